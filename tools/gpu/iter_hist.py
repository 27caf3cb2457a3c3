import sys, os, numpy as np, torch
sys.path.insert(0, os.getcwd())
import bench
from carmpc_amd.qp import solve_segments
ctrls = bench.build_controllers(bench.ENVS, 20, torch.device("cuda", 0))
probs = [c.qp for c in ctrls]
X, env, offsets = bench.sample_shard(0, 131072, [c.goal for c in ctrls])
u, s, i = solve_segments(probs, offsets, torch.as_tensor(X).cuda())
torch.cuda.synchronize()
s, i = s.cpu().numpy(), i.cpu().numpy()
print("optimal iters hist", np.bincount(i[s == 0]))
print("infeasible iters hist", np.bincount(i[s == 1]))
