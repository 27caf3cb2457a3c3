"""One call with 1,048,576 instances (bench's 131,072-instance shard tiled 8 times per environment) on one
GPU: statuses, iteration counts and inputs must equal the tiled results of the 131,072-instance call
(every instance is solved with the same arithmetic wherever it sits) -- checks the work-list indexing of
the three-launch form at the full size of configuration 5 and prints the time of the call."""
import sys, os, numpy as np, torch, time
sys.path.insert(0, os.getcwd())
import bench
from carmpc_amd.qp import solve_segments
ctrls = bench.build_controllers(bench.ENVS, 20, torch.device("cuda", 0))
probs = [c.qp for c in ctrls]
X, env, offsets = bench.sample_shard(0, 131072, [c.goal for c in ctrls])
u1, s1, i1 = solve_segments(probs, offsets, torch.as_tensor(X).cuda())
reps = 8
# per-environment tiling keeps the segments contiguous
Xb = np.concatenate([np.tile(X[offsets[j]:offsets[j+1]], (reps, 1)) for j in range(3)])
ob = np.array([0] + list(np.cumsum([(offsets[j+1]-offsets[j])*reps for j in range(3)])))
print("big batch", Xb.shape, ob, flush=True)
Xd = torch.as_tensor(Xb).cuda()
torch.cuda.synchronize(); t0 = time.time()
ub, sb, ib = solve_segments(probs, ob, Xd)
torch.cuda.synchronize(); dt = time.time() - t0
ok = True
for j in range(3):
    a = slice(int(offsets[j]), int(offsets[j+1])); b = slice(int(ob[j]), int(ob[j+1]))
    ok &= torch.equal(sb[b], s1[a].repeat(reps)) and torch.equal(ib[b], i1[a].repeat(reps))
    opt = (s1[a] == 0).repeat(reps)
    ok &= torch.equal(ub[b][opt], u1[a].repeat(reps, 1)[opt])
print("1,048,576 instances in %.1f ms (first call), equal to the tiled 131,072 results: %s" % (dt*1e3, ok))
assert ok
