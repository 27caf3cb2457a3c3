"""One batch of RoadMultipleCarsEnv N=20 QPs per kernel id (argv), for rocprofv3 counter passes."""
import os, sys
import numpy as np
import torch
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "."))
from oracle import assembly as oa
from carmpc_amd.qp import QPProblem, SolverSettings

name = os.environ.get("ENV", "RoadMultipleCarsEnv")
asm = oa.build(name, 20, terminal_set_dir="terminal_sets")
qp = QPProblem(N=20, A=asm.A, B=asm.B, Q=oa.STAGE_COST_Q, R=oa.STAGE_COST_R, P=asm.P, goal=asm.goal,
               state_A=np.asarray(asm.state_rows_A, float), state_b=np.asarray(asm.state_rows_b, float),
               term_A=asm.term_A[:, -4:], term_b=asm.term_b, u_lower=asm.input_lower, u_upper=asm.input_upper)
rng = np.random.default_rng(5)
B = 65536
gx = asm.goal[0]
X = torch.as_tensor(np.stack([rng.uniform(gx - 25, gx, B), rng.uniform(-3, 3, B), rng.uniform(-np.pi / 8, np.pi / 8, B),
                              rng.uniform(-1, 5, B)], axis=1)).cuda()
for k in [int(a) for a in sys.argv[1:]] or [7]:
    u, st, it = qp.solve(X, settings=SolverSettings(kernel=k))
    torch.cuda.synchronize()
    itn = it.cpu().numpy(); stn = st.cpu().numpy()
    print(k, "iters mean", itn.mean(), "status", np.bincount(stn, minlength=4).tolist(), flush=True)
