"""Problems whose terminal set is the goal box (rows paired into equalities) at N = 5 and 10: the grouped kernel
against the C oracle on 200 states, repeated, with the mismatching instances listed.  CARMPC_LIB selects the library."""
import os
import sys
import tempfile

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))
from oracle import assembly as oa  # noqa: E402
from oracle.cpu import CpuProblem  # noqa: E402
from carmpc_amd.qp import QPProblem, SolverSettings  # noqa: E402

tmp = tempfile.mkdtemp()
for N in (5, 10, 20):
    asm = oa.build("RoadEnv", N, terminal_set_dir=tmp)
    qp = QPProblem(N=N, A=asm.A, B=asm.B, Q=oa.STAGE_COST_Q, R=oa.STAGE_COST_R, P=asm.P, goal=asm.goal,
                   state_A=np.asarray(asm.state_rows_A, float), state_b=np.asarray(asm.state_rows_b, float),
                   term_A=asm.term_A[:, -4:], term_b=asm.term_b, u_lower=asm.input_lower, u_upper=asm.input_upper)
    rng = np.random.default_rng(N)
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 200
    X = np.stack([rng.uniform(30 - 0.2 * N, 30, B), rng.uniform(1, 2, B), rng.uniform(-0.05, 0.05, B), rng.uniform(-0.2, 0.2, B)], axis=1)
    uc, sc, ic = CpuProblem(asm).solve(X)
    Xd = torch.as_tensor(X).cuda()
    for rep in range(6):
        s = SolverSettings(kernel=7)
        u, st, it = qp.solve(Xd, settings=s)
        torch.cuda.synchronize()
        st = st.cpu().numpy(); it = it.cpu().numpy()
        bad = np.nonzero((st != sc) | (it != ic))[0]
        print("N", N, "rep", rep, "mismatches", len(bad), bad[:10].tolist(), "status", st[bad[:10]].tolist(), "oracle", sc[bad[:10]].tolist(),
              "iters", it[bad[:10]].tolist(), "oracle", ic[bad[:10]].tolist(), flush=True)
