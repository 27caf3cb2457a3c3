"""Parity/timing check of the grouped Riccati kernel (settings.kernel = 7) vs the C oracle."""
import os, sys, time, json
import numpy as np
import torch
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "."))
from oracle import assembly as oa
from oracle.cpu import CpuProblem
from carmpc_amd.qp import QPProblem, SolverSettings

out = {}
for name, N in [("RoadEnv", 10), ("RoadEnv", 20), ("RoadOneCarEnv", 20), ("RoadMultipleCarsEnv", 20)]:
    asm = oa.build(name, N, terminal_set_dir="terminal_sets")
    qp = QPProblem(N=N, A=asm.A, B=asm.B, Q=oa.STAGE_COST_Q, R=oa.STAGE_COST_R, P=asm.P, goal=asm.goal,
                   state_A=np.asarray(asm.state_rows_A, float), state_b=np.asarray(asm.state_rows_b, float),
                   term_A=asm.term_A[:, -4:], term_b=asm.term_b, u_lower=asm.input_lower, u_upper=asm.input_upper)
    rng = np.random.default_rng(11 + N)
    B = 2048
    gx = asm.goal[0]
    X = np.stack([rng.uniform(gx - 25, gx, B), rng.uniform(-3, 3, B), rng.uniform(-np.pi / 8, np.pi / 8, B),
                  rng.uniform(-1, 5, B)], axis=1)
    uc, sc, ic = CpuProblem(asm).solve(X)
    res = {}
    for k in (2, 7):
        u, st, it = qp.solve(torch.as_tensor(X).cuda(), settings=SolverSettings(kernel=k))
        torch.cuda.synchronize()
        u, st, it = u.cpu().numpy(), st.cpu().numpy(), it.cpu().numpy()
        both = (st == 0) & (sc == 0)
        res[k] = dict(agree=float((st == sc).mean()), status=np.bincount(st, minlength=4).tolist(),
                      err=float(np.abs(u[both] - uc[both]).max()) if both.any() else None,
                      iter_diff=np.unique(it[both] - ic[both], return_counts=True)[0].tolist()[:10],
                      bad=[(int(i), int(st[i]), int(sc[i]), int(it[i]), int(ic[i])) for i in np.where(st != sc)[0][:8]])
        # timing on a big batch
        Xb = torch.as_tensor(np.tile(X, (32, 1))).cuda()
        for _ in range(2):
            qp.solve(Xb, settings=SolverSettings(kernel=k))
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(3):
            qp.solve(Xb, settings=SolverSettings(kernel=k))
        torch.cuda.synchronize()
        res[k]["qps"] = 3 * Xb.shape[0] / (time.perf_counter() - t0)
    out[f"{name}_N{N}"] = res
    print(name, N, json.dumps(res), flush=True)
os.makedirs("gpurun_out", exist_ok=True)
json.dump(out, open("gpurun_out/ric_check.json", "w"), indent=1)
