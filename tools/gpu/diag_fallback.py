"""Diagnose status disagreements of the goal-box fallback case (RoadEnv N=10) per kernel."""
import os, sys, tempfile, json
import numpy as np
import torch
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "."))
from oracle import assembly as oa
from oracle import qp as oq
from oracle.cpu import CpuProblem
from carmpc_amd.qp import QPProblem, SolverSettings

tmp = tempfile.mkdtemp()
out = {}
for N in (10,):
    asm = oa.build("RoadEnv", N, terminal_set_dir=tmp)
    qp = QPProblem(N=N, A=asm.A, B=asm.B, Q=oa.STAGE_COST_Q, R=oa.STAGE_COST_R, P=asm.P, goal=asm.goal,
                   state_A=np.asarray(asm.state_rows_A, float), state_b=np.asarray(asm.state_rows_b, float),
                   term_A=asm.term_A[:, -4:], term_b=asm.term_b, u_lower=asm.input_lower, u_upper=asm.input_upper)
    rng = np.random.default_rng(N)
    X = np.stack([rng.uniform(28, 30, 200), rng.uniform(1, 2, 200), rng.uniform(-0.05, 0.05, 200),
                  rng.uniform(-0.2, 0.2, 200)], axis=1)
    uc, sc, ic = CpuProblem(asm).solve(X)
    for k in (1, 2):
        u, st, it = qp.solve(torch.as_tensor(X).cuda(), settings=SolverSettings(kernel=k))
        st, it, u = st.cpu().numpy(), it.cpu().numpy(), u.cpu().numpy()
        bad = np.where(st != sc)[0]
        out[f"N{N}_k{k}"] = dict(kernel=qp.kernel, mismatches=[dict(i=int(i), gpu=int(st[i]), gpu_it=int(it[i]), cpu=int(sc[i]),
                                  cpu_it=int(ic[i]), x0=X[i].tolist()) for i in bad],
                                  agree=float((st == sc).mean()), both_opt_err=float(np.abs(u[(st == 0) & (sc == 0)] - uc[(st == 0) & (sc == 0)]).max()),
                                  status_counts=np.bincount(st, minlength=4).tolist(), cpu_counts=np.bincount(sc, minlength=4).tolist(),
                                  it_gpu=it.tolist(), it_cpu=ic.tolist())
os.makedirs("gpurun_out", exist_ok=True)
json.dump(out, open("gpurun_out/diag_fallback.json", "w"), indent=1)
for k, v in out.items():
    print(k, v["agree"], v["status_counts"], v["cpu_counts"], v["both_opt_err"], v["mismatches"])
