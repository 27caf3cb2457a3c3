#!/usr/bin/env python3
"""Every instance of bench.py's seeded per-GPU shard (131,072 mixed Road* QPs, N = 20) and of the
N = 10 configuration, device solve against the C oracle (oracle/ipm.c on the host cores):
status agreement (disagreements listed with their LP feasibility margin), |u - u_oracle| on
instances both call optimal, iteration-count differences, constraint violation of the device
answers.  Prints one JSON object.  Evidence run, not part of the test suite (the suite checks a
stratified sample of the same shard)."""
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))


def main():
    import torch
    import bench
    from conftest import TERMINAL_SETS
    from oracle import assembly as oa
    from oracle import qp as oq
    from oracle.cpu import CpuProblem
    from carmpc_amd.qp import solve_segments

    out = {}
    ctrls = bench.build_controllers(bench.ENVS, 20, torch.device("cuda", 0))
    X, env, offsets = bench.sample_shard(0, bench.PER_GPU, [c.goal for c in ctrls])
    u, st, it = solve_segments([c.qp for c in ctrls], offsets, torch.as_tensor(X).cuda())
    torch.cuda.synchronize()
    u, st, it = u.cpu().numpy(), st.cpu().numpy(), it.cpu().numpy()
    cases = [(name, 20, X[offsets[j]:offsets[j + 1]], u[offsets[j]:offsets[j + 1]], st[offsets[j]:offsets[j + 1]],
              it[offsets[j]:offsets[j + 1]]) for j, name in enumerate(bench.ENVS)]
    # the N = 10 configuration at the same density
    c10 = bench.build_controllers(["RoadEnv"], 10, torch.device("cuda", 0))[0]
    X10, _, _ = bench.sample_shard(0, 32768, [c10.goal])
    u10, st10, it10 = c10.qp.solve(torch.as_tensor(X10).cuda())
    cases.append(("RoadEnv", 10, X10, u10.cpu().numpy(), st10.cpu().numpy(), it10.cpu().numpy()))

    for name, N, Xe, ue, se, ie in cases:
        asm = oa.build(name, N, terminal_set_dir=TERMINAL_SETS)
        t0 = time.time()
        uc, sc, ic = CpuProblem(asm).solve(Xe, threads=16)
        dt = time.time() - t0
        agree = se == sc
        Gn, w0n, En, keep, pw, pE = oq.normalize_rows(asm.G, asm.w0, asm.E)
        margins = [float(oq.lp_margin(Gn, w0n - En @ Xe[i], asm.lb, asm.ub)) for i in np.where(~agree)[0][:50]]
        both = (se == 0) & (sc == 0)
        ok = se == 0
        w = asm.w0[None, :] - Xe[ok] @ asm.E.T
        viol = float(max((ue[ok] @ asm.G.T - w).max(), (ue[ok] - asm.ub[None]).max(), (asm.lb[None] - ue[ok]).max()))
        d = ie[both].astype(int) - ic[both].astype(int)
        out[f"{name}_N{N}"] = {
            "instances": int(len(Xe)), "device_status": np.bincount(se, minlength=4).tolist(),
            "oracle_status": np.bincount(sc, minlength=4).tolist(), "status_disagreements": int((~agree).sum()),
            "disagreement_lp_margins": margins, "both_optimal": int(both.sum()),
            "max_abs_u_diff": float(np.abs(ue[both] - uc[both]).max()),
            "max_constraint_violation_device": viol,
            "iteration_diff_hist": {str(k): int(v) for k, v in zip(*np.unique(d, return_counts=True))},
            "iters_mean_device": float(ie[both].mean()), "iters_mean_oracle": float(ic[both].mean()),
            "oracle_seconds_16_threads": round(dt, 2)}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
