#!/usr/bin/env python3
"""Generate the committed golden fixtures under tests/golden/ (build container only).

Provenance
----------
* ``assembly_<env>_N<N>.npz`` -- T, S, H, h computed by the REFERENCE's own
  ``lib/matrix_gen.py`` (``predmod``/``costgen``, imported from /root/reference,
  which imports directly without stubs) from A, B, P restated in
  ``oracle/assembly.py`` (``lib/mpc.py`` itself needs cvxpy, which is absent, so
  it is not imported); environment rows/goal/name read from the REFERENCE's
  ``lib/environments.py`` objects; configuration constants from the REFERENCE's
  ``lib/configuration.py``; terminal-set rows from the reference's data files.
* ``plant.npz`` -- seeded (state, u) pairs stepped through the REFERENCE's
  ``lib/simulator.CarSimulator`` (dt = DT_SIMULATION).
* ``qp_<env>_N<N>.npz`` -- 64 seeded x0 per config with the oracle's status,
  the KKT-certified optimum ``u_star`` (active-set polish of oracle.qp), its
  iteration count, and the HiGHS LP feasibility margin.  QP parity is
  *unpinned* against the reference's solver (cvxpy absent); see oracle/__init__.py.
* ``closed_loop_statefb.npz`` -- the run_MPCStateFB loop (examples/run_MPCStateFB.py:29-41)
  on RoadMultipleCarsEnv N=20 from [5,-1.5,0.1,0], using the REFERENCE plant and
  the oracle QP.

Run:  PYTHONDONTWRITEBYTECODE=1 MPLBACKEND=Agg python tools/make_golden.py
"""
from __future__ import annotations

import os
import sys
import json

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF = "/root/reference"
OUT = os.path.join(REPO, "tests", "golden")
sys.path.insert(0, REPO)

from oracle import assembly as oa  # noqa: E402
from oracle import qp as oq        # noqa: E402

CONFIGS = [("RoadEnv", 10), ("RoadEnv", 20), ("RoadOneCarEnv", 20), ("RoadMultipleCarsEnv", 20)]


def sample_x0(rng, goal_x, k):
    """Survey §8d input distribution: x in [g_x-25, g_x], y in [-3,3], psi in [-pi/8,pi/8], v in [-1,5]."""
    return np.stack([rng.uniform(goal_x - 25, goal_x, k), rng.uniform(-3, 3, k),
                     rng.uniform(-np.pi / 8, np.pi / 8, k), rng.uniform(-1, 5, k)], axis=1)


def main():
    os.makedirs(OUT, exist_ok=True)
    os.environ.setdefault("MPLBACKEND", "Agg")
    sys.path.insert(0, REF)
    import lib.matrix_gen as ref_mg          # reference code, imported read-only
    import lib.environments as ref_env
    import lib.simulator as ref_sim
    import lib.configuration as ref_cfg
    sys.path.remove(REF)

    meta = {"reference": REF, "configs": CONFIGS,
            "configuration": {"DT_CONTROL": ref_cfg.DT_CONTROL, "N": ref_cfg.N,
                              "LINEARIZE_STATE": list(ref_cfg.LINEARIZE_STATE),
                              "LINEARIZE_INPUT": list(ref_cfg.LINEARIZE_INPUT),
                              "Q": ref_cfg.STAGE_COST_Q.tolist(), "R": ref_cfg.STAGE_COST_R.tolist(),
                              "STEPS_UPDATE": ref_cfg.STEPS_UPDATE}}
    envs = {}
    for cls in (ref_env.RoadEnv, ref_env.RoadOneCarEnv, ref_env.RoadMultipleCarsEnv):
        e = cls()
        envs[e.name] = {"constraints_A": np.asarray(e.constraints_A, float).tolist(),
                        "constraints_b": np.asarray(e.constraints_b, float).tolist(),
                        "goal": list(e.goal), "lim": e.lim}
    meta["environments"] = envs

    for name, N in CONFIGS:
        asm = oa.build(name, N, terminal_set_dir=os.path.join(REF, "terminal_sets"))
        T, S = ref_mg.predmod(asm.A, asm.B, N)
        H, h, const = ref_mg.costgen(ref_cfg.STAGE_COST_Q, ref_cfg.STAGE_COST_R, asm.P, T, S, 4)
        np.savez(os.path.join(OUT, f"assembly_{name}_N{N}.npz"), A=asm.A, B=asm.B, P=asm.P, K=asm.K,
                 T=T, S=S, H=H, h=h, const=const,
                 term=np.load(os.path.join(REF, "terminal_sets", oa.terminal_set_filename(name, envs[name]["goal"]))))

        rng = np.random.default_rng(1000 + N + len(name))
        X0 = sample_x0(rng, asm.goal[0], 64)
        status, iters, ustar, margin = [], [], [], []
        for x0 in X0:
            r = oq.solve_instance(asm, x0)
            Gn, w0n, En, keep, pw, pE = oq.normalize_rows(asm.G, asm.w0, asm.E)
            pre = pw - pE @ x0
            m = float(pre.min()) if pre.size and pre.min() < 0 else oq.lp_margin(Gn, w0n - En @ x0, asm.lb, asm.ub)
            if r["status"] == oq.STATUS_OPTIMAL:
                assert r["certified"], (name, N, x0, r.get("kkt"))
                ustar.append(r["u_exact"])
            else:
                ustar.append(np.full(2 * N, np.nan))
            assert (m >= 0) == (r["status"] == oq.STATUS_OPTIMAL), (name, N, x0, m, r["status"])
            status.append(r["status"]); iters.append(r["iters"]); margin.append(m)
        np.savez(os.path.join(OUT, f"qp_{name}_N{N}.npz"), x0=X0, status=np.array(status, np.int32),
                 iters=np.array(iters, np.int32), u_star=np.array(ustar), margin=np.array(margin))
        print(name, N, "feasible", int(np.sum(np.array(status) == 0)), "/ 64",
              "iters mean %.2f" % np.mean([i for i, s in zip(iters, status) if s == 0]))

    # plant golden: reference simulator on seeded pairs
    rng = np.random.default_rng(7)
    states = sample_x0(rng, 30.0, 32)
    us = np.stack([rng.uniform(-2, 2, 32), rng.uniform(-np.pi / 8, np.pi / 8, 32)], axis=1)
    nxt = []
    for s0, u in zip(states, us):
        sim = ref_sim.CarSimulator(dt=ref_cfg.DT_SIMULATION)
        sim.reset(np.array(s0))
        sim.step(u)
        nxt.append(sim.state.copy())
    np.savez(os.path.join(OUT, "plant.npz"), state=states, u=us, next=np.array(nxt))

    # closed loop: examples/run_MPCStateFB.py:29-41 with the reference plant + oracle QP
    asm = oa.build("RoadMultipleCarsEnv", 20, terminal_set_dir=os.path.join(REF, "terminal_sets"))
    sim = ref_sim.CarSimulator(dt=ref_cfg.DT_SIMULATION)
    sim.reset(np.array([5, -1.5, 0.1, 0]))
    u = [0, 0]
    traj, inputs = [], []
    for i in range(1000):
        sim.step(u)
        traj.append(sim.state.copy())
        if i % ref_cfg.STEPS_UPDATE == 0:
            r = oq.solve_instance(asm, sim.state)
            assert r["status"] == 0 and r["certified"]
            u = r["u_exact"][:2]
            inputs.append(u.copy())
        if np.all(np.abs(sim.state - asm.goal) <= 1e-1) or i > 30 / ref_cfg.DT_SIMULATION:
            break
    np.savez(os.path.join(OUT, "closed_loop_statefb.npz"), states=np.array(traj), inputs=np.array(inputs))
    print("closed loop steps", len(traj), "final", traj[-1])
    meta["closed_loop_steps"] = len(traj)
    with open(os.path.join(OUT, "meta.json"), "w") as f:
        json.dump(meta, f, indent=1)


if __name__ == "__main__":
    main()
