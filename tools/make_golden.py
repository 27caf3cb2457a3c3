#!/usr/bin/env python3
"""Generate the committed golden fixtures under tests/golden/ (build container only).

Provenance
----------
* ``assembly_<env>_N<N>.npz`` -- everything the REFERENCE's own constructor
  ``lib/mpc.py::MPCStateFB.__init__`` (mpc.py:22-117) leaves on the object: A, B, P, K, T, S,
  H, h, the terminal rows, and the stacks returned by its ``terminal_constraint()``,
  ``input_constraint()`` and ``state_constraint()`` (mpc.py:196-253).  ``lib/mpc.py`` does
  ``import cvxpy`` (absent here); the constructors and constraint builders never call it, so
  the module is imported with an EMPTY module object registered under that name -- nothing of
  cvxpy is emulated, and ``step`` (which needs the real solver) is never called.  The
  constructor runs with cwd = <reference>/examples, as the example scripts do, so its
  ``'../terminal_sets/'`` lookup finds the reference's data files.
  ``assembly_fallback_RoadEnv_N10.npz`` is the same dump for a goal without a terminal-set
  file (the goal-box fallback, mpc.py:107-117).
* ``observer.npz`` -- the REFERENCE's ``MPCOutputFB.luenberger_observer`` (mpc.py:439-448) and
  ``MPCOutputFBWithDisturbance.luenberger_observer`` (mpc.py:598-612) on seeded
  (x_estimate, previous_u, y0[, d_estimate]) tuples, with their C, L, Bd, Cd, L1, L2.
* ``plant.npz`` -- seeded (state, u) pairs stepped through the REFERENCE's
  ``lib/simulator.CarSimulator`` (dt = DT_SIMULATION); ``oob_*``: inputs outside the actuator
  limits with the outcome of the reference's ``check_input`` (simulator.py:83-97: raised or
  not) and the next state when it did not raise.
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
    """Input distribution of the benchmark configurations: x in [g_x-25, g_x], y in [-3,3], psi in [-pi/8,pi/8], v in [-1,5]."""
    return np.stack([rng.uniform(goal_x - 25, goal_x, k), rng.uniform(-3, 3, k),
                     rng.uniform(-np.pi / 8, np.pi / 8, k), rng.uniform(-1, 5, k)], axis=1)


def import_reference():
    """The reference's lib.* modules, imported read-only from /root/reference.  lib.mpc does
    ``import cvxpy``: an empty module object stands under that name (see the module docstring)."""
    import types
    os.environ.setdefault("MPLBACKEND", "Agg")
    sys.dont_write_bytecode = True
    sys.modules.setdefault("cvxpy", types.ModuleType("cvxpy"))
    # The reference's lib/ has no __init__.py (a namespace package), so a regular package of the
    # same name anywhere on sys.path -- this repository's own lib/ shim -- would win the import
    # whatever the path order.  Bind the name to the reference's directory explicitly and check
    # where every module came from.
    for k in [k for k in sys.modules if k == "lib" or k.startswith("lib.")]:
        del sys.modules[k]
    pkg = types.ModuleType("lib")
    pkg.__path__ = [os.path.join(REF, "lib")]
    sys.modules["lib"] = pkg
    import lib.matrix_gen as ref_mg          # reference code, imported read-only
    import lib.environments as ref_env
    import lib.simulator as ref_sim
    import lib.configuration as ref_cfg
    import lib.mpc as ref_mpc
    for m in (ref_mg, ref_env, ref_sim, ref_cfg, ref_mpc):
        assert os.path.realpath(m.__file__).startswith(os.path.join(REF, "lib") + os.sep), m.__file__
    return ref_mg, ref_env, ref_sim, ref_cfg, ref_mpc


def reference_constructor(ref_mpc, ref_env, ref_cfg, name, N, goal=None, cls="MPCStateFB", **kw):
    """Run the reference's own constructor (cwd = <reference>/examples, like its scripts)."""
    import contextlib
    import io
    env = getattr(ref_env, name)()
    if goal is not None:
        env.goal = list(goal)
    cwd = os.getcwd()
    os.chdir(os.path.join(REF, "examples"))
    try:
        with contextlib.redirect_stdout(io.StringIO()) as out:
            ctrl = getattr(ref_mpc, cls)(dt=ref_cfg.DT_CONTROL, N=N, lin_state=ref_cfg.LINEARIZE_STATE,
                                         lin_input=ref_cfg.LINEARIZE_INPUT, env=env, **kw)
    finally:
        os.chdir(cwd)
    return ctrl, env, out.getvalue()


def dump_constructor(ctrl, path, ref_mg):
    tA, tb = ctrl.terminal_constraint()
    iA, ib = ctrl.input_constraint()
    sA, sb = ctrl.state_constraint()
    const = ref_mg.costgen(ctrl.Q, ctrl.R, ctrl.P, ctrl.T, ctrl.S, ctrl.nx)[2]   # the constructor drops it (mpc.py:78)
    np.savez_compressed(path, const=const, A=ctrl.A, B=ctrl.B, P=ctrl.P, K=ctrl.K, T=ctrl.T, S=ctrl.S, H=ctrl.H, h=ctrl.h,
                        goal=np.asarray(ctrl.goal, float), input_upper=ctrl.input_upper, input_lower=ctrl.input_lower,
                        term_A=tA, term_b=tb, input_A=iA, input_b=ib, state_A=sA, state_b=sb,
                        term=np.hstack((tA[:, -4:], np.asarray(tb, float)[:, None])))


def qp_vectors():
    """qp_<env>_N<N>.npz: seeded x0 with the oracle's status, iteration counts (``iters``: with the
    oracle's polish -- early gate, correction round; ``iters_single``: the fallback kernels' variant,
    qp.FALLBACK_VARIANT),
    the certified optimum and the feasibility margin.  Needs the oracle and the reference's
    terminal-set files only."""
    for name, N in CONFIGS:
        asm = oa.build(name, N, terminal_set_dir=os.path.join(REF, "terminal_sets"))

        rng = np.random.default_rng(1000 + N + len(name))
        X0 = sample_x0(rng, asm.goal[0], 64)
        status, iters, iters1, ustar, margin = [], [], [], [], []
        for x0 in X0:
            r = oq.solve_instance(asm, x0)
            r1 = oq.solve_instance(asm, x0, **oq.FALLBACK_VARIANT)
            assert r1["status"] == r["status"]
            Gn, w0n, En, keep, pw, pE = oq.normalize_rows(asm.G, asm.w0, asm.E)
            pre = pw - pE @ x0
            m = float(pre.min()) if pre.size and pre.min() < 0 else oq.lp_margin(Gn, w0n - En @ x0, asm.lb, asm.ub)
            if r["status"] == oq.STATUS_OPTIMAL:
                assert r["certified"], (name, N, x0, r.get("kkt"))
                ustar.append(r["u_exact"])
            else:
                ustar.append(np.full(2 * N, np.nan))
            assert (m >= 0) == (r["status"] == oq.STATUS_OPTIMAL), (name, N, x0, m, r["status"])
            status.append(r["status"]); iters.append(r["iters"]); iters1.append(r1["iters"]); margin.append(m)
        np.savez(os.path.join(OUT, f"qp_{name}_N{N}.npz"), x0=X0, status=np.array(status, np.int32),
                 iters=np.array(iters, np.int32), iters_single=np.array(iters1, np.int32), u_star=np.array(ustar),
                 margin=np.array(margin))
        print(name, N, "feasible", int(np.sum(np.array(status) == 0)), "/ 64",
              "iters mean %.2f" % np.mean([i for i, s in zip(iters, status) if s == 0]),
              "(fallback polish variant %.2f)" % np.mean([i for i, s in zip(iters1, status) if s == 0]))


def main():
    os.makedirs(OUT, exist_ok=True)
    ref_mg, ref_env, ref_sim, ref_cfg, ref_mpc = import_reference()

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

    # constructor dumps: the reference's own MPCStateFB.__init__ and constraint builders
    for name, N in CONFIGS:
        ctrl, env, log = reference_constructor(ref_mpc, ref_env, ref_cfg, name, N)
        assert "Using" in log and "terminal set" in log, log
        dump_constructor(ctrl, os.path.join(OUT, f"assembly_{name}_N{N}.npz"), ref_mg)
    FALLBACK_GOAL = [25, 0.5, 0, 0]      # an equilibrium without a terminal-set file
    ctrl, env, log = reference_constructor(ref_mpc, ref_env, ref_cfg, "RoadEnv", 10, goal=FALLBACK_GOAL)
    assert "No terminal set found" in log, log
    dump_constructor(ctrl, os.path.join(OUT, "assembly_fallback_RoadEnv_N10.npz"), ref_mg)
    meta["fallback_goal"] = FALLBACK_GOAL

    # observers: the reference's own methods on seeded tuples
    rng = np.random.default_rng(11)
    import contextlib
    import io
    ofb, _, _ = reference_constructor(ref_mpc, ref_env, ref_cfg, "RoadMultipleCarsEnv", 20, cls="MPCOutputFB",
                                      init_state=[5, -1.5, 0, 0])
    dfb, _, _ = reference_constructor(ref_mpc, ref_env, ref_cfg, "RoadMultipleCarsEnv", 20,
                                      cls="MPCOutputFBWithDisturbance", init_state=[5, -1.5, 0, 0])
    xe = sample_x0(rng, 30.0, 32)
    up = np.stack([rng.uniform(-2, 2, 32), rng.uniform(-np.pi / 8, np.pi / 8, 32)], axis=1)
    y0 = xe[:, [0, 1, 3]] + rng.normal(0, 0.05, (32, 3))
    de = rng.normal(0, 0.1, 32)
    lo, dx, dd = [], [], []
    for i in range(32):
        ofb.x_estimate, ofb.previous_u = xe[i].copy(), up[i].copy()
        lo.append(ofb.luenberger_observer(y0[i]))
        dfb.x_estimate, dfb.previous_u, dfb.d_estimate = xe[i].copy(), up[i].copy(), float(de[i])
        with contextlib.redirect_stdout(io.StringIO()):     # the reference prints its innovations
            xn, dn = dfb.luenberger_observer(y0[i])
        dx.append(xn); dd.append(dn)
    np.savez(os.path.join(OUT, "observer.npz"), x_estimate=xe, previous_u=up, y0=y0, d_estimate=de,
             C=ofb.C, L=ofb.L, y_goal=ofb.y_goal, next=np.array(lo),
             Bd=np.asarray(dfb.Bd, float), Cd=np.asarray(dfb.Cd, float), L1=dfb.L1, L2=np.asarray(dfb.L2, float),
             next_dist_x=np.array(dx), next_dist_d=np.array(dd))

    qp_vectors()

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
    # inputs outside the actuator limits: what the reference's check_input does with them
    oob_u = np.array([[a, d] for a in (-5.0, -2.1, -2.05, 2.05, 2.1, 0.5)
                      for d in (-1.0, -np.pi / 4 - 0.05, 0.1, np.pi / 4 + 0.05, 1.0)])
    oob_state = sample_x0(rng, 30.0, len(oob_u))
    oob_raised, oob_next = [], []
    for s0, u in zip(oob_state, oob_u):
        sim = ref_sim.CarSimulator(dt=ref_cfg.DT_SIMULATION)
        sim.reset(np.array(s0))
        try:
            sim.step(u)
            oob_raised.append(0)
        except AssertionError:
            oob_raised.append(1)
        oob_next.append(np.asarray(sim.state, float).copy())     # unchanged when the check raised
    np.savez(os.path.join(OUT, "plant.npz"), state=states, u=us, next=np.array(nxt), oob_state=oob_state,
             oob_u=oob_u, oob_raised=np.array(oob_raised, np.int32), oob_next=np.array(oob_next))
    print("check_input raised on", int(np.sum(oob_raised)), "of", len(oob_u), "out-of-range inputs")

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

    # the plumbing configuration: the same runner on RoadEnv with N = 10.  The example's start
    # [5, -1.5, 0.1, 0] is infeasible at N = 10 (the reference raises at step 0), so the trace
    # starts at [22, 0, 0, 3]; it runs to the runner's time limit (i > 30 / DT_SIMULATION).
    asm = oa.build("RoadEnv", 10, terminal_set_dir=os.path.join(REF, "terminal_sets"))
    assert oq.solve_instance(asm, np.array([5, -1.5, 0.1, 0]))["status"] == oq.STATUS_INFEASIBLE
    sim = ref_sim.CarSimulator(dt=ref_cfg.DT_SIMULATION)
    sim.reset(np.array([22.0, 0.0, 0.0, 3.0]))
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
    np.savez(os.path.join(OUT, "closed_loop_statefb_RoadEnv_N10.npz"), states=np.array(traj), inputs=np.array(inputs))
    print("RoadEnv N=10 closed loop steps", len(traj), "final", traj[-1])
    meta["closed_loop_steps_RoadEnv_N10"] = len(traj)
    with open(os.path.join(OUT, "meta.json"), "w") as f:
        json.dump(meta, f, indent=1)


if __name__ == "__main__":
    if "--only-qp" in sys.argv:
        qp_vectors()      # (the other fixtures do not depend on the solver's iteration sequence)
    else:
        main()
