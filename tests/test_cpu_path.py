"""The product's CPU QP path (carmpc_cpu_*, carmpc_amd.qp.CpuQPProblem) and the controllers on
it (device="cpu", or no GPU present): BASELINE configuration 1 -- the run_MPCStateFB loop on
RoadEnv with N = 10 and the QP on the CPU, no GPU (examples/run_MPCStateFB.py:15-40 over
lib/mpc.py:312-349) -- plus the same parity checks the device path gets.

Tolerances as for the device path: |u - u*|_inf <= 1e-6 against the KKT-certified optimum,
constraint violation <= 1e-8, status identical to the oracle."""
import os
import subprocess
import sys

import numpy as np
import pytest

from conftest import CONFIGS, GOLDEN, REPO, TERMINAL_SETS
from costs import OBJ_RTOL, objective, objective_gap, stage_cost, terminal_cost

from oracle import assembly as oa
from oracle import qp as oq

U_TOL = 1e-6
VIOL_TOL = 1e-8


def _cpu_qp(asm, **kw):
    from carmpc_amd.qp import CpuQPProblem
    t, i, s = asm.flags
    return CpuQPProblem(N=asm.N, A=asm.A, B=asm.B, Q=oa.STAGE_COST_Q, R=oa.STAGE_COST_R, P=asm.P, goal=asm.goal,
                        state_A=np.asarray(asm.state_rows_A, float) if s else None,
                        state_b=np.asarray(asm.state_rows_b, float) if s else None,
                        term_A=asm.term_A[:, -4:] if t else None, term_b=asm.term_b if t else None,
                        u_lower=asm.input_lower if i else None, u_upper=asm.input_upper if i else None, **kw)


def _x0(rng, goal_x, B):
    return np.stack([rng.uniform(goal_x - 25, goal_x, B), rng.uniform(-3, 3, B),
                     rng.uniform(-np.pi / 8, np.pi / 8, B), rng.uniform(-1, 5, B)], axis=1)


@pytest.mark.parametrize("name,N", CONFIGS)
def test_cpu_path_golden_vectors(name, N):
    asm = oa.build(name, N, terminal_set_dir=TERMINAL_SETS)
    qp = _cpu_qp(asm)
    g = np.load(os.path.join(GOLDEN, f"qp_{name}_N{N}.npz"))
    u, st, it = qp.solve(g["x0"], threads=2)
    np.testing.assert_array_equal(st, g["status"])
    ok = st == 0
    assert np.abs(u[ok] - g["u_star"][ok]).max() <= U_TOL
    assert np.abs(it[ok] - g["iters"][ok]).max() <= 1          # same algorithm as the oracle
    for x0, uu, us in zip(g["x0"][ok], u[ok], g["u_star"][ok]):
        assert objective_gap(asm, x0, uu, us) <= OBJ_RTOL
        w = asm.w0 - asm.E @ x0
        assert (asm.G @ uu - w).max() <= VIOL_TOL and (uu - asm.ub).max() <= VIOL_TOL and (asm.lb - uu).max() <= VIOL_TOL
        xN = (asm.T @ x0 + asm.S @ uu)[-4:]
        assert (asm.term_A[:, -4:] @ xN - asm.term_b).max() <= VIOL_TOL       # terminal-set feasibility
    m = qp.matrices()                                           # host assembly against the oracle's
    np.testing.assert_allclose(m["G"], asm.G, rtol=0, atol=1e-12)
    np.testing.assert_allclose(m["E"], asm.E, rtol=0, atol=1e-12)
    np.testing.assert_array_equal(m["w0"], asm.w0)


@pytest.mark.parametrize("name,N", CONFIGS)
def test_cpu_path_random_batch_vs_oracle(name, N):
    from oracle.cpu import CpuProblem
    asm = oa.build(name, N, terminal_set_dir=TERMINAL_SETS)
    qp = _cpu_qp(asm)
    X = _x0(np.random.default_rng(31 + N), asm.goal[0], 1024)
    u, st, it = qp.solve(X, threads=4)
    uc, sc, ic = CpuProblem(asm).solve(X, threads=4)
    np.testing.assert_array_equal(st, sc)
    both = (st == 0) & (sc == 0)
    assert both.sum() > 256 and (st == 1).sum() > 0 and (st >= 2).sum() == 0
    assert np.abs(u[both] - uc[both]).max() <= U_TOL
    for i in np.where(both)[0][:12]:                            # and against the exact optimum
        r = oq.solve_instance(asm, X[i])
        assert r["certified"] and np.abs(u[i] - r["u_exact"]).max() <= U_TOL
    # thread count and batch order do not change a result
    u1, st1, _ = qp.solve(X[:100], threads=1)
    np.testing.assert_array_equal(u1, u[:100])
    np.testing.assert_array_equal(st1, st[:100])


def test_cpu_path_flags_fallback_and_edge_cases(tmp_path):
    from oracle.cpu import CpuProblem
    rng = np.random.default_rng(5)
    for kw in (dict(input_constraint_on=False), dict(terminal_constraint=False), dict(state_constraint_on=False)):
        asm = oa.build("RoadEnv", 20, terminal_set_dir=TERMINAL_SETS, **kw)
        X = _x0(rng, asm.goal[0], 200)
        u, st, _ = _cpu_qp(asm).solve(X, threads=2)
        uc, sc, _ = CpuProblem(asm).solve(X, threads=2)
        both = (st == 0) & (sc == 0)
        assert (st == sc).mean() > 0.99, kw
        assert np.abs(u[both] - uc[both]).max() <= U_TOL, kw
    # goal-box fallback: equality pairs (mpc.py:107-117)
    asm = oa.build("RoadEnv", 10, terminal_set_dir=str(tmp_path))
    X = np.stack([rng.uniform(28, 30, 100), rng.uniform(1, 2, 100), rng.uniform(-0.05, 0.05, 100),
                  rng.uniform(-0.2, 0.2, 100)], axis=1)
    u, st, _ = _cpu_qp(asm).solve(X, threads=2)
    uc, sc, _ = CpuProblem(asm).solve(X, threads=2)
    np.testing.assert_array_equal(st, sc)
    assert (st == 0).all() and np.abs(u - uc).max() <= U_TOL
    # empty batch, one instance at the goal, explicit xref
    asm = oa.build("RoadOneCarEnv", 20, terminal_set_dir=TERMINAL_SETS)
    qp = _cpu_qp(asm)
    u, st, it = qp.solve(np.zeros((0, 4)))
    assert u.shape == (0, 40) and st.shape == (0,)
    u, st, it = qp.solve(asm.goal.reshape(1, 4))
    assert st[0] == 0 and np.abs(u).max() <= 1e-9
    X = _x0(rng, asm.goal[0], 13)
    u1, s1, _ = qp.solve(X)
    u2, s2, _ = qp.solve(X, np.tile(asm.goal, (13, 1)))
    np.testing.assert_array_equal(u1, u2)
    np.testing.assert_array_equal(s1, s2)


def test_cpu_path_iteration_limit():
    """Small max_iter: last-resort polish and the max-iter status, identical to the oracle's."""
    from oracle.cpu import CpuProblem
    from carmpc_amd.qp import SolverSettings
    asm = oa.build("RoadMultipleCarsEnv", 20, terminal_set_dir=TERMINAL_SETS)
    X = _x0(np.random.default_rng(5), asm.goal[0], 512)
    qp = _cpu_qp(asm)
    for mi in (2, 4):
        uc, sc, ic = CpuProblem(asm).solve(X, max_iter=mi, threads=4)
        u, st, it = qp.solve(X, settings=SolverSettings(max_iter=mi), threads=4)
        np.testing.assert_array_equal(st, sc)
        np.testing.assert_array_equal(it, ic)
        assert (st == 2).sum() > 50 and (st == 0).sum() > 20
        both = st == 0
        assert np.abs(u[both] - uc[both]).max() <= U_TOL


def test_cpu_path_disturbance_offsets():
    asm = oa.build("RoadMultipleCarsEnv", 20, terminal_set_dir=TERMINAL_SETS)
    qp = _cpu_qp(asm)
    qp.set_disturbance(oa.BD_DIST)
    rng = np.random.default_rng(8)
    X = _x0(rng, 30.0, 24)
    d = rng.normal(0, 0.02, 24)
    u, st, _ = qp.solve(X, oa.XREF_DIST.reshape(1, 4), dist=d)
    for i in range(24):
        r = oq.solve_instance_dist(asm, X[i], d[i])
        assert st[i] == r["status"]
        if r["status"] == 0:
            assert r["certified"] and np.abs(u[i] - r["u_exact"]).max() <= U_TOL


def test_config1_statefb_loop_on_cpu_matches_golden_trace():
    """BASELINE configuration 1: the run_MPCStateFB loop (examples/run_MPCStateFB.py:29-40) on
    RoadEnv with N = 10, QP on the CPU.  The script's own start is infeasible at N = 10 (the
    controller raises, as the reference would); from [22, 0, 0, 3] the loop runs its 152 steps."""
    from lib.configuration import DT_CONTROL, DT_SIMULATION, LINEARIZE_INPUT, LINEARIZE_STATE, STEPS_UPDATE
    from lib.environments import RoadEnv
    from lib.mpc import MPCStateFB, OutsideTheRegionOfAttractionError
    from lib.simulator import CarSimulator
    g = np.load(os.path.join(GOLDEN, "closed_loop_statefb_RoadEnv_N10.npz"))
    env = RoadEnv()
    ctrl = MPCStateFB(dt=DT_CONTROL, N=10, lin_state=LINEARIZE_STATE, lin_input=LINEARIZE_INPUT, env=env,
                      terminal_set_dir=TERMINAL_SETS, device="cpu")
    ctrl.set_goal(env.goal)
    assert ctrl.on_cpu
    with pytest.raises(OutsideTheRegionOfAttractionError):
        ctrl.step(np.array([5, -1.5, 0.1, 0]))
    plant = CarSimulator(dt=DT_SIMULATION)
    plant.reset(np.array([22.0, 0.0, 0.0, 3.0]))
    u = [0, 0]
    step = 0
    while True:
        plant.step(u)
        np.testing.assert_allclose(plant.state, g["states"][step], rtol=0, atol=1e-6)
        if step % STEPS_UPDATE == 0:
            u = ctrl.step(plant.state)
            np.testing.assert_allclose(u, g["inputs"][step], rtol=0, atol=1e-6)
            assert ctrl.x_horizon.shape == (11, 4) and ctrl.u_horizon.shape == (10, 2)
            assert (ctrl.term_set_A[:, -4:] @ ctrl.x_horizon[-1] - ctrl.term_set_b).max() <= VIOL_TOL
        if np.all(np.abs(plant.state - ctrl.goal) <= 1e-1) or step > 30 / DT_SIMULATION:
            break
        step += 1
    assert step + 1 == len(g["states"]) == 152


@pytest.mark.parametrize("name,N", [("RoadEnv", 10), ("RoadMultipleCarsEnv", 20)])
def test_statefb_step_side_effects_on_cpu(name, N):
    """MPCStateFB.step's side-effect attributes (mpc.py:341-347) against the reference formulas
    evaluated at the golden optimum: x_horizon, u_horizon, terminal_cost (absolute x_N), stage_cost."""
    from carmpc_amd.environments import ENVIRONMENTS
    from carmpc_amd.mpc import MPCStateFB
    asm = oa.build(name, N, terminal_set_dir=TERMINAL_SETS)
    g = np.load(os.path.join(GOLDEN, f"qp_{name}_N{N}.npz"))
    c = MPCStateFB(0.2, N, [0, 0, 0, 3], [0, 0], env=ENVIRONMENTS[name](), terminal_set_dir=TERMINAL_SETS, device="cpu")
    for i in np.where(g["status"] == 0)[0][:6]:
        x0, us = g["x0"][i], g["u_star"][i]
        u0 = c.step(x0)
        np.testing.assert_allclose(u0, us[:2], rtol=0, atol=U_TOL)
        np.testing.assert_allclose(c.u_horizon, us.reshape(-1, 2), rtol=0, atol=U_TOL)
        np.testing.assert_allclose(c.x_horizon, (asm.T @ x0 + asm.S @ us).reshape(-1, 4), rtol=0, atol=1e-6)
        tc, sc = terminal_cost(asm, x0, us), stage_cost(asm, x0, us, oa.STAGE_COST_Q, oa.STAGE_COST_R)
        assert abs(c.terminal_cost - tc) <= 1e-7 * max(1.0, abs(tc))
        assert abs(c.stage_cost - sc) <= 1e-7 * max(1.0, abs(sc))


def test_outputfb_and_disturbance_controllers_on_cpu():
    """MPCOutputFB.step (mpc.py:450-492) and MPCOutputFBWithDisturbance.step (mpc.py:614-667) with
    the host observer forms and the CPU QP, against the oracle step by step."""
    from carmpc_amd.environments import RoadMultipleCarsEnv
    from carmpc_amd.mpc import MPCOutputFB, MPCOutputFBWithDisturbance
    from carmpc_amd.simulator import CarSimulator
    asm = oa.build("RoadMultipleCarsEnv", 20, terminal_set_dir=TERMINAL_SETS)
    env = RoadMultipleCarsEnv()
    start = [5, -1.5, 0, 0]
    c = MPCOutputFB(0.2, 20, [0, 0, 0, 3], [0, 0], init_state=start, env=env, terminal_set_dir=TERMINAL_SETS,
                    device="cpu")
    sim = CarSimulator(dt=0.2, C=c.C)
    sim.reset(np.array(start, float))
    xhat, u = np.array(start, float), np.zeros(2)
    for _ in range(12):
        sim.step(u)
        xhat = oa.luenberger_observer(asm.A, asm.B, xhat, u, sim.output)
        r = oq.solve_instance(asm, xhat, oa.optimal_target_selection(asm.A, asm.B, oa.C_OUT @ asm.goal)[0])
        u = c.step(sim.output)
        assert r["status"] == 0 and np.abs(u - r["u_exact"][:2]).max() <= U_TOL
        np.testing.assert_allclose(c.x_estimate, xhat, rtol=0, atol=1e-9)
        j_ref = objective(asm, xhat, r["u_exact"], asm.goal)                 # MPCOutputFB.cost (mpc.py:478, 487)
        assert abs(c.cost - j_ref) <= OBJ_RTOL * max(1.0, abs(j_ref))
        u = r["u_exact"][:2]
        c.previous_u = u.copy()
    cd = MPCOutputFBWithDisturbance(0.2, 20, [0, 0, 0, 3], [0, 0], start, env=env, terminal_set_dir=TERMINAL_SETS,
                                    device="cpu")
    y = np.array([5.02, -1.49, 0.01])
    xe, de = oa.disturbance_observer(asm.A, asm.B, np.array(start, float), 0.0, np.zeros(2), y)
    r = oq.solve_instance_dist(asm, xe, de)
    if r["status"] == 0:
        assert np.abs(cd.step(y) - r["u_exact"][:2]).max() <= U_TOL
        assert abs(cd.d_estimate - de) <= 1e-12


def test_example_script_runs_config1_without_gpu():
    """examples/run_MPCStateFB.py --env RoadEnv --horizon 10 in a process that sees no GPU."""
    out = subprocess.run([sys.executable, "run_MPCStateFB.py", "--env", "RoadEnv", "--horizon", "10", "--start", "22",
                          "0", "0", "3", "--no-plot"], cwd=os.path.join(REPO, "examples"), capture_output=True, text=True,
                         env={**os.environ, "CUDA_VISIBLE_DEVICES": "", "HIP_VISIBLE_DEVICES": "", "MPLBACKEND": "Agg"},
                         timeout=600)
    assert out.returncode == 0, out.stderr[-2000:]
    assert "steps 152" in out.stdout
