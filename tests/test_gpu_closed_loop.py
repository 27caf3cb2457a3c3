"""GPU parity of the device closed loop (carmpc_closed_loop_batch) against
the CPU restatement of the examples' runner loops (oracle/closed_loop.py).

Per instance: identical outcome (reached / infeasible / time-out ...) and step count, final
plant state and observer estimate within 1e-6 (the QP inputs agree to 1e-6 with the oracle's
KKT point, and the runner stops on exact thresholds; no start below sits within that distance
of a threshold)."""
import numpy as np
import pytest

from conftest import TERMINAL_SETS

pytestmark = pytest.mark.gpu

X_TOL = 1e-6


def _controller(kind, start=(5.0, -1.5, 0.0, 0.0), kernel=0, **flags):
    from carmpc_amd.configuration import DT_CONTROL, LINEARIZE_INPUT, LINEARIZE_STATE, N
    from carmpc_amd.environments import ENVIRONMENTS
    from carmpc_amd.qp import SolverSettings
    from lib.mpc import MPCOutputFB, MPCOutputFBWithDisturbance, MPCStateFB
    env = ENVIRONMENTS["RoadMultipleCarsEnv"]()
    if kind == 0:
        c = MPCStateFB(dt=DT_CONTROL, N=N, lin_state=LINEARIZE_STATE, lin_input=LINEARIZE_INPUT, env=env,
                       terminal_set_dir=TERMINAL_SETS, **flags)
    elif kind == 1:
        c = MPCOutputFB(dt=DT_CONTROL, N=N, lin_state=LINEARIZE_STATE, lin_input=LINEARIZE_INPUT,
                        init_state=list(start), env=env, terminal_set_dir=TERMINAL_SETS)
    else:
        c = MPCOutputFBWithDisturbance(DT_CONTROL, N, LINEARIZE_STATE, LINEARIZE_INPUT, list(start), env=env,
                                       terminal_set_dir=TERMINAL_SETS)
    if kind != 2:
        c.set_goal(env.goal)   # as the runners do
    c.settings = SolverSettings(kernel=kernel)
    return c


def _asm():
    from oracle import assembly as oa
    return oa.build("RoadMultipleCarsEnv", 20, terminal_set_dir=TERMINAL_SETS)


def _starts(n, seed):
    rng = np.random.default_rng(seed)
    s = np.column_stack([rng.uniform(0, 25, n), rng.uniform(-2.8, 2.8, n), rng.uniform(-0.3, 0.3, n),
                         rng.uniform(0, 5, n)])
    return np.vstack([[5.0, -1.5, 0.1, 0.0], [5.0, -1.5, 0.0, 0.0], s])


def _compare(res, refs, check_xhat=False):
    for b, r in enumerate(refs):
        assert int(res["outcome"][b]) == r["outcome"], (b, int(res["outcome"][b]), r["outcome"])
        assert int(res["steps"][b]) == r["steps"], (b, int(res["steps"][b]), r["steps"])
        np.testing.assert_allclose(res["state"][b], r["state"], rtol=0, atol=X_TOL, err_msg=str(b))
        if check_xhat:
            np.testing.assert_allclose(res["xhat"][b], r["xhat"], rtol=0, atol=X_TOL, err_msg=str(b))


@pytest.mark.parametrize("kernel", [0, 1, 2])
def test_state_feedback_loop(gpu_available, kernel):
    """run_MPCStateFB.py runner for 66 cars vs the oracle loop (C restatement of the IPM)."""
    from carmpc_amd.closed_loop import run_closed_loop
    from oracle import closed_loop as ocl
    asm = _asm()
    starts = _starts(64, 3)
    res = run_closed_loop(_controller(0, kernel=kernel), starts)
    solve = ocl.c_solver(asm, threads=8)
    refs = [ocl.run(asm, s, mode=0, last_step=151, goal_tol=0.1, solve=solve) for s in starts]
    assert refs[0]["outcome"] == ocl.REACHED and refs[0]["steps"] == 52   # the example's start
    outcomes = {r["outcome"] for r in refs}
    assert ocl.REACHED in outcomes and ocl.INFEASIBLE in outcomes
    _compare(res, refs)


def test_state_feedback_loop_without_input_constraint(gpu_available):
    """input_constraint=False: the QP's inputs leave the actuator range.  The reference's
    check_input compares Python lists (simulator.py:92-95), so only inputs ABOVE the upper
    limits stop a run; hard braking below -2.05 m/s^2 keeps driving."""
    from carmpc_amd.closed_loop import run_closed_loop
    from oracle import assembly as oa
    from oracle import closed_loop as ocl
    asm = oa.build("RoadMultipleCarsEnv", 20, terminal_set_dir=TERMINAL_SETS, input_constraint_on=False)
    rng = np.random.default_rng(21)
    n = 24
    starts = np.column_stack([rng.uniform(0, 29, n), rng.uniform(-2.8, 2.8, n), rng.uniform(-0.3, 0.3, n),
                              rng.uniform(0, 5, n)])
    starts = np.vstack([[27.0, 1.0, 0.0, 4.5], [29.0, 1.5, 0.0, 4.0], [5.0, -1.5, 0.0, 0.0], starts])
    base = ocl.c_solver(asm, threads=8)
    refs, braked = [], []
    for s0 in starts:
        amin = [0.0]

        def solve(x0, xr, d):
            st, u = base(x0, xr, d)
            if st == 0:
                amin[0] = min(amin[0], u[0])
            return st, u
        refs.append(ocl.run(asm, s0, mode=0, last_step=151, goal_tol=0.1, solve=solve))
        braked.append(amin[0] < -2.05 and refs[-1]["steps"] > 2)
    assert any(braked)                                              # ran on after an input below the range
    assert any(r["outcome"] == ocl.INPUT_VIOLATION for r in refs)   # stopped by one above it
    res = run_closed_loop(_controller(0, input_constraint=False), starts)
    _compare(res, refs)


def test_output_feedback_loop(gpu_available):
    """run_MPCOutputFB.py runner (Luenberger observer on device) for 18 cars."""
    from carmpc_amd.closed_loop import run_closed_loop
    from oracle import closed_loop as ocl
    asm = _asm()
    starts = _starts(16, 5)
    res = run_closed_loop(_controller(1), starts)
    solve = ocl.c_solver(asm, threads=8)
    refs = [ocl.run(asm, s, mode=1, last_step=75, goal_tol=0.0, solve=solve) for s in starts]
    assert refs[1]["outcome"] == ocl.TIMEOUT and refs[1]["steps"] == 76   # the example runs 76 steps
    _compare(res, refs, check_xhat=True)


def test_disturbance_loop(gpu_available):
    """Disturbance-observer output feedback in the same runner (numpy oracle, 6 cars)."""
    from carmpc_amd.closed_loop import run_closed_loop
    from oracle import closed_loop as ocl
    asm = _asm()
    starts = _starts(4, 9)
    res = run_closed_loop(_controller(2), starts)
    refs = [ocl.run(asm, s, mode=2, last_step=75, goal_tol=0.0) for s in starts]
    _compare(res, refs, check_xhat=True)
    for b, r in enumerate(refs):
        assert abs(res["dhat"][b] - r["dhat"]) <= X_TOL


def test_loop_matches_host_runner(gpu_available):
    """batch = 1 device loop == the example's own Python loop through lib.mpc + lib.simulator."""
    from carmpc_amd.closed_loop import run_closed_loop
    from carmpc_amd.configuration import DT_SIMULATION
    from lib.simulator import CarSimulator
    start = [5.0, -1.5, 0.1, 0.0]
    ctrl = _controller(0)
    sim = CarSimulator(dt=DT_SIMULATION)
    sim.reset(np.array(start))
    u = [0, 0]
    i = 0
    while True:
        sim.step(u)
        u = ctrl.step(sim.state)
        if np.all(np.abs(sim.state - ctrl.goal) <= 1e-1) or i > 30 / DT_SIMULATION:
            break
        i += 1
    res = run_closed_loop(_controller(0), [start])
    assert int(res["outcome"][0]) == 0 and int(res["steps"][0]) == i + 1
    np.testing.assert_allclose(res["state"][0], sim.state, rtol=0, atol=X_TOL)


def test_region_of_attraction_grid(gpu_available):
    """Paper-style grid search (4096 starts in one batched run): spot-check 24 cells against
    the oracle loop, and the outcome grid is independent of the solve kernel."""
    from carmpc_amd.closed_loop import region_of_attraction
    from oracle import closed_loop as ocl
    xs, ys = np.linspace(0.0, 28.0, 64), np.linspace(-2.9, 2.9, 64)
    roa = region_of_attraction(_controller(0), xs, ys, psi=0.0, v=2.0)
    assert roa["outcome"].shape == (64, 64)
    assert (roa["outcome"] >= 0).all()
    roa2 = region_of_attraction(_controller(0, kernel=2), xs, ys, psi=0.0, v=2.0)
    np.testing.assert_array_equal(roa["outcome"], roa2["outcome"])
    np.testing.assert_array_equal(roa["steps"], roa2["steps"])
    asm = _asm()
    solve = ocl.c_solver(asm, threads=8)
    rng = np.random.default_rng(1)
    for flat in rng.choice(64 * 64, 24, replace=False):
        iy, ix = divmod(int(flat), 64)
        r = ocl.run(asm, [xs[ix], ys[iy], 0.0, 2.0], mode=0, last_step=151, goal_tol=0.1, solve=solve)
        assert int(roa["outcome"][iy, ix]) == r["outcome"], (iy, ix)
        assert int(roa["steps"][iy, ix]) == r["steps"], (iy, ix)
