"""GPU: the drop-in controller API (lib.mpc / carmpc_amd.mpc) in the reference's closed loops.

run_MPCStateFB (examples/run_MPCStateFB.py:29-41) and run_MPCOutputFB
(examples/run_MPCOutputFB.py:29-43) with the controller's QP on the GPU, checked against
the oracle-driven golden trace and the oracle itself step by step."""
import os
import subprocess
import sys

import numpy as np
import pytest

from conftest import GOLDEN, REPO, TERMINAL_SETS

pytestmark = pytest.mark.gpu


def test_statefb_closed_loop_matches_golden(gpu_available):
    from carmpc_amd.environments import RoadMultipleCarsEnv
    from carmpc_amd.mpc import MPCStateFB
    from carmpc_amd.simulator import CarSimulator
    g = np.load(os.path.join(GOLDEN, "closed_loop_statefb.npz"))
    env = RoadMultipleCarsEnv()
    c = MPCStateFB(0.2, 20, [0, 0, 0, 3], [0, 0], env=env, terminal_set_dir=TERMINAL_SETS)
    c.set_goal(env.goal)
    sim = CarSimulator(dt=0.2)
    sim.reset(np.array([5, -1.5, 0.1, 0]))
    u = [0, 0]
    for i in range(len(g["states"])):
        sim.step(u)
        np.testing.assert_allclose(sim.state, g["states"][i], atol=1e-6)
        u = c.step(sim.state)
        np.testing.assert_allclose(u, g["inputs"][i], atol=1e-6)
        assert c.x_horizon.shape == (21, 4) and c.u_horizon.shape == (20, 2)
        # predicted terminal state inside the terminal set (terminal-set feasibility)
        tA, tb = c.term_set_A[:, -4:], c.term_set_b
        assert (tA @ c.x_horizon[-1] - tb).max() <= 1e-8
    assert np.all(np.abs(sim.state - c.goal) <= 1e-1)


def test_statefb_infeasible_start_raises(gpu_available):
    """Configuration 1 (run_MPCStateFB, RoadEnv, N=10): the example's start state is infeasible at N=10."""
    from carmpc_amd.environments import RoadEnv
    from carmpc_amd.mpc import MPCStateFB, OutsideTheRegionOfAttractionError
    c = MPCStateFB(0.2, 10, [0, 0, 0, 3], [0, 0], env=RoadEnv(), terminal_set_dir=TERMINAL_SETS)
    with pytest.raises(OutsideTheRegionOfAttractionError):
        c.step(np.array([5, -1.5, 0.1, 0]))
    u = c.step(np.array([22, 0, 0, 3.0]))       # feasible start (config 1 plumbing)
    assert u.shape == (2,)


def test_outputfb_closed_loop_against_oracle(gpu_available):
    from oracle import assembly as oa
    from oracle import qp as oq
    from carmpc_amd.environments import RoadMultipleCarsEnv
    from carmpc_amd.mpc import MPCOutputFB
    from carmpc_amd.simulator import CarSimulator
    env = RoadMultipleCarsEnv()
    start = [5, -1.5, 0, 0]
    c = MPCOutputFB(0.2, 20, [0, 0, 0, 3], [0, 0], init_state=start, env=env, terminal_set_dir=TERMINAL_SETS)
    c.set_goal(env.goal)
    asm = oa.build("RoadMultipleCarsEnv", 20, terminal_set_dir=TERMINAL_SETS)
    sim = CarSimulator(dt=0.2, C=c.C)
    sim.reset(np.array(start))
    u, xh, up = [0, 0], np.array(start, float), np.zeros(2)
    for i in range(76):
        sim.step(u)
        xh_ref = oa.luenberger_observer(asm.A, asm.B, xh, up, sim.output)
        u = c.step(sim.output)
        np.testing.assert_allclose(c.x_estimate, xh_ref, rtol=1e-12, atol=1e-10)
        r = oq.solve_instance(asm, c.x_estimate)
        assert r["status"] == 0
        ref = r["u_exact"] if r["certified"] else r["u"]
        np.testing.assert_allclose(u, ref[:2], atol=1e-6)
        xh, up = c.x_estimate.copy(), np.array(u)
    assert abs(sim.state[0] - 30) < 0.5 and abs(sim.state[1] - 1.5) < 0.1


def test_step_side_effect_costs(gpu_available):
    """terminal_cost (absolute x_N, mpc.py:344-345), stage_cost (mpc.py:347) of MPCStateFB.step and cost of
    MPCOutputFB.step (mpc.py:478, 487) on the GPU path, against the reference formulas at the golden optimum."""
    from costs import OBJ_RTOL, objective, stage_cost, terminal_cost
    from oracle import assembly as oa
    from oracle import qp as oq
    from carmpc_amd.environments import RoadMultipleCarsEnv
    from carmpc_amd.mpc import MPCOutputFB, MPCStateFB
    env = RoadMultipleCarsEnv()
    asm = oa.build("RoadMultipleCarsEnv", 20, terminal_set_dir=TERMINAL_SETS)
    g = np.load(os.path.join(GOLDEN, "qp_RoadMultipleCarsEnv_N20.npz"))
    c = MPCStateFB(0.2, 20, [0, 0, 0, 3], [0, 0], env=env, terminal_set_dir=TERMINAL_SETS)
    for i in np.where(g["status"] == 0)[0][:6]:
        x0, us = g["x0"][i], g["u_star"][i]
        c.step(x0)
        np.testing.assert_allclose(c.x_horizon, (asm.T @ x0 + asm.S @ us).reshape(-1, 4), rtol=0, atol=1e-6)
        tc, sc = terminal_cost(asm, x0, us), stage_cost(asm, x0, us, oa.STAGE_COST_Q, oa.STAGE_COST_R)
        assert abs(c.terminal_cost - tc) <= 1e-7 * max(1.0, abs(tc))
        assert abs(c.stage_cost - sc) <= 1e-7 * max(1.0, abs(sc))
    start = np.array([12.0, -1.0, 0.0, 2.0])
    co = MPCOutputFB(0.2, 20, [0, 0, 0, 3], [0, 0], init_state=start, env=env, terminal_set_dir=TERMINAL_SETS)
    y = oa.C_OUT @ start + np.array([0.02, -0.01, 0.03])
    xh = oa.luenberger_observer(asm.A, asm.B, start, np.zeros(2), y)
    r = oq.solve_instance(asm, xh)
    assert r["status"] == 0 and r["certified"]
    co.step(y)
    j_ref = objective(asm, xh, r["u_exact"])
    assert abs(co.cost - j_ref) <= OBJ_RTOL * max(1.0, abs(j_ref))


def test_step_batch_matches_scalar(gpu_available):
    from carmpc_amd.environments import RoadOneCarEnv
    from carmpc_amd.mpc import MPCStateFB
    c = MPCStateFB(0.2, 20, [0, 0, 0, 3], [0, 0], env=RoadOneCarEnv(), terminal_set_dir=TERMINAL_SETS)
    rng = np.random.default_rng(0)
    X = np.stack([rng.uniform(5, 29, 64), rng.uniform(-3, 3, 64), rng.uniform(-0.3, 0.3, 64),
                  rng.uniform(0, 4, 64)], axis=1)
    u0, u, st = c.step_batch(X)
    st = st.cpu().numpy()
    for i in np.where(st == 0)[0][:8]:
        np.testing.assert_array_equal(c.step(X[i]), u0[i].cpu().numpy())


def test_examples_run_headless(gpu_available):
    """The repository's example drivers (same loops as the reference's) run unchanged on the GPU."""
    for script in ("run_MPCStateFB.py", "run_MPCOutputFB.py"):
        out = subprocess.run([sys.executable, script], cwd=os.path.join(REPO, "examples"), capture_output=True,
                             text=True, timeout=600, env={**os.environ, "MPLBACKEND": "Agg", "CARMPC_NO_PLOT": "1"})
        assert out.returncode == 0, out.stderr[-2000:]
        assert "steps" in out.stdout
