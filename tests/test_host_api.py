"""Host-side mirror of the reference API (lib/*): constructor setup, constraint stacks,
constants, environments, plant and the drop-in import paths.  CPU only: no QP is solved
here (the product has no CPU solve path; that is asserted too)."""
import json
import os
import subprocess
import sys

import numpy as np
import pytest

from conftest import CONFIGS, GOLDEN, REPO, TERMINAL_SETS

from oracle import assembly as oa


def _ctrl(name, N, cls="MPCStateFB", **kw):
    from carmpc_amd import environments, mpc
    env = environments.ENVIRONMENTS[name]()
    lin_state = kw.pop("lin_state", [0, 0, 0, 3])
    if cls == "MPCOutputFB":
        return mpc.MPCOutputFB(0.2, N, lin_state, [0, 0], [5, -1.5, 0, 0], env=env,
                               terminal_set_dir=TERMINAL_SETS, **kw)
    return getattr(mpc, cls)(0.2, N, lin_state, [0, 0], env=env, terminal_set_dir=TERMINAL_SETS, **kw)


@pytest.mark.parametrize("name,N", CONFIGS)
def test_constructor_matches_reference_constructor(name, N):
    """Host mirror of MPC.__init__ against the dump of the reference's own constructor and
    constraint builders (tests/golden/assembly_*.npz, tools/make_golden.py)."""
    c = _ctrl(name, N)
    g = np.load(os.path.join(GOLDEN, f"assembly_{name}_N{N}.npz"))
    np.testing.assert_array_equal(c.A, g["A"])
    np.testing.assert_array_equal(c.B, g["B"])
    np.testing.assert_allclose(c.P, g["P"], rtol=1e-13, atol=0)
    np.testing.assert_allclose(c.K, g["K"], rtol=1e-12, atol=1e-14)
    np.testing.assert_array_equal(c.goal, g["goal"])
    np.testing.assert_array_equal(c.input_upper, g["input_upper"])
    np.testing.assert_array_equal(c.input_lower, g["input_lower"])
    for fn, key in ((c.terminal_constraint, "term"), (c.input_constraint, "input"), (c.state_constraint, "state")):
        A, b = fn()
        np.testing.assert_array_equal(A, g[key + "_A"])
        np.testing.assert_array_equal(b, g[key + "_b"])


def test_constructor_fallback_matches_reference(tmp_path):
    from carmpc_amd import environments, mpc
    meta = json.load(open(os.path.join(GOLDEN, "meta.json")))
    g = np.load(os.path.join(GOLDEN, "assembly_fallback_RoadEnv_N10.npz"))
    env = environments.RoadEnv()
    env.goal = list(meta["fallback_goal"])
    c = mpc.MPCStateFB(0.2, 10, [0, 0, 0, 3], [0, 0], env=env, terminal_set_dir=str(tmp_path))
    A, b = c.terminal_constraint()
    np.testing.assert_array_equal(A, g["term_A"])
    np.testing.assert_array_equal(b, g["term_b"])
    np.testing.assert_array_equal(c.goal, g["goal"])


@pytest.mark.parametrize("name,N", CONFIGS)
def test_constructor_matches_oracle(name, N):
    c = _ctrl(name, N)
    asm = oa.build(name, N, terminal_set_dir=TERMINAL_SETS)
    np.testing.assert_array_equal(c.A, asm.A)
    np.testing.assert_array_equal(c.B, asm.B)
    np.testing.assert_allclose(c.P, asm.P, rtol=1e-13)
    np.testing.assert_allclose(c.K, asm.K, rtol=1e-12)
    np.testing.assert_array_equal(c.goal, asm.goal)
    A, b = c.terminal_constraint()
    np.testing.assert_array_equal(A, asm.term_A)
    np.testing.assert_array_equal(b, asm.term_b)
    A, b = c.input_constraint()
    Ar, br = oa.input_constraint(N, 2, asm.input_upper, asm.input_lower)
    np.testing.assert_array_equal(A, Ar)
    np.testing.assert_array_equal(b, br)
    A, b = c.state_constraint()
    Ar, br = oa.state_constraint(N, 4, asm.state_rows_A, asm.state_rows_b)
    np.testing.assert_array_equal(A, Ar)
    np.testing.assert_array_equal(b, br)


def test_set_goal_equilibrium_assert():
    c = _ctrl("RoadEnv", 10)
    c.set_goal([30, 1.5, 0, 0])
    with pytest.raises(AssertionError):
        c.set_goal([30, 1.5, 0.1, 0])      # psi != 0 is not an equilibrium (mpc.py:190)
    with pytest.raises(AssertionError):
        c.set_goal([1, 2, 3])


def test_output_fb_target_and_observer_host_forms():
    c = _ctrl("RoadMultipleCarsEnv", 20, cls="MPCOutputFB")
    x_ref, u_ref = c.optimal_target_selection()
    np.testing.assert_allclose(x_ref, [30, 1.5, 0, 0], atol=1e-12)
    np.testing.assert_allclose(u_ref, [0, 0], atol=1e-12)
    y = np.array([5.1, -1.4, 0.2])
    ref = oa.luenberger_observer(c.A, c.B, np.array([5, -1.5, 0, 0.0]), np.zeros(2), y)
    np.testing.assert_allclose(c.luenberger_observer(y), ref, rtol=1e-15)
    np.testing.assert_array_equal(c.C, oa.C_OUT)
    np.testing.assert_array_equal(c.L, oa.L_OBS)
    # the reference's own method on seeded tuples (mpc.py:439-448)
    g = np.load(os.path.join(GOLDEN, "observer.npz"))
    np.testing.assert_array_equal(c.y_goal, g["y_goal"])
    for i in range(len(g["y0"])):
        c.x_estimate, c.previous_u = g["x_estimate"][i].copy(), g["previous_u"][i].copy()
        np.testing.assert_allclose(c.luenberger_observer(g["y0"][i]), g["next"][i], rtol=0, atol=1e-13)


def test_target_selection_with_a_family_of_steady_states():
    """The reference's target-selection QP (mpc.py:413-437) when its equalities leave freedom: min x'Qx + u'Ru
    over the admissible steady states that reach y_goal.  Checked against scipy's SLSQP on the same QP:
    (a) the bicycle linearised at standstill (v = 0: heading and steering drop out of the equalities, the cost
    sets them to zero), (b) a synthetic output map that measures only x and v, so that y, psi, delta are free
    and a state row y >= 2 is active at the optimum."""
    from scipy.optimize import minimize
    from carmpc_amd import mpc as m

    def slsqp(Hd, M, rhs, A_in, b_in):
        # (SLSQP wants independent equality rows: the row space of M, with the consistent right-hand side)
        _u, sv, vt = np.linalg.svd(M)
        rank = int((sv > 1e-10 * sv.max()).sum())
        z_p = np.linalg.lstsq(M, rhs, rcond=None)[0]
        M, rhs = vt[:rank], vt[:rank] @ z_p
        res = minimize(lambda z: z @ Hd @ z, np.zeros(6), jac=lambda z: 2 * Hd @ z, method="SLSQP",
                       constraints=[{"type": "eq", "fun": lambda z: M @ z - rhs, "jac": lambda z: M},
                                    {"type": "ineq", "fun": lambda z: b_in - A_in @ z, "jac": lambda z: -A_in}],
                       options={"ftol": 1e-14, "maxiter": 500})
        assert res.success
        return res.x

    c = _ctrl("RoadMultipleCarsEnv", 20, cls="MPCOutputFB")
    Hd = np.block([[c.Q, np.zeros((4, 2))], [np.zeros((2, 4)), c.R]])
    A_s, b_s = np.asarray(c.state_const_A, float), np.asarray(c.state_const_b, float)
    A_in = np.block([[A_s, np.zeros((len(b_s), 2))], [np.zeros((2, 4)), np.eye(2)], [np.zeros((2, 4)), -np.eye(2)]])
    b_in = np.concatenate((b_s, c.input_upper, -np.asarray(c.input_lower)))
    # (a) standstill linearisation
    c0 = _ctrl("RoadMultipleCarsEnv", 20, cls="MPCOutputFB", lin_state=[0, 0, 0, 0.0])
    M0 = np.block([[np.eye(4) - c0.A, -c0.B], [c0.C, np.zeros((3, 2))]])
    assert np.linalg.matrix_rank(M0) < 6
    x_ref, u_ref = c0.optimal_target_selection()
    ref = slsqp(Hd, M0, np.concatenate((np.zeros(4), c0.y_goal)), A_in, b_in)
    np.testing.assert_allclose(np.concatenate((x_ref, u_ref)), ref, atol=1e-6)
    np.testing.assert_allclose(x_ref, [30, 1.5, 0, 0], atol=1e-9)
    # (b) outputs x and v only, with an extra admissible-state row y >= 2
    C2 = np.array([[1.0, 0, 0, 0], [0, 0, 0, 1.0]])
    M2 = np.block([[np.eye(4) - c.A, -c.B], [C2, np.zeros((2, 2))]])
    rhs2 = np.concatenate((np.zeros(4), [30.0, 0.0]))
    A2 = np.vstack((A_in, [[0, -1.0, 0, 0, 0, 0]]))
    b2 = np.concatenate((b_in, [-2.0]))
    z = m._target_qp(Hd, M2, rhs2, A2, b2)
    np.testing.assert_allclose(z, slsqp(Hd, M2, rhs2, A2, b2), atol=1e-6)
    assert abs(z[1] - 2.0) <= 1e-9 and abs(z[2]) <= 1e-9           # the row is active, the free heading is zero
    # inconsistent constraints: y >= 2 against the road's y <= ... at a goal outside
    assert m._target_qp(Hd, M2, rhs2, np.vstack((A2, [[0, 1.0, 0, 0, 0, 0]])), np.concatenate((b2, [1.0]))) is None


def test_lqr_path():
    c = _ctrl("RoadMultipleCarsEnv", 20, cls="MPC", use_LQR=True)
    x0 = np.array([5, -1.5, 0, 0.0])
    u = c.step(x0)
    np.testing.assert_allclose(u, np.clip(c.K @ (x0 - c.goal), c.input_lower, c.input_upper))
    with pytest.raises(NotImplementedError):
        _ctrl("RoadEnv", 10, cls="MPC").step(x0)


def test_matrix_gen_mirror_matches_reference_outputs():
    from carmpc_amd import matrix_gen as mg
    for name, N in CONFIGS:
        g = np.load(os.path.join(GOLDEN, f"assembly_{name}_N{N}.npz"))
        T, S = mg.predmod(g["A"], g["B"], N)
        np.testing.assert_allclose(T, g["T"], rtol=0, atol=1e-13)   # powers of A by a different product order
        np.testing.assert_allclose(S, g["S"], rtol=0, atol=1e-13)
        H, h, const = mg.costgen(oa.STAGE_COST_Q, oa.STAGE_COST_R, g["P"], T, S, 4)
        np.testing.assert_allclose(H, g["H"], rtol=1e-13, atol=1e-10)
        np.testing.assert_allclose(h, g["h"], rtol=1e-13, atol=1e-10)
        np.testing.assert_allclose(const, g["const"], rtol=1e-13, atol=1e-9)


def test_simulator_mirror_matches_reference():
    from carmpc_amd.simulator import CarSimulator
    g = np.load(os.path.join(GOLDEN, "plant.npz"))
    for s0, u, nxt in zip(g["state"], g["u"], g["next"]):
        sim = CarSimulator(dt=0.2)
        sim.reset(np.array(s0))
        log = sim.step(u)
        np.testing.assert_array_equal(sim.state, nxt)     # same numpy expression -> same bits
        np.testing.assert_array_equal(log["inputs"], u)
    sim = CarSimulator(dt=0.2)
    with pytest.raises(AssertionError):
        sim.step([2.1, 0.0])                               # simulator.py:92-93
    with pytest.raises(AssertionError):
        sim.step([0.0, 1.0])
    # outside the limits: same outcome as the reference's check_input, whose list comparison
    # (simulator.py:92-95) only rejects inputs above the upper limits
    for s0, u, raised, nxt in zip(g["oob_state"], g["oob_u"], g["oob_raised"], g["oob_next"]):
        sim = CarSimulator(dt=0.2)
        sim.reset(np.array(s0))
        if raised:
            with pytest.raises(AssertionError):
                sim.step(u)
        else:
            sim.step(u)
        np.testing.assert_array_equal(sim.state, nxt)
    clipped = CarSimulator(dt=0.2, clip=True).check_input([5.0, -2.0])
    np.testing.assert_allclose(clipped, [2.05, -np.pi / 4 - 0.05])


def test_environments_mirror():
    meta = json.load(open(os.path.join(GOLDEN, "meta.json")))
    from carmpc_amd import environments as E
    for name, e in meta["environments"].items():
        env = E.ENVIRONMENTS[name]()
        assert env.name == name and list(env.goal) == e["goal"]
        np.testing.assert_array_equal(np.asarray(env.constraints_A, float), np.asarray(e["constraints_A"]))
        np.testing.assert_array_equal(np.asarray(env.constraints_b, float), np.asarray(e["constraints_b"]))
        assert env.lim == [tuple(x) for x in e["lim"]]


def test_configuration_mirror():
    meta = json.load(open(os.path.join(GOLDEN, "meta.json")))["configuration"]
    import carmpc_amd.configuration as C
    assert C.DT_CONTROL == meta["DT_CONTROL"] and C.N == meta["N"] and C.STEPS_UPDATE == meta["STEPS_UPDATE"]
    np.testing.assert_array_equal(C.STAGE_COST_Q, np.asarray(meta["Q"]))


def test_dropin_import_paths_and_cpu_path_without_gpu():
    """`from lib.mpc import MPCStateFB` works from the repo root and from examples/ (cwd-relative
    terminal sets); in a process that sees no GPU the controller solves on the CPU QP path, as the
    reference's controllers do."""
    code = ("import sys, numpy as np; sys.path.insert(0, 'examples'); "
            "from lib.mpc import MPCStateFB, OutsideTheRegionOfAttractionError; "
            "from lib.environments import RoadMultipleCarsEnv; from lib.configuration import *; "
            "from lib.simulator import CarSimulator; from lib.visualize_state import plot_live; "
            "from lib.matrix_gen import predmod, costgen; "
            "import carmpc_amd; e = RoadMultipleCarsEnv(); "
            "c = MPCStateFB(dt=DT_CONTROL, N=N, lin_state=LINEARIZE_STATE, lin_input=LINEARIZE_INPUT, env=e); "
            "c.set_goal(e.goal)\n"
            "u = c.step(np.array([5, -1.5, 0.1, 0]))\nprint('SOLVED', c.on_cpu, repr(u.tolist()))\n")
    out = subprocess.run([sys.executable, "-c", code], cwd=os.path.join(REPO, "examples"), capture_output=True,
                         text=True, env={**os.environ, "PYTHONPATH": REPO, "CUDA_VISIBLE_DEVICES": "",
                                         "HIP_VISIBLE_DEVICES": "", "MPLBACKEND": "Agg"}, timeout=300)
    assert out.returncode == 0, out.stderr
    assert "Using ../terminal_sets/RoadMultipleCarsEnv_30_1.5_0_0.npy" in out.stdout
    line = [ln for ln in out.stdout.splitlines() if ln.startswith("SOLVED")][0]
    assert line.split()[1] == "True"                      # no GPU visible -> CPU path
    u = np.array(eval(line.split(" ", 2)[2]))
    g = np.load(os.path.join(GOLDEN, "closed_loop_statefb.npz"))
    # first controller step of the golden trace solves the QP at plant(start, u = 0)
    from oracle import qp as oq
    asm = oa.build("RoadMultipleCarsEnv", 20, terminal_set_dir=TERMINAL_SETS)
    r = oq.solve_instance(asm, np.array([5, -1.5, 0.1, 0]))
    np.testing.assert_allclose(u, r["u_exact"][:2], rtol=0, atol=1e-6)
