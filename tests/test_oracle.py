"""The oracle against the golden vectors produced from the reference (CPU only).

Pins (see tests/golden/meta.json, tools/make_golden.py):
  * constructor (A, B, P, K, T, S, H, h, terminal rows, constraint stacks) == what the
    reference's own lib/mpc.py::MPCStateFB.__init__ and its terminal_constraint() /
    input_constraint() / state_constraint() produce, including the missing-file fallback;
  * observers == the reference's own luenberger_observer methods on seeded tuples;
  * environments / configuration == the reference's objects and constants;
  * terminal-set data == the reference's terminal_sets/*.npy;
  * plant == the reference's lib/simulator.CarSimulator on seeded pairs, and its check_input
    outcome (raised / not raised) on inputs outside the limits;
  * QP solutions: KKT-certified optimum (parity vs cvxpy itself is unpinned: absent).
"""
import json
import os

import numpy as np
import pytest

from conftest import CONFIGS, GOLDEN, REPO, TERMINAL_SETS

from oracle import assembly as oa
from oracle import qp as oq


def _meta():
    with open(os.path.join(GOLDEN, "meta.json")) as f:
        return json.load(f)


def _check_against_reference_constructor(asm, g):
    """asm (oracle restatement) against a dump of the reference's constructor and builders."""
    N = asm.N
    np.testing.assert_array_equal(asm.A, g["A"])
    np.testing.assert_array_equal(asm.B, g["B"])
    np.testing.assert_allclose(asm.P, g["P"], rtol=1e-13, atol=0)     # same LAPACK call (mpc.py:70)
    np.testing.assert_allclose(asm.K, g["K"], rtol=1e-12, atol=1e-14)
    np.testing.assert_allclose(asm.T, g["T"], rtol=0, atol=1e-14)   # BLAS rounding only
    np.testing.assert_allclose(asm.S, g["S"], rtol=0, atol=1e-14)
    np.testing.assert_allclose(asm.H, g["H"], rtol=1e-14, atol=1e-11)
    np.testing.assert_allclose(asm.h, g["h"], rtol=1e-14, atol=1e-11)
    np.testing.assert_array_equal(asm.goal, g["goal"])
    np.testing.assert_array_equal(asm.input_upper, g["input_upper"])
    np.testing.assert_array_equal(asm.input_lower, g["input_lower"])
    # the three stacks, exactly as the reference's builders return them (mpc.py:196-253)
    np.testing.assert_array_equal(asm.term_A, g["term_A"])
    np.testing.assert_array_equal(asm.term_b, g["term_b"])
    iA, ib = oa.input_constraint(N, 2, asm.input_upper, asm.input_lower)
    np.testing.assert_array_equal(iA, g["input_A"])
    np.testing.assert_array_equal(ib, g["input_b"])
    sA, sb = oa.state_constraint(N, 4, asm.state_rows_A, asm.state_rows_b)
    np.testing.assert_array_equal(sA, g["state_A"])
    np.testing.assert_array_equal(sb, g["state_b"])
    # condensed rows G u <= w0 - E x0: the reference's stacks composed with ITS T and S
    # (x = T x0 + S u, mpc.py:319; order terminal, then state: mpc.py:323-332)
    A_all = np.vstack((g["term_A"], g["state_A"]))
    np.testing.assert_allclose(asm.G, A_all @ g["S"], rtol=0, atol=1e-12)
    np.testing.assert_allclose(asm.E, A_all @ g["T"], rtol=0, atol=1e-12)
    np.testing.assert_array_equal(asm.w0, np.hstack((g["term_b"], g["state_b"])))
    np.testing.assert_array_equal(asm.ub, g["input_b"][:2 * N])
    np.testing.assert_array_equal(asm.lb, -g["input_b"][2 * N:])


@pytest.mark.parametrize("name,N", CONFIGS)
def test_assembly_matches_reference_constructor(name, N):
    g = np.load(os.path.join(GOLDEN, f"assembly_{name}_N{N}.npz"))
    asm = oa.build(name, N, terminal_set_dir=TERMINAL_SETS)
    _check_against_reference_constructor(asm, g)
    np.testing.assert_array_equal(asm.term_A[:, -4:], g["term"][:, :4])
    np.testing.assert_array_equal(asm.term_b, g["term"][:, 4])
    # DARE fixed point (mpc.py:70)
    A, B, P, Q, R = asm.A, asm.B, asm.P, oa.STAGE_COST_Q, oa.STAGE_COST_R
    res = A.T @ P @ A - P - A.T @ P @ B @ np.linalg.solve(R + B.T @ P @ B, B.T @ P @ A) + Q
    assert np.abs(res).max() < 1e-9
    assert abs(P[0, 0] - 60.13) < 5e-3 and abs(P[2, 2] - 843.30) < 5e-3


def test_fallback_matches_reference_constructor(tmp_path):
    """No terminal-set file for the goal -> the reference's goal box (mpc.py:107-117)."""
    g = np.load(os.path.join(GOLDEN, "assembly_fallback_RoadEnv_N10.npz"))
    goal = _meta()["fallback_goal"]
    asm = oa.build("RoadEnv", 10, terminal_set_dir=str(tmp_path), goal=goal)
    assert asm.term_file is None and g["term_A"].shape == (8, 44)
    _check_against_reference_constructor(asm, g)


def test_observer_restatements_match_reference_methods():
    """oracle luenberger_observer / disturbance_observer against the reference's own methods
    (mpc.py:439-448, 598-612) and their constants (mpc.py:387-404, 530-546)."""
    g = np.load(os.path.join(GOLDEN, "observer.npz"))
    np.testing.assert_array_equal(oa.C_OUT, g["C"])
    np.testing.assert_array_equal(oa.L_OBS, g["L"])
    np.testing.assert_array_equal(oa.BD_DIST, g["Bd"])
    np.testing.assert_array_equal(oa.CD_DIST, g["Cd"])
    np.testing.assert_array_equal(oa.L1_DIST, g["L1"])
    np.testing.assert_array_equal(oa.L2_DIST, g["L2"])
    asm = oa.build("RoadMultipleCarsEnv", 20, terminal_set_dir=TERMINAL_SETS)
    np.testing.assert_array_equal(oa.C_OUT @ asm.goal, g["y_goal"])
    for i in range(len(g["y0"])):
        x = oa.luenberger_observer(asm.A, asm.B, g["x_estimate"][i], g["previous_u"][i], g["y0"][i])
        np.testing.assert_allclose(x, g["next"][i], rtol=0, atol=1e-13)
        xd, dd = oa.disturbance_observer(asm.A, asm.B, g["x_estimate"][i], g["d_estimate"][i], g["previous_u"][i],
                                         g["y0"][i])
        np.testing.assert_allclose(xd, g["next_dist_x"][i], rtol=0, atol=1e-13)
        np.testing.assert_allclose(dd, g["next_dist_d"][i], rtol=0, atol=1e-13)


def test_environment_and_configuration_data():
    meta = _meta()
    for name, (rows, rhs, goal) in oa.ENVIRONMENTS.items():
        e = meta["environments"][name]
        np.testing.assert_array_equal(np.asarray(rows, float), np.asarray(e["constraints_A"]))
        np.testing.assert_array_equal(np.asarray(rhs, float), np.asarray(e["constraints_b"]))
        assert list(goal) == e["goal"]
    c = meta["configuration"]
    assert c["DT_CONTROL"] == oa.DT_CONTROL and c["N"] == oa.N_HORIZON
    assert c["LINEARIZE_STATE"] == oa.LINEARIZE_STATE and c["LINEARIZE_INPUT"] == oa.LINEARIZE_INPUT
    np.testing.assert_array_equal(np.asarray(c["Q"]), oa.STAGE_COST_Q)
    np.testing.assert_array_equal(np.asarray(c["R"]), oa.STAGE_COST_R)


def test_terminal_set_files_are_reference_copies():
    # byte-identical copies of the reference data
    import hashlib
    want = {"RoadEnv_30_1.5_0_0.npy": "b8e85fd87a9d03968feeb45884bce20f",
            "RoadMultipleCarsEnv_30_1.5_0_0.npy": "e51cd11d0a547780b53b624cc09eeacf",
            "RoadOneCarEnv_29.9_-1.5_0_0.npy": "19e967d9a5804a3ed5251c0699e112e6"}
    for f, h in want.items():
        with open(os.path.join(TERMINAL_SETS, f), "rb") as fh:
            assert hashlib.md5(fh.read()).hexdigest() == h
    assert oa.terminal_set_filename("RoadOneCarEnv", [29.9, -1.5, 0, 0]) == "RoadOneCarEnv_29.9_-1.5_0_0.npy"


def test_terminal_fallback_box(tmp_path):
    asm = oa.build("RoadEnv", 10, terminal_set_dir=str(tmp_path))
    assert asm.term_file is None and asm.term_A.shape == (8, 44)
    np.testing.assert_array_equal(asm.term_A[:4, -4:], np.diag([1, 1, 1, 0]))
    np.testing.assert_array_equal(asm.term_b, np.hstack((asm.goal, -asm.goal)))


@pytest.mark.parametrize("name,N", CONFIGS)
def test_numpy_ipm_against_golden(name, N):
    g = np.load(os.path.join(GOLDEN, f"qp_{name}_N{N}.npz"))
    asm = oa.build(name, N, terminal_set_dir=TERMINAL_SETS)
    for i in range(0, 64, 4):
        r = oq.solve_instance(asm, g["x0"][i])
        assert r["status"] == g["status"][i]
        assert r["iters"] == g["iters"][i]
        if r["status"] == 0:
            assert np.abs(r["u"] - g["u_star"][i]).max() <= 1e-8
        assert (g["margin"][i] >= 0) == (g["status"][i] == 0)


@pytest.mark.parametrize("name,N", CONFIGS)
def test_c_oracle_against_golden(name, N):
    from oracle.cpu import CpuProblem
    g = np.load(os.path.join(GOLDEN, f"qp_{name}_N{N}.npz"))
    asm = oa.build(name, N, terminal_set_dir=TERMINAL_SETS)
    u, st, it = CpuProblem(asm).solve(g["x0"], threads=2)
    np.testing.assert_array_equal(st, g["status"])
    np.testing.assert_array_equal(it, g["iters"])
    ok = st == 0
    assert np.abs(u[ok] - g["u_star"][ok]).max() <= 1e-8


def test_c_oracle_status_against_lp_ground_truth():
    """Box-Farkas infeasibility certificates and optimal statuses agree with HiGHS."""
    from oracle.cpu import CpuProblem
    asm = oa.build("RoadOneCarEnv", 20, terminal_set_dir=TERMINAL_SETS)
    rng = np.random.default_rng(123)
    B = 400
    X = np.stack([rng.uniform(4.9, 29.9, B), rng.uniform(-3, 3, B), rng.uniform(-np.pi / 8, np.pi / 8, B),
                  rng.uniform(-1, 5, B)], axis=1)
    u, st, it = CpuProblem(asm).solve(X, threads=2)
    Gn, w0n, En, keep, pw, pE = oq.normalize_rows(asm.G, asm.w0, asm.E)
    for i in range(B):
        pre = pw - pE @ X[i]
        if pre.size and pre.min() < -oq.PRE_TOL:
            assert st[i] == 1
            continue
        m = oq.lp_margin(Gn, w0n - En @ X[i], asm.lb, asm.ub)
        if abs(m) > 1e-7:
            assert (st[i] == 0) == (m > 0), (i, st[i], m)
    assert (st == 2).sum() == 0


def test_plant_restatement_matches_reference_simulator():
    from oracle import closed_loop as ocl
    g = np.load(os.path.join(GOLDEN, "plant.npz"))
    for s, u, nxt in zip(g["state"], g["u"], g["next"]):
        np.testing.assert_allclose(oa.plant_step(s, u), nxt, rtol=0, atol=1e-14)
        assert not ocl.input_bad(u)
    # inputs outside the limits: the reference's check_input compares lists lexicographically
    # (simulator.py:92-95), so only inputs above the UPPER limits raise
    assert g["oob_raised"].sum() == 10 and len(g["oob_raised"]) == 30
    for s, u, raised, nxt in zip(g["oob_state"], g["oob_u"], g["oob_raised"], g["oob_next"]):
        assert ocl.input_bad(u) == bool(raised), u
        if not raised:
            np.testing.assert_allclose(oa.plant_step(s, u), nxt, rtol=0, atol=1e-14)


def test_closed_loop_statefb_reproduces_golden_trace():
    """examples/run_MPCStateFB.py loop (RoadMultipleCarsEnv, N=20, start [5,-1.5,0.1,0]) with the
    oracle QP reaches the goal tolerance in 52 steps, as recorded from the reference plant."""
    g = np.load(os.path.join(GOLDEN, "closed_loop_statefb.npz"))
    asm = oa.build("RoadMultipleCarsEnv", 20, terminal_set_dir=TERMINAL_SETS)
    state, u = np.array([5, -1.5, 0.1, 0.0]), np.zeros(2)
    for i in range(len(g["states"])):
        state = oa.plant_step(state, u)
        np.testing.assert_allclose(state, g["states"][i], atol=1e-7)
        r = oq.solve_instance(asm, state)
        assert r["status"] == 0
        u = r["u_exact"][:2] if r["certified"] else r["u"][:2]
    assert np.all(np.abs(state - asm.goal) <= 1e-1)


def test_goal_box_fallback_equality_pairs(tmp_path):
    """Without a terminal-set file the reference constrains x_N to the goal box written as
    opposite row pairs (mpc.py:107-117): an equality with no strict interior.  The pairs are
    detected and the polish re-splits their multipliers, so every instance is solved and
    KKT-certified (before: iteration limit on ~1% of them)."""
    from oracle.cpu import CpuProblem
    asm = oa.build("RoadEnv", 10, terminal_set_dir=str(tmp_path))
    Gn, w0n, En, keep, pw, pE = oq.normalize_rows(asm.G, asm.w0, asm.E)
    partner = oq.opposite_pairs(Gn, w0n, En)
    paired = np.where(partner >= 0)[0]
    assert len(paired) == 6 and np.array_equal(partner[partner[paired]], paired)
    np.testing.assert_array_equal(Gn[paired], -Gn[partner[paired]])
    rng = np.random.default_rng(10)
    X = np.stack([rng.uniform(28, 30, 200), rng.uniform(1, 2, 200), rng.uniform(-0.05, 0.05, 200),
                  rng.uniform(-0.2, 0.2, 200)], axis=1)
    u, st, it = CpuProblem(asm).solve(X, threads=2)
    assert (st == 0).all() and it.max() <= 20
    for i in range(0, 200, 25):
        r = oq.solve_instance(asm, X[i])
        assert r["status"] == 0 and r["certified"] and r["iters"] == it[i]
        assert np.abs(r["u_exact"] - u[i]).max() <= 1e-8
    # the reference's own terminal sets have no such pairs
    for name, N in CONFIGS:
        a = oa.build(name, N, terminal_set_dir=TERMINAL_SETS)
        G2, w2, E2, *_ = oq.normalize_rows(a.G, a.w0, a.E)
        assert (oq.opposite_pairs(G2, w2, E2) < 0).all()
