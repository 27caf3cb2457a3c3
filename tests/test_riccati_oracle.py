"""The stage-form (Riccati) restatement of the IPM follows the dense oracle step for step.

oracle/riccati.py is the arithmetic of the grouped HIP kernel (ipm_riccati.hip): same
algorithm as oracle/qp.py::ipm, with M^{-1} applied by a backward Riccati
recursion + forward roll-out over the horizon instead of a dense Cholesky.
"""
import numpy as np
import pytest

from conftest import CONFIGS, GOLDEN, TERMINAL_SETS


@pytest.mark.parametrize("name,N", CONFIGS)
def test_riccati_oracle_golden(name, N):
    from oracle import assembly as oa
    from oracle import riccati as orc
    asm = oa.build(name, N, terminal_set_dir=TERMINAL_SETS)
    g = np.load(f"{GOLDEN}/qp_{name}_N{N}.npz")
    sq = orc.StageQP(asm)
    for i, x0 in enumerate(g["x0"][:32]):
        u, st, it = orc.ipm(sq, x0, asm.goal)
        assert st == g["status"][i]
        assert it == g["iters"][i]
        if st == 0:
            assert np.abs(u - g["u_star"][i]).max() <= 1e-8


def test_riccati_solve_matches_dense_normal_matrix():
    """M^{-1} b by the Riccati recursion == dense solve of M = H + G'DG + diag(box)."""
    from oracle import assembly as oa
    from oracle import riccati as orc
    asm = oa.build("RoadMultipleCarsEnv", 20, terminal_set_dir=TERMINAL_SETS)
    sq = orc.StageQP(asm)
    rng = np.random.default_rng(0)
    d = 10.0 ** rng.uniform(-6, 6, sq.p)
    dbox = 10.0 ** rng.uniform(-6, 6, sq.n)
    M = asm.H + (sq.Gn.T * d) @ sq.Gn + np.diag(dbox)
    M = 0.5 * (M + M.T)
    bu = rng.normal(size=sq.n)
    bx = np.zeros((sq.N + 1, 4))
    bx[1:] = rng.normal(size=(sq.N, 4))
    b = bu + sq.adjoint(bx)
    v, y = sq.riccati_solve(sq.riccati_factor(d, dbox), bu, bx)
    ref = np.linalg.solve(M, b)
    assert np.abs(v - ref).max() <= 1e-9 * (1 + np.abs(ref).max())
    assert np.allclose(y, sq.rollout(v), rtol=1e-12, atol=1e-12)


def test_riccati_oracle_random_vs_c_oracle():
    from oracle import assembly as oa
    from oracle import riccati as orc
    from oracle.cpu import CpuProblem
    asm = oa.build("RoadOneCarEnv", 20, terminal_set_dir=TERMINAL_SETS)
    sq = orc.StageQP(asm)
    rng = np.random.default_rng(3)
    B = 40
    gx = asm.goal[0]
    X = np.stack([rng.uniform(gx - 25, gx, B), rng.uniform(-3, 3, B), rng.uniform(-np.pi / 8, np.pi / 8, B),
                  rng.uniform(-1, 5, B)], axis=1)
    uc, sc, ic = CpuProblem(asm).solve(X)
    for i in range(B):
        u, st, it = orc.ipm(sq, X[i], asm.goal)
        assert st == sc[i] and it == ic[i]
        if st == 0:
            assert np.abs(u - uc[i]).max() <= 1e-9
