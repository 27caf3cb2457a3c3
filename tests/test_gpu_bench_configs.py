"""GPU: the BASELINE configurations at their full sizes, on bench.py's own seeded inputs.

Configuration 5's per-GPU shard (131,072 mixed Road* instances, the workload bench.py times):
status and u against the C oracle on a stratified sample, and -- on ALL optimal instances --
the size-independent properties: constraint violation <= 1e-8 with the un-normalised rows,
box, and terminal-set feasibility of the predicted x_N.  Configuration 4 (65,536 output-feedback
steps: observer kernel + QP) and configurations 3 and 2 likewise."""
import numpy as np
import pytest

from conftest import TERMINAL_SETS

pytestmark = pytest.mark.gpu

U_TOL = 1e-6
VIOL_TOL = 1e-8


def _check_all(asm, X, u, st):
    """Feasibility properties on every optimal instance of one environment."""
    ok = st == 0
    Xo, uo = X[ok], u[ok]
    w = asm.w0[None, :] - Xo @ asm.E.T
    viol = (uo @ asm.G.T - w).max()
    assert viol <= VIOL_TOL, viol
    assert (uo - asm.ub[None]).max() <= VIOL_TOL and (asm.lb[None] - uo).max() <= VIOL_TOL
    xN = (Xo @ asm.T.T + uo @ asm.S.T)[:, -4:]
    tv = (xN @ asm.term_A[:, -4:].T - asm.term_b[None]).max()
    assert tv <= VIOL_TOL, tv                                   # terminal-set feasibility
    assert (st[~ok] == 1).all()                                 # everything else: certified infeasible


def _check_sample(asm, X, u, st, idx, xref=None):
    """Status and u against the C oracle; a few against the exact KKT optimum."""
    from oracle import qp as oq
    from oracle.cpu import CpuProblem
    xr = None if xref is None else np.ascontiguousarray(np.broadcast_to(xref, (len(idx), 4)))
    uc, sc, _ = CpuProblem(asm).solve(X[idx], xr, threads=8)
    agree = st[idx] == sc
    if not agree.all():
        Gn, w0n, En, keep, pw, pE = oq.normalize_rows(asm.G, asm.w0, asm.E)
        for i in idx[~agree]:       # only at the feasibility boundary
            assert abs(oq.lp_margin(Gn, w0n - En @ X[i], asm.lb, asm.ub)) < 1e-7, (i, st[i])
    both = (st[idx] == 0) & (sc == 0)
    assert both.sum() > len(idx) // 4
    assert np.abs(u[idx][both] - uc[both]).max() <= U_TOL
    from costs import OBJ_RTOL, objective_gap
    assert max(objective_gap(asm, X[i], u[i], uc[k], xref) for k, i in enumerate(idx) if both[k]) <= OBJ_RTOL
    for i in idx[both][:8]:
        r = oq.solve_instance(asm, X[i], xref)
        assert r["certified"] and np.abs(u[i] - r["u_exact"]).max() <= U_TOL
        assert objective_gap(asm, X[i], u[i], r["u_exact"], xref) <= OBJ_RTOL


def test_config5_bench_shard(gpu_available):
    import torch
    import bench
    from oracle import assembly as oa
    from carmpc_amd.qp import solve_segments
    ctrls = bench.build_controllers(bench.ENVS, 20, torch.device("cuda", 0))
    probs = [c.qp for c in ctrls]
    X, env, offsets = bench.sample_shard(0, bench.PER_GPU, [c.goal for c in ctrls])
    assert X.shape == (131072, 4)
    u, st, it = solve_segments(probs, offsets, torch.as_tensor(X).cuda())
    torch.cuda.synchronize()
    u, st, it = u.cpu().numpy(), st.cpu().numpy(), it.cpu().numpy()
    assert ((st == 0) | (st == 1)).all()                        # no iteration-limit / numerical stops
    rng = np.random.default_rng(0)
    for j, name in enumerate(bench.ENVS):
        asm = oa.build(name, 20, terminal_set_dir=TERMINAL_SETS)
        sl = slice(int(offsets[j]), int(offsets[j + 1]))
        _check_all(asm, X[sl], u[sl], st[sl])
        idx = np.sort(rng.choice(offsets[j + 1] - offsets[j], 1024, replace=False))     # 3 x 1024 stratified
        _check_sample(asm, X[sl], u[sl], st[sl], idx)
    # one call over the three segments == one carmpc_solve_batch per environment
    for j, p in enumerate(probs):
        sl = slice(int(offsets[j]), int(offsets[j + 1]))
        u1, st1, it1 = p.solve(torch.as_tensor(X[sl]).cuda())
        np.testing.assert_array_equal(st1.cpu().numpy(), st[sl])
        np.testing.assert_array_equal(it1.cpu().numpy(), it[sl])
        ok = st[sl] == 0
        np.testing.assert_allclose(u1.cpu().numpy()[ok], u[sl][ok], rtol=0, atol=1e-12)


def test_config4_outputfb_batch(gpu_available):
    """65,536 output-feedback steps (mpc.py:450-478): observer kernel, then the QP at the estimate."""
    import torch
    import bench
    from oracle import assembly as oa
    from carmpc_amd.mpc import MPCOutputFB
    asm = oa.build("RoadMultipleCarsEnv", 20, terminal_set_dir=TERMINAL_SETS)
    c = bench.build_controllers(("RoadMultipleCarsEnv",), 20, torch.device("cuda", 0))[0]
    B = 65536
    xt, xhat0, uprev, y = bench.sample_outputfb(0, B, c.goal)
    xh = torch.as_tensor(xhat0.copy()).cuda()
    c.qp.observe(torch.as_tensor(y).cuda(), xh, torch.as_tensor(uprev).cuda(), MPCOutputFB.C_OUT, MPCOutputFB.L_GAIN)
    xref = torch.as_tensor(np.tile(c.goal, (B, 1))).cuda()
    u, st, it = c.qp.solve(xh, xref)
    torch.cuda.synchronize()
    xhat = xh.cpu().numpy()
    ref = xhat0 @ asm.A.T + uprev @ asm.B.T + (y - xhat0 @ oa.C_OUT.T) @ oa.L_OBS.T        # mpc.py:448
    np.testing.assert_allclose(xhat, ref, rtol=0, atol=1e-12)
    u, st = u.cpu().numpy(), st.cpu().numpy()
    assert ((st == 0) | (st == 1)).all() and (st == 0).sum() > B // 4
    _check_all(asm, xhat, u, st)
    idx = np.sort(np.random.default_rng(4).choice(B, 1024, replace=False))
    _check_sample(asm, xhat, u, st, idx, xref=c.goal)


@pytest.mark.parametrize("workload,name,N,B", [("config3", "RoadOneCarEnv", 20, 65536), ("config2", "RoadEnv", 10, 4096)])
def test_config3_and_config2_batches(gpu_available, workload, name, N, B):
    import torch
    import bench
    from oracle import assembly as oa
    asm = oa.build(name, N, terminal_set_dir=TERMINAL_SETS)
    c = bench.build_controllers((name,), N, torch.device("cuda", 0))[0]
    X, _, _ = bench.sample_shard(0, B, [c.goal], seed={"config3": 3, "config2": 2}[workload])
    u, st, _ = c.qp.solve(torch.as_tensor(X).cuda())
    u, st = u.cpu().numpy(), st.cpu().numpy()
    assert ((st == 0) | (st == 1)).all()
    _check_all(asm, X, u, st)
    idx = np.sort(np.random.default_rng(3).choice(B, 1024, replace=False))
    _check_sample(asm, X, u, st, idx)
