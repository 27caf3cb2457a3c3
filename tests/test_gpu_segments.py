"""carmpc_solve_segments: several problems in one call.  Segments that share a kernel
instantiation are solved by one launch whose workgroups move between the problems; the results
equal per-problem solves (every instance is solved by one 16-lane group with the same arithmetic
whichever workgroup claims it), mixed horizons and kernels fall back to per-problem launches, and
the call is ordered on the caller's stream."""
import numpy as np
import pytest

from conftest import TERMINAL_SETS

pytestmark = pytest.mark.gpu

ENVS = ("RoadEnv", "RoadOneCarEnv", "RoadMultipleCarsEnv")


def _problems():
    from carmpc_amd.configuration import DT_CONTROL, LINEARIZE_INPUT, LINEARIZE_STATE
    from carmpc_amd.environments import ENVIRONMENTS
    from carmpc_amd.mpc import MPCStateFB
    return [MPCStateFB(dt=DT_CONTROL, N=20, lin_state=LINEARIZE_STATE, lin_input=LINEARIZE_INPUT,
                       env=ENVIRONMENTS[e](), terminal_set_dir=TERMINAL_SETS).qp for e in ENVS]


def _states(n, seed):
    rng = np.random.default_rng(seed)
    return np.column_stack([rng.uniform(0, 28, n), rng.uniform(-2.5, 2.5, n), rng.uniform(-0.3, 0.3, n),
                            rng.uniform(0, 4, n)])


def test_one_launch_equals_per_problem_solves(gpu_available):
    import torch
    from carmpc_amd.qp import SolverSettings, solve_segments
    probs = _problems()
    for counts in ([3001, 1, 2500], [40, 7000, 3], [5000, 0, 4000]):
        offsets = np.concatenate([[0], np.cumsum(counts)])
        X = torch.as_tensor(_states(int(offsets[-1]), 1)).cuda()
        u_c, s_c, i_c = solve_segments(probs, offsets, X)
        u_k, s_k, i_k = solve_segments(probs, offsets, X, settings=SolverSettings(kernel=2))   # per-problem launches
        torch.cuda.synchronize()
        assert torch.equal(s_c, s_k)
        for j, p in enumerate(probs):
            sl = slice(int(offsets[j]), int(offsets[j + 1]))
            u1, s1, i1 = p.solve(X[sl])
            assert torch.equal(s1, s_c[sl]) and torch.equal(i1, i_c[sl])
            ok = (s1 == 0)
            assert torch.equal(u1[ok], u_c[sl, :p.n][ok])
            assert float((u_k[sl, :p.n][ok] - u1[ok]).abs().max()) <= 1e-6 if bool(ok.any()) else True


def test_mixed_horizons_and_many_segments(gpu_available):
    """N = 10 and N = 20 problems in one call (different instantiations: separate launches) and more
    segments than one launch carries."""
    import torch
    from carmpc_amd.configuration import DT_CONTROL, LINEARIZE_INPUT, LINEARIZE_STATE
    from carmpc_amd.environments import ENVIRONMENTS
    from carmpc_amd.mpc import MPCStateFB
    from carmpc_amd.qp import solve_segments
    p20 = _problems()
    p10 = MPCStateFB(dt=DT_CONTROL, N=10, lin_state=LINEARIZE_STATE, lin_input=LINEARIZE_INPUT,
                     env=ENVIRONMENTS["RoadEnv"](), terminal_set_dir=TERMINAL_SETS).qp
    probs = [p20[0], p20[1], p10, p20[2], p20[0], p20[1], p20[2], p20[0]]
    counts = [300, 200, 500, 100, 250, 1, 350, 299]
    offsets = np.concatenate([[0], np.cumsum(counts)])
    x = _states(int(offsets[-1]), 7)
    x[offsets[2]:offsets[3], 0] = np.random.default_rng(2).uniform(22, 30, 500)     # feasible range at N = 10
    X = torch.as_tensor(x).cuda()
    u, st, it = solve_segments(probs, offsets, X)
    torch.cuda.synchronize()
    assert u.shape[1] == 40
    for j, p in enumerate(probs):
        sl = slice(int(offsets[j]), int(offsets[j + 1]))
        u1, s1, i1 = p.solve(X[sl])
        assert torch.equal(s1, st[sl]) and torch.equal(i1, it[sl])
        ok = s1 == 0
        assert torch.equal(u1[ok], u[sl, :p.n][ok])


def test_stream_ordering_on_side_stream(gpu_available):
    """Called on a user stream, the results are complete once that stream is synchronised,
    including when x0 is written on the same stream right before the call."""
    import torch
    from carmpc_amd.qp import solve_segments
    probs = _problems()
    offsets = np.array([0, 1000, 2000, 3000])
    Xh = torch.as_tensor(_states(3000, 2))
    ref_u, ref_s, _ = solve_segments(probs, offsets, Xh.cuda())
    torch.cuda.synchronize()
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        X = torch.zeros((3000, 4), dtype=torch.float64, device="cuda")
        X.copy_(Xh.cuda(non_blocking=True))
        u, st, _ = solve_segments(probs, offsets, X, stream=s)
        done = torch.cuda.Event()
        done.record(s)
    done.synchronize()
    assert torch.equal(u, ref_u) and torch.equal(st, ref_s)


def test_empty_segments(gpu_available):
    import torch
    from carmpc_amd.qp import solve_segments
    probs = _problems()
    X = torch.as_tensor(_states(10, 3)).cuda()
    u, st, _ = solve_segments(probs, [0, 0, 10, 10], X)
    u2, st2, _ = probs[1].solve(X)
    torch.cuda.synchronize()
    assert torch.equal(st, st2) and torch.equal(u[:, :probs[1].n], u2)


@pytest.mark.parametrize("case", ["first_offset_positive", "leading_other_horizon", "six_segments"])
def test_pipeline_runs_that_do_not_start_at_instance_zero(gpu_available, case):
    """Runs of segments large enough for the three-launch form (49,152 instances and more) whose first
    instance is not row 0 of the call: a positive first offset, a run behind a segment of another
    horizon, and the second run of a call with more segments than one launch carries.  The hand-off
    and retry lists of such a run begin at the run's first instance."""
    import torch
    from carmpc_amd.configuration import DT_CONTROL, LINEARIZE_INPUT, LINEARIZE_STATE
    from carmpc_amd.environments import ENVIRONMENTS
    from carmpc_amd.mpc import MPCStateFB
    from carmpc_amd.qp import solve_segments
    p20 = _problems()
    if case == "first_offset_positive":
        probs, offsets = [p20[1], p20[2]], np.array([5000, 33000, 61000])
    elif case == "leading_other_horizon":
        p10 = MPCStateFB(dt=DT_CONTROL, N=10, lin_state=LINEARIZE_STATE, lin_input=LINEARIZE_INPUT,
                         env=ENVIRONMENTS["RoadEnv"](), terminal_set_dir=TERMINAL_SETS).qp
        probs, offsets = [p10, p20[0], p20[2]], np.array([0, 3000, 30000, 56000])
    else:
        probs = [p20[0], p20[1], p20[2], p20[0], p20[1], p20[2]]
        offsets = np.concatenate([[0], np.cumsum([2500, 2500, 2500, 2500, 26000, 26000])])
    B = int(offsets[-1]) + 100                     # rows beyond the last offset belong to no segment
    X = torch.as_tensor(_states(B, 21)).cuda()
    u = torch.full((B, 40), -7.0, dtype=torch.float64, device="cuda")
    st = torch.full((B,), -7, dtype=torch.int32, device="cuda")
    it = torch.full((B,), -7, dtype=torch.int32, device="cuda")
    solve_segments(probs, offsets, X, out=(u, st, it))
    torch.cuda.synchronize()
    outside = np.ones(B, bool)
    outside[int(offsets[0]):int(offsets[-1])] = False
    outside = torch.as_tensor(outside).cuda()
    assert bool((st[outside] == -7).all()) and bool((u[outside] == -7.0).all())     # nothing written outside the segments
    for j, p in enumerate(probs):
        sl = slice(int(offsets[j]), int(offsets[j + 1]))
        u1, s1, i1 = p.solve(X[sl])
        torch.cuda.synchronize()
        bad = ((s1 != st[sl]) | (i1 != it[sl])).nonzero().flatten()
        assert bad.numel() == 0, (case, j, bad[:8].tolist(), s1[bad[:8]].tolist(), st[sl][bad[:8]].tolist(),
                                  i1[bad[:8]].tolist(), it[sl][bad[:8]].tolist(), int(bad.numel()))
        ok = s1 == 0
        assert int(ok.sum()) > 0
        assert float((u1[ok] - u[sl, :p.n][ok]).abs().max()) <= 1e-12


def test_host_pipeline_equals_resident_solve(gpu_available):
    """States in host memory, results to host memory, copies overlapped with the solve chunk by chunk
    (carmpc_amd.qp.HostPipeline): same statuses, iteration counts and inputs as one call on resident data,
    for the default split and for chunks that cut through segments; repeated calls reuse the buffers."""
    import torch
    from carmpc_amd.qp import HostPipeline, solve_segments
    probs = _problems()
    counts = [30000, 41000, 27304]
    offsets = np.concatenate([[0], np.cumsum(counts)])
    B = int(offsets[-1])
    X = _states(B, 33)
    u0, s0, i0 = solve_segments(probs, offsets, torch.as_tensor(X).cuda())
    torch.cuda.synchronize()
    u0, s0, i0 = u0.cpu().numpy(), s0.cpu().numpy(), i0.cpu().numpy()
    ok = s0 == 0
    for chunks in (None, [50000, 20000, 28304]):
        hp = HostPipeline(probs, offsets, chunks)
        for rep in range(2):
            u, st, it = hp.solve(X)
            np.testing.assert_array_equal(st.numpy(), s0)
            np.testing.assert_array_equal(it.numpy(), i0)
            np.testing.assert_allclose(u.numpy()[ok], u0[ok], rtol=0, atol=1e-12)
    # only the first input of every sequence back to the host (what the reference's step() returns, mpc.py:349)
    hp = HostPipeline(probs, offsets, depth=1, first_action=True)
    u, st, it = hp.solve(X)
    assert u.shape == (B, 2)
    np.testing.assert_array_equal(st.numpy(), s0)
    np.testing.assert_allclose(u.numpy()[ok], u0[ok][:, :2], rtol=0, atol=1e-12)
    # a sequence of batches with two in flight: batch k's results are those of batch k's states
    hp = HostPipeline(probs, offsets, depth=2)
    Xs = [X, X[::-1].copy(), X]                 # (the reversed batch puts other states under each problem)
    refs = []
    for Xk in Xs[:2]:
        r = solve_segments(probs, offsets, torch.as_tensor(Xk).cuda())
        torch.cuda.synchronize()
        refs.append([t.cpu().numpy() for t in r])
    refs.append(refs[0])
    tickets = [hp.submit(Xs[0]), hp.submit(Xs[1])]
    for k in range(3):
        u, st, it = hp.wait(tickets[k])
        np.testing.assert_array_equal(st.numpy(), refs[k][1])
        np.testing.assert_array_equal(it.numpy(), refs[k][2])
        okk = refs[k][1] == 0
        np.testing.assert_allclose(u.numpy()[okk], refs[k][0][okk], rtol=0, atol=1e-12)
        if k == 0:
            tickets.append(hp.submit(Xs[2]))
    u1, s1, i1 = probs[1].solve_host(X[:5000])
    u2, s2, i2 = probs[1].solve(torch.as_tensor(X[:5000]).cuda())
    np.testing.assert_array_equal(s1, s2.cpu().numpy())
    np.testing.assert_allclose(u1[s1 == 0], u2.cpu().numpy()[s1 == 0], rtol=0, atol=1e-12)
