"""carmpc_solve_segments: several problems in one call, launches forked onto side streams and
joined back.  Concurrent and serial launching give bitwise-identical results,
equal to per-problem solves, and the call is ordered on the caller's stream."""
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


def test_concurrent_equals_serial_equals_single(gpu_available):
    import torch
    from carmpc_amd import _native
    from carmpc_amd.qp import solve_segments
    probs = _problems()
    counts = [3001, 1, 2500]
    offsets = np.concatenate([[0], np.cumsum(counts)])
    X = torch.as_tensor(_states(int(offsets[-1]), 1)).cuda()
    lib = _native.load()
    try:
        lib.carmpc_set_serial_segments(0)
        u_c, s_c, i_c = solve_segments(probs, offsets, X)
        lib.carmpc_set_serial_segments(1)
        u_s, s_s, i_s = solve_segments(probs, offsets, X)
    finally:
        lib.carmpc_set_serial_segments(0)
    torch.cuda.synchronize()
    assert torch.equal(u_c, u_s) and torch.equal(s_c, s_s) and torch.equal(i_c, i_s)
    for j, p in enumerate(probs):
        sl = slice(int(offsets[j]), int(offsets[j + 1]))
        u1, s1, _ = p.solve(X[sl])
        assert torch.equal(s1, s_c[sl])
        assert torch.equal(u1, u_c[sl, :p.n])


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
