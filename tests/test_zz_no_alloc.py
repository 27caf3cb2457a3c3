"""carmpc_solve_batch_noalloc (the entry point for callers that cannot allocate) against
carmpc_solve_batch, through the C ABI: same kernels, the claim counter in the library's static
device scratch instead of a stream-ordered allocation.

Two calls in a row on one stream, the second with a smaller batch (the scratch keeps the first
call's count until the second call clears it); every output must equal carmpc_solve_batch's:
status and iteration counts exactly, u to 1e-12 (each instance is solved by one 16-lane group with
the same arithmetic whichever group claims it; the tolerance of the parity suite is 1e-6)."""
import ctypes

import numpy as np
import pytest

from conftest import TERMINAL_SETS

pytestmark = pytest.mark.gpu


def _x0(rng, goal_x, B):
    return np.stack([rng.uniform(goal_x - 25, goal_x, B), rng.uniform(-3, 3, B),
                     rng.uniform(-np.pi / 8, np.pi / 8, B), rng.uniform(-1, 5, B)], axis=1)


def _call(fn, qp, X, settings):
    import torch
    from carmpc_amd import _native
    B = X.shape[0]
    u = torch.full((B, qp.n), float("nan"), dtype=torch.float64, device=qp.device)
    st = torch.full((B,), -1, dtype=torch.int32, device=qp.device)
    it = torch.full((B,), -1, dtype=torch.int32, device=qp.device)
    s = settings.c()
    stream = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    with torch.cuda.device(qp.device):
        rc = fn(qp._h, B, ctypes.c_void_p(X.data_ptr()), None, ctypes.c_void_p(u.data_ptr()),
                ctypes.c_void_p(st.data_ptr()), ctypes.c_void_p(it.data_ptr()), ctypes.byref(s), stream)
    _native.check(rc, fn.__name__)
    return u, st, it


@pytest.mark.parametrize("kernel", [0, 1, 2])
def test_noalloc_matches_solve_batch(gpu_available, kernel):
    import torch
    from oracle import assembly as oa
    from carmpc_amd import _native
    from carmpc_amd.qp import QPProblem, SolverSettings
    lib = _native.load()
    asm = oa.build("RoadMultipleCarsEnv", 20, terminal_set_dir=TERMINAL_SETS)
    qp = QPProblem(N=20, A=asm.A, B=asm.B, Q=oa.STAGE_COST_Q, R=oa.STAGE_COST_R, P=asm.P, goal=asm.goal,
                   state_A=np.asarray(asm.state_rows_A, float), state_b=np.asarray(asm.state_rows_b, float),
                   term_A=asm.term_A[:, -4:], term_b=asm.term_b, u_lower=asm.input_lower, u_upper=asm.input_upper)
    settings = SolverSettings(kernel=kernel)
    rng = np.random.default_rng(77)
    for B in (3001, 517):                     # two calls in a row, the second smaller
        X = torch.as_tensor(_x0(rng, asm.goal[0], B)).to(qp.device)
        u1, st1, it1 = _call(lib.carmpc_solve_batch_noalloc, qp, X, settings)
        u0, st0, it0 = _call(lib.carmpc_solve_batch, qp, X, settings)
        torch.cuda.synchronize()
        assert torch.equal(st1, st0) and torch.equal(it1, it0)
        assert int((st0 == 0).sum()) > B // 4 and int((st0 == 1).sum()) > 0
        ok = (st0 == 0).cpu().numpy()
        np.testing.assert_allclose(u1.cpu().numpy()[ok], u0.cpu().numpy()[ok], rtol=0, atol=1e-12)
    # beyond the stated maximum: a clear error, nothing launched
    rc = lib.carmpc_solve_batch_noalloc(qp._h, (1 << 30) + 1, ctypes.c_void_p(X.data_ptr()), None,
                                        ctypes.c_void_p(u1.data_ptr()), ctypes.c_void_p(st1.data_ptr()), None, None, None)
    assert rc == -2 and b"CARMPC_NOALLOC_MAX_BATCH" in lib.carmpc_last_error()


def _qp_multi():
    from oracle import assembly as oa
    from carmpc_amd.qp import QPProblem
    asm = oa.build("RoadMultipleCarsEnv", 20, terminal_set_dir=TERMINAL_SETS)
    return asm, QPProblem(N=20, A=asm.A, B=asm.B, Q=oa.STAGE_COST_Q, R=oa.STAGE_COST_R, P=asm.P, goal=asm.goal,
                          state_A=np.asarray(asm.state_rows_A, float), state_b=np.asarray(asm.state_rows_b, float),
                          term_A=asm.term_A[:, -4:], term_b=asm.term_b, u_lower=asm.input_lower, u_upper=asm.input_upper)


def test_noalloc_takes_no_device_memory(gpu_available):
    """Free device memory (hipMemGetInfo) is the same before and after calls of the entry point:
    nothing is allocated, by the call or by a pool on its behalf.  Outputs are allocated before the
    first reading; the caching allocator of torch is not touched in between."""
    import torch
    from carmpc_amd import _native
    from carmpc_amd.qp import SolverSettings
    lib = _native.load()
    asm, qp = _qp_multi()
    B = 20000
    X = torch.as_tensor(_x0(np.random.default_rng(3), asm.goal[0], B)).to(qp.device)
    u = torch.empty((B, qp.n), dtype=torch.float64, device=qp.device)
    st = torch.empty((B,), dtype=torch.int32, device=qp.device)
    it = torch.empty((B,), dtype=torch.int32, device=qp.device)
    s = SolverSettings().c()
    stream = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    args = (qp._h, B, ctypes.c_void_p(X.data_ptr()), None, ctypes.c_void_p(u.data_ptr()), ctypes.c_void_p(st.data_ptr()),
            ctypes.c_void_p(it.data_ptr()), ctypes.byref(s), stream)
    torch.cuda.synchronize()
    free0, _ = torch.cuda.mem_get_info()
    for _ in range(3):
        with torch.cuda.device(qp.device):
            _native.check(lib.carmpc_solve_batch_noalloc(*args), "carmpc_solve_batch_noalloc")
        torch.cuda.synchronize()
        assert torch.cuda.mem_get_info()[0] == free0
    assert int((st == 0).sum()) > B // 4


def test_noalloc_in_a_hip_graph(gpu_available):
    """The stated use: the call recorded into a HIP graph (stream capture) and replayed.  Every
    replay -- with eager work and synchronisations of the program in between, and with new inputs
    written into the captured buffers -- equals carmpc_solve_batch on the same inputs."""
    import torch
    from carmpc_amd import _native
    from carmpc_amd.qp import SolverSettings
    lib = _native.load()
    asm, qp = _qp_multi()
    B = 4096
    rng = np.random.default_rng(9)
    settings = SolverSettings()
    X = torch.as_tensor(_x0(rng, asm.goal[0], B)).to(qp.device)
    u = torch.full((B, qp.n), float("nan"), dtype=torch.float64, device=qp.device)
    st = torch.full((B,), -1, dtype=torch.int32, device=qp.device)
    it = torch.full((B,), -1, dtype=torch.int32, device=qp.device)
    s = settings.c()
    side = torch.cuda.Stream()
    graph = torch.cuda.CUDAGraph()
    torch.cuda.synchronize()
    with torch.cuda.graph(graph, stream=side):
        with torch.cuda.device(qp.device):
            rc = lib.carmpc_solve_batch_noalloc(qp._h, B, ctypes.c_void_p(X.data_ptr()), None, ctypes.c_void_p(u.data_ptr()),
                                                ctypes.c_void_p(st.data_ptr()), ctypes.c_void_p(it.data_ptr()),
                                                ctypes.byref(s), ctypes.c_void_p(torch.cuda.current_stream().cuda_stream))
    _native.check(rc, "carmpc_solve_batch_noalloc under capture")
    assert int((st == -1).sum()) == B                      # capture records, it does not run
    for rep in range(4):
        if rep:
            X.copy_(torch.as_tensor(_x0(rng, asm.goal[0], B)))
        u.fill_(float("nan")); st.fill_(-1); it.fill_(-1)
        torch.cuda.synchronize()
        graph.replay()
        torch.cuda.synchronize()
        u0, st0, it0 = _call(lib.carmpc_solve_batch, qp, X, settings)      # eager work between the replays
        torch.cuda.synchronize()
        assert torch.equal(st, st0) and torch.equal(it, it0), rep
        ok = (st0 == 0).cpu().numpy()
        assert ok.sum() > B // 4
        np.testing.assert_allclose(u.cpu().numpy()[ok], u0.cpu().numpy()[ok], rtol=0, atol=1e-12)
