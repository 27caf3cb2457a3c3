"""Batched condensed-QP problems on the GPU (thin wrapper over the C ABI).

One ``QPProblem`` = one environment / horizon / linearisation point, i.e. the
data ``MPC.__init__`` builds (lib/mpc.py:22-117).  Solving replaces the
per-step ``cp.Problem(...).solve()`` of lib/mpc.py:334-335 and 477-478 for a
whole batch of states at once.  torch-ROCm tensors are used only as device
buffers; all arithmetic runs in the HIP kernels of ``csrc/``.
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass

import numpy as np
import torch

from . import _native
from ._native import CarMPCNativeError, ModelDesc, Settings, check

NX = 4


def _dptr(a: np.ndarray | None):
    if a is None:
        return None
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_double))


def _f64(a) -> np.ndarray | None:
    if a is None:
        return None
    return np.ascontiguousarray(np.asarray(a, dtype=np.float64))


def _tptr(t: torch.Tensor | None):
    return None if t is None else ctypes.c_void_p(t.data_ptr())


def _stream_handle(stream: torch.cuda.Stream | None):
    s = stream if stream is not None else torch.cuda.current_stream()
    return ctypes.c_void_p(s.cuda_stream)


def require_gpu(device=None) -> torch.device:
    if not torch.cuda.is_available():
        raise CarMPCNativeError("this entry point needs a ROCm GPU (torch.cuda.is_available() is False); "
                                "only the per-step QP has a CPU path (carmpc_amd.qp.CpuQPProblem)")
    dev = torch.device("cuda", torch.cuda.current_device()) if device is None else torch.device(device)
    return dev


@dataclass
class SolverSettings:
    """carmpc_settings; defaults match oracle/qp.py."""
    tol: float = 1e-10
    tol_mu: float = 1e-12
    max_iter: int = 60
    #: 0 auto (grouped Riccati, else staged, else dense), 1 dense, 2 staged, 3 dense 4-wave,
    #: 4-6 staged A/B variants, 7 grouped Riccati
    kernel: int = 0

    def c(self) -> Settings:
        return Settings(self.tol, self.tol_mu, self.max_iter, self.kernel)


class QPProblem:
    """Device-resident condensed QP of one linear-MPC configuration.

        min 1/2 u'Hu + (h (x0 - xref))'u
        s.t. G u <= w0 - E x0   (terminal rows on x_N, state rows on x_1..x_N)
             lb <= u <= ub      (input box, optional)
    """

    def __init__(self, *, N: int, A, B, Q, R, P, goal, state_A=None, state_b=None, term_A=None, term_b=None,
                 u_lower=None, u_upper=None, device=None):
        self.device = require_gpu(device)
        lib = _native.load()
        A, B, Q, R, P, goal = (_f64(v) for v in (A, B, Q, R, P, goal))
        nu = B.shape[1]
        sA = _f64(state_A if state_A is not None else np.zeros((0, NX)))
        sb = _f64(state_b if state_b is not None else np.zeros(0))
        tA = _f64(term_A if term_A is not None else np.zeros((0, NX)))
        tb = _f64(term_b if term_b is not None else np.zeros(0))
        lo, hi = _f64(u_lower), _f64(u_upper)
        self._keep = (A, B, Q, R, P, goal, sA, sb, tA, tb, lo, hi)
        d = ModelDesc(N=N, nx=NX, nu=nu, A=_dptr(A), B=_dptr(B), Q=_dptr(Q), R=_dptr(R), P=_dptr(P),
                      n_state_rows=sA.shape[0], state_A=_dptr(sA), state_b=_dptr(sb),
                      n_term_rows=tA.shape[0], term_A=_dptr(tA), term_b=_dptr(tb),
                      u_lower=_dptr(lo), u_upper=_dptr(hi), goal=_dptr(goal))
        handle = ctypes.c_void_p()
        with torch.cuda.device(self.device):
            check(lib.carmpc_problem_create(ctypes.byref(d), ctypes.byref(handle)), "carmpc_problem_create")
        self._h = handle
        self.N, self.nu, self.assembled = N, nu, True
        self.goal = goal.copy()
        self._info()

    @classmethod
    def dense(cls, H, G, w0, E, hq, goal, lb=None, ub=None, device=None) -> "QPProblem":
        """Generic dense QP without stage structure (carmpc_problem_create_dense)."""
        self = cls.__new__(cls)
        self.device = require_gpu(device)
        lib = _native.load()
        H, G, w0, E, hq, goal, lb, ub = (_f64(v) for v in (H, G, w0, E, hq, goal, lb, ub))
        n = H.shape[0]
        p = 0 if G is None else G.shape[0]
        handle = ctypes.c_void_p()
        with torch.cuda.device(self.device):
            check(lib.carmpc_problem_create_dense(n, p, NX, _dptr(H), _dptr(G), _dptr(w0), _dptr(E), _dptr(hq),
                                                  _dptr(lb), _dptr(ub), _dptr(goal), ctypes.byref(handle)),
                  "carmpc_problem_create_dense")
        self._h = handle
        self.N, self.nu, self.assembled = None, None, False
        self.goal = goal.copy()
        self._keep = ()
        self._info()
        return self

    def _info(self):
        vals = [ctypes.c_int32() for _ in range(5)]
        check(_native.load().carmpc_problem_info(self._h, *[ctypes.byref(v) for v in vals]), "carmpc_problem_info")
        self.n, self.p, self.npre, self.nx, _ = (v.value for v in vals)
        #: solve kernel chosen by ``kernel=0`` (auto): 1 dense, 2 staged, 7 grouped Riccati
        self.kernel = int(_native.load().carmpc_problem_kernel(self._h))

    def __del__(self):
        h = getattr(self, "_h", None)
        if h is not None and h.value:
            try:
                _native.load().carmpc_problem_destroy(h)
            except Exception:
                pass
            self._h = None

    # ------------------------------------------------------------------ data
    def matrices(self) -> dict:
        """Assembled T, S, H, h, G, E, w0 (device assembly kernel output) as numpy."""
        if not self.assembled:
            raise ValueError("only assembled problems keep T/S/G")
        N, n = self.N, self.n
        pa = ctypes.c_int32()
        check(_native.load().carmpc_problem_get(self._h, None, None, None, None, None, None, None,
                                                ctypes.byref(pa)), "carmpc_problem_get")
        out = dict(T=np.zeros(((N + 1) * NX, NX)), S=np.zeros(((N + 1) * NX, n)), H=np.zeros((n, n)),
                   h=np.zeros((n, NX)), G=np.zeros((pa.value, n)), E=np.zeros((pa.value, NX)),
                   w0=np.zeros(pa.value))
        check(_native.load().carmpc_problem_get(self._h, *[_dptr(out[k]) for k in ("T", "S", "H", "h", "G", "E",
                                                                                     "w0")], ctypes.byref(pa)),
              "carmpc_problem_get")
        return out

    def canonical_flops_per_iter(self) -> float:
        """Canonical dense-IPM count: p n^2 + n^3/3 + 6 n^2 + 12 p n with p = general (QP) rows."""
        return float(_native.load().carmpc_canonical_flops_per_iter(self.n, self.p))

    def executed_flops_per_iter(self, kernel: int = 0) -> float:
        """Flops per IPM iteration the chosen kernel performs for one QP (every recursion counted once)."""
        return float(_native.load().carmpc_executed_flops_per_iter(self._h, kernel))

    def issued_flops_per_iter(self, kernel: int = 0) -> float:
        """The same with every matrix-core instruction counted as a full 4x4x4 product."""
        return float(_native.load().carmpc_issued_flops_per_iter(self._h, kernel))

    # ----------------------------------------------------------------- solve
    def set_disturbance(self, Bd) -> None:
        """Constant scalar disturbance model x+ = A x + B u + Bd d (mpc.py:508-512): stores the row
        offsets of x = T x0 + S u + ABd d (mpc.py:631-650) for ``solve(..., dist=d)``."""
        Bd = _f64(Bd).reshape(-1)
        if Bd.shape != (NX,):
            raise ValueError("Bd must have nx entries")
        with torch.cuda.device(self.device):
            check(_native.load().carmpc_problem_set_disturbance(self._h, _dptr(Bd)), "carmpc_problem_set_disturbance")
        self.Bd = Bd.copy()

    def solve(self, x0: torch.Tensor, xref: torch.Tensor | None = None, settings: SolverSettings | None = None,
              out: tuple | None = None, stream=None, dist: torch.Tensor | None = None):
        """Solve QP(x0) for every row of x0 (B x 4, float64, on this problem's device).
        ``dist`` (B,) per-instance disturbance estimates (needs ``set_disturbance``).

        Returns (u (B x n) float64, status (B,) int32, iters (B,) int32), all on device;
        stream-ordered, no host synchronisation."""
        x0 = _as_dev(x0, self.device)
        B = x0.shape[0]
        if dist is not None:
            if not isinstance(dist, torch.Tensor):
                dist = torch.as_tensor(np.asarray(dist, dtype=np.float64))
            dist = dist.reshape(-1).to(device=self.device, dtype=torch.float64).contiguous()
            if dist.shape[0] != B:
                raise ValueError("dist must have one entry per instance")
        if xref is not None:
            xref = _as_dev(xref, self.device)
            if xref.shape != x0.shape:
                raise ValueError("xref must have the shape of x0")
        if out is None:
            u = torch.empty((B, self.n), dtype=torch.float64, device=self.device)
            st = torch.empty(B, dtype=torch.int32, device=self.device)
            it = torch.empty(B, dtype=torch.int32, device=self.device)
        else:
            u, st, it = out
        s = (settings or SolverSettings()).c()
        with torch.cuda.device(self.device):
            if dist is None:
                check(_native.load().carmpc_solve_batch(self._h, B, _tptr(x0), _tptr(xref), _tptr(u), _tptr(st),
                                                        _tptr(it), ctypes.byref(s), _stream_handle(stream)),
                      "carmpc_solve_batch")
            else:
                check(_native.load().carmpc_solve_batch_dist(self._h, B, _tptr(x0), _tptr(xref), _tptr(dist), _tptr(u),
                                                             _tptr(st), _tptr(it), ctypes.byref(s),
                                                             _stream_handle(stream)), "carmpc_solve_batch_dist")
        return u, st, it

    def solve_host(self, x0_host, chunks=None, settings: SolverSettings | None = None):
        """QP(x0) for states in host memory, results to host memory, transfers overlapped with the solve
        (``HostPipeline``).  Returns numpy (u (B x n), status (B,), iters (B,))."""
        X = np.ascontiguousarray(np.asarray(x0_host, dtype=np.float64).reshape(-1, NX))
        return solve_segments_host([self], [0, X.shape[0]], X, chunks, settings)

    def observe(self, y: torch.Tensor, xhat: torch.Tensor, uprev: torch.Tensor, C, L, stream=None) -> None:
        """In-place Luenberger update xhat <- A xhat + B uprev + L (y - C xhat) (mpc.py:439-448)."""
        C, L = _f64(C), _f64(L)
        y = _as_dev(y, self.device, width=C.shape[0])
        if xhat.dtype != torch.float64 or not xhat.is_contiguous() or xhat.device != self.device:
            raise ValueError("xhat must be a contiguous float64 tensor on the problem device")
        if uprev.dtype != torch.float64 or uprev.stride(1) != 1:
            raise ValueError("uprev must be float64 with unit column stride")
        with torch.cuda.device(self.device):
            check(_native.load().carmpc_observer_batch(self._h, xhat.shape[0], _tptr(y), C.shape[0], _dptr(C),
                                                       _dptr(L), _tptr(xhat), _tptr(uprev), uprev.stride(0),
                                                       _stream_handle(stream)), "carmpc_observer_batch")


    def observe_dist(self, y: torch.Tensor, xhat: torch.Tensor, dhat: torch.Tensor, uprev: torch.Tensor,
                     C, L1, Cd, L2, Bd, stream=None) -> None:
        """In-place disturbance-augmented observer (mpc.py:598-612): e = y - C xhat - Cd dhat,
        xhat <- A xhat + Bd dhat + B uprev + L1 e, dhat <- dhat + L2 . e."""
        C, L1, Cd, L2, Bd = _f64(C), _f64(L1), _f64(Cd).reshape(-1), _f64(L2).reshape(-1), _f64(Bd).reshape(-1)
        y = _as_dev(y, self.device, width=C.shape[0])
        for t, nm in ((xhat, "xhat"), (dhat, "dhat")):
            if t.dtype != torch.float64 or not t.is_contiguous() or t.device != self.device:
                raise ValueError(f"{nm} must be a contiguous float64 tensor on the problem device")
        if uprev.dtype != torch.float64 or uprev.stride(1) != 1:
            raise ValueError("uprev must be float64 with unit column stride")
        with torch.cuda.device(self.device):
            check(_native.load().carmpc_observer_dist_batch(self._h, xhat.shape[0], _tptr(y), C.shape[0], _dptr(C),
                                                            _dptr(L1), _dptr(Cd), _dptr(L2), _dptr(Bd), _tptr(xhat),
                                                            _tptr(dhat), _tptr(uprev), uprev.stride(0),
                                                            _stream_handle(stream)), "carmpc_observer_dist_batch")


    def closed_loop(self, state: torch.Tensor, *, mode: int = 0, steps_update: int = 1, last_step: int = 151,
                    dt: float = 0.2, l1: float = 3.5, goal_tol: float = 0.1, goal=None,
                    xhat: torch.Tensor | None = None, dhat: torch.Tensor | None = None,
                    xref: torch.Tensor | None = None, C=None, L=None, Cd=None, L2=None, Bd=None,
                    settings: SolverSettings | None = None, check_every: int = 8, stream=None) -> dict:
        """Run the examples' runner loop for every row of ``state`` on the GPU
        (carmpc_closed_loop_batch): mode 0 state feedback, 1 output feedback (xhat, C, L),
        2 output feedback with disturbance (also dhat, Cd, L2, Bd; needs set_disturbance).
        ``state``, ``xhat`` and ``dhat`` are updated in place.  Returns a dict of device tensors
        {state, xhat, dhat, u (last QP solution), outcome, steps}."""
        for t, nm in ((state, "state"), (xhat, "xhat"), (dhat, "dhat")):
            if t is not None and (t.dtype != torch.float64 or not t.is_contiguous() or t.device != self.device):
                raise ValueError(f"{nm} must be a contiguous float64 tensor on the problem device")
        if state.dim() != 2 or state.shape[1] != NX:
            raise ValueError("state must be B x 4")
        B = state.shape[0]
        if xhat is not None and tuple(xhat.shape) != (B, NX):
            raise ValueError("xhat must be B x 4")
        if dhat is not None and dhat.numel() != B:
            raise ValueError("dhat must have one entry per instance")
        if xref is not None:
            xref = _as_dev(xref, self.device)
            if xref.shape[0] == 1 and B > 1:
                xref = xref.expand(B, NX).contiguous()
            if tuple(xref.shape) != (B, NX):
                raise ValueError("xref must be B x 4 (or 1 x 4)")
        C, L, Cd, L2, Bd = _f64(C), _f64(L), _f64(Cd), _f64(L2), _f64(Bd)
        goal = _f64(goal)
        desc = _native.LoopDesc(mode, steps_update, last_step, 0 if C is None else C.shape[0], dt, l1, goal_tol,
                                _dptr(goal), _dptr(C), _dptr(L), _dptr(None if Cd is None else Cd.reshape(-1)),
                                _dptr(None if L2 is None else L2.reshape(-1)),
                                _dptr(None if Bd is None else Bd.reshape(-1)))
        keep = (C, L, Cd, L2, Bd, goal)   # noqa: F841  (host arrays live through the call)
        u = torch.empty((B, self.n), dtype=torch.float64, device=self.device)
        outcome = torch.empty(B, dtype=torch.int32, device=self.device)
        steps = torch.empty(B, dtype=torch.int32, device=self.device)
        s = (settings or SolverSettings()).c()
        with torch.cuda.device(self.device):
            check(_native.load().carmpc_closed_loop_batch(self._h, B, ctypes.byref(desc), _tptr(state), _tptr(xhat),
                                                          _tptr(dhat), _tptr(xref), _tptr(u), _tptr(outcome),
                                                          _tptr(steps), check_every, ctypes.byref(s),
                                                          _stream_handle(stream)), "carmpc_closed_loop_batch")
        return {"state": state, "xhat": xhat, "dhat": dhat, "u": u, "outcome": outcome, "steps": steps}

class CpuQPProblem:
    """The same condensed QP solved on the host's cores (``carmpc_cpu_*``): the product's CPU QP
    path, as the reference's controllers have one (cvxpy, lib/mpc.py:334-335).  Used by the
    controllers when no GPU is present; the arguments are those of ``QPProblem``, batches are
    numpy arrays (or CPU tensors) and the results numpy arrays."""

    assembled = True
    kernel = 0
    device = torch.device("cpu")

    def __init__(self, *, N: int, A, B, Q, R, P, goal, state_A=None, state_b=None, term_A=None, term_b=None,
                 u_lower=None, u_upper=None, device=None, threads: int = 0):
        lib = _native.load()
        A, B, Q, R, P, goal = (_f64(v) for v in (A, B, Q, R, P, goal))
        nu = B.shape[1]
        sA = _f64(state_A if state_A is not None else np.zeros((0, NX)))
        sb = _f64(state_b if state_b is not None else np.zeros(0))
        tA = _f64(term_A if term_A is not None else np.zeros((0, NX)))
        tb = _f64(term_b if term_b is not None else np.zeros(0))
        lo, hi = _f64(u_lower), _f64(u_upper)
        self._model = (A, B, Q, R, P)
        d = ModelDesc(N=N, nx=NX, nu=nu, A=_dptr(A), B=_dptr(B), Q=_dptr(Q), R=_dptr(R), P=_dptr(P),
                      n_state_rows=sA.shape[0], state_A=_dptr(sA), state_b=_dptr(sb),
                      n_term_rows=tA.shape[0], term_A=_dptr(tA), term_b=_dptr(tb),
                      u_lower=_dptr(lo), u_upper=_dptr(hi), goal=_dptr(goal))
        handle = ctypes.c_void_p()
        check(lib.carmpc_cpu_problem_create(ctypes.byref(d), ctypes.byref(handle)), "carmpc_cpu_problem_create")
        self._h = handle
        self.N, self.nu, self.threads = N, nu, threads
        self.goal = goal.copy()
        self._rows = (tA, tb, sA, sb)
        vals = [ctypes.c_int32() for _ in range(5)]
        check(lib.carmpc_cpu_problem_info(self._h, *[ctypes.byref(v) for v in vals]), "carmpc_cpu_problem_info")
        self.n, self.p, self.npre, self.nx, _ = (v.value for v in vals)

    def __del__(self):
        h = getattr(self, "_h", None)
        if h is not None and h.value:
            try:
                _native.load().carmpc_cpu_problem_destroy(h)
            except Exception:
                pass
            self._h = None

    def matrices(self) -> dict:
        """T, S, H, h, G, E, w0 built on the host (matrix_gen.py:6-72, mpc.py:196-253), with the
        keys and row order of ``QPProblem.matrices``."""
        from .matrix_gen import costgen, predmod
        A, B, Q, R, P = self._model
        N = self.N
        T, S = predmod(A, B, N)
        H, h, _ = costgen(Q, R, P, T, S, NX)
        tA, tb, sA, sb = self._rows
        rows = np.zeros((len(tb) + len(sb) * N, (N + 1) * NX))
        rows[:len(tb), -NX:] = tA
        for j, c in enumerate(sA):
            for i in range(N):
                rows[len(tb) + j * N + i, (i + 1) * NX:(i + 2) * NX] = c
        return dict(T=T, S=S, H=H, h=h, G=rows @ S, E=rows @ T, w0=np.concatenate((tb, np.repeat(sb, N))))

    def set_disturbance(self, Bd) -> None:
        Bd = _f64(Bd).reshape(-1)
        if Bd.shape != (NX,):
            raise ValueError("Bd must have nx entries")
        check(_native.load().carmpc_cpu_problem_set_disturbance(self._h, _dptr(Bd)), "carmpc_cpu_problem_set_disturbance")
        self.Bd = Bd.copy()

    def solve(self, x0, xref=None, settings: SolverSettings | None = None, dist=None, threads: int | None = None):
        """(u (B x n), status (B,), iters (B,)) as numpy arrays for the rows of x0 (B x 4)."""
        def host(a, width):
            if isinstance(a, torch.Tensor):
                a = a.detach().cpu().numpy()
            a = np.ascontiguousarray(np.asarray(a, dtype=np.float64).reshape(-1, width))
            return a
        X = host(x0, NX)
        B = X.shape[0]
        R = None
        if xref is not None:
            R = host(xref, NX)
            if R.shape[0] == 1 and B > 1:
                R = np.ascontiguousarray(np.broadcast_to(R, (B, NX)))
            if R.shape != X.shape:
                raise ValueError("xref must have the shape of x0")
        u = np.empty((B, self.n))
        st = np.empty(B, dtype=np.int32)
        it = np.empty(B, dtype=np.int32)
        ip = ctypes.POINTER(ctypes.c_int32)
        s = (settings or SolverSettings()).c()
        nthr = self.threads if threads is None else threads
        lib = _native.load()
        if dist is None:
            check(lib.carmpc_cpu_solve_batch(self._h, B, _dptr(X), _dptr(R), _dptr(u), st.ctypes.data_as(ip),
                                             it.ctypes.data_as(ip), ctypes.byref(s), nthr), "carmpc_cpu_solve_batch")
        else:
            dv = host(dist, 1).reshape(-1)
            if dv.shape[0] != B:
                raise ValueError("dist must have one entry per instance")
            check(lib.carmpc_cpu_solve_batch_dist(self._h, B, _dptr(X), _dptr(R), _dptr(dv), _dptr(u),
                                                  st.ctypes.data_as(ip), it.ctypes.data_as(ip), ctypes.byref(s), nthr),
                  "carmpc_cpu_solve_batch_dist")
        return u, st, it


def solve_segments(problems: list, offsets, x0: torch.Tensor, xref: torch.Tensor | None = None,
                   settings: SolverSettings | None = None, stream=None, out: tuple | None = None):
    """Instances grouped by problem: rows [offsets[j], offsets[j+1]) use problems[j]; one call
    solves all segments, in one kernel launch where the problems share a kernel instantiation
    (stream-ordered on ``stream``).  ``xref`` is B x 4 or 1 x 4;
    ``out`` = (u (B x ld, unit column stride), status (B,), iters (B,)) preallocated device tensors."""
    if not problems:
        raise ValueError("no problems")
    dev = problems[0].device
    if any(p.device != dev for p in problems):
        raise ValueError("all problems of one call must live on one device")
    x0 = _as_dev(x0, dev)
    B = x0.shape[0]
    offs_l = [int(o) for o in offsets]
    if len(offs_l) != len(problems) + 1:
        raise ValueError(f"offsets must have len(problems) + 1 = {len(problems) + 1} entries")
    if offs_l[0] < 0 or offs_l[-1] > B or any(b < a for a, b in zip(offs_l, offs_l[1:])):
        raise ValueError(f"offsets must be non-decreasing within [0, {B}]")
    ld_min = max(p.n for p in problems)
    s_obj = stream if stream is not None else torch.cuda.current_stream(dev)
    if out is None:
        with torch.cuda.stream(s_obj):      # the fill below must be ordered before the solve on `stream`
            u = torch.zeros((B, ld_min), dtype=torch.float64, device=dev)
            st = torch.empty(B, dtype=torch.int32, device=dev)
            it = torch.empty(B, dtype=torch.int32, device=dev)
    else:
        u, st, it = out
        if u.dtype != torch.float64 or u.dim() != 2 or u.shape[0] < offs_l[-1] or u.shape[1] < ld_min or \
                u.stride(1) != 1 or u.device != dev:
            raise ValueError(f"out[0] must be float64 on {dev}, at least {offs_l[-1]} x {ld_min}, unit column stride")
        for t, nm in ((st, "status"), (it, "iters")):
            if t.dtype != torch.int32 or t.dim() != 1 or t.shape[0] < offs_l[-1] or not t.is_contiguous() or t.device != dev:
                raise ValueError(f"out {nm} must be a contiguous int32 vector on {dev} with at least {offs_l[-1]} entries")
    ld = u.stride(0)
    xr = None
    if xref is not None:
        xr = _as_dev(xref, dev)
        if xr.shape[0] == 1 and B > 1:
            xr = xr.expand(B, NX).contiguous()
        if xr.shape != x0.shape:
            raise ValueError("xref must be B x 4 (or 1 x 4)")
    handles = (ctypes.c_void_p * len(problems))(*[p._h.value for p in problems])
    offs = (ctypes.c_int64 * (len(problems) + 1))(*offs_l)
    s = (settings or SolverSettings()).c()
    with torch.cuda.device(dev):
        check(_native.load().carmpc_solve_segments(handles, len(problems), offs, _tptr(x0), _tptr(xr), _tptr(u), ld,
                                                   _tptr(st), _tptr(it), ctypes.byref(s), _stream_handle(s_obj)),
              "carmpc_solve_segments")
    for t in (x0, xr, u, st, it):
        if t is not None:
            t.record_stream(s_obj)
    return u, st, it


class HostPipeline:
    """Solves for callers whose states and results live in HOST memory (the scalar ``step`` API's batched use:
    states come from a plant or a network, inputs go back to it).  Copies run on streams of their own, of the
    same priority as the solve stream: host -> device of x0, ``carmpc_solve_segments``, device -> host of
    u / status / iterations.  Pinned staging buffers and device buffers are allocated once per pipeline, in
    ``depth`` sets, so that a caller with a sequence of batches keeps ``depth`` of them in flight
    (``submit`` / ``wait``): the copies of one batch run under the solve of another and the rate is that of
    the solve alone.  ``solve`` is submit + wait for one batch.  Results are those of one ``solve_segments``
    call on resident data.

    ``first_action`` returns what the reference's ``step`` returns -- the first input of every optimal sequence
    (mpc.py:349: ``u.value[:nu]``; the rest of the horizon is kept there for plots only) -- so the copy back to
    the host is nu instead of N nu doubles per instance: 2 MB instead of 42 MB for 131,072 instances at N = 20,
    and the host-memory rate is within a few per cent of the resident one.

    ``chunks`` (row counts) cuts one batch into several solve calls whose copies overlap inside the batch;
    measured on the 131,072-instance mixed shard this is slower than one call (every call ends with its own
    latency-bound launch tails), so the default is one.  Batches in flight, same shard, full sequences back:
    one 22M QP/s, two 19-21M, three 18-24M (resident data: 27M) -- a copy that runs beside a solve slows the
    solve by about what it saves."""

    def __init__(self, problems: list, offsets, chunks=None, settings: SolverSettings | None = None, depth: int = 3,
                 first_action: bool = False):
        self.problems = list(problems)
        self.dev = problems[0].device
        self.offsets = [int(o) for o in offsets]
        if len(self.offsets) != len(problems) + 1 or self.offsets[0] != 0:
            raise ValueError("offsets must start at 0 and have len(problems) + 1 entries")
        self.B = B = self.offsets[-1]
        self.ld = max(p.n for p in problems)
        #: columns of u copied back to the host: the whole sequence, or the first input (nu entries) of each
        self.ncopy = self.ld
        if first_action:
            nus = {p.nu for p in problems}
            if len(nus) != 1 or None in nus:
                raise ValueError("first_action needs stage-structured problems with one input dimension")
            self.ncopy = int(nus.pop())
        self.settings = settings or SolverSettings()
        chunks = [B] if chunks is None else [int(c) for c in chunks if int(c) > 0]
        if sum(chunks) != B:
            raise ValueError(f"chunks must sum to the batch ({B})")
        self.bounds = np.concatenate([[0], np.cumsum(chunks)]).astype(np.int64)
        self.depth = max(1, int(depth))
        with torch.cuda.device(self.dev):
            self.s_in, self.s_solve, self.s_out = torch.cuda.Stream(), torch.cuda.Stream(), torch.cuda.Stream()
        self.sets = []
        for _ in range(self.depth):
            with torch.cuda.device(self.dev):
                d = dict(Xd=torch.empty((B, NX), dtype=torch.float64, device=self.dev),
                         u=torch.zeros((B, self.ld), dtype=torch.float64, device=self.dev),
                         st=torch.empty(B, dtype=torch.int32, device=self.dev),
                         it=torch.empty(B, dtype=torch.int32, device=self.dev))
            d.update(Xh=torch.empty((B, NX), dtype=torch.float64).pin_memory(),
                     uh=torch.empty((B, self.ncopy), dtype=torch.float64).pin_memory(),
                     sth=torch.empty(B, dtype=torch.int32).pin_memory(),
                     ith=torch.empty(B, dtype=torch.int32).pin_memory(), done=None)
            self.sets.append(d)
        self._next = 0
        self._handles = (ctypes.c_void_p * len(problems))(*[p._h.value for p in problems])
        torch.cuda.synchronize(self.dev)

    def staging(self, k: int | None = None) -> torch.Tensor:
        """Pinned B x 4 input buffer of buffer set k (default: the set the next ``submit`` uses): callers that
        produce their states in place there save the staging copy."""
        return self.sets[self._next if k is None else k]["Xh"]

    def submit(self, x0_host=None) -> int:
        """Queue one batch (B x 4 float64 numpy / CPU tensor; None = already written into ``staging()``) and
        return its buffer-set index without waiting.  A set is reused only after its previous batch is complete."""
        k = self._next
        self._next = (k + 1) % self.depth
        d = self.sets[k]
        if d["done"] is not None:
            d["done"].synchronize()
            d["done"] = None
        if x0_host is not None:
            src = x0_host if isinstance(x0_host, torch.Tensor) else torch.as_tensor(np.asarray(x0_host, dtype=np.float64))
            if src.data_ptr() != d["Xh"].data_ptr():
                d["Xh"].copy_(src.reshape(self.B, NX))
        lib = _native.load()
        s = self.settings.c()
        nseg = len(self.problems)
        with torch.cuda.device(self.dev):
            for c in range(len(self.bounds) - 1):
                r0, r1 = int(self.bounds[c]), int(self.bounds[c + 1])
                with torch.cuda.stream(self.s_in):
                    d["Xd"][r0:r1].copy_(d["Xh"][r0:r1], non_blocking=True)
                    ev_in = torch.cuda.Event()
                    ev_in.record(self.s_in)
                self.s_solve.wait_event(ev_in)
                offs = (ctypes.c_int64 * (nseg + 1))(*[min(max(o, r0), r1) for o in self.offsets])
                check(lib.carmpc_solve_segments(self._handles, nseg, offs, _tptr(d["Xd"]), None, _tptr(d["u"]), self.ld,
                                                _tptr(d["st"]), _tptr(d["it"]), ctypes.byref(s),
                                                ctypes.c_void_p(self.s_solve.cuda_stream)), "carmpc_solve_segments")
                ev_done = torch.cuda.Event()
                ev_done.record(self.s_solve)
                self.s_out.wait_event(ev_done)
                with torch.cuda.stream(self.s_out):
                    d["uh"][r0:r1].copy_(d["u"][r0:r1, :self.ncopy], non_blocking=True)
                    d["sth"][r0:r1].copy_(d["st"][r0:r1], non_blocking=True)
                    d["ith"][r0:r1].copy_(d["it"][r0:r1], non_blocking=True)
            with torch.cuda.stream(self.s_out):
                d["done"] = torch.cuda.Event()
                d["done"].record(self.s_out)
        return k

    def wait(self, k: int):
        """Block until batch ``k`` is complete; (u, status, iters) as that set's pinned host tensors, valid until
        the set is submitted again."""
        d = self.sets[k]
        if d["done"] is not None:
            d["done"].synchronize()
        return d["uh"], d["sth"], d["ith"]

    def solve(self, x0_host):
        return self.wait(self.submit(x0_host))


def solve_segments_host(problems: list, offsets, x0_host, chunks=None, settings: SolverSettings | None = None):
    """One-shot form of ``HostPipeline`` (allocates its buffers per call; keep a ``HostPipeline`` for repeated
    calls).  Returns numpy copies (u (B x ld), status, iters)."""
    hp = HostPipeline(problems, offsets, chunks, settings, depth=1)
    u, st, it = hp.solve(x0_host)
    return u.numpy().copy(), st.numpy().copy(), it.numpy().copy()


class HeteroQP:
    """Per-instance linear-MPC QPs (carmpc_hetero_*): instance b is linearised at its own
    (lin_state[b], lin_input[b]); A, B, the DARE terminal cost P, K and the condensed QP are
    built on the device.  Constraint rows, Q, R, box and goal are shared."""

    def __init__(self, *, N: int, batch: int, dt: float, l1: float, Q, R, goal, state_A=None, state_b=None,
                 term_A=None, term_b=None, u_lower=None, u_upper=None, device=None):
        self.device = require_gpu(device)
        lib = _native.load()
        Q, R, goal = _f64(Q), _f64(R), _f64(goal)
        sA = _f64(state_A if state_A is not None else np.zeros((0, NX)))
        sb = _f64(state_b if state_b is not None else np.zeros(0))
        tA = _f64(term_A if term_A is not None else np.zeros((0, NX)))
        tb = _f64(term_b if term_b is not None else np.zeros(0))
        lo, hi = _f64(u_lower), _f64(u_upper)
        self._keep = (Q, R, goal, sA, sb, tA, tb, lo, hi)
        d = _native.HeteroDesc(N=N, dt=dt, l1=l1, Q=_dptr(Q), R=_dptr(R), n_state_rows=sA.shape[0],
                               state_A=_dptr(sA), state_b=_dptr(sb), n_term_rows=tA.shape[0], term_A=_dptr(tA),
                               term_b=_dptr(tb), u_lower=_dptr(lo), u_upper=_dptr(hi), goal=_dptr(goal))
        handle = ctypes.c_void_p()
        with torch.cuda.device(self.device):
            check(lib.carmpc_hetero_create(ctypes.byref(d), int(batch), ctypes.byref(handle)), "carmpc_hetero_create")
        self._h = handle
        self.N, self.batch, self.n = N, int(batch), 2 * N
        self.goal = goal.copy()

    def __del__(self):
        h = getattr(self, "_h", None)
        if h is not None and h.value:
            try:
                _native.load().carmpc_hetero_destroy(h)
            except Exception:
                pass
            self._h = None

    def linearize(self, lin_state, lin_input, stream=None) -> None:
        """(Re)build every instance's model and QP at its linearisation point (device, stream-ordered)."""
        ls = _as_dev(lin_state, self.device)
        li = _as_dev(lin_input, self.device, width=2)
        if ls.shape[0] != self.batch or li.shape[0] != self.batch:
            raise ValueError(f"expected {self.batch} linearisation points")
        self._lin = (ls, li)   # kernels read them asynchronously
        with torch.cuda.device(self.device):
            check(_native.load().carmpc_hetero_linearize(self._h, _tptr(ls), _tptr(li), _stream_handle(stream)),
                  "carmpc_hetero_linearize")

    def solve(self, x0, xref=None, settings: SolverSettings | None = None, stream=None):
        """(u (B x 2N), status, iters) on device for x0 (B x 4); xref defaults to the goal."""
        x0 = _as_dev(x0, self.device)
        if x0.shape[0] != self.batch:
            raise ValueError(f"x0 must have {self.batch} rows")
        if xref is not None:
            xref = _as_dev(xref, self.device)
            if xref.shape[0] == 1 and self.batch > 1:
                xref = xref.expand(self.batch, NX).contiguous()
        u = torch.empty((self.batch, self.n), dtype=torch.float64, device=self.device)
        st = torch.empty(self.batch, dtype=torch.int32, device=self.device)
        it = torch.empty(self.batch, dtype=torch.int32, device=self.device)
        s = (settings or SolverSettings()).c()
        with torch.cuda.device(self.device):
            check(_native.load().carmpc_hetero_solve(self._h, _tptr(x0), _tptr(xref), _tptr(u), _tptr(st), _tptr(it),
                                                     ctypes.byref(s), _stream_handle(stream)), "carmpc_hetero_solve")
        return u, st, it

    def get(self) -> dict:
        """Per-instance model and QP slices as host numpy (carmpc_hetero_get): A, B, P, K,
        dare_status, p, npre, G (B x R x ldg), H (B x nv x nv), hq (B x nv x 4), w0, E."""
        lib = _native.load()
        dims = (ctypes.c_int64 * 6)()
        check(lib.carmpc_hetero_get(self._h, *([None] * 12), dims), "carmpc_hetero_get")
        R, ldg, nv, _n, _pa, B = (int(v) for v in dims)
        out = dict(A=np.empty((B, 4, 4)), B=np.empty((B, 4, 2)), P=np.empty((B, 4, 4)), K=np.empty((B, 2, 4)),
                   dare_status=np.empty(B, np.int32), p=np.empty(B, np.int32), npre=np.empty(B, np.int32),
                   G=np.empty((B, R, ldg)), H=np.empty((B, nv, nv)), hq=np.empty((B, nv, NX)), w0=np.empty((B, R)),
                   E=np.empty((B, R, NX)))
        ptr = lambda a: a.ctypes.data_as(ctypes.c_void_p)  # noqa: E731
        with torch.cuda.device(self.device):
            check(lib.carmpc_hetero_get(self._h, *[ptr(out[k]) for k in ("A", "B", "P", "K", "dare_status", "p", "npre",
                                                                          "G", "H", "hq", "w0", "E")], dims),
                  "carmpc_hetero_get")
        return out

LP_OPTIMAL, LP_UNBOUNDED, LP_MAX_ITER, LP_NUMERICAL = 0, 1, 2, 3


def lp_batch(c, A_list, b_list, relax=None, relax_amount: float = 1.0, device=None, return_iters: bool = False):
    """max c_l'x s.t. A_l x <= b_l (x in R^4) for every l on the GPU (carmpc_lp_batch).
    ``A_list``/``b_list`` may repeat the same arrays: identical objects are uploaded once.
    ``relax`` (per LP row index or -1) raises that row's b by ``relax_amount``.
    Returns host arrays (value (+inf unbounded), x, status)."""
    dev = require_gpu(device)
    c = np.ascontiguousarray(np.asarray(c, dtype=np.float64).reshape(-1, 4))
    L = c.shape[0]
    if len(A_list) != L or len(b_list) != L:
        raise ValueError("one constraint set per objective")
    pools_a, pools_b, a_off, b_off, m = [], [], np.zeros(L, np.int64), np.zeros(L, np.int64), np.zeros(L, np.int32)
    seen_a, seen_b = {}, {}
    na = nb = 0
    for l_, (A, b) in enumerate(zip(A_list, b_list)):
        if id(A) not in seen_a:
            Af = np.ascontiguousarray(np.asarray(A, dtype=np.float64).reshape(-1, 4))
            seen_a[id(A)] = (na, Af.shape[0], A)
            pools_a.append(Af.ravel())
            na += Af.size
        if id(b) not in seen_b:
            bf = np.ascontiguousarray(np.asarray(b, dtype=np.float64).ravel())
            seen_b[id(b)] = (nb, bf.size, b)
            pools_b.append(bf)
            nb += bf.size
        a_off[l_], rows, _ = seen_a[id(A)]
        b_off[l_], nrhs, _ = seen_b[id(b)]
        if rows != nrhs:
            raise ValueError(f"LP {l_}: {rows} rows but {nrhs} right-hand sides")
        m[l_] = rows
    max_m = int(m.max()) if L else 0
    if max_m > 1016:
        raise ValueError("LPs are limited to 1016 rows")
    t = lambda a: torch.as_tensor(a).to(dev)  # noqa: E731
    da, db = t(np.concatenate(pools_a) if pools_a else np.zeros(4)), t(np.concatenate(pools_b) if pools_b else np.zeros(1))
    dao, dbo, dm, dc = t(a_off), t(b_off), t(m), t(c)
    drel = None if relax is None else t(np.ascontiguousarray(np.asarray(relax, dtype=np.int32).ravel()))
    val = torch.empty(L, dtype=torch.float64, device=dev)
    x = torch.empty((L, 4), dtype=torch.float64, device=dev)
    st = torch.empty(L, dtype=torch.int32, device=dev)
    its = torch.empty(L, dtype=torch.int32, device=dev)
    with torch.cuda.device(dev):
        check(_native.load().carmpc_lp_batch(L, max_m, _tptr(dao), _tptr(dbo), _tptr(dm), _tptr(da), _tptr(db),
                                             _tptr(dc), _tptr(drel), relax_amount, _tptr(val), _tptr(x), _tptr(st),
                                             _tptr(its), _stream_handle(None)), "carmpc_lp_batch")
    out = (val.cpu().numpy(), x.cpu().numpy(), st.cpu().numpy())
    return out + (its.cpu().numpy(),) if return_iters else out

def plant_step(state: torch.Tensor, u: torch.Tensor, dt: float, l1: float, stream=None) -> torch.Tensor:
    """Batched nonlinear plant (simulator.py:51-69), in place on device.  Returns the per-instance
    input-limit flags of check_input (simulator.py:83-97); flagged rows are stepped anyway."""
    if state.dtype != torch.float64 or not state.is_contiguous():
        raise ValueError("state must be contiguous float64")
    bad = torch.empty(state.shape[0], dtype=torch.int32, device=state.device)
    with torch.cuda.device(state.device):
        check(_native.load().carmpc_plant_step_batch(state.shape[0], _tptr(state), _tptr(u), u.stride(0), dt, l1,
                                                     _tptr(bad), _stream_handle(stream)), "carmpc_plant_step_batch")
    return bad


def _as_dev(t, device, width: int = NX) -> torch.Tensor:
    if not isinstance(t, torch.Tensor):
        t = torch.as_tensor(np.asarray(t, dtype=np.float64))
    if t.dim() == 1:
        t = t.reshape(1, -1)
    t = t.to(device=device, dtype=torch.float64)
    if not t.is_contiguous():
        t = t.contiguous()
    if t.shape[1] != width:
        raise ValueError(f"expected rows of length {width}, got {tuple(t.shape)}")
    return t
