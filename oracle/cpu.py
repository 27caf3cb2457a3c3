"""ctypes wrapper of oracle/ipm.c (ORACLE, tests + bench cpu_baseline only)."""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

from . import qp as oq

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "build", "liboracle_ipm.so")
_lib = None


def build():
    subprocess.run(["make", "-s", "-C", _HERE], check=True)


def load():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        lib = ctypes.CDLL(LIB_PATH)
        dp = ctypes.POINTER(ctypes.c_double)
        ip = ctypes.POINTER(ctypes.c_int32)
        lib.oracle_solve_batch.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, dp, dp, dp, dp, dp, dp, dp,
                                           dp, dp, ip, dp, ctypes.c_int64, dp, dp, dp, ip, ip,
                                           ctypes.c_double, ctypes.c_double, ctypes.c_int, ctypes.c_int]
        lib.oracle_solve_batch.restype = ctypes.c_int
        lib.oracle_set_variant.argtypes = [ctypes.c_int] + [ctypes.c_double] * 4 + [ctypes.c_int, ctypes.c_double]
        lib.oracle_set_variant.restype = None
        _lib = lib
    return _lib


def _p(a, t=ctypes.c_double):
    if a is None:
        return None
    return a.ctypes.data_as(ctypes.POINTER(t))


class CpuProblem:
    """Normalised QP data of one ``oracle.assembly.Assembly`` for the C oracle."""

    def __init__(self, asm):
        Gn, w0n, En, keep, pre_w0, pre_E = oq.normalize_rows(asm.G, asm.w0, asm.E)
        self.n = asm.G.shape[1]
        self.H = np.ascontiguousarray(asm.H, dtype=np.float64)
        self.G = np.ascontiguousarray(Gn); self.w0 = np.ascontiguousarray(w0n); self.E = np.ascontiguousarray(En)
        self.pre_w0 = np.ascontiguousarray(pre_w0); self.pre_E = np.ascontiguousarray(pre_E)
        self.hq = np.ascontiguousarray(asm.h)
        self.lb = None if asm.lb is None else np.ascontiguousarray(asm.lb)
        self.ub = None if asm.ub is None else np.ascontiguousarray(asm.ub)
        self.goal = np.ascontiguousarray(asm.goal, dtype=np.float64)
        self.partner = np.ascontiguousarray(oq.opposite_pairs(Gn, w0n, En), dtype=np.int32)

    def solve(self, x0, xref=None, tol=oq.TOL_RES, tol_mu=oq.TOL_MU, max_iter=oq.MAX_ITER, threads=0,
              polish_corrections=oq.POLISH_CORRECTIONS, polish_mu=oq.POLISH_MU, polish_res=oq.POLISH_RES,
              init_mu0=oq.INIT_MU0, init_sfloor=oq.INIT_SFLOOR, polish_refine=oq.POLISH_REFINE,
              polish_act=oq.POLISH_ACT):
        """``**oq.FALLBACK_VARIANT`` selects the algorithm variant of the fallback kernels."""
        lib = load()
        lib.oracle_set_variant(int(polish_corrections), float(polish_mu), float(polish_res), float(init_mu0),
                               float(init_sfloor), int(polish_refine), float(polish_act))
        x0 = np.ascontiguousarray(x0, dtype=np.float64).reshape(-1, 4)
        B = x0.shape[0]
        xr = None if xref is None else np.ascontiguousarray(xref, dtype=np.float64).reshape(-1, 4)
        u = np.zeros((B, self.n)); st = np.zeros(B, np.int32); it = np.zeros(B, np.int32)
        rc = lib.oracle_solve_batch(self.n, self.G.shape[0], self.pre_w0.shape[0], _p(self.H), _p(self.G),
                                    _p(self.w0), _p(self.E), _p(self.pre_w0), _p(self.pre_E), _p(self.hq),
                                    _p(self.lb), _p(self.ub), _p(self.partner, ctypes.c_int32), _p(self.goal), B,
                                    _p(x0), _p(xr), _p(u),
                                    _p(st, ctypes.c_int32), _p(it, ctypes.c_int32), tol, tol_mu, max_iter, threads)
        assert rc == 0
        return u, st, it
