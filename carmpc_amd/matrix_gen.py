"""Condensed prediction / cost matrices (API mirror of lib/matrix_gen.py).

The controllers in ``carmpc_amd.mpc`` never call these: their condensed QP is
assembled on the GPU by ``csrc/assembly.hip`` (``carmpc_problem_create``).
These host helpers exist so user code that imports ``lib.matrix_gen`` keeps
working, and are written as closed-form block constructions rather than
repeated matrix powers.

    x_bar = T x0 + S u_bar                          (matrix_gen.py:6-32)
    V_N   = u'Hu + 2 (h x0)'u + x0' const x0         (matrix_gen.py:35-72)
"""
from __future__ import annotations

import numpy as np


def _powers(A: np.ndarray, count: int) -> list:
    out = [np.eye(A.shape[0])]
    for _ in range(1, count):
        out.append(out[-1] @ A)
    return out


def predmod(A: np.ndarray, B: np.ndarray, N: int) -> tuple:
    """T = [I; A; ...; A^N] ((N+1)nx x nx) and block lower-triangular S ((N+1)nx x N nu)
    with block (i, j) = A^{i-j-1} B for i > j and a zero first block row."""
    nx, nu = B.shape
    Ap = _powers(A, N + 1)
    T = np.concatenate(Ap, axis=0)
    S = np.zeros(((N + 1) * nx, N * nu))
    for lag in range(N):                       # lag = i - j - 1
        blk = Ap[lag] @ B
        for j in range(N - lag):
            i = j + lag + 1
            S[i * nx:(i + 1) * nx, j * nu:(j + 1) * nu] = blk
    return T, S


def stack_matrix_along_diag(A: np.ndarray, N: int) -> np.ndarray:
    """blkdiag(A, ..., A) with N copies (matrix_gen.py:75-82)."""
    return np.kron(np.eye(N), A)


def costgen(Q: np.ndarray, R: np.ndarray, P: np.ndarray, T: np.ndarray, S: np.ndarray, nx: int) -> tuple:
    """H = R_hat + S'Q_hat S, h = S'Q_hat T, const = T'Q_hat T with Q_hat = blkdiag(Q..Q, P)."""
    N = S.shape[0] // nx - 1
    Q_hat = stack_matrix_along_diag(Q, N + 1)
    Q_hat[N * nx:, N * nx:] = P
    SQ = S.T @ Q_hat
    return stack_matrix_along_diag(R, N) + SQ @ S, SQ @ T, T.T @ Q_hat @ T
