"""CPU restatement of the terminal-set synthesis (ORACLE, tests only).

Restates ``lib/terminal_set.py:23-73`` (``compute_terminal_set``: maximal
constraint-admissible set of x+ = (A + BK) x by iterated LPs) and ``:135-213``
(``calc_terminal_set``: state set, intersection with the input set u = K(x - goal),
redundancy removal, ``[A | b]`` rows saved as ``<env>_<goal...>.npy``).

The reference solves its LPs with cvxpy and represents sets with the third-party
``polytope`` package (no version pinned upstream); neither is installed here.  The
polytope operations used are restated from that package's published algorithm:

* ``Polytope(A, b)`` normalises every row to unit norm (``normalize=True`` default);
* ``translation(d)`` returns ``{x : A (x - d) <= b}`` = ``(A, b + A d)``;
* ``intersect`` stacks the rows;
* ``reduce``: drop rows parallel to an earlier, at-least-as-tight row
  (``a_i . a_j > 1 - abs_tol``), then keep row k iff ``max a_k x`` over the set with
  ``b_k`` relaxed by 1 exceeds ``b_k + abs_tol`` (or is unbounded), rows kept in order.

LPs here use scipy's HiGHS (``scipy.optimize.linprog``).  Parity is pinned against the
reference's own outputs: the six ``terminal_sets/*.npy`` files it ships
(tests/test_terminal_set.py).
"""
from __future__ import annotations

import numpy as np
from scipy.optimize import linprog

from . import assembly as oa

ABS_TOL = 1e-7        # polytope's default abs_tol
RESULT_TOL = 1e-3     # terminal_set.py:60 (result <= 0 + 1e-3)
MAX_K = 100           # terminal_set.py:70


def normalize(A, b):
    """Polytope(A, b): unit-norm rows."""
    A = np.asarray(A, float)
    b = np.asarray(b, float)
    n = np.linalg.norm(A, axis=1)
    return A / n[:, None], b / n


def translation(A, b, d):
    return A, b + A @ np.asarray(d, float)


def lp_max(c, A, b):
    """max c'x s.t. A x <= b -> (value, x); value = inf when unbounded."""
    r = linprog(-np.asarray(c, float), A_ub=A, b_ub=b, bounds=[(None, None)] * A.shape[1], method="highs")
    if r.status == 3:
        return np.inf, None
    if r.status != 0:
        raise RuntimeError(f"LP status {r.status}: {r.message}")
    return -r.fun, r.x


def compute_terminal_set(A_k, A_con, b_con, goal):
    """terminal_set.py:23-73 -> (A, b) in absolute coordinates (unit rows), k."""
    A_k = np.asarray(A_k, float)
    nx = A_k.shape[0]
    A_con, b_con = normalize(A_con, b_con)
    A_con, b_con = translation(A_con, b_con, -np.asarray(goal, float))     # terminal_set.py:40-42
    s = len(A_con)
    for k in range(1, MAX_K + 2):
        A_ts = np.vstack([A_con @ np.linalg.matrix_power(A_k, t) for t in range(k + 1)])   # :52
        b_ts = np.hstack((b_con,) * (k + 1))                                              # :53
        Ak1 = np.linalg.matrix_power(A_k, k + 1)
        ok = True
        for i in range(s):                                                               # :45-67
            val, _ = lp_max(A_con[i] @ Ak1, A_ts, b_ts)
            if not val - b_con[i] <= RESULT_TOL:
                ok = False
                break
        if ok:
            A, b = normalize(A_ts, b_ts)
            return translation(A, b, goal) + (k,)
        if k > MAX_K:
            return None, None, None
    return None, None, None


def reduce(A, b, abs_tol=ABS_TOL):
    """polytope.reduce restated (see the module docstring); rows stay in order."""
    A, b = normalize(A, b)
    m = len(A)
    drop = np.zeros(m, bool)
    for i in range(m):
        if drop[i]:
            continue
        for j in range(i + 1, m):
            if drop[j]:
                continue
            if A[i] @ A[j] > 1 - abs_tol:
                if b[j] < b[i]:
                    drop[i] = True
                    break
                drop[j] = True
    idx = np.flatnonzero(~drop)
    A, b = A[idx], b[idx]
    keep = []
    for k in range(len(A)):
        t = b.copy()
        t[k] += 1.0
        val, _ = lp_max(A[k], A, t)
        if val - b[k] > abs_tol:
            keep.append(k)
    return A[keep], b[keep]


def controller_matrices(env_name, dt=oa.DT_CONTROL):
    """MPCStateFB(N=1, terminal off, input off, state on) pieces used by calc_terminal_set
    (terminal_set.py:146-151): A, B, K, the x_1 state rows, the input rows."""
    A, B = oa.discretized_model(*oa.linearized_model(oa.LINEARIZE_STATE, oa.LINEARIZE_INPUT), dt)
    Q, R = oa.STAGE_COST_Q, oa.STAGE_COST_R
    P = oa.terminal_cost(A, B, Q, R)
    K = -np.linalg.inv(R + B.T @ P @ B) @ B.T @ P @ A                         # mpc.py:80
    env_A, env_b, goal = oa.ENVIRONMENTS[env_name]
    base_A = [[0, 0, 1, 0], [0, 0, -1, 0], [0, 0, 0, 1], [0, 0, 0, -1]]       # mpc.py:88-93
    base_b = [np.pi / 8, np.pi / 8, 5, 1]
    A_con = np.asarray(base_A + list(env_A), float)
    b_con = np.asarray(base_b + list(env_b), float)
    upper = np.array([2, np.pi / 8])                                          # mpc.py:83-84
    A_in = np.vstack((np.eye(2), -np.eye(2)))
    b_in = np.hstack((upper, upper))
    return dict(A=A, B=B, K=K, A_con=A_con, b_con=b_con, A_in=A_in, b_in=b_in, goal=np.asarray(goal, float))


def calc_terminal_set(env_name, goal=None):
    """terminal_set.py:135-213 without plotting / saving: returns the [A | b] halfspaces."""
    m = controller_matrices(env_name)
    goal = m["goal"] if goal is None else np.asarray(goal, float)
    A_k = m["A"] + m["B"] @ m["K"]                                            # :150
    A_t, b_t, _k = compute_terminal_set(A_k, m["A_con"], m["b_con"], goal)   # :189
    A_u, b_u = normalize(m["A_in"] @ m["K"], m["b_in"])                      # :193
    A_u, b_u = translation(A_u, b_u, goal)                                    # :194
    A_f, b_f = reduce(np.vstack((A_t, A_u)), np.hstack((b_t, b_u)))           # :197
    return np.hstack((A_f, b_f[:, None]))
