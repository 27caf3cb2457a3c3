"""Terminal-set synthesis with the LPs on the GPU (mirrors lib/terminal_set.py).

Same functions and file format as the reference:

* ``compute_terminal_set(A_k, A_con, b_con, env)`` (terminal_set.py:23-73): the maximal
  constraint-admissible set of x+ = A_k x -- the smallest k such that every state row,
  propagated k+1 steps, is implied by the rows propagated 0..k steps.  The reference tests one
  k at a time with one cvxpy LP per row; here a window of k values (all rows, all k) is one
  ``carmpc_lp_batch`` launch and the smallest passing k is taken, which is the same answer.
* ``calc_terminal_set(env, ...)`` (terminal_set.py:135-213): intersect with the input set
  u = K (x - goal), remove redundant rows, save ``[A | b]`` as
  ``<env.name>_<goal...>.npy`` (the name rule ``mpc.py:97`` reads back).
* ``calc_terminal_sets(env, goals)``: many goals in lockstep (one launch per window for all).

The set operations follow the ``polytope`` package the reference uses (unit-norm rows,
``translation``, ``intersect``, ``reduce``); ``reduce``'s redundancy LPs run in one launch.
Parity: the reference's shipped ``terminal_sets/*.npy`` files (tests/test_gpu_terminal_set.py).
"""
from __future__ import annotations

import os

import numpy as np

from .configuration import DT_CONTROL, LINEARIZE_INPUT, LINEARIZE_STATE

ABS_TOL = 1e-7        # polytope's abs_tol (reduce)
RESULT_TOL = 1e-3     # terminal_set.py:60
MAX_K = 100           # terminal_set.py:70
_WINDOWS = (8, 16, 32, 48)


class Polytope:
    """H-representation {x : A x <= b} with unit-norm rows (as polytope.Polytope(A, b))."""

    def __init__(self, A, b, normalize: bool = True):
        A = np.atleast_2d(np.asarray(A, dtype=np.float64))
        b = np.asarray(b, dtype=np.float64).ravel()
        if normalize and len(A):
            n = np.linalg.norm(A, axis=1)
            A, b = A / n[:, None], b / n
        self.A, self.b = A, b

    def translation(self, d) -> "Polytope":
        """{x : A (x - d) <= b}."""
        return Polytope(self.A, self.b + self.A @ np.asarray(d, dtype=np.float64), normalize=False)

    def intersect(self, other: "Polytope") -> "Polytope":
        return Polytope(np.vstack((self.A, other.A)), np.hstack((self.b, other.b)))

    def __len__(self) -> int:
        return len(self.b)


def _check_lps(st, what):
    from .qp import LP_MAX_ITER, LP_NUMERICAL
    bad = np.flatnonzero((st == LP_MAX_ITER) | (st == LP_NUMERICAL))
    if bad.size:
        raise RuntimeError(f"{what} LP did not converge: {bad.size} of {st.size} (first {bad[:5].tolist()}, "
                           f"status {st[bad[:5]].tolist()})")


def _first_passing_k(A_k, A_con, b_cons, device=None):
    """Smallest k in 1..MAX_K+1 per right-hand side in b_cons (one per goal) with
    max_x A_con[i] A_k^(k+1) x - b[i] <= RESULT_TOL for all i over the rows of k (terminal_set.py:45-67)."""
    from .qp import lp_batch
    s = len(A_con)
    G = len(b_cons)
    powers = [np.eye(len(A_k))]
    found = [None] * G
    k0 = 1
    for w in _WINDOWS + (MAX_K + 1,):
        k1 = min(k0 + w - 1, MAX_K + 1)
        while len(powers) <= k1 + 1:
            powers.append(powers[-1] @ A_k)
        pending = [g for g in range(G) if found[g] is None]
        c, As, bs, owner = [], [], [], []
        for k in range(k0, k1 + 1):
            A_ts = np.vstack([A_con @ powers[t] for t in range(k + 1)])
            b_stack = [np.hstack((b_cons[g],) * (k + 1)) for g in pending]
            for gi, g in enumerate(pending):
                for i in range(s):
                    c.append(A_con[i] @ powers[k + 1])
                    As.append(A_ts)
                    bs.append(b_stack[gi])
                    owner.append((g, k, i))
        val, _x, st = lp_batch(np.array(c), As, bs, device=device)
        _check_lps(st, "terminal-set")
        ok = {}
        for (g, k, i), v in zip(owner, val):
            good = v - b_cons[g][i] <= RESULT_TOL
            ok[(g, k)] = ok.get((g, k), True) and bool(good)
        for g in pending:
            for k in range(k0, k1 + 1):
                if ok[(g, k)]:
                    found[g] = k
                    break
        if all(f is not None for f in found) or k1 > MAX_K:
            break
        k0 = k1 + 1
    return found


def compute_terminal_set(A_k, A_con, b_con, env=None, device=None):
    """terminal_set.py:23-73: (Polytope in absolute coordinates, k), or (None, None) when no k <= 100 works."""
    goal = np.zeros(len(A_k)) if env is None else np.asarray(env.goal, dtype=np.float64)
    return _compute_sets(A_k, A_con, b_con, [goal], device)[0]


def _compute_sets(A_k, A_con, b_con, goals, device=None):
    A_k = np.asarray(A_k, dtype=np.float64)
    base = Polytope(A_con, b_con)
    shifted = [base.translation(-g) for g in goals]                 # terminal_set.py:40-42
    A_n = shifted[0].A
    ks = _first_passing_k(A_k, A_n, [p.b for p in shifted], device)
    out = []
    for p, g, k in zip(shifted, goals, ks):
        if k is None:
            print("Unsuccesful search: too many iterations. The goal might be outside the constraints.")
            out.append((None, None))
            continue
        A_ts = np.vstack([A_n @ np.linalg.matrix_power(A_k, t) for t in range(k + 1)])
        b_ts = np.hstack((p.b,) * (k + 1))
        out.append((Polytope(A_ts, b_ts).translation(g), k))
    return out


def _dedupe(A, b, abs_tol=ABS_TOL):
    m = len(A)
    drop = np.zeros(m, bool)
    for i in range(m):
        if drop[i]:
            continue
        for j in range(i + 1, m):
            if not drop[j] and A[i] @ A[j] > 1 - abs_tol:
                if b[j] < b[i]:
                    drop[i] = True
                    break
                drop[j] = True
    return np.flatnonzero(~drop)


def reduce_batch(polys, abs_tol=ABS_TOL, device=None):
    """polytope.reduce for several polytopes: parallel-row elimination on the host, then one
    LP per remaining row (max a_k x with b_k relaxed by 1; redundant unless it exceeds b_k)."""
    from .qp import LP_UNBOUNDED, lp_batch
    cand = []
    c, As, bs, rel, owner = [], [], [], [], []
    for pi, p in enumerate(polys):
        idx = _dedupe(p.A, p.b, abs_tol)
        A, b = p.A[idx], p.b[idx]
        cand.append((A, b))
        for k in range(len(A)):
            c.append(A[k])
            As.append(A)
            bs.append(b)
            rel.append(k)
            owner.append((pi, k))
    val, _x, st = lp_batch(np.array(c).reshape(-1, 4), As, bs, relax=rel, relax_amount=1.0, device=device)
    _check_lps(st, "redundancy")
    keep = [[] for _ in polys]
    for (pi, k), v, s_ in zip(owner, val, st):
        b = cand[pi][1]
        if s_ == LP_UNBOUNDED or v - b[k] > abs_tol:
            keep[pi].append(k)
    return [Polytope(A[kp], b[kp], normalize=False) for (A, b), kp in zip(cand, keep)]


def reduce(poly: Polytope, abs_tol=ABS_TOL, device=None) -> Polytope:
    return reduce_batch([poly], abs_tol, device)[0]


def _controller(env):
    from .mpc import MPCStateFB
    # terminal_set.py:146-148: horizon 1, only the state constraints
    return MPCStateFB(dt=DT_CONTROL, N=1, lin_state=LINEARIZE_STATE, lin_input=LINEARIZE_INPUT,
                      terminal_constraint=False, input_constraint=False, state_constraint=True, env=env)


def filename_for(env, goal=None) -> str:
    goal = env.goal if goal is None else goal
    return env.name + "".join("_" + str(s) for s in goal) + ".npy"     # terminal_set.py:206


def calc_terminal_sets(env, goals, save: bool = False, directory: str = "../terminal_sets/", device=None):
    """calc_terminal_set for several goals of one environment; returns [(A, b) or (None, None)]."""
    ctrl = _controller(env)
    A_k = ctrl.A + ctrl.B @ ctrl.K                                           # terminal_set.py:150
    A_con, b_con = ctrl.state_constraint()
    A_con = A_con[..., 4:]                                                   # terminal_set.py:187
    goals_in = list(goals)
    goals = [np.asarray(g, dtype=np.float64) for g in goals_in]
    sets = _compute_sets(A_k, A_con, b_con, goals, device)                   # terminal_set.py:189
    # input set u = K (x - goal) (terminal_set.py:192-194), intersection and reduction (:197)
    A_in, b_in = ctrl.input_constraint()
    todo = [(gi, p.intersect(Polytope(A_in @ ctrl.K, b_in).translation(goals[gi])))
            for gi, (p, _k) in enumerate(sets) if p is not None]
    reduced = reduce_batch([p for _, p in todo], device=device) if todo else []
    out = [(None, None)] * len(goals)
    for (gi, _), r in zip(todo, reduced):
        out[gi] = (r.A, r.b)
        if save:
            np.save(os.path.join(directory, filename_for(env, goals_in[gi])), np.hstack((r.A, r.b[:, None])))
    return out


def calc_terminal_set(env, verbose: bool = False, save: bool = True, directory: str = "../terminal_sets/",
                      device=None):
    """terminal_set.py:135-213: returns (A, b) of the terminal set of env around env.goal and
    saves [A | b] as <env.name>_<goal...>.npy in ``directory`` (reference default ../terminal_sets/)."""
    (A, b), = calc_terminal_sets(env, [env.goal], save=False, device=device)
    if A is None:
        return None, None
    if verbose:
        print(f"Terminal set has {len(b)} constraints.")
    if save:
        fn = filename_for(env)
        print(f"Filename to save: {fn}")
        np.save(os.path.join(directory, fn), np.hstack((A, b[:, None])))
    return A, b
