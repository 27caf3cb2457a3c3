"""Cost values of a control step, written out from the reference's formulas, for the tests.

  objective      1/2 u'Hu + (h (x0 - x_ref))'u          lib/mpc.py:320-321, 477-478 (the QP's cost, constant dropped)
  terminal_cost  x_N' P x_N with the ABSOLUTE x_N       lib/mpc.py:344-345 (x_N = (T x0 + S u)[-4:], goal not subtracted)
  stage_cost     (x0 - goal)'Q(x0 - goal) + u_0'R u_0   lib/mpc.py:347
"""
import numpy as np

OBJ_RTOL = 1e-9      # relative objective difference against the certified optimum


def objective(asm, x0, u, xref=None):
    dx = np.asarray(x0, float) - (asm.goal if xref is None else np.asarray(xref, float))
    return 0.5 * u @ asm.H @ u + (asm.h @ dx) @ u


def objective_gap(asm, x0, u, u_ref, xref=None):
    """|J(u) - J(u_ref)| relative to max(1, |J(u_ref)|)."""
    j, jr = objective(asm, x0, u, xref), objective(asm, x0, u_ref, xref)
    return abs(j - jr) / max(1.0, abs(jr))


def terminal_cost(asm, x0, u):
    x_N = (asm.T @ np.asarray(x0, float) + asm.S @ u)[-4:]
    return x_N @ asm.P @ x_N


def stage_cost(asm, x0, u, Q, R, goal=None):
    dx = np.asarray(x0, float) - (asm.goal if goal is None else goal)
    return dx @ Q @ dx + u[:2] @ R @ u[:2]
