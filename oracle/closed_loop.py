"""CPU restatement of the reference's runner loops (ORACLE, tests only).

Checker for ``carmpc_closed_loop_batch``: the same loop as
``examples/run_MPCStateFB.py:26-43`` / ``examples/run_MPCOutputFB.py:28-50``, one car at a
time, with the oracle QP (``oracle.qp.solve_instance[_dist]``, or the C restatement
``oracle/ipm.c`` through ``oracle.cpu`` for speed), the plant of ``simulator.py:51-69,83-118``
and the observers of ``mpc.py:439-448,598-612``.  Loop per index i:

    check_input(u)                     simulator.py:83-97 (clip=False: assertion)
    state = plant(state, u)            simulator.py:99-118
    if i % STEPS_UPDATE == 0:          run_MPCStateFB.py:32-33 / run_MPCOutputFB.py:32-33
        u = controller.step(...)       infinite cost -> OutsideTheRegionOfAttractionError
    stop: all |x - goal| <= tol        run_MPCStateFB.py:40
          i >= last_step               run_MPCStateFB.py:40 (i > 30/DT) / run_MPCOutputFB.py:48
"""
from __future__ import annotations

import numpy as np

from . import assembly as oa
from . import qp as oq

REACHED, INFEASIBLE, INPUT_VIOLATION, TIMEOUT, SOLVER_FAILURE = 0, 1, 2, 3, 4
ACC_LO, ACC_HI = -2 - 0.05, 2 + 0.05                        # simulator.py:45
DEL_LO, DEL_HI = -np.pi / 4 - 0.05, np.pi / 4 + 0.05        # simulator.py:44


def input_bad(u) -> bool:
    """check_input with clip=False (simulator.py:88-95).  The reference compares Python LISTS,
    ``[a, -a] <= [acc_upper, -acc_lower]``: list order is lexicographic, so the second pair only
    counts when ``a == acc_upper`` -- inputs below the lower limit pass.  Restated with the same
    list comparison."""
    a, delta = float(u[0]), float(u[1])
    return not ([a, -a] <= [ACC_HI, -ACC_LO] and [delta, -delta] <= [DEL_HI, -DEL_LO])


def run(asm, start, mode=0, last_step=151, goal_tol=0.1, steps_update=1, dt=oa.DT_SIMULATION, xref=None,
        init_estimate=None, solve=None):
    """One car through the runner loop.  mode 0 state feedback, 1 output feedback, 2 output
    feedback with disturbance.  ``solve(x0, xref, d)`` -> (status, u) defaults to the numpy
    oracle.  Returns dict(outcome, steps, state, xhat, dhat, u, trajectory)."""
    if solve is None:
        def solve(x0, xr, d):
            r = oq.solve_instance(asm, x0, xr) if mode != 2 else oq.solve_instance_dist(asm, x0, d, xr)
            return r["status"], r["u"]
    state = np.asarray(start, float).copy()
    xhat = np.asarray(start if init_estimate is None else init_estimate, float).copy()
    dhat = 0.0
    u = np.zeros(2 * asm.N)
    if xref is None:
        xref = asm.goal if mode == 0 else (oa.optimal_target_selection(asm.A, asm.B, oa.C_OUT @ asm.goal)[0]
                                            if mode == 1 else oa.XREF_DIST)
    traj = []
    i = 0
    while True:
        if input_bad(u):
            return dict(outcome=INPUT_VIOLATION, steps=i, state=state, xhat=xhat, dhat=dhat, u=u, trajectory=traj)
        state = oa.plant_step(state, u[:2], dt)
        traj.append(state.copy())
        if i % steps_update == 0:
            if mode == 0:
                x0 = state
            elif mode == 1:
                xhat = oa.luenberger_observer(asm.A, asm.B, xhat, u[:2], oa.C_OUT @ state)
                x0 = xhat
            else:
                xhat, dhat = oa.disturbance_observer(asm.A, asm.B, xhat, dhat, u[:2], oa.C_OUT @ state)
                x0 = xhat
            st, u_new = solve(x0, xref, dhat)
            if st != oq.STATUS_OPTIMAL:
                return dict(outcome=INFEASIBLE if st == oq.STATUS_INFEASIBLE else SOLVER_FAILURE, steps=i + 1,
                            state=state, xhat=xhat, dhat=dhat, u=u, trajectory=traj)
            u = np.asarray(u_new, float)
        if goal_tol > 0 and np.all(np.abs(state - asm.goal) <= goal_tol):
            return dict(outcome=REACHED, steps=i + 1, state=state, xhat=xhat, dhat=dhat, u=u, trajectory=traj)
        if i >= last_step:
            return dict(outcome=TIMEOUT, steps=i + 1, state=state, xhat=xhat, dhat=dhat, u=u, trajectory=traj)
        i += 1


def c_solver(asm, threads=1):
    """``solve`` callback on the C restatement (oracle/ipm.c), modes 0 and 1."""
    from .cpu import CpuProblem
    cp_ = CpuProblem(asm)

    def solve(x0, xr, d):
        u, st, _ = cp_.solve(np.asarray(x0, float).reshape(1, 4), np.asarray(xr, float).reshape(1, 4),
                             threads=threads)
        return int(st[0]), u[0]
    return solve
