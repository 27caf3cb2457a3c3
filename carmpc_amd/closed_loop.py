"""Closed-loop runs of many cars at once, entirely on the GPU.

``run_closed_loop(controller, starts)`` is the runner loop of the reference examples
for a batch of start states:

* ``MPCStateFB``  -- ``examples/run_MPCStateFB.py:26-43``: plant step, ``controller.step(state)``,
  stop when every ``|x - goal| <= 0.1`` or ``i > 30 / DT_SIMULATION``;
* ``MPCOutputFB`` -- ``examples/run_MPCOutputFB.py:28-50``: plant step,
  ``controller.step(C x)`` (Luenberger observer + QP), stop at ``i >= 15 / DT_SIMULATION``;
* ``MPCOutputFBWithDisturbance`` -- the same runner with the disturbance observer.

An infeasible QP ends an instance as ``OutsideTheRegionOfAttractionError`` would end the
reference run.  Plant, observer, QP and the stop tests run as device kernels
(``carmpc_closed_loop_batch``); the host only launches.

``region_of_attraction(controller, grid)`` is the paper's grid search (many closed-loop simulations from a grid of start states) as one batched run.
"""
from __future__ import annotations

import math

import numpy as np

from . import _native
from .configuration import DT_SIMULATION, STEPS_UPDATE
from .simulator import CarTrailerDimension

OUTCOME_NAMES = _native.LOOP_NAMES
REACHED, INFEASIBLE, INPUT_VIOLATION, TIMEOUT, SOLVER_FAILURE = (
    _native.LOOP_REACHED, _native.LOOP_INFEASIBLE, _native.LOOP_INPUT_VIOLATION, _native.LOOP_TIMEOUT,
    _native.LOOP_SOLVER_FAILURE)


def first_index_above(t: float) -> int:
    """Smallest loop index i with i > t (run_MPCStateFB.py:40)."""
    return int(math.floor(t)) + 1


def first_index_at_least(t: float) -> int:
    """Smallest loop index i with i >= t (run_MPCOutputFB.py:48)."""
    return int(math.ceil(t))


def runner_defaults(controller, dt_sim: float = DT_SIMULATION) -> dict:
    """Mode, stop tests and references of the example runner for this controller type."""
    from .mpc import MPCOutputFB, MPCOutputFBWithDisturbance, MPCStateFB
    if isinstance(controller, MPCStateFB):
        return {"mode": 0, "last_step": first_index_above(30 / dt_sim), "goal_tol": 0.1}
    if isinstance(controller, MPCOutputFBWithDisturbance):
        return {"mode": 2, "last_step": first_index_at_least(15 / dt_sim), "goal_tol": 0.0}
    if isinstance(controller, MPCOutputFB):
        return {"mode": 1, "last_step": first_index_at_least(15 / dt_sim), "goal_tol": 0.0}
    raise TypeError(f"no closed-loop runner for {type(controller).__name__}")


def run_closed_loop(controller, starts, *, dt_sim: float = DT_SIMULATION, steps_update: int = STEPS_UPDATE,
                    last_step: int | None = None, goal_tol: float | None = None, init_estimates=None,
                    check_every: int = 8, stream=None) -> dict:
    """Run the example runner of ``controller``'s class from every row of ``starts`` (B x 4).

    ``init_estimates`` (B x 4) is the observers' ``init_state`` (output feedback; default:
    the start states, as the runner passes ``init_state=start_position``).  Returns host arrays
    {state (final plant state), xhat, dhat, u (last QP solution), outcome, steps}; outcome
    codes in ``OUTCOME_NAMES``, steps = loop indices executed."""
    import torch
    qp = controller.qp
    dev = qp.device
    d = runner_defaults(controller, dt_sim)
    if last_step is not None:
        d["last_step"] = last_step
    if goal_tol is not None:
        d["goal_tol"] = goal_tol
    starts = np.asarray(starts, dtype=np.float64).reshape(-1, 4)
    B = starts.shape[0]
    state = torch.as_tensor(starts.copy()).to(dev).contiguous()
    kw = {}
    xhat = dhat = xref = None
    if d["mode"] >= 1:
        est = starts if init_estimates is None else np.asarray(init_estimates, dtype=np.float64).reshape(B, 4)
        xhat = torch.as_tensor(est.copy()).to(dev).contiguous()
    if d["mode"] == 0:
        if not np.array_equal(controller.goal, qp.goal):
            xref = torch.as_tensor(controller.goal, dtype=torch.float64).to(dev).reshape(1, 4)
        kw = {}
    elif d["mode"] == 1:
        x_ref, _u_ref = controller.optimal_target_selection()
        xref = torch.as_tensor(x_ref, dtype=torch.float64).to(dev).reshape(1, 4)
        kw = {"C": controller.C, "L": controller.L}
    else:
        qp = controller._qp_dist()
        dhat = torch.full((B,), float(controller.d_estimate), dtype=torch.float64, device=dev)
        xref = torch.as_tensor(controller.X_REF, dtype=torch.float64).to(dev).reshape(1, 4)
        kw = {"C": controller.C, "L": controller.L1, "Cd": controller.Cd, "L2": controller.L2, "Bd": controller.Bd}
    res = qp.closed_loop(state, mode=d["mode"], steps_update=steps_update, last_step=d["last_step"], dt=dt_sim,
                         l1=CarTrailerDimension.l1, goal_tol=d["goal_tol"], goal=controller.goal, xhat=xhat,
                         dhat=dhat, xref=xref, settings=controller.settings, check_every=check_every,
                         stream=stream, **kw)
    out = {k: (None if v is None else v.cpu().numpy()) for k, v in res.items()}
    return out


def region_of_attraction(controller, x_values, y_values, psi: float = 0.0, v: float = 0.0, **kw) -> dict:
    """Closed-loop grid search over start positions (x, y) with heading psi and speed v:
    one batched run; returns the grid of outcomes and step counts (shape len(y) x len(x))."""
    X, Y = np.meshgrid(np.asarray(x_values, float), np.asarray(y_values, float))
    starts = np.stack([X.ravel(), Y.ravel(), np.full(X.size, psi), np.full(X.size, v)], axis=1)
    res = run_closed_loop(controller, starts, **kw)
    return {"x": X, "y": Y, "outcome": res["outcome"].reshape(X.shape), "steps": res["steps"].reshape(X.shape),
            "final_state": res["state"].reshape(X.shape + (4,))}
