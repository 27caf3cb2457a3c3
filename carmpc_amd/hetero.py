"""Many MPCStateFB controllers, each linearised at its own point, solved in one batch.

The reference builds one controller per linearisation point: ``MPC.__init__`` linearises
(mpc.py:128-161), discretises (mpc.py:164-180), solves the DARE (mpc.py:67-74), forms K
(mpc.py:80-81) and the condensed QP (matrix_gen.py:6-72).  ``MPCStateFBBatch`` does all of that
on the device for B controllers at once -- ``relinearize`` rebuilds every instance's model in
two kernel launches, so successive-linearisation loops never leave the GPU -- and
``step_batch`` solves the B QPs with MPCStateFB.step semantics (mpc.py:312-349).

Constraint rows, the terminal set file, the input box and the goal are shared: they do not
depend on the linearisation point (the reference loads the same terminal-set file for any).
"""
from __future__ import annotations

import numpy as np

from .configuration import DT_CONTROL, LINEARIZE_INPUT, LINEARIZE_STATE
from .simulator import CarTrailerDimension


class MPCStateFBBatch:
    """B state-feedback MPC controllers of one environment with per-instance linearisation."""

    def __init__(self, dt: float = DT_CONTROL, N: int = 20, lin_states=None, lin_inputs=None, *, batch: int | None = None,
                 terminal_constraint: bool = True, input_constraint: bool = True, state_constraint: bool = True,
                 env=None, terminal_set_dir: str | None = None, device=None, settings=None):
        from .mpc import MPCStateFB
        from .qp import HeteroQP
        if lin_states is None:
            if batch is None:
                raise ValueError("give lin_states/lin_inputs or batch")
            lin_states = np.tile(LINEARIZE_STATE, (batch, 1))
            lin_inputs = np.tile(LINEARIZE_INPUT, (batch, 1))
        lin_states = np.asarray(lin_states, dtype=np.float64).reshape(-1, 4)
        lin_inputs = np.asarray(lin_inputs, dtype=np.float64).reshape(-1, 2)
        if lin_inputs.shape[0] != lin_states.shape[0]:
            raise ValueError("one input linearisation point per state linearisation point")
        # the shared pieces (rows, terminal set, box, goal) of one reference controller
        tmpl = MPCStateFB(dt=dt, N=N, lin_state=LINEARIZE_STATE, lin_input=LINEARIZE_INPUT,
                          terminal_constraint=terminal_constraint, input_constraint=input_constraint,
                          state_constraint=state_constraint, env=env, terminal_set_dir=terminal_set_dir,
                          device=device, settings=settings)
        self.template = tmpl
        self.N, self.dt, self.nu, self.nx = N, dt, 2, 4
        self.goal = np.array(tmpl.goal, dtype=np.float64)
        self.settings = tmpl.settings
        rows, rhs = tmpl._stage_rows() if state_constraint else (None, None)
        term_A = term_b = None
        if terminal_constraint:
            term_A, term_b = tmpl.term_set_A[:, -4:], tmpl.term_set_b
        box = input_constraint
        self.qp = HeteroQP(N=N, batch=lin_states.shape[0], dt=dt, l1=CarTrailerDimension.l1, Q=tmpl.Q, R=tmpl.R,
                           goal=self.goal, state_A=rows, state_b=rhs, term_A=term_A, term_b=term_b,
                           u_lower=tmpl.input_lower if box else None, u_upper=tmpl.input_upper if box else None,
                           device=device)
        self.batch = lin_states.shape[0]
        self.relinearize(lin_states, lin_inputs)

    def relinearize(self, lin_states, lin_inputs) -> None:
        """New linearisation points (B x 4, B x 2; host arrays or device tensors)."""
        self.qp.linearize(lin_states, lin_inputs)

    def model(self) -> dict:
        """Per-instance A, B, P, K, dare_status (host copies)."""
        g = self.qp.get()
        return {k: g[k] for k in ("A", "B", "P", "K", "dare_status")}

    def step_batch(self, x0, xref=None):
        """Solve all B QPs: returns (u0 (B x 2), u (B x 2N), status (B,)) as device tensors;
        status 1 = outside the region of attraction (mpc.py:336-338)."""
        u, st, _ = self.qp.solve(x0, xref, self.settings)
        return u[:, :self.nu], u, st
