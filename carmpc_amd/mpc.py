"""Linear MPC controllers for the kinematic bicycle (API mirror of lib/mpc.py).

Same classes, constructor signatures, public attributes and exceptions as the
reference, so ``examples/`` style loops run unchanged.  What changed is where
the work happens:

* the condensed QP (T, S, H, h and the stacked constraint rows of
  lib/matrix_gen.py:6-72 and lib/mpc.py:196-253) is assembled by a HIP kernel
  when the controller's ``QPProblem`` is created (lazily, on first use);
* ``step`` solves the QP with the batched wavefront-per-QP IPM
  (csrc/ipm_dense.hip) instead of ``cp.Problem(...).solve()`` (mpc.py:334-335,
  477-478); ``step_batch`` solves many states at once;
* the OutputFB observer runs as a device kernel (mpc.py:439-448) and the
  optimal-target QP (mpc.py:413-437), which is constant, is solved once in
  closed form instead of every step.

Without a GPU (``torch.cuda.is_available()`` false, or ``device="cpu"``) the controllers solve
the same QP on the host's cores through the library's ``carmpc_cpu_*`` entry points -- the
reference's controllers are CPU programs (mpc.py:334-335), and its plumbing configuration
(run_MPCStateFB, N = 10) runs without a GPU.  With a GPU present the device path is always used;
a missing library raises ``CarMPCNativeError`` either way.
"""
from __future__ import annotations

import os
from typing import Union

import numpy as np
from scipy.linalg import solve_discrete_are

from ._native import OPTIMAL, PRIMAL_INFEASIBLE, STATUS_NAMES
from .configuration import STAGE_COST_Q, STAGE_COST_R
from .environments import BaseEnv
from .simulator import CarTrailerDimension


def _target_qp(Hd, M, rhs, A_in, b_in, tol=1e-9):
    """min z'Hd z  s.t.  M z = rhs, A_in z <= b_in  for the handful of variables of a target selection
    (mpc.py:413-437: x_ref and u_ref, Hd = blkdiag(Q, R) positive definite, so the minimiser is unique).
    Exact active-set enumeration: for every set W of at most dim(null(M)) inequality rows the KKT system with
    M z = rhs and the rows of W as equalities is solved; the feasible one with non-negative multipliers is the
    optimum.  Returns z, or None when the constraints are inconsistent."""
    from itertools import combinations
    n = Hd.shape[0]
    z_p, *_ = np.linalg.lstsq(M, rhs, rcond=None)
    if np.abs(M @ z_p - rhs).max() > tol * (1.0 + np.abs(rhs).max()):
        return None
    _u, sv, vt = np.linalg.svd(M)
    rank = int((sv > 1e-10 * max(sv.max(), 1.0)).sum())
    Z = vt[rank:].T                                   # z = z_p + Z t
    free = Z.shape[1]
    best = None
    for k in range(0, free + 1):
        for W in combinations(range(A_in.shape[0]), k):
            Aw = A_in[list(W)] @ Z if k else np.zeros((0, free))
            if k and np.linalg.matrix_rank(Aw) < k:
                continue
            # stationarity in the reduced space: Z'Hd(z_p + Z t) + Aw' lam = 0, Aw t = b_w - A_w z_p
            K = np.block([[Z.T @ Hd @ Z, Aw.T], [Aw, np.zeros((k, k))]]) if free else np.zeros((0, 0))
            r = np.concatenate((-Z.T @ Hd @ z_p, (b_in[list(W)] - A_in[list(W)] @ z_p) if k else np.zeros(0)))
            try:
                sol = np.linalg.solve(K, r) if free else np.zeros(0)
            except np.linalg.LinAlgError:
                continue
            z = z_p + Z @ sol[:free]
            lam = sol[free:]
            if (A_in @ z - b_in).max(initial=-np.inf) <= tol and (lam >= -tol).all():
                val = z @ Hd @ z
                if best is None or val < best[0]:
                    best = (val, z)
        if best is not None:
            return best[1]
    return None


class OutsideTheRegionOfAttractionError(Exception):
    """The QP is infeasible: the initial state lies outside the region of attraction (mpc.py:17-18)."""


class SolverError(Exception):
    """The IPM stopped without a certificate (iteration limit or numerical failure)."""


ArrayLike = Union[np.ndarray, list]


class MPC:
    """Base controller: model, costs, constraint sets and the device QP (mpc.py:21-276).

    Extra keyword-only arguments (not in the reference):
      terminal_set_dir -- directory searched for ``<name>_<goal...>.npy``
                          (default '../terminal_sets/', cwd-relative as in mpc.py:98)
      device           -- torch device for the QP problem (default: current GPU)
      settings         -- ``carmpc_amd.qp.SolverSettings``
    """

    def __init__(self, dt: float, N: int, lin_state: ArrayLike, lin_input: ArrayLike,
                 terminal_constraint: bool = True, input_constraint: bool = True, state_constraint: bool = True,
                 env: BaseEnv = None, use_LQR: bool = False, *, terminal_set_dir: str | None = None,
                 device=None, settings=None) -> None:
        self.dt, self.N = dt, N
        self.lin_state = np.array(lin_state) if isinstance(lin_state, list) else lin_state
        self.lin_input = np.array(lin_input) if isinstance(lin_input, list) else lin_input
        self.goal = np.array(env.goal)
        self.x_horizon, self.u_horizon = None, None
        self.cost = 0
        self.env = env
        self.use_LQR = use_LQR
        self.device = device
        self.settings = settings
        A_lin, B_lin = self.linearized_model(self.lin_state, self.lin_input)
        self.A, self.B = self.discretized_model(A_lin, B_lin, dt)
        self.state_const_A, self.state_const_b = [], []
        self.nx, self.nu = 4, 2
        self.Q, self.R = STAGE_COST_Q, STAGE_COST_R
        self.terminal_constraint_bool = terminal_constraint
        self.input_constraint_bool = input_constraint
        self.state_constraint_bool = state_constraint
        try:                                                                   # mpc.py:69-74
            self.P = solve_discrete_are(self.A, self.B, self.Q, self.R)
        except np.linalg.LinAlgError:
            print("\nNOT POSSIBLE TO SOLVE DARE\n")
            self.P = np.zeros((4, 4))
        self.K = -np.linalg.solve(self.R + self.B.T @ self.P @ self.B, self.B.T @ self.P @ self.A)   # mpc.py:81
        self.input_upper = np.array([2, np.pi / 8])                           # mpc.py:84-85
        self.input_lower = -self.input_upper
        self.state_const_A += [[0, 0, 1, 0], [0, 0, -1, 0], [0, 0, 0, 1], [0, 0, 0, -1]]   # mpc.py:89-93
        self.state_const_b += [np.pi / 8, np.pi / 8, 5, 1]
        self._load_terminal_set(terminal_set_dir)
        self._qp = None
        self._host_mats = None

    # ------------------------------------------------------------ model (host setup)
    @staticmethod
    def linearized_model(lin_state: np.ndarray, lin_input: np.ndarray) -> tuple:
        """Jacobians of the bicycle at (x_e, u_e) (mpc.py:128-161)."""
        if lin_state.shape != (4,):
            raise AssertionError(f"The state should have shape [4], but has {lin_state.shape}.")
        if lin_input.shape != (2,):
            raise AssertionError(f"The input should have shape [2], but has {lin_input.shape}.")
        psi, v = lin_state[2], lin_state[3]
        delta = lin_input[1]
        l1 = CarTrailerDimension.l1
        A_lin = np.zeros((4, 4))
        A_lin[0, 2], A_lin[0, 3] = -v * np.sin(psi), np.cos(psi)
        A_lin[1, 2], A_lin[1, 3] = v * np.cos(psi), np.sin(psi)
        A_lin[2, 3] = np.tan(delta) / l1
        B_lin = np.zeros((4, 2))
        B_lin[2, 1] = v / l1 * 1 / np.cos(delta) ** 2
        B_lin[3, 0] = 1
        return A_lin, B_lin

    @staticmethod
    def discretized_model(A: np.ndarray, B: np.ndarray, dt: float) -> tuple:
        """Forward Euler: A_d = dt A + I, B_d = dt B (mpc.py:164-180)."""
        if len(A) != len(B):
            raise AssertionError("Matrices A and B should have the same height.")
        return dt * A + np.eye(len(A)), dt * B

    def _load_terminal_set(self, directory: str | None) -> None:
        """Terminal half-spaces on x_N from ``<name>_<g0>_<g1>..npy`` or the goal box (mpc.py:95-117)."""
        if not self.terminal_constraint_bool:
            return
        filename = self.env.name + "".join("_" + str(s) for s in self.env.goal) + ".npy"
        directory = "../terminal_sets/" if directory is None else directory
        path = os.path.join(directory, filename)
        width = (self.N + 1) * self.nx
        try:
            data = np.load(path)
            A_hat = np.zeros((len(data), width))
            A_hat[:, -4:] = data[..., :4]
            self.term_set_A, self.term_set_b = A_hat, data[..., 4]
            print(f"Using {path} for the terminal set.")
        except FileNotFoundError:
            print(f"No terminal set found for the specific combination of environment{self.env.name} and "
                  f"goal{self.env.goal}.", "The goal state will be used as terminal constraint, but this "
                  "might be too strict.")
            sel = np.diag([1, 1, 1, 0])
            A_hat = np.zeros((2 * self.nx, width))
            A_hat[:self.nx, -self.nx:] = sel
            A_hat[self.nx:, -self.nx:] = -sel
            self.term_set_A, self.term_set_b = A_hat, np.hstack((self.goal, -self.goal))

    def check_constraints(self) -> None:
        if len(self.state_const_A) != len(self.state_const_b):
            raise AssertionError("The state constraint lists do not have the same length.")

    def set_goal(self, goal: ArrayLike) -> None:
        """Set the reference; must be an equilibrium of the linear model (mpc.py:182-194)."""
        if np.array(goal).shape != (4,):
            raise AssertionError("goal must have shape (4,)")
        if not np.all(goal == self.A @ goal):
            raise AssertionError("Goal is not an equilibrium point. At least not for the linearized model. "
                                 "E.g. psi != 0 is not an equilibrium point.")
        self.goal = np.array(goal) if isinstance(goal, list) else goal

    # ------------------------------------------------------------ constraint stacks
    def terminal_constraint(self) -> tuple:
        """(A, b) on the stacked state sequence (mpc.py:196-203)."""
        return self.term_set_A, self.term_set_b

    def input_constraint(self) -> tuple:
        """[I; -I] u <= [ub..; -lb..] over the horizon (mpc.py:205-220)."""
        if self.nu != len(self.input_upper) or self.nu != len(self.input_lower):
            raise AssertionError("input bound length differs from nu")
        eye = np.eye(self.N * self.nu)
        return np.vstack((eye, -eye)), np.concatenate((np.tile(self.input_upper, self.N),
                                                       np.tile(-self.input_lower, self.N)))

    def _stage_rows(self) -> tuple:
        rows = list(self.state_const_A) + (list(self.env.constraints_A) if self.env is not None else [])
        rhs = list(self.state_const_b) + (list(self.env.constraints_b) if self.env is not None else [])
        return np.asarray(rows, dtype=float).reshape(-1, 4), np.asarray(rhs, dtype=float)

    def state_constraint(self) -> tuple:
        """Per-step rows on x_1..x_N, one block of N rows per half-space (mpc.py:222-253)."""
        rows, rhs = self._stage_rows()
        N, nx = self.N, self.nx
        A = np.zeros((len(rows) * N, (N + 1) * nx))
        for j, c in enumerate(rows):
            for i in range(N):
                A[j * N + i, (i + 1) * nx:(i + 2) * nx] = c
        return A, np.repeat(rhs, N)

    # ------------------------------------------------------------ device QP
    @property
    def qp(self):
        """The controller's QP: on the device (assembled by the HIP kernel on first access), or the
        host twin when no GPU is present / ``device="cpu"``."""
        if self._qp is None:
            import torch
            from .qp import CpuQPProblem, QPProblem
            on_gpu = torch.cuda.is_available() if self.device is None else torch.device(self.device).type == "cuda"
            QPProblem = QPProblem if on_gpu else CpuQPProblem
            rows, rhs = self._stage_rows() if self.state_constraint_bool else (None, None)
            term_A = term_b = None
            if self.terminal_constraint_bool:
                term_A, term_b = self.term_set_A[:, -self.nx:], self.term_set_b
            box = self.input_constraint_bool
            self._qp = QPProblem(N=self.N, A=self.A, B=self.B, Q=self.Q, R=self.R, P=self.P, goal=self.goal,
                                 state_A=rows, state_b=rhs, term_A=term_A, term_b=term_b,
                                 u_lower=self.input_lower if box else None, u_upper=self.input_upper if box else None,
                                 device=self.device)
        return self._qp

    def _mats(self) -> dict:
        if self._host_mats is None:
            self._host_mats = self.qp.matrices()
        return self._host_mats

    T = property(lambda self: self._mats()["T"], doc="(N+1)nx x nx prediction matrix (device-assembled)")
    S = property(lambda self: self._mats()["S"], doc="(N+1)nx x N nu input-to-state matrix (device-assembled)")
    H = property(lambda self: self._mats()["H"], doc="condensed Hessian (device-assembled)")
    h = property(lambda self: self._mats()["h"], doc="condensed linear-term matrix (device-assembled)")

    @property
    def on_cpu(self) -> bool:
        """True when this controller solves on the host (no GPU present, or device="cpu")."""
        return self.qp.device.type == "cpu"

    def _solve_one(self, x0: np.ndarray, xref: np.ndarray) -> np.ndarray:
        if self.on_cpu:
            u, st, _ = self.qp.solve(np.asarray(x0, float).reshape(1, 4), np.asarray(xref, float).reshape(1, 4),
                                     self.settings)
            return self._check_status(int(st[0]), u[0])
        import torch
        dev = self.qp.device
        X = torch.as_tensor(np.asarray(x0, dtype=np.float64).reshape(1, 4)).to(dev)
        R = torch.as_tensor(np.asarray(xref, dtype=np.float64).reshape(1, 4)).to(dev)
        u, st, _ = self.qp.solve(X, R, self.settings)
        status = int(st.cpu()[0])
        return self._check_status(status, u[0].cpu().numpy())

    @staticmethod
    def _check_status(status: int, u: np.ndarray) -> np.ndarray:
        if status == PRIMAL_INFEASIBLE:
            raise OutsideTheRegionOfAttractionError
        if status != OPTIMAL:
            raise SolverError(f"QP solve ended with status {STATUS_NAMES.get(status, status)}")
        return u

    def step_batch(self, x0, xref=None):
        """Solve the MPC QP for a batch of states (B x 4) on the GPU.

        Returns (u0 (B x nu), u (B x N nu), status (B,)) as device tensors; status
        1 marks states outside the region of attraction.  xref defaults to the goal."""
        if self.on_cpu:     # host twin: numpy in, numpy out
            X = np.asarray(x0, dtype=np.float64).reshape(-1, 4)
            Rf = self.goal.reshape(1, 4) if xref is None else np.asarray(xref, dtype=np.float64).reshape(-1, 4)
            u, st, _ = self.qp.solve(X, Rf, self.settings)
            return u[:, :self.nu], u, st
        import torch
        X = torch.as_tensor(x0, dtype=torch.float64).to(self.qp.device).reshape(-1, 4)
        Rf = None
        if xref is not None:
            Rf = torch.as_tensor(xref, dtype=torch.float64).to(self.qp.device).reshape(-1, 4)
        elif not np.array_equal(self.goal, self.qp.goal):
            Rf = torch.as_tensor(self.goal, dtype=torch.float64).to(self.qp.device).expand(X.shape[0], 4)
        u, st, _ = self.qp.solve(X, Rf, self.settings)
        return u[:, :self.nu], u, st

    # ------------------------------------------------------------ LQR
    def LQR(self, x0) -> np.ndarray:
        """Unconstrained optimal law u = K (x0 - goal) (mpc.py:255-262)."""
        return self.K @ (x0 - self.goal)

    def step(self, x0) -> np.ndarray:
        """LQR step with input clipping if use_LQR, else NotImplementedError (mpc.py:264-276)."""
        if not self.use_LQR:
            raise NotImplementedError
        u0 = np.clip(self.LQR(x0), self.input_lower, self.input_upper)
        dx = x0 - self.goal
        self.stage_cost = dx @ self.Q @ dx + u0 @ self.R @ u0
        return u0


class MPCStateFB(MPC):
    """State-feedback MPC (mpc.py:279-349)."""

    def __init__(self, dt: float, N: int, lin_state: ArrayLike, lin_input: ArrayLike, terminal_constraint: bool = True,
                 input_constraint: bool = True, state_constraint: bool = True, env: BaseEnv = None, **kw) -> None:
        super().__init__(dt, N, lin_state, lin_input, terminal_constraint, input_constraint, state_constraint,
                         env, **kw)
        self.check_constraints()

    def step(self, x0) -> np.ndarray:
        """First input of the optimal sequence for QP(x0) (mpc.py:312-349); the QP runs on the GPU."""
        x0 = np.asarray(x0, dtype=float)
        u = self._solve_one(x0, self.goal)
        m = self._mats()
        dx = x0 - self.goal
        self.x_horizon = (m["T"] @ dx + m["S"] @ u).reshape(-1, self.nx) + self.goal    # mpc.py:341-342
        self.u_horizon = u.reshape(-1, 2)                                              # mpc.py:343
        x_N = (m["T"] @ x0 + m["S"] @ u)[-4:]                                          # mpc.py:344 (absolute)
        self.terminal_cost = x_N @ self.P @ x_N
        u0 = u[:self.nu]
        self.stage_cost = dx @ self.Q @ dx + u0 @ self.R @ u0                           # mpc.py:347
        return u[:self.nu]


class MPCOutputFB(MPC):
    """Output-feedback MPC: Luenberger observer + target selection + QP (mpc.py:352-492)."""

    C_OUT = np.array([[1, 0, 0, 0], [0, 1, 0, 0], [0, 0, 0, 1]])                     # mpc.py:387-389
    L_GAIN = np.array([[3.00000000e-01, 2.00284502e-16, 2.00000000e-01],             # mpc.py:401-404
                       [3.48682242e+00, 1.90000000e+00, 3.86733776e-01],
                       [1.74341121e+00, 8.00000000e-01, 1.93366888e-01],
                       [-3.36822969e-16, -2.07305381e-16, 3.00000000e-01]])

    def __init__(self, dt: float, N: int, lin_state: ArrayLike, lin_input: ArrayLike, init_state: ArrayLike,
                 terminal_constraint: bool = True, input_constraint: bool = True, state_constraint: bool = True,
                 env: BaseEnv = None, **kw) -> None:
        super().__init__(dt, N, lin_state, lin_input, terminal_constraint, input_constraint, state_constraint,
                         env, **kw)
        self.C = self.C_OUT.copy()
        self.y_goal = self.C @ env.goal
        self.L = self.L_GAIN.copy()
        self._x_est = np.array(init_state, dtype=float)
        self._x_dev = None
        self.previous_u = np.zeros(2)
        self._u_dev = None
        self._ots = None
        self.check_constraints()

    @property
    def x_estimate(self) -> np.ndarray:
        return self._x_est

    @x_estimate.setter
    def x_estimate(self, value) -> None:
        self._x_est = np.array(value, dtype=float)
        self._x_dev = None

    def optimal_target_selection(self) -> tuple:
        """(x_ref, u_ref) for y_goal (mpc.py:413-437).  The equality block [[I-A, -B], [C, 0]] has
        full column rank for the Road* setups, so the QP's feasible set is one point: solve it in
        closed form and check the state/input inequalities."""
        if self._ots is None:
            M = np.block([[np.eye(self.nx) - self.A, -self.B], [self.C, np.zeros((self.C.shape[0], self.nu))]])
            rhs = np.concatenate((np.zeros(self.nx), self.y_goal))
            A_s, b_s = np.asarray(self.state_const_A, float), np.asarray(self.state_const_b, float)
            if np.linalg.matrix_rank(M) == self.nx + self.nu:
                # the feasible set of the equalities is one point: closed form, then the inequalities are a check
                xu, *_ = np.linalg.lstsq(M, rhs, rcond=None)
                if np.abs(M @ xu - rhs).max() > 1e-9:
                    raise OutsideTheRegionOfAttractionError("no steady state reaches y_goal")
                if (A_s @ xu[:self.nx] - b_s).max() > 1e-9 or np.any(xu[self.nx:] > self.input_upper + 1e-9) or \
                        np.any(xu[self.nx:] < self.input_lower - 1e-9):
                    raise OutsideTheRegionOfAttractionError("target violates the constraints")
            else:
                # a family of steady states reaches y_goal: the reference's QP picks the cheapest admissible one
                A_in = np.block([[A_s, np.zeros((A_s.shape[0], self.nu))],
                                 [np.zeros((self.nu, self.nx)), np.eye(self.nu)],
                                 [np.zeros((self.nu, self.nx)), -np.eye(self.nu)]])
                b_in = np.concatenate((b_s, self.input_upper, -np.asarray(self.input_lower)))
                Hd = np.block([[self.Q, np.zeros((self.nx, self.nu))], [np.zeros((self.nu, self.nx)), self.R]])
                xu = _target_qp(Hd, M, rhs, A_in, b_in)
                if xu is None:
                    raise OutsideTheRegionOfAttractionError("no admissible steady state reaches y_goal")
            x_ref, u_ref = xu[:self.nx], xu[self.nx:]
            self._ots = (x_ref, u_ref)
        return self._ots

    def luenberger_observer(self, y0) -> np.ndarray:
        """Host form of x_hat+ = A x_hat + B u_prev + L (y - C x_hat) (mpc.py:439-448).
        ``step`` runs the same update on the GPU (carmpc_observer_batch)."""
        return self.A @ self.x_estimate + self.B @ self.previous_u + self.L @ (y0 - self.C @ self.x_estimate)

    def step(self, y0) -> np.ndarray:
        """Observer -> target -> QP (mpc.py:450-492), observer and QP on the GPU."""
        qp = self.qp
        if self.on_cpu:
            x0 = self.luenberger_observer(np.asarray(y0, dtype=float))          # mpc.py:456-458
            self._x_est = x0.copy()
            x_ref, _u_ref = self.optimal_target_selection()
            u = self._solve_one(x0, x_ref)
            return self._finish_step(x0, x_ref, u)
        import torch
        dev = qp.device
        if self._x_dev is None:
            self._x_dev = torch.as_tensor(self._x_est.reshape(1, 4)).to(dev).contiguous()
        if self._u_dev is None:
            self._u_dev = torch.as_tensor(np.asarray(self.previous_u, dtype=np.float64).reshape(1, -1)).to(dev)
        y = torch.as_tensor(np.asarray(y0, dtype=np.float64).reshape(1, -1)).to(dev)
        qp.observe(y, self._x_dev, self._u_dev, self.C, self.L)
        x_ref, _u_ref = self.optimal_target_selection()
        Rf = torch.as_tensor(x_ref.reshape(1, 4)).to(dev)
        u_all, st, _ = qp.solve(self._x_dev, Rf, self.settings)
        x0 = self._x_dev[0].cpu().numpy()
        self._x_est = x0.copy()
        u = self._check_status(int(st.cpu()[0]), u_all[0].cpu().numpy())
        self._u_dev = u_all[:, :self.nu].contiguous()
        return self._finish_step(x0, x_ref, u)

    def _finish_step(self, x0, x_ref, u) -> np.ndarray:
        m = self._mats()
        dx = x0 - x_ref
        self.x_horizon = (m["T"] @ dx + m["S"] @ u).reshape(-1, self.nx) + self.goal      # mpc.py:484-485
        self.u_horizon = u.reshape(-1, 2)
        self.cost = 0.5 * u @ m["H"] @ u + (m["h"] @ dx) @ u                             # mpc.py:478,487
        self.previous_u = u[:self.nu]
        return u[:self.nu]


class MPCOutputFBWithDisturbance(MPC):
    """Output-feedback MPC with a constant scalar disturbance d (mpc.py:495-667):
        x+ = A x + B u + Bd d,   y = C x + Cd d,
    a disturbance-augmented Luenberger observer, and the QP of MPCStateFB with the predicted
    states shifted by ABd d (x = T x0 + S u + ABd d, mpc.py:631-650).  Observer and QP run on
    the GPU (carmpc_observer_dist_batch, carmpc_solve_batch_dist)."""

    C_OUT = MPCOutputFB.C_OUT
    BD = np.array([1.0, 1.0, 1.0, 1.0])       # mpc.py:536 (the value the constructor leaves)
    CD = np.array([1.0, 1.0, 1.0])            # mpc.py:537
    L1_GAIN = MPCOutputFB.L_GAIN              # mpc.py:541-544
    L2_GAIN = np.array([1.0, 1.0, 1.0])       # mpc.py:546
    X_REF = np.array([30.0, 1.5, 0.0, 0.0])   # mpc.py:624 (target selection commented out in step)

    def __init__(self, dt: float, N: int, lin_state: ArrayLike, lin_input: ArrayLike, init_state: ArrayLike,
                 terminal_constraint: bool = True, input_constraint: bool = True, state_constraint: bool = True,
                 env: BaseEnv = None, **kw) -> None:
        super().__init__(dt, N, lin_state, lin_input, terminal_constraint, input_constraint, state_constraint,
                         env, **kw)
        self.C = self.C_OUT.copy()
        self.Bd = self.BD.copy()
        self.Cd = self.CD.copy()
        self.C_hat = np.hstack((self.C, self.Cd.reshape(-1, 1)))                                   # mpc.py:538
        self.L1 = self.L1_GAIN.copy()
        self.L2 = self.L2_GAIN.copy()
        self.A_hat = np.vstack((np.hstack((self.A, self.Bd.reshape(-1, 1))),
                                np.array([0, 0, 0, 0, 1]).reshape(1, -1)))                       # mpc.py:548
        self.B_hat = np.vstack((self.B, [0, 0]))                                                 # mpc.py:549
        self.x_estimate = np.array(init_state, dtype=float)
        self.d_estimate = 0.0
        self.previous_u = np.zeros(2)
        self.y_goal = self.C @ env.goal                                                          # mpc.py:567
        self._dist_ready = False
        self.check_constraints()

    def _qp_dist(self):
        qp = self.qp
        if not self._dist_ready:
            qp.set_disturbance(self.Bd)
            self._dist_ready = True
        return qp

    def optimal_target_selection(self) -> tuple:
        """(x_ref, u_ref) with the disturbance (mpc.py:572-596): the equality block
        [[I-A, -B], [C, 0]] [x; u] = [Bd d; y_goal - Cd d] has full column rank for the Road*
        setups, so the feasible set is one point; solved in closed form (not called by step,
        as in the reference)."""
        M = np.block([[np.eye(self.nx) - self.A, -self.B], [self.C, np.zeros((self.C.shape[0], self.nu))]])
        rhs = np.concatenate((self.Bd * self.d_estimate, self.y_goal - self.Cd * self.d_estimate))
        if np.linalg.matrix_rank(M) < self.nx + self.nu:
            raise NotImplementedError("target selection with a non-unique equality solution")
        xu, *_ = np.linalg.lstsq(M, rhs, rcond=None)
        if np.abs(M @ xu - rhs).max() > 1e-9:
            raise OutsideTheRegionOfAttractionError("no steady state reaches y_goal")
        return xu[:self.nx], xu[self.nx:]

    def luenberger_observer(self, y0) -> tuple:
        """Host form of the disturbance observer (mpc.py:598-612, without its debug prints):
        e = y - C x_hat - Cd d_hat; x_hat+ = A x_hat + Bd d_hat + B u_prev + L1 e; d_hat+ = d_hat + L2 . e.
        ``step`` runs the same update on the GPU."""
        e = np.asarray(y0, float) - self.C @ self.x_estimate - self.Cd * self.d_estimate
        x_new = self.A @ self.x_estimate + self.Bd * self.d_estimate + self.B @ self.previous_u + self.L1 @ e
        return x_new, float(self.d_estimate + self.L2 @ e)

    def step_batch(self, y, xhat, dhat, uprev):
        """Observer + QP for a batch on the GPU: y (B x 3), xhat (B x 4), dhat (B,), uprev (B x 2)
        device float64 tensors; xhat and dhat are updated in place.
        Returns (u0 (B x nu), u (B x N nu), status (B,))."""
        import torch
        qp = self._qp_dist()
        qp.observe_dist(y, xhat, dhat, uprev, self.C, self.L1, self.Cd, self.L2, self.Bd)
        Rf = torch.as_tensor(self.X_REF, dtype=torch.float64, device=qp.device).expand(xhat.shape[0], 4).contiguous()
        u, st, _ = qp.solve(xhat, Rf, self.settings, dist=dhat)
        return u[:, :self.nu], u, st

    def step(self, y0) -> np.ndarray:
        """Observer -> QP with the disturbance offset (mpc.py:614-667), both on the GPU."""
        qp = self._qp_dist()
        if self.on_cpu:
            x0, d0 = self.luenberger_observer(np.asarray(y0, dtype=float))      # mpc.py:620
            self.x_estimate, self.d_estimate = x0.copy(), d0
            u_all, st, _ = qp.solve(x0.reshape(1, 4), self.X_REF.reshape(1, 4), self.settings, dist=np.array([d0]))
            u = self._check_status(int(st[0]), u_all[0])
            return self._finish_step(x0, u)
        import torch
        dev = qp.device
        xh = torch.as_tensor(self.x_estimate.reshape(1, 4)).to(dev).contiguous()
        dh = torch.tensor([float(self.d_estimate)], dtype=torch.float64, device=dev)
        up = torch.as_tensor(np.asarray(self.previous_u, dtype=np.float64).reshape(1, -1)).to(dev)
        y = torch.as_tensor(np.asarray(y0, dtype=np.float64).reshape(1, -1)).to(dev)
        _, u_all, st = self.step_batch(y, xh, dh, up)
        x0 = xh[0].cpu().numpy()
        self.x_estimate = x0.copy()
        self.d_estimate = float(dh.cpu()[0])
        u = self._check_status(int(st.cpu()[0]), u_all[0].cpu().numpy())
        return self._finish_step(x0, u)

    def _finish_step(self, x0, u) -> np.ndarray:
        m = self._mats()
        dx = x0 - self.X_REF
        self.x_horizon = (m["T"] @ dx + m["S"] @ u).reshape(-1, self.nx) + self.goal     # mpc.py:659-660
        self.u_horizon = u.reshape(-1, 2)
        self.cost = 0.5 * u @ m["H"] @ u + (m["h"] @ dx) @ u                            # mpc.py:639,653
        self.previous_u = u[:self.nu]
        return u[:self.nu]
