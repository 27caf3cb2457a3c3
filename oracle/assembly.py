"""numpy restatement of the reference's constructor-time QP assembly (ORACLE, tests only).

Every function cites the reference lines it restates.  Nothing here is used by
the product package; ``carmpc_amd`` performs the same assembly with its own
HIP kernel (``carmpc_amd/csrc/carmpc_assembly.hip``) and the tests compare the
two.

Notation: nx=4, nu=2, n=N*nu decision variables
``ubar=(u_0..u_{N-1})``; the reference QP at state x0 is

    min_u  1/2 u'Hu + (h (x0-goal))'u
    s.t.   A_t (T x0 + S u) <= b_t          terminal rows   (mpc.py:324-326)
           [I;-I] u <= [ub..;-lb..]         input box       (mpc.py:327-329)
           A_s (T x0 + S u) <= b_s          state rows      (mpc.py:330-332)

which we write as ``G u <= w0 - E x0`` (general rows: terminal then state) plus
``lb <= u <= ub``.
"""
from __future__ import annotations

import os
from dataclasses import dataclass, field

import numpy as np
from scipy.linalg import solve_discrete_are

# --- lib/configuration.py:4-21 -------------------------------------------------
DT_CONTROL = 0.2                       # configuration.py:4
DT_SIMULATION = DT_CONTROL             # configuration.py:7
STEPS_UPDATE = int(DT_CONTROL / DT_SIMULATION)  # configuration.py:9
LINEARIZE_STATE = [0, 0, 0, 3]         # configuration.py:12
LINEARIZE_INPUT = [0, 0]               # configuration.py:13
N_HORIZON = 20                         # configuration.py:16
STAGE_COST_Q = np.diag([5, 5, 10, 10])  # configuration.py:19
STAGE_COST_R = np.diag([10, 100])       # configuration.py:21

# --- lib/simulator.py:5-13 -----------------------------------------------------
L1 = 3.5                               # CarTrailerDimension.l1 (simulator.py:6)

# --- lib/environments.py: constraint rows, goals, names ------------------------
# name -> (constraints_A, constraints_b, goal)
ENVIRONMENTS = {
    # RoadEnv.__init__ environments.py:52-63
    "RoadEnv": ([[0, 1, 0, 0], [0, -1, 0, 0]], [3, 3], [30, 1.5, 0, 0]),
    # RoadOneCarEnv.__init__ environments.py:81-91 (inherits RoadEnv rows)
    "RoadOneCarEnv": ([[0, 1, 0, 0], [0, -1, 0, 0], [1, 0, 0, 0]], [3, 3, 30],
                      [29.9, -1.5, 0, 0]),
    # RoadMultipleCarsEnv.__init__ environments.py:118-128
    "RoadMultipleCarsEnv": ([[0, 1, 0, 0], [0, -1, 0, 0], [-0.25, 1, 0, 0], [0.25, -1, 0, 0]],
                            [3, 3, -2, 6.25], [30, 1.5, 0, 0]),
}
ENV_NAMES = tuple(ENVIRONMENTS)


def linearized_model(lin_state, lin_input):
    """Jacobians of the kinematic bicycle at (x_e, u_e).  Restates mpc.py:128-161."""
    lin_state = np.asarray(lin_state)
    lin_input = np.asarray(lin_input)
    assert lin_state.shape == (4,) and lin_input.shape == (2,)
    _x, _y, psi_e, v_e = lin_state
    _a, delta_e = lin_input
    A_lin = np.array([[0, 0, -v_e * np.sin(psi_e), np.cos(psi_e)],
                      [0, 0, v_e * np.cos(psi_e), np.sin(psi_e)],
                      [0, 0, 0, np.tan(delta_e) / L1],
                      [0, 0, 0, 0]])
    B_lin = np.array([[0, 0],
                      [0, 0],
                      [0, v_e / L1 * 1 / np.cos(delta_e) ** 2],
                      [1, 0]])
    return A_lin, B_lin


def discretized_model(A, B, dt):
    """Forward-Euler discretisation A_d = dt*A + I, B_d = dt*B.  Restates mpc.py:164-180."""
    assert len(A) == len(B)
    return dt * A + np.eye(len(A)), dt * B


def terminal_cost(A, B, Q, R):
    """P = DARE(A, B, Q, R), zeros on failure.  Restates mpc.py:67-74."""
    try:
        return solve_discrete_are(A, B, Q, R)
    except np.linalg.LinAlgError:
        return np.zeros((4, 4))


def predmod(A, B, N):
    """x_bar = T x0 + S u_bar.  Restates matrix_gen.py:6-32."""
    T = np.vstack([np.linalg.matrix_power(A, i) for i in range(N + 1)])
    S = np.hstack([np.vstack([np.linalg.matrix_power(A, i - j - 1) @ B if i - j - 1 >= 0
                              else np.zeros_like(B) for i in range(N + 1)]) for j in range(N)])
    return T, S


def stack_matrix_along_diag(A, N):
    """Block-diagonal repetition.  Restates matrix_gen.py:75-82."""
    i, j = A.shape
    out = np.zeros((i * N, j * N))
    for k in range(N):
        out[i * k:i * (k + 1), j * k:j * (k + 1)] = A
    return out


def costgen(Q, R, P, T, S, nx):
    """H = R_hat + S'Q_hat S, h = S'Q_hat T, const = T'Q_hat T.  Restates matrix_gen.py:35-72."""
    N = len(S) // nx - 1
    Q_hat = stack_matrix_along_diag(Q, N + 1)
    Q_hat[N * nx:(N + 1) * nx, N * nx:(N + 1) * nx] = P
    R_hat = stack_matrix_along_diag(R, N)
    H = R_hat + S.T @ Q_hat @ S
    h = S.T @ Q_hat @ T
    const = T.T @ Q_hat @ T
    return H, h, const


def terminal_set_filename(name, goal):
    """File-name rule ``name + '_'+str(g) per goal entry + '.npy'``.  Restates mpc.py:97
    (writer side: terminal_set.py:206)."""
    return name + "".join("_" + str(s) for s in goal) + ".npy"


@dataclass
class Assembly:
    """Everything MPC.__init__ (mpc.py:22-117) computes, plus the stacked QP data."""
    name: str
    N: int
    dt: float
    A: np.ndarray
    B: np.ndarray
    P: np.ndarray
    K: np.ndarray
    T: np.ndarray
    S: np.ndarray
    H: np.ndarray
    h: np.ndarray
    goal: np.ndarray
    input_upper: np.ndarray
    input_lower: np.ndarray
    state_rows_A: list          # per-step state half-spaces, base then env (mpc.py:89-93 + env)
    state_rows_b: list
    term_A: np.ndarray | None   # (k, 4(N+1)) acting on x_N only (mpc.py:103-105 / 112-117)
    term_b: np.ndarray | None
    term_file: str | None
    flags: tuple = (True, True, True)   # terminal, input, state
    # stacked QP pieces
    G: np.ndarray = field(default=None)   # general rows p x n  (terminal then state)
    E: np.ndarray = field(default=None)   # p x 4
    w0: np.ndarray = field(default=None)  # p
    row_stage: np.ndarray = field(default=None)  # stage k of each general row (x_k it acts on)
    row_coef: np.ndarray = field(default=None)   # p x 4 coefficient on x_k
    lb: np.ndarray = field(default=None)  # n  (None if no input box)
    ub: np.ndarray = field(default=None)


def input_constraint(N, nu, upper, lower):
    """[I; -I] u <= [ub...; -lb...].  Restates mpc.py:205-220."""
    A = np.vstack((np.eye(N * nu), -np.eye(N * nu)))
    b = np.vstack(((upper,) * N, (-lower,) * N)).flatten()
    return A, b


def state_constraint(N, nx, rows_A, rows_b):
    """Stacked per-step state rows on x_1..x_N, one block of N rows per half-space.
    Restates mpc.py:222-253 (base rows first, then env rows)."""
    A, b = [], []
    for A_con, b_con in zip(rows_A, rows_b):
        A_hat = np.zeros((N, (N + 1) * nx))
        for i in range(N):
            A_hat[i, (i + 1) * nx:(i + 2) * nx] = A_con
        A.append(A_hat)
        b.append(np.hstack(((b_con,) * N)))
    return np.vstack(A), np.hstack(b)


def build(env_name: str, N: int = N_HORIZON, dt: float = DT_CONTROL,
          lin_state=LINEARIZE_STATE, lin_input=LINEARIZE_INPUT,
          terminal_constraint=True, input_constraint_on=True, state_constraint_on=True,
          terminal_set_dir: str | None = None, goal=None) -> Assembly:
    """Restates MPC.__init__ (mpc.py:22-117) for one environment and stacks the QP rows
    the way MPCStateFB.step builds them (mpc.py:323-332)."""
    nx, nu = 4, 2
    cA, cb, env_goal = ENVIRONMENTS[env_name]
    goal_list = list(env_goal if goal is None else goal)
    A_lin, B_lin = linearized_model(np.array(lin_state), np.array(lin_input))   # mpc.py:53
    A, B = discretized_model(A_lin, B_lin, dt)                                   # mpc.py:54
    Q, R = STAGE_COST_Q, STAGE_COST_R                                            # mpc.py:60-61
    P = terminal_cost(A, B, Q, R)                                                # mpc.py:69-74
    T, S = predmod(A, B, N)                                                      # mpc.py:77
    H, h, _ = costgen(Q, R, P, T, S, nx)                                         # mpc.py:78
    K = -np.linalg.inv(R + B.T @ P @ B) @ B.T @ P @ A                            # mpc.py:81
    upper = np.array([2, np.pi / 8])                                             # mpc.py:84
    lower = -upper                                                               # mpc.py:85
    rows_A = [[0, 0, 1, 0], [0, 0, -1, 0], [0, 0, 0, 1], [0, 0, 0, -1]]          # mpc.py:89,92
    rows_b = [np.pi / 8, np.pi / 8, 5, 1]                                        # mpc.py:90,93
    rows_A = rows_A + [list(r) for r in cA]                                      # mpc.py:240-248
    rows_b = rows_b + list(cb)
    goal_arr = np.array(goal_list)
    term_A = term_b = term_file = None
    if terminal_constraint:                                                      # mpc.py:96-117
        fname = terminal_set_filename(env_name, goal_list)
        directory = terminal_set_dir if terminal_set_dir is not None else "../terminal_sets/"
        path = os.path.join(directory, fname)
        if os.path.exists(path):
            ts = np.load(path)
            A_hat = np.zeros((len(ts), (N + 1) * nx))
            A_hat[:, -4:] = ts[..., :4]
            term_A, term_b, term_file = A_hat, ts[..., 4], path
        else:
            Af = np.zeros((2 * nx, (N + 1) * nx))
            Af[0:nx, N * nx:(N + 1) * nx] = np.diag([1, 1, 1, 0])
            Af[nx:2 * nx, N * nx:(N + 1) * nx] = -np.diag([1, 1, 1, 0])
            term_A, term_b = Af, np.hstack((goal_arr, -goal_arr))
    asm = Assembly(env_name, N, dt, A, B, P, K, T, S, H, h, goal_arr, upper, lower,
                   rows_A, rows_b, term_A, term_b, term_file,
                   (terminal_constraint, input_constraint_on, state_constraint_on))
    stack_qp(asm)
    return asm


def stack_qp(asm: Assembly) -> None:
    """Condensed general rows G u <= w0 - E x0 (terminal first, then state), as the
    reference feeds them to cvxpy in mpc.py:323-332 with x = T x0 + S u (mpc.py:319)."""
    N, nx = asm.N, 4
    blocks_A, blocks_b, stage, coef = [], [], [], []
    term_on, input_on, state_on = asm.flags
    if term_on:
        blocks_A.append(asm.term_A)
        blocks_b.append(asm.term_b)
        stage.append(np.full(len(asm.term_b), N))
        coef.append(asm.term_A[:, N * nx:(N + 1) * nx])
    if state_on:
        As, bs = state_constraint(N, nx, asm.state_rows_A, asm.state_rows_b)
        blocks_A.append(As)
        blocks_b.append(bs)
        for r in asm.state_rows_A:
            stage.append(np.arange(1, N + 1))
            coef.append(np.tile(np.asarray(r, dtype=float), (N, 1)))
    if blocks_A:
        A_all = np.vstack(blocks_A)
        asm.G = A_all @ asm.S
        asm.E = A_all @ asm.T
        asm.w0 = np.hstack(blocks_b).astype(float)
        asm.row_stage = np.hstack(stage).astype(np.int32)
        asm.row_coef = np.vstack(coef).astype(float)
    else:
        n = N * 2
        asm.G = np.zeros((0, n)); asm.E = np.zeros((0, nx)); asm.w0 = np.zeros(0)
        asm.row_stage = np.zeros(0, np.int32); asm.row_coef = np.zeros((0, nx))
    if input_on:
        asm.ub = np.tile(asm.input_upper, N).astype(float)
        asm.lb = np.tile(asm.input_lower, N).astype(float)


def qp_data(asm: Assembly, x0, xref=None):
    """Per-instance QP vectors: q = h (x0 - xref) (mpc.py:320-321), w = w0 - E x0 (mpc.py:319,326,332)."""
    x0 = np.asarray(x0, float)
    xref = asm.goal if xref is None else np.asarray(xref, float)
    q = asm.h @ (x0 - xref)
    w = asm.w0 - asm.E @ x0
    return q, w


# --- lib/mpc.py:387-404 (MPCOutputFB observer) ---------------------------------
C_OUT = np.array([[1, 0, 0, 0], [0, 1, 0, 0], [0, 0, 0, 1]])    # mpc.py:387-389
L_OBS = np.array([[3.00000000e-01, 2.00284502e-16, 2.00000000e-01],   # mpc.py:401-404
                  [3.48682242e+00, 1.90000000e+00, 3.86733776e-01],
                  [1.74341121e+00, 8.00000000e-01, 1.93366888e-01],
                  [-3.36822969e-16, -2.07305381e-16, 3.00000000e-01]])


def luenberger_observer(A, B, x_est, u_prev, y0, C=C_OUT, L=L_OBS):
    """x_hat+ = A x_hat + B u_prev + L (y - C x_hat).  Restates mpc.py:439-448."""
    return A @ x_est + B @ u_prev + L @ (y0 - C @ x_est)


def optimal_target_selection(A, B, y_goal, C=C_OUT):
    """Closed form of the OTS QP (mpc.py:413-437) when its 7x6 equality block
    [[I-A, -B],[C, 0]] [x;u] = [0; y_goal] has full column rank (all Road* goals):
    the unique feasible point is the least-squares solution."""
    M = np.hstack((np.vstack((np.eye(4) - A, C)), np.vstack((-B, np.zeros((C.shape[0], 2))))))
    rhs = np.hstack((np.zeros(4), y_goal))
    assert np.linalg.matrix_rank(M) == 6
    xu = np.linalg.lstsq(M, rhs, rcond=None)[0]
    return xu[:4], xu[4:]


# --- lib/mpc.py:495-667 (MPCOutputFBWithDisturbance) --------------------------
# x+ = A x + B u + Bd d,  y = C x + Cd d, d a scalar disturbance (mpc.py:508-512); the
# constants below are the values the constructor leaves in place (the second assignments,
# mpc.py:536-537), the observer gains of mpc.py:541-546 and the hard-coded reference of
# step() (mpc.py:624: the target selection call is commented out there).
BD_DIST = np.array([1.0, 1.0, 1.0, 1.0])                       # mpc.py:536
CD_DIST = np.array([1.0, 1.0, 1.0])                            # mpc.py:537
L1_DIST = L_OBS.copy()                                         # mpc.py:541-544
L2_DIST = np.array([1.0, 1.0, 1.0])                            # mpc.py:546
XREF_DIST = np.array([30.0, 1.5, 0.0, 0.0])                    # mpc.py:624


def disturbance_observer(A, B, x_est, d_est, u_prev, y0, C=C_OUT, Bd=BD_DIST, Cd=CD_DIST, L1=L1_DIST,
                         L2=L2_DIST):
    """(x_hat+, d_hat+) of the disturbance-augmented Luenberger observer.  Restates
    mpc.py:598-612 (without its debug prints): innovation e = y - C x_hat - Cd d_hat,
    x_hat+ = A x_hat + Bd d_hat + B u_prev + L1 e,  d_hat+ = d_hat + L2 . e."""
    e = np.asarray(y0, float) - C @ x_est - Cd * d_est
    return A @ x_est + Bd * d_est + B @ u_prev + L1 @ e, float(d_est + L2 @ e)


def abd_offsets(A, Bd, N):
    """ABd_k = sum_{m<k} A^m Bd, k = 0..N: the predicted-state offset of a constant
    disturbance, x = T x0 + S u + ABd d (mpc.py:631-637)."""
    out = np.zeros((N + 1, 4))
    acc = np.zeros(4)
    Am = np.eye(4)
    for k in range(1, N + 1):
        acc = acc + Am @ Bd
        Am = A @ Am
        out[k] = acc
    return out


def qp_data_dist(asm: Assembly, x0, d, xref=XREF_DIST, Bd=BD_DIST):
    """Per-instance QP vectors of MPCOutputFBWithDisturbance.step (mpc.py:630-650):
    q = h (x0 - xref), w = w0 - E x0 - (rows . ABd_k) d (constraints act on x with the offset)."""
    x0 = np.asarray(x0, float)
    q = asm.h @ (x0 - np.asarray(xref, float))
    abd = abd_offsets(asm.A, Bd, asm.N)
    Ed = np.einsum("ra,ra->r", asm.row_coef, abd[asm.row_stage]) if len(asm.w0) else np.zeros(0)
    w = asm.w0 - asm.E @ x0 - Ed * float(d)
    return q, w, Ed


# --- lib/simulator.py:51-69,83-118 (plant) ------------------------------------
def plant_step(state, u, dt=DT_SIMULATION, l1=L1):
    """Forward-Euler kinematic bicycle.  Restates simulator.py:51-69."""
    x, y, psi, v = state
    a, delta = u
    t = np.tan(delta)
    return np.array([v * np.cos(psi), v * np.sin(psi), v / l1 * t, a]) * dt + state
