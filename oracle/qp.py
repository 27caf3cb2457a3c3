"""numpy restatement of the per-step QP and its solution (ORACLE, tests only).

The reference solves, every control step, the strictly convex QP built in
``lib/mpc.py:318-335`` (MPCStateFB.step) / ``lib/mpc.py:461-478`` (MPCOutputFB.step)
with cvxpy.  cvxpy (and its default backend) is absent in this image and
unpinned upstream, so the QP arithmetic cannot be run from the reference; see
``oracle/__init__.py`` for how parity is anchored instead.

This module provides
  * ``ipm``        -- the dense Mehrotra predictor-corrector IPM (the algorithm
                      the HIP kernels implement),
                      vectorised numpy, one instance at a time;
  * ``certify``    -- an independent active-set KKT polish + certificate: returns
                      the exact optimum (to ~1e-13) and the KKT residuals, so a
                      solution is judged against the *unique* optimum, not
                      against another IPM;
  * ``lp_margin``  -- the HiGHS LP max-slack margin t* = max{t : G u + t <= w,
                      lb <= u <= ub}; t* >= 0 <=> feasible.  Ground truth for the
                      optimal / primal-infeasible status (mpc.py:336-338).
"""
from __future__ import annotations

import numpy as np
from scipy.optimize import linprog

STATUS_OPTIMAL, STATUS_INFEASIBLE, STATUS_MAXITER, STATUS_NUMERICAL = 0, 1, 2, 3
STATUS_NAMES = {0: "optimal", 1: "primal_infeasible", 2: "max_iter", 3: "numerical"}

# Settings shared with oracle/ipm.c and carmpc_amd/csrc
TOL_RES = 1e-10
TOL_MU = 1e-12
MAX_ITER = 60
STEP_FRAC = 0.99
REFINE = 1                 # iterative-refinement passes on the corrector direction
REFINE_MU = 1e-6           # ... only once mu <= REFINE_MU (D = z/s spans many decades)
POLISH_MU = 1e-2           # attempt the active-set polish once mu <= POLISH_MU ...
POLISH_RES = 2e-4          # ... and both residuals are within max(POLISH_RES, tol), relative.  An accepted
#                            polish is the exact optimum whenever it comes; the gate trades iterations for
#                            rejected attempts (most are repaired by the correction round).
# Initial point: slacks s = max(w - G u0, INIT_SFLOOR), multipliers on the central path, z = mu0 / s with
# mu0 = clamp((|q|_inf / (INIT_Q_PER_VAR n))^2, INIT_MU_MIN, INIT_MU0): a centred start whose distance from the
# boundary follows the size of the linear term -- far from the goal well inside the cone (about 1.3
# iterations fewer than z = 1 with the floor at 1), on closed-loop trajectories and near the goal close to
# it (3 to 4 iterations, as before; a fixed mu0 = 100 costs 5 there).
INIT_MU0 = 100.0
INIT_MU_MIN = 1.0
INIT_Q_PER_VAR = 3.5       # (the best scale grows with the horizon: about 140 at N = 20, 70 at N = 10, 35 at N = 5)
INIT_SFLOOR = 2.0
# First active set of a polish: the rows with s < POLISH_ACT z -- a conservative guess (few rows, the correction
# round adds the violated ones) is accepted far more often than s < z.
POLISH_ACT = 0.003
# the variant the fallback kernels (dense, staged, per-instance) run: z = 1 and slack floor 1 at the start,
# one polish attempt behind the conservative gate
FALLBACK_VARIANT = dict(polish_corrections=0, polish_mu=1e-6, polish_res=0.0, init_mu0=0.0, init_sfloor=1.0,
                        polish_refine=3, polish_act=1.0)
POLISH_DELTA = 1e-10        # regularisation of the polish KKT system
POLISH_REFINE = 2          # iterative-refinement passes of the polish (2: |u - u*| ~ 1e-10, same acceptances as 3)
POLISH_TOL = 1e-11         # acceptance: primal violation and negative multipliers, relative
POLISH_CORRECTIONS = 1     # correction rounds of a rejected polish (0: the single-attempt polish of the fallback kernels)
UNBOXED_BOUND = 1e9        # |u_i| bound assumed by the Farkas test for unboxed variables
PRE_TOL = 1e-9             # zero-row precondition tolerance
ZERO_ROW = 1e-12           # rows with ||G_r||_2 <= ZERO_ROW * max_r ||G_r||_2 are x0-only rows


def normalize_rows(G, w0, E):
    """Split general rows into QP rows (unit 2-norm) and x0-only rows (G_r == 0).
    Returns (Gn, w0n, En, keep_mask, pre_w0, pre_E)."""
    nrm = np.linalg.norm(G, axis=1) if G.size else np.zeros(len(w0))
    thr = ZERO_ROW * (nrm.max() if nrm.size else 0.0)
    keep = nrm > thr
    inv = 1.0 / nrm[keep]
    return (G[keep] * inv[:, None], w0[keep] * inv, E[keep] * inv[:, None], keep,
            w0[~keep], E[~keep])


def opposite_pairs(G, w0, E):
    """partner[r] = r' if row r' is the exact negation of row r (G, w0 and E), else -1.

    Such a pair writes an equality c'x = b as two inequalities -- the reference's
    fallback terminal set x_N = goal (lib/mpc.py:107-117) does exactly that.  When both
    rows are active the polish may re-split their multipliers."""
    p = G.shape[0]
    partner = np.full(p, -1, dtype=np.int32)
    if p == 0:
        return partner
    rows = np.hstack([G, np.asarray(w0, float).reshape(-1, 1), E]) + 0.0   # + 0.0: -0.0 -> 0.0
    neg = -rows + 0.0
    key = {}
    for r in range(p):
        key.setdefault(rows[r].tobytes(), r)
    for r in range(p):
        r2 = key.get(neg[r].tobytes())
        if r2 is not None and r2 != r:
            partner[r] = r2
    return partner


def ipm(H, q, G, w, lb=None, ub=None, tol=TOL_RES, tol_mu=TOL_MU, max_iter=MAX_ITER,
        trace=None, refine=REFINE, polish=True, info=None, partner=None, polish_corrections=None,
        polish_mu=None, polish_res=None, init_mu0=None, init_sfloor=None, polish_refine=None, polish_act=None):
    """Dense Mehrotra IPM for  min 1/2 u'Hu + q'u  s.t. G u <= w, lb <= u <= ub.

    G rows must be normalised (``normalize_rows``).  lb/ub None => no box.
    ``partner`` (``opposite_pairs``) marks rows that together form an equality.
    Returns (u, status, iterations, z_g)."""
    n = len(q)
    p = G.shape[0]
    boxed = lb is not None
    if boxed:
        lb = np.asarray(lb, float); ub = np.asarray(ub, float)
        blo, bhi = lb, ub
        u = np.clip(np.zeros(n), lb, ub)
    else:
        blo = np.full(n, -UNBOXED_BOUND); bhi = np.full(n, UNBOXED_BOUND)
        u = np.zeros(n)
    nb = n if boxed else 0
    m = p + 2 * nb
    mu0 = INIT_MU0 if init_mu0 is None else init_mu0
    if mu0 > 0:
        qrel = (1.0 / (INIT_Q_PER_VAR * n)) * (np.abs(q).max() if n else 0.0)
        mu0 = min(mu0, max(INIT_MU_MIN, qrel * qrel))
    sfl = INIT_SFLOOR if init_sfloor is None else init_sfloor
    s = np.maximum(w - G @ u, sfl); z = mu0 / s if mu0 > 0 else np.ones(p)
    if boxed:
        su = np.maximum(ub - u, sfl); sl = np.maximum(u - lb, sfl)
    else:
        su = np.ones(0); sl = np.ones(0)
    zu = mu0 / su if mu0 > 0 else np.ones(nb)
    zl = mu0 / sl if mu0 > 0 else np.ones(nb)
    bnorm = 1.0 + max(np.abs(w).max() if p else 0.0,
                      np.abs(ub).max() if boxed else 0.0, np.abs(lb).max() if boxed else 0.0)
    qnorm = 1.0 + (np.abs(q).max() if n else 0.0)
    bound_abs = np.maximum(np.abs(blo), np.abs(bhi))

    def box_T(vu, vl):  # contribution of box rows to A'v
        return (vu - vl) if boxed else 0.0

    for it in range(max_iter):
        Gu = G @ u
        rp = Gu + s - w
        rpu = (u + su - ub) if boxed else su
        rpl = (-u + sl + lb) if boxed else sl
        rd = H @ u + q + G.T @ z + box_T(zu, zl)
        mu = (s @ z + su @ zu + sl @ zl) / max(m, 1)
        rpn = max(np.abs(rp).max() if p else 0.0, np.abs(rpu).max() if nb else 0.0,
                  np.abs(rpl).max() if nb else 0.0)
        rdn = np.abs(rd).max()
        # tolerances scale with the magnitude of the terms each residual sums (roundoff floor)
        Hu = H @ u; Gtz = G.T @ z
        pscale = max(bnorm, 1.0 + (np.abs(Gu).max() if p else 0.0), 1.0 + (np.abs(u).max() if nb else 0.0))
        dscale = max(qnorm, 1.0 + np.abs(Hu).max(), 1.0 + np.abs(Gtz + box_T(zu, zl)).max())
        if trace is not None:
            trace.append((it, mu, rpn, rdn))
        if not np.isfinite(mu) or not np.isfinite(rdn):
            return u, STATUS_NUMERICAL, it, z
        ptol = max(POLISH_RES if polish_res is None else polish_res, tol)
        pmu = POLISH_MU if polish_mu is None else polish_mu
        if polish and rpn <= ptol * pscale and rdn <= ptol * dscale and mu <= pmu:
            up, ok = polish_step(H, q, G, w, lb if boxed else None, ub if boxed else None, s, z, su, zu, sl, zl,
                                 partner=partner, corrections=polish_corrections,
                                 refine=POLISH_REFINE if polish_refine is None else polish_refine, act=polish_act)
            if info is not None:
                info.setdefault("polish", []).append((it, ok))
            if ok:
                return up, STATUS_OPTIMAL, it, z
        if rpn <= tol * pscale and rdn <= tol * dscale and mu <= tol_mu:
            return u, STATUS_OPTIMAL, it, z
        # Farkas test: for every u in the box, (G'z)'u >= lo; if lo > w'z then no u
        # satisfies G u <= w (z >= 0).  Rigorous when all variables are boxed.
        if p:
            c = G.T @ z
            lo = np.minimum(c * blo, c * bhi).sum()
            wz = w @ z
            if lo - wz > 1e-12 * (np.abs(c) @ bound_abs + np.abs(w) @ z):
                return u, STATUS_INFEASIBLE, it, z
        d = z / s
        M = H + (G.T * d) @ G
        if boxed:
            M[np.diag_indices(n)] += zu / su + zl / sl
        Lc = _chol_guarded(M)

        def solve(rc, rcu, rcl):
            t = (rc - z * rp) / s
            rhs = -rd + G.T @ t
            if boxed:
                rhs = rhs + (rcu - zu * rpu) / su - (rcl - zl * rpl) / sl
            du = _chol_solve(Lc, rhs)
            ds = -rp - G @ du
            dz = (-rc - z * ds) / s
            if boxed:
                dsu = -rpu - du; dsl = -rpl + du
                dzu = (-rcu - zu * dsu) / su; dzl = (-rcl - zl * dsl) / sl
            else:
                dsu = dsl = dzu = dzl = np.zeros(0)
            return du, ds, dz, dsu, dzu, dsl, dzl

        du, ds, dz, dsu, dzu, dsl, dzl = solve(s * z, su * zu, sl * zl)
        a_aff = min(1.0, _maxstep(s, ds), _maxstep(z, dz), _maxstep(su, dsu),
                    _maxstep(zu, dzu), _maxstep(sl, dsl), _maxstep(zl, dzl))
        mu_aff = ((s + a_aff * ds) @ (z + a_aff * dz) + (su + a_aff * dsu) @ (zu + a_aff * dzu)
                  + (sl + a_aff * dsl) @ (zl + a_aff * dzl)) / max(m, 1)
        sigma = (mu_aff / mu) ** 3
        smu = sigma * mu
        du, ds, dz, dsu, dzu, dsl, dzl = solve(s * z + ds * dz - smu, su * zu + dsu * dzu - smu,
                                               sl * zl + dsl * dzl - smu)
        for _ in range(refine if mu <= REFINE_MU else 0):
            # residual of the dual equation H du + A'dz = -rd for the reconstructed direction;
            # correct with the same factor: M dU = -e, dS = -A dU, dZ = -z dS / s
            e = H @ du + G.T @ dz + rd + (box_T(dzu, dzl) if boxed else 0.0)
            cu = _chol_solve(Lc, -e)
            cs = -(G @ cu)
            du = du + cu; ds = ds + cs; dz = dz - z * cs / s
            if boxed:
                dsu = dsu - cu; dzu = dzu + zu * cu / su
                dsl = dsl + cu; dzl = dzl - zl * cu / sl
        a = min(1.0, STEP_FRAC * min(_maxstep(s, ds), _maxstep(z, dz), _maxstep(su, dsu),
                                     _maxstep(zu, dzu), _maxstep(sl, dsl), _maxstep(zl, dzl)))
        u = u + a * du; s = s + a * ds; z = z + a * dz
        su = su + a * dsu; zu = zu + a * dzu; sl = sl + a * dsl; zl = zl + a * dzl
    if polish:
        up, ok = polish_step(H, q, G, w, lb if boxed else None, ub if boxed else None, s, z, su, zu, sl, zl,
                             partner=partner, corrections=polish_corrections,
                             refine=POLISH_REFINE if polish_refine is None else polish_refine, act=polish_act)
        if ok:
            return up, STATUS_OPTIMAL, max_iter, z
    return u, STATUS_MAXITER, max_iter, z


def polish_step(H, q, G, w, lb, ub, s, z, su, zu, sl, zl, delta=POLISH_DELTA, refine=POLISH_REFINE,
                partner=None, corrections=None, act=None):
    """Active-set polish.  Active set from the IPM iterate (s < z); solve the
    equality-constrained KKT [[H, A'], [A, 0]] [x; y] = [-q; b_act] by iterative refinement on
    the regularised factor  H + A'A/delta  (the IPM's M with d = 1/delta on active rows, 0 else);
    accept only if x is primal feasible and the active multipliers are nonnegative.  Rows whose
    opposite partner is also active form an equality: their multipliers can be re-split as
    (max(y-y',0), max(y'-y,0)) without changing A'y, so they are exempt from the sign test.

    Correction rounds (POLISH_CORRECTIONS): a rejected attempt names what is wrong with its
    active set -- active rows whose multiplier fails the sign test, inactive rows that are
    violated -- and the polish is repeated on the set with those rows dropped / added.  A
    rejection with nothing to change, or of the last round, stands."""
    n = len(q)
    boxed = lb is not None
    if corrections is None:
        corrections = POLISH_CORRECTIONS
    act = POLISH_ACT if act is None else act
    ag = s < act * z
    au = su < act * zu if boxed else np.zeros(n, bool)
    al = sl < act * zl if boxed else np.zeros(n, bool)
    x = np.zeros(n)
    for attempt in range(corrections + 1):
        x, ok, fix = _polish_attempt(H, q, G, w, lb, ub, ag, au, al, delta, refine, partner)
        if ok or fix is None or attempt == corrections:
            return x, ok
        nag, nau, nal = fix
        if np.array_equal(nag, ag) and np.array_equal(nau, au) and np.array_equal(nal, al):
            return x, False
        ag, au, al = nag, nau, nal
    return x, False


def _polish_attempt(H, q, G, w, lb, ub, ag, au, al, delta, refine, partner):
    """One polish on the active set (ag rows, au / al upper / lower bounds).  Returns x, the outcome
    of the acceptance test and, for a rejected finite x, the corrected active set."""
    n = len(q)
    boxed = lb is not None
    dg = np.where(ag, 1.0 / delta, 0.0)
    M = H + (G.T * dg) @ G
    if boxed:
        du_ = np.where(au, 1.0 / delta, 0.0); dl_ = np.where(al, 1.0 / delta, 0.0)
        M[np.diag_indices(n)] += du_ + dl_
    else:
        du_ = dl_ = np.zeros(n)
    L = _chol_guarded(M)
    bg = np.where(ag, w, 0.0)
    bu = np.where(au, ub, 0.0) if boxed else np.zeros(n)
    bl = np.where(al, lb, 0.0) if boxed else np.zeros(n)

    def At(yg, yu, yl):
        return G.T @ yg + yu - yl

    def ksolve(rx, ryg, ryu, ryl):
        # [[H, A'], [A, -delta I]] on the active rows: dy = (A dx - ry)/delta
        dx = _chol_solve(L, rx + At(dg * ryg, du_ * ryu, dl_ * ryl))
        return dx, dg * (G @ dx - ryg), du_ * (dx - ryu), dl_ * (-dx - ryl)

    x, yg, yu, yl = ksolve(-q, bg, bu, -bl)
    for _ in range(refine):
        rx = -q - H @ x - At(yg, yu, yl)
        ryg = np.where(ag, bg - G @ x, 0.0)
        ryu = np.where(au, bu - x, 0.0)
        ryl = np.where(al, -bl + x, 0.0)
        dx, dyg, dyu, dyl = ksolve(rx, ryg, ryu, ryl)
        x = x + dx; yg = yg + dyg; yu = yu + dyu; yl = yl + dyl
    wscale = 1.0 + max(np.abs(w).max() if len(w) else 0.0, np.abs(ub).max() if boxed else 0.0,
                       np.abs(lb).max() if boxed else 0.0)
    gxw = G @ x - w
    viol = max(gxw.max() if len(w) else -np.inf, (x - ub).max() if boxed else -np.inf,
               (lb - x).max() if boxed else -np.inf)
    paired = np.zeros(len(yg), bool)
    if partner is not None and len(yg):
        paired = ag & (partner >= 0) & ag[np.maximum(partner, 0)]
    yg_sign = np.where(paired, 0.0, yg)
    ymin = min(yg_sign.min() if len(yg) else 0.0, yu.min() if boxed else 0.0, yl.min() if boxed else 0.0)
    yscale = 1.0 + max(np.abs(yg).max() if len(yg) else 0.0, np.abs(yu).max() if boxed else 0.0,
                       np.abs(yl).max() if boxed else 0.0)
    finite = bool(np.all(np.isfinite(x)))
    vtol, ytol = POLISH_TOL * wscale, -POLISH_TOL * yscale
    ok = bool(viol <= vtol and ymin >= ytol and finite)
    if ok or not finite:
        return x, ok, None
    nag = np.where(ag, ~(~paired & (yg < ytol)), gxw > vtol)
    nau, nal = au, al
    if boxed:
        nau = np.where(au, ~(yu < ytol), x - ub > vtol)
        nal = np.where(al, ~(yl < ytol), lb - x > vtol)
    return x, ok, (nag, nau, nal)


def _maxstep(v, dv):
    neg = dv < 0
    if not neg.any():
        return np.inf
    return float(np.min(-v[neg] / dv[neg]))


def _chol_guarded(M):
    """Right-looking Cholesky; a non-positive pivot is replaced by 1e128 (its
    direction is frozen) -- the same guard as oracle/ipm.c and the HIP kernel."""
    n = M.shape[0]
    L = np.array(M, dtype=float)
    for k in range(n):
        piv = L[k, k]
        if not piv > 0:
            piv = 1e128
        lkk = np.sqrt(piv)
        L[k, k] = lkk
        L[k + 1:, k] /= lkk
        L[k + 1:, k + 1:] -= np.outer(L[k + 1:, k], L[k + 1:, k])
    return np.tril(L)


def _chol_solve(L, b):
    from scipy.linalg import solve_triangular
    y = solve_triangular(L, b, lower=True)
    return solve_triangular(L.T, y, lower=False)


def certify(H, q, G, w, lb, ub, u_hint, act_tol=1e-7):
    """Active-set KKT polish + certificate.

    Takes the active set suggested by ``u_hint`` (rows with slack <= act_tol*(1+|b|)),
    solves the equality-constrained KKT system exactly, and reports
    (u_exact, certified, residuals) with residuals = (max primal violation,
    min multiplier, max stationarity residual).  certified <=> violation <= 1e-9,
    multipliers >= -1e-9, stationarity <= 1e-9 * (1 + |q|)."""
    n = len(q)
    rows = [G]; rhs = [w]
    if lb is not None:
        rows += [np.eye(n), -np.eye(n)]; rhs += [ub, -lb]
    A = np.vstack(rows); b = np.hstack(rhs)
    best = None
    for tol in (act_tol, 1e-9, 1e-6, 1e-5):
        slack = b - A @ u_hint
        act = np.where(slack <= tol * (1 + np.abs(b)))[0]
        Aa = A[act]; k = len(act)
        KKT = np.block([[H, Aa.T], [Aa, np.zeros((k, k))]])
        sol = np.linalg.lstsq(KKT, np.hstack([-q, b[act]]), rcond=None)[0]
        ue, lam = sol[:n], sol[n:]
        viol = float(max((A @ ue - b).max(), 0.0)) if len(b) else 0.0
        # active opposite pairs (an equality written as two rows): re-split the multipliers
        part = opposite_pairs(Aa, b[act], np.zeros((k, 0))) if k else np.zeros(0, np.int32)
        lam_s = lam.copy()
        for i in np.where(part >= 0)[0]:
            lam_s[i] = max(lam[i] - lam[part[i]], 0.0)
        lmin = float(lam_s.min()) if k else 0.0
        stn = float(np.abs(H @ ue + q + Aa.T @ lam_s).max())
        ok = viol <= 1e-9 and lmin >= -1e-9 and stn <= 1e-9 * (1 + np.abs(q).max())
        if ok:
            return ue, True, (viol, lmin, stn)
        if best is None:
            best = (ue, False, (viol, lmin, stn))
    return best


def lp_margin(G, w, lb, ub, cap=1.0):
    """HiGHS: t* = max t s.t. G u + t 1 <= w, lb <= u <= ub, t <= cap.
    Feasible iff t* >= 0 (G rows normalised => t* is a Euclidean slack)."""
    n = G.shape[1]
    c = np.zeros(n + 1); c[-1] = -1.0
    A = np.hstack([G, np.ones((G.shape[0], 1))])
    bounds = ([(l, h) for l, h in zip(lb, ub)] if lb is not None else [(None, None)] * n) + [(None, cap)]
    r = linprog(c, A_ub=A, b_ub=w, bounds=bounds, method="highs")
    if r.status != 0:
        raise RuntimeError(f"HiGHS failed: {r.message}")
    return float(r.x[-1])


def solve_instance(asm, x0, xref=None, info=None, **kw):
    """Full per-step oracle for one instance of an ``assembly.Assembly``:
    preconditions on x0-only rows, normalised IPM, certificate.
    Returns dict(status, iters, u, u_exact, certified, margin)."""
    from .assembly import qp_data
    q, w = qp_data(asm, x0, xref)
    Gn, w0n, En, keep, pre_w0, pre_E = normalize_rows(asm.G, asm.w0, asm.E)
    x0 = np.asarray(x0, float)
    wn = w0n - En @ x0
    pre = pre_w0 - pre_E @ x0
    out = dict(q=q, w=wn)
    if pre.size and pre.min() < -PRE_TOL:
        out.update(status=STATUS_INFEASIBLE, iters=0, u=np.zeros(len(q)), u_exact=None,
                   certified=False, margin=float(pre.min()))
        return out
    kw.setdefault("partner", opposite_pairs(Gn, w0n, En))
    u, st, it, _ = ipm(asm.H, q, Gn, wn, asm.lb, asm.ub, info=info, **kw)
    out.update(status=st, iters=it, u=u)
    if st == STATUS_OPTIMAL:
        ue, ok, res = certify(asm.H, q, Gn, wn, asm.lb, asm.ub, u)
        out.update(u_exact=ue, certified=ok, kkt=res)
    else:
        out.update(u_exact=None, certified=False)
    return out


def solve_instance_dist(asm, x0, d, xref=None, Bd=None, **kw):
    """Oracle for MPCOutputFBWithDisturbance.step's QP (mpc.py:630-656): the rows read
    w = w0 - E x0 - Ed d with Ed_r = c_r . ABd_{k_r} (assembly.qp_data_dist), the cost uses
    x0 - xref.  Same preconditions / normalisation / IPM / certificate as solve_instance."""
    from .assembly import BD_DIST, XREF_DIST, qp_data_dist
    xref = XREF_DIST if xref is None else xref
    q, w, Ed = qp_data_dist(asm, x0, d, xref, BD_DIST if Bd is None else Bd)
    nrm = np.linalg.norm(asm.G, axis=1) if asm.G.size else np.zeros(len(asm.w0))
    thr = ZERO_ROW * (nrm.max() if nrm.size else 0.0)
    keep = nrm > thr
    Gn, w0n, En, _, _, _ = normalize_rows(asm.G, asm.w0, asm.E)
    wn = w[keep] / nrm[keep]
    out = dict(q=q, w=wn)
    pre = w[~keep]
    if pre.size and pre.min() < -PRE_TOL:
        out.update(status=STATUS_INFEASIBLE, iters=0, u=np.zeros(len(q)), u_exact=None, certified=False)
        return out
    kw.setdefault("partner", opposite_pairs(Gn, w0n, En))
    u, st, it, _ = ipm(asm.H, q, Gn, wn, asm.lb, asm.ub, **kw)
    out.update(status=st, iters=it, u=u)
    if st == STATUS_OPTIMAL:
        ue, ok, res = certify(asm.H, q, Gn, wn, asm.lb, asm.ub, u)
        out.update(u_exact=ue, certified=ok, kkt=res)
    else:
        out.update(u_exact=None, certified=False)
    return out
