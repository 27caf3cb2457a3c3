"""Stage-form (Riccati) restatement of the per-step QP IPM (ORACLE, tests only).

Same algorithm, tolerances and trip structure as ``oracle/qp.py::ipm``:
the Newton system  M du = b,  M = H + G'DG + diag(box),  is the KKT system of a
linear-quadratic problem over the horizon, because every QP row of the reference acts
on ONE predicted state (``lib/mpc.py:196-253``: terminal rows on x_N, state rows on
x_1..x_N) and  H = R_hat + S'Q_hat S  (``lib/matrix_gen.py:35-72``, S from
``matrix_gen.py:6-32``).  With y_k = S_k v (y_0 = 0, y_{k+1} = A y_k + B v_k),

    v'Mv = sum_t v_t'(R + Db_t) v_t + sum_{k>=1} y_k'(Qbar_k + W_k) y_k,
    W_k  = sum_{r in k} d_r c_r c_r',

so M^{-1} b is a backward Riccati recursion plus a forward roll-out
(``riccati_factor`` / ``riccati_solve``) instead of a dense n x n Cholesky.  Right-hand
sides are kept in stage form  b = b^u + sum_k S_k' b^x_k, so the adjoints G'(.) and
S'Qbar(.) never have to be formed in u-space.  This is the arithmetic of the grouped
HIP kernel (``carmpc_amd/csrc/ipm_riccati.hip``); the tests check that it follows
``qp.ipm`` step for step (same status and iteration count, u to ~1e-9).
"""
from __future__ import annotations

import numpy as np

from .qp import (INIT_MU0, INIT_MU_MIN, INIT_Q_PER_VAR, INIT_SFLOOR, MAX_ITER, POLISH_ACT, POLISH_CORRECTIONS, POLISH_DELTA, POLISH_MU, POLISH_RES, POLISH_REFINE, POLISH_TOL, PRE_TOL, REFINE_MU, STEP_FRAC,
                 STATUS_INFEASIBLE, STATUS_MAXITER, STATUS_NUMERICAL, STATUS_OPTIMAL, TOL_MU, TOL_RES,
                 UNBOXED_BOUND, ZERO_ROW, _maxstep, opposite_pairs)


class StageQP:
    """Stage data of one assembled problem (oracle.assembly.Assembly), rows normalised
    exactly as ``qp.normalize_rows`` does (unit 2-norm of the condensed row)."""

    def __init__(self, asm):
        self.N = asm.N
        self.A = np.asarray(asm.A, float)
        self.B = np.asarray(asm.B, float)
        from .assembly import STAGE_COST_Q, STAGE_COST_R
        Q = np.asarray(STAGE_COST_Q, float)
        P = np.asarray(asm.P, float)
        self.R = 0.5 * (np.asarray(STAGE_COST_R, float) + np.asarray(STAGE_COST_R, float).T)
        self.Qbar = [None] + [0.5 * (Q + Q.T)] * (self.N - 1) + [0.5 * (P + P.T)]   # k = 1..N
        self.h = asm.h
        G, w0, E = asm.G, asm.w0, asm.E
        nrm = np.linalg.norm(G, axis=1) if G.size else np.zeros(len(w0))
        thr = ZERO_ROW * (nrm.max() if nrm.size else 0.0)
        keep = nrm > thr
        inv = 1.0 / nrm[keep]
        self.stage = np.asarray(asm.row_stage)[keep]
        self.coef = np.asarray(asm.row_coef, float)[keep] * inv[:, None]
        self.w0 = w0[keep] * inv
        self.E = E[keep] * inv[:, None]
        self.Gn = G[keep] * inv[:, None]
        self.pre_w0, self.pre_E = w0[~keep], E[~keep]
        self.partner = opposite_pairs(self.Gn, self.w0, self.E)
        self.lb, self.ub = asm.lb, asm.ub
        self.n = 2 * self.N
        self.p = len(self.w0)

    # ---- stage-form products ---------------------------------------------------------
    def rollout(self, v):
        """y_k = S_k v, k = 0..N."""
        y = np.zeros((self.N + 1, 4))
        for t in range(self.N):
            y[t + 1] = self.A @ y[t] + self.B @ v[2 * t:2 * t + 2]
        return y

    def grow(self, y):
        """(G v)_r = c_r . y_{k_r} for y = S v."""
        return np.einsum("ra,ra->r", self.coef, y[self.stage])

    def stage_sum(self, vals):
        """b^x_k = sum_{r in k} vals_r c_r (k = 0..N, k = 0 unused)."""
        bx = np.zeros((self.N + 1, 4))
        np.add.at(bx, self.stage, vals[:, None] * self.coef)
        return bx

    def adjoint(self, bx):
        """sum_k S_k' bx_k as an n-vector: psi_k = bx_k + A' psi_{k+1}, (.)_t = B' psi_{t+1}."""
        out = np.zeros(self.n)
        psi = np.zeros(4)
        for k in range(self.N, 0, -1):
            psi = bx[k] + self.A.T @ psi
            out[2 * (k - 1):2 * k] = self.B.T @ psi
        return out

    def qbar_y(self, y):
        out = np.zeros((self.N + 1, 4))
        for k in range(1, self.N + 1):
            out[k] = self.Qbar[k] @ y[k]
        return out

    # ---- Riccati factorization and solve --------------------------------------------
    def riccati_factor(self, d, dbox):
        """Factor M = R_hat + diag(dbox) + sum_k S_k'(Qbar_k + W_k)S_k, W_k from row weights d.
        Returns per-stage (L_t (2x2 Cholesky of Re_t, guarded as qp._chol_guarded), K_t = Re_t^{-1}F_t)."""
        W = np.zeros((self.N + 1, 4, 4))
        np.add.at(W, self.stage, d[:, None, None] * self.coef[:, :, None] * self.coef[:, None, :])
        A, B = self.A, self.B
        P = self.Qbar[self.N] + W[self.N]
        fac = [None] * self.N
        for t in range(self.N - 1, -1, -1):
            Re = self.R + np.diag(dbox[2 * t:2 * t + 2]) + B.T @ P @ B
            F = B.T @ P @ A
            L = _chol2(Re)
            K = _chol2_solve(L, F)
            fac[t] = (L, K)
            if t >= 1:
                P = self.Qbar[t] + W[t] + A.T @ P @ A - F.T @ K
                P = 0.5 * (P + P.T)
        return fac

    def riccati_solve(self, fac, bu, bx):
        """v = M^{-1}(bu + sum_k S_k' bx_k); also returns y = S v (stage states)."""
        A, B = self.A, self.B
        p = bx[self.N].copy()
        kap = [None] * self.N
        for t in range(self.N - 1, -1, -1):
            L, K = fac[t]
            g = bu[2 * t:2 * t + 2] + B.T @ p
            kap[t] = _chol2_solve(L, g)
            if t >= 1:
                p = bx[t] + A.T @ p - K.T @ g
        v = np.zeros(self.n)
        y = np.zeros((self.N + 1, 4))
        for t in range(self.N):
            L, K = fac[t]
            v[2 * t:2 * t + 2] = kap[t] - K @ y[t]
            y[t + 1] = A @ y[t] + B @ v[2 * t:2 * t + 2]
        return v, y


def _chol2(Re):
    p0 = Re[0, 0]
    if not p0 > 0:
        p0 = 1e128
    l00 = np.sqrt(p0)
    l10 = Re[1, 0] / l00
    p1 = Re[1, 1] - l10 * l10
    if not p1 > 0:
        p1 = 1e128
    return np.array([[l00, 0.0], [l10, np.sqrt(p1)]])


def _chol2_solve(L, b):
    y0 = b[0] / L[0, 0]
    y1 = (b[1] - L[1, 0] * y0) / L[1, 1]
    x1 = y1 / L[1, 1]
    x0 = (y0 - L[1, 0] * x1) / L[0, 0]
    return np.array([x0, x1]) if b.ndim == 1 else np.vstack([x0, x1])


def ipm(sq: StageQP, x0, xref, tol=TOL_RES, tol_mu=TOL_MU, max_iter=MAX_ITER, polish_corrections=None,
        polish_mu=None, polish_res=None, init_mu0=None, init_sfloor=None, polish_refine=None, polish_act=None):
    """qp.ipm + qp.polish_step in stage form for one instance.  Returns (u, status, iters)."""
    x0 = np.asarray(x0, float)
    xref = np.asarray(xref, float)
    n, p = sq.n, sq.p
    pre = sq.pre_w0 - sq.pre_E @ x0
    if pre.size and pre.min() < -PRE_TOL:
        return np.zeros(n), STATUS_INFEASIBLE, 0
    q = sq.h @ (x0 - xref)          # mpc.py:320-321
    w = sq.w0 - sq.E @ x0
    boxed = sq.lb is not None
    lb, ub = (sq.lb, sq.ub) if boxed else (np.full(n, -UNBOXED_BOUND), np.full(n, UNBOXED_BOUND))
    nb = n if boxed else 0
    m = p + 2 * nb
    R = sq.R

    def Rhat(v):
        return (R @ v.reshape(-1, 2).T).T.reshape(-1)

    u = np.clip(np.zeros(n), lb, ub) if boxed else np.zeros(n)
    mu0 = INIT_MU0 if init_mu0 is None else init_mu0
    if mu0 > 0:
        qrel = (1.0 / (INIT_Q_PER_VAR * n)) * np.abs(q).max()
        mu0 = min(mu0, max(INIT_MU_MIN, qrel * qrel))
    sfl = INIT_SFLOOR if init_sfloor is None else init_sfloor
    s = np.maximum(w - sq.grow(sq.rollout(u)), sfl); z = mu0 / s if mu0 > 0 else np.ones(p)
    su = np.maximum(ub - u, sfl) if boxed else np.ones(n)
    sl = np.maximum(u - lb, sfl) if boxed else np.ones(n)
    zu = (mu0 / su if mu0 > 0 else np.ones(n)) if boxed else np.zeros(n)
    zl = (mu0 / sl if mu0 > 0 else np.ones(n)) if boxed else np.zeros(n)
    bmask = 1.0 if boxed else 0.0
    bnorm = 1.0 + max(np.abs(w).max() if p else 0.0, np.maximum(np.abs(lb), np.abs(ub)).max() if boxed else 0.0)
    qnorm = 1.0 + np.abs(q).max()
    bound_abs = np.maximum(np.abs(lb), np.abs(ub))
    it = 0
    polish_failed = False
    while True:
        xs = sq.rollout(u)
        Gu = sq.grow(xs)
        rp = Gu + s - w
        rpu = (u + su - ub) * bmask
        rpl = (-u + sl + lb) * bmask
        Hu = Rhat(u) + sq.adjoint(sq.qbar_y(xs))
        Gtz = sq.adjoint(sq.stage_sum(z))
        gz = Gtz + (zu - zl) * bmask
        rd = Hu + q + gz
        mu = ((s @ z) + ((su @ zu + sl @ zl) if boxed else 0.0)) / max(m, 1)
        rpn = max(np.abs(rp).max() if p else 0.0, np.abs(rpu).max(), np.abs(rpl).max())
        rdn = np.abs(rd).max()
        pscale = max(bnorm, 1.0 + (np.abs(Gu).max() if p else 0.0), 1.0 + (np.abs(u).max() if boxed else 0.0))
        dscale = max(qnorm, 1.0 + np.abs(Hu).max(), 1.0 + np.abs(gz).max())
        if not np.isfinite(mu) or not np.isfinite(rdn):
            return u, STATUS_NUMERICAL, it
        res_ok = rpn <= tol * pscale and rdn <= tol * dscale
        last = it >= max_iter
        ptol = max(POLISH_RES if polish_res is None else polish_res, tol)
        pres_ok = rpn <= ptol * pscale and rdn <= ptol * dscale
        polish = not polish_failed and ((pres_ok and mu <= (POLISH_MU if polish_mu is None else polish_mu)) or last)
        if not polish:
            if last:
                return u, STATUS_MAXITER, it
            if res_ok and mu <= tol_mu:
                return u, STATUS_OPTIMAL, it
            if p:
                lo = np.minimum(Gtz * lb, Gtz * ub).sum()
                if lo - w @ z > 1e-12 * (np.abs(Gtz) @ bound_abs + np.abs(w) @ z):
                    return u, STATUS_INFEASIBLE, it
        if polish:
            x, ok = _polish(sq, q, w, lb, ub, boxed, s, z, su, zu, sl, zl, Rhat, polish_corrections,
                            POLISH_REFINE if polish_refine is None else polish_refine,
                            POLISH_ACT if polish_act is None else polish_act)
            if ok:
                return x, STATUS_OPTIMAL, it
            polish_failed = True
            continue
        d = z / s
        dbox = (zu / su + zl / sl) * bmask
        fac = sq.riccati_factor(d, dbox)

        def solve(rc, rcu, rcl):
            t = (rc - z * rp) / s
            bu = -rd + ((rcu - zu * rpu) / su - (rcl - zl * rpl) / sl) * bmask
            du, dy = sq.riccati_solve(fac, bu, sq.stage_sum(t))
            ds = -rp - sq.grow(dy)
            dz = (-rc - z * ds) / s
            dsu = (-rpu - du) * bmask; dsl = (-rpl + du) * bmask
            dzu = (-rcu - zu * dsu) / su * bmask; dzl = (-rcl - zl * dsl) / sl * bmask
            return du, dy, ds, dz, dsu, dzu, dsl, dzl

        du, dy, ds, dz, dsu, dzu, dsl, dzl = solve(s * z, su * zu * bmask, sl * zl * bmask)
        ms = [_maxstep(s, ds), _maxstep(z, dz)]
        if boxed:
            ms += [_maxstep(su, dsu), _maxstep(zu, dzu), _maxstep(sl, dsl), _maxstep(zl, dzl)]
        a_aff = min(1.0, *ms)
        mu_aff = ((s + a_aff * ds) @ (z + a_aff * dz) + (((su + a_aff * dsu) @ (zu + a_aff * dzu) +
                  (sl + a_aff * dsl) @ (zl + a_aff * dzl)) if boxed else 0.0)) / max(m, 1)
        smu = (mu_aff / mu) ** 3 * mu
        rcu = (su * zu + dsu * dzu - smu) * bmask
        rcl = (sl * zl + dsl * dzl - smu) * bmask
        du, dy, ds, dz, dsu, dzu, dsl, dzl = solve(s * z + ds * dz - smu, rcu, rcl)
        if mu <= REFINE_MU:
            # refinement: e = H du + G'dz + rd + box;  M c = -e
            bu = -(Rhat(du) + rd + (dzu - dzl) * bmask)
            bx = -(sq.qbar_y(dy) + sq.stage_sum(dz))
            cu, cy = sq.riccati_solve(fac, bu, bx)
            cs = -sq.grow(cy)
            du = du + cu; ds = ds + cs; dz = dz - z * cs / s
            if boxed:
                dsu = dsu - cu; dzu = dzu + zu * cu / su
                dsl = dsl + cu; dzl = dzl - zl * cu / sl
        ms = [_maxstep(s, ds), _maxstep(z, dz)]
        if boxed:
            ms += [_maxstep(su, dsu), _maxstep(zu, dzu), _maxstep(sl, dsl), _maxstep(zl, dzl)]
        a = min(1.0, STEP_FRAC * min(ms))
        u = u + a * du; s = s + a * ds; z = z + a * dz
        if boxed:
            su = su + a * dsu; zu = zu + a * dzu; sl = sl + a * dsl; zl = zl + a * dzl
        polish_failed = False
        it += 1


def _polish(sq, q, w, lb, ub, boxed, s, z, su, zu, sl, zl, Rhat, corrections=None, refine=POLISH_REFINE,
            act=POLISH_ACT):
    """qp.polish_step in stage form, with its correction rounds."""
    n = sq.n
    if corrections is None:
        corrections = POLISH_CORRECTIONS
    ag = s < act * z
    au = su < act * zu if boxed else np.zeros(n, bool)
    al = sl < act * zl if boxed else np.zeros(n, bool)
    x = np.zeros(n)
    for attempt in range(corrections + 1):
        x, ok, fix = _polish_attempt(sq, q, w, lb, ub, boxed, ag, au, al, Rhat, refine)
        if ok or fix is None or attempt == corrections:
            return x, ok
        nag, nau, nal = fix
        if np.array_equal(nag, ag) and np.array_equal(nau, au) and np.array_equal(nal, al):
            return x, False
        ag, au, al = nag, nau, nal
    return x, False


def _polish_attempt(sq, q, w, lb, ub, boxed, ag, au, al, Rhat, refine=POLISH_REFINE):
    """One polish on the active set (qp._polish_attempt in stage form)."""
    n = sq.n
    idl = 1.0 / POLISH_DELTA
    dg = np.where(ag, idl, 0.0)
    dbu = np.where(au, idl, 0.0)
    dbl = np.where(al, idl, 0.0)
    fac = sq.riccati_factor(dg, dbu + dbl)
    x = np.zeros(n); xv = np.zeros((sq.N + 1, 4))
    yg = np.zeros(sq.p); yu = np.zeros(n); yl = np.zeros(n)
    for _ in range(refine + 1):
        gx = sq.grow(xv)
        ryg = np.where(ag, w - gx, 0.0)
        ryu = np.where(dbu > 0, ub - x, 0.0)
        ryl = np.where(dbl > 0, -lb + x, 0.0)
        t = yg - dg * ryg
        bu = -q - Rhat(x) - yu + yl + dbu * ryu - dbl * ryl
        bx = -(sq.qbar_y(xv) + sq.stage_sum(t))
        dx, dy = sq.riccati_solve(fac, bu, bx)
        yg = yg + dg * (sq.grow(dy) - ryg)
        yu = yu + dbu * (dx - ryu)
        yl = yl + dbl * (-dx - ryl)
        x = x + dx; xv = xv + dy
    gxw = sq.grow(sq.rollout(x)) - w
    wscale = 1.0 + max(np.abs(w).max() if len(w) else 0.0, np.maximum(np.abs(lb), np.abs(ub)).max() if boxed else 0.0)
    viol = max(gxw.max() if len(w) else -np.inf, (x - ub).max() if boxed else -np.inf,
               (lb - x).max() if boxed else -np.inf)
    part = sq.partner
    paired = np.zeros(len(yg), bool)
    if len(yg):
        paired = ag & (part >= 0) & ag[np.maximum(part, 0)]
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


def solve_instance(asm, x0, xref=None, **kw):
    """Stage-form oracle for one instance (goal as the default reference, mpc.py:320-321)."""
    sq = StageQP(asm)
    return ipm(sq, x0, asm.goal if xref is None else xref, **kw)
