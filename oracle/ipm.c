/*
 * oracle/ipm.c -- plain-C restatement of the per-step CarMPC QP solve (ORACLE, tests only).
 *
 * TEST INFRASTRUCTURE: only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg load this library.  The product (carmpc_amd) never does.
 *
 * Restates, per instance, the QP that lib/mpc.py:312-349 (MPCStateFB.step) and
 * lib/mpc.py:450-492 (MPCOutputFB.step) hand to cvxpy:
 *     min 1/2 u'Hu + q'u,  q = hq (x0 - xref)          (mpc.py:320-321)
 *     s.t. G u <= w0 - E x0  (terminal + state rows)    (mpc.py:319,324-332)
 *          lb <= u <= ub     (input box)                (mpc.py:327-329)
 * with the algorithm of oracle/qp.py::ipm: dense Mehrotra
 * predictor-corrector on the normal equations, one refinement pass on the
 * corrector, rigorous box-Farkas infeasibility test, and the active-set polish.
 * OpenMP over instances.  G/w0/E rows are the normalised QP rows; pre_* are
 * the x0-only rows (G_r == 0), checked first.
 *
 * Status codes: 0 optimal, 1 primal infeasible, 2 max iterations, 3 numerical.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#define UNBOXED_BOUND 1e9
#define PRE_TOL 1e-9
#define STEP_FRAC 0.99
#define POLISH_MU 1e-2    /* polish gate: mu <= POLISH_MU and residuals within max(POLISH_RES, tol) */
#define POLISH_RES 2e-4
#define POLISH_ACT 0.003  /* first active set of a polish: rows with s < POLISH_ACT z */
#define INIT_MU0 100.0     /* initial point: s = max(w - G u0, INIT_SFLOOR), z = INIT_MU0 / s (qp.py) */
#define INIT_SFLOOR 2.0
#define INIT_MU_MIN 1.0     /* mu0 = clamp((|q|_inf / (INIT_Q_PER_VAR n))^2, INIT_MU_MIN, INIT_MU0) */
#define INIT_Q_PER_VAR 3.5
#define REFINE_MU 1e-6   /* refinement of the corrector only once mu <= REFINE_MU */
#define POLISH_DELTA 1e-10
#define POLISH_REFINE 2   /* refinement passes of the polish solve; 3 in the fallback variant */
#define POLISH_TOL 1e-11

typedef struct {
    int n, p, boxed;
    const double *H, *G, *lb, *ub;
    const int32_t* partner;   /* opposite row (equality pair) or -1; NULL = none (qp.py::opposite_pairs) */
} qp_t;

static double maxstep(const double* v, const double* dv, int k, double cur) {
    for (int i = 0; i < k; ++i)
        if (dv[i] < 0.0) {
            double a = -v[i] / dv[i];
            if (a < cur) cur = a;
        }
    return cur;
}

/* M = H + G' diag(dg) G + diag(dbox) (lower triangle), then guarded Cholesky in place. */
static void factor(const qp_t* P, const double* dg, const double* dbox, double* M) {
    const int n = P->n, p = P->p;
    for (int i = 0; i < n; ++i)
        for (int j = 0; j <= i; ++j) M[i * n + j] = P->H[i * n + j];
    for (int r = 0; r < p; ++r) {
        if (dg[r] == 0.0) continue;
        const double* g = P->G + r * n;
        for (int i = 0; i < n; ++i) {
            double t = dg[r] * g[i];
            for (int j = 0; j <= i; ++j) M[i * n + j] += t * g[j];
        }
    }
    if (dbox)
        for (int i = 0; i < n; ++i) M[i * n + i] += dbox[i];
    for (int k = 0; k < n; ++k) {
        double piv = M[k * n + k];
        if (!(piv > 0.0)) piv = 1e128;
        double lkk = sqrt(piv);
        M[k * n + k] = lkk;
        double inv = 1.0 / lkk;
        for (int i = k + 1; i < n; ++i) M[i * n + k] *= inv;
        for (int j = k + 1; j < n; ++j) {
            double ljk = M[j * n + k];
            for (int i = j; i < n; ++i) M[i * n + j] -= M[i * n + k] * ljk;
        }
    }
}

static void chol_solve(const double* L, int n, double* x) {
    for (int i = 0; i < n; ++i) {
        double v = x[i];
        for (int j = 0; j < i; ++j) v -= L[i * n + j] * x[j];
        x[i] = v / L[i * n + i];
    }
    for (int i = n - 1; i >= 0; --i) {
        double v = x[i];
        for (int j = i + 1; j < n; ++j) v -= L[j * n + i] * x[j];
        x[i] = v / L[i * n + i];
    }
}

static void gmul(const qp_t* P, const double* x, double* out) { /* out = G x */
    for (int r = 0; r < P->p; ++r) {
        double v = 0.0;
        for (int j = 0; j < P->n; ++j) v += P->G[r * P->n + j] * x[j];
        out[r] = v;
    }
}

static void gtmul(const qp_t* P, const double* y, double* out) { /* out = G' y */
    for (int i = 0; i < P->n; ++i) out[i] = 0.0;
    for (int r = 0; r < P->p; ++r) {
        if (y[r] == 0.0) continue;
        for (int i = 0; i < P->n; ++i) out[i] += P->G[r * P->n + i] * y[r];
    }
}

/* correction rounds of a rejected polish (qp.POLISH_CORRECTIONS); 0 = the single-attempt polish */
static int g_polish_corrections = 1;
static double g_polish_mu = POLISH_MU, g_polish_res = POLISH_RES;
static double g_init_mu0 = INIT_MU0, g_init_sfloor = INIT_SFLOOR;
static int g_polish_refine = POLISH_REFINE;
static double g_polish_act = POLISH_ACT;
/* qp.FALLBACK_VARIANT = (0, 1e-6, 0, 0, 1, 3, 1): the single-attempt polish (3 refinement passes, active set
 * s < z) behind the conservative gate, z = 1 and slack floor 1 at the start */
void oracle_set_variant(int corrections, double mu, double res, double init_mu0, double init_sfloor, int refine,
                        double act) {
    g_polish_refine = refine; g_polish_act = act;
    g_polish_corrections = corrections; g_polish_mu = mu; g_polish_res = res;
    g_init_mu0 = init_mu0; g_init_sfloor = init_sfloor;
}

typedef struct {   /* per-thread scratch */
    double *M, *s, *z, *rp, *ds, *dz, *dsa, *dza, *t, *rc, *gv, *pv1, *pv2;
    double *su, *sl, *zu, *zl, *rpu, *rpl, *rd, *du, *dsu, *dsl, *dzu, *dzl, *dsua, *dzua, *dsla, *dzla, *nv1,
        *nv2, *nv3, *nv4, *nv5;
    /* polish-only scratch (must not alias IPM state) */
    double *pdg, *pyg, *pryg, *pgx, *pdbu, *pdbl, *pyu, *pyl, *prhs, *pdx;
} work_t;

static void work_alloc(work_t* W, int n, int p) {
    size_t pn = (size_t)(p > 0 ? p : 1), nn = (size_t)(n > 0 ? n : 1);
    double* base = (double*)malloc(sizeof(double) * (nn * nn + 17 * pn + 28 * nn));
    W->M = base;
    double* c = base + nn * nn;
    double** pv[] = {&W->s, &W->z, &W->rp, &W->ds, &W->dz, &W->dsa, &W->dza, &W->t, &W->rc, &W->gv, &W->pv1, &W->pv2};
    for (size_t k = 0; k < sizeof(pv) / sizeof(pv[0]); ++k) { *pv[k] = c; c += pn; }
    c += pn;
    double** nvp[] = {&W->su, &W->sl, &W->zu, &W->zl, &W->rpu, &W->rpl, &W->rd, &W->du, &W->dsu, &W->dsl, &W->dzu,
                      &W->dzl, &W->dsua, &W->dzua, &W->dsla, &W->dzla, &W->nv1, &W->nv2, &W->nv3, &W->nv4, &W->nv5};
    for (size_t k = 0; k < sizeof(nvp) / sizeof(nvp[0]); ++k) { *nvp[k] = c; c += nn; }
    double** ppv[] = {&W->pdg, &W->pyg, &W->pryg, &W->pgx};
    for (size_t k = 0; k < sizeof(ppv) / sizeof(ppv[0]); ++k) { *ppv[k] = c; c += pn; }
    double** pnv[] = {&W->pdbu, &W->pdbl, &W->pyu, &W->pyl, &W->prhs, &W->pdx};
    for (size_t k = 0; k < sizeof(pnv) / sizeof(pnv[0]); ++k) { *pnv[k] = c; c += nn; }
}

/* Active-set polish (oracle/qp.py::polish_step).  Returns 1 and writes x if accepted. */
static int polish(const qp_t* P, const double* q, const double* w, work_t* W, double* x_out) {
    const int n = P->n, p = P->p, boxed = P->boxed;
    const double id = 1.0 / POLISH_DELTA;
    double* dg = W->pdg;   /* 1/delta on active rows */
    double* yg = W->pyg;
    double* ryg = W->pryg;
    double* gx = W->pgx;
    double* dbu = W->pdbu; double* dbl = W->pdbl;
    double* yu = W->pyu; double* yl = W->pyl;
    double* rhs = W->prhs;
    double* dx = W->pdx;
    double* x = x_out;
    double ryu[64], ryl[64], dbox[64];
    if (n > 64) return 0;
    for (int r = 0; r < p; ++r) dg[r] = W->s[r] < g_polish_act * W->z[r] ? id : 0.0;
    for (int i = 0; i < n; ++i) {
        dbu[i] = (boxed && W->su[i] < g_polish_act * W->zu[i]) ? id : 0.0;
        dbl[i] = (boxed && W->sl[i] < g_polish_act * W->zl[i]) ? id : 0.0;
    }
    /* attempt 0 on the active set of the iterate; correction rounds on the set the rejected
     * attempt names (oracle/qp.py::polish_step) */
    for (int attempt = 0;; ++attempt) {
    for (int i = 0; i < n; ++i) dbox[i] = dbu[i] + dbl[i];
    factor(P, dg, dbox, W->M);   /* M is rebuilt by the IPM before its next use */
    /* first solve: rx = -q, ry = b on active rows */
    for (int r = 0; r < p; ++r) ryg[r] = dg[r] != 0.0 ? w[r] : 0.0;
    for (int i = 0; i < n; ++i) {
        ryu[i] = dbu[i] != 0.0 ? P->ub[i] : 0.0;
        ryl[i] = dbl[i] != 0.0 ? -P->lb[i] : 0.0;
        x[i] = 0.0; yu[i] = 0.0; yl[i] = 0.0;
    }
    for (int r = 0; r < p; ++r) yg[r] = 0.0;
    for (int pass = 0; pass <= g_polish_refine; ++pass) {
        /* rx = -q - H x - A'y  (pass 0: x = y = 0) */
        for (int i = 0; i < n; ++i) {
            double v = -q[i];
            for (int j = 0; j < n; ++j) v -= P->H[i * n + j] * x[j];
            rhs[i] = v - yu[i] + yl[i];
        }
        gtmul(P, yg, dx);
        for (int i = 0; i < n; ++i) rhs[i] -= dx[i];
        if (pass > 0) {   /* ry = b - A x on active rows */
            gmul(P, x, gx);
            for (int r = 0; r < p; ++r) ryg[r] = dg[r] != 0.0 ? w[r] - gx[r] : 0.0;
            for (int i = 0; i < n; ++i) {
                ryu[i] = dbu[i] != 0.0 ? P->ub[i] - x[i] : 0.0;
                ryl[i] = dbl[i] != 0.0 ? -P->lb[i] + x[i] : 0.0;
            }
        }
        /* K_delta solve: (H + A'A/delta) dx = rx + A' ry/delta ; dy = (A dx - ry)/delta */
        for (int r = 0; r < p; ++r) gx[r] = dg[r] * ryg[r];
        gtmul(P, gx, dx);
        for (int i = 0; i < n; ++i) rhs[i] += dx[i] + dbu[i] * ryu[i] - dbl[i] * ryl[i];
        memcpy(dx, rhs, sizeof(double) * n);
        chol_solve(W->M, n, dx);
        gmul(P, dx, gx);
        for (int r = 0; r < p; ++r) yg[r] += dg[r] * (gx[r] - ryg[r]);
        for (int i = 0; i < n; ++i) {
            yu[i] += dbu[i] * (dx[i] - ryu[i]);
            yl[i] += dbl[i] * (-dx[i] - ryl[i]);
            x[i] += dx[i];
        }
    }
    /* accept: primal feasible and dual nonnegative (relative POLISH_TOL) */
    double wsc = 0.0, ysc = 0.0, viol = -INFINITY, ymin = 0.0;
    gmul(P, x, gx);
    for (int r = 0; r < p; ++r) {
        if (fabs(w[r]) > wsc) wsc = fabs(w[r]);
        if (gx[r] - w[r] > viol) viol = gx[r] - w[r];
        if (fabs(yg[r]) > ysc) ysc = fabs(yg[r]);
        /* both rows of an opposite pair active = an equality: multipliers re-splittable */
        const int pr = P->partner ? P->partner[r] : -1;
        const int paired = pr >= 0 && dg[r] != 0.0 && dg[pr] != 0.0;
        if (!paired && yg[r] < ymin) ymin = yg[r];
    }
    int finite = 1;
    for (int i = 0; i < n; ++i) {
        if (!isfinite(x[i])) finite = 0;
        if (boxed) {
            if (fabs(P->ub[i]) > wsc) wsc = fabs(P->ub[i]);
            if (fabs(P->lb[i]) > wsc) wsc = fabs(P->lb[i]);
            if (x[i] - P->ub[i] > viol) viol = x[i] - P->ub[i];
            if (P->lb[i] - x[i] > viol) viol = P->lb[i] - x[i];
        }
        if (fabs(yu[i]) > ysc) ysc = fabs(yu[i]);
        if (fabs(yl[i]) > ysc) ysc = fabs(yl[i]);
        if (yu[i] < ymin) ymin = yu[i];
        if (yl[i] < ymin) ymin = yl[i];
    }
    if (!finite) return 0;
    const double vtol = POLISH_TOL * (1.0 + wsc), ytol = -POLISH_TOL * (1.0 + ysc);
    if (viol <= vtol && ymin >= ytol) return 1;
    if (attempt >= g_polish_corrections) return 0;
    /* drop active rows that fail the sign test, add inactive rows that are violated */
    int changed = 0;
    for (int r = 0; r < p; ++r) {
        const int pr = P->partner ? P->partner[r] : -1;
        const int paired = pr >= 0 && dg[r] != 0.0 && dg[pr] != 0.0;
        if (dg[r] != 0.0) W->pryg[r] = (!paired && yg[r] < ytol) ? 0.0 : id;   /* pryg: next dg (ryg is rebuilt) */
        else W->pryg[r] = gx[r] - w[r] > vtol ? id : 0.0;
    }
    for (int r = 0; r < p; ++r) {
        if (W->pryg[r] != dg[r]) changed = 1;
        dg[r] = W->pryg[r];
    }
    for (int i = 0; i < n && boxed; ++i) {
        const double nu = dbu[i] != 0.0 ? (yu[i] < ytol ? 0.0 : id) : (x[i] - P->ub[i] > vtol ? id : 0.0);
        const double nl = dbl[i] != 0.0 ? (yl[i] < ytol ? 0.0 : id) : (P->lb[i] - x[i] > vtol ? id : 0.0);
        if (nu != dbu[i] || nl != dbl[i]) changed = 1;
        dbu[i] = nu; dbl[i] = nl;
    }
    if (!changed) return 0;
    }
}

static int solve_one(const qp_t* P, const double* q, const double* w, double* u, work_t* W, double tol,
                     double tol_mu, int max_iter, int* iters_out) {
    const int n = P->n, p = P->p, boxed = P->boxed;
    const int nb = boxed ? n : 0;
    const double *lb = P->lb, *ub = P->ub;
    double *s = W->s, *z = W->z, *rp = W->rp, *rd = W->rd, *du = W->du;
    double *su = W->su, *sl = W->sl, *zu = W->zu, *zl = W->zl, *rpu = W->rpu, *rpl = W->rpl;
    const int m = p + 2 * nb;
    double xpol[64];

    for (int i = 0; i < n; ++i) {
        double v = 0.0;
        if (boxed) { v = v < lb[i] ? lb[i] : v; v = v > ub[i] ? ub[i] : v; }
        u[i] = v;
    }
    double bnorm = 0.0, qnorm = 0.0;
    double mu0 = g_init_mu0;
    if (mu0 > 0.0) {
        double qn = 0.0;
        for (int i = 0; i < n; ++i) if (fabs(q[i]) > qn) qn = fabs(q[i]);
        double m = (1.0 / (INIT_Q_PER_VAR * n)) * qn;
        m = m * m;
        if (m < INIT_MU_MIN) m = INIT_MU_MIN;
        if (m < mu0) mu0 = m;
    }
    gmul(P, u, W->gv);
    for (int r = 0; r < p; ++r) {
        double sv = w[r] - W->gv[r];
        s[r] = sv > g_init_sfloor ? sv : g_init_sfloor;
        z[r] = mu0 > 0.0 ? mu0 / s[r] : 1.0;
        if (fabs(w[r]) > bnorm) bnorm = fabs(w[r]);
    }
    for (int i = 0; i < n; ++i) {
        su[i] = sl[i] = 1.0;
        zu[i] = zl[i] = boxed ? 1.0 : 0.0;
        if (boxed) {
            double a = ub[i] - u[i], b = u[i] - lb[i];
            su[i] = a > g_init_sfloor ? a : g_init_sfloor;
            sl[i] = b > g_init_sfloor ? b : g_init_sfloor;
            if (mu0 > 0.0) { zu[i] = mu0 / su[i]; zl[i] = mu0 / sl[i]; }
            if (fabs(ub[i]) > bnorm) bnorm = fabs(ub[i]);
            if (fabs(lb[i]) > bnorm) bnorm = fabs(lb[i]);
        }
        if (fabs(q[i]) > qnorm) qnorm = fabs(q[i]);
    }
    bnorm += 1.0; qnorm += 1.0;

    int status = 2, it;
    for (it = 0; it < max_iter; ++it) {
        /* ---- residuals and their scales ---- */
        double rpn = 0.0, rdn = 0.0, mu = 0.0, gun = 0.0, un = 0.0, hun = 0.0, gzn = 0.0;
        gmul(P, u, W->gv);
        for (int r = 0; r < p; ++r) {
            if (fabs(W->gv[r]) > gun) gun = fabs(W->gv[r]);
            rp[r] = W->gv[r] + s[r] - w[r];
            if (fabs(rp[r]) > rpn) rpn = fabs(rp[r]);
            mu += s[r] * z[r];
        }
        for (int i = 0; i < n; ++i) {
            rpu[i] = boxed ? u[i] + su[i] - ub[i] : 0.0;
            rpl[i] = boxed ? -u[i] + sl[i] + lb[i] : 0.0;
            if (fabs(rpu[i]) > rpn) rpn = fabs(rpu[i]);
            if (fabs(rpl[i]) > rpn) rpn = fabs(rpl[i]);
            if (boxed) mu += su[i] * zu[i] + sl[i] * zl[i];
            if (boxed && fabs(u[i]) > un) un = fabs(u[i]);
        }
        mu /= (m > 0 ? m : 1);
        gtmul(P, z, W->nv1);                      /* nv1 = G'z (Farkas c) */
        for (int i = 0; i < n; ++i) {
            double hu = 0.0;
            for (int j = 0; j < n; ++j) hu += P->H[i * n + j] * u[j];
            double gz = W->nv1[i] + (boxed ? zu[i] - zl[i] : 0.0);
            rd[i] = q[i] + hu + gz;
            if (fabs(rd[i]) > rdn) rdn = fabs(rd[i]);
            if (fabs(hu) > hun) hun = fabs(hu);
            if (fabs(gz) > gzn) gzn = fabs(gz);
        }
        double pscale = bnorm, dscale = qnorm;
        if (1.0 + gun > pscale) pscale = 1.0 + gun;
        if (1.0 + un > pscale) pscale = 1.0 + un;
        if (1.0 + hun > dscale) dscale = 1.0 + hun;
        if (1.0 + gzn > dscale) dscale = 1.0 + gzn;
        if (!isfinite(mu) || !isfinite(rdn)) { status = 3; break; }
        const int res_ok = rpn <= tol * pscale && rdn <= tol * dscale;
        const double ptol = g_polish_res > tol ? g_polish_res : tol;
        const int pres_ok = rpn <= ptol * pscale && rdn <= ptol * dscale;
        if (pres_ok && mu <= g_polish_mu && polish(P, q, w, W, xpol)) {
            memcpy(u, xpol, sizeof(double) * n);
            status = 0;
            break;
        }
        if (res_ok && mu <= tol_mu) { status = 0; break; }
        /* ---- Farkas test (rigorous when boxed): min_box (G'z)'u > w'z => infeasible ---- */
        if (p > 0) {
            double lo = 0.0, wz = 0.0, scale = 0.0;
            for (int i = 0; i < n; ++i) {
                double c = W->nv1[i];
                double bl = boxed ? lb[i] : -UNBOXED_BOUND, bh = boxed ? ub[i] : UNBOXED_BOUND;
                double a = c * bl, b = c * bh;
                lo += a < b ? a : b;
                double ab = fabs(bl) > fabs(bh) ? fabs(bl) : fabs(bh);
                scale += fabs(c) * ab;
            }
            for (int r = 0; r < p; ++r) { wz += w[r] * z[r]; scale += fabs(w[r]) * z[r]; }
            if (lo - wz > 1e-12 * scale) { status = 1; break; }
        }
        /* ---- factor M = H + G' diag(z/s) G + diag(box) ---- */
        for (int r = 0; r < p; ++r) W->pv1[r] = z[r] / s[r];
        for (int i = 0; i < n; ++i) W->nv2[i] = boxed ? zu[i] / su[i] + zl[i] / sl[i] : 0.0;
        factor(P, W->pv1, W->nv2, W->M);
        /* ---- predictor then corrector (+1 refinement pass on the corrector) ---- */
        double sigma_mu = 0.0;
        for (int pass = 0; pass < 2; ++pass) {
            double* dS = pass == 0 ? W->dsa : W->ds;
            double* dZ = pass == 0 ? W->dza : W->dz;
            double* dSu = pass == 0 ? W->dsua : W->dsu;
            double* dZu = pass == 0 ? W->dzua : W->dzu;
            double* dSl = pass == 0 ? W->dsla : W->dsl;
            double* dZl = pass == 0 ? W->dzla : W->dzl;
            double* rcu = W->nv3; double* rcl = W->nv4;
            for (int r = 0; r < p; ++r) {
                W->rc[r] = pass == 0 ? s[r] * z[r] : s[r] * z[r] + W->dsa[r] * W->dza[r] - sigma_mu;
                W->t[r] = (W->rc[r] - z[r] * rp[r]) / s[r];
            }
            gtmul(P, W->t, du);
            for (int i = 0; i < n; ++i) {
                double v = -rd[i] + du[i];
                if (boxed) {
                    rcu[i] = pass == 0 ? su[i] * zu[i] : su[i] * zu[i] + W->dsua[i] * W->dzua[i] - sigma_mu;
                    rcl[i] = pass == 0 ? sl[i] * zl[i] : sl[i] * zl[i] + W->dsla[i] * W->dzla[i] - sigma_mu;
                    v += (rcu[i] - zu[i] * rpu[i]) / su[i] - (rcl[i] - zl[i] * rpl[i]) / sl[i];
                }
                du[i] = v;
            }
            chol_solve(W->M, n, du);
            gmul(P, du, W->gv);
            for (int r = 0; r < p; ++r) {
                dS[r] = -rp[r] - W->gv[r];
                dZ[r] = (-W->rc[r] - z[r] * dS[r]) / s[r];
            }
            for (int i = 0; i < nb; ++i) {
                dSu[i] = -rpu[i] - du[i];
                dSl[i] = -rpl[i] + du[i];
                dZu[i] = (-rcu[i] - zu[i] * dSu[i]) / su[i];
                dZl[i] = (-rcl[i] - zl[i] * dSl[i]) / sl[i];
            }
            if (pass == 1 && mu <= REFINE_MU) {
                /* refinement (once mu <= REFINE_MU): e = H du + G'dz + box + rd ; M c = -e ;
                   du += c, ds -= G c, dz += z G c / s */
                double* e = W->nv5;
                gtmul(P, dZ, e);
                for (int i = 0; i < n; ++i) {
                    double v = e[i] + rd[i] + (boxed ? dZu[i] - dZl[i] : 0.0);
                    for (int j = 0; j < n; ++j) v += P->H[i * n + j] * du[j];
                    e[i] = -v;
                }
                chol_solve(W->M, n, e);
                gmul(P, e, W->gv);
                for (int r = 0; r < p; ++r) {
                    dS[r] -= W->gv[r];
                    dZ[r] += z[r] * W->gv[r] / s[r];
                }
                for (int i = 0; i < n; ++i) {
                    du[i] += e[i];
                    if (boxed) {
                        dSu[i] -= e[i]; dZu[i] += zu[i] * e[i] / su[i];
                        dSl[i] += e[i]; dZl[i] -= zl[i] * e[i] / sl[i];
                    }
                }
            }
            double amax = INFINITY;
            amax = maxstep(s, dS, p, amax);
            amax = maxstep(z, dZ, p, amax);
            amax = maxstep(su, dSu, nb, amax);
            amax = maxstep(zu, dZu, nb, amax);
            amax = maxstep(sl, dSl, nb, amax);
            amax = maxstep(zl, dZl, nb, amax);
            if (pass == 0) {
                double a = amax < 1.0 ? amax : 1.0;
                double mua = 0.0;
                for (int r = 0; r < p; ++r) mua += (s[r] + a * dS[r]) * (z[r] + a * dZ[r]);
                for (int i = 0; i < nb; ++i)
                    mua += (su[i] + a * dSu[i]) * (zu[i] + a * dZu[i]) + (sl[i] + a * dSl[i]) * (zl[i] + a * dZl[i]);
                mua /= (m > 0 ? m : 1);
                double sg = mua / mu;
                sigma_mu = sg * sg * sg * mu;
            } else {
                double a = STEP_FRAC * amax;
                if (a > 1.0) a = 1.0;
                for (int i = 0; i < n; ++i) u[i] += a * du[i];
                for (int r = 0; r < p; ++r) { s[r] += a * dS[r]; z[r] += a * dZ[r]; }
                for (int i = 0; i < nb; ++i) {
                    su[i] += a * dSu[i]; zu[i] += a * dZu[i];
                    sl[i] += a * dSl[i]; zl[i] += a * dZl[i];
                }
            }
        }
    }
    if (status == 2 && polish(P, q, w, W, xpol)) {   /* last resort at the iteration limit */
        memcpy(u, xpol, sizeof(double) * n);
        status = 0;
    }
    *iters_out = it < max_iter ? it : max_iter;
    return status;
}

/* Batched entry point.  Arrays are row-major fp64.  lb/ub NULL => no input box.
 * partner (p entries, -1 = none) or NULL: opposite-row pairs for the polish.
 * xref NULL => goal for every instance.  Returns 0, or -1 for n > 64. */
int oracle_solve_batch(int n, int p, int npre, const double* H, const double* G, const double* w0,
                       const double* E, const double* pre_w0, const double* pre_E, const double* hq,
                       const double* lb, const double* ub, const int32_t* partner, const double* goal, int64_t B,
                       const double* x0, const double* xref, double* u_out, int32_t* status,
                       int32_t* iters, double tol, double tol_mu, int max_iter, int nthreads) {
    if (n > 64) return -1;
    qp_t P = {n, p, lb != NULL && ub != NULL, H, G, lb, ub, partner};
#ifdef _OPENMP
    if (nthreads > 0) omp_set_num_threads(nthreads);
#else
    (void)nthreads;
#endif
#pragma omp parallel
    {
        work_t W;
        work_alloc(&W, n, p);
        double* q = (double*)malloc(sizeof(double) * (size_t)(n + 1));
        double* w = (double*)malloc(sizeof(double) * (size_t)(p + 1));
#pragma omp for schedule(dynamic, 16)
        for (int64_t b = 0; b < B; ++b) {
            const double* xb = x0 + 4 * b;
            const double* xr = xref ? xref + 4 * b : goal;
            double* u = u_out + (size_t)n * b;
            int bad = 0;
            for (int r = 0; r < npre; ++r) {
                double v = pre_w0[r];
                for (int k = 0; k < 4; ++k) v -= pre_E[r * 4 + k] * xb[k];
                if (v < -PRE_TOL) bad = 1;
            }
            if (bad) {
                for (int i = 0; i < n; ++i) u[i] = 0.0;
                status[b] = 1; iters[b] = 0;
                continue;
            }
            for (int i = 0; i < n; ++i) {
                double v = 0.0;
                for (int k = 0; k < 4; ++k) v += hq[i * 4 + k] * (xb[k] - xr[k]);
                q[i] = v;
            }
            for (int r = 0; r < p; ++r) {
                double v = w0[r];
                for (int k = 0; k < 4; ++k) v -= E[r * 4 + k] * xb[k];
                w[r] = v;
            }
            int it = 0;
            status[b] = solve_one(&P, q, w, u, &W, tol, tol_mu, max_iter, &it);
            iters[b] = it;
        }
        free(W.M); free(q); free(w);
    }
    return 0;
}
