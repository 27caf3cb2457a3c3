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
 * with the dense Mehrotra IPM of DESIGN.md §3 / oracle/qp.py::ipm (same
 * settings, same guard rules), OpenMP over instances.  G/w0/E rows are the
 * normalised QP rows; pre_* are the x0-only rows (G_r == 0), checked first.
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

static double maxstep(const double* v, const double* dv, int k, double cur) {
    for (int i = 0; i < k; ++i)
        if (dv[i] < 0.0) {
            double a = -v[i] / dv[i];
            if (a < cur) cur = a;
        }
    return cur;
}

typedef struct {
    int n, p, boxed;
    const double *H, *G, *lb, *ub;
} qp_t;

/* One instance.  work must hold n*n + 17*n + 9*p doubles (WORK_SIZE). */
static int solve_one(const qp_t* P, const double* q, const double* w, double* u, double* work,
                     double tol, double tol_mu, int max_iter, int* iters_out) {
    const int n = P->n, p = P->p, boxed = P->boxed;
    const int nb = boxed ? n : 0;
    const double *H = P->H, *G = P->G, *lb = P->lb, *ub = P->ub;
    double* M = work;               /* n*n */
    double* su = M + n * n;         /* n each */
    double* sl = su + n;
    double* zu = sl + n;
    double* zl = zu + n;
    double* rpu = zl + n;
    double* rpl = rpu + n;
    double* rd = rpl + n;
    double* du = rd + n;
    double* dsu = du + n;
    double* dsl = dsu + n;
    double* dzu = dsl + n;
    double* dzl = dzu + n;          /* 12n so far incl. M */
    double* s = dzl + n;            /* p each */
    double* z = s + p;
    double* rp = z + p;
    double* ds = rp + p;
    double* dz = ds + p;
    double* dsa = dz + p;
    double* dza = dsa + p;
    double* t = dza + p;
    double* rc = t + p;
    double* dsua_ = rc + p;         /* box affine directions, n each */
    double* dzua_ = dsua_ + n;
    double* dsla_ = dzua_ + n;
    double* dzla_ = dsla_ + n;
    const int m = p + 2 * nb;

    for (int i = 0; i < n; ++i) {
        double v = 0.0;
        if (boxed) { v = v < lb[i] ? lb[i] : v; v = v > ub[i] ? ub[i] : v; }
        u[i] = v;
    }
    double bnorm = 0.0, qnorm = 0.0;
    for (int r = 0; r < p; ++r) {
        double gu = 0.0;
        for (int j = 0; j < n; ++j) gu += G[r * n + j] * u[j];
        double sv = w[r] - gu;
        s[r] = sv > 1.0 ? sv : 1.0;
        z[r] = 1.0;
        if (fabs(w[r]) > bnorm) bnorm = fabs(w[r]);
    }
    for (int i = 0; i < nb; ++i) {
        double a = ub[i] - u[i], b = u[i] - lb[i];
        su[i] = a > 1.0 ? a : 1.0;
        sl[i] = b > 1.0 ? b : 1.0;
        zu[i] = zl[i] = 1.0;
        if (fabs(ub[i]) > bnorm) bnorm = fabs(ub[i]);
        if (fabs(lb[i]) > bnorm) bnorm = fabs(lb[i]);
    }
    for (int i = 0; i < n; ++i) if (fabs(q[i]) > qnorm) qnorm = fabs(q[i]);
    bnorm += 1.0; qnorm += 1.0;

    int status = 2, it;
    for (it = 0; it < max_iter; ++it) {
        /* residuals */
        double rpn = 0.0, rdn = 0.0, mu = 0.0;
        for (int r = 0; r < p; ++r) {
            double gu = 0.0;
            for (int j = 0; j < n; ++j) gu += G[r * n + j] * u[j];
            rp[r] = gu + s[r] - w[r];
            if (fabs(rp[r]) > rpn) rpn = fabs(rp[r]);
            mu += s[r] * z[r];
        }
        for (int i = 0; i < nb; ++i) {
            rpu[i] = u[i] + su[i] - ub[i];
            rpl[i] = -u[i] + sl[i] + lb[i];
            if (fabs(rpu[i]) > rpn) rpn = fabs(rpu[i]);
            if (fabs(rpl[i]) > rpn) rpn = fabs(rpl[i]);
            mu += su[i] * zu[i] + sl[i] * zl[i];
        }
        mu /= (m > 0 ? m : 1);
        for (int i = 0; i < n; ++i) {
            double v = q[i];
            for (int j = 0; j < n; ++j) v += H[i * n + j] * u[j];
            for (int r = 0; r < p; ++r) v += G[r * n + i] * z[r];
            if (boxed) v += zu[i] - zl[i];
            rd[i] = v;
            if (fabs(v) > rdn) rdn = fabs(v);
        }
        if (!isfinite(mu) || !isfinite(rdn)) { status = 3; break; }
        if (rpn <= tol * bnorm && rdn <= tol * qnorm && mu <= tol_mu) { status = 0; break; }
        /* Farkas test (rigorous when boxed): min_{box} (G'z)'u > w'z  =>  infeasible */
        if (p > 0) {
            double lo = 0.0, wz = 0.0, scale = 0.0;
            for (int i = 0; i < n; ++i) {
                double c = 0.0;
                for (int r = 0; r < p; ++r) c += G[r * n + i] * z[r];
                double bl = boxed ? lb[i] : -UNBOXED_BOUND, bh = boxed ? ub[i] : UNBOXED_BOUND;
                double a = c * bl, b = c * bh;
                lo += a < b ? a : b;
                double ab = fabs(bl) > fabs(bh) ? fabs(bl) : fabs(bh);
                scale += fabs(c) * ab;
            }
            for (int r = 0; r < p; ++r) { wz += w[r] * z[r]; scale += fabs(w[r]) * z[r]; }
            if (lo - wz > 1e-12 * scale) { status = 1; break; }
        }
        /* M = H + G' diag(z/s) G + diag(box) -- lower triangle only */
        for (int i = 0; i < n; ++i)
            for (int j = 0; j <= i; ++j) M[i * n + j] = H[i * n + j];
        for (int r = 0; r < p; ++r) {
            double d = z[r] / s[r];
            const double* g = G + r * n;
            for (int i = 0; i < n; ++i) {
                double dg = d * g[i];
                for (int j = 0; j <= i; ++j) M[i * n + j] += dg * g[j];
            }
        }
        for (int i = 0; i < nb; ++i) M[i * n + i] += zu[i] / su[i] + zl[i] / sl[i];
        /* guarded right-looking Cholesky, in place (lower) */
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
        /* two solves: predictor (affine) then corrector */
        double sigma_mu = 0.0;
        for (int pass = 0; pass < 2; ++pass) {
            double* dS = pass == 0 ? dsa : ds;
            double* dZ = pass == 0 ? dza : dz;
            double* dSu = pass == 0 ? dsua_ : dsu;
            double* dZu = pass == 0 ? dzua_ : dzu;
            double* dSl = pass == 0 ? dsla_ : dsl;
            double* dZl = pass == 0 ? dzla_ : dzl;
            /* rhs = -rd + G' t + box terms, t = (rc - z rp)/s */
            for (int r = 0; r < p; ++r) {
                rc[r] = pass == 0 ? s[r] * z[r] : s[r] * z[r] + dsa[r] * dza[r] - sigma_mu;
                t[r] = (rc[r] - z[r] * rp[r]) / s[r];
            }
            for (int i = 0; i < n; ++i) {
                double v = -rd[i];
                for (int r = 0; r < p; ++r) v += G[r * n + i] * t[r];
                if (boxed) {
                    double rcu = pass == 0 ? su[i] * zu[i] : su[i] * zu[i] + dsua_[i] * dzua_[i] - sigma_mu;
                    double rcl = pass == 0 ? sl[i] * zl[i] : sl[i] * zl[i] + dsla_[i] * dzla_[i] - sigma_mu;
                    v += (rcu - zu[i] * rpu[i]) / su[i] - (rcl - zl[i] * rpl[i]) / sl[i];
                    /* stash rc for the box dz computation */
                    dSu[i] = rcu; dSl[i] = rcl;
                }
                du[i] = v;
            }
            /* forward: L y = rhs */
            for (int i = 0; i < n; ++i) {
                double v = du[i];
                for (int j = 0; j < i; ++j) v -= M[i * n + j] * du[j];
                du[i] = v / M[i * n + i];
            }
            /* backward: L' x = y */
            for (int i = n - 1; i >= 0; --i) {
                double v = du[i];
                for (int j = i + 1; j < n; ++j) v -= M[j * n + i] * du[j];
                du[i] = v / M[i * n + i];
            }
            for (int r = 0; r < p; ++r) {
                double gd = 0.0;
                for (int j = 0; j < n; ++j) gd += G[r * n + j] * du[j];
                dS[r] = -rp[r] - gd;
                dZ[r] = (-rc[r] - z[r] * dS[r]) / s[r];
            }
            for (int i = 0; i < nb; ++i) {
                double rcu = dSu[i], rcl = dSl[i];
                dSu[i] = -rpu[i] - du[i];
                dSl[i] = -rpl[i] + du[i];
                dZu[i] = (-rcu - zu[i] * dSu[i]) / su[i];
                dZl[i] = (-rcl - zl[i] * dSl[i]) / sl[i];
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
                for (int r = 0; r < p; ++r) { s[r] += a * ds[r]; z[r] += a * dz[r]; }
                for (int i = 0; i < nb; ++i) {
                    su[i] += a * dsu[i]; zu[i] += a * dzu[i];
                    sl[i] += a * dsl[i]; zl[i] += a * dzl[i];
                }
            }
        }
    }
    *iters_out = it < max_iter ? it : max_iter;
    return status;
}

/* Batched entry point.  Arrays are row-major fp64.  lb/ub NULL => no input box.
 * xref NULL => goal for every instance.  Returns 0. */
int oracle_solve_batch(int n, int p, int npre, const double* H, const double* G, const double* w0,
                       const double* E, const double* pre_w0, const double* pre_E, const double* hq,
                       const double* lb, const double* ub, const double* goal, int64_t B,
                       const double* x0, const double* xref, double* u_out, int32_t* status,
                       int32_t* iters, double tol, double tol_mu, int max_iter, int nthreads) {
    qp_t P = {n, p, lb != NULL && ub != NULL, H, G, lb, ub};
#ifdef _OPENMP
    if (nthreads > 0) omp_set_num_threads(nthreads);
#else
    (void)nthreads;
#endif
#pragma omp parallel
    {
        double* work = (double*)malloc(sizeof(double) * (size_t)(n * n + 17 * n + 9 * p + 1));
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
            status[b] = solve_one(&P, q, w, u, work, tol, tol_mu, max_iter, &it);
            iters[b] = it;
        }
        free(work); free(q); free(w);
    }
    return 0;
}
