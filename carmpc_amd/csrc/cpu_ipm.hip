// cpu_ipm.hip -- host twins of the batched solve: carmpc_cpu_problem_create /
// carmpc_cpu_solve_batch / carmpc_cpu_solve_batch_dist (host code only; no device call).
//
// The reference solves its per-step QP on the CPU (cp.Problem(...).solve(), lib/mpc.py:334-335,
// 477-478, 652-653).  This is the product's CPU path for hosts without a GPU: the same
// stage-form Mehrotra IPM as the grouped device kernel (ipm_riccati.hip) -- every QP row of
// lib/mpc.py:196-253 acts on one predicted state, H = R_hat + S'Q_hat S
// (lib/matrix_gen.py:35-72), so each Newton system M du = b is one backward Riccati recursion
// plus a forward roll-out over the horizon -- with the device path's tolerances, row
// normalisation, x0-only preconditions, box-Farkas infeasibility test and active-set polish.
// One instance per call of Solver::solve; instances are spread over std::threads.
#include <algorithm>
#include <atomic>
#include <cmath>
#include <cstring>
#include <limits>
#include <string>
#include <thread>
#include <vector>

#include "carmpc_internal.h"

using namespace carmpc;

struct carmpc_cpu_problem {
    int N = 0, n = 0, p = 0, npre = 0;
    bool boxed = false, has_dist = false;
    double A[16], B[8], Q[16], Pt[16], R[4];   // Q, Pt (terminal cost), R symmetrised
    std::vector<int> row_begin;                // rows of stage k: [row_begin[k], row_begin[k+1]), k = 1..N
    std::vector<double> coef, w0, E, Ed;       // p x NX (unit condensed 2-norm), p, p x NX, p
    std::vector<int> partner;                  // p: the exactly opposite row or -1
    std::vector<double> pre_w0, pre_E, pre_Ed; // x0-only rows (raw)
    std::vector<double> hq;                    // n x NX: h = S'Q_hat T (matrix_gen.py:66)
    std::vector<double> lb, ub;                // n
    double goal[NX];
    // rows before the split, for carmpc_cpu_problem_set_disturbance
    std::vector<int> all_stage;
    std::vector<double> all_coef, all_norm;
    std::vector<int> qp_rows, pre_rows;        // indices into the rows before the split
};

namespace {

constexpr double kPolishMu = 1e-2, kPolishRes = 2e-4;   // polish gate of the grouped device kernel (ipm_riccati.hip)
constexpr double kPolishAct = 0.003;                    // ... and its first active set: rows with s < kPolishAct z
constexpr double kPolishDelta = 1e-10, kPolishTol = 1e-11;
// initial point s = max(w - G u0, floor), z = mu0 / s, mu0 = clamp((|q|_inf / (kInitQPerVar n))^2, kInitMuMin, kInitMu0) (ipm_riccati.hip)
constexpr double kInitMu0 = 100.0, kInitSFloor = 2.0, kInitMuMin = 1.0, kInitQPerVar = 3.5;
constexpr int kPolishRefine = 2;
constexpr int kPolishCorrections = 1;   // correction rounds of a rejected polish
constexpr double kInf = std::numeric_limits<double>::infinity();

inline void mat4(const double* X, const double* Y, double* Z) {   // Z = X Y
    for (int a = 0; a < 4; ++a)
        for (int b = 0; b < 4; ++b) {
            double v = 0.0;
            for (int c = 0; c < 4; ++c) v += X[a * 4 + c] * Y[c * 4 + b];
            Z[a * 4 + b] = v;
        }
}

// Per-thread solver state for one problem.
struct Solver {
    const carmpc_cpu_problem& P;
    const int N, n, p;
    std::vector<double> w, s, z, rp, gu, d, t, ds, dz, yg, ryg, tmp;
    // per input
    std::vector<double> u, q, su, sl, zu, zl, rd, hu, gtz, gz, rpu, rpl, dbox, du, dsu, dzu, dsl, dzl, bu, cu, x, yu,
        yl, dbu, dbl, ryu, ryl, v;
    // per stage (index k = 0..N)
    std::vector<double> xs, dy, cy, xv, bx, qy, W, K, Lc, kap;

    explicit Solver(const carmpc_cpu_problem& pr) : P(pr), N(pr.N), n(pr.n), p(pr.p) {
        for (auto* a : {&w, &s, &z, &rp, &gu, &d, &t, &ds, &dz, &yg, &ryg, &tmp}) a->assign(std::max(p, 1), 0.0);
        for (auto* a : {&u, &q, &su, &sl, &zu, &zl, &rd, &hu, &gtz, &gz, &rpu, &rpl, &dbox, &du, &dsu, &dzu, &dsl, &dzl,
                        &bu, &cu, &x, &yu, &yl, &dbu, &dbl, &ryu, &ryl, &v})
            a->assign(n, 0.0);
        for (auto* a : {&xs, &dy, &cy, &xv, &bx, &qy}) a->assign((size_t)(N + 1) * NX, 0.0);
        W.assign((size_t)(N + 1) * 16, 0.0);
        K.assign((size_t)N * 8, 0.0);
        Lc.assign((size_t)N * 3, 0.0);
        kap.assign((size_t)N * 2, 0.0);
    }

    // y_k = S_k v: y_0 = 0, y_{k+1} = A y_k + B v_k
    void rollout(const double* vv, double* y) const {
        for (int a = 0; a < NX; ++a) y[a] = 0.0;
        for (int tt = 0; tt < N; ++tt)
            for (int a = 0; a < NX; ++a) {
                double acc = P.B[a * 2] * vv[2 * tt] + P.B[a * 2 + 1] * vv[2 * tt + 1];
                for (int c = 0; c < NX; ++c) acc += P.A[a * 4 + c] * y[tt * NX + c];
                y[(tt + 1) * NX + a] = acc;
            }
    }
    // (G v)_r = c_r . y_{k_r}
    void grow(const double* y, double* out) const {
        for (int k = 1; k <= N; ++k)
            for (int r = P.row_begin[k]; r < P.row_begin[k + 1]; ++r) {
                double acc = 0.0;
                for (int a = 0; a < NX; ++a) acc += P.coef[(size_t)r * NX + a] * y[k * NX + a];
                out[r] = acc;
            }
    }
    // b^x_k = sum_{r in k} vals_r c_r
    void stage_sum(const double* vals, double* b) const {
        for (int a = 0; a < NX; ++a) b[a] = 0.0;
        for (int k = 1; k <= N; ++k) {
            double acc[NX] = {0, 0, 0, 0};
            for (int r = P.row_begin[k]; r < P.row_begin[k + 1]; ++r)
                for (int a = 0; a < NX; ++a) acc[a] += vals[r] * P.coef[(size_t)r * NX + a];
            for (int a = 0; a < NX; ++a) b[k * NX + a] = acc[a];
        }
    }
    // sum_k S_k' b_k: psi_k = b_k + A' psi_{k+1}, out_t = B' psi_{t+1}
    void adjoint(const double* b, double* out) const {
        double psi[NX] = {0, 0, 0, 0};
        for (int k = N; k >= 1; --k) {
            double np_[NX];
            for (int a = 0; a < NX; ++a) {
                double acc = b[k * NX + a];
                for (int c = 0; c < NX; ++c) acc += P.A[c * 4 + a] * psi[c];
                np_[a] = acc;
            }
            for (int a = 0; a < NX; ++a) psi[a] = np_[a];
            for (int c = 0; c < 2; ++c) {
                double acc = 0.0;
                for (int a = 0; a < NX; ++a) acc += P.B[a * 2 + c] * psi[a];
                out[2 * (k - 1) + c] = acc;
            }
        }
    }
    const double* qbar(int k) const { return k == N ? P.Pt : P.Q; }
    void qbar_y(const double* y, double* out) const {
        for (int a = 0; a < NX; ++a) out[a] = 0.0;
        for (int k = 1; k <= N; ++k) {
            const double* Qk = qbar(k);
            for (int a = 0; a < NX; ++a) {
                double acc = 0.0;
                for (int c = 0; c < NX; ++c) acc += Qk[a * 4 + c] * y[k * NX + c];
                out[k * NX + a] = acc;
            }
        }
    }
    void rhat(const double* vv, double* out) const {
        for (int tt = 0; tt < N; ++tt)
            for (int c = 0; c < 2; ++c) out[2 * tt + c] = P.R[c * 2] * vv[2 * tt] + P.R[c * 2 + 1] * vv[2 * tt + 1];
    }
    static void chol2(double r00, double r10, double r11, double* L) {   // guarded: non-positive pivot -> 1e128
        double p0 = r00;
        if (!(p0 > 0.0)) p0 = 1e128;
        const double l00 = std::sqrt(p0), l10 = r10 / l00;
        double p1 = r11 - l10 * l10;
        if (!(p1 > 0.0)) p1 = 1e128;
        L[0] = l00; L[1] = l10; L[2] = std::sqrt(p1);
    }
    static void chol2_solve(const double* L, double b0, double b1, double& x0, double& x1) {
        const double y0 = b0 / L[0], y1 = (b1 - L[1] * y0) / L[2];
        x1 = y1 / L[2];
        x0 = (y0 - L[1] * x1) / L[0];
    }
    // M = R_hat + diag(dbox) + sum_k S_k'(Qbar_k + W_k)S_k with W_k = sum d_r c_r c_r'
    void factor(const double* dr, const double* db) {
        for (int k = 1; k <= N; ++k) {
            double* Wk = &W[(size_t)k * 16];
            for (int e = 0; e < 16; ++e) Wk[e] = 0.0;
            for (int r = P.row_begin[k]; r < P.row_begin[k + 1]; ++r) {
                if (dr[r] == 0.0) continue;
                const double* c = &P.coef[(size_t)r * NX];
                for (int a = 0; a < NX; ++a)
                    for (int b = 0; b < NX; ++b) Wk[a * 4 + b] += dr[r] * c[a] * c[b];
            }
        }
        double Pm[16];
        for (int e = 0; e < 16; ++e) Pm[e] = P.Pt[e] + W[(size_t)N * 16 + e];
        for (int tt = N - 1; tt >= 0; --tt) {
            double PB[8], PA[16];
            for (int a = 0; a < NX; ++a)
                for (int c = 0; c < 2; ++c) {
                    double acc = 0.0;
                    for (int b = 0; b < NX; ++b) acc += Pm[a * 4 + b] * P.B[b * 2 + c];
                    PB[a * 2 + c] = acc;
                }
            mat4(Pm, P.A, PA);
            double re[4], F[8];   // Re = R + diag(db) + B'PB, F = B'PA
            for (int c = 0; c < 2; ++c)
                for (int e = 0; e < 2; ++e) {
                    double acc = P.R[c * 2 + e] + (c == e ? db[2 * tt + c] : 0.0);
                    for (int a = 0; a < NX; ++a) acc += P.B[a * 2 + c] * PB[a * 2 + e];
                    re[c * 2 + e] = acc;
                }
            for (int c = 0; c < 2; ++c)
                for (int m = 0; m < NX; ++m) {
                    double acc = 0.0;
                    for (int a = 0; a < NX; ++a) acc += P.B[a * 2 + c] * PA[a * 4 + m];
                    F[c * 4 + m] = acc;
                }
            double* L = &Lc[(size_t)tt * 3];
            chol2(re[0], re[2], re[3], L);
            double* Kt = &K[(size_t)tt * 8];
            for (int m = 0; m < NX; ++m) chol2_solve(L, F[m], F[4 + m], Kt[m], Kt[4 + m]);
            if (tt >= 1) {
                const double* Qt = qbar(tt);
                const double* Wt = &W[(size_t)tt * 16];
                double Pn[16];
                for (int a = 0; a < NX; ++a)
                    for (int b = 0; b < NX; ++b) {
                        double acc = Qt[a * 4 + b] + Wt[a * 4 + b];
                        for (int c = 0; c < NX; ++c) acc += P.A[c * 4 + a] * PA[c * 4 + b];
                        acc -= F[a] * Kt[b] + F[4 + a] * Kt[4 + b];
                        Pn[a * 4 + b] = acc;
                    }
                for (int a = 0; a < NX; ++a)
                    for (int b = 0; b < NX; ++b) Pm[a * 4 + b] = 0.5 * (Pn[a * 4 + b] + Pn[b * 4 + a]);
            }
        }
    }
    // v = M^{-1}(b^u + sum_k S_k' b^x_k), y = S v
    void riccati_solve(const double* b_u, const double* b_x, double* vv, double* y) {
        double pv[NX];
        for (int a = 0; a < NX; ++a) pv[a] = b_x[N * NX + a];
        for (int tt = N - 1; tt >= 0; --tt) {
            double g[2];
            for (int c = 0; c < 2; ++c) {
                double acc = b_u[2 * tt + c];
                for (int a = 0; a < NX; ++a) acc += P.B[a * 2 + c] * pv[a];
                g[c] = acc;
            }
            chol2_solve(&Lc[(size_t)tt * 3], g[0], g[1], kap[2 * tt], kap[2 * tt + 1]);
            if (tt >= 1) {
                const double* Kt = &K[(size_t)tt * 8];
                double np_[NX];
                for (int a = 0; a < NX; ++a) {
                    double acc = b_x[tt * NX + a];
                    for (int c = 0; c < NX; ++c) acc += P.A[c * 4 + a] * pv[c];
                    np_[a] = acc - Kt[a] * g[0] - Kt[4 + a] * g[1];
                }
                for (int a = 0; a < NX; ++a) pv[a] = np_[a];
            }
        }
        for (int a = 0; a < NX; ++a) y[a] = 0.0;
        for (int tt = 0; tt < N; ++tt) {
            const double* Kt = &K[(size_t)tt * 8];
            double v0 = kap[2 * tt], v1 = kap[2 * tt + 1];
            for (int a = 0; a < NX; ++a) {
                v0 -= Kt[a] * y[tt * NX + a];
                v1 -= Kt[4 + a] * y[tt * NX + a];
            }
            vv[2 * tt] = v0;
            vv[2 * tt + 1] = v1;
            for (int a = 0; a < NX; ++a) {
                double acc = P.B[a * 2] * v0 + P.B[a * 2 + 1] * v1;
                for (int c = 0; c < NX; ++c) acc += P.A[a * 4 + c] * y[tt * NX + c];
                y[(tt + 1) * NX + a] = acc;
            }
        }
    }
    static double maxstep(const double* vv, const double* dv, int len) {
        double m = kInf;
        for (int i = 0; i < len; ++i)
            if (dv[i] < 0.0) m = std::min(m, -vv[i] / dv[i]);
        return m;
    }
    static double amax(const double* vv, int len) {
        double m = 0.0;
        for (int i = 0; i < len; ++i) m = std::max(m, std::fabs(vv[i]));
        return m;
    }

    // One Newton solve of a normal trip: right-hand side from (rc, rcu, rcl) -> directions
    void newton(const double* rc, const double* rcu, const double* rcl, double bm, double* o_du, double* o_dy, double* o_ds,
                double* o_dz, double* o_dsu, double* o_dzu, double* o_dsl, double* o_dzl) {
        for (int r = 0; r < p; ++r) t[r] = (rc[r] - z[r] * rp[r]) / s[r];
        for (int i = 0; i < n; ++i)
            bu[i] = -rd[i] + ((rcu[i] - zu[i] * rpu[i]) / su[i] - (rcl[i] - zl[i] * rpl[i]) / sl[i]) * bm;
        stage_sum(t.data(), bx.data());
        riccati_solve(bu.data(), bx.data(), o_du, o_dy);
        grow(o_dy, tmp.data());
        for (int r = 0; r < p; ++r) {
            o_ds[r] = -rp[r] - tmp[r];
            o_dz[r] = (-rc[r] - z[r] * o_ds[r]) / s[r];
        }
        for (int i = 0; i < n; ++i) {
            o_dsu[i] = (-rpu[i] - o_du[i]) * bm;
            o_dsl[i] = (-rpl[i] + o_du[i]) * bm;
            o_dzu[i] = (-rcu[i] - zu[i] * o_dsu[i]) / su[i] * bm;
            o_dzl[i] = (-rcl[i] - zl[i] * o_dsl[i]) / sl[i] * bm;
        }
    }

    // Active-set polish: equality-constrained KKT on the rows with s < z, by iterative refinement
    // on the regularised factor (d = 1/delta on active rows).  Returns true when x is accepted.
    // A rejected attempt names what is wrong with its active set -- active rows whose multiplier
    // fails the sign test, inactive rows that are violated; the polish runs once more on the set
    // with those rows dropped / added (kPolishCorrections, as the grouped device kernel does).
    bool polish(const double* lbv, const double* ubv) {
        const double idl = 1.0 / kPolishDelta;
        const bool boxed = P.boxed;
        for (int r = 0; r < p; ++r) d[r] = s[r] < kPolishAct * z[r] ? idl : 0.0;
        for (int i = 0; i < n; ++i) {
            dbu[i] = (boxed && su[i] < kPolishAct * zu[i]) ? idl : 0.0;
            dbl[i] = (boxed && sl[i] < kPolishAct * zl[i]) ? idl : 0.0;
        }
        for (int attempt = 0;; ++attempt) {
            if (polish_attempt(lbv, ubv, attempt < kPolishCorrections)) return true;
            if (attempt >= kPolishCorrections || !polish_changed) return false;
        }
    }

    bool polish_changed = false;   // the last rejected attempt changed the active set
    // one attempt on the active set in d / dbu / dbl; when `correct`, a rejection updates the set
    bool polish_attempt(const double* lbv, const double* ubv, bool correct) {
        const double idl = 1.0 / kPolishDelta;
        const bool boxed = P.boxed;
        polish_changed = false;
        for (int i = 0; i < n; ++i) {
            dbox[i] = dbu[i] + dbl[i];
            x[i] = yu[i] = yl[i] = 0.0;
        }
        factor(d.data(), dbox.data());
        std::fill(xv.begin(), xv.end(), 0.0);
        for (int r = 0; r < p; ++r) yg[r] = 0.0;
        for (int pass = 0; pass <= kPolishRefine; ++pass) {
            grow(xv.data(), gu.data());
            for (int r = 0; r < p; ++r) {
                ryg[r] = d[r] > 0.0 ? w[r] - gu[r] : 0.0;
                t[r] = yg[r] - d[r] * ryg[r];
            }
            rhat(x.data(), hu.data());
            for (int i = 0; i < n; ++i) {
                ryu[i] = dbu[i] > 0.0 ? ubv[i] - x[i] : 0.0;
                ryl[i] = dbl[i] > 0.0 ? -lbv[i] + x[i] : 0.0;
                bu[i] = -q[i] - hu[i] - yu[i] + yl[i] + dbu[i] * ryu[i] - dbl[i] * ryl[i];
            }
            qbar_y(xv.data(), qy.data());
            stage_sum(t.data(), bx.data());
            for (size_t e = 0; e < bx.size(); ++e) bx[e] = -(qy[e] + bx[e]);
            riccati_solve(bu.data(), bx.data(), du.data(), dy.data());
            grow(dy.data(), tmp.data());
            for (int r = 0; r < p; ++r) yg[r] += d[r] * (tmp[r] - ryg[r]);
            for (int i = 0; i < n; ++i) {
                yu[i] += dbu[i] * (du[i] - ryu[i]);
                yl[i] += dbl[i] * (-du[i] - ryl[i]);
                x[i] += du[i];
            }
            for (size_t e = 0; e < xv.size(); ++e) xv[e] += dy[e];
        }
        rollout(x.data(), cy.data());
        grow(cy.data(), gu.data());
        double wsc = 0.0, viol = -kInf, ymin = 0.0, ysc = 0.0;
        bool fin = true;
        for (int r = 0; r < p; ++r) {
            wsc = std::max(wsc, std::fabs(w[r]));
            viol = std::max(viol, gu[r] - w[r]);
            ysc = std::max(ysc, std::fabs(yg[r]));
            const int pr = P.partner[r];
            const bool paired = d[r] > 0.0 && pr >= 0 && d[pr] > 0.0;   // an active equality pair: sign is free
            if (!paired) ymin = std::min(ymin, yg[r]);
        }
        for (int i = 0; i < n; ++i) {
            fin = fin && std::isfinite(x[i]);
            if (boxed) {
                wsc = std::max(wsc, std::max(std::fabs(lbv[i]), std::fabs(ubv[i])));
                viol = std::max(viol, std::max(x[i] - ubv[i], lbv[i] - x[i]));
                ysc = std::max(ysc, std::max(std::fabs(yu[i]), std::fabs(yl[i])));
                ymin = std::min(ymin, std::min(yu[i], yl[i]));
            }
        }
        const double vtol = kPolishTol * (1.0 + wsc), ytol = -kPolishTol * (1.0 + ysc);
        if (fin && viol <= vtol && ymin >= ytol) return true;
        if (!fin || !correct) return false;
        for (int r = 0; r < p; ++r) {   // (t: the next d, so that the pair test reads the old set)
            const int pr = P.partner[r];
            const bool paired = d[r] > 0.0 && pr >= 0 && d[pr] > 0.0;
            if (d[r] > 0.0) t[r] = (!paired && yg[r] < ytol) ? 0.0 : idl;
            else t[r] = gu[r] - w[r] > vtol ? idl : 0.0;
        }
        for (int r = 0; r < p; ++r) {
            polish_changed = polish_changed || t[r] != d[r];
            d[r] = t[r];
        }
        for (int i = 0; i < n && boxed; ++i) {
            const double nu = dbu[i] > 0.0 ? (yu[i] < ytol ? 0.0 : idl) : (x[i] - ubv[i] > vtol ? idl : 0.0);
            const double nl = dbl[i] > 0.0 ? (yl[i] < ytol ? 0.0 : idl) : (lbv[i] - x[i] > vtol ? idl : 0.0);
            polish_changed = polish_changed || nu != dbu[i] || nl != dbl[i];
            dbu[i] = nu;
            dbl[i] = nl;
        }
        return false;
    }

    // QP(x0): returns the status, writes n inputs and the iteration count
    int solve(const double* x0, const double* xref, double dist, double tol, double tol_mu, int max_iter, double* u_out,
              int32_t* iters_out) {
        for (int i = 0; i < n; ++i) u_out[i] = 0.0;
        *iters_out = 0;
        for (int r = 0; r < P.npre; ++r) {   // x0-only rows (G_r = 0)
            double vv = P.pre_w0[r];
            for (int a = 0; a < NX; ++a) vv -= P.pre_E[(size_t)r * NX + a] * x0[a];
            if (P.has_dist) vv -= P.pre_Ed[r] * dist;
            if (vv < -PRE_TOL) return CARMPC_PRIMAL_INFEASIBLE;
        }
        const bool boxed = P.boxed;
        const double bm = boxed ? 1.0 : 0.0;
        std::vector<double> lbv(n, -UNBOXED_BOUND), ubv(n, UNBOXED_BOUND);
        if (boxed) { lbv = P.lb; ubv = P.ub; }
        double dx[NX];
        for (int a = 0; a < NX; ++a) dx[a] = x0[a] - xref[a];
        for (int i = 0; i < n; ++i) {
            double acc = 0.0;
            for (int a = 0; a < NX; ++a) acc += P.hq[(size_t)i * NX + a] * dx[a];
            q[i] = acc;                                             // mpc.py:320-321
            u[i] = boxed ? std::min(std::max(0.0, lbv[i]), ubv[i]) : 0.0;
            su[i] = boxed ? std::max(ubv[i] - u[i], kInitSFloor) : 1.0;
            sl[i] = boxed ? std::max(u[i] - lbv[i], kInitSFloor) : 1.0;
            zu[i] = zl[i] = bm;
        }
        for (int r = 0; r < p; ++r) {
            double vv = P.w0[r];
            for (int a = 0; a < NX; ++a) vv -= P.E[(size_t)r * NX + a] * x0[a];
            if (P.has_dist) vv -= P.Ed[r] * dist;
            w[r] = vv;
        }
        rollout(u.data(), xs.data());
        grow(xs.data(), gu.data());
        const double qrel = (1.0 / (kInitQPerVar * n)) * amax(q.data(), n);
        const double mu0 = std::min(kInitMu0, std::max(kInitMuMin, qrel * qrel));
        for (int r = 0; r < p; ++r) { s[r] = std::max(w[r] - gu[r], kInitSFloor); z[r] = mu0 / s[r]; }
        for (int i = 0; i < n && boxed; ++i) { zu[i] = mu0 / su[i]; zl[i] = mu0 / sl[i]; }
        const int m = p + (boxed ? 2 * n : 0);
        const double inv_m = 1.0 / std::max(m, 1);
        double bnd = 0.0;
        for (int i = 0; i < n; ++i) bnd = std::max(bnd, std::max(std::fabs(lbv[i]), std::fabs(ubv[i])));
        const double bnorm = 1.0 + std::max(amax(w.data(), p), boxed ? bnd : 0.0);
        const double qnorm = 1.0 + amax(q.data(), n);
        int it = 0;
        bool polish_failed = false;
        std::vector<double> rc(std::max(p, 1)), rcu(n), rcl(n), dyT((size_t)(N + 1) * NX);
        for (;;) {
            rollout(u.data(), xs.data());
            grow(xs.data(), gu.data());
            double musum = 0.0;
            for (int r = 0; r < p; ++r) { rp[r] = gu[r] + s[r] - w[r]; musum += s[r] * z[r]; }
            for (int i = 0; i < n; ++i) {
                rpu[i] = (u[i] + su[i] - ubv[i]) * bm;
                rpl[i] = (-u[i] + sl[i] + lbv[i]) * bm;
                if (boxed) musum += su[i] * zu[i] + sl[i] * zl[i];
            }
            rhat(u.data(), hu.data());
            qbar_y(xs.data(), qy.data());
            adjoint(qy.data(), tmp_n());
            for (int i = 0; i < n; ++i) hu[i] += tmpn[i];
            stage_sum(z.data(), bx.data());
            adjoint(bx.data(), gtz.data());
            for (int i = 0; i < n; ++i) {
                gz[i] = gtz[i] + (zu[i] - zl[i]) * bm;
                rd[i] = hu[i] + q[i] + gz[i];
            }
            const double mu = musum * inv_m;
            const double rpn = std::max(amax(rp.data(), p), std::max(amax(rpu.data(), n), amax(rpl.data(), n)));
            const double rdn = amax(rd.data(), n);
            const double pscale = std::max(bnorm, std::max(1.0 + amax(gu.data(), p), 1.0 + (boxed ? amax(u.data(), n) : 0.0)));
            const double dscale = std::max(qnorm, std::max(1.0 + amax(hu.data(), n), 1.0 + amax(gz.data(), n)));
            *iters_out = it;
            if (!std::isfinite(mu) || !std::isfinite(rdn)) { copy_u(u_out, u.data()); return CARMPC_NUMERICAL; }
            const bool res_ok = rpn <= tol * pscale && rdn <= tol * dscale;
            const bool last = it >= max_iter;
            const double ptol = std::max(kPolishRes, tol);
            const bool pres_ok = rpn <= ptol * pscale && rdn <= ptol * dscale;
            const bool do_polish = !polish_failed && ((pres_ok && mu <= kPolishMu) || last);
            if (!do_polish) {
                if (last) { copy_u(u_out, u.data()); return CARMPC_MAX_ITER; }
                if (res_ok && mu <= tol_mu) { copy_u(u_out, u.data()); return CARMPC_OPTIMAL; }
                if (p > 0) {   // Farkas with the box: no u in [lb, ub] has G u <= w
                    double lo = 0.0, sc = 0.0, wz = 0.0, wza = 0.0;
                    for (int i = 0; i < n; ++i) {
                        lo += std::min(gtz[i] * lbv[i], gtz[i] * ubv[i]);
                        sc += std::fabs(gtz[i]) * std::max(std::fabs(lbv[i]), std::fabs(ubv[i]));
                    }
                    for (int r = 0; r < p; ++r) { wz += w[r] * z[r]; wza += std::fabs(w[r]) * z[r]; }
                    if (lo - wz > 1e-12 * (sc + wza)) { copy_u(u_out, u.data()); return CARMPC_PRIMAL_INFEASIBLE; }
                }
            } else {
                if (polish(lbv.data(), ubv.data())) { copy_u(u_out, x.data()); return CARMPC_OPTIMAL; }
                polish_failed = true;
                continue;
            }
            for (int r = 0; r < p; ++r) d[r] = z[r] / s[r];
            for (int i = 0; i < n; ++i) dbox[i] = (zu[i] / su[i] + zl[i] / sl[i]) * bm;
            factor(d.data(), dbox.data());
            // predictor
            for (int r = 0; r < p; ++r) rc[r] = s[r] * z[r];
            for (int i = 0; i < n; ++i) { rcu[i] = su[i] * zu[i] * bm; rcl[i] = sl[i] * zl[i] * bm; }
            newton(rc.data(), rcu.data(), rcl.data(), bm, du.data(), dy.data(), ds.data(), dz.data(), dsu.data(), dzu.data(),
                   dsl.data(), dzl.data());
            double a_aff = std::min(maxstep(s.data(), ds.data(), p), maxstep(z.data(), dz.data(), p));
            if (boxed)
                a_aff = std::min(std::min(a_aff, std::min(maxstep(su.data(), dsu.data(), n), maxstep(zu.data(), dzu.data(), n))),
                                 std::min(maxstep(sl.data(), dsl.data(), n), maxstep(zl.data(), dzl.data(), n)));
            a_aff = std::min(1.0, a_aff);
            double mua = 0.0;
            for (int r = 0; r < p; ++r) mua += (s[r] + a_aff * ds[r]) * (z[r] + a_aff * dz[r]);
            if (boxed)
                for (int i = 0; i < n; ++i)
                    mua += (su[i] + a_aff * dsu[i]) * (zu[i] + a_aff * dzu[i]) + (sl[i] + a_aff * dsl[i]) * (zl[i] + a_aff * dzl[i]);
            const double sg = mua * inv_m / mu;
            const double smu = sg * sg * sg * mu;
            // corrector
            for (int r = 0; r < p; ++r) rc[r] = s[r] * z[r] + ds[r] * dz[r] - smu;
            for (int i = 0; i < n; ++i) {
                rcu[i] = (su[i] * zu[i] + dsu[i] * dzu[i] - smu) * bm;
                rcl[i] = (sl[i] * zl[i] + dsl[i] * dzl[i] - smu) * bm;
            }
            newton(rc.data(), rcu.data(), rcl.data(), bm, du.data(), dy.data(), ds.data(), dz.data(), dsu.data(), dzu.data(),
                   dsl.data(), dzl.data());
            if (mu <= REFINE_MU) {
                // e = H du + G'dz + rd + box; M c = -e with the same factor
                rhat(du.data(), hu.data());
                for (int i = 0; i < n; ++i) bu[i] = -(hu[i] + rd[i] + (dzu[i] - dzl[i]) * bm);
                qbar_y(dy.data(), qy.data());
                stage_sum(dz.data(), bx.data());
                for (size_t e = 0; e < bx.size(); ++e) bx[e] = -(qy[e] + bx[e]);
                riccati_solve(bu.data(), bx.data(), cu.data(), cy.data());
                grow(cy.data(), tmp.data());
                for (int r = 0; r < p; ++r) {
                    const double cs = -tmp[r];
                    ds[r] += cs;
                    dz[r] -= z[r] * cs / s[r];
                }
                for (int i = 0; i < n; ++i) {
                    du[i] += cu[i];
                    if (boxed) {
                        dsu[i] -= cu[i]; dzu[i] += zu[i] * cu[i] / su[i];
                        dsl[i] += cu[i]; dzl[i] -= zl[i] * cu[i] / sl[i];
                    }
                }
            }
            double am = std::min(maxstep(s.data(), ds.data(), p), maxstep(z.data(), dz.data(), p));
            if (boxed)
                am = std::min(std::min(am, std::min(maxstep(su.data(), dsu.data(), n), maxstep(zu.data(), dzu.data(), n))),
                              std::min(maxstep(sl.data(), dsl.data(), n), maxstep(zl.data(), dzl.data(), n)));
            const double a = std::min(1.0, STEP_FRAC * am);
            for (int r = 0; r < p; ++r) { s[r] += a * ds[r]; z[r] += a * dz[r]; }
            for (int i = 0; i < n; ++i) {
                u[i] += a * du[i];
                if (boxed) { su[i] += a * dsu[i]; zu[i] += a * dzu[i]; sl[i] += a * dsl[i]; zl[i] += a * dzl[i]; }
            }
            polish_failed = false;
            ++it;
        }
    }

    std::vector<double> tmpn;
    double* tmp_n() {
        tmpn.resize(n);
        return tmpn.data();
    }
    void copy_u(double* dst, const double* src) const {
        for (int i = 0; i < n; ++i) dst[i] = src[i];
    }
};

int run_batch(const carmpc_cpu_problem* P, int64_t batch, const double* x0, const double* xref, const double* dist,
              double* u_out, int32_t* status, int32_t* iters, const carmpc_settings* st, int32_t threads) {
    if (!P) return set_error(CARMPC_EINVAL, "null problem");
    if (batch < 0) return set_error(CARMPC_EINVAL, "negative batch");
    if (batch == 0) return CARMPC_OK;
    if (!x0 || !u_out || !status) return set_error(CARMPC_EINVAL, "null batch pointer");
    if (dist && !P->has_dist) return set_error(CARMPC_EINVAL, "no disturbance model: call carmpc_cpu_problem_set_disturbance first");
    double tol = 1e-10, tol_mu = 1e-12;
    int max_iter = 60;
    if (st) {
        if (st->tol > 0) tol = st->tol;
        if (st->tol_mu > 0) tol_mu = st->tol_mu;
        if (st->max_iter > 0) max_iter = st->max_iter;
    }
    int nt = threads > 0 ? threads : (int)std::thread::hardware_concurrency();
    nt = (int)std::max<int64_t>(1, std::min<int64_t>(nt, (batch + 7) / 8));
    std::atomic<int64_t> next{0};
    auto worker = [&]() {
        Solver S(*P);
        for (;;) {
            const int64_t b0 = next.fetch_add(8);
            if (b0 >= batch) break;
            for (int64_t b = b0; b < std::min(batch, b0 + 8); ++b) {
                int32_t it = 0;
                status[b] = S.solve(x0 + b * NX, xref ? xref + b * NX : P->goal, dist ? dist[b] : 0.0, tol, tol_mu,
                                    max_iter, u_out + b * P->n, &it);
                if (iters) iters[b] = it;
            }
        }
    };
    if (nt == 1) {
        worker();
    } else {
        std::vector<std::thread> pool;
        for (int i = 0; i < nt; ++i) pool.emplace_back(worker);
        for (auto& th : pool) th.join();
    }
    return CARMPC_OK;
}

}  // namespace

extern "C" {

int carmpc_cpu_problem_create(const carmpc_model_desc* d, carmpc_cpu_problem** out) {
    if (!d || !out) return set_error(CARMPC_EINVAL, "null argument");
    *out = nullptr;
    if (d->nx != NX) return set_error(CARMPC_EUNSUPPORTED, "nx must be 4 (kinematic bicycle state)");
    if (d->nu != 2) return set_error(CARMPC_EUNSUPPORTED, "the CPU path needs nu = 2");
    if (d->N < 1 || d->N > 32) return set_error(CARMPC_EUNSUPPORTED, "N must be in [1,32]");
    if (!d->A || !d->B || !d->Q || !d->R || !d->P || !d->goal) return set_error(CARMPC_EINVAL, "null model matrix");
    if (d->n_state_rows < 0 || d->n_term_rows < 0) return set_error(CARMPC_EINVAL, "negative row count");
    if ((d->n_state_rows && (!d->state_A || !d->state_b)) || (d->n_term_rows && (!d->term_A || !d->term_b)))
        return set_error(CARMPC_EINVAL, "null constraint rows");
    if ((d->u_lower == nullptr) != (d->u_upper == nullptr)) return set_error(CARMPC_EINVAL, "u_lower/u_upper mismatch");
    auto* P = new carmpc_cpu_problem();
    const int N = d->N, n = 2 * N;
    P->N = N; P->n = n;
    std::memcpy(P->A, d->A, sizeof(P->A));
    std::memcpy(P->B, d->B, sizeof(P->B));
    std::memcpy(P->goal, d->goal, sizeof(P->goal));
    for (int i = 0; i < 4; ++i)
        for (int j = 0; j < 4; ++j) {
            P->Q[i * 4 + j] = 0.5 * (d->Q[i * 4 + j] + d->Q[j * 4 + i]);
            P->Pt[i * 4 + j] = 0.5 * (d->P[i * 4 + j] + d->P[j * 4 + i]);
        }
    for (int i = 0; i < 2; ++i)
        for (int j = 0; j < 2; ++j) P->R[i * 2 + j] = 0.5 * (d->R[i * 2 + j] + d->R[j * 2 + i]);
    // powers of A and Phi_m = A^m B (matrix_gen.py:6-32)
    std::vector<double> Ap((size_t)(N + 1) * 16), Phi((size_t)N * 8);
    for (int e = 0; e < 16; ++e) Ap[e] = (e % 5 == 0) ? 1.0 : 0.0;
    for (int m = 1; m <= N; ++m) mat4(P->A, &Ap[(size_t)(m - 1) * 16], &Ap[(size_t)m * 16]);
    for (int m = 0; m < N; ++m)
        for (int a = 0; a < NX; ++a)
            for (int c = 0; c < 2; ++c) {
                double acc = 0.0;
                for (int b = 0; b < NX; ++b) acc += Ap[(size_t)m * 16 + a * 4 + b] * P->B[b * 2 + c];
                Phi[(size_t)m * 8 + a * 2 + c] = acc;
            }
    // h = S'Q_hat T (matrix_gen.py:66): row (t, c) = sum_{k > t} Phi_{k-1-t}[:, c]' Qbar_k A^k, with the
    // reference's own (unsymmetrised) Q and P
    P->hq.assign((size_t)n * NX, 0.0);
    for (int k = 1; k <= N; ++k) {
        const double* Qk = k == N ? d->P : d->Q;
        double QA[16];
        mat4(Qk, &Ap[(size_t)k * 16], QA);
        for (int t = 0; t < k; ++t)
            for (int c = 0; c < 2; ++c)
                for (int b = 0; b < NX; ++b) {
                    double acc = 0.0;
                    for (int a = 0; a < NX; ++a) acc += Phi[(size_t)(k - 1 - t) * 8 + a * 2 + c] * QA[a * 4 + b];
                    P->hq[(size_t)(2 * t + c) * NX + b] += acc;
                }
    }
    // rows in the reference's order (mpc.py:323-332): terminal rows on x_N, then one block of N rows
    // per state half-space (x_1..x_N)
    const int nt = d->n_term_rows, ns = d->n_state_rows, pa = nt + ns * N;
    std::vector<double> G((size_t)pa * n, 0.0), E((size_t)pa * NX), rhs(pa);
    P->all_stage.resize(pa); P->all_coef.resize((size_t)pa * NX); P->all_norm.resize(pa);
    double nmax = 0.0;
    for (int r = 0; r < pa; ++r) {
        const double* c = r < nt ? d->term_A + (size_t)r * NX : d->state_A + (size_t)((r - nt) / N) * NX;
        const int k = r < nt ? N : (r - nt) % N + 1;
        rhs[r] = r < nt ? d->term_b[r] : d->state_b[(r - nt) / N];
        P->all_stage[r] = k;
        for (int a = 0; a < NX; ++a) P->all_coef[(size_t)r * NX + a] = c[a];
        double nn = 0.0;
        for (int t = 0; t < k; ++t)
            for (int cc = 0; cc < 2; ++cc) {
                double acc = 0.0;
                for (int a = 0; a < NX; ++a) acc += c[a] * Phi[(size_t)(k - 1 - t) * 8 + a * 2 + cc];
                G[(size_t)r * n + 2 * t + cc] = acc;
                nn += acc * acc;
            }
        for (int b = 0; b < NX; ++b) {
            double acc = 0.0;
            for (int a = 0; a < NX; ++a) acc += c[a] * Ap[(size_t)k * 16 + a * 4 + b];
            E[(size_t)r * NX + b] = acc;
        }
        P->all_norm[r] = std::sqrt(nn);
        nmax = std::max(nmax, P->all_norm[r]);
    }
    const double thr = ZERO_ROW * nmax;
    for (int r = 0; r < pa; ++r) (P->all_norm[r] > thr ? P->qp_rows : P->pre_rows).push_back(r);
    // QP rows sorted by stage (stable: keeps the reference order inside a stage)
    std::stable_sort(P->qp_rows.begin(), P->qp_rows.end(), [&](int a, int b) { return P->all_stage[a] < P->all_stage[b]; });
    P->p = (int)P->qp_rows.size();
    P->npre = (int)P->pre_rows.size();
    P->coef.resize((size_t)P->p * NX); P->w0.resize(P->p); P->E.resize((size_t)P->p * NX);
    P->row_begin.assign(N + 2, 0);
    std::vector<double> Gn((size_t)P->p * n);
    for (int i = 0; i < P->p; ++i) {
        const int r = P->qp_rows[i];
        const double inv = 1.0 / P->all_norm[r];
        for (int a = 0; a < NX; ++a) {
            P->coef[(size_t)i * NX + a] = P->all_coef[(size_t)r * NX + a] * inv;
            P->E[(size_t)i * NX + a] = E[(size_t)r * NX + a] * inv;
        }
        P->w0[i] = rhs[r] * inv;
        for (int j = 0; j < n; ++j) Gn[(size_t)i * n + j] = G[(size_t)r * n + j] * inv;
        ++P->row_begin[P->all_stage[r] + 1];
    }
    for (int k = 1; k <= N + 1; ++k) P->row_begin[k] += P->row_begin[k - 1];
    P->pre_w0.resize(P->npre); P->pre_E.resize((size_t)P->npre * NX);
    for (int i = 0; i < P->npre; ++i) {
        const int r = P->pre_rows[i];
        P->pre_w0[i] = rhs[r];
        for (int a = 0; a < NX; ++a) P->pre_E[(size_t)i * NX + a] = E[(size_t)r * NX + a];
    }
    // opposite-row pairs: an equality written as two rows (the goal-box fallback, mpc.py:107-117)
    P->partner.assign(P->p, -1);
    for (int r = 0; r < P->p; ++r)
        for (int r2 = 0; r2 < P->p && P->partner[r] < 0; ++r2) {
            if (r2 == r || P->w0[r2] != -P->w0[r]) continue;
            bool same = true;
            for (int a = 0; a < NX && same; ++a) same = P->E[(size_t)r2 * NX + a] == -P->E[(size_t)r * NX + a];
            for (int j = 0; j < n && same; ++j) same = Gn[(size_t)r2 * n + j] == -Gn[(size_t)r * n + j];
            if (same) P->partner[r] = r2;
        }
    P->boxed = d->u_lower != nullptr;
    P->lb.assign(n, -1.0); P->ub.assign(n, 1.0);
    if (P->boxed)
        for (int t = 0; t < N; ++t)
            for (int c = 0; c < 2; ++c) { P->lb[2 * t + c] = d->u_lower[c]; P->ub[2 * t + c] = d->u_upper[c]; }
    *out = P;
    return CARMPC_OK;
}

void carmpc_cpu_problem_destroy(carmpc_cpu_problem* prob) { delete prob; }

int carmpc_cpu_problem_info(const carmpc_cpu_problem* P, int32_t* n, int32_t* p, int32_t* npre, int32_t* nx, int32_t* N) {
    if (!P) return set_error(CARMPC_EINVAL, "null problem");
    if (n) *n = P->n;
    if (p) *p = P->p;
    if (npre) *npre = P->npre;
    if (nx) *nx = NX;
    if (N) *N = P->N;
    return CARMPC_OK;
}

int carmpc_cpu_problem_set_disturbance(carmpc_cpu_problem* P, const double* Bd) {
    if (!P || !Bd) return set_error(CARMPC_EINVAL, "null argument");
    const int N = P->N;
    // ABd_k = sum_{m<k} A^m Bd (mpc.py:631-635); row offset Ed_r = c_r . ABd_{k_r}
    std::vector<double> abd((size_t)(N + 1) * NX, 0.0);
    double Am[16], acc[NX] = {0, 0, 0, 0};
    for (int e = 0; e < 16; ++e) Am[e] = (e % 5 == 0) ? 1.0 : 0.0;
    for (int k = 1; k <= N; ++k) {
        for (int a = 0; a < NX; ++a)
            for (int b = 0; b < NX; ++b) acc[a] += Am[a * 4 + b] * Bd[b];
        for (int a = 0; a < NX; ++a) abd[(size_t)k * NX + a] = acc[a];
        double nx_[16];
        mat4(P->A, Am, nx_);
        std::memcpy(Am, nx_, sizeof(Am));
    }
    auto ed = [&](int r) {
        double v = 0.0;
        for (int a = 0; a < NX; ++a) v += P->all_coef[(size_t)r * NX + a] * abd[(size_t)P->all_stage[r] * NX + a];
        return v;
    };
    P->Ed.resize(P->p);
    for (int i = 0; i < P->p; ++i) P->Ed[i] = ed(P->qp_rows[i]) / P->all_norm[P->qp_rows[i]];
    P->pre_Ed.resize(P->npre);
    for (int i = 0; i < P->npre; ++i) P->pre_Ed[i] = ed(P->pre_rows[i]);
    P->has_dist = true;
    return CARMPC_OK;
}

int carmpc_cpu_solve_batch(const carmpc_cpu_problem* prob, int64_t batch, const double* x0, const double* xref,
                           double* u_out, int32_t* status, int32_t* iters, const carmpc_settings* settings,
                           int32_t threads) {
    return run_batch(prob, batch, x0, xref, nullptr, u_out, status, iters, settings, threads);
}

int carmpc_cpu_solve_batch_dist(const carmpc_cpu_problem* prob, int64_t batch, const double* x0, const double* xref,
                                const double* dist, double* u_out, int32_t* status, int32_t* iters,
                                const carmpc_settings* settings, int32_t threads) {
    if (!dist) return set_error(CARMPC_EINVAL, "null batch pointer");
    return run_batch(prob, batch, x0, xref, dist, u_out, status, iters, settings, threads);
}

}  // extern "C"
