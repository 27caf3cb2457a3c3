// ipm_riccati.hip -- grouped stage-form Mehrotra IPM: 16 lanes per QP, 4 QPs per wavefront.
//
// Replaces the per-step cvxpy solve of lib/mpc.py:334-335 / 477-478 with the algorithm of
// DESIGN.md §3 (oracle/qp.py::ipm), applying M^{-1} by a backward Riccati recursion and a
// forward roll-out over the horizon (oracle/riccati.py, the CPU restatement this kernel
// follows line by line).  Every QP row acts on one predicted state x_k (mpc.py:196-253),
// and H = R_hat + S'Q_hat S (matrix_gen.py:35-72), so
//     M = H + G'DG + diag(box) = R_hat + diag(Db) + sum_k S_k'(Qbar_k + W_k) S_k.
//
// Layout (one QP per 16-lane DPP row; group g = lane>>4, j = lane&15):
//   * row state in registers: lane j owns stage j+1 (segment 0) and j+17 (segment 1) -- the
//     rows of those stages sit in its 2 x 8 slots; stage-N rows that do not fit the owner
//     spill into the segments whose stage number exceeds N (capi.hip::riccati_layout);
//     the owner of stage t+1 also owns the input u_t (both components) and its box rows;
//   * stage recursions (adjoints, Riccati factorization, backward/forward solves) run
//     redundantly in all 16 lanes of the group -- scalar code, no cross-lane traffic --
//     reading/writing per-stage records in LDS (W_k, rhs, factor K_t / Re_t, y_k, v_t);
//   * per-QP reductions are 16-lane DPP butterflies (lanes.h), bitwise row-uniform.
// The 4 groups of a wave advance trip by trip together; a finished group idles until the
// wave's 4 instances are done.
#include "carmpc_internal.h"
#include "lanes.h"

#include <hip/hip_runtime.h>
#include <math.h>

namespace carmpc {

namespace {

using namespace lanes;

constexpr int G16 = kRicLanes;
constexpr int RSEG = kRicSeg;
constexpr int RS = kRicSlots;
constexpr int REC = 20;   // doubles per stage record (160 B)
// record t (stage t+1, input t):
//   [0..9]   W_{t+1} (packed) | lamZ_{t+1} [0..3], lamH_{t+1} [4..7] | factor: K_t [0..7], il00 l10 il11 [8..10]
//   [12..15] b^x_{t+1} | y_{t+1} | gz_t [12..13], hs_t [14..15]
//   [16..17] b^u_t | v_t
//   [18..19] Db_t | kappa_t
constexpr int O_K = 0, O_CH = 8, O_BX = 12, O_BU = 16, O_DB = 18;

constexpr double POLISH_MU = 1e-8;
constexpr double POLISH_DELTA = 1e-10;
constexpr int POLISH_REFINE = 3;
constexpr double POLISH_TOL = 1e-11;

template <int N>
struct RicShared {
    double2 cf01[RS * G16];   // slot (s, j): c~0, c~1
    double2 cf23[RS * G16];   // c~2, c~3
    int32_t partner[RS * G16];
    double lb[64], ub[64];
};
template <int N>
struct RicWave {
    double rec[4][N * REC];
    double w[RS][64];         // w = w0 - E x0 per (slot, lane)
    double scr[RS][64];       // polish verification scratch
};

__device__ __forceinline__ void wb() { __builtin_amdgcn_wave_barrier(); }

template <int N, int WPB>
__global__ void __launch_bounds__(WPB * 64) ipm_riccati_kernel(DevProblem P, int64_t batch, const double* __restrict__ x0,
                                                               const double* __restrict__ xref, double* __restrict__ u_out,
                                                               int64_t ld_u, int32_t* __restrict__ status_out,
                                                               int32_t* __restrict__ iters_out, Settings S) {
    __shared__ __attribute__((aligned(16))) RicShared<N> sh;
    __shared__ __attribute__((aligned(16))) RicWave<N> wscr[WPB];
    const StageMats& MT = P.mats;
    for (int i = threadIdx.x; i < RS * G16; i += blockDim.x) {
        sh.cf01[i] = make_double2(P.r_coef[i * 4 + 0], P.r_coef[i * 4 + 1]);
        sh.cf23[i] = make_double2(P.r_coef[i * 4 + 2], P.r_coef[i * 4 + 3]);
        sh.partner[i] = P.r_partner ? P.r_partner[i] : -1;
    }
    for (int i = threadIdx.x; i < 64; i += blockDim.x) {
        const bool bx = i < 2 * N && P.boxed;
        sh.lb[i] = bx ? P.lb[i] : -UNBOXED_BOUND;
        sh.ub[i] = bx ? P.ub[i] : UNBOXED_BOUND;
    }
    __syncthreads();

    const int lane = threadIdx.x & 63;
    const int wave = threadIdx.x >> 6;
    const int g = lane >> 4, j = lane & 15;
    RicWave<N>& wv = wscr[wave];
    double* rec = wv.rec[g];
    const bool boxed = P.boxed != 0;
    // segment stages: seg 0 -> j+1, seg 1 -> j+17 (overflow segments -> stage N)
    int kseg[2];
    bool own[2], isN[2];
#pragma unroll
    for (int sg = 0; sg < 2; ++sg) {
        const int k = j + 1 + 16 * sg;
        own[sg] = k <= N;
        kseg[sg] = k <= N ? k : N;
        isN[sg] = kseg[sg] == N;
    }
    bool rv[RS];
#pragma unroll
    for (int s = 0; s < RS; ++s) rv[s] = P.r_valid[s * G16 + j] != 0;
    const int p = P.p;
    const int m_rows = p + (boxed ? 4 * N : 0);
    const double inv_m = 1.0 / (double)(m_rows > 0 ? m_rows : 1);
    const double idl = 1.0 / POLISH_DELTA;

    // ---- helpers ----------------------------------------------------------------------
    auto cf = [&](int s, double (&c)[4]) {
        const double2 a = sh.cf01[s * G16 + j], b = sh.cf23[s * G16 + j];
        c[0] = a.x; c[1] = a.y; c[2] = b.x; c[3] = b.y;
    };
    auto dot4 = [&](const double (&c)[4], const double (&y)[4]) {
        return fma(c[3], y[3], fma(c[2], y[2], fma(c[1], y[1], c[0] * y[0])));
    };
    auto rd4 = [&](int off, double (&v)[4]) {   // rec[off..off+3]
        const double2 a = *reinterpret_cast<const double2*>(rec + off);
        const double2 b = *reinterpret_cast<const double2*>(rec + off + 2);
        v[0] = a.x; v[1] = a.y; v[2] = b.x; v[3] = b.y;
    };
    auto wr4 = [&](int off, const double (&v)[4]) {
        *reinterpret_cast<double2*>(rec + off) = make_double2(v[0], v[1]);
        *reinterpret_cast<double2*>(rec + off + 2) = make_double2(v[2], v[3]);
    };
    auto rd2 = [&](int off, double& a, double& b) {
        const double2 v = *reinterpret_cast<const double2*>(rec + off);
        a = v.x; b = v.y;
    };
    auto rdK = [&](int r, double (&K)[8]) {
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            const double2 v = *reinterpret_cast<const double2*>(rec + r + O_K + 2 * e);
            K[2 * e] = v.x;
            K[2 * e + 1] = v.y;
        }
    };
    auto wr2 = [&](int off, double a, double b) { *reinterpret_cast<double2*>(rec + off) = make_double2(a, b); };
    // y += Qbar_k v (k runtime, 1..N) -- only segment owners call it
    auto add_qbar = [&](bool termN, const double (&v)[4], double (&y)[4], double sgn) {
#pragma unroll
        for (int a = 0; a < 4; ++a) {
            double acc = 0.0;
#pragma unroll
            for (int b = 0; b < 4; ++b) acc = fma(termN ? MT.P[a * 4 + b] : MT.Q[a * 4 + b], v[b], acc);
            y[a] = fma(sgn, acc, y[a]);
        }
    };
    // sum the stage-N partials of the 16 lanes; owners write b^x (plus Qbar term) of their stages
    auto write_bx = [&](double (&acc)[2][4], const double (&qv)[2][4], double qsgn) {
        double pn[4];
#pragma unroll
        for (int a = 0; a < 4; ++a) pn[a] = (isN[0] ? acc[0][a] : 0.0) + (isN[1] ? acc[1][a] : 0.0);
#pragma unroll
        for (int a = 0; a < 4; ++a) pn[a] = row_sum(pn[a]);
#pragma unroll
        for (int sg = 0; sg < 2; ++sg) {
            if (own[sg]) {
                double v[4];
#pragma unroll
                for (int a = 0; a < 4; ++a) v[a] = isN[sg] ? pn[a] : acc[sg][a];
                if (qsgn != 0.0) add_qbar(kseg[sg] == N, qv[sg], v, qsgn);
                wr4((kseg[sg] - 1) * REC + O_BX, v);
            }
        }
    };

    // ---- stage recursions (redundant in the 16 lanes of a group) ----------------------
    // backward linear pass: p_N = b^x_N; g_t = b^u_t + B'p_{t+1}; kappa_t = Re_t^{-1} g_t;
    // p_t = b^x_t + A'p_{t+1} - K_t'g_t   (oracle/riccati.py::riccati_solve)
    auto back_linear = [&]() {
        wb();
        double pv[4];
        rd4((N - 1) * REC + O_BX, pv);
#pragma unroll
        for (int t = N - 1; t >= 0; --t) {
            const int r = t * REC;
            double bu0, bu1, il00, l10, il11, dummy;
            rd2(r + O_BU, bu0, bu1);
            rd2(r + O_CH, il00, l10);
            rd2(r + O_CH + 2, il11, dummy);
            double K[8];
            rdK(r, K);
            double g0 = bu0, g1 = bu1;
#pragma unroll
            for (int a = 0; a < 4; ++a) {
                g0 = fma(MT.B[a * 2 + 0], pv[a], g0);
                g1 = fma(MT.B[a * 2 + 1], pv[a], g1);
            }
            const double y0 = g0 * il00;
            const double y1 = fma(-l10, y0, g1) * il11;
            const double k1 = y1 * il11;
            const double k0 = fma(-l10, k1, y0) * il00;
            if (j == 0) wr2(r + O_DB, k0, k1);
            if (t >= 1) {
                double bx[4];
                rd4(r - REC + O_BX, bx);
                double np[4];
#pragma unroll
                for (int a = 0; a < 4; ++a) {
                    double acc = bx[a];
#pragma unroll
                    for (int c = 0; c < 4; ++c) acc = fma(MT.A[c * 4 + a], pv[c], acc);
                    acc = fma(-K[a], g0, acc);
                    np[a] = fma(-K[4 + a], g1, acc);
                }
#pragma unroll
                for (int a = 0; a < 4; ++a) pv[a] = np[a];
            }
        }
        wb();
    };
    // forward pass: y_0 = 0; v_t = kappa_t - K_t y_t; y_{t+1} = A y_t + B v_t -> rec
    auto forward = [&]() {
        wb();
        double y[4] = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
        for (int t = 0; t < N; ++t) {
            const int r = t * REC;
            double k0, k1;
            rd2(r + O_DB, k0, k1);
            double K[8];
            rdK(r, K);
            double v0 = k0, v1 = k1;
#pragma unroll
            for (int a = 0; a < 4; ++a) {
                v0 = fma(-K[a], y[a], v0);
                v1 = fma(-K[4 + a], y[a], v1);
            }
            double ny[4];
#pragma unroll
            for (int a = 0; a < 4; ++a) {
                double acc = MT.B[a * 2] * v0;
                acc = fma(MT.B[a * 2 + 1], v1, acc);
#pragma unroll
                for (int c = 0; c < 4; ++c) acc = fma(MT.A[a * 4 + c], y[c], acc);
                ny[a] = acc;
            }
#pragma unroll
            for (int a = 0; a < 4; ++a) y[a] = ny[a];
            if (j == 0) {
                wr4(r + O_BX, y);
                wr2(r + O_BU, v0, v1);
            }
        }
        wb();
    };
    // plain roll-out of v_t stored in rec[t][O_BU] (initial point): y -> rec[t][O_BX]
    auto rollout = [&]() {
        wb();
        double y[4] = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
        for (int t = 0; t < N; ++t) {
            const int r = t * REC;
            double v0, v1;
            rd2(r + O_BU, v0, v1);
            double ny[4];
#pragma unroll
            for (int a = 0; a < 4; ++a) {
                double acc = MT.B[a * 2] * v0;
                acc = fma(MT.B[a * 2 + 1], v1, acc);
#pragma unroll
                for (int c = 0; c < 4; ++c) acc = fma(MT.A[a * 4 + c], y[c], acc);
                ny[a] = acc;
            }
#pragma unroll
            for (int a = 0; a < 4; ++a) y[a] = ny[a];
            wb();
            if (j == 0) wr4(r + O_BX, y);
        }
        wb();
    };
    // Riccati factorization with W_k, Db_t from rec, fused with the backward linear pass
    // of the first right-hand side (b^x, b^u in rec)   (oracle/riccati.py::riccati_factor)
    auto factor_and_back = [&]() {
        wb();
        double Pm[10], pv[4];
        {
            double Wn[10];
#pragma unroll
            for (int e = 0; e < 5; ++e) rd2((N - 1) * REC + 2 * e, Wn[2 * e], Wn[2 * e + 1]);
#pragma unroll
            for (int a = 0; a < 4; ++a)
#pragma unroll
                for (int b = a; b < 4; ++b) Pm[sym10(a, b)] = MT.P[a * 4 + b] + Wn[sym10(a, b)];
            rd4((N - 1) * REC + O_BX, pv);
        }
#pragma unroll 1
        for (int t = N - 1; t >= 0; --t) {
            const int r = t * REC;
            double db0, db1, bu0, bu1;
            rd2(r + O_DB, db0, db1);
            rd2(r + O_BU, bu0, bu1);
            // PB = P B (4x2), PA = P A (4x4)
            double PB[4][2], PA[4][4];
#pragma unroll
            for (int a = 0; a < 4; ++a) {
#pragma unroll
                for (int c = 0; c < 2; ++c) {
                    double acc = 0.0;
#pragma unroll
                    for (int b = 0; b < 4; ++b) acc = fma(Pm[sym10(a, b)], MT.B[b * 2 + c], acc);
                    PB[a][c] = acc;
                }
#pragma unroll
                for (int m = 0; m < 4; ++m) {
                    double acc = 0.0;
#pragma unroll
                    for (int b = 0; b < 4; ++b) acc = fma(Pm[sym10(a, b)], MT.A[b * 4 + m], acc);
                    PA[a][m] = acc;
                }
            }
            // Re = R + diag(Db) + B'PB ; F = B'PA
            double re00 = MT.R[0] + db0, re10 = MT.R[2], re11 = MT.R[3] + db1;
#pragma unroll
            for (int a = 0; a < 4; ++a) {
                re00 = fma(MT.B[a * 2 + 0], PB[a][0], re00);
                re10 = fma(MT.B[a * 2 + 1], PB[a][0], re10);
                re11 = fma(MT.B[a * 2 + 1], PB[a][1], re11);
            }
            double F[2][4];
#pragma unroll
            for (int c = 0; c < 2; ++c)
#pragma unroll
                for (int m = 0; m < 4; ++m) {
                    double acc = 0.0;
#pragma unroll
                    for (int a = 0; a < 4; ++a) acc = fma(MT.B[a * 2 + c], PA[a][m], acc);
                    F[c][m] = acc;
                }
            // guarded 2x2 Cholesky (non-positive pivot -> 1e128, as qp._chol_guarded)
            double p0 = re00;
            if (!(p0 > 0.0)) p0 = 1e128;
            const double il00 = frsq(p0);
            const double l10 = re10 * il00;
            double p1 = fma(-l10, l10, re11);
            if (!(p1 > 0.0)) p1 = 1e128;
            const double il11 = frsq(p1);
            double K[2][4];
#pragma unroll
            for (int m = 0; m < 4; ++m) {
                const double y0 = F[0][m] * il00;
                const double y1 = fma(-l10, y0, F[1][m]) * il11;
                K[1][m] = y1 * il11;
                K[0][m] = fma(-l10, K[1][m], y0) * il00;
            }
            double g0 = bu0, g1 = bu1;
#pragma unroll
            for (int a = 0; a < 4; ++a) {
                g0 = fma(MT.B[a * 2 + 0], pv[a], g0);
                g1 = fma(MT.B[a * 2 + 1], pv[a], g1);
            }
            const double y0 = g0 * il00;
            const double y1 = fma(-l10, y0, g1) * il11;
            const double k1 = y1 * il11;
            const double k0 = fma(-l10, k1, y0) * il00;
            wb();
            if (j == 0) {
                wr4(r + O_K, K[0]);
                wr4(r + O_K + 4, K[1]);
                wr2(r + O_CH, il00, l10);
                wr2(r + O_CH + 2, il11, 0.0);
                wr2(r + O_DB, k0, k1);
            }
            if (t >= 1) {
                double Wt[10], bx[4];
#pragma unroll
                for (int e = 0; e < 5; ++e) rd2(r - REC + 2 * e, Wt[2 * e], Wt[2 * e + 1]);
                rd4(r - REC + O_BX, bx);
                // P_t = Qbar_t + W_t + A'PA - F'K  (upper triangle)
#pragma unroll
                for (int a = 0; a < 4; ++a)
#pragma unroll
                    for (int b = a; b < 4; ++b) {
                        double acc = MT.Q[a * 4 + b] + Wt[sym10(a, b)];
#pragma unroll
                        for (int c = 0; c < 4; ++c) acc = fma(MT.A[c * 4 + a], PA[c][b], acc);
                        acc = fma(-F[0][a], K[0][b], acc);
                        Pm[sym10(a, b)] = fma(-F[1][a], K[1][b], acc);
                    }
                double np[4];
#pragma unroll
                for (int a = 0; a < 4; ++a) {
                    double acc = bx[a];
#pragma unroll
                    for (int c = 0; c < 4; ++c) acc = fma(MT.A[c * 4 + a], pv[c], acc);
                    acc = fma(-K[0][a], g0, acc);
                    np[a] = fma(-K[1][a], g1, acc);
                }
#pragma unroll
                for (int a = 0; a < 4; ++a) pv[a] = np[a];
            }
        }
        wb();
    };

    const int64_t per_wave = 4;
    const int64_t stride = (int64_t)gridDim.x * WPB * per_wave;
    for (int64_t base = ((int64_t)blockIdx.x * WPB + wave) * per_wave; base < batch; base += stride) {
        const int64_t inst = base + g;
        bool active = inst < batch;
        const int64_t ii = active ? inst : 0;
        double xv0[NX], xr[NX];
#pragma unroll
        for (int k = 0; k < NX; ++k) {
            xv0[k] = x0[ii * NX + k];
            xr[k] = xref ? xref[ii * NX + k] : P.goal[k];
        }
        // x0-only rows (G_r = 0): preconditions
        {
            double bad = 0.0;
            for (int r = j; r < P.npre; r += G16) {
                double v = P.pre_w0[r];
#pragma unroll
                for (int k = 0; k < NX; ++k) v -= P.pre_E[r * NX + k] * xv0[k];
                bad = v < -PRE_TOL ? 1.0 : bad;
            }
            bad = row_max(bad);
            if (active && bad > 0.0) {
#pragma unroll
                for (int sg = 0; sg < 2; ++sg)
                    if (own[sg]) {
                        const int t = kseg[sg] - 1;
                        u_out[inst * ld_u + 2 * t] = 0.0;
                        u_out[inst * ld_u + 2 * t + 1] = 0.0;
                    }
                if (j == 0) {
                    status_out[inst] = CARMPC_PRIMAL_INFEASIBLE;
                    if (iters_out) iters_out[inst] = 0;
                }
                active = false;
            }
        }
        // per-slot w, q and box of the owned inputs, initial point
        double s_[RS], z_[RS], ra[RS], rb[RS];
        double u_[2][2], q_[2][2], su[2][2], sl[2][2], zu[2][2], zl[2][2];
        double xs[2][4];
        double bn = 0.0, qn = 0.0;
#pragma unroll
        for (int s = 0; s < RS; ++s) {
            double v = 0.0;
            if (rv[s]) {
                const int e = s * G16 + j;
                v = P.r_w0[e];
#pragma unroll
                for (int k = 0; k < NX; ++k) v -= P.r_E[e * NX + k] * xv0[k];
            }
            wv.w[s][lane] = v;
            bn = fmax(bn, fabs(v));
        }
#pragma unroll
        for (int sg = 0; sg < 2; ++sg) {
            const int t = kseg[sg] - 1;
#pragma unroll
            for (int c = 0; c < 2; ++c) {
                const int i = 2 * t + c;
                double q = 0.0;
#pragma unroll
                for (int k = 0; k < NX; ++k) q = fma(P.hq[i * NX + k], xv0[k] - xr[k], q);
                const double lb = sh.lb[i], ub = sh.ub[i];
                const bool bx = own[sg] && boxed;
                q_[sg][c] = own[sg] ? q : 0.0;
                u_[sg][c] = bx ? fmin(fmax(0.0, lb), ub) : 0.0;
                su[sg][c] = bx ? fmax(ub - u_[sg][c], 1.0) : 1.0;
                sl[sg][c] = bx ? fmax(u_[sg][c] - lb, 1.0) : 1.0;
                zu[sg][c] = bx ? 1.0 : 0.0;
                zl[sg][c] = bx ? 1.0 : 0.0;
                bn = bx ? fmax(bn, fmax(fabs(lb), fabs(ub))) : bn;
                qn = fmax(qn, fabs(q_[sg][c]));
            }
        }
        // xs = S u0 (u0 = clip(0, lb, ub))
#pragma unroll
        for (int sg = 0; sg < 2; ++sg)
            if (own[sg]) wr2((kseg[sg] - 1) * REC + O_BU, u_[sg][0], u_[sg][1]);
        rollout();
#pragma unroll
        for (int sg = 0; sg < 2; ++sg) rd4((kseg[sg] - 1) * REC + O_BX, xs[sg]);
#pragma unroll
        for (int s = 0; s < RS; ++s) {
            const int sg = s / RSEG;
            double c[4];
            cf(s, c);
            s_[s] = rv[s] ? fmax(wv.w[s][lane] - dot4(c, xs[sg]), 1.0) : 1.0;
            z_[s] = rv[s] ? 1.0 : 0.0;
            ra[s] = 0.0;
            rb[s] = 0.0;
        }
        const double bnorm = 1.0 + row_max(bn);
        const double qnorm = 1.0 + row_max(qn);

        int status = CARMPC_MAX_ITER;
        int it = 0;
        bool polish_failed = false;
        while (__any(active)) {
            // ================= residuals (R1 + B1) =================
            double rd_[2][2], mu = 0.0, rpn = 0.0, gun = 0.0, umax = 0.0, wz = 0.0, wzabs = 0.0;
            double lo = 0.0, scf = 0.0;
            bool polish = false;
            if (active) {
                double lz[2][4], musum = 0.0;
#pragma unroll
                for (int sg = 0; sg < 2; ++sg)
#pragma unroll
                    for (int a = 0; a < 4; ++a) lz[sg][a] = 0.0;
#pragma unroll
                for (int s = 0; s < RS; ++s) {
                    const int sg = s / RSEG;
                    double c[4];
                    cf(s, c);
                    const double w = wv.w[s][lane];
                    const double gu = rv[s] ? dot4(c, xs[sg]) : 0.0;
                    const double rp = rv[s] ? gu + s_[s] - w : 0.0;
                    rpn = fmax(rpn, fabs(rp));
                    gun = fmax(gun, fabs(gu));
                    musum = fma(s_[s], z_[s], musum);
#pragma unroll
                    for (int a = 0; a < 4; ++a) lz[sg][a] = fma(z_[s], c[a], lz[sg][a]);
                    wz = fma(w, z_[s], wz);
                    wzabs = fma(fabs(w), z_[s], wzabs);
                }
#pragma unroll
                for (int sg = 0; sg < 2; ++sg)
#pragma unroll
                    for (int c = 0; c < 2; ++c) {
                        const int i = 2 * (kseg[sg] - 1) + c;
                        if (own[sg] && boxed) {
                            const double rpu = u_[sg][c] + su[sg][c] - sh.ub[i];
                            const double rpl = -u_[sg][c] + sl[sg][c] + sh.lb[i];
                            rpn = fmax(rpn, fmax(fabs(rpu), fabs(rpl)));
                            musum = fma(su[sg][c], zu[sg][c], fma(sl[sg][c], zl[sg][c], musum));
                            umax = fmax(umax, fabs(u_[sg][c]));
                        }
                    }
                // stage-N sum of lamZ, owners write lamZ_k [0..3], lamH_k = Qbar_k xs_k [4..7]
                double pn[4];
#pragma unroll
                for (int a = 0; a < 4; ++a) pn[a] = row_sum((isN[0] ? lz[0][a] : 0.0) + (isN[1] ? lz[1][a] : 0.0));
                wb();
#pragma unroll
                for (int sg = 0; sg < 2; ++sg)
                    if (own[sg]) {
                        double v[4], h[4] = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
                        for (int a = 0; a < 4; ++a) v[a] = isN[sg] ? pn[a] : lz[sg][a];
                        add_qbar(kseg[sg] == N, xs[sg], h, 1.0);
                        wr4((kseg[sg] - 1) * REC + 0, v);
                        wr4((kseg[sg] - 1) * REC + 4, h);
                    }
                mu = row_sum(musum) * inv_m;
                rpn = row_max(rpn);
                gun = row_max(gun);
                umax = row_max(umax);
                wz = row_sum(wz);
                wzabs = row_sum(wzabs);
                // B1: psiZ_k = lamZ_k + A'psiZ_{k+1}, psiH likewise; gz_t = B'psiZ_{t+1}
                wb();
                {
                    double pz[4] = {0.0, 0.0, 0.0, 0.0}, ph[4] = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
                    for (int t = N - 1; t >= 0; --t) {
                        const int r = t * REC;
                        double lzv[4], lhv[4];
                        rd4(r + 0, lzv);
                        rd4(r + 4, lhv);
                        double nz[4], nh[4];
#pragma unroll
                        for (int a = 0; a < 4; ++a) {
                            double az = lzv[a], ah = lhv[a];
#pragma unroll
                            for (int c = 0; c < 4; ++c) {
                                az = fma(MT.A[c * 4 + a], pz[c], az);
                                ah = fma(MT.A[c * 4 + a], ph[c], ah);
                            }
                            nz[a] = az;
                            nh[a] = ah;
                        }
                        double gz[2], hs[2];
#pragma unroll
                        for (int c = 0; c < 2; ++c) {
                            double az = 0.0, ah = 0.0;
#pragma unroll
                            for (int a = 0; a < 4; ++a) {
                                pz[a] = nz[a];
                                ph[a] = nh[a];
                                az = fma(MT.B[a * 2 + c], nz[a], az);
                                ah = fma(MT.B[a * 2 + c], nh[a], ah);
                            }
                            gz[c] = az;
                            hs[c] = ah;
                            const double lb = sh.lb[2 * t + c], ub = sh.ub[2 * t + c];
                            lo += fmin(az * lb, az * ub);
                            scf = fma(fabs(az), fmax(fabs(lb), fabs(ub)), scf);
                        }
                        wb();
                        if (j == 0) {
                            wr2(r + 12, gz[0], gz[1]);
                            wr2(r + 14, hs[0], hs[1]);
                        }
                    }
                }
                wb();
                double rdn = 0.0, hun = 0.0, gzn = 0.0;
#pragma unroll
                for (int sg = 0; sg < 2; ++sg) {
                    const int r = (kseg[sg] - 1) * REC;
                    double gz0, gz1, hs0, hs1;
                    rd2(r + 12, gz0, gz1);
                    rd2(r + 14, hs0, hs1);
                    const double gzv[2] = {gz0, gz1}, hsv[2] = {hs0, hs1};
#pragma unroll
                    for (int c = 0; c < 2; ++c) {
                        const double hu = hsv[c] + fma(MT.R[c * 2], u_[sg][0], MT.R[c * 2 + 1] * u_[sg][1]);
                        const double gzb = gzv[c] + (boxed ? zu[sg][c] - zl[sg][c] : 0.0);
                        const double rd = hu + q_[sg][c] + gzb;
                        rd_[sg][c] = own[sg] ? rd : 0.0;
                        if (own[sg]) {
                            rdn = fmax(rdn, fabs(rd));
                            hun = fmax(hun, fabs(hu));
                            gzn = fmax(gzn, fabs(gzb));
                        }
                    }
                }
                rdn = row_max(rdn);
                hun = row_max(hun);
                gzn = row_max(gzn);
                const double pscale = fmax(bnorm, 1.0 + fmax(gun, umax));
                const double dscale = fmax(qnorm, 1.0 + fmax(hun, gzn));
                int done = -1;
                if (!isfinite(mu) || !isfinite(rdn)) {
                    done = CARMPC_NUMERICAL;
                } else {
                    const bool res_ok = rpn <= S.tol * pscale && rdn <= S.tol * dscale;
                    const bool last = it >= S.max_iter;
                    polish = !polish_failed && ((res_ok && mu <= POLISH_MU) || last);
                    if (!polish) {
                        if (last) done = CARMPC_MAX_ITER;
                        else if (res_ok && mu <= S.tol_mu) done = CARMPC_OPTIMAL;
                        else if (p > 0 && lo - wz > 1e-12 * (scf + wzabs)) done = CARMPC_PRIMAL_INFEASIBLE;
                    }
                }
                if (done >= 0) {
                    status = done;
#pragma unroll
                    for (int sg = 0; sg < 2; ++sg)
                        if (own[sg]) {
                            const int t = kseg[sg] - 1;
                            u_out[inst * ld_u + 2 * t] = u_[sg][0];
                            u_out[inst * ld_u + 2 * t + 1] = u_[sg][1];
                        }
                    if (j == 0) {
                        status_out[inst] = status;
                        if (iters_out) iters_out[inst] = it;
                    }
                    active = false;
                    polish = false;
                }
            }
            const bool any_polish = __any(polish);
            if (!__any(active)) break;
            // ================= factorization rows (R2) + first right-hand side =================
            // normal: d = z/s, predictor rhs; polish: d = 1/delta on the active set (s < z)
            // per owned input: normal e1..e4 = dsu, dzu, dsl, dzl of the direction, vx = du;
            // polish vx = x, e1 = yu, e2 = yl.  xvv: normal S du (corrector), polish S x.
            double e1[2][2], e2[2][2], e3[2][2], e4[2][2], vx[2][2];
            double xvv[2][4];
            double pua[2][2], pla[2][2];
            double smu = 0.0;
            if (active) {
                double Wa[2][10], acc[2][4];
#pragma unroll
                for (int sg = 0; sg < 2; ++sg) {
#pragma unroll
                    for (int e = 0; e < 10; ++e) Wa[sg][e] = 0.0;
#pragma unroll
                    for (int a = 0; a < 4; ++a) acc[sg][a] = 0.0;
                }
#pragma unroll
                for (int s = 0; s < RS; ++s) {
                    const int sg = s / RSEG;
                    double c[4];
                    cf(s, c);
                    const double w = wv.w[s][lane];
                    double d, t;
                    if (polish) {
                        d = (rv[s] && s_[s] < z_[s]) ? idl : 0.0;
                        rb[s] = d != 0.0 ? w : 0.0;       // ryg of the first polish solve (x = 0)
                        ra[s] = 0.0;                       // yg
                        t = -(ra[s] - d * rb[s]);          // b^x = -(Qbar xv + sum (yg - d ryg) c)
                    } else {
                        d = rv[s] ? z_[s] * frcp(s_[s]) : 0.0;
                        const double rp = rv[s] ? dot4(c, xs[sg]) + s_[s] - w : 0.0;
                        t = rv[s] ? (s_[s] * z_[s] - z_[s] * rp) * frcp(s_[s]) : 0.0;
                    }
#pragma unroll
                    for (int a = 0; a < 4; ++a) {
                        const double da = d * c[a];
#pragma unroll
                        for (int b = a; b < 4; ++b) Wa[sg][sym10(a, b)] = fma(da, c[b], Wa[sg][sym10(a, b)]);
                        acc[sg][a] = fma(t, c[a], acc[sg][a]);
                    }
                }
                // stage-N totals of W
                double wn[10];
#pragma unroll
                for (int e = 0; e < 10; ++e) wn[e] = row_sum((isN[0] ? Wa[0][e] : 0.0) + (isN[1] ? Wa[1][e] : 0.0));
                double zero4[2][4] = {{0.0, 0.0, 0.0, 0.0}, {0.0, 0.0, 0.0, 0.0}};
                wb();
                write_bx(acc, zero4, 0.0);
#pragma unroll
                for (int sg = 0; sg < 2; ++sg) {
                    const int t = kseg[sg] - 1;
                    const int r = t * REC;
                    double db[2], bu[2];
#pragma unroll
                    for (int c = 0; c < 2; ++c) {
                        const int i = 2 * t + c;
                        const double lb = sh.lb[i], ub = sh.ub[i];
                        vx[sg][c] = 0.0;
                        e1[sg][c] = 0.0;
                        e2[sg][c] = 0.0;
                        e3[sg][c] = 0.0;
                        e4[sg][c] = 0.0;
                        pua[sg][c] = 0.0;
                        pla[sg][c] = 0.0;
                        if (polish) {
                            const double dbu = (boxed && su[sg][c] < zu[sg][c]) ? idl : 0.0;
                            const double dbl = (boxed && sl[sg][c] < zl[sg][c]) ? idl : 0.0;
                            db[c] = dbu + dbl;
                            bu[c] = -q_[sg][c] + dbu * ub + dbl * lb;
                        } else if (boxed) {
                            const double rpu = u_[sg][c] + su[sg][c] - ub;
                            const double rpl = -u_[sg][c] + sl[sg][c] + lb;
                            db[c] = zu[sg][c] * frcp(su[sg][c]) + zl[sg][c] * frcp(sl[sg][c]);
                            bu[c] = -rd_[sg][c] + (su[sg][c] * zu[sg][c] - zu[sg][c] * rpu) * frcp(su[sg][c]) -
                                    (sl[sg][c] * zl[sg][c] - zl[sg][c] * rpl) * frcp(sl[sg][c]);
                        } else {
                            db[c] = 0.0;
                            bu[c] = -rd_[sg][c];
                        }
                    }
#pragma unroll
                    for (int a = 0; a < 4; ++a) xvv[sg][a] = 0.0;
                    if (own[sg]) {
#pragma unroll
                        for (int e = 0; e < 5; ++e)
                            wr2(r + 2 * e, isN[sg] ? wn[2 * e] : Wa[sg][2 * e], isN[sg] ? wn[2 * e + 1] : Wa[sg][2 * e + 1]);
                        wr2(r + O_BU, bu[0], bu[1]);
                        wr2(r + O_DB, db[0], db[1]);
                    }
                }
                factor_and_back();
            }
            // ================= solves =================
            const int nsolve = any_polish ? POLISH_REFINE + 1 : 3;
#pragma unroll 1
            for (int k = 0; k < nsolve; ++k) {
                const bool run = active && (polish || k < 3);
                if (k > 0 && run) back_linear();
                if (run) forward();
                if (!run) continue;
                double dy[2][4], dv[2][2];
#pragma unroll
                for (int sg = 0; sg < 2; ++sg) {
                    rd4((kseg[sg] - 1) * REC + O_BX, dy[sg]);
                    rd2((kseg[sg] - 1) * REC + O_BU, dv[sg][0], dv[sg][1]);
                }
                wb();
                if (polish) {
                    // update: yg += d (G dx - ryg); yu += dbu (dx - ryu); yl += dbl (-dx - ryl); x += dx
#pragma unroll
                    for (int s = 0; s < RS; ++s) {
                        const int sg = s / RSEG;
                        double c[4];
                        cf(s, c);
                        const double d = (rv[s] && s_[s] < z_[s]) ? idl : 0.0;
                        ra[s] = fma(d, dot4(c, dy[sg]) - rb[s], ra[s]);
                    }
#pragma unroll
                    for (int sg = 0; sg < 2; ++sg) {
                        const int t = kseg[sg] - 1;
#pragma unroll
                        for (int c = 0; c < 2; ++c) {
                            const int i = 2 * t + c;
                            const double dbu = (boxed && su[sg][c] < zu[sg][c]) ? idl : 0.0;
                            const double dbl = (boxed && sl[sg][c] < zl[sg][c]) ? idl : 0.0;
                            const double ryu = dbu != 0.0 ? sh.ub[i] - vx[sg][c] : 0.0;
                            const double ryl = dbl != 0.0 ? -sh.lb[i] + vx[sg][c] : 0.0;
                            e1[sg][c] = fma(dbu, dv[sg][c] - ryu, e1[sg][c]);
                            e2[sg][c] = fma(dbl, -dv[sg][c] - ryl, e2[sg][c]);
                            vx[sg][c] = own[sg] ? vx[sg][c] + dv[sg][c] : 0.0;
                        }
#pragma unroll
                        for (int a = 0; a < 4; ++a) xvv[sg][a] += dy[sg][a];
                    }
                    if (k < POLISH_REFINE) {
                        // next right-hand side of the refinement
                        double acc[2][4];
#pragma unroll
                        for (int sg = 0; sg < 2; ++sg)
#pragma unroll
                            for (int a = 0; a < 4; ++a) acc[sg][a] = 0.0;
#pragma unroll
                        for (int s = 0; s < RS; ++s) {
                            const int sg = s / RSEG;
                            double c[4];
                            cf(s, c);
                            const double d = (rv[s] && s_[s] < z_[s]) ? idl : 0.0;
                            const double gx = dot4(c, xvv[sg]);
                            rb[s] = d != 0.0 ? wv.w[s][lane] - gx : 0.0;
                            const double t = -(ra[s] - d * rb[s]);
#pragma unroll
                            for (int a = 0; a < 4; ++a) acc[sg][a] = fma(t, c[a], acc[sg][a]);
                        }
                        wb();
                        write_bx(acc, xvv, -1.0);
#pragma unroll
                        for (int sg = 0; sg < 2; ++sg) {
                            const int t = kseg[sg] - 1;
                            double bu[2];
#pragma unroll
                            for (int c = 0; c < 2; ++c) {
                                const int i = 2 * t + c;
                                const double dbu = (boxed && su[sg][c] < zu[sg][c]) ? idl : 0.0;
                                const double dbl = (boxed && sl[sg][c] < zl[sg][c]) ? idl : 0.0;
                                const double ryu = dbu != 0.0 ? sh.ub[i] - vx[sg][c] : 0.0;
                                const double ryl = dbl != 0.0 ? -sh.lb[i] + vx[sg][c] : 0.0;
                                const double rx = fma(MT.R[c * 2], vx[sg][0], MT.R[c * 2 + 1] * vx[sg][1]);
                                bu[c] = -q_[sg][c] - rx - e1[sg][c] + e2[sg][c] + dbu * ryu - dbl * ryl;
                            }
                            if (own[sg]) wr2(t * REC + O_BU, bu[0], bu[1]);
                        }
                    } else {
                        // verification (oracle/qp.py::polish_step acceptance test)
                        double viol = -INFINITY, wsc = 0.0, ysc = 0.0, ymin = 0.0;
                        bool fin = true;
#pragma unroll
                        for (int sg = 0; sg < 2; ++sg)
#pragma unroll
                            for (int c = 0; c < 2; ++c) {
                                const int i = 2 * (kseg[sg] - 1) + c;
                                if (own[sg]) {
                                    if (boxed) {
                                        viol = fmax(viol, fmax(vx[sg][c] - sh.ub[i], sh.lb[i] - vx[sg][c]));
                                        wsc = fmax(wsc, fmax(fabs(sh.lb[i]), fabs(sh.ub[i])));
                                    }
                                    ysc = fmax(ysc, fmax(fabs(e1[sg][c]), fabs(e2[sg][c])));
                                    ymin = fmin(ymin, fmin(e1[sg][c], e2[sg][c]));
                                    fin = fin && isfinite(vx[sg][c]);
                                }
                            }
                        bool paired[RS];
#pragma unroll
                        for (int s = 0; s < RS; ++s) paired[s] = false;
                        if (P.r_partner) {
#pragma unroll
                            for (int s = 0; s < RS; ++s)
                                wv.scr[s][lane] = (rv[s] && s_[s] < z_[s]) ? ra[s] : NAN;
                            wb();
#pragma unroll
                            for (int s = 0; s < RS; ++s) {
                                const int pr = rv[s] ? sh.partner[s * G16 + j] : -1;
                                paired[s] = pr >= 0 && s_[s] < z_[s] &&
                                            !isnan(wv.scr[pr / G16][(lane & 48) + (pr % G16)]);
                            }
                            wb();
                        }
#pragma unroll
                        for (int s = 0; s < RS; ++s) {
                            const int sg = s / RSEG;
                            if (rv[s]) {
                                double c[4];
                                cf(s, c);
                                const double w = wv.w[s][lane];
                                viol = fmax(viol, dot4(c, xvv[sg]) - w);
                                wsc = fmax(wsc, fabs(w));
                                ysc = fmax(ysc, fabs(ra[s]));
                                ymin = paired[s] ? ymin : fmin(ymin, ra[s]);
                            }
                        }
                        viol = row_max(viol);
                        wsc = row_max(wsc);
                        ysc = row_max(ysc);
                        ymin = row_min(ymin);
                        const double finv = row_min(fin ? 1.0 : 0.0);
                        if (finv > 0.0 && viol <= POLISH_TOL * (1.0 + wsc) && ymin >= -POLISH_TOL * (1.0 + ysc)) {
                            status = CARMPC_OPTIMAL;
#pragma unroll
                            for (int sg = 0; sg < 2; ++sg)
                                if (own[sg]) {
                                    const int t = kseg[sg] - 1;
                                    u_out[inst * ld_u + 2 * t] = vx[sg][0];
                                    u_out[inst * ld_u + 2 * t + 1] = vx[sg][1];
                                }
                            if (j == 0) {
                                status_out[inst] = status;
                                if (iters_out) iters_out[inst] = it;
                            }
                            active = false;
                        }
                        polish_failed = true;
                    }
                    continue;
                }
                // ---------------- normal trip ----------------
                if (k == 0) {
                    // predictor direction: ratio test, sigma, corrector right-hand side
                    double amax = INFINITY, mua = 0.0;
#pragma unroll
                    for (int s = 0; s < RS; ++s) {
                        const int sg = s / RSEG;
                        double c[4];
                        cf(s, c);
                        const double w = wv.w[s][lane];
                        const double rp = rv[s] ? dot4(c, xs[sg]) + s_[s] - w : 0.0;
                        const double ds = rv[s] ? -rp - dot4(c, dy[sg]) : 0.0;
                        const double dz = rv[s] ? (-s_[s] * z_[s] - z_[s] * ds) * frcp(s_[s]) : 0.0;
                        ra[s] = ds;
                        rb[s] = dz;
                        amax = fmin(amax, fmin(ratio(s_[s], ds), ratio(z_[s], dz)));
                    }
#pragma unroll
                    for (int sg = 0; sg < 2; ++sg)
#pragma unroll
                        for (int c = 0; c < 2; ++c) {
                            const int i = 2 * (kseg[sg] - 1) + c;
                            if (own[sg] && boxed) {
                                const double rpu = u_[sg][c] + su[sg][c] - sh.ub[i];
                                const double rpl = -u_[sg][c] + sl[sg][c] + sh.lb[i];
                                const double dsu = -rpu - dv[sg][c], dsl = -rpl + dv[sg][c];
                                const double dzu = (-su[sg][c] * zu[sg][c] - zu[sg][c] * dsu) * frcp(su[sg][c]);
                                const double dzl = (-sl[sg][c] * zl[sg][c] - zl[sg][c] * dsl) * frcp(sl[sg][c]);
                                amax = fmin(amax, fmin(fmin(ratio(su[sg][c], dsu), ratio(zu[sg][c], dzu)),
                                                       fmin(ratio(sl[sg][c], dsl), ratio(zl[sg][c], dzl))));
                                pua[sg][c] = dsu * dzu;
                                pla[sg][c] = dsl * dzl;
                                e1[sg][c] = dsu;
                                e2[sg][c] = dzu;
                                e3[sg][c] = dsl;
                                e4[sg][c] = dzl;
                            }
                        }
                    const double a = fmin(1.0, row_min(amax));
#pragma unroll
                    for (int s = 0; s < RS; ++s) mua = fma(fma(a, ra[s], s_[s]), fma(a, rb[s], z_[s]), mua);
#pragma unroll
                    for (int sg = 0; sg < 2; ++sg)
#pragma unroll
                        for (int c = 0; c < 2; ++c)
                            if (own[sg] && boxed) {
                                mua = fma(fma(a, e1[sg][c], su[sg][c]), fma(a, e2[sg][c], zu[sg][c]), mua);
                                mua = fma(fma(a, e3[sg][c], sl[sg][c]), fma(a, e4[sg][c], zl[sg][c]), mua);
                            }
                    const double sg3 = row_sum(mua) * inv_m / mu;
                    smu = sg3 * sg3 * sg3 * mu;
                    double acc[2][4];
#pragma unroll
                    for (int sg = 0; sg < 2; ++sg)
#pragma unroll
                        for (int aa = 0; aa < 4; ++aa) acc[sg][aa] = 0.0;
#pragma unroll
                    for (int s = 0; s < RS; ++s) {
                        const int sg = s / RSEG;
                        double c[4];
                        cf(s, c);
                        const double pa = ra[s] * rb[s];
                        ra[s] = pa;   // keep the predictor products for the corrector
                        const double rp = rv[s] ? dot4(c, xs[sg]) + s_[s] - wv.w[s][lane] : 0.0;
                        const double rc = s_[s] * z_[s] + pa - smu;
                        const double t = rv[s] ? (rc - z_[s] * rp) * frcp(s_[s]) : 0.0;
#pragma unroll
                        for (int aa = 0; aa < 4; ++aa) acc[sg][aa] = fma(t, c[aa], acc[sg][aa]);
                    }
                    double zero4[2][4] = {{0.0, 0.0, 0.0, 0.0}, {0.0, 0.0, 0.0, 0.0}};
                    wb();
                    write_bx(acc, zero4, 0.0);
#pragma unroll
                    for (int sg = 0; sg < 2; ++sg) {
                        const int t = kseg[sg] - 1;
                        double bu[2];
#pragma unroll
                        for (int c = 0; c < 2; ++c) {
                            const int i = 2 * t + c;
                            if (boxed) {
                                const double rpu = u_[sg][c] + su[sg][c] - sh.ub[i];
                                const double rpl = -u_[sg][c] + sl[sg][c] + sh.lb[i];
                                const double rcu = su[sg][c] * zu[sg][c] + pua[sg][c] - smu;
                                const double rcl = sl[sg][c] * zl[sg][c] + pla[sg][c] - smu;
                                bu[c] = -rd_[sg][c] + (rcu - zu[sg][c] * rpu) * frcp(su[sg][c]) -
                                        (rcl - zl[sg][c] * rpl) * frcp(sl[sg][c]);
                            } else {
                                bu[c] = -rd_[sg][c];
                            }
                        }
                        if (own[sg]) wr2(t * REC + O_BU, bu[0], bu[1]);
                    }
                } else if (k == 1) {
                    // corrector direction; refinement right-hand side -(H du + G'dz + rd + box)
                    double acc[2][4];
#pragma unroll
                    for (int sg = 0; sg < 2; ++sg)
#pragma unroll
                        for (int aa = 0; aa < 4; ++aa) acc[sg][aa] = 0.0;
#pragma unroll
                    for (int s = 0; s < RS; ++s) {
                        const int sg = s / RSEG;
                        double c[4];
                        cf(s, c);
                        const double rp = rv[s] ? dot4(c, xs[sg]) + s_[s] - wv.w[s][lane] : 0.0;
                        const double rc = s_[s] * z_[s] + ra[s] - smu;
                        const double ds = rv[s] ? -rp - dot4(c, dy[sg]) : 0.0;
                        const double dz = rv[s] ? (-rc - z_[s] * ds) * frcp(s_[s]) : 0.0;
                        ra[s] = ds;
                        rb[s] = dz;
#pragma unroll
                        for (int aa = 0; aa < 4; ++aa) acc[sg][aa] = fma(-dz, c[aa], acc[sg][aa]);
                    }
                    wb();
                    write_bx(acc, dy, -1.0);
#pragma unroll
                    for (int sg = 0; sg < 2; ++sg) {
                        const int t = kseg[sg] - 1;
                        double bu[2];
#pragma unroll
                        for (int c = 0; c < 2; ++c) {
                            const int i = 2 * t + c;
                            double dzu = 0.0, dzl = 0.0;
                            if (own[sg] && boxed) {
                                const double rpu = u_[sg][c] + su[sg][c] - sh.ub[i];
                                const double rpl = -u_[sg][c] + sl[sg][c] + sh.lb[i];
                                const double rcu = su[sg][c] * zu[sg][c] + pua[sg][c] - smu;
                                const double rcl = sl[sg][c] * zl[sg][c] + pla[sg][c] - smu;
                                const double dsu = -rpu - dv[sg][c], dsl = -rpl + dv[sg][c];
                                dzu = (-rcu - zu[sg][c] * dsu) * frcp(su[sg][c]);
                                dzl = (-rcl - zl[sg][c] * dsl) * frcp(sl[sg][c]);
                                e1[sg][c] = dsu;
                                e2[sg][c] = dzu;
                                e3[sg][c] = dsl;
                                e4[sg][c] = dzl;
                            }
                            const double rdu = fma(MT.R[c * 2], dv[sg][0], MT.R[c * 2 + 1] * dv[sg][1]);
                            bu[c] = -(rdu + rd_[sg][c] + (dzu - dzl));
                        }
#pragma unroll
                        for (int c = 0; c < 2; ++c) vx[sg][c] = dv[sg][c];
#pragma unroll
                        for (int aa = 0; aa < 4; ++aa) xvv[sg][aa] = dy[sg][aa];
                        if (own[sg]) wr2(t * REC + O_BU, bu[0], bu[1]);
                    }
                } else if (k == 2) {
                    // apply the correction, step length, update
                    double amax = INFINITY;
#pragma unroll
                    for (int s = 0; s < RS; ++s) {
                        const int sg = s / RSEG;
                        double c[4];
                        cf(s, c);
                        const double cs = rv[s] ? -dot4(c, dy[sg]) : 0.0;
                        ra[s] += cs;
                        rb[s] = rv[s] ? rb[s] - z_[s] * cs * frcp(s_[s]) : 0.0;
                        amax = fmin(amax, fmin(ratio(s_[s], ra[s]), ratio(z_[s], rb[s])));
                    }
#pragma unroll
                    for (int sg = 0; sg < 2; ++sg)
#pragma unroll
                        for (int c = 0; c < 2; ++c) {
                            vx[sg][c] += dv[sg][c];
                            if (own[sg] && boxed) {
                                const double cu = dv[sg][c];
                                e1[sg][c] -= cu;
                                e2[sg][c] = fma(zu[sg][c] * cu, frcp(su[sg][c]), e2[sg][c]);
                                e3[sg][c] += cu;
                                e4[sg][c] = fma(-zl[sg][c] * cu, frcp(sl[sg][c]), e4[sg][c]);
                                amax = fmin(amax, fmin(fmin(ratio(su[sg][c], e1[sg][c]), ratio(zu[sg][c], e2[sg][c])),
                                                       fmin(ratio(sl[sg][c], e3[sg][c]), ratio(zl[sg][c], e4[sg][c]))));
                            }
                        }
                    const double a = fmin(1.0, STEP_FRAC * row_min(amax));
#pragma unroll
                    for (int s = 0; s < RS; ++s) {
                        s_[s] = fma(a, ra[s], s_[s]);
                        z_[s] = fma(a, rb[s], z_[s]);
                    }
#pragma unroll
                    for (int sg = 0; sg < 2; ++sg) {
#pragma unroll
                        for (int c = 0; c < 2; ++c) {
                            if (own[sg]) u_[sg][c] = fma(a, vx[sg][c], u_[sg][c]);
                            if (own[sg] && boxed) {
                                su[sg][c] = fma(a, e1[sg][c], su[sg][c]);
                                zu[sg][c] = fma(a, e2[sg][c], zu[sg][c]);
                                sl[sg][c] = fma(a, e3[sg][c], sl[sg][c]);
                                zl[sg][c] = fma(a, e4[sg][c], zl[sg][c]);
                            }
                        }
#pragma unroll
                        for (int aa = 0; aa < 4; ++aa) xs[sg][aa] = fma(a, xvv[sg][aa] + dy[sg][aa], xs[sg][aa]);
                    }
                    polish_failed = false;
                    ++it;
                }
            }
        }
    }
}

}  // namespace

bool riccati_supported_N(int N) { return N == 10 || N == 20; }

hipError_t launch_riccati(const DevProblem& P, int64_t batch, const double* x0, const double* xref, double* u_out,
                          int64_t ld_u, int32_t* status, int32_t* iters, const Settings& s, hipStream_t stream,
                          int* unsupported) {
    *unsupported = 0;
    if (batch <= 0) return hipSuccess;
    if (!P.ric) {
        *unsupported = 1;
        return hipErrorInvalidValue;
    }
    constexpr int WPB = 4;
    auto go = [&](auto kern) -> hipError_t {
        int dev = 0, cus = 0, per_cu = 0;
        hipError_t e = hipGetDevice(&dev);
        if (e != hipSuccess) return e;
        e = hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
        if (e != hipSuccess) return e;
        e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, (const void*)kern, WPB * 64, 0);
        if (e != hipSuccess) return e;
        if (per_cu < 1) per_cu = 1;
        const int64_t per_block = (int64_t)WPB * 4;
        int64_t want = (batch + per_block - 1) / per_block;
        int64_t grid = (int64_t)cus * per_cu;
        if (want < grid) grid = want;
        if (grid < 1) grid = 1;
        hipLaunchKernelGGL(kern, dim3((unsigned)grid), dim3(WPB * 64), 0, stream, P, batch, x0, xref, u_out, ld_u,
                           status, iters, s);
        return hipGetLastError();
    };
    switch (P.N) {
        case 10: return go(ipm_riccati_kernel<10, WPB>);
        case 20: return go(ipm_riccati_kernel<20, WPB>);
        default: *unsupported = 1; return hipErrorInvalidValue;
    }
}

}  // namespace carmpc
