// Batched small LPs for the terminal-set synthesis:
//   maximise c'x  s.t.  A x <= b,  x in R^4,
// one LP per wavefront.  lib/terminal_set.py:45-67 solves one cvxpy LP per state row and
// horizon; polytope.reduce solves one per candidate half-space.  Here every LP of one
// synthesis round (all rows, all goals) is one launch.
//
// Method: Mehrotra predictor-corrector on the inequality form (slacks s, duals z), rows
// strided over the 64 lanes (RPL rows per lane in registers), the 4x4 normal matrix
// A' diag(z/s) A reduced across the wave and factorised redundantly in every lane.
// Unboundedness: 8 box rows |x_j| <= kBig are appended; a solution on the box is reported as
// unbounded (value +inf), which is what the reference's solver returns for those LPs.
#include "carmpc_internal.h"
#include "lanes.h"

namespace carmpc {

namespace {

constexpr double kBig = 1e6;
constexpr int kLpWPB = 4;

__device__ __forceinline__ double wave_sum(double v) {
    v = lanes::row_sum(v);
    v += __shfl_xor(v, 16);
    return v + __shfl_xor(v, 32);
}
__device__ __forceinline__ double wave_max(double v) {
    v = lanes::row_max(v);
    v = fmax(v, __shfl_xor(v, 16));
    return fmax(v, __shfl_xor(v, 32));
}
__device__ __forceinline__ double wave_min(double v) {
    v = lanes::row_min(v);
    v = fmin(v, __shfl_xor(v, 16));
    return fmin(v, __shfl_xor(v, 32));
}

// solve (L L') y = r for the packed symmetric 4x4 M (10 entries), in place on r.  Near a
// degenerate vertex z/s spans many decades and a pivot can cancel to ~0: such a pivot is
// replaced by a huge value, which zeroes that component of the direction (pivot
// replacement; a diagonal shift instead would stall the dual residual).
__device__ __forceinline__ bool chol4_solve(const double* M, double* r) {
    const double dmax = fmax(fmax(M[lanes::sym10(0, 0)], M[lanes::sym10(1, 1)]),
                             fmax(M[lanes::sym10(2, 2)], M[lanes::sym10(3, 3)]));
    if (!(dmax > 0.0) || !(dmax < INFINITY)) return false;
    double L[4][4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j <= i; ++j) {
            double v = M[lanes::sym10(j, i)];
#pragma unroll
            for (int k = 0; k < j; ++k) v -= L[i][k] * L[j][k];
            if (i == j) {
                L[i][i] = v > 1e-14 * dmax ? sqrt(v) : 1e64;
            } else {
                L[i][j] = v / L[j][j];
            }
        }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        double v = r[i];
#pragma unroll
        for (int k = 0; k < i; ++k) v -= L[i][k] * r[k];
        r[i] = v / L[i][i];
    }
#pragma unroll
    for (int i = 3; i >= 0; --i) {
        double v = r[i];
#pragma unroll
        for (int k = i + 1; k < 4; ++k) v -= L[k][i] * r[k];
        r[i] = v / L[i][i];
    }
    return true;
}

template <int RPL>
__global__ void __launch_bounds__(kLpWPB * 64) lp_kernel(LpArgs a) {
    const int lane = threadIdx.x & 63;
    const int64_t l = (int64_t)blockIdx.x * kLpWPB + (threadIdx.x >> 6);
    if (l >= a.nlp) return;
    const int m0 = a.m[l];
    const int m = m0 + 8;   // + box rows
    const double* A = a.a_pool + a.a_off[l];
    const double* bp = a.b_pool + a.b_off[l];
    const int relax = a.relax ? a.relax[l] : -1;
    double f[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) f[j] = -a.c[l * 4 + j];   // minimise f'x
    // row data in registers
    double ar[RPL][4], br[RPL], s[RPL], z[RPL];
    bool on[RPL];
#pragma unroll
    for (int q = 0; q < RPL; ++q) {
        const int r = lane + 64 * q;
        on[q] = r < m;
        if (r < m0) {
#pragma unroll
            for (int j = 0; j < 4; ++j) ar[q][j] = A[(int64_t)r * 4 + j];
            br[q] = bp[r] + (r == relax ? a.relax_amount : 0.0);
        } else if (r < m) {
            const int j = (r - m0) >> 1;
#pragma unroll
            for (int k = 0; k < 4; ++k) ar[q][k] = k == j ? (((r - m0) & 1) ? -1.0 : 1.0) : 0.0;
            br[q] = kBig;
        } else {
#pragma unroll
            for (int k = 0; k < 4; ++k) ar[q][k] = 0.0;
            br[q] = 0.0;
        }
        s[q] = on[q] ? fmax(br[q], 1.0) : 1.0;
        z[q] = on[q] ? 1.0 : 0.0;
    }
    double fmax_ = 0.0;
#pragma unroll
    for (int j = 0; j < 4; ++j) fmax_ = fmax(fmax_, fabs(f[j]));
    double x[4] = {0.0, 0.0, 0.0, 0.0};
    int status = 2;
    int it = 0;
    for (; it < a.max_iter; ++it) {
        // residuals: rp = A x + s - b, rd = f + A'z, mu = s'z / m
        double rp[RPL], rdl[4] = {0.0, 0.0, 0.0, 0.0}, sz = 0.0, rpm = 0.0;
#pragma unroll
        for (int q = 0; q < RPL; ++q) {
            double ax = 0.0;
#pragma unroll
            for (int j = 0; j < 4; ++j) ax += ar[q][j] * x[j];
            rp[q] = on[q] ? ax + s[q] - br[q] : 0.0;
            rpm = fmax(rpm, fabs(rp[q]) / (1.0 + fabs(br[q])));   // row-relative (box rows have b = kBig)
#pragma unroll
            for (int j = 0; j < 4; ++j) rdl[j] += ar[q][j] * z[q];
            sz += s[q] * z[q];
        }
        double rd[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) rd[j] = f[j] + wave_sum(rdl[j]);
        const double mu = wave_sum(sz) / m;
        rpm = wave_max(rpm);
        double rdm = 0.0, pobj = 0.0;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            rdm = fmax(rdm, fabs(rd[j]));
            pobj += f[j] * x[j];
        }
        if (rpm <= a.tol && rdm <= a.tol * (1.0 + fmax_) && mu * m <= a.tol_gap * (1.0 + fabs(pobj))) {
            status = 0;
            break;
        }
        // normal matrix and its two right-hand sides
        double Ml[10];
#pragma unroll
        for (int e = 0; e < 10; ++e) Ml[e] = 0.0;
        double w[RPL];
#pragma unroll
        for (int q = 0; q < RPL; ++q) {
            w[q] = on[q] ? z[q] / s[q] : 0.0;
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int j = i; j < 4; ++j) Ml[lanes::sym10(i, j)] += w[q] * ar[q][i] * ar[q][j];
        }
        double M[10];
#pragma unroll
        for (int e = 0; e < 10; ++e) M[e] = wave_sum(Ml[e]);
        // predictor: rc = s z
        auto direction = [&](const double* rc, double* dx, double* ds, double* dz) -> bool {
            double gl[4] = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
            for (int q = 0; q < RPL; ++q) {
                const double t = on[q] ? (rc[q] - z[q] * rp[q]) / s[q] : 0.0;
#pragma unroll
                for (int j = 0; j < 4; ++j) gl[j] += ar[q][j] * t;
            }
#pragma unroll
            for (int j = 0; j < 4; ++j) dx[j] = -rd[j] + wave_sum(gl[j]);
            if (!chol4_solve(M, dx)) return false;
#pragma unroll
            for (int q = 0; q < RPL; ++q) {
                double adx = 0.0;
#pragma unroll
                for (int j = 0; j < 4; ++j) adx += ar[q][j] * dx[j];
                ds[q] = on[q] ? -rp[q] - adx : 0.0;
                dz[q] = on[q] ? (-rc[q] - z[q] * ds[q]) / s[q] : 0.0;
            }
            return true;
        };
        double rc[RPL], dx[4], ds[RPL], dz[RPL];
#pragma unroll
        for (int q = 0; q < RPL; ++q) rc[q] = s[q] * z[q];
        if (!direction(rc, dx, ds, dz)) {
            status = (rpm <= 1e2 * a.tol && mu * m <= 1e2 * a.tol_gap * (1.0 + fabs(pobj))) ? 0 : 4;
            break;
        }
        double ap = 1.0, ad = 1.0;
#pragma unroll
        for (int q = 0; q < RPL; ++q)
            if (on[q]) {
                ap = fmin(ap, lanes::ratio(s[q], ds[q]));
                ad = fmin(ad, lanes::ratio(z[q], dz[q]));
            }
        ap = wave_min(ap);
        ad = wave_min(ad);
        double szl = 0.0;
#pragma unroll
        for (int q = 0; q < RPL; ++q) szl += on[q] ? (s[q] + ap * ds[q]) * (z[q] + ad * dz[q]) : 0.0;
        const double mu_aff = wave_sum(szl) / m;
        const double sig = mu > 0.0 ? (mu_aff / mu) * (mu_aff / mu) * (mu_aff / mu) : 0.0;
        // corrector
#pragma unroll
        for (int q = 0; q < RPL; ++q) rc[q] = on[q] ? s[q] * z[q] + ds[q] * dz[q] - sig * mu : 0.0;
        if (!direction(rc, dx, ds, dz)) {
            status = (rpm <= 1e2 * a.tol && mu * m <= 1e2 * a.tol_gap * (1.0 + fabs(pobj))) ? 0 : 4;
            break;
        }
        ap = 1.0 / 0.99;
        ad = 1.0 / 0.99;
#pragma unroll
        for (int q = 0; q < RPL; ++q)
            if (on[q]) {
                ap = fmin(ap, lanes::ratio(s[q], ds[q]));
                ad = fmin(ad, lanes::ratio(z[q], dz[q]));
            }
        ap = fmin(1.0, 0.99 * wave_min(ap));
        ad = fmin(1.0, 0.99 * wave_min(ad));
#pragma unroll
        for (int j = 0; j < 4; ++j) x[j] += ap * dx[j];
#pragma unroll
        for (int q = 0; q < RPL; ++q) {
            s[q] += ap * ds[q];
            z[q] += ad * dz[q];
        }
    }
    // on the box -> unbounded
    double boxmin = INFINITY;
#pragma unroll
    for (int q = 0; q < RPL; ++q) {
        const int r = lane + 64 * q;
        if (r >= m0 && r < m) boxmin = fmin(boxmin, s[q]);
    }
    boxmin = wave_min(boxmin);
    double val = 0.0;
#pragma unroll
    for (int j = 0; j < 4; ++j) val -= f[j] * x[j];
    int out_status = status == 0 ? CARMPC_LP_OPTIMAL : (status == 4 ? CARMPC_LP_NUMERICAL : CARMPC_LP_MAX_ITER);
    if (status == 0 && boxmin < 1e-3 * kBig) {
        out_status = CARMPC_LP_UNBOUNDED;
        val = INFINITY;
    }
    if (lane == 0) {
        a.value[l] = val;
        a.status[l] = out_status;
        if (a.iters) a.iters[l] = it;
    }
    if (a.x)
#pragma unroll
        for (int j = 0; j < 4; ++j)
            if (lane == j) a.x[l * 4 + j] = x[j];
}

}  // namespace

hipError_t launch_lp(const LpArgs& a, int max_m, hipStream_t s) {
    if (a.nlp <= 0) return hipSuccess;
    const int rows = max_m + 8;
    const dim3 grid((unsigned)((a.nlp + kLpWPB - 1) / kLpWPB)), block(kLpWPB * 64);
    if (rows <= 64) hipLaunchKernelGGL(lp_kernel<1>, grid, block, 0, s, a);
    else if (rows <= 128) hipLaunchKernelGGL(lp_kernel<2>, grid, block, 0, s, a);
    else if (rows <= 256) hipLaunchKernelGGL(lp_kernel<4>, grid, block, 0, s, a);
    else if (rows <= 512) hipLaunchKernelGGL(lp_kernel<8>, grid, block, 0, s, a);
    else if (rows <= 1024) hipLaunchKernelGGL(lp_kernel<16>, grid, block, 0, s, a);
    else return hipErrorInvalidValue;
    return hipGetLastError();
}

}  // namespace carmpc
