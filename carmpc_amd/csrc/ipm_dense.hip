// ipm_dense.hip -- dense condensed-QP Mehrotra IPM, one wavefront per QP (gfx950).
//
// Replaces the per-step cvxpy solve of lib/mpc.py:334-335 (MPCStateFB.step) and
// lib/mpc.py:477-478 (MPCOutputFB.step).  Algorithm: DESIGN.md §3 (restated on
// the CPU in oracle/qp.py::ipm and oracle/ipm.c).
//
// Layout:
//   * one workgroup = WPB wavefronts sharing one problem (environment);
//     G (p x ldg, unit rows, ldg = NV+2 doubles) and H (NV x NV) live in LDS;
//   * lane i < NV owns decision variable i: u_i, box slacks/duals, and column i
//     of M = H + G' diag(z/s) G in NV registers ("slot j" = M[j][i]);
//   * general row r lives in lane r%64, register slot r/64 (RS slots);
//   * cross-lane traffic: per-wave LDS broadcast buffers (bvec: an n-vector,
//     rvec: a p-vector) and v_readlane for the triangular-solve scalars.
// After the Cholesky, lane i's slot j holds L[i][j] (j<i), l_ii (j==i) and
// l_ii*L[j][i] (j>i), so both triangular solves run without data movement.
#include "carmpc_internal.h"

#include <hip/hip_runtime.h>
#include <math.h>

namespace carmpc {

namespace {

__device__ __forceinline__ double readlane_d(double v, int l) {
    const unsigned long long b = __builtin_bit_cast(unsigned long long, v);
    const unsigned lo = __builtin_amdgcn_readlane((unsigned)(b & 0xffffffffull), l);
    const unsigned hi = __builtin_amdgcn_readlane((unsigned)(b >> 32), l);
    return __builtin_bit_cast(double, ((unsigned long long)hi << 32) | lo);
}

__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}
__device__ __forceinline__ double wave_max(double v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = fmax(v, __shfl_xor(v, o, 64));
    return v;
}
__device__ __forceinline__ double wave_min(double v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = fmin(v, __shfl_xor(v, o, 64));
    return v;
}

// Step-to-boundary ratio -v/dv for dv < 0, +inf otherwise (masked lanes pass dv = 0).
// Branch-free with the hardware reciprocal: the result only feeds the
// fraction-to-boundary rule (x 0.99), so a few ulps do not matter.
__device__ __forceinline__ double ratio(double v, double dv) {
    const double r = -v * __builtin_amdgcn_rcp(dv);
    return dv < 0.0 ? r : INFINITY;
}

template <int RS>
__device__ __forceinline__ double dot_rows_lds(const double* Gs, int ldg, int row, const double* vec, int nv) {
    (void)RS;
    double acc = 0.0;
    const double2* g2 = reinterpret_cast<const double2*>(Gs + (size_t)row * ldg);
    const double2* v2 = reinterpret_cast<const double2*>(vec);
    for (int j = 0; j < nv / 2; ++j) {
        const double2 a = g2[j], b = v2[j];
        acc = fma(a.x, b.x, acc);
        acc = fma(a.y, b.y, acc);
    }
    return acc;
}

}  // namespace

template <int NV, int RS>
__global__ void __launch_bounds__(512) ipm_dense_kernel(DevProblem P, int64_t batch,
                                                        const double* __restrict__ x0,
                                                        const double* __restrict__ xref,
                                                        double* __restrict__ u_out, int64_t ld_u,
                                                        int32_t* __restrict__ status_out,
                                                        int32_t* __restrict__ iters_out, Settings S) {
    static_assert(NV % 2 == 0 && NV <= 64, "NV must be even and <= 64");
    extern __shared__ __attribute__((aligned(16))) double smem[];
    const int lane = threadIdx.x & 63;
    const int wave = threadIdx.x >> 6;
    const int wpb = blockDim.x >> 6;
    const int p = P.p;
    const int ldg = P.ldg;
    const int gsz = (p * ldg + 1) & ~1;
    double* Gs = smem;
    double* Hs = Gs + gsz;
    double* bvec = Hs + NV * NV + wave * (64 + 64 * RS);
    double* rvec = bvec + 64;

    for (int i = threadIdx.x; i < p * ldg; i += blockDim.x) Gs[i] = P.G[i];
    for (int i = threadIdx.x; i < NV * NV; i += blockDim.x) Hs[i] = P.H[i];
    __syncthreads();

    const bool act = lane < NV;
    const int li = act ? lane : 0;
    const bool boxact = act && P.boxed;
    const double lb = boxact ? P.lb[li] : -UNBOXED_BOUND;
    const double ub = boxact ? P.ub[li] : UNBOXED_BOUND;
    const double bndabs = fmax(fabs(lb), fabs(ub));
    bool rv[RS];
#pragma unroll
    for (int s = 0; s < RS; ++s) rv[s] = (s * 64 + lane) < p;
    const int m_rows = p + (P.boxed ? 2 * NV : 0);
    const double inv_m = 1.0 / (double)(m_rows > 0 ? m_rows : 1);

    for (int64_t inst = (int64_t)blockIdx.x * wpb + wave; inst < batch; inst += (int64_t)gridDim.x * wpb) {
        double xv[NX], xr[NX];
#pragma unroll
        for (int k = 0; k < NX; ++k) {
            xv[k] = x0[inst * NX + k];
            xr[k] = xref ? xref[inst * NX + k] : P.goal[k];
        }
        // ---- x0-only rows (G_r == 0): pure preconditions on x0 -------------
        bool bad = false;
        for (int r = lane; r < P.npre; r += 64) {
            double v = P.pre_w0[r];
#pragma unroll
            for (int k = 0; k < NX; ++k) v -= P.pre_E[r * NX + k] * xv[k];
            bad |= v < -PRE_TOL;
        }
        if (__any(bad)) {
            if (lane < P.n) u_out[inst * ld_u + lane] = 0.0;
            if (lane == 0) {
                status_out[inst] = CARMPC_PRIMAL_INFEASIBLE;
                if (iters_out) iters_out[inst] = 0;
            }
            continue;
        }
        // ---- per-instance data: q = hq (x0 - xref), w = w0 - E x0 ----------
        double q = 0.0;
        if (act) {
#pragma unroll
            for (int k = 0; k < NX; ++k) q += P.hq[li * NX + k] * (xv[k] - xr[k]);
        }
        double w[RS];
#pragma unroll
        for (int s = 0; s < RS; ++s) {
            const int r = s * 64 + lane;
            double v = 0.0;
            if (rv[s]) {
                v = P.w0[r];
#pragma unroll
                for (int k = 0; k < NX; ++k) v -= P.E[r * NX + k] * xv[k];
            }
            w[s] = v;
        }
        // ---- initial point --------------------------------------------------
        double u = boxact ? fmin(fmax(0.0, lb), ub) : 0.0;
        double su = boxact ? fmax(ub - u, 1.0) : 1.0;
        double sl = boxact ? fmax(u - lb, 1.0) : 1.0;
        double zu = boxact ? 1.0 : 0.0, zl = zu;
        bvec[lane] = act ? u : 0.0;
        __builtin_amdgcn_wave_barrier();
        double s_[RS], z_[RS];
#pragma unroll
        for (int s = 0; s < RS; ++s) {
            const int r = rv[s] ? s * 64 + lane : 0;
            const double gu = dot_rows_lds<RS>(Gs, ldg, r, bvec, NV);
            s_[s] = rv[s] ? fmax(w[s] - gu, 1.0) : 1.0;
            z_[s] = rv[s] ? 1.0 : 0.0;
        }
        double bn = boxact ? bndabs : 0.0;
#pragma unroll
        for (int s = 0; s < RS; ++s) bn = fmax(bn, rv[s] ? fabs(w[s]) : 0.0);
        const double bnorm = 1.0 + wave_max(bn);
        const double qnorm = 1.0 + wave_max(act ? fabs(q) : 0.0);

        int status = CARMPC_MAX_ITER;
        int it = 0;
        for (; it < S.max_iter; ++it) {
            // ---- residuals ----------------------------------------------------
            __builtin_amdgcn_wave_barrier();
            bvec[lane] = act ? u : 0.0;
#pragma unroll
            for (int s = 0; s < RS; ++s) rvec[s * 64 + lane] = z_[s];
            __builtin_amdgcn_wave_barrier();
            double rp[RS];
            double rpn = 0.0, musum = 0.0, wz = 0.0, wzabs = 0.0;
#pragma unroll
            for (int s = 0; s < RS; ++s) {
                const int r = rv[s] ? s * 64 + lane : 0;
                const double gu = dot_rows_lds<RS>(Gs, ldg, r, bvec, NV);
                rp[s] = rv[s] ? gu + s_[s] - w[s] : 0.0;
                rpn = fmax(rpn, fabs(rp[s]));
                musum += s_[s] * z_[s];
                wz += w[s] * z_[s];
                wzabs += fabs(w[s]) * z_[s];
            }
            const double rpu = boxact ? u + su - ub : 0.0;
            const double rpl = boxact ? -u + sl + lb : 0.0;
            rpn = fmax(rpn, fmax(fabs(rpu), fabs(rpl)));
            musum += boxact ? su * zu + sl * zl : 0.0;
            double gtz = 0.0, hu = 0.0;
            for (int r = 0; r < p; ++r) gtz = fma(Gs[r * ldg + li], rvec[r], gtz);
#pragma unroll
            for (int j = 0; j < NV; ++j) hu = fma(Hs[j * NV + li], bvec[j], hu);
            const double rd = act ? hu + q + gtz + (boxact ? zu - zl : 0.0) : 0.0;
            const double mu = wave_sum(musum) * inv_m;
            const double rpn_w = wave_max(rpn);
            const double rdn_w = wave_max(fabs(rd));
            if (!isfinite(mu) || !isfinite(rdn_w)) { status = CARMPC_NUMERICAL; break; }
            if (rpn_w <= S.tol * bnorm && rdn_w <= S.tol * qnorm && mu <= S.tol_mu) { status = CARMPC_OPTIMAL; break; }
            // ---- Farkas certificate: min_box (G'z)'u > w'z  =>  infeasible ----
            if (p > 0) {
                const double lo = act ? fmin(gtz * lb, gtz * ub) : 0.0;
                const double sc = act ? fabs(gtz) * bndabs : 0.0;
                const double lo_w = wave_sum(lo);
                const double wz_w = wave_sum(wz);
                const double sc_w = wave_sum(sc + wzabs);
                if (lo_w - wz_w > 1e-12 * sc_w) { status = CARMPC_PRIMAL_INFEASIBLE; break; }
            }
            // ---- M = H + G' diag(z/s) G + diag(box) : column `lane` ------------
            __builtin_amdgcn_wave_barrier();
#pragma unroll
            for (int s = 0; s < RS; ++s) rvec[s * 64 + lane] = rv[s] ? z_[s] / s_[s] : 0.0;
            __builtin_amdgcn_wave_barrier();
            double M[NV];
#pragma unroll
            for (int j = 0; j < NV; ++j) M[j] = Hs[j * NV + li];
            for (int r = 0; r < p; ++r) {
                const double2* g2 = reinterpret_cast<const double2*>(Gs + (size_t)r * ldg);
                const double t = rvec[r] * Gs[r * ldg + li];
#pragma unroll
                for (int j = 0; j < NV / 2; ++j) {
                    const double2 g = g2[j];
                    M[2 * j] = fma(g.x, t, M[2 * j]);
                    M[2 * j + 1] = fma(g.y, t, M[2 * j + 1]);
                }
            }
            const double dbox = boxact ? zu / su + zl / sl : 0.0;
#pragma unroll
            for (int j = 0; j < NV; ++j) M[j] += (j == lane) ? dbox : 0.0;
            // ---- guarded right-looking Cholesky, in registers -------------------
            double inv_ii = 1.0;
#pragma unroll
            for (int k = 0; k < NV; ++k) {
                double piv = readlane_d(M[k], k);
                if (!(piv > 0.0)) piv = 1e128;
                const double lkk = sqrt(piv);
                const double inv = 1.0 / lkk;
                const double l = (lane > k && act) ? M[k] * inv : 0.0;
                M[k] = (lane == k) ? lkk : ((lane > k) ? l : M[k]);
                inv_ii = (lane == k) ? inv : inv_ii;
                __builtin_amdgcn_wave_barrier();
                bvec[lane] = l;
                __builtin_amdgcn_wave_barrier();
#pragma unroll
                for (int j = k + 1; j < NV; ++j) M[j] = fma(-bvec[j], l, M[j]);
            }
            // ---- predictor / corrector solves ----------------------------------
            double du = 0.0, ds[RS], dz[RS], dsu = 0.0, dzu = 0.0, dsl = 0.0, dzl = 0.0;
            double dsa[RS], dza[RS], dsua = 0.0, dzua = 0.0, dsla = 0.0, dzla = 0.0;
            double sigma_mu = 0.0;
#pragma unroll
            for (int pass = 0; pass < 2; ++pass) {
                double rc[RS];
#pragma unroll
                for (int s = 0; s < RS; ++s)
                    rc[s] = pass == 0 ? s_[s] * z_[s] : s_[s] * z_[s] + dsa[s] * dza[s] - (rv[s] ? sigma_mu : 0.0);
                const double rcu = !boxact ? 0.0 : (pass == 0 ? su * zu : su * zu + dsua * dzua - sigma_mu);
                const double rcl = !boxact ? 0.0 : (pass == 0 ? sl * zl : sl * zl + dsla * dzla - sigma_mu);
                __builtin_amdgcn_wave_barrier();
#pragma unroll
                for (int s = 0; s < RS; ++s) rvec[s * 64 + lane] = rv[s] ? (rc[s] - z_[s] * rp[s]) / s_[s] : 0.0;
                __builtin_amdgcn_wave_barrier();
                double gtt = 0.0;
                for (int r = 0; r < p; ++r) gtt = fma(Gs[r * ldg + li], rvec[r], gtt);
                double b = act ? -rd + gtt + (boxact ? (rcu - zu * rpu) / su - (rcl - zl * rpl) / sl : 0.0) : 0.0;
                // forward: L y = b  (lane i: slot j<i holds L[i][j])
#pragma unroll
                for (int k = 0; k < NV; ++k) {
                    const double yk = readlane_d(b * inv_ii, k);
                    b = (lane == k) ? yk : ((lane > k) ? fma(-M[k], yk, b) : b);
                }
                // backward: L' x = y  (lane i: slot j>i holds l_ii L[j][i])
                double acc = 0.0;
#pragma unroll
                for (int k = NV - 1; k >= 0; --k) {
                    const double xk = readlane_d((b - inv_ii * acc) * inv_ii, k);
                    b = (lane == k) ? xk : b;
                    acc = (lane < k) ? fma(M[k], xk, acc) : acc;
                }
                const double dU = act ? b : 0.0;
                __builtin_amdgcn_wave_barrier();
                bvec[lane] = dU;
                __builtin_amdgcn_wave_barrier();
                double amax = INFINITY;
                double dS[RS], dZ[RS];
#pragma unroll
                for (int s = 0; s < RS; ++s) {
                    const int r = rv[s] ? s * 64 + lane : 0;
                    const double gd = dot_rows_lds<RS>(Gs, ldg, r, bvec, NV);
                    dS[s] = rv[s] ? -rp[s] - gd : 0.0;
                    dZ[s] = rv[s] ? (-rc[s] - z_[s] * dS[s]) / s_[s] : 0.0;
                    amax = fmin(amax, fmin(ratio(s_[s], dS[s]), ratio(z_[s], dZ[s])));
                }
                const double dSu = boxact ? -rpu - dU : 0.0;
                const double dSl = boxact ? -rpl + dU : 0.0;
                const double dZu = boxact ? (-rcu - zu * dSu) / su : 0.0;
                const double dZl = boxact ? (-rcl - zl * dSl) / sl : 0.0;
                amax = fmin(amax, fmin(fmin(ratio(su, dSu), ratio(zu, dZu)), fmin(ratio(sl, dSl), ratio(zl, dZl))));
                amax = wave_min(amax);
                if (pass == 0) {
                    const double a = fmin(1.0, amax);
                    double mua = 0.0;
#pragma unroll
                    for (int s = 0; s < RS; ++s) {
                        mua += (s_[s] + a * dS[s]) * (z_[s] + a * dZ[s]);
                        dsa[s] = dS[s];
                        dza[s] = dZ[s];
                    }
                    mua += boxact ? (su + a * dSu) * (zu + a * dZu) + (sl + a * dSl) * (zl + a * dZl) : 0.0;
                    const double sg = wave_sum(mua) * inv_m / mu;
                    sigma_mu = sg * sg * sg * mu;
                    dsua = dSu; dzua = dZu; dsla = dSl; dzla = dZl;
                } else {
                    du = dU;
#pragma unroll
                    for (int s = 0; s < RS; ++s) { ds[s] = dS[s]; dz[s] = dZ[s]; }
                    dsu = dSu; dzu = dZu; dsl = dSl; dzl = dZl;
                    const double a = fmin(1.0, STEP_FRAC * amax);
                    u += a * du;
#pragma unroll
                    for (int s = 0; s < RS; ++s) { s_[s] += a * ds[s]; z_[s] += a * dz[s]; }
                    su += a * dsu; zu += a * dzu; sl += a * dsl; zl += a * dzl;
                }
            }
        }
        if (lane < P.n) u_out[inst * ld_u + lane] = u;
        if (lane == 0) {
            status_out[inst] = status;
            if (iters_out) iters_out[inst] = it;
        }
    }
}

// ---------------------------------------------------------------------------
// Host-side dispatch
// ---------------------------------------------------------------------------
namespace {
#ifndef CARMPC_NVS
#define CARMPC_NVS 8, 16, 20, 24, 32, 40, 48, 64
#endif
constexpr int kNVs[] = {CARMPC_NVS};
constexpr int kMaxRS = 4;
constexpr int kWPB = 8;

size_t dense_lds(int nv, int p, int rs, int wpb) {
    const int ldg = nv + 2;
    const size_t gsz = (size_t)((p * ldg + 1) & ~1);
    return (gsz + (size_t)nv * nv + (size_t)wpb * (64 + 64 * rs)) * sizeof(double);
}

template <int NV, int RS>
hipError_t launch_t(const DevProblem& P, int64_t batch, const double* x0, const double* xref, double* u_out,
                    int64_t ld_u, int32_t* status, int32_t* iters, const Settings& s, hipStream_t stream) {
    const size_t lds = dense_lds(NV, P.p, RS, kWPB);
    auto kern = ipm_dense_kernel<NV, RS>;
    static bool attr_set = false;
    if (!attr_set) {
        hipError_t e = hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
        if (e != hipSuccess) return e;
        attr_set = true;
    }
    int dev = 0, cus = 0, per_cu = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e != hipSuccess) return e;
    e = hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    if (e != hipSuccess) return e;
    e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, (const void*)kern, kWPB * 64, lds);
    if (e != hipSuccess) return e;
    if (per_cu < 1) per_cu = 1;
    int64_t want = (batch + kWPB - 1) / kWPB;
    int64_t grid = (int64_t)cus * per_cu;
    if (want < grid) grid = want;
    if (grid < 1) grid = 1;
    hipLaunchKernelGGL(kern, dim3((unsigned)grid), dim3(kWPB * 64), lds, stream, P, batch, x0, xref, u_out, ld_u,
                       status, iters, s);
    return hipGetLastError();
}

template <int NV>
hipError_t launch_rs(int rs, const DevProblem& P, int64_t batch, const double* x0, const double* xref,
                     double* u_out, int64_t ld_u, int32_t* status, int32_t* iters, const Settings& s,
                     hipStream_t stream) {
    switch (rs) {
        case 1: return launch_t<NV, 1>(P, batch, x0, xref, u_out, ld_u, status, iters, s, stream);
        case 2: return launch_t<NV, 2>(P, batch, x0, xref, u_out, ld_u, status, iters, s, stream);
        case 3: return launch_t<NV, 3>(P, batch, x0, xref, u_out, ld_u, status, iters, s, stream);
        case 4: return launch_t<NV, 4>(P, batch, x0, xref, u_out, ld_u, status, iters, s, stream);
        default: return hipErrorInvalidValue;
    }
}
}  // namespace

int dense_pick_nv(int n) {
    for (int nv : kNVs)
        if (nv >= n) return nv;
    return -1;
}

bool dense_supported(int nv, int p, size_t* lds_bytes) {
    const int rs = (p + 63) / 64;
    if (dense_pick_nv(nv) != nv || rs > kMaxRS) return false;
    const size_t lds = dense_lds(nv, p, rs < 1 ? 1 : rs, kWPB);
    if (lds_bytes) *lds_bytes = lds;
    return lds <= 160 * 1024;
}

hipError_t launch_dense(const DevProblem& P, int64_t batch, const double* x0, const double* xref, double* u_out,
                        int64_t ld_u, int32_t* status, int32_t* iters, const Settings& s, hipStream_t stream,
                        int* unsupported) {
    *unsupported = 0;
    if (batch <= 0) return hipSuccess;
    size_t lds = 0;
    if (!dense_supported(P.nv, P.p, &lds)) {
        *unsupported = 1;
        return hipErrorInvalidValue;
    }
    int rs = (P.p + 63) / 64;
    if (rs < 1) rs = 1;
    switch (P.nv) {
        case 8: return launch_rs<8>(rs, P, batch, x0, xref, u_out, ld_u, status, iters, s, stream);
        case 16: return launch_rs<16>(rs, P, batch, x0, xref, u_out, ld_u, status, iters, s, stream);
        case 20: return launch_rs<20>(rs, P, batch, x0, xref, u_out, ld_u, status, iters, s, stream);
        case 24: return launch_rs<24>(rs, P, batch, x0, xref, u_out, ld_u, status, iters, s, stream);
        case 32: return launch_rs<32>(rs, P, batch, x0, xref, u_out, ld_u, status, iters, s, stream);
        case 40: return launch_rs<40>(rs, P, batch, x0, xref, u_out, ld_u, status, iters, s, stream);
        case 48: return launch_rs<48>(rs, P, batch, x0, xref, u_out, ld_u, status, iters, s, stream);
        case 64: return launch_rs<64>(rs, P, batch, x0, xref, u_out, ld_u, status, iters, s, stream);
        default: *unsupported = 1; return hipErrorInvalidValue;
    }
}

}  // namespace carmpc
