// ipm_dense.hip -- dense condensed-QP Mehrotra IPM, one wavefront per QP (gfx950).
//
// Replaces the per-step cvxpy solve of lib/mpc.py:334-335 (MPCStateFB.step) and
// lib/mpc.py:477-478 (MPCOutputFB.step).  Algorithm: Mehrotra predictor-corrector IPM, restated on the
// CPU in oracle/qp.py::ipm and oracle/ipm.c (same steps, same tolerances):
//   Mehrotra predictor-corrector on the normal equations M = H + G'diag(z/s)G + box,
//   one iterative-refinement pass on the corrector, box-Farkas infeasibility
//   certificate, and an active-set polish once mu <= POLISH_MU.
//
// Layout:
//   * one workgroup = WPB wavefronts sharing one problem (environment); G (p x ldg,
//     unit rows, ldg = NV+2 doubles, 16B-aligned rows) and H (NV x NV) live in LDS;
//   * lane i < NV owns decision variable i: u_i, its box slacks/duals, and column i
//     of M in NV registers ("slot j" = M[j][i]);
//   * general row r lives in lane r%64, register slot r/64 (RS slots);
//   * per-wave broadcast buffers (bvec: an NV-vector, rvec: a p-vector) sit at a
//     static LDS offset so every access is base + immediate;
//   * the Cholesky broadcasts lane k's column with v_readlane (no LDS round trip).
// After the Cholesky, lane i's slot j holds L[i][j] (j<i), l_ii (j==i) and
// l_ii*L[j][i] (j>i), so both triangular solves run without data movement.
#include "carmpc_internal.h"

#include <hip/hip_runtime.h>
#include <math.h>

namespace carmpc {

constexpr double POLISH_MU = 1e-6;
constexpr double POLISH_DELTA = 1e-10;
constexpr int POLISH_REFINE = 3;
constexpr double POLISH_TOL = 1e-11;

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
// Step-to-boundary ratio -v/dv for dv < 0, +inf otherwise.  The hardware reciprocal
// is enough: the result only feeds the fraction-to-boundary rule (x 0.99).
__device__ __forceinline__ double ratio(double v, double dv) {
    const double r = -v * __builtin_amdgcn_rcp(dv);
    return dv < 0.0 ? r : INFINITY;
}

// Per-wave view of the problem data and broadcast buffers.
template <int NV, int RS>
struct WaveCtx {
    const double* Gs;   // LDS, p x ldg
    const double* Hs;   // LDS, NV x NV
    double* bvec;       // LDS, 64 doubles (this wave)
    double* rvec;       // LDS, 64*RS doubles (this wave)
    int p, ldg, lane, li;
    bool act;
    bool rv[RS];

    // out[s] = (G v)_{row s}, v given per lane (lanes >= NV pass 0)
    __device__ __forceinline__ void gmul(double v, double (&out)[RS]) const {
        __builtin_amdgcn_wave_barrier();
        bvec[lane] = v;
        __builtin_amdgcn_wave_barrier();
        const double2* v2 = reinterpret_cast<const double2*>(bvec);
#pragma unroll
        for (int s = 0; s < RS; ++s) {
            const int r = rv[s] ? s * 64 + lane : 0;
            const double2* g2 = reinterpret_cast<const double2*>(Gs + (size_t)r * ldg);
            double acc = 0.0;
#pragma unroll
            for (int j = 0; j < NV / 2; ++j) {
                const double2 a = g2[j], b = v2[j];
                acc = fma(a.x, b.x, acc);
                acc = fma(a.y, b.y, acc);
            }
            out[s] = rv[s] ? acc : 0.0;
        }
    }
    // (H v)_lane, with v already in bvec (call right after gmul / put)
    __device__ __forceinline__ double hmul_bvec() const {
        const double2* v2 = reinterpret_cast<const double2*>(bvec);
        double acc = 0.0;
#pragma unroll
        for (int j = 0; j < NV / 2; ++j) {
            const double2 b = v2[j];
            acc = fma(Hs[(2 * j) * NV + li], b.x, acc);
            acc = fma(Hs[(2 * j + 1) * NV + li], b.y, acc);
        }
        return act ? acc : 0.0;
    }
    __device__ __forceinline__ void put(double v) const {
        __builtin_amdgcn_wave_barrier();
        bvec[lane] = v;
        __builtin_amdgcn_wave_barrier();
    }
    // (G' y)_lane for a row vector y
    __device__ __forceinline__ double gtmul(const double (&y)[RS]) const {
        __builtin_amdgcn_wave_barrier();
#pragma unroll
        for (int s = 0; s < RS; ++s) rvec[s * 64 + lane] = y[s];
        __builtin_amdgcn_wave_barrier();
        double acc = 0.0;
        for (int r = 0; r < p; ++r) acc = fma(Gs[r * ldg + li], rvec[r], acc);
        return act ? acc : 0.0;
    }
    // M = H + G' diag(d) G + diag(dbox): column `lane` in registers
    __device__ __forceinline__ void build_M(double (&M)[NV], const double (&d)[RS], double dbox) const {
        __builtin_amdgcn_wave_barrier();
#pragma unroll
        for (int s = 0; s < RS; ++s) rvec[s * 64 + lane] = d[s];
        __builtin_amdgcn_wave_barrier();
#pragma unroll
        for (int j = 0; j < NV; ++j) M[j] = Hs[j * NV + li];
        for (int r = 0; r < p; ++r) {
            const double dr = rvec[r];
            if (dr == 0.0) continue;   // wave-uniform
            const double2* g2 = reinterpret_cast<const double2*>(Gs + (size_t)r * ldg);
            const double t = dr * Gs[r * ldg + li];
#pragma unroll
            for (int j = 0; j < NV / 2; ++j) {
                const double2 g = g2[j];
                M[2 * j] = fma(g.x, t, M[2 * j]);
                M[2 * j + 1] = fma(g.y, t, M[2 * j + 1]);
            }
        }
#pragma unroll
        for (int j = 0; j < NV; ++j) M[j] += (j == lane) ? dbox : 0.0;
    }
};

// Guarded right-looking Cholesky in the slot layout.  Lane k's own column (slots
// j > k, still holding l_kk * L[j][k]) is broadcast with v_readlane.
template <int NV>
__device__ __forceinline__ double cholesky(double (&M)[NV], int lane) {
    asm volatile("" : "+v"(lane));   // keep the per-k lane masks local (no hoisting into SGPRs)
    double inv_ii = 1.0;
#pragma unroll
    for (int k = 0; k < NV; ++k) {
        double piv = readlane_d(M[k], k);
        if (!(piv > 0.0)) piv = 1e128;
        const double lkk = sqrt(piv);
        const double inv = 1.0 / lkk;
        const bool below = lane > k && lane < NV;
        const double l = below ? M[k] * inv : 0.0;     // L[lane][k]
        const double lt = l * inv;                      // L[lane][k] / l_kk
#pragma unroll
        for (int j = k + 1; j < NV; ++j) M[j] = fma(-readlane_d(M[j], k), lt, M[j]);
        M[k] = (lane == k) ? lkk : (below ? l : M[k]);
        inv_ii = (lane == k) ? inv : inv_ii;
    }
    return inv_ii;
}

// Solve L L' x = b (b per lane, lanes >= NV pass 0).
template <int NV>
__device__ __forceinline__ double chol_solve(const double (&M)[NV], double inv_ii, double b, int lane) {
    asm volatile("" : "+v"(lane));   // keep the per-k lane masks local (no hoisting into SGPRs)
#pragma unroll
    for (int k = 0; k < NV; ++k) {   // forward: lane i's slot k<i holds L[i][k]
        const double yk = readlane_d(b * inv_ii, k);
        const double upd = fma(M[k], -yk, b);
        b = (lane > k) ? upd : b;
        b = (lane == k) ? yk : b;
    }
    double acc = 0.0;
#pragma unroll
    for (int k = NV - 1; k >= 0; --k) {   // backward: lane i's slot k>i holds l_ii L[k][i]
        const double xk = readlane_d((b - inv_ii * acc) * inv_ii, k);
        const double upd = fma(M[k], xk, acc);
        b = (lane == k) ? xk : b;
        acc = (lane < k) ? upd : acc;
    }
    return lane < NV ? b : 0.0;
}

}  // namespace

// HET: every instance has its own problem slice (hetero.hip; G, H read from global memory,
// p / npre per instance); otherwise one problem per launch with G, H in LDS.
template <int NV, int RS, int kWPB, bool HET = false>
__global__ void __launch_bounds__(kWPB * 64) ipm_dense_kernel(DevProblem P, int64_t batch,
                                                              const double* __restrict__ x0,
                                                              const double* __restrict__ xref,
                                                              double* __restrict__ u_out, int64_t ld_u,
                                                              int32_t* __restrict__ status_out,
                                                              int32_t* __restrict__ iters_out, Settings S) {
    static_assert(NV % 2 == 0 && NV <= 64, "NV must be even and <= 64");
    __shared__ __attribute__((aligned(16))) double wscr[kWPB][64 + 64 * RS];
    extern __shared__ __attribute__((aligned(16))) double smem[];
    const int lane = threadIdx.x & 63;
    const int wave = threadIdx.x >> 6;
    int p = P.p;
    const int ldg = P.ldg;
    double* Gs = smem;
    double* Hs = Gs + ((p * ldg + 1) & ~1);
    if (!HET) {
        for (int i = threadIdx.x; i < p * ldg; i += blockDim.x) Gs[i] = P.G[i];
        for (int i = threadIdx.x; i < NV * NV; i += blockDim.x) Hs[i] = P.H[i];
        __syncthreads();
    }

    WaveCtx<NV, RS> W;
    W.Gs = Gs; W.Hs = Hs; W.bvec = wscr[wave]; W.rvec = wscr[wave] + 64;
    W.p = p; W.ldg = ldg; W.lane = lane; W.act = lane < NV; W.li = W.act ? lane : 0;
#pragma unroll
    for (int s = 0; s < RS; ++s) W.rv[s] = (s * 64 + lane) < p;
    const bool act = W.act;
    const bool boxact = act && P.boxed;
    const double lb = boxact ? P.lb[W.li] : -UNBOXED_BOUND;
    const double ub = boxact ? P.ub[W.li] : UNBOXED_BOUND;
    const double bndabs = fmax(fabs(lb), fabs(ub));
    int m_rows = p + (P.boxed ? 2 * NV : 0);
    double inv_m = 1.0 / (double)(m_rows > 0 ? m_rows : 1);

    // closed-loop runs solve only their live instances: slot -> row through S.index, count on device
    const int64_t nlive = S.count ? (int64_t)*S.count : batch;
    const int64_t stride = (int64_t)gridDim.x * kWPB;
    for (int64_t slot = S.claim ? wave_claim(S.claim) : (int64_t)blockIdx.x * kWPB + wave; slot < nlive;
         slot = S.claim ? wave_claim(S.claim) : slot + stride) {
        const int64_t inst = S.index ? (int64_t)S.index[slot] : slot;
        // this instance's rows (shared problem: the launch's; HET: its own slice)
        const double *Pw0 = P.w0, *PE = P.E, *Phq = P.hq, *Ppw = P.pre_w0, *PpE = P.pre_E;
        const int32_t* Ppart = P.partner;
        int npre = P.npre;
        if (HET) {
            p = P.het_p[inst];
            npre = P.het_npre[inst];
            W.Gs = P.G + inst * P.het_sG;
            W.Hs = P.H + inst * P.het_sH;
            W.p = p;
#pragma unroll
            for (int s = 0; s < RS; ++s) W.rv[s] = (s * 64 + lane) < p;
            m_rows = p + (P.boxed ? 2 * NV : 0);
            inv_m = 1.0 / (double)(m_rows > 0 ? m_rows : 1);
            Pw0 += inst * P.het_sRow;
            PE += inst * P.het_sRow * NX;
            Ppw += inst * P.het_sRow;
            PpE += inst * P.het_sRow * NX;
            Ppart += inst * P.het_sRow;
            Phq += inst * P.het_sHq;
        }
        double xv[NX], xr[NX];
#pragma unroll
        for (int k = 0; k < NX; ++k) {
            xv[k] = x0[inst * NX + k];
            xr[k] = xref ? xref[inst * NX + k] : P.goal[k];
        }
        // ---- x0-only rows (G_r == 0): preconditions on x0 ---------------------
        const double dd = S.dist ? S.dist[inst] : 0.0;   // disturbance estimate (w -= Ed d)
        bool bad = false;
        for (int r = lane; r < npre; r += 64) {
            double v = Ppw[r];
#pragma unroll
            for (int k = 0; k < NX; ++k) v -= PpE[r * NX + k] * xv[k];
            if (P.pre_Ed) v -= P.pre_Ed[r] * dd;
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
        // ---- per-instance data: q = hq (x0 - xref), w = w0 - E x0 -------------
        double q = 0.0;
        if (act) {
#pragma unroll
            for (int k = 0; k < NX; ++k) q += Phq[W.li * NX + k] * (xv[k] - xr[k]);
        }
        double w[RS];
#pragma unroll
        for (int s = 0; s < RS; ++s) {
            const int r = s * 64 + lane;
            double v = 0.0;
            if (W.rv[s]) {
                v = Pw0[r];
#pragma unroll
                for (int k = 0; k < NX; ++k) v -= PE[r * NX + k] * xv[k];
                if (P.Ed) v -= P.Ed[r] * dd;
            }
            w[s] = v;
        }
        // ---- initial point ----------------------------------------------------
        double u = boxact ? fmin(fmax(0.0, lb), ub) : 0.0;
        double su = boxact ? fmax(ub - u, 1.0) : 1.0;
        double sl = boxact ? fmax(u - lb, 1.0) : 1.0;
        double zu = boxact ? 1.0 : 0.0, zl = zu;
        double s_[RS], z_[RS];
        {
            double gu[RS];
            W.gmul(act ? u : 0.0, gu);
#pragma unroll
            for (int s = 0; s < RS; ++s) {
                s_[s] = W.rv[s] ? fmax(w[s] - gu[s], 1.0) : 1.0;
                z_[s] = W.rv[s] ? 1.0 : 0.0;
            }
        }
        double bn = boxact ? bndabs : 0.0;
#pragma unroll
        for (int s = 0; s < RS; ++s) bn = fmax(bn, W.rv[s] ? fabs(w[s]) : 0.0);
        const double bnorm = 1.0 + wave_max(bn);
        const double qnorm = 1.0 + wave_max(act ? fabs(q) : 0.0);

        int status = CARMPC_MAX_ITER;
        int it = 0;
        bool polish_failed = false;
        double M[NV];
        // One trip = residuals, then ONE factorization followed by a rolled loop of
        // solves with that factor, so the unrolled build_M / cholesky / chol_solve
        // bodies exist once in the binary (register allocation stays sane):
        //   IPM trip:    solve 0 predictor, 1 corrector, 2 refinement of the corrector
        //   polish trip: solves 0..POLISH_REFINE of the regularised active-set KKT
        for (;;) {
            // ---- residuals and their scales ------------------------------------
            double rp[RS];
            double gtz, rd, rpu, rpl, mu;
            bool res_ok;
            {
                double gu[RS];
                W.gmul(act ? u : 0.0, gu);
                const double hu = W.hmul_bvec();
                gtz = W.gtmul(z_);
                double rpn = 0.0, musum = 0.0, gun = 0.0;
#pragma unroll
                for (int s = 0; s < RS; ++s) {
                    rp[s] = W.rv[s] ? gu[s] + s_[s] - w[s] : 0.0;
                    rpn = fmax(rpn, fabs(rp[s]));
                    gun = fmax(gun, fabs(gu[s]));
                    musum += s_[s] * z_[s];
                }
                rpu = boxact ? u + su - ub : 0.0;
                rpl = boxact ? -u + sl + lb : 0.0;
                rpn = fmax(rpn, fmax(fabs(rpu), fabs(rpl)));
                musum += boxact ? su * zu + sl * zl : 0.0;
                const double gz = gtz + (boxact ? zu - zl : 0.0);
                rd = act ? hu + q + gz : 0.0;
                mu = wave_sum(musum) * inv_m;
                const double rpn_w = wave_max(rpn);
                const double rdn_w = wave_max(fabs(rd));
                const double pscale = fmax(bnorm, 1.0 + wave_max(fmax(gun, boxact ? fabs(u) : 0.0)));
                const double dscale = fmax(qnorm, 1.0 + wave_max(fmax(fabs(hu), fabs(gz))));
                if (!isfinite(mu) || !isfinite(rdn_w)) { status = CARMPC_NUMERICAL; break; }
                res_ok = rpn_w <= S.tol * pscale && rdn_w <= S.tol * dscale;
            }
            const bool last = it >= S.max_iter;
            const bool polish = !polish_failed && ((res_ok && mu <= POLISH_MU) || last);
            if (!polish) {
                if (last) break;
                if (res_ok && mu <= S.tol_mu) { status = CARMPC_OPTIMAL; break; }
                // ---- Farkas certificate: min_box (G'z)'u > w'z  =>  infeasible -----
                if (p > 0) {
                    double wz = 0.0, wzabs = 0.0;
#pragma unroll
                    for (int s = 0; s < RS; ++s) { wz += w[s] * z_[s]; wzabs += fabs(w[s]) * z_[s]; }
                    const double lo = act ? fmin(gtz * lb, gtz * ub) : 0.0;
                    const double sc = act ? fabs(gtz) * bndabs : 0.0;
                    const double lo_w = wave_sum(lo), wz_w = wave_sum(wz), sc_w = wave_sum(sc + wzabs);
                    if (lo_w - wz_w > 1e-12 * sc_w) { status = CARMPC_PRIMAL_INFEASIBLE; break; }
                }
            }
            // ---- factor: IPM M = H + G'diag(z/s)G + box, polish M = H + A_act'A_act/delta
            const double id = 1.0 / POLISH_DELTA;
            const double dbu = (polish && boxact && su < zu) ? id : 0.0;   // polish: active box rows
            const double dbl = (polish && boxact && sl < zl) ? id : 0.0;
            double dg[RS];
#pragma unroll
            for (int s = 0; s < RS; ++s)
                dg[s] = !W.rv[s] ? 0.0 : (polish ? (s_[s] < z_[s] ? id : 0.0) : z_[s] / s_[s]);
            W.build_M(M, dg, polish ? dbu + dbl : (boxact ? zu / su + zl / sl : 0.0));
            const double inv_ii = cholesky<NV>(M, lane);
            // ---- solve sequence ------------------------------------------------
            // row temporaries:  ra = dS (IPM) | y_g (polish);  rb = dZ (IPM) | ry_g (polish)
            //                   pa = dS_aff * dZ_aff (IPM predictor product)
            // lane temporaries: v0 = du | x;  v1 = dSu | y_u;  v2 = dSl | y_l;  v3 = dZu;  v4 = dZl
            double ra[RS], rb[RS], pa[RS];
#pragma unroll
            for (int s = 0; s < RS; ++s) { ra[s] = 0.0; rb[s] = 0.0; pa[s] = 0.0; }
            double v0 = 0.0, v1 = 0.0, v2 = 0.0, v3 = 0.0, v4 = 0.0, pua = 0.0, pla = 0.0, sigma_mu = 0.0;
            const int nsolve = polish ? POLISH_REFINE + 1 : (mu <= REFINE_MU ? 3 : 2);   // refinement late only
#pragma unroll 1
            for (int k = 0; k < nsolve; ++k) {
                double rhs, ryu = 0.0, ryl = 0.0;
                if (polish) {
                    double gx[RS], t[RS];
                    W.gmul(act ? v0 : 0.0, gx);
                    const double hx = W.hmul_bvec();
                    const double gty = W.gtmul(ra);
#pragma unroll
                    for (int s = 0; s < RS; ++s) {
                        rb[s] = dg[s] != 0.0 ? w[s] - gx[s] : 0.0;
                        t[s] = dg[s] * rb[s];
                    }
                    ryu = dbu != 0.0 ? ub - v0 : 0.0;
                    ryl = dbl != 0.0 ? -lb + v0 : 0.0;
                    const double gtt = W.gtmul(t);
                    rhs = act ? -q - hx - gty - v1 + v2 + gtt + dbu * ryu - dbl * ryl : 0.0;
                } else if (k < 2) {
                    double t[RS];
#pragma unroll
                    for (int s = 0; s < RS; ++s) {
                        const double rc = s_[s] * z_[s] + pa[s] - (k == 1 && W.rv[s] ? sigma_mu : 0.0);
                        t[s] = W.rv[s] ? (rc - z_[s] * rp[s]) / s_[s] : 0.0;
                    }
                    const double rcu = !boxact ? 0.0 : su * zu + pua - (k == 1 ? sigma_mu : 0.0);
                    const double rcl = !boxact ? 0.0 : sl * zl + pla - (k == 1 ? sigma_mu : 0.0);
                    const double gtt = W.gtmul(t);
                    rhs = act ? -rd + gtt + (boxact ? (rcu - zu * rpu) / su - (rcl - zl * rpl) / sl : 0.0) : 0.0;
                } else {
                    // refinement residual of the corrector: e = H du + G'dZ + rd + box
                    W.put(act ? v0 : 0.0);
                    const double hdu = W.hmul_bvec();
                    const double gtdz = W.gtmul(rb);
                    rhs = act ? -(hdu + gtdz + rd + (boxact ? v3 - v4 : 0.0)) : 0.0;
                }
                const double sol = chol_solve<NV>(M, inv_ii, rhs, lane);
                double gs[RS];
                W.gmul(sol, gs);
                if (polish) {
#pragma unroll
                    for (int s = 0; s < RS; ++s) ra[s] += dg[s] * (gs[s] - rb[s]);
                    v1 += dbu * (sol - ryu);
                    v2 += dbl * (-sol - ryl);
                    v0 += sol;
                } else if (k < 2) {
                    v0 = sol;
#pragma unroll
                    for (int s = 0; s < RS; ++s) {
                        const double rc = s_[s] * z_[s] + pa[s] - (k == 1 && W.rv[s] ? sigma_mu : 0.0);
                        ra[s] = W.rv[s] ? -rp[s] - gs[s] : 0.0;
                        rb[s] = W.rv[s] ? (-rc - z_[s] * ra[s]) / s_[s] : 0.0;
                    }
                    const double rcu = !boxact ? 0.0 : su * zu + pua - (k == 1 ? sigma_mu : 0.0);
                    const double rcl = !boxact ? 0.0 : sl * zl + pla - (k == 1 ? sigma_mu : 0.0);
                    v1 = boxact ? -rpu - sol : 0.0;
                    v2 = boxact ? -rpl + sol : 0.0;
                    v3 = boxact ? (-rcu - zu * v1) / su : 0.0;
                    v4 = boxact ? (-rcl - zl * v2) / sl : 0.0;
                    if (k == 0) {   // affine step -> centering parameter
                        double amax = fmin(fmin(ratio(su, v1), ratio(zu, v3)), fmin(ratio(sl, v2), ratio(zl, v4)));
#pragma unroll
                        for (int s = 0; s < RS; ++s) amax = fmin(amax, fmin(ratio(s_[s], ra[s]), ratio(z_[s], rb[s])));
                        const double a = fmin(1.0, wave_min(amax));
                        double mua = boxact ? (su + a * v1) * (zu + a * v3) + (sl + a * v2) * (zl + a * v4) : 0.0;
#pragma unroll
                        for (int s = 0; s < RS; ++s) {
                            mua += (s_[s] + a * ra[s]) * (z_[s] + a * rb[s]);
                            pa[s] = ra[s] * rb[s];
                        }
                        const double sg = wave_sum(mua) * inv_m / mu;
                        sigma_mu = sg * sg * sg * mu;
                        pua = v1 * v3;
                        pla = v2 * v4;
                    }
                } else {
#pragma unroll
                    for (int s = 0; s < RS; ++s) {
                        ra[s] -= gs[s];
                        rb[s] += W.rv[s] ? z_[s] * gs[s] / s_[s] : 0.0;
                    }
                    v0 += sol;
                    if (boxact) {
                        v1 -= sol; v3 += zu * sol / su;
                        v2 += sol; v4 -= zl * sol / sl;
                    }
                }
            }
            if (polish) {
                // accept iff primal feasible and active multipliers nonnegative
                double gx[RS];
                W.gmul(act ? v0 : 0.0, gx);
                double viol = boxact ? fmax(v0 - ub, lb - v0) : -INFINITY;
                double wsc = boxact ? bndabs : 0.0, ysc = fmax(fabs(v1), fabs(v2)), ymin = fmin(v1, v2);
                // rows whose opposite partner is also active form an equality: their
                // multipliers may be re-split, so they skip the sign test (oracle/qp.py)
                bool paired[RS];
#pragma unroll
                for (int s = 0; s < RS; ++s) paired[s] = false;
                if (Ppart) {
                    __builtin_amdgcn_wave_barrier();
#pragma unroll
                    for (int s = 0; s < RS; ++s) W.rvec[s * 64 + lane] = (W.rv[s] && dg[s] != 0.0) ? ra[s] : NAN;
                    __builtin_amdgcn_wave_barrier();
#pragma unroll
                    for (int s = 0; s < RS; ++s) {
                        const int pr = W.rv[s] ? Ppart[s * 64 + lane] : -1;
                        paired[s] = pr >= 0 && dg[s] != 0.0 && !isnan(W.rvec[pr]);
                    }
                }
#pragma unroll
                for (int s = 0; s < RS; ++s) {
                    if (W.rv[s]) {
                        viol = fmax(viol, gx[s] - w[s]);
                        wsc = fmax(wsc, fabs(w[s]));
                        ysc = fmax(ysc, fabs(ra[s]));
                        ymin = paired[s] ? ymin : fmin(ymin, ra[s]);
                    }
                }
                const bool fin = !act || isfinite(v0);
                viol = wave_max(viol); wsc = wave_max(wsc); ysc = wave_max(ysc); ymin = wave_min(ymin);
                if (__all(fin) && viol <= POLISH_TOL * (1.0 + wsc) && ymin >= -POLISH_TOL * (1.0 + ysc)) {
                    u = act ? v0 : 0.0;
                    status = CARMPC_OPTIMAL;
                    break;
                }
                polish_failed = true;
                continue;
            }
            // ---- step to the fraction-to-boundary and update ---------------------
            double amax = fmin(fmin(ratio(su, v1), ratio(zu, v3)), fmin(ratio(sl, v2), ratio(zl, v4)));
#pragma unroll
            for (int s = 0; s < RS; ++s) amax = fmin(amax, fmin(ratio(s_[s], ra[s]), ratio(z_[s], rb[s])));
            const double a = fmin(1.0, STEP_FRAC * wave_min(amax));
            u += a * v0;
#pragma unroll
            for (int s = 0; s < RS; ++s) { s_[s] += a * ra[s]; z_[s] += a * rb[s]; }
            su += a * v1; zu += a * v3; sl += a * v2; zl += a * v4;
            polish_failed = false;
            ++it;
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

size_t dense_lds(int nv, int p) {   // dynamic part only (G, H)
    const int ldg = nv + 2;
    return ((size_t)((p * ldg + 1) & ~1) + (size_t)nv * nv) * sizeof(double);
}

template <int NV, int RS, int kWPB>
hipError_t launch_t(const DevProblem& P, int64_t batch, const double* x0, const double* xref, double* u_out,
                    int64_t ld_u, int32_t* status, int32_t* iters, const Settings& s, hipStream_t stream) {
    const size_t lds = dense_lds(NV, P.p);
    auto kern = ipm_dense_kernel<NV, RS, kWPB>;
    static bool attr_set = false;
    if (!attr_set) {
        hipError_t e = hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize,
                                           160 * 1024 - (int)(sizeof(double) * kWPB * (64 + 64 * RS)));
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
    return launch_with_claim(s, batch, stream, [&](const Settings& sc) {
        hipLaunchKernelGGL(kern, dim3((unsigned)grid), dim3(kWPB * 64), lds, stream, P, batch, x0, xref, u_out, ld_u,
                           status, iters, sc);
        return hipGetLastError();
    });
}

template <int NV>
hipError_t launch_rs(int rs, const DevProblem& P, int64_t batch, const double* x0, const double* xref,
                     double* u_out, int64_t ld_u, int32_t* status, int32_t* iters, const Settings& s,
                     hipStream_t stream) {
    // kernel 3 selects the one-wave-per-SIMD variant (4 waves / workgroup, 512 registers)
    if (s.kernel == 3 && (NV == 20 || NV == 40)) {
        switch (rs) {
            case 1: return launch_t<NV, 1, 4>(P, batch, x0, xref, u_out, ld_u, status, iters, s, stream);
            case 2: return launch_t<NV, 2, 4>(P, batch, x0, xref, u_out, ld_u, status, iters, s, stream);
            case 3: return launch_t<NV, 3, 4>(P, batch, x0, xref, u_out, ld_u, status, iters, s, stream);
            case 4: return launch_t<NV, 4, 4>(P, batch, x0, xref, u_out, ld_u, status, iters, s, stream);
            default: return hipErrorInvalidValue;
        }
    }
    switch (rs) {
        case 1: return launch_t<NV, 1, 8>(P, batch, x0, xref, u_out, ld_u, status, iters, s, stream);
        case 2: return launch_t<NV, 2, 8>(P, batch, x0, xref, u_out, ld_u, status, iters, s, stream);
        case 3: return launch_t<NV, 3, 8>(P, batch, x0, xref, u_out, ld_u, status, iters, s, stream);
        case 4: return launch_t<NV, 4, 8>(P, batch, x0, xref, u_out, ld_u, status, iters, s, stream);
        default: return hipErrorInvalidValue;
    }
}
template <int NV, int RS>
hipError_t launch_het_t(const DevProblem& P, int64_t batch, const double* x0, const double* xref, double* u_out,
                        int64_t ld_u, int32_t* status, int32_t* iters, const Settings& s, hipStream_t stream) {
    constexpr int kWPB = 4;
    auto kern = ipm_dense_kernel<NV, RS, kWPB, true>;
    int dev = 0, cus = 0, per_cu = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e != hipSuccess) return e;
    e = hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    if (e != hipSuccess) return e;
    e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, (const void*)kern, kWPB * 64, 0);
    if (e != hipSuccess) return e;
    if (per_cu < 1) per_cu = 1;
    int64_t want = (batch + kWPB - 1) / kWPB;
    int64_t grid = (int64_t)cus * per_cu;
    if (want < grid) grid = want;
    if (grid < 1) grid = 1;
    return launch_with_claim(s, batch, stream, [&](const Settings& sc) {
        hipLaunchKernelGGL(kern, dim3((unsigned)grid), dim3(kWPB * 64), 0, stream, P, batch, x0, xref, u_out, ld_u,
                           status, iters, sc);
        return hipGetLastError();
    });
}
template <int NV>
hipError_t launch_het_rs(int rs, const DevProblem& P, int64_t batch, const double* x0, const double* xref,
                         double* u_out, int64_t ld_u, int32_t* status, int32_t* iters, const Settings& s,
                         hipStream_t stream) {
    switch (rs) {
        case 1: return launch_het_t<NV, 1>(P, batch, x0, xref, u_out, ld_u, status, iters, s, stream);
        case 2: return launch_het_t<NV, 2>(P, batch, x0, xref, u_out, ld_u, status, iters, s, stream);
        case 3: return launch_het_t<NV, 3>(P, batch, x0, xref, u_out, ld_u, status, iters, s, stream);
        case 4: return launch_het_t<NV, 4>(P, batch, x0, xref, u_out, ld_u, status, iters, s, stream);
        default: return hipErrorInvalidValue;
    }
}
}  // namespace

hipError_t launch_dense_het(const DevProblem& P, int p_max, int64_t batch, const double* x0, const double* xref,
                            double* u_out, int64_t ld_u, int32_t* status, int32_t* iters, const Settings& s,
                            hipStream_t stream, int* unsupported) {
    *unsupported = 0;
    if (batch <= 0) return hipSuccess;
    int rs = (p_max + 63) / 64;
    if (rs < 1) rs = 1;
    if (rs > kMaxRS) {
        *unsupported = 1;
        return hipErrorInvalidValue;
    }
    switch (P.nv) {
        case 8: return launch_het_rs<8>(rs, P, batch, x0, xref, u_out, ld_u, status, iters, s, stream);
        case 16: return launch_het_rs<16>(rs, P, batch, x0, xref, u_out, ld_u, status, iters, s, stream);
        case 20: return launch_het_rs<20>(rs, P, batch, x0, xref, u_out, ld_u, status, iters, s, stream);
        case 24: return launch_het_rs<24>(rs, P, batch, x0, xref, u_out, ld_u, status, iters, s, stream);
        case 32: return launch_het_rs<32>(rs, P, batch, x0, xref, u_out, ld_u, status, iters, s, stream);
        case 40: return launch_het_rs<40>(rs, P, batch, x0, xref, u_out, ld_u, status, iters, s, stream);
        case 48: return launch_het_rs<48>(rs, P, batch, x0, xref, u_out, ld_u, status, iters, s, stream);
        case 64: return launch_het_rs<64>(rs, P, batch, x0, xref, u_out, ld_u, status, iters, s, stream);
        default: *unsupported = 1; return hipErrorInvalidValue;
    }
}


int dense_pick_nv(int n) {
    for (int nv : kNVs)
        if (nv >= n) return nv;
    return -1;
}

bool dense_supported(int nv, int p, size_t* lds_bytes) {
    int rs = (p + 63) / 64;
    if (rs < 1) rs = 1;
    if (dense_pick_nv(nv) != nv || rs > kMaxRS) return false;
    const size_t lds = dense_lds(nv, p) + sizeof(double) * 8 * (64 + 64 * rs);
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
