// ipm_staged.hip -- stage-structured condensed-QP Mehrotra IPM, one wavefront per QP (gfx950).
//
// Same algorithm, tolerances and trip structure as ipm_dense.hip (CPU
// restatement oracle/qp.py::ipm, oracle/ipm.c), replacing the per-step cvxpy solve of
// lib/mpc.py:334-335 / 477-478.  What changes is how the products with G, H and the
// normal matrix are formed: every QP row of the reference acts on ONE predicted state
// (mpc.py:196-253: terminal rows on x_N, state rows on x_1..x_N), so with
// Phi_m = A^m B (matrix_gen.py:6-32)
//     (G v)_r   = c_r . Y_{k_r},            Y_k = sum_{t<k} Phi_{k-1-t} v_t
//     (G'y)_i   = sum_{k>t_i} Phi_{k-1-t_i}[:,c_i] . lam_k,   lam_k = sum_{r in k} y_r c_r
//     H         = R_hat + sum_k S_k' Qbar_k S_k            (matrix_gen.py:35-72)
//     M = H + G'DG = R_hat + sum_k S_k'(Qbar_k + W_k) S_k,  W_k = sum_{r in k} d_r c_r c_r'
// and M comes from the backward recursion  Z_{N-1} = Qt_N,  Z_t = Qt_{t+1} + A'Z_{t+1}A,
//     M[(t,c'),(s,c)] = B_c'' Z_t Phi_{t-s}[:,c]   (t >= s, + R on the diagonal block).
// The M build drops from p n^2 to ~N*(64+40) flops per lane and G never has to sit in
// LDS, which leaves room to keep the long-lived row vectors (w, predictor products,
// row weights) in LDS instead of registers.
//
// Lane roles (nu = 2, n = 2N = NV):
//   variable lane i = (t_i, c_i) = (i/2, i%2) owns u_i and column i of M (as dense);
//   row lanes: row slot (s, L) holds a row of stage k(L) = L%32 + 1 for L%32 < N, and a
//     terminal row (stage N) on the "tail" lanes L%32 >= N, so per-stage sums are a
//     pairwise (L, L^32) add plus one tail reduction (host layout: capi.hip::stage_layout);
//   state lanes L < 2N compute the two components (2(L&1), 2(L&1)+1) of Y_{L/2+1}.
#include "carmpc_internal.h"

#include <hip/hip_runtime.h>
#include <math.h>

// Optional per-phase cycle accounting (profiling build only: -DCARMPC_PHASE_TIMING,
// tools/phase_timing.py).  Phases: 0 residuals, 1 Farkas/decisions, 2 M build,
// 3 Cholesky, 4 right-hand sides, 5 triangular solves, 6 G dx + direction update,
// 7 step / polish verification.
#ifdef CARMPC_PHASE_TIMING
__device__ unsigned long long carmpc_phase_cycles[8];
#define PT_DECL                                   \
    unsigned long long pt_acc[8] = {0, 0, 0, 0, 0, 0, 0, 0}; \
    unsigned long long pt_t = clock64();
#define PT_MARK(i)                                \
    do {                                          \
        const unsigned long long n_ = clock64();  \
        pt_acc[i] += n_ - pt_t;                   \
        pt_t = n_;                                \
    } while (0)
#define PT_FLUSH()                                                              \
    do {                                                                        \
        if (lane == 0)                                                          \
            for (int i_ = 0; i_ < 8; ++i_) atomicAdd(&carmpc_phase_cycles[i_], pt_acc[i_]); \
    } while (0)
#else
#define PT_DECL
#define PT_MARK(i) do {} while (0)
#define PT_FLUSH() do {} while (0)
#endif

namespace carmpc {

namespace {

constexpr double POLISH_MU = 1e-6;
constexpr double POLISH_DELTA = 1e-10;
constexpr int POLISH_REFINE = 3;
constexpr double POLISH_TOL = 1e-11;

__device__ __forceinline__ double readlane_d(double v, int l) {
    const unsigned long long b = __builtin_bit_cast(unsigned long long, v);
    const unsigned lo = __builtin_amdgcn_readlane((unsigned)(b & 0xffffffffull), l);
    const unsigned hi = __builtin_amdgcn_readlane((unsigned)(b >> 32), l);
    return __builtin_bit_cast(double, ((unsigned long long)hi << 32) | lo);
}
// ---- cross-lane reductions without the LDS crossbar ---------------------------------
// Butterfly pairings only (quad xor 1, quad xor 2, row half-mirror, row mirror, then the
// gfx950 row-16 / half-32 swaps): both lanes of a pair combine the same two operands, so
// every lane ends with a bitwise-identical result (the step length, mu and the Farkas
// sums drive wave-uniform decisions).  ~3 VALU per step instead of a ds_bpermute round
// trip per 32 bits.
template <int CTRL>
__device__ __forceinline__ double dpp_d(double v) {
    const unsigned long long b = __builtin_bit_cast(unsigned long long, v);
    const int lo = __builtin_amdgcn_update_dpp(0, (int)(unsigned)b, CTRL, 0xf, 0xf, false);
    const int hi = __builtin_amdgcn_update_dpp(0, (int)(unsigned)(b >> 32), CTRL, 0xf, 0xf, false);
    return __builtin_bit_cast(double, ((unsigned long long)(unsigned)hi << 32) | (unsigned)lo);
}
// the two operands of the row-16 pair (rows 0<->1, 2<->3) resp. the half-32 pair
__device__ __forceinline__ void swap16_d(double v, double& a, double& b) {
    const unsigned long long x = __builtin_bit_cast(unsigned long long, v);
    const auto lo = __builtin_amdgcn_permlane16_swap((unsigned)x, (unsigned)x, false, false);
    const auto hi = __builtin_amdgcn_permlane16_swap((unsigned)(x >> 32), (unsigned)(x >> 32), false, false);
    a = __builtin_bit_cast(double, ((unsigned long long)hi[0] << 32) | lo[0]);
    b = __builtin_bit_cast(double, ((unsigned long long)hi[1] << 32) | lo[1]);
}
__device__ __forceinline__ void swap32_d(double v, double& a, double& b) {
    const unsigned long long x = __builtin_bit_cast(unsigned long long, v);
    const auto lo = __builtin_amdgcn_permlane32_swap((unsigned)x, (unsigned)x, false, false);
    const auto hi = __builtin_amdgcn_permlane32_swap((unsigned)(x >> 32), (unsigned)(x >> 32), false, false);
    a = __builtin_bit_cast(double, ((unsigned long long)hi[0] << 32) | lo[0]);
    b = __builtin_bit_cast(double, ((unsigned long long)hi[1] << 32) | lo[1]);
}
constexpr int DPP_QXOR1 = 0xB1, DPP_QXOR2 = 0x4E, DPP_HMIRROR = 0x141, DPP_MIRROR = 0x140;
struct OpSum { __device__ static double f(double a, double b) { return a + b; } };
struct OpMax { __device__ static double f(double a, double b) { return fmax(a, b); } };
struct OpMin { __device__ static double f(double a, double b) { return fmin(a, b); } };
// reduction over each 16-lane row
template <class Op>
__device__ __forceinline__ double row_reduce(double v) {
    v = Op::f(v, dpp_d<DPP_QXOR1>(v));
    v = Op::f(v, dpp_d<DPP_QXOR2>(v));
    v = Op::f(v, dpp_d<DPP_HMIRROR>(v));
    return Op::f(v, dpp_d<DPP_MIRROR>(v));
}
// reduction over each 32-lane half
template <class Op>
__device__ __forceinline__ double half_reduce(double v) {
    v = row_reduce<Op>(v);
    double a, b;
    swap16_d(v, a, b);
    return Op::f(a, b);
}
// the result is identical in all lanes: hand it to the compiler as a scalar (SGPR pair)
__device__ __forceinline__ double uniform_d(double v) {
    const unsigned long long b = __builtin_bit_cast(unsigned long long, v);
    const unsigned lo = __builtin_amdgcn_readfirstlane((unsigned)b);
    const unsigned hi = __builtin_amdgcn_readfirstlane((unsigned)(b >> 32));
    return __builtin_bit_cast(double, ((unsigned long long)hi << 32) | lo);
}
template <class Op>
__device__ __forceinline__ double wave_reduce(double v) {
    v = half_reduce<Op>(v);
    double a, b;
    swap32_d(v, a, b);
    return uniform_d(Op::f(a, b));
}
__device__ __forceinline__ double wave_sum(double v) { return wave_reduce<OpSum>(v); }
__device__ __forceinline__ double wave_max(double v) { return wave_reduce<OpMax>(v); }
__device__ __forceinline__ double wave_min(double v) { return wave_reduce<OpMin>(v); }
// Reciprocal / reciprocal square root: hardware approximation + two Newton steps
// (to the last ulp or so; ~5 instructions instead of the ~10 of an IEEE divide).
__device__ __forceinline__ double frcp(double b) {
    double r = __builtin_amdgcn_rcp(b);
    r = fma(fma(-b, r, 1.0), r, r);
    return fma(fma(-b, r, 1.0), r, r);
}
__device__ __forceinline__ double frsq(double a) {
    double r = __builtin_amdgcn_rsq(a);
    const double h = 0.5 * a;
    r = r * fma(-h * r, r, 1.5);
    return r * fma(-h * r, r, 1.5);
}
__device__ __forceinline__ double ratio(double v, double dv) {
    const double r = -v * __builtin_amdgcn_rcp(dv);
    return dv < 0.0 ? r : INFINITY;
}
// index of the symmetric 4x4 entry (a <= b) in the packed 10-vector
__host__ __device__ constexpr int sym10(int a, int b) { return a * 4 - a * (a - 1) / 2 + (b - a); }

// Block-shared problem data (LDS).
template <int N, int RS>
struct StageShared {
    // Phi_m = A^m B tables indexed by a shifted q in [0, 2N-2] so that every gather in a
    // loop over stages is lane_base + (compile-time offset): no per-step index math.
    double fa[(2 * N - 1) * 8];   // [c][a]: Phi_{q-(N-1)} for q >= N-1, else 0
    double fb[(2 * N - 1) * 8];   // [c][a]: Phi_{(N-1)-q} for q <  N-1, else 0
    double fs[(2 * N - 1) * 8];   // [a][c]: Phi_{(N-1)-q} for q <= N-1, else 0
    double2 cf01[RS * 64];        // row coefficients (c0, c1) of slot (s, lane)
    double2 cf23[RS * 64];        // (c2, c3)
    double qp[2][16];             // Q (stages < N), P (stage N)
    double A[16];
    double B[8];                  // [a][c]
    double R[4];
    double lb[64], ub[64];        // input box per variable (+-UNBOXED_BOUND when unboxed)
};
// Per-wave scratch (LDS).
template <int N, int RS>
struct StageWave {
    double bvec[64];              // broadcast of a lane vector
    double Y[(N + 1) * 4];        // predicted states Y_k (k = 1..N)
    double lam[(N + 1) * 4];      // adjoint input lam_k
    double lamH[(N + 1) * 4];     // second adjoint input (residual: H part)
    double Wf[(N + 1) * 10 >= 64 ? (N + 1) * 10 : 64];   // W_k packed symmetric; 2nd Cholesky buffer
    double Z[N * 16];             // Z_t (t = 0..N-1)
    double Gam[N * 8];            // Gam_t[c][a] = (B' Z_t)[c][a]
    double w[RS * 64];            // w = w0 - E x0 per row slot
    double pa[RS * 64];           // predictor products dS_aff dZ_aff
    double rp[RS * 64];           // primal residual G u + s - w of the current iterate
    double dg[RS * 64];           // row weights of the current factorization
};

template <int N, int RS>
struct StageCtx {
    static constexpr int NV = 2 * N;
    const StageShared<N, RS>* sh;
    StageWave<N, RS>* wv;
    int lane;
    bool act, tail;
    bool rv[RS];

    // Lane-role indices are re-derived from an opaque copy of the lane id inside every
    // primitive: otherwise the compiler hoists the (loop-invariant) per-t LDS addresses
    // out of the IPM loop and keeps dozens of them live in VGPRs.
    __device__ __forceinline__ int olane() const {
        int l = lane;
        asm volatile("" : "+v"(l));
        return l;
    }
    __device__ __forceinline__ static int var_t(int l) { return l < NV ? (l >> 1) : N - 1; }

    // ---- Y = S v (into wv->Y) and (G v)_slot ---------------------------------------
    __device__ __forceinline__ void state_pred(double v) const {
        __builtin_amdgcn_wave_barrier();
        wv->bvec[lane] = v;
        __builtin_amdgcn_wave_barrier();
        const int L = olane();
        const int ap = L & 1;
        const int yk = L < 2 * N ? (L >> 1) + 1 : 1;
        const double2* v2 = reinterpret_cast<const double2*>(wv->bvec);
        double y0 = 0.0, y1 = 0.0, z0 = 0.0, z1 = 0.0;   // split chains
        const double* fbase = sh->fs + (N - yk) * 8 + ap * 4;   // q = t + N - yk: Phi_{yk-1-t}
#pragma unroll 4
        for (int t = 0; t < N; ++t) {
            const double2* ph = reinterpret_cast<const double2*>(fbase + t * 8);
            const double2 a = ph[0], b = ph[1];
            const double2 vv = v2[t];
            y0 = fma(a.x, vv.x, y0);
            z0 = fma(a.y, vv.y, z0);
            y1 = fma(b.x, vv.x, y1);
            z1 = fma(b.y, vv.y, z1);
        }
        if (L < 2 * N) reinterpret_cast<double2*>(wv->Y)[yk * 2 + ap] = make_double2(y0 + z0, y1 + z1);
        __builtin_amdgcn_wave_barrier();
    }
    __device__ __forceinline__ void rows_from_Y(double (&out)[RS]) const {
        const int L = olane();
        const int ystage = (L & 31) >= N ? N : (L & 31) + 1;
        const double2* Y2 = reinterpret_cast<const double2*>(wv->Y + ystage * 4);
        const double2 ya = Y2[0], yb = Y2[1];
#pragma unroll
        for (int s = 0; s < RS; ++s) {
            const double2 c01 = sh->cf01[s * 64 + L], c23 = sh->cf23[s * 64 + L];
            double acc = c01.x * ya.x;
            acc = fma(c01.y, ya.y, acc);
            acc = fma(c23.x, yb.x, acc);
            acc = fma(c23.y, yb.y, acc);
            out[s] = rv[s] ? acc : 0.0;
        }
    }
    __device__ __forceinline__ void gmul(double v, double (&out)[RS]) const {
        state_pred(v);
        rows_from_Y(out);
    }
    // (R_hat v)_lane with v in bvec
    __device__ __forceinline__ double rhat_bvec() const {
        const int L = olane();
        const int vc = L & 1;
        const double2 v = reinterpret_cast<const double2*>(wv->bvec)[var_t(L)];
        const double r0 = vc ? sh->R[2] : sh->R[0];
        const double r1 = vc ? sh->R[3] : sh->R[1];
        return act ? fma(r0, v.x, r1 * v.y) : 0.0;
    }

    // ---- per-stage sums of lane partials ----------------------------------------------
    // After the call, lanes L < N hold the sum over all lanes of stage L+1.
    template <int K>
    __device__ __forceinline__ void stage_reduce(double (&v)[K]) const {
#pragma unroll
        for (int e = 0; e < K; ++e) {
            double a, b;
            swap32_d(v[e], a, b);   // lanes L and L^32 hold rows of the same stage
            v[e] = a + b;
        }
        if (N < 32) {
#pragma unroll
            for (int e = 0; e < K; ++e) {
                const double t = half_reduce<OpSum>(tail ? v[e] : 0.0);
                v[e] += (lane == N - 1) ? t : 0.0;
            }
        }
    }
    // lam_k = sum_{r in k} y_r c_r  (+ Qbar_k Y_k when withH), into dst (LDS)
    __device__ __forceinline__ void build_lam(const double (&y)[RS], bool withH, double* dst) const {
        const int L = olane();
        double l[4] = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
        for (int s = 0; s < RS; ++s) {
            const double2 c01 = sh->cf01[s * 64 + L], c23 = sh->cf23[s * 64 + L];
            const double ys = rv[s] ? y[s] : 0.0;
            l[0] = fma(ys, c01.x, l[0]);
            l[1] = fma(ys, c01.y, l[1]);
            l[2] = fma(ys, c23.x, l[2]);
            l[3] = fma(ys, c23.y, l[3]);
        }
        stage_reduce<4>(l);
        if (withH) addQY(l);
        if (lane < N) {
            double2* d2 = reinterpret_cast<double2*>(dst + (lane + 1) * 4);
            d2[0] = make_double2(l[0], l[1]);
            d2[1] = make_double2(l[2], l[3]);
        }
        __builtin_amdgcn_wave_barrier();
    }
    // l += Qbar_k Y_k for lanes L < N (k = L+1)
    __device__ __forceinline__ void addQY(double (&l)[4]) const {
        const int L = olane();
        const int k = L < N ? L + 1 : 1;
        const double2* Y2 = reinterpret_cast<const double2*>(wv->Y + k * 4);
        const double2 ya = Y2[0], yb = Y2[1];
        const double* Qb = sh->qp[k == N ? 1 : 0];
#pragma unroll
        for (int a = 0; a < 4; ++a) {
            const double2 q01 = reinterpret_cast<const double2*>(Qb + a * 4)[0];
            const double2 q23 = reinterpret_cast<const double2*>(Qb + a * 4)[1];
            double acc = fma(q01.x, ya.x, l[a]);
            acc = fma(q01.y, ya.y, acc);
            acc = fma(q23.x, yb.x, acc);
            l[a] = fma(q23.y, yb.y, acc);
        }
    }
    // Qbar_k Y_k alone (residual H part), into lamH
    __device__ __forceinline__ void build_lamH() const {
        double l[4] = {0.0, 0.0, 0.0, 0.0};
        addQY(l);
        if (lane < N) {
            double2* d2 = reinterpret_cast<double2*>(wv->lamH + (lane + 1) * 4);
            d2[0] = make_double2(l[0], l[1]);
            d2[1] = make_double2(l[2], l[3]);
        }
        __builtin_amdgcn_wave_barrier();
    }
    // (S' lam)_lane
    __device__ __forceinline__ double adjoint(const double* lp) const {
        const int L = olane();
        const int vt = var_t(L), vc = L & 1;
        double g = 0.0, h = 0.0;   // two chains: shorter FMA dependency
        const double* fbase = sh->fa + (N - 1 - vt) * 8 + vc * 4;   // q = k-1 + N-1-vt: Phi_{k-1-vt}
#pragma unroll 4
        for (int k = 1; k <= N; ++k) {
            const double2* ph = reinterpret_cast<const double2*>(fbase + (k - 1) * 8);
            const double2 p0 = ph[0], p1 = ph[1];
            const double2* l2 = reinterpret_cast<const double2*>(lp + k * 4);
            const double2 l0 = l2[0], l1 = l2[1];
            g = fma(p0.x, l0.x, g);
            h = fma(p0.y, l0.y, h);
            g = fma(p1.x, l1.x, g);
            h = fma(p1.y, l1.y, h);
        }
        return act ? g + h : 0.0;
    }
    // two adjoints sharing the Phi gathers
    __device__ __forceinline__ void adjoint2(const double* lp, const double* lq, double& g1, double& g2) const {
        const int L = olane();
        const int vt = var_t(L), vc = L & 1;
        double a1 = 0.0, a2 = 0.0, b1 = 0.0, b2 = 0.0;
        const double* fbase = sh->fa + (N - 1 - vt) * 8 + vc * 4;
#pragma unroll 4
        for (int k = 1; k <= N; ++k) {
            const double2* ph = reinterpret_cast<const double2*>(fbase + (k - 1) * 8);
            const double2 p0 = ph[0], p1 = ph[1];
            const double2* l2 = reinterpret_cast<const double2*>(lp + k * 4);
            const double2* q2 = reinterpret_cast<const double2*>(lq + k * 4);
            const double2 l0 = l2[0], l1 = l2[1], q0 = q2[0], q1 = q2[1];
            a1 = fma(p0.x, l0.x, a1);
            b1 = fma(p0.y, l0.y, b1);
            a1 = fma(p1.x, l1.x, a1);
            b1 = fma(p1.y, l1.y, b1);
            a2 = fma(p0.x, q0.x, a2);
            b2 = fma(p0.y, q0.y, b2);
            a2 = fma(p1.x, q1.x, a2);
            b2 = fma(p1.y, q1.y, b2);
        }
        g1 = act ? a1 + b1 : 0.0;
        g2 = act ? a2 + b2 : 0.0;
    }

    // ---- normal matrix -----------------------------------------------------------------
    // M = R_hat + sum_k S_k'(Qbar_k + W_k)S_k + diag(dbox), column `lane` in registers;
    // row weights d in wv->dg.
    __device__ __forceinline__ void build_M(double (&M)[NV], double dbox) const {
        const int L = olane();
        // W partials of this lane's rows
        double wp[10];
#pragma unroll
        for (int e = 0; e < 10; ++e) wp[e] = 0.0;
#pragma unroll
        for (int s = 0; s < RS; ++s) {
            const double2 c01 = sh->cf01[s * 64 + L], c23 = sh->cf23[s * 64 + L];
            const double d = rv[s] ? wv->dg[s * 64 + L] : 0.0;
            const double c[4] = {c01.x, c01.y, c23.x, c23.y};
#pragma unroll
            for (int a = 0; a < 4; ++a) {
                const double ta = d * c[a];
#pragma unroll
                for (int b = a; b < 4; ++b) wp[sym10(a, b)] = fma(ta, c[b], wp[sym10(a, b)]);
            }
        }
        stage_reduce<10>(wp);
        if (lane < N) {
            double2* d2 = reinterpret_cast<double2*>(wv->Wf + (lane + 1) * 10);
#pragma unroll
            for (int e = 0; e < 5; ++e) d2[e] = make_double2(wp[2 * e], wp[2 * e + 1]);
        }
        __builtin_amdgcn_wave_barrier();
        // backward recursion on 16 lanes (entry (a,b) computed as (min,max): exactly symmetric)
        {
            const int e = L & 15;
            const int a0 = e >> 2, b0 = e & 3;
            const int a = a0 < b0 ? a0 : b0, b = a0 < b0 ? b0 : a0;
            const int wi = sym10(a, b);
            double Aa[4], Ab[4];
#pragma unroll
            for (int c = 0; c < 4; ++c) { Aa[c] = sh->A[c * 4 + a]; Ab[c] = sh->A[c * 4 + b]; }
            const double qv = sh->qp[0][a * 4 + b];
            double z = sh->qp[1][a * 4 + b] + wv->Wf[N * 10 + wi];
            if (lane < 16) wv->Z[(N - 1) * 16 + e] = z;
#pragma unroll 1
            for (int t = N - 2; t >= 0; --t) {
                __builtin_amdgcn_wave_barrier();
                const double2* z2 = reinterpret_cast<const double2*>(wv->Z + (t + 1) * 16);
                double acc = qv + wv->Wf[(t + 1) * 10 + wi];
#pragma unroll
                for (int c = 0; c < 4; ++c) {
                    const double2 zc0 = z2[2 * c], zc1 = z2[2 * c + 1];
                    double tc = zc0.x * Ab[0];
                    tc = fma(zc0.y, Ab[1], tc);
                    tc = fma(zc1.x, Ab[2], tc);
                    tc = fma(zc1.y, Ab[3], tc);
                    acc = fma(Aa[c], tc, acc);
                }
                if (lane < 16) wv->Z[t * 16 + e] = acc;
            }
        }
        __builtin_amdgcn_wave_barrier();
        // Gam_t[c][a] = sum_b B[b][c] Z_t[b][a]
#pragma unroll
        for (int j = 0; j < (N * 8 + 63) / 64; ++j) {
            const int e = j * 64 + L;
            if (e < N * 8) {
                const int t = e >> 3, c = (e >> 2) & 1, a = e & 3;
                double g = 0.0;
#pragma unroll
                for (int b = 0; b < 4; ++b) g = fma(sh->B[b * 2 + c], wv->Z[t * 16 + b * 4 + a], g);
                wv->Gam[e] = g;
            }
        }
        __builtin_amdgcn_wave_barrier();
        // column assembly
        const int vt = var_t(L), vc = L & 1;
        const double2* gs2 = reinterpret_cast<const double2*>(wv->Gam + vt * 8 + vc * 4);
        const double2 g01 = gs2[0], g23 = gs2[1];
        // diagonal 2x2 block: R[c'][c] plus the box barrier on the diagonal entry c' == c
        const double rr0 = (vc ? sh->R[1] : sh->R[0]) + (vc ? 0.0 : dbox);   // R[0][c]
        const double rr1 = (vc ? sh->R[3] : sh->R[2]) + (vc ? dbox : 0.0);   // R[1][c]
        const double* abase = sh->fa + (N - 1 - vt) * 8 + vc * 4;   // q = t + N-1-vt
        const double* bbase = sh->fb + (N - 1 - vt) * 8;
#pragma unroll
        for (int t = 0; t < N; ++t) {
            const int d = t - vt;
            const double2* pa2 = reinterpret_cast<const double2*>(abase + t * 8);   // Phi_d (d >= 0)
            const double2 fa0 = pa2[0], fa1 = pa2[1];
            const double2* pb2 = reinterpret_cast<const double2*>(bbase + t * 8);   // Phi_{-d} (d < 0)
            const double2 fb00 = pb2[0], fb01 = pb2[1], fb10 = pb2[2], fb11 = pb2[3];
            const double2* gt2 = reinterpret_cast<const double2*>(wv->Gam + t * 8);
            const double2 G00 = gt2[0], G01 = gt2[1], G10 = gt2[2], G11 = gt2[3];
            double m0 = G00.x * fa0.x;
            m0 = fma(G00.y, fa0.y, m0);
            m0 = fma(G01.x, fa1.x, m0);
            m0 = fma(G01.y, fa1.y, m0);
            m0 = fma(fb00.x, g01.x, m0);
            m0 = fma(fb00.y, g01.y, m0);
            m0 = fma(fb01.x, g23.x, m0);
            m0 = fma(fb01.y, g23.y, m0);
            double m1 = G10.x * fa0.x;
            m1 = fma(G10.y, fa0.y, m1);
            m1 = fma(G11.x, fa1.x, m1);
            m1 = fma(G11.y, fa1.y, m1);
            m1 = fma(fb10.x, g01.x, m1);
            m1 = fma(fb10.y, g01.y, m1);
            m1 = fma(fb11.x, g23.x, m1);
            m1 = fma(fb11.y, g23.y, m1);
            M[2 * t] = m0 + (d == 0 ? rr0 : 0.0);
            M[2 * t + 1] = m1 + (d == 0 ? rr1 : 0.0);
        }
    }
};

// Guarded square-root-free LDL' in the slot layout (M = L~ D L~', D = diag(d_k)), the
// UNSCALED column k broadcast through LDS: every lane publishes c_i = M_i[k] once, then
// reads c_j (j > k) with b128 broadcasts; lane i updates with t_i = c_i / d_k.  One
// reciprocal per step and no diagonal store (the solves use 1/d_i).  Result layout:
// lane i's slot j < i = L~[i][j]; slot j > i = d_i L~[j][i]; returns 1/d_lane.
template <int NV>
__device__ __forceinline__ double cholesky_lds(double (&M)[NV], int lane, double* col) {
    asm volatile("" : "+v"(lane));
    double invd = 1.0;
#pragma unroll
    for (int k = 0; k < NV; ++k) {
        double piv = readlane_d(M[k], k);
        if (!(piv > 0.0)) piv = 1e128;
        const double rp = frcp(piv);
        const bool below = lane > k && lane < NV;
        const double t = below ? M[k] * rp : 0.0;      // L~[lane][k]
        if (k + 1 < NV) {
            __builtin_amdgcn_wave_barrier();
            // lanes <= k write t (never read): the store, and with it the broadcast reads,
            // wait for the reciprocal, so the column is not held in registers meanwhile
            col[lane] = below ? M[k] : t;
            __builtin_amdgcn_wave_barrier();
#pragma unroll
            for (int j = k + 1; j < NV; ++j) M[j] = fma(-col[j], t, M[j]);
        }
        M[k] = below ? t : M[k];
        invd = (lane == k) ? rp : invd;
    }
    __builtin_amdgcn_wave_barrier();
    return invd;
}

// Cholesky with square roots, scaled column L[.][k] broadcast through LDS (same result
// layout as cholesky_lds: row part L~, column part d_i L~; returns 1/d_lane).
template <int NV>
__device__ __forceinline__ double cholesky_lds_sqrt(double (&M)[NV], int lane, double* col) {
    asm volatile("" : "+v"(lane));
    double inv_ii = 1.0;
#pragma unroll
    for (int k = 0; k < NV; ++k) {
        double piv = readlane_d(M[k], k);
        if (!(piv > 0.0)) piv = 1e128;
        const double inv = frsq(piv);
        const double lkk = piv * inv;
        const bool below = lane > k && lane < NV;
        const double l = below ? M[k] * inv : 0.0;     // L[lane][k]
        if (k + 1 < NV) {
            __builtin_amdgcn_wave_barrier();
            col[lane] = l;
            __builtin_amdgcn_wave_barrier();
#pragma unroll
            for (int j = k + 1; j < NV; ++j) M[j] = fma(-col[j], l, M[j]);
        }
        M[k] = (lane == k) ? lkk : (below ? l * inv : M[k]);
        inv_ii = (lane == k) ? inv : inv_ii;
    }
    __builtin_amdgcn_wave_barrier();
    return inv_ii * inv_ii;
}

// Same factorization with the column broadcast by v_readlane (kernel id 4, for A/B).
template <int NV>
__device__ __forceinline__ double cholesky(double (&M)[NV], int lane) {
    asm volatile("" : "+v"(lane));
    double inv_ii = 1.0;
#pragma unroll
    for (int k = 0; k < NV; ++k) {
        double piv = readlane_d(M[k], k);
        if (!(piv > 0.0)) piv = 1e128;
        const double inv = frsq(piv);
        const double lkk = piv * inv;
        const bool below = lane > k && lane < NV;
        const double l = below ? M[k] * inv : 0.0;
        const double lt = l * inv;
#pragma unroll
        for (int j = k + 1; j < NV; ++j) M[j] = fma(-readlane_d(M[j], k), lt, M[j]);
        M[k] = (lane == k) ? lkk : (below ? lt : M[k]);   // row part: L~ = L / l_kk
        inv_ii = (lane == k) ? inv : inv_ii;
    }
    return inv_ii * inv_ii;   // 1/d_lane, d = l^2
}

// Solve M x = b with M = L~ D^2 L~' (L~ unit lower, D = diag(l_kk)) in the slot layout:
// lane i's slot j < i holds L~[i][j], slot j > i holds l_ii L[j][i] = l_ii^2 L~[j][i], and
// inv2 = 1 / l_ii^2.  b per lane, lanes >= NV pass 0.
template <int NV>
__device__ __forceinline__ double chol_solve(const double (&M)[NV], double inv2, double b, int lane) {
    asm volatile("" : "+v"(lane));
#pragma unroll
    for (int k = 0; k < NV; ++k) {   // forward, unit diagonal: w = L~^{-1} b
        const double yk = readlane_d(b, k);
        const double upd = fma(M[k], -yk, b);
        b = (lane > k) ? upd : b;
    }
    const double v = b * inv2;       // D^{-2} w
    double acc = 0.0;                // sum_{j>i} slot_j x_j
#pragma unroll
    for (int k = NV - 1; k >= 0; --k) {   // backward: x_k = v_k - inv2_k acc_k
        const double xk = readlane_d(fma(-inv2, acc, v), k);
        const double upd = fma(M[k], xk, acc);
        acc = (lane < k) ? upd : acc;
    }
    return lane < NV ? fma(-inv2, acc, v) : 0.0;
}

}  // namespace

// kChol: 0 readlane broadcast, 1 LDS broadcast with square roots, 2 LDS square-root-free LDL'
template <int N, int RS, int kChol, int kWPB>
__global__ void __launch_bounds__(kWPB * 64) ipm_staged_kernel(DevProblem P, int64_t batch, const double* __restrict__ x0,
                                                         const double* __restrict__ xref, double* __restrict__ u_out,
                                                         int64_t ld_u, int32_t* __restrict__ status_out,
                                                         int32_t* __restrict__ iters_out, Settings S) {
    constexpr int NV = 2 * N;
    __shared__ __attribute__((aligned(16))) StageShared<N, RS> sh;
    __shared__ __attribute__((aligned(16))) StageWave<N, RS> wscr[kWPB];
    const int lane = threadIdx.x & 63;
    const int wave = threadIdx.x >> 6;
    for (int i = threadIdx.x; i < (2 * N - 1) * 8; i += blockDim.x) {
        const int q = i >> 3, e = i & 7;
        const int mf = q - (N - 1), mr = (N - 1) - q;   // P.phi_*: entry m+1 = Phi_m
        sh.fa[i] = mf >= 0 ? P.phi_ca[(mf + 1) * 8 + e] : 0.0;
        sh.fb[i] = mr > 0 ? P.phi_ca[(mr + 1) * 8 + e] : 0.0;
        sh.fs[i] = mr >= 0 ? P.phi_ac[(mr + 1) * 8 + e] : 0.0;
    }
    for (int i = threadIdx.x; i < RS * 64; i += blockDim.x) {
        sh.cf01[i] = make_double2(P.s_coef[i * 4 + 0], P.s_coef[i * 4 + 1]);
        sh.cf23[i] = make_double2(P.s_coef[i * 4 + 2], P.s_coef[i * 4 + 3]);
    }
    for (int i = threadIdx.x; i < 64; i += blockDim.x) {
        const bool bx = i < 2 * N && P.boxed;
        sh.lb[i] = bx ? P.lb[i] : -UNBOXED_BOUND;
        sh.ub[i] = bx ? P.ub[i] : UNBOXED_BOUND;
    }
    for (int i = threadIdx.x; i < 60; i += blockDim.x) {
        const double v = P.s_mats[i];   // Q 16, P 16, A 16, B 8, R 4
        if (i < 32) sh.qp[i >> 4][i & 15] = v;
        else if (i < 48) sh.A[i - 32] = v;
        else if (i < 56) sh.B[i - 48] = v;
        else sh.R[i - 56] = v;
    }
    __syncthreads();

    StageCtx<N, RS> W;
    W.sh = &sh;
    W.wv = &wscr[wave];
    W.lane = lane;
    W.act = lane < NV;
    W.tail = (lane & 31) >= N;
#pragma unroll
    for (int s = 0; s < RS; ++s) W.rv[s] = P.s_valid[s * 64 + lane] != 0;
    StageWave<N, RS>& wv = wscr[wave];
    const bool act = W.act;
    const bool boxact = act && P.boxed;
    const int li = act ? lane : 0;
    // lb / ub are re-read from LDS at every use (fewer live registers across the loops)
#define LB_ (sh.lb[lane])
#define UB_ (sh.ub[lane])
#define BNDABS_ fmax(fabs(LB_), fabs(UB_))
    const int p = P.p;
    const int m_rows = p + (P.boxed ? 2 * NV : 0);
    const double inv_m = 1.0 / (double)(m_rows > 0 ? m_rows : 1);

    // closed-loop runs solve only their live instances: slot -> row through S.index, count on device
    const int64_t nlive = S.count ? (int64_t)*S.count : batch;
    const int64_t stride = (int64_t)gridDim.x * kWPB;
    for (int64_t slot = S.claim ? wave_claim(S.claim) : (int64_t)blockIdx.x * kWPB + wave; slot < nlive;
         slot = S.claim ? wave_claim(S.claim) : slot + stride) {
        const int64_t inst = S.index ? (int64_t)S.index[slot] : slot;
        double xv[NX], xr[NX];
#pragma unroll
        for (int k = 0; k < NX; ++k) {
            xv[k] = x0[inst * NX + k];
            xr[k] = xref ? xref[inst * NX + k] : P.goal[k];
        }
        const double dd = S.dist ? S.dist[inst] : 0.0;   // disturbance estimate (w -= Ed d)
        bool bad = false;
        for (int r = lane; r < P.npre; r += 64) {
            double v = P.pre_w0[r];
#pragma unroll
            for (int k = 0; k < NX; ++k) v -= P.pre_E[r * NX + k] * xv[k];
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
        double q = 0.0;
        if (act) {
#pragma unroll
            for (int k = 0; k < NX; ++k) q += P.hq[li * NX + k] * (xv[k] - xr[k]);
        }
        double bn = boxact ? BNDABS_ : 0.0;
#pragma unroll
        for (int s = 0; s < RS; ++s) {
            double v = 0.0;
            if (W.rv[s]) {
                const int e = s * 64 + lane;
                v = P.s_w0[e];
#pragma unroll
                for (int k = 0; k < NX; ++k) v -= P.s_E[e * NX + k] * xv[k];
                if (P.s_Ed) v -= P.s_Ed[e] * dd;
            }
            wv.w[s * 64 + lane] = v;
            bn = fmax(bn, fabs(v));
        }
        double u = boxact ? fmin(fmax(0.0, LB_), UB_) : 0.0;
        double su = boxact ? fmax(UB_ - u, 1.0) : 1.0;
        double sl = boxact ? fmax(u - LB_, 1.0) : 1.0;
        double zu = boxact ? 1.0 : 0.0, zl = zu;
        double s_[RS], z_[RS];
        {
            double gu[RS];
            W.gmul(act ? u : 0.0, gu);
#pragma unroll
            for (int s = 0; s < RS; ++s) {
                s_[s] = W.rv[s] ? fmax(wv.w[s * 64 + lane] - gu[s], 1.0) : 1.0;
                z_[s] = W.rv[s] ? 1.0 : 0.0;
            }
        }
        const double bnorm = 1.0 + wave_max(bn);
        const double qnorm = 1.0 + wave_max(act ? fabs(q) : 0.0);

        int status = CARMPC_MAX_ITER;
        int it = 0;
        bool polish_failed = false;
        double M[NV];
        PT_DECL
        for (;;) {
            double gtz, rd, rpu, rpl, mu;
            bool res_ok;
            {
                double gu[RS];
                W.gmul(act ? u : 0.0, gu);
                const double ru = W.rhat_bvec();
                W.build_lam(z_, false, wv.lam);
                W.build_lamH();
                double hs;
                W.adjoint2(wv.lam, wv.lamH, gtz, hs);
                const double hu = hs + ru;
                double rpn = 0.0, musum = 0.0, gun = 0.0;
#pragma unroll
                for (int s = 0; s < RS; ++s) {
                    const double rps = W.rv[s] ? gu[s] + s_[s] - wv.w[s * 64 + lane] : 0.0;
                    wv.rp[s * 64 + lane] = rps;
                    rpn = fmax(rpn, fabs(rps));
                    gun = fmax(gun, fabs(gu[s]));
                    musum += s_[s] * z_[s];
                }
                rpu = boxact ? u + su - UB_ : 0.0;
                rpl = boxact ? -u + sl + LB_ : 0.0;
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
            PT_MARK(0);
            const bool last = it >= S.max_iter;
            const bool polish = !polish_failed && ((res_ok && mu <= POLISH_MU) || last);
            if (!polish) {
                if (last) break;
                if (res_ok && mu <= S.tol_mu) { status = CARMPC_OPTIMAL; break; }
                if (p > 0) {
                    double wz = 0.0, wzabs = 0.0;
#pragma unroll
                    for (int s = 0; s < RS; ++s) {
                        const double wsv = wv.w[s * 64 + lane];
                        wz += wsv * z_[s];
                        wzabs += fabs(wsv) * z_[s];
                    }
                    const double lo = act ? fmin(gtz * LB_, gtz * UB_) : 0.0;
                    const double sc = act ? fabs(gtz) * BNDABS_ : 0.0;
                    const double lo_w = wave_sum(lo), wz_w = wave_sum(wz), sc_w = wave_sum(sc + wzabs);
                    if (lo_w - wz_w > 1e-12 * sc_w) { status = CARMPC_PRIMAL_INFEASIBLE; break; }
                }
            }
            const double id = 1.0 / POLISH_DELTA;
            const double dbu = (polish && boxact && su < zu) ? id : 0.0;
            const double dbl = (polish && boxact && sl < zl) ? id : 0.0;
#pragma unroll
            for (int s = 0; s < RS; ++s)
                wv.dg[s * 64 + lane] = !W.rv[s] ? 0.0 : (polish ? (s_[s] < z_[s] ? id : 0.0) : z_[s] * frcp(s_[s]));
            __builtin_amdgcn_wave_barrier();
            PT_MARK(1);
            W.build_M(M, polish ? dbu + dbl : (boxact ? zu * frcp(su) + zl * frcp(sl) : 0.0));
            PT_MARK(2);
            const double inv2 = kChol == 2   ? cholesky_lds<NV>(M, lane, wv.bvec)
                                 : kChol == 1 ? cholesky_lds_sqrt<NV>(M, lane, wv.bvec)
                                              : cholesky<NV>(M, lane);
            PT_MARK(3);
            // row temporaries: ra = dS | y_g ; rb = dZ | ry_g ; (LDS) pa = dS_aff dZ_aff
            double ra[RS], rb[RS];
#pragma unroll
            for (int s = 0; s < RS; ++s) { ra[s] = 0.0; rb[s] = 0.0; }
            double v0 = 0.0, v1 = 0.0, v2 = 0.0, v3 = 0.0, v4 = 0.0, pua = 0.0, pla = 0.0, sigma_mu = 0.0;
            const int nsolve = polish ? POLISH_REFINE + 1 : (mu <= REFINE_MU ? 3 : 2);   // refinement late only
#pragma unroll 1
            for (int k = 0; k < nsolve; ++k) {
                double rhs, ryu = 0.0, ryl = 0.0;
                if (polish) {
                    double gx[RS], t[RS];
                    W.gmul(act ? v0 : 0.0, gx);
                    const double rx = W.rhat_bvec();
#pragma unroll
                    for (int s = 0; s < RS; ++s) {
                        const double dgs = wv.dg[s * 64 + lane];
                        rb[s] = dgs != 0.0 ? wv.w[s * 64 + lane] - gx[s] : 0.0;
                        t[s] = ra[s] - dgs * rb[s];
                    }
                    W.build_lam(t, true, wv.lam);
                    const double hg = W.adjoint(wv.lam);
                    ryu = dbu != 0.0 ? UB_ - v0 : 0.0;
                    ryl = dbl != 0.0 ? -LB_ + v0 : 0.0;
                    rhs = act ? -q - (hg + rx) - v1 + v2 + dbu * ryu - dbl * ryl : 0.0;
                } else if (k < 2) {
                    double t[RS];
#pragma unroll
                    for (int s = 0; s < RS; ++s) {
                        const double rc = s_[s] * z_[s] + (k == 1 ? wv.pa[s * 64 + lane] : 0.0) -
                                          (k == 1 && W.rv[s] ? sigma_mu : 0.0);
                        t[s] = W.rv[s] ? (rc - z_[s] * wv.rp[s * 64 + lane]) * frcp(s_[s]) : 0.0;
                    }
                    const double rcu = !boxact ? 0.0 : su * zu + pua - (k == 1 ? sigma_mu : 0.0);
                    const double rcl = !boxact ? 0.0 : sl * zl + pla - (k == 1 ? sigma_mu : 0.0);
                    W.build_lam(t, false, wv.lam);
                    const double gtt = W.adjoint(wv.lam);
                    rhs = act ? -rd + gtt + (boxact ? (rcu - zu * rpu) * frcp(su) - (rcl - zl * rpl) * frcp(sl) : 0.0) : 0.0;
                } else {
                    // refinement of the corrector: e = H du + G'dZ + rd + box.  Y(du) and du
                    // are still in wv.Y / wv.bvec from the gmul that followed solve 1.
                    const double rdu = W.rhat_bvec();
                    W.build_lam(rb, true, wv.lam);
                    const double hg = W.adjoint(wv.lam);
                    rhs = act ? -(hg + rdu + rd + (boxact ? v3 - v4 : 0.0)) : 0.0;
                }
                PT_MARK(4);
                const double sol = chol_solve<NV>(M, inv2, rhs, lane);
                PT_MARK(5);
                double gs[RS];
                W.gmul(sol, gs);
                if (polish) {
#pragma unroll
                    for (int s = 0; s < RS; ++s) ra[s] += wv.dg[s * 64 + lane] * (gs[s] - rb[s]);
                    v1 += dbu * (sol - ryu);
                    v2 += dbl * (-sol - ryl);
                    v0 += sol;
                } else if (k < 2) {
                    v0 = sol;
#pragma unroll
                    for (int s = 0; s < RS; ++s) {
                        const double rc = s_[s] * z_[s] + (k == 1 ? wv.pa[s * 64 + lane] : 0.0) -
                                          (k == 1 && W.rv[s] ? sigma_mu : 0.0);
                        ra[s] = W.rv[s] ? -wv.rp[s * 64 + lane] - gs[s] : 0.0;
                        rb[s] = W.rv[s] ? (-rc - z_[s] * ra[s]) * frcp(s_[s]) : 0.0;
                    }
                    const double rcu = !boxact ? 0.0 : su * zu + pua - (k == 1 ? sigma_mu : 0.0);
                    const double rcl = !boxact ? 0.0 : sl * zl + pla - (k == 1 ? sigma_mu : 0.0);
                    v1 = boxact ? -rpu - sol : 0.0;
                    v2 = boxact ? -rpl + sol : 0.0;
                    v3 = boxact ? (-rcu - zu * v1) * frcp(su) : 0.0;
                    v4 = boxact ? (-rcl - zl * v2) * frcp(sl) : 0.0;
                    if (k == 0) {
                        double amax = fmin(fmin(ratio(su, v1), ratio(zu, v3)), fmin(ratio(sl, v2), ratio(zl, v4)));
#pragma unroll
                        for (int s = 0; s < RS; ++s) amax = fmin(amax, fmin(ratio(s_[s], ra[s]), ratio(z_[s], rb[s])));
                        const double a = fmin(1.0, wave_min(amax));
                        double mua = boxact ? (su + a * v1) * (zu + a * v3) + (sl + a * v2) * (zl + a * v4) : 0.0;
#pragma unroll
                        for (int s = 0; s < RS; ++s) {
                            mua += (s_[s] + a * ra[s]) * (z_[s] + a * rb[s]);
                            wv.pa[s * 64 + lane] = ra[s] * rb[s];
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
                        rb[s] += W.rv[s] ? z_[s] * gs[s] * frcp(s_[s]) : 0.0;
                    }
                    v0 += sol;
                    if (boxact) {
                        v1 -= sol; v3 += zu * sol * frcp(su);
                        v2 += sol; v4 -= zl * sol * frcp(sl);
                    }
                }
            }
            PT_MARK(6);
            if (polish) {
                double gx[RS];
                W.gmul(act ? v0 : 0.0, gx);
                double viol = boxact ? fmax(v0 - UB_, LB_ - v0) : -INFINITY;
                double wsc = boxact ? BNDABS_ : 0.0, ysc = fmax(fabs(v1), fabs(v2)), ymin = fmin(v1, v2);
                // active opposite pairs form an equality: exempt from the sign test (oracle/qp.py)
                bool paired[RS];
#pragma unroll
                for (int s = 0; s < RS; ++s) paired[s] = false;
                if (P.s_partner) {
                    __builtin_amdgcn_wave_barrier();
#pragma unroll
                    for (int s = 0; s < RS; ++s)
                        wv.pa[s * 64 + lane] = (W.rv[s] && wv.dg[s * 64 + lane] != 0.0) ? ra[s] : NAN;
                    __builtin_amdgcn_wave_barrier();
#pragma unroll
                    for (int s = 0; s < RS; ++s) {
                        const int pr = W.rv[s] ? P.s_partner[s * 64 + lane] : -1;
                        paired[s] = pr >= 0 && wv.dg[s * 64 + lane] != 0.0 && !isnan(wv.pa[pr]);
                    }
                }
#pragma unroll
                for (int s = 0; s < RS; ++s) {
                    if (W.rv[s]) {
                        const double wsv = wv.w[s * 64 + lane];
                        viol = fmax(viol, gx[s] - wsv);
                        wsc = fmax(wsc, fabs(wsv));
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
            PT_MARK(7);
        }
        PT_MARK(7);
        PT_FLUSH();
        if (lane < P.n) u_out[inst * ld_u + lane] = u;
        if (lane == 0) {
            status_out[inst] = status;
            if (iters_out) iters_out[inst] = it;
        }
    }
}

#undef LB_
#undef UB_
#undef BNDABS_

// ---------------------------------------------------------------------------
// Host-side dispatch
// ---------------------------------------------------------------------------
namespace {
#ifndef CARMPC_STAGED_NS
#define CARMPC_STAGED_NS 10, 20
#endif
constexpr int kStagedNs[] = {CARMPC_STAGED_NS};

template <int N, int RS, int kChol, int kWPB>
hipError_t launch_t(const DevProblem& P, int64_t batch, const double* x0, const double* xref, double* u_out,
                    int64_t ld_u, int32_t* status, int32_t* iters, const Settings& s, hipStream_t stream) {
    auto kern = ipm_staged_kernel<N, RS, kChol, kWPB>;
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

template <int N>
hipError_t launch_rs(const DevProblem& P, int64_t batch, const double* x0, const double* xref, double* u_out,
                     int64_t ld_u, int32_t* status, int32_t* iters, const Settings& s, hipStream_t stream) {
    // default (2): LDS-broadcast Cholesky with square roots, 8 waves per workgroup (fastest
    // measured).  The variants it was measured against -- 4 readlane-broadcast Cholesky, 5 four
    // waves per workgroup (one wave per SIMD, 512 registers), 6 square-root-free LDL' -- are
    // only instantiated in experiment builds (-DCARMPC_AB_KERNELS); the product library rejects
    // settings.kernel 4..6 (launch_staged).
#define CARMPC_RS_SWITCH(LDS, WPB)                                                                    \
    switch (P.srs) {                                                                                  \
        case 1: return launch_t<N, 1, LDS, WPB>(P, batch, x0, xref, u_out, ld_u, status, iters, s, stream); \
        case 2: return launch_t<N, 2, LDS, WPB>(P, batch, x0, xref, u_out, ld_u, status, iters, s, stream); \
        case 3: return launch_t<N, 3, LDS, WPB>(P, batch, x0, xref, u_out, ld_u, status, iters, s, stream); \
        case 4: return launch_t<N, 4, LDS, WPB>(P, batch, x0, xref, u_out, ld_u, status, iters, s, stream); \
        default: return hipErrorInvalidValue;                                                         \
    }
#ifdef CARMPC_AB_KERNELS
    if (s.kernel == 4) { CARMPC_RS_SWITCH(0, 8) }
    if (s.kernel == 5) { CARMPC_RS_SWITCH(1, 4) }
    if (s.kernel == 6) { CARMPC_RS_SWITCH(2, 8) }
#endif
    CARMPC_RS_SWITCH(1, 8)
#undef CARMPC_RS_SWITCH
}
}  // namespace

bool staged_supported_N(int N) {
    for (int v : kStagedNs)
        if (v == N) return true;
    return false;
}

hipError_t launch_staged(const DevProblem& P, int64_t batch, const double* x0, const double* xref, double* u_out,
                         int64_t ld_u, int32_t* status, int32_t* iters, const Settings& s, hipStream_t stream,
                         int* unsupported) {
    *unsupported = 0;
    if (batch <= 0) return hipSuccess;
    if (!P.staged || P.srs < 1 || P.srs > kStagedMaxRS) {
        *unsupported = 1;
        return hipErrorInvalidValue;
    }
#ifndef CARMPC_AB_KERNELS
    if (s.kernel >= 4 && s.kernel <= 6) {
        *unsupported = 1;
        return hipErrorInvalidValue;
    }
#endif
    switch (P.N) {
        case 10: return launch_rs<10>(P, batch, x0, xref, u_out, ld_u, status, iters, s, stream);
        case 20: return launch_rs<20>(P, batch, x0, xref, u_out, ld_u, status, iters, s, stream);
        default: *unsupported = 1; return hipErrorInvalidValue;
    }
}

}  // namespace carmpc

#ifdef CARMPC_PHASE_TIMING
// Profiling build only: read (and optionally reset) the per-phase cycle counters.
extern "C" int carmpc_debug_phase_cycles(unsigned long long* out8, int reset) {
    if (hipMemcpyFromSymbol(out8, HIP_SYMBOL(carmpc_phase_cycles), sizeof(unsigned long long) * 8) != hipSuccess)
        return -1;
    if (reset) {
        const unsigned long long z[8] = {0, 0, 0, 0, 0, 0, 0, 0};
        if (hipMemcpyToSymbol(HIP_SYMBOL(carmpc_phase_cycles), z, sizeof(z)) != hipSuccess) return -1;
    }
    return 0;
}
#endif
