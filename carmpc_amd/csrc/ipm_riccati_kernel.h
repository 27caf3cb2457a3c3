#pragma once
// ipm_riccati_kernel.h -- grouped stage-form Mehrotra IPM: 16 lanes per QP, 4 QPs per wavefront.
//
// Replaces the per-step cvxpy solve of lib/mpc.py:334-335 / 477-478 with a Mehrotra
// predictor-corrector IPM (restated on the CPU in oracle/qp.py::ipm), applying M^{-1} by a backward
// Riccati recursion and a forward roll-out over the horizon (oracle/riccati.py, the CPU restatement
// this kernel follows line by line).  Every QP row acts on one predicted state x_k (mpc.py:196-253),
// and H = R_hat + S'Q_hat S (matrix_gen.py:35-72), so
//     M = H + G'DG + diag(box) = R_hat + diag(Db) + sum_k S_k'(Qbar_k + W_k) S_k.
//
// Layout (one QP per 16-lane DPP row; group g = lane>>4, j = lane&15):
//   * row state in registers: lane j owns stage j+1 (segment 0) and j+17 (segment 1) -- the
//     rows of those stages sit in its 2 x 8 slots; stage-N rows that do not fit the owner
//     go to the segments whose stage number exceeds N (capi.hip::riccati_layout);
//     the owner of stage t+1 also owns the input u_t (both components) and its box rows (LDS);
//   * stage recursions (adjoints, Riccati factorization, backward/forward solves) exchange
//     per-stage records in LDS (W_k, rhs, factor K_t / Re_t, y_k, v_t) with the row phases.
//     Shared-model problems run them on the matrix cores, one 4x4 matrix entry per lane (see
//     "stage recursions on the matrix cores" below); per-instance models (HET) run them as scalar
//     code repeated in the 16 lanes of the group;
//   * per-QP reductions are 16-lane DPP butterflies (lanes.h), bitwise row-uniform.
// The 4 groups of a wave advance trip by trip together (one trip = one IPM iteration or one
// polish); a group that finishes an instance claims its next one from an atomic counter at once.
// Large solves run as three launches of this kernel (MODE, launch pipeline at the end of the file).
#include "carmpc_internal.h"
#include "lanes.h"

#include <algorithm>
#include <cstdlib>
#include <type_traits>

#include <hip/hip_runtime.h>
#include <math.h>

// Optional per-phase cycle accounting (profiling build only: -DCARMPC_PHASE_TIMING,
// tools/ric_timing.py): 0 init, 1 residual rows, 2 adjoint pass, 3 decisions, 4 factor rows,
// 5 factorization pass, 6 backward passes, 7 forward passes, 8-10 row phases k = 0..2,
// 11 polish rows.
#ifdef CARMPC_PHASE_TIMING
// (one accumulator per translation unit that instantiates the kernel; RIC_TIMING_READER defines its reader)
static __device__ unsigned long long carmpc_ric_cycles[12];
#define RIC_TIMING_READER(NAME)                                                                                  \
    extern "C" int carmpc_debug_ric_cycles_##NAME(unsigned long long* out12, int reset) {                         \
        if (hipMemcpyFromSymbol(out12, HIP_SYMBOL(carmpc_ric_cycles), sizeof(unsigned long long) * 12) != hipSuccess) \
            return -1;                                                                                           \
        if (reset) {                                                                                             \
            const unsigned long long z[12] = {};                                                                 \
            if (hipMemcpyToSymbol(HIP_SYMBOL(carmpc_ric_cycles), z, sizeof(z)) != hipSuccess) return -1;         \
        }                                                                                                        \
        return 0;                                                                                                \
    }
#define RT_DECL                                                        \
    unsigned long long rt_acc[12] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0}; \
    unsigned long long rt_t = clock64();
#define RT_MARK(i)                               \
    do {                                         \
        const unsigned long long n_ = clock64(); \
        rt_acc[i] += n_ - rt_t;                  \
        rt_t = n_;                               \
    } while (0)
#define RT_FLUSH()                                                                           \
    do {                                                                                     \
        if (lane == 0)                                                                       \
            for (int i_ = 0; i_ < 12; ++i_) atomicAdd(&carmpc_ric_cycles[i_], rt_acc[i_]); \
    } while (0)
#else
#define RIC_TIMING_READER(NAME)
#define RT_DECL
#define RT_MARK(i) do {} while (0)
#define RT_FLUSH() do {} while (0)
#endif

// Unroll factor of the scalar stage loops (per-instance models and the initial roll-out; forward,
// backward, factorization, adjoint): > 1 lets the compiler rename the one-stage-ahead prefetch
// registers instead of copying them every stage.  Measured when the shared-model kernels still ran
// these loops (1 GPU, QP/s) for unroll 1 / 2 / 4 / 5 / 10: 7.05M / 7.52M / 7.73M / 7.80M / 7.76M.
#ifndef CARMPC_RIC_UNROLL
#define CARMPC_RIC_UNROLL 5
#endif
#ifndef CARMPC_RIC_UNROLL_ADJ
#define CARMPC_RIC_UNROLL_ADJ 5
#endif
// Scalar stage loops: all 16 lanes of a group hold bitwise-identical values (redundant
// recursions), and every lane stores them (same address, same bits) -- no exec-mask branch
// per stage.  Lane-0-only stores (CARMPC_RIC_LANE0_WRITE) measured 7.81M vs 8.05M QP/s.
#ifdef CARMPC_RIC_LANE0_WRITE
#define RIC_WRITER (j == 0)
#else
#define RIC_WRITER true
#endif
// Stages of read-ahead of the matrix-core passes (see the comment at kPre).
#ifndef CARMPC_RIC_FACTOR_SPLIT   // 1: with two QPs per wave, blocks 2 and 3 take the vector half of the factorization
#define CARMPC_RIC_FACTOR_SPLIT 1
#endif
#ifndef CARMPC_RIC_KPRE
#define CARMPC_RIC_KPRE 1
#endif
// Scheduling barrier after every k-th row slot of the slot loops (0: none): bounds the live set of the loop.
#ifndef CARMPC_RIC_SLOT_FENCE
#define CARMPC_RIC_SLOT_FENCE 1
#endif
#ifndef CARMPC_HET_LEGACY
#define CARMPC_HET_LEGACY 0
#endif
#ifndef CARMPC_RIC_UNROLL_HET   // per-instance (HET) variant, both loop kinds: its A, B in registers
                                // leave no room to unroll (hetero_bench 7.1M QP/s rolled, 6.4M at 5)
#define CARMPC_RIC_UNROLL_HET 1
#endif

namespace carmpc {

namespace ric {

using namespace lanes;

constexpr int G16 = kRicLanes;
constexpr int RSEG = kRicSeg;
constexpr int RS = kRicSlots;
// Doubles per stage record: 20 fields; two more of padding where the LDS has room for them (ric_rec below), which
// spreads the records of consecutive stages -- one per lane in the row phases -- over all banks.
constexpr int kRecFields = 20;
// record t (stage t+1, input t):
//   [0..9]   W_{t+1} (packed) | lamZ_{t+1} [0..3], lamH_{t+1} [4..7] | factor: K_t [0..7], il00 l10 il11 [8..10]
//   [12..15] b^x_{t+1} | y_{t+1} | gz_t [12..13], hs_t [14..15]
//   [16..17] b^u_t | v_t
//   [18..19] Db_t | kappa_t
constexpr int O_K = 0, O_CH = 8, O_ZERO = 11, O_BX = 12, O_BU = 16, O_DB = 18;

// The polish is attempted once mu <= POLISH_MU with both residuals within POLISH_RES (relative, like the
// termination tolerance): far earlier than the IPM would terminate.  An accepted polish is the exact
// optimum whenever it comes, so the gate only trades iterations saved (about 3 per instance against the
// conservative gate mu <= 1e-6, residuals within the termination tolerance) for more rejected attempts,
// most of which the correction round repairs (measured with the conservative first active set below: gates
// from 5e-5 / 3e-6 to 2e-2 / 3e-4, best from 5e-3 / 1e-4 on; beyond 2e-2 the retry launch outgrows the
// gain).  Overridable for such sweeps (tools/gpu/mkvar.sh).
// The per-instance kernels keep the conservative gate, like the fallback kernels.
#ifndef CARMPC_POLISH_MU
#define CARMPC_POLISH_MU 1e-2
#endif
#ifndef CARMPC_POLISH_RES
#define CARMPC_POLISH_RES 2e-4
#endif
constexpr double POLISH_MU = CARMPC_POLISH_MU, POLISH_RES = CARMPC_POLISH_RES;
constexpr double POLISH_MU_CONSERVATIVE = 1e-6;
// First active set of a polish: the rows with s < POLISH_ACT z.  A conservative guess (few rows active, the
// correction round adds the violated ones) is accepted far more often than s < z: 76 % instead of 50 % at
// this gate, and 1.7 % instead of 13 % rejected after the correction (swept 0.001..30 for several gates).
#ifndef CARMPC_POLISH_ACT
#define CARMPC_POLISH_ACT 0.003
#endif
constexpr double POLISH_ACT = CARMPC_POLISH_ACT;
// Initial point: slacks s = max(w - G u0, INIT_SFLOOR), multipliers on the central path z = mu0 / s with
// mu0 = clamp((|q|_inf / (INIT_Q_PER_VAR n))^2, INIT_MU_MIN, INIT_MU0): a centred start whose distance from the
// boundary follows the size of the linear term.  States far from the goal (large q, many active rows at the
// optimum) start well inside the cone -- about 1.3 iterations fewer than z = 1 with the floor at 1 on the
// bench's states --, states on closed-loop trajectories and near the goal (little or nothing active) start
// close to the boundary and keep their 3 to 4 iterations, where a fixed mu0 = 100 costs them 5 (measured:
// linear and quadratic rules; the best scale is 100..200 at N = 20, 50..70 at N = 10, about 35 at N = 5, hence
// proportional to the number of variables).  INIT_MU0 = 0 means z = 1 (the per-instance kernels, like the
// fallback kernels).
#ifndef CARMPC_INIT_MU0
#define CARMPC_INIT_MU0 100.0
#endif
#ifndef CARMPC_INIT_MU_MIN
#define CARMPC_INIT_MU_MIN 1.0
#endif
#ifndef CARMPC_INIT_Q_PER_VAR
#define CARMPC_INIT_Q_PER_VAR 3.5
#endif
#ifndef CARMPC_INIT_SFLOOR
#define CARMPC_INIT_SFLOOR 2.0
#endif
constexpr double POLISH_DELTA = 1e-10;
constexpr int POLISH_REFINE = 2;            // refinement passes of the polish solve (2: |u - u*| ~ 1e-10, same acceptances as 3)
constexpr int POLISH_REFINE_CONSERVATIVE = 3;   // ... of the per-instance kernels, like the fallback kernels
constexpr double POLISH_TOL = 1e-11;

// Slot table of a problem: kTab = 256 entries, entry (sg * 8 + i) * 16 + j16 = slot i of segment sg of
// table lane j16 (capi.hip::riccati_layout).  With 16 lanes per QP a lane holds both segments of its table
// lane (16 slots); with 32 lanes per QP lane l holds segment l >> 4 of table lane l & 15 (8 slots).
constexpr int kTab = RS * G16;
template <int N>
struct RicShared {
    double2 cf01[kTab];   // c~0, c~1
    double2 cf23[kTab];   // c~2, c~3
    int16_t partner[kTab];
    double lb[2 * N], ub[2 * N];
};
// per-input state of the owned inputs: 12 fields x 2 components per input pair t (row t; row N: dummy row
// written by lanes whose segment owns no input)
enum { F_U = 0, F_Q, F_SU, F_SL, F_ZU, F_ZL, F_RD, F_E1, F_E2, F_E3, F_E4, F_VX, F_COUNT };
// REC_ doubles per stage record, QS_ doubles between the records of two groups (see ric_rec, ric_qstride)
template <int N, int LPQ, int SEGS, int REC_, int QS_>
struct RicWaveT {
    static constexpr int NG = 64 / LPQ, SL = SEGS * kRicSeg;   // groups per wave, slots per lane
    // stage records of the groups; the polish verification scratch [SL][64] aliases them
    double recbuf[NG * QS_ > SL * 64 ? NG * QS_ : SL * 64];
    double w[SL][64];         // w = w0 - E x0 per (slot, lane)
    // Field-major: the N + 1 rows of one field are contiguous (16 bytes per row), so the lanes of a group -- lane l on
    // row l -- read and write consecutive 16-byte slots, one per bank group.  (Row-major rows of 192 bytes put lanes
    // l, l + 4, l + 8, ... on the same banks: five-way conflicts on every access.)
    double vbox[NG][F_COUNT][N + 1][2];
};
// LDS banking of the stage records (64 banks of 4 bytes for 8- and 16-byte reads, 32 for stores; a 16-byte access is
// served in groups of 8 or 16 lanes).  In the row phases lane l works on record l: at 20 doubles per record lanes
// l, l + 8, l + 16 share banks; 22 doubles put the 16-byte slots of 16 consecutive records on 16 different bank
// groups.  In the matrix-core passes the blocks of two QPs access the same fields of their records at once: the
// distance between the two QPs' records decides whether those meet on a bank.  Two QPs per wave: the distance in
// dwords is kept at 16..24 or 40..48 modulo 64 (reads: 14 banks per QP) and away from 0 modulo 32 (stores).
constexpr int ric_qstride(int N, int rec, int ng) {
    if (ng != 2) return N * rec;
    for (int pad = 0; pad < 32; pad += 2) {
        const int d = 2 * (N * rec + pad);
        if ((d % 64 >= 16 && d % 64 <= 24) || (d % 64 >= 40 && d % 64 <= 48)) return N * rec + pad;
    }
    return N * rec;
}
constexpr int ric_waves_wanted(int SEGS) { return 8 / SEGS; }
template <int N, int LPQ, int SEGS, int REC_>
constexpr size_t ric_lds_bytes(int waves) {
    return sizeof(RicShared<N>) + 16 + (size_t)waves * sizeof(RicWaveT<N, LPQ, SEGS, REC_, ric_qstride(N, REC_, 64 / LPQ)>);
}
// waves per workgroup: as many as a CU's LDS (160 KB) holds, up to eight with one slot segment per lane and four with two
template <int N, int LPQ, int SEGS, int REC_>
constexpr int ric_wpb_rec() {
    int w = ric_waves_wanted(SEGS);
    while (w > 1 && ric_lds_bytes<N, LPQ, SEGS, REC_>(w) > 160u * 1024u) --w;
    return w;
}
// the padded record where it costs no wave
template <int N, int LPQ, int SEGS>
constexpr int ric_rec() {
    return (64 / LPQ == 2 && ric_wpb_rec<N, LPQ, SEGS, kRecFields + 2>() == ric_wpb_rec<N, LPQ, SEGS, kRecFields>()) ? kRecFields + 2 : kRecFields;
}
template <int N, int LPQ, int SEGS = 32 / LPQ>
using RicWave = RicWaveT<N, LPQ, SEGS, ric_rec<N, LPQ, SEGS>(), ric_qstride(N, ric_rec<N, LPQ, SEGS>(), 64 / LPQ)>;

__device__ __forceinline__ void wb() { __builtin_amdgcn_wave_barrier(); }

// Compile-time sparsity of the stage matrices: entries outside a mask are exactly zero and,
// with AUNIT, diag(A) == 1 exactly (verified on the host, capi.hip::riccati_layout), so the
// unrolled products skip them.  DenseModel is the general fallback.
constexpr unsigned bit4(int a, int b) { return 1u << (a * 4 + b); }
constexpr unsigned bit2(int a, int b) { return 1u << (a * 2 + b); }
struct DenseModel {
    static constexpr unsigned A = 0xFFFFu, B = 0xFFu, Q = 0xFFFFu, R = 0xFu;
    static constexpr bool AUNIT = false;
};
// kinematic bicycle linearised and discretised as in mpc.py:128-180: A = I + dt A_lin with
// A_lin nonzero only in rows 0-1 (columns 2-3) and entry (2,3); B = dt B_lin with B_lin[2][1],
// B_lin[3][0]; Q, R diagonal (configuration.py:19-21).
struct BicycleModel {
    static constexpr unsigned A = bit4(0, 0) | bit4(0, 2) | bit4(0, 3) | bit4(1, 1) | bit4(1, 2) | bit4(1, 3) |
                                  bit4(2, 2) | bit4(2, 3) | bit4(3, 3);
    static constexpr unsigned B = bit2(2, 1) | bit2(3, 0);
    static constexpr unsigned Q = bit4(0, 0) | bit4(1, 1) | bit4(2, 2) | bit4(3, 3);
    static constexpr unsigned R = bit2(0, 0) | bit2(1, 1);
    static constexpr bool AUNIT = true;
};
template <class SP>
struct Mt {
    const StageMats& m;
    // acc + X[a][b] * x, skipping structural zeros (indices are unrolled constants)
    __device__ __forceinline__ double A_(int a, int b, double x, double acc) const {
        if (!((SP::A >> (a * 4 + b)) & 1u)) return acc;
        if (SP::AUNIT && a == b) return acc + x;
        return fma(m.A[a * 4 + b], x, acc);
    }
    __device__ __forceinline__ double B_(int a, int c, double x, double acc) const {
        return ((SP::B >> (a * 2 + c)) & 1u) ? fma(m.B[a * 2 + c], x, acc) : acc;
    }
    __device__ __forceinline__ double Q_(int a, int b, double x, double acc) const {
        return ((SP::Q >> (a * 4 + b)) & 1u) ? fma(m.Q[a * 4 + b], x, acc) : acc;
    }
    __device__ __forceinline__ double R_(int c, int d, double x, double acc) const {
        return ((SP::R >> (c * 2 + d)) & 1u) ? fma(m.R[c * 2 + d], x, acc) : acc;
    }
    // structural zeros are returned / accumulated as -0.0: x + (-0.0) == x and
    // fma(a, b, -0.0) == a * b exactly, so the compiler drops them
    __device__ __forceinline__ double Qv(int a, int b) const { return ((SP::Q >> (a * 4 + b)) & 1u) ? m.Q[a * 4 + b] : -0.0; }
    __device__ __forceinline__ double Rv(int c, int d) const { return ((SP::R >> (c * 2 + d)) & 1u) ? m.R[c * 2 + d] : -0.0; }
    // (R v)_c
    __device__ __forceinline__ double Rmul(int c, double v0, double v1) const { return R_(c, 0, v0, R_(c, 1, v1, -0.0)); }
};

// Per-instance model (carmpc_hetero_*): A, B of the group's own instance in registers (only the
// entries inside the sparsity masks are ever read), Q, R shared from the kernel argument.
template <class SP>
struct MtH {
    const StageMats& m;
    double A[16], B[8];
    __device__ explicit MtH(const StageMats& s) : m(s), A{}, B{} {}
    __device__ __forceinline__ double A_(int a, int b, double x, double acc) const {
        if (!((SP::A >> (a * 4 + b)) & 1u)) return acc;
        if (SP::AUNIT && a == b) return acc + x;
        return fma(A[a * 4 + b], x, acc);
    }
    __device__ __forceinline__ double B_(int a, int c, double x, double acc) const {
        return ((SP::B >> (a * 2 + c)) & 1u) ? fma(B[a * 2 + c], x, acc) : acc;
    }
    __device__ __forceinline__ double Q_(int a, int b, double x, double acc) const {
        return ((SP::Q >> (a * 4 + b)) & 1u) ? fma(m.Q[a * 4 + b], x, acc) : acc;
    }
    __device__ __forceinline__ double R_(int c, int d, double x, double acc) const {
        return ((SP::R >> (c * 2 + d)) & 1u) ? fma(m.R[c * 2 + d], x, acc) : acc;
    }
    __device__ __forceinline__ double Qv(int a, int b) const { return ((SP::Q >> (a * 4 + b)) & 1u) ? m.Q[a * 4 + b] : -0.0; }
    __device__ __forceinline__ double Rv(int c, int d) const { return ((SP::R >> (c * 2 + d)) & 1u) ? m.R[c * 2 + d] : -0.0; }
    __device__ __forceinline__ double Rmul(int c, double v0, double v1) const { return R_(c, 0, v0, R_(c, 1, v1, -0.0)); }
};

// HET: every instance has its own linearisation (hetero.hip): A, B, P, slot row norms, w0, E,
// hq and x0-only rows come from the instance's slices; the row layout is the template's.
// One launch serves up to kRicMaxSeg problems (instance segments, carmpc_solve_segments); a
// single problem is the one-segment case.  The descriptors travel by value in the kernel arguments
// (scalar loads), every segment has its own claim counter (S.claim + 16 seg), and the workgroups
// are dealt to "home" segments in proportion to the instance counts.  A workgroup serves its home
// segment until that counter runs out, then moves on round-robin to help with the others
// (reloading the problem's slot tables), so the launch ends when every segment is drained -- no
// per-problem launch tail, no side streams.
//
// MODE splits the solve over three launches (launch pipeline below) so that each one runs lean code:
//   1  interior-point iterations only.  An instance that reaches its polish point is handed off --
//      its active set (one bit per row slot and box row) and iteration count go to the work lists --
//      and the group claims its next instance at once.  No polish code, no polish state.
//   2  polish only, over the hand-off list: every instance runs the same fixed sequence (active-set
//      factorization, solve, three refinements, acceptance test), so the four groups of a wave polish
//      in lock-step instead of one at a time beside three iterating groups.  A group whose polish
//      is rejected keeps the instance for the correction round (its next trip, see act_next); what
//      is rejected again goes to the retry list.
//   0  the complete algorithm in one kernel (iterations and polish interleaved per group): solves the
//      retry list from scratch -- the arithmetic is deterministic, so this reproduces the rejected
//      polish and carries on exactly as a single-kernel solve would -- and serves callers that bring
//      their own instance lists or claim counter (closed loops, per-instance models, no-allocation entry).
//
// LPQ = lanes per QP.  16: one DPP row per QP, four QPs per wavefront, every lane holds two segments of row
// slots.  32: two QPs per wavefront, lane l holds ONE segment (stage l + 1; lanes beyond the horizon hold
// overflow rows of the last stage) -- half the per-lane state, so that two wavefronts fit one SIMD's register
// file and the LDS of a CU holds the same sixteen QPs in eight waves instead of four: the second wave fills
// the issue slots the first leaves idle while it waits for its own dependent results.  The matrix-core passes
// then carry two QPs in blocks 0 and 1; blocks 2 and 3 repeat them (same loads, same values stored).
//
// SEGS = slot segments per lane.  With 16 lanes per QP the default is two (the original layout, 16 row slots per
// lane); SEGS = 1 with 16 lanes is the layout for short horizons whose rows fit the first segment alone (N <= 16,
// capi.hip::riccati_layout, DevProblem::rone): FOUR QPs per wavefront at the per-lane state of the 32-lane
// layout, so eight waves of four QPs share a CU -- twice the QPs per instruction.
template <int N, int WPB, class SP, bool HET = false, int MODE = 0, int LPQ = 16, int SEGS = 32 / LPQ>
__global__ void __launch_bounds__(WPB * 64) ipm_riccati_kernel(RicSegs T, RicWork W, const double* __restrict__ x0_all,
                                                               const double* __restrict__ xref_all,
                                                               double* __restrict__ u_all, int64_t ld_u,
                                                               int32_t* __restrict__ status_all,
                                                               int32_t* __restrict__ iters_all, Settings S_all) {
    static_assert(!(HET && MODE != 0), "per-instance models run the single-kernel algorithm");
    // Per-instance models run the algorithm and the matrix-core passes of the shared-model kernels (their stage
    // matrices are reloaded per block whenever a group takes a new instance); HL selects their former variant --
    // scalar stage passes with A, B in registers, one polish attempt behind the conservative gate, z = 1 start --
    // in experiment builds (-DCARMPC_HET_LEGACY=1).
    constexpr bool HL = HET && CARMPC_HET_LEGACY != 0;
    constexpr double kMu0 = HL ? 0.0 : CARMPC_INIT_MU0, kSFloor = HL ? 1.0 : CARMPC_INIT_SFLOOR;
    constexpr int kPolRefine = HL ? POLISH_REFINE_CONSERVATIVE : POLISH_REFINE;
    constexpr double kAct = HL ? 1.0 : POLISH_ACT;   // a row starts the polish active when s < kAct z
    constexpr int kSolves = kPolRefine + 1 > 3 ? kPolRefine + 1 : 3;   // solves per trip: 3 of a step, kPolRefine + 1 of a polish
    constexpr double kMuMin = CARMPC_INIT_MU_MIN, kQInv = 1.0 / (CARMPC_INIT_Q_PER_VAR * 2 * N);
    constexpr int kUnroll = HET ? CARMPC_RIC_UNROLL_HET : CARMPC_RIC_UNROLL;
    constexpr int kUnrollAdj = HET ? CARMPC_RIC_UNROLL_HET : CARMPC_RIC_UNROLL_ADJ;
    __shared__ __attribute__((aligned(16))) RicShared<N> sh;
    constexpr int GL = LPQ;            // lanes of a group (one QP)
    constexpr int NG = 64 / LPQ;       // groups per wavefront
    constexpr int NSG = SEGS;          // row-slot segments per lane
    static_assert(LPQ * SEGS <= 32 && (SEGS == 1 || SEGS == 2), "a group's lanes hold at most the table's 32 segments");
    constexpr int SL = NSG * RSEG;     // row slots per lane
    constexpr int REC = ric_rec<N, LPQ, SEGS>();               // doubles per stage record
    constexpr int QS = ric_qstride(N, REC, NG);                // doubles between the records of two groups
    __shared__ __attribute__((aligned(16))) RicWave<N, LPQ, SEGS> wscr[WPB];
    const int nseg = T.nseg;
    int home = 0;
    if (nseg > 1) {
        const int64_t first = T.off[0], total = T.off[nseg] - first;
        const int64_t pos = first + (int64_t)blockIdx.x * total / gridDim.x;
        while (home + 1 < nseg && pos >= T.off[home + 1]) ++home;
    }
    for (int kseg_i = 0; kseg_i < nseg; ++kseg_i) {
    const int seg = nseg > 1 ? (home + kseg_i) % nseg : 0;
    const DevProblem& P = T.P[seg];
    const int64_t seg0 = T.off[seg], batch = T.off[seg + 1] - seg0;
    const int64_t lst0 = seg0 - T.off[0];   // the segment's start in the work lists, which begin at the run's first instance
    const double* __restrict__ x0 = x0_all + seg0 * NX;
    const double* __restrict__ xref = xref_all ? xref_all + seg0 * NX : nullptr;
    double* __restrict__ u_out = u_all + seg0 * ld_u;
    int32_t* __restrict__ status_out = status_all + seg0;
    int32_t* __restrict__ iters_out = iters_all ? iters_all + seg0 : nullptr;
    Settings S = S_all;
    if (W.cnt) {   // launch pipeline: this segment's counters and work lists of round W.round (RicWork)
        unsigned* wc = W.cnt + kRicClaimStride * seg;
        if constexpr (MODE == 1) {
            if (W.round == 0) {
                S.claim = wc + 0;
            } else {   // the previous round's rejected polishes
                S.index = W.retry_idx + lst0;
                S.count = reinterpret_cast<const int32_t*>(wc + 4 * W.round - 1);
                S.claim = wc + 4 * W.round;
            }
        } else if constexpr (MODE == 2) {
            S.index = nullptr;   // (rows come from the hand-off records)
            S.count = reinterpret_cast<const int32_t*>(wc + 4 * W.round + 1);
            S.claim = wc + 4 * W.round + 2;
        } else {   // after the last round
            S.index = W.retry_idx + lst0;
            S.count = reinterpret_cast<const int32_t*>(wc + 4 * W.round - 1);
            S.claim = wc + 4 * W.round;
        }
    } else if (S.claim) {
        S.claim += kRicClaimStride * seg;
    }
    if (kseg_i > 0) __syncthreads();   // every wave is done with the previous problem's tables
    if (batch <= 0) continue;
    const StageMats& MT = P.mats;
    std::conditional_t<HL, MtH<SP>, const Mt<SP>> M{P.mats};
    int64_t hinst = 0;   // HET: the group's current instance (slice index)
    for (int i = threadIdx.x; i < kTab; i += blockDim.x) {
        sh.cf01[i] = make_double2(P.r_coef[i * 4 + 0], P.r_coef[i * 4 + 1]);
        sh.cf23[i] = make_double2(P.r_coef[i * 4 + 2], P.r_coef[i * 4 + 3]);
        sh.partner[i] = (int16_t)(P.r_partner ? P.r_partner[i] : -1);
    }
    for (int i = threadIdx.x; i < 2 * N; i += blockDim.x) {
        const bool bx = P.boxed;
        sh.lb[i] = bx ? P.lb[i] : -UNBOXED_BOUND;
        sh.ub[i] = bx ? P.ub[i] : UNBOXED_BOUND;
    }
    __syncthreads();

    const int lane = threadIdx.x & 63;
    const int wave = threadIdx.x >> 6;
    const int g = lane / GL, j = lane % GL;
    // slot s of this lane in the problem's slot table (see kTab)
    const int j16 = lane & 15, sbase = LPQ == 32 ? ((lane >> 4) & 1) * RSEG : 0;
    auto tix = [&](int s) { return (sbase + s) * G16 + j16; };
    RicWave<N, LPQ, SEGS>& wv = wscr[wave];
    double* rec = wv.recbuf + g * QS;
    double(*scr)[64] = reinterpret_cast<double(*)[64]>(wv.recbuf);
    const bool boxed = P.boxed != 0;
    // segment stages: seg 0 -> j+1, seg 1 -> j+17 (overflow segments -> stage N)
    int kseg[NSG];
    bool own[NSG], isN[NSG];
#pragma unroll
    for (int sg = 0; sg < NSG; ++sg) {
        const int k = j + 1 + 16 * sg;
        own[sg] = k <= N;
        kseg[sg] = k <= N ? k : N;
        isN[sg] = kseg[sg] == N;
    }
    double* vb[NSG];
#pragma unroll
    for (int sg = 0; sg < NSG; ++sg) vb[sg] = &wv.vbox[g][0][own[sg] ? kseg[sg] - 1 : N][0];
#define BX(F, sg, c) vb[sg][(F) * ((N + 1) * 2) + (c)]
    // Unused row slots are made inert instead of being masked: their coefficients are zero, w = 1,
    // s = 1, z = 0, so every residual, direction and sum below gets an exact zero from them and the
    // slot loops are straight-line code (no exec-mask region per slot).  The validity bits are only
    // consulted where the instance is set up and in the polish acceptance test.
    unsigned rvm = 0;
#pragma unroll
    for (int s = 0; s < SL; ++s) rvm |= (P.r_valid[tix(s)] != 0 ? 1u : 0u) << s;
    auto valid = [&](int s) { return ((rvm >> s) & 1u) != 0; };
    const int p = P.p;
    const int m_rows = p + (boxed ? 4 * N : 0);
    const double inv_m = 1.0 / (double)(m_rows > 0 ? m_rows : 1);
    const double idl = 1.0 / POLISH_DELTA;

    // ---- helpers ----------------------------------------------------------------------
    // reductions over the lanes of the group (they shadow the 16-lane row reductions of lanes.h)
    auto row_sum = [](double v) __attribute__((always_inline)) { return grp_reduce<LPQ, OpSum>(v); };
    auto row_max = [](double v) __attribute__((always_inline)) { return grp_reduce<LPQ, OpMax>(v); };
    auto row_min = [](double v) __attribute__((always_inline)) { return grp_reduce<LPQ, OpMin>(v); };
    // Totals over the rows of stage N, wanted by the owner of stage N alone.  With 32 lanes per QP and N >= 17 that
    // owner (lane N - 1) and every overflow lane sit in the group's upper DPP row, the lower row contributes
    // zeros: the 16-lane butterfly is the whole sum there (the lower row's lanes get a value nobody reads).
    constexpr bool kStageNUpperRow = LPQ == 32 && N >= 17;
    // Two totals at a time (lanes.h: the second value rides in the lower row through the same butterfly).
    auto stageN_sum2 = [&](double& a, double& b) __attribute__((always_inline)) {
        if constexpr (kStageNUpperRow) upper_row_sum2(a, b);
        else grp_reduce2<LPQ, OpSum>(a, b);
    };
    // this lane's part of a stage-N total: the entries of its segments that belong to stage N
    auto stageN_part = [&](const auto& v, int e) __attribute__((always_inline)) {
        double t = isN[0] ? v[0][e] : 0.0;
        if constexpr (NSG == 2) t += isN[1] ? v[1][e] : 0.0;
        return t;
    };
    // Row-slot loops.  Slots are visited pairwise -- slot i of segment 0, then slot i of segment 1 --
    // for i below the problem's slots-per-segment count (wave-uniform: a scalar branch ahead of the
    // pairs i >= kSegMin, none below).  The next slot's coefficients and w are loaded one slot ahead
    // and a scheduling barrier closes every slot: the live set stays one slot wide instead of
    // growing with however many slots the compiler chooses to interleave.
    struct SlotIn { double2 c01, c23; double w, iv; };
    auto ld_slot = [&](int s) __attribute__((always_inline)) {
        SlotIn in;
        in.c01 = sh.cf01[tix(s)];
        in.c23 = sh.cf23[tix(s)];
        in.w = wv.w[s][lane];
        in.iv = 1.0;
        if constexpr (HET) in.iv = P.het_ric_invn[hinst * kTab + tix(s)];
        return in;
    };
    auto coef = [&](const SlotIn& in, double (&c)[4]) __attribute__((always_inline)) {
        c[0] = in.c01.x; c[1] = in.c01.y; c[2] = in.c23.x; c[3] = in.c23.y;
        if constexpr (HET) {   // raw template coefficients x this instance's 1/||G_r||
#pragma unroll
            for (int a2 = 0; a2 < 4; ++a2) c[a2] *= in.iv;
        }
    };
    constexpr int kSegMin = 6;
    const int rseg = P.rseg;
    auto for_slots = [&](auto&& body) __attribute__((always_inline)) {
        SlotIn cur = ld_slot(0);
#pragma unroll
        for (int q = 0; q < SL; ++q) {
            const int i = q / NSG, s = (q % NSG) * RSEG + i;
            if (i >= kSegMin && i >= rseg) break;   // uniform; the remaining slots are unused in every lane
            const int qn = q + 1 < SL ? q + 1 : q;
            const SlotIn nxt = ld_slot((qn % NSG) * RSEG + (qn / NSG));
            body(s, cur);
            if (CARMPC_RIC_SLOT_FENCE != 0 && (q + 1) % (CARMPC_RIC_SLOT_FENCE != 0 ? CARMPC_RIC_SLOT_FENCE : 1) == 0)
                __builtin_amdgcn_sched_barrier(0);
            cur = nxt;
        }
    };
    // the same visit without the loads (slot state in registers only)
    auto for_used = [&](auto&& body) __attribute__((always_inline)) {
#pragma unroll
        for (int q = 0; q < SL; ++q) {
            const int i = q / NSG;
            if (i >= kSegMin && i >= rseg) break;
            body((q % NSG) * RSEG + i);
        }
    };
#define FOR_SLOTS_BEGIN                                                                        \
    for_slots([&](const int s, const SlotIn& in) __attribute__((always_inline)) {              \
        const int sg = s / RSEG;                                                               \
        double c[4];                                                                           \
        coef(in, c);
#define FOR_SLOTS_END });
    auto cf = [&](int s, double (&c)[4]) {
        const double2 a = sh.cf01[tix(s)], b = sh.cf23[tix(s)];
        c[0] = a.x; c[1] = a.y; c[2] = b.x; c[3] = b.y;
        if constexpr (HET) {   // raw template coefficients x this instance's 1/||G_r||
            const double iv = P.het_ric_invn[hinst * kTab + tix(s)];
#pragma unroll
            for (int a2 = 0; a2 < 4; ++a2) c[a2] *= iv;
        }
    };
    // terminal cost P (upper triangle read): shared, or this instance's DARE solution
    auto Pv = [&](int idx) -> double {
        if constexpr (HET) return P.het_P[hinst * 16 + idx];
        else return MT.P[idx];
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
            double accp = -0.0, accq = -0.0;
#pragma unroll
            for (int b = 0; b < 4; ++b) {
                accp = fma(Pv((a < b ? a : b) * 4 + (a < b ? b : a)), v[b], accp);
                accq = M.Q_(a, b, v[b], accq);
            }
            y[a] = fma(sgn, termN ? accp : accq, y[a]);
        }
    };
    // sum the stage-N partials of the 16 lanes; owners write b^x (plus Qbar term) of their stages
    auto write_bx = [&](double (&acc)[NSG][4], const double (&qv)[NSG][4], double qsgn) {
        double pn[4];
#pragma unroll
        for (int a = 0; a < 4; ++a) pn[a] = stageN_part(acc, a);
#pragma unroll
        for (int a = 0; a < 4; a += 2) stageN_sum2(pn[a], pn[a + 1]);
#pragma unroll
        for (int sg = 0; sg < NSG; ++sg) {
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
        // stage data one stage ahead (software pipelining of the LDS latency)
        auto ld = [&](int t, double (&bu)[2], double (&ch)[4], double (&K)[8], double (&bx)[4]) {
            const int r = t * REC;
            rd2(r + O_BU, bu[0], bu[1]);
            rd2(r + O_CH, ch[0], ch[1]);
            rd2(r + O_CH + 2, ch[2], ch[3]);
            rdK(r, K);
            rd4((t >= 1 ? r - REC : 0) + O_BX, bx);
        };
        double bu[2], ch[4], K[8], bx[4];
        ld(N - 1, bu, ch, K, bx);
#pragma unroll kUnroll
        for (int t = N - 1; t >= 0; --t) {
            double nbu[2], nch[4], nK[8], nbx[4];
            ld(t >= 1 ? t - 1 : 0, nbu, nch, nK, nbx);
            double g0 = bu[0], g1 = bu[1];
#pragma unroll
            for (int a = 0; a < 4; ++a) {
                g0 = M.B_(a, 0, pv[a], g0);
                g1 = M.B_(a, 1, pv[a], g1);
            }
            const double il00 = ch[0], l10 = ch[1], il11 = ch[2];
            const double y0 = g0 * il00;
            const double y1 = fma(-l10, y0, g1) * il11;
            const double k1 = y1 * il11;
            const double k0 = fma(-l10, k1, y0) * il00;
            if (RIC_WRITER) wr2(t * REC + O_DB, k0, k1);
            double np[4];
#pragma unroll
            for (int a = 0; a < 4; ++a) {
                double acc = bx[a];
#pragma unroll
                for (int c = 0; c < 4; ++c) acc = M.A_(c, a, pv[c], acc);
                acc = fma(-K[a], g0, acc);
                np[a] = fma(-K[4 + a], g1, acc);
            }
#pragma unroll
            for (int a = 0; a < 4; ++a) pv[a] = np[a];
#pragma unroll
            for (int e = 0; e < 8; ++e) K[e] = nK[e];
#pragma unroll
            for (int e = 0; e < 4; ++e) { ch[e] = nch[e]; bx[e] = nbx[e]; }
            bu[0] = nbu[0];
            bu[1] = nbu[1];
        }
        wb();
    };
    // forward pass: y_0 = 0; v_t = kappa_t - K_t y_t; y_{t+1} = A y_t + B v_t -> rec
    auto forward = [&]() {
        wb();
        double y[4] = {0.0, 0.0, 0.0, 0.0};
        double K[8], kp[2];
        rdK(0, K);
        rd2(O_DB, kp[0], kp[1]);
#pragma unroll kUnroll
        for (int t = 0; t < N; ++t) {
            const int r = t * REC;
            const int rn = (t + 1 < N ? t + 1 : t) * REC;
            double nK[8], nkp[2];
            rdK(rn, nK);
            rd2(rn + O_DB, nkp[0], nkp[1]);
            double v0 = kp[0], v1 = kp[1];
#pragma unroll
            for (int a = 0; a < 4; ++a) {
                v0 = fma(-K[a], y[a], v0);
                v1 = fma(-K[4 + a], y[a], v1);
            }
            double ny[4];
#pragma unroll
            for (int a = 0; a < 4; ++a) {
                double acc = M.B_(a, 0, v0, -0.0);
                acc = M.B_(a, 1, v1, acc);
#pragma unroll
                for (int c = 0; c < 4; ++c) acc = M.A_(a, c, y[c], acc);
                ny[a] = acc;
            }
#pragma unroll
            for (int a = 0; a < 4; ++a) y[a] = ny[a];
            if (RIC_WRITER) {
                wr4(r + O_BX, y);
                wr2(r + O_BU, v0, v1);
            }
#pragma unroll
            for (int e = 0; e < 8; ++e) K[e] = nK[e];
            kp[0] = nkp[0];
            kp[1] = nkp[1];
        }
        wb();
    };
    // plain roll-out of v_t stored in rec[t][O_BU] (initial point): y -> rec[t][O_BX]
    auto rollout = [&]() {
        auto run = [&](const auto& MM) __attribute__((always_inline)) {
            wb();
            double y[4] = {0.0, 0.0, 0.0, 0.0};
            for (int t = 0; t < N; ++t) {   // (rolled: this runs once per instance, and only when 0 lies outside the input box)
                const int r = t * REC;
                double v0, v1;
                rd2(r + O_BU, v0, v1);
                double ny[4];
#pragma unroll
                for (int a = 0; a < 4; ++a) {
                    double acc = MM.B_(a, 0, v0, -0.0);
                    acc = MM.B_(a, 1, v1, acc);
#pragma unroll
                    for (int c = 0; c < 4; ++c) acc = MM.A_(a, c, y[c], acc);
                    ny[a] = acc;
                }
#pragma unroll
                for (int a = 0; a < 4; ++a) y[a] = ny[a];
                wb();
                if (RIC_WRITER) wr4(r + O_BX, y);
            }
            wb();
        };
        if constexpr (HET && !HL) {   // this instance's A, B (the only scalar stage loop of the per-instance kernels)
            MtH<SP> Mh(P.mats);
#pragma unroll
            for (int e = 0; e < 16; ++e) Mh.A[e] = P.het_A[hinst * 16 + e];
#pragma unroll
            for (int e = 0; e < 8; ++e) Mh.B[e] = P.het_B[hinst * 8 + e];
            run(Mh);
        } else {
            run(M);
        }
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
                for (int b = a; b < 4; ++b) Pm[sym10(a, b)] = Pv(a * 4 + b) + Wn[sym10(a, b)];
            rd4((N - 1) * REC + O_BX, pv);
        }
        // stage data one stage ahead: Db_t, b^u_t (record t), W_t, b^x_t (record t-1)
        auto ld = [&](int t, double (&du)[4], double (&Wt)[10], double (&bx)[4]) {
            const int r = t * REC, rp = (t >= 1 ? t - 1 : 0) * REC;
            rd2(r + O_DB, du[0], du[1]);
            rd2(r + O_BU, du[2], du[3]);
#pragma unroll
            for (int e = 0; e < 5; ++e) rd2(rp + 2 * e, Wt[2 * e], Wt[2 * e + 1]);
            rd4(rp + O_BX, bx);
        };
        double du[4], Wt[10], bx[4];
        ld(N - 1, du, Wt, bx);
#pragma unroll kUnroll
        for (int t = N - 1; t >= 0; --t) {
            const int r = t * REC;
            double ndu[4], nWt[10], nbx[4];
            ld(t >= 1 ? t - 1 : 0, ndu, nWt, nbx);
            const double db0 = du[0], db1 = du[1], bu0 = du[2], bu1 = du[3];
            // PB = P B (4x2); Re = R + diag(Db) + B'PB; F = B'PA = (PB)'A
            double PB[4][2];
#pragma unroll
            for (int a = 0; a < 4; ++a)
#pragma unroll
                for (int c = 0; c < 2; ++c) {
                    double acc = -0.0;
#pragma unroll
                    for (int b = 0; b < 4; ++b) acc = M.B_(b, c, Pm[sym10(a, b)], acc);
                    PB[a][c] = acc;
                }
            double re00 = M.Rv(0, 0) + db0, re10 = M.Rv(1, 0), re11 = M.Rv(1, 1) + db1;
#pragma unroll
            for (int a = 0; a < 4; ++a) {
                re00 = M.B_(a, 0, PB[a][0], re00);
                re10 = M.B_(a, 1, PB[a][0], re10);
                re11 = M.B_(a, 1, PB[a][1], re11);
            }
            double F[2][4];
#pragma unroll
            for (int c = 0; c < 2; ++c)
#pragma unroll
                for (int mm = 0; mm < 4; ++mm) {
                    double acc = -0.0;
#pragma unroll
                    for (int a = 0; a < 4; ++a) acc = M.A_(a, mm, PB[a][c], acc);
                    F[c][mm] = acc;
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
                g0 = M.B_(a, 0, pv[a], g0);
                g1 = M.B_(a, 1, pv[a], g1);
            }
            const double y0 = g0 * il00;
            const double y1 = fma(-l10, y0, g1) * il11;
            const double k1 = y1 * il11;
            const double k0 = fma(-l10, k1, y0) * il00;
            wb();
            if (RIC_WRITER) {
                wr4(r + O_K, K[0]);
                wr4(r + O_K + 4, K[1]);
                wr2(r + O_CH, il00, l10);
                wr2(r + O_CH + 2, il11, 0.0);
                wr2(r + O_DB, k0, k1);
            }
            if (t >= 1) {
                // P_t = Qbar_t + W_t + A'PA - F'K  (upper triangle), PA one column at a time
                double Pn[10];
#pragma unroll
                for (int b = 0; b < 4; ++b) {
                    double col[4];
#pragma unroll
                    for (int c = 0; c < 4; ++c) {
                        double acc = -0.0;
#pragma unroll
                        for (int d = 0; d < 4; ++d) acc = M.A_(d, b, Pm[sym10(c, d)], acc);
                        col[c] = acc;
                    }
#pragma unroll
                    for (int a = 0; a <= b; ++a) {
                        double acc = M.Qv(a, b) + Wt[sym10(a, b)];
#pragma unroll
                        for (int c = 0; c < 4; ++c) acc = M.A_(c, a, col[c], acc);
                        acc = fma(-F[0][a], K[0][b], acc);
                        Pn[sym10(a, b)] = fma(-F[1][a], K[1][b], acc);
                    }
                }
#pragma unroll
                for (int e = 0; e < 10; ++e) Pm[e] = Pn[e];
                double np[4];
#pragma unroll
                for (int a = 0; a < 4; ++a) {
                    double acc = bx[a];
#pragma unroll
                    for (int c = 0; c < 4; ++c) acc = M.A_(c, a, pv[c], acc);
                    acc = fma(-K[0][a], g0, acc);
                    np[a] = fma(-K[1][a], g1, acc);
                }
#pragma unroll
                for (int a = 0; a < 4; ++a) pv[a] = np[a];
            }
#pragma unroll
            for (int e = 0; e < 10; ++e) Wt[e] = nWt[e];
#pragma unroll
            for (int e = 0; e < 4; ++e) { du[e] = ndu[e]; bx[e] = nbx[e]; }
        }
        wb();
    };


    // ---- stage recursions on the matrix cores (shared-model problems) -------------------
    // v_mfma_f64_4x4x4f64 multiplies four independent 4x4 blocks per wavefront; block b lives in
    // lanes 16 r + 4 b + c (r, c = 0..3), and with X^ the 4x4 matrix whose entry (r, c) is the
    // value lane (r, c) holds in register X, the instruction computes  D^ = A^' B^ + C^
    // (operand A enters transposed; the neg modifier negates an operand for free).  In the
    // recursion phases block b therefore works on QP group b with ONE matrix entry per lane --
    // P, K, the 2x2 pivots are single registers -- instead of every lane of a group repeating the
    // whole 4x4 recursion; vectors are 4x4 operands whose columns all hold the vector (the adjoint
    // pass carries psiZ / psiH in columns 0 / 1).  Stage data is exchanged with the row phases
    // through the same LDS records.  The passes are straight-line code without exec masking:
    //   * all four blocks always compute (MFMA needs the whole wave); a block whose group sits out
    //     a pass only overwrites record fields that are dead until the group's next trip;
    //   * structural zeros (rows 2-3 of K, of b^u, ...) are loaded from slot 11 of each record,
    //     which always holds 0.0, and lanes whose result is a structural zero store it there;
    //   * lanes that hold copies of one value (the columns of a vector) all store it.
    const int mb = (lane >> 2) & 3, mr = lane >> 4, mc = lane & 3;
    double* recm = wv.recbuf + (mb % NG) * QS;
    auto mm = [](double a, double b, double c) { return __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, c, 0, 0, 0); };
    auto mm_na = [](double a, double b, double c) { return __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, c, 0, 0, 1); };
    const bool m_top = mr < 2, m_left = mc < 2;
    const int oW = sym10(mr, mc);                              // W^, P^ entry in the packed 10-vector
    const int oK = m_top ? O_K + 4 * mr + mc : O_ZERO;         // K^ (rows 0-1)
    const int oKT = m_left ? O_K + 4 * mc + mr : O_ZERO;       // K'^ (columns 0-1)
    const int oLam = m_left ? 4 * mc + mr : O_ZERO;            // [lamZ lamH 0 0]
    const int oGH = (m_top && m_left) ? 12 + 2 * mc + mr : O_ZERO;   // gz, hs
    const int oBUt = m_top ? O_BU + mr : O_ZERO;               // b^u / v in rows 0-1
    const int oBU1 = mr == 1 ? O_BU : O_ZERO;                  // b^u_0 in row 1 (for E b^u)
    const int oKPt = m_top ? O_DB + mr : O_ZERO;               // kappa in rows 0-1
    const int oDrow = O_CH + (mr == 0 ? 1 : 2);                // 1/p0 in row 0, 1/p1 below
    double cA = 0.0, cBp = 0.0, cB0r = 0.0, cB1r = 0.0, cQ = 0.0, cPt = 0.0;
    if constexpr (HET) cQ = MT.Q[mr * 4 + mc];   // (A, B, P of a per-instance model: reloaded when a group takes a new instance)
    if constexpr (!HET) {
        cA = MT.A[mr * 4 + mc];                       // A^
        cBp = m_left ? MT.B[mr * 2 + mc] : 0.0;       // [B 0 0]^
        cB0r = MT.B[mr * 2];                          // column 0 of B in every column
        cB1r = MT.B[mr * 2 + 1];                      // column 1 of B in every column
        cQ = MT.Q[mr * 4 + mc];
        cPt = MT.P[mr * 4 + mc];
    }
    // Constants that only one kind of pass needs are rebuilt at its start (a dozen instructions, or two
    // matrix-core transposes) instead of occupying registers through the row phases; the lane index goes
    // through an empty asm so that the compiler does not hoist them back out of the trip loop.
    struct PassK { double cB0m1, k10, kd, cI; };
    auto pass_consts = [&]() __attribute__((always_inline)) {
        int lz = lane;
        asm volatile("" : "+v"(lz));
        const int r_ = lz >> 4, c_ = lz & 3;
        PassK k;
        k.cB0m1 = c_ == 1 ? cB0r : 0.0;                          // column 0 of B in column 1
        k.k10 = (r_ == 1 && c_ == 0) ? 1.0 : 0.0;
        k.kd = (r_ == c_ && r_ < 2) ? 1.0 : 0.0;                 // identity of the leading 2x2 block
        k.cI = r_ == c_ ? 1.0 : 0.0;
        return k;
    };
    // One wave per SIMD leaves nothing to hide an LDS round trip (~70 cycles) or an MFMA result
    // (28 cycles to a dependent MFMA, 16 cycles of pipe each) behind, so the passes are software
    // pipelined by hand: stage t's record fields are read kPre stages ahead, side products and
    // stores trail the recursion by a stage, and a scheduling barrier closes every stage -- without
    // it the compiler sinks the stores (nothing waits for them) and, since it cannot rule out an
    // alias between lane-dependent LDS offsets, every later load sinks behind them, back onto the
    // critical path.  The loops are fully unrolled; staged values sit in registers.
    constexpr int kPre = CARMPC_RIC_KPRE;
    auto stage_fence = [] { __builtin_amdgcn_sched_barrier(0); };
    // adjoint pass: psi_k = lam_k + A'psi_{k+1} for lamZ (column 0) and lamH (column 1);
    // gz_t, hs_t = B'psi_{t+1} -> rec[t][12..15]
    auto adjoint_mm = [&]() __attribute__((always_inline)) {
        wb();
        double lam[N], psi[N + 1], gh[N];
        psi[N] = 0.0;
#pragma unroll
        for (int t = N - 1; t >= 0 && t > N - 1 - kPre; --t) lam[t] = recm[t * REC + oLam];
        stage_fence();
#pragma unroll
        for (int t = N - 1; t >= -2; --t) {
            if (t - kPre >= 0) lam[t - kPre] = recm[(t - kPre) * REC + oLam];
            if (t >= 0) psi[t] = mm(cA, psi[t + 1], lam[t]);
            if (t + 1 >= 0 && t + 1 < N) gh[t + 1] = mm(cBp, psi[t + 1], 0.0);
            if (t + 2 < N) recm[(t + 2) * REC + oGH] = gh[t + 2];
            stage_fence();
        }
        wb();
    };
    // Riccati factorization (W_k, Db_t in rec) fused with the backward pass of the first
    // right-hand side.  Re_t = R + Db_t + B'PB = L D^{-1} L' with L = [[1, 0], [l, 1]] and
    // D = diag(1/p0, 1/p1), guarded like the Cholesky it replaces (a non-positive pivot becomes
    // 1e128), and Re_t^{-1} = E'D E with E = L^{-1} is applied in that factored form -- E F first,
    // then D, then E' -- never as an explicit inverse: when B'PB is nearly singular the rows of
    // F = B'PA are nearly dependent, and only the factored form subtracts them before scaling (an
    // explicit inverse stalled the IPM on such instances).  The three entries of Re_t come out of
    // MFMAs with B's columns replicated, so every lane of the block holds them (no cross-lane
    // broadcast).  K_t -> rec[t][0..7], (l, 1/p0, 1/p1) -> rec[t][8..10], kappa_t -> rec[t][18..19]
    auto factor_mm = [&]() __attribute__((always_inline)) {
        wb();
        const PassK pk = pass_consts();
        const double cB0m1 = pk.cB0m1, k10 = pk.k10, kd = pk.kd;
        struct In { double db0, db1, buT, bu01, Wt, bxv; };
        struct Out { double En, Z, zg, l, drow; };
        In in[N];
        Out o[N];
        auto load = [&](int t) {
            const int r = t * REC, rp = (t >= 1 ? t - 1 : 0) * REC;
            in[t].db0 = recm[r + O_DB];
            in[t].db1 = recm[r + O_DB + 1];
            in[t].buT = recm[r + oBUt];
            in[t].bu01 = recm[r + oBU1];
            in[t].Wt = recm[rp + oW];
            in[t].bxv = recm[rp + O_BX + mr];
        };
        double Pm = cPt + recm[(N - 1) * REC + oW];
        double pv = recm[(N - 1) * REC + O_BX + mr];
#pragma unroll
        for (int t = N - 1; t >= 0 && t > N - 1 - kPre; --t) load(t);
        stage_fence();
#pragma unroll
        for (int t = N - 1; t >= -1; --t) {
            if (t - kPre >= 0) load(t - kPre);
            if (t >= 0) {
                const double T = mm(Pm, cA, 0.0);             // P A
                const double PB0 = mm(Pm, cB0r, 0.0);         // every column: P b0
                const double PB1 = mm(Pm, cB1r, 0.0);         // every column: P b1
                const double re00 = mm(cB0r, PB0, MT.R[0] + in[t].db0);   // every entry: (R + Db + B'PB)_00
                const double re10 = mm(cB1r, PB0, MT.R[2]);
                const double re11 = mm(cB1r, PB1, MT.R[3] + in[t].db1);
                const double apT = mm(cA, T, cQ + in[t].Wt);  // Qbar_t + W_t + A'(P A)
                const double app = mm(cA, pv, in[t].bxv);     // b^x_t + A'p
                const double p0 = re00 > 0.0 ? re00 : 1e128;
                const double det = fma(p0, re11, -(re10 * re10));   // p0 p1
                const double r0 = frcp(p0);
                const double rd = frcp(det > 0.0 ? det : 1.0);
                const double ip1 = det > 0.0 ? p0 * rd : 1e-128;    // 1/p1, p1 = re11 - re10^2/p0
                const double l = re10 * r0;
                const double drow = mr == 0 ? r0 : ip1;
                const double Xl = fma(-l, cB0m1, cBp);              // [B 0 0] E'
                const double Y = mm(Xl, T, 0.0);                    // rows 0-1: E B'PA
                const double yg = mm(Xl, pv, fma(-l, in[t].bu01, in[t].buT));   // rows 0-1: E (b^u + B'p)
                o[t].En = fma(-l, k10, kd);                         // E (2x2 block)
                o[t].Z = Y * drow;
                o[t].zg = yg * drow;
                o[t].l = l;
                o[t].drow = drow;
                // P_t = Qbar_t + W_t + A'(P A) - F'K with F'K = Y'Z;  p_t = b^x_t + A'p - K'g, K'g = Y'zg
                Pm = mm_na(Y, o[t].Z, apT);
                pv = mm_na(Y, o[t].zg, app);
            }
            if (t + 1 < N) {   // the previous stage's gain, multiplier and factor, off the recursion's path
                const int r = (t + 1) * REC;
                recm[r + oK] = mm(o[t + 1].En, o[t + 1].Z, 0.0);       // rows 0-1: E'D E F = Re^{-1} F
                recm[r + oKPt] = mm(o[t + 1].En, o[t + 1].zg, 0.0);    // rows 0-1: Re^{-1} g
                recm[r + O_CH] = o[t + 1].l;
                recm[r + oDrow] = o[t + 1].drow;
            }
            stage_fence();
        }
        wb();
    };
    // The same with two QPs per wave.  Blocks 2 and 3 would repeat blocks 0 and 1 (same loads, same products); instead
    // they carry the VECTOR half of every stage -- b^x + A'p, E (b^u + B'p), the p recursion, kappa -- in the very
    // instructions whose matrix half (Qbar + W + A'PA, E B'PA, the P recursion, K) blocks 0 and 1 compute: the two
    // halves share the left operand (A, [B 0 0] E', Y, E) and differ in the right operand and the addend, which are one
    // register each with the matrix value in lanes 0..7 of a DPP row and the vector value in lanes 8..15.  What the
    // vector half needs from the matrix half -- l, the pivots' reciprocals, Y -- crosses once per stage (row_shr:8).
    // Ten products per stage instead of fourteen, three record loads instead of six; every product is the one the
    // unsplit pass computes, bit for bit.
    constexpr bool kFactorSplit = NG == 2 && CARMPC_RIC_FACTOR_SPLIT != 0;
    auto factor_mm_split = [&]() __attribute__((always_inline)) {
        wb();
        const PassK pk = pass_consts();
        const double cB0m1 = pk.cB0m1, k10 = pk.k10, kd = pk.kd;
        int lz = lane;
        asm volatile("" : "+v"(lz));
        const bool vrole = ((lz >> 3) & 1) != 0;   // blocks 2, 3
        const double cAm = vrole ? 0.0 : cA, cQm = vrole ? 0.0 : cQ;
        // the three record fields per stage: (Db_0, Db_1, W_t) for the matrix half, (b^u in rows 0-1, b^u_0 in row 1,
        // b^x_t) for the vector half; W_t and b^x_t sit in the record of stage t - 1
        const int o1 = vrole ? oBUt : O_DB, o2 = vrole ? oBU1 : O_DB + 1, o3 = vrole ? O_BX + (lz >> 4) : oW;
        const int oKK = vrole ? oKPt : oK;
        struct In { double l1, l2, l3; };
        struct Out { double En, ZZ, l, drow; };
        In in[N];
        Out o[N];
        auto load = [&](int t) {
            const int r = t * REC, rp = (t >= 1 ? t - 1 : 0) * REC;
            in[t].l1 = recm[r + o1];
            in[t].l2 = recm[r + o2];
            in[t].l3 = recm[rp + o3];
        };
        double PP = (vrole ? 0.0 : cPt) + recm[(N - 1) * REC + o3];   // P + W_N | b^x_N
#pragma unroll
        for (int t = N - 1; t >= 0 && t > N - 1 - kPre; --t) load(t);
        stage_fence();
#pragma unroll
        for (int t = N - 1; t >= -1; --t) {
            if (t - kPre >= 0) load(t - kPre);
            if (t >= 0) {
                const double X = mm(PP, cAm, vrole ? PP : 0.0);   // P A | p
                const double PB0 = mm(PP, cB0r, 0.0);             // (matrix half; the vector half's results are not used)
                const double PB1 = mm(PP, cB1r, 0.0);
                const double re00 = mm(cB0r, PB0, MT.R[0] + in[t].l1);
                const double re10 = mm(cB1r, PB0, MT.R[2]);
                const double re11 = mm(cB1r, PB1, MT.R[3] + in[t].l2);
                const double AP = mm(cA, X, cQm + in[t].l3);      // Qbar_t + W_t + A'(P A) | b^x_t + A'p
                const double p0 = re00 > 0.0 ? re00 : 1e128;
                const double det = fma(p0, re11, -(re10 * re10));
                const double r0 = frcp(p0);
                const double rd = frcp(det > 0.0 ? det : 1.0);
                const double ip1 = det > 0.0 ? p0 * rd : 1e-128;
                const double l = upper_half_from_lower(re10 * r0);
                const double drow = upper_half_from_lower(mr == 0 ? r0 : ip1);
                const double Xl = fma(-l, cB0m1, cBp);            // [B 0 0] E'
                const double YY = mm(Xl, X, vrole ? fma(-l, in[t].l2, in[t].l1) : 0.0);   // E B'PA | E (b^u + B'p)
                o[t].En = fma(-l, k10, kd);
                o[t].ZZ = YY * drow;
                o[t].l = l;
                o[t].drow = drow;
                PP = mm_na(upper_half_from_lower(YY), o[t].ZZ, AP);   // P_t | p_t
            }
            if (t + 1 < N) {
                const int r = (t + 1) * REC;
                recm[r + oKK] = mm(o[t + 1].En, o[t + 1].ZZ, 0.0);     // Re^{-1} F | Re^{-1} g   (rows 0-1)
                recm[r + O_CH] = o[t + 1].l;
                recm[r + oDrow] = o[t + 1].drow;
            }
            stage_fence();
        }
        wb();
    };
    // backward linear pass with the stored factor: kappa_t = Re_t^{-1}(b^u_t + B'p_{t+1}) in the
    // factored form above, p_t = b^x_t + A'p_{t+1} - K_t'g_t
    auto back_mm = [&]() __attribute__((always_inline)) {
        wb();
        const PassK pk = pass_consts();
        const double cB0m1 = pk.cB0m1, k10 = pk.k10, kd = pk.kd;
        struct In { double buT, bu01, l, drow, K, bxv; };
        In in[N];
        double En[N], zg[N];
        auto load = [&](int t) {
            const int r = t * REC, rp = (t >= 1 ? t - 1 : 0) * REC;
            in[t].buT = recm[r + oBUt];
            in[t].bu01 = recm[r + oBU1];
            in[t].l = recm[r + O_CH];
            in[t].drow = recm[r + oDrow];
            in[t].K = recm[r + oK];
            in[t].bxv = recm[rp + O_BX + mr];
        };
        double pv = recm[(N - 1) * REC + O_BX + mr];
#pragma unroll
        for (int t = N - 1; t >= 0 && t > N - 1 - kPre; --t) load(t);
        stage_fence();
#pragma unroll
        for (int t = N - 1; t >= -1; --t) {
            if (t - kPre >= 0) load(t - kPre);
            if (t >= 0) {
                const double l = in[t].l;
                const double g = mm(cBp, pv, in[t].buT);
                const double app = mm(cA, pv, in[t].bxv);
                const double yg = mm(fma(-l, cB0m1, cBp), pv, fma(-l, in[t].bu01, in[t].buT));
                En[t] = fma(-l, k10, kd);
                if (t >= 1) pv = mm_na(in[t].K, g, app);
                zg[t] = yg * in[t].drow;
            }
            if (t + 1 < N) recm[(t + 1) * REC + oKPt] = mm(En[t + 1], zg[t + 1], 0.0);
            stage_fence();
        }
        wb();
    };
    // forward pass: v_t = kappa_t - K_t y_t -> rec[t][16..17]; y_{t+1} = A y_t + B v_t -> rec[t][12..15]
    auto forward_mm = [&]() __attribute__((always_inline)) {
        wb();
        const PassK pk = pass_consts();
        const double cAT = mm(cA, pk.cI, 0.0), cBpT = mm(cBp, pk.cI, 0.0);   // (A')^ and [B 0 0]'^
        double KT[N], kp[N], y[N + 1], v[N];
        y[0] = 0.0;
#pragma unroll
        for (int t = 0; t < N && t < kPre; ++t) {
            KT[t] = recm[t * REC + oKT];
            kp[t] = recm[t * REC + oKPt];
        }
        stage_fence();
#pragma unroll
        for (int t = 0; t <= N; ++t) {
            if (t + kPre < N) {
                KT[t + kPre] = recm[(t + kPre) * REC + oKT];
                kp[t + kPre] = recm[(t + kPre) * REC + oKPt];
            }
            if (t < N) {
                v[t] = mm_na(KT[t], y[t], kp[t]);              // rows 0-1: kappa - K y
                const double ay = mm(cAT, y[t], 0.0);          // A y
                y[t + 1] = mm(cBpT, v[t], ay);                 // + B v
            }
            if (t >= 1) {
                recm[(t - 1) * REC + O_BX + mr] = y[t];
                recm[(t - 1) * REC + oBUt] = v[t - 1];
            }
            stage_fence();
        }
        wb();
    };

    // Each group claims its next instance from the launch's counter (S.claim, one atomic per
    // instance by the group's lane 0) at the first trip after finishing one, so the 4 groups
    // of a wave never wait for the slowest instance and no group is left with a heavier static
    // share at the end of the launch.  Without a counter: static stride over the grid.
    const int64_t stride = (int64_t)gridDim.x * WPB * NG;
    auto claim = [&]() -> int64_t {
        unsigned v = 0;
        if (j == 0) v = atomicAdd(S.claim, 1u);
        return (int64_t)__shfl(v, lane & ~(GL - 1), 64);
    };
    // closed-loop runs solve only their live instances: slot -> row through S.index, count on device
    // launch pipeline: the iteration launch leaves the segment's last W.tail instances to the final launch, which takes
    // them as fresh instances behind its retry list (slots nretry .. nretry + tail - 1)
    const int64_t ntail = W.cnt ? (int64_t)W.tail[seg] : 0;
    const int64_t nretry = (MODE == 0 && W.cnt) ? (int64_t)*S.count : 0;
    const int64_t nlive = (MODE == 0 && W.cnt) ? nretry + ntail
                          : S.count            ? (int64_t)*S.count
                          : (MODE == 1 && W.cnt) ? batch - ntail
                                                 : batch;
    int64_t slot = S.claim ? claim() : ((int64_t)blockIdx.x * WPB + wave) * NG + g;
    bool live = slot < nlive;   // the group has an instance to work on
    // slot -> row: the caller's list, the hand-off record (polish launch), or the slot itself
    auto row_of = [&](int64_t sl, bool lv) -> int64_t {
        if constexpr (MODE == 2) return lv ? (int64_t)(int32_t)W.pend_rec[(lst0 + sl) * kRicRecWords + kRicRecRow] : sl;
        else if (MODE == 0 && W.cnt)   // a retry (its entry names the hand-off record, which holds the row) or a fresh instance of the tail
            return !lv ? sl
                   : sl < nretry ? (int64_t)(int32_t)W.pend_rec[(lst0 + S.index[sl]) * kRicRecWords + kRicRecRow]
                                 : batch - ntail + (sl - nretry);
        else return lv && S.index ? (int64_t)S.index[sl] : sl;
    };
    int64_t inst = row_of(slot, live);
    bool fresh = true;          // ... that still needs its initial point
    double s_[SL], z_[SL];
    double xs[NSG][4];
    double bnorm = 1.0, qnorm = 1.0;
    int it = 0, npol = 0;   // iterations; polish points passed over (pipeline rounds > 0)
    bool polish_failed = false;
    // Polish correction (shared-model kernels): when the acceptance test rejects the first attempt at a polish
    // point and names rows to drop (active, negative multiplier) or to add (inactive, violated), the group's
    // next trip polishes again on that corrected set (act_next: the set, bit 31 = such a trip is due); a second
    // rejection stands.
    unsigned act_next = 0;
    // write the result of the current instance and move the group to its next one
    auto finish = [&](int st, bool zero_u, bool write = true) {
        if (write) {
#pragma unroll
            for (int sg = 0; sg < NSG; ++sg)
                if (own[sg]) {
                    const int t = kseg[sg] - 1;
                    u_out[inst * ld_u + 2 * t] = zero_u ? 0.0 : BX(F_U, sg, 0);
                    u_out[inst * ld_u + 2 * t + 1] = zero_u ? 0.0 : BX(F_U, sg, 1);
                }
            if (j == 0) {
                status_out[inst] = st;
                if (iters_out) iters_out[inst] = it;
            }
        }
        slot = S.claim ? claim() : slot + stride;
        live = slot < nlive;
        inst = row_of(slot, live);
        fresh = true;
    };
    RT_DECL
    while (__any(live)) {
        bool active = live;
        RT_MARK(11);
        const bool setup_now = live && fresh;
        if (live && fresh) {
            fresh = false;
            if constexpr (!HL) {   // slot 11 of every record is the matrix-core passes' source of structural zeros
                for (int t = j; t < N; t += GL) rec[t * REC + O_ZERO] = 0.0;
            }
            // this instance's data (HET) / the launch's problem
            const double *Ipw = P.pre_w0, *IpE = P.pre_E, *Irw = P.r_w0, *IrE = P.r_E, *Ihq = P.hq;
            const double *IpEd = P.pre_Ed, *IrEd = P.r_Ed, *Igoal = P.goal;
            // The problem's data never changes inside the instance loop, and the compiler would hoist
            // the loads below out of it -- dozens of registers of copies held for the whole kernel,
            // which pushes row state out to scratch memory.  Passing the pointers through an empty asm
            // makes them opaque, so the loads stay here.
            asm volatile("" : "+s"(Ipw), "+s"(IpE), "+s"(Irw), "+s"(IrE), "+s"(Ihq), "+s"(IpEd), "+s"(IrEd), "+s"(Igoal));
            int lzi = lane;   // likewise the lane's indices into them (per-slot address offsets would be kept otherwise)
            asm volatile("" : "+v"(lzi));
            const int ji = lzi % GL, tb = (LPQ == 32 ? ((lzi >> 4) & 1) * RSEG : 0) * G16 + (lzi & 15);
            if constexpr (HET) {
                hinst = inst;
                if constexpr (HL) {
#pragma unroll
                    for (int e = 0; e < 16; ++e) M.A[e] = P.het_A[inst * 16 + e];
#pragma unroll
                    for (int e = 0; e < 8; ++e) M.B[e] = P.het_B[inst * 8 + e];
                }
                Ipw += inst * P.het_sRow;
                IpE += inst * P.het_sRow * NX;
                Irw = P.het_ric_w0 + inst * kTab;
                IrE = P.het_ric_E + inst * kTab * NX;
                Ihq += inst * P.het_sHq;
            }
            double xv0[NX], xr[NX];
#pragma unroll
            for (int k = 0; k < NX; ++k) {
                if constexpr (MODE == 2)
                    xv0[k] = reinterpret_cast<const double*>(W.pend_rec + (lst0 + slot) * kRicRecWords + kRicRecX0)[k];
                else
                    xv0[k] = x0[inst * NX + k];
                xr[k] = xref ? xref[inst * NX + k] : Igoal[k];
            }
            // x0-only rows (G_r = 0): preconditions
            const double dd = S.dist ? S.dist[inst] : 0.0;   // disturbance estimate (w -= Ed d)
            double bad = 0.0;
            if constexpr (MODE != 2)   // (handed-off instances have passed this test)
            for (int r = ji; r < P.npre; r += GL) {
                double v = Ipw[r];
#pragma unroll
                for (int k = 0; k < NX; ++k) v -= IpE[r * NX + k] * xv0[k];
                if (IpEd) v -= IpEd[r] * dd;
                bad = v < -PRE_TOL ? 1.0 : bad;
            }
            it = 0;
            npol = 0;
            polish_failed = false;
            if constexpr (!HL) act_next = 0;
            if (row_max(bad) > 0.0) {
                finish(CARMPC_PRIMAL_INFEASIBLE, true);
                active = false;
            } else {
                // per-slot w, q and box of the owned inputs, initial point
                double bn = 0.0, qn = 0.0, u0n = 0.0;
#pragma unroll
                for (int s = 0; s < SL; ++s) {
                    double v = 0.0;
                    if (valid(s)) {
                        const int e = s * G16 + tb;
                        v = Irw[e];
#pragma unroll
                        for (int k = 0; k < NX; ++k) v -= IrE[e * NX + k] * xv0[k];
                        if (IrEd) v -= IrEd[e] * dd;
                    }
                    wv.w[s][lane] = valid(s) ? v : 1.0;
                    bn = fmax(bn, fabs(v));
                }
#pragma unroll
                for (int sg = 0; sg < NSG; ++sg) {
                    const int t = kseg[sg] - 1;
#pragma unroll
                    for (int c = 0; c < 2; ++c) {
                        const int i = 2 * t + c;
                        double q = 0.0;
#pragma unroll
                        for (int k = 0; k < NX; ++k) q = fma(Ihq[i * NX + k], xv0[k] - xr[k], q);
                        const double lb = sh.lb[i], ub = sh.ub[i];
                        const bool bx = own[sg] && boxed;
                        const double u0 = bx ? fmin(fmax(0.0, lb), ub) : 0.0;
                        BX(F_Q, sg, c) = own[sg] ? q : 0.0;
                        BX(F_U, sg, c) = u0;
                        const double su0 = fmax(ub - u0, kSFloor), sl0 = fmax(u0 - lb, kSFloor);
                        BX(F_SU, sg, c) = bx ? su0 : 1.0;
                        BX(F_SL, sg, c) = bx ? sl0 : 1.0;
                        BX(F_ZU, sg, c) = bx ? 1.0 : 0.0;
                        BX(F_ZL, sg, c) = bx ? 1.0 : 0.0;
                        bn = bx ? fmax(bn, fmax(fabs(lb), fabs(ub))) : bn;
                        qn = fmax(qn, own[sg] ? fabs(q) : 0.0);
                        u0n = fmax(u0n, fabs(u0));
                    }
                }
                // multipliers on the central path: z = mu0 / s with mu0 following the size of the linear term
                double mu0 = 0.0;
                if constexpr (!HL && MODE != 2) {
                    if (kMu0 > 0.0) {
                        const double qrel = kQInv * row_max(qn);
                        mu0 = fmin(kMu0, fmax(kMuMin, qrel * qrel));
#pragma unroll
                        for (int sg = 0; sg < NSG; ++sg)
#pragma unroll
                            for (int c = 0; c < 2; ++c)
                                if (own[sg] && boxed) {
                                    BX(F_ZU, sg, c) = mu0 / BX(F_SU, sg, c);
                                    BX(F_ZL, sg, c) = mu0 / BX(F_SL, sg, c);
                                }
                    }
                }
                if constexpr (MODE != 2) {   // the polish starts from the active set alone
                // xs = S u0 (u0 = clip(0, lb, ub); zero whenever the box contains 0)
                if (row_max(u0n) > 0.0) {
#pragma unroll
                    for (int sg = 0; sg < NSG; ++sg)
                        if (own[sg]) wr2((kseg[sg] - 1) * REC + O_BU, BX(F_U, sg, 0), BX(F_U, sg, 1));
                    rollout();
#pragma unroll
                    for (int sg = 0; sg < NSG; ++sg) rd4((kseg[sg] - 1) * REC + O_BX, xs[sg]);
                } else {
#pragma unroll
                    for (int sg = 0; sg < NSG; ++sg)
#pragma unroll
                        for (int a = 0; a < 4; ++a) xs[sg][a] = 0.0;
                }
#pragma unroll
                for (int s = 0; s < SL; ++s) {
                    const int sg = s / RSEG;
                    double c[4];
                    cf(s, c);
                    const double s0 = fmax(wv.w[s][lane] - dot4(c, xs[sg]), kSFloor);
                    s_[s] = valid(s) ? s0 : 1.0;
                    z_[s] = valid(s) ? (mu0 > 0.0 ? mu0 / s0 : 1.0) : 0.0;
                }
                }
                bnorm = 1.0 + row_max(bn);
                qnorm = 1.0 + row_max(qn);
                if constexpr (MODE == 0 && !HET) {
                    // A retry whose iterate the iteration launch saved resumes from it: the same point from which the
                    // single kernel carries on after a rejected polish (the trip below passes that polish over).
                    if (W.cnt && slot < nretry) {
                        const int64_t h = lst0 + S.index[slot];
                        if (h < W.state_cap) {
                            const double* st = W.state + h * kRicStateDoubles + j;
#pragma unroll
                            for (int s = 0; s < SL; ++s) {
                                s_[s] = st[s * GL];
                                z_[s] = st[(SL + s) * GL];
                            }
#pragma unroll
                            for (int sg = 0; sg < NSG; ++sg) {
#pragma unroll
                                for (int a = 0; a < 4; ++a) xs[sg][a] = st[(2 * SL + sg * 14 + a) * GL];
#pragma unroll
                                for (int c = 0; c < 2; ++c) {
                                    BX(F_U, sg, c) = st[(2 * SL + sg * 14 + 4 + c) * GL];
                                    BX(F_SU, sg, c) = st[(2 * SL + sg * 14 + 6 + c) * GL];
                                    BX(F_SL, sg, c) = st[(2 * SL + sg * 14 + 8 + c) * GL];
                                    BX(F_ZU, sg, c) = st[(2 * SL + sg * 14 + 10 + c) * GL];
                                    BX(F_ZL, sg, c) = st[(2 * SL + sg * 14 + 12 + c) * GL];
                                }
                            }
                            it = (int)W.pend_rec[h * kRicRecWords + kRicRecIt];
                        }
                    }
                }
            }
        }
        if constexpr (HET && !HL) {
            // a group has taken a new instance: the lanes of its matrix-core block (spread over all four rows of the
            // wave) fetch that instance's A, B and terminal cost -- one matrix entry per lane, as for a shared model
            if (__any(setup_now)) {
                const int64_t hb = (int64_t)__shfl((int)hinst, (mb % NG) * GL, 64);
                cA = P.het_A[hb * 16 + mr * 4 + mc];
                cBp = m_left ? P.het_B[hb * 8 + mr * 2 + mc] : 0.0;
                cB0r = P.het_B[hb * 8 + mr * 2];
                cB1r = P.het_B[hb * 8 + mr * 2 + 1];
                cPt = P.het_P[hb * 16 + (mr < mc ? mr : mc) * 4 + (mr < mc ? mc : mr)];
            }
        }
        RT_MARK(0);
        if (!__any(active)) continue;
        {
            // ================= residuals (R1 + B1) =================
            double mu = 0.0, rpn = 0.0, gun = 0.0, umax = 0.0, wz = 0.0, wzabs = 0.0;
            double lo = 0.0, scf = 0.0;
            bool polish = false;
            // polish: the active set (rows with s < z) as a bit per slot, fixed when the polish factorizes;
            // the polish loops test it instead of reading s and z (which they leave alone)
            // (shared-model kernels: bits 16.. hold the box rows of the lane's inputs, upper and lower bound of
            // input (sg, c) at 16 + 4 sg + 2 c and the bit above; per-instance kernels compare slack and multiplier)
            unsigned actm = 0;
#define RIC_REPOL (!HL && (act_next >> 31) != 0)   // this trip is the second attempt of a polish
            if constexpr (!HL) {
                if (RIC_REPOL) actm = act_next & 0xFFFFFFu;
            }
            auto act = [&](int s) { return ((actm >> s) & 1u) != 0; };
            auto box_bit = [](int sg, int c, int lower) { return 16 + (sg * 2 + c) * 2 + lower; };
            auto act_ub = [&](int sg, int c) {
                if constexpr (HL) return boxed && BX(F_SU, sg, c) < BX(F_ZU, sg, c);
                else return ((actm >> box_bit(sg, c, 0)) & 1u) != 0;
            };
            auto act_lb = [&](int sg, int c) {
                if constexpr (HL) return boxed && BX(F_SL, sg, c) < BX(F_ZL, sg, c);
                else return ((actm >> box_bit(sg, c, 1)) & 1u) != 0;
            };
            if (MODE != 2 && active) {
                double lz[NSG][4], musum = -0.0;
#pragma unroll
                for (int sg = 0; sg < NSG; ++sg)
#pragma unroll
                    for (int a = 0; a < 4; ++a) lz[sg][a] = -0.0;
                FOR_SLOTS_BEGIN
                    const double w = in.w;
                    const double gu = dot4(c, xs[sg]);
                    const double rp = gu + s_[s] - w;
                    rpn = fmax(rpn, fabs(rp));
                    gun = fmax(gun, fabs(gu));
                    musum = fma(s_[s], z_[s], musum);
#pragma unroll
                    for (int a = 0; a < 4; ++a) lz[sg][a] = fma(z_[s], c[a], lz[sg][a]);
                    wz = fma(w, z_[s], wz);
                    wzabs = fma(fabs(w), z_[s], wzabs);
                FOR_SLOTS_END
#pragma unroll
                for (int sg = 0; sg < NSG; ++sg)
#pragma unroll
                    for (int c = 0; c < 2; ++c) {
                        const int i = 2 * (kseg[sg] - 1) + c;
                        if (own[sg] && boxed) {
                            const double rpu = BX(F_U, sg, c) + BX(F_SU, sg, c) - sh.ub[i];
                            const double rpl = -BX(F_U, sg, c) + BX(F_SL, sg, c) + sh.lb[i];
                            rpn = fmax(rpn, fmax(fabs(rpu), fabs(rpl)));
                            musum = fma(BX(F_SU, sg, c), BX(F_ZU, sg, c), fma(BX(F_SL, sg, c), BX(F_ZL, sg, c), musum));
                            umax = fmax(umax, fabs(BX(F_U, sg, c)));
                        }
                    }
                // stage-N sum of lamZ, owners write lamZ_k [0..3], lamH_k = Qbar_k xs_k [4..7]
                double pn[4];
#pragma unroll
                for (int a = 0; a < 4; ++a) pn[a] = stageN_part(lz, a);
#pragma unroll
                for (int a = 0; a < 4; a += 2) stageN_sum2(pn[a], pn[a + 1]);
                wb();
#pragma unroll
                for (int sg = 0; sg < NSG; ++sg)
                    if (own[sg]) {
                        double v[4], h[4] = {-0.0, -0.0, -0.0, -0.0};
#pragma unroll
                        for (int a = 0; a < 4; ++a) v[a] = isN[sg] ? pn[a] : lz[sg][a];
                        add_qbar(kseg[sg] == N, xs[sg], h, 1.0);
                        wr4((kseg[sg] - 1) * REC + 0, v);
                        wr4((kseg[sg] - 1) * REC + 4, h);
                        // The passes' source of structural zeros, rewritten with the record's other inputs: the passes
                        // run for the whole wave, and while a group sits one out on records that hold non-finite
                        // leftovers (the pair check's NaN marks, an overflow on stale data), its lanes store 0 x that
                        // = NaN into this slot.
                        if constexpr (!HL) rec[(kseg[sg] - 1) * REC + O_ZERO] = 0.0;
                    }
                RT_MARK(1);
                mu = row_sum(musum) * inv_m;
                gun = fmax(gun, umax);   // (only their maximum is used)
                grp_reduce2<LPQ, OpMax>(rpn, gun);
                grp_reduce2<LPQ, OpSum>(wz, wzabs);
            }
            // B1 (per-instance models): psiZ_k = lamZ_k + A'psiZ_{k+1}, psiH likewise; gz_t = B'psiZ_{t+1},
            // redundantly in the 16 lanes of the group
            auto adjoint_scalar = [&]() {
                wb();
                    double pz[4] = {0.0, 0.0, 0.0, 0.0}, ph[4] = {0.0, 0.0, 0.0, 0.0};
                    double lzv[4], lhv[4];
                    rd4((N - 1) * REC + 0, lzv);
                    rd4((N - 1) * REC + 4, lhv);
#pragma unroll kUnrollAdj
                    for (int t = N - 1; t >= 0; --t) {
                        const int r = t * REC;
                        double nlz[4], nlh[4];
                        rd4((t >= 1 ? r - REC : 0), nlz);
                        rd4((t >= 1 ? r - REC : 0) + 4, nlh);
                        double nz[4], nh[4];
#pragma unroll
                        for (int a = 0; a < 4; ++a) {
                            double az = lzv[a], ah = lhv[a];
#pragma unroll
                            for (int c = 0; c < 4; ++c) {
                                az = M.A_(c, a, pz[c], az);
                                ah = M.A_(c, a, ph[c], ah);
                            }
                            nz[a] = az;
                            nh[a] = ah;
                        }
                        double gz[2], hs[2];
#pragma unroll
                        for (int c = 0; c < 2; ++c) {
                            double az = -0.0, ah = -0.0;
#pragma unroll
                            for (int a = 0; a < 4; ++a) {
                                pz[a] = nz[a];
                                ph[a] = nh[a];
                                az = M.B_(a, c, nz[a], az);
                                ah = M.B_(a, c, nh[a], ah);
                            }
                            gz[c] = az;
                            hs[c] = ah;
                            const double lb = sh.lb[2 * t + c], ub = sh.ub[2 * t + c];
                            lo += fmin(az * lb, az * ub);
                            scf = fma(fabs(az), fmax(fabs(lb), fabs(ub)), scf);
                        }
                        if (RIC_WRITER) {
                            wr2(r + 12, gz[0], gz[1]);
                            wr2(r + 14, hs[0], hs[1]);
                        }
#pragma unroll
                        for (int a = 0; a < 4; ++a) { lzv[a] = nlz[a]; lhv[a] = nlh[a]; }
                    }
                wb();
            };
            // B1: psiZ_k = lamZ_k + A'psiZ_{k+1}, psiH likewise; gz_t = B'psiZ_{t+1}
            if constexpr (HL) {
                if (active) adjoint_scalar();
            } else if constexpr (MODE != 2) {
                adjoint_mm();
            }
            if (MODE != 2 && active) {
                RT_MARK(2);
                double rdn = 0.0, hun = 0.0, gzn = 0.0;
#pragma unroll
                for (int sg = 0; sg < NSG; ++sg) {
                    const int r = (kseg[sg] - 1) * REC;
                    double gz0, gz1, hs0, hs1;
                    rd2(r + 12, gz0, gz1);
                    rd2(r + 14, hs0, hs1);
                    const double gzv[2] = {gz0, gz1}, hsv[2] = {hs0, hs1};
#pragma unroll
                    for (int c = 0; c < 2; ++c) {
                        if constexpr (!HL) {   // box-Farkas sums over the owned inputs (summed over the group below)
                            const double lb = sh.lb[2 * (kseg[sg] - 1) + c], ub = sh.ub[2 * (kseg[sg] - 1) + c];
                            if (own[sg]) {
                                lo += fmin(gzv[c] * lb, gzv[c] * ub);
                                scf = fma(fabs(gzv[c]), fmax(fabs(lb), fabs(ub)), scf);
                            }
                        }
                        const double hu = hsv[c] + M.Rmul(c, BX(F_U, sg, 0), BX(F_U, sg, 1));
                        const double gzb = gzv[c] + (boxed ? BX(F_ZU, sg, c) - BX(F_ZL, sg, c) : 0.0);
                        const double rd = hu + BX(F_Q, sg, c) + gzb;
                        BX(F_RD, sg, c) = own[sg] ? rd : 0.0;
                        if (own[sg]) {
                            rdn = fmax(rdn, fabs(rd));
                            hun = fmax(hun, fabs(hu));
                            gzn = fmax(gzn, fabs(gzb));
                        }
                    }
                }
                hun = fmax(hun, gzn);    // (only their maximum is used)
                grp_reduce2<LPQ, OpMax>(rdn, hun);
                if constexpr (!HL) grp_reduce2<LPQ, OpSum>(lo, scf);
                const double pscale = fmax(bnorm, 1.0 + gun);
                const double dscale = fmax(qnorm, 1.0 + hun);
                int done = -1;
                if (!isfinite(mu) || !isfinite(rdn)) {
                    done = CARMPC_NUMERICAL;
                } else {
                    const bool res_ok = rpn <= S.tol * pscale && rdn <= S.tol * dscale;
                    const bool last = it >= S.max_iter;
                    const double ptol = HL ? S.tol : fmax(POLISH_RES, S.tol);
                    const bool pres_ok = rpn <= ptol * pscale && rdn <= ptol * dscale;
                    polish = !polish_failed && ((pres_ok && mu <= (HL ? POLISH_MU_CONSERVATIVE : POLISH_MU)) || last);
                    if constexpr (MODE != 2) {
                        // round r of the pipeline (the single kernel after the last round included): the
                        // instance's first r polishes are known to be rejected -- that is why it is here;
                        // pass them over the way the single kernel carries on after a rejection: same
                        // iterate, no polish until a step has been taken
                        if (W.cnt && polish && npol < W.round && slot < nretry) {
                            ++npol;
                            polish = false;
                        }
                    }
                    if (!polish) {
                        if (last) done = CARMPC_MAX_ITER;
                        else if (res_ok && mu <= S.tol_mu) done = CARMPC_OPTIMAL;
                        else if (p > 0 && lo - wz > 1e-12 * (scf + wzabs)) done = CARMPC_PRIMAL_INFEASIBLE;
                    }
                }
                if (done >= 0) {
                    finish(done, false);
                    active = false;
                    polish = false;
                }
                if constexpr (MODE == 1) {
                    if (polish) {
                        // hand the instance to the polish launch: active rows (s < z) and active box rows
                        unsigned m = 0;
                        for_used([&](const int s) __attribute__((always_inline)) { m |= (s_[s] < kAct * z_[s] ? 1u : 0u) << s; });
#pragma unroll
                        for (int sg = 0; sg < NSG; ++sg)
#pragma unroll
                            for (int c = 0; c < 2; ++c)
                                if (own[sg] && boxed) {
                                    m |= (BX(F_SU, sg, c) < kAct * BX(F_ZU, sg, c) ? 1u : 0u) << box_bit(sg, c, 0);
                                    m |= (BX(F_SL, sg, c) < kAct * BX(F_ZL, sg, c) ? 1u : 0u) << box_bit(sg, c, 1);
                                }
                        unsigned pos = 0;
                        if (j == 0) pos = atomicAdd(W.cnt + kRicClaimStride * seg + 4 * W.round + 1, 1u);
                        pos = __shfl(pos, lane & ~(GL - 1), 64);
                        uint32_t* hrec = W.pend_rec + (lst0 + pos) * kRicRecWords;
                        // record word j16 = the masks of both segments of table lane j16, whichever lanes hold them
                        if constexpr (LPQ == 32) {
                            if ((lane >> 4) & 1) m = ((m & 0xFFu) << RSEG) | ((m & 0xF0000u) << 4);
                            m |= (unsigned)__shfl_xor((int)m, 16, 64);
                        }
                        if (j < G16) hrec[j] = m;
                        if (j < NX) reinterpret_cast<double*>(hrec + kRicRecX0)[j] = x0[inst * NX + j];
                        if (j == 0) {
                            hrec[kRicRecRow] = (uint32_t)inst;
                            hrec[kRicRecIt] = (uint32_t)it;
                        }
                        // the iterate itself, for the final launch should the polish be rejected (RicWork::state):
                        // [quantity][lane of the group], every lane its own slots and inputs
                        if ((int64_t)(lst0 + pos) < W.state_cap) {
                            static_assert((2 * SL + 14 * NSG) * GL <= kRicStateDoubles, "state record");
                            double* st = W.state + (int64_t)(lst0 + pos) * kRicStateDoubles + j;
#pragma unroll
                            for (int s = 0; s < SL; ++s) {
                                st[s * GL] = s_[s];
                                st[(SL + s) * GL] = z_[s];
                            }
#pragma unroll
                            for (int sg = 0; sg < NSG; ++sg) {
#pragma unroll
                                for (int a = 0; a < 4; ++a) st[(2 * SL + sg * 14 + a) * GL] = xs[sg][a];
#pragma unroll
                                for (int c = 0; c < 2; ++c) {
                                    st[(2 * SL + sg * 14 + 4 + c) * GL] = BX(F_U, sg, c);
                                    st[(2 * SL + sg * 14 + 6 + c) * GL] = BX(F_SU, sg, c);
                                    st[(2 * SL + sg * 14 + 8 + c) * GL] = BX(F_SL, sg, c);
                                    st[(2 * SL + sg * 14 + 10 + c) * GL] = BX(F_ZU, sg, c);
                                    st[(2 * SL + sg * 14 + 12 + c) * GL] = BX(F_ZL, sg, c);
                                }
                            }
                        }
                        finish(0, false, false);
                        active = false;
                        polish = false;
                    }
                }
            }
            if constexpr (MODE == 1) polish = false;   // (compile-time fact for the code below)
            if constexpr (MODE == 2) {
                // the hand-off record replaces residuals and decisions
                polish = true;
                if (active && !RIC_REPOL) {
                    const uint32_t* hrec = W.pend_rec + (lst0 + slot) * kRicRecWords;
                    actm = hrec[j16];
                    if constexpr (LPQ == 32) actm = ((lane >> 4) & 1) ? ((actm >> RSEG) & 0xFFu) | ((actm >> 4) & 0xF0000u) : actm & 0xF00FFu;
                    it = (int)hrec[kRicRecIt];
                }
            }
            const bool any_polish = __any(polish);
            RT_MARK(3);
#ifdef CARMPC_HET_TWO_FORM   // build-only switch for code inspection (tools/kernel_meta.py); never part of the product library
            constexpr bool kInterleaved = false;
#else
            constexpr bool kInterleaved = HET;
#endif
            if constexpr (kInterleaved) {
                // per-instance models: both forms interleaved per group (flags per lane)
                if (!__any(active)) continue;
#define RIC_GO active
#define RIC_POLISH polish
#define RIC_ANY_POLISH any_polish
#include "ipm_riccati_solve.inc"
#undef RIC_GO
#undef RIC_POLISH
#undef RIC_ANY_POLISH
            } else {
                // Shared model: the rest of the trip exists in two compile-time forms, the interior-point step and the
                // active-set polish.  The single kernel (MODE 0) runs the polish form first for the groups that polish
                // in this trip, then the step form for the others: each form keeps only its own vectors live, where
                // code that interleaves them per group keeps the union (and spilled to scratch).  MODE 1 / 2
                // instantiate one form each.
                auto solve_phase = [&](auto pol_c, bool go) __attribute__((always_inline)) {
                    constexpr bool POL = decltype(pol_c)::value;
                    if (!__any(go)) return;
#define RIC_GO go
#define RIC_POLISH POL
#define RIC_ANY_POLISH POL
#include "ipm_riccati_solve.inc"
#undef RIC_GO
#undef RIC_POLISH
#undef RIC_ANY_POLISH
                };
                if constexpr (MODE != 1) {
                    if (any_polish) solve_phase(std::true_type{}, active && polish);
                }
                if constexpr (MODE != 2) solve_phase(std::false_type{}, active && !polish);
            }
        }
    }
    RT_FLUSH();
    }   // segments
#undef RIC_REPOL
}

// Lanes per QP of each launch kind (MODE 1 iterations, MODE 2 polish, MODE 0 single kernel; see LPQ at the
// kernel).  A workgroup always carries 16 QPs -- what one CU's LDS holds at N = 20 --, as 4 wavefronts of
// four 16-lane groups (one wave per SIMD) or 8 wavefronts of two 32-lane groups (two waves per SIMD, 256
// registers each).  Measured on the 131,072-instance mixed shard, QP/s: all launches with 16 lanes 19.9M; the
// iteration launch with 32 lanes 21.0M; iteration and single kernel 21.4M; all three 21.6M (and only with all
// three on one layout do the pipeline and the single kernel perform bit-identical arithmetic).
#ifndef CARMPC_RIC_LPQ_M1
#define CARMPC_RIC_LPQ_M1 32
#endif
#ifndef CARMPC_RIC_LPQ_M2
#define CARMPC_RIC_LPQ_M2 32
#endif
#ifndef CARMPC_RIC_LPQ_M0
#define CARMPC_RIC_LPQ_M0 32
#endif
#ifndef CARMPC_RIC_LPQ_HET   // per-instance models: 14.9M QP/s with 16 lanes, 17.3M with 32 (131,072 instances)
#define CARMPC_RIC_LPQ_HET 32
#endif
constexpr int ric_lpq(int mode, bool het) {
    return het ? CARMPC_RIC_LPQ_HET : mode == 1 ? CARMPC_RIC_LPQ_M1 : mode == 2 ? CARMPC_RIC_LPQ_M2 : CARMPC_RIC_LPQ_M0;
}
// Wavefronts per workgroup: eight with one slot segment per lane (two waves per SIMD at 256 registers), four with
// two segments (one wave per SIMD), fewer where a CU's LDS (160 KB) does not hold that many.
template <int N, int LPQ, int SEGS = 32 / LPQ>
constexpr int ric_wpb_for() {
    return ric_wpb_rec<N, LPQ, SEGS, ric_rec<N, LPQ, SEGS>()>();
}
// Horizons with a compiled instantiation (others run on the staged / dense kernels) ...
#define RIC_FOR_EACH_N(X, ...) X(5, __VA_ARGS__) X(10, __VA_ARGS__) X(15, __VA_ARGS__) X(20, __VA_ARGS__) X(25, __VA_ARGS__)
// ... and those that also have the four-QPs-per-wave form (16 lanes, one segment) for shared-model problems.
#define RIC_FOR_EACH_N_ONESEG(X, ...) X(5, __VA_ARGS__) X(10, __VA_ARGS__)
#ifdef CARMPC_NO_ONESEG   // A/B builds
constexpr bool ric_has_oneseg(int) { return false; }
#else
constexpr bool ric_has_oneseg(int N) { return N == 5 || N == 10; }
#endif

// The kernel is compiled in several translation units (ipm_riccati_m0 / _m1 / _m2 / _het.hip: one per launch
// kind, each with the code-generation flags that suit it, carmpc_amd/build.py) and launched from
// ipm_riccati.hip, which only declares the instantiations.
#define RIC_KERNEL_ARGS RicSegs, RicWork, const double*, const double*, double*, int64_t, int32_t*, int32_t*, Settings
#define RIC_INST_N(NN, PREFIX, HET, MODE)                                                                              \
    PREFIX template __global__ void                                                                                   \
    ipm_riccati_kernel<NN, ric_wpb_for<NN, ric_lpq(MODE, HET)>(), BicycleModel, HET, MODE, ric_lpq(MODE, HET)>(RIC_KERNEL_ARGS); \
    PREFIX template __global__ void                                                                                   \
    ipm_riccati_kernel<NN, ric_wpb_for<NN, ric_lpq(MODE, HET)>(), DenseModel, HET, MODE, ric_lpq(MODE, HET)>(RIC_KERNEL_ARGS);
#define RIC_INST_N1(NN, PREFIX, MODE)                                                                                  \
    PREFIX template __global__ void ipm_riccati_kernel<NN, ric_wpb_for<NN, 16, 1>(), BicycleModel, false, MODE, 16, 1>(RIC_KERNEL_ARGS); \
    PREFIX template __global__ void ipm_riccati_kernel<NN, ric_wpb_for<NN, 16, 1>(), DenseModel, false, MODE, 16, 1>(RIC_KERNEL_ARGS);
#define RIC_INST(PREFIX, HET, MODE) RIC_FOR_EACH_N(RIC_INST_N, PREFIX, HET, MODE)
#define RIC_INST_ONESEG(PREFIX, MODE) RIC_FOR_EACH_N_ONESEG(RIC_INST_N1, PREFIX, MODE)

}  // namespace ric
}  // namespace carmpc
