// lanes.h -- cross-lane and arithmetic primitives for gfx950 solve kernels.
#pragma once

#include <hip/hip_runtime.h>
#include <math.h>

namespace carmpc {
namespace lanes {

// DPP butterflies inside a 16-lane row: quad xor 1, quad xor 2, half-row mirror, row
// mirror.  Both lanes of each pair combine the same two operands, so every lane of the
// row ends with a bitwise-identical result (row-uniform decisions stay consistent).
constexpr int DPP_QXOR1 = 0xB1, DPP_QXOR2 = 0x4E, DPP_HMIRROR = 0x141, DPP_MIRROR = 0x140;

template <int CTRL>
__device__ __forceinline__ double dpp_d(double v) {
    const unsigned long long b = __builtin_bit_cast(unsigned long long, v);
    const int lo = __builtin_amdgcn_update_dpp(0, (int)(unsigned)b, CTRL, 0xf, 0xf, false);
    const int hi = __builtin_amdgcn_update_dpp(0, (int)(unsigned)(b >> 32), CTRL, 0xf, 0xf, false);
    return __builtin_bit_cast(double, ((unsigned long long)(unsigned)hi << 32) | (unsigned)lo);
}
struct OpSum { __device__ static double f(double a, double b) { return a + b; } };
struct OpMax { __device__ static double f(double a, double b) { return fmax(a, b); } };
struct OpMin { __device__ static double f(double a, double b) { return fmin(a, b); } };

// reduction over each 16-lane row (one QP group), result in every lane of the row
template <class Op>
__device__ __forceinline__ double row_reduce(double v) {
    v = Op::f(v, dpp_d<DPP_QXOR1>(v));
    v = Op::f(v, dpp_d<DPP_QXOR2>(v));
    v = Op::f(v, dpp_d<DPP_HMIRROR>(v));
    return Op::f(v, dpp_d<DPP_MIRROR>(v));
}
__device__ __forceinline__ double row_sum(double v) { return row_reduce<OpSum>(v); }
__device__ __forceinline__ double row_max(double v) { return row_reduce<OpMax>(v); }
__device__ __forceinline__ double row_min(double v) { return row_reduce<OpMin>(v); }

// Exchange between the two 16-lane rows of a 32-lane half-wave (lane l <-> lane l ^ 16) with
// v_permlane16_swap_b32 (gfx950: swaps the odd rows of its first operand with the even rows of its
// second).  Given two copies of x, the first ends up holding the even row's value in both rows and
// the second the odd row's value, so every lane of the pair combines (even, odd) in the same order:
// the result is bitwise identical in both rows.
template <class Op>
__device__ __forceinline__ double pair_rows(double v) {
    const unsigned long long b = __builtin_bit_cast(unsigned long long, v);
    const unsigned lo = (unsigned)b, hi = (unsigned)(b >> 32);
    const auto rl = __builtin_amdgcn_permlane16_swap(lo, lo, false, false);
    const auto rh = __builtin_amdgcn_permlane16_swap(hi, hi, false, false);
    const double ev = __builtin_bit_cast(double, ((unsigned long long)rh[0] << 32) | rl[0]);
    const double od = __builtin_bit_cast(double, ((unsigned long long)rh[1] << 32) | rl[1]);
    return Op::f(ev, od);
}
// Two reductions over a 32-lane group for little more than the price of one: the lower row takes over `a` and the
// upper row `b` (one swap: afterwards the first register holds the lower lane's value in both rows, the second the
// upper lane's), one 16-lane butterfly then reduces `a` in the lower row and `b` in the upper row at the same
// time, and a last swap hands each row the other's total.  Both results bitwise uniform over the 32 lanes.
__device__ __forceinline__ void swap16(double& x, double& y) {   // rows of x: (x.even, y.even); of y: (x.odd, y.odd)
    const unsigned long long bx = __builtin_bit_cast(unsigned long long, x), by = __builtin_bit_cast(unsigned long long, y);
    const auto rl = __builtin_amdgcn_permlane16_swap((unsigned)bx, (unsigned)by, false, false);
    const auto rh = __builtin_amdgcn_permlane16_swap((unsigned)(bx >> 32), (unsigned)(by >> 32), false, false);
    x = __builtin_bit_cast(double, ((unsigned long long)rh[0] << 32) | rl[0]);
    y = __builtin_bit_cast(double, ((unsigned long long)rh[1] << 32) | rl[1]);
}
// Lanes 8..15 of every DPP row take the value of the lane 8 below them, lanes 0..7 keep theirs (row_shr:8 into
// banks 2 and 3).  In the matrix-core layout (block b = lanes 4 b .. 4 b + 3 of each row) that copies blocks 0, 1
// onto blocks 2, 3.
__device__ __forceinline__ double upper_half_from_lower(double v) {
    const unsigned long long b = (unsigned long long)__double_as_longlong(v);
    const int lo = __builtin_amdgcn_update_dpp((int)(unsigned)b, (int)(unsigned)b, 0x118, 0xf, 0xc, false);
    const int hi = __builtin_amdgcn_update_dpp((int)(unsigned)(b >> 32), (int)(unsigned)(b >> 32), 0x118, 0xf, 0xc, false);
    return __longlong_as_double((long long)(((unsigned long long)(unsigned)hi << 32) | (unsigned)lo));
}

template <int LPQ, class Op>
__device__ __forceinline__ void grp_reduce2(double& a, double& b) {
    if constexpr (LPQ == 32) {
        double x = a, y = b;
        swap16(x, y);                       // x: (a_lower, b_lower), y: (a_upper, b_upper)  [even row, odd row]
        double t = row_reduce<Op>(Op::f(x, y));
        double u = t;
        swap16(t, u);                       // t: total of a in both rows, u: total of b
        a = t;
        b = u;
    } else {
        a = row_reduce<Op>(a);
        b = row_reduce<Op>(b);
    }
}
// The same for two sums whose addends all sit in the UPPER row of each 32-lane group (the lower row's inputs are
// ignored): b's addends move to the lower row, one butterfly, and the upper row gets b's total back.  Results valid
// in the upper row only.
__device__ __forceinline__ void upper_row_sum2(double& a, double& b) {
    double x = b, y = a;
    swap16(x, y);                           // y: (b_upper, a_upper)
    y = row_reduce<OpSum>(y);               // lower row: total of b, upper row: total of a
    double z = y;
    swap16(z, y);                           // z.odd row = y.even row = total of b
    a = y;                                  // (upper row: total of a)
    b = z;
}
// reduction over each group of LPQ lanes (LPQ = 16: one row; 32: two rows), result in every lane of the group
template <int LPQ, class Op>
__device__ __forceinline__ double grp_reduce(double v) {
    static_assert(LPQ == 16 || LPQ == 32, "lanes per group");
    if constexpr (LPQ == 32) v = pair_rows<Op>(v);
    return row_reduce<Op>(v);
}

// Reciprocal: v_rcp_f64 is good to ~2^-25 (measured, tools/probe/rcp_probe.hip: max 2.5e8 ulp), so
// one Newton step leaves <= 11 ulp (mean 0.6) -- enough for the scalings it is used for (z/s, step
// ratios, pivots; the IPM's iterates are insensitive at that level and statuses and iteration
// counts are unchanged on every test vector).  CARMPC_FRCP_NR2 adds the second step (<= 1 ulp).
__device__ __forceinline__ double frcp(double b) {
    double r = __builtin_amdgcn_rcp(b);
    r = fma(fma(-b, r, 1.0), r, r);
#ifdef CARMPC_FRCP_NR2
    r = fma(fma(-b, r, 1.0), r, r);
#endif
    return r;
}
// Reciprocal square root: hardware approximation + two Newton steps.
__device__ __forceinline__ double frsq(double a) {
    double r = __builtin_amdgcn_rsq(a);
    const double h = 0.5 * a;
    r = r * fma(-h * r, r, 1.5);
    return r * fma(-h * r, r, 1.5);
}
// step to the boundary along dv (inf when dv >= 0)
__device__ __forceinline__ double ratio(double v, double dv) {
    const double r = -v * __builtin_amdgcn_rcp(dv);
    return dv < 0.0 ? r : INFINITY;
}
// index of the symmetric 4x4 entry (a <= b) in the packed 10-vector
__host__ __device__ constexpr int sym10(int a, int b) {
    return a <= b ? a * 4 - a * (a - 1) / 2 + (b - a) : b * 4 - b * (b - 1) / 2 + (a - b);
}

}  // namespace lanes
}  // namespace carmpc
