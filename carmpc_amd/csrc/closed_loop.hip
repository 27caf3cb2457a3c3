// Closed-loop simulation on the device: the examples' runner loops
// (examples/run_MPCStateFB.py:26-43, examples/run_MPCOutputFB.py:28-50) for a batch of
// independent cars, with the plant (simulator.py:51-69,83-97,99-118), the observers
// (mpc.py:439-448, 598-612) and the QP kernels all on the GPU and no host round trip per
// control step.
//
// One loop index i per launch pair, around the QP launch:
//   loop_advance_kernel  check_input -> plant step -> (every steps_update) observer
//   <QP kernel on the live slots: S.index / S.count>
//   loop_finish_kernel   QP status -> outcome, goal / time-out test, compaction of the
//                        still-running instances into the other slot list
// Live-instance lists are double-buffered; the count lives on the device, so the QP
// kernels size their work from it without a host read.
#include "carmpc_internal.h"

namespace carmpc {

namespace {

__global__ void loop_advance_kernel(LoopArgs a, int32_t i) {
    const int64_t slot = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (slot == 0) *a.cnt_next = 0;   // the other list is rebuilt by loop_finish_kernel
    if (slot >= *a.cnt_cur) return;
    const int64_t b = a.idx_cur[slot];
    double* st = a.state + b * NX;
    const double acc = a.u[b * a.ld_u + 0], delta = a.u[b * a.ld_u + 1];
    if (input_rejected(acc, delta)) {   // check_input, clip=False (simulator.py:83-97)
        a.outcome[b] = CARMPC_LOOP_INPUT_VIOLATION;   // the runner stops at the assertion, before the step
        a.steps[b] = i;
        return;
    }
    // forward Euler of the kinematic bicycle (simulator.py:51-69)
    const double x = st[0], y = st[1], psi = st[2], v = st[3];
    const double t = tan(delta);
    double xn[NX];
    xn[0] = v * cos(psi) * a.dt + x;
    xn[1] = v * sin(psi) * a.dt + y;
    xn[2] = v / a.l1 * t * a.dt + psi;
    xn[3] = acc * a.dt + v;
#pragma unroll
    for (int k = 0; k < NX; ++k) st[k] = xn[k];
    if (a.mode == 0 || i % a.steps_update != 0) return;
    // observer on y = C x (the runners step the plant without an output disturbance)
    double* xh = a.xhat + b * NX;
    double xe[NX], innov[8];
#pragma unroll
    for (int k = 0; k < NX; ++k) xe[k] = xh[k];
    const double d = a.mode == 2 ? a.dhat[b] : 0.0;
    for (int r = 0; r < a.ny; ++r) {
        double yr = 0.0, v2 = 0.0;
#pragma unroll
        for (int k = 0; k < NX; ++k) {
            yr += a.C[r * NX + k] * xn[k];
            v2 += a.C[r * NX + k] * xe[k];
        }
        double e = yr - v2;
        if (a.mode == 2) e -= a.Cd[r] * d;
        innov[r] = e;
    }
    double out[NX];
#pragma unroll
    for (int r = 0; r < NX; ++r) {
        double v3 = 0.0;
#pragma unroll
        for (int k = 0; k < NX; ++k) v3 += a.A[r * NX + k] * xe[k];
        if (a.mode == 2) v3 += a.Bd[r] * d;
        v3 += a.B[r * 2 + 0] * acc + a.B[r * 2 + 1] * delta;   // previous_u = the input held by the plant
        for (int q = 0; q < a.ny; ++q) v3 += a.L[r * a.ny + q] * innov[q];
        out[r] = v3;
    }
#pragma unroll
    for (int k = 0; k < NX; ++k) xh[k] = out[k];
    if (a.mode == 2) {
        double dn = d;
        for (int q = 0; q < a.ny; ++q) dn += a.L2[q] * innov[q];
        a.dhat[b] = dn;
    }
}

__global__ void loop_finish_kernel(LoopArgs a, int32_t i) {
    const int64_t slot = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (slot >= *a.cnt_cur) return;
    const int64_t b = a.idx_cur[slot];
    if (a.outcome[b] != CARMPC_LOOP_RUNNING) return;   // input violation in this step
    if (i % a.steps_update == 0) {
        const int32_t s = a.qp_status[b];
        if (s != CARMPC_OPTIMAL) {
            // infinite cost -> OutsideTheRegionOfAttractionError (mpc.py:336-338, 479-481)
            a.outcome[b] = s == CARMPC_PRIMAL_INFEASIBLE ? CARMPC_LOOP_INFEASIBLE : CARMPC_LOOP_SOLVER_FAILURE;
            a.steps[b] = i + 1;
            return;
        }
    }
    const double* st = a.state + b * NX;
    if (a.goal_tol > 0.0) {
        bool at = true;
#pragma unroll
        for (int k = 0; k < NX; ++k) at = at && fabs(st[k] - a.goal[k]) <= a.goal_tol;
        if (at) {   // run_MPCStateFB.py:40
            a.outcome[b] = CARMPC_LOOP_REACHED;
            a.steps[b] = i + 1;
            return;
        }
    }
    if (i >= a.last_step) {   // run_MPCStateFB.py:40 (i > 30/DT), run_MPCOutputFB.py:48 (i >= 15/DT)
        a.outcome[b] = CARMPC_LOOP_TIMEOUT;
        a.steps[b] = i + 1;
        return;
    }
    a.idx_next[atomicAdd(a.cnt_next, 1)] = (int32_t)b;
}

__global__ void loop_init_kernel(LoopArgs a) {
    const int64_t b = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (b == 0) *a.cnt_cur = (int32_t)a.batch;
    if (b >= a.batch) return;
    a.idx_cur[b] = (int32_t)b;
    a.outcome[b] = CARMPC_LOOP_RUNNING;
    a.steps[b] = 0;
    for (int c = 0; c < a.ld_u; ++c) a.u[b * a.ld_u + c] = 0.0;   // control_input = [0, 0] before the first step
}

unsigned blocks_for(int64_t n) { return (unsigned)((n + 255) / 256); }

}  // namespace

hipError_t launch_loop_init(const LoopArgs& a, hipStream_t s) {
    hipLaunchKernelGGL(loop_init_kernel, dim3(blocks_for(a.batch)), dim3(256), 0, s, a);
    return hipGetLastError();
}
hipError_t launch_loop_advance(const LoopArgs& a, int32_t i, hipStream_t s) {
    hipLaunchKernelGGL(loop_advance_kernel, dim3(blocks_for(a.batch)), dim3(256), 0, s, a, i);
    return hipGetLastError();
}
hipError_t launch_loop_finish(const LoopArgs& a, int32_t i, hipStream_t s) {
    hipLaunchKernelGGL(loop_finish_kernel, dim3(blocks_for(a.batch)), dim3(256), 0, s, a, i);
    return hipGetLastError();
}

}  // namespace carmpc
