// ipm_riccati.hip -- launch side of the grouped stage-form IPM kernel (ipm_riccati_kernel.h): grid sizing,
// dispatch by horizon and model structure, the three-launch pipeline, several problems per launch.
#include <mutex>
#include "ipm_riccati_kernel.h"

namespace carmpc {

using namespace ric;
namespace ric {
RIC_INST(extern, false, 0)
RIC_INST(extern, false, 1)
RIC_INST(extern, false, 2)
RIC_INST(extern, true, 0)
RIC_INST_ONESEG(extern, 0)
RIC_INST_ONESEG(extern, 1)
RIC_INST_ONESEG(extern, 2)
}  // namespace ric

bool riccati_supported_N(int N) {
#define RIC_IS_N(NN, ...) if (N == NN) return true;
    RIC_FOR_EACH_N(RIC_IS_N, )
#undef RIC_IS_N
    return false;
}

bool riccati_oneseg_N(int N) { return ric_has_oneseg(N); }
constexpr int64_t kRicOneSegMin = 16384;
#ifndef CARMPC_RIC_TAIL_DIV
#define CARMPC_RIC_TAIL_DIV 32
#endif
constexpr int kRicTailDiv = CARMPC_RIC_TAIL_DIV;
#ifndef CARMPC_RIC_SAVE_STATE   // 0: A/B builds without the saved iterates (every retry starts over)
#define CARMPC_RIC_SAVE_STATE 1
#endif
constexpr bool kRicSaveState = CARMPC_RIC_SAVE_STATE != 0;

namespace {
// grid = one workgroup per CU slot (persistent workgroups), at most one per 16 instances
template <int WPB, int LPQ, class Kern>
hipError_t ric_launch(Kern kern, const RicSegs& T, const RicWork& W, int64_t total, const double* x0, const double* xref,
                      double* u_out, int64_t ld_u, int32_t* status, int32_t* iters, const Settings& s, hipStream_t stream) {
    int dev = 0, cus = 0, per_cu = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e != hipSuccess) return e;
    e = hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    if (e != hipSuccess) return e;
    e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, (const void*)kern, WPB * 64, 0);
    if (e != hipSuccess) return e;
    if (per_cu < 1) per_cu = 1;
    const int64_t per_block = (int64_t)WPB * (64 / LPQ);
    int64_t grid = std::min<int64_t>((int64_t)cus * per_cu, (total + per_block - 1) / per_block);
    if (grid < 1) grid = 1;
    hipLaunchKernelGGL(kern, dim3((unsigned)grid), dim3(WPB * 64), 0, stream, T, W, x0, xref, u_out, ld_u, status, iters, s);
    return hipGetLastError();
}
template <bool HET, int MODE>
hipError_t ric_dispatch(const RicSegs& T, const RicWork& W, int64_t total, const double* x0, const double* xref,
                        double* u_out, int64_t ld_u, int32_t* status, int32_t* iters, const Settings& s, hipStream_t stream,
                        int* unsupported) {
    const bool bike = T.P[0].ric == 2;
    constexpr int LQ = ric_lpq(MODE, HET);
    if (HET && !bike) {   // per-instance models are always bicycle-structured (hetero.hip::linearize_kernel)
        *unsupported = 1;
        return hipErrorInvalidValue;
    }
#define RIC_GO(NN, MODEL)                                                                                              \
    ric_launch<ric_wpb_for<NN, LQ>(), LQ>(ipm_riccati_kernel<NN, ric_wpb_for<NN, LQ>(), MODEL, HET, MODE, LQ>, T, W, total, x0, xref, \
                                          u_out, ld_u, status, iters, s, stream)
#define RIC_GO1(NN, MODEL)                                                                                             \
    ric_launch<ric_wpb_for<NN, 16, 1>(), 16>(ipm_riccati_kernel<NN, ric_wpb_for<NN, 16, 1>(), MODEL, false, MODE, 16, 1>, T, W, total, \
                                             x0, xref, u_out, ld_u, status, iters, s, stream)
#define RIC_CASE(NN, ...) case NN: return bike ? RIC_GO(NN, BicycleModel) : RIC_GO(NN, DenseModel);
#define RIC_CASE1(NN, ...) case NN: return bike ? RIC_GO1(NN, BicycleModel) : RIC_GO1(NN, DenseModel);
    if constexpr (!HET) {
        // rows in the first slot segment alone (short horizons): four QPs per wavefront
        // (from kRicOneSegMin instances on: a small batch spreads over twice the wavefronts, hence CUs, with two QPs per
        // wave, and its time is the latency of one solve -- 4,096 instances at N = 10: 15.0M QP/s with two per wave,
        // 13.7M with four; 65,536: 29.1M against 37.4M; 131,072: 32.7M against 43.3M)
        if (T.P[0].rone && ric_has_oneseg(T.P[0].N) && total >= kRicOneSegMin) {
            switch (T.P[0].N) {
                RIC_FOR_EACH_N_ONESEG(RIC_CASE1, )
                default: break;
            }
        }
    }
    switch (T.P[0].N) {
        RIC_FOR_EACH_N(RIC_CASE, )
        default: *unsupported = 1; return hipErrorInvalidValue;
    }
#undef RIC_CASE1
#undef RIC_GO1
#undef RIC_CASE
#undef RIC_GO
}

// The launch pipeline: rounds of iterations with hand-off and lock-step polish, then the single kernel for
// what the last round rejected (see MODE at the kernel).  Work lists and counters live for the call,
// stream-ordered.  The last launch usually finds an empty list; its workgroups read the count and return.
// The pipeline's work memory (lists, counters, saved iterates: up to kRicStateMaxBytes + 132 B per instance, per call
// in flight) is stream-ordered memory from a pool of the library's own per device, which keeps what a call frees for
// the next one (release threshold: none) -- a caller that synchronises after every call would otherwise pay a device
// allocation of that size per call.  Without such a pool (creation refused) the device's default pool serves.
hipMemPool_t pipeline_pool() {
    static std::mutex mu;
    static hipMemPool_t pools[64] = {};
    static bool tried[64] = {};
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return nullptr;
    std::lock_guard<std::mutex> lock(mu);
    if (!tried[dev]) {
        tried[dev] = true;
        hipMemPoolProps props{};
        props.allocType = hipMemAllocationTypePinned;
        props.handleTypes = hipMemHandleTypeNone;
        props.location.type = hipMemLocationTypeDevice;
        props.location.id = dev;
        hipMemPool_t p = nullptr;
        if (hipMemPoolCreate(&p, &props) == hipSuccess) {
            uint64_t keep = UINT64_MAX;
            if (hipMemPoolSetAttribute(p, hipMemPoolAttrReleaseThreshold, &keep) == hipSuccess) pools[dev] = p;
            else (void)hipMemPoolDestroy(p);
        }
        (void)hipGetLastError();   // (a refused pool is not an error of the call)
    }
    return pools[dev];
}
hipError_t pipeline_alloc(void** ptr, size_t bytes, hipStream_t stream) {
    if (hipMemPool_t pool = pipeline_pool()) return hipMallocFromPoolAsync(ptr, bytes, pool, stream);
    return hipMallocAsync(ptr, bytes, stream);
}

hipError_t ric_pipeline(const RicSegs& T, int64_t total, const double* x0, const double* xref, double* u_out, int64_t ld_u,
                        int32_t* status, int32_t* iters, const Settings& s, hipStream_t stream, int* unsupported) {
    static_assert(kRicRounds == 1, "the retry list names hand-off records: a second round of iterations would need their rows");
    const size_t n = (size_t)total, ncnt = (size_t)kRicClaimStride * kRicMaxSeg;
    const size_t bytes = sizeof(unsigned) * ncnt + sizeof(uint32_t) * kRicRecWords * n + sizeof(int32_t) * n;
    static_assert(kRicLanes == kRicRecX0 && (kRicClaimStride * kRicMaxSeg * sizeof(unsigned)) % 128 == 0, "record layout");
    char* base = nullptr;
    hipError_t e = pipeline_alloc(reinterpret_cast<void**>(&base), bytes, stream);
    if (e != hipSuccess) return e;
    RicWork W{};
    W.cnt = reinterpret_cast<unsigned*>(base);
    W.pend_rec = reinterpret_cast<uint32_t*>(W.cnt + ncnt);   // (ncnt words = 256 bytes: records stay line-aligned)
    W.retry_idx = reinterpret_cast<int32_t*>(W.pend_rec + (size_t)kRicRecWords * n);
    // saved iterates of the hand-offs (RicWork::state); without the memory every retry starts over, as beyond the cap
    const size_t state_one = sizeof(double) * kRicStateDoubles;
    W.state_cap = kRicSaveState ? (int64_t)std::min(n, kRicStateMaxBytes / state_one) : 0;
    void* state = nullptr;
    if (W.state_cap > 0 && pipeline_alloc(&state, state_one * (size_t)W.state_cap, stream) != hipSuccess) {
        (void)hipGetLastError();
        state = nullptr;
        W.state_cap = 0;
    }
    W.state = static_cast<double*>(state);
    e = launch_zero_u32(W.cnt, (int)ncnt, stream);
    // the final launch's fresh instances (RicWork::tail): 1/kRicTailDiv of every segment when its retries start over
    // (no memory for their iterates, or more hand-offs than the memory holds).  Resumed retries are short -- three
    // trips on average instead of nine, eleven instead of twenty-one at most -- and fresh instances beside them only
    // add their own stragglers: 27.15M QP/s without, 27.13M with 1/128, 26.8M with 1/32 on the 131,072-instance shard.
#ifdef CARMPC_RIC_TAIL_ENV   // experiment builds only: divisor from the environment
    static const int tail_div = [] {
        const char* v = getenv("CARMPC_RIC_TAIL_DIV");
        return v ? atoi(v) : kRicTailDiv;
    }();
#else
    constexpr int tail_div = kRicTailDiv;
#endif
    const bool fill = tail_div > 0 && W.state_cap < (int64_t)n;
    for (int j = 0; j < T.nseg; ++j) W.tail[j] = fill ? (int32_t)((T.off[j + 1] - T.off[j]) / tail_div) : 0;
    // rounds of (iterations, polish): round r takes the instances whose first r polishes were rejected
    // (two or three per cent after round 0); what is left after the last round goes to the single kernel
    for (W.round = 0; W.round < kRicRounds && e == hipSuccess; ++W.round) {
        e = ric_dispatch<false, 1>(T, W, total, x0, xref, u_out, ld_u, status, iters, s, stream, unsupported);
        if (e == hipSuccess) e = ric_dispatch<false, 2>(T, W, total, x0, xref, u_out, ld_u, status, iters, s, stream, unsupported);
    }
    if (e == hipSuccess) e = ric_dispatch<false, 0>(T, W, total, x0, xref, u_out, ld_u, status, iters, s, stream, unsupported);
    hipError_t ef = hipFreeAsync(base, stream);
    if (state) {
        const hipError_t es = hipFreeAsync(state, stream);
        if (ef == hipSuccess) ef = es;
    }
    return e != hipSuccess ? e : ef;
}
// Callers with their own instance list (closed loops: live slots, few per step) or claim counter (the
// no-allocation entry) get the single kernel, and so do small batches: the pipeline's last launch has
// the latency of one complete solve however few instances it holds.
bool ric_wants_pipeline(const Settings& s, int64_t total) {
#ifdef CARMPC_RIC_PIPELINE_MIN_ENV   // experiment builds only (tools/gpu/pipe_threshold.sh): threshold from the environment
    static const long long min_total = [] {
        const char* v = getenv("CARMPC_RIC_PIPELINE_MIN");
        return v ? atoll(v) : (long long)kRicPipelineMin;
    }();
#else
    constexpr long long min_total = kRicPipelineMin;
#endif
    return !s.index && !s.count && !s.claim && total >= min_total;
}
}  // namespace

hipError_t launch_riccati(const DevProblem& P, int64_t batch, const double* x0, const double* xref, double* u_out,
                          int64_t ld_u, int32_t* status, int32_t* iters, const Settings& s, hipStream_t stream,
                          int* unsupported, bool het) {
    *unsupported = 0;
    if (batch <= 0) return hipSuccess;
    if (!P.ric) {
        *unsupported = 1;
        return hipErrorInvalidValue;
    }
    RicSegs T{};
    T.nseg = 1;
    T.off[0] = 0;
    T.off[1] = batch;
    T.P[0] = P;
    if (!het && ric_wants_pipeline(s, batch) && riccati_supported_N(P.N))
        return ric_pipeline(T, batch, x0, xref, u_out, ld_u, status, iters, s, stream, unsupported);
    // per-launch claim counter, stream-ordered (allocated, zeroed, freed on `stream`)
    const RicWork none{};
    return launch_with_claim(s, batch, stream, [&](const Settings& sc) {
        return het ? ric_dispatch<true, 0>(T, none, batch, x0, xref, u_out, ld_u, status, iters, sc, stream, unsupported)
                   : ric_dispatch<false, 0>(T, none, batch, x0, xref, u_out, ld_u, status, iters, sc, stream, unsupported);
    });
}

hipError_t launch_riccati_segs(const RicSegs& T, const double* x0, const double* xref, double* u_out, int64_t ld_u,
                               int32_t* status, int32_t* iters, const Settings& s, hipStream_t stream, int* unsupported) {
    *unsupported = 0;
    static_assert(sizeof(RicSegs) + sizeof(RicWork) + 6 * sizeof(void*) + sizeof(Settings) + 64 <= 4096,
                  "kernel arguments exceed 4 KB");
    const int nseg = T.nseg;
    if (nseg < 1 || nseg > kRicMaxSeg) {
        *unsupported = 1;
        return hipErrorInvalidValue;
    }
    for (int j = 0; j < nseg; ++j)
        if (!T.P[j].ric || T.P[j].N != T.P[0].N || T.P[j].ric != T.P[0].ric || T.P[j].rone != T.P[0].rone) {
            *unsupported = 1;
            return hipErrorInvalidValue;
        }
    const int64_t total = T.off[nseg] - T.off[0];
    if (total <= 0) return hipSuccess;
    if (ric_wants_pipeline(s, total))
        return ric_pipeline(T, total, x0, xref, u_out, ld_u, status, iters, s, stream, unsupported);
    // a single kernel over several segments claims from one counter per segment (kRicClaimStride words apart)
    const RicWork none{};
    if (s.claim) return ric_dispatch<false, 0>(T, none, total, x0, xref, u_out, ld_u, status, iters, s, stream, unsupported);
    unsigned* counters = nullptr;
    const int ncnt = kRicClaimStride * nseg;
    hipError_t e = hipMallocAsync(reinterpret_cast<void**>(&counters), sizeof(unsigned) * ncnt, stream);
    if (e != hipSuccess) return e;
    Settings sc = s;
    sc.claim = counters;
    e = launch_zero_u32(counters, ncnt, stream);
    if (e == hipSuccess) e = ric_dispatch<false, 0>(T, none, total, x0, xref, u_out, ld_u, status, iters, sc, stream, unsupported);
    const hipError_t ef = hipFreeAsync(counters, stream);
    return e != hipSuccess ? e : ef;
}

}  // namespace carmpc

#ifdef CARMPC_PHASE_TIMING
// Profiling build only: read (and optionally reset) the Riccati kernels' phase cycles, summed over the
// translation units that instantiate the kernel.
extern "C" int carmpc_debug_ric_cycles_m0(unsigned long long*, int);
extern "C" int carmpc_debug_ric_cycles_m1(unsigned long long*, int);
extern "C" int carmpc_debug_ric_cycles_m2(unsigned long long*, int);
extern "C" int carmpc_debug_ric_cycles_het(unsigned long long*, int);
extern "C" int carmpc_debug_ric_cycles(unsigned long long* out12, int reset) {
    for (int i = 0; i < 12; ++i) out12[i] = 0;
    for (auto fn : {carmpc_debug_ric_cycles_m0, carmpc_debug_ric_cycles_m1, carmpc_debug_ric_cycles_m2, carmpc_debug_ric_cycles_het}) {
        unsigned long long part[12];
        if (fn(part, reset) != 0) return -1;
        for (int i = 0; i < 12; ++i) out12[i] += part[i];
    }
    return 0;
}
#endif
