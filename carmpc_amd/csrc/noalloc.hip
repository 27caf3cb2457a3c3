// noalloc.hip -- carmpc_solve_batch_noalloc: the batched solve for callers that cannot allocate
// (code under HIP graph capture, tight serving loops, harnesses that forbid hipMalloc).
//
// carmpc_solve_batch takes the solve kernels' claim counter -- the only device memory the solve
// uses beyond its inputs and outputs -- from a stream-ordered allocation per launch.  Here the
// counter lives in a static device array, so the call makes no hipMalloc / hipFree / allocating
// library call at all.  Every GPU the library runs on holds its own 256-byte copy of the array
// until the process ends.
#include <hip/hip_runtime.h>

#include <mutex>
#include <string>

#include "carmpc_internal.h"

using namespace carmpc;

// Word 0 is the claim counter; the rest pads the array to its alignment unit.  In host code
// this name is only a handle for hipGetSymbolAddress, never an address to hand to a kernel.
static __device__ __align__(256) unsigned scratch[64];

namespace {
// Device address of `scratch` on each GPU (every GPU has its own copy at its own address),
// resolved once per device with that device current: when a problem is created on it
// (noalloc_prepare_device), else on the first call of the entry point.
int scratch_address(int dev, unsigned** out) {
    static std::mutex mu;
    static unsigned* ptr[64] = {};
    if (dev < 0 || dev >= 64) return set_error(CARMPC_EUNSUPPORTED, "carmpc_solve_batch_noalloc: device index above 63");
    std::lock_guard<std::mutex> lock(mu);
    if (!ptr[dev]) {
        unsigned* p = nullptr;
        const hipError_t e = hipGetSymbolAddress(reinterpret_cast<void**>(&p), HIP_SYMBOL(scratch));
        if (e != hipSuccess || !p)
            return set_error(CARMPC_EHIP, (std::string("hipGetSymbolAddress(scratch): ") + hipGetErrorName(e)).c_str());
        ptr[dev] = p;
    }
    *out = ptr[dev];
    return CARMPC_OK;
}
}  // namespace

int carmpc::noalloc_prepare_device(int dev) {
    unsigned* p = nullptr;
    return scratch_address(dev, &p);
}

extern "C" int carmpc_solve_batch_noalloc(const carmpc_problem* P, int64_t batch, const double* x0, const double* xref,
                                          double* u_out, int32_t* status, int32_t* iters,
                                          const carmpc_settings* settings, hipStream_t stream) {
    if (!P) return set_error(CARMPC_EINVAL, "null problem");
    if (batch < 0) return set_error(CARMPC_EINVAL, "negative batch");
    if (batch > CARMPC_NOALLOC_MAX_BATCH)
        return set_error(CARMPC_EUNSUPPORTED,
                         ("carmpc_solve_batch_noalloc: batch " + std::to_string(batch) + " exceeds CARMPC_NOALLOC_MAX_BATCH (" +
                          std::to_string((long long)CARMPC_NOALLOC_MAX_BATCH) +
                          "): the 32-bit claim counter in the static scratch cannot index it").c_str());
    if (batch == 0) return CARMPC_OK;
    if (!x0 || !u_out || !status) return set_error(CARMPC_EINVAL, "null batch pointer");
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return set_error(CARMPC_EHIP, "hipGetDevice failed");
    if (dev != problem_device(P))
        return set_error(CARMPC_EINVAL, "carmpc_solve_batch_noalloc: the problem belongs to another device than the current one");
    unsigned* counter = nullptr;
    const int rc = scratch_address(dev, &counter);
    if (rc != CARMPC_OK) return rc;
    // the array keeps the last call's count: clear it with a fill kernel on the caller's stream
    const hipError_t e = launch_zero_u32(counter, 1, stream);
    if (e != hipSuccess) return set_error(CARMPC_EHIP, (std::string("clear claim counter: ") + hipGetErrorName(e)).c_str());
    // the kernels take the counter's device address as an argument, as in carmpc_solve_batch
    return solve_batch_with_claim(P, batch, x0, xref, u_out, status, iters, settings, counter, stream);
}
