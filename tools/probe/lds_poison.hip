// Test tool: fills the LDS of every CU (and a block of stream-ordered pool memory) with a chosen bit pattern, so that a
// kernel which reads LDS or work-list memory before writing it meets that pattern instead of the leftovers of the
// previous launch.  Build: hipcc --offload-arch=gfx950 -O2 -shared -fPIC tools/probe/lds_poison.hip -o build/probe/libpoison.so
#include <hip/hip_runtime.h>
#include <cstdint>

namespace {
constexpr int kWords = 160 * 1024 / 8;
__global__ void __launch_bounds__(512) fill_lds(uint64_t pattern, uint64_t* sink) {
    __shared__ uint64_t buf[kWords];
    for (int i = threadIdx.x; i < kWords; i += blockDim.x) buf[i] = pattern;
    __syncthreads();
    // keep the workgroup resident for a moment so that the grid spreads over every CU
    uint64_t acc = 0;
    for (int r = 0; r < 64; ++r)
        for (int i = threadIdx.x; i < kWords; i += blockDim.x) acc += buf[i] ^ (uint64_t)r;
    if (acc == 0x1234567u) sink[0] = acc;
}
__global__ void fill_mem(uint64_t* p, size_t n, uint64_t pattern) {
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) p[i] = pattern;
}
// occupies CU slots for a while: `spin` rounds over `lds_bytes` of dynamic LDS per workgroup
__global__ void __launch_bounds__(256) hog_kernel(int lds_words, int spin, uint64_t* sink) {
    extern __shared__ uint64_t dyn[];
    for (int i = threadIdx.x; i < lds_words; i += blockDim.x) dyn[i] = (uint64_t)i;
    __syncthreads();
    uint64_t acc = threadIdx.x;
    for (int r = 0; r < spin; ++r) {
        for (int i = threadIdx.x; i < lds_words; i += blockDim.x) acc += dyn[i] ^ (uint64_t)r;
        acc = acc * 6364136223846793005ull + 1442695040888963407ull;
    }
    if (acc == 0x1234567u) sink[0] = acc;
}
}  // namespace
extern "C" int hog(int workgroups, int lds_bytes, int spin, void* stream) {
    static uint64_t* sink = nullptr;
    if (!sink && hipMalloc(reinterpret_cast<void**>(&sink), 8) != hipSuccess) return -1;
    hipLaunchKernelGGL(hog_kernel, dim3(workgroups), dim3(256), (size_t)lds_bytes, static_cast<hipStream_t>(stream), lds_bytes / 8, spin, sink);
    return (int)hipGetLastError();
}

extern "C" int poison_lds(uint64_t pattern, int workgroups, void* stream) {
    static uint64_t* sink = nullptr;
    if (!sink && hipMalloc(reinterpret_cast<void**>(&sink), 8) != hipSuccess) return -1;
    hipLaunchKernelGGL(fill_lds, dim3(workgroups), dim3(512), 0, static_cast<hipStream_t>(stream), pattern, sink);
    return (int)hipGetLastError();
}
// allocate `bytes` from the stream-ordered pool, fill, free: the next hipMallocAsync on the stream reuses it
extern "C" int poison_pool(uint64_t pattern, size_t bytes, void* stream) {
    uint64_t* p = nullptr;
    hipStream_t s = static_cast<hipStream_t>(stream);
    if (hipMallocAsync(reinterpret_cast<void**>(&p), bytes, s) != hipSuccess) return -1;
    hipLaunchKernelGGL(fill_mem, dim3(1024), dim3(256), 0, s, p, bytes / 8, pattern);
    if (hipGetLastError() != hipSuccess) return -2;
    return (int)hipFreeAsync(p, s);
}
