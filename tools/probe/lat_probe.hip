// lat_probe.hip -- latencies that bound the stage passes of the Riccati kernel at one wave per SIMD
// (gfx950): dependent v_mfma_f64_4x4x4 chain, independent MFMA issue rate, LDS read round trip,
// dependent FP64 FMA chain, v_rcp_f64 chain, ds_bpermute round trip.  One wave, cycles by clock64.
// Build: hipcc -O2 --offload-arch=gfx950 tools/probe/lat_probe.hip -o build/lat_probe
#include <hip/hip_runtime.h>
#include <cstdio>

#define REP 256
// keep a value (and the clock reads around its chain) where the source puts them
#define PIN(v) asm volatile("" : "+v"(v) : : "memory")
__device__ __forceinline__ long long now() {
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n s_nop 0" ::: "memory");
    const long long t = __builtin_readcyclecounter();
    asm volatile("" ::: "memory");
    return t;
}

__global__ void probe(double* out, long long* cyc, const double* in) {
    __shared__ double lds[4096];
    const int l = threadIdx.x;
    for (int i = l; i < 4096; i += 64) lds[i] = in[i & 63] * 1e-3 + (i & 1023);
    __syncthreads();
    double a = in[l], b = in[64 + l] * 1e-3, c = in[128 + l];
    long long t0, t1;
    // 1. dependent MFMA chain (result feeds operand B of the next)
    double x = c;
    t0 = now();
#pragma unroll
    for (int i = 0; i < REP; ++i) { x = __builtin_amdgcn_mfma_f64_4x4x4f64(b, x, c, 0, 0, 0); PIN(x); }
    t1 = now();
    if (l == 0) cyc[0] = t1 - t0;
    out[l] = x;
    // 2. independent MFMAs (8 accumulators)
    double y[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) y[j] = c + j;
    t0 = now();
#pragma unroll
    for (int i = 0; i < REP / 8; ++i)
#pragma unroll
        for (int j = 0; j < 8; ++j) { y[j] = __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, y[j], 0, 0, 0); PIN(y[j]); }
    t1 = now();
    if (l == 0) cyc[1] = t1 - t0;
    for (int j = 0; j < 8; ++j) out[64 + l] += y[j];
    // 3. dependent LDS reads (pointer chase through an index kept in the loaded double)
    int idx = l;
    double acc = 0.0;
    t0 = now();
#pragma unroll
    for (int i = 0; i < REP; ++i) {
        const double v = lds[idx];
        acc += v;
        idx = ((int)v + l) & 1023;
    }
    t1 = now();
    if (l == 0) cyc[2] = t1 - t0;
    out[128 + l] = acc;
    // 4. dependent FP64 FMA chain
    double f = a;
    t0 = now();
#pragma unroll
    for (int i = 0; i < REP; ++i) { f = fma(f, b, c); PIN(f); }
    t1 = now();
    if (l == 0) cyc[3] = t1 - t0;
    out[192 + l] = f;
    // 5. dependent v_rcp_f64 chain
    double r = a + 2.0;
    t0 = now();
#pragma unroll
    for (int i = 0; i < REP; ++i) { r = __builtin_amdgcn_rcp(r); PIN(r); }
    t1 = now();
    if (l == 0) cyc[4] = t1 - t0;
    out[256 + l] = r;
    // 6. dependent ds_bpermute round trips (32-bit)
    int p = l;
    t0 = now();
#pragma unroll
    for (int i = 0; i < REP; ++i) { p = __builtin_amdgcn_ds_bpermute(((p + 1) & 63) << 2, p); PIN(p); }
    t1 = now();
    if (l == 0) cyc[5] = t1 - t0;
    out[320 + l] = p;
    // 7. LDS store then load of another lane's value (write -> read round trip)
    double w = a;
    t0 = now();
#pragma unroll
    for (int i = 0; i < REP; ++i) {
        lds[2048 + l] = w;
        __builtin_amdgcn_wave_barrier();
        w = lds[2048 + ((l + 1) & 63)] + 1.0;
        __builtin_amdgcn_wave_barrier();
    }
    t1 = now();
    if (l == 0) cyc[6] = t1 - t0;
    out[384 + l] = w;
    // 8. MFMA -> LDS store -> LDS load -> MFMA (the per-stage loop of the vector passes)
    double z = c;
    t0 = now();
#pragma unroll
    for (int i = 0; i < REP; ++i) {
        z = __builtin_amdgcn_mfma_f64_4x4x4f64(b, z, lds[(i * 64 + l) & 2047], 0, 0, 0);
        lds[2048 + ((i * 64 + l) & 2047)] = z;
    }
    t1 = now();
    if (l == 0) cyc[7] = t1 - t0;
    out[448 + l] = z;
}

int main() {
    double hin[192];
    for (int i = 0; i < 192; ++i) hin[i] = 1.0 + 0.01 * i;
    double *din, *dout;
    long long* dc;
    if (hipMalloc(&din, sizeof(hin)) != hipSuccess || hipMalloc(&dout, 512 * 8) != hipSuccess ||
        hipMalloc(&dc, 8 * 8) != hipSuccess)
        return 1;
    (void)hipMemcpy(din, hin, sizeof(hin), hipMemcpyHostToDevice);
    (void)hipMemset(dout, 0, 512 * 8);
    for (int rep = 0; rep < 2; ++rep) {
        hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, dout, dc, din);
        if (hipDeviceSynchronize() != hipSuccess) { printf("kernel failed\n"); return 1; }
    }
    long long c[8];
    (void)hipMemcpy(c, dc, sizeof(c), hipMemcpyDeviceToHost);
    const char* nm[8] = {"dependent MFMA f64 4x4x4 chain", "independent MFMA f64 4x4x4 (8 accumulators)",
                         "dependent LDS read (ds_read_b64)", "dependent FP64 FMA chain", "dependent v_rcp_f64 chain",
                         "dependent ds_bpermute_b32", "LDS store -> wave barrier -> load (other lane)",
                         "MFMA <- LDS load, MFMA -> LDS store per step"};
    for (int i = 0; i < 8; ++i) printf("%-50s %7.1f clock64 ticks per step\n", nm[i], (double)c[i] / REP);
    return 0;
}
