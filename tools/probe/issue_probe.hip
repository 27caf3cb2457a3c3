// issue_probe.hip -- instruction issue cost of one wavefront per SIMD on gfx950: how many cycles
// independent instructions of each class take back to back, and whether scalar, LDS and
// register-move instructions placed between vector FP64 instructions are hidden or add to them.
// One workgroup of 4 waves (one per SIMD), then 8 waves (two per SIMD) for the same per-wave work.
// Build: hipcc -O2 --offload-arch=gfx950 tools/probe/issue_probe.hip -o build/issue_probe
#include <hip/hip_runtime.h>
#include <cstdio>

#define REP 64   // repetitions of an 8-instruction group
__device__ __forceinline__ long long now() {
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n s_nop 0" ::: "memory");
    const long long t = __builtin_readcyclecounter();
    asm volatile("" ::: "memory");
    return t;
}

#define FMA8                                                                                          \
    "v_fma_f64 %0, %0, %8, %9\n v_fma_f64 %1, %1, %8, %9\n v_fma_f64 %2, %2, %8, %9\n v_fma_f64 %3, %3, %8, %9\n" \
    "v_fma_f64 %4, %4, %8, %9\n v_fma_f64 %5, %5, %8, %9\n v_fma_f64 %6, %6, %8, %9\n v_fma_f64 %7, %7, %8, %9\n"
#define ACC8 "+v"(y[0]), "+v"(y[1]), "+v"(y[2]), "+v"(y[3]), "+v"(y[4]), "+v"(y[5]), "+v"(y[6]), "+v"(y[7])

__global__ void probe(double* out, long long* cyc, const double* in) {
    __shared__ double lds[8 * 1024];
    const int l = threadIdx.x & 63, w = threadIdx.x >> 6;
    for (int i = threadIdx.x; i < 8 * 1024; i += blockDim.x) lds[i] = in[i & 63];
    __syncthreads();
    double y[8];
    for (int j = 0; j < 8; ++j) y[j] = in[l] + j;
    const double b = in[64 + l] * 1e-3, c = in[128 + l];
    long long t0, t1;
    int sk = 0;
    int vi = l, vj = l + 1;
    const unsigned la = (unsigned)(((w & 3) * 1024 + l) * 8);   // stays inside the 64 KB array with the offsets
    double ld0 = 0, ld1 = 0, ld2 = 0, ld3 = 0;
    auto rec = [&](int i) {
        if (l == 0) cyc[w * 16 + i] = t1 - t0;
    };
    // 0. independent FP64 FMAs
    t0 = now();
    for (int i = 0; i < REP; ++i) asm volatile(FMA8 : ACC8 : "v"(b), "v"(c));
    t1 = now();
    rec(0);
    // 1. FMA + scalar add, 1:1
    t0 = now();
    for (int i = 0; i < REP; ++i)
        asm volatile("v_fma_f64 %0, %0, %8, %9\n s_mov_b32 s40, 1\n v_fma_f64 %1, %1, %8, %9\n s_mov_b32 s40, 1\n"
                     "v_fma_f64 %2, %2, %8, %9\n s_mov_b32 s40, 1\n v_fma_f64 %3, %3, %8, %9\n s_mov_b32 s40, 1\n"
                     "v_fma_f64 %4, %4, %8, %9\n s_mov_b32 s40, 1\n v_fma_f64 %5, %5, %8, %9\n s_mov_b32 s40, 1\n"
                     "v_fma_f64 %6, %6, %8, %9\n s_mov_b32 s40, 1\n v_fma_f64 %7, %7, %8, %9\n s_mov_b32 s40, 1\n"
                     : ACC8 : "v"(b), "v"(c) : "s40", "scc");
    t1 = now();
    rec(1);
    // 2. FMA + 32-bit vector move, 1:1
    t0 = now();
    for (int i = 0; i < REP; ++i)
        asm volatile("v_fma_f64 %0, %0, %8, %9\n v_mov_b32 %10, %11\n v_fma_f64 %1, %1, %8, %9\n v_mov_b32 %11, %10\n"
                     "v_fma_f64 %2, %2, %8, %9\n v_mov_b32 %10, %11\n v_fma_f64 %3, %3, %8, %9\n v_mov_b32 %11, %10\n"
                     "v_fma_f64 %4, %4, %8, %9\n v_mov_b32 %10, %11\n v_fma_f64 %5, %5, %8, %9\n v_mov_b32 %11, %10\n"
                     "v_fma_f64 %6, %6, %8, %9\n v_mov_b32 %10, %11\n v_fma_f64 %7, %7, %8, %9\n v_mov_b32 %11, %10\n"
                     : ACC8 : "v"(b), "v"(c), "v"(vi), "v"(vj));
    t1 = now();
    rec(2);
    // 3. FMA + LDS read (b64, independent destinations), 1:1 pairs of four
    t0 = now();
    for (int i = 0; i < REP; ++i)
        asm volatile("v_fma_f64 %0, %0, %12, %13\n ds_read_b64 %8, %14\n v_fma_f64 %1, %1, %12, %13\n ds_read_b64 %9, %14 offset:512\n"
                     "v_fma_f64 %2, %2, %12, %13\n ds_read_b64 %10, %14 offset:1024\n v_fma_f64 %3, %3, %12, %13\n ds_read_b64 %11, %14 offset:1536\n"
                     "v_fma_f64 %4, %4, %12, %13\n v_fma_f64 %5, %5, %12, %13\n v_fma_f64 %6, %6, %12, %13\n v_fma_f64 %7, %7, %12, %13\n"
                     "s_waitcnt lgkmcnt(0)\n"
                     : ACC8, "=&v"(ld0), "=&v"(ld1), "=&v"(ld2), "=&v"(ld3) : "v"(b), "v"(c), "v"(la));
    t1 = now();
    rec(3);
    // 4. 32-bit vector moves only (16 per group)
    t0 = now();
    for (int i = 0; i < REP; ++i)
        asm volatile("v_mov_b32 %0, %1\n v_mov_b32 %1, %0\n v_mov_b32 %0, %1\n v_mov_b32 %1, %0\n v_mov_b32 %0, %1\n v_mov_b32 %1, %0\n"
                     "v_mov_b32 %0, %1\n v_mov_b32 %1, %0\n"
                     : "+v"(vi), "+v"(vj));
    t1 = now();
    rec(4);
    // 5. scalar adds only (8 per group, dependent)
    t0 = now();
    for (int i = 0; i < REP; ++i)
        asm volatile("s_mov_b32 s40, 1\n s_mov_b32 s40, 1\n s_mov_b32 s40, 1\n s_mov_b32 s40, 1\n"
                     "s_mov_b32 s40, 1\n s_mov_b32 s40, 1\n s_mov_b32 s40, 1\n s_mov_b32 s40, 1\n"
                     ::: "s40", "scc");
    t1 = now();
    rec(5);
    // 6. FMA + s_nop 0, 1:1
    t0 = now();
    for (int i = 0; i < REP; ++i)
        asm volatile("v_fma_f64 %0, %0, %8, %9\n s_nop 0\n v_fma_f64 %1, %1, %8, %9\n s_nop 0\n v_fma_f64 %2, %2, %8, %9\n s_nop 0\n"
                     "v_fma_f64 %3, %3, %8, %9\n s_nop 0\n v_fma_f64 %4, %4, %8, %9\n s_nop 0\n v_fma_f64 %5, %5, %8, %9\n s_nop 0\n"
                     "v_fma_f64 %6, %6, %8, %9\n s_nop 0\n v_fma_f64 %7, %7, %8, %9\n s_nop 0\n"
                     : ACC8 : "v"(b), "v"(c));
    t1 = now();
    rec(6);
    // 7. two dependent chains of FMAs (distance 2)
    t0 = now();
    for (int i = 0; i < REP; ++i)
        asm volatile("v_fma_f64 %0, %0, %2, %3\n v_fma_f64 %1, %1, %2, %3\n v_fma_f64 %0, %0, %2, %3\n v_fma_f64 %1, %1, %2, %3\n"
                     "v_fma_f64 %0, %0, %2, %3\n v_fma_f64 %1, %1, %2, %3\n v_fma_f64 %0, %0, %2, %3\n v_fma_f64 %1, %1, %2, %3\n"
                     : "+v"(y[0]), "+v"(y[1]) : "v"(b), "v"(c));
    t1 = now();
    rec(7);
    // 8. FMA + accumulation-register read, 1:1
    t0 = now();
    for (int i = 0; i < REP; ++i)
        asm volatile("v_fma_f64 %0, %0, %8, %9\n v_accvgpr_read_b32 %10, a0\n v_fma_f64 %1, %1, %8, %9\n v_accvgpr_read_b32 %11, a1\n"
                     "v_fma_f64 %2, %2, %8, %9\n v_accvgpr_read_b32 %10, a2\n v_fma_f64 %3, %3, %8, %9\n v_accvgpr_read_b32 %11, a3\n"
                     "v_fma_f64 %4, %4, %8, %9\n v_accvgpr_read_b32 %10, a0\n v_fma_f64 %5, %5, %8, %9\n v_accvgpr_read_b32 %11, a1\n"
                     "v_fma_f64 %6, %6, %8, %9\n v_accvgpr_read_b32 %10, a2\n v_fma_f64 %7, %7, %8, %9\n v_accvgpr_read_b32 %11, a3\n"
                     : ACC8 : "v"(b), "v"(c), "v"(vi), "v"(vj) : "a0", "a1", "a2", "a3");
    t1 = now();
    rec(8);
    // 9. FMA + compare + 2 cndmask (a 64-bit select), per FMA
    t0 = now();
    for (int i = 0; i < REP; ++i)
        asm volatile("v_fma_f64 %0, %0, %8, %9\n v_cmp_lt_f64 vcc, %1, %8\n v_cndmask_b32 %10, %10, %11, vcc\n v_cndmask_b32 %11, %11, %10, vcc\n"
                     "v_fma_f64 %2, %2, %8, %9\n v_cmp_lt_f64 vcc, %3, %8\n v_cndmask_b32 %10, %10, %11, vcc\n v_cndmask_b32 %11, %11, %10, vcc\n"
                     "v_fma_f64 %4, %4, %8, %9\n v_cmp_lt_f64 vcc, %5, %8\n v_cndmask_b32 %10, %10, %11, vcc\n v_cndmask_b32 %11, %11, %10, vcc\n"
                     "v_fma_f64 %6, %6, %8, %9\n v_cmp_lt_f64 vcc, %7, %8\n v_cndmask_b32 %10, %10, %11, vcc\n v_cndmask_b32 %11, %11, %10, vcc\n"
                     : ACC8 : "v"(b), "v"(c), "v"(vi), "v"(vj) : "vcc");
    t1 = now();
    rec(9);
    // 10. LDS reads only: 8 x ds_read_b128 then wait
    t0 = now();
    for (int i = 0; i < REP; ++i) {
        double2 q0, q1, q2, q3;
        asm volatile("ds_read_b128 %0, %4\n ds_read_b128 %1, %4 offset:1024\n ds_read_b128 %2, %4 offset:2048\n ds_read_b128 %3, %4 offset:3072\n"
                     "ds_read_b128 %0, %4 offset:4096\n ds_read_b128 %1, %4 offset:5120\n ds_read_b128 %2, %4 offset:6144\n ds_read_b128 %3, %4 offset:7168\n"
                     "s_waitcnt lgkmcnt(0)\n"
                     : "=&v"(q0), "=&v"(q1), "=&v"(q2), "=&v"(q3) : "v"((unsigned)(l * 16)));
        ld0 += q0.x + q1.x + q2.x + q3.x;
    }
    t1 = now();
    rec(10);
    out[threadIdx.x] = y[0] + y[1] + y[2] + y[3] + y[4] + y[5] + y[6] + y[7] + sk + vi + vj + ld0 + ld1 + ld2 + ld3;
}

int main() {
    double hin[192];
    for (int i = 0; i < 192; ++i) hin[i] = 1.0 + 0.01 * i;
    double *din, *dout;
    long long* dc;
    if (hipMalloc(&din, sizeof(hin)) != hipSuccess || hipMalloc(&dout, 1024 * 8) != hipSuccess ||
        hipMalloc(&dc, 16 * 16 * 8) != hipSuccess)
        return 1;
    (void)hipMemcpy(din, hin, sizeof(hin), hipMemcpyHostToDevice);
    const char* nm[11] = {"8 independent v_fma_f64",
                          "8 x (v_fma_f64 + s_mov_b32)",
                          "8 x (v_fma_f64 + v_mov_b32)",
                          "8 v_fma_f64 + 4 ds_read_b64 + wait",
                          "8 v_mov_b32 (dependent pairs)",
                          "8 s_mov_b32",
                          "8 x (v_fma_f64 + s_nop 0)",
                          "8 v_fma_f64 in two dependent chains",
                          "8 x (v_fma_f64 + v_accvgpr_read_b32)",
                          "4 x (v_fma_f64 + v_cmp_f64 + 2 v_cndmask_b32)",
                          "8 ds_read_b128 + wait (ld0 sum outside)"};
    for (int waves : {4, 8, 16}) {
        (void)hipMemset(dc, 0, 16 * 16 * 8);
        for (int rep = 0; rep < 2; ++rep) {
            hipLaunchKernelGGL(probe, dim3(1), dim3(64 * waves), 0, 0, dout, dc, din);
            if (hipDeviceSynchronize() != hipSuccess) { printf("kernel failed\n"); return 1; }
        }
        long long c[16 * 16];
        (void)hipMemcpy(c, dc, sizeof(c), hipMemcpyDeviceToHost);
        printf("%d waves in the workgroup (%d per SIMD): cycles per group, wave 0 / last wave\n", waves, waves / 4);
        for (int i = 0; i < 11; ++i)
            printf("  %-48s %7.1f %7.1f\n", nm[i], (double)c[i] / REP, (double)c[(waves - 1) * 16 + i] / REP);
    }
    return 0;
}
