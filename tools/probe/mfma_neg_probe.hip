// mfma_neg_probe.hip -- does the BLGP field of v_mfma_f64_4x4x4f64 act as per-operand negation
// on gfx950 (bit 0: A, bit 1: B, bit 2: C), as documented for the FP64 MFMAs of gfx940+?
// Build: hipcc -O2 --offload-arch=gfx950 tools/probe/mfma_neg_probe.hip -o build/mfma_neg_probe
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <cstdlib>

__global__ void probe(const double* a, const double* b, const double* c, double* d) {
    const int l = threadIdx.x;
    d[l] = __builtin_amdgcn_mfma_f64_4x4x4f64(a[l], b[l], c[l], 0, 0, 0);
    d[64 + l] = __builtin_amdgcn_mfma_f64_4x4x4f64(a[l], b[l], c[l], 0, 0, 1);
    d[128 + l] = __builtin_amdgcn_mfma_f64_4x4x4f64(a[l], b[l], c[l], 0, 0, 2);
    d[192 + l] = __builtin_amdgcn_mfma_f64_4x4x4f64(a[l], b[l], c[l], 0, 0, 4);
}

int main() {
    double ha[64], hb[64], hc[64], hd[256];
    srand(5);
    for (int i = 0; i < 64; ++i) {
        ha[i] = 1.0 + (rand() % 97) / 7.0;
        hb[i] = -2.0 + (rand() % 89) / 5.0;
        hc[i] = (rand() % 13) / 3.0;
    }
    double *da, *db, *dc, *dd;
    if (hipMalloc(&da, 512) != hipSuccess || hipMalloc(&db, 512) != hipSuccess || hipMalloc(&dc, 512) != hipSuccess ||
        hipMalloc(&dd, 2048) != hipSuccess)
        return 1;
    (void)hipMemcpy(da, ha, 512, hipMemcpyHostToDevice);
    (void)hipMemcpy(db, hb, 512, hipMemcpyHostToDevice);
    (void)hipMemcpy(dc, hc, 512, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, da, db, dc, dd);
    if (hipDeviceSynchronize() != hipSuccess) { printf("kernel failed\n"); return 1; }
    (void)hipMemcpy(hd, dd, 2048, hipMemcpyDeviceToHost);
    // with D = A B + C: neg A or neg B -> D' = 2 C - D ; neg C -> D' = D - 2 C
    const char* what[3] = {"blgp=1", "blgp=2", "blgp=4"};
    for (int v = 0; v < 3; ++v) {
        double e_ab = 0, e_c = 0, e_same = 0;
        for (int l = 0; l < 64; ++l) {
            const double d0 = hd[l], dv = hd[64 * (v + 1) + l];
            e_ab = fmax(e_ab, fabs(dv - (2 * hc[l] - d0)));
            e_c = fmax(e_c, fabs(dv - (d0 - 2 * hc[l])));
            e_same = fmax(e_same, fabs(dv - d0));
        }
        printf("%s: %s\n", what[v], e_ab < 1e-9 ? "negates the product (A or B)" : e_c < 1e-9 ? "negates C" :
                                    e_same < 1e-9 ? "no effect" : "something else");
    }
    return 0;
}
