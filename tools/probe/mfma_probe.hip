// mfma_probe.hip -- operand layout of v_mfma_f64_4x4x4f64 on gfx950 (4 blocks of 4x4x4 per wave).
// Every lane holds one element of A, B and C/D.  The probe feeds distinct values, reads D back
// and searches, per operand, the lane -> (block, row, col) map among the candidate maps
//   lane = 16*blk + 4*r + c   ("rowmajor")  or  lane = 16*blk + r + 4*c ("colmajor")
// that reproduces D = A*B + C computed on the host.  It also reports whether lanes masked out of
// EXEC still take part (MFMA under a divergent branch).
// Build: hipcc -O2 --offload-arch=gfx950 tools/probe/mfma_probe.hip -o build/mfma_probe
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <cstdlib>

__global__ void probe(const double* a, const double* b, const double* c, double* d, double* d_masked,
                      double* bc) {
    const int l = threadIdx.x;
    double acc = __builtin_amdgcn_mfma_f64_4x4x4f64(a[l], b[l], c[l], 0, 0, 0);
    d[l] = acc;
    double m = -7.0;
    if ((l >> 4) != 2) m = __builtin_amdgcn_mfma_f64_4x4x4f64(a[l], b[l], c[l], 0, 0, 0);   // block 2 masked off
    d_masked[l] = m;
    // DPP row_newbcast: lane 5 of each 16-lane row to the whole row (ctrl 0x150 + n)
    const unsigned long long bits = __builtin_bit_cast(unsigned long long, a[l]);
    const int lo = __builtin_amdgcn_update_dpp(0, (int)(unsigned)bits, 0x155, 0xf, 0xf, false);
    const int hi = __builtin_amdgcn_update_dpp(0, (int)(unsigned)(bits >> 32), 0x155, 0xf, 0xf, false);
    bc[l] = __builtin_bit_cast(double, ((unsigned long long)(unsigned)hi << 32) | (unsigned)lo);
}

static int lane_of(int layout, int blk, int r, int c) { return 16 * blk + (layout ? r + 4 * c : 4 * r + c); }

int main() {
    double ha[64], hb[64], hc[64], hd[64], hm[64], hbc[64];
    srand(3);
    for (int i = 0; i < 64; ++i) {
        ha[i] = 1.0 + (rand() % 97) / 7.0;
        hb[i] = -2.0 + (rand() % 89) / 5.0;
        hc[i] = (rand() % 13) / 3.0;
    }
    double *da, *db, *dc, *dd, *dm, *dbc;
    hipMalloc(&da, 512); hipMalloc(&db, 512); hipMalloc(&dc, 512); hipMalloc(&dd, 512); hipMalloc(&dm, 512);
    hipMalloc(&dbc, 512);
    hipMemcpy(da, ha, 512, hipMemcpyHostToDevice);
    hipMemcpy(db, hb, 512, hipMemcpyHostToDevice);
    hipMemcpy(dc, hc, 512, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, da, db, dc, dd, dm, dbc);
    if (hipDeviceSynchronize() != hipSuccess) { printf("kernel failed\n"); return 1; }
    hipMemcpy(hd, dd, 512, hipMemcpyDeviceToHost);
    hipMemcpy(hm, dm, 512, hipMemcpyDeviceToHost);
    hipMemcpy(hbc, dbc, 512, hipMemcpyDeviceToHost);
    const char* nm[2] = {"rowmajor(4r+c)", "colmajor(r+4c)"};
    int found = 0;
    for (int la = 0; la < 2; ++la)
        for (int lb = 0; lb < 2; ++lb)
            for (int lc = 0; lc < 2; ++lc) {
                double err = 0.0;
                for (int blk = 0; blk < 4; ++blk)
                    for (int i = 0; i < 4; ++i)
                        for (int j = 0; j < 4; ++j) {
                            double s = hc[lane_of(lc, blk, i, j)];
                            for (int k = 0; k < 4; ++k) s += ha[lane_of(la, blk, i, k)] * hb[lane_of(lb, blk, k, j)];
                            err = fmax(err, fabs(s - hd[lane_of(lc, blk, i, j)]));
                        }
                if (err < 1e-9) {
                    printf("LAYOUT A=%s B=%s C/D=%s  (max err %.2e)\n", nm[la], nm[lb], nm[lc], err);
                    ++found;
                }
            }
    if (!found) {
        printf("no candidate layout matches; D by lane:\n");
        for (int i = 0; i < 64; ++i) printf("%d %.6f\n", i, hd[i]);
    }
    int same = 1, sentinel = 1;
    for (int l = 0; l < 64; ++l) {
        if ((l >> 4) == 2) sentinel &= hm[l] == -7.0;
        else same &= hm[l] == hd[l];
    }
    printf("MASKED: active blocks %s, masked block keeps its old value: %s\n", same ? "correct" : "WRONG",
           sentinel ? "yes" : "no");
    int bc_ok = 1;
    for (int l = 0; l < 64; ++l) bc_ok &= hbc[l] == ha[(l & ~15) + 5];
    printf("ROW_NEWBCAST lane 5: %s\n", bc_ok ? "ok" : "WRONG");
    return 0;
}
