// Probe of the cross-lane primitives used by the reductions in ipm_staged.hip:
// prints, for lane values v = lane, what each primitive returns in every lane.
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ void probe(int* out) {
    const int l = threadIdx.x;
    const unsigned v = (unsigned)l;
    auto p32 = __builtin_amdgcn_permlane32_swap(v, v, false, false);
    auto p16 = __builtin_amdgcn_permlane16_swap(v, v, false, false);
    out[0 * 64 + l] = (int)p32[0];
    out[1 * 64 + l] = (int)p32[1];
    out[2 * 64 + l] = (int)p16[0];
    out[3 * 64 + l] = (int)p16[1];
    out[4 * 64 + l] = __builtin_amdgcn_update_dpp(-1, (int)v, 0xB1, 0xf, 0xf, false);   // quad_perm [1,0,3,2]
    out[5 * 64 + l] = __builtin_amdgcn_update_dpp(-1, (int)v, 0x4E, 0xf, 0xf, false);   // quad_perm [2,3,0,1]
    out[6 * 64 + l] = __builtin_amdgcn_update_dpp(-1, (int)v, 0x124, 0xf, 0xf, false);  // row_ror:4
    out[7 * 64 + l] = __builtin_amdgcn_update_dpp(-1, (int)v, 0x128, 0xf, 0xf, false);  // row_ror:8
}

int main() {
    int* d;
    int h[8 * 64];
    if (hipMalloc(&d, sizeof(h)) != hipSuccess) return 1;
    hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, d);
    if (hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost) != hipSuccess) return 2;
    const char* names[8] = {"p32[0]", "p32[1]", "p16[0]", "p16[1]", "qp1032", "qp2301", "ror4", "ror8"};
    for (int r = 0; r < 8; ++r) {
        printf("%-7s", names[r]);
        for (int l = 0; l < 64; ++l) printf(" %d", h[r * 64 + l]);
        printf("\n");
    }
    return 0;
}
