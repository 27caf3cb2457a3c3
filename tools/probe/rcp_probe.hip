// Accuracy of v_rcp_f64 / v_rsq_f64 (raw and with one Newton step) against the
// correctly rounded 1/x and 1/sqrt(x), in ulps, over log-uniform x in [1e-30, 1e30].
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <cstdint>

__device__ double ulps(double a, double b) {
    const long long ia = __builtin_bit_cast(long long, a), ib = __builtin_bit_cast(long long, b);
    return fabs((double)(ia - ib));
}
__global__ void probe(double* out, int n) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    unsigned long long s = 0x9E3779B97F4A7C15ull * (i + 1);
    s ^= s >> 29; s *= 0xBF58476D1CE4E5B9ull; s ^= s >> 32;
    const double u = (double)(s >> 11) * (1.0 / 9007199254740992.0);
    const double x = pow(10.0, -30.0 + 60.0 * u);
    const double rc = 1.0 / x, rs = 1.0 / sqrt(x);
    const double r0 = __builtin_amdgcn_rcp(x);
    const double r1 = fma(fma(-x, r0, 1.0), r0, r0);
    const double q0 = __builtin_amdgcn_rsq(x);
    const double q1 = q0 * fma(-0.5 * x * q0, q0, 1.5);
    out[4 * i + 0] = ulps(r0, rc);
    out[4 * i + 1] = ulps(r1, rc);
    out[4 * i + 2] = ulps(q0, rs);
    out[4 * i + 3] = ulps(q1, rs);
}
int main() {
    const int n = 1 << 20;
    double* d;
    if (hipMalloc(&d, sizeof(double) * 4 * n) != hipSuccess) return 1;
    hipLaunchKernelGGL(probe, dim3(n / 256), dim3(256), 0, 0, d, n);
    double* h = new double[4 * n];
    if (hipMemcpy(h, d, sizeof(double) * 4 * n, hipMemcpyDeviceToHost) != hipSuccess) return 2;
    const char* names[4] = {"rcp raw", "rcp+1NR", "rsq raw", "rsq+1NR"};
    for (int k = 0; k < 4; ++k) {
        double mx = 0, sum = 0;
        for (int i = 0; i < n; ++i) { mx = fmax(mx, h[4 * i + k]); sum += h[4 * i + k]; }
        printf("%s: max %.0f ulp, mean %.3f ulp\n", names[k], mx, sum / n);
    }
    return 0;
}
