// assembly.hip -- condensed-QP assembly on the device (one workgroup per problem).
//
// Restates, as a CDNA4 kernel, what the reference computes in MPC.__init__ and
// rebuilds every step in Python loops:
//   predmod  lib/matrix_gen.py:6-32   T = [A^0;..;A^N], S block (i,j) = A^{i-j-1}B
//   costgen  lib/matrix_gen.py:35-72  H = R_hat + S'Q_hat S, h = S'Q_hat T (Q_hat[N] = P)
//   stacks   lib/mpc.py:196-253       terminal rows on x_N, then per constraint row j
//                                     a block of N rows on x_1..x_N
//   step     lib/mpc.py:319,326,332   G = A_rows S, E = A_rows T, w0 = b_rows
// Also writes Phi_m = A^m B (m = 0..N-1) and the 2-norm of every general row
// (the host uses them to split x0-only rows and normalise).
//
// Sizes are tiny (N <= 32): one 256-thread workgroup, LDS for the powers of A.
#include "carmpc_internal.h"

namespace carmpc {


__global__ void __launch_bounds__(256) assembly_kernel(AsmArgs a) {
    __shared__ double Ap[33 * NX * NX];  // A^0 .. A^N (N <= 32)
    const int tid = threadIdx.x;
    const int N = a.N, nu = a.nu, n = a.n;
    // powers of A: sequential in k, 16 threads per product
    if (tid < NX * NX) Ap[tid] = (tid / NX == tid % NX) ? 1.0 : 0.0;
    __syncthreads();
    for (int k = 1; k <= N; ++k) {
        double v = 0.0;
        if (tid < NX * NX) {
            const int i = tid / NX, j = tid % NX;
#pragma unroll
            for (int m = 0; m < NX; ++m) v += Ap[(k - 1) * NX * NX + i * NX + m] * a.A[m * NX + j];
        }
        __syncthreads();
        if (tid < NX * NX) Ap[k * NX * NX + tid] = v;
        __syncthreads();
    }
    // T and Phi
    for (int e = tid; e < (N + 1) * NX * NX; e += blockDim.x) a.T[e] = Ap[e];
    for (int e = tid; e < N * NX * nu; e += blockDim.x) {
        const int m = e / (NX * nu), r = (e / nu) % NX, c = e % nu;
        double v = 0.0;
        for (int q = 0; q < NX; ++q) v += Ap[m * NX * NX + r * NX + q] * a.B[q * nu + c];
        a.Phi[e] = v;
    }
    __syncthreads();
    // S: row 4i+r, col j*nu+c  = (A^{i-j-1} B)[r][c] for i > j
    const int srows = (N + 1) * NX;
    for (int e = tid; e < srows * n; e += blockDim.x) {
        const int row = e / n, col = e % n;
        const int i = row / NX, r = row % NX, j = col / nu, c = col % nu;
        a.S[e] = (i > j) ? a.Phi[(i - j - 1) * NX * nu + r * nu + c] : 0.0;
    }
    __syncthreads();
    // H = R_hat + sum_k S_k' Q_k S_k ; h = sum_k S_k' Q_k A^k   (Q_N = P)
    for (int e = tid; e < n * n; e += blockDim.x) {
        const int x = e / n, y = e % n;
        double v = (x / nu == y / nu) ? a.R[(x % nu) * nu + (y % nu)] : 0.0;
        for (int k = 1; k <= N; ++k) {
            const double* Qk = (k == N) ? a.P : a.Q;
            for (int r = 0; r < NX; ++r) {
                const double sx = a.S[(k * NX + r) * n + x];
                if (sx == 0.0) continue;
                double t = 0.0;
                for (int q = 0; q < NX; ++q) t += Qk[r * NX + q] * a.S[(k * NX + q) * n + y];
                v += sx * t;
            }
        }
        a.H[e] = v;
    }
    for (int e = tid; e < n * NX; e += blockDim.x) {
        const int x = e / NX, y = e % NX;
        double v = 0.0;
        for (int k = 1; k <= N; ++k) {
            const double* Qk = (k == N) ? a.P : a.Q;
            for (int r = 0; r < NX; ++r) {
                const double sx = a.S[(k * NX + r) * n + x];
                if (sx == 0.0) continue;
                double t = 0.0;
                for (int q = 0; q < NX; ++q) t += Qk[r * NX + q] * Ap[k * NX * NX + q * NX + y];
                v += sx * t;
            }
        }
        a.h[e] = v;
    }
    // general rows: terminal (stage N) then state blocks (row j, stage 1..N)
    const int p_all = a.nt + a.ns * N;
    for (int e = tid; e < p_all; e += blockDim.x) {
        int stage;
        const double* c;
        double b;
        if (e < a.nt) {
            stage = N; c = a.term_A + e * NX; b = a.term_b[e];
        } else {
            const int j = (e - a.nt) / N, k = (e - a.nt) % N + 1;
            stage = k; c = a.state_A + j * NX; b = a.state_b[j];
        }
        a.w0[e] = b;
        a.row_stage[e] = stage;
        double nrm = 0.0;
        for (int col = 0; col < n; ++col) {
            double v = 0.0;
            for (int r = 0; r < NX; ++r) v += c[r] * a.S[(stage * NX + r) * n + col];
            a.G[e * n + col] = v;
            nrm += v * v;
        }
        for (int col = 0; col < NX; ++col) {
            double v = 0.0;
            for (int r = 0; r < NX; ++r) v += c[r] * Ap[stage * NX * NX + r * NX + col];
            a.E[e * NX + col] = v;
            a.row_coef[e * NX + col] = c[col];
        }
        a.rownorm[e] = sqrt(nrm);
    }
}

// Pack the normalised QP rows into the solver layout: G (p x ldg, padded), w0, E,
// stage/coef scaled by 1/||G_r||; x0-only rows go to pre_w0/pre_E.
__global__ void pack_rows_kernel(PackArgs a) {
    const int tid = blockIdx.x * blockDim.x + threadIdx.x;
    const int stride = gridDim.x * blockDim.x;
    for (int e = tid; e < a.p * a.ldg; e += stride) {
        const int r = e / a.ldg, col = e % a.ldg;
        const int src = a.qp_rows[r];
        a.Gp[e] = col < a.n ? a.G[src * a.n + col] / a.rownorm[src] : 0.0;
    }
    for (int e = tid; e < a.p * NX; e += stride) {
        const int r = e / NX, k = e % NX;
        const int src = a.qp_rows[r];
        a.Ep[e] = a.E[src * NX + k] / a.rownorm[src];
        a.coefp[e] = a.row_coef[src * NX + k] / a.rownorm[src];
    }
    for (int r = tid; r < a.p; r += stride) {
        const int src = a.qp_rows[r];
        a.w0p[r] = a.w0[src] / a.rownorm[src];
        a.stagep[r] = a.row_stage[src];
    }
    for (int e = tid; e < a.npre * NX; e += stride) {
        const int r = e / NX, k = e % NX;
        a.pre_E[e] = a.E[a.pre_rows[r] * NX + k];
    }
    for (int r = tid; r < a.npre; r += stride) a.pre_w0[r] = a.w0[a.pre_rows[r]];
}

// Luenberger observer (mpc.py:439-448): xhat <- A xhat + B uprev + L (y - C xhat)

// With a.dhat (MPCOutputFBWithDisturbance, mpc.py:598-612): innovation e = y - C xhat - Cd d,
// xhat <- A xhat + Bd d + B uprev + L e,  d <- d + L2 . e.
__global__ void observer_kernel(ObsArgs a) {
    const int64_t b = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= a.batch) return;
    double x[NX], innov[8];
#pragma unroll
    for (int k = 0; k < NX; ++k) x[k] = a.xhat[b * NX + k];
    const double d = a.dhat ? a.dhat[b] : 0.0;
    for (int r = 0; r < a.ny; ++r) {
        double v = a.y[b * a.ny + r];
#pragma unroll
        for (int k = 0; k < NX; ++k) v -= a.C[r * NX + k] * x[k];
        if (a.dhat) v -= a.Cd[r] * d;
        innov[r] = v;
    }
    double out[NX];
#pragma unroll
    for (int i = 0; i < NX; ++i) {
        double v = 0.0;
#pragma unroll
        for (int k = 0; k < NX; ++k) v += a.A[i * NX + k] * x[k];
        if (a.dhat) v += a.Bd[i] * d;
        for (int c = 0; c < a.nu; ++c) v += a.B[i * a.nu + c] * a.uprev[b * a.ld_uprev + c];
        for (int r = 0; r < a.ny; ++r) v += a.L[i * a.ny + r] * innov[r];
        out[i] = v;
    }
#pragma unroll
    for (int k = 0; k < NX; ++k) a.xhat[b * NX + k] = out[k];
    if (a.dhat) {
        double dn = d;
        for (int r = 0; r < a.ny; ++r) dn += a.L2[r] * innov[r];
        a.dhat[b] = dn;
    }
}

// Nonlinear kinematic bicycle, forward Euler (simulator.py:51-69); input
// limits of check_input (simulator.py:83-97) flagged per instance.
__global__ void plant_kernel(int64_t batch, double* state, const double* u, int64_t ld_u, double dt, double l1,
                             int32_t* bad) {
    const int64_t b = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= batch) return;
    const double x = state[b * 4 + 0], y = state[b * 4 + 1], psi = state[b * 4 + 2], v = state[b * 4 + 3];
    const double acc = u[b * ld_u + 0], delta = u[b * ld_u + 1];
    const double t = tan(delta);
    state[b * 4 + 0] = v * cos(psi) * dt + x;
    state[b * 4 + 1] = v * sin(psi) * dt + y;
    state[b * 4 + 2] = v / l1 * t * dt + psi;
    state[b * 4 + 3] = acc * dt + v;
    if (bad) bad[b] = input_rejected(acc, delta) ? 1 : 0;
}

__global__ void zero_u32_kernel(unsigned* ptr, int n) {
    for (int i = threadIdx.x; i < n; i += blockDim.x) ptr[i] = 0u;
}
hipError_t launch_zero_u32(unsigned* ptr, int n, hipStream_t s) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(zero_u32_kernel, dim3(1), dim3(64), 0, s, ptr, n);
    return hipGetLastError();
}

hipError_t launch_assembly(const AsmArgs& a, hipStream_t s) {
    hipLaunchKernelGGL(assembly_kernel, dim3(1), dim3(256), 0, s, a);
    return hipGetLastError();
}
hipError_t launch_pack(const PackArgs& a, hipStream_t s) {
    const int work = a.p * a.ldg > 256 ? a.p * a.ldg : 256;
    const int blocks = (work + 255) / 256 < 1024 ? (work + 255) / 256 : 1024;
    hipLaunchKernelGGL(pack_rows_kernel, dim3(blocks), dim3(256), 0, s, a);
    return hipGetLastError();
}
hipError_t launch_observer(const ObsArgs& a, hipStream_t s) {
    if (a.batch <= 0) return hipSuccess;
    hipLaunchKernelGGL(observer_kernel, dim3((unsigned)((a.batch + 255) / 256)), dim3(256), 0, s, a);
    return hipGetLastError();
}
hipError_t launch_plant(int64_t batch, double* state, const double* u, int64_t ld_u, double dt, double l1,
                        int32_t* bad, hipStream_t s) {
    if (batch <= 0) return hipSuccess;
    hipLaunchKernelGGL(plant_kernel, dim3((unsigned)((batch + 255) / 256)), dim3(256), 0, s, batch, state, u, ld_u,
                       dt, l1, bad);
    return hipGetLastError();
}

}  // namespace carmpc
