// Per-instance linearisation and condensed-QP assembly on the device.
//
// Every instance b carries its own linearisation point (x_e, u_e); the reference computes one
// per controller in MPC.__init__:
//   linearized_model    mpc.py:128-161   Jacobians of the kinematic bicycle at (x_e, u_e)
//   discretized_model   mpc.py:164-180   A = I + dt A_lin, B = dt B_lin
//   dare                mpc.py:67-74     P = DARE(A, B, Q, R) (scipy.linalg.solve_discrete_are),
//                                        zeros when it has no stabilising solution
//   K                   mpc.py:80-81     K = -(R + B'PB)^-1 B'PA
//   predmod / costgen   matrix_gen.py:6-72, constraint stacks mpc.py:196-253
//
// linearize_kernel: one thread per instance; the DARE by the structure-preserving doubling
// algorithm (W = I + G_k H_k, A_{k+1} = A_k W^-1 A_k, G_{k+1} = G_k + A_k W^-1 G_k A_k',
// H_{k+1} = H_k + A_k' H_k W^-1 A_k, H_k -> P quadratically in the closed-loop spectral radius).
// hetero_assembly_kernel: one 256-thread workgroup per instance -- the assembly of assembly.hip
// plus the row split / normalisation / opposite-pair search the host does for a shared
// problem -- into per-instance slices read by the dense solve kernel (ipm_dense.hip, HET).
#include "carmpc_internal.h"

namespace carmpc {

namespace {

// in-place inverse of a 4x4 matrix (Gauss-Jordan, partial pivoting); false if singular
__device__ bool inv4(double* M) {
    double a[4][8];
    for (int i = 0; i < 4; ++i)
        for (int j = 0; j < 4; ++j) {
            a[i][j] = M[i * 4 + j];
            a[i][j + 4] = i == j ? 1.0 : 0.0;
        }
    for (int c = 0; c < 4; ++c) {
        int piv = c;
        double best = fabs(a[c][c]);
        for (int r = c + 1; r < 4; ++r)
            if (fabs(a[r][c]) > best) {
                best = fabs(a[r][c]);
                piv = r;
            }
        if (!(best > 0.0)) return false;
        if (piv != c)
            for (int j = 0; j < 8; ++j) {
                const double t = a[c][j];
                a[c][j] = a[piv][j];
                a[piv][j] = t;
            }
        const double inv = 1.0 / a[c][c];
        for (int j = 0; j < 8; ++j) a[c][j] *= inv;
        for (int r = 0; r < 4; ++r)
            if (r != c) {
                const double f = a[r][c];
                for (int j = 0; j < 8; ++j) a[r][j] = fma(-f, a[c][j], a[r][j]);
            }
    }
    for (int i = 0; i < 4; ++i)
        for (int j = 0; j < 4; ++j) M[i * 4 + j] = a[i][j + 4];
    return true;
}

__device__ void mm4(const double* X, const double* Y, double* Z) {   // Z = X Y
    for (int i = 0; i < 4; ++i)
        for (int j = 0; j < 4; ++j) {
            double v = 0.0;
            for (int k = 0; k < 4; ++k) v = fma(X[i * 4 + k], Y[k * 4 + j], v);
            Z[i * 4 + j] = v;
        }
}

__global__ void linearize_kernel(LinArgs a) {
    const int64_t b = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= a.batch) return;
    const double psi = a.lin_state[b * 4 + 2], v = a.lin_state[b * 4 + 3];
    const double delta = a.lin_input[b * 2 + 1];
    const double dt = a.dt, l1 = a.l1;
    // mpc.py:128-161, then A = dt A_lin + I, B = dt B_lin (mpc.py:164-180)
    double A[16], B[8];
    for (int i = 0; i < 16; ++i) A[i] = (i % 5 == 0) ? 1.0 : 0.0;
    A[0 * 4 + 2] = dt * (-v * sin(psi));
    A[0 * 4 + 3] = dt * cos(psi);
    A[1 * 4 + 2] = dt * (v * cos(psi));
    A[1 * 4 + 3] = dt * sin(psi);
    A[2 * 4 + 3] = dt * (tan(delta) / l1);
    const double cd = cos(delta);
    for (int i = 0; i < 8; ++i) B[i] = 0.0;
    B[2 * 2 + 1] = dt * (v / l1 * 1.0 / (cd * cd));
    B[3 * 2 + 0] = dt * 1.0;
    const double* R = a.R;
    const double det = R[0] * R[3] - R[1] * R[2];
    const double Ri[4] = {R[3] / det, -R[1] / det, -R[2] / det, R[0] / det};
    double Ak[16], G[16], H[16];
    for (int i = 0; i < 16; ++i) {
        Ak[i] = A[i];
        H[i] = a.Q[i];
    }
    for (int i = 0; i < 4; ++i)
        for (int j = 0; j < 4; ++j) {
            double s = 0.0;
            for (int c = 0; c < 2; ++c)
                for (int d = 0; d < 2; ++d) s += B[i * 2 + c] * Ri[c * 2 + d] * B[j * 2 + d];
            G[i * 4 + j] = s;
        }
    int it = 0;
    bool conv = false;
    for (; it < kDareMaxIter; ++it) {
        double W[16], AW[16], An[16], T1[16], T2[16];
        mm4(G, H, W);
        for (int i = 0; i < 4; ++i) W[i * 5] += 1.0;
        if (!inv4(W)) break;
        mm4(Ak, W, AW);        // A W^-1
        mm4(AW, Ak, An);       // A W^-1 A
        mm4(AW, G, T1);        // A W^-1 G
        mm4(H, W, T2);         // H W^-1
        double Gn[16], Hn[16], dmax = 0.0, hmax = 0.0;
        for (int i = 0; i < 4; ++i)
            for (int j = 0; j < 4; ++j) {
                double s = 0.0, t = 0.0;
                for (int k = 0; k < 4; ++k) {
                    s = fma(T1[i * 4 + k], Ak[j * 4 + k], s);   // (A W^-1 G) A'
                    double u = 0.0;
                    for (int m = 0; m < 4; ++m) u = fma(T2[k * 4 + m], Ak[m * 4 + j], u);   // (H W^-1 A)_{kj}
                    t = fma(Ak[k * 4 + i], u, t);                // A' (H W^-1 A)
                }
                Gn[i * 4 + j] = G[i * 4 + j] + s;
                Hn[i * 4 + j] = H[i * 4 + j] + t;
            }
        for (int i = 0; i < 16; ++i) {
            dmax = fmax(dmax, fabs(Hn[i] - H[i]));
            hmax = fmax(hmax, fabs(Hn[i]));
            Ak[i] = An[i];
            G[i] = Gn[i];
            H[i] = Hn[i];
        }
        if (!(hmax < INFINITY)) break;
        if (dmax <= 1e-15 * hmax) {
            conv = true;
            break;
        }
    }
    // no stabilising solution: P = 0 as the reference's except-branch (mpc.py:71-74)
    double P[16];
    for (int i = 0; i < 4; ++i)
        for (int j = 0; j < 4; ++j) P[i * 4 + j] = conv ? 0.5 * (H[i * 4 + j] + H[j * 4 + i]) : 0.0;
    double PB[8], PA[16];
    for (int i = 0; i < 4; ++i)
        for (int c = 0; c < 2; ++c) {
            double s = 0.0;
            for (int k = 0; k < 4; ++k) s = fma(P[i * 4 + k], B[k * 2 + c], s);
            PB[i * 2 + c] = s;
        }
    mm4(P, A, PA);
    double S2[4], BPA[8];
    for (int c = 0; c < 2; ++c) {
        for (int d = 0; d < 2; ++d) {
            double s = R[c * 2 + d];
            for (int k = 0; k < 4; ++k) s = fma(B[k * 2 + c], PB[k * 2 + d], s);
            S2[c * 2 + d] = s;
        }
        for (int j = 0; j < 4; ++j) {
            double s = 0.0;
            for (int k = 0; k < 4; ++k) s = fma(B[k * 2 + c], PA[k * 4 + j], s);
            BPA[c * 4 + j] = s;
        }
    }
    const double d2 = S2[0] * S2[3] - S2[1] * S2[2];
    const double Si[4] = {S2[3] / d2, -S2[1] / d2, -S2[2] / d2, S2[0] / d2};
    for (int i = 0; i < 16; ++i) {
        a.A[b * 16 + i] = A[i];
        a.P[b * 16 + i] = P[i];
    }
    for (int i = 0; i < 8; ++i) a.B[b * 8 + i] = B[i];
    if (a.K)
        for (int c = 0; c < 2; ++c)
            for (int j = 0; j < 4; ++j) a.K[b * 8 + c * 4 + j] = -(Si[c * 2 + 0] * BPA[j] + Si[c * 2 + 1] * BPA[4 + j]);
    if (a.status) a.status[b] = conv ? it + 1 : -1;
}

__global__ void __launch_bounds__(256) hetero_assembly_kernel(HetAsmArgs a) {
    __shared__ double Ap[33 * 16];      // A^0 .. A^N (N <= 32)
    __shared__ double Phi[32 * 8];      // Phi_m = A^m B, m < N
    __shared__ double Qk[2][16];        // Q (k < N) and P (k = N) of this instance
    __shared__ double nrm[kHetMaxRows];
    __shared__ int32_t qp_of[kHetMaxRows], pre_of[kHetMaxRows];
    __shared__ int32_t counts[2];
    const int64_t b = blockIdx.x;
    const int tid = threadIdx.x;
    const int N = a.N, n = 2 * N, nv = a.nv, ldg = a.ldg, p_all = a.nt + a.ns * N;
    const double* A = a.A + b * 16;
    const double* B = a.B + b * 8;
    if (tid < 16) {
        Ap[tid] = (tid / 4 == tid % 4) ? 1.0 : 0.0;
        Qk[0][tid] = 0.5 * (a.Q[tid] + a.Q[(tid % 4) * 4 + tid / 4]);
        Qk[1][tid] = 0.5 * (a.P[b * 16 + tid] + a.P[b * 16 + (tid % 4) * 4 + tid / 4]);
    }
    __syncthreads();
    for (int k = 1; k <= N; ++k) {
        double v = 0.0;
        if (tid < 16) {
            const int i = tid / 4, j = tid % 4;
            for (int m = 0; m < 4; ++m) v += Ap[(k - 1) * 16 + i * 4 + m] * A[m * 4 + j];
        }
        __syncthreads();
        if (tid < 16) Ap[k * 16 + tid] = v;
        __syncthreads();
    }
    for (int e = tid; e < N * 8; e += blockDim.x) {
        const int m = e / 8, r = (e / 2) % 4, c = e % 2;
        double v = 0.0;
        for (int q = 0; q < 4; ++q) v += Ap[m * 16 + r * 4 + q] * B[q * 2 + c];
        Phi[e] = v;
    }
    __syncthreads();
    // S_k[r][(j, c)] = Phi_{k-j-1}[r][c] for j < k, else 0 (matrix_gen.py:6-32)
    auto S = [&](int k, int r, int col) -> double {
        const int j = col >> 1, c = col & 1;
        return j < k ? Phi[(k - j - 1) * 8 + r * 2 + c] : 0.0;
    };
    double* H = a.H + b * a.strideH;
    double* hq = a.hq + b * a.strideHq;
    // H = R_hat + sum_k S_k' Q_k S_k (Q_N = P), symmetric by construction, padded to nv
    for (int e = tid; e < nv * nv; e += blockDim.x) {
        const int x = e / nv, y = e % nv;
        if (x > y) continue;
        double v;
        if (y >= n) {
            v = (x == y) ? 1.0 : 0.0;
        } else {
            v = (x / 2 == y / 2) ? 0.5 * (a.R[(x % 2) * 2 + (y % 2)] + a.R[(y % 2) * 2 + (x % 2)]) : 0.0;
            for (int k = y / 2 + 1; k <= N; ++k) {
                const double* Q = Qk[k == N ? 1 : 0];
                for (int r = 0; r < 4; ++r) {
                    double t = 0.0;
                    for (int q = 0; q < 4; ++q) t += Q[r * 4 + q] * S(k, q, y);
                    v += S(k, r, x) * t;
                }
            }
        }
        H[x * nv + y] = v;
        H[y * nv + x] = v;
    }
    // hq = S' Q_hat T (matrix_gen.py:35-72), rows padded to nv
    for (int e = tid; e < nv * 4; e += blockDim.x) {
        const int x = e / 4, y = e % 4;
        double v = 0.0;
        if (x < n)
            for (int k = x / 2 + 1; k <= N; ++k) {
                const double* Q = Qk[k == N ? 1 : 0];
                for (int r = 0; r < 4; ++r) {
                    double t = 0.0;
                    for (int q = 0; q < 4; ++q) t += Q[r * 4 + q] * Ap[k * 16 + q * 4 + y];
                    v += S(k, r, x) * t;
                }
            }
        hq[e] = v;
    }
    // general rows: terminal (stage N) then state blocks (row j on x_1..x_N), mpc.py:196-253
    auto row = [&](int e, int* stage, const double** c, double* bb) {
        if (e < a.nt) {
            *stage = N;
            *c = a.term_A + e * 4;
            *bb = a.term_b[e];
        } else {
            const int j = (e - a.nt) / N, k = (e - a.nt) % N + 1;
            *stage = k;
            *c = a.state_A + j * 4;
            *bb = a.state_b[j];
        }
    };
    for (int e = tid; e < p_all; e += blockDim.x) {
        int st;
        const double* c;
        double bb;
        row(e, &st, &c, &bb);
        double s2 = 0.0;
        for (int col = 0; col < n; ++col) {
            double v = 0.0;
            for (int r = 0; r < 4; ++r) v += c[r] * S(st, r, col);
            s2 += v * v;
        }
        nrm[e] = sqrt(s2);
    }
    __syncthreads();
    // QP rows and x0-only rows in order (capi.hip::classify: ZERO_ROW x the largest norm)
    if (tid == 0) {
        double mx = 0.0;
        for (int e = 0; e < p_all; ++e) mx = fmax(mx, nrm[e]);
        const double thr = ZERO_ROW * mx;
        int nq = 0, np = 0;
        for (int e = 0; e < p_all; ++e) {
            if (nrm[e] > thr) qp_of[nq++] = e;
            else pre_of[np++] = e;
        }
        counts[0] = nq;
        counts[1] = np;
        a.p[b] = nq;
        a.npre[b] = np;
    }
    __syncthreads();
    const int nq = counts[0], np = counts[1];
    double* G = a.G + b * a.strideG;
    double* w0 = a.w0 + b * a.strideRow;
    double* E = a.E + b * a.strideRow * 4;
    double* pw = a.pre_w0 + b * a.strideRow;
    double* pE = a.pre_E + b * a.strideRow * 4;
    int32_t* partner = a.partner + b * a.strideRow;
    for (int r = tid; r < nq; r += blockDim.x) {
        const int e = qp_of[r];
        int st;
        const double* c;
        double bb;
        row(e, &st, &c, &bb);
        const double inv = 1.0 / nrm[e];
        for (int col = 0; col < ldg; ++col) {
            double v = 0.0;
            if (col < n)
                for (int q = 0; q < 4; ++q) v += c[q] * S(st, q, col);
            G[(int64_t)r * ldg + col] = v * inv;
        }
        for (int y = 0; y < 4; ++y) {
            double v = 0.0;
            for (int q = 0; q < 4; ++q) v += c[q] * Ap[st * 16 + q * 4 + y];
            E[r * 4 + y] = v * inv;
        }
        w0[r] = bb * inv;
        // opposite row (an equality as two rows): same stage, negated coefficients and bound
        int pr = -1;
        for (int r2 = 0; r2 < nq && pr < 0; ++r2) {
            if (r2 == r) continue;
            int st2;
            const double* c2;
            double b2;
            row(qp_of[r2], &st2, &c2, &b2);
            if (st2 != st || b2 != -bb) continue;
            bool same = true;
            for (int q = 0; q < 4 && same; ++q) same = c2[q] == -c[q];
            if (same) pr = r2;
        }
        partner[r] = pr;
    }
    // Riccati layout of the template: per-slot 1/||G_r||, w0 / ||G_r||, E / ||G_r|| (unused slots 0)
    if (a.tmpl_slot) {
        constexpr int kSlots = kRicSlots * kRicLanes;
        double* iv = a.ric_invn + b * kSlots;
        double* rw = a.ric_w0 + b * kSlots;
        double* rE = a.ric_E + b * kSlots * 4;
        for (int e = tid; e < kSlots; e += blockDim.x) {
            iv[e] = 0.0;
            rw[e] = 0.0;
            for (int y = 0; y < 4; ++y) rE[e * 4 + y] = 0.0;
        }
        __syncthreads();
        const double thr = ZERO_ROW * [&] {
            double mx = 0.0;
            for (int e = 0; e < p_all; ++e) mx = fmax(mx, nrm[e]);
            return mx;
        }();
        int bad = 0;
        for (int e = tid; e < p_all; e += blockDim.x) {
            const bool qp = nrm[e] > thr;
            const int slot = a.tmpl_slot[e];
            if (qp != (slot >= 0)) {
                bad = 1;
                continue;
            }
            if (!qp) continue;
            int st;
            const double* c;
            double bb;
            row(e, &st, &c, &bb);
            const double inv = 1.0 / nrm[e];
            iv[slot] = inv;
            rw[slot] = bb * inv;
            for (int y = 0; y < 4; ++y) {
                double v = 0.0;
                for (int q = 0; q < 4; ++q) v += c[q] * Ap[st * 16 + q * 4 + y];
                rE[slot * 4 + y] = v * inv;
            }
        }
        bad = __syncthreads_or(bad);
        if (tid == 0) a.layout_ok[b] = bad ? 0 : 1;
    }
    for (int r = tid; r < np; r += blockDim.x) {
        const int e = pre_of[r];
        int st;
        const double* c;
        double bb;
        row(e, &st, &c, &bb);
        for (int y = 0; y < 4; ++y) {
            double v = 0.0;
            for (int q = 0; q < 4; ++q) v += c[q] * Ap[st * 16 + q * 4 + y];
            pE[r * 4 + y] = v;
        }
        pw[r] = bb;
    }
}

// split the instances into those the Riccati kernel takes (template layout) and the rest
__global__ void het_split_kernel(int64_t batch, const int32_t* ok, int32_t* idx_ok, int32_t* cnt_ok, int32_t* idx_bad,
                                 int32_t* cnt_bad) {
    const int64_t b = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= batch) return;
    if (ok[b]) idx_ok[atomicAdd(cnt_ok, 1)] = (int32_t)b;
    else idx_bad[atomicAdd(cnt_bad, 1)] = (int32_t)b;
}

}  // namespace

hipError_t launch_het_split(int64_t batch, const int32_t* ok, int32_t* idx_ok, int32_t* cnt_ok, int32_t* idx_bad,
                            int32_t* cnt_bad, hipStream_t s) {
    if (batch <= 0) return hipSuccess;
    // cleared by the fill kernel, like every counter of the library (a caller may capture the launches)
    hipError_t e = launch_zero_u32(reinterpret_cast<unsigned*>(cnt_ok), 1, s);
    if (e == hipSuccess) e = launch_zero_u32(reinterpret_cast<unsigned*>(cnt_bad), 1, s);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(het_split_kernel, dim3((unsigned)((batch + 255) / 256)), dim3(256), 0, s, batch, ok, idx_ok,
                       cnt_ok, idx_bad, cnt_bad);
    return hipGetLastError();
}

hipError_t launch_linearize(const LinArgs& a, hipStream_t s) {
    if (a.batch <= 0) return hipSuccess;
    hipLaunchKernelGGL(linearize_kernel, dim3((unsigned)((a.batch + 63) / 64)), dim3(64), 0, s, a);
    return hipGetLastError();
}

hipError_t launch_hetero_assembly(const HetAsmArgs& a, hipStream_t s) {
    if (a.batch <= 0) return hipSuccess;
    hipLaunchKernelGGL(hetero_assembly_kernel, dim3((unsigned)a.batch), dim3(256), 0, s, a);
    return hipGetLastError();
}

}  // namespace carmpc
