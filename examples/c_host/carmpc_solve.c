/*
 * Minimal C host of the drop-in boundary (include/carmpc.h): no Python, no torch.
 *
 *   carmpc_solve <problem.bin> <x0.bin> <u.bin> <status.bin>
 *
 * problem.bin (little endian): int32 N, n_state_rows, n_term_rows; double A[16], B[8], Q[16],
 * R[4], P[16], state_A[ns*4], state_b[ns], term_A[nt*4], term_b[nt], u_lower[2], u_upper[2],
 * goal[4].  x0.bin: batch x 4 doubles.  Writes u (batch x 2N doubles) and status (batch int32).
 * This is what a maintainer's MPC.__init__ / MPCStateFB.step would call through an FFI
 * (mpc.py:22-117 -> carmpc_problem_create, mpc.py:318-338 -> carmpc_solve_batch).
 */
#include <stdio.h>
#include <stdlib.h>

#include <hip/hip_runtime_api.h>

#include "carmpc.h"

static void* slurp(const char* path, size_t* len) {
    FILE* f = fopen(path, "rb");
    if (!f) return NULL;
    fseek(f, 0, SEEK_END);
    *len = (size_t)ftell(f);
    fseek(f, 0, SEEK_SET);
    void* buf = malloc(*len ? *len : 1);
    if (fread(buf, 1, *len, f) != *len) {
        fclose(f);
        free(buf);
        return NULL;
    }
    fclose(f);
    return buf;
}

#define CHECK(x)                                                                      \
    do {                                                                              \
        int rc_ = (x);                                                                \
        if (rc_ != 0) {                                                               \
            fprintf(stderr, "%s failed: %d (%s)\n", #x, rc_, carmpc_last_error());   \
            return 1;                                                                 \
        }                                                                             \
    } while (0)
#define HCHECK(x)                                                                 \
    do {                                                                          \
        hipError_t e_ = (x);                                                      \
        if (e_ != hipSuccess) {                                                   \
            fprintf(stderr, "%s failed: %s\n", #x, hipGetErrorString(e_));        \
            return 1;                                                             \
        }                                                                         \
    } while (0)

int main(int argc, char** argv) {
    if (argc != 5) {
        fprintf(stderr, "usage: %s problem.bin x0.bin u.bin status.bin\n", argv[0]);
        return 2;
    }
    size_t plen = 0, xlen = 0;
    char* pb = (char*)slurp(argv[1], &plen);
    double* x0 = (double*)slurp(argv[2], &xlen);
    if (!pb || !x0 || plen < 12) {
        fprintf(stderr, "cannot read inputs\n");
        return 2;
    }
    const int32_t* hdr = (const int32_t*)pb;
    const int N = hdr[0], ns = hdr[1], nt = hdr[2];
    const double* d = (const double*)(pb + 12);
    carmpc_model_desc desc = {0};
    desc.N = N; desc.nx = 4; desc.nu = 2;
    desc.A = d; d += 16;
    desc.B = d; d += 8;
    desc.Q = d; d += 16;
    desc.R = d; d += 4;
    desc.P = d; d += 16;
    desc.n_state_rows = ns; desc.state_A = d; d += 4 * ns;
    desc.state_b = d; d += ns;
    desc.n_term_rows = nt; desc.term_A = d; d += 4 * nt;
    desc.term_b = d; d += nt;
    desc.u_lower = d; d += 2;
    desc.u_upper = d; d += 2;
    desc.goal = d; d += 4;
    if ((size_t)((const char*)d - pb) != plen) {
        fprintf(stderr, "problem.bin size mismatch\n");
        return 2;
    }
    const int64_t batch = (int64_t)(xlen / (4 * sizeof(double)));
    const int n = 2 * N;

    carmpc_problem* prob = NULL;
    CHECK(carmpc_problem_create(&desc, &prob));
    double *dx0, *du;
    int32_t* dst;
    HCHECK(hipMalloc((void**)&dx0, xlen));
    HCHECK(hipMalloc((void**)&du, sizeof(double) * batch * n));
    HCHECK(hipMalloc((void**)&dst, sizeof(int32_t) * batch));
    HCHECK(hipMemcpy(dx0, x0, xlen, hipMemcpyHostToDevice));
    hipStream_t s;
    HCHECK(hipStreamCreate(&s));
    CHECK(carmpc_solve_batch(prob, batch, dx0, NULL, du, dst, NULL, NULL, s));
    HCHECK(hipStreamSynchronize(s));
    double* u = (double*)malloc(sizeof(double) * batch * n);
    int32_t* st = (int32_t*)malloc(sizeof(int32_t) * batch);
    HCHECK(hipMemcpy(u, du, sizeof(double) * batch * n, hipMemcpyDeviceToHost));
    HCHECK(hipMemcpy(st, dst, sizeof(int32_t) * batch, hipMemcpyDeviceToHost));
    FILE* fu = fopen(argv[3], "wb");
    FILE* fs = fopen(argv[4], "wb");
    if (!fu || !fs) return 2;
    fwrite(u, sizeof(double), (size_t)batch * n, fu);
    fwrite(st, sizeof(int32_t), (size_t)batch, fs);
    fclose(fu);
    fclose(fs);
    printf("solved %lld instances with kernel %d (%s)\n", (long long)batch, carmpc_problem_kernel(prob),
           carmpc_version());
    carmpc_problem_destroy(prob);
    hipFree(dx0);
    hipFree(du);
    hipFree(dst);
    hipStreamDestroy(s);
    return 0;
}
