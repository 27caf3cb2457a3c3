// carmpc_internal.h -- device-side problem layout shared by the HIP kernels and the C ABI.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/carmpc.h"

namespace carmpc {

constexpr int NX = 4;                 // bicycle state dimension (mpc.py:59)
constexpr double UNBOXED_BOUND = 1e9; // |u_i| assumed by the Farkas test for unboxed variables
constexpr double PRE_TOL = 1e-9;      // x0-only row tolerance
constexpr double STEP_FRAC = 0.99;
constexpr double ZERO_ROW = 1e-12;    // relative row-norm threshold for x0-only rows
constexpr double REFINE_MU = 1e-6;    // corrector refinement only once mu <= REFINE_MU

// Small stage matrices by value (symmetrised Q, P, R): kernel arguments, so the grouped
// kernel reads them through the scalar cache.
struct StageMats {
    double A[16];   // [a][b]
    double B[8];    // [a][c]
    double Q[16];   // Qbar_k, k < N
    double P[16];   // Qbar_N (DARE terminal cost)
    double R[4];
};

// Everything a solve kernel reads, as device pointers.  Lives in the problem
// handle; passed to kernels by value.
struct DevProblem {
    int32_t n;      // decision variables (N*nu)
    int32_t nv;     // kernel width (n padded up to a compiled size)
    int32_t p;      // normalised QP rows
    int32_t npre;   // x0-only rows (G_r == 0)
    int32_t ldg;    // row stride of G in doubles (nv + 2: 16B-aligned, conflict-free)
    int32_t boxed;  // input box present
    int32_t N, nu;
    const double* G;      // p x ldg, unit-norm rows, padded columns 0
    const double* H;      // nv x nv (padded diagonal 1)
    const double* w0;     // p
    const double* E;      // p x NX
    const double* pre_w0; // npre
    const double* pre_E;  // npre x NX
    const double* hq;     // nv x NX
    const double* lb;     // nv
    const double* ub;     // nv
    const double* goal;   // NX
    const double* A;      // NX x NX
    const double* B;      // NX x nu
    // stage structure (staged kernel): row r acts on x_{stage[r]} with coef[r]
    const int32_t* row_stage; // p
    const double* row_coef;   // p x NX (normalised with the row)
    const double* Phi;        // N x NX x nu : Phi_m = A^m B
    // staged-kernel layout (capi.hip::stage_layout); staged == 0 -> dense kernel only
    int32_t staged;           // layout present (nu == 2, compiled N, rows fit)
    int32_t srs;              // row slots per lane
    const double* s_coef;     // srs*64 x NX   row coefficients per (slot, lane)
    const double* s_w0;       // srs*64
    const double* s_E;        // srs*64 x NX
    const int32_t* s_valid;   // srs*64
    const double* phi_ac;     // (N+1) x 8: zero block, then Phi_m as [a][c]
    const double* phi_ca;     // (N+1) x 8: zero block, then Phi_m as [c][a]
    const double* s_mats;     // Q 16, P 16 (symmetrised), A 16, B 8, R 4
    // opposite-row pairs (an equality written as two rows, e.g. the goal-box fallback
    // terminal set, mpc.py:107-117); nullptr when the problem has none
    const int32_t* partner;   // p: packed index of the opposite row or -1 (dense kernel)
    const int32_t* s_partner; // srs*64: slot index of the opposite row or -1 (staged kernel)
    // grouped Riccati layout (ipm_riccati.hip, capi.hip::riccati_layout): 16 lanes per QP,
    // lane j owns stage j+1 (segment 0) and j+17 (segment 1); slot e = (seg*8 + s)*16 + j
    int32_t ric;              // layout present: 1 dense stage matrices, 2 bicycle sparsity
    int32_t rseg;             // slots per segment in use (every lane): the kernels skip the rest
    int32_t rone;             // every row sits in segment 0 (horizons <= 16 whose rows fit 16 lanes x 8 slots)
    const double* r_coef;     // 256 x NX  normalised row coefficients c~ of each slot
    const double* r_w0;       // 256
    const double* r_E;        // 256 x NX
    const int32_t* r_valid;   // 256
    const int32_t* r_partner; // 256: slot of the opposite row or -1; nullptr when none
    StageMats mats;
    // constant-disturbance offsets (MPCOutputFBWithDisturbance, mpc.py:631-650): with
    // x = T x0 + S u + ABd d the rows read w = w0 - E x0 - Ed d.  nullptr until
    // carmpc_problem_set_disturbance; per layout (packed rows, x0-only rows, slots)
    const double* Ed;         // p (normalised like w0)
    const double* pre_Ed;     // npre
    const double* s_Ed;       // srs*64 (staged slots)
    const double* r_Ed;       // 256 (Riccati slots)
    // per-instance problems (hetero.hip, ipm_dense.hip HET): G, H, w0, E, hq, pre_w0, pre_E,
    // partner above are the bases of per-instance slices; p / npre per instance
    const int32_t* het_p;     // batch (nullptr: shared problem)
    const int32_t* het_npre;  // batch
    int64_t het_sG, het_sH, het_sHq, het_sRow;   // slice strides in elements
    // per-instance Riccati layout (template slot map): 256 slots per instance
    const double *het_ric_invn, *het_ric_w0, *het_ric_E;   // B x 256, B x 256, B x 256 x NX
    const double *het_A, *het_B, *het_P;                    // B x 16, B x 8, B x 16
};

// CarSimulator.check_input with clip=False (simulator.py:88-95) asserts
//   [a, -a] <= [acc_upper, -acc_lower]   and   [delta, -delta] <= [delta_upper, -delta_lower]
// on Python lists, whose order is lexicographic: the second pair is only compared when the
// first elements are equal.  So an input is rejected when it exceeds the UPPER limit only
// (2 + 0.05, pi/4 + 0.05, simulator.py:44-45); large negative inputs pass.  NaN is rejected
// (NaN != hi, then NaN <= hi is false).
__host__ __device__ inline bool list_le2(double a0, double a1, double b0, double b1) {
    return a0 < b0 || (a0 == b0 && a1 <= b1);
}
__host__ __device__ inline bool input_rejected(double acc, double delta) {
    const double acc_hi = 2.0 + 0.05, acc_lo = -2.0 - 0.05;
    const double del_hi = 3.14159265358979323846 / 4 + 0.05, del_lo = -3.14159265358979323846 / 4 - 0.05;
    return !list_le2(acc, -acc, acc_hi, -acc_lo) || !list_le2(delta, -delta, del_hi, -del_lo);
}

struct Settings {
    double tol, tol_mu;
    int32_t max_iter;
    int32_t kernel;        // 0 auto (riccati, staged, dense), 1 dense, 2 staged, 3 dense 4-wave, 4-6 staged A/B, 7 riccati
    const double* dist;    // per-instance disturbance estimate d (device, batch) or nullptr
    const int32_t* index;  // slot -> instance row (device) or nullptr = identity
    const int32_t* count;  // number of slots (device scalar) or nullptr = batch
    unsigned* claim;       // dynamic instance counter of one launch (zeroed), Riccati kernel; nullptr = static
};


// Dynamic instance claiming (one atomic per instance on a per-launch counter): the
// wavefront-per-QP kernels take the next instance with wave_claim; the counter lives for one
// launch, stream-ordered (launch_with_claim), unless the caller already set s.claim to a zeroed
// counter of its own (carmpc_solve_segments zeroes all segments' counters before its fork).
__device__ __forceinline__ int64_t wave_claim(unsigned* c) {
    unsigned v = 0;
    if ((threadIdx.x & 63) == 0) v = atomicAdd(c, 1u);
    return (int64_t)__builtin_amdgcn_readfirstlane(v);
}
// Clear n 32-bit words with a small kernel (not hipMemsetAsync, so that a caller may record
// the launch sequence into a HIP graph).
hipError_t launch_zero_u32(unsigned* ptr, int n, hipStream_t stream);
template <class Launch>
inline hipError_t launch_with_claim(Settings s, int64_t batch, hipStream_t stream, Launch&& launch) {
    unsigned* counter = nullptr;
    hipError_t e = hipSuccess;
    if (batch > 1 && !s.claim) {
        if ((e = hipMallocAsync(reinterpret_cast<void**>(&counter), sizeof(unsigned), stream)) != hipSuccess) return e;
        if ((e = launch_zero_u32(counter, 1, stream)) != hipSuccess) return e;
        s.claim = counter;
    }
    e = launch(s);
    if (counter) {
        const hipError_t ef = hipFreeAsync(counter, stream);
        if (e == hipSuccess) e = ef;
    }
    return e;
}

// capi.hip internals shared with the other translation units of the C ABI.
int solve_batch_with_claim(const carmpc_problem* P, int64_t batch, const double* x0, const double* xref, double* u_out,
                           int32_t* status, int32_t* iters, const carmpc_settings* settings, unsigned* claim,
                           hipStream_t stream);
int problem_device(const carmpc_problem* P);
// noalloc.hip: resolve the device address of the static scratch of GPU `dev` (current device) once; problem
// creation calls it, so that carmpc_solve_batch_noalloc itself makes no symbol lookup on that GPU any more
int noalloc_prepare_device(int dev);
int set_error(int code, const char* msg);   // records the calling thread's last-error message, returns code

// Argument blocks of the setup kernels (assembly.hip).
struct AsmArgs {
    int N, nu, n, nt, ns;
    const double *A, *B, *Q, *R, *P;   // NX*NX, NX*nu, NX*NX, nu*nu, NX*NX
    const double *term_A, *term_b;     // nt*NX, nt
    const double *state_A, *state_b;   // ns*NX, ns
    double *T, *S, *H, *h;             // (N+1)NX*NX, (N+1)NX*n, n*n, n*NX
    double *G, *E, *w0, *rownorm;      // p_all*n, p_all*NX, p_all, p_all
    double* Phi;                       // N*NX*nu
    int32_t* row_stage;                // p_all
    double* row_coef;                  // p_all*NX
};
struct PackArgs {
    int n, nv, ldg, p, npre, p_all;
    const int32_t* qp_rows;   // p indices into the assembled rows
    const int32_t* pre_rows;  // npre
    const double *G, *E, *w0, *rownorm, *row_coef;
    const int32_t* row_stage;
    double *Gp, *Ep, *w0p, *pre_w0, *pre_E, *coefp;
    int32_t* stagep;
};
struct ObsArgs {
    int64_t batch;
    int ny, nu;
    int64_t ld_uprev;
    const double *A, *B, *C, *L;   // device: NX*NX, NX*nu, ny*NX, NX*ny
    const double* y;
    const double* uprev;
    double* xhat;
    // disturbance-augmented observer (mpc.py:598-612) when dhat != nullptr
    const double *Bd, *Cd, *L2;    // device: NX, ny, ny
    double* dhat;                  // batch
};
// Closed-loop runner (closed_loop.hip): one launch pair per loop index around the QP launch.
struct LoopArgs {
    int64_t batch;
    int32_t mode, ny, steps_update, last_step;
    int64_t ld_u;
    double dt, l1, goal_tol;
    const double *A, *B;                 // device, from the problem
    const double *C, *L, *Cd, *L2, *Bd;  // device copies of the observer data (modes 1, 2)
    const double* goal;                  // device NX
    double *state, *xhat, *dhat, *u;     // B*NX, B*NX, B, B*ld_u
    const int32_t* qp_status;            // B
    int32_t *outcome, *steps;            // B
    int32_t *idx_cur, *cnt_cur, *idx_next, *cnt_next;
};
hipError_t launch_loop_init(const LoopArgs& a, hipStream_t s);
hipError_t launch_loop_advance(const LoopArgs& a, int32_t i, hipStream_t s);
hipError_t launch_loop_finish(const LoopArgs& a, int32_t i, hipStream_t s);
// Batched 4-variable LPs (lp.hip): max c'x s.t. A x <= b, one per wavefront.
struct LpArgs {
    int64_t nlp;
    const int64_t *a_off, *b_off;   // per LP offsets into the pools (doubles)
    const int32_t* m;               // rows per LP
    const double *a_pool, *b_pool;  // rows (m x 4, row-major) and right-hand sides
    const double* c;                // nlp x 4
    const int32_t* relax;           // per LP row index whose b is raised by relax_amount, -1 none (nullable)
    double relax_amount;
    double tol, tol_gap;
    int32_t max_iter;
    double* value;                  // nlp: max c'x (+inf unbounded)
    double* x;                      // nlp x 4 (nullable)
    int32_t *status, *iters;        // nlp (iters nullable)
};
hipError_t launch_lp(const LpArgs& a, int max_m, hipStream_t s);
// Per-instance linearisation / DARE / assembly (hetero.hip).
constexpr int kHetMaxRows = 1024;
constexpr int kDareMaxIter = 60;
struct LinArgs {
    int64_t batch;
    double dt, l1;
    const double *lin_state, *lin_input;   // B x 4, B x 2
    const double *Q, *R;                   // 16, 4 (device)
    double *A, *B, *P, *K;                 // B x 16, B x 8, B x 16, B x 8 (K nullable)
    int32_t* status;                       // B: doubling steps, -1 = no stabilising solution (P = 0)
};
struct HetAsmArgs {
    int64_t batch;
    int N, nv, ldg, nt, ns;
    const double *A, *B, *P;               // per instance, from LinArgs
    const double *Q, *R;
    const double *term_A, *term_b, *state_A, *state_b;
    double *G, *H, *hq, *w0, *E, *pre_w0, *pre_E;
    int32_t *partner, *p, *npre;
    int64_t strideG, strideH, strideHq, strideRow;
    // Riccati layout of the template (nullptr: none): slot of each assembled row, -1 = x0-only
    const int32_t* tmpl_slot;
    double *ric_invn, *ric_w0, *ric_E;   // B x 256, B x 256, B x 256 x NX
    int32_t* layout_ok;                  // B: the instance splits its rows like the template
};
hipError_t launch_linearize(const LinArgs& a, hipStream_t s);
hipError_t launch_hetero_assembly(const HetAsmArgs& a, hipStream_t s);
hipError_t launch_het_split(int64_t batch, const int32_t* ok, int32_t* idx_ok, int32_t* cnt_ok, int32_t* idx_bad,
                            int32_t* cnt_bad, hipStream_t s);
hipError_t launch_dense_het(const DevProblem& P, int p_max, int64_t batch, const double* x0, const double* xref,
                            double* u_out, int64_t ld_u, int32_t* status, int32_t* iters, const Settings& s,
                            hipStream_t stream, int* unsupported);
hipError_t launch_assembly(const AsmArgs& a, hipStream_t s);
hipError_t launch_pack(const PackArgs& a, hipStream_t s);
hipError_t launch_observer(const ObsArgs& a, hipStream_t s);
hipError_t launch_plant(int64_t batch, double* state, const double* u, int64_t ld_u, double dt, double l1,
                        int32_t* bad, hipStream_t s);

// Solve-kernel launch helpers (ipm_dense.hip).
hipError_t launch_dense(const DevProblem& P, int64_t batch, const double* x0, const double* xref,
                        double* u_out, int64_t ld_u, int32_t* status, int32_t* iters,
                        const Settings& s, hipStream_t stream, int* unsupported);
bool dense_supported(int nv, int p, size_t* lds_bytes);
int dense_pick_nv(int n);

// Grouped stage-form (Riccati) kernel (ipm_riccati.hip).
constexpr int kRicLanes = 16, kRicSeg = 8, kRicSlots = 2 * kRicSeg;
bool riccati_supported_N(int N);
bool riccati_oneseg_N(int N);   // ... with the four-QPs-per-wave instantiation for rows that fit one slot segment
hipError_t launch_riccati(const DevProblem& P, int64_t batch, const double* x0, const double* xref,
                          double* u_out, int64_t ld_u, int32_t* status, int32_t* iters,
                          const Settings& s, hipStream_t stream, int* unsupported, bool het = false);

// Several problems in one Riccati launch (carmpc_solve_segments): descriptors by value in the
// kernel arguments, segment j = instances [off[j], off[j+1]), claim counter j at claim + 16 j.
constexpr int kRicMaxSeg = 4, kRicClaimStride = 16;
struct RicSegs {
    int32_t nseg;
    int64_t off[kRicMaxSeg + 1];
    DevProblem P[kRicMaxSeg];
};
// Work lists of the Riccati launch pipeline (ipm_riccati.hip: rounds of iterations -> polish, then the
// single kernel), device memory for one call.  cnt holds kRicClaimStride words per segment: [0] claim
// counter of round 0's iteration launch; for round r: [4r+1] number of handed-off instances, [4r+2]
// claim counter of the polish launch, [4r+3] number of rejected polishes, [4r+4] claim counter of the
// launch that takes them (round r+1's iterations, or the single kernel after the last round).  The lists
// are per segment, starting at the segment's first instance, and reused from round to round.  A hand-off
// is one 128-byte record (kRicRecWords 32-bit words, one cache line written by the iteration launch and
// read by the polish launch): words 0..15 the lanes' active-set masks (bit s = row slot s active, bits
// 16.. = box rows of the lane's inputs), 16..23 the instance's x0 (4 doubles), 24 the segment-relative
// row, 25 the iterations done.  cnt null: no pipeline.
constexpr int kRicRecWords = 32, kRicRecX0 = 16, kRicRecRow = 24, kRicRecIt = 25;
struct RicWork {
    unsigned* cnt;
    uint32_t* pend_rec;   // total x kRicRecWords: hand-off records in hand-off order
    int32_t* retry_idx;   // total: hand-off records (positions in the segment's list) whose polish was rejected
    int32_t round;        // pipeline round of this launch
    // The last tail[j] instances of segment j skip the iteration and polish launches: the final launch (single kernel)
    // takes them as fresh instances behind the retry list, so that it has work for the group slots that its few, long
    // retries leave idle.
    int32_t tail[kRicMaxSeg];
    // The iterate of every handed-off instance (slacks, multipliers, inputs, stage states: kRicStateDoubles per
    // instance, indexed like pend_rec) for the first state_cap hand-offs of the run: a retry whose state is here resumes
    // from it instead of repeating the iterations that led to the hand-off.  Null / 0: every retry starts over.
    double* state;
    int64_t state_cap;
};
// (2 x 8 row slots + 4 state entries + 5 box quantities x 2 inputs per lane, 32 lanes per QP; the 16-lane layouts need
// as much or half of it)
constexpr int kRicStateDoubles = 960;
constexpr size_t kRicStateMaxBytes = (size_t)2 << 30;   // per call; hand-offs beyond it are not saved
// One round of (iterations, polish): a second one for the instances whose polish was rejected measured
// slower on the 131,072-instance mixed shard (10.9M vs 11.45M QP/s when 6 % were rejected; 2-3 % with the
// correction round and the early polish gate) -- it solves them with the lean kernels but still leaves a
// latency-bound single-kernel tail for the ones rejected again.
constexpr int kRicRounds = 1;
// smallest batch (instances of one call) solved by the pipeline: measured cross-over between 32,768 (single
// kernel 14.3M QP/s, pipeline 14.4M) and 65,536 (14.9M, 16.7M) on RoadOneCarEnv, N = 20
constexpr int kRicPipelineMin = 49152;
static_assert(4 * kRicRounds < kRicClaimStride, "counter slots per segment");
hipError_t launch_riccati_segs(const RicSegs& T, const double* x0, const double* xref, double* u_out, int64_t ld_u,
                               int32_t* status, int32_t* iters, const Settings& s, hipStream_t stream, int* unsupported);

// Stage-structured kernel (ipm_staged.hip).
constexpr int kStagedMaxRS = 4;
bool staged_supported_N(int N);
hipError_t launch_staged(const DevProblem& P, int64_t batch, const double* x0, const double* xref,
                         double* u_out, int64_t ld_u, int32_t* status, int32_t* iters,
                         const Settings& s, hipStream_t stream, int* unsupported);

}  // namespace carmpc
