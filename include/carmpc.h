/*
 * carmpc.h -- C ABI of the MI355X-native batched linear-MPC QP solver.
 *
 * Drop-in boundary for the per-step QP of CarMPC's controllers.  In the
 * reference the boundary is a Python call into cvxpy (no FFI exists):
 *
 *   MPC.__init__                lib/mpc.py:22-117   -> carmpc_problem_create (assembly on device)
 *     predmod / costgen         lib/matrix_gen.py:6-72
 *     constraint stacks         lib/mpc.py:196-253
 *   MPCStateFB.step  cp.Problem(...).solve()   lib/mpc.py:318-335  -> carmpc_solve_batch
 *   MPCOutputFB.step cp.Problem(...).solve()   lib/mpc.py:461-478  -> carmpc_solve_batch
 *   MPCOutputFB.luenberger_observer            lib/mpc.py:439-448  -> carmpc_observer_batch
 *   MPCOutputFBWithDisturbance.step            lib/mpc.py:614-667  -> carmpc_solve_batch_dist
 *     ABd offsets of the constraints           lib/mpc.py:631-650  -> carmpc_problem_set_disturbance
 *   MPCOutputFBWithDisturbance.luenberger_observer lib/mpc.py:598-612 -> carmpc_observer_dist_batch
 *   OutsideTheRegionOfAttractionError          lib/mpc.py:17,336-338 -> status CARMPC_PRIMAL_INFEASIBLE
 *   CarSimulator.step (plant)                  lib/simulator.py:51-69,99-118 -> carmpc_plant_step_batch
 *
 * Conventions
 *   - All matrices are row-major fp64.  Descriptor (host) pointers are read
 *     during the call only.  Batch pointers (x0, u_out, ...) are DEVICE
 *     pointers owned by the caller (e.g. torch-ROCm tensors).
 *   - Every launch is stream-ordered on the given hipStream_t (NULL = default
 *     stream); no hidden host synchronisation in the solve path.
 *   - Functions return 0 on success or a negative CARMPC_E* code; the message
 *     of the last error on the calling thread is available from
 *     carmpc_last_error().
 *   - One problem handle per (environment, horizon, linearisation point);
 *     handles are bound to the device current at creation.
 */
#ifndef CARMPC_H
#define CARMPC_H

#include <stdint.h>
#include <hip/hip_runtime_api.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- status of one QP instance (int32 per instance) ---------------------- */
enum {
    CARMPC_OPTIMAL = 0,            /* KKT residuals within tolerance                    */
    CARMPC_PRIMAL_INFEASIBLE = 1,  /* certificate found; reference raises               */
                                   /* OutsideTheRegionOfAttractionError (mpc.py:336-338) */
    CARMPC_MAX_ITER = 2,
    CARMPC_NUMERICAL = 3
};

/* ---- error codes --------------------------------------------------------- */
enum {
    CARMPC_OK = 0,
    CARMPC_EINVAL = -1,     /* bad argument / shape                                    */
    CARMPC_EUNSUPPORTED = -2, /* size outside the compiled kernel set (e.g. n > 64)    */
    CARMPC_EHIP = -3,       /* HIP runtime error (message has the hipError_t name)     */
    CARMPC_ENOMEM = -4
};

typedef struct carmpc_problem carmpc_problem;

/* Linear-MPC model description: the inputs of MPC.__init__ after linearisation
 * and discretisation (mpc.py:53-54) and DARE (mpc.py:70).  The library builds
 * T, S, H = R_hat + S'Q_hat S, h = S'Q_hat T (matrix_gen.py:6-72) and the
 * stacked constraint rows (mpc.py:196-253) with a device assembly kernel.  */
typedef struct {
    int32_t N;            /* horizon (configuration.py:16), 1..32                      */
    int32_t nx, nu;       /* 4, 2 for the bicycle model                                */
    const double* A;      /* nx*nx  discrete dynamics (mpc.py:164-180)                 */
    const double* B;      /* nx*nu                                                     */
    const double* Q;      /* nx*nx  stage cost (configuration.py:19)                   */
    const double* R;      /* nu*nu  (configuration.py:21)                              */
    const double* P;      /* nx*nx  terminal cost (mpc.py:70)                          */
    int32_t n_state_rows; /* per-step half-spaces c'x_k <= d on x_1..x_N (mpc.py:222-253) */
    const double* state_A;/* n_state_rows*nx                                           */
    const double* state_b;/* n_state_rows                                              */
    int32_t n_term_rows;  /* terminal half-spaces on x_N (mpc.py:96-117), 0 = none      */
    const double* term_A; /* n_term_rows*nx                                            */
    const double* term_b; /* n_term_rows                                               */
    const double* u_lower;/* nu, NULL => no input box (input_constraint=False)         */
    const double* u_upper;/* nu                                                        */
    const double* goal;   /* nx  default reference (mpc.py:46,182-194)                 */
} carmpc_model_desc;

/* Solver settings.  Pass NULL for the defaults
 * {1e-10, 1e-12, 60}. */
typedef struct {
    double tol;        /* primal/dual residual tolerance, relative to 1+||.||_inf */
    double tol_mu;     /* complementarity tolerance (absolute)                     */
    int32_t max_iter;
    int32_t kernel;    /* 0 = auto (grouped Riccati, else staged, else dense), 1 = dense
                          (G,H in LDS), 2 = staged (stage structure, assembled problems
                          with nu=2 and a compiled N), 3 = dense with 4 waves per
                          workgroup, 4-6 = staged variants of experiment builds only (rejected
                          with CARMPC_EUNSUPPORTED otherwise), 7 = grouped stage-form
                          (Riccati) kernel, 32 lanes per QP (assembled, nu=2, N in
                          {5,10,15,20,25}, <= 8 rows per stage; N = 5, 10 with all rows in
                          the first 16 lanes' slots: 16 lanes per QP from 16,384 instances on) */
} carmpc_settings;

/* Which solve kernel `auto` picks for this problem: 1 dense, 2 staged, 7 grouped Riccati. */
int carmpc_problem_kernel(const carmpc_problem* prob);

/* Flops per IPM iteration the given kernel (0 auto, 1 dense, 2 staged, 7 Riccati) performs on
 * behalf of one QP, counting every stage recursion once (useful work); the canonical dense-IPM
 * count is carmpc_canonical_flops_per_iter. */
double carmpc_executed_flops_per_iter(const carmpc_problem* prob, int32_t kernel);
/* Flops per IPM iteration the hardware is asked to perform for one QP: as above, except that
 * every matrix-core instruction of the Riccati kernel counts as a full 4x4x4 product (128 flops
 * per QP) although part of its operands are structural zeros or replicated columns.  Equals
 * carmpc_executed_flops_per_iter for kernels that issue no matrix-core instructions. */
double carmpc_issued_flops_per_iter(const carmpc_problem* prob, int32_t kernel);

/* Build one problem on the current device (assembly kernel + row normalisation). */
int carmpc_problem_create(const carmpc_model_desc* desc, carmpc_problem** out);

/* Generic dense variant (no stage structure): min 1/2u'Hu + (hq(x0-xref))'u
 * s.t. G u <= w0 - E x0, lb <= u <= ub.  H n*n, G p*n, w0 p, E p*nx, hq n*nx,
 * lb/ub n (NULL = no box), goal nx.  Host pointers. */
int carmpc_problem_create_dense(int32_t n, int32_t p, int32_t nx, const double* H, const double* G,
                                const double* w0, const double* E, const double* hq,
                                const double* lb, const double* ub, const double* goal,
                                carmpc_problem** out);

void carmpc_problem_destroy(carmpc_problem* prob);

/* Sizes: n decision variables, p QP rows after normalisation, npre x0-only rows. */
int carmpc_problem_info(const carmpc_problem* prob, int32_t* n, int32_t* p, int32_t* npre,
                        int32_t* nx, int32_t* N);

/* Copy assembled matrices back to HOST buffers (any pointer may be NULL):
 * T (N+1)nx*nx, S (N+1)nx*n, H n*n, h n*nx, G p_all*n, E p_all*nx, w0 p_all
 * (p_all = rows before normalisation, order: terminal then state blocks as in
 * mpc.py:323-332).  Only valid for carmpc_problem_create problems. */
int carmpc_problem_get(const carmpc_problem* prob, double* T, double* S, double* H, double* h,
                       double* G, double* E, double* w0, int32_t* p_all);

/* Solve B independent QP(x0) instances (MPCStateFB.step semantics, mpc.py:312-349):
 *   x0    B*nx  device, absolute state (constraints use it as is, mpc.py:319)
 *   xref  B*nx  device or NULL (NULL = goal; cost uses x0 - xref, mpc.py:320)
 *   u_out B*n   device, optimal input sequence u_0..u_{N-1}
 *   status, iters  B int32 device (iters may be NULL)
 * Stream-ordered on `stream`.  Device memory beyond the arguments comes from the stream-ordered
 * allocator: a claim counter, and for large batches of the grouped kernel (which then runs as
 * an iteration launch, a polish launch and a launch for the instances whose polish was rejected)
 * the work memory between those launches: 132 bytes per instance of lists, and 7,680 bytes per
 * instance (at most 2 GiB per call) for the iterates from which rejected instances resume.  That
 * memory comes from a pool of the library's own per device, which keeps it between calls and until
 * the process ends (up to that much per call in flight).  Results do not depend on which form
 * ran.  carmpc_solve_batch_noalloc below never takes any of it. */
int carmpc_solve_batch(const carmpc_problem* prob, int64_t batch, const double* x0, const double* xref,
                       double* u_out, int32_t* status, int32_t* iters,
                       const carmpc_settings* settings, hipStream_t stream);

/* carmpc_solve_batch for callers that cannot allocate: code under HIP graph capture, tight
 * serving loops, harnesses that forbid hipMalloc.  It has no counterpart in the reference.  Same
 * arguments and results as carmpc_solve_batch; it always runs the single-launch form of the
 * kernels, whose claim counter (the only device memory that form uses beyond its inputs and
 * outputs) lives in a 256-byte static device array of the library instead of a stream-ordered
 * allocation, and the call makes no hipMalloc, hipFree or other allocating call.  batch <= CARMPC_NOALLOC_MAX_BATCH, else CARMPC_EUNSUPPORTED.
 * All calls on one GPU share that array: the counter is cleared at the start of each call (on
 * `stream`), and two calls whose kernels overlap on one GPU -- from different streams or threads --
 * race on it.  Call it with the problem's device current.  The array's device address is looked up
 * when a problem is created on the GPU, so the call may be the first thing a capturing stream
 * records; a captured call replays like any kernel sequence (the counter is cleared by a small
 * fill kernel, not a memset node). */
#define CARMPC_NOALLOC_MAX_BATCH ((int64_t)1 << 30)
int carmpc_solve_batch_noalloc(const carmpc_problem* prob, int64_t batch, const double* x0, const double* xref,
                               double* u_out, int32_t* status, int32_t* iters,
                               const carmpc_settings* settings, hipStream_t stream);

/* Several problems in one call: instances grouped by problem, segment j is
 * [offsets[j], offsets[j+1]) (host array of nprobs+1).  Row strides follow each problem's n; u_out
 * uses a common row stride ld_u >= max n.  Consecutive segments that run on the same instantiation
 * of the grouped kernel (same horizon, same model structure; up to 4 per launch) are solved by ONE launch whose
 * workgroups move from a drained segment to the remaining ones, so no segment ends with a launch
 * tail of its own; other segments are launched one after another.  Stream-ordered on `stream`. */
int carmpc_solve_segments(const carmpc_problem* const* probs, int32_t nprobs, const int64_t* offsets,
                          const double* x0, const double* xref, double* u_out, int64_t ld_u,
                          int32_t* status, int32_t* iters, const carmpc_settings* settings,
                          hipStream_t stream);

/* MPCOutputFBWithDisturbance (mpc.py:495-667): constant scalar disturbance d with
 * x+ = A x + B u + Bd d.  set_disturbance stores the row offsets Ed (x = T x0 + S u + ABd d,
 * ABd_k = sum_{m<k} A^m Bd, mpc.py:631-637); solve_batch_dist then solves the QPs with
 * w = w0 - E x0 - Ed d_b for per-instance device estimates dist[b]. */
int carmpc_problem_set_disturbance(carmpc_problem* prob, const double* Bd /* NX, host */);
int carmpc_solve_batch_dist(const carmpc_problem* prob, int64_t batch, const double* x0, const double* xref,
                            const double* dist, double* u_out, int32_t* status, int32_t* iters,
                            const carmpc_settings* settings, hipStream_t stream);
/* Disturbance-augmented Luenberger observer (mpc.py:598-612), in place on device:
 * e = y - C xhat - Cd dhat; xhat <- A xhat + Bd dhat + B uprev + L1 e; dhat <- dhat + L2 . e.
 * C (ny x NX), L1 (NX x ny), Cd, L2 (ny), Bd (NX) are host arrays, compared by value with the
 * sets already staged on the problem (carmpc_problem_set_observer). */
int carmpc_observer_dist_batch(const carmpc_problem* prob, int64_t batch, const double* y, int32_t ny,
                               const double* C, const double* L1, const double* Cd, const double* L2,
                               const double* Bd, double* xhat, double* dhat, const double* uprev,
                               int64_t ld_uprev, hipStream_t stream);

/* Stage a set of observer constants on the device ahead of time (MPCOutputFB.__init__ sets C
 * and L once, mpc.py:387-404; MPCOutputFBWithDisturbance Bd, Cd, L1, L2, mpc.py:530-546).  The
 * observer entry points do this themselves on the first call with a given set of values; calls
 * with values already staged only launch the kernel (no copy, no host synchronisation).
 * Cd, L2, Bd may all be NULL (plain Luenberger observer).  Blocking; at most 64 distinct sets. */
int carmpc_problem_set_observer(const carmpc_problem* prob, int32_t ny, const double* C, const double* L,
                                const double* Cd, const double* L2, const double* Bd);

/* Luenberger observer (mpc.py:439-448), in place on device:
 *   xhat <- A xhat + B uprev + L (y - C xhat)
 * y B*ny, xhat B*nx, uprev rows at stride ld_uprev (first nu entries used),
 * C ny*nx, L nx*ny host arrays (staged on the device at their first use, see
 * carmpc_problem_set_observer).  A, B come from the problem. */
int carmpc_observer_batch(const carmpc_problem* prob, int64_t batch, const double* y, int32_t ny,
                          const double* C, const double* L, double* xhat, const double* uprev,
                          int64_t ld_uprev, hipStream_t stream);

/* Nonlinear kinematic bicycle plant, forward Euler (simulator.py:51-69):
 * state <- state + dt*[v cos psi, v sin psi, v/l1 tan delta, a];
 * u rows at stride ld_u (first 2 entries).  Returns CARMPC_OK; per-instance
 * input-limit violations (simulator.py:83-97) are flagged in bad (nullable). */
int carmpc_plant_step_batch(int64_t batch, double* state, const double* u, int64_t ld_u, double dt,
                            double l1, int32_t* bad, hipStream_t stream);

/* ---- closed loop on the device -------------------------------------
 * The examples' runner loops for B independent cars, entirely on the GPU:
 *   examples/run_MPCStateFB.py:26-43   mode 0: u = controller.step(state)
 *   examples/run_MPCOutputFB.py:28-50  mode 1: u = controller.step(C state) (Luenberger, mpc.py:439-492)
 *   MPCOutputFBWithDisturbance         mode 2: observer mpc.py:598-612 + ABd offsets (needs
 *                                      carmpc_problem_set_disturbance)
 * Per loop index i = 0, 1, ...: check_input(u) (simulator.py:83-97, clip=False), plant step
 * (simulator.py:51-69,99-118), every steps_update-th index the controller step (observer + QP),
 * then the runner's stop tests: QP infeasible -> OutsideTheRegionOfAttractionError; all
 * |x - goal| <= goal_tol (goal_tol <= 0: no goal test); i >= last_step.
 * The reference loop is the special case batch = 1. */
enum {
    CARMPC_LOOP_RUNNING = -1,
    CARMPC_LOOP_REACHED = 0,          /* goal test passed (run_MPCStateFB.py:40)              */
    CARMPC_LOOP_INFEASIBLE = 1,       /* QP infeasible: OutsideTheRegionOfAttractionError     */
    CARMPC_LOOP_INPUT_VIOLATION = 2,  /* check_input assertion (simulator.py:92-95)           */
    CARMPC_LOOP_TIMEOUT = 3,          /* i >= last_step                                       */
    CARMPC_LOOP_SOLVER_FAILURE = 4    /* QP status MAX_ITER / NUMERICAL                       */
};

typedef struct {
    int32_t mode;          /* 0 state feedback, 1 output feedback, 2 output feedback with disturbance */
    int32_t steps_update;  /* STEPS_UPDATE (configuration.py:13)                                       */
    int32_t last_step;     /* loop index of the time-out: 151 (i > 30/DT), 75 (i >= 15/DT)             */
    int32_t ny;            /* output rows (modes 1, 2), <= 8                                           */
    double dt;             /* DT_SIMULATION                                                            */
    double l1;             /* wheelbase (simulator.py:6-13)                                            */
    double goal_tol;       /* 0.1 in run_MPCStateFB.py:40; <= 0 disables the goal test                 */
    const double* goal;    /* NX host, NULL = the problem's goal                                       */
    const double *C, *L;   /* ny*NX, NX*ny host (modes 1, 2; L = L1 in mode 2)                         */
    const double *Cd, *L2, *Bd; /* ny, ny, NX host (mode 2)                                            */
} carmpc_loop_desc;

/* Runs the loop to completion for every instance.  Device buffers: state B*NX (in: start,
 * out: final), xhat B*NX (modes 1, 2: in init_state, out estimate), dhat B (mode 2), xref B*NX
 * or NULL (QP reference, NULL = goal), u B*n (out: last QP solution), outcome/steps B int32
 * (steps = loop indices executed).  Synchronises the stream once every check_every indices to
 * stop when no instance is left (check_every <= 0: never, run to last_step). */
int carmpc_closed_loop_batch(const carmpc_problem* prob, int64_t batch, const carmpc_loop_desc* loop,
                             double* state, double* xhat, double* dhat, const double* xref, double* u,
                             int32_t* outcome, int32_t* steps, int32_t check_every,
                             const carmpc_settings* settings, hipStream_t stream);

/* ---- batched small LPs (terminal-set synthesis) ------------------------
 * lib/terminal_set.py:45-67 (one LP per state row and horizon k) and the redundancy removal of
 * the final set (polytope.reduce, called at terminal_set.py:197) as one launch:
 *   LP l:  maximise c_l'x  s.t.  A_l x <= b_l (+ relax_amount on row relax[l]),  x in R^4
 * A_l = a_pool[a_off[l] ...] (m[l] x 4 row-major), b_l = b_pool[b_off[l] ...] (m[l]); all
 * DEVICE pointers; relax may be NULL.  value[l] = optimum (+inf when unbounded), x (nullable)
 * nlp x 4, status/iters (iters nullable) nlp.  m[l] <= 1016; max_m is the largest m[l]. */
enum {
    CARMPC_LP_OPTIMAL = 0,
    CARMPC_LP_UNBOUNDED = 1,
    CARMPC_LP_MAX_ITER = 2,
    CARMPC_LP_NUMERICAL = 3
};
int carmpc_lp_batch(int64_t nlp, int32_t max_m, const int64_t* a_off, const int64_t* b_off, const int32_t* m,
                    const double* a_pool, const double* b_pool, const double* c, const int32_t* relax,
                    double relax_amount, double* value, double* x, int32_t* status, int32_t* iters,
                    hipStream_t stream);

/* ---- per-instance linearisation -------------------------------------
 * Every instance b has its own linearisation point (lin_state[b], lin_input[b]): A, B
 * (mpc.py:128-180), P = DARE (mpc.py:67-74; zeros when no stabilising solution), K (mpc.py:80-81)
 * and the condensed QP (matrix_gen.py:6-72, mpc.py:196-253) are built on the device, one slice per
 * instance, and solved by the dense kernel reading each instance's slice.  Rows, Q, R, box and goal
 * are shared (they do not depend on the linearisation point). */
typedef struct carmpc_hetero carmpc_hetero;
typedef struct {
    int32_t N;             /* horizon, 2N <= 64                                   */
    double dt, l1;         /* DT_CONTROL, wheelbase (simulator.py:6)              */
    const double *Q, *R;   /* 4x4, 2x2 host                                       */
    int32_t n_state_rows;  /* per-step rows on x_1..x_N (mpc.py:222-253)          */
    const double *state_A, *state_b;
    int32_t n_term_rows;   /* terminal rows on x_N (mpc.py:96-117)                 */
    const double *term_A, *term_b;
    const double *u_lower, *u_upper; /* nu = 2 host, NULL = no input box       */
    const double* goal;    /* NX host, default reference                          */
} carmpc_hetero_desc;
/* Allocates per-instance slices for `batch` instances (n_term + N n_state <= 256 rows). */
int carmpc_hetero_create(const carmpc_hetero_desc* desc, int64_t batch, carmpc_hetero** out);
void carmpc_hetero_destroy(carmpc_hetero* h);
/* (Re)linearise every instance at lin_state (B x 4) / lin_input (B x 2), DEVICE pointers, and
 * assemble its QP; stream-ordered, no host synchronisation (successive linearisation loops). */
int carmpc_hetero_linearize(carmpc_hetero* h, const double* lin_state, const double* lin_input,
                            hipStream_t stream);
/* carmpc_solve_batch semantics over the handle's instances (x0, xref B x 4, u_out B x 2N). */
int carmpc_hetero_solve(const carmpc_hetero* h, const double* x0, const double* xref, double* u_out,
                        int32_t* status, int32_t* iters, const carmpc_settings* settings, hipStream_t stream);
/* Copy the per-instance model and QP slices to HOST buffers (any pointer may be NULL; synchronous):
 * A B x 16, B B x 8, P B x 16, K B x 8, dare_status B (doubling steps, -1 = no stabilising solution,
 * P = 0), p / npre B (QP rows / x0-only rows), G B x R x ldg (unit rows), H B x nv x nv,
 * hq B x nv x 4, w0 B x R, E B x R x 4 with dims = {R, ldg, nv, n, rows before the split, B}. */
int carmpc_hetero_get(const carmpc_hetero* h, double* A, double* B, double* P, double* K, int32_t* dare_status,
                      int32_t* p, int32_t* npre, double* G, double* H, double* hq, double* w0, double* E,
                      int64_t* dims);

/* ---- CPU twins: the same QP on the host's cores -----------------------------------------
 * The reference solves its per-step QP on the CPU (cp.Problem(...).solve(), lib/mpc.py:334-335,
 * 477-478, 652-653).  These entry points are that path for hosts without a GPU and the plumbing
 * configuration "run_MPCStateFB, N = 10, CPU QP path": the same stage-form interior-point method
 * as the device kernel (tolerances, row normalisation, x0-only preconditions, infeasibility
 * certificate, active-set polish), in plain host code.  They make no device call and work in a
 * process that never touches a GPU.  Same descriptors and argument meaning as the device entry
 * points, except that every batch pointer is a HOST pointer and the last argument is a thread
 * count (<= 0: all hardware threads) instead of a stream.  nu = 2. */
typedef struct carmpc_cpu_problem carmpc_cpu_problem;
int carmpc_cpu_problem_create(const carmpc_model_desc* desc, carmpc_cpu_problem** out);   /* <-> carmpc_problem_create */
void carmpc_cpu_problem_destroy(carmpc_cpu_problem* prob);
int carmpc_cpu_problem_info(const carmpc_cpu_problem* prob, int32_t* n, int32_t* p, int32_t* npre, int32_t* nx,
                            int32_t* N);
int carmpc_cpu_problem_set_disturbance(carmpc_cpu_problem* prob, const double* Bd /* NX */);
/* MPCStateFB.step / MPCOutputFB.step QP (mpc.py:318-335, 461-478) for `batch` states. */
int carmpc_cpu_solve_batch(const carmpc_cpu_problem* prob, int64_t batch, const double* x0, const double* xref,
                           double* u_out, int32_t* status, int32_t* iters, const carmpc_settings* settings,
                           int32_t threads);
/* MPCOutputFBWithDisturbance.step QP (mpc.py:630-653): w = w0 - E x0 - Ed d_b. */
int carmpc_cpu_solve_batch_dist(const carmpc_cpu_problem* prob, int64_t batch, const double* x0, const double* xref,
                                const double* dist, double* u_out, int32_t* status, int32_t* iters,
                                const carmpc_settings* settings, int32_t threads);

/* Canonical per-iteration flop count of the dense condensed IPM
 * p*n^2 + n^3/3 + 6n^2 + 12pn with p = general rows. */
double carmpc_canonical_flops_per_iter(int32_t n, int32_t p);

const char* carmpc_last_error(void);
const char* carmpc_version(void);

#ifdef __cplusplus
}
#endif
#endif /* CARMPC_H */
