// capi.hip -- the extern "C" boundary declared in include/carmpc.h.
//
// Setup (carmpc_problem_create) mirrors MPC.__init__ (lib/mpc.py:22-117): the
// caller passes the discretised model, costs, DARE terminal cost and the
// constraint half-spaces; the device assembly kernel builds the condensed QP
// (matrix_gen.py:6-72, mpc.py:196-253).  The solve path (carmpc_solve_batch)
// replaces cp.Problem(...).solve() of mpc.py:334-335 / 477-478.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

#include "carmpc_internal.h"

using namespace carmpc;


struct carmpc_problem {
    DevProblem dev{};
    int device = 0;
    int nx = NX;
    int p_all = 0;        // rows before normalisation (assembled problems)
    bool assembled = false;
    std::vector<void*> allocs;
    // assembled full matrices (device), for carmpc_problem_get
    double *T = nullptr, *S = nullptr, *H = nullptr, *h = nullptr, *G_all = nullptr, *E_all = nullptr,
           *w0_all = nullptr;
    // host bookkeeping for the disturbance offsets (carmpc_problem_set_disturbance)
    double A_host[16] = {};
    const double* coef_all_dev = nullptr;   // p_all x NX row coefficients on x_k
    const int32_t* stage_all_dev = nullptr; // p_all
    std::vector<double> nrm_all;            // p_all condensed row norms
    std::vector<int32_t> qp_rows, pre_rows; // packed QP rows / x0-only rows (assembled indices)
    std::vector<int32_t> stage_slot, ric_slot;   // slot of each packed row per layout (empty: none)
    // Observer constants (C, L | Cd, L2, Bd) staged on the device once per distinct value set
    // (carmpc_problem_set_observer, or the first carmpc_observer*_batch call that passes them):
    // later calls with the same host values only launch.  Superseded sets stay allocated until the
    // problem is destroyed, so a launch still queued on some stream never loses its operands.
    static constexpr int kObsStage = 2 * 8 * NX + 8 + 8 + NX;   // C 8xNX | L NXx8 | Cd 8 | L2 8 | Bd NX
    struct ObsSet {
        double host[kObsStage];
        double* dev;
    };
    mutable std::mutex obs_mu;
    mutable std::vector<std::unique_ptr<ObsSet>> obs_sets;
    ~carmpc_problem() {
        for (void* p : allocs) (void)hipFree(p);
        for (auto& set : obs_sets) (void)hipFree(set->dev);
    }
    template <class T_>
    hipError_t alloc(T_** ptr, size_t count) {
        void* p = nullptr;
        hipError_t e = hipMalloc(&p, std::max<size_t>(count, 1) * sizeof(T_));
        if (e == hipSuccess) {
            allocs.push_back(p);
            *ptr = static_cast<T_*>(p);
        }
        return e;
    }
};

struct carmpc_hetero {
    DevProblem dev{};     // shared part (n, nv, ldg, boxed, N, nu, lb, ub, goal) + slice bases
    int64_t batch = 0;
    int p_all = 0, nt = 0, ns = 0;
    double dt = 0.0, l1 = 0.0;
    int device = 0;
    bool ready = false;   // carmpc_hetero_linearize ran
    std::vector<void*> allocs;
    double *Q = nullptr, *R = nullptr, *tA = nullptr, *tb = nullptr, *sA = nullptr, *sb = nullptr;
    double *A = nullptr, *B = nullptr, *P = nullptr, *K = nullptr;
    int32_t* lin_status = nullptr;
    double *G = nullptr, *H = nullptr, *hq = nullptr, *w0 = nullptr, *E = nullptr, *pw = nullptr, *pE = nullptr;
    int32_t *partner = nullptr, *p = nullptr, *npre = nullptr;
    // Riccati path: the template problem's layout and per-instance slot data
    carmpc_problem* tmpl = nullptr;
    DevProblem ric{};     // template dev + per-instance slice pointers (ipm_riccati HET)
    int32_t* tmpl_slot = nullptr;
    double *ric_invn = nullptr, *ric_w0 = nullptr, *ric_E = nullptr;
    int32_t *layout_ok = nullptr, *idx_ok = nullptr, *idx_bad = nullptr, *cnt = nullptr;
    ~carmpc_hetero() {
        for (void* q : allocs) (void)hipFree(q);
        delete tmpl;
    }
    template <class T_>
    hipError_t alloc(T_** ptr, size_t count) {
        void* q = nullptr;
        hipError_t e = hipMalloc(&q, std::max<size_t>(count, 1) * sizeof(T_));
        if (e == hipSuccess) {
            allocs.push_back(q);
            *ptr = static_cast<T_*>(q);
        }
        return e;
    }
    template <class T_>
    hipError_t upload(T_** ptr, const T_* src, size_t count) {
        hipError_t e = alloc(ptr, count);
        if (e == hipSuccess && count) e = hipMemcpy(*ptr, src, count * sizeof(T_), hipMemcpyHostToDevice);
        return e;
    }
};

namespace {
thread_local std::string g_err;

int fail(int code, const std::string& msg) {
    g_err = msg;
    return code;
}
int hipfail(hipError_t e, const char* what) {
    g_err = std::string(what) + ": " + hipGetErrorName(e) + " (" + hipGetErrorString(e) + ")";
    return CARMPC_EHIP;
}
#define HIP_TRY(expr, what)                          \
    do {                                             \
        hipError_t _e = (expr);                      \
        if (_e != hipSuccess) return hipfail(_e, what); \
    } while (0)

template <class T_>
hipError_t upload(carmpc_problem* P, T_** dst, const T_* src, size_t count) {
    hipError_t e = P->alloc(dst, count);
    if (e != hipSuccess) return e;
    if (count && src) e = hipMemcpy(*dst, src, count * sizeof(T_), hipMemcpyHostToDevice);
    return e;
}

Settings make_settings(const carmpc_settings* s) {
    Settings out{1e-10, 1e-12, 60, 0, nullptr};
    if (s) {
        if (s->tol > 0) out.tol = s->tol;
        if (s->tol_mu > 0) out.tol_mu = s->tol_mu;
        if (s->max_iter > 0) out.max_iter = s->max_iter;
        out.kernel = s->kernel;
    }
    return out;
}

// Split rows into QP rows (nonzero G_r) and x0-only rows, given host row norms.
void classify(const std::vector<double>& nrm, std::vector<int32_t>& qp, std::vector<int32_t>& pre) {
    double mx = 0.0;
    for (double v : nrm) mx = std::max(mx, v);
    const double thr = ZERO_ROW * mx;
    for (size_t r = 0; r < nrm.size(); ++r) (nrm[r] > thr ? qp : pre).push_back((int32_t)r);
}

// Upload the per-variable arrays padded to nv (H: identity on the pad; hq rows 0;
// box [-1,1] on the pad so padded variables sit at 0).
int finish_padded(carmpc_problem* P, const double* H, const double* hq, const double* lb, const double* ub,
                  const double* goal) {
    const int n = P->dev.n, nv = P->dev.nv;
    std::vector<double> Hp((size_t)nv * nv, 0.0), hqp((size_t)nv * NX, 0.0), lbp(nv, -1.0), ubp(nv, 1.0);
    for (int i = 0; i < nv; ++i)
        for (int j = 0; j < nv; ++j)
            Hp[(size_t)i * nv + j] = (i < n && j < n) ? 0.5 * (H[(size_t)i * n + j] + H[(size_t)j * n + i])
                                                      : (i == j ? 1.0 : 0.0);
    for (int i = 0; i < n; ++i)
        for (int k = 0; k < NX; ++k) hqp[(size_t)i * NX + k] = hq[(size_t)i * NX + k];
    if (lb && ub)
        for (int i = 0; i < n; ++i) { lbp[i] = lb[i]; ubp[i] = ub[i]; }
    double *dH, *dhq, *dlb, *dub, *dgoal;
    HIP_TRY(upload(P, &dH, Hp.data(), Hp.size()), "upload H");
    HIP_TRY(upload(P, &dhq, hqp.data(), hqp.size()), "upload hq");
    HIP_TRY(upload(P, &dlb, lbp.data(), lbp.size()), "upload lb");
    HIP_TRY(upload(P, &dub, ubp.data(), ubp.size()), "upload ub");
    HIP_TRY(upload(P, &dgoal, goal, NX), "upload goal");
    P->dev.H = dH; P->dev.hq = dhq; P->dev.lb = dlb; P->dev.ub = dub; P->dev.goal = dgoal;
    P->dev.boxed = (lb && ub) ? 1 : 0;
    return CARMPC_OK;
}

// Opposite-row pairs of the packed rows (oracle/qp.py::opposite_pairs): row r' with
// G_r' = -G_r, w0_r' = -w0_r, E_r' = -E_r exactly.  G is p x ldg (first n columns used).
std::vector<int32_t> find_pairs(const std::vector<double>& G, int p, int ldg, int n, const std::vector<double>& w0,
                                const std::vector<double>& E, int* npairs) {
    std::vector<int32_t> partner(p, -1);
    *npairs = 0;
    for (int r = 0; r < p; ++r) {
        for (int r2 = 0; r2 < p && partner[r] < 0; ++r2) {
            if (r2 == r || w0[r2] != -w0[r]) continue;
            bool same = true;
            for (int k = 0; k < NX && same; ++k) same = E[(size_t)r2 * NX + k] == -E[(size_t)r * NX + k];
            for (int j = 0; j < n && same; ++j) same = G[(size_t)r2 * ldg + j] == -G[(size_t)r * ldg + j];
            if (same) {
                partner[r] = r2;
                ++*npairs;
            }
        }
    }
    return partner;
}

// Download the packed rows, find opposite pairs, upload D.partner (left null when none).
int setup_pairs(carmpc_problem* P, std::vector<int32_t>& partner) {
    DevProblem& D = P->dev;
    partner.assign(D.p, -1);
    if (D.p == 0) return CARMPC_OK;
    std::vector<double> G((size_t)D.p * D.ldg), w0(D.p), E((size_t)D.p * NX);
    HIP_TRY(hipMemcpy(G.data(), D.G, sizeof(double) * G.size(), hipMemcpyDeviceToHost), "readback G");
    HIP_TRY(hipMemcpy(w0.data(), D.w0, sizeof(double) * w0.size(), hipMemcpyDeviceToHost), "readback w0");
    HIP_TRY(hipMemcpy(E.data(), D.E, sizeof(double) * E.size(), hipMemcpyDeviceToHost), "readback E");
    int np = 0;
    partner = find_pairs(G, D.p, D.ldg, D.n, w0, E, &np);
    if (np > 0) {
        int32_t* dp = nullptr;
        HIP_TRY(upload(P, &dp, partner.data(), partner.size()), "upload partner");
        D.partner = dp;
    }
    return CARMPC_OK;
}

// Row layout of the staged kernel (ipm_staged.hip): a lane's row slots all act on one
// predicted state.  State row j of stage k -> lane (k-1) + 32*(j%2), slot j/2; terminal
// row t (stage N) -> the t-th "tail" lane (L%32 >= N) round-robin, slot t / #tail.
// qp[r] is the assembled index of packed row r (terminal rows first, then N rows per
// state row j: mpc.py:196-253).  Returns false when the problem does not fit.
int stage_layout(carmpc_problem* P, const carmpc_model_desc* d, const std::vector<int32_t>& qp, const double* Phi_dev,
                 const std::vector<int32_t>& partner, bool* ok) {
    *ok = false;
    DevProblem& D = P->dev;
    const int N = D.N, nt = d->n_term_rows;
    if (D.nu != 2 || !staged_supported_N(N) || D.n != D.nv) return CARMPC_OK;
    std::vector<int> tail;
    for (int L = 0; L < 64; ++L)
        if ((L & 31) >= N) tail.push_back(L);
    if (nt > 0 && tail.empty()) return CARMPC_OK;
    std::vector<int> lane_of(D.p), slot_of(D.p);
    int rs = 1;
    for (int r = 0; r < D.p; ++r) {
        const int e = qp[r];
        if (e < nt) {
            lane_of[r] = tail[e % tail.size()];
            slot_of[r] = e / (int)tail.size();
        } else {
            const int j = (e - nt) / N, k = (e - nt) % N + 1;
            lane_of[r] = (k - 1) + 32 * (j % 2);
            slot_of[r] = j / 2;
        }
        rs = std::max(rs, slot_of[r] + 1);
    }
    if (rs > kStagedMaxRS) return CARMPC_OK;
    // packed rows (normalised on the device) back to the host
    std::vector<double> coefp((size_t)D.p * NX), w0p(D.p), Ep((size_t)D.p * NX), phi((size_t)N * NX * 2);
    if (D.p > 0) {
        HIP_TRY(hipMemcpy(coefp.data(), D.row_coef, sizeof(double) * coefp.size(), hipMemcpyDeviceToHost), "readback coef");
        HIP_TRY(hipMemcpy(w0p.data(), D.w0, sizeof(double) * w0p.size(), hipMemcpyDeviceToHost), "readback w0");
        HIP_TRY(hipMemcpy(Ep.data(), D.E, sizeof(double) * Ep.size(), hipMemcpyDeviceToHost), "readback E");
    }
    HIP_TRY(hipMemcpy(phi.data(), Phi_dev, sizeof(double) * phi.size(), hipMemcpyDeviceToHost), "readback Phi");
    const size_t ns = (size_t)rs * 64;
    std::vector<double> sc(ns * NX, 0.0), sw(ns, 0.0), sE(ns * NX, 0.0);
    std::vector<int32_t> sv(ns, 0), spart(ns, -1);
    P->stage_slot.assign(D.p, -1);
    for (int r = 0; r < D.p; ++r) {
        const size_t e = (size_t)slot_of[r] * 64 + lane_of[r];
        P->stage_slot[r] = (int32_t)e;
        if (sv[e]) return fail(CARMPC_EINVAL, "stage layout collision");
        sv[e] = 1;
        if (partner[r] >= 0) spart[e] = slot_of[partner[r]] * 64 + lane_of[partner[r]];
        sw[e] = w0p[r];
        for (int a = 0; a < NX; ++a) { sc[e * NX + a] = coefp[(size_t)r * NX + a]; sE[e * NX + a] = Ep[(size_t)r * NX + a]; }
    }
    std::vector<double> pac((size_t)(N + 1) * 8, 0.0), pca((size_t)(N + 1) * 8, 0.0);
    for (int m = 0; m < N; ++m)
        for (int a = 0; a < NX; ++a)
            for (int c = 0; c < 2; ++c) {
                const double v = phi[((size_t)m * NX + a) * 2 + c];
                pac[(size_t)(m + 1) * 8 + a * 2 + c] = v;
                pca[(size_t)(m + 1) * 8 + c * 4 + a] = v;
            }
    std::vector<double> mats(60);
    for (int i = 0; i < 4; ++i)
        for (int j = 0; j < 4; ++j) {
            mats[i * 4 + j] = 0.5 * (d->Q[i * 4 + j] + d->Q[j * 4 + i]);
            mats[16 + i * 4 + j] = 0.5 * (d->P[i * 4 + j] + d->P[j * 4 + i]);
            mats[32 + i * 4 + j] = d->A[i * 4 + j];
        }
    for (int i = 0; i < 8; ++i) mats[48 + i] = d->B[i];
    for (int i = 0; i < 2; ++i)
        for (int j = 0; j < 2; ++j) mats[56 + i * 2 + j] = 0.5 * (d->R[i * 2 + j] + d->R[j * 2 + i]);
    double *dsc, *dsw, *dsE, *dpac, *dpca, *dmats;
    int32_t* dsv;
    HIP_TRY(upload(P, &dsc, sc.data(), sc.size()), "upload s_coef");
    HIP_TRY(upload(P, &dsw, sw.data(), sw.size()), "upload s_w0");
    HIP_TRY(upload(P, &dsE, sE.data(), sE.size()), "upload s_E");
    HIP_TRY(upload(P, &dsv, sv.data(), sv.size()), "upload s_valid");
    HIP_TRY(upload(P, &dpac, pac.data(), pac.size()), "upload phi_ac");
    HIP_TRY(upload(P, &dpca, pca.data(), pca.size()), "upload phi_ca");
    HIP_TRY(upload(P, &dmats, mats.data(), mats.size()), "upload mats");
    D.s_coef = dsc; D.s_w0 = dsw; D.s_E = dsE; D.s_valid = dsv; D.phi_ac = dpac; D.phi_ca = dpca; D.s_mats = dmats;
    if (D.partner) {
        int32_t* dsp = nullptr;
        HIP_TRY(upload(P, &dsp, spart.data(), spart.size()), "upload s_partner");
        D.s_partner = dsp;
    }
    D.srs = rs;
    D.staged = 1;
    *ok = true;
    return CARMPC_OK;
}

// Row layout of the grouped Riccati kernel (ipm_riccati.hip): 16 lanes per QP; lane j owns
// stage j+1 (segment 0) and stage j+17 (segment 1), 8 row slots each.  Rows of stage k < N go
// to the owner's segment; stage-N rows (terminal set + state rows on x_N) fill the owner of
// N first, then the "overflow" segments whose stage number exceeds N (least-filled first).
// Slot e = (seg*8 + s)*16 + j.  Returns ok=false (kernel unavailable) when it does not fit.
// (set while the template problem of a per-instance batch is created: its kernels read both segments, 32 lanes per QP)
thread_local bool g_two_segments_only = false;
int riccati_layout(carmpc_problem* P, const carmpc_model_desc* d, const std::vector<int32_t>& partner, bool* ok) {
    *ok = false;
    DevProblem& D = P->dev;
    const int N = D.N;
    if (D.nu != 2 || !riccati_supported_N(N) || D.n != 2 * N || N > 32) return CARMPC_OK;
    std::vector<int32_t> stage(D.p);
    std::vector<double> coefp((size_t)D.p * NX), w0p(D.p), Ep((size_t)D.p * NX);
    if (D.p > 0) {
        HIP_TRY(hipMemcpy(stage.data(), D.row_stage, sizeof(int32_t) * stage.size(), hipMemcpyDeviceToHost), "readback stage");
        HIP_TRY(hipMemcpy(coefp.data(), D.row_coef, sizeof(double) * coefp.size(), hipMemcpyDeviceToHost), "readback coef");
        HIP_TRY(hipMemcpy(w0p.data(), D.w0, sizeof(double) * w0p.size(), hipMemcpyDeviceToHost), "readback w0");
        HIP_TRY(hipMemcpy(Ep.data(), D.E, sizeof(double) * Ep.size(), hipMemcpyDeviceToHost), "readback E");
    }
    // slots per segment: the smallest count that holds every stage k < N in its owner's segment and
    // the stage-N rows in the owner of N plus the overflow segments (kernels skip the slots above it)
    int per_stage[33] = {};
    for (int r = 0; r < D.p; ++r) {
        const int k = stage[r];
        if (k < 1 || k > N) return CARMPC_OK;
        ++per_stage[k];
    }
    // Placement with `nsg` segments of 16 table lanes: stage k <= 16 nsg in segment (k - 1) / 16, lane (k - 1) % 16;
    // segments whose stage number exceeds N take the stage-N rows that do not fit the owner.  One segment (short
    // horizons) is tried first: the kernels then carry four QPs per wavefront instead of two.
    std::vector<int32_t> slot_of;
    int rseg = 0, rone = 0;
    auto place = [&](int nsg) {
        if (N > 16 * nsg) return false;
        int rs = 1, n_over = 0;
        for (int k = 1; k < N; ++k) rs = std::max(rs, per_stage[k]);
        for (int s2 = 0; s2 < nsg; ++s2)
            for (int j2 = 0; j2 < 16; ++j2) n_over += (j2 + 1 + 16 * s2 > N) ? 1 : 0;
        rs = std::max(rs, (per_stage[N] + n_over) / (n_over + 1));   // ceil(rows_N / (owner + overflow segments))
        if (rs > kRicSeg) return false;
        int cnt[2][16] = {};
        std::vector<int32_t> so(D.p, -1);
        for (int r = 0; r < D.p; ++r) {
            const int k = stage[r];
            int sg = (k - 1) / 16, j = (k - 1) % 16;
            if (cnt[sg][j] >= rs) {
                if (k != N) return false;
                int best = -1;
                for (int s2 = 0; s2 < nsg; ++s2)
                    for (int j2 = 0; j2 < 16; ++j2)
                        if (j2 + 1 + 16 * s2 > N && cnt[s2][j2] < rs && (best < 0 || cnt[s2][j2] < cnt[best / 16][best % 16]))
                            best = s2 * 16 + j2;
                if (best < 0) return false;
                sg = best / 16;
                j = best % 16;
            }
            so[r] = ((sg * kRicSeg + cnt[sg][j]) * 16) + j;
            ++cnt[sg][j];
        }
        slot_of = so;
        rseg = rs;
        return true;
    };
    if (!g_two_segments_only && riccati_oneseg_N(N) && place(1)) rone = 1;
    else if (!place(2)) return CARMPC_OK;
    const int ns = kRicSlots * kRicLanes;
    std::vector<double> sc((size_t)ns * NX, 0.0), sw(ns, 0.0), sE((size_t)ns * NX, 0.0);
    std::vector<int32_t> sv(ns, 0), sp(ns, -1);
    bool any_pair = false;
    for (int r = 0; r < D.p; ++r) {
        const int e = slot_of[r];
        sv[e] = 1;
        sw[e] = w0p[r];
        for (int a = 0; a < NX; ++a) { sc[(size_t)e * NX + a] = coefp[(size_t)r * NX + a]; sE[(size_t)e * NX + a] = Ep[(size_t)r * NX + a]; }
        if (!partner.empty() && partner[r] >= 0) {
            sp[e] = slot_of[partner[r]];
            any_pair = true;
        }
    }
    double *dsc, *dsw, *dsE;
    int32_t* dsv;
    HIP_TRY(upload(P, &dsc, sc.data(), sc.size()), "upload r_coef");
    HIP_TRY(upload(P, &dsw, sw.data(), sw.size()), "upload r_w0");
    HIP_TRY(upload(P, &dsE, sE.data(), sE.size()), "upload r_E");
    HIP_TRY(upload(P, &dsv, sv.data(), sv.size()), "upload r_valid");
    D.r_coef = dsc; D.r_w0 = dsw; D.r_E = dsE; D.r_valid = dsv; D.r_partner = nullptr;
    if (any_pair) {
        int32_t* dsp = nullptr;
        HIP_TRY(upload(P, &dsp, sp.data(), sp.size()), "upload r_partner");
        D.r_partner = dsp;
    }
    StageMats& M = D.mats;
    for (int i = 0; i < 4; ++i)
        for (int jj = 0; jj < 4; ++jj) {
            M.A[i * 4 + jj] = d->A[i * 4 + jj];
            M.Q[i * 4 + jj] = 0.5 * (d->Q[i * 4 + jj] + d->Q[jj * 4 + i]);
            M.P[i * 4 + jj] = 0.5 * (d->P[i * 4 + jj] + d->P[jj * 4 + i]);
        }
    for (int i = 0; i < 8; ++i) M.B[i] = d->B[i];
    for (int i = 0; i < 2; ++i)
        for (int jj = 0; jj < 2; ++jj) M.R[i * 2 + jj] = 0.5 * (d->R[i * 2 + jj] + d->R[jj * 2 + i]);
    // structural zeros of the bicycle model (ipm_riccati.hip::BicycleModel): exact zeros outside
    // the masks and a unit diagonal of A select the sparse instantiation
    auto zero_outside = [](const double* X, int rows, int cols, const int* keep, int nkeep) {
        for (int i = 0; i < rows * cols; ++i) {
            bool k = false;
            for (int t = 0; t < nkeep; ++t) k = k || keep[t] == i;
            if (!k && X[i] != 0.0) return false;
        }
        return true;
    };
    const int keepA[] = {0, 2, 3, 5, 6, 7, 10, 11, 15}, keepB[] = {5, 6}, keepQ[] = {0, 5, 10, 15}, keepR[] = {0, 3};
    const bool bike = zero_outside(M.A, 4, 4, keepA, 9) && M.A[0] == 1.0 && M.A[5] == 1.0 && M.A[10] == 1.0 &&
                      M.A[15] == 1.0 && zero_outside(M.B, 4, 2, keepB, 2) && zero_outside(M.Q, 4, 4, keepQ, 4) &&
                      zero_outside(M.R, 2, 2, keepR, 2);
    D.ric = bike ? 2 : 1;
    D.rseg = rseg;
    D.rone = rone;
    P->ric_slot = slot_of;
    *ok = true;
    return CARMPC_OK;
}

// Kernel choice for one launch (settings.kernel).
hipError_t launch_solve(const DevProblem& D, int64_t batch, const double* x0, const double* xref, double* u_out,
                        int64_t ld_u, int32_t* status, int32_t* iters, const Settings& s, hipStream_t stream,
                        int* unsupported) {
    if (s.kernel == 7 || (s.kernel == 0 && D.ric))
        return launch_riccati(D, batch, x0, xref, u_out, ld_u, status, iters, s, stream, unsupported);
    const bool staged = (s.kernel >= 4 && s.kernel <= 6) || s.kernel == 2 || (s.kernel == 0 && D.staged);
    if (staged) return launch_staged(D, batch, x0, xref, u_out, ld_u, status, iters, s, stream, unsupported);
    return launch_dense(D, batch, x0, xref, u_out, ld_u, status, iters, s, stream, unsupported);
}
}  // namespace

// Riccati layout for per-instance problems: a template problem with the same rows at a generic
// linearisation point (v = 1: every input reaches the psi and v rows at stage 1) gives the slot of
// every QP row; instances whose rows split the same way (layout_ok) run on the Riccati kernel, the
// rest on the dense per-instance kernel.
int carmpc_problem_create(const carmpc_model_desc* d, carmpc_problem** out);
namespace {
int hetero_riccati_template(carmpc_hetero* h, const carmpc_hetero_desc* d) {
    const int N = d->N;
    if (!riccati_supported_N(N)) return CARMPC_OK;
    const double dt = d->dt, v = 1.0;
    double A[16] = {1, 0, 0, dt, 0, 1, dt * v, 0, 0, 0, 1, 0, 0, 0, 0, 1};
    double B[8] = {0, 0, 0, 0, 0, dt * v / d->l1, dt, 0};
    double Pm[16] = {1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1};
    carmpc_model_desc md{};
    md.N = N; md.nx = NX; md.nu = 2; md.A = A; md.B = B; md.Q = d->Q; md.R = d->R; md.P = Pm;
    md.n_state_rows = d->n_state_rows; md.state_A = d->state_A; md.state_b = d->state_b;
    md.n_term_rows = d->n_term_rows; md.term_A = d->term_A; md.term_b = d->term_b;
    md.u_lower = d->u_lower; md.u_upper = d->u_upper; md.goal = d->goal;
    carmpc_problem* T = nullptr;
    g_two_segments_only = true;
    const int rc = carmpc_problem_create(&md, &T);
    g_two_segments_only = false;
    if (rc != CARMPC_OK) return rc;
    h->tmpl = T;
    if (T->dev.ric != 2 || T->ric_slot.size() != T->qp_rows.size()) return CARMPC_OK;   // no bicycle layout
    const int nt = d->n_term_rows, pa = h->p_all;
    constexpr int kSlots = kRicSlots * kRicLanes;
    std::vector<int32_t> slot_of_row(pa, -1);
    std::vector<double> raw((size_t)kSlots * NX, 0.0);
    for (size_t i = 0; i < T->qp_rows.size(); ++i) {
        const int e = T->qp_rows[i], slot = T->ric_slot[i];
        slot_of_row[e] = slot;
        const double* c = e < nt ? d->term_A + (size_t)e * NX : d->state_A + (size_t)((e - nt) / N) * NX;
        for (int a = 0; a < NX; ++a) raw[(size_t)slot * NX + a] = c[a];
    }
    const int64_t B_ = h->batch;
    double* draw = nullptr;
    hipError_t e = hipSuccess;
    auto chk = [&](hipError_t r) { if (e == hipSuccess) e = r; };
    chk(h->upload(&h->tmpl_slot, slot_of_row.data(), slot_of_row.size()));
    chk(h->upload(&draw, raw.data(), raw.size()));
    chk(h->alloc(&h->ric_invn, (size_t)B_ * kSlots));
    chk(h->alloc(&h->ric_w0, (size_t)B_ * kSlots));
    chk(h->alloc(&h->ric_E, (size_t)B_ * kSlots * NX));
    chk(h->alloc(&h->layout_ok, (size_t)B_));
    chk(h->alloc(&h->idx_ok, (size_t)B_));
    chk(h->alloc(&h->idx_bad, (size_t)B_));
    chk(h->alloc(&h->cnt, 2));
    if (e != hipSuccess) return hipfail(e, "hetero Riccati slices");
    DevProblem R = T->dev;   // rows, slots, partners, box, Q, R of the template
    R.r_coef = draw;         // raw row coefficients: the kernel scales them by each instance's 1/||G_r||
    R.r_w0 = nullptr; R.r_E = nullptr;
    R.hq = h->hq; R.pre_w0 = h->pw; R.pre_E = h->pE;
    R.het_p = h->p; R.het_npre = h->npre;
    R.het_sG = h->dev.het_sG; R.het_sH = h->dev.het_sH; R.het_sHq = h->dev.het_sHq; R.het_sRow = h->dev.het_sRow;
    R.het_ric_invn = h->ric_invn; R.het_ric_w0 = h->ric_w0; R.het_ric_E = h->ric_E;
    R.het_A = h->A; R.het_B = h->B; R.het_P = h->P;
    R.Ed = R.pre_Ed = R.s_Ed = R.r_Ed = nullptr;
    h->ric = R;
    return CARMPC_OK;
}
}  // namespace

namespace {
// Device copy of one set of observer constants, keyed by value.  The first use of a value set
// uploads it with a blocking copy (a setup cost, like carmpc_problem_create); every later call
// finds it and returns without touching the device, so the observer entry points only launch.
int stage_observer(const carmpc_problem* P, int32_t ny, const double* C, const double* L, const double* Cd,
                   const double* L2, const double* Bd, const double** dev) {
    if (!P || !C || !L) return fail(CARMPC_EINVAL, "null argument");
    if (!P->assembled) return fail(CARMPC_EINVAL, "observer needs an assembled problem (A, B)");
    if (ny < 1 || ny > 8) return fail(CARMPC_EUNSUPPORTED, "ny must be in [1,8]");
    if ((Cd != nullptr) != (L2 != nullptr) || (Cd != nullptr) != (Bd != nullptr))
        return fail(CARMPC_EINVAL, "Cd, L2 and Bd go together");
    double host[carmpc_problem::kObsStage] = {};
    std::memcpy(host, C, sizeof(double) * ny * NX);
    std::memcpy(host + 8 * NX, L, sizeof(double) * NX * ny);
    if (Cd) {
        std::memcpy(host + 16 * NX, Cd, sizeof(double) * ny);
        std::memcpy(host + 16 * NX + 8, L2, sizeof(double) * ny);
        std::memcpy(host + 16 * NX + 16, Bd, sizeof(double) * NX);
    }
    std::lock_guard<std::mutex> lock(P->obs_mu);
    for (const auto& set : P->obs_sets)
        if (std::memcmp(set->host, host, sizeof(host)) == 0) {
            *dev = set->dev;
            return CARMPC_OK;
        }
    if (P->obs_sets.size() >= 64) return fail(CARMPC_ENOMEM, "more than 64 distinct observer constant sets on one problem");
    int cur = 0;
    HIP_TRY(hipGetDevice(&cur), "hipGetDevice");
    if (cur != P->device) return fail(CARMPC_EINVAL, "the problem belongs to another device than the current one");
    auto set = std::make_unique<carmpc_problem::ObsSet>();
    std::memcpy(set->host, host, sizeof(host));
    HIP_TRY(hipMalloc(reinterpret_cast<void**>(&set->dev), sizeof(host)), "hipMalloc observer constants");
    const hipError_t e = hipMemcpy(set->dev, host, sizeof(host), hipMemcpyHostToDevice);
    if (e != hipSuccess) {
        (void)hipFree(set->dev);
        return hipfail(e, "upload observer constants");
    }
    *dev = set->dev;
    P->obs_sets.push_back(std::move(set));
    return CARMPC_OK;
}
}  // namespace

extern "C" {

const char* carmpc_last_error(void) { return g_err.c_str(); }
const char* carmpc_version(void) { return "carmpc-mi355x 0.6 (gfx950: riccati launch pipeline / staged / dense IPM, closed loop, batched LP, per-instance linearisation, CPU path)"; }

int carmpc_problem_kernel(const carmpc_problem* P) {
    if (!P) return fail(CARMPC_EINVAL, "null problem");
    return P->dev.ric ? 7 : (P->dev.staged ? 2 : 1);
}

// Flops one IPM iteration (predictor + corrector + one refinement) of the given kernel
// actually performs (multiply-add = 2).  Masked/padded lanes not counted.
double carmpc_executed_flops_per_iter(const carmpc_problem* P, int32_t kernel) {
    if (!P) return 0.0;
    const double n = P->dev.n, p = P->dev.p, N = P->dev.N;
    if (kernel == 7 || (kernel == 0 && P->dev.ric)) {
        // grouped Riccati kernel, every stage recursion counted once (the matrix-core passes pad it
        // to full 4x4x4 products, see carmpc_issued_flops_per_iter):
        // per stage factorization + adjoint + 2 backward + 3 forward passes, per row the five
        // row phases (~212 flops), per input the box rows; bicycle sparsity when selected
        const bool bike = P->dev.ric == 2;
        const double fac = bike ? 250.0 : 470.0, adj = bike ? 44.0 : 104.0, back = bike ? 42.0 : 72.0,
                     fwd = bike ? 34.0 : 64.0;
        return N * (fac + adj + 2.0 * back + 3.0 * fwd) + 212.0 * p + 60.0 * n;
    }
    const bool staged = (kernel >= 4 && kernel <= 6) || kernel == 2 || (kernel == 0 && P->dev.staged);
    const double chol = n * n * n / 3.0, trisolve = 2.0 * n * n;
    if (!staged) {
        const double gv = 2.0 * p * n, hv = 2.0 * n * n;
        // M build, Cholesky, residual (Gu, Hu, G'z), 3 x (G't, solve, G dx), refinement H du + G'dZ
        return p * n * n + chol + (gv + hv + gv) + 3.0 * (gv + trisolve + gv) + (hv + gv);
    }
    const double pred = 8.0 * N * (N + 1), adj = 8.0 * N * (N + 1);   // Y = S v ; S' lam
    const double rows = 8.0 * p;                                     // c_r . Y / lam scatter
    const double qy = 32.0 * N;                                      // Qbar_k Y_k
    const double mbuild = 24.0 * p + 640.0 * (N - 1) + 64.0 * N + 32.0 * n * N;
    const double resid = pred + rows + 4.0 * n + rows + qy + 2.0 * adj;
    const double solve = rows + adj + trisolve + pred + rows;
    return mbuild + chol + resid + 3.0 * solve + (qy + 4.0 * n);
}

double carmpc_issued_flops_per_iter(const carmpc_problem* P, int32_t kernel) {
    if (!P) return 0.0;
    if ((kernel == 7 || (kernel == 0 && P->dev.ric))) {
        // v_mfma_f64_4x4x4 per stage: factorization 14, adjoint 2, backward pass 5, forward pass 3
        // (ipm_riccati.hip: factor_mm, adjoint_mm, back_mm, forward_mm), 128 flops per QP each;
        // per iteration one factorization, one adjoint, two backward and three forward passes
        const double n = P->dev.n, p = P->dev.p, N = P->dev.N;
        return N * 128.0 * (14.0 + 2.0 + 2.0 * 5.0 + 3.0 * 3.0) + 212.0 * p + 60.0 * n;
    }
    return carmpc_executed_flops_per_iter(P, kernel);
}

double carmpc_canonical_flops_per_iter(int32_t n, int32_t p) {
    const double N_ = n, P_ = p;
    return P_ * N_ * N_ + N_ * N_ * N_ / 3.0 + 6.0 * N_ * N_ + 12.0 * P_ * N_;
}

int carmpc_problem_create(const carmpc_model_desc* d, carmpc_problem** out) {
    if (!d || !out) return fail(CARMPC_EINVAL, "null argument");
    *out = nullptr;
    if (d->nx != NX) return fail(CARMPC_EUNSUPPORTED, "nx must be 4 (kinematic bicycle state)");
    if (d->nu < 1 || d->nu > 4) return fail(CARMPC_EUNSUPPORTED, "nu must be in [1,4]");
    if (d->N < 1 || d->N > 32) return fail(CARMPC_EUNSUPPORTED, "N must be in [1,32]");
    if (!d->A || !d->B || !d->Q || !d->R || !d->P || !d->goal) return fail(CARMPC_EINVAL, "null model matrix");
    if (d->n_state_rows < 0 || d->n_term_rows < 0) return fail(CARMPC_EINVAL, "negative row count");
    if ((d->n_state_rows && (!d->state_A || !d->state_b)) || (d->n_term_rows && (!d->term_A || !d->term_b)))
        return fail(CARMPC_EINVAL, "null constraint rows");
    if ((d->u_lower == nullptr) != (d->u_upper == nullptr)) return fail(CARMPC_EINVAL, "u_lower/u_upper mismatch");
    const int N = d->N, nu = d->nu, n = N * nu;
    const int nv = dense_pick_nv(n);
    if (nv < 0) return fail(CARMPC_EUNSUPPORTED, "N*nu must be <= 64");
    int dev = 0;
    HIP_TRY(hipGetDevice(&dev), "hipGetDevice");
    auto* P = new carmpc_problem();
    P->device = dev;
    noalloc_prepare_device(dev);   // (resolves the no-allocation entry's scratch address now: that entry may first run under graph capture)
    P->assembled = true;
    const int nt = d->n_term_rows, ns = d->n_state_rows;
    const int p_all = nt + ns * N;
    P->p_all = p_all;
    AsmArgs a{};
    a.N = N; a.nu = nu; a.n = n; a.nt = nt; a.ns = ns;
    double *dA, *dB, *dQ, *dR, *dP, *dtA, *dtb, *dsA, *dsb;
    hipError_t e;
#define UP(dst, src, cnt)                                             \
    if ((e = upload(P, &dst, src, cnt)) != hipSuccess) {              \
        delete P;                                                     \
        return hipfail(e, "upload " #src);                            \
    }
    UP(dA, d->A, NX * NX); UP(dB, d->B, NX * nu); UP(dQ, d->Q, NX * NX); UP(dR, d->R, nu * nu);
    UP(dP, d->P, NX * NX); UP(dtA, d->term_A, (size_t)nt * NX); UP(dtb, d->term_b, nt);
    UP(dsA, d->state_A, (size_t)ns * NX); UP(dsb, d->state_b, ns);
#undef UP
    double *rownorm, *Phi, *coef;
    int32_t* stage;
    if ((e = P->alloc(&P->T, (size_t)(N + 1) * NX * NX)) != hipSuccess ||
        (e = P->alloc(&P->S, (size_t)(N + 1) * NX * n)) != hipSuccess ||
        (e = P->alloc(&P->H, (size_t)n * n)) != hipSuccess || (e = P->alloc(&P->h, (size_t)n * NX)) != hipSuccess ||
        (e = P->alloc(&P->G_all, (size_t)p_all * n)) != hipSuccess ||
        (e = P->alloc(&P->E_all, (size_t)p_all * NX)) != hipSuccess ||
        (e = P->alloc(&P->w0_all, (size_t)p_all)) != hipSuccess || (e = P->alloc(&rownorm, (size_t)p_all)) != hipSuccess ||
        (e = P->alloc(&Phi, (size_t)N * NX * nu)) != hipSuccess || (e = P->alloc(&coef, (size_t)p_all * NX)) != hipSuccess ||
        (e = P->alloc(&stage, (size_t)p_all)) != hipSuccess) {
        delete P;
        return hipfail(e, "hipMalloc (assembly)");
    }
    a.A = dA; a.B = dB; a.Q = dQ; a.R = dR; a.P = dP;
    a.term_A = dtA; a.term_b = dtb; a.state_A = dsA; a.state_b = dsb;
    a.T = P->T; a.S = P->S; a.H = P->H; a.h = P->h; a.G = P->G_all; a.E = P->E_all; a.w0 = P->w0_all;
    a.rownorm = rownorm; a.Phi = Phi; a.row_stage = stage; a.row_coef = coef;
    if ((e = launch_assembly(a, nullptr)) != hipSuccess || (e = hipDeviceSynchronize()) != hipSuccess) {
        delete P;
        return hipfail(e, "assembly kernel");
    }
    std::vector<double> nrm(p_all), Hh((size_t)n * n), hh((size_t)n * NX);
    if ((e = hipMemcpy(nrm.data(), rownorm, sizeof(double) * p_all, hipMemcpyDeviceToHost)) != hipSuccess ||
        (e = hipMemcpy(Hh.data(), P->H, sizeof(double) * n * n, hipMemcpyDeviceToHost)) != hipSuccess ||
        (e = hipMemcpy(hh.data(), P->h, sizeof(double) * n * NX, hipMemcpyDeviceToHost)) != hipSuccess) {
        delete P;
        return hipfail(e, "readback");
    }
    std::vector<int32_t> qp, pre;
    classify(nrm, qp, pre);
    P->qp_rows = qp;
    P->pre_rows = pre;
    P->nrm_all = nrm;
    P->coef_all_dev = coef;
    P->stage_all_dev = stage;
    std::memcpy(P->A_host, d->A, sizeof(double) * NX * NX);
    DevProblem& D = P->dev;
    D.n = n; D.nv = nv; D.p = (int)qp.size(); D.npre = (int)pre.size(); D.ldg = nv + 2; D.N = N; D.nu = nu;
    // (a problem the dense kernel cannot hold in LDS is accepted when a stage-structured layout takes it, below)
    const bool dense_ok = dense_supported(nv, D.p, nullptr);
    int32_t *dqp, *dpre, *stagep;
    double *Gp, *Ep, *w0p, *prew, *preE, *coefp;
    if ((e = upload(P, &dqp, qp.data(), qp.size())) != hipSuccess ||
        (e = upload(P, &dpre, pre.data(), pre.size())) != hipSuccess ||
        (e = P->alloc(&Gp, (size_t)D.p * D.ldg)) != hipSuccess || (e = P->alloc(&Ep, (size_t)D.p * NX)) != hipSuccess ||
        (e = P->alloc(&w0p, (size_t)D.p)) != hipSuccess || (e = P->alloc(&prew, (size_t)D.npre)) != hipSuccess ||
        (e = P->alloc(&preE, (size_t)D.npre * NX)) != hipSuccess || (e = P->alloc(&coefp, (size_t)D.p * NX)) != hipSuccess ||
        (e = P->alloc(&stagep, (size_t)D.p)) != hipSuccess) {
        delete P;
        return hipfail(e, "hipMalloc (pack)");
    }
    PackArgs pk{};
    pk.n = n; pk.nv = nv; pk.ldg = D.ldg; pk.p = D.p; pk.npre = D.npre; pk.p_all = p_all;
    pk.qp_rows = dqp; pk.pre_rows = dpre; pk.G = P->G_all; pk.E = P->E_all; pk.w0 = P->w0_all; pk.rownorm = rownorm;
    pk.row_coef = coef; pk.row_stage = stage; pk.Gp = Gp; pk.Ep = Ep; pk.w0p = w0p; pk.pre_w0 = prew; pk.pre_E = preE;
    pk.coefp = coefp; pk.stagep = stagep;
    if ((D.p + D.npre) > 0 && ((e = launch_pack(pk, nullptr)) != hipSuccess || (e = hipDeviceSynchronize()) != hipSuccess)) {
        delete P;
        return hipfail(e, "pack kernel");
    }
    D.G = Gp; D.E = Ep; D.w0 = w0p; D.pre_w0 = prew; D.pre_E = preE; D.row_coef = coefp; D.row_stage = stagep;
    D.Phi = Phi; D.A = dA; D.B = dB;
    // box: tile u_lower/u_upper over the horizon (mpc.py:217-218)
    std::vector<double> lbv, ubv;
    if (d->u_lower) {
        lbv.resize(n); ubv.resize(n);
        for (int k = 0; k < N; ++k)
            for (int c = 0; c < nu; ++c) { lbv[k * nu + c] = d->u_lower[c]; ubv[k * nu + c] = d->u_upper[c]; }
    }
    int rc = finish_padded(P, Hh.data(), hh.data(), d->u_lower ? lbv.data() : nullptr, d->u_lower ? ubv.data() : nullptr,
                       d->goal);
    bool staged = false;
    std::vector<int32_t> partner;
    if (rc == CARMPC_OK) rc = setup_pairs(P, partner);
    if (rc == CARMPC_OK) rc = stage_layout(P, d, qp, Phi, partner, &staged);
    bool ric = false;
    if (rc == CARMPC_OK) rc = riccati_layout(P, d, partner, &ric);
    if (rc == CARMPC_OK && !dense_ok && !staged && !ric)
        rc = fail(CARMPC_EUNSUPPORTED, "problem too large for the LDS-resident dense kernel (p=" + std::to_string(D.p) +
                                           ", n=" + std::to_string(n) + ") and without a stage-structured layout");
    if (rc != CARMPC_OK) {
        delete P;
        return rc;
    }
    *out = P;
    return CARMPC_OK;
}

int carmpc_problem_create_dense(int32_t n, int32_t p, int32_t nx, const double* H, const double* G, const double* w0,
                                const double* E, const double* hq, const double* lb, const double* ub,
                                const double* goal, carmpc_problem** out) {
    if (!out || !H || !hq || !goal || (p > 0 && (!G || !w0 || !E))) return fail(CARMPC_EINVAL, "null argument");
    *out = nullptr;
    if (nx != NX) return fail(CARMPC_EUNSUPPORTED, "nx must be 4");
    if (n < 1 || p < 0) return fail(CARMPC_EINVAL, "bad sizes");
    if ((lb == nullptr) != (ub == nullptr)) return fail(CARMPC_EINVAL, "lb/ub mismatch");
    const int nv = dense_pick_nv(n);
    if (nv < 0) return fail(CARMPC_EUNSUPPORTED, "n must be <= 64");
    std::vector<double> nrm(p);
    for (int r = 0; r < p; ++r) {
        double s = 0.0;
        for (int j = 0; j < n; ++j) s += G[(size_t)r * n + j] * G[(size_t)r * n + j];
        nrm[r] = std::sqrt(s);
    }
    std::vector<int32_t> qp, pre;
    classify(nrm, qp, pre);
    auto* P = new carmpc_problem();
    HIP_TRY(hipGetDevice(&P->device), "hipGetDevice");
    noalloc_prepare_device(P->device);
    DevProblem& D = P->dev;
    D.n = n; D.nv = nv; D.p = (int)qp.size(); D.npre = (int)pre.size(); D.ldg = nv + 2; D.N = 0; D.nu = 0;
    size_t lds = 0;
    if (!dense_supported(nv, D.p, &lds)) {
        delete P;
        return fail(CARMPC_EUNSUPPORTED, "problem too large for the LDS-resident dense kernel");
    }
    std::vector<double> Gp((size_t)D.p * D.ldg, 0.0), w0p(D.p), Ep((size_t)D.p * NX), prew(D.npre), preE((size_t)D.npre * NX);
    for (int r = 0; r < D.p; ++r) {
        const int s = qp[r];
        for (int j = 0; j < n; ++j) Gp[(size_t)r * D.ldg + j] = G[(size_t)s * n + j] / nrm[s];
        w0p[r] = w0[s] / nrm[s];
        for (int k = 0; k < NX; ++k) Ep[(size_t)r * NX + k] = E[(size_t)s * NX + k] / nrm[s];
    }
    for (int r = 0; r < D.npre; ++r) {
        prew[r] = w0[pre[r]];
        for (int k = 0; k < NX; ++k) preE[(size_t)r * NX + k] = E[(size_t)pre[r] * NX + k];
    }
    double *dG, *dw0, *dE, *dprew, *dpreE;
    hipError_t e;
    if ((e = upload(P, &dG, Gp.data(), Gp.size())) != hipSuccess || (e = upload(P, &dw0, w0p.data(), w0p.size())) != hipSuccess ||
        (e = upload(P, &dE, Ep.data(), Ep.size())) != hipSuccess || (e = upload(P, &dprew, prew.data(), prew.size())) != hipSuccess ||
        (e = upload(P, &dpreE, preE.data(), preE.size())) != hipSuccess) {
        delete P;
        return hipfail(e, "upload dense problem");
    }
    D.G = dG; D.w0 = dw0; D.E = dE; D.pre_w0 = dprew; D.pre_E = dpreE;
    int rc = finish_padded(P, H, hq, lb, ub, goal);
    std::vector<int32_t> partner;
    if (rc == CARMPC_OK) rc = setup_pairs(P, partner);
    if (rc != CARMPC_OK) {
        delete P;
        return rc;
    }
    *out = P;
    return CARMPC_OK;
}

void carmpc_problem_destroy(carmpc_problem* prob) { delete prob; }

int carmpc_problem_info(const carmpc_problem* P, int32_t* n, int32_t* p, int32_t* npre, int32_t* nx, int32_t* N) {
    if (!P) return fail(CARMPC_EINVAL, "null problem");
    if (n) *n = P->dev.n;
    if (p) *p = P->dev.p;
    if (npre) *npre = P->dev.npre;
    if (nx) *nx = NX;
    if (N) *N = P->dev.N;
    return CARMPC_OK;
}

int carmpc_problem_get(const carmpc_problem* P, double* T, double* S, double* H, double* h, double* G, double* E,
                       double* w0, int32_t* p_all) {
    if (!P) return fail(CARMPC_EINVAL, "null problem");
    if (!P->assembled) return fail(CARMPC_EINVAL, "not an assembled problem");
    const int N = P->dev.N, n = P->dev.n, pa = P->p_all;
    if (p_all) *p_all = pa;
    struct Item { void* dst; const void* src; size_t bytes; } items[] = {
        {T, P->T, sizeof(double) * (N + 1) * NX * NX}, {S, P->S, sizeof(double) * (N + 1) * NX * n},
        {H, P->H, sizeof(double) * n * n},             {h, P->h, sizeof(double) * n * NX},
        {G, P->G_all, sizeof(double) * pa * n},        {E, P->E_all, sizeof(double) * pa * NX},
        {w0, P->w0_all, sizeof(double) * pa}};
    for (auto& it : items)
        if (it.dst && it.bytes) HIP_TRY(hipMemcpy(it.dst, it.src, it.bytes, hipMemcpyDeviceToHost), "problem_get");
    return CARMPC_OK;
}

int carmpc_solve_batch(const carmpc_problem* P, int64_t batch, const double* x0, const double* xref, double* u_out,
                       int32_t* status, int32_t* iters, const carmpc_settings* settings, hipStream_t stream) {
    return solve_batch_with_claim(P, batch, x0, xref, u_out, status, iters, settings, nullptr, stream);
}

int carmpc_solve_segments(const carmpc_problem* const* probs, int32_t nprobs, const int64_t* offsets,
                          const double* x0, const double* xref, double* u_out, int64_t ld_u, int32_t* status,
                          int32_t* iters, const carmpc_settings* settings, hipStream_t stream) {
    if (!probs || !offsets || nprobs < 0) return fail(CARMPC_EINVAL, "null argument");
    const Settings s = make_settings(settings);
    std::vector<int> live;
    for (int j = 0; j < nprobs; ++j) {
        const int64_t b0 = offsets[j], b1 = offsets[j + 1];
        if (b0 < 0 || b1 < b0) return fail(CARMPC_EINVAL, "offsets must be non-negative and non-decreasing");
        // (32-bit claim counters and int32 rows in the work lists, as in carmpc_solve_batch)
        if (b1 - offsets[0] > INT32_MAX) return fail(CARMPC_EUNSUPPORTED, "segments exceed 2^31 - 1 instances");
        if (b1 == b0) continue;
        if (!probs[j]) return fail(CARMPC_EINVAL, "null problem in segment list");
        if (ld_u < probs[j]->dev.n) return fail(CARMPC_EINVAL, "ld_u smaller than n");
        live.push_back(j);
    }
    if (live.empty()) return CARMPC_OK;
    if (!x0 || !u_out || !status) return fail(CARMPC_EINVAL, "null batch pointer");
    // Runs of consecutive segments that share one instantiation of the grouped Riccati kernel go out
    // as ONE launch sequence (ipm_riccati.hip: workgroups move from a drained segment to the others),
    // so no segment ends with its own launch tail; anything else is launched per problem.  All
    // launches are queued on `stream`; counters and work lists are stream-ordered allocations of
    // the launch helpers.
    auto ric_ok = [&](int j) { return (s.kernel == 0 || s.kernel == 7) && probs[j]->dev.ric != 0; };
    int rc = CARMPC_OK;
    for (size_t i = 0; i < live.size() && rc == CARMPC_OK;) {
        size_t i1 = i + 1;
        if (ric_ok(live[i]))
            while (i1 < live.size() && i1 - i < (size_t)kRicMaxSeg && live[i1] == live[i1 - 1] + 1 && ric_ok(live[i1]) &&
                   probs[live[i1]]->dev.N == probs[live[i]]->dev.N && probs[live[i1]]->dev.ric == probs[live[i]]->dev.ric &&
                   probs[live[i1]]->dev.rone == probs[live[i]]->dev.rone)
                ++i1;
        int unsupported = 0;
        hipError_t e = hipSuccess;
        if (i1 - i >= 2) {
            RicSegs T{};
            T.nseg = (int)(i1 - i);
            for (size_t k = i; k < i1; ++k) {
                T.off[k - i] = offsets[live[k]];
                T.P[k - i] = probs[live[k]]->dev;
            }
            T.off[i1 - i] = offsets[live[i1 - 1] + 1];
            e = launch_riccati_segs(T, x0, xref, u_out, ld_u, status, iters, s, stream, &unsupported);
        } else {
            const int j = live[i];
            const int64_t b0 = offsets[j], b1 = offsets[j + 1];
            e = launch_solve(probs[j]->dev, b1 - b0, x0 + b0 * NX, xref ? xref + b0 * NX : nullptr, u_out + b0 * ld_u, ld_u,
                             status + b0, iters ? iters + b0 : nullptr, s, stream, &unsupported);
        }
        if (unsupported) rc = fail(CARMPC_EUNSUPPORTED, "no compiled kernel for this problem size");
        else if (e != hipSuccess) rc = hipfail(e, "segment launch");
        i = i1;
    }
    return rc;
}

int carmpc_problem_set_disturbance(carmpc_problem* P, const double* Bd) {
    if (!P || !Bd) return fail(CARMPC_EINVAL, "null argument");
    if (!P->assembled || P->dev.nu < 1) return fail(CARMPC_EUNSUPPORTED, "disturbance offsets need an assembled problem");
    DevProblem& D = P->dev;
    const int N = D.N, pa = P->p_all;
    // ABd_k = sum_{m<k} A^m Bd  (mpc.py:631-635)
    std::vector<double> abd((size_t)(N + 1) * NX, 0.0);
    double Am[16], acc[NX] = {0, 0, 0, 0};
    for (int i = 0; i < 16; ++i) Am[i] = (i % 5 == 0) ? 1.0 : 0.0;
    for (int k = 1; k <= N; ++k) {
        for (int a = 0; a < NX; ++a)
            for (int b = 0; b < NX; ++b) acc[a] += Am[a * NX + b] * Bd[b];
        for (int a = 0; a < NX; ++a) abd[(size_t)k * NX + a] = acc[a];
        double nx_[16];
        for (int a = 0; a < NX; ++a)
            for (int b = 0; b < NX; ++b) {
                double v = 0.0;
                for (int c = 0; c < NX; ++c) v += P->A_host[a * NX + c] * Am[c * NX + b];
                nx_[a * NX + b] = v;
            }
        std::memcpy(Am, nx_, sizeof(Am));
    }
    std::vector<double> coef((size_t)pa * NX);
    std::vector<int32_t> stage(pa);
    if (pa > 0) {
        HIP_TRY(hipMemcpy(coef.data(), P->coef_all_dev, sizeof(double) * coef.size(), hipMemcpyDeviceToHost), "readback coef");
        HIP_TRY(hipMemcpy(stage.data(), P->stage_all_dev, sizeof(int32_t) * pa, hipMemcpyDeviceToHost), "readback stage");
    }
    std::vector<double> ed_all(pa, 0.0);
    for (int r = 0; r < pa; ++r)
        for (int a = 0; a < NX; ++a) ed_all[r] += coef[(size_t)r * NX + a] * abd[(size_t)stage[r] * NX + a];
    std::vector<double> ed(D.p), pre_ed(D.npre);
    for (int i = 0; i < D.p; ++i) ed[i] = ed_all[P->qp_rows[i]] / P->nrm_all[P->qp_rows[i]];   // packed rows are normalised
    for (int i = 0; i < D.npre; ++i) pre_ed[i] = ed_all[P->pre_rows[i]];
    double *ded, *dpre;
    HIP_TRY(upload(P, &ded, ed.data(), ed.size()), "upload Ed");
    HIP_TRY(upload(P, &dpre, pre_ed.data(), pre_ed.size()), "upload pre_Ed");
    D.Ed = ded;
    D.pre_Ed = dpre;
    if (!P->stage_slot.empty()) {
        std::vector<double> sed((size_t)D.srs * 64, 0.0);
        for (int i = 0; i < D.p; ++i) sed[P->stage_slot[i]] = ed[i];
        double* dsed;
        HIP_TRY(upload(P, &dsed, sed.data(), sed.size()), "upload s_Ed");
        D.s_Ed = dsed;
    }
    if (!P->ric_slot.empty()) {
        std::vector<double> red((size_t)kRicSlots * kRicLanes, 0.0);
        for (int i = 0; i < D.p; ++i) red[P->ric_slot[i]] = ed[i];
        double* dred;
        HIP_TRY(upload(P, &dred, red.data(), red.size()), "upload r_Ed");
        D.r_Ed = dred;
    }
    return CARMPC_OK;
}

int carmpc_solve_batch_dist(const carmpc_problem* P, int64_t batch, const double* x0, const double* xref,
                            const double* dist, double* u_out, int32_t* status, int32_t* iters,
                            const carmpc_settings* settings, hipStream_t stream) {
    if (!P) return fail(CARMPC_EINVAL, "null problem");
    if (batch < 0) return fail(CARMPC_EINVAL, "negative batch");
    if (batch == 0) return CARMPC_OK;
    if (!x0 || !u_out || !status || !dist) return fail(CARMPC_EINVAL, "null batch pointer");
    if (!P->dev.Ed) return fail(CARMPC_EINVAL, "no disturbance model: call carmpc_problem_set_disturbance first");
    Settings s = make_settings(settings);
    s.dist = dist;
    int unsupported = 0;
    hipError_t e = launch_solve(P->dev, batch, x0, xref, u_out, P->dev.n, status, iters, s, stream, &unsupported);
    if (unsupported) return fail(CARMPC_EUNSUPPORTED, "no compiled kernel for this problem size");
    if (e != hipSuccess) return hipfail(e, "solve launch");
    return CARMPC_OK;
}

int carmpc_hetero_create(const carmpc_hetero_desc* d, int64_t batch, carmpc_hetero** out) {
    if (!d || !out) return fail(CARMPC_EINVAL, "null argument");
    *out = nullptr;
    if (batch < 1) return fail(CARMPC_EINVAL, "batch must be >= 1");
    if (d->N < 1 || d->N > 32) return fail(CARMPC_EUNSUPPORTED, "N must be in [1,32]");
    if (!d->Q || !d->R || !d->goal) return fail(CARMPC_EINVAL, "null model matrix");
    if (!(d->dt > 0.0) || !(d->l1 > 0.0)) return fail(CARMPC_EINVAL, "dt and l1 must be positive");
    if (d->n_state_rows < 0 || d->n_term_rows < 0) return fail(CARMPC_EINVAL, "negative row count");
    if ((d->n_state_rows && (!d->state_A || !d->state_b)) || (d->n_term_rows && (!d->term_A || !d->term_b)))
        return fail(CARMPC_EINVAL, "null constraint rows");
    if ((d->u_lower == nullptr) != (d->u_upper == nullptr)) return fail(CARMPC_EINVAL, "u_lower/u_upper mismatch");
    const int N = d->N, n = 2 * N;
    const int nv = dense_pick_nv(n);
    const int p_all = d->n_term_rows + d->n_state_rows * N;
    if (nv < 0) return fail(CARMPC_EUNSUPPORTED, "2N must be <= 64");
    if (p_all > 256 || p_all > kHetMaxRows)
        return fail(CARMPC_EUNSUPPORTED, "per-instance problems are limited to 256 general rows (p_all=" +
                                             std::to_string(p_all) + ")");
    int dev = 0;
    HIP_TRY(hipGetDevice(&dev), "hipGetDevice");
    auto* h = new carmpc_hetero();
    h->device = dev;
    h->batch = batch; h->p_all = p_all; h->nt = d->n_term_rows; h->ns = d->n_state_rows; h->dt = d->dt; h->l1 = d->l1;
    DevProblem& D = h->dev;
    D.n = n; D.nv = nv; D.ldg = nv + 2; D.N = N; D.nu = 2; D.p = p_all;
    std::vector<double> lbp(nv, -1.0), ubp(nv, 1.0);
    if (d->u_lower)
        for (int k = 0; k < N; ++k)
            for (int c = 0; c < 2; ++c) { lbp[k * 2 + c] = d->u_lower[c]; ubp[k * 2 + c] = d->u_upper[c]; }
    D.boxed = d->u_lower ? 1 : 0;
    const int64_t sG = (int64_t)std::max(p_all, 1) * D.ldg, sH = (int64_t)nv * nv, sHq = (int64_t)nv * NX,
                  sRow = std::max(p_all, 1);
    double *dlb, *dub, *dgoal;
    hipError_t e = hipSuccess;
    auto chk = [&](hipError_t r) { if (e == hipSuccess) e = r; };
    chk(h->upload(&dlb, lbp.data(), lbp.size()));
    chk(h->upload(&dub, ubp.data(), ubp.size()));
    chk(h->upload(&dgoal, d->goal, NX));
    chk(h->upload(&h->Q, d->Q, 16));
    chk(h->upload(&h->R, d->R, 4));
    chk(h->upload(&h->tA, d->term_A, (size_t)h->nt * NX));
    chk(h->upload(&h->tb, d->term_b, (size_t)h->nt));
    chk(h->upload(&h->sA, d->state_A, (size_t)h->ns * NX));
    chk(h->upload(&h->sb, d->state_b, (size_t)h->ns));
    chk(h->alloc(&h->A, (size_t)batch * 16)); chk(h->alloc(&h->B, (size_t)batch * 8));
    chk(h->alloc(&h->P, (size_t)batch * 16)); chk(h->alloc(&h->K, (size_t)batch * 8));
    chk(h->alloc(&h->lin_status, (size_t)batch));
    chk(h->alloc(&h->G, (size_t)batch * sG)); chk(h->alloc(&h->H, (size_t)batch * sH));
    chk(h->alloc(&h->hq, (size_t)batch * sHq)); chk(h->alloc(&h->w0, (size_t)batch * sRow));
    chk(h->alloc(&h->E, (size_t)batch * sRow * NX)); chk(h->alloc(&h->pw, (size_t)batch * sRow));
    chk(h->alloc(&h->pE, (size_t)batch * sRow * NX)); chk(h->alloc(&h->partner, (size_t)batch * sRow));
    chk(h->alloc(&h->p, (size_t)batch)); chk(h->alloc(&h->npre, (size_t)batch));
    if (e != hipSuccess) {
        delete h;
        return hipfail(e, "hetero allocation (per-instance problem slices)");
    }
    D.lb = dlb; D.ub = dub; D.goal = dgoal;
    D.G = h->G; D.H = h->H; D.hq = h->hq; D.w0 = h->w0; D.E = h->E; D.pre_w0 = h->pw; D.pre_E = h->pE;
    D.partner = h->partner; D.het_p = h->p; D.het_npre = h->npre;
    D.het_sG = sG; D.het_sH = sH; D.het_sHq = sHq; D.het_sRow = sRow;
    const int rc = hetero_riccati_template(h, d);
    if (rc != CARMPC_OK) {
        delete h;
        return rc;
    }
    *out = h;
    return CARMPC_OK;
}

void carmpc_hetero_destroy(carmpc_hetero* h) { delete h; }

int carmpc_hetero_linearize(carmpc_hetero* h, const double* lin_state, const double* lin_input, hipStream_t stream) {
    if (!h || !lin_state || !lin_input) return fail(CARMPC_EINVAL, "null argument");
    LinArgs l{};
    l.batch = h->batch; l.dt = h->dt; l.l1 = h->l1; l.lin_state = lin_state; l.lin_input = lin_input;
    l.Q = h->Q; l.R = h->R; l.A = h->A; l.B = h->B; l.P = h->P; l.K = h->K; l.status = h->lin_status;
    HIP_TRY(launch_linearize(l, stream), "linearize launch");
    HetAsmArgs a{};
    a.batch = h->batch; a.N = h->dev.N; a.nv = h->dev.nv; a.ldg = h->dev.ldg; a.nt = h->nt; a.ns = h->ns;
    a.A = h->A; a.B = h->B; a.P = h->P; a.Q = h->Q; a.R = h->R;
    a.term_A = h->tA; a.term_b = h->tb; a.state_A = h->sA; a.state_b = h->sb;
    a.G = h->G; a.H = h->H; a.hq = h->hq; a.w0 = h->w0; a.E = h->E; a.pre_w0 = h->pw; a.pre_E = h->pE;
    a.partner = h->partner; a.p = h->p; a.npre = h->npre;
    a.strideG = h->dev.het_sG; a.strideH = h->dev.het_sH; a.strideHq = h->dev.het_sHq; a.strideRow = h->dev.het_sRow;
    a.tmpl_slot = h->tmpl_slot;
    a.ric_invn = h->ric_invn; a.ric_w0 = h->ric_w0; a.ric_E = h->ric_E; a.layout_ok = h->layout_ok;
    HIP_TRY(launch_hetero_assembly(a, stream), "hetero assembly launch");
    if (h->tmpl_slot)
        HIP_TRY(launch_het_split(h->batch, h->layout_ok, h->idx_ok, h->cnt, h->idx_bad, h->cnt + 1, stream),
                "hetero split");
    h->ready = true;
    return CARMPC_OK;
}

int carmpc_hetero_solve(const carmpc_hetero* h, const double* x0, const double* xref, double* u_out, int32_t* status,
                        int32_t* iters, const carmpc_settings* settings, hipStream_t stream) {
    if (!h) return fail(CARMPC_EINVAL, "null handle");
    if (!h->ready) return fail(CARMPC_EINVAL, "call carmpc_hetero_linearize first");
    if (!x0 || !u_out || !status) return fail(CARMPC_EINVAL, "null batch pointer");
    const Settings s = make_settings(settings);
    int unsupported = 0;
    hipError_t e = hipSuccess;
    if (h->tmpl_slot && (s.kernel == 0 || s.kernel == 7)) {
        // Riccati kernel on the instances with the template's row layout, dense kernel on the rest
        // (e.g. v = 0 linearisations, where the steering input leaves the psi rows at stage 1)
        Settings so = s, sb = s;
        so.index = h->idx_ok; so.count = h->cnt;
        sb.index = h->idx_bad; sb.count = h->cnt + 1;
        e = launch_riccati(h->ric, h->batch, x0, xref, u_out, h->dev.n, status, iters, so, stream, &unsupported, true);
        if (e == hipSuccess && !unsupported)
            e = launch_dense_het(h->dev, h->p_all, h->batch, x0, xref, u_out, h->dev.n, status, iters, sb, stream,
                                 &unsupported);
    } else {
        e = launch_dense_het(h->dev, h->p_all, h->batch, x0, xref, u_out, h->dev.n, status, iters, s, stream,
                             &unsupported);
    }
    if (unsupported) return fail(CARMPC_EUNSUPPORTED, "no compiled kernel for this problem size");
    if (e != hipSuccess) return hipfail(e, "hetero solve launch");
    return CARMPC_OK;
}

int carmpc_hetero_get(const carmpc_hetero* h, double* A, double* B, double* P, double* K, int32_t* dare_status,
                      int32_t* p, int32_t* npre, double* G, double* H, double* hq, double* w0, double* E,
                      int64_t* dims) {
    if (!h) return fail(CARMPC_EINVAL, "null handle");
    const size_t b = (size_t)h->batch;
    const DevProblem& D = h->dev;
    if (dims) {
        dims[0] = D.het_sRow; dims[1] = D.ldg; dims[2] = D.nv; dims[3] = D.n; dims[4] = h->p_all; dims[5] = h->batch;
    }
    if (!h->ready && (A || B || P || K || dare_status || p || npre || G || H || hq || w0 || E))
        return fail(CARMPC_EINVAL, "call carmpc_hetero_linearize first");
    struct Item { void* dst; const void* src; size_t bytes; } items[] = {
        {A, h->A, sizeof(double) * b * 16},          {B, h->B, sizeof(double) * b * 8},
        {P, h->P, sizeof(double) * b * 16},          {K, h->K, sizeof(double) * b * 8},
        {dare_status, h->lin_status, sizeof(int32_t) * b},
        {p, h->p, sizeof(int32_t) * b},              {npre, h->npre, sizeof(int32_t) * b},
        {G, h->G, sizeof(double) * b * D.het_sG},    {H, h->H, sizeof(double) * b * D.het_sH},
        {hq, h->hq, sizeof(double) * b * D.het_sHq}, {w0, h->w0, sizeof(double) * b * D.het_sRow},
        {E, h->E, sizeof(double) * b * D.het_sRow * NX}};
    HIP_TRY(hipDeviceSynchronize(), "hetero_get sync");
    for (auto& it : items)
        if (it.dst) HIP_TRY(hipMemcpy(it.dst, it.src, it.bytes, hipMemcpyDeviceToHost), "hetero_get");
    return CARMPC_OK;
}

int carmpc_lp_batch(int64_t nlp, int32_t max_m, const int64_t* a_off, const int64_t* b_off, const int32_t* m,
                    const double* a_pool, const double* b_pool, const double* c, const int32_t* relax,
                    double relax_amount, double* value, double* x, int32_t* status, int32_t* iters,
                    hipStream_t stream) {
    if (nlp < 0) return fail(CARMPC_EINVAL, "negative LP count");
    if (nlp == 0) return CARMPC_OK;
    if (!a_off || !b_off || !m || !a_pool || !b_pool || !c || !value || !status)
        return fail(CARMPC_EINVAL, "null LP pointer");
    if (max_m < 0 || max_m > 1016) return fail(CARMPC_EUNSUPPORTED, "LPs with more than 1016 rows");
    LpArgs a{};
    a.nlp = nlp; a.a_off = a_off; a.b_off = b_off; a.m = m; a.a_pool = a_pool; a.b_pool = b_pool; a.c = c;
    a.relax = relax; a.relax_amount = relax_amount; a.tol = 1e-10; a.tol_gap = 1e-10; a.max_iter = 200;
    a.value = value; a.x = x; a.status = status; a.iters = iters;
    HIP_TRY(launch_lp(a, max_m, stream), "LP launch");
    return CARMPC_OK;
}

int carmpc_closed_loop_batch(const carmpc_problem* P, int64_t batch, const carmpc_loop_desc* L, double* state,
                             double* xhat, double* dhat, const double* xref, double* u, int32_t* outcome,
                             int32_t* steps, int32_t check_every, const carmpc_settings* settings,
                             hipStream_t stream) {
    if (!P || !L) return fail(CARMPC_EINVAL, "null argument");
    if (batch < 0 || batch > INT32_MAX) return fail(CARMPC_EINVAL, "batch out of range");
    if (batch == 0) return CARMPC_OK;
    if (!state || !u || !outcome || !steps) return fail(CARMPC_EINVAL, "null batch pointer");
    if (!P->assembled || P->dev.nu != 2) return fail(CARMPC_EUNSUPPORTED, "closed loop needs an assembled problem with nu = 2");
    if (L->mode < 0 || L->mode > 2) return fail(CARMPC_EINVAL, "mode must be 0, 1 or 2");
    if (L->steps_update < 1 || L->last_step < 0 || !(L->dt > 0.0) || !(L->l1 > 0.0))
        return fail(CARMPC_EINVAL, "steps_update >= 1, last_step >= 0, dt > 0, l1 > 0 required");
    if (L->mode >= 1) {
        if (!xhat || !L->C || !L->L) return fail(CARMPC_EINVAL, "output feedback needs xhat, C and L");
        if (L->ny < 1 || L->ny > 8) return fail(CARMPC_EUNSUPPORTED, "ny must be in [1,8]");
    }
    if (L->mode == 2) {
        if (!dhat || !L->Cd || !L->L2 || !L->Bd) return fail(CARMPC_EINVAL, "disturbance mode needs dhat, Cd, L2, Bd");
        if (!P->dev.Ed) return fail(CARMPC_EINVAL, "no disturbance model: call carmpc_problem_set_disturbance first");
    }
    const int64_t n = P->dev.n;
    // loop constants: C 8*NX | L NX*8 | Cd 8 | L2 8 | Bd NX | goal NX
    constexpr int kC = 0, kL = 8 * NX, kCd = 16 * NX, kL2 = 16 * NX + 8, kBd = 16 * NX + 16, kGoal = 17 * NX + 16,
                  kConst = 18 * NX + 16;
    std::vector<double> host(kConst, 0.0);
    const int ny = L->mode >= 1 ? L->ny : 0;
    if (ny) {
        std::memcpy(host.data() + kC, L->C, sizeof(double) * ny * NX);
        std::memcpy(host.data() + kL, L->L, sizeof(double) * NX * ny);
    }
    if (L->mode == 2) {
        std::memcpy(host.data() + kCd, L->Cd, sizeof(double) * ny);
        std::memcpy(host.data() + kL2, L->L2, sizeof(double) * ny);
        std::memcpy(host.data() + kBd, L->Bd, sizeof(double) * NX);
    }
    HIP_TRY(hipMemcpy(host.data() + kGoal, P->dev.goal, sizeof(double) * NX, hipMemcpyDeviceToHost), "read goal");
    if (L->goal) std::memcpy(host.data() + kGoal, L->goal, sizeof(double) * NX);
    // workspace: constants, QP status, two slot lists and their counts (stream-ordered)
    const size_t bytes = sizeof(double) * kConst + sizeof(int32_t) * (3 * (size_t)batch + 2);
    void* ws = nullptr;
    HIP_TRY(hipMallocAsync(&ws, bytes, stream), "hipMallocAsync loop workspace");
    double* dconst = static_cast<double*>(ws);
    int32_t* ibase = reinterpret_cast<int32_t*>(dconst + kConst);
    hipError_t e = hipMemcpyAsync(dconst, host.data(), sizeof(double) * kConst, hipMemcpyHostToDevice, stream);
    if (e == hipSuccess) e = hipStreamSynchronize(stream);   // host staging buffer goes out of scope
    LoopArgs a{};
    a.batch = batch; a.mode = L->mode; a.ny = ny; a.steps_update = L->steps_update; a.last_step = L->last_step;
    a.ld_u = n; a.dt = L->dt; a.l1 = L->l1; a.goal_tol = L->goal_tol;
    a.A = P->dev.A; a.B = P->dev.B;
    a.C = dconst + kC; a.L = dconst + kL; a.Cd = dconst + kCd; a.L2 = dconst + kL2; a.Bd = dconst + kBd;
    a.goal = dconst + kGoal;
    a.state = state; a.xhat = xhat; a.dhat = dhat; a.u = u;
    int32_t* qp_status = ibase;
    a.qp_status = qp_status;
    a.outcome = outcome; a.steps = steps;
    a.idx_cur = ibase + batch; a.idx_next = ibase + 2 * batch;
    a.cnt_cur = ibase + 3 * batch; a.cnt_next = ibase + 3 * batch + 1;
    if (e == hipSuccess) e = launch_loop_init(a, stream);
    Settings s = make_settings(settings);
    if (L->mode == 2) s.dist = dhat;
    const double* x_qp = L->mode == 0 ? state : xhat;
    int unsupported = 0;
    for (int32_t i = 0; i <= L->last_step && e == hipSuccess; ++i) {
        e = launch_loop_advance(a, i, stream);
        if (e == hipSuccess && i % L->steps_update == 0) {
            s.index = a.idx_cur;
            s.count = a.cnt_cur;
            e = launch_solve(P->dev, batch, x_qp, xref, u, n, qp_status, nullptr, s, stream, &unsupported);
        }
        if (e == hipSuccess) e = launch_loop_finish(a, i, stream);
        std::swap(a.idx_cur, a.idx_next);
        std::swap(a.cnt_cur, a.cnt_next);
        if (e == hipSuccess && check_every > 0 && (i + 1) % check_every == 0 && i < L->last_step) {
            int32_t left = 0;
            e = hipMemcpyAsync(&left, a.cnt_cur, sizeof(int32_t), hipMemcpyDeviceToHost, stream);
            if (e == hipSuccess) e = hipStreamSynchronize(stream);
            if (e == hipSuccess && left == 0) break;
        }
    }
    const hipError_t ef = hipFreeAsync(ws, stream);
    if (unsupported) return fail(CARMPC_EUNSUPPORTED, "no compiled kernel for this problem size");
    if (e != hipSuccess) return hipfail(e, "closed loop");
    if (ef != hipSuccess) return hipfail(ef, "hipFreeAsync loop workspace");
    return CARMPC_OK;
}

int carmpc_problem_set_observer(const carmpc_problem* P, int32_t ny, const double* C, const double* L,
                                const double* Cd, const double* L2, const double* Bd) {
    const double* dev = nullptr;
    return stage_observer(P, ny, C, L, Cd, L2, Bd, &dev);
}

int carmpc_observer_dist_batch(const carmpc_problem* P, int64_t batch, const double* y, int32_t ny, const double* C,
                               const double* L1, const double* Cd, const double* L2, const double* Bd, double* xhat,
                               double* dhat, const double* uprev, int64_t ld_uprev, hipStream_t stream) {
    if (!P || !y || !C || !L1 || !Cd || !L2 || !Bd || !xhat || !dhat || !uprev) return fail(CARMPC_EINVAL, "null argument");
    const double* dCL = nullptr;
    const int rc = stage_observer(P, ny, C, L1, Cd, L2, Bd, &dCL);
    if (rc != CARMPC_OK) return rc;
    ObsArgs a{};
    a.batch = batch; a.ny = ny; a.nu = P->dev.nu; a.ld_uprev = ld_uprev;
    a.A = P->dev.A; a.B = P->dev.B; a.C = dCL; a.L = dCL + 8 * NX; a.y = y; a.uprev = uprev; a.xhat = xhat;
    a.Cd = dCL + 16 * NX; a.L2 = dCL + 16 * NX + 8; a.Bd = dCL + 16 * NX + 16; a.dhat = dhat;
    HIP_TRY(launch_observer(a, stream), "observer launch");
    return CARMPC_OK;
}

int carmpc_observer_batch(const carmpc_problem* P, int64_t batch, const double* y, int32_t ny, const double* C,
                          const double* L, double* xhat, const double* uprev, int64_t ld_uprev, hipStream_t stream) {
    if (!P || !y || !C || !L || !xhat || !uprev) return fail(CARMPC_EINVAL, "null argument");
    const double* dCL = nullptr;
    const int rc = stage_observer(P, ny, C, L, nullptr, nullptr, nullptr, &dCL);
    if (rc != CARMPC_OK) return rc;
    ObsArgs a{};
    a.batch = batch; a.ny = ny; a.nu = P->dev.nu; a.ld_uprev = ld_uprev;
    a.A = P->dev.A; a.B = P->dev.B; a.C = dCL; a.L = dCL + 8 * NX; a.y = y; a.uprev = uprev; a.xhat = xhat;
    HIP_TRY(launch_observer(a, stream), "observer launch");
    return CARMPC_OK;
}

int carmpc_plant_step_batch(int64_t batch, double* state, const double* u, int64_t ld_u, double dt, double l1,
                            int32_t* bad, hipStream_t stream) {
    if (batch < 0 || (batch > 0 && (!state || !u))) return fail(CARMPC_EINVAL, "bad argument");
    HIP_TRY(launch_plant(batch, state, u, ld_u, dt, l1, bad, stream), "plant launch");
    return CARMPC_OK;
}

}  // extern "C"

// carmpc_solve_batch with the claim counter supplied by the caller (already zeroed, stream-ordered
// before the launch); claim == nullptr: a stream-ordered allocation per launch.
namespace carmpc {
int solve_batch_with_claim(const carmpc_problem* P, int64_t batch, const double* x0, const double* xref, double* u_out,
                           int32_t* status, int32_t* iters, const carmpc_settings* settings, unsigned* claim,
                           hipStream_t stream) {
    if (!P) return fail(CARMPC_EINVAL, "null problem");
    if (batch < 0) return fail(CARMPC_EINVAL, "negative batch");
    if (batch == 0) return CARMPC_OK;
    // the kernels count instances in 32-bit claim counters and keep rows as int32 in their work lists
    if (batch > INT32_MAX) return fail(CARMPC_EUNSUPPORTED, "batch exceeds 2^31 - 1 instances");
    if (!x0 || !u_out || !status) return fail(CARMPC_EINVAL, "null batch pointer");
    Settings s = make_settings(settings);
    s.claim = claim;
    int unsupported = 0;
    hipError_t e = launch_solve(P->dev, batch, x0, xref, u_out, P->dev.n, status, iters, s, stream, &unsupported);
    if (unsupported) return fail(CARMPC_EUNSUPPORTED, "no compiled kernel for this problem size");
    if (e != hipSuccess) return hipfail(e, "solve launch");
    return CARMPC_OK;
}
int problem_device(const carmpc_problem* P) { return P ? P->device : -1; }
int set_error(int code, const char* msg) { return fail(code, msg); }
}  // namespace carmpc
