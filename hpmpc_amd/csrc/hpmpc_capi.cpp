// hpmpc_capi.cpp -- host side of libhpmpc_mi355x.so: the reference-named C ABI (drop-in for
// HPMPC's lqcp_solvers.h / mpc_solvers.h hot path) and the batched device API.  Every call runs on
// the GPU through the kernels in hpmpc_kernels.hip; there is no CPU fallback.
//
// Host marshalling of the single-problem entry points:
//   * the caller's per-stage lib4 blocks (pointers may alias across stages) are copied stage by stage
//     into a pinned staging arena, uploaded with one hipMemcpyAsync and solved by a 1-problem launch;
//   * the reference's documented in-place side effects on hpRSQrq / hpBAbt (update_q / update_b
//     rows, box diagonal and gradient, d_back_ric_rec.c:197-209, :249-291) are applied to the caller's
//     buffers in the reference's stage order, and each stage's device copy receives exactly the
//     values the reference factorises for that stage;
//   * "memory" / "double_work_memory" hold this library's private device image (factor + persistent
//     IPM iterate) so that trs and d_kkt_solve_new_rhs_res_mpc_hard_tv can re-use it.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <mutex>
#include <vector>

#include "hpmpc_api.h"
#include "hpmpc_kargs.h"
#include "hk_wide_args.h"

extern "C" int hk_launch(int which, const KArgs* a, int count, hipStream_t stream);
#ifdef HK_RIC2  // the two-wave sv (hk_ric2.hip), a measured negative result: only in the ric2 build variant
extern "C" int hk_launch_ric2(int which, const KArgs* a, int count, hipStream_t stream);
#endif
extern "C" int hk_fixcls(int nu, int nx);
// wide-stage path (hpmpc_capi_wide.cpp, hpmpc_capi_wide_ipm.cpp)
extern "C" long long hk_wide_ipm_bytes(int N, const int* nx, const int* nu, const int* nb, const int* ng);
extern "C" int hk_wide_ipm_entry(int mode, int* kk, int k_max, double mu0, double mu_tol, double alpha_min,
                                 int warm_start, double* stat, int N, int* nx, int* nu_N, int* nb, int** idxb, int* ng,
                                 double** pBAbt, double** pQ, double** pDCt, double** d, double** ux,
                                 int compute_mult, double** pi, double** lam, double** t, double* work, double** ux0,
                                 double** pi0, double** lam0, double** t0);
extern "C" void hk_wide_kkt_entry(int p1, int N, int* nx, int* nu_N, int* nb, int** idxb, int* ng, double** pBAbt,
                                  double** b, double** pQ, double** q, double** pDCt, double** d, double** ux,
                                  int compute_mult, double** pi, double** lam, double** t, double* work);
extern "C" void hk_wide_res_entry(int plain, int N, int* nx, int* nu, int* nb, int** idxb, int* ng, double** hpBAbt,
                                  double** hb, double** hpQ, double** hq, double** hux, double** hpDCt, double** hd,
                                  double** hpi, double** hlam, double** ht, double** hrq, double** hrb, double** hrd,
                                  double** hrm, double* mu);
extern "C" long long hk_wide_factor_bytes(int N, const int* nx, const int* nu);
extern "C" void hk_wide_sv_entry(int N, int* nx, int* nu, int* nb, int** idxb, int* ng, int update_b, double** hpBAbt,
                                 double** b, int update_q, double** hpQ, double** q, double** bd, double** hpDCt,
                                 double** Qx, double** qx, double** hux, int compute_pi, double** hpi, int compute_Pb,
                                 double** hPb, double* memory);
extern "C" void hk_wide_trf_entry(int N, int* nx, int* nu, int* nb, int** idxb, int* ng, double** hpBAbt,
                                  double** hpQ, double** hpDCt, double** Qx, double** bd, double* memory);
extern "C" void hk_wide_trs_entry(int N, int* nx, int* nu, int* nb, int** idxb, int* ng, double** hpBAbt,
                                  double** hb, double** hq, double** hpDCt, double** qx, double** hux, int compute_pi,
                                  double** hpi, int compute_Pb, double** hPb, double* memory);

namespace {

enum { K_SV = 0, K_TRF = 1, K_TRS = 2, K_RES = 3, K_IPM = 4, K_KKT = 5, K_KKT_P1 = 6, K_SOLO = 15 };
constexpr int FSTRIDE = 352, V16 = 16, V32 = 32, BS = 4, NCL = 2;

// d_back_ric_rec_sv_tv_res runs the two-wave kernel (hk_ric2.hip: the tile recursion on one wave, fetch / row half /
// stores on the other) when the library is the ric2 build variant (hpmpc_amd.build.build_ric2, -DHK_RIC2),
// HPMPC_MI355X_RIC_WAVES=2 asks for it and its launch guard accepts the launch (HK_LAUNCH_REFUSED = -2,
// hk_launch_guard.h).  The product library has the one-wave kernel only: it measured faster at every batch (DESIGN.md
// §4, round 5).  Every other entry point is hk_launch's.
int launch(int which, const KArgs* a, int count, hipStream_t s) {
#ifdef HK_RIC2
    if (which == K_SV) {
        const char* e = getenv("HPMPC_MI355X_RIC_WAVES");
        if (e && e[0] == '2') {
            const int r = hk_launch_ric2(which, a, count, s);
            if (r != -2) return r;
        }
    }
#endif
    return hk_launch(which, a, count, s);
}

struct StageInfoH {  // mirror of hk::StageInfo
    int nu, nx, nb, ng, xo, nx1, nu1, xo1, sdB, sdR, oB, oR, oD, pnb, r0, oG;
};

inline int rup(int n, int m) { return (n + m - 1) / m * m; }
inline double& P4(double* A, int sd, int i, int j) { return A[(i / BS) * BS * sd + i % BS + BS * j]; }

thread_local int g_err = 0;

void set_err(int code, const char* what) {
    g_err = code;
    if (code) fprintf(stderr, "[hpmpc_mi355x] %s (code %d)\n", what, code);
}

bool hip_ok(hipError_t e, const char* what) {
    if (e == hipSuccess) return true;
    char msg[256];
    snprintf(msg, sizeof msg, "HIP error in %s: %s", what, hipGetErrorString(e));
    set_err(HPMPC_MI355X_EHIP, msg);
    return false;
}

}  // namespace

// error reporting shared with the wide-stage translation unit
extern "C" void hk_set_error(int code, const char* what) {
    if (code)
        set_err(code, what);
    else
        g_err = 0;
}

// ------------------------------------------------------------------------------------------------
// Plan: stage tables shared by every problem of a batch.
// ------------------------------------------------------------------------------------------------
struct hpmpc_mi355x_plan {
    int N = 0;
    std::vector<int> nx, nu, nb, ng;
    std::vector<std::vector<int>> idxb;
    std::vector<StageInfoH> st;
    std::vector<signed char> tileslot, slotvar;
    std::vector<long long> offB, offR;  // packed default layout
    long long packB = 0, packR = 0;
    void* d_st = nullptr;  // the stage table of the packed default layout (uploaded once, never rewritten)
    signed char *d_tileslot = nullptr, *d_slotvar = nullptr;
    // one device stage table per caller layout (hpmpc_mi355x_layout: offsets and shared-block flags differ), uploaded
    // the first time a layout is used and never rewritten: a launch still running on another stream keeps reading its
    // own layout's offsets while the next call uses a different one
    struct LayoutTable {
        std::vector<StageInfoH> st;
        void* d = nullptr;
    };
    std::vector<LayoutTable> ltabs;  // at most kMaxLayouts, guarded by ltabs_mu (calls on one plan from several threads)
    std::mutex ltabs_mu;
    int fixcls = 0;                             // compiled inner-stage class (kernel instance)
    int nbt = 0;                                // sum of nb + ng
    int ngt = 0;                                // sum of ng
    std::vector<long long> offG;                // DCt_k offsets (packed), per stage
    long long packG = 0;
};

namespace {

bool plan_supported(int N, const int* nx, const int* nu, const int* nb, const int* const* idxb, const int* ng,
                    const char** why) {
    // the tile kernels stage the plan's tables in LDS, 256 B + 104 B per stage (hpmpc_kernels.hip launch_t: Scratch +
    // StageInfo + tile / slot tables + the certificate bounds), within the 160 KiB one workgroup may use
    if (256 + 104LL * (N + 1) > 160 * 1024) {
        *why = "horizon beyond the LDS stage tables of the tile kernels (N <= 1571)";
        return false;
    }
    for (int k = 0; k <= N; k++) {
        const int u = k < N ? nu[k] : 0;
        if (ng[k] < 0 || rup(nb[k], 4) + rup(ng[k], 4) > 16) {
            *why = "round_up(nb[k],4) + round_up(ng[k],4) must be <= 16 (one 32-slot constraint vector per stage)";
            return false;
        }
        if (u < 0 || nx[k] < 0 || u + nx[k] > 16 || rup(u, 4) + nx[k] > 16) {
            *why = "stage size beyond the 16-wide tile (nu+nx <= 16, round_up(nu,4)+nx <= 16)";
            return false;
        }
        if (nb[k] < 0 || nb[k] > u + nx[k]) {
            *why = "nb[k] > nu[k]+nx[k]";
            return false;
        }
        if (idxb) {  // box indices: in range and distinct (one box per variable)
            unsigned seen = 0;
            for (int j = 0; j < nb[k]; j++) {
                const int v = idxb[k][j];
                if (v < 0 || v >= u + nx[k] || (seen >> v & 1u)) {
                    *why = "idxb[k] must hold distinct variable indices in [0, nu[k]+nx[k])";
                    return false;
                }
                seen |= 1u << v;
            }
        }
    }
    if (N < 1) {
        *why = "N must be >= 1";
        return false;
    }
    return true;
}

// Stage offsets (and the shared-block flags, StageInfo r0 bits 1 / 2: the block of stage k sits at the batch's
// base + offset for every problem) into the device stage table; re-uploaded only when they change.
// The device stage table for the given stage offsets and shared-block flags: the plan's default table when they are
// the packed defaults, else the table of that layout (uploaded on first use, cached for the plan's lifetime).
const void* plan_stage_table(hpmpc_mi355x_plan* P, const long long* offB, const long long* offR,
                             const unsigned char* shB = nullptr, const unsigned char* shR = nullptr) {
    const int N = P->N;
    std::vector<StageInfoH> st = P->st;
    for (int k = 0; k <= N; k++) {
        st[k].oB = k < N ? (int)offB[k] : 0;
        st[k].oR = (int)offR[k];
        st[k].r0 = (P->st[k].r0 & 1) | ((shB && k < N && shB[k]) ? 2 : 0) | ((shR && shR[k]) ? 4 : 0);
    }
    const size_t bytes = sizeof(StageInfoH) * (N + 1);
    if (!memcmp(st.data(), P->st.data(), bytes)) return P->d_st;
    std::lock_guard<std::mutex> lock(P->ltabs_mu);
    for (const auto& t : P->ltabs)
        if (!memcmp(st.data(), t.st.data(), bytes)) return t.d;
    // each distinct layout keeps a device table (and its first use a synchronous upload) until the plan is destroyed:
    // a caller whose offsets change from call to call would grow it without bound, so the cache is capped
    constexpr size_t kMaxLayouts = 64;
    if (P->ltabs.size() >= kMaxLayouts) {
        set_err(HPMPC_MI355X_EUNSUPPORTED, "more than 64 distinct stage layouts on one plan (create a plan per layout "
                                           "family, or keep the offsets fixed)");
        return nullptr;
    }
    void* d = nullptr;
    if (!hip_ok(hipMalloc(&d, bytes), "layout stage table")) return nullptr;
    if (!hip_ok(hipMemcpy(d, st.data(), bytes, hipMemcpyHostToDevice), "layout stage table")) {
        (void)hipFree(d);
        return nullptr;
    }
    P->ltabs.push_back({std::move(st), d});
    return d;
}

// Per-problem workspace (device carve in hpmpc_kernels.hip): rounded to 256 B, so that every slot of a batch or queue
// starts on a cache-line boundary and its 16- / 32-double stage vectors stay line-aligned (the certificate's N+1
// doubles alone would shift each slot by 8 B per stage: +50 % on the element-wise update pass, measured)
long long ws_doubles(int N) {
    const long long n = (long long)(N + 1) * (FSTRIDE + 9 * V16 + 8 * V32 + 1) + 16;
    return (n + 31) / 32 * 32;
}

}  // namespace

extern "C" hpmpc_mi355x_plan* hpmpc_mi355x_plan_create(int N, const int* nx, const int* nu, const int* nb,
                                                       const int* const* idxb, const int* ng) {
    const char* why = nullptr;
    if (!plan_supported(N, nx, nu, nb, idxb, ng, &why)) {
        set_err(HPMPC_MI355X_EUNSUPPORTED, why);
        return nullptr;
    }
    auto* P = new hpmpc_mi355x_plan();
    P->N = N;
    P->nx.assign(nx, nx + N + 1);
    P->nu.assign(nu, nu + N + 1);
    P->nu[N] = 0;
    P->nb.assign(nb, nb + N + 1);
    P->ng.assign(ng, ng + N + 1);
    P->idxb.resize(N + 1);
    P->st.resize(N + 1);
    P->tileslot.assign((N + 1) * 16, -1);
    P->slotvar.assign((N + 1) * 16, 0);
    P->offB.resize(N);
    P->offR.resize(N + 1);
    P->offG.resize(N + 1);
    for (int k = 0; k <= N; k++) {
        StageInfoH& s = P->st[k];
        s.nu = P->nu[k];
        s.nx = nx[k];
        s.nb = nb[k];
        s.ng = ng[k];
        s.xo = rup(s.nu, 4);
        s.nx1 = k < N ? nx[k + 1] : 0;
        s.nu1 = k + 1 < N ? P->nu[k + 1] : 0;
        s.xo1 = rup(s.nu1, 4);
        s.sdB = rup(s.nx1, NCL);
        s.sdR = rup(s.nu + s.nx, NCL);
        s.pnb = rup(nb[k], BS);
        s.oD = k * V32;
        s.r0 = 0;
        s.oG = (int)P->packG;
        P->offG[k] = P->packG;
        if (ng[k] > 0) P->packG += (long long)rup(s.nu + s.nx, BS) * rup(ng[k], NCL);
        P->nbt += ng[k];
        P->ngt += ng[k];
        const int nux = s.nu + s.nx;
        if (k < N) {
            P->offB[k] = P->packB;
            P->packB += (long long)rup(nux + 1, BS) * s.sdB;
        }
        P->offR[k] = P->packR;
        P->packR += (long long)rup(nux + 1, BS) * s.sdR;
        // idxb[k] is read only for a stage with boxes: callers without boxes may pass idxb = NULL (the reference's
        // test_d_ric_mpc.c does), exactly as the reference never touches it there
        if (nb[k] > 0) P->idxb[k].assign(idxb[k], idxb[k] + nb[k]);
        P->nbt += nb[k];
        for (int l = 0; l < nb[k]; l++) {
            const int v = idxb[k][l];
            const int t = v < s.nu ? v : s.xo + (v - s.nu);
            P->tileslot[k * 16 + t] = (signed char)l;
            P->slotvar[k * 16 + l] = (signed char)v;
        }
    }
    // Inner stages of one compiled class run the constant-shape kernel path (StageInfo.r0 = 1).
    if (N >= 3) {
        const int nuc = P->nu[1], nxc = nx[1];
        P->fixcls = hk_fixcls(nuc, nxc);
        if (P->fixcls)
            for (int k = 1; k <= N - 2; k++)
                P->st[k].r0 = (P->nu[k] == nuc && nx[k] == nxc && P->nu[k + 1] == nuc && nx[k + 1] == nxc &&
                               ng[k] == 0)
                                  ? 1
                                  : 0;
    }
    for (int k = 0; k <= N; k++) {  // the packed default layout
        P->st[k].oB = k < N ? (int)P->offB[k] : 0;
        P->st[k].oR = (int)P->offR[k];
    }
    bool ok = hip_ok(hipMalloc(&P->d_st, sizeof(StageInfoH) * (N + 1)), "plan alloc") &&
              hip_ok(hipMalloc((void**)&P->d_tileslot, (N + 1) * 16), "plan alloc") &&
              hip_ok(hipMalloc((void**)&P->d_slotvar, (N + 1) * 16), "plan alloc") &&
              hip_ok(hipMemcpy(P->d_tileslot, P->tileslot.data(), (N + 1) * 16, hipMemcpyHostToDevice), "plan") &&
              hip_ok(hipMemcpy(P->d_slotvar, P->slotvar.data(), (N + 1) * 16, hipMemcpyHostToDevice), "plan") &&
              hip_ok(hipMemcpy(P->d_st, P->st.data(), sizeof(StageInfoH) * (N + 1), hipMemcpyHostToDevice), "plan");
    if (!ok) {
        hpmpc_mi355x_plan_destroy(P);
        return nullptr;
    }
    g_err = 0;
    return P;
}

extern "C" void hpmpc_mi355x_plan_destroy(hpmpc_mi355x_plan* P) {
    if (!P) return;
    if (P->d_st) (void)hipFree(P->d_st);
    for (auto& t : P->ltabs) (void)hipFree(t.d);
    if (P->d_tileslot) (void)hipFree(P->d_tileslot);
    if (P->d_slotvar) (void)hipFree(P->d_slotvar);
    delete P;
}

extern "C" long long hpmpc_mi355x_ws_doubles(const hpmpc_mi355x_plan* P) { return P ? ws_doubles(P->N) : 0; }

extern "C" int hpmpc_mi355x_last_error(void) { return g_err; }

// Diagnostic builds (-DHK_STAMPS, build.py build_stamps) record s_memtime stamps of problem 0 into this device
// buffer; only that build exports the setter (tools/stamps*.py load it through HPMPC_MI355X_LIB).
static unsigned long long* g_dbg_buf = nullptr;
#ifdef HK_STAMPS
extern "C" __attribute__((visibility("default"))) void hpmpc_mi355x_debug_buffer(void* dev_ptr) {
    g_dbg_buf = (unsigned long long*)dev_ptr;
}
#endif

extern "C" const char* hpmpc_mi355x_version(void) {
    return "hpmpc_mi355x 0.1 gfx950 (wave-per-problem, f64 MFMA 16x16x4 stage contractions)";
}

namespace {

KArgs base_args(const hpmpc_mi355x_plan* P, int nprob, int p0) {
    KArgs a;
    memset(&a, 0, sizeof a);
    a.N = P->N;
    a.nprob = nprob;
    a.p0 = p0;
    a.st = P->d_st;
    a.tileslot = P->d_tileslot;
    a.slotvar = P->d_slotvar;
    a.sV16 = (long long)(P->N + 1) * V16;
    a.sV32 = (long long)(P->N + 1) * V32;
    a.sW = ws_doubles(P->N);
    a.fixcls = P->fixcls;
    a.nbt = P->nbt;
    a.ngt = P->ngt;
    a.sG = P->packG;
    a.dbg = g_dbg_buf;
    return a;
}

bool layout_apply(hpmpc_mi355x_plan* P, const hpmpc_mi355x_layout* lay, KArgs& a) {
    if (P->ngt) {  // the batched entry points carry no DCt array
        set_err(HPMPC_MI355X_EUNSUPPORTED, "batched entry points: general constraints (ng > 0) need the "
                                           "reference-named entry points");
        return false;
    }
    if (lay && lay->BAbt_off && lay->RSQrq_off) {
        a.st = plan_stage_table(P, lay->BAbt_off, lay->RSQrq_off, lay->BAbt_shared, lay->RSQrq_shared);
        if (!a.st) return false;
    }
    a.sB = lay ? lay->BAbt_stride : P->packB;
    a.sR = lay ? lay->RSQrq_stride : P->packR;
    return true;
}

}  // namespace

namespace {

int ipm_launch(const hpmpc_mi355x_plan* plan, const hpmpc_mi355x_layout* lay, int nprob, int p0, int count,
               const double* BAbt, const double* RSQrq, const double* d, double* ux, double* pi, double* lam,
               double* t, double* ws, int k_max, double mu0, double mu_tol, double alpha_min, int warm_start,
               int compute_mult, int* kk, int* ret, double* stat, int which, void* stream) {
    auto* P = const_cast<hpmpc_mi355x_plan*>(plan);
    if (!P) return g_err = HPMPC_MI355X_EUNSUPPORTED;
    KArgs a = base_args(P, nprob, p0);
    if (!layout_apply(P, lay, a)) return g_err;
    a.BAbt = BAbt;
    a.RSQ = RSQrq;
    a.d = d;
    a.ux = ux;
    a.pi = pi;
    a.lam = lam;
    a.t = t;
    a.ws = ws;
    a.k_max = k_max;
    a.mu0 = mu0;
    a.mu_tol = mu_tol;
    a.alpha_min = alpha_min;
    a.warm_start = warm_start;
    a.compute_mult = compute_mult;
    a.kk = kk;
    a.ret = ret;
    a.stat = stat;
    int e = hk_launch(which, &a, count, (hipStream_t)stream);
    if (e) {
        set_err(HPMPC_MI355X_EHIP, "hk_ipm launch failed");
        return HPMPC_MI355X_EHIP;
    }
    return g_err = 0;
}

// hipEvents owned by one API call.  The destructor first waits for every event recorded on them.
struct CallEvents {
    std::vector<hipEvent_t> e;
    bool create(int n) {
        e.reserve(n);
        for (int i = 0; i < n; i++) {
            hipEvent_t x;
            if (!hip_ok(hipEventCreate(&x), "event create")) return false;
            e.push_back(x);
        }
        return true;
    }
    hipEvent_t& operator[](size_t i) { return e[i]; }
    ~CallEvents() {
        for (hipEvent_t x : e) {
            (void)hipEventSynchronize(x);
            (void)hipEventDestroy(x);
        }
    }
};

}  // namespace

extern "C" int hpmpc_mi355x_ipm_batch(const hpmpc_mi355x_plan* plan, const hpmpc_mi355x_layout* lay, int nprob,
                                      int p0, int count, const double* BAbt, const double* RSQrq, const double* d,
                                      double* ux, double* pi, double* lam, double* t, double* ws, int k_max,
                                      double mu0, double mu_tol, double alpha_min, int warm_start, int compute_mult,
                                      int* kk, int* ret, double* stat, void* stream) {
    return ipm_launch(plan, lay, nprob, p0, count, BAbt, RSQrq, d, ux, pi, lam, t, ws, k_max, mu0, mu_tol, alpha_min,
                      warm_start, compute_mult, kk, ret, stat, K_IPM, stream);
}

extern "C" int hpmpc_mi355x_ipm_solo(const hpmpc_mi355x_plan* plan, const hpmpc_mi355x_layout* lay, int nprob, int p0,
                                     int count, const double* BAbt, const double* RSQrq, const double* d, double* ux,
                                     double* pi, double* lam, double* t, double* ws, int k_max, double mu0,
                                     double mu_tol, double alpha_min, int warm_start, int compute_mult, int* kk,
                                     int* ret, double* stat, void* stream) {
    return ipm_launch(plan, lay, nprob, p0, count, BAbt, RSQrq, d, ux, pi, lam, t, ws, k_max, mu0, mu_tol, alpha_min,
                      warm_start, compute_mult, kk, ret, stat, K_SOLO, stream);
}

extern "C" int hpmpc_mi355x_ipm_batch_profiled(const hpmpc_mi355x_plan* plan, const hpmpc_mi355x_layout* lay,
                                               int nprob, int p0, int count, const double* BAbt, const double* RSQrq,
                                               const double* d, double* ux, double* pi, double* lam, double* t,
                                               double* ws, int k_max, double mu0, double mu_tol, double alpha_min,
                                               int warm_start, int compute_mult, int* kk, int* ret, double* stat,
                                               double* pass_ms, void* stream) {
    // the same launch sequence as hpmpc_mi355x_ipm_batch, with a hipEvent pair around every pass kernel
    // (events are per call: they belong to the current device, and nothing outlives the call)
    const int npass = 1 + 4 * (k_max > 0 ? k_max : 0);
    CallEvents ev;
    if (!ev.create(2 * npass)) return g_err;
    hipStream_t st = (hipStream_t)stream;
    for (int i = 0; i < npass; i++) {
        const int which = i == 0 ? 10 : 11 + (i - 1) % 4;
        if (!hip_ok(hipEventRecord(ev[2 * i], st), "event record")) return g_err;
        int rc = ipm_launch(plan, lay, nprob, p0, count, BAbt, RSQrq, d, ux, pi, lam, t, ws, k_max, mu0, mu_tol,
                            alpha_min, warm_start, compute_mult, kk, ret, stat, which, stream);
        if (rc) return rc;
        if (!hip_ok(hipEventRecord(ev[2 * i + 1], st), "event record")) return g_err;
    }
    if (!hip_ok(hipStreamSynchronize(st), "sync")) return g_err;
    for (int p = 0; p < 5; p++) pass_ms[p] = 0.0;
    for (int i = 0; i < npass; i++) {
        float ms = 0.f;
        if (!hip_ok(hipEventElapsedTime(&ms, ev[2 * i], ev[2 * i + 1]), "event time")) return g_err;
        pass_ms[i == 0 ? 0 : 1 + (i - 1) % 4] += ms;
    }
    return g_err = 0;
}

extern "C" int hpmpc_mi355x_ipm_pass(const hpmpc_mi355x_plan* plan, const hpmpc_mi355x_layout* lay, int nprob,
                                     int p0, int count, const double* BAbt, const double* RSQrq, const double* d,
                                     double* ux, double* pi, double* lam, double* t, double* ws, int k_max,
                                     double mu0, double mu_tol, double alpha_min, int warm_start, int compute_mult,
                                     int* kk, int* ret, double* stat, int pass, void* stream) {
    if (pass < 0 || pass > 4) return g_err = HPMPC_MI355X_EUNSUPPORTED;
    return ipm_launch(plan, lay, nprob, p0, count, BAbt, RSQrq, d, ux, pi, lam, t, ws, k_max, mu0, mu_tol, alpha_min,
                      warm_start, compute_mult, kk, ret, stat, 10 + pass, stream);
}

// Problem queue: n_slots workgroups each solve queue entries back to back, so a slot whose problem has
// converged starts the next entry at the following iteration instead of idling until the slowest
// problem of a batch finishes.  The host enqueues ticks (fact, pred, corr, update) in chunks and stops
// once the device-side finished counter reaches nq, checking a chunk behind so the stream never drains.
namespace {
// Polling state of the queue driver (hipEvents + a pinned copy of the device's finished counter), pooled per
// host thread and (device, stream).  A call does not wait for the chunk it enqueued last: the next call that
// reuses the same entry is on the same in-order stream, so its own records and counter copies land after every
// copy the earlier call left queued, and it reads a counter only after waiting on its own event.  Calls on other
// streams (or devices) use other entries and never see each other's counts.  Entries live as long as the thread.
struct PollState {
    int dev = -1;
    hipStream_t stream = nullptr;
    std::vector<hipEvent_t> e;
    int* hint = nullptr;
    ~PollState() {
        for (hipEvent_t x : e) {
            (void)hipEventSynchronize(x);
            (void)hipEventDestroy(x);
        }
        if (hint) (void)hipHostFree(hint);
    }
};

constexpr int kPollEvents = 2 * (8 * 4 + 1) + 4;  // queue lanes with R <= 8: chunk events, 2 copies, drain, fork/join
constexpr int HK_LAUNCH_REFUSED_H = -2;  // hk_launch_guard.h HK_LAUNCH_REFUSED

PollState* poll_state(hipStream_t st) {
    thread_local std::vector<std::unique_ptr<PollState>> pool;
    int dev = 0;
    if (!hip_ok(hipGetDevice(&dev), "get device")) return nullptr;
    for (auto& p : pool)
        if (p->dev == dev && p->stream == st) return p.get();
    auto p = std::make_unique<PollState>();
    p->dev = dev;
    p->stream = st;
    p->e.reserve(kPollEvents);
    for (int i = 0; i < kPollEvents; i++) {
        hipEvent_t x;
        if (!hip_ok(hipEventCreate(&x), "event create")) return nullptr;
        p->e.push_back(x);
    }
    if (!hip_ok(hipHostMalloc((void**)&p->hint, 8 * sizeof(int), hipHostMallocDefault), "host alloc")) return nullptr;
    for (int i = 0; i < 8; i++) p->hint[i] = 0;
    pool.push_back(std::move(p));
    return pool.back().get();
}

// Streams of the queue's extra lanes (lane i >= 1), pooled per host thread and (device, caller stream): created
// once, non-blocking, alive as long as the thread.
struct LaneStreams {
    int dev = -1;
    hipStream_t caller = nullptr;
    std::vector<hipStream_t> s;
    ~LaneStreams() {
        for (hipStream_t x : s) (void)hipStreamDestroy(x);
    }
};

hipStream_t lane_stream(hipStream_t caller, int i) {
    thread_local std::vector<std::unique_ptr<LaneStreams>> pool;
    int dev = 0;
    if (!hip_ok(hipGetDevice(&dev), "get device")) return nullptr;
    LaneStreams* ls = nullptr;
    for (auto& p : pool)
        if (p->dev == dev && p->caller == caller) ls = p.get();
    if (!ls) {
        pool.push_back(std::make_unique<LaneStreams>());
        ls = pool.back().get();
        ls->dev = dev;
        ls->caller = caller;
    }
    while ((int)ls->s.size() < i) {
        hipStream_t x;
        if (!hip_ok(hipStreamCreateWithFlags(&x, hipStreamNonBlocking), "stream create")) return nullptr;
        ls->s.push_back(x);
    }
    return ls->s[i - 1];
}

// One lane of the queue: an independent queue over its own slots, entries, control block and stream.  R ticks
// per chunk; the host enqueues chunk c and then looks at chunk c - 1 (waiting for it), so the stream never runs dry.
// A tick of the queue: three launches, hk_ipm_fact, hk_ipm_predcorr (predictor + corrector of a problem back to back)
// and hk_ipm_update; their device time goes to pass_ms[1], [2] and [4] ([3] stays 0: the corrector runs inside [2]).
constexpr int TL = 3;
constexpr int kTick[TL] = {11, 18, 14};
constexpr int kTickPass[TL] = {1, 2, 4};

template <int R>
struct QueueLane {
    static constexpr int nev = R * TL + 1;
    KArgs a;
    int nq = 0, ns = 0, drain_max = 0;  // nq: the whole queue's entries (the lanes share the entry counter)
    hipStream_t st = nullptr;
    // 2 chunk parities x nev kernel boundaries, then the two "counters copied" events and the drain's end event
    // (the (device, stream) poll pool); hdone: the pinned host copy of the counters
    hipEvent_t* ev = nullptr;
    int* hdone = nullptr;
    double* pass_ms = nullptr;  // [init + drain, fact, pred, corr, update] of this lane, or null
    long ticks = 0, cap = 0;
    bool pending = false, drained = false, done = false;

    bool launch(int which) {
        if (hk_launch(which, &a, ns, st)) {
            set_err(HPMPC_MI355X_EHIP, "hk_ipm_queue launch failed");
            return false;
        }
        return true;
    }
    bool harvest(int par) {  // chunk parity par has completed: accumulate its kernel times
        hipEvent_t* e = &ev[par * nev];
        for (int i = 0; i < R * TL; i++) {
            float ms = 0.f;
            if (!hip_ok(hipEventElapsedTime(&ms, e[i], e[i + 1]), "event time")) return false;
            pass_ms[kTickPass[i % TL]] += ms;
        }
        return true;
    }
    // the lane's counters and the init launch (every slot takes its first entry; the iterating ones form list 0)
    bool begin(int k_max) {
        if (!hip_ok(hipMemsetAsync(a.qctl + 1, 0, sizeof(int), st), "memset") ||
            !hip_ok(hipMemsetAsync(a.qctl + 2 + ns, 0, 2 * sizeof(int), st), "memset"))
            return false;
        if (pass_ms && !hip_ok(hipEventRecord(ev[0], st), "event record")) return false;
        if (!launch(10)) return false;
        if (pass_ms) {
            if (!hip_ok(hipEventRecord(ev[1], st), "event record") || !hip_ok(hipStreamSynchronize(st), "sync"))
                return false;
            float ms = 0.f;
            if (!hip_ok(hipEventElapsedTime(&ms, ev[0], ev[1]), "event time")) return false;
            pass_ms[0] = ms;
        }
        // every entry retires within k_max ticks of being handed out, and a slot is handed a new entry at
        // least every k_max ticks, so this bound is never reached by a correct run
        cap = (long)k_max * ((nq + ns - 1) / ns + 1) + R;
        return true;
    }
    // chunk c: R ticks of the four passes, then the copy of the counters
    bool enqueue(int c) {
        const int par = c & 1;
        hipEvent_t* e = &ev[par * nev];
        if (pass_ms && !hip_ok(hipEventRecord(e[0], st), "event record")) return false;
        for (int i = 0; i < R; i++) {
            a.qpar = (int)((ticks + i) & 1);  // active-slot list of this iteration (kernel args are copied at launch)
            for (int k = 0; k < TL; k++) {
                if (!launch(kTick[k])) return false;
                if (pass_ms && !hip_ok(hipEventRecord(e[TL * i + k + 1], st), "event record")) return false;
            }
        }
        ticks += R;
        // per chunk parity: [4 par] handed out (all lanes), [4 par + 1] finished (this lane), [4 par + 2 .. 3] the
        // two active-list lengths
        int* hc = &hdone[4 * par];
        return hip_ok(hipMemcpyAsync(hc, a.qnext, sizeof(int), hipMemcpyDeviceToHost, st), "copy") &&
               hip_ok(hipMemcpyAsync(hc + 1, a.qctl + 1, sizeof(int), hipMemcpyDeviceToHost, st), "copy") &&
               hip_ok(hipMemcpyAsync(hc + 2, a.qctl + 2 + ns, 2 * sizeof(int), hipMemcpyDeviceToHost, st), "copy") &&
               hip_ok(hipEventRecord(ev[2 * nev + par], st), "event record");
    }
    // after chunk c is enqueued: look at chunk c - 1; every entry handed out and none left iterating in this lane,
    // or the drain launched -> done
    bool poll(int c) {
        const int par = c & 1;
        if (pending) {
            if (!hip_ok(hipEventSynchronize(ev[2 * nev + (par ^ 1)]), "event sync")) return false;
            if (pass_ms && !harvest(par ^ 1)) return false;
            const int* hp = &hdone[4 * (par ^ 1)];
            // slots still iterating after chunk c - 1 (the active list its last update filled)
            const int nact = hp[2 + (int)((ticks - R) & 1)];
            if (hp[0] >= nq && nact == 0) {
                done = true;
                return true;
            }
            // Drain: every entry handed out and at most drain_max slots still iterating (as of the previous
            // chunk): the survivors finish in one multi-wave launch (hk_ipm_qdrain_mw) after the chunk just
            // enqueued, on the active list its last update filled
            if (drain_max > 0 && hp[0] >= nq && nact <= drain_max) {
                a.qpar = (int)(ticks & 1);
                const int r = hk_launch(17, &a, ns, st);
                if (r == 0) {
                    drained = done = true;
                    return true;
                }
                if (r != HK_LAUNCH_REFUSED_H) {
                    set_err(HPMPC_MI355X_EHIP, "hk_ipm_qdrain_mw launch failed");
                    return false;
                }
                drain_max = 0;  // refused: keep ticking
            }
        }
        pending = true;
        if (ticks >= cap) {
            set_err(HPMPC_MI355X_EHIP, "hk_ipm_queue did not drain");
            return false;
        }
        return true;
    }
    // the chunk enqueued last finds every slot idle; profiled runs wait for it so that pass_ms covers every
    // launch (ticks of each pass kernel), otherwise it completes on the stream.  A drain goes to pass_ms[0].
    bool end() {
        if (!pass_ms) return true;
        const int par = (int)((ticks / R - 1) & 1);
        hipEvent_t* done_ev = &ev[2 * nev];
        if (drained && !hip_ok(hipEventRecord(ev[2 * nev + 2], st), "event record")) return false;
        if (!hip_ok(hipEventSynchronize(done_ev[par]), "event sync") || !harvest(par)) return false;
        if (drained) {
            float ms = 0.f;
            if (!hip_ok(hipEventSynchronize(ev[2 * nev + 2]), "event sync") ||
                !hip_ok(hipEventElapsedTime(&ms, done_ev[par], ev[2 * nev + 2]), "event time"))
                return false;
            pass_ms[0] += ms;
        }
        return true;
    }
};

// The problem-queue driver (hpmpc_mi355x_ipm_queue).  `a` carries the problem data and solver parameters.  The
// slots are split into `lanes` contiguous lanes, each a queue with its own control block in qctl and its own stream
// (lane 0 on the caller's; the others forked from it and joined back into it at the end), all handing out entries
// from one shared counter: one lane's pass kernels fill the tail of another's, where a single queue's launch waits
// for its last waves, and no lane runs out of entries before the others.  Each entry's solve is the same whatever
// its lane and slot.
template <int R>
int queue_run(KArgs a, int nq, int n_slots, int* qctl, int* dctr, int lanes, int k_max, double* pass_ms,
              int* n_ticks, hipStream_t st) {
    static_assert(2 * (R * TL + 1) + 3 < kPollEvents, "poll pool sized for R <= 8, plus the fork / join event");
    if (n_ticks) *n_ticks = 0;
    if (pass_ms)
        for (int i = 0; i < 5; i++) pass_ms[i] = 0.0;
    if (nq == 0) return g_err = 0;
    lanes = std::max(1, std::min({lanes, HPMPC_MI355X_QUEUE_LANES_MAX, nq, n_slots}));
    // the drain threshold (slots still iterating once the queue is empty; split over the lanes in proportion to
    // their slots): HPMPC_MI355X_QUEUE_DRAIN, default 768 (tools/slots_probe.py: 512 / 768 / 1024 / 1536 within
    // 1 % at 6144-8192 slots); 0 keeps the ticks to the end (results then bitwise the batched solve's)
    int drain_max = 768;
    if (const char* e = getenv("HPMPC_MI355X_QUEUE_DRAIN")) drain_max = atoi(e);
    QueueLane<R> L[HPMPC_MI355X_QUEUE_LANES_MAX];
    double lane_ms[HPMPC_MI355X_QUEUE_LANES_MAX][5] = {};
    a.dctr = dctr;
    a.qnext = qctl;  // lane 0's [0]: the entry counter every lane hands out from
    if (!hip_ok(hipMemsetAsync(dctr, 0, 2 * sizeof(int), st), "memset") ||
        !hip_ok(hipMemsetAsync(qctl, 0, sizeof(int), st), "memset"))
        return g_err;
    PollState* ps0 = poll_state(st);
    if (!ps0) return g_err;
    hipEvent_t fork = ps0->e[kPollEvents - 1];
    if (lanes > 1 && !hip_ok(hipEventRecord(fork, st), "event record")) return g_err;
    int s0 = 0;
    for (int i = 0; i < lanes; i++) {
        QueueLane<R>& l = L[i];
        l.ns = n_slots / lanes + (i < n_slots % lanes);
        l.nq = nq;
        l.st = i == 0 ? st : lane_stream(st, i);  // (the caller's may be the null stream)
        if (i > 0 && !l.st) return g_err;
        PollState* ps = poll_state(l.st);
        if (!ps) return g_err;
        l.ev = ps->e.data();
        l.hdone = ps->hint;
        if (i > 0 && !hip_ok(hipStreamWaitEvent(l.st, fork, 0), "stream wait")) return g_err;
        l.a = a;
        l.a.nq = nq;
        l.a.nslots = l.ns;
        l.a.qctl = qctl + 6 * i + 3 * s0;
        l.a.qpar = 0;
        l.a.ws = a.ws + (long)s0 * a.sW;
        l.drain_max = drain_max > 0 ? std::max(1, (int)((long)drain_max * l.ns / n_slots)) : 0;
        l.pass_ms = pass_ms ? lane_ms[i] : nullptr;
        s0 += l.ns;
    }
    // Each lane runs the protocol "enqueue chunk c, then look at chunk c - 1" on its own: a lane whose chunk c - 1
    // has completed is looked at and given chunk c + 1 at once, whatever the other lanes are doing (polled without
    // blocking; with one lane this is the same sequence as waiting for the event).
    int c[HPMPC_MI355X_QUEUE_LANES_MAX] = {};
    for (int i = 0; i < lanes; i++) {
        QueueLane<R>& l = L[i];
        if (!l.begin(k_max) || !l.enqueue(0) || !l.poll(0) || !l.enqueue(1)) return g_err;
        c[i] = 1;
    }
    for (int left = lanes; left > 0;) {
        for (int i = 0; i < lanes; i++) {
            QueueLane<R>& l = L[i];
            if (l.done) continue;
            const hipError_t q = hipEventQuery(l.ev[2 * QueueLane<R>::nev + ((c[i] - 1) & 1)]);
            if (q == hipErrorNotReady) continue;
            if (!hip_ok(q, "event query") || !l.poll(c[i])) return g_err;
            if (l.done) {
                left--;
                continue;
            }
            if (!l.enqueue(++c[i])) return g_err;
        }
    }
    long ticks = 0;
    for (int i = 0; i < lanes; i++) {
        QueueLane<R>& l = L[i];
        if (!l.end()) return g_err;
        if (i > 0) {  // join: the caller's stream waits for the lane's last chunk (and drain)
            hipEvent_t join = l.ev[kPollEvents - 1];
            if (!hip_ok(hipEventRecord(join, l.st), "event record") ||
                !hip_ok(hipStreamWaitEvent(st, join, 0), "stream wait"))
                return g_err;
        }
        ticks += l.ticks;
        if (pass_ms)
            for (int k = 0; k < 5; k++) pass_ms[k] += lane_ms[i][k];
    }
    if (n_ticks) *n_ticks = (int)ticks;
    return g_err = 0;
}
}  // namespace

extern "C" int hpmpc_mi355x_ipm_queue(const hpmpc_mi355x_plan* plan, const hpmpc_mi355x_layout* lay, int nprob,
                                      int nq, int n_slots, const double* BAbt, const double* RSQrq, const double* d,
                                      double* ux, double* pi, double* lam, double* t, double* ws, int* qctl,
                                      int k_max, double mu0, double mu_tol, double alpha_min, int warm_start,
                                      int compute_mult, int* kk, int* ret, double* stat, double* pass_ms,
                                      int* n_ticks, void* stream) {
    auto* P = const_cast<hpmpc_mi355x_plan*>(plan);
    if (!P || nprob <= 0 || nq < 0 || n_slots <= 0 || !qctl) return g_err = HPMPC_MI355X_EUNSUPPORTED;
    KArgs a = base_args(P, nprob, 0);
    if (!layout_apply(P, lay, a)) return g_err;
    a.BAbt = BAbt;
    a.RSQ = RSQrq;
    a.d = d;
    a.ux = ux;
    a.pi = pi;
    a.lam = lam;
    a.t = t;
    a.ws = ws;
    a.k_max = k_max;
    a.mu0 = mu0;
    a.mu_tol = mu_tol;
    a.alpha_min = alpha_min;
    a.warm_start = warm_start;
    a.compute_mult = compute_mult;
    a.kk = kk;
    a.ret = ret;
    a.stat = stat;
    a.no_bkp = 1;  // slots are reused and no KKT re-solve follows a queue solve (header): backups are dead stores
    // lanes: HPMPC_MI355X_QUEUE_LANES (default 4), at most one per 1024 slots (a smaller queue keeps one lane)
    int lanes = 4;
    if (const char* e = getenv("HPMPC_MI355X_QUEUE_LANES")) lanes = atoi(e);
    lanes = std::min(lanes, n_slots / 1024);
    int* dctr = qctl + 6 * HPMPC_MI355X_QUEUE_LANES_MAX + 3 * n_slots;
    return queue_run<8>(a, nq, n_slots, qctl, dctr, lanes, k_max, pass_ms, n_ticks, (hipStream_t)stream);
}

extern "C" int hpmpc_mi355x_ric_sv_batch(const hpmpc_mi355x_plan* plan, const hpmpc_mi355x_layout* lay, int nprob,
                                         int p0, int count, const double* BAbt, const double* RSQrq, double* ux,
                                         double* pi, double* ws, int compute_pi, int compute_Pb, double* Pb,
                                         void* stream) {
    auto* P = const_cast<hpmpc_mi355x_plan*>(plan);
    if (!P) return g_err = HPMPC_MI355X_EUNSUPPORTED;
    KArgs a = base_args(P, nprob, p0);
    if (!layout_apply(P, lay, a)) return g_err;
    a.BAbt = BAbt;
    a.RSQ = RSQrq;
    a.ux = ux;
    a.pi = pi;
    a.ws = ws;
    a.compute_pi = compute_pi;
    a.compute_Pb = compute_Pb && Pb;
    a.vPb = Pb;
    int e = launch(K_SV, &a, count, (hipStream_t)stream);
    if (e) {
        set_err(HPMPC_MI355X_EHIP, "hk_ric_sv launch failed");
        return HPMPC_MI355X_EHIP;
    }
    return g_err = 0;
}

extern "C" int hpmpc_mi355x_ric_trf_batch(const hpmpc_mi355x_plan* plan, const hpmpc_mi355x_layout* lay, int nprob,
                                          int p0, int count, const double* BAbt, const double* RSQrq, double* ws,
                                          void* stream) {
    auto* P = const_cast<hpmpc_mi355x_plan*>(plan);
    if (!P) return g_err = HPMPC_MI355X_EUNSUPPORTED;
    KArgs a = base_args(P, nprob, p0);
    if (!layout_apply(P, lay, a)) return g_err;
    a.BAbt = BAbt;
    a.RSQ = RSQrq;
    a.ws = ws;
    int e = hk_launch(K_TRF, &a, count, (hipStream_t)stream);
    if (e) {
        set_err(HPMPC_MI355X_EHIP, "hk_ric_trf launch failed");
        return HPMPC_MI355X_EHIP;
    }
    return g_err = 0;
}

extern "C" int hpmpc_mi355x_ric_trs_batch(const hpmpc_mi355x_plan* plan, const hpmpc_mi355x_layout* lay, int nprob,
                                          int p0, int count, const double* BAbt, const double* RSQrq, const double* b,
                                          const double* q, double* ux, double* pi, double* ws, int compute_pi,
                                          int compute_Pb, double* Pb, void* stream) {
    auto* P = const_cast<hpmpc_mi355x_plan*>(plan);
    if (!P) return g_err = HPMPC_MI355X_EUNSUPPORTED;
    KArgs a = base_args(P, nprob, p0);
    if (!layout_apply(P, lay, a)) return g_err;
    a.BAbt = BAbt;
    a.RSQ = RSQrq;
    a.vb = b;
    a.vq = q;
    a.ux = ux;
    a.pi = pi;
    a.ws = ws;
    a.compute_pi = compute_pi;
    a.compute_Pb = compute_Pb;
    a.vPb = Pb;
    int e = hk_launch(K_TRS, &a, count, (hipStream_t)stream);
    if (e) {
        set_err(HPMPC_MI355X_EHIP, "hk_ric_trs launch failed");
        return HPMPC_MI355X_EHIP;
    }
    return g_err = 0;
}

// ================================================================================================
// Single-problem reference entry points
// ================================================================================================
namespace {

// Thread-local device context: one stream, growable device arena, pinned staging arena, plan cache.
struct Ctx {
    hipStream_t stream = nullptr;
    double* dev = nullptr;
    size_t dev_cap = 0;
    double* host = nullptr;
    size_t host_cap = 0;
    hpmpc_mi355x_plan* plan = nullptr;
    std::vector<int> key;
    ~Ctx() {
        if (plan) hpmpc_mi355x_plan_destroy(plan);
        if (dev) (void)hipFree(dev);
        if (host) (void)hipHostFree(host);
        if (stream) (void)hipStreamDestroy(stream);
    }
    bool ensure(size_t n) {
        if (!stream && !hip_ok(hipStreamCreateWithFlags(&stream, hipStreamNonBlocking), "stream create"))
            return false;
        if (n > dev_cap) {
            if (dev) (void)hipFree(dev);
            dev = nullptr;
            dev_cap = 0;
            if (!hip_ok(hipMalloc((void**)&dev, n * sizeof(double)), "device arena")) return false;
            dev_cap = n;
        }
        if (n > host_cap) {
            if (host) (void)hipHostFree(host);
            host = nullptr;
            host_cap = 0;
            if (!hip_ok(hipHostMalloc((void**)&host, n * sizeof(double), 0), "pinned arena")) return false;
            host_cap = n;
        }
        memset(host, 0, n * sizeof(double));
        return true;
    }
    hpmpc_mi355x_plan* get_plan(int N, const int* nx, const int* nu, const int* nb, int** idxb, const int* ng) {
        std::vector<int> k;
        k.push_back(N);
        for (int i = 0; i <= N; i++) {
            k.push_back(nx[i]);
            k.push_back(i < N ? nu[i] : 0);
            k.push_back(nb[i]);
            k.push_back(ng[i]);
            for (int l = 0; l < nb[i]; l++) k.push_back(idxb[i][l]);
        }
        if (plan && k == key) return plan;
        if (plan) hpmpc_mi355x_plan_destroy(plan);
        plan = hpmpc_mi355x_plan_create(N, nx, nu, nb, idxb, ng);
        key = plan ? k : std::vector<int>();
        return plan;
    }
};

thread_local Ctx g_ctx;

// Arena carve (doubles) for one problem.
struct Arena {
    size_t BAbt, RSQ, DCt, d, ux, pi, lam, t, ws, vb, vq, vQx, vqx, vPb, stat, ints, qctl, total;
};

Arena arena(const hpmpc_mi355x_plan* P, int k_max) {
    Arena A;
    size_t o = 0;
    auto take = [&](size_t n) {  // 128-B granules: every array starts on a cache line
        size_t r = o;
        o += (n + 15) / 16 * 16;
        return r;
    };
    const size_t n1 = P->N + 1;
    A.BAbt = take(P->packB);
    A.RSQ = take(P->packR);
    A.DCt = take(P->packG > 0 ? P->packG : 1);
    A.d = take(n1 * V32);
    A.ux = take(n1 * V16);
    A.pi = take(n1 * V16);
    A.lam = take(n1 * V32);
    A.t = take(n1 * V32);
    A.ws = take(ws_doubles(P->N));
    A.vb = take(n1 * V16);
    A.vq = take(n1 * V16);
    A.vQx = take(n1 * V16);
    A.vqx = take(n1 * V16);
    A.vPb = take(n1 * V16);
    A.stat = take(5 * (size_t)(k_max > 0 ? k_max : 1) + 8);
    A.ints = take(8);
    A.qctl = take(8);  // queue control of the one-entry queue the IPM entry points run (16 ints >= 6 + 3 slots)
    A.total = o;
    return A;
}

KArgs arena_args(const hpmpc_mi355x_plan* P, const Arena& A, double* dev) {
    KArgs a = base_args(P, 1, 0);
    a.sB = P->packB;
    a.sR = P->packR;
    a.BAbt = dev + A.BAbt;
    a.RSQ = dev + A.RSQ;
    a.DCt = P->ngt ? dev + A.DCt : nullptr;
    a.d = dev + A.d;
    a.ux = dev + A.ux;
    a.pi = dev + A.pi;
    a.lam = dev + A.lam;
    a.t = dev + A.t;
    a.ws = dev + A.ws;
    a.vb = dev + A.vb;
    a.vq = dev + A.vq;
    a.vQx = dev + A.vQx;
    a.vqx = dev + A.vqx;
    a.vPb = dev + A.vPb;
    a.stat = dev + A.stat;
    a.kk = reinterpret_cast<int*>(dev + A.ints);
    a.ret = a.kk + 1;
    a.mu_out = dev + A.ints + 2;
    return a;
}

// copy stage blocks (lib4, possibly aliased) into the packed arena layout
void stage_BAbt(const hpmpc_mi355x_plan* P, double* H, const Arena& A, double** hpBAbt) {
    for (int k = 0; k < P->N; k++) {
        const auto& s = P->st[k];
        const size_t n = (size_t)rup(s.nu + s.nx + 1, BS) * s.sdB;
        memcpy(H + A.BAbt + P->offB[k], hpBAbt[k], n * sizeof(double));
    }
}
void stage_RSQ(const hpmpc_mi355x_plan* P, double* H, const Arena& A, double** hpQ) {
    for (int k = 0; k <= P->N; k++) {
        const auto& s = P->st[k];
        const size_t n = (size_t)rup(s.nu + s.nx + 1, BS) * s.sdR;
        memcpy(H + A.RSQ + P->offR[k], hpQ[k], n * sizeof(double));
    }
}
// constraint vectors per stage: [lb (pnb) | ub (pnb) | lg (png) | ug (png)]
int cvec_len(const hpmpc_mi355x_plan* P, int k) { return 2 * P->st[k].pnb + 2 * rup(P->ng[k], BS); }
void stage_d(const hpmpc_mi355x_plan* P, double* H, const Arena& A, double** d) {
    for (int k = 0; k <= P->N; k++)
        if (P->nb[k] + P->ng[k] > 0) memcpy(H + A.d + k * V32, d[k], cvec_len(P, k) * sizeof(double));
}
void stage_DCt(const hpmpc_mi355x_plan* P, double* H, const Arena& A, double** hpDCt) {
    for (int k = 0; k <= P->N; k++) {
        if (P->ng[k] == 0) continue;
        const auto& s = P->st[k];
        memcpy(H + A.DCt + P->offG[k], hpDCt[k],
               (size_t)rup(s.nu + s.nx, BS) * rup(P->ng[k], NCL) * sizeof(double));
    }
}
// Qx / qx of the general constraints ([box (pnb) | general (png)]): the box halves are applied on the
// host for sv / trf, so the device sees zeros there and only adds the general terms.
void stage_gen_q(const hpmpc_mi355x_plan* P, double* H, size_t off, double** v) {
    for (int k = 0; k <= P->N; k++)
        for (int l = 0; l < P->ng[k]; l++) H[off + k * V16 + P->st[k].pnb + l] = v[k][P->st[k].pnb + l];
}

bool run(int which, const KArgs& a, const char* name) {
    int e = launch(which, &a, 1, g_ctx.stream);
    if (e) {
        char msg[128];
        snprintf(msg, sizeof msg, "%s launch failed (%d)", name, e);
        set_err(HPMPC_MI355X_EHIP, msg);
        return false;
    }
    return true;
}

bool up(const Arena& A) {
    return hip_ok(hipMemcpyAsync(g_ctx.dev, g_ctx.host, A.total * sizeof(double), hipMemcpyHostToDevice,
                                 g_ctx.stream),
                  "H2D");
}
bool down(const Arena& A) {
    return hip_ok(hipMemcpyAsync(g_ctx.host, g_ctx.dev, A.total * sizeof(double), hipMemcpyDeviceToHost,
                                 g_ctx.stream),
                  "D2H") &&
           hip_ok(hipStreamSynchronize(g_ctx.stream), "sync");
}

}  // namespace

extern "C" int d_back_ric_rec_sv_tv_work_space_size_bytes(int N, int* nx, int* nu, int* nb, int* ng) {
    (void)N;
    (void)nx;
    (void)nu;
    (void)nb;
    (void)ng;
    return 64;  // all temporaries live on the device
}

extern "C" int d_back_ric_rec_sv_tv_memory_space_size_bytes(int N, int* nx, int* nu, int* nb, int* ng) {
    (void)nx;
    (void)nu;
    (void)nb;
    (void)ng;
    // the larger of the tile image and the wide-stage factor (nu+nx > 16 stages run on the wide path)
    const long long tile = (long long)(N + 1) * FSTRIDE * 8, wide = hk_wide_factor_bytes(N, nx, nu);
    return (int)(((tile > wide ? tile : wide) + 63) / 64 * 64);
}

extern "C" void d_back_ric_rec_sv_tv_res(int N, int* nx, int* nu, int* nb, int** idxb, int* ng, int update_b,
                                         double** hpBAbt, double** b, int update_q, double** hpQ, double** q,
                                         double** bd, double** hpDCt, double** Qx, double** qx, double** hux,
                                         int compute_pi, double** hpi, int compute_Pb, double** hPb, double* memory,
                                         double* work) {
    (void)work;
    g_err = 0;
    {
        const char* why = nullptr;
        if (!plan_supported(N, nx, nu, nb, idxb, ng, &why)) {  // stages beyond the 16-wide tile
            hk_wide_sv_entry(N, nx, nu, nb, idxb, ng, update_b, hpBAbt, b, update_q, hpQ, q, bd, hpDCt, Qx, qx, hux,
                             compute_pi, hpi, compute_Pb, hPb, memory);
            return;
        }
    }
    hpmpc_mi355x_plan* P = g_ctx.get_plan(N, nx, nu, nb, idxb, ng);
    if (!P) return;
    Arena A = arena(P, 1);
    if (!g_ctx.ensure(A.total)) return;
    double* H = g_ctx.host;
    // Stage copies receive exactly what the reference factorises for that stage; the caller's
    // buffers get the reference's side effects, applied in its stage order (N .. 0).
    for (int k = N; k >= 0; k--) {
        const auto& s = P->st[k];
        const int nux = s.nu + s.nx, cnux = s.sdR;
        if (update_q)
            for (int j = 0; j < nux; j++) P4(hpQ[k], cnux, nux, j) = q[k][j];
        for (int l = 0; l < nb[k]; l++) {
            const int ii = idxb[k][l];
            P4(hpQ[k], cnux, ii, ii) = bd[k][l] + Qx[k][l];
        }
        for (int l = 0; l < nb[k]; l++) P4(hpQ[k], cnux, nux, idxb[k][l]) += qx[k][l];
        memcpy(H + A.RSQ + P->offR[k], hpQ[k], (size_t)rup(nux + 1, BS) * cnux * sizeof(double));
        if (k < N) {
            if (update_b)
                for (int j = 0; j < s.nx1; j++) P4(hpBAbt[k], s.sdB, nux, j) = b[k][j];
            memcpy(H + A.BAbt + P->offB[k], hpBAbt[k], (size_t)rup(nux + 1, BS) * s.sdB * sizeof(double));
        }
    }
    KArgs a = arena_args(P, A, g_ctx.dev);
    a.compute_pi = compute_pi;
    a.compute_Pb = compute_Pb;
    if (P->ngt) {  // general constraints: DCt diag(Qx_g) DCt' and DCt qx_g on the device
        stage_DCt(P, H, A, hpDCt);
        stage_gen_q(P, H, A.vQx, Qx);
        stage_gen_q(P, H, A.vqx, qx);
        a.use_box = 1;
    }
    if (!up(A) || !run(K_SV, a, "hk_ric_sv") || !down(A)) return;
    for (int k = 0; k <= N; k++) {
        const int nux = P->st[k].nu + P->st[k].nx;
        memcpy(hux[k], H + A.ux + k * V16, nux * sizeof(double));
        if (k < N && compute_pi) memcpy(hpi[k], H + A.pi + k * V16, nx[k + 1] * sizeof(double));
        if (k < N && compute_Pb) memcpy(hPb[k], H + A.vPb + k * V16, nx[k + 1] * sizeof(double));
    }
    memcpy(memory, H + A.ws, (size_t)(N + 1) * FSTRIDE * sizeof(double));
}

extern "C" void d_back_ric_rec_trf_tv_res(int N, int* nx, int* nu, int* nb, int** idxb, int* ng, double** hpBAbt,
                                          double** hpQ, double** hpDCt, double** Qx, double** bd, double* memory,
                                          double* work) {
    (void)work;
    g_err = 0;
    {
        const char* why = nullptr;
        if (!plan_supported(N, nx, nu, nb, idxb, ng, &why)) {  // stages beyond the 16-wide tile
            hk_wide_trf_entry(N, nx, nu, nb, idxb, ng, hpBAbt, hpQ, hpDCt, Qx, bd, memory);
            return;
        }
    }
    hpmpc_mi355x_plan* P = g_ctx.get_plan(N, nx, nu, nb, idxb, ng);
    if (!P) return;
    Arena A = arena(P, 1);
    if (!g_ctx.ensure(A.total)) return;
    double* H = g_ctx.host;
    for (int k = N; k >= 0; k--) {
        const auto& s = P->st[k];
        const int nux = s.nu + s.nx, cnux = s.sdR;
        for (int l = 0; l < nb[k]; l++) {
            const int ii = idxb[k][l];
            P4(hpQ[k], cnux, ii, ii) = bd[k][l] + Qx[k][l];
        }
        memcpy(H + A.RSQ + P->offR[k], hpQ[k], (size_t)rup(nux + 1, BS) * cnux * sizeof(double));
        if (k < N) memcpy(H + A.BAbt + P->offB[k], hpBAbt[k], (size_t)rup(nux + 1, BS) * s.sdB * sizeof(double));
    }
    KArgs a = arena_args(P, A, g_ctx.dev);
    if (P->ngt) {
        stage_DCt(P, H, A, hpDCt);
        stage_gen_q(P, H, A.vQx, Qx);
        a.use_box = 1;
    }
    if (!up(A) || !run(K_TRF, a, "hk_ric_trf") || !down(A)) return;
    memcpy(memory, H + A.ws, (size_t)(N + 1) * FSTRIDE * sizeof(double));
}

extern "C" void d_back_ric_rec_trs_tv_res(int N, int* nx, int* nu, int* nb, int** idxb, int* ng, double** hpBAbt,
                                          double** hb, double** hq, double** hpDCt, double** qx, double** hux,
                                          int compute_pi, double** hpi, int compute_Pb, double** hPb, double* memory,
                                          double* work) {
    (void)work;
    g_err = 0;
    {
        const char* why = nullptr;
        if (!plan_supported(N, nx, nu, nb, idxb, ng, &why)) {  // stages beyond the 16-wide tile
            hk_wide_trs_entry(N, nx, nu, nb, idxb, ng, hpBAbt, hb, hq, hpDCt, qx, hux, compute_pi, hpi, compute_Pb,
                              hPb, memory);
            return;
        }
    }
    hpmpc_mi355x_plan* P = g_ctx.get_plan(N, nx, nu, nb, idxb, ng);
    if (!P) return;
    Arena A = arena(P, 1);
    if (!g_ctx.ensure(A.total)) return;
    double* H = g_ctx.host;
    stage_BAbt(P, H, A, hpBAbt);
    memcpy(H + A.ws, memory, (size_t)(N + 1) * FSTRIDE * sizeof(double));
    for (int k = 0; k <= N; k++) {
        const int nux = P->st[k].nu + P->st[k].nx;
        memcpy(H + A.vq + k * V16, hq[k], nux * sizeof(double));
        if (k < N) memcpy(H + A.vb + k * V16, hb[k], nx[k + 1] * sizeof(double));
        if (k < N && !compute_Pb) memcpy(H + A.vPb + k * V16, hPb[k], nx[k + 1] * sizeof(double));
        if (nb[k] > 0) memcpy(H + A.vqx + k * V16, qx[k], nb[k] * sizeof(double));
    }
    if (P->ngt) {
        stage_DCt(P, H, A, hpDCt);
        stage_gen_q(P, H, A.vqx, qx);
    }
    KArgs a = arena_args(P, A, g_ctx.dev);
    a.use_box = 1;
    a.compute_pi = compute_pi;
    a.compute_Pb = compute_Pb;
    if (!up(A) || !run(K_TRS, a, "hk_ric_trs") || !down(A)) return;
    for (int k = 0; k <= N; k++) {
        const int nux = P->st[k].nu + P->st[k].nx;
        memcpy(hux[k], H + A.ux + k * V16, nux * sizeof(double));
        if (k < N && compute_pi) memcpy(hpi[k], H + A.pi + k * V16, nx[k + 1] * sizeof(double));
        if (k < N && compute_Pb) memcpy(hPb[k], H + A.vPb + k * V16, nx[k + 1] * sizeof(double));
    }
}

extern "C" int d_ip2_res_mpc_hard_tv_work_space_size_bytes(int N, int* nx, int* nu, int* nb, int* ng) {
    // the larger of the tile path's image and the wide-stage IPM's (problems beyond the tile run there)
    std::vector<int> nuN(nu, nu + N + 1);
    nuN[N] = 0;
    const long long tile = ws_doubles(N) * 8, wide = hk_wide_ipm_bytes(N, nx, nuN.data(), nb, ng);
    return (int)(((tile > wide ? tile : wide) + 63) / 64 * 64);
}

namespace {
// stages beyond the 16-wide tile (or its 32 constraint slots) run on the wide-stage path
bool wide_path(int N, const int* nx, const int* nu, const int* nb, int** idxb, const int* ng) {
    const char* why = nullptr;
    return !plan_supported(N, nx, nu, nb, idxb, ng, &why);
}
}  // namespace

namespace {

// Shared body of d_ip2_res_mpc_hard_tv and its single-Newton variant.  For the variant, ux0/pi0/lam0/t0
// hold the start iterate (lam0/t0 as [lower(nb) | upper(nb)], d_aux_ip_hard_lib4.c:153-213).
int ipm_entry(int single_newton, int phase1_only, int* kk, int k_max, double mu0, double mu_tol, double alpha_min, int warm_start,
              double* stat, int N, int* nx, int* nu_N, int* nb, int** idxb, int* ng, double** pBAbt, double** pQ,
              double** pDCt, double** d, double** ux, int compute_mult, double** pi, double** lam, double** t,
              double* double_work_memory, double** ux0, double** pi0, double** lam0, double** t0) {
    g_err = 0;
    if (wide_path(N, nx, nu_N, nb, idxb, ng))
        return hk_wide_ipm_entry(single_newton ? WI_NEWTON : phase1_only ? WI_IPM_P1 : WI_IPM_RES, kk, k_max, mu0,
                                 mu_tol, alpha_min, warm_start, stat, N, nx, nu_N, nb, idxb, ng, pBAbt, pQ, pDCt, d, ux,
                                 compute_mult, pi, lam, t, double_work_memory, ux0, pi0, lam0, t0);
    hpmpc_mi355x_plan* P = g_ctx.get_plan(N, nx, nu_N, nb, idxb, ng);
    if (!P) return g_err;
    if (single_newton && P->ngt) {  // the reference stops here too (d_aux_ip_hard_lib4.c:197-208)
        set_err(HPMPC_MI355X_EUNSUPPORTED, "single Newton step with general constraints");
        return g_err;
    }
    Arena A = arena(P, k_max);
    if (!g_ctx.ensure(A.total)) return g_err;
    double* H = g_ctx.host;
    stage_BAbt(P, H, A, pBAbt);
    stage_RSQ(P, H, A, pQ);
    stage_d(P, H, A, d);
    stage_DCt(P, H, A, pDCt);
    if (single_newton) {
        for (int k = 0; k <= N; k++) {
            memcpy(H + A.ux + k * V16, ux0[k], (P->st[k].nu + nx[k]) * sizeof(double));
            if (k < N) memcpy(H + A.pi + k * V16, pi0[k], nx[k + 1] * sizeof(double));
            const int pnb = P->st[k].pnb;
            for (int l = 0; l < nb[k]; l++) {
                H[A.lam + k * V32 + l] = lam0[k][l];
                H[A.lam + k * V32 + pnb + l] = lam0[k][nb[k] + l];
                H[A.t + k * V32 + l] = t0[k][l];
                H[A.t + k * V32 + pnb + l] = t0[k][nb[k] + l];
            }
        }
    } else if (warm_start) {
        for (int k = 0; k <= N; k++) memcpy(H + A.ux + k * V16, ux[k], (P->st[k].nu + nx[k]) * sizeof(double));
    }
    KArgs a = arena_args(P, A, g_ctx.dev);
    a.k_max = k_max;
    a.mu0 = mu0;
    a.mu_tol = mu_tol;
    a.alpha_min = alpha_min;
    a.warm_start = warm_start;
    a.compute_mult = compute_mult;
    a.single_newton = single_newton;
    a.phase1_only = phase1_only;
    // the whole solve in one launch (hk_ipm_solo): one workgroup runs init and every iteration's passes back to
    // back, its stage data and factor records resident in one XCD's L2
    if (!up(A)) return g_err;
    if (hk_launch(K_SOLO, &a, 1, g_ctx.stream)) {
        set_err(HPMPC_MI355X_EHIP, "hk_ipm_solo launch failed");
        return g_err;
    }
    if (!down(A)) return g_err;
    const int* iv = reinterpret_cast<const int*>(H + A.ints);
    *kk = iv[0];
    if (iv[1] == HPMPC_MI355X_EMW) {
        // the multi-wave kernel abandoned the solve (an expired hand-over wait: a bug, never a data condition); its
        // stat holds diagnostics and its iterate is not a solution, so nothing is copied out
        set_err(HPMPC_MI355X_EMW, "hk_ipm_solo_mw: expired hand-over wait, solve abandoned");
        return g_err;
    }
    for (int i = 0; i < 5 * iv[0]; i++) stat[i] = H[A.stat + i];
    // d_ip2_mpc_hard_tv without constraints solves into its workspace only (d_ip2_hard.c:282-291)
    const bool outputs = !(phase1_only && P->nbt == 0);
    for (int k = 0; outputs && k <= N; k++) {
        memcpy(ux[k], H + A.ux + k * V16, (P->st[k].nu + nx[k]) * sizeof(double));
        if (k < N) memcpy(pi[k], H + A.pi + k * V16, nx[k + 1] * sizeof(double));
        if (nb[k] + ng[k] > 0) {
            memcpy(lam[k], H + A.lam + k * V32, cvec_len(P, k) * sizeof(double));
            memcpy(t[k], H + A.t + k * V32, cvec_len(P, k) * sizeof(double));
        }
    }
    memcpy(double_work_memory, H + A.ws, ws_doubles(N) * sizeof(double));
    return iv[1];
}

}  // namespace

extern "C" int d_ip2_res_mpc_hard_tv(int* kk, int k_max, double mu0, double mu_tol, double alpha_min, int warm_start,
                                     double* stat, int N, int* nx, int* nu_N, int* nb, int** idxb, int* ng,
                                     double** pBAbt, double** pQ, double** pDCt, double** d, double** ux,
                                     int compute_mult, double** pi, double** lam, double** t,
                                     double* double_work_memory) {
    return ipm_entry(0, 0, kk, k_max, mu0, mu_tol, alpha_min, warm_start, stat, N, nx, nu_N, nb, idxb, ng, pBAbt, pQ,
                     pDCt, d, ux, compute_mult, pi, lam, t, double_work_memory, nullptr, nullptr, nullptr, nullptr);
}

extern "C" int d_ip2_res_mpc_hard_tv_single_newton_step(int* kk, int k_max, double mu0, double mu_tol,
                                                        double alpha_min, int warm_start, double* stat, int N,
                                                        int* nx, int* nu_N, int* nb, int** idxb, int* ng,
                                                        double** pBAbt, double** pQ, double** pDCt, double** d,
                                                        double** ux, int compute_mult, double** pi, double** lam,
                                                        double** t, double* double_work_memory, double** ux0,
                                                        double** pi0, double** lam0, double** t0) {
    return ipm_entry(1, 0, kk, k_max, mu0, mu_tol, alpha_min, warm_start, stat, N, nx, nu_N, nb, idxb, ng, pBAbt, pQ,
                     pDCt, d, ux, compute_mult, pi, lam, t, double_work_memory, ux0, pi0, lam0, t0);
}

extern "C" void d_kkt_solve_new_rhs_res_mpc_hard_tv(int N, int* nx, int* nu_N, int* nb, int** idxb, int* ng,
                                                    double** pBAbt, double** b, double** pQ, double** q,
                                                    double** pDCt, double** d, double** ux, int compute_mult,
                                                    double** pi, double** lam, double** t,
                                                    double* double_work_memory) {
    g_err = 0;
    if (wide_path(N, nx, nu_N, nb, idxb, ng)) {
        hk_wide_kkt_entry(0, N, nx, nu_N, nb, idxb, ng, pBAbt, b, pQ, q, pDCt, d, ux, compute_mult, pi, lam, t,
                          double_work_memory);
        return;
    }
    hpmpc_mi355x_plan* P = g_ctx.get_plan(N, nx, nu_N, nb, idxb, ng);
    if (!P) return;
    Arena A = arena(P, 1);
    if (!g_ctx.ensure(A.total)) return;
    double* H = g_ctx.host;
    stage_BAbt(P, H, A, pBAbt);
    stage_RSQ(P, H, A, pQ);
    stage_d(P, H, A, d);
    stage_DCt(P, H, A, pDCt);
    memcpy(H + A.ws, double_work_memory, ws_doubles(N) * sizeof(double));
    for (int k = 0; k <= N; k++) {
        memcpy(H + A.vq + k * V16, q[k], (P->st[k].nu + nx[k]) * sizeof(double));
        if (k < N) memcpy(H + A.vb + k * V16, b[k], nx[k + 1] * sizeof(double));
    }
    KArgs a = arena_args(P, A, g_ctx.dev);
    a.compute_mult = compute_mult;
    if (!up(A) || !run(K_KKT, a, "hk_kkt_new_rhs") || !down(A)) return;
    for (int k = 0; k <= N; k++) {
        memcpy(ux[k], H + A.ux + k * V16, (P->st[k].nu + nx[k]) * sizeof(double));
        if (k < N) memcpy(pi[k], H + A.pi + k * V16, nx[k + 1] * sizeof(double));
        if (nb[k] + ng[k] > 0) {
            memcpy(lam[k], H + A.lam + k * V32, cvec_len(P, k) * sizeof(double));
            memcpy(t[k], H + A.t + k * V32, cvec_len(P, k) * sizeof(double));
        }
    }
}

extern "C" void d_res_res_mpc_hard_tv(int N, int* nx, int* nu, int* nb, int** idxb, int* ng, double** hpBAbt,
                                      double** hb, double** hpQ, double** hq, double** hux, double** hpDCt,
                                      double** hd, double** hpi, double** hlam, double** ht, double* work,
                                      double** hrq, double** hrb, double** hrd, double** hrm, double* mu) {
    (void)work;
    g_err = 0;
    if (wide_path(N, nx, nu, nb, idxb, ng)) {
        hk_wide_res_entry(0, N, nx, nu, nb, idxb, ng, hpBAbt, hb, hpQ, hq, hux, hpDCt, hd, hpi, hlam, ht, hrq, hrb, hrd,
                          hrm, mu);
        return;
    }
    hpmpc_mi355x_plan* P = g_ctx.get_plan(N, nx, nu, nb, idxb, ng);
    if (!P) return;
    Arena A = arena(P, 1);
    if (!g_ctx.ensure(A.total)) return;
    double* H = g_ctx.host;
    stage_BAbt(P, H, A, hpBAbt);
    stage_RSQ(P, H, A, hpQ);
    stage_d(P, H, A, hd);
    stage_DCt(P, H, A, hpDCt);
    for (int k = 0; k <= N; k++) {
        const int nux = P->st[k].nu + nx[k];
        memcpy(H + A.vq + k * V16, hq[k], nux * sizeof(double));
        memcpy(H + A.ux + k * V16, hux[k], nux * sizeof(double));
        if (k < N) {
            memcpy(H + A.vb + k * V16, hb[k], nx[k + 1] * sizeof(double));
            memcpy(H + A.pi + k * V16, hpi[k], nx[k + 1] * sizeof(double));
        }
        if (nb[k] + ng[k] > 0) {
            memcpy(H + A.lam + k * V32, hlam[k], cvec_len(P, k) * sizeof(double));
            memcpy(H + A.t + k * V32, ht[k], cvec_len(P, k) * sizeof(double));
        }
    }
    KArgs a = arena_args(P, A, g_ctx.dev);
    H[A.ints + 2] = *mu;  // mu is left untouched when there are no constraints (d_res_ip_res_hard.c:309-313)
    if (!up(A) || !run(K_RES, a, "hk_res") || !down(A)) return;
    const size_t n1 = N + 1;
    const double* rq = H + A.ws;
    const double* rb = rq + n1 * V16;
    const double* rd = rb + n1 * V16;
    const double* rm = rd + n1 * V32;
    for (int k = 0; k <= N; k++) {
        const int nux = P->st[k].nu + nx[k];
        memcpy(hrq[k], rq + k * V16, nux * sizeof(double));
        if (k < N) memcpy(hrb[k], rb + k * V16, nx[k + 1] * sizeof(double));
        if (nb[k] + ng[k] > 0) {
            memcpy(hrd[k], rd + k * V32, cvec_len(P, k) * sizeof(double));
            memcpy(hrm[k], rm + k * V32, cvec_len(P, k) * sizeof(double));
        }
    }
    *mu = H[A.ints + 2];
}

// ------------------------------------------------------------------------------------------------
// The alternate IPM of mpc_solvers/d_ip2_hard.c (phase-1 Mehrotra loop alone), its KKT re-solve and the
// plain residuals of mpc_solvers/d_res_ip_hard.c, on the same kernels (KArgs.phase1_only / res_plain).
// ------------------------------------------------------------------------------------------------
extern "C" int d_ip2_mpc_hard_tv_work_space_size_bytes(int N, int* nx, int* nu, int* nb, int* ng) {
    return d_ip2_res_mpc_hard_tv_work_space_size_bytes(N, nx, nu, nb, ng);
}

extern "C" int d_ip2_mpc_hard_tv(int* kk, int k_max, double mu0, double mu_tol, double alpha_min, int warm_start,
                                 double* stat, int N, int* nx, int* nu_N, int* nb, int** idxb, int* ng,
                                 double** pBAbt, double** pQ, double** pDCt, double** d, double** ux,
                                 int compute_mult, double** pi, double** lam, double** t,
                                 double* double_work_memory) {
    return ipm_entry(0, 1, kk, k_max, mu0, mu_tol, alpha_min, warm_start, stat, N, nx, nu_N, nb, idxb, ng, pBAbt,
                     pQ, pDCt, d, ux, compute_mult, pi, lam, t, double_work_memory, nullptr, nullptr, nullptr,
                     nullptr);
}

extern "C" void d_kkt_solve_new_rhs_mpc_hard_tv(int N, int* nx, int* nu_N, int* nb, int** idxb, int* ng,
                                                double** pBAbt, double** r_A, double** pQ, double** r_H,
                                                double** pDCt, double** r_C, double** ux, int compute_mult,
                                                double** pi, double** lam, double** t, double* double_work_memory) {
    g_err = 0;
    if (wide_path(N, nx, nu_N, nb, idxb, ng)) {
        hk_wide_kkt_entry(1, N, nx, nu_N, nb, idxb, ng, pBAbt, r_A, pQ, r_H, pDCt, r_C, ux, compute_mult, pi, lam, t,
                          double_work_memory);
        return;
    }
    (void)pQ;  // the factor of the IPM's last iteration is in the workspace
    hpmpc_mi355x_plan* P = g_ctx.get_plan(N, nx, nu_N, nb, idxb, ng);
    if (!P) return;
    Arena A = arena(P, 1);
    if (!g_ctx.ensure(A.total)) return;
    double* H = g_ctx.host;
    stage_BAbt(P, H, A, pBAbt);
    stage_d(P, H, A, r_C);
    stage_DCt(P, H, A, pDCt);
    memcpy(H + A.ws, double_work_memory, ws_doubles(N) * sizeof(double));
    for (int k = 0; k <= N; k++) {
        memcpy(H + A.vq + k * V16, r_H[k], (P->st[k].nu + nx[k]) * sizeof(double));
        memcpy(H + A.ux + k * V16, ux[k], (P->st[k].nu + nx[k]) * sizeof(double));
        if (k < N) memcpy(H + A.vb + k * V16, r_A[k], nx[k + 1] * sizeof(double));
    }
    KArgs a = arena_args(P, A, g_ctx.dev);
    a.compute_mult = compute_mult;
    if (!up(A) || !run(K_KKT_P1, a, "hk_kkt_new_rhs_p1") || !down(A)) return;
    for (int k = 0; k <= N; k++) {
        memcpy(ux[k], H + A.ux + k * V16, (P->st[k].nu + nx[k]) * sizeof(double));
        if (k < N && compute_mult) memcpy(pi[k], H + A.pi + k * V16, nx[k + 1] * sizeof(double));
        if (nb[k] + ng[k] > 0) {
            memcpy(lam[k], H + A.lam + k * V32, cvec_len(P, k) * sizeof(double));
            memcpy(t[k], H + A.t + k * V32, cvec_len(P, k) * sizeof(double));
        }
    }
    // the persisted factor / workspace is left as the IPM wrote it, apart from qx and Pb (as the reference)
    memcpy(double_work_memory, H + A.ws, ws_doubles(N) * sizeof(double));
}

extern "C" void d_res_mpc_hard_tv(int N, int* nx, int* nu, int* nb, int** idxb, int* ng, double** hpBAbt,
                                  double** hb, double** hpQ, double** hq, double** hux, double** hpDCt, double** hd,
                                  double** hpi, double** hlam, double** ht, double** hrq, double** hrb, double** hrd,
                                  double* mu) {
    g_err = 0;
    if (wide_path(N, nx, nu, nb, idxb, ng)) {
        hk_wide_res_entry(1, N, nx, nu, nb, idxb, ng, hpBAbt, hb, hpQ, hq, hux, hpDCt, hd, hpi, hlam, ht, hrq, hrb, hrd,
                          nullptr, mu);
        return;
    }
    hpmpc_mi355x_plan* P = g_ctx.get_plan(N, nx, nu, nb, idxb, ng);
    if (!P) return;
    Arena A = arena(P, 1);
    if (!g_ctx.ensure(A.total)) return;
    double* H = g_ctx.host;
    stage_BAbt(P, H, A, hpBAbt);
    stage_RSQ(P, H, A, hpQ);
    stage_d(P, H, A, hd);
    stage_DCt(P, H, A, hpDCt);
    for (int k = 0; k <= N; k++) {
        const int nux = P->st[k].nu + nx[k];
        memcpy(H + A.vq + k * V16, hq[k], nux * sizeof(double));
        memcpy(H + A.ux + k * V16, hux[k], nux * sizeof(double));
        if (k < N) {
            memcpy(H + A.vb + k * V16, hb[k], nx[k + 1] * sizeof(double));
            memcpy(H + A.pi + k * V16, hpi[k], nx[k + 1] * sizeof(double));
        }
        if (nb[k] + ng[k] > 0) {
            memcpy(H + A.lam + k * V32, hlam[k], cvec_len(P, k) * sizeof(double));
            memcpy(H + A.t + k * V32, ht[k], cvec_len(P, k) * sizeof(double));
        }
    }
    KArgs a = arena_args(P, A, g_ctx.dev);
    a.res_plain = 1;
    if (!up(A) || !run(K_RES, a, "hk_res") || !down(A)) return;
    const size_t n1 = N + 1;
    const double* rq = H + A.ws;
    const double* rb = rq + n1 * V16;
    const double* rd = rb + n1 * V16;
    for (int k = 0; k <= N; k++) {
        const int nux = P->st[k].nu + nx[k];
        memcpy(hrq[k], rq + k * V16, nux * sizeof(double));
        if (k < N) memcpy(hrb[k], rb + k * V16, nx[k + 1] * sizeof(double));
        if (nb[k] + ng[k] > 0) memcpy(hrd[k], rd + k * V32, cvec_len(P, k) * sizeof(double));
    }
    *mu = H[A.ints + 2];
}

// ================================================================================================
// Soft-constraint IPM d_ip2_mpc_soft_tv (mpc_solvers/d_ip2_soft.c:42-547, include/mpc_solvers.h:69-70):
// the constraint passes of hk_soft.hip around the tile Riccati kernels, one host round trip (the exit
// flag) per iteration.  Limits (HPMPC_MI355X_EUNSUPPORTED, DESIGN.md soft constraints): ng = 0, nu[N] = 0,
// round_up(nb + ns, 4) <= 16 per stage, b_k read inside BAbt_k with the reference's stride
// (d_ip2_soft.c:172), and no soft-gradient write of the reference into a Zl its pass still reads.
// ================================================================================================
#include "hk_soft_args.h"

extern "C" int hk_soft_launch(int which, const SoftArgs* a, int count, hipStream_t stream);

namespace {

const char* soft_unsupported(int N, const int* nx, const int* nu, const int* ng) {
    if (N < 1 || nu[N] != 0) return "soft IPM: N >= 1 and nu[N] = 0 required";
    for (int k = 0; k <= N; k++)
        if (ng[k] != 0) return "soft IPM with general constraints (ng > 0)";
    for (int k = 0; k < N; k++) {
        const int nux = nu[k] + nx[k], nx1 = nx[k + 1];
        const long idx = (long)(nux / BS) * BS * rup(nx1, BS) + nux % BS + BS * (long)(nx1 > 0 ? nx1 - 1 : 0);
        if (nx1 > 0 && idx >= (long)rup(nux + 1, BS) * rup(nx1, NCL))
            return "soft IPM: the reference reads b_k outside BAbt_k here (stride round_up(nx,4), d_ip2_soft.c:172)";
    }
    return nullptr;
}

bool soft_launch(int which, const SoftArgs& s) {
    if (hk_soft_launch(which, &s, 1, g_ctx.stream)) {
        set_err(HPMPC_MI355X_EHIP, "hk_soft_pass launch failed");
        return false;
    }
    return true;
}

}  // namespace

extern "C" int d_ip2_mpc_soft_tv_work_space_size_bytes(int N, int* nx, int* nu, int* nb, int* ng, int* ns) {
    (void)N;
    (void)nx;
    (void)nu;
    (void)nb;
    (void)ng;
    (void)ns;
    return 64;  // iterate, factor and work vectors live on the device
}

extern "C" int d_ip2_mpc_soft_tv(int* kk, int k_max, double mu0, double mu_tol, double alpha_min, int warm_start,
                                 double* stat, int N, int* nx, int* nu, int* nb, int** idxb, int* ng, int* ns,
                                 double** pBAbt, double** pQ, double** Z, double** z, double** pDCt, double** d,
                                 double** ux, int compute_mult, double** pi, double** lam, double** t,
                                 double* double_work_memory) {
    (void)pDCt;
    (void)double_work_memory;
    g_err = 0;
    if (const char* why = soft_unsupported(N, nx, nu, ng)) {
        set_err(HPMPC_MI355X_EUNSUPPORTED, why);
        return g_err;
    }
    double mu_scal = 0.0;
    for (int k = 0; k <= N; k++) mu_scal += 2 * nb[k] + 2 * ng[k] + 4 * ns[k];
    if (mu_scal == 0.0) {  // the reference solves into its workspace and leaves every output untouched (:273-284)
        *kk = 0;
        return 0;
    }
    mu_scal = 1.0 / mu_scal;
    std::vector<int> nbs(N + 1);
    for (int k = 0; k <= N; k++) nbs[k] = nb[k] + ns[k];
    hpmpc_mi355x_plan* P = g_ctx.get_plan(N, nx, nu, nbs.data(), idxb, ng);
    if (!P) return g_err;
    // soft layout (doubles): per-stage constraint vectors, then the flat Qx / qx | Zl / zl block
    std::vector<SoftStage> ss(N + 1);
    long sC = 0, sD = 0, sZ = 0, F = 0;
    int padM = 0;
    for (int k = 0; k <= N; k++) {
        SoftStage& s = ss[k];
        memset(&s, 0, sizeof s);
        s.nu = P->st[k].nu;
        s.nx = nx[k];
        s.nx1 = k < N ? nx[k + 1] : 0;
        s.nb = nb[k];
        s.ns = ns[k];
        s.pnb = rup(nb[k], BS);
        s.pns = rup(ns[k], BS);
        s.oC = (int)sC;
        sC += 2 * s.pnb + 4 * s.pns;
        s.oD = (int)sD;
        sD += 2 * s.pnb + 2 * s.pns;
        s.oZ = (int)sZ;
        sZ += 2 * s.pns;
        s.oQ = (int)F;
        F += 2 * (s.pnb + s.pns);
        padM = std::max(padM, 2 * (s.pnb + s.pns));
    }
    for (int k = 0; k <= N; k++) {
        ss[k].oZl = (int)F;
        F += 4 * ss[k].pns;
    }
    const long sF = F + padM + 16;
    for (int k = 0; k <= N; k++) {  // where the soft gradient term goes (d_aux_ip_soft_lib4.c:557, :601)
        SoftStage& s = ss[k];
        const int pnbs = rup(s.nb + s.ns, BS);
        s.oS = s.oQ + s.pnb + s.pns + (s.nb > 0 ? pnbs + s.nb : s.nb);
        for (int i = 0; s.nb > 0 && i < s.ns; i++)
            for (int j = k; j <= N; j++)
                if (s.oS + i >= ss[j].oZl && s.oS + i < ss[j].oZl + 2 * ss[j].pns) {
                    set_err(HPMPC_MI355X_EUNSUPPORTED,
                            "soft IPM: the reference's soft-gradient write lands in a Zl read later in the same pass");
                    return g_err;
                }
    }
    Arena A = arena(P, 1);
    const size_t n1 = N + 1, v16 = n1 * V16;
    size_t o = A.total;
    auto take = [&](size_t n) {
        size_t r = o;
        o += (n + 7) / 8 * 8;
        return r;
    };
    const size_t oScal = take(4), oIst = take(4), oStat = take(5 * (size_t)(k_max > 0 ? k_max : 1) + 8),
                 oTab = take((sizeof(SoftStage) * n1 + 7) / 8), oIdx = take((n1 * 16 * sizeof(int) + 7) / 8),
                 oD = take(sD + 1), oZ = take(sZ + 1), oz = take(sZ + 1), oF = take(sF), oUx = take(v16),
                 oPi = take(v16);
    size_t oCv[6];
    for (int i = 0; i < 6; i++) oCv[i] = take(sC + 1);
    const size_t total = o;
    if (!g_ctx.ensure(total)) return g_err;
    double* H = g_ctx.host;
    stage_BAbt(P, H, A, pBAbt);
    stage_RSQ(P, H, A, pQ);
    memcpy(H + oTab, ss.data(), sizeof(SoftStage) * n1);
    int* hidx = reinterpret_cast<int*>(H + oIdx);
    for (int k = 0; k <= N; k++) {
        const SoftStage& s = ss[k];
        const int nux = s.nu + s.nx;
        for (int l = 0; l < nbs[k]; l++) hidx[k * 16 + l] = idxb[k][l];
        for (int l = 0; l < nux; l++) H[A.vq + k * V16 + l] = P4(pQ[k], rup(nux, NCL), nux, l);
        if (k < N) {  // b_k with the reference's stride round_up(nx_{k+1}, 4) (d_ip2_soft.c:172)
            const double* row = pBAbt[k] + (nux / BS) * BS * rup(s.nx1, BS) + nux % BS;
            for (int j = 0; j < s.nx1; j++) H[A.vb + k * V16 + j] = row[BS * j];
        }
        memcpy(H + oD + s.oD, d[k], (2 * s.pnb + 2 * s.pns) * sizeof(double));
        if (s.ns > 0) {
            memcpy(H + oZ + s.oZ, Z[k], 2 * s.pns * sizeof(double));
            memcpy(H + oz + s.oZ, z[k], 2 * s.pns * sizeof(double));
        }
        if (warm_start) memcpy(H + oUx + k * V16, ux[k], nux * sizeof(double));
    }
    double* D = g_ctx.dev;
    KArgs a = arena_args(P, A, D);
    a.use_box = 1;
    a.update_q = 1;
    a.update_b = 0;
    a.compute_pi = compute_mult;
    a.compute_Pb = 1;
    KArgs a2 = a;
    a2.compute_Pb = 0;
    SoftArgs s;
    memset(&s, 0, sizeof s);
    s.N = N;
    s.nprob = 1;
    s.k_max = k_max;
    s.warm_start = warm_start;
    s.nq = (N + 4) / 4;
    s.st = reinterpret_cast<const SoftStage*>(D + oTab);
    s.idxb = reinterpret_cast<const int*>(D + oIdx);
    s.d = D + oD;
    s.Z = D + oZ;
    s.z = D + oz;
    s.t = D + oCv[0];
    s.lam = D + oCv[1];
    s.dt = D + oCv[2];
    s.dlam = D + oCv[3];
    s.lamt = D + oCv[4];
    s.tinv = D + oCv[5];
    s.flat = D + oF;
    s.ux = D + oUx;
    s.pi = D + oPi;
    s.dux = D + A.ux;
    s.dpi = D + A.pi;
    s.vQx = D + A.vQx;
    s.vqx = D + A.vqx;
    s.mu0 = mu0;
    s.mu_tol = mu_tol;
    s.alpha_min = alpha_min;
    s.mu_scal = mu_scal;
    s.scal = D + oScal;
    s.ist = reinterpret_cast<int*>(D + oIst);
    s.stat = D + oStat;
    if (!hip_ok(hipMemcpyAsync(D, H, total * sizeof(double), hipMemcpyHostToDevice, g_ctx.stream), "H2D") ||
        !soft_launch(0, s))
        return g_err;
    const int* hist = reinterpret_cast<const int*>(H + oIst);
    for (int it = 0; it < k_max; it++) {
        if (!soft_launch(1, s) || !run(K_SV, a, "hk_ric_sv") || !soft_launch(2, s) || !run(K_TRS, a2, "hk_ric_trs") ||
            !soft_launch(3, s))
            return g_err;
        if (!hip_ok(hipMemcpyAsync(H + oIst, D + oIst, 4 * sizeof(int), hipMemcpyDeviceToHost, g_ctx.stream),
                    "D2H") ||
            !hip_ok(hipStreamSynchronize(g_ctx.stream), "sync"))
            return g_err;
        if (!hist[1]) break;
    }
    if (!hip_ok(hipMemcpyAsync(H, D, total * sizeof(double), hipMemcpyDeviceToHost, g_ctx.stream), "D2H") ||
        !hip_ok(hipStreamSynchronize(g_ctx.stream), "sync"))
        return g_err;
    *kk = hist[0];
    for (int i = 0; i < 5 * hist[0]; i++) stat[i] = H[oStat + i];
    for (int k = 0; k <= N; k++) {
        const SoftStage& st = ss[k];
        memcpy(ux[k], H + oUx + k * V16, (st.nu + st.nx) * sizeof(double));
        if (k < N) memcpy(pi[k], H + oPi + k * V16, st.nx1 * sizeof(double));
        const int nc = 2 * st.pnb + 4 * st.pns;
        if (nc > 0) {
            memcpy(lam[k], H + oCv[1] + st.oC, nc * sizeof(double));
            memcpy(t[k], H + oCv[0] + st.oC, nc * sizeof(double));
        }
    }
    return hist[2];
}

// ------------------------------------------------------------------------------------------------
// d_res_mpc_soft_tv (mpc_solvers/d_res_ip_soft.c:38-268, include/mpc_solvers.h:71): hk_soft_res on a copy of
// every array of the call.  The output vectors are uploaded first, so the entries the reference does not write
// (padding, and stage N's input rows of r_q, :199-200) come back as the caller left them.  General constraints
// are supported (the residual has no soft-gradient quirk); stage 0's pi_{-1} (nx_0 > 0) reads as zero.
// ------------------------------------------------------------------------------------------------
extern "C" int hk_soft_res_launch(const SoftResArgs* a, hipStream_t stream);

extern "C" void d_res_mpc_soft_tv(int N, int* nx, int* nu, int* nb, int** idxb, int* ng, int* ns, double** hpBAbt,
                                  double** hpQ, double** hq, double** hZ, double** hz, double** hux, double** hpDCt,
                                  double** hd, double** hpi, double** hlam, double** ht, double** hrq, double** hrb,
                                  double** hrd, double** hrz, double* mu) {
    g_err = 0;
    if (N < 0) {
        set_err(HPMPC_MI355X_EUNSUPPORTED, "d_res_mpc_soft_tv: N < 0");
        return;
    }
    std::vector<SoftResStage> st(N + 1);
    std::vector<int> ints;
    size_t o = 0;
    auto take = [&](size_t n) {
        size_t r = o;
        o += (n + 7) / 8 * 8;
        return (int)r;
    };
    for (int k = 0; k <= N; k++) {
        SoftResStage& s = st[k];
        s.nu = nu[k];
        s.nx = nx[k];
        s.nb = nb[k];
        s.ng = ng[k];
        s.ns = ns[k];
        s.nx1 = k < N ? nx[k + 1] : 0;
        s.nu1 = k < N ? nu[k + 1] : 0;
        s.pnb = rup(nb[k], BS);
        s.png = rup(ng[k], BS);
        s.pns = rup(ns[k], BS);
        const int nux = s.nu + s.nx, ncv = 2 * s.pnb + 2 * s.png + 4 * s.pns, nrd = 2 * s.pnb + 2 * s.png + 2 * s.pns;
        s.sdB = rup(s.nx1, NCL);
        s.sdQ = rup(nux, NCL);
        s.sdG = rup(ng[k], NCL);
        s.oB = k < N ? take((size_t)rup(nux + 1, BS) * s.sdB) : -1;
        s.oQ = take((size_t)rup(nux + 1, BS) * s.sdQ);
        s.oq = take(nux);
        s.oZ = take(2 * s.pns);
        s.oz = take(2 * s.pns);
        s.oux = take(nux);
        s.oG = ng[k] > 0 ? take((size_t)rup(nux, BS) * s.sdG) : -1;
        s.od = take(nrd);
        s.opi = k < N ? take(s.nx1) : -1;
        s.olam = take(ncv);
        s.ot = take(ncv);
        s.orq = take(nux);
        s.orb = k < N ? take(s.nx1) : -1;
        s.ord = take(nrd);
        s.orz = take(2 * s.pns);
        s.oI = (int)ints.size();
        // the soft constraints read idxb[k][nu_k + i] (:107), so the row is copied that far
        const int nI = std::max(nb[k], ns[k] > 0 ? nu[k] + ns[k] : 0);
        for (int j = 0; j < nI; j++) ints.push_back(idxb[k][j]);
    }
    for (int k = 0; k <= N; k++) {
        st[k].oux1 = k < N ? st[k + 1].oux : -1;
        st[k].opim1 = k > 0 ? st[k - 1].opi : -1;
    }
    const int omu = take(1);
    const size_t oSt = take((sizeof(SoftResStage) * (N + 1) + 7) / 8), oIdx = take((4 * ints.size() + 7) / 8 + 1);
    Arena A{};
    A.total = o;
    if (!g_ctx.ensure(A.total)) return;
    double* H = g_ctx.host;
    memset(H, 0, A.total * sizeof(double));
    auto cp = [&](int off, const double* src, size_t n) {
        if (off >= 0 && n > 0) memcpy(H + off, src, n * sizeof(double));
    };
    for (int k = 0; k <= N; k++) {
        const SoftResStage& s = st[k];
        const int nux = s.nu + s.nx, ncv = 2 * s.pnb + 2 * s.png + 4 * s.pns, nrd = 2 * s.pnb + 2 * s.png + 2 * s.pns;
        if (k < N) cp(s.oB, hpBAbt[k], (size_t)rup(nux + 1, BS) * s.sdB);
        cp(s.oQ, hpQ[k], (size_t)rup(nux + 1, BS) * s.sdQ);
        cp(s.oq, hq[k], nux);
        if (ns[k] > 0) {
            cp(s.oZ, hZ[k], 2 * s.pns);
            cp(s.oz, hz[k], 2 * s.pns);
            cp(s.orz, hrz[k], 2 * s.pns);
        }
        cp(s.oux, hux[k], nux);
        if (ng[k] > 0) cp(s.oG, hpDCt[k], (size_t)rup(nux, BS) * s.sdG);
        if (nrd > 0) {
            cp(s.od, hd[k], nrd);
            cp(s.ord, hrd[k], nrd);
            cp(s.olam, hlam[k], ncv);
            cp(s.ot, ht[k], ncv);
        }
        if (k < N) {
            cp(s.opi, hpi[k], s.nx1);
            cp(s.orb, hrb[k], s.nx1);
        }
        cp(s.orq, hrq[k], nux);
    }
    memcpy(H + oSt, st.data(), sizeof(SoftResStage) * (N + 1));
    if (!ints.empty()) memcpy(H + oIdx, ints.data(), 4 * ints.size());
    SoftResArgs a;
    a.N = N;
    a.st = reinterpret_cast<const SoftResStage*>(g_ctx.dev + oSt);
    a.idxb = reinterpret_cast<const int*>(g_ctx.dev + oIdx);
    a.buf = g_ctx.dev;
    a.omu = omu;
    if (!up(A)) return;
    if (hk_soft_res_launch(&a, g_ctx.stream)) {
        set_err(HPMPC_MI355X_EHIP, "hk_soft_res launch failed");
        return;
    }
    if (!down(A)) return;
    for (int k = 0; k <= N; k++) {
        const SoftResStage& s = st[k];
        const int nux = s.nu + s.nx, nrd = 2 * s.pnb + 2 * s.png + 2 * s.pns;
        memcpy(hrq[k], H + s.orq, nux * sizeof(double));
        if (k < N && s.nx1 > 0) memcpy(hrb[k], H + s.orb, s.nx1 * sizeof(double));
        if (nrd > 0) memcpy(hrd[k], H + s.ord, nrd * sizeof(double));
        if (ns[k] > 0) memcpy(hrz[k], H + s.orz, 2 * s.pns * sizeof(double));
    }
    *mu = H[omu];
}
