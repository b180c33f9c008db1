// hpmpc_capi_wide_ipm.cpp -- host side of the IPM on wide stages (hk_wide_ipm.hip).
//
// hpmpc_capi.cpp routes the reference-named IPM entry points here when a problem does not fit the 16-wide
// register tile (nu+nx > 16, round_up(nu,4)+nx > 16, or more than 16 box + general slots in a stage):
//   d_ip2_res_mpc_hard_tv, d_ip2_res_mpc_hard_tv_single_newton_step, d_kkt_solve_new_rhs_res_mpc_hard_tv,
//   d_res_res_mpc_hard_tv (mpc_solvers/d_ip2_res_hard.c, c99/d_res_ip_res_hard.c), and d_ip2_mpc_hard_tv,
//   d_kkt_solve_new_rhs_mpc_hard_tv, d_res_mpc_hard_tv (mpc_solvers/d_ip2_hard.c, d_res_ip_hard.c).
// Arguments are the reference's host lib4 buffers.  Each call stages them into a pinned arena, uploads it with
// one copy, runs ONE launch of hk_wide_ipm (the whole solve on the device) and copies the results back.
// `double_work_memory` holds this library's private work image (factor, IPM vectors, iterate backup), so the
// KKT re-solves find what the IPM left; its size is d_ip2_res_mpc_hard_tv_work_space_size_bytes.
#include "hk_wide_host.h"

extern "C" int hk_wide_ipm_launch(const WideIpmArgs* a, int count, int lds_doubles, hipStream_t stream);
namespace {
// the wide IPM's LDS: the Riccati carve, 8 doubles of reduction scratch, the DCt chunk-limit table ((N+1) x 8 ints
// and a flag, hk_wide_core.h)
inline int ipm_lds(const WLayout& L) { return L.lds + 8 + ((L.N + 1) * KC_STRIDE + 2) / 2; }
}  // namespace

namespace {

// The per-problem work image of the wide IPM (offsets in doubles).
struct WIpm {
    WLayout L;
    int oF, oDux, oDpi, oPb, oRq, oRb, oUb, oPib, oC[10];
    long long nIW;
    std::vector<WideCSlot> cs;
    std::vector<int> vbox;
    long long nbt = 0;  // sum(nb + ng)
};

WIpm make_ipm(int N, const int* nx, const int* nu, const int* nb, const int* ng) {
    WIpm W;
    W.L = make_layout(N, nx, nu, nb, ng);
    const WLayout& L = W.L;
    long long o = 0;
    auto take = [&](long long n) {
        const long long r = o;
        o += (n + 7) / 8 * 8;
        return (int)r;
    };
    W.oF = take(L.nL);
    W.oDux = take(L.nU);
    W.oDpi = take(L.nP);
    W.oPb = take(L.nP);
    W.oRq = take(L.nU);
    W.oRb = take(L.nP);
    W.oUb = take(L.nU);
    W.oPib = take(L.nP);
    for (int i = 0; i < 10; i++) W.oC[i] = take(L.nD);
    W.nIW = o;
    for (int k = 0; k <= N; k++) W.nbt += nb[k] + ng[k];
    return W;
}

// constraint slots and the variable -> box map (needs idxb)
void fill_slots(WIpm& W, int N, int** idxb) {
    const WLayout& L = W.L;
    W.cs.clear();
    W.vbox.assign(L.nU, -1);
    for (int k = 0; k <= N; k++) {
        const WideStage& s = L.st[k];
        const int png = rup(s.ng, BS);
        for (int l = 0; l < s.nb; l++) {
            WideCSlot c;
            c.lo = s.oD + l;
            c.up = s.oD + s.pnb + l;
            c.q = s.oD + l;
            c.var = s.oU + idxb[k][l];
            c.g = 0;
            W.cs.push_back(c);
            W.vbox[s.oU + idxb[k][l]] = c.lo;
        }
        for (int g = 0; g < s.ng; g++) {
            WideCSlot c;
            c.lo = s.oD + 2 * s.pnb + g;
            c.up = s.oD + 2 * s.pnb + png + g;
            c.q = s.oD + s.pnb + g;
            c.var = -1 - k;
            c.g = g;
            W.cs.push_back(c);
        }
    }
}

// sizes the wide IPM serves: any nb <= nu+nx with distinct indices, any ng, stage tiles within the kernel limits
bool ipm_check(const WIpm& W, int N, const int* nx, const int* nu, const int* nb, int* const* idxb, const int* ng) {
    if (N < 1) {
        hk_set_error(HPMPC_MI355X_EUNSUPPORTED, "N must be >= 1");
        return false;
    }
    for (int k = 0; k <= N; k++) {
        const int nux = (k < N ? nu[k] : 0) + nx[k];
        if (nb[k] < 0 || nb[k] > nux || ng[k] < 0 || nx[k] < 0 || (k < N && nu[k] < 0)) {
            hk_set_error(HPMPC_MI355X_EUNSUPPORTED, "negative size or nb[k] > nu[k]+nx[k]");
            return false;
        }
        if (idxb) {
            std::vector<char> seen(nux > 0 ? nux : 1, 0);
            for (int l = 0; l < nb[k]; l++) {
                const int v = idxb[k][l];
                if (v < 0 || v >= nux || seen[v]) {
                    hk_set_error(HPMPC_MI355X_EUNSUPPORTED, "idxb[k] must hold distinct variable indices in [0, nu[k]+nx[k])");
                    return false;
                }
                seen[v] = 1;
            }
        }
    }
    if (!W.L.fits || ipm_lds(W.L) > LDS_MAX_DOUBLES) {
        hk_set_error(HPMPC_MI355X_EUNSUPPORTED, "wide stage beyond the kernel's tile limits (64 KiB LDS, nu+nx < 128, "
                                                "nx <= 64)");
        return false;
    }
    return true;
}

// Device arena of one call (byte offsets) and the argument block.
struct Stage {
    size_t oSt, oCs, oVb, oI, oB, oR, oG, oD, oU, oP, oLam, oT, ovb, ovq, oIW, oStat, oCtl, total;
};

Stage carve(const WIpm& W, int N, int k_max) {
    const WLayout& L = W.L;
    Carve c;
    Stage S;
    S.oSt = c.take(sizeof(WideStage) * (N + 1));
    S.oCs = c.take(sizeof(WideCSlot) * (W.cs.size() + 1));
    S.oVb = c.take(sizeof(int) * L.nU);
    S.oI = c.take(sizeof(int) * L.nI);
    S.oB = c.take(8 * L.nB);
    S.oR = c.take(8 * L.nR);
    S.oG = c.take(8 * L.nG);
    S.oD = c.take(8 * L.nD);
    S.oU = c.take(8 * L.nU);
    S.oP = c.take(8 * L.nP);
    S.oLam = c.take(8 * L.nD);
    S.oT = c.take(8 * L.nD);
    S.ovb = c.take(8 * L.nP);
    S.ovq = c.take(8 * L.nU);
    S.oIW = c.take(8 * W.nIW);
    S.oStat = c.take(8 * (5 * (size_t)(k_max > 0 ? k_max : 1) + 8));
    S.oCtl = c.take(64);
    S.total = c.o;
    return S;
}

// stage the problem data (lib4 blocks, possibly aliased stage pointers) and the tables
void stage_common(const WIpm& W, const Stage& S, char* H, int N, int** idxb, double** pBAbt, double** pQ,
                  double** pDCt) {
    const WLayout& L = W.L;
    memcpy(H + S.oSt, L.st.data(), sizeof(WideStage) * (N + 1));
    if (!W.cs.empty()) memcpy(H + S.oCs, W.cs.data(), sizeof(WideCSlot) * W.cs.size());
    memcpy(H + S.oVb, W.vbox.data(), sizeof(int) * L.nU);
    int* HI = reinterpret_cast<int*>(H + S.oI);
    double* HB = reinterpret_cast<double*>(H + S.oB);
    double* HR = reinterpret_cast<double*>(H + S.oR);
    double* HG = reinterpret_cast<double*>(H + S.oG);
    for (int k = 0; k <= N; k++) {
        const WideStage& s = L.st[k];
        const int nux = s.nu + s.nx;
        memcpy(HR + s.oR, pQ[k], (size_t)rup(nux + 1, BS) * s.sdR * sizeof(double));
        if (k < N) memcpy(HB + s.oB, pBAbt[k], (size_t)rup(nux + 1, BS) * s.sdB * sizeof(double));
        if (s.ng > 0) memcpy(HG + s.oG, pDCt[k], (size_t)rup(nux, BS) * s.sdG * sizeof(double));
        if (s.nb > 0) memcpy(HI + s.oI, idxb[k], s.nb * sizeof(int));
    }
}

void cvec_in(const WIpm& W, const Stage& S, size_t off, char* H, int N, double** v) {
    if (!v) return;
    double* Hv = reinterpret_cast<double*>(H + off);
    for (int k = 0; k <= N; k++) {
        const WideStage& s = W.L.st[k];
        const int n = 2 * s.pnb + 2 * rup(s.ng, BS);
        if (s.nb + s.ng > 0) memcpy(Hv + s.oD, v[k], n * sizeof(double));
    }
}
void cvec_out(const WIpm& W, const double* Hv, int N, double** v) {
    for (int k = 0; k <= N; k++) {
        const WideStage& s = W.L.st[k];
        const int n = 2 * s.pnb + 2 * rup(s.ng, BS);
        if (s.nb + s.ng > 0) memcpy(v[k], Hv + s.oD, n * sizeof(double));
    }
}
void uvec_in(const WIpm& W, double* Hv, int N, double** v) {
    for (int k = 0; k <= N; k++) memcpy(Hv + W.L.st[k].oU, v[k], (W.L.st[k].nu + W.L.st[k].nx) * sizeof(double));
}
void pvec_in(const WIpm& W, double* Hv, int N, double** v) {
    for (int k = 0; k < N; k++) memcpy(Hv + W.L.st[k].oP, v[k], W.L.st[k].nx1 * sizeof(double));
}

void fill_args(const WIpm& W, const Stage& S, char* D, int N, WideIpmArgs& a) {
    const WLayout& L = W.L;
    memset(&a, 0, sizeof a);
    a.w.N = N;
    a.w.nprob = 1;
    a.w.st = reinterpret_cast<const WideStage*>(D + S.oSt);
    a.w.BAbt = reinterpret_cast<const double*>(D + S.oB);
    a.w.RSQ = reinterpret_cast<const double*>(D + S.oR);
    a.w.DCt = reinterpret_cast<const double*>(D + S.oG);
    a.w.idxb = reinterpret_cast<const int*>(D + S.oI);
    a.w.offW = L.offW;
    a.w.offX = L.offX;
    a.w.offV = L.offV;
    a.w.offST = L.offST;
    a.w.ldW = L.ldW;
    a.w.ldX = L.ldX;
    a.mu_scal = W.nbt ? 1.0 / (2.0 * (double)W.nbt) : 0.0;
    a.nbt2 = 2.0 * (double)W.nbt;
    a.ncs = (int)W.cs.size();
    a.cs = reinterpret_cast<const WideCSlot*>(D + S.oCs);
    a.vbox = reinterpret_cast<const int*>(D + S.oVb);
    a.nU = (int)L.nU;
    a.nP = (int)L.nP;
    a.d = reinterpret_cast<const double*>(D + S.oD);
    a.ux = reinterpret_cast<double*>(D + S.oU);
    a.pi = reinterpret_cast<double*>(D + S.oP);
    a.lam = reinterpret_cast<double*>(D + S.oLam);
    a.t = reinterpret_cast<double*>(D + S.oT);
    a.iw = reinterpret_cast<double*>(D + S.oIW);
    a.oF = W.oF;
    a.oDux = W.oDux;
    a.oDpi = W.oDpi;
    a.oPb = W.oPb;
    a.oRq = W.oRq;
    a.oRb = W.oRb;
    a.oUb = W.oUb;
    a.oPib = W.oPib;
    int* oc[10] = {&a.oDlam, &a.oDt, &a.oTinv, &a.oLamt, &a.oRd, &a.oRm, &a.oTb, &a.oLb, &a.oQx, &a.oqx};
    for (int i = 0; i < 10; i++) *oc[i] = W.oC[i];
    a.stat = reinterpret_cast<double*>(D + S.oStat);
    a.kk = reinterpret_cast<int*>(D + S.oCtl);
    a.ret = a.kk + 1;
    a.mu = reinterpret_cast<double*>(D + S.oCtl + 8);
    a.offR = L.lds;
    a.offKC = L.lds + 8;
}

bool run(const WIpm& W, const Stage& S, const WideIpmArgs& a) {
    if (!g_w.up(S.total)) return false;
    const int e = hk_wide_ipm_launch(&a, 1, ipm_lds(W.L), g_w.stream);
    if (e) {
        char msg[96];
        snprintf(msg, sizeof msg, "hk_wide_ipm launch %s (%d)", e == -2 ? "refused: scratch / LDS beyond the limits" : "failed", e);
        hk_set_error(e == -2 ? HPMPC_MI355X_EUNSUPPORTED : HPMPC_MI355X_EHIP, msg);
        return false;
    }
    return g_w.down(S.total);
}

}  // namespace

// bytes of the wide IPM's work image for these sizes (hpmpc_capi.cpp reports the larger of this and the tile
// path's image as d_ip2_res_mpc_hard_tv_work_space_size_bytes)
extern "C" long long hk_wide_ipm_bytes(int N, const int* nx, const int* nu, const int* nb, const int* ng) {
    return make_ipm(N, nx, nu, nb, ng).nIW * 8;
}

// d_ip2_res_mpc_hard_tv (mode WI_IPM_RES), its single-Newton variant (WI_NEWTON) and d_ip2_mpc_hard_tv
// (WI_IPM_P1) on wide stages.
extern "C" int hk_wide_ipm_entry(int mode, int* kk, int k_max, double mu0, double mu_tol, double alpha_min,
                                 int warm_start, double* stat, int N, int* nx, int* nu_N, int* nb, int** idxb, int* ng,
                                 double** pBAbt, double** pQ, double** pDCt, double** d, double** ux,
                                 int compute_mult, double** pi, double** lam, double** t, double* work, double** ux0,
                                 double** pi0, double** lam0, double** t0) {
    hk_set_error(0, nullptr);
    std::vector<int> nu(nu_N, nu_N + N + 1);
    nu[N] = 0;
    WIpm W = make_ipm(N, nx, nu.data(), nb, ng);
    if (!ipm_check(W, N, nx, nu.data(), nb, idxb, ng)) return HPMPC_MI355X_EUNSUPPORTED;
    if (mode == WI_NEWTON) {
        for (int k = 0; k <= N; k++)
            if (ng[k] > 0) {  // the reference stops here too (d_aux_ip_hard_lib4.c:197-208)
                hk_set_error(HPMPC_MI355X_EUNSUPPORTED, "single Newton step with general constraints");
                return HPMPC_MI355X_EUNSUPPORTED;
            }
    }
    fill_slots(W, N, idxb);
    const Stage S = carve(W, N, k_max);
    if (!g_w.ensure(S.total)) return HPMPC_MI355X_EHIP;
    char* H = g_w.host;
    stage_common(W, S, H, N, idxb, pBAbt, pQ, pDCt);
    cvec_in(W, S, S.oD, H, N, d);
    double* HU = reinterpret_cast<double*>(H + S.oU);
    double* HP = reinterpret_cast<double*>(H + S.oP);
    if (mode == WI_NEWTON) {  // start iterate; lam0 / t0 as [lower (nb) | upper (nb)] (d_aux_ip_hard_lib4.c:153-213)
        uvec_in(W, HU, N, ux0);
        pvec_in(W, HP, N, pi0);
        double* HL = reinterpret_cast<double*>(H + S.oLam);
        double* HT = reinterpret_cast<double*>(H + S.oT);
        for (int k = 0; k <= N; k++) {
            const WideStage& s = W.L.st[k];
            for (int l = 0; l < nb[k]; l++) {
                HL[s.oD + l] = lam0[k][l];
                HL[s.oD + s.pnb + l] = lam0[k][nb[k] + l];
                HT[s.oD + l] = t0[k][l];
                HT[s.oD + s.pnb + l] = t0[k][nb[k] + l];
            }
        }
    } else if (warm_start) {
        uvec_in(W, HU, N, ux);
    }
    WideIpmArgs a;
    fill_args(W, S, g_w.dev, N, a);
    a.mode = mode;
    a.k_max = k_max;
    a.warm_start = warm_start;
    a.compute_mult = compute_mult;
    a.mu0 = mu0;
    a.mu_tol = mu_tol;
    a.alpha_min = alpha_min;
    if (!run(W, S, a)) return HPMPC_MI355X_EHIP;
    const int* iv = reinterpret_cast<const int*>(H + S.oCtl);
    *kk = iv[0];
    const double* Hs = reinterpret_cast<const double*>(H + S.oStat);
    for (int i = 0; i < 5 * iv[0]; i++) stat[i] = Hs[i];
    // d_ip2_mpc_hard_tv without constraints solves into its workspace only (d_ip2_hard.c:282-291)
    const bool outputs = !(mode == WI_IPM_P1 && W.nbt == 0);
    if (outputs) {
        for (int k = 0; k <= N; k++) {
            memcpy(ux[k], HU + W.L.st[k].oU, (W.L.st[k].nu + nx[k]) * sizeof(double));
            if (k < N) memcpy(pi[k], HP + W.L.st[k].oP, nx[k + 1] * sizeof(double));
        }
        cvec_out(W, reinterpret_cast<const double*>(H + S.oLam), N, lam);
        cvec_out(W, reinterpret_cast<const double*>(H + S.oT), N, t);
    }
    memcpy(work, H + S.oIW, W.nIW * sizeof(double));
    return iv[1];
}

// d_kkt_solve_new_rhs_res_mpc_hard_tv (p1 = 0: b / q / d) and d_kkt_solve_new_rhs_mpc_hard_tv (p1 = 1:
// r_A / r_H / r_C) over the work image the IPM left.
extern "C" void hk_wide_kkt_entry(int p1, int N, int* nx, int* nu_N, int* nb, int** idxb, int* ng, double** pBAbt,
                                  double** b, double** pQ, double** q, double** pDCt, double** d, double** ux,
                                  int compute_mult, double** pi, double** lam, double** t, double* work) {
    hk_set_error(0, nullptr);
    std::vector<int> nu(nu_N, nu_N + N + 1);
    nu[N] = 0;
    WIpm W = make_ipm(N, nx, nu.data(), nb, ng);
    if (!ipm_check(W, N, nx, nu.data(), nb, idxb, ng)) return;
    fill_slots(W, N, idxb);
    const Stage S = carve(W, N, 1);
    if (!g_w.ensure(S.total)) return;
    char* H = g_w.host;
    stage_common(W, S, H, N, idxb, pBAbt, pQ, pDCt);
    cvec_in(W, S, S.oD, H, N, d);
    uvec_in(W, reinterpret_cast<double*>(H + S.ovq), N, q);
    pvec_in(W, reinterpret_cast<double*>(H + S.ovb), N, b);
    memcpy(H + S.oIW, work, W.nIW * sizeof(double));
    WideIpmArgs a;
    fill_args(W, S, g_w.dev, N, a);
    a.mode = p1 ? WI_KKT_P1 : WI_KKT_RES;
    a.compute_mult = compute_mult;
    a.vb = reinterpret_cast<const double*>(g_w.dev + S.ovb);
    a.vq = reinterpret_cast<const double*>(g_w.dev + S.ovq);
    if (!run(W, S, a)) return;
    const double* HU = reinterpret_cast<const double*>(H + S.oU);
    const double* HP = reinterpret_cast<const double*>(H + S.oP);
    for (int k = 0; k <= N; k++) {
        memcpy(ux[k], HU + W.L.st[k].oU, (W.L.st[k].nu + nx[k]) * sizeof(double));
        if (k < N && (compute_mult || !p1)) memcpy(pi[k], HP + W.L.st[k].oP, nx[k + 1] * sizeof(double));
    }
    cvec_out(W, reinterpret_cast<const double*>(H + S.oLam), N, lam);
    cvec_out(W, reinterpret_cast<const double*>(H + S.oT), N, t);
    if (p1) memcpy(work, H + S.oIW, W.nIW * sizeof(double));  // qx / Pb of the re-solve, as the reference leaves them
}

// d_res_res_mpc_hard_tv (plain = 0: r_q, r_b, r_d, r_m, mu) and d_res_mpc_hard_tv (plain = 1: r_q, r_b, r_d, mu).
extern "C" void hk_wide_res_entry(int plain, int N, int* nx, int* nu, int* nb, int** idxb, int* ng, double** hpBAbt,
                                  double** hb, double** hpQ, double** hq, double** hux, double** hpDCt, double** hd,
                                  double** hpi, double** hlam, double** ht, double** hrq, double** hrb, double** hrd,
                                  double** hrm, double* mu) {
    hk_set_error(0, nullptr);
    WIpm W = make_ipm(N, nx, nu, nb, ng);
    if (!ipm_check(W, N, nx, nu, nb, idxb, ng)) return;
    fill_slots(W, N, idxb);
    const Stage S = carve(W, N, 1);
    if (!g_w.ensure(S.total)) return;
    char* H = g_w.host;
    stage_common(W, S, H, N, idxb, hpBAbt, hpQ, hpDCt);
    cvec_in(W, S, S.oD, H, N, hd);
    cvec_in(W, S, S.oLam, H, N, hlam);
    cvec_in(W, S, S.oT, H, N, ht);
    uvec_in(W, reinterpret_cast<double*>(H + S.oU), N, hux);
    pvec_in(W, reinterpret_cast<double*>(H + S.oP), N, hpi);
    uvec_in(W, reinterpret_cast<double*>(H + S.ovq), N, hq);
    pvec_in(W, reinterpret_cast<double*>(H + S.ovb), N, hb);
    reinterpret_cast<double*>(H + S.oCtl + 8)[0] = *mu;  // unchanged without constraints (d_res_ip_res_hard.c:309-313)
    WideIpmArgs a;
    fill_args(W, S, g_w.dev, N, a);
    a.mode = plain ? WI_RES_PLAIN : WI_RES;
    a.vb = reinterpret_cast<const double*>(g_w.dev + S.ovb);
    a.vq = reinterpret_cast<const double*>(g_w.dev + S.ovq);
    if (!run(W, S, a)) return;
    const double* IW = reinterpret_cast<const double*>(H + S.oIW);
    for (int k = 0; k <= N; k++) {
        const WideStage& s = W.L.st[k];
        memcpy(hrq[k], IW + W.oRq + s.oU, (s.nu + s.nx) * sizeof(double));
        if (k < N) memcpy(hrb[k], IW + W.oRb + s.oP, s.nx1 * sizeof(double));
    }
    cvec_out(W, IW + W.oC[4], N, hrd);
    if (!plain) cvec_out(W, IW + W.oC[5], N, hrm);
    *mu = reinterpret_cast<const double*>(H + S.oCtl + 8)[0];
}

// ------------------------------------------------------------------------------------------------
// Batched device API of the wide-stage IPM (include/hpmpc_mi355x.h, Part 2): many problems that share the
// stage sizes and box index sets, data resident in HBM, one workgroup per problem, one launch per batch.
// ------------------------------------------------------------------------------------------------
struct hpmpc_mi355x_wide_plan {
    WIpm W;
    int N = 0;
    WideStage* d_st = nullptr;
    WideCSlot* d_cs = nullptr;
    int* d_vbox = nullptr;
    int* d_idxb = nullptr;
};

extern "C" void hpmpc_mi355x_wide_plan_destroy(hpmpc_mi355x_wide_plan* q) {
    if (!q) return;
    if (q->d_st) (void)hipFree(q->d_st);
    if (q->d_cs) (void)hipFree(q->d_cs);
    if (q->d_vbox) (void)hipFree(q->d_vbox);
    if (q->d_idxb) (void)hipFree(q->d_idxb);
    delete q;
}

extern "C" hpmpc_mi355x_wide_plan* hpmpc_mi355x_wide_plan_create(int N, const int* nx, const int* nu_in, const int* nb,
                                                                 const int* const* idxb, const int* ng) {
    hk_set_error(0, nullptr);
    std::vector<int> nu(nu_in, nu_in + N + 1);
    nu[N] = 0;
    auto* q = new hpmpc_mi355x_wide_plan();
    q->N = N;
    q->W = make_ipm(N, nx, nu.data(), nb, ng);
    int** ib = const_cast<int**>(idxb);
    if (!ipm_check(q->W, N, nx, nu.data(), nb, ib, ng)) {
        delete q;
        return nullptr;
    }
    fill_slots(q->W, N, ib);
    const WLayout& L = q->W.L;
    std::vector<int> hidx(L.nI, 0);
    for (int k = 0; k <= N; k++)
        for (int l = 0; l < nb[k]; l++) hidx[L.st[k].oI + l] = idxb[k][l];
    const size_t ncs = q->W.cs.size() + 1;
    bool ok = hip_ok(hipMalloc((void**)&q->d_st, sizeof(WideStage) * (N + 1)), "wide plan") &&
              hip_ok(hipMalloc((void**)&q->d_cs, sizeof(WideCSlot) * ncs), "wide plan") &&
              hip_ok(hipMalloc((void**)&q->d_vbox, sizeof(int) * L.nU), "wide plan") &&
              hip_ok(hipMalloc((void**)&q->d_idxb, sizeof(int) * L.nI), "wide plan") &&
              hip_ok(hipMemcpy(q->d_st, L.st.data(), sizeof(WideStage) * (N + 1), hipMemcpyHostToDevice), "plan") &&
              (q->W.cs.empty() || hip_ok(hipMemcpy(q->d_cs, q->W.cs.data(), sizeof(WideCSlot) * q->W.cs.size(),
                                                   hipMemcpyHostToDevice), "plan")) &&
              hip_ok(hipMemcpy(q->d_vbox, q->W.vbox.data(), sizeof(int) * L.nU, hipMemcpyHostToDevice), "plan") &&
              hip_ok(hipMemcpy(q->d_idxb, hidx.data(), sizeof(int) * L.nI, hipMemcpyHostToDevice), "plan");
    if (!ok) {
        hpmpc_mi355x_wide_plan_destroy(q);
        return nullptr;
    }
    return q;
}

// out[8]: doubles per problem of BAbt, RSQrq, DCt, d (= lam = t), ux, pi, the work image; N
extern "C" int hpmpc_mi355x_wide_sizes(const hpmpc_mi355x_wide_plan* q, long long* out) {
    if (!q) return HPMPC_MI355X_EUNSUPPORTED;
    const WLayout& L = q->W.L;
    const long long v[8] = {L.nB, L.nR, L.nG, L.nD, L.nU, L.nP, q->W.nIW, q->N};
    memcpy(out, v, sizeof v);
    return 0;
}

// out[6*(N+1)]: oB, oR, oG, oD, oU, oP of every stage (doubles inside one problem's arrays)
extern "C" int hpmpc_mi355x_wide_offsets(const hpmpc_mi355x_wide_plan* q, long long* out) {
    if (!q) return HPMPC_MI355X_EUNSUPPORTED;
    for (int k = 0; k <= q->N; k++) {
        const WideStage& s = q->W.L.st[k];
        const long long v[6] = {s.oB, s.oR, s.oG, s.oD, s.oU, s.oP};
        memcpy(out + 6 * k, v, sizeof v);
    }
    return 0;
}

// d_ip2_res_mpc_hard_tv on problems [p0, p0 + count) of a device-resident batch (problem-major arrays with the
// per-problem sizes of hpmpc_mi355x_wide_sizes); kk / ret per problem, stat 5 * k_max per problem; `work` holds
// each problem's work image (the factor and iterate backup of its last iteration).  Asynchronous on `stream`.
extern "C" int hpmpc_mi355x_wide_ipm_batch(const hpmpc_mi355x_wide_plan* q, int nprob, int p0, int count,
                                           const double* BAbt, const double* RSQrq, const double* DCt, const double* d,
                                           double* ux, double* pi, double* lam, double* t, double* work, int k_max,
                                           double mu0, double mu_tol, double alpha_min, int warm_start,
                                           int compute_mult, int* kk, int* ret, double* stat, void* stream) {
    hk_set_error(0, nullptr);
    if (!q || nprob <= 0 || p0 < 0 || count < 0 || p0 + count > nprob || k_max < 0)
        return HPMPC_MI355X_EUNSUPPORTED;
    const WIpm& W = q->W;
    const WLayout& L = W.L;
    // every array the kernel dereferences unconditionally (DCt only when a stage has general constraints; stat is
    // nullable): a null one is a caller error, reported instead of faulting on the device
    if (!BAbt || !RSQrq || !d || !ux || !pi || !lam || !t || !work || !kk || !ret || (L.any_ng && !DCt)) {
        hk_set_error(HPMPC_MI355X_EUNSUPPORTED, "hpmpc_mi355x_wide_ipm_batch: null array");
        return HPMPC_MI355X_EUNSUPPORTED;
    }
    WideIpmArgs a;
    memset(&a, 0, sizeof a);
    a.w.N = q->N;
    a.w.nprob = nprob;
    a.w.p0 = p0;
    a.w.st = q->d_st;
    a.w.BAbt = BAbt;
    a.w.sB = L.nB;
    a.w.RSQ = RSQrq;
    a.w.sR = L.nR;
    a.w.DCt = DCt;
    a.w.sG = L.nG;
    a.w.idxb = q->d_idxb;
    a.w.offW = L.offW;
    a.w.offX = L.offX;
    a.w.offV = L.offV;
    a.w.offST = L.offST;
    a.w.ldW = L.ldW;
    a.w.ldX = L.ldX;
    a.w.sU = L.nU;
    a.w.sP = L.nP;
    a.mode = WI_IPM_RES;
    a.k_max = k_max;
    a.warm_start = warm_start;
    a.compute_mult = compute_mult;
    a.mu0 = mu0;
    a.mu_tol = mu_tol;
    a.alpha_min = alpha_min;
    a.mu_scal = W.nbt ? 1.0 / (2.0 * (double)W.nbt) : 0.0;
    a.nbt2 = 2.0 * (double)W.nbt;
    a.ncs = (int)W.cs.size();
    a.cs = q->d_cs;
    a.vbox = q->d_vbox;
    a.nU = (int)L.nU;
    a.nP = (int)L.nP;
    a.d = d;
    a.ux = ux;
    a.pi = pi;
    a.lam = lam;
    a.t = t;
    a.sC = L.nD;
    a.iw = work;
    a.sI = W.nIW;
    a.oF = W.oF;
    a.oDux = W.oDux;
    a.oDpi = W.oDpi;
    a.oPb = W.oPb;
    a.oRq = W.oRq;
    a.oRb = W.oRb;
    a.oUb = W.oUb;
    a.oPib = W.oPib;
    int* oc[10] = {&a.oDlam, &a.oDt, &a.oTinv, &a.oLamt, &a.oRd, &a.oRm, &a.oTb, &a.oLb, &a.oQx, &a.oqx};
    for (int i = 0; i < 10; i++) *oc[i] = W.oC[i];
    a.stat = stat;
    a.sS = 5LL * (k_max > 0 ? k_max : 1);
    a.kk = kk;
    a.ret = ret;
    a.mu = nullptr;
    a.offR = L.lds;
    a.offKC = L.lds + 8;
    if (count == 0) return 0;
    const int e = hk_wide_ipm_launch(&a, count, ipm_lds(L), (hipStream_t)stream);
    if (e) {
        char msg[96];
        snprintf(msg, sizeof msg, "hk_wide_ipm launch %s (%d)", e == -2 ? "refused: scratch / LDS beyond the limits" : "failed", e);
        const int code = e == -2 ? HPMPC_MI355X_EUNSUPPORTED : HPMPC_MI355X_EHIP;
        hk_set_error(code, msg);
        return code;
    }
    return 0;
}
