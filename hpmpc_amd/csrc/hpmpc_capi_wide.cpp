// hpmpc_capi_wide.cpp -- host side of the wide-stage path (hk_wide.hip):
//   * d_back_ric_rec_sv_tv_res for stages beyond the 16-wide register tile (routed here by hpmpc_capi.cpp);
//   * partial condensing, the §8f #1 row: d_part_cond_compute_problem_size / _work_space_size_bytes /
//     _memory_space_size_bytes / d_part_cond / d_part_expand_work_space_size_bytes / d_part_expand_solution
//     (lqcp_solvers/d_part_cond.c:694-1308) with the reference prototypes, on host lib4 buffers;
//   * the batched device API of the same pipeline (hpmpc_mi355x_pcond_*), data resident in HBM.
// Every computation runs on the GPU; the host only packs stage tables and copies buffers.
#include "hk_wide_host.h"


// ------------------------------------------------------------------------------------------------
// d_back_ric_rec_sv_tv_res on wide stages (called by hpmpc_capi.cpp when the tile path does not fit).
// ------------------------------------------------------------------------------------------------
extern "C" long long hk_wide_factor_bytes(int N, const int* nx, const int* nu) {
    long long s = 0;
    for (int k = 0; k <= N; k++) {
        const int nux = (k < N ? nu[k] : 0) + nx[k];
        s += poff(nux, nux + 1) + nux;
        s = (s + 7) / 8 * 8;
    }
    return s * 8;
}

namespace {
// General constraints of the drop-in Riccati calls: DCt_k and the general halves of Qx / qx ([box (pnb) |
// general (png)]) staged for the device (DCt diag(Qx_g) DCt' and DCt qx_g are added there, d_back_ric_rec.c:
// 210-231, :292-317, :620-633); the box halves stay on the host path (the reference's in-place side effects).
struct GenStage {
    size_t oG = 0, oQx = 0, oqx = 0;
};
GenStage carve_general(const WLayout& L, Carve& c) {
    GenStage g;
    if (!L.any_ng) return g;
    g.oG = c.take(8 * L.nG);
    g.oQx = c.take(8 * L.nD);
    g.oqx = c.take(8 * L.nD);
    return g;
}
void stage_general(const WLayout& L, const GenStage& g, char* H, double** hpDCt, double** Qx, double** qx) {
    if (!L.any_ng) return;
    double* HG = reinterpret_cast<double*>(H + g.oG);
    for (int k = 0; k <= L.N; k++) {
        const WideStage& s = L.st[k];
        if (s.ng == 0) continue;
        memcpy(HG + s.oG, hpDCt[k], (size_t)rup(s.nu + s.nx, BS) * s.sdG * sizeof(double));
        for (int l = 0; l < s.ng; l++) {
            if (Qx) reinterpret_cast<double*>(H + g.oQx)[s.oD + s.pnb + l] = Qx[k][s.pnb + l];
            if (qx) reinterpret_cast<double*>(H + g.oqx)[s.oD + s.pnb + l] = qx[k][s.pnb + l];
        }
    }
}
void general_args(const WLayout& L, const GenStage& g, char* D, WideArgs& a) {
    if (!L.any_ng) return;
    a.DCt = reinterpret_cast<const double*>(D + g.oG);
    a.Qx = reinterpret_cast<const double*>(D + g.oQx);
    a.qx = reinterpret_cast<const double*>(D + g.oqx);
}
bool fits_check(const WLayout& L) {
    if (L.lds > LDS_MAX_DOUBLES || !L.fits) {
        hk_set_error(HPMPC_MI355X_EUNSUPPORTED, "wide stage beyond the kernel's tile limits (64 KiB LDS, "
                                                "nu+nx < 128, nx <= 64)");
        return false;
    }
    return true;
}
}  // namespace

extern "C" void hk_wide_sv_entry(int N, int* nx, int* nu, int* nb, int** idxb, int* ng, int update_b, double** hpBAbt,
                                 double** b, int update_q, double** hpQ, double** q, double** bd, double** hpDCt,
                                 double** Qx, double** qx, double** hux, int compute_pi, double** hpi, int compute_Pb,
                                 double** hPb, double* memory) {
    hk_set_error(0, nullptr);
    WLayout L = make_layout(N, nx, nu, nb, ng);
    if (!fits_check(L)) return;
    Carve c;
    const size_t oSt = c.take(sizeof(WideStage) * (N + 1)), oB = c.take(8 * L.nB), oR = c.take(8 * L.nR),
                 oF = c.take(8 * L.nL), oU = c.take(8 * L.nU), oP = c.take(8 * L.nP), oPb = c.take(8 * L.nP);
    const GenStage gs = carve_general(L, c);
    if (!g_w.ensure(c.o)) return;
    char* H = g_w.host;
    memcpy(H + oSt, L.st.data(), sizeof(WideStage) * (N + 1));
    double* HB = reinterpret_cast<double*>(H + oB);
    double* HR = reinterpret_cast<double*>(H + oR);
    // the reference's in-place side effects, in its stage order (d_back_ric_rec.c:197-209, :249-291)
    for (int k = N; k >= 0; k--) {
        const WideStage& s = L.st[k];
        const int nux = s.nu + s.nx;
        if (update_q)
            for (int j = 0; j < nux; j++) P4(hpQ[k], s.sdR, nux, j) = q[k][j];
        for (int l = 0; l < nb[k]; l++) {
            const int ii = idxb[k][l];
            P4(hpQ[k], s.sdR, ii, ii) = bd[k][l] + Qx[k][l];
        }
        for (int l = 0; l < nb[k]; l++) P4(hpQ[k], s.sdR, nux, idxb[k][l]) += qx[k][l];
        memcpy(HR + s.oR, hpQ[k], (size_t)rup(nux + 1, BS) * s.sdR * sizeof(double));
        if (k < N) {
            if (update_b)
                for (int j = 0; j < s.nx1; j++) P4(hpBAbt[k], s.sdB, nux, j) = b[k][j];
            memcpy(HB + s.oB, hpBAbt[k], (size_t)rup(nux + 1, BS) * s.sdB * sizeof(double));
        }
    }
    stage_general(L, gs, H, hpDCt, Qx, qx);
    char* D = g_w.dev;
    WideArgs a;
    memset(&a, 0, sizeof a);
    general_args(L, gs, D, a);
    a.N = N;
    a.nprob = 1;
    a.st = reinterpret_cast<const WideStage*>(D + oSt);
    a.BAbt = reinterpret_cast<const double*>(D + oB);
    a.RSQ = reinterpret_cast<const double*>(D + oR);
    a.ws = reinterpret_cast<double*>(D + oF);
    a.ux = reinterpret_cast<double*>(D + oU);
    a.pi = reinterpret_cast<double*>(D + oP);
    a.Pb = reinterpret_cast<double*>(D + oPb);
    a.compute_pi = compute_pi;
    a.compute_Pb = compute_Pb;
    a.offW = L.offW;
    a.offX = L.offX;
    a.offV = L.offV;
    a.offST = L.offST;
    a.ldW = L.ldW;
    a.ldX = L.ldX;
    if (!g_w.up(c.o) || !launch(0, &a, 1, L.lds, g_w.stream, "hk_wide_sv") || !g_w.down(c.o)) return;
    const double* HU = reinterpret_cast<const double*>(H + oU);
    const double* HP = reinterpret_cast<const double*>(H + oP);
    const double* HPb = reinterpret_cast<const double*>(H + oPb);
    for (int k = 0; k <= N; k++) {
        const WideStage& s = L.st[k];
        memcpy(hux[k], HU + s.oU, (s.nu + s.nx) * sizeof(double));
        if (k < N && compute_pi) memcpy(hpi[k], HP + s.oP, s.nx1 * sizeof(double));
        if (k < N && compute_Pb) memcpy(hPb[k], HPb + s.oP, s.nx1 * sizeof(double));
    }
    memcpy(memory, H + oF, 8 * L.nL);
}

namespace {
bool wide_check(const WLayout& L) { return fits_check(L); }
void wide_args(const WLayout& L, WideArgs& a) {
    memset(&a, 0, sizeof a);
    a.N = L.N;
    a.nprob = 1;
    a.offW = L.offW;
    a.offX = L.offX;
    a.offV = L.offV;
    a.offST = L.offST;
    a.ldW = L.ldW;
    a.ldX = L.ldX;
}
}  // namespace

// d_back_ric_rec_trf_tv_res on wide stages: hk_wide_sv in factor-only mode (no augmented row, no forward).
extern "C" void hk_wide_trf_entry(int N, int* nx, int* nu, int* nb, int** idxb, int* ng, double** hpBAbt,
                                  double** hpQ, double** hpDCt, double** Qx, double** bd, double* memory) {
    hk_set_error(0, nullptr);
    WLayout L = make_layout(N, nx, nu, nb, ng);
    if (!wide_check(L)) return;
    Carve c;
    const size_t oSt = c.take(sizeof(WideStage) * (N + 1)), oB = c.take(8 * L.nB), oR = c.take(8 * L.nR),
                 oF = c.take(8 * L.nL), oU = c.take(8 * L.nU), oP = c.take(8 * L.nP);
    const GenStage gs = carve_general(L, c);
    if (!g_w.ensure(c.o)) return;
    char* H = g_w.host;
    memcpy(H + oSt, L.st.data(), sizeof(WideStage) * (N + 1));
    double* HB = reinterpret_cast<double*>(H + oB);
    double* HR = reinterpret_cast<double*>(H + oR);
    for (int k = N; k >= 0; k--) {  // the reference's side effect: box diagonal = bd + Qx (d_back_ric_rec.c:468, :520)
        const WideStage& s = L.st[k];
        const int nux = s.nu + s.nx;
        for (int l = 0; l < nb[k]; l++) {
            const int ii = idxb[k][l];
            P4(hpQ[k], s.sdR, ii, ii) = bd[k][l] + Qx[k][l];
        }
        memcpy(HR + s.oR, hpQ[k], (size_t)rup(nux + 1, BS) * s.sdR * sizeof(double));
        if (k < N) memcpy(HB + s.oB, hpBAbt[k], (size_t)rup(nux + 1, BS) * s.sdB * sizeof(double));
    }
    stage_general(L, gs, H, hpDCt, Qx, nullptr);
    char* D = g_w.dev;
    WideArgs a;
    wide_args(L, a);
    general_args(L, gs, D, a);
    a.trf = 1;
    a.st = reinterpret_cast<const WideStage*>(D + oSt);
    a.BAbt = reinterpret_cast<const double*>(D + oB);
    a.RSQ = reinterpret_cast<const double*>(D + oR);
    a.ws = reinterpret_cast<double*>(D + oF);
    a.ux = reinterpret_cast<double*>(D + oU);
    a.pi = a.Pb = reinterpret_cast<double*>(D + oP);
    if (!g_w.up(c.o) || !launch(0, &a, 1, L.lds, g_w.stream, "hk_wide_sv(trf)") || !g_w.down(c.o)) return;
    memcpy(memory, H + oF, 8 * L.nL);
}

// d_back_ric_rec_trs_tv_res on wide stages (hk_wide_trs) over the factor hk_wide_trf_entry left in memory.
extern "C" void hk_wide_trs_entry(int N, int* nx, int* nu, int* nb, int** idxb, int* ng, double** hpBAbt,
                                  double** hb, double** hq, double** hpDCt, double** qx, double** hux, int compute_pi,
                                  double** hpi, int compute_Pb, double** hPb, double* memory) {
    hk_set_error(0, nullptr);
    WLayout L = make_layout(N, nx, nu, nb, ng);
    if (!wide_check(L)) return;
    Carve c;
    const size_t oSt = c.take(sizeof(WideStage) * (N + 1)), oB = c.take(8 * L.nB), oF = c.take(8 * L.nL),
                 oU = c.take(8 * L.nU), oP = c.take(8 * L.nP), oPb = c.take(8 * L.nP), ob = c.take(8 * L.nP),
                 oq = c.take(8 * L.nU), oqx = c.take(8 * L.nD), oI = c.take(4 * L.nI), oG = c.take(8 * L.nG);
    if (!g_w.ensure(c.o)) return;
    char* H = g_w.host;
    memcpy(H + oSt, L.st.data(), sizeof(WideStage) * (N + 1));
    memcpy(H + oF, memory, 8 * L.nL);
    double* HB = reinterpret_cast<double*>(H + oB);
    double* HPb = reinterpret_cast<double*>(H + oPb);
    double* Hb = reinterpret_cast<double*>(H + ob);
    double* Hq = reinterpret_cast<double*>(H + oq);
    double* Hqx = reinterpret_cast<double*>(H + oqx);
    int* HI = reinterpret_cast<int*>(H + oI);
    for (int k = 0; k <= N; k++) {
        const WideStage& s = L.st[k];
        const int nux = s.nu + s.nx;
        memcpy(Hq + s.oU, hq[k], nux * sizeof(double));
        if (nb[k] > 0) {
            memcpy(Hqx + s.oD, qx[k], nb[k] * sizeof(double));
            memcpy(HI + s.oI, idxb[k], nb[k] * sizeof(int));
        }
        if (ng[k] > 0) {  // DCt qx_g on the device (general half of qx at pnb)
            memcpy(Hqx + s.oD + s.pnb, qx[k] + s.pnb, ng[k] * sizeof(double));
            memcpy(reinterpret_cast<double*>(H + oG) + s.oG, hpDCt[k],
                   (size_t)rup(nux, BS) * s.sdG * sizeof(double));
        }
        if (k < N) {
            memcpy(HB + s.oB, hpBAbt[k], (size_t)rup(nux + 1, BS) * s.sdB * sizeof(double));
            memcpy(Hb + s.oP, hb[k], s.nx1 * sizeof(double));
            if (!compute_Pb) memcpy(HPb + s.oP, hPb[k], s.nx1 * sizeof(double));
        }
    }
    char* D = g_w.dev;
    WideArgs a;
    wide_args(L, a);
    a.st = reinterpret_cast<const WideStage*>(D + oSt);
    a.BAbt = reinterpret_cast<const double*>(D + oB);
    a.ws = reinterpret_cast<double*>(D + oF);
    a.ux = reinterpret_cast<double*>(D + oU);
    a.pi = reinterpret_cast<double*>(D + oP);
    a.Pb = reinterpret_cast<double*>(D + oPb);
    a.hb = reinterpret_cast<const double*>(D + ob);
    a.hq = reinterpret_cast<const double*>(D + oq);
    a.qx = reinterpret_cast<const double*>(D + oqx);
    a.idxb = reinterpret_cast<const int*>(D + oI);
    if (L.any_ng) a.DCt = reinterpret_cast<const double*>(D + oG);
    a.compute_pi = compute_pi;
    a.compute_Pb = compute_Pb;
    if (!g_w.up(c.o) || !launch(3, &a, 1, L.lds, g_w.stream, "hk_wide_trs") || !g_w.down(c.o)) return;
    const double* HU = reinterpret_cast<const double*>(H + oU);
    const double* HP = reinterpret_cast<const double*>(H + oP);
    for (int k = 0; k <= N; k++) {
        const WideStage& s = L.st[k];
        memcpy(hux[k], HU + s.oU, (s.nu + s.nx) * sizeof(double));
        if (k < N && compute_pi) memcpy(hpi[k], HP + s.oP, s.nx1 * sizeof(double));
        if (k < N && compute_Pb) memcpy(hPb[k], HPb + s.oP, s.nx1 * sizeof(double));
    }
}

// ------------------------------------------------------------------------------------------------
// Partial condensing: host bookkeeping shared by the single-problem and the batched entry points.
// ------------------------------------------------------------------------------------------------
namespace {

int block_len(int N, int N2, int ii) {
    const int N1 = N / N2, R1 = N - N2 * N1, M1 = R1 > 0 ? N1 + 1 : N1;
    return ii < R1 ? M1 : N1;
}

struct PcPlan {
    int N = 0, N2 = 0;
    WLayout orig, cond;
    std::vector<int> nx2, nu2, nb2, ng2;
    std::vector<int> idxb2;  // condensed box indices packed per stage (cond.st[ii].oI), as hk_pcond writes them
    std::vector<PcBlock> blk;
    std::vector<int> idxb;  // original idxb packed per stage (orig.st[k].oI)
    long long nG = 0;       // Gamma scratch (doubles per problem)
    long long nG2 = 0;      // condensed DCt2 (doubles per problem)
    long long ref_d = 0;    // the reference's memory carve: doubles before the idxb2 ints
    int pc_lds = 0, ldP = 0, ldX = 0, ldW = 0, ldB = 0, offP = 0, offX = 0, offW = 0, offB = 0, offGA = 0, offGB = 0;
    int px_lds = 0, ldT = 0, xoB = 0, xoR = 0, xoV = 0, xoW = 0, xoQ = 0;
    int pc_gm = 4;  // hk_pcond's gemm tiles per wave (4 or 8)
    int offST = 0;  // hk_pcond's LDS stage table
    int offU = 0;   // hk_pcond's P-form u columns
    int offGT = 0;  // hk_pcond's P-form certificate bounds
    bool pform_ok = true;
    bool pc_dm_ok = true;  // hk_pcond's deferred cross terms fit the Gamma scratch
};

void problem_size(int N, const int* nx, const int* nu, const int* nb, const int* const* hidxb, const int* ng, int N2,
                  int* nx2, int* nu2, int* nb2, int* ng2) {
    int N_tmp = 0;
    for (int ii = 0; ii < N2; ii++) {
        const int T1 = block_len(N, N2, ii);
        nx2[ii] = nx[N_tmp];
        nu2[ii] = nu[N_tmp];
        nb2[ii] = nb[N_tmp];
        ng2[ii] = ng[N_tmp];
        for (int jj = 1; jj < T1; jj++) {
            const int s = N_tmp + jj;
            int nbb = 0, nbg = 0;
            for (int kk = 0; kk < nb[s]; kk++) (hidxb[s][kk] < nu[s] ? nbb : nbg)++;
            nu2[ii] += nu[s];
            nb2[ii] += nbb;
            ng2[ii] += ng[s] + nbg;
        }
        N_tmp += T1;
    }
    nx2[N2] = nx[N];
    nu2[N2] = nu[N];
    nb2[N2] = nb[N];
    ng2[N2] = ng[N];
}

bool pc_plan(PcPlan& P, int N, const int* nx, const int* nu_in, const int* nb, const int* const* idxb, const int* ng,
             int N2) {
    if (N2 < 1 || N2 > N) {  // N2 == N: blocks of one stage (d_part_cond itself aliases instead, :936)
        hk_set_error(HPMPC_MI355X_EUNSUPPORTED, "partial condensing needs 1 <= N2 <= N (:962-967)");
        return false;
    }
    for (int k = 0; k < N; k++)
        if (ng[k] > 0) {  // d_part_cond.c:971-976: only ng[N] > 0 is supported by the reference
            hk_set_error(HPMPC_MI355X_EUNSUPPORTED, "partial condensing with ng > 0 before the last stage");
            return false;
        }
    std::vector<int> nu(nu_in, nu_in + N + 1);
    nu[N] = 0;
    P.N = N;
    P.N2 = N2;
    P.orig = make_layout(N, nx, nu.data(), nb, ng);
    P.idxb.assign(P.orig.nI, 0);
    for (int k = 0; k <= N; k++)
        for (int l = 0; l < nb[k]; l++) P.idxb[P.orig.st[k].oI + l] = idxb[k][l];
    P.nx2.resize(N2 + 1);
    P.nu2.resize(N2 + 1);
    P.nb2.resize(N2 + 1);
    P.ng2.resize(N2 + 1);
    problem_size(N, nx, nu.data(), nb, idxb, ng, N2, P.nx2.data(), P.nu2.data(), P.nb2.data(), P.ng2.data());
    P.cond = make_layout(N2, P.nx2.data(), P.nu2.data(), P.nb2.data(), P.ng2.data());
    P.blk.resize(N2);
    int N_tmp = 0, nzM = 1, nxM = 1;
    long long oG2 = 0, ref_d = 0;
    for (int ii = 0; ii < N2; ii++) {
        PcBlock& b = P.blk[ii];
        memset(&b, 0, sizeof b);
        b.s0 = N_tmp;
        b.T = block_len(N, N2, ii);
        b.nx0 = nx[N_tmp];
        b.nut = 0;
        b.oG = (int)P.nG;
        int rows = b.nx0 + 1;
        long long sneed = 0;  // hk_pcond's deferred cross terms: (nx_s + 1) x nu_s per stage s >= 1 of the block
        for (int j = 0; j < b.T; j++) {
            const int s = N_tmp + j;
            b.nut += nu[s];
            rows += nu[s];
            P.nG += (long long)rows * nx[s + 1];
            if (j > 0) sneed += (long long)(nx[s] + 1) * nu[s];
            nzM = std::max(nzM, nu[s] + nx[s] + 1);
            nxM = std::max(nxM, nx[s + 1]);
        }
        if (sneed > P.nG - b.oG) P.pc_dm_ok = false;  // the block's Gamma scratch holds them (it always does at nu <= nx)
        b.oB2 = P.cond.st[ii].oB;
        b.oR2 = P.cond.st[ii].oR;
        b.oD2 = P.cond.st[ii].oD;
        b.oI2 = P.cond.st[ii].oI;
        b.oG2 = (int)oG2;
        oG2 += (long long)rup(P.nu2[ii] + P.nx2[ii], BS) * rup(P.ng2[ii], NCL);
        b.nx2n = P.nx2[ii + 1];
        b.nb2 = P.nb2[ii];
        b.ng2 = P.ng2[ii];
        N_tmp += b.T;
        // the reference's carve of `memory` (d_part_cond.c:1013-1041), doubles part
        const int pnz2 = rup(P.nu2[ii] + P.nx2[ii] + 1, BS);
        ref_d += (long long)pnz2 * rup(P.nx2[ii + 1], NCL) + (long long)pnz2 * rup(P.nu2[ii] + P.nx2[ii], NCL) +
                 (long long)rup(P.nu2[ii] + P.nx2[ii], BS) * rup(P.ng2[ii], NCL) + 2 * rup(P.nb2[ii], BS) +
                 2 * rup(P.ng2[ii], BS);
    }
    P.nG2 = oG2 > 0 ? oG2 : 1;
    P.ref_d = ref_d;
    // condensed box indices (d_cond_DCtd, d_part_cond.c:579-688): input boxes of the block's later stages keep
    // their position in [u_{T-1}; ..; u_0; x_0], stage 0's boxes stay boxes, inner state boxes become general
    P.idxb2.assign(P.cond.nI, 0);
    for (int ii = 0; ii < N2; ii++) {
        const PcBlock& b = P.blk[ii];
        int* i2 = P.idxb2.data() + P.cond.st[ii].oI;
        int ib = 0, nu_tmp = 0;
        for (int sI = b.T - 1; sI >= 1; sI--) {
            const int s = b.s0 + sI;
            nu_tmp += nu[s];
            for (int jj = 0; jj < nb[s]; jj++)
                if (idxb[s][jj] < nu[s]) i2[ib++] = nu_tmp - nu[s] + idxb[s][jj];
        }
        nu_tmp += nu[b.s0];
        for (int jj = 0; jj < nb[b.s0]; jj++) i2[ib++] = nu_tmp - nu[b.s0] + idxb[b.s0][jj];
    }
    for (int l = 0; l < nb[N]; l++) P.idxb2[P.cond.st[N2].oI + l] = idxb[N][l];
    // Gamma tiles: the largest (rows x nx_{j+1}) of any block, also used as the RSQrq_{s-1} tile
    long long gmax = (long long)nzM * nzM;
    int tmax = 0;  // output tiles of hk_pcond's largest gemm: Gamma_{j-1} A_j, and W / W W' of d_cond_RSQrq
    auto tiles = [](int m, int n) { return ((m + 15) / 16) * ((n + 15) / 16); };
    {
        int Nt = 0;
        for (int ii = 0; ii < N2; ii++) {
            int rows = nx[Nt] + 1;
            for (int j = 0; j < P.blk[ii].T; j++) {
                const int s = Nt + j;
                if (j > 0) tmax = std::max(tmax, tiles(rows, nx[s + 1]));  // rows = rows(j - 1)
                rows += nu[s];
                gmax = std::max(gmax, (long long)rows * nx[s + 1]);
                if (j > 0) {  // d_cond_RSQrq at stage s: W (nz_{s-1} x nx_s), W W' (nz_{s-1} x nux_{s-1})
                    const int nzp = nu[s - 1] + nx[s - 1] + 1;
                    tmax = std::max(tmax, std::max(tiles(nzp, nx[s]), tiles(nzp, nzp - 1)));
                }
            }
            Nt += P.blk[ii].T;
        }
    }
    if (tmax > 32) {
        hk_set_error(HPMPC_MI355X_EUNSUPPORTED, "condensing block beyond hk_pcond's gemm tiles (32 16x16 tiles)");
        return false;
    }
    P.pc_gm = tmax <= 16 ? 4 : 8;
    // LDS carve (doubles, every tile 32-byte aligned for the 16-byte LDS DMA): pL as a lib4 RSQrq block
    // (rup(nz, 4) x sdR), Lx dense, the BAbt tile dense (d_cond_BAbt) or as a lib4 block (d_cond_RSQrq), Gamma_{j-1}
    int nuxM = 1;
    for (int k = 0; k < N; k++) nuxM = std::max(nuxM, nu[k] + nx[k]);
    P.ldP = P.ldW = P.ldB = nzM;
    P.ldX = nxM + 1;
    P.offP = 0;
    P.offX = rup(std::max(P.ldP * nzM, rup(nzM, BS) * rup(nuxM, NCL)), 4);
    P.offB = P.offX + rup(P.ldX * nzM, 4);  // Lx, or the P form's T = X^ [BAbt | e]' ((nx+1) x nz)
    P.offW = P.offB;  // W is formed in place in the BAbt tile
    P.offGA = P.offB + rup(std::max(P.ldB * nxM, rup(nzM, BS) * rup(nxM, NCL)), 4);
    P.offGB = 0;
    int Tmax = 1;
    for (int ii = 0; ii < N2; ii++) Tmax = std::max(Tmax, P.blk[ii].T);
    P.offST = P.offGA + rup((int)gmax, 4);
    int nuM = 1;
    for (int k = 0; k < N; k++) nuM = std::max(nuM, nu[k]);
    P.offU = P.offST + rup(Tmax * (int)(sizeof(WideStage) / sizeof(double)), 2);
    P.offGT = P.offU + P.ldX * nuM;
    P.pc_lds = P.offGT + Tmax;
    // the P form's per-row scratch (one row value per stage and state) lives in the Gamma tile before d_cond_RSQrq
    P.pform_ok = (long long)(Tmax - 1) * nxM <= gmax;
    if (gmax > 12 * 256 || nxM > 63) {  // hk_pcond: PC_GCH Gamma outputs per lane; the state Cholesky in one wave
        hk_set_error(HPMPC_MI355X_EUNSUPPORTED, "condensing block beyond the kernel's tile limits "
                                                "(Gamma rows x nx <= 3072, nx <= 63)");
        return false;
    }
    // expansion tiles: BAbt (nzM x nxM), RSQrq (nzM x nzM), ux_j, box terms, pi_j
    P.ldT = nzM;
    P.xoB = 0;
    P.xoR = P.xoB + nzM * nxM;
    P.xoV = P.xoR + nzM * nzM;
    P.xoW = P.xoV + nzM;
    P.xoQ = P.xoW + nzM;
    P.px_lds = P.xoQ + std::max(nzM, nxM);
    for (int ii = 0; ii < N2; ii++)  // hk_pcond's d_cond_DCtd bookkeeping: 6 ints per stage + 1 per general row
        if (6 * P.blk[ii].T + P.ng2[ii] > 2 * P.offST) {  // below the LDS stage table
            hk_set_error(HPMPC_MI355X_EUNSUPPORTED, "condensing block with more state boxes than the LDS tiles hold");
            return false;
        }
    if (P.pc_lds > LDS_MAX_DOUBLES || P.px_lds > LDS_MAX_DOUBLES) {
        hk_set_error(HPMPC_MI355X_EUNSUPPORTED, "condensing stage tiles beyond the 64 KiB LDS budget");
        return false;
    }
    return true;
}

void fill_pc_args(const PcPlan& P, PcArgs& a) {
    memset(&a, 0, sizeof a);
    a.N = P.N;
    a.N2 = P.N2;
    a.sB = P.orig.nB;
    a.sR = P.orig.nR;
    a.sD = P.orig.nD;
    a.sG = P.nG;
    a.sB2 = P.cond.nB;
    a.sR2 = P.cond.nR;
    a.sG2 = P.nG2;
    a.sD2 = P.cond.nD;
    a.oR2N = P.cond.st[P.N2].oR;
    a.oD2N = P.cond.st[P.N2].oD;
    a.nDN = 2 * P.orig.st[P.N].pnb + 2 * rup(P.orig.st[P.N].ng, BS);
    a.sdRN = P.orig.st[P.N].sdR;
    a.nzN = P.orig.st[P.N].nu + P.orig.st[P.N].nx + 1;
    a.offP = P.offP;
    a.offX = P.offX;
    a.offW = P.offW;
    a.offB = P.offB;
    a.ldP = P.ldP;
    a.ldX = P.ldX;
    a.ldW = P.ldW;
    a.ldB = P.ldB;
    a.offGA = P.offGA;
    a.offGB = P.offGB;
    a.ph = PC_ALL;
    a.gm = P.pc_gm;
    a.offST = P.offST;
    a.offU = P.offU;
    // HPMPC_MI355X_PCOND_PFORM=0: every stage takes the Cholesky route (read per call: tests compare the two routes)
    const char* pf = getenv("HPMPC_MI355X_PCOND_PFORM");
    a.pform = P.pform_ok && (pf ? atoi(pf) : 1);
    a.offGT = P.offGT;
    // d_cond_RSQrq before d_cond_BAbt with the cross terms deferred (no Gamma through HBM) unless
    // HPMPC_MI355X_PCOND_DM=0 (read per call: tests compare the two orders bitwise)
    const char* dmv = getenv("HPMPC_MI355X_PCOND_DM");
    a.dm = P.pc_dm_ok && (dmv ? atoi(dmv) : 1);
}

void fill_px_args(const PcPlan& P, PxArgs& a) {
    memset(&a, 0, sizeof a);
    a.N = P.N;
    a.N2 = P.N2;
    a.sB = P.orig.nB;
    a.sR = P.orig.nR;
    a.sU = P.orig.nU;
    a.sP = P.orig.nP;
    a.sC = P.orig.nD;
    a.sU2 = P.cond.nU;
    a.sP2 = P.cond.nP;
    a.sC2 = P.cond.nD;
    a.offB = P.xoB;
    a.offR = P.xoR;
    a.offV = P.xoV;
    a.offW = P.xoW;
    a.offQ = P.xoQ;
    a.ldT = P.ldT;
}

}  // namespace

// d_part_cond.c:694-738 -- integer bookkeeping (no device work)
extern "C" void d_part_cond_compute_problem_size(int N, int* nx, int* nu, int* nb, int** hidxb, int* ng, int N2,
                                                 int* nx2, int* nu2, int* nb2, int* ng2) {
    problem_size(N, nx, nu, nb, hidxb, ng, N2, nx2, nu2, nb2, ng2);
}

// every temporary of the condensing lives on the device
extern "C" int d_part_cond_work_space_size_bytes(int N, int* nx, int* nu, int* nb, int** hidxb, int* ng, int N2,
                                                 int* nx2, int* nu2, int* nb2, int* ng2) {
    return 64;
}

// d_part_cond.c:868-924: the condensed data are written into `memory` with the reference's carve
extern "C" int d_part_cond_memory_space_size_bytes(int N, int* nx, int* nu, int* nb, int** hidxb, int* ng, int N2,
                                                   int* nx2, int* nu2, int* nb2, int* ng2) {
    if (N2 == N) return 0;
    long long d_size = 0, i_size = 0;
    for (int ii = 0; ii < N2; ii++) {
        const int pnz2 = rup(nu2[ii] + nx2[ii] + 1, BS), pnux2 = rup(nu2[ii] + nx2[ii], BS);
        d_size += (long long)pnz2 * rup(nx2[ii + 1], NCL) + (long long)pnz2 * rup(nu2[ii] + nx2[ii], NCL) +
                  (long long)pnux2 * rup(ng2[ii], NCL) + 2 * rup(nb2[ii], BS) + 2 * rup(ng2[ii], BS);
        i_size += nb2[ii];
    }
    return (int)((d_size * 8 + i_size * 4 + 63) / 64 * 64);
}

// d_part_cond.c:926-1062
extern "C" void d_part_cond(int N, int* nx, int* nu, int* nb, int** hidxb, int* ng, double** hpBAbt, double** hpRSQrq,
                            double** hpDCt, double** hd, int N2, int* nx2, int* nu2, int* nb2, int** hidxb2, int* ng2,
                            double** hpBAbt2, double** hpRSQrq2, double** hpDCt2, double** hd2, void* memory,
                            void* work) {
    (void)work;
    hk_set_error(0, nullptr);
    if (N2 == N) {  // :936-960: the condensed problem aliases the original
        for (int ii = 0; ii <= N; ii++) {
            nx2[ii] = nx[ii];
            nu2[ii] = nu[ii];
            nb2[ii] = nb[ii];
            hidxb2[ii] = hidxb[ii];
            ng2[ii] = ng[ii];
            if (ii < N) hpBAbt2[ii] = hpBAbt[ii];
            hpRSQrq2[ii] = hpRSQrq[ii];
            hpDCt2[ii] = hpDCt[ii];
            hd2[ii] = hd[ii];
        }
        return;
    }
    PcPlan P;
    if (!pc_plan(P, N, nx, nu, nb, hidxb, ng, N2)) return;
    const WLayout &O = P.orig, &C = P.cond;
    // the condensed outputs go into one buffer with the reference's carve (BAbt2 | RSQrq2 | DCt2 | d2 | idxb2,
    // d_part_cond.c:1013-1041), downloaded into `memory` as is; the kernel's copy of the terminal RSQrq
    // lands past it (the reference aliases hpRSQrq[N] there instead)
    const long long term_off = P.ref_d + (4 * C.nI + 7) / 8 + 8;
    const long long mem_doubles = term_off + (long long)rup(O.st[N].nu + O.st[N].nx + 1, BS) * O.st[N].sdR;
    Carve c;
    const size_t oSt = c.take(sizeof(WideStage) * (N + 1)), oBlk = c.take(sizeof(PcBlock) * N2),
                 oIdx = c.take(4 * O.nI), oB = c.take(8 * O.nB), oR = c.take(8 * O.nR), oD = c.take(8 * O.nD),
                 oG = c.take(8 * P.nG), oMem = c.take(8 * mem_doubles);
    if (!g_w.ensure(c.o)) return;
    char* H = g_w.host;
    memcpy(H + oSt, O.st.data(), sizeof(WideStage) * (N + 1));
    // condensed outputs go straight into the reference carve inside one buffer (oMem): BAbt2 | RSQrq2 |
    // DCt2 | d2 | idxb2, so the block offsets are absolute within that buffer
    std::vector<PcBlock> blk = P.blk;
    long long o = 0;
    std::vector<long long> cB(N2), cR(N2), cG(N2), cD(N2);
    for (int ii = 0; ii < N2; ii++) {
        cB[ii] = o;
        o += (long long)rup(P.nu2[ii] + P.nx2[ii] + 1, BS) * rup(P.nx2[ii + 1], NCL);
    }
    for (int ii = 0; ii < N2; ii++) {
        cR[ii] = o;
        o += (long long)rup(P.nu2[ii] + P.nx2[ii] + 1, BS) * rup(P.nu2[ii] + P.nx2[ii], NCL);
    }
    for (int ii = 0; ii < N2; ii++) {
        cG[ii] = o;
        o += (long long)rup(P.nu2[ii] + P.nx2[ii], BS) * rup(P.ng2[ii], NCL);
    }
    for (int ii = 0; ii < N2; ii++) {
        cD[ii] = o;
        o += 2 * rup(P.nb2[ii], BS) + 2 * rup(P.ng2[ii], BS);
    }
    int oi = 0;
    for (int ii = 0; ii < N2; ii++) {
        blk[ii].oB2 = (int)cB[ii];
        blk[ii].oR2 = (int)cR[ii];
        blk[ii].oG2 = (int)cG[ii];
        blk[ii].oD2 = (int)cD[ii];
        blk[ii].oI2 = oi;
        oi += P.nb2[ii];
    }
    memcpy(H + oBlk, blk.data(), sizeof(PcBlock) * N2);
    memcpy(H + oIdx, P.idxb.data(), 4 * O.nI);
    double* HB = reinterpret_cast<double*>(H + oB);
    double* HR = reinterpret_cast<double*>(H + oR);
    double* HD = reinterpret_cast<double*>(H + oD);
    for (int k = 0; k <= N; k++) {
        const WideStage& s = O.st[k];
        const int nux = s.nu + s.nx;
        if (k < N) memcpy(HB + s.oB, hpBAbt[k], (size_t)rup(nux + 1, BS) * s.sdB * sizeof(double));
        memcpy(HR + s.oR, hpRSQrq[k], (size_t)rup(nux + 1, BS) * s.sdR * sizeof(double));
        if (nb[k] + ng[k] > 0) memcpy(HD + s.oD, hd[k], (size_t)(2 * s.pnb + 2 * rup(ng[k], BS)) * sizeof(double));
    }
    char* D = g_w.dev;
    PcArgs a;
    fill_pc_args(P, a);
    a.nprob = 1;
    a.st = reinterpret_cast<const WideStage*>(D + oSt);
    a.blk = reinterpret_cast<const PcBlock*>(D + oBlk);
    a.idxb = reinterpret_cast<const int*>(D + oIdx);
    a.BAbt = reinterpret_cast<const double*>(D + oB);
    a.RSQ = reinterpret_cast<const double*>(D + oR);
    a.d = reinterpret_cast<const double*>(D + oD);
    a.G = reinterpret_cast<double*>(D + oG);
    double* mem = reinterpret_cast<double*>(D + oMem);
    a.BAbt2 = a.RSQ2 = a.DCt2 = a.d2 = mem;
    a.idxb2 = reinterpret_cast<int*>(mem + P.ref_d);
    a.oR2N = (int)term_off;
    a.nDN = 0;  // the reference aliases hd2[N2] = hd[N] (d_part_cond.c), nothing to copy into the carve
    if (!g_w.up(c.o) || !launch(1, &a, 1, P.pc_lds, g_w.stream, "hk_pcond") || !g_w.down(c.o)) return;
    for (int ii = 0; ii <= N2; ii++) {
        nx2[ii] = P.nx2[ii];
        nu2[ii] = P.nu2[ii];
        nb2[ii] = P.nb2[ii];
        ng2[ii] = P.ng2[ii];
    }
    memcpy(memory, H + oMem, 8 * P.ref_d + 4 * (C.nI > 0 ? oi : 0));
    double* m = static_cast<double*>(memory);
    int* mi = reinterpret_cast<int*>(m + P.ref_d);
    for (int ii = 0; ii < N2; ii++) {
        hpBAbt2[ii] = m + cB[ii];
        hpRSQrq2[ii] = m + cR[ii];
        hpDCt2[ii] = m + cG[ii];
        hd2[ii] = m + cD[ii];
        hidxb2[ii] = mi + blk[ii].oI2;
    }
    hpRSQrq2[N2] = hpRSQrq[N];
    hpDCt2[N2] = hpDCt[N];
    hd2[N2] = hd[N];
    hidxb2[N2] = hidxb[N];
}

// ------------------------------------------------------------------------------------------------
// The building blocks of one condensing block (d_cond_BAbt / d_cond_RSQrq / d_cond_DCtd, d_part_cond.c:214-688):
// the block is a horizon-N problem condensed with N2 = 1 by hk_pcond restricted to one phase (PC_PART).  Gammas
// move between the caller's lib4 matrices and the kernel's dense column-major scratch on the host; the outputs
// the reference writes only in part are uploaded first, so what it leaves alone comes back unchanged.
// ------------------------------------------------------------------------------------------------
namespace {
inline long long l4(int sd, int i, int j) { return (long long)(i / BS) * BS * sd + i % BS + BS * j; }

void cond_part(int ph, int N, const int* nx, const int* nu, const int* nb, int* const* hidxb, double* const* hpBAbt,
               double* const* hpRSQrq, double* const* hd, double** hpGamma, double* pBAbt2, double* pRSQrq2,
               double* pDCt2, double* d2, int* idxb2) {
    hk_set_error(0, nullptr);
    if (N < 1) return;  // the reference returns early (d_part_cond.c:315, :583)
    std::vector<int> nxv(nx, nx + N + 1), nuv(nu, nu + N), nbv(N + 1, 0), ngv(N + 1, 0);
    nuv.push_back(0);
    std::vector<const int*> idx(N + 1, nullptr);
    if (ph == PC_DCTD)
        for (int k = 0; k < N; k++) {
            nbv[k] = nb[k];
            idx[k] = hidxb[k];
        }
    PcPlan P;
    if (!pc_plan(P, N, nxv.data(), nuv.data(), nbv.data(), idx.data(), ngv.data(), 1)) return;
    const WLayout& O = P.orig;
    const PcBlock& b0 = P.blk[0];
    const int nv = b0.nut + b0.nx0, nbb = b0.nb2, nbg = b0.ng2;
    const int pnbb = rup(nbb, BS), pnbg = rup(nbg, BS), cnbg = rup(nbg, NCL), cnux2 = rup(nv, NCL);
    // Gamma_j: rows r_j, dense at go[j] in the scratch
    std::vector<int> rj(N);
    std::vector<long long> go(N + 1, 0);
    for (int j = 0, acc = b0.nx0 + 1; j < N; j++) {
        acc += nuv[j];
        rj[j] = acc;
        go[j + 1] = go[j] + (long long)acc * nxv[j + 1];
    }
    // extents the reference touches in the partly-written outputs (last element + 1)
    long long nR2 = l4(cnux2, nv, nv - 1) + 1, nG2 = 0, nD2 = nbg > 0 ? 2 * pnbb + pnbg + nbg : (nbb > 0 ? pnbb + nbb : 0);
    if (ph == PC_DCTD) {  // d_part_cond.c:637-668: the column of general constraint ig spans rows nu_tmp .. +idx_gammab
        int ig = 0, nu_tmp = 0, idx_gammab = b0.nx0;
        for (int j = 0; j < N - 1; j++) idx_gammab += nuv[j];
        for (int s = N - 1; s >= 1; s--) {
            nu_tmp += nuv[s];
            for (int jj = 0; jj < nb[s]; jj++)
                if (hidxb[s][jj] >= nuv[s]) {
                    if (idx_gammab > 0) nG2 = std::max(nG2, l4(cnbg, nu_tmp + idx_gammab - 1, ig) + 1);
                    ig++;
                }
            idx_gammab -= nuv[s - 1];
        }
    }
    const long long nB2 = (long long)rup(nv + 1, BS) * rup(nxv[N], NCL);
    Carve c;
    const size_t oSt = c.take(sizeof(WideStage) * (N + 1)), oBlk = c.take(sizeof(PcBlock)), oIdx = c.take(4 * O.nI + 4),
                 oB = c.take(8 * O.nB), oR = c.take(8 * O.nR), oD = c.take(8 * O.nD + 8), oG = c.take(8 * P.nG),
                 oB2 = c.take(8 * nB2), oR2 = c.take(8 * nR2), oG2 = c.take(8 * nG2 + 8), oD2 = c.take(8 * nD2 + 8),
                 oI2 = c.take(4 * nbb + 4);
    if (!g_w.ensure(c.o)) return;
    char* H = g_w.host;
    memset(H, 0, c.o);
    memcpy(H + oSt, O.st.data(), sizeof(WideStage) * (N + 1));
    PcBlock blk = b0;
    blk.oB2 = blk.oR2 = blk.oG2 = blk.oD2 = blk.oI2 = 0;
    memcpy(H + oBlk, &blk, sizeof blk);
    memcpy(H + oIdx, P.idxb.data(), 4 * O.nI);
    double* HB = reinterpret_cast<double*>(H + oB);
    double* HR = reinterpret_cast<double*>(H + oR);
    double* HD = reinterpret_cast<double*>(H + oD);
    double* HG = reinterpret_cast<double*>(H + oG);
    for (int k = 0; k < N; k++) {
        const WideStage& s = O.st[k];
        const int nz = s.nu + s.nx + 1;
        if (ph != PC_DCTD) memcpy(HB + s.oB, hpBAbt[k], (size_t)rup(nz, BS) * s.sdB * sizeof(double));
        if (ph == PC_RSQ) memcpy(HR + s.oR, hpRSQrq[k], (size_t)rup(nz, BS) * s.sdR * sizeof(double));
        if (ph == PC_DCTD && nb[k] > 0) memcpy(HD + s.oD, hd[k], (size_t)2 * s.pnb * sizeof(double));
    }
    if (ph != PC_BABT)  // the given Gammas (RSQrq reads Gamma_0..N-2, DCtd those of stages with state boxes)
        for (int j = 0; j + 1 < N; j++) {
            const int sd = rup(nxv[j + 1], NCL);
            for (int cc = 0; cc < nxv[j + 1]; cc++)
                for (int i = 0; i < rj[j]; i++) HG[go[j] + i + (long long)cc * rj[j]] = hpGamma[j][l4(sd, i, cc)];
        }
    if (ph == PC_RSQ) memcpy(H + oR2, pRSQrq2, 8 * nR2);
    if (ph == PC_DCTD) {
        if (nG2) memcpy(H + oG2, pDCt2, 8 * nG2);
        if (nD2) memcpy(H + oD2, d2, 8 * nD2);
    }
    char* D = g_w.dev;
    PcArgs a;
    fill_pc_args(P, a);
    a.ph = ph | PC_PART;
    a.nprob = 1;
    a.st = reinterpret_cast<const WideStage*>(D + oSt);
    a.blk = reinterpret_cast<const PcBlock*>(D + oBlk);
    a.idxb = reinterpret_cast<const int*>(D + oIdx);
    a.BAbt = reinterpret_cast<const double*>(D + oB);
    a.RSQ = reinterpret_cast<const double*>(D + oR);
    a.d = reinterpret_cast<const double*>(D + oD);
    a.G = reinterpret_cast<double*>(D + oG);
    a.BAbt2 = reinterpret_cast<double*>(D + oB2);
    a.RSQ2 = reinterpret_cast<double*>(D + oR2);
    a.DCt2 = reinterpret_cast<double*>(D + oG2);
    a.d2 = reinterpret_cast<double*>(D + oD2);
    a.idxb2 = reinterpret_cast<int*>(D + oI2);
    if (!g_w.up(c.o) || !launch(1, &a, 1, P.pc_lds, g_w.stream, "hk_pcond") || !g_w.down(c.o)) return;
    if (ph == PC_BABT) {  // d_part_cond.c:262-303: Gamma_j (r_j x nx_{j+1}) and BAbt2 = Gamma_{N-1}
        const double* B2 = reinterpret_cast<const double*>(H + oB2);
        for (int j = 0; j < N; j++) {
            const int sd = rup(nxv[j + 1], NCL);
            for (int cc = 0; cc < nxv[j + 1]; cc++)
                for (int i = 0; i < rj[j]; i++) hpGamma[j][l4(sd, i, cc)] = HG[go[j] + i + (long long)cc * rj[j]];
        }
        const int sd = rup(nxv[N], NCL);
        for (int cc = 0; cc < nxv[N]; cc++)
            for (int i = 0; i < rj[N - 1]; i++) pBAbt2[l4(sd, i, cc)] = B2[l4(sd, i, cc)];
    } else if (ph == PC_RSQ) {
        memcpy(pRSQrq2, H + oR2, 8 * nR2);
    } else {
        if (nG2) memcpy(pDCt2, H + oG2, 8 * nG2);
        if (nD2) memcpy(d2, H + oD2, 8 * nD2);
        if (nbb) memcpy(idxb2, H + oI2, 4 * nbb);
    }
}
}  // namespace

// d_part_cond.c:214-308
extern "C" void d_cond_BAbt(int N, int* nx, int* nu, double** hpBAbt, double* work, double** hpGamma, double* pBAbt2) {
    (void)work;
    cond_part(PC_BABT, N, nx, nu, nullptr, nullptr, hpBAbt, nullptr, nullptr, hpGamma, pBAbt2, nullptr, nullptr,
              nullptr, nullptr);
}

// d_part_cond.c:312-574
extern "C" void d_cond_RSQrq(int N, int* nx, int* nu, double** hpBAbt, double** hpRSQrq, double** hpGamma,
                             double* work, double* pRSQrq2) {
    (void)work;
    cond_part(PC_RSQ, N, nx, nu, nullptr, nullptr, hpBAbt, hpRSQrq, nullptr, hpGamma, nullptr, pRSQrq2, nullptr,
              nullptr, nullptr);
}

// d_part_cond.c:579-689
extern "C" void d_cond_DCtd(int N, int* nx, int* nu, int* nb, int** hidxb, double** hd, double** hpGamma,
                            double* pDCt2, double* d2, int* idxb2) {
    cond_part(PC_DCTD, N, nx, nu, nb, hidxb, nullptr, nullptr, hd, hpGamma, nullptr, nullptr, pDCt2, d2, idxb2);
}

extern "C" int d_part_expand_work_space_size_bytes(int N, int* nx, int* nu, int* nb, int* ng) { return 64; }

// d_part_cond.c:1103-1308
extern "C" void d_part_expand_solution(int N, int* nx, int* nu, int* nb, int** hidxb, int* ng, double** hpBAbt,
                                       double** hb, double** hpRSQrq, double** hrq, double** hpDCt, double** hux,
                                       double** hpi, double** hlam, double** ht, int N2, int* nx2, int* nu2, int* nb2,
                                       int** hidxb2, int* ng2, double** hux2, double** hpi2, double** hlam2,
                                       double** ht2, void* work) {
    (void)work;
    (void)hpDCt;  // only the last stage may carry general constraints (d_part_cond.c:971-976): copied, not used
    (void)hidxb2;
    hk_set_error(0, nullptr);
    PcPlan P;
    if (!pc_plan(P, N, nx, nu, nb, hidxb, ng, N2)) return;
    const WLayout &O = P.orig, &C = P.cond;
    Carve c;
    const size_t oSt = c.take(sizeof(WideStage) * (N + 1)), oSt2 = c.take(sizeof(WideStage) * (N2 + 1)),
                 oBlk = c.take(sizeof(PcBlock) * N2), oIdx = c.take(4 * O.nI), oB = c.take(8 * O.nB),
                 oR = c.take(8 * O.nR), ohb = c.take(8 * O.nP), orq = c.take(8 * O.nU), oU2 = c.take(8 * C.nU),
                 oP2 = c.take(8 * C.nP), oL2 = c.take(8 * C.nD), oT2 = c.take(8 * C.nD), oU = c.take(8 * O.nU),
                 oP = c.take(8 * O.nP), oL = c.take(8 * O.nD), oT = c.take(8 * O.nD);
    if (!g_w.ensure(c.o)) return;
    char* H = g_w.host;
    memcpy(H + oSt, O.st.data(), sizeof(WideStage) * (N + 1));
    memcpy(H + oSt2, C.st.data(), sizeof(WideStage) * (N2 + 1));
    memcpy(H + oBlk, P.blk.data(), sizeof(PcBlock) * N2);
    memcpy(H + oIdx, P.idxb.data(), 4 * O.nI);
    auto dp = [&](size_t off) { return reinterpret_cast<double*>(H + off); };
    for (int k = 0; k <= N; k++) {
        const WideStage& s = O.st[k];
        const int nux = s.nu + s.nx;
        if (k < N) {
            memcpy(dp(oB) + s.oB, hpBAbt[k], (size_t)rup(nux + 1, BS) * s.sdB * sizeof(double));
            memcpy(dp(ohb) + s.oP, hb[k], s.nx1 * sizeof(double));
        }
        memcpy(dp(oR) + s.oR, hpRSQrq[k], (size_t)rup(nux + 1, BS) * s.sdR * sizeof(double));
        memcpy(dp(orq) + s.oU, hrq[k], nux * sizeof(double));
    }
    for (int k = 0; k <= N2; k++) {
        const WideStage& s = C.st[k];
        memcpy(dp(oU2) + s.oU, hux2[k], (s.nu + s.nx) * sizeof(double));
        if (k < N2) memcpy(dp(oP2) + s.oP, hpi2[k], s.nx1 * sizeof(double));
        const int nc = 2 * s.pnb + 2 * rup(s.ng, BS);
        if (nc > 0) {
            memcpy(dp(oL2) + s.oD, hlam2[k], nc * sizeof(double));
            memcpy(dp(oT2) + s.oD, ht2[k], nc * sizeof(double));
        }
    }
    char* D = g_w.dev;
    auto dd = [&](size_t off) { return reinterpret_cast<double*>(D + off); };
    PxArgs a;
    fill_px_args(P, a);
    a.nprob = 1;
    a.st = reinterpret_cast<const WideStage*>(D + oSt);
    a.st2 = reinterpret_cast<const WideStage*>(D + oSt2);
    a.blk = reinterpret_cast<const PcBlock*>(D + oBlk);
    a.idxb = reinterpret_cast<const int*>(D + oIdx);
    a.BAbt = dd(oB);
    a.RSQ = dd(oR);
    a.hb = dd(ohb);
    a.hrq = dd(orq);
    a.ux2 = dd(oU2);
    a.pi2 = dd(oP2);
    a.lam2 = dd(oL2);
    a.t2 = dd(oT2);
    a.ux = dd(oU);
    a.pi = dd(oP);
    a.lam = dd(oL);
    a.t = dd(oT);
    if (!g_w.up(c.o) || !launch(2, &a, 1, P.px_lds, g_w.stream, "hk_pexpand") || !g_w.down(c.o)) return;
    for (int k = 0; k <= N; k++) {
        const WideStage& s = O.st[k];
        memcpy(hux[k], dp(oU) + s.oU, (s.nu + s.nx) * sizeof(double));
        if (k < N) memcpy(hpi[k], dp(oP) + s.oP, s.nx1 * sizeof(double));
        const int nc = 2 * s.pnb + 2 * rup(s.ng, BS);
        if (s.nb + s.ng > 0) {
            // only the slots the reference writes: boxes [0, nb) / [pnb, pnb+nb) and, at N, the generals
            for (int l = 0; l < s.nb; l++) {
                hlam[k][l] = dp(oL)[s.oD + l];
                hlam[k][s.pnb + l] = dp(oL)[s.oD + s.pnb + l];
                ht[k][l] = dp(oT)[s.oD + l];
                ht[k][s.pnb + l] = dp(oT)[s.oD + s.pnb + l];
            }
            if (k == N)
                for (int l = 2 * s.pnb; l < nc; l++) {
                    hlam[k][l] = dp(oL)[s.oD + l];
                    ht[k][l] = dp(oT)[s.oD + l];
                }
        }
    }
}

// ------------------------------------------------------------------------------------------------
// Batched device API of the partial-condensing pipeline (data resident in HBM, problem-major).
// ------------------------------------------------------------------------------------------------
extern "C" hpmpc_mi355x_wide_plan* hpmpc_mi355x_wide_plan_create(int N, const int* nx, const int* nu, const int* nb,
                                                                 const int* const* idxb, const int* ng);
extern "C" void hpmpc_mi355x_wide_plan_destroy(hpmpc_mi355x_wide_plan* q);

struct hpmpc_mi355x_pcond_plan {
    PcPlan P;
    hpmpc_mi355x_wide_plan* wide = nullptr;  // the condensed problem's IPM plan (null: beyond the wide IPM)
    WideStage *d_st = nullptr, *d_st2 = nullptr;
    PcBlock* d_blk = nullptr;
    int* d_idxb = nullptr;
    int* d_idxb2 = nullptr;
};

extern "C" void hpmpc_mi355x_pcond_plan_destroy(hpmpc_mi355x_pcond_plan* q) {
    if (!q) return;
    if (q->d_st) (void)hipFree(q->d_st);
    if (q->d_st2) (void)hipFree(q->d_st2);
    if (q->d_blk) (void)hipFree(q->d_blk);
    if (q->d_idxb) (void)hipFree(q->d_idxb);
    if (q->d_idxb2) (void)hipFree(q->d_idxb2);
    hpmpc_mi355x_wide_plan_destroy(q->wide);
    delete q;
}

extern "C" hpmpc_mi355x_pcond_plan* hpmpc_mi355x_pcond_plan_create(int N, const int* nx, const int* nu, const int* nb,
                                                                   const int* const* idxb, const int* ng, int N2) {
    hk_set_error(0, nullptr);
    auto* q = new hpmpc_mi355x_pcond_plan();
    if (!pc_plan(q->P, N, nx, nu, nb, idxb, ng, N2)) {
        delete q;
        return nullptr;
    }
    const PcPlan& P = q->P;
    bool ok = hip_ok(hipMalloc((void**)&q->d_st, sizeof(WideStage) * (N + 1)), "pcond plan") &&
              hip_ok(hipMalloc((void**)&q->d_st2, sizeof(WideStage) * (N2 + 1)), "pcond plan") &&
              hip_ok(hipMalloc((void**)&q->d_blk, sizeof(PcBlock) * N2), "pcond plan") &&
              hip_ok(hipMalloc((void**)&q->d_idxb, 4 * P.orig.nI), "pcond plan") &&
              hip_ok(hipMalloc((void**)&q->d_idxb2, 4 * P.cond.nI), "pcond plan") &&
              hip_ok(hipMemcpy(q->d_st, P.orig.st.data(), sizeof(WideStage) * (N + 1), hipMemcpyHostToDevice), "plan") &&
              hip_ok(hipMemcpy(q->d_st2, P.cond.st.data(), sizeof(WideStage) * (N2 + 1), hipMemcpyHostToDevice),
                     "plan") &&
              hip_ok(hipMemcpy(q->d_blk, P.blk.data(), sizeof(PcBlock) * N2, hipMemcpyHostToDevice), "plan") &&
              hip_ok(hipMemcpy(q->d_idxb, P.idxb.data(), 4 * P.orig.nI, hipMemcpyHostToDevice), "plan");
    if (!ok) {
        hpmpc_mi355x_pcond_plan_destroy(q);
        return nullptr;
    }
    // the condensed problem's wide-stage IPM plan (hpmpc_mi355x_pcond_wide_plan); its DCt2 holds the blocks'
    // general constraints only, so a terminal stage with ng[N] > 0 leaves the plan without it
    if (ng[N] == 0) {
        std::vector<int*> i2(N2 + 1);
        for (int k = 0; k <= N2; k++) i2[k] = q->P.idxb2.data() + P.cond.st[k].oI;
        q->wide = hpmpc_mi355x_wide_plan_create(N2, P.nx2.data(), P.nu2.data(), P.nb2.data(), i2.data(),
                                                P.ng2.data());
        // the wide IPM indexes BAbt2 / RSQrq2 / DCt2 / d2 / ux2 / pi2 with its own layout: it must be exactly the
        // condensing kernels' carve (same per-problem sizes, same stage offsets), or it would read other blocks
        if (q->wide) {
            long long ws[8];
            std::vector<long long> wo(6 * (size_t)(N2 + 1));
            bool same = hpmpc_mi355x_wide_sizes(q->wide, ws) == 0 && hpmpc_mi355x_wide_offsets(q->wide, wo.data()) == 0;
            same = same && ws[0] == P.cond.nB && ws[1] == P.cond.nR && ws[2] == P.nG2 && ws[3] == P.cond.nD &&
                   ws[4] == P.cond.nU && ws[5] == P.cond.nP;
            for (int k = 0; same && k <= N2; k++) {
                const WideStage& s2 = P.cond.st[k];
                const long long* o = wo.data() + 6 * k;  // oB, oR, oG, oD, oU, oP
                same = o[0] == s2.oB && o[1] == s2.oR && o[3] == s2.oD && o[4] == s2.oU && o[5] == s2.oP &&
                       (k == N2 || P.ng2[k] == 0 || o[2] == P.blk[k].oG2);
            }
            if (!same) {
                fprintf(stderr, "hpmpc_mi355x: condensed wide IPM layout differs from the condensing carve\n");
                hpmpc_mi355x_wide_plan_destroy(q->wide);
                q->wide = nullptr;
            }
        }
    }
    hk_set_error(0, nullptr);  // a condensed problem beyond the wide IPM keeps the condense / Riccati pipeline
    return q;
}

// The condensed problem's IPM plan (owned by the pcond plan; null when the condensed stages exceed the wide
// IPM's limits or ng[N] > 0): hpmpc_mi355x_wide_ipm_batch on BAbt2 / RSQrq2 / DCt2 / d2 solves the condensed
// problems, hpmpc_mi355x_pexpand_batch expands their solution and multipliers.
extern "C" const hpmpc_mi355x_wide_plan* hpmpc_mi355x_pcond_wide_plan(const hpmpc_mi355x_pcond_plan* q) {
    if (!q || !q->wide) {
        hk_set_error(HPMPC_MI355X_EUNSUPPORTED, "no wide IPM plan for this condensed problem");
        return nullptr;
    }
    return q->wide;
}

// Per-problem sizes (doubles): [0] BAbt [1] RSQrq [2] d (=lam/t) [3] ux [4] pi of the original layout;
// [5] BAbt2 [6] RSQrq2 [7] DCt2 [8] d2 [9] ux2 [10] pi2 [11] condensed factor [12] Gamma scratch;
// [13] condensed stages N2, [14] max ng2 (the condensed Riccati needs 0).
extern "C" int hpmpc_mi355x_pcond_sizes(const hpmpc_mi355x_pcond_plan* q, long long* out) {
    if (!q) return HPMPC_MI355X_EUNSUPPORTED;
    const PcPlan& P = q->P;
    long long v[15] = {P.orig.nB, P.orig.nR, P.orig.nD, P.orig.nU, P.orig.nP, P.cond.nB, P.cond.nR, P.nG2,
                       P.cond.nD, P.cond.nU, P.cond.nP, P.cond.nL, P.nG, P.N2, 0};
    for (int k = 0; k <= P.N2; k++) v[14] = std::max<long long>(v[14], P.ng2[k]);
    memcpy(out, v, sizeof v);
    return 0;
}

// Stage offsets (doubles) of the layouts, for callers that fill / read the packed arrays:
// which = 0 original, 1 condensed; out[k*6 + 0..5] = oB, oR, oD, oU, oP, oL of stage k.
extern "C" int hpmpc_mi355x_pcond_offsets(const hpmpc_mi355x_pcond_plan* q, int which, long long* out) {
    if (!q) return HPMPC_MI355X_EUNSUPPORTED;
    const WLayout& L = which ? q->P.cond : q->P.orig;
    for (int k = 0; k <= L.N; k++) {
        const WideStage& s = L.st[k];
        const long long v[6] = {s.oB, s.oR, s.oD, s.oU, s.oP, s.oL};
        memcpy(out + 6 * k, v, sizeof v);
    }
    return 0;
}

extern "C" int hpmpc_mi355x_pcond_batch(const hpmpc_mi355x_pcond_plan* q, int nprob, int p0, int count,
                                        const double* BAbt, const double* RSQrq, const double* d, double* G,
                                        double* BAbt2, double* RSQrq2, double* DCt2, double* d2, void* stream) {
    if (!q) return HPMPC_MI355X_EUNSUPPORTED;
    hk_set_error(0, nullptr);
    if (((uintptr_t)BAbt | (uintptr_t)RSQrq) & 15) {  // hk_pcond copies their lib4 blocks by 16-byte LDS DMA
        hk_set_error(HPMPC_MI355X_EUNSUPPORTED, "pcond_batch: BAbt / RSQrq must be 16-byte aligned");
        return HPMPC_MI355X_EUNSUPPORTED;
    }
    PcArgs a;
    fill_pc_args(q->P, a);
    a.nprob = nprob;
    a.p0 = p0;
    a.st = q->d_st;
    a.blk = q->d_blk;
    a.idxb = q->d_idxb;
    a.BAbt = BAbt;
    a.RSQ = RSQrq;
    a.d = d;
    a.G = G;
    a.BAbt2 = BAbt2;
    a.RSQ2 = RSQrq2;
    a.DCt2 = DCt2;
    a.d2 = d2;
    a.idxb2 = q->d_idxb2;
    if (const char* e = getenv("HK_PCOND_SKIP")) a.skip = atoi(e);  // profiling only
    return launch(1, &a, count, q->P.pc_lds, (hipStream_t)stream, "hk_pcond") ? 0 : HPMPC_MI355X_EHIP;
}

extern "C" int hpmpc_mi355x_pcond_ric_sv_batch(const hpmpc_mi355x_pcond_plan* q, int nprob, int p0, int count,
                                               const double* BAbt2, const double* RSQrq2, double* ws, double* ux2,
                                               double* pi2, int compute_pi, void* stream) {
    if (!q) return HPMPC_MI355X_EUNSUPPORTED;
    hk_set_error(0, nullptr);
    const WLayout& C = q->P.cond;
    if (C.any_ng || !C.fits) {
        hk_set_error(HPMPC_MI355X_EUNSUPPORTED, "condensed Riccati with general constraints (state boxes) or "
                                                "beyond the wide-stage tile limits");
        return HPMPC_MI355X_EUNSUPPORTED;
    }
    WideArgs a;
    memset(&a, 0, sizeof a);
    a.N = C.N;
    a.nprob = nprob;
    a.p0 = p0;
    a.st = q->d_st2;
    a.BAbt = BAbt2;
    a.sB = C.nB;
    a.RSQ = RSQrq2;
    a.sR = C.nR;
    a.ws = ws;
    a.sW = C.nL;
    a.ux = ux2;
    a.pi = pi2;
    a.sU = C.nU;
    a.sP = C.nP;
    a.compute_pi = compute_pi;
    a.offW = C.offW;
    a.offX = C.offX;
    a.offV = C.offV;
    a.offST = C.offST;
    a.ldW = C.ldW;
    a.ldX = C.ldX;
    if (const char* e = getenv("HK_WIDE_SKIP")) a.skip = atoi(e);  // profiling only
    return launch(0, &a, count, C.lds, (hipStream_t)stream, "hk_wide_sv") ? 0 : HPMPC_MI355X_EHIP;
}

extern "C" int hpmpc_mi355x_pexpand_batch(const hpmpc_mi355x_pcond_plan* q, int nprob, int p0, int count,
                                          const double* BAbt, const double* RSQrq, const double* ux2,
                                          const double* pi2, const double* lam2, const double* t2, double* ux,
                                          double* pi, double* lam, double* t, void* stream) {
    if (!q) return HPMPC_MI355X_EUNSUPPORTED;
    hk_set_error(0, nullptr);
    PxArgs a;
    fill_px_args(q->P, a);
    a.nprob = nprob;
    a.p0 = p0;
    a.st = q->d_st;
    a.st2 = q->d_st2;
    a.blk = q->d_blk;
    a.idxb = q->d_idxb;
    a.BAbt = BAbt;
    a.RSQ = RSQrq;
    a.ux2 = ux2;
    a.pi2 = pi2;
    a.lam2 = lam2;
    a.t2 = t2;
    a.ux = ux;
    a.pi = pi;
    a.lam = lam;
    a.t = t;
    return launch(2, &a, count, q->P.px_lds, (hipStream_t)stream, "hk_pexpand") ? 0 : HPMPC_MI355X_EHIP;
}
