// hk_wide_args.h -- argument blocks of the wide-stage kernels (hk_wide.hip), shared with the host C-ABI.
//
// The wide path serves stages beyond the 16-wide register tile of hk_riccati.h: the condensed stages of
// partial condensing (nu+nx = 84 at the C5 configuration) and any caller problem with nu+nx > 16.  One
// 256-thread workgroup owns a problem (Riccati) or a (problem, block) pair (condensing); stage data are
// staged through LDS as dense column-major tiles.  Plain C layout; every pointer is a device pointer.
#pragma once

// One stage of a wide problem (ints; offsets in doubles inside one problem's arrays).
struct WideStage {
    int nu, nx, nx1, nu1;  // sizes of stage k and k+1 (nx1 = nu1 = 0 at k = N)
    int sdB, sdR;          // lib4 panel strides of BAbt_k / RSQrq_k
    int oB, oR;            // BAbt_k / RSQrq_k in the problem's packed stage arrays
    int oL;                // factor of stage k in ws: packed lower columns (nux+1 rows) then 1/diag (nux)
    int oU, oP;            // ux_k / pi_k (and Pb_k) in the problem's solution vectors
    int nb, pnb, oD, oI;   // boxes: count, padded count, d_k offset, idxb_k offset (ints)
    int ng;                // general constraints
    int oG, sdG;           // DCt_k (lib4, nux x ng, panel stride round_up(ng, 2)) in the problem's DCt array
};

static_assert(sizeof(WideStage) % sizeof(double) == 0, "LDS stage tables are carved in doubles");
// per stage: the last nonzero DCt column + 1 of each 16-row tile of M (8 tiles), then a 'recorded' flag
constexpr int KC_STRIDE = 9;

struct WideArgs {
    int N, nprob, p0;
    const WideStage* st;
    const double* BAbt;
    long long sB;
    const double* RSQ;
    long long sR;
    double* ws;  // factor per problem
    long long sW;
    double *ux, *pi, *Pb;  // solution vectors per problem (stage offsets oU / oP)
    long long sU, sP;
    int compute_pi, compute_Pb;
    int offW, offX, offV;  // dynamic LDS carve (doubles): M packed | W | X | v | stage table (offST)
    int offST;
    int ldW, ldX;
    int skip;  // profiling only (HK_WIDE_SKIP): bit 0 forward, bit 1 Cholesky, bit 2 trmm/syrk -- results invalid
    int trf;   // d_back_ric_rec_trf_tv_res: no augmented row (stored as zeros), no forward
    // d_back_ric_rec_trs_tv_res (hk_wide_trs): b (offsets oP), q (offsets oU), qx (offsets oD, stride sC), idxb (oI)
    const double *hb, *hq, *qx;
    const int* idxb;
    long long sC;
    // optional device-side terms of hk_wide_sv (the drop-in path applies them on the host instead):
    //   vb / vq: b_k / q_k from vectors (offsets oP / oU) instead of the augmented rows of BAbt_k / RSQrq_k;
    //   Qx (with qx): box terms diag[idxb] += Qx, row[idxb] += qx (dev_box), and the general terms
    //   DCt diag(Qx_g) DCt' / DCt qx_g, in the reference's [box (pnb) | general (png)] layout at offset oD;
    //   DCt: the general-constraint blocks (offsets oG, stride sG).  hk_wide_trs adds DCt qx_g when DCt is set.
    const double *vb, *vq, *Qx, *DCt;
    long long sG;
    int dev_box;  // hk_wide_sv: box terms from Qx / qx at idxb (else pre-applied in the staged RSQrq)
};

// Partial condensing (d_part_cond): one workgroup per (block ii, problem p).
struct PcBlock {
    int s0, T;                // first original stage of the block, its length
    int nx0, nut;             // the block's first state size, sum of its inputs
    int oG;                   // Gamma scratch of the block (doubles, inside the problem's scratch)
    int oB2, oR2, oG2, oD2;   // condensed BAbt2 / RSQrq2 / DCt2 / d2 of the block (packed condensed arrays)
    int oI2;                  // condensed idxb2 (ints)
    int nx2n;                 // nx of the next condensed stage (= nx[s0+T])
    int nb2, ng2;             // condensed box / general constraint counts
    int pad[2];
};

struct PcArgs {
    int N, N2, nprob, p0;
    const WideStage* st;     // original stages (oB, oR, oD, oI, nb, pnb)
    const PcBlock* blk;      // N2 blocks
    const double *BAbt, *RSQ, *d;
    const int* idxb;         // original idxb, packed per stage (oI), shared by the batch
    long long sB, sR, sD;
    double* G;               // Gamma scratch per problem
    long long sG;
    double *BAbt2, *RSQ2, *DCt2, *d2;
    int* idxb2;              // condensed idxb (written by problem 0 only: shared by the batch)
    long long sB2, sR2, sG2, sD2;
    int oR2N;                // terminal condensed RSQrq2 (a copy of RSQrq_N) in the packed condensed array
    int sdRN, nzN;           // its lib4 panel stride and rows
    int offP, offX, offW, offB, ldP, ldX, ldW, ldB;  // dynamic LDS carve
    int offGA, offGB;                                // Gamma_{j-1} / Gamma_j tiles (and stage scratch)
    int offST;                                       // the block's stage records (WideStage, T of them)
    int offU;                                        // P form: the u columns of pL_s ((nx+1) x nu, ld ldX)
    int pform;                                       // 0: every stage takes the Cholesky route (A/B, tests)
    int offGT;                                       // P form: the certificate bounds g_s of the block's stages
    int skip;  // profiling only (HK_PCOND_SKIP): bit 0 Gamma, 1 RSQ phase, 2 its Cholesky, 3 M product, 4 W/syrk
    int oD2N, nDN;  // terminal stage: its bounds d_N (original offset st[N].oD, nDN doubles) -> d2 at oD2N
    // phases (d_part_cond: PC_ALL).  Without PC_BABT the Gammas are inputs, already in the scratch G; PC_PART runs
    // one building block alone (d_cond_BAbt / _RSQrq / _DCtd): outputs are not cleared first (the caller's
    // contents stay where the reference writes nothing) and the terminal stage is not copied
    int ph;
    int gm;  // output tiles per wave of the kernel's gemms (4 or 8: the hk_pcond instance)
    int dm;  // full condensing (PC_ALL): d_cond_RSQrq first, the cross terms deferred to d_cond_BAbt (hk_pcond)
};
enum { PC_BABT = 1, PC_RSQ = 2, PC_DCTD = 4, PC_ALL = 7, PC_PART = 8 };

// Expansion (d_part_expand_solution): one workgroup per (block, problem).
struct PxArgs {
    int N, N2, nprob, p0;
    const WideStage* st;     // original stages (oU, oP for the full-space vectors)
    const PcBlock* blk;
    const WideStage* st2;    // condensed stages (oU, oP, pnb for the condensed vectors)
    const double *BAbt, *RSQ, *hb, *hrq;  // hb / hrq: per-stage b / rq (stage offsets oP / oU, strides sP / sU);
                                          // null = read from the augmented rows of BAbt / RSQrq
    const int* idxb;
    long long sB, sR, sU, sP, sC;   // sC: per-problem stride of the constraint vectors (lam/t)
    const double *ux2, *pi2, *lam2, *t2;
    long long sU2, sP2, sC2;
    double *ux, *pi, *lam, *t;
    int offB, offR, offV, offW, offQ, ldT;  // dynamic LDS carve: BAbt tile, RSQrq tile, ux_j, box terms, pi_j
};

// ------------------------------------------------------------------------------------------------
// The IPM on wide stages (hk_wide_ipm.hip): one workgroup runs a whole solve of one problem.
// ------------------------------------------------------------------------------------------------
// One constraint pair (lower / upper) of a problem's flattened constraint list (shared by the batch).
struct WideCSlot {
    int lo, up;  // its lower / upper slot in the constraint vectors ([lb | ub | lg | ug] at stage offset oD)
    int q;       // its Qx / qx entry ([box (pnb) | general (png)] at stage offset oD)
    int var;     // box: offset of its variable in ux (>= 0); general: -1 - stage
    int g;       // general: constraint index in the stage (column of DCt_k)
};

enum {
    WI_IPM_RES = 0,    // d_ip2_res_mpc_hard_tv            (mpc_solvers/d_ip2_res_hard.c:116-1345)
    WI_IPM_P1 = 1,     // d_ip2_mpc_hard_tv                (mpc_solvers/d_ip2_hard.c:88-614)
    WI_NEWTON = 2,     // d_ip2_res_mpc_hard_tv_single_newton_step (d_ip2_res_hard.c:1348-1919)
    WI_KKT_RES = 3,    // d_kkt_solve_new_rhs_res_mpc_hard_tv (d_ip2_res_hard.c:1922-2299)
    WI_KKT_P1 = 4,     // d_kkt_solve_new_rhs_mpc_hard_tv  (d_ip2_hard.c:626-825)
    WI_RES = 5,        // d_res_res_mpc_hard_tv            (mpc_solvers/c99/d_res_ip_res_hard.c:39-319)
    WI_RES_PLAIN = 6,  // d_res_mpc_hard_tv                (mpc_solvers/d_res_ip_hard.c:38-330)
};

struct WideIpmArgs {
    WideArgs w;  // stage table, LDS carve, BAbt / RSQ / DCt (+ strides), idxb; its vector slots are unused
    int mode, k_max, warm_start, compute_mult;
    double mu0, mu_tol, alpha_min;
    double mu_scal;  // 1 / (2 sum(nb + ng)); 0 without constraints
    double nbt2;     // 2 sum(nb + ng) (the residual routines divide by it)
    int ncs;
    const WideCSlot* cs;
    const int* vbox;  // per ux entry: lo slot of the box on that variable, -1 if none (problem-relative)
    int nU, nP;       // per-problem vector lengths (ux / pi layouts)
    const double* d;  // bounds (or r_C of the phase-1 KKT re-solve), stride sC
    double *ux, *pi, *lam, *t;  // iterate: strides w.sU, w.sP, sC
    long long sC;
    const double *vb, *vq;  // b / q vectors of the KKT re-solves and the residual routines (strides w.sP / w.sU)
    double* iw;             // per-problem work image (stride sI), offsets below
    long long sI;
    int oF, oDux, oDpi, oPb, oRq, oRb, oUb, oPib;
    int oDlam, oDt, oTinv, oLamt, oRd, oRm, oTb, oLb, oQx, oqx;
    double* stat;  // 5 * k_max per problem (stride sS)
    long long sS;
    int* kk;       // per problem: kk, return code
    int* ret;
    double* mu;    // per problem: final mu (residual routines: in / out)
    int offR;      // LDS reduction scratch (8 doubles) after the Riccati carve
    int offKC;     // LDS: the general-constraint chunk limits ((N+1) x KC_STRIDE ints) and their valid flag
};
