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
    int ng;                // general constraints (wide Riccati: 0)
};

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
    int offW, offX, offV;  // dynamic LDS carve (doubles): M packed | W | X | v
    int ldW, ldX;
    int skip;  // profiling only (HK_WIDE_SKIP): bit 0 forward, bit 1 Cholesky, bit 2 trmm/syrk -- results invalid
    int trf;   // d_back_ric_rec_trf_tv_res: no augmented row (stored as zeros), no forward
    // d_back_ric_rec_trs_tv_res (hk_wide_trs): b (offsets oP), q (offsets oU), qx (offsets oD, stride sC), idxb (oI)
    const double *hb, *hq, *qx;
    const int* idxb;
    long long sC;
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
    int skip;  // profiling only (HK_PCOND_SKIP): bit 0 Gamma, 1 RSQ phase, 2 its Cholesky, 3 M product, 4 W/syrk
};

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
