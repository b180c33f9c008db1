// hpmpc_kargs.h -- kernel argument block shared by the host C-ABI and the HIP kernels.
// Plain C layout; every pointer is a device pointer.  Per-problem arrays are problem-major with the
// stride given next to them (0 = shared by all problems, i.e. time-invariant / aliased data).
#pragma once

struct KArgs {
    int N, nprob, p0;             // horizon, problems in the batch, first problem of this launch
    int nbt;                      // sum of nb + ng over the stages
    int ngt;                      // sum of ng over the stages
    int fixcls;                   // compiled inner-stage class of the plan (0: generic kernels)
    const void* st;               // hk::StageInfo[N+1]
    const signed char* tileslot;  // (N+1)*16
    const signed char* slotvar;   // (N+1)*16
    const double* BAbt;           // lib4 stage blocks
    long long sB;
    const double* RSQ;
    long long sR;
    const double* d;  // bounds, V32 per stage: [lb (pnb) | ub (pnb) | lg (png) | ug (png)]
    const double* DCt;  // general constraints D_k' (lib4 nux x ng per stage, offsets in the stage table)
    long long sG;
    double* ws;       // per-problem workspace / factor memory
    long long sW;
    double *ux, *pi;  // V16 per stage (variable order / state order)
    double *lam, *t;  // V32 per stage
    long long sV16, sV32;
    // Riccati entry points: optional inputs (V16 per stage, same strides as ux)
    const double *vb, *vq, *vQx, *vqx;
    double* vPb;
    int update_b, update_q, use_box, compute_pi, compute_Pb;
    // IPM
    int k_max, warm_start, compute_mult, single_newton;
    int phase1_only;  // d_ip2_mpc_hard_tv (mpc_solvers/d_ip2_hard.c:88): the phase-1 loop alone, run to mu_tol
    int res_plain;    // d_res_mpc_hard_tv sign convention (mpc_solvers/d_res_ip_hard.c:305-326), no r_m
    double mu0, mu_tol, alpha_min;
    int *kk, *ret;
    double* stat;    // 5*k_max per problem
    double* mu_out;  // per problem (residual kernel)
    // problem queue (hpmpc_mi355x_ipm_queue): nq > 0 makes the grid a set of slots; slot s solves queue
    // entries one after another (entry q: data problem q % nprob, iterate/outputs at q, workspace s)
    int nq;
    int* qctl;  // [0] next entry to hand out, [1] entries finished, [2 + s] entry held by slot s (-1 none),
                // [2 + nslots + p] length of active-slot list p, [4 + nslots + p nslots ..] list p (p = 0, 1)
    unsigned long long* dbg;  // diagnostic stamp buffer (HK_STAMPS builds only)
    int nslots;  // queue slots
    int no_bkp;  // public queue API: the update pass writes no iterate backups (only the KKT re-solve reads them)
    int qpar;    // queue tick parity: workgroup i of an iteration kernel runs slot list[qpar][i]; the update
                 // pass lists the slots that iterate again in list qpar ^ 1 (hk_ipm_init fills list qpar)
    int* dctr;   // queue: [0] iterations and [1] problems the multi-wave drain finished (summed over lanes)
    int* qnext;  // queue: the next entry to hand out, shared by the lanes
};
