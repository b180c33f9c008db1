// hk_soft_args.h -- argument block of the soft-constraint IPM passes (hk_soft.hip), shared with the host C-ABI.
//
// d_ip2_mpc_soft_tv (mpc_solvers/d_ip2_soft.c:83-547): the Riccati steps run on the tile kernels (hk_ric_sv /
// hk_ric_trs with the box terms given per slot); these passes own the constraint vectors.  Per stage k the
// reference's vectors keep their layout (d_aux_ip_soft_lib4.c):
//   d             [lb (pnb) | ub (pnb) | ls (pns) | us (pns)]
//   t, lam, ...   [lo (pnb) | up (pnb) | s0 | s1 | s2 | s3 (pns each)]
//   Z, z          [lower (pns) | upper (pns)]
// and Qx / qx / Zl / zl live in one flat block in the reference's order (d_ip2_soft.c:244-260), because its
// soft gradient update writes past qx_k (d_aux_ip_soft_lib4.c:557, :601) and that write must land where it
// lands in the reference.  Plain C layout; every pointer is a device pointer; offsets in doubles.
#pragma once

struct SoftStage {
    int nu, nx, nx1;      // sizes (nx1 = nx_{k+1}, 0 at k = N)
    int nb, ns, pnb, pns;  // hard / soft boxes and their padded counts
    int oC;                // t / lam / dt / dlam / lamt / t_inv of stage k (2 pnb + 4 pns)
    int oD;                // d (2 pnb + 2 pns)
    int oZ;                // Z / z (2 pns)
    int oQ;                // Qx_k in the flat block; qx_k = oQ + pnb + pns
    int oZl;               // Zl_k in the flat block; zl_k = oZl + 2 pns
    int oS;                // target of the soft gradient term in the flat block (qx_k + pnbs + nb when nb > 0)
    int pad;
};

struct SoftArgs {
    int N, nprob, p0, k_max, warm_start, nq;  // nq = ceil((N+1)/4) stage quads
    const SoftStage* st;
    const int* idxb;  // 16 per stage (hard then soft), shared by the batch
    const double *d, *Z, *z;
    long long sD, sZ;
    double *t, *lam, *dt, *dlam, *lamt, *tinv;
    long long sC;
    double* flat;
    long long sF;
    double *ux, *pi;    // iterate, V16 per stage
    double *dux, *dpi;  // Riccati outputs, V16 per stage
    double *vQx, *vqx;  // Riccati box terms, V16 per stage (slot = position in idxb)
    long long sV;
    double mu0, mu_tol, alpha_min, mu_scal;
    double* scal;  // per problem, 4: mu, alpha, sigma, mu_aff
    int* ist;      // per problem, 4: kk, active, ret
    double* stat;  // per problem, 5 k_max
    long long sS;
};

// d_res_mpc_soft_tv (mpc_solvers/d_res_ip_soft.c:38-268): one 256-thread workgroup walks the stages of one
// problem.  Every input and output array of the call is copied into one buffer; SoftResStage holds each stage's
// sizes and offsets (doubles, -1 = absent).
struct SoftResStage {
    int nu, nx, nb, ng, ns, nx1, nu1;
    int pnb, png, pns, sdB, sdQ, sdG;
    int oB, oQ, oq, oZ, oz, oux, oux1, oG, od, opi, opim1, olam, ot, orq, orb, ord, orz, oI;
};

struct SoftResArgs {
    int N;
    const SoftResStage* st;
    const int* idxb;  // the caller's idxb rows, packed (oI)
    double* buf;      // inputs and outputs
    int omu;          // mu
};
