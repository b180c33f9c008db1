/*
 * hpmpc_oracle.c -- TEST INFRASTRUCTURE ONLY (parity checker; see hpmpc_oracle.h).
 *
 * A clean-room, scalar, dense restatement of the HPMPC c99 hot path.  Matrices are read from and
 * written to the caller's lib4 panel-major buffers exactly where the reference reads/writes them
 * (including its documented in-place side effects on hpRSQrq / hpBAbt); all arithmetic happens on
 * small dense column-major temporaries.  Summation order follows the mathematical statement, not
 * the reference's 4x4 register blocking, so results agree with the reference to rounding
 * (|diff| ~ 1e-15 relative), not bit for bit.  The pinning of this restatement against the real
 * reference (oracle/_ref) is in tests/golden + tests/test_oracle_golden.py.
 *
 * Reference anchors (relative to the reference checkout):
 *   lib4 addressing         include/block_size.h:62-72, auxiliary/d_aux_lib4.c:1310
 *   Riccati sv              lqcp_solvers/d_back_ric_rec.c:112-399
 *   Riccati trf             lqcp_solvers/d_back_ric_rec.c:403-560
 *   Riccati trs             lqcp_solvers/d_back_ric_rec.c:564-791
 *   fused syrk+potrf clamp  kernel/c99/kernel_dpotrf_c99_lib4.c:555-640 (pivot > 1e-15 else 0)
 *   IPM                     mpc_solvers/d_ip2_res_hard.c:116-1345, 1348-1919, 1922-2299
 *   IPM vector kernels      mpc_solvers/c99/d_aux_ip_hard_lib4.c:43-1639
 *   KKT residuals           mpc_solvers/c99/d_res_ip_res_hard.c:39-319
 */
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "hpmpc_oracle.h"

#define BS 4  /* D_MR   (include/block_size.h:62-72, TARGET_C99_4X4) */
#define NCL 2 /* D_NCL */

static inline int rup(int n, int m) { return (n + m - 1) / m * m; }

/* element (i,j) of a lib4 matrix with panel stride sd (columns per panel) */
static inline double *P4(double *pA, int sd, int i, int j) { return pA + (i / BS) * BS * sd + i % BS + BS * j; }

/* ------------------------------------------------------------------------------------------------
 * Riccati "memory" (oracle-private layout): for every stage k = 0..N a dense column-major factor
 * L_k of (nux_k+1) rows x nux_k cols (ld = nux_k+1; last row = transformed gradient l_k), followed
 * by the inverse diagonal dL_k (nux_k).
 * ---------------------------------------------------------------------------------------------- */
static int stage_nux(int k, int N, const int *nx, const int *nu) { return (k < N ? nu[k] : 0) + nx[k]; }

static void carve_factor(int N, const int *nx, const int *nu, double *memory, double **L, double **dL) {
    double *p = memory;
    for (int k = 0; k <= N; k++) {
        int nux = stage_nux(k, N, nx, nu);
        L[k] = p;
        p += (nux + 1) * nux;
        dL[k] = p;
        p += nux;
    }
}

int orc_d_back_ric_rec_sv_tv_memory_space_size_bytes(int N, int *nx, int *nu, int *nb, int *ng) {
    long s = 0;
    for (int k = 0; k <= N; k++) {
        int nux = stage_nux(k, N, nx, nu);
        s += (nux + 1) * nux + nux;
    }
    return (int)((s * 8 + 63) / 64 * 64);
}

int orc_d_back_ric_rec_sv_tv_work_space_size_bytes(int N, int *nx, int *nu, int *nb, int *ng) {
    /* dense W (nz x (nx'+ng)), Wg, M (nz x nux), 3 vectors */
    int nzM = 0, nxgM = 0;
    for (int k = 0; k <= N; k++) {
        int nux = stage_nux(k, N, nx, nu);
        if (nux + 1 > nzM) nzM = nux + 1;
        int g = (k < N ? nx[k + 1] : 0) + ng[k];
        if (g > nxgM) nxgM = g;
    }
    long s = 2L * nzM * nxgM + (long)nzM * nzM + 4L * nzM + 8;
    return (int)((s * 8 + 63) / 64 * 64);
}

/* Cholesky of the leading n x n block of the dense symmetric M (lower part used), with the extra
 * rows n..m-1 solved against it (the "augmented row" trick, d_back_ric_rec.c:146,194,259,345).
 * Left-looking; pivot d > 1e-15 else the column is zeroed (kernel_dpotrf_c99_lib4.c:555-640). */
void orc__chol_aug(int m, int n, double *M, int ldm, double *L, int ldl, double *dL);
static void chol_aug(int m, int n, double *M, int ldm, double *L, int ldl, double *dL) {
    for (int j = 0; j < n; j++) {
        for (int i = j; i < m; i++) {
            double c = M[i + j * ldm];
            for (int l = 0; l < j; l++) c -= L[i + l * ldl] * L[j + l * ldl];
            M[i + j * ldm] = c;
        }
        double d = M[j + j * ldm], s, inv;
        if (d > 1e-15) {
            s = sqrt(d);
            inv = 1.0 / s;
        } else {
            s = 0.0;
            inv = 0.0;
        }
        L[j + j * ldl] = s;
        dL[j] = inv;
        for (int i = j + 1; i < m; i++) L[i + j * ldl] = M[i + j * ldm] * inv;
        for (int i = 0; i < j; i++) L[i + j * ldl] = 0.0; /* strictly upper part kept zero */
    }
}

/* Factorise one stage.  aug=1: (nux+1) rows (sv); aug=0: nux rows (trf).
 * Side effects on hpRSQrq / hpBAbt mirror d_back_ric_rec.c:186-244 (terminal) and :248-335. */
static void stage_factor(int k, int N, int *nx, int *nu, int *nb, int **idxb, int *ng, int aug, int update_b,
                         double **hpBAbt, double **b, int update_q, double **hpRSQrq, double **q, double **bd,
                         double **hpDCt, double **Qx, double **qx, int compute_Pb, double **hPb, double **L,
                         double **dL, double *work) {
    const int nuk = k < N ? nu[k] : 0;
    const int nux = nuk + nx[k];
    const int cnux = rup(nux, NCL);
    const int nz = nux + (aug ? 1 : 0);
    const int ldm = nux + 1;
    const int nx1 = k < N ? nx[k + 1] : 0;
    const int ngk = ng[k];
    const int pnb = rup(nb[k], BS);
    const int cng = rup(ngk, NCL);
    double *M = work;                    /* ldm x nux */
    double *W = M + ldm * (nux > 0 ? nux : 1); /* ldm x (nx1+ngk) */
    double *RSQ = hpRSQrq[k];

    /* update_q: write q into the augmented row of RSQrq (:197-201, :279-283) */
    if (aug && update_q)
        for (int j = 0; j < nux; j++) *P4(RSQ, cnux, nux, j) = q[k][j];
    /* box: diag[idxb] = bd + Qx (ddiaadin_libsp), aug row[idxb] += qx (drowad_libsp) (:203-209, :284-291) */
    if (nb[k] > 0) {
        for (int l = 0; l < nb[k]; l++) {
            int ii = idxb[k][l];
            *P4(RSQ, cnux, ii, ii) = bd[k][l] + Qx[k][l];
        }
        if (aug)
            for (int l = 0; l < nb[k]; l++) *P4(RSQ, cnux, nux, idxb[k][l]) += qx[k][l];
    }

    /* M = lower(RSQrq) including the augmented row */
    for (int j = 0; j < nux; j++)
        for (int i = j; i < nz; i++) M[i + j * ldm] = *P4(RSQ, cnux, i, j);

    if (k < N) {
        /* W = BAbt_k * Lxx_{k+1}, Lxx lower (dtrmm_nt_u_lib on the transposed copy, :262-264) */
        const int nu1 = (k + 1 < N) ? nu[k + 1] : 0;
        const int nux1 = nu1 + nx1;
        const int ld1 = nux1 + 1;
        const int cnx1 = rup(nx1, NCL);
        double *BAbt = hpBAbt[k];
        double *L1 = L[k + 1];
        if (aug && update_b)
            for (int j = 0; j < nx1; j++) *P4(BAbt, cnx1, nux, j) = b[k][j];
        for (int j = 0; j < nx1; j++)
            for (int i = 0; i < nz; i++) {
                double c = 0.0;
                for (int r = j; r < nx1; r++) c += *P4(BAbt, cnx1, i, r) * L1[(nu1 + r) + (nu1 + j) * ld1];
                W[i + j * ldm] = c;
            }
        if (aug) {
            /* Pb_k = Lxx (Lxx' b) from the last row of W before adding l (:266-276) */
            if (compute_Pb)
                for (int i = 0; i < nx1; i++) {
                    double c = 0.0;
                    for (int j = 0; j <= i; j++) c += L1[(nu1 + i) + (nu1 + j) * ld1] * W[nux + j * ldm];
                    hPb[k][i] = c;
                }
            /* dgead: last row of W += l_{k+1,x} (:276) */
            for (int j = 0; j < nx1; j++) W[nux + j * ldm] += L1[nux1 + (nu1 + j) * ld1];
        }
        /* M += W W' (lower, incl. augmented row) */
        for (int j = 0; j < nux; j++)
            for (int i = j; i < nz; i++) {
                double c = 0.0;
                for (int r = 0; r < nx1; r++) c += W[i + r * ldm] * W[j + r * ldm];
                M[i + j * ldm] += c;
            }
    }
    if (ngk > 0) {
        /* general constraints: Wg = DCt diag(Qx_g), last row qx_g; M += Wg DCt' (:210-231, :292-317) */
        double *DCt = hpDCt[k];
        for (int j = 0; j < nux; j++)
            for (int i = j; i < nz; i++) {
                double c = 0.0;
                for (int g = 0; g < ngk; g++) {
                    double wig = (i < nux) ? *P4(DCt, cng, i, g) * Qx[k][pnb + g] : qx[k][pnb + g];
                    c += wig * *P4(DCt, cng, j, g);
                }
                M[i + j * ldm] += c;
            }
    }
    chol_aug(nz, nux, M, ldm, L[k], ldm, dL[k]);
    if (!aug)
        for (int j = 0; j < nux; j++) L[k][nux + j * ldm] = 0.0;
}

/* y[0:n] = solve L[0:n,0:n]' y1 = x1 - L[n:m,0:n]' x2   (dtrsv_t_lib, blas_d_lib4.c:5276; inv_diag) */
static void trsv_t(int m, int n, const double *L, int ld, const double *dL, double *x) {
    for (int i = n - 1; i >= 0; i--) {
        double c = x[i];
        for (int j = i + 1; j < m; j++) c -= L[j + i * ld] * x[j];
        x[i] = c * dL[i];
    }
}

/* L[0:n,0:n] y1 = x1 ; y2 = x2 - L[n:m,0:n] y1    (dtrsv_n_lib, blas_d_lib4.c:5204; inv_diag) */
static void trsv_n(int m, int n, const double *L, int ld, const double *dL, double *x) {
    for (int j = 0; j < n; j++) {
        double yj = x[j];
        for (int l = 0; l < j; l++) yj -= L[j + l * ld] * x[l];
        x[j] = yj * dL[j];
    }
    for (int i = n; i < m; i++) {
        double c = x[i];
        for (int l = 0; l < n; l++) c -= L[i + l * ld] * x[l];
        x[i] = c;
    }
}

/* pi = Lxx (Lxx' x + p)  (dtrmv_u_n + dtrmv_u_t on the transposed copy, d_back_ric_rec.c:355-365) */
static void pi_from_x(int nx1, const double *L1, int ld1, int nu1, const double *x, const double *p, double *pi,
                      double *tmp) {
    for (int j = 0; j < nx1; j++) {
        double c = p ? p[j] : 0.0;
        for (int i = j; i < nx1; i++) c += L1[(nu1 + i) + (nu1 + j) * ld1] * x[i];
        tmp[j] = c;
    }
    for (int i = 0; i < nx1; i++) {
        double c = 0.0;
        for (int j = 0; j <= i; j++) c += L1[(nu1 + i) + (nu1 + j) * ld1] * tmp[j];
        pi[i] = c;
    }
}

void orc_d_back_ric_rec_sv_tv_res(int N, int *nx, int *nu, int *nb, int **idxb, int *ng, int update_b,
                                  double **hpBAbt, double **b, int update_q, double **hpRSQrq, double **q,
                                  double **bd, double **hpDCt, double **Qx, double **qx, double **hux,
                                  int compute_pi, double **hpi, int compute_Pb, double **hPb, double *memory,
                                  double *work) {
    double *L[N + 1], *dL[N + 1];
    carve_factor(N, nx, nu, memory, L, dL);
    for (int k = N; k >= 0; k--)
        stage_factor(k, N, nx, nu, nb, idxb, ng, 1, update_b, hpBAbt, b, update_q, hpRSQrq, q, bd, hpDCt, Qx, qx,
                     compute_Pb, hPb, L, dL, work);
    /* forward substitution (:339-397) */
    int nxM = 1;
    for (int k = 0; k <= N; k++) nxM = nx[k] > nxM ? nx[k] : nxM;
    double tmp[nxM], p[nxM];
    for (int k = 0; k < N; k++) {
        const int nux = nu[k] + nx[k], ld = nux + 1;
        const int nx1 = nx[k + 1];
        const int nu1 = (k + 1 < N) ? nu[k + 1] : 0;
        const int ld1 = nu1 + nx1 + 1;
        const int cnx1 = rup(nx1, NCL);
        const int ns = (k == 0) ? nux : nu[k]; /* stage 0 solves the full block */
        for (int j = 0; j < ns; j++) hux[k][j] = -L[k][nux + j * ld];
        trsv_t(nux, ns, L[k], ld, dL[k], hux[k]);
        for (int j = 0; j < nx1; j++) {
            double c = *P4(hpBAbt[k], cnx1, nux, j);
            for (int i = 0; i < nux; i++) c += *P4(hpBAbt[k], cnx1, i, j) * hux[k][i];
            hux[k + 1][nu1 + j] = c;
        }
        if (compute_pi) {
            for (int j = 0; j < nx1; j++) p[j] = L[k + 1][(nu1 + nx1) + (nu1 + j) * ld1];
            pi_from_x(nx1, L[k + 1], ld1, nu1, hux[k + 1] + nu1, p, hpi[k], tmp);
        }
    }
}

void orc_d_back_ric_rec_trf_tv_res(int N, int *nx, int *nu, int *nb, int **idxb, int *ng, double **hpBAbt,
                                   double **hpRSQrq, double **hpDCt, double **Qx, double **bd, double *memory,
                                   double *work) {
    double *L[N + 1], *dL[N + 1];
    carve_factor(N, nx, nu, memory, L, dL);
    for (int k = N; k >= 0; k--)
        stage_factor(k, N, nx, nu, nb, idxb, ng, 0, 0, hpBAbt, NULL, 0, hpRSQrq, NULL, bd, hpDCt, Qx, NULL, 0,
                     NULL, L, dL, work);
}

/* g_k = q_k + qx at idxb + DCt qx_g  (dvecad_libsp + dgemv_n_lib, d_back_ric_rec.c:612-633) */
static void stage_gradient(int k, int N, int *nx, int *nu, int *nb, int **idxb, int *ng, double **hq,
                           double **hpDCt, double **qx, double *g) {
    const int nux = (k < N ? nu[k] : 0) + nx[k];
    for (int i = 0; i < nux; i++) g[i] = hq[k][i];
    const int pnb = rup(nb[k], BS);
    for (int l = 0; l < nb[k]; l++) g[idxb[k][l]] += qx[k][l];
    if (ng[k] > 0) {
        const int cng = rup(ng[k], NCL);
        for (int i = 0; i < nux; i++) {
            double c = 0.0;
            for (int l = 0; l < ng[k]; l++) c += *P4(hpDCt[k], cng, i, l) * qx[k][pnb + l];
            g[i] += c;
        }
    }
}

void orc_d_back_ric_rec_trs_tv_res(int N, int *nx, int *nu, int *nb, int **idxb, int *ng, double **hpBAbt,
                                   double **hb, double **hq, double **hpDCt, double **qx, double **hux,
                                   int compute_pi, double **hpi, int compute_Pb, double **hPb, double *memory,
                                   double *work) {
    double *L[N + 1], *dL[N + 1];
    carve_factor(N, nx, nu, memory, L, dL);
    int nxM = 1;
    for (int k = 0; k <= N; k++) nxM = nx[k] > nxM ? nx[k] : nxM;
    double tmp[nxM], w[nxM], pk[nxM];
    /* backward (:604-700) */
    stage_gradient(N, N, nx, nu, nb, idxb, ng, hq, hpDCt, qx, hux[N]);
    for (int k = N - 1; k >= 0; k--) {
        const int nux = nu[k] + nx[k], ld = nux + 1;
        const int nx1 = nx[k + 1];
        const int nu1 = (k + 1 < N) ? nu[k + 1] : 0;
        const int ld1 = nu1 + nx1 + 1;
        const int cnx1 = rup(nx1, NCL);
        if (compute_Pb) pi_from_x(nx1, L[k + 1], ld1, nu1, hb[k], NULL, hPb[k], tmp);
        stage_gradient(k, N, nx, nu, nb, idxb, ng, hq, hpDCt, qx, hux[k]);
        for (int j = 0; j < nx1; j++) w[j] = hPb[k][j] + hux[k + 1][nu1 + j];
        for (int i = 0; i < nux; i++) {
            double c = 0.0;
            for (int j = 0; j < nx1; j++) c += *P4(hpBAbt[k], cnx1, i, j) * w[j];
            hux[k][i] += c;
        }
        trsv_n(nux, k == 0 ? nux : nu[k], L[k], ld, dL[k], hux[k]);
    }
    /* forward (:704-790) */
    for (int k = 0; k < N; k++) {
        const int nux = nu[k] + nx[k], ld = nux + 1;
        const int nx1 = nx[k + 1];
        const int nu1 = (k + 1 < N) ? nu[k + 1] : 0;
        const int ld1 = nu1 + nx1 + 1;
        const int cnx1 = rup(nx1, NCL);
        const int ns = (k == 0) ? nux : nu[k];
        if (compute_pi)
            for (int j = 0; j < nx1; j++) hpi[k][j] = hux[k + 1][nu1 + j];
        for (int j = 0; j < ns; j++) hux[k][j] = -hux[k][j];
        trsv_t(nux, ns, L[k], ld, dL[k], hux[k]);
        for (int j = 0; j < nx1; j++) {
            double c = hb[k][j];
            for (int i = 0; i < nux; i++) c += *P4(hpBAbt[k], cnx1, i, j) * hux[k][i];
            hux[k + 1][nu1 + j] = c;
        }
        if (compute_pi) {
            for (int j = 0; j < nx1; j++) pk[j] = hpi[k][j];
            pi_from_x(nx1, L[k + 1], ld1, nu1, hux[k + 1] + nu1, NULL, hpi[k], tmp);
            for (int j = 0; j < nx1; j++) hpi[k][j] += pk[j];
        }
    }
}

/* ================================================================================================
 * Residuals  (mpc_solvers/c99/d_res_ip_res_hard.c:39-319)
 * ============================================================================================== */
void orc_d_res_res_mpc_hard_tv(int N, int *nx, int *nu, int *nb, int **idxb, int *ng, double **hpBAbt, double **hb,
                               double **hpQ, double **hq, double **hux, double **hpDCt, double **hd, double **hpi,
                               double **hlam, double **ht, double *work, double **hrq, double **hrb, double **hrd,
                               double **hrm, double *mu) {
    int nb_tot = 0;
    double mu2 = 0.0;
    for (int k = 0; k <= N; k++) {
        const int nuk = nu[k]; /* nu[N] == 0 */
        const int nux = nuk + nx[k];
        const int cnux = rup(nux, NCL);
        const int pnb = rup(nb[k], BS), png = rup(ng[k], BS), cng = rup(ng[k], NCL);
        for (int j = 0; j < nux; j++) hrq[k][j] = hq[k][j];
        if (k > 0)
            for (int j = 0; j < nx[k]; j++) hrq[k][nuk + j] -= hpi[k - 1][j];
        if (nb[k] > 0) {
            nb_tot += nb[k];
            for (int l = 0; l < nb[k]; l++) {
                int ii = idxb[k][l];
                hrq[k][ii] += -hlam[k][l] + hlam[k][pnb + l];
                hrd[k][l] = hd[k][l] - hux[k][ii] + ht[k][l];
                hrd[k][pnb + l] = hd[k][pnb + l] - hux[k][ii] - ht[k][pnb + l];
                hrm[k][l] = hlam[k][l] * ht[k][l];
                hrm[k][pnb + l] = hlam[k][pnb + l] * ht[k][pnb + l];
                mu2 += hrm[k][l] + hrm[k][pnb + l];
            }
        }
        /* r_q += RSQ ux  (dsymv_lib, lower triangle) */
        for (int i = 0; i < nux; i++) {
            double c = 0.0;
            for (int j = 0; j < nux; j++) c += (i >= j ? *P4(hpQ[k], cnux, i, j) : *P4(hpQ[k], cnux, j, i)) * hux[k][j];
            hrq[k][i] += c;
        }
        if (k < N) {
            const int nx1 = nx[k + 1], nu1 = (k + 1 < N) ? nu[k + 1] : 0, cnx1 = rup(nx1, NCL);
            for (int j = 0; j < nx1; j++) hrb[k][j] = hb[k][j] - hux[k + 1][nu1 + j];
            /* dgemv_nt: r_q += BAbt pi ; r_b += BAbt' ux */
            for (int i = 0; i < nux; i++) {
                double c = 0.0;
                for (int j = 0; j < nx1; j++) c += *P4(hpBAbt[k], cnx1, i, j) * hpi[k][j];
                hrq[k][i] += c;
            }
            for (int j = 0; j < nx1; j++) {
                double c = 0.0;
                for (int i = 0; i < nux; i++) c += *P4(hpBAbt[k], cnx1, i, j) * hux[k][i];
                hrb[k][j] += c;
            }
        }
        if (ng[k] > 0) {
            nb_tot += ng[k];
            double *wl = work, *wc = work + png;
            for (int l = 0; l < ng[k]; l++) {
                wl[l] = hlam[k][2 * pnb + png + l] - hlam[k][2 * pnb + l];
                hrd[k][2 * pnb + l] = hd[k][2 * pnb + l] + ht[k][2 * pnb + l];
                hrd[k][2 * pnb + png + l] = hd[k][2 * pnb + png + l] - ht[k][2 * pnb + png + l];
                hrm[k][2 * pnb + l] = hlam[k][2 * pnb + l] * ht[k][2 * pnb + l];
                hrm[k][2 * pnb + png + l] = hlam[k][2 * pnb + png + l] * ht[k][2 * pnb + png + l];
                mu2 += hrm[k][2 * pnb + l] + hrm[k][2 * pnb + png + l];
            }
            for (int i = 0; i < nux; i++) {
                double c = 0.0;
                for (int l = 0; l < ng[k]; l++) c += *P4(hpDCt[k], cng, i, l) * wl[l];
                hrq[k][i] += c;
            }
            for (int l = 0; l < ng[k]; l++) {
                double c = 0.0;
                for (int i = 0; i < nux; i++) c += *P4(hpDCt[k], cng, i, l) * hux[k][i];
                wc[l] = c;
                hrd[k][2 * pnb + l] -= c;
                hrd[k][2 * pnb + png + l] -= c;
            }
        }
    }
    if (nb_tot != 0) *mu = mu2 / (2.0 * nb_tot);
}

/* ================================================================================================
 * IPM vector kernels (mpc_solvers/c99/d_aux_ip_hard_lib4.c).  Constraint vectors use the padded
 * [lb (pnb) | ub (pnb) | lg (png) | ug (png)] layout; Qx/qx use [box (pnb) | general (png)].
 * ============================================================================================== */
typedef struct {
    int nb, pnb, ng, png;
} cdim_t;
static cdim_t cdim(int *nb, int *ng, int k) {
    cdim_t c = {nb[k], rup(nb[k], BS), ng[k], rup(ng[k], BS)};
    return c;
}

/* step length update, sequential over stages and constraints exactly as :541-565 */
static inline void alpha_upd_pair(double *alpha, double *lam, double *dlam, double *t, double *dt, int i, int off) {
    if (-*alpha * dlam[i] > lam[i]) *alpha = -lam[i] / dlam[i];
    if (-*alpha * dlam[i + off] > lam[i + off]) *alpha = -lam[i + off] / dlam[i + off];
    if (-*alpha * dt[i] > t[i]) *alpha = -t[i] / dt[i];
    if (-*alpha * dt[i + off] > t[i + off]) *alpha = -t[i + off] / dt[i + off];
}

/* DCt' v  (dgemv_t_lib with alg 0) */
static void dct_t(int k, int *nu, int *nx, int *ng, double **hpDCt, const double *v, double *out) {
    const int nux = nu[k] + nx[k], cng = rup(ng[k], NCL);
    for (int l = 0; l < ng[k]; l++) {
        double c = 0.0;
        for (int i = 0; i < nux; i++) c += *P4(hpDCt[k], cng, i, l) * v[i];
        out[l] = c;
    }
}

/* d_aux_ip_hard_lib4.c:43-149 */
static void init_var(int N, int *nx, int *nu, int *nb, int **idxb, int *ng, double **ux, double **pi,
                     double **pDCt, double **db, double **t, double **lam, double mu0, int warm_start) {
    const double thr0 = 0.1;
    if (!warm_start)
        for (int k = 0; k <= N; k++)
            for (int l = 0; l < nu[k] + nx[k]; l++) ux[k][l] = 0.0;
    for (int k = 0; k <= N; k++) {
        cdim_t c = cdim(nb, ng, k);
        for (int l = 0; l < c.nb; l++) {
            int ii = idxb[k][l];
            t[k][l] = -db[k][l] + ux[k][ii];
            t[k][c.pnb + l] = db[k][c.pnb + l] - ux[k][ii];
            if (t[k][l] < thr0) {
                if (t[k][c.pnb + l] < thr0) {
                    ux[k][ii] = (-db[k][c.pnb + l] + db[k][l]) * 0.5;
                    t[k][l] = thr0;
                    t[k][c.pnb + l] = thr0;
                } else {
                    t[k][l] = thr0;
                    ux[k][ii] = db[k][l] + thr0;
                }
            } else if (t[k][c.pnb + l] < thr0) {
                t[k][c.pnb + l] = thr0;
                ux[k][ii] = db[k][c.pnb + l] - thr0;
            }
            lam[k][l] = mu0 / t[k][l];
            lam[k][c.pnb + l] = mu0 / t[k][c.pnb + l];
        }
    }
    for (int k = 0; k < N; k++)
        for (int l = 0; l < nx[k + 1]; l++) pi[k][l] = 0.0;
    for (int k = 0; k <= N; k++) {
        cdim_t c = cdim(nb, ng, k);
        if (c.ng > 0) {
            double *tt = t[k] + 2 * c.pnb, *ll = lam[k] + 2 * c.pnb, *dd = db[k] + 2 * c.pnb;
            dct_t(k, nu, nx, ng, pDCt, ux[k], tt);
            for (int l = 0; l < c.ng; l++) {
                tt[l + c.png] = -tt[l];
                tt[l] += -dd[l];
                tt[l + c.png] += dd[l + c.png];
                tt[l] = fmax(thr0, tt[l]);
                tt[c.png + l] = fmax(thr0, tt[c.png + l]);
                ll[l] = mu0 / tt[l];
                ll[c.png + l] = mu0 / tt[c.png + l];
            }
        }
    }
}

/* d_aux_ip_hard_lib4.c:217-383 */
static void update_hessian(int N, int *nb, int *ng, double **db, double sigma_mu, double **t, double **t_inv,
                           double **lam, double **lamt, double **dlam, double **Qx, double **qx) {
    for (int k = 0; k <= N; k++) {
        cdim_t c = cdim(nb, ng, k);
        int segs[2][3] = {{c.nb, c.pnb, 0}, {c.ng, c.png, 2 * c.pnb}};
        int qoff[2] = {0, c.pnb};
        for (int s = 0; s < 2; s++) {
            int n = segs[s][0], p = segs[s][1], o = segs[s][2];
            for (int i = 0; i < n; i++) {
                int a = o + i, b2 = o + p + i;
                t_inv[k][a] = 1.0 / t[k][a];
                t_inv[k][b2] = 1.0 / t[k][b2];
                lamt[k][a] = lam[k][a] * t_inv[k][a];
                lamt[k][b2] = lam[k][b2] * t_inv[k][b2];
                dlam[k][a] = t_inv[k][a] * sigma_mu;
                dlam[k][b2] = t_inv[k][b2] * sigma_mu;
                Qx[k][qoff[s] + i] = lamt[k][a] + lamt[k][b2];
                qx[k][qoff[s] + i] = lam[k][b2] - lamt[k][b2] * db[k][b2] + dlam[k][b2] - lam[k][a] -
                                     lamt[k][a] * db[k][a] - dlam[k][a];
            }
        }
    }
}

/* d_aux_ip_hard_lib4.c:387-485 */
static void update_gradient(int N, int *nb, int *ng, double sigma_mu, double **dt, double **dlam, double **t_inv,
                            double **qx) {
    for (int k = 0; k <= N; k++) {
        cdim_t c = cdim(nb, ng, k);
        int segs[2][3] = {{c.nb, c.pnb, 0}, {c.ng, c.png, 2 * c.pnb}};
        int qoff[2] = {0, c.pnb};
        for (int s = 0; s < 2; s++) {
            int n = segs[s][0], p = segs[s][1], o = segs[s][2];
            for (int i = 0; i < n; i++) {
                int a = o + i, b2 = o + p + i;
                dlam[k][a] = t_inv[k][a] * (sigma_mu - dlam[k][a] * dt[k][a]);
                dlam[k][b2] = t_inv[k][b2] * (sigma_mu - dlam[k][b2] * dt[k][b2]);
                qx[k][qoff[s] + i] += dlam[k][b2] - dlam[k][a];
            }
        }
    }
}

/* d_aux_ip_hard_lib4.c:489-614 */
static void compute_alpha(int N, int *nx, int *nu, int *nb, int **idxb, int *ng, double *ptr_alpha, double **t,
                          double **dt, double **lam, double **dlam, double **lamt, double **dux, double **pDCt,
                          double **db) {
    double alpha = *ptr_alpha;
    for (int k = 0; k <= N; k++) {
        cdim_t c = cdim(nb, ng, k);
        for (int l = 0; l < c.nb; l++) {
            int ii = idxb[k][l], u = c.pnb + l;
            dt[k][l] = dux[k][ii] - db[k][l] - t[k][l];
            dt[k][u] = -dux[k][ii] + db[k][u] - t[k][u];
            dlam[k][l] -= lamt[k][l] * dt[k][l] + lam[k][l];
            dlam[k][u] -= lamt[k][u] * dt[k][u] + lam[k][u];
            alpha_upd_pair(&alpha, lam[k], dlam[k], t[k], dt[k], l, c.pnb);
        }
        if (c.ng > 0) {
            double *tt = t[k] + 2 * c.pnb, *dd = dt[k] + 2 * c.pnb, *ll = lam[k] + 2 * c.pnb,
                   *dl = dlam[k] + 2 * c.pnb, *lt = lamt[k] + 2 * c.pnb, *bb = db[k] + 2 * c.pnb;
            dct_t(k, nu, nx, ng, pDCt, dux[k], dd);
            for (int l = 0; l < c.ng; l++) {
                int u = c.png + l;
                dd[u] = -dd[l];
                dd[l] += -bb[l] - tt[l];
                dd[u] += bb[u] - tt[u];
                dl[l] -= lt[l] * dd[l] + ll[l];
                dl[u] -= lt[u] * dd[u] + ll[u];
                alpha_upd_pair(&alpha, ll, dl, tt, dd, l, c.png);
            }
        }
    }
    *ptr_alpha = alpha;
}

/* d_aux_ip_hard_lib4.c:618-711 */
static void update_var(int N, int *nx, int *nu, int *nb, int *ng, double *ptr_mu, double mu_scal, double alpha,
                       double **ux, double **dux, double **t, double **dt, double **lam, double **dlam, double **pi,
                       double **dpi) {
    double mu = 0.0;
    for (int k = 0; k <= N; k++) {
        cdim_t c = cdim(nb, ng, k);
        int nx1 = k < N ? nx[k + 1] : 0;
        for (int l = 0; l < nu[k] + nx[k]; l++) ux[k][l] += alpha * (dux[k][l] - ux[k][l]);
        for (int l = 0; l < nx1; l++) pi[k][l] += alpha * (dpi[k][l] - pi[k][l]);
        for (int l = 0; l < c.nb; l++) {
            int u = c.pnb + l;
            lam[k][l] += alpha * dlam[k][l];
            lam[k][u] += alpha * dlam[k][u];
            t[k][l] += alpha * dt[k][l];
            t[k][u] += alpha * dt[k][u];
            mu += lam[k][l] * t[k][l] + lam[k][u] * t[k][u];
        }
        for (int l = 0; l < c.ng; l++) {
            int a = 2 * c.pnb + l, u = 2 * c.pnb + c.png + l;
            lam[k][a] += alpha * dlam[k][a];
            lam[k][u] += alpha * dlam[k][u];
            t[k][a] += alpha * dt[k][a];
            t[k][u] += alpha * dt[k][u];
            mu += lam[k][a] * t[k][a] + lam[k][u] * t[k][u];
        }
    }
    *ptr_mu = mu * mu_scal;
}

/* d_aux_ip_hard_lib4.c:715-770 and :1453-1508 (identical arithmetic) */
static void compute_mu(int N, int *nb, int *ng, double *ptr_mu, double mu_scal, double alpha, double **lam,
                       double **dlam, double **t, double **dt) {
    double mu = 0.0;
    for (int k = 0; k <= N; k++) {
        cdim_t c = cdim(nb, ng, k);
        for (int l = 0; l < c.nb; l++) {
            int u = c.pnb + l;
            mu += (lam[k][l] + alpha * dlam[k][l]) * (t[k][l] + alpha * dt[k][l]) +
                  (lam[k][u] + alpha * dlam[k][u]) * (t[k][u] + alpha * dt[k][u]);
        }
        for (int l = 0; l < c.ng; l++) {
            int a = 2 * c.pnb + l, u = 2 * c.pnb + c.png + l;
            mu += (lam[k][a] + alpha * dlam[k][a]) * (t[k][a] + alpha * dt[k][a]) +
                  (lam[k][u] + alpha * dlam[k][u]) * (t[k][u] + alpha * dt[k][u]);
        }
    }
    *ptr_mu = mu * mu_scal;
}

/* d_aux_ip_hard_lib4.c:954-1078 */
static void update_hessian_gradient_res(int N, int *nb, int *ng, double **res_d, double **res_m, double **t,
                                        double **lam, double **t_inv, double **Qx, double **qx) {
    for (int k = 0; k <= N; k++) {
        cdim_t c = cdim(nb, ng, k);
        int segs[2][3] = {{c.nb, c.pnb, 0}, {c.ng, c.png, 2 * c.pnb}};
        int qoff[2] = {0, c.pnb};
        for (int s = 0; s < 2; s++) {
            int n = segs[s][0], p = segs[s][1], o = segs[s][2];
            for (int i = 0; i < n; i++) {
                int a = o + i, u = o + p + i;
                t_inv[k][a] = 1.0 / t[k][a];
                t_inv[k][u] = 1.0 / t[k][u];
                Qx[k][qoff[s] + i] = t_inv[k][a] * lam[k][a] + t_inv[k][u] * lam[k][u];
                qx[k][qoff[s] + i] = t_inv[k][a] * (res_m[k][a] - lam[k][a] * res_d[k][a]) -
                                     t_inv[k][u] * (res_m[k][u] + lam[k][u] * res_d[k][u]);
            }
        }
    }
}

/* d_aux_ip_hard_lib4.c:1550-1639 */
static void update_gradient_res(int N, int *nb, int *ng, double **res_d, double **res_m, double **lam,
                                double **t_inv, double **qx) {
    for (int k = 0; k <= N; k++) {
        cdim_t c = cdim(nb, ng, k);
        int segs[2][3] = {{c.nb, c.pnb, 0}, {c.ng, c.png, 2 * c.pnb}};
        int qoff[2] = {0, c.pnb};
        for (int s = 0; s < 2; s++) {
            int n = segs[s][0], p = segs[s][1], o = segs[s][2];
            for (int i = 0; i < n; i++) {
                int a = o + i, u = o + p + i;
                qx[k][qoff[s] + i] = t_inv[k][a] * (res_m[k][a] - lam[k][a] * res_d[k][a]) -
                                     t_inv[k][u] * (res_m[k][u] + lam[k][u] * res_d[k][u]);
            }
        }
    }
}

/* d_aux_ip_hard_lib4.c:1082-1176 (with_alpha=0) and :1180-1313 (with_alpha=1) */
static void dt_dlam_res(int with_alpha, int N, int *nx, int *nu, int *nb, int **idxb, int *ng, double **dux,
                        double **t, double **t_inv, double **lam, double **pDCt, double **res_d, double **res_m,
                        double **dt, double **dlam, double *ptr_alpha) {
    double alpha = with_alpha ? *ptr_alpha : 1.0;
    for (int k = 0; k <= N; k++) {
        cdim_t c = cdim(nb, ng, k);
        for (int l = 0; l < c.nb; l++) {
            int ii = idxb[k][l], u = c.pnb + l;
            dt[k][l] = dux[k][ii] - res_d[k][l];
            dt[k][u] = -dux[k][ii] + res_d[k][u];
            dlam[k][l] = -t_inv[k][l] * (lam[k][l] * dt[k][l] + res_m[k][l]);
            dlam[k][u] = -t_inv[k][u] * (lam[k][u] * dt[k][u] + res_m[k][u]);
            if (with_alpha) alpha_upd_pair(&alpha, lam[k], dlam[k], t[k], dt[k], l, c.pnb);
        }
        if (c.ng > 0) {
            const int o = 2 * c.pnb;
            double *dd = dt[k] + o;
            dct_t(k, nu, nx, ng, pDCt, dux[k], dd);
            for (int l = 0; l < c.ng; l++) {
                int a = o + l, u = o + c.png + l;
                dt[k][u] = -dt[k][a];
                dt[k][a] -= res_d[k][a];
                dt[k][u] += res_d[k][u];
                dlam[k][a] = -t_inv[k][a] * (lam[k][a] * dt[k][a] + res_m[k][a]);
                dlam[k][u] = -t_inv[k][u] * (lam[k][u] * dt[k][u] + res_m[k][u]);
                if (with_alpha) alpha_upd_pair(&alpha, lam[k] + o, dlam[k] + o, t[k] + o, dt[k] + o, l, c.png);
            }
        }
    }
    if (with_alpha) *ptr_alpha = alpha;
}

/* d_aux_ip_hard_lib4.c:1512-1546 */
static void centering_correction(int N, int *nb, int *ng, double sigma_mu, double **dt, double **dlam,
                                 double **res_m) {
    for (int k = 0; k <= N; k++) {
        cdim_t c = cdim(nb, ng, k);
        for (int l = 0; l < c.nb; l++) {
            res_m[k][l] += dt[k][l] * dlam[k][l] - sigma_mu;
            res_m[k][c.pnb + l] += dt[k][c.pnb + l] * dlam[k][c.pnb + l] - sigma_mu;
        }
        for (int l = 0; l < c.ng; l++) {
            int a = 2 * c.pnb + l, u = 2 * c.pnb + c.png + l;
            res_m[k][a] += dt[k][a] * dlam[k][a] - sigma_mu;
            res_m[k][u] += dt[k][u] * dlam[k][u] - sigma_mu;
        }
    }
}

/* y += alpha x, optional backup z = y first  (daxpy_lib :5321 / daxpy_bkp_lib :5389) */
static void axpy_bkp(int n, double alpha, const double *x, double *y, double *z) {
    for (int i = 0; i < n; i++) {
        if (z) z[i] = y[i];
        y[i] += alpha * x[i];
    }
}

/* d_aux_ip_hard_lib4.c:1317-1378 (bkp == NULL) and :1382-1449 */
static void update_var_res(int N, int *nx, int *nu, int *nb, int *ng, double alpha, double **ux_bkp, double **ux,
                           double **dux, double **pi_bkp, double **pi, double **dpi, double **t_bkp, double **t,
                           double **dt, double **lam_bkp, double **lam, double **dlam) {
    for (int k = 0; k <= N; k++) {
        cdim_t c = cdim(nb, ng, k);
        int nx1 = k < N ? nx[k + 1] : 0;
        axpy_bkp(nu[k] + nx[k], alpha, dux[k], ux[k], ux_bkp ? ux_bkp[k] : NULL);
        if (k < N) /* pi, dpi, pi_bkp hold N stage pointers: there is no pi[N] to touch */
            axpy_bkp(nx1, alpha, dpi[k], pi[k], pi_bkp ? pi_bkp[k] : NULL);
        int offs[4] = {0, c.pnb, 2 * c.pnb, 2 * c.pnb + c.png};
        int lens[4] = {c.nb, c.nb, c.ng, c.ng};
        for (int s = 0; s < 4; s++) {
            axpy_bkp(lens[s], alpha, dlam[k] + offs[s], lam[k] + offs[s], lam_bkp ? lam_bkp[k] + offs[s] : NULL);
            axpy_bkp(lens[s], alpha, dt[k] + offs[s], t[k] + offs[s], t_bkp ? t_bkp[k] + offs[s] : NULL);
        }
    }
}

/* ================================================================================================
 * IPM workspace (oracle-private carve).  Persistent between orc_d_ip2_res_mpc_hard_tv and
 * orc_d_kkt_solve_new_rhs_res_mpc_hard_tv: factor, t_inv and the *_bkp iterate (d_ip2_res_hard.c:1922+).
 * ============================================================================================== */
typedef struct {
    double *work, *memory;
    double **b, **q, **dux, **dpi, **Pb, **bd, **dlam, **dt, **t_inv, **lamt, **Qx, **qx, *res_work, **res_q,
        **res_b, **res_d, **res_m, **ux_bkp, **pi_bkp, **t_bkp, **lam_bkp;
} ipws_t;

static long ipws_carve(int N, int *nx, int *nu, int *nb, int *ng, double *base, ipws_t *w, double **ptrs) {
    /* ptrs: storage for the per-stage pointer tables, 19*(N+1) entries */
    long off = 0;
    int nuN[N + 1];
    for (int k = 0; k <= N; k++) nuN[k] = k < N ? nu[k] : 0;
    int pngM = 0;
    for (int k = 0; k <= N; k++)
        if (rup(ng[k], BS) > pngM) pngM = rup(ng[k], BS);
    if (w) w->work = base + off;
    off += orc_d_back_ric_rec_sv_tv_work_space_size_bytes(N, nx, nuN, nb, ng) / 8;
    if (w) w->memory = base + off;
    off += orc_d_back_ric_rec_sv_tv_memory_space_size_bytes(N, nx, nuN, nb, ng) / 8;
    double ***tabs[18];
    if (w) {
        double ***t[18] = {&w->b,     &w->q,     &w->dux,   &w->dpi,    &w->Pb,     &w->bd,
                           &w->dlam,  &w->dt,    &w->t_inv, &w->lamt,   &w->Qx,     &w->res_q,
                           &w->res_b, &w->res_d, &w->res_m, &w->ux_bkp, &w->pi_bkp, &w->t_bkp};
        memcpy(tabs, t, sizeof(t));
        for (int i = 0; i < 18; i++) *tabs[i] = ptrs + i * (N + 1);
        w->lam_bkp = ptrs + 18 * (N + 1);
        w->qx = ptrs + 19 * (N + 1);
    }
    for (int k = 0; k <= N; k++) {
        int nux = nuN[k] + nx[k], pnz = rup(nux + 1, BS), pnx1 = k < N ? rup(nx[k + 1], BS) : 0;
        int pnb = rup(nb[k], BS), png = rup(ng[k], BS), nc = 2 * pnb + 2 * png;
#define TAKE(field, n)                  \
    do {                                \
        if (w) w->field[k] = base + off; \
        off += (n);                      \
    } while (0)
        TAKE(b, pnx1);
        TAKE(q, pnz);
        TAKE(dux, pnz);
        TAKE(dpi, pnx1);
        TAKE(Pb, pnx1);
        TAKE(bd, pnb);
        TAKE(dlam, nc);
        TAKE(dt, nc);
        TAKE(t_inv, nc);
        TAKE(lamt, nc);
        TAKE(Qx, pnb + png);
        TAKE(qx, pnb + png);
        TAKE(res_q, pnz);
        TAKE(res_b, pnx1);
        TAKE(res_d, nc);
        TAKE(res_m, nc);
        TAKE(ux_bkp, pnz);
        TAKE(pi_bkp, pnx1);
        TAKE(t_bkp, nc);
        TAKE(lam_bkp, nc);
#undef TAKE
    }
    if (w) w->res_work = base + off;
    off += 2 * pngM + 4;
    return off;
}

int orc_d_ip2_res_mpc_hard_tv_work_space_size_bytes(int N, int *nx, int *nu, int *nb, int *ng) {
    long n = ipws_carve(N, nx, nu, nb, ng, NULL, NULL, NULL);
    return (int)((n * 8 + 63) / 64 * 64);
}

/* restore hpRSQrq diag / aug row and (optionally) hpBAbt aug row from the backups (:721-732, :1231-1245) */
static void restore_data(int N, int *nx, int *nu, int *nb, int **idxb, double **pBAbt, double **pQ, ipws_t *w,
                         int restore_b) {
    for (int k = 0; k <= N; k++) {
        int nux = nu[k] + nx[k], cnux = rup(nux, NCL);
        for (int l = 0; l < nb[k]; l++) {
            int ii = idxb[k][l];
            *P4(pQ[k], cnux, ii, ii) = w->bd[k][l];
        }
        for (int l = 0; l < nux; l++) *P4(pQ[k], cnux, nux, l) = w->q[k][l];
    }
    if (restore_b)
        for (int k = 0; k < N; k++) {
            int nux = nu[k] + nx[k], cnx1 = rup(nx[k + 1], NCL);
            for (int j = 0; j < nx[k + 1]; j++) *P4(pBAbt[k], cnx1, nux, j) = w->b[k][j];
        }
}

static void ip_setup(int N, int *nx, int *nu, int *nb, int **idxb, int *ng, double **pBAbt, double **pQ,
                     ipws_t *w) {
    for (int k = 0; k < N; k++) {
        int nux = nu[k] + nx[k], cnx1 = rup(nx[k + 1], NCL);
        for (int j = 0; j < nx[k + 1]; j++) w->b[k][j] = *P4(pBAbt[k], cnx1, nux, j);
    }
    for (int k = 0; k <= N; k++) {
        int nux = nu[k] + nx[k], cnux = rup(nux, NCL);
        for (int l = 0; l < nux; l++) w->q[k][l] = *P4(pQ[k], cnux, nux, l);
        for (int l = 0; l < nb[k]; l++) {
            int ii = idxb[k][l];
            w->bd[k][l] = *P4(pQ[k], cnux, ii, ii);
        }
    }
}

static void backup_iterate(int N, int *nx, int *nu, int *nb, int *ng, double **ux, double **pi, double **lam,
                           double **t, ipws_t *w) {
    for (int k = 0; k <= N; k++) {
        for (int j = 0; j < nu[k] + nx[k]; j++) w->ux_bkp[k][j] = ux[k][j];
        if (k < N)
            for (int j = 0; j < nx[k + 1]; j++) w->pi_bkp[k][j] = pi[k][j];
        cdim_t c = cdim(nb, ng, k);
        int offs[4] = {0, c.pnb, 2 * c.pnb, 2 * c.pnb + c.png}, lens[4] = {c.nb, c.nb, c.ng, c.ng};
        for (int s = 0; s < 4; s++)
            for (int j = 0; j < lens[s]; j++) {
                w->lam_bkp[k][offs[s] + j] = lam[k][offs[s] + j];
                w->t_bkp[k][offs[s] + j] = t[k][offs[s] + j];
            }
    }
}

#define IPWS_DECL(N)                 \
    double *ptrs_[20 * ((N) + 1)];   \
    ipws_t w_;                       \
    int nu_[(N) + 1];

static int ipm_core(int single_newton, int phase1_only, int *kk, int k_max, double mu0, double mu_tol, double alpha_min,
                    int warm_start, double *stat, int N, int *nx, int *nu_N, int *nb, int **idxb, int *ng,
                    double **pBAbt, double **pQ, double **pDCt, double **d, double **ux, int compute_mult,
                    double **pi, double **lam, double **t, double *double_work_memory, double **ux0, double **pi0,
                    double **lam0, double **t0) {
    IPWS_DECL(N);
    int *nu = nu_;
    for (int k = 0; k < N; k++) nu[k] = nu_N[k];
    nu[N] = 0;
    ipws_t *w = &w_;
    ipws_carve(N, nx, nu, nb, ng, double_work_memory, w, ptrs_);
    ip_setup(N, nx, nu, nb, idxb, ng, pBAbt, pQ, w);

    double mu_scal = 0.0;
    for (int k = 0; k <= N; k++) mu_scal += 2 * nb[k] + 2 * ng[k];
    if (mu_scal == 0.0 && phase1_only) {
        /* d_ip2_hard.c:282-291: the sv solves into the workspace (dux, dpi); ux/pi/lam/t are untouched */
        orc_d_back_ric_rec_sv_tv_res(N, nx, nu, nb, idxb, ng, 0, pBAbt, w->b, 0, pQ, w->q, NULL, NULL, NULL, NULL,
                                     w->dux, compute_mult, w->dpi, 1, w->Pb, w->memory, w->work);
        *kk = 0;
        return 0;
    }
    if (mu_scal == 0.0) {
        /* unconstrained: one sv and return (:428-450) */
        orc_d_back_ric_rec_sv_tv_res(N, nx, nu, nb, idxb, ng, 0, pBAbt, w->b, 0, pQ, w->q, NULL, NULL, NULL, NULL,
                                     ux, compute_mult, pi, 1, w->Pb, w->memory, w->work);
        for (int k = 0; k <= N; k++)
            for (int j = 0; j < nu[k] + nx[k]; j++) w->ux_bkp[k][j] = ux[k][j];
        for (int k = 0; k < N; k++)
            for (int j = 0; j < nx[k + 1]; j++) w->pi_bkp[k][j] = pi[k][j];
        *kk = 0;
        return 0;
    }
    mu_scal = 1.0 / mu_scal;
    double sigma = 0.0, alpha = 1.0, mu = mu0, mu_aff = 0.0;
    *kk = 0;

    if (!single_newton) {
        init_var(N, nx, nu, nb, idxb, ng, ux, pi, pDCt, d, t, lam, mu0, warm_start);
        /* phase 1: no residuals (:498-718).  d_ip2_mpc_hard_tv (d_ip2_hard.c:329-520) is this loop alone, run
         * to mu_tol itself */
        const double mu_tol_low = phase1_only ? mu_tol : (mu_tol < 1e-5 ? 1e-5 : mu_tol);
        while (*kk < k_max && mu > mu_tol_low && alpha >= alpha_min) {
            update_hessian(N, nb, ng, d, 0.0, t, w->t_inv, lam, w->lamt, w->dlam, w->Qx, w->qx);
            orc_d_back_ric_rec_sv_tv_res(N, nx, nu, nb, idxb, ng, 0, pBAbt, w->b, 1, pQ, w->q, w->bd, pDCt, w->Qx,
                                         w->qx, w->dux, compute_mult, w->dpi, 1, w->Pb, w->memory, w->work);
            alpha = 1.0;
            compute_alpha(N, nx, nu, nb, idxb, ng, &alpha, t, w->dt, lam, w->dlam, w->lamt, w->dux, pDCt, d);
            stat[5 * *kk] = sigma;
            stat[5 * *kk + 1] = alpha;
            alpha *= 0.995;
            compute_mu(N, nb, ng, &mu_aff, mu_scal, alpha, lam, w->dlam, t, w->dt);
            stat[5 * *kk + 2] = mu_aff;
            sigma = mu_aff / mu;
            sigma = sigma * sigma * sigma;
            update_gradient(N, nb, ng, sigma * mu, w->dt, w->dlam, w->t_inv, w->qx);
            orc_d_back_ric_rec_trs_tv_res(N, nx, nu, nb, idxb, ng, pBAbt, w->b, w->q, pDCt, w->qx, w->dux,
                                          compute_mult, w->dpi, 0, w->Pb, w->memory, w->work);
            alpha = 1.0;
            compute_alpha(N, nx, nu, nb, idxb, ng, &alpha, t, w->dt, lam, w->dlam, w->lamt, w->dux, pDCt, d);
            stat[5 * *kk] = sigma;
            stat[5 * *kk + 3] = alpha;
            alpha *= 0.995;
            backup_iterate(N, nx, nu, nb, ng, ux, pi, lam, t, w);
            update_var(N, nx, nu, nb, ng, &mu, mu_scal, alpha, ux, w->dux, t, w->dt, lam, w->dlam, pi, w->dpi);
            stat[5 * *kk + 4] = mu;
            (*kk)++;
        }
        restore_data(N, nx, nu, nb, idxb, pBAbt, pQ, w, 0);
        if (phase1_only) { /* d_ip2_hard.c:604-612 */
            if (mu <= mu_tol) return 0;
            if (*kk >= k_max) return 1;
            if (alpha < alpha_min) return 2;
            return -1;
        }
    } else {
        /* d_init_var_mpc_hard_tv_single_newton (d_aux_ip_hard_lib4.c:153-213) */
        for (int k = 0; k <= N; k++) {
            for (int l = 0; l < nu[k] + nx[k]; l++) ux[k][l] = ux0[k][l];
            int pnb = rup(nb[k], BS);
            for (int l = 0; l < nb[k]; l++) {
                lam[k][l] = lam0[k][l];
                lam[k][pnb + l] = lam0[k][nb[k] + l];
                t[k][l] = t0[k][l];
                t[k][pnb + l] = t0[k][nb[k] + l];
            }
            if (ng[k] > 0) {
                fprintf(stderr, "General constraints not supported yet!!\n");
                exit(1);
            }
        }
        for (int k = 0; k < N; k++)
            for (int l = 0; l < nx[k + 1]; l++) pi[k][l] = pi0[k][l];
        mu = mu0;
        restore_data(N, nx, nu, nb, idxb, pBAbt, pQ, w, 0);
    }

    orc_d_res_res_mpc_hard_tv(N, nx, nu, nb, idxb, ng, pBAbt, w->b, pQ, w->q, ux, pDCt, d, pi, lam, t, w->res_work,
                              w->res_q, w->res_b, w->res_d, w->res_m, &mu);

    /* phase 2: residual-based Mehrotra (:783-1273); single Newton: :1640-1905 */
    while (*kk < k_max && (single_newton || (mu > mu_tol && alpha >= alpha_min))) {
        update_hessian_gradient_res(N, nb, ng, w->res_d, w->res_m, t, lam, w->t_inv, w->Qx, w->qx);
        if (!single_newton)
            orc_d_back_ric_rec_sv_tv_res(N, nx, nu, nb, idxb, ng, 1, pBAbt, w->res_b, 1, pQ, w->res_q, w->bd, pDCt,
                                         w->Qx, w->qx, w->dux, compute_mult, w->dpi, 1, w->Pb, w->memory, w->work);
        else /* the reference's single-Newton step factorises with update_b=0,b / update_q=1,q */
            orc_d_back_ric_rec_sv_tv_res(N, nx, nu, nb, idxb, ng, 0, pBAbt, w->b, 1, pQ, w->q, w->bd, pDCt, w->Qx,
                                         w->qx, w->dux, compute_mult, w->dpi, 1, w->Pb, w->memory, w->work);
        alpha = 1.0;
        dt_dlam_res(1, N, nx, nu, nb, idxb, ng, w->dux, t, w->t_inv, lam, pDCt, w->res_d, w->res_m, w->dt, w->dlam,
                    &alpha);
        stat[5 * *kk] = sigma;
        stat[5 * *kk + 1] = alpha;
        alpha *= 0.995;
        compute_mu(N, nb, ng, &mu_aff, mu_scal, alpha, lam, w->dlam, t, w->dt);
        stat[5 * *kk + 2] = mu_aff;
        if (!single_newton) {
            sigma = mu_aff / mu;
            sigma = sigma * sigma * sigma;
            centering_correction(N, nb, ng, sigma * mu, w->dt, w->dlam, w->res_m);
        } else {
            centering_correction(N, nb, ng, mu0, w->dt, w->dlam, w->res_m);
        }
        update_gradient_res(N, nb, ng, w->res_d, w->res_m, lam, w->t_inv, w->qx);
        orc_d_back_ric_rec_trs_tv_res(N, nx, nu, nb, idxb, ng, pBAbt, w->res_b, w->res_q, pDCt, w->qx, w->dux,
                                      compute_mult, w->dpi, 0, w->Pb, w->memory, w->work);
        alpha = 1.0;
        dt_dlam_res(1, N, nx, nu, nb, idxb, ng, w->dux, t, w->t_inv, lam, pDCt, w->res_d, w->res_m, w->dt, w->dlam,
                    &alpha);
        stat[5 * *kk] = sigma;
        stat[5 * *kk + 3] = alpha;
        alpha *= 0.995;
        update_var_res(N, nx, nu, nb, ng, alpha, w->ux_bkp, ux, w->dux, w->pi_bkp, pi, w->dpi, w->t_bkp, t, w->dt,
                       w->lam_bkp, lam, w->dlam);
        restore_data(N, nx, nu, nb, idxb, pBAbt, pQ, w, 1);
        orc_d_res_res_mpc_hard_tv(N, nx, nu, nb, idxb, ng, pBAbt, w->b, pQ, w->q, ux, pDCt, d, pi, lam, t,
                                  w->res_work, w->res_q, w->res_b, w->res_d, w->res_m, &mu);
        stat[5 * *kk + 4] = mu;
        (*kk)++;
    }
    if (!single_newton && mu <= mu_tol) return 0;
    if (*kk >= k_max) return 1;
    if (alpha < alpha_min) return 2;
    return -1;
}

int orc_d_ip2_res_mpc_hard_tv(int *kk, int k_max, double mu0, double mu_tol, double alpha_min, int warm_start,
                              double *stat, int N, int *nx, int *nu_N, int *nb, int **idxb, int *ng, double **pBAbt,
                              double **pQ, double **pDCt, double **d, double **ux, int compute_mult, double **pi,
                              double **lam, double **t, double *double_work_memory) {
    return ipm_core(0, 0, kk, k_max, mu0, mu_tol, alpha_min, warm_start, stat, N, nx, nu_N, nb, idxb, ng, pBAbt, pQ,
                    pDCt, d, ux, compute_mult, pi, lam, t, double_work_memory, NULL, NULL, NULL, NULL);
}

int orc_d_ip2_res_mpc_hard_tv_single_newton_step(int *kk, int k_max, double mu0, double mu_tol, double alpha_min,
                                                 int warm_start, double *stat, int N, int *nx, int *nu_N, int *nb,
                                                 int **idxb, int *ng, double **pBAbt, double **pQ, double **pDCt,
                                                 double **d, double **ux, int compute_mult, double **pi,
                                                 double **lam, double **t, double *double_work_memory, double **ux0,
                                                 double **pi0, double **lam0, double **t0) {
    return ipm_core(1, 0, kk, k_max, mu0, mu_tol, alpha_min, warm_start, stat, N, nx, nu_N, nb, idxb, ng, pBAbt, pQ,
                    pDCt, d, ux, compute_mult, pi, lam, t, double_work_memory, ux0, pi0, lam0, t0);
}

void orc_d_kkt_solve_new_rhs_res_mpc_hard_tv(int N, int *nx, int *nu_N, int *nb, int **idxb, int *ng,
                                             double **pBAbt, double **b, double **pQ, double **q, double **pDCt,
                                             double **d, double **ux, int compute_mult, double **pi, double **lam,
                                             double **t, double *double_work_memory) {
    IPWS_DECL(N);
    int *nu = nu_;
    for (int k = 0; k < N; k++) nu[k] = nu_N[k];
    nu[N] = 0;
    ipws_t *w = &w_;
    ipws_carve(N, nx, nu, nb, ng, double_work_memory, w, ptrs_);
    double mu = 0.0;
    /* restore the last iterate from the backup (:2139-2172) */
    for (int k = 0; k <= N; k++) {
        for (int j = 0; j < nu[k] + nx[k]; j++) ux[k][j] = w->ux_bkp[k][j];
        if (k < N)
            for (int j = 0; j < nx[k + 1]; j++) pi[k][j] = w->pi_bkp[k][j];
        cdim_t c = cdim(nb, ng, k);
        int offs[4] = {0, c.pnb, 2 * c.pnb, 2 * c.pnb + c.png}, lens[4] = {c.nb, c.nb, c.ng, c.ng};
        for (int s = 0; s < 4; s++)
            for (int j = 0; j < lens[s]; j++) {
                t[k][offs[s] + j] = w->t_bkp[k][offs[s] + j];
                lam[k][offs[s] + j] = w->lam_bkp[k][offs[s] + j];
            }
    }
    orc_d_res_res_mpc_hard_tv(N, nx, nu, nb, idxb, ng, pBAbt, b, pQ, q, ux, pDCt, d, pi, lam, t, w->res_work,
                              w->res_q, w->res_b, w->res_d, w->res_m, &mu);
    update_gradient_res(N, nb, ng, w->res_d, w->res_m, lam, w->t_inv, w->qx);
    orc_d_back_ric_rec_trs_tv_res(N, nx, nu, nb, idxb, ng, pBAbt, w->res_b, w->res_q, pDCt, w->qx, w->dux,
                                  compute_mult, w->dpi, 1, w->Pb, w->memory, w->work);
    dt_dlam_res(0, N, nx, nu, nb, idxb, ng, w->dux, t, w->t_inv, lam, pDCt, w->res_d, w->res_m, w->dt, w->dlam,
                NULL);
    update_var_res(N, nx, nu, nb, ng, 1.0, NULL, ux, w->dux, NULL, pi, w->dpi, NULL, t, w->dt, NULL, lam, w->dlam);
}

/* ================================================================================================
 * Alternate IPM (mpc_solvers/d_ip2_hard.c): the phase-1 Mehrotra loop alone, its KKT re-solve and
 * the plain residuals of mpc_solvers/d_res_ip_hard.c.
 * ============================================================================================== */
int orc_d_ip2_mpc_hard_tv_work_space_size_bytes(int N, int *nx, int *nu, int *nb, int *ng) {
    /* the oracle shares one private workspace carve between both IPMs (d_ip2_hard.c:31-87 sizes its own) */
    return orc_d_ip2_res_mpc_hard_tv_work_space_size_bytes(N, nx, nu, nb, ng);
}

/* d_ip2_hard.c:88-614 */
int orc_d_ip2_mpc_hard_tv(int *kk, int k_max, double mu0, double mu_tol, double alpha_min, int warm_start,
                          double *stat, int N, int *nx, int *nu_N, int *nb, int **idxb, int *ng, double **pBAbt,
                          double **pQ, double **pDCt, double **d, double **ux, int compute_mult, double **pi,
                          double **lam, double **t, double *double_work_memory) {
    return ipm_core(0, 1, kk, k_max, mu0, mu_tol, alpha_min, warm_start, stat, N, nx, nu_N, nb, idxb, ng, pBAbt, pQ,
                    pDCt, d, ux, compute_mult, pi, lam, t, double_work_memory, NULL, NULL, NULL, NULL);
}

/* d_ip2_hard.c:626-825 as built for the reference's default target X64_AVX (Makefile.rule:38), where
 * d_update_gradient_new_rhs_mpc_hard_tv takes (db, t_inv, lamt, qx) (avx/d_aux_ip_hard_lib4.c:1735-1838).
 * lamt / the factor are those of the IPM's last iteration, left in the workspace. */
void orc_d_kkt_solve_new_rhs_mpc_hard_tv(int N, int *nx, int *nu_N, int *nb, int **idxb, int *ng, double **pBAbt,
                                         double **r_A, double **pQ, double **r_H, double **pDCt, double **r_C,
                                         double **ux, int compute_mult, double **pi, double **lam, double **t,
                                         double *double_work_memory) {
    IPWS_DECL(N);
    int *nu = nu_;
    for (int k = 0; k < N; k++) nu[k] = nu_N[k];
    nu[N] = 0;
    ipws_t *w = &w_;
    ipws_carve(N, nx, nu, nb, ng, double_work_memory, w, ptrs_);
    /* d_update_gradient_new_rhs_mpc_hard_tv (avx/d_aux_ip_hard_lib4.c:1735-1838) */
    for (int k = 0; k <= N; k++) {
        cdim_t c = cdim(nb, ng, k);
        for (int i = 0; i < c.nb; i++)
            w->qx[k][i] = -w->lamt[k][c.pnb + i] * r_C[k][c.pnb + i] - w->lamt[k][i] * r_C[k][i];
        const int o = 2 * c.pnb;
        for (int i = 0; i < c.ng; i++)
            w->qx[k][c.pnb + i] = -w->lamt[k][o + c.png + i] * r_C[k][o + c.png + i] - w->lamt[k][o + i] * r_C[k][o + i];
    }
    orc_d_back_ric_rec_trs_tv_res(N, nx, nu, nb, idxb, ng, pBAbt, r_A, r_H, pDCt, w->qx, ux, compute_mult, pi, 1,
                                  w->Pb, w->memory, w->work);
    /* d_compute_t_lam_new_rhs_mpc_hard_tv (c99/d_aux_ip_hard_lib4.c:864-935) */
    for (int k = 0; k <= N; k++) {
        cdim_t c = cdim(nb, ng, k);
        for (int l = 0; l < c.nb; l++) {
            const int ii = idxb[k][l];
            t[k][l] = ux[k][ii] - r_C[k][l];
            t[k][c.pnb + l] = -ux[k][ii] + r_C[k][c.pnb + l];
            lam[k][l] = -w->lamt[k][l] * t[k][l];
            lam[k][c.pnb + l] = -w->lamt[k][c.pnb + l] * t[k][c.pnb + l];
        }
        if (c.ng > 0) {
            const int o = 2 * c.pnb;
            double *tt = t[k] + o, *ll = lam[k] + o, *lt = w->lamt[k] + o, *dd = r_C[k] + o;
            dct_t(k, nu, nx, ng, pDCt, ux[k], tt);
            for (int l = 0; l < c.ng; l++) {
                tt[l + c.png] = -tt[l];
                tt[l] -= dd[l];
                tt[l + c.png] += dd[l + c.png];
                ll[l] = -lt[l] * tt[l];
                ll[l + c.png] = -lt[l + c.png] * tt[l + c.png];
            }
        }
    }
}

/* mpc_solvers/d_res_ip_hard.c:38-330: r_q, r_b, r_d of the KKT system (no r_m), mu = lam't / (2 sum(nb+ng)),
 * 0 without constraints.  Computed with the reference's signs, then negated (:305-326). */
void orc_d_res_mpc_hard_tv(int N, int *nx, int *nu, int *nb, int **idxb, int *ng, double **hpBAbt, double **hb,
                           double **hpQ, double **hq, double **hux, double **hpDCt, double **hd, double **hpi,
                           double **hlam, double **ht, double **hrq, double **hrb, double **hrd, double *mu) {
    int nb_tot = 0;
    mu[0] = 0.0;
    for (int k = 0; k <= N; k++) {
        const int nuk = nu[k], nxk = nx[k], nux = nuk + nxk, cnux = rup(nux, NCL); /* nu[N] == 0 */
        cdim_t c = cdim(nb, ng, k);
        nb_tot += c.nb + c.ng;
        for (int j = 0; j < c.nb; j++) mu[0] += hlam[k][j] * ht[k][j] + hlam[k][c.pnb + j] * ht[k][c.pnb + j];
        for (int j = 0; j < c.ng; j++)
            mu[0] += hlam[k][2 * c.pnb + j] * ht[k][2 * c.pnb + j] +
                     hlam[k][2 * c.pnb + c.png + j] * ht[k][2 * c.pnb + c.png + j];
        for (int j = 0; j < c.nb; j++) {
            const int ii = idxb[k][j];
            hrd[k][j] = hux[k][ii] - hd[k][j] - ht[k][j];
            hrd[k][c.pnb + j] = -hux[k][ii] + hd[k][c.pnb + j] - ht[k][c.pnb + j];
        }
        if (c.ng > 0) {
            double *r = hrd[k] + 2 * c.pnb;
            const double *dd = hd[k] + 2 * c.pnb, *tt = ht[k] + 2 * c.pnb;
            dct_t(k, nu, nx, ng, hpDCt, hux[k], r);
            for (int j = 0; j < c.ng; j++) {
                r[c.png + j] = -r[j];
                r[j] += -dd[j] - tt[j];
                r[c.png + j] += dd[c.png + j] - tt[c.png + j];
            }
        }
        for (int j = 0; j < nuk; j++) hrq[k][j] = -hq[k][j];
        for (int j = 0; j < nxk; j++) hrq[k][nuk + j] = k > 0 ? -hq[k][nuk + j] + hpi[k - 1][j] : -hq[k][nuk + j];
        for (int j = 0; j < c.nb; j++) hrq[k][idxb[k][j]] += hlam[k][j] - hlam[k][c.pnb + j];
        for (int i = 0; i < nux; i++) { /* dsymv_lib, alg -1 */
            double a = 0.0;
            for (int j = 0; j < nux; j++) a += (i >= j ? *P4(hpQ[k], cnux, i, j) : *P4(hpQ[k], cnux, j, i)) * hux[k][j];
            hrq[k][i] -= a;
        }
        if (c.ng > 0) {
            const int cng = rup(c.ng, NCL);
            for (int i = 0; i < nux; i++) {
                double a = 0.0, b = 0.0;
                for (int l = 0; l < c.ng; l++) a += *P4(hpDCt[k], cng, i, l) * hlam[k][2 * c.pnb + l];
                for (int l = 0; l < c.ng; l++) b += *P4(hpDCt[k], cng, i, l) * hlam[k][2 * c.pnb + c.png + l];
                hrq[k][i] += a;
                hrq[k][i] -= b;
            }
        }
        if (k < N) {
            const int nx1 = nx[k + 1], nu1 = nu[k + 1], cnx1 = rup(nx1, NCL);
            for (int j = 0; j < nx1; j++) hrb[k][j] = hux[k + 1][nu1 + j] - hb[k][j];
            for (int i = 0; i < nux; i++) { /* dgemv_nt_lib, alg -1 / -1 */
                double a = 0.0;
                for (int j = 0; j < nx1; j++) a += *P4(hpBAbt[k], cnx1, i, j) * hpi[k][j];
                hrq[k][i] -= a;
            }
            for (int j = 0; j < nx1; j++) {
                double a = 0.0;
                for (int i = 0; i < nux; i++) a += *P4(hpBAbt[k], cnx1, i, j) * hux[k][i];
                hrb[k][j] -= a;
            }
        }
    }
    if (nb_tot != 0) mu[0] /= 2.0 * nb_tot;
    for (int k = 0; k <= N; k++) {
        const int nux = nu[k] + nx[k];
        cdim_t c = cdim(nb, ng, k);
        for (int j = 0; j < nux; j++) hrq[k][j] = -hrq[k][j];
        if (k < N)
            for (int j = 0; j < nx[k + 1]; j++) hrb[k][j] = -hrb[k][j];
        for (int j = 0; j < c.nb; j++) {
            hrd[k][j] = -hrd[k][j];
            hrd[k][c.pnb + j] = -hrd[k][c.pnb + j];
        }
        for (int j = 0; j < c.ng; j++) {
            hrd[k][2 * c.pnb + j] = -hrd[k][2 * c.pnb + j];
            hrd[k][2 * c.pnb + c.png + j] = -hrd[k][2 * c.pnb + c.png + j];
        }
    }
}

/* shared with hpmpc_oracle_cond.c (partial condensing propagates the state cost-to-go with it) */
void orc__chol_aug(int m, int n, double *M, int ldm, double *L, int ldl, double *dL) { chol_aug(m, n, M, ldm, L, ldl, dL); }
