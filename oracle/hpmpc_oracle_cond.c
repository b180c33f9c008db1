/*
 * hpmpc_oracle_cond.c -- TEST INFRASTRUCTURE ONLY (parity checker; see hpmpc_oracle.h).
 *
 * Clean-room restatement of HPMPC's partial condensing (lqcp_solvers/d_part_cond.c, non-BLASFEO
 * branches): a horizon-N OCP QP is condensed into N2 blocks; block i eliminates the states inside
 * its T stages, keeping [u_{T-1}; ...; u_0; x_0] (inputs in reverse stage order, then the block's
 * first state) as the condensed stage variable.  Matrices are unpacked from / packed to lib4; all
 * arithmetic runs on dense column-major temporaries in the mathematical summation order.
 *
 *   problem size         d_part_cond.c:694-738
 *   work / memory sizes  :743-924 (memory carve and sizes reproduced: callers read the condensed
 *                        data through the pointer arrays d_part_cond fills, :1013-1041)
 *   condensing           :926-1062 -> d_cond_BAbt :214-308, d_cond_RSQrq :312-574, d_cond_DCtd :579-689
 *                        (each also exported alone, orc_d_cond_*, with the reference prototypes)
 *   expansion            :1103-1308
 */
#include <math.h>
#include <stdlib.h>
#include <string.h>

#include "hpmpc_oracle.h"

#define BS 4
#define NCL 2

static inline int rup(int n, int m) { return (n + m - 1) / m * m; }
static inline double *P4(double *pA, int sd, int i, int j) { return pA + (i / BS) * BS * sd + i % BS + BS * j; }

/* the augmented Cholesky of hpmpc_oracle.c (pivot > 1e-15 else the column is zeroed) */
void orc__chol_aug(int m, int n, double *M, int ldm, double *L, int ldl, double *dL);

/* block partition (d_part_cond.c:699-701): the first R1 blocks have M1 = N1+1 stages */
static int block_len(int N, int N2, int ii) {
    int N1 = N / N2, R1 = N - N2 * N1, M1 = R1 > 0 ? N1 + 1 : N1;
    return ii < R1 ? M1 : N1;
}

/* d_part_cond.c:694-738 */
void orc_d_part_cond_compute_problem_size(int N, int *nx, int *nu, int *nb, int **hidxb, int *ng, int N2, int *nx2,
                                          int *nu2, int *nb2, int *ng2) {
    int N_tmp = 0;
    for (int ii = 0; ii < N2; ii++) {
        int T1 = block_len(N, N2, ii);
        nx2[ii] = nx[N_tmp];
        nu2[ii] = nu[N_tmp];
        nb2[ii] = nb[N_tmp];
        ng2[ii] = ng[N_tmp];
        for (int jj = 1; jj < T1; jj++) {
            int nbb = 0, nbg = 0, s = N_tmp + jj;
            for (int kk = 0; kk < nb[s]; kk++) {
                if (hidxb[s][kk] < nu[s])
                    nbb++;
                else
                    nbg++;
            }
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

/* oracle-private: the lib4 and dense Gamma matrices of the largest block plus the stage temporaries */
int orc_d_part_cond_work_space_size_bytes(int N, int *nx, int *nu, int *nb, int **hidxb, int *ng, int N2, int *nx2,
                                          int *nu2, int *nb2, int *ng2) {
    long best = 0;
    int N_tmp = 0;
    for (int ii = 0; ii < N2; ii++) {
        int T1 = block_len(N, N2, ii);
        long s = 0, nut = 0, nzM = 0;
        for (int jj = 0; jj < T1; jj++) {
            int st = N_tmp + jj;
            nut += nu[st];
            s += (nut + nx[N_tmp] + 1) * (long)nx[st + 1] +
                 (long)rup(nut + nx[N_tmp] + 1, BS) * rup(nx[st + 1], NCL);
            if (nu[st] + nx[st] + 1 > nzM) nzM = nu[st] + nx[st] + 1;
        }
        s += 4 * nzM * nzM + 4 * (nut + nx[N_tmp] + 1) * (nut + nx[N_tmp] + 1);
        if (s > best) best = s;
        N_tmp += T1;
    }
    return (int)((best * 8 + 8 * 64 + 63) / 64 * 64);
}

/* d_part_cond.c:868-924 (the reference's memory carve; reproduced so callers see the same layout) */
int orc_d_part_cond_memory_space_size_bytes(int N, int *nx, int *nu, int *nb, int **hidxb, int *ng, int N2,
                                            int *nx2, int *nu2, int *nb2, int *ng2) {
    if (N2 == N) return 0;
    long d_size = 0, i_size = 0;
    for (int ii = 0; ii < N2; ii++) {
        int pnz2 = rup(nu2[ii] + nx2[ii] + 1, BS), pnux2 = rup(nu2[ii] + nx2[ii], BS);
        d_size += (long)pnz2 * rup(nx2[ii + 1], NCL) + (long)pnz2 * rup(nu2[ii] + nx2[ii], NCL) +
                  (long)pnux2 * rup(ng2[ii], NCL) + 2 * rup(nb2[ii], BS) + 2 * rup(ng2[ii], BS);
        i_size += nb2[ii];
    }
    return (int)((d_size * 8 + i_size * 4 + 63) / 64 * 64);
}

static void unpack(double *pA, int sd, int m, int n, double *A, int lda) {
    for (int j = 0; j < n; j++)
        for (int i = 0; i < m; i++) A[i + j * lda] = *P4(pA, sd, i, j);
}

static void pack(const double *A, int lda, int m, int n, double *pA, int sd) {
    for (int j = 0; j < n; j++)
        for (int i = 0; i < m; i++) *P4(pA, sd, i, j) = A[i + j * lda];
}

/* rows of Gamma_j: [u_j .. u_0, x_0, 1] -> r_j = sum_{i<=j} nu_i + nx_0 + 1 */
static int gamma_rows(int j, int *nx, int *nu) {
    int r = nx[0] + 1;
    for (int i = 0; i <= j; i++) r += nu[i];
    return r;
}

/* the dense copies of hpGamma[0..n) laid end to end in work; returns the first double past them */
static double *gamma_dense(int n, int *nx, int *nu, double **hpGamma, double *work, double **G) {
    double *p = work;
    for (int j = 0; j < n; j++) {
        const int r = gamma_rows(j, nx, nu);
        G[j] = p;
        unpack(hpGamma[j], rup(nx[j + 1], NCL), r, nx[j + 1], G[j], r);
        p += (long)r * nx[j + 1];
    }
    return p;
}

/* d_part_cond.c:214-308: Gamma_0 = BAbt_0, Gamma_j = [B_j ; Gamma_{j-1} A_j] + b_j e_last (lib4, rows r_j, panel
 * stride cnx_{j+1}); pBAbt2 = Gamma_{N-1}.  Dense column-major temporaries in work. */
void orc_d_cond_BAbt(int N, int *nx, int *nu, double **hpBAbt, double *work, double **hpGamma, double *pBAbt2) {
    if (N < 1) return;
    double *G[N];
    double *p = work;
    for (int j = 0; j < N; j++) {
        G[j] = p;
        p += (long)gamma_rows(j, nx, nu) * nx[j + 1];
    }
    {
        const int nux = nu[0] + nx[0], cnx1 = rup(nx[1], NCL);
        unpack(hpBAbt[0], cnx1, nux + 1, nx[1], G[0], gamma_rows(0, nx, nu));
    }
    for (int j = 1; j < N; j++) {
        const int nuj = nu[j], nxj = nx[j], nx1 = nx[j + 1], cnx1 = rup(nx1, NCL), r0 = gamma_rows(j - 1, nx, nu),
                  rj = r0 + nuj;
        double *Gj = G[j], *Gp = G[j - 1];
        for (int c = 0; c < nx1; c++) {
            for (int i = 0; i < nuj; i++) Gj[i + c * rj] = *P4(hpBAbt[j], cnx1, i, c);
            for (int i = 0; i < r0; i++) {
                double a = 0.0;
                for (int l = 0; l < nxj; l++) a += Gp[i + l * r0] * *P4(hpBAbt[j], cnx1, nuj + l, c);
                Gj[nuj + i + c * rj] = a;
            }
            Gj[rj - 1 + c * rj] += *P4(hpBAbt[j], cnx1, nuj + nxj, c);
        }
    }
    for (int j = 0; j < N; j++) {
        const int r = gamma_rows(j, nx, nu);
        pack(G[j], r, r, nx[j + 1], hpGamma[j], rup(nx[j + 1], NCL));
    }
    pack(G[N - 1], gamma_rows(N - 1, nx, nu), gamma_rows(N - 1, nx, nu), nx[N], pBAbt2, rup(nx[N], NCL));
}

/* d_part_cond.c:312-574: the condensed Hessian [D M'; M P] with its gradient row, from the given Gammas.  Writes
 * the lower triangle of every column block the reference writes (the reference also copies the strict upper
 * triangle of the u_s x u_s blocks from its work matrix; not part of the result). */
void orc_d_cond_RSQrq(int N, int *nx, int *nu, double **hpBAbt, double **hpRSQrq, double **hpGamma, double *work,
                      double *pRSQ2) {
    if (N < 1) return;
    const int T = N, nx0 = nx[0];
    int nut = 0;
    for (int j = 0; j < T; j++) nut += nu[j];
    const int nv = nut + nx0, cnux2 = rup(nv, NCL);
    if (T == 1) {
        const int nux = nu[0] + nx[0], cnux = rup(nux, NCL);
        for (int c = 0; c < nux; c++)
            for (int i = c; i <= nux; i++) *P4(pRSQ2, cnux2, i, c) = *P4(hpRSQrq[0], cnux, i, c);
        return;
    }
    double *G[T];
    double *p = gamma_dense(T - 1, nx, nu, hpGamma, work, G);
    /* off[s]: column of u_s in the condensed variables = sum_{r > s} nu_r (nu3 in d_cond_RSQrq) */
    int off[T + 1];
    off[T] = 0;
    for (int s = T - 1; s >= 0; s--) off[s] = (s == T - 1 ? 0 : off[s + 1] + nu[s + 1]);
    /* pL: dense (nux_s+1) x nux_s accumulated Hessian of stage s (lower triangle + last row) */
    int nzM = 0;
    for (int j = 0; j < T; j++)
        if (nu[j] + nx[j] + 1 > nzM) nzM = nu[j] + nx[j] + 1;
    double *pL = p, *Lx = pL + nzM * nzM, *W = Lx + nzM * nzM, *tmp = W + nzM * nzM, *dLx = tmp + nzM * nzM;
    int s = T - 1;
    {
        const int nux = nu[s] + nx[s], cnux = rup(nux, NCL);
        for (int c = 0; c < nux; c++)
            for (int i = c; i <= nux; i++) pL[i + c * (nux + 1)] = *P4(hpRSQrq[s], cnux, i, c);
    }
    for (;;) {
        const int nus = nu[s], nxs = nx[s], nux = nus + nxs, ld = nux + 1;
        if (s == 0) {
            /* D, M, m, P, p of the first stage: the whole pL at (off_0, off_0) */
            for (int c = 0; c < nux; c++)
                for (int i = c; i <= nux; i++) *P4(pRSQ2, cnux2, off[0] + i, off[0] + c) = pL[i + c * ld];
            break;
        }
        /* D: the u_s x u_s block */
        for (int c = 0; c < nus; c++)
            for (int i = c; i < nus; i++) *P4(pRSQ2, cnux2, off[s] + i, off[s] + c) = pL[i + c * ld];
        /* M: Gamma_{s-1} (rows [u_{s-1}..u_0, x_0, 1]) times the x_s x u_s block; its last row is the
         * gradient row, to which m (the r row of pL) is added */
        const int r0 = gamma_rows(s - 1, nx, nu);
        for (int c = 0; c < nus; c++) {
            for (int i = 0; i < r0; i++) {
                double a = 0.0;
                for (int l = 0; l < nxs; l++) a += G[s - 1][i + l * r0] * pL[nus + l + c * ld];
                if (i == r0 - 1) a += pL[nux + c * ld];
                *P4(pRSQ2, cnux2, off[s] + nus + i, off[s] + c) = a;
            }
        }
        /* state cost-to-go of x_s: Lx = chol_aug(pL[x, x] with its gradient row) */
        const int ldx = nxs + 1;
        for (int c = 0; c < nxs; c++)
            for (int i = c; i <= nxs; i++) tmp[i + c * ldx] = pL[nus + i + (nus + c) * ld];
        orc__chol_aug(nxs + 1, nxs, tmp, ldx, Lx, ldx, dLx);
        /* W = BAbt_{s-1} Lx (dtrmm_nt_u), last row += l (dgead), pL = RSQ_{s-1} + W W' (dsyrk_nt) */
        const int sp = s - 1, nuxp = nu[sp] + nx[sp], ldp = nuxp + 1, cnx1 = rup(nxs, NCL), cnuxp = rup(nuxp, NCL);
        for (int c = 0; c < nxs; c++)
            for (int i = 0; i <= nuxp; i++) {
                double a = 0.0;
                for (int l = c; l < nxs; l++) a += *P4(hpBAbt[sp], cnx1, i, l) * Lx[l + c * ldx];
                W[i + c * ldp] = a;
            }
        for (int c = 0; c < nxs; c++) W[nuxp + c * ldp] += Lx[nxs + c * ldx];
        for (int c = 0; c < nuxp; c++)
            for (int i = c; i <= nuxp; i++) {
                double a = 0.0;
                for (int l = 0; l < nxs; l++) a += W[i + l * ldp] * W[c + l * ldp];
                pL[i + c * ldp] = *P4(hpRSQrq[sp], cnuxp, i, c) + a;
            }
        s = sp;
    }
}

/* d_part_cond.c:579-689: input boxes stay boxes, state boxes of stages 1..N-1 become general constraints on
 * [u_{s-1} .. u_0, x_0] through Gamma_{s-1}; stage 0's boxes all stay boxes.  Only the slots the reference
 * assigns are written. */
void orc_d_cond_DCtd(int N, int *nx, int *nu, int *nb, int **hidxb, double **hd, double **hpGamma, double *pDCt2,
                     double *d2, int *idxb2) {
    if (N < 1) return;
    const int T = N;
    int nbb = nb[0], nbg = 0;
    for (int s = 1; s < T; s++)
        for (int jj = 0; jj < nb[s]; jj++) {
            if (hidxb[s][jj] < nu[s])
                nbb++;
            else
                nbg++;
        }
    const int pnbb = rup(nbb, BS), pnbg = rup(nbg, BS), cnbg = rup(nbg, NCL);
    int ib = 0, ig = 0, nu_tmp = 0, idx_gammab = nx[0];
    for (int j = 0; j < T - 1; j++) idx_gammab += nu[j];
    for (int s = T - 1; s >= 1; s--) {
        nu_tmp += nu[s];
        const int pnbs = rup(nb[s], BS), sdg = rup(nx[s], NCL);
        for (int jj = 0; jj < nb[s]; jj++) {
            const int v = hidxb[s][jj];
            if (v < nu[s]) {
                d2[ib] = hd[s][jj];
                d2[pnbb + ib] = hd[s][pnbs + jj];
                idxb2[ib] = nu_tmp - nu[s] + v;
                ib++;
            } else {
                const int g = v - nu[s];
                const double c0 = *P4(hpGamma[s - 1], sdg, idx_gammab, g);
                d2[2 * pnbb + ig] = hd[s][jj] - c0;
                d2[2 * pnbb + pnbg + ig] = hd[s][pnbs + jj] - c0;
                for (int i = 0; i < idx_gammab; i++) *P4(pDCt2, cnbg, nu_tmp + i, ig) = *P4(hpGamma[s - 1], sdg, i, g);
                ig++;
            }
        }
        idx_gammab -= nu[s - 1];
    }
    nu_tmp += nu[0];
    const int pnb0 = rup(nb[0], BS);
    for (int jj = 0; jj < nb[0]; jj++) {
        d2[ib] = hd[0][jj];
        d2[pnbb + ib] = hd[0][pnb0 + jj];
        idxb2[ib] = nu_tmp - nu[0] + hidxb[0][jj];
        ib++;
    }
}

/* Condense one block of T stages: the three building blocks on cleared outputs (the condensed arrays of
 * d_part_cond), the Gammas as lib4 matrices at the start of work.  Outputs are lib4 (BAbt2 sd cnx2',
 * RSQ2 sd cnux2, DCt2 sd cng2) and the padded d2/idxb2. */
static void cond_block(int T, int *nx, int *nu, int *nb, int **hidxb, double **hpBAbt, double **hpRSQrq, double **hd,
                       double *pBAbt2, double *pRSQ2, double *pDCt2, double *d2, int *idxb2, double *work) {
    int nut = 0;
    for (int j = 0; j < T; j++) nut += nu[j];
    const int nv = nut + nx[0];
    double *hpGamma[T];
    double *p = work;
    for (int j = 0; j < T; j++) {
        hpGamma[j] = p;
        p += (long)rup(gamma_rows(j, nx, nu), BS) * rup(nx[j + 1], NCL);
    }
    int nbb = nb[0], nbg = 0;
    for (int s = 1; s < T; s++)
        for (int jj = 0; jj < nb[s]; jj++) {
            if (hidxb[s][jj] < nu[s])
                nbb++;
            else
                nbg++;
        }
    for (int i = 0; i < rup(nv + 1, BS) * rup(nv, NCL); i++) pRSQ2[i] = 0.0;
    for (int i = 0; i < rup(nv, BS) * rup(nbg, NCL); i++) pDCt2[i] = 0.0;
    for (int i = 0; i < 2 * rup(nbb, BS) + 2 * rup(nbg, BS); i++) d2[i] = 0.0;
    orc_d_cond_BAbt(T, nx, nu, hpBAbt, p, hpGamma, pBAbt2);
    orc_d_cond_RSQrq(T, nx, nu, hpBAbt, hpRSQrq, hpGamma, p, pRSQ2);
    orc_d_cond_DCtd(T, nx, nu, nb, hidxb, hd, hpGamma, pDCt2, d2, idxb2);
}

/* d_part_cond.c:926-1062 */
void orc_d_part_cond(int N, int *nx, int *nu, int *nb, int **hidxb, int *ng, double **hpBAbt, double **hpRSQrq,
                     double **hpDCt, double **hd, int N2, int *nx2, int *nu2, int *nb2, int **hidxb2, int *ng2,
                     double **hpBAbt2, double **hpRSQrq2, double **hpDCt2, double **hd2, void *memory, void *work) {
    if (N2 == N) { /* :936-960: the condensed problem aliases the original */
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
    /* the reference carve (:1013-1041) */
    double *ptr = (double *)memory;
    for (int ii = 0; ii < N2; ii++) {
        hpBAbt2[ii] = ptr;
        ptr += rup(nu2[ii] + nx2[ii] + 1, BS) * rup(nx2[ii + 1], NCL);
    }
    for (int ii = 0; ii < N2; ii++) {
        hpRSQrq2[ii] = ptr;
        ptr += rup(nu2[ii] + nx2[ii] + 1, BS) * rup(nu2[ii] + nx2[ii], NCL);
    }
    for (int ii = 0; ii < N2; ii++) {
        hpDCt2[ii] = ptr;
        ptr += rup(nu2[ii] + nx2[ii], BS) * rup(ng2[ii], NCL);
    }
    for (int ii = 0; ii < N2; ii++) {
        hd2[ii] = ptr;
        ptr += 2 * rup(nb2[ii], BS) + 2 * rup(ng2[ii], BS);
    }
    int *iptr = (int *)ptr;
    for (int ii = 0; ii < N2; ii++) {
        hidxb2[ii] = iptr;
        iptr += nb2[ii];
    }
    int N_tmp = 0;
    for (int ii = 0; ii < N2; ii++) {
        const int T1 = block_len(N, N2, ii);
        cond_block(T1, nx + N_tmp, nu + N_tmp, nb + N_tmp, hidxb + N_tmp, hpBAbt + N_tmp, hpRSQrq + N_tmp, hd + N_tmp,
                   hpBAbt2[ii], hpRSQrq2[ii], hpDCt2[ii], hd2[ii], hidxb2[ii], (double *)work);
        N_tmp += T1;
    }
    hpRSQrq2[N2] = hpRSQrq[N];
    hpDCt2[N2] = hpDCt[N];
    hd2[N2] = hd[N];
    hidxb2[N2] = hidxb[N];
}

/* d_part_cond.c:1066-1099 */
int orc_d_part_expand_work_space_size_bytes(int N, int *nx, int *nu, int *nb, int *ng) {
    int nzM = 0, ngM = 0;
    for (int ii = 0; ii <= N; ii++) {
        if (nu[ii] + nx[ii] + 1 > nzM) nzM = nu[ii] + nx[ii] + 1;
        if (ng[ii] > ngM) ngM = ng[ii];
    }
    return ((rup(nzM, BS) + rup(ngM, BS)) * 8 + 63) / 64 * 64;
}

/* d_part_cond.c:1103-1308 */
void orc_d_part_expand_solution(int N, int *nx, int *nu, int *nb, int **hidxb, int *ng, double **hpBAbt, double **hb,
                                double **hpRSQrq, double **hrq, double **hpDCt, double **hux, double **hpi,
                                double **hlam, double **ht, int N2, int *nx2, int *nu2, int *nb2, int **hidxb2,
                                int *ng2, double **hux2, double **hpi2, double **hlam2, double **ht2, void *work) {
    double *w0 = (double *)work;
    int nzM = 0;
    for (int ii = 0; ii <= N; ii++)
        if (nu[ii] + nx[ii] + 1 > nzM) nzM = nu[ii] + nx[ii] + 1;
    double *w1 = w0 + rup(nzM, BS);
    /* inputs (reverse stage order) and each block's first state */
    int N_tmp = 0;
    for (int ii = 0; ii < N2; ii++) {
        const int T1 = block_len(N, N2, ii);
        int nu_tmp = 0;
        for (int jj = 0; jj < T1 - 1; jj++) {
            const int s = N_tmp + T1 - 1 - jj;
            for (int l = 0; l < nu[s]; l++) hux[s][l] = hux2[ii][nu_tmp + l];
            nu_tmp += nu[s];
        }
        for (int l = 0; l < nu[N_tmp] + nx[N_tmp]; l++) hux[N_tmp][l] = hux2[ii][nu_tmp + l];
        N_tmp += T1;
    }
    for (int l = 0; l < nx[N]; l++) hux[N][l] = hux2[N2][l];
    /* states inside each block by simulation, x_{j+1} = b_j + BAbt_j' ux_j (dgemv_t, alg 1) */
    N_tmp = 0;
    for (int ii = 0; ii < N2; ii++) {
        const int T1 = block_len(N, N2, ii);
        for (int jj = 0; jj < T1 - 1; jj++) {
            const int s = N_tmp + jj, nux = nu[s] + nx[s], nx1 = nx[s + 1], cnx1 = rup(nx1, NCL);
            double *x1 = hux[s + 1] + nu[s + 1];
            for (int c = 0; c < nx1; c++) {
                double a = 0.0;
                for (int i = 0; i < nux; i++) a += *P4(hpBAbt[s], cnx1, i, c) * hux[s][i];
                x1[c] = hb[s][c] + a;
            }
        }
        N_tmp += T1;
    }
    /* slacks and inequality multipliers: boxes of later stages first, state boxes from the generals */
    N_tmp = 0;
    for (int ii = 0; ii < N2; ii++) {
        const int T1 = block_len(N, N2, ii), pnb2 = rup(nb2[ii], BS), png2 = rup(ng2[ii], BS);
        int nbb2_tmp = 0, nbg2_tmp = 0;
        for (int jj = 0; jj < T1 - 1; jj++) {
            const int s = N_tmp + T1 - 1 - jj, pnb = rup(nb[s], BS);
            int nbb2 = 0, nbg2 = 0;
            for (int l = 0; l < nb[s]; l++) {
                if (hidxb[s][l] < nu[s])
                    nbb2++;
                else
                    nbg2++;
            }
            for (int l = 0; l < nbb2; l++) {
                hlam[s][l] = hlam2[ii][nbb2_tmp + l];
                hlam[s][pnb + l] = hlam2[ii][pnb2 + nbb2_tmp + l];
                ht[s][l] = ht2[ii][nbb2_tmp + l];
                ht[s][pnb + l] = ht2[ii][pnb2 + nbb2_tmp + l];
            }
            for (int l = 0; l < nbg2; l++) {
                hlam[s][nbb2 + l] = hlam2[ii][2 * pnb2 + nbg2_tmp + l];
                hlam[s][pnb + nbb2 + l] = hlam2[ii][2 * pnb2 + png2 + nbg2_tmp + l];
                ht[s][nbb2 + l] = ht2[ii][2 * pnb2 + nbg2_tmp + l];
                ht[s][pnb + nbb2 + l] = ht2[ii][2 * pnb2 + png2 + nbg2_tmp + l];
            }
            nbb2_tmp += nbb2;
            nbg2_tmp += nbg2;
        }
        const int s = N_tmp, pnb = rup(nb[s], BS);
        for (int l = 0; l < nb[s]; l++) {
            hlam[s][l] = hlam2[ii][nbb2_tmp + l];
            hlam[s][pnb + l] = hlam2[ii][pnb2 + nbb2_tmp + l];
            ht[s][l] = ht2[ii][nbb2_tmp + l];
            ht[s][pnb + l] = ht2[ii][pnb2 + nbb2_tmp + l];
        }
        N_tmp += T1;
    }
    {
        const int pnb = rup(nb[N], BS), png = rup(ng[N], BS), pnb2 = rup(nb2[N2], BS), png2 = rup(ng2[N2], BS);
        for (int j = 0; j < nb[N]; j++) {
            hlam[N][j] = hlam2[N2][j];
            hlam[N][pnb + j] = hlam2[N2][pnb2 + j];
            ht[N][j] = ht2[N2][j];
            ht[N][pnb + j] = ht2[N2][pnb2 + j];
        }
        for (int j = 0; j < ng[N]; j++) {
            hlam[N][2 * pnb + j] = hlam2[N2][2 * pnb2 + j];
            hlam[N][2 * pnb + png + j] = hlam2[N2][2 * pnb2 + png2 + j];
            ht[N][2 * pnb + j] = ht2[N2][2 * pnb2 + j];
            ht[N][2 * pnb + png + j] = ht2[N2][2 * pnb2 + png2 + j];
        }
    }
    /* equality multipliers: the block's last pi is the condensed one; inner ones by the backward
     * stationarity recursion pi_{s-1} = [RSQ_s ux_s + rq_s + box terms + BAbt_s pi_s + DCt_s (lam_u - lam_l)]_x */
    N_tmp = 0;
    for (int ii = 0; ii < N2; ii++) {
        const int T1 = block_len(N, N2, ii);
        for (int l = 0; l < nx[N_tmp + T1]; l++) hpi[N_tmp + T1 - 1][l] = hpi2[ii][l];
        for (int jj = 0; jj < T1 - 1; jj++) {
            const int s = N_tmp + T1 - 1 - jj, nux = nu[s] + nx[s], cnux = rup(nux, NCL), pnb = rup(nb[s], BS),
                      png = rup(ng[s], BS), nx1 = nx[s + 1], cnx1 = rup(nx1, NCL), cng = rup(ng[s], NCL);
            for (int l = 0; l < nux; l++) w0[l] = hrq[s][l];
            for (int l = 0; l < nb[s]; l++) w0[hidxb[s][l]] += -hlam[s][l] + hlam[s][pnb + l];
            for (int i = 0; i < nux; i++) { /* dsymv_lib, lower triangle */
                double a = 0.0;
                for (int j = 0; j < nux; j++)
                    a += (i >= j ? *P4(hpRSQrq[s], cnux, i, j) : *P4(hpRSQrq[s], cnux, j, i)) * hux[s][j];
                w0[i] += a;
            }
            for (int i = 0; i < nux; i++) { /* dgemv_n_lib, alg 1 */
                double a = 0.0;
                for (int j = 0; j < nx1; j++) a += *P4(hpBAbt[s], cnx1, i, j) * hpi[s][j];
                w0[i] += a;
            }
            for (int l = 0; l < ng[s]; l++) w1[l] = hlam[s][2 * pnb + png + l] - hlam[s][2 * pnb + l];
            for (int i = 0; i < nux && ng[s] > 0; i++) {
                double a = 0.0;
                for (int j = 0; j < ng[s]; j++) a += *P4(hpDCt[s], cng, i, j) * w1[j];
                w0[i] += a;
            }
            for (int l = 0; l < nx[s]; l++) hpi[s - 1][l] = w0[nu[s] + l];
        }
        N_tmp += T1;
    }
}
