/*
 * hpmpc_oracle_soft.c -- TEST INFRASTRUCTURE ONLY (parity checker; see hpmpc_oracle.h).
 *
 * CPU restatement of the soft-constraint IPM d_ip2_mpc_soft_tv (mpc_solvers/d_ip2_soft.c:83-547) and
 * its vector routines (mpc_solvers/c99/d_aux_ip_soft_lib4.c:38-999), over the restated Riccati
 * (orc_d_back_ric_rec_sv_tv_res / _trs_, hpmpc_oracle.c).  Pinned by the reference build's outputs
 * (tests/golden/soft_*.npz, tests/golden/make_golden.py soft).
 *
 * The reference is restated as it behaves, including two layout quirks (soft constraints):
 *   - b_k is read from the augmented row of BAbt_k with the panel stride round_up(nx_{k+1}, 4) instead of
 *     the lib4 stride round_up(nx_{k+1}, 2) (d_ip2_soft.c:172); where the two differ the read leaves the
 *     buffer for nu+nx >= 4, so such sizes are rejected (-10) rather than restated;
 *   - d_update_gradient_mpc_soft_tv adds the soft corrector term at qx[k] + pnbs + nb + i when nb > 0
 *     (d_aux_ip_soft_lib4.c:557, :601) -- past the slots the Riccati reads -- so Qx / qx and Zl / zl
 *     live in one flat block in the reference's order (d_ip2_soft.c:244-260) and the stray write lands
 *     where it lands in the reference.
 * General constraints with soft constraints (ng > 0) are rejected (-10): the reference's general-constraint
 * branch of the soft gradient update indexes past its own vectors (d_aux_ip_soft_lib4.c:565-576).
 */
#include <math.h>
#include <stdlib.h>
#include <string.h>

#include "hpmpc_oracle.h"

#define BS 4
#define NCL 2

static inline int rup(int n, int m) { return (n + m - 1) / m * m; }
static inline double *P4(double *pA, int sd, int i, int j) { return pA + (i / BS) * BS * sd + i % BS + BS * j; }

typedef struct {
    double *work, *memory, *flat;
    double **b, **q, **dux, **dpi, **Pb, **bd, **dlam, **dt, **lamt, **t_inv, **Qx, **qx, **Zl, **zl;
} sws_t;

/* workspace carve (doubles); ptrs: 14 (N+1) pointer slots */
static long sws_carve(int N, int *nx, int *nu, int *nb, int *ng, int *ns, double *base, sws_t *w, double **ptrs) {
    int nbs[N + 1];
    for (int k = 0; k <= N; k++) nbs[k] = nb[k] + ns[k];
    long off = 0;
    if (w) {
        double ***t[14] = {&w->b,  &w->q,    &w->dux,  &w->dpi,   &w->Pb, &w->bd, &w->dlam,
                           &w->dt, &w->lamt, &w->t_inv, &w->Qx,    &w->qx, &w->Zl, &w->zl};
        for (int i = 0; i < 14; i++) *t[i] = ptrs + i * (N + 1);
        w->work = base + off;
    }
    off += orc_d_back_ric_rec_sv_tv_work_space_size_bytes(N, nx, nu, nbs, ng) / 8;
    if (w) w->memory = base + off;
    off += orc_d_back_ric_rec_sv_tv_memory_space_size_bytes(N, nx, nu, nbs, ng) / 8;
#define TAKE(field, n)                   \
    do {                                 \
        if (w) w->field[k] = base + off; \
        off += (n);                      \
    } while (0)
    for (int k = 0; k <= N; k++) {
        const int pnz = rup(nu[k] + nx[k] + 1, BS), pnx1 = k < N ? rup(nx[k + 1], BS) : 0;
        const int pnb = rup(nb[k], BS), png = rup(ng[k], BS), pns = rup(ns[k], BS);
        const int nc = 2 * pnb + 2 * png + 4 * pns;
        TAKE(b, pnx1);
        TAKE(q, pnz);
        TAKE(dux, pnz);
        TAKE(dpi, pnx1);
        TAKE(Pb, pnx1);
        TAKE(bd, pnb + pns);
        TAKE(dlam, nc);
        TAKE(dt, nc);
        TAKE(lamt, nc);
        TAKE(t_inv, nc);
    }
    /* Qx/qx then Zl/zl in the reference's order (d_ip2_soft.c:244-260), then room for the stray writes */
    if (w) w->flat = base + off;
    int padM = 0;
    for (int k = 0; k <= N; k++) {
        const int pnb = rup(nb[k], BS), png = rup(ng[k], BS), pns = rup(ns[k], BS);
        if (w) {
            w->Qx[k] = base + off;
            w->qx[k] = base + off + pnb + png + pns;
        }
        off += 2 * (pnb + png + pns);
        if (2 * (pnb + pns) > padM) padM = 2 * (pnb + pns);
    }
    for (int k = 0; k <= N; k++) {
        const int pns = rup(ns[k], BS);
        if (w) {
            w->Zl[k] = base + off;
            w->zl[k] = base + off + 2 * pns;
        }
        off += 4 * pns;
    }
    off += padM + 8;
#undef TAKE
    return off;
}

int orc_d_ip2_mpc_soft_tv_work_space_size_bytes(int N, int *nx, int *nu, int *nb, int *ng, int *ns) {
    long n = sws_carve(N, nx, nu, nb, ng, ns, NULL, NULL, NULL);
    return (int)((n * 8 + 63) / 64 * 64);
}

/* d_init_var_mpc_soft_tv (d_aux_ip_soft_lib4.c:38-165), ng = 0 */
static void init_var_soft(int N, int *nx, int *nu, int *nb, int **idxb, int *ns, double **ux, double **pi,
                          double **db, double **t, double **lam, double mu0, int warm_start) {
    const double thr0 = 0.1;
    if (!warm_start)
        for (int k = 0; k <= N; k++)
            for (int l = 0; l < nu[k] + nx[k]; l++) ux[k][l] = 0.0;
    for (int k = 0; k <= N; k++) {
        const int pnb = rup(nb[k], BS);
        for (int l = 0; l < nb[k]; l++) {
            const int i = idxb[k][l];
            t[k][l] = -db[k][l] + ux[k][i];
            t[k][pnb + l] = db[k][pnb + l] - ux[k][i];
            if (t[k][l] < thr0) {
                if (t[k][pnb + l] < thr0) {
                    ux[k][i] = (-db[k][pnb + l] + db[k][l]) * 0.5;
                    t[k][l] = thr0;
                    t[k][pnb + l] = thr0;
                } else {
                    t[k][l] = thr0;
                    ux[k][i] = db[k][l] + thr0;
                }
            } else if (t[k][pnb + l] < thr0) {
                t[k][pnb + l] = thr0;
                ux[k][i] = db[k][pnb + l] - thr0;
            }
            lam[k][l] = mu0 / t[k][l];
            lam[k][pnb + l] = mu0 / t[k][pnb + l];
        }
    }
    for (int k = 0; k <= N; k++) {
        const int pnb = rup(nb[k], BS), pns = rup(ns[k], BS);
        for (int l = 0; l < ns[k]; l++)
            for (int s = 0; s < 4; s++) {
                t[k][2 * pnb + s * pns + l] = 1.0;
                lam[k][2 * pnb + s * pns + l] = mu0;
            }
    }
    for (int k = 0; k < N; k++)
        for (int l = 0; l < nx[k + 1]; l++) pi[k][l] = 0.0;
}

/* d_update_hessian_mpc_soft_tv (:167-506) */
static void update_hessian_soft(int N, int *nb, int *ns, double **db, double sigma_mu, double **t, double **tinv,
                                double **lam, double **lamt, double **dlam, double **Qx, double **qx, double **Z,
                                double **z, double **Zl, double **zl) {
    for (int k = 0; k <= N; k++) {
        const int nb0 = nb[k], ns0 = ns[k], pnb = rup(nb0, BS), pns = rup(ns0, BS);
        double *pt = t[k], *pl = lam[k], *plt = lamt[k], *pdl = dlam[k], *pti = tinv[k], *pd = db[k];
        for (int i = 0; i < nb0; i++) {
            pti[i] = 1.0 / pt[i];
            pti[pnb + i] = 1.0 / pt[pnb + i];
            plt[i] = pl[i] * pti[i];
            plt[pnb + i] = pl[pnb + i] * pti[pnb + i];
            pdl[i] = pti[i] * sigma_mu;
            pdl[pnb + i] = pti[pnb + i] * sigma_mu;
            Qx[k][i] = plt[i] + plt[pnb + i];
            qx[k][i] = pl[pnb + i] - plt[pnb + i] * pd[pnb + i] + pdl[pnb + i] - pl[i] - plt[i] * pd[i] - pdl[i];
        }
        if (nb0 > 0) {
            pt += 2 * pnb;
            pl += 2 * pnb;
            plt += 2 * pnb;
            pdl += 2 * pnb;
            pti += 2 * pnb;
            pd += 2 * pnb;
        }
        for (int i = 0; i < ns0; i++) {
            for (int s = 0; s < 4; s++) {
                pti[s * pns + i] = 1.0 / pt[s * pns + i];
                plt[s * pns + i] = pl[s * pns + i] * pti[s * pns + i];
                pdl[s * pns + i] = pti[s * pns + i] * sigma_mu;
            }
            double rQx0 = plt[i], rQx1 = plt[pns + i];
            double rqx0 = pl[i] + pdl[i] + plt[i] * pd[i];
            double rqx1 = pl[pns + i] + pdl[pns + i] - plt[pns + i] * pd[pns + i];
            Zl[k][i] = 1.0 / (Z[k][i] + rQx0 + plt[2 * pns + i]);
            Zl[k][pns + i] = 1.0 / (Z[k][pns + i] + rQx1 + plt[3 * pns + i]);
            zl[k][i] = -z[k][i] + rqx0 + pl[2 * pns + i] + pdl[2 * pns + i];
            zl[k][pns + i] = -z[k][pns + i] + rqx1 + pl[3 * pns + i] + pdl[3 * pns + i];
            rqx0 = rqx0 - rQx0 * zl[k][i] * Zl[k][i];
            rqx1 = rqx1 - rQx1 * zl[k][pns + i] * Zl[k][pns + i];
            rQx0 = rQx0 - rQx0 * rQx0 * Zl[k][i];
            rQx1 = rQx1 - rQx1 * rQx1 * Zl[k][pns + i];
            Qx[k][nb0 + i] = rQx1 + rQx0;
            qx[k][nb0 + i] = rqx1 - rqx0;
        }
    }
}

/* d_update_gradient_mpc_soft_tv (:508-609), ng = 0: the soft term goes to qx[k] + pnbs + nb + i when nb > 0 */
static void update_gradient_soft(int N, int *nb, int *ns, double sigma_mu, double **dt, double **dlam,
                                 double **t_inv, double **lamt, double **qx, double **Zl, double **zl) {
    for (int k = 0; k <= N; k++) {
        const int nb0 = nb[k], ns0 = ns[k], pnb = rup(nb0, BS), pns = rup(ns0, BS), pnbs = rup(nb0 + ns0, BS);
        double *pdl = dlam[k], *pdt = dt[k], *plt = lamt[k], *pti = t_inv[k], *pq = qx[k];
        if (nb0 > 0) {
            for (int i = 0; i < nb0; i++) {
                pdl[i] = pti[i] * (sigma_mu - pdl[i] * pdt[i]);
                pdl[pnb + i] = pti[pnb + i] * (sigma_mu - pdl[pnb + i] * pdt[pnb + i]);
                pq[i] += pdl[pnb + i] - pdl[i];
            }
            pdl += 2 * pnb;
            pdt += 2 * pnb;
            plt += 2 * pnb;
            pti += 2 * pnb;
            pq = qx[k] + pnbs;
        }
        for (int i = 0; i < ns0; i++) {
            for (int s = 0; s < 4; s++) pdl[s * pns + i] = pti[s * pns + i] * (sigma_mu - pdl[s * pns + i] * pdt[s * pns + i]);
            const double rQx0 = plt[i], rQx1 = plt[pns + i];
            double rqx0 = pdl[i], rqx1 = pdl[pns + i];
            zl[k][i] += rqx0 + pdl[2 * pns + i];
            zl[k][pns + i] += rqx1 + pdl[3 * pns + i];
            rqx0 = rqx0 - rQx0 * (rqx0 + pdl[2 * pns + i]) * Zl[k][i];
            rqx1 = rqx1 - rQx1 * (rqx1 + pdl[3 * pns + i]) * Zl[k][pns + i];
            pq[nb0 + i] += rqx1 - rqx0;
        }
    }
}

static inline void alpha_rule(double *alpha, double v, double dv) {
    if (-*alpha * dv > v) *alpha = -v / dv;
}

/* d_compute_alpha_mpc_soft_tv (:611-804), ng = 0 */
static void compute_alpha_soft(int N, int *nb, int **idxb, int *ns, double *ptr_alpha, double **t, double **dt,
                               double **lam, double **dlam, double **lamt, double **dux, double **db, double **Zl,
                               double **zl) {
    double alpha = *ptr_alpha;
    for (int k = 0; k <= N; k++) {
        const int nb0 = nb[k], ns0 = ns[k], pnb = rup(nb0, BS), pns = rup(ns0, BS);
        double *pd = db[k], *pt = t[k], *pdt = dt[k], *plt = lamt[k], *pl = lam[k], *pdl = dlam[k], *ux = dux[k];
        if (nb0 > 0) {
            for (int l = 0; l < nb0; l++) {
                const double x = ux[idxb[k][l]];
                pdt[l] = x - pd[l] - pt[l];
                pdt[pnb + l] = -x + pd[pnb + l] - pt[pnb + l];
                pdl[l] -= plt[l] * pdt[l] + pl[l];
                pdl[pnb + l] -= plt[pnb + l] * pdt[pnb + l] + pl[pnb + l];
                alpha_rule(&alpha, pl[l], pdl[l]);
                alpha_rule(&alpha, pl[pnb + l], pdl[pnb + l]);
                alpha_rule(&alpha, pt[l], pdt[l]);
                alpha_rule(&alpha, pt[pnb + l], pdt[pnb + l]);
            }
            pd += 2 * pnb;
            pt += 2 * pnb;
            pdt += 2 * pnb;
            plt += 2 * pnb;
            pl += 2 * pnb;
            pdl += 2 * pnb;
        }
        for (int l = 0; l < ns0; l++) {
            const double x = ux[idxb[k][nb0 + l]];
            pdt[2 * pns + l] = (zl[k][l] - plt[l] * x) * Zl[k][l];
            pdt[3 * pns + l] = (zl[k][pns + l] + plt[pns + l] * x) * Zl[k][pns + l];
            pdt[l] = pdt[2 * pns + l] + x - pd[l] - pt[l];
            pdt[pns + l] = pdt[3 * pns + l] - x + pd[pns + l] - pt[pns + l];
            pdt[2 * pns + l] -= pt[2 * pns + l];
            pdt[3 * pns + l] -= pt[3 * pns + l];
            for (int s = 0; s < 4; s++) pdl[s * pns + l] -= plt[s * pns + l] * pdt[s * pns + l] + pl[s * pns + l];
            for (int s = 0; s < 4; s++) alpha_rule(&alpha, pl[s * pns + l], pdl[s * pns + l]);
            for (int s = 0; s < 4; s++) alpha_rule(&alpha, pt[s * pns + l], pdt[s * pns + l]);
        }
    }
    *ptr_alpha = alpha;
}

/* d_compute_mu_mpc_soft_tv (:926-999) */
static void compute_mu_soft(int N, int *nb, int *ns, double *ptr_mu, double mu_scal, double alpha, double **lam,
                            double **dlam, double **t, double **dt) {
    double mu = 0.0;
    for (int k = 0; k <= N; k++) {
        const int pnb = rup(nb[k], BS), pns = rup(ns[k], BS);
        const double *pl = lam[k], *pdl = dlam[k], *pt = t[k], *pdt = dt[k];
        for (int l = 0; l < nb[k]; l++)
            mu += (pl[l] + alpha * pdl[l]) * (pt[l] + alpha * pdt[l]) +
                  (pl[pnb + l] + alpha * pdl[pnb + l]) * (pt[pnb + l] + alpha * pdt[pnb + l]);
        pl += 2 * pnb;
        pdl += 2 * pnb;
        pt += 2 * pnb;
        pdt += 2 * pnb;
        for (int l = 0; l < ns[k]; l++)
            mu += (pl[l] + alpha * pdl[l]) * (pt[l] + alpha * pdt[l]) +
                  (pl[pns + l] + alpha * pdl[pns + l]) * (pt[pns + l] + alpha * pdt[pns + l]) +
                  (pl[2 * pns + l] + alpha * pdl[2 * pns + l]) * (pt[2 * pns + l] + alpha * pdt[2 * pns + l]) +
                  (pl[3 * pns + l] + alpha * pdl[3 * pns + l]) * (pt[3 * pns + l] + alpha * pdt[3 * pns + l]);
    }
    *ptr_mu = mu * mu_scal;
}

/* d_update_var_mpc_soft_tv (:806-924) */
static void update_var_soft(int N, int *nx, int *nu, int *nb, int *ns, double *ptr_mu, double mu_scal, double alpha,
                            double **ux, double **dux, double **t, double **dt, double **lam, double **dlam,
                            double **pi, double **dpi) {
    double mu = 0.0;
    for (int k = 0; k <= N; k++) {
        const int pnb = rup(nb[k], BS), pns = rup(ns[k], BS), nx1 = k < N ? nx[k + 1] : 0;
        for (int l = 0; l < nu[k] + nx[k]; l++) ux[k][l] += alpha * (dux[k][l] - ux[k][l]);
        for (int l = 0; l < nx1; l++) pi[k][l] += alpha * (dpi[k][l] - pi[k][l]);
        double *pl = lam[k], *pdl = dlam[k], *pt = t[k], *pdt = dt[k];
        for (int l = 0; l < nb[k]; l++) {
            pl[l] += alpha * pdl[l];
            pl[pnb + l] += alpha * pdl[pnb + l];
            pt[l] += alpha * pdt[l];
            pt[pnb + l] += alpha * pdt[pnb + l];
            mu += pl[l] * pt[l] + pl[pnb + l] * pt[pnb + l];
        }
        pl += 2 * pnb;
        pdl += 2 * pnb;
        pt += 2 * pnb;
        pdt += 2 * pnb;
        for (int l = 0; l < ns[k]; l++) {
            for (int s = 0; s < 4; s++) {
                pl[s * pns + l] += alpha * pdl[s * pns + l];
                pt[s * pns + l] += alpha * pdt[s * pns + l];
            }
            mu += pl[l] * pt[l] + pl[pns + l] * pt[pns + l] + pl[2 * pns + l] * pt[2 * pns + l] +
                  pl[3 * pns + l] * pt[3 * pns + l];
        }
    }
    *ptr_mu = mu * mu_scal;
}

/* sizes the restatement (and the HIP path) accept; 0 when supported */
int orc_soft_supported(int N, int *nx, int *nu, int *ng) {
    if (N < 1 || nu[N] != 0) return -10;
    for (int k = 0; k <= N; k++)
        if (ng[k] != 0) return -10;
    for (int k = 0; k < N; k++) {  /* b_k read with stride pnx (d_ip2_soft.c:172) must stay in BAbt_k */
        const int nux = nu[k] + nx[k], nx1 = nx[k + 1];
        const long idx = (long)(nux / BS) * BS * rup(nx1, BS) + nux % BS + BS * (long)(nx1 > 0 ? nx1 - 1 : 0);
        if (nx1 > 0 && idx >= (long)rup(nux + 1, BS) * rup(nx1, NCL)) return -10;
    }
    return 0;
}

int orc_d_ip2_mpc_soft_tv(int *kk, int k_max, double mu0, double mu_tol, double alpha_min, int warm_start,
                          double *stat, int N, int *nx, int *nu, int *nb, int **idxb, int *ng, int *ns,
                          double **pBAbt, double **pQ, double **Z, double **z, double **pDCt, double **d,
                          double **ux, int compute_mult, double **pi, double **lam, double **t,
                          double *double_work_memory) {
    if (orc_soft_supported(N, nx, nu, ng)) return -10;
    int nbs[N + 1];
    for (int k = 0; k <= N; k++) nbs[k] = nb[k] + ns[k];
    double *ptrs[14 * (N + 1)];
    sws_t w;
    sws_carve(N, nx, nu, nb, ng, ns, double_work_memory, &w, ptrs);
    /* b_k, q_k and the box diagonal backups (:168-216) */
    for (int k = 0; k < N; k++) {
        const int nux = nu[k] + nx[k], nx1 = nx[k + 1];
        const double *row = pBAbt[k] + (nux / BS) * BS * rup(nx1, BS) + nux % BS;
        for (int j = 0; j < nx1; j++) w.b[k][j] = row[BS * j];
    }
    for (int k = 0; k <= N; k++) {
        const int nux = nu[k] + nx[k], cnux = rup(nux, NCL);
        for (int l = 0; l < nux; l++) w.q[k][l] = *P4(pQ[k], cnux, nux, l);
        for (int l = 0; l < nbs[k]; l++) {
            const int i = idxb[k][l];
            w.bd[k][l] = *P4(pQ[k], cnux, i, i);
        }
    }
    double mu_scal = 0.0;
    for (int k = 0; k <= N; k++) mu_scal += 2 * nb[k] + 2 * ng[k] + 4 * ns[k];
    if (mu_scal == 0.0) {  /* (:273-284) */
        orc_d_back_ric_rec_sv_tv_res(N, nx, nu, nb, idxb, ng, 0, pBAbt, w.b, 0, pQ, w.q, NULL, NULL, NULL, NULL, w.dux,
                                     compute_mult, w.dpi, 1, w.Pb, w.memory, w.work);
        *kk = 0;
        return 0;
    }
    mu_scal = 1.0 / mu_scal;
    double sigma = 1.0;
    init_var_soft(N, nx, nu, nb, idxb, ns, ux, pi, d, t, lam, mu0, warm_start);
    for (int k = 0; k < N; k++)
        for (int l = 0; l < nx[k + 1]; l++) w.dpi[k][l] = 0.0;
    for (int l = 0; l < nx[0]; l++) w.dux[0][nu[0] + l] = ux[0][nu[0] + l];
    double mu = mu0, alpha = 1.0, mu_aff;
    *kk = 0;
    while (*kk < k_max && mu > mu_tol && alpha >= alpha_min) {
        update_hessian_soft(N, nb, ns, d, 0.0, t, w.t_inv, lam, w.lamt, w.dlam, w.Qx, w.qx, Z, z, w.Zl, w.zl);
        orc_d_back_ric_rec_sv_tv_res(N, nx, nu, nbs, idxb, ng, 0, pBAbt, w.b, 1, pQ, w.q, w.bd, pDCt, w.Qx, w.qx,
                                     w.dux, compute_mult, w.dpi, 1, w.Pb, w.memory, w.work);
        alpha = 1.0;
        compute_alpha_soft(N, nb, idxb, ns, &alpha, t, w.dt, lam, w.dlam, w.lamt, w.dux, d, w.Zl, w.zl);
        stat[5 * *kk] = sigma;
        stat[5 * *kk + 1] = alpha;
        alpha *= 0.995;
        compute_mu_soft(N, nb, ns, &mu_aff, mu_scal, alpha, lam, w.dlam, t, w.dt);
        stat[5 * *kk + 2] = mu_aff;
        sigma = mu_aff / mu;
        sigma = sigma * sigma * sigma;
        update_gradient_soft(N, nb, ns, sigma * mu, w.dt, w.dlam, w.t_inv, w.lamt, w.qx, w.Zl, w.zl);
        orc_d_back_ric_rec_trs_tv_res(N, nx, nu, nbs, idxb, ng, pBAbt, w.b, w.q, pDCt, w.qx, w.dux, compute_mult,
                                      w.dpi, 0, w.Pb, w.memory, w.work);
        alpha = 1.0;
        compute_alpha_soft(N, nb, idxb, ns, &alpha, t, w.dt, lam, w.dlam, w.lamt, w.dux, d, w.Zl, w.zl);
        stat[5 * *kk] = sigma;
        stat[5 * *kk + 3] = alpha;
        alpha *= 0.995;
        update_var_soft(N, nx, nu, nb, ns, &mu, mu_scal, alpha, ux, w.dux, t, w.dt, lam, w.dlam, pi, w.dpi);
        stat[5 * *kk + 4] = mu;
        (*kk)++;
    }
    /* restore the Hessian diagonal and gradient row (:512-526) */
    for (int k = 0; k <= N; k++) {
        const int nux = nu[k] + nx[k], cnux = rup(nux, NCL);
        for (int l = 0; l < nbs[k]; l++) {
            const int i = idxb[k][l];
            *P4(pQ[k], cnux, i, i) = w.bd[k][l];
        }
        for (int l = 0; l < nux; l++) *P4(pQ[k], cnux, nux, l) = w.q[k][l];
    }
    if (mu <= mu_tol) return 0;
    if (*kk >= k_max) return 1;
    if (alpha < alpha_min) return 2;
    return -1;
}

/* d_res_mpc_soft_tv (mpc_solvers/d_res_ip_soft.c:38-268): residuals r_q, r_b, r_d, r_z and mu of a soft-constraint
 * iterate, restated with the reference's layout and quirks:
 *   - soft constraint i of stage k acts on ux[idxb[k][nu_k + i]] (the reference indexes idxb past the nu_k
 *     inputs, not past the nb_k hard boxes: :107-108, :134);
 *   - its multipliers enter r_q as lam_0 - lam_1 on stages k < N (:134) but as -lam_2 + lam_3 on stage N (:220);
 *   - on stage N r_q starts from pi_{N-1} - q on the state rows only (:199-200; the input rows, empty when
 *     nu_N = 0, keep what the caller's vector holds) and its symv covers the leading nx_N x nx_N block (:204-207);
 *   - mu = sum(lam t) over the hard, general and all four soft blocks / (2 (nb + ng + ns)) (:51-84, :231);
 *   - r_q, r_b and r_d (hard, general and the first two soft blocks) change sign at the end (:237-264), r_z
 *     does not.
 * pi_{-1} (stage 0 with nx_0 > 0) is read as zero (the reference reads before hpi[0]). */
void orc_d_res_mpc_soft_tv(int N, int *nx, int *nu, int *nb, int **idxb, int *ng, int *ns, double **hpBAbt,
                           double **hpQ, double **hq, double **hZ, double **hz, double **hux, double **hpDCt,
                           double **hd, double **hpi, double **hlam, double **ht, double **hrq, double **hrb,
                           double **hrd, double **hrz, double *mu) {
    double m = 0.0;
    long ntot = 0;
    for (int k = 0; k <= N; k++) {
        const int nu0 = nu[k], nx0 = nx[k], nux = nu0 + nx0, cnux = rup(nux, NCL);
        const int pnb = rup(nb[k], BS), png = rup(ng[k], BS), pns = rup(ns[k], BS), cng = rup(ng[k], NCL);
        const int ob = 0, og = 2 * pnb, os = 2 * pnb + 2 * png;
        const double *lam = hlam[k], *t = ht[k], *ux = hux[k], *d = hd[k];
        double *rq = hrq[k], *rd = hrd[k];
        ntot += nb[k] + ng[k] + ns[k];
        for (int j = 0; j < nb[k]; j++) m += lam[ob + j] * t[ob + j] + lam[ob + pnb + j] * t[ob + pnb + j];
        for (int j = 0; j < ng[k]; j++) m += lam[og + j] * t[og + j] + lam[og + png + j] * t[og + png + j];
        for (int j = 0; j < ns[k]; j++)
            for (int b = 0; b < 4; b++) m += lam[os + b * pns + j] * t[os + b * pns + j];
        /* r_d */
        for (int j = 0; j < nb[k]; j++) {
            const double x = ux[idxb[k][j]];
            rd[j] = x - d[j] - t[j];
            rd[pnb + j] = -x + d[pnb + j] - t[pnb + j];
        }
        for (int j = 0; j < ng[k]; j++) {
            double g = 0.0;
            for (int i = 0; i < nux; i++) g += *P4(hpDCt[k], cng, i, j) * ux[i];
            rd[og + j] = g - d[og + j] - t[og + j];
            rd[og + png + j] = -g + d[og + png + j] - t[og + png + j];
        }
        for (int j = 0; j < ns[k]; j++) {
            const double x = ux[idxb[k][nu0 + j]];
            rd[os + j] = t[os + 2 * pns + j] + x - d[os + j] - t[os + j];
            rd[os + pns + j] = t[os + 3 * pns + j] - x + d[os + pns + j] - t[os + pns + j];
        }
        /* r_q */
        const int nsym = k < N ? nux : nx0;
        if (k < N)
            for (int i = 0; i < nu0; i++) rq[i] = -hq[k][i];
        for (int i = 0; i < nx0; i++) rq[nu0 + i] = -hq[k][nu0 + i] + (k > 0 ? hpi[k - 1][i] : 0.0);
        if (k == N)
            for (int j = 0; j < nb[k]; j++) rq[idxb[k][j]] += lam[j] - lam[pnb + j];
        for (int i = 0; i < nsym; i++) {
            double s = 0.0;
            for (int j = 0; j < nsym; j++) s += (i >= j ? *P4(hpQ[k], cnux, i, j) : *P4(hpQ[k], cnux, j, i)) * ux[j];
            rq[i] -= s;
        }
        if (k < N)
            for (int j = 0; j < nb[k]; j++) rq[idxb[k][j]] += lam[j] - lam[pnb + j];
        for (int i = 0; i < nux; i++) {
            double s = 0.0;
            for (int j = 0; j < ng[k]; j++) s += *P4(hpDCt[k], cng, i, j) * (lam[og + j] - lam[og + png + j]);
            rq[i] += s;
        }
        for (int j = 0; j < ns[k]; j++)
            rq[idxb[k][nu0 + j]] += k < N ? lam[os + j] - lam[os + pns + j] : -lam[os + 2 * pns + j] + lam[os + 3 * pns + j];
        if (k < N) {
            const int nx1 = nx[k + 1], nu1 = nu[k + 1], cnx1 = rup(nx1, NCL);
            for (int j = 0; j < nx1; j++) {
                double s = 0.0;
                for (int i = 0; i < nux; i++) s += *P4(hpBAbt[k], cnx1, i, j) * ux[i];
                hrb[k][j] = hux[k + 1][nu1 + j] - *P4(hpBAbt[k], cnx1, nux, j) - s;
            }
            for (int i = 0; i < nux; i++) {
                double s = 0.0;
                for (int j = 0; j < nx1; j++) s += *P4(hpBAbt[k], cnx1, i, j) * hpi[k][j];
                rq[i] -= s;
            }
        }
        /* r_z */
        for (int j = 0; j < ns[k]; j++) {
            hrz[k][j] = hz[k][j] + hZ[k][j] * t[os + 2 * pns + j] - lam[os + j] - lam[os + 2 * pns + j];
            hrz[k][pns + j] = hz[k][pns + j] + hZ[k][pns + j] * t[os + 3 * pns + j] - lam[os + pns + j] - lam[os + 3 * pns + j];
        }
    }
    *mu = ntot != 0 ? m / (2.0 * ntot) : 0.0;
    for (int k = 0; k <= N; k++) {
        const int pnb = rup(nb[k], BS), png = rup(ng[k], BS), pns = rup(ns[k], BS), os = 2 * pnb + 2 * png;
        for (int i = 0; i < nu[k] + nx[k]; i++) hrq[k][i] = -hrq[k][i];
        if (k < N)
            for (int j = 0; j < nx[k + 1]; j++) hrb[k][j] = -hrb[k][j];
        for (int j = 0; j < nb[k]; j++) {
            hrd[k][j] = -hrd[k][j];
            hrd[k][pnb + j] = -hrd[k][pnb + j];
        }
        for (int j = 0; j < ng[k]; j++) {
            hrd[k][2 * pnb + j] = -hrd[k][2 * pnb + j];
            hrd[k][2 * pnb + png + j] = -hrd[k][2 * pnb + png + j];
        }
        for (int j = 0; j < ns[k]; j++) {
            hrd[k][os + j] = -hrd[k][os + j];
            hrd[k][os + pns + j] = -hrd[k][os + pns + j];
        }
    }
}
