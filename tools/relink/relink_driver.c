/*
 * relink_driver.c -- link-level proof of the drop-in.
 *
 * The reference's own drivers test_problems/test_d_ip_hard.c:937-1042 and test_d_ric_mpc.c:536-590 include the
 * BLASFEO headers (blasfeo_target.h, blasfeo_common.h, ...), which this image does not have, so they cannot be
 * compiled here.  This driver makes the same call sequence through the reference's OWN public headers
 * (include/mpc_solvers.h, lqcp_solvers.h, aux_d.h, taken from the reference tree at build time, not copied) and
 * the reference's own auxiliary objects (d_zeros_align, d_cvt_mat2pmat, ...).  tools/relink/Makefile links it
 * against the reference objects MINUS the replaced solver files, plus -lhpmpc_mi355x; tests/test_relink.py
 * checks with nm that every replaced entry point resolves to the shim.  The same driver linked against the whole
 * reference (relink_driver_ref, run here) prints the reference's answers (tests/golden/drivers/relink_driver.txt);
 * the relinked binary travels to the GPU box (oracle/_ref/drivers/relink_driver), where
 * tests/test_gpu_ref_driver.py runs it and compares every printed number.
 *
 * (test_problems/test_d_ip_hard.c itself compiles only with include/target.h, which the reference's build system
 * generates (Makefile:472-518); this tree does not stand in for generated reference files, DESIGN.md.)
 */
#include <stdio.h>
#include <stdlib.h>

#include "aux_d.h"
#include "lqcp_solvers.h"
#include "mpc_solvers.h"

/* every printed number at full precision: "<tag> <k> v0 v1 ..." */
static void dump(const char *tag, int k, const double *v, int n) {
    printf("%s %d", tag, k);
    for (int i = 0; i < n; i++) printf(" %.17g", v[i]);
    printf("\n");
}

static void dump_sol(const char *tag, int N, const int *nx, const int *nu, const int *nb, double **ux, double **pi,
                     double **lam, double **t) {
    for (int k = 0; k <= N; k++) {
        const int pnb = (nb[k] + 3) / 4 * 4;
        char nm[64];
        snprintf(nm, sizeof nm, "%s.ux", tag);
        dump(nm, k, ux[k], nu[k] + nx[k]);
        if (k < N) {
            snprintf(nm, sizeof nm, "%s.pi", tag);
            dump(nm, k, pi[k], nx[k + 1]);
        }
        if (lam && nb[k]) {
            snprintf(nm, sizeof nm, "%s.lam", tag);
            dump(nm, k, lam[k], 2 * pnb);
            snprintf(nm, sizeof nm, "%s.t", tag);
            dump(nm, k, t[k], 2 * pnb);
        }
    }
}

int main(void) {
    enum { N = 10, NX = 8, NU = 3, BS = 4 };
    int nx[N + 1], nu[N + 1], nb[N + 1], ng[N + 1];
    int *idxb[N + 1];
    double *pBAbt[N], *pRSQ[N + 1], *pDCt[N + 1], *d[N + 1], *ux[N + 1], *pi[N], *lam[N + 1], *t[N + 1];
    double *b[N], *q[N + 1], *rq[N + 1], *rb[N], *rd[N + 1], *rm[N + 1], *Pb[N];
    for (int k = 0; k <= N; k++) {
        nx[k] = k == 0 ? 0 : NX;
        nu[k] = k < N ? NU : 0;
        nb[k] = nu[k] + nx[k] / 2;
        ng[k] = 0;
    }
    /* mass-spring-like stage data in column-major, converted to the lib4 panel-major layout by the
     * reference's own d_cvt_mat2pmat */
    for (int k = 0; k <= N; k++) {
        const int nux = nu[k] + nx[k], nx1 = k < N ? nx[k + 1] : 0;
        const int pnz = (nux + 1 + BS - 1) / BS * BS, cnux = (nux + 1) / 2 * 2, cnx1 = (nx1 + 1) / 2 * 2;
        double *M;
        d_zeros(&M, nux + 1, nux > 0 ? nux : 1);
        for (int i = 0; i < nux; i++) M[i + i * (nux + 1)] = 2.0;
        for (int j = 0; j < nux; j++) M[nux + j * (nux + 1)] = 0.1;
        d_zeros_align(&pRSQ[k], pnz, cnux > 0 ? cnux : 2);
        d_cvt_mat2pmat(nux + 1, nux, M, nux + 1, 0, pRSQ[k], cnux);
        d_free(M);
        if (k < N) {
            double *B;
            d_zeros(&B, nux + 1, nx1);
            for (int i = 0; i < nx1; i++) B[(nu[k] + i % (nx[k] > 0 ? nx[k] : 1)) + i * (nux + 1)] = 1.0;
            for (int i = 0; i < nx1; i++) B[i % (nu[k] > 0 ? nu[k] : 1) + i * (nux + 1)] += 0.1;
            for (int i = 0; i < nx1; i++) B[nux + i * (nux + 1)] = 0.05;
            d_zeros_align(&pBAbt[k], pnz, cnx1);
            d_cvt_mat2pmat(nux + 1, nx1, B, nux + 1, 0, pBAbt[k], cnx1);
            d_free(B);
            d_zeros_align(&pi[k], nx1 + 4, 1);
            d_zeros_align(&b[k], nx1 + 4, 1);
            d_zeros_align(&rb[k], nx1 + 4, 1);
            d_zeros_align(&Pb[k], nx1 + 4, 1);
        }
        idxb[k] = malloc(sizeof(int) * (nb[k] > 0 ? nb[k] : 1));
        for (int l = 0; l < nb[k]; l++) idxb[k][l] = l;
        const int pnb = (nb[k] + BS - 1) / BS * BS;
        d_zeros_align(&d[k], 2 * pnb + 4, 1);
        for (int l = 0; l < nb[k]; l++) {
            d[k][l] = -1.0;
            d[k][pnb + l] = 1.0;
        }
        d_zeros_align(&lam[k], 2 * pnb + 4, 1);
        d_zeros_align(&t[k], 2 * pnb + 4, 1);
        d_zeros_align(&rd[k], 2 * pnb + 4, 1);
        d_zeros_align(&rm[k], 2 * pnb + 4, 1);
        d_zeros_align(&ux[k], nux + 4, 1);
        d_zeros_align(&q[k], nux + 4, 1);
        d_zeros_align(&rq[k], nux + 4, 1);
        pDCt[k] = NULL;
    }
    int kk = 0;
    double stat[5 * 50], mu = 0.0;
    double *work, *mem, *ws;
    /* IPM (test_d_ip_hard.c:688-939), its KKT re-solve (:1040) and residuals */
    d_zeros_align(&work, d_ip2_res_mpc_hard_tv_work_space_size_bytes(N, nx, nu, nb, ng) / sizeof(double) + 8, 1);
    int status = d_ip2_res_mpc_hard_tv(&kk, 50, 2.0, 1e-12, 1e-8, 0, stat, N, nx, nu, nb, idxb, ng, pBAbt, pRSQ, pDCt,
                                       d, ux, 1, pi, lam, t, work);
    printf("ipm status %d kk %d\n", status, kk);
    dump("ipm.stat", 0, stat, 5 * kk);
    dump_sol("ipm", N, nx, nu, nb, ux, pi, lam, t);
    /* new right-hand sides for the re-solves: b, q */
    for (int k = 0; k <= N; k++) {
        for (int i = 0; i < nu[k] + nx[k]; i++) q[k][i] = 0.01 * (i + 1) - 0.02 * k;
        if (k < N)
            for (int i = 0; i < nx[k + 1]; i++) b[k][i] = 0.03 * ((i + k) % 3);
    }
    d_kkt_solve_new_rhs_res_mpc_hard_tv(N, nx, nu, nb, idxb, ng, pBAbt, b, pRSQ, q, pDCt, d, ux, 1, pi, lam, t, work);
    dump_sol("kkt", N, nx, nu, nb, ux, pi, lam, t);
    d_res_res_mpc_hard_tv(N, nx, nu, nb, idxb, ng, pBAbt, b, pRSQ, q, ux, pDCt, d, pi, lam, t, work, rq, rb, rd, rm, &mu);
    for (int k = 0; k <= N; k++) {
        dump("res.rq", k, rq[k], nu[k] + nx[k]);
        if (k < N) dump("res.rb", k, rb[k], nx[k + 1]);
    }
    dump("res.mu", 0, &mu, 1);
    int st2 = d_ip2_mpc_hard_tv(&kk, 50, 2.0, 1e-8, 1e-8, 0, stat, N, nx, nu, nb, idxb, ng, pBAbt, pRSQ, pDCt, d, ux,
                                1, pi, lam, t, work);
    printf("ipm2 status %d kk %d\n", st2, kk);
    status |= st2;
    dump_sol("ipm2", N, nx, nu, nb, ux, pi, NULL, NULL);
    d_kkt_solve_new_rhs_mpc_hard_tv(N, nx, nu, nb, idxb, ng, pBAbt, b, pRSQ, q, pDCt, d, ux, 1, pi, lam, t, work);
    dump_sol("kkt2", N, nx, nu, nb, ux, pi, NULL, NULL);
    d_res_mpc_hard_tv(N, nx, nu, nb, idxb, ng, pBAbt, b, pRSQ, q, ux, pDCt, d, pi, lam, t, rq, rb, rd, &mu);
    dump("res2.mu", 0, &mu, 1);
    /* Riccati factorisation + solve (test_d_ric_mpc.c:536-560) and trf / trs */
    d_zeros_align(&mem, d_back_ric_rec_sv_tv_memory_space_size_bytes(N, nx, nu, nb, ng) / sizeof(double) + 8, 1);
    d_zeros_align(&ws, d_back_ric_rec_sv_tv_work_space_size_bytes(N, nx, nu, nb, ng) / sizeof(double) + 8, 1);
    d_back_ric_rec_sv_tv_res(N, nx, nu, nb, idxb, ng, 0, pBAbt, b, 0, pRSQ, q, d, pDCt, d, d, ux, 1, pi, 1, Pb, mem, ws);
    dump_sol("sv", N, nx, nu, nb, ux, pi, NULL, NULL);
    for (int k = 0; k < N; k++) dump("sv.Pb", k, Pb[k], nx[k + 1]);
    d_back_ric_rec_trf_tv_res(N, nx, nu, nb, idxb, ng, pBAbt, pRSQ, pDCt, d, d, mem, ws);
    d_back_ric_rec_trs_tv_res(N, nx, nu, nb, idxb, ng, pBAbt, b, q, pDCt, d, ux, 1, pi, 1, Pb, mem, ws);
    dump_sol("trs", N, nx, nu, nb, ux, pi, NULL, NULL);
    /* partial condensing (test_d_part_cond.c) */
    int N2 = 2, nx2[3], nu2[3], nb2[3], ng2[3];
    d_part_cond_compute_problem_size(N, nx, nu, nb, idxb, ng, N2, nx2, nu2, nb2, ng2);
    printf("status %d kk %d mu %e size %d %d\n", status, kk, mu,
           d_part_cond_work_space_size_bytes(N, nx, nu, nb, idxb, ng, N2, nx2, nu2, nb2, ng2),
           d_part_expand_work_space_size_bytes(N, nx, nu, nb, ng));
    return 0;
}
