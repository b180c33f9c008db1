/*
 * hpmpc_oracle.h -- TEST INFRASTRUCTURE ONLY.
 *
 * Clean-room CPU restatement of the HPMPC hot path (backward Riccati recursion + residual-based
 * Mehrotra IPM on lib4 panel-major data).  It is the parity checker for the MI355X build: only
 * tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load it.  The product
 * (libhpmpc_mi355x.so) never links, calls or falls back to it.
 *
 * Every entry point has the SAME argument list and meaning as the reference routine it restates
 * (file:line relative to the reference checkout), prefixed with orc_ so that it can live in one
 * process next to the product's reference-named symbols.  Workspace/memory layouts are private to
 * the oracle and sized by the oracle's own *_size_bytes functions.
 */
#ifndef HPMPC_ORACLE_H_
#define HPMPC_ORACLE_H_

#ifdef __cplusplus
extern "C" {
#endif

/* lqcp_solvers/d_back_ric_rec.c:43 */
int orc_d_back_ric_rec_sv_tv_work_space_size_bytes(int N, int *nx, int *nu, int *nb, int *ng);
/* lqcp_solvers/d_back_ric_rec.c:79 */
int orc_d_back_ric_rec_sv_tv_memory_space_size_bytes(int N, int *nx, int *nu, int *nb, int *ng);
/* lqcp_solvers/d_back_ric_rec.c:112 */
void orc_d_back_ric_rec_sv_tv_res(int N, int *nx, int *nu, int *nb, int **idxb, int *ng, int update_b,
    double **hpBAbt, double **b, int update_q, double **hpRSQrq, double **q, double **bd, double **hpDCt,
    double **Qx, double **qx, double **hux, int compute_pi, double **hpi, int compute_Pb, double **hPb,
    double *memory, double *work);
/* lqcp_solvers/d_back_ric_rec.c:403 */
void orc_d_back_ric_rec_trf_tv_res(int N, int *nx, int *nu, int *nb, int **idxb, int *ng, double **hpBAbt,
    double **hpRSQrq, double **hpDCt, double **Qx, double **bd, double *memory, double *work);
/* lqcp_solvers/d_back_ric_rec.c:564 */
void orc_d_back_ric_rec_trs_tv_res(int N, int *nx, int *nu, int *nb, int **idxb, int *ng, double **hpBAbt,
    double **hb, double **hq, double **hpDCt, double **qx, double **hux, int compute_pi, double **hpi,
    int compute_Pb, double **hPb, double *memory, double *work);

/* mpc_solvers/d_ip2_res_hard.c:57 */
int orc_d_ip2_res_mpc_hard_tv_work_space_size_bytes(int N, int *nx, int *nu, int *nb, int *ng);
/* mpc_solvers/d_ip2_res_hard.c:116 */
int orc_d_ip2_res_mpc_hard_tv(int *kk, int k_max, double mu0, double mu_tol, double alpha_min, int warm_start,
    double *stat, int N, int *nx, int *nu_N, int *nb, int **idxb, int *ng, double **pBAbt, double **pQ,
    double **pDCt, double **d, double **ux, int compute_mult, double **pi, double **lam, double **t,
    double *double_work_memory);
/* mpc_solvers/d_ip2_res_hard.c:1348 */
int orc_d_ip2_res_mpc_hard_tv_single_newton_step(int *kk, int k_max, double mu0, double mu_tol, double alpha_min,
    int warm_start, double *stat, int N, int *nx, int *nu_N, int *nb, int **idxb, int *ng, double **pBAbt,
    double **pQ, double **pDCt, double **d, double **ux, int compute_mult, double **pi, double **lam, double **t,
    double *double_work_memory, double **ux0, double **pi0, double **lam0, double **t0);
/* mpc_solvers/d_ip2_res_hard.c:1922 */
void orc_d_kkt_solve_new_rhs_res_mpc_hard_tv(int N, int *nx, int *nu_N, int *nb, int **idxb, int *ng,
    double **pBAbt, double **b, double **pQ, double **q, double **pDCt, double **d, double **ux, int compute_mult,
    double **pi, double **lam, double **t, double *double_work_memory);
/* mpc_solvers/c99/d_res_ip_res_hard.c:39 */
void orc_d_res_res_mpc_hard_tv(int N, int *nx, int *nu, int *nb, int **idxb, int *ng, double **hpBAbt, double **hb,
    double **hpQ, double **hq, double **hux, double **hpDCt, double **hd, double **hpi, double **hlam, double **ht,
    double *work, double **hrq, double **hrb, double **hrd, double **hrm, double *mu);

/* alternate IPM (mpc_solvers/d_ip2_hard.c) and its residuals (mpc_solvers/d_res_ip_hard.c) */
int orc_d_ip2_mpc_hard_tv_work_space_size_bytes(int N, int *nx, int *nu, int *nb, int *ng);
int orc_d_ip2_mpc_hard_tv(int *kk, int k_max, double mu0, double mu_tol, double alpha_min, int warm_start,
                          double *stat, int N, int *nx, int *nu_N, int *nb, int **idxb, int *ng, double **pBAbt,
                          double **pQ, double **pDCt, double **d, double **ux, int compute_mult, double **pi,
                          double **lam, double **t, double *double_work_memory);
void orc_d_kkt_solve_new_rhs_mpc_hard_tv(int N, int *nx, int *nu_N, int *nb, int **idxb, int *ng, double **pBAbt,
                                         double **r_A, double **pQ, double **r_H, double **pDCt, double **r_C,
                                         double **ux, int compute_mult, double **pi, double **lam, double **t,
                                         double *double_work_memory);
void orc_d_res_mpc_hard_tv(int N, int *nx, int *nu, int *nb, int **idxb, int *ng, double **hpBAbt, double **hb,
                           double **hpQ, double **hq, double **hux, double **hpDCt, double **hd, double **hpi,
                           double **hlam, double **ht, double **hrq, double **hrb, double **hrd, double *mu);

/* partial condensing (lqcp_solvers/d_part_cond.c) */
void orc_d_cond_BAbt(int N, int *nx, int *nu, double **hpBAbt, double *work, double **hpGamma, double *pBAbt2);
void orc_d_cond_RSQrq(int N, int *nx, int *nu, double **hpBAbt, double **hpRSQrq, double **hpGamma, double *work,
                      double *pRSQrq2);
void orc_d_cond_DCtd(int N, int *nx, int *nu, int *nb, int **hidxb, double **hd, double **hpGamma, double *pDCt2,
                     double *d2, int *idxb2);
void orc_d_part_cond_compute_problem_size(int N, int *nx, int *nu, int *nb, int **hidxb, int *ng, int N2, int *nx2,
                                          int *nu2, int *nb2, int *ng2);
int orc_d_part_cond_work_space_size_bytes(int N, int *nx, int *nu, int *nb, int **hidxb, int *ng, int N2, int *nx2,
                                          int *nu2, int *nb2, int *ng2);
int orc_d_part_cond_memory_space_size_bytes(int N, int *nx, int *nu, int *nb, int **hidxb, int *ng, int N2,
                                            int *nx2, int *nu2, int *nb2, int *ng2);
void orc_d_part_cond(int N, int *nx, int *nu, int *nb, int **hidxb, int *ng, double **hpBAbt, double **hpRSQrq,
                     double **hpDCt, double **hd, int N2, int *nx2, int *nu2, int *nb2, int **hidxb2, int *ng2,
                     double **hpBAbt2, double **hpRSQrq2, double **hpDCt2, double **hd2, void *memory, void *work);
int orc_d_part_expand_work_space_size_bytes(int N, int *nx, int *nu, int *nb, int *ng);
void orc_d_part_expand_solution(int N, int *nx, int *nu, int *nb, int **hidxb, int *ng, double **hpBAbt, double **hb,
                                double **hpRSQrq, double **hrq, double **hpDCt, double **hux, double **hpi,
                                double **hlam, double **ht, int N2, int *nx2, int *nu2, int *nb2, int **hidxb2,
                                int *ng2, double **hux2, double **hpi2, double **hlam2, double **ht2, void *work);

/* soft-constraint IPM (hpmpc_oracle_soft.c; mpc_solvers/d_ip2_soft.c:42-547) */
int orc_soft_supported(int N, int *nx, int *nu, int *ng);
void orc_d_res_mpc_soft_tv(int N, int *nx, int *nu, int *nb, int **idxb, int *ng, int *ns, double **hpBAbt,
                           double **hpQ, double **hq, double **hZ, double **hz, double **hux, double **hpDCt,
                           double **hd, double **hpi, double **hlam, double **ht, double **hrq, double **hrb,
                           double **hrd, double **hrz, double *mu);
int orc_d_ip2_mpc_soft_tv_work_space_size_bytes(int N, int *nx, int *nu, int *nb, int *ng, int *ns);
int orc_d_ip2_mpc_soft_tv(int *kk, int k_max, double mu0, double mu_tol, double alpha_min, int warm_start,
                          double *stat, int N, int *nx, int *nu, int *nb, int **idxb, int *ng, int *ns,
                          double **pBAbt, double **pQ, double **Z, double **z, double **pDCt, double **d,
                          double **ux, int compute_mult, double **pi, double **lam, double **t,
                          double *double_work_memory);

#ifdef __cplusplus
}
#endif
#endif
