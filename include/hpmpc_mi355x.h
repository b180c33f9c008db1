/*
 * hpmpc_mi355x.h -- C ABI of libhpmpc_mi355x.so, the MI355X (gfx950) drop-in for HPMPC's
 * Riccati / interior-point hot path.
 *
 * Part 1 re-exports the reference's own low-level entry points with byte-identical prototypes, so
 * that the reference drivers (test_problems/test_d_ip_hard.c, test_d_ric_mpc.c) and the high-level
 * wrappers (interfaces/c/fortran_order_interface.c) relink against this library unchanged.  Each
 * prototype cites the reference declaration it replaces (paths relative to the reference checkout).
 * All data are the reference's lib4 panel-major buffers (bs = 4, ncl = 2) on the HOST; every call
 * runs on the GPU (no CPU fallback).  Workspace / memory contents are private to this library and
 * are sized by this library's *_size_bytes functions.
 *
 * Part 2 is the additive batched API: many independent QPs that share stage sizes, with all data
 * already resident in device memory (HBM).
 *
 * GPU paths (selected per call from the stage sizes):
 *   tile path -- nu[k] + nx[k] <= 16, round_up(nu[k],4) + nx[k] <= 16 and round_up(nb[k],4) + round_up(ng[k],4)
 *     <= 16 for every stage: one wavefront per problem, the stage in MFMA registers;
 *   wide path -- every other problem with nu[k] + nx[k] + 1 <= 128, nx[k] <= 64 and the stage tiles within
 *     64 KiB of LDS (any nb <= nu+nx, any ng): one 256-thread workgroup per problem, stage tiles in LDS; the
 *     IPMs run whole on the device in one launch.
 *   Part 1 serves both; the batched Part 2 takes tile-path plans (plus the partial-condensing pipeline).
 *   Beyond these limits, and for duplicate box indices, calls report HPMPC_MI355X_EUNSUPPORTED.
 * Error reporting: the reference's int entry points keep their codes 0/1/2/-1; this library adds
 *   HPMPC_MI355X_EUNSUPPORTED (-10), HPMPC_MI355X_EHIP (-11) and HPMPC_MI355X_EMW (-20: the one-problem latency
 *   kernel abandoned a solve after an expired hand-over wait between its waves -- a bug, never a data condition;
 *   see hpmpc_mi355x_ipm_solo).  void entry points set the thread-local code returned by
 *   hpmpc_mi355x_last_error() and print one line to stderr; int entry points set it too.
 */
#ifndef HPMPC_MI355X_H_
#define HPMPC_MI355X_H_

#ifdef __cplusplus
extern "C" {
#endif

#define HPMPC_MI355X_EUNSUPPORTED (-10)
#define HPMPC_MI355X_EHIP (-11)
#define HPMPC_MI355X_EMW (-20)
/* Problem queue control block (hpmpc_mi355x_ipm_queue's qctl): ints for n_slots slots, up to
 * HPMPC_MI355X_QUEUE_LANES_MAX lanes. */
#define HPMPC_MI355X_QUEUE_LANES_MAX 4
#define HPMPC_MI355X_QUEUE_CTL_INTS(n_slots) (6 * HPMPC_MI355X_QUEUE_LANES_MAX + 2 + 3 * (n_slots))

/* ================================ Part 1: reference entry points ================================ */

/* include/lqcp_solvers.h:37 (lqcp_solvers/d_back_ric_rec.c:43) */
int d_back_ric_rec_sv_tv_work_space_size_bytes(int N, int *nx, int *nu, int *nb, int *ng);
/* include/lqcp_solvers.h:39 (d_back_ric_rec.c:79) */
int d_back_ric_rec_sv_tv_memory_space_size_bytes(int N, int *nx, int *nu, int *nb, int *ng);
/* include/lqcp_solvers.h:41 (d_back_ric_rec.c:112) -- factorise + solve */
void d_back_ric_rec_sv_tv_res(int N, int *nx, int *nu, int *nb, int **idxb, int *ng, int update_b, double **hpBAbt,
                              double **b, int update_q, double **hpQ, double **q, double **bd, double **hpDCt,
                              double **Qx, double **qx, double **hux, int compute_pi, double **hpi, int compute_Pb,
                              double **hPb, double *memory, double *work);
/* include/lqcp_solvers.h:43 (d_back_ric_rec.c:403) -- factorise */
void d_back_ric_rec_trf_tv_res(int N, int *nx, int *nu, int *nb, int **idxb, int *ng, double **hpBAbt, double **hpQ,
                               double **hpDCt, double **Qx, double **bd, double *memory, double *work);
/* include/lqcp_solvers.h:45 (d_back_ric_rec.c:564) -- solve with the factor left in memory */
void d_back_ric_rec_trs_tv_res(int N, int *nx, int *nu, int *nb, int **idxb, int *ng, double **hpBAbt, double **hb,
                               double **hq, double **hpDCt, double **qx, double **hux, int compute_pi, double **hpi,
                               int compute_Pb, double **hPb, double *memory, double *work);

/* include/mpc_solvers.h:41 (mpc_solvers/d_ip2_res_hard.c:57) */
int d_ip2_res_mpc_hard_tv_work_space_size_bytes(int N, int *nx, int *nu, int *nb, int *ng);
/* include/mpc_solvers.h:42 (d_ip2_res_hard.c:116) */
int d_ip2_res_mpc_hard_tv(int *kk, int k_max, double mu0, double mu_tol, double alpha_min, int warm_start,
                          double *stat, int N, int *nx, int *nu_N, int *nb, int **idxb, int *ng, double **pBAbt,
                          double **pQ, double **pDCt, double **d, double **ux, int compute_mult, double **pi,
                          double **lam, double **t, double *double_work_memory);
/* include/mpc_solvers.h:44 (d_ip2_res_hard.c:1348) -- k_max Newton steps from (ux0, pi0, lam0, t0), fixed
 * centering target mu0, no exit test on mu; lam0/t0 as [lower(nb) | upper(nb)] */
int d_ip2_res_mpc_hard_tv_single_newton_step(int *kk, int k_max, double mu0, double mu_tol, double alpha_min,
                                             int warm_start, double *stat, int N, int *nx, int *nu_N, int *nb,
                                             int **idxb, int *ng, double **pBAbt, double **pQ, double **pDCt,
                                             double **d, double **ux, int compute_mult, double **pi, double **lam,
                                             double **t, double *double_work_memory, double **ux0, double **pi0,
                                             double **lam0, double **t0);
/* include/mpc_solvers.h:46 (d_ip2_res_hard.c:1922) -- re-solve with the persisted factor/iterate */
void d_kkt_solve_new_rhs_res_mpc_hard_tv(int N, int *nx, int *nu_N, int *nb, int **idxb, int *ng, double **pBAbt,
                                         double **b, double **pQ, double **q, double **pDCt, double **d,
                                         double **ux, int compute_mult, double **pi, double **lam, double **t,
                                         double *double_work_memory);
/* include/mpc_solvers.h:47 (mpc_solvers/c99/d_res_ip_res_hard.c:39) */
void d_res_res_mpc_hard_tv(int N, int *nx, int *nu, int *nb, int **idxb, int *ng, double **hpBAbt, double **hb,
                           double **hpQ, double **hq, double **hux, double **hpDCt, double **hd, double **hpi,
                           double **hlam, double **ht, double *work, double **hrq, double **hrb, double **hrd,
                           double **hrm, double *mu);

/* The alternate IPM of mpc_solvers/d_ip2_hard.c: the phase-1 Mehrotra loop alone, run to mu_tol. */
/* include/mpc_solvers.h:33 (mpc_solvers/d_ip2_hard.c:31) */
int d_ip2_mpc_hard_tv_work_space_size_bytes(int N, int *nx, int *nu, int *nb, int *ng);
/* include/mpc_solvers.h:34 (d_ip2_hard.c:88) */
int d_ip2_mpc_hard_tv(int *kk, int k_max, double mu0, double mu_tol, double alpha_min, int warm_start, double *stat,
                      int N, int *nx, int *nu, int *nb, int **idxb, int *ng, double **pBAbt, double **pQ,
                      double **pDCt, double **d, double **ux, int compute_mult, double **pi, double **lam, double **t,
                      double *double_work_memory);
/* include/mpc_solvers.h:35 (d_ip2_hard.c:626) -- re-solve on the factor and lam/t that d_ip2_mpc_hard_tv left in
 * the workspace, for new r_A (b), r_H (q) and r_C (bounds) */
void d_kkt_solve_new_rhs_mpc_hard_tv(int N, int *nx, int *nu_N, int *nb, int **idxb, int *ng, double **pBAbt,
                                     double **r_A, double **pQ, double **r_H, double **pDCt, double **r_C,
                                     double **ux, int compute_mult, double **pi, double **lam, double **t,
                                     double *double_work_memory);
/* Soft-constraint IPM (phase-1 Mehrotra loop with slack variables for the ns soft boxes listed after the nb
 * hard ones in idxb; d = [lb | ub | ls | us], lam / t = [lo | up | 4 soft blocks], Z / z slack penalties).
 * include/mpc_solvers.h:69 (mpc_solvers/d_ip2_soft.c:42) */
int d_ip2_mpc_soft_tv_work_space_size_bytes(int N, int *nx, int *nu, int *nb, int *ng, int *ns);
/* include/mpc_solvers.h:70 (d_ip2_soft.c:83).  HPMPC_MI355X_EUNSUPPORTED for ng > 0, nu[N] != 0, and the sizes
 * where the reference itself reads outside BAbt (soft constraints). */
int d_ip2_mpc_soft_tv(int *kk, int k_max, double mu0, double mu_tol, double alpha_min, int warm_start, double *stat,
                      int N, int *nx, int *nu, int *nb, int **idxb, int *ng, int *ns, double **pBAbt, double **pQ,
                      double **Z, double **z, double **pDCt, double **d, double **ux, int compute_mult, double **pi,
                      double **lam, double **t, double *double_work_memory);
/* include/mpc_solvers.h:71 (mpc_solvers/d_res_ip_soft.c:38) -- r_q, r_b, r_d (hard | general | 2 soft blocks),
 * r_z and mu of a soft-constraint iterate, with the reference's indexing (soft constraint i of stage k on
 * ux[idxb[k][nu_k + i]]) and signs; general constraints allowed.  Entries the reference does not write keep the
 * caller's values. */
void d_res_mpc_soft_tv(int N, int *nx, int *nu, int *nb, int **idxb, int *ng, int *ns, double **hpBAbt, double **hpQ,
                       double **hq, double **hZ, double **hz, double **hux, double **hpDCt, double **hd, double **hpi,
                       double **hlam, double **ht, double **hrq, double **hrb, double **hrd, double **hrz, double *mu);
/* include/mpc_solvers.h:36 (mpc_solvers/d_res_ip_hard.c:38) -- r_q, r_b, r_d and mu (no r_m) */
void d_res_mpc_hard_tv(int N, int *nx, int *nu, int *nb, int **idxb, int *ng, double **hpBAbt, double **hb,
                       double **hpQ, double **hq, double **hux, double **hpDCt, double **hd, double **hpi,
                       double **hlam, double **ht, double **hrq, double **hrb, double **hrd, double *mu);

/* Partial condensing: N stages -> N2 blocks, block i keeping [u_{T-1}; ..; u_0; x_0] as its
 * stage variable.  The condensed data are written into `memory` with the reference's own carve, the pointer
 * arrays hpBAbt2 .. hidxb2 are set into it, and the terminal stage aliases the caller's (d_part_cond.c:1052-1056).
 * Stages with nu+nx > 16 (e.g. the condensed nu2+nx2 = 84 of configs[4]) are solved by
 * d_back_ric_rec_sv_tv_res on the wide-stage path. */
/* The three building blocks of one condensing block (horizon N, condensed variable [u_{N-1}; ..; u_0; x_0]), each
 * one hk_pcond launch.  Gamma_j = hpGamma[j] is lib4 with (sum_{i<=j} nu_i + nx_0 + 1) rows, nx_{j+1} columns,
 * panel stride round_up(nx_{j+1}, 2); work is not used (every temporary is on the device).  Only the elements the
 * reference writes are written, except the strict upper triangle of pRSQrq2 (of each u_s x u_s diagonal block
 * and of the first stage's square), which the reference copies from its work matrix: it is left as the caller
 * had it (every consumer reads the lower triangle).  Limits as for d_part_cond (nx <= 63, Gamma rows x nx <= 3072): else no output and
 * hpmpc_mi355x_last_error() = HPMPC_MI355X_EUNSUPPORTED. */
/* include/lqcp_solvers.h:80 (lqcp_solvers/d_part_cond.c:214) -- Gamma_0..Gamma_{N-1} and pBAbt2 = Gamma_{N-1} */
void d_cond_BAbt(int N, int *nx, int *nu, double **hpBAbt, double *work, double **hpGamma, double *pBAbt2);
/* include/lqcp_solvers.h:82 (d_part_cond.c:312) -- the condensed Hessian from the given Gamma_0..Gamma_{N-2} */
void d_cond_RSQrq(int N, int *nx, int *nu, double **hpBAbt, double **hpRSQrq, double **hpGamma, double *work,
                  double *pRSQrq2);
/* include/lqcp_solvers.h:84 (d_part_cond.c:579) -- boxes of stage 0 and input boxes stay boxes (d2 lower/upper
 * at 0 / round_up(nbb,4), idxb2), state boxes of stages 1..N-1 become rows of pDCt2 with bounds at
 * 2 round_up(nbb,4) / + round_up(nbg,4) */
void d_cond_DCtd(int N, int *nx, int *nu, int *nb, int **hidxb, double **hd, double **hpGamma, double *pDCt2,
                 double *d2, int *idxb2);
/* include/lqcp_solvers.h:86 (lqcp_solvers/d_part_cond.c:694) */
void d_part_cond_compute_problem_size(int N, int *nx, int *nu, int *nb, int **hidxb, int *ng, int N2, int *nx2,
                                      int *nu2, int *nb2, int *ng2);
/* include/lqcp_solvers.h:88 (d_part_cond.c:743) -- every temporary lives on the device: 64 bytes */
int d_part_cond_work_space_size_bytes(int N, int *nx, int *nu, int *nb, int **hidxb, int *ng, int N2, int *nx2,
                                      int *nu2, int *nb2, int *ng2);
/* include/lqcp_solvers.h:90 (d_part_cond.c:868) */
int d_part_cond_memory_space_size_bytes(int N, int *nx, int *nu, int *nb, int **hidxb, int *ng, int N2, int *nx2,
                                        int *nu2, int *nb2, int *ng2);
/* include/lqcp_solvers.h:92 (d_part_cond.c:926) */
void d_part_cond(int N, int *nx, int *nu, int *nb, int **hidxb, int *ng, double **hpBAbt, double **hpRSQrq,
                 double **hpDCt, double **hd, int N2, int *nx2, int *nu2, int *nb2, int **hidxb2, int *ng2,
                 double **hpBAbt2, double **hpRSQrq2, double **hpDCt2, double **hd2, void *memory, void *work);
/* include/lqcp_solvers.h:94 (d_part_cond.c:1066) */
int d_part_expand_work_space_size_bytes(int N, int *nx, int *nu, int *nb, int *ng);
/* include/lqcp_solvers.h:96 (d_part_cond.c:1103) */
void d_part_expand_solution(int N, int *nx, int *nu, int *nb, int **hidxb, int *ng, double **hpBAbt, double **hb,
                            double **hpRSQrq, double **hrq, double **hpDCt, double **hux, double **hpi,
                            double **hlam, double **ht, int N2, int *nx2, int *nu2, int *nb2, int **hidxb2,
                            int *ng2, double **hux2, double **hpi2, double **hlam2, double **ht2, void *work);

/* High-level wrappers of include/c_interface.h: dense problem data in column-major
 * (fortran_order_*) or row-major (c_order_*) layout, packed to lib4 on the host, then partial condensing (N2 < N,
 * ng == 0 before stage N) or not, the residual IPM, the expansion and the residual infinity norms
 * inf_norm_res = [max|r_q|, max|r_b|, max|r_d|, mu], all through the entry points above (on the GPU).
 * lam is returned compact as [lam_lb (nb) | lam_ub (nb) | lam_lg (ng) | lam_ug (ng)].  The KKT re-solve wrappers
 * re-use the factor the IPM wrapper left in work0 (full-space solves only). */
/* include/c_interface.h:59 (interfaces/c/c_interface_work_space.c:70) */
int hpmpc_d_ip_ocp_hard_tv_work_space_size_bytes(int N, int *nx, int *nu, int *nb, int **hidxb, int *ng, int N2);
/* include/c_interface.h:60 (defined by the reference only in interfaces/c/fortran_order_interface_libstr.c:110): the
 * same size for boxes given by count, nbu[k] inputs and nbx[k] states */
int hpmpc_d_ip_ocp_hard_tv_work_space_size_bytes_noidxb(int N, int *nx, int *nu, int *nb, int *nbx, int *nbu, int *ng, int N2);
/* include/c_interface.h:66 (interfaces/c/fortran_order_interface.c:690) -- k_max Newton steps from (ux0, pi0, lam0,
 * t0) with centering target mu0 on the full space; lam and t returned compact like the IPM wrapper's lam */
int fortran_order_d_ip_ocp_hard_tv_single_newton_step(int *kk, int k_max, double mu0, double mu_tol, int N, int *nx, int *nu_N, int *nb, int **hidxb, int *ng, int N2, int warm_start, double **A, double **B, double **b, double **Q, double **S, double **R, double **q, double **r, double **lb, double **ub, double **C, double **D, double **lg, double **ug, double **x, double **u, double **pi, double **lam, double **t, double *inf_norm_res, void *work0, double *stat, double **ux0, double **pi0, double **lam0, double **t0);
/* include/c_interface.h:70 (interfaces/c/c_interface_work_space.c:177) -- the reference's formula over this library's
 * d_ip2_mpc_soft_tv work space */
int hpmpc_d_ip_ocp_soft_tv_work_space_size_bytes(int N, int *nx, int *nu, int *nb, int **hidxb, int *ng, int *ns);
/* include/c_interface.h:71 (interfaces/c/fortran_order_interface.c:1442) -- soft-constraint IPM wrapper: idxb / lb /
 * ub list the nb hard boxes then the ns soft ones, Z / z = [lower (ns) | upper (ns)]; full space; lam returned as
 * [lo nb | up nb | lg ng | ug ng | 4 soft blocks of ns].  As the reference's IPM sees it, z is not used (the
 * reference never copies it, :1712-1719); inf_norm_res comes from d_res_mpc_soft_tv called as declared (the
 * reference's call is shifted by one argument, :1880).  Limits of d_ip2_mpc_soft_tv apply. */
int fortran_order_d_ip_ocp_soft_tv(int *kk, int k_max, double mu0, double mu_tol, int N, int *nx, int *nu_N, int *nb,
                                   int **hidxb, int *ng, int *ns, int warm_start, double **A, double **B, double **b,
                                   double **Q, double **S, double **R, double **q, double **r, double **Z, double **z,
                                   double **lb, double **ub, double **C, double **D, double **lg, double **ug,
                                   double **x, double **u, double **pi, double **lam, double *inf_norm_res,
                                   void *work0, double *stat);
/* include/c_interface.h:62 (interfaces/c/c_order_interface.c:53) */
int c_order_d_ip_ocp_hard_tv(int *kk, int k_max, double mu0, double mu_tol, int N, int *nx, int *nu, int *nb,
                             int **hidxb, int *ng, int N2, int warm_start, double **A, double **B, double **b,
                             double **Q, double **S, double **R, double **q, double **r, double **lb, double **ub,
                             double **C, double **D, double **lg, double **ug, double **x, double **u, double **pi,
                             double **lam, double *inf_norm_res, void *work0, double *stat);
/* include/c_interface.h:63 (interfaces/c/c_order_interface.c:692) */
void c_order_d_solve_kkt_new_rhs_ocp_hard_tv(int N, int *nx, int *nu, int *nb, int **hidxb, int *ng, double **A,
                                             double **B, double **b, double **Q, double **S, double **R, double **q,
                                             double **r, double **lb, double **ub, double **C, double **D, double **lg,
                                             double **ug, double **x, double **u, double **pi, double **lam,
                                             double *inf_norm_res, double *work0);
/* include/c_interface.h:65 (interfaces/c/fortran_order_interface.c:53) */
int fortran_order_d_ip_ocp_hard_tv(int *kk, int k_max, double mu0, double mu_tol, int N, int *nx, int *nu, int *nb,
                                   int **hidxb, int *ng, int N2, int warm_start, double **A, double **B, double **b,
                                   double **Q, double **S, double **R, double **q, double **r, double **lb,
                                   double **ub, double **C, double **D, double **lg, double **ug, double **x,
                                   double **u, double **pi, double **lam, double *inf_norm_res, void *work0,
                                   double *stat);
/* include/c_interface.h:67 (interfaces/c/fortran_order_interface.c:1082) */
void fortran_order_d_solve_kkt_new_rhs_ocp_hard_tv(int N, int *nx, int *nu, int *nb, int **hidxb, int *ng,
                                                   double **A, double **B, double **b, double **Q, double **S,
                                                   double **R, double **q, double **r, double **lb, double **ub,
                                                   double **C, double **D, double **lg, double **ug, double **x,
                                                   double **u, double **pi, double **lam, double *inf_norm_res,
                                                   double *work0);

/* Legacy uniform-size wrappers (include/c_interface.h:40-53; interfaces/c/fortran_order_interface.c:1975,3017,
 * c_order_interface.c:1052,2083): N stages of nx states / nu inputs in flat arrays (time_invariant: one copy of each
 * stage array; lg / ug are read per stage either way), x0 = x[0..nx) folded into stage 0, nb boxes per stage
 * ([inputs | states]; nb - nu state boxes on stage N), ng general constraints per stage and ngN on stage N; the
 * alternate IPM d_ip2_mpc_hard_tv, then d_res_mpc_hard_tv for inf_norm_res.  u (N nu), x (stages 1..N), pi (N nx),
 * lam / t with stage stride 2 nb + 2 ng.  The KKT twins re-solve on the factor the IPM wrapper left in work0 with
 * new x0, b, r, q, qf and bounds.  The reference's quirks and the reads it makes of unwritten memory are listed in
 * hpmpc_amd/csrc/hpmpc_capi_mpc.cpp. */
/* include/c_interface.h:40 -- declared, never defined by the reference: the doubles of work0 these wrappers use */
int hpmpc_d_ip_mpc_hard_tv_work_space_size_doubles(int N, int nx, int nu, int nb, int ng, int ngN);
/* include/c_interface.h:45 (interfaces/c/c_order_interface.c:1052) */
int c_order_d_ip_mpc_hard_tv(int *kk, int k_max, double mu0, double mu_tol, int N, int nx, int nu, int nb, int ng,
                             int ngN, int time_invariant, int free_x0, int warm_start, double *A, double *B,
                             double *b, double *Q, double *Qf, double *S, double *R, double *q, double *qf, double *r,
                             double *lb, double *ub, double *C, double *D, double *lg, double *ug, double *Cf,
                             double *lgf, double *ugf, double *x, double *u, double *pi, double *lam, double *t,
                             double *inf_norm_res, double *work0, double *stat);
/* include/c_interface.h:46 (interfaces/c/c_order_interface.c:2083) */
void c_order_d_solve_kkt_new_rhs_mpc_hard_tv(int N, int nx, int nu, int nb, int ng, int ngN, int time_invariant,
                                             int free_x0, double *A, double *B, double *b, double *Q, double *Qf,
                                             double *S, double *R, double *q, double *qf, double *r, double *lb,
                                             double *ub, double *C, double *D, double *lg, double *ug, double *Cf,
                                             double *lgf, double *ugf, double *x, double *u, double *pi, double *lam,
                                             double *t, double *inf_norm_res, double *work0);
/* include/c_interface.h:52 (interfaces/c/fortran_order_interface.c:1975) */
int fortran_order_d_ip_mpc_hard_tv(int *kk, int k_max, double mu0, double mu_tol, int N, int nx, int nu, int nb,
                                   int ng, int ngN, int time_invariant, int free_x0, int warm_start, double *A,
                                   double *B, double *b, double *Q, double *Qf, double *S, double *R, double *q,
                                   double *qf, double *r, double *lb, double *ub, double *C, double *D, double *lg,
                                   double *ug, double *Cf, double *lgf, double *ugf, double *x, double *u, double *pi,
                                   double *lam, double *t, double *inf_norm_res, double *work0, double *stat);
/* include/c_interface.h:53 (interfaces/c/fortran_order_interface.c:3017) */
void fortran_order_d_solve_kkt_new_rhs_mpc_hard_tv(int N, int nx, int nu, int nb, int ng, int ngN, int time_invariant,
                                                   int free_x0, double *A, double *B, double *b, double *Q, double *Qf,
                                                   double *S, double *R, double *q, double *qf, double *r, double *lb,
                                                   double *ub, double *C, double *D, double *lg, double *ug,
                                                   double *Cf, double *lgf, double *ugf, double *x, double *u,
                                                   double *pi, double *lam, double *t, double *inf_norm_res,
                                                   double *work0);

/* ================================ Part 2: batched device API ==================================== */

/* Opaque plan: stage sizes, box indices and device tables shared by every problem of a batch. */
typedef struct hpmpc_mi355x_plan hpmpc_mi355x_plan;

/* Create a plan for horizon N with per-stage sizes (nu[N] is ignored and treated as 0; idxb[k]
 * lists the nb[k] boxed variables of stage k).  Returns NULL on unsupported sizes. */
hpmpc_mi355x_plan *hpmpc_mi355x_plan_create(int N, const int *nx, const int *nu, const int *nb,
                                            const int *const *idxb, const int *ng);
void hpmpc_mi355x_plan_destroy(hpmpc_mi355x_plan *plan);

/* Device-array geometry of a problem-major batch (all sizes in doubles).  Stage k of problem p reads its BAbt
 * block at BAbt + p * BAbt_stride + BAbt_off[k], or -- when BAbt_shared[k] is nonzero -- at BAbt + BAbt_off[k] for
 * every problem (likewise RSQrq).  Shared blocks give the time-invariant / aliased mode of the reference drivers
 * (test_problems/test_d_ip_hard.c:652-662: every inner stage points at one block) across a whole batch: e.g. only
 * stage 0 per problem (its b row carries A x0 + b) and one shared inner block for every other stage.  The offsets
 * must fit in 32 bits.  A plan keeps one device table per distinct layout it has seen (its first use uploads it,
 * synchronously), up to 64: a call with a 65th distinct layout fails with HPMPC_MI355X_EUNSUPPORTED. */
typedef struct {
    long long BAbt_stride;   /* doubles between problems (0: shared by all problems) */
    long long RSQrq_stride;
    const long long *BAbt_off;   /* host array [N]   : lib4 block of stage k inside one problem */
    const long long *RSQrq_off;  /* host array [N+1] */
    const unsigned char *BAbt_shared;   /* host array [N] or NULL (no shared block) */
    const unsigned char *RSQrq_shared;  /* host array [N+1] or NULL */
} hpmpc_mi355x_layout;

/* Doubles of per-problem device workspace the batched calls need (factor + IPM iterate). */
long long hpmpc_mi355x_ws_doubles(const hpmpc_mi355x_plan *plan);

/* Batched d_ip2_res_mpc_hard_tv on problems [p0, p0+count) of a batch of nprob problems.
 * d, lam, t: 32 doubles per stage ([lb(pnb) | ub(pnb)], reference padded layout inside the stride);
 * ux, pi: 16 doubles per stage (ux in the reference variable order, pi over x_{k+1}).
 * kk, ret: per problem; stat: 5*k_max per problem.  Asynchronous on `stream` (hipStream_t). */
int hpmpc_mi355x_ipm_batch(const hpmpc_mi355x_plan *plan, const hpmpc_mi355x_layout *lay, int nprob, int p0,
                           int count, const double *BAbt, const double *RSQrq, const double *d, double *ux, double *pi,
                           double *lam, double *t, double *ws, int k_max, double mu0, double mu_tol, double alpha_min,
                           int warm_start, int compute_mult, int *kk, int *ret, double *stat, void *stream);

/* Latency path: hpmpc_mi355x_ipm_batch with each problem's WHOLE solve in one launch -- one workgroup per problem
 * runs init and every iteration's passes back to back on one CU, so its stage data and factor stay in that XCD's L2
 * and no launch or host poll separates the passes.  For a lone problem or a handful (configs[1]); for throughput
 * over many problems use hpmpc_mi355x_ipm_queue.  Same arguments as hpmpc_mi355x_ipm_batch; the results agree with
 * it to rounding (the four-wave kernel splits each sweep over waves and hipcc contracts a few products
 * differently), with the same kk and ret on every tested problem.  One exception: if a hand-over wait between the
 * kernel's waves expires (~2^22 polls; a bug, never a data condition) the solve stops after that iteration with
 * ret[p] = HPMPC_MI355X_EMW and stat[5 k_max p + 0..3] = diagnostic integers (flag, expected, found, wave); the
 * reference-named entry points then return HPMPC_MI355X_EMW, set hpmpc_mi355x_last_error() and copy nothing. */
int hpmpc_mi355x_ipm_solo(const hpmpc_mi355x_plan *plan, const hpmpc_mi355x_layout *lay, int nprob, int p0, int count,
                          const double *BAbt, const double *RSQrq, const double *d, double *ux, double *pi,
                          double *lam, double *t, double *ws, int k_max, double mu0, double mu_tol, double alpha_min,
                          int warm_start, int compute_mult, int *kk, int *ret, double *stat, void *stream);

/* One pass of the batched IPM, for callers that interleave their own work or timing: the batched
 * solve above is pass 0 (init) followed by k_max rounds of passes 1 (factorisation), 2 (predictor
 * solve + step length + mu_aff), 3 (corrector solve + step length), 4 (update + residuals); problems
 * that have finished return immediately.  Same arguments as hpmpc_mi355x_ipm_batch plus `pass`. */
int hpmpc_mi355x_ipm_pass(const hpmpc_mi355x_plan *plan, const hpmpc_mi355x_layout *lay, int nprob, int p0,
                          int count, const double *BAbt, const double *RSQrq, const double *d, double *ux, double *pi,
                          double *lam, double *t, double *ws, int k_max, double mu0, double mu_tol, double alpha_min,
                          int warm_start, int compute_mult, int *kk, int *ret, double *stat, int pass, void *stream);

/* hpmpc_mi355x_ipm_batch with a hipEvent pair around every pass kernel; synchronises `stream` and
 * returns in pass_ms[0..4] the summed device time of passes 0..4 (benchmark / profiling use). */
int hpmpc_mi355x_ipm_batch_profiled(const hpmpc_mi355x_plan *plan, const hpmpc_mi355x_layout *lay, int nprob,
                                    int p0, int count, const double *BAbt, const double *RSQrq, const double *d,
                                    double *ux, double *pi, double *lam, double *t, double *ws, int k_max, double mu0,
                                    double mu_tol, double alpha_min, int warm_start, int compute_mult, int *kk,
                                    int *ret, double *stat, double *pass_ms, void *stream);

/* Problem queue (continuous batching): solve nq problems with n_slots resident solver slots.  Queue
 * entry q solves data problem q % nprob (BAbt/RSQrq/d as in hpmpc_mi355x_ipm_batch, nprob problems);
 * ux/pi/lam/t/kk/ret/stat are per queue entry (nq of each, same strides); ws holds n_slots
 * workspaces; qctl is device scratch of HPMPC_MI355X_QUEUE_CTL_INTS(n_slots) ints.  A slot whose problem has
 * finished takes the next entry at the following iteration, so the GPU is not left idle behind the slowest
 * problem of a batch.  Lanes: the slots are split into L contiguous lanes (HPMPC_MI355X_QUEUE_LANES, environment,
 * default 4, at most one per 1024 slots and HPMPC_MI355X_QUEUE_LANES_MAX), each a queue on its own stream (lane 0
 * on `stream`, the others forked from it and joined back into it) handing out entries from one shared counter
 * (qctl[0]), so that one lane's pass kernels fill the tail of another's.  Lane i's control block starts at
 * qctl[6 i + 3 s_i] (s_i: its first slot): [0] (lane 0: the shared counter of entries handed out), [1] entries
 * the lane finished, [2 + s] the entry its slot s holds (-1 none), then the lengths and entries of two lists of
 * the slots that iterate (workgroup i of an iteration runs the i-th listed slot, so a draining queue keeps one
 * slot per SIMD).  qctl[6 HPMPC_MI355X_QUEUE_LANES_MAX + 3 n_slots] and the
 * next int hold the iterations / problems the drain finished.  Drain: once a lane has handed out every entry and
 * at most its share (by slots) of HPMPC_MI355X_QUEUE_DRAIN (environment, default 768) slots still iterate, its
 * survivors finish one per four-wave workgroup (the multi-wave body of hpmpc_mi355x_ipm_solo) in one launch.  Results are those of hpmpc_mi355x_ipm_batch on each entry: bitwise
 * for the entries finished by the iteration passes (all of them with HPMPC_MI355X_QUEUE_DRAIN=0), to rounding
 * for those finished in the drain (the multi-wave bodies contract a few products differently).  The per-slot
 * workspace is reused, so a queue solve leaves no factor behind for d_kkt_solve_new_rhs_res_mpc_hard_tv; for
 * the same reason its update pass writes neither the iterate backups nor r_m, which only that re-solve reads.
 * Synchronises with the device once per chunk of iterations (it polls the finished counter); on
 * return the last chunk may still be running on `stream`.  An iteration (tick) is three launches: the
 * factorisation, the predictor and corrector of each problem back to back, and the update.  pass_ms (nullable):
 * device time of [init + drain, fact, pred + corr, 0, update] summed over the run and the lanes (the lanes'
 * kernels overlap); n_ticks (nullable): iterations enqueued, summed over the lanes (launches of each kernel). */
int hpmpc_mi355x_ipm_queue(const hpmpc_mi355x_plan *plan, const hpmpc_mi355x_layout *lay, int nprob, int nq,
                           int n_slots, const double *BAbt, const double *RSQrq, const double *d, double *ux,
                           double *pi, double *lam, double *t, double *ws, int *qctl, int k_max, double mu0,
                           double mu_tol, double alpha_min, int warm_start, int compute_mult, int *kk, int *ret,
                           double *stat, double *pass_ms, int *n_ticks, void *stream);

/* Batched d_back_ric_rec_sv_tv_res (no box / no update rows): factor into ws, ux/pi as above. */
int hpmpc_mi355x_ric_sv_batch(const hpmpc_mi355x_plan *plan, const hpmpc_mi355x_layout *lay, int nprob, int p0,
                              int count, const double *BAbt, const double *RSQrq, double *ux, double *pi, double *ws,
                              int compute_pi, int compute_Pb, double *Pb, void *stream);

/* Batched d_back_ric_rec_trf_tv_res (factorisation only, no box terms) into ws. */
int hpmpc_mi355x_ric_trf_batch(const hpmpc_mi355x_plan *plan, const hpmpc_mi355x_layout *lay, int nprob, int p0,
                               int count, const double *BAbt, const double *RSQrq, double *ws, void *stream);

/* Batched d_back_ric_rec_trs_tv_res re-using the factor in ws; b (16/stage, state order), q (16/stage,
 * variable order). */
int hpmpc_mi355x_ric_trs_batch(const hpmpc_mi355x_plan *plan, const hpmpc_mi355x_layout *lay, int nprob, int p0,
                               int count, const double *BAbt, const double *RSQrq, const double *b, const double *q,
                               double *ux, double *pi, double *ws, int compute_pi, int compute_Pb, double *Pb,
                               void *stream);

/* Thread-local status of the last call (0 = success). */
int hpmpc_mi355x_last_error(void);
/* Library build string (architecture, kernel variant). */
const char *hpmpc_mi355x_version(void);


/* ---- partial-condensing pipeline on device-resident batches (configs[4]) ----
 * A pcond plan holds the original and the condensed stage layouts shared by a batch.  Arrays are
 * problem-major with the per-problem sizes of hpmpc_mi355x_pcond_sizes and the stage offsets of
 * hpmpc_mi355x_pcond_offsets (lib4 blocks / padded vectors at those offsets). */
typedef struct hpmpc_mi355x_pcond_plan hpmpc_mi355x_pcond_plan;
hpmpc_mi355x_pcond_plan *hpmpc_mi355x_pcond_plan_create(int N, const int *nx, const int *nu, const int *nb,
                                                        const int *const *idxb, const int *ng, int N2);
void hpmpc_mi355x_pcond_plan_destroy(hpmpc_mi355x_pcond_plan *plan);
/* out[15]: original BAbt, RSQrq, d, ux, pi | condensed BAbt2, RSQrq2, DCt2, d2, ux2, pi2, factor | Gamma
 * scratch | N2 | max ng2 (doubles per problem) */
int hpmpc_mi355x_pcond_sizes(const hpmpc_mi355x_pcond_plan *plan, long long *out);
/* out[6*(N+1)] (which 0: original) or out[6*(N2+1)] (which 1: condensed): oB, oR, oD, oU, oP, oL per stage */
int hpmpc_mi355x_pcond_offsets(const hpmpc_mi355x_pcond_plan *plan, int which, long long *out);
/* d_part_cond of problems [p0, p0+count): one workgroup per (block, problem); G is the Gamma scratch */
int hpmpc_mi355x_pcond_batch(const hpmpc_mi355x_pcond_plan *plan, int nprob, int p0, int count, const double *BAbt,
                             const double *RSQrq, const double *d, double *G, double *BAbt2, double *RSQrq2,
                             double *DCt2, double *d2, void *stream);
/* d_back_ric_rec_sv_tv_res on the condensed problems (wide stages; no constraints) */
int hpmpc_mi355x_pcond_ric_sv_batch(const hpmpc_mi355x_pcond_plan *plan, int nprob, int p0, int count,
                                    const double *BAbt2, const double *RSQrq2, double *ws, double *ux2, double *pi2,
                                    int compute_pi, void *stream);
/* d_part_expand_solution (b / rq read from the augmented rows of BAbt / RSQrq) */
int hpmpc_mi355x_pexpand_batch(const hpmpc_mi355x_pcond_plan *plan, int nprob, int p0, int count, const double *BAbt,
                               const double *RSQrq, const double *ux2, const double *pi2, const double *lam2,
                               const double *t2, double *ux, double *pi, double *lam, double *t, void *stream);

/* ---- the IPM on wide stages for device-resident batches ----
 * d_ip2_res_mpc_hard_tv (mpc_solvers/d_ip2_res_hard.c:116) for problems whose stages exceed the 16-wide tile
 * (nu+nx+1 <= 128, nx <= 64, stage tiles within 64 KiB of LDS; any nb <= nu+nx, any ng): one 256-thread
 * workgroup runs a whole solve, one launch per batch.  Arrays are problem-major with the per-problem sizes of
 * hpmpc_mi355x_wide_sizes and the stage offsets of hpmpc_mi355x_wide_offsets; the lib4 blocks, the padded
 * [lb | ub | lg | ug] vectors and the DCt blocks sit at those offsets. */
typedef struct hpmpc_mi355x_wide_plan hpmpc_mi355x_wide_plan;
hpmpc_mi355x_wide_plan *hpmpc_mi355x_wide_plan_create(int N, const int *nx, const int *nu, const int *nb,
                                                      const int *const *idxb, const int *ng);
void hpmpc_mi355x_wide_plan_destroy(hpmpc_mi355x_wide_plan *plan);
/* out[8]: doubles per problem of BAbt, RSQrq, DCt, d (= lam = t), ux, pi, the work image; N */
int hpmpc_mi355x_wide_sizes(const hpmpc_mi355x_wide_plan *plan, long long *out);
/* out[6*(N+1)]: oB, oR, oG, oD, oU, oP per stage */
int hpmpc_mi355x_wide_offsets(const hpmpc_mi355x_wide_plan *plan, long long *out);
/* problems [p0, p0+count) of the batch; kk / ret per problem, stat 5*k_max per problem (nullable), work: each
 * problem's work image (factor, iterate backup).  Every other array is required (DCt only when some stage has
 * ng > 0): a null one returns HPMPC_MI355X_EUNSUPPORTED.  Asynchronous on `stream` (a hipStream_t, or null). */
int hpmpc_mi355x_wide_ipm_batch(const hpmpc_mi355x_wide_plan *plan, int nprob, int p0, int count, const double *BAbt,
                                const double *RSQrq, const double *DCt, const double *d, double *ux, double *pi,
                                double *lam, double *t, double *work, int k_max, double mu0, double mu_tol,
                                double alpha_min, int warm_start, int compute_mult, int *kk, int *ret, double *stat,
                                void *stream);
/* the condensed problem's wide plan of a pcond plan (owned by it; null when ng[N] > 0 or beyond the limits):
 * condense -> hpmpc_mi355x_wide_ipm_batch on BAbt2 / RSQrq2 / DCt2 / d2 -> hpmpc_mi355x_pexpand_batch is the
 * IPM on a partially condensed batch (the c_interface wrappers' N2 < N path, batched) */
const hpmpc_mi355x_wide_plan *hpmpc_mi355x_pcond_wide_plan(const hpmpc_mi355x_pcond_plan *plan);

#ifdef __cplusplus
}
#endif
#endif /* HPMPC_MI355X_H_ */
