// hk_wide_ipm.hip -- MI355X (gfx950) interior-point solver for problems whose stages exceed the 16-wide register
// tile of hk_riccati.h: caller problems with nu+nx > 16 or more than 16 constraint slots per stage, and the
// partially condensed problems of d_part_cond (nu2+nx2 = 84 at configs[4], inner state boxes turned into
// general constraints).  SURVEY.md §8a rows a7-a16 on wide stages.
//
// One 256-thread workgroup runs a WHOLE solve of one problem in a single launch: the Mehrotra loop with its
// convergence test lives on the device, so there is no host round trip and no pass launch per iteration, and a
// problem that converges frees its CU slot at once.  Per iteration:
//   * the element-wise IPM work over the problem's flattened constraint list (WideCSlot): box slots read their
//     variable, general slots a dot product with their column of DCt_k (HBM); step lengths and mu are
//     workgroup reductions;
//   * the Riccati factorisation + solve (wide_sv_body) and the solve with the corrector right-hand side
//     (wide_trs_body) of hk_wide_core.h, with the box terms, the general-constraint terms DCt diag(Qx_g) DCt'
//     (MFMA) and b / q taken on the device from the IPM vectors;
//   * the residuals (d_res_res_mpc_hard_tv): one row of r_q / r_b per thread, r_d / r_m per constraint slot.
// The control flow, iteration statistics and return codes follow mpc_solvers/d_ip2_res_hard.c:116-1345 (the
// restatement is oracle/hpmpc_oracle.c ipm_core); each pass below names the reference routine it restates.
#include <hip/hip_runtime.h>

#include "hk_launch_guard.h"

#ifdef HK_STAMPS
// Diagnostic build only: per-phase s_memtime cycle totals of workgroup 0 (tools/wide_phases.py); WSUB marks the
// sub-phases of the Riccati bodies (hk_wide_core.h)
__device__ unsigned long long* g_wdbg;
__device__ unsigned long long g_wsub_t0;
#define WSUB(i)                                                                             \
    do {                                                                                    \
        unsigned long long t_;                                                              \
        asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t_)::"memory");           \
        if (g_wdbg && blockIdx.x == 0 && threadIdx.x == 0) {                                \
            if ((i) > 0) g_wdbg[11 + (i)] += t_ - g_wsub_t0;                                \
            g_wsub_t0 = t_;                                                                 \
        }                                                                                   \
    } while (0)
#define TSUB(i)                                                                             \
    do {                                                                                    \
        unsigned long long t_;                                                              \
        asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t_)::"memory");           \
        if (g_wdbg && blockIdx.x == 0 && threadIdx.x == 0) {                                \
            if ((i) > 0) g_wdbg[22 + (i)] += t_ - g_wsub_t0;                                \
            g_wsub_t0 = t_;                                                                 \
        }                                                                                   \
    } while (0)
#endif
#include "hk_wide_core.h"

namespace {

// Per-problem pointers of one solve.
struct IP {
    const double *BAbt, *RSQ, *DCt, *d;
    double *ux, *pi, *lam, *t;
    double *F, *dux, *dpi, *Pb, *rq, *rb, *uxb, *pib;
    double *dlam, *dt, *tinv, *lamt, *rd, *rm, *tb, *lb, *Qx, *qx;
    double* stat;
    const double *vb, *vq;
};

__device__ __forceinline__ IP ip_ptrs(const WideIpmArgs& A, int p) {
    IP P;
    P.BAbt = A.w.BAbt + (long)p * A.w.sB;
    P.RSQ = A.w.RSQ + (long)p * A.w.sR;
    P.DCt = A.w.DCt ? A.w.DCt + (long)p * A.w.sG : nullptr;
    P.d = A.d ? A.d + (long)p * A.sC : nullptr;
    P.ux = A.ux + (long)p * A.w.sU;
    P.pi = A.pi + (long)p * A.w.sP;
    P.lam = A.lam + (long)p * A.sC;
    P.t = A.t + (long)p * A.sC;
    double* w = A.iw + (long)p * A.sI;
    P.F = w + A.oF;
    P.dux = w + A.oDux;
    P.dpi = w + A.oDpi;
    P.Pb = w + A.oPb;
    P.rq = w + A.oRq;
    P.rb = w + A.oRb;
    P.uxb = w + A.oUb;
    P.pib = w + A.oPib;
    P.dlam = w + A.oDlam;
    P.dt = w + A.oDt;
    P.tinv = w + A.oTinv;
    P.lamt = w + A.oLamt;
    P.rd = w + A.oRd;
    P.rm = w + A.oRm;
    P.tb = w + A.oTb;
    P.lb = w + A.oLb;
    P.Qx = w + A.oQx;
    P.qx = w + A.oqx;
    P.stat = A.stat ? A.stat + (long)p * A.sS : nullptr;
    P.vb = A.vb ? A.vb + (long)p * A.w.sP : nullptr;
    P.vq = A.vq ? A.vq + (long)p * A.w.sU : nullptr;
    return P;
}

// the stage table in LDS (wide_stage_table; per-lane reads here: the stage index may differ between lanes)
__device__ __forceinline__ const WideStage* wst(const WideIpmArgs& A) {
    extern __shared__ double sm[];
    return reinterpret_cast<const WideStage*>(sm + A.w.offST);
}

// workgroup reductions (every thread gets the result); red = 8 doubles of LDS
__device__ __forceinline__ double wg_sum(double v, double* red) {
    v = hk::wave_sum(v);
    bar();
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
    bar();
    return (red[0] + red[1]) + (red[2] + red[3]);
}
__device__ __forceinline__ double wg_min(double v, double* red) {
    v = hk::wave_min(v);
    bar();
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
    bar();
    return fmin(fmin(red[0], red[1]), fmin(red[2], red[3]));
}

// the reference's step-length rule (d_aux_ip_hard_lib4.c:541-565): each thread applies it in slot order to
// its own slots; the workgroup result is the minimum of the per-thread values
__device__ __forceinline__ void alpha_rule(double& al, double v, double dv) {
    if (-al * dv > v) al = -v / dv;
}

// x at a constraint: the boxed variable, or DCt_k' x_k for a general constraint (dgemv_t_lib)
__device__ __forceinline__ double cval(const WideIpmArgs& A, const IP& P, const double* x, const WideCSlot& c) {
    if (c.var >= 0) return x[c.var];
    const WideStage s = wst(A)[-1 - c.var];
    // the slots of one wave may sit on different stages: the problem's (wave-uniform) bases, per-lane offsets
    return bdot(
        s.nu + s.nx, [&](int i, bool ok) { return hk::gld(P.DCt, s.oG + p4i(i, c.g, s.sdG), ok); },
        [&](int i, bool ok) { return hk::gld(x, s.oU + i, ok); });
}

// ---- d_init_var_mpc_hard_tv (d_aux_ip_hard_lib4.c:43-149) ----
__device__ __forceinline__ void init_var(const WideIpmArgs& A, const IP& P) {
    const int tid = threadIdx.x;
    const double thr0 = 0.1, mu0 = A.mu0;
    if (!A.warm_start)
        for (int e = tid; e < A.nU; e += WT) P.ux[e] = 0.0;
    bar();
    for (int e = tid; e < A.ncs; e += WT) {
        const WideCSlot c = A.cs[e];
        if (c.var < 0) continue;
        const double dl = P.d[c.lo], du = P.d[c.up];
        double x = P.ux[c.var];
        double tl = -dl + x, tu = du - x;
        if (tl < thr0) {
            if (tu < thr0) {
                x = (-du + dl) * 0.5;
                tl = thr0;
                tu = thr0;
            } else {
                tl = thr0;
                x = dl + thr0;
            }
        } else if (tu < thr0) {
            tu = thr0;
            x = du - thr0;
        }
        P.ux[c.var] = x;
        P.t[c.lo] = tl;
        P.t[c.up] = tu;
        P.lam[c.lo] = mu0 / tl;
        P.lam[c.up] = mu0 / tu;
    }
    for (int e = tid; e < A.nP; e += WT) P.pi[e] = 0.0;
    bar();
    for (int e = tid; e < A.ncs; e += WT) {
        const WideCSlot c = A.cs[e];
        if (c.var >= 0) continue;
        const double v = cval(A, P, P.ux, c);
        double tl = v + -P.d[c.lo];
        double tu = -v + P.d[c.up];
        tl = fmax(thr0, tl);
        tu = fmax(thr0, tu);
        P.t[c.lo] = tl;
        P.t[c.up] = tu;
        P.lam[c.lo] = mu0 / tl;
        P.lam[c.up] = mu0 / tu;
    }
    bar();
}

// ---- d_update_hessian_mpc_hard_tv (d_aux_ip_hard_lib4.c:217-383) ----
__device__ __forceinline__ void update_hessian(const WideIpmArgs& A, const IP& P, double smu) {
    for (int e = threadIdx.x; e < A.ncs; e += WT) {
        const WideCSlot c = A.cs[e];
        const double til = 1.0 / P.t[c.lo], tiu = 1.0 / P.t[c.up];
        const double ll = P.lam[c.lo], lu = P.lam[c.up];
        const double ltl = ll * til, ltu = lu * tiu, dll = til * smu, dlu = tiu * smu;
        P.tinv[c.lo] = til;
        P.tinv[c.up] = tiu;
        P.lamt[c.lo] = ltl;
        P.lamt[c.up] = ltu;
        P.dlam[c.lo] = dll;
        P.dlam[c.up] = dlu;
        P.Qx[c.q] = ltl + ltu;
        P.qx[c.q] = lu - ltu * P.d[c.up] + dlu - ll - ltl * P.d[c.lo] - dll;
    }
    bar();
}

// ---- d_compute_alpha_mpc_hard_tv (d_aux_ip_hard_lib4.c:489-614) ----
__device__ __forceinline__ double compute_alpha(const WideIpmArgs& A, const IP& P, double* red) {
    double al = 1.0;
    for (int e = threadIdx.x; e < A.ncs; e += WT) {
        const WideCSlot c = A.cs[e];
        const double x = cval(A, P, P.dux, c);
        const double tl = P.t[c.lo], tu = P.t[c.up], ll = P.lam[c.lo], lu = P.lam[c.up];
        double dtl, dtu;
        if (c.var >= 0) {
            dtl = x - P.d[c.lo] - tl;
            dtu = -x + P.d[c.up] - tu;
        } else {
            dtl = x + (-P.d[c.lo] - tl);
            dtu = -x + (P.d[c.up] - tu);
        }
        const double dll = P.dlam[c.lo] - (P.lamt[c.lo] * dtl + ll);
        const double dlu = P.dlam[c.up] - (P.lamt[c.up] * dtu + lu);
        P.dt[c.lo] = dtl;
        P.dt[c.up] = dtu;
        P.dlam[c.lo] = dll;
        P.dlam[c.up] = dlu;
        alpha_rule(al, ll, dll);
        alpha_rule(al, lu, dlu);
        alpha_rule(al, tl, dtl);
        alpha_rule(al, tu, dtu);
    }
    return wg_min(al, red);
}

// ---- d_compute_mu_mpc_hard_tv (d_aux_ip_hard_lib4.c:715-770) ----
__device__ __forceinline__ double compute_mu(const WideIpmArgs& A, const IP& P, double alpha, double* red) {
    double s = 0.0;
    for (int e = threadIdx.x; e < A.ncs; e += WT) {
        const WideCSlot c = A.cs[e];
        s += (P.lam[c.lo] + alpha * P.dlam[c.lo]) * (P.t[c.lo] + alpha * P.dt[c.lo]) +
             (P.lam[c.up] + alpha * P.dlam[c.up]) * (P.t[c.up] + alpha * P.dt[c.up]);
    }
    return wg_sum(s, red) * A.mu_scal;
}

// ---- d_update_gradient_mpc_hard_tv (d_aux_ip_hard_lib4.c:387-485) ----
__device__ __forceinline__ void update_gradient(const WideIpmArgs& A, const IP& P, double smu) {
    for (int e = threadIdx.x; e < A.ncs; e += WT) {
        const WideCSlot c = A.cs[e];
        const double dll = P.tinv[c.lo] * (smu - P.dlam[c.lo] * P.dt[c.lo]);
        const double dlu = P.tinv[c.up] * (smu - P.dlam[c.up] * P.dt[c.up]);
        P.dlam[c.lo] = dll;
        P.dlam[c.up] = dlu;
        P.qx[c.q] += dlu - dll;
    }
    bar();
}

// iterate backup (ux, pi, lam, t -> *_bkp)
__device__ __forceinline__ void backup(const WideIpmArgs& A, const IP& P) {
    const int tid = threadIdx.x;
    for (int e = tid; e < A.nU; e += WT) P.uxb[e] = P.ux[e];
    for (int e = tid; e < A.nP; e += WT) P.pib[e] = P.pi[e];
    for (int e = tid; e < A.ncs; e += WT) {
        const WideCSlot c = A.cs[e];
        P.lb[c.lo] = P.lam[c.lo];
        P.lb[c.up] = P.lam[c.up];
        P.tb[c.lo] = P.t[c.lo];
        P.tb[c.up] = P.t[c.up];
    }
}

// ---- d_update_var_mpc_hard_tv (d_aux_ip_hard_lib4.c:618-711); returns mu ----
__device__ __forceinline__ double update_var(const WideIpmArgs& A, const IP& P, double alpha, double* red) {
    const int tid = threadIdx.x;
    for (int e = tid; e < A.nU; e += WT) P.ux[e] += alpha * (P.dux[e] - P.ux[e]);
    for (int e = tid; e < A.nP; e += WT) P.pi[e] += alpha * (P.dpi[e] - P.pi[e]);
    double s = 0.0;
    for (int e = tid; e < A.ncs; e += WT) {
        const WideCSlot c = A.cs[e];
        const double ll = P.lam[c.lo] + alpha * P.dlam[c.lo], lu = P.lam[c.up] + alpha * P.dlam[c.up];
        const double tl = P.t[c.lo] + alpha * P.dt[c.lo], tu = P.t[c.up] + alpha * P.dt[c.up];
        P.lam[c.lo] = ll;
        P.lam[c.up] = lu;
        P.t[c.lo] = tl;
        P.t[c.up] = tu;
        s += ll * tl + lu * tu;
    }
    return wg_sum(s, red) * A.mu_scal;
}

// ---- d_update_hessian_gradient_res_mpc_hard_tv (d_aux_ip_hard_lib4.c:954-1078) ----
__device__ __forceinline__ void update_hessian_gradient_res(const WideIpmArgs& A, const IP& P) {
    for (int e = threadIdx.x; e < A.ncs; e += WT) {
        const WideCSlot c = A.cs[e];
        const double til = 1.0 / P.t[c.lo], tiu = 1.0 / P.t[c.up];
        const double ll = P.lam[c.lo], lu = P.lam[c.up];
        P.tinv[c.lo] = til;
        P.tinv[c.up] = tiu;
        P.Qx[c.q] = til * ll + tiu * lu;
        P.qx[c.q] = til * (P.rm[c.lo] - ll * P.rd[c.lo]) - tiu * (P.rm[c.up] + lu * P.rd[c.up]);
    }
    bar();
}

// ---- d_update_gradient_res_mpc_hard_tv (d_aux_ip_hard_lib4.c:1550-1639) ----
__device__ __forceinline__ void update_gradient_res(const WideIpmArgs& A, const IP& P) {
    for (int e = threadIdx.x; e < A.ncs; e += WT) {
        const WideCSlot c = A.cs[e];
        P.qx[c.q] = P.tinv[c.lo] * (P.rm[c.lo] - P.lam[c.lo] * P.rd[c.lo]) -
                    P.tinv[c.up] * (P.rm[c.up] + P.lam[c.up] * P.rd[c.up]);
    }
    bar();
}

// ---- d_compute_dt_dlam_res_mpc_hard_tv (:1082-1176) / d_compute_alpha_res_mpc_hard_tv (:1180-1313) ----
__device__ __forceinline__ double dt_dlam_res(const WideIpmArgs& A, const IP& P, bool with_alpha, double* red) {
    double al = 1.0;
    for (int e = threadIdx.x; e < A.ncs; e += WT) {
        const WideCSlot c = A.cs[e];
        const double x = cval(A, P, P.dux, c);
        const double dtl = x - P.rd[c.lo], dtu = -x + P.rd[c.up];
        const double ll = P.lam[c.lo], lu = P.lam[c.up];
        const double dll = -P.tinv[c.lo] * (ll * dtl + P.rm[c.lo]);
        const double dlu = -P.tinv[c.up] * (lu * dtu + P.rm[c.up]);
        P.dt[c.lo] = dtl;
        P.dt[c.up] = dtu;
        P.dlam[c.lo] = dll;
        P.dlam[c.up] = dlu;
        if (with_alpha) {
            alpha_rule(al, ll, dll);
            alpha_rule(al, lu, dlu);
            alpha_rule(al, P.t[c.lo], dtl);
            alpha_rule(al, P.t[c.up], dtu);
        }
    }
    if (!with_alpha) {
        bar();
        return 1.0;
    }
    return wg_min(al, red);
}

// ---- d_compute_centering_correction_res_mpc_hard_tv (:1512-1546) ----
__device__ __forceinline__ void centering_correction(const WideIpmArgs& A, const IP& P, double smu) {
    for (int e = threadIdx.x; e < A.ncs; e += WT) {
        const WideCSlot c = A.cs[e];
        P.rm[c.lo] += P.dt[c.lo] * P.dlam[c.lo] - smu;
        P.rm[c.up] += P.dt[c.up] * P.dlam[c.up] - smu;
    }
    bar();
}

// ---- d_update_var_res_mpc_hard_tv (:1317-1378, bkp: :1382-1449) ----
__device__ __forceinline__ void update_var_res(const WideIpmArgs& A, const IP& P, double alpha, bool bkp) {
    const int tid = threadIdx.x;
    for (int e = tid; e < A.nU; e += WT) {
        if (bkp) P.uxb[e] = P.ux[e];
        P.ux[e] += alpha * P.dux[e];
    }
    for (int e = tid; e < A.nP; e += WT) {
        if (bkp) P.pib[e] = P.pi[e];
        P.pi[e] += alpha * P.dpi[e];
    }
    for (int e = tid; e < A.ncs; e += WT) {
        const WideCSlot c = A.cs[e];
        if (bkp) {
            P.lb[c.lo] = P.lam[c.lo];
            P.lb[c.up] = P.lam[c.up];
            P.tb[c.lo] = P.t[c.lo];
            P.tb[c.up] = P.t[c.up];
        }
        P.lam[c.lo] += alpha * P.dlam[c.lo];
        P.lam[c.up] += alpha * P.dlam[c.up];
        P.t[c.lo] += alpha * P.dt[c.lo];
        P.t[c.up] += alpha * P.dt[c.up];
    }
    bar();
}

// ---- residuals: d_res_res_mpc_hard_tv (c99/d_res_ip_res_hard.c:39-319) and, plain = true, d_res_mpc_hard_tv
// (d_res_ip_hard.c:38-330, the KKT residuals with the reference's signs, negated at the end) ----
// b_k / q_k come from vb / vq when given, else from the augmented rows.  Returns mu (unchanged without
// constraints for the res variant, 0 for the plain one).
__device__ __forceinline__ double residuals(const WideIpmArgs& A, const IP& P, bool plain, double mu_in, double* red) {
    using hk::gld;
    const int tid = threadIdx.x, N = A.w.N;
    // the rows of every stage (nux r_q rows, then nx1 r_b rows) form one flat range that all threads share, so a
    // stage's ~100 rows do not leave most of the workgroup idle; each row's dot products load 8 terms at a time
    // from the problem's (wave-uniform) bases.  Every row sums in the reference's order, as before.
    // a general-constraint row term stops at the row's 16-row tile's last nonzero DCt column once the factorisation
    // has recorded it (kct): the skipped terms are products of exact zeros
    extern __shared__ double sm[];
    const int* kct = reinterpret_cast<const int*>(sm + A.offKC);
    const bool kcu = __builtin_amdgcn_readfirstlane(kct[(N + 1) * KC_STRIDE]) != 0;
    int k = 0, rbase = 0;
    for (int rr = tid;; rr += WT) {
        while (k <= N && rr >= rbase + wst(A)[k].nu + wst(A)[k].nx + wst(A)[k].nx1) {
            rbase += wst(A)[k].nu + wst(A)[k].nx + wst(A)[k].nx1;
            k++;
        }
        if (k > N) break;
        const int r = rr - rbase;
        const WideStage s = wst(A)[k];
        const int nux = s.nu + s.nx;
        const double* R = P.RSQ + s.oR;
        const double* B = P.BAbt + s.oB;
        const int pnb = s.pnb, png = (s.ng + 3) & ~3;
        const int olg = s.oD + 2 * pnb;  // general multipliers: lam[olg + g] (lower), lam[olg + png + g] (upper)
        {
            if (r < nux) {
                const int i = r;
                const double q = P.vq ? P.vq[s.oU + i] : P4(R, s.sdR, nux, i);
                const int glim = (kcu && kct[k * KC_STRIDE + KC_STRIDE - 1]) ? kct[k * KC_STRIDE + (i >> 4)] : s.ng;
                const double sy = bdot<16>(
                    nux,
                    [&](int j, bool ok) {
                        return gld(P.RSQ, s.oR + (i >= j ? p4i(i, j, s.sdR) : p4i(j, i, s.sdR)), ok);
                    },
                    [&](int j, bool ok) { return gld(P.ux, s.oU + j, ok); });
                const double bp = bdot(
                    s.nx1, [&](int j, bool ok) { return gld(P.BAbt, s.oB + p4i(i, j, s.sdB), ok); },
                    [&](int j, bool ok) { return gld(P.pi, s.oP + j, ok); });
                const int lo = A.vbox[s.oU + i];
                double v;
                if (!plain) {
                    v = q;
                    if (k > 0 && i >= s.nu) v -= P.pi[wst(A)[k - 1].oP + i - s.nu];
                    if (lo >= 0) v += -P.lam[lo] + P.lam[lo + pnb];
                    v += sy;
                    if (k < N) v += bp;
                    if (s.ng > 0)
                        v += bdot<16>(
                            glim, [&](int g, bool ok) { return gld(P.DCt, s.oG + p4i(i, g, s.sdG), ok); },
                            [&](int g, bool ok) { return gld(P.lam, olg + png + g, ok) - gld(P.lam, olg + g, ok); });
                } else {
                    v = -q;
                    if (k > 0 && i >= s.nu) v = -q + P.pi[wst(A)[k - 1].oP + i - s.nu];
                    if (lo >= 0) v += P.lam[lo] - P.lam[lo + pnb];
                    v -= sy;
                    if (s.ng > 0) {
                        auto dg = [&](int g, bool ok) { return gld(P.DCt, s.oG + p4i(i, g, s.sdG), ok); };
                        const double ca = bdot<16>(glim, dg, [&](int g, bool ok) { return gld(P.lam, olg + g, ok); });
                        const double cb =
                            bdot<16>(glim, dg, [&](int g, bool ok) { return gld(P.lam, olg + png + g, ok); });
                        v += ca;
                        v -= cb;
                    }
                    if (k < N) v -= bp;
                    v = -v;
                }
                P.rq[s.oU + i] = v;
            } else {
                const int j = r - nux;
                const WideStage s1 = wst(A)[k + 1];
                const double b = P.vb ? P.vb[s.oP + j] : P4(B, s.sdB, nux, j);
                const double x1 = P.ux[s1.oU + s1.nu + j];
                const double c = bdot<16>(
                    nux, [&](int i, bool ok) { return gld(P.BAbt, s.oB + p4i(i, j, s.sdB), ok); },
                    [&](int i, bool ok) { return gld(P.ux, s.oU + i, ok); });
                P.rb[s.oP + j] = plain ? -((x1 - b) - c) : (b - x1) + c;
            }
        }
    }
    bar();  // r_q / r_b complete before anything reads them
    double s2 = 0.0;
    for (int e = tid; e < A.ncs; e += WT) {
        const WideCSlot c = A.cs[e];
        const double x = cval(A, P, P.ux, c);
        const double tl = P.t[c.lo], tu = P.t[c.up], ll = P.lam[c.lo], lu = P.lam[c.up];
        const double dl = P.d[c.lo], du = P.d[c.up];
        if (!plain) {
            if (c.var >= 0) {
                P.rd[c.lo] = dl - x + tl;
                P.rd[c.up] = du - x - tu;
            } else {
                P.rd[c.lo] = (dl + tl) - x;
                P.rd[c.up] = (du - tu) - x;
            }
            const double ml = ll * tl, mu = lu * tu;
            P.rm[c.lo] = ml;
            P.rm[c.up] = mu;
            s2 += ml + mu;
        } else {
            if (c.var >= 0) {
                P.rd[c.lo] = -(x - dl - tl);
                P.rd[c.up] = -(-x + du - tu);
            } else {
                P.rd[c.lo] = -(x + (-dl - tl));
                P.rd[c.up] = -(-x + (du - tu));
            }
            s2 += ll * tl + lu * tu;
        }
    }
    const double tot = wg_sum(s2, red);
    if (A.ncs == 0) return plain ? 0.0 : mu_in;
    return tot / A.nbt2;
}

// Riccati calls on the IPM's vectors
__device__ __forceinline__ void ric_sv(const WideIpmArgs& A, const IP& P, const double* vb, const double* vq, bool box, double* ux,
                       double* pi) {
    WideProb q;
    q.BAbt = P.BAbt;
    q.RSQ = P.RSQ;
    q.DCt = box ? P.DCt : nullptr;
    q.F = P.F;
    q.ux = ux;
    q.pi = pi;
    q.Pb = P.Pb;
    q.vb = vb;
    q.vq = vq;
    q.Qx = box ? P.Qx : nullptr;
    q.qx = box ? P.qx : nullptr;
    q.hb = q.hq = nullptr;
    q.compute_pi = A.compute_mult;
    q.compute_Pb = 1;
    q.dev_box = box;
    extern __shared__ double sm[];
    int* kct = reinterpret_cast<int*>(sm + A.offKC);
    q.kct = kct;
    q.kc_use = __builtin_amdgcn_readfirstlane(kct[(A.w.N + 1) * KC_STRIDE]) != 0;
    bar();
    wide_sv_body(A.w, q);
    bar();
    if (threadIdx.x == 0 && box) kct[(A.w.N + 1) * KC_STRIDE] = 1;  // every chunk has been scanned once (read after a barrier)
}

__device__ __forceinline__ void ric_trs(const WideIpmArgs& A, const IP& P, const double* hb, const double* hq, int compute_Pb,
                        double* ux, double* pi) {
    WideProb q;
    q.BAbt = P.BAbt;
    q.RSQ = P.RSQ;
    q.DCt = P.DCt;
    q.F = P.F;
    q.ux = ux;
    q.pi = pi;
    q.Pb = P.Pb;
    q.vb = q.vq = q.Qx = nullptr;
    q.qx = P.qx;
    q.hb = hb;
    q.hq = hq;
    q.compute_pi = A.compute_mult;
    q.compute_Pb = compute_Pb;
    q.dev_box = false;
    extern __shared__ double sm[];
    int* kct = reinterpret_cast<int*>(sm + A.offKC);  // the general-constraint column limits of the factorisation
    q.kct = kct;
    q.kc_use = __builtin_amdgcn_readfirstlane(kct[(A.w.N + 1) * KC_STRIDE]) != 0;
    bar();
    wide_trs_body(A.w, q);
    bar();
}

}  // namespace

#ifdef HK_STAMPS
extern "C" __attribute__((visibility("default"))) int hpmpc_mi355x_wide_ipm_debug(void* dev_ptr) {
    return (int)hipMemcpyToSymbol(HIP_SYMBOL(g_wdbg), &dev_ptr, sizeof(void*));
}
#define WPH(i)                                                                              \
    do {                                                                                    \
        unsigned long long t_;                                                              \
        asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t_)::"memory");           \
        if (g_wdbg && blockIdx.x == 0 && threadIdx.x == 0) {                                \
            if (ph_ >= 0) g_wdbg[ph_] += t_ - t0_;                                          \
            g_wdbg[31] += 1;                                                                \
        }                                                                                   \
        t0_ = t_;                                                                           \
        ph_ = (i);                                                                          \
    } while (0)
#else
#define WPH(i) \
    do {       \
    } while (0)
#endif

__global__ __launch_bounds__(WT, 2) void hk_wide_ipm(WideIpmArgs A) {
#ifdef HK_STAMPS
    unsigned long long t0_ = 0;
    int ph_ = -1;
#endif
    extern __shared__ double sm[];
    const int p = blockIdx.x + A.w.p0;
    if (p >= A.w.nprob) return;
    {
        int* kct = reinterpret_cast<int*>(sm + A.offKC);  // the DCt chunk limits, empty
        for (int e = threadIdx.x; e < (A.w.N + 1) * KC_STRIDE + 1; e += WT) kct[e] = 0;
    }
    wide_stage_table(A.w);
    const int tid = threadIdx.x;
    double* red = sm + A.offR;
    const IP P = ip_ptrs(A, p);
    const int mode = A.mode;
    auto put_stat = [&](int kk, int j, double v) {
        if (tid == 0 && P.stat) P.stat[5 * kk + j] = v;
    };
    auto finish = [&](int kk, int ret, double mu) {
        if (tid == 0) {
            A.kk[p] = kk;
            A.ret[p] = ret;
            if (A.mu) A.mu[p] = mu;
        }
    };

    if (mode == WI_RES || mode == WI_RES_PLAIN) {
        const double mu = residuals(A, P, mode == WI_RES_PLAIN, A.mu ? A.mu[p] : 0.0, red);
        finish(0, 0, mu);
        return;
    }
    if (mode == WI_KKT_RES) {  // d_ip2_res_hard.c:2139-2299: last iterate from the backup, residuals, trs
        for (int e = tid; e < A.nU; e += WT) P.ux[e] = P.uxb[e];
        for (int e = tid; e < A.nP; e += WT) P.pi[e] = P.pib[e];
        for (int e = tid; e < A.ncs; e += WT) {
            const WideCSlot c = A.cs[e];
            P.t[c.lo] = P.tb[c.lo];
            P.t[c.up] = P.tb[c.up];
            P.lam[c.lo] = P.lb[c.lo];
            P.lam[c.up] = P.lb[c.up];
        }
        bar();
        const double mu = residuals(A, P, false, 0.0, red);
        bar();
        update_gradient_res(A, P);
        ric_trs(A, P, P.rb, P.rq, 1, P.dux, P.dpi);
        dt_dlam_res(A, P, false, red);
        update_var_res(A, P, 1.0, false);
        finish(0, 0, mu);
        return;
    }
    if (mode == WI_KKT_P1) {  // d_ip2_hard.c:626-825 (qx from lamt and r_C, trs, t / lam from the solution)
        for (int e = tid; e < A.ncs; e += WT) {
            const WideCSlot c = A.cs[e];
            P.qx[c.q] = -P.lamt[c.up] * P.d[c.up] - P.lamt[c.lo] * P.d[c.lo];
        }
        bar();
        ric_trs(A, P, P.vb, P.vq, 1, P.ux, P.pi);
        for (int e = tid; e < A.ncs; e += WT) {
            const WideCSlot c = A.cs[e];
            const double x = cval(A, P, P.ux, c);
            const double tl = x - P.d[c.lo], tu = -x + P.d[c.up];
            P.t[c.lo] = tl;
            P.t[c.up] = tu;
            P.lam[c.lo] = -P.lamt[c.lo] * tl;
            P.lam[c.up] = -P.lamt[c.up] * tu;
        }
        finish(0, 0, 0.0);
        return;
    }

    // ---- the IPMs ----
    const bool newton = mode == WI_NEWTON, p1only = mode == WI_IPM_P1;
    if (A.mu_scal == 0.0) {  // no constraints: one Riccati solve (d_ip2_res_hard.c:428-450, d_ip2_hard.c:282-291)
        if (p1only) {
            ric_sv(A, P, nullptr, nullptr, false, P.dux, P.dpi);
        } else {
            ric_sv(A, P, nullptr, nullptr, false, P.ux, P.pi);
            for (int e = tid; e < A.nU; e += WT) P.uxb[e] = P.ux[e];
            for (int e = tid; e < A.nP; e += WT) P.pib[e] = P.pi[e];
        }
        finish(0, 0, 0.0);
        return;
    }
    double sigma = 0.0, alpha = 1.0, mu = A.mu0, mu_aff = 0.0;
    int kk = 0;
    if (!newton) {
        init_var(A, P);
        // phase 1 (d_ip2_res_hard.c:498-718): no residuals; d_ip2_mpc_hard_tv is this loop run to mu_tol
        const double mu_tol_low = p1only ? A.mu_tol : (A.mu_tol < 1e-5 ? 1e-5 : A.mu_tol);
        while (kk < A.k_max && mu > mu_tol_low && alpha >= A.alpha_min) {
            update_hessian(A, P, 0.0);
            ric_sv(A, P, nullptr, nullptr, true, P.dux, P.dpi);
            alpha = compute_alpha(A, P, red);
            put_stat(kk, 0, sigma);
            put_stat(kk, 1, alpha);
            alpha *= 0.995;
            mu_aff = compute_mu(A, P, alpha, red);
            put_stat(kk, 2, mu_aff);
            sigma = mu_aff / mu;
            sigma = sigma * sigma * sigma;
            update_gradient(A, P, sigma * mu);
            ric_trs(A, P, nullptr, nullptr, 0, P.dux, P.dpi);
            alpha = compute_alpha(A, P, red);
            put_stat(kk, 0, sigma);
            put_stat(kk, 3, alpha);
            alpha *= 0.995;
            backup(A, P);
            mu = update_var(A, P, alpha, red);
            put_stat(kk, 4, mu);
            kk++;
        }
        if (p1only) {  // d_ip2_hard.c:604-612
            const int ret = mu <= A.mu_tol ? 0 : kk >= A.k_max ? 1 : alpha < A.alpha_min ? 2 : -1;
            finish(kk, ret, mu);
            return;
        }
    }
    bar();
    mu = residuals(A, P, false, mu, red);
    bar();
    // phase 2: residual-based Mehrotra (d_ip2_res_hard.c:783-1273); single Newton step: :1640-1905
    while (kk < A.k_max && (newton || (mu > A.mu_tol && alpha >= A.alpha_min))) {
        WPH(0);
        update_hessian_gradient_res(A, P);
        WPH(1);
        if (!newton)
            ric_sv(A, P, P.rb, P.rq, true, P.dux, P.dpi);
        else  // the single-Newton step factorises with the data's own b / q rows
            ric_sv(A, P, nullptr, nullptr, true, P.dux, P.dpi);
        WPH(2);
        alpha = dt_dlam_res(A, P, true, red);
        WPH(3);
        put_stat(kk, 0, sigma);
        put_stat(kk, 1, alpha);
        alpha *= 0.995;
        mu_aff = compute_mu(A, P, alpha, red);
        put_stat(kk, 2, mu_aff);
        if (!newton) {
            sigma = mu_aff / mu;
            sigma = sigma * sigma * sigma;
            centering_correction(A, P, sigma * mu);
        } else {
            centering_correction(A, P, A.mu0);
        }
        WPH(4);
        update_gradient_res(A, P);
        WPH(5);
        ric_trs(A, P, P.rb, P.rq, 0, P.dux, P.dpi);
        WPH(6);
        alpha = dt_dlam_res(A, P, true, red);
        put_stat(kk, 0, sigma);
        put_stat(kk, 3, alpha);
        alpha *= 0.995;
        WPH(7);
        update_var_res(A, P, alpha, true);
        WPH(8);
        mu = residuals(A, P, false, mu, red);
        bar();
        put_stat(kk, 4, mu);
        kk++;
        WPH(9);
    }
    WPH(10);
    const int ret = (!newton && mu <= A.mu_tol) ? 0 : kk >= A.k_max ? 1 : alpha < A.alpha_min ? 2 : -1;
    finish(kk, ret, mu);
}

extern "C" int hk_wide_ipm_launch(const WideIpmArgs* a, int count, int lds_doubles, hipStream_t stream) {
    if (count <= 0) return 0;
    // scratch / LDS need against what the device reserves (round-2 noinline-build fault)
    static const HkKernelLimits lim(reinterpret_cast<const void*>(&hk_wide_ipm));
    if (const int g = lim.check((size_t)lds_doubles * sizeof(double), WT)) return g;
    hipLaunchKernelGGL(hk_wide_ipm, dim3(count), dim3(WT), (size_t)lds_doubles * sizeof(double), stream, *a);
    return (int)hipGetLastError();
}
