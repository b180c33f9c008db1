// hk_soft.hip -- MI355X (gfx950) passes of the soft-constraint IPM d_ip2_mpc_soft_tv
// (mpc_solvers/d_ip2_soft.c:83-547, vector routines mpc_solvers/c99/d_aux_ip_soft_lib4.c:38-999).
//
// One wave per problem.  Lane l = 16 g + c owns constraint slot c (hard boxes first, then soft ones, the
// order of idxb) of stage 4 q + g, q = 0, 1, ..: the per-stage vector routines are element-wise, so a pass
// sweeps the horizon four stages at a time and reduces alpha / mu across the wave.  The Riccati steps between
// the passes are the tile kernels (hk_ric_sv / hk_ric_trs with box terms given per slot):
//   init  d_init_var_mpc_soft_tv
//   hess  d_update_hessian_mpc_soft_tv (sigma mu = 0) -> Qx, qx slots for hk_ric_sv
//   pred  d_compute_alpha + d_compute_mu + d_update_gradient_mpc_soft_tv -> qx slots for hk_ric_trs
//   corr  d_compute_alpha + d_update_var_mpc_soft_tv, iteration count, exit test
// Divisions are IEEE (the reference's 1.0/t and -v/dv).  Every pass returns at once for a problem whose
// loop has ended, so a batch can run a fixed number of iterations without host round trips.
#include <hip/hip_runtime.h>

#include "hk_prims.h"
#include "hk_soft_args.h"

namespace {

using hk::wave_min;
using hk::wave_sum;

constexpr int V16 = 16;

struct Lane {
    int k, c;
    bool ok;
};

__device__ __forceinline__ Lane lane_at(const SoftArgs& a, int q) {
    const int l = threadIdx.x & 63;
    Lane L;
    L.k = 4 * q + (l >> 4);
    L.c = l & 15;
    L.ok = L.k <= a.N;
    return L;
}

__device__ __forceinline__ void alpha_rule(double& al, double v, double dv) {
    if (-al * dv > v) al = -v / dv;
}

__device__ __forceinline__ int exit_code(double mu, double mu_tol, int kk, int k_max, double alpha, double alpha_min) {
    if (mu <= mu_tol) return 0;
    if (kk >= k_max) return 1;
    if (alpha < alpha_min) return 2;
    return -1;
}

struct Prob {
    const double *d, *Z, *z;
    double *t, *lam, *dt, *dlam, *lamt, *tinv, *flat, *ux, *pi, *dux, *dpi, *vQx, *vqx, *scal, *stat;
    int* ist;
};

__device__ __forceinline__ Prob prob(const SoftArgs& a, int p) {
    Prob P;
    P.d = a.d + (long)p * a.sD;
    P.Z = a.Z + (long)p * a.sZ;
    P.z = a.z + (long)p * a.sZ;
    const long oc = (long)p * a.sC;
    P.t = a.t + oc;
    P.lam = a.lam + oc;
    P.dt = a.dt + oc;
    P.dlam = a.dlam + oc;
    P.lamt = a.lamt + oc;
    P.tinv = a.tinv + oc;
    P.flat = a.flat + (long)p * a.sF;
    const long ov = (long)p * a.sV;
    P.ux = a.ux + ov;
    P.pi = a.pi + ov;
    P.dux = a.dux + ov;
    P.dpi = a.dpi + ov;
    P.vQx = a.vQx + ov;
    P.vqx = a.vqx + ov;
    P.scal = a.scal + 4L * p;
    P.ist = a.ist + 4L * p;
    P.stat = a.stat + (long)p * a.sS;
    return P;
}

// d_compute_alpha_mpc_soft_tv (d_aux_ip_soft_lib4.c:611-804): dt, dlam from the Riccati solution dux; the
// largest step in (0, 1] keeping t, lam >= 0 (per lane, then the wave minimum)
__device__ double soft_alpha(const SoftArgs& a, const Prob& P) {
    double al = 1.0;
    for (int q = 0; q < a.nq; q++) {
        const Lane L = lane_at(a, q);
        if (!L.ok) continue;
        const SoftStage s = a.st[L.k];
        if (L.c < s.nb) {
            const int lo = s.oC + L.c, up = lo + s.pnb;
            const double x = P.dux[L.k * V16 + a.idxb[L.k * 16 + L.c]];
            const double dtl = x - P.d[s.oD + L.c] - P.t[lo];
            const double dtu = -x + P.d[s.oD + s.pnb + L.c] - P.t[up];
            const double dll = P.dlam[lo] - (P.lamt[lo] * dtl + P.lam[lo]);
            const double dlu = P.dlam[up] - (P.lamt[up] * dtu + P.lam[up]);
            P.dt[lo] = dtl;
            P.dt[up] = dtu;
            P.dlam[lo] = dll;
            P.dlam[up] = dlu;
            alpha_rule(al, P.lam[lo], dll);
            alpha_rule(al, P.lam[up], dlu);
            alpha_rule(al, P.t[lo], dtl);
            alpha_rule(al, P.t[up], dtu);
        } else if (L.c < s.nb + s.ns) {
            const int i = L.c - s.nb, b0 = s.oC + 2 * s.pnb + i, pns = s.pns;
            const double x = P.dux[L.k * V16 + a.idxb[L.k * 16 + L.c]];
            const double* Zl = P.flat + s.oZl;
            const double* zl = Zl + 2 * pns;
            double dt[4];
            dt[2] = (zl[i] - P.lamt[b0] * x) * Zl[i];
            dt[3] = (zl[pns + i] + P.lamt[b0 + pns] * x) * Zl[pns + i];
            dt[0] = dt[2] + x - P.d[s.oD + 2 * s.pnb + i] - P.t[b0];
            dt[1] = dt[3] - x + P.d[s.oD + 2 * s.pnb + pns + i] - P.t[b0 + pns];
            dt[2] -= P.t[b0 + 2 * pns];
            dt[3] -= P.t[b0 + 3 * pns];
            double dl[4];
#pragma unroll
            for (int j = 0; j < 4; j++) {
                const int e = b0 + j * pns;
                dl[j] = P.dlam[e] - (P.lamt[e] * dt[j] + P.lam[e]);
                P.dt[e] = dt[j];
                P.dlam[e] = dl[j];
            }
#pragma unroll
            for (int j = 0; j < 4; j++) alpha_rule(al, P.lam[b0 + j * pns], dl[j]);
#pragma unroll
            for (int j = 0; j < 4; j++) alpha_rule(al, P.t[b0 + j * pns], dt[j]);
        }
    }
    return wave_min(al);
}

}  // namespace

// which: 0 init, 1 hess, 2 pred, 3 corr
__global__ __launch_bounds__(64) void hk_soft_pass(SoftArgs a, int which) {
    const int p = blockIdx.x + a.p0;
    if (p >= a.nprob) return;
    const int l = threadIdx.x & 63;
    const Prob P = prob(a, p);

    if (which == 0) {  // d_init_var_mpc_soft_tv (d_aux_ip_soft_lib4.c:38-165), ng = 0
        if (!a.warm_start)
            for (int q = 0; q < a.nq; q++) {
                const Lane L = lane_at(a, q);
                if (L.ok && L.c < a.st[L.k].nu + a.st[L.k].nx) P.ux[L.k * V16 + L.c] = 0.0;
            }
        __syncthreads();
        const double thr0 = 0.1;
        for (int q = 0; q < a.nq; q++) {
            const Lane L = lane_at(a, q);
            if (!L.ok) continue;
            const SoftStage s = a.st[L.k];
            if (L.c < s.nb) {
                const int lo = s.oC + L.c, up = lo + s.pnb, iv = L.k * V16 + a.idxb[L.k * 16 + L.c];
                const double dl = P.d[s.oD + L.c], du = P.d[s.oD + s.pnb + L.c];
                double x = P.ux[iv];
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
                P.ux[iv] = x;
                P.t[lo] = tl;
                P.t[up] = tu;
                P.lam[lo] = a.mu0 / tl;
                P.lam[up] = a.mu0 / tu;
            } else if (L.c < s.nb + s.ns) {
                const int b0 = s.oC + 2 * s.pnb + (L.c - s.nb);
#pragma unroll
                for (int j = 0; j < 4; j++) {
                    P.t[b0 + j * s.pns] = 1.0;
                    P.lam[b0 + j * s.pns] = a.mu0;
                }
            }
            if (L.c < s.nx1) {
                P.pi[L.k * V16 + L.c] = 0.0;
                P.dpi[L.k * V16 + L.c] = 0.0;
            }
        }
        if (l == 0) {
            P.scal[0] = a.mu0;
            P.scal[1] = 1.0;
            P.scal[2] = 1.0;
            P.scal[3] = 0.0;
            P.ist[0] = 0;
            P.ist[1] = (0 < a.k_max && a.mu0 > a.mu_tol && 1.0 >= a.alpha_min) ? 1 : 0;
            P.ist[2] = exit_code(a.mu0, a.mu_tol, 0, a.k_max, 1.0, a.alpha_min);
        }
        return;
    }
    if (!P.ist[1]) return;
    const int kk = P.ist[0];
    double* stat = P.stat + 5 * kk;

    if (which == 1) {  // d_update_hessian_mpc_soft_tv (:167-506), sigma mu = 0
        for (int q = 0; q < a.nq; q++) {
            const Lane L = lane_at(a, q);
            if (!L.ok) continue;
            const SoftStage s = a.st[L.k];
            double* Qx = P.flat + s.oQ;
            double* qx = Qx + s.pnb + s.pns;
            if (L.c < s.nb) {
                const int lo = s.oC + L.c, up = lo + s.pnb;
                const double til = 1.0 / P.t[lo], tiu = 1.0 / P.t[up];
                const double ltl = P.lam[lo] * til, ltu = P.lam[up] * tiu;
                const double dll = til * 0.0, dlu = tiu * 0.0;
                P.tinv[lo] = til;
                P.tinv[up] = tiu;
                P.lamt[lo] = ltl;
                P.lamt[up] = ltu;
                P.dlam[lo] = dll;
                P.dlam[up] = dlu;
                const double Q = ltl + ltu;
                const double g = P.lam[up] - ltu * P.d[s.oD + s.pnb + L.c] + dlu - P.lam[lo] -
                                 ltl * P.d[s.oD + L.c] - dll;
                Qx[L.c] = Q;
                qx[L.c] = g;
                P.vQx[L.k * V16 + L.c] = Q;
                P.vqx[L.k * V16 + L.c] = g;
            } else if (L.c < s.nb + s.ns) {
                const int i = L.c - s.nb, pns = s.pns, b0 = s.oC + 2 * s.pnb + i;
                double lt[4], dl[4];
#pragma unroll
                for (int j = 0; j < 4; j++) {
                    const int e = b0 + j * pns;
                    const double ti = 1.0 / P.t[e];
                    P.tinv[e] = ti;
                    lt[j] = P.lam[e] * ti;
                    P.lamt[e] = lt[j];
                    dl[j] = ti * 0.0;
                    P.dlam[e] = dl[j];
                }
                const double* Z = P.Z + s.oZ;
                const double* zz = P.z + s.oZ;
                const double dls = P.d[s.oD + 2 * s.pnb + i], dus = P.d[s.oD + 2 * s.pnb + pns + i];
                double rQx0 = lt[0], rQx1 = lt[1];
                double rqx0 = P.lam[b0] + dl[0] + lt[0] * dls;
                double rqx1 = P.lam[b0 + pns] + dl[1] - lt[1] * dus;
                double* Zl = P.flat + s.oZl;
                double* zl = Zl + 2 * pns;
                const double Zl0 = 1.0 / (Z[i] + rQx0 + lt[2]);
                const double Zl1 = 1.0 / (Z[pns + i] + rQx1 + lt[3]);
                const double zl0 = -zz[i] + rqx0 + P.lam[b0 + 2 * pns] + dl[2];
                const double zl1 = -zz[pns + i] + rqx1 + P.lam[b0 + 3 * pns] + dl[3];
                Zl[i] = Zl0;
                Zl[pns + i] = Zl1;
                zl[i] = zl0;
                zl[pns + i] = zl1;
                rqx0 = rqx0 - rQx0 * zl0 * Zl0;
                rqx1 = rqx1 - rQx1 * zl1 * Zl1;
                rQx0 = rQx0 - rQx0 * rQx0 * Zl0;
                rQx1 = rQx1 - rQx1 * rQx1 * Zl1;
                const double Q = rQx1 + rQx0, g = rqx1 - rqx0;
                Qx[L.c] = Q;
                qx[L.c] = g;
                P.vQx[L.k * V16 + L.c] = Q;
                P.vqx[L.k * V16 + L.c] = g;
            }
        }
        return;
    }

    if (which == 2) {  // predictor: alpha, mu_aff, sigma, then the corrector gradient
        double alpha = soft_alpha(a, P);
        if (l == 0) {
            stat[0] = P.scal[2];
            stat[1] = alpha;
        }
        alpha *= 0.995;
        // d_compute_mu_mpc_soft_tv (:926-999)
        double part = 0.0;
        for (int q = 0; q < a.nq; q++) {
            const Lane L = lane_at(a, q);
            if (!L.ok) continue;
            const SoftStage s = a.st[L.k];
            if (L.c < s.nb) {
                const int lo = s.oC + L.c, up = lo + s.pnb;
                part += (P.lam[lo] + alpha * P.dlam[lo]) * (P.t[lo] + alpha * P.dt[lo]) +
                        (P.lam[up] + alpha * P.dlam[up]) * (P.t[up] + alpha * P.dt[up]);
            } else if (L.c < s.nb + s.ns) {
                const int b0 = s.oC + 2 * s.pnb + (L.c - s.nb), pns = s.pns;
                double v = 0.0;
#pragma unroll
                for (int j = 0; j < 4; j++) {
                    const int e = b0 + j * pns;
                    v += (P.lam[e] + alpha * P.dlam[e]) * (P.t[e] + alpha * P.dt[e]);
                }
                part += v;
            }
        }
        const double mu_aff = wave_sum(part) * a.mu_scal;
        const double mu = P.scal[0];
        double sigma = mu_aff / mu;
        sigma = sigma * sigma * sigma;
        const double smu = sigma * mu;
        if (l == 0) stat[2] = mu_aff;
        // d_update_gradient_mpc_soft_tv (:508-609).  The soft term goes to flat[oS + i] (qx_k + pnbs + nb + i when
        // nb > 0, past the slots of qx_k): it is parked in this lane's vqx slot and added once every stage has
        // made its own update (the targets are only ever accumulated into in this pass, or read back in later
        // passes; the host rejects layouts where one would land in a Zl this pass reads)
        for (int q = 0; q < a.nq; q++) {
            const Lane L = lane_at(a, q);
            if (!L.ok) continue;
            const SoftStage s = a.st[L.k];
            double* qx = P.flat + s.oQ + s.pnb + s.pns;
            if (L.c < s.nb) {
                const int lo = s.oC + L.c, up = lo + s.pnb;
                const double dll = P.tinv[lo] * (smu - P.dlam[lo] * P.dt[lo]);
                const double dlu = P.tinv[up] * (smu - P.dlam[up] * P.dt[up]);
                P.dlam[lo] = dll;
                P.dlam[up] = dlu;
                qx[L.c] += dlu - dll;
            } else if (L.c < s.nb + s.ns) {
                const int i = L.c - s.nb, pns = s.pns, b0 = s.oC + 2 * s.pnb + i;
                double dl[4];
#pragma unroll
                for (int j = 0; j < 4; j++) {
                    const int e = b0 + j * pns;
                    dl[j] = P.tinv[e] * (smu - P.dlam[e] * P.dt[e]);
                    P.dlam[e] = dl[j];
                }
                const double rQx0 = P.lamt[b0], rQx1 = P.lamt[b0 + pns];
                double rqx0 = dl[0], rqx1 = dl[1];
                double* Zl = P.flat + s.oZl;
                double* zl = Zl + 2 * pns;
                zl[i] += rqx0 + dl[2];
                zl[pns + i] += rqx1 + dl[3];
                rqx0 = rqx0 - rQx0 * (rqx0 + dl[2]) * Zl[i];
                rqx1 = rqx1 - rQx1 * (rqx1 + dl[3]) * Zl[pns + i];
                P.vqx[L.k * V16 + L.c] = rqx1 - rqx0;
            }
        }
        __syncthreads();
        for (int q = 0; q < a.nq; q++) {
            const Lane L = lane_at(a, q);
            if (!L.ok) continue;
            const SoftStage s = a.st[L.k];
            if (L.c >= s.nb && L.c < s.nb + s.ns)
                atomicAdd(P.flat + s.oS + (L.c - s.nb), P.vqx[L.k * V16 + L.c]);
        }
        __syncthreads();
        for (int q = 0; q < a.nq; q++) {
            const Lane L = lane_at(a, q);
            if (!L.ok) continue;
            const SoftStage s = a.st[L.k];
            if (L.c < s.nb + s.ns) P.vqx[L.k * V16 + L.c] = P.flat[s.oQ + s.pnb + s.pns + L.c];
        }
        if (l == 0) {
            P.scal[1] = alpha;
            P.scal[2] = sigma;
            P.scal[3] = mu_aff;
        }
        return;
    }

    // which == 3: corrector alpha, d_update_var_mpc_soft_tv (:806-924), exit test (d_ip2_soft.c:333-535)
    double alpha = soft_alpha(a, P);
    if (l == 0) {
        stat[0] = P.scal[2];
        stat[3] = alpha;
    }
    alpha *= 0.995;
    double part = 0.0;
    for (int q = 0; q < a.nq; q++) {
        const Lane L = lane_at(a, q);
        if (!L.ok) continue;
        const SoftStage s = a.st[L.k];
        if (L.c < s.nu + s.nx) {
            const int e = L.k * V16 + L.c;
            P.ux[e] += alpha * (P.dux[e] - P.ux[e]);
        }
        if (L.c < s.nx1) {
            const int e = L.k * V16 + L.c;
            P.pi[e] += alpha * (P.dpi[e] - P.pi[e]);
        }
        if (L.c < s.nb) {
            const int lo = s.oC + L.c, up = lo + s.pnb;
            P.lam[lo] += alpha * P.dlam[lo];
            P.lam[up] += alpha * P.dlam[up];
            P.t[lo] += alpha * P.dt[lo];
            P.t[up] += alpha * P.dt[up];
            part += P.lam[lo] * P.t[lo] + P.lam[up] * P.t[up];
        } else if (L.c < s.nb + s.ns) {
            const int b0 = s.oC + 2 * s.pnb + (L.c - s.nb), pns = s.pns;
            double v = 0.0;
#pragma unroll
            for (int j = 0; j < 4; j++) {
                const int e = b0 + j * pns;
                P.lam[e] += alpha * P.dlam[e];
                P.t[e] += alpha * P.dt[e];
            }
#pragma unroll
            for (int j = 0; j < 4; j++) v += P.lam[b0 + j * pns] * P.t[b0 + j * pns];
            part += v;
        }
    }
    const double mu = wave_sum(part) * a.mu_scal;
    if (l == 0) {
        stat[4] = mu;
        const int k1 = kk + 1;
        P.scal[0] = mu;
        P.scal[1] = alpha;
        P.ist[0] = k1;
        P.ist[1] = (k1 < a.k_max && mu > a.mu_tol && alpha >= a.alpha_min) ? 1 : 0;
        P.ist[2] = exit_code(mu, a.mu_tol, k1, a.k_max, alpha, a.alpha_min);
    }
}

extern "C" int hk_soft_launch(int which, const SoftArgs* a, int count, hipStream_t stream) {
    if (count <= 0) return 0;
    hipLaunchKernelGGL(hk_soft_pass, dim3(count), dim3(64), 0, stream, *a, which);
    return hipGetLastError() == hipSuccess ? 0 : 1;
}

// ------------------------------------------------------------------------------------------------
// d_res_mpc_soft_tv (mpc_solvers/d_res_ip_soft.c:38-268), one workgroup of RT threads per call: the stages in
// order, a thread per row of r_q / r_b and per constraint of r_d / r_z, signs as the reference leaves them (r_q,
// r_b, r_d negated at the end, r_z not).  The reference's layout quirks are kept (soft residual): the
// soft constraint i of stage k acts on ux[idxb[k][nu_k + i]]; its multipliers enter r_q as lam_0 - lam_1 on
// k < N and as -lam_2 + lam_3 on k = N; on stage N, r_q starts from pi_{N-1} - q on the state rows (the input
// rows keep the caller's values) and its symv covers the leading nx_N x nx_N block; mu averages lam t over
// 2 (nb + ng + ns).
// ------------------------------------------------------------------------------------------------
namespace {
constexpr int RT = 256;
__device__ __forceinline__ double q4(const double* A, int sd, int i, int j) {
    return A[(i >> 2) * 4 * sd + (i & 3) + 4 * j];
}
}  // namespace

__global__ __launch_bounds__(RT) void hk_soft_res(SoftResArgs a) {
    __shared__ double red[RT];
    double* B = a.buf;
    const int tid = threadIdx.x;
    double musum = 0.0;
    long ntot = 0;
    for (int k = 0; k <= a.N; k++) {
        const SoftResStage s = a.st[k];
        const int nux = s.nu + s.nx, og = 2 * s.pnb, os = 2 * s.pnb + 2 * s.png, pns = s.pns;
        const bool last = k == a.N;
        const int* ib = a.idxb + s.oI;
        const double *ux = B + s.oux, *lam = B + s.olam, *t = B + s.ot, *d = B + s.od;
        ntot += s.nb + s.ng + s.ns;
        // mu partial sums
        for (int j = tid; j < s.nb; j += RT) musum += lam[j] * t[j] + lam[s.pnb + j] * t[s.pnb + j];
        for (int j = tid; j < s.ng; j += RT) musum += lam[og + j] * t[og + j] + lam[og + s.png + j] * t[og + s.png + j];
        for (int j = tid; j < s.ns; j += RT)
            musum += lam[os + j] * t[os + j] + lam[os + pns + j] * t[os + pns + j] + lam[os + 2 * pns + j] * t[os + 2 * pns + j] +
                     lam[os + 3 * pns + j] * t[os + 3 * pns + j];
        // r_d (negated) and r_z
        double* rd = B + s.ord;
        for (int j = tid; j < s.nb; j += RT) {
            const double x = ux[ib[j]];
            rd[j] = -(x - d[j] - t[j]);
            rd[s.pnb + j] = -(-x + d[s.pnb + j] - t[s.pnb + j]);
        }
        for (int j = tid; j < s.ng; j += RT) {
            const double* G = B + s.oG;
            double g = 0.0;
            for (int i = 0; i < nux; i++) g += q4(G, s.sdG, i, j) * ux[i];
            rd[og + j] = -(g - d[og + j] - t[og + j]);
            rd[og + s.png + j] = -(-g + d[og + s.png + j] - t[og + s.png + j]);
        }
        for (int j = tid; j < s.ns; j += RT) {
            const double x = ux[ib[s.nu + j]];
            rd[os + j] = -(t[os + 2 * pns + j] + x - d[os + j] - t[os + j]);
            rd[os + pns + j] = -(t[os + 3 * pns + j] - x + d[os + pns + j] - t[os + pns + j]);
            const double *Z = B + s.oZ, *z = B + s.oz;
            double* rz = B + s.orz;
            rz[j] = z[j] + Z[j] * t[os + 2 * pns + j] - lam[os + j] - lam[os + 2 * pns + j];
            rz[pns + j] = z[pns + j] + Z[pns + j] * t[os + 3 * pns + j] - lam[os + pns + j] - lam[os + 3 * pns + j];
        }
        // r_q (negated): row i by one thread
        double* rq = B + s.orq;
        const double* q = B + s.oq;
        const int nsym = last ? s.nx : nux;
        for (int i = tid; i < nux; i += RT) {
            double v;
            if (i < s.nu)
                v = last ? rq[i] : -q[i];  // stage N input rows: the caller's values (:199-200 writes only x rows)
            else
                v = -q[i] + (s.opim1 >= 0 ? B[s.opim1 + i - s.nu] : 0.0);
            if (i < nsym) {
                const double* Q = B + s.oQ;
                double acc = 0.0;
                for (int j = 0; j < nsym; j++) acc += (i >= j ? q4(Q, s.sdQ, i, j) : q4(Q, s.sdQ, j, i)) * ux[j];
                v -= acc;
            }
            for (int j = 0; j < s.nb; j++)
                if (ib[j] == i) v += lam[j] - lam[s.pnb + j];
            if (s.ng > 0) {
                const double* G = B + s.oG;
                double acc = 0.0;
                for (int j = 0; j < s.ng; j++) acc += q4(G, s.sdG, i, j) * (lam[og + j] - lam[og + s.png + j]);
                v += acc;
            }
            for (int j = 0; j < s.ns; j++)
                if (ib[s.nu + j] == i)
                    v += last ? -lam[os + 2 * pns + j] + lam[os + 3 * pns + j] : lam[os + j] - lam[os + pns + j];
            if (!last) {
                const double* Bt = B + s.oB;
                const double* pi = B + s.opi;
                double acc = 0.0;
                for (int j = 0; j < s.nx1; j++) acc += q4(Bt, s.sdB, i, j) * pi[j];
                v -= acc;
            }
            rq[i] = -v;
        }
        // r_b (negated): x_{k+1} - A x - B u - b
        if (!last) {
            const double* Bt = B + s.oB;
            const double* ux1 = B + s.oux1;
            double* rb = B + s.orb;
            for (int j = tid; j < s.nx1; j += RT) {
                double acc = 0.0;
                for (int i = 0; i < nux; i++) acc += q4(Bt, s.sdB, i, j) * ux[i];
                rb[j] = -(ux1[s.nu1 + j] - q4(Bt, s.sdB, nux, j) - acc);
            }
        }
    }
    red[tid] = musum;
    __syncthreads();
    for (int w = RT / 2; w > 0; w >>= 1) {
        if (tid < w) red[tid] += red[tid + w];
        __syncthreads();
    }
    if (tid == 0) B[a.omu] = ntot != 0 ? red[0] / (2.0 * ntot) : 0.0;
}

extern "C" int hk_soft_res_launch(const SoftResArgs* a, hipStream_t stream) {
    hipLaunchKernelGGL(hk_soft_res, dim3(1), dim3(RT), 0, stream, *a);
    return (int)hipGetLastError();
}
