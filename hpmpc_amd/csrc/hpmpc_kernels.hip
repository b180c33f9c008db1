// hpmpc_kernels.hip -- MI355X (gfx950) kernels for HPMPC's Riccati / interior-point hot path.
//
// Execution model: one wavefront (64-thread workgroup) owns one QP instance for the whole call; a
// launch covers a batch (grid = number of problems).  Stage data are read straight from HBM in the
// reference's lib4 layout; the recursion state (the previous stage's factor) stays in registers.
// All IPM control flow (iteration count, step length, mu) is per wave, so problems that converge
// early simply retire their wave.
#include "hk_ipm.h"
#include "hpmpc_kargs.h"

using namespace hk;

namespace {

struct Ws {  // per-problem workspace carve (doubles), persistent between an IPM and a KKT re-solve
    double *F, *dux, *dpi, *Pb, *Qx, *qx, *res_q, *res_b, *ux_bkp, *pi_bkp;
    double *dlam, *dt, *t_inv, *lamt, *res_d, *res_m, *t_bkp, *lam_bkp;
};

__device__ __forceinline__ Ws carve(double* W, int N) {
    Ws w;
    const long n1 = N + 1, a = n1 * V16, b = n1 * V32;
    w.F = W;
    W += n1 * FSTRIDE;
    w.dux = W;
    w.dpi = W + a;
    w.Pb = W + 2 * a;
    w.Qx = W + 3 * a;
    w.qx = W + 4 * a;
    w.res_q = W + 5 * a;
    w.res_b = W + 6 * a;
    w.ux_bkp = W + 7 * a;
    w.pi_bkp = W + 8 * a;
    W += 9 * a;
    w.dlam = W;
    w.dt = W + b;
    w.t_inv = W + 2 * b;
    w.lamt = W + 3 * b;
    w.res_d = W + 4 * b;
    w.res_m = W + 5 * b;
    w.t_bkp = W + 6 * b;
    w.lam_bkp = W + 7 * b;
    return w;
}

// Per-batch stage tables (StageInfo, tile->box slot, box slot->variable) are copied into LDS at
// kernel start: every stage iteration reads them with ds_read (lgkmcnt), so the HBM prefetch queue
// (vmcnt) is never drained just to learn the next stage's sizes.
extern __shared__ __attribute__((aligned(16))) char hk_smem[];

struct LdsTabs {
    Scratch* sm;
    const StageInfo* st;
    const signed char* tileslot;
    const signed char* slotvar;
};

__device__ __forceinline__ LdsTabs lds_tables(const KArgs& a) {
    LdsTabs T;
    T.sm = reinterpret_cast<Scratch*>(hk_smem);
    StageInfo* st = reinterpret_cast<StageInfo*>(hk_smem + sizeof(Scratch));
    signed char* ts = reinterpret_cast<signed char*>(st + (a.N + 1));
    signed char* sv = ts + (a.N + 1) * 16;
    const int l = lane_id(), n1 = a.N + 1;
    const int* gst = reinterpret_cast<const int*>(a.st);
    int* lst = reinterpret_cast<int*>(st);
    for (int i = l; i < n1 * 16; i += 64) lst[i] = gst[i];
    const int* gts = reinterpret_cast<const int*>(a.tileslot);
    const int* gsv = reinterpret_cast<const int*>(a.slotvar);
    int* lts = reinterpret_cast<int*>(ts);
    int* lsv = reinterpret_cast<int*>(sv);
    for (int i = l; i < n1 * 4; i += 64) {
        lts[i] = gts[i];
        lsv[i] = gsv[i];
    }
    __syncthreads();
    T.st = st;
    T.tileslot = ts;
    T.slotvar = sv;
    return T;
}

__device__ __forceinline__ RicIO make_io(const KArgs& a, const LdsTabs& T, int p, double* F) {
    RicIO io;
    io.N = a.N;
    io.st = T.st;
    io.tileslot = T.tileslot;
    io.BAbt = a.BAbt + (long)p * a.sB;
    io.RSQ = a.RSQ + (long)p * a.sR;
    io.F = F;
    return io;
}

__device__ __forceinline__ void wsync() { __syncthreads(); }

}  // namespace

// ------------------------------------------------------------------------------------------------
// d_back_ric_rec_sv_tv_res / _trf_ / _trs_ over a batch (one problem per workgroup)
// ------------------------------------------------------------------------------------------------
extern "C" __global__ __launch_bounds__(64) void hk_ric_sv(KArgs a) {
    const LdsTabs T = lds_tables(a);
    Scratch& sm = *T.sm;
    const int p = blockIdx.x + a.p0;
    if (p >= a.nprob) return;
    double* F = a.ws + (long)p * a.sW;
    RicIO io = make_io(a, T, p, F);
    const long o16 = (long)p * a.sV16;
    const double* b = a.vb ? a.vb + o16 : nullptr;
    const double* q = a.vq ? a.vq + o16 : nullptr;
    const double* Qx = a.vQx ? a.vQx + o16 : nullptr;
    const double* qx = a.vqx ? a.vqx + o16 : nullptr;
    double* Pb = a.vPb ? a.vPb + o16 : nullptr;
    ric_backward<true>(io, &sm, a.update_b, b, a.update_q, q, a.use_box, Qx, qx, a.compute_Pb, Pb);
    wsync();
    ric_forward_sv(io, &sm, a.update_b, b, a.ux + o16, a.compute_pi, a.pi + o16);
}

extern "C" __global__ __launch_bounds__(64) void hk_ric_trf(KArgs a) {
    const LdsTabs T = lds_tables(a);
    Scratch& sm = *T.sm;
    const int p = blockIdx.x + a.p0;
    if (p >= a.nprob) return;
    double* F = a.ws + (long)p * a.sW;
    RicIO io = make_io(a, T, p, F);
    const long o16 = (long)p * a.sV16;
    const double* Qx = a.vQx ? a.vQx + o16 : nullptr;
    ric_backward<false>(io, &sm, 0, nullptr, 0, nullptr, a.use_box, Qx, nullptr, 0, nullptr);
}

extern "C" __global__ __launch_bounds__(64) void hk_ric_trs(KArgs a) {
    const LdsTabs T = lds_tables(a);
    Scratch& sm = *T.sm;
    const int p = blockIdx.x + a.p0;
    if (p >= a.nprob) return;
    double* F = a.ws + (long)p * a.sW;
    RicIO io = make_io(a, T, p, F);
    const long o16 = (long)p * a.sV16;
    const double* qx = a.vqx ? a.vqx + o16 : nullptr;
    ric_trs(io, &sm, a.vb + o16, a.vq + o16, a.use_box, qx, a.ux + o16, a.compute_pi, a.pi + o16, a.compute_Pb,
            a.vPb + o16);
}

extern "C" __global__ __launch_bounds__(64) void hk_res(KArgs a) {
    const LdsTabs T = lds_tables(a);
    Scratch& sm = *T.sm;
    const int p = blockIdx.x + a.p0;
    if (p >= a.nprob) return;
    RicIO io = make_io(a, T, p, nullptr);
    BoxTab bt{T.tileslot, T.slotvar};
    const long o16 = (long)p * a.sV16, o32 = (long)p * a.sV32;
    double* out = a.ws + (long)p * a.sW;  // [rq | rb] V16, [rd | rm] V32
    const long n1 = a.N + 1;
    double mu = 0.0;
    const bool have = residuals(io, bt, &sm, a.vb ? a.vb + o16 : nullptr, a.vq ? a.vq + o16 : nullptr,
                                a.ux + o16, a.pi + o16, a.d + o32, a.lam + o32, a.t + o32, out, out + n1 * V16,
                                out + 2 * n1 * V16, out + 2 * n1 * V16 + n1 * V32, mu);
    if (lane_id() == 0 && have) a.mu_out[p] = mu;
}

// ------------------------------------------------------------------------------------------------
// IPM vector passes (d_aux_ip_hard_lib4.c), box constraints, four stages per pass.
// ------------------------------------------------------------------------------------------------
namespace {

__device__ void init_var(const RicIO& io, const BoxTab& bt, const double* dv, double* ux, double* pi, double* lam,
                         double* t, double mu0, int warm_start) {
    const int l = lane_id();
    const double thr0 = 0.1;
    if (!warm_start)
        for (int i = l; i < (io.N + 1) * V16; i += 64) ux[i] = 0.0;
    for (int i = l; i < io.N * V16; i += 64) pi[i] = 0.0;
    wsync();
    HK_FOR_BOX(io, k, {
        const int v = bt.slotvar[k * 16 + slot];
        double x = ux[k * V16 + v];
        const double dl = dv[lo], du = dv[up];
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
        ux[k * V16 + v] = x;
        t[lo] = tl;
        t[up] = tu;
        lam[lo] = mu0 / tl;
        lam[up] = mu0 / tu;
    });
    wsync();
}

// sequential step-length rule of d_compute_alpha_* (:541-565): per lane, min-reduced afterwards
__device__ __forceinline__ void alpha_rule(double& al, double lam, double dlam, double t, double dt) {
    (void)t;
    (void)dt;
    if (-al * dlam > lam) al = -lam / dlam;
}

}  // namespace

extern "C" __global__ __launch_bounds__(64) void hk_ipm(KArgs a) {
    const LdsTabs T = lds_tables(a);
    Scratch& sm = *T.sm;
    const int p = blockIdx.x + a.p0;
    if (p >= a.nprob) return;
    const int N = a.N;
    Ws w = carve(a.ws + (long)p * a.sW, N);
    RicIO io = make_io(a, T, p, w.F);
    BoxTab bt{T.tileslot, T.slotvar};
    const long o16 = (long)p * a.sV16, o32 = (long)p * a.sV32;
    double* ux = a.ux + o16;
    double* pi = a.pi + o16;
    double* lam = a.lam + o32;
    double* t = a.t + o32;
    const double* dv = a.d + o32;
    double* stat = a.stat + (long)p * 5 * a.k_max;
    const int l = lane_id();

    int nbt = 0;
    for (int k = 0; k <= N; k++) nbt += io.st[k].nb;
    int kk = 0, ret;
    if (nbt == 0) {
        // no constraints: one sv and return (d_ip2_res_hard.c:428-450)
        ric_backward<true>(io, &sm, 0, nullptr, 0, nullptr, 0, nullptr, nullptr, 1, w.Pb);
        wsync();
        ric_forward_sv(io, &sm, 0, nullptr, ux, a.compute_mult, pi);
        wsync();
        for (int i = l; i < (N + 1) * V16; i += 64) {
            w.ux_bkp[i] = ux[i];
            w.pi_bkp[i] = pi[i];
        }
        if (l == 0) {
            a.kk[p] = 0;
            a.ret[p] = 0;
        }
        return;
    }
    const double mu_scal = 1.0 / (2.0 * nbt);
    // single Newton step (d_ip2_res_hard.c:1348-1919): the caller's ux/pi/lam/t already hold the start
    // iterate (d_init_var_mpc_hard_tv_single_newton is a copy, done by the host), no phase 1.
    const bool sn = a.single_newton != 0;
    if (!sn) init_var(io, bt, dv, ux, pi, lam, t, a.mu0, a.warm_start);
    for (int i = l; i < (N + 1) * V16; i += 64) w.dpi[i] = 0.0;

    double mu = a.mu0, alpha = 1.0, sigma = 0.0;
    const double mu_tol_low = a.mu_tol < 1e-5 ? 1e-5 : a.mu_tol;

    // ------------------------------ phase 1 (d_ip2_res_hard.c:498-718) ------------------------------
    while (!sn && kk < a.k_max && mu > mu_tol_low && alpha >= a.alpha_min) {
        HK_FOR_BOX(io, k, {  // d_update_hessian_mpc_hard_tv, sigma_mu = 0
            const double til = 1.0 / t[lo], tiu = 1.0 / t[up];
            const double ltl = lam[lo] * til, ltu = lam[up] * tiu;
            const double dll = til * 0.0, dlu = tiu * 0.0;
            w.t_inv[lo] = til;
            w.t_inv[up] = tiu;
            w.lamt[lo] = ltl;
            w.lamt[up] = ltu;
            w.dlam[lo] = dll;
            w.dlam[up] = dlu;
            w.Qx[k * V16 + slot] = ltl + ltu;
            w.qx[k * V16 + slot] = lam[up] - ltu * dv[up] + dlu - lam[lo] - ltl * dv[lo] - dll;
        });
        wsync();
        ric_backward<true>(io, &sm, 0, nullptr, 0, nullptr, 1, w.Qx, w.qx, 1, w.Pb);
        wsync();
        ric_forward_sv(io, &sm, 0, nullptr, w.dux, a.compute_mult, w.dpi);
        wsync();
        double al = 1.0;
        HK_FOR_BOX(io, k, {  // d_compute_alpha_mpc_hard_tv
            const int v = bt.slotvar[k * 16 + slot];
            const double x = w.dux[k * V16 + v];
            const double dtl = x - dv[lo] - t[lo], dtu = -x + dv[up] - t[up];
            const double dll = w.dlam[lo] - (w.lamt[lo] * dtl + lam[lo]);
            const double dlu = w.dlam[up] - (w.lamt[up] * dtu + lam[up]);
            w.dt[lo] = dtl;
            w.dt[up] = dtu;
            w.dlam[lo] = dll;
            w.dlam[up] = dlu;
            alpha_rule(al, lam[lo], dll, 0, 0);
            alpha_rule(al, lam[up], dlu, 0, 0);
            alpha_rule(al, t[lo], dtl, 0, 0);
            alpha_rule(al, t[up], dtu, 0, 0);
        });
        al = wave_min(al);
        wsync();
        if (l == 0) {
            stat[5 * kk] = sigma;
            stat[5 * kk + 1] = al;
        }
        alpha = al * 0.995;
        double ms = 0.0;
        HK_FOR_BOX(io, k, {  // d_compute_mu_mpc_hard_tv
            ms += (lam[lo] + alpha * w.dlam[lo]) * (t[lo] + alpha * w.dt[lo]) +
                  (lam[up] + alpha * w.dlam[up]) * (t[up] + alpha * w.dt[up]);
        });
        const double mu_aff = wave_sum(ms) * mu_scal;
        if (l == 0) stat[5 * kk + 2] = mu_aff;
        sigma = mu_aff / mu;
        sigma = sigma * sigma * sigma;
        const double smu = sigma * mu;
        HK_FOR_BOX(io, k, {  // d_update_gradient_mpc_hard_tv
            const double dll = w.t_inv[lo] * (smu - w.dlam[lo] * w.dt[lo]);
            const double dlu = w.t_inv[up] * (smu - w.dlam[up] * w.dt[up]);
            w.dlam[lo] = dll;
            w.dlam[up] = dlu;
            w.qx[k * V16 + slot] += dlu - dll;
        });
        wsync();
        ric_trs(io, &sm, nullptr, nullptr, 1, w.qx, w.dux, a.compute_mult, w.dpi, 0, w.Pb);
        wsync();
        al = 1.0;
        HK_FOR_BOX(io, k, {
            const int v = bt.slotvar[k * 16 + slot];
            const double x = w.dux[k * V16 + v];
            const double dtl = x - dv[lo] - t[lo], dtu = -x + dv[up] - t[up];
            const double dll = w.dlam[lo] - (w.lamt[lo] * dtl + lam[lo]);
            const double dlu = w.dlam[up] - (w.lamt[up] * dtu + lam[up]);
            w.dt[lo] = dtl;
            w.dt[up] = dtu;
            w.dlam[lo] = dll;
            w.dlam[up] = dlu;
            alpha_rule(al, lam[lo], dll, 0, 0);
            alpha_rule(al, lam[up], dlu, 0, 0);
            alpha_rule(al, t[lo], dtl, 0, 0);
            alpha_rule(al, t[up], dtu, 0, 0);
        });
        al = wave_min(al);
        wsync();
        if (l == 0) {
            stat[5 * kk] = sigma;
            stat[5 * kk + 3] = al;
        }
        alpha = al * 0.995;
        // backup + d_update_var_mpc_hard_tv (phase-1 dux/dpi are full iterates)
        for (int k = 0; k <= N; k++) {
            const StageInfo si = load_stage(io.st, k);
            if (l < si.nu + si.nx) {
                const int i = k * V16 + l;
                const double x = ux[i];
                w.ux_bkp[i] = x;
                ux[i] = x + alpha * (w.dux[i] - x);
            }
            if (k < N && l < si.nx1) {
                const int i = k * V16 + l;
                const double y = pi[i];
                w.pi_bkp[i] = y;
                pi[i] = y + alpha * (w.dpi[i] - y);
            }
        }
        ms = 0.0;
        HK_FOR_BOX(io, k, {
            w.lam_bkp[lo] = lam[lo];
            w.lam_bkp[up] = lam[up];
            w.t_bkp[lo] = t[lo];
            w.t_bkp[up] = t[up];
            const double ll = lam[lo] + alpha * w.dlam[lo], lu = lam[up] + alpha * w.dlam[up];
            const double tl = t[lo] + alpha * w.dt[lo], tu = t[up] + alpha * w.dt[up];
            lam[lo] = ll;
            lam[up] = lu;
            t[lo] = tl;
            t[up] = tu;
            ms += ll * tl + lu * tu;
        });
        mu = wave_sum(ms) * mu_scal;
        if (l == 0) stat[5 * kk + 4] = mu;
        kk++;
        wsync();
    }

    // ------------------------------ phase 2 (d_ip2_res_hard.c:756-1273) ------------------------------
    residuals(io, bt, &sm, nullptr, nullptr, ux, pi, dv, lam, t, w.res_q, w.res_b, w.res_d, w.res_m, mu);
    wsync();
    const int kk_p2 = kk;  // first phase-2 iteration (diagnostic stamps only)
    (void)kk_p2;
    while (kk < a.k_max && (sn || (mu > a.mu_tol && alpha >= a.alpha_min))) {
        HK_STAMP(32, kk == kk_p2 ? 50 : -1);
        HK_FOR_BOX(io, k, {  // d_update_hessian_gradient_res_mpc_hard_tv
            const double til = 1.0 / t[lo], tiu = 1.0 / t[up];
            w.t_inv[lo] = til;
            w.t_inv[up] = tiu;
            w.Qx[k * V16 + slot] = til * lam[lo] + tiu * lam[up];
            w.qx[k * V16 + slot] = til * (w.res_m[lo] - lam[lo] * w.res_d[lo]) -
                                   tiu * (w.res_m[up] + lam[up] * w.res_d[up]);
        });
        wsync();
        HK_STAMP(33, kk == kk_p2 ? 50 : -1);
        // the single-Newton variant factorises with the data's own b/q rows (d_ip2_res_hard.c:1700-1760)
        ric_backward<true>(io, &sm, !sn, w.res_b, !sn, w.res_q, 1, w.Qx, w.qx, 1, w.Pb);
        wsync();
        HK_STAMP(34, kk == kk_p2 ? 50 : -1);
        ric_forward_sv(io, &sm, !sn, w.res_b, w.dux, a.compute_mult, w.dpi);
        wsync();
        HK_STAMP(35, kk == kk_p2 ? 50 : -1);
        double al = 1.0;
        HK_FOR_BOX(io, k, {  // d_compute_alpha_res_mpc_hard_tv
            const int v = bt.slotvar[k * 16 + slot];
            const double x = w.dux[k * V16 + v];
            const double dtl = x - w.res_d[lo], dtu = -x + w.res_d[up];
            const double dll = -w.t_inv[lo] * (lam[lo] * dtl + w.res_m[lo]);
            const double dlu = -w.t_inv[up] * (lam[up] * dtu + w.res_m[up]);
            w.dt[lo] = dtl;
            w.dt[up] = dtu;
            w.dlam[lo] = dll;
            w.dlam[up] = dlu;
            alpha_rule(al, lam[lo], dll, 0, 0);
            alpha_rule(al, lam[up], dlu, 0, 0);
            alpha_rule(al, t[lo], dtl, 0, 0);
            alpha_rule(al, t[up], dtu, 0, 0);
        });
        al = wave_min(al);
        wsync();
        if (l == 0) {
            stat[5 * kk] = sigma;
            stat[5 * kk + 1] = al;
        }
        alpha = al * 0.995;
        HK_STAMP(36, kk == kk_p2 ? 50 : -1);
        double ms = 0.0;
        HK_FOR_BOX(io, k, {  // d_compute_mu_res_mpc_hard_tv
            ms += (lam[lo] + alpha * w.dlam[lo]) * (t[lo] + alpha * w.dt[lo]) +
                  (lam[up] + alpha * w.dlam[up]) * (t[up] + alpha * w.dt[up]);
        });
        const double mu_aff = wave_sum(ms) * mu_scal;
        if (l == 0) stat[5 * kk + 2] = mu_aff;
        HK_STAMP(37, kk == kk_p2 ? 50 : -1);
        double smu = a.mu0;  // single Newton: sigma*mu is supplied by the caller as mu0 (:1788-1790)
        if (!sn) {
            sigma = mu_aff / mu;
            sigma = sigma * sigma * sigma;
            smu = sigma * mu;
        }
        HK_FOR_BOX(io, k, {  // centering correction + d_update_gradient_res_mpc_hard_tv
            const double rml = w.res_m[lo] + (w.dt[lo] * w.dlam[lo] - smu);
            const double rmu = w.res_m[up] + (w.dt[up] * w.dlam[up] - smu);
            w.res_m[lo] = rml;
            w.res_m[up] = rmu;
            w.qx[k * V16 + slot] = w.t_inv[lo] * (rml - lam[lo] * w.res_d[lo]) -
                                   w.t_inv[up] * (rmu + lam[up] * w.res_d[up]);
        });
        wsync();
        HK_STAMP(38, kk == kk_p2 ? 50 : -1);
        ric_trs(io, &sm, w.res_b, w.res_q, 1, w.qx, w.dux, a.compute_mult, w.dpi, 0, w.Pb);
        wsync();
        HK_STAMP(39, kk == kk_p2 ? 50 : -1);
        al = 1.0;
        HK_FOR_BOX(io, k, {
            const int v = bt.slotvar[k * 16 + slot];
            const double x = w.dux[k * V16 + v];
            const double dtl = x - w.res_d[lo], dtu = -x + w.res_d[up];
            const double dll = -w.t_inv[lo] * (lam[lo] * dtl + w.res_m[lo]);
            const double dlu = -w.t_inv[up] * (lam[up] * dtu + w.res_m[up]);
            w.dt[lo] = dtl;
            w.dt[up] = dtu;
            w.dlam[lo] = dll;
            w.dlam[up] = dlu;
            alpha_rule(al, lam[lo], dll, 0, 0);
            alpha_rule(al, lam[up], dlu, 0, 0);
            alpha_rule(al, t[lo], dtl, 0, 0);
            alpha_rule(al, t[up], dtu, 0, 0);
        });
        al = wave_min(al);
        wsync();
        if (l == 0) {
            stat[5 * kk] = sigma;
            stat[5 * kk + 3] = al;
        }
        alpha = al * 0.995;
        HK_STAMP(40, kk == kk_p2 ? 50 : -1);
        // d_backup_update_var_res_mpc_hard_tv (phase-2 dux/dpi are deltas)
        for (int k = 0; k <= N; k++) {
            const StageInfo si = load_stage(io.st, k);
            if (l < si.nu + si.nx) {
                const int i = k * V16 + l;
                const double x = ux[i];
                w.ux_bkp[i] = x;
                ux[i] = x + alpha * w.dux[i];
            }
            if (k < N && l < si.nx1) {
                const int i = k * V16 + l;
                const double y = pi[i];
                w.pi_bkp[i] = y;
                pi[i] = y + alpha * w.dpi[i];
            }
        }
        HK_FOR_BOX(io, k, {
            w.lam_bkp[lo] = lam[lo];
            w.lam_bkp[up] = lam[up];
            w.t_bkp[lo] = t[lo];
            w.t_bkp[up] = t[up];
            lam[lo] += alpha * w.dlam[lo];
            lam[up] += alpha * w.dlam[up];
            t[lo] += alpha * w.dt[lo];
            t[up] += alpha * w.dt[up];
        });
        wsync();
        HK_STAMP(41, kk == kk_p2 ? 50 : -1);
        residuals(io, bt, &sm, nullptr, nullptr, ux, pi, dv, lam, t, w.res_q, w.res_b, w.res_d, w.res_m, mu);
        wsync();
        if (l == 0) stat[5 * kk + 4] = mu;
        HK_STAMP(42, kk == kk_p2 ? 50 : -1);
        kk++;
    }
    if (!sn && mu <= a.mu_tol)
        ret = 0;
    else if (kk >= a.k_max)
        ret = 1;
    else if (alpha < a.alpha_min)
        ret = 2;
    else
        ret = -1;
    if (l == 0) {
        a.kk[p] = kk;
        a.ret[p] = ret;
    }
}

// ------------------------------------------------------------------------------------------------
// d_kkt_solve_new_rhs_res_mpc_hard_tv: re-solve with the factor + iterate persisted in ws.
// vb/vq hold the new b (state order) / q (variable order).
// ------------------------------------------------------------------------------------------------
extern "C" __global__ __launch_bounds__(64) void hk_kkt_new_rhs(KArgs a) {
    const LdsTabs T = lds_tables(a);
    Scratch& sm = *T.sm;
    const int p = blockIdx.x + a.p0;
    if (p >= a.nprob) return;
    const int N = a.N;
    Ws w = carve(a.ws + (long)p * a.sW, N);
    RicIO io = make_io(a, T, p, w.F);
    BoxTab bt{T.tileslot, T.slotvar};
    const long o16 = (long)p * a.sV16, o32 = (long)p * a.sV32;
    double* ux = a.ux + o16;
    double* pi = a.pi + o16;
    double* lam = a.lam + o32;
    double* t = a.t + o32;
    const double* dv = a.d + o32;
    const int l = lane_id();
    for (int i = l; i < (N + 1) * V16; i += 64) {
        ux[i] = w.ux_bkp[i];
        pi[i] = w.pi_bkp[i];
    }
    for (int i = l; i < (N + 1) * V32; i += 64) {
        t[i] = w.t_bkp[i];
        lam[i] = w.lam_bkp[i];
    }
    wsync();
    double mu = 0.0;
    residuals(io, bt, &sm, a.vb + o16, a.vq + o16, ux, pi, dv, lam, t, w.res_q, w.res_b, w.res_d, w.res_m, mu);
    wsync();
    HK_FOR_BOX(io, k, {
        w.qx[k * V16 + slot] = w.t_inv[lo] * (w.res_m[lo] - lam[lo] * w.res_d[lo]) -
                               w.t_inv[up] * (w.res_m[up] + lam[up] * w.res_d[up]);
    });
    wsync();
    ric_trs(io, &sm, w.res_b, w.res_q, 1, w.qx, w.dux, a.compute_mult, w.dpi, 1, w.Pb);
    wsync();
    HK_FOR_BOX(io, k, {  // d_compute_dt_dlam_res + d_update_var_res (alpha = 1)
        const int v = bt.slotvar[k * 16 + slot];
        const double x = w.dux[k * V16 + v];
        const double dtl = x - w.res_d[lo], dtu = -x + w.res_d[up];
        const double dll = -w.t_inv[lo] * (lam[lo] * dtl + w.res_m[lo]);
        const double dlu = -w.t_inv[up] * (lam[up] * dtu + w.res_m[up]);
        w.dt[lo] = dtl;
        w.dt[up] = dtu;
        w.dlam[lo] = dll;
        w.dlam[up] = dlu;
    });
    wsync();
    for (int k = 0; k <= N; k++) {
        const StageInfo si = load_stage(io.st, k);
        if (l < si.nu + si.nx) ux[k * V16 + l] += 1.0 * w.dux[k * V16 + l];
        if (k < N && l < si.nx1) pi[k * V16 + l] += 1.0 * w.dpi[k * V16 + l];
    }
    HK_FOR_BOX(io, k, {
        lam[lo] += 1.0 * w.dlam[lo];
        lam[up] += 1.0 * w.dlam[up];
        t[lo] += 1.0 * w.dt[lo];
        t[up] += 1.0 * w.dt[up];
    });
}

// ------------------------------------------------------------------------------------------------
// Host launch helpers (called from the C-ABI translation unit).
// ------------------------------------------------------------------------------------------------
extern "C" int hk_launch(int which, const KArgs* a, int count, hipStream_t stream) {
    if (count <= 0) return 0;
#ifdef HK_STAMPS
    if (a->dbg) {
        unsigned long long* p = a->dbg;
        int st = 50;
        (void)hipMemcpyToSymbol(HIP_SYMBOL(g_dbg), &p, sizeof(p));
        (void)hipMemcpyToSymbol(HIP_SYMBOL(g_dbg_stage), &st, sizeof(st));
    }
#endif
    dim3 grid(count), block(64);
    const size_t lds = sizeof(Scratch) + (size_t)(a->N + 1) * (sizeof(StageInfo) + 32);
    switch (which) {
        case 0: hipLaunchKernelGGL(hk_ric_sv, grid, block, lds, stream, *a); break;
        case 1: hipLaunchKernelGGL(hk_ric_trf, grid, block, lds, stream, *a); break;
        case 2: hipLaunchKernelGGL(hk_ric_trs, grid, block, lds, stream, *a); break;
        case 3: hipLaunchKernelGGL(hk_res, grid, block, lds, stream, *a); break;
        case 4: hipLaunchKernelGGL(hk_ipm, grid, block, lds, stream, *a); break;
        case 5: hipLaunchKernelGGL(hk_kkt_new_rhs, grid, block, lds, stream, *a); break;
        default: return -1;
    }
    return (int)hipGetLastError();
}
