// hk_ipm.h -- residuals and interior-point vector passes, one problem per wavefront (gfx950).
//
// Restates mpc_solvers/c99/d_res_ip_res_hard.c:39-319 (KKT residuals) and the vector kernels of
// mpc_solvers/c99/d_aux_ip_hard_lib4.c (box constraints; ng == 0 on the GPU path).  Box-slot vectors
// use the reference's per-stage [lb (pnb) | ub (pnb)] layout inside a V32 stride.
//
// Every pass here is latency-tolerant: the residual pass is a stage loop with the same one-stage-ahead
// register prefetch as the Riccati passes, and the purely element-wise passes (mu_aff, the phase-1
// update) load a whole chunk of stages before computing any of it.  A pass never waits for a global
// load right after issuing it (per-stage load -> use -> store chains cost a full memory round trip
// per stage, which dominated the IPM before).
#pragma once
#include "hk_riccati.h"

namespace hk {

struct BoxTab {
    const signed char* tileslot;  // (N+1)*16 box slot of tile t or -1
    const signed char* slotvar;   // (N+1)*16 variable index of box slot l
};

// Iterate (stage k, slot c) pairs four stages per pass (one-off passes only: init, KKT re-solve).
#define HK_FOR_BOX(io, KV, ...)                                                       \
    for (int j4_ = 0; j4_ <= (io).N; j4_ += 4) {                                       \
        const int KV = j4_ + (lane_id() >> 4);                                         \
        const int slot = lane_id() & 15;                                               \
        if (KV <= (io).N) {                                                            \
            const int nb_ = (io).st[KV].nb, pnb_ = (io).st[KV].pnb;                    \
            if (slot < nb_) {                                                          \
                const int lo = KV * V32 + slot, up = KV * V32 + pnb_ + slot;           \
                (void)lo; (void)up;                                                    \
                __VA_ARGS__                                                            \
            }                                                                          \
        }                                                                              \
    }

// Iterate (stage k, general constraint l) pairs four stages per pass (one-off passes only).
#define HK_FOR_GEN(io, KV, ...)                                                       \
    for (int j4_ = 0; j4_ <= (io).N; j4_ += 4) {                                       \
        const int KV = j4_ + (lane_id() >> 4);                                         \
        const int gl_ = lane_id() & 15;                                                \
        if (KV <= (io).N) {                                                            \
            const int ng_ = (io).st[KV].ng, pnb_ = (io).st[KV].pnb;                    \
            if (gl_ < ng_) {                                                           \
                const int png_ = (ng_ + 3) & ~3;                                       \
                const int lo = KV * V32 + 2 * pnb_ + gl_, up = lo + png_;               \
                const int s16 = KV * V16 + pnb_ + gl_;                                 \
                (void)lo; (void)up; (void)s16;                                         \
                __VA_ARGS__                                                            \
            }                                                                          \
        }                                                                              \
    }

// ------------------------------------------------------------------------------------------------
// Element-wise box passes over quads of stages: lane (g, c) handles stage 4q+g, slot c.  CH quads
// (4*CH stages) are loaded before any is used.
// ------------------------------------------------------------------------------------------------
// Lane c of row group g owns constraint pair c of stage 4q+g: box c (c < nb) or general constraint
// c - nb (nb <= c < nb + ng), with its lower / upper slot in the [lb | ub | lg | ug] layout.
struct QuadLane {
    int lo, up;
    bool ok;
    bool box;  // a box pair (its variable is slotvar[c])
};

__device__ __forceinline__ QuadLane quad_lane(const RicIO& io, int q) {
    const int l = lane_id(), g = l >> 4, c = l & 15;
    const int k = 4 * q + g;
    const bool kv = k <= io.N;
    const int kc = kv ? k : io.N;
    const StageInfo& s = io.st[kc];
    QuadLane b;
    b.ok = kv && c < s.nb + s.ng;
    b.box = c < s.nb;
    const int png = (s.ng + 3) & ~3;
    b.lo = kc * V32 + (b.box ? c : 2 * s.pnb + (c - s.nb));
    b.up = b.lo + (b.box ? s.pnb : png);
    return b;
}

// Multi-wave split of the element-wise update passes (the one-problem-per-workgroup solo kernel, hk_mw.h): wave w
// of NW takes the quad chunks w, w + NW, ...; each quad's per-lane r_m contribution goes to red[q * 64 + lane] and
// every wave then sums all of them in quad order -- the single-wave loop's order, so mu is bitwise the same.
typedef __attribute__((address_space(3))) double lds_f64;  // an LDS pointer that stays one through memory

struct MwSplit {
    int w;
    lds_f64* red;  // round_up(nq, CH) x 64 doubles
};

template <int NW>
__device__ __forceinline__ double mw_quad_sum(const MwSplit& ms, int nq_pad, double ms_local) {
    if constexpr (NW == 1) {
        return ms_local;
    } else {
        const int l = lane_id();
        __syncthreads();
        double m = 0.0;
        for (int q = 0; q < nq_pad; q++) m += ms.red[q * 64 + l];
        __syncthreads();  // red is written again by the next pass
        return m;
    }
}

// d_compute_mu_[res_]mpc_hard_tv: mu_aff = sum (lam + alpha dlam)(t + alpha dt) * mu_scal
template <int CH>
__device__ double mu_aff_pass(const RicIO& io, const BoxCtx& bc, double alpha, double mu_scal) {
    const int nq = (io.N + 4) / 4;
    double ms = 0.0;
    for (int q0 = 0; q0 < nq; q0 += CH) {
        double v[CH][8];
#pragma unroll
        for (int j = 0; j < CH; j++) {
            const QuadLane b = quad_lane(io, q0 + j);
            v[j][0] = gld(bc.lam, b.lo, b.ok);
            v[j][1] = gld(bc.dlam, b.lo, b.ok);
            v[j][2] = gld(bc.t, b.lo, b.ok);
            v[j][3] = gld(bc.dt, b.lo, b.ok);
            v[j][4] = gld(bc.lam, b.up, b.ok);
            v[j][5] = gld(bc.dlam, b.up, b.ok);
            v[j][6] = gld(bc.t, b.up, b.ok);
            v[j][7] = gld(bc.dt, b.up, b.ok);
        }
#pragma unroll
        for (int j = 0; j < CH; j++)
            ms += (v[j][0] + alpha * v[j][1]) * (v[j][2] + alpha * v[j][3]) +
                  (v[j][4] + alpha * v[j][5]) * (v[j][6] + alpha * v[j][7]);
    }
    return wave_sum(ms) * mu_scal;
}

// Phase-1 update (d_update_var_mpc_hard_tv :618-711 with the backups of :721-732): the phase-1 dux/dpi
// are full iterates, so ux += alpha (dux - ux).  Returns mu = sum lam t * mu_scal of the new iterate.
template <int CH, int NW = 1>
__device__ double update_p1_pass(const RicIO& io, const BoxCtx& bc, double alpha, double mu_scal, double* ux,
                                 double* pi, const double* dux, const double* dpi, double* ux_bkp, double* pi_bkp,
                                 double* lam_bkp, double* t_bkp, const MwSplit& mws = MwSplit{0, nullptr}) {
    const int l = lane_id(), g = l >> 4, c = l & 15;
    const int nq = (io.N + 4) / 4;
    double ms = 0.0;
    for (int q0 = NW > 1 ? mws.w * CH : 0; q0 < nq; q0 += NW * CH) {
        double v[CH][12];
        int i16[CH];
        bool oku[CH], okp[CH];
        QuadLane bl[CH];
#pragma unroll
        for (int j = 0; j < CH; j++) {
            const int k = 4 * (q0 + j) + g;
            const bool kv = k <= io.N;
            const StageInfo& s = io.st[kv ? k : io.N];
            i16[j] = (kv ? k : io.N) * V16 + c;
            oku[j] = kv && c < s.nu + s.nx;
            okp[j] = kv && k < io.N && c < s.nx1;
            bl[j] = quad_lane(io, q0 + j);
            const QuadLane& b = bl[j];
            v[j][0] = gld(ux, i16[j], oku[j]);
            v[j][1] = gld(dux, i16[j], oku[j]);
            v[j][2] = gld(pi, i16[j], okp[j]);
            v[j][3] = gld(dpi, i16[j], okp[j]);
            v[j][4] = gld(bc.lam, b.lo, b.ok);
            v[j][5] = gld(bc.dlam, b.lo, b.ok);
            v[j][6] = gld(bc.t, b.lo, b.ok);
            v[j][7] = gld(bc.dt, b.lo, b.ok);
            v[j][8] = gld(bc.lam, b.up, b.ok);
            v[j][9] = gld(bc.dlam, b.up, b.ok);
            v[j][10] = gld(bc.t, b.up, b.ok);
            v[j][11] = gld(bc.dt, b.up, b.ok);
        }
#pragma unroll
        for (int j = 0; j < CH; j++) {
            const QuadLane& b = bl[j];
            const double x = v[j][0], y = v[j][2];
            gst(ux_bkp, i16[j], x, oku[j]);
            gst(ux, i16[j], x + alpha * (v[j][1] - x), oku[j]);
            gst(pi_bkp, i16[j], y, okp[j]);
            gst(pi, i16[j], y + alpha * (v[j][3] - y), okp[j]);
            gst(lam_bkp, b.lo, v[j][4], b.ok);
            gst(lam_bkp, b.up, v[j][8], b.ok);
            gst(t_bkp, b.lo, v[j][6], b.ok);
            gst(t_bkp, b.up, v[j][10], b.ok);
            const double ll = v[j][4] + alpha * v[j][5], lu = v[j][8] + alpha * v[j][9];
            const double tl = v[j][6] + alpha * v[j][7], tu = v[j][10] + alpha * v[j][11];
            gst(bc.lam, b.lo, ll, b.ok);
            gst(bc.lam, b.up, lu, b.ok);
            gst(bc.t, b.lo, tl, b.ok);
            gst(bc.t, b.up, tu, b.ok);
            const double mc = b.ok ? ll * tl + lu * tu : 0.0;
            if constexpr (NW > 1)
                mws.red[(q0 + j) * 64 + l] = mc;
            else
                ms += mc;
        }
    }
    ms = mw_quad_sum<NW>(mws, (nq + CH - 1) / CH * CH, ms);
    return wave_sum(ms) * mu_scal;
}

// Phase-2 update (d_update_var_res_mpc_hard_tv with the backups of d_backup_update_var_res_mpc_hard_tv)
// and the element-wise residuals of the new iterate, r_d = [lb - x + t_lo | ub - x - t_up], r_m = lam t;
// returns mu = sum r_m * mu_scal.  With UPD false it only computes r_d, r_m and mu of the current
// iterate (phase-2 start).  r_q and r_b, the residuals that need the stage matrices, are computed by
// the next factorisation pass (BX_P2R).  The box variable's x is recomputed from (ux, dux) in the
// slot lane with the same arithmetic as in its own lane.
// BKP = false (the public queue API, whose per-slot workspace never feeds a KKT re-solve): the iterate
// backups and r_m, which only hk_kkt_new_rhs (and general constraints) read, are not written.
template <int CH, bool UPD, bool BKP = true, int NW = 1>
__device__ double update_p2_pass(const RicIO& io, const BoxCtx& bc, const signed char* slotvar, double alpha,
                                 double mu_scal, double* ux, double* pi, const double* dux, const double* dpi,
                                 double* ux_bkp, double* pi_bkp, double* lam_bkp, double* t_bkp, double* res_d,
                                 double* res_m, const MwSplit& mws = MwSplit{0, nullptr}) {
    const int l = lane_id(), g = l >> 4, c = l & 15;
    const int nq = (io.N + 4) / 4;
    double ms = 0.0;
    for (int q0 = NW > 1 ? mws.w * CH : 0; q0 < nq; q0 += NW * CH) {
        double v[CH][16];
        int i16[CH], iv[CH];
        bool oku[CH], okp[CH];
        QuadLane bl[CH];
#pragma unroll
        for (int j = 0; j < CH; j++) {
            const int k = 4 * (q0 + j) + g;
            const bool kv = k <= io.N;
            const int kc = kv ? k : io.N;
            const StageInfo& s = io.st[kc];
            i16[j] = kc * V16 + c;
            oku[j] = kv && c < s.nu + s.nx;
            okp[j] = kv && k < io.N && c < s.nx1;
            bl[j] = quad_lane(io, q0 + j);
            const QuadLane& b = bl[j];
            iv[j] = kc * V16 + ((b.ok && b.box) ? slotvar[kc * 16 + c] : 0);
            v[j][0] = UPD ? gld(ux, i16[j], oku[j]) : 0.0;
            v[j][1] = UPD ? gld(dux, i16[j], oku[j]) : 0.0;
            v[j][2] = UPD ? gld(pi, i16[j], okp[j]) : 0.0;
            v[j][3] = UPD ? gld(dpi, i16[j], okp[j]) : 0.0;
            v[j][4] = gld(bc.lam, b.lo, b.ok);
            v[j][5] = UPD ? gld(bc.dlam, b.lo, b.ok) : 0.0;
            v[j][6] = gld(bc.t, b.lo, b.ok);
            v[j][7] = UPD ? gld(bc.dt, b.lo, b.ok) : 0.0;
            v[j][8] = gld(bc.lam, b.up, b.ok);
            v[j][9] = UPD ? gld(bc.dlam, b.up, b.ok) : 0.0;
            v[j][10] = gld(bc.t, b.up, b.ok);
            v[j][11] = UPD ? gld(bc.dt, b.up, b.ok) : 0.0;
            v[j][12] = gld(ux, iv[j], b.ok && b.box);
            v[j][13] = UPD ? gld(dux, iv[j], b.ok && b.box) : 0.0;
            v[j][14] = gld(bc.d, b.lo, b.ok);
            v[j][15] = gld(bc.d, b.up, b.ok);
        }
#pragma unroll
        for (int j = 0; j < CH; j++) {
            const QuadLane& b = bl[j];
            if (UPD) {
                if (BKP) gst(ux_bkp, i16[j], v[j][0], oku[j]);
                gst(ux, i16[j], v[j][0] + alpha * v[j][1], oku[j]);
                if (BKP) gst(pi_bkp, i16[j], v[j][2], okp[j]);
                gst(pi, i16[j], v[j][2] + alpha * v[j][3], okp[j]);
                if (BKP) {
                    gst(lam_bkp, b.lo, v[j][4], b.ok);
                    gst(lam_bkp, b.up, v[j][8], b.ok);
                    gst(t_bkp, b.lo, v[j][6], b.ok);
                    gst(t_bkp, b.up, v[j][10], b.ok);
                }
            }
            const double ll = UPD ? v[j][4] + alpha * v[j][5] : v[j][4];
            const double lu = UPD ? v[j][8] + alpha * v[j][9] : v[j][8];
            const double tl = UPD ? v[j][6] + alpha * v[j][7] : v[j][6];
            const double tu = UPD ? v[j][10] + alpha * v[j][11] : v[j][10];
            const double x = UPD ? v[j][12] + alpha * v[j][13] : v[j][12];
            if (UPD) {
                gst(bc.lam, b.lo, ll, b.ok);
                gst(bc.lam, b.up, lu, b.ok);
                gst(bc.t, b.lo, tl, b.ok);
                gst(bc.t, b.up, tu, b.ok);
            }
            const double rml = ll * tl, rmu = lu * tu;
            // r_d of the general pairs needs D x: the next factorisation forms it (gen_hessian)
            gst(res_d, b.lo, v[j][14] - x + tl, b.ok && b.box);
            gst(res_d, b.up, v[j][15] - x - tu, b.ok && b.box);
            // r_m = lam t is re-formed at use by every phase-2 pass (and the corrector stores its own centred
            // r_m before its forward reads it): only the KKT re-solve and the general-constraint halves load
            // this store, and the queue API has neither (BKP = false; layout_apply refuses ng > 0)
            if (BKP) {
                gst(res_m, b.lo, rml, b.ok);
                gst(res_m, b.up, rmu, b.ok);
            }
            const double mc = b.ok ? rml + rmu : 0.0;
            if constexpr (NW > 1)
                mws.red[(q0 + j) * 64 + l] = mc;
            else
                ms += mc;
        }
    }
    ms = mw_quad_sum<NW>(mws, (nq + CH - 1) / CH * CH, ms);
    return wave_sum(ms) * mu_scal;
}

// ------------------------------------------------------------------------------------------------
// d_res_res_mpc_hard_tv as a prefetched stage pass.  With UPD it first applies the phase-2 update
// x += alpha dx to (ux, pi, lam, t) and writes the backups (d_backup_update_var_res_mpc_hard_tv
// :1382), then computes the residuals of the NEW iterate:
//   r_q = q - [0; pi_{k-1}] + (lam_up - lam_lo) + RSQ ux + BAbt pi,   r_b = b - x_{k+1} + BAbt' ux,
//   r_d = [lb - x + t_lo | ub - x - t_up],   r_m = lam t,   mu = sum r_m / (2 sum nb).
// b: state order (the BAbt augmented row if bsrc == nullptr), q: variable order (RSQrq row if null).
// ------------------------------------------------------------------------------------------------
struct ResIO {
    const double *bsrc, *qsrc;
    double *ux, *pi;
    const double *dux, *dpi;   // UPD
    double *ux_bkp, *pi_bkp;   // UPD
    double *lam_bkp, *t_bkp;   // UPD
    double *rq, *rb, *rd, *rm; // outputs (V16 / V16 / V32 / V32)
    double alpha;
};

template <bool UPD>
struct ResFrag {
    d4 Mi;                 // RSQrq tile (mirrored lower part)
    double q;              // q[var(c)]
    d4 bop;                // BAbt_k[var(c)][g+4r-xo1]      (BAbt pi)
    d4 bt;                 // BAbt_k[var(g+4r)][c-xo1]      (BAbt' ux)
    double bval;           // b_k[c-xo1]
    double uc, duc;        // ux_k[var(c)]
    double ur[4], dur[4];  // ux_k[var(g+4r)]
    double pr[4], dpr[4];  // pi_k[g+4r-xo1]
    double pc, dpc;        // pi_k[c-xo1]
    double x1, dx1;        // ux_{k+1}[nu1 + c-xo1]
    double bx[10];         // d lo/up, lam lo/up, t lo/up, dlam lo/up, dt lo/up
    BoxLane bl;
};

template <bool UPD, class SH>
__device__ __forceinline__ void res_fetch(const RicIO& io, const SH& si, const BoxCtx& bc, const ResIO& ro, int k,
                                          ResFrag<UPD>& f) {
    const int l = lane_id(), g = l >> 4, c = l & 15;
    const int nu = si.nu, nx = si.nx, xo = si.xo, nux = nu + nx;
    const double* R = stage_R(io, si);
    const int vc = tile_var(c, nu, nx, xo);
    const bool live = SH::fixed || k < io.N;
#pragma unroll
    for (int r = 0; r < 4; r++) {
        const int vi = tile_var(g + 4 * r, nu, nx, xo);
        const int hi = vi > vc ? vi : vc, lo = vi > vc ? vc : vi;
        f.Mi[r] = ldsel(R, lib4_idx(si.sdR, hi, lo), vi >= 0 && vc >= 0);
        f.ur[r] = ldsel(ro.ux, k * V16 + vi, vi >= 0);
        f.dur[r] = UPD ? ldsel(ro.dux, k * V16 + vi, vi >= 0) : 0.0;
    }
    f.q = ro.qsrc ? ldsel(ro.qsrc, k * V16 + vc, vc >= 0) : ldsel(R, lib4_idx(si.sdR, nux, vc), vc >= 0);
    f.uc = ldsel(ro.ux, k * V16 + vc, vc >= 0);
    f.duc = UPD ? ldsel(ro.dux, k * V16 + vc, vc >= 0) : 0.0;
    const double* Bk = stage_B(io, si);
    const int nx1 = si.nx1, xo1 = si.xo1;
    const int s = c - xo1;
    const bool oks = live && s >= 0 && s < nx1;
#pragma unroll
    for (int r = 0; r < 4; r++) {
        const int sr = g + 4 * r - xo1;
        const bool okr = live && sr >= 0 && sr < nx1;
        const int vi = tile_var(g + 4 * r, nu, nx, xo);
        f.bop[r] = ldsel(Bk, lib4_idx(si.sdB, vc, sr), okr && vc >= 0);
        f.bt[r] = ldsel(Bk, lib4_idx(si.sdB, vi, s), oks && vi >= 0);
        f.pr[r] = ldsel(ro.pi, k * V16 + sr, okr);
        f.dpr[r] = UPD ? ldsel(ro.dpi, k * V16 + sr, okr) : 0.0;
    }
    f.bval = ro.bsrc ? ldsel(ro.bsrc, k * V16 + s, oks) : ldsel(Bk, lib4_idx(si.sdB, nux, s), oks);
    f.pc = ldsel(ro.pi, k * V16 + s, oks);
    f.dpc = UPD ? ldsel(ro.dpi, k * V16 + s, oks) : 0.0;
    f.x1 = ldsel(ro.ux, (k + 1) * V16 + si.nu1 + s, oks);
    f.dx1 = UPD ? ldsel(ro.dux, (k + 1) * V16 + si.nu1 + s, oks) : 0.0;
    const BoxLane b = box_lane(io.tileslot, si.pnb, k);
    f.bl = b;
    f.bx[0] = ldsel(bc.d, b.lo, b.ok);
    f.bx[1] = ldsel(bc.d, b.up, b.ok);
    f.bx[2] = ldsel(bc.lam, b.lo, b.ok);
    f.bx[3] = ldsel(bc.lam, b.up, b.ok);
    f.bx[4] = ldsel(bc.t, b.lo, b.ok);
    f.bx[5] = ldsel(bc.t, b.up, b.ok);
    f.bx[6] = UPD ? ldsel(bc.dlam, b.lo, b.ok) : 0.0;
    f.bx[7] = UPD ? ldsel(bc.dlam, b.up, b.ok) : 0.0;
    f.bx[8] = UPD ? ldsel(bc.dt, b.lo, b.ok) : 0.0;
    f.bx[9] = UPD ? ldsel(bc.dt, b.up, b.ok) : 0.0;
}

// One residual stage (with the phase-2 update when UPD).  pim1: pi_{k-1} (new) in stage-k tile col
// layout, replaced by pi_k (new) for the next stage; ms: partial sum of r_m.
template <bool UPD, class SH>
__device__ __forceinline__ void res_step(const RicIO& io, const SH& sh, int k, const ResFrag<UPD>& cur,
                                         const BoxCtx& bc, const ResIO& ro, double& pim1, double& ms) {
    const int l = lane_id(), g = l >> 4, c = l & 15;
    const double al = ro.alpha;
    const bool live = SH::fixed || k < io.N;
    const int nu = sh.nu;
    const int vc = tile_var(c, sh.nu, sh.nx, sh.xo);
    const int s = c - sh.xo1;
    const bool oks = live && s >= 0 && s < sh.nx1;
    // updated iterate (UPD) in every layout this stage needs; identical arithmetic per element
    const double ucn = UPD ? cur.uc + al * cur.duc : cur.uc;
    double urn[4], prn[4];
#pragma unroll
    for (int r = 0; r < 4; r++) {
        urn[r] = UPD ? cur.ur[r] + al * cur.dur[r] : cur.ur[r];
        prn[r] = UPD ? cur.pr[r] + al * cur.dpr[r] : cur.pr[r];
    }
    const double pcn = UPD ? cur.pc + al * cur.dpc : cur.pc;
    const double x1n = UPD ? cur.x1 + al * cur.dx1 : cur.x1;
    const BoxLane& b = cur.bl;
    const double lml = UPD ? cur.bx[2] + al * cur.bx[6] : cur.bx[2];
    const double lmu = UPD ? cur.bx[3] + al * cur.bx[7] : cur.bx[3];
    const double tl = UPD ? cur.bx[4] + al * cur.bx[8] : cur.bx[4];
    const double tu = UPD ? cur.bx[5] + al * cur.bx[9] : cur.bx[5];
    const bool st0 = g == 0;
    if (UPD) {
        gst(ro.ux_bkp, k * V16 + vc, cur.uc, st0 && vc >= 0);
        gst(ro.ux, k * V16 + vc, ucn, st0 && vc >= 0);
        gst(ro.pi_bkp, k * V16 + s, cur.pc, st0 && oks);
        gst(ro.pi, k * V16 + s, pcn, st0 && oks);
        gst(ro.lam_bkp, b.lo, cur.bx[2], st0 && b.ok);
        gst(ro.lam_bkp, b.up, cur.bx[3], st0 && b.ok);
        gst(ro.t_bkp, b.lo, cur.bx[4], st0 && b.ok);
        gst(ro.t_bkp, b.up, cur.bx[5], st0 && b.ok);
        gst(bc.lam, b.lo, lml, st0 && b.ok);
        gst(bc.lam, b.up, lmu, st0 && b.ok);
        gst(bc.t, b.lo, tl, st0 && b.ok);
        gst(bc.t, b.up, tu, st0 && b.ok);
    }
    // r_q
    double h = cur.q;
    if (k > 0 && vc >= nu) h -= pim1;
    if (b.ok) h += -lml + lmu;
    double part = 0.0;
#pragma unroll
    for (int r = 0; r < 4; r++) part += cur.Mi[r] * urn[r];
    h += xrow_sum(part);
    double p2 = 0.0, p3 = 0.0;
#pragma unroll
    for (int r = 0; r < 4; r++) {
        p2 += cur.bop[r] * prn[r];
        p3 += cur.bt[r] * urn[r];
    }
    const double bpi = xrow_sum(p2);
    const double atu = xrow_sum(p3);
    if (live) h += bpi;
    gst(ro.rq, k * V16 + vc, h, st0 && vc >= 0);
    // r_b
    gst(ro.rb, k * V16 + s, cur.bval - x1n + atu, st0 && oks);
    // r_d, r_m
    const double x = ucn;
    const double rml = lml * tl, rmu = lmu * tu;
    gst(ro.rd, b.lo, cur.bx[0] - x + tl, st0 && b.ok);
    gst(ro.rd, b.up, cur.bx[1] - x - tu, st0 && b.ok);
    gst(ro.rm, b.lo, rml, st0 && b.ok);
    gst(ro.rm, b.up, rmu, st0 && b.ok);
    ms += (st0 && b.ok) ? rml + rmu : 0.0;
    if constexpr (!SH::fixed) {
        if (sh.ng > 0) {  // general constraints (d_res_ip_res_hard.c:393-416); never on the UPD path
            static_assert(!UPD || SH::fixed, "the update pass handles general slots element-wise");
            const double tq = gen_rq(io, sh, k, bc.lam);
            gst(ro.rq, k * V16 + vc, h + tq, st0 && vc >= 0);
            double dg[4];
            gen_dg(io, sh, dg);
#pragma unroll
            for (int lc = 0; lc < 4; lc++) {
                if (4 * lc >= sh.ng) continue;
                const GenLane q = gen_lane(k, sh.pnb, sh.ng, lc);
                const bool st = q.ok && c == 0;
                const double dx = row_sum16(dg[lc] * x);
                const double tgl = gld(bc.t, q.lo, q.ok), tgu = gld(bc.t, q.up, q.ok);
                const double lgl = gld(bc.lam, q.lo, q.ok), lgu = gld(bc.lam, q.up, q.ok);
                gst(ro.rd, q.lo, gld(bc.d, q.lo, q.ok) - dx + tgl, st);
                gst(ro.rd, q.up, gld(bc.d, q.up, q.ok) - dx - tgu, st);
                const double gml = lgl * tgl, gmu = lgu * tgu;
                gst(ro.rm, q.lo, gml, st);
                gst(ro.rm, q.up, gmu, st);
                ms += st ? gml + gmu : 0.0;  // constraint 4 lc + g is counted once, in lane (g, 0)
            }
        }
    }
    pim1 = pcn;
}

// Returns false (mu untouched) when the problem has no constraints (d_res_ip_res_hard.c:309-313).
template <bool UPD, class FX>
__device__ bool residual_pass(const RicIO& io, const BoxCtx& bc, const ResIO& ro, double& mu_out) {
    double ms = 0.0, pim1 = 0.0;
    int nbt = 0;
    ResFrag<UPD> cur, nxt;
    {
        const StageRef s0{io.st, 0};
        with_shape<FX>(s0, [&](const auto& sh) { res_fetch<UPD>(io, sh, bc, ro, 0, cur); });
    }
    for (int k = 0; k <= io.N; k++) {
        const int kn = k < io.N ? k + 1 : io.N;
        const StageRef sn{io.st, kn};
        with_shape<FX>(sn, [&](const auto& sh) { res_fetch<UPD>(io, sh, bc, ro, kn, nxt); });
        asm volatile("" ::: "memory");
        const StageRef si{io.st, k};
        nbt += srd(si, &StageInfo::nb) + srd(si, &StageInfo::ng);
        with_shape<FX>(si, [&](const auto& sh) { res_step<UPD>(io, sh, k, cur, bc, ro, pim1, ms); });
        cur = nxt;
    }
    ms = wave_sum(ms);
    if (nbt != 0) {
        mu_out = ms / (2.0 * nbt);
        return true;
    }
    return false;
}

}  // namespace hk
