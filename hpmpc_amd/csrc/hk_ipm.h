// hk_ipm.h -- residuals and interior-point vector kernels, one problem per wavefront (gfx950).
//
// Restates mpc_solvers/c99/d_res_ip_res_hard.c:39-319 (KKT residuals) and the vector kernels of
// mpc_solvers/c99/d_aux_ip_hard_lib4.c (box constraints; ng == 0 on the GPU path).  Box-slot vectors
// use the reference's per-stage [lb (pnb) | ub (pnb)] layout inside a V32 stride.  The element-wise
// passes process four stages at once: row group g of the wave handles stage 4j+g, column c slot c.
#pragma once
#include "hk_riccati.h"

namespace hk {

struct BoxTab {
    const signed char* tileslot;  // (N+1)*16 box slot of tile t or -1
    const signed char* slotvar;   // (N+1)*16 variable index of box slot l
};

// Iterate (stage k, slot c) pairs four stages per pass.  Body sees k, slot, lo (lower index), up.
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

// d_res_res_mpc_hard_tv: r_q, r_b, r_d, r_m and mu (returned; NaN-free 0 if no constraints means
// "leave mu untouched", signalled by the bool).
// b: state order (the BAbt augmented row if bsrc == nullptr), q: variable order (RSQrq aug row if null).
__device__ bool residuals(const RicIO& io, const BoxTab& bt, Scratch* sm, const double* bsrc, const double* qsrc,
                          const double* ux, const double* pi, const double* dvec, const double* lam, const double* t,
                          double* rq, double* rb, double* rd, double* rm, double& mu_out) {
    const int l = lane_id(), g = l >> 4, c = l & 15;
    for (int k = 0; k <= io.N; k++) {
        const StageInfo si = load_stage(io.st, k);
        const int nu = si.nu, nx = si.nx, xo = si.xo, nux = nu + nx;
        const double* R = io.RSQ + si.oR;
        const int vc = tile_var(c, nu, nx, xo);
        double uxrow[4], pirow[4];
        d4 M;
#pragma unroll
        for (int r = 0; r < 4; r++) {
            const int vi = tile_var(g + 4 * r, nu, nx, xo);
            uxrow[r] = vi >= 0 ? ux[k * V16 + vi] : 0.0;
            M[r] = (vi >= 0 && vc >= 0) ? lib4_at(R, si.sdR, vi > vc ? vi : vc, vi > vc ? vc : vi) : 0.0;
        }
        // r_q = q - [0; pi_{k-1}] + box terms + RSQ ux + BAbt pi
        double h = 0.0;
        if (vc >= 0) {
            h = qsrc ? qsrc[k * V16 + vc] : lib4_at(R, si.sdR, nux, vc);
            if (k > 0 && vc >= nu) h -= pi[(k - 1) * V16 + (vc - nu)];
            if (si.nb > 0) {
                const int slot = bt.tileslot[k * 16 + c];
                if (slot >= 0) h += -lam[k * V32 + slot] + lam[k * V32 + si.pnb + slot];
            }
        }
        double part = 0.0;
#pragma unroll
        for (int r = 0; r < 4; r++) part += M[r] * uxrow[r];
        h += xrow_sum(part);
        if (k < io.N) {
            const double* Bk = io.BAbt + si.oB;
            const int nx1 = si.nx1, xo1 = si.xo1;
            double p2 = 0.0, p3 = 0.0;
#pragma unroll
            for (int r = 0; r < 4; r++) {
                const int sr = g + 4 * r - xo1;  // state index of stage-(k+1) tile row g+4r
                pirow[r] = (sr >= 0 && sr < nx1) ? pi[k * V16 + sr] : 0.0;
                if (vc >= 0 && sr >= 0 && sr < nx1) p2 += lib4_at(Bk, si.sdB, vc, sr) * pirow[r];
                const int vi = tile_var(g + 4 * r, nu, nx, xo);
                const int s = c - xo1;
                if (vi >= 0 && s >= 0 && s < nx1) p3 += lib4_at(Bk, si.sdB, vi, s) * uxrow[r];
            }
            h += xrow_sum(p2);
            const double atu = xrow_sum(p3);
            const int s = c - xo1;
            if (g == 0 && s >= 0 && s < nx1) {
                const StageInfo s1 = load_stage(io.st, k + 1);
                const double bb = bsrc ? bsrc[k * V16 + s] : lib4_at(Bk, si.sdB, nux, s);
                rb[k * V16 + s] = bb - ux[(k + 1) * V16 + s1.nu + s] + atu;
            }
        }
        if (g == 0 && vc >= 0) rq[k * V16 + vc] = h;
    }
    // r_d, r_m, mu
    double mus = 0.0;
    int nbt = 0;
    for (int k = 0; k <= io.N; k++) nbt += io.st[k].nb;
    HK_FOR_BOX(io, k, {
        const int v = bt.slotvar[k * 16 + slot];
        const double x = ux[k * V16 + v];
        rd[lo] = dvec[k * V32 + slot] - x + t[lo];
        rd[up] = dvec[k * V32 + pnb_ + slot] - x - t[up];
        const double ml = lam[lo] * t[lo], mu_ = lam[up] * t[up];
        rm[lo] = ml;
        rm[up] = mu_;
        mus += ml + mu_;
    });
    mus = wave_sum(mus);
    if (nbt != 0) {
        mu_out = mus / (2.0 * nbt);
        return true;
    }
    return false;
}

}  // namespace hk
