// hk_riccati.h -- device-side Riccati recursion for one problem per wavefront (gfx950).
//
// Restates, per wave, lqcp_solvers/d_back_ric_rec.c (reference):
//   sv  :112-399   backward factorisation with the augmented gradient row + forward substitution
//   trf :403-560   factorisation only
//   trs :564-791   backward/forward substitution with an existing factor
// The per-stage dtrmm (kernel_dtrmm_nt_u_4x4) and the dsyrk part of dsyrk_dpotrf are two chains of
// v_mfma_f64_16x16x4_f64 on the stage tile; the Cholesky (kernel_dsyrk_dpotrf_nt_4x4 /
// kernel_dgemm_dtrsm_nt_4x4 with the >1e-15 pivot clamp) runs on the tile registers with DPP and
// permlane broadcasts; the triangular solves (dtrsv_n/t) and gemv/trmv are wave reductions.
//
// Tile coordinates: variable v of stage k (u first, then x) sits at tile index
//     tile(v) = v < nu ? v : xo + (v - nu),   xo = round_up(nu, 4),
// so that the state block always starts on an MFMA K-chunk boundary.  Tile indices in [nu, xo) and
// beyond xo+nx are zero padding (their pivots clamp to 0 and contribute nothing).
#pragma once
#include "hk_prims.h"

namespace hk {

// Per-stage static description (shared by all problems of a batch).  64 bytes.
struct StageInfo {
    int nu, nx, nb, ng;
    int xo;             // round_up(nu, 4)
    int nx1, nu1, xo1;  // next stage (0 for k = N)
    int sdB, sdR;       // lib4 panel strides of BAbt_k (cnx_{k+1}) and RSQrq_k (cnux_k)
    int oB, oR, oD;     // offsets (doubles) of BAbt_k / RSQrq_k / d_k inside one problem's arrays
    int pnb;            // round_up(nb, 4)
    int r0, r1;
};

constexpr int FSTRIDE = 288;  // factor doubles per stage: 4 regs x 64 lanes + l (16) + inv_diag (16)
constexpr int V16 = 16;       // per-stage stride of tile/state vectors
constexpr int V32 = 32;       // per-stage stride of constraint vectors ([lb | pad | ub | pad])

__device__ __forceinline__ int tile_var(int t, int nu, int nx, int xo) {
    return t < nu ? t : ((t >= xo && t < xo + nx) ? nu + (t - xo) : -1);
}

__device__ __forceinline__ double lib4_at(const double* A, int sd, int i, int j) {
    return A[(i >> 2) * 4 * sd + (i & 3) + 4 * j];
}

// LDS scratch for col->row layout conversion: 16 doubles per wave.
struct Scratch {
    double v[32];
};

// col layout value (lane (g,c) holds v[c]) -> row layout (reg r holds v[g+4r])
__device__ __forceinline__ void col2row(Scratch* sm, double vc, double vr[4]) {
    const int l = lane_id(), g = l >> 4, c = l & 15;
    if (g == 0) sm->v[c] = vc;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int r = 0; r < 4; r++) vr[r] = sm->v[g + 4 * r];
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    __builtin_amdgcn_wave_barrier();
}

// ------------------------------------------------------------------------------------------------
// Stage Cholesky with the augmented row.  In: M (tile, full symmetric), ml (aug row, col layout).
// Out: S = lower(L) + strict_upper(L') (symmetric storage: row p of S == column p of L),
//      lc / lr : aug row l in col / row layout, invd : inverse diagonal (col layout).
// Pivots outside [0,nu) U [xo, xo+nx) are skipped (zero padding, inv_diag = 0 as the clamp gives).
// ------------------------------------------------------------------------------------------------
template <bool AUG>
__device__ __forceinline__ void stage_chol(double M[4], double& ml, double lr[4], double& invd, int nu, int nx,
                                           int xo) {
    const int l = lane_id(), g = l >> 4, c = l & 15;
    invd = 0.0;
#pragma unroll
    for (int r = 0; r < 4; r++) lr[r] = 0.0;
#pragma unroll
    for (int p = 0; p < 16; p++) {
        const bool act = (p < nu) || (p >= xo && p < xo + nx);
        if (!act) continue;  // wave-uniform
        const int rp = p >> 2, gp = p & 3;
        double d;
        switch (rp) {  // p is a compile-time constant after unrolling
            case 0: d = readlane(M[0], gp * 16 + p); break;
            case 1: d = readlane(M[1], gp * 16 + p); break;
            case 2: d = readlane(M[2], gp * 16 + p); break;
            default: d = readlane(M[3], gp * 16 + p); break;
        }
        double s, inv;
        chol_pivot(d, s, inv);
        // column p in row layout: L[g+4r][p] = M[g+4r][p] * inv   (DPP row_newbcast:p)
        double cr[4];
#pragma unroll
        for (int r = 0; r < 4; r++) {
            double v;
            switch (p) {
#define HK_CASE(P) \
    case P: v = row_bcast<P>(M[r]); break;
                HK_CASE(0) HK_CASE(1) HK_CASE(2) HK_CASE(3) HK_CASE(4) HK_CASE(5) HK_CASE(6) HK_CASE(7)
                HK_CASE(8) HK_CASE(9) HK_CASE(10) HK_CASE(11) HK_CASE(12) HK_CASE(13) HK_CASE(14)
                default: v = row_bcast<15>(M[r]); break;
#undef HK_CASE
            }
            cr[r] = (g + 4 * r > p) ? v * inv : 0.0;
        }
        // column p in col layout: L[c][p] = M[p][c] * inv   (row p broadcast from row group gp)
        double mrow;
        {
            double src = (rp == 0) ? M[0] : (rp == 1) ? M[1] : (rp == 2) ? M[2] : M[3];
            switch (gp) {
                case 0: mrow = rowgroup_bcast<0>(src); break;
                case 1: mrow = rowgroup_bcast<1>(src); break;
                case 2: mrow = rowgroup_bcast<2>(src); break;
                default: mrow = rowgroup_bcast<3>(src); break;
            }
        }
        const double cc = (c > p) ? mrow * inv : 0.0;
        // trailing update (both triangles) + write column p and row p (= column p, symmetric storage)
#pragma unroll
        for (int r = 0; r < 4; r++) {
            const int row = g + 4 * r;
            double m = M[r] - cr[r] * cc;
            if (c == p) m = (row > p) ? cr[r] : (row == p ? s : M[r]);
            if (row == p && c > p) m = cc;
            M[r] = m;
        }
        if (AUG) {
            const double lp = readlane(ml, p) * inv;  // l_p = m_last[p] / L[p][p]
            ml = (c == p) ? lp : ((c > p) ? ml - lp * cc : ml);
#pragma unroll
            for (int r = 0; r < 4; r++)
                if (r == rp) lr[r] = (g == gp) ? lp : lr[r];
        }
        if (c == p) invd = inv;
    }
    // rows/cols that were never pivoted (padding) are zero already; strictly-upper part of inactive
    // rows is zero too.
}


// ------------------------------------------------------------------------------------------------
// Per-problem views used by the stage passes.
// ------------------------------------------------------------------------------------------------
struct RicIO {
    int N;
    const StageInfo* st;
    const signed char* tileslot;  // (N+1)*16: box slot owning tile t, or -1
    const double* BAbt;           // this problem's BAbt base (stage k block at st[k].oB)
    const double* RSQ;            // this problem's RSQrq base (stage k block at st[k].oR)
    double* F;                    // factor store (N+1)*FSTRIDE (private layout)
};

__device__ __forceinline__ StageInfo load_stage(const StageInfo* st, int k) { return st[k]; }

__device__ __forceinline__ bool tile_active(int t, int nu, int nx, int xo) {
    return t < nu || (t >= xo && t < xo + nx);
}

// lower / upper part of the symmetric factor storage S (lane (g,c), reg r = S[g+4r][c])
__device__ __forceinline__ double lowS(const d4& S, int r, int g, int c) { return (g + 4 * r >= c) ? S[r] : 0.0; }

__device__ __forceinline__ void load_factor(const double* Fk, d4& S, double& lc, double& invd) {
    const int l = lane_id(), c = l & 15;
#pragma unroll
    for (int r = 0; r < 4; r++) S[r] = Fk[r * 64 + l];
    lc = Fk[256 + c];
    invd = Fk[272 + c];
}

// Backward Riccati recursion (sv when AUG, trf otherwise), d_back_ric_rec.c:186-335 / :447-558.
//   b  (state order) / q (variable order) : update_b / update_q replacement rows
//   Qx, qx (box-slot order)               : box Hessian / gradient terms (use_box)
//   Pb (state order)                      : P_{k+1} b_k (compute_Pb, AUG only)
// Vector arguments use a per-stage stride of V16.
template <bool AUG>
__device__ void ric_backward(const RicIO& io, Scratch* sm, int update_b, const double* bsrc, int update_q,
                             const double* qsrc, int use_box, const double* Qx, const double* qx, int compute_Pb,
                             double* Pb) {
    const int l = lane_id(), g = l >> 4, c = l & 15;
    d4 S = {0.0, 0.0, 0.0, 0.0};
    double lr_prev[4] = {0.0, 0.0, 0.0, 0.0};
    for (int k = io.N; k >= 0; k--) {
        const StageInfo si = load_stage(io.st, k);
        const int nu = si.nu, nx = si.nx, xo = si.xo, nux = nu + nx;
        const double* R = io.RSQ + si.oR;
        const int vc = tile_var(c, nu, nx, xo);
        // M = lower(RSQrq) mirrored to a full symmetric tile
        d4 M;
#pragma unroll
        for (int r = 0; r < 4; r++) {
            const int vi = tile_var(g + 4 * r, nu, nx, xo);
            M[r] = (vi >= 0 && vc >= 0) ? lib4_at(R, si.sdR, vi > vc ? vi : vc, vi > vc ? vc : vi) : 0.0;
        }
        double ml = 0.0;
        if (AUG && vc >= 0) ml = update_q ? qsrc[k * V16 + vc] : lib4_at(R, si.sdR, nux, vc);
        if (use_box && si.nb > 0) {
            const int slot = io.tileslot[k * 16 + c];
            if (slot >= 0) {
                const double dq = Qx[k * V16 + slot];
#pragma unroll
                for (int r = 0; r < 4; r++)
                    if (g + 4 * r == c) M[r] += dq;  // ddiaadin: diag = bd + Qx
                if (AUG) ml += qx[k * V16 + slot];   // drowad: aug row += qx
            }
        }
        if (k < io.N) {
            const int nx1 = si.nx1, xo1 = si.xo1;
            const double* Bk = io.BAbt + si.oB;
            // W' = Lxx_{k+1}' BAbt_k'  (dtrmm_nt_u, d_back_ric_rec.c:262-264), rows in stage-(k+1) tile coords
            d4 acc = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
            for (int kc = 0; kc < 4; kc++) {
                if (4 * kc + 3 < xo1 || 4 * kc >= xo1 + nx1) continue;  // uniform
                const int qt = 4 * kc + g, s = qt - xo1;
                const double bop = (vc >= 0 && s >= 0 && s < nx1) ? lib4_at(Bk, si.sdB, vc, s) : 0.0;
                const double aop = (c >= xo1 && qt >= c) ? S[kc] : 0.0;
                acc = mfma(aop, bop, acc);
            }
            // M += W W'  (dsyrk part of dsyrk_dpotrf_lib, :325)
#pragma unroll
            for (int r = 0; r < 4; r++) {
                if (4 * r + 3 < xo1 || 4 * r >= xo1 + nx1) continue;
                M = mfma(acc[r], acc[r], M);
            }
            if (AUG) {
                // v = Lxx' b (col layout, stage k+1 tile), b from the BAbt augmented row or update_b
                double part = 0.0;
#pragma unroll
                for (int r = 0; r < 4; r++) {
                    const int s = g + 4 * r - xo1;
                    double bv = 0.0;
                    if (s >= 0 && s < nx1) bv = update_b ? bsrc[k * V16 + s] : lib4_at(Bk, si.sdB, nux, s);
                    part += (c >= xo1 ? lowS(S, r, g, c) : 0.0) * bv;
                }
                const double vcol = xrow_sum(part);
                double vrow[4];
                col2row(sm, vcol, vrow);
                if (compute_Pb) {
                    // Pb_k = Lxx (Lxx' b)  (dtrmv_u_t on W's last row, :266-275)
                    double pp = 0.0;
#pragma unroll
                    for (int r = 0; r < 4; r++) {
                        const int j = g + 4 * r;
                        pp += (j <= c && j >= xo1) ? S[r] * vrow[r] : 0.0;
                    }
                    const double pb = xrow_sum(pp);
                    if (g == 0 && c >= xo1 && c < xo1 + nx1) Pb[k * V16 + (c - xo1)] = pb;
                }
                // w_last = b' Lxx + l_{k+1,x}   (dgead, :276)  -> m_last += W w_last
                double mp = 0.0;
#pragma unroll
                for (int r = 0; r < 4; r++) {
                    const double w = (g + 4 * r >= xo1) ? vrow[r] + lr_prev[r] : 0.0;
                    mp += acc[r] * w;
                }
                ml += xrow_sum(mp);
            }
        }
        double Ml[4] = {M[0], M[1], M[2], M[3]};
        double lr[4], invd;
        stage_chol<AUG>(Ml, ml, lr, invd, nu, nx, xo);
        double* Fk = io.F + (long)k * FSTRIDE;
#pragma unroll
        for (int r = 0; r < 4; r++) {
            S[r] = Ml[r];
            Fk[r * 64 + l] = Ml[r];
            lr_prev[r] = lr[r];
        }
        if (g == 0) {
            Fk[256 + c] = AUG ? ml : 0.0;
            Fk[272 + c] = invd;
        }
    }
}

// Solve the unknown part of L_k' y = rhs (dtrsv_t_lib, blas_d_lib4.c:5276) in row layout, descending.
// rrow: rhs in row layout (reduced by the known part already); y written into ur (row layout) at the
// unknown tile indices.  unknown(t) = active(t) && (all || t < nu).
__device__ __forceinline__ void solve_lt(const d4& S, double invd, double rrow[4], double ur[4], int nu, int nx,
                                         int xo, bool all) {
    const int l = lane_id(), g = l >> 4;
#pragma unroll
    for (int p = 15; p >= 0; p--) {
        const bool unk = all ? tile_active(p, nu, nx, xo) : (p < nu);
        if (!unk) continue;
        const int rp = p >> 2, gp = p & 3;
        const double rv = (rp == 0) ? rrow[0] : (rp == 1) ? rrow[1] : (rp == 2) ? rrow[2] : rrow[3];
        const double y = readlane(rv, gp * 16) * readlane(invd, p);
#pragma unroll
        for (int r = 0; r < 4; r++) {
            double sv;
            switch (p) {
#define HK_CASE(P) \
    case P: sv = row_bcast<P>(S[r]); break;
                HK_CASE(0) HK_CASE(1) HK_CASE(2) HK_CASE(3) HK_CASE(4) HK_CASE(5) HK_CASE(6) HK_CASE(7)
                HK_CASE(8) HK_CASE(9) HK_CASE(10) HK_CASE(11) HK_CASE(12) HK_CASE(13) HK_CASE(14)
                default: sv = row_bcast<15>(S[r]); break;
#undef HK_CASE
            }
            if (g + 4 * r < p) rrow[r] -= sv * y;  // L[p][j] = S[j][p] (upper storage), j = g+4r < p
            if (r == rp && g == gp) ur[r] = y;
        }
    }
}

// Forward solve of the unknown part of L_k y = h (dtrsv_n_lib, :5204) in col layout, ascending;
// rows beyond the unknown block get the rectangular update.
__device__ __forceinline__ double solve_ln(const d4& S, double invd, double h, int nu, int nx, int xo, bool all) {
    const int l = lane_id(), c = l & 15;
#pragma unroll
    for (int p = 0; p < 16; p++) {
        const bool unk = all ? tile_active(p, nu, nx, xo) : (p < nu);
        if (!unk) continue;
        const int rp = p >> 2, gp = p & 3;
        const double y = readlane(h, p) * readlane(invd, p);
        const double src = (rp == 0) ? S[0] : (rp == 1) ? S[1] : (rp == 2) ? S[2] : S[3];
        double colp;  // L[c][p] for c > p = S[p][c]
        switch (gp) {
            case 0: colp = rowgroup_bcast<0>(src); break;
            case 1: colp = rowgroup_bcast<1>(src); break;
            case 2: colp = rowgroup_bcast<2>(src); break;
            default: colp = rowgroup_bcast<3>(src); break;
        }
        h = (c == p) ? y : ((c > p) ? h - colp * y : h);
    }
    return h;
}

// x_{k+1} = b + BAbt_k' ux_k  (dgemv_t_lib alg 1, :347-351), col layout over stage-(k+1) tile.
__device__ __forceinline__ double gemv_t_next(const double* Bk, const StageInfo& si, const double ur[4], double bval) {
    const int l = lane_id(), g = l >> 4, c = l & 15;
    const int s = c - si.xo1;
    double part = 0.0;
#pragma unroll
    for (int r = 0; r < 4; r++) {
        const int vi = tile_var(g + 4 * r, si.nu, si.nx, si.xo);
        if (vi >= 0 && s >= 0 && s < si.nx1) part += lib4_at(Bk, si.sdB, vi, s) * ur[r];
    }
    return bval + xrow_sum(part);
}

// pi = Lxx (Lxx' x + p)  on the next-stage factor S1 (dtrmv_u_n + dtrmv_u_t, :355-365), col layout.
__device__ __forceinline__ double pi_from_x(Scratch* sm, const d4& S1, int xo1, const double x1row[4], double pcol) {
    const int l = lane_id(), g = l >> 4, c = l & 15;
    double part = 0.0;
#pragma unroll
    for (int r = 0; r < 4; r++) part += (c >= xo1 && g + 4 * r >= c) ? S1[r] * x1row[r] : 0.0;
    const double tcol = (c >= xo1) ? xrow_sum(part) + pcol : 0.0;
    double trow[4];
    col2row(sm, tcol, trow);
    double p2 = 0.0;
#pragma unroll
    for (int r = 0; r < 4; r++) {
        const int j = g + 4 * r;
        p2 += (j <= c && j >= xo1) ? S1[r] * trow[r] : 0.0;
    }
    return xrow_sum(p2);
}

// Forward substitution of the sv (d_back_ric_rec.c:339-397).  ux: variable order; pi: state order.
__device__ void ric_forward_sv(const RicIO& io, Scratch* sm, int update_b, const double* bsrc, double* ux,
                               int compute_pi, double* pi) {
    const int l = lane_id(), g = l >> 4, c = l & 15;
    double xcol = 0.0;  // x_k in col layout (stage-k tile coords)
    d4 S;
    double lc, invd;
    load_factor(io.F, S, lc, invd);
    for (int k = 0; k < io.N; k++) {
        const StageInfo si = load_stage(io.st, k);
        const int nu = si.nu, nx = si.nx, xo = si.xo, nux = nu + nx;
        const bool all = (k == 0);
        double xrow[4];
        col2row(sm, xcol, xrow);
        double part = 0.0;
        if (!all) {
#pragma unroll
            for (int r = 0; r < 4; r++) part += (g + 4 * r >= xo) ? lowS(S, r, g, c) * xrow[r] : 0.0;
        }
        const double rc = -lc - xrow_sum(part);
        double rrow[4], ur[4];
        col2row(sm, rc, rrow);
#pragma unroll
        for (int r = 0; r < 4; r++) ur[r] = all ? 0.0 : xrow[r];
        solve_lt(S, invd, rrow, ur, nu, nx, xo, all);
        // store ux_k (variable order) from row layout (lanes c == 0)
        if (c == 0) {
#pragma unroll
            for (int r = 0; r < 4; r++) {
                const int v = tile_var(g + 4 * r, nu, nx, xo);
                if (v >= 0) ux[k * V16 + v] = ur[r];
            }
        }
        const double* Bk = io.BAbt + si.oB;
        const int s = c - si.xo1;
        double bval = 0.0;
        if (s >= 0 && s < si.nx1) bval = update_b ? bsrc[k * V16 + s] : lib4_at(Bk, si.sdB, nux, s);
        const double x1 = gemv_t_next(Bk, si, ur, bval);
        xcol = (s >= 0 && s < si.nx1) ? x1 : 0.0;
        d4 S1;
        double lc1, invd1;
        load_factor(io.F + (long)(k + 1) * FSTRIDE, S1, lc1, invd1);
        if (compute_pi) {
            double x1row[4];
            col2row(sm, xcol, x1row);
            const double pv = pi_from_x(sm, S1, si.xo1, x1row, lc1);
            if (g == 0 && s >= 0 && s < si.nx1) pi[k * V16 + s] = pv;
        }
        S = S1;
        lc = lc1;
        invd = invd1;
    }
    // x_N
    const StageInfo sN = load_stage(io.st, io.N);
    const int v = tile_var(c, sN.nu, sN.nx, sN.xo);
    if (g == 0 && v >= 0) ux[io.N * V16 + v] = xcol;
}

// stage gradient g_k[c] = q_k + qx at the box slots (dvecad_libsp, :612-620), col layout
__device__ __forceinline__ double stage_grad(const RicIO& io, int k, const StageInfo& si, const double* hq,
                                             int use_box, const double* qx) {
    const int c = lane_id() & 15;
    const int v = tile_var(c, si.nu, si.nx, si.xo);
    double h = 0.0;
    if (v >= 0) h = hq ? hq[k * V16 + v] : lib4_at(io.RSQ + si.oR, si.sdR, si.nu + si.nx, v);
    if (use_box && si.nb > 0) {
        const int slot = io.tileslot[k * 16 + c];
        if (slot >= 0) h += qx[k * V16 + slot];
    }
    return h;
}

// Riccati solve with an existing factor (d_back_ric_rec.c:564-791).
// hb: state order, hq: variable order, qx: slot order; ux (variable order) doubles as the backward
// work vector exactly like hux in the reference.
__device__ void ric_trs(const RicIO& io, Scratch* sm, const double* hb, const double* hq, int use_box,
                        const double* qx, double* ux, int compute_pi, double* pi, int compute_Pb, double* Pb) {
    const int l = lane_id(), g = l >> 4, c = l & 15;
    // ---- backward
    StageInfo sn = load_stage(io.st, io.N);
    double h = stage_grad(io, io.N, sn, hq, use_box, qx);
    {
        const int v = tile_var(c, sn.nu, sn.nx, sn.xo);
        if (g == 0 && v >= 0) ux[io.N * V16 + v] = h;
    }
    double pcol = h;  // hux_{k+1} in col layout (stage-(k+1) tile coords)
    d4 S1;
    double lc1, invd1;
    load_factor(io.F + (long)io.N * FSTRIDE, S1, lc1, invd1);
    for (int k = io.N - 1; k >= 0; k--) {
        const StageInfo si = load_stage(io.st, k);
        const int nu = si.nu, nx = si.nx, xo = si.xo, xo1 = si.xo1, nx1 = si.nx1;
        const double* Bk = io.BAbt + si.oB;
        const int vc = tile_var(c, nu, nx, xo);
        double pbc;
        const int s = c - xo1;
        if (compute_Pb) {
            double brow[4], part = 0.0;
#pragma unroll
            for (int r = 0; r < 4; r++) {
                const int sr = g + 4 * r - xo1;
                brow[r] = (sr >= 0 && sr < nx1) ? (hb ? hb[k * V16 + sr] : lib4_at(Bk, si.sdB, nu + nx, sr)) : 0.0;
                part += (c >= xo1 ? lowS(S1, r, g, c) : 0.0) * brow[r];
            }
            const double vcol = xrow_sum(part);
            double vrow[4];
            col2row(sm, vcol, vrow);
            double pp = 0.0;
#pragma unroll
            for (int r = 0; r < 4; r++) {
                const int j = g + 4 * r;
                pp += (j <= c && j >= xo1) ? S1[r] * vrow[r] : 0.0;
            }
            pbc = xrow_sum(pp);
            if (g == 0 && s >= 0 && s < nx1) Pb[k * V16 + s] = pbc;
        } else {
            pbc = (s >= 0 && s < nx1) ? Pb[k * V16 + s] : 0.0;
        }
        const double wc = (s >= 0 && s < nx1) ? pbc + pcol : 0.0;
        double wrow[4];
        col2row(sm, wc, wrow);
        h = stage_grad(io, k, si, hq, use_box, qx);
        double part = 0.0;
#pragma unroll
        for (int r = 0; r < 4; r++) {
            const int sr = g + 4 * r - xo1;
            if (vc >= 0 && sr >= 0 && sr < nx1) part += lib4_at(Bk, si.sdB, vc, sr) * wrow[r];
        }
        h += xrow_sum(part);
        d4 S;
        double lc, invd;
        load_factor(io.F + (long)k * FSTRIDE, S, lc, invd);
        h = solve_ln(S, invd, h, nu, nx, xo, k == 0);
        if (g == 0 && vc >= 0) ux[k * V16 + vc] = h;
        pcol = h;
        S1 = S;
        lc1 = lc;
        invd1 = invd;
    }
    // ---- forward
    double xcol = 0.0;
    d4 S;
    double lc, invd;
    load_factor(io.F, S, lc, invd);
    for (int k = 0; k < io.N; k++) {
        const StageInfo si = load_stage(io.st, k);
        const int nu = si.nu, nx = si.nx, xo = si.xo;
        const bool all = (k == 0);
        const int vc = tile_var(c, nu, nx, xo);
        const int s = c - si.xo1;
        const StageInfo s1 = load_stage(io.st, k + 1);
        double pk = 0.0;
        if (compute_pi) {
            const int v1 = tile_var(c, s1.nu, s1.nx, s1.xo);
            pk = (v1 >= 0 && c >= s1.xo) ? ux[(k + 1) * V16 + v1] : 0.0;  // p_{k+1} = hux_{k+1}[x]
        }
        const double hc = (vc >= 0) ? ux[k * V16 + vc] : 0.0;
        double xrow[4];
        col2row(sm, xcol, xrow);
        double part = 0.0;
        if (!all) {
#pragma unroll
            for (int r = 0; r < 4; r++) part += (g + 4 * r >= xo) ? lowS(S, r, g, c) * xrow[r] : 0.0;
        }
        const double rc = -hc - xrow_sum(part);
        double rrow[4], ur[4];
        col2row(sm, rc, rrow);
#pragma unroll
        for (int r = 0; r < 4; r++) ur[r] = all ? 0.0 : xrow[r];
        solve_lt(S, invd, rrow, ur, nu, nx, xo, all);
        if (c == 0) {
#pragma unroll
            for (int r = 0; r < 4; r++) {
                const int v = tile_var(g + 4 * r, nu, nx, xo);
                if (v >= 0) ux[k * V16 + v] = ur[r];
            }
        }
        const double* Bk = io.BAbt + si.oB;
        double bval = 0.0;
        if (s >= 0 && s < si.nx1) bval = hb ? hb[k * V16 + s] : lib4_at(Bk, si.sdB, nu + nx, s);
        const double x1 = gemv_t_next(Bk, si, ur, bval);
        xcol = (s >= 0 && s < si.nx1) ? x1 : 0.0;
        d4 Sn;
        double lcn, invdn;
        load_factor(io.F + (long)(k + 1) * FSTRIDE, Sn, lcn, invdn);
        if (compute_pi) {
            double x1row[4];
            col2row(sm, xcol, x1row);
            // pi_k = p_{k+1} + Lxx (Lxx' x_{k+1})   (:735-745)
            const double pv = pi_from_x(sm, Sn, si.xo1, x1row, 0.0) + pk;
            if (g == 0 && s >= 0 && s < si.nx1) pi[k * V16 + s] = pv;
        }
        S = Sn;
        lc = lcn;
        invd = invdn;
    }
    const StageInfo sN = load_stage(io.st, io.N);
    const int v = tile_var(c, sN.nu, sN.nx, sN.xo);
    if (g == 0 && v >= 0) ux[io.N * V16 + v] = xcol;
}

}  // namespace hk
