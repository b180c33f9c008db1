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
    int r0;             // flags: bit 0 the stage belongs to the compiled inner class (constant shapes); bits 1 / 2
                        // its BAbt / RSQrq block is shared by every problem of the batch (no problem stride:
                        // the time-invariant / aliased layouts, hpmpc_mi355x_layout.BAbt_shared / RSQrq_shared)
    int oG;             // offset (doubles) of DCt_k inside one problem's general-constraint array
};

constexpr int FSTRIDE = 352;  // factor doubles per stage: 4 regs x 64 lanes + l (16) + inv_diag (16) + KG (64)
constexpr int V16 = 16;       // per-stage stride of tile/state vectors
constexpr int V32 = 32;       // per-stage stride of constraint vectors ([lb | pad | ub | pad])

__device__ __forceinline__ bool tile_active(int t, int nu, int nx, int xo) {
    return t < nu || (t >= xo && t < xo + nx);
}

__device__ __forceinline__ int tile_var(int t, int nu, int nx, int xo) {
    return t < nu ? t : ((t >= xo && t < xo + nx) ? nu + (t - xo) : -1);
}

__device__ __forceinline__ double lib4_at(const double* A, int sd, int i, int j) {
    return A[(i >> 2) * 4 * sd + (i & 3) + 4 * j];
}

__device__ __forceinline__ int lib4_idx(int sd, int i, int j) { return (i >> 2) * 4 * sd + (i & 3) + 4 * j; }

// Unconditional load + select: every lane issues the load (at a clamped, valid address), so the
// number of outstanding vector-memory ops is the same on every path and hipcc can wait with a
// counted s_waitcnt vmcnt(N) instead of draining the whole prefetch queue.
__device__ __forceinline__ double ldsel(const double* p, int idx, bool ok) { return gld(p, idx, ok); }

// LDS scratch for col->row layout conversion: 16 doubles per wave.
struct Scratch {
    double v[32];
};

// col layout value (lane (g,c) holds v[c]) -> row layout (reg r holds v[g+4r])
__device__ __forceinline__ void col2row(Scratch* sm, double vc, double vr[4]) {
    const int l = lane_id(), g = l >> 4, c = l & 15;
    sm->v[c] = vc;  // the four row groups write the same value (no exec-mask branch)
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int r = 0; r < 4; r++) vr[r] = sm->v[g + 4 * r];
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    __builtin_amdgcn_wave_barrier();
}

// two col-layout values -> row layout in one LDS round trip
__device__ __forceinline__ void col2row2(Scratch* sm, double ac, double bc, double ar[4], double br[4]) {
    const int l = lane_id(), g = l >> 4, c = l & 15;
    sm->v[c] = ac;
    sm->v[16 + c] = bc;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int r = 0; r < 4; r++) {
        ar[r] = sm->v[g + 4 * r];
        br[r] = sm->v[16 + g + 4 * r];
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    __builtin_amdgcn_wave_barrier();
}

// row layout (reg r holds v[g+4r], replicated over the columns) -> col layout (lane (g,c) holds v[c])
__device__ __forceinline__ double row2col(Scratch* sm, const double vr[4]) {
    const int l = lane_id(), g = l >> 4, c = l & 15;
#pragma unroll
    for (int r = 0; r < 4; r++) sm->v[16 + g + 4 * r] = vr[r];  // replicas write identical values
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    const double v = sm->v[16 + c];
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    return v;
}

// ------------------------------------------------------------------------------------------------
// Stage Cholesky with the augmented row, blocked by 4 (one tile register per block row).
// In : M (tile, full symmetric), ml (aug row, col layout).
// Out: M = S = lower(L) + strict_upper(L') (symmetric storage: row p of S == column p of L),
//      ml = aug row l (col layout), lr = l in row layout, invd = inverse diagonal (col layout).
// Block b holds pivots 4b..4b+3 in register b (row group q = pivot 4b+q).  Inside a block the four
// pivots only touch register b (row-group broadcast + readlane); the rank-4 trailing update of the
// whole tile is ONE v_mfma_f64_16x16x4_f64 whose A and B fragments are register b itself (upper
// storage of the panel), and the lower triangle is restored at the end by an identity-MFMA
// transpose.  Pivots outside [0,nu) U [xo, xo+nx) are skipped (zero padding, inv_diag = 0).
// Pivot clamp d > 1e-15 as in kernel_dpotrf_c99_lib4.c:555-640.
// ------------------------------------------------------------------------------------------------
// One 4-pivot block of the stage Cholesky.  Column block b of the tile (rows 4b..4b+3 of the upper
// storage, i.e. register b) is gathered so that every lane holds the four entries x_j = A[c][4b+j]
// of its own tile row c.  The 4x4 diagonal block is then broadcast (DPP row_newbcast) and factorised
// redundantly in every lane -- a short scalar dependency chain with no cross-lane traffic -- while
// each lane solves its own panel row against it (kernel_dsyrk_dpotrf_nt_4x4 / kernel_dgemm_dtrsm_nt_4x4,
// same operation order, same >1e-15 pivot clamp).  Padded tile indices carry exact zeros, so their
// pivots clamp to 0 and contribute nothing.
template <int B, bool AUG, bool KGEN = false>
__device__ __forceinline__ void chol_block(d4& M, double& ml, double& invd, double* kg = nullptr, int kdbg = -1) {
    const int l = lane_id(), c = l & 15;
    (void)kdbg;
#define HK_BSTAMP(i) \
    if (B == 1) HK_STAMP(24 + (i), kdbg)
    HK_BSTAMP(0);
    double x[4];
    rowgroup_gather(M[B], x);
    // diagonal block A[4B+i][4B+j] (i >= j), uniform across the wave
    const double a00 = row_bcast<4 * B + 0>(x[0]);
    const double a10 = row_bcast<4 * B + 1>(x[0]), a11 = row_bcast<4 * B + 1>(x[1]);
    const double a20 = row_bcast<4 * B + 2>(x[0]), a21 = row_bcast<4 * B + 2>(x[1]);
    const double a22 = row_bcast<4 * B + 2>(x[2]);
    const double a30 = row_bcast<4 * B + 3>(x[0]), a31 = row_bcast<4 * B + 3>(x[1]);
    const double a32 = row_bcast<4 * B + 3>(x[2]), a33 = row_bcast<4 * B + 3>(x[3]);
    double m0 = 0.0, m1 = 0.0, m2 = 0.0, m3 = 0.0;
    if (AUG) {
        m0 = row_bcast<4 * B + 0>(ml);
        m1 = row_bcast<4 * B + 1>(ml);
        m2 = row_bcast<4 * B + 2>(ml);
        m3 = row_bcast<4 * B + 3>(ml);
    }
    // The diagonal entry is not formed separately: in lane c = 4B+g the panel formula for y_g is
    // d_g * i_g with exactly the operations that produce d_g in the uniform chain, i.e. s_g bitwise.
    const double i0 = chol_inv(a00);
    const double l10 = a10 * i0, l20 = a20 * i0, l30 = a30 * i0;
    const double y0 = x[0] * i0;
    const double p0 = m0 * i0;
    HK_BSTAMP(2);
    const double i1 = chol_inv(fma(-l10, l10, a11));
    const double l21 = fma(-l20, l10, a21) * i1, l31 = fma(-l30, l10, a31) * i1;
    const double y1 = fma(-y0, l10, x[1]) * i1;
    const double p1 = fma(-p0, l10, m1) * i1;
    HK_BSTAMP(3);
    const double i2 = chol_inv(fma(-l21, l21, fma(-l20, l20, a22)));
    const double l32 = fma(-l31, l21, fma(-l30, l20, a32)) * i2;
    const double y2 = fma(-y1, l21, fma(-y0, l20, x[2])) * i2;
    const double p2 = fma(-p1, l21, fma(-p0, l20, m2)) * i2;
    HK_BSTAMP(4);
    const double i3 = chol_inv(fma(-l32, l32, fma(-l31, l31, fma(-l30, l30, a33))));
    const double y3 = fma(-y2, l32, fma(-y1, l31, fma(-y0, l30, x[3]))) * i3;
    const double p3 = fma(-p2, l32, fma(-p1, l31, fma(-p0, l30, m3))) * i3;
    HK_BSTAMP(5);
    if (KGEN && B == 0) {
        // Gain form of the u-block (stages with nu <= 4, u in tile block 0): KG[g][c] = (-L_uu^{-T} y)_g with
        // y = e_c for the u tiles (c < 4: G = -L_uu^{-T}) and y = L[c][0..3] for the state tiles
        // (K = -L_uu^{-T} L_xu').  The forward then gets u = G rhs_u + K x as one 4x16 mat-vec
        // instead of the dtrsv_t back-substitution (same quantity, d_back_ric_rec.c:339-346).
        const bool ut = c < 4;
        const double e0 = ut ? (c == 0 ? 1.0 : 0.0) : y0, e1 = ut ? (c == 1 ? 1.0 : 0.0) : y1;
        const double e2 = ut ? (c == 2 ? 1.0 : 0.0) : y2, e3 = ut ? (c == 3 ? 1.0 : 0.0) : y3;
        const double z3 = e3 * i3;
        const double z2 = fma(-l32, z3, e2) * i2;
        const double z1 = fma(-l31, z3, fma(-l21, z2, e1)) * i1;
        const double z0 = fma(-l30, z3, fma(-l20, z2, fma(-l10, z1, e0))) * i0;
        *kg = -sel_g(z0, z1, z2, z3);
    }
    // upper storage row 4B+g: L[c][4B+g] = y_g for c >= 4B+g (diagonal included).  Branch-free selects.
    const double yg = sel_g(y0, y1, y2, y3);
    M[B] = yg;
    const int j = c - 4 * B;
    const bool inb = (c >> 2) == B, below = c > 4 * B + 3;
    invd = inb ? sel_q(i0, i1, i2, i3) : invd;
    if (AUG) {
        const double mt = fma(-p3, y3, fma(-p2, y2, fma(-p1, y1, fma(-p0, y0, ml))));
        const double mb = sel_q(p0, p1, p2, p3);
        ml = below ? mt : (inb ? mb : ml);
    }
    HK_BSTAMP(6);
    (void)j;
    if (B < 3) {
        const double a = below ? yg : 0.0;
        M = mfma(-a, a, M);
    }
#undef HK_BSTAMP
}

// The augmented row's terms (AUG) and the gain block (KGEN) of chol_block<B>, formed after the fact from the
// block's final factor S[B] (upper storage: lane c of row group j holds y_j = L[c][4B+j]) and the pivots' inverse
// diagonal (lane 4B+j holds i_j): the same operations on the same operands as chol_block, so ml and kg are bitwise
// chol_block's.  The multi-wave solo kernel runs the tile half of the factorisation on one wave and this row half
// one stage behind on another (hk_mw.h).
template <int B, bool AUG, bool KGEN>
__device__ __forceinline__ void chol_block_row(const d4& S, double invd, double& ml, double* kg) {
    const int l = lane_id(), c = l & 15;
    double y[4];
    rowgroup_gather(S[B], y);
    const double i0 = row_bcast<4 * B + 0>(invd), i1 = row_bcast<4 * B + 1>(invd);
    const double i2 = row_bcast<4 * B + 2>(invd), i3 = row_bcast<4 * B + 3>(invd);
    const double l10 = row_bcast<4 * B + 1>(y[0]), l20 = row_bcast<4 * B + 2>(y[0]), l30 = row_bcast<4 * B + 3>(y[0]);
    const double l21 = row_bcast<4 * B + 2>(y[1]), l31 = row_bcast<4 * B + 3>(y[1]);
    const double l32 = row_bcast<4 * B + 3>(y[2]);
    if (KGEN && B == 0) {
        const bool ut = c < 4;
        const double e0 = ut ? (c == 0 ? 1.0 : 0.0) : y[0], e1 = ut ? (c == 1 ? 1.0 : 0.0) : y[1];
        const double e2 = ut ? (c == 2 ? 1.0 : 0.0) : y[2], e3 = ut ? (c == 3 ? 1.0 : 0.0) : y[3];
        const double z3 = e3 * i3;
        const double z2 = fma(-l32, z3, e2) * i2;
        const double z1 = fma(-l31, z3, fma(-l21, z2, e1)) * i1;
        const double z0 = fma(-l30, z3, fma(-l20, z2, fma(-l10, z1, e0))) * i0;
        *kg = -sel_g(z0, z1, z2, z3);
    }
    if (AUG) {
        const double m0 = row_bcast<4 * B + 0>(ml), m1 = row_bcast<4 * B + 1>(ml);
        const double m2 = row_bcast<4 * B + 2>(ml), m3 = row_bcast<4 * B + 3>(ml);
        const double p0 = m0 * i0;
        const double p1 = fma(-p0, l10, m1) * i1;
        const double p2 = fma(-p1, l21, fma(-p0, l20, m2)) * i2;
        const double p3 = fma(-p2, l32, fma(-p1, l31, fma(-p0, l30, m3))) * i3;
        const bool inb = (c >> 2) == B, below = c > 4 * B + 3;
        const double mt = fma(-p3, y[3], fma(-p2, y[2], fma(-p1, y[1], fma(-p0, y[0], ml))));
        const double mb = sel_q(p0, p1, p2, p3);
        ml = below ? mt : (inb ? mb : ml);
    }
}

// stage_chol's row half over the blocks it factorised (same block conditions)
template <bool AUG, bool KGEN>
__device__ __forceinline__ void stage_chol_row(const d4& S, double invd, double& ml, int nu, int nx, int xo, bool full,
                                               double* kg) {
    const int hi = full ? xo + nx : nu;
    if (0 < nu || (full && 3 >= xo && 0 < hi)) chol_block_row<0, AUG, KGEN>(S, invd, ml, kg);
    if (4 < nu || (full && 7 >= xo && 4 < hi)) chol_block_row<1, AUG, false>(S, invd, ml, nullptr);
    if (8 < nu || (full && 11 >= xo && 8 < hi)) chol_block_row<2, AUG, false>(S, invd, ml, nullptr);
    if (12 < nu || (full && 15 >= xo && 12 < hi)) chol_block_row<3, AUG, false>(S, invd, ml, nullptr);
}

// ------------------------------------------------------------------------------------------------
// The reference's inner-stage x-pivot clamp on the P form (kernel_dpotrf_c99_lib4.c:555-640, SURVEY.md
// Appendix C).  The reference factorises every stage completely and clamps a pivot d <= 1e-15 to 0 (its column of
// L becomes 0), so what it carries to the next stage is not P_k but P_eff = Lxx Lxx' and p_eff = Lxx l_x of the
// clamped factor.  Without a clamp the two are the same quantity (the P form below); with one they differ by the
// dropped rank-one term.  A stage therefore keeps the cheap P form only when a certificate shows that none of the
// reference's x pivots can reach the clamp, and otherwise factorises its x block as the reference does and stores
// P_eff / p_eff in the record instead of P / p (all consumers of the record read P and p only).
//
// The certificate (per stage, per factorisation):
//   g  = Gershgorin lower bound of the stage's DATA block RSQ_k (min_i M_ii - sum_{j != i} |M_ij| over the active
//        rows): every later term (box Hessian >= 0, DCt diag(Q) DCt' >= 0, BAbt P_{k+1} BAbt' >= 0 -- the
//        reference's W W' is an exact Gram product of its own W) only raises the smallest eigenvalue, and every
//        Cholesky pivot of the full stage matrix -- the x pivots are those of the Schur complement -- is at least
//        M_ii lambda_min(D^-1/2 M D^-1/2) >= M_ii g / e_max, with e_max = max_i (M_ii - box_i) (the box terms are
//        diagonal and cancel from that ratio);
//   the reference's computed pivots are exact pivots of M + dM with |dM_ij| <= c n eps sqrt(M_ii M_jj) (Cholesky's
//        componentwise backward error; the reference's own M differs from ours by rounding of the same order), so
//        with 1e-11 >> 16 n eps as the allowance the certificate is  g (g / e_max - 1e-11) > 1e-15, i.e.
//        e_max (1e-11 g + 1e-15) < g^2 with g > 0.
// g depends on the data only: an IPM solve forms it in its first factorisation (from the data tiles that pass loads
// anyway) and its later factorisations load it; the Riccati entry points form it per stage (cert_g).  The e_max test is one product and compare per diagonal
// entry and a ballot.
// ------------------------------------------------------------------------------------------------
// The tile's diagonal entry held by this lane: lane (g,c) holds element (g+4r, c) of register r, so it holds the
// diagonal entry (c, c) iff c % 4 == g, in register c / 4 (callers mask the other lanes with diag_lane()).
__device__ __forceinline__ double diag_sel(const d4& v) {
    const int c = lane_id() & 15;
    const bool b0 = (c & 4) != 0, b1 = (c & 8) != 0;
    const double lo = b0 ? v[1] : v[0], hi = b0 ? v[3] : v[2];
    return b1 ? hi : lo;
}
__device__ __forceinline__ bool diag_lane() {
    const int l = lane_id();
    return (l & 3) == (l >> 4);
}

// Wave minimum of a double to a conservative f32 bound (<= the exact minimum): one DPP-sourced f32 min per row step
// (v_min_f32 with its first operand read through row_ror: no separate move, no NaN canonicalisation) and two row-group
// swaps instead of the f64 butterfly; the certificate needs a bound, not the exact value.
__device__ __forceinline__ double wave_min_lb(double x) {
    float f = (float)x;  // round to nearest, then step down one ulp-ish so that f <= x
    f = f - fabsf(f) * 0x1p-22f - 0x1p-126f;
    asm volatile(
        "s_nop 1\n\t"
        "v_min_f32_dpp %0, %0, %0 row_ror:8 row_mask:0xf bank_mask:0xf\n\t"
        "s_nop 1\n\t"
        "v_min_f32_dpp %0, %0, %0 row_ror:4 row_mask:0xf bank_mask:0xf\n\t"
        "s_nop 1\n\t"
        "v_min_f32_dpp %0, %0, %0 row_ror:2 row_mask:0xf bank_mask:0xf\n\t"
        "s_nop 1\n\t"
        "v_min_f32_dpp %0, %0, %0 row_ror:1 row_mask:0xf bank_mask:0xf"
        : "+v"(f));
    int v = __builtin_bit_cast(int, f);
    const auto a = __builtin_amdgcn_permlane32_swap(v, v, false, false);
    f = __builtin_fminf(__builtin_bit_cast(float, (int)a[0]), __builtin_bit_cast(float, (int)a[1]));
    v = __builtin_bit_cast(int, f);
    const auto b = __builtin_amdgcn_permlane16_swap(v, v, false, false);
    return (double)__builtin_fminf(__builtin_bit_cast(float, (int)b[0]), __builtin_bit_cast(float, (int)b[1]));
}

// Gershgorin's g of a stage from its data tile Mi (symmetric -- load_rsq_tile mirrors the lower triangle -- and zero
// outside the active rows / columns): the absolute row sums are column sums, so a lane adds its four registers and
// the four row groups are summed across (xrow_sum): a handful of VALU ops instead of four f64 MFMAs against a ones
// operand (64 cycles of the matrix pipe each on gfx950).  Then the diagonal margin on the lane that holds the diagonal
// entry and a wave minimum (as a conservative f32 bound).  cert_g (after stage_chol below) falls back to a shifted
// Cholesky where this bound is not positive.
template <class SH>
__device__ __forceinline__ double cert_g_gersh(const d4& Mi, const SH& sh) {
    const int c = lane_id() & 15;
    const double rs = xrow_sum((fabs(Mi[0]) + fabs(Mi[1])) + (fabs(Mi[2]) + fabs(Mi[3])));
    const double d = diag_sel(Mi);
    const double m = (diag_lane() && tile_active(c, sh.nu, sh.nx, sh.xo)) ? d + fabs(d) - rs : 1e300;
    return wave_min_lb(m);
}

#ifdef HK_STAMPS
// P-form stages tested, failed at CERT_ALLOW, at 1e-12, at 1e-13; backward sweeps, sweeps with a failed stage
__device__ unsigned long long g_xfac_stat[6];
__device__ unsigned g_xfac_sweep[1 << 16];  // per workgroup: this sweep has failed a stage (one wave per workgroup)
#endif
constexpr double CERT_ALLOW = 1e-11;  // the backward-error allowance (>> 16 n eps, n = 16)

// The certificate on the stage matrix M (after the tile update, before the factorisation): g > 0 and, on every
// diagonal entry, (M_ii - dq_i) (1e-11 g + 1e-15) < g^2 -- i.e. g (g / e_max - 1e-11) > 1e-15 without a division.
// Wave-uniform (ballot of the failing lanes).
__device__ __forceinline__ bool cert_ok(const d4& M, double dq, double gc, double allow = CERT_ALLOW) {
    const double cc = fma(allow, gc, 1e-15), g2 = gc * gc;
    // a negative given box term (BX_GIVEN) is not covered by the bound: no certificate
    const bool bad = !(gc > 0.0) || dq < 0.0 || (diag_lane() && !((diag_sel(M) - dq) * cc < g2));
    return __builtin_amdgcn_ballot_w64(bad) == 0;
}

// The same test in threshold form, for the IPM's factorisations, whose bounds are formed once per solve: the stage
// stores T = g^2 / (1e-11 g + 1e-15) (cert_thr; -inf when g <= 0, rounded down by 2^-40 so that e < T implies the
// division-free test above), and the test is max_i (M_ii - dq_i) < T.  The diagonal entry comes from per-lane 0/1
// weights (cert_diag_w, loop-invariant VGPRs) instead of lane-mask selects: no SGPR mask stays live across the
// stage loop, and lanes without a diagonal entry test -dq_c < T, which holds whenever the stage can pass at all.
// (dq >= 0 in these modes: it is a sum of lam / t terms.)
__device__ __forceinline__ double cert_thr(double g) {
    const double T = (g * g) * rcp_nr(fma(CERT_ALLOW, g, 1e-15)) * (1.0 - 0x1p-40);
    return g > 0.0 ? T : -__builtin_inf();
}
__device__ __forceinline__ d4 cert_diag_w() {
    const int l = lane_id(), g = l >> 4, c = l & 15;
    d4 w;
#pragma unroll
    for (int r = 0; r < 4; r++) w[r] = (c == g + 4 * r) ? 1.0 : 0.0;
    return w;
}
__device__ __forceinline__ bool cert_ok_thr(const d4& M, double dq, double T, const d4& w) {
    const double d = w[0] * M[0] + w[1] * M[1] + w[2] * M[2] + w[3] * M[3];
    return __builtin_amdgcn_ballot_w64(!(d - dq < T)) == 0;
}

// The stage's data part of the certificate, the threshold T_k (a negative given box term folded into T_k = -inf).
// (A test off the chain, on the trace of the record the stage starts from against a data threshold tau_k, measured
// slower in every kernel in round 5: profiles/r05/ab_cert/)
template <class SH>
__device__ __forceinline__ double cert_form(const d4& Mi, double dq, const SH& sh) {
    const double T = cert_thr(cert_g(Mi, sh));
    return __builtin_amdgcn_ballot_w64(dq < 0.0) != 0 ? -__builtin_inf() : T;
}
// The per-stage test on the stage matrix M after its products.
__device__ __forceinline__ bool cert_test(const d4& M, double dq, double gc) {
    return cert_ok_thr(M, dq, gc, cert_diag_w());
}

// l[4R + g] (row layout of a col-layout vector over tile block R): the pivot entries of block R
template <int R>
__device__ __forceinline__ double lrow_blk(double v) {
    return sel_g(row_bcast<4 * R + 0>(v), row_bcast<4 * R + 1>(v), row_bcast<4 * R + 2>(v), row_bcast<4 * R + 3>(v));
}

// The x columns of the factor as MFMA operands: lane (g,c) of block R holds L[c][4R+g] (upper storage, c >= 4R+g)
// for the x pivots 4R+g >= xo, zero elsewhere.
__device__ __forceinline__ double xcol_op(const d4& L, int R, int xo) {
    const int l = lane_id(), g = l >> 4, c = l & 15;
    const int p = 4 * R + g;
    return (p >= xo && c >= p) ? L[R] : 0.0;
}

// P_eff = Lxx Lxx' (one MFMA per x block, A = B = the block's columns of L) written over the x block of M (both
// triangles).
__device__ __forceinline__ void pform_eff_tile(const d4& L, int nx, int xo, d4& M) {
    const int l = lane_id(), g = l >> 4, c = l & 15;
    const d4 z = {0.0, 0.0, 0.0, 0.0};
    d4 Pe = z;
#pragma unroll
    for (int R = 0; R < 4; R++) {
        if (4 * R + 3 < xo || 4 * R >= xo + nx) continue;  // uniform
        const double a = xcol_op(L, R, xo);
        Pe = mfma(a, a, Pe);
    }
#pragma unroll
    for (int r = 0; r < 4; r++) M[r] = (g + 4 * r >= xo && c >= xo) ? Pe[r] : M[r];
}

// p_eff = Lxx l_x (col layout) written over the x part of ml; lx holds the clamped factor's row l (x part).
__device__ __forceinline__ void pform_eff_row(const d4& L, double lx, int nx, int xo, double& ml) {
    const int c = lane_id() & 15;
    double part = 0.0;
    if (4 * 0 + 3 >= xo && 0 < xo + nx) part += xcol_op(L, 0, xo) * lrow_blk<0>(lx);
    if (4 * 1 + 3 >= xo && 4 < xo + nx) part += xcol_op(L, 1, xo) * lrow_blk<1>(lx);
    if (4 * 2 + 3 >= xo && 8 < xo + nx) part += xcol_op(L, 2, xo) * lrow_blk<2>(lx);
    if (4 * 3 + 3 >= xo && 12 < xo + nx) part += xcol_op(L, 3, xo) * lrow_blk<3>(lx);
    const double pe = xrow_sum(part);
    ml = c >= xo ? pe : ml;
}

// The x-block factorisation of a stage whose u pivots are done (the reference's remaining dsyrk_dpotrf pivots,
// with the same clamp): M (in: u rows factorised, x block = P; out: x rows = upper storage of Lxx), ml (x part: p ->
// l_x), invd (x pivots' inverse diagonal added).
template <bool AUG>
__device__ __forceinline__ void xblocks_chol(d4& M, double& ml, double& invd, int nx, int xo) {
    const int hi = xo + nx;
    if (0 >= xo && 0 < hi) chol_block<0, AUG>(M, ml, invd);
    if (4 >= xo && 4 < hi) chol_block<1, AUG>(M, ml, invd);
    if (8 >= xo && 8 < hi) chol_block<2, AUG>(M, ml, invd);
    if (12 >= xo && 12 < hi) chol_block<3, AUG>(M, ml, invd);
}

// Its row half on another wave (hk_mw.h: the row recursion), from the x factor L and its inverse diagonal.
__device__ __forceinline__ void xblocks_chol_row(const d4& L, double invd, double& ml, int nx, int xo) {
    const int hi = xo + nx;
    if (0 >= xo && 0 < hi) chol_block_row<0, true, false>(L, invd, ml, nullptr);
    if (4 >= xo && 4 < hi) chol_block_row<1, true, false>(L, invd, ml, nullptr);
    if (8 >= xo && 8 < hi) chol_block_row<2, true, false>(L, invd, ml, nullptr);
    if (12 >= xo && 12 < hi) chol_block_row<3, true, false>(L, invd, ml, nullptr);
}

// What a clamped stage hands the row recursion of the multi-wave kernel: the x factor and its inverse diagonal.
struct XFac {
    d4 L;
    double invd;
};

// Stage factorisation with the augmented row.
// In : M (tile, full symmetric), ml (aug row, col layout).
// full == true : the whole stage Cholesky (d_back_ric_rec.c:325, dsyrk_dpotrf_lib), M = S = lower(L) +
//                strict_upper(L'), ml = l, invd = inverse diagonal of every pivot.
// full == false: "P form" -- only the u pivots are factorised.  The rank-|u| trailing update that the last
//                u block applies leaves the Schur complement P_k = M_xx - L_xu L_xu' in the x block and
//                p_k = m_x - L_xu l_u in the x part of ml: exactly the value function's Hessian and gradient
//                that the reference carries as Lxx Lxx' and Lxx l_x (:262-276 multiply them back), so the
//                x pivots (and their triangular factor) are never needed on stages k >= 1: the next
//                stage uses P and p directly (M += BAbt P BAbt', ml += BAbt (P b + p)), pi = P x + p, and
//                the trs / KKT recursions only ever solve the u pivots.  Stage 0 keeps the full factor (its
//                forward may solve for x_0 too).  u-block rows keep L's columns in upper storage (row p of S
//                == column p of L, p < nu), invd holds the u pivots only.
// Generic shapes restore the lower triangle by an identity-MFMA transpose (L_xu for the generic forward,
// and P symmetrised); fixed shapes skip it (their consumers read the upper u rows and the P block only).
// xfac (P form only, wave-uniform): the stage failed the clamp certificate (cert_ok) -- its x block is factorised
// as the reference does and the record carries P_eff = Lxx Lxx' and p_eff = Lxx l_x (the x factor and its inverse
// diagonal also go to *xf when given); invd keeps the u pivots only, as in every P-form record.
template <bool AUG, bool KGEN = false>
__device__ __forceinline__ void stage_chol(d4& M, double& ml, double& invd, int nu, int nx, int xo, bool full,
                                           bool transpose, double* kg = nullptr, int kdbg = -1, bool xfac = false,
                                           XFac* xf = nullptr) {
    const int l = lane_id(), g = l >> 4, c = l & 15;
    (void)kdbg;
    invd = 0.0;
    // blocks without an active pivot are skipped (wave-uniform); their rows/columns are zero
    const int hi = full ? xo + nx : nu;  // pivots [0, hi) are factorised (padding ones clamp to 0)
    if (0 < nu || (full && 3 >= xo && 0 < hi)) chol_block<0, AUG, KGEN>(M, ml, invd, kg, kdbg);
    HK_STAMP(16, kdbg);
    if (4 < nu || (full && 7 >= xo && 4 < hi)) chol_block<1, AUG>(M, ml, invd, nullptr, kdbg);
    HK_STAMP(18, kdbg);
    if (8 < nu || (full && 11 >= xo && 8 < hi)) chol_block<2, AUG>(M, ml, invd, nullptr, kdbg);
    HK_STAMP(20, kdbg);
    if (12 < nu || (full && 15 >= xo && 12 < hi)) chol_block<3, AUG>(M, ml, invd, nullptr, kdbg);
    HK_STAMP(22, kdbg);
    const bool xf_now = xfac;
#ifdef HK_COUNT_NOFALLBACK  // static instruction counts of the certified path (tools/loop_icount.py): the test stays,
    // the clamped factorisation is compiled out
    asm volatile("" ::"s"(__builtin_amdgcn_readfirstlane((int)xf_now)));
    if (false) {
#else
    if (!full && xf_now) {
#endif
        d4 L = M;
        double lx = ml, ivx = invd;
        xblocks_chol<AUG>(L, lx, ivx, nx, xo);
        pform_eff_tile(L, nx, xo, M);
        if (AUG) pform_eff_row(L, lx, nx, xo, ml);
        if (xf) {
            xf->L = L;
            xf->invd = ivx;
        }
    }
    if (!transpose) return;
    // lower triangle <- transpose of the upper storage:  T = S' via MFMA with an identity B operand
    // (two accumulator chains: the identity products are exact, so the split does not change T)
    const d4 z = {0.0, 0.0, 0.0, 0.0};
    d4 T0 = mfma(M[0], (c == g) ? 1.0 : 0.0, z);
    d4 T1 = mfma(M[1], (c == 4 + g) ? 1.0 : 0.0, z);
    T0 = mfma(M[2], (c == 8 + g) ? 1.0 : 0.0, T0);
    T1 = mfma(M[3], (c == 12 + g) ? 1.0 : 0.0, T1);
    const d4 T = T0 + T1;
#pragma unroll
    for (int r = 0; r < 4; r++) M[r] = (g + 4 * r > c) ? T[r] : M[r];
}

// A sharper lower bound on lambda_min of the data block where Gershgorin's is not positive (strongly coupled stage
// Hessians, e.g. Q = G G' / n + I: every such stage used to fail the certificate and take the clamped x-block
// factorisation).  tau = 2^-10 max_i Mi_ii; a Cholesky of Mi - tau I that keeps every active pivot
// above the clamp proves lambda_min(Mi) >= tau - (eps + n gamma_{n+1}) max_i Mi_ii: the computed factor is the exact
// factor of Mi - tau I + E with |E_ij| <= gamma_{n+1} sqrt(a_ii a_jj) (Cholesky's componentwise backward error), so
// ||E||_2 <= n gamma_{n+1} max_i a_ii ~ 3e-14 max_i Mi_ii at n = 16; 1e-12 max_i Mi_ii is subtracted.  Any lower bound
// on lambda_min(RSQ_k) can stand in for Gershgorin's g in the certificate (its derivation only uses that one).
// Returns -1 (no bound) when the shifted factorisation clamps a pivot.  Wave-uniform.
template <class SH>
__device__ __forceinline__ double cert_g_shift(const d4& Mi, const SH& sh) {
    const int l = lane_id(), g = l >> 4, c = l & 15;
    const bool act = tile_active(c, sh.nu, sh.nx, sh.xo);
    const double dm = -wave_min((diag_lane() && act) ? -diag_sel(Mi) : 0.0);  // max_i Mi_ii (exact)
    const double tau = dm * 0x1p-10;
    d4 A = Mi;
#pragma unroll
    for (int r = 0; r < 4; r++) A[r] -= (g + 4 * r == c && act) ? tau : 0.0;
    double ml = 0.0, invd = 0.0;
    stage_chol<false, false>(A, ml, invd, sh.nu, sh.nx, sh.xo, true, false);
    const bool ok = dm > 0.0 && __builtin_amdgcn_ballot_w64(act && !(invd > 0.0)) == 0;
    return ok ? tau - 1e-12 * dm : -1.0;
}

// The certificate's data part: a lower bound g on the smallest eigenvalue of the stage's data block RSQ_k -- Gershgorin's,
// or where that one is not positive the shifted-Cholesky bound (wave-uniform branch; the benchmark data never take it).
template <class SH>
__device__ __forceinline__ double cert_g(const d4& Mi, const SH& sh) {
    const double g = cert_g_gersh(Mi, sh);
#ifdef HK_COUNT_NOSHIFT  // static instruction counts of the Gershgorin path alone (tools/loop_icount.py)
    return g;
#endif
    if (g > 0.0) return g;
    return cert_g_shift(Mi, sh);
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
    const double* BAbtS;          // the batch's BAbt / RSQrq base: a stage block shared by every problem (StageInfo
    const double* RSQS;           // r0 bits 1 / 2) sits at BAbtS + oB / RSQS + oR
    double* F;                    // factor store (N+1)*FSTRIDE (private layout)
    const double* DCt;            // this problem's general-constraint base (stage k block at st[k].oG)
};

// Stage record from the LDS table, forced into SGPRs (readfirstlane) so that every address derived
// from it is provably wave-uniform (otherwise hipcc wraps each buffer op in a waterfall loop).
__device__ __forceinline__ StageInfo load_stage(const StageInfo* st, int k) {
    const StageInfo v = st[k];
    StageInfo u;
    u.nu = __builtin_amdgcn_readfirstlane(v.nu);
    u.nx = __builtin_amdgcn_readfirstlane(v.nx);
    u.nb = __builtin_amdgcn_readfirstlane(v.nb);
    u.ng = __builtin_amdgcn_readfirstlane(v.ng);
    u.xo = __builtin_amdgcn_readfirstlane(v.xo);
    u.nx1 = __builtin_amdgcn_readfirstlane(v.nx1);
    u.nu1 = __builtin_amdgcn_readfirstlane(v.nu1);
    u.xo1 = __builtin_amdgcn_readfirstlane(v.xo1);
    u.sdB = __builtin_amdgcn_readfirstlane(v.sdB);
    u.sdR = __builtin_amdgcn_readfirstlane(v.sdR);
    u.oB = __builtin_amdgcn_readfirstlane(v.oB);
    u.oR = __builtin_amdgcn_readfirstlane(v.oR);
    u.oD = __builtin_amdgcn_readfirstlane(v.oD);
    u.pnb = __builtin_amdgcn_readfirstlane(v.pnb);
    u.r0 = __builtin_amdgcn_readfirstlane(v.r0);  // stage belongs to the compiled inner class
    u.oG = __builtin_amdgcn_readfirstlane(v.oG);
    return u;
}

// A stage of the LDS table by reference: the shape objects below read (readfirstlane) only the fields they use, where
// they are built, so a stage loop does not hold a whole StageInfo in SGPRs across its body (the compiled-class path
// needs five fields; the full record would add some thirty live SGPRs per loop, and the stage kernels run at the
// SGPR limit, spilling to VGPR lanes).
struct StageRef {
    const StageInfo* p;
    int k;
};
__device__ __forceinline__ int srd(const StageRef& s, int StageInfo::*m) {
    return __builtin_amdgcn_readfirstlane(s.p[s.k].*m);
}

// ------------------------------------------------------------------------------------------------
// Stage-shape policies.  Every per-stage routine is written once against a shape object `sh`:
//   DynSh          -- all sizes from the stage table (any problem the plan accepts);
//   FixSh<NU, NX>  -- the batch's uniform inner stages (1 <= k <= N-2: nu = NU, nx = NX, next stage
//                     the same), sizes as compile-time constants, so every tile mask, loop bound and
//                     "is this pivot active" test folds away.
// A kernel compiled for FixSh<NU,NX> takes the constant path on every stage the host flagged
// (StageInfo.r0) and the runtime path elsewhere (first / last stages, irregular problems).
// ------------------------------------------------------------------------------------------------
struct DynSh {
    static constexpr bool fixed = false;
    int nu, nx, xo, nx1, nu1, xo1, sdB, sdR, nb, pnb, oB, oR, ng, oG, fl;
    __device__ __forceinline__ explicit DynSh(const StageInfo& s)
        : nu(s.nu), nx(s.nx), xo(s.xo), nx1(s.nx1), nu1(s.nu1), xo1(s.xo1), sdB(s.sdB), sdR(s.sdR), nb(s.nb),
          pnb(s.pnb), oB(s.oB), oR(s.oR), ng(s.ng), oG(s.oG), fl(s.r0) {}
    __device__ __forceinline__ explicit DynSh(const StageRef& s)
        : nu(srd(s, &StageInfo::nu)), nx(srd(s, &StageInfo::nx)), xo(srd(s, &StageInfo::xo)),
          nx1(srd(s, &StageInfo::nx1)), nu1(srd(s, &StageInfo::nu1)), xo1(srd(s, &StageInfo::xo1)),
          sdB(srd(s, &StageInfo::sdB)), sdR(srd(s, &StageInfo::sdR)), nb(srd(s, &StageInfo::nb)),
          pnb(srd(s, &StageInfo::pnb)), oB(srd(s, &StageInfo::oB)), oR(srd(s, &StageInfo::oR)),
          ng(srd(s, &StageInfo::ng)), oG(srd(s, &StageInfo::oG)), fl(srd(s, &StageInfo::r0)) {}
};

template <int NU, int NX>
struct FixSh {
    static constexpr bool fixed = true, enabled = true;
    static constexpr int nu = NU, nx = NX, xo = (NU + 3) / 4 * 4, nx1 = NX, nu1 = NU, xo1 = xo,
                         sdB = (NX + 1) / 2 * 2, sdR = (NU + NX + 1) / 2 * 2;
    int nb, pnb, oB, oR, fl;
    __device__ __forceinline__ explicit FixSh(const StageInfo& s)
        : nb(s.nb), pnb(s.pnb), oB(s.oB), oR(s.oR), fl(s.r0) {}
    __device__ __forceinline__ explicit FixSh(const StageRef& s)
        : nb(srd(s, &StageInfo::nb)), pnb(srd(s, &StageInfo::pnb)), oB(srd(s, &StageInfo::oB)),
          oR(srd(s, &StageInfo::oR)), fl(srd(s, &StageInfo::r0)) {}
};


// The stage's data blocks: per problem, or shared by the batch (StageInfo r0 bits 1 / 2; wave-uniform selects).
__device__ __forceinline__ int stage_flags(const StageInfo& s) { return s.r0; }
template <class SH>
__device__ __forceinline__ int stage_flags(const SH& s) { return s.fl; }
template <class SH>
__device__ __forceinline__ const double* stage_B(const RicIO& io, const SH& sh) {
    return ((stage_flags(sh) & 2) ? io.BAbtS : io.BAbt) + sh.oB;
}
template <class SH>
__device__ __forceinline__ const double* stage_R(const RicIO& io, const SH& sh) {
    return ((stage_flags(sh) & 4) ? io.RSQS : io.RSQ) + sh.oR;
}

struct NoFix {  // generic kernels: no compile-time stage class
    static constexpr bool enabled = false;
    __device__ __forceinline__ explicit NoFix(const StageInfo&) {}
    __device__ __forceinline__ explicit NoFix(const StageRef&) {}
};

// Run f(sh) with the stage's shape object: the constant one when the stage belongs to FX's class.
template <class FX, class F>
__device__ __forceinline__ void with_shape(const StageInfo& s, F&& f) {
#ifdef HK_COUNT_FIXED
    if constexpr (FX::enabled) { f(FX(s)); return; }
#endif
    if constexpr (FX::enabled) {
        if (s.r0 & 1) {
            f(FX(s));
            return;
        }
    }
    f(DynSh(s));
}
template <class FX, class F>
__device__ __forceinline__ void with_shape(const StageRef& s, F&& f) {
#ifdef HK_COUNT_FIXED
    if constexpr (FX::enabled) { f(FX(s)); return; }
#endif
    if constexpr (FX::enabled) {
        if (srd(s, &StageInfo::r0) & 1) {
            f(FX(s));
            return;
        }
    }
    f(DynSh(s));
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

// factor record of one stage: 4 tile registers in register order (4 x 512 B coalesced), l, inv_diag
// (ok == false still issues the six stores, out of range, so that every path through a stage loop has
// the same number of vector-memory ops and the compiler's counted s_waitcnt stays exact)
__device__ __forceinline__ void store_factor(double* Fk, const d4& S, double lc, double invd, double kg,
                                             bool ok = true) {
    const int l = lane_id(), g = l >> 4, c = l & 15;
#pragma unroll
    for (int r = 0; r < 4; r++) gst(Fk, r * 64 + l, S[r], ok);
    gst(Fk, 256 + 16 * g + c, g == 0 ? lc : invd, ok && g < 2);  // l (row group 0) and inv_diag (row group 1)
    gst(Fk, 288 + l, kg, ok);
}

// Packed record of a compiled-class stage (nu <= 4, so the u block is tile block 0 and the state block starts at
// tile index xo = 4).  What the solves read of it, and nothing else:
//   [0, 64)    unused (was S0, the u columns of L: the trs u solve now runs in gain form on KG, trs_usolve)
//   [64, 80)   l = [l_u; p_k] (the sv forward's right-hand side; pi's p_{k+1})
//   [80, 96)   the u pivots' inverse diagonal (stored with l by one instruction; no compiled-class solve reads it)
//   [96, 160)  the gain block KG (4 x 16, the forward's u = KG [rhs_u; x])
//   [160, ..)  P_k, the state block, packed lower by rows (NX (NX+1) / 2 doubles; symmetric, so the tile's upper
//              half is not stored): 1 392 B against the 2 816 B of the full record at nx = 12 (S1..S3 are 1 536 B
//              of which 1 152 B hold P in both triangles)
constexpr int FXR_L = 64, FXR_INVD = 80, FXR_KG = 96, FXR_P = 160;

// element (i, j) of the packed-lower P block (either triangle)
__device__ __forceinline__ int fxr_pidx(int i, int j) {
    const int a = i > j ? i : j, b = i > j ? j : i;
    return FXR_P + (a * (a + 1) >> 1) + b;
}

// Store of a packed record (same six stores as store_factor: the vector-memory count per stage stays fixed).
template <int NX>
__device__ __forceinline__ void store_factor_fixed(double* Fk, const d4& S, double lc, double invd, double kg,
                                                   bool ok) {
    const int l = lane_id(), g = l >> 4, c = l & 15;
    // S0 is not stored (every solve of a compiled-class stage runs its u block in gain form: fwd_step, trs_usolve);
    // the masked store keeps the per-stage vector-memory count of store_factor
    gst(Fk, l, S[0], false);
    gst(Fk, FXR_L + 16 * g + c, g == 0 ? lc : invd, ok && g < 2);
    gst(Fk, FXR_KG + l, kg, ok);
    const int j = c - 4;
#pragma unroll
    for (int r = 1; r < 4; r++) {  // lane (g, c) of tile register r holds P[g + 4r - 4][c - 4] (c >= 4)
        const int i = g + 4 * r - 4;
        gst(Fk, fxr_pidx(i, j), S[r], ok && j >= 0 && j <= i && i < NX);
    }
}

// Tile registers 1..3 (the state rows) of a packed record: P in the tile layout (lanes c < 4 read 0).
template <int NX>
__device__ __forceinline__ void load_p_fixed(const double* Fk, d4& S, bool ok) {
    const int l = lane_id(), g = l >> 4, c = l & 15;
    const int j = c - 4;
#pragma unroll
    for (int r = 1; r < 4; r++) {
        const int i = g + 4 * r - 4;
        S[r] = gld(Fk, fxr_pidx(i, j), ok && j >= 0 && i < NX && j < NX);
    }
}

// ------------------------------------------------------------------------------------------------
// IPM box terms fused into the stage passes (mpc_solvers/c99/d_aux_ip_hard_lib4.c).  Instead of
// separate element-wise passes over all stages (each paying a full memory round trip per stage), the
// box-constraint vectors of stage k are prefetched together with the stage's Riccati data and
// combined where the stage pass needs them:
//   backward (sv)  : Hessian / gradient terms   d_update_hessian_[res_]mpc_hard_tv
//   forward        : step, dual step and alpha  d_compute_alpha_[res_]mpc_hard_tv
//   backward (trs) : corrector gradient         d_update_gradient_[res_]mpc_hard_tv (+ centering)
// A lane of tile column c handles the box attached to tile index c (if any); row group 0 stores.
// ------------------------------------------------------------------------------------------------
// BX_P2R: BX_P2 whose update rows are the residuals r_q, r_b of the current iterate, computed (and
// stored) inside the backward pass instead of by a separate residual pass (backward only).
enum BoxMode { BX_NONE = 0, BX_GIVEN = 1, BX_P1 = 2, BX_P2 = 3, BX_P2R = 4 };

// the IPM's box modes read the certificate bound g that the solve's init formed (cert_pass); the others form it
constexpr bool cert_loaded(int bm) { return bm == BX_P1 || bm == BX_P2 || bm == BX_P2R; }

struct BoxCtx {
    const double* d;                                   // bounds [lb (pnb) | ub (pnb)], V32 per stage
    double *lam, *t;                                   // iterate (V32)
    double *dlam, *dt, *t_inv, *lamt, *res_d, *res_m;  // IPM work vectors (V32)
    double* qxs;                                       // phase-1 gradient (V16, slot order)
    const double *Qx, *qx;                             // BX_GIVEN terms (V16, slot order)
    double smu;                                        // centering target of the trs box modes
    int pred;                                          // forward BX_P1: predictor step (dlam = 0)
    // BX_P2R: iterate, residual outputs, and whether the residuals (1) or the data rows (0) are the
    // right-hand side of the factorisation
    const double *ux, *pi;
    double *res_q, *res_b;
    int res_rhs;
    // BX_P2 / BX_P2R: the factorisation skips its t^-1 store (queue API: the solves re-form 1/t from t, and
    // only the KKT re-solve and the general-constraint halves load it; wave-uniform)
    int no_tinv;
    // the clamp certificate's data part g per stage, for the IPM's factorisations (BX_P1 / BX_P2 / BX_P2R): the first
    // factorisation of a solve forms it from the data tiles it loads anyway (cert_new, wave-uniform) and stores it to
    // cert_out; the later ones read it from cert (staged in LDS by fact_body, the workspace in the multi-wave kernel)
    const double* cert;
    double* cert_out;
    int cert_new;
};

struct BoxLane {
    int lo, up, s16;  // element indices of this lane's box in the V32 / V16 arrays
    bool ok;          // tile index c carries a box
};

__device__ __forceinline__ BoxLane box_lane(const signed char* tileslot, int pnb, int k) {
    const int c = lane_id() & 15;
    const int slot = tileslot[k * 16 + c];
    BoxLane b;
    b.ok = slot >= 0;
    b.lo = k * V32 + slot;
    b.up = b.lo + pnb;
    b.s16 = k * V16 + slot;
    return b;
}

// A box pair's lower and upper value with ONE load: row groups 0/2 read the lower slot, 1/3 the upper one,
// and one v_permlane16_swap per dword gives every lane both (after the swap, [0] holds the even row's dword
// and [1] the odd row's, in all lanes -- the order rowgroup_gather relies on).  Rows g and g^1 have the same
// c, so the same box and mask; a masked lane reads 0 like ldsel.
__device__ __forceinline__ void ld_lu(const double* p, const BoxLane& b, double& vlo, double& vup) {
    const bool odd = (lane_id() & 16) != 0;
    // the slot by a bit mask: a select between the two fields was lowered to a stack round trip
    const int m = -(int)odd;
    const double x = gld(p, (b.up & m) | (b.lo & ~m), b.ok);
    const int xl = __double2loint(x), xh = __double2hiint(x);
    const auto cl = __builtin_amdgcn_permlane16_swap(xl, xl, false, false);
    const auto ch = __builtin_amdgcn_permlane16_swap(xh, xh, false, false);
    vlo = mk((int)ch[0], (int)cl[0]);
    vup = mk((int)ch[1], (int)cl[1]);
}

// The solves' prefetched fragments load a box pair's lower and upper value separately: a paired load (ld_lu) needs its
// exchange at the use, and a same-box A/B measured that 0.5-1 % slower in pred and corr (profiles/ab_solve_pairs/).
__device__ __forceinline__ void fetch_pair(const double* p, const BoxLane& b, double& e0, double& e1) {
    e0 = gld(p, b.lo, b.ok);
    e1 = gld(p, b.up, b.ok);
}
__device__ __forceinline__ void use_pair(double e0, double e1, double& vlo, double& vup) {
    vlo = e0;
    vup = e1;
}

// A box pair's lower and upper value with ONE store: row group 0 writes the lower slot, row group 1 the
// upper one (every lane holds both values; rows 2/3 are masked off).
__device__ __forceinline__ void st_lu(double* p, const BoxLane& b, double vlo, double vup, bool ok) {
    const bool odd = (lane_id() & 16) != 0;
    const int m = -(int)odd;
    gst(p, (b.up & m) | (b.lo & ~m), odd ? vup : vlo, ok && lane_id() < 32);
}

// sequential step-length rule of d_compute_alpha_* (d_aux_ip_hard_lib4.c:541-565), per lane
__device__ __forceinline__ void alpha_rule(double& al, double v, double dv) {
    const double cand = -v * rcp_nr(dv);
    al = (-al * dv > v) ? cand : al;
}


// ------------------------------------------------------------------------------------------------
// General constraints lg <= D_k ux_k <= ug (ng_k > 0; such stages always run the generic shape).
// DCt_k = D_k' is a lib4 block (nux x ng, sd = round_up(ng, 2)).  Constraint l = 4*lc + g belongs to
// row group g in chunk lc, so a lane holds dg[lc] = DCt[var(c)][4 lc + g] and
//   (D v)_l      = row_sum16(dg[lc] * v_col)             (every lane of row group g)
//   (DCt w)_c    = xrow_sum(sum_lc dg[lc] * w_l)          (col layout)
//   DCt W DCt'   = sum_lc mfma(dg[lc] * W_l, dg[lc])      (tile layout, W diagonal)
// Slots: [lb (pnb) | ub (pnb) | lg (png) | ug (png)] in the V32 vectors, [box (pnb) | general (png)] in
// Qx / qx (d_aux_ip_hard_lib4.c, the "general" halves of every box routine).
// ------------------------------------------------------------------------------------------------
struct GenLane {
    int lo, up, s16;
    bool ok;
};

__device__ __forceinline__ GenLane gen_lane(int k, int pnb, int ng, int lc) {
    const int gl = 4 * lc + (lane_id() >> 4);
    const int png = (ng + 3) & ~3;
    GenLane q;
    q.ok = gl < ng;
    q.lo = k * V32 + 2 * pnb + gl;
    q.up = q.lo + png;
    q.s16 = k * V16 + pnb + gl;
    return q;
}

__device__ __forceinline__ void gen_dg(const RicIO& io, const DynSh& sh, double dg[4]) {
    const int l = lane_id(), g = l >> 4, c = l & 15;
    const int vc = tile_var(c, sh.nu, sh.nx, sh.xo);
    const int cng = (sh.ng + 1) & ~1;
    const double* D = io.DCt + sh.oG;
#pragma unroll
    for (int lc = 0; lc < 4; lc++) {
        const int gl = 4 * lc + g;
        dg[lc] = (4 * lc < sh.ng) ? gld(D, lib4_idx(cng, vc, gl), vc >= 0 && gl < sh.ng) : 0.0;
    }
}

// Backward: M += DCt diag(Qg) DCt', ml += DCt qg with the box routine of mode BM applied to the general
// slots (d_update_hessian_mpc_hard_tv / d_update_hessian_gradient_res_mpc_hard_tv general halves).
// BX_P2R also forms r_d of the general slots from the current iterate (x: ux_k in col layout).
template <int BM>
__device__ void gen_hessian(const RicIO& io, const DynSh& sh, int k, const BoxCtx& bc, double x, d4& M, double& ml,
                            bool aug) {
    const int c = lane_id() & 15;
    double dg[4];
    gen_dg(io, sh, dg);
    double part = 0.0;
#pragma unroll
    for (int lc = 0; lc < 4; lc++) {
        if (4 * lc >= sh.ng) continue;
        const GenLane q = gen_lane(k, sh.pnb, sh.ng, lc);
        const bool st = q.ok && c == 0;
        double Q = 0.0, qv = 0.0;
        if (BM == BX_GIVEN) {
            Q = gld(bc.Qx, q.s16, q.ok);
            qv = aug ? gld(bc.qx, q.s16, q.ok) : 0.0;
        } else if (BM == BX_P1) {
            const double lml = gld(bc.lam, q.lo, q.ok), lmu = gld(bc.lam, q.up, q.ok);
            const double tl = gld(bc.t, q.lo, q.ok), tu = gld(bc.t, q.up, q.ok);
            const double dl = gld(bc.d, q.lo, q.ok), du = gld(bc.d, q.up, q.ok);
            const double til = rcp_nr(tl), tiu = rcp_nr(tu);
            const double ltl = lml * til, ltu = lmu * tiu;
            const double dll = til * 0.0, dlu = tiu * 0.0;
            qv = lmu - ltu * du + dlu - lml - ltl * dl - dll;
            Q = ltl + ltu;
            gst(bc.t_inv, q.lo, til, st);
            gst(bc.t_inv, q.up, tiu, st);
            gst(bc.lamt, q.lo, ltl, st);
            gst(bc.lamt, q.up, ltu, st);
            gst(bc.qxs, q.s16, qv, st);
        } else if (BM == BX_P2 || BM == BX_P2R) {
            const double lml = gld(bc.lam, q.lo, q.ok), lmu = gld(bc.lam, q.up, q.ok);
            const double tl = gld(bc.t, q.lo, q.ok), tu = gld(bc.t, q.up, q.ok);
            const double rml = gld(bc.res_m, q.lo, q.ok), rmu = gld(bc.res_m, q.up, q.ok);
            double rdl, rdu;
            if (BM == BX_P2R) {  // r_d = [lg - D x + t_lg | ug - D x - t_ug]  (d_res_ip_res_hard.c:393-416)
                const double dx = row_sum16(dg[lc] * x);
                rdl = gld(bc.d, q.lo, q.ok) - dx + tl;
                rdu = gld(bc.d, q.up, q.ok) - dx - tu;
                gst(bc.res_d, q.lo, rdl, st);
                gst(bc.res_d, q.up, rdu, st);
            } else {
                rdl = gld(bc.res_d, q.lo, q.ok);
                rdu = gld(bc.res_d, q.up, q.ok);
            }
            const double til = rcp_nr(tl), tiu = rcp_nr(tu);
            qv = til * (rml - lml * rdl) - tiu * (rmu + lmu * rdu);
            Q = til * lml + tiu * lmu;
            gst(bc.t_inv, q.lo, til, st);
            gst(bc.t_inv, q.up, tiu, st);
        }
        Q = q.ok ? Q : 0.0;
        qv = q.ok ? qv : 0.0;
        M = mfma(dg[lc] * Q, dg[lc], M);
        part += dg[lc] * qv;
    }
    if (aug) ml += xrow_sum(part);
}

// r_q term DCt (lam_ug - lam_lg) of the residuals (d_res_ip_res_hard.c:393-407), col layout.
__device__ double gen_rq(const RicIO& io, const DynSh& sh, int k, const double* lam) {
    double dg[4];
    gen_dg(io, sh, dg);
    double part = 0.0;
#pragma unroll
    for (int lc = 0; lc < 4; lc++) {
        if (4 * lc >= sh.ng) continue;
        const GenLane q = gen_lane(k, sh.pnb, sh.ng, lc);
        const double w = gld(lam, q.up, q.ok) - gld(lam, q.lo, q.ok);
        part += dg[lc] * (q.ok ? w : 0.0);
    }
    return xrow_sum(part);
}

// Forward: steps of the general slots from the primal step x (col layout) and their step-length
// candidates (d_compute_alpha_mpc_hard_tv / d_compute_alpha_res_mpc_hard_tv general halves).
template <int FM>
__device__ void gen_alpha(const RicIO& io, const DynSh& sh, int k, const BoxCtx& bc, double x, double& al) {
    if (FM == BX_NONE) return;
    const int c = lane_id() & 15;
    double dg[4];
    gen_dg(io, sh, dg);
#pragma unroll
    for (int lc = 0; lc < 4; lc++) {
        if (4 * lc >= sh.ng) continue;
        const GenLane q = gen_lane(k, sh.pnb, sh.ng, lc);
        const bool st = q.ok && c == 0;
        const double dx = row_sum16(dg[lc] * x);
        const double lml = gld(bc.lam, q.lo, q.ok), lmu = gld(bc.lam, q.up, q.ok);
        const double tl = gld(bc.t, q.lo, q.ok), tu = gld(bc.t, q.up, q.ok);
        double dtl, dtu, dll, dlu;
        if (FM == BX_P1) {
            dtl = dx - gld(bc.d, q.lo, q.ok) - tl;
            dtu = -dx + gld(bc.d, q.up, q.ok) - tu;
            const double d0l = gld(bc.dlam, q.lo, q.ok && !bc.pred), d0u = gld(bc.dlam, q.up, q.ok && !bc.pred);
            dll = d0l - (gld(bc.lamt, q.lo, q.ok) * dtl + lml);
            dlu = d0u - (gld(bc.lamt, q.up, q.ok) * dtu + lmu);
        } else {
            dtl = dx - gld(bc.res_d, q.lo, q.ok);
            dtu = -dx + gld(bc.res_d, q.up, q.ok);
            dll = -gld(bc.t_inv, q.lo, q.ok) * (lml * dtl + gld(bc.res_m, q.lo, q.ok));
            dlu = -gld(bc.t_inv, q.up, q.ok) * (lmu * dtu + gld(bc.res_m, q.up, q.ok));
        }
        gst(bc.dt, q.lo, dtl, st);
        gst(bc.dt, q.up, dtu, st);
        gst(bc.dlam, q.lo, dll, st);
        gst(bc.dlam, q.up, dlu, st);
        if (q.ok) {
            alpha_rule(al, lml, dll);
            alpha_rule(al, lmu, dlu);
            alpha_rule(al, tl, dtl);
            alpha_rule(al, tu, dtu);
        }
    }
}

// trs backward: the general part of the gradient, DCt qg (col layout), with the corrector updates of
// the general slots (d_update_gradient_mpc_hard_tv / centering correction + d_update_gradient_res).
template <int TM>
__device__ double gen_gradient(const RicIO& io, const DynSh& sh, int k, const BoxCtx& bc) {
    if (TM == BX_NONE) return 0.0;
    const int c = lane_id() & 15;
    double dg[4];
    gen_dg(io, sh, dg);
    double part = 0.0;
#pragma unroll
    for (int lc = 0; lc < 4; lc++) {
        if (4 * lc >= sh.ng) continue;
        const GenLane q = gen_lane(k, sh.pnb, sh.ng, lc);
        const bool st = q.ok && c == 0;
        double qv = 0.0;
        if (TM == BX_GIVEN) {
            qv = gld(bc.qx, q.s16, q.ok);
        } else if (TM == BX_P1) {
            const double dll = gld(bc.t_inv, q.lo, q.ok) * (bc.smu - gld(bc.dlam, q.lo, q.ok) * gld(bc.dt, q.lo, q.ok));
            const double dlu = gld(bc.t_inv, q.up, q.ok) * (bc.smu - gld(bc.dlam, q.up, q.ok) * gld(bc.dt, q.up, q.ok));
            gst(bc.dlam, q.lo, dll, st);
            gst(bc.dlam, q.up, dlu, st);
            qv = gld(bc.qxs, q.s16, q.ok) + (dlu - dll);
        } else if (TM == BX_P2) {
            const double rml = gld(bc.res_m, q.lo, q.ok) + (gld(bc.dt, q.lo, q.ok) * gld(bc.dlam, q.lo, q.ok) - bc.smu);
            const double rmu = gld(bc.res_m, q.up, q.ok) + (gld(bc.dt, q.up, q.ok) * gld(bc.dlam, q.up, q.ok) - bc.smu);
            gst(bc.res_m, q.lo, rml, st);
            gst(bc.res_m, q.up, rmu, st);
            qv = gld(bc.t_inv, q.lo, q.ok) * (rml - gld(bc.lam, q.lo, q.ok) * gld(bc.res_d, q.lo, q.ok)) -
                 gld(bc.t_inv, q.up, q.ok) * (rmu + gld(bc.lam, q.up, q.ok) * gld(bc.res_d, q.up, q.ok));
        }
        part += dg[lc] * (q.ok ? qv : 0.0);
    }
    return xrow_sum(part);
}

// ------------------------------------------------------------------------------------------------
// Backward factorisation.  Every pass over the stages issues the HBM loads of the NEXT stage (into
// registers) before it computes the current one, so the dependent recursion never waits on memory.
// ------------------------------------------------------------------------------------------------
struct BwdFrag {
    d4 Mi;         // RSQrq tile (mirrored lower part), tile coords of stage k
    double mlq;    // augmented-row source: q (update_q) or the RSQrq last row
    d4 bop;        // MFMA B operand per K-chunk: BAbt_k[var(c)][4kc+g-xo1]
    d4 brow;       // b_k in row layout over the stage-(k+1) tile rows (BX_P2R: b_k, col layout, in [0])
    double bx[8];  // box-mode inputs of tile c
    BoxLane bl;
    // BX_P2R residual inputs: ux_k (col c / rows g+4r), pi_k (rows), pi_{k-1} (col), BAbt_k' (col
    // c-xo1 over rows g+4r), x_{k+1} (col)
    double uc, pc, pim1;
    double gc;  // the stored certificate bound g (IPM box modes)
};

// The stage's RSQ block as a full symmetric tile (its lower triangle mirrored), zero outside the active variables.
template <class SH>
__device__ __forceinline__ void load_rsq_tile(const double* R, const SH& sh, d4& Mi) {
    const int l = lane_id(), g = l >> 4, c = l & 15;
    const int vc = tile_var(c, sh.nu, sh.nx, sh.xo);
#pragma unroll
    for (int r = 0; r < 4; r++) {
        const int vi = tile_var(g + 4 * r, sh.nu, sh.nx, sh.xo);
        const int hi = vi > vc ? vi : vc, lo = vi > vc ? vc : vi;
        Mi[r] = ldsel(R, lib4_idx(sh.sdR, hi, lo), vi >= 0 && vc >= 0);
    }
}

// The certificate's threshold T_k of every stage into cert[0..N], as its own pass (stages in groups of
// eight, the group's tile and BAbt-operand loads issued before its math): the single-Newton start, whose first
// factorisation is a phase-2 one.
__device__ void cert_pass(const RicIO& io, double* cert) {
    const int l = lane_id(), g = l >> 4, c = l & 15;
    for (int k0 = 0; k0 <= io.N; k0 += 8) {
        d4 Mi[8], bop[8];
#pragma unroll
        for (int j = 0; j < 8; j++) {
            const int k = k0 + j <= io.N ? k0 + j : io.N;
            const DynSh sh(StageRef{io.st, k});
            load_rsq_tile(stage_R(io, sh), sh, Mi[j]);
            const int vc = tile_var(c, sh.nu, sh.nx, sh.xo);
            const double* Bk = stage_B(io, sh);
#pragma unroll
            for (int r = 0; r < 4; r++) {
                const int s = 4 * r + g - sh.xo1;
                bop[j][r] = ldsel(Bk, lib4_idx(sh.sdB, vc, s), k < io.N && s >= 0 && s < sh.nx1 && vc >= 0);
            }
        }
#pragma unroll
        for (int j = 0; j < 8; j++) {
            const int k = k0 + j <= io.N ? k0 + j : io.N;
            const DynSh sh(StageRef{io.st, k});
            const double tau = cert_form(Mi[j], 0.0, sh);
            gst(cert, k0 + j, tau, lane_id() == 0 && k0 + j <= io.N);
        }
    }
}

template <bool AUG, int BM, class SH>
__device__ __forceinline__ void bwd_fetch(const RicIO& io, const SH& sh, int k, int update_b, const double* bsrc,
                                          int update_q, const double* qsrc, const BoxCtx& bc, BwdFrag& f) {
    const int l = lane_id(), g = l >> 4, c = l & 15;
    const int nux = sh.nu + sh.nx;
    const double* R = stage_R(io, sh);
    const int vc = tile_var(c, sh.nu, sh.nx, sh.xo);
    load_rsq_tile(R, sh, f.Mi);
    f.mlq = 0.0;
    if (AUG) {
        const double* qp = update_q ? qsrc + k * V16 : R;
        const int qi = update_q ? vc : lib4_idx(sh.sdR, nux, vc);
        f.mlq = ldsel(qp, qi, vc >= 0);
    }
    const BoxLane b = box_lane(io.tileslot, sh.pnb, k);
    f.bl = b;
    f.gc = cert_loaded(BM) ? bc.cert[k] : 0.0;  // LDS (fact_body) or the workspace (multi-wave); unused when cert_new
#pragma unroll
    for (int i = 0; i < 8; i++) f.bx[i] = 0.0;
    if (BM == BX_GIVEN) {
        f.bx[0] = ldsel(bc.Qx, b.s16, b.ok);
        f.bx[1] = AUG ? ldsel(bc.qx, b.s16, b.ok) : 0.0;
    } else if (BM == BX_P1) {
        f.bx[0] = ldsel(bc.lam, b.lo, b.ok);
        f.bx[1] = ldsel(bc.lam, b.up, b.ok);
        f.bx[2] = ldsel(bc.t, b.lo, b.ok);
        f.bx[3] = ldsel(bc.t, b.up, b.ok);
        f.bx[4] = ldsel(bc.d, b.lo, b.ok);
        f.bx[5] = ldsel(bc.d, b.up, b.ok);
    } else if (BM == BX_P2 || BM == BX_P2R) {
        ld_lu(bc.lam, b, f.bx[0], f.bx[1]);
        ld_lu(bc.t, b, f.bx[2], f.bx[3]);
        // BX_P2R: r_m of the current iterate is lam * t, exactly the product the update pass stored
        // (update_p2_pass), so it is formed at use instead of loaded
        if (BM == BX_P2) ld_lu(bc.res_m, b, f.bx[4], f.bx[5]);
        ld_lu(bc.res_d, b, f.bx[6], f.bx[7]);
    }
    const bool live = SH::fixed || k < io.N;
    const double* Bk = stage_B(io, sh);
    const double* bp = update_b ? bsrc + k * V16 : Bk;
#pragma unroll
    for (int r = 0; r < 4; r++) {
        const int s = 4 * r + g - sh.xo1;
        const bool ok = live && s >= 0 && s < sh.nx1;
        f.bop[r] = ldsel(Bk, lib4_idx(sh.sdB, vc, s), ok && vc >= 0);
        if (BM != BX_P2R) f.brow[r] = AUG ? ldsel(bp, update_b ? s : lib4_idx(sh.sdB, nux, s), ok) : 0.0;
    }
    if (BM == BX_P2R) {
        static_assert(BM != BX_P2R || AUG, "residual right-hand sides need the augmented row");
        const int sc = c - sh.xo1;
        const bool oks = live && sc >= 0 && sc < sh.nx1;
        // ux_k and pi_k in col layout (the residual turns them into row layout through LDS: two loads
        // instead of eight row-layout loads with four distinct addresses each)
        f.uc = ldsel(bc.ux, k * V16 + vc, vc >= 0);
        f.pc = ldsel(bc.pi, k * V16 + sc, oks);
        f.pim1 = ldsel(bc.pi, (k - 1) * V16 + (vc - sh.nu), k > 0 && vc >= sh.nu);
        f.brow[0] = ldsel(Bk, lib4_idx(sh.sdB, nux, sc), oks);
    }
}

// Box Hessian (dq, on the tile diagonal) and gradient (qxv, on the augmented row) of tile c.
template <bool AUG, int BM>
__device__ __forceinline__ void box_hessian(const BoxCtx& bc, const BwdFrag& f, double& dq, double& qxv) {
    const int g = lane_id() >> 4;
    const BoxLane& b = f.bl;
    const bool st = b.ok && g == 0;
    dq = 0.0;
    qxv = 0.0;
    if (BM == BX_GIVEN) {
        dq = f.bx[0];
        qxv = f.bx[1];
    } else if (BM == BX_P1) {  // d_update_hessian_mpc_hard_tv with sigma*mu = 0 (phase 1)
        const double til = rcp_nr(f.bx[2]), tiu = rcp_nr(f.bx[3]);
        const double ltl = f.bx[0] * til, ltu = f.bx[1] * tiu;
        const double dll = til * 0.0, dlu = tiu * 0.0;
        const double q = f.bx[1] - ltu * f.bx[5] + dlu - f.bx[0] - ltl * f.bx[4] - dll;
        gst(bc.t_inv, b.lo, til, st);
        gst(bc.t_inv, b.up, tiu, st);
        gst(bc.lamt, b.lo, ltl, st);
        gst(bc.lamt, b.up, ltu, st);
        gst(bc.qxs, b.s16, q, st);
        dq = b.ok ? ltl + ltu : 0.0;
        qxv = (AUG && b.ok) ? q : 0.0;
    } else if (BM == BX_P2 || BM == BX_P2R) {  // d_update_hessian_gradient_res_mpc_hard_tv
        const double til = rcp_nr(f.bx[2]), tiu = rcp_nr(f.bx[3]);
        const double rml = BM == BX_P2R ? f.bx[0] * f.bx[2] : f.bx[4];
        const double rmu = BM == BX_P2R ? f.bx[1] * f.bx[3] : f.bx[5];
        const double q = til * (rml - f.bx[0] * f.bx[6]) - tiu * (rmu + f.bx[1] * f.bx[7]);
        if (!bc.no_tinv) st_lu(bc.t_inv, b, til, tiu, b.ok);  // lower / upper: one store
        dq = b.ok ? til * f.bx[0] + tiu * f.bx[1] : 0.0;
        qxv = (AUG && b.ok) ? q : 0.0;
    }
}

// BX_P2R: residuals of the current iterate (d_res_res_mpc_hard_tv, d_res_ip_res_hard.c:39-319) for the
// prefetched stage k, computed one stage ahead (at the end of stage k+1's step) so that only the
// right-hand side it produces stays live across the next step:
//   r_q = q - [0; pi_{k-1}] + (lam_up - lam_lo) + RSQ ux + BAbt pi,   r_b = b - x_{k+1} + BAbt' ux
// The factorisation's rows become (mlq, brow) = (r_q, r_b) (res_rhs) or the data's own (q, b).
template <class SH>
// x1c: x_{k+1} in col layout over stage-(k+1) tiles -- the ux_{k+1} the previous stage's fragment holds.
__device__ __forceinline__ void bwd_residual(const RicIO& io, Scratch* sm, const SH& sh, int k, const BoxCtx& bc,
                                             BwdFrag& f, double x1c, bool store) {
    const int l = lane_id(), g = l >> 4, c = l & 15;
    const bool live = SH::fixed || k < io.N;
    const int vc = tile_var(c, sh.nu, sh.nx, sh.xo);
    const int sc = c - sh.xo1;
    const bool oks = live && sc >= 0 && sc < sh.nx1;
    double h = f.mlq;
    if (k > 0 && vc >= sh.nu) h -= f.pim1;
    if (f.bl.ok) h += -f.bx[0] + f.bx[1];
    double ur[4], pr[4];  // ux_k (tile rows g+4r) and pi_k (stage-(k+1) tile rows g+4r) in row layout
    col2row2(sm, f.uc, f.pc, ur, pr);
    // BAbt_k' as a tile (reg r: BAbt_k[var(g+4r)][c - xo1]) is the transpose of the fragment's BAbt operand
    // tile: identity MFMAs (exact) on the otherwise idle matrix unit instead of four more loads
    d4 bt = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
    for (int r = 0; r < 4; r++) {
        if (4 * r + 3 < sh.xo1 || 4 * r >= sh.xo1 + sh.nx1) continue;  // uniform: chunk without a state
        bt = mfma(f.bop[r], (c == 4 * r + g) ? 1.0 : 0.0, bt);
    }
    double part = 0.0, p2 = 0.0, p3 = 0.0;
#pragma unroll
    for (int r = 0; r < 4; r++) part += f.Mi[r] * ur[r];
    h += xrow_sum(part);
#pragma unroll
    for (int r = 0; r < 4; r++) {
        p2 += f.bop[r] * pr[r];
        p3 += bt[r] * ur[r];
    }
    const double bpi = xrow_sum(p2);
    const double atu = xrow_sum(p3);
    if (live) h += bpi;
    if constexpr (!SH::fixed) {
        if (sh.ng > 0) h += gen_rq(io, sh, k, bc.lam);
    }
    const double rb = f.brow[0] - (oks ? x1c : 0.0) + atu;
    // r_q (row group 0) and r_b (row group 1) in one store: both live in the IPM workspace carve (hpmpc_kernels.hip
    // carve: res_b = res_q + (N+1)*16), so r_b is a positive offset from r_q's base
    const int db = (int)(bc.res_b - bc.res_q);
    gst(bc.res_q, g == 0 ? k * V16 + vc : db + k * V16 + sc, g == 0 ? h : rb,
        store && ((g == 0 && vc >= 0) || (g == 1 && oks)));
    f.mlq = bc.res_rhs ? h : f.mlq;
    double bcol = bc.res_rhs ? rb : f.brow[0];
    bcol = oks ? bcol : 0.0;
    double br[4];
    col2row(sm, bcol, br);
#pragma unroll
    for (int r = 0; r < 4; r++) f.brow[r] = br[r];
}

// First half of a backward stage: the stage tile and augmented row with the box (and general) Hessian /
// gradient terms added -- everything that does not depend on the recursion (the multi-wave solo kernel runs it
// on a helper wave, hk_mw.h).
// dq (col layout): the box term on the diagonal; gc: the stage's clamp-certificate bound g (cert_g: loaded in the
// IPM's box modes, formed from the data tile otherwise; unused on a stage that is fully factorised).
// CN (IPM box modes): how the stage's certificate bound g is had -- CERT_LOAD: from bc.cert (a later factorisation
// of the solve); CERT_FORM: formed from the data tile and stored to bc.cert_out (the solve's first factorisation);
// CERT_RT: either, by bc.cert_new at run time (the multi-wave kernel's helpers, which have the issue slots to spare).
// The pass kernels pick CERT_LOAD or CERT_FORM once per launch, so neither stage loop carries the other's code.
enum CertMode { CERT_LOAD = 0, CERT_FORM = 1, CERT_RT = 2 };
template <bool AUG, int BM, int CN = CERT_RT, class SH>
__device__ __forceinline__ void bwd_pre(const RicIO& io, const SH& sh, int k, const BwdFrag& cur, const BoxCtx& bc,
                                        d4& M, double& ml, double& dq, double& gc) {
    const int l = lane_id(), g = l >> 4, c = l & 15;
    double qxv;
    box_hessian<AUG, BM>(bc, cur, dq, qxv);
#ifdef HK_COUNT_NOCERT
    gc = 0.0;
#else
    // gc: the stage's certificate threshold T_k (cert_thr), from its data alone
    if constexpr (cert_loaded(BM)) {
        // the solve's first factorisation forms T_k from the tile (stage 0 too: a later one may be a P-form stage of
        // another plan shape) and keeps it for the others; masked store otherwise (fixed vector-memory count).  The box
        // terms (lam / t >= 0) are the iterate's, not the data's: no dq in these modes
        if constexpr (CN == CERT_LOAD) {
            gc = cur.gc;
        } else if constexpr (CN == CERT_FORM) {
            gc = cert_form(cur.Mi, 0.0, sh);
            gst(bc.cert_out, k, gc, lane_id() == 0);
        } else {
            gc = bc.cert_new ? cert_form(cur.Mi, 0.0, sh) : cur.gc;
            gst(bc.cert_out, k, gc, bc.cert_new && lane_id() == 0);
        }
    } else {
        gc = (SH::fixed || k > 0) ? cert_form(cur.Mi, dq, sh) : 0.0;
    }
#endif
    M = cur.Mi;
    ml = cur.mlq + qxv;  // update_q row (or RSQrq row) + drowad qx
#pragma unroll
    for (int r = 0; r < 4; r++) M[r] += (g + 4 * r == c) ? dq : 0.0;  // ddiaadin: diag = bd + Qx
    if constexpr (!SH::fixed && BM != BX_NONE) {
        if (sh.ng > 0) gen_hessian<BM>(io, sh, k, bc, BM == BX_P2R ? cur.uc : 0.0, M, ml, AUG);
    }
}

// M += BAbt_k P_{k+1} BAbt_k' (the tile half of the recursion; P form, see stage_chol).
template <class SH>
__device__ __forceinline__ void bwd_tile_update(const SH& sh, bool live, const d4& bop, const d4& S, d4& M) {
    const int nx1 = sh.nx1, xo1 = sh.xo1;
    if (live) {
        // T' = P_{k+1} BAbt_k'  (rows in stage-(k+1) tile coords): the A fragment of K-chunk kc is P's
        // register kc itself (P symmetric: lane (g,c) holds P[4kc+g][c] = P[c][4kc+g]), its u columns masked;
        // two accumulator chains (even / odd K-chunks) halve the dependent MFMA latency
        d4 a0 = {0.0, 0.0, 0.0, 0.0}, a1 = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
        for (int kc = 0; kc < 4; kc++) {
            if (4 * kc + 3 < xo1 || 4 * kc >= xo1 + nx1) continue;  // uniform
            // lanes c < xo1 (u rows of stage k+1) only produce rows of T' that the second chain skips: no mask
            const double aop = S[kc];
            if (kc & 1)
                a1 = mfma(aop, bop[kc], a1);
            else
                a0 = mfma(aop, bop[kc], a0);
        }
        const d4 acc = a0 + a1;
        // M += BAbt_k T'  (A fragment of chunk r = the BAbt operand already in registers), two chains
        d4 m1 = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
        for (int r = 0; r < 4; r++) {
            if (4 * r + 3 < xo1 || 4 * r >= xo1 + nx1) continue;
            if (r & 1)
                m1 = mfma(bop[r], acc[r], m1);
            else
                M = mfma(bop[r], acc[r], M);
        }
        M = M + m1;
    }
}

// The augmented row's update before the stage factorisation: Pb_k = P_{k+1} b_k (stored when compute_Pb) and
// ml += BAbt_k (P b + p_{k+1}) (the row half of the recursion).
template <class SH>
__device__ __forceinline__ void bwd_row_update(const RicIO& io, Scratch* sm, const SH& sh, int k, bool live,
                                               const d4& bop, const d4& brow, const d4& S, double ml_prev,
                                               int compute_Pb, double* Pb, double& ml) {
    const int l = lane_id(), g = l >> 4, c = l & 15;
    const int nx1 = sh.nx1, xo1 = sh.xo1;
    const bool xc = c >= xo1;  // tile column c is a state of stage k+1 (padding beyond xo1+nx1 is zero)
    // Pb_k = P_{k+1} b_k (col layout, stage-(k+1) tile); zero at k = N (S = 0, b = 0).  Stored masked,
    // never skipped: the row update below needs it anyway
    double part = 0.0;
#pragma unroll
    for (int r = 0; r < 4; r++) part += S[r] * brow[r];  // columns c < xo1: unused (masked below)
    const double pb = xrow_sum(part);
    gst(Pb, k * V16 + (c - xo1), pb, compute_Pb && live && g == 0 && xc && c < xo1 + nx1);
    // m_last += BAbt_k (P b + p_{k+1})
    const double wc = xc ? pb + ml_prev : 0.0;
    double wrow[4];
    col2row(sm, wc, wrow);
    double mp = 0.0;
#pragma unroll
    for (int r = 0; r < 4; r++) mp += bop[r] * wrow[r];
    if (live) ml += xrow_sum(mp);
}

// Second half: M += BAbt P BAbt', the row update and the stage factorisation (the recursion's chain).
// THR: gc is the certificate threshold T of the IPM's modes (cert_ok_thr), else the bound g (cert_ok).
template <bool AUG, bool THR, class SH>
__device__ __forceinline__ void bwd_core(const RicIO& io, Scratch* sm, const SH& sh, int k, const d4& bop,
                                         const d4& brow, d4 M, double ml, double dq, double gc, int compute_Pb,
                                         double* Pb, d4& S, double& ml_prev, double& invd_prev, double& kg_prev) {
    const bool live = SH::fixed || k < io.N;
    bwd_tile_update(sh, live, bop, S, M);
    // stage 0 of a generic problem keeps the full factor; every other stage is factorised in P form, with its x
    // block factorised as well where the clamp certificate fails (stage_chol)
    const bool full = !SH::fixed && k == 0;
#ifdef HK_COUNT_NOCERT  // static counts without the clamp certificate (tools/loop_icount.py)
    const bool xcert = false;
    (void)dq;
    (void)gc;
#else
    // on the stage matrix after its products (cert_ok_thr)
    const bool xcert = !full && !cert_test(M, dq, gc);
#endif
#ifdef HK_STAMPS  // diagnostic build: how often the certificate fails, at this allowance and (with g) at 10x / 100x
    // smaller ones -- the threshold form only knows its own allowance, so those two count its failures
    if (!full) {
        // (the threshold form knows its own allowance only: the 1e-12 / 1e-13 slots count its failures too)
        const bool xfac = xcert, f12 = xcert, f13 = xcert;
        if (lane_id() == 0) {
            atomicAdd(&g_xfac_stat[0], 1ull);
            if (xfac) atomicAdd(&g_xfac_stat[1], 1ull);
            if (xfac) g_xfac_sweep[blockIdx.x & 0xffff] = 1u;
            if (f12) atomicAdd(&g_xfac_stat[2], 1ull);
            if (f13) atomicAdd(&g_xfac_stat[3], 1ull);
        }
    }
#endif
    if (AUG) bwd_row_update(io, sm, sh, k, live, bop, brow, S, ml_prev, compute_Pb, Pb, ml);
    HK_STAMP(2, k);
    double invd, kg = 0.0;
    stage_chol<AUG, SH::fixed>(M, ml, invd, sh.nu, sh.nx, sh.xo, full, !SH::fixed, &kg, k, xcert);
    kg_prev = kg;
    HK_STAMP(3, k);
#pragma unroll
    for (int r = 0; r < 4; r++) S[r] = M[r];
    ml_prev = ml;
    invd_prev = invd;
}

// One backward stage: M = RSQ + BAbt P BAbt' (+ box terms), then the stage factorisation (P form on
// stages k >= 1, see stage_chol).  S (in: record of stage k+1, whose x block is P_{k+1}; out: record of
// stage k), ml/invd/kg likewise.  The reference forms the same M as RSQ + W W' with W = BAbt Lxx
// (dtrmm_nt_u + dsyrk, d_back_ric_rec.c:262-264, :325) and the same row as W (Lxx' b + l_x) (:266-276).
template <bool AUG, int BM, int CN, class SH>
__device__ __forceinline__ void bwd_step(const RicIO& io, Scratch* sm, const SH& sh, int k, const BwdFrag& cur,
                                         const BoxCtx& bc, int compute_Pb, double* Pb, d4& S, double& ml_prev,
                                         double& invd_prev, double& kg_prev) {
    d4 M;
    double ml, dq, gc;
    bwd_pre<AUG, BM, CN>(io, sh, k, cur, bc, M, ml, dq, gc);
    bwd_core<AUG, cert_loaded(BM)>(io, sm, sh, k, cur.bop, cur.brow, M, ml, dq, gc, compute_Pb, Pb, S, ml_prev, invd_prev, kg_prev);
}

// Backward Riccati recursion (sv when AUG, trf otherwise), d_back_ric_rec.c:186-335 / :447-558.
//   b  (state order) / q (variable order) : update_b / update_q replacement rows
//   BM                                    : box Hessian / gradient terms (BoxMode)
//   Pb (state order)                      : P_{k+1} b_k (compute_Pb, AUG only)
// Vector arguments use a per-stage stride of V16.
// Prefetch depth one stage (two measured no faster in the Riccati entry points: N=100 3.48 vs 3.50 M fact/s, configs[2]
// 7.14 vs 7.25 M, profiles/r04/ab_ric_LO.txt; the IPM passes have no registers for a third fragment).
template <bool AUG, int BM, class FX, int CN = CERT_LOAD>
__device__ void ric_backward(const RicIO& io, Scratch* sm, int update_b, const double* bsrc, int update_q,
                             const double* qsrc, const BoxCtx& bc, int compute_Pb, double* Pb) {
    d4 S = {0.0, 0.0, 0.0, 0.0};
    double ml_prev = 0.0, invd_prev = 0.0, kg_prev = 0.0;
#ifdef HK_STAMPS
    if (lane_id() == 0) g_xfac_sweep[blockIdx.x & 0xffff] = 0u;
#endif
    StageRef si{io.st, io.N};
    BwdFrag cur;
    with_shape<FX>(si, [&](const auto& sh) {
        bwd_fetch<AUG, BM>(io, sh, io.N, update_b, bsrc, update_q, qsrc, bc, cur);
        if constexpr (BM == BX_P2R) bwd_residual(io, sm, sh, io.N, bc, cur, 0.0, true);
    });
    // One stage: prefetch stage kn into `nxt` while stage k runs on `cur`.  The loop is unrolled by two
    // with the fragments swapping roles, so no stage pays a register copy of the prefetched fragment.
    bool rec_fixed = false;  // the record in registers (stage k+1's) belongs to the compiled class: packed format
    auto stage = [&](int k, const BwdFrag& cur, BwdFrag& nxt) __attribute__((always_inline)) {
        HK_STAMP(0, k);
        const int kn = k > 0 ? k - 1 : 0;  // unconditional prefetch (stage 0 re-read on the last pass)
        const StageRef sn{io.st, kn};
        HK_STAMP(5, k);
        with_shape<FX>(sn, [&](const auto& sh) { bwd_fetch<AUG, BM>(io, sh, kn, update_b, bsrc, update_q, qsrc, bc, nxt); });
        HK_STAMP(6, k);
        // factor of stage k+1 (still in registers): stored one stage late, behind the prefetch, so
        // that no s_waitcnt of this stage has to wait for the store acknowledgements
        double* Fk1 = io.F + (long)(k + 1) * FSTRIDE;
        if constexpr (FX::enabled) {
            if (rec_fixed)
                store_factor_fixed<FX::nx>(Fk1, S, AUG ? ml_prev : 0.0, invd_prev, kg_prev, k < io.N);
            else
                store_factor(Fk1, S, AUG ? ml_prev : 0.0, invd_prev, kg_prev, k < io.N);
        } else {
            store_factor(Fk1, S, AUG ? ml_prev : 0.0, invd_prev, kg_prev, k < io.N);
        }
        asm volatile("" ::: "memory");  // keep those stores here, ahead of this stage's math
        HK_STAMP(1, k);
        with_shape<FX>(si, [&](const auto& sh) {
            bwd_step<AUG, BM, CN>(io, sm, sh, k, cur, bc, compute_Pb, Pb, S, ml_prev, invd_prev, kg_prev);
            rec_fixed = std::remove_reference_t<decltype(sh)>::fixed;
        });
        if constexpr (BM == BX_P2R)
            with_shape<FX>(sn, [&](const auto& sh) { bwd_residual(io, sm, sh, kn, bc, nxt, cur.uc, k > 0); });
        HK_STAMP(4, k);
        si = sn;
    };
    BwdFrag alt;
    for (int k = io.N;;) {
        stage(k, cur, alt);
        if (--k < 0) break;
        stage(k, alt, cur);
        if (--k < 0) break;
    }
    store_factor(io.F, S, AUG ? ml_prev : 0.0, invd_prev, kg_prev);
#ifdef HK_STAMPS
    if (lane_id() == 0) {
        atomicAdd(&g_xfac_stat[4], 1ull);
        if (g_xfac_sweep[blockIdx.x & 0xffff]) atomicAdd(&g_xfac_stat[5], 1ull);
    }
#endif
}

// ------------------------------------------------------------------------------------------------
// Triangular solves on the stage factor (upper storage S: row p of S = column p of L).
// ------------------------------------------------------------------------------------------------
// Solve the unknown part of L_k' y = rhs (dtrsv_t_lib, blas_d_lib4.c:5276) in row layout, descending.
// rrow: rhs in row layout (reduced by the known part already); y written into ur (row layout) at the
// unknown tile indices.  unknown(t) = active(t) && (all || t < nu).
template <class SH>
__device__ __forceinline__ void solve_lt(const SH& sh, const d4& S, double invd, double rrow[4], double ur[4],
                                         bool all) {
    const int l = lane_id(), g = l >> 4;
#pragma unroll
    for (int p = 15; p >= 0; p--) {
        const bool unk = all ? tile_active(p, sh.nu, sh.nx, sh.xo) : (p < sh.nu);
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
template <class SH>
__device__ __forceinline__ double solve_ln(const SH& sh, const d4& S, double invd, double h, bool all) {
    const int l = lane_id(), c = l & 15;
#pragma unroll
    for (int p = 0; p < 16; p++) {
        const bool unk = all ? tile_active(p, sh.nu, sh.nx, sh.xo) : (p < sh.nu);
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

// The trs backward's u solve of stage k (the rectangular dtrsv_n_lib over the nu pivots, d_back_ric_rec.c:687).  A
// fixed-shape stage (nu <= 4, u block = tile block 0) runs it in gain form on the record's gain block KG, which the
// trs fetch puts in S[0]: with N = L_uu^-1, the solve is y = N h_u and h_x' = h_x - L_xu N h_u, and KG (stage_chol
// KGEN: KG[g][c] = -(L_uu^-T e_c)_g on the u tiles, -(L_uu^-T L[c][0..3]')_g on the state tiles) is exactly
// [-N' | -(L_xu N)'] -- transposes of the substitution's own matrices (also with clamped pivots: the forward and the
// backward substitution with the same zeroed inverse diagonal are transposes of each other).  So
//   t[c] = sum_g KG[g][c] h[g],   y[c] = -t[c] (c < 4),   h'[c] = h[c] + t[c] (c >= 4):
// four row broadcasts, one product and a row-group sum instead of four dependent pivot steps.
template <class SH>
__device__ __forceinline__ double trs_usolve(const SH& sh, const d4& S, double invd, double h, bool all) {
    if constexpr (SH::fixed) {
        static_assert(SH::xo == 4, "gain form needs the u block in tile block 0");
        const int c = lane_id() & 15;
        // h[g] in every lane of row group g (h is in col layout: lane (g, j) holds h[j])
        const double hg = sel_g(row_bcast<0>(h), row_bcast<1>(h), row_bcast<2>(h), row_bcast<3>(h));
        const double t = xrow_sum(S[0] * hg);
        return c < 4 ? -t : h + t;
    } else {
        return solve_ln(sh, S, invd, h, all);
    }
}

// pi = P x + p on the next stage's record S1 (P form; the reference's Lxx (Lxx' x + l_x), dtrmv_u_n +
// dtrmv_u_t, d_back_ric_rec.c:355-365), x in row layout, result in col layout.
__device__ __forceinline__ double pi_from_x(const d4& S1, int xo1, const double x1row[4], double pcol) {
    (void)xo1;
    double part = 0.0;
#pragma unroll
    for (int r = 0; r < 4; r++) part += S1[r] * x1row[r];  // columns c < xo1 are never stored
    return xrow_sum(part) + pcol;
}

// ------------------------------------------------------------------------------------------------
// Forward substitution (sv and trs).
// ------------------------------------------------------------------------------------------------
struct FwdFrag {
    d4 S;
    double lc, invd;
    double kg;    // gain form: KG[g][c] (fixed stages)
    d4 bt;        // bt[r] = BAbt_k[var(g+4r)][c - xo1]
    double bval;  // b_k[c - xo1]
    double hc;    // trs: backward vector hux_k[var(c)]
    double pk;    // trs: p_{k+1} = hux_{k+1}[x part] (col layout over stage-(k+1) tile)
    double bx[10];
    BoxLane bl;
};

// Fetch of stage k (sh: shape of stage min(k, N-1), whose BAbt block the pass reads; pnbk: pnb of k).
// mode 0: sv (b from update_b source or the BAbt row); mode 1: trs (b from hb or the BAbt row, plus hc/pk)
// PRED: the IPM predictor sweep.  It never asks for pi (the record rows pi would read are not loaded), and its
// r_m is still lam * t as the update pass stored it (formed at use instead of loaded).  The step rule's 1/t is
// recomputed from t in every sweep (bitwise the factorisation's stored t^-1: the same rcp_nr of the same t).
template <int MODE, int FM, bool PRED, class SH>
__device__ __forceinline__ void fwd_fetch(const RicIO& io, const SH& sh, int k, int pnbk, const double* bsrc,
                                          int use_bsrc, const double* ux, int compute_pi_, const BoxCtx& bc,
                                          FwdFrag& f) {
    const int compute_pi = PRED ? 0 : compute_pi_;
    const int l = lane_id(), g = l >> 4, c = l & 15;
    const double* Fk = io.F + (long)k * FSTRIDE;
    // The factor tile is read by the u-block solve of generic stages and by pi (compute_pi) only, inv_diag by
    // the generic solve, l by the sv forward: the gain-form predictor masks the rest off (a masked lane reads
    // nothing, and every path keeps the same load count for the counted vmcnt waits).
    const bool needS = !SH::fixed || compute_pi;
    // S[0] (tile rows 0..3) holds the u block's columns of L: a fixed-shape stage (nu <= 4, xo = 4) solves
    // its u block in gain form, and pi_from_x reads rows >= xo only, so S[0] is never needed there
    if constexpr (SH::fixed) {  // packed record (store_factor_fixed): P only, and only for pi
        f.S[0] = 0.0;
        if (PRED) {
            f.S[1] = f.S[2] = f.S[3] = 0.0;
        } else {
            load_p_fixed<SH::nx>(Fk, f.S, needS);
        }
        f.lc = MODE == 0 ? gld(Fk, FXR_L + c) : 0.0;
        f.invd = 0.0;
        f.kg = gld(Fk, FXR_KG + l);
    } else {
#pragma unroll
        for (int r = 0; r < 4; r++) f.S[r] = gld(Fk, r * 64 + l, needS);
        f.lc = MODE == 0 ? gld(Fk, 256 + c) : 0.0;
        f.invd = gld(Fk, 272 + c);
        f.kg = gld(Fk, 288 + l);
    }
    const int kk = k < io.N ? k : io.N - 1;  // stage N has no BAbt block: loads clamped, values masked
    const bool live = k < io.N;
    const double* Bk = stage_B(io, sh);
    const int s = c - sh.xo1;
    const bool ok = live && s >= 0 && s < sh.nx1;
#pragma unroll
    for (int r = 0; r < 4; r++) {
        const int vi = tile_var(g + 4 * r, sh.nu, sh.nx, sh.xo);
        f.bt[r] = ldsel(Bk, lib4_idx(sh.sdB, vi, s), vi >= 0 && ok);
    }
    f.bval = use_bsrc ? ldsel(bsrc + kk * V16, s, ok) : ldsel(Bk, lib4_idx(sh.sdB, sh.nu + sh.nx, s), ok);
    f.hc = 0.0;
    f.pk = 0.0;
    if (MODE == 1) {
        const int vc = tile_var(c, sh.nu, sh.nx, sh.xo);
        f.hc = ldsel(ux + kk * V16, vc, live && vc >= 0);
        // p_{k+1} for pi_k is not loaded: fwd_step forms pi_{k-1} from its own fragment's hc (= hux_k)
    }
#pragma unroll
    for (int i = 0; i < 10; i++) f.bx[i] = 0.0;
    if (FM != BX_NONE) {
        const BoxLane b = box_lane(io.tileslot, pnbk, k);
        f.bl = b;
        if (FM == BX_P1) {
            f.bx[0] = ldsel(bc.d, b.lo, b.ok);
            f.bx[1] = ldsel(bc.d, b.up, b.ok);
            f.bx[2] = ldsel(bc.t, b.lo, b.ok);
            f.bx[3] = ldsel(bc.t, b.up, b.ok);
            f.bx[4] = ldsel(bc.lamt, b.lo, b.ok);
            f.bx[5] = ldsel(bc.lamt, b.up, b.ok);
            f.bx[6] = ldsel(bc.lam, b.lo, b.ok);
            f.bx[7] = ldsel(bc.lam, b.up, b.ok);
            f.bx[8] = ldsel(bc.dlam, b.lo, b.ok && !bc.pred);
            f.bx[9] = ldsel(bc.dlam, b.up, b.ok && !bc.pred);
        } else if (FM == BX_P2) {  // [2..3] (1/t) and, in the predictor, [6..7] (r_m) are formed at use
            // lower / upper pairs in one load each (even slot: the raw value, split at use by box_alpha)
            fetch_pair(bc.res_d, b, f.bx[0], f.bx[1]);
            fetch_pair(bc.lam, b, f.bx[4], f.bx[5]);
            if (!PRED) fetch_pair(bc.res_m, b, f.bx[6], f.bx[7]);
            fetch_pair(bc.t, b, f.bx[8], f.bx[9]);
        }
    }
}

template <int MODE, int FM, class FX, bool PRED>
__device__ __forceinline__ void fwd_fetch_k(const RicIO& io, int k, const double* bsrc, int use_bsrc,
                                            const double* ux, int compute_pi, const BoxCtx& bc, FwdFrag& f) {
    const int kk = k < io.N ? k : io.N - 1;
    const StageRef sk{io.st, kk};
    const int pnbk = srd(StageRef{io.st, k}, &StageInfo::pnb);
    with_shape<FX>(sk, [&](const auto& sh) {
        fwd_fetch<MODE, FM, PRED>(io, sh, k, pnbk, bsrc, use_bsrc, ux, compute_pi, bc, f);
    });
}

// Step of the box slacks / multipliers of tile c given the primal step x = dux_k[var(c)] (col layout)
// and the per-lane step-length candidate (d_compute_alpha_mpc_hard_tv :489-614 / _res_ :1180-1313).
template <int FM, bool PRED>
__device__ __forceinline__ void box_alpha(const BoxCtx& bc, const FwdFrag& f, double x, double& al) {
    if (FM == BX_NONE) return;
    const BoxLane& b = f.bl;
    double dtl, dtu, dll, dlu, lml, lmu, tl, tu;
    if (FM == BX_P1) {
        dtl = x - f.bx[0] - f.bx[2];
        dtu = -x + f.bx[1] - f.bx[3];
        dll = f.bx[8] - (f.bx[4] * dtl + f.bx[6]);
        dlu = f.bx[9] - (f.bx[5] * dtu + f.bx[7]);
        lml = f.bx[6];
        lmu = f.bx[7];
        tl = f.bx[2];
        tu = f.bx[3];
    } else {
        double bx[10];
        use_pair(f.bx[0], f.bx[1], bx[0], bx[1]);
        use_pair(f.bx[4], f.bx[5], bx[4], bx[5]);
        if (!PRED) use_pair(f.bx[6], f.bx[7], bx[6], bx[7]);
        use_pair(f.bx[8], f.bx[9], bx[8], bx[9]);
        const double til = rcp_nr(bx[8]), tiu = rcp_nr(bx[9]);
        const double rml = PRED ? __dmul_rn(bx[4], bx[8]) : bx[6];
        const double rmu = PRED ? __dmul_rn(bx[5], bx[9]) : bx[7];
        dtl = x - bx[0];
        dtu = -x + bx[1];
        dll = -til * (bx[4] * dtl + rml);
        dlu = -tiu * (bx[5] * dtu + rmu);
        lml = bx[4];
        lmu = bx[5];
        tl = bx[8];
        tu = bx[9];
    }
    st_lu(bc.dt, b, dtl, dtu, b.ok);
    st_lu(bc.dlam, b, dll, dlu, b.ok);
    if (b.ok) {
        alpha_rule(al, lml, dll);
        alpha_rule(al, lmu, dlu);
        alpha_rule(al, tl, dtl);
        alpha_rule(al, tu, dtu);
    }
}

// pi_{k-1} = P_k x_k + p_k (the reference's Lxx (Lxx' x + l_x): dtrmv_u_n + dtrmv_u_t, d_back_ric_rec.c:355-365) from
// stage k's record S (P_k in its state rows), x_k in row layout and p_k in col layout (the record's l row in the sv,
// hux_k in the trs), stored over stage k's state tiles.  Formed at the start of stage k, where x_k is in row layout
// for the u solve anyway, instead of at the end of stage k-1 with a second layout change of the same x_k.
template <int MODE>
__device__ __forceinline__ void fwd_pi(int xo, int nx, int k, const d4& S, const double xrow[4], double pc,
                                       int compute_pi, double* pi) {
    const int g = lane_id() >> 4, c = lane_id() & 15;
    const int s = c - xo;
    const bool okp = s >= 0 && s < nx;
    double pv = 0.0;
    if (compute_pi && k > 0) pv = pi_from_x(S, xo, xrow, okp ? pc : 0.0);  // wave-uniform
    gst(pi, (k - 1) * V16 + s, pv, compute_pi && k > 0 && g == 0 && okp);
}

// One forward stage k < N: pi_{k-1}, u_k from the factor, x_{k+1} = b + BAbt' ux, box steps.
template <int MODE, int FM, bool PRED, class SH>
__device__ __forceinline__ void fwd_step(const RicIO& io, Scratch* sm, const SH& sh, int k, const FwdFrag& cur,
                                         double& xcol, double* ux, int compute_pi, double* pi, const BoxCtx& bc,
                                         double& al) {
    const int l = lane_id(), g = l >> 4, c = l & 15;
    const bool all = !SH::fixed && k == 0;
    double xrow[4];
    col2row(sm, xcol, xrow);
    if constexpr (!PRED) fwd_pi<MODE>(sh.xo, sh.nx, k, cur.S, xrow, MODE == 0 ? cur.lc : cur.hc, compute_pi, pi);
    const double rhs = (MODE == 0) ? cur.lc : cur.hc;
    double ur[4];
    if constexpr (SH::fixed) {
        // gain form (nu <= 4): u_g = sum_c KG[g][c] v[c], v = [rhs_u ; x] -- the reference's
        // u = -L_uu^{-T} (rhs_u + L_xu' x) as one 4x16 mat-vec (row sums over the 16 columns)
        const double v = (c < sh.xo) ? rhs : xcol;
        ur[0] = row_sum16(cur.kg * v);
#pragma unroll
        for (int r = 1; r < 4; r++) ur[r] = xrow[r];
        static_assert(SH::xo <= 4, "gain form needs the u block in tile block 0");
    } else {
        double part = 0.0;
        if (!all) {
#pragma unroll
            for (int r = 0; r < 4; r++) part += (g + 4 * r >= sh.xo) ? lowS(cur.S, r, g, c) * xrow[r] : 0.0;
        }
        const double rc = -rhs - xrow_sum(part);
        double rrow[4];
        col2row(sm, rc, rrow);
#pragma unroll
        for (int r = 0; r < 4; r++) ur[r] = all ? 0.0 : xrow[r];
        HK_STAMP(9, k);
        solve_lt(sh, cur.S, cur.invd, rrow, ur, all);
        HK_STAMP(10, k);
    }
    // ux_k, col layout (tile c): one coalesced store from row group 0, and the box steps
    const double ucol = row2col(sm, ur);
    const int vcs = tile_var(c, sh.nu, sh.nx, sh.xo);
    // the predictor's step is never read (the corrector's trs overwrites dux before reading it, and mu_aff
    // needs dt / dlam only): it is not stored
    if (!PRED) gst(ux, k * V16 + vcs, ucol, g == 0 && vcs >= 0);
    box_alpha<FM, PRED>(bc, cur, ucol, al);
    if constexpr (!SH::fixed && FM != BX_NONE) {
        if (sh.ng > 0) gen_alpha<FM>(io, sh, k, bc, ucol, al);
    }
    // x_{k+1} = b + BAbt_k' ux_k  (dgemv_t_lib alg 1, :347-351), col layout over stage-(k+1) tile
    double gp = 0.0;
#pragma unroll
    for (int r = 0; r < 4; r++) gp += cur.bt[r] * ur[r];
    const int s = c - sh.xo1;
    const bool ok = s >= 0 && s < sh.nx1;
    const double x1 = cur.bval + xrow_sum(gp);
    xcol = ok ? x1 : 0.0;
    HK_STAMP(11, k);
}

// Shared forward substitution (sv: rhs = -l_k ; trs: rhs = -hux_k), d_back_ric_rec.c:339-397 / :704-790.
// ux: variable order; pi: state order.  FM != BX_NONE also computes the box steps of every stage and
// the per-lane step-length candidate `al` (caller reduces it with wave_min).
template <int MODE, int FM, class FX, bool PRED = false>
__device__ void ric_forward(const RicIO& io, Scratch* sm, const double* bsrc, int use_bsrc, double* ux,
                            int compute_pi, double* pi, const BoxCtx& bc, double& al) {
    const int l = lane_id(), g = l >> 4, c = l & 15;
    double xcol = 0.0;  // x_k in col layout (stage-k tile coords)
    // Stage k runs on fa (its record) while stage k+2 is fetched into fc (fb, stage k+1's, is in flight); the
    // loop is unrolled by three with the fragments rotating roles (no register copies between stages).
    FwdFrag f0, f1, f2;
    fwd_fetch_k<MODE, FM, FX, PRED>(io, 0, bsrc, use_bsrc, ux, compute_pi, bc, f0);
    fwd_fetch_k<MODE, FM, FX, PRED>(io, 1, bsrc, use_bsrc, ux, compute_pi, bc, f1);
    auto stage = [&](int k, const FwdFrag& fa, const FwdFrag& fb, FwdFrag& fc) __attribute__((always_inline)) {
        (void)fb;  // stage k+1's fragment stays in flight (the prefetch depth), it is no longer read here
        HK_STAMP(8, k);
        fwd_fetch_k<MODE, FM, FX, PRED>(io, k + 2 <= io.N ? k + 2 : io.N, bsrc, use_bsrc, ux, compute_pi, bc, fc);
        const StageRef si{io.st, k};
        with_shape<FX>(si, [&](const auto& sh) {
            fwd_step<MODE, FM, PRED>(io, sm, sh, k, fa, xcol, ux, compute_pi, pi, bc, al);
        });
        HK_STAMP(12, k);
    };
    auto finish = [&](const FwdFrag& fN) __attribute__((always_inline)) {  // stage N: nu = 0, every tile a state
        const DynSh sN(StageRef{io.st, io.N});
        const int v = tile_var(c, sN.nu, sN.nx, sN.xo);
        if constexpr (!PRED) {
            // pi_{N-1} = P_N x_N + p_N: the fragment of stage N carries the record's l row but not hux_N (it is fetched
            // with stage N-1's shape), so the trs reads p_N here, before x_N overwrites ux_N
            double pc = MODE == 0 ? fN.lc : ldsel(ux + io.N * V16, v, compute_pi && v >= 0);
            double xrow[4] = {0.0, 0.0, 0.0, 0.0};
            if (compute_pi) col2row(sm, xcol, xrow);
            fwd_pi<MODE>(sN.xo, sN.nx, io.N, fN.S, xrow, pc, compute_pi, pi);
            gst(ux, io.N * V16 + v, xcol, g == 0 && v >= 0);
        }
        box_alpha<FM, PRED>(bc, fN, xcol, al);
    };
    for (int k = 0;;) {
        if (k >= io.N) { finish(f0); break; }
        stage(k, f0, f1, f2);
        if (++k >= io.N) { finish(f1); break; }
        stage(k, f1, f2, f0);
        if (++k >= io.N) { finish(f2); break; }
        stage(k, f2, f0, f1);
        ++k;
    }
    if (FM != BX_NONE) {
        const DynSh sN(StageRef{io.st, io.N});
        if (sN.ng > 0) gen_alpha<FM>(io, sN, io.N, bc, xcol, al);
    }
}

template <class FX>
__device__ __forceinline__ void ric_forward_sv(const RicIO& io, Scratch* sm, int update_b, const double* bsrc,
                                               double* ux, int compute_pi, double* pi) {
    BoxCtx bc{};
    double al = 1.0;
    ric_forward<0, BX_NONE, FX>(io, sm, bsrc, update_b, ux, compute_pi, pi, bc, al);
}

// ------------------------------------------------------------------------------------------------
// Riccati solve with an existing factor (trs).
// ------------------------------------------------------------------------------------------------
struct TrsFrag {
    d4 S;
    double invd;
    d4 bop;      // BAbt_k[var(c)][g+4r-xo1]
    d4 brow;     // hb_k in row layout over stage-(k+1) tile rows (compute_Pb)
    double h0;   // gradient q (col layout), box term added at use
    double pbc;  // stored Pb_k (col layout over stage-(k+1) tile) when !compute_Pb
    double bx[12];
    BoxLane bl;
};

// RPB = false: the caller never recomputes P b (the IPM corrector reuses the stored Pb), so the loads that
// only serve that product are not issued at all.
template <int TM, bool RPB, class SH>
__device__ __forceinline__ void trs_fetch(const RicIO& io, const SH& sh, int k, const double* hb, const double* hq,
                                          const BoxCtx& bc, int compute_Pb_, const double* Pb, TrsFrag& f) {
    const int compute_Pb = RPB ? compute_Pb_ : 0;
    const int l = lane_id(), g = l >> 4, c = l & 15;
    const double* Fk = io.F + (long)k * FSTRIDE;
    // a fixed-shape stage solves its u block in gain form (trs_usolve: KG in S[0], no pivots); rows 4..15 are
    // needed by the generic solve and by P_{k} b_{k-1} (compute_Pb, the KKT re-solve)
    if constexpr (SH::fixed) {  // packed record: the gain block KG into S[0] (trs_usolve), P only for a P b recompute
        f.S[0] = gld(Fk, FXR_KG + l);
        if (RPB) {
            load_p_fixed<SH::nx>(Fk, f.S, compute_Pb);
        } else {
            f.S[1] = f.S[2] = f.S[3] = 0.0;
        }
        f.invd = 0.0;
    } else {
#pragma unroll
        for (int r = 0; r < 4; r++) f.S[r] = gld(Fk, r * 64 + l);
        f.invd = gld(Fk, 272 + c);
    }
    const int nux = sh.nu + sh.nx;
    const int vc = tile_var(c, sh.nu, sh.nx, sh.xo);
    const double* R = stage_R(io, sh);
    f.h0 = hq ? ldsel(hq + k * V16, vc, vc >= 0) : ldsel(R, lib4_idx(sh.sdR, nux, vc), vc >= 0);
    const BoxLane b = box_lane(io.tileslot, sh.pnb, k);
    f.bl = b;
#pragma unroll
    for (int i = 0; i < 12; i++) f.bx[i] = 0.0;
    if (TM == BX_GIVEN) {
        f.bx[0] = ldsel(bc.qx, b.s16, b.ok);
    } else if (TM == BX_P1) {
        f.bx[0] = ldsel(bc.t_inv, b.lo, b.ok);
        f.bx[1] = ldsel(bc.t_inv, b.up, b.ok);
        f.bx[2] = ldsel(bc.dlam, b.lo, b.ok);
        f.bx[3] = ldsel(bc.dlam, b.up, b.ok);
        f.bx[4] = ldsel(bc.dt, b.lo, b.ok);
        f.bx[5] = ldsel(bc.dt, b.up, b.ok);
        f.bx[6] = ldsel(bc.qxs, b.s16, b.ok);
    } else if (TM == BX_P2) {  // [0..1]: t (r_m = lam t and 1/t are formed at use, bitwise the stored ones)
        // lower / upper pairs in one load each (even slot: the raw value, split at use by box_gradient)
        fetch_pair(bc.t, b, f.bx[0], f.bx[1]);
        fetch_pair(bc.dt, b, f.bx[2], f.bx[3]);
        fetch_pair(bc.dlam, b, f.bx[4], f.bx[5]);
        fetch_pair(bc.lam, b, f.bx[8], f.bx[9]);
        fetch_pair(bc.res_d, b, f.bx[10], f.bx[11]);
    }
    const bool live = SH::fixed || k < io.N;
    const double* Bk = stage_B(io, sh);
    const double* bp = hb ? hb + k * V16 : Bk;
#pragma unroll
    for (int r = 0; r < 4; r++) {
        const int sr = g + 4 * r - sh.xo1;
        const bool ok = live && sr >= 0 && sr < sh.nx1;
        f.bop[r] = ldsel(Bk, lib4_idx(sh.sdB, vc, sr), ok && vc >= 0);
        f.brow[r] = RPB ? ldsel(bp, hb ? sr : lib4_idx(sh.sdB, nux, sr), ok && compute_Pb) : 0.0;
    }
    const int s = c - sh.xo1;
    f.pbc = ldsel(Pb + k * V16, s, !compute_Pb && live && s >= 0 && s < sh.nx1);
}

// Corrector gradient of tile c (d_update_gradient_mpc_hard_tv :387-485 / centering correction +
// d_update_gradient_res_mpc_hard_tv :1512-1600): the box term added to the trs gradient.
template <int TM>
__device__ __forceinline__ double box_gradient(const BoxCtx& bc, const TrsFrag& f) {
    const int g = lane_id() >> 4;
    const BoxLane& b = f.bl;
    const bool st = b.ok && g == 0;
    if (TM == BX_GIVEN) return f.bx[0];
    if (TM == BX_P1) {
        const double dll = f.bx[0] * (bc.smu - f.bx[2] * f.bx[4]);
        const double dlu = f.bx[1] * (bc.smu - f.bx[3] * f.bx[5]);
        gst(bc.dlam, b.lo, dll, st);
        gst(bc.dlam, b.up, dlu, st);
        return b.ok ? f.bx[6] + (dlu - dll) : 0.0;
    }
    if (TM == BX_P2) {
        // r_m of the current iterate = lam t (the update pass's rounded product), 1/t = rcp_nr(t) (the
        // factorisation's stored t^-1): formed here instead of loaded
        double bx[12];
        use_pair(f.bx[0], f.bx[1], bx[0], bx[1]);
        use_pair(f.bx[2], f.bx[3], bx[2], bx[3]);
        use_pair(f.bx[4], f.bx[5], bx[4], bx[5]);
        use_pair(f.bx[8], f.bx[9], bx[8], bx[9]);
        use_pair(f.bx[10], f.bx[11], bx[10], bx[11]);
        const double til = rcp_nr(bx[0]), tiu = rcp_nr(bx[1]);
        const double rml = __dmul_rn(bx[8], bx[0]) + (bx[2] * bx[4] - bc.smu);
        const double rmu = __dmul_rn(bx[9], bx[1]) + (bx[3] * bx[5] - bc.smu);
        st_lu(bc.res_m, b, rml, rmu, b.ok);
        return b.ok ? til * (rml - bx[8] * bx[10]) - tiu * (rmu + bx[9] * bx[11]) : 0.0;
    }
    return 0.0;
}

// One backward trs stage k < N: hux_k = q_k + box + BAbt_k (P_{k+1} b_k + p_{k+1}), then the solve.
template <int TM, bool RPB, class SH>
__device__ __forceinline__ void trs_step(const RicIO& io, Scratch* sm, const SH& sh, int k, const TrsFrag& cur,
                                         const BoxCtx& bc, double* ux, int compute_Pb_, double* Pb, d4& S1,
                                         double& pcol) {
    const int compute_Pb = RPB ? compute_Pb_ : 0;
    const int l = lane_id(), g = l >> 4, c = l & 15;
    const int xo1 = sh.xo1, nx1 = sh.nx1;
    const int vc = tile_var(c, sh.nu, sh.nx, sh.xo);
    const int s = c - xo1;
    double pbc = cur.pbc;
    // P_{k+1} b_k is recomputed only on request (wave-uniform branch): the IPM corrector passes
    // compute_Pb = 0 and reuses the Pb its factorisation stored (d_ip2_res_hard.c:628, :1168)
    if (compute_Pb) {  // P_{k+1} b_k on the P-form record
        double part = 0.0;
#pragma unroll
        for (int r = 0; r < 4; r++) part += S1[r] * cur.brow[r];  // columns c < xo1: masked at use
        pbc = xrow_sum(part);
    }
    gst(Pb, k * V16 + s, pbc, compute_Pb && g == 0 && s >= 0 && s < nx1);
    const double wc = (s >= 0 && s < nx1) ? pbc + pcol : 0.0;
    double wrow[4];
    col2row(sm, wc, wrow);
    double part = 0.0;
#pragma unroll
    for (int r = 0; r < 4; r++) part += cur.bop[r] * wrow[r];
    double h = cur.h0 + box_gradient<TM>(bc, cur);  // dvecad_libsp (:612-620)
    if constexpr (!SH::fixed) {
        if (sh.ng > 0) h += gen_gradient<TM>(io, sh, k, bc);  // dgemv_n on DCt (:621-633)
    }
    h += xrow_sum(part);
    h = trs_usolve(sh, cur.S, cur.invd, h, !SH::fixed && k == 0);
    gst(ux, k * V16 + vc, h, g == 0 && vc >= 0);
    pcol = h;
    S1 = cur.S;
}

// Riccati solve with an existing factor (d_back_ric_rec.c:564-791).
// hb: state order, hq: variable order (null: the BAbt / RSQrq augmented rows), TM: box gradient term;
// ux (variable order) doubles as the backward work vector exactly like hux in the reference.
// FM != BX_NONE: box steps + step-length candidate `al` in the forward substitution.
template <int TM, int FM, class FX, bool RPB = true>
__device__ void ric_trs(const RicIO& io, Scratch* sm, const double* hb, const double* hq, const BoxCtx& bc,
                        double* ux, int compute_pi, double* pi, int compute_Pb, double* Pb, double& al) {
    const int l = lane_id(), g = l >> 4, c = l & 15;
    // ---- backward
    TrsFrag cur;
    with_shape<FX>(StageRef{io.st, io.N}, [&](const auto& sh) { trs_fetch<TM, RPB>(io, sh, io.N, hb, hq, bc, compute_Pb, Pb, cur); });
    double hN = cur.h0 + box_gradient<TM>(bc, cur);
    {
        const DynSh sN(StageRef{io.st, io.N});
        if (sN.ng > 0) hN += gen_gradient<TM>(io, sN, io.N, bc);
        const int v = tile_var(c, sN.nu, sN.nx, sN.xo);
        gst(ux, io.N * V16 + v, hN, g == 0 && v >= 0);
    }
    double pcol = hN;  // hux_{k+1} in col layout (stage-(k+1) tile coords)
    d4 S1 = cur.S;
    TrsFrag nxt;
    {
        with_shape<FX>(StageRef{io.st, io.N - 1}, [&](const auto& sh) { trs_fetch<TM, RPB>(io, sh, io.N - 1, hb, hq, bc, compute_Pb, Pb, nxt); });
    }
    // stage k on fa while stage k-1 is fetched into fb; unrolled by two, the fragments swap roles
    auto stage = [&](int k, const TrsFrag& fa, TrsFrag& fb) __attribute__((always_inline)) {
        const int kn = k > 0 ? k - 1 : 0;
        with_shape<FX>(StageRef{io.st, kn}, [&](const auto& sh) { trs_fetch<TM, RPB>(io, sh, kn, hb, hq, bc, compute_Pb, Pb, fb); });
        asm volatile("" ::: "memory");
        const StageRef si{io.st, k};
        with_shape<FX>(si, [&](const auto& sh) { trs_step<TM, RPB>(io, sm, sh, k, fa, bc, ux, compute_Pb, Pb, S1, pcol); });
    };
    for (int k = io.N - 1;;) {
        if (k < 0) break;
        stage(k, nxt, cur);
        if (--k < 0) break;
        stage(k, cur, nxt);
        --k;
    }
    __syncthreads();  // hux_k written by row group 0 is re-read by every lane below
    // ---- forward
    ric_forward<1, FM, FX>(io, sm, hb, hb != nullptr, ux, compute_pi, pi, bc, al);
}

}  // namespace hk
