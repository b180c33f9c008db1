// hk_mw.h -- the stage sweeps with one problem per WORKGROUP of four waves (configs[1]: a lone QP).
//
// A lone problem on one wavefront is bound by the wave's instruction issue: every stage of every sweep runs its
// recursion (the chain: the MFMA products of P, the u-block Cholesky, the triangular solves and mat-vecs from one
// stage to the next) interleaved with work that does not depend on the recursion at all -- the stage's loads, the
// box Hessian / gradient terms, the KKT residuals of the iterate, the box steps and the step-length rule, the
// multipliers pi and every store.  Here wave 0 runs the chain only and waves 1..3 ("helpers") run the rest, each
// helper taking every third stage:
//   backward (factorisation, d_back_ric_rec.c:186-335 inside d_ip2_res_hard.c's loop): a helper fetches stage k,
//     forms its residuals (BX_P2R) and box terms (bwd_pre) and hands wave 0 the ready stage tile M, the row ml
//     and the BAbt operands; wave 0 runs bwd_core (M += BAbt P BAbt', row update, u-block Cholesky) and stores
//     the stage record;
//   trs backward (:564-700): a helper hands over q + box gradient, the BAbt operand and the factor's u block;
//     wave 0 runs P b + p -> BAbt (.) -> the u solve;
//   forward (:339-397 / :704-790): wave 0 computes u_k and x_{k+1} and hands them (and p_{k+1}) to the helper of
//     stage k, which stores ux, forms the box steps, the step-length candidates and pi.
// The hand-over is a ring of MW_D slots in LDS (16 doubles per lane each) with a full / free flag per slot; the
// flags carry tickets that grow over the whole launch, so no sweep has to reset them.  Every value is computed by
// the same routine with the same operands as in the single-wave sweeps (hk_riccati.h); the step length is the
// minimum of the helpers' per-lane candidates.  The results are bitwise those of hk_ipm_solo only when the product
// terms are contracted into FMAs the same way in both kernels (they are with -ffp-contract=on, measured); under the
// default contraction hipcc fuses a few a * b + c differently once the bodies are split over waves, and the two
// agree to rounding (tests/test_gpu_parity.py test_solo_matches_batch).
// A wait that does not end (a bug, not a data condition) sets MwShared.err after ~2^22 polls and falls through,
// so every wave still reaches the end of the launch; the kernel then reports ret = HK_MW_ERR.
#pragma once
#include "hk_ipm.h"

namespace hk {

constexpr int MW_WAVES = 4, MW_HELP = 3;
constexpr int MW_D = 6;      // ring slots
constexpr int MW_SLOT = 16;  // doubles per lane per slot
constexpr int MW_DP = 6;     // tile wave -> row wave ring (backward sweep)
constexpr int MW_NMAX = 300;  // horizon limit of the multi-wave kernel (the update's reduction rows live in LDS)
constexpr int MW_RED = ((MW_NMAX + 4) / 4 + 3) / 4 * 4;
constexpr int HK_MW_ERR = -20;  // HPMPC_MI355X_EMW

struct MwShared {
    double ring[MW_D][MW_SLOT][64];
    double red[MW_RED][64];  // the update passes' per-quad r_m contributions (MwSplit)
    Scratch sm[MW_WAVES];
    double al[MW_WAVES];
    int full[MW_D], freed[MW_D];
    // backward sweep: the row wave's own free flags of the helpers' ring, and the tile wave -> row wave ring
    int freedB[MW_D];
    // [stage record tile (4) | inverse diagonal | a clamped stage's x factor (4) and its inverse diagonal]
    double ringP[MW_DP][10][64];
    int fullP[MW_DP], freedP[MW_DP];
    int xfacP[MW_DP];  // the stage failed the clamp certificate (stage_chol xfac): rows 5..9 are valid
    int err;
    int dbg[4];  // the first expired wait: flag index (full: slot, freed: MW_D + slot), expected, found, wave
#ifdef HK_STAMPS
    unsigned long long wait_cyc[MW_WAVES];  // cycles each wave spent in mw_wait (diagnostic build)
    unsigned long long seg[4];              // the tile wave's backward step by segment (diagnostic build)
#endif
};

// One object per workgroup of the multi-wave kernel, referred to by name everywhere (never through a pointer that
// could lose its address space): every access is a ds_ op, so a flag poll never waits on the global-memory counter.
__shared__ MwShared hk_mw;

#ifdef HK_STAMPS
// Diagnostic build only: a helper that "forgets" one hand-over (HPMPC_MI355X_MW_FAULT=1 at launch, hk_launch), so
// that tests/test_gpu_parity.py can check the expired-wait path: the waits expire, the launch drains, ret = -20.
__device__ int g_mw_fault;
#endif


__device__ __forceinline__ int mw_flag(const int* f) { return __atomic_load_n(f, __ATOMIC_RELAXED); }

// The hand-over's ordering.  Everything a hand-over moves -- slot data and flags -- is LDS, and the LDS performs one
// wave's ds_ instructions in issue order (for LDS-only traffic they also complete in order, which is why lgkmcnt
// can count them): a flag written after the slot data by the same wave cannot become visible before the data, and a
// consumer issues its slot reads only after the poll that saw the flag has returned.  The compiler keeps that order
// through the "memory" clobbers below (no LDS access moves across a post or a successful poll).
// HK_MW_FENCE=1 states the same order in the memory model instead -- a workgroup-scope release (LDS only) before
// each flag store and the matching acquire after each successful poll -- at the price of an s_waitcnt lgkmcnt(0)
// before every post, which also waits for the poster's unrelated scalar loads: a same-box A/B measured 350.4 vs
// 367.1-367.5 us per lone-QP IP iteration (3 pairs, profiles/r04/ab_latency.txt), 4.7 %, above the 2 % the fenced
// form was allowed, so it is a build option (tools/gpu_ab.sh variants) and not the default.
#ifndef HK_MW_FENCE
#define HK_MW_FENCE 0
#endif
__device__ __forceinline__ void mw_release_fence() {
#if HK_MW_FENCE
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
#else
    asm volatile("" ::: "memory");
#endif
}
__device__ __forceinline__ void mw_acquire_fence() {
#if HK_MW_FENCE
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
#else
    asm volatile("" ::: "memory");
#endif
}

__device__ __forceinline__ unsigned long long mw_clock() {
    unsigned long long t;
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
    return t;
}

// wait until flag *f (one of hk_mw's; always inlined, so it stays an LDS access) reaches v; i names the flag in the
// diagnostics
__device__ __forceinline__ void mw_wait_at(const int* f, int v, int i) {
#ifdef HK_STAMPS
    const unsigned long long t0 = mw_clock();
    struct Acc {
        unsigned long long t0;
        __device__ ~Acc() {
            if (lane_id() == 0) hk_mw.wait_cyc[threadIdx.x >> 6] += mw_clock() - t0;
        }
    } acc_{t0};
#endif
    int n = 0;
    while (mw_flag(f) < v) {
        if (++n > 64) __builtin_amdgcn_s_sleep(1);
        if (n > (1 << 22)) {
            if (lane_id() == 0 && mw_flag(&hk_mw.err) == 0) {
                hk_mw.dbg[0] = i;
                hk_mw.dbg[1] = v;
                hk_mw.dbg[2] = mw_flag(f);
                hk_mw.dbg[3] = (int)(threadIdx.x >> 6);
            }
            __atomic_store_n(&hk_mw.err, 1, __ATOMIC_RELAXED);
        }
        if (mw_flag(&hk_mw.err)) break;  // after one expired wait every wait falls through: the launch drains
    }
    mw_acquire_fence();
}

// wait until the flag (full[i] for i < MW_D, freed[i - MW_D] otherwise) reaches v
__device__ __forceinline__ void mw_wait(int i, int v) {
    mw_wait_at(i < MW_D ? &hk_mw.full[i] : &hk_mw.freed[i - MW_D], v, i);
}

// publish *f = v behind this wave's earlier LDS accesses (the slot data): a release (mw_release_fence) and a relaxed
// store from one lane.
__device__ __forceinline__ void mw_post_at(int* f, int v) {
    mw_release_fence();
    if (lane_id() == 0) __atomic_store_n(f, v, __ATOMIC_RELAXED);
    asm volatile("" ::: "memory");
}

// publish flag i (full[i] for i < MW_D, freed[i - MW_D] otherwise) = v
__device__ __forceinline__ void mw_post(int i, int v) {
    mw_post_at(i < MW_D ? &hk_mw.full[i] : &hk_mw.freed[i - MW_D], v);
}

// producer side of step j: wait for the slot's previous occupant (step j - MW_D of this sweep) to be consumed
__device__ __forceinline__ void mw_acquire(int tb, int j) {
    if (j >= MW_D) mw_wait(MW_D + j % MW_D, tb + j - MW_D + 1);
}

__device__ __forceinline__ void mw_put(int j, int i, double v) { hk_mw.ring[j % MW_D][i][lane_id()] = v; }
__device__ __forceinline__ double mw_get(int j, int i) { return hk_mw.ring[j % MW_D][i][lane_id()]; }

// ------------------------------------------------------------------------------------------------
// Backward factorisation (ric_backward), split over two recursions:
//   wave 0 (tile): M += BAbt P_{k+1} BAbt' and the tile half of the stage Cholesky -> P_k (bwd_tile_update,
//                  stage_chol without the row), handed to wave 1 through ringP = [record tile (4) | inv diag];
//   wave 1 (row):  P_{k+1} b, the row update ml += BAbt (P b + p_{k+1}), the row half of each Cholesky block, the
//                  gain block (stage_chol_row) and the stage record -- a second recursion (p_{k+1} -> p_k) that
//                  needs the tile wave's factor but never feeds it, so it runs one stage behind;
//   waves 2, 3 (helpers, every other stage): fetch, residuals, box terms -> ring = [M (4) | ml | bop (4) | brow (4) |
//                  dq | g] (dq, g: the box diagonal and the clamp-certificate bound, cert_ok), read by both
//                  recursions (its slot is free once both have read it).
// A stage that fails the clamp certificate is factorised as the reference does (stage_chol xfac): the tile wave
// carries P_eff on and hands the x factor to the row wave, which adds its row half and p_eff = Lxx l_x.
// ------------------------------------------------------------------------------------------------
constexpr int MW_BHELP = 2;

template <bool AUG, int BM, class FX>
__device__ __forceinline__ int ric_backward_mw(const RicIO& io, int tb, int w, int update_b, const double* bsrc,
                                               int update_q, const double* qsrc, const BoxCtx& bc, int compute_Pb,
                                               double* Pb) {
    const int N = io.N, l = lane_id(), c = l & 15;
    Scratch* sm = &hk_mw.sm[w];
    if (w >= 2) {
        // each helper walks its stages with one-step register prefetch: step j + MW_BHELP is fetched before step
        // j is computed (the unrolled pair swaps the fragments' roles)
        auto fetch = [&](int j, BwdFrag& f, double& x1c) __attribute__((always_inline)) {
            const int k = N - j;
            const StageInfo si = load_stage(io.st, k);
            with_shape<FX>(si, [&](const auto& sh) {
                bwd_fetch<AUG, BM>(io, sh, k, update_b, bsrc, update_q, qsrc, bc, f);
            });
            x1c = 0.0;
            if constexpr (BM == BX_P2R) {
                // x_{k+1} in col layout over the stage-(k+1) tile: the ux_{k+1} that the single-wave sweep's
                // previous fragment holds
                if (k < N) {
                    const StageInfo s1 = load_stage(io.st, k + 1);
                    const int v1 = tile_var(c, s1.nu, s1.nx, s1.xo);
                    x1c = ldsel(bc.ux, (k + 1) * V16 + v1, v1 >= 0);
                }
            }
        };
        auto work = [&](int j, BwdFrag& f, double x1c) __attribute__((always_inline)) {
            const int k = N - j;
            const StageInfo si = load_stage(io.st, k);
            d4 M;
            double ml, dq, gc;
            with_shape<FX>(si, [&](const auto& sh) {
                if constexpr (BM == BX_P2R) bwd_residual(io, sm, sh, k, bc, f, x1c, true);
                bwd_pre<AUG, BM>(io, sh, k, f, bc, M, ml, dq, gc);
            });
            if (j >= MW_D) {  // the slot's previous occupant read by both recursions
                mw_wait_at(&hk_mw.freed[j % MW_D], tb + j - MW_D + 1, MW_D + j % MW_D);
                mw_wait_at(&hk_mw.freedB[j % MW_D], tb + j - MW_D + 1, 2 * MW_D + j % MW_D);
            }
#pragma unroll
            for (int r = 0; r < 4; r++) {
                mw_put(j, r, M[r]);
                mw_put(j, 5 + r, f.bop[r]);
                mw_put(j, 9 + r, f.brow[r]);
            }
            mw_put(j, 4, ml);
            mw_put(j, 13, dq);
            mw_put(j, 14, gc);
#ifdef HK_STAMPS
            if (g_mw_fault && j == 3) return;  // the lost hand-over (diagnostic build)
#endif
            mw_post(j % MW_D, tb + j + 1);
        };
        BwdFrag fa, fb;
        double xa = 0.0, xb = 0.0;
        int j = w - 2;
        if (j <= N) fetch(j, fa, xa);
        for (;;) {
            if (j > N) break;
            if (j + MW_BHELP <= N) fetch(j + MW_BHELP, fb, xb);
            work(j, fa, xa);
            j += MW_BHELP;
            if (j > N) break;
            if (j + MW_BHELP <= N) fetch(j + MW_BHELP, fa, xa);
            work(j, fb, xb);
            j += MW_BHELP;
        }
    } else if (w == 0) {
        // the next step's slot is read while this step computes (its LDS latency off the recursion); the slot is
        // released once this step is done, by which time those reads have long completed
        d4 P = {0.0, 0.0, 0.0, 0.0};  // record tile of stage k+1 (its x block is P_{k+1})
        d4 Mn, bopn;
        double dqn, gcn;
        auto take = [&](int j) __attribute__((always_inline)) {
            mw_wait(j % MW_D, tb + j + 1);
#pragma unroll
            for (int r = 0; r < 4; r++) {
                Mn[r] = mw_get(j, r);
                bopn[r] = mw_get(j, 5 + r);
            }
            dqn = mw_get(j, 13);
            gcn = mw_get(j, 14);
        };
        take(0);
        StageInfo sn = load_stage(io.st, N);
#ifdef HK_STAMPS
        unsigned long long seg[4] = {0, 0, 0, 0}, tq = mw_clock();
#define MW_SEG(i)                                 \
    do {                                          \
        const unsigned long long t_ = mw_clock(); \
        seg[i] += t_ - tq;                        \
        tq = t_;                                  \
    } while (0)
#else
#define MW_SEG(i) \
    do {          \
    } while (0)
#endif
        for (int j = 0; j <= N; j++) {
            const int k = N - j;
            const StageInfo si = sn;
            d4 M = Mn;
            const d4 bop = bopn;
            const double dq = dqn, gc = gcn;
            if (j < N) {
                take(j + 1);
                sn = load_stage(io.st, k - 1);
            }
            MW_SEG(0);
            double invd;
            bool xfac = false;
            XFac xf;
            with_shape<FX>(si, [&](const auto& sh) {
                using SHT = std::remove_reference_t<decltype(sh)>;
                const bool live = SHT::fixed || k < N;
                bwd_tile_update(sh, live, bop, P, M);
                MW_SEG(1);
                double mld = 0.0;
                const bool full = !SHT::fixed && k == 0;
                // gc: the threshold T_k, tested on M after the tile update (cert_ok_thr)
                xfac = !full && !cert_test(M, dq, gc);
                stage_chol<false, false>(M, mld, invd, sh.nu, sh.nx, sh.xo, full, !SHT::fixed, nullptr, k, xfac, &xf);
                MW_SEG(2);
            });
            P = M;
            mw_post(MW_D + j % MW_D, tb + j + 1);  // step j's slot (read one step ago)
            if (j >= MW_DP) mw_wait_at(&hk_mw.freedP[j % MW_DP], tb + j - MW_DP + 1, 3 * MW_D + j % MW_DP);
#pragma unroll
            for (int r = 0; r < 4; r++) hk_mw.ringP[j % MW_DP][r][l] = P[r];
            hk_mw.ringP[j % MW_DP][4][l] = invd;
            if (xfac) {  // wave-uniform
#pragma unroll
                for (int r = 0; r < 4; r++) hk_mw.ringP[j % MW_DP][5 + r][l] = xf.L[r];
                hk_mw.ringP[j % MW_DP][9][l] = xf.invd;
            }
            if (l == 0) hk_mw.xfacP[j % MW_DP] = xfac ? 1 : 0;
            mw_post_at(&hk_mw.fullP[j % MW_DP], tb + j + 1);
            MW_SEG(3);
        }
#ifdef HK_STAMPS
        if (l == 0)
            for (int i = 0; i < 4; i++) hk_mw.seg[i] += seg[i];
#endif
#undef MW_SEG
    } else {
        d4 P1 = {0.0, 0.0, 0.0, 0.0};  // record tile of stage k+1
        double ml_prev = 0.0;           // its row [l_u; p_{k+1}]
        for (int j = 0; j <= N; j++) {
            const int k = N - j;
            const StageInfo si = load_stage(io.st, k);
            mw_wait(j % MW_D, tb + j + 1);
            d4 bop, brow;
#pragma unroll
            for (int r = 0; r < 4; r++) {
                bop[r] = mw_get(j, 5 + r);
                brow[r] = mw_get(j, 9 + r);
            }
            double ml = mw_get(j, 4);
            mw_post_at(&hk_mw.freedB[j % MW_D], tb + j + 1);
            // the row update needs only P_{k+1} (held from the previous step): it runs while the tile wave
            // factorises stage k
            with_shape<FX>(si, [&](const auto& sh) {
                using SHT = std::remove_reference_t<decltype(sh)>;
                if (AUG) bwd_row_update(io, sm, sh, k, SHT::fixed || k < N, bop, brow, P1, ml_prev, compute_Pb, Pb, ml);
            });
            mw_wait_at(&hk_mw.fullP[j % MW_DP], tb + j + 1, 4 * MW_D + j % MW_DP);
            d4 S;
#pragma unroll
            for (int r = 0; r < 4; r++) S[r] = hk_mw.ringP[j % MW_DP][r][l];
            const double invd = hk_mw.ringP[j % MW_DP][4][l];
            const bool xfac = __builtin_amdgcn_readfirstlane(hk_mw.xfacP[j % MW_DP]) != 0;
            XFac xf;
            if (xfac) {
#pragma unroll
                for (int r = 0; r < 4; r++) xf.L[r] = hk_mw.ringP[j % MW_DP][5 + r][l];
                xf.invd = hk_mw.ringP[j % MW_DP][9][l];
            }
            mw_post_at(&hk_mw.freedP[j % MW_DP], tb + j + 1);
            double kg = 0.0;
            with_shape<FX>(si, [&](const auto& sh) {
                using SHT = std::remove_reference_t<decltype(sh)>;
                stage_chol_row<AUG, SHT::fixed>(S, invd, ml, sh.nu, sh.nx, sh.xo, !SHT::fixed && k == 0, &kg);
                if (AUG && xfac) {  // the clamped x block's row half and p_eff = Lxx l_x (stage_chol xfac)
                    double lx = ml;
                    xblocks_chol_row(xf.L, xf.invd, lx, sh.nx, sh.xo);
                    pform_eff_row(xf.L, lx, sh.nx, sh.xo, ml);
                }
                // the stage record, in the format of the stage's shape class (as ric_backward)
                double* Fk = io.F + (long)k * FSTRIDE;
                if constexpr (SHT::fixed)
                    store_factor_fixed<SHT::nx>(Fk, S, AUG ? ml : 0.0, invd, kg, true);
                else
                    store_factor(Fk, S, AUG ? ml : 0.0, invd, kg);
            });
            P1 = S;
            ml_prev = ml;
        }
    }
    return tb + N + 2;
}

// ------------------------------------------------------------------------------------------------
// Forward substitution (ric_forward), wave 0 -> helpers: slot = [u_k (col) | x_{k+1} (col, masked) | p_{k+1}].
// ------------------------------------------------------------------------------------------------
// What wave 0 reads of stage k: the gain block (fixed shapes) or the factor (generic), the rhs row, BAbt' and b;
// MODE 1 also hux_k and, for pi on generic stages, p_{k+1} (read here, before any helper overwrites ux_{k+1}).
template <int MODE, class SH>
__device__ __forceinline__ void fwd_fetch_chain(const RicIO& io, const SH& sh, int k, const double* bsrc,
                                                int use_bsrc, const double* ux, int compute_pi, FwdFrag& f) {
    const int l = lane_id(), g = l >> 4, c = l & 15;
    const double* Fk = io.F + (long)k * FSTRIDE;
    if constexpr (SH::fixed) {
        f.lc = MODE == 0 ? gld(Fk, FXR_L + c) : 0.0;
        f.kg = gld(Fk, FXR_KG + l);
    } else {
#pragma unroll
        for (int r = 0; r < 4; r++) f.S[r] = gld(Fk, r * 64 + l);
        f.lc = MODE == 0 ? gld(Fk, 256 + c) : 0.0;
        f.invd = gld(Fk, 272 + c);
    }
    const int kk = k < io.N ? k : io.N - 1;
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
        f.pk = SH::fixed ? 0.0 : ldsel(ux + (kk + 1) * V16, sh.nu1 + s, compute_pi && ok);
    }
}

template <int MODE, class FX>
__device__ __forceinline__ void fwd_fetch_chain_k(const RicIO& io, int k, const double* bsrc, int use_bsrc,
                                                  const double* ux, int compute_pi, FwdFrag& f) {
    const int kk = k < io.N ? k : io.N - 1;
    const StageInfo sk = load_stage(io.st, kk);
    with_shape<FX>(sk, [&](const auto& sh) { fwd_fetch_chain<MODE>(io, sh, k, bsrc, use_bsrc, ux, compute_pi, f); });
}

// The chain half of fwd_step: u_k (the gain form or the dtrsv_t solve) and x_{k+1} = b + BAbt' ux.
template <int MODE, class SH>
__device__ __forceinline__ void fwd_chain(Scratch* sm, const SH& sh, int k, const FwdFrag& cur, double& xcol,
                                          double& ucol) {
    const int l = lane_id(), g = l >> 4, c = l & 15;
    const bool all = !SH::fixed && k == 0;
    double xrow[4];
    col2row(sm, xcol, xrow);
    const double rhs = (MODE == 0) ? cur.lc : cur.hc;
    double ur[4];
    if constexpr (SH::fixed) {
        const double v = (c < sh.xo) ? rhs : xcol;
        ur[0] = row_sum16(cur.kg * v);
#pragma unroll
        for (int r = 1; r < 4; r++) ur[r] = xrow[r];
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
        solve_lt(sh, cur.S, cur.invd, rrow, ur, all);
    }
    ucol = row2col(sm, ur);
    double gp = 0.0;
#pragma unroll
    for (int r = 0; r < 4; r++) gp += cur.bt[r] * ur[r];
    const int s = c - sh.xo1;
    const bool ok = s >= 0 && s < sh.nx1;
    const double x1 = cur.bval + xrow_sum(gp);
    xcol = ok ? x1 : 0.0;
}

template <int MODE, int FM, class FX, bool PRED = false>
__device__ __forceinline__ int ric_forward_mw(const RicIO& io, int tb, int w, const double* bsrc, int use_bsrc,
                               double* ux, int compute_pi_, double* pi, const BoxCtx& bc, double& al_out) {
    const int N = io.N, l = lane_id(), g = l >> 4, c = l & 15;
    const int compute_pi = PRED ? 0 : compute_pi_;
    Scratch* sm = &hk_mw.sm[w];
    double al = 1.0;
    if (w == 0) {
        double xcol = 0.0;
        FwdFrag f0, f1, f2;
        fwd_fetch_chain_k<MODE, FX>(io, 0, bsrc, use_bsrc, ux, compute_pi, f0);
        fwd_fetch_chain_k<MODE, FX>(io, 1 <= N ? 1 : N, bsrc, use_bsrc, ux, compute_pi, f1);
        auto stage = [&](int k, const FwdFrag& fa, const FwdFrag& fb, FwdFrag& fc) __attribute__((always_inline)) {
            fwd_fetch_chain_k<MODE, FX>(io, k + 2 <= N ? k + 2 : N, bsrc, use_bsrc, ux, compute_pi, fc);
            const StageInfo si = load_stage(io.st, k);
            double ucol = 0.0, p1 = 0.0;
            with_shape<FX>(si, [&](const auto& sh) {
                fwd_chain<MODE>(sm, sh, k, fa, xcol, ucol);
                if (MODE == 1) {
                    // p_{k+1} for pi_k: the next fragment's hux_{k+1} (fixed stages) or the loaded x part (as
                    // fwd_step); masked lanes are never stored
                    const int s = c - sh.xo1;
                    const bool ok = s >= 0 && s < sh.nx1;
                    p1 = std::remove_reference_t<decltype(sh)>::fixed ? (ok ? fb.hc : 0.0) : fa.pk;
                }
            });
            mw_acquire(tb, k);
            mw_put(k, 0, ucol);
            mw_put(k, 1, xcol);
            mw_put(k, 2, p1);
            mw_post(k % MW_D, tb + k + 1);
        };
        for (int k = 0;;) {
            if (k >= N) break;
            stage(k, f0, f1, f2);
            if (++k >= N) break;
            stage(k, f1, f2, f0);
            if (++k >= N) break;
            stage(k, f2, f0, f1);
            ++k;
        }
        mw_acquire(tb, N);  // stage N: x_N
        mw_put(N, 0, xcol);
        mw_put(N, 1, 0.0);
        mw_put(N, 2, 0.0);
        mw_post(N % MW_D, tb + N + 1);
    } else {
        auto fetch = [&](int k, FwdFrag& fc, FwdFrag& fn) __attribute__((always_inline)) {
            fwd_fetch_k<MODE, FM, FX, PRED>(io, k, bsrc, use_bsrc, ux, 0, bc, fc);
            if (compute_pi && k < N) fwd_fetch_k<MODE, FM, FX, PRED>(io, k + 1, bsrc, use_bsrc, ux, compute_pi, bc, fn);
        };
        auto work = [&](int k, const FwdFrag& fc, const FwdFrag& fn) __attribute__((always_inline)) {
            mw_wait(k % MW_D, tb + k + 1);
            const double ucol = mw_get(k, 0), x1 = mw_get(k, 1), p1 = mw_get(k, 2);
            mw_post(MW_D + k % MW_D, tb + k + 1);
            if (k < N) {
                const StageInfo si = load_stage(io.st, k);
                with_shape<FX>(si, [&](const auto& sh) {
                    using SHT = std::remove_reference_t<decltype(sh)>;
                    const int vcs = tile_var(c, sh.nu, sh.nx, sh.xo);
                    if (!PRED) gst(ux, k * V16 + vcs, ucol, g == 0 && vcs >= 0);
                    box_alpha<FM, PRED>(bc, fc, ucol, al);
                    if constexpr (!SHT::fixed && FM != BX_NONE) {
                        if (sh.ng > 0) gen_alpha<FM>(io, sh, k, bc, ucol, al);
                    }
                    const int s = c - sh.xo1;
                    const bool ok = s >= 0 && s < sh.nx1;
                    double pv = 0.0;
                    if (compute_pi) {
                        double x1row[4];
                        col2row(sm, x1, x1row);
                        pv = pi_from_x(fn.S, sh.xo1, x1row, MODE == 0 ? fn.lc : p1);
                    }
                    gst(pi, k * V16 + s, pv, compute_pi && g == 0 && ok);
                });
            } else {
                const StageInfo sN = load_stage(io.st, N);
                const int v = tile_var(c, sN.nu, sN.nx, sN.xo);
                if (!PRED) gst(ux, N * V16 + v, ucol, g == 0 && v >= 0);
                box_alpha<FM, PRED>(bc, fc, ucol, al);
                if (FM != BX_NONE && sN.ng > 0) gen_alpha<FM>(io, DynSh(sN), N, bc, ucol, al);
            }
        };
        FwdFrag ca, na, cb, nb;
        int k = w - 1;
        if (k <= N) fetch(k, ca, na);
        for (;;) {
            if (k > N) break;
            if (k + MW_HELP <= N) fetch(k + MW_HELP, cb, nb);
            work(k, ca, na);
            k += MW_HELP;
            if (k > N) break;
            if (k + MW_HELP <= N) fetch(k + MW_HELP, ca, na);
            work(k, cb, nb);
            k += MW_HELP;
        }
    }
    al = wave_min(al);
    if (l == 0) hk_mw.al[w] = al;
    __syncthreads();
    al_out = fmin(fmin(hk_mw.al[0], hk_mw.al[1]), fmin(hk_mw.al[2], hk_mw.al[3]));
    return tb + N + 2;
}

// ------------------------------------------------------------------------------------------------
// Riccati solve with the existing factor (ric_trs, RPB = false: the stored P b), helpers -> wave 0:
// slot = [q + box gradient | bop (4) | S (4) | invd | Pb].
// ------------------------------------------------------------------------------------------------
template <int TM, int FM, class FX>
__device__ __forceinline__ int ric_trs_mw(const RicIO& io, int tb, int w, const double* hb, const double* hq,
                           const BoxCtx& bc, double* ux, int compute_pi, double* pi, double* Pb, double& al) {
    const int N = io.N, l = lane_id(), g = l >> 4, c = l & 15;
    Scratch* sm = &hk_mw.sm[w];
    if (w > 0) {
        auto fetch = [&](int j, TrsFrag& f) __attribute__((always_inline)) {
            const int k = N - j;
            const StageInfo si = load_stage(io.st, k);
            with_shape<FX>(si, [&](const auto& sh) { trs_fetch<TM, false>(io, sh, k, hb, hq, bc, 0, Pb, f); });
        };
        auto work = [&](int j, const TrsFrag& f) __attribute__((always_inline)) {
            const int k = N - j;
            const StageInfo si = load_stage(io.st, k);
            double hpre = 0.0;
            with_shape<FX>(si, [&](const auto& sh) {
                using SHT = std::remove_reference_t<decltype(sh)>;
                hpre = f.h0 + box_gradient<TM>(bc, f);  // dvecad_libsp (:612-620)
                if constexpr (!SHT::fixed) {
                    if (sh.ng > 0) hpre += gen_gradient<TM>(io, sh, k, bc);  // dgemv_n on DCt (:621-633)
                }
            });
            mw_acquire(tb, j);
            mw_put(j, 0, hpre);
#pragma unroll
            for (int r = 0; r < 4; r++) {
                mw_put(j, 1 + r, f.bop[r]);
                mw_put(j, 5 + r, f.S[r]);
            }
            mw_put(j, 9, f.invd);
            mw_put(j, 10, f.pbc);
            mw_post(j % MW_D, tb + j + 1);
        };
        TrsFrag fa, fb;
        int j = w - 1;
        if (j <= N) fetch(j, fa);
        for (;;) {
            if (j > N) break;
            if (j + MW_HELP <= N) fetch(j + MW_HELP, fb);
            work(j, fa);
            j += MW_HELP;
            if (j > N) break;
            if (j + MW_HELP <= N) fetch(j + MW_HELP, fa);
            work(j, fb);
            j += MW_HELP;
        }
    } else {
        // as the factorisation's tile wave: the next step's slot is read while this step computes
        double pcol = 0.0;
        double hn, invdn, pbcn;
        d4 bopn, Sn;
        auto take = [&](int j) __attribute__((always_inline)) {
            mw_wait(j % MW_D, tb + j + 1);
            hn = mw_get(j, 0);
#pragma unroll
            for (int r = 0; r < 4; r++) {
                bopn[r] = mw_get(j, 1 + r);
                Sn[r] = mw_get(j, 5 + r);
            }
            invdn = mw_get(j, 9);
            pbcn = mw_get(j, 10);
        };
        take(0);
        StageInfo sn = load_stage(io.st, N);
        for (int j = 0; j <= N; j++) {
            const int k = N - j;
            const StageInfo si = sn;
            const double hpre = hn, invd = invdn, pbc = pbcn;
            const d4 bop = bopn, Sk = Sn;
            if (j < N) {
                take(j + 1);
                sn = load_stage(io.st, k - 1);
            }
            if (k == N) {  // stage N: hux_N = q_N + box (+ general) gradient, no u block
                const int v = tile_var(c, si.nu, si.nx, si.xo);
                gst(ux, N * V16 + v, hpre, g == 0 && v >= 0);
                pcol = hpre;
            } else {
                with_shape<FX>(si, [&](const auto& sh) {
                    using SHT = std::remove_reference_t<decltype(sh)>;
                    const int xo1 = sh.xo1, nx1 = sh.nx1;
                    const int vc = tile_var(c, sh.nu, sh.nx, sh.xo);
                    const int s = c - xo1;
                    const double wc = (s >= 0 && s < nx1) ? pbc + pcol : 0.0;
                    double wrow[4];
                    col2row(sm, wc, wrow);
                    double part = 0.0;
#pragma unroll
                    for (int r = 0; r < 4; r++) part += bop[r] * wrow[r];
                    double h = hpre;
                    h += xrow_sum(part);
                    h = trs_usolve(sh, Sk, invd, h, !SHT::fixed && k == 0);
                    gst(ux, k * V16 + vc, h, g == 0 && vc >= 0);
                    pcol = h;
                });
            }
            mw_post(MW_D + j % MW_D, tb + j + 1);
        }
    }
    __syncthreads();  // hux written by wave 0 is read by the forward below
    return ric_forward_mw<1, FM, FX>(io, tb + N + 2, w, hb, hb != nullptr, ux, compute_pi, pi, bc, al);
}

}  // namespace hk
