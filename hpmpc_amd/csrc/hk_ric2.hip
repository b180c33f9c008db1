// hk_ric2.hip -- d_back_ric_rec_sv_tv_res over a batch with TWO waves per problem (gfx950).
//
// At the benchmark batches (1024 problems) the one-wave kernel (hpmpc_kernels.hip hk_ric_sv) leaves one wave per
// SIMD, and that wave is bound by its own issue: a backward stage of the compiled (4, 12) class executes ~440
// instructions (tools/loop_icount.py), the SIMD's VALU is ~25 % busy and the wave parks on s_waitcnt for ~47 % of its
// cycles (profiles/r04b_pmc_mix.json).  Here each problem gets a 128-thread workgroup and the work is split by
// dependency, as in the multi-wave lone-QP kernel (hk_mw.h) but with two roles and a small LDS footprint (four
// workgroups per CU):
//
//   backward sweep (lqcp_solvers/d_back_ric_rec.c:186-335), step j = stage k = N - j
//     wave 0 (tile): M += BAbt_k P_{k+1} BAbt_k' (MFMA), the clamp certificate (cert_ok) and the tile half of the
//                    u-block Cholesky -> P_k -- the only chain that carries the recursion forward;
//     wave 1 (row):  one step behind wave 0, the augmented row (P b, ml += BAbt (P b + p), the row half of the Cholesky,
//                    the gain block) and the stage record -- a second recursion (p_{k+1} -> p_k) that needs wave 0's
//                    factor but never feeds it (hk_mw.h, same routines) -- then, two steps ahead of wave 0, the fetch
//                    and the ready tile of stage j + 2 (RSQ + box terms, bwd_pre) with the BAbt operand.
//   forward sweep (:339-397), in blocks of R2_H stages
//     wave 0: u_k = KG [rhs_u; x_k] and x_{k+1} = b_k + BAbt_k' ux_k (fwd_chain, the chain only);
//     wave 1, one block behind: stores ux_k and forms pi_{k-1} = P_k x_k + p_k from stage k's record (fwd_pi).
// Every value is produced by the same routine on the same operands as in hk_ric_sv (hk_riccati.h), so the results
// agree with it up to the compiler's FMA contraction (tests/test_gpu_ric2.py holds both to the goldens and the oracle).
//
// Synchronisation: the waves exchange through LDS rings and meet at one s_barrier per backward step and one per
// forward block.  A waiting wave sleeps at the barrier instead of polling a flag (a polling wave takes issue slots from
// the wave it waits for when they share a SIMD).  The barrier is preceded by s_waitcnt lgkmcnt(0) only: the ring writes
// are complete, wave 1's prefetched loads stay in flight across it.  Every slot's reuse is ordered by a barrier (the
// comments at each ring say which).
#include "hk_mw.h"
#include "hk_launch_guard.h"
#include "hpmpc_kargs.h"

using namespace hk;

namespace {

constexpr int R2_D = 3;       // backward stage slots (wave 1 writes step j + 2 while wave 0 reads step j + 1)
constexpr int R2_ROWS = 10;   // M (4) | bop (4) | dq | ml
constexpr int R2_DP = 2;      // backward factor slots (wave 0 writes step j, wave 1 reads step j - 1)
constexpr int R2_PROWS = 10;  // record tile (4) | inverse diagonal | a clamped stage's x factor (4) and inverse diagonal
constexpr int R2_H = 6;       // forward block (stages per barrier)

struct R2Shared {
    union {
        double mring[R2_D][R2_ROWS][64];
        double fring[2 * R2_H][2][64];  // forward: [ucol | xcol] of two blocks, over the backward's stage ring
    };
    double pring[R2_DP][R2_PROWS][64];
    Scratch sm[2];
    double mgc[R2_D];  // the stage's certificate bound g (wave-uniform)
    int xfac[R2_DP];
};
static_assert(2 * R2_H * 2 <= R2_D * R2_ROWS, "forward ring overlay");

// one object per workgroup, referred to by name (every access stays a ds_ op; hk_mw.h)
__shared__ R2Shared r2;

// The two waves' meeting point: this wave's LDS writes are complete, then the workgroup barrier (no vmcnt wait).
__device__ __forceinline__ void r2_bar() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

// Diagnostic build (-DHK_STAMPS, tools/ric_waves_probe.py --stamps): s_memtime totals of problem 0 into KArgs.dbg --
// [0] / [1] wave 0's backward work / barrier wait, [2] / [3] wave 1's, [4] / [5] wave 0's forward work / wait, [6] / [7]
// wave 1's; wave 0's backward step by segment: [8] shape dispatch, [9] tile update + certificate, [10] Cholesky tile
// half, [11] the whole step before the barrier.  Stamps wait for the wave's LDS operations.
#ifdef HK_STAMPS
__device__ unsigned long long* r2_dbg;
#define R2_T0(v) unsigned long long v = mw_clock()
#define R2_ADD(i, d)                                                         \
    do {                                                                     \
        if (r2_dbg && blockIdx.x == 0 && lane_id() == 0) r2_dbg[i] += (d); \
    } while (0)
// a barrier whose wait is charged to stamp slot i, the work since the previous barrier to slot i - 1
#define R2_STEP_BAR(tprev, i)                      \
    do {                                           \
        const unsigned long long t_a = mw_clock(); \
        r2_bar();                                  \
        const unsigned long long t_b = mw_clock(); \
        R2_ADD((i) - 1, t_a - tprev);              \
        R2_ADD(i, t_b - t_a);                      \
        tprev = t_b;                               \
    } while (0)
#else
#define R2_T0(v) \
    do {         \
    } while (0)
#define R2_STEP_BAR(tprev, i) r2_bar()
#endif
#ifdef HK_STAMPS
#define R2_SEG(i, d) R2_ADD(i, d)
#else
#define R2_SEG(i, d) \
    do {             \
    } while (0)
#endif

// The stage-table copies of lds_tables (hpmpc_kernels.hip) for a 128-thread workgroup: StageInfo[N+1] and the
// tile -> box-slot table (the sv's box terms); the rings are the static r2 object.
struct R2Tabs {
    const StageInfo* st;
    const signed char* tileslot;
};
extern __shared__ __attribute__((aligned(16))) char hk_smem2[];

__device__ __forceinline__ R2Tabs r2_tables(const KArgs& a) {
    StageInfo* st = reinterpret_cast<StageInfo*>(hk_smem2);
    signed char* ts = reinterpret_cast<signed char*>(st + (a.N + 1));
    const int t = threadIdx.x, n1 = a.N + 1;
    const int* gs = reinterpret_cast<const int*>(a.st);
    int* ls = reinterpret_cast<int*>(st);
    for (int i = t; i < n1 * 16; i += 128) ls[i] = gs[i];
    const int* gt = reinterpret_cast<const int*>(a.tileslot);
    int* lt = reinterpret_cast<int*>(ts);
    for (int i = t; i < n1 * 4; i += 128) lt[i] = gt[i];
    __syncthreads();
    return R2Tabs{st, ts};
}

__host__ __device__ constexpr size_t r2_lds_bytes(int N) { return (size_t)(N + 1) * (sizeof(StageInfo) + 16); }

// What wave 1's row half reads of stage k beside the ring: the BAbt operand and b (as bwd_fetch, AUG).
struct RowFrag {
    d4 bop, brow;
};
template <class SH>
__device__ __forceinline__ void row_fetch(const RicIO& io, const SH& sh, int k, int update_b, const double* bsrc,
                                          RowFrag& f) {
    const int l = lane_id(), g = l >> 4, c = l & 15;
    const int nux = sh.nu + sh.nx;
    const int vc = tile_var(c, sh.nu, sh.nx, sh.xo);
    const bool live = SH::fixed || k < io.N;
    const double* Bk = stage_B(io, sh);
    const double* bp = update_b ? bsrc + k * V16 : Bk;
#pragma unroll
    for (int r = 0; r < 4; r++) {
        const int s = 4 * r + g - sh.xo1;
        const bool ok = live && s >= 0 && s < sh.nx1;
        f.bop[r] = ldsel(Bk, lib4_idx(sh.sdB, vc, s), ok && vc >= 0);
        f.brow[r] = ldsel(bp, update_b ? s : lib4_idx(sh.sdB, nux, s), ok);
    }
}

// ------------------------------------------------------------------------------------------------
// Backward sweep.  Step j is stage k = N - j; steps 0 .. N + 1 (wave 1's row half of stage 0 is step N + 1), each
// ending at one barrier of both waves; a prologue barrier hands over the first two tiles.
//   stage slot s % 3: written by wave 1 (prep) at step s - 2 (s = 0, 1: the prologue), read by wave 0 at step s - 1
//     (its next tile, into registers at the end of the step) and by wave 1's row half at step s + 1 (ml), before
//     wave 1 overwrites it with stage s + 3 in the same step;
//   factor slot s % 2: written by wave 0 at step s, read by wave 1 at step s + 1; rewritten at step s + 2.
// ------------------------------------------------------------------------------------------------
template <int BM, class FX>
__device__ __forceinline__ void ric_backward2(const RicIO& io, int w, int update_b, const double* bsrc, int update_q,
                                              const double* qsrc, const BoxCtx& bc, int compute_Pb, double* Pb) {
    const int N = io.N, l = lane_id();
    if (w == 0) {
        d4 P = {0.0, 0.0, 0.0, 0.0};  // record tile of stage k+1 (its x block is P_{k+1})
        d4 M, bop;
        double dq, gc;
        auto take = [&](int s) __attribute__((always_inline)) {
            const int q = s % R2_D;
#pragma unroll
            for (int r = 0; r < 4; r++) {
                M[r] = r2.mring[q][r][l];
                bop[r] = r2.mring[q][4 + r][l];
            }
            dq = r2.mring[q][8][l];
            gc = r2.mgc[q];
        };
        R2_T0(tp);
        r2_bar();  // prologue: stage slots 0 and 1
        take(0);
        for (int j = 0; j <= N + 1; j++) {
            if (j <= N) {
                const int k = N - j;
                double invd;
                bool xfac = false;
                XFac xf;
                R2_T0(ts0);
                with_shape<FX>(StageRef{io.st, k}, [&](const auto& sh) {
                    using SHT = std::remove_reference_t<decltype(sh)>;
                    R2_T0(ts1);
                    bwd_tile_update(sh, SHT::fixed || k < N, bop, P, M);
                    double mld = 0.0;
                    const bool full = !SHT::fixed && k == 0;
                    xfac = !full && !cert_test(M, dq, gc);  // gc: cert_form's T_k
                    R2_T0(ts2);
                    stage_chol<false, false>(M, mld, invd, sh.nu, sh.nx, sh.xo, full, !SHT::fixed, nullptr, k, xfac,
                                             &xf);
                    R2_T0(ts3);
                    R2_SEG(8, ts1 - ts0);
                    R2_SEG(9, ts2 - ts1);
                    R2_SEG(10, ts3 - ts2);
                });
                P = M;
                const int s = j % R2_DP;
#pragma unroll
                for (int r = 0; r < 4; r++) r2.pring[s][r][l] = P[r];
                r2.pring[s][4][l] = invd;
                if (xfac) {  // wave-uniform
#pragma unroll
                    for (int r = 0; r < 4; r++) r2.pring[s][5 + r][l] = xf.L[r];
                    r2.pring[s][9][l] = xf.invd;
                }
                if (l == 0) r2.xfac[s] = xfac ? 1 : 0;
                if (j < N) take(j + 1);  // written by wave 1 at step j - 1 (or the prologue)
                R2_T0(ts4);
                R2_SEG(11, ts4 - ts0);
            }
            R2_STEP_BAR(tp, 1);
        }
    } else {
        Scratch* sm = &r2.sm[1];
        auto fetch = [&](int j, BwdFrag& f) __attribute__((always_inline)) {
            const int k = N - j;
            with_shape<FX>(StageRef{io.st, k}, [&](const auto& sh) {
                bwd_fetch<true, BM>(io, sh, k, update_b, bsrc, update_q, qsrc, bc, f);
            });
        };
        auto prep = [&](int j, const BwdFrag& f) __attribute__((always_inline)) {
            const int k = N - j;
            d4 M;
            double ml, dq, gc;
            with_shape<FX>(StageRef{io.st, k}, [&](const auto& sh) {
                bwd_pre<true, BM, CERT_RT>(io, sh, k, f, bc, M, ml, dq, gc);
            });
            const int q = j % R2_D;
#pragma unroll
            for (int r = 0; r < 4; r++) {
                r2.mring[q][r][l] = M[r];
                r2.mring[q][4 + r][l] = f.bop[r];
            }
            r2.mring[q][8][l] = dq;
            r2.mring[q][9][l] = ml;
            if (l == 0) r2.mgc[q] = gc;
        };
        d4 P1 = {0.0, 0.0, 0.0, 0.0};  // record tile of stage k+1
        double ml_prev = 0.0;           // its row [l_u; p_{k+1}]
        auto row = [&](int j, const RowFrag& rf) __attribute__((always_inline)) {
            const int k = N - j;
            double ml = r2.mring[j % R2_D][9][l];
            with_shape<FX>(StageRef{io.st, k}, [&](const auto& sh) {
                using SHT = std::remove_reference_t<decltype(sh)>;
                bwd_row_update(io, sm, sh, k, SHT::fixed || k < N, rf.bop, rf.brow, P1, ml_prev, compute_Pb, Pb, ml);
            });
            const int sp = j % R2_DP;
            d4 S;
#pragma unroll
            for (int r = 0; r < 4; r++) S[r] = r2.pring[sp][r][l];
            const double invd = r2.pring[sp][4][l];
            const bool xfac = __builtin_amdgcn_readfirstlane(r2.xfac[sp]) != 0;
            XFac xf;
            if (xfac) {
#pragma unroll
                for (int r = 0; r < 4; r++) xf.L[r] = r2.pring[sp][5 + r][l];
                xf.invd = r2.pring[sp][9][l];
            }
            double kg = 0.0;
            with_shape<FX>(StageRef{io.st, k}, [&](const auto& sh) {
                using SHT = std::remove_reference_t<decltype(sh)>;
                stage_chol_row<true, SHT::fixed>(S, invd, ml, sh.nu, sh.nx, sh.xo, !SHT::fixed && k == 0, &kg);
                if (xfac) {  // the clamped x block's row half and p_eff = Lxx l_x (stage_chol xfac)
                    double lx = ml;
                    xblocks_chol_row(xf.L, xf.invd, lx, sh.nx, sh.xo);
                    pform_eff_row(xf.L, lx, sh.nx, sh.xo, ml);
                }
                double* Fk = io.F + (long)k * FSTRIDE;
                if constexpr (SHT::fixed)
                    store_factor_fixed<SHT::nx>(Fk, S, ml, invd, kg, true);
                else
                    store_factor(Fk, S, ml, invd, kg);
            });
            P1 = S;
            ml_prev = ml;
        };
        auto rfetch = [&](int j, RowFrag& f) __attribute__((always_inline)) {
            const int k = N - j;
            with_shape<FX>(StageRef{io.st, k}, [&](const auto& sh) { row_fetch(io, sh, k, update_b, bsrc, f); });
        };
        R2_T0(tp);
        BwdFrag fa, fb;
        RowFrag ra, rb;
        fetch(0, fa);
        if (1 <= N) fetch(1, fb);
        prep(0, fa);
        if (2 <= N) fetch(2, fa);
        if (1 <= N) prep(1, fb);
        if (3 <= N) fetch(3, fb);
        rfetch(0, ra);
        r2_bar();  // prologue
        // step j: the row half of step j - 1 (row fragment fetched at step j - 1), the row fragment of step j, then
        // prep(j + 2) from the fragment fetched at step j - 2 and fetch(j + 4) into it; a pair of steps swaps the roles
        for (int j = 0;;) {
            if (j >= 1) row(j - 1, rb);
            if (j + 1 <= N) rfetch(j + 1, rb);
            if (j + 2 <= N) prep(j + 2, fa);
            if (j + 4 <= N) fetch(j + 4, fa);
            R2_STEP_BAR(tp, 3);
            if (++j > N + 1) break;
            row(j - 1, ra);
            if (j + 1 <= N) rfetch(j + 1, ra);
            if (j + 2 <= N) prep(j + 2, fb);
            if (j + 4 <= N) fetch(j + 4, fb);
            R2_STEP_BAR(tp, 3);
            if (++j > N + 1) break;
        }
    }
}

// ------------------------------------------------------------------------------------------------
// Forward sweep in blocks of R2_H items (item k < N: stage k; item N: x_N): at block b wave 0 computes items
// [b H, b H + H) into forward slots k % 2H = [ux_k (col) | x_k (col, state tiles only)] while wave 1 stores / forms pi
// for block b - 1; one barrier per block.  A slot written at block b is read at block b + 1 and rewritten at b + 2.
// ------------------------------------------------------------------------------------------------
template <class FX>
__device__ __forceinline__ void ric_forward2(const RicIO& io, int w, int update_b, const double* bsrc, double* ux,
                                             int compute_pi, double* pi) {
    const int N = io.N, l = lane_id(), g = l >> 4, c = l & 15;
    const int nblk = (N + R2_H) / R2_H;  // blocks covering items 0 .. N
    if (w == 0) {
        Scratch* sm = &r2.sm[0];
        double xcol = 0.0;
        FwdFrag f0, f1, f2;
        fwd_fetch_chain_k<0, FX>(io, 0, bsrc, update_b, ux, compute_pi, f0);
        fwd_fetch_chain_k<0, FX>(io, 1 <= N ? 1 : N, bsrc, update_b, ux, compute_pi, f1);
        auto put = [&](int k, double u, double x) __attribute__((always_inline)) {
            const int s = k % (2 * R2_H);
            r2.fring[s][0][l] = u;
            r2.fring[s][1][l] = x;
        };
        auto stage = [&](int k, const FwdFrag& fa, FwdFrag& fc) __attribute__((always_inline)) {
            fwd_fetch_chain_k<0, FX>(io, k + 2 <= N ? k + 2 : N, bsrc, update_b, ux, compute_pi, fc);
            const double xk = xcol;
            double ucol = 0.0;
            with_shape<FX>(StageRef{io.st, k}, [&](const auto& sh) { fwd_chain<0>(sm, sh, k, fa, xcol, ucol); });
            put(k, ucol, xk);
        };
        R2_T0(tp);
        int k = 0, r = 0;  // next item; a stage's fragment is f[r] (three rotating roles)
        for (int b = 0; b <= nblk; b++) {
            const int kend = (b + 1) * R2_H < N + 1 ? (b + 1) * R2_H : N + 1;
            for (; k < kend; k++) {
                if (k == N) {
                    put(N, xcol, xcol);
                } else if (r == 0) {
                    stage(k, f0, f2);
                } else if (r == 1) {
                    stage(k, f1, f0);
                } else {
                    stage(k, f2, f1);
                }
                r = r == 2 ? 0 : r + 1;
            }
            R2_STEP_BAR(tp, 5);
        }
    } else {
        Scratch* sm = &r2.sm[1];
        // stage k's record: P_k (pi) and the row [l_u; p_k], in the format of stage k's shape class
        struct PiFrag {
            d4 S;
            double lc;
        };
        auto fetch = [&](int k, PiFrag& f) __attribute__((always_inline)) {
            const double* Fk = io.F + (long)k * FSTRIDE;
            with_shape<FX>(StageRef{io.st, k < N ? k : N - 1}, [&](const auto& sh) {
                using SHT = std::remove_reference_t<decltype(sh)>;
                if constexpr (SHT::fixed) {
                    f.S[0] = 0.0;
                    load_p_fixed<SHT::nx>(Fk, f.S, compute_pi && k > 0);
                    f.lc = gld(Fk, FXR_L + c);
                } else {
#pragma unroll
                    for (int r = 0; r < 4; r++) f.S[r] = gld(Fk, r * 64 + l, compute_pi && k > 0);
                    f.lc = gld(Fk, 256 + c);
                }
            });
        };
        auto work = [&](int k, const PiFrag& f) __attribute__((always_inline)) {
            const int s = k % (2 * R2_H);
            const double ucol = r2.fring[s][0][l], xk = r2.fring[s][1][l];
            const DynSh sk(StageRef{io.st, k});
            if (compute_pi && k > 0) {
                double xrow[4];
                col2row(sm, xk, xrow);
                fwd_pi<0>(sk.xo, sk.nx, k, f.S, xrow, f.lc, compute_pi, pi);
            }
            const int v = tile_var(c, sk.nu, sk.nx, sk.xo);
            gst(ux, k * V16 + v, k < N ? ucol : xk, g == 0 && v >= 0);
        };
        R2_T0(tp);
        PiFrag fa, fb;
        fetch(0, fa);
        int k = 0;
        bool alt = false;
        for (int b = 0; b <= nblk; b++) {
            const int kend = b * R2_H < N + 1 ? b * R2_H : N + 1;  // items of blocks 0 .. b - 1
            for (; k < kend; k++) {
                if (!alt) {
                    if (k + 1 <= N) fetch(k + 1, fb);
                    work(k, fa);
                } else {
                    if (k + 1 <= N) fetch(k + 1, fa);
                    work(k, fb);
                }
                alt = !alt;
            }
            R2_STEP_BAR(tp, 7);
        }
    }
}

__device__ __forceinline__ RicIO r2_io(const KArgs& a, const R2Tabs& T, int p) {
    RicIO io;
    io.N = a.N;
    io.st = T.st;
    io.tileslot = T.tileslot;
    io.BAbt = a.BAbt + (long)p * a.sB;
    io.RSQ = a.RSQ + (long)p * a.sR;
    io.BAbtS = a.BAbt;
    io.RSQS = a.RSQ;
    io.F = a.ws + (long)p * a.sW;
    io.DCt = a.DCt ? a.DCt + (long)p * a.sG : a.RSQ;
    return io;
}

}  // namespace

// two waves per SIMD (<= 256 VGPRs): four problems' workgroups per CU put 1024 problems on 256 CUs in one wave
template <class FX>
__global__ __launch_bounds__(128) __attribute__((amdgpu_waves_per_eu(2))) void hk_ric_sv2(KArgs a) {
    const R2Tabs T = r2_tables(a);
    const int p = blockIdx.x + a.p0;
    if (p >= a.nprob) return;
    const int w = threadIdx.x >> 6;
    const RicIO io = r2_io(a, T, p);
    const long o16 = (long)p * a.sV16;
    const double* b = a.vb ? a.vb + o16 : nullptr;
    const double* q = a.vq ? a.vq + o16 : nullptr;
    BoxCtx bc{};
    bc.Qx = a.vQx ? a.vQx + o16 : nullptr;
    bc.qx = a.vqx ? a.vqx + o16 : nullptr;
    double* Pb = a.vPb ? a.vPb + o16 : nullptr;
    if (a.use_box)
        ric_backward2<BX_GIVEN, FX>(io, w, a.update_b, b, a.update_q, q, bc, a.compute_Pb, Pb);
    else
        ric_backward2<BX_NONE, FX>(io, w, a.update_b, b, a.update_q, q, bc, a.compute_Pb, Pb);
    __syncthreads();  // the records stored by wave 1 are read by both waves below; the stage ring is re-used
    ric_forward2<FX>(io, w, a.update_b, b, a.ux + o16, a.compute_pi, a.pi + o16);
}

template <class FX>
static int launch2_t(const KArgs* a, int count, hipStream_t stream) {
#ifdef HK_STAMPS
    (void)hipMemcpyToSymbol(HIP_SYMBOL(r2_dbg), &a->dbg, sizeof(a->dbg));
#endif
    static const HkKernelLimits lim(reinterpret_cast<const void*>(&hk_ric_sv2<FX>));
    const size_t lds = r2_lds_bytes(a->N);
    if (lim.check(lds, 128) != 0) return HK_LAUNCH_REFUSED;
    hipLaunchKernelGGL(hk_ric_sv2<FX>, dim3(count), dim3(128), lds, stream, *a);
    return (int)hipGetLastError();
}

// which: 0 = d_back_ric_rec_sv_tv_res (the only entry point with a two-wave kernel).  HK_LAUNCH_REFUSED: the caller
// runs the one-wave kernel instead.
extern "C" int hk_launch_ric2(int which, const KArgs* a, int count, hipStream_t stream) {
    if (count <= 0) return 0;
    if (which != 0) return HK_LAUNCH_REFUSED;
    switch (a->fixcls) {
        case 1: return launch2_t<FixSh<4, 12>>(a, count, stream);
        case 2: return launch2_t<FixSh<3, 8>>(a, count, stream);
        default: return launch2_t<NoFix>(a, count, stream);
    }
}
