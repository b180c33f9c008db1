// hk_ric2.hip -- d_back_ric_rec_sv_tv_res over a batch with TWO waves per problem (gfx950).
//
// At the benchmark batches (1024 problems) the one-wave kernel (hpmpc_kernels.hip hk_ric_sv) leaves one wave per
// SIMD, and that wave is latency-bound: it parks on s_waitcnt for ~47 % of its cycles and issues one instruction per
// ~17 cycles (profiles/r04b_pmc_mix.json), because every stage interleaves the recursion's dependent chain with
// the work around it.  Here each problem gets a 128-thread workgroup and the work is split by dependency, as in the
// multi-wave lone-QP kernel (hk_mw.h) but with two roles and a small LDS footprint (four workgroups per CU):
//
//   backward sweep (lqcp_solvers/d_back_ric_rec.c:186-335)
//     wave 0 (tile): M += BAbt_k P_{k+1} BAbt_k' (MFMA), the clamp certificate (cert_ok) and the tile half of the
//                    u-block Cholesky -> P_k -- the only chain that carries the recursion forward;
//     wave 1 (row):  fetches stage k two stages ahead of wave 0 and hands it the ready tile (RSQ + box, bwd_pre) with
//                    the BAbt operand; then, one stage behind wave 0, the augmented row (P b, ml += BAbt (P b + p),
//                    the row half of the Cholesky, the gain block) and the stage record -- a second recursion
//                    (p_{k+1} -> p_k) that needs wave 0's factor but never feeds it (hk_mw.h, same routines).
//   forward sweep (:339-397)
//     wave 0: u_k = KG [rhs_u; x_k] and x_{k+1} = b_k + BAbt_k' ux_k (fwd_chain, the chain only);
//     wave 1: stores ux_k and forms pi_{k-1} = P_k x_k + p_k from stage k's record (fwd_pi).
// Every value is produced by the same routine on the same operands as in hk_ric_sv (hk_riccati.h), so results agree
// with it up to the compiler's FMA contraction (tests/test_gpu_ric2.py holds both to the goldens and the oracle).
//
// Hand-over: rings in LDS with ticketed flags (one lane stores the flag after the slot data; the LDS performs one
// wave's ds_ operations in issue order -- the hk_mw.h argument, including its HK_MW_FENCE option).  Slot reuse needs
// no "free" flags: the order of the other ring's flags implies it (comments at each ring).  A wait that does not end
// (a bug, never a data condition) sets r2.err after ~2^22 polls, every later wait falls through, and the problem's
// ux / pi are overwritten with NaN so that the failure is loud.
#include "hk_mw.h"
#include "hk_launch_guard.h"
#include "hpmpc_kargs.h"

using namespace hk;

namespace {

constexpr int R2_D = 3;      // wave 1 -> wave 0 stage slots (wave 1 runs two stages ahead)
constexpr int R2_ROWS = 10;  // M (4) | bop (4) | dq | ml
constexpr int R2_DP = 2;     // wave 0 -> wave 1 factor slots
constexpr int R2_PROWS = 10; // record tile (4) | inverse diagonal | a clamped stage's x factor (4) and inverse diagonal
constexpr int R2_FD = 8;     // forward slots: [ucol | xcol]
constexpr int R2_ERR_POLLS = 1 << 22;

struct R2Shared {
    union {
        double mring[R2_D][R2_ROWS][64];
        double fring[R2_FD][2][64];  // the forward sweep re-uses the backward's stage ring
    };
    double pring[R2_DP][R2_PROWS][64];
    Scratch sm[2];
    double mgc[R2_D];  // the stage's certificate bound g (wave-uniform)
    int mfull[R2_D], pfull[R2_DP], xfac[R2_DP], ffull[R2_FD];
    int fdone;  // forward stages wave 1 has read
    int rdone;  // backward steps whose row half wave 1 has finished (read at the last step only)
    int err;
};
static_assert(sizeof(double) * R2_FD * 2 * 64 <= sizeof(double) * R2_D * R2_ROWS * 64, "forward ring overlay");

// one object per workgroup, referred to by name (every access stays a ds_ op; hk_mw.h)
__shared__ R2Shared r2;

// Diagnostic build (-DHK_STAMPS, tools/ric_waves_probe.py --stamps): s_memtime segment totals of problem 0 into
// KArgs.dbg -- [0..3] wave 0's backward step by segment (hand-over in, tile update + certificate, Cholesky, hand-over
// out), [4] / [5] each wave's backward sweep, [6] / [7] each wave's forward sweep, [8] wave 1's waits for the factor,
// [9] wave 0's forward waits for free slots, [10] wave 1's forward waits.  Stamps wait for the wave's LDS operations.
#ifdef HK_STAMPS
__device__ unsigned long long* r2_dbg;
#define R2_CLK(v) const unsigned long long v = mw_clock()
#define R2_ADD(i, d)                                                         \
    do {                                                                     \
        if (r2_dbg && blockIdx.x == 0 && lane_id() == 0) r2_dbg[i] += (d); \
    } while (0)
#else
#define R2_CLK(v) \
    do {          \
    } while (0)
#define R2_ADD(i, d) \
    do {             \
    } while (0)
#endif

__device__ __forceinline__ int r2_flag(const int* f) { return __atomic_load_n(f, __ATOMIC_RELAXED); }

__device__ __forceinline__ void r2_wait(const int* f, int v) {
    int n = 0;
    while (r2_flag(f) < v) {
        if (++n > 64) __builtin_amdgcn_s_sleep(1);
        if (n > R2_ERR_POLLS) __atomic_store_n(&r2.err, 1, __ATOMIC_RELAXED);
        if (r2_flag(&r2.err)) break;
    }
    mw_acquire_fence();
}

__device__ __forceinline__ void r2_post(int* f, int v) {
    mw_release_fence();
    if (lane_id() == 0) __atomic_store_n(f, v, __ATOMIC_RELAXED);
    asm volatile("" ::: "memory");
}

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
    if (t < R2_D) r2.mfull[t] = 0;
    if (t < R2_DP) r2.pfull[t] = 0;
    if (t < R2_FD) r2.ffull[t] = 0;
    if (t == 0) {
        r2.fdone = 0;
        r2.rdone = 0;
        r2.err = 0;
    }
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
// Backward sweep.  Step j is stage k = N - j.
// ------------------------------------------------------------------------------------------------
template <int BM, class FX>
__device__ __forceinline__ void ric_backward2(const RicIO& io, int w, int update_b, const double* bsrc, int update_q,
                                              const double* qsrc, const BoxCtx& bc, int compute_Pb, double* Pb) {
    const int N = io.N, l = lane_id();
    if (w == 0) {
        // The tile recursion.  Stage slot j + 1 is read at the start of step j (one step ahead), so its LDS latency is
        // off the chain.  Factor slot j % R2_DP is free when written at step j: its previous occupant (step j - 2) was
        // read by wave 1's row half of step j - 2, which precedes (program order) wave 1's post of stage slot j + 1
        // (its step j - 1), and this wave waited for that post (take) at the start of step j.  The last step has no
        // take: it waits for the row half of step N - 2 explicitly.
        d4 P = {0.0, 0.0, 0.0, 0.0};  // record tile of stage k+1 (its x block is P_{k+1})
        d4 Mn, bopn;
        double dqn, gcn;
        auto take = [&](int j) __attribute__((always_inline)) {
            const int s = j % R2_D;
            r2_wait(&r2.mfull[s], j + 1);
#pragma unroll
            for (int r = 0; r < 4; r++) {
                Mn[r] = r2.mring[s][r][l];
                bopn[r] = r2.mring[s][4 + r][l];
            }
            dqn = r2.mring[s][8][l];
            gcn = r2.mgc[s];
        };
        R2_CLK(tb0);
        take(0);
        for (int j = 0; j <= N; j++) {
            const int k = N - j;
            d4 M = Mn;
            const d4 bop = bopn;
            const double dq = dqn, gc = gcn;
            R2_CLK(ta);
            if (j < N) take(j + 1);
            else if (N >= 2) r2_wait(&r2.rdone, N - 1);
            R2_CLK(tt);
            R2_ADD(0, tt - ta);
            double invd;
            bool xfac = false;
            XFac xf;
            with_shape<FX>(StageRef{io.st, k}, [&](const auto& sh) {
                using SHT = std::remove_reference_t<decltype(sh)>;
                bwd_tile_update(sh, SHT::fixed || k < N, bop, P, M);
                double mld = 0.0;
                const bool full = !SHT::fixed && k == 0;
                xfac = !full && !cert_ok(M, dq, gc);
                R2_CLK(tc);
                R2_ADD(1, tc - tt);
                stage_chol<false, false>(M, mld, invd, sh.nu, sh.nx, sh.xo, full, !SHT::fixed, nullptr, k, xfac, &xf);
                R2_CLK(td);
                R2_ADD(2, td - tc);
            });
            R2_CLK(te);
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
            r2_post(&r2.pfull[s], j + 1);
            R2_CLK(tf);
            R2_ADD(3, tf - te);
        }
        R2_CLK(tb1);
        R2_ADD(4, tb1 - tb0);
    } else {
        // Wave 1: at step j it prepares stage j + 2 for wave 0 (fragments fetched two steps ahead), then runs the row
        // half and the record of stage j.  Stage slot (j + 2) % R2_D last held step j - 1: wave 1 itself read its
        // row data at step j - 1, and wave 0 read the rest one step before posting factor slot j - 1, which wave 1's
        // step j - 1 waited for.
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
            const int s = j % R2_D;
#pragma unroll
            for (int r = 0; r < 4; r++) {
                r2.mring[s][r][l] = M[r];
                r2.mring[s][4 + r][l] = f.bop[r];
            }
            r2.mring[s][8][l] = dq;
            r2.mring[s][9][l] = ml;
            if (l == 0) r2.mgc[s] = gc;
            r2_post(&r2.mfull[s], j + 1);
        };
        d4 P1 = {0.0, 0.0, 0.0, 0.0};  // record tile of stage k+1
        double ml_prev = 0.0;           // its row [l_u; p_{k+1}]
        auto row = [&](int j, const RowFrag& rf) __attribute__((always_inline)) {
            const int k = N - j;
            const int s = j % R2_D;
            double ml = r2.mring[s][9][l];
            with_shape<FX>(StageRef{io.st, k}, [&](const auto& sh) {
                using SHT = std::remove_reference_t<decltype(sh)>;
                bwd_row_update(io, sm, sh, k, SHT::fixed || k < N, rf.bop, rf.brow, P1, ml_prev, compute_Pb, Pb, ml);
            });
            const int sp = j % R2_DP;
            R2_CLK(tw0);
            r2_wait(&r2.pfull[sp], j + 1);
            R2_CLK(tw1);
            R2_ADD(8, tw1 - tw0);
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
            r2_post(&r2.rdone, j + 1);
        };
        auto rfetch = [&](int j, RowFrag& f) __attribute__((always_inline)) {
            const int k = N - j;
            with_shape<FX>(StageRef{io.st, k}, [&](const auto& sh) { row_fetch(io, sh, k, update_b, bsrc, f); });
        };
        R2_CLK(tb0);
        BwdFrag fa, fb;
        RowFrag ra, rb;
        fetch(0, fa);
        if (1 <= N) fetch(1, fb);
        rfetch(0, ra);
        prep(0, fa);
        if (2 <= N) fetch(2, fa);
        if (1 <= N) prep(1, fb);
        if (3 <= N) fetch(3, fb);
        // step j: prep(j + 2) from the fragment fetched at step j - 2, then fetch(j + 4) into it; the row fragment of
        // step j + 1 is issued before the row half of step j
        for (int j = 0;;) {
            if (j + 2 <= N) prep(j + 2, fa);
            if (j + 4 <= N) fetch(j + 4, fa);
            if (j + 1 <= N) rfetch(j + 1, rb);
            row(j, ra);
            if (++j > N) break;
            if (j + 2 <= N) prep(j + 2, fb);
            if (j + 4 <= N) fetch(j + 4, fb);
            if (j + 1 <= N) rfetch(j + 1, ra);
            row(j, rb);
            if (++j > N) break;
        }
        R2_CLK(tb1);
        R2_ADD(5, tb1 - tb0);
    }
}

// ------------------------------------------------------------------------------------------------
// Forward sweep: wave 0 -> wave 1 slot k % R2_FD = [ux_k (col) | x_k (col, state tiles only)].  Wave 1 posts fdone
// every R2_FD / 2 stages; wave 0 checks it once per R2_FD / 2 stages: slots k .. k + R2_FD/2 - 1 are free once
// stage k + R2_FD/2 - 1 - R2_FD has been read, i.e. fdone >= k + R2_FD/2 - R2_FD.
// ------------------------------------------------------------------------------------------------
template <class FX>
__device__ __forceinline__ void ric_forward2(const RicIO& io, int w, int update_b, const double* bsrc, double* ux,
                                             int compute_pi, double* pi) {
    const int N = io.N, l = lane_id(), g = l >> 4, c = l & 15;
    constexpr int H = R2_FD / 2;
    if (w == 0) {
        Scratch* sm = &r2.sm[0];
        double xcol = 0.0;
        FwdFrag f0, f1, f2;
        fwd_fetch_chain_k<0, FX>(io, 0, bsrc, update_b, ux, compute_pi, f0);
        fwd_fetch_chain_k<0, FX>(io, 1 <= N ? 1 : N, bsrc, update_b, ux, compute_pi, f1);
        R2_CLK(tf0);
        auto put = [&](int k, double u, double x) __attribute__((always_inline)) {
            if (k >= R2_FD && k % H == 0) {
                R2_CLK(tw0);
                r2_wait(&r2.fdone, k + H - R2_FD);
                R2_CLK(tw1);
                R2_ADD(9, tw1 - tw0);
            }
            const int s = k % R2_FD;
            r2.fring[s][0][l] = u;
            r2.fring[s][1][l] = x;
            r2_post(&r2.ffull[s], k + 1);
        };
        auto stage = [&](int k, const FwdFrag& fa, FwdFrag& fc) __attribute__((always_inline)) {
            fwd_fetch_chain_k<0, FX>(io, k + 2 <= N ? k + 2 : N, bsrc, update_b, ux, compute_pi, fc);
            const double xk = xcol;
            double ucol = 0.0;
            with_shape<FX>(StageRef{io.st, k}, [&](const auto& sh) { fwd_chain<0>(sm, sh, k, fa, xcol, ucol); });
            put(k, ucol, xk);
        };
        for (int k = 0;;) {
            if (k >= N) break;
            stage(k, f0, f2);
            if (++k >= N) break;
            stage(k, f1, f0);
            if (++k >= N) break;
            stage(k, f2, f1);
            ++k;
        }
        put(N, xcol, xcol);
        R2_CLK(tf1);
        R2_ADD(6, tf1 - tf0);
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
        R2_CLK(tf0);
        auto work = [&](int k, const PiFrag& f) __attribute__((always_inline)) {
            const int s = k % R2_FD;
            R2_CLK(tw0);
            r2_wait(&r2.ffull[s], k + 1);
            R2_CLK(tw1);
            R2_ADD(10, tw1 - tw0);
            const double ucol = r2.fring[s][0][l], xk = r2.fring[s][1][l];
            if (k % H == H - 1 || k == N) r2_post(&r2.fdone, k + 1);
            const DynSh sk(StageRef{io.st, k});
            if (compute_pi && k > 0) {
                double xrow[4];
                col2row(sm, xk, xrow);
                fwd_pi<0>(sk.xo, sk.nx, k, f.S, xrow, f.lc, compute_pi, pi);
            }
            const int v = tile_var(c, sk.nu, sk.nx, sk.xo);
            gst(ux, k * V16 + v, k < N ? ucol : xk, g == 0 && v >= 0);
        };
        PiFrag fa, fb;
        fetch(0, fa);
        for (int k = 0;;) {
            if (k + 1 <= N) fetch(k + 1, fb);
            work(k, fa);
            if (++k > N) break;
            if (k + 1 <= N) fetch(k + 1, fa);
            work(k, fb);
            if (++k > N) break;
        }
        R2_CLK(tf1);
        R2_ADD(7, tf1 - tf0);
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
    __syncthreads();  // the records stored by wave 1 are read by both waves below; the ring is re-used
    ric_forward2<FX>(io, w, a.update_b, b, a.ux + o16, a.compute_pi, a.pi + o16);
    __syncthreads();
    if (r2_flag(&r2.err)) {  // an expired hand-over wait (a bug): make the problem's outputs NaN
        const double nan = __builtin_nan("");
        for (int i = threadIdx.x; i < (a.N + 1) * V16; i += 128) {
            a.ux[o16 + i] = nan;
            a.pi[o16 + i] = nan;
        }
    }
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
