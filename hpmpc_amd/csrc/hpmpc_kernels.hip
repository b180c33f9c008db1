// hpmpc_kernels.hip -- MI355X (gfx950) kernels for HPMPC's Riccati / interior-point hot path.
//
// Execution model: one wavefront (64-thread workgroup) owns one QP instance for the whole call; a
// launch covers a batch (grid = number of problems).  Stage data are read straight from HBM in the
// reference's lib4 layout; the recursion state (the previous stage's factor) stays in registers.
// All IPM control flow (iteration count, step length, mu) is per wave, so problems that converge
// early simply retire their wave.
#include "hk_ipm_body.h"
#include "hk_mw.h"
#include <cstdlib>

// ------------------------------------------------------------------------------------------------
// d_back_ric_rec_sv_tv_res / _trf_ / _trs_ over a batch (one problem per workgroup)
// ------------------------------------------------------------------------------------------------
template <class FX>
__global__ __launch_bounds__(64) void hk_ric_sv(KArgs a) {
    const LdsTabs T = lds_tables(a);
    Scratch& sm = *T.sm;
    const int p = blockIdx.x + a.p0;
    if (p >= a.nprob) return;
    double* F = a.ws + (long)p * a.sW;
    RicIO io = make_io(a, T, p, F);
    const long o16 = (long)p * a.sV16;
    const double* b = a.vb ? a.vb + o16 : nullptr;
    const double* q = a.vq ? a.vq + o16 : nullptr;
    BoxCtx bc{};
    bc.Qx = a.vQx ? a.vQx + o16 : nullptr;
    bc.qx = a.vqx ? a.vqx + o16 : nullptr;
    double* Pb = a.vPb ? a.vPb + o16 : nullptr;
#ifdef HK_STAMPS  // diagnostic build: the two sweeps of problem 0 (cycles), a.dbg[60] backward, [61] forward
    const unsigned long long t0 = mw_clock();
#endif
    if (a.use_box)
        ric_backward<true, BX_GIVEN, FX, CERT_LOAD>(io, &sm, a.update_b, b, a.update_q, q, bc, a.compute_Pb, Pb);
    else
        ric_backward<true, BX_NONE, FX, CERT_LOAD>(io, &sm, a.update_b, b, a.update_q, q, bc, a.compute_Pb, Pb);
    wsync();
#ifdef HK_STAMPS
    const unsigned long long t1 = mw_clock();
#endif
    ric_forward_sv<FX>(io, &sm, a.update_b, b, a.ux + o16, a.compute_pi, a.pi + o16);
#ifdef HK_STAMPS
    const unsigned long long t2 = mw_clock();
    if (a.dbg && p == 0 && lane_id() == 0) {
        a.dbg[60] = t1 - t0;
        a.dbg[61] = t2 - t1;
    }
#endif
}

template <class FX>
__global__ __launch_bounds__(64) void hk_ric_trf(KArgs a) {
    const LdsTabs T = lds_tables(a);
    Scratch& sm = *T.sm;
    const int p = blockIdx.x + a.p0;
    if (p >= a.nprob) return;
    double* F = a.ws + (long)p * a.sW;
    RicIO io = make_io(a, T, p, F);
    const long o16 = (long)p * a.sV16;
    BoxCtx bc{};
    bc.Qx = a.vQx ? a.vQx + o16 : nullptr;
    if (a.use_box)
        ric_backward<false, BX_GIVEN, FX, CERT_LOAD>(io, &sm, 0, nullptr, 0, nullptr, bc, 0, nullptr);
    else
        ric_backward<false, BX_NONE, FX, CERT_LOAD>(io, &sm, 0, nullptr, 0, nullptr, bc, 0, nullptr);
}

template <class FX>
__global__ __launch_bounds__(64) void hk_ric_trs(KArgs a) {
    const LdsTabs T = lds_tables(a);
    Scratch& sm = *T.sm;
    const int p = blockIdx.x + a.p0;
    if (p >= a.nprob) return;
    double* F = a.ws + (long)p * a.sW;
    RicIO io = make_io(a, T, p, F);
    const long o16 = (long)p * a.sV16;
    BoxCtx bc{};
    bc.qx = a.vqx ? a.vqx + o16 : nullptr;
    double al = 1.0;
    if (a.use_box)
        ric_trs<BX_GIVEN, BX_NONE, FX>(io, &sm, a.vb + o16, a.vq + o16, bc, a.ux + o16, a.compute_pi, a.pi + o16,
                                   a.compute_Pb, a.vPb + o16, al);
    else
        ric_trs<BX_NONE, BX_NONE, FX>(io, &sm, a.vb + o16, a.vq + o16, bc, a.ux + o16, a.compute_pi, a.pi + o16,
                                  a.compute_Pb, a.vPb + o16, al);
}

template <class FX>
__global__ __launch_bounds__(64) void hk_res(KArgs a) {
    const LdsTabs T = lds_tables(a);
    const int p = blockIdx.x + a.p0;
    if (p >= a.nprob) return;
    RicIO io = make_io(a, T, p, nullptr);
    const long o16 = (long)p * a.sV16, o32 = (long)p * a.sV32;
    double* out = a.ws + (long)p * a.sW;  // [rq | rb] V16, [rd | rm] V32
    const long n1 = a.N + 1;
    BoxCtx bc{};
    bc.d = a.d + o32;
    bc.lam = a.lam + o32;
    bc.t = a.t + o32;
    ResIO ro{};
    ro.bsrc = a.vb ? a.vb + o16 : nullptr;
    ro.qsrc = a.vq ? a.vq + o16 : nullptr;
    ro.ux = a.ux + o16;
    ro.pi = a.pi + o16;
    ro.rq = out;
    ro.rb = out + n1 * V16;
    ro.rd = out + 2 * n1 * V16;
    ro.rm = out + 2 * n1 * V16 + n1 * V32;
    double mu = 0.0;
    const bool have = residual_pass<false, FX>(io, bc, ro, mu);
    if (a.res_plain) {
        // d_res_mpc_hard_tv (mpc_solvers/d_res_ip_hard.c:38-330): the same r_q, r_b and lower r_d; its
        // upper r_d is (x - ub + t_up), the negation of the residual IPM's, and mu is 0 without constraints
        wsync();
        HK_FOR_BOX(io, k, { ro.rd[up] = -ro.rd[up]; });
        HK_FOR_GEN(io, k, { ro.rd[up] = -ro.rd[up]; });
        if (lane_id() == 0) a.mu_out[p] = have ? mu : 0.0;
        return;
    }
    if (lane_id() == 0 && have) a.mu_out[p] = mu;
}

// ------------------------------------------------------------------------------------------------
// IPM (d_ip2_res_mpc_hard_tv), persistent per problem.
// ------------------------------------------------------------------------------------------------
template <class FX>
__global__ __launch_bounds__(64) HK_TWO_WAVES void hk_ipm_init(KArgs a) {
    const LdsTabs T = lds_tables(a);
    if (a.nq) {  // every slot takes its first entry; the iterating ones form the first active list
        if (ipm_refill<FX, 7, true>(a, T, blockIdx.x)) qlist_push(a, a.qpar, blockIdx.x);
        return;
    }
    Who who;
    if (!who_am_i(a, who)) return;
    IpmView v = ipm_view(a, T, who);
    ipm_start<FX, 7, true>(a, T, v);
}


template <class FX>
__global__ __launch_bounds__(64) HK_TWO_WAVES void hk_ipm_fact(KArgs a) {
    // queue: empty the list this iteration's update pass fills (nothing reads it before then)
    if (a.nq && blockIdx.x == 0 && lane_id() == 0) *qcount(a, a.qpar ^ 1) = 0;
    Who who;
    if (!who_am_i(a, who) || !slot_active(a, who)) return;  // idle slots leave before staging the tables
    const LdsTabs T = lds_tables(a);
    IpmView v = ipm_view(a, T, who);
    if (v.w.state[S_ACTIVE] == 0.0) return;
    fact_body<FX>(a, T, v);
}

template <class FX>
__global__ __launch_bounds__(64) HK_TWO_WAVES void hk_ipm_pred(KArgs a) {
    Who who;
    if (!who_am_i(a, who) || !slot_active(a, who)) return;  // idle slots leave before staging the tables
    const LdsTabs T = lds_tables(a);
    IpmView v = ipm_view(a, T, who);
    if (v.w.state[S_ACTIVE] == 0.0) return;
    pred_body<FX>(a, T, v);
}

template <class FX>
__global__ __launch_bounds__(64) HK_TWO_WAVES void hk_ipm_corr(KArgs a) {
    Who who;
    if (!who_am_i(a, who) || !slot_active(a, who)) return;  // idle slots leave before staging the tables
    const LdsTabs T = lds_tables(a);
    IpmView v = ipm_view(a, T, who);
    if (v.w.state[S_ACTIVE] == 0.0) return;
    corr_body<FX>(a, T, v);
}

// The queue's second launch of a tick: the predictor and the corrector of one problem back to back (one launch
// boundary, one launch tail and one set of workgroup prologues fewer per tick than two pass kernels; the corrector's
// trs backward starts on the stages the predictor's forward ended on).  Each body gets a fresh view (the slot, entry
// and problem made opaque in between), so each keeps the register allocation it has in its own pass kernel.
template <class FX>
__global__ __launch_bounds__(64) HK_TWO_WAVES void hk_ipm_predcorr(KArgs a) {
    Who who;
    if (!who_am_i(a, who) || !slot_active(a, who)) return;  // idle slots leave before staging the tables
    const LdsTabs T = lds_tables(a);
    {
        IpmView v = ipm_view(a, T, who);
        if (v.w.state[S_ACTIVE] == 0.0) return;
        pred_body<FX>(a, T, v);
    }
    wsync();
    int s = who.s, q = who.q, d = who.d;
    asm volatile("" : "+v"(s), "+v"(q), "+v"(d));
    const Who w2{__builtin_amdgcn_readfirstlane(s), __builtin_amdgcn_readfirstlane(q), __builtin_amdgcn_readfirstlane(d)};
    IpmView v = ipm_view(a, T, w2);
    corr_body<FX>(a, T, v);
}

// The update pass loads 4 quads (16 stages) before using any (6 measured slower: profiles/r04/ab_headline_OP.txt)
template <class FX>
__global__ __launch_bounds__(64) HK_TWO_WAVES void hk_ipm_update(KArgs a) {
    Who who;
    if (!who_am_i(a, who) || !slot_active(a, who)) return;  // idle slots leave before staging the tables
    const LdsTabs T = lds_tables(a);
    IpmView v = ipm_view(a, T, who);
    if (v.w.state[S_ACTIVE] == 0.0) return;
    bool again = update_body<FX, 4>(a, v);
    if (!again && a.nq) {
        if (v.l == 0) atomicAdd(&a.qctl[1], 1);
        again = ipm_refill<FX, 4, false>(a, T, who.s);  // queue mode: the slot takes the next entry
    }
    if (a.nq && again) qlist_push(a, a.qpar ^ 1, who.s);
}

// One problem per workgroup, every iteration in ONE launch after hk_ipm_init (configs[1]: a lone QP): the same
// workgroup runs each iteration's four passes back to back on one CU, so no launch or host poll separates them and
// the problem's ~1 MB of stage data and factor records stay in that XCD's L2.
template <class FX>
__global__ __launch_bounds__(64) void hk_ipm_solo(KArgs a) {
    const LdsTabs T = lds_tables(a);
    const int p = blockIdx.x + a.p0;
    if (p >= a.nprob) return;
    // init is its own launch (hk_ipm_init, right before this one): inlined here it pushed the kernel into scratch
    // spills (852 B per lane) on top of the four iteration bodies
    if (carve(a.ws + (long)p * a.sW, a.N).state[S_ACTIVE] == 0.0) return;
    // every body gets a fresh view (its pointers are re-derived from the kernel arguments), so no register of one
    // pass is live across the next: each body keeps the allocation it has in its own pass kernel
    // (the problem index is made opaque before each view, so that nothing derived from it is hoisted out of the
    // loop and kept live across the bodies)
    auto view = [&]() __attribute__((always_inline)) {
        int q = p;
        asm volatile("" : "+v"(q));
        q = __builtin_amdgcn_readfirstlane(q);
        const Who w{q, q, q};
        return ipm_view(a, T, w);
    };
    for (int it = 0; it < a.k_max; it++) {  // ipm_continue ends the loop; k_max bounds it regardless
        wsync();
        {
            IpmView v = view();
            fact_body<FX>(a, T, v);
        }
        wsync();
        {
            IpmView v = view();
            pred_body<FX>(a, T, v);
        }
        wsync();
        {
            IpmView v = view();
            corr_body<FX>(a, T, v);
        }
        wsync();
        IpmView v = view();
        if (!update_body<FX, 4>(a, v)) break;
    }
}

// ------------------------------------------------------------------------------------------------
// The same solve with one problem per 256-thread workgroup (hk_mw.h): wave 0 runs each sweep's recursion, waves
// 1..3 everything off it, and the element-wise update is split over the four waves.  Every body keeps the
// single-wave body's arithmetic (same routines, same operands, mu summed in the same order), so the iterates are
// bitwise hk_ipm_solo's when both are built with -ffp-contract=on; under the build's default contraction hipcc fuses
// a few a * b + c differently once the bodies are split over waves and the two agree to rounding (hk_mw.h).  All four
// waves run every body, so that they meet the same barriers in the same order;
// the loop-control state is read by all and written by thread 0 (IpmView.l = threadIdx.x here).
// ------------------------------------------------------------------------------------------------
namespace {

template <class FX>
__device__ __forceinline__ void fact_body_mw(const KArgs& a, IpmView& v, int& tb, int w) {
    const double* st = v.w.state;
    const bool sn = a.single_newton != 0;
    v.bc.cert_new = st[S_KK] == 0.0;  // the helpers form the certificate bounds in the solve's first factorisation
    if (st[S_PHASE] == 1.0)
        tb = ric_backward_mw<true, BX_P1, FX>(v.io, tb, w, 0, nullptr, 0, nullptr, v.bc, 1, v.w.Pb);
    else {
        v.bc.res_rhs = !sn;
        v.bc.no_tinv = a.no_bkp;
        tb = ric_backward_mw<true, BX_P2R, FX>(v.io, tb, w, 0, nullptr, 0, nullptr, v.bc, 1, v.w.Pb);
    }
}

template <class FX>
__device__ __forceinline__ void pred_body_mw(const KArgs& a, IpmView& v, int& tb, int w) {
    double* st = v.w.state;
    const bool sn = a.single_newton != 0;
    const int phase = (int)st[S_PHASE], kk = (int)st[S_KK];
    const double mu = st[S_MU];
    double sigma = st[S_SIGMA];
    double al = 1.0;
    if (phase == 1) {
        v.bc.pred = 1;
        tb = ric_forward_mw<0, BX_P1, FX, true>(v.io, tb, w, nullptr, 0, v.w.dux, 0, v.w.dpi, v.bc, al);
    } else {
        tb = ric_forward_mw<0, BX_P2, FX, true>(v.io, tb, w, v.w.res_b, !sn, v.w.dux, 0, v.w.dpi, v.bc, al);
    }
    // al is the workgroup minimum in every wave, and the helpers' dt / dlam stores are visible (the sweep ends with
    // a barrier): every wave forms the same mu_aff and sigma
    const double alpha = al * 0.995;
    double mu_aff;
    {  // callees that may stay out of line get their own copies, so that the view itself never escapes to memory
        const RicIO io = v.io;
        const BoxCtx bc = v.bc;
        mu_aff = mu_aff_pass<7>(io, bc, alpha, st[S_MUSCAL]);
    }
    double smu = a.mu0;
    if (!sn) {
        sigma = mu_aff / mu;
        sigma = sigma * sigma * sigma;
        smu = sigma * mu;
    }
    __syncthreads();  // every wave has read the state before thread 0 rewrites it
    if (v.l == 0) {
        v.stat[5 * kk] = st[S_SIGMA];
        v.stat[5 * kk + 1] = al;
        v.stat[5 * kk + 2] = mu_aff;
        st[S_SIGMA] = sigma;
        st[S_SMU] = smu;
    }
}

template <class FX>
__device__ __forceinline__ void corr_body_mw(const KArgs& a, IpmView& v, int& tb, int w) {
    double* st = v.w.state;
    const int phase = (int)st[S_PHASE], kk = (int)st[S_KK];
    v.bc.smu = st[S_SMU];
    double al = 1.0;
    if (phase == 1)
        tb = ric_trs_mw<BX_P1, BX_P1, FX>(v.io, tb, w, nullptr, nullptr, v.bc, v.w.dux, a.compute_mult, v.w.dpi,
                                     v.w.Pb, al);
    else
        tb = ric_trs_mw<BX_P2, BX_P2, FX>(v.io, tb, w, v.w.res_b, v.w.res_q, v.bc, v.w.dux, a.compute_mult, v.w.dpi,
                                     v.w.Pb, al);
    if (v.l == 0) {
        v.stat[5 * kk] = st[S_SIGMA];
        v.stat[5 * kk + 3] = al;
        st[S_ALPHA] = al * 0.995;
    }
}

template <class FX, int CI>
__device__ __forceinline__ bool update_body_mw(const KArgs& a, const IpmView& v0, const MwSplit& mws0) {
    IpmView v = v0;  // a copy: the out-of-line passes below take it by reference
    const MwSplit mws = mws0;
    double* st = v.w.state;
    const int phase = (int)st[S_PHASE];
    int kk = (int)st[S_KK];
    const double alpha = st[S_ALPHA];
    const double sigma = st[S_SIGMA];
    double mu;
    if (phase == 1) {
        mu = update_p1_pass<CI, MW_WAVES>(v.io, v.bc, alpha, st[S_MUSCAL], v.ux, v.pi, v.w.dux, v.w.dpi, v.w.ux_bkp,
                                          v.w.pi_bkp, v.w.lam_bkp, v.w.t_bkp, mws);
    } else {
        if (a.no_bkp)
            mu = update_p2_pass<CI, true, false, MW_WAVES>(v.io, v.bc, v.bt.slotvar, alpha, st[S_MUSCAL], v.ux, v.pi,
                                                           v.w.dux, v.w.dpi, v.w.ux_bkp, v.w.pi_bkp, v.w.lam_bkp,
                                                           v.w.t_bkp, v.w.res_d, v.w.res_m, mws);
        else
            mu = update_p2_pass<CI, true, true, MW_WAVES>(v.io, v.bc, v.bt.slotvar, alpha, st[S_MUSCAL], v.ux, v.pi,
                                                          v.w.dux, v.w.dpi, v.w.ux_bkp, v.w.pi_bkp, v.w.lam_bkp,
                                                          v.w.t_bkp, v.w.res_d, v.w.res_m, mws);
    }
    wsync();
    if (v.l == 0) v.stat[5 * kk + 4] = mu;
    kk++;
    return ipm_continue<FX, CI, MW_WAVES>(a, v, kk, mu, alpha, sigma, phase, mws);
}

// LDS of the multi-wave kernel: the stage tables (lds_tables, dynamic) beside the static hk_mw object
__host__ __device__ constexpr size_t mw_lds_bytes(int N) {
    return sizeof(Scratch) + (size_t)(N + 1) * (sizeof(StageInfo) + 40);
}

}  // namespace

// The multi-wave solve of one problem (its workspace, iterate and data: who), from the loop-control state its
// workspace holds (a fresh start after hk_ipm_init, or a queue slot's problem in the middle of its iterations) to
// its end.  Every thread of the 256-thread workgroup calls it.
template <class FX>
__device__ __forceinline__ void mw_solve(const KArgs& a, const LdsTabs& T, const Who& who) {
    const int p = who.q;
    const int w = threadIdx.x >> 6;
    if (threadIdx.x < MW_D) {
        hk_mw.full[threadIdx.x] = 0;
        hk_mw.freed[threadIdx.x] = 0;
        hk_mw.freedB[threadIdx.x] = 0;
    }
    if (threadIdx.x < MW_DP) {
        hk_mw.fullP[threadIdx.x] = 0;
        hk_mw.freedP[threadIdx.x] = 0;
    }
    if (threadIdx.x == 0) hk_mw.err = 0;
    __syncthreads();
    int tb = 0;
    const MwSplit mws{w, (lds_f64*)&hk_mw.red[0][0]};
#ifdef HK_STAMPS
    // diagnostic build: cycles per body (summed over the iterations) and per wave in hand-over waits, problem 0
    unsigned long long tph[4] = {0, 0, 0, 0}, tm = 0;
    if (threadIdx.x < MW_WAVES) hk_mw.wait_cyc[threadIdx.x] = hk_mw.seg[threadIdx.x] = 0;
#define HK_MW_PHASE(i)                            \
    do {                                          \
        const unsigned long long t_ = mw_clock(); \
        if (i >= 0) tph[(i) & 3] += t_ - tm;      \
        tm = t_;                                  \
    } while (0)
#else
#define HK_MW_PHASE(i) \
    do {               \
    } while (0)
#endif
    for (int it = 0; it < a.k_max; it++) {
        __syncthreads();
        HK_MW_PHASE(-1);
        {
            IpmView v = ipm_view(a, T, who);
            v.l = threadIdx.x;  // thread 0 alone writes the control state and the statistics
            fact_body_mw<FX>(a, v, tb, w);
        }
        __syncthreads();
        HK_MW_PHASE(0);
        {
            IpmView v = ipm_view(a, T, who);
            v.l = threadIdx.x;
            pred_body_mw<FX>(a, v, tb, w);
        }
        __syncthreads();
        HK_MW_PHASE(1);
        {
            IpmView v = ipm_view(a, T, who);
            v.l = threadIdx.x;
            corr_body_mw<FX>(a, v, tb, w);
        }
        __syncthreads();
        HK_MW_PHASE(2);
        IpmView v = ipm_view(a, T, who);
        v.l = threadIdx.x;
        const bool again = update_body_mw<FX, 4>(a, v, mws);
        __syncthreads();
        HK_MW_PHASE(3);
        // an expired hand-over wait (a bug, never a data condition) ends the solve with HK_MW_ERR
        if (!again || __atomic_load_n(&hk_mw.err, __ATOMIC_RELAXED)) break;
    }
#ifdef HK_STAMPS
    if (a.dbg && p == 0 && threadIdx.x == 0) {
        for (int i = 0; i < 4; i++) a.dbg[32 + i] = tph[i];
        for (int i = 0; i < MW_WAVES; i++) a.dbg[40 + i] = hk_mw.wait_cyc[i];
        for (int i = 0; i < 4; i++) a.dbg[48 + i] = hk_mw.seg[i];
    }
#endif
#undef HK_MW_PHASE
    if (threadIdx.x == 0 && hk_mw.err) {
        a.ret[p] = HK_MW_ERR;
        for (int i = 0; i < 4; i++) a.stat[(long)p * 5 * a.k_max + i] = hk_mw.dbg[i];
    }
}

template <class FX>
__global__ __launch_bounds__(256) void hk_ipm_solo_mw(KArgs a) {
    const LdsTabs T = lds_tables(a);
    const int p = blockIdx.x + a.p0;
    if (p >= a.nprob) return;
    if (carve(a.ws + (long)p * a.sW, a.N).state[S_ACTIVE] == 0.0) return;
    mw_solve<FX>(a, T, Who{p, p, p});
}

// Queue drain (hpmpc_mi355x_ipm_queue): once every entry has been handed out and few slots still iterate, the host
// stops the four-launch ticks and finishes the survivors here, one problem per four-wave workgroup (workgroup i takes
// the i-th slot of active list qpar, the list the next tick would run).  In the drain the problems that stop on
// alpha_min or k_max run alone on the chip, one wavefront each, bound by the latency of their own chain: the
// multi-wave solve (hk_mw.h) gives each of them a CU.  Same routines on the same operands as the single-wave bodies
// (results to rounding, hk_mw.h).
template <class FX>
__global__ __launch_bounds__(256) void hk_ipm_qdrain_mw(KArgs a) {
    const LdsTabs T = lds_tables(a);
    const int n = __builtin_amdgcn_readfirstlane(*qcount(a, a.qpar));
    if ((int)blockIdx.x >= n) return;
    const int s = __builtin_amdgcn_readfirstlane(qlist(a, a.qpar)[blockIdx.x]);
    const int q = __builtin_amdgcn_readfirstlane(a.qctl[2 + s]);
    const double* st = carve(a.ws + (long)s * a.sW, a.N).state;
    if (q < 0 || st[S_ACTIVE] == 0.0) return;
    const int kk0 = (int)st[S_KK];
    __syncthreads();  // every wave has read the state before the solve rewrites it
    mw_solve<FX>(a, T, Who{s, q, q % a.nprob});
    __syncthreads();
    if (threadIdx.x == 0) {
        a.qctl[2 + s] = -1;
        atomicAdd(&a.dctr[0], a.kk[q] - kk0);  // the drain's iterations and problems
        atomicAdd(&a.dctr[1], 1);
        atomicAdd(&a.qctl[1], 1);
    }
}

// ------------------------------------------------------------------------------------------------
// d_kkt_solve_new_rhs_res_mpc_hard_tv: re-solve with the factor + iterate persisted in ws.
// vb/vq hold the new b (state order) / q (variable order).
// ------------------------------------------------------------------------------------------------
template <class FX>
__global__ __launch_bounds__(64) void hk_kkt_new_rhs(KArgs a) {
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
    BoxCtx bc = box_ctx(w, dv, lam, t);
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
    ResIO ro{};
    ro.bsrc = a.vb + o16;
    ro.qsrc = a.vq + o16;
    ro.ux = ux;
    ro.pi = pi;
    ro.rq = w.res_q;
    ro.rb = w.res_b;
    ro.rd = w.res_d;
    ro.rm = w.res_m;
    residual_pass<false, FX>(io, bc, ro, mu);
    wsync();
    HK_FOR_BOX(io, k, {
        w.qx[k * V16 + slot] = w.t_inv[lo] * (w.res_m[lo] - lam[lo] * w.res_d[lo]) -
                               w.t_inv[up] * (w.res_m[up] + lam[up] * w.res_d[up]);
    });
    HK_FOR_GEN(io, k, {
        w.qx[s16] = w.t_inv[lo] * (w.res_m[lo] - lam[lo] * w.res_d[lo]) -
                    w.t_inv[up] * (w.res_m[up] + lam[up] * w.res_d[up]);
    });
    wsync();
    double al = 1.0;
    ric_trs<BX_GIVEN, BX_NONE, FX>(io, &sm, w.res_b, w.res_q, bc, w.dux, a.compute_mult, w.dpi, 1, w.Pb, al);
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
    if (a.ngt) {  // the general slots: the same update from D dux (gen_alpha's phase-2 branch)
        for (int k = 0; k <= N; k++) {
            const StageInfo si = load_stage(io.st, k);
            if (si.ng == 0) continue;
            const DynSh sh(si);
            const int vc = tile_var(l & 15, sh.nu, sh.nx, sh.xo);
            double dummy = 1.0;
            gen_alpha<BX_P2>(io, sh, k, bc, gld(w.dux, k * V16 + vc, vc >= 0), dummy);
        }
    }
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
    HK_FOR_GEN(io, k, {
        lam[lo] += 1.0 * w.dlam[lo];
        lam[up] += 1.0 * w.dlam[up];
        t[lo] += 1.0 * w.dt[lo];
        t[up] += 1.0 * w.dt[up];
    });
}

// ------------------------------------------------------------------------------------------------
// d_kkt_solve_new_rhs_mpc_hard_tv (mpc_solvers/d_ip2_hard.c:626-825): re-solve of the alternate IPM's
// last KKT system for new b (r_A, in vb), q (r_H, in vq) and bounds (r_C, in d), on the factor and the
// lamt = lam/t that d_ip2_mpc_hard_tv left in ws.  ux / pi are solved for directly (not as a step).
// ------------------------------------------------------------------------------------------------
template <class FX>
__global__ __launch_bounds__(64) void hk_kkt_new_rhs_p1(KArgs a) {
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
    const double* rC = a.d + o32;
    const int l = lane_id();
    BoxCtx bc = box_ctx(w, rC, lam, t);
    // d_update_gradient_new_rhs_mpc_hard_tv (the reference's default X64_AVX build,
    // avx/d_aux_ip_hard_lib4.c:1735-1838): qx = -lamt_u r_C,u - lamt_l r_C,l
    HK_FOR_BOX(io, k, { w.qx[k * V16 + slot] = -w.lamt[up] * rC[up] - w.lamt[lo] * rC[lo]; });
    HK_FOR_GEN(io, k, { w.qx[s16] = -w.lamt[up] * rC[up] - w.lamt[lo] * rC[lo]; });
    wsync();
    double al = 1.0;
    ric_trs<BX_GIVEN, BX_NONE, FX>(io, &sm, a.vb + o16, a.vq + o16, bc, ux, a.compute_mult, pi, 1, w.Pb, al);
    wsync();
    // d_compute_t_lam_new_rhs_mpc_hard_tv (c99/d_aux_ip_hard_lib4.c:864-935)
    HK_FOR_BOX(io, k, {
        const double x = ux[k * V16 + bt.slotvar[k * 16 + slot]];
        const double tl = x - rC[lo], tu = -x + rC[up];
        t[lo] = tl;
        t[up] = tu;
        lam[lo] = -w.lamt[lo] * tl;
        lam[up] = -w.lamt[up] * tu;
    });
    if (a.ngt) {
        const int c = l & 15;
        for (int k = 0; k <= N; k++) {
            const StageInfo si = load_stage(io.st, k);
            if (si.ng == 0) continue;
            const DynSh sh(si);
            const int vc = tile_var(c, sh.nu, sh.nx, sh.xo);
            const double x = gld(ux, k * V16 + vc, vc >= 0);
            double dg[4];
            gen_dg(io, sh, dg);
#pragma unroll
            for (int lc = 0; lc < 4; lc++) {
                if (4 * lc >= sh.ng) continue;
                const GenLane q = gen_lane(k, sh.pnb, sh.ng, lc);
                const bool st = q.ok && c == 0;
                const double dx = row_sum16(dg[lc] * x);
                const double tl = dx - gld(rC, q.lo, q.ok), tu = -dx + gld(rC, q.up, q.ok);
                gst(t, q.lo, tl, st);
                gst(t, q.up, tu, st);
                gst(lam, q.lo, -gld(w.lamt, q.lo, q.ok) * tl, st);
                gst(lam, q.up, -gld(w.lamt, q.up, q.ok) * tu, st);
            }
        }
    }
}

// ------------------------------------------------------------------------------------------------
// Host launch helpers (called from the C-ABI translation unit).
// ------------------------------------------------------------------------------------------------
template <class FX>
static int launch_t(int which, const KArgs* a, int count, hipStream_t stream) {
    dim3 grid(count), block(64);
    const size_t lds = sizeof(Scratch) + (size_t)(a->N + 1) * (sizeof(StageInfo) + 40);
    switch (which) {
        case 0: hipLaunchKernelGGL(hk_ric_sv<FX>, grid, block, lds, stream, *a); break;
        case 1: hipLaunchKernelGGL(hk_ric_trf<FX>, grid, block, lds, stream, *a); break;
        case 2: hipLaunchKernelGGL(hk_ric_trs<FX>, grid, block, lds, stream, *a); break;
        case 3: hipLaunchKernelGGL(hk_res<FX>, grid, block, lds, stream, *a); break;
        case 4:
            hipLaunchKernelGGL(hk_ipm_init<FX>, grid, block, lds, stream, *a);
            for (int it = 0; it < a->k_max; it++) {
                hipLaunchKernelGGL(hk_ipm_fact<FX>, grid, block, lds, stream, *a);
                hipLaunchKernelGGL(hk_ipm_pred<FX>, grid, block, lds, stream, *a);
                hipLaunchKernelGGL(hk_ipm_corr<FX>, grid, block, lds, stream, *a);
                hipLaunchKernelGGL(hk_ipm_update<FX>, grid, block, lds, stream, *a);
            }
            break;
        case 5: hipLaunchKernelGGL(hk_kkt_new_rhs<FX>, grid, block, lds, stream, *a); break;
        case 6: hipLaunchKernelGGL(hk_kkt_new_rhs_p1<FX>, grid, block, lds, stream, *a); break;
        // single IPM pass kernels (hpmpc_mi355x_ipm_pass): the batched solve is 10, then k_max x (11..14)
        case 10: hipLaunchKernelGGL(hk_ipm_init<FX>, grid, block, lds, stream, *a); break;
        case 11: hipLaunchKernelGGL(hk_ipm_fact<FX>, grid, block, lds, stream, *a); break;
        case 12: hipLaunchKernelGGL(hk_ipm_pred<FX>, grid, block, lds, stream, *a); break;
        case 13: hipLaunchKernelGGL(hk_ipm_corr<FX>, grid, block, lds, stream, *a); break;
        case 14: hipLaunchKernelGGL(hk_ipm_update<FX>, grid, block, lds, stream, *a); break;
        // the queue's tick: fact (11), predictor + corrector (18), update (14)
        case 18: hipLaunchKernelGGL(hk_ipm_predcorr<FX>, grid, block, lds, stream, *a); break;
        // the whole IPM per problem in one launch (hk_ipm_solo)
        case 15:
        case 16: {
            // one problem per 256-thread workgroup (hk_ipm_solo_mw) unless HPMPC_MI355X_SOLO=1 asks for the
            // single-wave kernel (which == 16 forces it), the horizon exceeds the kernel's LDS tables, or the
            // launch guard (static + dynamic LDS, private segment vs the stack limit, launch bound; read once, with
            // thread-safe static initialisation) refuses it: then the single-wave kernel runs instead
            static const HkKernelLimits lim_mw(reinterpret_cast<const void*>(&hk_ipm_solo_mw<FX>));
            const char* env = getenv("HPMPC_MI355X_SOLO");
            const bool single = which == 16 || (env && env[0] == '1');
            const size_t lds_mw = mw_lds_bytes(a->N);
            hipLaunchKernelGGL(hk_ipm_init<FX>, grid, block, lds, stream, *a);
            if (!single && a->N <= MW_NMAX && lim_mw.check(lds_mw, 256) == 0)
                hipLaunchKernelGGL(hk_ipm_solo_mw<FX>, grid, dim3(256), lds_mw, stream, *a);
            else
                hipLaunchKernelGGL(hk_ipm_solo<FX>, grid, block, lds, stream, *a);
            break;
        }
        // the queue's drain (hk_ipm_qdrain_mw): grid = slots, four waves per workgroup; HK_LAUNCH_REFUSED when the
        // horizon or the launch guard rules the multi-wave kernel out (the host then keeps ticking)
        case 17: {
            static const HkKernelLimits lim_dr(reinterpret_cast<const void*>(&hk_ipm_qdrain_mw<FX>));
            const size_t lds_mw = mw_lds_bytes(a->N);
            if (a->N > MW_NMAX || lim_dr.check(lds_mw, 256) != 0) return HK_LAUNCH_REFUSED;
            hipLaunchKernelGGL(hk_ipm_qdrain_mw<FX>, grid, dim3(256), lds_mw, stream, *a);
            break;
        }
        default: return -1;
    }
    return (int)hipGetLastError();
}

// Compiled inner-stage classes (KArgs.fixcls): 0 generic, 1 nu=4 nx=12, 2 nu=3 nx=8.  The plan picks
// the class and flags its stages (StageInfo.r0); any other problem runs the generic kernels.
extern "C" int hk_fixcls(int nu, int nx) {
    if (nu == 4 && nx == 12) return 1;
    if (nu == 3 && nx == 8) return 2;
    return 0;
}

#ifdef HK_STAMPS
// Diagnostic build only: the clamp-certificate counters of the tile kernels (g_xfac_stat), read and optionally reset.
extern "C" __attribute__((visibility("default"))) int hpmpc_mi355x_diag_xfac(unsigned long long* out, int reset) {
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_xfac_stat), 6 * sizeof(unsigned long long)) != hipSuccess) return -11;
    if (reset) {
        const unsigned long long z[6] = {0, 0, 0, 0, 0, 0};
        if (hipMemcpyToSymbol(HIP_SYMBOL(g_xfac_stat), z, sizeof(z)) != hipSuccess) return -11;
    }
    return 0;
}
#endif

extern "C" int hk_launch(int which, const KArgs* a, int count, hipStream_t stream) {
    if (count <= 0) return 0;
#ifdef HK_STAMPS
    if (a->dbg) {
        unsigned long long* p = a->dbg;
        int st = 50;
        (void)hipMemcpyToSymbol(HIP_SYMBOL(g_dbg), &p, sizeof(p));
        (void)hipMemcpyToSymbol(HIP_SYMBOL(g_dbg_stage), &st, sizeof(st));
    }
    {
        const char* f = getenv("HPMPC_MI355X_MW_FAULT");
        const int fault = (f && f[0] == '1') ? 1 : 0;
        (void)hipMemcpyToSymbol(HIP_SYMBOL(g_mw_fault), &fault, sizeof(fault));
    }
#endif
    switch (a->fixcls) {
        case 1: return launch_t<FixSh<4, 12>>(which, a, count, stream);
        case 2: return launch_t<FixSh<3, 8>>(which, a, count, stream);
        default: return launch_t<NoFix>(which, a, count, stream);
    }
}
