// hk_ipm_body.h -- the per-problem IPM building blocks shared by the pass kernels (hpmpc_kernels.hip) and the
// persistent problem-queue kernel (hk_qloop.hip): workspace carve, LDS stage tables, problem views, init / start /
// refill of a solve and the bodies of the four iteration passes (d_ip2_res_hard.c:116-1345).
#pragma once
#include "hk_ipm.h"
#include "hk_launch_guard.h"
#include "hpmpc_kargs.h"

using namespace hk;

// IPM pass kernels fit two waves per SIMD (<= 256 VGPRs), so a problem queue with two slots per SIMD
// interleaves two problems' dependency chains.
#ifndef HK_WAVES
#define HK_WAVES 2
#endif
#define HK_TWO_WAVES __attribute__((amdgpu_waves_per_eu(HK_WAVES)))

namespace {

struct Ws {  // per-problem workspace carve (doubles), persistent between an IPM and a KKT re-solve
    double *F, *dux, *dpi, *Pb, *Qx, *qx, *res_q, *res_b, *ux_bkp, *pi_bkp;
    double *dlam, *dt, *t_inv, *lamt, *res_d, *res_m, *t_bkp, *lam_bkp;
    double* state;  // IpmState (16 doubles) carried between the IPM pass kernels
    double* cert;   // N+1: the clamp certificate's threshold per stage (the first factorisation of a solve)
};

// Per-problem IPM control state between the pass kernels of one batched solve.
enum { S_MU = 0, S_ALPHA, S_SIGMA, S_SMU, S_KK, S_PHASE, S_ACTIVE, S_MUSCAL, S_RET };

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
    w.state = W + 8 * b;
    w.cert = w.state + 16;
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
    double* gc;  // N+1: the problem's clamp-certificate bounds (filled by the factorisation pass, fact_body)
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
    T.gc = reinterpret_cast<double*>(sv + n1 * 16);
    return T;
}

__device__ __forceinline__ RicIO make_io(const KArgs& a, const LdsTabs& T, int p, double* F) {
    RicIO io;
    io.N = a.N;
    io.st = T.st;
    io.tileslot = T.tileslot;
    io.BAbt = a.BAbt + (long)p * a.sB;
    io.RSQ = a.RSQ + (long)p * a.sR;
    io.BAbtS = a.BAbt;
    io.RSQS = a.RSQ;
    io.F = F;
    io.DCt = a.DCt ? a.DCt + (long)p * a.sG : a.RSQ;  // never read when every ng = 0
    return io;
}

__device__ __forceinline__ void wsync() { __syncthreads(); }

}  // namespace

namespace {

// d_init_var_mpc_hard_tv (d_aux_ip_hard_lib4.c:59-130) as a quad pass: lane (g, c) owns variable c of
// stage 4q+g and, when c is boxed, its box slot; CH quads are loaded before any is computed, so a
// refill costs a few memory round trips instead of one per stage.  Also zeroes pi and dpi.
template <int CH>
__device__ void init_var(const RicIO& io, const double* dv, double* ux, double* pi, double* dpi, double* lam,
                         double* t, double mu0, int warm_start) {
    const int l = lane_id(), g = l >> 4, c = l & 15;
    const double thr0 = 0.1;
    const int nq = (io.N + 4) / 4;
    for (int q0 = 0; q0 < nq; q0 += CH) {
        double dl[CH], du[CH], xv[CH];
        int lo[CH], up[CH], iv[CH];
        bool kv[CH], bx[CH], kp[CH];
#pragma unroll
        for (int j = 0; j < CH; j++) {
            const int k = 4 * (q0 + j) + g;
            kv[j] = k <= io.N;
            kp[j] = k < io.N;
            const int kc = kv[j] ? k : io.N;
            const StageInfo& si = io.st[kc];
            const bool okv = c < si.nu + si.nx;
            const int tile = c < si.nu ? c : si.xo + (c - si.nu);
            const int slot = okv ? io.tileslot[kc * 16 + (okv ? tile : 0)] : -1;
            bx[j] = kv[j] && slot >= 0;
            lo[j] = kc * V32 + (slot >= 0 ? slot : 0);
            up[j] = lo[j] + si.pnb;
            iv[j] = kc * V16 + c;
            dl[j] = gld(dv, lo[j], bx[j]);
            du[j] = gld(dv, up[j], bx[j]);
            xv[j] = warm_start ? gld(ux, iv[j], kv[j]) : 0.0;
        }
#pragma unroll
        for (int j = 0; j < CH; j++) {
            double x = xv[j];
            double tl = -dl[j] + x, tu = du[j] - x;
            if (tl < thr0) {
                if (tu < thr0) {
                    x = (-du[j] + dl[j]) * 0.5;
                    tl = thr0;
                    tu = thr0;
                } else {
                    tl = thr0;
                    x = dl[j] + thr0;
                }
            } else if (tu < thr0) {
                tu = thr0;
                x = du[j] - thr0;
            }
            x = bx[j] ? x : xv[j];
            gst(ux, iv[j], x, kv[j]);
            gst(pi, iv[j], 0.0, kp[j]);
            gst(dpi, iv[j], 0.0, kv[j]);
            gst(t, lo[j], tl, bx[j]);
            gst(t, up[j], tu, bx[j]);
            gst(lam, lo[j], mu0 / tl, bx[j]);
            gst(lam, up[j], mu0 / tu, bx[j]);
        }
    }
}

// General-constraint part of d_init_var_mpc_hard_tv (d_aux_ip_hard_lib4.c:131-149): slacks from D ux of
// the (box-adjusted) start point, clipped at thr0.  Call after init_var's stores are visible.
__device__ void init_var_gen(const RicIO& io, const double* dv, const double* ux, double* lam, double* t,
                             double mu0) {
    const int l = lane_id(), c = l & 15;
    const double thr0 = 0.1;
    for (int k = 0; k <= io.N; k++) {
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
            const double tl = fmax(thr0, dx + (-gld(dv, q.lo, q.ok)));
            const double tu = fmax(thr0, -dx + gld(dv, q.up, q.ok));
            gst(t, q.lo, tl, st);
            gst(t, q.up, tu, st);
            gst(lam, q.lo, mu0 / tl, st);
            gst(lam, q.up, mu0 / tu, st);
        }
    }
}

__device__ __forceinline__ BoxCtx box_ctx(const Ws& w, const double* dv, double* lam, double* t) {
    BoxCtx bc{};
    bc.d = dv;
    bc.lam = lam;
    bc.t = t;
    bc.dlam = w.dlam;
    bc.dt = w.dt;
    bc.t_inv = w.t_inv;
    bc.lamt = w.lamt;
    bc.res_d = w.res_d;
    bc.res_m = w.res_m;
    bc.qxs = w.qx;
    bc.Qx = w.Qx;
    bc.qx = w.qx;
    bc.cert = w.cert;
    bc.cert_out = w.cert;
    bc.cert_new = 0;
    bc.res_q = w.res_q;
    bc.res_b = w.res_b;
    return bc;
}

}  // namespace

// The IPM runs as one init kernel and then, per iteration, four pass kernels (factorisation, solve +
// step length + mu_aff, corrector, update + residuals).  Every kernel handles the whole batch; a
// problem that has finished returns at once.  Each pass kernel is a single stage loop, so it gets
// its own register allocation, and rocprof reports the passes separately.
namespace {

struct IpmView {
    int N, q, l;  // q: iterate / output index (the problem in batch mode, the queue entry in queue mode)
    Ws w;
    RicIO io;
    BoxTab bt;
    double *ux, *pi, *lam, *t, *stat;
    const double* dv;
    BoxCtx bc;
};

// Queue active-slot lists (KArgs.qctl layout): length and entries of list p.
__device__ __forceinline__ int* qcount(const KArgs& a, int p) { return a.qctl + 2 + a.nslots + p; }
__device__ __forceinline__ int* qlist(const KArgs& a, int p) { return a.qctl + 4 + a.nslots + p * a.nslots; }
__device__ __forceinline__ void qlist_push(const KArgs& a, int p, int s) {
    if (lane_id() == 0) qlist(a, p)[atomicAdd(qcount(a, p), 1)] = s;
}

// Which workspace (s), iterate/output (q) and data problem (d) this workgroup works on.
struct Who {
    int s, q, d;
};

__device__ __forceinline__ bool who_am_i(const KArgs& a, Who& w) {
    if (a.nq == 0) {
        const int p = blockIdx.x + a.p0;
        w.s = w.q = w.d = p;
        return p < a.nprob;
    }
    // queue: workgroup i takes the i-th listed active slot, so a draining queue runs a dense grid prefix (one
    // wave per SIMD once fewer slots than SIMDs iterate) instead of scattered slots that share SIMDs
    const int n = __builtin_amdgcn_readfirstlane(*qcount(a, a.qpar));
    if ((int)blockIdx.x >= n) return false;
    w.s = __builtin_amdgcn_readfirstlane(qlist(a, a.qpar)[blockIdx.x]);
    w.q = __builtin_amdgcn_readfirstlane(a.qctl[2 + w.s]);
    w.d = w.q >= 0 ? w.q % a.nprob : 0;
    return w.q >= 0;
}

// Whether this workgroup's problem still iterates (its control state in the slot's workspace); read before
// the stage tables are staged, so the finished problems of a batch and the idle slots of a draining queue
// return at once.
__device__ __forceinline__ bool slot_active(const KArgs& a, const Who& who) {
    return carve(a.ws + (long)who.s * a.sW, a.N).state[S_ACTIVE] != 0.0;
}

__device__ __forceinline__ IpmView ipm_view(const KArgs& a, const LdsTabs& T, const Who& who) {
    IpmView v;
    v.N = a.N;
    v.q = who.q;
    v.l = lane_id();
    v.w = carve(a.ws + (long)who.s * a.sW, a.N);
    v.io = make_io(a, T, who.d, v.w.F);
    v.bt = BoxTab{T.tileslot, T.slotvar};
    const long o16 = (long)who.q * a.sV16, o32 = (long)who.q * a.sV32;
    v.ux = a.ux + o16;
    v.pi = a.pi + o16;
    v.lam = a.lam + o32;
    v.t = a.t + o32;
    v.dv = a.d + (long)who.d * a.sV32;
    v.stat = a.stat + (long)who.q * 5 * a.k_max;
    v.bc = box_ctx(v.w, v.dv, v.lam, v.t);
    v.bc.ux = v.ux;
    v.bc.pi = v.pi;
    return v;
}

__device__ __forceinline__ ResIO res_io(const IpmView& v) {
    ResIO ro{};
    ro.ux = v.ux;
    ro.pi = v.pi;
    ro.dux = v.w.dux;
    ro.dpi = v.w.dpi;
    ro.ux_bkp = v.w.ux_bkp;
    ro.pi_bkp = v.w.pi_bkp;
    ro.lam_bkp = v.w.lam_bkp;
    ro.t_bkp = v.w.t_bkp;
    ro.rq = v.w.res_q;
    ro.rb = v.w.res_b;
    ro.rd = v.w.res_d;
    ro.rm = v.w.res_m;
    return ro;
}

// Phase-2 start residuals: r_d, r_m and mu here; r_q, r_b in the first phase-2 factorisation.  CI: stages
// per chunk of the element-wise passes (7 in hk_ipm_init; 2 inside hk_ipm_update, where the problem-start and
// phase-switch paths run once per problem and must not raise the update loop's register allocation).
template <class FX, int CI, int NW = 1>
__device__ double p2_start(const KArgs& a, IpmView& v, const MwSplit& mws = MwSplit{0, nullptr}) {
    const double mu = update_p2_pass<CI, false, true, NW>(v.io, v.bc, v.bt.slotvar, 0.0, 1.0 / (2.0 * a.nbt), v.ux,
                                                          v.pi, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr,
                                                          v.w.res_d, v.w.res_m, mws);
    wsync();
    return mu;
}

// End of an iteration (or of init): decide whether the problem continues, switching from phase 1 to
// phase 2 (with the phase-2 start residuals) when phase 1's loop condition fails.
template <class FX, int CI, int NW = 1>
__device__ bool ipm_continue(const KArgs& a, IpmView& v, int kk, double mu, double alpha, double sigma, int phase,
                             const MwSplit& mws = MwSplit{0, nullptr}) {
    const bool sn = a.single_newton != 0;
    bool active;
    if (a.phase1_only) {  // d_ip2_mpc_hard_tv: the phase-1 loop run to mu_tol (d_ip2_hard.c:329-520)
        active = kk < a.k_max && mu > a.mu_tol && alpha >= a.alpha_min;
    } else {
        if (phase == 1) {
            const double mu_tol_low = a.mu_tol < 1e-5 ? 1e-5 : a.mu_tol;
            if (!(kk < a.k_max && mu > mu_tol_low && alpha >= a.alpha_min)) {
                mu = p2_start<FX, CI, NW>(a, v, mws);  // phase-2 start (d_ip2_res_hard.c:756-781)
                phase = 2;
            }
        }
        active = phase == 1;
        if (phase == 2) active = kk < a.k_max && (sn || (mu > a.mu_tol && alpha >= a.alpha_min));
    }
    int ret = 0;
    if (!active) {
        if (!sn && mu <= a.mu_tol)
            ret = 0;
        else if (kk >= a.k_max)
            ret = 1;
        else if (alpha < a.alpha_min)
            ret = 2;
        else
            ret = -1;
    }
    if (v.l == 0) {
        double* st = v.w.state;
        st[S_MU] = mu;
        st[S_ALPHA] = alpha;
        st[S_SIGMA] = sigma;
        st[S_KK] = kk;
        st[S_PHASE] = phase;
        st[S_ACTIVE] = active ? 1.0 : 0.0;
        if (!active) {
            a.kk[v.q] = kk;
            a.ret[v.q] = ret;
        }
    }
    return active;
}

// Start of a solve: init_var and the loop-control state.  Returns whether the problem iterates.
// SHORTCUT: compile the unconstrained one-Riccati-solve exits (nbt == 0, a plan-wide constant).  hk_ipm_update
// leaves them out: with nbt == 0 every entry finishes inside ipm_start, so hk_ipm_init's refill loop drains the
// whole queue and no update pass ever refills a slot.
template <class FX, int CI, bool SHORTCUT>
__device__ bool ipm_start(const KArgs& a, const LdsTabs& T, IpmView& v) {
    Scratch& sm = *T.sm;
    const int N = v.N, l = v.l;
    const int nbt = a.nbt;
    if (!SHORTCUT && nbt == 0) return false;
    if (SHORTCUT && nbt == 0 && a.phase1_only) {
        // d_ip2_mpc_hard_tv without constraints: one sv into the workspace's dux / dpi, the caller's
        // ux / pi stay untouched (d_ip2_hard.c:282-291)
        ric_backward<true, BX_NONE, FX>(v.io, &sm, 0, nullptr, 0, nullptr, v.bc, 1, v.w.Pb);
        wsync();
        ric_forward_sv<FX>(v.io, &sm, 0, nullptr, v.w.dux, a.compute_mult, v.w.dpi);
        if (l == 0) {
            v.w.state[S_ACTIVE] = 0.0;
            a.kk[v.q] = 0;
            a.ret[v.q] = 0;
        }
        return false;
    }
    if (SHORTCUT && nbt == 0) {
        // no constraints: one sv and return (d_ip2_res_hard.c:428-450)
        ric_backward<true, BX_NONE, FX>(v.io, &sm, 0, nullptr, 0, nullptr, v.bc, 1, v.w.Pb);
        wsync();
        ric_forward_sv<FX>(v.io, &sm, 0, nullptr, v.ux, a.compute_mult, v.pi);
        wsync();
        for (int i = l; i < (N + 1) * V16; i += 64) {
            v.w.ux_bkp[i] = v.ux[i];
            v.w.pi_bkp[i] = v.pi[i];
        }
        if (l == 0) {
            v.w.state[S_ACTIVE] = 0.0;
            a.kk[v.q] = 0;
            a.ret[v.q] = 0;
        }
        return false;
    }
    // single Newton step (d_ip2_res_hard.c:1348-1919): the caller's ux/pi/lam/t already hold the start
    // iterate (d_init_var_mpc_hard_tv_single_newton is a copy, done by the host), no phase 1.
    const bool sn = a.single_newton != 0;
    if (!sn) {
        init_var<CI>(v.io, v.dv, v.ux, v.pi, v.w.dpi, v.lam, v.t, a.mu0, a.warm_start);
        if (a.ngt) {
            wsync();
            init_var_gen(v.io, v.dv, v.ux, v.lam, v.t, a.mu0);
        }
    } else {
        for (int i = l; i < (N + 1) * V16; i += 64) v.w.dpi[i] = 0.0;
    }
    if (l == 0) v.w.state[S_MUSCAL] = 1.0 / (2.0 * nbt);
    wsync();
    double mu = a.mu0;
    if (sn) mu = p2_start<FX, CI>(a, v);  // straight to phase 2: its start residuals
    return ipm_continue<FX, CI>(a, v, 0, mu, 1.0, 0.0, sn ? 2 : 1);
}

// Queue mode: hand slot s the next queue entries until one of them iterates (true) or the queue is empty.
template <class FX, int CI, bool SHORTCUT>
__device__ bool ipm_refill(const KArgs& a, const LdsTabs& T, int s) {
    const bool l0 = lane_id() == 0;
    for (;;) {
        int q = 0;
        if (l0) q = atomicAdd(a.qnext, 1);
        q = __builtin_amdgcn_readfirstlane(q);
        if (q >= a.nq) {
            if (l0) a.qctl[2 + s] = -1;
            return false;
        }
        if (l0) a.qctl[2 + s] = q;
        const Who who{s, q, q % a.nprob};
        IpmView v = ipm_view(a, T, who);
        if (ipm_start<FX, CI, SHORTCUT>(a, T, v)) return true;
        if (l0) atomicAdd(&a.qctl[1], 1);
    }
}

}  // namespace

// The bodies of the four iteration passes.  Each runs one pass of one problem (its IpmView) and reads / writes
// the problem's control state in its workspace; the pass kernels run one body over a batch or queue, the solo
// kernel runs them all in sequence for one problem per workgroup.
namespace {

// Factorisation of the iteration's KKT system, Hessian / gradient box terms fused into the fetch.
template <class FX>
__device__ __forceinline__ void fact_body(const KArgs& a, const LdsTabs& T, IpmView& v) {
    Scratch& sm = *T.sm;
    const double* st = v.w.state;
    const bool sn = a.single_newton != 0;
    // The clamp certificate's bounds: the solve's first factorisation forms them from the data tiles it loads anyway
    // (CERT_FORM: a phase-1 one, except in the single-Newton variant, which starts in phase 2 and runs the bounds'
    // own pass first); the later ones read them, staged in LDS (ds_read in the stage loop instead of one more buffer
    // descriptor in SGPRs).
    const bool first = st[S_KK] == 0.0;
    if (first && st[S_PHASE] != 1.0) {
        cert_pass(v.io, v.w.cert);
        wsync();
    }
    if (!first || st[S_PHASE] != 1.0)
        for (int i = v.l; i <= v.N; i += 64) T.gc[i] = v.w.cert[i];
    wsync();
    v.bc.cert = T.gc;
    if (st[S_PHASE] == 1.0) {
        if (first)
            ric_backward<true, BX_P1, FX, CERT_FORM>(v.io, &sm, 0, nullptr, 0, nullptr, v.bc, 1, v.w.Pb);
        else
            ric_backward<true, BX_P1, FX, CERT_LOAD>(v.io, &sm, 0, nullptr, 0, nullptr, v.bc, 1, v.w.Pb);
    } else {  // the single-Newton variant factorises with the data's own b/q rows (d_ip2_res_hard.c:1700-1760)
        v.bc.res_rhs = !sn;
        v.bc.no_tinv = a.no_bkp;
        ric_backward<true, BX_P2R, FX, CERT_LOAD>(v.io, &sm, 0, nullptr, 0, nullptr, v.bc, 1, v.w.Pb);
    }
}

// Predictor solve with the box steps and step length fused in, then mu_aff and the centering target.
template <class FX>
__device__ __forceinline__ void pred_body(const KArgs& a, const LdsTabs& T, IpmView& v) {
    Scratch& sm = *T.sm;
    double* st = v.w.state;
    const bool sn = a.single_newton != 0;
    const int phase = (int)st[S_PHASE], kk = (int)st[S_KK];
    const double mu = st[S_MU];
    double sigma = st[S_SIGMA];
    double al = 1.0;
    // The predictor's multipliers are never read: the corrector's solve overwrites dpi before the
    // update uses it (d_ip2_res_hard.c:527 vs :628 and :948 vs :1168), so the predictor skips them.
    if (phase == 1) {
        v.bc.pred = 1;
        ric_forward<0, BX_P1, FX, true>(v.io, &sm, nullptr, 0, v.w.dux, 0, v.w.dpi, v.bc, al);
    } else {
        ric_forward<0, BX_P2, FX, true>(v.io, &sm, v.w.res_b, !sn, v.w.dux, 0, v.w.dpi, v.bc, al);
    }
    al = wave_min(al);
    wsync();
    const double alpha = al * 0.995;
    const double mu_aff = mu_aff_pass<7>(v.io, v.bc, alpha, st[S_MUSCAL]);
    double smu = a.mu0;  // single Newton: sigma*mu is supplied by the caller as mu0 (:1788-1790)
    if (!sn) {
        sigma = mu_aff / mu;
        sigma = sigma * sigma * sigma;
        smu = sigma * mu;
    }
    if (v.l == 0) {
        v.stat[5 * kk] = st[S_SIGMA];
        v.stat[5 * kk + 1] = al;
        v.stat[5 * kk + 2] = mu_aff;
        st[S_SIGMA] = sigma;
        st[S_SMU] = smu;
    }
}

// Corrector: centering / gradient update fused into the trs backward, box steps + alpha into its forward.
template <class FX>
__device__ __forceinline__ void corr_body(const KArgs& a, const LdsTabs& T, IpmView& v) {
    Scratch& sm = *T.sm;
    double* st = v.w.state;
    const int phase = (int)st[S_PHASE], kk = (int)st[S_KK];
    v.bc.smu = st[S_SMU];
    double al = 1.0;
    if (phase == 1)
        ric_trs<BX_P1, BX_P1, FX, false>(v.io, &sm, nullptr, nullptr, v.bc, v.w.dux, a.compute_mult, v.w.dpi, 0, v.w.Pb,
                                         al);
    else
        ric_trs<BX_P2, BX_P2, FX, false>(v.io, &sm, v.w.res_b, v.w.res_q, v.bc, v.w.dux, a.compute_mult, v.w.dpi, 0,
                                         v.w.Pb, al);
    al = wave_min(al);
    if (v.l == 0) {
        v.stat[5 * kk] = st[S_SIGMA];
        v.stat[5 * kk + 3] = al;
        st[S_ALPHA] = al * 0.995;
    }
}

// Update of the iterate (with backups) and, in phase 2, the residuals of the new iterate; loop control.  Returns
// whether the problem iterates again (CI: stages per chunk of the element-wise passes).
template <class FX, int CI>
__device__ __forceinline__ bool update_body(const KArgs& a, IpmView& v) {
    double* st = v.w.state;
    const int phase = (int)st[S_PHASE];
    int kk = (int)st[S_KK];
    const double alpha = st[S_ALPHA];
    double mu;
    if (phase == 1) {
        mu = update_p1_pass<CI>(v.io, v.bc, alpha, st[S_MUSCAL], v.ux, v.pi, v.w.dux, v.w.dpi, v.w.ux_bkp,
                                v.w.pi_bkp, v.w.lam_bkp, v.w.t_bkp);
    } else {
        if (a.no_bkp)  // wave-uniform: the public queue API keeps no backups (nothing re-solves its slots)
            mu = update_p2_pass<CI, true, false>(v.io, v.bc, v.bt.slotvar, alpha, st[S_MUSCAL], v.ux, v.pi, v.w.dux,
                                                 v.w.dpi, v.w.ux_bkp, v.w.pi_bkp, v.w.lam_bkp, v.w.t_bkp, v.w.res_d,
                                                 v.w.res_m);
        else
            mu = update_p2_pass<CI, true>(v.io, v.bc, v.bt.slotvar, alpha, st[S_MUSCAL], v.ux, v.pi, v.w.dux, v.w.dpi,
                                          v.w.ux_bkp, v.w.pi_bkp, v.w.lam_bkp, v.w.t_bkp, v.w.res_d, v.w.res_m);
    }
    wsync();
    if (v.l == 0) v.stat[5 * kk + 4] = mu;
    kk++;
    return ipm_continue<FX, CI>(a, v, kk, mu, alpha, st[S_SIGMA], phase);
}

}  // namespace
