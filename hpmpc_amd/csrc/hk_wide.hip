// hk_wide.hip -- MI355X (gfx950) kernels for stages wider than the 16-wide register tile:
//   hk_wide_sv  d_back_ric_rec_sv_tv_res (lqcp_solvers/d_back_ric_rec.c:112-399) for nu+nx > 16, one
//               256-thread workgroup per problem, the stage Hessian in LDS as packed lower columns;
//   hk_pcond    d_part_cond (lqcp_solvers/d_part_cond.c:926-1062): one workgroup per (block, problem),
//               every block of every problem condensed concurrently;
//   hk_pexpand  d_part_expand_solution (d_part_cond.c:1103-1308): one workgroup per (block, problem).
//
// These are the "next" rows of SURVEY.md §8f #1 (configs[4]: N=200 -> 20 blocks of 10, nx=24 nu=6).
// Every stage matrix is read from HBM once per pass in the reference's lib4 layout and staged into LDS
// as a dense column-major tile; the per-stage work is spread over the 256 lanes of the workgroup with
// one barrier per dependency step (one per Cholesky column).
#include <hip/hip_runtime.h>

#include "hk_wide_core.h"

#ifdef HK_STAMPS
// Diagnostic build only: per-phase s_memtime cycle totals of hk_pcond workgroup (0, 0) (tools/pcond_phases.py)
__device__ unsigned long long* g_pdbg;
extern "C" __attribute__((visibility("default"))) int hpmpc_mi355x_pcond_debug(void* dev_ptr) {
    return (int)hipMemcpyToSymbol(HIP_SYMBOL(g_pdbg), &dev_ptr, sizeof(void*));
}
// per-phase totals kept in (wave-uniform) registers and written once at the end, so a stamp costs no memory access
#define PST_DECL unsigned long long pst_acc[16] = {}, pst_t0 = 0
#define PST(i)                                                                    \
    do {                                                                          \
        unsigned long long t_;                                                    \
        asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t_)::"memory"); \
        if ((i) > 0) pst_acc[i] += t_ - pst_t0;                                   \
        pst_t0 = t_;                                                              \
    } while (0)
#define PST_FLUSH()                                                               \
    do {                                                                          \
        if (g_pdbg && blockIdx.x == 0 && blockIdx.y == 0 && threadIdx.x == 0)     \
            for (int q_ = 0; q_ < 16; q_++) g_pdbg[q_] += pst_acc[q_];            \
    } while (0)
#else
#define PST_DECL (void)0
#define PST(i) \
    do {       \
    } while (0)
#define PST_FLUSH() (void)0
#endif


// d_back_ric_rec_sv_tv_res / _trf_tv_res on wide stages (wide_sv_body, hk_wide_core.h)
__global__ __launch_bounds__(WT) void hk_wide_sv(WideArgs a) {
    const int p = blockIdx.x + a.p0;
    if (p >= a.nprob) return;
    wide_stage_table(a);
    wide_sv_body(a, wide_prob(a, p));
}

// ------------------------------------------------------------------------------------------------
// The condensing's state-block Cholesky with its gradient row (d_cond_RSQrq's dpotrf_l on [pL_xx; pL_r],
// d_part_cond.c:436-470) on one wave, for nx <= 28, as 16x16 MFMA tiles of the 32x32 padded block (the gradient row
// sits at padded row 31, padding is zero):
//   T00 rows / cols 0..15 and T11 rows / cols 16..31, symmetric storage (register r at lane (g,c) = A[4r+g][c]);
//   U the off-diagonal rows 16..31 transposed (register r at lane (g,c) = A[16+c][4r+g]).
// Pivot block B (4 pivots): its 4x4 diagonal block is broadcast (DPP row_newbcast) and factorised redundantly in
// every lane, each lane solves its own row of the block column (T00 and U rows, a row-group gather each), and the
// rank-4 trailing update is one v_mfma_f64_16x16x4 per tile.  Pivot clamp d > 1e-15 else 0 (kernel_dpotrf_c99_lib4.c
// :555-640) with 1/sqrt(d) from v_rsq_f64 + one refinement (hk::chol_inv); padded pivots clamp to 0.  Replaces the
// per-pivot readlane broadcasts (two v_readlane per entry of the pivot column).
// ------------------------------------------------------------------------------------------------
// The same factorisation for nx > 28 (row i on lane i, nx + 1 <= 64 rows): 16-column panels in registers, the pivot
// column broadcast by readlane, each panel followed by its update of the later columns.  In place on X.
__device__ __attribute__((noinline)) void xchol_rows(double* X, int ldX, int nxs) {
    const int i = threadIdx.x & 63;
    for (int p0 = 0; p0 < nxs; p0 += 16) {
        const int pw = nxs - p0 < 16 ? nxs - p0 : 16;
        double cl[16];
#pragma unroll
        for (int jj = 0; jj < 16; jj++) cl[jj] = (jj < pw && i >= p0 + jj && i <= nxs) ? X[i + (p0 + jj) * ldX] : 0.0;
#pragma unroll
        for (int jj = 0; jj < 16; jj++) {
            if (jj < pw) {
                const double d = rdlane(cl[jj], p0 + jj);
                double sq, inv;
                hk::chol_pivot(d, sq, inv);
                cl[jj] = i == p0 + jj ? sq : (i > p0 + jj ? cl[jj] * inv : 0.0);
#pragma unroll
                for (int cc = jj + 1; cc < 16; cc++) cl[cc] -= cl[jj] * rdlane(cl[jj], p0 + cc);
            }
        }
#pragma unroll
        for (int jj = 0; jj < 16; jj++)
            if (jj < pw && i >= p0 + jj && i <= nxs) X[i + (p0 + jj) * ldX] = cl[jj];
        for (int c = p0 + 16; c < nxs; c++) {  // the panel's update of column c (rows >= c)
            double acc = 0.0;
#pragma unroll
            for (int jj = 0; jj < 16; jj++) acc += cl[jj] * rdlane(cl[jj], c);
            if (i >= c && i <= nxs) X[i + c * ldX] -= acc;
        }
        wave_sync();
    }
}

// The block is read through S(i, j) (i >= j: row i, column j; row nx = the gradient row) and the factor written to X
// ((nx+1) x nx lower, dense, ld ldX).  Wave-level (one wave calls it).
template <class FS>
__device__ __forceinline__ void xchol_tiles(FS S, double* X, int ldX, int nx) {  // the P form's fallback
    const int l = threadIdx.x & 63, g = l >> 4, c = l & 15;
    auto src = [&](int t) { return t < nx ? t : (t == 31 ? nx : -1); };
    auto at = [&](int t1, int t2) -> double {  // A[t1][t2] of the padded symmetric block
        const int i1 = src(t1), i2 = src(t2);
        const int r = i1 > i2 ? i1 : i2, q = i1 > i2 ? i2 : i1;
        const bool ok = q >= 0 && q < nx;
        const double v = S(ok ? r : 0, ok ? q : 0);  // unconditional load (no exec-masked branch), then a select
        return ok ? v : 0.0;
    };
    hk::d4 T00, U, T11;
#pragma unroll
    for (int r = 0; r < 4; r++) {
        T00[r] = at(4 * r + g, c);
        U[r] = at(16 + c, 4 * r + g);
        T11[r] = at(16 + 4 * r + g, 16 + c);
    }
    double inv = 0.0;  // not needed: the condensing keeps L only
    if (nx > 0) tile_chol_block<0, 1, true>(T00, &U, 1, &T11, inv);
    if (nx > 4) tile_chol_block<1, 1, true>(T00, &U, 1, &T11, inv);
    if (nx > 8) tile_chol_block<2, 1, true>(T00, &U, 1, &T11, inv);
    if (nx > 12) tile_chol_block<3, 1, true>(T00, &U, 1, &T11, inv);
    if (nx > 16) tile_chol_block<0, 1, false>(T11, &U, 0, &T11, inv);
    if (nx > 20) tile_chol_block<1, 1, false>(T11, &U, 0, &T11, inv);
    if (nx > 24) tile_chol_block<2, 1, false>(T11, &U, 0, &T11, inv);
#pragma unroll
    for (int r = 0; r < 4; r++) {
        const int col = 4 * r + g, c1 = 16 + col, row1 = src(16 + c);
        if (c >= col && c < nx && col < nx) X[c + col * ldX] = T00[r];
        if (row1 >= 0 && col < nx) X[row1 + col * ldX] = U[r];
        if (c >= col && row1 >= 0 && c1 < nx) X[row1 + c1 * ldX] = T11[r];
    }
}

// ------------------------------------------------------------------------------------------------
// Partial condensing of one block (d_cond_BAbt :214-303, d_cond_RSQrq :307-574, d_cond_DCtd :579-688).
// Condensed stage variables: [u_{T-1}; ...; u_0; x_0].  Gamma_j (rows [u_j..u_0, x_0, 1] x nx_{j+1},
// dense column-major) is formed once and read again by the RSQrq and DCtd phases through the problem's HBM scratch,
// with only Gamma_{j-1} in LDS; the stage tiles (pL, Lx, BAbt, W) are in LDS too.  Keeping a whole block's Gammas in
// LDS instead (130 KiB at configs[4]) measured 2.7x slower: the workgroup's own time fell 17 %, but one workgroup
// per CU instead of four leaves nothing to hide its dependency chains behind.
// ------------------------------------------------------------------------------------------------
// GM: output tiles per wave of its gemms (host-chosen from the block shapes: 4, or 8 at two workgroups per CU)
template <int GM>
__global__ __launch_bounds__(WT, GM <= 4 ? 4 : 2) void hk_pcond(PcArgs a) {  // 4 waves per SIMD at GM 4: four workgroups per CU (the LDS fits four)
    extern __shared__ double sm[];
    const int ii = blockIdx.x, p = blockIdx.y + a.p0;
    if (p >= a.nprob || ii >= a.N2) return;
    const int tid = threadIdx.x;
    const PcBlock blk = a.blk[ii];
    const int T = blk.T, nx0 = blk.nx0, nv = blk.nut + nx0;
    WideStage* stl = reinterpret_cast<WideStage*>(sm + a.offST);  // the block's stage records, in LDS
    stage_table_to_lds(stl, a.st + blk.s0, T);
    bar();
    const StTab st{stl};
    const double* BAbt = a.BAbt + (long)p * a.sB;
    const double* RSQ = a.RSQ + (long)p * a.sR;
    const double* dv = a.d + (long)p * a.sD;
    const int* idxb = a.idxb;
    double* G = a.G + (long)p * a.sG + blk.oG;
    double* B2 = a.BAbt2 + (long)p * a.sB2 + blk.oB2;
    double* R2 = a.RSQ2 + (long)p * a.sR2 + blk.oR2;
    double* G2 = a.DCt2 + (long)p * a.sG2 + blk.oG2;
    double* d2 = a.d2 + (long)p * a.sD2 + blk.oD2;
    double* Pl = sm + a.offP;  // pL (RSQrq_s + W W', a lib4 block in the layout of its stage)
    double* X = sm + a.offX;   // Lx / chol scratch (ld ldX)
    double* Bt = sm + a.offB;  // stage BAbt tile, then W in place (ld ldB)
    double* Ucol = sm + a.offU;  // P form: the u columns of pL_s (x rows and gradient row), ld ldU
    const int ldU = a.ldX;
    const int ldX = a.ldX, ldB = a.ldB;

    // Gamma row counts / offsets (rows r_j = sum_{i<=j} nu_i + nx0 + 1)
    auto rows = [&](int j) {
        int acc = nx0 + 1;
        for (int i = 0; i <= j; i++) acc += st[i].nu;
        return acc;
    };
    auto goff = [&](int j) {
        int o = 0, acc = nx0 + 1;
        for (int i = 0; i < j; i++) {
            acc += st[i].nu;
            o += acc * st[i].nx1;
        }
        return o;
    };

    // ---- d_cond_BAbt: Gamma_{j-1} stays in LDS (GA); Gamma_j = [B_j; Gamma_{j-1} A_j] comes from MFMA tiles
    // held in registers, then overwrites GA and streams to HBM ----
    double* GA = sm + a.offGA;
    const int ph = a.ph;
    // Deferred cross terms (full condensing only): d_cond_RSQrq runs first and leaves, per stage s, the operand of its
    // cross term M_s = Gamma_{s-1} pL_s[x, u] (the (nx_s + 1) x nu_s u columns of pL_s: x rows and gradient row) in the
    // scratch; d_cond_BAbt runs second and forms M_s, and the general constraints of stage s (d_cond_DCtd), while
    // Gamma_{s-1} is in LDS.  No Gamma goes through HBM (the scratch carries ~(nx + 1) nu doubles per stage instead of
    // a Gamma of (sum nu + nx + 1) x nx), and every value is formed by the same operations on the same operands.
    const bool dm = ph == PC_ALL && a.dm;
    int* I = reinterpret_cast<int*>(sm);  // d_cond_DCtd's bookkeeping (the LDS tiles are free when it runs)
    int *cU = I, *cX = I + T, *iob = I + 2 * T, *iog = I + 3 * T, *ntmp = I + 4 * T, *igb = I + 5 * T;
    int* gd = I + 6 * T;  // general constraint ig: (stage << 16) | state index g
    int* gj = gd + blk.ng2;  // ... and its box index in the stage (dm)
    auto soff = [&](int sI) {  // dm: stage sI's cross-term operand in the scratch, (nx + 1) x nu, ld nx + 1
        int o = 0;
        for (int r = 1; r < sI; r++) o += (st[r].nx + 1) * st[r].nu;
        return o;
    };
    // dm: stage s's cross term from Gamma_{s-1} (in GA, leading dimension r0 = rows(s-1)) and the general constraints
    // of its state boxes (DCt2 columns and the bounds' constant terms), as d_cond_RSQrq's M_product and d_cond_DCtd
    // form them from the scratch Gammas
    auto dm_stage = [&](int sI, int r0) __attribute__((always_inline)) {
        const WideStage q = st[sI];
        const int nus = q.nu, nxs = q.nx, ldS = nxs + 1;
        const double* Ss = G + soff(sI);
        for (int e = tid; e < ldS * nus; e += WT) Ucol[e] = Ss[e];
        lds_bar();
        const int os = ntmp[sI] - nus;
        const float rr0 = 1.0f / r0;
        for (int e = tid; e < ((a.skip & 8) ? 0 : r0 * nus); e += WT) {
            const int c = fdiv(e, rr0), i = e - c * r0;
            double acc = 0.0;
            for (int l = 0; l < nxs; l++) acc += GA[i + l * r0] * Ucol[l + c * ldS];
            if (i == r0 - 1) acc += Ucol[nxs + c * ldS];
            *P4w(R2, (nv + 1) / 2 * 2, os + nus + i, os + c) = acc;
        }
        const int nbb = blk.nb2, nbg = blk.ng2, pnbb = (nbb + 3) / 4 * 4, pnbg = (nbg + 3) / 4 * 4;
        const int cnbg = (nbg + 1) / 2 * 2, rowsI = igb[sI], nt = ntmp[sI];
        const int wv = tid >> 6, ln = tid & 63;
        for (int ig = iog[sI] + wv; ig < iog[sI] + cX[sI]; ig += WT / 64) {
            const int g = gd[ig] & 0xffff, jj = gj[ig];
            for (int i = ln; i < rowsI; i += 64) *P4w(G2, cnbg, nt + i, ig) = GA[i + g * r0];
            if (ln == 0) {
                const double c0 = GA[rowsI + g * r0];
                d2[2 * pnbb + ig] = dv[q.oD + jj] - c0;
                d2[2 * pnbb + pnbg + ig] = dv[q.oD + q.pnb + jj] - c0;
            }
        }
    };
    PST_DECL;
    PST(0);
    auto babt_phase = [&]() __attribute__((always_inline)) {
    {
        const WideStage s = st[0];
        const int r0 = s.nu + s.nx + 1;
        load_dense<8>(GA, r0, BAbt + s.oB, s.sdB, r0, s.nx1);
        lds_bar();
        if (!dm && (T > 1 || (ph & PC_PART)))
            for (int e = tid; e < r0 * s.nx1; e += WT) G[e] = GA[e];
        if (dm && T > 1) dm_stage(1, r0);
    }
    // BAbt_{j+1} is loaded into registers while Gamma_j is formed (Staged), and stored into LDS at the top of the
    // next step: one memory round trip per block instead of one per stage
    Staged<4> nb;
    bool staged = false;
    int rp = st[0].nu + nx0 + 1, go = rp * st[0].nx1;  // rows(j - 1) and goff(j), carried along the loop
    for (int j = 1; j < ((a.skip & 1) ? 1 : T); j++) {
        const WideStage s = st[j];
        const int nuj = s.nu, nxj = s.nx, nx1 = s.nx1, nzj = nuj + nxj + 1;
        const int rj = rp + nuj, n = rj * nx1;
        double* Gj = G + go;
        // the later phases read Gamma_0 .. Gamma_{T-2}; Gamma_{T-1} only goes to B2 (d_cond_BAbt alone returns all)
        const bool keep = !dm && (j < T - 1 || (ph & PC_PART));
        PST(1);
        if (staged)
            put_dense(nb, Bt, ldB);
        else
            load_dense<8>(Bt, ldB, BAbt + s.oB, s.sdB, nzj, nx1);
        lds_bar();
        PST(2);
        staged = false;
        if (j + 1 < ((a.skip & 1) ? 1 : T)) {
            const WideStage sn = st[j + 1];
            const int nzn = sn.nu + sn.nx + 1;
            if (nzn * sn.nx1 <= 4 * WT) {  // uniform
                pre_dense(nb, BAbt + sn.oB, sn.sdB, nzn, sn.nx1);
                staged = true;
            }
        }
        PST(11);
        // rows nuj.. : Gamma_{j-1} A_j (+ b_j on the last row) on MFMA; rows ..nuj: B_j.  The results overwrite
        // GA (leading dimension rp -> rj) after mfma_gemm's barrier, when every operand read is done.
        {
            auto fa = [&](int i, int l) { return GA[i + l * rp]; };
            auto fb = [&](int l, int c) { return Bt[nuj + l + c * ldB]; };
            auto fo = [&](int i, int c, double v) {
                if (i == rp - 1) v += Bt[nuj + nxj + c * ldB];
                GA[nuj + i + c * rj] = v;
                if (keep) Gj[nuj + i + c * rj] = v;
            };
            if (nxj <= 32)  // uniform: all K chunks unrolled
                mfma_gemm<GM, 8>(rp, nx1, nxj, fa, fb, fo);
            else
                mfma_gemm<GM, 0>(rp, nx1, nxj, fa, fb, fo);
        }
        const float rnu = 1.0f / nuj;
        PST(12);
        for (int e = tid; e < nuj * nx1; e += WT) {
            const int c = fdiv(e, rnu), i = e - c * nuj;
            GA[i + c * rj] = Bt[i + c * ldB];
            if (keep) Gj[i + c * rj] = Bt[i + c * ldB];
        }
        (void)n;
        lds_bar();
        PST(3);
        if (dm && j + 1 < T) dm_stage(j + 1, rj);
        rp = rj;
        go += rj * nx1;
    }
    {
        const int rT = rp, nxT = st[T - 1].nx1;  // rows(T - 1)
        const int sd = (nxT + 1) / 2 * 2;
        const float rrT = 1.0f / rT;
        for (int e = tid; e < rT * nxT; e += WT) {
            const int c = fdiv(e, rrT), i = e - c * rT;
            *P4w(B2, sd, i, c) = GA[i + c * rT];
        }
    }
    };  // babt_phase
    if ((ph & PC_BABT) && !dm) babt_phase();
    bar();  // Gamma scratch complete (written by this block's threads) before the later phases read it
    PST(4);

    // ---- d_cond_RSQrq ----
    const int cnux2 = (nv + 1) / 2 * 2;
    if (ph & PC_RSQ) {
    if (!(ph & PC_PART)) {
        // zeros only where the recursion below writes nothing: the strict upper triangle and the padding (every
        // entry i >= j, i <= nv, j < nv is stored exactly once by the D / M / final blocks)
        const int npan = (nv + 1 + 3) / 4, pan = 4 * cnux2;  // lib4 panels of 4 rows x cnux2 columns
        for (int pb = 0; pb < npan; pb++)
            for (int q = tid; q < pan; q += WT) {
                const int i = 4 * pb + (q & 3), j = q >> 2;
                if (i < j || i > nv || j >= nv) R2[pb * pan + q] = 0.0;
            }
    }
    bar();
    if (T == 1) {
        const WideStage s = st[0];
        const int nux = s.nu + s.nx;
        for (int j = tid >> 6; j < nux; j += WT / 64)
            for (int i = j + (tid & 63); i <= nux; i += 64) *P4w(R2, cnux2, i, j) = P4(RSQ + s.oR, s.sdR, i, j);
    } else {
        // pL (RSQrq_s + W W'), BAbt_{s-1} (then W) and Gamma_{s-1} sit in LDS in the layouts they have in memory:
        // pL and BAbt as lib4 panels (panel stride sd of their stage), Gamma flat.  Each arrives by an asynchronous
        // LDS DMA (dma_copy) issued as soon as its buffer is free: Gamma_{s-2} and RSQrq_{s-1} when the Cholesky and
        // M are done, BAbt_{s-2} when the step's gemms are done, so the round trips overlap the work in between.
        auto PL = [&](int sd, int i, int j) -> double& { return Pl[p4i(i, j, sd)]; };
        auto BT = [&](int sd, int i, int j) -> double& { return Bt[p4i(i, j, sd)]; };
        auto lib4n = [&](const WideStage& q, int sd) { return (q.nu + q.nx + 1 + 3) / 4 * 4 * sd; };
        // The clamp certificate of the state-block Cholesky (the reference clamps a pivot
        // d <= 1e-15 to 0, kernel_dpotrf_c99_lib4.c:555-640): X = pL_s[x,x] = RSQrq_s[x,x] + (W W')[x,x] >= RSQrq_s[x,x],
        // so every exact pivot of X is at least g_s = the Gershgorin bound of RSQrq_s[x,x] (from the data), and the
        // reference's computed pivots (exact pivots of X + dX, |dX_ij| <= c n eps max_i X_ii) stay above the clamp when
        // g_s - 1e-11 max_i X_ii > 1e-15.  Then L L' = X (to rounding) and d_cond_RSQrq's W W' = [BAbt | e] X^ [BAbt | e]'
        // with X^ the state block and its gradient row (P form): no Cholesky on the stage chain.  Otherwise the stage
        // takes the reference's route (Cholesky, W = BAbt L + l, W W').
        // g_s for every stage of the block, before the loop: one thread per (stage, row) forms the row's Gershgorin
        // value of RSQrq_s[x,x] from memory (eight loads in flight), GA holds them until the per-stage minimum
        // (GA is free between the d_cond_BAbt phase and the first Gamma copy below).
        double* gtab = sm + a.offGT;  // g_1 .. g_{T-1}
        const int nxw = a.ldX - 1;    // rows per stage in the scratch (the largest nx)
        if (a.pform) {
            for (int e = tid; e < (T - 1) * nxw; e += WT) {
                const int sg = 1 + e / nxw, i = e - (sg - 1) * nxw;
                const WideStage q = st[sg];
                double r = 1e300;
                if (i < q.nx) {
                    const double* R = RSQ + q.oR;
                    const double off = bdot(
                        q.nx,
                        [&](int j, bool ok) {
                            const int a1 = i > j ? i : j, a2 = i > j ? j : i;
                            return j == i ? 0.0 : fabs(gld(R, p4i(q.nu + a1, q.nu + a2, q.sdR), ok));
                        },
                        [&](int, bool) { return 1.0; });
                    r = gld(R, p4i(q.nu + i, q.nu + i, q.sdR)) - off;
                }
                GA[e] = r;
            }
            bar();
            for (int sg = 1 + tid; sg < T; sg += WT) {
                double g = 1e300;
                for (int i = 0; i < nxw; i++) g = fmin(g, GA[(sg - 1) * nxw + i]);
                gtab[sg] = g;
            }
            bar();
        }
        // Outstanding DMA at the top of step s: RSQrq_s -> pL and Gamma_{s-1} -> GA (issued after step s+1's Cholesky,
        // needed now), then BAbt_{s-1} -> Bt (issued at the end of step s+1, needed only after this step's Cholesky):
        // the top waits for all but the BAbt copy (nbk = its instruction count in this wave).
        int nbk;            // this wave's DMA instructions of the BAbt copy the next top may leave in flight
        bool bpend = true;  // workgroup-uniform: that copy may be in flight at the next top
        // carried along the loop: os = sum_{r > sI} nu_r (the offset of u_sI in the condensed variables),
        // r1 = rows(sI - 1), g1 = goff(sI - 1)
        int os = 0, r1 = rows(T - 2), g1 = goff(T - 2);
        {
            const WideStage s = st[T - 1], sp = st[T - 2];
            dma_copy<WT, 16>(Pl, RSQ + s.oR, lib4n(s, s.sdR), tid);
            if (!dm) dma_copy_any<WT>(GA, G + g1, r1 * s.nx, tid);
            nbk = dma_copy<WT, 16>(Bt, BAbt + sp.oB, lib4n(sp, sp.sdB), tid);
        }
        for (int sI = (a.skip & 2) ? 0 : T - 1;; sI--) {
            const WideStage s = st[sI];
            const int nus = s.nu, nxs = s.nx, nux = nus + nxs, sdP = s.sdR;
            dma_wait_keep(nbk);  // pL_s and Gamma_{s-1} have landed (this wave's part)
            lds_bar();
            if (sI == 0) {
                for (int j = tid >> 6; j < nux; j += WT / 64)
                    for (int i = j + (tid & 63); i <= nux; i += 64) *P4w(R2, cnux2, os + i, os + j) = PL(sdP, i, j);
                break;
            }
            // D: the u_s x u_s block
            for (int j = tid >> 6; j < nus; j += WT / 64)
                for (int i = j + (tid & 63); i < nus; i += 64) *P4w(R2, cnux2, os + i, os + j) = PL(sdP, i, j);
            const WideStage sp = st[sI - 1];
            const int nuxp = sp.nu + sp.nx, nzp = nuxp + 1;
            const int r0 = r1;
            const int r2 = r1 - sp.nu, g2 = sI >= 2 ? g1 - r2 * st[sI - 2].nx1 : 0;  // rows / goff(sI - 2)
            const int sdB = sp.sdB, sdQ = sp.sdR;
            // the stage gemms fit one 16x16 tile per wave and eight K chunks at nz, nx <= 32 (configs[4]: 31 x 24)
            const bool small = nzp <= 32 && nuxp <= 32 && nxs <= 32;  // uniform
            double emax = 0.0;  // max_i X_ii
            {
                const int i = tid & 63;
                emax = -hk::wave_min(i < nxs ? -PL(sdP, nus + i, nus + i) : 0.0);
            }
            // the P form's T = X^ [BAbt | e]' is (nx+1) x nz_{s-1}: one tile per wave covers it only with nx + 1 <= 32
            // (nx = 32 would need a third tile row: those stages take the Cholesky route)
            const bool pf = a.pform && small && nxs + 1 <= 32 && gtab[sI] - 1e-11 * emax > 1e-15;  // uniform
            auto M_product = [&](auto&& pxu, int t0, int nt) {  // M = Gamma_{s-1} pL_s[x,u] (+ the r row)
                const float rr0 = 1.0f / r0;
                for (int e = tid - t0; e < ((a.skip & 8) ? 0 : r0 * nus); e += nt) {
                    const int c = fdiv(e, rr0), i = e - c * r0;
                    double acc = 0.0;
                    for (int l = 0; l < nxs; l++) acc += GA[i + l * r0] * pxu(l, c);
                    if (i == r0 - 1) acc += pxu(nxs, c);
                    *P4w(R2, cnux2, os + nus + i, os + c) = acc;
                }
            };
            auto M_store = [&](auto&& pxu, int t0, int nt) {  // dm: the cross term's operand to the scratch
                double* Ss = G + soff(sI);
                for (int e = tid - t0; e < (nxs + 1) * nus; e += nt) {
                    const int c = e / (nxs + 1), l = e - c * (nxs + 1);
                    Ss[e] = pxu(l, c);
                }
            };
            PST(5);
            int ngm = 0;
            if (pf) {
                // ---- P form: T = X^ [BAbt | e]' ((nx+1) x nz_{s-1}, in the X tile, ld ldX), pL_{s-1} = RSQrq_{s-1} +
                // [BAbt | e] T (lower).  RSQrq_{s-1} arrives by LDS DMA while M is formed.
                if (bpend) {  // BAbt_{s-1} may still be in flight (the top left it): T needs it now
                    dma_wait();
                    lds_bar();
                }
                // the u columns of pL_s (x rows and the gradient row) for M, so pL's buffer is free after T
                for (int e = tid; e < (nxs + 1) * nus; e += WT) {
                    const int c = e / (nxs + 1), i = e - c * (nxs + 1);
                    Ucol[i + c * ldU] = PL(sdP, nus + i, c);
                }
                auto xh = [&](int i, int l) {  // X^[i][l], symmetric; the corner X^[nx][nx] is never used
                    const int a1 = i > l ? i : l, a2 = i > l ? l : i;
                    return PL(sdP, nus + a1, nus + a2);
                };
                // the e column's term X^[i][nx] of this wave's output tile (one tile per wave), read before the gemm's
                // barrier so that pL's buffer is free when the gemm returns
                double xr[4];
                {
                    const int nI2 = (nxs + 1 + 15) >> 4, t = __builtin_amdgcn_readfirstlane(tid >> 6), ti = t / nI2;
                    const int col = 16 * ti + (tid & 15), rb = 16 * (t - ti * nI2) + ((tid & 63) >> 4);
#pragma unroll
                    for (int r = 0; r < 4; r++) {
                        const int i = rb + 4 * r;
                        const double v = xh(nxs, i < nxs ? i : nxs - 1);
                        xr[r] = (col == nuxp && i < nxs) ? v : 0.0;
                    }
                }
                mfma_gemm<1, 8>(
                    nxs + 1, nzp, nxs, xh, [&](int l, int c) { return BT(sdB, c, l); },
                    [&](int i, int c, double v) { X[i + c * ldX] = v + xr[(i & 15) >> 2]; });
                PST(6);
                // every read of pL_s is done: RSQrq_{s-1} into its buffer
                dma_copy<WT, 16>(Pl, RSQ + sp.oR, lib4n(sp, sdQ), tid);
                if (dm)
                    M_store([&](int l, int c) { return Ucol[l + c * ldU]; }, 0, WT);
                else
                    M_product([&](int l, int c) { return Ucol[l + c * ldU]; }, 0, WT);
                dma_wait();
                lds_bar();  // M is done (GA free), RSQrq_{s-1} and T are in LDS
                PST(7);
                ngm = (sI >= 2 && !dm) ? dma_copy_any<WT>(GA, G + g2, r2 * sp.nx, tid) : 0;
                PST(13);
                mfma_gemm<1, 8>(
                    nzp, nuxp, nxs, [&](int i, int l) { return BT(sdB, i, l); },
                    [&](int l, int j) { return X[l + j * ldX]; },
                    [&](int i, int j, double v) {
                        if (i == nuxp) v += X[nxs + j * ldX];  // the e row of [BAbt | e]
                        if (i >= j) PL(sdQ, i, j) += v;
                    });
                lds_bar();  // BAbt_{s-1} and T are read
                PST(14);
                if (sI >= 2) {  // (register staging of this copy across the step measured the same: 1.567 ms)
                    const WideStage sq = st[sI - 2];
                    dma_copy<WT, 16>(Bt, BAbt + sq.oB, lib4n(sq, sq.sdB), tid);
                }
                nbk = 0;  // the next step's top waits for anything still in flight (a P-form step needs BAbt at once)
                bpend = false;
                PST(8);
            } else {
            const bool xt = nxs <= 28;  // uniform: the tile Cholesky reads pL directly
            if (!xt) {
                for (int j = tid >> 6; j < nxs; j += WT / 64)
                    for (int i = j + (tid & 63); i <= nxs; i += 64) X[i + j * ldX] = PL(sdP, nus + i, nus + j);
                lds_bar();
            }
            if (__builtin_amdgcn_readfirstlane(tid) < 64) {  // wave-uniform branch
                // Lx = chol_aug(pL_xx; pL_r) on wave 0 while the other three form M
                if (!(a.skip & 4)) {
                    if (xt)
                        xchol_tiles([&](int i, int j) { return PL(sdP, nus + i, nus + j); }, X, ldX, nxs);
                    else
                        xchol_rows(X, ldX, nxs);
                }
            } else {
                if (dm)
                    M_store([&](int l, int c) { return PL(sdP, nus + l, c); }, 64, WT - 64);
                else
                    M_product([&](int l, int c) { return PL(sdP, nus + l, c); }, 64, WT - 64);
            }
            dma_wait();  // BAbt_{s-1} has landed
            lds_bar();       // pL and GA are read until here
            // RSQrq_{s-1} into pL and Gamma_{s-2} into GA while W = BAbt_{s-1} Lx (+ l on the last row) forms in place
            // over BAbt_{s-1}; then pL += W W' (lower); both products on MFMA
            dma_copy<WT, 16>(Pl, RSQ + sp.oR, lib4n(sp, sp.sdR), tid);
            ngm = (sI >= 2 && !dm) ? dma_copy_any<WT>(GA, G + g2, r2 * sp.nx, tid) : 0;
            auto wa = [&](int i, int l) { return BT(sdB, i, l); };
            auto wb = [&](int l, int c) {
                const double v = X[l + c * ldX];
                return l >= c ? v : 0.0;
            };
            auto wo = [&](int i, int c, double v) {
                if (i == nuxp) v += X[nxs + c * ldX];
                BT(sdB, i, c) = v;
            };
            if (!(a.skip & 16)) {
                if (small)
                    mfma_gemm<1, 8>(nzp, nxs, nxs, wa, wb, wo);
                else
                    mfma_gemm<GM, 0>(nzp, nxs, nxs, wa, wb, wo);
            }
            dma_wait_keep(ngm);  // RSQrq_{s-1} has landed; Gamma_{s-2} may still be in flight
            lds_bar();
            auto pa = [&](int i, int l) { return BT(sdB, i, l); };
            auto pb = [&](int l, int j) { return BT(sdB, j, l); };
            auto po = [&](int i, int j, double v) {
                if (i >= j) PL(sdQ, i, j) += v;
            };
            if (!(a.skip & 16)) {
                if (small)
                    mfma_gemm<1, 8>(nzp, nuxp, nxs, pa, pb, po);
                else
                    mfma_gemm<GM, 0>(nzp, nuxp, nxs, pa, pb, po);
            }
            lds_bar();  // W is read
            nbk = 0;
            if (sI >= 2) {
                const WideStage sq = st[sI - 2];
                nbk = dma_copy<WT, 16>(Bt, BAbt + sq.oB, lib4n(sq, sq.sdB), tid);
            }
            bpend = true;
            }
            (void)ngm;
            os += nus;
            r1 = r2;
            g1 = g2;
            PST(9);
        }
    }
    }  // PC_RSQ

    // ---- d_cond_DCtd: input boxes stay boxes, state boxes of stages 1..T-1 become general constraints.  The
    // reference walks the stages backwards assigning box / general slots in order (:637-678); here each wave
    // takes whole stages and ranks its entries with ballots, after a per-stage count and a prefix over stages
    // (the LDS tiles are free by now and hold the integer bookkeeping), then the general constraints' Gamma
    // rows are copied one column per wave ----
    if (ph & PC_DCTD) {
        const int nbb = blk.nb2, nbg = blk.ng2, pnbb = (nbb + 3) / 4 * 4, pnbg = (nbg + 3) / 4 * 4;
        const int cnbg = (nbg + 1) / 2 * 2, pnv = (nv + 3) / 4 * 4;
        const int wv = tid >> 6, ln = tid & 63;
        const unsigned long long below = (1ull << ln) - 1ull;
        bar();                // the RSQ phase's last LDS reads are done
        if (!(ph & PC_PART))
            for (int e = tid; e < 2 * pnbb + 2 * pnbg; e += WT) d2[e] = 0.0;
        for (int sI = wv; sI < T; sI += WT / 64) {  // input / state box counts of each stage
            const WideStage s = st[sI];
            int nU = 0, nX = 0;
            for (int j0 = 0; j0 < s.nb; j0 += 64) {
                const int jj = j0 + ln;
                const int vv = jj < s.nb ? idxb[s.oI + jj] : -1;
                const unsigned long long mu = __ballot(jj < s.nb && vv < s.nu), mx = __ballot(jj < s.nb && vv >= s.nu);
                nU += __popcll(mu);
                nX += __popcll(mx);
            }
            if (ln == 0) {
                cU[sI] = nU;
                cX[sI] = nX;
            }
        }
        bar();
        if (tid == 0) {  // slots in the reference's order: stages T-1 .. 1, then all of stage 0's boxes
            int ib = 0, ig = 0, nt = 0;
            for (int sI = T - 1; sI >= 1; sI--) {
                nt += st[sI].nu;
                iob[sI] = ib;
                iog[sI] = ig;
                ntmp[sI] = nt;
                ib += cU[sI];
                ig += cX[sI];
            }
            iob[0] = ib;
            iog[0] = ig;
            ntmp[0] = nt + st[0].nu;
            int acc = nx0;  // idx_gammab of stage s: nx0 + sum_{j<s} nu_j (= rows(s-1) - 1)
            for (int sI = 0; sI < T; sI++) {
                igb[sI] = acc;
                acc += st[sI].nu;
            }
        }
        bar();
        int* i2 = p == 0 ? a.idxb2 + blk.oI2 : nullptr;
        for (int sI = wv; sI < T; sI += WT / 64) {
            const WideStage s = st[sI];
            const int r0 = sI > 0 ? igb[sI] + 1 : 0, gb = igb[sI];
            const double* Gp = (sI > 0 && !dm) ? G + goff(sI - 1) : nullptr;
            int rU = iob[sI], rX = iog[sI];
            for (int j0 = 0; j0 < s.nb; j0 += 64) {
                const int jj = j0 + ln;
                const bool in = jj < s.nb;
                const int vv = in ? idxb[s.oI + jj] : -1;
                const bool isb = in && (sI == 0 || vv < s.nu), isg = in && !isb;
                const unsigned long long mb = __ballot(isb), mg = __ballot(isg);
                if (isb) {
                    const int ib = rU + __popcll(mb & below);
                    d2[ib] = dv[s.oD + jj];
                    d2[pnbb + ib] = dv[s.oD + s.pnb + jj];
                    if (i2) i2[ib] = ntmp[sI] - s.nu + vv;
                }
                if (isg) {
                    const int ig = rX + __popcll(mg & below), g = vv - s.nu;
                    if (!dm) {  // dm: the bounds' constant terms come with Gamma_{s-1} (dm_stage)
                        const double c0 = Gp[gb + g * r0];
                        d2[2 * pnbb + ig] = dv[s.oD + jj] - c0;
                        d2[2 * pnbb + pnbg + ig] = dv[s.oD + s.pnb + jj] - c0;
                    }
                    gd[ig] = (sI << 16) | g;
                    gj[ig] = jj;
                }
                rU += __popcll(mb);
                rX += __popcll(mg);
            }
        }
        bar();
        const float rpan = 1.0f / (4 * cnbg);
        if (!(ph & PC_PART))  // DCt2 zeros only outside the rows the copy below writes
            for (int e = tid; e < pnv * cnbg; e += WT) {
                const int pq = fdiv(e, rpan), q = e - pq * (4 * cnbg), i = pq * 4 + (q & 3), ig = q >> 2;
                bool z = ig >= nbg;
                if (!z) {
                    const int sI = gd[ig] >> 16, nt = ntmp[sI];
                    z = i < nt || i >= nt + igb[sI];
                }
                if (z) G2[e] = 0.0;
            }
        for (int ig = wv; ig < (dm ? 0 : nbg); ig += WT / 64) {  // DCt2 column ig: rows nu_tmp + i <- Gamma_{s-1}(i, g)
            const int sI = gd[ig] >> 16, g = gd[ig] & 0xffff, rowsI = igb[sI], r0 = rowsI + 1, nt = ntmp[sI];
            const double* Gp = G + goff(sI - 1);
            for (int i = ln; i < rowsI; i += 64) *P4w(G2, cnbg, nt + i, ig) = Gp[i + g * r0];
        }
    }
    if (dm) {  // d_cond_BAbt last: Gamma_j in LDS forms the cross terms and general constraints of stage j + 1
        bar();  // the bookkeeping and the cross-term operands in the scratch are complete
        babt_phase();
    }
    PST(10);
    // the terminal condensed stage is the original's (d_part_cond.c:1052-1056): block N2-1 copies it
    if (ii == a.N2 - 1 && !(ph & PC_PART)) {
        const WideStage sN = a.st[a.N];
        const int n = (a.nzN + 3) / 4 * 4 * a.sdRN;
        double* RN = a.RSQ2 + (long)p * a.sR2 + a.oR2N;
        for (int e = tid; e < n; e += WT) RN[e] = RSQ[sN.oR + e];
        double* dN = a.d2 + (long)p * a.sD2 + a.oD2N;  // and its bounds (the IPM on the condensed problem reads them)
        for (int e = tid; e < a.nDN; e += WT) dN[e] = dv[sN.oD + e];
    }
    PST_FLUSH();
}

// ------------------------------------------------------------------------------------------------
// Expansion of the condensed solution (d_part_expand_solution), one workgroup per (block, problem):
// the blocks are independent (each starts from its own x_0 and ends at the condensed pi).
// ------------------------------------------------------------------------------------------------
__global__ __launch_bounds__(WT) void hk_pexpand(PxArgs a) {
    extern __shared__ double sm[];
    const int ii = blockIdx.x, p = blockIdx.y + a.p0;
    if (p >= a.nprob || ii >= a.N2) return;
    const int tid = threadIdx.x;
    const WideStage* st = a.st;
    const WideStage* st2 = a.st2;
    const PcBlock blk = a.blk[ii];
    const int T = blk.T, s0 = blk.s0;
    const double* BAbt = a.BAbt + (long)p * a.sB;
    const double* RSQ = a.RSQ + (long)p * a.sR;
    const double* u2 = a.ux2 + (long)p * a.sU2 + st2[ii].oU;
    const double* lam2 = a.lam2 + (long)p * a.sC2;
    const double* t2 = a.t2 + (long)p * a.sC2;
    double* ux = a.ux + (long)p * a.sU;
    double* pi = a.pi + (long)p * a.sP;
    double* lam = a.lam + (long)p * a.sC;
    double* t = a.t + (long)p * a.sC;
    const double* hb = a.hb ? a.hb + (long)p * a.sP : nullptr;
    const double* hrq = a.hrq ? a.hrq + (long)p * a.sU : nullptr;
    const int ld = a.ldT;
    double* Bt = sm + a.offB;  // BAbt_j tile (ld x nxM)
    double* Rt = sm + a.offR;  // RSQrq_j tile (ld x ld)
    double* vu = sm + a.offV;  // ux_j (ld)
    double* w = sm + a.offW;   // box terms (ld)
    double* vp = sm + a.offQ;  // pi_j (ld)

    // u of the block's later stages come first in the condensed vector (reverse order), then u_0, x_0
    auto upos = [&](int j) {  // position of u_{s0+j} in u2
        int o = 0;
        for (int r = T - 1; r > j; r--) o += st[s0 + r].nu;
        return o;
    };
    // stage s0: u and x straight from u2
    {
        const WideStage s = st[s0];
        const int o = upos(0);
        for (int l = tid; l < s.nu + s.nx; l += WT) {
            const double x = u2[o + l];
            vu[l] = x;
            ux[s.oU + l] = x;
        }
    }
    if (ii == a.N2 - 1) {  // the final state, and stage N's multipliers (box and general slots)
        const WideStage sN = st[a.N], c = st2[a.N2];
        for (int l = tid; l < sN.nx; l += WT) ux[sN.oU + l] = a.ux2[(long)p * a.sU2 + c.oU + l];
        if (tid == 0) {
            const int png = (sN.ng + 3) / 4 * 4, png2 = (c.ng + 3) / 4 * 4;
            for (int j = 0; j < sN.nb; j++) {
                lam[sN.oD + j] = lam2[c.oD + j];
                lam[sN.oD + sN.pnb + j] = lam2[c.oD + c.pnb + j];
                t[sN.oD + j] = t2[c.oD + j];
                t[sN.oD + sN.pnb + j] = t2[c.oD + c.pnb + j];
            }
            for (int j = 0; j < sN.ng; j++) {
                lam[sN.oD + 2 * sN.pnb + j] = lam2[c.oD + 2 * c.pnb + j];
                lam[sN.oD + 2 * sN.pnb + png + j] = lam2[c.oD + 2 * c.pnb + png2 + j];
                t[sN.oD + 2 * sN.pnb + j] = t2[c.oD + 2 * c.pnb + j];
                t[sN.oD + 2 * sN.pnb + png + j] = t2[c.oD + 2 * c.pnb + png2 + j];
            }
        }
    }
    if (tid == 0) {  // slacks and multipliers of the block's stages (the slot order is a prefix scan)
        const int pnb2 = st2[ii].pnb, png2 = (st2[ii].ng + 3) / 4 * 4, o2 = st2[ii].oD;
        int nbb2_tmp = 0, nbg2_tmp = 0;
        for (int jj = 0; jj < T - 1; jj++) {
            const WideStage s = st[s0 + T - 1 - jj];
            int nbb2 = 0, nbg2 = 0;
            for (int l = 0; l < s.nb; l++) {
                if (a.idxb[s.oI + l] < s.nu)
                    nbb2++;
                else
                    nbg2++;
            }
            for (int l = 0; l < nbb2; l++) {
                lam[s.oD + l] = lam2[o2 + nbb2_tmp + l];
                lam[s.oD + s.pnb + l] = lam2[o2 + pnb2 + nbb2_tmp + l];
                t[s.oD + l] = t2[o2 + nbb2_tmp + l];
                t[s.oD + s.pnb + l] = t2[o2 + pnb2 + nbb2_tmp + l];
            }
            for (int l = 0; l < nbg2; l++) {
                lam[s.oD + nbb2 + l] = lam2[o2 + 2 * pnb2 + nbg2_tmp + l];
                lam[s.oD + s.pnb + nbb2 + l] = lam2[o2 + 2 * pnb2 + png2 + nbg2_tmp + l];
                t[s.oD + nbb2 + l] = t2[o2 + 2 * pnb2 + nbg2_tmp + l];
                t[s.oD + s.pnb + nbb2 + l] = t2[o2 + 2 * pnb2 + png2 + nbg2_tmp + l];
            }
            nbb2_tmp += nbb2;
            nbg2_tmp += nbg2;
        }
        const WideStage s = st[s0];
        for (int l = 0; l < s.nb; l++) {
            lam[s.oD + l] = lam2[o2 + nbb2_tmp + l];
            lam[s.oD + s.pnb + l] = lam2[o2 + pnb2 + nbb2_tmp + l];
            t[s.oD + l] = t2[o2 + nbb2_tmp + l];
            t[s.oD + s.pnb + l] = t2[o2 + pnb2 + nbb2_tmp + l];
        }
    }
    // states inside the block by simulation, x_{j+1} = b_j + BAbt_j' ux_j; u_{j+1} from u2
    for (int jj = 0; jj < T - 1; jj++) {
        const WideStage s = st[s0 + jj], s1 = st[s0 + jj + 1];
        const int nux = s.nu + s.nx;
        load_dense<4>(Bt, ld, BAbt + s.oB, s.sdB, nux + 1, s.nx1);
        bar();
        double xn = 0.0;
        if (tid < s.nx1) {
            double acc = 0.0;
            for (int i = 0; i < nux; i++) acc += Bt[i + tid * ld] * vu[i];
            xn = (hb ? hb[s.oP + tid] : Bt[nux + tid * ld]) + acc;
        }
        bar();
        const int o = upos(jj + 1);
        for (int l = tid; l < s1.nu; l += WT) {
            const double x = u2[o + l];
            vu[l] = x;
            ux[s1.oU + l] = x;
        }
        if (tid < s.nx1) {
            vu[s1.nu + tid] = xn;
            ux[s1.oU + s1.nu + tid] = xn;
        }
    }
    bar();
    // equality multipliers: the block's last pi is the condensed one; inner ones by the backward
    // stationarity recursion pi_{s-1} = [rq_s + box terms + RSQ_s ux_s + BAbt_s pi_s]_x
    {
        const WideStage sl = st[s0 + T - 1];
        const double* p2 = a.pi2 + (long)p * a.sP2 + st2[ii].oP;
        for (int l = tid; l < sl.nx1; l += WT) {
            const double x = p2[l];
            vp[l] = x;
            pi[sl.oP + l] = x;
        }
    }
    for (int jj = 0; jj < T - 1; jj++) {
        const int sI = s0 + T - 1 - jj;
        const WideStage s = st[sI], sm1 = st[sI - 1];
        const int nux = s.nu + s.nx;
        load_dense<4>(Bt, ld, BAbt + s.oB, s.sdB, nux, s.nx1);
        load_dense<4>(Rt, ld, RSQ + s.oR, s.sdR, nux + 1, nux);
        load_flat<2>(vu, ux + s.oU, nux);
        for (int l = tid; l < nux; l += WT) w[l] = 0.0;
        bar();
        if (tid == 0)
            for (int l = 0; l < s.nb; l++) w[a.idxb[s.oI + l]] += -lam[s.oD + l] + lam[s.oD + s.pnb + l];
        bar();
        double acc = 0.0;
        if (tid < s.nx) {
            const int i = s.nu + tid;
            acc = hrq ? hrq[s.oU + i] : Rt[nux + i * ld];
            acc += w[i];
            double sy = 0.0;
            for (int j = 0; j < nux; j++) sy += (i >= j ? Rt[i + j * ld] : Rt[j + i * ld]) * vu[j];
            acc += sy;
            double sg = 0.0;
            for (int j = 0; j < s.nx1; j++) sg += Bt[i + j * ld] * vp[j];
            acc += sg;
        }
        bar();
        if (tid < s.nx) {
            vp[tid] = acc;
            pi[sm1.oP + tid] = acc;
        }
    }
}

// d_back_ric_rec_trs_tv_res on wide stages (wide_trs_body, hk_wide_core.h)
__global__ __launch_bounds__(WT) void hk_wide_trs(WideArgs a) {
    const int p = blockIdx.x + a.p0;
    if (p >= a.nprob) return;
    wide_stage_table(a);
    wide_trs_body(a, wide_prob(a, p));
}

// ------------------------------------------------------------------------------------------------
// Host launchers
// ------------------------------------------------------------------------------------------------
extern "C" int hk_wide_launch(int which, const void* args, int count, int lds_doubles, hipStream_t stream) {
    if (count <= 0) return 0;
    const size_t lds = (size_t)lds_doubles * sizeof(double);
    switch (which) {
        case 0: {
            const WideArgs& a = *static_cast<const WideArgs*>(args);
            hipLaunchKernelGGL(hk_wide_sv, dim3(count), dim3(WT), lds, stream, a);
            break;
        }
        case 1: {
            const PcArgs& a = *static_cast<const PcArgs*>(args);
            if (a.gm <= 4)
                hipLaunchKernelGGL(hk_pcond<4>, dim3(a.N2, count), dim3(WT), lds, stream, a);
            else
                hipLaunchKernelGGL(hk_pcond<8>, dim3(a.N2, count), dim3(WT), lds, stream, a);
            break;
        }
        case 2: {
            const PxArgs& a = *static_cast<const PxArgs*>(args);
            hipLaunchKernelGGL(hk_pexpand, dim3(a.N2, count), dim3(WT), lds, stream, a);
            break;
        }
        case 3: {
            const WideArgs& a = *static_cast<const WideArgs*>(args);
            hipLaunchKernelGGL(hk_wide_trs, dim3(count), dim3(WT), lds, stream, a);
            break;
        }
        default:
            return -1;
    }
    return (int)hipGetLastError();
}
