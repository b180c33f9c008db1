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

#include "hk_prims.h"
#include "hk_wide_args.h"

namespace {

using hk::gld;

constexpr int WT = 256;  // threads per workgroup
constexpr int WS_TILES = 8;  // W = BAbt Lxx output tiles per wave (nz <= 128, nx <= 64: <= 32 tiles, host-checked)
constexpr int BS = 4;

__device__ __forceinline__ int p4i(int i, int j, int sd) { return (i / BS) * BS * sd + i % BS + BS * j; }

__device__ __forceinline__ double P4(const double* A, int sd, int i, int j) {
    return A[(i / BS) * BS * sd + i % BS + BS * j];
}
__device__ __forceinline__ double* P4w(double* A, int sd, int i, int j) {
    return A + (i / BS) * BS * sd + i % BS + BS * j;
}
// packed lower columns of an nz-row matrix: column j holds rows j..nz-1
__device__ __forceinline__ int poff(int j, int nz) { return j * nz - (j * (j - 1)) / 2; }

__device__ __forceinline__ void bar() { __syncthreads(); }

// Global -> LDS staging with CH loads in flight per lane: every load of a batch is issued before the first
// LDS store (raw buffer loads, masked lanes read out of range), so a stage tile costs one or two memory
// round trips instead of one per element.
template <int CH>
__device__ void load_flat(double* D, const double* src, int n) {
    const int tid = threadIdx.x;
    for (int base = 0; base < n; base += WT * CH) {
        double r[CH];
#pragma unroll
        for (int u = 0; u < CH; u++) r[u] = gld(src, base + u * WT + tid, base + u * WT + tid < n);
#pragma unroll
        for (int u = 0; u < CH; u++)
            if (base + u * WT + tid < n) D[base + u * WT + tid] = r[u];
    }
}
// lib4 block rows [0, nr) x cols [0, nc) -> dense column-major (ld)
template <int CH>
__device__ void load_dense(double* D, int ld, const double* src, int sd, int nr, int nc) {
    const int tid = threadIdx.x, n = nr * nc;
    for (int base = 0; base < n; base += WT * CH) {
        double r[CH];
#pragma unroll
        for (int u = 0; u < CH; u++) {
            const int e = base + u * WT + tid, i = e % nr, c = e / nr;
            r[u] = gld(src, p4i(i, c, sd), e < n);
        }
#pragma unroll
        for (int u = 0; u < CH; u++) {
            const int e = base + u * WT + tid, i = e % nr, c = e / nr;
            if (e < n) D[i + c * ld] = r[u];
        }
    }
}
// lib4 lower trapezoid rows [j, nz) of cols [0, nc) -> packed lower columns (nz <= 128: two rows per lane)
template <int CU>
__device__ void load_lower(double* M, const double* src, int sd, int nz, int nc) {
    const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
    for (int j0 = w; j0 < nc; j0 += 4 * CU) {
        double r[CU][2];
#pragma unroll
        for (int u = 0; u < CU; u++)
#pragma unroll
            for (int h = 0; h < 2; h++) {
                const int j = j0 + 4 * u, i = j + l + 64 * h;
                r[u][h] = gld(src, p4i(i, j, sd), j < nc && i < nz);
            }
#pragma unroll
        for (int u = 0; u < CU; u++)
#pragma unroll
            for (int h = 0; h < 2; h++) {
                const int j = j0 + 4 * u, i = j + l + 64 * h;
                if (j < nc && i < nz) M[poff(j, nz) + i - j] = r[u][h];
            }
    }
}
// broadcast lane l's double (l wave-uniform) through SGPRs
__device__ __forceinline__ double rdlane(double v, int l) {
    const int lo = __builtin_amdgcn_readlane(__double2loint(v), l);
    const int hi = __builtin_amdgcn_readlane(__double2hiint(v), l);
    return __hiloint2double(hi, lo);
}

// In-wave ordering of LDS traffic between lanes (single-wave phases need no workgroup barrier): wait for this
// wave's LDS operations only (a release fence would also drain its outstanding global stores).
__device__ __forceinline__ void wave_sync() {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_wave_barrier();
}

// C (m x n) = A (m x K) B (K x n) on v_mfma_f64_16x16x4: wave w takes output tiles w, w+4, ..; a(i, k) / b(k, j)
// read the operands (0 outside), out(i, j, v) stores a result after a workgroup barrier, so C may overwrite
// an operand.  All threads of the workgroup must call it.  At most 4 * GM_TILES output tiles.
constexpr int GM_TILES = 8;
template <class FA, class FB, class FO>
__device__ __forceinline__ void mfma_gemm(int m, int n, int K, FA a, FB b, FO out) {
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6, c16 = lane & 15, g4 = lane >> 4;
    const int nI = (m + 15) >> 4, nT = nI * ((n + 15) >> 4), nK = (K + 3) >> 2;
    hk::d4 acc[GM_TILES];
#pragma unroll
    for (int u = 0; u < GM_TILES; u++) {
        acc[u] = hk::d4{0.0, 0.0, 0.0, 0.0};
        const int t = wv + 4 * u;
        if (t < nT) {
            const int ra = 16 * (t % nI) + c16, cb = 16 * (t / nI) + c16;
            for (int kc = 0; kc < nK; kc++) {
                const int kk = 4 * kc + g4;
                const double av = (ra < m && kk < K) ? a(ra, kk) : 0.0;
                const double bv = (cb < n && kk < K) ? b(kk, cb) : 0.0;
                acc[u] = hk::mfma(av, bv, acc[u]);
            }
        }
    }
    __syncthreads();
#pragma unroll
    for (int u = 0; u < GM_TILES; u++) {
        const int t = wv + 4 * u;
        if (t < nT) {
            const int col = 16 * (t / nI) + c16;
#pragma unroll
            for (int r = 0; r < 4; r++) {
                const int row = 16 * (t % nI) + g4 + 4 * r;
                if (row < m && col < n) out(row, col, acc[u][r]);
            }
        }
    }
}

}  // namespace

// ------------------------------------------------------------------------------------------------
// Riccati factorisation + solve on wide stages (d_back_ric_rec_sv_tv_res, no box / general terms:
// the host applies the box terms to the staged RSQrq copies, as the reference does in place).
// Per stage k = N..0 (d_back_ric_rec.c:186-335):
//   W = BAbt_k Lxx_{k+1} (dtrmm_nt_u), Pb = Lxx (W_last)', W_last += l_{k+1,x} (dgead),
//   M = RSQrq_k + W W' (dsyrk), L_k = chol_aug(M) with the pivot clamp d > 1e-15 else 0
//   (kernel_dpotrf_c99_lib4.c:555-640): right-looking, one barrier per column; the scaled column goes
//   straight to the factor in HBM (and, for the state block, to LDS as Lxx for stage k-1).
// Forward (:339-397): ux_k = -L_k^{-T}(l_k ...) over the u block (the whole block at k = 0),
//   x_{k+1} = b_k + BAbt_k' ux_k (dgemv_t), pi_k = Lxx_{k+1}(Lxx_{k+1}' x_{k+1} + l_{k+1,x}).
// ------------------------------------------------------------------------------------------------
__global__ __launch_bounds__(WT) void hk_wide_sv(WideArgs a) {
    extern __shared__ double sm[];
    const int p = blockIdx.x + a.p0;
    if (p >= a.nprob) return;
    const int tid = threadIdx.x;
    double* M = sm;
    double* W = sm + a.offW;
    double* X = sm + a.offX;
    double* v = sm + a.offV;
    const int ldW = a.ldW, ldX = a.ldX;
    const int lane = tid & 63, wv = tid >> 6, c16 = lane & 15, g4 = lane >> 4;  // MFMA lane coordinates
    const double* BAbt = a.BAbt + (long)p * a.sB;
    const double* RSQ = a.RSQ + (long)p * a.sR;
    double* F = a.ws + (long)p * a.sW;
    double* ux = a.ux + (long)p * a.sU;
    double* pi = a.pi + (long)p * a.sP;
    double* Pb = a.Pb ? a.Pb + (long)p * a.sP : nullptr;

    for (int k = a.N; k >= 0; k--) {
        const WideStage s = a.st[k];
        const int nu = s.nu, nux = s.nu + s.nx, nz = nux + 1, nx1 = s.nx1;
        load_lower<4>(M, RSQ + s.oR, s.sdR, nz, nux);
        if (k < a.N && !(a.skip & 4)) {
            load_dense<8>(W, ldW, BAbt + s.oB, s.sdB, nz, nx1);
            bar();
            if (a.trf) {  // trf factorises without the augmented row: the b row and the gradient row read as 0
                for (int j = tid; j < nux + nx1; j += WT) {
                    if (j < nx1) W[nux + j * ldW] = 0.0;
                    if (j < nux) M[poff(j, nz) + nux - j] = 0.0;
                }
                bar();
            }
            // W = BAbt_k Lxx_{k+1} (dtrmm_nt_u) on MFMA: 16x16 output tiles, K over the nx1 columns of BAbt; the
            // tiles are kept in registers and written back over BAbt after a barrier
            {
                const int nI = (nz + 15) >> 4, nJ = (nx1 + 15) >> 4, nK = (nx1 + 3) >> 2;
                hk::d4 acc[WS_TILES];
#pragma unroll
                for (int u = 0; u < WS_TILES; u++) {
                    acc[u] = hk::d4{0.0, 0.0, 0.0, 0.0};
                    const int t = wv + 4 * u;
                    if (t < nI * nJ) {
                        const int I = t % nI, J = t / nI, ra = 16 * I + c16, cb = 16 * J + c16;
                        for (int kc = 0; kc < nK; kc++) {
                            const int kk = 4 * kc + g4;
                            const double av = (ra < nz && kk < nx1) ? W[ra + kk * ldW] : 0.0;
                            const double bv = (cb < nx1 && kk < nx1) ? X[kk + cb * ldX] : 0.0;
                            acc[u] = hk::mfma(av, bv, acc[u]);
                        }
                    }
                }
                bar();
#pragma unroll
                for (int u = 0; u < WS_TILES; u++) {
                    const int t = wv + 4 * u;
                    if (t < nI * nJ) {
                        const int I = t % nI, J = t / nI, col = 16 * J + c16;
#pragma unroll
                        for (int r = 0; r < 4; r++) {
                            const int row = 16 * I + g4 + 4 * r;
                            if (row < nz && col < nx1) W[row + col * ldW] = acc[u][r];
                        }
                    }
                }
            }
            bar();
            if (a.compute_Pb && tid < nx1) {  // Pb_k = Lxx (Lxx' b_k) from W's last row before + l
                double acc = 0.0;
                for (int j = 0; j <= tid; j++) acc += X[tid + j * ldX] * W[nux + j * ldW];
                Pb[s.oP + tid] = acc;
            }
            bar();
            if (tid < nx1) W[nux + tid * ldW] += X[nx1 + tid * ldX];
            bar();
            // M += W W' (dsyrk) on MFMA over the lower 16x16 tiles
            {
                const int nI = (nz + 15) >> 4, nK = (nx1 + 3) >> 2, nT = nI * (nI + 1) / 2;
                for (int t = wv; t < nT; t += 4) {
                    int I = 0;
                    while ((I + 1) * (I + 2) / 2 <= t) I++;
                    const int J = t - I * (I + 1) / 2;
                    const int ra = 16 * I + c16, rb = 16 * J + c16;
                    hk::d4 acc = {0.0, 0.0, 0.0, 0.0};
                    for (int kc = 0; kc < nK; kc++) {
                        const int kk = 4 * kc + g4;
                        const double av = (ra < nz && kk < nx1) ? W[ra + kk * ldW] : 0.0;
                        const double bv = (rb < nux && kk < nx1) ? W[rb + kk * ldW] : 0.0;
                        acc = hk::mfma(av, bv, acc);
                    }
                    const int col = 16 * J + c16;
#pragma unroll
                    for (int r = 0; r < 4; r++) {
                        const int row = 16 * I + g4 + 4 * r;
                        if (row < nz && col < nux && row >= col) M[poff(col, nz) + row - col] += acc[r];
                    }
                }
            }
        } else if (a.trf) {
            bar();
            for (int j = tid; j < nux; j += WT) M[poff(j, nz) + nux - j] = 0.0;
        }
        bar();
        // Cholesky with the augmented row, blocked by 16-column panels: wave 0 factors the panel (row i on
        // lanes i - j0 and i - j0 + 64, shuffles for the pivot row, no workgroup barrier), then all waves
        // apply the panel's rank-16 update to the trailing lower tiles on MFMA
        double* Lk = F + s.oL;
        double* dL = Lk + poff(nux, nz);
        for (int p0 = 0; p0 < ((a.skip & 2) ? 0 : nux); p0 += 16) {
            const int pe = p0 + 16 < nux ? p0 + 16 : nux;
            if (wv == 0) {
                // the panel (rows p0.., its <= 16 columns) in registers: lane L holds rows p0+L and p0+L+64
                const int pw = pe - p0, r0 = p0 + lane, r1 = r0 + 64;
                double c0[16], c1[16];
#pragma unroll
                for (int jj = 0; jj < 16; jj++) {
                    const int j = p0 + jj, cj = poff(j < nux ? j : 0, nz);
                    c0[jj] = (jj < pw && r0 >= j && r0 < nz) ? M[cj + r0 - j] : 0.0;
                    c1[jj] = (jj < pw && r1 < nz) ? M[cj + r1 - j] : 0.0;
                }
#pragma unroll
                for (int jj = 0; jj < 16; jj++) {
                    if (jj < pw) {
                        const double d = rdlane(c0[jj], jj);
                        double sq = 0.0, inv = 0.0;
                        if (d > 1e-15) {
                            sq = sqrt(d);
                            inv = 1.0 / sq;
                        }
                        c0[jj] = lane == jj ? sq : (lane > jj ? c0[jj] * inv : 0.0);
                        c1[jj] = c1[jj] * inv;
                        if (lane == 0) M[poff(nux, nz) + p0 + jj] = inv;
#pragma unroll
                        for (int cc = jj + 1; cc < 16; cc++) {
                            const double lc = rdlane(c0[jj], cc);
                            c0[cc] -= c0[jj] * lc;
                            c1[cc] -= c1[jj] * lc;
                        }
                    }
                }
#pragma unroll
                for (int jj = 0; jj < 16; jj++) {
                    const int j = p0 + jj;
                    if (jj < pw) {
                        const int cj = poff(j, nz);
                        if (r0 >= j && r0 < nz) {
                            M[cj + r0 - j] = c0[jj];
                            if (j >= nu) X[(r0 - nu) + (j - nu) * ldX] = c0[jj];
                        }
                        if (r1 < nz) {
                            M[cj + r1 - j] = c1[jj];
                            if (j >= nu) X[(r1 - nu) + (j - nu) * ldX] = c1[jj];
                        }
                    }
                }
            }
            bar();
            if (pe < nux) {  // trailing update: M[i, jj] -= sum_{k in panel} L[i, k] L[jj, k], tiles from pe
                const int T0 = pe >> 4, nI = (nz + 15) >> 4, nTI = nI - T0;
                const int nT = nTI * (nTI + 1) / 2, nK = (pe - p0 + 3) >> 2;
                for (int t = wv; t < nT; t += 4) {
                    int I = 0;
                    while ((I + 1) * (I + 2) / 2 <= t) I++;
                    const int J = t - I * (I + 1) / 2;
                    const int ra = 16 * (T0 + I) + c16, rb = 16 * (T0 + J) + c16;
                    hk::d4 acc = {0.0, 0.0, 0.0, 0.0};
                    for (int kc = 0; kc < nK; kc++) {
                        const int kk = p0 + 4 * kc + g4;
                        const bool kok = kk < pe;
                        const double av = (ra < nz && kok) ? M[poff(kk, nz) + ra - kk] : 0.0;
                        const double bv = (rb < nux && kok) ? M[poff(kk, nz) + rb - kk] : 0.0;
                        acc = hk::mfma(av, bv, acc);
                    }
                    const int col = 16 * (T0 + J) + c16;
#pragma unroll
                    for (int r = 0; r < 4; r++) {
                        const int row = 16 * (T0 + I) + g4 + 4 * r;
                        if (row < nz && col < nux && row >= col) M[poff(col, nz) + row - col] -= acc[r];
                    }
                }
                bar();
            }
        }
        // the factor (packed columns + 1/diag) to HBM in one coalesced sweep
        for (int e = tid; e < poff(nux, nz) + nux; e += WT) Lk[e] = M[e];
        (void)dL;
        // strictly upper part of the copied Lxx stays zero (the next stage's MFMA trmm reads whole tiles)
        for (int e = tid; e < s.nx * s.nx; e += WT) {
            const int i = e % s.nx, cc = e / s.nx;
            if (i < cc) X[i + cc * ldX] = 0.0;
        }
        bar();
    }

    // forward substitution: L_k (packed + 1/diag) and BAbt_k are staged into LDS (M, W) per stage
    double* tmp = X;  // Lxx is no longer needed: nx1 doubles of scratch for pi
    {
        const WideStage s0 = a.st[0];
        const int nz0 = s0.nu + s0.nx + 1;
        load_flat<16>(M, F + s0.oL, poff(nz0 - 1, nz0) + nz0 - 1);
    }
    for (int k = 0; k < ((a.skip & 1) || a.trf ? 0 : a.N); k++) {
        const WideStage s = a.st[k];
        const int nux = s.nu + s.nx, nz = nux + 1, nx1 = s.nx1, nu1 = s.nu1;
        const int ns = k == 0 ? nux : s.nu;
        const double* dL = M + poff(nux, nz);
        load_dense<8>(W, ldW, BAbt + s.oB, s.sdB, nz, nx1);
        bar();
        // v[0:ns] = -l[0:ns] - L[ns:nux, 0:ns]' v[ns:nux]   (v[ns:nux] = x_k from the previous stage)
        for (int j = tid; j < ns; j += WT) {
            const int cj = poff(j, nz) - j;
            double r = -M[cj + nux];
            for (int m = ns; m < nux; m++) r -= M[cj + m] * v[m];
            v[j] = r;
        }
        bar();
        // back substitution with L[0:ns, 0:ns]' (inv_diag multiply), column-oriented inside wave 0
        if (tid < 64) {
            for (int i = ns - 1; i >= 0; i--) {
                const double y = v[i] * dL[i];
                for (int j = tid; j < i; j += 64) v[j] -= M[poff(j, nz) + i - j] * y;
                if (tid == 0) v[i] = y;
                wave_sync();
            }
        }
        bar();
        for (int j = tid; j < nux; j += WT) ux[s.oU + j] = v[j];
        // x_{k+1} = b_k + BAbt_k' ux_k
        double xn = 0.0;
        if (tid < nx1) {
            xn = W[nux + tid * ldW];
            for (int i = 0; i < nux; i++) xn += W[i + tid * ldW] * v[i];
        }
        bar();
        const WideStage s1 = a.st[k + 1];
        const int nux1 = nu1 + nx1, nz1 = nux1 + 1;
        if (tid < nx1) {
            v[nu1 + tid] = xn;
            ux[s1.oU + nu1 + tid] = xn;
        }
        load_flat<16>(M, F + s1.oL, poff(nux1, nz1) + nux1);
        bar();
        if (a.compute_pi) {  // pi_k = Lxx (Lxx' x + l), Lxx of stage k+1 (rows / cols nu1..)
            if (tid < nx1) {
                const int cj = poff(nu1 + tid, nz1) - (nu1 + tid);
                double tj = M[cj + nux1];
                for (int i = tid; i < nx1; i++) tj += M[cj + nu1 + i] * v[nu1 + i];
                tmp[tid] = tj;
            }
            bar();
            if (tid < nx1) {
                double acc = 0.0;
                for (int j = 0; j <= tid; j++) acc += M[poff(nu1 + j, nz1) + tid - j] * tmp[j];
                pi[s.oP + tid] = acc;
            }
            bar();
        }
    }
}

// ------------------------------------------------------------------------------------------------
// Partial condensing of one block (d_cond_BAbt :214-303, d_cond_RSQrq :307-574, d_cond_DCtd :579-688).
// Condensed stage variables: [u_{T-1}; ...; u_0; x_0].  Gamma_j (rows [u_j..u_0, x_0, 1] x nx_{j+1},
// dense column-major) lives in the problem's scratch; the stage tiles (pL, Lx, BAbt, W) in LDS.
// ------------------------------------------------------------------------------------------------
__global__ __launch_bounds__(WT) void hk_pcond(PcArgs a) {
    extern __shared__ double sm[];
    const int ii = blockIdx.x, p = blockIdx.y + a.p0;
    if (p >= a.nprob || ii >= a.N2) return;
    const int tid = threadIdx.x;
    const PcBlock blk = a.blk[ii];
    const int T = blk.T, nx0 = blk.nx0, nv = blk.nut + nx0;
    const WideStage* st = a.st + blk.s0;
    const double* BAbt = a.BAbt + (long)p * a.sB;
    const double* RSQ = a.RSQ + (long)p * a.sR;
    const double* dv = a.d + (long)p * a.sD;
    const int* idxb = a.idxb;
    double* G = a.G + (long)p * a.sG + blk.oG;
    double* B2 = a.BAbt2 + (long)p * a.sB2 + blk.oB2;
    double* R2 = a.RSQ2 + (long)p * a.sR2 + blk.oR2;
    double* G2 = a.DCt2 + (long)p * a.sG2 + blk.oG2;
    double* d2 = a.d2 + (long)p * a.sD2 + blk.oD2;
    double* Pl = sm + a.offP;  // pL (dense, ld ldP)
    double* X = sm + a.offX;   // Lx / chol scratch (ld ldX)
    double* Bt = sm + a.offB;  // stage BAbt tile, then W in place (ld ldB)
    const int ldP = a.ldP, ldX = a.ldX, ldB = a.ldB;

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
    {
        const WideStage s = st[0];
        const int r0 = s.nu + s.nx + 1;
        load_dense<8>(GA, r0, BAbt + s.oB, s.sdB, r0, s.nx1);
        bar();
        for (int e = tid; e < r0 * s.nx1; e += WT) G[e] = GA[e];
    }
    for (int j = 1; j < ((a.skip & 1) ? 1 : T); j++) {
        const WideStage s = st[j];
        const int nuj = s.nu, nxj = s.nx, nx1 = s.nx1, nzj = nuj + nxj + 1;
        const int rp = rows(j - 1), rj = rp + nuj, n = rj * nx1;
        double* Gj = G + goff(j);
        load_dense<8>(Bt, ldB, BAbt + s.oB, s.sdB, nzj, nx1);
        bar();
        // rows nuj.. : Gamma_{j-1} A_j (+ b_j on the last row) on MFMA; rows ..nuj: B_j.  The results overwrite
        // GA (leading dimension rp -> rj) after mfma_gemm's barrier, when every operand read is done.
        mfma_gemm(
            rp, nx1, nxj, [&](int i, int l) { return GA[i + l * rp]; },
            [&](int l, int c) { return Bt[nuj + l + c * ldB]; },
            [&](int i, int c, double v) {
                if (i == rp - 1) v += Bt[nuj + nxj + c * ldB];
                GA[nuj + i + c * rj] = v;
                Gj[nuj + i + c * rj] = v;
            });
        for (int e = tid; e < nuj * nx1; e += WT) {
            const int i = e % nuj, c = e / nuj;
            GA[i + c * rj] = Bt[i + c * ldB];
            Gj[i + c * rj] = Bt[i + c * ldB];
        }
        (void)n;
        bar();
    }
    {
        const int rT = rows(T - 1), nxT = st[T - 1].nx1;
        const int sd = (nxT + 1) / 2 * 2;
        for (int e = tid; e < rT * nxT; e += WT) {
            const int i = e % rT, c = e / rT;
            *P4w(B2, sd, i, c) = GA[i + c * rT];
        }
    }

    // ---- d_cond_RSQrq ----
    const int cnux2 = (nv + 1) / 2 * 2;
    {
        const int n = ((nv + 1 + 3) / 4 * 4) * cnux2;
        for (int e = tid; e < n; e += WT) R2[e] = 0.0;
    }
    // offsets of u_s in the condensed variables: off(s) = sum_{r > s} nu_r
    auto uoff = [&](int s) {
        int o = 0;
        for (int r = s + 1; r < T; r++) o += st[r].nu;
        return o;
    };
    bar();
    if (T == 1) {
        const WideStage s = st[0];
        const int nux = s.nu + s.nx;
        for (int j = tid >> 6; j < nux; j += WT / 64)
            for (int i = j + (tid & 63); i <= nux; i += 64) *P4w(R2, cnux2, i, j) = P4(RSQ + s.oR, s.sdR, i, j);
    } else {
        {
            const WideStage s = st[T - 1];
            load_dense<8>(Pl, ldP, RSQ + s.oR, s.sdR, s.nu + s.nx + 1, s.nu + s.nx);
        }
        bar();
        for (int sI = (a.skip & 2) ? 0 : T - 1;; sI--) {
            const WideStage s = st[sI];
            const int nus = s.nu, nxs = s.nx, nux = nus + nxs, os = uoff(sI);
            if (sI == 0) {
                for (int j = tid >> 6; j < nux; j += WT / 64)
                    for (int i = j + (tid & 63); i <= nux; i += 64) *P4w(R2, cnux2, os + i, os + j) = Pl[i + j * ldP];
                break;
            }
            // D: the u_s x u_s block
            for (int j = tid >> 6; j < nus; j += WT / 64)
                for (int i = j + (tid & 63); i < nus; i += 64) *P4w(R2, cnux2, os + i, os + j) = Pl[i + j * ldP];
            // Gamma_{s-1} into GA; the state block of pL (with its gradient row) into X
            const int r0 = rows(sI - 1);
            load_flat<8>(GA, G + goff(sI - 1), r0 * nxs);
            for (int j = tid >> 6; j < nxs; j += WT / 64)
                for (int i = j + (tid & 63); i <= nxs; i += 64) X[i + j * ldX] = Pl[nus + i + (nus + j) * ldP];
            bar();
            // M: Gamma_{s-1} times the x_s x u_s block of pL; m: + the r row on the gradient row
            for (int e = tid; e < ((a.skip & 8) ? 0 : r0 * nus); e += WT) {
                const int i = e % r0, c = e / r0;
                double acc = 0.0;
                for (int l = 0; l < nxs; l++) acc += GA[i + l * r0] * Pl[nus + l + c * ldP];
                if (i == r0 - 1) acc += Pl[nux + c * ldP];
                *P4w(R2, cnux2, os + nus + i, os + c) = acc;
            }
            // Lx = chol_aug(X) inside wave 0 (row i on lane i, nxs + 1 <= 64 rows): 16-column panels factored in
            // registers (pivot values broadcast by readlane), each followed by its update of the later columns
            if (tid < 64 && !(a.skip & 4)) {
                const int i = tid;
                for (int p0 = 0; p0 < nxs; p0 += 16) {
                    const int pw = nxs - p0 < 16 ? nxs - p0 : 16;
                    double cl[16];
#pragma unroll
                    for (int jj = 0; jj < 16; jj++)
                        cl[jj] = (jj < pw && i >= p0 + jj && i <= nxs) ? X[i + (p0 + jj) * ldX] : 0.0;
#pragma unroll
                    for (int jj = 0; jj < 16; jj++) {
                        if (jj < pw) {
                            const double d = rdlane(cl[jj], p0 + jj);
                            double sq = 0.0, inv = 0.0;
                            if (d > 1e-15) {
                                sq = sqrt(d);
                                inv = 1.0 / sq;
                            }
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
            bar();
            // W = BAbt_{s-1} Lx (in place in Bt, row i by one thread), last row += l; pL = RSQ_{s-1} + W W'
            const WideStage sp = st[sI - 1];
            const int nuxp = sp.nu + sp.nx, nzp = nuxp + 1;
            load_dense<8>(Bt, ldB, BAbt + sp.oB, sp.sdB, nzp, nxs);
            load_dense<8>(Pl, ldP, RSQ + sp.oR, sp.sdR, nzp, nuxp);
            bar();
            if (!(a.skip & 16)) {
                // W = BAbt_{s-1} Lx (+ l on the last row) in place over Bt, then pL += W W' (lower), both on MFMA
                mfma_gemm(
                    nzp, nxs, nxs, [&](int i, int l) { return Bt[i + l * ldB]; },
                    [&](int l, int c) { return l >= c ? X[l + c * ldX] : 0.0; },
                    [&](int i, int c, double v) {
                        if (i == nuxp) v += X[nxs + c * ldX];
                        Bt[i + c * ldB] = v;
                    });
                bar();
                mfma_gemm(
                    nzp, nuxp, nxs, [&](int i, int l) { return Bt[i + l * ldB]; },
                    [&](int l, int j) { return Bt[j + l * ldB]; },
                    [&](int i, int j, double v) {
                        if (i >= j) Pl[i + j * ldP] += v;
                    });
            }
            bar();
        }
    }

    // ---- d_cond_DCtd: input boxes stay boxes, state boxes of stages 1..T-1 become general constraints ----
    {
        const int nbb = blk.nb2, nbg = blk.ng2, pnbb = (nbb + 3) / 4 * 4, pnbg = (nbg + 3) / 4 * 4;
        const int cnbg = (nbg + 1) / 2 * 2, pnv = (nv + 3) / 4 * 4;
        for (int e = tid; e < pnv * cnbg; e += WT) G2[e] = 0.0;
        for (int e = tid; e < 2 * pnbb + 2 * pnbg; e += WT) d2[e] = 0.0;
        bar();
        if (tid == 0) {
            int* i2 = p == 0 ? a.idxb2 + blk.oI2 : nullptr;
            int ib = 0, ig = 0, nu_tmp = 0, idx_gammab = nx0;
            for (int j = 0; j < T - 1; j++) idx_gammab += st[j].nu;
            for (int sI = T - 1; sI >= 1; sI--) {
                const WideStage s = st[sI];
                nu_tmp += s.nu;
                const int r0 = rows(sI - 1);
                const double* Gp = G + goff(sI - 1);
                for (int jj = 0; jj < s.nb; jj++) {
                    const int vv = idxb[s.oI + jj];
                    if (vv < s.nu) {
                        d2[ib] = dv[s.oD + jj];
                        d2[pnbb + ib] = dv[s.oD + s.pnb + jj];
                        if (i2) i2[ib] = nu_tmp - s.nu + vv;
                        ib++;
                    } else {
                        const int g = vv - s.nu;
                        const double c0 = Gp[idx_gammab + g * r0];
                        d2[2 * pnbb + ig] = dv[s.oD + jj] - c0;
                        d2[2 * pnbb + pnbg + ig] = dv[s.oD + s.pnb + jj] - c0;
                        for (int i = 0; i < idx_gammab; i++) *P4w(G2, cnbg, nu_tmp + i, ig) = Gp[i + g * r0];
                        ig++;
                    }
                }
                idx_gammab -= st[sI - 1].nu;
            }
            const WideStage s = st[0];
            nu_tmp += s.nu;
            for (int jj = 0; jj < s.nb; jj++) {
                d2[ib] = dv[s.oD + jj];
                d2[pnbb + ib] = dv[s.oD + s.pnb + jj];
                if (i2) i2[ib] = nu_tmp - s.nu + idxb[s.oI + jj];
                ib++;
            }
        }
    }
    // the terminal condensed stage is the original's (d_part_cond.c:1052-1056): block N2-1 copies it
    if (ii == a.N2 - 1) {
        const WideStage sN = a.st[a.N];
        const int n = (a.nzN + 3) / 4 * 4 * a.sdRN;
        double* RN = a.RSQ2 + (long)p * a.sR2 + a.oR2N;
        for (int e = tid; e < n; e += WT) RN[e] = RSQ[sN.oR + e];
    }
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

// ------------------------------------------------------------------------------------------------
// d_back_ric_rec_trs_tv_res on wide stages (d_back_ric_rec.c:564-791, restated in oracle/hpmpc_oracle.c):
// backward, per stage k = N..0: g_k = q_k + qx at idxb; v_k = g_k + BAbt_k (Pb_k + v_{k+1,x}) (k < N), with
// Pb_k = Lxx_{k+1}(Lxx_{k+1}' b_k); then L_k's n-form solve on the first nu_k columns (all of stage 0) with the
// rectangular update of the later rows.  Forward as the sv forward, pi_k = Lxx(Lxx' x_{k+1}) + v_{k+1,x}.
// The processed v_k are parked in ux (the forward overwrites them).  No general constraints (host-checked).
// ------------------------------------------------------------------------------------------------
__global__ __launch_bounds__(WT) void hk_wide_trs(WideArgs a) {
    extern __shared__ double sm[];
    const int p = blockIdx.x + a.p0;
    if (p >= a.nprob) return;
    const int tid = threadIdx.x, lane = tid & 63;
    double* M = sm;
    double* W = sm + a.offW;
    double* X = sm + a.offX;  // w = Pb + v_{k+1,x} (backward) / pi scratch (forward)
    double* v = sm + a.offV;
    const int ldW = a.ldW;
    const double* BAbt = a.BAbt + (long)p * a.sB;
    const double* F = a.ws + (long)p * a.sW;
    double* ux = a.ux + (long)p * a.sU;
    double* pi = a.pi + (long)p * a.sP;
    double* Pb = a.Pb + (long)p * a.sP;
    const double* hb = a.hb + (long)p * a.sP;
    const double* hq = a.hq + (long)p * a.sU;
    const double* qx = a.qx + (long)p * a.sC;
    for (int k = a.N; k >= 0; k--) {
        const WideStage s = a.st[k];
        const int nux = s.nu + s.nx, nz = nux + 1, nx1 = s.nx1;
        const int ns = k == 0 ? nux : s.nu;
        load_flat<16>(M, F + s.oL, poff(nux, nz) + nux);
        if (k < a.N) load_dense<8>(W, ldW, BAbt + s.oB, s.sdB, nux, nx1);
        for (int i = tid; i < nux; i += WT) v[i] = hq[s.oU + i];
        bar();
        if (tid == 0)
            for (int l = 0; l < s.nb; l++) v[a.idxb[s.oI + l]] += qx[s.oD + l];
        bar();
        if (k < a.N) {
            double c = 0.0;
            if (tid < nux)
                for (int j = 0; j < nx1; j++) c += W[tid + j * ldW] * X[j];
            bar();
            if (tid < nux) v[tid] += c;
            bar();
            // n-form solve on the first ns columns with the rectangular update (column-oriented, one wave)
            const double* dL = M + poff(nux, nz);
            if (tid < 64) {
                for (int j = 0; j < ns; j++) {
                    const double y = v[j] * dL[j];
                    const int cj = poff(j, nz) - j;
                    for (int i = j + 1 + lane; i < nux; i += 64) v[i] -= M[cj + i] * y;
                    if (lane == 0) v[j] = y;
                    wave_sync();
                }
            }
            bar();
        }
        for (int i = tid; i < nux; i += WT) ux[s.oU + i] = v[i];
        if (k > 0) {  // w for stage k-1: Pb_{k-1} = Lxx_k (Lxx_k' b_{k-1}), plus v_{k,x}
            const WideStage sp = a.st[k - 1];
            const int nu = s.nu, nx = s.nx;
            double t = 0.0;
            if (tid < nx) {
                const int cj = poff(nu + tid, nz) - (nu + tid);
                for (int i = tid; i < nx; i++) t += M[cj + nu + i] * hb[sp.oP + i];
            }
            bar();
            if (tid < nx) W[tid] = t;  // W is free: scratch
            bar();
            if (tid < nx) {
                double acc = 0.0;
                for (int j = 0; j <= tid; j++) acc += M[poff(nu + j, nz) + tid - j] * W[j];
                if (a.compute_Pb) Pb[sp.oP + tid] = acc;
                X[tid] = (a.compute_Pb ? acc : Pb[sp.oP + tid]) + v[nu + tid];
            }
        }
        bar();
    }
    // forward
    {
        const WideStage s0 = a.st[0];
        const int nz0 = s0.nu + s0.nx + 1;
        load_flat<16>(M, F + s0.oL, poff(nz0 - 1, nz0) + nz0 - 1);
        load_flat<4>(v, ux + s0.oU, nz0 - 1);
        bar();
    }
    for (int k = 0; k < a.N; k++) {
        const WideStage s = a.st[k], s1 = a.st[k + 1];
        const int nux = s.nu + s.nx, nz = nux + 1, nx1 = s.nx1, nu1 = s.nu1;
        const int ns = k == 0 ? nux : s.nu;
        const double* dL = M + poff(nux, nz);
        load_dense<8>(W, ldW, BAbt + s.oB, s.sdB, nux, nx1);
        double pk = 0.0;
        if (tid < nx1) pk = ux[s1.oU + nu1 + tid];  // v_{k+1,x} of the backward, before x_{k+1} replaces it
        for (int j = tid; j < ns; j += WT) v[j] = -v[j];
        bar();
        double r = 0.0;
        if (tid < ns) {  // - L[ns:nux, 0:ns]' x_k
            const int cj = poff(tid, nz) - tid;
            r = v[tid];
            for (int m = ns; m < nux; m++) r -= M[cj + m] * v[m];
        }
        bar();
        if (tid < ns) v[tid] = r;
        bar();
        if (tid < 64) {
            for (int i = ns - 1; i >= 0; i--) {
                const double y = v[i] * dL[i];
                for (int j = tid; j < i; j += 64) v[j] -= M[poff(j, nz) + i - j] * y;
                if (tid == 0) v[i] = y;
                wave_sync();
            }
        }
        bar();
        for (int j = tid; j < nux; j += WT) ux[s.oU + j] = v[j];
        double xn = 0.0;
        if (tid < nx1) {
            xn = hb[s.oP + tid];
            for (int i = 0; i < nux; i++) xn += W[i + tid * ldW] * v[i];
        }
        bar();
        const int nux1 = nu1 + nx1, nz1 = nux1 + 1;
        load_flat<16>(M, F + s1.oL, poff(nux1, nz1) + nux1);
        // v <- stage k+1: the backward's processed u part, and the actual state x_{k+1}
        for (int j = tid; j < nu1; j += WT) v[j] = ux[s1.oU + j];
        if (tid < nx1) v[nu1 + tid] = xn;
        bar();
        if (a.compute_pi) {
            if (tid < nx1) {
                const int cj = poff(nu1 + tid, nz1) - (nu1 + tid);
                double tj = 0.0;
                for (int i = tid; i < nx1; i++) tj += M[cj + nu1 + i] * v[nu1 + i];
                X[tid] = tj;
            }
            bar();
            if (tid < nx1) {
                double acc = 0.0;
                for (int j = 0; j <= tid; j++) acc += M[poff(nu1 + j, nz1) + tid - j] * X[j];
                pi[s.oP + tid] = acc + pk;
            }
            bar();
        }
    }
    if (tid < a.st[a.N].nx) ux[a.st[a.N].oU + tid] = v[tid];
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
            hipLaunchKernelGGL(hk_pcond, dim3(a.N2, count), dim3(WT), lds, stream, a);
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
