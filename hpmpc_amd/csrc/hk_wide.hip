// hk_wide.hip -- MI355X (gfx950) kernels for stages wider than the 16-wide register tile:
//   hk_wide_sv  d_back_ric_rec_sv_tv_res (lqcp_solvers/d_back_ric_rec.c:112-399) for nu+nx > 16, one
//               256-thread workgroup per problem, the stage Hessian in LDS as packed lower columns;
//   hk_pcond    d_part_cond (lqcp_solvers/d_part_cond.c:926-1062): one workgroup per (block, problem),
//               every block of every problem condensed concurrently;
//   hk_pexpand  d_part_expand_solution (d_part_cond.c:1103-1308): one workgroup per problem.
//
// These are the "next" rows of SURVEY.md §8f #1 (configs[4]: N=200 -> 20 blocks of 10, nx=24 nu=6).
// Every stage matrix is read from HBM once per pass in the reference's lib4 layout and staged into LDS
// as a dense column-major tile; the per-stage work is spread over the 256 lanes of the workgroup with
// one barrier per dependency step (one per Cholesky column).
#include <hip/hip_runtime.h>

#include "hk_wide_args.h"

namespace {

constexpr int WT = 256;  // threads per workgroup
constexpr int BS = 4;

__device__ __forceinline__ double P4(const double* A, int sd, int i, int j) {
    return A[(i / BS) * BS * sd + i % BS + BS * j];
}
__device__ __forceinline__ double* P4w(double* A, int sd, int i, int j) {
    return A + (i / BS) * BS * sd + i % BS + BS * j;
}
// packed lower columns of an nz-row matrix: column j holds rows j..nz-1
__device__ __forceinline__ int poff(int j, int nz) { return j * nz - (j * (j - 1)) / 2; }

__device__ __forceinline__ void bar() { __syncthreads(); }

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
    const double* BAbt = a.BAbt + (long)p * a.sB;
    const double* RSQ = a.RSQ + (long)p * a.sR;
    double* F = a.ws + (long)p * a.sW;
    double* ux = a.ux + (long)p * a.sU;
    double* pi = a.pi + (long)p * a.sP;
    double* Pb = a.Pb ? a.Pb + (long)p * a.sP : nullptr;

    for (int k = a.N; k >= 0; k--) {
        const WideStage s = a.st[k];
        const int nu = s.nu, nux = s.nu + s.nx, nz = nux + 1, nx1 = s.nx1;
        const double* R = RSQ + s.oR;
        for (int j = tid >> 6; j < nux; j += WT / 64)
            for (int i = j + (tid & 63); i < nz; i += 64) M[poff(j, nz) + i - j] = P4(R, s.sdR, i, j);
        if (k < a.N) {
            const double* B = BAbt + s.oB;
            for (int e = tid; e < nz * nx1; e += WT) {
                const int i = e % nz, c = e / nz;
                W[i + c * ldW] = P4(B, s.sdB, i, c);
            }
            bar();
            // W = BAbt Lxx (in place, row i by thread: w_c needs W[i, l >= c] only)
            for (int i = tid; i < nz; i += WT)
                for (int c = 0; c < nx1; c++) {
                    double acc = 0.0;
                    for (int l = c; l < nx1; l++) acc += W[i + l * ldW] * X[l + c * ldX];
                    W[i + c * ldW] = acc;
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
            for (int j = tid >> 6; j < nux; j += WT / 64)
                for (int i = j + (tid & 63); i < nz; i += 64) {
                    double acc = 0.0;
                    for (int r = 0; r < nx1; r++) acc += W[i + r * ldW] * W[j + r * ldW];
                    M[poff(j, nz) + i - j] += acc;
                }
        }
        bar();
        double* Lk = F + s.oL;
        double* dL = Lk + poff(nux, nz);
        for (int j = 0; j < nux; j++) {
            const int cj = poff(j, nz);
            const double d = M[cj];
            double sq = 0.0, inv = 0.0;
            if (d > 1e-15) {
                sq = sqrt(d);
                inv = 1.0 / sq;
            }
            for (int i = j + tid; i < nz; i += WT) {
                const double l = i == j ? sq : M[cj + i - j] * inv;
                Lk[cj + i - j] = l;
                if (j >= nu) X[(i - nu) + (j - nu) * ldX] = l;
            }
            if (tid == 0) dL[j] = inv;
            for (int c = j + 1 + (tid >> 6); c < nux; c += WT / 64) {
                const double lc = M[cj + c - j] * inv;
                const int cc = poff(c, nz);
                for (int i = c + (tid & 63); i < nz; i += 64) M[cc + i - c] -= (M[cj + i - j] * inv) * lc;
            }
            bar();
        }
        // strictly upper part of the copied Lxx stays zero
        for (int e = tid; e < s.nx * s.nx; e += WT) {
            const int i = e % s.nx, c = e / s.nx;
            if (i < c) X[i + c * ldX] = 0.0;
        }
        bar();
    }

    // forward substitution
    for (int k = 0; k < a.N; k++) {
        const WideStage s = a.st[k];
        const int nux = s.nu + s.nx, nz = nux + 1, nx1 = s.nx1, nu1 = s.nu1;
        const int ns = k == 0 ? nux : s.nu;
        const double* Lk = F + s.oL;
        const double* dL = Lk + poff(nux, nz);
        // v[0:ns] = -l[0:ns] - L[ns:nux, 0:ns]' v[ns:nux]   (v[ns:nux] = x_k from the previous stage)
        for (int j = tid; j < ns; j += WT) {
            double r = -Lk[poff(j, nz) + nux - j];
            for (int m = ns; m < nux; m++) r -= Lk[poff(j, nz) + m - j] * v[m];
            v[j] = r;
        }
        bar();
        // back substitution with L[0:ns, 0:ns]' (column-oriented, inv_diag multiply)
        for (int i = ns - 1; i >= 0; i--) {
            const double y = v[i] * dL[i];
            bar();
            for (int j = tid; j < i; j += WT) v[j] -= Lk[poff(j, nz) + i - j] * y;
            if (tid == 0) v[i] = y;
            bar();
        }
        for (int j = tid; j < nux; j += WT) ux[s.oU + j] = v[j];
        // x_{k+1} = b_k + BAbt_k' ux_k
        const double* B = BAbt + s.oB;
        double xn = 0.0;
        if (tid < nx1) {
            xn = P4(B, s.sdB, nux, tid);
            for (int i = 0; i < nux; i++) xn += P4(B, s.sdB, i, tid) * v[i];
        }
        bar();
        const WideStage s1 = a.st[k + 1];
        if (tid < nx1) {
            v[nu1 + tid] = xn;
            ux[s1.oU + nu1 + tid] = xn;
        }
        bar();
        if (a.compute_pi) {  // pi_k = Lxx (Lxx' x + l), Lxx of stage k+1 (rows / cols nu1.., packed)
            const int nux1 = nu1 + nx1, nz1 = nux1 + 1;
            const double* L1 = F + s1.oL;
            double tj = 0.0;
            if (tid < nx1) {
                const int cj = poff(nu1 + tid, nz1);
                tj = L1[cj + nux1 - (nu1 + tid)];
                for (int i = tid; i < nx1; i++) tj += L1[cj + i - tid] * v[nu1 + i];
            }
            bar();
            if (tid < nx1) W[tid] = tj;
            bar();
            if (tid < nx1) {
                double acc = 0.0;
                for (int j = 0; j <= tid; j++) acc += L1[poff(nu1 + j, nz1) + tid - j] * W[j];
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
    double* W = sm + a.offW;   // W (ld ldW)
    double* Bt = sm + a.offB;  // stage BAbt tile (ld ldB)
    const int ldP = a.ldP, ldX = a.ldX, ldW = a.ldW, ldB = a.ldB;

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

    // ---- d_cond_BAbt ----
    {
        const WideStage s = st[0];
        const int r0 = s.nu + s.nx + 1;
        const double* B = BAbt + s.oB;
        for (int e = tid; e < r0 * s.nx1; e += WT) {
            const int i = e % r0, c = e / r0;
            G[i + c * r0] = P4(B, s.sdB, i, c);
        }
    }
    bar();
    for (int j = 1; j < T; j++) {
        const WideStage s = st[j];
        const int nuj = s.nu, nxj = s.nx, nx1 = s.nx1, nzj = nuj + nxj + 1;
        const int rp = rows(j - 1), rj = rp + nuj;
        const double* Gp = G + goff(j - 1);
        double* Gj = G + goff(j);
        const double* B = BAbt + s.oB;
        for (int e = tid; e < nzj * nx1; e += WT) {
            const int i = e % nzj, c = e / nzj;
            Bt[i + c * ldB] = P4(B, s.sdB, i, c);
        }
        bar();
        for (int e = tid; e < rj * nx1; e += WT) {
            const int i = e % rj, c = e / rj;
            double val;
            if (i < nuj) {
                val = Bt[i + c * ldB];
            } else {
                const int ip = i - nuj;
                double acc = 0.0;
                for (int l = 0; l < nxj; l++) acc += Gp[ip + l * rp] * Bt[nuj + l + c * ldB];
                val = acc;
                if (i == rj - 1) val += Bt[nuj + nxj + c * ldB];
            }
            Gj[i + c * rj] = val;
        }
        bar();
    }
    {
        const int rT = rows(T - 1), nxT = st[T - 1].nx1;
        const double* GT = G + goff(T - 1);
        const int sd = (nxT + 1) / 2 * 2;
        for (int e = tid; e < rT * nxT; e += WT) {
            const int i = e % rT, c = e / rT;
            *P4w(B2, sd, i, c) = GT[i + c * rT];
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
            const int nux = s.nu + s.nx;
            for (int j = tid >> 6; j < nux; j += WT / 64)
                for (int i = j + (tid & 63); i <= nux; i += 64) Pl[i + j * ldP] = P4(RSQ + s.oR, s.sdR, i, j);
        }
        bar();
        for (int sI = T - 1;; sI--) {
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
            // M: Gamma_{s-1} times the x_s x u_s block of pL; m: + the r row on the gradient row
            {
                const int r0 = rows(sI - 1);
                const double* Gp = G + goff(sI - 1);
                for (int e = tid; e < r0 * nus; e += WT) {
                    const int i = e % r0, c = e / r0;
                    double acc = 0.0;
                    for (int l = 0; l < nxs; l++) acc += Gp[i + l * r0] * Pl[nus + l + c * ldP];
                    if (i == r0 - 1) acc += Pl[nux + c * ldP];
                    *P4w(R2, cnux2, os + nus + i, os + c) = acc;
                }
            }
            // Lx = chol_aug(pL[x, x] with its gradient row), right-looking in X
            for (int j = tid >> 6; j < nxs; j += WT / 64)
                for (int i = j + (tid & 63); i <= nxs; i += 64) X[i + j * ldX] = Pl[nus + i + (nus + j) * ldP];
            bar();
            for (int j = 0; j < nxs; j++) {
                const double d = X[j + j * ldX];
                double sq = 0.0, inv = 0.0;
                if (d > 1e-15) {
                    sq = sqrt(d);
                    inv = 1.0 / sq;
                }
                // trailing update reads the unscaled column j, then the column is scaled (after a barrier)
                for (int c = j + 1 + (tid >> 6); c < nxs; c += WT / 64) {
                    const double lc = X[c + j * ldX] * inv;
                    for (int i = c + (tid & 63); i <= nxs; i += 64) X[i + c * ldX] -= (X[i + j * ldX] * inv) * lc;
                }
                bar();
                for (int i = j + tid; i <= nxs; i += WT) X[i + j * ldX] = i == j ? sq : X[i + j * ldX] * inv;
                bar();
            }
            // W = BAbt_{s-1} Lx, last row += l; pL = RSQ_{s-1} + W W'
            const WideStage sp = st[sI - 1];
            const int nuxp = sp.nu + sp.nx, nzp = nuxp + 1;
            {
                const double* B = BAbt + sp.oB;
                for (int e = tid; e < nzp * nxs; e += WT) {
                    const int i = e % nzp, c = e / nzp;
                    Bt[i + c * ldB] = P4(B, sp.sdB, i, c);
                }
            }
            bar();
            for (int e = tid; e < nzp * nxs; e += WT) {
                const int i = e % nzp, c = e / nzp;
                double acc = 0.0;
                for (int l = c; l < nxs; l++) acc += Bt[i + l * ldB] * X[l + c * ldX];
                if (i == nuxp) acc += X[nxs + c * ldX];
                W[i + c * ldW] = acc;
            }
            bar();
            for (int j = tid >> 6; j < nuxp; j += WT / 64)
                for (int i = j + (tid & 63); i <= nuxp; i += 64) {
                    double acc = 0.0;
                    for (int l = 0; l < nxs; l++) acc += W[i + l * ldW] * W[j + l * ldW];
                    Pl[i + j * ldP] = P4(RSQ + sp.oR, sp.sdR, i, j) + acc;
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
// Expansion of the condensed solution (d_part_expand_solution).
// ------------------------------------------------------------------------------------------------
__global__ __launch_bounds__(WT) void hk_pexpand(PxArgs a) {
    extern __shared__ double sm[];
    const int p = blockIdx.x + a.p0;
    if (p >= a.nprob) return;
    const int tid = threadIdx.x;
    const WideStage* st = a.st;
    const WideStage* st2 = a.st2;
    const double* BAbt = a.BAbt + (long)p * a.sB;
    const double* RSQ = a.RSQ + (long)p * a.sR;
    const double* ux2 = a.ux2 + (long)p * a.sU2;
    const double* pi2 = a.pi2 + (long)p * a.sP2;
    const double* lam2 = a.lam2 + (long)p * a.sC2;
    const double* t2 = a.t2 + (long)p * a.sC2;
    double* ux = a.ux + (long)p * a.sU;
    double* pi = a.pi + (long)p * a.sP;
    double* lam = a.lam + (long)p * a.sC;
    double* t = a.t + (long)p * a.sC;
    const double* hb = a.hb ? a.hb + (long)p * a.sP : nullptr;
    const double* hrq = a.hrq ? a.hrq + (long)p * a.sU : nullptr;
    double* w = sm + a.offW;

    // inputs (reverse stage order) and the blocks' first states; the final state
    for (int ii = 0; ii < a.N2; ii++) {
        const PcBlock blk = a.blk[ii];
        const double* u2 = ux2 + st2[ii].oU;
        int nu_tmp = 0;
        for (int jj = 0; jj < blk.T - 1; jj++) {
            const WideStage s = st[blk.s0 + blk.T - 1 - jj];
            for (int l = tid; l < s.nu; l += WT) ux[s.oU + l] = u2[nu_tmp + l];
            nu_tmp += s.nu;
        }
        const WideStage s = st[blk.s0];
        for (int l = tid; l < s.nu + s.nx; l += WT) ux[s.oU + l] = u2[nu_tmp + l];
    }
    for (int l = tid; l < st[a.N].nx; l += WT) ux[st[a.N].oU + l] = ux2[st2[a.N2].oU + l];
    bar();
    // states inside the blocks by simulation, x_{j+1} = b_j + BAbt_j' ux_j
    for (int ii = 0; ii < a.N2; ii++) {
        const PcBlock blk = a.blk[ii];
        for (int jj = 0; jj < blk.T - 1; jj++) {
            const WideStage s = st[blk.s0 + jj], s1 = st[blk.s0 + jj + 1];
            const int nux = s.nu + s.nx;
            const double* B = BAbt + s.oB;
            if (tid < s.nx1) {
                double acc = 0.0;
                for (int i = 0; i < nux; i++) acc += P4(B, s.sdB, i, tid) * ux[s.oU + i];
                const double b = hb ? hb[s.oP + tid] : P4(B, s.sdB, nux, tid);
                ux[s1.oU + s1.nu + tid] = b + acc;
            }
            bar();
        }
    }
    // slacks and inequality multipliers (one thread per block: the slot order is a prefix scan)
    for (int ii = tid; ii < a.N2; ii += WT) {
        const PcBlock blk = a.blk[ii];
        const int pnb2 = st2[ii].pnb, png2 = (st2[ii].ng + 3) / 4 * 4, o2 = st2[ii].oD;
        int nbb2_tmp = 0, nbg2_tmp = 0;
        for (int jj = 0; jj < blk.T - 1; jj++) {
            const WideStage s = st[blk.s0 + blk.T - 1 - jj];
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
        const WideStage s = st[blk.s0];
        for (int l = 0; l < s.nb; l++) {
            lam[s.oD + l] = lam2[o2 + nbb2_tmp + l];
            lam[s.oD + s.pnb + l] = lam2[o2 + pnb2 + nbb2_tmp + l];
            t[s.oD + l] = t2[o2 + nbb2_tmp + l];
            t[s.oD + s.pnb + l] = t2[o2 + pnb2 + nbb2_tmp + l];
        }
    }
    if (tid == 0) {  // last stage: box and general slots copied
        const WideStage s = st[a.N], c = st2[a.N2];
        const int png = (s.ng + 3) / 4 * 4, png2 = (c.ng + 3) / 4 * 4;
        for (int j = 0; j < s.nb; j++) {
            lam[s.oD + j] = lam2[c.oD + j];
            lam[s.oD + s.pnb + j] = lam2[c.oD + c.pnb + j];
            t[s.oD + j] = t2[c.oD + j];
            t[s.oD + s.pnb + j] = t2[c.oD + c.pnb + j];
        }
        for (int j = 0; j < s.ng; j++) {
            lam[s.oD + 2 * s.pnb + j] = lam2[c.oD + 2 * c.pnb + j];
            lam[s.oD + 2 * s.pnb + png + j] = lam2[c.oD + 2 * c.pnb + png2 + j];
            t[s.oD + 2 * s.pnb + j] = t2[c.oD + 2 * c.pnb + j];
            t[s.oD + 2 * s.pnb + png + j] = t2[c.oD + 2 * c.pnb + png2 + j];
        }
    }
    bar();
    // equality multipliers: pi_{s-1} = [rq_s + box terms + RSQ_s ux_s + BAbt_s pi_s]_x inside each block
    for (int ii = 0; ii < a.N2; ii++) {
        const PcBlock blk = a.blk[ii];
        const WideStage sl = st[blk.s0 + blk.T - 1];
        for (int l = tid; l < sl.nx1; l += WT) pi[sl.oP + l] = pi2[st2[ii].oP + l];
        bar();
        for (int jj = 0; jj < blk.T - 1; jj++) {
            const int sI = blk.s0 + blk.T - 1 - jj;
            const WideStage s = st[sI], sm1 = st[sI - 1];
            const int nux = s.nu + s.nx;
            // box terms by variable (w holds -lam_l + lam_u at idxb, 0 elsewhere)
            for (int l = tid; l < nux; l += WT) w[l] = 0.0;
            bar();
            if (tid == 0)
                for (int l = 0; l < s.nb; l++) w[a.idxb[s.oI + l]] += -lam[s.oD + l] + lam[s.oD + s.pnb + l];
            bar();
            const double* R = RSQ + s.oR;
            const double* B = BAbt + s.oB;
            if (tid < s.nx) {
                const int i = s.nu + tid;
                double acc = hrq ? hrq[s.oU + i] : P4(R, s.sdR, nux, i);
                acc += w[i];
                double sy = 0.0;
                for (int j = 0; j < nux; j++) sy += (i >= j ? P4(R, s.sdR, i, j) : P4(R, s.sdR, j, i)) * ux[s.oU + j];
                acc += sy;
                double sg = 0.0;
                for (int j = 0; j < s.nx1; j++) sg += P4(B, s.sdB, i, j) * pi[s.oP + j];
                acc += sg;
                pi[sm1.oP + tid] = acc;
            }
            bar();
        }
    }
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
            hipLaunchKernelGGL(hk_pexpand, dim3(count), dim3(WT), lds, stream, a);
            break;
        }
        default:
            return -1;
    }
    return (int)hipGetLastError();
}
