// hk_wide_core.h -- device building blocks of the wide-stage path (stages beyond the 16-wide register tile),
// shared by hk_wide.hip (Riccati sv / trf / trs, condensing, expansion) and hk_wide_ipm.hip (the IPM on wide
// stages): LDS staging helpers, the MFMA gemm, and the per-problem bodies of the wide Riccati factorisation +
// solve (d_back_ric_rec_sv_tv_res / _trf_tv_res, lqcp_solvers/d_back_ric_rec.c:112-560) and of the solve with a
// new right-hand side (d_back_ric_rec_trs_tv_res, :564-791).  One 256-thread workgroup owns a problem; stage
// tiles live in LDS as dense column-major (or packed lower) blocks.
#pragma once
#include <hip/hip_runtime.h>

#include "hk_prims.h"
#include "hk_wide_args.h"

namespace {

using hk::gld;

constexpr int WT = 256;  // threads per workgroup
constexpr int WS_TILES = 8;  // W = BAbt Lxx output tiles per wave (nz <= 128, nx <= 64: <= 32 tiles, host-checked)
constexpr int DT_TILES = 6;  // DCt diag DCt' lower tiles per wave on the LDS-staged path (nz <= 96; larger stages read HBM directly)
constexpr int DS_LD = 17;   // row stride (doubles) of the staged DCt block: 16 columns + 1 pad against LDS bank conflicts

constexpr int BS = 4;

// lib4 index of (i, j), i >= 0 (shifts: the signed / and % by 4 cost a sign fix-up each)
__device__ __forceinline__ int p4i(int i, int j, int sd) { return (i >> 2) * (BS * sd) + (i & 3) + BS * j; }

__device__ __forceinline__ double P4(const double* A, int sd, int i, int j) { return A[p4i(i, j, sd)]; }
__device__ __forceinline__ double* P4w(double* A, int sd, int i, int j) { return A + p4i(i, j, sd); }

// e / n for 0 <= e < 2^20 from rn = 1.0f / n (a float multiply instead of the ~35-instruction integer division):
// (e + 0.5) / n lies at least 0.5 / n from an integer, far more than the float rounding of the product.
__device__ __forceinline__ int fdiv(int e, float rn) { return (int)(((float)e + 0.5f) * rn); }
// packed lower columns of an nz-row matrix: column j holds rows j..nz-1
__device__ __forceinline__ int poff(int j, int nz) { return j * nz - (j * (j - 1)) / 2; }

__device__ __forceinline__ void bar() { __syncthreads(); }
// A workgroup barrier for LDS data only: this wave's LDS operations are complete, then s_barrier.  Unlike
// __syncthreads it does not wait for outstanding global loads and stores (a prefetch or an LDS DMA in flight, the
// stores of a finished tile), so it may only order LDS traffic; global data passed between threads needs bar().
__device__ __forceinline__ void lds_bar() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

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
    const float rn = 1.0f / nr;
    for (int base = 0; base < n; base += WT * CH) {
        double r[CH];
        int dof[CH];
#pragma unroll
        for (int u = 0; u < CH; u++) {
            const int e = base + u * WT + tid, c = fdiv(e, rn), i = e - c * nr;
            r[u] = gld(src, p4i(i, c, sd), e < n);
            dof[u] = i + c * ld;
        }
#pragma unroll
        for (int u = 0; u < CH; u++)
            if (base + u * WT + tid < n) D[dof[u]] = r[u];
    }
}
// The same copy split in two: pre_dense issues the loads of a block of at most CH * WT elements into registers,
// put_dense stores them into LDS later, so their memory latency overlaps whatever work runs in between.
template <int CH>
struct Staged {
    double r[CH];
    int nr, nc;
};
template <int CH>
__device__ __forceinline__ void pre_dense(Staged<CH>& S, const double* src, int sd, int nr, int nc) {
    const int tid = threadIdx.x, n = nr * nc;
    S.nr = nr;
    S.nc = nc;
    const float rn = 1.0f / nr;
#pragma unroll
    for (int u = 0; u < CH; u++) {
        const int e = u * WT + tid, c = fdiv(e, rn), i = e - c * nr;
        S.r[u] = gld(src, p4i(i, c, sd), e < n);
    }
}
template <int CH>
__device__ __forceinline__ void put_dense(const Staged<CH>& S, double* D, int ld) {
    const int tid = threadIdx.x, nr = S.nr, n = S.nr * S.nc;
    const float rn = 1.0f / nr;
#pragma unroll
    for (int u = 0; u < CH; u++) {
        const int e = u * WT + tid, c = fdiv(e, rn), i = e - c * nr;
        if (e < n) D[i + c * ld] = S.r[u];
    }
}
// A flat block of at most CH * WT doubles staged in registers (pre_flat issues the loads, put_flat stores to LDS)
template <int CH>
struct Flat {
    double r[CH];
};
template <int CH>
__device__ __forceinline__ void pre_flat(Flat<CH>& S, const double* src, int n) {
#pragma unroll
    for (int u = 0; u < CH; u++) S.r[u] = gld(src, u * WT + threadIdx.x, u * WT + (int)threadIdx.x < n);
}
template <int CH>
__device__ __forceinline__ void put_flat(const Flat<CH>& S, double* D, int n) {
#pragma unroll
    for (int u = 0; u < CH; u++)
        if (u * WT + (int)threadIdx.x < n) D[u * WT + threadIdx.x] = S.r[u];
}
// The same staging done by a group of NT threads (t = index in the group): at most CH * NT elements
template <int NT, int CH>
__device__ __forceinline__ void pre_dense_g(Staged<CH>& S, const double* src, int sd, int nr, int nc, int t) {
    const int n = nr * nc;
    S.nr = nr;
    S.nc = nc;
    const float rn = 1.0f / nr;
#pragma unroll
    for (int u = 0; u < CH; u++) {
        const int e = u * NT + t, c = fdiv(e, rn), i = e - c * nr;
        S.r[u] = gld(src, p4i(i, c, sd), e < n);
    }
}
template <int NT, int CH>
__device__ __forceinline__ void put_dense_g(const Staged<CH>& S, double* D, int ld, int t) {
    const int nr = S.nr, n = S.nr * S.nc;
    const float rn = 1.0f / nr;
#pragma unroll
    for (int u = 0; u < CH; u++) {
        const int e = u * NT + t, c = fdiv(e, rn), i = e - c * nr;
        if (e < n) D[i + c * ld] = S.r[u];
    }
}
template <int NT, int CH>
__device__ __forceinline__ void pre_flat_g(Flat<CH>& S, const double* src, int n, int t) {
#pragma unroll
    for (int u = 0; u < CH; u++) S.r[u] = gld(src, u * NT + t, u * NT + t < n);
}
template <int NT, int CH>
__device__ __forceinline__ void put_flat_g(const Flat<CH>& S, double* D, int n, int t) {
#pragma unroll
    for (int u = 0; u < CH; u++)
        if (u * NT + t < n) D[u * NT + t] = S.r[u];
}
// A stage record from an LDS table with every field made wave-uniform (readfirstlane).  Stage tables in global memory
// cannot be read with scalar loads (the kernels store to global memory, so the compiler cannot prove the table
// unchanged): each read would be a vector load followed by a wait for ALL outstanding vector-memory operations,
// prefetches and LDS DMA included.  Kernels copy their stage table into LDS once (stage_table_to_lds) and read it
// through StTab.
__device__ __forceinline__ WideStage rfl_stage(const WideStage& v) {
    constexpr int NI = sizeof(WideStage) / sizeof(int);
    const int* a = reinterpret_cast<const int*>(&v);
    WideStage u;
    int* b = reinterpret_cast<int*>(&u);
#pragma unroll
    for (int i = 0; i < NI; i++) b[i] = __builtin_amdgcn_readfirstlane(a[i]);
    return u;
}
struct StTab {
    const WideStage* p;
    __device__ __forceinline__ WideStage operator[](int i) const { return rfl_stage(p[i]); }
};
// n stage records from global memory into an LDS table (all threads of the workgroup; a barrier must follow)
__device__ __forceinline__ void stage_table_to_lds(WideStage* dst, const WideStage* src, int n) {
    constexpr int NI = sizeof(WideStage) / sizeof(int);
    const int* a = reinterpret_cast<const int*>(src);
    int* b = reinterpret_cast<int*>(dst);
    for (int e = threadIdx.x; e < n * NI; e += WT) b[e] = a[e];
}

// The wide kernels' stage table into LDS at offST (every thread; ends with a barrier)
__device__ __forceinline__ void wide_stage_table(const WideArgs& a) {
    extern __shared__ double sm[];
    stage_table_to_lds(reinterpret_cast<WideStage*>(sm + a.offST), a.st, a.N + 1);
    __syncthreads();
}

// Asynchronous global -> LDS copy of n doubles (v_global_load_lds): a lane's B bytes land at its wave's LDS base +
// lane * B without passing through registers, so the copy costs no VGPRs and its round trip overlaps whatever the
// wave does next.  The NT threads of a group (t = index in the group) split the copy; a wave's part is in LDS after
// its dma_wait(), and other waves see it after a barrier that follows.  B = 16 needs src and dst 16-byte aligned and
// n even; B = 4 only 4-byte alignment.
typedef __attribute__((address_space(3))) void* lds_void_ptr;
template <int NT, int B>
__device__ __forceinline__ int dma_copy(double* dst, const double* src, int n, int t) {
    constexpr int PER = B / 4;  // dwords per lane
    const int nd = 2 * n, lane = t & 63;
    int cnt = 0;  // DMA instructions this wave issued (for dma_wait_keep)
    for (int base = 64 * PER * (t >> 6); base < nd; base += 64 * PER * (NT / 64), cnt++) {  // dwords, wave-uniform
        if (base + PER * lane < nd) {
            const void* g = reinterpret_cast<const unsigned*>(src) + base + PER * lane;
            lds_void_ptr l = (lds_void_ptr)(reinterpret_cast<unsigned*>(dst) + base);
            if constexpr (B == 16)
                __builtin_amdgcn_global_load_lds(g, l, 16, 0, 0);
            else
                __builtin_amdgcn_global_load_lds(g, l, 4, 0, 0);
        }
    }
    return cnt;
}
// 16-byte DMA when both ends are 16-byte aligned and n is even, else 4-byte (uniform choice)
template <int NT>
__device__ __forceinline__ int dma_copy_any(double* dst, const double* src, int n, int t) {
    if ((((unsigned long long)src | (unsigned long long)dst) & 15) == 0 && (n & 1) == 0)
        return dma_copy<NT, 16>(dst, src, n, t);
    return dma_copy<NT, 4>(dst, src, n, t);
}
__device__ __forceinline__ void dma_wait() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }
// Wait until at most `keep` of this wave's vector-memory operations are outstanding (they complete in issue order):
// the copies issued before the last `keep` have landed.  keep is wave-uniform; beyond 31 it waits for all.
__device__ __forceinline__ void dma_wait_keep(int keep) {
    switch (__builtin_amdgcn_readfirstlane(keep)) {
#define HK_VMW(n) \
    case n: asm volatile("s_waitcnt vmcnt(" #n ")" ::: "memory"); break;
        HK_VMW(1) HK_VMW(2) HK_VMW(3) HK_VMW(4) HK_VMW(5) HK_VMW(6) HK_VMW(7) HK_VMW(8)
        HK_VMW(9) HK_VMW(10) HK_VMW(11) HK_VMW(12) HK_VMW(13) HK_VMW(14) HK_VMW(15) HK_VMW(16)
        HK_VMW(17) HK_VMW(18) HK_VMW(19) HK_VMW(20) HK_VMW(21) HK_VMW(22) HK_VMW(23) HK_VMW(24)
        HK_VMW(25) HK_VMW(26) HK_VMW(27) HK_VMW(28) HK_VMW(29) HK_VMW(30) HK_VMW(31)
#undef HK_VMW
        default: asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
}

// lib4 lower trapezoid rows [j, nz) of cols [0, nc) -> packed lower columns by DMA, no VGPRs for the data: one
// wave instruction moves 32 doubles of a packed column, two lanes per double (4 bytes each) gathered from the lib4
// panels, so the whole trapezoid is one memory round trip.  In LDS after dma_wait() and a barrier.
__device__ __forceinline__ void dma_lower(double* M, const double* src, int sd, int nz, int nc) {
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), l = threadIdx.x & 63;
    for (int j = w; j < nc; j += WT / 64)
        for (int r0 = j; r0 < nz; r0 += 32) {
            const int i = r0 + (l >> 1);
            if (i < nz) {
                const void* g = reinterpret_cast<const unsigned*>(src + p4i(i, j, sd)) + (l & 1);
                lds_void_ptr d = (lds_void_ptr)(M + poff(j, nz) + r0 - j);
                __builtin_amdgcn_global_load_lds(g, d, 4, 0, 0);
            }
        }
}
// lib4 rows [0, nr) x cols [0, nc) -> dense column-major (ld) by DMA, no VGPRs for the data: one wave instruction per
// 32 rows of a column (two lanes per double, 4 bytes each); returns the instructions this wave issued (dma_wait_keep)
__device__ __forceinline__ int dma_dense(double* D, int ld, const double* src, int sd, int nr, int nc) {
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), l = threadIdx.x & 63;
    int cnt = 0;
    for (int j = w; j < nc; j += WT / 64)
        for (int r0 = 0; r0 < nr; r0 += 32, cnt++) {
            const int i = r0 + (l >> 1);
            if (i < nr) {
                const void* g = reinterpret_cast<const unsigned*>(src + p4i(i, j, sd)) + (l & 1);
                lds_void_ptr d = (lds_void_ptr)(D + r0 + j * ld);
                __builtin_amdgcn_global_load_lds(g, d, 4, 0, 0);
            }
        }
    return cnt;
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

// In-register triangular solves for wave 0 on a packed-lower factor M (poff columns, nz rows) with inverse diagonal
// dL: v[0..n) sits in registers, two entries per lane (v[l], v[l + 64], n <= 128), each pivot is broadcast by
// readlane.  Every entry sees the same operations in the same order as the column loops over LDS they replace
// (one LDS round trip and wave barrier per pivot), so the results are the same.
// The pivots go in groups of four whose factor entries and inverse diagonals are read before the group's chain of
// broadcasts (clamped in-range reads, then a select), so the LDS latency is paid once per group.
// L' y = v on the first ns unknowns, descending (dtrsv_t over the u block): v[j] -= L[i][j] y_i for j < i.
__device__ __forceinline__ void wave_solve_lt(double* v, const double* M, const double* dL, int nz, int ns) {
    const int l = threadIdx.x & 63;
    double v0 = l < ns ? v[l] : 0.0, v1 = l + 64 < ns ? v[l + 64] : 0.0;
    const int c0 = l < ns ? poff(l, nz) - l : 0, c1 = l + 64 < ns ? poff(l + 64, nz) - l - 64 : 0;
    auto step = [&](int i, double m0, double m1, double d) {
        const double y = rdlane(i < 64 ? v0 : v1, i & 63) * d;
        if (l < i) v0 -= m0 * y;
        if (l + 64 < i) v1 -= m1 * y;
        if (l == i) v0 = y;
        if (l + 64 == i) v1 = y;
    };
    int i = ns - 1;
    for (; i >= 3; i -= 4) {
        double m0[4], m1[4], d[4];
#pragma unroll
        for (int q = 0; q < 4; q++) {
            m0[q] = M[c0 + (l < i - q ? i - q : l)];
            m1[q] = M[c1 + (l + 64 < i - q ? i - q : l + 64)];
            d[q] = dL[i - q];
        }
#pragma unroll
        for (int q = 0; q < 4; q++) step(i - q, m0[q], m1[q], d[q]);
    }
    for (; i >= 0; i--) step(i, M[c0 + (l < i ? i : l)], M[c1 + (l + 64 < i ? i : l + 64)], dL[i]);
    if (l < ns) v[l] = v0;
    if (l + 64 < ns) v[l + 64] = v1;
}
// L y = v on the first ns columns with the rectangular update of rows up to n (dtrsv_n): v[i] -= L[i][j] y_j.
__device__ __forceinline__ void wave_solve_ln(double* v, const double* M, const double* dL, int nz, int ns, int n) {
    const int l = threadIdx.x & 63;
    double v0 = l < n ? v[l] : 0.0, v1 = l + 64 < n ? v[l + 64] : 0.0;
    const int r0 = l < n ? l : 0, r1 = l + 64 < n ? l + 64 : 0;  // in-range rows for the unconditional reads
    auto step = [&](int j, double m0, double m1, double d) {
        const double y = rdlane(j < 64 ? v0 : v1, j & 63) * d;
        if (l > j && l < n) v0 -= m0 * y;
        if (l + 64 > j && l + 64 < n) v1 -= m1 * y;
        if (l == j) v0 = y;
        if (l + 64 == j) v1 = y;
    };
    auto rd = [&](int j, int r) { return M[poff(j, nz) - j + (r > j ? r : j)]; };
    int j = 0;
    for (; j + 3 < ns; j += 4) {
        double m0[4], m1[4], d[4];
#pragma unroll
        for (int q = 0; q < 4; q++) {
            m0[q] = rd(j + q, r0);
            m1[q] = rd(j + q, r1);
            d[q] = dL[j + q];
        }
#pragma unroll
        for (int q = 0; q < 4; q++) step(j + q, m0[q], m1[q], d[q]);
    }
    for (; j < ns; j++) step(j, rd(j, r0), rd(j, r1), dL[j]);
    if (l < n) v[l] = v0;
    if (l + 64 < n) v[l + 64] = v1;
}

// One 4-pivot block B of a Cholesky held as 16x16 MFMA tiles (the C/D layout: register r at lane (g,c) holds tile
// row 4r+g, column c).  D is the diagonal tile in symmetric storage (register r = rows / columns 4r..4r+3, so the
// tile's row c is its column c); U[0..nU) are the tiles below it, transposed (register r at lane (g,c) = A[16(I+1)+c]
// [4r+g]: tile row c of U[I] is matrix row 16(I+1)+c).  The block's 4x4 diagonal is broadcast (DPP row_newbcast) and
// factorised redundantly in every lane (pivot clamp d > 1e-15 else 0, kernel_dpotrf_c99_lib4.c:555-640, 1/sqrt(d)
// from v_rsq_f64 + one refinement, hk::chol_inv), each lane solves its own row of the block column in D and in
// every U[I] (one row-group gather each, the reference's in-block operation order), and the rank-4 update of the
// block's later columns is one v_mfma_f64_16x16x4 per tile.  On return register B of D and of each U[I] holds the
// factor's block column (lane (g,c): L[row c][4B+g]; D's diagonal is d_g i_g = sqrt(d_g)) and invd the inverse
// diagonal at lanes c = 4B..4B+3.  T11 (optional, D-shaped): the trailing tile of the rows below, updated by
// -U[0] U[0]' (the two-tile Cholesky of the condensing).  A pivot index with a zero diagonal entry (padding, or a
// row that is not a column) clamps to a zero column.
template <int B, int NB, bool T11UPD>
__device__ __forceinline__ void tile_chol_block(hk::d4& D, hk::d4* U, int nU, hk::d4* T11, double& invd) {
    using hk::row_bcast;
    const int c = threadIdx.x & 15;
    double x[4];
    hk::rowgroup_gather(D[B], x);
    const double a00 = row_bcast<4 * B + 0>(x[0]);
    const double a10 = row_bcast<4 * B + 1>(x[0]), a11 = row_bcast<4 * B + 1>(x[1]);
    const double a20 = row_bcast<4 * B + 2>(x[0]), a21 = row_bcast<4 * B + 2>(x[1]);
    const double a22 = row_bcast<4 * B + 2>(x[2]);
    const double a30 = row_bcast<4 * B + 3>(x[0]), a31 = row_bcast<4 * B + 3>(x[1]);
    const double a32 = row_bcast<4 * B + 3>(x[2]), a33 = row_bcast<4 * B + 3>(x[3]);
    const double i0 = hk::chol_inv(a00);
    const double l10 = a10 * i0, l20 = a20 * i0, l30 = a30 * i0;
    const double y0 = x[0] * i0;
    const double i1 = hk::chol_inv(fma(-l10, l10, a11));
    const double l21 = fma(-l20, l10, a21) * i1, l31 = fma(-l30, l10, a31) * i1;
    const double y1 = fma(-y0, l10, x[1]) * i1;
    const double i2 = hk::chol_inv(fma(-l21, l21, fma(-l20, l20, a22)));
    const double l32 = fma(-l31, l21, fma(-l30, l20, a32)) * i2;
    const double y2 = fma(-y1, l21, fma(-y0, l20, x[2])) * i2;
    const double i3 = hk::chol_inv(fma(-l32, l32, fma(-l31, l31, fma(-l30, l30, a33))));
    const double y3 = fma(-y2, l32, fma(-y1, l31, fma(-y0, l30, x[3]))) * i3;
    const double yg = hk::sel_g(y0, y1, y2, y3);
    D[B] = yg;
    if ((c >> 2) == B) invd = hk::sel_q(i0, i1, i2, i3);
    const double a = c > 4 * B + 3 ? yg : 0.0;
    if (B < 3) D = hk::mfma(-a, a, D);
#pragma unroll
    for (int I = 0; I < NB; I++) {
        if (I < nU) {  // uniform
            double z[4];
            hk::rowgroup_gather(U[I][B], z);
            const double w0 = z[0] * i0;
            const double w1 = fma(-w0, l10, z[1]) * i1;
            const double w2 = fma(-w1, l21, fma(-w0, l20, z[2])) * i2;
            const double w3 = fma(-w2, l32, fma(-w1, l31, fma(-w0, l30, z[3]))) * i3;
            const double wg = hk::sel_g(w0, w1, w2, w3);
            U[I][B] = wg;
            if (B < 3) U[I] = hk::mfma(-a, wg, U[I]);  // A[row j][i] -= sum_k L[i][4B+k] L[row j][4B+k], i below
            if (T11UPD && I == 0) *T11 = hk::mfma(-wg, wg, *T11);
        }
    }
}

// C (m x n) = A (m x K) B (K x n) on v_mfma_f64_16x16x4: wave w takes output tiles w, w+4, .. (at most GM per
// wave, host-checked); a(i, k) / b(k, j) read the operands (LDS; 0 outside), out(i, j, v) stores a result after a
// workgroup barrier, so C may overwrite an operand.  All threads of the workgroup must call it.  The K chunks are the
// outer loop and the wave's tiles the inner one, so each chunk issues every tile's operand loads before their MFMAs:
// one LDS round trip per chunk for all tiles, and independent MFMAs back to back instead of one dependent chain per
// tile after another.
template <int GM, int KM, class FA, class FB, class FO>
__device__ __forceinline__ void mfma_gemm(int m, int n, int K, FA a, FB b, FO out) {
    const int lane = threadIdx.x & 63, wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), c16 = lane & 15,
              g4 = lane >> 4;
    const int nI = (m + 15) >> 4, nT = nI * ((n + 15) >> 4), nK = (K + 3) >> 2;
    int ra[GM], cb[GM];
    hk::d4 acc[GM];
#pragma unroll
    for (int u = 0; u < GM; u++) {
        const int t = wv + 4 * u, ti = t / nI;
        ra[u] = 16 * (t - ti * nI) + c16;
        cb[u] = 16 * ti + c16;
        acc[u] = hk::d4{0.0, 0.0, 0.0, 0.0};
    }
    // K chunks in groups of KG: every load of a group is issued before its MFMAs.  Loads are unconditional, at
    // clamped (valid) indices, followed by a select -- a conditional load is compiled to an exec-masked branch with
    // its own lgkmcnt wait per operand.  KM (the caller's bound on the chunk count, or 0) only sets the group size.
    constexpr int KG = KM == 0 ? 1 : (GM >= 8 ? 1 : (8 / GM < KM ? 8 / GM : KM));
    for (int kc0 = 0; kc0 < nK; kc0 += KG) {
        double av[KG][GM], bv[KG][GM];
#pragma unroll
        for (int j = 0; j < KG; j++) {
            const int kk = 4 * (kc0 + j) + g4, kq = kk < K ? kk : K - 1;
#pragma unroll
            for (int u = 0; u < GM; u++) {
                if (wv + 4 * u < nT) {  // uniform
                    const double x = a(ra[u] < m ? ra[u] : m - 1, kq), y = b(kq, cb[u] < n ? cb[u] : n - 1);
                    av[j][u] = (ra[u] < m && kk < K) ? x : 0.0;
                    bv[j][u] = (cb[u] < n && kk < K) ? y : 0.0;
                }
            }
        }
#pragma unroll
        for (int j = 0; j < KG; j++)
            if (kc0 + j < nK)  // uniform
#pragma unroll
                for (int u = 0; u < GM; u++)
                    if (wv + 4 * u < nT) acc[u] = hk::mfma(av[j][u], bv[j][u], acc[u]);
    }
    lds_bar();  // every operand read is done (the operands live in LDS)
#pragma unroll
    for (int u = 0; u < GM; u++) {
        if (wv + 4 * u < nT) {
#pragma unroll
            for (int r = 0; r < 4; r++) {
                const int row = ra[u] - c16 + g4 + 4 * r;
                if (row < m && cb[u] < n) out(row, cb[u], acc[u][r]);
            }
        }
    }
}

// sum_{j < n} a(j) b(j), accumulated in the order j = 0, 1, .. exactly as the plain loop (so bitwise the same
// result), with the operands of NB terms loaded before their multiply-adds: a global-memory dot product then costs
// one memory latency per NB terms instead of one per term.  a(j, ok) / b(j, ok) load term j (0 when !ok).
template <int NB = 8, class FA, class FB>
__device__ __forceinline__ double bdot(int n, FA a, FB b, double acc = 0.0) {
    for (int j0 = 0; j0 < n; j0 += NB) {
        double x[NB], y[NB];
#pragma unroll
        for (int u = 0; u < NB; u++) {
            const bool ok = j0 + u < n;
            x[u] = a(j0 + u, ok);
            y[u] = b(j0 + u, ok);
        }
#pragma unroll
        for (int u = 0; u < NB; u++)
            if (j0 + u < n) acc += x[u] * y[u];
    }
    return acc;
}

// Per-problem pointers of one wide Riccati call (already offset to the problem).
struct WideProb {
    const double *BAbt, *RSQ, *DCt;
    double *F, *ux, *pi, *Pb;               // factor (ws), solution, Pb
    const double *vb, *vq, *Qx, *qx;        // sv: optional b / q vectors and box / general terms
    const double *hb, *hq;                  // trs: b / q vectors (null: the augmented rows)
    int compute_pi, compute_Pb;
    bool dev_box;                           // sv: apply the box terms Qx / qx at idxb on the device
    int* kct;                               // LDS (nullable): per stage (KC_STRIDE) and 16-row tile of M, 1 + the last
                                            // DCt column with a nonzero entry in the tile's rows; then the stage's
                                            // 'recorded' flag
    bool kc_use;                            // kct is complete (a factorisation has scanned every chunk): use it
};

__device__ __forceinline__ WideProb wide_prob(const WideArgs& a, int p) {
    WideProb q;
    q.BAbt = a.BAbt + (long)p * a.sB;
    q.RSQ = a.RSQ ? a.RSQ + (long)p * a.sR : nullptr;
    q.DCt = a.DCt ? a.DCt + (long)p * a.sG : nullptr;
    q.F = a.ws + (long)p * a.sW;
    q.ux = a.ux + (long)p * a.sU;
    q.pi = a.pi + (long)p * a.sP;
    q.Pb = a.Pb ? a.Pb + (long)p * a.sP : nullptr;
    q.vb = a.vb ? a.vb + (long)p * a.sP : nullptr;
    q.vq = a.vq ? a.vq + (long)p * a.sU : nullptr;
    q.Qx = a.Qx ? a.Qx + (long)p * a.sC : nullptr;
    q.qx = a.qx ? a.qx + (long)p * a.sC : nullptr;
    q.hb = a.hb ? a.hb + (long)p * a.sP : nullptr;
    q.hq = a.hq ? a.hq + (long)p * a.sU : nullptr;
    q.compute_pi = a.compute_pi;
    q.compute_Pb = a.compute_Pb;
    q.dev_box = a.dev_box != 0;
    q.kct = nullptr;
    q.kc_use = false;
    return q;
}

// ------------------------------------------------------------------------------------------------
// Riccati factorisation + solve on wide stages (d_back_ric_rec_sv_tv_res).  Box / general terms and b / q
// come either pre-applied in the staged RSQrq / BAbt copies (the drop-in entry points, which apply the
// reference's in-place side effects on the host) or from WideProb's vectors (the wide IPM).
// Per stage k = N..0 (d_back_ric_rec.c:186-335):
//   W = BAbt_k Lxx_{k+1} (dtrmm_nt_u), Pb = Lxx (W_last)', W_last += l_{k+1,x} (dgead),
//   M = RSQrq_k + W W' (dsyrk) [+ DCt diag(Qx_g) DCt'], L_k = chol_aug(M) with the pivot clamp d > 1e-15
//   else 0 (kernel_dpotrf_c99_lib4.c:555-640): 16-column panels; the factor goes to HBM (and, for the
//   state block, to LDS as Lxx for stage k-1).
// Forward (:339-397): ux_k = -L_k^{-T}(l_k ...) over the u block (the whole block at k = 0),
//   x_{k+1} = b_k + BAbt_k' ux_k (dgemv_t), pi_k = Lxx_{k+1}(Lxx_{k+1}' x_{k+1} + l_{k+1,x}).
// ------------------------------------------------------------------------------------------------
// HK_WIDE_NOINLINE (probe builds only, tools/wide_noinline.sh): the two bodies as real calls
#ifdef HK_WIDE_NOINLINE
#define HK_WIDE_BODY __attribute__((noinline))
#else
#define HK_WIDE_BODY
#endif
#ifndef WSUB
#define WSUB(i) \
    do {        \
    } while (0)
#endif
#ifndef TSUB
#define TSUB(i) \
    do {        \
    } while (0)
#endif
__device__ HK_WIDE_BODY void wide_sv_body(const WideArgs& a, const WideProb& q) {
    extern __shared__ double sm[];
    const StTab st{reinterpret_cast<const WideStage*>(sm + a.offST)};  // filled by the kernel (wide_stage_table)
    const int tid = threadIdx.x;
    double* M = sm;
    double* W = sm + a.offW;
    double* X = sm + a.offX;
    double* v = sm + a.offV;
    const int ldW = a.ldW, ldX = a.ldX;
    const int lane = tid & 63, wv = tid >> 6, c16 = lane & 15, g4 = lane >> 4;  // MFMA lane coordinates
    const double* BAbt = q.BAbt;
    const double* RSQ = q.RSQ;
    double* F = q.F;
    double* ux = q.ux;
    double* pi = q.pi;
    double* Pb = q.Pb;

    for (int k = a.N; k >= 0; k--) {
        const WideStage s = st[k];
        const int nu = s.nu, nux = s.nu + s.nx, nz = nux + 1, nx1 = s.nx1;
        WSUB(0);
        dma_lower(M, RSQ + s.oR, s.sdR, nz, nux);
        dma_wait();
        if (q.vq || q.dev_box) {  // device-side q_k row and box terms (d_back_ric_rec.c:197-209, :249-291): the
            bar();           // staged RSQrq is the caller's original, so diag[idxb] = bd + Qx is a += Qx
            if (q.vq && !a.trf)
                for (int j = tid; j < nux; j += WT) M[poff(j, nz) + nux - j] = q.vq[s.oU + j];
            bar();
            if (q.dev_box)
                for (int l = tid; l < s.nb; l += WT) {
                    const int ii = a.idxb[s.oI + l];
                    M[poff(ii, nz)] += q.Qx[s.oD + l];
                    if (!a.trf) M[poff(ii, nz) + nux - ii] += q.qx[s.oD + l];
                }
        }
        if (k < a.N && !(a.skip & 4)) {
            WSUB(1);
            load_dense<8>(W, ldW, BAbt + s.oB, s.sdB, nz, nx1);
            bar();
            WSUB(2);
            if (a.trf) {  // trf factorises without the augmented row: the b row and the gradient row read as 0
                for (int j = tid; j < nux + nx1; j += WT) {
                    if (j < nx1) W[nux + j * ldW] = 0.0;
                    if (j < nux) M[poff(j, nz) + nux - j] = 0.0;
                }
                bar();
            } else if (q.vb) {  // update_b: b_k from a vector (d_back_ric_rec.c:249-251)
                for (int j = tid; j < nx1; j += WT) W[nux + j * ldW] = q.vb[s.oP + j];
                bar();
            }
            // W = BAbt_k Lxx_{k+1} (dtrmm_nt_u) on MFMA: 16x16 output tiles, K over the nx1 columns of BAbt; the
            // tiles are kept in registers and written back over BAbt after a barrier
            {
                const int nI = (nz + 15) >> 4, nJ = (nx1 + 15) >> 4, nK = (nx1 + 3) >> 2, nT = nI * nJ;
                const int w = __builtin_amdgcn_readfirstlane(wv);
                hk::d4 acc[WS_TILES];
                int ra[WS_TILES], cb[WS_TILES];
#pragma unroll
                for (int u = 0; u < WS_TILES; u++) {
                    acc[u] = hk::d4{0.0, 0.0, 0.0, 0.0};
                    const int t = w + 4 * u, J = t / nI;
                    ra[u] = 16 * (t - J * nI) + c16;
                    cb[u] = 16 * J + c16;
                }
                // K chunks outer, the wave's tiles inner (independent MFMAs back to back); operand loads at clamped
                // indices and a select (a conditional LDS load becomes an exec-masked branch with its own wait)
                for (int kc = 0; kc < nK; kc++) {
                    const int kk = 4 * kc + g4, kq = kk < nx1 ? kk : nx1 - 1;
#pragma unroll
                    for (int u = 0; u < WS_TILES; u++) {
                        if (w + 4 * u < nT) {  // uniform
                            const double x = W[(ra[u] < nz ? ra[u] : nz - 1) + kq * ldW];
                            const double y = X[kq + (cb[u] < nx1 ? cb[u] : nx1 - 1) * ldX];
                            acc[u] = hk::mfma((ra[u] < nz && kk < nx1) ? x : 0.0, (cb[u] < nx1 && kk < nx1) ? y : 0.0,
                                              acc[u]);
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
            WSUB(3);
            if (q.compute_Pb && tid < nx1) {  // Pb_k = Lxx (Lxx' b_k) from W's last row before + l
                double acc = 0.0;
                for (int j = 0; j <= tid; j++) acc += X[tid + j * ldX] * W[nux + j * ldW];
                Pb[s.oP + tid] = acc;
            }
            bar();
            if (tid < nx1) W[nux + tid * ldW] += X[nx1 + tid * ldX];
            bar();
            WSUB(4);
            // M += W W' (dsyrk) on MFMA over the lower 16x16 tiles
            {
                const int nI = (nz + 15) >> 4, nK = (nx1 + 3) >> 2, nT = nI * (nI + 1) / 2;
                for (int t = wv; t < nT; t += 4) {
                    int I = 0;
                    while ((I + 1) * (I + 2) / 2 <= t) I++;
                    const int J = t - I * (I + 1) / 2;
                    const int ra = 16 * I + c16, rb = 16 * J + c16;
                    const int rac = ra < nz ? ra : nz - 1, rbc = rb < nux ? rb : nux - 1;
                    hk::d4 acc = {0.0, 0.0, 0.0, 0.0};
                    for (int kc = 0; kc < nK; kc++) {
                        const int kk = 4 * kc + g4, kq = kk < nx1 ? kk : nx1 - 1;
                        const double x = W[rac + kq * ldW], y = W[rbc + kq * ldW];  // unconditional, then a select
                        const double av = (ra < nz && kk < nx1) ? x : 0.0;
                        const double bv = (rb < nux && kk < nx1) ? y : 0.0;
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
        WSUB(5);
        if (q.DCt && s.ng > 0) {
            // general constraints: M += [DCt diag(Qx_g) ; qx_g'] DCt' over the lower tiles on MFMA, K = ng
            // (d_back_ric_rec.c:210-231, :292-317); DCt is read from HBM (nux x ng may exceed LDS)
            bar();
            WSUB(6);
            const double* D = q.DCt + s.oG;
            const double* Qg = q.Qx + s.oD + s.pnb;
            const double* qg = q.qx + s.oD + s.pnb;
            const int ng = s.ng, sdG = s.sdG, nI = (nz + 15) >> 4, nK = (ng + 3) >> 2, nT = nI * (nI + 1) / 2;
            const int ldS = 16 * nI;
            const float rS = 1.0f / ldS;
            if (nT <= 4 * DT_TILES && DS_LD * ldS + 32 <= a.offV - a.offW) {  // uniform
                // K blocks of 16 constraints staged in LDS (W and X are free between the syrk and the Cholesky):
                // the block's DCt columns (zero beyond nux / ng), diag(Qx_g) and the qx_g entries, one memory round
                // trip per block for the whole workgroup.  Each wave keeps its output tiles in registers across
                // the blocks; the MFMA chain of a tile runs over the same K chunks in the same order as the direct
                // loop below, so M gets the same sums.
                double* Ds = W;  // Ds[kk + DS_LD i]: a chunk's four columns are compile-time offsets from a row
                double* dqs = W + DS_LD * ldS;
                double* qrs = dqs + 16;
                // In an IPM the DCt blocks are the same in every factorisation and often block-staircase (the
                // condensed problem's state boxes of inner stage s have no entries above its nu_tmp): the first
                // factorisation records per 16-row tile of M the last column with a nonzero entry in the tile's rows
                // (kct), the later ones skip the 16-column K blocks beyond it for tiles whose B operand lies in those
                // rows -- products of exact zeros, so M is unchanged.
                int* kck = q.kct ? q.kct + k * KC_STRIDE : nullptr;
                const bool kcu = kck && q.kc_use, kcr = kck && !q.kc_use;  // uniform
                hk::d4 acc[DT_TILES];
                int kcl[DT_TILES], tI[DT_TILES], tJ[DT_TILES];  // wave-uniform: the tile's K limit and block row / col
#pragma unroll
                for (int u = 0; u < DT_TILES; u++) {
                    acc[u] = hk::d4{0.0, 0.0, 0.0, 0.0};
                    int I = 0;
                    const int t = wv + 4 * u;
                    while ((I + 1) * (I + 2) / 2 <= t) I++;
                    tI[u] = I;
                    tJ[u] = t - I * (I + 1) / 2;
                    kcl[u] = t >= nT ? 0 : kcu ? __builtin_amdgcn_readfirstlane(kck[tJ[u]]) : ng;
                }
                // the next block's loads are issued before this block's MFMAs, so their latency hides behind them
                double r[8], dq, qq;
                auto stage_load = [&](int kb) {
#pragma unroll
                    for (int u = 0; u < 8; u++) {
                        const int e = u * WT + tid, kk = fdiv(e, rS), i = e - kk * ldS;
                        r[u] = gld(D, p4i(i, kb + kk, sdG), e < 16 * ldS && i < nux && kb + kk < ng);
                    }
                    dq = gld(Qg, kb + (tid & 15), tid < 16 && kb + tid < ng);
                    qq = gld(qg, kb + (tid & 15), tid < 16 && kb + tid < ng);
                };
                for (int kb = 0; kb < ng; kb += 16) {
                    stage_load(kb);
                    bar();  // the previous block's operands are read
#pragma unroll
                    for (int u = 0; u < 8; u++) {
                        const int e = u * WT + tid, kk = fdiv(e, rS), i = e - kk * ldS;
                        if (e < 16 * ldS) Ds[kk + DS_LD * i] = r[u];
                        if (kcr && e < 16 * ldS && r[u] != 0.0) atomicMax(&kck[i >> 4], kb + kk + 1);
                    }
                    if (tid < 16) {
                        dqs[tid] = dq;
                        qrs[tid] = qq;
                    }
                    lds_bar();
                    // a tile runs the block if its B rows have a nonzero column in it (the block's chunks beyond the
                    // limit are products of zeros); the four chunks' operands are read before the four MFMAs
#pragma unroll
                    for (int u = 0; u < DT_TILES; u++) {
                        if (kb < kcl[u]) {
                            int ti = __builtin_amdgcn_readfirstlane(tI[u]), tj = __builtin_amdgcn_readfirstlane(tJ[u]);
                            asm volatile("" : "+s"(ti), "+s"(tj));  // tile addresses per block, not hoisted (VGPRs)
                            const int ra = 16 * ti + c16;
                            const double* pa = Ds + g4 + DS_LD * ra;
                            const double* pb = Ds + g4 + DS_LD * (16 * tj + c16);
                            double av[4], bv[4];
                            // row nux of Ds is zero: its A operand is qx_g (0 in a pure factorisation), the others'
                            // is diag(Qx_g) DCt.  qx_g is read on every row and selected as a value (v_cndmask, no
                            // branch over the reads); a select rather than a product with 0 keeps a non-finite qx_g
                            // out of the other rows, as in the reference.  Finite values: the same two
                            // roundings as the former fma(qx_g, 0 or 1, product), so the same sums.
                            const bool sq = ra == nux && !a.trf;
#pragma unroll
                            for (int kc = 0; kc < 4; kc++) {
                                const double qv = qrs[4 * kc + g4];
                                av[kc] = __dadd_rn(sq ? qv : 0.0, __dmul_rn(pa[4 * kc], dqs[4 * kc + g4]));
                                bv[kc] = pb[4 * kc];
                            }
#pragma unroll
                            for (int kc = 0; kc < 4; kc++) acc[u] = hk::mfma(av[kc], bv[kc], acc[u]);
                        }
                    }
                }
                if (kcr && tid == 0) kck[KC_STRIDE - 1] = 1;  // this stage's limits are recorded
#pragma unroll
                for (int u = 0; u < DT_TILES; u++) {
                    if (wv + 4 * u < nT) {
                        const int col = 16 * tJ[u] + c16;
#pragma unroll
                        for (int rr = 0; rr < 4; rr++) {
                            const int row = 16 * tI[u] + g4 + 4 * rr;
                            if (row < nz && col < nux && row >= col) M[poff(col, nz) + row - col] += acc[u][rr];
                        }
                    }
                }
            } else
            for (int t = wv; t < nT; t += 4) {
                int I = 0;
                while ((I + 1) * (I + 2) / 2 <= t) I++;
                const int J = t - I * (I + 1) / 2;
                const int ra = 16 * I + c16, rb = 16 * J + c16;
                hk::d4 acc = {0.0, 0.0, 0.0, 0.0};
                // K chunks in batches of 8: every operand of a batch is loaded before its MFMAs (the MFMA chain
                // keeps the chunk order, so the sum is the same as one chunk at a time)
                for (int kc0 = 0; kc0 < nK; kc0 += 8) {
                    double avs[8], bvs[8];
#pragma unroll
                    for (int u = 0; u < 8; u++) {
                        const int kk = 4 * (kc0 + u) + g4;
                        const bool kok = kk < ng;
                        const double dq = gld(Qg, kk, kok);
                        double av = gld(D, p4i(ra, kk, sdG), kok && ra < nux) * dq;
                        if (ra == nux) av = a.trf ? 0.0 : gld(qg, kk, kok);
                        avs[u] = av;
                        bvs[u] = gld(D, p4i(rb, kk, sdG), kok && rb < nux);
                    }
#pragma unroll
                    for (int u = 0; u < 8; u++)
                        if (kc0 + u < nK) acc = hk::mfma(avs[u], bvs[u], acc);
                }
                const int col = 16 * J + c16;
#pragma unroll
                for (int r = 0; r < 4; r++) {
                    const int row = 16 * I + g4 + 4 * r;
                    if (row < nz && col < nux && row >= col) M[poff(col, nz) + row - col] += acc[r];
                }
            }
        }
        bar();
        WSUB(7);
        // Cholesky with the augmented row, blocked by 16-column panels: the four waves factor the panel as MFMA tiles
        // (each its own rows, no workgroup barrier inside), then apply its rank-16 update to the trailing lower
        // tiles on MFMA
        double* Lk = F + s.oL;
        double* dL = Lk + poff(nux, nz);
        for (int p0 = 0; p0 < ((a.skip & 2) ? 0 : nux); p0 += 16) {
            const int pe = p0 + 16 < nux ? p0 + 16 : nux;
            {
                // the panel as MFMA tiles (tile_chol_block): D = rows / columns p0..p0+15, factorised redundantly
                // by every wave; the tiles below it (rows p0+16(I+1).., nz <= 128: I < 7) are solved by wave I % 4
                // (U[t] = tile wv + 4t); entries outside the panel's columns read as 0
                const int pw = pe - p0, nUt = (nz - p0 - 1) >> 4, g = lane >> 4;
                const int w = __builtin_amdgcn_readfirstlane(wv);
                const int nU = (w < nUt) + (w + 4 < nUt);
                auto ld = [&](int r, int j) -> double {  // A[r][j], r >= j
                    return (j < pe && r < nz) ? M[poff(j, nz) + r - j] : 0.0;
                };
                hk::d4 D, U[2];
#pragma unroll
                for (int r = 0; r < 4; r++) {
                    const int i = p0 + 4 * r + g, j = p0 + c16;
                    D[r] = i >= j ? ld(i, j) : ld(j, i);
#pragma unroll
                    for (int t = 0; t < 2; t++)
                        U[t][r] = t < nU ? ld(p0 + 16 * (w + 4 * t + 1) + c16, p0 + 4 * r + g) : 0.0;
                }
                double invd = 0.0;
                if (pw > 0) tile_chol_block<0, 2, false>(D, U, nU, nullptr, invd);
                if (pw > 4) tile_chol_block<1, 2, false>(D, U, nU, nullptr, invd);
                if (pw > 8) tile_chol_block<2, 2, false>(D, U, nU, nullptr, invd);
                if (pw > 12) tile_chol_block<3, 2, false>(D, U, nU, nullptr, invd);
                auto put = [&](int row, int j, double v) {
                    if (row < nz) {
                        M[poff(j, nz) + row - j] = v;
                        if (j >= nu) X[(row - nu) + (j - nu) * ldX] = v;
                    }
                };
#pragma unroll
                for (int r = 0; r < 4; r++) {
                    const int j = p0 + 4 * r + g;
                    if (j < pe) {
                        if (w == 0 && c16 >= 4 * r + g) put(p0 + c16, j, D[r]);
#pragma unroll
                        for (int t = 0; t < 2; t++)
                            if (t < nU) put(p0 + 16 * (w + 4 * t + 1) + c16, j, U[t][r]);
                    }
                }
                if (w == 0 && g == 0 && p0 + c16 < pe) M[poff(nux, nz) + p0 + c16] = invd;
            }
            bar();
            WSUB(8);
            if (pe < nux) {  // trailing update: M[i, jj] -= sum_{k in panel} L[i, k] L[jj, k], tiles from pe
                const int T0 = pe >> 4, nI = (nz + 15) >> 4, nTI = nI - T0;
                const int nT = nTI * (nTI + 1) / 2, nK = (pe - p0 + 3) >> 2;
                for (int t = wv; t < nT; t += 4) {
                    int I = 0;
                    while ((I + 1) * (I + 2) / 2 <= t) I++;
                    const int J = t - I * (I + 1) / 2;
                    const int ra = 16 * (T0 + I) + c16, rb = 16 * (T0 + J) + c16;
                    hk::d4 acc = {0.0, 0.0, 0.0, 0.0};
                    const int rac = ra < nz ? ra : nz - 1, rbc = rb < nux ? rb : nux - 1;
                    // the panel's (at most four) K chunks: every operand read before the first MFMA
                    double av[4], bv[4];
#pragma unroll
                    for (int kc = 0; kc < 4; kc++) {
                        const int kk = p0 + 4 * kc + g4;
                        const bool kok = kk < pe;
                        const int kq = kok ? kk : pe - 1, ck = poff(kq, nz) - kq;
                        const double x = M[ck + rac], y = M[ck + rbc];  // unconditional (rows >= pe > kq), then a select
                        av[kc] = (ra < nz && kok) ? x : 0.0;
                        bv[kc] = (rb < nux && kok) ? y : 0.0;
                    }
#pragma unroll
                    for (int kc = 0; kc < 4; kc++)
                        if (kc < nK) acc = hk::mfma(av[kc], bv[kc], acc);
                    const int col = 16 * (T0 + J) + c16;
#pragma unroll
                    for (int r = 0; r < 4; r++) {
                        const int row = 16 * (T0 + I) + g4 + 4 * r;
                        if (row < nz && col < nux && row >= col) M[poff(col, nz) + row - col] -= acc[r];
                    }
                }
                bar();
            }
            WSUB(9);
        }
        // the factor (packed columns + 1/diag) to HBM in one coalesced sweep
        for (int e = tid; e < poff(nux, nz) + nux; e += WT) Lk[e] = M[e];
        (void)dL;
        // strictly upper part of the copied Lxx stays zero (the next stage's MFMA trmm reads whole tiles)
        const float rnx = 1.0f / s.nx;
        for (int e = tid; e < s.nx * s.nx; e += WT) {
            const int cc = fdiv(e, rnx), i = e - cc * s.nx;
            if (i < cc) X[i + cc * ldX] = 0.0;
        }
        bar();
        WSUB(10);
    }

    // forward substitution: L_k (packed + 1/diag) and BAbt_k are staged into LDS (M, W) per stage by DMA, each issued
    // as soon as its buffer is free -- L_{k+1} while x_{k+1} is formed, BAbt_{k+1} during pi_k and stage k+1's solve --
    // with LDS-only barriers in between so that the copies stay in flight
    double* tmp = X;  // Lxx is no longer needed: nx1 doubles of scratch for pi
    const int nfw = (a.skip & 1) || a.trf ? 0 : a.N;
    if (nfw > 0) {
        const WideStage s0 = st[0];
        const int nz0 = s0.nu + s0.nx + 1;
        dma_copy_any<WT>(M, F + s0.oL, poff(nz0 - 1, nz0) + nz0 - 1, tid);
        dma_dense(W, ldW, BAbt + s0.oB, s0.sdB, nz0, s0.nx1);
        dma_wait();
        bar();
    }
    for (int k = 0; k < nfw; k++) {
        const WideStage s = st[k];
        const int nux = s.nu + s.nx, nz = nux + 1, nx1 = s.nx1, nu1 = s.nu1;
        const int ns = k == 0 ? nux : s.nu;
        const double* dL = M + poff(nux, nz);
        // v[0:ns] = -l[0:ns] - L[ns:nux, 0:ns]' v[ns:nux]   (v[ns:nux] = x_k from the previous stage)
        for (int j = tid; j < ns; j += WT) {
            const int cj = poff(j, nz) - j;
            double r = -M[cj + nux];
            #pragma unroll 8
            for (int m = ns; m < nux; m++) r -= M[cj + m] * v[m];
            v[j] = r;
        }
        lds_bar();
        // back substitution with L[0:ns, 0:ns]' (inv_diag multiply), column-oriented inside wave 0
        if (tid < 64) wave_solve_lt(v, M, dL, nz, ns);
        dma_wait();  // BAbt_k (issued during the previous stage) has landed, every wave's part after the barrier
        bar();
        const WideStage s1 = st[k + 1];
        const int nux1 = nu1 + nx1, nz1 = nux1 + 1;
        dma_copy_any<WT>(M, F + s1.oL, poff(nux1, nz1) + nux1, tid);  // L_k is done with
        for (int j = tid; j < nux; j += WT) ux[s.oU + j] = v[j];
        // x_{k+1} = b_k + BAbt_k' ux_k
        double xn = 0.0;
        if (tid < nx1) {
            xn = q.vb ? q.vb[s.oP + tid] : W[nux + tid * ldW];  // b_k: the update_b vector when given
            #pragma unroll 8
            for (int i = 0; i < nux; i++) xn += W[i + tid * ldW] * v[i];
        }
        lds_bar();  // W is read
        if (tid < nx1) {
            v[nu1 + tid] = xn;
            ux[s1.oU + nu1 + tid] = xn;
        }
        const int nB = k + 1 < nfw ? dma_dense(W, ldW, BAbt + s1.oB, s1.sdB, nz1, st[k + 1].nx1) : 0;
        dma_wait_keep(nB);  // L_{k+1} has landed (this wave's part); BAbt_{k+1} stays in flight
        lds_bar();
        if (q.compute_pi) {  // pi_k = Lxx (Lxx' x + l), Lxx of stage k+1 (rows / cols nu1..)
            if (tid < nx1) {
                const int cj = poff(nu1 + tid, nz1) - (nu1 + tid);
                double tj = M[cj + nux1];
                #pragma unroll 8
                for (int i = tid; i < nx1; i++) tj += M[cj + nu1 + i] * v[nu1 + i];
                tmp[tid] = tj;
            }
            lds_bar();
            if (tid < nx1) {
                double acc = 0.0;
                #pragma unroll 8
                for (int j = 0; j <= tid; j++) acc += M[poff(nu1 + j, nz1) + tid - j] * tmp[j];
                pi[s.oP + tid] = acc;
            }
            lds_bar();
        }
    }
    dma_wait();
    WSUB(11);
}

// ------------------------------------------------------------------------------------------------
// d_back_ric_rec_trs_tv_res on wide stages (d_back_ric_rec.c:564-791, restated in oracle/hpmpc_oracle.c):
// backward, per stage k = N..0: g_k = q_k + qx at idxb (+ DCt qx_g); v_k = g_k + BAbt_k (Pb_k + v_{k+1,x})
// (k < N), with Pb_k = Lxx_{k+1}(Lxx_{k+1}' b_k); then L_k's n-form solve on the first nu_k columns (all of
// stage 0) with the rectangular update of the later rows.  Forward as the sv forward,
// pi_k = Lxx(Lxx' x_{k+1}) + v_{k+1,x}.  The processed v_k are parked in ux (the forward overwrites them).
// ------------------------------------------------------------------------------------------------
__device__ HK_WIDE_BODY void wide_trs_body(const WideArgs& a, const WideProb& q) {
    extern __shared__ double sm[];
    const StTab st{reinterpret_cast<const WideStage*>(sm + a.offST)};  // filled by the kernel (wide_stage_table)
    const int tid = threadIdx.x;
    double* M = sm;
    double* W = sm + a.offW;
    double* X = sm + a.offX;  // w = Pb + v_{k+1,x} (backward) / pi scratch (forward)
    double* v = sm + a.offV;
    const int ldW = a.ldW;
    const double* BAbt = q.BAbt;
    const double* F = q.F;
    double* ux = q.ux;
    double* pi = q.pi;
    double* Pb = q.Pb;
    const double* qx = q.qx;
    // b_k / q_k: the given vectors, or the augmented rows of BAbt_k / RSQrq_k
    auto bk = [&](const WideStage& sk, int j) {
        return q.hb ? q.hb[sk.oP + j] : P4(BAbt + sk.oB, sk.sdB, sk.nu + sk.nx, j);
    };
    auto qk = [&](const WideStage& sk, int i) {
        return q.hq ? q.hq[sk.oU + i] : P4(q.RSQ + sk.oR, sk.sdR, sk.nu + sk.nx, i);
    };
    for (int k = a.N; k >= 0; k--) {
        const WideStage s = st[k];
        const int nux = s.nu + s.nx, nz = nux + 1, nx1 = s.nx1;
        const int ns = k == 0 ? nux : s.nu;
        TSUB(0);
        load_flat<16>(M, F + s.oL, poff(nux, nz) + nux);
        if (k < a.N) load_dense<8>(W, ldW, BAbt + s.oB, s.sdB, nux, nx1);
        for (int i = tid; i < nux; i += WT) v[i] = qk(s, i);
        if (k > 0)  // b_{k-1} for Pb_{k-1} into W's unused row nux, read with the other loads of the stage
            for (int i = tid; i < s.nx; i += WT) W[nux + i * ldW] = bk(st[k - 1], i);
        bar();
        TSUB(1);
        for (int l = tid; l < s.nb; l += WT) v[a.idxb[s.oI + l]] += qx[s.oD + l];  // distinct indices (as the sv)
        bar();
        if (q.DCt && s.ng > 0) {  // + DCt qx_g (dgemv_n_lib, d_back_ric_rec.c:620-633)
            // nch lanes of one wave per row, each summing a contiguous column chunk (12 loads in flight per batch),
            // the chunk sums gathered by the row's first lane; columns past the last nonzero of the row's 16-row
            // tile (kct, recorded by the factorisation) are products of zeros and skipped
            const double* D = q.DCt + s.oG;
            const double* qg = qx + s.oD + s.pnb;
            const int nch = nux <= 64 ? 4 : nux <= 84 ? 3 : nux <= 128 ? 2 : 1, R = 64 / nch;
            const int w = tid >> 6, l = tid & 63, il = l / nch, ch = l - il * nch, i = w * R + il;
            const int* kck = q.kct ? q.kct + k * KC_STRIDE : nullptr;
            const bool kcu = kck && q.kc_use && __builtin_amdgcn_readfirstlane(kck[KC_STRIDE - 1]) != 0;
            const bool row = il < R && i < nux;
            const int lim = (kcu && row) ? kck[i >> 4] : s.ng;
            const int cs = (s.ng + nch - 1) / nch, g0 = ch * cs, g1 = min(g0 + cs, lim);
            const double part = row ? bdot<12>(
                                          g1 - g0, [&](int g, bool ok) { return gld(D, p4i(i, g0 + g, s.sdG), ok); },
                                          [&](int g, bool ok) { return gld(qg, g0 + g, ok); })
                                    : 0.0;
            double c = 0.0;
            for (int h = 0; h < nch; h++) c += __shfl(part, il * nch + h);  // chunk order
            if (row && ch == 0) v[i] += c;
            bar();
        }
        TSUB(2);
        if (k < a.N) {
            double c = 0.0;
            if (tid < nux)
                #pragma unroll 8
                for (int j = 0; j < nx1; j++) c += W[tid + j * ldW] * X[j];
            bar();
            if (tid < nux) v[tid] += c;
            bar();
            // n-form solve on the first ns columns with the rectangular update (column-oriented, one wave)
            const double* dL = M + poff(nux, nz);
            if (tid < 64) wave_solve_ln(v, M, dL, nz, ns, nux);
            bar();
        }
        TSUB(3);
        for (int i = tid; i < nux; i += WT) ux[s.oU + i] = v[i];
        if (k > 0) {  // w for stage k-1: Pb_{k-1} = Lxx_k (Lxx_k' b_{k-1}), plus v_{k,x}
            const WideStage sp = st[k - 1];
            const int nu = s.nu, nx = s.nx;
            double t = 0.0;
            if (tid < nx) {
                const int cj = poff(nu + tid, nz) - (nu + tid);
                #pragma unroll 8
                for (int i = tid; i < nx; i++) t += M[cj + nu + i] * W[nux + i * ldW];
            }
            bar();
            if (tid < nx) W[tid] = t;  // W is free: scratch
            bar();
            if (tid < nx) {
                double acc = 0.0;
                #pragma unroll 8
                for (int j = 0; j <= tid; j++) acc += M[poff(nu + j, nz) + tid - j] * W[j];
                if (q.compute_Pb) Pb[sp.oP + tid] = acc;
                X[tid] = (q.compute_Pb ? acc : Pb[sp.oP + tid]) + v[nu + tid];
            }
        }
        bar();
        TSUB(4);
    }
    // forward: as the sv forward, L_{k+1} and BAbt_{k+1} by DMA as soon as their buffers are free, the stage's vector
    // reads issued at its top, LDS-only barriers while the copies are in flight
    if (a.N > 0) {
        const WideStage s0 = st[0];
        const int nz0 = s0.nu + s0.nx + 1;
        dma_copy_any<WT>(M, F + s0.oL, poff(nz0 - 1, nz0) + nz0 - 1, tid);
        dma_dense(W, ldW, BAbt + s0.oB, s0.sdB, nz0 - 1, s0.nx1);
        load_flat<4>(v, ux + s0.oU, nz0 - 1);
        dma_wait();
        bar();
    }
    for (int k = 0; k < a.N; k++) {
        const WideStage s = st[k], s1 = st[k + 1];
        const int nux = s.nu + s.nx, nz = nux + 1, nx1 = s.nx1, nu1 = s.nu1;
        const int ns = k == 0 ? nux : s.nu;
        const double* dL = M + poff(nux, nz);
        TSUB(0);
        double pk = 0.0, bq = 0.0;
        if (tid < nx1) {
            pk = ux[s1.oU + nu1 + tid];  // v_{k+1,x} of the backward, before x_{k+1} replaces it
            bq = bk(s, tid);
        }
        const double un = tid < nu1 ? ux[s1.oU + tid] : 0.0;  // the backward's processed u part of stage k+1
        for (int j = tid; j < ns; j += WT) v[j] = -v[j];
        lds_bar();
        double r = 0.0;
        if (tid < ns) {  // - L[ns:nux, 0:ns]' x_k
            const int cj = poff(tid, nz) - tid;
            r = v[tid];
            #pragma unroll 8
            for (int m = ns; m < nux; m++) r -= M[cj + m] * v[m];
        }
        lds_bar();
        if (tid < ns) v[tid] = r;
        lds_bar();
        TSUB(5);
        if (tid < 64) wave_solve_lt(v, M, dL, nz, ns);
        dma_wait();  // BAbt_k (issued during the previous stage) has landed, every wave's part after the barrier
        bar();
        TSUB(6);
        const int nux1 = nu1 + nx1, nz1 = nux1 + 1;
        dma_copy_any<WT>(M, F + s1.oL, poff(nux1, nz1) + nux1, tid);  // L_k is done with
        for (int j = tid; j < nux; j += WT) ux[s.oU + j] = v[j];
        double xn = 0.0;
        if (tid < nx1) {
            xn = bq;
            #pragma unroll 8
            for (int i = 0; i < nux; i++) xn += W[i + tid * ldW] * v[i];
        }
        lds_bar();  // W and v are read
        // v <- stage k+1: the backward's processed u part, and the actual state x_{k+1}
        if (tid < nu1) v[tid] = un;
        if (tid < nx1) v[nu1 + tid] = xn;
        const int nB = k + 1 < a.N ? dma_dense(W, ldW, BAbt + s1.oB, s1.sdB, nux1, st[k + 1].nx1) : 0;
        dma_wait_keep(nB);  // L_{k+1} has landed (this wave's part); BAbt_{k+1} stays in flight
        lds_bar();
        TSUB(7);
        if (q.compute_pi) {
            if (tid < nx1) {
                const int cj = poff(nu1 + tid, nz1) - (nu1 + tid);
                double tj = 0.0;
                #pragma unroll 8
                for (int i = tid; i < nx1; i++) tj += M[cj + nu1 + i] * v[nu1 + i];
                X[tid] = tj;
            }
            lds_bar();
            if (tid < nx1) {
                double acc = 0.0;
                #pragma unroll 8
                for (int j = 0; j <= tid; j++) acc += M[poff(nu1 + j, nz1) + tid - j] * X[j];
                pi[s.oP + tid] = acc + pk;
            }
            lds_bar();
        }
        TSUB(8);
    }
    dma_wait();
    if (tid < st[a.N].nx) ux[st[a.N].oU + tid] = v[tid];
}

}  // namespace
