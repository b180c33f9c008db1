// hk_prims.h -- wave64 cross-lane primitives for the MI355X (gfx950) Riccati/IPM kernels.
//
// One problem is owned by one wavefront.  A stage's (nu+nx) x (nu+nx) block lives in the f64 MFMA
// C/D register layout of v_mfma_f64_16x16x4_f64 ("tile layout"):
//     lane l = 16*g + c  (g = l>>4 in 0..3 "row group", c = l&15 "column"),
//     register r in 0..3 holds element (row g+4r, col c).
// Vectors use one of two replicated layouts:
//     col layout : one double per lane, value v[c]           (identical in the 4 row groups)
//     row layout : double[4] per lane,  value v[g+4r] in r   (identical in the 16 columns)
// Every primitive below keeps replicated values bitwise identical across their replicas.
#pragma once
#include <hip/hip_runtime.h>

namespace hk {

// Diagnostic build only (-DHK_STAMPS): s_memtime stamps of one (problem, stage) into a debug buffer.
#ifdef HK_STAMPS
__device__ unsigned long long* g_dbg;
__device__ int g_dbg_stage;
#define HK_STAMP(slot, k)                                                                  \
    do {                                                                                   \
        unsigned long long t_;                                                             \
        __builtin_amdgcn_sched_barrier(0);                                                 \
        asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t_)::"memory");         \
        __builtin_amdgcn_sched_barrier(0);                                                 \
        if (g_dbg && blockIdx.x == 0 && (k) == g_dbg_stage && (threadIdx.x & 63) == 0)     \
            g_dbg[slot] = t_;                                                              \
    } while (0)
#else
#define HK_STAMP(slot, k) \
    do {                  \
    } while (0)
#endif

typedef double d4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ int lane_id() { return threadIdx.x & 63; }

__device__ __forceinline__ double mk(int hi, int lo) { return __hiloint2double(hi, lo); }

// DPP move of a double; CTRL is the DPP control word.  row_newbcast (0x150 + lane) is one v_mov_b64_dpp
// on gfx950 (DPP64); the other controls split into two v_mov_b32_dpp.
template <int CTRL>
__device__ __forceinline__ double dpp_mov(double x) {
    const long v = __builtin_bit_cast(long, x);
    return __builtin_bit_cast(double, (long)__builtin_amdgcn_mov_dpp(v, CTRL, 0xf, 0xf, true));
}

// broadcast lane P of every 16-lane row to the whole row (DPP row_newbcast, gfx90a+)
template <int P>
__device__ __forceinline__ double row_bcast(double x) { return dpp_mov<0x150 + P>(x); }

// value of lane `src` (wave-uniform) as a scalar
__device__ __forceinline__ double readlane(double x, int src) {
    int lo = __builtin_amdgcn_readlane(__double2loint(x), src);
    int hi = __builtin_amdgcn_readlane(__double2hiint(x), src);
    return mk(hi, lo);
}

// Broadcast row group GS (lanes 16*GS..16*GS+15) to all four row groups, lane-column preserving:
// result at lane (g,c) = x at lane (GS,c).  v_permlane32_swap + v_permlane16_swap (gfx950).
template <int GS>
__device__ __forceinline__ double rowgroup_bcast(double x) {
    int lo = __double2loint(x), hi = __double2hiint(x);
    // step 1: replicate the 32-lane half that holds GS
    auto a = __builtin_amdgcn_permlane32_swap(lo, lo, false, false);
    auto b = __builtin_amdgcn_permlane32_swap(hi, hi, false, false);
    int lo1 = (GS < 2) ? (int)a[0] : (int)a[1];
    int hi1 = (GS < 2) ? (int)b[0] : (int)b[1];
    // step 2: replicate the 16-lane row (even/odd) inside the half
    auto c = __builtin_amdgcn_permlane16_swap(lo1, lo1, false, false);
    auto d = __builtin_amdgcn_permlane16_swap(hi1, hi1, false, false);
    int lo2 = (GS % 2 == 0) ? (int)c[0] : (int)c[1];
    int hi2 = (GS % 2 == 0) ? (int)d[0] : (int)d[1];
    return mk(hi2, lo2);
}

// Branch-free 4-way selects.  Written as bit tests on the lane index so that the optimiser keeps
// them as v_cndmask (equality chains on one variable get turned into a switch, i.e. exec-mask
// branches).  sel_g: by row group g = lane >> 4; sel_q: by q = c & 3 (c = lane & 15).
__device__ __forceinline__ double sel_g(double a0, double a1, double a2, double a3) {
    const int l = __builtin_amdgcn_workitem_id_x() & 63;
    const bool b0 = (l & 16) != 0, b1 = (l & 32) != 0;
    const double lo = b0 ? a1 : a0, hi = b0 ? a3 : a2;
    return b1 ? hi : lo;
}
__device__ __forceinline__ double sel_q(double a0, double a1, double a2, double a3) {
    const int l = __builtin_amdgcn_workitem_id_x() & 63;
    const bool b0 = (l & 1) != 0, b1 = (l & 2) != 0;
    const double lo = b0 ? a1 : a0, hi = b0 ? a3 : a2;
    return b1 ? hi : lo;
}

// Gather the four row groups: x[j] at lane (g,c) = v at lane (j,c), for all j at once.
// One v_permlane32_swap per dword splits the halves, one v_permlane16_swap per dword and half
// splits the rows: 6 cross-lane ops for the whole 4x16 transpose-by-row-group.
__device__ __forceinline__ void rowgroup_gather(double v, double x[4]) {
    const int lo = __double2loint(v), hi = __double2hiint(v);
    const auto a = __builtin_amdgcn_permlane32_swap(lo, lo, false, false);  // [0]: rows {0,1}, [1]: rows {2,3}
    const auto b = __builtin_amdgcn_permlane32_swap(hi, hi, false, false);
    const auto c0 = __builtin_amdgcn_permlane16_swap((int)a[0], (int)a[0], false, false);  // rows 0 | 1
    const auto d0 = __builtin_amdgcn_permlane16_swap((int)b[0], (int)b[0], false, false);
    const auto c1 = __builtin_amdgcn_permlane16_swap((int)a[1], (int)a[1], false, false);  // rows 2 | 3
    const auto d1 = __builtin_amdgcn_permlane16_swap((int)b[1], (int)b[1], false, false);
    x[0] = mk((int)d0[0], (int)c0[0]);
    x[1] = mk((int)d0[1], (int)c0[1]);
    x[2] = mk((int)d1[0], (int)c1[0]);
    x[3] = mk((int)d1[1], (int)c1[1]);
}

// Sum over the four row groups: result at (g,c) = sum_g' x(g',c); identical in all row groups.
__device__ __forceinline__ double xrow_sum(double x) {
    int lo = __double2loint(x), hi = __double2hiint(x);
    auto a = __builtin_amdgcn_permlane32_swap(lo, lo, false, false);
    auto b = __builtin_amdgcn_permlane32_swap(hi, hi, false, false);
    double s1 = mk((int)b[0], (int)a[0]) + mk((int)b[1], (int)a[1]);  // rows {0,1}+{2,3}
    lo = __double2loint(s1);
    hi = __double2hiint(s1);
    auto c = __builtin_amdgcn_permlane16_swap(lo, lo, false, false);
    auto d = __builtin_amdgcn_permlane16_swap(hi, hi, false, false);
    return mk((int)d[0], (int)c[0]) + mk((int)d[1], (int)c[1]);
}

// Sum over the 16 lanes of each row (rotate-and-add butterfly); identical in all 16 lanes.
__device__ __forceinline__ double row_sum16(double x) {
    x += dpp_mov<0x128>(x);  // row_ror:8
    x += dpp_mov<0x124>(x);  // row_ror:4
    x += dpp_mov<0x122>(x);  // row_ror:2
    x += dpp_mov<0x121>(x);  // row_ror:1
    return x;
}

// wave-wide reductions (all lanes get the result)
__device__ __forceinline__ double wave_sum(double x) {
    x = row_sum16(x);
    return xrow_sum(x);
}
__device__ __forceinline__ double wave_min(double x) {
    x = fmin(x, dpp_mov<0x128>(x));
    x = fmin(x, dpp_mov<0x124>(x));
    x = fmin(x, dpp_mov<0x122>(x));
    x = fmin(x, dpp_mov<0x121>(x));
    int lo = __double2loint(x), hi = __double2hiint(x);
    auto a = __builtin_amdgcn_permlane32_swap(lo, lo, false, false);
    auto b = __builtin_amdgcn_permlane32_swap(hi, hi, false, false);
    x = fmin(mk((int)b[0], (int)a[0]), mk((int)b[1], (int)a[1]));
    lo = __double2loint(x);
    hi = __double2hiint(x);
    auto c = __builtin_amdgcn_permlane16_swap(lo, lo, false, false);
    auto d = __builtin_amdgcn_permlane16_swap(hi, hi, false, false);
    return fmin(mk((int)d[0], (int)c[0]), mk((int)d[1], (int)c[1]));
}

// Cholesky pivot with the reference's clamp (kernel_dpotrf_c99_lib4.c:555-640): d > 1e-15 gives
// s = sqrt(d), inv = 1/s; otherwise both 0.  v_rsq_f64 (rel. error 5e-8 on gfx950, measured by
// tools/rsq_precision.py) refined by ONE third-order step y(1 + e/2 + 3e^2/8), e = 1 - d y^2:
// truncation ~e^3 ~ 1e-22, i.e. the result is rounding-limited (~1 ulp), and the dependent chain is
// four f64 ops after the rsq instead of six for two Newton steps.  The clamp select sits at the end,
// off the chain.
__device__ __forceinline__ void chol_pivot(double d, double &s, double &inv) {
    const bool ok = d > 1e-15;
    const double y = __builtin_amdgcn_rsq(d);
    const double dy = d * y;
    const double e = fma(-dy, y, 1.0);
    const double p = fma(0.375, e, 0.5);
    const double ye = y * e;
    const double y1 = fma(ye, p, y);
    inv = ok ? y1 : 0.0;
    s = ok ? d * y1 : 0.0;
}

// Pivot inverse only (the diagonal entry itself comes out of the panel formula, see chol_block).
__device__ __forceinline__ double chol_inv(double d) {
    const bool ok = d > 1e-15;
    const double y = __builtin_amdgcn_rsq(d);
    const double dy = d * y;
    const double e = fma(-dy, y, 1.0);
    const double p = fma(0.375, e, 0.5);
    const double ye = y * e;
    const double y1 = fma(ye, p, y);
    return ok ? y1 : 0.0;
}

// 1/x from v_rcp_f64 plus two Newton steps (<= 1 ulp from the IEEE quotient; the reference's 1.0/t and
// -lam/dlam are reproduced to the parity tolerance, at 5 VALU ops instead of the 10-op IEEE divide).
__device__ __forceinline__ double rcp_nr(double x) {
    double y = __builtin_amdgcn_rcp(x);
    double e = fma(-x, y, 1.0);
    y = fma(y, e, y);
    e = fma(-x, y, 1.0);
    return fma(y, e, y);
}

// Raw-buffer global access.  Masked lanes use an out-of-range offset: the hardware range check
// returns 0 for the load and drops the store, so no exec-masked branch is emitted around the memory
// op and the vector-memory counter stays exact (hipcc can then wait with a counted vmcnt instead of
// draining every prefetch).  `base` must be wave-uniform; idx is per lane (doubles).
__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void* base) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), 0, 0x7FFFFFF0, 0x00020000);
}
__device__ __forceinline__ double gld(const double* base, int idx, bool ok = true) {
    const int off = ok ? idx * 8 : (int)0xFFFFFFF0;
    return __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(rsrc(base), off, 0, 0));
}
__device__ __forceinline__ void gst(double* base, int idx, double v, bool ok = true) {
    const int off = ok ? idx * 8 : (int)0xFFFFFFF0;
    typedef unsigned int u2 __attribute__((ext_vector_type(2)));
    __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u2, v), rsrc(base), off, 0, 0);
}

__device__ __forceinline__ d4 mfma(double a, double b, d4 c) {
    return __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0);
}

}  // namespace hk
