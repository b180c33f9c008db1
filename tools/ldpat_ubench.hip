// ldpat_ubench.hip -- cost of the stage kernels' vector loads by ADDRESS PATTERN (tools/ldpat_ubench.py).
//
// One wave (or a grid of waves) repeatedly issues 16 raw 8-B buffer loads (hk::gld's instruction) and waits for
// them, over a buffer that stays L2-resident.  Patterns, per load instruction:
//   0 contiguous   lane l reads element base + l           (512 B, 4 cache lines: the factor record's loads)
//   1 lib4 tile    lane (g,c) reads lower-lib4 element (max(r,c), min(r,c)) of a 20 x 16 block, r = g + 4j
//                  (the RSQrq fetch of bwd_fetch: ~10 lines spread over 2.5 KB)
//   2 lib4 trans   lane (g,c) reads BAbt element (c, g + 4j) of a 20 x 12 block (the bop fetch)
//   3 b128 contig  lane l reads 16 B at base + 2l with one buffer_load_dwordx4 (two doubles per lane)
// Reported: cycles (s_memtime) per iteration of 16 loads + wait, for the grid's wave 0.
#include <hip/hip_runtime.h>

namespace {
__device__ __forceinline__ __amdgpu_buffer_rsrc_t rs(const void* p) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), 0, 0x7FFFFFF0, 0x00020000);
}
__device__ __forceinline__ double ld8(const double* b, int idx) {
    return __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(rs(b), idx * 8, 0, 0));
}
typedef double d2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ d2 ld16(const double* b, int idx) {
    typedef unsigned int u4 __attribute__((ext_vector_type(4)));
    return __builtin_bit_cast(d2, __builtin_amdgcn_raw_buffer_load_b128(rs(b), idx * 8, 0, 0));
}
__device__ __forceinline__ int lib4(int sd, int i, int j) { return (i >> 2) * 4 * sd + (i & 3) + 4 * j; }
}  // namespace

extern "C" __global__ __launch_bounds__(64) void ldpat(const double* buf, double* out, unsigned long long* cyc,
                                                        int pattern, int iters, long long stride) {
    const int l = threadIdx.x & 63, g = l >> 4, c = l & 15;
    const double* base = buf + (long long)blockIdx.x * stride;
    double acc = 0.0;
    unsigned long long t0 = 0;
    for (int it = -2; it < iters; it++) {
        if (it == 0) t0 = __builtin_amdgcn_s_memtime();
        const double* b = base + (it & 7) * 640;  // 8 rotating 5 KB blocks
        double v[16];
        if (pattern == 0) {
#pragma unroll
            for (int j = 0; j < 16; j++) v[j] = ld8(b, j * 64 + l);
        } else if (pattern == 1) {
#pragma unroll
            for (int j = 0; j < 16; j++) {
                const int r = g + 4 * (j & 3), cc = (c + 4 * (j >> 2)) & 15;
                v[j] = ld8(b, lib4(16, r > cc ? r : cc, r > cc ? cc : r) + (j >> 2) * 8);
            }
        } else if (pattern == 2) {
#pragma unroll
            for (int j = 0; j < 16; j++) v[j] = ld8(b, lib4(12, c + (j >> 2), (g + 4 * (j & 3)) % 12));
        } else {
#pragma unroll
            for (int j = 0; j < 8; j++) {
                const d2 x = ld16(b, j * 128 + 2 * l);
                v[2 * j] = x[0];
                v[2 * j + 1] = x[1];
            }
        }
        double s = 0.0;
#pragma unroll
        for (int j = 0; j < 16; j++) s += v[j];
        acc = acc * 0.5 + s;
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    out[(long long)blockIdx.x * 64 + l] = acc;
    if (blockIdx.x == 0 && l == 0) cyc[0] = t1 - t0;
}

extern "C" int ldpat_run(const double* buf, double* out, unsigned long long* cyc, int pattern, int iters, int grid,
                         long long stride, hipStream_t st) {
    hipLaunchKernelGGL(ldpat, dim3(grid), dim3(64), 0, st, buf, out, cyc, pattern, iters, stride);
    return (int)hipGetLastError();
}
