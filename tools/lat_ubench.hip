// lat_ubench.hip -- single-wave latency / issue cost of the instructions the stage kernels are
// built from (inline asm so that nothing is folded), measured with s_memtime.
#include <hip/hip_runtime.h>

#define REP 64
__device__ __forceinline__ unsigned long long now() {
    unsigned long long t;
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
    return t;
}
#define FMA(a, b, c) asm volatile("v_fma_f64 %0, %1, %2, %0" : "+v"(a) : "v"(b), "v"(c))
#define MUL(a, b) asm volatile("v_mul_f64 %0, %0, %1" : "+v"(a) : "v"(b))
#define RSQ(a) asm volatile("v_rsq_f64 %0, %0" : "+v"(a))
#define CND(a, b) asm volatile("v_cndmask_b32 %0, %0, %1, vcc" : "+v"(a) : "v"(b))
#define DPP(a) asm volatile("v_mov_b32_dpp %0, %0 row_newbcast:3 row_mask:0xf bank_mask:0xf" : "+v"(a))
#define PL16(a, b) asm volatile("v_permlane16_swap_b32 %0, %1" : "+v"(a), "+v"(b))
#define FMA32(a, b, c) asm volatile("v_fma_f32 %0, %1, %2, %0" : "+v"(a) : "v"(b), "v"(c))
// f64 MFMA 16x16x4: dependent accumulator chain, and its result read by a VALU op
#define MFMA64(acc, a, b) asm volatile("v_mfma_f64_16x16x4_f64 %0, %1, %2, %0" : "+v"(acc) : "v"(a), "v"(b))
#define MFMA64USE(acc, a, b)                                             \
    do {                                                                 \
        acc = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc, 0, 0, 0); \
        a = a + acc[0];                                                  \
    } while (0)
#define DPP64(a) asm volatile("v_mov_b64_dpp %0, %0 row_newbcast:3 row_mask:0xf bank_mask:0xf" : "+v"(a))
#define PL32(a, b) asm volatile("v_permlane32_swap_b32 %0, %1" : "+v"(a), "+v"(b))
// LDS round trip: write then read back the same address (dependent through the value)
#define LDSRT(p, a) asm volatile("ds_write_b64 %1, %0\n\ts_waitcnt lgkmcnt(0)\n\tds_read_b64 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "+v"(a) : "v"(p) : "memory")
// readlane of a double's low half + scalar compare + branch (a ballot-like wave-uniform decision)
#define RDL(a, i) asm volatile("v_readfirstlane_b32 %0, %1\n\ts_add_u32 %0, %0, 1\n\tv_mov_b32 %1, %0" : "=s"(i) : "v"(a))

#define TIME(slot, ...)                      \
    {                                         \
        t0 = now();                           \
        _Pragma("unroll") for (int i = 0; i < REP; i++) { __VA_ARGS__; } \
        t1 = now();                           \
        if (l == 0) cyc[slot] = t1 - t0;      \
    }

extern "C" __global__ __launch_bounds__(64) void lat(double* out, unsigned long long* cyc, double seed) {
    const int l = threadIdx.x;
    double a = seed + l, b = 1.0000001, c = 0.5, d0 = a, d1 = a + 1, d2 = a + 2, d3 = a + 3;
    double e0 = a, e1 = a, e2 = a, e3 = a, e4 = a, e5 = a, e6 = a, e7 = a;
    float f0 = a, f1 = a, f2 = a, f3 = a, f4 = a, f5 = a, f6 = a, f7 = a, fb = 1.0f, fc = 0.5f;
    int i0 = l, i1 = l + 1, i2 = l + 2, i3 = l + 3;
    unsigned long long t0, t1;
    TIME(0, FMA(a, b, c));                                  // dependent fma_f64
    TIME(1, MUL(a, b));                                     // dependent mul_f64
    TIME(2, RSQ(a));                                        // dependent rsq_f64
    TIME(3, FMA(e0, b, c); FMA(e1, b, c); FMA(e2, b, c); FMA(e3, b, c); FMA(e4, b, c); FMA(e5, b, c);
             FMA(e6, b, c); FMA(e7, b, c));                // 8 independent fma_f64
    TIME(4, FMA32(f0, fb, fc); FMA32(f1, fb, fc); FMA32(f2, fb, fc); FMA32(f3, fb, fc); FMA32(f4, fb, fc);
             FMA32(f5, fb, fc); FMA32(f6, fb, fc); FMA32(f7, fb, fc));  // 8 independent fma_f32
    TIME(5, CND(i0, i1); CND(i1, i2); CND(i2, i3); CND(i3, i0));       // cndmask stream
    TIME(6, DPP(i0));                                       // dependent dpp mov
    TIME(7, DPP(i0); DPP(i1); DPP(i2); DPP(i3));          // 4 independent dpp movs
    TIME(8, PL16(i0, i1));                                  // dependent permlane16_swap
    TIME(9, RSQ(e0); RSQ(e1); RSQ(e2); RSQ(e3));          // 4 independent rsq
    typedef double d4v __attribute__((ext_vector_type(4)));
    d4v acc = {a, a, a, a};
    TIME(10, MFMA64(acc, b, c));                            // dependent f64 MFMA (accumulator)
    double u = a;
    TIME(11, MFMA64USE(acc, u, c));                         // MFMA -> VALU use -> next MFMA operand
    TIME(12, DPP64(d0));                                    // dependent v_mov_b64_dpp row_newbcast
    TIME(13, PL32(i0, i1));                                 // dependent permlane32_swap
    __shared__ double sh[64];
    const unsigned lp = (unsigned)(l * 8) + (unsigned)(size_t)sh;
    TIME(14, LDSRT(lp, d1));                                // LDS write -> read round trip
    int sreg = 0;
    TIME(15, RDL(i2, sreg));                                // readfirstlane -> SALU -> VALU
    out[l] = a + d0 + d1 + d2 + d3 + e0 + e1 + e2 + e3 + e4 + e5 + e6 + e7 + f0 + f1 + f2 + f3 + f4 + f5 +
             f6 + f7 + i0 + i1 + i2 + i3 + acc[0] + acc[3] + u + sreg;
}

extern "C" int lat_run(double* out, unsigned long long* cyc, void* stream) {
    hipLaunchKernelGGL(lat, dim3(1), dim3(64), 0, (hipStream_t)stream, out, cyc, 1.25);
    return (int)hipGetLastError();
}
