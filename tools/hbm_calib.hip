// hbm_calib.hip -- calibration of rocprofv3 FETCH_SIZE / WRITE_SIZE for the access pattern of the
// Riccati/IPM kernels (8-byte raw buffer loads/stores per lane, hk::gld / hk::gst), on a known byte
// count far beyond the 256 MiB Infinity Cache.  MI355X_MICROARCH.md: "calibrate on a known byte count
// in your own access pattern before trusting an absolute".
#include <hip/hip_runtime.h>

#include "../hpmpc_amd/csrc/hk_prims.h"

// each wave streams a contiguous 64 x 8 B = 512 B segment per instruction, grid-stride
extern "C" __global__ __launch_bounds__(256) void calib_copy(const double* x, double* y, long n) {
    const long stride = (long)gridDim.x * blockDim.x;
    for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        const long base = i & ~63L;  // 64-element chunk the wave works on
        const double v = hk::gld(x + base, (int)(i - base));
        hk::gst(y + base, (int)(i - base), v * 1.0000001);
    }
}

// read-only stream in the same pattern (one 8-B store per thread at the end, so the loads are not dead)
extern "C" __global__ __launch_bounds__(256) void calib_read(const double* x, double* y, long n) {
    const long stride = (long)gridDim.x * blockDim.x;
    double acc = 0.0;
    for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        const long base = i & ~63L;
        acc += hk::gld(x + base, (int)(i - base));
    }
    y[(long)blockIdx.x * blockDim.x + threadIdx.x] = acc;
}

extern "C" int calib_read_run(const double* x, double* y, long n, void* stream) {
    hipLaunchKernelGGL(calib_read, dim3(8192), dim3(256), 0, (hipStream_t)stream, x, y, n);
    return (int)hipGetLastError();
}

extern "C" int calib_run(const double* x, double* y, long n, void* stream) {
    hipLaunchKernelGGL(calib_copy, dim3(8192), dim3(256), 0, (hipStream_t)stream, x, y, n);
    return (int)hipGetLastError();
}

// ---- load-width / memory-level-parallelism probes (tools/hbm_bw.py): 8-B and 16-B raw buffer loads per lane, each
// thread keeping U loads in flight (independent addresses, unrolled), over the same 1 GiB
typedef unsigned int u4v __attribute__((ext_vector_type(4)));
typedef unsigned int u2v __attribute__((ext_vector_type(2)));

template <int U>
__global__ __launch_bounds__(256) void read8_u(const double* x, double* y, long n) {
    const long nthr = (long)gridDim.x * blockDim.x, t = (long)blockIdx.x * blockDim.x + threadIdx.x;
    double acc[U];
#pragma unroll
    for (int u = 0; u < U; u++) acc[u] = 0.0;
    for (long i0 = 0; i0 < n; i0 += nthr * U) {
#pragma unroll
        for (int u = 0; u < U; u++) {
            const long i = i0 + u * nthr + t;
            const long base = i & ~63L;
            acc[u] += hk::gld(x + base, (int)(i - base), i < n);
        }
    }
    double s = 0.0;
#pragma unroll
    for (int u = 0; u < U; u++) s += acc[u];
    y[t] = s;
}

template <int U>
__global__ __launch_bounds__(256) void read16_u(const double* x, double* y, long n) {
    const long n2 = n / 2, nthr = (long)gridDim.x * blockDim.x, t = (long)blockIdx.x * blockDim.x + threadIdx.x;
    double acc[U];
#pragma unroll
    for (int u = 0; u < U; u++) acc[u] = 0.0;
    for (long i0 = 0; i0 < n2; i0 += nthr * U) {
#pragma unroll
        for (int u = 0; u < U; u++) {
            const long i = i0 + u * nthr + t;  // pair index
            const long base = i & ~63L;
            const int off = i < n2 ? (int)(i - base) * 16 : (int)0xFFFFFFF0;
            const u4v v = __builtin_amdgcn_raw_buffer_load_b128(hk::rsrc(x + 2 * base), off, 0, 0);
            const double a = __builtin_bit_cast(double, (unsigned long long)v.x | ((unsigned long long)v.y << 32));
            const double b = __builtin_bit_cast(double, (unsigned long long)v.z | ((unsigned long long)v.w << 32));
            acc[u] += a + b;
        }
    }
    double s = 0.0;
#pragma unroll
    for (int u = 0; u < U; u++) s += acc[u];
    y[t] = s;
}

template <int U>
__global__ __launch_bounds__(256) void copy16_u(const double* x, double* y, long n) {
    const long n2 = n / 2, nthr = (long)gridDim.x * blockDim.x, t = (long)blockIdx.x * blockDim.x + threadIdx.x;
    for (long i0 = 0; i0 < n2; i0 += nthr * U) {
        u4v v[U];
#pragma unroll
        for (int u = 0; u < U; u++) {
            const long i = i0 + u * nthr + t;
            const long base = i & ~63L;
            const int off = i < n2 ? (int)(i - base) * 16 : (int)0xFFFFFFF0;
            v[u] = __builtin_amdgcn_raw_buffer_load_b128(hk::rsrc(x + 2 * base), off, 0, 0);
        }
#pragma unroll
        for (int u = 0; u < U; u++) {
            const long i = i0 + u * nthr + t;
            const long base = i & ~63L;
            const int off = i < n2 ? (int)(i - base) * 16 : (int)0xFFFFFFF0;
            __builtin_amdgcn_raw_buffer_store_b128(v[u], hk::rsrc(y + 2 * base), off, 0, 0);
        }
    }
}

template <int U>
__global__ __launch_bounds__(256) void copy8_u(const double* x, double* y, long n) {
    const long nthr = (long)gridDim.x * blockDim.x, t = (long)blockIdx.x * blockDim.x + threadIdx.x;
    for (long i0 = 0; i0 < n; i0 += nthr * U) {
        double v[U];
#pragma unroll
        for (int u = 0; u < U; u++) {
            const long i = i0 + u * nthr + t;
            const long base = i & ~63L;
            v[u] = hk::gld(x + base, (int)(i - base), i < n);
        }
#pragma unroll
        for (int u = 0; u < U; u++) {
            const long i = i0 + u * nthr + t;
            const long base = i & ~63L;
            hk::gst(y + base, (int)(i - base), v[u], i < n);
        }
    }
}

// which: 0 read8 U=1, 1 read8 U=4, 2 read16 U=1, 3 read16 U=4, 4 copy8 U=4, 5 copy16 U=4
extern "C" int probe_run(int which, const double* x, double* y, long n, int grid, void* stream) {
    const dim3 g(grid), b(256);
    hipStream_t s = (hipStream_t)stream;
    switch (which) {
        case 0: hipLaunchKernelGGL(read8_u<1>, g, b, 0, s, x, y, n); break;
        case 1: hipLaunchKernelGGL(read8_u<4>, g, b, 0, s, x, y, n); break;
        case 2: hipLaunchKernelGGL(read16_u<1>, g, b, 0, s, x, y, n); break;
        case 3: hipLaunchKernelGGL(read16_u<4>, g, b, 0, s, x, y, n); break;
        case 4: hipLaunchKernelGGL(copy8_u<4>, g, b, 0, s, x, y, n); break;
        case 5: hipLaunchKernelGGL(copy16_u<4>, g, b, 0, s, x, y, n); break;
        default: return -1;
    }
    return (int)hipGetLastError();
}
