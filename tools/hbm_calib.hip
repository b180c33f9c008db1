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
