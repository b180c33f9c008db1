// rsq_precision.hip -- accuracy of v_rsq_f64 and of its Newton refinements (decides how many
// refinement steps chol_pivot needs for the 1e-12 parity gate).
#include <hip/hip_runtime.h>
extern "C" __global__ void rsq_prec(const double* d, double* y0, double* y1, double* y2, int n) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const double x = d[i];
    double y = __builtin_amdgcn_rsq(x);
    y0[i] = y;
    const double h = 0.5 * x;
    double e = fma(-h * y, y, 0.5);
    y = fma(y, e, y);
    y1[i] = y;
    e = fma(-h * y, y, 0.5);
    y = fma(y, e, y);
    (void)y;
    // one third-order step (chol_pivot)
    const double r = __builtin_amdgcn_rsq(x);
    const double dy = x * r;
    const double ee = fma(-dy, r, 1.0);
    const double pp = fma(0.375, ee, 0.5);
    y2[i] = fma(r * ee, pp, r);
}
extern "C" int rsq_run(const double* d, double* y0, double* y1, double* y2, int n, void* s) {
    hipLaunchKernelGGL(rsq_prec, dim3((n + 255) / 256), dim3(256), 0, (hipStream_t)s, d, y0, y1, y2, n);
    return (int)hipGetLastError();
}
