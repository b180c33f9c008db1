// checks that an out-of-range raw buffer load with the LDS flag writes zero into LDS
#include <hip/hip_runtime.h>
#include <cstdio>
typedef __attribute__((address_space(3))) void* lds_void_ptr;
__global__ void k(const float* src, float* out) {
    __shared__ float sm[128];
    sm[threadIdx.x] = -7.0f;
    sm[threadIdx.x + 64] = -7.0f;
    __syncthreads();
    __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(src), 0, 0x7FFFFFF0, 0x00020000);
    int off = (threadIdx.x & 1) ? (int)threadIdx.x * 4 : (int)0xFFFFFFF0;
    __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (lds_void_ptr)(sm + 32), 4, off, 0, 0, 0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    out[threadIdx.x] = sm[threadIdx.x];
    out[threadIdx.x + 64] = sm[threadIdx.x + 64];
}
int main() {
    float h[64], o[128];
    for (int i = 0; i < 64; i++) h[i] = 100.0f + i;
    float *d, *dout;
    hipMalloc(&d, sizeof h);
    hipMalloc(&dout, sizeof o);
    hipMemcpy(d, h, sizeof h, hipMemcpyHostToDevice);
    k<<<1, 64>>>(d, dout);
    hipMemcpy(o, dout, sizeof o, hipMemcpyDeviceToHost);
    int bad = 0;
    for (int i = 0; i < 128; i++) {
        float want = (i < 32 || i >= 96) ? -7.0f : (((i - 32) & 1) ? 100.0f + (i - 32) : 0.0f);
        if (o[i] != want) { bad++; if (bad < 8) printf("slot %d got %g want %g\n", i, o[i], want); }
    }
    printf("dma_oob: %s (%d bad)\n", bad ? "FAIL" : "zero-fill confirmed", bad);
    return bad != 0;
}
