// hk_launch_guard.h -- host-side check before launching a workgroup kernel: the kernel's private segment (scratch
// per lane, from its code object) must fit the device's stack limit, its static + dynamic LDS the per-workgroup
// maximum, and the block size its launch bound.  A launch that would exceed any is refused (HK_LAUNCH_REFUSED)
// instead of being issued.  The kernel's attributes and the device limits are read once per kernel.
#pragma once
#include <hip/hip_runtime.h>

constexpr int HK_LAUNCH_REFUSED = -2;

struct HkKernelLimits {
    hipFuncAttributes fa{};
    size_t stack = 0;
    int lds_max = 0, err = 0;
    explicit HkKernelLimits(const void* kernel) {
        if (hipFuncGetAttributes(&fa, kernel) != hipSuccess || hipDeviceGetLimit(&stack, hipLimitStackSize) != hipSuccess) {
            err = (int)hipGetLastError();
            return;
        }
        int dev = 0;
        (void)hipGetDevice(&dev);
        (void)hipDeviceGetAttribute(&lds_max, hipDeviceAttributeMaxSharedMemoryPerBlock, dev);
    }
    int check(size_t dyn_lds, int threads) const {
        if (err) return err;
        if (fa.localSizeBytes > stack) return HK_LAUNCH_REFUSED;
        if (lds_max > 0 && fa.sharedSizeBytes + dyn_lds > (size_t)lds_max) return HK_LAUNCH_REFUSED;
        if (fa.maxThreadsPerBlock > 0 && threads > fa.maxThreadsPerBlock) return HK_LAUNCH_REFUSED;
        return 0;
    }
};
