// hk_wide_host.h -- host-side helpers of the wide-stage path shared by hpmpc_capi_wide.cpp (Riccati, condensing)
// and hpmpc_capi_wide_ipm.cpp (the IPM on wide stages): the packed per-problem layout of a wide problem, a
// thread-local device context for the host-buffer entry points, and the launch wrapper.
#pragma once
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "hpmpc_api.h"
#include "hk_wide_args.h"

extern "C" int hk_wide_launch(int which, const void* args, int count, int lds_doubles, hipStream_t stream);
extern "C" void hk_set_error(int code, const char* what);

namespace {

constexpr int BS = 4, NCL = 2;
constexpr int LDS_MAX_DOUBLES = 65536 / 8;

inline int rup(int n, int m) { return (n + m - 1) / m * m; }
inline double& P4(double* A, int sd, int i, int j) { return A[(i / BS) * BS * sd + i % BS + BS * j]; }
inline int poff(int j, int nz) { return j * nz - (j * (j - 1)) / 2; }

bool hip_ok(hipError_t e, const char* what) {
    if (e == hipSuccess) return true;
    char msg[256];
    snprintf(msg, sizeof msg, "HIP error in %s: %s", what, hipGetErrorString(e));
    hk_set_error(HPMPC_MI355X_EHIP, msg);
    return false;
}

// One problem's packed layout on the wide path (offsets in doubles; idxb in ints).
struct WLayout {
    int N = 0;
    std::vector<WideStage> st;
    long long nB = 0, nR = 0, nL = 0, nU = 0, nP = 0, nD = 0, nI = 0, nG = 0;
    int lds = 0, offW = 0, offX = 0, offV = 0, ldW = 0, ldX = 0, offST = 0;
    bool any_ng = false;
    bool fits = true;  // hk_wide_sv limits: nu+nx+1 <= 128 (two rows per lane), nx <= 64 (MFMA tiles per wave)
};

WLayout make_layout(int N, const int* nx, const int* nu, const int* nb, const int* ng) {
    WLayout L;
    L.N = N;
    L.st.resize(N + 1);
    int Mmax = 1, nzM = 1, nxM = 1;
    for (int k = 0; k <= N; k++) {
        WideStage& s = L.st[k];
        memset(&s, 0, sizeof s);
        s.nu = k < N ? nu[k] : 0;
        s.nx = nx[k];
        s.nx1 = k < N ? nx[k + 1] : 0;
        s.nu1 = k + 1 < N ? nu[k + 1] : 0;
        const int nux = s.nu + s.nx;
        s.sdB = rup(s.nx1, NCL);
        s.sdR = rup(nux, NCL);
        s.oB = (int)L.nB;
        if (k < N) L.nB += (long long)rup(nux + 1, BS) * s.sdB;
        s.oR = (int)L.nR;
        L.nR += (long long)rup(nux + 1, BS) * s.sdR;
        s.oL = (int)L.nL;
        L.nL += poff(nux, nux + 1) + nux;
        L.nL = (L.nL + 7) / 8 * 8;
        s.oU = (int)L.nU;
        L.nU += rup(nux + 1, 8);
        s.oP = (int)L.nP;
        L.nP += rup(s.nx1 + 1, 8);
        s.nb = nb[k];
        s.pnb = rup(nb[k], BS);
        s.ng = ng[k];
        s.sdG = rup(ng[k], NCL);
        s.oG = (int)L.nG;
        L.nG += (long long)rup(nux, BS) * s.sdG;
        s.oD = (int)L.nD;
        L.nD += 2 * s.pnb + 2 * rup(ng[k], BS);
        s.oI = (int)L.nI;
        L.nI += nb[k];
        if (ng[k] > 0) L.any_ng = true;
        Mmax = std::max(Mmax, poff(nux, nux + 1));
        nzM = std::max(nzM, nux + 1);
        nxM = std::max(nxM, std::max(s.nx1, s.nx));  // X also receives stage k's own Lxx
    }
    L.fits = nzM <= 128 && nxM <= 64;
    L.ldW = nzM;
    L.ldX = nxM + 1;
    L.offW = Mmax + nzM;  // the forward stages L_k with its 1/diag tail into M
    L.offX = L.offW + L.ldW * nxM;
    L.offV = L.offX + L.ldX * nxM;
    L.offST = rup(L.offV + nzM, 2);  // the stage table (WideStage records) in LDS
    L.lds = L.offST + (N + 1) * (int)(sizeof(WideStage) / sizeof(double));
    if (L.nD == 0) L.nD = 1;
    if (L.nI == 0) L.nI = 1;
    if (L.nB == 0) L.nB = 1;
    if (L.nG == 0) L.nG = 1;
    return L;
}

// Thread-local device context of the host-buffer entry points: one stream, a growable device arena and
// its pinned staging twin.
struct WCtx {
    hipStream_t stream = nullptr;
    char* dev = nullptr;
    char* host = nullptr;
    size_t cap = 0;
    ~WCtx() {
        if (dev) (void)hipFree(dev);
        if (host) (void)hipHostFree(host);
        if (stream) (void)hipStreamDestroy(stream);
    }
    bool ensure(size_t bytes) {
        if (!stream && !hip_ok(hipStreamCreateWithFlags(&stream, hipStreamNonBlocking), "stream create")) return false;
        if (bytes > cap) {
            if (dev) (void)hipFree(dev);
            if (host) (void)hipHostFree(host);
            dev = host = nullptr;
            cap = 0;
            if (!hip_ok(hipMalloc((void**)&dev, bytes), "wide device arena")) return false;
            if (!hip_ok(hipHostMalloc((void**)&host, bytes, 0), "wide pinned arena")) return false;
            cap = bytes;
        }
        memset(host, 0, bytes);
        return true;
    }
    bool up(size_t bytes) {
        return hip_ok(hipMemcpyAsync(dev, host, bytes, hipMemcpyHostToDevice, stream), "H2D");
    }
    bool down(size_t bytes) {
        return hip_ok(hipMemcpyAsync(host, dev, bytes, hipMemcpyDeviceToHost, stream), "D2H") &&
               hip_ok(hipStreamSynchronize(stream), "sync");
    }
};
thread_local WCtx g_w;

// Byte carve of the staging arena.
struct Carve {
    size_t o = 0;
    size_t take(size_t bytes) {
        size_t r = o;
        o += (bytes + 255) / 256 * 256;
        return r;
    }
};

bool launch(int which, const void* args, int count, int lds, hipStream_t stream, const char* name) {
    if (lds > LDS_MAX_DOUBLES) {
        hk_set_error(HPMPC_MI355X_EUNSUPPORTED, "wide stage beyond the 64 KiB LDS tile budget");
        return false;
    }
    int e = hk_wide_launch(which, args, count, lds, stream);
    if (e) {
        char msg[128];
        snprintf(msg, sizeof msg, "%s launch failed (%d)", name, e);
        hk_set_error(HPMPC_MI355X_EHIP, msg);
        return false;
    }
    return true;
}

}  // namespace
