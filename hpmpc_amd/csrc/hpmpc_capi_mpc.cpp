// hpmpc_capi_mpc.cpp -- the legacy uniform-size wrappers of include/c_interface.h:40-53:
// fortran_order_d_ip_mpc_hard_tv / c_order_d_ip_mpc_hard_tv (interfaces/c/fortran_order_interface.c:1975-3013,
// c_order_interface.c:1052-2082), their KKT re-solves (fortran_order_interface.c:3017-3779, c_order_interface.c:
// 2083-2848) and hpmpc_d_ip_mpc_hard_tv_work_space_size_doubles (declared at c_interface.h:40, defined nowhere in the
// reference).  Uniform stage sizes in flat arrays, a time_invariant flag (one copy of each stage array), x0 folded
// into stage 0 (nx[0] = 0: b0 = A x0 + b, r0 = r + S x0), lib4 packing on the host, then this library's
// d_ip2_mpc_hard_tv / d_kkt_solve_new_rhs_mpc_hard_tv and d_res_mpc_hard_tv -- every solve runs on the GPU.
//
// The reference's deterministic quirks are kept (oracle/iface_oracle.py restates the same steps):
//   * an input with lb == ub is folded into b and its B column zeroed; the b row is addressed with panel
//     (nxx + nuu) / 4 but in-panel row (nx + nu) % 4 (:2698), so on stage 0 the update lands on row
//     4 (nu / 4) + (nx + nu) % 4; the box becomes [lb + 1e3, ub - 1e3] (:2704);
//   * time-invariant general-constraint bounds are read per stage (lg + ng k) into one shared vector, so every
//     middle stage gets stage N-1's (:2425-2433);
//   * the residual's q is the data's r, q (stage 0: r without S x0, :2846-2867); b is the packed b;
//   * the KKT wrapper re-packs stage 0's B' over the IPM's data (:3264), copies the bounds as they are (no equality
//     folding) and does no input-equality fix on u; the c_order KKT norm skips the general constraints of stages
//     0..N-1 (c_order_interface.c:2761);
//   * outputs: lam / t with stage stride 2 nb + 2 ng, box lower at 0, upper at nb + ng, general lower at nb, upper
//     at 2 nb + ng, stage N boxes at nu + j with the upper offset nb + ngN (:2953-3007).
// Where the reference reads memory it never wrote or reads past an array, the evident intent is taken instead:
//   * time-invariant packing of the middle stages happens only if a stale loop index (nx) is below N
//     (`if(jj<N)`, :2235 / :2259); here always;
//   * the c_order time-variant / time-invariant wrappers never write hb[k] for k >= 1 (resp. k >= 2), which the
//     residual reads (c_order_interface.c:1651-1657, :1296); here hb[k] = b_k;
//   * mu0 <= 0 reads qf[nx] (one past qf) and, time-invariant, the stage-1 slots of single-stage arrays
//     (:2325-2339); here qf[0..nx) and the single stage (absolute values time-invariant, plain time-variant, as
//     the reference);
//   * the stage-N box term of inf_norm_res[2] reads r_q of stage N, partly memory d_res never writes
//     (:2920-2925); here r_d of stage N;
//   * the time-invariant KKT wrapper tests an uninitialised index before copying b into hb[1] (:3268); here always.
// work0 holds the idxb tables, then (64-byte aligned) per-stage BAbt, DCt, RSQrq, the IPM work space and the
// vectors, in one carve shared by the IPM and KKT wrappers (the KKT re-solve reads the IPM's packed matrices,
// iterate and work space from it, as the reference does).
#include <cmath>
#include <cstdint>
#include <cstring>
#include <vector>

#include "hpmpc_api.h"

extern "C" void hk_set_error(int code, const char* what);

namespace {

constexpr int BS = 4, NCL = 2;
inline int rup(int n, int m) { return (n + m - 1) / m * m; }
inline long li(int sd, int i, int j) { return (long)(i / BS) * BS * sd + i % BS + BS * j; }

struct Mpc {
    int N, nx, nu, nb, ng, ngN, nbu;
    bool ti, rowmajor;
    int pnz, pnx, pnb, png, pngN, cnux, cnu, cnx, cng, cngN;
    std::vector<int> nxx, nuu, nbb, ngg;
    std::vector<int*> idxb;
    std::vector<double*> BAbt, DCt, RSQ, b, rq, d, ux, pi, lam, t, rb, rrq, rd;
    double* work = nullptr;
    long long ipm_bytes = 0;
    long long total = 0;  // bytes of work0 used (from its start)
    std::vector<double> dummy;

    // element (i, j) of the m x n stage-k block of a flat stage array (time-invariant: the single copy)
    double el(const double* M, int m, int n, int k, int i, int j) const {
        const double* p = M + (ti ? 0 : (long)k * m * n);
        return rowmajor ? p[(long)i * n + j] : p[i + (long)j * m];
    }
    double el1(const double* M, int m, int n, int i, int j) const {  // a single block (Qf, Cf)
        return rowmajor ? M[(long)i * n + j] : M[i + (long)j * m];
    }
    const double* vec(const double* v, int k, int n) const { return v + (ti ? 0 : (long)k * n); }
    int blk(int k) const { return ti ? 0 : nb * k; }  // start of stage k's bounds in lb / ub
};

void dims(Mpc& P, int N, int nx, int nu, int nb, int ng, int ngN, bool ti, bool rowmajor) {
    P.N = N;
    P.nx = nx;
    P.nu = nu;
    P.nb = nb;
    P.ng = ng;
    P.ngN = ngN;
    P.ti = ti;
    P.rowmajor = rowmajor;
    P.nbu = nb < nu ? nb : nu;
    P.pnz = rup(nx + nu + 1, BS);
    P.pnx = rup(nx, BS);
    P.pnb = rup(nb, BS);
    P.png = rup(ng, BS);
    P.pngN = rup(ngN, BS);
    P.cnux = rup(nu + nx, NCL);
    P.cnu = rup(nu, NCL);
    P.cnx = rup(nx, NCL);
    P.cng = rup(ng, NCL);
    P.cngN = rup(ngN, NCL);
    P.nxx.assign(N + 1, nx);
    P.nxx[0] = 0;
    P.nuu.assign(N + 1, nu);
    P.nuu[N] = 0;
    P.nbb.assign(N + 1, nb);
    P.nbb[0] = P.nbu;
    P.nbb[N] = nb - nu > 0 ? nb - nu : 0;
    if (N == 0) P.nbb[0] = 0;
    P.ngg.assign(N + 1, ng);
    P.ngg[N] = ngN;
}

// Carve of work0 (base == nullptr: sizes only).  Returns false on sizes the wrapper cannot take.
bool carve(Mpc& P, void* work0) {
    const int N = P.N;
    char* w = reinterpret_cast<char*>(work0);
    long long o = 0;  // bytes from work0
    P.idxb.assign(N + 1, nullptr);
    for (int k = 0; k <= N; k++) {
        int* ip = w ? reinterpret_cast<int*>(w + o) : nullptr;
        P.idxb[k] = ip;
        if (ip)
            for (int j = 0; j < P.nbb[k]; j++) ip[j] = j;  // :2039-2061: stage N's idxb[j] = nuu[N] + j = j
        o += 4LL * P.nbb[k];
    }
    const uintptr_t a0 = (uintptr_t)w + o;
    o += (long long)(((a0 + 63) / 64 * 64) - a0);
    if (!w) o += 64;  // sizes only: the worst-case alignment gap
    auto take = [&](std::vector<double*>& v, int n, auto size) {
        v.resize(n);
        for (int k = 0; k < n; k++) {
            v[k] = w ? reinterpret_cast<double*>(w + o) : nullptr;
            o += 8LL * size(k);
        }
    };
    const int cgm = P.cng > P.cngN ? P.cng : P.cngN;
    take(P.BAbt, N, [&](int) { return (long long)P.pnz * P.cnx; });
    take(P.DCt, N + 1, [&](int k) { return (k < N ? P.ng : P.ngN) > 0 ? (long long)P.pnz * cgm : 0LL; });
    take(P.RSQ, N + 1, [&](int) { return (long long)P.pnz * P.cnux; });
    P.ipm_bytes = d_ip2_mpc_hard_tv_work_space_size_bytes(N, P.nxx.data(), P.nuu.data(), P.nbb.data(), P.ngg.data());
    P.work = w ? reinterpret_cast<double*>(w + o) : nullptr;
    o += (P.ipm_bytes + 63) / 64 * 64;
    auto nc = [&](int k) { return 2LL * P.pnb + 2LL * (k < N ? P.png : P.pngN) + 4; };
    take(P.b, N, [&](int) { return (long long)P.pnx + 4; });
    take(P.rq, N + 1, [&](int) { return (long long)P.pnz + 4; });
    take(P.d, N + 1, nc);
    take(P.ux, N + 1, [&](int) { return (long long)P.pnz + 4; });
    take(P.pi, N, [&](int) { return (long long)P.pnx + 4; });
    take(P.lam, N + 1, nc);
    take(P.t, N + 1, nc);
    take(P.rb, N, [&](int) { return (long long)P.pnx + 4; });
    take(P.rrq, N + 1, [&](int) { return (long long)P.pnz + 4; });
    take(P.rd, N + 1, nc);
    P.total = o;
    P.dummy.assign(8, 0.0);
    for (int k = 0; k <= N; k++)
        if (!P.DCt[k] || (k < N ? P.ng : P.ngN) == 0) P.DCt[k] = P.dummy.data();
    return true;
}

bool check(int N, int nx, int nu, int nb, int ng, int ngN) {
    if (N < 1 || nx < 1 || nu < 0 || nb < 0 || ng < 0 || ngN < 0 || nb > nu + nx) {
        hk_set_error(HPMPC_MI355X_EUNSUPPORTED, "legacy MPC wrapper: need N >= 1, nx >= 1, 0 <= nb <= nu + nx");
        return false;
    }
    return true;
}

struct Data {
    const double *A, *B, *b, *Q, *Qf, *S, *R, *q, *qf, *r, *lb, *ub, *C, *D, *lg, *ug, *Cf, *lgf, *ugf, *x0;
};

// Stage-0 right-hand sides: b0 = A0 x0 + b0 (:2561-2567), r0 = r0 + S0 x0 (:2628-2634).
void stage0_rhs(const Mpc& P, const Data& X, double* b0, double* r0) {
    for (int i = 0; i < P.nx; i++) {
        double s = 0.0;
        for (int j = 0; j < P.nx; j++) s += P.el(X.A, P.nx, P.nx, 0, i, j) * X.x0[j];
        b0[i] = s + P.vec(X.b, 0, P.nx)[i];
    }
    for (int i = 0; i < P.nu; i++) {
        double s = 0.0;
        for (int j = 0; j < P.nx; j++) s += P.el(X.S, P.nu, P.nx, 0, i, j) * X.x0[j];
        r0[i] = P.vec(X.r, 0, P.nu)[i] + s;
    }
}

// The IPM wrapper's packing (:2213-2757), or with kkt == true the KKT wrapper's re-pack of the right-hand sides over
// the IPM's data (:3248-3366, time-variant :3480-3560).
void pack(Mpc& P, const Data& X, bool kkt) {
    const int N = P.N, nx = P.nx, nu = P.nu, ng = P.ng, ngN = P.ngN;
    const int cnx = P.cnx, cnu = P.cnu, cnux = P.cnux;
    std::vector<double> r0(nu > 0 ? nu : 1);
    for (int k = 0; k < N; k++) memset(P.b[k], 0, sizeof(double) * (P.pnx + 4));
    for (int k = 0; k <= N; k++) {
        memset(P.rq[k], 0, sizeof(double) * (P.pnz + 4));
        memset(P.d[k], 0, sizeof(double) * (2 * P.pnb + 2 * (k < N ? P.png : P.pngN) + 4));
    }
    if (!kkt) {
        for (int k = 0; k < N; k++) memset(P.BAbt[k], 0, sizeof(double) * P.pnz * cnx);
        for (int k = 0; k <= N; k++) {
            memset(P.RSQ[k], 0, sizeof(double) * P.pnz * cnux);
            if (P.DCt[k] != P.dummy.data())
                memset(P.DCt[k], 0, sizeof(double) * P.pnz * (P.cng > P.cngN ? P.cng : P.cngN));
        }
    }
    stage0_rhs(P, X, P.b[0], r0.data());
    for (int i = 0; i < nu; i++)  // B0' (the KKT wrapper restores it over the IPM's data, :3264)
        for (int j = 0; j < nx; j++) P.BAbt[0][li(cnx, i, j)] = P.el(X.B, nx, nu, 0, j, i);
    if (kkt) {
        for (int i = 0; i < nu; i++) P.rq[0][i] = r0[i];
    } else {
        for (int j = 0; j < nx; j++) P.BAbt[0][li(cnx, nu, j)] = P.b[0][j];
        for (int i = 0; i < nu; i++) {
            for (int j = 0; j < nu; j++) P.RSQ[0][li(cnu, i, j)] = P.el(X.R, nu, nu, 0, i, j);
            P.RSQ[0][li(cnu, nu, i)] = r0[i];
        }
    }
    for (int k = 1; k < N; k++) {
        const double *bk = P.vec(X.b, k, nx), *rk = P.vec(X.r, k, nu), *qk = P.vec(X.q, k, nx);
        for (int j = 0; j < nx; j++) P.b[k][j] = bk[j];
        if (kkt) {
            for (int i = 0; i < nu; i++) P.rq[k][i] = rk[i];
            for (int i = 0; i < nx; i++) P.rq[k][nu + i] = qk[i];
            continue;
        }
        double* Bk = P.BAbt[k];
        for (int j = 0; j < nx; j++) {
            for (int i = 0; i < nu; i++) Bk[li(cnx, i, j)] = P.el(X.B, nx, nu, k, j, i);
            for (int i = 0; i < nx; i++) Bk[li(cnx, nu + i, j)] = P.el(X.A, nx, nx, k, j, i);
            Bk[li(cnx, nu + nx, j)] = bk[j];
        }
        double* Rk = P.RSQ[k];
        for (int i = 0; i < nu; i++) {
            for (int j = 0; j < nu; j++) Rk[li(cnux, i, j)] = P.el(X.R, nu, nu, k, i, j);
            Rk[li(cnux, nu + nx, i)] = rk[i];
        }
        for (int i = 0; i < nx; i++) {
            for (int j = 0; j < nu; j++) Rk[li(cnux, nu + i, j)] = P.el(X.S, nu, nx, k, j, i);
            for (int j = 0; j < nx; j++) Rk[li(cnux, nu + i, nu + j)] = P.el(X.Q, nx, nx, k, i, j);
            Rk[li(cnux, nu + nx, nu + i)] = qk[i];
        }
    }
    if (kkt) {
        for (int i = 0; i < nx; i++) P.rq[N][i] = X.qf[i];
    } else {
        for (int i = 0; i < nx; i++) {
            for (int j = 0; j < nx; j++) P.RSQ[N][li(cnx, i, j)] = P.el1(X.Qf, nx, nx, i, j);
            P.RSQ[N][li(cnx, nx, i)] = X.qf[i];
        }
        if (ng > 0)  // [D'; C'] (stage 0: D' only), :2592-2603
            for (int k = 0; k < N; k++) {
                for (int i = 0; i < nu; i++)
                    for (int j = 0; j < ng; j++) P.DCt[k][li(P.cng, i, j)] = P.el(X.D, ng, nu, k, j, i);
                if (k > 0)
                    for (int i = 0; i < nx; i++)
                        for (int j = 0; j < ng; j++) P.DCt[k][li(P.cng, nu + i, j)] = P.el(X.C, ng, nx, k, j, i);
            }
        if (ngN > 0)
            for (int i = 0; i < nx; i++)
                for (int j = 0; j < ngN; j++) P.DCt[N][li(P.cngN, i, j)] = P.el1(X.Cf, ngN, nx, j, i);
    }
    // bounds (:2683-2753)
    for (int k = 0; k < N; k++) {
        const int p0 = rup(P.nbb[k], BS);
        for (int i = 0; i < P.nbu; i++) {
            const double lo = X.lb[i + P.blk(k)], up = X.ub[i + P.blk(k)];
            if (kkt || lo != up) {
                P.d[k][i] = lo;
                P.d[k][i + p0] = up;
            } else {  // input equality constraint folded into b (:2695-2705), b row addressed as the reference does
                for (int l = 0; l < nx; l++) {
                    const long row = (long)((P.nxx[k] + P.nuu[k]) / BS) * cnx * BS + (nx + nu) % BS + (long)l * BS;
                    P.BAbt[k][row] += P.BAbt[k][li(cnx, i, l)] * lo;
                    P.BAbt[k][li(cnx, i, l)] = 0.0;
                }
                P.d[k][i] = lo + 1e3;
                P.d[k][i + p0] = up - 1e3;
            }
        }
    }
    for (int k = 1; k < N; k++) {
        const int p0 = rup(P.nbb[k], BS);
        for (int i = nu; i < P.nbb[k]; i++) {
            P.d[k][i] = X.lb[i + P.blk(k)];
            P.d[k][i + p0] = X.ub[i + P.blk(k)];
        }
    }
    {
        const int p0 = rup(P.nbb[N], BS);
        for (int i = 0; i < P.nbb[N]; i++) {
            P.d[N][i] = X.lb[nu + i + P.blk(N)];
            P.d[N][i + p0] = X.ub[nu + i + P.blk(N)];
        }
    }
    if (ng > 0)
        for (int k = 0; k < N; k++) {
            const int p0 = rup(P.nbb[k], BS), g0 = rup(P.ngg[k], BS);
            const int ks = (P.ti && k > 0) ? N - 1 : k;  // time-invariant: one shared vector, stage N-1's bounds win
            for (int i = 0; i < ng; i++) {
                P.d[k][2 * p0 + i] = X.lg[i + ng * ks];
                P.d[k][2 * p0 + g0 + i] = X.ug[i + ng * ks];
            }
        }
    if (ngN > 0) {
        const int p0 = rup(P.nbb[N], BS), g0 = rup(ngN, BS);
        for (int i = 0; i < ngN; i++) {
            P.d[N][2 * p0 + i] = X.lgf[i];
            P.d[N][2 * p0 + g0 + i] = X.ugf[i];
        }
    }
}

// The residual's q (:2846-2867): the data's r, q (stage 0: r without S x0), qf.
void residual_q(Mpc& P, const Data& X) {
    for (int k = 0; k <= P.N; k++) memset(P.rq[k], 0, sizeof(double) * (P.pnz + 4));
    for (int k = 0; k < P.N; k++) {
        for (int i = 0; i < P.nu; i++) P.rq[k][i] = P.vec(X.r, k, P.nu)[i];
        if (k > 0)
            for (int i = 0; i < P.nx; i++) P.rq[k][P.nu + i] = P.vec(X.q, k, P.nx)[i];
    }
    for (int i = 0; i < P.nx; i++) P.rq[P.N][i] = X.qf[i];
}

// mu0 <= 0 (:2320-2340 time-invariant, absolute values; :2659-2675 time-variant, plain values)
double auto_mu0(const Mpc& P, const Data& X) {
    const int N = P.N, nx = P.nx, nu = P.nu;
    double m = 0.0;
    auto f = [&](double v) { return P.ti ? fabs(v) : v; };
    auto blkmax = [&](const double* M, int rows, int cols, int k) {
        const double* p = M + (P.ti ? 0 : (long)k * rows * cols);
        for (long i = 0; i < (long)rows * cols; i++) m = fmax(m, f(p[i]));
    };
    blkmax(X.R, nu, nu, 0);
    blkmax(X.r, nu, 1, 0);
    const int kend = P.ti ? (N > 1 ? 2 : 1) : N;
    for (int k = 1; k < kend; k++) {
        blkmax(X.R, nu, nu, k);
        blkmax(X.S, nu, nx, k);
        blkmax(X.Q, nx, nx, k);
        blkmax(X.r, nu, 1, k);
        blkmax(X.q, nx, 1, k);
    }
    for (int i = 0; i < nx * nx; i++) m = fmax(m, f(X.Qf[i]));
    for (int i = 0; i < nx; i++) m = fmax(m, f(X.qf[i]));
    return m;
}

// Outputs (:2802-3007): u, x (stages 1..N), the input-equality fix, inf_norm_res, pi, lam / t.
void outputs(Mpc& P, const Data& X, bool eqfix, bool gen_norm, double mu, double* x, double* u, double* pi,
             double* lam, double* t, double* inf_norm_res) {
    const int N = P.N, nx = P.nx, nu = P.nu, nb = P.nb, ng = P.ng, ngN = P.ngN;
    for (int k = 0; k < N; k++)
        for (int i = 0; i < nu; i++) u[i + nu * k] = P.ux[k][i];
    for (int k = 1; k <= N; k++)
        for (int i = 0; i < nx; i++) x[i + nx * k] = P.ux[k][P.nuu[k] + i];
    if (eqfix)
        for (int k = 0; k < N; k++)
            for (int i = 0; i < P.nbu; i++)
                if (X.lb[i + P.blk(k)] == X.ub[i + P.blk(k)]) u[i + nu * k] = X.lb[i + P.blk(k)];
    double tmp = fabs(P.rrq[0][0]);
    for (int i = 0; i < nu; i++) tmp = fmax(tmp, fabs(P.rrq[0][i]));
    for (int k = 1; k < N; k++)
        for (int i = 0; i < nu + nx; i++) tmp = fmax(tmp, fabs(P.rrq[k][i]));
    for (int i = 0; i < nx; i++) tmp = fmax(tmp, fabs(P.rrq[N][i]));
    inf_norm_res[0] = tmp;
    tmp = fabs(P.rb[0][0]);
    for (int k = 0; k < N; k++)
        for (int i = 0; i < nx; i++) tmp = fmax(tmp, fabs(P.rb[k][i]));
    inf_norm_res[1] = tmp;
    tmp = fabs(P.rd[0][0]);
    for (int k = 0; k <= N; k++) {
        const int p0 = rup(P.nbb[k], BS), cnt = k == 0 ? P.nbu : (k < N ? nb : P.nbb[N]);
        for (int j = 0; j < cnt; j++) tmp = fmax(tmp, fmax(fabs(P.rd[k][j]), fabs(P.rd[k][p0 + j])));
    }
    for (int k = 0; k <= N; k++) {
        if (k < N && !gen_norm) continue;
        const int p0 = rup(P.nbb[k], BS), g0 = rup(P.ngg[k], BS);
        for (int j = 2 * p0; j < 2 * p0 + P.ngg[k]; j++)
            tmp = fmax(tmp, fmax(fabs(P.rd[k][j]), fabs(P.rd[k][g0 + j])));
    }
    inf_norm_res[2] = tmp;
    inf_norm_res[3] = mu;
    for (int k = 0; k < N; k++)
        for (int i = 0; i < nx; i++) pi[i + k * nx] = P.pi[k][i];
    const int s = 2 * nb + 2 * ng;
    for (int w = 0; w < 2; w++) {
        double* dst = w == 0 ? lam : t;
        const std::vector<double*>& src = w == 0 ? P.lam : P.t;
        if (!dst) continue;
        for (int k = 0; k < N; k++) {
            const int p0 = rup(P.nbb[k], BS);
            for (int j = 0; j < (k == 0 ? P.nbu : nb); j++) {
                dst[j + k * s] = src[k][j];
                dst[j + k * s + nb + ng] = src[k][p0 + j];
            }
        }
        {
            const int p0 = rup(P.nbb[N], BS);
            for (int j = 0; j < P.nbb[N]; j++) {
                dst[nu + j + N * s] = src[N][j];
                dst[nu + j + N * s + nb + ngN] = src[N][p0 + j];
            }
        }
        for (int k = 0; k < N; k++) {
            const int p0 = rup(P.nbb[k], BS), g0 = rup(P.ngg[k], BS);
            for (int j = 0; j < ng; j++) {
                dst[j + k * s + nb] = src[k][2 * p0 + j];
                dst[j + k * s + nb + ng + nb] = src[k][2 * p0 + g0 + j];
            }
        }
        {
            const int p0 = rup(P.nbb[N], BS), g0 = rup(ngN, BS);
            for (int j = 0; j < ngN; j++) {
                dst[j + N * s + nb] = src[N][2 * p0 + j];
                dst[j + N * s + nb + ngN + nb] = src[N][2 * p0 + g0 + j];
            }
        }
    }
}

double residuals(Mpc& P) {
    double mu = 0.0;
    d_res_mpc_hard_tv(P.N, P.nxx.data(), P.nuu.data(), P.nbb.data(), P.idxb.data(), P.ngg.data(), P.BAbt.data(),
                      P.b.data(), P.RSQ.data(), P.rq.data(), P.ux.data(), P.DCt.data(), P.d.data(), P.pi.data(),
                      P.lam.data(), P.t.data(), P.rrq.data(), P.rb.data(), P.rd.data(), &mu);
    return mu;
}

int ip_mpc(bool rowmajor, int* kk, int k_max, double mu0, double mu_tol, int N, int nx, int nu, int nb, int ng,
           int ngN, int time_invariant, int warm_start, const Data& X, double* x, double* u, double* pi, double* lam,
           double* t, double* inf_norm_res, double* work0, double* stat) {
    hk_set_error(0, nullptr);
    if (!check(N, nx, nu, nb, ng, ngN)) return HPMPC_MI355X_EUNSUPPORTED;
    Mpc P;
    dims(P, N, nx, nu, nb, ng, ngN, time_invariant != 0, rowmajor);
    carve(P, work0);
    pack(P, X, false);
    if (mu0 <= 0) mu0 = auto_mu0(P, X);
    for (int k = 0; k <= N; k++) {
        memset(P.ux[k], 0, sizeof(double) * (P.pnz + 4));
        if (k < N) memset(P.pi[k], 0, sizeof(double) * (P.pnx + 4));
    }
    if (warm_start) {  // :2764-2775
        for (int k = 0; k < N; k++)
            for (int i = 0; i < nu; i++) P.ux[k][i] = u[i + nu * k];
        for (int k = 1; k <= N; k++)
            for (int i = 0; i < nx; i++) P.ux[k][P.nuu[k] + i] = x[i + nx * k];
    }
    const int status = d_ip2_mpc_hard_tv(kk, k_max, mu0, mu_tol, 1e-8, warm_start, stat, N, P.nxx.data(),
                                         P.nuu.data(), P.nbb.data(), P.idxb.data(), P.ngg.data(), P.BAbt.data(),
                                         P.RSQ.data(), P.DCt.data(), P.d.data(), P.ux.data(), 1, P.pi.data(),
                                         P.lam.data(), P.t.data(), P.work);
    if (status <= HPMPC_MI355X_EUNSUPPORTED) return status;
    residual_q(P, X);
    const double mu = residuals(P);
    if (hpmpc_mi355x_last_error()) return hpmpc_mi355x_last_error();
    outputs(P, X, true, true, mu, x, u, pi, lam, t, inf_norm_res);
    return status;
}

void kkt_mpc(bool rowmajor, int N, int nx, int nu, int nb, int ng, int ngN, int time_invariant, const Data& X,
             double* x, double* u, double* pi, double* lam, double* t, double* inf_norm_res, double* work0) {
    hk_set_error(0, nullptr);
    if (!check(N, nx, nu, nb, ng, ngN)) return;
    Mpc P;
    dims(P, N, nx, nu, nb, ng, ngN, time_invariant != 0, rowmajor);
    carve(P, work0);
    pack(P, X, true);
    d_kkt_solve_new_rhs_mpc_hard_tv(N, P.nxx.data(), P.nuu.data(), P.nbb.data(), P.idxb.data(), P.ngg.data(),
                                    P.BAbt.data(), P.b.data(), P.RSQ.data(), P.rq.data(), P.DCt.data(), P.d.data(),
                                    P.ux.data(), 1, P.pi.data(), P.lam.data(), P.t.data(), P.work);
    if (hpmpc_mi355x_last_error()) return;
    residual_q(P, X);
    const double mu = residuals(P);
    if (hpmpc_mi355x_last_error()) return;
    outputs(P, X, false, !rowmajor, mu, x, u, pi, lam, t, inf_norm_res);
}

Data data(double* A, double* B, double* b, double* Q, double* Qf, double* S, double* R, double* q, double* qf,
          double* r, double* lb, double* ub, double* C, double* D, double* lg, double* ug, double* Cf, double* lgf,
          double* ugf, double* x) {
    return Data{A, B, b, Q, Qf, S, R, q, qf, r, lb, ub, C, D, lg, ug, Cf, lgf, ugf, x};
}

}  // namespace

// include/c_interface.h:40 -- declared by the reference, defined nowhere in it: the doubles of work0 the legacy
// wrappers below need (idxb tables, lib4 blocks, this library's d_ip2_mpc_hard_tv work space, vectors).
extern "C" int hpmpc_d_ip_mpc_hard_tv_work_space_size_doubles(int N, int nx, int nu, int nb, int ng, int ngN) {
    if (N < 1 || nx < 1) return 0;
    Mpc P;
    dims(P, N, nx, nu, nb, ng, ngN, false, false);
    carve(P, nullptr);
    return (int)((P.total + 7) / 8 + 8);
}

// include/c_interface.h:52 (interfaces/c/fortran_order_interface.c:1975)
extern "C" int fortran_order_d_ip_mpc_hard_tv(int* kk, int k_max, double mu0, double mu_tol, int N, int nx, int nu,
                                              int nb, int ng, int ngN, int time_invariant, int free_x0,
                                              int warm_start, double* A, double* B, double* b, double* Q, double* Qf,
                                              double* S, double* R, double* q, double* qf, double* r, double* lb,
                                              double* ub, double* C, double* D, double* lg, double* ug, double* Cf,
                                              double* lgf, double* ugf, double* x, double* u, double* pi, double* lam,
                                              double* t, double* inf_norm_res, double* work0, double* stat) {
    (void)free_x0;  // unused by the reference too
    return ip_mpc(false, kk, k_max, mu0, mu_tol, N, nx, nu, nb, ng, ngN, time_invariant, warm_start,
                  data(A, B, b, Q, Qf, S, R, q, qf, r, lb, ub, C, D, lg, ug, Cf, lgf, ugf, x), x, u, pi, lam, t,
                  inf_norm_res, work0, stat);
}

// include/c_interface.h:45 (interfaces/c/c_order_interface.c:1052); warm start as the fortran twin (the reference's
// c_order copies u, x in either case, which a cold start then zeroes)
extern "C" int c_order_d_ip_mpc_hard_tv(int* kk, int k_max, double mu0, double mu_tol, int N, int nx, int nu, int nb,
                                        int ng, int ngN, int time_invariant, int free_x0, int warm_start, double* A,
                                        double* B, double* b, double* Q, double* Qf, double* S, double* R, double* q,
                                        double* qf, double* r, double* lb, double* ub, double* C, double* D,
                                        double* lg, double* ug, double* Cf, double* lgf, double* ugf, double* x,
                                        double* u, double* pi, double* lam, double* t, double* inf_norm_res,
                                        double* work0, double* stat) {
    (void)free_x0;
    return ip_mpc(true, kk, k_max, mu0, mu_tol, N, nx, nu, nb, ng, ngN, time_invariant, warm_start,
                  data(A, B, b, Q, Qf, S, R, q, qf, r, lb, ub, C, D, lg, ug, Cf, lgf, ugf, x), x, u, pi, lam, t,
                  inf_norm_res, work0, stat);
}

// include/c_interface.h:53 (interfaces/c/fortran_order_interface.c:3017)
extern "C" void fortran_order_d_solve_kkt_new_rhs_mpc_hard_tv(
    int N, int nx, int nu, int nb, int ng, int ngN, int time_invariant, int free_x0, double* A, double* B, double* b,
    double* Q, double* Qf, double* S, double* R, double* q, double* qf, double* r, double* lb, double* ub, double* C,
    double* D, double* lg, double* ug, double* Cf, double* lgf, double* ugf, double* x, double* u, double* pi,
    double* lam, double* t, double* inf_norm_res, double* work0) {
    (void)free_x0;
    kkt_mpc(false, N, nx, nu, nb, ng, ngN, time_invariant,
            data(A, B, b, Q, Qf, S, R, q, qf, r, lb, ub, C, D, lg, ug, Cf, lgf, ugf, x), x, u, pi, lam, t,
            inf_norm_res, work0);
}

// include/c_interface.h:46 (interfaces/c/c_order_interface.c:2083)
extern "C" void c_order_d_solve_kkt_new_rhs_mpc_hard_tv(
    int N, int nx, int nu, int nb, int ng, int ngN, int time_invariant, int free_x0, double* A, double* B, double* b,
    double* Q, double* Qf, double* S, double* R, double* q, double* qf, double* r, double* lb, double* ub, double* C,
    double* D, double* lg, double* ug, double* Cf, double* lgf, double* ugf, double* x, double* u, double* pi,
    double* lam, double* t, double* inf_norm_res, double* work0) {
    (void)free_x0;
    kkt_mpc(true, N, nx, nu, nb, ng, ngN, time_invariant,
            data(A, B, b, Q, Qf, S, R, q, qf, r, lb, ub, C, D, lg, ug, Cf, lgf, ugf, x), x, u, pi, lam, t,
            inf_norm_res, work0);
}
