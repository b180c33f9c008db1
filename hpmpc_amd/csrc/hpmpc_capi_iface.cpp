// hpmpc_capi_iface.cpp -- the high-level entry points of include/c_interface.h:
// column-major (fortran_order_*) and row-major (c_order_*) problem data in, lib4 packing on the host, then the
// reference-named hot path of this library (d_ip2_res_mpc_hard_tv, d_part_cond / d_part_expand_solution,
// d_kkt_solve_new_rhs_res_mpc_hard_tv, d_res_mpc_hard_tv) -- every solve runs on the GPU.
//
// Follows interfaces/c/fortran_order_interface.c:53-688 (IPM wrapper), :1082-1300 (KKT re-solve wrapper) and
// interfaces/c/c_order_interface.c:53-691,692-1050 (row-major twins), interfaces/c/c_interface_work_space.c:70
// (work space size).  Differences, all documented in DESIGN.md:
//   * size errors return HPMPC_MI355X_EUNSUPPORTED with one stderr line instead of printf + exit(1);
//   * work0 is carved once by both wrappers (the reference's KKT wrapper looks for the IPM work space at a
//     different offset than its IPM wrapper leaves it, fortran_order_interface.c:1163-1174 vs :480-520); the
//     KKT re-solve therefore needs the IPM wrapper to have run on the full space (N2 == N), as in the reference;
//   * c_order with general constraints reads C[N] row-major like every other C[k] (the reference transposes
//     C[N] once more, c_order_interface.c:283).
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <vector>

#include "hpmpc_api.h"

extern "C" void hk_set_error(int code, const char* what);

namespace {

constexpr int BS = 4, NCL = 2;
inline int rup(int n, int m) { return (n + m - 1) / m * m; }
inline double& P4(double* A, int sd, int i, int j) { return A[(i / BS) * BS * sd + i % BS + BS * j]; }

// Dense m x n block (element (i, j) at A[i + j*lda]) into a lib4 matrix at row offset r0; tran: its transpose.
void pack(const double* A, int m, int n, int lda, bool tran, double* pA, int sd, int r0) {
    for (int j = 0; j < n; j++)
        for (int i = 0; i < m; i++) {
            if (tran)
                P4(pA, sd, r0 + j, i) = A[i + j * lda];
            else
                P4(pA, sd, r0 + i, j) = A[i + j * lda];
        }
}

// The carve of work0 shared by the IPM and KKT wrappers (all offsets in doubles from the aligned base).
struct Carve {
    int N = 0, N2 = 0;
    std::vector<int> nu, pnx, pnz, pnb, png, cnx, cnux, cng;
    std::vector<int> nx2, nu2, nb2, ng2;
    std::vector<double*> BAbt, DCt, RSQ, b, rq, d, ux, pi, lam, t, rb, rrq, rd;
    double* ws = nullptr;     // full-space IPM work space, or the condensed pipeline's memory
    long long ipm_bytes = 0, pc_mem = 0, pc_work = 0, ipm2_bytes = 0, px_work = 0;
    long long total = 0;      // bytes from the aligned base
};

bool carve(Carve& C, char* base, int N, int* nx, const int* nu_N, int* nb, int** hidxb, int* ng, int N2) {
    C.N = N;
    C.nu.assign(nu_N, nu_N + N + 1);
    C.nu[N] = 0;
    int ngM = 0;
    for (int k = 0; k < N; k++) ngM = ng[k] > ngM ? ng[k] : ngM;
    if (N2 > N || ngM > 0) N2 = N;  // fortran_order_interface.c:86-101
    if (N2 < 1) N2 = N;
    C.N2 = N2;
    auto& nu = C.nu;
    for (auto* v : {&C.pnx, &C.pnz, &C.pnb, &C.png, &C.cnx, &C.cnux, &C.cng}) v->resize(N + 1);
    for (int k = 0; k <= N; k++) {
        C.pnx[k] = rup(nx[k], BS);
        C.pnz[k] = rup(nu[k] + nx[k] + 1, BS);
        C.pnb[k] = rup(nb[k], BS);
        C.png[k] = rup(ng[k], BS);
        C.cnx[k] = rup(nx[k], NCL);
        C.cnux[k] = rup(nu[k] + nx[k], NCL);
        C.cng[k] = rup(ng[k], NCL);
    }
    long long o = 64 / 8;  // header: [0] = N2 the IPM ran on
    auto take = [&](std::vector<double*>& v, int n, auto size) {
        v.resize(n);
        for (int k = 0; k < n; k++) {
            v[k] = base ? reinterpret_cast<double*>(base) + o : nullptr;
            o += size(k);
        }
    };
    take(C.BAbt, N, [&](int k) { return (long long)C.pnz[k] * C.cnx[k + 1]; });
    take(C.DCt, N + 1, [&](int k) { return (long long)C.pnz[k] * C.cng[k]; });
    take(C.RSQ, N + 1, [&](int k) { return (long long)C.pnz[k] * C.cnux[k]; });
    take(C.b, N, [&](int k) { return (long long)C.pnx[k + 1]; });
    take(C.rq, N + 1, [&](int k) { return (long long)C.pnz[k]; });
    take(C.d, N + 1, [&](int k) { return 2LL * C.pnb[k] + 2 * C.png[k]; });
    take(C.ux, N + 1, [&](int k) { return (long long)C.pnz[k]; });
    take(C.pi, N, [&](int k) { return (long long)C.pnx[k + 1]; });
    take(C.lam, N + 1, [&](int k) { return 2LL * C.pnb[k] + 2 * C.png[k] + 4; });
    take(C.t, N + 1, [&](int k) { return 2LL * C.pnb[k] + 2 * C.png[k] + 4; });
    take(C.rb, N, [&](int k) { return (long long)C.pnx[k + 1]; });
    take(C.rrq, N + 1, [&](int k) { return (long long)C.pnz[k]; });
    take(C.rd, N + 1, [&](int k) { return 2LL * C.pnb[k] + 2 * C.png[k] + 4; });
    o = (o + 7) / 8 * 8;
    C.ws = base ? reinterpret_cast<double*>(base) + o : nullptr;
    if (N2 == N) {
        C.ipm_bytes = d_ip2_res_mpc_hard_tv_work_space_size_bytes(N, nx, C.nu.data(), nb, ng);
        o += (C.ipm_bytes + 63) / 64 * 8;
    } else {
        C.nx2.resize(N2 + 1);
        C.nu2.resize(N2 + 1);
        C.nb2.resize(N2 + 1);
        C.ng2.resize(N2 + 1);
        d_part_cond_compute_problem_size(N, nx, C.nu.data(), nb, hidxb, ng, N2, C.nx2.data(), C.nu2.data(),
                                         C.nb2.data(), C.ng2.data());
        C.pc_mem = d_part_cond_memory_space_size_bytes(N, nx, C.nu.data(), nb, hidxb, ng, N2, C.nx2.data(),
                                                       C.nu2.data(), C.nb2.data(), C.ng2.data());
        C.pc_work = d_part_cond_work_space_size_bytes(N, nx, C.nu.data(), nb, hidxb, ng, N2, C.nx2.data(),
                                                      C.nu2.data(), C.nb2.data(), C.ng2.data());
        C.ipm2_bytes = d_ip2_res_mpc_hard_tv_work_space_size_bytes(N2, C.nx2.data(), C.nu2.data(), C.nb2.data(),
                                                                   C.ng2.data());
        C.px_work = d_part_expand_work_space_size_bytes(N, nx, C.nu.data(), nb, ng);
        long long s = (C.pc_mem + 63) / 64 * 64 + (C.pc_work + 63) / 64 * 64 + (C.ipm2_bytes + 63) / 64 * 64 +
                      (C.px_work + 63) / 64 * 64;
        for (int k = 0; k <= N2; k++) {
            const int pz = rup(C.nu2[k] + C.nx2[k] + 1, BS), pc = 2 * rup(C.nb2[k], BS) + 2 * rup(C.ng2[k], BS) + 4;
            s += 8LL * (pz + (k < N2 ? rup(C.nx2[k + 1], BS) : 0) + 2 * pc);
        }
        o += (s + 63) / 64 * 8;
    }
    C.total = o * 8;
    return true;
}

char* aligned(void* work0) { return reinterpret_cast<char*>(((uintptr_t)work0 + 63) / 64 * 64); }

bool check_sizes(int N, int* nx, const int* nu, int* nb) {
    for (int k = 0; k <= N; k++) {
        const int u = k < N ? nu[k] : 0;
        if (nb[k] > u + nx[k]) {
            char msg[160];
            snprintf(msg, sizeof msg, "stage %d: nb=%d larger than nu+nx=%d (fortran_order_interface.c:106-114)", k,
                     nb[k], u + nx[k]);
            hk_set_error(HPMPC_MI355X_EUNSUPPORTED, msg);
            return false;
        }
    }
    return true;
}

// Problem data -> lib4 stage blocks, b / rq vectors and bounds.  rowmajor: the c_order layout.
void pack_problem(Carve& C, int* nx, int* nb, int** hidxb, int* ng, bool rowmajor, double** A, double** B, double** b,
                  double** Q, double** S, double** R, double** q, double** r, double** lb, double** ub, double** Cm,
                  double** D, double** lg, double** ug, bool matrices) {
    const int N = C.N;
    const auto& nu = C.nu;
    for (int k = 0; k < N; k++) {
        const int sd = C.cnx[k + 1], nx1 = nx[k + 1];
        if (matrices) {
            memset(C.BAbt[k], 0, sizeof(double) * C.pnz[k] * sd);
            if (rowmajor) {  // B (nx1 x nu) row-major == B' col-major
                pack(B[k], nu[k], nx1, nu[k], false, C.BAbt[k], sd, 0);
                pack(A[k], nx[k], nx1, nx[k], false, C.BAbt[k], sd, nu[k]);
            } else {
                pack(B[k], nx1, nu[k], nx1, true, C.BAbt[k], sd, 0);
                pack(A[k], nx1, nx[k], nx1, true, C.BAbt[k], sd, nu[k]);
            }
        }
        for (int j = 0; j < nx1; j++) {
            C.b[k][j] = b[k][j];
            P4(C.BAbt[k], sd, nu[k] + nx[k], j) = b[k][j];
        }
    }
    if (matrices)
        for (int k = 0; k <= N; k++) {
            const int sd = C.cng[k];
            memset(C.DCt[k], 0, sizeof(double) * C.pnz[k] * sd);
            if (ng[k] == 0) continue;
            if (rowmajor) {
                if (k < N) pack(D[k], nu[k], ng[k], nu[k], false, C.DCt[k], sd, 0);
                pack(Cm[k], nx[k], ng[k], nx[k], false, C.DCt[k], sd, nu[k]);
            } else {
                if (k < N) pack(D[k], ng[k], nu[k], ng[k], true, C.DCt[k], sd, 0);
                pack(Cm[k], ng[k], nx[k], ng[k], true, C.DCt[k], sd, nu[k]);
            }
        }
    for (int k = 0; k <= N; k++) {
        const int sd = C.cnux[k], nuk = nu[k], nxk = nx[k], nux = nuk + nxk;
        if (matrices) {
            memset(C.RSQ[k], 0, sizeof(double) * C.pnz[k] * sd);
            if (k < N) {
                if (rowmajor) {
                    pack(R[k], nuk, nuk, nuk, true, C.RSQ[k], sd, 0);
                    pack(S[k], nxk, nuk, nxk, false, C.RSQ[k], sd, nuk);
                } else {
                    pack(R[k], nuk, nuk, nuk, false, C.RSQ[k], sd, 0);
                    pack(S[k], nuk, nxk, nuk, true, C.RSQ[k], sd, nuk);
                }
            }
            for (int j = 0; j < nxk; j++)  // Q into rows / cols nu.. (symmetric: either order)
                for (int i = 0; i < nxk; i++)
                    P4(C.RSQ[k], sd, nuk + i, nuk + j) = rowmajor ? Q[k][j + i * nxk] : Q[k][i + j * nxk];
        }
        for (int j = 0; j < nuk; j++) {
            C.rq[k][j] = r[k][j];
            P4(C.RSQ[k], sd, nux, j) = r[k][j];
        }
        for (int j = 0; j < nxk; j++) {
            C.rq[k][nuk + j] = q[k][j];
            P4(C.RSQ[k], sd, nux, nuk + j) = q[k][j];
        }
    }
    for (int k = 0; k <= N; k++) {
        memset(C.d[k], 0, sizeof(double) * (2 * C.pnb[k] + 2 * C.png[k]));
        for (int j = 0; j < nb[k]; j++) {  // :331-375 (inputs and states alike)
            C.d[k][j] = lb[k][j];
            C.d[k][j + C.pnb[k]] = ub[k][j];
        }
        for (int j = 0; j < ng[k]; j++) {
            C.d[k][2 * C.pnb[k] + j] = lg[k][j];
            C.d[k][2 * C.pnb[k] + C.png[k] + j] = ug[k][j];
        }
    }
}

// Outputs shared by both wrappers (:590-686): u, x, the equality-box fix, residual infinity norms, pi, lam.
void outputs(Carve& C, int* nx, int* nb, int** hidxb, int* ng, double** lb, double** ub, double** x, double** u,
             double** pi, double** lam, double* inf_norm_res, double** t = nullptr) {
    const int N = C.N;
    const auto& nu = C.nu;
    for (int k = 0; k < N; k++)
        for (int j = 0; j < nu[k]; j++) u[k][j] = C.ux[k][j];
    for (int k = 0; k <= N; k++)
        for (int j = 0; j < nx[k]; j++) x[k][j] = C.ux[k][nu[k] + j];
    for (int k = 0; k < N; k++)
        for (int j = 0; j < nb[k] && hidxb[k][j] < nu[k]; j++)
            if (lb[k][j] == ub[k][j]) u[k][hidxb[k][j]] = lb[k][j];
    double mu = 0.0;
    d_res_mpc_hard_tv(N, nx, C.nu.data(), nb, hidxb, ng, C.BAbt.data(), C.b.data(), C.RSQ.data(), C.rq.data(),
                      C.ux.data(), C.DCt.data(), C.d.data(), C.pi.data(), C.lam.data(), C.t.data(), C.rrq.data(),
                      C.rb.data(), C.rd.data(), &mu);
    double tmp = fabs(C.rrq[0][0]);
    for (int k = 0; k < N; k++)
        for (int j = 0; j < nu[k] + nx[k]; j++) tmp = fmax(tmp, fabs(C.rrq[k][j]));
    for (int j = 0; j < nx[N]; j++) tmp = fmax(tmp, fabs(C.rrq[N][j]));
    inf_norm_res[0] = tmp;
    tmp = fabs(C.rb[0][0]);
    for (int k = 0; k < N; k++)
        for (int j = 0; j < nx[k + 1]; j++) tmp = fmax(tmp, fabs(C.rb[k][j]));
    inf_norm_res[1] = tmp;
    tmp = fabs(C.rd[0][0]);
    for (int k = 0; k <= N; k++)
        for (int j = 0; j < nb[k]; j++) {
            tmp = fmax(tmp, fabs(C.rd[k][j]));
            tmp = fmax(tmp, fabs(C.rd[k][j + C.pnb[k]]));
        }
    for (int k = 0; k <= N; k++)
        for (int j = 0; j < ng[k]; j++) {
            tmp = fmax(tmp, fabs(C.rd[k][2 * C.pnb[k] + j]));
            tmp = fmax(tmp, fabs(C.rd[k][2 * C.pnb[k] + j + C.png[k]]));
        }
    inf_norm_res[2] = tmp;
    inf_norm_res[3] = mu;
    for (int k = 0; k < N; k++)
        for (int j = 0; j < nx[k + 1]; j++) pi[k][j] = C.pi[k][j];
    for (int k = 0; k <= N; k++) {
        for (int j = 0; j < nb[k]; j++) {
            lam[k][j] = C.lam[k][j];
            lam[k][j + nb[k]] = C.lam[k][j + C.pnb[k]];
        }
        for (int j = 0; j < ng[k]; j++) {
            lam[k][2 * nb[k] + j] = C.lam[k][2 * C.pnb[k] + j];
            lam[k][2 * nb[k] + j + ng[k]] = C.lam[k][2 * C.pnb[k] + j + C.png[k]];
        }
    }
    if (!t) return;
    for (int k = 0; k <= N; k++) {  // the single-Newton wrapper's t, compact like lam (:1057-1075)
        for (int j = 0; j < nb[k]; j++) {
            t[k][j] = C.t[k][j];
            t[k][j + nb[k]] = C.t[k][j + C.pnb[k]];
        }
        for (int j = 0; j < ng[k]; j++) {
            t[k][2 * nb[k] + j] = C.t[k][2 * C.pnb[k] + j];
            t[k][2 * nb[k] + j + ng[k]] = C.t[k][2 * C.pnb[k] + j + C.png[k]];
        }
    }
}

// work0's header (the first 64 bytes of the carve): [0] the horizon the IPM ran on (N2), [1] a tag, [2] N -- so that
// the KKT re-solve can tell a work space the IPM wrapper wrote from one it never saw.
constexpr double WORK0_TAG = 0x1.48504d5043e5fp+33;
// Set only after a solve that left its factor in work0; cleared (clear_work0) when a wrapper call starts, so that a
// call that returns early (size error, condensing error, a device failure) leaves a work space the re-solve refuses.
void mark_work0(char* base, int N2, int N) {
    double* h = reinterpret_cast<double*>(base);
    h[0] = N2;
    h[1] = WORK0_TAG;
    h[2] = N;
}
void clear_work0(char* base) { reinterpret_cast<double*>(base)[1] = 0.0; }

int ip_ocp(bool rowmajor, int* kk, int k_max, double mu0, double mu_tol, int N, int* nx, int* nu_N, int* nb,
           int** hidxb, int* ng, int N2, int warm_start, double** A, double** B, double** b, double** Q, double** S,
           double** R, double** q, double** r, double** lb, double** ub, double** Cm, double** D, double** lg,
           double** ug, double** x, double** u, double** pi, double** lam, double* inf_norm_res, void* work0,
           double* stat) {
    hk_set_error(0, nullptr);
    if (!check_sizes(N, nx, nu_N, nb)) return HPMPC_MI355X_EUNSUPPORTED;
    char* base = aligned(work0);
    Carve C;
    carve(C, base, N, nx, nu_N, nb, hidxb, ng, N2);
    const auto& nu = C.nu;
    pack_problem(C, nx, nb, hidxb, ng, rowmajor, A, B, b, Q, S, R, q, r, lb, ub, Cm, D, lg, ug, true);
    if (mu0 <= 0) {  // :311-329: the largest cost entry
        for (int k = 0; k < N; k++) {
            for (int j = 0; j < nu[k] * nu[k]; j++) mu0 = fmax(mu0, R[k][j]);
            for (int j = 0; j < nx[k] * nu[k]; j++) mu0 = fmax(mu0, S[k][j]);
            for (int j = 0; j < nx[k] * nx[k]; j++) mu0 = fmax(mu0, Q[k][j]);
            for (int j = 0; j < nu[k]; j++) mu0 = fmax(mu0, r[k][j]);
            for (int j = 0; j < nx[k]; j++) mu0 = fmax(mu0, q[k][j]);
        }
        for (int j = 0; j < nx[N] * nx[N]; j++) mu0 = fmax(mu0, Q[N][j]);
        for (int j = 0; j < nx[N]; j++) mu0 = fmax(mu0, q[N][j]);
    }
    const double alpha_min = 1e-8;
    clear_work0(base);
    int status;
    if (C.N2 < N) {  // partial condensing (:388-545)
        const int N2c = C.N2;
        char* p = reinterpret_cast<char*>(C.ws);
        void* mem = p;
        p += (C.pc_mem + 63) / 64 * 64;
        void* wpc = p;
        p += (C.pc_work + 63) / 64 * 64;
        double* wipm = reinterpret_cast<double*>(p);
        p += (C.ipm2_bytes + 63) / 64 * 64;
        void* wpx = p;
        p += (C.px_work + 63) / 64 * 64;
        std::vector<double*> BAbt2(N2c + 1), RSQ2(N2c + 1), DCt2(N2c + 1), d2(N2c + 1), ux2(N2c + 1), pi2(N2c + 1),
            lam2(N2c + 1), t2(N2c + 1);
        std::vector<int*> idxb2(N2c + 1);
        double* dp = reinterpret_cast<double*>(p);
        for (int k = 0; k <= N2c; k++) {
            ux2[k] = dp;
            dp += rup(C.nu2[k] + C.nx2[k] + 1, BS);
        }
        for (int k = 0; k < N2c; k++) {
            pi2[k] = dp;
            dp += rup(C.nx2[k + 1], BS);
        }
        for (int k = 0; k <= N2c; k++) {
            const int pc = 2 * rup(C.nb2[k], BS) + 2 * rup(C.ng2[k], BS) + 4;
            lam2[k] = dp;
            dp += pc;
            t2[k] = dp;
            dp += pc;
        }
        d_part_cond(N, nx, C.nu.data(), nb, hidxb, ng, C.BAbt.data(), C.RSQ.data(), C.DCt.data(), C.d.data(), N2c,
                    C.nx2.data(), C.nu2.data(), C.nb2.data(), idxb2.data(), C.ng2.data(), BAbt2.data(), RSQ2.data(),
                    DCt2.data(), d2.data(), mem, wpc);
        int e = hpmpc_mi355x_last_error();
        if (e) return e;
        status = d_ip2_res_mpc_hard_tv(kk, k_max, mu0, mu_tol, alpha_min, 0, stat, N2c, C.nx2.data(), C.nu2.data(),
                                       C.nb2.data(), idxb2.data(), C.ng2.data(), BAbt2.data(), RSQ2.data(),
                                       DCt2.data(), d2.data(), ux2.data(), 1, pi2.data(), lam2.data(), t2.data(), wipm);
        if (status <= HPMPC_MI355X_EUNSUPPORTED) return status;
        d_part_expand_solution(N, nx, C.nu.data(), nb, hidxb, ng, C.BAbt.data(), C.b.data(), C.RSQ.data(),
                               C.rq.data(), C.DCt.data(), C.ux.data(), C.pi.data(), C.lam.data(), C.t.data(), N2c,
                               C.nx2.data(), C.nu2.data(), C.nb2.data(), idxb2.data(), C.ng2.data(), ux2.data(),
                               pi2.data(), lam2.data(), t2.data(), wpx);
        if (hpmpc_mi355x_last_error()) return hpmpc_mi355x_last_error();
    } else {
        if (warm_start) {
            for (int k = 0; k < N; k++)
                for (int j = 0; j < nu[k]; j++) C.ux[k][j] = u[k][j];
            for (int k = 0; k <= N; k++)
                for (int j = 0; j < nx[k]; j++) C.ux[k][nu[k] + j] = x[k][j];
        }
        status = d_ip2_res_mpc_hard_tv(kk, k_max, mu0, mu_tol, alpha_min, warm_start, stat, N, nx, C.nu.data(), nb,
                                       hidxb, ng, C.BAbt.data(), C.RSQ.data(), C.DCt.data(), C.d.data(), C.ux.data(),
                                       1, C.pi.data(), C.lam.data(), C.t.data(), C.ws);
        if (status <= HPMPC_MI355X_EUNSUPPORTED) return status;
    }
    mark_work0(base, C.N2, N);
    outputs(C, nx, nb, hidxb, ng, lb, ub, x, u, pi, lam, inf_norm_res);
    return status;
}

void kkt_ocp(bool rowmajor, int N, int* nx, int* nu, int* nb, int** hidxb, int* ng, double** A, double** B,
             double** b, double** Q, double** S, double** R, double** q, double** r, double** lb, double** ub,
             double** Cm, double** D, double** lg, double** ug, double** x, double** u, double** pi, double** lam,
             double* inf_norm_res, double* work0) {
    hk_set_error(0, nullptr);
    char* base = aligned(work0);
    Carve C;
    carve(C, base, N, nx, nu, nb, hidxb, ng, N);
    const double* hd = reinterpret_cast<const double*>(base);
    if (hd[1] != WORK0_TAG || hd[2] != (double)N) {
        // e.g. test_problems/test_d_ip_hard.c:892 calls the re-solve on a work space no IPM wrapper has written (its
        // IPM call at :849 is commented out): the reference then reads whatever the buffer holds, this library
        // refuses instead of solving with an undefined factor
        hk_set_error(HPMPC_MI355X_EUNSUPPORTED, "KKT re-solve: work0 holds no factor of this problem's IPM wrapper "
                                                "call (call fortran_order_ / c_order_d_ip_ocp_hard_tv on it first)");
        return;
    }
    if ((int)hd[0] != N) {
        hk_set_error(HPMPC_MI355X_EUNSUPPORTED, "KKT re-solve after a partially condensed IPM (the wrapper keeps "
                                                "the full-space factor only when N2 == N)");
        return;
    }
    // new right-hand sides only: the stage matrices packed by the IPM wrapper stay in work0 (:1232-1290)
    pack_problem(C, nx, nb, hidxb, ng, rowmajor, A, B, b, Q, S, R, q, r, lb, ub, Cm, D, lg, ug, false);
    d_kkt_solve_new_rhs_res_mpc_hard_tv(N, nx, C.nu.data(), nb, hidxb, ng, C.BAbt.data(), C.b.data(), C.RSQ.data(),
                                        C.rq.data(), C.DCt.data(), C.d.data(), C.ux.data(), 1, C.pi.data(),
                                        C.lam.data(), C.t.data(), C.ws);
    if (hpmpc_mi355x_last_error()) return;
    outputs(C, nx, nb, hidxb, ng, lb, ub, x, u, pi, lam, inf_norm_res);
}

}  // namespace

// include/c_interface.h:66 (interfaces/c/fortran_order_interface.c:690-1080): k_max Newton steps of the residual IPM
// from the caller's (ux0, pi0, lam0, t0) with the fixed centering target mu0 (d_ip2_res_mpc_hard_tv_single_newton_step),
// always on the full space (the reference computes N2 but never condenses here), then the common outputs plus t.
extern "C" int fortran_order_d_ip_ocp_hard_tv_single_newton_step(
    int* kk, int k_max, double mu0, double mu_tol, int N, int* nx, int* nu_N, int* nb, int** hidxb, int* ng, int N2,
    int warm_start, double** A, double** B, double** b, double** Q, double** S, double** R, double** q, double** r,
    double** lb, double** ub, double** Cm, double** D, double** lg, double** ug, double** x, double** u, double** pi,
    double** lam, double** t, double* inf_norm_res, void* work0, double* stat, double** ux0, double** pi0,
    double** lam0, double** t0) {
    (void)N2;
    hk_set_error(0, nullptr);
    if (!check_sizes(N, nx, nu_N, nb)) return HPMPC_MI355X_EUNSUPPORTED;
    char* base = aligned(work0);
    Carve C;
    carve(C, base, N, nx, nu_N, nb, hidxb, ng, N);
    pack_problem(C, nx, nb, hidxb, ng, false, A, B, b, Q, S, R, q, r, lb, ub, Cm, D, lg, ug, true);
    clear_work0(base);
    const double alpha_min = 1e-8;
    const int status = d_ip2_res_mpc_hard_tv_single_newton_step(
        kk, k_max, mu0, mu_tol, alpha_min, warm_start, stat, N, nx, C.nu.data(), nb, hidxb, ng, C.BAbt.data(),
        C.RSQ.data(), C.DCt.data(), C.d.data(), C.ux.data(), 1, C.pi.data(), C.lam.data(), C.t.data(), C.ws, ux0, pi0,
        lam0, t0);
    if (status <= HPMPC_MI355X_EUNSUPPORTED) return status;
    mark_work0(base, N, N);
    outputs(C, nx, nb, hidxb, ng, lb, ub, x, u, pi, lam, inf_norm_res, t);
    return status;
}

// include/c_interface.h:60.  The reference defines it only in its BLASFEO interface
// (interfaces/c/fortran_order_interface_libstr.c:110): the work space of hpmpc_d_ip_ocp_hard_tv_work_space_size_bytes
// for a problem whose boxes are given by count -- nbu[k] boxed inputs and nbx[k] boxed states per stage -- instead
// of by index.  This library's carve depends on the box positions only through how many are input / state boxes
// (partial condensing turns inner state boxes into general constraints, d_part_cond.c:716-731), so the size is that
// of the canonical index set [0, nbu[k]) u [nu[k], nu[k] + nbx[k]).
extern "C" int hpmpc_d_ip_ocp_hard_tv_work_space_size_bytes_noidxb(int N, int* nx, int* nu, int* nb, int* nbx, int* nbu,
                                                                   int* ng, int N2) {
    std::vector<std::vector<int>> idx(N + 1);
    std::vector<int*> hidxb(N + 1);
    std::vector<int> nbk(N + 1);
    for (int k = 0; k <= N; k++) {
        const int u = k < N ? nu[k] : 0;
        const int bu = nbu[k] < u ? nbu[k] : u, bx = nbx[k] < nx[k] ? nbx[k] : nx[k];
        for (int j = 0; j < bu; j++) idx[k].push_back(j);
        for (int j = 0; j < bx; j++) idx[k].push_back(u + j);
        nbk[k] = nb[k] > bu + bx ? nb[k] : bu + bx;
        while ((int)idx[k].size() < nbk[k]) idx[k].push_back((int)idx[k].size());  // nb beyond nbu + nbx (sizes only)
        hidxb[k] = idx[k].data();
    }
    return hpmpc_d_ip_ocp_hard_tv_work_space_size_bytes(N, nx, nu, nbk.data(), hidxb.data(), ng, N2);
}

// include/c_interface.h:59 (interfaces/c/c_interface_work_space.c:70)
extern "C" int hpmpc_d_ip_ocp_hard_tv_work_space_size_bytes(int N, int* nx, int* nu, int* nb, int** hidxb, int* ng,
                                                            int N2) {
    Carve C;
    carve(C, nullptr, N, nx, nu, nb, hidxb, ng, N2);
    return (int)(C.total + 2 * 64);
}

// include/c_interface.h:65 (interfaces/c/fortran_order_interface.c:53)
extern "C" int fortran_order_d_ip_ocp_hard_tv(int* kk, int k_max, double mu0, double mu_tol, int N, int* nx, int* nu,
                                              int* nb, int** hidxb, int* ng, int N2, int warm_start, double** A,
                                              double** B, double** b, double** Q, double** S, double** R, double** q,
                                              double** r, double** lb, double** ub, double** C, double** D,
                                              double** lg, double** ug, double** x, double** u, double** pi,
                                              double** lam, double* inf_norm_res, void* work0, double* stat) {
    return ip_ocp(false, kk, k_max, mu0, mu_tol, N, nx, nu, nb, hidxb, ng, N2, warm_start, A, B, b, Q, S, R, q, r, lb,
                  ub, C, D, lg, ug, x, u, pi, lam, inf_norm_res, work0, stat);
}

// include/c_interface.h:62 (interfaces/c/c_order_interface.c:53)
extern "C" int c_order_d_ip_ocp_hard_tv(int* kk, int k_max, double mu0, double mu_tol, int N, int* nx, int* nu, int* nb,
                                        int** hidxb, int* ng, int N2, int warm_start, double** A, double** B,
                                        double** b, double** Q, double** S, double** R, double** q, double** r,
                                        double** lb, double** ub, double** C, double** D, double** lg, double** ug,
                                        double** x, double** u, double** pi, double** lam, double* inf_norm_res,
                                        void* work0, double* stat) {
    return ip_ocp(true, kk, k_max, mu0, mu_tol, N, nx, nu, nb, hidxb, ng, N2, warm_start, A, B, b, Q, S, R, q, r, lb,
                  ub, C, D, lg, ug, x, u, pi, lam, inf_norm_res, work0, stat);
}

// include/c_interface.h:67 (interfaces/c/fortran_order_interface.c:1082)
extern "C" void fortran_order_d_solve_kkt_new_rhs_ocp_hard_tv(int N, int* nx, int* nu, int* nb, int** hidxb, int* ng,
                                                              double** A, double** B, double** b, double** Q,
                                                              double** S, double** R, double** q, double** r,
                                                              double** lb, double** ub, double** C, double** D,
                                                              double** lg, double** ug, double** x, double** u,
                                                              double** pi, double** lam, double* inf_norm_res,
                                                              double* work0) {
    kkt_ocp(false, N, nx, nu, nb, hidxb, ng, A, B, b, Q, S, R, q, r, lb, ub, C, D, lg, ug, x, u, pi, lam, inf_norm_res,
            work0);
}

// include/c_interface.h:63 (interfaces/c/c_order_interface.c:692)
extern "C" void c_order_d_solve_kkt_new_rhs_ocp_hard_tv(int N, int* nx, int* nu, int* nb, int** hidxb, int* ng,
                                                        double** A, double** B, double** b, double** Q, double** S,
                                                        double** R, double** q, double** r, double** lb, double** ub,
                                                        double** C, double** D, double** lg, double** ug, double** x,
                                                        double** u, double** pi, double** lam, double* inf_norm_res,
                                                        double* work0) {
    kkt_ocp(true, N, nx, nu, nb, hidxb, ng, A, B, b, Q, S, R, q, r, lb, ub, C, D, lg, ug, x, u, pi, lam, inf_norm_res,
            work0);
}

// ------------------------------------------------------------------------------------------------
// Soft constraints: fortran_order_d_ip_ocp_soft_tv (interfaces/c/fortran_order_interface.c:1442-1971) and its
// work-space size (interfaces/c/c_interface_work_space.c:177-236).  Packing on the host into private buffers (work0
// is not used), then this library's d_ip2_mpc_soft_tv and d_res_mpc_soft_tv -- both on the GPU.  As the reference:
// no partial condensing; idxb = the nb hard boxes then the ns soft ones, lb / ub hold nb + ns bounds; Z[k] =
// [lower (ns) | upper (ns)]; mu0 <= 0 -> the largest entry (not absolute value) of R, S, Q, r, q, Z, z.  Two
// reference defects are handled as follows (soft constraints):
//   * the reference never copies z into the IPM's hz (:1712-1719 fill hZ only), so its IPM sees the contents of
//     work0 there -- zeros for a zeroed work0; the linear slack penalty passed to the IPM here is zero;
//   * its residual call passes the arguments shifted by one (an extra hb after hpBAbt and no hrz, :1880 against
//     mpc_solvers.h:71), so its inf_norm_res comes from scrambled inputs; here d_res_mpc_soft_tv is called as
//     declared (r_q / r_b / r_d of the returned iterate, with the same zero z).
// ------------------------------------------------------------------------------------------------
extern "C" int hpmpc_d_ip_ocp_soft_tv_work_space_size_bytes(int N, int* nx, int* nu, int* nb, int** hidxb, int* ng,
                                                             int* ns) {
    (void)hidxb;
    long long d_size = BS;
    for (int k = 0; k <= N; k++) {
        const int u = k < N ? nu[k] : 0;
        const int pnx = rup(nx[k], BS), pnz = rup(u + nx[k] + 1, BS), pnb = rup(nb[k], BS), png = rup(ng[k], BS),
                  pns = rup(ns[k], BS), cnx1 = k < N ? rup(nx[k + 1], NCL) : 0, cnux = rup(u + nx[k], NCL),
                  cng = rup(ng[k], NCL);
        d_size += (long long)pnz * cnx1 + (long long)pnz * cng + (long long)pnz * cnux + 3 * pnx + 3 * pnz + 8 * pnb +
                  8 * png + 16 * pns;
    }
    std::vector<int> nuv(nu, nu + N + 1);
    nuv[N] = 0;
    long long size = 2 * 64 + d_ip2_mpc_soft_tv_work_space_size_bytes(N, nx, nuv.data(), nb, ng, ns) + d_size * 8;
    return (int)((size + 63) / 64 * 64);
}

// include/c_interface.h:71 (interfaces/c/fortran_order_interface.c:1442)
extern "C" int fortran_order_d_ip_ocp_soft_tv(int* kk, int k_max, double mu0, double mu_tol, int N, int* nx, int* nu_N,
                                              int* nb, int** hidxb, int* ng, int* ns, int warm_start, double** A,
                                              double** B, double** b, double** Q, double** S, double** R, double** q,
                                              double** r, double** Z, double** z, double** lb, double** ub, double** C,
                                              double** D, double** lg, double** ug, double** x, double** u,
                                              double** pi, double** lam, double* inf_norm_res, void* work0,
                                              double* stat) {
    (void)work0;
    hk_set_error(0, nullptr);
    std::vector<int> nu(nu_N, nu_N + N + 1);
    nu[N] = 0;
    if (!check_sizes(N, nx, nu.data(), nb)) return HPMPC_MI355X_EUNSUPPORTED;
    const int n1 = N + 1;
    std::vector<std::vector<double>> vBAbt(N), vDCt(n1), vRSQ(n1), vrq(n1), vZ(n1), vz(n1), vd(n1), vux(n1),
        vpi(N), vlam(n1), vt(n1), vrb(N), vrrq(n1), vrd(n1), vrz(n1);
    std::vector<double*> pBAbt(N), pDCt(n1), pRSQ(n1), prq(n1), pZ(n1), pz(n1), pd(n1), pux(n1), ppi(N), plam(n1),
        pt(n1), prb(N), prrq(n1), prd(n1), prz(n1);
    std::vector<int> pnb(n1), png(n1), pns(n1);
    for (int k = 0; k <= N; k++) {
        const int nuk = nu[k], nxk = nx[k], nux = nuk + nxk, pnz = rup(nux + 1, BS), cnux = rup(nux, NCL);
        pnb[k] = rup(nb[k], BS);
        png[k] = rup(ng[k], BS);
        pns[k] = rup(ns[k], BS);
        const int ncv = 2 * pnb[k] + 2 * png[k] + 4 * pns[k], nd = 2 * pnb[k] + 2 * png[k] + 2 * pns[k];
        auto mk = [](std::vector<double>& v, size_t n, std::vector<double*>& p, int k) {
            v.assign(n + 8, 0.0);
            p[k] = v.data();
        };
        if (k < N) {
            const int nx1 = nx[k + 1], cnx1 = rup(nx1, NCL);
            mk(vBAbt[k], (size_t)pnz * cnx1, pBAbt, k);
            mk(vpi[k], rup(nx1, BS), ppi, k);
            mk(vrb[k], rup(nx1, BS), prb, k);
            double* M = pBAbt[k];
            pack(B[k], nx1, nuk, nx1, true, M, cnx1, 0);
            pack(A[k], nx1, nxk, nx1, true, M, cnx1, nuk);
            for (int j = 0; j < nx1; j++) P4(M, cnx1, nux, j) = b[k][j];
        }
        mk(vDCt[k], (size_t)pnz * rup(ng[k], NCL), pDCt, k);
        if (ng[k] > 0) {
            const int cng = rup(ng[k], NCL);
            if (k < N) pack(D[k], ng[k], nuk, ng[k], true, pDCt[k], cng, 0);
            pack(C[k], ng[k], nxk, ng[k], true, pDCt[k], cng, nuk);
        }
        mk(vRSQ[k], (size_t)pnz * cnux, pRSQ, k);
        mk(vrq[k], pnz, prq, k);
        double* M = pRSQ[k];
        if (k < N) {
            pack(R[k], nuk, nuk, nuk, false, M, cnux, 0);
            pack(S[k], nuk, nxk, nuk, true, M, cnux, nuk);  // S' below R
        }
        for (int j = 0; j < nxk; j++)  // Q at (nu, nu)
            for (int i = 0; i < nxk; i++) P4(M, cnux, nuk + i, nuk + j) = Q[k][i + j * nxk];
        for (int j = 0; j < nuk; j++) P4(M, cnux, nux, j) = prq[k][j] = r[k][j];
        for (int j = 0; j < nxk; j++) P4(M, cnux, nux, nuk + j) = prq[k][nuk + j] = q[k][j];
        mk(vZ[k], 2 * pns[k], pZ, k);
        mk(vz[k], 2 * pns[k], pz, k);  // never filled by the reference wrapper (see above)
        for (int j = 0; j < ns[k]; j++) {
            pZ[k][j] = Z[k][j];
            pZ[k][pns[k] + j] = Z[k][ns[k] + j];
        }
        mk(vd[k], nd, pd, k);
        for (int j = 0; j < nb[k]; j++) {
            pd[k][j] = lb[k][j];
            pd[k][pnb[k] + j] = ub[k][j];
        }
        for (int j = 0; j < ns[k]; j++) {
            pd[k][2 * pnb[k] + 2 * png[k] + j] = lb[k][nb[k] + j];
            pd[k][2 * pnb[k] + 2 * png[k] + pns[k] + j] = ub[k][nb[k] + j];
        }
        for (int j = 0; j < ng[k]; j++) {
            pd[k][2 * pnb[k] + j] = lg[k][j];
            pd[k][2 * pnb[k] + png[k] + j] = ug[k][j];
        }
        mk(vux[k], pnz, pux, k);
        mk(vlam[k], ncv, plam, k);
        mk(vt[k], ncv, pt, k);
        mk(vrrq[k], pnz, prrq, k);
        mk(vrd[k], nd, prd, k);
        mk(vrz[k], 2 * pns[k], prz, k);
        if (warm_start) {
            for (int j = 0; j < nuk; j++) pux[k][j] = u[k][j];
            for (int j = 0; j < nxk; j++) pux[k][nuk + j] = x[k][j];
        }
    }
    if (mu0 <= 0) {  // :1723-1740 (no absolute value)
        for (int k = 0; k <= N; k++) {
            const int nuk = nu[k], nxk = nx[k];
            if (k < N) {
                for (int i = 0; i < nuk * nuk; i++) mu0 = fmax(mu0, R[k][i]);
                for (int i = 0; i < nxk * nuk; i++) mu0 = fmax(mu0, S[k][i]);
                for (int i = 0; i < nuk; i++) mu0 = fmax(mu0, r[k][i]);
            }
            for (int i = 0; i < nxk * nxk; i++) mu0 = fmax(mu0, Q[k][i]);
            for (int i = 0; i < nxk; i++) mu0 = fmax(mu0, q[k][i]);
            for (int i = 0; i < 2 * ns[k]; i++) mu0 = fmax(mu0, Z[k][i]);
            for (int i = 0; i < 2 * ns[k]; i++) mu0 = fmax(mu0, z[k][i]);
        }
    }
    std::vector<double> work(8);
    const int status = d_ip2_mpc_soft_tv(kk, k_max, mu0, mu_tol, 1e-8, warm_start, stat, N, nx, nu.data(), nb, hidxb,
                                         ng, ns, pBAbt.data(), pRSQ.data(), pZ.data(), pz.data(), pDCt.data(),
                                         pd.data(), pux.data(), 1, ppi.data(), plam.data(), pt.data(), work.data());
    if (hpmpc_mi355x_last_error() != 0) return status;
    for (int k = 0; k < N; k++)
        for (int j = 0; j < nu[k]; j++) u[k][j] = pux[k][j];
    for (int k = 0; k <= N; k++)
        for (int j = 0; j < nx[k]; j++) x[k][j] = pux[k][nu[k] + j];
    double mu = 0.0;
    d_res_mpc_soft_tv(N, nx, nu.data(), nb, hidxb, ng, ns, pBAbt.data(), pRSQ.data(), prq.data(), pZ.data(), pz.data(),
                      pux.data(), pDCt.data(), pd.data(), ppi.data(), plam.data(), pt.data(), prrq.data(), prb.data(),
                      prd.data(), prz.data(), &mu);
    if (hpmpc_mi355x_last_error() != 0) return status;
    double tq = fabs(prrq[0][0]);
    for (int k = 0; k < N; k++)
        for (int j = 0; j < nu[k] + nx[k]; j++) tq = fmax(tq, fabs(prrq[k][j]));
    for (int j = 0; j < nx[N]; j++) tq = fmax(tq, fabs(prrq[N][j]));
    double tb = N > 0 ? fabs(prb[0][0]) : 0.0;
    for (int k = 0; k < N; k++)
        for (int j = 0; j < nx[k + 1]; j++) tb = fmax(tb, fabs(prb[k][j]));
    double td = fabs(prd[0][0]);
    for (int k = 0; k <= N; k++) {
        const int os = 2 * pnb[k] + 2 * png[k];
        for (int j = 0; j < nb[k]; j++) td = fmax(td, fmax(fabs(prd[k][j]), fabs(prd[k][pnb[k] + j])));
        for (int j = 0; j < ng[k]; j++)
            td = fmax(td, fmax(fabs(prd[k][2 * pnb[k] + j]), fabs(prd[k][2 * pnb[k] + png[k] + j])));
        for (int j = 0; j < ns[k]; j++) td = fmax(td, fmax(fabs(prd[k][os + j]), fabs(prd[k][os + pns[k] + j])));
    }
    inf_norm_res[0] = tq;
    inf_norm_res[1] = tb;
    inf_norm_res[2] = td;
    inf_norm_res[3] = mu;
    for (int k = 0; k < N; k++)
        for (int j = 0; j < nx[k + 1]; j++) pi[k][j] = ppi[k][j];
    for (int k = 0; k <= N; k++) {  // compact lam: [lo nb | up nb | lg ng | ug ng | 4 soft blocks of ns]
        const int os = 2 * pnb[k] + 2 * png[k];
        for (int j = 0; j < nb[k]; j++) {
            lam[k][j] = plam[k][j];
            lam[k][nb[k] + j] = plam[k][pnb[k] + j];
        }
        for (int j = 0; j < ng[k]; j++) {
            lam[k][2 * nb[k] + j] = plam[k][2 * pnb[k] + j];
            lam[k][2 * nb[k] + ng[k] + j] = plam[k][2 * pnb[k] + png[k] + j];
        }
        for (int s = 0; s < 4; s++)
            for (int j = 0; j < ns[k]; j++) lam[k][2 * nb[k] + 2 * ng[k] + s * ns[k] + j] = plam[k][os + s * pns[k] + j];
    }
    return status;
}
