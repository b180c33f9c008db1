#!/usr/bin/env python3
"""Benchmark of the MI355X Riccati / interior-point hot path (BASELINE.json metric).

Workload (BASELINE.json configs[1] shape at the metric's batch): 1024 box-constrained mass-spring
MPC QPs per GPU, N=100, nx=12, nu=4 (nb = 4 / 10 / 6 on stage 0 / inner / N), fp64, time-variant
stage data (no aliased buffers), solved by the residual-based Mehrotra IPM
(d_ip2_res_mpc_hard_tv: mu0=2, mu_tol=1e-12, alpha_min=1e-8, k_max=50).

A "step" is one batch of 1024 problems (default K = 20 steps, the driver's count; the same line reports K = 40 in
"k40").  The K timed steps are solved through one problem queue (hpmpc_mi355x_ipm_queue): 8 x 1024 resident solver
slots in four lanes of 2048 on four streams, each slot taking the next problem (one shared counter) as soon as its
own has converged (iterations are ticks of the pass kernels hk_ipm_fact, hk_ipm_pred, hk_ipm_corr, hk_ipm_update over
a lane's slots; once the queue is empty and few slots still iterate, they finish on the multi-wave kernel
hk_ipm_qdrain_mw).  value = IP iterations per second over all ranks (sum of per-problem iteration counts /
max-over-ranks time).  The lanes run the four passes concurrently, so the roofline's unit of work is one step (all
four passes' algorithmic bytes over the step's IP iterations, over the step's wall time); the dominant pass's
per-launch figures (hipEvents at every kernel boundary inside the timed region) and `per_pass` are kept beside it.
An isolated single-batch solve is reported beside it.
The Riccati factorisation rate (d_back_ric_rec_sv_tv_res, nb = 0, compute_pi = 1) of the same
batch is reported in the same JSON line, and so is configs[4] ("pcond": 512 x N=200 nx=24 nu=6 condensed into
20 blocks, the condensed Riccati and the expansion, with its own roofline and CPU baseline).

Multi-GPU: one process per GPU (torch.distributed.run); every rank generates its own shard of
problems from the global problem seeds (no data-path collective: weak scaling); RCCL is used only
for the barrier and the max-time / sum-of-iterations reductions.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

PEAK_HBM_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8 TB/s spec
BASELINE_METRIC = "Riccati factorisations/sec + IP iters/sec, fp64, N=100 nx=12 nu=4 batch=1024"  # BASELINE.json
PEAK_FP64_TFS = 78.6   # MI355X fp64 (vector = MFMA dense)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    # 20 batches, the driver's count; the line also reports 40 batches ("k40": the queue's drain -- the last
    # problems, ~9 % of which run to k_max or alpha_min -- is a fixed cost per run)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--batch", type=int, default=1024, help="problems per GPU")
    ap.add_argument("--N", type=int, default=100)
    ap.add_argument("--nx", type=int, default=12)
    ap.add_argument("--nu", type=int, default=4)
    ap.add_argument("--k-max", type=int, default=50)
    ap.add_argument("--slots", type=int, default=0, help="resident solver slots (default max(8 x batch, 8192): "
                    "two problems per SIMD resident, the rest dispatched as they finish; tools/slots_probe.py)")
    ap.add_argument("--no-k40", action="store_true", help="skip the 40-batch queue run reported beside the headline")
    ap.add_argument("--sv-streams", type=int, default=2, help="Riccati legs: batches in flight (one stream and one set "
                    "of output buffers each; tools/sv_streams_probe.py: 2 best, 1.48x / 1.41x over one at N=100 / 50)")
    ap.add_argument("--cpu-seconds", type=float, default=15.0)
    ap.add_argument("--cpu-threads", type=int, default=16, help="host threads for the CPU baseline "
                    "(the GPU box's CPU share is 16 per GPU)")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-pcond", action="store_true", help="skip the configs[4] partial-condensing leg")
    ap.add_argument("--pcond-batch", type=int, default=512)
    ap.add_argument("--no-isolated", action="store_true", help="skip the isolated single-batch solve (profiling "
                    "runs: then every hk_ipm_* launch of the command belongs to the timed queue)")
    ap.add_argument("--global-batch", type=int, default=0, help="fixed total problems split over the ranks "
                    "(strong scaling, e.g. configs[3]: 4096 over 8 GPUs = 512 per GPU); default: --batch per GPU "
                    "(weak scaling)")
    ap.add_argument("--no-scatter", action="store_true", help="skip the rank-0 scatter / gather leg (N > 1)")
    ap.add_argument("--no-queue-batch-slots", action="store_true", help="skip the queue run with one slot per "
                    "problem of the batch")
    ap.add_argument("--no-aliased", action="store_true", help="skip the time-invariant / aliased leg")
    ap.add_argument("--no-coupled", action="store_true", help="skip the coupled-Hessian IPM leg")
    ap.add_argument("--check-launch", action="store_true", help="start the ranks, join the process group (gloo) "
                    "and print each rank's world size, without touching the GPU (launcher test)")
    return ap.parse_args()


def launch_ranks(args):
    """--gpus N > 1 outside a torch.distributed launcher: run this script under torch.distributed.run with N
    ranks as a child process (nothing here has touched the GPU) and exit with its code."""
    import socket
    import subprocess

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr", "127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + sys.argv[1:]
    sys.exit(subprocess.call(cmd))


def host_cpu():
    """Host CPU model and logical CPU count (the lscpu facts SURVEY.md §8d asks for beside the baseline)."""
    model = None
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    return {"model": model, "nproc": os.cpu_count(),
            "affinity": len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else None}


def physical_cores():
    """Physical cores of the host (distinct (package, core) pairs in /proc/cpuinfo), or None."""
    ids, pkg = set(), None
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("physical id"):
                    pkg = line.split(":", 1)[1].strip()
                elif line.startswith("core id"):
                    ids.add((pkg, line.split(":", 1)[1].strip()))
    except OSError:
        return None
    return len(ids) or None


def ref_api():
    """The reference c99 build (oracle/_ref/libhpmpc_ref.so) for the parity samples, or None when absent."""
    from hpmpc_amd.cabi import HpmpcAPI, load

    path = os.path.join(ROOT, "oracle", "_ref", "libhpmpc_ref.so")
    return HpmpcAPI(load(path)) if os.path.exists(path) else None


def rel_err(a, b):
    a, b = np.asarray(a, dtype=np.float64), np.asarray(b, dtype=np.float64)
    return float(np.max(np.abs(a - b) / np.maximum(1.0, np.abs(b)), initial=0.0))


def parity_ipm(ref, qp, sol, idx):
    """SURVEY.md §5 'max parity error' of timed IPM solves: problems `idx` (pairs of (entry in sol, problem of qp))
    re-solved by the reference c99 build after the timed region; max relative error of ux / pi / lam / t over the
    valid entries, kk / ret equality.  A problem the reference itself stops on alpha_min with |lam| > 1e12 (an
    infeasible draw, where last bits grow without bound) contributes only kk / ret."""
    if ref is None:
        return None
    rows_t = sol["ux"].new_tensor([q for q, _ in idx], dtype=sol["kk"].dtype).long()
    ux, pi, lam, t, kk, ret = (sol[n][rows_t].cpu().numpy() for n in ("ux", "pi", "lam", "t", "kk", "ret"))
    idx = [(i, p) for i, (_, p) in enumerate(idx)]
    e, same, div, rows = 0.0, 0, 0, []
    for q, p in idx:
        one = qp.problem(int(p))
        r = ref.ipm(one.copy(), k_max=int(sol["k_max"]))
        ok = int(kk[q]) == r["kk"] and int(ret[q]) == r["ret"]
        same += ok
        if r["ret"] == 2 and max(float(np.max(np.abs(x))) for x in r["lam"]) > 1e12:
            div += 1
            rows.append({"problem": int(p), "kk": int(kk[q]), "ret": int(ret[q]), "divergent": True})
            continue
        ep = 0.0
        for k in range(qp.N + 1):
            ep = max(ep, rel_err(ux[q, k, :qp.nux(k)], r["ux"][k][:qp.nux(k)]))
            if k < qp.N:
                ep = max(ep, rel_err(pi[q, k, :int(qp.nx[k + 1])], r["pi"][k][:int(qp.nx[k + 1])]))
            nb, pnb = int(qp.nb[k]), qp.pnb(k)
            ib = np.r_[0:nb, pnb:pnb + nb].astype(int)
            ep = max(ep, rel_err(lam[q, k, ib], r["lam"][k][ib]), rel_err(t[q, k, ib], r["t"][k][ib]))
        e = max(e, ep)
        rows.append({"problem": int(p), "kk": int(kk[q]), "ret": int(ret[q]), "max_rel_err": ep})
    return {"reference": "oracle/_ref c99 build, d_ip2_res_mpc_hard_tv", "problems": len(idx), "max_rel_err": e,
            "kk_ret_equal": same, "divergent_kk_ret_only": div, "per_problem": rows}


def parity_sv(ref, qp, ux_t, pi_t, problems, compute_pi=1):
    """The same for timed Riccati solves (d_back_ric_rec_sv_tv_res): ux and pi of `problems` against the reference."""
    if ref is None:
        return None
    sel = ux_t.new_tensor(list(problems)).long()
    ux, pi = ux_t[sel].cpu().numpy(), pi_t[sel].cpu().numpy()
    e = 0.0
    for i, p in enumerate(problems):
        u2, p2, _, _ = ref.ric_sv(qp.problem(int(p)), compute_pi=compute_pi, compute_Pb=0)
        for k in range(qp.N + 1):
            e = max(e, rel_err(ux[i, k, :qp.nux(k)], u2[k][:qp.nux(k)]))
            if k < qp.N and compute_pi:
                e = max(e, rel_err(pi[i, k, :int(qp.nx[k + 1])], p2[k][:int(qp.nx[k + 1])]))
    return {"reference": "oracle/_ref c99 build, d_back_ric_rec_sv_tv_res", "problems": [int(p) for p in problems],
            "max_rel_err": e}


def spread(n, total):
    """n indices spread over [0, total)."""
    return sorted({int(round(x)) for x in np.linspace(0, total - 1, n)})


def cpu_baseline(qp, seconds, k_max, threads):
    """IP iterations/s of the reference c99 build (oracle/_ref, kind 'reference') -- or of the
    clean-room oracle (kind 'port') when the reference build is absent -- on the GPU box's host cores,
    over the first problems of this rank's batch.  Calls are pre-marshalled; each thread cycles over
    its own problems until the time budget ends.  Reported for `threads` threads and for 1 thread."""
    import threading

    from hpmpc_amd.cabi import HpmpcAPI, load

    ref = os.path.join(ROOT, "oracle", "_ref", "libhpmpc_ref.so")
    orc = os.path.join(ROOT, "oracle", "liboracle.so")
    if os.path.exists(ref):
        api, kind = HpmpcAPI(load(ref)), "reference"
    elif os.path.exists(orc):
        api, kind = HpmpcAPI(load(orc), "orc_"), "port"
    else:
        return None
    nprob = min(qp.batch, max(64, threads * 4))
    calls = [api.prepare_ipm(qp.problem(p), k_max=k_max) for p in range(nprob)]

    def run(nthr, secs):
        counts = [0] * nthr
        solves = [0] * nthr
        stop = time.perf_counter() + secs

        def worker(i):
            mine = calls[i::nthr]
            j = 0
            while time.perf_counter() < stop:
                call, kk = mine[j % len(mine)]
                call()
                counts[i] += kk.value
                solves[i] += 1
                j += 1

        th = [threading.Thread(target=worker, args=(i,)) for i in range(nthr)]
        t0 = time.perf_counter()
        for t in th:
            t.start()
        for t in th:
            t.join()
        el = time.perf_counter() - t0
        return sum(counts) / el, sum(counts), sum(solves), el

    v1, it1, s1, e1 = run(1, seconds * 0.3)
    vn, itn, sn, en = run(threads, seconds * 0.7)
    host = host_cpu()
    phys = physical_cores()
    host["physical_cores"] = phys
    out = {"value": vn, "unit": "IP-iter/s", "cores": threads, "kind": kind, "host": host,
           "sample": f"first {nprob} problems of the benchmark batch, cold-start d_ip2_res_mpc_hard_tv "
                     f"(k_max={k_max}) cycled by {threads} host threads for {en:.1f} s ({sn} solves, {itn} IP "
                     f"iterations); pre-marshalled ctypes calls",
           "single_core": {"value": v1, "solves": s1, "iters": it1, "seconds": e1}}
    if phys and phys > threads:
        # the GPU box is one GPU's share of a shared host (16 CPUs per GPU): the run stays inside that share, and
        # the all-core figure is the measured per-thread rate at `threads` threads times the physical cores (the
        # per-thread rate is flat from 1 to `threads` threads: single_core vs value / threads)
        out["all_cores_estimate"] = {"cores": phys, "value": vn / threads * phys, "unit": "IP-iter/s",
                                     "basis": f"measured {vn / threads:.0f} IP-iter/s per thread at {threads} threads "
                                              f"(1 thread: {v1:.0f}) x {phys} physical cores; not measured"}
    return out


def cpu_pcond_baseline(qp, N2, seconds, threads):
    """Pipelines/s of the reference c99 build (oracle/_ref: d_part_cond + d_back_ric_rec_sv_tv_res on the
    condensed problem + d_part_expand_solution), or of the oracle (kind 'port') without it, on the host cores:
    a bounded sample of this rank's configs[4] batch, `threads` host threads and 1 thread."""
    import threading

    from hpmpc_amd.cabi import HpmpcAPI, load

    ref = os.path.join(ROOT, "oracle", "_ref", "libhpmpc_ref.so")
    orc = os.path.join(ROOT, "oracle", "liboracle.so")
    if os.path.exists(ref):
        api, kind = HpmpcAPI(load(ref)), "reference"
    elif os.path.exists(orc):
        api, kind = HpmpcAPI(load(orc), "orc_"), "port"
    else:
        return None
    calls = [api.prepare_pcond(qp.problem(p), N2) for p in range(min(qp.batch, 2 * threads))]

    def run(nthr, secs):
        done = [0] * nthr
        stop = time.perf_counter() + secs

        def worker(i):
            j = 0
            while time.perf_counter() < stop:
                calls[(i + nthr * j) % len(calls)]()
                done[i] += 1
                j += 1

        th = [threading.Thread(target=worker, args=(i,)) for i in range(nthr)]
        t0 = time.perf_counter()
        for t in th:
            t.start()
        for t in th:
            t.join()
        return sum(done) / (time.perf_counter() - t0), sum(done)

    v1, n1 = run(1, seconds * 0.3)
    vn, nn = run(threads, seconds * 0.7)
    return {"value": vn, "unit": "solves/s", "cores": threads, "kind": kind, "host": host_cpu(),
            "sample": f"{len(calls)} problems of the configs[4] batch, d_part_cond + condensed "
                      f"d_back_ric_rec_sv_tv_res + d_part_expand_solution, pre-marshalled ctypes calls, {threads} host threads "
                      f"({nn} pipelines) and 1 thread ({n1}); the reference c99 condensing is numerically wrong "
                      f"for nu > 4 (DESIGN.md) but does the same work",
            "single_core": {"value": v1, "solves": n1}}


def pcond_traffic(kernel, B):
    """Calibrated HBM bytes per launch of a configs[4] kernel (profiles/pmc_hk_ipm.json, tools/pmc_mix.sh: the
    same pipeline at batch 512 under rocprofv3 FETCH_SIZE / WRITE_SIZE passes), scaled to this run's batch."""
    pmc = os.path.join(ROOT, "profiles", "pmc_hk_ipm.json")
    try:
        with open(pmc) as f:
            k = json.load(f)["kernels"][kernel]
        return k["hbm_bytes_per_launch"] * B / 512.0
    except Exception:
        return None


def bench_pcond(args, torch, red, rank, world, barrier):
    """configs[4]: 512 problems per GPU, N=200 nx=24 nu=6 condensed into N2=20 blocks of 10, then the
    condensed Riccati factorisation + solve and the expansion (d_part_cond -> d_back_ric_rec_sv_tv_res ->
    d_part_expand_solution).  A step is the whole pipeline over the batch; per-kernel hipEvents on the solve
    stream give the roofline of the dominant kernel."""
    from hpmpc_amd.pcond import PcondSolver, pcond_algorithmic_bytes, pcond_flops
    from hpmpc_amd.shard import make_shard

    B, N, nx, nu, N2 = args.pcond_batch, 200, 24, 6, 20
    qp = make_shard(N, nx, nu, rank, world, B, boxes=False)
    s = PcondSolver(qp, N2)
    for _ in range(max(args.warmup, 1)):
        s.solve()
    stream = torch.cuda.current_stream()
    K = args.steps
    ev = [[torch.cuda.Event(enable_timing=True) for _ in range(4)] for _ in range(K)]
    barrier()
    t0 = time.perf_counter()
    for i in range(K):
        ev[i][0].record(stream)
        s.condense()
        ev[i][1].record(stream)
        s.riccati()
        ev[i][2].record(stream)
        s.expand()
        ev[i][3].record(stream)
    barrier()
    dt = red.max(time.perf_counter() - t0)
    ms = np.array([[e[j].elapsed_time(e[j + 1]) for j in range(3)] for e in ev]).mean(axis=0)
    # the same K pipelines with args.sv_streams batches in flight (own solver buffers per stream): the condensing of
    # one batch overlaps the condensed Riccati of the other, whose one workgroup per problem leaves CUs idle
    # (tools/pcond_streams_probe.py: +10 %); the per-kernel roofline below is the one-stream run's
    sols = [s] + [PcondSolver(qp, N2) for _ in range(max(args.sv_streams, 1) - 1)]
    streams = [stream] + side_streams(torch, len(sols) - 1)
    for x, st in zip(sols[1:], streams[1:]):  # untimed: each stream's first use pays its queue's set-up
        st.wait_stream(stream)
        with torch.cuda.stream(st):
            x.solve()
    torch.cuda.synchronize()
    barrier()
    t0 = time.perf_counter()
    for i in range(K):
        j = i % len(sols)
        with torch.cuda.stream(streams[j]):
            sols[j].solve()
    for st in streams[1:]:
        stream.wait_stream(st)
    barrier()
    dt_f = red.max(time.perf_counter() - t0)
    names = ["hk_pcond", "hk_wide_sv", "hk_pexpand"]
    by = pcond_algorithmic_bytes(qp, N2)
    fl = pcond_flops(qp, N2)
    dom = int(np.argmax(ms))
    ach = B * by[dom] / (ms[dom] * 1e-3) / 1e9
    kern = {n: {"ms": float(m), "algorithmic_bytes_per_problem": b, "flops_per_problem": f,
                "achieved_GBps": B * b / (m * 1e-3) / 1e9, "fp64_tflops": B * f / (m * 1e-3) / 1e12}
            for n, m, b, f in zip(names, ms, by, fl)}
    out = {"workload": f"pcond_N{N}_nx{nx}_nu{nu}_N2_{N2}_batch{B}", "value": B * world * K / dt_f,
           "unit": "solves/s", "ms_per_step": dt_f / K * 1e3, "batch_per_gpu": B, "batches_in_flight": len(sols),
           "one_batch_in_flight": {"value": B * world * K / dt, "ms_per_step": dt / K * 1e3,
                                   "note": "the run the per-kernel roofline and 'kernels' are measured on"},
           "condensed": {"N2": N2, "nu2": 60, "nx2": 24},
           "riccati_fact_per_s": B * world / (ms[1] * 1e-3),
           "roofline": {"bound": "hbm", "kernel": names[dom], "achieved": ach, "peak": PEAK_HBM_GBS, "unit": "GB/s",
                        "frac": ach / PEAK_HBM_GBS, "traffic": pcond_traffic(names[dom], B),
                        "launch_ms": float(ms[dom])},
           "kernels": kern}
    for n in names:
        kern[n]["traffic_bytes_per_launch"] = pcond_traffic(n, B)
    ref = ref_api() if rank == 0 else None
    if ref is not None:
        # the reference's own condensing is wrong for nu > 4: the expanded solution is held to its direct
        # Riccati solve of the uncondensed problem
        torch.cuda.synchronize()
        e = 0.0
        for p in spread(8, B):
            u2, p2, _, _ = ref.ric_sv(qp.problem(p), compute_pi=1, compute_Pb=0)
            for x in sols:  # every stream's buffers
                U, Pi = x.solution(p)
                for k in range(N + 1):
                    e = max(e, rel_err(U[k], u2[k][:qp.nux(k)]))
                    if k < N:
                        e = max(e, rel_err(Pi[k], p2[k][:int(qp.nx[k + 1])]))
        out["parity"] = {"reference": "oracle/_ref c99 d_back_ric_rec_sv_tv_res on the uncondensed problem",
                         "problems": spread(8, B), "max_rel_err": e}
    if rank == 0 and world == 1 and not args.no_cpu:
        out["cpu_baseline"] = cpu_pcond_baseline(qp, N2, args.cpu_seconds * 0.5, args.cpu_threads)
    out["ipm"] = bench_pcond_ipm(args, torch, red, rank, world, barrier)
    return out


def bench_pcond_ipm(args, torch, red, rank, world, barrier):
    """configs[4] with box constraints: d_part_cond (inner state boxes become the condensed problem's general
    constraints, ng2 = 108 per block) -> d_ip2_res_mpc_hard_tv on the condensed N2=20 system (nu2=60 nx2=24,
    the batched wide-stage IPM: one 256-thread workgroup per problem, one launch) -> d_part_expand_solution, on
    the same 512-problem batch shape.  value = IP iterations per second of the condensed IPMs."""
    from hpmpc_amd.pcond import PcondSolver
    from hpmpc_amd.shard import make_shard

    from hpmpc_amd.pcond import wide_ipm_algorithmic_bytes

    B, N, nx, nu, N2 = args.pcond_batch, 200, 24, 6, 20
    k_max = 50
    # x0 ~ U(-0.5, 0.5) (0.2 x the other legs' draw): over N = 200 stages most U(-2.5, 2.5) draws are box-infeasible
    # (measured: 70 % of the batch diverge or hit k_max at scale 1, none at 0.2), and iterations of diverging
    # problems would dominate the rate
    x0_scale = 0.2
    qp = make_shard(N, nx, nu, rank, world, B, boxes=True, x0_scale=x0_scale)
    s = PcondSolver(qp, N2)
    s.solve_ipm(k_max=k_max)  # warmup (plans, workspaces)
    stream = torch.cuda.current_stream()
    K = max(1, min(args.steps, 3))
    ev = [[torch.cuda.Event(enable_timing=True) for _ in range(4)] for _ in range(K)]
    iters = 0.0
    barrier()
    t0 = time.perf_counter()
    for i in range(K):
        ev[i][0].record(stream)
        s.condense()
        ev[i][1].record(stream)
        s.ipm(k_max=k_max)
        ev[i][2].record(stream)
        s.expand()
        ev[i][3].record(stream)
    barrier()
    dt = red.max(time.perf_counter() - t0)
    kk = s.kk2.cpu().numpy()
    ret = s.ret2.cpu().numpy()
    iters = red.sum(float(kk.sum()) * K)
    ms = np.array([[e[j].elapsed_time(e[j + 1]) for j in range(3)] for e in ev]).mean(axis=0)
    # the same K pipelines with args.sv_streams batches in flight (own solver buffers per stream): one workgroup per
    # problem and 512 problems leave room on the chip for a second batch (tools/pcond_streams_probe.py: +10 %); the
    # roofline below is the one-stream run's
    sols = [s] + [PcondSolver(qp, N2) for _ in range(max(args.sv_streams, 1) - 1)]
    streams = [stream] + side_streams(torch, len(sols) - 1)
    for x, st in zip(sols[1:], streams[1:]):  # untimed: each stream's first use pays its queue's set-up
        st.wait_stream(stream)
        with torch.cuda.stream(st):
            x.solve_ipm(k_max=k_max)
    torch.cuda.synchronize()
    barrier()
    t0 = time.perf_counter()
    for i in range(K * len(sols)):
        j = i % len(sols)
        with torch.cuda.stream(streams[j]):
            sols[j].solve_ipm(k_max=k_max)
    for st in streams[1:]:
        stream.wait_stream(st)
    barrier()
    dt_f = red.max(time.perf_counter() - t0)
    iters_f = red.sum(sum(float(x.kk2.sum().item()) for x in sols) * K)
    # roofline of the wide-stage IPM (one launch solves the batch): algorithmic bytes of one condensed IP
    # iteration (pcond.wide_ipm_algorithmic_bytes) x the launch's iterations / its duration
    c = s.cond_sizes()
    bpi = wide_ipm_algorithmic_bytes(c["nx"], c["nu"], c["nb"], c["ng"])
    ach = float(kk.sum()) * bpi / (ms[1] * 1e-3) / 1e9
    out = {"workload": f"pcond_ipm_N{N}_nx{nx}_nu{nu}_N2_{N2}_boxes_batch{B}", "value": iters_f / dt_f,
           "unit": "IP-iter/s", "x0_scale": x0_scale, "batches_in_flight": len(sols),
           "one_batch_in_flight": {"value": iters / dt, "solves_per_s": B * world * K / dt,
                                   "note": "the run the roofline, 'ms' and 'solves_per_s' are measured on"},
           "roofline": {"bound": "hbm", "kernel": "hk_wide_ipm", "achieved": ach, "peak": PEAK_HBM_GBS, "unit": "GB/s",
                        "frac": ach / PEAK_HBM_GBS, "bytes_per_ip_iter": bpi, "launch_ms": float(ms[1]),
                        "ip_iters_per_launch": float(kk.sum())},
           "solves_per_s": B * world * K / dt, "ms_per_step": dt / K * 1e3, "steps": K,
           "k_max": k_max, "condensed": {"N2": N2, "nu2": nu * (N // N2), "nx2": nx,
                                         "ng2": int(sum(int(qp.nb[k]) - nu for k in range(1, N // N2)))},
           "ms": {"hk_pcond": float(ms[0]), "hk_wide_ipm": float(ms[1]), "hk_pexpand": float(ms[2])},
           "sum_kk_per_step": float(kk.sum()),
           "ret_counts": {str(int(v)): int((ret == v).sum()) for v in np.unique(ret)}}
    if rank == 0 and world == 1 and not args.no_cpu:
        out["cpu_baseline"] = cpu_pcond_ipm_baseline(qp, N2, k_max, args.cpu_seconds * 0.5, args.cpu_threads)
    return out


def cpu_pcond_ipm_baseline(qp, N2, k_max, seconds, threads):
    """IP iterations/s of the configs[4] IPM pipeline on the host cores: d_part_cond -> d_ip2_res_mpc_hard_tv on the
    condensed problem -> d_part_expand_solution from the reference's c99 build (oracle/_ref, kind 'reference': its
    condensing is numerically wrong for nu > 4, DESIGN.md §3b, so its IPM solves a slightly different condensed problem
    -- the same work per iteration), or the oracle (kind 'port') without it; `threads` host threads over a bounded
    sample of the batch, and one thread."""
    import threading

    from hpmpc_amd.cabi import HpmpcAPI, load

    ref = os.path.join(ROOT, "oracle", "_ref", "libhpmpc_ref.so")
    orc = os.path.join(ROOT, "oracle", "liboracle.so")
    if os.path.exists(ref):
        api, kind = HpmpcAPI(load(ref)), "reference"
    elif os.path.exists(orc):
        api, kind = HpmpcAPI(load(orc), "orc_"), "port"
    else:
        return None
    calls = [api.prepare_pcond_ipm(qp.problem(p), N2, k_max=k_max) for p in range(min(qp.batch, 2 * threads))]

    def run(nthr, secs):
        done, iters = [0] * nthr, [0] * nthr
        stop = time.perf_counter() + secs

        def worker(i):
            j = 0
            while time.perf_counter() < stop:
                call, kk = calls[(i + nthr * j) % len(calls)]
                call()
                iters[i] += kk.value
                done[i] += 1
                j += 1

        th = [threading.Thread(target=worker, args=(i,)) for i in range(nthr)]
        t0 = time.perf_counter()
        for t in th:
            t.start()
        for t in th:
            t.join()
        dt = time.perf_counter() - t0
        return sum(iters) / dt, sum(done), sum(iters)

    v1, n1, i1 = run(1, seconds * 0.3)
    vn, nn, itn = run(threads, seconds * 0.7)
    return {"value": vn, "unit": "IP-iter/s", "cores": threads, "kind": kind, "host": host_cpu(),
            "sample": f"{len(calls)} problems of the configs[4] batch with boxes, d_part_cond + condensed "
                      f"d_ip2_res_mpc_hard_tv (k_max={k_max}) + d_part_expand_solution, pre-marshalled ctypes calls, "
                      f"{threads} host threads ({nn} pipelines, {itn} IP iterations) and 1 thread ({n1}, {i1})",
            "single_core": {"value": v1, "solves": n1, "iters": i1}}


def bench_single_qp(args, torch, stream):
    """configs[1]: one QP (the drivers' x0, test_d_ip_hard.c:306-322) solved alone on the GPU: the device time of
    the latency path (hpmpc_mi355x_ipm_solo, data resident in HBM; the kernel the drop-in runs), of a one-entry
    problem queue, of the batched API with a batch of one, and the drop-in d_ip2_res_mpc_hard_tv call on host lib4
    buffers (PCIe staging included).  Latency-bound: the stages are walked serially; the solo kernel gives one problem
    a 256-thread workgroup (hk_ipm_solo_mw: wave 0 runs the recursion, waves 1..3 everything off it), and the line also
    reports the single-wave solo kernel (HPMPC_MI355X_SOLO=1) beside it."""
    from hpmpc_amd.batch import LIBPATH, BatchSolver
    from hpmpc_amd.cabi import HpmpcAPI, load
    from hpmpc_amd.ocp import mass_spring_qp

    one = mass_spring_qp(args.N, args.nx, args.nu, batch=1)
    s = BatchSolver(one, k_max=args.k_max)
    reps = max(min(args.steps, 20), 5)
    # the latency path (hpmpc_mi355x_ipm_solo, what the drop-in calls): the whole solve in one launch; beside it a
    # queue of one entry in one slot (pass kernels, chunks of 8 iterations) and the batched solve
    # (hpmpc_mi355x_ipm_batch: k_max x 4 pass launches)
    Q = s.queue(1, 1)
    for _ in range(2):
        Q.run()
        s.ipm()
        s.ipm_solo()

    def timed(fn):
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(reps)]
        for a, b in ev:
            a.record(stream)
            fn()
            b.record(stream)
        torch.cuda.synchronize()
        return float(np.median([a.elapsed_time(b) for a, b in ev]))

    ms = timed(s.ipm_solo)
    kk = int(s.kk[0].item())
    os.environ["HPMPC_MI355X_SOLO"] = "1"  # read at each launch: the single-wave solo kernel
    try:
        s.ipm_solo()
        ms_single = timed(s.ipm_solo)
        assert int(s.kk[0].item()) == kk
    finally:
        os.environ.pop("HPMPC_MI355X_SOLO", None)
    ms_queue = timed(Q.run)
    assert int(Q.kk[0].item()) == kk
    evb = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(reps)]
    for a, b in evb:
        a.record(stream)
        s.ipm()
        b.record(stream)
    torch.cuda.synchronize()
    ms_batch = float(np.median([a.elapsed_time(b) for a, b in evb]))
    assert int(s.kk[0].item()) == kk
    s.ipm_solo()
    torch.cuda.synchronize()
    par = parity_ipm(ref_api(), one, dict(ux=s.ux, pi=s.pi, lam=s.lam, t=s.t, kk=s.kk, ret=s.ret, k_max=args.k_max),
                     [(0, 0)])
    call, kkc = HpmpcAPI(load(LIBPATH)).prepare_ipm(one.problem(0), k_max=args.k_max)
    call()
    t0 = time.perf_counter()
    for _ in range(reps):
        call()
    host_ms = (time.perf_counter() - t0) / reps * 1e3
    return {"workload": f"single_qp_N{args.N}_nx{args.nx}_nu{args.nu}", "kk": kk, "device_ms_per_solve": ms,
            "device_us_per_ip_iter": ms * 1e3 / max(kk, 1),
            "path": "hpmpc_mi355x_ipm_solo (one launch per solve, one problem per 4-wave workgroup: hk_ipm_solo_mw)",
            "single_wave_ms_per_solve": ms_single, "single_wave_us_per_ip_iter": ms_single * 1e3 / max(kk, 1),
            "queue1_ms_per_solve": ms_queue, "batch_api_ms_per_solve": ms_batch,
            "dropin_ms_per_solve": host_ms, "dropin_kk": int(kkc.value), "parity": par}


_SIDE = []


def side_streams(torch, n):
    """The streams the legs with several batches in flight use beside the current one, created once and shared by
    every such leg: the process has four hardware queues (GPU_MAX_HW_QUEUES), the queue's lanes hold three of them,
    and a stream created later can land on the current stream's queue and serialise behind it."""
    while len(_SIDE) < n:
        _SIDE.append(torch.cuda.Stream())
    return _SIDE[:n]


def sv_timed(torch, solvers, steps, barrier, red):
    """K = steps batched sv launches (one batch each) issued round-robin on len(solvers) streams, each solver with its
    own output buffers: len(solvers) batches in flight.  One wave per problem, so one batch of 1024 fills one wave per
    SIMD and a second batch in flight is a second wave on every SIMD.  The launches are pre-marshalled foreign calls
    (BatchSolver.ric_sv_bound), so that the host keeps ahead of kernels of ~0.1 ms.  Returns (max-over-ranks wall
    seconds, mean launch ms: a hipEvent pair per launch on its own stream, one stream only -- with several the events
    would overlap and cost host time between the launches)."""
    S = len(solvers)
    streams = [torch.cuda.current_stream()] + side_streams(torch, S - 1)
    calls = [x.ric_sv_bound(st) for x, st in zip(solvers, streams)]
    for c in calls:  # one untimed launch per stream: a stream's first launch pays its queue's set-up
        if c():
            raise RuntimeError("hpmpc_mi355x_ric_sv_batch failed")
    torch.cuda.synchronize()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(steps)]
    barrier()
    t0 = time.perf_counter()
    if S == 1:
        for i in range(steps):
            ev[i][0].record(streams[0])
            if calls[0]():
                raise RuntimeError("hpmpc_mi355x_ric_sv_batch failed")
            ev[i][1].record(streams[0])
    else:
        for i in range(steps):
            if calls[i % S]():
                raise RuntimeError("hpmpc_mi355x_ric_sv_batch failed")
    for st in streams[1:]:
        streams[0].wait_stream(st)
    barrier()
    dt = red.max(time.perf_counter() - t0)
    return dt, (float(np.mean([a.elapsed_time(b) for a, b in ev])) if S == 1 else None)


def bench_riccati_small(args, torch, red, rank, world, barrier, stream):
    """configs[2]: batch x mass-spring N=50 nx=8 nu=3, Riccati only (d_back_ric_rec_sv_tv_res, nb = 0,
    compute_pi = 1); fact/s over all ranks, hipEvents around each batched launch for the roofline."""
    from hpmpc_amd.batch import BatchSolver, algorithmic_bytes_per_sv
    from hpmpc_amd.shard import make_shard

    B, N, nx, nu = args.batch, 50, 8, 3
    qp = make_shard(N, nx, nu, rank, world, B, boxes=False)
    sols = [BatchSolver(qp, k_max=1) for _ in range(max(args.sv_streams, 1))]
    for _ in range(max(args.warmup, 1)):
        for s in sols:
            s.ric_sv()
    dt1, ms1 = sv_timed(torch, sols[:1], args.steps, barrier, red)
    dt, ms = sv_timed(torch, sols, args.steps, barrier, red)
    ms = ms1 if ms is None else ms
    by = algorithmic_bytes_per_sv(qp)
    ach = B * args.steps * by / dt / 1e9  # device level: every launch's bytes over the wall time of the K launches
    ref = ref_api() if rank == 0 else None
    par = None
    if ref is not None:
        ps = [parity_sv(ref, qp, s.ux, s.pi, spread(8, B)) for s in sols]
        par = max(ps, key=lambda x: x["max_rel_err"]) if all(ps) else None
    return {"workload": f"riccati_N{N}_nx{nx}_nu{nu}_batch{B}", "value": B * world * args.steps / dt, "unit": "fact/s",
            "batches_in_flight": len(sols), "launch_ms": ms, "parity": par,
            "roofline": {"bound": "hbm", "kernel": "hk_ric_sv", "achieved": ach, "peak": PEAK_HBM_GBS,
                         "unit": "GB/s", "frac": ach / PEAK_HBM_GBS, "algorithmic_bytes_per_sv": by,
                         "unit_of_work": f"K = {args.steps} launches of one batch, {len(sols)} in flight, over their "
                                         f"wall time (the launches overlap; launch_ms is the one-stream run's)"},
            "one_batch_in_flight": {"value": B * world * args.steps / dt1, "launch_ms": ms1,
                                    "frac": B * by / (ms1 * 1e-3) / 1e9 / PEAK_HBM_GBS}}


def bench_aliased(args, torch, red, rank, world, barrier, slots):
    """SURVEY.md §8d's aliased "time-invariant" mode, reported beside the headline: the same IPM workload, but every
    problem shares one A / B / Q / R (time-invariant mass-spring data, the drivers' aliasing, test_d_ip_hard.c:652-662)
    and the problems differ only in x0, so the batched layout holds one copy of every stage block except stage 0's
    (hpmpc_mi355x_layout BAbt_shared / RSQrq_shared) and the stage data stay in L2 / the Infinity Cache.  Timed
    through the same problem queue; beside it the same data in the ordinary per-problem layout."""
    from hpmpc_amd.batch import BatchSolver, IpmQueue
    from hpmpc_amd.shard import make_shard

    B, N, nx, nu = args.batch, args.N, args.nx, args.nu
    qa = make_shard(N, nx, nu, rank, world, B, time_variant=False)
    out = {"workload": f"ipm_N{N}_nx{nx}_nu{nu}_batch{B}_time_invariant_aliased", "unit": "IP-iter/s"}
    for name, aliased in (("aliased", True), ("per_problem_layout", False)):
        s = BatchSolver(qa, k_max=args.k_max, aliased=aliased)
        s.queue(B, slots).run()
        Q = s.queue(args.steps * B, slots)
        barrier()
        t0 = time.perf_counter()
        pm, ticks = Q.run(profiled=True)
        barrier()
        dt = red.max(time.perf_counter() - t0)
        it = red.sum(float(Q.kk.sum().item()))
        r = {"value": it / dt, "ms_per_step": dt / args.steps * 1e3,
             "stage_data_bytes": int((s.BAbt.numel() + s.RSQrq.numel()) * 8),
             "pass_ms_per_step": {n: float(v) / args.steps for n, v in
                                  zip(IpmQueue.PASS_KERNELS, pm) if n}}
        if aliased:
            out.update(r)
            ref = ref_api() if rank == 0 else None
            out["parity"] = parity_ipm(ref, qa, dict(ux=Q.ux, pi=Q.pi, lam=Q.lam, t=Q.t, kk=Q.kk, ret=Q.ret,
                                                     k_max=args.k_max), [(q, q % B) for q in spread(8, args.steps * B)])
        else:
            out[name] = r
        del Q, s
    return out


def bench_coupled(args, torch, red, rank, world, barrier, slots, headline_value):
    """the headline IPM workload with strongly coupled stage Hessians (hpmpc_amd.shard.coupled_shard:
    diag(R, Q) + G G' / nux, positive definite but not diagonally dominant, so Gershgorin's bound is negative on every
    inner stage).  The clamp certificate then rests on the shifted-Cholesky bound (hk_riccati.h cert_g_shift); before
    it, every stage of every factorisation took the clamped x-block fallback.  Same queue, slots and steps as the
    headline; the ratio to the headline's rate is reported beside it."""
    from hpmpc_amd.batch import BatchSolver, IpmQueue
    from hpmpc_amd.shard import coupled_shard

    B, N, nx, nu = args.batch, args.N, args.nx, args.nu
    qc = coupled_shard(N, nx, nu, rank, world, B)
    s = BatchSolver(qc, k_max=args.k_max)
    s.queue(B, slots).run()
    K = min(args.steps, 20)
    Q = s.queue(K * B, slots)
    barrier()
    t0 = time.perf_counter()
    pm, ticks = Q.run(profiled=True)
    barrier()
    dt = red.max(time.perf_counter() - t0)
    it = red.sum(float(Q.kk.sum().item()))
    ret = Q.ret.cpu().numpy()
    out = {"workload": f"ipm_N{N}_nx{nx}_nu{nu}_batch{B}_coupled_hessians", "value": it / dt, "unit": "IP-iter/s",
           "steps": K, "ms_per_step": dt / K * 1e3, "vs_headline": (it / dt) / headline_value,
           "ret_counts": {str(int(r)): int((ret == r).sum()) for r in np.unique(ret)},
           "pass_ms_per_step": {n: float(v) / K for n, v in
                                zip(IpmQueue.PASS_KERNELS, pm) if n}}
    ref = ref_api() if rank == 0 else None
    out["parity"] = parity_ipm(ref, qc, dict(ux=Q.ux, pi=Q.pi, lam=Q.lam, t=Q.t, kk=Q.kk, ret=Q.ret, k_max=args.k_max),
                               [(q, q % B) for q in spread(8, K * B)])
    del Q, s
    return out


def bench_scatter(args, torch, dist, rank, world, solver, template, B, barrier):
    """configs[3]'s data path (SURVEY.md §8e scatter mode): rank 0 holds every rank's block in HBM and sends
    it over RCCL point-to-point (xGMI), each rank solves its block through the problem queue, and ux / pi /
    kk / ret come back to rank 0.  Times the scatter, the solve and the gather separately (max over ranks)."""
    from hpmpc_amd.batch import pack_batch
    from hpmpc_amd.shard import gather_to_root, make_shard, scatter_from_root

    N, nx, nu = args.N, args.nx, args.nu
    local = [solver.BAbt, solver.RSQrq, solver.d]
    blocks = None
    if rank == 0:
        blocks = [[torch.from_numpy(a).cuda() for a in pack_batch(make_shard(N, nx, nu, r, world, B))]
                  for r in range(world)]
    ref = [t.clone() for t in local]  # the seed-mode block of this rank: the scatter must reproduce it
    for t in local:
        t.zero_()
    red = solver._red

    def timed(fn):
        barrier()
        t0 = time.perf_counter()
        out = fn()
        barrier()
        return red.max(time.perf_counter() - t0), out

    t_sc, _ = timed(lambda: scatter_from_root(dist, rank, world, local, blocks))
    same = all(torch.equal(a, b) for a, b in zip(local, ref))
    del blocks, ref
    Q = solver.queue(B, 2 * B)
    t_solve, _ = timed(lambda: Q.run())
    res = [Q.ux, Q.pi, Q.kk, Q.ret]
    t_ga, got = timed(lambda: gather_to_root(dist, rank, world, res))
    iters = red.sum(float(Q.kk.sum().item()))
    out = {"scatter_ms": t_sc * 1e3, "solve_ms": t_solve * 1e3, "gather_ms": t_ga * 1e3,
           "scattered_bytes_per_rank": int(sum(t.numel() * t.element_size() for t in local)),
           "gathered_bytes_per_rank": int(sum(t.numel() * t.element_size() for t in res)),
           "scatter_matches_seed_block": bool(red.min(1.0 if same else 0.0) == 1.0),
           "value_with_scatter_gather": iters / (t_sc + t_solve + t_ga), "value_solve_only": iters / t_solve,
           "unit": "IP-iter/s", "note": "one batch per rank; value_* over all ranks"}
    if rank == 0:
        out["gathered_iters"] = int(sum(int(g[2].sum().item()) for g in got))
    return out


def main():
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        launch_ranks(args)  # does not return
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        print(f"bench.py: rank {rank}: WORLD_SIZE={world} but --gpus {args.gpus}; using the launcher's "
              f"world size", file=sys.stderr)
    if args.check_launch:
        import torch.distributed as cdist

        if world > 1:
            cdist.init_process_group("gloo")
        # one write() per line: the ranks share the launcher's stdout pipe, and print() may split the text
        # and its newline into two writes that interleave with the other rank's
        sys.stdout.flush()
        os.write(1, (json.dumps({"rank": rank, "world": cdist.get_world_size() if world > 1 else 1}) + "\n").encode())
        if world > 1:
            cdist.destroy_process_group()
        return
    import torch

    torch.cuda.set_device(local)
    dist = None
    if world > 1:
        import torch.distributed as dist

        dist.init_process_group("nccl")
    print(f"bench.py: rank {rank} of world {world} on cuda:{local}", file=sys.stderr, flush=True)

    from hpmpc_amd.batch import (BatchSolver, IpmQueue, algorithmic_bytes_per_ip_iter, algorithmic_bytes_per_pass,
                                 algorithmic_bytes_per_sv, flops_ip_iter, flops_sv)
    from hpmpc_amd.shard import Reducer, make_shard

    from hpmpc_amd.shard import split_batch

    B, N, nx, nu = args.batch, args.N, args.nx, args.nu
    strong = args.global_batch > 0
    if strong:
        B = split_batch(args.global_batch, world)
    qp = make_shard(N, nx, nu, rank, world, B)
    solver = BatchSolver(qp, k_max=args.k_max)
    qp_ric = make_shard(N, nx, nu, rank, world, B, boxes=False)
    ric = BatchSolver(qp_ric, k_max=1)
    stream = torch.cuda.current_stream()
    red = Reducer(dist, "cuda")
    solver._red = red

    def barrier():
        torch.cuda.synchronize()
        red.barrier()
        torch.cuda.synchronize()

    max_over_ranks, sum_over_ranks = red.max, red.sum

    # ---------------- IPM (headline) ----------------
    # A step is one batch of B problems.  The K timed steps go through one problem queue
    # (hpmpc_mi355x_ipm_queue): `slots` resident solver slots, each taking the next problem of the
    # queue as soon as its own has converged, so K batches cost ~K x (mean iterations), not
    # K x (max iterations).  Profiled run: one hipEvent per kernel boundary on the solve's stream.
    # two resident problems per SIMD of the chip (256 CUs x 4 SIMDs): a per-GPU batch below 1024 (the strong-
    # scaling split of configs[3], 4096 over 8 GPUs = 512 per GPU) still fills every SIMD twice from the queue
    # more slots than the chip holds resident (2 per SIMD = 2048): each pass launch then dispatches the waiting slots
    # as earlier ones finish, so a launch no longer waits for its slowest resident slot (tools/slots_probe.py: 2048 /
    # 4096 / 6144 / 8192 slots 1.53 / 1.56 / 1.59 / 1.61 M IP-iter/s at K = 20 with the drain).  The queue runs its
    # slots as four lanes of 2048 on four streams (one shared entry counter), whose pass kernels overlap one another's
    # launch tails (tools/mstream_probe.py: 1.60 -> 1.70 M at K = 20; the lanes' kernel times overlap, so the per-pass
    # launch_ms below are per lane launch, summed over the lanes' concurrent streams by rocprofv3 alike)
    slots = args.slots if args.slots > 0 else max(8 * B, 8192)
    if args.warmup > 0:
        wq = solver.queue(args.warmup * B, slots)
        wq.run()
        torch.cuda.synchronize()
        del wq
    Q = solver.queue(args.steps * B, slots)
    barrier()
    t0 = time.perf_counter()
    pass_ms, ticks = Q.run(profiled=True)
    barrier()
    t1 = time.perf_counter()
    dt = max_over_ranks(t1 - t0)
    kk = Q.kk.cpu().numpy()
    ret = Q.ret.cpu().numpy()
    iters_rank = float(kk.sum())
    drain_iters, drain_probs = Q.drained()
    iters_total = sum_over_ranks(iters_rank)
    value = iters_total / dt
    # a tick is three launches (IpmQueue.PASS_KERNELS: fact, predictor + corrector, update); names[i] times pass_ms[i]
    names = list(IpmQueue.PASS_KERNELS)
    # the dominant launch (largest device time per step): each kernel runs one launch per tick; per launch, the
    # problem-iterations it processes (sum kk / ticks) x that kernel's algorithmic bytes (algorithmic_bytes_per_pass),
    # over its average launch duration (both from this timed run)
    dom = max((i for i in range(1, len(names)) if names[i]), key=lambda i: pass_ms[i])
    bytes_pass = algorithmic_bytes_per_pass(qp)
    # the problem-iterations the tick launches ran (the drain's own are not in the pass kernels)
    probs_per_launch = (iters_rank - drain_iters) / ticks
    per_pass = {}
    for i in range(1, len(names)):
        if not names[i]:
            continue
        lm = pass_ms[i] / ticks
        per_pass[names[i]] = {"launch_ms": float(lm), "algorithmic_bytes_per_problem_iter": bytes_pass[names[i]],
                              "achieved_GBps": probs_per_launch * bytes_pass[names[i]] / (lm * 1e-3) / 1e9}
    launch_ms = per_pass[names[dom]]["launch_ms"]
    bytes_dom = bytes_pass[names[dom]]
    achieved = per_pass[names[dom]]["achieved_GBps"]
    bytes_iter = algorithmic_bytes_per_ip_iter(qp)
    dt_rank = t1 - t0
    step_achieved = iters_rank * bytes_iter / dt_rank / 1e9
    n_lanes = len(Q.lanes())
    fl_iter = flops_ip_iter(N, nx, nu)
    # parity sample of the timed run (after it): 8 queue entries spread over the K batches against the reference
    ref = ref_api() if rank == 0 else None
    nq = args.steps * B
    par_ipm = parity_ipm(ref, qp, dict(ux=Q.ux, pi=Q.pi, lam=Q.lam, t=Q.t, kk=Q.kk, ret=Q.ret, k_max=args.k_max),
                         [(q, q % B) for q in spread(8, nq)])
    del Q

    # the same queue with 40 batches (the drain's fixed cost amortised over twice the work), beside the driver's K
    k40 = None
    if not args.no_k40 and args.steps != 40:
        Q = solver.queue(40 * B, slots)
        barrier()
        q0 = time.perf_counter()
        Q.run()
        barrier()
        qdt = max_over_ranks(time.perf_counter() - q0)
        k40 = {"steps": 40, "value": sum_over_ranks(float(Q.kk.sum().item())) / qdt, "unit": "IP-iter/s",
               "ms_per_step": qdt / 40 * 1e3}
        del Q

    # the same K batches through a queue with one resident slot per problem of the batch (B slots: the
    # metric's literal batch resident at once), beside the headline's 2 x B slots
    qb = None
    if not args.no_queue_batch_slots and slots != B:
        Q = solver.queue(args.steps * B, B)
        barrier()
        q0 = time.perf_counter()
        Q.run()
        barrier()
        qdt = max_over_ranks(time.perf_counter() - q0)
        qb = {"slots": B, "value": sum_over_ranks(float(Q.kk.sum().item())) / qdt, "unit": "IP-iter/s",
              "ms_per_step": qdt / args.steps * 1e3}
        del Q

    # the generic-shape kernels (DynSh: stage sizes read from the stage table, no compile-time class) on a shape
    # with no compiled class, nx = 10 nu = 3, same N / constraints / queue: what any other caller shape runs at
    dyn = None
    if not args.no_isolated and rank == 0:
        qd = make_shard(N, 10, 3, 0, 1, B)
        sd = BatchSolver(qd, k_max=args.k_max)
        Kd = min(args.steps, 10)
        sd.queue(B, slots).run()
        Qd = sd.queue(Kd * B, slots)
        torch.cuda.synchronize()
        d0 = time.perf_counter()
        pd, td = Qd.run(profiled=True)
        torch.cuda.synchronize()
        ddt = time.perf_counter() - d0
        itd = float(Qd.kk.sum().item())
        dyn = {"workload": f"ipm_N{N}_nx10_nu3_batch{B}_generic_kernels", "value": itd / ddt, "unit": "IP-iter/s",
               "steps": Kd, "fact_us_per_problem_iter": pd[1] * 1e3 / itd,
               "headline_fact_us_per_problem_iter": pass_ms[1] * 1e3 / iters_rank,
               "pass_ms_per_step": {n: float(v) / Kd for n, v in zip(names, pd) if n}}
        del Qd, sd

    # one isolated batch (no queue): the latency of a batch solve, reported beside the queue rate
    iso = None
    if not args.no_isolated:
        solver.ipm_profiled()
        torch.cuda.synchronize()
        iso_ms = float(solver.ipm_profiled().sum())
        iso_iters = float(solver.kk.sum().item())
        # the same batch through the other two entry points: a queue of one batch in as many slots (ticks, then
        # the multi-wave drain of the survivors) and the solo kernel over the batch (one 4-wave workgroup per
        # problem from the first iteration)
        def dev_ms(fn):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            fn()
            e0.record(stream)
            fn()
            e1.record(stream)
            torch.cuda.synchronize()
            return e0.elapsed_time(e1)

        q1 = solver.queue(B, B)
        q_ms = dev_ms(q1.run)
        q_iters = float(q1.kk.sum().item())
        so_ms = dev_ms(solver.ipm_solo)
        so_iters = float(solver.kk.sum().item())
        del q1
        iso = {"ms": iso_ms, "value": iso_iters / (iso_ms * 1e-3), "unit": "IP-iter/s",
               "note": "one batch solved alone (hpmpc_mi355x_ipm_batch): every pass runs k_max times, so the "
                       "slowest problem sets the time",
               "queue_one_batch": {"ms": q_ms, "value": q_iters / (q_ms * 1e-3),
                                   "path": "hpmpc_mi355x_ipm_queue, nq = n_slots = batch (ticks, then the drain)"},
               "solo_batch": {"ms": so_ms, "value": so_iters / (so_ms * 1e-3),
                              "path": "hpmpc_mi355x_ipm_solo over the batch (hk_ipm_solo_mw, one 4-wave "
                                      "workgroup per problem)"}}

    ali = None if args.no_aliased else bench_aliased(args, torch, red, rank, world, barrier, slots)
    cpl = None if args.no_coupled else bench_coupled(args, torch, red, rank, world, barrier, slots, value)

    # ---------------- Riccati factorisation + solve ----------------
    # K steps of one batch each with args.sv_streams batches in flight (own output buffers per stream), and the same
    # K steps on one stream beside it
    rics = [ric] + [BatchSolver(qp_ric, k_max=1) for _ in range(max(args.sv_streams, 1) - 1)]
    for _ in range(args.warmup):
        for r_ in rics:
            r_.ric_sv()
    rdt1, sv_ms1 = sv_timed(torch, rics[:1], args.steps, barrier, red)
    rdt, sv_ms = sv_timed(torch, rics, args.steps, barrier, red)
    sv_ms = sv_ms1 if sv_ms is None else sv_ms
    fact_total = B * world * args.steps
    par_sv = None
    if ref is not None:
        ps = [parity_sv(ref, qp_ric, r_.ux, r_.pi, spread(8, B)) for r_ in rics]
        par_sv = max(ps, key=lambda x: x["max_rel_err"]) if all(ps) else None
    sv_bytes = algorithmic_bytes_per_sv(qp_ric)
    sv_achieved = B * args.steps * sv_bytes / rdt / 1e9  # this rank's launches over the (max-over-ranks) wall time

    traffic = traffic_dom_launch = None
    pmc = os.path.join(ROOT, "profiles", "pmc_hk_ipm.json")
    if os.path.exists(pmc):
        try:
            with open(pmc) as f:
                pm = json.load(f)
            if pm.get("workload") == f"ipm_queue_N{N}_nx{nx}_nu{nu}_batch{B}_slots{slots}":
                # measured HBM bytes per problem-iteration of each pass (the PMC run's bytes per launch x its
                # launches / its sum kk; two passes of the same run are averaged) x this run's problems per launch
                for n, pp in per_pass.items():
                    kp = pm["kernels"].get(n)
                    if kp:
                        nl = len(kp["raw_fetch"]) / 2
                        per_it = kp["hbm_bytes_per_launch"] * nl / pm["kk_sum_per_solve"]
                        pp["traffic_bytes_per_problem_iter"] = per_it
                        pp["traffic_over_algorithmic"] = per_it / pp["algorithmic_bytes_per_problem_iter"]
                t_dom = per_pass[names[dom]].get("traffic_bytes_per_problem_iter")
                traffic_dom_launch = None if t_dom is None else t_dom * probs_per_launch
                # per step: the four passes' measured bytes per problem-iteration x this run's iterations per step
                # (the drained iterations priced at the pass kernels' rate)
                t_it = [pp.get("traffic_bytes_per_problem_iter") for pp in per_pass.values()]
                if all(x is not None for x in t_it):
                    traffic = sum(t_it) * iters_rank / args.steps
        except Exception:
            traffic = None

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu:
        cpu = cpu_baseline(qp, args.cpu_seconds, args.k_max, args.cpu_threads)

    sc = None
    if world > 1 and not args.no_scatter:
        sc = bench_scatter(args, torch, dist, rank, world, solver, qp, B, barrier)
    pc = None if args.no_pcond else bench_pcond(args, torch, red, rank, world, barrier)
    # configs[2] and configs[1]; skipped in profiling runs so every hk_ipm_* launch belongs to the timed queue
    rs = None if args.no_isolated else bench_riccati_small(args, torch, red, rank, world, barrier, stream)
    sq = bench_single_qp(args, torch, stream) if (rank == 0 and not args.no_isolated) else None

    if rank == 0:
        line = {
            "metric": BASELINE_METRIC,
            "value": value,
            "unit": "IP-iter/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": dt / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": "strong" if strong else "weak",
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic (mass-spring MPC, per-problem x0 ~ U(-2.5,2.5) from PCG64(20261015+p), time-variant "
                    "A/B/Q perturbations; each rank generates its block (seed mode); the rank-0 scatter / gather of "
                    "the same blocks is timed separately in 'scatter')",
            "config": {"workload": f"ipm_N{N}_nx{nx}_nu{nu}_batch{B}", "N": N, "nx": nx, "nu": nu,
                       "batch_per_gpu": B, "global_batch": B * world, "k_max": args.k_max, "mu_tol": 1e-12,
                       "parallelism": f"dp{world}" if world > 1 else "single",
                       "resident_slots": slots,
                       "schedule": f"problem queue: {args.steps} batches of {B} per rank through {slots} resident "
                                   f"slots (hpmpc_mi355x_ipm_queue); 'queue_batch_slots' is the same run with "
                                   f"{B} slots",
                       "sum_kk_per_step": iters_total / args.steps, "ret_counts": {
                           str(int(r)): int((ret == r).sum()) for r in np.unique(ret)}},
            # The queue's four lanes run the four pass kernels concurrently on four streams, so a pass launch's
            # duration overlaps the other lanes' launches and per-launch rates understate the device: the roofline's
            # unit of work is one step (a batch of B problems solved through the queue, init and drain included),
            # its algorithmic bytes the sum over the step's IP iterations of the four passes' algorithmic bytes,
            # over the step's wall time (conservative: host gaps, init and drain included).  The dominant pass's
            # per-lane-launch figures (which rocprofv3's kernel stats reproduce) are kept beside it.
            "roofline": {"bound": "hbm", "achieved": step_achieved, "peak": PEAK_HBM_GBS, "unit": "GB/s",
                         "frac": step_achieved / PEAK_HBM_GBS, "traffic": traffic,
                         "kernel": "hk_ipm_fact + hk_ipm_pred + hk_ipm_corr + hk_ipm_update (one IP iteration, "
                                   f"{n_lanes} concurrent lanes)",
                         "unit_of_work": "one step: a batch of B problems through the queue (per rank)",
                         "algorithmic_bytes_per_step": bytes_iter * iters_rank / args.steps,
                         "traffic_over_algorithmic": (None if traffic is None else
                                                      traffic / (bytes_iter * iters_rank / args.steps)),
                         "lanes": n_lanes,
                         "dominant_pass": {"kernel": names[dom], "launch_ms": launch_ms, "launches": int(ticks),
                                           "problem_iters_per_launch": probs_per_launch,
                                           "achieved_GBps_per_launch": achieved,
                                           "frac_per_launch": achieved / PEAK_HBM_GBS,
                                           "traffic_per_launch": traffic_dom_launch},
                         "drain": {"kernel": "hk_ipm_qdrain_mw", "problems": drain_probs, "iterations": drain_iters,
                                   "ms_with_init": float(pass_ms[0])},
                         "algorithmic_bytes_per_problem_iter": bytes_dom,
                         "per_pass": per_pass,
                         "pass_ms_per_step": {n: float(v / args.steps) for n, v in zip(names, pass_ms) if n},
                         # fixed fields: the two largest launches (per lane launch) and the whole iteration
                         "frac_fact": per_pass["hk_ipm_fact"]["achieved_GBps"] / PEAK_HBM_GBS,
                         "frac_predcorr": per_pass["hk_ipm_predcorr"]["achieved_GBps"] / PEAK_HBM_GBS,
                         "frac_whole_iteration": step_achieved / PEAK_HBM_GBS,
                         "ipm_whole_solve": {"achieved_GBps": step_achieved,
                                             "algorithmic_bytes_per_ip_iter": bytes_iter,
                                             "fp64_tflops": iters_rank * fl_iter / dt_rank / 1e12}},
            "k40": k40,
            "queue_batch_slots": qb,
            "aliased": ali,
            "coupled": cpl,
            "generic_shape": dyn,
            "isolated_batch": iso,
            "scatter": sc,
            "parity": par_ipm,
            "riccati": {"value": fact_total / rdt, "unit": "fact/s", "kernel": "hk_ric_sv", "launch_ms": sv_ms,
                        "batches_in_flight": len(rics), "parity": par_sv,
                        "roofline": {"bound": "hbm", "achieved": sv_achieved, "peak": PEAK_HBM_GBS, "unit": "GB/s",
                                     "frac": sv_achieved / PEAK_HBM_GBS,
                                     "algorithmic_bytes_per_sv": sv_bytes,
                                     "unit_of_work": f"K = {args.steps} launches of one batch, {len(rics)} in flight, "
                                                     "over their wall time (the launches overlap; launch_ms is the "
                                                     "one-stream run's per-launch time)",
                                     "fp64_tflops": B * args.steps * flops_sv(N, nx, nu) / rdt / 1e12},
                        "one_batch_in_flight": {"value": fact_total / rdt1, "launch_ms": sv_ms1,
                                                "frac": B * sv_bytes / (sv_ms1 * 1e-3) / 1e9 / PEAK_HBM_GBS}},
            "cpu_baseline": cpu,
            "pcond": pc,
            "riccati_batch_N50": rs,
            "single_qp": sq,
        }
        print(json.dumps(line), flush=True)
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
