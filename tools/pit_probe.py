"""configs[1] (one QP, N=100 nx=12 nu=4) through a partitioned-in-time Riccati: the horizon split into N2 segments,
each segment condensed to a problem in its boundary state by its own workgroup (hk_pcond, all segments in parallel:
the per-segment chain), the N2-stage condensed Riccati on one workgroup (hk_wide_sv: the combine), and the segments'
forward recursions in parallel again (hk_pexpand).  This is the reference's own partial condensing
(d_part_cond.c / d_part_expand_solution) used as a latency device for one problem, timed per kernel against the
serial one-wave Riccati (hk_ric_sv) and, for the IPM, against the multi-wave solo kernel.
    python3 tools/pit_probe.py  ->  one JSON line per measurement"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from hpmpc_amd.batch import BatchSolver  # noqa: E402
from hpmpc_amd.ocp import mass_spring_qp  # noqa: E402
from hpmpc_amd.pcond import PcondSolver  # noqa: E402

REPS = 20


def med(fns):
    """Median device time (ms) of each callable in fns over REPS back-to-back repetitions of the sequence."""
    st = torch.cuda.current_stream()
    ev = [[torch.cuda.Event(enable_timing=True) for _ in range(len(fns) + 1)] for _ in range(REPS)]
    for e in ev:
        e[0].record(st)
        for j, f in enumerate(fns):
            f()
            e[j + 1].record(st)
    torch.cuda.synchronize()
    return [float(np.median([e[j].elapsed_time(e[j + 1]) for e in ev])) for j in range(len(fns))]


def main():
    N, nx, nu = 100, 12, 4
    out = []
    # serial Riccati, one problem (one wave walks the 100 stages back and forth)
    one = mass_spring_qp(N, nx, nu, boxes=False, batch=1)
    s = BatchSolver(one, k_max=1)
    s.ric_sv()
    (t_sv,) = med([s.ric_sv])
    uxs = s.ux[0].cpu().numpy()
    ux_ref = np.concatenate([uxs[k, :one.nux(k)] for k in range(N + 1)])
    out.append({"what": "serial_sv", "kernel": "hk_ric_sv", "us": t_sv * 1e3})
    for N2 in (4, 5, 10, 20, 25, 50):
        try:
            pc = PcondSolver(one, N2)
            pc.solve()
            torch.cuda.synchronize()
        except Exception as e:  # noqa: BLE001
            out.append({"what": "pit_sv", "N2": N2, "refused": str(e)})
            continue
        ux = np.concatenate(pc.solution(0)[0])
        err = float(np.abs(ux - ux_ref).max() / max(np.abs(ux_ref).max(), 1e-300))
        tc, tr, te = med([pc.condense, pc.riccati, pc.expand])
        out.append({"what": "pit_sv", "N2": N2, "segment_len": -(-N // N2), "condense_us": tc * 1e3,
                    "combine_sv_us": tr * 1e3, "expand_us": te * 1e3, "total_us": (tc + tr + te) * 1e3,
                    "vs_serial": t_sv / (tc + tr + te), "ux_rel_err_vs_serial": err})
        print(json.dumps(out[-1]), flush=True)
    # the IPM of configs[1] (boxes): multi-wave solo kernel vs condense -> wide IPM -> expand
    qb = mass_spring_qp(N, nx, nu, batch=1)
    sb = BatchSolver(qb, k_max=50)
    sb.ipm_solo()
    (t_solo,) = med([sb.ipm_solo])
    kk = int(sb.kk[0].item())
    out.append({"what": "solo_ipm", "kernel": "hk_ipm_solo_mw", "kk": kk, "us": t_solo * 1e3,
                "us_per_iter": t_solo * 1e3 / kk})
    for N2 in (5, 10, 20, 25):
        try:
            pc = PcondSolver(qb, N2)
            pc.solve_ipm(k_max=50)
            torch.cuda.synchronize()
        except Exception as e:  # noqa: BLE001
            out.append({"what": "pit_ipm", "N2": N2, "refused": str(e)})
            continue
        tc, ti, te = med([pc.condense, lambda: pc.ipm(k_max=50), pc.expand])
        k2 = int(pc.kk2[0].item())
        out.append({"what": "pit_ipm", "N2": N2, "kk": k2, "ret": int(pc.ret2[0].item()), "condense_us": tc * 1e3,
                    "wide_ipm_us": ti * 1e3, "expand_us": te * 1e3, "us_per_iter": ti * 1e3 / max(k2, 1),
                    "total_us": (tc + ti + te) * 1e3})
        print(json.dumps(out[-1]), flush=True)
    for o in out:
        print(json.dumps(o))


if __name__ == "__main__":
    main()
