"""Headline workload (K batches of 1024 x N=100 nx=12 nu=4) split over L independent problem queues, each driven by
its own host thread on its own HIP stream, so that one queue's pass kernels fill the tail of another's
(L=1 is the bench's single queue).  Prints IP-iter/s per (L, slots per queue).
    python3 tools/mstream_probe.py [K]"""
import os
import sys
import threading
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from hpmpc_amd.batch import BatchSolver  # noqa: E402
from hpmpc_amd.shard import make_shard  # noqa: E402


def run(s, K, L, slots):
    nq = K * 1024 // L
    qs = [s.queue(nq, slots) for _ in range(L)]
    sts = [torch.cuda.Stream() for _ in range(L)]
    torch.cuda.synchronize()
    err = []

    def go(i):
        try:
            with torch.cuda.stream(sts[i]):
                qs[i].run()
        except Exception as e:  # noqa: BLE001
            err.append(e)

    th = [threading.Thread(target=go, args=(i,)) for i in range(L)]
    t0 = time.perf_counter()
    for t in th:
        t.start()
    for t in th:
        t.join()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    if err:
        raise err[0]
    it = sum(float(q.kk.sum().item()) for q in qs)
    return it / dt, dt


def main():
    """Three rounds of: the library's own lanes (one queue of 8192 slots, HPMPC_MI355X_QUEUE_LANES=4), four host
    threads each driving a one-lane queue of 2048 slots, and one one-lane queue of 8192 slots."""
    K = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    s = BatchSolver(make_shard(100, 12, 4, 0, 1, 1024), k_max=50)
    run(s, 4, 1, 8192)
    for rnd in range(3):
        for name, lanes_env, L, slots in (("C lanes", "4", 1, 8192), ("py threads", "1", 4, 2048),
                                          ("one lane", "1", 1, 8192)):
            os.environ["HPMPC_MI355X_QUEUE_LANES"] = lanes_env
            run(s, 4, L, slots)
            best = max(run(s, K, L, slots) for _ in range(2))
            print(f"round {rnd} K={K} {name}: queues={L} slots/queue={slots} lanes env={lanes_env}: "
                  f"{best[0]:.0f} IP-iter/s ({best[1] * 1e3:.1f} ms)", flush=True)


if __name__ == "__main__":
    main()
