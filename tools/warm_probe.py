"""Does the headline rate depend on how long the GPU has been busy?  The K=20 queue timed again and again in one
process, with the elapsed time since the first launch: IP-iter/s per repetition.
    python3 tools/warm_probe.py [reps]"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from hpmpc_amd.batch import BatchSolver  # noqa: E402
from hpmpc_amd.shard import make_shard  # noqa: E402


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 12
    s = BatchSolver(make_shard(100, 12, 4, 0, 1, 1024), k_max=50)
    T0 = time.perf_counter()
    for r in range(reps):
        Q = s.queue(20 * 1024, 8192)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        Q.run()
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        print(f"rep {r} at {t0 - T0:6.1f} s: {float(Q.kk.sum().item()) / dt:.0f} IP-iter/s ({dt * 1e3:.1f} ms)",
              flush=True)


if __name__ == "__main__" and not os.environ.get("WARM_ADDR"):
    main()


def addresses():
    """The alternating rate above follows the queue's buffer set: print each buffer's address (mod 2 MiB and 1 GiB)
    per repetition, then time the queue with its slot workspace shifted by a few offsets inside one allocation."""
    s = BatchSolver(make_shard(100, 12, 4, 0, 1, 1024), k_max=50)
    for r in range(4):
        Q = s.queue(20 * 1024, 8192)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        Q.run()
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        ptrs = {n: getattr(Q, n).data_ptr() for n in ("ws", "ux", "pi", "lam", "t", "kk", "ret", "stat", "qctl")}
        print(f"rep {r}: {float(Q.kk.sum().item()) / dt:.0f} IP-iter/s; " +
              " ".join(f"{n}={p % (1 << 21):#x}/{(p >> 30) % 1024}G" for n, p in ptrs.items()), flush=True)
    Q = s.queue(20 * 1024, 8192)
    base = Q.ws
    for off in (0, 256, 4096, 65536, 1 << 20, 0, 256, 4096, 65536, 1 << 20):
        Q.ws = torch.zeros(base.numel() + (1 << 21) // 8, dtype=torch.float64, device=base.device)[off // 8:]
        Q.ws = Q.ws[:base.numel()].view(base.shape)
        Q.run()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        Q.run()
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        print(f"ws offset {off}: {float(Q.kk.sum().item()) / dt:.0f} IP-iter/s (ws at {Q.ws.data_ptr() % (1 << 21):#x})",
              flush=True)


if __name__ == "__main__" and os.environ.get("WARM_ADDR"):
    addresses()
