"""Cycle breakdown of the multi-wave solo kernel (hk_ipm_solo_mw) on one configs[1] problem (N=100 nx=12 nu=4), from
the -DHK_STAMPS build (build.py build_stamps, loaded through HPMPC_MI355X_LIB): s_memtime totals per IPM body over
the whole solve, and the cycles each wave spent waiting on the LDS hand-over (wave 0: the recursion; 1..3: helpers).
Ticks are s_memtime units; the solo time per iteration (latency_probe.py) converts them."""
import ctypes as C
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from hpmpc_amd.batch import BatchSolver, lib  # noqa: E402
from hpmpc_amd.ocp import mass_spring_qp  # noqa: E402

dbg = torch.zeros(64, dtype=torch.int64, device="cuda")
lib().hpmpc_mi355x_debug_buffer.argtypes = [C.c_void_p]
lib().hpmpc_mi355x_debug_buffer(dbg.data_ptr())
s = BatchSolver(mass_spring_qp(100, 12, 4, batch=1), k_max=50)
s.ipm_solo()
s.ipm_solo()
torch.cuda.synchronize()
t = dbg.cpu().tolist()
kk = int(s.kk[0])
tot = sum(t[32:36])
print(f"kk {kk}; per iteration (s_memtime ticks): " + " ".join(
    f"{n} {t[32 + i] / kk:.0f}" for i, n in enumerate(["fact", "pred", "corr", "update"])) +
    f" | total {tot / kk:.0f}")
print("hand-over waits per iteration (ticks): " + " ".join(f"w{i} {t[40 + i] / kk:.0f}" for i in range(4)))
# one backward stage of the tile wave (stage 50, the solve's last factorisation): stamps 0 (step start),
# 5 (slot ready), 6 (slot read), 2 (M += BAbt P BAbt' done), 16 (u block factorised), 3 (end)
st = {i: t[i] for i in (0, 5, 6, 2, 16, 3)}
if all(st.values()):
    seq = [0, 5, 6, 2, 16, 3]
    print("wave-0 backward stage 50 (ticks): " + " ".join(f"{a}->{b} {st[b] - st[a]}" for a, b in zip(seq, seq[1:])) +
          f" | total {st[3] - st[0]}")
# the tile wave's backward steps by segment, summed over every factorisation of the solve: the hand-over in (slot
# poll and reads, stage table), M += BAbt P BAbt', the tile Cholesky, the hand-over out
seg = t[48:52]
if sum(seg):
    n = kk * 101
    print("tile wave per backward step (ticks): " + " ".join(
        f"{nm} {v / n:.0f}" for nm, v in zip(["handover-in", "mfma", "chol", "handover-out"], seg)))
