"""Run tools/lat_ubench.hip: cycles per instruction (dependent chains and independent streams)."""
import ctypes as C, os
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
import torch
L = C.CDLL(os.path.join(ROOT, "hpmpc_amd", "lib", "liblat_ubench.so"))
L.lat_run.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p]
out = torch.zeros(64, dtype=torch.float64, device="cuda")
cyc = torch.zeros(16, dtype=torch.int64, device="cuda")
for _ in range(3):
    L.lat_run(out.data_ptr(), cyc.data_ptr(), torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
c = cyc.cpu().numpy()
rows = [("dependent v_fma_f64", 0, 64), ("dependent v_mul_f64", 1, 64), ("dependent v_rsq_f64", 2, 64),
        ("independent v_fma_f64", 3, 512), ("independent v_fma_f32", 4, 512), ("v_cndmask_b32 stream", 5, 256),
        ("dependent v_mov_dpp", 6, 64), ("independent v_mov_dpp", 7, 256), ("dependent permlane16_swap", 8, 64),
        ("independent v_rsq_f64", 9, 256), ("dependent mfma_f64_16x16x4", 10, 64),
        ("mfma_f64 -> v_add_f64 -> mfma", 11, 64), ("dependent v_mov_b64_dpp", 12, 64),
        ("dependent permlane32_swap", 13, 64), ("LDS write+read round trip", 14, 64),
        ("readfirstlane -> salu -> vmov", 15, 64)]
for name, i, n in rows:
    print(f"{name:28s} {c[i] / n:6.2f} cyc/instr")
