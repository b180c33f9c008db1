import ctypes as C, os, numpy as np, torch
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
L = C.CDLL(os.path.join(ROOT, "hpmpc_amd", "lib", "librsq_precision.so"))
L.rsq_run.argtypes = [C.c_void_p] * 4 + [C.c_int, C.c_void_p]
rng = np.random.default_rng(0)
n = 1 << 20
d = np.exp(rng.uniform(np.log(1e-12), np.log(1e12), n))
D = torch.from_numpy(d).cuda()
Y = [torch.empty_like(D) for _ in range(3)]
L.rsq_run(D.data_ptr(), Y[0].data_ptr(), Y[1].data_ptr(), Y[2].data_ptr(), n, torch.cuda.current_stream().cuda_stream)
torch.cuda.synchronize()
ref = 1.0 / np.sqrt(d.astype(np.longdouble))
for i, y in enumerate(Y):
    y = y.cpu().numpy().astype(np.longdouble)
    rel = np.abs((y - ref) / ref).astype(np.float64)
    print(f"variant {['raw', 'newton1', 'third-order'][i]}: max rel err {rel.max():.3e} ({rel.max() / 2.0**-53:.1f} half-ulps), mean {rel.mean():.3e}")
# sqrt reference check: s = d*y vs sqrt(d)
