import ctypes as C, os, torch
L = C.CDLL(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "hpmpc_amd", "lib", "libsoff_test.so"))
L.run.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p]
b = torch.arange(20000, dtype=torch.float64, device="cuda") + 1
o = torch.full((128,), -7.0, dtype=torch.float64, device="cuda")
L.run(b.data_ptr(), o.data_ptr(), torch.cuda.current_stream().cuda_stream); torch.cuda.synchronize()
o = o.cpu().numpy()
print("valid lanes (expect 129 + l):", o[0:8:2])
print("masked lanes soff=1024 (expect 0):", o[1:8:2])
print("valid soff=64K (expect 8193 + l):", o[64:72:2], " masked:", o[65:72:2])
