import time, torch, os, subprocess
t0=time.time()
print("torch", torch.__version__, "hip", torch.version.hip, flush=True)
print("avail", torch.cuda.is_available(), "n", torch.cuda.device_count(), flush=True)
p = torch.cuda.get_device_properties(0)
print(p, flush=True)
print("gcnArch", getattr(p, "gcnArchName", None), flush=True)
a = torch.randn(8192, 8192, device="cuda", dtype=torch.bfloat16)
b = torch.randn(8192, 8192, device="cuda", dtype=torch.bfloat16)
for _ in range(3): c = a @ b
torch.cuda.synchronize()
t=time.time(); n=20
for _ in range(n): c = a @ b
torch.cuda.synchronize(); dt=(time.time()-t)/n
print("bf16 8192^3 TFLOPs", 2*8192**3/dt/1e12, flush=True)
try:
    c32 = torch.mm(a, b, out_dtype=torch.float32); print("out_dtype ok", c32.dtype, flush=True)
except Exception as e: print("out_dtype fail", e, flush=True)
try:
    g = torch.zeros(8192, 8192, device="cuda", dtype=torch.float32)
    torch.addmm(g, a, b, out_dtype=torch.float32, out=g); print("addmm out_dtype inplace ok", flush=True)
except Exception as e: print("addmm out_dtype fail", e, flush=True)
print("sdpa backends", torch.backends.cuda.flash_sdp_enabled(), torch.backends.cuda.mem_efficient_sdp_enabled(), flush=True)
print("elapsed", time.time()-t0)
