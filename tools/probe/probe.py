import ctypes, os, time, subprocess, torch
here = os.path.dirname(os.path.abspath(__file__))
print("torch", torch.__version__, "hip", torch.version.hip, torch.cuda.get_device_name(0))
p = torch.cuda.get_device_properties(0); print("CUs", p.multi_processor_count, "mem GB", p.total_memory/2**30)
lib = ctypes.CDLL(os.path.join(here, "probe.so"))
s = torch.cuda.current_stream().cuda_stream
def run(which, M, N, K, dt):
    A = torch.randint(-4, 5, (M, K), device="cuda").to(dt)
    Bt = torch.randint(-4, 5, (N, K), device="cuda").to(dt)
    C = torch.zeros(M, N, device="cuda")
    rc = lib.probe_run(which, ctypes.c_void_p(A.data_ptr()), ctypes.c_void_p(Bt.data_ptr()), ctypes.c_void_p(C.data_ptr()), ctypes.c_void_p(s))
    torch.cuda.synchronize()
    ref = A.float() @ Bt.float().t()
    print("mfma", which, "rc", rc, "maxerr", (C - ref).abs().max().item())
run(0, 16, 16, 32, torch.bfloat16); run(1, 32, 32, 16, torch.bfloat16); run(2, 16, 16, 4, torch.float32)
# conv timing (fp32, DPT-like) via torch/MIOpen
import torch.nn.functional as F
for (C_in, C_out, H) in [(256, 256, 256), (256, 128, 512)]:
    x = torch.randn(1, C_in, H, H, device="cuda"); w = torch.randn(C_out, C_in, 3, 3, device="cuda")
    t0 = time.time(); y = F.conv2d(x, w, padding=1); torch.cuda.synchronize(); t1 = time.time()
    for _ in range(3): y = F.conv2d(x, w, padding=1)
    torch.cuda.synchronize(); t2 = time.time()
    fl = 2 * H * H * C_in * C_out * 9
    print(f"conv {C_in}->{C_out} @{H}: first {t1-t0:.2f}s, then {(t2-t1)/3*1e3:.2f} ms = {fl/((t2-t1)/3)/1e12:.1f} TF")
a = torch.randn(8192, 8192, device="cuda", dtype=torch.bfloat16); b = torch.randn(8192, 8192, device="cuda", dtype=torch.bfloat16)
for _ in range(2): c = a @ b
torch.cuda.synchronize(); t = time.time()
for _ in range(10): c = a @ b
torch.cuda.synchronize(); dt = (time.time() - t) / 10
print(f"torch bf16 gemm 8192^3: {2*8192**3/dt/1e12:.0f} TF")
print(subprocess.run("lscpu | head -20; nproc; cat /sys/fs/cgroup/cpu.max 2>/dev/null", shell=True, capture_output=True, text=True).stdout)
