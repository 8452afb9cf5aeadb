"""Probe: vendor FP64 GEMM rate via torch.matmul (rocBLAS/hipBLASLt) on the box.
Only a yardstick for our own HIP DGEMM; not used by the product."""
import torch, time
d = torch.device("cuda:0")
for (m, n, k) in [(4096, 4096, 4096), (2048, 1024, 65536), (8192, 8192, 8192)]:
    a = torch.randn(m, k, dtype=torch.float64, device=d)
    b = torch.randn(k, n, dtype=torch.float64, device=d)
    for _ in range(2):
        c = a @ b
    torch.cuda.synchronize()
    t = time.perf_counter(); r = 5
    for _ in range(r):
        c = a @ b
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t) / r
    print(f"torch fp64 matmul {m}x{n}x{k}: {2*m*n*k/dt/1e12:.2f} TFLOP/s")
