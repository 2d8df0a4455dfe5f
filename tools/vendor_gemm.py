"""Reference point only (not the product path): torch.matmul (hipBLASLt/rocBLAS) fp64/fp32 on the box."""
import time, torch
for dt, n in [(torch.float64, 8192), (torch.float64, 16384), (torch.float32, 16384)]:
    a = torch.rand(n, n, dtype=dt, device="cuda") - 0.5
    b = torch.rand(n, n, dtype=dt, device="cuda") - 0.5
    for _ in range(2): c = a @ b
    torch.cuda.synchronize(); t = time.perf_counter()
    for _ in range(3): c = a @ b
    torch.cuda.synchronize(); dtm = (time.perf_counter() - t) / 3
    print(f"vendor matmul {dt} n={n}: {2*n**3/dtm/1e12:.1f} TFLOP/s")
