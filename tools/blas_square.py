"""Practical f16 GEMM peak on this box: torch half matmul (hipBLASLt) on square shapes (measurement aid)."""
import torch
torch.cuda.init()
for n in (8192, 16384):
    a = torch.randn(n, n, device="cuda", dtype=torch.float16); b = torch.randn(n, n, device="cuda", dtype=torch.float16)
    for _ in range(3): c = a @ b
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(10): c = a @ b
    e.record(); torch.cuda.synchronize()
    ms = s.elapsed_time(e) / 10
    print(f"f16 square {n}: {ms:.3f} ms, {2.0 * n**3 / ms / 1e9:.1f} TF/s", flush=True)
