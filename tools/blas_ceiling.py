"""Library GEMM ceilings on the C4 FVP shapes (one MI355X, torch -> hipBLASLt / rocBLAS), to size what the
hand-written split k-loops leave on the table. f16 in / f32 accumulate (torch's half matmul) and bf16, M = 8M rows:
  [M x 512] x [512 x 256]   the two-segment row GEMMs (fvp_rfwd_l1, the R-backward k-loop of fvp_rbwdwg)
  [M x 256] x [256 x 256]   the one-segment forwards
  [256 x M] x [M x 256]     the weight gradients (K = rows)
Prints TF/s of the issued f16 work; the fp32-work rate of a 3-product split is a third of it."""
import torch

torch.cuda.init()


def bench(a, b, reps=5):
    for _ in range(2):
        c = a @ b
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        c = a @ b
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps, c


M = 8_000_000
for dt in (torch.float16, torch.bfloat16):
    for (m, k, n, name) in ((M, 512, 256, "row K=512"), (M, 256, 256, "row K=256")):
        a = torch.randn(m, k, device="cuda", dtype=dt)
        b = torch.randn(k, n, device="cuda", dtype=dt)
        ms, _ = bench(a, b)
        fl = 2.0 * m * k * n
        by = (m * k + m * n) * a.element_size()
        print(f"{str(dt):15s} {name:10s} {ms:7.3f} ms  {fl / ms / 1e9:7.1f} TF/s  {by / ms / 1e6:6.0f} GB/s", flush=True)
        del a, b
    a = torch.randn(256, M, device="cuda", dtype=dt)
    b = torch.randn(M, 256, device="cuda", dtype=dt)
    ms, _ = bench(a, b)
    print(f"{str(dt):15s} {'wgrad':10s} {ms:7.3f} ms  {2.0 * 256 * M * 256 / ms / 1e9:7.1f} TF/s", flush=True)
    del a, b
    torch.cuda.empty_cache()
