"""Library bf16 GEMM ceiling on this GPU for reference shapes (hipBLASLt via torch.mm):
what a plain MFMA GEMM reaches at K=768 / K=1024 vs the filter kernel."""
import torch

def t(m, n, k, reps=20):
    a = torch.randn(m, k, device="cuda", dtype=torch.bfloat16)
    b = torch.randn(n, k, device="cuda", dtype=torch.bfloat16)
    for _ in range(3):
        c = a @ b.T
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record()
    for _ in range(reps):
        c = a @ b.T
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / reps
    tf = 2 * m * n * k / ms / 1e9
    print(f"m={m} n={n} k={k}: {ms:.3f} ms  {tf:.1f} TF/s  frac {tf/2500:.3f}  (out {m*n*2/1e9:.2f} GB)", flush=True)

for shape in [(8192, 8192, 8192), (16384, 16384, 8192), (10240, 65536, 768), (10240, 131072, 768), (4096, 262144, 768),
              (10240, 65536, 1024)]:
    t(*shape)
