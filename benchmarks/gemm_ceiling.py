"""hipBLASLt (torch.matmul) bf16 TF/s on large square shapes vs the GPT-2 B128 projection shapes.

Calibrates the practical GEMM ceiling of the chip under sustained load (DVFS included): random N(0,1)
operands, 3 warmup + 10 timed calls per shape, HIP events.  One JSON line per shape.
"""
import json

import torch


def tflops(m, n, k, iters=10):
    a = torch.randn(m, k, device="cuda", dtype=torch.bfloat16)
    b = torch.randn(n, k, device="cuda", dtype=torch.bfloat16)
    for _ in range(3):
        torch.matmul(a, b.t())
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        torch.matmul(a, b.t())
    e.record()
    torch.cuda.synchronize()
    ms = s.elapsed_time(e) / iters
    return ms, 2 * m * n * k / ms / 1e9


if __name__ == "__main__":
    shapes = [(8192, 8192, 8192), (16384, 16384, 16384), (16384, 16384, 4096), (131072, 2304, 768),
              (131072, 4096, 768), (131072, 768, 2048), (131072, 50432, 768), (32768, 8192, 8192)]
    for m, n, k in shapes:
        ms, tf = tflops(m, n, k)
        print(json.dumps({"m": m, "n": n, "k": k, "ms": round(ms, 3), "tflops": round(tf, 1)}), flush=True)
