"""Timing diagnostics of the 4-wave GEMM (variant build ``python -m bpe_transformer.ops.build --variant w4diag -D
BPE_W4_DIAG``, run with ``BPE_HIP_VARIANT=w4diag``): the kernel with pieces of its main loop removed (numerically
wrong), interleaved in one process.  0 full, 1 no in-loop DMA, 2 no fragment reads, 3 no MFMAs, 4 no waits/barriers, 5 DMA never waited
for, 6 DMA as one burst per section.
"""
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from bpe_transformer.ops._ext import ops  # noqa: E402


def timeit(fn, iters=10):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters


def main():
    h = ops()
    bf = dict(device="cuda", dtype=torch.bfloat16)
    shapes = [("square 8192", 8192, 8192, 8192), ("gpt2 qkv", 131072, 2304, 768), ("gpt2 w13", 131072, 4096, 768),
              ("llama w2", 65536, 2048, 5632)]
    for name, M, N, K in shapes:
        a = torch.randn(M, K, **bf)
        b = torch.randn(N, K, **bf)
        c = torch.empty(M, N, **bf)
        t = {d: [] for d in range(7)}
        for d in range(7):
            os.environ["BPE_W4_DIAG"] = str(d)
            h.gemm_w4(a, True, b, True, c, 0.0)
        torch.cuda.synchronize()
        for _ in range(7):
            for d in range(7):
                os.environ["BPE_W4_DIAG"] = str(d)
                t[d].append(timeit(lambda: h.gemm_w4(a, True, b, True, c, 0.0)))
        f = 2.0 * M * N * K
        print(json.dumps({"shape": name, **{f"diag{d}_ms": round(statistics.median(v), 4) for d, v in t.items()},
                          **{f"diag{d}_tf": round(f / statistics.median(v) / 1e9, 1) for d, v in t.items()}}),
              flush=True)


if __name__ == "__main__":
    main()
