"""GPT-2 LM-head GEMMs (131 072 tokens x 50 432 vocab x 768) under the ping-pong kernel's tile orders
(``gpp_order_config``) against hipBLASLt with the bench's TunableOp table:

* forward logits = h W^T: library (``torch.mm``) vs the persistent ping-pong kernel at gm 0 / 2 / 4 / 8 / 16;
* weight gradient dW += dlogits^T h: the ``ppt`` route (split-K ping-pong kernel on h^T) at the same orders.

    python benchmarks/head_tile_order.py [--tokens 131072]

One JSON line per case: median ms of interleaved repetitions and TF/s.
"""
import argparse
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from bpe_transformer.ops._ext import ops  # noqa: E402
from bpe_transformer.ops.gemm import choose_splits_pp  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tokens", type=int, default=131072)
    ap.add_argument("--orders", default="0,2,4,8,16")
    a = ap.parse_args()
    import torch.cuda.tunable as tunable

    table = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "bpe_transformer", "ops",
                         "tuning", "gpt2-small_b128_s1024.csv")
    tunable.enable(True)
    tunable.tuning_enable(False)
    tunable.record_untuned_enable(False)
    tunable.read_file(table)
    h = ops()
    T, V, d = a.tokens, 50432, 768
    orders = [int(x) for x in a.orders.split(",")]
    torch.manual_seed(0)
    x = torch.randn(T, d, device="cuda", dtype=torch.bfloat16)
    w = (0.05 * torch.randn(V, d, device="cuda")).to(torch.bfloat16)
    logits = torch.empty(T, V, device="cuda", dtype=torch.bfloat16)
    xt = h.transpose_bf16(x)
    g = torch.zeros(V, d, device="cuda", dtype=torch.bfloat16)
    sp = choose_splits_pp(V, d, T)
    flop = 2.0 * T * V * d
    arms = {"fwd_lib": lambda: torch.mm(x, w.t(), out=logits)}
    for o in orders:
        arms[f"fwd_pp_gm{o}"] = (lambda o=o: (h.gpp_order_config(o), h.gemm_pp(x, True, w, True, logits, 0.0, 1)))
    for o in orders:
        arms[f"dw_ppt_gm{o}"] = (lambda o=o: (h.gpp_order_config(o), h.gemm_pp(logits, False, xt, True, g, 0.0, sp)))
    prev = h.gpp_order_config(-1)
    for fn in arms.values():  # warm
        fn()
    torch.cuda.synchronize()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    times = {n: [] for n in arms}
    for _ in range(5):
        for name, fn in arms.items():
            fn()
            ev[0].record()
            for _ in range(2):
                fn()
            ev[1].record()
            torch.cuda.synchronize()
            times[name].append(ev[0].elapsed_time(ev[1]) / 2)
    h.gpp_order_config(prev)
    for name in arms:
        ms = statistics.median(times[name])
        print(json.dumps({"case": name, "tokens": T, "splits": sp if name.startswith("dw") else 1, "ms": round(ms, 4),
                          "tflops": round(flop / ms / 1e9, 1)}), flush=True)


if __name__ == "__main__":
    main()
