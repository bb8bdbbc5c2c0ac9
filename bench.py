#!/usr/bin/env python3
"""Headline benchmark: GPT-2-small-shape LM training throughput on MI355X.

Metric (BASELINE.json): "training tokens/sec (whole node), GPT-2-small config
at 1/2/4/8 MI355X".  Model: 12 layers, d_model 768, 12 heads, SwiGLU d_ff 2048,
RoPE, RMSNorm, vocab 50257, seq 1024, bf16 compute with fp32 master weights
and fp32 optimizer state; random-init weights, synthetic uniform token data.
Every timed step is a full training step: forward, fused LM-head+CE,
backward, RCCL bucketed all-reduce (N>1), global-norm clip, AdamW update.

    python bench.py --gpus 1 --steps 20 --warmup 5
    python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 \
        --master-port 29511 bench.py --gpus 8 --steps 20 --warmup 5

Weak scaling: the per-GPU micro-batch is fixed, global batch = N * micro-batch.
Rank 0 prints one JSON line; the time is the MAX over ranks of K steps
bracketed by barrier + device synchronize.
"""

from __future__ import annotations

import argparse
import json
import os
import sys
import time

os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")

import torch  # noqa: E402

METRIC = "training tokens/sec (whole node), GPT-2-small config at 1/2/4/8 MI355X"
TUNING_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "bpe_transformer", "ops", "tuning")


# per-GPU micro-batch when --batch is not given: GPT-2-small 128 sequences; Llama-1.1B 65 536 tokens (32 x 2048,
# 16 x 4096: +5-6 % over 16 384 tokens, ~110 GB of the 288 GB HBM; profiles/bench/ab_llama_microbatch_65k_tokens.log)
DEFAULT_BATCH = {"gpt2-small": 128}
DEFAULT_TOKENS = {"llama-1.1b": 65536}


def load_gemm_tuning(spec: str, model: str, batch: int, seq: int) -> str | None:
    """Point PyTorch's TunableOp at a pre-measured hipBLASLt/rocBLAS solution table (no tuning at run time).

    The tables in ``bpe_transformer/ops/tuning`` were produced on MI355X by running this benchmark with
    ``PYTORCH_TUNABLEOP_TUNING=1``; they only choose among the libraries' own GEMM solutions.
    """
    if spec == "off":
        return None
    path = spec
    if spec == "auto":
        path = os.path.join(TUNING_DIR, f"{model}_b{batch}_s{seq}.csv")
    if not os.path.exists(path):
        return None
    import torch.cuda.tunable as tunable

    tunable.enable(True)
    tunable.tuning_enable(False)
    tunable.record_untuned_enable(False)
    tunable.read_file(path)
    return os.path.basename(path)


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--batch", type=int, default=None,
                    help="per-GPU micro-batch (sequences); default per model: gpt2-small 128 (128 x 1024 tokens "
                         "uses a fraction of the 288 GB HBM and runs ~2 percent faster than 64; library GEMM tables "
                         "for both in ops/tuning), llama-1.1b 65536 tokens (32 x 2048, 16 x 4096), otherwise 8")
    ap.add_argument("--seq", type=int, default=1024)
    ap.add_argument("--model", default="gpt2-small")
    ap.add_argument("--bucket-mb", type=float, default=64.0)
    ap.add_argument("--zero", type=int, choices=[0, 1], default=0,
                    help="1 = sharded data parallelism (reduce-scatter gradients, AdamW on 1/N of the parameters, "
                         "weight all-gather overlapped with the next forward; parallel/zero.py); N>1 only")
    ap.add_argument("--gemm-tuning", default="auto",
                    help="hipBLASLt/rocBLAS solution table (TunableOp CSV) for the library GEMMs; 'auto' = the "
                         "shipped table for this model/batch if present, 'off' = library heuristics")
    ap.add_argument("--precision", choices=["bf16", "fp8"], default="bf16",
                    help="fp8 = block projections' forward GEMMs in e4m3fn with delayed scaling (bf16 backward)")
    ap.add_argument("--grad-dtype", choices=["bf16", "fp32"], default="bf16",
                    help="flat gradient buffer dtype (fp32: weight gradients written unrounded through the dW "
                         "kernels' fp32 slab; the default bf16 is the measured-faster form for one micro-batch)")
    ap.add_argument("--comm-dtype", choices=["auto", "bf16", "fp32"], default="auto",
                    help="data-parallel all-reduce dtype (auto = the gradient dtype; fp32 with bf16 gradients "
                         "sums across ranks without a bf16 rounding per ring hop)")
    ap.add_argument("--lm-head-mode", choices=["logits", "streamed"], default="logits",
                    help="LM head + CE: one [tokens, vocab] logits buffer (default) or streamed token chunks with "
                         "dh / dW formed in the forward (no full logits; ops/loss.py)")
    ap.add_argument("--lm-head-chunk", type=int, default=0, help="token rows per chunk (0 = the mode's default)")
    ap.add_argument("--device", choices=["cuda", "cpu"], default="cuda",
                    help="cpu = the plumbing config path (fp32, no HIP kernels), e.g. --model tinystories-17m --seq 256")
    ap.add_argument("--json-out", default=None)
    ap.add_argument("--no-dp-check", action="store_true",
                    help="N>1: skip the untimed replica-consistency step after warmup (default: run it)")
    ap.add_argument("--debug-corrupt-rank", type=int, default=-1,
                    help=argparse.SUPPRESS)  # tests: perturb this rank's weights before the consistency step
    args = ap.parse_args()
    if args.batch is None:
        if args.model in DEFAULT_TOKENS:
            args.batch = max(1, DEFAULT_TOKENS[args.model] // args.seq)
        else:
            args.batch = DEFAULT_BATCH.get(args.model, 8)

    from bpe_transformer.data import synthetic_tokens
    from bpe_transformer.models import TransformerLM, get_preset
    from bpe_transformer.parallel import all_reduce_max, barrier, cleanup, init_distributed
    from bpe_transformer.train.engine import TrainEngine

    info = init_distributed(args.device)
    on_gpu = info.device.type == "cuda"
    sync = torch.cuda.synchronize if on_gpu else (lambda: None)
    tuning = load_gemm_tuning(args.gemm_tuning, args.model, args.batch, args.seq)
    if args.gpus != info.world_size:
        print(f"warning: --gpus {args.gpus} but WORLD_SIZE={info.world_size}", file=sys.stderr)
    dev = info.device
    torch.manual_seed(1234)  # identical init on every rank (rank-0 broadcast also enforces it)
    cfg = get_preset(args.model, context_length=args.seq)
    dtype = torch.bfloat16 if on_gpu else torch.float32
    model = TransformerLM.from_config(cfg, device=dev, dtype=dtype)
    if args.precision == "fp8":
        model.enable_fp8()
    model.lm_head_mode, model.lm_head_chunk = args.lm_head_mode, args.lm_head_chunk or None
    # phase timing: device events around forward / backward / exposed collective wait / clip + AdamW, read once
    # after the timed loop (stderr; the driver's scaling run then shows how much all-reduce stays exposed)
    gdt = {"bf16": torch.bfloat16, "fp32": torch.float32}[args.grad_dtype] if on_gpu else None
    cdt = None if args.comm_dtype == "auto" else {"bf16": torch.bfloat16, "fp32": torch.float32}[args.comm_dtype]
    engine = TrainEngine(model, info, lr=3e-4, weight_decay=0.1, max_grad_norm=1.0, bucket_mb=args.bucket_mb,
                         zero=args.zero, time_phases=on_gpu, grad_dtype=gdt, comm_dtype=cdt)

    # synthetic token stream, different per rank; batches staged on the device up front
    data = synthetic_tokens(cfg.vocab_size, args.batch * (args.seq + 1) * 8, seed=1000 + info.rank)
    data_t = torch.from_numpy(data.astype("int64")).to(dev)
    nwin = len(data) // (args.seq + 1)

    def batch(i: int):
        j = (i * args.batch) % (nwin - args.batch)
        w = data_t[j * (args.seq + 1) : (j + args.batch) * (args.seq + 1)].view(args.batch, args.seq + 1)
        return [(w[:, :-1].contiguous(), w[:, 1:].contiguous())]

    for i in range(args.warmup):
        engine.train_step(batch(i))
    # N > 1: one more untimed step with the replica-consistency detector on (parallel/ddp.py check_consistency):
    # per-bucket fp64 checksums of the all-reduced gradients and of the updated weights compared across ranks; a
    # mismatch raises, so the first multi-GPU record can only be written by replicas that stayed bit-identical
    dp_check = None
    if engine.ddp is not None and not args.no_dp_check:
        if args.debug_corrupt_rank == info.rank:
            with torch.no_grad():
                engine.flat.data[:64].add_(1.0)
        prev_every = engine.ddp_check_every
        engine.ddp_check_every = 1
        engine.train_step(batch(args.warmup))
        sync()
        engine.ddp_check_every = prev_every
        dp_check = "grad+data bit-identical across ranks" if not engine.zero else "data bit-identical across ranks"
    sync()
    engine.phase_times()  # drop the warmup steps' events
    if on_gpu:
        torch.cuda.reset_peak_memory_stats(dev)
    barrier()
    sync()
    t0 = time.perf_counter()
    loss = None
    for i in range(args.steps):
        loss = engine.train_step(batch(args.warmup + i))
    sync()
    barrier()
    sync()
    dt = time.perf_counter() - t0
    dt = all_reduce_max(dt, dev)
    phases = {k: round(all_reduce_max(v, dev), 3) for k, v in sorted(engine.phase_times().items())}
    loss_v = float(loss.item()) if loss is not None else float("nan")

    n = info.world_size
    tokens = args.steps * args.batch * args.seq * n
    value = tokens / dt
    flops_tok = cfg.train_flops_per_token(args.seq)
    out = {
        # the headline metric names the GPT-2-small config; other models report under their own name
        "metric": METRIC if args.model == "gpt2-small" else f"training tokens/sec (whole node), {args.model}",
        "value": round(value, 1),
        "unit": "tokens/s",
        "n_gpus": n,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(dt / args.steps * 1000.0, 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": ("bf16" if args.precision == "bf16" else "fp8(e4m3 fwd GEMMs)+bf16") if on_gpu else "fp32",
        "data": "synthetic (uniform random tokens, random-init weights)",
        "config": {
            "model": f"{args.model} ({cfg.num_layers}L/{cfg.d_model}d/{cfg.num_heads}H, RoPE+SwiGLU+RMSNorm, "
                     f"vocab {cfg.vocab_size})",
            "global_batch": args.batch * n,
            "seq_len": args.seq,
            "parallelism": f"dp{n}" + ("-zero1" if engine.zero else ""),
            "micro_batch_per_gpu": args.batch,
        },
        "mfu_bf16_dense_2.5PF": round(value / n * flops_tok / 2.5e15, 4),
        "final_loss": round(loss_v, 4),
        "gemm_tuning": tuning,
        "grad_dtype": str(engine.flat.grad.dtype).replace("torch.", ""),
        "lm_head_mode": args.lm_head_mode,
        "allreduce_dtype": (str(engine.ddp.comm_dtype if hasattr(engine.ddp, "comm_dtype") else
                                engine.flat.grad.dtype).replace("torch.", "") if engine.ddp is not None else None),
    }
    if engine.ddp is not None:
        import torch.distributed as dist

        bk = engine.ddp.buckets
        esz = engine.flat.grad.element_size()
        out["dist"] = {
            "world_size": dist.get_world_size(),
            "backend": dist.get_backend(),
            "collective": "reduce-scatter + all-gather (ZeRO-1)" if engine.zero else "all-reduce (AVG)",
            "buckets": len(bk),
            "bucket_mb": [round((e - s_) * esz / 2**20, 2) for s_, e in bk],
            "comm_dtype": str(getattr(engine.ddp, "comm_dtype", engine.flat.grad.dtype)).replace("torch.", ""),
            "consistency_check": dp_check,
        }
    if phases:
        out["phases_ms"] = phases  # max over ranks; comm_ms = the all-reduce wait left exposed after the backward
        out["comm_ms"] = phases.get("comm_ms")
    if on_gpu:
        # peak HBM allocated by PyTorch's caching allocator over the timed steps (max over ranks), and reserved
        out["peak_mem_gb"] = round(all_reduce_max(torch.cuda.max_memory_allocated(dev) / 1e9, dev), 2)
        out["peak_reserved_gb"] = round(all_reduce_max(torch.cuda.max_memory_reserved(dev) / 1e9, dev), 2)
        from bpe_transformer.ops import gemm as _gemm

        out["dw_gemm_routes"] = _gemm.routes_summary()  # weight-gradient kernel per shape (ops/tuning/dw_routes.json)
        out["dw_gemm_groups"] = _gemm.groups_summary()  # grouped dW launches: shapes -> split count
    if info.is_main:
        if phases:  # max over ranks of each phase's mean ms per step (comm_ms = exposed collective wait)
            print(json.dumps({"phases_ms_per_step_max_over_ranks": phases}), file=sys.stderr, flush=True)
        line = json.dumps(out)
        print(line, flush=True)
        if args.json_out:
            with open(args.json_out, "w") as f:
                f.write(line + "\n")
    cleanup()
    return 0


if __name__ == "__main__":
    sys.exit(main())
