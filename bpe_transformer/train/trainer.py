"""Training loop: data -> model -> kernels -> optimizer -> DP -> metrics -> checkpoint.

One process per GPU (``torchrun``); single-process runs work unchanged on a
GPU or the CPU (the TinyStories ~17M plumbing config of BASELINE.json).

Failure handling:
  * non-finite gradient norm -> the AdamW kernel skips the step on the device
    (no host sync); the loss is checked on the host at every log step and the
    run aborts after ``max_nonfinite`` consecutive non-finite checks;
  * a hung RCCL collective times out (``init_distributed(timeout_s=...)``);
  * checkpoints are written atomically by rank 0, every ``ckpt_every`` steps,
    and ``resume="latest"`` restarts from the newest one (model, optimizer
    state incl. fp32 master weights, iteration, RNG seeds).
"""

from __future__ import annotations

import math
import time
from pathlib import Path

import numpy as np
import torch

from ..data import BatchLoader, load_tokens, synthetic_tokens
from ..models import TransformerLM
from ..optim.schedule import CosineSchedule
from ..parallel import all_reduce_mean_, barrier, init_distributed
from ..utils.checkpoint import latest_checkpoint, read_checkpoint, save_checkpoint
from ..utils.metrics import MetricsLogger, device_memory_gb, log, setup_logging
from ..utils.profiling import MI355X_BF16_DENSE_FLOPS, torch_profile
from .config import TrainConfig
from .engine import TrainEngine


class _EngineOptimizerView:
    """Adapter so :func:`save_checkpoint` can call ``optimizer.state_dict()`` on the engine."""

    def __init__(self, engine: TrainEngine):
        self.engine = engine

    def state_dict(self):
        return self.engine.state_dict()


class Trainer:
    def __init__(self, cfg: TrainConfig):
        self.cfg = cfg
        want = cfg.device if cfg.device != "auto" else ("cuda" if torch.cuda.is_available() else "cpu")
        self.info = init_distributed(want)
        setup_logging(self.info.rank)
        dev = self.info.device
        if cfg.dtype == "auto":
            dtype = torch.bfloat16 if dev.type == "cuda" else torch.float32
        else:
            dtype = {"bf16": torch.bfloat16, "fp32": torch.float32}[cfg.dtype]
        self.dtype = dtype
        torch.manual_seed(cfg.seed)  # identical init everywhere; rank 0 is broadcast anyway
        self.model = TransformerLM.from_config(cfg.model, device=dev, dtype=dtype)
        if cfg.precision == "fp8":
            if dev.type != "cuda":
                raise ValueError("precision=fp8 needs the GPU path (MI355X fp8 MFMA)")
            self.model.enable_fp8()
        if cfg.lm_head_mode not in ("logits", "streamed"):
            raise ValueError(f"lm_head_mode must be 'logits' or 'streamed', got {cfg.lm_head_mode!r}")
        self.model.lm_head_mode = cfg.lm_head_mode
        self.model.lm_head_chunk = cfg.lm_head_chunk or None
        o = cfg.optim
        self.engine = TrainEngine(self.model, self.info, lr=o.lr, betas=o.betas, eps=o.eps,
                                  weight_decay=o.weight_decay, max_grad_norm=o.max_grad_norm,
                                  bucket_mb=cfg.bucket_mb, time_phases=cfg.phase_timing,
                                  ddp_check_every=cfg.ddp_check_every, zero=cfg.zero,
                                  grad_dtype=cfg.resolved_grad_dtype(next(self.model.parameters()).dtype),
                                  comm_dtype=cfg.resolved_comm_dtype())
        self.schedule = CosineSchedule(o.lr, o.min_lr, o.warmup_iters, o.cosine_cycle_iters or cfg.max_iters)
        ctx = cfg.model.context_length
        if cfg.data.train_path:
            train = load_tokens(cfg.data.train_path, cfg.data.vocab_size_for_dtype)
        else:
            train = synthetic_tokens(cfg.model.vocab_size, cfg.data.synthetic_tokens, seed=cfg.seed)
        self.val = load_tokens(cfg.data.val_path, cfg.data.vocab_size_for_dtype) if cfg.data.val_path else None
        self.train_data = train
        self.loader = BatchLoader(train, cfg.batch_size, ctx, dev, seed=cfg.seed + 1000 * self.info.rank)
        self.metrics = MetricsLogger(cfg.metrics_path, self.info.rank)
        self.start_iter = 0
        if cfg.resume:
            self._resume(cfg.resume)
        n = sum(p.numel() for p in self.model.parameters())
        log.info(f"model {n / 1e6:.1f}M params | dtype {dtype} | world {self.info.world_size} | device {dev}")

    # ------------------------------------------------------------------ checkpoint
    def _ckpt_path(self, it: int) -> Path:
        return Path(self.cfg.ckpt_dir) / f"ckpt_{it:08d}.pt"

    def save(self, it: int) -> None:
        # sharded DP: every rank joins the collectives that make the weights and the full optimizer state
        # current on rank 0 (no-ops otherwise)
        self.engine.sync_params()
        self.engine.gather_optimizer_state()
        extra = {"rng": {"torch": torch.get_rng_state(),
                         "cuda": torch.cuda.get_rng_state_all() if torch.cuda.is_available() else []}}
        if self.model.fp8_state is not None:
            extra["fp8"] = [st.state_dict() for st in self.model.fp8_states()]
        save_checkpoint(self.model, _EngineOptimizerView(self.engine), it, self._ckpt_path(it), rank=self.info.rank,
                        config=self.cfg.to_dict(), **extra)

    def _resume(self, spec: str) -> None:
        path = latest_checkpoint(self.cfg.ckpt_dir) if spec == "latest" else Path(spec)
        if path is None:
            log.info("resume: no checkpoint found, starting fresh")
            return
        obj = read_checkpoint(path, map_location=self.info.device)
        with torch.no_grad():
            self.model.load_state_dict(obj["model"])
        self.engine.load_state_dict(obj["optimizer"])
        if self.model.fp8_state is not None and "fp8" in obj:
            for st, sd in zip(self.model.fp8_states(), obj["fp8"]):
                st.load_state_dict(sd)
        rng = obj.get("rng")
        if rng is not None:
            torch.set_rng_state(rng["torch"].cpu())
            if torch.cuda.is_available() and len(rng["cuda"]) == torch.cuda.device_count():
                torch.cuda.set_rng_state_all([t.cpu() for t in rng["cuda"]])
        self.start_iter = int(obj["iteration"])
        # the prefetching loader runs ahead of the step counter, so its generator state is not checkpointed;
        # a resumed run draws a fresh, deterministic stream keyed by (seed, rank, resume iteration)
        self.loader.close()
        self.loader = BatchLoader(self.train_data, self.cfg.batch_size, self.cfg.model.context_length, self.info.device,
                                  seed=self.cfg.seed + 1000 * self.info.rank + 7919 * self.start_iter)
        log.info(f"resumed from {path} at iteration {self.start_iter}")

    # ------------------------------------------------------------------ eval
    @torch.no_grad()
    def evaluate(self) -> float:
        data = self.val
        if data is None:
            return float("nan")
        self.model.eval()
        rng = np.random.default_rng(self.cfg.seed + 7)
        from ..data import get_batch

        tot = torch.zeros((), device=self.info.device)
        self.engine.sync_params()
        for _ in range(self.cfg.eval_iters):
            x, y = get_batch(data, self.cfg.batch_size, self.cfg.model.context_length, self.info.device, rng)
            tot += self.model.loss(x, y).float()
        tot /= self.cfg.eval_iters
        all_reduce_mean_(tot)
        self.model.train()
        return float(tot.item())

    # ------------------------------------------------------------------ loop
    def fit(self) -> dict:
        cfg = self.cfg
        tok_per_step = cfg.batch_size * cfg.grad_accum * cfg.model.context_length * self.info.world_size
        flops_tok = cfg.model.train_flops_per_token()
        last_t = time.perf_counter()
        last_it = self.start_iter
        bad = 0
        loss_v = float("nan")
        prof_cm = torch_profile(Path(cfg.ckpt_dir) / "profile") if cfg.profile else None
        prof = prof_cm.__enter__() if prof_cm else None
        try:
            routes_logged = False
            for it in range(self.start_iter, cfg.max_iters):
                lr = self.schedule(it)
                batches = [next(self.loader) for _ in range(cfg.grad_accum)]
                loss = self.engine.train_step(batches, lr)
                if prof is not None:
                    prof.step()
                step = it + 1
                if step % cfg.log_every == 0 or step == cfg.max_iters:
                    lt = loss.detach().float().clone()
                    all_reduce_mean_(lt)
                    loss_v = float(lt.item())
                    now = time.perf_counter()
                    dt = (now - last_t) / max(step - last_it, 1)
                    last_t, last_it = now, step
                    gn = self.engine.last_grad_norm
                    gn_v = float(gn.item()) if gn is not None else float("nan")
                    tps = tok_per_step / dt
                    self.metrics.log(step=step, loss=loss_v, lr=lr, grad_norm=gn_v, ms_per_step=1000 * dt,
                                     tokens_per_s=tps,
                                     mfu=tps * flops_tok / (MI355X_BF16_DENSE_FLOPS * self.info.world_size),
                                     mem_gb=device_memory_gb(), **self.engine.phase_times())
                    if not routes_logged and self.engine.flat.data.is_cuda:
                        from ..ops.gemm import routes_summary

                        self.metrics.log(step=step, dw_gemm_routes=routes_summary())  # kernel per dW shape
                        routes_logged = True
                    if cfg.nan_guard and not math.isfinite(loss_v):
                        bad += 1
                        log.warning(f"non-finite loss at step {step} ({bad} consecutive)")
                        if bad >= 3:
                            raise FloatingPointError("loss diverged (3 consecutive non-finite checks)")
                    else:
                        bad = 0
                if cfg.eval_every and step % cfg.eval_every == 0:
                    self.metrics.log(step=step, val_loss=self.evaluate())
                if cfg.ckpt_every and step % cfg.ckpt_every == 0:
                    self.save(step)
        finally:
            if prof_cm is not None:
                prof_cm.__exit__(None, None, None)
            self.loader.close()
            self.metrics.close()
        barrier()
        return {"final_loss": loss_v, "iterations": cfg.max_iters}
