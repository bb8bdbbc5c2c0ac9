"""The full training loop on one MI355X: bf16 fused blocks, eval, JSONL metrics, checkpoint and resume.

The CPU trainer tests (tests/test_trainer.py) cover the loop logic in fp32; this runs the same loop through the
HIP path, where the state that must survive a checkpoint is the bf16 weights, the fp32 master, both moments
and the device step counter.  The resumed state must equal the checkpoint exactly.
"""

from __future__ import annotations

import json

import numpy as np
import pytest
import torch

from bpe_transformer.models.config import ModelConfig
from bpe_transformer.train.config import TrainConfig
from bpe_transformer.train.trainer import Trainer

pytestmark = pytest.mark.gpu


def _cfg(tmp_path, **kw):
    model = ModelConfig(vocab_size=512, context_length=128, d_model=256, num_layers=2, num_heads=4, d_ff=512)
    cfg = TrainConfig(model=model, batch_size=4, max_iters=8, device="cuda", log_every=2, eval_every=4,
                      eval_iters=2, ckpt_dir=str(tmp_path / "ck"), metrics_path=str(tmp_path / "m.jsonl"))
    cfg.optim.warmup_iters = 2
    cfg.optim.lr = 2e-3
    cfg.data.synthetic_tokens = 50_000
    for k, v in kw.items():
        setattr(cfg, k, v)
    return cfg


def test_trainer_gpu_loop_checkpoint_resume(gpu_device, tmp_path):
    from bpe_transformer.data import write_tokens

    rng = np.random.default_rng(0)
    write_tokens(rng.integers(0, 512, 40_000), tmp_path / "val.bin", vocab_size=512)
    cfg = _cfg(tmp_path, ckpt_every=4)
    cfg.data.val_path = str(tmp_path / "val.bin")
    cfg.data.vocab_size_for_dtype = 512
    full = Trainer(cfg)
    assert full.dtype == torch.bfloat16 and full.engine.flat.data.is_cuda
    out = full.fit()
    assert np.isfinite(out["final_loss"])
    recs = [json.loads(line) for line in open(tmp_path / "m.jsonl")]
    assert any("val_loss" in r and np.isfinite(r["val_loss"]) for r in recs)
    assert all(r["tokens_per_s"] > 0 for r in recs if "tokens_per_s" in r)
    ck = tmp_path / "ck" / "ckpt_00000004.pt"
    saved = torch.load(ck, weights_only=True)
    assert saved["optimizer"]["step"] == 4

    cfg2 = _cfg(tmp_path, resume=str(ck))
    cfg2.data.val_path = cfg.data.val_path
    cfg2.data.vocab_size_for_dtype = 512
    resumed = Trainer(cfg2)
    assert resumed.start_iter == 4
    assert resumed.engine.opt.step_count == 4
    torch.testing.assert_close(resumed.engine.opt.master.cpu(), saved["optimizer"]["master"].cpu())
    assert torch.equal(resumed.engine.flat.data.cpu(), resumed.engine.opt.master.to(torch.bfloat16).cpu())
    out2 = resumed.fit()
    # the loader re-seeds at the resume point (trainer._resume), so the two runs see different batches after
    # step 4: compare update counts and health, not weights
    assert np.isfinite(out2["final_loss"])
    assert resumed.engine.opt.step_count == full.engine.opt.step_count == 8
