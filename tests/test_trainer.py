"""Trainer loop, config/CLI, checkpoint-resume and failure guards (CPU)."""

from __future__ import annotations

import json

import numpy as np
import pytest
import torch

from bpe_transformer.models import get_preset
from bpe_transformer.train.__main__ import main as cli_main
from bpe_transformer.train.config import TrainConfig, apply_overrides
from bpe_transformer.train.trainer import Trainer


def _cfg(tmp_path, **kw):
    cfg = TrainConfig(model=get_preset("ts-tests", vocab_size=256, context_length=16), batch_size=4, max_iters=12,
                      device="cpu", log_every=4, ckpt_dir=str(tmp_path / "ck"),
                      metrics_path=str(tmp_path / "m.jsonl"))
    cfg.optim.warmup_iters = 2
    cfg.optim.lr = 3e-3
    cfg.data.synthetic_tokens = 20_000
    for k, v in kw.items():
        setattr(cfg, k, v)
    return cfg


def test_trainer_runs_and_logs(tmp_path):
    out = Trainer(_cfg(tmp_path)).fit()
    assert np.isfinite(out["final_loss"])
    recs = [json.loads(line) for line in open(tmp_path / "m.jsonl")]
    assert [r["step"] for r in recs] == [4, 8, 12]
    assert all(r["tokens_per_s"] > 0 for r in recs)


def test_trainer_learns_real_tokens(tmp_path):
    from bpe_transformer import train_bpe
    from bpe_transformer.data import write_tokens
    from bpe_transformer.tokenization import BPETokenizer

    from .conftest import FIXTURES

    vocab, merges = train_bpe(FIXTURES / "tinystories_sample.txt", 300, ["<|endoftext|>"])
    tok = BPETokenizer(vocab, merges, ["<|endoftext|>"])
    ids = tok.encode_file(FIXTURES / "tinystories_sample.txt", 2)
    write_tokens(np.tile(ids, 5), tmp_path / "train.bin", vocab_size=300)
    cfg = _cfg(tmp_path, max_iters=40, log_every=20)
    cfg.model = get_preset("ts-tests", vocab_size=300, context_length=16)
    cfg.data.train_path = str(tmp_path / "train.bin")
    cfg.data.val_path = str(tmp_path / "train.bin")
    cfg.data.vocab_size_for_dtype = 300
    tr = Trainer(cfg)
    before = tr.evaluate()
    tr.fit()
    assert tr.evaluate() < before - 0.5


def test_checkpoint_resume_is_exact(tmp_path):
    full = Trainer(_cfg(tmp_path / "a", max_iters=8, ckpt_every=4))
    full.fit()
    resumed = Trainer(_cfg(tmp_path / "a", max_iters=8, resume=str(tmp_path / "a" / "ck" / "ckpt_00000004.pt")))
    assert resumed.start_iter == 4
    torch.testing.assert_close(resumed.engine.opt.master, torch.load(
        tmp_path / "a" / "ck" / "ckpt_00000004.pt", weights_only=True)["optimizer"]["master"])


def test_nonfinite_grad_skips_update():
    from bpe_transformer.optim import FlatAdamW, FlatParameters

    lin = torch.nn.Linear(4, 4)
    flat = FlatParameters.from_module(lin)
    opt = FlatAdamW(flat, lr=1e-2)
    before = flat.data.clone()
    flat.grad.fill_(float("nan"))
    _, coef = opt.clip_grad_norm(1.0)
    opt.step(grad_scale=coef)
    assert torch.equal(flat.data, before)


def _flat_opt_run(device, skip_at=None, steps=4, wd=0.1):
    from bpe_transformer.optim import FlatAdamW, FlatParameters

    torch.manual_seed(0)
    lin = torch.nn.Linear(8, 8).to(device)
    flat = FlatParameters.from_module(lin)
    opt = FlatAdamW(flat, lr=1e-2, weight_decay=wd)
    g = torch.Generator().manual_seed(3)
    grads = [torch.randn(flat.numel, generator=g).to(device) for _ in range(steps)]
    it = iter(grads)
    for i in range(steps + (skip_at is not None)):
        if i == skip_at:
            flat.grad.fill_(float("inf"))
        else:
            flat.grad.copy_(next(it))
        _, coef = opt.clip_grad_norm(1e9)
        opt.step(grad_scale=coef)
    return opt, flat


def test_skipped_step_does_not_advance_bias_correction():
    """A non-finite step is skipped WITHOUT counting: the updates after it equal a run that never saw it, and the
    checkpointed step is the number of applied updates (bias correction drifted on skipped steps)."""
    ref, fref = _flat_opt_run("cpu")
    opt, flat = _flat_opt_run("cpu", skip_at=2)
    assert opt.calls == 5 and opt.step_count == 4 and opt.state_dict()["step"] == 4
    torch.testing.assert_close(flat.data, fref.data, rtol=0, atol=0)


def test_load_state_dict_rebuilds_weight_decay_segments():
    from bpe_transformer.optim import FlatAdamW, FlatParameters

    lin = torch.nn.Linear(4, 4)
    flat = FlatParameters.from_module(lin)
    src = FlatAdamW(flat, lr=1e-2, weight_decay=0.3)
    dst = FlatAdamW(flat, lr=1e-2, weight_decay=0.0)
    dst.load_state_dict(src.state_dict())
    assert dst.weight_decay == 0.3
    assert {wd for _, _, wd in dst.segments} == {0.3, 0.0}  # weight decayed, bias not
    assert dst.segments == src.segments


def test_config_overrides_and_cli(tmp_path, capsys):
    cfg = apply_overrides(TrainConfig(), ["optim.lr=0.01", "batch_size=3", "model.num_layers=1"])
    assert cfg.optim.lr == 0.01 and cfg.batch_size == 3 and cfg.model.num_layers == 1
    with pytest.raises(KeyError):
        apply_overrides(TrainConfig(), ["nope=1"])
    assert cli_main(["--preset", "gpt2-small", "--print-config"]) == 0
    assert json.loads(capsys.readouterr().out)["model"]["d_model"] == 768
    rc = cli_main(["--preset", "ts-tests", "device=cpu", "max_iters=2", "batch_size=2", "log_every=1",
                   "model.vocab_size=128", f"ckpt_dir={tmp_path}", "data.synthetic_tokens=5000"])
    assert rc == 0


def test_training_is_deterministic_on_cpu():
    """two runs from the same seed give bitwise-identical losses and weights (fp32, CPU)."""
    import torch

    from bpe_transformer.models import TransformerLM
    from bpe_transformer.train.engine import TrainEngine

    def run():
        torch.manual_seed(0)
        m = TransformerLM(300, 32, 32, 2, 2, 64)
        eng = TrainEngine(m, lr=1e-2, weight_decay=0.1, max_grad_norm=1.0)
        g = torch.Generator().manual_seed(5)
        losses = []
        for _ in range(4):
            x = torch.randint(0, 300, (2, 32), generator=g)
            losses.append(eng.train_step([(x, torch.roll(x, -1, 1))]).item())
        return losses, eng.flat.data.clone()

    (l1, w1), (l2, w2) = run(), run()
    assert l1 == l2
    assert torch.equal(w1, w2)


def test_phase_timing_is_a_noop_on_cpu():
    import torch

    from bpe_transformer.models import TransformerLM
    from bpe_transformer.train.engine import TrainEngine

    m = TransformerLM(100, 16, 32, 1, 2, 64)
    eng = TrainEngine(m, time_phases=True)
    x = torch.randint(0, 100, (2, 16))
    eng.train_step([(x, x)])
    assert eng.phase_times() == {}
