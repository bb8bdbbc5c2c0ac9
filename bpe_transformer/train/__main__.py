"""CLI: ``python -m bpe_transformer.train [--config cfg.json] [--preset NAME] [key=value ...]``.

Examples::

    # TinyStories ~17M plumbing config on the CPU (fp32), synthetic data
    python -m bpe_transformer.train --preset tinystories-17m max_iters=50 batch_size=4 device=cpu

    # GPT-2-small on 8 MI355X over RCCL, real tokens
    torchrun --nproc-per-node 8 --master-addr 127.0.0.1 -m bpe_transformer.train --preset gpt2-small \
        data.train_path=data/train.bin batch_size=32 max_iters=20000 ckpt_every=1000 resume=latest
"""

from __future__ import annotations

import argparse
import json
import os
import sys

from ..models.config import get_preset
from .config import TrainConfig, apply_overrides
from .trainer import Trainer


def main(argv: list[str] | None = None) -> int:
    ap = argparse.ArgumentParser(prog="python -m bpe_transformer.train")
    ap.add_argument("--config", default=None, help="TrainConfig JSON")
    ap.add_argument("--preset", default=None, help="model preset (tinystories-17m, gpt2-small, llama-1.1b, ...)")
    ap.add_argument("--print-config", action="store_true")
    ap.add_argument("overrides", nargs="*", help="dotted key=value overrides, e.g. optim.lr=1e-3")
    a = ap.parse_args(argv)
    cfg = TrainConfig.from_json(a.config) if a.config else TrainConfig()
    if a.preset:
        cfg.model = get_preset(a.preset)
    cfg = apply_overrides(cfg, a.overrides)
    if a.print_config:
        print(json.dumps(cfg.to_dict(), indent=2))
        return 0
    out = Trainer(cfg).fit()
    if int(os.environ.get("RANK", "0")) == 0:
        print(json.dumps(out))
    return 0


if __name__ == "__main__":
    sys.exit(main())
