"""Checkpoint save / load (reference contract K18, ``tests/adapters.py:505-542``;
test ``tests/test_serialization.py:57-121``).

A checkpoint is one ``torch.save`` dict ``{"model", "optimizer", "iteration",
...extra}`` written to a path or a binary file object.  Loading uses
``torch.load(weights_only=True)`` (nothing in the file is executed) and maps
tensors to the model's device.  In data-parallel runs only rank 0 writes
(``save_checkpoint(..., rank=r)``) and every rank waits at a barrier.
Writes to a path are atomic (temp file + rename) so a crash mid-save never
corrupts the last good checkpoint.
"""

from __future__ import annotations

import os
from pathlib import Path
from typing import IO, BinaryIO

import torch


def save_checkpoint(model: torch.nn.Module, optimizer, iteration: int,
                    out: str | os.PathLike | BinaryIO | IO[bytes], rank: int = 0, **extra) -> None:
    if rank == 0:
        obj = {"model": model.state_dict(), "optimizer": optimizer.state_dict(), "iteration": int(iteration)}
        obj.update(extra)
        if isinstance(out, (str, os.PathLike)):
            path = Path(out)
            path.parent.mkdir(parents=True, exist_ok=True)
            tmp = path.with_suffix(path.suffix + ".tmp")
            torch.save(obj, tmp)
            os.replace(tmp, path)
        else:
            torch.save(obj, out)
    if torch.distributed.is_available() and torch.distributed.is_initialized():
        torch.distributed.barrier()


def load_checkpoint(src: str | os.PathLike | BinaryIO | IO[bytes], model: torch.nn.Module, optimizer=None) -> int:
    try:
        dev = next(model.parameters()).device
    except StopIteration:
        dev = torch.device("cpu")
    obj = torch.load(src, map_location=dev, weights_only=True)
    model.load_state_dict(obj["model"])
    if optimizer is not None and "optimizer" in obj:
        optimizer.load_state_dict(obj["optimizer"])
    return int(obj["iteration"])


def read_checkpoint(src, map_location="cpu") -> dict:
    return torch.load(src, map_location=map_location, weights_only=True)


def latest_checkpoint(directory: str | os.PathLike, pattern: str = "ckpt_*.pt") -> Path | None:
    d = Path(directory)
    if not d.is_dir():
        return None
    cands = sorted(d.glob(pattern), key=lambda p: p.stat().st_mtime)
    return cands[-1] if cands else None
