"""Loader for the in-tree gfx950 kernel library ``_bpe_hip.so``.

The library registers ``torch.ops.bpe_hip.*``.  GPU code paths call
:func:`ops` which loads it once; when the library is missing on a machine with
a GPU this raises loudly (there is deliberately no silent PyTorch fallback on
the device: a GPU run either uses the HIP kernels or fails).  Set
``BPE_AUTOBUILD=1`` to compile it on first use.
"""

from __future__ import annotations

import os
import threading
from pathlib import Path

import torch

_VARIANT = os.environ.get("BPE_HIP_VARIANT") or None  # A/B builds: _bpe_hip_<variant>.so (ops/build.py)
LIB_PATH = Path(__file__).resolve().parent / ("_bpe_hip.so" if not _VARIANT else f"_bpe_hip_{_VARIANT}.so")
_lock = threading.Lock()
_loaded = False


def library_path() -> Path:
    return LIB_PATH


def is_built() -> bool:
    return LIB_PATH.exists()


def load() -> None:
    global _loaded
    if _loaded:
        return
    with _lock:
        if _loaded:
            return
        if not LIB_PATH.exists():
            if os.environ.get("BPE_AUTOBUILD", "0") == "1" and not _VARIANT:
                from .build import build

                build()
            else:
                raise RuntimeError(
                    f"bpe_transformer HIP kernels are not built ({LIB_PATH} missing). "
                    "Run `python -m bpe_transformer.ops.build` (hipcc --offload-arch=gfx950)."
                )
        torch.ops.load_library(str(LIB_PATH))
        _loaded = True


def ops():
    """Return the ``torch.ops.bpe_hip`` namespace, loading the library if needed."""
    load()
    return torch.ops.bpe_hip
