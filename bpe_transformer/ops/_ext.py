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
        autobuild = os.environ.get("BPE_AUTOBUILD", "0") == "1" and not _VARIANT
        if not LIB_PATH.exists():
            if autobuild:
                from .build import build

                build()
            else:
                raise RuntimeError(
                    f"bpe_transformer HIP kernels are not built ({LIB_PATH} missing). "
                    "Run `python -m bpe_transformer.ops.build` (hipcc --offload-arch=gfx950)."
                )
        if not _VARIANT:  # A/B variants are built from other sources / defines: their stamps name those
            check_fresh(autobuild)
        torch.ops.load_library(str(LIB_PATH))
        _loaded = True


def check_fresh(rebuild: bool = False) -> None:
    """Refuse a library whose content stamp does not match the kernel sources next to it (ops/build.py): it was
    built from other sources, so its kernels are not the ones in the tree.  ``rebuild``: rebuild instead."""
    from .build import read_stamp, source_digest

    if read_stamp(LIB_PATH) == source_digest():
        return
    if rebuild:
        from .build import build

        build()
        if read_stamp(LIB_PATH) == source_digest():
            return
    raise RuntimeError(
        f"{LIB_PATH.name} is stale: its content stamp does not match bpe_transformer/ops/csrc (sources changed "
        "since it was built). Run `python -m bpe_transformer.ops.build`, or set BPE_AUTOBUILD=1.")


def ops():
    """Return the ``torch.ops.bpe_hip`` namespace, loading the library if needed."""
    load()
    return torch.ops.bpe_hip
