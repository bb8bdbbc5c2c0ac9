"""bpe_transformer for AMD Instinct MI355X (gfx950).

A GPT-2-style byte-level BPE tokenizer (C++ core) and a decoder-only
Transformer LM training stack whose hot path is hand-written HIP for CDNA4,
scaling over RCCL/xGMI.  API-compatible with ``milasd/BPE-Transformer``
(``bpe_transformer.train_bpe``, ``bpe_transformer.tokenization``).
"""

from __future__ import annotations

try:  # the reference reads installed metadata and fails from a bare checkout
    from importlib.metadata import PackageNotFoundError, version

    __version__ = version("bpe_transformer")
except Exception:  # noqa: BLE001
    __version__ = "0.5.0+mi355x"

__all__ = ["train_bpe", "__version__"]


def __getattr__(name):
    if name == "train_bpe":
        from .main import train_bpe

        return train_bpe
    raise AttributeError(name)
