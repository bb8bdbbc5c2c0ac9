"""Package-wide constants.

Parity: reference ``bpe_transformer/settings.py:4-10``.  ``PAT`` is the GPT-2
pre-tokenisation regex, byte-for-byte the same string.  ``DEFAULT_OUTPUT_DIR``
is *fixed* here: the reference resolves ``Path(__file__) / "output"`` to a path
*under the settings.py file* (SURVEY §0.6), so a no-argument ``save_trainer()``
could never create its directory.  We anchor it next to the package instead.
"""

from pathlib import Path

ENCODING_STD = "utf-8"

# GPT-2 pre-tokenisation pattern (Radford et al., 2019; tiktoken PR #234).
PAT = r"""'(?:[sdmt]|ll|ve|re)| ?\p{L}+| ?\p{N}+| ?[^\s\p{L}\p{N}]+|\s+(?!\S)|\s+"""

DEFAULT_OUTPUT_DIR = Path(__file__).resolve().parent.parent / "output"
