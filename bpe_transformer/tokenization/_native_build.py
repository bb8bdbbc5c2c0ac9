"""In-tree build of the C++ tokenizer core (``_bpe_native`` pybind11 module).

``python -m bpe_transformer.tokenization._native_build`` compiles
``csrc/tokenizer/bpe_native.cpp`` with g++ (-O3, C++20, pthreads) into
``bpe_transformer/tokenization/_bpe_native<ext-suffix>``.  Incremental by CONTENT:
the library carries a stamp (``<lib>.stamp``, untracked) with the sha256 of the compile
command and every source / header, and of the library bytes themselves; a mismatch (sources edited, whatever their
mtimes) rebuilds, and ``_native.py`` checks the stamp before importing.
"""

from __future__ import annotations

import hashlib
import subprocess
import sys
import sysconfig
from pathlib import Path

HERE = Path(__file__).resolve().parent
REPO = HERE.parent.parent
SRC_DIR = REPO / "csrc" / "tokenizer"
SUFFIX = sysconfig.get_config_var("EXT_SUFFIX") or ".so"
LIB = HERE / f"_bpe_native{SUFFIX}"


STAMP = LIB.with_name(LIB.name + ".stamp")


def _cmd() -> tuple[list[str], list[Path]]:
    import pybind11

    srcs = [SRC_DIR / "bpe_native.cpp"]
    cmd = [
        "g++", "-O3", "-std=c++20", "-shared", "-fPIC", "-pthread", "-fvisibility=hidden",
        "-I", pybind11.get_include(), "-I", sysconfig.get_paths()["include"], "-I", str(SRC_DIR),
        *map(str, srcs), "-o", str(LIB),
    ]
    return cmd, srcs + sorted(SRC_DIR.glob("*.h"))


def digest() -> str:
    """sha256 of the compile flags (not the paths: the tree is copied elsewhere to run) and every source."""
    cmd, deps = _cmd()
    h = hashlib.sha256("\0".join(c for c in cmd if c.startswith("-") and c not in ("-I", "-o")).encode())
    for d in deps:
        h.update(d.name.encode() + b"\0" + d.read_bytes())
    return h.hexdigest()


def _lib_sha() -> str:
    return hashlib.sha256(LIB.read_bytes()).hexdigest()


def is_fresh() -> bool:
    """The stamp (never committed: .gitignore) names both the source digest and the sha256 of the library bytes it
    was written for, so a library and a stamp that did not come out of one build never pass together."""
    try:
        src, lib = STAMP.read_text().split()
        return LIB.exists() and src == digest() and lib == _lib_sha()
    except (OSError, ValueError):
        return False


def build(force: bool = False, verbose: bool = False) -> Path:
    if not force and is_fresh():
        return LIB
    cmd, _ = _cmd()
    STAMP.unlink(missing_ok=True)
    if verbose:
        print(" ".join(cmd))
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        sys.stderr.write(r.stdout + r.stderr)
        raise RuntimeError("building the native tokenizer failed")
    STAMP.write_text(f"{digest()} {_lib_sha()}\n")
    return LIB


if __name__ == "__main__":
    print(build(force="-f" in sys.argv, verbose=True))
