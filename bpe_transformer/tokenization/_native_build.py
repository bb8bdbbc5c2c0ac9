"""In-tree build of the C++ tokenizer core (``_bpe_native`` pybind11 module).

``python -m bpe_transformer.tokenization._native_build`` compiles
``csrc/tokenizer/bpe_native.cpp`` with g++ (-O3, C++20, pthreads) into
``bpe_transformer/tokenization/_bpe_native<ext-suffix>``.  Incremental: only
rebuilds when the sources are newer than the library.
"""

from __future__ import annotations

import subprocess
import sys
import sysconfig
from pathlib import Path

HERE = Path(__file__).resolve().parent
REPO = HERE.parent.parent
SRC_DIR = REPO / "csrc" / "tokenizer"
SUFFIX = sysconfig.get_config_var("EXT_SUFFIX") or ".so"
LIB = HERE / f"_bpe_native{SUFFIX}"


def build(force: bool = False, verbose: bool = False) -> Path:
    import pybind11

    srcs = [SRC_DIR / "bpe_native.cpp"]
    deps = srcs + list(SRC_DIR.glob("*.h"))
    if not force and LIB.exists() and all(d.stat().st_mtime <= LIB.stat().st_mtime for d in deps):
        return LIB
    cmd = [
        "g++", "-O3", "-std=c++20", "-shared", "-fPIC", "-pthread", "-fvisibility=hidden",
        "-I", pybind11.get_include(), "-I", sysconfig.get_paths()["include"], "-I", str(SRC_DIR),
        *map(str, srcs), "-o", str(LIB),
    ]
    if verbose:
        print(" ".join(cmd))
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        sys.stderr.write(r.stdout + r.stderr)
        raise RuntimeError("building the native tokenizer failed")
    return LIB


if __name__ == "__main__":
    print(build(force="-f" in sys.argv, verbose=True))
