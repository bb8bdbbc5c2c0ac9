"""In-tree build of the gfx950 HIP kernel library.

``python -m bpe_transformer.ops.build`` compiles every ``csrc/*.hip`` with
``hipcc --offload-arch=gfx950`` (device code, no torch headers: seconds per
file), the single torch-binding translation unit, and links
``bpe_transformer/ops/_bpe_hip.so`` next to this file, so the library travels
with the source tree (no JIT cache, no site-packages install).  Rebuilds are
incremental (mtime of each source and every header).

No hipify step and no CUDA sources: the kernels are written for CDNA4 directly.
"""

from __future__ import annotations

import argparse
import concurrent.futures as cf
import os
import subprocess
import sys
import sysconfig
from pathlib import Path

HERE = Path(__file__).resolve().parent
CSRC = HERE / "csrc"
REPO = HERE.parent.parent
BUILD = REPO / "build" / "hip"
LIB = HERE / "_bpe_hip.so"
ARCH = os.environ.get("BPE_OFFLOAD_ARCH", "gfx950")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")


def _torch_paths():
    import torch
    from torch.utils import cpp_extension

    inc = cpp_extension.include_paths()
    lib = cpp_extension.library_paths()
    abi = int(torch._C._GLIBCXX_USE_CXX11_ABI)
    return inc, lib, abi


def _needs_build(obj: Path, src: Path, headers: list[Path]) -> bool:
    if not obj.exists():
        return True
    t = obj.stat().st_mtime
    return src.stat().st_mtime > t or any(h.stat().st_mtime > t for h in headers)


def _run(cmd: list[str], verbose: bool) -> None:
    if verbose:
        print(" ".join(cmd), flush=True)
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        sys.stderr.write(r.stdout + r.stderr)
        raise RuntimeError(f"compile failed: {' '.join(cmd[:4])} ...")
    if verbose and r.stderr.strip():
        sys.stderr.write(r.stderr)


def lib_path(variant: str | None = None) -> Path:
    return LIB if not variant else HERE / f"_bpe_hip_{variant}.so"


def build(verbose: bool = False, jobs: int | None = None, force: bool = False, variant: str | None = None,
          defines: list[str] | None = None, src_dir: Path | None = None) -> Path:
    """Build the library; ``variant`` + ``defines`` build an A/B copy (``_bpe_hip_<variant>.so``, own object
    directory) compiled with extra ``-D`` flags, selected at run time with ``BPE_HIP_VARIANT=<variant>``.
    ``src_dir``: compile another copy of ``csrc`` (e.g. an older revision, ``tools/ab_build.sh``) into the
    variant, for same-process / same-box A/B runs."""
    csrc = Path(src_dir) if src_dir else CSRC
    build_dir = BUILD if not variant else BUILD.parent / f"hip_{variant}"
    lib = lib_path(variant)
    build_dir.mkdir(parents=True, exist_ok=True)
    headers = sorted(csrc.glob("*.h"))
    hip_srcs = sorted(csrc.glob("*.hip"))
    inc, libdirs, abi = _torch_paths()
    common = ["-O3", "-fPIC", "-std=c++17", f"--offload-arch={ARCH}", "-I", str(csrc)]
    common += [f"-D{d}" for d in (defines or [])]
    jobs_list = []
    objs = []
    for src in hip_srcs:
        obj = build_dir / (src.stem + ".o")
        objs.append(obj)
        if force or _needs_build(obj, src, headers):
            jobs_list.append([HIPCC, *common, "-c", str(src), "-o", str(obj)])
    bind_src = csrc / "torch_bindings.cpp"
    bind_obj = build_dir / "torch_bindings.o"
    objs.append(bind_obj)
    if force or _needs_build(bind_obj, bind_src, headers):
        cmd = [HIPCC, "-O2", "-fPIC", "-std=c++17", f"-D_GLIBCXX_USE_CXX11_ABI={abi}", "-DUSE_ROCM=1",
               "-I", str(csrc)]
        for i in inc:
            cmd += ["-I", i]
        cmd += ["-I", sysconfig.get_paths()["include"], "-c", str(bind_src), "-o", str(bind_obj)]
        jobs_list.append(cmd)
    if jobs_list:
        n = jobs or min(8, os.cpu_count() or 4)
        with cf.ThreadPoolExecutor(n) as ex:
            list(ex.map(lambda c: _run(c, verbose), jobs_list))
    if force or jobs_list or not lib.exists():
        link = [HIPCC, "-shared", "-fPIC", f"--offload-arch={ARCH}", "-o", str(lib), *map(str, objs)]
        for d in libdirs:
            link += ["-L", d, f"-Wl,-rpath,{d}"]
        link += ["-lc10", "-lc10_hip", "-ltorch", "-ltorch_cpu", "-ltorch_hip"]
        _run(link, verbose)
    return lib


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("-v", "--verbose", action="store_true")
    ap.add_argument("-f", "--force", action="store_true")
    ap.add_argument("-j", "--jobs", type=int, default=None)
    ap.add_argument("--variant", default=None, help="build an A/B copy _bpe_hip_<variant>.so")
    ap.add_argument("-D", dest="defines", action="append", default=[], help="extra preprocessor define")
    ap.add_argument("--src", default=None, help="csrc directory to compile instead of the in-tree one (--variant)")
    a = ap.parse_args()
    if a.src and not a.variant:
        ap.error("--src needs --variant (never overwrite the in-tree library with other sources)")
    print(build(verbose=a.verbose, jobs=a.jobs, force=a.force, variant=a.variant, defines=a.defines,
                src_dir=a.src))


if __name__ == "__main__":
    main()
