"""In-tree build of the gfx950 HIP kernel library.

``python -m bpe_transformer.ops.build`` compiles every ``csrc/*.hip`` with
``hipcc --offload-arch=gfx950`` (device code, no torch headers: seconds per
file), the single torch-binding translation unit, and links
``bpe_transformer/ops/_bpe_hip.so`` next to this file, so the library travels
with the source tree (no JIT cache, no site-packages install).

Staleness is decided by CONTENT, not mtimes: every object records the sha256 of
its compile command, its source and every header (``<obj>.sha``), and the linked
library carries a stamp (``_bpe_hip.so.stamp``, never committed) with the digest of all sources,
headers and flags AND the sha256 of the library bytes it was written for.  ``_ext.load()`` recomputes that digest and refuses a library
whose stamp does not match the tree (or rebuilds it with ``BPE_AUTOBUILD=1``), so a
newer-but-stale ``.so`` shipped with a snapshot can never run in place of the
sources next to it.

No hipify step and no CUDA sources: the kernels are written for CDNA4 directly.
"""

from __future__ import annotations

import argparse
import concurrent.futures as cf
import hashlib
import json
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


COMMON_FLAGS = ["-O3", "-fPIC", "-std=c++17"]


def _digest(paths: list[Path], extra: list[str]) -> str:
    h = hashlib.sha256()
    for x in extra:
        h.update(x.encode() + b"\0")
    for p in paths:
        h.update(p.name.encode() + b"\0")
        h.update(p.read_bytes())
        h.update(b"\0")
    return h.hexdigest()


def source_digest(csrc: Path = CSRC, defines: list[str] | None = None, flags: list[str] | None = None) -> str:
    """sha256 over every kernel source, header and the binding unit plus the arch and flags: the library stamp."""
    files = sorted(csrc.glob("*.h")) + sorted(csrc.glob("*.hip")) + [csrc / "torch_bindings.cpp"]
    return _digest(files, [ARCH, *COMMON_FLAGS, *[f"-D{d}" for d in (defines or [])], *(flags or [])])


def file_flags(src: Path) -> list[str]:
    """Per-file compiler flags: a ``// build-flags: ...`` line among the first 40 lines of the source (part of the
    source, so covered by its digest).  The attention and GEMM kernels use it for ``-fno-slp-vectorize``: packed f32
    VALU (``v_pk_mul_f32`` / ``v_pk_fma_f32``) issued beside MFMAs costs more than the two scalar instructions it
    replaces (MI355X_MICROARCH, price of one filler beside MFMAs)."""
    for line in src.read_text().splitlines()[:40]:
        if line.startswith("// build-flags:"):
            out = []
            for tok in line.split(":", 1)[1].split():  # flags up to the first word that is not one (a remark)
                if not tok.startswith("-"):
                    break
                out.append(tok)
            return out
    return []


def stamp_path(lib: Path) -> Path:
    return lib.with_name(lib.name + ".stamp")


def lib_sha(lib: Path) -> str:
    return hashlib.sha256(lib.read_bytes()).hexdigest()


def read_stamp(lib: Path) -> str | None:
    """The source digest the library was built from, or None when there is no stamp or the stamp was written for
    other library bytes (a stamp and a library that did not come out of one build)."""
    try:
        st = json.loads(stamp_path(lib).read_text())
        return st["digest"] if st.get("lib_sha256") == lib_sha(lib) else None
    except (OSError, ValueError, KeyError):
        return None


def _needs_build(obj: Path, key: str) -> bool:
    """Rebuild unless the object exists and was compiled from exactly this command + source + headers."""
    sha = obj.with_name(obj.name + ".sha")
    return not obj.exists() or not sha.exists() or sha.read_text().strip() != key


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
          defines: list[str] | None = None, src_dir: Path | None = None, flags: list[str] | None = None) -> Path:
    """Build the library; ``variant`` + ``defines`` build an A/B copy (``_bpe_hip_<variant>.so``, own object
    directory) compiled with extra ``-D`` flags, selected at run time with ``BPE_HIP_VARIANT=<variant>``.
    ``src_dir``: compile another copy of ``csrc`` (e.g. an older revision, ``tools/ab_build.sh``) into the
    variant, for same-process / same-box A/B runs.  ``flags``: extra compiler flags after every file's own (a
    variant's ``-fslp-vectorize`` undoes the per-file ``-fno-slp-vectorize``, for instance)."""
    csrc = Path(src_dir) if src_dir else CSRC
    build_dir = BUILD if not variant else BUILD.parent / f"hip_{variant}"
    lib = lib_path(variant)
    build_dir.mkdir(parents=True, exist_ok=True)
    headers = sorted(csrc.glob("*.h"))
    hip_srcs = sorted(csrc.glob("*.hip"))
    inc, libdirs, abi = _torch_paths()
    common = [*COMMON_FLAGS, f"--offload-arch={ARCH}", "-I", str(csrc)]
    common += [f"-D{d}" for d in (defines or [])]
    jobs_list = []  # (command, object, content key)
    objs = []
    for src in hip_srcs:
        obj = build_dir / (src.stem + ".o")
        objs.append(obj)
        cmd = [HIPCC, *common, *file_flags(src), *(flags or []), "-c", str(src), "-o", str(obj)]
        key = _digest([src, *headers], cmd)
        if force or _needs_build(obj, key):
            jobs_list.append((cmd, obj, key))
    bind_src = csrc / "torch_bindings.cpp"
    bind_obj = build_dir / "torch_bindings.o"
    objs.append(bind_obj)
    cmd = [HIPCC, "-O2", "-fPIC", "-std=c++17", f"-D_GLIBCXX_USE_CXX11_ABI={abi}", "-DUSE_ROCM=1",
           "-I", str(csrc)]
    for i in inc:
        cmd += ["-I", i]
    cmd += ["-I", sysconfig.get_paths()["include"], "-c", str(bind_src), "-o", str(bind_obj)]
    key = _digest([bind_src, *headers], cmd)
    if force or _needs_build(bind_obj, key):
        jobs_list.append((cmd, bind_obj, key))

    def compile_one(job):
        cmd, obj, key = job
        obj.with_name(obj.name + ".sha").unlink(missing_ok=True)
        _run(cmd, verbose)
        obj.with_name(obj.name + ".sha").write_text(key + "\n")

    if jobs_list:
        n = jobs or min(8, os.cpu_count() or 4)
        with cf.ThreadPoolExecutor(n) as ex:
            list(ex.map(compile_one, jobs_list))
    digest = source_digest(csrc, defines, flags)
    if force or jobs_list or not lib.exists() or read_stamp(lib) != digest:  # (read_stamp checks the lib bytes)
        stamp_path(lib).unlink(missing_ok=True)
        link = [HIPCC, "-shared", "-fPIC", f"--offload-arch={ARCH}", "-o", str(lib), *map(str, objs)]
        for d in libdirs:
            link += ["-L", d, f"-Wl,-rpath,{d}"]
        link += ["-lc10", "-lc10_hip", "-ltorch", "-ltorch_cpu", "-ltorch_hip"]
        _run(link, verbose)
        stamp_path(lib).write_text(json.dumps({"digest": digest, "lib_sha256": lib_sha(lib), "arch": ARCH,
                                               "defines": defines or [], "flags": flags or [], "src": str(csrc)}) + "\n")
    return lib


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("-v", "--verbose", action="store_true")
    ap.add_argument("-f", "--force", action="store_true")
    ap.add_argument("-j", "--jobs", type=int, default=None)
    ap.add_argument("--variant", default=None, help="build an A/B copy _bpe_hip_<variant>.so")
    ap.add_argument("-D", dest="defines", action="append", default=[], help="extra preprocessor define")
    ap.add_argument("--flag", dest="flags", action="append", default=[],
                    help="extra compiler flag for every source (variants only), e.g. --flag=-fslp-vectorize")
    ap.add_argument("--src", default=None, help="csrc directory to compile instead of the in-tree one (--variant)")
    a = ap.parse_args()
    if a.src and not a.variant:
        ap.error("--src needs --variant (never overwrite the in-tree library with other sources)")
    if a.flags and not a.variant:
        ap.error("--flag needs --variant (the in-tree library takes its flags from the sources)")
    print(build(verbose=a.verbose, jobs=a.jobs, force=a.force, variant=a.variant, defines=a.defines, flags=a.flags,
                src_dir=a.src))


if __name__ == "__main__":
    main()
