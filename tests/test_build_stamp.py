"""The HIP library's staleness check is content-based (``ops/build.py``, ``ops/_ext.py``).

A source whose bytes change while its mtime does not must be recompiled, and a library whose stamp does not
match the sources next to it must refuse to load.  The compiler is replaced by a recorder here (the real build
is the driver's ``__graft_entry__.build()``), so the test runs in a second.
"""

from __future__ import annotations

import json
import os
import shutil
from pathlib import Path

import pytest

from bpe_transformer.ops import _ext
from bpe_transformer.ops import build as B


@pytest.fixture
def fake_tree(tmp_path, monkeypatch):
    src = tmp_path / "csrc"
    shutil.copytree(B.CSRC, src)
    calls: list[list[str]] = []

    def fake_run(cmd, verbose):
        calls.append(cmd)
        out = Path(cmd[cmd.index("-o") + 1])
        out.write_bytes(b"obj")

    monkeypatch.setattr(B, "_run", fake_run)
    monkeypatch.setattr(B, "BUILD", tmp_path / "build" / "hip")
    monkeypatch.setattr(B, "HERE", tmp_path)
    return src, calls


def _compiled(calls):
    return sorted(Path(c[c.index("-c") + 1]).name for c in calls if "-c" in c)


def test_content_change_with_same_mtime_rebuilds(fake_tree):
    src, calls = fake_tree
    lib = B.build(variant="t", src_dir=src)
    n_src = len(list(src.glob("*.hip"))) + 1
    assert len(_compiled(calls)) == n_src and lib.exists()
    digest = B.read_stamp(lib)
    assert digest == B.source_digest(src)

    calls.clear()
    B.build(variant="t", src_dir=src)
    assert calls == [], "an unchanged tree must not recompile or relink"

    # edit one kernel's bytes but keep its mtime (a checkout / copy can do exactly this)
    f = src / "softmax.hip"
    st = f.stat()
    f.write_text(f.read_text() + "\n// edited\n")
    os.utime(f, ns=(st.st_atime_ns, st.st_mtime_ns))
    calls.clear()
    B.build(variant="t", src_dir=src)
    assert _compiled(calls) == ["softmax.hip"]
    assert any("-shared" in c for c in calls), "the library must be relinked"
    assert B.read_stamp(lib) == B.source_digest(src) != digest

    # a header edit recompiles every unit that includes headers (all of them)
    h = src / "common.h"
    h.write_text(h.read_text() + "\n// edited\n")
    calls.clear()
    B.build(variant="t", src_dir=src)
    assert len(_compiled(calls)) == n_src


def test_stale_library_refuses_to_load(tmp_path, monkeypatch):
    lib = tmp_path / "_bpe_hip.so"
    lib.write_bytes(b"x")
    monkeypatch.setattr(_ext, "LIB_PATH", lib)
    B.stamp_path(lib).write_text(json.dumps({"digest": "0" * 64}))
    with pytest.raises(RuntimeError, match="stale"):
        _ext.check_fresh()
    B.stamp_path(lib).write_text(json.dumps({"digest": B.source_digest(), "lib_sha256": B.lib_sha(lib)}))
    _ext.check_fresh()  # matching stamp: accepted
    # a current stamp next to OTHER library bytes (a library replaced after its build, e.g. a stale copy beside a
    # stamp rewritten for a newer checkout): refused
    lib.write_bytes(b"y")
    with pytest.raises(RuntimeError, match="stale"):
        _ext.check_fresh()
    B.stamp_path(lib).write_text(json.dumps({"digest": B.source_digest()}))  # no library hash: refused
    with pytest.raises(RuntimeError, match="stale"):
        _ext.check_fresh()
    B.stamp_path(lib).unlink()
    with pytest.raises(RuntimeError, match="stale"):
        _ext.check_fresh()


def test_shipped_library_matches_tree():
    """The in-tree library (built by __graft_entry__.build / ops.build) carries the stamp of these sources."""
    if not B.LIB.exists():
        pytest.skip("library not built")
    assert B.read_stamp(B.LIB) == B.source_digest()


def test_shipped_library_loads_on_cpu():
    """The library resolves every symbol (dlopen, no GPU needed): an undefined symbol -- e.g. a declaration that
    landed in an anonymous namespace -- would otherwise only show up on the GPU box."""
    import subprocess
    import sys

    if not B.LIB.exists():
        pytest.skip("library not built")
    code = f"import torch; torch.ops.load_library({str(B.LIB)!r}); print(hasattr(torch.ops.bpe_hip, 'fa_fwd'))"
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0 and r.stdout.strip().endswith("True"), r.stderr[-2000:]
