"""Static schedule checks on the ping-pong GEMM's gfx950 assembly (hipcc cross-compiles here, no GPU needed).

The ping-pong schedule (csrc/gemm_pp.hip) relies on each wave issuing exactly one quadrant of MFMAs between two
phase barriers.  hipcc once sank every fp8 MFMA of a K-tile past those barriers (24 + 8 MFMAs in two sections,
three sections empty), which silently serialised the two wave groups; `pin_quadrant` fixed it.  This test
compiles the kernels and fails if any section holds more than one quadrant: 16 bf16 (16x16x32) or 8 fp8
(16x16x128) MFMAs.
"""

from __future__ import annotations

import re
import shutil
import subprocess
import sys
from pathlib import Path

import pytest

REPO = Path(__file__).resolve().parent.parent
CSRC = REPO / "bpe_transformer" / "ops" / "csrc"
HIPCC = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"

sys.path.insert(0, str(REPO / "tools"))
from isa_mfma_sections import sections  # noqa: E402


@pytest.fixture(scope="module")
def gemm_pp_asm(tmp_path_factory):
    if not Path(HIPCC).exists():
        pytest.skip("hipcc not available")
    out = tmp_path_factory.mktemp("isa") / "gemm_pp.s"
    r = subprocess.run([HIPCC, "-O3", "-std=c++17", "--offload-arch=gfx950", "-I", str(CSRC), "-S",
                        "--cuda-device-only", str(CSRC / "gemm_pp.hip"), "-o", str(out)],
                       capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-2000:]
    return out.read_text()


def _kernels(src: str):
    for m in re.finditer(r"^(_Z\S*gemm_pp_kernel\S*):(?:\s*;.*)?$", src, re.M):
        end = src.find(".Lfunc_end", m.end())
        yield m.group(1), sections(src[m.end():end])


def test_one_quadrant_per_section(gemm_pp_asm):
    seen_f8 = seen_bf16 = 0
    for name, sec in _kernels(gemm_pp_asm):
        # template <AK, BKM, SLAB, DIAG, EPI, SPREAD, F8>: the seventh argument is F8
        targs = re.findall(r"L[bi](\d+)E", name[name.index("gemm_pp_kernelI"):name.index("EEv")])
        f8 = int(targs[6])
        limit = 8 if f8 else 16
        assert max(sec) <= limit, (name[:80], sec)
        assert sum(sec) % limit == 0, (name[:80], sec)
        seen_f8 += bool(f8)
        seen_bf16 += not f8
    assert seen_f8 >= 2 and seen_bf16 >= 10
