"""Host-side race / memory checks of the native tokenizer core (SURVEY §5 "Race detection / sanitizers").

Builds csrc/tokenizer/native_selftest.cpp with AddressSanitizer + UndefinedBehaviorSanitizer and with
ThreadSanitizer (tools/native_sanitize.sh) and runs the threaded count / train / encode / decode paths on a
fixture corpus with 8 threads.  GPU sanitizers are not available on the MI355X pool; the HIP side is
checked by the kernel-vs-oracle tests instead.
"""

import shutil
import subprocess
from pathlib import Path

import pytest

REPO = Path(__file__).resolve().parent.parent


@pytest.mark.skipif(shutil.which("g++") is None, reason="needs g++")
def test_native_tokenizer_asan_ubsan_tsan():
    r = subprocess.run([str(REPO / "tools" / "native_sanitize.sh")], cwd=REPO, capture_output=True, text=True,
                       timeout=600)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "native sanitizers: clean" in r.stdout
