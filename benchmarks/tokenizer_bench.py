"""CPU tokenizer benchmark on the workloads BASELINE.md measured with the reference code on this 8-vCPU box.

The reference's only published numbers are tokenizer timings (its notebooks, M3 Pro laptop); the survey re-ran
the reference code here on ``tests/fixtures/corpus.en`` and on that file repeated 150x (19.96 MB).  This script
times the same four workloads through this package's public API (the native C++ core underneath) and prints one
JSON line per workload with the reference's time on the same box:

  1. ``train_bpe(corpus.en, vocab_size=500)``                       reference 0.31-0.42 s (speed gate < 1.5 s)
  2. pre-tokenize 19.96 MB, parallel (8 workers) / serial          reference 0.51 s / 3.05 s
  3. BPE training on 19.96 MB, vocab 10 000                          reference 1.30 s
  4. ``encode_iterable`` over 19.96 MB, serial / 8 workers           reference 11.63 s / 195.1 s

    python benchmarks/tokenizer_bench.py [--repeat 150] [--workers 8]
"""
import argparse
import json
import os
import sys
import tempfile
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from bpe_transformer import train_bpe  # noqa: E402
from bpe_transformer.tokenization.bpe_tokenizer import BPETokenizer  # noqa: E402
from bpe_transformer.tokenization.preprocessing.pretokenization import pretokenize  # noqa: E402

FIXTURE = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests", "fixtures",
                       "corpus.en")
SPECIAL = ["<|endoftext|>"]
# reference code on this box (BASELINE.md "Measured here"), seconds
REF = {"train_bpe_corpus_en_v500": 0.365, "pretokenize_parallel": 0.51, "pretokenize_serial": 3.05,
       "train_bpe_20MB_v10000": 1.30, "encode_iterable_serial": 11.63, "encode_iterable_parallel": 195.1}


def timed(fn, reps=1):
    best, out = float("inf"), None
    for _ in range(reps):
        t0 = time.perf_counter()
        out = fn()
        best = min(best, time.perf_counter() - t0)
    return best, out


def effective_cores(n: int = 8, mb: int = 32) -> float:
    """How many threads actually run at once right now: n GIL-free sha256 threads against one.  On a shared or
    oversubscribed box this is far below os.cpu_count(), and parallel rows then measure no thread scaling."""
    import hashlib
    import threading

    data = b"x" * (mb << 20)

    def run(k: int) -> float:
        ts = [threading.Thread(target=lambda: hashlib.sha256(data).digest()) for _ in range(k)]
        t0 = time.perf_counter()
        for t in ts:
            t.start()
        for t in ts:
            t.join()
        return time.perf_counter() - t0

    one = min(run(1) for _ in range(2))
    return round(n * one / min(run(n) for _ in range(2)), 2)


def emit(name, seconds, **extra):
    ref = REF.get(name)
    row = {"workload": name, "seconds": round(seconds, 4), "reference_seconds": ref,
           "speedup_vs_reference": round(ref / seconds, 2) if ref else None}
    row.update(extra)
    print(json.dumps(row), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--repeat", type=int, default=150, help="corpus.en copies in the large file (150 = 19.96 MB)")
    ap.add_argument("--workers", type=int, default=8)
    a = ap.parse_args()
    # printed first, and again last: parallel rows only show thread scaling where this is near --workers
    print(json.dumps({"cpu_count": os.cpu_count(), "effective_cores_8_threads": effective_cores()}), flush=True)

    t, (vocab, merges) = timed(lambda: train_bpe(FIXTURE, 500, SPECIAL), reps=3)
    emit("train_bpe_corpus_en_v500", t, merges=len(merges))

    with tempfile.TemporaryDirectory() as td:
        big = os.path.join(td, "corpus_x.txt")
        with open(FIXTURE, "rb") as f:
            data = f.read()
        with open(big, "wb") as f:
            for _ in range(a.repeat):
                f.write(data)
        mb = os.path.getsize(big) / 1e6

        t, counts = timed(lambda: pretokenize(big, special_tokens=SPECIAL, parallel_processing=True,
                                              n_workers=a.workers), reps=3)
        emit("pretokenize_parallel", t, MB=round(mb, 2), pretokens=sum(counts.values()), unique=len(counts))
        t, counts = timed(lambda: pretokenize(big, special_tokens=SPECIAL, parallel_processing=False,
                                              n_workers=1), reps=3)
        emit("pretokenize_serial", t, MB=round(mb, 2), pretokens=sum(counts.values()))

        t, (vocab, merges) = timed(lambda: train_bpe(big, 10_000, SPECIAL, n_workers=a.workers))
        emit("train_bpe_20MB_v10000", t, merges=len(merges))

        tok = BPETokenizer(vocab, merges, special_tokens=SPECIAL)

        def run(n_workers):
            n = 0
            with open(big, encoding="utf-8") as f:
                for _ in tok.encode_iterable(f, n_workers):
                    n += 1
            return n

        t, n = timed(lambda: run(None))
        emit("encode_iterable_serial", t, tokens=n, tok_per_s=round(n / t))
        t, n = timed(lambda: run(a.workers))
        emit("encode_iterable_parallel", t, tokens=n, tok_per_s=round(n / t))
    print(json.dumps({"effective_cores_8_threads_after": effective_cores()}), flush=True)


if __name__ == "__main__":
    main()
