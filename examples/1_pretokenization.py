"""Pre-tokenization timing, parallel vs serial (the reference's notebooks/1_pretokenization.ipynb).

    python examples/1_pretokenization.py corpus.txt [--workers 8]

Counts GPT-2-regex pre-tokens (special tokens split out) with the native threaded counter and with the
single-threaded path, and prints totals, unique pre-tokens and wall times.
"""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from bpe_transformer.tokenization.preprocessing.pretokenization import pretokenize  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("path")
    ap.add_argument("--workers", type=int, default=os.cpu_count())
    ap.add_argument("--special", default="<|endoftext|>")
    a = ap.parse_args()
    for parallel in (True, False):
        t0 = time.perf_counter()
        counts = pretokenize(a.path, special_tokens=[a.special], parallel_processing=parallel,
                             n_workers=a.workers if parallel else 1)
        dt = time.perf_counter() - t0
        print(f"{'parallel' if parallel else 'serial  '}: {sum(counts.values()):,} pre-tokens, "
              f"{len(counts):,} unique, {dt:.2f} s")


if __name__ == "__main__":
    main()
