"""BPE training: time and peak traced memory (the reference's notebooks/2_bpe_tokenization_training.ipynb).

    python examples/2_bpe_training.py corpus.txt --vocab-size 10000 --out output/tokenizer
"""
import argparse
import os
import sys
import time
import tracemalloc

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from bpe_transformer.tokenization.bpe_trainer import BPETrainer  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("path")
    ap.add_argument("--vocab-size", type=int, default=10_000)
    ap.add_argument("--special", default="<|endoftext|>")
    ap.add_argument("--workers", type=int, default=None)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    tracemalloc.start()
    t0 = time.perf_counter()
    tr = BPETrainer(a.vocab_size, [a.special])
    tr.train(a.path, n_workers=a.workers)
    dt = time.perf_counter() - t0
    _, peak = tracemalloc.get_traced_memory()
    print(f"trained {len(tr.vocab):,} vocab / {len(tr.merges):,} merges in {dt:.2f} s; "
          f"peak traced Python memory {peak / 1e9:.2f} GB")
    longest = max(tr.vocab.values(), key=len)
    print(f"longest token ({len(longest)} bytes): {longest!r}")
    if a.out:
        tr.save_trainer(a.out)
        print(f"saved {a.out}/vocab.pkl, {a.out}/merges.pkl")


if __name__ == "__main__":
    main()
