"""Encode / decode with a trained tokenizer (the reference's notebooks/3_bpe_tokenization_encode_decode.ipynb).

    python examples/3_encode_decode.py output/tokenizer/vocab.pkl output/tokenizer/merges.pkl valid.txt \
        [--tokens-out valid.bin]

Round-trips a sample string, then streams the file through ``encode_iterable`` (constant memory) and
through the threaded ``encode_file``, printing throughput and the compression ratio (bytes / token).
"""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402

from bpe_transformer.tokenization.bpe_tokenizer import BPETokenizer  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("vocab")
    ap.add_argument("merges")
    ap.add_argument("text")
    ap.add_argument("--special", default="<|endoftext|>")
    ap.add_argument("--tokens-out", default=None, help="write the token ids as a flat uint16/uint32 file")
    a = ap.parse_args()
    tok = BPETokenizer.from_files(a.vocab, a.merges, special_tokens=[a.special])
    sample = f"Once upon a time, there was a little robot.{a.special} The end."
    ids = tok.encode(sample)
    assert tok.decode(ids) == sample
    print(f"sample -> {len(ids)} tokens: {ids[:16]}...")

    nbytes = os.path.getsize(a.text)
    t0 = time.perf_counter()
    with open(a.text, encoding="utf-8") as f:
        n = sum(1 for _ in tok.encode_iterable(f))
    dt = time.perf_counter() - t0
    print(f"encode_iterable: {n:,} tokens in {dt:.2f} s ({n / dt / 1e3:.0f} k tok/s), {nbytes / n:.2f} bytes/token")
    t0 = time.perf_counter()
    arr = tok.encode_file(a.text)
    dt = time.perf_counter() - t0
    print(f"encode_file (threaded): {len(arr):,} tokens in {dt:.2f} s ({len(arr) / dt / 1e3:.0f} k tok/s)")
    if a.tokens_out:
        dtype = np.uint16 if len(tok.vocab) <= 65536 else np.uint32
        np.asarray(arr, dtype=dtype).tofile(a.tokens_out)
        print(f"wrote {a.tokens_out} ({dtype.__name__})")


if __name__ == "__main__":
    main()
