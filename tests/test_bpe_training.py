"""BPE training: fixture parity, speed gate, special tokens, canonical-BPE oracle.

Fixture parity and the 1.5 s speed gate are the reference's
(``tests/test_train_bpe.py:8-63``).  The reference's special-token snapshot
(``tests/test_train_bpe.py:66-89``, ``_snapshots/test_train_bpe_special_tokens.pkl``) is vendored and read with
the restricted pickle reader (nothing from the file is executed); its input, ``tinystories_sample_5M.txt``, is
missing from the mirror, so the snapshot comparison skips until that fixture is dropped into ``tests/fixtures``
(parity unpinned), and the special-token behaviour itself runs on a corpus built from the present fixtures.
"""

from __future__ import annotations

import json
import random
import time
from collections import Counter

import pytest
import regex

from bpe_transformer.tokenization import BPETrainer
from bpe_transformer.tokenization.serialization import gpt2_bytes_to_unicode

from .adapters import run_train_bpe
from .conftest import FIXTURES

PAT = regex.compile(r"""'(?:[sdmt]|ll|ve|re)| ?\p{L}+| ?\p{N}+| ?[^\s\p{L}\p{N}]+|\s+(?!\S)|\s+""")


def _decode_gpt2(s: str) -> bytes:
    dec = {v: k for k, v in gpt2_bytes_to_unicode().items()}
    return bytes(dec[c] for c in s)


def test_train_bpe_speed():
    t0 = time.time()
    run_train_bpe(FIXTURES / "corpus.en", 500, ["<|endoftext|>"])
    assert time.time() - t0 < 1.5


def test_train_bpe_matches_reference_fixture():
    vocab, merges = run_train_bpe(FIXTURES / "corpus.en", 500, ["<|endoftext|>"])
    lines = (FIXTURES / "train-bpe-reference-merges.txt").read_text(encoding="utf-8").splitlines()
    ref_merges = [tuple(_decode_gpt2(p) for p in ln.split(" ")) for ln in lines]
    assert merges == ref_merges
    ref_vocab = {i: _decode_gpt2(t) for t, i in
                 json.loads((FIXTURES / "train-bpe-reference-vocab.json").read_text(encoding="utf-8")).items()}
    assert set(vocab) == set(ref_vocab)
    assert set(vocab.values()) == set(ref_vocab.values())


def _special_snapshot():
    from bpe_transformer.tokenization.safe_pickle import load

    from .conftest import SNAPSHOTS

    return load(SNAPSHOTS / "test_train_bpe_special_tokens.pkl")


def test_special_token_snapshot_is_consistent():
    """The vendored reference snapshot loads without unpickling and is a 1 000-entry vocabulary with the special
    token, 256 bytes and 743 merges, none of which touches ``<|``."""
    snap = _special_snapshot()
    assert set(snap) == {"vocab_keys", "vocab_values", "merges"}
    assert snap["vocab_keys"] == set(range(1000))
    assert b"<|endoftext|>" in snap["vocab_values"]
    assert {bytes([b]) for b in range(256)} <= snap["vocab_values"]
    assert len(snap["merges"]) == 1000 - 256 - 1
    assert all(b"<|" not in a + b for a, b in snap["merges"])
    assert {a + b for a, b in snap["merges"]} <= snap["vocab_values"]


def test_train_bpe_special_tokens():
    """The reference's snapshot test (``tests/test_train_bpe.py:66-89``), verbatim in what it compares."""
    path = FIXTURES / "tinystories_sample_5M.txt"
    if not path.exists():
        pytest.skip("tinystories_sample_5M.txt is not in the mirror (reference snapshot vendored, parity unpinned)")
    vocab, merges = run_train_bpe(path, 1000, ["<|endoftext|>"])
    for word in vocab.values():
        if word != b"<|endoftext|>":
            assert b"<|" not in word
    snap = _special_snapshot()
    assert set(vocab.keys()) == snap["vocab_keys"]
    assert set(vocab.values()) == snap["vocab_values"]
    assert merges == snap["merges"]


def test_special_tokens_never_merged(tmp_path):
    parts = [(FIXTURES / f).read_text(encoding="utf-8") for f in ("tinystories_sample.txt", "corpus.en", "german.txt")]
    corpus = tmp_path / "c.txt"
    corpus.write_text("<|endoftext|>".join(parts * 3), encoding="utf-8")
    vocab, merges = run_train_bpe(corpus, 700, ["<|endoftext|>"])
    assert len(vocab) == 700
    assert b"<|endoftext|>" in vocab.values()
    for tok in vocab.values():
        if tok != b"<|endoftext|>":
            assert b"<|" not in tok


def test_special_token_ids_follow_list_order(tmp_path):
    f = tmp_path / "a.txt"
    f.write_text("hello world <|pad|> hello", encoding="utf-8")
    specials = ["<|endoftext|>", "<|pad|>", "<|bos|>"]
    vocab, _ = run_train_bpe(f, 270, specials)
    assert [vocab[256], vocab[257], vocab[258]] == [s.encode() for s in specials]


def test_vocab_size_validation(tmp_path):
    f = tmp_path / "a.txt"
    f.write_text("abc", encoding="utf-8")
    with pytest.raises(ValueError):
        run_train_bpe(f, 256, ["<|endoftext|>"])


def _naive_bpe(text: str, vocab_size: int, specials: list[str]):
    """Recount-every-step canonical BPE (the oracle the reference's own trainer diverges from)."""
    words = Counter()
    chunks = regex.split("|".join(regex.escape(s) for s in sorted(specials, key=len, reverse=True)), text) \
        if specials else [text]
    for ch in chunks:
        for m in PAT.finditer(ch):
            words[tuple(bytes([b]) for b in m.group().encode())] += 1
    merges = []
    n_vocab = 256 + len(specials)
    while n_vocab < vocab_size:
        pairs = Counter()
        for w, c in words.items():
            for a, b in zip(w, w[1:]):
                pairs[(a, b)] += c
        if not pairs:
            break
        best = max(pairs, key=lambda p: (pairs[p], p))
        merges.append(best)
        new = Counter()
        for w, c in words.items():
            out, i = [], 0
            while i < len(w):
                if i + 1 < len(w) and (w[i], w[i + 1]) == best:
                    out.append(w[i] + w[i + 1])
                    i += 2
                else:
                    out.append(w[i])
                    i += 1
            new[tuple(out)] += c
        words = new
        n_vocab += 1
    return merges


@pytest.mark.parametrize("seed", range(12))
def test_canonical_bpe_on_adversarial_corpora(tmp_path, seed):
    rnd = random.Random(seed)
    alphabet = ["a", "aa", "b", "ab", " ", "  ", "\n", "é", "xy", "<|eot|>", "1", "!"]
    text = "".join(rnd.choice(alphabet) for _ in range(rnd.randint(50, 400)))
    f = tmp_path / "c.txt"
    f.write_text(text, encoding="utf-8")
    specials = ["<|eot|>"]
    _, merges = run_train_bpe(f, 256 + 1 + 40, specials)
    assert merges == _naive_bpe(text, 256 + 1 + 40, specials)


def test_self_pair_counts_are_exact(tmp_path):
    """'aaaa' has ONE (aa, aa) pair after the first merge (the reference counts 2)."""
    f = tmp_path / "a.txt"
    f.write_text("aaaa aaaa aaaa bbbb", encoding="utf-8")
    _, merges = run_train_bpe(f, 262, [])
    assert merges == _naive_bpe("aaaa aaaa aaaa bbbb", 262, [])


def test_results_independent_of_worker_count(tmp_path):
    text = ((FIXTURES / "corpus.en").read_text(encoding="utf-8") + "\n") * 4
    f = tmp_path / "big.txt"
    f.write_text(text, encoding="utf-8")
    out = [run_train_bpe(f, 600, [], n_workers=n) for n in (1, 3, 8)]
    assert out[0] == out[1] == out[2]


def test_trainer_save_roundtrip(tmp_path):
    from bpe_transformer.tokenization.serialization import load_merges, load_vocab

    tr = BPETrainer(300, ["<|endoftext|>"])
    tr.train(FIXTURES / "corpus.en", n_workers=2)
    tr.save_trainer(tmp_path / "tok")
    assert load_vocab(tmp_path / "tok" / "vocab.pkl") == tr.vocab
    assert load_merges(tmp_path / "tok" / "merges.pkl") == tr.merges


@pytest.mark.parametrize("seed", range(6))
def test_parallel_pretoken_counts_match_regex_oracle(tmp_path, seed):
    """Chunked multi-threaded counting (safe cuts at control-space runs, special-token starts) gives exactly the
    GPT-2 regex's pre-tokens over the whole text: blank lines, CRLF, tabs, space runs, Unicode spaces, specials."""
    from bpe_transformer.tokenization._native import native

    rng = random.Random(seed)
    atoms = ["word", " word", "x", "7", "!!", "'s", " ", "  ", "\n", "\n\n", "\r\n", "\t", "　", " ", "é",
             "<|endoftext|>", "\n<|endoftext|>\n", " \n", "\n ", "\v", "\f"]
    text = "".join(rng.choice(atoms) for _ in range(rng.randint(2000, 6000)))
    path = tmp_path / "t.txt"
    path.write_bytes(text.encode("utf-8"))
    want = Counter()
    for part in regex.split(r"<\|endoftext\|>", text):
        want.update(m.group().encode("utf-8") for m in PAT.finditer(part))
    for n in (1, 3, 8):
        got = native.count_pretokens_file(str(path), ["<|endoftext|>"], n)
        assert Counter(got) == want, n
    assert Counter(native.count_pretokens_file(str(path), [], 8)) == Counter(
        m.group().encode("utf-8") for m in PAT.finditer(text))


def test_pretoken_counts_many_unique_tokens(tmp_path):
    """The native counter (open addressing over text views, grown from 4096 slots) on ~40 000 distinct
    pre-tokens of 1-40 bytes -- letters, digits, punctuation runs, multi-byte letters -- equals the regex oracle,
    for one thread and for per-thread tables merged at the end."""
    from bpe_transformer.tokenization._native import native

    rng = random.Random(7)
    alpha = "abcdefghijklmnopqrstuvwxyzABCDEFGHIJKLMNOPQRSTUVWXYZéüßжπ"
    parts = []
    for _ in range(60000):
        k = rng.random()
        if k < 0.7:
            parts.append(" " * rng.randint(0, 1) + "".join(rng.choice(alpha) for _ in range(rng.randint(1, 20))))
        elif k < 0.85:
            parts.append(" " + str(rng.randint(0, 10 ** rng.randint(1, 12))))
        else:
            parts.append(" " + "".join(rng.choice("!?.,;:-_=+*") for _ in range(rng.randint(1, 6))) + "\n")
    text = "".join(parts)
    path = tmp_path / "u.txt"
    path.write_bytes(text.encode("utf-8"))
    want = Counter(m.group().encode("utf-8") for m in PAT.finditer(text))
    assert len(want) > 30000
    for n in (1, 4):
        assert Counter(native.count_pretokens_file(str(path), [], n)) == want, n


@pytest.mark.parametrize("seed", range(4))
def test_native_utf8_sanitizer_matches_python(seed):
    """sanitize_utf8 (in place, 8-byte ASCII skip) == Python's decode(errors="ignore").encode() on byte soup:
    ASCII runs straddling 8-byte words, valid 2-4 byte sequences, overlongs, surrogates, truncations, stray
    continuation bytes."""
    from bpe_transformer.tokenization._native import native

    rng = random.Random(seed)
    atoms = [b"plain ascii text ", b"abcdefg", b"\xc3\xa9", b"\xe2\x82\xac", b"\xf0\x9f\x98\x80", b"\x80", b"\xbf",
             b"\xc0\xaf", b"\xed\xa0\x80", b"\xf4\x90\x80\x80", b"\xe2\x82", b"\xf0\x9f", b"\xff", b"\n", b"x"]
    data = b"".join(rng.choice(atoms) for _ in range(rng.randint(500, 3000)))
    assert native.sanitize_utf8(data) == data.decode("utf-8", errors="ignore").encode("utf-8")
