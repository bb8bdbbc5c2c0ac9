"""BPE encode / decode: GPT-2 parity, round trips, specials, streaming, artifacts.

The reference checks parity against ``tiktoken`` (``tests/test_tokenizer.py``),
which cannot be installed offline; ``tests/gpt2_oracle.py`` is an independent
pure-Python GPT-2 BPE over the same vocab/merges fixtures.
"""

from __future__ import annotations

import io
import os
from pathlib import Path
import pickle

import pytest

from bpe_transformer.tokenization import BPETokenizer
from bpe_transformer.tokenization.serialization import load_gpt2_files

from .adapters import get_tokenizer
from .conftest import FIXTURES
from .gpt2_oracle import GPT2Oracle

EOT = "<|endoftext|>"


@pytest.fixture(scope="module")
def oracle():
    return GPT2Oracle()


@pytest.fixture(scope="module")
def gpt2_files():
    return load_gpt2_files(FIXTURES / "gpt2_vocab.json", FIXTURES / "gpt2_merges.txt", [EOT])


@pytest.fixture(scope="module")
def tok(gpt2_files):
    return get_tokenizer(*gpt2_files, special_tokens=[EOT])


@pytest.fixture(scope="module")
def tok_plain():
    return get_tokenizer(*load_gpt2_files(FIXTURES / "gpt2_vocab.json", FIXTURES / "gpt2_merges.txt"))


STRINGS = [
    "", "s", "🙃", "Hello, how are you?", "Héllò hôw are ü? 🙃",
    "Hello, how <|endoftext|><|endoftext|> are you?<|endoftext|>",
    "x  \n\n y\n", "  leading and trailing  ", "tabs\tand\r\nCRLF\n\n\n", "numbers 12345 and ١٢٣ and ²",
    "don't can't we'll they've you're I'm he'd", "'s 's''s", "日本語のテキスト", "a" * 300, " " * 50 + "x",
]


@pytest.mark.parametrize("text", STRINGS)
def test_roundtrip(tok, text):
    assert tok.decode(tok.encode(text)) == text


@pytest.mark.parametrize("text", [s for s in STRINGS if EOT not in s])
def test_matches_gpt2_without_specials(tok_plain, oracle, text):
    assert tok_plain.encode(text) == oracle.encode(text)


@pytest.mark.parametrize("text", STRINGS)
def test_matches_gpt2_with_specials(tok, oracle, text):
    assert tok.encode(text) == oracle.encode(text, allowed_special={EOT})


@pytest.mark.parametrize("name", ["address.txt", "german.txt", "tinystories_sample.txt",
                                  "special_token_trailing_newlines.txt",
                                  "special_token_double_newlines_non_whitespace.txt", "corpus.en"])
def test_fixture_files_match_gpt2(tok, oracle, name):
    text = (FIXTURES / name).read_text(encoding="utf-8")
    ids = tok.encode(text)
    assert ids == oracle.encode(text, allowed_special={EOT})
    assert tok.decode(ids) == text


def test_overlapping_special_tokens(gpt2_files):
    vocab, merges = gpt2_files
    specials = [EOT, EOT + EOT]
    t = get_tokenizer(dict(vocab), merges, specials)
    s = "Hello, how <|endoftext|><|endoftext|> are you?<|endoftext|>"
    ids = t.encode(s)
    toks = [t.decode([i]) for i in ids]
    assert toks.count(EOT) == 1 and toks.count(EOT + EOT) == 1
    assert t.decode(ids) == s


def test_special_tokens_kept_whole(tok):
    ids = tok.encode("a<|endoftext|>b")
    assert [tok.decode([i]) for i in ids] == ["a", EOT, "b"]


@pytest.mark.parametrize("name", ["tinystories_sample.txt", "german.txt", "address.txt", "corpus.en"])
@pytest.mark.parametrize("workers", [None, 4])
def test_encode_iterable_equals_encode(tok, name, workers):
    path = FIXTURES / name
    whole = tok.encode(path.read_text(encoding="utf-8"))
    with open(path, encoding="utf-8") as f:
        assert list(tok.encode_iterable(f, n_workers=workers)) == whole


def test_encode_iterable_whitespace_boundary(tok):
    """The reference's streaming encode split '\\n\\n' across lines."""
    text = "x  \n\n y\n"
    assert list(tok.encode_iterable(io.StringIO(text))) == tok.encode(text)
    lines = ["x  \n", "\n", " y\n"]
    assert list(tok.encode_iterable(lines)) == tok.encode(text)


def test_encode_iterable_specials_split_across_chunks(tok):
    text = "one\nmore <|endoftext|>\nline\n" * 50
    pieces = [text[i:i + 3] for i in range(0, len(text), 3)]
    assert list(tok.encode_iterable(pieces)) == tok.encode(text)


def test_encode_batch_and_file(tok):
    import numpy as np

    texts = [(FIXTURES / n).read_text(encoding="utf-8") for n in ("german.txt", "address.txt")]
    assert tok.encode_batch(texts, 2) == [tok.encode(t) for t in texts]
    arr = tok.encode_file(FIXTURES / "corpus.en", 4)
    assert isinstance(arr, np.ndarray)
    assert arr.tolist() == tok.encode((FIXTURES / "corpus.en").read_text(encoding="utf-8"))


def test_decode_unknown_id(tok):
    assert tok.decode([99999999]) == "�"


def test_from_files_roundtrip(tmp_path, gpt2_files):
    vocab, merges = gpt2_files
    t = BPETokenizer(vocab, merges, [EOT])
    t.save(tmp_path)
    t2 = BPETokenizer.from_files(tmp_path / "vocab.pkl", tmp_path / "merges.pkl", [EOT, "<|pad|>"])
    s = "Hi <|pad|> there<|endoftext|>"
    assert t2.decode(t2.encode(s)) == s
    assert t2.encode("Hello world") == t.encode("Hello world")


def test_restricted_unpickler_refuses_code(tmp_path):
    class Evil:
        def __reduce__(self):
            return (print, ("pwned",))

    p = tmp_path / "vocab.pkl"
    with open(p, "wb") as f:
        pickle.dump({0: Evil()}, f)
    from bpe_transformer.tokenization.safe_pickle import UnsafePickleError

    with pytest.raises(UnsafePickleError):
        BPETokenizer.load_vocab(p)


def test_safe_pickle_reads_what_pickle_writes(tmp_path):
    """The opcode-level reader decodes builtin data in protocols 3-5 (the reference's artifacts are protocol 4).
    Protocol 2 has no bytes opcode -- it pickles bytes as a call to ``_codecs.encode`` -- and is refused."""
    from bpe_transformer.tokenization import safe_pickle

    obj = {0: b"a", 300: b"\xff" * 300, 70000: b"", 2**40: [(b"x", b"y"), (b"x", b"y")]}
    for proto in (3, 4, 5):
        data = pickle.dumps(obj, protocol=proto)
        assert safe_pickle.loads(data) == obj
    with pytest.raises(safe_pickle.UnsafePickleError):
        safe_pickle.loads(pickle.dumps(obj, protocol=2))
    shared = [b"ab", b"cd"]
    merges = [(shared[0], shared[1]), (shared[1], shared[0])]  # memoised bytes referenced twice
    assert safe_pickle.loads(pickle.dumps(merges, protocol=4)) == merges


SAMPLE = FIXTURES / "sample_tokenizer"  # the reference's notebooks/sample_data/bpe_tokenizer/{vocab,merges}.pkl


def test_reference_sample_tokenizer_parity():
    """The reference's shipped TinyStories tokenizer (10 000 vocab, 9 743 merges) loads through the
    non-executing reader and reproduces the reference notebook's outputs
    (``notebooks/3_bpe_tokenization_encode_decode.ipynb`` cells 11, 16, 18)."""
    t = BPETokenizer.from_files(SAMPLE / "vocab.pkl", SAMPLE / "merges.pkl")
    assert len(t.vocab) == 10000 and len(t.merges) == 9743
    text = "Hello, I am encoding my text. How are you?"
    ids = t.encode(text)
    assert ids == [1183, 44, 338, 740, 835, 1262, 5686, 622, 799, 983, 46, 2687, 483, 349, 63]
    assert t.decode(ids) == text
    with open(FIXTURES / "tinystories_sample.txt", encoding="utf-8") as f:
        stream = list(t.encode_iterable(f))
    assert len(stream) == 927
    assert stream[-10:] == [10, 60, 124, 353, 111, 791, 3279, 124, 62, 10]


def test_trained_tokenizer_end_to_end(tmp_path):
    from bpe_transformer import train_bpe

    vocab, merges = train_bpe(FIXTURES / "tinystories_sample.txt", 400, [EOT])
    t = BPETokenizer(vocab, merges, [EOT])
    text = (FIXTURES / "tinystories_sample.txt").read_text(encoding="utf-8")
    ids = t.encode(text)
    assert t.decode(ids) == text and len(ids) < len(text.encode())


@pytest.mark.parametrize("workers", [None, 4])
def test_encode_iterable_memory_is_bounded(tok, workers):
    """The reference's ``test_encode_iterable_memory_usage`` (5 MB TinyStories stream under a 1 MB rlimit; the
    5 MB blob is not shipped) as a tracemalloc bound: streaming ~5 MB through ``encode_iterable`` while only
    counting ids keeps Python-side peak allocation O(chunk), independent of the stream length (the serial path
    buffers <= one line + 1 KiB, the parallel one <= one 4 MiB batch)."""
    import tracemalloc

    sample = (FIXTURES / "tinystories_sample.txt").read_text(encoding="utf-8")
    lines = sample.splitlines(keepends=True)
    reps = (5 << 20) // len(sample) + 1

    def stream():
        for _ in range(reps):
            yield from lines

    expect = len(tok.encode(sample))
    tracemalloc.start()
    try:
        n = sum(1 for _ in tok.encode_iterable(stream(), n_workers=workers))
        _, peak = tracemalloc.get_traced_memory()
    finally:
        tracemalloc.stop()
    assert abs(n - reps * expect) <= reps  # chunk cuts may merge a boundary token differently at most once each
    limit = (1 << 20) if workers is None else (24 << 20)
    assert peak < limit, peak


_RLIMIT_CHILD = r"""
import os, resource, sys
sys.path.insert(0, sys.argv[1])
from bpe_transformer.tokenization.bpe_tokenizer import BPETokenizer

sample_dir, workers, headroom_mb, stream_mb = sys.argv[2], int(sys.argv[3]), int(sys.argv[4]), int(sys.argv[5])
tok = BPETokenizer.from_files(os.path.join(sample_dir, "sample_tokenizer", "vocab.pkl"),
                              os.path.join(sample_dir, "sample_tokenizer", "merges.pkl"), ["<|endoftext|>"])
with open(os.path.join(sample_dir, "tinystories_sample.txt"), encoding="utf-8") as f:
    lines = f.read().splitlines(keepends=True)
per = sum(len(x) for x in lines)
reps = (stream_mb << 20) // per + 1
expect = len(tok.encode("".join(lines)))
tok.encode("".join(lines) * 4)  # warm every lazily built structure before the limit
if workers > 1:
    list(tok.encode_iterable(iter(lines * 64), n_workers=workers))  # and the worker threads' caches


def vm_bytes():
    with open("/proc/self/status") as f:
        for ln in f:
            if ln.startswith("VmSize:"):
                return int(ln.split()[1]) * 1024


limit = vm_bytes() + (headroom_mb << 20)
resource.setrlimit(resource.RLIMIT_AS, (limit, limit))
try:  # the limit bites: one allocation of the headroom (+ 8 MB of slack for pages freed since) must fail
    bytearray((headroom_mb + 8) << 20)
    print("LIMIT_NOT_EFFECTIVE")
    sys.exit(3)
except MemoryError:
    pass


def stream():
    for _ in range(reps):
        yield from lines


n = 0
for _ in tok.encode_iterable(stream(), n_workers=workers if workers > 1 else None):
    n += 1
assert abs(n - reps * expect) <= reps, (n, reps * expect)
print("OK", n, reps)
"""


@pytest.mark.parametrize("workers,headroom_mb", [(1, 40), (4, 64)])
def test_encode_iterable_rlimit_address_space(tmp_path, workers, headroom_mb):
    """The reference's ``test_encode_iterable_memory_usage`` with a real address-space limit (RLIMIT_AS,
    ``/root/reference/tests/test_tokenizer.py:19-36,416-446``), which -- unlike tracemalloc -- also bounds the C++
    core's allocations.  A fresh interpreter (tokenizer only, no torch) warms up, caps its address space at the
    current size + ``headroom`` (checked to bite: one allocation of the headroom + 8 MB fails), then streams a generated
    96 MB text through ``encode_iterable``: any O(text) buffer, Python or native, would exceed the cap.  Worker
    threads get 1 MB stacks (RLIMIT_STACK before exec) and one malloc arena, so thread reservations stay small."""
    import resource
    import subprocess
    import sys

    if not sys.platform.startswith("linux"):
        pytest.skip("RLIMIT_AS is Linux-specific")
    root = Path(__file__).resolve().parents[1]
    script = tmp_path / "child.py"
    script.write_text(_RLIMIT_CHILD)

    def small_stacks():
        resource.setrlimit(resource.RLIMIT_STACK, (1 << 20, 1 << 20))

    env = dict(os.environ, MALLOC_ARENA_MAX="1", OMP_NUM_THREADS="1")
    r = subprocess.run([sys.executable, str(script), str(root), str(FIXTURES), str(workers), str(headroom_mb), "96"],
                       capture_output=True, text=True, timeout=600, env=env, preexec_fn=small_stacks)
    assert r.returncode == 0 and r.stdout.startswith("OK"), (r.stdout[-500:], r.stderr[-2000:])


def test_safe_pickle_malformed_streams_raise_unsafe_error():
    """Malformed or hostile opcode streams raise UnsafePickleError (a ValueError), never a bare KeyError /
    IndexError / TypeError / AttributeError, so a caller rejecting bad artifacts by that type catches them all."""
    import random

    from bpe_transformer.tokenization import safe_pickle

    P = pickle
    bad = [
        b"\x80\x04h\x00.",                       # BINGET before any PUT
        b"\x80\x04s.",                           # SETITEM on an empty stack
        b"\x80\x04]K\x01K\x02s.",                # SETITEM on a list
        b"\x80\x04}]K\x01s.",                    # unhashable (list) dict key
        b"\x80\x04}K\x01a.",                     # APPEND on a dict
        b"\x80\x04e.",                           # APPENDS with no MARK
        b"\x80\x04\x86.",                        # TUPLE2 on an empty stack
        b"\x80\x04K\x01K\x02",                   # no STOP
        b"\x80\x04",                             # truncated
    ]
    good = P.dumps({1: [(b"a", b"b")], 2: "x"}, protocol=4)
    rng = random.Random(0)
    for _ in range(300):  # random single-byte corruptions and truncations of a valid stream
        d = bytearray(good)
        if rng.random() < 0.5:
            d[rng.randrange(len(d))] = rng.randrange(256)
        else:
            d = d[: rng.randrange(len(d))]
        bad.append(bytes(d))
    for data in bad:
        try:
            safe_pickle.loads(data)
        except safe_pickle.UnsafePickleError:
            pass
