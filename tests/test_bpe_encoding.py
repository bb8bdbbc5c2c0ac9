"""BPE encode / decode: GPT-2 parity, round trips, specials, streaming, artifacts.

The reference checks parity against ``tiktoken`` (``tests/test_tokenizer.py``),
which cannot be installed offline; ``tests/gpt2_oracle.py`` is an independent
pure-Python GPT-2 BPE over the same vocab/merges fixtures.
"""

from __future__ import annotations

import io
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
