// Sanitizer driver for the native tokenizer core (no Python): run under AddressSanitizer +
// UndefinedBehaviorSanitizer or ThreadSanitizer by tools/native_sanitize.sh.
//
//   native_selftest <text file> <vocab size> <threads>
//
// Exercises every threaded path the Python API reaches -- parallel pre-token counting, the trainer,
// the threaded encoder (per-thread caches, chunk boundaries at safe cuts), decode -- and checks
// decode(encode(text)) == text and that threaded and serial encodings agree.
#define BPE_NATIVE_NO_PYTHON 1
#include "bpe_native.cpp"

#include <cstdlib>
#include <iostream>

using namespace bpe_tok;

int main(int argc, char** argv) {
    if (argc < 4) {
        std::cerr << "usage: native_selftest <file> <vocab_size> <threads>\n";
        return 2;
    }
    const std::string text = read_file(argv[1]);
    const int vocab_size = std::atoi(argv[2]), nthreads = std::atoi(argv[3]);
    const std::vector<std::string> specials{"<|endoftext|>"};
    SpecialSplitter sp(specials);
    CountMap counts = count_text_parallel(text, sp, nthreads);
    CountMap serial = count_text_parallel(text, sp, 1);
    if (counts != serial) {
        std::cerr << "FAIL: threaded pre-token counts differ from serial\n";
        return 1;
    }
    Trainer tr;
    tr.train(counts, vocab_size, specials);
    std::unordered_map<int32_t, std::string> vocab;
    for (size_t i = 0; i < tr.vocab.size(); ++i) vocab[(int32_t)i] = tr.vocab[i];
    std::vector<std::pair<std::string, std::string>> merges;
    for (auto& m : tr.merges) merges.emplace_back(tr.vocab[m.first], tr.vocab[m.second]);
    Encoder enc(vocab, merges, specials);
    const std::string clean = sanitize_utf8(text.data(), text.size());
    std::vector<int32_t> par = enc.encode_parallel(clean, nthreads);
    std::vector<int32_t> ser;
    {
        Encoder::Cache c;
        enc.encode_into(clean, ser, c);
    }
    if (par != ser) {
        std::cerr << "FAIL: threaded encoding differs from serial\n";
        return 1;
    }
    std::vector<int64_t> ids(par.begin(), par.end());
    if (enc.decode(ids) != clean) {
        std::cerr << "FAIL: decode(encode(text)) != text\n";
        return 1;
    }
    std::cout << "ok: " << counts.size() << " unique pre-tokens, " << tr.vocab.size() << " vocab, " << tr.merges.size()
              << " merges, " << par.size() << " tokens\n";
    return 0;
}
