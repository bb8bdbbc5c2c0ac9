// Native core of the byte-level BPE tokenizer (pybind11 module `_bpe_native`).
//
// Rebuilds, natively and threaded, what the reference does in Python:
//   * GPT-2 pre-tokenisation  (reference: pretokenization.py:238-252 `regex.finditer(PAT)`,
//     PAT at settings.py:8).  A hand-written matcher for
//       '(?:[sdmt]|ll|ve|re)| ?\p{L}+| ?\p{N}+| ?[^\s\p{L}\p{N}]+|\s+(?!\S)|\s+
//     including the one-code-point backtrack of `\s+(?!\S)`; character classes
//     come from tables generated from the `regex` module (unicode_tables.h).
//   * special-token splitting, longest token first at equal positions
//     (reference: pretokenization.py:211-235).
//   * chunked, multi-threaded pre-token counting of a file (reference:
//     pretokenization.py:73-111 used a process pool; here: std::thread, no
//     pickling, no GIL, chunk boundaries chosen so counts do not depend on the
//     number of threads).
//   * BPE training (reference: bpe_trainer.py:141-445): CANONICAL BPE -- each
//     affected word's pairs are recounted exactly (the reference double-counts
//     self-pairs); most frequent pair first, ties to the
//     lexicographically greater (bytes, bytes); a lazy max-heap plus a
//     pair -> words index.
//   * encoding (reference: bpe_tokenizer.py:139-290, O(n^2) per pre-token):
//     rank-ordered merges with a linked list + min-heap (O(n log n)), a
//     pre-token cache, and a threaded batch/file encoder.
#ifndef BPE_NATIVE_NO_PYTHON  // the core below is plain C++; tools/native_selftest builds it without Python
#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>
#endif

#include <algorithm>
#include <atomic>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <functional>
#include <queue>
#include <stdexcept>
#include <string>
#include <string_view>
#include <memory>
#include <mutex>
#include <thread>
#include <unordered_map>
#include <utility>
#include <vector>

#include "unicode_tables.h"

#ifndef BPE_NATIVE_NO_PYTHON
namespace py = pybind11;
#endif

namespace bpe_tok {

// ------------------------------------------------------------------ Unicode
enum : uint8_t { C_OTHER = 0, C_LETTER = 1, C_NUMBER = 2, C_SPACE = 4 };

static bool in_ranges(uint32_t cp, const CpRange* r, int n) {
    int lo = 0, hi = n - 1;
    while (lo <= hi) {
        const int mid = (lo + hi) >> 1;
        if (cp < r[mid].lo) hi = mid - 1;
        else if (cp > r[mid].hi) lo = mid + 1;
        else return true;
    }
    return false;
}

struct ClassTable {
    uint8_t ascii[128];
    ClassTable() {
        for (uint32_t c = 0; c < 128; ++c) ascii[c] = slow(c);
    }
    static uint8_t slow(uint32_t cp) {
        uint8_t k = C_OTHER;
        if (in_ranges(cp, kLetterRanges, kLetterCount)) k = C_LETTER;
        else if (in_ranges(cp, kNumberRanges, kNumberCount)) k = C_NUMBER;
        if (in_ranges(cp, kSpaceRanges, kSpaceCount)) k |= C_SPACE;
        return k;
    }
};
static const ClassTable g_cls;

static inline uint8_t classify(uint32_t cp) { return cp < 128 ? g_cls.ascii[cp] : ClassTable::slow(cp); }

// Decode one code point of VALID utf-8 at s[i] (input has been sanitised).
static inline uint32_t decode(const uint8_t* s, size_t i, size_t n, int* len) {
    const uint8_t c = s[i];
    if (c < 0x80) { *len = 1; return c; }
    if ((c >> 5) == 6 && i + 1 < n) { *len = 2; return ((c & 0x1F) << 6) | (s[i + 1] & 0x3F); }
    if ((c >> 4) == 14 && i + 2 < n) {
        *len = 3;
        return ((c & 0x0F) << 12) | ((s[i + 1] & 0x3F) << 6) | (s[i + 2] & 0x3F);
    }
    if ((c >> 3) == 30 && i + 3 < n) {
        *len = 4;
        return ((c & 0x07) << 18) | ((s[i + 1] & 0x3F) << 12) | ((s[i + 2] & 0x3F) << 6) | (s[i + 3] & 0x3F);
    }
    *len = 1;
    return 0xFFFD;
}

// Length of a valid utf-8 sequence at s[i], or 0 if invalid (overlong, surrogate, > U+10FFFF, truncated).
static inline int valid_seq(const uint8_t* s, size_t i, size_t n) {
    const uint8_t c = s[i];
    if (c < 0x80) return 1;
    auto cont = [&](size_t k) { return k < n && (s[k] & 0xC0) == 0x80; };
    if (c >= 0xC2 && c <= 0xDF) return cont(i + 1) ? 2 : 0;
    if (c >= 0xE0 && c <= 0xEF) {
        if (!cont(i + 1) || !cont(i + 2)) return 0;
        if (c == 0xE0 && s[i + 1] < 0xA0) return 0;
        if (c == 0xED && s[i + 1] >= 0xA0) return 0;
        return 3;
    }
    if (c >= 0xF0 && c <= 0xF4) {
        if (!cont(i + 1) || !cont(i + 2) || !cont(i + 3)) return 0;
        if (c == 0xF0 && s[i + 1] < 0x90) return 0;
        if (c == 0xF4 && s[i + 1] >= 0x90) return 0;
        return 4;
    }
    return 0;
}

// Python `bytes.decode("utf-8", errors="ignore").encode("utf-8")` (reference pretokenization.py:194), in
// place: invalid bytes are dropped by compacting the buffer.  ASCII is skipped 8 bytes per step and a valid
// buffer (the usual case) is never copied; the byte-at-a-time copy this replaces cost ~50 ms per 20 MB.
static void sanitize_utf8_inplace(std::string& buf) {
    uint8_t* s = reinterpret_cast<uint8_t*>(buf.data());
    const size_t n = buf.size();
    size_t i = 0, o = 0;  // read / write positions (o == i until the first invalid byte)
    while (i < n) {
        if (i + 8 <= n) {
            uint64_t v;
            std::memcpy(&v, s + i, 8);
            if ((v & 0x8080808080808080ull) == 0) {
                if (o != i) std::memmove(s + o, s + i, 8);
                i += 8;
                o += 8;
                continue;
            }
        }
        const int l = valid_seq(s, i, n);
        if (l == 0) {
            ++i;
            continue;
        }
        if (o != i) std::memmove(s + o, s + i, (size_t)l);
        i += l;
        o += l;
    }
    buf.resize(o);
}

static std::string sanitize_utf8(const char* data, size_t n) {
    std::string out(data, n);
    sanitize_utf8_inplace(out);
    return out;
}

// ------------------------------------------------------------------ GPT-2 pattern matcher
// Byte length of the pre-token starting at byte i (i < n) of valid utf-8 text.
static size_t match_at(const uint8_t* s, size_t i, size_t n) {
    int l0;
    const uint32_t cp0 = decode(s, i, n, &l0);
    // 1. contractions '(?:[sdmt]|ll|ve|re)   (ASCII, case-sensitive)
    if (cp0 == '\'' && i + 1 < n) {
        const uint8_t a = s[i + 1];
        if (a == 's' || a == 'd' || a == 'm' || a == 't') return 2;
        if (i + 2 < n) {
            const uint8_t b = s[i + 2];
            if ((a == 'l' && b == 'l') || (a == 'v' && b == 'e') || (a == 'r' && b == 'e')) return 3;
        }
    }
    uint8_t c0 = classify(cp0);
    // 2-4: optional single ' ' then a run of letters | numbers | other
    size_t j = i;
    int lj = l0;
    uint8_t cj = c0;
    if (cp0 == ' ' && i + 1 < n) {
        int l1;
        const uint32_t cp1 = decode(s, i + 1, n, &l1);
        const uint8_t c1 = classify(cp1);
        if (!(c1 & C_SPACE)) { j = i + 1; lj = l1; cj = c1; }
    }
    if (!(cj & C_SPACE)) {
        const uint8_t kind = cj;  // C_LETTER, C_NUMBER or C_OTHER
        size_t k = j + lj;
        while (k < n) {
            const uint8_t b = s[k];
            if (b < 0x80) {  // ASCII: one table lookup, no decode
                if (g_cls.ascii[b] != kind) break;
                ++k;
                continue;
            }
            int l;
            const uint32_t cp = decode(s, k, n, &l);
            if (classify(cp) != kind) break;
            k += l;
        }
        return k - i;
    }
    // 5/6: whitespace run; \s+(?!\S) backtracks one code point when followed by non-space
    size_t k = i, last = i;
    while (k < n) {
        const uint8_t b = s[k];
        if (b < 0x80) {
            if (!(g_cls.ascii[b] & C_SPACE)) break;
            last = k;
            ++k;
            continue;
        }
        int l;
        const uint32_t cp = decode(s, k, n, &l);
        if (!(classify(cp) & C_SPACE)) break;
        last = k;
        k += l;
    }
    if (k == n) return k - i;
    if (last > i) return last - i;
    return k - i;
}

template <typename F>
static void for_each_pretoken(const std::string_view text, F&& f) {
    const uint8_t* s = reinterpret_cast<const uint8_t*>(text.data());
    const size_t n = text.size();
    size_t i = 0;
    while (i < n) {
        const size_t l = match_at(s, i, n);
        f(text.substr(i, l));
        i += l;
    }
}

// ------------------------------------------------------------------ special tokens
struct SpecialSplitter {
    std::vector<std::string> toks;  // sorted by length, longest first
    explicit SpecialSplitter(std::vector<std::string> t) : toks(std::move(t)) {
        std::stable_sort(toks.begin(), toks.end(), [](const std::string& a, const std::string& b) {
            return a.size() > b.size();
        });
        toks.erase(std::remove_if(toks.begin(), toks.end(), [](const std::string& x) { return x.empty(); }), toks.end());
    }
    // Earliest special occurrence at or after `from`; ties -> longest.  Returns {pos, index} or {npos, -1}.
    std::pair<size_t, int> next(std::string_view text, size_t from) const {
        size_t best = std::string_view::npos;
        int bi = -1;
        for (int t = 0; t < (int)toks.size(); ++t) {
            const size_t p = text.find(toks[t], from);
            if (p != std::string_view::npos && (p < best)) { best = p; bi = t; }
        }
        return {best, bi};
    }
    // Visit text segments and specials in order: seg(string_view), special(index).
    template <typename FS, typename FT>
    void split(std::string_view text, FS&& seg, FT&& special) const {
        if (toks.empty()) { seg(text); return; }
        size_t pos = 0;
        // cache of next occurrence per token
        std::vector<size_t> nxt(toks.size());
        for (size_t t = 0; t < toks.size(); ++t) nxt[t] = text.find(toks[t], 0);
        while (pos <= text.size()) {
            size_t best = std::string_view::npos;
            int bi = -1;
            for (size_t t = 0; t < toks.size(); ++t) {
                if (nxt[t] != std::string_view::npos && nxt[t] < pos) nxt[t] = text.find(toks[t], pos);
                if (nxt[t] != std::string_view::npos && nxt[t] < best) { best = nxt[t]; bi = (int)t; }
            }
            if (bi < 0) { seg(text.substr(pos)); return; }
            seg(text.substr(pos, best - pos));
            special(bi);
            pos = best + toks[bi].size();
        }
    }
};

// ------------------------------------------------------------------ safe cut points
// A position p where text[:p] and text[p:] tokenise independently to the same
// pre-tokens as the whole: text[p] is non-whitespace, text[p-1] is a single
// whitespace code point other than ' ', and the code point before that is
// non-whitespace.  (No pre-token alternative can span such a boundary.)
static size_t last_safe_cut(std::string_view text, size_t lo = 0) {
    const uint8_t* s = reinterpret_cast<const uint8_t*>(text.data());
    const size_t n = text.size();
    if (n < 3) return std::string_view::npos;
    for (size_t p = n - 1; p >= lo + 2 && p > 1; --p) {
        const uint8_t c = s[p - 1];
        if (c != '\n' && c != '\r' && c != '\t' && c != 0x0B && c != 0x0C) continue;
        if ((s[p] & 0xC0) == 0x80) continue;
        int l;
        const uint32_t cpn = decode(s, p, n, &l);
        if (classify(cpn) & C_SPACE) continue;
        // code point before p-1
        size_t q = p - 2;
        while (q > 0 && (s[q] & 0xC0) == 0x80) --q;
        const uint32_t cpp = decode(s, q, n, &l);
        if (classify(cpp) & C_SPACE) continue;
        return p;
    }
    return std::string_view::npos;
}

// A position where both halves pre-tokenize to exactly the whole text's pre-tokens: right before the LAST
// character w of a whitespace run when w is an ASCII control space (\n \r \t \v \f) and the next character is not
// whitespace.  In the whole text the run then always ends in a token boundary before w (the ` ?` prefixes only
// take a ' ', and `\s+(?!\S)` stops one short of a run followed by \S); the left half's trailing run matches
// `\s+(?!\S)` to its end, and the right half starts with `w` + non-space, which `\s+` takes alone.  Blank-line
// separated text (".\n\nNext") cuts between the two newlines.  "Next" must not be a special token: a run that
// ends at a special ends its segment, where `\s+(?!\S)` takes the whole run.
static size_t first_safe_cut(std::string_view text, size_t from, const std::vector<std::string>& specials) {
    const uint8_t* s = reinterpret_cast<const uint8_t*>(text.data());
    const size_t n = text.size();
    for (size_t p = std::max<size_t>(from, 1); p + 1 < n; ++p) {
        const uint8_t c = s[p];
        if (c != '\n' && c != '\r' && c != '\t' && c != 0x0B && c != 0x0C) continue;
        int l;
        if (classify(decode(s, p + 1, n, &l)) & C_SPACE) continue;
        bool special_next = false;
        for (const auto& t : specials) special_next |= text.compare(p + 1, t.size(), t) == 0;
        if (special_next) continue;
        return p;
    }
    return std::string_view::npos;
}

// chunk boundaries for parallel processing: at safe cuts or special-token starts, whichever comes first
static std::vector<size_t> chunk_bounds(std::string_view text, const SpecialSplitter& sp, int nchunks) {
    std::vector<size_t> b{0};
    const size_t n = text.size();
    for (int c = 1; c < nchunks; ++c) {
        size_t guess = n * (size_t)c / nchunks;
        if (guess <= b.back()) continue;
        // a pre-token-safe cut after the guess; with special tokens, the start of one that begins first (or
        // straddles the guess) instead -- a file with few or no specials still splits into nchunks pieces
        size_t cut = first_safe_cut(text, guess, sp.toks);
        if (!sp.toks.empty()) {
            const size_t maxlen = sp.toks[0].size();  // longest first
            const size_t from = std::max(b.back(), guess > maxlen ? guess - maxlen : (size_t)0);
            const size_t p = sp.next(text, from).first;
            if (p != std::string_view::npos && (cut == std::string_view::npos || p < cut)) cut = p;
        }
        if (cut == std::string_view::npos || cut >= n) break;
        if (cut > b.back()) b.push_back(cut);
    }
    b.push_back(n);
    return b;
}

// ------------------------------------------------------------------ pre-token counting
struct SvHash {
    using is_transparent = void;
    size_t operator()(std::string_view s) const noexcept { return std::hash<std::string_view>{}(s); }
    size_t operator()(const std::string& s) const noexcept { return std::hash<std::string_view>{}(s); }
};
using CountMap = std::unordered_map<std::string, int64_t, SvHash, std::equal_to<>>;

// Pre-token counter over views into the text being counted (which outlives it): open addressing, linear
// probing, one multiply-mix hash and on a hit one memcmp per pre-token.  The node-based unordered_map it
// replaces allocated a node per new key and chased a bucket pointer per lookup; this table keeps the
// (hash, view, count) slots contiguous.  Keys are copied into std::strings only once, at the end (into()).
// 64-bit multiply-mix hash of a short byte string (pre-tokens average ~5 bytes)
static inline uint64_t pretok_hash(const char* p, size_t n) {
    uint64_t h = 0x9E3779B97F4A7C15ull ^ (n * 0xff51afd7ed558ccdull);
    while (n >= 8) {
        uint64_t v;
        std::memcpy(&v, p, 8);
        h = (h ^ v) * 0xff51afd7ed558ccdull;
        h ^= h >> 32;
        p += 8;
        n -= 8;
    }
    if (n) {
        uint64_t v = 0;
        std::memcpy(&v, p, n);
        h = (h ^ v) * 0xc4ceb9fe1a85ec53ull;
    }
    h ^= h >> 29;
    h *= 0x9E3779B97F4A7C15ull;
    return h ^ (h >> 32);
}

class ViewCounter {
    struct Slot {
        uint64_t h;
        const char* p;  // nullptr: empty
        uint32_t n;
        int64_t c;
    };
    std::vector<Slot> t_;
    size_t used_ = 0;

    void grow() {
        std::vector<Slot> old(t_.size() * 2, Slot{0, nullptr, 0, 0});
        old.swap(t_);
        const size_t mask = t_.size() - 1;
        for (const Slot& x : old) {
            if (!x.p) continue;
            size_t i = x.h & mask;
            while (t_[i].p) i = (i + 1) & mask;
            t_[i] = x;
        }
    }

  public:
    ViewCounter() : t_(size_t(1) << 12, Slot{0, nullptr, 0, 0}) {}
    void add(std::string_view s) {
        const uint64_t h = pretok_hash(s.data(), s.size());
        const size_t mask = t_.size() - 1;
        for (size_t i = h & mask;; i = (i + 1) & mask) {
            Slot& x = t_[i];
            if (!x.p) {
                x = Slot{h, s.data(), (uint32_t)s.size(), 1};
                if (2 * ++used_ > t_.size()) grow();
                return;
            }
            if (x.h == h && x.n == s.size() && std::memcmp(x.p, s.data(), s.size()) == 0) {
                ++x.c;
                return;
            }
        }
    }
    void into(CountMap& m) const {
        for (const Slot& x : t_)
            if (x.p) m[std::string(x.p, x.n)] += x.c;
    }
};

static void count_segment(std::string_view seg, ViewCounter& m) {
    for_each_pretoken(seg, [&](std::string_view tok) { m.add(tok); });
}

static CountMap count_text_parallel(const std::string& text, const SpecialSplitter& sp, int nthreads) {
    nthreads = std::max(1, nthreads);
    const auto bounds = chunk_bounds(text, sp, nthreads * 4);
    const int nchunks = (int)bounds.size() - 1;
    std::vector<ViewCounter> maps(nthreads);
    std::atomic<int> nextc{0};
    auto work = [&](int t) {
        for (;;) {
            const int c = nextc.fetch_add(1);
            if (c >= nchunks) break;
            std::string_view chunk(text.data() + bounds[c], bounds[c + 1] - bounds[c]);
            sp.split(chunk, [&](std::string_view seg) { count_segment(seg, maps[t]); }, [](int) {});
        }
    };
    std::vector<std::thread> th;
    for (int t = 1; t < nthreads; ++t) th.emplace_back(work, t);
    work(0);
    for (auto& x : th) x.join();
    CountMap out;
    for (int t = 0; t < nthreads; ++t) maps[t].into(out);
    return out;
}

static std::string read_file(const std::string& path) {
    std::ifstream f(path, std::ios::binary);
    if (!f) throw std::runtime_error("cannot open " + path);
    f.seekg(0, std::ios::end);
    const std::streamoff n = f.tellg();
    f.seekg(0);
    std::string buf((size_t)n, '\0');
    f.read(buf.data(), n);
    return buf;
}

// ------------------------------------------------------------------ BPE training
struct Trainer {
    std::vector<std::string> vocab;  // id -> bytes
    std::vector<std::pair<int, int>> merges;

    struct Word {
        std::vector<int32_t> sym;
        int64_t cnt;
    };

    static inline uint64_t key(int32_t a, int32_t b) { return ((uint64_t)(uint32_t)a << 32) | (uint32_t)b; }

    void train(const CountMap& counts, int vocab_size, const std::vector<std::string>& specials) {
        // vocab: 256 single bytes, then specials in list order (deterministic, unlike the reference's set)
        vocab.clear();
        for (int b = 0; b < 256; ++b) vocab.emplace_back(1, (char)b);
        for (auto& s : specials) vocab.push_back(s);
        if ((int)vocab.size() > vocab_size) throw std::invalid_argument("vocab_size smaller than 256 + #special tokens");

        std::vector<Word> words;
        words.reserve(counts.size());
        // deterministic word order (sorted keys) so that nothing depends on hash order
        std::vector<const std::pair<const std::string, int64_t>*> items;
        items.reserve(counts.size());
        for (auto& kv : counts) items.push_back(&kv);
        std::sort(items.begin(), items.end(), [](auto* a, auto* b) { return a->first < b->first; });
        for (auto* kv : items) {
            Word w;
            w.cnt = kv->second;
            w.sym.reserve(kv->first.size());
            for (unsigned char c : kv->first) w.sym.push_back(c);
            words.push_back(std::move(w));
        }
        std::unordered_map<uint64_t, int64_t> pc;
        std::unordered_map<uint64_t, std::vector<int32_t>> where;
        pc.reserve(1 << 16);
        for (int32_t wi = 0; wi < (int32_t)words.size(); ++wi) {
            const auto& s = words[wi].sym;
            for (size_t i = 0; i + 1 < s.size(); ++i) {
                const uint64_t k = key(s[i], s[i + 1]);
                pc[k] += words[wi].cnt;
                auto& v = where[k];
                if (v.empty() || v.back() != wi) v.push_back(wi);
            }
        }
        struct Entry {
            int64_t cnt;
            int32_t a, b;
        };
        auto less = [this](const Entry& x, const Entry& y) {  // true if x has LOWER priority than y
            if (x.cnt != y.cnt) return x.cnt < y.cnt;
            const int c = vocab[x.a].compare(vocab[y.a]);
            if (c != 0) return c < 0;
            return vocab[x.b].compare(vocab[y.b]) < 0;
        };
        std::priority_queue<Entry, std::vector<Entry>, decltype(less)> heap(less);
        for (auto& kv : pc)
            if (kv.second > 0) heap.push({kv.second, (int32_t)(kv.first >> 32), (int32_t)(kv.first & 0xFFFFFFFF)});

        std::vector<int> seen(words.size(), -1);
        std::unordered_map<uint64_t, int64_t> delta;
        std::vector<int32_t> tmp;
        int step = 0;
        while ((int)vocab.size() < vocab_size) {
            Entry top{};
            bool found = false;
            while (!heap.empty()) {
                top = heap.top();
                heap.pop();
                auto it = pc.find(key(top.a, top.b));
                if (it != pc.end() && it->second == top.cnt && top.cnt > 0) { found = true; break; }
            }
            if (!found) break;
            const int32_t a = top.a, b = top.b, z = (int32_t)vocab.size();
            vocab.push_back(vocab[a] + vocab[b]);
            merges.emplace_back(a, b);
            std::vector<int32_t> list;
            {
                auto it = where.find(key(a, b));
                if (it != where.end()) { list.swap(it->second); where.erase(it); }
            }
            delta.clear();
            for (int32_t wi : list) {
                if (seen[wi] == step) continue;
                seen[wi] = step;
                Word& w = words[wi];
                const auto& s = w.sym;
                bool has = false;
                for (size_t i = 0; i + 1 < s.size(); ++i)
                    if (s[i] == a && s[i + 1] == b) { has = true; break; }
                if (!has) continue;
                for (size_t i = 0; i + 1 < s.size(); ++i) delta[key(s[i], s[i + 1])] -= w.cnt;
                tmp.clear();
                for (size_t i = 0; i < s.size();) {
                    if (i + 1 < s.size() && s[i] == a && s[i + 1] == b) { tmp.push_back(z); i += 2; }
                    else { tmp.push_back(s[i]); ++i; }
                }
                w.sym.assign(tmp.begin(), tmp.end());
                for (size_t i = 0; i + 1 < w.sym.size(); ++i) {
                    const uint64_t k = key(w.sym[i], w.sym[i + 1]);
                    delta[k] += w.cnt;
                    if (w.sym[i] == z || w.sym[i + 1] == z) {
                        auto& v = where[k];
                        if (v.empty() || v.back() != wi) v.push_back(wi);
                    }
                }
            }
            for (auto& kv : delta) {
                if (kv.second == 0) continue;
                int64_t& c = pc[kv.first];
                c += kv.second;
                if (c > 0) heap.push({c, (int32_t)(kv.first >> 32), (int32_t)(kv.first & 0xFFFFFFFF)});
                else if (c == 0) pc.erase(kv.first);
            }
            ++step;
        }
    }
};

// ------------------------------------------------------------------ encoder
// Pre-token -> token ids cache: open addressing over (hash, key, ids) slots, keys and ids appended to two
// arenas (no node or vector allocation per entry; a hit is one probe sequence, one memcmp and a copy of a
// contiguous id run).
class PretokCache {
    struct Slot {
        uint64_t h;
        uint32_t koff, klen, ioff, ilen;  // ilen == 0: empty (every pre-token has at least one id)
    };
    std::vector<Slot> t_;
    std::string keys_;
    std::vector<int32_t> ids_;
    size_t used_ = 0;

    void grow() {
        std::vector<Slot> old(t_.size() * 2, Slot{0, 0, 0, 0, 0});
        old.swap(t_);
        const size_t mask = t_.size() - 1;
        for (const Slot& x : old) {
            if (!x.ilen) continue;
            size_t i = x.h & mask;
            while (t_[i].ilen) i = (i + 1) & mask;
            t_[i] = x;
        }
    }

  public:
    PretokCache() : t_(size_t(1) << 12, Slot{0, 0, 0, 0, 0}) {}
    size_t size() const { return used_; }
    void clear() {
        t_.assign(size_t(1) << 12, Slot{0, 0, 0, 0, 0});
        keys_.clear();
        ids_.clear();
        used_ = 0;
    }
    // ids of `s` appended to out; false if absent
    bool get(std::string_view s, uint64_t h, std::vector<int32_t>& out) const {
        const size_t mask = t_.size() - 1;
        for (size_t i = h & mask;; i = (i + 1) & mask) {
            const Slot& x = t_[i];
            if (!x.ilen) return false;
            if (x.h == h && x.klen == s.size() && std::memcmp(keys_.data() + x.koff, s.data(), s.size()) == 0) {
                out.insert(out.end(), ids_.begin() + x.ioff, ids_.begin() + x.ioff + x.ilen);
                return true;
            }
        }
    }
    void put(std::string_view s, uint64_t h, const int32_t* ids, size_t n) {
        if (n == 0 || keys_.size() + s.size() > UINT32_MAX || ids_.size() + n > UINT32_MAX) return;
        const size_t mask = t_.size() - 1;
        size_t i = h & mask;
        while (t_[i].ilen) i = (i + 1) & mask;
        t_[i] = Slot{h, (uint32_t)keys_.size(), (uint32_t)s.size(), (uint32_t)ids_.size(), (uint32_t)n};
        keys_.append(s.data(), s.size());
        ids_.insert(ids_.end(), ids, ids + n);
        if (2 * ++used_ > t_.size()) grow();
    }
};

struct Encoder {
    std::unordered_map<int32_t, std::string> id2bytes;
    std::unordered_map<std::string, int32_t, SvHash, std::equal_to<>> bytes2id;
    int32_t byte_id[256];
    std::unordered_map<uint64_t, std::pair<int32_t, int32_t>> ranks;  // (a,b) -> (rank, merged id)
    SpecialSplitter specials;
    std::vector<int32_t> special_ids;
    using Cache = PretokCache;
    Cache cache;  // the calling thread's pre-token cache (worker 0 of every threaded call)
    // persistent caches of workers 1.. of the threaded calls: a 4 MiB encode_iterable batch then starts warm
    // instead of with an empty map per thread per call (the pre-token vocabulary of a corpus is small)
    std::vector<std::unique_ptr<Cache>> worker_cache;
    std::mutex mu;  // one call at a time per Encoder (calls release the GIL; the caches are not shared-safe)
    size_t cache_limit = 1 << 20;

    Cache& cache_of(int t) {
        if (t == 0) return cache;
        while ((int)worker_cache.size() < t) worker_cache.emplace_back(new Cache());
        return *worker_cache[t - 1];
    }

    // run fn(worker, cache) on nthreads threads (the caller is worker 0), each with its own persistent cache
    template <typename F> void run_workers(int nthreads, F&& fn) {
        nthreads = std::max(1, nthreads);
        for (int t = 1; t < nthreads; ++t) cache_of(t);  // allocate before the threads start
        std::vector<std::thread> th;
        for (int t = 1; t < nthreads; ++t) th.emplace_back([&, t]() { fn(cache_of(t)); });
        fn(cache);
        for (auto& x : th) x.join();
    }

    Encoder(const std::unordered_map<int32_t, std::string>& vocab, const std::vector<std::pair<std::string, std::string>>& mg,
            const std::vector<std::string>& sp)
        : id2bytes(vocab), specials(sp) {
        for (auto& kv : id2bytes) {
            auto it = bytes2id.find(kv.second);
            if (it == bytes2id.end() || kv.first < it->second) bytes2id[kv.second] = kv.first;
        }
        for (int b = 0; b < 256; ++b) {
            auto it = bytes2id.find(std::string(1, (char)b));
            byte_id[b] = it == bytes2id.end() ? -1 : it->second;
        }
        for (size_t r = 0; r < mg.size(); ++r) {
            auto ia = bytes2id.find(mg[r].first), ib = bytes2id.find(mg[r].second);
            auto iz = bytes2id.find(mg[r].first + mg[r].second);
            if (ia == bytes2id.end() || ib == bytes2id.end() || iz == bytes2id.end()) continue;
            const uint64_t k = Trainer::key(ia->second, ib->second);
            if (!ranks.count(k)) ranks[k] = {(int32_t)r, iz->second};
        }
        for (auto& s : specials.toks) {
            auto it = bytes2id.find(s);
            if (it == bytes2id.end()) throw std::invalid_argument("special token missing from vocab: " + s);
            special_ids.push_back(it->second);
        }
    }

    void bpe(std::string_view tok, std::vector<int32_t>& out) const {
        const size_t n = tok.size();
        if (n == 1) {
            out.push_back(byte_id[(uint8_t)tok[0]]);
            return;
        }
        std::vector<int32_t> sym(n), nxt(n), prv(n);
        for (size_t i = 0; i < n; ++i) {
            sym[i] = byte_id[(uint8_t)tok[i]];
            nxt[i] = i + 1 < n ? (int32_t)(i + 1) : -1;
            prv[i] = (int32_t)i - 1;
        }
        using E = std::pair<int32_t, int32_t>;  // (rank, pos)
        std::priority_queue<E, std::vector<E>, std::greater<E>> h;
        auto rank_of = [&](int32_t p, int32_t* merged) -> int32_t {
            const int32_t q = nxt[p];
            if (q < 0) return -1;
            auto it = ranks.find(Trainer::key(sym[p], sym[q]));
            if (it == ranks.end()) return -1;
            if (merged) *merged = it->second.second;
            return it->second.first;
        };
        for (int32_t p = 0; p + 1 < (int32_t)n; ++p) {
            const int32_t r = rank_of(p, nullptr);
            if (r >= 0) h.push({r, p});
        }
        std::vector<char> alive(n, 1);
        while (!h.empty()) {
            const auto [r, p] = h.top();
            h.pop();
            if (!alive[p]) continue;
            int32_t z;
            if (rank_of(p, &z) != r) continue;
            const int32_t q = nxt[p];
            sym[p] = z;
            alive[q] = 0;
            nxt[p] = nxt[q];
            if (nxt[q] >= 0) prv[nxt[q]] = p;
            if (prv[p] >= 0) {
                const int32_t r2 = rank_of(prv[p], nullptr);
                if (r2 >= 0) h.push({r2, prv[p]});
            }
            const int32_t r3 = rank_of(p, nullptr);
            if (r3 >= 0) h.push({r3, p});
        }
        for (int32_t p = 0; p >= 0; p = nxt[p]) out.push_back(sym[p]);
    }

    void encode_pretoken(std::string_view tok, std::vector<int32_t>& out, Cache& c) const {
        if (tok.size() == 1) {  // single byte: one table read, no cache
            out.push_back(byte_id[(uint8_t)tok[0]]);
            return;
        }
        const uint64_t h = pretok_hash(tok.data(), tok.size());
        if (c.get(tok, h, out)) return;
        const size_t start = out.size();
        bpe(tok, out);
        if (c.size() < cache_limit) c.put(tok, h, out.data() + start, out.size() - start);
    }

    void encode_into(std::string_view text, std::vector<int32_t>& out, Cache& c) const {
        specials.split(
            text,
            [&](std::string_view seg) { for_each_pretoken(seg, [&](std::string_view t) { encode_pretoken(t, out, c); }); },
            [&](int si) { out.push_back(special_ids[si]); });
    }

    std::vector<int32_t> encode_parallel(const std::string& text, int nthreads) {
        if (nthreads <= 1 || text.size() < (1u << 16)) {
            std::vector<int32_t> out;
            encode_into(text, out, cache);
            return out;
        }
        // boundaries that are safe for pre-tokenisation AND never inside a special token
        std::vector<size_t> b{0};
        const size_t n = text.size();
        const int nchunks = nthreads * 4;
        for (int c = 1; c < nchunks; ++c) {
            size_t cut = first_safe_cut(text, std::max(b.back() + 1, n * (size_t)c / nchunks), specials.toks);
            while (cut != std::string_view::npos && inside_special(text, cut))
                cut = first_safe_cut(text, cut + 1, specials.toks);
            if (cut == std::string_view::npos) break;
            b.push_back(cut);
        }
        b.push_back(n);
        const int nc = (int)b.size() - 1;
        std::vector<std::vector<int32_t>> parts(nc);
        std::atomic<int> nextc{0};
        run_workers(nthreads, [&](Cache& local) {
            for (;;) {
                const int c = nextc.fetch_add(1);
                if (c >= nc) break;
                encode_into(std::string_view(text.data() + b[c], b[c + 1] - b[c]), parts[c], local);
            }
        });
        size_t total = 0;
        for (auto& p : parts) total += p.size();
        std::vector<int32_t> out;
        out.reserve(total);
        for (auto& p : parts) out.insert(out.end(), p.begin(), p.end());
        return out;
    }

    bool inside_special(std::string_view text, size_t cut) const {
        for (auto& s : specials.toks) {
            const size_t lo = cut >= s.size() ? cut - s.size() + 1 : 0;
            const size_t p = text.find(s, lo);
            if (p != std::string_view::npos && p < cut && p + s.size() > cut) return true;
        }
        return false;
    }

    std::string decode(const std::vector<int64_t>& ids) const {
        std::string out;
        for (int64_t id : ids) {
            auto it = id2bytes.find((int32_t)id);
            if (it == id2bytes.end()) out += "\xef\xbf\xbd";
            else out += it->second;
        }
        return out;
    }
};

}  // namespace bpe_tok

// ------------------------------------------------------------------ bindings
#ifndef BPE_NATIVE_NO_PYTHON
using namespace bpe_tok;

static std::string to_str(const py::bytes& b) { return std::string(b); }

static py::dict counts_to_dict(const CountMap& m) {
    py::dict d;
    for (auto& kv : m) d[py::bytes(kv.first)] = kv.second;
    return d;
}

static std::pair<py::dict, py::list> trainer_result(const Trainer& t) {
    py::dict vocab;
    for (size_t i = 0; i < t.vocab.size(); ++i) vocab[py::int_(i)] = py::bytes(t.vocab[i]);
    py::list merges;
    for (auto& m : t.merges) merges.append(py::make_tuple(py::bytes(t.vocab[m.first]), py::bytes(t.vocab[m.second])));
    return {vocab, merges};
}

PYBIND11_MODULE(_bpe_native, m) {
    m.doc() = "Native (C++) core of the bpe_transformer byte-level BPE tokenizer";

    m.def("pretokenize", [](const py::bytes& text) {
        const std::string s = to_str(text);
        py::list out;
        for_each_pretoken(s, [&](std::string_view t) { out.append(py::bytes(t.data(), t.size())); });
        return out;
    }, "GPT-2 pre-tokenisation of utf-8 text -> list of bytes");

    m.def("sanitize_utf8", [](const py::bytes& b) {
        const std::string s = to_str(b);
        return py::bytes(sanitize_utf8(s.data(), s.size()));
    });

    m.def("last_safe_cut", [](const py::bytes& b) -> int64_t {
        const std::string s = to_str(b);
        const size_t p = last_safe_cut(s);
        return p == std::string_view::npos ? -1 : (int64_t)p;
    });

    m.def("count_pretokens_text", [](const py::bytes& text, std::vector<std::string> specials, int nthreads) {
        const std::string s = to_str(text);
        CountMap cm;
        {
            py::gil_scoped_release nogil;
            SpecialSplitter sp(std::move(specials));
            cm = count_text_parallel(s, sp, nthreads);
        }
        return counts_to_dict(cm);
    }, py::arg("text"), py::arg("special_tokens"), py::arg("n_threads") = 1);

    m.def("count_pretokens_file", [](const std::string& path, std::vector<std::string> specials, int nthreads) {
        CountMap cm;
        {
            py::gil_scoped_release nogil;
            std::string raw = read_file(path);
            sanitize_utf8_inplace(raw);
            std::string s = std::move(raw);
            SpecialSplitter sp(std::move(specials));
            cm = count_text_parallel(s, sp, nthreads);
        }
        return counts_to_dict(cm);
    }, py::arg("path"), py::arg("special_tokens"), py::arg("n_threads") = 1);

    m.def("train_from_counts", [](const py::dict& counts, int vocab_size, std::vector<std::string> specials) {
        CountMap cm;
        for (auto item : counts) cm[std::string(py::cast<py::bytes>(item.first))] = py::cast<int64_t>(item.second);
        Trainer t;
        {
            py::gil_scoped_release nogil;
            t.train(cm, vocab_size, specials);
        }
        return trainer_result(t);
    });

    m.def("train_file", [](const std::string& path, int vocab_size, std::vector<std::string> specials, int nthreads) {
        Trainer t;
        {
            py::gil_scoped_release nogil;
            std::string raw = read_file(path);
            sanitize_utf8_inplace(raw);
            std::string s = std::move(raw);
            SpecialSplitter sp(specials);
            CountMap cm = count_text_parallel(s, sp, nthreads);
            t.train(cm, vocab_size, specials);
        }
        return trainer_result(t);
    }, py::arg("path"), py::arg("vocab_size"), py::arg("special_tokens"), py::arg("n_threads") = 1);

    py::class_<Encoder>(m, "Encoder")
        .def(py::init([](const py::dict& vocab, const py::list& merges, std::vector<std::string> specials) {
            std::unordered_map<int32_t, std::string> v;
            for (auto item : vocab) v[py::cast<int32_t>(item.first)] = std::string(py::cast<py::bytes>(item.second));
            std::vector<std::pair<std::string, std::string>> mg;
            mg.reserve(merges.size());
            for (auto item : merges) {
                auto t = py::cast<py::tuple>(item);
                mg.emplace_back(std::string(py::cast<py::bytes>(t[0])), std::string(py::cast<py::bytes>(t[1])));
            }
            return new Encoder(v, mg, specials);
        }))
        .def("encode", [](Encoder& e, const py::bytes& text) {
            const std::string s = to_str(text);
            std::vector<int32_t> out;
            {
                py::gil_scoped_release nogil;
                std::lock_guard<std::mutex> lk(e.mu);
                e.encode_into(s, out, e.cache);
            }
            return out;
        })
        .def("encode_parallel", [](Encoder& e, const py::bytes& text, int nthreads) {
            const std::string s = to_str(text);
            std::vector<int32_t> out;
            {
                py::gil_scoped_release nogil;
                std::lock_guard<std::mutex> lk(e.mu);
                out = e.encode_parallel(s, nthreads);
            }
            return py::array_t<int32_t>(out.size(), out.data());
        })
        .def("encode_batch", [](Encoder& e, const std::vector<std::string>& texts, int nthreads) {
            std::vector<std::vector<int32_t>> outs(texts.size());
            {
                py::gil_scoped_release nogil;
                std::lock_guard<std::mutex> lk(e.mu);
                std::atomic<size_t> nx{0};
                e.run_workers(std::min<int>(nthreads, (int)texts.size()), [&](Encoder::Cache& local) {
                    for (;;) {
                        const size_t i = nx.fetch_add(1);
                        if (i >= texts.size()) break;
                        e.encode_into(texts[i], outs[i], local);
                    }
                });
            }
            return outs;
        })
        // same as encode_batch, returned compactly: (int32 ids of all texts concatenated, int64 offsets [n + 1])
        .def("encode_batch_flat", [](Encoder& e, const std::vector<std::string>& texts, int nthreads) {
            std::vector<std::vector<int32_t>> outs(texts.size());
            {
                py::gil_scoped_release nogil;
                std::lock_guard<std::mutex> lk(e.mu);
                std::atomic<size_t> nx{0};
                e.run_workers(std::min<int>(nthreads, (int)texts.size()), [&](Encoder::Cache& local) {
                    for (;;) {
                        const size_t i = nx.fetch_add(1);
                        if (i >= texts.size()) break;
                        e.encode_into(texts[i], outs[i], local);
                    }
                });
            }
            std::vector<int64_t> off(texts.size() + 1, 0);
            for (size_t i = 0; i < outs.size(); ++i) off[i + 1] = off[i] + (int64_t)outs[i].size();
            py::array_t<int32_t> ids((size_t)off.back());
            int32_t* dst = ids.mutable_data();
            for (size_t i = 0; i < outs.size(); ++i) std::copy(outs[i].begin(), outs[i].end(), dst + off[i]);
            return py::make_tuple(ids, py::array_t<int64_t>(off.size(), off.data()));
        })
        .def("encode_file", [](Encoder& e, const std::string& path, int nthreads) {
            std::vector<int32_t> out;
            {
                py::gil_scoped_release nogil;
                std::string s = read_file(path);
                sanitize_utf8_inplace(s);
                std::lock_guard<std::mutex> lk(e.mu);
                out = e.encode_parallel(s, nthreads);
            }
            return py::array_t<int32_t>(out.size(), out.data());
        })
        .def("decode", [](const Encoder& e, const std::vector<int64_t>& ids) { return py::bytes(e.decode(ids)); })
        .def("cache_size", [](const Encoder& e) { return e.cache.size(); })
        .def("worker_cache_sizes", [](const Encoder& e) {
            std::vector<size_t> n;
            for (auto& c : e.worker_cache) n.push_back(c->size());
            return n;
        })
        .def("clear_cache", [](Encoder& e) {
            std::lock_guard<std::mutex> lk(e.mu);
            e.cache.clear();
            e.worker_cache.clear();
        });
}
#endif  // BPE_NATIVE_NO_PYTHON
