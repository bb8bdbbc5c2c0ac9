#!/bin/bash
# Race / memory checks for the native tokenizer core (host code only; no GPU involved):
#   ASan + UBSan build, then a ThreadSanitizer build of csrc/tokenizer/native_selftest.cpp,
#   each run on a fixture corpus with 8 threads.
# usage: tools/native_sanitize.sh [text file] [vocab size]
set -euo pipefail
cd "$(dirname "$0")/.."
TEXT=${1:-tests/fixtures/corpus.en}
VOCAB=${2:-1000}
OUT=build/sanitize
mkdir -p "$OUT"
SRC=csrc/tokenizer/native_selftest.cpp
g++ -std=c++20 -O1 -g -fno-omit-frame-pointer -fsanitize=address,undefined -fno-sanitize-recover=all -pthread \
    -Icsrc/tokenizer "$SRC" -o "$OUT/selftest_asan"
ASAN_OPTIONS=detect_leaks=1:abort_on_error=1 "$OUT/selftest_asan" "$TEXT" "$VOCAB" 8
g++ -std=c++20 -O1 -g -fsanitize=thread -pthread -Icsrc/tokenizer "$SRC" -o "$OUT/selftest_tsan"
TSAN_OPTIONS=halt_on_error=1 "$OUT/selftest_tsan" "$TEXT" "$VOCAB" 8
echo "native sanitizers: clean"
