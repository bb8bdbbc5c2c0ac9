// Token-embedding gather (forward) and deterministic scatter-add (backward).
//
// Parity target: reference contract K2, `tests/adapters.py:38-57` (W[ids]).
//
// Forward: one wave64 per output row, 16-byte vector copies.
// Backward: the host sorts the ids once (stable); then one wave per sorted
// position.  Only the wave at the START of a run of equal ids works: it sums
// the run's gradient rows in sorted order in fp32 registers and writes the
// table row once.  No float atomics (guide G12: they cap at ~1.3 TB/s and are
// order-nondeterministic), bitwise reproducible, and rows never hit by a
// token stay zero (the output is zero-initialised by the caller).
#include "common.h"
#include "kernels.h"

namespace bpe {

template <typename T>
__global__ void __launch_bounds__(256) embed_fwd_kernel(const T* __restrict__ W, const int64_t* __restrict__ ids,
                                                        T* __restrict__ out, int M, int D, long vocab) {
    constexpr int V = Vec<T>::N;
    const int lane = threadIdx.x & 63;
    const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (row >= M) return;
    long id = ids[row];
    if (id < 0 || id >= vocab) id = 0;  // host validates; never read out of bounds
    const T* src = W + id * (long)D;
    T* dst = out + (long)row * D;
    for (int i = lane * V; i < D; i += 64 * V) {
        *reinterpret_cast<u16x8*>(dst + i) = *reinterpret_cast<const u16x8*>(src + i);
    }
}

// C = ceil(D / V / 64) column chunks per lane
template <typename T, int C>
__global__ void __launch_bounds__(256) embed_bwd_kernel(const T* __restrict__ dout, const int64_t* __restrict__ sorted_ids,
                                                        const int64_t* __restrict__ perm, T* __restrict__ dW, int M,
                                                        int D) {
    constexpr int V = Vec<T>::N;
    const int lane = threadIdx.x & 63;
    const int pos = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (pos >= M) return;
    const long id = sorted_ids[pos];
    if (pos > 0 && sorted_ids[pos - 1] == id) return;  // not the start of a run
    const int nvec = D / V;
    float acc[C][V];
#pragma unroll
    for (int c = 0; c < C; ++c)
#pragma unroll
        for (int j = 0; j < V; ++j) acc[c][j] = 0.f;
    for (int p = pos; p < M && sorted_ids[p] == id; ++p) {
        const T* src = dout + perm[p] * (long)D;
#pragma unroll
        for (int c = 0; c < C; ++c) {
            const int i = c * 64 + lane;
            if (i < nvec) {
                Vec<T> a;
                a.load(src + i * V);
#pragma unroll
                for (int j = 0; j < V; ++j) acc[c][j] += a.v[j];
            }
        }
    }
    T* dst = dW + id * (long)D;
#pragma unroll
    for (int c = 0; c < C; ++c) {
        const int i = c * 64 + lane;
        if (i < nvec) {
            Vec<T> o;
#pragma unroll
            for (int j = 0; j < V; ++j) o.v[j] = acc[c][j];
            o.store(dst + i * V);
        }
    }
}

}  // namespace bpe

using namespace bpe;

void launch_embed_fwd(int dtype, const void* W, const int64_t* ids, void* out, int M, int D, long vocab,
                      hipStream_t s) {
    dim3 grid((M + 3) / 4);
    if (dtype == DT_BF16)
        embed_fwd_kernel<__bf16><<<grid, 256, 0, s>>>((const __bf16*)W, ids, (__bf16*)out, M, D, vocab);
    else
        embed_fwd_kernel<float><<<grid, 256, 0, s>>>((const float*)W, ids, (float*)out, M, D, vocab);
}

template <typename T>
static void embed_bwd_dispatch(const T* dout, const int64_t* sorted_ids, const int64_t* perm, T* dW, int M, int D,
                               hipStream_t s) {
    constexpr int V = Vec<T>::N;
    const int chunks = (D / V + 63) / 64;
    dim3 grid((M + 3) / 4);
#define EMB_CASE(CC)                                                                        \
    if (chunks <= CC) {                                                                     \
        embed_bwd_kernel<T, CC><<<grid, 256, 0, s>>>(dout, sorted_ids, perm, dW, M, D);     \
        return;                                                                             \
    }
    EMB_CASE(1) EMB_CASE(2) EMB_CASE(4) EMB_CASE(8) EMB_CASE(16)
#undef EMB_CASE
}

void launch_embed_bwd(int dtype, const void* dout, const int64_t* sorted_ids, const int64_t* perm, void* dW, int M,
                      int D, hipStream_t s) {
    if (M == 0) return;
    if (dtype == DT_BF16)
        embed_bwd_dispatch<__bf16>((const __bf16*)dout, sorted_ids, perm, (__bf16*)dW, M, D, s);
    else
        embed_bwd_dispatch<float>((const float*)dout, sorted_ids, perm, (float*)dW, M, D, s);
}
