// Row softmax (last dim) forward / backward for gfx950.
//
// Parity target: reference contract K6 (`tests/adapters.py:424-437`, stable
// under x + 100, `tests/test_nn_utils.py:9-24`).  In the training step softmax
// lives inside the attention and cross-entropy kernels; this standalone op is
// the contract's GPU path.  One 256-thread block per row: an online
// (max, sum-exp) pass, then a normalising pass (row re-read from L2).
#include "common.h"
#include "kernels.h"

namespace bpe {

template <typename T>
__global__ void __launch_bounds__(256) softmax_fwd_kernel(const T* __restrict__ x, T* __restrict__ y, int N) {
    __shared__ float red_m[4], red_s[4];
    const long row = blockIdx.x;
    const T* xr = x + row * (long)N;
    T* yr = y + row * (long)N;
    float m = -INFINITY, s = 0.f;
    for (int i = threadIdx.x; i < N; i += 256) {
        const float v = ld1<T>(xr + i);
        const float mn = fmaxf(m, v);
        s = s * __expf(m - mn) + __expf(v - mn);
        m = mn;
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        const float m2 = __shfl_xor(m, o, 64), s2 = __shfl_xor(s, o, 64);
        const float mn = fmaxf(m, m2);
        if (mn != -INFINITY) { s = s * __expf(m - mn) + s2 * __expf(m2 - mn); m = mn; }
    }
    if ((threadIdx.x & 63) == 0) { red_m[threadIdx.x >> 6] = m; red_s[threadIdx.x >> 6] = s; }
    __syncthreads();
    m = red_m[0]; s = red_s[0];
    for (int w = 1; w < 4; ++w) {
        const float mn = fmaxf(m, red_m[w]);
        if (mn != -INFINITY) { s = s * __expf(m - mn) + red_s[w] * __expf(red_m[w] - mn); m = mn; }
    }
    const float inv = 1.f / s;
    for (int i = threadIdx.x; i < N; i += 256) st1<T>(yr + i, __expf(ld1<T>(xr + i) - m) * inv);
}

template <typename T>
__global__ void __launch_bounds__(256) softmax_bwd_kernel(const T* __restrict__ dy, const T* __restrict__ y,
                                                          T* __restrict__ dx, int N) {
    __shared__ float red[16];
    const long row = blockIdx.x;
    float acc = 0.f;
    for (int i = threadIdx.x; i < N; i += 256) acc += ld1<T>(dy + row * N + i) * ld1<T>(y + row * N + i);
    acc = block_sum(acc, red);
    for (int i = threadIdx.x; i < N; i += 256) {
        const float yy = ld1<T>(y + row * N + i);
        st1<T>(dx + row * N + i, yy * (ld1<T>(dy + row * N + i) - acc));
    }
}

}  // namespace bpe

using namespace bpe;

void launch_softmax_fwd(int dtype, const void* x, void* y, int M, int N, hipStream_t s) {
    if (M == 0) return;
    if (dtype == DT_BF16)
        softmax_fwd_kernel<__bf16><<<M, 256, 0, s>>>((const __bf16*)x, (__bf16*)y, N);
    else
        softmax_fwd_kernel<float><<<M, 256, 0, s>>>((const float*)x, (float*)y, N);
}

void launch_softmax_bwd(int dtype, const void* dy, const void* y, void* dx, int M, int N, hipStream_t s) {
    if (M == 0) return;
    if (dtype == DT_BF16)
        softmax_bwd_kernel<__bf16><<<M, 256, 0, s>>>((const __bf16*)dy, (const __bf16*)y, (__bf16*)dx, N);
    else
        softmax_bwd_kernel<float><<<M, 256, 0, s>>>((const float*)dy, (const float*)y, (float*)dx, N);
}
