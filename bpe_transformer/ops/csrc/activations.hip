// FFN activations for gfx950: SwiGLU gate (K5), SiLU (K3), tanh-GELU.
//
// Parity targets:
//   * SwiGLU / SiLU: reference contract `tests/adapters.py:60-89, 387-398`.
//   * GELU: the reference's only GPU kernel, the Triton tanh-GELU at
//     `bpe_transformer/kernels/triton/gelu.py:33-64`.  Rebuilt here with an
//     overflow-safe tanh (the reference's e^{2a} form is inf/inf = NaN for
//     large x) and with a backward, which the reference lacks.
//
// SwiGLU input is the output of ONE fused GEMM against cat([W1; W3]):
// gu = [M, 2F] with g = gu[:, :F] and u = gu[:, F:].  The gate kernel reads
// both halves with 16-byte vectors and writes a = silu(g) * u, [M, F].
// Memory-bound; vectorised per guide G13; grid-stride with a capped grid.
#include "common.h"
#include "kernels.h"

namespace bpe {

__device__ __forceinline__ float sigmoidf_(float x) { return fast_sigmoid(x); }

__device__ __forceinline__ float gelu_f(float x) {
    const float c = 0.7978845608028654f;  // sqrt(2/pi)
    const float a = c * (x + 0.044715f * x * x * x);
    return 0.5f * x * (1.f + tanhf(a));
}
__device__ __forceinline__ float gelu_grad(float x) {
    const float c = 0.7978845608028654f;
    const float x2 = x * x;
    const float a = c * (x + 0.044715f * x2 * x);
    const float t = tanhf(a);
    return 0.5f * (1.f + t) + 0.5f * x * (1.f - t * t) * c * (1.f + 3.f * 0.044715f * x2);
}

template <typename T>
__global__ void __launch_bounds__(256) swiglu_fwd_kernel(const T* __restrict__ gu, T* __restrict__ out, size_t M,
                                                         int F) {
    constexpr int V = Vec<T>::N;
    const int fv = F / V;
    const size_t total = M * (size_t)fv;
    for (size_t idx = blockIdx.x * (size_t)256 + threadIdx.x; idx < total; idx += (size_t)gridDim.x * 256) {
        const size_t m = idx / fv;
        const int f = (int)(idx - m * fv) * V;
        const T* row = gu + m * (size_t)(2 * F);
        Vec<T> g, u;
        g.load(row + f);
        u.load(row + F + f);
#pragma unroll
        for (int j = 0; j < V; ++j) g.v[j] = g.v[j] * sigmoidf_(g.v[j]) * u.v[j];
        g.store(out + m * (size_t)F + f);
    }
}

template <typename T>
__global__ void __launch_bounds__(256) swiglu_bwd_kernel(const T* __restrict__ dout, const T* __restrict__ gu,
                                                         T* __restrict__ dgu, size_t M, int F) {
    constexpr int V = Vec<T>::N;
    const int fv = F / V;
    const size_t total = M * (size_t)fv;
    for (size_t idx = blockIdx.x * (size_t)256 + threadIdx.x; idx < total; idx += (size_t)gridDim.x * 256) {
        const size_t m = idx / fv;
        const int f = (int)(idx - m * fv) * V;
        const T* row = gu + m * (size_t)(2 * F);
        Vec<T> g, u, d, dg, du;
        g.load(row + f);
        u.load(row + F + f);
        d.load(dout + m * (size_t)F + f);
#pragma unroll
        for (int j = 0; j < V; ++j) {
            const float s = sigmoidf_(g.v[j]);
            const float silu = g.v[j] * s;
            du.v[j] = d.v[j] * silu;
            dg.v[j] = d.v[j] * u.v[j] * s * (1.f + g.v[j] * (1.f - s));
        }
        T* orow = dgu + m * (size_t)(2 * F);
        dg.store(orow + f);
        du.store(orow + F + f);
    }
}

// kind: 0 = silu, 1 = gelu(tanh)
template <typename T, int KIND>
__global__ void __launch_bounds__(256) act_fwd_kernel(const T* __restrict__ x, T* __restrict__ y, size_t nvec) {
    constexpr int V = Vec<T>::N;
    for (size_t i = blockIdx.x * (size_t)256 + threadIdx.x; i < nvec; i += (size_t)gridDim.x * 256) {
        Vec<T> a;
        a.load(x + i * V);
#pragma unroll
        for (int j = 0; j < V; ++j) a.v[j] = KIND == 0 ? a.v[j] * sigmoidf_(a.v[j]) : gelu_f(a.v[j]);
        a.store(y + i * V);
    }
}

template <typename T, int KIND>
__global__ void __launch_bounds__(256) act_bwd_kernel(const T* __restrict__ dy, const T* __restrict__ x,
                                                      T* __restrict__ dx, size_t nvec) {
    constexpr int V = Vec<T>::N;
    for (size_t i = blockIdx.x * (size_t)256 + threadIdx.x; i < nvec; i += (size_t)gridDim.x * 256) {
        Vec<T> a, d;
        a.load(x + i * V);
        d.load(dy + i * V);
#pragma unroll
        for (int j = 0; j < V; ++j) {
            float g;
            if (KIND == 0) {
                const float s = sigmoidf_(a.v[j]);
                g = s * (1.f + a.v[j] * (1.f - s));
            } else {
                g = gelu_grad(a.v[j]);
            }
            a.v[j] = d.v[j] * g;
        }
        a.store(dx + i * V);
    }
}

}  // namespace bpe

using namespace bpe;

void launch_swiglu_fwd(int dtype, const void* gu, void* out, size_t M, int F, hipStream_t s) {
    const int V = dtype == DT_BF16 ? 8 : 4;
    const int grid = stream_grid(M * (size_t)(F / V), 256, 4096);
    if (dtype == DT_BF16)
        swiglu_fwd_kernel<__bf16><<<grid, 256, 0, s>>>((const __bf16*)gu, (__bf16*)out, M, F);
    else
        swiglu_fwd_kernel<float><<<grid, 256, 0, s>>>((const float*)gu, (float*)out, M, F);
}

void launch_swiglu_bwd(int dtype, const void* dout, const void* gu, void* dgu, size_t M, int F, hipStream_t s) {
    const int V = dtype == DT_BF16 ? 8 : 4;
    const int grid = stream_grid(M * (size_t)(F / V), 256, 4096);
    if (dtype == DT_BF16)
        swiglu_bwd_kernel<__bf16><<<grid, 256, 0, s>>>((const __bf16*)dout, (const __bf16*)gu, (__bf16*)dgu, M, F);
    else
        swiglu_bwd_kernel<float><<<grid, 256, 0, s>>>((const float*)dout, (const float*)gu, (float*)dgu, M, F);
}

void launch_act_fwd(int dtype, int kind, const void* x, void* y, size_t n, hipStream_t s) {
    const int V = dtype == DT_BF16 ? 8 : 4;
    const size_t nvec = n / V;
    const int grid = stream_grid(nvec, 256, 4096);
#define ACT_F(T, K) act_fwd_kernel<T, K><<<grid, 256, 0, s>>>((const T*)x, (T*)y, nvec)
    if (dtype == DT_BF16) { if (kind == 0) ACT_F(__bf16, 0); else ACT_F(__bf16, 1); }
    else { if (kind == 0) ACT_F(float, 0); else ACT_F(float, 1); }
#undef ACT_F
}

void launch_act_bwd(int dtype, int kind, const void* dy, const void* x, void* dx, size_t n, hipStream_t s) {
    const int V = dtype == DT_BF16 ? 8 : 4;
    const size_t nvec = n / V;
    const int grid = stream_grid(nvec, 256, 4096);
#define ACT_B(T, K) act_bwd_kernel<T, K><<<grid, 256, 0, s>>>((const T*)dy, (const T*)x, (T*)dx, nvec)
    if (dtype == DT_BF16) { if (kind == 0) ACT_B(__bf16, 0); else ACT_B(__bf16, 1); }
    else { if (kind == 0) ACT_B(float, 0); else ACT_B(float, 1); }
#undef ACT_B
}
