// Standalone rotary positional embedding (interleaved pairs) for gfx950.
//
// Parity target: reference contract K8, `tests/adapters.py:187-206`; pairing
// verified against `tests/_snapshots/test_rope.npz`: pairs are
// (x[2i], x[2i+1]), inv_freq_i = theta^(-2i/d), angle = pos * inv_freq_i.
//
// Training hot path: at D = 64 rope_qk_kernel rotates Q and K of the fused
// qkv buffer in place before the attention kernels (which un-rotate dQ / dK
// in their epilogues); other head sizes rotate inside the attention kernels.
// rope_kernel serves the standalone op and its backward (inverse rotation).  cos/sin come from a host-precomputed fp32
// table [max_seq, d/2] (guide App. B: no on-device trig in memory-bound ops).
// x is [R, H, D] contiguous, position of row r = pos[r].
#include "common.h"

#include <climits>
#include <cstdint>
#include <stdexcept>
#include "kernels.h"

namespace bpe {

template <typename T>
__global__ void __launch_bounds__(256) rope_kernel(const T* __restrict__ x, T* __restrict__ y,
                                                   const int64_t* __restrict__ pos, const float* __restrict__ cosT,
                                                   const float* __restrict__ sinT, size_t R, int H, int D,
                                                   float sign) {
    constexpr int V = Vec<T>::N;
    const int dv = D / V;
    const size_t total = R * (size_t)H * dv;
    const int half = D / 2;
    for (size_t idx = blockIdx.x * (size_t)256 + threadIdx.x; idx < total; idx += (size_t)gridDim.x * 256) {
        const size_t r = idx / ((size_t)H * dv);
        const int d0 = (int)(idx % dv) * V;
        const long p = pos[r];
        const float* c = cosT + p * half + d0 / 2;
        const float* s = sinT + p * half + d0 / 2;
        Vec<T> a;
        a.load(x + idx * V);
#pragma unroll
        for (int j = 0; j < V; j += 2) {
            const float cc = c[j / 2], ss = sign * s[j / 2];
            const float x1 = a.v[j], x2 = a.v[j + 1];
            a.v[j] = x1 * cc - x2 * ss;
            a.v[j + 1] = x1 * ss + x2 * cc;
        }
        a.store(y + idx * V);
    }
}

// In-place RoPE on the Q and K column ranges of a fused QKV activation [B*S, (H + 2 Hkv) * D] (row stride ld,
// positions 0..S-1 in every sequence): the training path rotates Q and K ONCE here, so the flash-attention
// forward stages K tiles by LDS-DMA with no per-tile rotation and the backward re-reads rotated Q / K (it
// un-rotates dQ / dK on output).  One 16-byte chunk (4 pairs) per thread step; V columns are not touched.
// 2-D grid: blockIdx.x selects 64 chunk columns of a row (a chunk = 8 values = 4 pairs), blockIdx.y a group of
// 4 * RQK_RPT rows; thread (col, sub) rotates chunk col of rows sub, sub + 4, ...  All index math is 32-bit per
// row (the flat 64-bit `i / cpr`, `r % S` form ran at 3.2 TB/s: profiles/gpt2small_bf16_s1024_b128_kernels_v10.md).
constexpr int RQK_RPT = 8;
__global__ void __launch_bounds__(256) rope_qk_kernel(__bf16* __restrict__ qkv, long ld, const float* __restrict__ cosT,
                                                     const float* __restrict__ sinT, int rows, int S, int cpr,
                                                     int D) {
    const int c = blockIdx.x * 64 + (threadIdx.x & 63);
    if (c >= cpr) return;
    const int half = D / 2, d2 = ((c * 8) % D) / 2;
    const int r0 = blockIdx.y * (4 * RQK_RPT) + (threadIdx.x >> 6);
#pragma unroll 4
    for (int k = 0; k < RQK_RPT; ++k) {
        const int r = r0 + 4 * k;
        if (r >= rows) break;
        const int p = r % S;
        __bf16* px = qkv + (long)r * ld + c * 8;
        const u16x8 v = *reinterpret_cast<const u16x8*>(px);
        const f32x4 cs = *reinterpret_cast<const f32x4*>(cosT + p * half + d2);
        const f32x4 sn = *reinterpret_cast<const f32x4*>(sinT + p * half + d2);
        u16x8 o;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const float a = bf2f(v[2 * j]), b = bf2f(v[2 * j + 1]);
            o[2 * j] = f2bf(a * cs[j] - b * sn[j]);
            o[2 * j + 1] = f2bf(a * sn[j] + b * cs[j]);
        }
        *reinterpret_cast<u16x8*>(px) = o;
    }
}

}  // namespace bpe

using namespace bpe;

void launch_rope_qk(void* qkv, long ld, const float* cosT, const float* sinT, long rows, int S, int H, int Hkv, int D,
                    hipStream_t s) {
    const int cpr = (H + Hkv) * D / 8;
    if (rows > INT32_MAX / 2) throw std::runtime_error("rope_qk_: too many rows");
    const dim3 grid((cpr + 63) / 64, (unsigned)((rows + 4 * RQK_RPT - 1) / (4 * RQK_RPT)));
    rope_qk_kernel<<<grid, 256, 0, s>>>((__bf16*)qkv, ld, cosT, sinT, (int)rows, S, cpr, D);
}

void launch_rope(int dtype, const void* x, void* y, const int64_t* pos, const float* cosT, const float* sinT,
                 size_t R, int H, int D, int inverse, hipStream_t s) {
    const int V = dtype == DT_BF16 ? 8 : 4;
    const int grid = stream_grid(R * H * (size_t)(D / V), 256, 4096);
    const float sign = inverse ? -1.f : 1.f;
    if (dtype == DT_BF16)
        rope_kernel<__bf16><<<grid, 256, 0, s>>>((const __bf16*)x, (__bf16*)y, pos, cosT, sinT, R, H, D, sign);
    else
        rope_kernel<float><<<grid, 256, 0, s>>>((const float*)x, (float*)y, pos, cosT, sinT, R, H, D, sign);
}
