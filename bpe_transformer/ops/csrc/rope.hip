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
// One thread per (row, chunk column c of a head): the cos / sin of that column (32 bytes, from L2) are loaded once
// and applied to the chunk of every Q and K head of the row (16 bytes each, 4 heads' loads in flight per step).
// The flat form -- one (row, chunk) per thread, cos / sin re-read per chunk, 64-bit index math -- moved 3x the
// data bytes through L2 and ran at 3.2 TB/s (profiles/gpt2small_bf16_s1024_b128_kernels_v10.md).
__global__ void __launch_bounds__(256) rope_qk_kernel(__bf16* __restrict__ qkv, long ld, const float* __restrict__ cosT,
                                                     const float* __restrict__ sinT, int rows, int S, int nh,
                                                     int D) {
    const int cph = D / 8, rpb = 256 / cph;
    const int r = blockIdx.x * rpb + (int)threadIdx.x / cph, c = (int)threadIdx.x % cph;
    if (r >= rows || (int)threadIdx.x >= rpb * cph) return;
    const int p = r % S;
    const f32x4 cs = *reinterpret_cast<const f32x4*>(cosT + p * (D / 2) + 4 * c);
    const f32x4 sn = *reinterpret_cast<const f32x4*>(sinT + p * (D / 2) + 4 * c);
    __bf16* row = qkv + (long)r * ld + c * 8;
    auto rot = [&](const u16x8 v) {
        u16x8 o;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const float a = bf2f(v[2 * j]), b = bf2f(v[2 * j + 1]);
            o[2 * j] = f2bf(a * cs[j] - b * sn[j]);
            o[2 * j + 1] = f2bf(a * sn[j] + b * cs[j]);
        }
        return o;
    };
    int h = 0;
    for (; h + 4 <= nh; h += 4) {
        u16x8 v[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) v[i] = *reinterpret_cast<const u16x8*>(row + (h + i) * D);
#pragma unroll
        for (int i = 0; i < 4; ++i) *reinterpret_cast<u16x8*>(row + (h + i) * D) = rot(v[i]);
    }
    for (; h < nh; ++h) *reinterpret_cast<u16x8*>(row + h * D) = rot(*reinterpret_cast<const u16x8*>(row + h * D));
}

}  // namespace bpe

using namespace bpe;

void launch_rope_qk(void* qkv, long ld, const float* cosT, const float* sinT, long rows, int S, int H, int Hkv, int D,
                    hipStream_t s) {
    if (rows > INT32_MAX / 2) throw std::runtime_error("rope_qk_: too many rows");
    if (D % 8 != 0 || D > 256) throw std::runtime_error("rope_qk_: head size must be a multiple of 8, at most 256");
    const int rpb = 256 / (D / 8);
    rope_qk_kernel<<<(unsigned)((rows + rpb - 1) / rpb), 256, 0, s>>>((__bf16*)qkv, ld, cosT, sinT, (int)rows, S,
                                                                      H + Hkv, D);
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
