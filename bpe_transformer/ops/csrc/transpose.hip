// bf16 matrix transpose through LDS (gfx950): dst[C, R] = src[R, C]^T.
//
// Used for the input-gradient GEMMs of the fused transformer block: dX = dY . W runs ~10-20 % faster in
// hipBLASLt's "TN" layout (both operands contiguous along the reduction) than in the "NN" layout of the
// parameter as stored (benchmarks/gemm_layouts.py at 131072 tokens: qkv 0.359 vs 0.407 ms, o 0.138 vs 0.176,
// w13 0.606 vs 0.689), so the block transposes [Wq;Wk;Wv], Wo and [W1;W3] once per backward (~12 us of copies
// per layer against ~0.13 ms saved).  torch's strided copy moves these shapes at ~0.5 TB/s; this kernel
// stages 64 x 64 tiles through LDS so both the reads and the writes are 16-byte row vectors.
#include "common.h"
#include "kernels.h"

namespace bpe {

// one 64 x 64 tile per 256-thread workgroup; thread t reads 16 elements of row t / 4 and writes 16 elements of
// output row t / 4 (= tile column t / 4)
// scale (optional, device fp32 scalar): dst = bf16(scale * src)^T -- the LM head's backward folds the loss
// gradient into the transposed operand copies it makes anyway, instead of two elementwise passes over [T, d]
__global__ void __launch_bounds__(256) transpose_bf16_kernel(const __bf16* __restrict__ src, long ld_src,
                                                             __bf16* __restrict__ dst, long ld_dst, int R, int C,
                                                             const float* __restrict__ scale) {
    __shared__ u16 tile[64][64 + 2];  // +2: the column reads of one wave spread over the banks
    const int tid = threadIdx.x;
    const int tiles_c = C / 64;
    const int r0 = (blockIdx.x / tiles_c) * 64, c0 = (blockIdx.x % tiles_c) * 64;
    const int r = tid >> 2, c = (tid & 3) * 16;
    const __bf16* sp = src + (long)(r0 + r) * ld_src + c0 + c;
    u16x8 a = *reinterpret_cast<const u16x8*>(sp);
    u16x8 b = *reinterpret_cast<const u16x8*>(sp + 8);
    if (scale != nullptr) {
        const float sc = *scale;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            a[j] = f2bf(bf2f(a[j]) * sc);
            b[j] = f2bf(bf2f(b[j]) * sc);
        }
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        tile[r][c + j] = a[j];
        tile[r][c + 8 + j] = b[j];
    }
    __syncthreads();
    u16x8 o0, o1;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        o0[j] = tile[c + j][r];
        o1[j] = tile[c + 8 + j][r];
    }
    __bf16* dp = dst + (long)(c0 + r) * ld_dst + r0 + c;
    *reinterpret_cast<u16x8*>(dp) = o0;
    *reinterpret_cast<u16x8*>(dp + 8) = o1;
}

}  // namespace bpe

using namespace bpe;

void launch_transpose_bf16(const void* src, long ld_src, void* dst, long ld_dst, int R, int C, hipStream_t s,
                           const float* scale) {
    transpose_bf16_kernel<<<(R / 64) * (C / 64), 256, 0, s>>>((const __bf16*)src, ld_src, (__bf16*)dst, ld_dst, R,
                                                              C, scale);
}
