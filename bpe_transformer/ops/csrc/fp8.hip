// FP8 (OCP e4m3fn / e5m2) quantisation kernels for gfx950, delayed scaling.
//
// The fp8 training path (BASELINE.json config "Llama-style 1.1B fp8 MFMA
// path") runs every block projection's GEMMs as fp8 x fp8 on the MFMA fp8
// units, with per-tensor scales.  Which kernel runs them (ops/fp8.py):
//   * the QKV forward: the hand-written f8f6f4 kernel (gemm_pp.hip, F8) with
//     RoPE in its epilogue (gemm_fp8_rope);
//   * every weight gradient dW = dY^T X (e5m2 x e4m3): the hand kernel's
//     split-K form (gemm_fp8_acc, fp32 partials, ordered reduce into the
//     gradient buffer);
//   * the W13 forward (with fp8 weight gradients): the hand kernel with the
//     SwiGLU gate and its two-layout e4m3 cast in the epilogue
//     (gemm_pp.hip EPI_SWIGLU_FWD8; round 6), replacing swiglu_cast_fp8's
//     forward pass;
//   * the other forward and the input-gradient GEMMs: hipBLASLt
//     (torch._scaled_mm) -- it leads the hand kernel by 3-12 % at the
//     65 536-token shapes (profiles/bench/fp8_gemm_orders_r6.log) -- except
//     the shapes routed to the hand kernel in ops/tuning/fp8_routes.json (two
//     16 384-token shapes).
// The casts here produce their operands:
//
//   x8 = sat(x * s)            s = FMAX / (max over the amax history), FMAX = 448 (e4m3) / 57344 (e5m2)
//   y  = (x8 / s_x) . (w8 / s_w)^T
//
// Everything that touches the scales stays on the device -- no host sync:
//   * cast_fp8: one streaming pass that writes x8 with the CURRENT scale and
//     folds |x|max into this step's amax slot (block max + one atomicMax per
//     block on the float bit pattern, valid because amax >= 0);
//   * update_scales: one tiny launch per step for ALL fp8 tensors: push each
//     amax into its history ring, recompute scale and 1/scale.
// gfx950 uses the OCP e4m3fn encoding (not MI300's fnuz); the conversion is
// v_cvt_pk_fp8_f32 after an explicit clamp to +-448 (saturating cast).
#include "common.h"
#include "kernels.h"

namespace bpe {

// FP8_E4M3_MAX / FP8_E5M2_MAX and the saturating pack4_fp8<FMT> live in common.h (the GEMM epilogues cast too)

template <typename T, int FMT>
__global__ void __launch_bounds__(256) cast_fp8_kernel(const T* __restrict__ x, size_t n, const float* __restrict__ scale,
                                                       uint8_t* __restrict__ out, unsigned* __restrict__ amax_bits) {
    constexpr int V = Vec<T>::N;  // 8 bf16 / 4 fp32 per 16-byte load
    const float s = *scale;
    float am = 0.f;
    const size_t nv = n / V;
    for (size_t i = blockIdx.x * (size_t)256 + threadIdx.x; i < nv; i += (size_t)gridDim.x * 256) {
        Vec<T> a;
        a.load(x + i * V);
#pragma unroll
        for (int j = 0; j < V; ++j) am = fmaxf(am, fabsf(a.v[j]));
        if constexpr (V == 8) {
            uint2 o = {pack4_fp8<FMT>(a.v[0] * s, a.v[1] * s, a.v[2] * s, a.v[3] * s),
                       pack4_fp8<FMT>(a.v[4] * s, a.v[5] * s, a.v[6] * s, a.v[7] * s)};
            *reinterpret_cast<uint2*>(out + i * V) = o;
        } else {
            *reinterpret_cast<unsigned*>(out + i * V) =
                pack4_fp8<FMT>(a.v[0] * s, a.v[1] * s, a.v[2] * s, a.v[3] * s);
        }
    }
    // scalar tail
    const size_t t = nv * V + blockIdx.x * (size_t)256 + threadIdx.x;
    if (blockIdx.x == 0 && t < n) {
        const float v = ld1<T>(x + t);
        am = fmaxf(am, fabsf(v));
        out[t] = (uint8_t)(pack4_fp8<FMT>(v * s, 0.f, 0.f, 0.f) & 0xFF);
    }
    // one atomic per block: thousands of same-address atomics serialise at the L2 (measured 170 us per
    // 67 MB cast with per-wave atomics vs ~25 us of streaming)
    __shared__ float red[4];
    am = block_max(am, red);
    if (threadIdx.x == 0 && amax_bits) atomicMax(amax_bits, __float_as_uint(am));
}

// Two-layout cast: W [N][K] bf16 -> w8 [N][K] AND w8t [K][N] (FMT 0 e4m3 / 1 e5m2), one pass, amax folded in.
// Weights: the input-gradient GEMM dX = dY . W needs W with the reduction index (N) contiguous; writing that
// copy here replaces a strided PyTorch transpose of the fp8 weight per GEMM (~0.3 TB/s).  Activations and output
// gradients: the fp8 weight-gradient GEMM dW = dY^T . X reduces over tokens, so both operands are wanted with the
// token index contiguous ([N][T], [K][T]) -- the layout of the fp8 kernel and of the library.  64 x 64 tiles
// through LDS (row stride 68 B: the transposed byte reads of one wave spread over the banks); a grid-stride loop
// over the tiles, so one amax atomic per workgroup stays a few thousand at most.
template <int FMT>
__global__ void __launch_bounds__(256) cast_fp8_t_kernel(const __bf16* __restrict__ w, int N, int K,
                                                         const float* __restrict__ scale, uint8_t* __restrict__ w8,
                                                         uint8_t* __restrict__ w8t, unsigned* __restrict__ amax_bits) {
    __shared__ uint8_t tile[64][68];
    __shared__ float red[4];
    const int tid = threadIdx.x;
    const int tiles_k = K / 64, ntiles = (N / 64) * tiles_k;
    const float sc = *scale;
    const int r = tid >> 2, c = (tid & 3) * 16;
    float am = 0.f;
    for (int t = blockIdx.x; t < ntiles; t += gridDim.x) {
        const int n0 = (t / tiles_k) * 64, k0 = (t % tiles_k) * 64;
        const __bf16* src = w + (long)(n0 + r) * K + k0 + c;
        const u16x8 a = *reinterpret_cast<const u16x8*>(src);
        const u16x8 b = *reinterpret_cast<const u16x8*>(src + 8);
        float v[16];
#pragma unroll
        for (int j = 0; j < 8; ++j) { v[j] = bf2f(a[j]); v[8 + j] = bf2f(b[j]); }
#pragma unroll
        for (int j = 0; j < 16; ++j) am = fmaxf(am, fabsf(v[j]));
        uint4 q;
        q.x = pack4_fp8<FMT>(v[0] * sc, v[1] * sc, v[2] * sc, v[3] * sc);
        q.y = pack4_fp8<FMT>(v[4] * sc, v[5] * sc, v[6] * sc, v[7] * sc);
        q.z = pack4_fp8<FMT>(v[8] * sc, v[9] * sc, v[10] * sc, v[11] * sc);
        q.w = pack4_fp8<FMT>(v[12] * sc, v[13] * sc, v[14] * sc, v[15] * sc);
        *reinterpret_cast<uint4*>(w8 + (long)(n0 + r) * K + k0 + c) = q;
        const unsigned qq[4] = {q.x, q.y, q.z, q.w};
        __syncthreads();  // the previous tile's transposed reads are done
#pragma unroll
        for (int j = 0; j < 4; ++j) *reinterpret_cast<unsigned*>(&tile[r][c + 4 * j]) = qq[j];
        __syncthreads();
        // transposed: thread -> output row k0 + r (a column of the tile), 16 consecutive n
        unsigned o[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            unsigned x = 0;
#pragma unroll
            for (int e = 0; e < 4; ++e) x |= (unsigned)tile[c + 4 * j + e][r] << (8 * e);
            o[j] = x;
        }
        *reinterpret_cast<uint4*>(w8t + (long)(k0 + r) * N + n0 + c) = uint4{o[0], o[1], o[2], o[3]};
    }
    am = block_max(am, red);
    if (tid == 0 && amax_bits) atomicMax(amax_bits, __float_as_uint(am));
}

// 128 x 128 fp8 tile transpose through LDS (the two-layout casts below).  Row-major phase (c128_put): thread t holds
// tile rows 16 i + (t >> 4), i = 0 .. 7, columns 8 (t & 15) .. + 7 -- one load instruction of a wave reads 4 whole
// tile rows (8 whole 128-byte lines of bf16) and one row-major fp8 store writes 4 whole 128-byte lines.  Transposed
// phase (t128_get_store): thread t emits output rows 4 kq .. 4 kq + 3 (kq = t >> 3) over tile rows 16 ns .. 16 ns +
// 15 (ns = t & 7): the 8 ns of one kq are adjacent lanes, so one store instruction of a wave writes 8 whole 128-byte
// output rows.  LDS word column c of tile row n sits at c ^ sw(n), so the column reads of a 32-lane half (4 kq x 8
// ns) hit 32 distinct banks.
// Measured, round 5 (profiles/bench/ab_fp8_cast_coalesced_r5.log): the earlier row-pair mapping (thread pair t, t + 1
// on the two 64-column halves of tile row t >> 1, so one load instruction touched 64 lines 16 bytes at a time) ran the
// two-layout cast at 4.4-4.5 TB/s and the SwiGLU casts at 4.1-4.2; this mapping 4.9 / 4.8-4.9 TB/s (the same bytes),
// fp8 Llama step 191.5-192.9 k -> 195.7-196.4 k tok/s.  Prefetching the next tile's bf16 rows in the SwiGLU casts
// measured the same and is not kept.
// Plain (temporal) loads and stores in the 128 x 128 casts.  Measured and dropped, round 5: the non-temporal hint
// (common.h ld_stream / st_stream, which took the softmax-CE kernel from 5.1 to 5.5 TB/s) halved these kernels -- the
// two-layout cast 4.5 -> 2.5 TB/s, the SwiGLU casts 4.0-4.2 -> 1.8-1.9 TB/s, the fp8 Llama step 192.0 k -> 166.6 k
// tok/s (profiles/bench/ab_fp8_cast_nt_r5.log): their transposed stores write 16-byte pieces of many lines per
// instruction, which non-temporal stores do not combine.
__device__ __forceinline__ u16x8 ld8(const __bf16* p) { return *reinterpret_cast<const u16x8*>(p); }
__device__ __forceinline__ void st16(uint8_t* p, unsigned a, unsigned b, unsigned c, unsigned d) {
    *reinterpret_cast<uint4*>(p) = uint4{a, b, c, d};
}

constexpr int T128_TS = 132;  // LDS row stride (bytes): 33 words
__device__ __forceinline__ int t128_sw(int n) { return ((n >> 4) & 7) << 2; }

// dst = output row 4 kq of the transposed tile at column 16 ns; ld = output row stride (bytes)
__device__ __forceinline__ void t128_get_store(const uint8_t* tile, int kq, int ns, uint8_t* dst, long ld) {
    unsigned o[4][4];  // [k offset e][n group g]: bytes n = 16 ns + 4 g .. +3 of output row 4 kq + e
#pragma unroll
    for (int g = 0; g < 4; ++g) {
        const int n = 16 * ns + 4 * g, cw = 4 * (kq ^ t128_sw(n));  // sw is the same for the 16 rows of ns
        const unsigned x0 = *reinterpret_cast<const unsigned*>(&tile[(n + 0) * T128_TS + cw]);
        const unsigned x1 = *reinterpret_cast<const unsigned*>(&tile[(n + 1) * T128_TS + cw]);
        const unsigned x2 = *reinterpret_cast<const unsigned*>(&tile[(n + 2) * T128_TS + cw]);
        const unsigned x3 = *reinterpret_cast<const unsigned*>(&tile[(n + 3) * T128_TS + cw]);
        // v_perm_b32(s0, s1, sel): selector byte 0-3 takes that byte of s1, 4-7 byte (sel - 4) of s0
        const unsigned lo01 = __builtin_amdgcn_perm(x1, x0, 0x05010400u);  // x0.0 x1.0 x0.1 x1.1
        const unsigned hi01 = __builtin_amdgcn_perm(x1, x0, 0x07030602u);  // x0.2 x1.2 x0.3 x1.3
        const unsigned lo23 = __builtin_amdgcn_perm(x3, x2, 0x05010400u);
        const unsigned hi23 = __builtin_amdgcn_perm(x3, x2, 0x07030602u);
        o[0][g] = __builtin_amdgcn_perm(lo23, lo01, 0x05040100u);  // x0.0 x1.0 x2.0 x3.0
        o[1][g] = __builtin_amdgcn_perm(lo23, lo01, 0x07060302u);
        o[2][g] = __builtin_amdgcn_perm(hi23, hi01, 0x05040100u);
        o[3][g] = __builtin_amdgcn_perm(hi23, hi01, 0x07060302u);
    }
#pragma unroll
    for (int e = 0; e < 4; ++e) st16(dst + e * ld, o[e][0], o[e][1], o[e][2], o[e][3]);
}

// raw barrier behind lgkmcnt(0) only: LDS hand-off without waiting for outstanding global loads / stores
__device__ __forceinline__ void lds_barrier() {
    __builtin_amdgcn_s_waitcnt(0xc07f);
    __builtin_amdgcn_s_barrier();
}

// SwiGLU with the two-layout fp8 cast fused in (the fp8 weight-gradient path, where no bf16 copy of these tensors
// is kept): MODE 0 forms a = silu(g) u from gu = [g | u] ([M][2F]) and writes a8 [M][F] and a8t [F][M] (FMT e4m3, the
// W2 projection's input); MODE 1 forms the gate gradient [dg | du] from dout = dA [M][F] and gu and writes dgu8
// [M][2F] and dgu8t [2F][M] (FMT e5m2, the W13 projection's output gradient).  Each value is rounded to bf16 exactly
// as swiglu_fwd / swiglu_bwd (activations.hip) store it before it is scaled and converted, so the outputs and the
// amax equal those of the two-pass form (SwiGLU kernel, then cast_fp8_t) while the bf16 tensor's write and re-read
// disappear.  64 x 64 tiles of (tokens, F columns) through LDS as in cast_fp8_t_kernel.
template <int MODE, int FMT>
__global__ void __launch_bounds__(256) swiglu_cast_fp8_t_kernel(const __bf16* __restrict__ gu,
                                                                const __bf16* __restrict__ dout, int M, int F,
                                                                const float* __restrict__ scale,
                                                                uint8_t* __restrict__ o8, uint8_t* __restrict__ o8t,
                                                                unsigned* __restrict__ amax_bits) {
    constexpr int NO = MODE == 0 ? 1 : 2;  // output column blocks per tile: a, or dg and du
    __shared__ uint8_t tile[NO][64][68];
    __shared__ float red[4];
    const int tid = threadIdx.x;
    const int tiles_f = F / 64, ntiles = (M / 64) * tiles_f;
    const long W = (long)NO * F;  // output row length
    const float sc = *scale;
    const int r = tid >> 2, c = (tid & 3) * 16;
    float am = 0.f;
    for (int t = blockIdx.x; t < ntiles; t += gridDim.x) {
        const int m0 = (t / tiles_f) * 64, f0 = (t % tiles_f) * 64;
        const __bf16* row = gu + (long)(m0 + r) * 2 * F + f0 + c;
        const u16x8 g0 = *reinterpret_cast<const u16x8*>(row), g1 = *reinterpret_cast<const u16x8*>(row + 8);
        const u16x8 u0 = *reinterpret_cast<const u16x8*>(row + F), u1 = *reinterpret_cast<const u16x8*>(row + F + 8);
        u16x8 d0{}, d1{};
        if constexpr (MODE == 1) {
            const __bf16* dr = dout + (long)(m0 + r) * F + f0 + c;
            d0 = *reinterpret_cast<const u16x8*>(dr);
            d1 = *reinterpret_cast<const u16x8*>(dr + 8);
        }
        float v[NO][16];
#pragma unroll
        for (int j = 0; j < 16; ++j) {
            const float g = bf2f(j < 8 ? g0[j] : g1[j - 8]), u = bf2f(j < 8 ? u0[j] : u1[j - 8]);
            const float sg = fast_sigmoid(g);
            if constexpr (MODE == 0) {
                v[0][j] = bf2f(f2bf(g * sg * u));
            } else {
                const float d = bf2f(j < 8 ? d0[j] : d1[j - 8]);
                const float silu = g * sg;
                v[1][j] = bf2f(f2bf(d * silu));                            // du
                v[0][j] = bf2f(f2bf(d * u * sg * (1.f + g * (1.f - sg))));  // dg
            }
        }
        uint4 q[NO];
#pragma unroll
        for (int o = 0; o < NO; ++o) {
#pragma unroll
            for (int j = 0; j < 16; ++j) am = fmaxf(am, fabsf(v[o][j]));
            q[o].x = pack4_fp8<FMT>(v[o][0] * sc, v[o][1] * sc, v[o][2] * sc, v[o][3] * sc);
            q[o].y = pack4_fp8<FMT>(v[o][4] * sc, v[o][5] * sc, v[o][6] * sc, v[o][7] * sc);
            q[o].z = pack4_fp8<FMT>(v[o][8] * sc, v[o][9] * sc, v[o][10] * sc, v[o][11] * sc);
            q[o].w = pack4_fp8<FMT>(v[o][12] * sc, v[o][13] * sc, v[o][14] * sc, v[o][15] * sc);
            *reinterpret_cast<uint4*>(o8 + (long)(m0 + r) * W + (long)o * F + f0 + c) = q[o];
        }
        __syncthreads();  // the previous tile's transposed reads are done
#pragma unroll
        for (int o = 0; o < NO; ++o) {
            const unsigned qq[4] = {q[o].x, q[o].y, q[o].z, q[o].w};
#pragma unroll
            for (int j = 0; j < 4; ++j) *reinterpret_cast<unsigned*>(&tile[o][r][c + 4 * j]) = qq[j];
        }
        __syncthreads();
        // transposed: thread -> output row (o F + f0 + r), 16 consecutive tokens m0 + c ..
#pragma unroll
        for (int o = 0; o < NO; ++o) {
            unsigned w4[4];
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                unsigned x = 0;
#pragma unroll
                for (int e = 0; e < 4; ++e) x |= (unsigned)tile[o][c + 4 * j + e][r] << (8 * e);
                w4[j] = x;
            }
            *reinterpret_cast<uint4*>(o8t + ((long)o * F + f0 + r) * M + m0 + c) = uint4{w4[0], w4[1], w4[2], w4[3]};
        }
    }
    am = block_max(am, red);
    if (tid == 0 && amax_bits) atomicMax(amax_bits, __float_as_uint(am));
}

// q[2 i], q[2 i + 1]: fp8 words cw, cw + 1 of tile row r0 + 16 i (the row-major phase above)
__device__ __forceinline__ void c128_put(uint8_t* tile, const unsigned (&q)[16], int r0, int cw) {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        const int r = r0 + 16 * i;
#pragma unroll
        for (int j = 0; j < 2; ++j) *reinterpret_cast<unsigned*>(&tile[r * T128_TS + 4 * ((cw + j) ^ t128_sw(r))]) = q[2 * i + j];
    }
}

// The two-layout cast on 128 x 128 tiles (N, K multiples of 128): every output row segment a thread group writes is a
// whole 128-byte line in both layouts (the 64 x 64 kernel writes 64-byte halves, 3.4-3.5 TB/s effective against
// 5.4-5.5 for the one-layout cast, profiles/bench/cast_bench_r4.log), and the next tile's loads are issued as soon as
// this tile's values are converted, so they are in flight through the stores and the LDS transpose (raw barriers
// behind lgkmcnt(0) only: __syncthreads would also wait for those loads).  Transposed reads: a thread takes one 32-bit
// word (4 k values) from each of 16 tile rows and turns every 4 x 4 byte block around with v_perm_b32, so it stores 16
// consecutive n for each of its 4 output rows.
template <int FMT>
__global__ void __launch_bounds__(256) cast_fp8_c128_kernel(const __bf16* __restrict__ w, int N, int K,
                                                            const float* __restrict__ scale, uint8_t* __restrict__ w8,
                                                            uint8_t* __restrict__ w8t,
                                                            unsigned* __restrict__ amax_bits) {
    __shared__ __attribute__((aligned(16))) uint8_t tile[128 * T128_TS];
    __shared__ float red[4];
    const int tid = threadIdx.x;
    const int tiles_k = K / 128, ntiles = (N / 128) * tiles_k;
    const float sc = *scale;
    const int r0 = tid >> 4, c8 = (tid & 15) * 8;
    const int kq = tid >> 3, ns = tid & 7;
    float am = 0.f;
    u16x8 a[8];
    auto load = [&](int tt) {
        const int n0 = (tt / tiles_k) * 128, k0 = (tt % tiles_k) * 128;
        const __bf16* src = w + (long)(n0 + r0) * K + k0 + c8;
#pragma unroll
        for (int i = 0; i < 8; ++i) a[i] = ld8(src + (long)16 * i * K);
    };
    if (blockIdx.x < ntiles) load(blockIdx.x);
    for (int t = blockIdx.x; t < ntiles; t += gridDim.x) {
        const int n0 = (t / tiles_k) * 128, k0 = (t % tiles_k) * 128;
        unsigned q[16];
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            float v[8];
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                v[j] = bf2f(a[i][j]);
                am = fmaxf(am, fabsf(v[j]));
            }
            q[2 * i] = pack4_fp8<FMT>(v[0] * sc, v[1] * sc, v[2] * sc, v[3] * sc);
            q[2 * i + 1] = pack4_fp8<FMT>(v[4] * sc, v[5] * sc, v[6] * sc, v[7] * sc);
        }
        if (t + (int)gridDim.x < ntiles) load(t + gridDim.x);
        uint8_t* dst = w8 + (long)(n0 + r0) * K + k0 + c8;
#pragma unroll
        for (int i = 0; i < 8; ++i) *reinterpret_cast<uint2*>(dst + (long)16 * i * K) = uint2{q[2 * i], q[2 * i + 1]};
        lds_barrier();  // the previous tile's transposed reads are done
        c128_put(tile, q, r0, c8 / 4);
        lds_barrier();
        t128_get_store(tile, kq, ns, w8t + (long)(k0 + 4 * kq) * N + n0 + 16 * ns, N);
    }
    am = block_max(am, red);
    if (tid == 0 && amax_bits) atomicMax(amax_bits, __float_as_uint(am));
}

// The SwiGLU + two-layout cast on 128 x 128 tiles (M and F multiples of 128).  Values, rounding and amax as
// swiglu_cast_fp8_t_kernel; the thread mapping of cast_fp8_c128_kernel.
template <int MODE, int FMT>
__global__ void __launch_bounds__(256) swiglu_cast_fp8_c128_kernel(const __bf16* __restrict__ gu,
                                                                   const __bf16* __restrict__ dout, int M, int F,
                                                                   const float* __restrict__ scale,
                                                                   uint8_t* __restrict__ o8, uint8_t* __restrict__ o8t,
                                                                   unsigned* __restrict__ amax_bits) {
    constexpr int NO = MODE == 0 ? 1 : 2;
    __shared__ __attribute__((aligned(16))) uint8_t tile[NO][128 * T128_TS];
    __shared__ float red[4];
    const int tid = threadIdx.x;
    const int tiles_f = F / 128, ntiles = (M / 128) * tiles_f;
    const long W = (long)NO * F;
    const float sc = *scale;
    const int r0 = tid >> 4, c8 = (tid & 15) * 8;
    const int kq = tid >> 3, ns = tid & 7;
    float am = 0.f;
    u16x8 g[8], u[8], d[MODE == 1 ? 8 : 1];
    auto load = [&](int tt) {
        const int m0 = (tt / tiles_f) * 128, f0 = (tt % tiles_f) * 128;
        const __bf16* row = gu + (long)(m0 + r0) * 2 * F + f0 + c8;
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            g[i] = ld8(row + (long)16 * i * 2 * F);
            u[i] = ld8(row + (long)16 * i * 2 * F + F);
        }
        if constexpr (MODE == 1) {
            const __bf16* dr = dout + (long)(m0 + r0) * F + f0 + c8;
#pragma unroll
            for (int i = 0; i < 8; ++i) d[i] = ld8(dr + (long)16 * i * F);
        }
    };
    for (int t = blockIdx.x; t < ntiles; t += gridDim.x) {
        const int m0 = (t / tiles_f) * 128, f0 = (t % tiles_f) * 128;
        load(t);
        unsigned q[NO][16];
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            float v[NO][8];
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                const float gg = bf2f(g[i][j]), uu = bf2f(u[i][j]);
                const float sg = fast_sigmoid(gg);
                if constexpr (MODE == 0) {
                    v[0][j] = bf2f(f2bf(gg * sg * uu));
                } else {
                    const float dd = bf2f(d[i][j]);
                    const float silu = gg * sg;
                    v[1][j] = bf2f(f2bf(dd * silu));                               // du
                    v[0][j] = bf2f(f2bf(dd * uu * sg * (1.f + gg * (1.f - sg))));  // dg
                }
            }
#pragma unroll
            for (int o = 0; o < NO; ++o) {
#pragma unroll
                for (int j = 0; j < 8; ++j) am = fmaxf(am, fabsf(v[o][j]));
                q[o][2 * i] = pack4_fp8<FMT>(v[o][0] * sc, v[o][1] * sc, v[o][2] * sc, v[o][3] * sc);
                q[o][2 * i + 1] = pack4_fp8<FMT>(v[o][4] * sc, v[o][5] * sc, v[o][6] * sc, v[o][7] * sc);
            }
        }
#pragma unroll
        for (int o = 0; o < NO; ++o) {
            uint8_t* dst = o8 + (long)(m0 + r0) * W + (long)o * F + f0 + c8;
#pragma unroll
            for (int i = 0; i < 8; ++i)
                *reinterpret_cast<uint2*>(dst + (long)16 * i * W) = uint2{q[o][2 * i], q[o][2 * i + 1]};
        }
        lds_barrier();  // the previous tile's transposed reads are done
#pragma unroll
        for (int o = 0; o < NO; ++o) c128_put(tile[o], q[o], r0, c8 / 4);
        lds_barrier();
#pragma unroll
        for (int o = 0; o < NO; ++o)
            t128_get_store(tile[o], kq, ns, o8t + ((long)o * F + f0 + 4 * kq) * M + m0 + 16 * ns, M);
    }
    am = block_max(am, red);
    if (tid == 0 && amax_bits) atomicMax(amax_bits, __float_as_uint(am));
}

// Residual add + RMSNorm with an fp8 output (the fp8 weight-gradient path, where the normalised activation only
// feeds fp8 GEMMs): s = x + d (bf16, stored: the residual stream; d == nullptr: s = x, not stored), rstd stored,
// and y = s * rstd * w -- rounded to bf16 exactly as add_rmsnorm_fwd / rmsnorm_fwd store it -- written only as
// e4m3 [M][N] (scale, amax folded in); transpose_fp8_c128_kernel then writes [N][M].  One wave per row, C 16-byte
// chunks per lane (N / 8 <= 64 C).  Against the norm + two-layout cast pair it drops the bf16 y write and its re-read.
template <int C>
__global__ void __launch_bounds__(256) add_rmsnorm_fp8_kernel(const __bf16* __restrict__ x, const __bf16* __restrict__ d,
                                                              const __bf16* __restrict__ w, __bf16* __restrict__ sum,
                                                              uint8_t* __restrict__ y8, float* __restrict__ rstd_out,
                                                              int M, int N, float eps, const float* __restrict__ scale,
                                                              unsigned* __restrict__ amax_bits) {
    __shared__ float red[4];
    const int lane = threadIdx.x & 63;
    const int nvec = N / 8;
    float am = 0.f;
    // a grid-stride loop over rows (one wave per row) on a capped grid: one amax atomic per workgroup stays a few
    // hundred (one per 4 rows serialised at the L2: 236 us per 65 536 x 2048 call against ~170 us)
    for (int row = blockIdx.x * 4 + (threadIdx.x >> 6); row < M; row += gridDim.x * 4) {
        const size_t off = (size_t)row * N;
        float ss = 0.f;
        Vec<__bf16> keep[C];
#pragma unroll
        for (int c = 0; c < C; ++c) {
            const int i = c * 64 + lane;
            if (i < nvec) {
                Vec<__bf16> a;
                a.load(x + off + i * 8);
                if (d != nullptr) {
                    Vec<__bf16> b;
                    b.load(d + off + i * 8);
#pragma unroll
                    for (int j = 0; j < 8; ++j) a.v[j] = bf2f(f2bf(a.v[j] + b.v[j]));
                    a.store(sum + off + i * 8);
                }
#pragma unroll
                for (int j = 0; j < 8; ++j) ss += a.v[j] * a.v[j];
                keep[c] = a;
            }
        }
        ss = wave_sum(ss);
        const float r = rsqrtf(ss / (float)N + eps);
        if (lane == 0) rstd_out[row] = r;
        const float sc = *scale;
#pragma unroll
        for (int c = 0; c < C; ++c) {
            const int i = c * 64 + lane;
            if (i < nvec) {
                Vec<__bf16> g;
                g.load(w + i * 8);
                float v[8];
#pragma unroll
                for (int j = 0; j < 8; ++j) {
                    v[j] = bf2f(f2bf(keep[c].v[j] * r * g.v[j]));
                    am = fmaxf(am, fabsf(v[j]));
                }
                *reinterpret_cast<uint2*>(y8 + off + i * 8) =
                    uint2{pack4_fp8<0>(v[0] * sc, v[1] * sc, v[2] * sc, v[3] * sc),
                          pack4_fp8<0>(v[4] * sc, v[5] * sc, v[6] * sc, v[7] * sc)};
            }
        }
    }
    am = block_max(am, red);
    if (threadIdx.x == 0) atomicMax(amax_bits, __float_as_uint(am));
}

// fp8 [M][N] -> [N][M] (M, N multiples of 128) through the 128 x 128 tile helpers above: thread t reads tile rows
// 32 i + (t >> 3), i = 0 .. 3, bytes 16 (t & 7) .. + 15, so one load instruction of a wave reads 8 whole 128-byte rows
__global__ void __launch_bounds__(256) transpose_fp8_c128_kernel(const uint8_t* __restrict__ a, uint8_t* __restrict__ at,
                                                                 int M, int N) {
    __shared__ __attribute__((aligned(16))) uint8_t tile[128 * T128_TS];
    const int tid = threadIdx.x;
    const int tiles_n = N / 128, ntiles = (M / 128) * tiles_n;
    const int r0 = tid >> 3, cw = (tid & 7) * 4, kq = tid >> 3, ns = tid & 7;
    for (int t = blockIdx.x; t < ntiles; t += gridDim.x) {
        const int m0 = (t / tiles_n) * 128, n0 = (t % tiles_n) * 128;
        const uint8_t* src = a + (long)(m0 + r0) * N + n0 + 4 * cw;
        uint4 q[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) q[i] = *reinterpret_cast<const uint4*>(src + (long)32 * i * N);
        lds_barrier();  // the previous tile's transposed reads are done
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int r = r0 + 32 * i;
            const unsigned w[4] = {q[i].x, q[i].y, q[i].z, q[i].w};
#pragma unroll
            for (int j = 0; j < 4; ++j) *reinterpret_cast<unsigned*>(&tile[r * T128_TS + 4 * ((cw + j) ^ t128_sw(r))]) = w[j];
        }
        lds_barrier();
        t128_get_store(tile, kq, ns, at + (long)(n0 + 4 * kq) * M + m0 + 16 * ns, M);
    }
}

// amax_cur [n] (float bits, zeroed here after use), hist [n][H], scale/inv [n]
__global__ void __launch_bounds__(256) update_scales_kernel(unsigned* __restrict__ amax_cur, float* __restrict__ hist,
                                                            float* __restrict__ scale, float* __restrict__ inv_scale,
                                                            int n, int H, int pos, float margin, float fmax) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    const float a = __uint_as_float(amax_cur[i]);
    amax_cur[i] = 0u;
    hist[(size_t)i * H + pos] = a;
    float m = 0.f;
    for (int k = 0; k < H; ++k) m = fmaxf(m, hist[(size_t)i * H + k]);
    float s = (m > 0.f && isfinite(m)) ? fmax / (m * margin) : 1.f;
    // keep scales powers of two: exact dequantisation, no rounding drift between steps
    s = exp2f(floorf(log2f(s)));
    scale[i] = s;
    inv_scale[i] = 1.f / s;
}

}  // namespace bpe

using namespace bpe;

// 1: the 128 x 128 tile kernels where the shape allows (a variant build with 0 keeps the 64 x 64 ones for A/B)
#ifndef BPE_CAST_T128
#define BPE_CAST_T128 1
#endif

void launch_cast_fp8(int dtype, int fmt, const void* x, size_t n, const float* scale, void* out,
                     unsigned* amax_bits, hipStream_t s) {
    if (n == 0) return;
    const int V = dtype == DT_BF16 ? 8 : 4;
    const int grid = stream_grid(n / V + 1, 256, 1024);
#define CAST(T, F) cast_fp8_kernel<T, F><<<grid, 256, 0, s>>>((const T*)x, n, scale, (uint8_t*)out, amax_bits)
    if (dtype == DT_BF16) { if (fmt == 0) CAST(__bf16, 0); else CAST(__bf16, 1); }
    else { if (fmt == 0) CAST(float, 0); else CAST(float, 1); }
#undef CAST
}

void launch_cast_fp8_t(const void* w, int N, int K, const float* scale, void* w8, void* w8t, unsigned* amax_bits,
                       int fmt, hipStream_t s) {
    if (BPE_CAST_T128 && N % 128 == 0 && K % 128 == 0) {
        const int nt = (N / 128) * (K / 128);
        const int g = nt < 2048 ? nt : 2048;
        if (fmt == 0)
            cast_fp8_c128_kernel<0><<<g, 256, 0, s>>>((const __bf16*)w, N, K, scale, (uint8_t*)w8, (uint8_t*)w8t,
                                                      amax_bits);
        else
            cast_fp8_c128_kernel<1><<<g, 256, 0, s>>>((const __bf16*)w, N, K, scale, (uint8_t*)w8, (uint8_t*)w8t,
                                                      amax_bits);
        return;
    }
    const int ntiles = (N / 64) * (K / 64);
    const int grid = ntiles < 2048 ? ntiles : 2048;
    if (fmt == 0)
        cast_fp8_t_kernel<0><<<grid, 256, 0, s>>>((const __bf16*)w, N, K, scale, (uint8_t*)w8, (uint8_t*)w8t,
                                                  amax_bits);
    else
        cast_fp8_t_kernel<1><<<grid, 256, 0, s>>>((const __bf16*)w, N, K, scale, (uint8_t*)w8, (uint8_t*)w8t,
                                                  amax_bits);
}

void launch_swiglu_cast_fp8_t(int mode, const void* gu, const void* dout, int M, int F, const float* scale, void* o8,
                              void* o8t, unsigned* amax_bits, hipStream_t s) {
    if (BPE_CAST_T128 && M % 128 == 0 && F % 128 == 0) {
        const int nt = (M / 128) * (F / 128);
        const int g = nt < 2048 ? nt : 2048;
        if (mode == 0)
            swiglu_cast_fp8_c128_kernel<0, 0><<<g, 256, 0, s>>>((const __bf16*)gu, nullptr, M, F, scale,
                                                                (uint8_t*)o8, (uint8_t*)o8t, amax_bits);
        else
            swiglu_cast_fp8_c128_kernel<1, 1><<<g, 256, 0, s>>>((const __bf16*)gu, (const __bf16*)dout, M, F, scale,
                                                                (uint8_t*)o8, (uint8_t*)o8t, amax_bits);
        return;
    }
    const int ntiles = (M / 64) * (F / 64);
    const int grid = ntiles < 2048 ? ntiles : 2048;
    if (mode == 0)
        swiglu_cast_fp8_t_kernel<0, 0><<<grid, 256, 0, s>>>((const __bf16*)gu, nullptr, M, F, scale, (uint8_t*)o8,
                                                            (uint8_t*)o8t, amax_bits);
    else
        swiglu_cast_fp8_t_kernel<1, 1><<<grid, 256, 0, s>>>((const __bf16*)gu, (const __bf16*)dout, M, F, scale,
                                                            (uint8_t*)o8, (uint8_t*)o8t, amax_bits);
}

void launch_add_rmsnorm_cast_fp8_t(const void* x, const void* d, const void* w, void* sum, void* y8, void* y8t,
                                   float* rstd, int M, int N, float eps, const float* scale, unsigned* amax_bits,
                                   hipStream_t s) {
    const int rows4 = (M + 3) / 4;
    const int grid = rows4 < 1024 ? rows4 : 1024;
    const int chunks = (N / 8 + 63) / 64;
#define ARF(CC)                                                                                                  \
    add_rmsnorm_fp8_kernel<CC><<<grid, 256, 0, s>>>((const __bf16*)x, (const __bf16*)d, (const __bf16*)w,        \
                                                    (__bf16*)sum, (uint8_t*)y8, rstd, M, N, eps, scale, amax_bits)
    if (chunks <= 1) ARF(1);
    else if (chunks <= 2) ARF(2);
    else ARF(4);
#undef ARF
    const int nt = (M / 128) * (N / 128);
    transpose_fp8_c128_kernel<<<nt < 2048 ? nt : 2048, 256, 0, s>>>((const uint8_t*)y8, (uint8_t*)y8t, M, N);
}

void launch_update_scales(unsigned* amax_cur, float* hist, float* scale, float* inv_scale, int n, int H, int pos,
                          float margin, int fmt, hipStream_t s) {
    update_scales_kernel<<<(n + 255) / 256, 256, 0, s>>>(amax_cur, hist, scale, inv_scale, n, H, pos, margin,
                                                         fmt == 0 ? FP8_E4M3_MAX : FP8_E5M2_MAX);
}
