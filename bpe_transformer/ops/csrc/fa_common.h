// Shared device helpers of the flash-attention kernels (gfx950).
//
// LDS tile layout: rows of RB = 2*D bytes; 16-byte chunk c of row r is stored
// at chunk c ^ sigma(r).  For 128-byte rows (D = 64)
//     sigma(r) = ((r >> 1) & 1) << 2 | ((r >> 2) & 3)
// makes BOTH access kinds conflict-free (bank rule: MI355X_MICROARCH §LDS):
//   * ds_read_b128 row reads (MFMA operand rows): every 16-lane group reads 16
//     distinct rows r at one logical chunk; (r & 1, sigma(r)) are distinct over
//     the group, i.e. 16 distinct 16-byte slots of the 256-byte bank row;
//   * ds_read_b64_tr_b16 column reads: a 32-lane half reads 4 rows r0..r0+3
//     (r0 % 4 == 0) x one 64-byte column half; rows r0 and r0+2 differ in bit 2
//     of sigma, so the four rows land in the four distinct 64-byte quarters.
// For 256-byte rows (D = 128) sigma(r) = (r & 3) << 2 | ((r >> 2) & 3)
// (guide T10 image (b)).
#pragma once
#include "common.h"

#include <cstdlib>

namespace bpe {
namespace fa {

typedef short v4s __attribute__((ext_vector_type(4)));
typedef short v8s __attribute__((ext_vector_type(8)));
typedef __attribute__((address_space(3))) v4s lds_v4s;

constexpr float LOG2E = 1.4426950408889634f;

template <int RB>
__device__ __forceinline__ int swz(int row, int c) {
    if constexpr (RB == 128) {
        const int sg = (((row >> 1) & 1) << 2) | ((row >> 2) & 3);
        return row * 128 + ((c ^ sg) << 4);
    } else {
        const int sg = ((row & 3) << 2) | ((row >> 2) & 3);
        return row * 256 + ((c ^ sg) << 4);
    }
}

// byte offset of the 8-byte granule at (row, col) of a swizzled tile (tr reads / 8-byte writes)
template <int RB>
__device__ __forceinline__ int tr_off(int row, int col) {
    return swz<RB>(row, col >> 3) + ((col & 7) << 1);
}

__device__ __forceinline__ bf16x8 lds_row16(const char* smem, int off) {
    return __builtin_bit_cast(bf16x8, *reinterpret_cast<const u16x8*>(smem + off));
}

// Two transposed 4x16 reads (ds_read_b64_tr_b16) -> one 8-element MFMA operand.
__device__ __forceinline__ bf16x8 lds_tr_pair(char* smem, int off0, int off1) {
    v4s lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s*)(smem + off0));
    v4s hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s*)(smem + off1));
    v8s c = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
    return __builtin_bit_cast(bf16x8, c);
}

__device__ __forceinline__ f32x16 mfma(bf16x8 a, bf16x8 b, f32x16 c) {
    return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}

// 32x32 accumulator register r of lane-half hh -> row inside the tile (column = lane & 31)
__device__ __forceinline__ int acc_row(int r, int hh) { return (r & 3) + 8 * (r >> 2) + 4 * hh; }

__device__ __forceinline__ float fast_exp2(float x) { return __builtin_amdgcn_exp2f(x); }

__device__ __forceinline__ void unpack8(const u16x8& t, float* x) {
#pragma unroll
    for (int i = 0; i < 8; ++i) x[i] = bf2f(t[i]);
}

// interleaved RoPE on 8 consecutive elements (4 pairs); cs/sn point at the pair index of x[0]
__device__ __forceinline__ void rope8(float* x, const float* cs, const float* sn) {
    const f32x4 c = *reinterpret_cast<const f32x4*>(cs);
    const f32x4 s = *reinterpret_cast<const f32x4*>(sn);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const float a = x[2 * i], b = x[2 * i + 1];
        x[2 * i] = a * c[i] - b * s[i];
        x[2 * i + 1] = a * s[i] + b * c[i];
    }
}

__device__ __forceinline__ void rope8v(float* x, const f32x4 c, const f32x4 s) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const float a = x[2 * i], b = x[2 * i + 1];
        x[2 * i] = a * c[i] - b * s[i];
        x[2 * i + 1] = a * s[i] + b * c[i];
    }
}

__device__ __forceinline__ u16x8 pack8(const float* x, float mul) {
    u16x8 t;
#pragma unroll
    for (int i = 0; i < 8; ++i) t[i] = f2bf(x[i] * mul);
    return t;
}

__device__ __forceinline__ u16x8 rope_u16x8(u16x8 v, const float* cs, const float* sn, float mul) {
    float x[8];
    unpack8(v, x);
    rope8(x, cs, sn);
    return pack8(x, mul);
}

// LDS-DMA staging of a 64-row x 128-byte tile (D = 64; dma_tile64_buf also 256-byte rows, D = 128) into the swizzled image of swz<128>: the DMA writes lane-
// linearly (wave-instruction i of wave w fills physical chunks 64 (cpw w + i) + lane), so each lane loads the
// SOURCE chunk the swizzle puts at its physical slot (c = pc ^ sigma(r)).  Rows past the end are loaded clamped
// (row S - 1): the kernels mask their scores, so those rows only ever meet a zero P / dS.  No registers hold the
// tile and no VALU touches it; completion is the issuing wave's vmcnt (the kernels' closing __syncthreads).
typedef __attribute__((address_space(3))) void lds_void_t;
typedef __attribute__((address_space(1))) const void gbl_void_t;

template <int NW>
__device__ __forceinline__ void dma_tile64(const __bf16* base, long ld, int r0, int S, char* img, int w, int l) {
    constexpr int CPW = 512 / (NW * 64);  // wave-instructions per wave (512 chunks of 16 bytes per tile)
#pragma unroll
    for (int i = 0; i < CPW; ++i) {
        const int slot = 64 * (CPW * w + i);  // wave-uniform first chunk of this instruction
        const int e = slot + l, r = e >> 3, pc = e & 7;
        const int sg = (((r >> 1) & 1) << 2) | ((r >> 2) & 3);
        const long row = min(r0 + r, S - 1);
        __builtin_amdgcn_global_load_lds((gbl_void_t*)(base + row * ld + ((pc ^ sg) << 3)),
                                         (lds_void_t*)(img + slot * 16), 16, 0, 0);
    }
}

// The same DMA through a buffer resource (guide T8): the resource covers one head's rows [0, S) of a row-major
// tensor (base = the head's first element, head_bytes = ((S - 1) * ld + D) * 2), the lane's byte offset inside a
// tile is fixed for the kernel (dma_voff, once) and the tile's row offset is the wave-uniform soffset -- no per-tile
// vector address arithmetic (the 64-bit clamped addresses of dma_tile64 cost ~30 VALU per tile).  Rows at or past S
// are out of range and read as zeros; the kernels mask their scores.  The resource is built inside the helper from
// wave-uniform values (scalar instructions only); its type exists for the device target alone, so the body is
// compiled in the device pass only.
__device__ __forceinline__ int head_bytes(long ld, int S, int D) { return (int)(((long)(S - 1) * ld + D) * 2); }

template <int NW, int RB = 128>
struct DmaVoff {
    static constexpr int CPW = 4 * RB / (NW * 64);  // wave-instructions per wave: 4 RB chunks of 16 bytes per tile
    unsigned v[CPW];
};

// RB = 128 (D = 64) or 256 (D = 128): the tile image of swz<RB>, 64 rows of RB bytes
template <int NW, int RB = 128>
__device__ __forceinline__ DmaVoff<NW, RB> dma_voff(long ld, int w, int l) {
    constexpr int CPR = RB / 16;  // chunks per row
    DmaVoff<NW, RB> o;
#pragma unroll
    for (int i = 0; i < DmaVoff<NW, RB>::CPW; ++i) {
        const unsigned e = 64 * (DmaVoff<NW, RB>::CPW * w + i) + l;
        const int r = e / CPR, pc = e % CPR;
        const int sg = RB == 128 ? ((((r >> 1) & 1) << 2) | ((r >> 2) & 3)) : (((r & 3) << 2) | ((r >> 2) & 3));
        o.v[i] = (unsigned)((r * ld + ((pc ^ sg) << 3)) * 2);
    }
    return o;
}

template <int NW, int RB = 128>
__device__ __forceinline__ void dma_tile64_buf(const __bf16* base, int nbytes, const DmaVoff<NW, RB>& vo, int r0,
                                               long ld, char* img, int w) {
#if defined(__HIP_DEVICE_COMPILE__)  // device pass only: the host pass cannot instantiate the resource type
    constexpr int CPW = DmaVoff<NW, RB>::CPW;
    const auto rsrc = __builtin_amdgcn_make_buffer_rsrc((void*)base, 0, nbytes, 0x00020000);
    const unsigned soff = (unsigned)((long)r0 * ld * 2);
#pragma unroll
    for (int i = 0; i < CPW; ++i)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rsrc, (lds_void_t*)(img + 64 * (CPW * w + i) * 16), 16, vo.v[i], soff,
                                                 0, 0);
#endif
}

// Prologue priority.  A workgroup that starts while its CU's other waves run their MFMA loops is the youngest there,
// and VALU issue goes by priority, then age (MI355X_MICROARCH, two waves per SIMD, item 2): its prologue -- ~200 VALU
// of index math (integer divisions by the grid's shape) and address set-up before the first load can issue --
// got the leftover slots.  Stamps (profiles/attention_stamps_r5.md): the 16-row dQ kernel's last wave issued its
// prologue loads ~6.4 k cycles after entry, its rows arrived 1.6 k later.  The prologue runs at s_setprio 3 and the
// loop at 0 (BPE_FA_PRIO=0 builds the old form for A/B).
#ifndef BPE_FA_PRIO
#define BPE_FA_PRIO 1
#endif
__device__ __forceinline__ void prologue_prio_begin() {
    if (BPE_FA_PRIO) __builtin_amdgcn_s_setprio(3);
}
__device__ __forceinline__ void prologue_prio_end() {
    if (BPE_FA_PRIO) __builtin_amdgcn_s_setprio(0);
}

// (Measured and dropped, round 5: pinning the prologue's Q rows / LSE before the barrier with an empty asm use --
// hipcc otherwise sinks those loads into the loop preheader, after the barrier -- together with float-reciprocal
// divisions for the work-item decomposition.  The dQ prologue shortened 8.1 k -> 7.5 k cycles, but the forward ran
// 1.5-3.7 % and the backward 0.3-1.2 % slower, end to end -0.15 % (profiles/bench/ab_attn_keep_sdiv_r5.log).)

// Launch order of the (block, batch*head) work items: heads are taken in groups of `group` (batch, head) pairs
// and, inside a group, the `nblk` blocks of every pair run heaviest first (index 0 = heaviest).  All blocks of a
// pair thus run close together in time, so the K / V (forward) or Q / dO (backward) rows they share are re-read
// from L2 / the Infinity Cache instead of HBM: with the plain "all pairs' heaviest block first" order the whole
// grid's K / V (393 MB at GPT-2 B 128) streamed through between two uses of a pair.  With group % 8 == 0 the
// blocks of one pair share blockIdx % 8, i.e. an XCD L2 under round-robin dispatch (speed only, not
// correctness).  Returns the block rank (0 = heaviest) and the pair index.
__device__ __forceinline__ void grouped_order(int bid, int nblk, int BH, int group, int& rank, int& bh) {
    const int per = nblk * group;
    const int g = bid / per;
    const int r = bid - g * per;
    const int gs = min(group, BH - g * group);  // the last group may be short
    rank = r / gs;
    bh = g * group + (r - rank * gs);
}

// Host: pairs per launch-order group, BPE_FA_GROUP (default 64; 0 = one group of all pairs, the old order).
inline int fa_group(int BH) {
    static const int g = [] {
        const char* e = getenv("BPE_FA_GROUP");
        return e ? atoi(e) : 64;
    }();
    return (g <= 0 || g > BH) ? BH : g;
}

}  // namespace fa
}  // namespace bpe
