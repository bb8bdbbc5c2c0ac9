// 8-wave ping-pong bf16 MFMA GEMM for gfx950 (all three GEMMs of a linear layer).
// build-flags: -fno-slp-vectorize   (no packed f32 VALU beside the MFMAs: ops/build.py file_flags)
//
//   C[M, N] = beta * C + sum_r A(i, r) B(r, j)        (fp32 accumulation, bf16 or fp32-slab output)
//
// Each operand is row-major and either K-major (reduction index contiguous:
// X [M][R] or W [N][R]) or MN-major (output index contiguous: dY [R][M],
// W [R][N], X [R][N]).  The forward Y = X W^T is (K, K), the input gradient
// dX = dY W is (K, MN), the weight gradient dW = dY^T X is (MN, MN).
//
// Geometry (guide §5 "The 256² 8-phase template", designed here for both
// operand layouts): 256 x 256 output tile, BK = 64, 512 threads = 8 waves in
// two groups of four.  Group g (waves 4g..4g+3) owns output rows
// [128g, 128g+128); wave wl = w & 3 owns columns [64 wl, 64 wl + 64), i.e.
// 8 x 4 accumulators of mfma_f32_16x16x32_bf16 (128 registers).  The MFMA is
// issued as (B fragment, A fragment) so an accumulator register holds four
// CONSECUTIVE output columns of one row (8-byte packed stores).
//
// Ping-pong: waves w and w+4 share a SIMD.  Group 1 runs one barrier behind
// group 0, so in every barrier interval one wave of each SIMD issues 16 MFMAs
// (one 64 x 32 quadrant of its tile over K = 64, 256 cycles) while its partner
// reads the next quadrant's fragments from LDS and issues LDS-DMA for the
// next K-tile: the matrix pipe alternates between the two waves and never
// waits for LDS.  Quadrant order (m0,n0) (m0,n1) (m1,n1) (m1,n0) reuses one
// operand's fragments between neighbours: 12 / 4 / 8 / 4 ds_read_b128 per
// phase.
//
// Staging: two 64 KiB stages (A image 32 KiB + B image 32 KiB), filled by
// global_load_lds_dwordx4 (LDS-DMA).  K-major images are [256][64] (128-byte
// rows, 16-byte chunk c of row r at c ^ ((r >> 1) & 7): conflict-free for the
// 16x16x32 ds_read_b128 lane groups); MN-major images are [64][256] (512-byte
// rows, chunk c at c ^ sig(r), read with ds_read_b64_tr_b16).  The DMA image
// is lane-linear, so the swizzle is applied to the SOURCE address.  K-tile
// kt+1 is DMA'd during phases 0-1 of kt (group 0 the first halves of A and B,
// group 1 the second halves), retired by each issuing wave's vmcnt(0) in
// phase 3 before the barrier that precedes the first read of kt+1.  WAR: the
// buffer refilled in phase 0 of kt was last read in phase 3 of kt-1, whose
// reads retire (lgkmcnt(0)) before that phase's closing barrier.  Raw
// s_barrier only: __syncthreads() would drain the DMA (guide §5 "Pipelining
// across barriers").
//
// Split-K (weight gradients: R = all tokens) writes fp32 partial tiles to a
// slab reduced by splitk_reduce_kernel (gemm.hip) in a fixed order.
// Epilogue (bf16 output): the tile is staged through the then-free LDS as a
// [256][512 B] image and written back as whole 512-byte rows.
#include "fa_common.h"
#include "kernels.h"

#include <algorithm>
#include <cstdlib>

namespace bpe {
namespace gpp {

constexpr int NT = 512, BT = 256, BK = 64;
constexpr int OPB = 32768;          // one operand image per stage
constexpr int STAGE = 2 * OPB;      // 64 KiB
constexpr int LDS_BYTES = 2 * STAGE;  // 128 KiB
#ifdef BPE_GPP_PHASE_STAMPS
constexpr int LDS_LAUNCH = LDS_BYTES + 8 * 64 * 8;  // + the phase stamps of 8 waves
#else
constexpr int LDS_LAUNCH = LDS_BYTES;
#endif

typedef __attribute__((address_space(3))) void lds_void;
typedef __attribute__((address_space(1))) void gbl_void;

__device__ __forceinline__ int fk(int r) { return (r >> 1) & 7; }
__device__ __forceinline__ int sig(int r) { return ((r & 3) << 2) | ((r >> 2) & 3); }

// Source offset (elements, relative to the tile origin) of 16-byte image chunk e (0..2047).
template <bool KM>
__device__ __forceinline__ int src_off(int e, int ld) {
    if constexpr (KM) {
        const int row = e >> 3, lc = (e & 7) ^ fk(row);
        return row * ld + lc * 8;
    } else {
        const int row = e >> 5, lc = (e & 31) ^ sig(row);
        return row * ld + lc * 8;
    }
}

// Tile origin of an operand for K-tile starting at k0 (t0 = first output row/column of the tile).
template <bool KM>
__device__ __forceinline__ const __bf16* tile_ptr(const __bf16* P, long ld, int t0, long k0) {
    return KM ? P + (long)t0 * ld + k0 : P + k0 * ld + t0;
}

// DMA half h (= the issuing group) of one operand image: 4 wave-instructions of 1 KiB.
__device__ __forceinline__ void dma_half(const __bf16* tile0, const int (&off)[4], char* img, int g, int wl) {
#pragma unroll
    for (int j = 0; j < 4; ++j)
        __builtin_amdgcn_global_load_lds((gbl_void*)(tile0 + off[j]),
                                         (lds_void*)(img + (g * 1024 + (wl * 4 + j) * 64) * 16), 16, 0, 0);
}

// MN-major image of the spread schedule: eight [64 k][32 col] sub-images of 4 KiB (64-byte rows), so that
// every set of columns the phases read (a 64-column A block, the 32-column halves of the B blocks) is a whole
// number of 1-KiB DMA pieces.  The 32-byte halves of a row are swapped on odd 8-row groups, which keeps the
// ds_read_b64_tr_b16 reads conflict-free (the 8 rows a 32-lane group reads, r0..r0+3 and r0+8..r0+11, land
// on 8 distinct 32-byte bank groups).
__device__ __forceinline__ int sub_off(int r, int c) {
    return (c >> 5) * 4096 + r * 64 + ((((c >> 4) & 1) ^ ((r >> 3) & 1)) << 5) + ((c & 15) << 1);
}

// Source offset (elements, from the tile origin) of 16-byte chunk e (0..2047) of a sub-image MN-major image:
// sub-image e >> 8, piece (16 k-rows) ((e >> 6) & 3), lane e & 63 -> k-row 16 piece + lane / 4, physical
// 16-byte chunk lane & 3 of the 64-byte row, which holds logical chunk (lane & 3) ^ (2 * bit 3 of the row).
__device__ __forceinline__ int src_off_sub(int e, int ld) {
    const int s = e >> 8, q = (e >> 6) & 3, ln = e & 63;
    const int row = 16 * q + (ln >> 2);
    const int ql = (ln & 3) ^ (((row >> 3) & 1) << 1);
    return row * ld + 32 * s + 8 * ql;
}

// A64 (build define, default on): the MN-major A operand of the spread schedule (the weight gradient's dY) in four
// [64 k][64 col] sub-images of 8 KiB with 128-byte rows instead of eight [64 k][32 col] ones: a 1-KiB DMA piece is
// then 8 whole 128-byte lines of 8 token rows instead of 16 half lines of 16 rows (the A pieces the schedule issues
// are whole 64-column blocks either way, so the schedule is unchanged; B keeps the 32-column halves it needs).  The
// 32-byte segment of a row is swizzled by a64_f(row), which keeps the ds_read_b64_tr_b16 fragment reads
// conflict-free (each 32-lane group reads rows {r0..r0+3, r0+8..r0+11} x one 32-byte segment: 8 distinct bank
// groups; checked exhaustively on the host when the layout was written).
#ifndef BPE_GPP_A64
#define BPE_GPP_A64 1
#endif
__device__ __forceinline__ int a64_f(int r) { return ((r >> 1) & 1) | (((r >> 3) & 1) << 1); }
__device__ __forceinline__ int sub64_off(int r, int c) {  // byte offset of (k-row r, column c) in the A64 image
    const int cc = c & 63;
    return (c >> 6) * 8192 + r * 128 + (((cc >> 4) ^ a64_f(r)) << 5) + ((cc & 15) << 1);
}
// source offset (elements from the tile origin) of 16-byte image chunk e (0..2047) of the A64 image: sub-image
// e >> 9, piece (8 k-rows) (e >> 6) & 7, lane e & 63 -> k-row 8 piece + lane / 8, physical chunk lane & 7
__device__ __forceinline__ int src_off_sub64(int e, int ld) {
    const int s = e >> 9, q = (e >> 6) & 7, ln = e & 63;
    const int row = 8 * q + (ln >> 3), ch = ln & 7;
    const int lc = (((ch >> 1) ^ a64_f(row)) << 1) | (ch & 1);
    return row * ld + 64 * s + 8 * lc;
}
__device__ __forceinline__ bf16x8 frag_a64(char* img, int tb, int ks, int l) {
    const int r = 32 * ks + 8 * (l >> 4) + ((l & 15) >> 2);
    const int c = tb * 16 + 4 * (l & 3);
    return fa::lds_tr_pair(img, sub64_off(r, c), sub64_off(r + 4, c));
}

// MFMA operand fragment of 16-row/col block tb, k-step ks: lane l gets X[t = 16 tb + (l & 15)][k = 32 ks + 8 (l >> 4) + j].
// SUB: MN-major operands use the sub-image layout above (spread schedule) instead of [64][256] 512-byte rows.
template <bool KM, bool SUB = false>
__device__ __forceinline__ bf16x8 frag(char* img, int tb, int ks, int l) {
    if constexpr (KM) {
        const int row = tb * 16 + (l & 15);
        const int ch = (4 * ks + (l >> 4)) ^ fk(l & 15);
        return fa::lds_row16(img, row * 128 + (ch << 4));
    } else if constexpr (SUB) {
        const int r = 32 * ks + 8 * (l >> 4) + ((l & 15) >> 2);
        const int c = tb * 16 + 4 * (l & 3);
        return fa::lds_tr_pair(img, sub_off(r, c), sub_off(r + 4, c));
    } else {
        const int r = 32 * ks + 8 * (l >> 4) + ((l & 15) >> 2);
        const int c = tb * 16 + 4 * (l & 3);
        const int o0 = r * 512 + (((c >> 3) ^ sig(r)) << 4) + ((c & 7) << 1);
        const int o1 = (r + 4) * 512 + (((c >> 3) ^ sig(r + 4)) << 4) + ((c & 7) << 1);
        return fa::lds_tr_pair(img, o0, o1);
    }
}

__device__ __forceinline__ f32x4 mfma16(bf16x8 a, bf16x8 b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

// fp8 operands (F8 != 0, K-major images only).  An fp8 K-tile of 128 values is byte-for-byte the 128-byte row
// segment of a bf16 K-tile of 64, so the staging (DMA, swizzle, fragment reads) is the bf16 kernel's, run on
// the matrices reinterpreted as bf16 rows of half the length.  The two bf16 k-step fragments of a lane (16-byte
// chunks g and 4 + g of its row, g = lane >> 4) together are the 32 bytes one
// v_mfma_scale_f32_16x16x128_f8f6f4 takes per lane: the lanes then cover every k of the 128 exactly once, in
// the same order for both operands, so the products sum over k correctly.  Block scales are 1 (E8M0 127);
// the per-tensor inverse scales are applied in the epilogue.  F8: 1 = e4m3 x e4m3, 2 = e5m2 (A) x e4m3 (B).
typedef int i32x8 __attribute__((ext_vector_type(8)));

__device__ __forceinline__ i32x8 cat8(bf16x8 lo, bf16x8 hi) {
    typedef int i32x4 __attribute__((ext_vector_type(4)));
    const i32x4 a = __builtin_bit_cast(i32x4, lo), b = __builtin_bit_cast(i32x4, hi);
    return i32x8{a[0], a[1], a[2], a[3], b[0], b[1], b[2], b[3]};
}

// C += B-operand x A-operand (the kernel issues (B, A) so a register holds 4 consecutive output columns);
// cbsz = format of the first operand (B = the weight, e4m3), blgp = the second's (A: e4m3, or e5m2 for F8 2)
template <int F8>
__device__ __forceinline__ f32x4 mfma_f8(const bf16x8 (&b)[2], const bf16x8 (&a)[2], f32x4 c) {
    return __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(cat8(b[0], b[1]), cat8(a[0], a[1]), c, 0,
                                                             F8 == 2 ? 1 : 0, 0, 127, 0, 127);
}

struct Frags {
    bf16x8 a[4][2];  // A (output rows): 4 i-blocks of the current m half x 2 k-steps
    bf16x8 b[2][2];  // B (output cols): 2 j-blocks of the current n half x 2 k-steps
};

__device__ __forceinline__ void bar() {
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
}

// Per-wave phase stamps (a diagnostic variant build: ops.build --variant pstamps -D BPE_GPP_PHASE_STAMPS; read by
// benchmarks/gemm_phase_stamps.py): every wave records s_memtime at four events of each phase of K-tiles
// PST_KT0 .. PST_KT0 + PST_NKT - 1 of the one-tile kernel's spread schedule -- 0 section start (before its
// fragment reads), 1 after its wait (reads / DMA retired), 2 after the barrier (MFMA section start), 3 after the
// MFMA issue (before the closing barrier) -- into LDS above the two stages (no VMEM traffic, so the kernel's
// vmcnt accounting is untouched), copied to g_gpp_phase at the end for workgroups 0 .. 1023.
#ifdef BPE_GPP_PHASE_STAMPS
constexpr int PST_KT0 = 2, PST_NKT = 4, PST_VALS = PST_NKT * 4 * 4;  // per wave
__device__ long long g_gpp_phase[1024 * 8 * PST_VALS];
__device__ __forceinline__ void pst(int kt, int p, int e) {
    extern __shared__ __attribute__((aligned(16))) char pst_smem[];
    if (kt >= PST_KT0 && kt < PST_KT0 + PST_NKT) {
        const long long t = __builtin_amdgcn_s_memtime();
        const int w = threadIdx.x >> 6;
        if ((threadIdx.x & 63) == 0)
            *reinterpret_cast<long long*>(pst_smem + 2 * 2 * 32768 +
                                          ((w * PST_NKT + kt - PST_KT0) * 16 + 4 * p + e) * 8) = t;
    }
}
#define PST(p, e) pst(kt_idx, p, e)
#else
#define PST(p, e)
#endif

template <bool AK, bool BKM, bool SUB = false>
__device__ __forceinline__ void load_a(Frags& f, char* img, int g, int m, int l) {
#pragma unroll
    for (int ib = 0; ib < 4; ++ib)
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) {
            if constexpr (!AK && SUB && BPE_GPP_A64) f.a[ib][ks] = frag_a64(img, 8 * g + 4 * m + ib, ks, l);
            else f.a[ib][ks] = frag<AK, SUB>(img, 8 * g + 4 * m + ib, ks, l);
        }
}
template <bool AK, bool BKM, bool SUB = false>
__device__ __forceinline__ void load_b(Frags& f, char* img, int wl, int n, int l) {
#pragma unroll
    for (int jb = 0; jb < 2; ++jb)
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) f.b[jb][ks] = frag<BKM, SUB>(img, 4 * wl + 2 * n + jb, ks, l);
}

// An empty asm "use" of the accumulators a section just issued MFMAs into (no instruction is emitted).
// Without it hipcc sinks every v_mfma_scale_f32_16x16x128_f8f6f4 of a K-tile past the phase barriers into the
// loop latch (the MFMA results are only read after the loop, the barriers are in other basic blocks, and
// sched_barrier only fences the scheduler inside a block): all 32 fp8 MFMAs of a K-tile then issued in one
// barrier interval and the ping-pong was gone (24 + 8 MFMAs in two sections, three sections empty).  Pinned,
// each section issues its own 8.  The bf16 MFMAs are not sunk (tools/isa_mfma_sections.py checks both).
__device__ __forceinline__ void pin_quadrant(f32x4 (&acc)[8][4], int m, int n, int ib0, int ib1) {
#pragma unroll
    for (int ib = ib0; ib < ib1; ++ib)
#pragma unroll
        for (int jb = 0; jb < 2; ++jb) asm volatile("" ::"v"(acc[4 * m + ib][2 * n + jb]));
}

template <int F8 = 0>
__device__ __forceinline__ void mma_quadrant(f32x4 (&acc)[8][4], const Frags& f, int m, int n) {
#pragma unroll
    for (int ib = 0; ib < 4; ++ib)
#pragma unroll
        for (int jb = 0; jb < 2; ++jb) {
            if constexpr (F8 != 0) {
                acc[4 * m + ib][2 * n + jb] = mfma_f8<F8>(f.b[jb], f.a[ib], acc[4 * m + ib][2 * n + jb]);
            } else {
#pragma unroll
                for (int ks = 0; ks < 2; ++ks)
                    acc[4 * m + ib][2 * n + jb] = mfma16(f.b[jb][ks], f.a[ib][ks], acc[4 * m + ib][2 * n + jb]);
            }
        }
    if constexpr (F8 != 0) pin_quadrant(acc, m, n, 0, 4);
}

// Half of a quadrant (i-blocks 2h, 2h+1): the MFMA section can then issue one DMA piece between its halves.
template <int F8 = 0>
__device__ __forceinline__ void mma_half(f32x4 (&acc)[8][4], const Frags& f, int m, int n, int h) {
#pragma unroll
    for (int ib = 2 * h; ib < 2 * h + 2; ++ib)
#pragma unroll
        for (int jb = 0; jb < 2; ++jb) {
            if constexpr (F8 != 0) {
                acc[4 * m + ib][2 * n + jb] = mfma_f8<F8>(f.b[jb], f.a[ib], acc[4 * m + ib][2 * n + jb]);
            } else {
#pragma unroll
                for (int ks = 0; ks < 2; ++ks)
                    acc[4 * m + ib][2 * n + jb] = mfma16(f.b[jb][ks], f.a[ib][ks], acc[4 * m + ib][2 * n + jb]);
            }
        }
    if constexpr (F8 != 0) pin_quadrant(acc, m, n, 2 * h, 2 * h + 2);
}

// (Measured and dropped, round 5 (docs/performance.md, ping-pong phase stamps): reading the next K-tile's phase-0 A
// fragments inside phase 3's MFMA section, so phase 0 reads only its B half -- the loaders' lateness at phase 0
// halved in the stamps build, but GPT-2 GEMMs moved -1 to +1 % and the Llama SwiGLU / fp8 GEMMs lost 0.7-1.4 %,
// profiles/bench/ab_r5_prea_fused.log; and issuing the barrier that ends an MFMA section before its last i-block --
// 6-10 % slower, profiles/bench/ab_r5_earlybar_prio.log.)

// One K-tile: four (load section, barrier, MFMA section, barrier) phases.  `cur` is read, `nxt` is the DMA
// target (the __restrict__ parameters let the wait-count pass see that the fragment reads do not alias the
// in-flight DMA; without it hipcc drains the DMA before the first read).
// DIAG (timing diagnostics, numerically wrong): 1 = no DMA in the loop, 2 = fragment reads only in phase 0,
// 6 = no epilogue global stores (gemm_pp_kernel),
// 3 = no MFMA, 4 = no stagger between the groups, 5 = DMA issued but never waited for (issue cost only)
template <bool AK, bool BKM, int DIAG>
__device__ __forceinline__ void ktile(char* __restrict__ cur, char* __restrict__ nxt, bool dma, const __bf16* an,
                                      const __bf16* bn, const int (&oa)[4], const int (&ob)[4], int g, int wl,
                                      int l, f32x4 (&acc)[8][4]) {
    Frags f;
    char* Ac = cur;
    char* Bc = cur + OPB;
    // phase 0: (m0, n0)
    load_a<AK, BKM>(f, Ac, g, 0, l);
    load_b<AK, BKM>(f, Bc, wl, 0, l);
    if (DIAG == 1) dma = false;
    if (dma) dma_half(an, oa, nxt, g, wl);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    bar();
    if (DIAG != 3) mma_quadrant(acc, f, 0, 0);
    bar();
    // phase 1: (m0, n1)
    if (DIAG != 2) load_b<AK, BKM>(f, Bc, wl, 1, l);
    if (dma) dma_half(bn, ob, nxt + OPB, g, wl);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    bar();
    if (DIAG != 3) mma_quadrant(acc, f, 0, 1);
    bar();
    // phase 2: (m1, n1)
    if (DIAG != 2) load_a<AK, BKM>(f, Ac, g, 1, l);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    bar();
    if (DIAG != 3) mma_quadrant(acc, f, 1, 1);
    bar();
    // phase 3: (m1, n0); retire this wave's DMA of the next K-tile before the barrier
    if (DIAG != 2) load_b<AK, BKM>(f, Bc, wl, 0, l);
    if (DIAG == 5)
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // DMA issued but never waited for
    else
        asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    bar();
    if (DIAG != 3) mma_quadrant(acc, f, 1, 0);
    bar();
    if (DIAG == 3) {  // keep the fragments live
#pragma unroll
        for (int ib = 0; ib < 4; ++ib) acc[ib][0][0] += (float)f.a[ib][0][0] + (float)f.b[ib & 1][1][1];
    }
}

// ---------------------------------------------------------------------------------------------------------
// Spread DMA schedule (both operands K-major, i.e. the forward GEMM).  A diagnostic build showed where the
// burst schedule above loses: issuing the next K-tile's 8 LDS-DMA instructions per wave in phases 0-1 only
// (4 per load section, each ~100-185 cycles to issue beside the fragment reads) makes those load sections
// longer than the partner wave's 256-cycle MFMA section; with the DMA removed (DIAG 1) the same loop runs
// 1.45-1.55x faster, and issuing it without ever waiting for it (DIAG 5) is no faster than waiting for it
// (profiles/bench/gpp_diag_b128.log) -- issue placement, not latency.  Here every load section issues 2
// pieces, in the order the next K-tile's phases read them:
//   phase 0: A rows [128g, +64)   (read by this group in phase 0 of kt+1)
//   phase 1: half g of B rows {64w' + [0, 32)}   (both groups, phase 0 / 3)
//   phase 2: half g of B rows {64w' + [32, 64)}  (both groups, phase 1)
//   phase 3: A rows [128g + 64, +64)  (this group, phase 2)
// and then waits vmcnt(4): the two newest issues stay in flight, the one issued three load sections ago is
// retired before the barrier that precedes its first read (by either group: group 1 reads a piece one barrier
// after group 0, never before the issuing wave's wait).  WAR: a region of the other buffer is refilled at
// least one barrier after its last read of K-tile kt-1 (A rows: phases 0 / 2, B halves: phases 3 / 1).
// Last K-tile (no issue): vmcnt(2) in phase 0 (B rows [32, 64) of this tile), vmcnt(0) afterwards.
#ifndef BPE_GPP_RELAX  // build define: phase 2 of the spread schedule waits vmcnt(6) (1) or vmcnt(4) (0)
#define BPE_GPP_RELAX 1
#endif

struct SpreadOff {
    int a0[2], a1[2], b0[2], b1[2];  // source offsets (elements from the K-tile origin) of this thread's pieces
    int la0, la1, lb0, lb1;          // wave-uniform LDS chunk index of each piece pair (piece j at + 64 j)
};

// Chunk e of either image kind: K-major [256][64] (A rows / B rows = output index) or the MN-major sub-image
// layout.  The piece sets line up in both: chunks [1024 g + 512 m, +512) are output rows / columns
// [128 g + 64 m, +64) and chunks {512 w' + 256 h + [0, 256)} the 32-wide half h of block w'.
template <bool KM>
__device__ __forceinline__ int spread_src(int e, int ld) {
    if constexpr (KM) return src_off<true>(e, ld);
    else return src_off_sub(e, ld);
}

template <bool AK, bool BKM>
__device__ __forceinline__ SpreadOff spread_offsets(int g, int wl, int l, int lda, int ldb) {
    SpreadOff o;
    o.la0 = 1024 * g + 128 * wl;
    o.la1 = o.la0 + 512;
    o.lb0 = 512 * (2 * g + (wl >> 1)) + 128 * (wl & 1);
    o.lb1 = o.lb0 + 256;
#pragma unroll
    for (int j = 0; j < 2; ++j) {
        if constexpr (!AK && BPE_GPP_A64) {
            o.a0[j] = src_off_sub64(o.la0 + 64 * j + l, lda);
            o.a1[j] = src_off_sub64(o.la1 + 64 * j + l, lda);
        } else {
            o.a0[j] = spread_src<AK>(o.la0 + 64 * j + l, lda);
            o.a1[j] = spread_src<AK>(o.la1 + 64 * j + l, lda);
        }
        o.b0[j] = spread_src<BKM>(o.lb0 + 64 * j + l, ldb);
        o.b1[j] = spread_src<BKM>(o.lb1 + 64 * j + l, ldb);
    }
    return o;
}

// Cache policy of the in-loop LDS-DMA loads per operand (variant builds; 0 = default, 2 = nt: the line is the first
// evicted from the XCD's L2).  Measured and left at 0 (profiles/bench/ab_dma_policy_r6.log): nt on A (activations)
// -2 to -3 % on the MN x MN weight-gradient GEMMs on one box, +1 to +6 % on another, and slower K-major forward /
// QKV + RoPE / ppt LM-head GEMMs (end to end -0.6-0.9 %); nt on B (weights, re-read every round) slower everywhere.
#ifndef BPE_GPP_DMA_POL_A
#define BPE_GPP_DMA_POL_A 0
#endif
#ifndef BPE_GPP_DMA_POL_B
#define BPE_GPP_DMA_POL_B 0
#endif

template <int POL>
__device__ __forceinline__ void dma_ld(const __bf16* src, char* dst) {
    __builtin_amdgcn_global_load_lds((gbl_void*)src, (lds_void*)dst, 16, 0, POL);
}

template <int POL = 0>
__device__ __forceinline__ void dma_one(const __bf16* tile0, int off, char* img, int lbase) {
    dma_ld<POL>(tile0 + off, img + lbase * 16);
}

template <int POL = 0>
__device__ __forceinline__ void dma_pair(const __bf16* tile0, const int (&off)[2], char* img, int lbase) {
#pragma unroll
    for (int j = 0; j < 2; ++j) dma_ld<POL>(tile0 + off[j], img + (lbase + 64 * j) * 16);
}

// SPLIT (spread mode 2, the weight-gradient layout): the second piece of each
// pair is issued by the same wave in its MFMA section,
// between the two halves of the quadrant, so a load section carries one piece; the waits become vmcnt(3).
// FIRST: K-tile 0 of a tile, whose image was retired (vmcnt(0)) before the loop.  Its phases 0-1 would only retire
// pieces of that image, so they wait for LDS only; phases 2-3 retire the first pieces of K-tile 1 (read before any
// wait of K-tile 1) as always.  In the persistent kernel this lets the previous tile's epilogue stores, which
// share the vmcnt counter with the DMA, drain during the first two phases instead of before them.
template <bool AK, bool BKM, int DIAG, bool SPLIT = false, int F8 = 0>
__device__ __forceinline__ void ktile_spread(char* __restrict__ cur, char* __restrict__ nxt, bool dma,
                                             const __bf16* an, const __bf16* bn, const SpreadOff& so, int g, int wl,
                                             int l, f32x4 (&acc)[8][4], bool first = false, int kt_idx = -1) {
    (void)kt_idx;  // phase stamps builds only
    Frags f;
    char* Ac = cur;
    char* Bc = cur + OPB;
    constexpr int PA = BPE_GPP_DMA_POL_A, PB = BPE_GPP_DMA_POL_B;
    if (DIAG == 1) dma = false;
    // one phase: fragment reads (done by the caller), pieces of (tile, off, img, lbase), wait, barrier, MFMAs
    // RELAX: phase 2 (m1, n1) retires nothing that a read before phase 3's barrier needs (its own A rows of K-tile
    // kt + 1 are first read in phase 0 of kt + 1; the group's B halves it issued are retired in phase 3 / phase 0),
    // so it waits vmcnt(6) and leaves the piece pair issued two load sections ago in flight one section longer
    auto phase = [&](const __bf16* t0, const int (&off)[2], char* img, int lb, int m, int n, bool last_nodma_wait2,
                     bool relax = false) {
        const bool is_a = img == nxt;  // the A image sits at the stage origin, B at + OPB
        const int ph = 2 * m + (m ? 1 - n : n);  // (m0,n0) 0, (m0,n1) 1, (m1,n1) 2, (m1,n0) 3
        (void)ph;
        if (dma) {
            if constexpr (SPLIT) is_a ? dma_one<PA>(t0, off[0], img, lb) : dma_one<PB>(t0, off[0], img, lb);
            else is_a ? dma_pair<PA>(t0, off, img, lb) : dma_pair<PB>(t0, off, img, lb);
        }
        if (first && m == 0) {
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        } else if (dma) {
            if constexpr (SPLIT) asm volatile("s_waitcnt vmcnt(3) lgkmcnt(0)" ::: "memory");
            else if (BPE_GPP_RELAX && relax) asm volatile("s_waitcnt vmcnt(6) lgkmcnt(0)" ::: "memory");
            else asm volatile("s_waitcnt vmcnt(4) lgkmcnt(0)" ::: "memory");
        } else if (last_nodma_wait2) {
            asm volatile("s_waitcnt vmcnt(2) lgkmcnt(0)" ::: "memory");
        } else {
            asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
        }
        PST(ph, 1);
        bar();
        PST(ph, 2);
        if constexpr (SPLIT) {
            mma_half<F8>(acc, f, m, n, 0);
            if (dma) {
                __builtin_amdgcn_sched_barrier(0);
                is_a ? dma_one<PA>(t0, off[1], img, lb + 64) : dma_one<PB>(t0, off[1], img, lb + 64);
                __builtin_amdgcn_sched_barrier(0);
            }
            mma_half<F8>(acc, f, m, n, 1);
        } else {
            mma_quadrant<F8>(acc, f, m, n);
        }
        PST(ph, 3);
        bar();
    };
    // phase 0: (m0, n0)
    PST(0, 0);
    load_a<AK, BKM, true>(f, Ac, g, 0, l);
    load_b<AK, BKM, true>(f, Bc, wl, 0, l);
    phase(an, so.a0, nxt, so.la0, 0, 0, true);
    // phase 1: (m0, n1)
    PST(1, 0);
    load_b<AK, BKM, true>(f, Bc, wl, 1, l);
    phase(bn, so.b0, nxt + OPB, so.lb0, 0, 1, false);
    // phase 2: (m1, n1)
    PST(2, 0);
    load_a<AK, BKM, true>(f, Ac, g, 1, l);
    phase(bn, so.b1, nxt + OPB, so.lb1, 1, 1, false, true);
    // phase 3: (m1, n0)
    PST(3, 0);
    load_b<AK, BKM, true>(f, Bc, wl, 0, l);
    phase(an, so.a1, nxt, so.la1, 1, 0, false);
}

// Fused epilogues of the one-tile-per-workgroup kernel.  EPI_SWIGLU_BWD: the GEMM result is da = dY W2 (the
// gradient of a = silu(g) * u); instead of storing da the epilogue reads g and u from gu = [g | u] ([M][2F])
// and writes dgu = [dg | du] -- the SwiGLU backward without the da round trip through HBM.  Same math and
// rounding as swiglu_bwd_kernel (da rounded to bf16 first).
// EPI_SWIGLU_FWD: the forward gu = X [W1; W3]^T with a = silu(g) * u in the epilogue.  A workgroup's 256 output
// columns are 128 columns of g and the SAME 128 columns of u (B rows [128 t, +128) and [F + 128 t, +128) of
// [W1; W3]), so the epilogue writes both halves of gu and the gate a from one tile -- the separate swiglu_fwd
// pass over gu (read 2F, write F per token) disappears.  Same rounding as swiglu_fwd_kernel (a from bf16 g, u).
// Per-workgroup s_memtime stamps (a diagnostic variant build: ops.build --variant stamps -D BPE_GPP_STAMPS; read
// by benchmarks/gemm_stamps.py): slot 0 entry, 1 prologue retired, 2 main loop done, 3 epilogue staged, 4 stores
// issued, 6 work id, 7 hardware XCC id.  Thread 0 writes them (wave 0's view of the workgroup).
#ifdef BPE_GPP_STAMPS
__device__ long long g_gpp_stamps[65536 * 8];
#define GPP_STAMP(i)                                                                                       \
    do {                                                                                                   \
        if (threadIdx.x == 0) g_gpp_stamps[(long)(blockIdx.x & 65535) * 8 + (i)] = __builtin_amdgcn_s_memtime(); \
    } while (0)
#define GPP_STAMP_VAL(i, v)                                                                                \
    do {                                                                                                   \
        if (threadIdx.x == 0) g_gpp_stamps[(long)(blockIdx.x & 65535) * 8 + (i)] = (v);                      \
    } while (0)
#define GPP_STAMP_T(t, i)                                                                                  \
    do {                                                                                                   \
        if (threadIdx.x == 0) g_gpp_stamps[(long)((t) & 65535) * 8 + (i)] = __builtin_amdgcn_s_memtime();    \
    } while (0)
#else
#define GPP_STAMP(i)
#define GPP_STAMP_VAL(i, v)
#define GPP_STAMP_T(t, i)
#endif

// EPI_ROPE: the QKV projection with RoPE on its Q / K columns (output columns [0, rot_cols)), applied to the
// bf16-rounded products exactly as rope_qk_kernel (rope.hip) applies it to the stored activation: interleaved
// pairs, position = row % S, fp32 cos / sin tables [S][D / 2].  Saves the separate in-place pass over Q / K.
// EPI_SWIGLU_FWD8: the fp8 forward [W1; W3] GEMM (e4m3 x e4m3) with the SwiGLU gate AND its two-layout e4m3 cast
// in the epilogue: writes gu (bf16, for the backward), a8 = e4m3(a * scale) [M][F] and a8t [F][M] (the W2 GEMM's
// operands) and folds max |a| into the slot's amax -- the swiglu_cast_fp8 pass over gu (0.43 ms per Llama layer at
// 65 536 tokens) disappears.  Same values, rounding and amax as launch_gemm_fp8 + swiglu_cast_fp8_t (bitwise).
// Persistent kernel only (the a8 tile is transposed through 18 KiB of LDS past the two stages).
// EPI_SWIGLU_BWD8: the fp8 input-gradient GEMM da = dY8 . W2_8 (e5m2 x e4m3, both K-major) with the SwiGLU backward
// AND the two-layout e5m2 cast of its result in the epilogue: reads g / u from gu, writes dgu8 = e5m2([dg | du] *
// scale) [M][2F] and dgu8t [2F][M] and folds max(|dg|, |du|) into the slot's amax -- neither da nor a bf16 dgu
// reaches HBM, and the swiglu_cast_fp8 backward pass (0.71 ms per Llama layer) disappears.  Same values as the hand
// fp8 GEMM + swiglu_cast_fp8_t (bitwise).  Persistent kernel only (the transposes go through the A8T tile).  Opt-in
// (ops/fp8.py BPE_FP8_SWIGLU_BWD_GEMM): 1.89 vs 1.34 ms per Llama layer against hipBLASLt + the cast pass -- the
// epilogue's 512 KiB of traffic per tile serialises behind the main loop, and the kernel spills 476 B per lane.
enum { EPI_NONE = 0, EPI_SWIGLU_BWD = 1, EPI_SWIGLU_FWD = 2, EPI_ROPE = 3, EPI_SWIGLU_FWD8 = 4, EPI_SWIGLU_BWD8 = 5 };
constexpr bool is_swf(int e) { return e == EPI_SWIGLU_FWD || e == EPI_SWIGLU_FWD8; }
constexpr int A8T_STRIDE = 144;               // bytes per token row of the a8 transpose tile (conflict-free reads)
constexpr int A8T_BYTES = 128 * A8T_STRIDE;   // one pass: 128 token rows x 128 a columns
// 1: the SwiGLU epilogues' arithmetic on the packed fp32 VALU, two elements per instruction (common.h
// fast_sigmoid2; bitwise the same results); 0: one element per instruction (A/B variant builds)
#ifndef BPE_GPP_PK
#define BPE_GPP_PK 1
#endif
// SwiGLU-backward epilogue timing diagnostics (variant builds only, numerically wrong): bit 0 = no g / u loads,
// bit 1 = no dg / du stores
#ifndef BPE_GPP_EPIDIAG
#define BPE_GPP_EPIDIAG 0
#endif
// Store policy of the fused epilogues' outputs (MI355X_MICROARCH store flavours): 0 = plain (the line stays in
// the XCD's L2), 1 = sc1 (written through and dropped from L2), 2 = nt.  The outputs are 0.6-1.1 GB streams read
// by later kernels only; kept in L2 they evict the main loop's operand tiles.  Per output, measured per call at
// GPT-2 B 128 (profiles/bench/ab_epilogue_store_policy_r6.log):
#ifndef BPE_GPP_POL_SWB  // SwiGLU backward dg / du (sc1: 0.67 vs 0.70-0.71 ms per GPT-2 call)
#define BPE_GPP_POL_SWB 1
#endif
#ifndef BPE_GPP_POL_SWF_GU  // SwiGLU forward gu (nt; sc1 on gu and a: 0.85 vs 0.82 ms)
#define BPE_GPP_POL_SWF_GU 2
#endif
#ifndef BPE_GPP_POL_SWF_A  // SwiGLU forward a
#define BPE_GPP_POL_SWF_A 0
#endif
#ifndef BPE_GPP_POL_ROPE  // QKV + RoPE output (sc1: 0.426-0.428 vs 0.433-0.434 ms)
#define BPE_GPP_POL_ROPE 1
#endif

// 16-byte store of v at byte offset off from the wave-uniform base (a buffer resource for the cache-policy forms:
// built from uniform values, so it lives in SGPRs -- no waterfall)
template <int POL>
__device__ __forceinline__ void st16(__bf16* base, unsigned off, const u16x8& v) {
#if defined(__HIP_DEVICE_COMPILE__)
    if constexpr (POL == 0) {
        *reinterpret_cast<u16x8*>(reinterpret_cast<char*>(base) + off) = v;
    } else {
        typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
        const auto rsrc = __builtin_amdgcn_make_buffer_rsrc((void*)base, 0, 0x7fffffff, 0x00020000);
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v), rsrc, off, 0, POL == 1 ? 16 : 2);
    }
#endif
}
struct Epi {
    const __bf16* gu;
    __bf16* dgu;  // EPI_SWIGLU_BWD: dgu out; EPI_SWIGLU_FWD: gu out
    long ld;      // row stride of gu / dgu (elements)
    int F;
    __bf16* act = nullptr;  // EPI_SWIGLU_FWD: a = silu(g) * u, [M][F]
    long ld_act = 0;
    int prio = 0;  // 1: group 1 (the younger waves 4-7) runs at s_setprio 1 (guide T5, static form)
    const float* sa = nullptr;  // F8: device-resident per-tensor inverse scales of A and B (output x sa x sb)
    const float* sb = nullptr;
    const float* cosT = nullptr;  // EPI_ROPE: [S][D / 2] tables, S, head dim, rotated column count
    const float* sinT = nullptr;
    int S = 0, D = 0, rot_cols = 0;
    uint8_t* a8 = nullptr;        // EPI_SWIGLU_FWD8: a8 [M][F], a8t [F][M] (ld M), the slot's scale and amax bits
    uint8_t* a8t = nullptr;
    long ld_a8t = 0;
    const float* a_scale = nullptr;
    unsigned* a_amax = nullptr;
    int gm = 0;  // tile order (tile_rc): 0 = row-major, gm > 0 = column-major within bands of gm row blocks
};

// Output tile t -> (row block ti, column block tj).  gm 0: row-major.  gm > 0: the tile grid cut into bands of gm
// row blocks, column-major inside a band, so the 32 consecutive work ids of one XCD in a round cover 32 / gm
// columns x gm rows instead of 32 / tiles_n rows x every column: when 256 is a multiple of gm x tiles_n, an XCD
// then keeps the same B column blocks in every round and its L2 holds them, instead of re-reading all of B (3.5-6.3
// MiB at GPT-2 K = 768, more than the 4 MiB L2) every round.
__device__ __forceinline__ void tile_rc(int t, int tiles_m, int tiles_n, int gm, int& ti, int& tj) {
    if (gm <= 0) {
        ti = t / tiles_n;
        tj = t % tiles_n;
        return;
    }
    const int band = t / (gm * tiles_n);
    const int r0 = band * gm;
    const int rows = tiles_m - r0 < gm ? tiles_m - r0 : gm;
    const int wb = t - band * gm * tiles_n;
    ti = r0 + wb % rows;
    tj = wb / rows;
}

// bf16 epilogue: the tile is staged through LDS at stg as [256 / NPASS][512 B] images (16-byte chunk c of row i at
// c ^ (i & 15)) and written back as whole rows.  NPASS 1: the whole tile at once (128 KiB, the one-tile kernel);
// NPASS 2: group h's rows [128 h, +128) in pass h through one 64 KiB image (the persistent kernel, whose other
// stage already holds the next tile's K-tile 0).  Raw barriers with LDS-only waits: the stores of a pass stay in
// flight.  TAIL: a barrier after the last pass too (the image is the next tile's DMA target).
template <int EPI, int F8, int NPASS>
__device__ __forceinline__ void epilogue_bf16(const f32x4 (&acc)[8][4], char* stg, int g, int wl, int l, int tid,
                                              int i0, int j0, int jb, __bf16* C, long ldc, float beta, const Epi& ep,
                                              bool st_on, bool tail, int sid, char* xtra = nullptr,
                                              float* amx = nullptr) {
    constexpr int RP = BT / NPASS;  // tile rows per pass
    float osc = 1.f;  // F8: the product of the operands' inverse scales (device-resident, one load)
    if constexpr (F8 != 0) osc = ep.sa[0] * ep.sb[0];
#pragma unroll
    for (int h = 0; h < NPASS; ++h) {
        const int r0 = h * RP;  // first tile row of this pass
        if (NPASS == 1 || g == h) {
#pragma unroll
            for (int ib = 0; ib < 8; ++ib)
#pragma unroll
                for (int jq = 0; jq < 4; ++jq) {
                    const int i = 128 * g + 16 * ib + (l & 15) - r0;
                    const int j = 64 * wl + 16 * jq + 4 * (l >> 4);
                    const f32x4 v = F8 != 0 ? acc[ib][jq] * osc : acc[ib][jq];
                    const u16x4 p = u16x4{f2bf(v[0]), f2bf(v[1]), f2bf(v[2]), f2bf(v[3])};
                    *reinterpret_cast<u16x4*>(stg + i * 512 + ((((j >> 3) ^ (i & 15))) << 4) + ((j & 7) << 1)) = p;
                }
        }
        if constexpr (EPI == EPI_SWIGLU_BWD) {
            // every g / u load of this thread's row segments is issued before the barrier (the accumulators are in
            // LDS now, their registers free): one memory round trip per pass instead of one per unrolled group of
            // rows, overlapped with the other waves' staging writes
            constexpr int NQ = 16 / NPASS;
            const int c = tid & 31;
            u16x8 gv[NQ], uv[NQ];
#pragma unroll
            for (int q = 0; q < NQ; ++q) {
                const long ro = (long)(i0 + r0 + q * 16 + (tid >> 5)) * ep.ld + j0 + c * 8;
                if (BPE_GPP_EPIDIAG & 1) {  // timing diagnostic: no g / u loads (numerically wrong)
                    gv[q] = u16x8{(unsigned short)ro, 1, 2, 3, 4, 5, 6, 7};
                    uv[q] = u16x8{(unsigned short)(ro >> 16), 1, 2, 3, 4, 5, 6, 7};
                    continue;
                }
                gv[q] = ld_stream(reinterpret_cast<const u16x8*>(ep.gu + ro));  // read once
                uv[q] = ld_stream(reinterpret_cast<const u16x8*>(ep.gu + ro + ep.F));
            }
            // raw barrier after the staging writes only: __syncthreads() would also wait for the loads (vmcnt(0))
            // before the first row's math; this way row q waits for its own pair (in-order vmcnt) and its math and
            // stores overlap the later rows' loads
            __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0) only
            bar();
            if (h == 0) GPP_STAMP_T(sid, 3);
#pragma unroll
            for (int q = 0; q < NQ; ++q) {
                const int i = q * 16 + (tid >> 5);
                const u16x8 v = *reinterpret_cast<const u16x8*>(stg + i * 512 + ((c ^ (i & 15)) << 4));
                const long ro = (long)(i0 + r0 + i) * ep.ld + j0 + c * 8;
                u16x8 dg, du;
#if BPE_GPP_PK
#pragma unroll
                for (int e = 0; e < 8; e += 2) {  // pairs on the packed fp32 VALU (same math and rounding)
                    const f32x2 gg = {bf2f(gv[q][e]), bf2f(gv[q][e + 1])}, uu = {bf2f(uv[q][e]), bf2f(uv[q][e + 1])};
                    const f32x2 d = {bf2f(v[e]), bf2f(v[e + 1])};
                    const f32x2 sg = fast_sigmoid2(gg);
                    const f32x2 a = d * (gg * sg), b = d * uu * sg * (1.f + gg * (1.f - sg));
                    du[e] = f2bf(a.x);
                    du[e + 1] = f2bf(a.y);
                    dg[e] = f2bf(b.x);
                    dg[e + 1] = f2bf(b.y);
                }
#else
#pragma unroll
                for (int e = 0; e < 8; ++e) {
                    const float gg = bf2f(gv[q][e]), uu = bf2f(uv[q][e]), d = bf2f(v[e]);
                    const float sg = fast_sigmoid(gg);
                    du[e] = f2bf(d * (gg * sg));
                    dg[e] = f2bf(d * uu * sg * (1.f + gg * (1.f - sg)));
                }
#endif
                if (st_on && (!(BPE_GPP_EPIDIAG & 2) || ep.prio == 77)) {  // EPIDIAG 2: no stores (timing)
                    // offsets from the tile's first output element (wave-uniform base)
                    __bf16* tb = ep.dgu + (long)(i0 + r0) * ep.ld + j0;
                    const unsigned o = (unsigned)(((long)i * ep.ld + c * 8) * 2);
                    st16<BPE_GPP_POL_SWB>(tb, o, dg);
                    st16<BPE_GPP_POL_SWB>(tb, o + (unsigned)ep.F * 2, du);
                }
            }
        } else if constexpr (EPI == EPI_SWIGLU_FWD) {
            // row i: g = staged columns [0, 128), u = [128, 256); 16 threads x 16 bytes per 256-byte segment
            __builtin_amdgcn_s_waitcnt(0xc07f);
            bar();
            if (h == 0) GPP_STAMP_T(sid, 3);
            const int c = tid & 15;
#pragma unroll 4
            for (int q = 0; q < 8 / NPASS; ++q) {
                const int i = q * 32 + (tid >> 4);
                const u16x8 gv = *reinterpret_cast<const u16x8*>(stg + i * 512 + ((c ^ (i & 15)) << 4));
                const u16x8 uv = *reinterpret_cast<const u16x8*>(stg + i * 512 + (((16 + c) ^ (i & 15)) << 4));
                u16x8 av;
#if BPE_GPP_PK
#pragma unroll
                for (int e = 0; e < 8; e += 2) {
                    const f32x2 gg = {bf2f(gv[e]), bf2f(gv[e + 1])};
                    const f32x2 a = gg * fast_sigmoid2(gg) * f32x2{bf2f(uv[e]), bf2f(uv[e + 1])};
                    av[e] = f2bf(a.x);
                    av[e + 1] = f2bf(a.y);
                }
#else
#pragma unroll
                for (int e = 0; e < 8; ++e) {
                    const float gg = bf2f(gv[e]);
                    av[e] = f2bf(gg * fast_sigmoid(gg) * bf2f(uv[e]));
                }
#endif
                const long r = i0 + r0 + i;
                // gu is next read by the backward, long after this step's forward: streaming stores
                if (st_on) {
                    __bf16* tg = ep.dgu + (long)(i0 + r0) * ep.ld + jb;
                    const unsigned og = (unsigned)(((long)i * ep.ld + c * 8) * 2);
                    st16<BPE_GPP_POL_SWF_GU>(tg, og, gv);
                    st16<BPE_GPP_POL_SWF_GU>(tg, og + (unsigned)ep.F * 2, uv);
                    st16<BPE_GPP_POL_SWF_A>(ep.act + (long)(i0 + r0) * ep.ld_act + jb,
                                            (unsigned)(((long)i * ep.ld_act + c * 8) * 2), av);
                }
            }
        } else if constexpr (EPI == EPI_SWIGLU_BWD8) {
            // in two 64-row halves (registers: one half's g / u and e5m2 results at a time); per half, dg then du go
            // through the 64 x 256 byte transpose tile (xtra, rows of 272 bytes) into dgu8t
            static_assert(NPASS == 2, "the transpose tile covers half of one 128-row pass");
            constexpr int QB = 4;  // 16-row groups per half
            constexpr int TS = 272;  // transpose-tile row stride (bytes)
            const int c = tid & 31;
            u16x8 gv[QB], uv[QB];
            auto load_gu = [&](int b) {
#pragma unroll
                for (int qq = 0; qq < QB; ++qq) {
                    const long ro = (long)(i0 + r0 + (b * QB + qq) * 16 + (tid >> 5)) * ep.ld + j0 + c * 8;
                    gv[qq] = ld_stream(reinterpret_cast<const u16x8*>(ep.gu + ro));
                    uv[qq] = ld_stream(reinterpret_cast<const u16x8*>(ep.gu + ro + ep.F));
                }
            };
            load_gu(0);  // the first half's operands before the barrier (as EPI_SWIGLU_BWD)
            __builtin_amdgcn_s_waitcnt(0xc07f);
            bar();
            if (h == 0) GPP_STAMP_T(sid, 3);
            const float sc = ep.a_scale[0];
            float am = *amx;
            const long W = 2L * ep.F;  // dgu8 row length
            const int f4 = tid & 63, tg = tid >> 6;
#pragma unroll
            for (int b = 0; b < 2; ++b) {
                if (b == 1) load_gu(1);
                uint2 qg[QB], qu[QB];  // e5m2 dg / du of this thread's 8 columns in rows (b QB + qq) 16 + (tid >> 5)
#pragma unroll
                for (int qq = 0; qq < QB; ++qq) {
                    const int i = (b * QB + qq) * 16 + (tid >> 5);
                    const u16x8 v = *reinterpret_cast<const u16x8*>(stg + i * 512 + ((c ^ (i & 15)) << 4));
                    float dgv[8], duv[8];
#pragma unroll
                    for (int e = 0; e < 8; ++e) {  // swiglu_cast_fp8_c128_kernel<1, 1>'s arithmetic, in its order
                        const float gg = bf2f(gv[qq][e]), uu = bf2f(uv[qq][e]), dd = bf2f(v[e]);
                        const float sg = fast_sigmoid(gg);
                        const float silu = gg * sg;
                        duv[e] = bf2f(f2bf(dd * silu));
                        dgv[e] = bf2f(f2bf(dd * uu * sg * (1.f + gg * (1.f - sg))));
                        am = fmaxf(am, fabsf(dgv[e]));
                        am = fmaxf(am, fabsf(duv[e]));
                    }
                    qg[qq] = uint2{pack4_fp8<1>(dgv[0] * sc, dgv[1] * sc, dgv[2] * sc, dgv[3] * sc),
                                   pack4_fp8<1>(dgv[4] * sc, dgv[5] * sc, dgv[6] * sc, dgv[7] * sc)};
                    qu[qq] = uint2{pack4_fp8<1>(duv[0] * sc, duv[1] * sc, duv[2] * sc, duv[3] * sc),
                                   pack4_fp8<1>(duv[4] * sc, duv[5] * sc, duv[6] * sc, duv[7] * sc)};
                    if (st_on) {
                        uint8_t* row = ep.a8 + (long)(i0 + r0 + i) * W + j0 + c * 8;
                        *reinterpret_cast<uint2*>(row) = qg[qq];
                        *reinterpret_cast<uint2*>(row + ep.F) = qu[qq];
                    }
                }
#pragma unroll
                for (int o = 0; o < 2; ++o) {  // dg, then du: [64 tokens][256 columns] -> [256 columns][64 tokens]
                    if (b + o > 0) {  // the previous round's transposed reads are done before the tile is rewritten
                        __builtin_amdgcn_s_waitcnt(0xc07f);
                        bar();
                    }
#pragma unroll
                    for (int qq = 0; qq < QB; ++qq)
                        *reinterpret_cast<uint2*>(xtra + (qq * 16 + (tid >> 5)) * TS + c * 8) = o == 0 ? qg[qq] : qu[qq];
                    __builtin_amdgcn_s_waitcnt(0xc07f);
                    bar();
                    unsigned wv[8];
#pragma unroll
                    for (int k = 0; k < 8; ++k)
                        wv[k] = *reinterpret_cast<const unsigned*>(xtra + (8 * tg + k) * TS + 4 * f4);
#pragma unroll
                    for (int j = 0; j < 4; ++j) {
                        unsigned lo = 0, hi = 0;
#pragma unroll
                        for (int k = 0; k < 4; ++k) {
                            lo |= ((wv[k] >> (8 * j)) & 0xffu) << (8 * k);
                            hi |= ((wv[k + 4] >> (8 * j)) & 0xffu) << (8 * k);
                        }
                        if (st_on)
                            *reinterpret_cast<uint2*>(ep.a8t + ((long)o * ep.F + j0 + 4 * f4 + j) * ep.ld_a8t + i0 + r0 +
                                                      64 * b + 8 * tg) = uint2{lo, hi};
                    }
                }
            }
            *amx = am;
        } else if constexpr (EPI == EPI_SWIGLU_FWD8) {
            // as EPI_SWIGLU_FWD for gu; a = bf16(silu(g) u) (swiglu_cast_fp8_c128_kernel's values) is cast to e4m3
            // with the slot's scale, stored row-major from registers and, through the a8 tile in LDS (xtra), as
            // a8t; max |a| accumulates in *amx (one atomic per workgroup, by the caller)
            static_assert(NPASS == 2, "the a8 transpose tile covers one 128-row pass");
            __builtin_amdgcn_s_waitcnt(0xc07f);
            bar();
            if (h == 0) GPP_STAMP_T(sid, 3);
            const int c = tid & 15;
            const float sc = ep.a_scale[0];
            float am = *amx;
#pragma unroll 2
            for (int q = 0; q < 8 / NPASS; ++q) {
                const int i = q * 32 + (tid >> 4);
                const u16x8 gv = *reinterpret_cast<const u16x8*>(stg + i * 512 + ((c ^ (i & 15)) << 4));
                const u16x8 uv = *reinterpret_cast<const u16x8*>(stg + i * 512 + (((16 + c) ^ (i & 15)) << 4));
                float v[8];
#pragma unroll
                for (int e = 0; e < 8; ++e) {
                    const float gg = bf2f(gv[e]);
                    v[e] = bf2f(f2bf(gg * fast_sigmoid(gg) * bf2f(uv[e])));
                    am = fmaxf(am, fabsf(v[e]));
                }
                const uint2 q8 = {pack4_fp8<0>(v[0] * sc, v[1] * sc, v[2] * sc, v[3] * sc),
                                  pack4_fp8<0>(v[4] * sc, v[5] * sc, v[6] * sc, v[7] * sc)};
                if (st_on) {
                    __bf16* tg = ep.dgu + (long)(i0 + r0) * ep.ld + jb;
                    const unsigned og = (unsigned)(((long)i * ep.ld + c * 8) * 2);
                    st16<BPE_GPP_POL_SWF_GU>(tg, og, gv);
                    st16<BPE_GPP_POL_SWF_GU>(tg, og + (unsigned)ep.F * 2, uv);
                    *reinterpret_cast<uint2*>(ep.a8 + (long)(i0 + r0 + i) * ep.F + jb + c * 8) = q8;
                }
                *reinterpret_cast<uint2*>(xtra + i * A8T_STRIDE + c * 8) = q8;
            }
            *amx = am;
            __builtin_amdgcn_s_waitcnt(0xc07f);
            bar();
            // a8t rows jb + 4 f4 + j (j < 4), tokens i0 + r0 + 8 tg .. + 7: 8 words of 4 columns -> 4 x 8 bytes
            const int f4 = tid & 31, tg = tid >> 5;
            unsigned wv[8];
#pragma unroll
            for (int k = 0; k < 8; ++k) wv[k] = *reinterpret_cast<const unsigned*>(xtra + (8 * tg + k) * A8T_STRIDE + 4 * f4);
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                unsigned lo = 0, hi = 0;
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    lo |= ((wv[k] >> (8 * j)) & 0xffu) << (8 * k);
                    hi |= ((wv[k + 4] >> (8 * j)) & 0xffu) << (8 * k);
                }
                if (st_on)
                    *reinterpret_cast<uint2*>(ep.a8t + (long)(jb + 4 * f4 + j) * ep.ld_a8t + i0 + r0 + 8 * tg) =
                        uint2{lo, hi};
            }
        } else if constexpr (EPI == EPI_ROPE) {
            // this thread's 8 columns are one quarter of a pair block of one head: the cos / sin loads of its rows
            // (positions) are issued before the barrier, like the SwiGLU-backward operands
            constexpr int NQ = 16 / NPASS;
            const int c = tid & 31;
            const int col = j0 + c * 8;
            const bool rot = col < ep.rot_cols;
            const int pb = (col % ep.D) >> 1;  // first pair of the 8 columns
            f32x4 cs[NQ], sn[NQ];
            if (rot) {
#pragma unroll
                for (int q = 0; q < NQ; ++q) {
                    const long pos = (long)((i0 + r0 + q * 16 + (tid >> 5)) % ep.S) * (ep.D >> 1) + pb;
                    cs[q] = *reinterpret_cast<const f32x4*>(ep.cosT + pos);
                    sn[q] = *reinterpret_cast<const f32x4*>(ep.sinT + pos);
                }
            }
            __builtin_amdgcn_s_waitcnt(0xc07f);
            bar();
            if (h == 0) GPP_STAMP_T(sid, 3);
#pragma unroll
            for (int q = 0; q < NQ; ++q) {
                const int i = q * 16 + (tid >> 5);
                u16x8 v = *reinterpret_cast<const u16x8*>(stg + i * 512 + ((c ^ (i & 15)) << 4));
                if (rot) {
#pragma unroll
                    for (int j = 0; j < 4; ++j) {
                        const float a = bf2f(v[2 * j]), b = bf2f(v[2 * j + 1]);
                        v[2 * j] = f2bf(a * cs[q][j] - b * sn[q][j]);
                        v[2 * j + 1] = f2bf(a * sn[q][j] + b * cs[q][j]);
                    }
                }
                if (st_on) st16<BPE_GPP_POL_ROPE>(C + (long)(i0 + r0) * ldc + j0, (unsigned)(((long)i * ldc + c * 8) * 2), v);
            }
        } else {
            __builtin_amdgcn_s_waitcnt(0xc07f);
            bar();
            if (h == 0) GPP_STAMP_T(sid, 3);
#pragma unroll 4
            for (int q = 0; q < 16 / NPASS; ++q) {
                const int i = q * 16 + (tid >> 5), c = tid & 31;
                u16x8 v = *reinterpret_cast<const u16x8*>(stg + i * 512 + ((c ^ (i & 15)) << 4));
                __bf16* cp = C + (long)(i0 + r0 + i) * ldc + j0 + c * 8;
                if (beta != 0.f) {
                    const u16x8 o = *reinterpret_cast<const u16x8*>(cp);
#pragma unroll
                    for (int e = 0; e < 8; ++e) v[e] = f2bf(bf2f(v[e]) + beta * bf2f(o[e]));
                }
                if (st_on) *reinterpret_cast<u16x8*>(cp) = v;
            }
        }
        if (h + 1 < NPASS || tail) {  // every read of the image retired before it is rewritten
            __builtin_amdgcn_s_waitcnt(0xc07f);
            bar();
        }
    }
}


template <bool AK, bool BKM, bool SLAB, int DIAG, int EPI = EPI_NONE, int SPREAD = 0, int F8 = 0>
__global__ void __launch_bounds__(NT, 1)
gemm_pp_kernel(const __bf16* __restrict__ A, long lda, const __bf16* __restrict__ B, long ldb,
               float* __restrict__ slab, __bf16* __restrict__ C, long ldc, float beta, int M, int N, int R,
               int splits, Epi ep = Epi{}) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int tid = threadIdx.x, l = tid & 63;
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int g = w >> 2, wl = w & 3;
    // XCD-aware bijective remap: consecutive work ids run on one XCD (guide §5, T1)
    const int nwg = gridDim.x, orig = blockIdx.x;
    const int xcd = orig & 7, qq = nwg >> 3, rr = nwg & 7;
    const int wid = (xcd < rr ? xcd * (qq + 1) : rr * (qq + 1) + (xcd - rr) * qq) + (orig >> 3);
    const int tiles_n = N / BT;
    const int ntiles = (M / BT) * tiles_n;
    const int split = wid / ntiles, tile = wid % ntiles;
    int ti, tj;
    tile_rc(tile, M / BT, tiles_n, ep.gm, ti, tj);
    const int i0 = ti * BT, j0 = tj * BT;
    // B tile origin: EPI_SWIGLU_FWD tiles 128 g columns (+ the matching u columns, offset F rows in B)
    const int jb = is_swf(EPI) ? tj * (BT / 2) : j0;
    const int nkt = R / BK;
    const int kb = (int)((long)split * nkt / splits);
    const int nk = (int)((long)(split + 1) * nkt / splits) - kb;
    GPP_STAMP(0);
    GPP_STAMP_VAL(6, wid);
#ifdef BPE_GPP_STAMPS
    {
        unsigned xcc, hw;
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
        GPP_STAMP_VAL(7, (long long)(xcc & 15));
        GPP_STAMP_VAL(5, (long long)hw);
    }
#endif

    constexpr bool SPR = SPREAD != 0;
    if (ep.prio && g == 1) __builtin_amdgcn_s_setprio(1);  // g is wave-uniform (readfirstlane): a scalar branch
    f32x4 acc[8][4];
#pragma unroll
    for (int a = 0; a < 8; ++a)
#pragma unroll
        for (int b = 0; b < 4; ++b) acc[a][b] = f32x4{0.f, 0.f, 0.f, 0.f};

    if constexpr (SPR) {
        SpreadOff so = spread_offsets<AK, BKM>(g, wl, l, (int)lda, (int)ldb);
        if constexpr (is_swf(EPI)) {
            // group g DMAs B rows [128 g, +128) of the tile: group 1's are the u rows, F - 128 rows further on
            static_assert(BKM, "SwiGLU forward: B = [W1; W3] is K-major");
            if (g == 1) {
                const int du = (ep.F - BT / 2) * (int)ldb;
#pragma unroll
                for (int j = 0; j < 2; ++j) {
                    so.b0[j] += du;
                    so.b1[j] += du;
                }
            }
        }
        {  // prologue: all of K-tile 0 (this wave's 8 pieces of the schedule), retired before the first read
            const long k0 = (long)kb * BK;
            const __bf16* a0 = tile_ptr<AK>(A, lda, i0, k0);
            const __bf16* b0 = tile_ptr<BKM>(B, ldb, jb, k0);
            dma_pair<BPE_GPP_DMA_POL_A>(a0, so.a0, smem, so.la0);
            dma_pair<BPE_GPP_DMA_POL_B>(b0, so.b0, smem + OPB, so.lb0);
            dma_pair<BPE_GPP_DMA_POL_B>(b0, so.b1, smem + OPB, so.lb1);
            dma_pair<BPE_GPP_DMA_POL_A>(a0, so.a1, smem, so.la1);
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            bar();
        }
        GPP_STAMP(1);
        if (g == 1) bar();  // the stagger
        for (int kt = 0; kt < nk; ++kt) {
            char* cur = smem + (kt & 1) * STAGE;
            char* nxt = smem + ((kt + 1) & 1) * STAGE;
            const long k1 = (long)(kb + kt + 1) * BK;
            ktile_spread<AK, BKM, DIAG, SPREAD == 2, F8>(cur, nxt, kt + 1 < nk, tile_ptr<AK>(A, lda, i0, k1),
                                                         tile_ptr<BKM>(B, ldb, jb, k1), so, g, wl, l, acc, false, kt);
        }
    } else {
        int oa[4], ob[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int e = g * 1024 + (wl * 4 + j) * 64 + l;
            oa[j] = src_off<AK>(e, (int)lda);
            ob[j] = src_off<BKM>(e, (int)ldb);
        }
        // prologue: K-tile 0, both halves (each group its own), then retire + barrier
        {
            const long k0 = (long)kb * BK;
            dma_half(tile_ptr<AK>(A, lda, i0, k0), oa, smem, g, wl);
            dma_half(tile_ptr<BKM>(B, ldb, j0, k0), ob, smem + OPB, g, wl);
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            bar();
        }
        if (g == 1 && DIAG != 4) bar();  // the stagger: group 1 runs one barrier interval behind group 0
        for (int kt = 0; kt < nk; ++kt) {
            char* cur = smem + (kt & 1) * STAGE;
            char* nxt = smem + ((kt + 1) & 1) * STAGE;
            const bool dma = kt + 1 < nk;
            const long k1 = (long)(kb + kt + 1) * BK;
            ktile<AK, BKM, DIAG>(cur, nxt, dma, tile_ptr<AK>(A, lda, i0, k1), tile_ptr<BKM>(B, ldb, j0, k1), oa, ob, g,
                                 wl, l, acc);
        }
    }
    GPP_STAMP(2);
    if (g == 0 && DIAG != 4) bar();
    // every fragment read and LDS-DMA done: the LDS is free for the epilogue.  The builtin (not inline asm)
    // tells the compiler's wait-count model that the DMA has retired; after an asm wait it still counts the
    // LDS-DMA loads as pending, a second kind of VMEM event beside the epilogue's own loads, and then waits
    // vmcnt(0) before the first use of any of them (the SwiGLU-backward epilogue's 32 g / u loads drained
    // completely before the first row's math; now row q waits for its own pair)
    __builtin_amdgcn_s_waitcnt(0x70);  // vmcnt(0) expcnt(7) lgkmcnt(0)
    bar();

    // DIAG 6 (timing only): the epilogue's global stores are skipped (kept in the code behind a runtime test
    // that is never true, so the MFMAs and the LDS staging stay): prices the store burst at the end of each tile
    // DIAG 6 (timing only): the epilogue's global stores are skipped (kept in the code behind a runtime test
    // that is never true, so the MFMAs and the LDS staging stay): prices the store burst at the end of each tile
    const bool st_on = DIAG != 6 || ep.prio == 77;
    // accumulator (ib, jb) register r of lane l: row i = 128 g + 16 ib + (l & 15), col j = 64 wl + 16 jb + 4 (l >> 4) + r
    if constexpr (SLAB) {
        float* sp = slab + (long)split * M * N;
        float osc = 1.f;  // F8: the operands' inverse scales, applied to each partial (the reduce only sums)
        if constexpr (F8 != 0) osc = ep.sa[0] * ep.sb[0];
#pragma unroll
        for (int ib = 0; ib < 8; ++ib)
#pragma unroll
            for (int jb = 0; jb < 4; ++jb) {
                const long i = i0 + 128 * g + 16 * ib + (l & 15);
                const long j = j0 + 64 * wl + 16 * jb + 4 * (l >> 4);
                if (st_on) *reinterpret_cast<f32x4*>(sp + i * N + j) = F8 != 0 ? acc[ib][jb] * osc : acc[ib][jb];
            }
        GPP_STAMP(4);
    } else {
        epilogue_bf16<EPI, F8, 1>(acc, smem, g, wl, l, tid, i0, j0, jb, C, ldc, beta, ep, st_on, false, blockIdx.x);
        GPP_STAMP(4);
    }
#ifdef BPE_GPP_PHASE_STAMPS
    if (blockIdx.x < 1024 && l < PST_VALS)  // each wave its own values (LDS above the stages; written by itself)
        g_gpp_phase[((long)blockIdx.x * 8 + w) * PST_VALS + l] =
            *reinterpret_cast<const long long*>(smem + LDS_BYTES + (w * PST_VALS + l) * 8);
#endif
}


// Persistent form of the bf16 (or fp8) one-pass GEMM: one workgroup per CU walks tiles wid, wid + grid, ... (the
// same tile order as the one-tile kernel's XCD-aware grid).  What it removes, measured with the stamps build at
// GPT-2 B 128 (benchmarks/gemm_stamps.py): a one-tile workgroup spends ~10-12 % of its time in the prologue (K-tile
// 0's round trip) and then ~2-3k cycles pass before the CU's next workgroup runs.  Here the next tile's K-tile 0
// is DMA'd during the last K-tile of the current one (the in-loop prefetch simply continues across the seam), so
// its image is resident before the epilogue; the epilogue stages through the other 64 KiB stage in two passes
// (NPASS 2), and its stores stay in flight into the first two phases of the next tile's K-tile 0 (which wait for
// LDS only); phase 2's vmcnt wait retires them.
// (An earlier persistent form stored the accumulators from registers as 8-byte row pieces during the next tile's
// first load section and lost to the one-tile kernel: 0.74-0.89 vs 1.0 PF/s on the K = 768 forward GEMMs.)
template <bool AK, bool BKM, int EPI, int SPREAD, int F8 = 0>
__global__ void __launch_bounds__(NT, 1)
gemm_pp_persist_kernel(const __bf16* __restrict__ A, long lda, const __bf16* __restrict__ B, long ldb,
                       __bf16* __restrict__ C, long ldc, float beta, int M, int N, int R, Epi ep = Epi{}) {
    static_assert(SPREAD != 0, "the persistent kernel runs the spread DMA schedule");
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int tid = threadIdx.x, l = tid & 63;
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int g = w >> 2, wl = w & 3;
    const int nwg = gridDim.x, orig = blockIdx.x;
    const int xcd = orig & 7, qq = nwg >> 3, rr = nwg & 7;
    const int wid = (xcd < rr ? xcd * (qq + 1) : rr * (qq + 1) + (xcd - rr) * qq) + (orig >> 3);
    const int tiles_n = N / BT;
    const int ntiles = (M / BT) * tiles_n;
    const int nk = R / BK;
    if (ep.prio && g == 1) __builtin_amdgcn_s_setprio(1);
    SpreadOff so = spread_offsets<AK, BKM>(g, wl, l, (int)lda, (int)ldb);
    if constexpr (is_swf(EPI)) {
        static_assert(BKM, "SwiGLU forward: B = [W1; W3] is K-major");
        if (g == 1) {
            const int du = (ep.F - BT / 2) * (int)ldb;
#pragma unroll
            for (int j = 0; j < 2; ++j) {
                so.b0[j] += du;
                so.b1[j] += du;
            }
        }
    }
    // tile t: output origin (i0, j0) and B origin jb (EPI_SWIGLU_FWD: 128 g columns + the matching u columns)
    auto origin = [&](int t, int& i0, int& j0, int& jb) {
        int ti, tj;
        tile_rc(t, M / BT, tiles_n, ep.gm, ti, tj);
        i0 = ti * BT;
        j0 = tj * BT;
        jb = is_swf(EPI) ? tj * (BT / 2) : j0;
    };
    int t = wid, i0, j0, jb;
    origin(t, i0, j0, jb);
    {  // prologue of the first tile: all of its K-tile 0, retired before the first read
        const __bf16* a0 = tile_ptr<AK>(A, lda, i0, 0);
        const __bf16* b0 = tile_ptr<BKM>(B, ldb, jb, 0);
        dma_pair<BPE_GPP_DMA_POL_A>(a0, so.a0, smem, so.la0);
        dma_pair<BPE_GPP_DMA_POL_B>(b0, so.b0, smem + OPB, so.lb0);
        dma_pair<BPE_GPP_DMA_POL_B>(b0, so.b1, smem + OPB, so.lb1);
        dma_pair<BPE_GPP_DMA_POL_A>(a0, so.a1, smem, so.la1);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        bar();
    }
    int st = 0;  // the stage holding the current K-tile
    f32x4 acc[8][4];
    float amx = 0.f;  // EPI_SWIGLU_FWD8: this thread's max |a| over its tiles
#ifdef BPE_GPP_STAMPS
    unsigned xcc_id, hw_id;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc_id));
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw_id));
#endif
    for (;;) {
        GPP_STAMP_T(t, 0);
#ifdef BPE_GPP_STAMPS
        if (threadIdx.x == 0) {
            g_gpp_stamps[(long)(t & 65535) * 8 + 5] = hw_id;
            g_gpp_stamps[(long)(t & 65535) * 8 + 6] = wid;
            g_gpp_stamps[(long)(t & 65535) * 8 + 7] = xcc_id & 15;
        }
#endif
        const int tn = t + nwg;
        const bool more = tn < ntiles;
        int i0n = i0, j0n = j0, jbn = jb;
        if (more) origin(tn, i0n, j0n, jbn);
#pragma unroll
        for (int a = 0; a < 8; ++a)
#pragma unroll
            for (int b = 0; b < 4; ++b) acc[a][b] = f32x4{0.f, 0.f, 0.f, 0.f};
        if (g == 1) bar();  // the stagger
        GPP_STAMP_T(t, 1);
        for (int kt = 0; kt < nk; ++kt) {
            char* cur = smem + st * STAGE;
            char* nxt = smem + (st ^ 1) * STAGE;
            const bool last = kt + 1 == nk;
            // the next K-tile of this tile, or K-tile 0 of the next tile
            const __bf16* an = last ? tile_ptr<AK>(A, lda, i0n, 0) : tile_ptr<AK>(A, lda, i0, (long)(kt + 1) * BK);
            const __bf16* bn = last ? tile_ptr<BKM>(B, ldb, jbn, 0) : tile_ptr<BKM>(B, ldb, jb, (long)(kt + 1) * BK);
            ktile_spread<AK, BKM, 0, SPREAD == 2, F8>(cur, nxt, !last || more, an, bn, so, g, wl, l, acc, kt == 0);
            st ^= 1;
        }
        GPP_STAMP_T(t, 2);
        if (g == 0) bar();
        // the next tile's K-tile 0 (stage st) retired; the stage just read (st ^ 1) is free for the staging
        __builtin_amdgcn_s_waitcnt(0x70);
        bar();
        // (Measured and dropped, round 6: the SwiGLU-backward epilogue straight from the accumulators -- no LDS
        // staging, lane pairs swapping halves into 16-byte chunks, every g / u load issued before the first store
        // -- 0.77 vs 0.69 ms, profiles/bench/ab_swiglu_bwd_reg_epilogue_r6.log: each access instruction then covers
        // 16 rows x 2 x 32 B instead of 2 rows x 512 B.)
        epilogue_bf16<EPI, F8, 2>(acc, smem + (st ^ 1) * STAGE, g, wl, l, tid, i0, j0, jb, C, ldc, beta, ep, true,
                                  more, t, smem + LDS_LAUNCH, &amx);
        GPP_STAMP_T(t, 4);
        if (!more) break;
        t = tn;
        i0 = i0n;
        j0 = j0n;
        jb = jbn;
    }
    if constexpr (EPI == EPI_SWIGLU_FWD8 || EPI == EPI_SWIGLU_BWD8) {  // the workgroup's max: one atomic per workgroup
        float m = amx;
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o, 64));
        float* red = reinterpret_cast<float*>(smem + LDS_LAUNCH);
        __syncthreads();  // every wave is done with the a8 tile
        if (l == 0) red[w] = m;
        __syncthreads();
        if (tid == 0) {
#pragma unroll
            for (int i = 1; i < NT / 64; ++i) m = fmaxf(m, red[i]);
            atomicMax(ep.a_amax, __float_as_uint(m));  // amax >= 0: the bit pattern orders as the float
        }
    }
}

// Grouped weight gradients: the dW GEMMs of one layer that become ready together (W2 + [W1; W3] after the
// SwiGLU-backward GEMM, Wo + [Wq; Wk; Wv] after the attention backward) in ONE split-K launch.  Each problem p is
// dW_p[M_p][N_p] += dY_p^T X_p with dY_p [R][M_p] and X_p [R][N_p] token-major (or X_p^T [N_p][R] when BKM: the
// transposed-copy route) over the same R tokens; their tiles are concatenated into one tile list and every tile
// is split over K the same `splits` ways.  Why: a layer's dW shapes have 9-48 output tiles each, and a tile count
// times a split count rarely fills whole waves of 256 CUs -- alone, GPT-2's W2 / W13 / Wo / Wqkv dW ran 240 / 240 /
// 243 / 243 workgroups for 256 CUs, 5-6 % of the chip idle, plus a separate reduce launch each
// (profiles/bench/dw_stamps_r6.log).  Grouped, the tiles x splits product is chosen for the whole set
// (ops/gemm.py choose_splits_group).  The workgroup order is split-major with consecutive work ids on one XCD,
// so the workgroups that read the same tokens (one split) share their dY / X rows in that XCD's L2.  Partials
// go to each problem's fp32 slab region [splits][M_p][N_p] and dwg_reduce_kernel sums them in split order:
// deterministic, bitwise equal to the single-problem split-K kernel at the same split count.
constexpr int DWG_MAX = 4;
struct DwGroup {
    const __bf16* A[DWG_MAX];
    const __bf16* B[DWG_MAX];
    long lda[DWG_MAX], ldb[DWG_MAX];
    long slab_off[DWG_MAX];  // float offset of problem p's slab region [splits][M_p][N_p]
    int M[DWG_MAX], N[DWG_MAX];
    int tile_end[DWG_MAX];  // inclusive prefix sums of the problems' tile counts
    int np, ntiles, splits, R;
    int prio;
};

template <bool BKM>
__global__ void __launch_bounds__(NT, 1) gemm_pp_dwg_kernel(DwGroup gp, float* __restrict__ slab) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int tid = threadIdx.x, l = tid & 63;
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int g = w >> 2, wl = w & 3;
    const int nwg = gridDim.x, orig = blockIdx.x;
    const int xcd = orig & 7, qq = nwg >> 3, rr = nwg & 7;
    const int wid = (xcd < rr ? xcd * (qq + 1) : rr * (qq + 1) + (xcd - rr) * qq) + (orig >> 3);
    const int split = wid / gp.ntiles, gt = wid % gp.ntiles;
    // the problem of global tile gt, selected with constant indices only (no dynamic indexing of the kernarg
    // arrays, which hipcc would copy to scratch)
    const __bf16* A = gp.A[0];
    const __bf16* B = gp.B[0];
    long lda = gp.lda[0], ldb = gp.ldb[0], soff = gp.slab_off[0];
    int M = gp.M[0], N = gp.N[0], t0 = 0;
#pragma unroll
    for (int q = 1; q < DWG_MAX; ++q) {
        if (q < gp.np && gt >= gp.tile_end[q - 1]) {
            A = gp.A[q];
            B = gp.B[q];
            lda = gp.lda[q];
            ldb = gp.ldb[q];
            soff = gp.slab_off[q];
            M = gp.M[q];
            N = gp.N[q];
            t0 = gp.tile_end[q - 1];
        }
    }
    const int tile = gt - t0, tiles_n = N / BT;
    const int i0 = (tile / tiles_n) * BT, j0 = (tile % tiles_n) * BT;
    const int nkt = gp.R / BK;
    const int kb = (int)((long)split * nkt / gp.splits);
    const int nk = (int)((long)(split + 1) * nkt / gp.splits) - kb;
    GPP_STAMP(0);
    GPP_STAMP_VAL(6, wid);
#ifdef BPE_GPP_STAMPS
    {
        unsigned xcc, hw;
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
        GPP_STAMP_VAL(7, (long long)(xcc & 15));
        GPP_STAMP_VAL(5, (long long)hw);
    }
#endif
    if (gp.prio && g == 1) __builtin_amdgcn_s_setprio(1);
    f32x4 acc[8][4];
#pragma unroll
    for (int a = 0; a < 8; ++a)
#pragma unroll
        for (int b = 0; b < 4; ++b) acc[a][b] = f32x4{0.f, 0.f, 0.f, 0.f};
    // BKM (X^T copy, B K-major): the forward GEMM's spread schedule (1); both token-major: the weight-gradient
    // one with a DMA piece inside each MFMA section (2) -- the same choices as the single-problem routes
    constexpr bool SPLIT = !BKM;
    const SpreadOff so = spread_offsets<false, BKM>(g, wl, l, (int)lda, (int)ldb);
    {
        const long k0 = (long)kb * BK;
        const __bf16* a0 = tile_ptr<false>(A, lda, i0, k0);
        const __bf16* b0 = tile_ptr<BKM>(B, ldb, j0, k0);
        dma_pair<BPE_GPP_DMA_POL_A>(a0, so.a0, smem, so.la0);
        dma_pair<BPE_GPP_DMA_POL_B>(b0, so.b0, smem + OPB, so.lb0);
        dma_pair<BPE_GPP_DMA_POL_B>(b0, so.b1, smem + OPB, so.lb1);
        dma_pair<BPE_GPP_DMA_POL_A>(a0, so.a1, smem, so.la1);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        bar();
    }
    GPP_STAMP(1);
    if (g == 1) bar();  // the stagger
    for (int kt = 0; kt < nk; ++kt) {
        char* cur = smem + (kt & 1) * STAGE;
        char* nxt = smem + ((kt + 1) & 1) * STAGE;
        const long k1 = (long)(kb + kt + 1) * BK;
        ktile_spread<false, BKM, 0, SPLIT, 0>(cur, nxt, kt + 1 < nk, tile_ptr<false>(A, lda, i0, k1),
                                              tile_ptr<BKM>(B, ldb, j0, k1), so, g, wl, l, acc, false, kt);
    }
    GPP_STAMP(2);
    if (g == 0) bar();
    __builtin_amdgcn_s_waitcnt(0x70);
    bar();
    float* sp = slab + soff + (long)split * M * N;
#pragma unroll
    for (int ib = 0; ib < 8; ++ib)
#pragma unroll
        for (int jq = 0; jq < 4; ++jq) {
            const long i = i0 + 128 * g + 16 * ib + (l & 15);
            const long j = j0 + 64 * wl + 16 * jq + 4 * (l >> 4);
            *reinterpret_cast<f32x4*>(sp + i * N + j) = acc[ib][jq];
        }
    GPP_STAMP(4);
}

// C_p = beta * C_p + sum over splits of problem p's slab region, in split order (the grouped form of
// splitk_reduce_kernel: one launch for every problem of a group).  end4[p]: inclusive prefix sums of M_p N_p / 4.
struct DwOut {
    void* C[DWG_MAX];
    long ldc[DWG_MAX];
    long slab_off[DWG_MAX];
    long end4[DWG_MAX];
    int N[DWG_MAX];
    int np, splits;
    float beta;
};

template <typename CT>
__global__ void __launch_bounds__(256) dwg_reduce_kernel(const float* __restrict__ slab, DwOut o) {
    const long total4 = o.end4[o.np - 1];
    for (long t = blockIdx.x * 256L + threadIdx.x; t < total4; t += (long)gridDim.x * 256) {
        CT* C = (CT*)o.C[0];
        long ldc = o.ldc[0], soff = o.slab_off[0], b4 = 0, mn = o.end4[0] * 4;
        int N = o.N[0];
#pragma unroll
        for (int q = 1; q < DWG_MAX; ++q) {
            if (q < o.np && t >= o.end4[q - 1]) {
                C = (CT*)o.C[q];
                ldc = o.ldc[q];
                soff = o.slab_off[q];
                b4 = o.end4[q - 1];
                mn = (o.end4[q] - o.end4[q - 1]) * 4;
                N = o.N[q];
            }
        }
        const long e = (t - b4) * 4;
        const long i = e / N, j = e % N;
        const float* sp = slab + soff + e;
        f32x4 s = *reinterpret_cast<const f32x4*>(sp);
        for (int k = 1; k < o.splits; ++k) s += *reinterpret_cast<const f32x4*>(sp + (long)k * mn);
        if constexpr (sizeof(CT) == 4) {
            f32x4* cp = reinterpret_cast<f32x4*>(C + i * ldc + j);
            if (o.beta != 0.f) s += o.beta * *cp;
            *cp = s;
        } else {
            u16x4* cp = reinterpret_cast<u16x4*>(C + i * ldc + j);
            if (o.beta != 0.f) {
                const u16x4 c = *cp;
                s[0] += o.beta * bf2f(c[0]);
                s[1] += o.beta * bf2f(c[1]);
                s[2] += o.beta * bf2f(c[2]);
                s[3] += o.beta * bf2f(c[3]);
            }
            *cp = u16x4{f2bf(s[0]), f2bf(s[1]), f2bf(s[2]), f2bf(s[3])};
        }
    }
}

}  // namespace gpp
}  // namespace bpe

using namespace bpe::gpp;

// Static s_setprio 1 for the younger wave group: end to end +0.1-0.6 % (profiles/bench/ab_e2e_gpp_prio.log).
static int prio_mode() { return 1; }

// DMA schedule: 1 = the spread schedule (ktile_spread), 2 = spread with one piece per section moved into the MFMA
// section: 2 for the weight gradient (both operands MN-major: +1-3 %), 1 for the rest (2 is 3 % slower there;
// profiles/bench/ab_gpp_dma_split.log).  0, the burst schedule of ktile, serves the DIAG 5 build only.
static int spread_mode(bool weight_grad = false) { return weight_grad ? 2 : 1; }

// Persistent kernel (gemm_pp_persist_kernel) for the one-pass bf16 / fp8 GEMMs: 1 = on (one workgroup per CU),
// 0 = the one-tile kernel, n >= 2 = on with at most n workgroups (tests: many tiles per workgroup on small shapes).
#ifndef BPE_GPP_PERSIST  // build define: the default form (variant builds A/B the one-tile kernel with 0)
#define BPE_GPP_PERSIST 1
#endif
static int g_persist = BPE_GPP_PERSIST;
int gpp_persist_config(int mode) {
    const int prev = g_persist;
    if (mode >= 0) g_persist = mode;
    return prev;
}

// Tile order of the one-pass GEMMs (Epi::gm, tile_rc): 0 = row-major; n > 0 = column-major within bands of n row
// blocks; -2 = auto: bands of 2 row blocks up to 10 column tiles, 4 above.  Measured per GEMM at GPT-2 B 128 and
// Llama s2048 (benchmarks/gemm_tile_order.py, profiles/bench/gemm_tile_order_r6.log): the SwiGLU forward -9 / -10 %,
// the plain W13 forward -4 / -7 %, the Llama SwiGLU backward -3 %, QKV + RoPE -1.5 % at 9 column tiles with 2 (4
// is 2 % slower there).  Set at run time for A/B (gpp_order_config, or BPE_GPP_GM in the environment); the split-K
// weight-gradient launches keep row-major, the fp8 ones too in auto mode (order_fp8).
static int g_gm = [] {
    const char* e = getenv("BPE_GPP_GM");
    return e && *e ? atoi(e) : -2;
}();
int gpp_order_config(int gm) {
    const int prev = g_gm;
    if (gm >= 0 || gm < -1) g_gm = gm < -1 ? -2 : gm;
    return prev;
}
static int order_for(int tiles_n) { return g_gm >= 0 ? g_gm : (tiles_n <= 10 ? 2 : 4); }
// the fp8 one-pass GEMMs stay row-major in auto mode: the Llama fp8 s4096 step ran 0.5 % slower with the bf16 rule
static int order_fp8() { return g_gm >= 0 ? g_gm : 0; }

static int num_cus() {
    static int n[16] = {};
    int dev = 0;
    (void)hipGetDevice(&dev);
    int& c = n[dev & 15];
    if (c == 0 && hipDeviceGetAttribute(&c, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) c = 256;
    return c;
}

// launch the persistent kernel k over ntiles tiles: one workgroup per CU
template <typename K, typename... Args>
static void launch_persist(K* k, int ntiles, hipStream_t s, Args... args) {
    static_assert(sizeof...(Args) > 0, "");
    const int cap = g_persist >= 2 ? g_persist : num_cus();  // mode >= 2: a test hook, at most `mode` workgroups
    const int grid = ntiles < cap ? ntiles : cap;
    k<<<grid, NT, LDS_LAUNCH, s>>>(args...);
}

template <typename K>
static void lds_attr(K* k) {  // > 64 KiB dynamic LDS must be opted into once per instantiation
    (void)hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, LDS_LAUNCH);
}

// dgu = swiglu_bwd(dY . W2, gu): A = dY [M][R] (K-major), B = W2 [R][F] (MN-major)
void launch_gemm_pp_swiglu_bwd(const void* dY, long ldy, const void* W2, long ldw, const void* gu, void* dgu,
                               long ldg, int M, int F, int R, hipStream_t s) {
    static bool attr = false;
    auto* k = &gemm_pp_kernel<true, false, false, 0, EPI_SWIGLU_BWD, 1>;
    if (!attr) {
        (void)hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, LDS_LAUNCH);
        attr = true;
    }
    const int grid = (M / BT) * (F / BT);
    Epi ep{(const __bf16*)gu, (__bf16*)dgu, ldg, F};
    ep.prio = prio_mode();
    ep.gm = order_for(F / BT);
    if (g_persist) {
        static bool pattr = false;
        auto* kp = &gemm_pp_persist_kernel<true, false, EPI_SWIGLU_BWD, 1>;
        if (!pattr) lds_attr(kp), pattr = true;
        return launch_persist(kp, grid, s, (const __bf16*)dY, ldy, (const __bf16*)W2, ldw, (__bf16*)nullptr, 0L, 0.f,
                              M, F, R, ep);
    }
    k<<<grid, NT, LDS_LAUNCH, s>>>((const __bf16*)dY, ldy, (const __bf16*)W2, ldw, nullptr, nullptr, 0, 0.f, M, F, R,
                                  1, ep);
}

// gu = X . [W1; W3]^T and a = silu(g) * u (EPI_SWIGLU_FWD): X [M][R], W13 [2F][R] (both K-major)
void launch_gemm_pp_swiglu_fwd(const void* X, long ldx, const void* W13, long ldw, void* gu, long ldg, void* act,
                               long lda_, int M, int F, int R, hipStream_t s) {
    static bool attr = false;
    auto* k = &gemm_pp_kernel<true, true, false, 0, EPI_SWIGLU_FWD, 1>;
    if (!attr) {
        (void)hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, LDS_LAUNCH);
        attr = true;
    }
    const int grid = (M / BT) * (F / (BT / 2));
    Epi ep{nullptr, (__bf16*)gu, ldg, F, (__bf16*)act, lda_};
    ep.prio = prio_mode();
    ep.gm = order_for(F / (BT / 2));
    if (g_persist) {
        static bool pattr = false;
        auto* kp = &gemm_pp_persist_kernel<true, true, EPI_SWIGLU_FWD, 1>;
        if (!pattr) lds_attr(kp), pattr = true;
        return launch_persist(kp, grid, s, (const __bf16*)X, ldx, (const __bf16*)W13, ldw, (__bf16*)nullptr, 0L, 0.f,
                              M, 2 * F, R, ep);
    }
    k<<<grid, NT, LDS_LAUNCH, s>>>((const __bf16*)X, ldx, (const __bf16*)W13, ldw, nullptr, nullptr, 0, 0.f, M, 2 * F,
                                  R, 1, ep);
}

// qkv = X . Wqkv^T with RoPE on columns [0, rot_cols) (EPI_ROPE): X [M][R], Wqkv [N][R] (both K-major)
void launch_gemm_pp_rope(const void* X, long ldx, const void* W, long ldw, void* C, long ldc, int M, int N, int R,
                         const float* cosT, const float* sinT, int S, int D, int rot_cols, hipStream_t s) {
    Epi ep{};
    ep.prio = prio_mode();
    ep.gm = order_for(N / BT);
    ep.cosT = cosT;
    ep.sinT = sinT;
    ep.S = S;
    ep.D = D;
    ep.rot_cols = rot_cols;
    const int ntiles = (M / BT) * (N / BT);
    if (g_persist) {
        static bool pattr = false;
        auto* kp = &gemm_pp_persist_kernel<true, true, EPI_ROPE, 1>;
        if (!pattr) lds_attr(kp), pattr = true;
        return launch_persist(kp, ntiles, s, (const __bf16*)X, ldx, (const __bf16*)W, ldw, (__bf16*)C, ldc, 0.f, M,
                              N, R, ep);
    }
    static bool attr = false;
    auto* k = &gemm_pp_kernel<true, true, false, 0, EPI_ROPE, 1>;
    if (!attr) lds_attr(k), attr = true;
    k<<<ntiles, NT, LDS_LAUNCH, s>>>((const __bf16*)X, ldx, (const __bf16*)W, ldw, nullptr, (__bf16*)C, ldc, 0.f, M,
                                    N, R, 1, ep);
}

// C[M][N] (bf16) = (A8 . B8^T) * sa * sb with A8 [M][K], B8 [N][K] fp8 row-major (K-major), row strides in
// bytes; fmt_a 0 = e4m3, 1 = e5m2; B is e4m3.  M, N multiples of 256, K of 128, strides of 16 bytes.
void launch_gemm_fp8(const void* A, long lda, const void* B, long ldb, void* C, long ldc, int M, int N, int K,
                     int fmt_a, const float* sa, const float* sb, hipStream_t s) {
    static bool attr1 = false, attr2 = false;
    auto* k1 = &gemm_pp_kernel<true, true, false, 0, EPI_NONE, 1, 1>;
    auto* k2 = &gemm_pp_kernel<true, true, false, 0, EPI_NONE, 1, 2>;
    auto* k = fmt_a == 1 ? k2 : k1;
    bool& attr = fmt_a == 1 ? attr2 : attr1;
    if (!attr) {
        (void)hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, LDS_LAUNCH);
        attr = true;
    }
    Epi ep{};
    ep.prio = prio_mode();
    ep.gm = order_fp8();
    ep.sa = sa;
    ep.sb = sb;
    // the fp8 rows as bf16 rows of half the length: R = K / 2 "bf16" elements = K / 128 K-tiles of 128 fp8
    if (g_persist) {
        static bool pattr1 = false, pattr2 = false;
        auto* kp = fmt_a == 1 ? &gemm_pp_persist_kernel<true, true, EPI_NONE, 1, 2>
                              : &gemm_pp_persist_kernel<true, true, EPI_NONE, 1, 1>;
        bool& pa = fmt_a == 1 ? pattr2 : pattr1;
        if (!pa) lds_attr(kp), pa = true;
        return launch_persist(kp, (M / BT) * (N / BT), s, (const __bf16*)A, lda / 2, (const __bf16*)B, ldb / 2,
                              (__bf16*)C, ldc, 0.f, M, N, K / 2, ep);
    }
    k<<<(M / BT) * (N / BT), NT, LDS_LAUNCH, s>>>((const __bf16*)A, lda / 2, (const __bf16*)B, ldb / 2, nullptr,
                                                  (__bf16*)C, ldc, 0.f, M, N, K / 2, 1, ep);
}

// qkv = (X8 . Wqkv8^T) * sa * sb (e4m3 x e4m3, K-major) with RoPE on output columns [0, rot_cols) in the epilogue:
// the fp8 QKV projection and the in-place rope_qk_ pass in one kernel (the scaled product is rounded to bf16 and
// rotated exactly as launch_gemm_fp8 + rope_qk_kernel do it)
void launch_gemm_fp8_rope(const void* A, long lda, const void* B, long ldb, void* C, long ldc, int M, int N, int K,
                          const float* sa, const float* sb, const float* cosT, const float* sinT, int S, int D,
                          int rot_cols, hipStream_t s) {
    Epi ep{};
    ep.prio = prio_mode();
    ep.gm = order_fp8();
    ep.sa = sa;
    ep.sb = sb;
    ep.cosT = cosT;
    ep.sinT = sinT;
    ep.S = S;
    ep.D = D;
    ep.rot_cols = rot_cols;
    if (g_persist) {
        static bool pattr = false;
        auto* kp = &gemm_pp_persist_kernel<true, true, EPI_ROPE, 1, 1>;
        if (!pattr) lds_attr(kp), pattr = true;
        return launch_persist(kp, (M / BT) * (N / BT), s, (const __bf16*)A, lda / 2, (const __bf16*)B, ldb / 2,
                              (__bf16*)C, ldc, 0.f, M, N, K / 2, ep);
    }
    static bool attr = false;
    auto* k = &gemm_pp_kernel<true, true, false, 0, EPI_ROPE, 1, 1>;
    if (!attr) lds_attr(k), attr = true;
    k<<<(M / BT) * (N / BT), NT, LDS_LAUNCH, s>>>((const __bf16*)A, lda / 2, (const __bf16*)B, ldb / 2, nullptr,
                                                  (__bf16*)C, ldc, 0.f, M, N, K / 2, 1, ep);
}

// gu = (X8 . W13_8^T) * sa * sb (e4m3 x e4m3, K-major; W13_8 = [W1; W3] [2F][K]) with a = silu(g) u cast to e4m3
// (scale a_scale) in both layouts a8 [M][F], a8t [F][M] and max |a| folded into *a_amax (EPI_SWIGLU_FWD8).  M a
// multiple of 256, F of 128, K of 128.  Always the persistent kernel (g_persist >= 2 caps its grid, as elsewhere).
void launch_gemm_fp8_swiglu(const void* A8, long lda, const void* B8, long ldb, void* gu, long ldg, void* a8,
                            void* a8t, int M, int F, int K, const float* sa, const float* sb, const float* a_scale,
                            unsigned* a_amax, hipStream_t s) {
    Epi ep{nullptr, (__bf16*)gu, ldg, F};
    ep.prio = prio_mode();
    // bands of 8 row blocks: the Llama fp8 W13 GEMM 1.17 vs 1.32 ms row-major (profiles/bench/fp8_gemm_orders_r6.log)
    ep.gm = g_gm >= 0 ? g_gm : 8;
    ep.sa = sa;
    ep.sb = sb;
    ep.a8 = (uint8_t*)a8;
    ep.a8t = (uint8_t*)a8t;
    ep.ld_a8t = M;
    ep.a_scale = a_scale;
    ep.a_amax = a_amax;
    auto* kp = &gemm_pp_persist_kernel<true, true, EPI_SWIGLU_FWD8, 1, 1>;
    static bool pattr = false;
    if (!pattr) {
        (void)hipFuncSetAttribute((const void*)kp, hipFuncAttributeMaxDynamicSharedMemorySize, LDS_LAUNCH + A8T_BYTES);
        pattr = true;
    }
    const int ntiles = (M / BT) * (F / (BT / 2));
    const int cap = g_persist >= 2 ? g_persist : num_cus();
    kp<<<ntiles < cap ? ntiles : cap, NT, LDS_LAUNCH + A8T_BYTES, s>>>((const __bf16*)A8, lda / 2,
                                                                       (const __bf16*)B8, ldb / 2, (__bf16*)nullptr,
                                                                       0L, 0.f, M, 2 * F, K / 2, ep);
}

// da = (G8 . W2t_8^T) * sa * sb (G8 e5m2 [M][K], W2t_8 e4m3 [F][K], both K-major) with the SwiGLU backward over gu
// ([M][2F] bf16) and the two-layout e5m2 cast of [dg | du] (scale d_scale) into dgu8 [M][2F] / dgu8t [2F][M], the
// max folded into *d_amax (EPI_SWIGLU_BWD8).  M a multiple of 256, F of 256, K of 128.  Persistent kernel only.
void launch_gemm_fp8_swiglu_bwd(const void* G8, long ldg8, const void* W8, long ldw8, const void* gu, void* dgu8,
                                void* dgu8t, int M, int F, int K, const float* sa, const float* sb,
                                const float* d_scale, unsigned* d_amax, hipStream_t s) {
    Epi ep{(const __bf16*)gu, nullptr, 2L * F, F};
    ep.prio = prio_mode();
    ep.gm = g_gm >= 0 ? g_gm : 8;
    ep.sa = sa;
    ep.sb = sb;
    ep.a8 = (uint8_t*)dgu8;
    ep.a8t = (uint8_t*)dgu8t;
    ep.ld_a8t = M;
    ep.a_scale = d_scale;
    ep.a_amax = d_amax;
    auto* kp = &gemm_pp_persist_kernel<true, true, EPI_SWIGLU_BWD8, 1, 2>;
    static bool pattr = false;
    if (!pattr) {
        (void)hipFuncSetAttribute((const void*)kp, hipFuncAttributeMaxDynamicSharedMemorySize, LDS_LAUNCH + A8T_BYTES);
        pattr = true;
    }
    const int ntiles = (M / BT) * (F / BT);
    const int cap = g_persist >= 2 ? g_persist : num_cus();
    kp<<<ntiles < cap ? ntiles : cap, NT, LDS_LAUNCH + A8T_BYTES, s>>>((const __bf16*)G8, ldg8 / 2,
                                                                       (const __bf16*)W8, ldw8 / 2, (__bf16*)nullptr,
                                                                       0L, 0.f, M, F, K / 2, ep);
}

// C = beta * C + (A8 . B8^T) * sa * sb, split over K into `splits` fp32 partials (slab [splits][M][N]) summed in a
// fixed order by splitk_reduce: the fp8 weight-gradient GEMM (few output tiles, K = all tokens).  C bf16 or fp32.
void launch_gemm_fp8_splitk(const void* A, long lda, const void* B, long ldb, void* C, long ldc, int M, int N, int K,
                            int fmt_a, const float* sa, const float* sb, float beta, int splits, float* slab,
                            int c_f32, hipStream_t s) {
    static bool attr1 = false, attr2 = false;
    auto* k1 = &gemm_pp_kernel<true, true, true, 0, EPI_NONE, 1, 1>;
    auto* k2 = &gemm_pp_kernel<true, true, true, 0, EPI_NONE, 1, 2>;
    auto* k = fmt_a == 1 ? k2 : k1;
    bool& attr = fmt_a == 1 ? attr2 : attr1;
    if (!attr) lds_attr(k), attr = true;
    Epi ep{};
    ep.prio = prio_mode();
    ep.sa = sa;
    ep.sb = sb;
    k<<<(M / BT) * (N / BT) * splits, NT, LDS_LAUNCH, s>>>((const __bf16*)A, lda / 2, (const __bf16*)B, ldb / 2, slab,
                                                           nullptr, 0, 0.f, M, N, K / 2, splits, ep);
    splitk_reduce(slab, C, ldc, beta, M, N, splits, c_f32, s);
}

bool gemm_pp_shape_ok(int M, int N, int R, int splits) {
    return M % BT == 0 && N % BT == 0 && R % BK == 0 && splits >= 1 && R / BK >= splits;
}


template <bool AK, bool BKM, bool SLAB, int DIAG, int SPREAD>
static void launch_pp1s(const __bf16* a, long lda, const __bf16* b, long ldb, float* slab, __bf16* c, long ldc,
                        float beta, int M, int N, int R, int splits, hipStream_t s) {
    static bool attr = false;  // > 64 KiB dynamic LDS must be opted into once per instantiation
    auto* k = &gemm_pp_kernel<AK, BKM, SLAB, DIAG, EPI_NONE, SPREAD>;
    if (!attr) {
        (void)hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, LDS_LAUNCH);
        attr = true;
    }
    const int grid = (M / BT) * (N / BT) * splits;
    Epi ep{};
    ep.prio = prio_mode();
    ep.gm = SLAB ? (g_gm >= 0 ? g_gm : 0) : order_for(N / BT);
    if constexpr (!SLAB && DIAG == 0 && SPREAD != 0) {
        if (g_persist) {
            static bool pattr = false;
            auto* kp = &gemm_pp_persist_kernel<AK, BKM, EPI_NONE, SPREAD>;
            if (!pattr) lds_attr(kp), pattr = true;
            return launch_persist(kp, grid, s, a, lda, b, ldb, c, ldc, beta, M, N, R, ep);
        }
    }
    k<<<grid, NT, LDS_LAUNCH, s>>>(a, lda, b, ldb, slab, c, ldc, beta, M, N, R, splits, ep);
}

template <bool AK, bool BKM, bool SLAB, int DIAG>
static void launch_pp1(const __bf16* a, long lda, const __bf16* b, long ldb, float* slab, __bf16* c, long ldc,
                      float beta, int M, int N, int R, int splits, hipStream_t s) {
    const int sm = DIAG == 5 ? 0 : spread_mode(!AK && !BKM);
    if (sm == 2) return launch_pp1s<AK, BKM, SLAB, DIAG, 2>(a, lda, b, ldb, slab, c, ldc, beta, M, N, R, splits, s);
    if (sm == 1) return launch_pp1s<AK, BKM, SLAB, DIAG, 1>(a, lda, b, ldb, slab, c, ldc, beta, M, N, R, splits, s);
    launch_pp1s<AK, BKM, SLAB, DIAG, 0>(a, lda, b, ldb, slab, c, ldc, beta, M, N, R, splits, s);
}

// BPE_GPP_DIAG (a build define, ``python -m bpe_transformer.ops.build --variant diag -D BPE_GPP_DIAG=<n>``): the
// timing diagnostics of ktile / ktile_spread (numerically wrong) in an A/B copy of the library
#ifndef BPE_GPP_DIAG
#define BPE_GPP_DIAG 0
#endif
template <bool AK, bool BKM, bool SLAB>
static void launch_pp(const __bf16* a, long lda, const __bf16* b, long ldb, float* slab, __bf16* c, long ldc,
                      float beta, int M, int N, int R, int splits, hipStream_t s) {
    launch_pp1<AK, BKM, SLAB, BPE_GPP_DIAG>(a, lda, b, ldb, slab, c, ldc, beta, M, N, R, splits, s);
}

// Grouped weight gradients (gemm_pp_dwg_kernel, then dwg_reduce_kernel): np <= 4 problems C_p[M_p][N_p] =
// beta C_p + dY_p^T X_p over R tokens, every tile split `splits` ways; slab: splits * sum M_p N_p floats.
void launch_gemm_pp_dw_group(int np, const void* const* A, const long* lda, const void* const* B, const long* ldb,
                             int b_kmajor, void* const* C, const long* ldc, const int* M, const int* N, int R,
                             int splits, float beta, float* slab, int c_f32, hipStream_t s) {
    DwGroup gp{};
    DwOut o{};
    long off = 0, e4 = 0;
    int tiles = 0;
    for (int p = 0; p < np; ++p) {
        gp.A[p] = (const __bf16*)A[p];
        gp.B[p] = (const __bf16*)B[p];
        gp.lda[p] = lda[p];
        gp.ldb[p] = ldb[p];
        gp.slab_off[p] = o.slab_off[p] = off;
        gp.M[p] = M[p];
        gp.N[p] = o.N[p] = N[p];
        tiles += (M[p] / BT) * (N[p] / BT);
        gp.tile_end[p] = tiles;
        off += (long)splits * M[p] * N[p];
        o.C[p] = C[p];
        o.ldc[p] = ldc[p];
        e4 += (long)M[p] * N[p] / 4;
        o.end4[p] = e4;
    }
    gp.np = o.np = np;
    gp.ntiles = tiles;
    gp.splits = o.splits = splits;
    gp.R = R;
    gp.prio = prio_mode();
    o.beta = beta;
    if (b_kmajor) {
        static bool attr = false;
        auto* k = &gemm_pp_dwg_kernel<true>;
        if (!attr) lds_attr(k), attr = true;
        k<<<tiles * splits, NT, LDS_LAUNCH, s>>>(gp, slab);
    } else {
        static bool attr = false;
        auto* k = &gemm_pp_dwg_kernel<false>;
        if (!attr) lds_attr(k), attr = true;
        k<<<tiles * splits, NT, LDS_LAUNCH, s>>>(gp, slab);
    }
    const int g = (int)std::min<long>((e4 + 255) / 256, 2048);
    if (c_f32)
        dwg_reduce_kernel<float><<<g, 256, 0, s>>>(slab, o);
    else
        dwg_reduce_kernel<__bf16><<<g, 256, 0, s>>>(slab, o);
}

void launch_gemm_pp(int a_kmajor, int b_kmajor, const void* A, long lda, const void* B, long ldb, void* C, long ldc,
                    float beta, int M, int N, int R, int splits, float* slab, int c_f32, hipStream_t s) {
    const __bf16* a = (const __bf16*)A;
    const __bf16* b = (const __bf16*)B;
    __bf16* c = (__bf16*)C;
#define L(AK, BKM, SL) launch_pp<AK, BKM, SL>(a, lda, b, ldb, slab, c, ldc, beta, M, N, R, splits, s)
    if (slab != nullptr) {  // splits > 1, or an fp32 C: fp32 partials, then the ordered reduce
        if (a_kmajor) { if (b_kmajor) L(true, true, true); else L(true, false, true); }
        else { if (b_kmajor) L(false, true, true); else L(false, false, true); }
        splitk_reduce(slab, C, ldc, beta, M, N, splits, c_f32, s);
    } else {
        if (a_kmajor) { if (b_kmajor) L(true, true, false); else L(true, false, false); }
        else { if (b_kmajor) L(false, true, false); else L(false, false, false); }
    }
#undef L
}

// copy the last gemm_pp launch's stamps out (BPE_GPP_STAMPS builds; false otherwise)
// phase stamps of the last one-tile launch: n workgroups x 8 waves x PST_VALS (BPE_GPP_PHASE_STAMPS builds)
bool gpp_read_phase_stamps(long long* host, int n) {
#ifdef BPE_GPP_PHASE_STAMPS
    (void)hipDeviceSynchronize();
    return hipMemcpyFromSymbol(host, HIP_SYMBOL(bpe::gpp::g_gpp_phase), (size_t)n * 8 * PST_VALS * sizeof(long long),
                               0, hipMemcpyDeviceToHost) == hipSuccess;
#else
    (void)host;
    (void)n;
    return false;
#endif
}

bool gpp_read_stamps(long long* host, int n) {
#ifdef BPE_GPP_STAMPS
    (void)hipDeviceSynchronize();
    return hipMemcpyFromSymbol(host, HIP_SYMBOL(bpe::gpp::g_gpp_stamps), (size_t)n * 8 * sizeof(long long), 0,
                               hipMemcpyDeviceToHost) == hipSuccess;
#else
    (void)host;
    (void)n;
    return false;
#endif
}
