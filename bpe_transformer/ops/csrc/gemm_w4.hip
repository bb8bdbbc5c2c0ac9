// 4-wave bf16 MFMA GEMM for gfx950: 256 x 256 x 64 tiles, one wave per SIMD, each wave a 128 x 128 block.
//
//   C[M, N] = beta * C + sum_r A(i, r) B(r, j)        (fp32 accumulation in 256 accumulator registers per lane)
//
// Operand layouts as gemm_pp.hip: K-major (X [M][R], W [N][R]) or MN-major (dY [R][M], W [R][N]).
//
// Why a second main loop beside the 8-wave ping-pong (gemm_pp.hip).  The ping-pong kernel splits a SIMD between two
// waves of 128 accumulator registers that alternate MFMA and load sections between raw barriers: 8 barriers and 28
// ds_read_b128 per wave per K-tile, and its diagnostic builds measured the loop skeleton WITHOUT any MFMA at the same
// ~2.75 k cycles per K-tile as the real loop (2.05 k of MFMA issue): the sections and their hand-offs, not the matrix
// pipe, set its pace.  Here one wave owns a whole SIMD (512 registers: 256 accumulators as AGPRs, two sets of
// fragments), computes a 128 x 128 block (8 x 8 accumulators of mfma_f32_16x16x32_bf16) and issues its own LDS reads
// and LDS-DMA between its MFMAs:
//   * per K-tile and wave 128 MFMAs (2 048 matrix cycles) against 32 ds_read_b128 (16 KiB of A, 16 KiB of B: every
//     fragment feeds 8 MFMAs, vs 2.3 in the ping-pong sections) and 16 LDS-DMA pieces;
//   * ONE barrier per K-tile, placed between the two 32-deep k-steps: the fragments of k-step 1 are in registers
//     before it, so the MFMAs never wait for LDS across it; the fragments of the next K-tile's k-step 0 are read
//     during k-step 1 (from the other stage, whose DMA the barrier retired).
// This is the structure of the library's own 256 x 256 x 64 MI16x16 kernel (4 waves, Tensile metadata), written
// in HIP with the staging of gemm_pp (LDS-DMA, source-address swizzles, raw barriers, counted waits).
//
// Pipeline, K-tile kt in stage s = kt & 1 (two 64 KiB stages, A image 32 KiB + B image 32 KiB):
//   section (kt, 0): 64 MFMAs on fragment set X = (kt, k-step 0); reads set Y = (kt, k-step 1) from stage s
//   wait vmcnt(0) lgkmcnt(0), barrier            -- Y landed; every wave's reads of stage s done; the DMA of
//                                                   K-tile kt + 1 (stage s ^ 1) retired by every issuing wave
//   section (kt, 1): 64 MFMAs on Y; reads X = (kt + 1, k-step 0) from stage s ^ 1; DMA of K-tile kt + 2 into s
// So a DMA piece has one full section (>= 1 024 matrix cycles) to land, and a stage is refilled only after the
// barrier that follows its last read.  Raw s_barrier only (__syncthreads would drain the in-flight DMA).
//
// Persistent: one workgroup per CU walks tiles wid, wid + grid, ... (XCD-aware order).  The K-tile sequence simply
// continues across the seam: the last two sections of a tile DMA the next tile's K-tiles 0 and 1 and read its first
// fragments.  The epilogue stages the bf16 tile through a third, 32 KiB LDS region (4 passes of 64 rows x 512 B,
// whole-row stores), so the next tile's K-tile 1 DMA (issued before the stores) and the stores overlap the next
// tile's first section: its barrier waits with vmcnt(stores) -- the DMA is older than the stores.
#include "fa_common.h"
#include "kernels.h"

#include <cstdlib>

namespace bpe {
namespace gw4 {

constexpr int NT = 256, BT = 256, BK = 64;
constexpr int OPB = 32768;              // one operand image
constexpr int STAGE = 2 * OPB;          // 64 KiB: A image + B image
constexpr int EPI_OFF = 2 * STAGE;      // epilogue staging region
constexpr int EPI_BYTES = 32768;        // 64 rows x 512 B
constexpr int LDS_BYTES = EPI_OFF + EPI_BYTES;  // 160 KiB: one workgroup per CU

typedef __attribute__((address_space(3))) void lds_void;
typedef __attribute__((address_space(1))) void gbl_void;

__device__ __forceinline__ int fk(int r) { return (r >> 1) & 7; }

// MN-major sub-image layout (gemm_pp.hip sub_off): eight [64 k][32 col] sub-images of 4 KiB with 64-byte rows, the
// 32-byte halves of a row swapped on odd 8-row groups (conflict-free ds_read_b64_tr_b16)
__device__ __forceinline__ int sub_off(int r, int c) {
    return (c >> 5) * 4096 + r * 64 + ((((c >> 4) & 1) ^ ((r >> 3) & 1)) << 5) + ((c & 15) << 1);
}

// Source offset (elements, from the K-tile origin) of 16-byte image chunk e (0..2047): K-major [256][64] images
// (chunk c of row r at c ^ fk(r)) or the MN-major sub-image layout.  The DMA writes lane-linearly, so the swizzle
// lives on the source address.
template <bool KM>
__device__ __forceinline__ int src_off(int e, int ld) {
    if constexpr (KM) {
        const int row = e >> 3, lc = (e & 7) ^ fk(row);
        return row * ld + lc * 8;
    } else {
        const int s = e >> 8, q = (e >> 6) & 3, ln = e & 63;
        const int row = 16 * q + (ln >> 2);
        const int ql = (ln & 3) ^ (((row >> 3) & 1) << 1);
        return row * ld + 32 * s + 8 * ql;
    }
}

template <bool KM>
__device__ __forceinline__ const __bf16* tile_ptr(const __bf16* P, long ld, int t0, long k0) {
    return KM ? P + (long)t0 * ld + k0 : P + k0 * ld + t0;
}

// Per-lane LDS byte offsets of the fragment reads (a k-step's 8 blocks differ by immediates only).
// K-major [256][64] image: lane l reads row 16 tb + (l & 15), chunk (4 ks + (l >> 4)) ^ fk(l & 15): tb adds 2048.
// MN-major sub-image image: lane l reads k-rows r, r + 4 (r = 32 ks + 8 (l >> 4) + ((l & 15) >> 2)) at columns
// 16 tb + 4 (l & 3): sub-image tb >> 1 (+4096 each), 32-byte half (tb & 1) ^ ((r >> 3) & 1) -- one offset per parity.
template <bool KM>
struct FragOff {
    int o[2][2];  // [k-step][K-major: unused second / MN-major: tb parity]
};

template <bool KM>
__device__ __forceinline__ FragOff<KM> frag_offsets(int l) {
    FragOff<KM> f;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
        if constexpr (KM) {
            f.o[ks][0] = (l & 15) * 128 + (((4 * ks + (l >> 4)) ^ fk(l & 15)) << 4);
            f.o[ks][1] = f.o[ks][0];
        } else {
            const int r = 32 * ks + 8 * (l >> 4) + ((l & 15) >> 2);
#pragma unroll
            for (int par = 0; par < 2; ++par) f.o[ks][par] = r * 64 + ((par ^ ((r >> 3) & 1)) << 5) + 8 * (l & 3);
        }
    }
    return f;
}

// MFMA operand fragment of 16-row block tb (compile-time after unrolling) at per-lane offset base:
// lane l gets X[16 tb + (l & 15)][32 ks + 8 (l >> 4) + j]
template <bool KM>
__device__ __forceinline__ bf16x8 frag(const char* img, const FragOff<KM>& fo, int ks, int tb) {
    if constexpr (KM) {
        return fa::lds_row16(img, fo.o[ks][0] + tb * 2048);
    } else {
        const int o = fo.o[ks][tb & 1] + (tb >> 1) * 4096;
        return fa::lds_tr_pair(const_cast<char*>(img), o, o + 256);
    }
}

struct Set {
    bf16x8 a[8];  // A fragments of this wave's 8 row blocks
    bf16x8 b[8];  // B fragments of its 8 column blocks
};

// img_a / img_b: this wave's first block (row block 8 wm of A, column block 8 wn of B) inside the stage
template <bool AK, bool BKM>
__device__ __forceinline__ void read_set(Set& f, const char* __restrict__ img_a, const char* __restrict__ img_b,
                                         const FragOff<AK>& fa_, const FragOff<BKM>& fb_, int ks) {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        f.a[i] = frag<AK>(img_a, fa_, ks, i);
        f.b[i] = frag<BKM>(img_b, fb_, ks, i);
    }
}

__device__ __forceinline__ f32x4 mfma16(bf16x8 a, bf16x8 b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

// 64 MFMAs of one k-step; FIRST: the tile's first k-step starts from zero (inline-constant C, no zeroing pass)
template <bool FIRST>
__device__ __forceinline__ void mma_set(f32x4 (&acc)[8][8], const Set& f) {
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < 8; ++j)
            acc[i][j] = mfma16(f.b[j], f.a[i], FIRST ? f32x4{0.f, 0.f, 0.f, 0.f} : acc[i][j]);
}

// DMA of this wave's 8 pieces (1 KiB each) of one operand image through a buffer resource based at the K-tile's
// origin (guide T8: 32-bit per-lane offsets fixed for the kernel, no 64-bit address arithmetic per K-tile)
__device__ __forceinline__ void dma8(const __bf16* tile0, const unsigned (&voff)[8], char* img, int w) {
#if defined(__HIP_DEVICE_COMPILE__)
    const auto rsrc = __builtin_amdgcn_make_buffer_rsrc((void*)tile0, 0, 0xFFFFFFFF, 0x00020000);
#pragma unroll
    for (int j = 0; j < 8; ++j)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rsrc, (lds_void*)(img + (8 * w + j) * 1024), 16, voff[j], 0, 0, 0);
#endif
}

__device__ __forceinline__ void bar() {
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
}

// interleave: per group, NRD fragment reads and NDMA LDS-DMA pieces, then NMF MFMAs (the reads lead, so the last
// group's MFMAs cover the last reads' latency before the section's wait)
template <int NGRP, int NMF, int NRD, int NDMA>
__device__ __forceinline__ void interleave() {
#pragma unroll
    for (int i = 0; i < NGRP; ++i) {
        if constexpr (NRD > 0) __builtin_amdgcn_sched_group_barrier(0x100, NRD, 0);
        if constexpr (NDMA > 0) __builtin_amdgcn_sched_group_barrier(0x020, NDMA, 0);
        __builtin_amdgcn_sched_group_barrier(0x008, NMF, 0);
    }
}

// Section k-step 0 of a K-tile: MFMAs on X, reads of Y (k-step 1 of the same stage)
// DIAG (timing diagnostics of a variant build, numerically wrong): 1 no DMA in the loop, 2 no fragment reads in the
// loop, 3 no MFMAs, 4 no waits / barriers in the loop, 5 DMA issued but never waited for, 6 the section's 16 DMA
// pieces as one burst at its start (correct: diagnostic of the issue placement)
template <int DIAG>
__device__ __forceinline__ void keep_live(const Set& f) {
#pragma unroll
    for (int i = 0; i < 8; ++i) asm volatile("" ::"v"(f.a[i]), "v"(f.b[i]));
}

template <bool AK, bool BKM, bool FIRST, int DIAG = 0>
__device__ __forceinline__ void section0(f32x4 (&acc)[8][8], const Set& X, Set& Y, const char* __restrict__ cur,
                                         int wm, int wn, const FragOff<AK>& fa_, const FragOff<BKM>& fb_) {
    if (DIAG != 2) read_set<AK, BKM>(Y, cur + 16384 * wm, cur + OPB + 16384 * wn, fa_, fb_, 1);
    if (DIAG != 3) mma_set<FIRST>(acc, X);
    else keep_live<DIAG>(X);
    // 64 MFMAs in 8 groups; 16 fragments = 16 ds_read_b128 (K-major) or 32 ds_read_b64_tr_b16 (MN-major) reads
    interleave<8, 8, (AK ? 1 : 2) + (BKM ? 1 : 2), 0>();
}

// Section k-step 1: MFMAs on Y, reads of X (next K-tile's k-step 0) from nxt, DMA of the K-tile after next into dst
// (unconditional: past the last K-tile of the last tile the sources are clamped to valid rows and the reads / DMA
// land in a stage no later read uses, so the section stays one basic block for the interleave)
template <bool AK, bool BKM, int DIAG = 0>
__device__ __forceinline__ void section1(f32x4 (&acc)[8][8], const Set& Y, Set& X, const char* __restrict__ nxt,
                                         char* __restrict__ dst, const __bf16* an, const __bf16* bn,
                                         const unsigned (&oa)[8], const unsigned (&ob)[8], int w, int wm, int wn,
                                         const FragOff<AK>& fa_, const FragOff<BKM>& fb_) {
    if (DIAG != 2) read_set<AK, BKM>(X, nxt + 16384 * wm, nxt + OPB + 16384 * wn, fa_, fb_, 0);
    if (DIAG != 1) {
        dma8(an, oa, dst, w);
        dma8(bn, ob, dst + OPB, w);
    }
    if (DIAG != 3) mma_set<false>(acc, Y);
    else keep_live<DIAG>(Y);
    if constexpr (DIAG == 6) {
        __builtin_amdgcn_sched_group_barrier(0x020, 16, 0);
        interleave<8, 8, (AK ? 1 : 2) + (BKM ? 1 : 2), 0>();
    } else {
        interleave<8, 8, (AK ? 1 : 2) + (BKM ? 1 : 2), 2>();
    }
}

// bf16 epilogue, 4 passes through the 32 KiB region: pass p holds rows [32 p, +32) of each wave's 128-row block
// (tile rows 32 p + [0, 32) and 128 + 32 p + [0, 32)) as [64][512 B] (16-byte chunk c of row i at c ^ (i & 15)),
// then every thread stores 8 x 16 bytes of whole rows.  Returns nothing; the stores stay in flight.
__device__ __forceinline__ int pass_row(int p, int i) { return i < 32 ? 32 * p + i : 96 + 32 * p + i; }

template <int EPI, bool BETA>
__device__ __forceinline__ void epilogue(const f32x4 (&acc)[8][8], char* stg, int wm, int wn, int l, int tid, int i0,
                                         int j0, __bf16* C, long ldc, float beta) {
    // the lane's epilogue addresses are recomputed per tile: hoisted out of the persistent loop they stay live
    // through the main loop and spill (tens of VGPRs beside 128 fragment registers)
    asm volatile("" : "+v"(l), "+v"(tid));
#pragma unroll
    for (int p = 0; p < 4; ++p) {
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const int ib = 2 * p + h;
#pragma unroll
            for (int jb = 0; jb < 8; ++jb) {
                const int i = 32 * wm + 16 * h + (l & 15);
                const int j = 128 * wn + 16 * jb + 4 * (l >> 4);
                const f32x4 v = acc[ib][jb];
                const u16x4 q = u16x4{f2bf(v[0]), f2bf(v[1]), f2bf(v[2]), f2bf(v[3])};
                *reinterpret_cast<u16x4*>(stg + i * 512 + (((j >> 3) ^ (i & 15)) << 4) + ((j & 7) << 1)) = q;
            }
        }
        __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): this wave's staging writes
        bar();
        const int c = tid & 31;
#pragma unroll
        for (int q = 0; q < 8; ++q) {
            const int i = 8 * q + (tid >> 5);
            u16x8 v = *reinterpret_cast<const u16x8*>(stg + i * 512 + ((c ^ (i & 15)) << 4));
            __bf16* cp = C + (long)(i0 + pass_row(p, i)) * ldc + j0 + c * 8;
            if constexpr (BETA) {
                const u16x8 o = *reinterpret_cast<const u16x8*>(cp);
#pragma unroll
                for (int e = 0; e < 8; ++e) v[e] = f2bf(bf2f(v[e]) + beta * bf2f(o[e]));
            }
            *reinterpret_cast<u16x8*>(cp) = v;
        }
        __builtin_amdgcn_s_waitcnt(0xc07f);  // the image's reads retired before the next pass rewrites it
        bar();
    }
}

template <bool AK, bool BKM, int EPI, bool BETA, int DIAG = 0>
__global__ void __launch_bounds__(NT, 1)
gemm_w4_kernel(const __bf16* __restrict__ A, long lda, const __bf16* __restrict__ B, long ldb, __bf16* __restrict__ C,
               long ldc, float beta, int M, int N, int R) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int tid = threadIdx.x, l = tid & 63;
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wm = w >> 1, wn = w & 1;
    const int nwg = gridDim.x, orig = blockIdx.x;
    const int xcd = orig & 7, qq = nwg >> 3, rr = nwg & 7;
    const int wid = (xcd < rr ? xcd * (qq + 1) : rr * (qq + 1) + (xcd - rr) * qq) + (orig >> 3);
    const int tiles_n = N / BT;
    const int ntiles = (M / BT) * tiles_n;
    const int nk = R / BK;  // >= 2 (host check)

    unsigned oa[8], ob[8];  // byte offsets of this lane's source chunks from the K-tile origin
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        const int e = 64 * (8 * w + j) + l;
        oa[j] = 2u * (unsigned)src_off<AK>(e, (int)lda);
        ob[j] = 2u * (unsigned)src_off<BKM>(e, (int)ldb);
    }
    const FragOff<AK> foa = frag_offsets<AK>(l);
    const FragOff<BKM> fob = frag_offsets<BKM>(l);
    int t = wid;
    int i0 = (t / tiles_n) * BT, j0 = (t % tiles_n) * BT;
    // prologue: K-tiles 0 and 1 of the first tile; K-tile 0 retired (vmcnt leaves K-tile 1's 16 pieces in flight)
    dma8(tile_ptr<AK>(A, lda, i0, 0), oa, smem, w);
    dma8(tile_ptr<BKM>(B, ldb, j0, 0), ob, smem + OPB, w);
    dma8(tile_ptr<AK>(A, lda, i0, BK), oa, smem + STAGE, w);
    dma8(tile_ptr<BKM>(B, ldb, j0, BK), ob, smem + STAGE + OPB, w);
    asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
    bar();
    Set X, Y;
    f32x4 acc[8][8];
    bool stores_pending = false;
    int sb = 0;  // stage of the tile's K-tile 0 (the K-tile sequence runs on across tiles: flips per tile when nk is odd)
    for (;;) {
        const int tn = t + nwg;
        const bool more = tn < ntiles;
        const int i0n = more ? (tn / tiles_n) * BT : i0, j0n = more ? (tn % tiles_n) * BT : j0;
        // k-step 0 fragments of K-tile 0 (read here, not at the end of the previous tile: keeps them out of the
        // epilogue's live registers)
        {
            const char* st0 = smem + sb * STAGE;
            read_set<AK, BKM>(X, st0 + 16384 * wm, st0 + OPB + 16384 * wn, foa, fob, 0);
        }
        for (int kt = 0; kt < nk; ++kt) {
            char* cur = smem + ((kt + sb) & 1) * STAGE;
            char* nxt = smem + ((kt + 1 + sb) & 1) * STAGE;
            if (kt == 0) section0<AK, BKM, true, DIAG>(acc, X, Y, cur, wm, wn, foa, fob);
            else section0<AK, BKM, false, DIAG>(acc, X, Y, cur, wm, wn, foa, fob);
            // Y landed, stage cur fully read by this wave, K-tile kt + 1's DMA retired.  After an epilogue the
            // previous tile's 32 stores are the youngest VMEM operations of this wave (the DMA of K-tile 1 was
            // issued before them): leave them in flight.
            if (DIAG == 5) {
                asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                bar();
            } else if (DIAG != 4) {
                if (kt == 0 && stores_pending) asm volatile("s_waitcnt vmcnt(32) lgkmcnt(0)" ::: "memory");
                else asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
                bar();
            }
            // reads: K-tile kt + 1 (the last K-tile's reads are dead: the next tile re-reads its K-tile 0 after the
            // epilogue); DMA: K-tile kt + 2 (or the next tile's kt + 2 - nk; after the last tile, this tile's again --
            // a dummy into a stage nothing reads any more)
            const int q = kt + 2;
            const long kq = (long)(q < nk ? q : q - nk) * BK;
            const __bf16* an = tile_ptr<AK>(A, lda, q < nk ? i0 : i0n, kq);
            const __bf16* bn = tile_ptr<BKM>(B, ldb, q < nk ? j0 : j0n, kq);
            section1<AK, BKM, DIAG>(acc, Y, X, nxt, cur, an, bn, oa, ob, w, wm, wn, foa, fob);
        }
        epilogue<EPI, BETA>(acc, smem + EPI_OFF, wm, wn, l, tid, i0, j0, C, ldc, beta);
        if (!more) {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // no LDS-DMA may land after the workgroup ends
            break;
        }
        stores_pending = true;
        sb = (sb + nk) & 1;
        t = tn;
        i0 = i0n;
        j0 = j0n;
    }
}

// ---------------------------------------------------------------------------------------------------------
// Ring form: 32-deep K-steps in a ring of four 32 KiB stages (A image [256][32] + B image [256][32], or the MN-major
// [32 k][256] sub-image layout), the epilogue region unchanged.  The 2-stage form above waits for every DMA piece of
// the next K-tile at each barrier (vmcnt(0)): a piece has 1-2 sections of flight and the wave's bytes in flight
// drain to zero once per K-tile, so the loop runs at the L2 -> LDS round trip, not at the matrix rate (its variant
// without in-loop DMA is 1.4x faster).  Here section j (64 MFMAs on F_j) reads F_{j+1} from stage (j+1) % 4 and DMAs
// step j + 4 into stage j % 4 (whose fragments F_j are in registers: their reads retired before the barrier that
// opened the section); the barrier closing section j waits vmcnt(16): step j + 2's pieces, issued three sections
// earlier, and leaves steps j + 3, j + 4 (16 pieces) in flight.  One barrier per 64 MFMAs.
namespace ring {

constexpr int SBK = 32;                 // K per step
constexpr int OP = 16384;               // one operand image
constexpr int STG = 2 * OP;             // 32 KiB
constexpr int NST = 4;                  // stages
constexpr int EOFF = NST * STG;         // epilogue staging region (32 KiB)
constexpr int LDS = EOFF + EPI_BYTES;   // 160 KiB

// K-major [256][32] image: 64-byte rows, 16-byte chunk c of row r at c ^ ((r >> 2) & 2) (conflict-free for the
// 16x16x32 ds_read_b128 lane groups: every group covers the 16 slots of a bank row)
__device__ __forceinline__ int fr(int r) { return (r >> 2) & 2; }

// MN-major [32 k][256] image: eight [32 k][32 col] sub-images of 2 KiB (gemm_pp's sub-image layout, 32 rows)
__device__ __forceinline__ int rsub_off(int r, int c) {
    return (c >> 5) * 2048 + r * 64 + ((((c >> 4) & 1) ^ ((r >> 3) & 1)) << 5) + ((c & 15) << 1);
}

// source offset (elements from the step origin) of image chunk e (0..1023)
template <bool KM>
__device__ __forceinline__ int rsrc_off(int e, int ld) {
    if constexpr (KM) {
        const int row = e >> 2, lc = (e & 3) ^ fr(row);
        return row * ld + lc * 8;
    } else {
        const int s = e >> 7, q = (e >> 6) & 1, ln = e & 63;
        const int row = 16 * q + (ln >> 2);
        const int ql = (ln & 3) ^ (((row >> 3) & 1) << 1);
        return row * ld + 32 * s + 8 * ql;
    }
}

template <bool KM>
struct ROff {
    int o[2];  // K-major: o[0]; MN-major: per block parity
};

template <bool KM>
__device__ __forceinline__ ROff<KM> roffsets(int l) {
    ROff<KM> f;
    if constexpr (KM) {
        const int r = l & 15;
        f.o[0] = r * 64 + (((l >> 4) ^ fr(r)) << 4);
        f.o[1] = f.o[0];
    } else {
        const int r = 8 * (l >> 4) + ((l & 15) >> 2);
#pragma unroll
        for (int par = 0; par < 2; ++par) f.o[par] = r * 64 + ((par ^ ((r >> 3) & 1)) << 5) + 8 * (l & 3);
    }
    return f;
}

// fragment of 16-row block tb (compile-time): lane l gets X[16 tb + (l & 15)][8 (l >> 4) + j]
template <bool KM>
__device__ __forceinline__ bf16x8 rfrag(const char* img, const ROff<KM>& fo, int tb) {
    if constexpr (KM) {
        return fa::lds_row16(img, fo.o[0] + tb * 1024);
    } else {
        const int o = fo.o[tb & 1] + (tb >> 1) * 2048;
        return fa::lds_tr_pair(const_cast<char*>(img), o, o + 256);
    }
}

// this wave's blocks start 8 blocks in: K-major 8 * 1024 bytes, MN-major 4 sub-images = 8 KiB as well
template <bool AK, bool BKM>
__device__ __forceinline__ void rread(Set& f, const char* __restrict__ st, int wm, int wn, const ROff<AK>& fa_,
                                      const ROff<BKM>& fb_) {
    const char* ia = st + 8192 * wm;
    const char* ib = st + OP + 8192 * wn;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        f.a[i] = rfrag<AK>(ia, fa_, i);
        f.b[i] = rfrag<BKM>(ib, fb_, i);
    }
}

// this wave's 4 pieces of one operand image of a step
__device__ __forceinline__ void rdma4(const __bf16* step0, const unsigned (&voff)[4], char* img, int w) {
#if defined(__HIP_DEVICE_COMPILE__)
    const auto rsrc = __builtin_amdgcn_make_buffer_rsrc((void*)step0, 0, 0xFFFFFFFF, 0x00020000);
#pragma unroll
    for (int j = 0; j < 4; ++j)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rsrc, (lds_void*)(img + (4 * w + j) * 1024), 16, voff[j], 0, 0, 0);
#endif
}

template <bool KM>
__device__ __forceinline__ const __bf16* rstep_ptr(const __bf16* P, long ld, int t0, int step) {
    return KM ? P + (long)t0 * ld + (long)step * SBK : P + (long)step * SBK * ld + t0;
}

// the ring form's epilogue: epilogue() with the next tile's F_0 read (into X) before the last pass's closing wait,
// which is vmcnt(48): the next tile's step 1 retired, its steps 2, 3 (16 pieces) and this epilogue's 32 stores in
// flight.  That barrier then opens the next tile's section 0 (stage 0 of the tile refilled only after it).
template <int EPI, bool BETA, bool AK, bool BKM>
__device__ __forceinline__ void epilogue_r(const f32x4 (&acc)[8][8], char* stg, int wm, int wn, int l, int tid,
                                           int i0, int j0, __bf16* C, long ldc, float beta, Set& X,
                                           const char* __restrict__ st0, const ROff<AK>& fa_, const ROff<BKM>& fb_) {
    asm volatile("" : "+v"(l), "+v"(tid));  // recomputed per tile (see epilogue())
#pragma unroll
    for (int p = 0; p < 4; ++p) {
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const int ib = 2 * p + h;
#pragma unroll
            for (int jb = 0; jb < 8; ++jb) {
                const int i = 32 * wm + 16 * h + (l & 15);
                const int j = 128 * wn + 16 * jb + 4 * (l >> 4);
                const f32x4 v = acc[ib][jb];
                const u16x4 q = u16x4{f2bf(v[0]), f2bf(v[1]), f2bf(v[2]), f2bf(v[3])};
                *reinterpret_cast<u16x4*>(stg + i * 512 + (((j >> 3) ^ (i & 15)) << 4) + ((j & 7) << 1)) = q;
            }
        }
        __builtin_amdgcn_s_waitcnt(0xc07f);
        bar();
        const int c = tid & 31;
#pragma unroll
        for (int q = 0; q < 8; ++q) {
            const int i = 8 * q + (tid >> 5);
            u16x8 v = *reinterpret_cast<const u16x8*>(stg + i * 512 + ((c ^ (i & 15)) << 4));
            __bf16* cp = C + (long)(i0 + pass_row(p, i)) * ldc + j0 + c * 8;
            if constexpr (BETA) {
                const u16x8 o = *reinterpret_cast<const u16x8*>(cp);
#pragma unroll
                for (int e = 0; e < 8; ++e) v[e] = f2bf(bf2f(v[e]) + beta * bf2f(o[e]));
            }
            *reinterpret_cast<u16x8*>(cp) = v;
        }
        if (p == 3) {
            rread<AK, BKM>(X, st0, wm, wn, fa_, fb_);
            asm volatile("s_waitcnt vmcnt(48) lgkmcnt(0)" ::: "memory");
        } else {
            __builtin_amdgcn_s_waitcnt(0xc07f);
        }
        bar();
    }
}

// one section: 64 MFMAs on X; (RD) reads of the next step's fragments into Y from rd_st; 8 DMA pieces of step q
// into dst
template <bool AK, bool BKM, bool FIRST, bool RD>
__device__ __forceinline__ void rsection(f32x4 (&acc)[8][8], const Set& X, Set& Y, const char* __restrict__ rd_st,
                                         char* __restrict__ dst, const __bf16* an, const __bf16* bn,
                                         const unsigned (&oa)[4], const unsigned (&ob)[4], int w, int wm, int wn,
                                         const ROff<AK>& fa_, const ROff<BKM>& fb_) {
    if constexpr (RD) rread<AK, BKM>(Y, rd_st, wm, wn, fa_, fb_);
    rdma4(an, oa, dst, w);
    rdma4(bn, ob, dst + OP, w);
    mma_set<FIRST>(acc, X);
    // 8 groups: 2-4 fragment reads, 1 DMA piece, 8 MFMAs
    interleave<8, 8, RD ? (AK ? 1 : 2) + (BKM ? 1 : 2) : 0, 1>();
}

template <bool AK, bool BKM, int EPI, bool BETA>
__global__ void __launch_bounds__(NT, 1)
gemm_w4r_kernel(const __bf16* __restrict__ A, long lda, const __bf16* __restrict__ B, long ldb,
                __bf16* __restrict__ C, long ldc, float beta, int M, int N, int R) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int tid = threadIdx.x, l = tid & 63;
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wm = w >> 1, wn = w & 1;
    const int nwg = gridDim.x, orig = blockIdx.x;
    const int xcd = orig & 7, qq = nwg >> 3, rr = nwg & 7;
    const int wid = (xcd < rr ? xcd * (qq + 1) : rr * (qq + 1) + (xcd - rr) * qq) + (orig >> 3);
    const int tiles_n = N / BT;
    const int ntiles = (M / BT) * tiles_n;
    const int nk = R / SBK;  // >= 4 (host check: R >= 128)

    unsigned oa[4], ob[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const int e = 64 * (4 * w + j) + l;
        oa[j] = 2u * (unsigned)rsrc_off<AK>(e, (int)lda);
        ob[j] = 2u * (unsigned)rsrc_off<BKM>(e, (int)ldb);
    }
    const ROff<AK> foa = roffsets<AK>(l);
    const ROff<BKM> fob = roffsets<BKM>(l);
    int t = wid;
    int i0 = (t / tiles_n) * BT, j0 = (t % tiles_n) * BT;
    // prologue: steps 0-3 into stages 0-3; steps 0, 1 retired; F_0 read; its reads retired before the barrier that
    // lets section 0 refill stage 0
#pragma unroll
    for (int q = 0; q < NST; ++q) {
        rdma4(rstep_ptr<AK>(A, lda, i0, q), oa, smem + q * STG, w);
        rdma4(rstep_ptr<BKM>(B, ldb, j0, q), ob, smem + q * STG + OP, w);
    }
    asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
    bar();
    Set X, Y;
    rread<AK, BKM>(X, smem, wm, wn, foa, fob);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    bar();
    f32x4 acc[8][8];
    bool stores_pending = false;
    int g = 0;  // global step index of the tile's step 0 (stage = step % 4)
    for (;;) {
        const int tn = t + nwg;
        const bool more = tn < ntiles;
        const int i0n = more ? (tn / tiles_n) * BT : i0, j0n = more ? (tn % tiles_n) * BT : j0;
        // sections 0 .. nk - 2 in pairs (X / Y swap roles), then the last one (no fragment read)
        auto dma_src = [&](int q, const __bf16*& an, const __bf16*& bn) {
            an = rstep_ptr<AK>(A, lda, q < nk ? i0 : i0n, q < nk ? q : q - nk);
            bn = rstep_ptr<BKM>(B, ldb, q < nk ? j0 : j0n, q < nk ? q : q - nk);
        };
        auto stage = [&](int j) { return smem + ((g + j) & 3) * STG; };
        auto wait_bar = [&](int j) {  // closing barrier of section j
            if (stores_pending && j <= 1) asm volatile("s_waitcnt vmcnt(48) lgkmcnt(0)" ::: "memory");
            else asm volatile("s_waitcnt vmcnt(16) lgkmcnt(0)" ::: "memory");
            bar();
        };
        int j = 0;
        for (; j + 2 < nk; j += 2) {
            const __bf16 *an, *bn;
            dma_src(j + 4, an, bn);
            if (j == 0) rsection<AK, BKM, true, true>(acc, X, Y, stage(1), stage(0), an, bn, oa, ob, w, wm, wn, foa, fob);
            else rsection<AK, BKM, false, true>(acc, X, Y, stage(j + 1), stage(j), an, bn, oa, ob, w, wm, wn, foa, fob);
            wait_bar(j);
            dma_src(j + 5, an, bn);
            rsection<AK, BKM, false, true>(acc, Y, X, stage(j + 2), stage(j + 1), an, bn, oa, ob, w, wm, wn, foa, fob);
            wait_bar(j + 1);
        }
        {  // j = nk - 2 (nk is even): reads F_{nk-1}; j = nk - 1: no read
            const __bf16 *an, *bn;
            dma_src(j + 4, an, bn);
            rsection<AK, BKM, false, true>(acc, X, Y, stage(j + 1), stage(j), an, bn, oa, ob, w, wm, wn, foa, fob);
            wait_bar(j);
            dma_src(j + 5, an, bn);
            rsection<AK, BKM, false, false>(acc, Y, X, stage(j + 2), stage(j + 1), an, bn, oa, ob, w, wm, wn, foa,
                                            fob);
        }
        g += nk;
        // epilogue; the next tile's F_0 (stage g % 4) is read inside it, before its last barrier, which also retires
        // the next tile's step 1 (younger: steps 2, 3 and the 32 stores)
        epilogue_r<EPI, BETA, AK, BKM>(acc, smem + EOFF, wm, wn, l, tid, i0, j0, C, ldc, beta, X,
                                       smem + (g & 3) * STG, foa, fob);
        if (!more) {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // no LDS-DMA may land after the workgroup ends
            break;
        }
        stores_pending = true;
        t = tn;
        i0 = i0n;
        j0 = j0n;
    }
}

}  // namespace ring

// ---------------------------------------------------------------------------------------------------------
// Register-staged ring (the "g" form): the same 4-stage ring and fragment reads, but the step data travels
// global_load_dwordx4 -> VGPRs -> ds_write_b128 (the lane-linear image the DMA would write, so the same swizzled
// sources and reads).  Why: in the DMA forms the computing wave pays each LDS-DMA piece's issue (~60 cycles among
// bare MFMAs, guide; measured here: the 2-stage loop without its in-loop DMA runs 1.4-2x faster, with the DMA issued
// but never waited for no faster than the real loop).  Step s is loaded in section s - 3 (8 loads into register
// set S[s & 1]), written in section s - 2 into stage s % 4 (free: its previous step's fragments were read in section
// s - 5 .. s - 6), read as F_s in section s - 1 and multiplied in section s.  The loads' waits are the compiler's
// own counted vmcnt (plain loads).
namespace ring {

template <int EPI, bool BETA, bool AK, bool BKM>
__device__ __forceinline__ void epilogue_g(const f32x4 (&acc)[8][8], char* stg, int wm, int wn, int l, int tid,
                                           int i0, int j0, __bf16* C, long ldc, float beta, Set& X,
                                           const char* __restrict__ st0, const ROff<AK>& fa_, const ROff<BKM>& fb_) {
    asm volatile("" : "+v"(l), "+v"(tid));
#pragma unroll
    for (int p = 0; p < 4; ++p) {
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const int ib = 2 * p + h;
#pragma unroll
            for (int jb = 0; jb < 8; ++jb) {
                const int i = 32 * wm + 16 * h + (l & 15);
                const int j = 128 * wn + 16 * jb + 4 * (l >> 4);
                const f32x4 v = acc[ib][jb];
                const u16x4 q = u16x4{f2bf(v[0]), f2bf(v[1]), f2bf(v[2]), f2bf(v[3])};
                *reinterpret_cast<u16x4*>(stg + i * 512 + (((j >> 3) ^ (i & 15)) << 4) + ((j & 7) << 1)) = q;
            }
        }
        __builtin_amdgcn_s_waitcnt(0xc07f);
        bar();
        const int c = tid & 31;
#pragma unroll
        for (int q = 0; q < 8; ++q) {
            const int i = 8 * q + (tid >> 5);
            u16x8 v = *reinterpret_cast<const u16x8*>(stg + i * 512 + ((c ^ (i & 15)) << 4));
            __bf16* cp = C + (long)(i0 + pass_row(p, i)) * ldc + j0 + c * 8;
            if constexpr (BETA) {
                const u16x8 o = *reinterpret_cast<const u16x8*>(cp);
#pragma unroll
                for (int e = 0; e < 8; ++e) v[e] = f2bf(bf2f(v[e]) + beta * bf2f(o[e]));
            }
            *reinterpret_cast<u16x8*>(cp) = v;
        }
        if (p == 3) rread<AK, BKM>(X, st0, wm, wn, fa_, fb_);
        __builtin_amdgcn_s_waitcnt(0xc07f);
        bar();
    }
}

template <bool KM>
__device__ __forceinline__ void gload4(u16x8 (&r)[4], const __bf16* step0, const unsigned (&voff)[4]) {
#pragma unroll
    for (int j = 0; j < 4; ++j)
        r[j] = *reinterpret_cast<const u16x8*>(reinterpret_cast<const char*>(step0) + voff[j]);
}

__device__ __forceinline__ void gwrite4(const u16x8 (&r)[4], char* img, int w, int l) {
#pragma unroll
    for (int j = 0; j < 4; ++j) *reinterpret_cast<u16x8*>(img + (4 * w + j) * 1024 + 16 * l) = r[j];
}

struct Stg {
    u16x8 a[4], b[4];
};

// section: MFMAs on X; reads of F_{j+1} (RD) into Y; loads of step j + 3 into `ld`; writes of `wr` (step j + 2) into
// the stage wdst
template <bool AK, bool BKM, bool FIRST, bool RD>
__device__ __forceinline__ void gsection(f32x4 (&acc)[8][8], const Set& X, Set& Y, const char* __restrict__ rd_st,
                                         char* __restrict__ wdst, Stg& ld, const Stg& wr, const __bf16* an,
                                         const __bf16* bn, const unsigned (&oa)[4], const unsigned (&ob)[4], int w,
                                         int wm, int wn, int l, const ROff<AK>& fa_, const ROff<BKM>& fb_) {
    if constexpr (RD) rread<AK, BKM>(Y, rd_st, wm, wn, fa_, fb_);
    gload4<AK>(ld.a, an, oa);
    gload4<BKM>(ld.b, bn, ob);
    gwrite4(wr.a, wdst, w, l);
    gwrite4(wr.b, wdst + OP, w, l);
    mma_set<FIRST>(acc, X);
    constexpr int NRD = RD ? (AK ? 1 : 2) + (BKM ? 1 : 2) : 0;
    // first half: reads, the 8 loads, MFMAs; second half: reads, the 8 writes (their loads a section old), MFMAs
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        if constexpr (NRD > 0) __builtin_amdgcn_sched_group_barrier(0x100, NRD, 0);
        __builtin_amdgcn_sched_group_barrier(0x020, 2, 0);
        __builtin_amdgcn_sched_group_barrier(0x008, 8, 0);
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        if constexpr (NRD > 0) __builtin_amdgcn_sched_group_barrier(0x100, NRD, 0);
        __builtin_amdgcn_sched_group_barrier(0x200, 2, 0);
        __builtin_amdgcn_sched_group_barrier(0x008, 8, 0);
    }
}

template <bool AK, bool BKM, int EPI, bool BETA>
__global__ void __launch_bounds__(NT, 1)
gemm_w4g_kernel(const __bf16* __restrict__ A, long lda, const __bf16* __restrict__ B, long ldb,
                __bf16* __restrict__ C, long ldc, float beta, int M, int N, int R) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int tid = threadIdx.x, l = tid & 63;
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wm = w >> 1, wn = w & 1;
    const int nwg = gridDim.x, orig = blockIdx.x;
    const int xcd = orig & 7, qq = nwg >> 3, rr = nwg & 7;
    const int wid = (xcd < rr ? xcd * (qq + 1) : rr * (qq + 1) + (xcd - rr) * qq) + (orig >> 3);
    const int tiles_n = N / BT;
    const int ntiles = (M / BT) * tiles_n;
    const int nk = R / SBK;  // >= 4, even

    unsigned oa[4], ob[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const int e = 64 * (4 * w + j) + l;
        oa[j] = 2u * (unsigned)rsrc_off<AK>(e, (int)lda);
        ob[j] = 2u * (unsigned)rsrc_off<BKM>(e, (int)ldb);
    }
    const ROff<AK> foa = roffsets<AK>(l);
    const ROff<BKM> fob = roffsets<BKM>(l);
    int t = wid;
    int i0 = (t / tiles_n) * BT, j0 = (t % tiles_n) * BT;
    // prologue: steps 0, 1 into stages 0, 1 (DMA), step 2 into register set S1 (as if loaded in section -1)
    Stg S0, S1;
#pragma unroll
    for (int q = 0; q < 2; ++q) {
        rdma4(rstep_ptr<AK>(A, lda, i0, q), oa, smem + q * STG, w);
        rdma4(rstep_ptr<BKM>(B, ldb, j0, q), ob, smem + q * STG + OP, w);
    }
    gload4<AK>(S1.a, rstep_ptr<AK>(A, lda, i0, 2), oa);
    gload4<BKM>(S1.b, rstep_ptr<BKM>(B, ldb, j0, 2), ob);
    asm volatile("s_waitcnt vmcnt(8)" ::: "memory");  // the DMA of steps 0, 1 (older than the 8 register loads)
    bar();
    Set X, Y;
    rread<AK, BKM>(X, smem, wm, wn, foa, fob);
    __builtin_amdgcn_s_waitcnt(0xc07f);
    bar();
    f32x4 acc[8][8];
    int g = 0;
    for (;;) {
        const int tn = t + nwg;
        const bool more = tn < ntiles;
        const int i0n = more ? (tn / tiles_n) * BT : i0, j0n = more ? (tn % tiles_n) * BT : j0;
        auto src = [&](int q, const __bf16*& an, const __bf16*& bn) {
            an = rstep_ptr<AK>(A, lda, q < nk ? i0 : i0n, q < nk ? q : q - nk);
            bn = rstep_ptr<BKM>(B, ldb, q < nk ? j0 : j0n, q < nk ? q : q - nk);
        };
        auto stage = [&](int j) { return smem + ((g + j) & 3) * STG; };
        auto close = [&]() {  // the section's writes and reads retired, then the barrier
            __builtin_amdgcn_s_waitcnt(0xc07f);
            bar();
        };
        int j = 0;
        for (; j + 2 < nk; j += 2) {
            const __bf16 *an, *bn;
            src(j + 3, an, bn);
            if (j == 0)
                gsection<AK, BKM, true, true>(acc, X, Y, stage(1), stage(2), S0, S1, an, bn, oa, ob, w, wm, wn, l, foa,
                                              fob);
            else
                gsection<AK, BKM, false, true>(acc, X, Y, stage(j + 1), stage(j + 2), S0, S1, an, bn, oa, ob, w, wm,
                                               wn, l, foa, fob);
            close();
            src(j + 4, an, bn);
            gsection<AK, BKM, false, true>(acc, Y, X, stage(j + 2), stage(j + 3), S1, S0, an, bn, oa, ob, w, wm, wn,
                                           l, foa, fob);
            close();
        }
        {
            const __bf16 *an, *bn;
            src(j + 3, an, bn);
            gsection<AK, BKM, false, true>(acc, X, Y, stage(j + 1), stage(j + 2), S0, S1, an, bn, oa, ob, w, wm, wn,
                                           l, foa, fob);
            close();
            src(j + 4, an, bn);
            gsection<AK, BKM, false, false>(acc, Y, X, stage(j + 2), stage(j + 3), S1, S0, an, bn, oa, ob, w, wm, wn,
                                            l, foa, fob);
        }
        g += nk;
        // the next tile's F_0 (stage g % 4, written two sections ago) is read inside the epilogue before its last
        // barrier; S1 holds the next tile's step 2 (loaded in the last section)
        epilogue_g<EPI, BETA, AK, BKM>(acc, smem + EOFF, wm, wn, l, tid, i0, j0, C, ldc, beta, X,
                                       smem + (g & 3) * STG, foa, fob);
        if (!more) break;
        t = tn;
        i0 = i0n;
        j0 = j0n;
    }
}

}  // namespace ring
}  // namespace gw4
}  // namespace bpe

using namespace bpe::gw4;

static int num_cus_w4() {
    static int n[16] = {};
    int dev = 0;
    (void)hipGetDevice(&dev);
    int& c = n[dev & 15];
    if (c == 0 && hipDeviceGetAttribute(&c, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) c = 256;
    return c;
}

static int g_w4_grid_cap = 0;  // tests: at most this many workgroups (many tiles per workgroup on small shapes)
static int g_w4_ring = 1;      // 1: the ring form (32-deep steps, 4 stages), 0: the 2-stage 64-deep form
int gw4_ring_config(int mode) {
    const int prev = g_w4_ring;
    if (mode >= 0) g_w4_ring = mode;
    return prev;
}
int gw4_grid_config(int cap) {
    const int prev = g_w4_grid_cap;
    if (cap >= 0) g_w4_grid_cap = cap;
    return prev;
}

bool gemm_w4_shape_ok(int M, int N, int R) { return M % BT == 0 && N % BT == 0 && R % BK == 0 && R >= 2 * BK; }

#ifdef BPE_W4_DIAG  // variant build: BPE_W4_DIAG=<mode> in the environment picks a timing diagnostic (K-major A, B)
template <int DIAG>
static void launch_w4_diag(const __bf16* a, long lda, const __bf16* b, long ldb, __bf16* c, long ldc, int M, int N,
                           int R, int grid, hipStream_t s) {
    auto* k = &gemm_w4_kernel<true, true, 0, false, DIAG>;
    (void)hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, LDS_BYTES);
    k<<<grid, NT, LDS_BYTES, s>>>(a, lda, b, ldb, c, ldc, 0.f, M, N, R);
}
#endif

template <bool AK, bool BKM>
static void launch_w4(const __bf16* a, long lda, const __bf16* b, long ldb, __bf16* c, long ldc, float beta, int M,
                      int N, int R, hipStream_t s) {
#ifdef BPE_W4_DIAG
    if (AK && BKM && beta == 0.f) {
        const char* e = getenv("BPE_W4_DIAG");
        const int d = e ? atoi(e) : 0;
        const int ntiles = (M / BT) * (N / BT), cap = num_cus_w4();
        const int grid = ntiles < cap ? ntiles : cap;
        if (d == 1) return launch_w4_diag<1>(a, lda, b, ldb, c, ldc, M, N, R, grid, s);
        if (d == 2) return launch_w4_diag<2>(a, lda, b, ldb, c, ldc, M, N, R, grid, s);
        if (d == 3) return launch_w4_diag<3>(a, lda, b, ldb, c, ldc, M, N, R, grid, s);
        if (d == 4) return launch_w4_diag<4>(a, lda, b, ldb, c, ldc, M, N, R, grid, s);
        if (d == 5) return launch_w4_diag<5>(a, lda, b, ldb, c, ldc, M, N, R, grid, s);
        if (d == 6) return launch_w4_diag<6>(a, lda, b, ldb, c, ldc, M, N, R, grid, s);
    }
#endif
    static bool attr = false;
    if (!attr) {
        (void)hipFuncSetAttribute((const void*)&gemm_w4_kernel<AK, BKM, 0, true>,
                                  hipFuncAttributeMaxDynamicSharedMemorySize, LDS_BYTES);
        (void)hipFuncSetAttribute((const void*)&gemm_w4_kernel<AK, BKM, 0, false>,
                                  hipFuncAttributeMaxDynamicSharedMemorySize, LDS_BYTES);
        (void)hipFuncSetAttribute((const void*)&ring::gemm_w4r_kernel<AK, BKM, 0, true>,
                                  hipFuncAttributeMaxDynamicSharedMemorySize, ring::LDS);
        (void)hipFuncSetAttribute((const void*)&ring::gemm_w4r_kernel<AK, BKM, 0, false>,
                                  hipFuncAttributeMaxDynamicSharedMemorySize, ring::LDS);
        attr = true;
    }
    const int ntiles = (M / BT) * (N / BT);
    const int cap = g_w4_grid_cap > 0 ? g_w4_grid_cap : num_cus_w4();
    const int grid = ntiles < cap ? ntiles : cap;
    if (g_w4_ring == 2) {
        static bool gattr = false;
        if (!gattr) {
            (void)hipFuncSetAttribute((const void*)&ring::gemm_w4g_kernel<AK, BKM, 0, true>,
                                      hipFuncAttributeMaxDynamicSharedMemorySize, ring::LDS);
            (void)hipFuncSetAttribute((const void*)&ring::gemm_w4g_kernel<AK, BKM, 0, false>,
                                      hipFuncAttributeMaxDynamicSharedMemorySize, ring::LDS);
            gattr = true;
        }
        auto* k = beta != 0.f ? &ring::gemm_w4g_kernel<AK, BKM, 0, true> : &ring::gemm_w4g_kernel<AK, BKM, 0, false>;
        k<<<grid, NT, ring::LDS, s>>>(a, lda, b, ldb, c, ldc, beta, M, N, R);
        return;
    }
    if (g_w4_ring) {
        auto* k = beta != 0.f ? &ring::gemm_w4r_kernel<AK, BKM, 0, true> : &ring::gemm_w4r_kernel<AK, BKM, 0, false>;
        k<<<grid, NT, ring::LDS, s>>>(a, lda, b, ldb, c, ldc, beta, M, N, R);
        return;
    }
    auto* k = beta != 0.f ? &gemm_w4_kernel<AK, BKM, 0, true> : &gemm_w4_kernel<AK, BKM, 0, false>;
    k<<<grid, NT, LDS_BYTES, s>>>(a, lda, b, ldb, c, ldc, beta, M, N, R);
}

void launch_gemm_w4(int a_kmajor, int b_kmajor, const void* A, long lda, const void* B, long ldb, void* C, long ldc,
                    float beta, int M, int N, int R, hipStream_t s) {
    const __bf16* a = (const __bf16*)A;
    const __bf16* b = (const __bf16*)B;
    __bf16* c = (__bf16*)C;
    if (a_kmajor) {
        if (b_kmajor) launch_w4<true, true>(a, lda, b, ldb, c, ldc, beta, M, N, R, s);
        else launch_w4<true, false>(a, lda, b, ldb, c, ldc, beta, M, N, R, s);
    } else {
        if (b_kmajor) launch_w4<false, true>(a, lda, b, ldb, c, ldc, beta, M, N, R, s);
        else launch_w4<false, false>(a, lda, b, ldb, c, ldc, beta, M, N, R, s);
    }
}
