// bf16 MFMA GEMM with split-K for gfx950, used for the weight-gradient products.
// build-flags: -fno-slp-vectorize   (no packed f32 VALU beside the MFMAs: ops/build.py file_flags)
//
//   C[Mo, No] = beta * C + sum_r A(i, r) * B(r, j)         (fp32 accumulation)
//
// Operands are row-major in memory; each may be "K-major" (the reduction index
// is the contiguous one) or "MN-major" (the output index is contiguous):
//   forward  Y  = X  . W^T : A = X  [i][r] K-major,  B = W [j][r] K-major
//   dX           = dY . W   : A = dY [i][r] K-major,  B = W [r][j] MN-major
//   dW           = dY^T . X : A = dY [r][i] MN-major, B = X [r][j] MN-major
// The weight-gradient case (reduction over all B*S tokens, small Mo x No) is
// the one hipBLASLt handles poorly (few output tiles, no split-K: 170-680 TF
// measured); here the token range is split across workgroups so even a
// 768 x 768 gradient fills the chip, and partial sums go to an fp32 slab that
// a small kernel reduces in a fixed order into C (deterministic; beta = 1
// accumulates straight into the flat bf16 gradient buffer).
//
// Tile: 128 x 128 x 64, 4 waves as 2 x 2, each wave 64 x 64 = 2 x 2 MFMA
// 32x32x16 tiles.  Operands are staged global -> registers -> LDS (double
// buffered, one barrier per K step, loads of step t+1 issued before the MFMAs
// of step t).  K-major tiles ([128][64], 128-byte rows) are read as MFMA
// fragments with ds_read_b128; MN-major tiles ([64][128], 256-byte rows) with
// ds_read_b64_tr_b16 (hardware transpose, guide T10) -- no transposition pass
// in global memory.  Both LDS images use the XOR swizzles of fa_common.h that
// make their read kind conflict-free.
#include "fa_common.h"
#include "kernels.h"

#include <algorithm>
#include <cstdlib>

namespace bpe {
namespace gemm {

using fa::acc_row;
using fa::lds_row16;
using fa::lds_tr_pair;
using fa::mfma;
using fa::swz;
using fa::tr_off;

constexpr int BM = 128, BN = 128, BK = 64;
constexpr int TILE_BYTES = 128 * 64 * 2;  // 16 KiB per operand tile

// Stage one operand tile into registers: 1024 16-byte chunks, 4 per thread.
// K-major: tile [128 rows (i or j)][64 r]  (8 chunks per row)
// MN-major: tile [64 r][128 cols]          (16 chunks per row)
template <bool KMAJ>
__device__ __forceinline__ void load_tile(const __bf16* __restrict__ base, long ld, int i0, int r0, u16x8* reg) {
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const int e = threadIdx.x + 256 * q;
        if constexpr (KMAJ) {
            const int row = e >> 3, c = e & 7;
            reg[q] = *reinterpret_cast<const u16x8*>(base + (long)(i0 + row) * ld + r0 + c * 8);
        } else {
            const int row = e >> 4, c = e & 15;
            reg[q] = *reinterpret_cast<const u16x8*>(base + (long)(r0 + row) * ld + i0 + c * 8);
        }
    }
}

template <bool KMAJ>
__device__ __forceinline__ void store_tile(char* lds, const u16x8* reg) {
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const int e = threadIdx.x + 256 * q;
        if constexpr (KMAJ) {
            *reinterpret_cast<u16x8*>(lds + swz<128>(e >> 3, e & 7)) = reg[q];
        } else {
            *reinterpret_cast<u16x8*>(lds + swz<256>(e >> 4, e & 15)) = reg[q];
        }
    }
}

// MFMA operand fragment (32 output rows/cols starting at t0, k-step ks of the 64-deep tile).
template <bool KMAJ>
__device__ __forceinline__ bf16x8 frag(char* lds, int t0, int ks, int l) {
    const int hh = l >> 5;
    if constexpr (KMAJ) {
        return lds_row16(lds, swz<128>(t0 + (l & 31), 2 * ks + hh));
    } else {
        const int r = 16 * ks + 8 * hh + ((l & 15) >> 2);
        const int c = t0 + 16 * ((l >> 4) & 1) + 4 * (l & 3);
        return lds_tr_pair(lds, tr_off<256>(r, c), tr_off<256>(r + 4, c));
    }
}

template <bool AK, bool BK_>
__global__ void __launch_bounds__(256, 2)
gemm_kernel(const __bf16* __restrict__ A, long lda, const __bf16* __restrict__ B, long ldb, float* __restrict__ slab,
            __bf16* __restrict__ C, long ldc, float beta, int Mo, int No, int R, int splits) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int tid = threadIdx.x, w = tid >> 6, l = tid & 63, l31 = l & 31, hh = l >> 5;
    const int tiles_n = No / BN;
    const int ntiles = (Mo / BM) * tiles_n;
    const int tile = blockIdx.x % ntiles, split = blockIdx.x / ntiles;
    const int i0 = (tile / tiles_n) * BM, j0 = (tile % tiles_n) * BN;
    // split s owns k-steps [s*nkt/splits, (s+1)*nkt/splits): any split count, ranges differ by <= 1 step
    const int nkt = R / BK;
    const int kb = (int)((long)split * nkt / splits), nk = (int)((long)(split + 1) * nkt / splits) - kb;
    const int rbeg = kb * BK;
    char* As = smem;                    // [2][16 KiB]
    char* Bs = smem + 2 * TILE_BYTES;   // [2][16 KiB]
    const int wr = (w >> 1) * 64, wc = (w & 1) * 64;

    f32x16 acc[2][2];
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int b = 0; b < 2; ++b)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[a][b][r] = 0.f;

    u16x8 ra[4], rb[4];
    load_tile<AK>(A, lda, i0, rbeg, ra);
    load_tile<BK_>(B, ldb, j0, rbeg, rb);
    store_tile<AK>(As, ra);
    store_tile<BK_>(Bs, rb);
    __syncthreads();
    for (int kt = 0; kt < nk; ++kt) {
        const int cur = kt & 1;
        if (kt + 1 < nk) {
            load_tile<AK>(A, lda, i0, rbeg + (kt + 1) * BK, ra);
            load_tile<BK_>(B, ldb, j0, rbeg + (kt + 1) * BK, rb);
        }
        char* Ac = As + cur * TILE_BYTES;
        char* Bc = Bs + cur * TILE_BYTES;
#pragma unroll
        for (int ks = 0; ks < BK / 16; ++ks) {
            bf16x8 fa0 = frag<AK>(Ac, wr, ks, l), fa1 = frag<AK>(Ac, wr + 32, ks, l);
            bf16x8 fb0 = frag<BK_>(Bc, wc, ks, l), fb1 = frag<BK_>(Bc, wc + 32, ks, l);
            acc[0][0] = mfma(fa0, fb0, acc[0][0]);
            acc[0][1] = mfma(fa0, fb1, acc[0][1]);
            acc[1][0] = mfma(fa1, fb0, acc[1][0]);
            acc[1][1] = mfma(fa1, fb1, acc[1][1]);
        }
        if (kt + 1 < nk) {
            store_tile<AK>(As + (cur ^ 1) * TILE_BYTES, ra);
            store_tile<BK_>(Bs + (cur ^ 1) * TILE_BYTES, rb);
        }
        __syncthreads();
    }
    // epilogue.  MFMA(A-frag, B-frag): column = lane -> output column j, registers -> rows i.
    if (slab == nullptr) {  // one split straight into C; else fp32 partials (splits > 1, or an fp32 C)
#pragma unroll
        for (int a = 0; a < 2; ++a)
#pragma unroll
            for (int b = 0; b < 2; ++b)
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    const long i = i0 + wr + a * 32 + acc_row(r, hh);
                    const long j = j0 + wc + b * 32 + l31;
                    float v = acc[a][b][r];
                    if (beta != 0.f) v += beta * bf2f(*reinterpret_cast<const u16*>(C + i * ldc + j));
                    *reinterpret_cast<u16*>(C + i * ldc + j) = f2bf(v);
                }
    } else {
        float* sp = slab + (long)split * Mo * No;
#pragma unroll
        for (int a = 0; a < 2; ++a)
#pragma unroll
            for (int b = 0; b < 2; ++b)
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    const long i = i0 + wr + a * 32 + acc_row(r, hh);
                    const long j = j0 + wc + b * 32 + l31;
                    sp[i * No + j] = acc[a][b][r];
                }
    }
}

// C = beta*C + sum_s slab[s]  (fixed order -> deterministic); 4 outputs per thread.  CT = __bf16 or float (fp32
// gradient buffers: the sum is added to C without a bf16 rounding)
template <typename CT>
__global__ void __launch_bounds__(256) splitk_reduce_kernel(const float* __restrict__ slab, CT* __restrict__ C,
                                                            long ldc, float beta, int Mo, int No, int splits) {
    const long total4 = (long)Mo * No / 4;
    for (long t = blockIdx.x * 256L + threadIdx.x; t < total4; t += (long)gridDim.x * 256) {
        const long e = t * 4;
        const long i = e / No, j = e % No;
        f32x4 s = *reinterpret_cast<const f32x4*>(slab + e);
        for (int k = 1; k < splits; ++k) {
            const f32x4 v = *reinterpret_cast<const f32x4*>(slab + (long)k * Mo * No + e);
            s += v;
        }
        if constexpr (sizeof(CT) == 4) {
            f32x4* cp = reinterpret_cast<f32x4*>(C + i * ldc + j);
            if (beta != 0.f) s += beta * *cp;
            *cp = s;
        } else {
            u16x4* cp = reinterpret_cast<u16x4*>(C + i * ldc + j);
            if (beta != 0.f) {
                const u16x4 c = *cp;
                s[0] += beta * bf2f(c[0]); s[1] += beta * bf2f(c[1]);
                s[2] += beta * bf2f(c[2]); s[3] += beta * bf2f(c[3]);
            }
            *cp = u16x4{f2bf(s[0]), f2bf(s[1]), f2bf(s[2]), f2bf(s[3])};
        }
    }
}



// ---------------------------------------------------------------------------
// Weight-gradient kernel: dW[Mo, No] (+)= A^T B with A [R, Mo], B [R, No] both
// token-major (MN-major), R = tokens.  256 x 256 output tile, 8 waves (2 x 4,
// each 128 x 64 = 4 x 2 MFMA 32x32x16), one workgroup per CU.
//
// Operands go global -> LDS by LDS-DMA (global_load_lds_dwordx4): the LDS
// image is lane-linear, so the XOR swizzle is applied to the SOURCE address
// and the same involution on the fragment read (guide §5.4 rule 21).  Tiles
// are [32 tokens][256 cols] (16 KiB per operand), 4 stages (128 KiB) with TWO
// stages in flight while the MFMAs consume a third: one LDS-DMA takes ~1 us
// to land, longer than one 64-deep step of MFMA work, so a single stage of
// prefetch (measured: 660-985 TF) leaves the matrix cores waiting on every
// barrier.  The wait is a counted `s_waitcnt vmcnt(8)` (the two newer stages
// stay in flight) before a raw s_barrier -- __syncthreads() would drain every
// DMA (guide §5 "Pipelining across barriers").
namespace g256 {

constexpr int BM = 256, BN = 256, BK = 32, NT = 512, NSTAGE = 4;
constexpr int TILE_BYTES = BK * 256 * 2;  // 16 KiB per operand per stage
constexpr int STAGE_BYTES = 2 * TILE_BYTES;
constexpr int LDS_BYTES = NSTAGE * STAGE_BYTES;  // 128 KiB

// 512-byte rows: chunk c of row r stored at c ^ sigma(r); the 4 rows r0..r0+3 read by one
// ds_read_b64_tr_b16 half-wave (64 contiguous bytes each) land in the 4 distinct 64-byte quarters of the
// 256-byte bank row (conflict-free).
__device__ __forceinline__ int sig512(int r) { return ((r & 3) << 2) | ((r >> 2) & 3); }

typedef __attribute__((address_space(3))) void lds_void;
typedef __attribute__((address_space(1))) void gbl_void;

// Per-thread source offsets (elements, relative to the tile's first token row) of the 2 chunks it DMAs per tile.
__device__ __forceinline__ void dma_offsets(long ld, int c0, int w, int l, long (&off)[2]) {
#pragma unroll
    for (int q = 0; q < 2; ++q) {
        const int e = q * NT + w * 64 + l;
        const int row = e >> 5, lc = (e & 31) ^ sig512(row);
        off[q] = (long)row * ld + c0 + lc * 8;
    }
}

// DMA one [32 r][256 cols] operand tile (1024 16-byte chunks, 2 per thread) into a lane-linear LDS image;
// `tile0` = base + r0 * ld (wave-uniform).
__device__ __forceinline__ void dma_tile(const __bf16* tile0, const long (&off)[2], char* lds, int w) {
#pragma unroll
    for (int q = 0; q < 2; ++q)
        __builtin_amdgcn_global_load_lds((gbl_void*)(tile0 + off[q]), (lds_void*)(lds + (q * NT + w * 64) * 16), 16,
                                         0, 0);
}

// MFMA operands by two transposed reads (ds_read_b64_tr_b16; lane groups of 16 read 4 k-rows x 16 columns and
// receive one column each).  32x32x16: lane l holds X[k = 8(l>>5) + j][t0 + (l&31)] of k-step ks (16 deep);
// 16x16x32: lane l holds X[k = 8(l>>4) + j][t0 + (l&15)] (32 deep).
__device__ __forceinline__ int off512(int r, int c) { return r * 512 + (((c >> 3) ^ sig512(r)) << 4) + ((c & 7) << 1); }

__device__ __forceinline__ bf16x8 frag32(char* lds, int t0, int ks, int l) {
    const int r = 16 * ks + 8 * (l >> 5) + ((l & 15) >> 2);
    const int c = t0 + 16 * ((l >> 4) & 1) + 4 * (l & 3);
    return lds_tr_pair(lds, off512(r, c), off512(r + 4, c));
}

__device__ __forceinline__ bf16x8 frag16(char* lds, int t0, int l) {
    const int r = 8 * (l >> 4) + ((l & 15) >> 2);
    const int c = t0 + 4 * (l & 3);
    return lds_tr_pair(lds, off512(r, c), off512(r + 4, c));
}

__device__ __forceinline__ f32x4 mfma16(bf16x8 a, bf16x8 b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

// Accumulators of one wave's 128 x 64 output block.
template <int MF>
struct Acc;
template <>
struct Acc<32> {
    f32x16 v[4][2];
};
template <>
struct Acc<16> {
    f32x4 v[8][4];
};

// One K-step: DMA a future stage, then fragments + MFMAs on the current one.  The two stages are __restrict__
// parameters so that, once inlined, the LDS reads carry alias-scope metadata proving they do not touch the DMA
// destination; without it the compiler's wait-count pass drains the DMA (vmcnt(0)) before the first fragment read.
// PRIO: all fragments first, then the MFMA cluster between s_setprio(1)/(0) (keeps hipcc from moving MFMAs
// across the barriers; guide T5).
// DSPLIT (MF = 32, no PRIO): the 4 LDS-DMA instructions per wave and step spread over the step instead of one
// burst at its start -- 1: the A tile's pair before the first 16-deep k-step, the B tile's between the two;
// 2: one instruction after every quarter of the MFMAs.
__device__ __forceinline__ void dma_one(const __bf16* tile0, long off, char* lds, int q, int w) {
    __builtin_amdgcn_global_load_lds((gbl_void*)(tile0 + off), (lds_void*)(lds + (q * NT + w * 64) * 16), 16, 0, 0);
}

template <int MF, bool PRIO, int DSPLIT = 0>
__device__ __forceinline__ void kstep(char* __restrict__ cur, char* __restrict__ nxt, const __bf16* an,
                                      const long (&oa)[2], const __bf16* bn, const long (&ob)[2], int wr, int wc,
                                      int w, int l, Acc<MF>& acc) {
    char* Bs = cur + TILE_BYTES;
    if constexpr (DSPLIT == 2 && MF == 32 && !PRIO) {
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) {
            bf16x8 fb0 = frag32(Bs, wc, ks, l), fb1 = frag32(Bs, wc + 32, ks, l);
#pragma unroll
            for (int a = 0; a < 4; ++a) {
                if ((a & 1) == 0) {  // quarters: A chunk 0, A chunk 1, B chunk 0, B chunk 1
                    const int qi = 2 * ks + (a >> 1);
                    __builtin_amdgcn_sched_barrier(0);
                    if (qi < 2)
                        dma_one(an, oa[qi], nxt, qi, w);
                    else
                        dma_one(bn, ob[qi - 2], nxt + TILE_BYTES, qi - 2, w);
                    __builtin_amdgcn_sched_barrier(0);
                }
                bf16x8 fa = frag32(cur, wr + 32 * a, ks, l);
                acc.v[a][0] = mfma(fa, fb0, acc.v[a][0]);
                acc.v[a][1] = mfma(fa, fb1, acc.v[a][1]);
            }
        }
        return;
    }
    if constexpr (DSPLIT == 1 && MF == 32 && !PRIO) {
        dma_tile(an, oa, nxt, w);
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) {
            bf16x8 fb0 = frag32(Bs, wc, ks, l), fb1 = frag32(Bs, wc + 32, ks, l);
#pragma unroll
            for (int a = 0; a < 4; ++a) {
                bf16x8 fa = frag32(cur, wr + 32 * a, ks, l);
                acc.v[a][0] = mfma(fa, fb0, acc.v[a][0]);
                acc.v[a][1] = mfma(fa, fb1, acc.v[a][1]);
            }
            if (ks == 0) {
                __builtin_amdgcn_sched_barrier(0);
                dma_tile(bn, ob, nxt + TILE_BYTES, w);
                __builtin_amdgcn_sched_barrier(0);
            }
        }
        return;
    }
    dma_tile(an, oa, nxt, w);
    dma_tile(bn, ob, nxt + TILE_BYTES, w);
    __builtin_amdgcn_sched_barrier(0);  // issue the DMA first: it needs all the MFMA time to land
    if constexpr (MF == 32) {
        if constexpr (PRIO) {
            bf16x8 fa[2][4], fb[2][2];
#pragma unroll
            for (int ks = 0; ks < 2; ++ks) {
                fb[ks][0] = frag32(Bs, wc, ks, l);
                fb[ks][1] = frag32(Bs, wc + 32, ks, l);
#pragma unroll
                for (int a = 0; a < 4; ++a) fa[ks][a] = frag32(cur, wr + 32 * a, ks, l);
            }
            __builtin_amdgcn_s_setprio(1);
#pragma unroll
            for (int ks = 0; ks < 2; ++ks)
#pragma unroll
                for (int a = 0; a < 4; ++a) {
                    acc.v[a][0] = mfma(fa[ks][a], fb[ks][0], acc.v[a][0]);
                    acc.v[a][1] = mfma(fa[ks][a], fb[ks][1], acc.v[a][1]);
                }
            __builtin_amdgcn_s_setprio(0);
        } else {
#pragma unroll
            for (int ks = 0; ks < 2; ++ks) {
                bf16x8 fb0 = frag32(Bs, wc, ks, l), fb1 = frag32(Bs, wc + 32, ks, l);
#pragma unroll
                for (int a = 0; a < 4; ++a) {
                    bf16x8 fa = frag32(cur, wr + 32 * a, ks, l);
                    acc.v[a][0] = mfma(fa, fb0, acc.v[a][0]);
                    acc.v[a][1] = mfma(fa, fb1, acc.v[a][1]);
                }
            }
        }
    } else {
        bf16x8 fb[4];
#pragma unroll
        for (int b = 0; b < 4; ++b) fb[b] = frag16(Bs, wc + 16 * b, l);
        if constexpr (PRIO) {
            bf16x8 fa[8];
#pragma unroll
            for (int a = 0; a < 8; ++a) fa[a] = frag16(cur, wr + 16 * a, l);
            __builtin_amdgcn_s_setprio(1);
#pragma unroll
            for (int a = 0; a < 8; ++a)
#pragma unroll
                for (int b = 0; b < 4; ++b) acc.v[a][b] = mfma16(fa[a], fb[b], acc.v[a][b]);
            __builtin_amdgcn_s_setprio(0);
        } else {
#pragma unroll
            for (int a = 0; a < 8; ++a) {
                bf16x8 fa = frag16(cur, wr + 16 * a, l);
#pragma unroll
                for (int b = 0; b < 4; ++b) acc.v[a][b] = mfma16(fa, fb[b], acc.v[a][b]);
            }
        }
    }
}

// Epilogue element visitor: f(i_local, j_local, value) for every accumulator element of the wave.
template <typename F>
__device__ __forceinline__ void for_each_acc(const Acc<32>& acc, int l, F&& f) {
#pragma unroll
    for (int a = 0; a < 4; ++a)
#pragma unroll
        for (int b = 0; b < 2; ++b)
#pragma unroll
            for (int r = 0; r < 16; ++r) f(a * 32 + acc_row(r, l >> 5), b * 32 + (l & 31), acc.v[a][b][r]);
}
template <typename F>
__device__ __forceinline__ void for_each_acc(const Acc<16>& acc, int l, F&& f) {
#pragma unroll
    for (int a = 0; a < 8; ++a)
#pragma unroll
        for (int b = 0; b < 4; ++b)
#pragma unroll
            for (int r = 0; r < 4; ++r) f(a * 16 + 4 * (l >> 4) + r, b * 16 + (l & 15), acc.v[a][b][r]);
}

// NS = LDS stages (4 = 128 KiB, NS - 2 = 2 in flight while one is consumed; 5 = 160 KiB, the whole LDS, 3 in
// flight; measured no faster)
template <int MF, bool PRIO, int DSPLIT = 0, int NS = NSTAGE>
__global__ void __launch_bounds__(NT, 1)
gemm256_tn_kernel(const __bf16* __restrict__ A, long lda, const __bf16* __restrict__ B, long ldb,
                  float* __restrict__ slab, __bf16* __restrict__ C, long ldc, float beta, int Mo, int No, int R,
                  int splits, int prio) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int tid = threadIdx.x, w = __builtin_amdgcn_readfirstlane(tid >> 6), l = tid & 63;
    if (prio && w >= 4) __builtin_amdgcn_s_setprio(1);  // static form of guide T5: the younger wave half
    // XCD-aware bijective remap: consecutive work ids (same split, neighbouring tiles sharing token rows)
    // run on one XCD and its L2 (guide §5 "XCD swizzle must be bijective").
    const int nwg = gridDim.x, orig = blockIdx.x;
    const int xcd = orig & 7, qq = nwg >> 3, rr = nwg & 7;
    const int wid = (xcd < rr ? xcd * (qq + 1) : rr * (qq + 1) + (xcd - rr) * qq) + (orig >> 3);
    const int tiles_n = No / BN;
    const int ntiles = (Mo / BM) * tiles_n;
    const int split = wid / ntiles, tile = wid % ntiles;
    const int i0 = (tile / tiles_n) * BM, j0 = (tile % tiles_n) * BN;
    // split s owns k-steps [s*nkt/splits, (s+1)*nkt/splits) -- any split count (the cost model picks counts
    // that fill whole waves of CUs, e.g. 28 splits x 9 tiles); nk >= NSTAGE - 1 (host-checked)
    const int nkt = R / BK;
    const int kb = (int)((long)split * nkt / splits);
    const int nk = (int)((long)(split + 1) * nkt / splits) - kb;
    const int rbeg = kb * BK;
    const int rlast = rbeg + (nk - 1) * BK;
    const int wr = (w >> 2) * 128, wc = (w & 3) * 64;

    Acc<MF> acc;
    {
        float* z = reinterpret_cast<float*>(&acc);
#pragma unroll
        for (int i = 0; i < (int)(sizeof(acc) / 4); ++i) z[i] = 0.f;
    }

    long oa[2], ob[2];
    dma_offsets(lda, i0, w, l, oa);
    dma_offsets(ldb, j0, w, l, ob);
    // prologue: stages 0 .. NS-2 in flight (4 DMA instructions per wave each); retire stage 0
#pragma unroll
    for (int st = 0; st < NS - 1; ++st) {
        char* d = smem + st * STAGE_BYTES;
        dma_tile(A + (long)(rbeg + st * BK) * lda, oa, d, w);
        dma_tile(B + (long)(rbeg + st * BK) * ldb, ob, d + TILE_BYTES, w);
    }
    if constexpr (NS == 5)
        asm volatile("s_waitcnt vmcnt(12)" ::: "memory");
    else
        asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    for (int kt = 0; kt < nk; ++kt) {
        char* cur = smem + (kt % NS) * STAGE_BYTES;
        char* nxt = smem + ((kt + NS - 1) % NS) * STAGE_BYTES;
        // every step issues exactly one stage so the counted wait below stays exact; past the end it re-loads
        // the last stage into a buffer nobody reads again
        const int rn = min(rbeg + (kt + NS - 1) * BK, rlast);
        kstep<MF, PRIO, DSPLIT>(cur, nxt, A + (long)rn * lda, oa, B + (long)rn * ldb, ob, wr, wc, w, l, acc);
        // stage kt+1 landed; the NS - 2 newer stages stay in flight
        if constexpr (NS == 5)
            asm volatile("s_waitcnt vmcnt(12)" ::: "memory");
        else
            asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (slab == nullptr) {  // one split straight into C; else fp32 partials (splits > 1, or an fp32 C)
        for_each_acc(acc, l, [&](int il, int jl, float v) {
            const long i = i0 + wr + il, j = j0 + wc + jl;
            if (beta != 0.f) v += beta * bf2f(*reinterpret_cast<const u16*>(C + i * ldc + j));
            *reinterpret_cast<u16*>(C + i * ldc + j) = f2bf(v);
        });
    } else {
        float* sp = slab + (long)split * Mo * No;
        for_each_acc(acc, l, [&](int il, int jl, float v) {
            sp[(long)(i0 + wr + il) * No + j0 + wc + jl] = v;
        });
    }
}

}  // namespace g256
}  // namespace gemm
}  // namespace bpe

using namespace bpe::gemm;

size_t gemm_lds_bytes() { return 4 * (size_t)TILE_BYTES; }

bool gemm_shape_ok(int Mo, int No, int R, int splits, int tile) {
    if (tile == 256)
        return Mo % 256 == 0 && No % 256 == 0 && splits >= 1 && R % g256::BK == 0 &&
               R / g256::BK / splits >= g256::NSTAGE - 1;
    return Mo % BM == 0 && No % BN == 0 && splits >= 1 && R % BK == 0 && R / BK >= splits;
}

template <int MF, bool PRIO, int DSPLIT = 0, int NS = g256::NSTAGE>
static void launch_g256_v(const __bf16* a, long lda, const __bf16* b, long ldb, float* slab, __bf16* c, long ldc,
                          float beta, int Mo, int No, int R, int splits, hipStream_t s, int prio) {
    static bool attr = false;  // > 64 KiB dynamic LDS must be opted into once per instantiation
    auto* k = &g256::gemm256_tn_kernel<MF, PRIO, DSPLIT, NS>;
    constexpr int lds = NS * g256::STAGE_BYTES;
    if (!attr) {
        (void)hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, lds);
        attr = true;
    }
    const int grid = (Mo / 256) * (No / 256) * splits;
    k<<<grid, g256::NT, lds, s>>>(a, lda, b, ldb, slab, c, ldc, beta, Mo, No, R, splits, prio);
}

// The dW configuration: 32x32x16 MFMA, the DMA of a stage split over the 16-deep k-step in 2 places (+3-4 % over
// one burst, profiles/bench/ab_dw_dma_split.log), 4 stages.  Measured and not kept: 16x16x32 MFMA and a setprio'd
// MFMA cluster (+-3 %), the DMA split in 4 places (-7 %), a static s_setprio for waves 4-7 (+-0.3 %), 5 stages.
static void launch_g256(const __bf16* a, long lda, const __bf16* b, long ldb, float* slab, __bf16* c, long ldc,
                        float beta, int Mo, int No, int R, int splits, hipStream_t s) {
    launch_g256_v<32, false, 1>(a, lda, b, ldb, slab, c, ldc, beta, Mo, No, R, splits, s, 0);
}

void splitk_reduce(const float* slab, void* C, long ldc, float beta, int M, int N, int splits, int c_f32,
                   hipStream_t s) {
    const long total4 = (long)M * N / 4;
    const int g = (int)std::min<long>((total4 + 255) / 256, 2048);
    if (c_f32)
        splitk_reduce_kernel<float><<<g, 256, 0, s>>>(slab, (float*)C, ldc, beta, M, N, splits);
    else
        splitk_reduce_kernel<__bf16><<<g, 256, 0, s>>>(slab, (__bf16*)C, ldc, beta, M, N, splits);
}

void launch_gemm(int a_kmajor, int b_kmajor, const void* A, long lda, const void* B, long ldb, void* C, long ldc,
                 float beta, int Mo, int No, int R, int splits, float* slab, int tile, int c_f32, hipStream_t s) {
    const __bf16* a = (const __bf16*)A;
    const __bf16* b = (const __bf16*)B;
    __bf16* c = (__bf16*)C;
    if (tile == 256) {  // token-major operands only (host-checked)
        launch_g256(a, lda, b, ldb, slab, c, ldc, beta, Mo, No, R, splits, s);
    } else {
        const int grid = (Mo / BM) * (No / BN) * splits;
        const size_t lds = gemm_lds_bytes();
#define G(AK, BKK) gemm_kernel<AK, BKK><<<grid, 256, lds, s>>>(a, lda, b, ldb, slab, c, ldc, beta, Mo, No, R, splits)
        if (a_kmajor) { if (b_kmajor) G(true, true); else G(true, false); }
        else { if (b_kmajor) G(false, true); else G(false, false); }
#undef G
    }
    if (slab != nullptr) splitk_reduce(slab, C, ldc, beta, Mo, No, splits, c_f32, s);
}
