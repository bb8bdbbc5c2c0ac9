// bf16 MFMA GEMM with split-K for gfx950, used for the weight-gradient products.
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
    const int rlen = R / splits;  // multiple of BK (host-checked)
    const int rbeg = split * rlen;
    const int nk = rlen / BK;
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
    if (splits == 1) {
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

// C = beta*C + sum_s slab[s]  (fixed order -> deterministic); 4 outputs per thread
__global__ void __launch_bounds__(256) splitk_reduce_kernel(const float* __restrict__ slab, __bf16* __restrict__ C,
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
        u16x4* cp = reinterpret_cast<u16x4*>(C + i * ldc + j);
        if (beta != 0.f) {
            const u16x4 c = *cp;
            s[0] += beta * bf2f(c[0]); s[1] += beta * bf2f(c[1]);
            s[2] += beta * bf2f(c[2]); s[3] += beta * bf2f(c[3]);
        }
        *cp = u16x4{f2bf(s[0]), f2bf(s[1]), f2bf(s[2]), f2bf(s[3])};
    }
}

}  // namespace gemm
}  // namespace bpe

using namespace bpe::gemm;

size_t gemm_lds_bytes() { return 4 * (size_t)TILE_BYTES; }

bool gemm_shape_ok(int Mo, int No, int R, int splits) {
    return Mo % BM == 0 && No % BN == 0 && splits >= 1 && R % (BK * splits) == 0;
}

void launch_gemm(int a_kmajor, int b_kmajor, const void* A, long lda, const void* B, long ldb, void* C, long ldc,
                 float beta, int Mo, int No, int R, int splits, float* slab, hipStream_t s) {
    const int grid = (Mo / BM) * (No / BN) * splits;
    const size_t lds = gemm_lds_bytes();
    const __bf16* a = (const __bf16*)A;
    const __bf16* b = (const __bf16*)B;
    __bf16* c = (__bf16*)C;
#define G(AK, BKK) gemm_kernel<AK, BKK><<<grid, 256, lds, s>>>(a, lda, b, ldb, slab, c, ldc, beta, Mo, No, R, splits)
    if (a_kmajor) { if (b_kmajor) G(true, true); else G(true, false); }
    else { if (b_kmajor) G(false, true); else G(false, false); }
#undef G
    if (splits > 1) {
        const long total4 = (long)Mo * No / 4;
        const int g = (int)std::min<long>((total4 + 255) / 256, 2048);
        splitk_reduce_kernel<<<g, 256, 0, s>>>(slab, c, ldc, beta, Mo, No, splits);
    }
}
