// Flash attention forward v4 (D = 64, Q / K pre-rotated or no RoPE), gfx950 (MI355X).
// build-flags: -fno-slp-vectorize   (no packed f32 VALU beside the MFMAs: ops/build.py file_flags)
//
// Parity target: reference contracts K7/K9/K10 (`tests/adapters.py:92-184`), as fa_fwd_kernel.
//
// Same geometry as fa_fwd_kernel (4 waves x 32 queries, swapped S^T = K.Q^T with the query on the lane,
// double-buffered K / V, one barrier per 64-key tile, deferred rescale), restructured for the VALU budget, which
// is what bounds D = 64 (a 32 x 64 score tile per wave costs 16 MFMAs but ~1000 cycles of VALU in fa_fwd_kernel:
// per score a subtract, an exponential, a row-sum add, plus zeroing moves).  3 waves per SIMD (162 VGPRs):
//   * the running max is folded into the S accumulator's starting value (guide: "row constants as the initial
//     accumulator"; the query is the lane, so it is one broadcast tuple): S' = K.(cQ)^T - m comes out of the
//     MFMA ready for P = exp2(S'), no subtraction.  Only the rare rescale (a tile max more than 8 above m, or
//     the first tile) subtracts, and then moves m and the tuple;
//   * no tile max on the common path: P = exp2(S') and its row sum (an MFMA, ones^T . P^T: it sums the
//     bf16-rounded P that O sums) first; only a tile whose P sum exceeds 2^THR -- and the first tile -- takes the
//     max, rescales and forms P again (below);
//   * K / V tiles by LDS-DMA through buffer resources (fa_common.h dma_tile64_buf): no staging registers, no
//     per-tile address VALU; rows past the sequence end read as zeros and are masked to -inf.
// Measured (docs/performance.md, attention): the max-less form 0.3125 vs 0.3225 ms (GPT-2 B 128), the DMA staging
// 0.342 vs 0.356-0.362 ms for register staging at 3 / 2 waves per SIMD.
#include "fa_common.h"
#include "kernels.h"

#include <cstdlib>

namespace bpe {
namespace fa {
namespace v4 {

constexpr int D = 64, RB = 128, TILE = 64 * RB, KS = 4;
constexpr float TSUM = 256.0f;  // 2^THR (THR = 8, log2 units): the P-sum threshold of the deferred rescale

template <bool CAUSAL>
__global__ void __launch_bounds__(256, 3)
fa_fwd_v4_kernel(const __bf16* __restrict__ Q, const __bf16* __restrict__ K, const __bf16* __restrict__ Vv,
                 long ld_q, long ld_kv, __bf16* __restrict__ O, long ld_o, float* __restrict__ LSE, int B, int H,
                 int Hkv, int S, float scale_log2, int group, float* __restrict__ DQZ) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    char* Ks = smem;             // [2][64][128 B]
    char* Vs = smem + 2 * TILE;  // [2][64][128 B]
    prologue_prio_begin();  // (fa_common.h)
    const int tid = threadIdx.x, w = tid >> 6, l = tid & 63, l31 = l & 31, hh = l >> 5;
    const int nqb = (S + 127) / 128;
    int qrank, bh;
    grouped_order((int)blockIdx.x, nqb, B * H, group, qrank, bh);
    const int qb = nqb - 1 - qrank;  // heaviest (last) query blocks first
    const int b = bh / H, h = bh % H, hk = h / (H / Hkv);
    const int q0 = qb * 128, qw0 = q0 + 32 * w, qrow = qw0 + l31;

    // prologue: the Q rows and K / V tile 0 are all requested before any is waited for (one memory round trip)
    u16x8 qr[KS];
    {
        const long qpos = min(qrow, S - 1);  // rows past the end clamped
        const __bf16* qp = Q + ((long)b * S + qpos) * ld_q + (long)h * D;
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) qr[ks] = *reinterpret_cast<const u16x8*>(qp + 16 * ks + 8 * hh);
    }
    const int n_end = CAUSAL ? min(S, q0 + 128) : S;
    const int ntiles = (n_end + 63) / 64;
    const __bf16* kbase = K + (long)b * S * ld_kv + (long)hk * D;
    const __bf16* vbase = Vv + (long)b * S * ld_kv + (long)hk * D;

    f32x16 o[2], nm;  // O^T (d rows, query lane), -m (S accumulator start)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
        o[0][r] = 0.f;
        o[1][r] = 0.f;
        nm[r] = 0.f;
    }
    float m_run = 0.f, lsum_t = 0.f;  // lsum_t: the row sum
    bf16x8 ones;
#pragma unroll
    for (int j = 0; j < 8; ++j) ones[j] = (__bf16)1.0f;

    const int trow = 4 * hh + ((l & 15) >> 2);
    const int tcol = 16 * ((l >> 4) & 1) + 4 * (l & 3);

    // K / V tiles by LDS-DMA through buffer resources (fa_common.h dma_tile64_buf; rows past the end read as 0 and
    // are masked below)
    const int wu = __builtin_amdgcn_readfirstlane(w);
    // K and V share the row stride: one set of lane offsets and one extent serve both buffer resources
    const int hbytes = head_bytes(ld_kv, S, D);
    const DmaVoff<4> vo = dma_voff<4>(ld_kv, wu, l);
    dma_tile64_buf(kbase, hbytes, vo, 0, ld_kv, Ks, wu);
    dma_tile64_buf(vbase, hbytes, vo, 0, ld_kv, Vs, wu);
    // Q fragments (B operand of S^T = K.Q^T), softmax scale * log2(e) folded in
    bf16x8 qf[KS];
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
        float x[8];
        unpack8(qr[ks], x);
        qf[ks] = __builtin_bit_cast(bf16x8, pack8(x, scale_log2));
    }
    __syncthreads();
    prologue_prio_end();
    for (int t = 0; t < ntiles; ++t) {
        const int cur = t & 1, n0 = t * 64;
        if (t + 1 < ntiles) {  // buffer cur ^ 1 was last read in tile t - 1, before its closing barrier
            dma_tile64_buf(kbase, hbytes, vo, n0 + 64, ld_kv, Ks + (cur ^ 1) * TILE, wu);
            dma_tile64_buf(vbase, hbytes, vo, n0 + 64, ld_kv, Vs + (cur ^ 1) * TILE, wu);
        }
        if (!CAUSAL || n0 <= qw0 + 31) {
            const char* Kc = Ks + cur * TILE;
            char* Vc = Vs + cur * TILE;
            f32x16 s[2];
#pragma unroll
            for (int kt = 0; kt < 2; ++kt) {
                s[kt] = nm;
#pragma unroll
                for (int ks = 0; ks < KS; ++ks)
                    s[kt] = mfma(lds_row16(Kc, swz<RB>(kt * 32 + l31, 2 * ks + hh)), qf[ks], s[kt]);
            }
            if ((CAUSAL && n0 + 63 > qw0) || (n0 + 64 > S)) {  // diagonal / ragged tile (wave-uniform)
                // key n0 + 32 kt + acc_row(r, hh) is valid iff it is <= min(qrow, S - 1) (causal) / S - 1: one
                // compare of the per-lane limit against the register's compile-time row offset (acc_row minus its
                // lane-half term) and one select per score
                const int qlim = (CAUSAL ? min(qrow, S - 1) : S - 1) - n0 - 4 * hh;
#pragma unroll
                for (int kt = 0; kt < 2; ++kt)
#pragma unroll
                    for (int r = 0; r < 16; ++r)
                        if ((r & 3) + 8 * (r >> 2) > qlim - 32 * kt) s[kt][r] = -INFINITY;
            }
            // No tile max on the common path: P = exp2(S') is formed at once and its row sum taken by MFMA into
            // a fresh accumulator; only a tile whose P sum exceeds 2^THR (some score more than ~THR above the
            // running max, or inf / NaN) -- and the first tile -- takes the max, rescales, and forms P and its
            // sum again, before any of this tile's P reaches O (guide T13 hazard).  Every P that reaches O is
            // <= 2^THR, as with the max test.  Saves the ~20 max instructions and the lane exchange per tile.
            bf16x8 pf[4];
            auto exp_tile = [&]() {
#pragma unroll
                for (int kk = 0; kk < 4; ++kk) {
                    const int kt = kk >> 1, ss = kk & 1;
#pragma unroll
                    for (int j = 0; j < 8; ++j) pf[kk][j] = (__bf16)fast_exp2(s[kt][8 * ss + j]);
                }
            };
            auto tile_sum = [&]() {  // every register of the result holds the lane's row sum
                f32x16 lt = mfma(ones, pf[0], f32x16{});
#pragma unroll
                for (int kk = 1; kk < 4; ++kk) lt = mfma(ones, pf[kk], lt);
                return lt[0];
            };
            float lt = 0.f;
            if (t > 0) {
                exp_tile();
                lt = tile_sum();
            }
            const bool grow = t == 0 || !(lt <= TSUM);
            if (!__all(!grow)) {
                float mt = s[0][0];
#pragma unroll
                for (int kt = 0; kt < 2; ++kt)
#pragma unroll
                    for (int r = 0; r < 16; ++r) mt = fmaxf(mt, s[kt][r]);
                mt = fmaxf(mt, __shfl_xor(mt, 32, 64));
                const float d = grow ? mt : 0.f;
                const float alpha = t == 0 ? 0.f : fast_exp2(-d);
                m_run += d;
                lsum_t *= alpha;
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    o[0][r] *= alpha;
                    o[1][r] *= alpha;
                    nm[r] = -m_run;
                    s[0][r] -= d;
                    s[1][r] -= d;
                }
                exp_tile();
                lt = tile_sum();
            }
            lsum_t += lt;
#pragma unroll
            for (int kk = 0; kk < 4; ++kk) {
                const int kb = (kk >> 1) * 32 + 16 * (kk & 1);
#pragma unroll
                for (int dt = 0; dt < 2; ++dt)
                    o[dt] = mfma(lds_tr_pair(Vc, tr_off<RB>(kb + trow, dt * 32 + tcol),
                                             tr_off<RB>(kb + 8 + trow, dt * 32 + tcol)),
                                 pf[kk], o[dt]);
            }
        }
        // no barrier after the last (diagonal) tile: a wave done with it does not wait for the others
        if (t + 1 < ntiles) __syncthreads();
    }

    // ---- epilogue: O = O^T / l (query on the lane, 4 consecutive d per register group), LSE = m + log2 l
    if (qrow < S) {
        const float lsum = lsum_t;
        const float inv = lsum > 0.f ? 1.f / lsum : 0.f;
        __bf16* op = O + ((long)b * S + qrow) * ld_o + (long)h * D;
#pragma unroll
        for (int dt = 0; dt < 2; ++dt)
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const u16x4 v = {f2bf(o[dt][4 * i] * inv), f2bf(o[dt][4 * i + 1] * inv),
                                 f2bf(o[dt][4 * i + 2] * inv), f2bf(o[dt][4 * i + 3] * inv)};
                *reinterpret_cast<u16x4*>(op + dt * 32 + 8 * i + 4 * hh) = v;
            }
        if (hh == 0) LSE[((long)b * H + h) * S + qrow] = lsum > 0.f ? m_run + __log2f(lsum) : INFINITY;
    }
    if (DQZ != nullptr) {  // the fused (atomics) backward's fp32 dQ accumulator, zeroed as fa_fwd_kernel does
        constexpr int C4 = D / 4;
        const int spad = (S + 63) & ~63;
        const int rows = min(128, spad - q0);
        float* zb = DQZ + ((long)b * spad + q0) * ((long)H * D) + (long)h * D;
        for (int e = tid; e < rows * C4; e += 256) {
            const int r = e / C4, c = e % C4;
            *reinterpret_cast<float4*>(zb + (long)r * H * D + 4 * c) = float4{0.f, 0.f, 0.f, 0.f};
        }
    }
}

}  // namespace v4
}  // namespace fa
}  // namespace bpe

using namespace bpe;
using namespace bpe::fa;

// The D = 64 forward without in-kernel RoPE: 8 (default, this file's kernel) or 2 (fa_fwd_kernel, the general
// kernel of flash_attn_fwd.hip, which also serves D = 128 and the fused-RoPE form); fa_fwd_config switches it at run
// time (tests compare the two).  Earlier versions (register staging at 2 / 3 waves per SIMD, a ping-pong schedule,
// the tile max on every tile) were measured slower and removed (docs/performance.md, attention).
static int g_fwd_ver = 8;

int fa_fwd_config(int ver) {
    const int prev = g_fwd_ver;
    if (ver > 0) g_fwd_ver = ver == 2 ? 2 : 8;
    return prev;
}

bool launch_fa_fwd_v4(const FaArgs& a, hipStream_t s) {
    if (a.D != 64 || a.rope == 1 || g_fwd_ver == 2) return false;
    const int nqb = (a.S + 127) / 128;
    auto* k = a.causal ? &v4::fa_fwd_v4_kernel<true> : &v4::fa_fwd_v4_kernel<false>;
    k<<<nqb * a.B * a.H, 256, 4 * v4::TILE, s>>>(a.q, a.k, a.v, a.ld_q, a.ld_kv, a.o, a.ld_o, a.lse, a.B, a.H, a.Hkv,
                                                 a.S, a.scale * LOG2E, fa_group(a.B * a.H), a.dq_acc);
    return true;
}
