// Flash attention forward with fused interleaved RoPE, gfx950 (MI355X).
// build-flags: -fno-slp-vectorize   (no packed f32 VALU beside the MFMAs: ops/build.py file_flags)
//
// Parity targets: reference contracts K7/K9/K10 (`tests/adapters.py:92-184`):
// softmax(Q K^T / sqrt(d) [causal]) V with RoPE on Q and K (interleaved
// pairs).
//
// Structure (one workgroup = 4 waves = 128 query rows of one (batch, head)):
//   * MFMA v_mfma_f32_32x32x16_bf16; each wave owns 32 query rows.  The
//     SWAPPED product S^T = K.Q^T puts one query on each lane (query =
//     lane & 31, 16 keys per 32-key tile in its registers), so the online
//     softmax max / sum are register-local plus one lane^32 exchange
//     (guide §B attention, T12).
//   * The fp32 S^T accumulator becomes, after exp2 and a bf16 convert, the B
//     operand of O^T += V^T.P^T directly (guide §3: an accumulator tile is the
//     next MFMA's operand when the product sums over its row index); the
//     permuted k order inside each 16-key step is matched on the V side by
//     the rows the transposed reads fetch.  O^T also keeps the query on the
//     lane, so the per-row rescale is a register multiply.
//   * V^T fragments come from ds_read_b64_tr_b16; K rows from ds_read_b128;
//     both through the one swizzled image described in fa_common.h.
//   * Register-staged double-buffered K/V (guide T14): the global loads of
//     tile t+1 are issued before tile t's MFMAs, written to the other LDS
//     buffer after them; one barrier per 64-key tile.
//   * RoPE: Q is rotated and pre-scaled by softmax_scale * log2(e) once when it
//     is loaded to registers; K is rotated while it is staged to LDS (fp32
//     cos/sin table, no device trig; the table entries are loaded together with
//     the K/V tile, not at the write: 0.292 -> 0.283 ms at the GPT-2 shape).  Scores are therefore in log2 units and
//     the exponentials are raw v_exp_f32.
//   * Deferred rescale (guide T13): the running max only moves when a tile's
//     max exceeds it by more than 8 (log2 units), so most tiles skip the O
//     rescale; P is bounded by 2^8, safe in bf16 and fp32 accumulators.  The
//     decision covers the whole tile before any of its P is formed.
//   * Work order: heaviest causal blocks first; the blocks of one (batch,
//     head) are 8-aligned apart in launch order so they share an XCD L2 under
//     round-robin dispatch (speed only).
#include "fa_common.h"
#include "kernels.h"

#include <cstdlib>
#include <type_traits>

namespace bpe {
namespace fa {

constexpr float RESCALE_THRESHOLD = 8.0f;


template <int D, bool CAUSAL, bool ROPE>
__global__ void __launch_bounds__(256, 2)
fa_fwd_kernel(const __bf16* __restrict__ Q, const __bf16* __restrict__ K, const __bf16* __restrict__ Vv, long ld_q,
              long ld_kv, __bf16* __restrict__ O, long ld_o, float* __restrict__ LSE, const float* __restrict__ cosT,
              const float* __restrict__ sinT, int B, int H, int Hkv, int S, float scale_log2, int group,
              float* __restrict__ DQZ) {
    constexpr int RB = D * 2;            // bytes per LDS row
    constexpr int CPR = D / 8;           // 16-byte chunks per row
    constexpr int TILE = 64 * RB;        // bytes per 64-row tile
    constexpr int SPT = 64 * CPR / 256;  // staged chunks per thread per tile
    constexpr int KS = D / 16;           // k-steps over the head dim
    constexpr int DT = D / 32;           // 32-wide d tiles of O
    extern __shared__ __attribute__((aligned(16))) char smem[];
    char* Ks = smem;             // [2][64][D]
    char* Vs = smem + 2 * TILE;  // [2][64][D]

    const int tid = threadIdx.x, w = tid >> 6, l = tid & 63, l31 = l & 31, hh = l >> 5;
    const int nqb = (S + 127) / 128;
    const int BH = B * H;
    int qrank, bh;
    grouped_order((int)blockIdx.x, nqb, BH, group, qrank, bh);
    const int qb = nqb - 1 - qrank;
    const int b = bh / H, h = bh % H;
    const int hk = h / (H / Hkv);
    const int q0 = qb * 128, qw0 = q0 + 32 * w;
    const int qrow = qw0 + l31;

    // ---- Q fragments (B operand of S^T = K.Q^T): RoPE + softmax scale * log2(e) folded in
    bf16x8 qf[KS];
    {
        const bool ok = qrow < S;
        const long qpos = ok ? qrow : 0;
        const __bf16* qp = Q + ((long)b * S + qpos) * ld_q + (long)h * D;
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) {
            const int d0 = 16 * ks + 8 * hh;
            u16x8 t = ok ? *reinterpret_cast<const u16x8*>(qp + d0) : u16x8{0, 0, 0, 0, 0, 0, 0, 0};
            if (ROPE) {
                t = rope_u16x8(t, cosT + qpos * (D / 2) + d0 / 2, sinT + qpos * (D / 2) + d0 / 2, scale_log2);
            } else {
                float x[8];
                unpack8(t, x);
                t = pack8(x, scale_log2);
            }
            qf[ks] = __builtin_bit_cast(bf16x8, t);
        }
    }

    const int n_end = CAUSAL ? min(S, q0 + 128) : S;
    const int ntiles = (n_end + 63) / 64;
    const __bf16* kbase = K + (long)b * S * ld_kv + (long)hk * D;
    const __bf16* vbase = Vv + (long)b * S * ld_kv + (long)hk * D;

    u16x8 kreg[SPT], vreg[SPT];
    // the K tile's rope table entries, loaded with it (off the write path); D = 128 has no VGPRs to spare
    constexpr bool PFT = ROPE && D == 64;
    f32x4 creg[SPT], sreg[SPT];
    auto load_tile = [&](int t) {
#pragma unroll
        for (int i = 0; i < SPT; ++i) {
            const int e = tid + 256 * i, row = e / CPR, c = e % CPR;
            const int key = t * 64 + row;
            if (key < S) {
                kreg[i] = *reinterpret_cast<const u16x8*>(kbase + (long)key * ld_kv + c * 8);
                vreg[i] = *reinterpret_cast<const u16x8*>(vbase + (long)key * ld_kv + c * 8);
            } else {
                kreg[i] = u16x8{0, 0, 0, 0, 0, 0, 0, 0};
                vreg[i] = u16x8{0, 0, 0, 0, 0, 0, 0, 0};
            }
            if (PFT) {
                const long kk = min(key, S - 1);
                creg[i] = *reinterpret_cast<const f32x4*>(cosT + kk * (D / 2) + c * 4);
                sreg[i] = *reinterpret_cast<const f32x4*>(sinT + kk * (D / 2) + c * 4);
            }
        }
    };
    auto write_tile = [&](int t, int buf) {
#pragma unroll
        for (int i = 0; i < SPT; ++i) {
            const int e = tid + 256 * i, row = e / CPR, c = e % CPR;
            u16x8 kv = kreg[i];
            if (PFT) {
                float x[8];
                unpack8(kv, x);
                rope8v(x, creg[i], sreg[i]);
                kv = pack8(x, 1.f);
            } else if (ROPE) {
                const long key = min(t * 64 + row, S - 1);
                kv = rope_u16x8(kv, cosT + key * (D / 2) + c * 4, sinT + key * (D / 2) + c * 4, 1.f);
            }
            *reinterpret_cast<u16x8*>(Ks + buf * TILE + swz<RB>(row, c)) = kv;
            *reinterpret_cast<u16x8*>(Vs + buf * TILE + swz<RB>(row, c)) = vreg[i];
        }
    };

    f32x16 o[DT];
#pragma unroll
    for (int dt = 0; dt < DT; ++dt)
#pragma unroll
        for (int r = 0; r < 16; ++r) o[dt][r] = 0.f;
    float m_run = -INFINITY, l_run = 0.f;

    const int trow = 4 * hh + ((l & 15) >> 2);          // tr-read row inside a 16-key step
    const int tcol = 16 * ((l >> 4) & 1) + 4 * (l & 3);  // tr-read column inside a 32-wide d tile

    load_tile(0);
    write_tile(0, 0);
    __syncthreads();

    for (int t = 0; t < ntiles; ++t) {
        const int cur = t & 1;
        if (t + 1 < ntiles) load_tile(t + 1);
        const int n0 = t * 64;
        const bool active = !CAUSAL || (n0 <= qw0 + 31);
        if (active) {
            const char* Kc = Ks + cur * TILE;
            char* Vc = Vs + cur * TILE;
            f32x16 s[2];
#pragma unroll
            for (int kt = 0; kt < 2; ++kt) {
#pragma unroll
                for (int r = 0; r < 16; ++r) s[kt][r] = 0.f;
#pragma unroll
                for (int ks = 0; ks < KS; ++ks)
                    s[kt] = mfma(lds_row16(Kc, swz<RB>(kt * 32 + l31, 2 * ks + hh)), qf[ks], s[kt]);
            }
            if ((CAUSAL && n0 + 63 > qw0) || (n0 + 64 > S)) {
#pragma unroll
                for (int kt = 0; kt < 2; ++kt)
#pragma unroll
                    for (int r = 0; r < 16; ++r) {
                        const int key = n0 + kt * 32 + acc_row(r, hh);
                        if ((CAUSAL && key > qrow) || key >= S) s[kt][r] = -INFINITY;
                    }
            }
            float mt = s[0][0];
#pragma unroll
            for (int kt = 0; kt < 2; ++kt)
#pragma unroll
                for (int r = 0; r < 16; ++r) mt = fmaxf(mt, s[kt][r]);
            mt = fmaxf(mt, __shfl_xor(mt, 32, 64));
            // deferred rescale: move the running max only when this tile exceeds it by > threshold
            const bool grow = mt > m_run + RESCALE_THRESHOLD;
            float alpha = 1.f;
            if (grow) {
                alpha = fast_exp2(m_run - mt);  // m_run = -inf on the first tile -> 0
                m_run = mt;
            }
            const float mu = (m_run == -INFINITY) ? 0.f : m_run;
            float ls = 0.f;
#pragma unroll
            for (int kt = 0; kt < 2; ++kt)
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    const float p = fast_exp2(s[kt][r] - mu);
                    s[kt][r] = p;
                    ls += p;
                }
            ls += __shfl_xor(ls, 32, 64);
            l_run = l_run * alpha + ls;
            if (!__all(!grow)) {
#pragma unroll
                for (int dt = 0; dt < DT; ++dt)
#pragma unroll
                    for (int r = 0; r < 16; ++r) o[dt][r] *= alpha;
            }
            // P^T fragments: k-step kk = (key tile kt, half ss) in the accumulator's permuted k order
            bf16x8 pf[4];
#pragma unroll
            for (int kk = 0; kk < 4; ++kk) {
                const int kt = kk >> 1, ss = kk & 1;
#pragma unroll
                for (int j = 0; j < 8; ++j) pf[kk][j] = (__bf16)s[kt][8 * ss + j];
            }
#pragma unroll
            for (int dt = 0; dt < DT; ++dt)
#pragma unroll
                for (int kk = 0; kk < 4; ++kk) {
                    const int kb = (kk >> 1) * 32 + 16 * (kk & 1);
                    const bf16x8 va = lds_tr_pair(Vc, tr_off<RB>(kb + trow, dt * 32 + tcol),
                                                  tr_off<RB>(kb + 8 + trow, dt * 32 + tcol));
                    o[dt] = mfma(va, pf[kk], o[dt]);
                }
        }
        if (t + 1 < ntiles) write_tile(t + 1, cur ^ 1);
        __syncthreads();
    }

    // ---- epilogue: O = O^T / l, query on the lane, 4 consecutive d per register group
    if (qrow < S) {
        const float inv = l_run > 0.f ? 1.f / l_run : 0.f;
        __bf16* op = O + ((long)b * S + qrow) * ld_o + (long)h * D;
#pragma unroll
        for (int dt = 0; dt < DT; ++dt)
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                u16x4 t = {f2bf(o[dt][4 * i] * inv), f2bf(o[dt][4 * i + 1] * inv), f2bf(o[dt][4 * i + 2] * inv),
                           f2bf(o[dt][4 * i + 3] * inv)};
                *reinterpret_cast<u16x4*>(op + dt * 32 + 8 * i + 4 * hh) = t;
            }
        if (hh == 0) LSE[((long)b * H + h) * S + qrow] = (l_run > 0.f) ? m_run + __log2f(l_run) : INFINITY;
    }
    // training: zero this block's rows of the backward's fp32 dQ accumulator ([B][Spad][H][D], rows padded to
    // 64), after every other store -- fire-and-forget stores under a compute-bound kernel replace the zeroing
    // pass of fa_bwd_pre_kernel (one 4 x [tokens, H*D]-byte HBM write per layer).  Blocks cover [0, Spad).
    if (DQZ != nullptr) {
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

}  // namespace fa
}  // namespace bpe

using namespace bpe;
using namespace bpe::fa;

size_t fa_fwd_lds_bytes(int D) { return (size_t)4 * 64 * D * 2; }

template <int D, bool C, bool R>
static void fwd_launch(const FaArgs& a, hipStream_t s) {
    const int nqb = (a.S + 127) / 128;
    fa_fwd_kernel<D, C, R><<<nqb * a.B * a.H, 256, fa_fwd_lds_bytes(D), s>>>(
        a.q, a.k, a.v, a.ld_q, a.ld_kv, a.o, a.ld_o, a.lse, a.cos, a.sin, a.B, a.H, a.Hkv, a.S, a.scale * LOG2E, fa_group(a.B * a.H),
        a.dq_acc);
}

void launch_fa_fwd(const FaArgs& a, hipStream_t s) {
    if (launch_fa_fwd_v4(a, s)) return;  // D = 64 without in-kernel RoPE (flash_attn_fwd_v4.hip)
    // rope 2 = Q / K already rotated: no RoPE inside the kernel
    const bool r = a.rope == 1;
#define FWD_CASE(DD)                                                                                        \
    if (a.D == DD) {                                                                                        \
        if (a.causal) { if (r) fwd_launch<DD, true, true>(a, s); else fwd_launch<DD, true, false>(a, s); } \
        else { if (r) fwd_launch<DD, false, true>(a, s); else fwd_launch<DD, false, false>(a, s); }     \
        return;                                                                                             \
    }
    FWD_CASE(64) FWD_CASE(128)
#undef FWD_CASE
}
