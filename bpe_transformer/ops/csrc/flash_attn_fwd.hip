// Flash attention forward with fused interleaved RoPE, gfx950 (MI355X).
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

// ---------------------------------------------------------------------------------------------------------
// v3 forward for D = 64 with Q / K already rotated (ops.rope_qk_, rope mode 2) or no RoPE.
//
// Same per-wave math as fa_fwd_kernel (swapped S^T = K.Q^T, query on the lane, P^T straight from the S
// accumulator into O^T += V^T.P^T, deferred rescale), restructured for the VALU budget that bounded it
// (~270 VALU per 64-key tile and wave, ~22 per MFMA: rocprofv3, profiles/attention_pmc.md):
//   * no per-tile RoPE: K and V tiles go global -> LDS by LDS-DMA (global_load_lds_dwordx4, guide §5), no
//     VGPR staging, no staging VALU.  The swizzled image of fa_common.h is produced by permuting the SOURCE
//     address of each lane (lane-linear LDS destination).  4 DMA instructions per wave and tile.
//   * software pipeline (guide T15): S(t+1) = K(t+1).Q^T is issued in the same block as the softmax of
//     tile t, so the matrix pipe works on the next tile while the VALU exponentiates this one; S is
//     double-buffered in registers (the loop is unrolled by two so both buffers are static).
//   * buffers: K(j) in Ks[j & 1], V(j) in Vs[j & 1]; iteration t waits for K(t+1), V(t) (DMA issued one
//     iteration earlier) with ONE barrier, then issues K(t+2), V(t+1) into the buffers iteration t-1 read.
// ---------------------------------------------------------------------------------------------------------

struct FwdV3 {
    static constexpr int D = 64, RB = 128, TILE = 64 * RB, KS = 4;
    // per-wave constants
    int l31, hh, qw0, qrow, S, trow, tcol;
    long ld_kv;
    int prow[2], pcol[2];
    bf16x8 qf[KS];
    // running state
    f32x16 o[2];
    float m_run, l_run;

    // 2 LDS-DMA pieces (8 rows x 128 B each) of tile t of one operand into `img`; rows past the end of the
    // sequence load row S-1 (valid memory, masked out of the softmax)
    __device__ __forceinline__ void dma(const __bf16* base, char* __restrict__ img, int t, int w) const {
        const bool tail = t * 64 + 64 > S;
#pragma unroll
        for (int i = 0; i < 2; ++i) {
            int key = t * 64 + prow[i];
            if (tail) key = min(key, S - 1);
            __builtin_amdgcn_global_load_lds((gbl_void_t*)(base + (long)key * ld_kv + pcol[i]),
                                             (lds_void_t*)(img + (16 * w + 8 * i) * RB), 16, 0, 0);
        }
    }

    __device__ __forceinline__ void qk(const char* __restrict__ Kc, f32x16 (&s)[2]) const {
#pragma unroll
        for (int kt = 0; kt < 2; ++kt) {
#pragma unroll
            for (int r = 0; r < 16; ++r) s[kt][r] = 0.f;
#pragma unroll
            for (int ks = 0; ks < KS; ++ks)
                s[kt] = mfma(lds_row16(Kc, swz<RB>(kt * 32 + l31, 2 * ks + hh)), qf[ks], s[kt]);
        }
    }

    // mask + running-max update of tile t (the rare rescale branch included); returns the exponent offset
    template <bool CAUSAL>
    __device__ __forceinline__ float prep(int t, f32x16 (&s)[2]) {
        const int n0 = t * 64;
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
        const bool grow = mt > m_run + RESCALE_THRESHOLD;
        if (!__all(!grow)) {  // rare (first tile, or a large jump): rescale O and l by the max update
            const float alpha = grow ? fast_exp2(m_run - mt) : 1.f;  // m_run = -inf on the first tile -> 0
            m_run = grow ? mt : m_run;
            l_run *= alpha;
#pragma unroll
            for (int dt = 0; dt < 2; ++dt)
#pragma unroll
                for (int r = 0; r < 16; ++r) o[dt][r] *= alpha;
        }
        return (m_run == -INFINITY) ? 0.f : m_run;
    }

    // exp2 + row sum + P^T fragments + O^T += V^T.P^T of the current tile, with the 8 MFMAs of S(t+1) from Kn
    // issued in the same basic block so the scheduler interleaves them with the exponentials.  On a wave's
    // last active tile S(t+1) comes from a stale K buffer and is never used (8 wasted MFMAs, one code path).
    __device__ __forceinline__ void finish(f32x16 (&s)[2], float mu, const char* __restrict__ Kn,
                                           const char* __restrict__ Vc, f32x16 (&nxt)[2]) {
        float ls = 0.f;
#pragma unroll
        for (int kt = 0; kt < 2; ++kt) {
#pragma unroll
            for (int r = 0; r < 16; ++r) nxt[kt][r] = 0.f;
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                if ((r & 3) == 0)
                    nxt[kt] = mfma(lds_row16(Kn, swz<RB>(kt * 32 + l31, 2 * (r >> 2) + hh)), qf[r >> 2], nxt[kt]);
                const float p = fast_exp2(s[kt][r] - mu);
                s[kt][r] = p;
                ls += p;
            }
        }
        ls += __shfl_xor(ls, 32, 64);
        l_run += ls;
        bf16x8 pf[4];
#pragma unroll
        for (int kk = 0; kk < 4; ++kk) {
            const int kt = kk >> 1, ss = kk & 1;
#pragma unroll
            for (int j = 0; j < 8; ++j) pf[kk][j] = (__bf16)s[kt][8 * ss + j];
        }
#pragma unroll
        for (int dt = 0; dt < 2; ++dt)
#pragma unroll
            for (int kk = 0; kk < 4; ++kk) {
                const int kb = (kk >> 1) * 32 + 16 * (kk & 1);
                const bf16x8 va = lds_tr_pair(const_cast<char*>(Vc), tr_off<RB>(kb + trow, dt * 32 + tcol),
                                              tr_off<RB>(kb + 8 + trow, dt * 32 + tcol));
                o[dt] = mfma(va, pf[kk], o[dt]);
            }
    }

    // one pipelined iteration: consumes S(t) in `cur`, produces S(t+1) in `nxt`.  The four LDS regions are
    // __restrict__ so that, inlined, the fragment reads carry alias scopes proving they do not touch the DMA
    // targets (without it the wait-count pass drains the just-issued DMA, vmcnt(0), before the V reads).
    template <bool CAUSAL>
    __device__ __forceinline__ void iter(int t, int ntiles, int w, const __bf16* kbase, const __bf16* vbase,
                                         char* __restrict__ k_dma, char* __restrict__ v_dma,
                                         const char* __restrict__ k_next, const char* __restrict__ v_cur,
                                         f32x16 (&cur)[2], f32x16 (&nxt)[2]) {
        __syncthreads();  // K(t+1), V(t) landed (the barrier's vmcnt(0) drains this wave's DMA); iteration t-1
                          // is done reading the buffers the DMA below overwrites
        if (t + 2 < ntiles) dma(kbase, k_dma, t + 2, w);
        if (t + 1 < ntiles) dma(vbase, v_dma, t + 1, w);
        if (!CAUSAL || t * 64 <= qw0 + 31) {
            const float mu = prep<CAUSAL>(t, cur);
            finish(cur, mu, k_next, v_cur, nxt);
        }
    }
};

template <bool CAUSAL>
__global__ void __launch_bounds__(256, 2)
fa_fwd_v3_kernel(const __bf16* __restrict__ Q, const __bf16* __restrict__ K, const __bf16* __restrict__ Vv, long ld_q,
                 long ld_kv, __bf16* __restrict__ O, long ld_o, float* __restrict__ LSE, int B, int H, int Hkv,
                 int S, float scale_log2, int group) {
    using F = FwdV3;
    constexpr int D = F::D, TILE = F::TILE;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    char* K0 = smem;            // K(j) in K0 / K1 by the parity of j
    char* K1 = smem + TILE;
    char* V0 = smem + 2 * TILE; // V(j) in V0 / V1
    char* V1 = smem + 3 * TILE;

    const int tid = threadIdx.x, l = tid & 63;
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int nqb = (S + 127) / 128;
    const int BH = B * H;
    int qrank, bh;
    grouped_order((int)blockIdx.x, nqb, BH, group, qrank, bh);
    const int qb = nqb - 1 - qrank;
    const int b = bh / H, h = bh % H;
    const int hk = h / (H / Hkv);
    const int q0 = qb * 128;

    F f;
    f.l31 = l & 31;
    f.hh = l >> 5;
    f.qw0 = q0 + 32 * w;
    f.qrow = f.qw0 + f.l31;
    f.S = S;
    f.ld_kv = ld_kv;
    f.trow = 4 * f.hh + ((l & 15) >> 2);
    f.tcol = 16 * ((l >> 4) & 1) + 4 * (l & 3);
#pragma unroll
    for (int i = 0; i < 2; ++i) {
        // lane l of piece i writes LDS slot l of the piece = row 16w + 8i + (l >> 3), physical chunk l & 7,
        // which holds logical chunk (l & 7) ^ sigma(row) (fa_common.h swz<128>)
        const int r = 16 * w + 8 * i + (l >> 3);
        const int sg = (((r >> 1) & 1) << 2) | ((r >> 2) & 3);
        f.prow[i] = r;
        f.pcol[i] = ((l & 7) ^ sg) * 8;
    }
    {  // Q fragments (B operand of S^T = K.Q^T), pre-rotated; softmax scale * log2(e) folded in
        const bool ok = f.qrow < S;
        const __bf16* qp = Q + ((long)b * S + (ok ? f.qrow : 0)) * ld_q + (long)h * D;
#pragma unroll
        for (int ks = 0; ks < F::KS; ++ks) {
            const int d0 = 16 * ks + 8 * f.hh;
            u16x8 t = ok ? *reinterpret_cast<const u16x8*>(qp + d0) : u16x8{0, 0, 0, 0, 0, 0, 0, 0};
            float x[8];
            unpack8(t, x);
            f.qf[ks] = __builtin_bit_cast(bf16x8, pack8(x, scale_log2));
        }
    }
#pragma unroll
    for (int dt = 0; dt < 2; ++dt)
#pragma unroll
        for (int r = 0; r < 16; ++r) f.o[dt][r] = 0.f;
    f.m_run = -INFINITY;
    f.l_run = 0.f;

    const int n_end = CAUSAL ? min(S, q0 + 128) : S;
    const int ntiles = (n_end + 63) / 64;
    const __bf16* kbase = K + (long)b * S * ld_kv + (long)hk * D;
    const __bf16* vbase = Vv + (long)b * S * ld_kv + (long)hk * D;

    f32x16 sa[2], sb[2];
    f.dma(kbase, K0, 0, w);
    __syncthreads();
    if (ntiles > 1) f.dma(kbase, K1, 1, w);
    f.dma(vbase, V0, 0, w);
    f.qk(K0, sa);  // tile 0 is active for every wave
    for (int t = 0; t < ntiles; t += 2) {
        f.iter<CAUSAL>(t, ntiles, w, kbase, vbase, K0, V1, K1, V0, sa, sb);
        if (t + 1 < ntiles) f.iter<CAUSAL>(t + 1, ntiles, w, kbase, vbase, K1, V0, K0, V1, sb, sa);
    }

    // ---- epilogue: O = O^T / l, query on the lane, 4 consecutive d per register group
    if (f.qrow < S) {
        const float inv = f.l_run > 0.f ? 1.f / f.l_run : 0.f;
        __bf16* op = O + ((long)b * S + f.qrow) * ld_o + (long)h * D;
#pragma unroll
        for (int dt = 0; dt < 2; ++dt)
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                u16x4 t = {f2bf(f.o[dt][4 * i] * inv), f2bf(f.o[dt][4 * i + 1] * inv),
                           f2bf(f.o[dt][4 * i + 2] * inv), f2bf(f.o[dt][4 * i + 3] * inv)};
                *reinterpret_cast<u16x4*>(op + dt * 32 + 8 * i + 4 * f.hh) = t;
            }
        if (f.hh == 0) LSE[((long)b * H + h) * S + f.qrow] = (f.l_run > 0.f) ? f.m_run + __log2f(f.l_run) : INFINITY;
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

template <bool C>
static void fwd_v3_launch(const FaArgs& a, hipStream_t s) {
    const int nqb = (a.S + 127) / 128;
    fa_fwd_v3_kernel<C><<<nqb * a.B * a.H, 256, fa_fwd_lds_bytes(64), s>>>(
        a.q, a.k, a.v, a.ld_q, a.ld_kv, a.o, a.ld_o, a.lse, a.B, a.H, a.Hkv, a.S, a.scale * LOG2E, fa_group(a.B * a.H));
}

// v3 is opt-in (BPE_FA_FWD_V3=1): at 184 VGPRs it runs 2 waves per SIMD against 3 for fa_fwd_kernel, and
// measured 0.397 vs 0.370 ms at GPT-2 B 128 without RoPE (docs/performance.md, attention section)
static bool fwd_v3_enabled() {
    static const bool on = [] {
        const char* e = getenv("BPE_FA_FWD_V3");
        return e && e[0] == '1';
    }();
    return on;
}

void launch_fa_fwd(const FaArgs& a, hipStream_t s) {
    if (launch_fa_fwd_v4(a, s)) return;  // D = 64 without in-kernel RoPE (flash_attn_fwd_v4.hip)
    // rope 2 = Q / K already rotated: no RoPE inside the kernel
    if (a.D == 64 && a.rope != 1 && fwd_v3_enabled()) {
        if (a.causal) fwd_v3_launch<true>(a, s); else fwd_v3_launch<false>(a, s);
        if (a.dq_acc != nullptr)  // v3 has no zeroing epilogue
            (void)hipMemsetAsync(a.dq_acc, 0, (size_t)a.B * ((a.S + 63) & ~63) * a.H * a.D * sizeof(float), s);
        return;
    }
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
