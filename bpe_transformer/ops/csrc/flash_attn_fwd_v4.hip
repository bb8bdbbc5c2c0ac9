// Flash attention forward v4 (D = 64, Q / K pre-rotated or no RoPE), gfx950 (MI355X).
//
// Parity target: reference contracts K7/K9/K10 (`tests/adapters.py:92-184`), as fa_fwd_kernel.
//
// Same geometry as fa_fwd_kernel (4 waves x 32 queries, swapped S^T = K.Q^T with the query on the lane,
// register-staged double-buffered K / V, one barrier per 64-key tile, deferred rescale), restructured for the
// VALU budget, which is what bounds D = 64 (a 32 x 64 score tile per wave costs 16 MFMAs but ~1000 cycles of
// VALU in fa_fwd_kernel: per score a subtract, an exponential, a row-sum add, plus zeroing moves):
//   * the running max is folded into the S accumulator's starting value (guide: "row constants as the initial
//     accumulator"; the query is the lane, so it is one broadcast tuple): S' = K.(cQ)^T - m comes out of the
//     MFMA ready for P = exp2(S'), no subtraction.  Only the rare rescale (a tile max more than 8 above m, or
//     the first tile) subtracts, and then moves m and the tuple;
//   * the row sum l is an MFMA: ones^T . P^T (a constant bf16 1.0 A operand, the same P^T fragments as P.V),
//     accumulated -- and rescaled -- like O.  It sums the bf16-rounded P that O sums, and the 33 adds + the
//     cross-lane exchange per tile leave the VALU for the matrix pipe, which has room;
//   * K / V rows past the sequence end are loaded clamped (valid rows) instead of zero-filled behind a branch:
//     their scores are masked to -inf, so P = 0 there; no zeroing moves, no branch around the loads.
#include "fa_common.h"
#include "kernels.h"

#include <cstdlib>

namespace bpe {
namespace fa {
namespace v4 {

constexpr int D = 64, RB = 128, TILE = 64 * RB, KS = 4, SPT = 2;  // SPT: 16-byte chunks per thread and tensor
constexpr float THR = 8.0f;                                        // deferred-rescale threshold (log2 units)
constexpr float TSUM = 256.0f;                                     // 2^THR: the MAXLESS form's P-sum threshold

template <bool CAUSAL, int OCC = 2, bool DMA = false, bool MAXLESS = false>
__global__ void __launch_bounds__(256, OCC)
fa_fwd_v4_kernel(const __bf16* __restrict__ Q, const __bf16* __restrict__ K, const __bf16* __restrict__ Vv,
                 long ld_q, long ld_kv, __bf16* __restrict__ O, long ld_o, float* __restrict__ LSE, int B, int H,
                 int Hkv, int S, float scale_log2, int group, float* __restrict__ DQZ) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    char* Ks = smem;             // [2][64][128 B]
    char* Vs = smem + 2 * TILE;  // [2][64][128 B]
    const int tid = threadIdx.x, w = tid >> 6, l = tid & 63, l31 = l & 31, hh = l >> 5;
    const int nqb = (S + 127) / 128;
    int qrank, bh;
    grouped_order((int)blockIdx.x, nqb, B * H, group, qrank, bh);
    const int qb = nqb - 1 - qrank;  // heaviest (last) query blocks first
    const int b = bh / H, h = bh % H, hk = h / (H / Hkv);
    const int q0 = qb * 128, qw0 = q0 + 32 * w, qrow = qw0 + l31;

    // Q fragments (B operand of S^T = K.Q^T), softmax scale * log2(e) folded in; rows past the end clamped
    bf16x8 qf[KS];
    {
        const long qpos = min(qrow, S - 1);
        const __bf16* qp = Q + ((long)b * S + qpos) * ld_q + (long)h * D;
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) {
            float x[8];
            unpack8(*reinterpret_cast<const u16x8*>(qp + 16 * ks + 8 * hh), x);
            qf[ks] = __builtin_bit_cast(bf16x8, pack8(x, scale_log2));
        }
    }
    const int n_end = CAUSAL ? min(S, q0 + 128) : S;
    const int ntiles = (n_end + 63) / 64;
    const __bf16* kbase = K + (long)b * S * ld_kv + (long)hk * D;
    const __bf16* vbase = Vv + (long)b * S * ld_kv + (long)hk * D;
    u16x8 kreg[SPT], vreg[SPT];
    auto load_tile = [&](int t) {
#pragma unroll
        for (int i = 0; i < SPT; ++i) {
            const int e = tid + 256 * i, row = e >> 3, c = e & 7;
            const long key = min(t * 64 + row, S - 1);
            kreg[i] = *reinterpret_cast<const u16x8*>(kbase + key * ld_kv + c * 8);
            vreg[i] = *reinterpret_cast<const u16x8*>(vbase + key * ld_kv + c * 8);
        }
    };
    auto write_tile = [&](int buf) {
#pragma unroll
        for (int i = 0; i < SPT; ++i) {
            const int e = tid + 256 * i, row = e >> 3, c = e & 7;
            *reinterpret_cast<u16x8*>(Ks + buf * TILE + swz<RB>(row, c)) = kreg[i];
            *reinterpret_cast<u16x8*>(Vs + buf * TILE + swz<RB>(row, c)) = vreg[i];
        }
    };

    f32x16 o[2], lacc, nm;  // O^T (d rows, query lane), row sums (every register), -m (S accumulator start)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
        o[0][r] = 0.f;
        o[1][r] = 0.f;
        lacc[r] = 0.f;
        nm[r] = 0.f;
    }
    float m_run = 0.f, lsum_t = 0.f;  // lsum_t: the row sum (MAXLESS)
    bf16x8 ones;
#pragma unroll
    for (int j = 0; j < 8; ++j) ones[j] = (__bf16)1.0f;

    const int trow = 4 * hh + ((l & 15) >> 2);
    const int tcol = 16 * ((l >> 4) & 1) + 4 * (l & 3);

    // DMA: K / V tiles by LDS-DMA through buffer resources (fa_common.h dma_tile64_buf; rows past the end read as 0
    // and are masked below)
    const int wu = __builtin_amdgcn_readfirstlane(w);
    // K and V share the row stride: one set of lane offsets and one extent serve both buffer resources
    const int hbytes = head_bytes(ld_kv, S, D);
    const DmaVoff<4> vo = dma_voff<4>(ld_kv, wu, l);
    if constexpr (DMA) {
        dma_tile64_buf(kbase, hbytes, vo, 0, ld_kv, Ks, wu);
        dma_tile64_buf(vbase, hbytes, vo, 0, ld_kv, Vs, wu);
    } else {
        load_tile(0);
        write_tile(0);
    }
    __syncthreads();
    for (int t = 0; t < ntiles; ++t) {
        const int cur = t & 1, n0 = t * 64;
        if (t + 1 < ntiles) {
            if constexpr (DMA) {  // buffer cur ^ 1 was last read in tile t - 1, before its closing barrier
                dma_tile64_buf(kbase, hbytes, vo, n0 + 64, ld_kv, Ks + (cur ^ 1) * TILE, wu);
                dma_tile64_buf(vbase, hbytes, vo, n0 + 64, ld_kv, Vs + (cur ^ 1) * TILE, wu);
            } else {
                load_tile(t + 1);
            }
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
            if constexpr (MAXLESS) {
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
            } else {
            float mt = s[0][0];
#pragma unroll
            for (int kt = 0; kt < 2; ++kt)
#pragma unroll
                for (int r = 0; r < 16; ++r) mt = fmaxf(mt, s[kt][r]);
            mt = fmaxf(mt, __shfl_xor(mt, 32, 64));
            // rescale (rare): the first tile sets m; later, a tile whose max exceeds m by more than THR moves it.
            // Every P of this tile is formed after the decision (guide T13 hazard).
            const bool grow = t == 0 || mt > THR;
            if (!__all(!grow)) {
                const float d = grow ? mt : 0.f;
                const float alpha = t == 0 ? 0.f : fast_exp2(-d);  // tile 0: O, l are still zero
                m_run += d;
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    o[0][r] *= alpha;
                    o[1][r] *= alpha;
                    lacc[r] *= alpha;
                    nm[r] = -m_run;
                    s[0][r] -= d;
                    s[1][r] -= d;
                }
            }
            bf16x8 pf[4];  // P^T fragments: k-step kk = (key half kt, 16-key step ss) in the permuted k order
#pragma unroll
            for (int kk = 0; kk < 4; ++kk) {
                const int kt = kk >> 1, ss = kk & 1;
#pragma unroll
                for (int j = 0; j < 8; ++j) pf[kk][j] = (__bf16)fast_exp2(s[kt][8 * ss + j]);
            }
#pragma unroll
            for (int kk = 0; kk < 4; ++kk) {
                const int kb = (kk >> 1) * 32 + 16 * (kk & 1);
#pragma unroll
                for (int dt = 0; dt < 2; ++dt)
                    o[dt] = mfma(lds_tr_pair(Vc, tr_off<RB>(kb + trow, dt * 32 + tcol),
                                             tr_off<RB>(kb + 8 + trow, dt * 32 + tcol)),
                                 pf[kk], o[dt]);
                lacc = mfma(ones, pf[kk], lacc);
            }
            }
        }
        if (!DMA && t + 1 < ntiles) write_tile(cur ^ 1);
        __syncthreads();
    }

    // ---- epilogue: O = O^T / l (query on the lane, 4 consecutive d per register group), LSE = m + log2 l
    if (qrow < S) {
        const float lsum = MAXLESS ? lsum_t : lacc[0];
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

// ---------------------------------------------------------------------------------------------------------
// v5: the v4 math on the ping-pong schedule of the split backward kernels (flash_attn_bwd_split.hip): 8 waves in
// two groups of four, waves w and w + 4 (one SIMD) owning adjacent 32-query blocks (queries q0 + 64 (w & 3) +
// 32 (w >> 2); a workgroup covers 256 queries), group 1 one barrier interval behind group 0.  Per 64-key tile t:
//   M(t): O^T += V^T.P^T and l += ones.P^T of tile t - 1 (12 MFMAs; operands from V(t - 1)), then
//         S'^T = K.(cQ)^T - m of tile t (8 MFMAs, K rows read at the top)
//   V(t): mask, tile max, the rare rescale, P^T = exp2(S'^T) in bf16, the V^T reads for M(t + 1), and staging.
// Three K / V buffers: tile t + 2 is written in V(t) into buffer (t + 2) % 3 (group g its rows [32 g, +32), from
// registers loaded in V(t - 1)); that buffer's tile t - 1 was last read in V(t - 1), which group 1 runs in the
// interval before group 0's V(t), and tile t + 2 is first read in M(t + 2), two intervals after group 1's write.
constexpr int PPW = 8;

__device__ __forceinline__ void pbar() {
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
}

template <bool CAUSAL>
__global__ void __launch_bounds__(PPW * 64, 1)
fa_fwd_pp_kernel(const __bf16* __restrict__ Q, const __bf16* __restrict__ K, const __bf16* __restrict__ Vv,
                 long ld_q, long ld_kv, __bf16* __restrict__ O, long ld_o, float* __restrict__ LSE, int B, int H,
                 int Hkv, int S, float scale_log2, int group, float* __restrict__ DQZ) {
    constexpr int QB = 32 * PPW;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    char* Ks = smem;             // [3][64][128 B]
    char* Vs = smem + 3 * TILE;  // [3][64][128 B]
    const int tid = threadIdx.x, l = tid & 63, l31 = l & 31, hh = l >> 5;
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int g = w >> 2, wl = w & 3, gt = tid & 255;
    const int nqb = (S + QB - 1) / QB;
    int qrank, bh;
    grouped_order((int)blockIdx.x, nqb, B * H, group, qrank, bh);
    const int qb = nqb - 1 - qrank;
    const int b = bh / H, h = bh % H, hk = h / (H / Hkv);
    const int q0 = qb * QB, qw0 = q0 + 64 * wl + 32 * g, qrow = qw0 + l31;

    bf16x8 qf[KS];
    {
        const long qpos = min(qrow, S - 1);
        const __bf16* qp = Q + ((long)b * S + qpos) * ld_q + (long)h * D;
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) {
            float x[8];
            unpack8(*reinterpret_cast<const u16x8*>(qp + 16 * ks + 8 * hh), x);
            qf[ks] = __builtin_bit_cast(bf16x8, pack8(x, scale_log2));
        }
    }
    const int n_end = CAUSAL ? min(S, q0 + QB) : S;
    const int ntiles = (n_end + 63) / 64;
    const __bf16* kbase = K + (long)b * S * ld_kv + (long)hk * D;
    const __bf16* vbase = Vv + (long)b * S * ld_kv + (long)hk * D;
    const int srow = 32 * g + (gt >> 3), sc = gt & 7;
    u16x8 kreg, vreg;
    auto load_tile = [&](int t) {
        const long key = min(t * 64 + srow, S - 1);
        kreg = *reinterpret_cast<const u16x8*>(kbase + key * ld_kv + sc * 8);
        vreg = *reinterpret_cast<const u16x8*>(vbase + key * ld_kv + sc * 8);
    };
    auto write_tile = [&](int t) {
        const int buf = t % 3;
        *reinterpret_cast<u16x8*>(Ks + buf * TILE + swz<RB>(srow, sc)) = kreg;
        *reinterpret_cast<u16x8*>(Vs + buf * TILE + swz<RB>(srow, sc)) = vreg;
    };

    f32x16 o[2], lacc, nm;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
        o[0][r] = 0.f;
        o[1][r] = 0.f;
        lacc[r] = 0.f;
        nm[r] = 0.f;
    }
    float m_run = 0.f;
    bf16x8 ones;
#pragma unroll
    for (int j = 0; j < 8; ++j) ones[j] = (__bf16)1.0f;
    const int trow = 4 * hh + ((l & 15) >> 2);
    const int tcol = 16 * ((l >> 4) & 1) + 4 * (l & 3);

    // prologue: tiles 0 and 1 staged and visible, tile 2 in registers
    load_tile(0);
    write_tile(0);
    if (ntiles > 1) {
        load_tile(1);
        write_tile(1);
    }
    if (ntiles > 2) load_tile(2);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    pbar();
    if (g == 1) pbar();

    f32x16 s[2];
    bf16x8 pf[4];       // bf16 P^T of the previous tile, k-steps kk
    bf16x8 vt[4][2];    // its V^T fragments [kk][dt]
    bool prev_active = false;
    for (int t = 0; t <= ntiles; ++t) {
        const int n0 = t * 64;
        const bool active = t < ntiles && (!CAUSAL || n0 <= qw0 + 31);
        // ---------------- M(t)
        if (prev_active) {
#pragma unroll
            for (int kk = 0; kk < 4; ++kk) {
#pragma unroll
                for (int dt = 0; dt < 2; ++dt) o[dt] = mfma(vt[kk][dt], pf[kk], o[dt]);
                lacc = mfma(ones, pf[kk], lacc);
            }
        }
        __builtin_amdgcn_sched_barrier(0);
        if (active) {
            const char* Kc = Ks + (t % 3) * TILE;
#pragma unroll
            for (int kt = 0; kt < 2; ++kt) {
                s[kt] = nm;
#pragma unroll
                for (int ks = 0; ks < KS; ++ks)
                    s[kt] = mfma(lds_row16(Kc, swz<RB>(kt * 32 + l31, 2 * ks + hh)), qf[ks], s[kt]);
            }
        }
        pbar();
        if (t == ntiles) break;
        // ---------------- V(t)
        if (active) {
            char* Vc = Vs + (t % 3) * TILE;
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
            // O and l hold tiles < t only (tile t - 1 was added in M(t)): a rescale here covers exactly them
            const bool grow = t == 0 || mt > THR;
            if (!__all(!grow)) {
                const float d = grow ? mt : 0.f;
                const float alpha = t == 0 ? 0.f : fast_exp2(-d);
                m_run += d;
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    o[0][r] *= alpha;
                    o[1][r] *= alpha;
                    lacc[r] *= alpha;
                    nm[r] = -m_run;
                    s[0][r] -= d;
                    s[1][r] -= d;
                }
            }
#pragma unroll
            for (int kk = 0; kk < 4; ++kk) {
                const int kt = kk >> 1, ss = kk & 1;
#pragma unroll
                for (int j = 0; j < 8; ++j) pf[kk][j] = (__bf16)fast_exp2(s[kt][8 * ss + j]);
                const int kb = kt * 32 + 16 * ss;
#pragma unroll
                for (int dt = 0; dt < 2; ++dt)
                    vt[kk][dt] = lds_tr_pair(Vc, tr_off<RB>(kb + trow, dt * 32 + tcol),
                                             tr_off<RB>(kb + 8 + trow, dt * 32 + tcol));
            }
        }
        prev_active = active;
        if (t + 2 < ntiles) {
            write_tile(t + 2);
            if (t + 3 < ntiles) load_tile(t + 3);
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        pbar();
    }
    if (g == 0) pbar();

    if (qrow < S) {
        const float lsum = lacc[0];
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
    if (DQZ != nullptr) {
        constexpr int C4 = D / 4;
        const int spad = (S + 63) & ~63;
        const int rows = min(QB, spad - q0);
        float* zb = DQZ + ((long)b * spad + q0) * ((long)H * D) + (long)h * D;
        for (int e = tid; e < rows * C4; e += PPW * 64) {
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

// forward version for D = 64 without in-kernel RoPE: 8 (default: this file's kernel at 3 waves per SIMD, K / V
// staged by LDS-DMA, no tile max on the common path), 7 (with the tile max), 6 (register staging), 4 (register
// staging at 2 waves per SIMD) or 2 (fa_fwd_kernel); BPE_FA_FWD sets the initial value, fa_fwd_config changes it at
// run time (A/B, tests).  Same box, op-level: GPT-2 B 128 0.342 / 0.356 / 0.362 ms for 7 / 6 / 4, Llama GQA
// (8, 2048, 32, 4) 0.178 / 0.196 / 0.193 ms (profiles/bench/ab_attn_fwd_dma.log); 8 vs 7 0.314 vs 0.324 ms
// (ab_attn_mask_maxless.log).
static int g_fwd_ver = -1;

// 2 (fa_fwd_kernel), 4 (fa_fwd_v4_kernel), 5 (fa_fwd_pp_kernel), 6 (fa_fwd_v4_kernel at 3 waves per SIMD: 162-168
// VGPRs, no spills), 7 (6 with LDS-DMA staging) or 8 (7 with the P-sum rescale test, MAXLESS; the default)
static int fwd_ver_code(int v) { return (v == 2 || v == 4 || v == 5 || v == 6 || v == 7) ? v : 8; }

int fa_fwd_config(int ver) {
    if (g_fwd_ver < 0) {
        const char* e = getenv("BPE_FA_FWD");
        g_fwd_ver = fwd_ver_code(e ? atoi(e) : 8);
    }
    if (ver > 0) g_fwd_ver = fwd_ver_code(ver);
    return g_fwd_ver;
}

bool launch_fa_fwd_v4(const FaArgs& a, hipStream_t s) {
    const int ver = fa_fwd_config(0);
    if (a.D != 64 || a.rope == 1 || ver == 2) return false;
    if (ver == 5) {
        const int nqb = (a.S + 32 * v4::PPW - 1) / (32 * v4::PPW);
        auto* k = a.causal ? &v4::fa_fwd_pp_kernel<true> : &v4::fa_fwd_pp_kernel<false>;
        k<<<nqb * a.B * a.H, v4::PPW * 64, 6 * v4::TILE, s>>>(a.q, a.k, a.v, a.ld_q, a.ld_kv, a.o, a.ld_o, a.lse, a.B,
                                                              a.H, a.Hkv, a.S, a.scale * LOG2E, fa_group(a.B * a.H),
                                                              a.dq_acc);
        return true;
    }
    const int nqb = (a.S + 127) / 128;
    auto* k = ver == 6   ? (a.causal ? &v4::fa_fwd_v4_kernel<true, 3> : &v4::fa_fwd_v4_kernel<false, 3>)
              : ver == 7 ? (a.causal ? &v4::fa_fwd_v4_kernel<true, 3, true> : &v4::fa_fwd_v4_kernel<false, 3, true>)
              : ver == 8 ? (a.causal ? &v4::fa_fwd_v4_kernel<true, 3, true, true>
                                     : &v4::fa_fwd_v4_kernel<false, 3, true, true>)
                         : (a.causal ? &v4::fa_fwd_v4_kernel<true> : &v4::fa_fwd_v4_kernel<false>);
    k<<<nqb * a.B * a.H, 256, 4 * v4::TILE, s>>>(a.q, a.k, a.v, a.ld_q, a.ld_kv, a.o, a.ld_o, a.lse, a.B, a.H, a.Hkv,
                                                 a.S, a.scale * LOG2E, fa_group(a.B * a.H), a.dq_acc);
    return true;
}
