// Flash attention backward, split form (D = 64 and D = 128), gfx950 (MI355X).
// build-flags: -fno-slp-vectorize   (no packed f32 VALU beside the MFMAs: ops/build.py file_flags)
//
// Parity target: the gradient of reference contracts K7/K10 (`tests/adapters.py:92-184`); checked against
// autograd of the fp32 oracle (tests/test_kernels_gpu.py).
//
// Why split: the fused backward (flash_attn_bwd.hip) owns 256 keys per workgroup and adds dQ = dS.K into an fp32
// buffer with float atomics.  At GPT-2 B 128 that is 983 MB of atomics per layer, whose chip-wide rate (1.3 TB/s,
// MI355X_MICROARCH 'Global float atomics') floors the kernel at 0.76 ms; it also needs a zeroed 402 MB fp32
// accumulator per layer, a delta pre-pass and a dQ convert pass.  Here the five products are computed by two
// kernels that each own their output, so nothing is summed across workgroups:
//
//   fa_bwd_dq_kernel   (query-major, first):  delta = rowsum(dO * O) for its queries (written for the second
//       kernel), then per 64-key tile  S^T = K.(cQ)^T - lse,  dP^T = V.dO^T - delta,  P^T = exp2(S^T),
//       dS^T = P^T * dP^T,  dQ^T += K^T.dS^T.   Q and dO are the lane-resident B operands (query on the lane),
//       pinned in registers for the whole key sweep; K / V tiles of 128 keys are staged in LDS by LDS-DMA through
//       buffer resources (fa_common.h), tile t+1 issued before tile t's MFMAs; one barrier per tile.  dS^T
//       is the B operand of the dQ^T product straight from its accumulator (guide §3).  dQ is scaled,
//       un-rotated (RoPE) and written as bf16 in the epilogue.
//   fa_bwd_dkv_kernel  (key-major):  per 64-query tile  S = Q.(cK)^T - lse,  dP = dO.V^T - delta (row constants
//       as the initial accumulators), P = exp2(S), dS = P dP,  dV^T += dO^T.P,  dK^T += Q^T.dS.  K and V are
//       the pinned B operands (key on the lane); Q / dO rows and their transposed reads come from one LDS image
//       (fa_common.h).  No dS LDS round trip, no second barrier, no atomics.
//
// c = softmax scale * log2(e) is folded into the pinned operand (Q in the dQ kernel, as in the forward; K in the
// dK/dV kernel, whose Q also feeds dK), so the only VALU between an S accumulator and its exponential is none.
// The price is the recomputation of S and dP in the dQ kernel (7 MFMA products instead of 5); in exchange the
// atomics floor, the 402 MB/layer accumulator (4.8 GB at GPT-2 B 128), the zeroing and the two side passes go.
// GQA: one dK / dV workgroup per KV head sweeps the G query heads of its group (no partials, no reduce kernel).
// With RoPE fused into the kernels (ROPE_IN: Q / K rotated on their way to LDS) the tiles are register-staged,
// 64 rows each (D = 64 only).
//
// D = 128: the same two kernels on 256-byte rows (swz<256>), 64-row tiles (LDS: 64 KiB per workgroup), K / V (dQ
// kernel) and Q / dO (dK/dV kernel) always by LDS-DMA; the pinned operands and accumulators double, so the dQ
// kernel reads its K / V fragments per k-step instead of in one batch and the dK/dV kernel (256 accumulator
// registers per lane for dK^T and dV^T alone) runs one wave per SIMD.  RoPE is applied before (fa_bwd rotates a copy
// of Q / K when the forward rotated inside its kernel).  This replaces the fused form's fp32 dQ atomics, dQ
// accumulator, delta pre-pass and convert pass for D = 128 as well, and makes it deterministic.
#include "fa_common.h"
#include "kernels.h"

#include <cstdlib>

namespace bpe {
namespace fa {
namespace split {

// 4 waves x 32 rows per workgroup, 2 workgroups per CU (2 waves per SIMD at <= 256 VGPRs)
constexpr int NW = 4;

// per head size: tile row bytes, 64-row tile bytes, 16-deep k-steps over d, 32-wide d tiles of an accumulator, and
// staged 16-byte chunks per thread and tensor for one register-staged 64-row tile
template <int D>
struct Geo {
    static_assert(D == 64 || D == 128, "split backward: D = 64 or 128");
    static constexpr int RB = 2 * D, TILE = 64 * RB, KS = D / 16, ND = D / 32, CPT = 4 * RB / (NW * 64);
};

// Per-workgroup s_memtime stamps (a diagnostic variant build: ops.build --variant stamps -D BPE_FA_STAMPS): slot 0
// entry, 1 after the prologue barrier, 2 at the start of the last tile, 3 after the tile loop, 5 the tile count; rows 0.. the dQ kernel's workgroups,
// rows 32768.. the dK/dV kernel's; read with ops.fa_stamps().  The normal build compiles them out.
#ifdef BPE_FA_STAMPS
__device__ long long g_stamps[65536 * 8];
#define FA_STAMP(base, i, v)                                                                         \
    if (threadIdx.x == 0) {                                                                          \
        g_stamps[((base) + (long)(blockIdx.x & 32767)) * 8 + (i)] = __builtin_amdgcn_s_memtime();   \
        if ((i) == 3) g_stamps[((base) + (long)(blockIdx.x & 32767)) * 8 + 5] = (v);               \
    }
#else
#define FA_STAMP(base, i, v)
#endif

// (D = 128: 2 waves per SIMD with 7-9 VGPRs spilled measured 0.44 / 0.71 ms against 0.49 / 0.80 ms at one wave
// per SIMD without spills, B 4 S 2048 H 16 / GQA 32:8, profiles/bench/attn_d128_split_r4.log)
template <int D, bool CAUSAL, bool ROPE, bool ROPE_IN>
__global__ void __launch_bounds__(NW * 64, 2)
fa_bwd_dq_kernel(const __bf16* __restrict__ Q, const __bf16* __restrict__ K, const __bf16* __restrict__ Vv,
                 long ld_q, long ld_kv, const __bf16* __restrict__ O, long ld_o, const __bf16* __restrict__ dO,
                 long ld_do, const float* __restrict__ LSE, float* __restrict__ DELTA, __bf16* __restrict__ dQ,
                 long ld_dq, const float* __restrict__ cosT, const float* __restrict__ sinT, int B, int H, int Hkv,
                 int S, float scale_log2, float scale, int group) {
    using G = Geo<D>;
    constexpr int RB = G::RB, TILE = G::TILE, KS = G::KS, ND = G::ND, CPT = G::CPT;
    static_assert(D == 64 || !ROPE_IN, "D = 128: Q / K are rotated before the kernels");
    constexpr int NT = NW * 64, QB = 32 * NW;
    // keys per K / V tile (one barrier each): 128 with LDS-DMA staging (two 64-row images side by side), 64 with
    // register staging (ROPE_IN: K is rotated on its way to LDS) and at D = 128 (64 KiB of LDS already)
    constexpr bool DM = !ROPE_IN;
    constexpr int KT = (DM && D == 64) ? 128 : 64, NSUB = KT / 64, BUF = NSUB * TILE;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    char* Ks = smem;            // [2][KT keys][RB]  (roped K)
    char* Vs = smem + 2 * BUF;  // [2][KT keys][RB]

    const int tid = threadIdx.x, w = tid >> 6, l = tid & 63, l31 = l & 31, hh = l >> 5;
    prologue_prio_begin();
    FA_STAMP(0, 0, 0);
    const int nqb = (S + QB - 1) / QB;
    int rank, bh;
    grouped_order((int)blockIdx.x, nqb, B * H, group, rank, bh);
    const int qblk = CAUSAL ? nqb - 1 - rank : rank;  // causal: the last (heaviest) query blocks first
    const int b = bh / H, h = bh % H, hk = h / (H / Hkv);
    const int q0 = qblk * QB, qw = q0 + 32 * w, q = qw + l31;
    const bool q_ok = q < S;
    const long qc = q_ok ? q : S - 1;
    const long qrow = (long)b * S + qc;

    // ---- prologue: every load issued before any of them is waited for -- the pinned Q / dO rows, the O rows of
    // delta, the LSE and K / V tile 0 -- so the prologue costs one memory round trip, not three (per-workgroup
    // s_memtime stamps at GPT-2 B 128: ~8k of a ~42k-cycle workgroup went to the serial form)
    u16x8 tqr[KS], tgr[KS], tor[KS];
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
        const int d0 = 16 * ks + 8 * hh;
        tqr[ks] = *reinterpret_cast<const u16x8*>(Q + qrow * ld_q + (long)h * D + d0);
        tgr[ks] = *reinterpret_cast<const u16x8*>(dO + qrow * ld_do + (long)h * D + d0);
        tor[ks] = *reinterpret_cast<const u16x8*>(O + qrow * ld_o + (long)h * D + d0);
    }
    const float lse = LSE[((long)b * H + h) * S + qc];

    const int kend = CAUSAL ? min(S, q0 + QB) : S;
    const int nkt = (kend + KT - 1) / KT;
    const __bf16* kb = K + (long)b * S * ld_kv + (long)hk * D;
    const __bf16* vb = Vv + (long)b * S * ld_kv + (long)hk * D;
    u16x8 kreg[CPT], vreg[CPT];
    auto load_tile = [&](int it) {
#pragma unroll
        for (int i = 0; i < CPT; ++i) {
            const int e = tid + NT * i, r = (unsigned)e / (RB / 16), c = (unsigned)e % (RB / 16);
            const long kk = min(it * 64 + r, S - 1);  // rows past the end: valid memory, zeroed at the write
            kreg[i] = *reinterpret_cast<const u16x8*>(kb + kk * ld_kv + c * 8);
            vreg[i] = *reinterpret_cast<const u16x8*>(vb + kk * ld_kv + c * 8);
        }
    };
    auto write_tile = [&](int it, int buf) {
#pragma unroll
        for (int i = 0; i < CPT; ++i) {
            const int e = tid + NT * i, r = (unsigned)e / (RB / 16), c = (unsigned)e % (RB / 16);
            const bool ok = it * 64 + r < S;
            u16x8 kv = ok ? kreg[i] : u16x8{0, 0, 0, 0, 0, 0, 0, 0};
            const u16x8 vv = ok ? vreg[i] : u16x8{0, 0, 0, 0, 0, 0, 0, 0};
            if (ROPE_IN) {
                const long kk = min(it * 64 + r, S - 1);
                kv = rope_u16x8(kv, cosT + kk * (D / 2) + c * 4, sinT + kk * (D / 2) + c * 4, 1.f);
            }
            *reinterpret_cast<u16x8*>(Ks + buf * TILE + swz<RB>(r, c)) = kv;
            *reinterpret_cast<u16x8*>(Vs + buf * TILE + swz<RB>(r, c)) = vv;
        }
    };

    // DM: K / V tiles by LDS-DMA through buffer resources (no staging registers, no per-tile address VALU; rows
    // past the end read as 0 and are masked below)
    const int wu = __builtin_amdgcn_readfirstlane(w);
    const int hbytes = head_bytes(ld_kv, S, D);
    const DmaVoff<NW, RB> kvo = dma_voff<NW, RB>(ld_kv, wu, l);
    if constexpr (DM) {
#pragma unroll
        for (int sb = 0; sb < NSUB; ++sb) {
            dma_tile64_buf(kb, hbytes, kvo, 64 * sb, ld_kv, Ks + sb * TILE, wu);
            dma_tile64_buf(vb, hbytes, kvo, 64 * sb, ld_kv, Vs + sb * TILE, wu);
        }
    } else {
        load_tile(0);
    }

    // ---- pinned B operands (query on the lane, d = 16 ks + 8 hh + j) and delta = rowsum(dO * O)
    bf16x8 qf[KS], of[KS];
    float dsum = 0.f;
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
        const int d0 = 16 * ks + 8 * hh;
        u16x8 tq = tqr[ks];
        // softmax scale * log2(e) folded into the pinned Q (as the forward does): S^T comes out in log2 units
        if (ROPE_IN) {
            tq = rope_u16x8(tq, cosT + qc * (D / 2) + d0 / 2, sinT + qc * (D / 2) + d0 / 2, scale_log2);
        } else {
            float x[8];
            unpack8(tq, x);
            tq = pack8(x, scale_log2);
        }
        qf[ks] = __builtin_bit_cast(bf16x8, tq);
#pragma unroll
        for (int i = 0; i < 8; ++i) dsum += bf2f(tgr[ks][i]) * bf2f(tor[ks][i]);
        of[ks] = __builtin_bit_cast(bf16x8, tgr[ks]);
    }
    dsum += __shfl_xor(dsum, 32, 64);
    // (delta is stored for the dK/dV kernel in the epilogue, not here: a store before the prologue barrier, whose
    // vmcnt(0) also waits for it, put its write-acknowledge latency into the prologue)
    // row constants as the initial accumulators (query = lane): S^T starts at -lse, so P = exp2(S^T) with no
    // VALU before the exponential (-inf for empty / pad rows: P = 0); dP^T starts at -delta
    const float nl = (q_ok && lse < INFINITY) ? -lse : -INFINITY;
    f32x16 ns, nd;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
        ns[r] = nl;
        nd[r] = -dsum;
    }

    f32x16 acc[ND];
#pragma unroll
    for (int dt = 0; dt < ND; ++dt)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[dt][r] = 0.f;

    if constexpr (!DM) write_tile(0, 0);
    __syncthreads();
    prologue_prio_end();
    FA_STAMP(0, 1, 0);

    const int trow = 4 * hh + ((l & 15) >> 2);          // tr-read row inside a 16-key step
    const int tcol = 16 * ((l >> 4) & 1) + 4 * (l & 3);  // tr-read column inside a 32-wide d tile
    for (int it = 0; it < nkt; ++it) {
        const int cur = it & 1, k0 = it * KT;
        if (it + 1 == nkt) FA_STAMP(0, 2, 0);
        // the current and next buffers as __restrict__ parameters (see fa_bwd_dkv_kernel): no DMA drain mid-tile
        auto body = [&](char* __restrict__ Kc, const char* __restrict__ Vc, char* __restrict__ Kn,
                        char* __restrict__ Vn) {
            if (it + 1 < nkt) {
                if constexpr (DM) {  // buffer cur ^ 1 was last read in iteration it - 1, before its closing barrier
#pragma unroll
                    for (int sb = 0; sb < NSUB; ++sb) {
                        dma_tile64_buf(kb, hbytes, kvo, k0 + KT + 64 * sb, ld_kv, Kn + sb * TILE, wu);
                        dma_tile64_buf(vb, hbytes, kvo, k0 + KT + 64 * sb, ld_kv, Vn + sb * TILE, wu);
                    }
                } else {
                    load_tile(it + 1);
                }
            }
            if (!CAUSAL || k0 <= qw + 31) {
#pragma unroll
                for (int kq = 0; kq < KT / 32; ++kq) {
                    if (CAUSAL && k0 + 32 * kq > qw + 31) break;  // this 32-key step is past every query of the wave
                    // masked only where a key of the step can pass a query of the wave (the diagonal 32 x 32 step)
                    // or the sequence end: the other steps of a diagonal tile take the unmasked path
                    const bool need_mask = (CAUSAL && k0 + 32 * kq + 31 > qw) || (k0 + 32 * kq + 32 > S);
                    // step kq: image kq / 2 of the tile, its 32-key half kh
                    char* Kh = Kc + (kq >> 1) * TILE;
                    const char* Vh = Vc + (kq >> 1) * TILE;
                    const int kh = kq & 1;
                    f32x16 sp, dp;
                    if constexpr (D == 64) {
                        sp = ns;
                        dp = nd;
                    } else {  // D = 128: no 32 registers held for the row constants
#pragma unroll
                        for (int r = 0; r < 16; ++r) {
                            sp[r] = nl;
                            dp[r] = -dsum;
                        }
                    }
                    // every operand read of the step is issued ahead of its MFMAs: the K / V rows before the S / dP
                    // chains, the transposed K fragments of the dQ products before the softmax VALU, so their LDS
                    // latency is paid once per batch (hipcc's own schedule waits lgkmcnt(0) before every MFMA pair).
                    // D = 128: the K / V rows per k-step (a batch would hold 64 more registers)
                    bf16x8 tk[2][ND];  // the transposed K fragments of the dQ products (s, dt)
                    if constexpr (D == 64) {
                        bf16x8 fk[KS], fv[KS];
#pragma unroll
                        for (int ks = 0; ks < KS; ++ks) {
                            const int koff = swz<RB>(32 * kh + l31, 2 * ks + hh);
                            fk[ks] = lds_row16(Kh, koff);
                            fv[ks] = lds_row16(Vh, koff);
                        }
                        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
                        for (int ks = 0; ks < KS; ++ks) {
                            sp = mfma(fk[ks], qf[ks], sp);
                            dp = mfma(fv[ks], of[ks], dp);
                        }
                    } else {
#pragma unroll
                        for (int ks = 0; ks < KS; ++ks) {
                            const int koff = swz<RB>(32 * kh + l31, 2 * ks + hh);
                            sp = mfma(lds_row16(Kh, koff), qf[ks], sp);
                            dp = mfma(lds_row16(Vh, koff), of[ks], dp);
                        }
                    }
                    __builtin_amdgcn_sched_barrier(0);
                    if constexpr (D == 64) {  // (D = 128 reads them per k-step of the dQ products)
#pragma unroll
                        for (int s = 0; s < 2; ++s)
#pragma unroll
                            for (int dt = 0; dt < ND; ++dt) {
                                const int kr = 32 * kh + 16 * s;
                                tk[s][dt] = lds_tr_pair(Kh, tr_off<RB>(kr + trow, 32 * dt + tcol),
                                                        tr_off<RB>(kr + 8 + trow, 32 * dt + tcol));
                            }
                    }
                    __builtin_amdgcn_sched_barrier(0);
                    // P^T = exp2(S^T c - lse), dS^T = P^T (dP^T - delta); key = row of the accumulator, query = lane
                    if (need_mask) {
                        // key k0 + 32 kq + acc_row(r, hh) is valid iff <= min(q, S - 1) (causal) / S - 1: the
                        // per-lane limit against the register's compile-time row offset, one compare per score
                        const int klim = (CAUSAL ? min(q, S - 1) : S - 1) - k0 - 32 * kq - 4 * hh;
#pragma unroll
                        for (int r = 0; r < 16; ++r) {
                            const float p = fast_exp2(sp[r]);
                            const bool ok = (r & 3) + 8 * (r >> 2) <= klim;
                            dp[r] = ok ? p * dp[r] : 0.f;
                        }
                    } else {
#pragma unroll
                        for (int r = 0; r < 16; ++r) dp[r] = fast_exp2(sp[r]) * dp[r];
                    }
                    // dQ^T += K^T.dS^T: registers 8s..8s+7 are k-step s (keys 16 s ..) in the MFMA's permuted order
#pragma unroll
                    for (int s = 0; s < 2; ++s) {
                        bf16x8 db;
#pragma unroll
                        for (int j = 0; j < 8; ++j) db[j] = (__bf16)dp[8 * s + j];
                        const int kr = 32 * kh + 16 * s;
                        if constexpr (D == 128) {
#pragma unroll
                            for (int dt = 0; dt < ND; ++dt)
                                tk[s][dt] = lds_tr_pair(Kh, tr_off<RB>(kr + trow, 32 * dt + tcol),
                                                        tr_off<RB>(kr + 8 + trow, 32 * dt + tcol));
                        }
#pragma unroll
                        for (int dt = 0; dt < ND; ++dt) acc[dt] = mfma(tk[s][dt], db, acc[dt]);
                    }
                }
            }
        };
        body(Ks + cur * BUF, Vs + cur * BUF, Ks + (cur ^ 1) * BUF, Vs + (cur ^ 1) * BUF);
        if (it + 1 < nkt) {  // (no barrier after the last tile: a wave done with the diagonal leaves early)
            if (!DM) write_tile(it + 1, cur ^ 1);
            __syncthreads();
        }
    }

    FA_STAMP(0, 3, nkt);
    // ---- epilogue: delta for the dK/dV kernel; dQ = scale * R(-pos) dQ^T (query on the lane, 4 consecutive d per
    // register group)
    if (q_ok && hh == 0) DELTA[((long)b * H + h) * S + q] = dsum;
    if (q_ok) {
        __bf16* dqp = dQ + ((long)b * S + q) * ld_dq + (long)h * D;
#pragma unroll
        for (int dt = 0; dt < ND; ++dt)
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int d0 = 32 * dt + 8 * i + 4 * hh;
                float x[4] = {acc[dt][4 * i] * scale, acc[dt][4 * i + 1] * scale, acc[dt][4 * i + 2] * scale,
                              acc[dt][4 * i + 3] * scale};
                if (ROPE) {
#pragma unroll
                    for (int pr = 0; pr < 2; ++pr) {
                        const float c = cosT[(long)q * (D / 2) + d0 / 2 + pr];
                        const float sn = sinT[(long)q * (D / 2) + d0 / 2 + pr];
                        const float a = x[2 * pr], bb = x[2 * pr + 1];
                        x[2 * pr] = a * c + bb * sn;
                        x[2 * pr + 1] = -a * sn + bb * c;
                    }
                }
                *reinterpret_cast<u16x4*>(dqp + d0) = u16x4{f2bf(x[0]), f2bf(x[1]), f2bf(x[2]), f2bf(x[3])};
            }
    }
}

template <int D, bool CAUSAL, bool ROPE, bool ROPE_IN>
__global__ void __launch_bounds__(NW * 64, D == 64 ? 2 : 1)
fa_bwd_dkv_kernel(const __bf16* __restrict__ Q, const __bf16* __restrict__ K, const __bf16* __restrict__ Vv,
                  long ld_q, long ld_kv, const __bf16* __restrict__ dO, long ld_do, const float* __restrict__ LSE,
                  const float* __restrict__ DELTA, __bf16* __restrict__ dK, __bf16* __restrict__ dV, long ld_dkv,
                  const float* __restrict__ cosT, const float* __restrict__ sinT, int B,
                  int H, int Hkv, int S, float scale_log2, float scale, int group) {
    using Gm = Geo<D>;
    constexpr int RB = Gm::RB, TILE = Gm::TILE, KS = Gm::KS, ND = Gm::ND, CPT = Gm::CPT;
    static_assert(D == 64 || !ROPE_IN, "D = 128: Q / K are rotated before the kernels");
    constexpr int NT = NW * 64, KB = 32 * NW;
    // queries per Q / dO tile (one barrier each): 128 with LDS-DMA staging (two 64-row images side by side), 64
    // with register staging (ROPE_IN: Q is rotated on its way to LDS) and at D = 128
    constexpr bool DM = !ROPE_IN;
    constexpr int QT = (DM && D == 64) ? 128 : 64, NSUB = QT / 64, BUF = NSUB * TILE;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    char* Qs = smem;                                            // [2][QT q][RB]  (roped Q)
    char* dOs = smem + 2 * BUF;                                 // [2][QT q][RB]
    float* lseS = reinterpret_cast<float*>(smem + 4 * BUF);     // [2][QT]  -lse / c
    float* dltS = lseS + 2 * QT;                                // [2][QT]  -delta

    const int tid = threadIdx.x, w = tid >> 6, l = tid & 63, l31 = l & 31, hh = l >> 5;
    prologue_prio_begin();
    FA_STAMP(32768, 0, 0);
    const int nkb = (S + KB - 1) / KB;
    // One workgroup per (batch, KV head, key block) sweeps the G = H / Hkv query heads of its group one after the
    // other, summing their dK / dV in the accumulators: no fp32 partials, no reduce kernel (GQA).
    const int G = H / Hkv, GL = G;
    int kblk, bh;  // causal: key block 0 (the most query tiles) first
    grouped_order((int)blockIdx.x, nkb, B * Hkv, group, kblk, bh);
    const int b = bh / Hkv;
    const int h = (bh % Hkv) * G;  // first query head
    const int hk = h / G;
    const int kb0 = kblk * KB, kw0 = kb0 + 32 * w, key = kw0 + l31;
    const bool key_ok = key < S;
    const long kpos = key_ok ? key : S - 1;

    // ---- prologue: every load issued before any of them is waited for -- the pinned K / V rows, tile 0's row
    // constants and its Q / dO (LDS-DMA) -- one memory round trip instead of three (per-workgroup s_memtime stamps
    // at GPT-2 B 128: the serial form spent ~8k cycles of a ~42k-cycle workgroup here)
    u16x8 tkr[KS], tvr[KS];
    {
        const __bf16* kp = K + ((long)b * S + kpos) * ld_kv + (long)hk * D;
        const __bf16* vp = Vv + ((long)b * S + kpos) * ld_kv + (long)hk * D;
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) {
            // unconditional loads (kpos is clamped), consumed by a VALU select below in this prologue.  (As a branch
            // around the loads, the wait-count pass placed a vmcnt(0) before the first use of V inside the tile loop
            // -- draining the next tile's prefetch in every half-tile.)
            tkr[ks] = *reinterpret_cast<const u16x8*>(kp + 16 * ks + 8 * hh);
            tvr[ks] = *reinterpret_cast<const u16x8*>(vp + 16 * ks + 8 * hh);
        }
    }
    const int m_start = CAUSAL ? kb0 : 0;  // kb0 is a multiple of 64
    const int nqt = m_start < S ? (S - m_start + QT - 1) / QT : 0;
    const int nsteps = GL * nqt;  // (query head, query tile) steps, head-major
    // step j: query head h + j / nqt, query tile j % nqt
    auto q_of = [&](int j) { return Q + (long)b * S * ld_q + (long)(h + j / nqt) * D; };
    auto o_of = [&](int j) { return dO + (long)b * S * ld_do + (long)(h + j / nqt) * D; };
    // query tiles last to first: the diagonal tile (whose waves have 4, 3, 2, 1 half-steps) comes last, with no
    // barrier after it, so a wave done with it leaves its SIMD to the co-resident workgroup instead of waiting; and
    // the key blocks of one (batch, head) pair, launched together, start on the same Q / dO tile (L2 reuse)
    auto m0_of = [&](int j) { return m_start + (nqt - 1 - j % nqt) * QT; };
    u16x8 qreg[CPT], oreg[CPT];
    float lreg = 0.f, dreg = 0.f;
    // DM: Q / dO tiles by LDS-DMA through per-head buffer resources (no staging registers, no per-tile address
    // VALU); only the row constants go through registers
    const int wu = __builtin_amdgcn_readfirstlane(w);
    const DmaVoff<NW, RB> qvo = dma_voff<NW, RB>(ld_q, wu, l), ovo = dma_voff<NW, RB>(ld_do, wu, l);
    auto load_tile = [&](int it) {
        const int m0 = m0_of(it);
        const __bf16* qb = q_of(it);
        const __bf16* ob = o_of(it);
        const long sbase = ((long)b * H + h + it / nqt) * S;
        // every wave loads the stats of tile rows 64 (w & 1) + lane (waves 0 .. QT / 64 - 1 write them)
        const long idx = sbase + min(m0 + (QT == 128 ? 64 * (w & 1) : 0) + l, S - 1);
        lreg = LSE[idx];
        dreg = DELTA[idx];
        if constexpr (!DM) {  // DM: the tile itself is DMA'd by the loop body (after these loads)
#pragma unroll
            for (int i = 0; i < CPT; ++i) {
                const int e = tid + NT * i, r = (unsigned)e / (RB / 16), c = (unsigned)e % (RB / 16);
                const long qq = min(m0 + r, S - 1);
                qreg[i] = *reinterpret_cast<const u16x8*>(qb + qq * ld_q + c * 8);
                oreg[i] = *reinterpret_cast<const u16x8*>(ob + qq * ld_do + c * 8);
            }
        }
    };
    auto write_tile = [&](int it, int buf) {
        const int m0 = m0_of(it);
#pragma unroll
        for (int i = 0; i < (DM ? 0 : CPT); ++i) {
            const int e = tid + NT * i, r = (unsigned)e / (RB / 16), c = (unsigned)e % (RB / 16);
            const bool ok = m0 + r < S;
            u16x8 qv = ok ? qreg[i] : u16x8{0, 0, 0, 0, 0, 0, 0, 0};
            const u16x8 ov = ok ? oreg[i] : u16x8{0, 0, 0, 0, 0, 0, 0, 0};
            if (ROPE_IN) {
                const long qq = min(m0 + r, S - 1);
                qv = rope_u16x8(qv, cosT + qq * (D / 2) + c * 4, sinT + qq * (D / 2) + c * 4, 1.f);
            }
            *reinterpret_cast<u16x8*>(Qs + buf * TILE + swz<RB>(r, c)) = qv;
            *reinterpret_cast<u16x8*>(dOs + buf * TILE + swz<RB>(r, c)) = ov;
        }
        if (tid < QT) {  // the S / dP accumulators' starting values: -lse and -delta
            const bool ok = m0 + tid < S;
            lseS[buf * QT + tid] = (!ok || lreg == INFINITY) ? -INFINITY : -lreg;
            dltS[buf * QT + tid] = ok ? -dreg : 0.f;
        }
    };


    if (nqt > 0) {
        load_tile(0);
        if constexpr (DM) {
#pragma unroll
            for (int sb = 0; sb < NSUB; ++sb) {
                dma_tile64_buf(q_of(0), head_bytes(ld_q, S, D), qvo, m0_of(0) + 64 * sb, ld_q, Qs + sb * TILE, wu);
                dma_tile64_buf(o_of(0), head_bytes(ld_do, S, D), ovo, m0_of(0) + 64 * sb, ld_do, dOs + sb * TILE, wu);
            }
        }
    }

    // ---- pinned B operands: K (roped) and V rows of the lane's key, d = 16 ks + 8 hh + j
    bf16x8 kf[KS], vf[KS];
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
        const int d0 = 16 * ks + 8 * hh;
        const u16x8 z = {0, 0, 0, 0, 0, 0, 0, 0};
        u16x8 tk = key_ok ? tkr[ks] : z;
        const u16x8 tv = key_ok ? tvr[ks] : z;
        // softmax scale * log2(e) folded into the pinned K: S comes out in log2 units
        if (ROPE_IN) {
            tk = rope_u16x8(tk, cosT + kpos * (D / 2) + d0 / 2, sinT + kpos * (D / 2) + d0 / 2, scale_log2);
        } else {
            float x[8];
            unpack8(tk, x);
            tk = pack8(x, scale_log2);
        }
        kf[ks] = __builtin_bit_cast(bf16x8, tk);
        vf[ks] = __builtin_bit_cast(bf16x8, tv);
    }

    f32x16 dk[ND], dv[ND];
#pragma unroll
    for (int dt = 0; dt < ND; ++dt)
#pragma unroll
        for (int r = 0; r < 16; ++r) { dk[dt][r] = 0.f; dv[dt][r] = 0.f; }

    if (nqt > 0) write_tile(0, 0);
    __syncthreads();
    prologue_prio_end();
    FA_STAMP(32768, 1, 0);
    const int trow = 4 * hh + ((l & 15) >> 2);
    const int tcol = 16 * ((l >> 4) & 1) + 4 * (l & 3);
    const int klim = CAUSAL ? (key_ok ? key : S) : (key_ok ? 0 : S);
    const unsigned span = (unsigned)(S - klim);  // valid query q: (unsigned)(q - klim) < span
    for (int it = 0; it < nsteps; ++it) {
        const int cur = it & 1, m0 = m0_of(it);
        if (it + 1 == nsteps) FA_STAMP(32768, 2, 0);
        // One iteration with the current and the next buffers as __restrict__ parameters: the DMA into the next
        // buffer and the fragment reads of the current one are then provably disjoint to the wait-count pass
        // (without it hipcc drains the DMA, vmcnt(0), before the first transposed read of every half-tile).
        auto body = [&](char* __restrict__ Qc, char* __restrict__ Oc, char* __restrict__ Qn, char* __restrict__ On) {
            if (it + 1 < nsteps) {
                load_tile(it + 1);
                if constexpr (DM) {  // buffer cur ^ 1 was last read in iteration it - 1, before its closing barrier
#pragma unroll
                    for (int sb = 0; sb < NSUB; ++sb) {
                        dma_tile64_buf(q_of(it + 1), head_bytes(ld_q, S, D), qvo, m0_of(it + 1) + 64 * sb, ld_q,
                                       Qn + sb * TILE, wu);
                        dma_tile64_buf(o_of(it + 1), head_bytes(ld_do, S, D), ovo, m0_of(it + 1) + 64 * sb, ld_do,
                                       On + sb * TILE, wu);
                    }
                }
            }
            const float* lc = lseS + cur * QT;
            const float* dc = dltS + cur * QT;
            if (!CAUSAL || m0 + QT - 1 >= kw0) {
#pragma unroll
                for (int qq = 0; qq < QT / 32; ++qq) {
                    if (CAUSAL && m0 + 32 * qq + 31 < kw0) continue;  // every query of this step precedes every key
                    // masked only where a query of the step can precede a key of the wave (the diagonal 32 x 32
                    // step) or at the sequence end: the other steps of a diagonal tile take the unmasked path
                    const bool need_mask =
                        (CAUSAL && m0 + 32 * qq < kw0 + 31) || (m0 + 32 * qq + 32 > S) || (kw0 + 32 > S);
                    // step qq: image qq / 2 of the tile, its 32-query half qt
                    char* Qh = Qc + (qq >> 1) * TILE;
                    char* Oh = Oc + (qq >> 1) * TILE;
                    const int qt = qq & 1;
                    f32x16 sp, dp;
                    // (the dQ kernel's batched operand reads measured slower here: 256 VGPRs with 2 spilled, 1.1465
                    // vs 1.1437 ms at GPT-2 B 128, profiles/bench/ab_attn_sched128.log)
#pragma unroll
                    for (int i = 0; i < 4; ++i) {
                        const int qi = qq * 32 + 8 * i + 4 * hh;  // rows qi..qi+3 of registers 4i..4i+3
                        const f32x4 lv = *reinterpret_cast<const f32x4*>(lc + qi);
                        const f32x4 dl = *reinterpret_cast<const f32x4*>(dc + qi);
#pragma unroll
                        for (int j = 0; j < 4; ++j) { sp[4 * i + j] = lv[j]; dp[4 * i + j] = dl[j]; }
                    }
#pragma unroll
                    for (int ks = 0; ks < KS; ++ks) {
                        const int off = swz<RB>(qt * 32 + l31, 2 * ks + hh);
                        sp = mfma(lds_row16(Qh, off), kf[ks], sp);
                        dp = mfma(lds_row16(Oh, off), vf[ks], dp);
                    }
                    if (need_mask) {
                        const int qoff = m0 + qq * 32 - klim;
#pragma unroll
                        for (int r = 0; r < 16; ++r) {
                            const float p = fast_exp2(sp[r]);
                            const bool ok = (unsigned)(qoff + acc_row(r, hh)) < span;
                            sp[r] = ok ? p : 0.f;
                            dp[r] = ok ? p * dp[r] : 0.f;
                        }
                    } else {
#pragma unroll
                        for (int r = 0; r < 16; ++r) {
                            const float p = fast_exp2(sp[r]);
                            sp[r] = p;
                            dp[r] *= p;
                        }
                    }
#pragma unroll
                    for (int ss = 0; ss < 2; ++ss) {
                        bf16x8 pb, db;
#pragma unroll
                        for (int j = 0; j < 8; ++j) {
                            pb[j] = (__bf16)sp[8 * ss + j];
                            db[j] = (__bf16)dp[8 * ss + j];
                        }
                        const int qr = qt * 32 + 16 * ss;
#pragma unroll
                        for (int dt = 0; dt < ND; ++dt) {
                            const int o0 = tr_off<RB>(qr + trow, dt * 32 + tcol);
                            const int o1 = tr_off<RB>(qr + 8 + trow, dt * 32 + tcol);
                            dv[dt] = mfma(lds_tr_pair(Oh, o0, o1), pb, dv[dt]);
                            dk[dt] = mfma(lds_tr_pair(Qh, o0, o1), db, dk[dt]);
                        }
                    }
                }
            }
        };
        body(Qs + cur * BUF, dOs + cur * BUF, Qs + (cur ^ 1) * BUF, dOs + (cur ^ 1) * BUF);
        if (it + 1 < nsteps) {  // (no barrier after the last tile: see m0_of)
            write_tile(it + 1, cur ^ 1);
            __syncthreads();
        }
    }

    FA_STAMP(32768, 3, nsteps);
    if (!key_ok) return;
    // ---- dK = scale * R(-pos) dK^T, dV = dV^T (key on the lane, d in registers)
    __bf16* dkp = dK + ((long)b * S + key) * ld_dkv + (long)hk * D;
    __bf16* dvp = dV + ((long)b * S + key) * ld_dkv + (long)hk * D;
#pragma unroll
    for (int dt = 0; dt < ND; ++dt)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int d0 = dt * 32 + 8 * i + 4 * hh;
            float x[4] = {dk[dt][4 * i] * scale, dk[dt][4 * i + 1] * scale, dk[dt][4 * i + 2] * scale,
                          dk[dt][4 * i + 3] * scale};
            if (ROPE) {
#pragma unroll
                for (int pr = 0; pr < 2; ++pr) {
                    const float c = cosT[kpos * (D / 2) + d0 / 2 + pr];
                    const float sn = sinT[kpos * (D / 2) + d0 / 2 + pr];
                    const float a = x[2 * pr], bb = x[2 * pr + 1];
                    x[2 * pr] = a * c + bb * sn;
                    x[2 * pr + 1] = -a * sn + bb * c;
                }
            }
            *reinterpret_cast<u16x4*>(dkp + d0) = u16x4{f2bf(x[0]), f2bf(x[1]), f2bf(x[2]), f2bf(x[3])};
            *reinterpret_cast<u16x4*>(dvp + d0) = u16x4{f2bf(dv[dt][4 * i]), f2bf(dv[dt][4 * i + 1]),
                                                        f2bf(dv[dt][4 * i + 2]), f2bf(dv[dt][4 * i + 3])};
        }
}

}  // namespace split
}  // namespace fa
}  // namespace bpe

using namespace bpe;
using namespace bpe::fa;

// Backward form: 0 = split (default), 1 = fused (flash_attn_bwd.hip, the atomics form);
// switched at run time by fa_bwd_config (tests compare the two).  The split kernels run at 4 waves, 2 workgroups per
// CU, with LDS-DMA staging and 128-row tiles (the dQ kernel with batched operand reads).  Measured and removed (same
// box, op-level, GPT-2 B 128; docs/performance.md, attention): register staging (1.207-1.277 vs 1.178-1.204 ms),
// 8 waves (+10 %), 3 waves per SIMD (spills, 2.5x), a two-half software pipeline of the dK/dV kernel (+2.3 %), the
// ping-pong pair (8 waves in two staggered groups: +13-27 %), 64-row tiles (dQ 1.162 vs 1.159, dK/dV 1.179 vs
// 1.168 ms), the per-query-head dK / dV partials + reduce for GQA (Llama B 32 2.64 vs 2.31 ms).
static int g_mode = 0;

// D = 128 takes the split form for pre-rotated Q / K (rope 2) or no RoPE; fa_bwd rotates a copy for rope 1
bool fa_bwd_split_active(int D, int rope) { return (D == 64 || (D == 128 && rope != 1)) && g_mode == 0; }

// mode < 0 leaves the form unchanged; returns the form in force BEFORE the call
int fa_bwd_config(int mode) {
    const int prev = g_mode;
    if (mode >= 0) g_mode = mode ? 1 : 0;
    return prev;
}

template <int D, bool C, bool R, bool RIN>
static void split_launch(const FaArgs& a, hipStream_t s) {
    constexpr int NSUB = (RIN || D == 128) ? 1 : 2;  // 64-row images per LDS buffer (128-row tiles with LDS-DMA)
    constexpr int TILE = split::Geo<D>::TILE;
    const int nblk = (a.S + 32 * split::NW - 1) / (32 * split::NW);
    // the 16-queries-per-wave dQ kernel when selected (fa_dq_config; D = 64 without in-kernel RoPE)
    if (!launch_fa_bwd_dq16(a, s))
        split::fa_bwd_dq_kernel<D, C, R, RIN><<<nblk * a.B * a.H, split::NW * 64, 4 * TILE * NSUB, s>>>(
            a.q, a.k, a.v, a.ld_q, a.ld_kv, a.o, a.ld_o, a.dout, a.ld_do, a.lse, a.delta, a.dq, a.ld_dq, a.cos,
            a.sin, a.B, a.H, a.Hkv, a.S, a.scale * LOG2E, a.scale, fa_group(a.B * a.H));
    // Q / dO buffers + the -lse / -delta rows
    const int lds = 4 * TILE * NSUB + 16 * 64 * NSUB;
    split::fa_bwd_dkv_kernel<D, C, R, RIN><<<nblk * a.B * a.Hkv, split::NW * 64, lds, s>>>(
        a.q, a.k, a.v, a.ld_q, a.ld_kv, a.dout, a.ld_do, a.lse, a.delta, a.dk, a.dv, a.ld_dkv, a.cos,
        a.sin, a.B, a.H, a.Hkv, a.S, a.scale * LOG2E, a.scale, fa_group(a.B * a.Hkv));
}

// whether a GQA backward of head size D needs the fp32 dK / dV partials buffer (FaArgs::dkv_part): only the fused
// backward does (the split dK/dV kernel sweeps the query heads of its KV head)
bool fa_dkv_partials_needed(int D, int rope) { return !fa_bwd_split_active(D, rope); }

// copy the last launch's stamps out (BPE_FA_STAMPS builds; false otherwise)
bool fa_read_stamps(long long* host, int n) {
#ifdef BPE_FA_STAMPS
    (void)hipDeviceSynchronize();
    const bool ok = hipMemcpyFromSymbol(host, HIP_SYMBOL(split::g_stamps), (size_t)n * 8 * sizeof(long long), 0,
                                        hipMemcpyDeviceToHost) == hipSuccess;
    fa_read_stamps_dq16(host, n);  // rows 0.. from the 16-row dQ kernel when it ran
    return ok;
#else
    (void)host;
    (void)n;
    return false;
#endif
}

bool launch_fa_bwd_split(const FaArgs& a, hipStream_t s) {
    if (!fa_bwd_split_active(a.D, a.rope)) return false;
    // rope: 0 none, 1 rotate Q / K on load and dQ / dK on output, 2 outputs only (Q / K pre-rotated)
    if (a.D == 128) {
        if (a.causal) {
            if (a.rope == 2) split_launch<128, true, true, false>(a, s);
            else split_launch<128, true, false, false>(a, s);
        } else {
            if (a.rope == 2) split_launch<128, false, true, false>(a, s);
            else split_launch<128, false, false, false>(a, s);
        }
        return true;
    }
    if (a.causal) {
        if (a.rope == 1) split_launch<64, true, true, true>(a, s);
        else if (a.rope == 2) split_launch<64, true, true, false>(a, s);
        else split_launch<64, true, false, false>(a, s);
    } else {
        if (a.rope == 1) split_launch<64, false, true, true>(a, s);
        else if (a.rope == 2) split_launch<64, false, true, false>(a, s);
        else split_launch<64, false, false, false>(a, s);
    }
    return true;
}
