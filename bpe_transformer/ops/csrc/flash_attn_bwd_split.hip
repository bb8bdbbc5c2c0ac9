// Flash attention backward, split form (D = 64), gfx950 (MI355X).
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
//       pinned in registers for the whole key sweep; K / V tiles are staged in LDS (register staging, guide
//       T14: loads of tile t+1 issued before tile t's MFMAs, written after them; one barrier per tile).  dS^T
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
// GQA: the dK / dV kernel runs per query head and writes fp32 partials summed by fa_dkv_reduce_kernel.
#include "fa_common.h"
#include "kernels.h"

#include <cstdlib>

namespace bpe {
namespace fa {
namespace split {

constexpr int D = 64, RB = 128, TILE = 64 * RB, KS = 4;

// staged 16-byte chunks per thread and tensor for one 64-row tile (512 chunks)
template <int NW> constexpr int cpt() { return 512 / (NW * 64); }

template <bool CAUSAL, bool ROPE, bool ROPE_IN, int NW, int OCC = 2, bool DMA = false, bool SCHED = false,
          int KTT = 64>
__global__ void __launch_bounds__(NW * 64, OCC)
fa_bwd_dq_kernel(const __bf16* __restrict__ Q, const __bf16* __restrict__ K, const __bf16* __restrict__ Vv,
                 long ld_q, long ld_kv, const __bf16* __restrict__ O, long ld_o, const __bf16* __restrict__ dO,
                 long ld_do, const float* __restrict__ LSE, float* __restrict__ DELTA, __bf16* __restrict__ dQ,
                 long ld_dq, const float* __restrict__ cosT, const float* __restrict__ sinT, int B, int H, int Hkv,
                 int S, float scale_log2, float scale, int group) {
    constexpr int NT = NW * 64, QB = 32 * NW, CPT = cpt<NW>();
    // keys per K / V tile (one barrier each): KTT (64 or 128) with LDS-DMA staging, 64 with register staging; a
    // 128-key tile is two 64-row images side by side
    constexpr bool DM = DMA && !ROPE_IN;
    constexpr int KT = DM ? KTT : 64, NSUB = KT / 64, BUF = NSUB * TILE;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    char* Ks = smem;            // [2][KT keys][128 B]  (roped K)
    char* Vs = smem + 2 * BUF;  // [2][KT keys][128 B]

    const int tid = threadIdx.x, w = tid >> 6, l = tid & 63, l31 = l & 31, hh = l >> 5;
    const int nqb = (S + QB - 1) / QB;
    int rank, bh;
    grouped_order((int)blockIdx.x, nqb, B * H, group, rank, bh);
    const int qblk = CAUSAL ? nqb - 1 - rank : rank;  // causal: the last (heaviest) query blocks first
    const int b = bh / H, h = bh % H, hk = h / (H / Hkv);
    const int q0 = qblk * QB, qw = q0 + 32 * w, q = qw + l31;
    const bool q_ok = q < S;
    const long qc = q_ok ? q : S - 1;
    const long qrow = (long)b * S + qc;

    // ---- pinned B operands (query on the lane, d = 16 ks + 8 hh + j) and delta = rowsum(dO * O)
    bf16x8 qf[KS], of[KS];
    float dsum = 0.f;
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
        const int d0 = 16 * ks + 8 * hh;
        u16x8 tq = *reinterpret_cast<const u16x8*>(Q + qrow * ld_q + (long)h * D + d0);
        // softmax scale * log2(e) folded into the pinned Q (as the forward does): S^T comes out in log2 units
        if (ROPE_IN) {
            tq = rope_u16x8(tq, cosT + qc * (D / 2) + d0 / 2, sinT + qc * (D / 2) + d0 / 2, scale_log2);
        } else {
            float x[8];
            unpack8(tq, x);
            tq = pack8(x, scale_log2);
        }
        qf[ks] = __builtin_bit_cast(bf16x8, tq);
        const u16x8 tg = *reinterpret_cast<const u16x8*>(dO + qrow * ld_do + (long)h * D + d0);
        const u16x8 to = *reinterpret_cast<const u16x8*>(O + qrow * ld_o + (long)h * D + d0);
#pragma unroll
        for (int i = 0; i < 8; ++i) dsum += bf2f(tg[i]) * bf2f(to[i]);
        of[ks] = __builtin_bit_cast(bf16x8, tg);
    }
    dsum += __shfl_xor(dsum, 32, 64);
    if (q_ok && hh == 0) DELTA[((long)b * H + h) * S + q] = dsum;
    const float lse = LSE[((long)b * H + h) * S + qc];
    // row constants as the initial accumulators (query = lane): S^T starts at -lse, so P = exp2(S^T) with no
    // VALU before the exponential (-inf for empty / pad rows: P = 0); dP^T starts at -delta
    const float nl = (q_ok && lse < INFINITY) ? -lse : -INFINITY;
    f32x16 ns, nd;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
        ns[r] = nl;
        nd[r] = -dsum;
    }

    f32x16 acc[2];
#pragma unroll
    for (int dt = 0; dt < 2; ++dt)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[dt][r] = 0.f;

    const int kend = CAUSAL ? min(S, q0 + QB) : S;
    const int nkt = (kend + KT - 1) / KT;
    const __bf16* kb = K + (long)b * S * ld_kv + (long)hk * D;
    const __bf16* vb = Vv + (long)b * S * ld_kv + (long)hk * D;
    u16x8 kreg[CPT], vreg[CPT];
    auto load_tile = [&](int it) {
#pragma unroll
        for (int i = 0; i < CPT; ++i) {
            const int e = tid + NT * i, r = e >> 3, c = e & 7;
            const long kk = min(it * 64 + r, S - 1);  // rows past the end: valid memory, zeroed at the write
            kreg[i] = *reinterpret_cast<const u16x8*>(kb + kk * ld_kv + c * 8);
            vreg[i] = *reinterpret_cast<const u16x8*>(vb + kk * ld_kv + c * 8);
        }
    };
    auto write_tile = [&](int it, int buf) {
#pragma unroll
        for (int i = 0; i < CPT; ++i) {
            const int e = tid + NT * i, r = e >> 3, c = e & 7;
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
    const DmaVoff<NW> kvo = dma_voff<NW>(ld_kv, wu, l);
    if constexpr (DM) {
#pragma unroll
        for (int sb = 0; sb < NSUB; ++sb) {
            dma_tile64_buf(kb, hbytes, kvo, 64 * sb, ld_kv, Ks + sb * TILE, wu);
            dma_tile64_buf(vb, hbytes, kvo, 64 * sb, ld_kv, Vs + sb * TILE, wu);
        }
    } else {
        load_tile(0);
        write_tile(0, 0);
    }
    __syncthreads();

    const int trow = 4 * hh + ((l & 15) >> 2);          // tr-read row inside a 16-key step
    const int tcol = 16 * ((l >> 4) & 1) + 4 * (l & 3);  // tr-read column inside a 32-wide d tile
    for (int it = 0; it < nkt; ++it) {
        const int cur = it & 1, k0 = it * KT;
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
                const bool need_mask = (CAUSAL && k0 + KT - 1 > qw) || (k0 + KT > S);
#pragma unroll
                for (int kq = 0; kq < KT / 32; ++kq) {
                    if (CAUSAL && k0 + 32 * kq > qw + 31) break;  // this 32-key step is past every query of the wave
                    // step kq: image kq / 2 of the tile, its 32-key half kh
                    char* Kh = Kc + (kq >> 1) * TILE;
                    const char* Vh = Vc + (kq >> 1) * TILE;
                    const int kh = kq & 1;
                    f32x16 sp = ns, dp = nd;
                    bf16x8 tk[2][2];  // SCHED: the transposed K fragments of the dQ products (s, dt)
                    if constexpr (SCHED) {  // operand reads batched ahead of their uses (see fa_bwd_dkv_kernel)
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
                        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
                        for (int s = 0; s < 2; ++s)
#pragma unroll
                            for (int dt = 0; dt < 2; ++dt) {
                                const int kr = 32 * kh + 16 * s;
                                tk[s][dt] = lds_tr_pair(Kh, tr_off<RB>(kr + trow, 32 * dt + tcol),
                                                        tr_off<RB>(kr + 8 + trow, 32 * dt + tcol));
                            }
                        __builtin_amdgcn_sched_barrier(0);
                    } else {
#pragma unroll
                        for (int ks = 0; ks < KS; ++ks) {
                            const int koff = swz<RB>(32 * kh + l31, 2 * ks + hh);
                            sp = mfma(lds_row16(Kh, koff), qf[ks], sp);
                            dp = mfma(lds_row16(Vh, koff), of[ks], dp);
                        }
                    }
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
#pragma unroll
                        for (int dt = 0; dt < 2; ++dt) {
                            if constexpr (SCHED)
                                acc[dt] = mfma(tk[s][dt], db, acc[dt]);
                            else
                                acc[dt] = mfma(lds_tr_pair(Kh, tr_off<RB>(kr + trow, 32 * dt + tcol),
                                                           tr_off<RB>(kr + 8 + trow, 32 * dt + tcol)),
                                               db, acc[dt]);
                        }
                    }
                }
            }
        };
        body(Ks + cur * BUF, Vs + cur * BUF, Ks + (cur ^ 1) * BUF, Vs + (cur ^ 1) * BUF);
        if (!DM && it + 1 < nkt) write_tile(it + 1, cur ^ 1);
        __syncthreads();
    }

    // ---- epilogue: dQ = scale * R(-pos) dQ^T (query on the lane, 4 consecutive d per register group)
    if (q_ok) {
        __bf16* dqp = dQ + ((long)b * S + q) * ld_dq + (long)h * D;
#pragma unroll
        for (int dt = 0; dt < 2; ++dt)
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

template <bool CAUSAL, bool ROPE, bool ROPE_IN, int NW, int OCC = 2, bool DMA = false, bool SCHED = false,
          bool LOOPG = false, int QTT = 64>
__global__ void __launch_bounds__(NW * 64, OCC)
fa_bwd_dkv_kernel(const __bf16* __restrict__ Q, const __bf16* __restrict__ K, const __bf16* __restrict__ Vv,
                  long ld_q, long ld_kv, const __bf16* __restrict__ dO, long ld_do, const float* __restrict__ LSE,
                  const float* __restrict__ DELTA, __bf16* __restrict__ dK, __bf16* __restrict__ dV, long ld_dkv,
                  float* __restrict__ dKVpart, const float* __restrict__ cosT, const float* __restrict__ sinT, int B,
                  int H, int Hkv, int S, float scale_log2, float scale, int group) {
    constexpr int NT = NW * 64, KB = 32 * NW, CPT = cpt<NW>();
    // queries per Q / dO tile (one barrier each): QTT (64 or 128) with LDS-DMA staging, 64 with register staging;
    // a 128-query tile is two 64-row images side by side
    constexpr int QT = (DMA && !ROPE_IN) ? QTT : 64, NSUB = QT / 64, BUF = NSUB * TILE;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    char* Qs = smem;                                            // [2][QT q][128 B]  (roped Q)
    char* dOs = smem + 2 * BUF;                                 // [2][QT q][128 B]
    float* lseS = reinterpret_cast<float*>(smem + 4 * BUF);     // [2][QT]  -lse / c
    float* dltS = lseS + 2 * QT;                                // [2][QT]  -delta

    const int tid = threadIdx.x, w = tid >> 6, l = tid & 63, l31 = l & 31, hh = l >> 5;
    const int nkb = (S + KB - 1) / KB;
    // LOOPG (GQA): one workgroup per (batch, KV head, key block) sweeps the G query heads of its group one after
    // the other, summing their dK / dV in the accumulators -- no fp32 partials, no reduce kernel.  Otherwise one
    // workgroup per (batch, query head, key block).
    const int G = H / Hkv, GL = LOOPG ? G : 1;
    int kblk, bh;  // causal: key block 0 (the most query tiles) first
    grouped_order((int)blockIdx.x, nkb, B * (LOOPG ? Hkv : H), group, kblk, bh);
    const int b = LOOPG ? bh / Hkv : bh / H;
    const int h = LOOPG ? (bh % Hkv) * G : bh % H;  // (first) query head
    const int hk = h / G;
    const int kb0 = kblk * KB, kw0 = kb0 + 32 * w, key = kw0 + l31;
    const bool key_ok = key < S;
    const long kpos = key_ok ? key : S - 1;

    // ---- pinned B operands: K (roped) and V rows of the lane's key, d = 16 ks + 8 hh + j
    bf16x8 kf[KS], vf[KS];
    {
        const __bf16* kp = K + ((long)b * S + kpos) * ld_kv + (long)hk * D;
        const __bf16* vp = Vv + ((long)b * S + kpos) * ld_kv + (long)hk * D;
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) {
            const int d0 = 16 * ks + 8 * hh;
            // unconditional loads (kpos is clamped) consumed by a VALU select here: the wait for them then sits in
            // this prologue.  (As a branch around the loads, the wait-count pass placed a vmcnt(0) before the first
            // use of V inside the tile loop -- draining the next tile's prefetch in every half-tile.)
            u16x8 tk = *reinterpret_cast<const u16x8*>(kp + d0);
            u16x8 tv = *reinterpret_cast<const u16x8*>(vp + d0);
            const u16x8 z = {0, 0, 0, 0, 0, 0, 0, 0};
            tk = key_ok ? tk : z;
            tv = key_ok ? tv : z;
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
    }

    f32x16 dk[2], dv[2];
#pragma unroll
    for (int dt = 0; dt < 2; ++dt)
#pragma unroll
        for (int r = 0; r < 16; ++r) { dk[dt][r] = 0.f; dv[dt][r] = 0.f; }

    const int m_start = CAUSAL ? kb0 : 0;  // kb0 is a multiple of 64
    const int nqt = m_start < S ? (S - m_start + QT - 1) / QT : 0;
    const int nsteps = GL * nqt;  // (query head, query tile) steps, head-major
    // step j: query head h + j / nqt, query tile j % nqt
    auto q_of = [&](int j) { return Q + (long)b * S * ld_q + (long)(h + j / nqt) * D; };
    auto o_of = [&](int j) { return dO + (long)b * S * ld_do + (long)(h + j / nqt) * D; };
    auto m0_of = [&](int j) { return m_start + (j % nqt) * QT; };
    u16x8 qreg[CPT], oreg[CPT];
    float lreg = 0.f, dreg = 0.f;
    // DM: Q / dO tiles by LDS-DMA through per-head buffer resources (no staging registers, no per-tile address
    // VALU); only the row constants go through registers
    constexpr bool DM = DMA && !ROPE_IN;
    const int wu = __builtin_amdgcn_readfirstlane(w);
    const DmaVoff<NW> qvo = dma_voff<NW>(ld_q, wu, l), ovo = dma_voff<NW>(ld_do, wu, l);
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
                const int e = tid + NT * i, r = e >> 3, c = e & 7;
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
            const int e = tid + NT * i, r = e >> 3, c = e & 7;
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
                dma_tile64_buf(q_of(0), head_bytes(ld_q, S, D), qvo, m_start + 64 * sb, ld_q, Qs + sb * TILE, wu);
                dma_tile64_buf(o_of(0), head_bytes(ld_do, S, D), ovo, m_start + 64 * sb, ld_do, dOs + sb * TILE, wu);
            }
        }
        write_tile(0, 0);
    }
    __syncthreads();

    const int trow = 4 * hh + ((l & 15) >> 2);
    const int tcol = 16 * ((l >> 4) & 1) + 4 * (l & 3);
    const int klim = CAUSAL ? (key_ok ? key : S) : (key_ok ? 0 : S);
    const unsigned span = (unsigned)(S - klim);  // valid query q: (unsigned)(q - klim) < span
    for (int it = 0; it < nsteps; ++it) {
        const int cur = it & 1, m0 = m0_of(it);
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
                const bool need_mask = (CAUSAL && m0 < kw0 + 31) || (m0 + QT > S) || (kw0 + 32 > S);
#pragma unroll
                for (int qq = 0; qq < QT / 32; ++qq) {
                    if (CAUSAL && m0 + 32 * qq + 31 < kw0) continue;  // every query of this step precedes every key
                    // step qq: image qq / 2 of the tile, its 32-query half qt
                    char* Qh = Qc + (qq >> 1) * TILE;
                    char* Oh = Oc + (qq >> 1) * TILE;
                    const int qt = qq & 1;
                    f32x16 sp, dp;
                    // every operand read of the half is issued before its first use (SCHED): the S / dP row
                    // fragments before the chains, the transposed dV / dK fragments before the softmax VALU, so
                    // their LDS latency is paid once per batch instead of once per MFMA (hipcc's own schedule
                    // waits lgkmcnt(0) in front of every MFMA pair)
                    bf16x8 fq[KS], fo[KS], tq[2][2], to[2][2];
                    if constexpr (SCHED) {
#pragma unroll
                        for (int ks = 0; ks < KS; ++ks) {
                            const int off = swz<RB>(qt * 32 + l31, 2 * ks + hh);
                            fq[ks] = lds_row16(Qh, off);
                            fo[ks] = lds_row16(Oh, off);
                        }
                    }
#pragma unroll
                    for (int i = 0; i < 4; ++i) {
                        const int qi = qq * 32 + 8 * i + 4 * hh;  // rows qi..qi+3 of registers 4i..4i+3
                        const f32x4 lv = *reinterpret_cast<const f32x4*>(lc + qi);
                        const f32x4 dl = *reinterpret_cast<const f32x4*>(dc + qi);
#pragma unroll
                        for (int j = 0; j < 4; ++j) { sp[4 * i + j] = lv[j]; dp[4 * i + j] = dl[j]; }
                    }
                    if constexpr (SCHED) {
                        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
                        for (int ks = 0; ks < KS; ++ks) {
                            sp = mfma(fq[ks], kf[ks], sp);
                            dp = mfma(fo[ks], vf[ks], dp);
                        }
                        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
                        for (int ss = 0; ss < 2; ++ss)
#pragma unroll
                            for (int dt = 0; dt < 2; ++dt) {
                                const int qr = qt * 32 + 16 * ss;
                                const int o0 = tr_off<RB>(qr + trow, dt * 32 + tcol);
                                const int o1 = tr_off<RB>(qr + 8 + trow, dt * 32 + tcol);
                                to[ss][dt] = lds_tr_pair(Oh, o0, o1);
                                tq[ss][dt] = lds_tr_pair(Qh, o0, o1);
                            }
                        __builtin_amdgcn_sched_barrier(0);
                    } else {
#pragma unroll
                        for (int ks = 0; ks < KS; ++ks) {
                            const int off = swz<RB>(qt * 32 + l31, 2 * ks + hh);
                            sp = mfma(lds_row16(Qh, off), kf[ks], sp);
                            dp = mfma(lds_row16(Oh, off), vf[ks], dp);
                        }
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
                        for (int dt = 0; dt < 2; ++dt) {
                            if constexpr (SCHED) {
                                dv[dt] = mfma(to[ss][dt], pb, dv[dt]);
                                dk[dt] = mfma(tq[ss][dt], db, dk[dt]);
                            } else {
                                const int o0 = tr_off<RB>(qr + trow, dt * 32 + tcol);
                                const int o1 = tr_off<RB>(qr + 8 + trow, dt * 32 + tcol);
                                dv[dt] = mfma(lds_tr_pair(Oh, o0, o1), pb, dv[dt]);
                                dk[dt] = mfma(lds_tr_pair(Qh, o0, o1), db, dk[dt]);
                            }
                        }
                    }
                }
            }
        };
        body(Qs + cur * BUF, dOs + cur * BUF, Qs + (cur ^ 1) * BUF, dOs + (cur ^ 1) * BUF);
        if (it + 1 < nsteps) write_tile(it + 1, cur ^ 1);
        __syncthreads();
    }

    if (!key_ok) return;
    if (G > 1 && !LOOPG) {  // GQA: fp32 partials of this query head -> [b, s, h, {dK, dV}, D] for fa_dkv_reduce_kernel
        float* pk = dKVpart + (((long)b * S + key) * H + h) * 2 * D;
#pragma unroll
        for (int dt = 0; dt < 2; ++dt)
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int d0 = dt * 32 + 8 * i + 4 * hh;
                *reinterpret_cast<f32x4*>(pk + d0) =
                    f32x4{dk[dt][4 * i], dk[dt][4 * i + 1], dk[dt][4 * i + 2], dk[dt][4 * i + 3]};
                *reinterpret_cast<f32x4*>(pk + D + d0) =
                    f32x4{dv[dt][4 * i], dv[dt][4 * i + 1], dv[dt][4 * i + 2], dv[dt][4 * i + 3]};
            }
        return;
    }
    // ---- dK = scale * R(-pos) dK^T, dV = dV^T (key on the lane, d in registers)
    __bf16* dkp = dK + ((long)b * S + key) * ld_dkv + (long)hk * D;
    __bf16* dvp = dV + ((long)b * S + key) * ld_dkv + (long)hk * D;
#pragma unroll
    for (int dt = 0; dt < 2; ++dt)
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

// ---------------------------------------------------------------------------------------------------------
// Ping-pong dK / dV kernel (the default for the split form).  Same math as fa_bwd_dkv_kernel; the schedule is the
// one that keeps the ping-pong GEMM's matrix pipe busy (gemm_pp.hip, guide §5 8-phase template): 8 waves in two
// groups of four; waves w and w + 4 share a SIMD and own adjacent 32-key blocks (keys kb0 + 64 (w & 3) +
// 32 (w >> 2)); group 1 runs one barrier interval behind group 0.  A wave's work is a chain of half-steps
// j = 2 t + h (query tile t, 32-query half h), each cut into two segments separated by barriers:
//   M(j): MFMA section -- dV^T += dO^T.P and dK^T += Q^T.dS of half-step j - 1 (operands read in V(j - 1)),
//         then S = Q.(cK)^T - lse and dP = dO.V^T - delta of half-step j (16 MFMAs, the rows and the row
//         constants read at the top of the section so they land under the first 8 MFMAs)
//   V(j): VALU section -- P = exp2(S), dS = P dP, bf16 packing, the transposed reads dV/dK(j) will need,
//         and the staging of the next query tile.
// So in every barrier interval one wave of each SIMD issues 16 MFMAs while its partner exponentiates: the
// softmax VALU (~300 cycles per half-step) hides under the partner's 512 MFMA cycles.
// Staging: query tile t + 1 is written into LDS buffer (t + 1) & 1 in V(2t) -- group g the rows [32 g, +32) of
// Q and dO and their row constants -- from registers loaded in V(2t - 2), and is first read in M(2t + 2).
// WAR: that buffer's previous tile (t - 1) was last read in V(2t - 1) (transposed reads), which group 1 runs in
// the interval before group 0's V(2t).  RAW: group 1's writes (its V(2t)) land two intervals before group 0's
// M(2t + 2).  Every section that writes LDS retires its writes (lgkmcnt(0)) before its closing barrier.
constexpr int PPNW = 8;

__device__ __forceinline__ void pp_bar() {
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
}

template <bool CAUSAL, bool ROPE, bool ROPE_IN>
__global__ void __launch_bounds__(PPNW * 64, 1)
fa_bwd_dkv_pp_kernel(const __bf16* __restrict__ Q, const __bf16* __restrict__ K, const __bf16* __restrict__ Vv,
                     long ld_q, long ld_kv, const __bf16* __restrict__ dO, long ld_do, const float* __restrict__ LSE,
                     const float* __restrict__ DELTA, __bf16* __restrict__ dK, __bf16* __restrict__ dV, long ld_dkv,
                     float* __restrict__ dKVpart, const float* __restrict__ cosT, const float* __restrict__ sinT,
                     int B, int H, int Hkv, int S, float scale_log2, float scale, int group) {
    constexpr int KB = 32 * PPNW;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    char* Qs = smem;                                          // [2][64 q][128 B]  (roped Q)
    char* dOs = smem + 2 * TILE;                              // [2][64 q][128 B]
    float* lseS = reinterpret_cast<float*>(smem + 4 * TILE);  // [2][64]  -lse
    float* dltS = lseS + 128;                                 // [2][64]  -delta

    const int tid = threadIdx.x, l = tid & 63, l31 = l & 31, hh = l >> 5;
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int g = w >> 2, wl = w & 3, gt = tid & 255;  // group, wave in group, thread in group
    const int nkb = (S + KB - 1) / KB;
    int kblk, bh;
    grouped_order((int)blockIdx.x, nkb, B * H, group, kblk, bh);
    const int b = bh / H, h = bh % H, G = H / Hkv, hk = h / G;
    const int kb0 = kblk * KB, kw0 = kb0 + 64 * wl + 32 * g, key = kw0 + l31;
    const bool key_ok = key < S;
    const long kpos = key_ok ? key : S - 1;

    bf16x8 kf[KS], vf[KS];
    {
        const __bf16* kp = K + ((long)b * S + kpos) * ld_kv + (long)hk * D;
        const __bf16* vp = Vv + ((long)b * S + kpos) * ld_kv + (long)hk * D;
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) {
            const int d0 = 16 * ks + 8 * hh;
            u16x8 tk = *reinterpret_cast<const u16x8*>(kp + d0);
            u16x8 tv = *reinterpret_cast<const u16x8*>(vp + d0);
            const u16x8 z = {0, 0, 0, 0, 0, 0, 0, 0};
            tk = key_ok ? tk : z;
            tv = key_ok ? tv : z;
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
    }
    f32x16 dk[2], dv[2];
#pragma unroll
    for (int dt = 0; dt < 2; ++dt)
#pragma unroll
        for (int r = 0; r < 16; ++r) { dk[dt][r] = 0.f; dv[dt][r] = 0.f; }

    const int m_start = CAUSAL ? kb0 : 0;
    const int nqt = m_start < S ? (S - m_start + 63) / 64 : 0;
    const int J = 2 * nqt;  // half-steps
    const __bf16* qb = Q + (long)b * S * ld_q + (long)h * D;
    const __bf16* ob = dO + (long)b * S * ld_do + (long)h * D;
    const long sbase = ((long)b * H + h) * S;
    // staging: group g owns rows [32 g, +32) of every tile: one Q chunk and one dO chunk per thread, and (threads
    // gt < 32) that row's lse / delta
    const int srow = 32 * g + (gt >> 3), sc = gt & 7;
    u16x8 qreg, oreg;
    float lreg = 0.f, dreg = 0.f;
    auto load_tile = [&](int t) {
        const long qq = min(m_start + t * 64 + srow, S - 1);
        qreg = *reinterpret_cast<const u16x8*>(qb + qq * ld_q + sc * 8);
        oreg = *reinterpret_cast<const u16x8*>(ob + qq * ld_do + sc * 8);
        const long idx = sbase + min(m_start + t * 64 + 32 * g + (gt & 31), S - 1);
        lreg = LSE[idx];
        dreg = DELTA[idx];
    };
    auto write_tile = [&](int t) {
        const int buf = t & 1, m0 = m_start + t * 64;
        const bool ok = m0 + srow < S;
        u16x8 qv = ok ? qreg : u16x8{0, 0, 0, 0, 0, 0, 0, 0};
        const u16x8 ov = ok ? oreg : u16x8{0, 0, 0, 0, 0, 0, 0, 0};
        if (ROPE_IN) {
            const long qq = min(m0 + srow, S - 1);
            qv = rope_u16x8(qv, cosT + qq * (D / 2) + sc * 4, sinT + qq * (D / 2) + sc * 4, 1.f);
        }
        *reinterpret_cast<u16x8*>(Qs + buf * TILE + swz<RB>(srow, sc)) = qv;
        *reinterpret_cast<u16x8*>(dOs + buf * TILE + swz<RB>(srow, sc)) = ov;
        if (gt < 32) {
            const int r = 32 * g + gt;
            const bool okr = m0 + r < S;
            lseS[buf * 64 + r] = (!okr || lreg == INFINITY) ? -INFINITY : -lreg;
            dltS[buf * 64 + r] = okr ? -dreg : 0.f;
        }
    };

    const int trow = 4 * hh + ((l & 15) >> 2);
    const int tcol = 16 * ((l >> 4) & 1) + 4 * (l & 3);
    const int klim = CAUSAL ? (key_ok ? key : S) : (key_ok ? 0 : S);
    const unsigned span = (unsigned)(S - klim);

    // prologue: tile 0 staged and visible; tile 1 in registers
    if (nqt > 0) {
        load_tile(0);
        write_tile(0);
        if (nqt > 1) load_tile(1);
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    pp_bar();
    if (g == 1) pp_bar();  // the stagger

    f32x16 sp, dp;          // S / dP of the current half-step (from its M section to its V section)
    bf16x8 pb[2], db[2];    // bf16 P / dS of the previous half-step (V -> next M)
    bf16x8 tq[2][2], to[2][2];  // its transposed Q / dO fragments [ss][dt]
    bool prev_active = false;
    for (int j = 0; j <= J; ++j) {
        const int t = j >> 1, hf = j & 1, m0 = m_start + t * 64;
        const bool active = j < J && (!CAUSAL || m0 + 32 * hf + 31 >= kw0);
        // ---------------- M(j): the previous half-step's dV / dK MFMAs (operands already in registers) are issued
        // first; the row reads of this half-step follow (a scheduling fence keeps the compiler from hoisting all
        // of them above: register pressure) and land while those MFMAs run.
        {
            if (prev_active) {
#pragma unroll
                for (int ss = 0; ss < 2; ++ss)
#pragma unroll
                    for (int dt = 0; dt < 2; ++dt) {
                        dv[dt] = mfma(to[ss][dt], pb[ss], dv[dt]);
                        dk[dt] = mfma(tq[ss][dt], db[ss], dk[dt]);
                    }
            }
            __builtin_amdgcn_sched_barrier(0);
            if (active) {
                char* Qc = Qs + (t & 1) * TILE;
                char* Oc = dOs + (t & 1) * TILE;
                const float* lc = lseS + (t & 1) * 64;
                const float* dc = dltS + (t & 1) * 64;
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    const int qi = hf * 32 + 8 * i + 4 * hh;
                    const f32x4 lv = *reinterpret_cast<const f32x4*>(lc + qi);
                    const f32x4 dl = *reinterpret_cast<const f32x4*>(dc + qi);
#pragma unroll
                    for (int jj = 0; jj < 4; ++jj) { sp[4 * i + jj] = lv[jj]; dp[4 * i + jj] = dl[jj]; }
                }
#pragma unroll
                for (int ks = 0; ks < KS; ++ks) {
                    const int off = swz<RB>(hf * 32 + l31, 2 * ks + hh);
                    sp = mfma(lds_row16(Qc, off), kf[ks], sp);
                    dp = mfma(lds_row16(Oc, off), vf[ks], dp);
                }
            }
        }
        pp_bar();
        if (j == J) break;
        // ---------------- V(j)
        {
            char* Qc = Qs + (t & 1) * TILE;
            char* Oc = dOs + (t & 1) * TILE;
            if (active) {
                const bool need_mask = (CAUSAL && m0 + 32 * hf < kw0 + 31) || (m0 + 32 * hf + 32 > S) || (kw0 + 32 > S);
                if (need_mask) {
                    const int qoff = m0 + hf * 32 - klim;
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
#pragma unroll
                    for (int jj = 0; jj < 8; ++jj) {
                        pb[ss][jj] = (__bf16)sp[8 * ss + jj];
                        db[ss][jj] = (__bf16)dp[8 * ss + jj];
                    }
                    const int qr = hf * 32 + 16 * ss;
#pragma unroll
                    for (int dt = 0; dt < 2; ++dt) {
                        const int o0 = tr_off<RB>(qr + trow, dt * 32 + tcol);
                        const int o1 = tr_off<RB>(qr + 8 + trow, dt * 32 + tcol);
                        to[ss][dt] = lds_tr_pair(Oc, o0, o1);
                        tq[ss][dt] = lds_tr_pair(Qc, o0, o1);
                    }
                }
            }
            prev_active = active;
            if (hf == 0 && t + 1 < nqt) {  // stage tile t + 1 (loaded two half-steps ago), then load tile t + 2
                write_tile(t + 1);
                if (t + 2 < nqt) load_tile(t + 2);
            }
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        }
        pp_bar();
    }
    if (g == 0) pp_bar();

    if (!key_ok) return;
    if (G > 1) {
        float* pk = dKVpart + (((long)b * S + key) * H + h) * 2 * D;
#pragma unroll
        for (int dt = 0; dt < 2; ++dt)
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int d0 = dt * 32 + 8 * i + 4 * hh;
                *reinterpret_cast<f32x4*>(pk + d0) =
                    f32x4{dk[dt][4 * i], dk[dt][4 * i + 1], dk[dt][4 * i + 2], dk[dt][4 * i + 3]};
                *reinterpret_cast<f32x4*>(pk + D + d0) =
                    f32x4{dv[dt][4 * i], dv[dt][4 * i + 1], dv[dt][4 * i + 2], dv[dt][4 * i + 3]};
            }
        return;
    }
    __bf16* dkp = dK + ((long)b * S + key) * ld_dkv + (long)hk * D;
    __bf16* dvp = dV + ((long)b * S + key) * ld_dkv + (long)hk * D;
#pragma unroll
    for (int dt = 0; dt < 2; ++dt)
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

// ---------------------------------------------------------------------------------------------------------
// Ping-pong dQ kernel (the default for the split form).  Same math as fa_bwd_dq_kernel, on the schedule of
// fa_bwd_dkv_pp_kernel: 8 waves in two staggered groups, waves w and w + 4 (one SIMD) owning adjacent 32-query
// blocks (queries q0 + 64 (w & 3) + 32 (w >> 2)); per half-step j = 2 t + h (key tile t, 32-key half h):
//   M(j): dQ^T += K^T.dS^T of half-step j - 1 (its transposed K fragments and bf16 dS read / packed in V(j - 1)),
//         then S^T = K.(cQ)^T - lse and dP^T = V.dO^T - delta of half-step j (12 MFMAs)
//   V(j): P^T = exp2(S^T), dS^T = P^T dP^T, bf16 packing, the transposed K reads for M(j + 1), and the staging of
//         the next key tile (group g the rows [32 g, +32) of K and V, from registers loaded in V(2t - 2)).
// delta = rowsum(dO * O) is computed in the prologue and written for the dK/dV kernel, as in fa_bwd_dq_kernel.
template <bool CAUSAL, bool ROPE, bool ROPE_IN>
__global__ void __launch_bounds__(PPNW * 64, 1)
fa_bwd_dq_pp_kernel(const __bf16* __restrict__ Q, const __bf16* __restrict__ K, const __bf16* __restrict__ Vv,
                    long ld_q, long ld_kv, const __bf16* __restrict__ O, long ld_o, const __bf16* __restrict__ dO,
                    long ld_do, const float* __restrict__ LSE, float* __restrict__ DELTA, __bf16* __restrict__ dQ,
                    long ld_dq, const float* __restrict__ cosT, const float* __restrict__ sinT, int B, int H, int Hkv,
                    int S, float scale_log2, float scale, int group) {
    constexpr int QB = 32 * PPNW;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    char* Ks = smem;             // [2][64 keys][128 B]  (roped K)
    char* Vs = smem + 2 * TILE;  // [2][64 keys][128 B]

    const int tid = threadIdx.x, l = tid & 63, l31 = l & 31, hh = l >> 5;
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int g = w >> 2, wl = w & 3, gt = tid & 255;
    const int nqb = (S + QB - 1) / QB;
    int rank, bh;
    grouped_order((int)blockIdx.x, nqb, B * H, group, rank, bh);
    const int qblk = CAUSAL ? nqb - 1 - rank : rank;
    const int b = bh / H, h = bh % H, hk = h / (H / Hkv);
    const int q0 = qblk * QB, qw = q0 + 64 * wl + 32 * g, q = qw + l31;
    const bool q_ok = q < S;
    const long qc = q_ok ? q : S - 1;
    const long qrow = (long)b * S + qc;

    bf16x8 qf[KS], of[KS];
    float dsum = 0.f;
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
        const int d0 = 16 * ks + 8 * hh;
        u16x8 tq = *reinterpret_cast<const u16x8*>(Q + qrow * ld_q + (long)h * D + d0);
        if (ROPE_IN) {
            tq = rope_u16x8(tq, cosT + qc * (D / 2) + d0 / 2, sinT + qc * (D / 2) + d0 / 2, scale_log2);
        } else {
            float x[8];
            unpack8(tq, x);
            tq = pack8(x, scale_log2);
        }
        qf[ks] = __builtin_bit_cast(bf16x8, tq);
        const u16x8 tg = *reinterpret_cast<const u16x8*>(dO + qrow * ld_do + (long)h * D + d0);
        const u16x8 to = *reinterpret_cast<const u16x8*>(O + qrow * ld_o + (long)h * D + d0);
#pragma unroll
        for (int i = 0; i < 8; ++i) dsum += bf2f(tg[i]) * bf2f(to[i]);
        of[ks] = __builtin_bit_cast(bf16x8, tg);
    }
    dsum += __shfl_xor(dsum, 32, 64);
    if (q_ok && hh == 0) DELTA[((long)b * H + h) * S + q] = dsum;
    const float lse = LSE[((long)b * H + h) * S + qc];
    const float nl = (q_ok && lse < INFINITY) ? -lse : -INFINITY;
    f32x16 ns, nd;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
        ns[r] = nl;
        nd[r] = -dsum;
    }
    f32x16 acc[2];
#pragma unroll
    for (int dt = 0; dt < 2; ++dt)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[dt][r] = 0.f;

    const int kend = CAUSAL ? min(S, q0 + QB) : S;
    const int nkt = (kend + 63) / 64;
    const int J = 2 * nkt;
    const __bf16* kb = K + (long)b * S * ld_kv + (long)hk * D;
    const __bf16* vb = Vv + (long)b * S * ld_kv + (long)hk * D;
    const int srow = 32 * g + (gt >> 3), sc = gt & 7;
    u16x8 kreg, vreg;
    auto load_tile = [&](int t) {
        const long kk = min(t * 64 + srow, S - 1);
        kreg = *reinterpret_cast<const u16x8*>(kb + kk * ld_kv + sc * 8);
        vreg = *reinterpret_cast<const u16x8*>(vb + kk * ld_kv + sc * 8);
    };
    auto write_tile = [&](int t) {
        const bool ok = t * 64 + srow < S;
        u16x8 kv = ok ? kreg : u16x8{0, 0, 0, 0, 0, 0, 0, 0};
        const u16x8 vv = ok ? vreg : u16x8{0, 0, 0, 0, 0, 0, 0, 0};
        if (ROPE_IN) {
            const long kk = min(t * 64 + srow, S - 1);
            kv = rope_u16x8(kv, cosT + kk * (D / 2) + sc * 4, sinT + kk * (D / 2) + sc * 4, 1.f);
        }
        *reinterpret_cast<u16x8*>(Ks + (t & 1) * TILE + swz<RB>(srow, sc)) = kv;
        *reinterpret_cast<u16x8*>(Vs + (t & 1) * TILE + swz<RB>(srow, sc)) = vv;
    };

    const int trow = 4 * hh + ((l & 15) >> 2);
    const int tcol = 16 * ((l >> 4) & 1) + 4 * (l & 3);
    if (nkt > 0) {
        load_tile(0);
        write_tile(0);
        if (nkt > 1) load_tile(1);
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    pp_bar();
    if (g == 1) pp_bar();

    f32x16 sp, dp;
    bf16x8 db[2];      // bf16 dS^T of the previous half-step, k-steps s = 0, 1
    bf16x8 kt_[2][2];  // its transposed K fragments [s][dt]
    bool prev_active = false;
    for (int j = 0; j <= J; ++j) {
        const int t = j >> 1, hf = j & 1, k0 = t * 64 + 32 * hf;
        const bool active = j < J && (!CAUSAL || k0 <= qw + 31);
        // ---------------- M(j)
        {
            if (prev_active) {
#pragma unroll
                for (int ss = 0; ss < 2; ++ss)
#pragma unroll
                    for (int dt = 0; dt < 2; ++dt) acc[dt] = mfma(kt_[ss][dt], db[ss], acc[dt]);
            }
            __builtin_amdgcn_sched_barrier(0);
            if (active) {
                const char* Kc = Ks + (t & 1) * TILE;
                const char* Vc = Vs + (t & 1) * TILE;
                sp = ns;
                dp = nd;
#pragma unroll
                for (int ks = 0; ks < KS; ++ks) {
                    const int koff = swz<RB>(32 * hf + l31, 2 * ks + hh);
                    sp = mfma(lds_row16(Kc, koff), qf[ks], sp);
                    dp = mfma(lds_row16(Vc, koff), of[ks], dp);
                }
            }
        }
        pp_bar();
        if (j == J) break;
        // ---------------- V(j)
        {
            char* Kc = Ks + (t & 1) * TILE;
            if (active) {
                const bool need_mask = (CAUSAL && k0 + 31 > qw) || (k0 + 32 > S);
                if (need_mask) {
#pragma unroll
                    for (int r = 0; r < 16; ++r) {
                        const int key = k0 + acc_row(r, hh);
                        const float p = fast_exp2(sp[r]);
                        const bool ok = key < S && (!CAUSAL || key <= q);
                        dp[r] = ok ? p * dp[r] : 0.f;
                    }
                } else {
#pragma unroll
                    for (int r = 0; r < 16; ++r) dp[r] = fast_exp2(sp[r]) * dp[r];
                }
#pragma unroll
                for (int ss = 0; ss < 2; ++ss) {
#pragma unroll
                    for (int jj = 0; jj < 8; ++jj) db[ss][jj] = (__bf16)dp[8 * ss + jj];
                    const int kr = 32 * hf + 16 * ss;
#pragma unroll
                    for (int dt = 0; dt < 2; ++dt)
                        kt_[ss][dt] = lds_tr_pair(Kc, tr_off<RB>(kr + trow, 32 * dt + tcol),
                                                  tr_off<RB>(kr + 8 + trow, 32 * dt + tcol));
                }
            }
            prev_active = active;
            if (hf == 0 && t + 1 < nkt) {
                write_tile(t + 1);
                if (t + 2 < nkt) load_tile(t + 2);
            }
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        }
        pp_bar();
    }
    if (g == 0) pp_bar();

    if (q_ok) {
        __bf16* dqp = dQ + ((long)b * S + q) * ld_dq + (long)h * D;
#pragma unroll
        for (int dt = 0; dt < 2; ++dt)
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

}  // namespace split
}  // namespace fa
}  // namespace bpe

using namespace bpe;
using namespace bpe::fa;

// Backward form: 0 = split (default for D = 64), 1 = fused (flash_attn_bwd.hip, the atomics form).  Initial value
// from BPE_FA_BWD ("fused" / "split"), changeable at run time (fa_bwd_config) for same-process A/B and tests.
// Waves per workgroup of the two split kernels: BPE_FA_SPLIT_NW="<dq>,<dkv>", each 4 or 8 (the plain kernels with
// register-staged tiles), 42 / 43 (4 waves, tiles staged by LDS-DMA, 2 / 3 waves per SIMD), 44 (42 with every
// operand read of a half-step issued ahead of its MFMAs, SCHED), 47 / 48 (42 / 44 with 128-key / 128-query tiles,
// one barrier per 128 rows), 82 (8 waves, LDS-DMA) or 2 (the ping-pong kernels: 8 waves in two staggered groups).
// Default 48,47 (the dK/dV kernel without the batched reads: 215 VGPRs instead of 256 with 2 spilled, and
// 1.1437 vs 1.1465 ms for 48,48; ab_attn_sched128.log).  Op-level, same box each: LDS-DMA staging 1.178-1.204 vs
// 1.207-1.277 ms for 4,4 (GPT-2 B 128) and 0.666 vs 0.702 ms (Llama GQA) (profiles/bench/ab_attn_dma_occ.log); the
// batched reads another -0.4-0.5 % (ab_attn_sched.log); 128-row tiles: dQ 1.159 vs 1.162 ms (ab_attn_dq128.log),
// dK/dV 1.168 vs 1.179 ms, Llama B 32 2.159 vs 2.208 ms (ab_attn_dkv128.log).
// Measured and dropped: 43 (168 VGPRs: 27-275 spilled, 2.5x slower), 82 (+10 %), a two-half software pipeline of
// the dK/dV kernel (S/dP of half 1 under the softmax of half 0, sched_group_barrier 1 MFMA : 5 VALU; +2.3 %), the
// ping-pong pair (+13-27 %, ab_attn_pp_b128.log).
static int g_mode = -1, g_nw_dq = 48, g_nw_dkv = 47;
// GQA dK / dV: 1 = one workgroup per KV head sweeping its G query heads (the plain split kernels), 0 = one per query
// head with fp32 partials summed by fa_dkv_reduce_kernel.  BPE_FA_GQA_LOOP sets it, fa_gqa_loop_config at run time.
static int g_gqa_loop = 1;

static int nw_code(int v) {
    return (v == 8 || v == 4 || v == 42 || v == 43 || v == 82 || v == 44 || v == 48 || v == 47) ? v : 2;
}

static void config_init() {
    if (g_mode >= 0) return;
    if (const char* e = getenv("BPE_FA_GQA_LOOP")) g_gqa_loop = atoi(e) ? 1 : 0;
    const char* e = getenv("BPE_FA_BWD");
    g_mode = (e && e[0] == 'f') ? 1 : 0;
    if (const char* n = getenv("BPE_FA_SPLIT_NW")) {
        int a = 4, c = 4;
        if (sscanf(n, "%d,%d", &a, &c) >= 1) {
            g_nw_dq = nw_code(a);
            g_nw_dkv = nw_code(c);
        }
    }
}

bool fa_bwd_split_active(int D) {
    config_init();
    return D == 64 && g_mode == 0;
}

// mode < 0 / nw <= 0 leave a setting unchanged; returns the mode in force afterwards
int fa_bwd_config(int mode, int nw_dq, int nw_dkv) {
    config_init();
    if (mode >= 0) g_mode = mode ? 1 : 0;
    if (nw_dq > 0) g_nw_dq = nw_code(nw_dq);
    if (nw_dkv > 0) g_nw_dkv = nw_code(nw_dkv);
    return g_mode;
}

template <bool C, bool R, bool RIN, int NW, int OCC = 2, bool DMA = false, bool SCHED = false, int KT = 64>
static void dq_launch(const FaArgs& a, hipStream_t s) {
    const int nqb = (a.S + 32 * NW - 1) / (32 * NW);
    const int lds = 4 * split::TILE * ((DMA && !RIN) ? KT / 64 : 1);
    split::fa_bwd_dq_kernel<C, R, RIN, NW, OCC, DMA, SCHED, KT><<<nqb * a.B * a.H, NW * 64, lds, s>>>(
        a.q, a.k, a.v, a.ld_q, a.ld_kv, a.o, a.ld_o, a.dout, a.ld_do, a.lse, a.delta, a.dq, a.ld_dq, a.cos, a.sin,
        a.B, a.H, a.Hkv, a.S, a.scale * LOG2E, a.scale, fa_group(a.B * a.H));
}

template <bool C, bool R, bool RIN, int NW, int OCC = 2, bool DMA = false, bool SCHED = false, int QT = 64>
static void dkv_launch(const FaArgs& a, hipStream_t s) {
    const int nkb = (a.S + 32 * NW - 1) / (32 * NW);
    const int qt = (DMA && !RIN) ? QT : 64;
    const int lds = 4 * split::TILE * (qt / 64) + 16 * qt;  // Q / dO buffers + the -lse / -delta rows
    if (a.Hkv < a.H && g_gqa_loop) {  // GQA: one workgroup per KV head sweeps its query heads (no partials / reduce)
        split::fa_bwd_dkv_kernel<C, R, RIN, NW, OCC, DMA, SCHED, true, QT>
            <<<nkb * a.B * a.Hkv, NW * 64, lds, s>>>(
                a.q, a.k, a.v, a.ld_q, a.ld_kv, a.dout, a.ld_do, a.lse, a.delta, a.dk, a.dv, a.ld_dkv, a.dkv_part,
                a.cos, a.sin, a.B, a.H, a.Hkv, a.S, a.scale * LOG2E, a.scale, fa_group(a.B * a.Hkv));
        return;
    }
    split::fa_bwd_dkv_kernel<C, R, RIN, NW, OCC, DMA, SCHED, false, QT><<<nkb * a.B * a.H, NW * 64, lds, s>>>(
        a.q, a.k, a.v, a.ld_q, a.ld_kv, a.dout, a.ld_do, a.lse, a.delta, a.dk, a.dv, a.ld_dkv, a.dkv_part, a.cos,
        a.sin, a.B, a.H, a.Hkv, a.S, a.scale * LOG2E, a.scale, fa_group(a.B * a.H));
}

template <bool C, bool R, bool RIN>
static void dq_pp_launch(const FaArgs& a, hipStream_t s) {
    const int nqb = (a.S + 32 * split::PPNW - 1) / (32 * split::PPNW);
    split::fa_bwd_dq_pp_kernel<C, R, RIN><<<nqb * a.B * a.H, split::PPNW * 64, 4 * split::TILE, s>>>(
        a.q, a.k, a.v, a.ld_q, a.ld_kv, a.o, a.ld_o, a.dout, a.ld_do, a.lse, a.delta, a.dq, a.ld_dq, a.cos, a.sin,
        a.B, a.H, a.Hkv, a.S, a.scale * LOG2E, a.scale, fa_group(a.B * a.H));
}

template <bool C, bool R, bool RIN>
static void dkv_pp_launch(const FaArgs& a, hipStream_t s) {
    const int nkb = (a.S + 32 * split::PPNW - 1) / (32 * split::PPNW);
    split::fa_bwd_dkv_pp_kernel<C, R, RIN><<<nkb * a.B * a.H, split::PPNW * 64, 4 * split::TILE + 1024, s>>>(
        a.q, a.k, a.v, a.ld_q, a.ld_kv, a.dout, a.ld_do, a.lse, a.delta, a.dk, a.dv, a.ld_dkv, a.dkv_part, a.cos,
        a.sin, a.B, a.H, a.Hkv, a.S, a.scale * LOG2E, a.scale, fa_group(a.B * a.H));
}

template <bool C, bool R, bool RIN>
static void split_launch(const FaArgs& a, hipStream_t s) {
    config_init();
    const int nq = g_nw_dq, nk = g_nw_dkv;
    if (nq == 2) dq_pp_launch<C, R, RIN>(a, s);
    else if (nq == 8) dq_launch<C, R, RIN, 8>(a, s);
    else if (nq == 42) dq_launch<C, R, RIN, 4, 2, true>(a, s);
    else if (nq == 43) dq_launch<C, R, RIN, 4, 3, true>(a, s);
    else if (nq == 82) dq_launch<C, R, RIN, 8, 2, true>(a, s);
    else if (nq == 44) dq_launch<C, R, RIN, 4, 2, true, true>(a, s);
    else if (nq == 48) dq_launch<C, R, RIN, 4, 2, true, true, 128>(a, s);
    else if (nq == 47) dq_launch<C, R, RIN, 4, 2, true, false, 128>(a, s);
    else dq_launch<C, R, RIN, 4>(a, s);
    if (nk == 2) dkv_pp_launch<C, R, RIN>(a, s);
    else if (nk == 8) dkv_launch<C, R, RIN, 8>(a, s);
    else if (nk == 42) dkv_launch<C, R, RIN, 4, 2, true>(a, s);
    else if (nk == 43) dkv_launch<C, R, RIN, 4, 3, true>(a, s);
    else if (nk == 82) dkv_launch<C, R, RIN, 8, 2, true>(a, s);
    else if (nk == 44) dkv_launch<C, R, RIN, 4, 2, true, true>(a, s);
    else if (nk == 48) dkv_launch<C, R, RIN, 4, 2, true, true, 128>(a, s);
    else if (nk == 47) dkv_launch<C, R, RIN, 4, 2, true, false, 128>(a, s);
    else dkv_launch<C, R, RIN, 4>(a, s);
}

void launch_fa_dkv_reduce(const FaArgs& a, hipStream_t s);  // flash_attn_bwd.hip

// whether a GQA backward of head size D needs the fp32 dK / dV partials buffer (FaArgs::dkv_part): the fused
// backward and the ping-pong dK / dV kernel always do, the plain split kernels only with the KV-head sweep off
bool fa_dkv_partials_needed(int D) {
    config_init();
    return !fa_bwd_split_active(D) || !g_gqa_loop || g_nw_dkv == 2;
}

// set the GQA dK / dV form (v >= 0), return the one in force
int fa_gqa_loop_config(int v) {
    config_init();
    if (v >= 0) g_gqa_loop = v ? 1 : 0;
    return g_gqa_loop;
}

bool launch_fa_bwd_split(const FaArgs& a, hipStream_t s) {
    if (!fa_bwd_split_active(a.D)) return false;
    // rope: 0 none, 1 rotate Q / K on load and dQ / dK on output, 2 outputs only (Q / K pre-rotated)
    if (a.causal) {
        if (a.rope == 1) split_launch<true, true, true>(a, s);
        else if (a.rope == 2) split_launch<true, true, false>(a, s);
        else split_launch<true, false, false>(a, s);
    } else {
        if (a.rope == 1) split_launch<false, true, true>(a, s);
        else if (a.rope == 2) split_launch<false, true, false>(a, s);
        else split_launch<false, false, false>(a, s);
    }
    if (a.Hkv < a.H && fa_dkv_partials_needed(a.D)) launch_fa_dkv_reduce(a, s);
    return true;
}
