// Flash attention backward with fused RoPE, gfx950 (MI355X).
// build-flags: -fno-slp-vectorize   (no packed f32 VALU beside the MFMAs: ops/build.py file_flags)
//
// Parity target: the gradient of reference contracts K7/K10
// (`tests/adapters.py:92-184`); checked against autograd of the fp32 oracle.
//
// Structure: one workgroup = NW waves x 32 keys of one (batch, kv-head)
// (NW = 8 -> 256 keys for D = 64; NW = 4 -> 128 keys for D = 128, where LDS
// is the limit).  Each wave keeps its 32 keys' K and V rows as MFMA B-operand
// fragments in registers and its dK^T / dV^T tiles in accumulators for the
// whole sweep over query tiles (64 queries per step), so dK and dV never need
// a cross-workgroup sum.  Per query tile:
//   S  = Q.K^T   and  dP = dO.V^T      (key on the lane, queries in registers;
//                                        A operands: Q / dO rows, ds_read_b128)
//   P  = exp2(S * scale*log2e - LSE2),  dS = P * (dP - delta)
//   dV^T += dO^T.P,  dK^T += Q^T.dS     (B operands straight from the P / dS
//                                        accumulators; A = dO^T / Q^T via
//                                        ds_read_b64_tr_b16 of the same images)
//   dS^T -> LDS (8-byte writes), then dQ = dS.K for the workgroup's keys:
//   16x16x32 MFMA blocks, 2 (D = 64) per wave over all the workgroup's keys
//   (no key split, no partial-sum exchange), added to an fp32 buffer with
//   float atomics (guide G12).  256-key workgroups halve the atomic bytes of a
//   128-key design.
// RoPE: Q tiles are rotated while staged, K once at the start; dK is
// un-rotated in the epilogue and dQ in the convert kernel.  GQA: one
// workgroup per query head; the G partial dK / dV of a kv head are summed in
// fp32 by fa_dkv_reduce_kernel.  Order: heaviest key blocks first.
#include "fa_common.h"
#include "kernels.h"

#include <algorithm>
#include <cstdlib>

namespace bpe {
namespace fa {

template <int D> struct BwdCfg {
    // waves per workgroup, Q / dO buffers, workgroups per CU.  (Measured alternative: two independent
    // 4-wave / 128-key workgroups per CU with single-buffered Q / dO -- 20-30 % slower: twice the dQ atomics
    // and no gain from the de-phased waves.)
    static constexpr int NW = (D == 64) ? 8 : 4, QBUF = 2, WGS = 1;
    static constexpr int KB = 32 * NW;                                  // keys per workgroup
    static constexpr int RB = D * 2;
    static constexpr int QT = 64 * RB;                                  // bytes per 64-query tile
    static constexpr int DT = D / 32;
    static constexpr size_t LDS_Q = QBUF * QT, LDS_DO = QBUF * QT;
    static constexpr size_t LDS_K = (size_t)KB * RB;  // K (roped) and V of the workgroup's keys, each
    static constexpr size_t LDS_DST = (size_t)KB * 128;
    static constexpr size_t LDS_STATS = 4 * 64 * 4;
    static constexpr size_t LDS = LDS_Q + LDS_DO + 2 * LDS_K + LDS_DST + LDS_STATS;
};

// delta = rowsum(dO * O) per (b, h, s)
template <int D, bool NT>
__global__ void __launch_bounds__(256) fa_bwd_pre_kernel(const __bf16* __restrict__ O, long ld_o,
                                                         const __bf16* __restrict__ dO, long ld_do,
                                                         float* __restrict__ delta, float* __restrict__ dq_acc,
                                                         int B, int H, int S, int spad) {
    // one row per (b, s < spad, h): delta = rowsum(O * dO) for s < S, and -- unless the forward already did
    // (dq_acc == nullptr) -- the row's fp32 dQ accumulator zeroed (pad rows s >= S only get the zeros)
    constexpr int LPR = D / 8;
    const long row = ((long)blockIdx.x * 256 + threadIdx.x) / LPR;
    const int sub = threadIdx.x % LPR;
    const long total = (long)B * spad * H;
    float acc = 0.f;
    const bool in = row < total;
    long b = 0;
    int s = 0, h = 0;
    if (in) {
        const long bsp = row / H;
        h = (int)(row % H);
        b = bsp / spad;
        s = (int)(bsp % spad);
        if (dq_acc != nullptr) {
            float4* z = reinterpret_cast<float4*>(dq_acc + row * D + sub * 8);
            z[0] = float4{0.f, 0.f, 0.f, 0.f};
            z[1] = float4{0.f, 0.f, 0.f, 0.f};
        }
    }
    const bool ok = in && s < S;
    if (ok) {
        const long bs = b * S + s;
        const u16x8* op = reinterpret_cast<const u16x8*>(O + bs * ld_o + (long)h * D + sub * 8);
        u16x8 a = NT ? ld_stream(op) : *op;  // O is read once
        u16x8 g = *reinterpret_cast<const u16x8*>(dO + bs * ld_do + (long)h * D + sub * 8);
#pragma unroll
        for (int i = 0; i < 8; ++i) acc += bf2f(a[i]) * bf2f(g[i]);
    }
#pragma unroll
    for (int o = LPR / 2; o > 0; o >>= 1) acc += __shfl_xor(acc, o, 64);
    if (ok && sub == 0) delta[(b * H + h) * S + s] = acc;
}

// P and dS of one 32-query half from its S / dP accumulators (key on the lane, 4 consecutive queries per
// register group), two elements per packed instruction.  The accumulators STARTED at the row constants
// (guide: "row constants as the initial accumulator"): S' = S - LSE2 / (scale*log2e), dP' = dP - delta, so
// P = exp2(scale*log2e * S') and dS = P * dP'.  MASK: zero P where (unsigned)(q - klim) >= span, with
// q = half start + row, passed as qoff = half start - klim.
template <bool MASK>
__device__ __forceinline__ void softmax_ds(f32x16& sp, f32x16& dp, int hh, float scale_log2, int qoff,
                                           unsigned span) {
    typedef float f2 __attribute__((ext_vector_type(2)));
    const f2 sc = {scale_log2, scale_log2};
#pragma unroll
    for (int r = 0; r < 16; r += 2) {
        const f2 x = f2{sp[r], sp[r + 1]} * sc;
        f2 p = {fast_exp2(x[0]), fast_exp2(x[1])};
        if constexpr (MASK) {
            const int q = qoff + acc_row(r, hh);
            p[0] = ((unsigned)q < span) ? p[0] : 0.f;
            p[1] = ((unsigned)(q + 1) < span) ? p[1] : 0.f;
        }
        const f2 d = p * f2{dp[r], dp[r + 1]};
        sp[r] = p[0];
        sp[r + 1] = p[1];
        dp[r] = d[0];
        dp[r + 1] = d[1];
    }
}

// ROPE: dK is un-rotated on output (and dQ by the convert kernel); ROPE_IN: Q / K are rotated on load too
// (false when ops.rope_qk_ rotated them in the QKV activation already, rope mode 2).
template <int D, bool CAUSAL, bool ROPE, bool ROPE_IN = ROPE>
__global__ void __launch_bounds__(BwdCfg<D>::NW * 64, BwdCfg<D>::WGS)
fa_bwd_kernel(const __bf16* __restrict__ Q, const __bf16* __restrict__ K, const __bf16* __restrict__ Vv, long ld_q,
              long ld_kv, const __bf16* __restrict__ dO, long ld_do, const float* __restrict__ LSE,
              const float* __restrict__ DELTA, float* __restrict__ dQacc, __bf16* __restrict__ dK,
              __bf16* __restrict__ dV, long ld_dkv, float* __restrict__ dKVpart, const float* __restrict__ cosT,
              const float* __restrict__ sinT, int B, int H, int Hkv, int S, float scale_log2, float scale,
              int group) {
    using C = BwdCfg<D>;
    constexpr int NW = C::NW, NT = NW * 64, RB = C::RB, CPR = D / 8, QT = C::QT;
    constexpr int SPT = (64 * CPR + NT - 1) / NT;  // staged chunks per thread per tile (Q and dO each)
    constexpr int KS = D / 16, DT = C::DT;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    char* Qs = smem;                                  // [2][64][D]
    char* dOs = Qs + C::LDS_Q;                        // [2][64][D]
    char* Kl = dOs + C::LDS_DO;                       // [KB][D]  roped K of this workgroup's keys
    char* Vl = Kl + C::LDS_K;                         // [KB][D]  V of this workgroup's keys
    char* dST = Vl + C::LDS_K;                        // [KB keys][64 q] bf16
    float* lseS = reinterpret_cast<float*>(dST + C::LDS_DST);  // [2][64]
    float* dltS = lseS + 128;                                              // [2][64]

    const int tid = threadIdx.x, w = tid >> 6, l = tid & 63, l31 = l & 31, hh = l >> 5;
    // one workgroup per (key block, batch, QUERY head): with GQA the G query heads of a kv head run in
    // parallel (their dK / dV partials are summed by fa_dkv_reduce_kernel) instead of one workgroup sweeping
    // all G heads -- with causal masking that serial sweep left most CUs idle behind the key-block-0 groups.
    const int BH = B * H;
    int kb, bh;  // kb 0 (the most query tiles under the causal mask) first inside each group of pairs
    grouped_order((int)blockIdx.x, (S + C::KB - 1) / C::KB, BH, group, kb, bh);
    const int b = bh / H, h = bh % H;
    const int G = H / Hkv;
    const int hk = h / G;
    const int kb0 = kb * C::KB, kw0 = kb0 + 32 * w;
    const int key = kw0 + l31;
    const bool key_ok = key < S;
    const long kpos = key_ok ? key : 0;

    // ---- this wave's K (roped) and V rows -> LDS (B operands of S / dP re-read per query tile,
    //      K also the B operand of dQ); nothing stays pinned in registers across the sweep
    {
        const __bf16* kp = K + ((long)b * S + kpos) * ld_kv + (long)hk * D;
        const __bf16* vp = Vv + ((long)b * S + kpos) * ld_kv + (long)hk * D;
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) {
            const int d0 = 16 * ks + 8 * hh;
            u16x8 tk = key_ok ? *reinterpret_cast<const u16x8*>(kp + d0) : u16x8{0, 0, 0, 0, 0, 0, 0, 0};
            u16x8 tv = key_ok ? *reinterpret_cast<const u16x8*>(vp + d0) : u16x8{0, 0, 0, 0, 0, 0, 0, 0};
            if (ROPE_IN) tk = rope_u16x8(tk, cosT + kpos * (D / 2) + d0 / 2, sinT + kpos * (D / 2) + d0 / 2, 1.f);
            *reinterpret_cast<u16x8*>(Kl + swz<RB>(32 * w + l31, 2 * ks + hh)) = tk;
            *reinterpret_cast<u16x8*>(Vl + swz<RB>(32 * w + l31, 2 * ks + hh)) = tv;
        }
    }

    f32x16 dk[DT], dv[DT];
#pragma unroll
    for (int dt = 0; dt < DT; ++dt)
#pragma unroll
        for (int r = 0; r < 16; ++r) { dk[dt][r] = 0.f; dv[dt][r] = 0.f; }

    const int m_start = CAUSAL ? kb0 : 0;  // kb0 is a multiple of 128 -> 64-aligned
    const int nqt = (S - m_start + 63) / 64;
    const int total_it = nqt;

    u16x8 qreg[SPT], oreg[SPT];
    float lreg = 0.f, dreg = 0.f;
    auto load_tile = [&](int it) {
        // every load unconditional (rows past the end clamped to S-1, their values zeroed at the LDS write; the
        // stats rows loaded by all waves, used by wave 0): straight-line code keeps the wait-count pass's
        // in-order vmcnt count exact, so write_tile waits for these loads and not for the dQ atomics after them
        const int m0 = m_start + it * 64;
        const __bf16* qb = Q + (long)b * S * ld_q + (long)h * D;
        const __bf16* ob = dO + (long)b * S * ld_do + (long)h * D;
#pragma unroll
        for (int i = 0; i < SPT; ++i) {
            const int e = min(tid + NT * i, 64 * CPR - 1), row = e / CPR, c = e % CPR;
            const long qq = min(m0 + row, S - 1);
            qreg[i] = *reinterpret_cast<const u16x8*>(qb + qq * ld_q + c * 8);
            oreg[i] = *reinterpret_cast<const u16x8*>(ob + qq * ld_do + c * 8);
        }
        {
            const long idx = ((long)b * H + h) * S + min(m0 + l, S - 1);
            lreg = LSE[idx];
            dreg = DELTA[idx];
        }
    };
    auto write_tile = [&](int it, int buf) {
        const int m0 = m_start + it * 64;
#pragma unroll
        for (int i = 0; i < SPT; ++i) {
            const int e = tid + NT * i, row = e / CPR, c = e % CPR;
            if (e >= 64 * CPR) break;
            const bool ok = m0 + row < S;
            u16x8 qv = ok ? qreg[i] : u16x8{0, 0, 0, 0, 0, 0, 0, 0};
            const u16x8 ov = ok ? oreg[i] : u16x8{0, 0, 0, 0, 0, 0, 0, 0};
            if (ROPE_IN) {
                const long qq = min(m0 + row, S - 1);
                qv = rope_u16x8(qv, cosT + qq * (D / 2) + c * 4, sinT + qq * (D / 2) + c * 4, 1.f);
            }
            *reinterpret_cast<u16x8*>(Qs + buf * QT + swz<RB>(row, c)) = qv;
            *reinterpret_cast<u16x8*>(dOs + buf * QT + swz<RB>(row, c)) = ov;
        }
        if (tid < 64) {
            // the S / dP accumulators' starting values: -LSE2 / (scale*log2e) and -delta
            const bool ok = m0 + tid < S;
            lseS[buf * 64 + tid] = (!ok || lreg == INFINITY) ? -INFINITY : -lreg / scale_log2;
            dltS[buf * 64 + tid] = ok ? -dreg : 0.f;
        }
    };

    load_tile(0);
    write_tile(0, 0);
    __syncthreads();

    const int trow = 4 * hh + ((l & 15) >> 2);          // tr-read row inside a 16-row k-step
    const int tcol = 16 * ((l >> 4) & 1) + 4 * (l & 3);  // tr-read column inside a 32-wide tile

    // one query tile.  (Unrolling by two so the buffer index becomes an immediate offset was measured:
    // the hoisted per-buffer addresses push the kernel past 256 VGPRs and it spills.)
    auto body = [&](int it) {
        const int cur = C::QBUF == 2 ? (it & 1) : 0;
        const int m0 = m_start + it * 64;
        if (it + 1 < total_it) load_tile(it + 1);
        char* Qc = Qs + cur * QT;
        char* Oc = dOs + cur * QT;
        const float* lc = lseS + cur * 64;
        const float* dc = dltS + cur * 64;
        const bool active = !CAUSAL || (m0 + 63 >= kw0);
        if (active) {
            // the two 32-query halves one after the other: only one S / dP accumulator pair is live
            const bool need_mask = (CAUSAL && m0 < kw0 + 31) || (m0 + 64 > S) || (kw0 + 32 > S);
            const int klim = CAUSAL ? (key_ok ? key : S) : (key_ok ? 0 : S);
            const unsigned span = (unsigned)(S - klim);
#pragma unroll
            for (int qt = 0; qt < 2; ++qt) {
                f32x16 sp, dp;
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    const int qi = qt * 32 + 8 * i + 4 * hh;  // rows qi..qi+3 of registers 4i..4i+3
                    const f32x4 lv = *reinterpret_cast<const f32x4*>(lc + qi);
                    const f32x4 dl = *reinterpret_cast<const f32x4*>(dc + qi);
#pragma unroll
                    for (int j = 0; j < 4; ++j) { sp[4 * i + j] = lv[j]; dp[4 * i + j] = dl[j]; }
                }
#pragma unroll
                for (int ks = 0; ks < KS; ++ks) {
                    const int koff = swz<RB>(32 * w + l31, 2 * ks + hh);
                    const int off = swz<RB>(qt * 32 + l31, 2 * ks + hh);
                    sp = mfma(lds_row16(Qc, off), lds_row16(Kl, koff), sp);
                    dp = mfma(lds_row16(Oc, off), lds_row16(Vl, koff), dp);
                }
                // P = exp2(S * scale*log2e - LSE2), dS = P * (dP - delta); diagonal / ragged tiles (wave-uniform
                // test, scalar branch) zero P where (unsigned)(q - klim) >= span
                if (need_mask)
                    softmax_ds<true>(sp, dp, hh, scale_log2, m0 + qt * 32 - klim, span);
                else
                    softmax_ds<false>(sp, dp, hh, scale_log2, 0, 0u);
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
                    for (int dt = 0; dt < DT; ++dt) {
                        const int o0 = tr_off<RB>(qr + trow, dt * 32 + tcol);
                        const int o1 = tr_off<RB>(qr + 8 + trow, dt * 32 + tcol);
                        dv[dt] = mfma(lds_tr_pair(Oc, o0, o1), pb, dv[dt]);
                        dk[dt] = mfma(lds_tr_pair(Qc, o0, o1), db, dk[dt]);
                    }
                    // dS^T -> LDS [key row][q] from the same bf16 values: elements 4g..4g+3 of db are
                    // registers 8ss+4g.. = 4 consecutive queries of group i = 2ss+g
                    const u16x8 du = __builtin_bit_cast(u16x8, db);
#pragma unroll
                    for (int g = 0; g < 2; ++g) {
                        const u16x4 t = {du[4 * g], du[4 * g + 1], du[4 * g + 2], du[4 * g + 3]};
                        *reinterpret_cast<u16x4*>(dST + swz<128>(32 * w + l31, qt * 4 + 2 * ss + g) + 8 * hh) = t;
                    }
                }
            }
        } else {
#pragma unroll
            for (int c = 0; c < 4; ++c)
                *reinterpret_cast<u16x8*>(dST + swz<128>(32 * w + l31, 2 * c + hh)) = u16x8{0, 0, 0, 0, 0, 0, 0, 0};
        }
        __syncthreads();
        // ---- dQ = dS.K over this workgroup's keys with 16x16x32 MFMA: the 64 x D tile is 4 x D/16 blocks
        //      of 16 x 16, TPW per wave over ALL keys (no key split, no partial-sum exchange); the TPW blocks
        //      of a wave share their query block, so the dS^T fragments are read once per 32-key step.
        //      dQacc rows are padded to a multiple of 64 per batch: rows q >= S of the last tile land in
        //      padding (carrying zeros: P = 0 there), so the atomics need no per-element guard.
        {
            constexpr int DB = D / 16, TPW = 4 * DB / NW;
            const int t0 = w * TPW, qb = t0 / DB;
            f32x4 acc[TPW];
#pragma unroll
            for (int u = 0; u < TPW; ++u) acc[u] = f32x4{0.f, 0.f, 0.f, 0.f};
            const int lr = 8 * (l >> 4) + ((l & 15) >> 2), lc4 = 4 * (l & 3);
#pragma unroll
            for (int ks = 0; ks < C::KB / 32; ++ks) {
                const int kr = 32 * ks + lr;
                const bf16x8 a = lds_tr_pair(dST, tr_off<128>(kr, qb * 16 + lc4), tr_off<128>(kr + 4, qb * 16 + lc4));
#pragma unroll
                for (int u = 0; u < TPW; ++u) {
                    const int dc2 = ((t0 + u) % DB) * 16 + lc4;
                    const bf16x8 bb = lds_tr_pair(Kl, tr_off<RB>(kr, dc2), tr_off<RB>(kr + 4, dc2));
                    acc[u] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, bb, acc[u], 0, 0, 0);
                }
            }
            // unconditional (no runtime skip flag): a conditional atomic block makes the wait-count pass take
            // the count of the path WITHOUT the atomics at the join, i.e. vmcnt(1) / vmcnt(0) before the next
            // tile's LDS writes -- which drains these atomics (~600-3000 cycles) every query tile
            {
                const long HD = (long)H * D;
                const int Spad = (S + 63) & ~63;
                float* dqp = dQacc + ((long)b * Spad + m0 + qb * 16 + 4 * (l >> 4)) * HD + (long)h * D + (l & 15);
#pragma unroll
                for (int u = 0; u < TPW; ++u)
#pragma unroll
                    for (int r = 0; r < 4; ++r) atomicAdd(dqp + r * HD + ((t0 + u) % DB) * 16, acc[u][r]);
            }
        }
        if (it + 1 < total_it) write_tile(it + 1, C::QBUF == 2 ? cur ^ 1 : 0);
        __syncthreads();
    };
    for (int it = 0; it < total_it; ++it) body(it);

    // ---- GQA: fp32 partials of this query head -> [b, s, h, {dK, dV}, D] for the reduce kernel
    if (G > 1) {
        if (key_ok) {
            float* pk = dKVpart + (((long)b * S + key) * H + h) * 2 * D;
#pragma unroll
            for (int dt = 0; dt < DT; ++dt)
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    const int d0 = dt * 32 + 8 * i + 4 * hh;
                    *reinterpret_cast<f32x4*>(pk + d0) =
                        f32x4{dk[dt][4 * i], dk[dt][4 * i + 1], dk[dt][4 * i + 2], dk[dt][4 * i + 3]};
                    *reinterpret_cast<f32x4*>(pk + D + d0) =
                        f32x4{dv[dt][4 * i], dv[dt][4 * i + 1], dv[dt][4 * i + 2], dv[dt][4 * i + 3]};
                }
        }
        return;
    }
    // ---- epilogue: dK = scale * R(-pos) dK^T, dV = dV^T  (key on the lane, d in registers)
    if (key_ok) {
        __bf16* dkp = dK + ((long)b * S + key) * ld_dkv + (long)hk * D;
        __bf16* dvp = dV + ((long)b * S + key) * ld_dkv + (long)hk * D;
#pragma unroll
        for (int dt = 0; dt < DT; ++dt)
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int d0 = dt * 32 + 8 * i + 4 * hh;
                float x[4] = {dk[dt][4 * i] * scale, dk[dt][4 * i + 1] * scale, dk[dt][4 * i + 2] * scale,
                              dk[dt][4 * i + 3] * scale};
                if (ROPE) {
#pragma unroll
                    for (int pr = 0; pr < 2; ++pr) {
                        const float c = cosT[kpos * (D / 2) + d0 / 2 + pr];
                        const float s = sinT[kpos * (D / 2) + d0 / 2 + pr];
                        const float a = x[2 * pr], bb = x[2 * pr + 1];
                        x[2 * pr] = a * c + bb * s;
                        x[2 * pr + 1] = -a * s + bb * c;
                    }
                }
                u16x4 tk = {f2bf(x[0]), f2bf(x[1]), f2bf(x[2]), f2bf(x[3])};
                u16x4 tv = {f2bf(dv[dt][4 * i]), f2bf(dv[dt][4 * i + 1]), f2bf(dv[dt][4 * i + 2]),
                            f2bf(dv[dt][4 * i + 3])};
                *reinterpret_cast<u16x4*>(dkp + d0) = tk;
                *reinterpret_cast<u16x4*>(dvp + d0) = tv;
            }
    }
}

// GQA: dK = scale * R(-pos) sum_g dK_g, dV = sum_g dV_g over the G query heads of each kv head
template <int D, bool ROPE>
__global__ void __launch_bounds__(256) fa_dkv_reduce_kernel(const float* __restrict__ part, __bf16* __restrict__ dK,
                                                            __bf16* __restrict__ dV, long ld_dkv,
                                                            const float* __restrict__ cosT,
                                                            const float* __restrict__ sinT, int B, int H, int Hkv,
                                                            int S, float scale) {
    const int G = H / Hkv;
    const long total = (long)B * S * Hkv * (D / 4);
    for (long i = blockIdx.x * 256L + threadIdx.x; i < total; i += (long)gridDim.x * 256) {
        const long row = i / (D / 4);  // (b, s, hk)
        const int d0 = (int)(i % (D / 4)) * 4;
        const long bs = row / Hkv;
        const int hk = (int)(row % Hkv);
        const long s = bs % S;
        const float* p = part + (bs * H + (long)hk * G) * 2 * D + d0;
        f32x4 k4 = {0.f, 0.f, 0.f, 0.f}, v4 = {0.f, 0.f, 0.f, 0.f};
        for (int g = 0; g < G; ++g) {
            k4 += *reinterpret_cast<const f32x4*>(p + (long)g * 2 * D);
            v4 += *reinterpret_cast<const f32x4*>(p + (long)g * 2 * D + D);
        }
        float x[4] = {k4[0] * scale, k4[1] * scale, k4[2] * scale, k4[3] * scale};
        if (ROPE) {
#pragma unroll
            for (int pr = 0; pr < 2; ++pr) {
                const float c = cosT[s * (D / 2) + d0 / 2 + pr];
                const float sn = sinT[s * (D / 2) + d0 / 2 + pr];
                const float a = x[2 * pr], bb = x[2 * pr + 1];
                x[2 * pr] = a * c + bb * sn;
                x[2 * pr + 1] = -a * sn + bb * c;
            }
        }
        *reinterpret_cast<u16x4*>(dK + bs * ld_dkv + (long)hk * D + d0) = u16x4{f2bf(x[0]), f2bf(x[1]), f2bf(x[2]),
                                                                                 f2bf(x[3])};
        *reinterpret_cast<u16x4*>(dV + bs * ld_dkv + (long)hk * D + d0) = u16x4{f2bf(v4[0]), f2bf(v4[1]),
                                                                                 f2bf(v4[2]), f2bf(v4[3])};
    }
}

// dQ (fp32, roped space, unscaled) -> bf16 output slice: dq = scale * R(-pos) dQacc
template <int D, bool ROPE, bool NT>
__global__ void __launch_bounds__(256) fa_dq_convert_kernel(const float* __restrict__ dQacc, __bf16* __restrict__ dq,
                                                            long ld_dq, const float* __restrict__ cosT,
                                                            const float* __restrict__ sinT, int B, int H, int S,
                                                            float scale) {
    const long total = (long)B * S * H * (D / 4);
    for (long i = blockIdx.x * 256L + threadIdx.x; i < total; i += (long)gridDim.x * 256) {
        const long row = i / (D / 4);  // (b, s, h)
        const int d0 = (int)(i % (D / 4)) * 4;
        const long bs = row / H;
        const int h = (int)(row % H);
        const long s = bs % S;
        const long src = ((bs / S) * ((S + 63) & ~63) + s) * H + h;  // padded dQacc row
        const f32x4* vp = reinterpret_cast<const f32x4*>(dQacc + src * D + d0);
        f32x4 v = NT ? ld_stream(vp) : *vp;  // read once
        float x[4] = {v[0] * scale, v[1] * scale, v[2] * scale, v[3] * scale};
        if (ROPE) {
#pragma unroll
            for (int pr = 0; pr < 2; ++pr) {
                const float c = cosT[s * (D / 2) + d0 / 2 + pr];
                const float sn = sinT[s * (D / 2) + d0 / 2 + pr];
                const float a = x[2 * pr], bb = x[2 * pr + 1];
                x[2 * pr] = a * c + bb * sn;
                x[2 * pr + 1] = -a * sn + bb * c;
            }
        }
        u16x4 t = {f2bf(x[0]), f2bf(x[1]), f2bf(x[2]), f2bf(x[3])};
        *reinterpret_cast<u16x4*>(dq + bs * ld_dq + (long)h * D + d0) = t;
    }
}

}  // namespace fa
}  // namespace bpe

using namespace bpe;
using namespace bpe::fa;

size_t fa_bwd_lds_bytes(int D) { return D == 64 ? BwdCfg<64>::LDS : BwdCfg<128>::LDS; }

template <int D, bool C, bool R, bool RIN>
static void bwd_main_k(const FaArgs& a, hipStream_t s, int nkb) {
    using Cfg = BwdCfg<D>;
    static bool lds_attr = false;  // > 64 KiB of dynamic LDS: opt in once (before any graph capture)
    if (!lds_attr) {
        (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&fa_bwd_kernel<D, C, R, RIN>),
                                  hipFuncAttributeMaxDynamicSharedMemorySize, (int)Cfg::LDS);
        lds_attr = true;
    }
    fa_bwd_kernel<D, C, R, RIN><<<nkb * a.B * a.H, Cfg::NW * 64, Cfg::LDS, s>>>(
        a.q, a.k, a.v, a.ld_q, a.ld_kv, a.dout, a.ld_do, a.lse, a.delta, a.dq_acc, a.dk, a.dv, a.ld_dkv,
        a.dkv_part, a.cos, a.sin, a.B, a.H, a.Hkv, a.S, a.scale * LOG2E, a.scale, fa_group(a.B * a.H));
}

// stream non-temporally when a [tokens, H * D] bf16 activation is past 128 MB: GPT-2 B 128 (201 MB; its fp32 dQ
// accumulator 402 MB) gains, Llama-1.1B B 8 s2048 (67 MB, fits the 256 MB Infinity Cache with room) loses
static bool big_stream(const FaArgs& a) { return (size_t)a.B * a.S * a.H * a.D * 2 > ((size_t)128 << 20); }

template <int D, bool C, bool R>
static void bwd_launch(const FaArgs& a, hipStream_t s) {
    using Cfg = BwdCfg<D>;
    {
        const int spad = (a.S + 63) & ~63;  // dq_acc is [B][spad][H][D] fp32
        const long rows = (long)a.B * spad * a.H;
        const long threads = rows * (D / 8);
        // non-temporal loads only for large activations (big_stream: GPT-2 B 128 3-5 % faster pre / convert
        // kernels; Llama B 8, 67 MB O: 3-4 % slower with them)
        auto* pre = big_stream(a) ? &fa_bwd_pre_kernel<D, true> : &fa_bwd_pre_kernel<D, false>;
        pre<<<(unsigned)((threads + 255) / 256), 256, 0, s>>>(
            a.o, a.ld_o, a.dout, a.ld_do, a.delta, a.dq_zeroed ? nullptr : a.dq_acc, a.B, a.H, a.S, spad);
    }
    {
        const int nkb = (a.S + Cfg::KB - 1) / Cfg::KB;
        if (R && a.rope == 2)
            bwd_main_k<D, C, R, false>(a, s, nkb);  // Q / K pre-rotated: only the outputs are rotated back
        else
            bwd_main_k<D, C, R, R>(a, s, nkb);
    }
    if (a.Hkv < a.H) {
        const long tkv = (long)a.B * a.S * a.Hkv * (D / 4);
        const int g2 = (int)std::min<long>((tkv + 255) / 256, 4096);
        fa_dkv_reduce_kernel<D, R><<<g2, 256, 0, s>>>(a.dkv_part, a.dk, a.dv, a.ld_dkv, a.cos, a.sin, a.B, a.H, a.Hkv,
                                                      a.S, a.scale);
    }
    const long total = (long)a.B * a.S * a.H * (D / 4);
    const int grid = (int)std::min<long>((total + 255) / 256, 4096);
    auto* conv = big_stream(a) ? &fa_dq_convert_kernel<D, R, true> : &fa_dq_convert_kernel<D, R, false>;
    conv<<<grid, 256, 0, s>>>(a.dq_acc, a.dq, a.ld_dq, a.cos, a.sin, a.B, a.H, a.S, a.scale);
}

bool launch_fa_bwd_split(const FaArgs& a, hipStream_t s);  // flash_attn_bwd_split.hip

void launch_fa_bwd(const FaArgs& a, hipStream_t s) {
    if (launch_fa_bwd_split(a, s)) return;  // D = 64: the split (dQ kernel + dK/dV kernel) form
    // a.rope: 0 none, 1 rotate Q / K on load and dQ / dK on output, 2 outputs only (Q / K pre-rotated)
#define BWD_CASE(DD)                                                                                        \
    if (a.D == DD) {                                                                                        \
        if (a.causal) { if (a.rope) bwd_launch<DD, true, true>(a, s); else bwd_launch<DD, true, false>(a, s); } \
        else { if (a.rope) bwd_launch<DD, false, true>(a, s); else bwd_launch<DD, false, false>(a, s); }     \
        return;                                                                                             \
    }
    BWD_CASE(64) BWD_CASE(128)
#undef BWD_CASE
}
