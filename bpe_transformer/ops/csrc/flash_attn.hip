// Flash attention (forward + backward) with fused interleaved RoPE, for gfx950.
//
// Parity targets: reference contracts K7/K9/K10 (`tests/adapters.py:92-184`):
// softmax(QK^T / sqrt(d) [causal]) V, RoPE on Q and K per head with the
// interleaved pairing verified in SURVEY §0.5.
//
// Design for CDNA4 (MI355X):
//   * MFMA v_mfma_f32_32x32x16_bf16, one wave = 32 query rows (fwd) or 32 keys
//     (bwd).  Forward computes S^T = K.Q^T ("swapped" product) so each lane owns
//     ONE query row: the online-softmax max/sum are lane-local plus a single
//     lane^32 exchange (guide §B attention, T12).  The fp32 S^T accumulator is
//     reused directly, converted to bf16, as the B operand of O^T += V^T.P^T
//     (guide §3 "accumulator tile as the next MFMA's operand"), so P never
//     touches LDS.  O^T keeps the query on the lane too, so the per-row rescale
//     is a plain register multiply.
//   * V^T operands come from ds_read_b64_tr_b16 (hardware transposed LDS read,
//     guide T10).  All LDS tiles use one XOR swizzle (16-byte chunk c of row r
//     stored at c ^ sigma(r)) that is conflict-free for BOTH the ds_read_b128
//     row reads and the tr_b16 column reads (derivation in docs/kernels.md).
//   * Register-staged K/V pipeline (guide T14): global loads for tile t+1 are
//     issued before tile t's MFMAs and written to the other LDS buffer after
//     them; one barrier per tile.
//   * RoPE is applied while Q is loaded to registers and while K is staged to
//     LDS (fp32 cos/sin table, no device trig); the backward un-rotates dQ and
//     dK in its epilogues.  softmax scale * log2(e) is folded into Q so the
//     exponentials are exp2; LSE is kept in that base-2 domain.
//   * Backward: one workgroup = 4 waves = 128 keys of one (batch, kv-head);
//     dK^T/dV^T live in accumulators for the whole sweep over query tiles
//     (no cross-workgroup sum for dK/dV).  dS^T goes through LDS once and the
//     4 waves then each produce one 32x32 dQ tile for the block's 128 keys,
//     added to an fp32 dQ buffer with float atomics shaped as full 128-B row
//     segments (guide G12).  GQA: the block sweeps every query head of its
//     kv head.
//   * Block order: heaviest causal blocks first; blocks of one (batch, head)
//     differ by multiples of 8 in launch order so they share an XCD's L2 under
//     round-robin dispatch (speed only, never correctness).
#include "common.h"
#include "kernels.h"
#include <algorithm>

namespace bpe {
namespace fa {

typedef short v4s __attribute__((ext_vector_type(4)));
typedef short v8s __attribute__((ext_vector_type(8)));
typedef __attribute__((address_space(3))) v4s lds_v4s;

constexpr float LOG2E = 1.4426950408889634f;

// byte offset of 16-byte chunk c of row `row` in a swizzled tile with rows of
// RB bytes (RB = 128 or 256).
template <int RB>
__device__ __forceinline__ int swz(int row, int c) {
    if constexpr (RB == 128) {
        const int sg = (((row >> 1) & 1) << 2) | ((row >> 2) & 3);
        return row * 128 + ((c ^ sg) << 4);
    } else {
        const int sg = ((row & 3) << 2) | ((row >> 2) & 3);
        return row * 256 + ((c ^ sg) << 4);
    }
}

__device__ __forceinline__ bf16x8 lds_row16(const char* smem, int off) {
    return __builtin_bit_cast(bf16x8, *reinterpret_cast<const u16x8*>(smem + off));
}
// Two transposed 4x16 reads -> one 8-element MFMA operand fragment.
__device__ __forceinline__ bf16x8 lds_tr_pair(char* smem, int off0, int off1) {
    v4s lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s*)(smem + off0));
    v4s hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s*)(smem + off1));
    v8s c = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
    return __builtin_bit_cast(bf16x8, c);
}
// byte offset of the 8-byte tr-read granule at (row, col) of a swizzled tile
template <int RB>
__device__ __forceinline__ int tr_off(int row, int col) {
    return swz<RB>(row, col >> 3) + ((col & 7) << 1);
}

__device__ __forceinline__ f32x16 mfma(bf16x8 a, bf16x8 b, f32x16 c) {
    return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}

// accumulator register r, lane-half hh -> row index inside the 32-row tile
__device__ __forceinline__ int acc_row(int r, int hh) { return (r & 3) + 8 * (r >> 2) + 4 * hh; }

// 8 bf16 (16 B) -> fp32, optional interleaved RoPE at (pos, first pair index f0)
__device__ __forceinline__ void unpack8(const u16x8& t, float* x) {
#pragma unroll
    for (int i = 0; i < 8; ++i) x[i] = bf2f(t[i]);
}
__device__ __forceinline__ void rope8(float* x, const float* cs, const float* sn, float sign) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const float c = cs[i], s = sign * sn[i];
        const float a = x[2 * i], b = x[2 * i + 1];
        x[2 * i] = a * c - b * s;
        x[2 * i + 1] = a * s + b * c;
    }
}
__device__ __forceinline__ u16x8 pack8(const float* x, float mul) {
    u16x8 t;
#pragma unroll
    for (int i = 0; i < 8; ++i) t[i] = f2bf(x[i] * mul);
    return t;
}

// ---------------------------------------------------------------------------
// Forward
// ---------------------------------------------------------------------------
template <int D, bool CAUSAL, bool ROPE>
__global__ void __launch_bounds__(256, 2)
fa_fwd_kernel(const __bf16* __restrict__ Q, const __bf16* __restrict__ K, const __bf16* __restrict__ Vv, long ld_q,
              long ld_kv, __bf16* __restrict__ O, long ld_o, float* __restrict__ LSE, const float* __restrict__ cosT,
              const float* __restrict__ sinT, int B, int H, int Hkv, int S, float scale_log2) {
    constexpr int RB = D * 2;            // bytes per LDS row
    constexpr int CPR = D / 8;           // 16-byte chunks per row
    constexpr int TILE = 64 * RB;        // bytes per 64-row tile
    constexpr int SPT = 64 * CPR / 256;  // staged chunks per thread per tile
    constexpr int KS = D / 16;           // k-steps over head dim
    constexpr int DT = D / 32;           // 32-wide d tiles
    extern __shared__ __attribute__((aligned(16))) char smem[];
    char* Ks = smem;                 // [2][64][D]
    char* Vs = smem + 2 * TILE;      // [2][64][D]

    const int tid = threadIdx.x, w = tid >> 6, l = tid & 63, l31 = l & 31, hh = l >> 5;
    const int nqb = (S + 127) / 128;
    const int BH = B * H;
    const int qb = nqb - 1 - (int)(blockIdx.x / BH);
    const int bh = blockIdx.x % BH;
    const int b = bh / H, h = bh % H;
    const int hk = h / (H / Hkv);
    const int q0 = qb * 128, qw0 = q0 + 32 * w;
    const int qrow = qw0 + l31;
    const float* cosp = cosT;
    const float* sinp = sinT;

    // ---- Q fragments (B operand of S^T = K.Q^T), RoPE + scale folded in
    bf16x8 qf[KS];
    {
        const bool ok = qrow < S;
        const __bf16* qp = Q + ((long)b * S + (ok ? qrow : 0)) * ld_q + (long)h * D;
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) {
            const int d0 = 16 * ks + 8 * hh;
            u16x8 t = ok ? *reinterpret_cast<const u16x8*>(qp + d0) : u16x8{0, 0, 0, 0, 0, 0, 0, 0};
            float x[8];
            unpack8(t, x);
            const long qpos = ok ? qrow : 0;
            if (ROPE) rope8(x, cosp + qpos * (D / 2) + d0 / 2, sinp + qpos * (D / 2) + d0 / 2, 1.f);
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
            const int e = tid + 256 * i, row = e / CPR, c = e % CPR;
            const int key = t * 64 + row;
            if (key < S) {
                kreg[i] = *reinterpret_cast<const u16x8*>(kbase + (long)key * ld_kv + c * 8);
                vreg[i] = *reinterpret_cast<const u16x8*>(vbase + (long)key * ld_kv + c * 8);
            } else {
                kreg[i] = u16x8{0, 0, 0, 0, 0, 0, 0, 0};
                vreg[i] = u16x8{0, 0, 0, 0, 0, 0, 0, 0};
            }
        }
    };
    auto write_tile = [&](int t, int buf) {
#pragma unroll
        for (int i = 0; i < SPT; ++i) {
            const int e = tid + 256 * i, row = e / CPR, c = e % CPR;
            u16x8 kv = kreg[i];
            if (ROPE) {
                const int key = min(t * 64 + row, S - 1);
                float x[8];
                unpack8(kv, x);
                rope8(x, cosp + (long)key * (D / 2) + c * 4, sinp + (long)key * (D / 2) + c * 4, 1.f);
                kv = pack8(x, 1.f);
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
            const bool need_mask = (CAUSAL && n0 + 63 > qw0) || (n0 + 64 > S);
            if (need_mask) {
#pragma unroll
                for (int kt = 0; kt < 2; ++kt)
#pragma unroll
                    for (int r = 0; r < 16; ++r) {
                        const int key = n0 + kt * 32 + acc_row(r, hh);
                        if ((CAUSAL && key > qrow) || key >= S) s[kt][r] = -INFINITY;
                    }
            }
            float mt = -INFINITY;
#pragma unroll
            for (int kt = 0; kt < 2; ++kt)
#pragma unroll
                for (int r = 0; r < 16; ++r) mt = fmaxf(mt, s[kt][r]);
            mt = fmaxf(mt, __shfl_xor(mt, 32, 64));
            const float mn = fmaxf(m_run, mt);
            const float mu = (mn == -INFINITY) ? 0.f : mn;
            const float alpha = exp2f(m_run - mu);
            float ls = 0.f;
#pragma unroll
            for (int kt = 0; kt < 2; ++kt)
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    const float p = exp2f(s[kt][r] - mu);
                    s[kt][r] = p;
                    ls += p;
                }
            ls += __shfl_xor(ls, 32, 64);
            l_run = l_run * alpha + ls;
            m_run = mn;
#pragma unroll
            for (int dt = 0; dt < DT; ++dt)
#pragma unroll
                for (int r = 0; r < 16; ++r) o[dt][r] *= alpha;
            // P^T fragments: k-step kk = (kt, sstep) covers keys kt*32 + 16*sstep + permuted
            bf16x8 pf[4];
#pragma unroll
            for (int kk = 0; kk < 4; ++kk) {
                const int kt = kk >> 1, ss = kk & 1;
#pragma unroll
                for (int j = 0; j < 8; ++j) pf[kk][j] = (__bf16)s[kt][8 * ss + j];
            }
            // O^T += V^T . P^T   (A = V^T via transposed reads)
            const int trow = 4 * hh + ((l & 15) >> 2);
            const int tcol = 16 * ((l >> 4) & 1) + 4 * (l & 3);
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

    // ---- epilogue: O = O^T / l, stored row-per-lane (query on the lane)
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
        if (hh == 0) LSE[((long)b * H + h) * S + qrow] = (l_run > 0.f) ? m_run + log2f(l_run) : INFINITY;
    }
}

// ---------------------------------------------------------------------------
// Backward preprocess: delta = rowsum(dO * O)   [B, H, S]
// ---------------------------------------------------------------------------
template <int D>
__global__ void __launch_bounds__(256) fa_bwd_pre_kernel(const __bf16* __restrict__ O, long ld_o,
                                                         const __bf16* __restrict__ dO, long ld_do,
                                                         float* __restrict__ delta, int B, int H, int S) {
    constexpr int LPR = D / 8;  // lanes per row
    const long row = ((long)blockIdx.x * 256 + threadIdx.x) / LPR;  // (b, s, h) flattened
    const int sub = threadIdx.x % LPR;
    const long total = (long)B * S * H;
    float acc = 0.f;
    const bool ok = row < total;
    long bs = 0;
    int h = 0;
    if (ok) {
        bs = row / H;
        h = (int)(row % H);
        u16x8 a = *reinterpret_cast<const u16x8*>(O + bs * ld_o + (long)h * D + sub * 8);
        u16x8 g = *reinterpret_cast<const u16x8*>(dO + bs * ld_do + (long)h * D + sub * 8);
#pragma unroll
        for (int i = 0; i < 8; ++i) acc += bf2f(a[i]) * bf2f(g[i]);
    }
#pragma unroll
    for (int o = LPR / 2; o > 0; o >>= 1) acc += __shfl_xor(acc, o, 64);
    if (ok && sub == 0) {
        const long b = bs / S, s = bs % S;
        delta[(b * H + h) * S + s] = acc;
    }
}

// ---------------------------------------------------------------------------
// Backward main kernel
// ---------------------------------------------------------------------------
template <int D, bool CAUSAL, bool ROPE>
__global__ void __launch_bounds__(256, D == 64 ? 2 : 1)
fa_bwd_kernel(const __bf16* __restrict__ Q, const __bf16* __restrict__ K, const __bf16* __restrict__ Vv, long ld_q,
              long ld_kv, const __bf16* __restrict__ dO, long ld_do, const float* __restrict__ LSE,
              const float* __restrict__ DELTA, float* __restrict__ dQacc, __bf16* __restrict__ dK,
              __bf16* __restrict__ dV, long ld_dkv, const float* __restrict__ cosT, const float* __restrict__ sinT,
              int B, int H, int Hkv, int S, float scale_log2, float scale) {
    constexpr int RB = D * 2;
    constexpr int CPR = D / 8;
    constexpr int QT = 64 * RB;          // bytes of a 64-query tile
    constexpr int SPT = 64 * CPR / 256;  // staged chunks per thread per tile (each of Q, dO)
    constexpr int KS = D / 16;
    constexpr int DT = D / 32;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    char* Qs = smem;                      // [2][64][D]
    char* dOs = smem + 2 * QT;            // [2][64][D]
    char* Kl = smem + 4 * QT;             // [128][D]  roped K of the block's keys
    char* dST = Kl + 128 * RB;            // [128 keys][64 q] bf16, rows of 128 B
    float* lseS = reinterpret_cast<float*>(dST + 128 * 128);  // [2][64]
    float* dltS = lseS + 128;                                  // [2][64]

    const int tid = threadIdx.x, w = tid >> 6, l = tid & 63, l31 = l & 31, hh = l >> 5;
    const int BHk = B * Hkv;
    const int kb = (int)(blockIdx.x / BHk);
    const int bhk = blockIdx.x % BHk;
    const int b = bhk / Hkv, hk = bhk % Hkv;
    const int G = H / Hkv;
    const int kb0 = kb * 128, kw0 = kb0 + 32 * w;
    const int key = kw0 + l31;
    const bool key_ok = key < S;

    // ---- this wave's K (roped) and V rows as B-operand fragments; K also to LDS
    bf16x8 kf[KS], vf[KS];
    {
        const __bf16* kp = K + ((long)b * S + (key_ok ? key : 0)) * ld_kv + (long)hk * D;
        const __bf16* vp = Vv + ((long)b * S + (key_ok ? key : 0)) * ld_kv + (long)hk * D;
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) {
            const int d0 = 16 * ks + 8 * hh;
            u16x8 tk = key_ok ? *reinterpret_cast<const u16x8*>(kp + d0) : u16x8{0, 0, 0, 0, 0, 0, 0, 0};
            u16x8 tv = key_ok ? *reinterpret_cast<const u16x8*>(vp + d0) : u16x8{0, 0, 0, 0, 0, 0, 0, 0};
            if (ROPE) {
                float x[8];
                unpack8(tk, x);
                const int kpos = key_ok ? key : 0;
                rope8(x, cosT + (long)kpos * (D / 2) + d0 / 2, sinT + (long)kpos * (D / 2) + d0 / 2, 1.f);
                tk = pack8(x, 1.f);
            }
            kf[ks] = __builtin_bit_cast(bf16x8, tk);
            vf[ks] = __builtin_bit_cast(bf16x8, tv);
            *reinterpret_cast<u16x8*>(Kl + swz<RB>(32 * w + l31, 2 * ks + hh)) = tk;
        }
    }

    f32x16 dk[DT], dv[DT];
#pragma unroll
    for (int dt = 0; dt < DT; ++dt)
#pragma unroll
        for (int r = 0; r < 16; ++r) { dk[dt][r] = 0.f; dv[dt][r] = 0.f; }

    const int m_start = CAUSAL ? kb0 : 0;  // kb0 is a multiple of 128 -> 64-aligned
    const int nqt = (S - m_start + 63) / 64;
    const int total_it = nqt * G;

    u16x8 qreg[SPT], oreg[SPT];
    float lreg = 0.f, dreg = 0.f;
    auto load_tile = [&](int it) {
        const int h = hk * G + it / nqt;
        const int m0 = m_start + (it % nqt) * 64;
        const __bf16* qb = Q + (long)b * S * ld_q + (long)h * D;
        const __bf16* ob = dO + (long)b * S * ld_do + (long)h * D;
#pragma unroll
        for (int i = 0; i < SPT; ++i) {
            const int e = tid + 256 * i, row = e / CPR, c = e % CPR;
            const int qq = m0 + row;
            if (qq < S) {
                qreg[i] = *reinterpret_cast<const u16x8*>(qb + (long)qq * ld_q + c * 8);
                oreg[i] = *reinterpret_cast<const u16x8*>(ob + (long)qq * ld_do + c * 8);
            } else {
                qreg[i] = u16x8{0, 0, 0, 0, 0, 0, 0, 0};
                oreg[i] = u16x8{0, 0, 0, 0, 0, 0, 0, 0};
            }
        }
        if (tid < 64) {
            const int qq = m0 + tid;
            const long idx = ((long)b * H + h) * S + qq;
            lreg = qq < S ? LSE[idx] : INFINITY;
            dreg = qq < S ? DELTA[idx] : 0.f;
        }
    };
    auto write_tile = [&](int it, int buf) {
        const int m0 = m_start + (it % nqt) * 64;
#pragma unroll
        for (int i = 0; i < SPT; ++i) {
            const int e = tid + 256 * i, row = e / CPR, c = e % CPR;
            u16x8 qv = qreg[i];
            if (ROPE) {
                const int qq = min(m0 + row, S - 1);
                float x[8];
                unpack8(qv, x);
                rope8(x, cosT + (long)qq * (D / 2) + c * 4, sinT + (long)qq * (D / 2) + c * 4, 1.f);
                qv = pack8(x, 1.f);
            }
            *reinterpret_cast<u16x8*>(Qs + buf * QT + swz<RB>(row, c)) = qv;
            *reinterpret_cast<u16x8*>(dOs + buf * QT + swz<RB>(row, c)) = oreg[i];
        }
        if (tid < 64) {
            lseS[buf * 64 + tid] = lreg;
            dltS[buf * 64 + tid] = dreg;
        }
    };

    load_tile(0);
    write_tile(0, 0);
    __syncthreads();

    const int trow = 4 * hh + ((l & 15) >> 2);          // tr-read row inside a 16-row k-step
    const int tcol = 16 * ((l >> 4) & 1) + 4 * (l & 3);  // tr-read column inside a 32-col tile

    for (int it = 0; it < total_it; ++it) {
        const int cur = it & 1;
        const int h = hk * G + it / nqt;
        const int m0 = m_start + (it % nqt) * 64;
        if (it + 1 < total_it) load_tile(it + 1);
        char* Qc = Qs + cur * QT;
        char* Oc = dOs + cur * QT;
        const float* lc = lseS + cur * 64;
        const float* dc = dltS + cur * 64;
        const bool active = !CAUSAL || (m0 + 63 >= kw0);
        if (active) {
            f32x16 sp[2], dp[2];
#pragma unroll
            for (int qt = 0; qt < 2; ++qt) {
#pragma unroll
                for (int r = 0; r < 16; ++r) { sp[qt][r] = 0.f; dp[qt][r] = 0.f; }
#pragma unroll
                for (int ks = 0; ks < KS; ++ks) {
                    const int off = swz<RB>(qt * 32 + l31, 2 * ks + hh);
                    sp[qt] = mfma(lds_row16(Qc, off), kf[ks], sp[qt]);
                    dp[qt] = mfma(lds_row16(Oc, off), vf[ks], dp[qt]);
                }
            }
            // P and dS (col = key on the lane, rows = queries)
#pragma unroll
            for (int qt = 0; qt < 2; ++qt)
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    const int qi = qt * 32 + 8 * i + 4 * hh;  // rows qi..qi+3
                    const f32x4 lv = *reinterpret_cast<const f32x4*>(lc + qi);
                    const f32x4 dlt = *reinterpret_cast<const f32x4*>(dc + qi);
#pragma unroll
                    for (int j = 0; j < 4; ++j) {
                        const int r = 4 * i + j;
                        const int qg = m0 + qi + j;
                        float p = exp2f(sp[qt][r] * scale_log2 - lv[j]);
                        if ((CAUSAL && key > qg) || qg >= S || !key_ok) p = 0.f;
                        sp[qt][r] = p;
                        dp[qt][r] = p * (dp[qt][r] - dlt[j]);
                    }
                }
            // dV^T += dO^T P ; dK^T += Q^T dS   (B operands straight from accumulators)
#pragma unroll
            for (int qt = 0; qt < 2; ++qt)
#pragma unroll
                for (int ss = 0; ss < 2; ++ss) {
                    bf16x8 pb, db;
#pragma unroll
                    for (int j = 0; j < 8; ++j) {
                        pb[j] = (__bf16)sp[qt][8 * ss + j];
                        db[j] = (__bf16)dp[qt][8 * ss + j];
                    }
                    const int qr = qt * 32 + 16 * ss;
#pragma unroll
                    for (int dt = 0; dt < DT; ++dt) {
                        const int o0 = tr_off<RB>(qr + trow, dt * 32 + tcol);
                        const int o1 = tr_off<RB>(qr + 8 + trow, dt * 32 + tcol);
                        dv[dt] = mfma(lds_tr_pair(Oc, o0, o1), pb, dv[dt]);
                        dk[dt] = mfma(lds_tr_pair(Qc, o0, o1), db, dk[dt]);
                    }
                }
            // dS^T -> LDS [key row][q]: registers 4i..4i+3 are 4 consecutive queries
#pragma unroll
            for (int qt = 0; qt < 2; ++qt)
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    u16x4 t = {f2bf(dp[qt][4 * i]), f2bf(dp[qt][4 * i + 1]), f2bf(dp[qt][4 * i + 2]),
                               f2bf(dp[qt][4 * i + 3])};
                    *reinterpret_cast<u16x4*>(dST + swz<128>(32 * w + l31, qt * 4 + i) + 8 * hh) = t;
                }
        } else {
#pragma unroll
            for (int c = 0; c < 4; ++c)
                *reinterpret_cast<u16x8*>(dST + swz<128>(32 * w + l31, 2 * c + hh)) = u16x8{0, 0, 0, 0, 0, 0, 0, 0};
        }
        __syncthreads();
        // dQ tiles: wave w -> query rows (w>>1)*32, d tiles (w&1)*DT/2 .. ; k = 128 keys
        {
            const int qt2 = w >> 1;
#pragma unroll
            for (int dd = 0; dd < DT / 2; ++dd) {
                const int dt2 = (w & 1) * (DT / 2) + dd;
                f32x16 acc;
#pragma unroll
                for (int r = 0; r < 16; ++r) acc[r] = 0.f;
#pragma unroll
                for (int ks = 0; ks < 8; ++ks) {
                    const int kr = 16 * ks + 8 * hh + ((l & 15) >> 2);
                    const int qc = qt2 * 32 + 16 * ((l >> 4) & 1) + 4 * (l & 3);
                    const bf16x8 a = lds_tr_pair(dST, tr_off<128>(kr, qc), tr_off<128>(kr + 4, qc));
                    const int dc2 = dt2 * 32 + 16 * ((l >> 4) & 1) + 4 * (l & 3);
                    const bf16x8 bb = lds_tr_pair(Kl, tr_off<RB>(kr, dc2), tr_off<RB>(kr + 4, dc2));
                    acc = mfma(a, bb, acc);
                }
                float* dqp = dQacc + ((long)b * S) * H * D + (long)h * D + dt2 * 32 + l31;
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    const int qg = m0 + qt2 * 32 + acc_row(r, hh);
                    if (qg < S) atomicAdd(dqp + (long)qg * H * D, acc[r]);
                }
            }
        }
        if (it + 1 < total_it) write_tile(it + 1, cur ^ 1);
        __syncthreads();
    }

    // ---- epilogue: dK = scale * R(-pos) dK^T, dV = dV^T; key on the lane, d in registers
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
                        const float c = cosT[(long)key * (D / 2) + d0 / 2 + pr];
                        const float s = sinT[(long)key * (D / 2) + d0 / 2 + pr];
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

// dQ (fp32, roped space, unscaled) -> bf16 output slice: dq = scale * R(-pos) dQacc
template <int D, bool ROPE>
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
        const int s = (int)(bs % S);
        f32x4 v = *reinterpret_cast<const f32x4*>(dQacc + row * D + d0);
        float x[4] = {v[0] * scale, v[1] * scale, v[2] * scale, v[3] * scale};
        if (ROPE) {
#pragma unroll
            for (int pr = 0; pr < 2; ++pr) {
                const float c = cosT[(long)s * (D / 2) + d0 / 2 + pr];
                const float sn = sinT[(long)s * (D / 2) + d0 / 2 + pr];
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

size_t fa_fwd_lds_bytes(int D) { return (size_t)4 * 64 * D * 2; }
size_t fa_bwd_lds_bytes(int D) { return (size_t)4 * 64 * D * 2 + 128 * D * 2 + 128 * 128 + 4 * 64 * 4; }

template <int D, bool C, bool R>
static void fwd_launch(const FaArgs& a, hipStream_t s) {
    const int nqb = (a.S + 127) / 128;
    const size_t lds = fa_fwd_lds_bytes(D);
    fa_fwd_kernel<D, C, R><<<nqb * a.B * a.H, 256, lds, s>>>(a.q, a.k, a.v, a.ld_q, a.ld_kv, a.o, a.ld_o, a.lse,
                                                            a.cos, a.sin, a.B, a.H, a.Hkv, a.S, a.scale * LOG2E);
}

void launch_fa_fwd(const FaArgs& a, hipStream_t s) {
#define FWD_CASE(DD)                                                                  \
    if (a.D == DD) {                                                                  \
        if (a.causal) { if (a.rope) fwd_launch<DD, true, true>(a, s); else fwd_launch<DD, true, false>(a, s); } \
        else { if (a.rope) fwd_launch<DD, false, true>(a, s); else fwd_launch<DD, false, false>(a, s); }       \
        return;                                                                       \
    }
    FWD_CASE(64) FWD_CASE(128)
#undef FWD_CASE
}

template <int D, bool C, bool R>
static void bwd_launch(const FaArgs& a, hipStream_t s) {
    // delta
    {
        const long rows = (long)a.B * a.S * a.H;
        const long threads = rows * (D / 8);
        fa_bwd_pre_kernel<D><<<(unsigned)((threads + 255) / 256), 256, 0, s>>>(a.o, a.ld_o, a.dout, a.ld_do, a.delta,
                                                                               a.B, a.H, a.S);
    }
    (void)hipMemsetAsync(a.dq_acc, 0, (size_t)a.B * a.S * a.H * D * sizeof(float), s);
    const int nkb = (a.S + 127) / 128;
    const size_t lds = fa_bwd_lds_bytes(D);
    fa_bwd_kernel<D, C, R><<<nkb * a.B * a.Hkv, 256, lds, s>>>(
        a.q, a.k, a.v, a.ld_q, a.ld_kv, a.dout, a.ld_do, a.lse, a.delta, a.dq_acc, a.dk, a.dv, a.ld_dkv, a.cos, a.sin,
        a.B, a.H, a.Hkv, a.S, a.scale * LOG2E, a.scale);
    const long total = (long)a.B * a.S * a.H * (D / 4);
    const int grid = (int)std::min<long>((total + 255) / 256, 4096);
    fa_dq_convert_kernel<D, R><<<grid, 256, 0, s>>>(a.dq_acc, a.dq, a.ld_dq, a.cos, a.sin, a.B, a.H, a.S, a.scale);
}

void launch_fa_bwd(const FaArgs& a, hipStream_t s) {
#define BWD_CASE(DD)                                                                  \
    if (a.D == DD) {                                                                  \
        if (a.causal) { if (a.rope) bwd_launch<DD, true, true>(a, s); else bwd_launch<DD, true, false>(a, s); } \
        else { if (a.rope) bwd_launch<DD, false, true>(a, s); else bwd_launch<DD, false, false>(a, s); }       \
        return;                                                                       \
    }
    BWD_CASE(64) BWD_CASE(128)
#undef BWD_CASE
}
