// Flash attention backward, dK/dV kernel with 16 keys per wave (D = 64), gfx950 (MI355X).
// build-flags: -fno-slp-vectorize   (no packed f32 VALU beside the MFMAs: ops/build.py file_flags)
//
// Parity target: dK / dV of the split backward (flash_attn_bwd_split.hip fa_bwd_dkv_kernel; reference contracts
// K7/K10, `tests/adapters.py:92-184`); checked against the 32-row kernel and the fp32 oracle's autograd
// (tests/test_kernels_gpu.py).
//
// The key-major counterpart of flash_attn_bwd_dq16.hip: v_mfma_f32_16x16x32_bf16 on 16 keys per wave, 8 waves per
// 128-key workgroup, <= 128 VGPRs so four waves per SIMD (two workgroups per CU) instead of two.  Per wave and
// 32-query step (two 16-query blocks qb):
//
//   S  [query][key] = Q . (cK)^T - lse     A = Q rows (ds_read_b128), B = the pinned c*K (key on the lane)
//   dP              = dO . V^T - delta     A = dO rows,               B = the pinned V
//   P = exp2(S), dS = P * dP               accumulator rows = queries 16 qb + 4 g + i (g = lane >> 4)
//   dV^T [d][key] += dO^T . P              A = dO^T (two ds_read_b64_tr_b16), B = P packed in the permuted query
//   dK^T [d][key] += Q^T . dS              order 16 (j >> 2) + 4 g + (j & 3) -- the k order of those reads
//
// Q / dO tiles of 128 queries (two 64-row images each, LDS-DMA through buffer resources, the c ^ (r & 6) image of
// the dq16 kernel: conflict-free for both read kinds), the -lse / -delta rows beside them; GQA: one workgroup per
// KV head sweeps the query heads of its group; query tiles last to first, the diagonal tile last, no barrier after
// it.  The loop structure, masking and epilogue follow fa_bwd_dkv_kernel.
#include "fa_common.h"
#include "kernels.h"

namespace bpe {
namespace fa {
namespace dkv16 {

constexpr int NW = 8;           // waves per workgroup, 16 keys each
constexpr int KB = 16 * NW;     // keys per workgroup
constexpr int QT = 128;         // queries per Q / dO tile
constexpr int TILE = 64 * 128;  // one 64-row image of 128-byte rows
constexpr int BUF = 2 * TILE;   // one tile (two images)

__device__ __forceinline__ int sw(int row, int c) { return row * 128 + ((c ^ (row & 6)) << 4); }
__device__ __forceinline__ int sw_tr(int row, int col) { return sw(row, col >> 3) + ((col & 7) << 1); }

__device__ __forceinline__ f32x4 mfma16(bf16x8 a, bf16x8 b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

// lane offset (bytes) of the source chunk wave w's one wave-instruction per 64-row image fills (physical chunk
// 64 w + lane of the c ^ (r & 6) image)
__device__ __forceinline__ unsigned dma_lane_off(long ld, int w, int l) {
    const int e = 64 * w + l, r = e >> 3, pc = e & 7;
    return (unsigned)((r * ld + ((pc ^ (r & 6)) << 3)) * 2);
}

__device__ __forceinline__ void dma_image(const __bf16* base, int nbytes, unsigned voff, int r0, long ld, char* img,
                                          int w) {
#if defined(__HIP_DEVICE_COMPILE__)
    const auto rsrc = __builtin_amdgcn_make_buffer_rsrc((void*)base, 0, nbytes, 0x00020000);
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rsrc, (lds_void_t*)(img + 1024 * w), 16, voff,
                                             (unsigned)((long)r0 * ld * 2), 0, 0);
#endif
}

template <bool CAUSAL, bool ROPE>
__global__ void __launch_bounds__(NW * 64, 2)
fa_bwd_dkv16_kernel(const __bf16* __restrict__ Q, const __bf16* __restrict__ K, const __bf16* __restrict__ Vv,
                    long ld_q, long ld_kv, const __bf16* __restrict__ dO, long ld_do, const float* __restrict__ LSE,
                    const float* __restrict__ DELTA, __bf16* __restrict__ dK, __bf16* __restrict__ dV, long ld_dkv,
                    const float* __restrict__ cosT, const float* __restrict__ sinT, int B, int H, int Hkv, int S,
                    float scale_log2, float scale, int group) {
    constexpr int D = 64;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    char* Qs = smem;                                         // [2][QT][128 B]
    char* dOs = smem + 2 * BUF;                              // [2][QT][128 B]
    float* lseS = reinterpret_cast<float*>(smem + 4 * BUF);  // [2][QT]  -lse
    float* dltS = lseS + 2 * QT;                             // [2][QT]  -delta

    prologue_prio_begin();
    const int tid = threadIdx.x, w = tid >> 6, l = tid & 63, g = l >> 4, i16 = l & 15;
    const int nkb = (S + KB - 1) / KB;
    const int G = H / Hkv;
    int kblk, bh;
    grouped_order((int)blockIdx.x, nkb, B * Hkv, group, kblk, bh);
    const int b = bh / Hkv;
    const int h = (bh % Hkv) * G;  // first query head of the group
    const int hk = h / G;
    const int kb0 = kblk * KB, kw0 = kb0 + 16 * w, key = kw0 + i16;
    const bool key_ok = key < S;
    const long kpos = key_ok ? key : S - 1;

    // ---- prologue: pinned K / V rows (lane: key i16, d = 32 ks + 8 g + j), tile 0's row constants and its DMA
    u16x8 tkr[2], tvr[2];
    {
        const __bf16* kp = K + ((long)b * S + kpos) * ld_kv + (long)hk * D;
        const __bf16* vp = Vv + ((long)b * S + kpos) * ld_kv + (long)hk * D;
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) {
            tkr[ks] = *reinterpret_cast<const u16x8*>(kp + 32 * ks + 8 * g);
            tvr[ks] = *reinterpret_cast<const u16x8*>(vp + 32 * ks + 8 * g);
        }
    }
    const int m_start = CAUSAL ? kb0 : 0;  // kb0 is a multiple of 128
    const int nqt = m_start < S ? (S - m_start + QT - 1) / QT : 0;
    const int nsteps = G * nqt;  // (query head, query tile) steps, head-major
    auto q_of = [&](int j) { return Q + (long)b * S * ld_q + (long)(h + j / nqt) * D; };
    auto o_of = [&](int j) { return dO + (long)b * S * ld_do + (long)(h + j / nqt) * D; };
    auto m0_of = [&](int j) { return m_start + (nqt - 1 - j % nqt) * QT; };  // the diagonal tile last
    float lreg = 0.f, dreg = 0.f;
    const int wu = __builtin_amdgcn_readfirstlane(w);
    const unsigned qvo = dma_lane_off(ld_q, wu, l), ovo = dma_lane_off(ld_do, wu, l);
    const int qbytes = head_bytes(ld_q, S, D), obytes = head_bytes(ld_do, S, D);
    auto load_consts = [&](int it) {  // waves 0, 1: the -lse / -delta of tile rows 64 (w & 1) + lane
        const long sbase = ((long)b * H + h + it / nqt) * S;
        const long idx = sbase + min(m0_of(it) + 64 * (w & 1) + l, S - 1);
        lreg = LSE[idx];
        dreg = DELTA[idx];
    };
    auto write_consts = [&](int it, int buf) {
        if (tid < QT) {
            const bool ok = m0_of(it) + tid < S;
            lseS[buf * QT + tid] = (!ok || lreg == INFINITY) ? -INFINITY : -lreg;
            dltS[buf * QT + tid] = ok ? -dreg : 0.f;
        }
    };
    auto dma_tile = [&](int it, char* Qd, char* Od) {
#pragma unroll
        for (int sb = 0; sb < 2; ++sb) {
            dma_image(q_of(it), qbytes, qvo, m0_of(it) + 64 * sb, ld_q, Qd + sb * TILE, wu);
            dma_image(o_of(it), obytes, ovo, m0_of(it) + 64 * sb, ld_do, Od + sb * TILE, wu);
        }
    };
    if (nqt > 0) {
        load_consts(0);
        dma_tile(0, Qs, dOs);
    }

    // ---- pinned B operands: c*K (roped, softmax scale * log2(e) folded in) and V
    bf16x8 kf[2], vf[2];
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
        const u16x8 z = {0, 0, 0, 0, 0, 0, 0, 0};
        float x[8];
        unpack8(key_ok ? tkr[ks] : z, x);
        kf[ks] = __builtin_bit_cast(bf16x8, pack8(x, scale_log2));
        vf[ks] = __builtin_bit_cast(bf16x8, key_ok ? tvr[ks] : z);
    }
    f32x4 dk[4], dv[4];
#pragma unroll
    for (int mt = 0; mt < 4; ++mt) {
        dk[mt] = f32x4{0.f, 0.f, 0.f, 0.f};
        dv[mt] = f32x4{0.f, 0.f, 0.f, 0.f};
    }
    if (nqt > 0) write_consts(0, 0);
    __syncthreads();
    prologue_prio_end();

    const int trq = i16 >> 2, trc = 4 * (i16 & 3);
    const int klim = CAUSAL ? (key_ok ? key : S) : (key_ok ? 0 : S);
    const unsigned span = (unsigned)(S - klim);  // valid query q: (unsigned)(q - klim) < span
    for (int it = 0; it < nsteps; ++it) {
        const int cur = it & 1, m0 = m0_of(it);
        auto body = [&](char* __restrict__ Qc, char* __restrict__ Oc, char* __restrict__ Qn, char* __restrict__ On) {
            if (it + 1 < nsteps) {  // buffer cur ^ 1 was last read in iteration it - 1, before its closing barrier
                load_consts(it + 1);
                dma_tile(it + 1, Qn, On);
            }
            const float* lc = lseS + cur * QT;
            const float* dc = dltS + cur * QT;
            if (CAUSAL && m0 + QT - 1 < kw0) return;
#pragma unroll
            for (int qq = 0; qq < QT / 32; ++qq) {
                if (CAUSAL && m0 + 32 * qq + 31 < kw0) continue;  // every query of the step precedes every key
                const bool need_mask =
                    (CAUSAL && m0 + 32 * qq < kw0 + 15) || (m0 + 32 * qq + 32 > S) || (kw0 + 16 > S);
                char* Qh = Qc + (qq >> 1) * TILE;
                char* Oh = Oc + (qq >> 1) * TILE;
                const int qr = 32 * (qq & 1);  // first row of the step inside its image
                f32x4 sp[2], dp[2];
#pragma unroll
                for (int qb = 0; qb < 2; ++qb) {  // row constants: queries 32 qq + 16 qb + 4 g + i
                    sp[qb] = *reinterpret_cast<const f32x4*>(lc + 32 * qq + 16 * qb + 4 * g);
                    dp[qb] = *reinterpret_cast<const f32x4*>(dc + 32 * qq + 16 * qb + 4 * g);
                }
#pragma unroll
                for (int ks = 0; ks < 2; ++ks)
#pragma unroll
                    for (int qb = 0; qb < 2; ++qb) {
                        const int off = sw(qr + 16 * qb + i16, 4 * ks + g);
                        sp[qb] = mfma16(lds_row16(Qh, off), kf[ks], sp[qb]);
                        dp[qb] = mfma16(lds_row16(Oh, off), vf[ks], dp[qb]);
                    }
                if (need_mask) {
                    const int qoff = m0 + 32 * qq - klim + 4 * g;
#pragma unroll
                    for (int qb = 0; qb < 2; ++qb)
#pragma unroll
                        for (int r = 0; r < 4; ++r) {
                            const float p = fast_exp2(sp[qb][r]);
                            const bool ok = (unsigned)(qoff + 16 * qb + r) < span;
                            sp[qb][r] = ok ? p : 0.f;
                            dp[qb][r] = ok ? p * dp[qb][r] : 0.f;
                        }
                } else {
#pragma unroll
                    for (int qb = 0; qb < 2; ++qb)
#pragma unroll
                        for (int r = 0; r < 4; ++r) {
                            const float p = fast_exp2(sp[qb][r]);
                            sp[qb][r] = p;
                            dp[qb][r] *= p;
                        }
                }
                bf16x8 pb, db;
#pragma unroll
                for (int j = 0; j < 8; ++j) {
                    pb[j] = (__bf16)sp[j >> 2][j & 3];
                    db[j] = (__bf16)dp[j >> 2][j & 3];
                }
#pragma unroll
                for (int mt = 0; mt < 4; ++mt) {
                    const int o0 = sw_tr(qr + 4 * g + trq, 16 * mt + trc);
                    const int o1 = sw_tr(qr + 16 + 4 * g + trq, 16 * mt + trc);
                    dv[mt] = mfma16(lds_tr_pair(Oh, o0, o1), pb, dv[mt]);
                    dk[mt] = mfma16(lds_tr_pair(Qh, o0, o1), db, dk[mt]);
                }
            }
        };
        body(Qs + cur * BUF, dOs + cur * BUF, Qs + (cur ^ 1) * BUF, dOs + (cur ^ 1) * BUF);
        if (it + 1 < nsteps) {  // (no barrier after the last tile: see m0_of)
            write_consts(it + 1, cur ^ 1);
            __syncthreads();
        }
    }

    if (!key_ok) return;
    // ---- dK = scale * R(-pos) dK^T, dV = dV^T (lane: key i16, d = 16 mt + 4 g + i)
    __bf16* dkp = dK + ((long)b * S + key) * ld_dkv + (long)hk * D;
    __bf16* dvp = dV + ((long)b * S + key) * ld_dkv + (long)hk * D;
#pragma unroll
    for (int mt = 0; mt < 4; ++mt) {
        const int d0 = 16 * mt + 4 * g;
        float x[4] = {dk[mt][0] * scale, dk[mt][1] * scale, dk[mt][2] * scale, dk[mt][3] * scale};
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
        *reinterpret_cast<u16x4*>(dvp + d0) =
            u16x4{f2bf(dv[mt][0]), f2bf(dv[mt][1]), f2bf(dv[mt][2]), f2bf(dv[mt][3])};
    }
}

}  // namespace dkv16
}  // namespace fa
}  // namespace bpe

using namespace bpe;
using namespace bpe::fa;

// dK/dV form of the split backward at D = 64 without in-kernel RoPE: 0 = 32 keys per wave (fa_bwd_dkv_kernel),
// 1 = 16 keys per wave (this file); switched at run time (tests compare them)
static int g_dkv_form = 0;

int fa_dkv_config(int form) {
    const int prev = g_dkv_form;
    if (form >= 0) g_dkv_form = form ? 1 : 0;
    return prev;
}

// launches the 16-row dK/dV kernel when selected and applicable (D = 64, rope 0 / 2); false otherwise
bool launch_fa_bwd_dkv16(const FaArgs& a, hipStream_t s) {
    if (g_dkv_form == 0 || a.D != 64 || a.rope == 1) return false;
    const int nblk = (a.S + dkv16::KB - 1) / dkv16::KB;
    const int lds = 4 * dkv16::BUF + 16 * dkv16::QT;  // Q / dO buffers + the -lse / -delta rows
    auto go = [&](auto kern) {
        kern<<<nblk * a.B * a.Hkv, dkv16::NW * 64, lds, s>>>(a.q, a.k, a.v, a.ld_q, a.ld_kv, a.dout, a.ld_do, a.lse,
                                                             a.delta, a.dk, a.dv, a.ld_dkv, a.cos, a.sin, a.B, a.H,
                                                             a.Hkv, a.S, a.scale * LOG2E, a.scale,
                                                             fa_group(a.B * a.Hkv));
    };
    if (a.causal) {
        if (a.rope == 2) go(dkv16::fa_bwd_dkv16_kernel<true, true>);
        else go(dkv16::fa_bwd_dkv16_kernel<true, false>);
    } else {
        if (a.rope == 2) go(dkv16::fa_bwd_dkv16_kernel<false, true>);
        else go(dkv16::fa_bwd_dkv16_kernel<false, false>);
    }
    return true;
}
