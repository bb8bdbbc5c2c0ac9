// Flash attention backward, dQ kernel with 16 queries per wave (D = 64), gfx950 (MI355X).
// build-flags: -fno-slp-vectorize   (no packed f32 VALU beside the MFMAs: ops/build.py file_flags)
//
// Parity target: the dQ of the split backward (flash_attn_bwd_split.hip fa_bwd_dq_kernel; reference contracts
// K7/K10, `tests/adapters.py:92-184`); checked against autograd of the fp32 oracle and against the 32-row kernel
// (tests/test_kernels_gpu.py).
//
// Why: the 32-row split dQ kernel runs at mfma_util 0.29 (profiles/attention_pmc.md): each wave's 32-key step is a
// dependency chain (S / dP MFMAs -> exp -> dS -> dQ MFMAs) and two waves per SIMD cannot cover it.  This form
// computes the same products with v_mfma_f32_16x16x32_bf16 on 16 queries per wave, so a wave holds half the
// registers (<= 128: four waves per SIMD, two 512-thread workgroups per CU) and each SIMD has twice as many
// independent chains to interleave.  Per 32-key step and wave: S^T and dP^T as two 16-key blocks each
// (4 + 4 MFMAs over d = 64), dQ^T += K^T dS^T over 4 d-tiles (4 MFMAs); the same VALU per score as before.
// Measured: backward -1.1 % (GPT-2 B 128) / -1.0 % (Llama s2048 GQA), mfma_util 0.298 vs 0.288 -- the default.  The
// gain is small because a 16x16x32 MFMA holds the SIMD's vector issue for half its cycles (8 of 16, against 8 of 32
// for 32x32x16), so the extra waves buy latency cover but lose VALU issue slots; the same form of the dK/dV kernel,
// with more MFMA work per score, measured 1-2.5 % slower and was dropped (docs/performance.md).
//
//   S^T [key][query]  = K . (cQ)^T - lse     A = K rows (ds_read_b128), B = the pinned c*Q (query on the lane)
//   dP^T              = V . dO^T - delta     A = V rows,                B = the pinned dO
//   dS^T = exp2(S^T) * dP^T                  accumulator rows = keys 16 kb + 4 g + i (g = lane >> 4)
//   dQ^T [d][query]  += K^T . dS^T           A = K^T (two ds_read_b64_tr_b16), B = dS^T packed from the two
//                                            accumulators in the permuted key order 16 (j >> 2) + 4 g + (j & 3)
//
// LDS image: 128-byte rows, chunk c of row r at c ^ (r & 6).  Both fragment reads are conflict-free on it (found by
// a search over per-row chunk XORs; SQ_LDS_BANK_CONFLICT 0, profiles/pmc/attn_dq16_pmc_r5.txt): the ds_read_b128 row
// reads (rows 16 m + lane & 15, chunk 4 ks + lane >> 4) and the ds_read_b64_tr_b16 reads (4-row blocks 16 rows apart,
// one 32-byte column pair).  The 32-row kernels' image (fa_common.h swz<128>) leaves both 2-way conflicted for these
// fragments.  K / V tiles are DMA'd through buffer resources, CPW wave-instructions per wave and 64-row image.
#include "fa_common.h"
#include "kernels.h"

#include <type_traits>

namespace bpe {
namespace fa {
namespace dq16 {

// Two geometries, both at four waves per SIMD: (NW, KT) = (8, 128) -- 128 queries per workgroup, 128-key tiles, two
// workgroups per CU (64 KiB of LDS each), the default -- and (4, 64) -- 64 queries, 64-key tiles, four workgroups per
// CU (32 KiB), meant to cover the ~30 % prologue with three other workgroups; it measured no faster (GPT-2) and 0.7-1.6 %
// slower (Llama), the prologue staying at ~8.8 k cycles (profiles/attention_stamps_r5.md).
constexpr int TILE = 64 * 128;   // one 64-row image of 128-byte rows

__device__ __forceinline__ int sw(int row, int c) { return row * 128 + ((c ^ (row & 6)) << 4); }
// byte offset of the 8-byte granule at (row, col) (transposed reads)
__device__ __forceinline__ int sw_tr(int row, int col) { return sw(row, col >> 3) + ((col & 7) << 1); }

// Per-workgroup s_memtime stamps (BPE_FA_STAMPS variant builds; read through fa_read_stamps, rows 0.. when this
// kernel is selected), taken by the LAST wave (the one with the most steps on the diagonal tile): slot 0 entry, 6
// every prologue load issued, 4 its row loads arrived, 1 after the prologue barrier, 2 at the start of the last
// tile, 3 after the tile loop, 5 the tile count
#ifdef BPE_FA_STAMPS
__device__ long long g_stamps16[32768 * 8];
#define DQ16_STAMP(i, v)                                                                             \
    if (threadIdx.x == (NW - 1) * 64) {                                                              \
        g_stamps16[(long)(blockIdx.x & 32767) * 8 + (i)] = __builtin_amdgcn_s_memtime();            \
        if ((i) == 3) g_stamps16[(long)(blockIdx.x & 32767) * 8 + 5] = (v);                        \
    }
#else
#define DQ16_STAMP(i, v)
#endif

__device__ __forceinline__ f32x4 mfma16(bf16x8 a, bf16x8 b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

// lane offset (bytes, inside a 64-row tile of a row-major tensor of row stride ld) of the source chunk this lane's
// DMA slot holds: wave-instruction i of wave w (CPW per wave and image) fills physical chunks 64 (CPW w + i) + lane
template <int CPW>
__device__ __forceinline__ void dma_lane_off(long ld, int w, int l, unsigned (&v)[CPW]) {
#pragma unroll
    for (int i = 0; i < CPW; ++i) {
        const int e = 64 * (CPW * w + i) + l, r = e >> 3, pc = e & 7;
        v[i] = (unsigned)((r * ld + ((pc ^ (r & 6)) << 3)) * 2);
    }
}

template <int CPW>
__device__ __forceinline__ void dma_image(const __bf16* base, int nbytes, const unsigned (&voff)[CPW], int r0, long ld,
                                          char* img, int w) {
#if defined(__HIP_DEVICE_COMPILE__)
    const auto rsrc = __builtin_amdgcn_make_buffer_rsrc((void*)base, 0, nbytes, 0x00020000);
#pragma unroll
    for (int i = 0; i < CPW; ++i)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rsrc, (lds_void_t*)(img + 1024 * (CPW * w + i)), 16, voff[i],
                                                 (unsigned)((long)r0 * ld * 2), 0, 0);
#endif
}

template <int NW, int KT, bool CAUSAL, bool ROPE>
__global__ void __launch_bounds__(NW * 64, 16 / NW)
fa_bwd_dq16_kernel(const __bf16* __restrict__ Q, const __bf16* __restrict__ K, const __bf16* __restrict__ Vv,
                   long ld_q, long ld_kv, const __bf16* __restrict__ O, long ld_o, const __bf16* __restrict__ dO,
                   long ld_do, const float* __restrict__ LSE, float* __restrict__ DELTA, __bf16* __restrict__ dQ,
                   long ld_dq, const float* __restrict__ cosT, const float* __restrict__ sinT, int B, int H, int Hkv,
                   int S, float scale_log2, float scale, int group) {
    constexpr int D = 64, QB = 16 * NW, NSUB = KT / 64, BUF = NSUB * TILE, CPW = 512 / (NW * 64);
    extern __shared__ __attribute__((aligned(16))) char smem[];
    char* Ks = smem;            // [2][KT keys][128 B]
    char* Vs = smem + 2 * BUF;  // [2][KT keys][128 B]

    const int tid = threadIdx.x, w = tid >> 6, l = tid & 63, g = l >> 4, i16 = l & 15;
    prologue_prio_begin();
    DQ16_STAMP(0, 0);
    const int nqb = (S + QB - 1) / QB;
    int rank, bh;
    grouped_order((int)blockIdx.x, nqb, B * H, group, rank, bh);
    const int qblk = CAUSAL ? nqb - 1 - rank : rank;  // causal: the heaviest query blocks first
    const int b = bh / H, h = bh % H, hk = h / (H / Hkv);
    const int q0 = qblk * QB, qw = q0 + 16 * w, q = qw + i16;
    const bool q_ok = q < S;
    const long qc = q_ok ? q : S - 1;
    const long qrow = (long)b * S + qc;

    // ---- prologue: every load issued before any is waited for (pinned Q / dO rows, O rows of delta, LSE, tile 0)
    // lane: query i16, d = 32 ks + 8 g + j
    u16x8 tqr[2], tgr[2], tor[2];
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
        const int d0 = 32 * ks + 8 * g;
        tqr[ks] = *reinterpret_cast<const u16x8*>(Q + qrow * ld_q + (long)h * D + d0);
        tgr[ks] = *reinterpret_cast<const u16x8*>(dO + qrow * ld_do + (long)h * D + d0);
        tor[ks] = *reinterpret_cast<const u16x8*>(O + qrow * ld_o + (long)h * D + d0);
    }
    const float lse = LSE[((long)b * H + h) * S + qc];

    const int kend = CAUSAL ? min(S, q0 + QB) : S;
    const int nkt = (kend + KT - 1) / KT;
    const __bf16* kb = K + (long)b * S * ld_kv + (long)hk * D;
    const __bf16* vb = Vv + (long)b * S * ld_kv + (long)hk * D;
    const int wu = __builtin_amdgcn_readfirstlane(w);
    const int hbytes = head_bytes(ld_kv, S, D);
    unsigned voff[CPW];
    dma_lane_off<CPW>(ld_kv, wu, l, voff);
#pragma unroll
    for (int sb = 0; sb < NSUB; ++sb) {
        dma_image(kb, hbytes, voff, 64 * sb, ld_kv, Ks + sb * TILE, wu);
        dma_image(vb, hbytes, voff, 64 * sb, ld_kv, Vs + sb * TILE, wu);
    }
    DQ16_STAMP(6, 0);  // every prologue load issued

    // ---- pinned B operands (c folded into Q: S^T in log2 units) and delta = rowsum(dO * O)
    bf16x8 qf[2], of[2];
    float dsum = 0.f;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
        float x[8];
        unpack8(tqr[ks], x);
        qf[ks] = __builtin_bit_cast(bf16x8, pack8(x, scale_log2));
#pragma unroll
        for (int i = 0; i < 8; ++i) dsum += bf2f(tgr[ks][i]) * bf2f(tor[ks][i]);
        of[ks] = __builtin_bit_cast(bf16x8, tgr[ks]);
    }
    dsum += __shfl_xor(dsum, 16, 64);
    dsum += __shfl_xor(dsum, 32, 64);
    DQ16_STAMP(4, 0);  // the wave's own row loads have arrived (its DMA and the other waves' may not have)
    // row constants as the initial accumulators: S^T starts at -lse (-inf on pad rows: P = 0), dP^T at -delta
    const float nl = (q_ok && lse < INFINITY) ? -lse : -INFINITY;

    f32x4 acc[4];
#pragma unroll
    for (int mt = 0; mt < 4; ++mt) acc[mt] = f32x4{0.f, 0.f, 0.f, 0.f};

    __syncthreads();
    prologue_prio_end();
    DQ16_STAMP(1, 0);

    const int trq = i16 >> 2, trc = 4 * (i16 & 3);  // transposed read: row 4 g + trq of a block, column trc
    for (int it = 0; it < nkt; ++it) {
        const int cur = it & 1, k0 = it * KT;
        if (it + 1 == nkt) DQ16_STAMP(2, 0);
        // current / next buffers as __restrict__ parameters: the next tile's DMA and this tile's reads are disjoint
        // to the wait-count pass (no vmcnt(0) drain before the first transposed read; flash_attn_bwd_split.hip)
        auto body = [&](char* __restrict__ Kc, const char* __restrict__ Vc, char* __restrict__ Kn,
                        char* __restrict__ Vn) {
            if (it + 1 < nkt) {  // buffer cur ^ 1 was last read in iteration it - 1, before its closing barrier
#pragma unroll
                for (int sb = 0; sb < NSUB; ++sb) {
                    dma_image(kb, hbytes, voff, k0 + KT + 64 * sb, ld_kv, Kn + sb * TILE, wu);
                    dma_image(vb, hbytes, voff, k0 + KT + 64 * sb, ld_kv, Vn + sb * TILE, wu);
                }
            }
            if (CAUSAL && k0 > qw + 15) return;
#pragma unroll
            for (int kq = 0; kq < KT / 32; ++kq) {
                if (CAUSAL && k0 + 32 * kq > qw + 15) break;  // the step is past every query of the wave
                const bool need_mask = (CAUSAL && k0 + 32 * kq + 31 > qw) || (k0 + 32 * kq + 32 > S);
                char* Kh = Kc + (kq >> 1) * TILE;
                const char* Vh = Vc + (kq >> 1) * TILE;
                const int kr = 32 * (kq & 1);
                bf16x8 fk[2][2], fv[2][2];
#pragma unroll
                for (int kb2 = 0; kb2 < 2; ++kb2)
#pragma unroll
                    for (int ks = 0; ks < 2; ++ks) {
                        const int off = sw(kr + 16 * kb2 + i16, 4 * ks + g);
                        fk[kb2][ks] = lds_row16(Kh, off);
                        fv[kb2][ks] = lds_row16(Vh, off);
                    }
                f32x4 sp[2], dp[2];
#pragma unroll
                for (int kb2 = 0; kb2 < 2; ++kb2) {
                    sp[kb2] = f32x4{nl, nl, nl, nl};
                    dp[kb2] = f32x4{-dsum, -dsum, -dsum, -dsum};
                }
#pragma unroll
                for (int ks = 0; ks < 2; ++ks)
#pragma unroll
                    for (int kb2 = 0; kb2 < 2; ++kb2) {
                        sp[kb2] = mfma16(fk[kb2][ks], qf[ks], sp[kb2]);
                        dp[kb2] = mfma16(fv[kb2][ks], of[ks], dp[kb2]);
                    }
                bf16x8 tk[4];
#pragma unroll
                for (int mt = 0; mt < 4; ++mt)
                    tk[mt] = lds_tr_pair(Kh, sw_tr(kr + 4 * g + trq, 16 * mt + trc),
                                         sw_tr(kr + 16 + 4 * g + trq, 16 * mt + trc));
                // P^T = exp2(S^T), dS^T = P^T dP^T; key = k0 + 32 kq + 16 kb + 4 g + r, query = q
                if (need_mask) {
                    const int klim = (CAUSAL ? min(q, S - 1) : S - 1) - k0 - 32 * kq - 4 * g;
#pragma unroll
                    for (int kb2 = 0; kb2 < 2; ++kb2)
#pragma unroll
                        for (int r = 0; r < 4; ++r) {
                            const float p = fast_exp2(sp[kb2][r]);
                            dp[kb2][r] = (16 * kb2 + r <= klim) ? p * dp[kb2][r] : 0.f;
                        }
                } else {
#pragma unroll
                    for (int kb2 = 0; kb2 < 2; ++kb2)
#pragma unroll
                        for (int r = 0; r < 4; ++r) dp[kb2][r] = fast_exp2(sp[kb2][r]) * dp[kb2][r];
                }
                bf16x8 db;
#pragma unroll
                for (int j = 0; j < 8; ++j) db[j] = (__bf16)dp[j >> 2][j & 3];
#pragma unroll
                for (int mt = 0; mt < 4; ++mt) acc[mt] = mfma16(tk[mt], db, acc[mt]);
            }
        };
        body(Ks + cur * BUF, Vs + cur * BUF, Ks + (cur ^ 1) * BUF, Vs + (cur ^ 1) * BUF);
        if (it + 1 < nkt) __syncthreads();  // (none after the last tile: a wave done with the diagonal leaves early)
    }

    DQ16_STAMP(3, nkt);
    // ---- epilogue: delta for the dK/dV kernel; dQ = scale * R(-pos) dQ^T (lane: query i16, d = 16 mt + 4 g + i)
    if (q_ok && g == 0) DELTA[((long)b * H + h) * S + q] = dsum;
    if (!q_ok) return;
    __bf16* dqp = dQ + ((long)b * S + q) * ld_dq + (long)h * D;
#pragma unroll
    for (int mt = 0; mt < 4; ++mt) {
        const int d0 = 16 * mt + 4 * g;
        float x[4] = {acc[mt][0] * scale, acc[mt][1] * scale, acc[mt][2] * scale, acc[mt][3] * scale};
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

}  // namespace dq16
}  // namespace fa
}  // namespace bpe

using namespace bpe;
using namespace bpe::fa;

// dQ form of the split backward at D = 64 without in-kernel RoPE: 0 = 32 queries per wave (fa_bwd_dq_kernel),
// 1 = 16 queries per wave, 8 waves, 128-key tiles, 2 = 16 queries per wave, 4 waves, 64-key tiles (this file),
// 3 = form 1 up to S = 2048 and form 0 above (the default); switched at run time (tests compare them).  Form 1 against
// form 0, op-level, interleaved: backward -1.9 % (S 1024, GPT-2 B 128), -0.3 % (S 2048, Llama GQA B 32), +0.1 %
// (S 4096), +0.5 % (S 8192) (profiles/bench/ab_attn_dq_forms_r5.log, ab_attn_dq_vs_seq_r5.log): the gain is in the
// per-workgroup fixed cost, which long sequences amortise.  Form 2 measured no gain (four workgroups per CU do not
// shorten the prologue, profiles/attention_stamps_r5.md).
static int g_dq_form = 3;
static bool g_dq16_ran = false;  // the last backward launched this file's kernel (stamps)

int fa_dq_config(int form) {
    const int prev = g_dq_form;
    if (form >= 0) g_dq_form = form > 3 ? 3 : form;
    return prev;
}

// copy the 16-row dQ kernel's stamps of the last launch into rows [0, 32768) (BPE_FA_STAMPS builds; false
// otherwise or when the kernel is not selected)
bool fa_read_stamps_dq16(long long* host, int n) {
#ifdef BPE_FA_STAMPS
    if (!g_dq16_ran) return false;
    (void)hipDeviceSynchronize();
    const int rows = n < 32768 ? n : 32768;
    return hipMemcpyFromSymbol(host, HIP_SYMBOL(dq16::g_stamps16), (size_t)rows * 8 * sizeof(long long), 0,
                               hipMemcpyDeviceToHost) == hipSuccess;
#else
    (void)host;
    (void)n;
    return false;
#endif
}

// launches the 16-row dQ kernel when selected and applicable (D = 64, rope 0 / 2); false otherwise
bool launch_fa_bwd_dq16(const FaArgs& a, hipStream_t s) {
    const int form = g_dq_form == 3 ? (a.S <= 2048 ? 1 : 0) : g_dq_form;
    g_dq16_ran = form != 0 && a.D == 64 && a.rope != 1;
    if (!g_dq16_ran) return false;
    auto run = [&](auto nw, auto kt) {
        constexpr int NW = decltype(nw)::value, KT = decltype(kt)::value;
        const int nblk = (a.S + 16 * NW - 1) / (16 * NW);
        const int lds = 2 * 2 * (KT / 64) * dq16::TILE;  // K and V, two buffers
        auto go = [&](auto kern) {
            kern<<<nblk * a.B * a.H, NW * 64, lds, s>>>(a.q, a.k, a.v, a.ld_q, a.ld_kv, a.o, a.ld_o, a.dout, a.ld_do,
                                                        a.lse, a.delta, a.dq, a.ld_dq, a.cos, a.sin, a.B, a.H, a.Hkv,
                                                        a.S, a.scale * LOG2E, a.scale, fa_group(a.B * a.H));
        };
        if (a.causal) {
            if (a.rope == 2) go(dq16::fa_bwd_dq16_kernel<NW, KT, true, true>);
            else go(dq16::fa_bwd_dq16_kernel<NW, KT, true, false>);
        } else {
            if (a.rope == 2) go(dq16::fa_bwd_dq16_kernel<NW, KT, false, true>);
            else go(dq16::fa_bwd_dq16_kernel<NW, KT, false, false>);
        }
    };
    if (form == 1) run(std::integral_constant<int, 8>{}, std::integral_constant<int, 128>{});
    else run(std::integral_constant<int, 4>{}, std::integral_constant<int, 64>{});
    return true;
}
