// Skinny GEMM (GEMV-like, M <= 8 token rows) with fused prologue / epilogues for the decode step, gfx950.
//
// At decode time a projection is y[m, n] = sum_k h[m, k] W[n, k] with M = batch (1..8): pure weight streaming
// (HBM-bound), where library GEMMs cost ~7 us per call and each elementwise op around them another launch.
// This kernel folds the neighbours in, so a transformer layer is 4 of these launches + the decode attention:
//   prologue  h = RMSNorm(x (+ xd)) * ln, computed redundantly by every workgroup from the (L2-resident) input
//             rows; workgroup 0 also writes the residual sum x + xd for the next layer;
//   epilogue  0: y = h W^T                                   (output projection, W2, LM head)
//             1: y[:, j] = silu(g_j) * u_j over [W1; W3]    (SwiGLU; rows j and F + j in one wave)
//             2: fused-QKV with RoPE at the device-side position and the K / V cache write (rows n, n + 1 of
//                a rotation pair in one wave) -- replaces the separate kv_append launch.
// Rounding matches the training kernels exactly (bf16 residual sum, (s * rstd) * g, bf16 GEMM outputs before
// SwiGLU / RoPE), so decode logits agree with the model's forward pass.
//
// Mapping (wave64): a 256-thread workgroup owns 16 weight rows, 4 per wave, 16 lanes per row; lane l of a row
// reads 16-byte W vectors l, l + 16, ... (coalesced 256 B per row per step) and the matching normalized-input
// vectors from LDS; the 16 partial dots are reduced with xor shuffles inside the row's lanes.  The first 8 W
// vectors of each lane (the whole row for K <= 1024) are loaded before the prologue, so the weight stream's
// latency overlaps the input read / normalization; the rest streams 4 vectors in flight.
// Prologue variant (GemvArgs::part): the input rows are the split-K decode attention's partial (o, m, l)
// triples, merged here -- the output projection absorbs the flash-decoding combine launch.
#include <cstdlib>

#include "common.h"
#include "kernels.h"

namespace bpe {
namespace gv {

// Weight rows are streamed once per decode step, each by one workgroup: non-temporal loads (same-box A/B,
// GPT-2-small decode step: batch 1 0.372 -> 0.350 ms, batch 8 0.502 -> 0.490 ms)
__device__ __forceinline__ u16x8 wload(const u16* p) {
    return __builtin_nontemporal_load(reinterpret_cast<const u16x8*>(p));
}

constexpr int LPR = 16;  // lanes per weight row
constexpr int RPW = 4;   // rows per wave
constexpr int UNR = 4;   // W vectors in flight per lane

constexpr int PF = 8;     // W vectors per lane issued before the prologue (all of a row for K <= 1024)

// Prologue shared by both kernels: input row m (< M) -> LDS row m (stride ldh): x (+ xd, with the sum written
// to xsum by workgroup 0), RMSNorm'd when ln is given; or, with part, the merged decode-attention partials.
__device__ __forceinline__ void gemv_prologue_rows(const GemvArgs& a, u16* hs, int ldh, int tid) {
    const int lane = tid & 63, wv = tid >> 6, K = a.K, nv = K / 8;
    for (int m = wv; m < a.M; m += 4) {
        u16* hr = hs + (long)m * ldh;
        if (a.part != nullptr) {
            const int D = a.D, ns = a.nsplit;
            for (int i = lane; i < nv; i += 64) {
                const int h = (8 * i) / D, d0 = (8 * i) % D;
                const float* pb = a.part + ((long)m * a.H + h) * ns * (D + 2);
                float mx = -INFINITY;
                for (int sp = 0; sp < ns; ++sp) mx = fmaxf(mx, pb[sp * (D + 2) + D]);
                float ls = 0.f, o[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
                for (int sp = 0; sp < ns; ++sp) {
                    const float* pr = pb + sp * (D + 2);
                    const float ms = pr[D];
                    if (ms == -INFINITY) continue;
                    const float c = __expf(ms - mx);
                    ls += c * pr[D + 1];
#pragma unroll
                    for (int e = 0; e < 8; ++e) o[e] += c * pr[d0 + e];
                }
                u16x8 hv;
#pragma unroll
                for (int e = 0; e < 8; ++e) hv[e] = f2bf(ls > 0.f ? o[e] / ls : 0.f);
                *reinterpret_cast<u16x8*>(hr + 8 * i) = hv;
            }
            continue;
        }
        float ss = 0.f;
        for (int i = lane; i < nv; i += 64) {
            u16x8 xv = *reinterpret_cast<const u16x8*>(a.x + (long)m * a.ldx + 8 * i);
            if (a.xd != nullptr) {
                const u16x8 dv = *reinterpret_cast<const u16x8*>(a.xd + (long)m * a.ldx + 8 * i);
#pragma unroll
                for (int j = 0; j < 8; ++j) xv[j] = f2bf(bf2f(xv[j]) + bf2f(dv[j]));
                if (a.xsum != nullptr && blockIdx.x == 0)
                    *reinterpret_cast<u16x8*>(a.xsum + (long)m * K + 8 * i) = xv;
            }
#pragma unroll
            for (int j = 0; j < 8; ++j) ss += bf2f(xv[j]) * bf2f(xv[j]);
            *reinterpret_cast<u16x8*>(hr + 8 * i) = xv;
        }
        if (a.ln != nullptr) {
            ss = wave_sum(ss);
            const float r = rsqrtf(ss / (float)K + a.eps);
            for (int i = lane; i < nv; i += 64) {
                u16x8 hv = *reinterpret_cast<const u16x8*>(hr + 8 * i);
                const u16x8 g = *reinterpret_cast<const u16x8*>(a.ln + 8 * i);
#pragma unroll
                for (int j = 0; j < 8; ++j) hv[j] = f2bf(bf2f(hv[j]) * r * bf2f(g[j]));
                *reinterpret_cast<u16x8*>(hr + 8 * i) = hv;
            }
        }
    }
}

template <int MM, int EPI>
__global__ void __launch_bounds__(256) gemv_kernel(const GemvArgs a) {
    extern __shared__ __attribute__((aligned(16))) u16 hs[];  // [MM][K] normalized input rows (bf16)
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const int K = a.K, nv = K / 8;
    // ---- this lane's weight row (4 rows per wave, 16 lanes per row)
    const int slot = lane / LPR, l16 = lane % LPR;
    const int wslot = wv * RPW + slot;  // row slot within the workgroup (0..15)
    int n, j = 0;
    bool valid;
    if constexpr (EPI == 1) {  // slots (2s, 2s+1) = rows (j, F + j) of logical output column j
        const int F = a.N / 2;
        j = blockIdx.x * 8 + wslot / 2;
        valid = j < F;
        n = (wslot & 1) ? F + j : j;
    } else {
        n = blockIdx.x * 16 + wslot;
        valid = n < a.N;
    }
    const u16* wr = reinterpret_cast<const u16*>(a.W) + (long)(valid ? n : 0) * a.ldw;
    // the first PF weight vectors are in flight while the prologue reads and normalizes the input rows: the
    // decode step is latency-bound, and the weight stream does not depend on the prologue
    u16x8 wp[PF];
#pragma unroll
    for (int u = 0; u < PF; ++u) {
        const int i = l16 + LPR * u;
        wp[u] = (valid && i < nv) ? wload(wr + 8 * i) : u16x8{};
    }
    // ---- prologue: rows M..MM-1 of the (rounded-up) LDS tile are zero, rows < M from the shared prologue
    for (int m = a.M + wv; m < MM; m += 4)
        for (int i = lane; i < nv; i += 64) *reinterpret_cast<u16x8*>(hs + (long)m * K + 8 * i) = u16x8{};
    gemv_prologue_rows(a, hs, K, tid);
    __syncthreads();
    // ---- main loop: 4 rows per wave, 16 lanes per row
    float acc[MM];
#pragma unroll
    for (int m = 0; m < MM; ++m) acc[m] = 0.f;
    if (valid) {
#pragma unroll
        for (int u = 0; u < PF; ++u) {
            const int i = l16 + LPR * u;
            if (i >= nv) break;
#pragma unroll
            for (int m = 0; m < MM; ++m) {
                const u16x8 hv = *reinterpret_cast<const u16x8*>(hs + (long)m * K + 8 * i);
#pragma unroll
                for (int e = 0; e < 8; ++e) acc[m] += bf2f(wp[u][e]) * bf2f(hv[e]);
            }
        }
        for (int i0 = l16 + LPR * PF; i0 < nv; i0 += LPR * UNR) {
            u16x8 w[UNR];
#pragma unroll
            for (int u = 0; u < UNR; ++u) {
                const int i = i0 + LPR * u;
                w[u] = i < nv ? wload(wr + 8 * i) : u16x8{};
            }
#pragma unroll
            for (int u = 0; u < UNR; ++u) {
                const int i = i0 + LPR * u;
                if (i >= nv) break;
#pragma unroll
                for (int m = 0; m < MM; ++m) {
                    const u16x8 hv = *reinterpret_cast<const u16x8*>(hs + (long)m * K + 8 * i);
#pragma unroll
                    for (int e = 0; e < 8; ++e) acc[m] += bf2f(w[u][e]) * bf2f(hv[e]);
                }
            }
        }
    }
#pragma unroll
    for (int m = 0; m < MM; ++m) {
#pragma unroll
        for (int off = LPR / 2; off > 0; off >>= 1) acc[m] += __shfl_xor(acc[m], off);
    }
    // ---- epilogues (lane l16 == 0 of each row holds the dots; partners are one row slot apart = 16 lanes)
    if constexpr (EPI == 0) {
        if (valid && l16 == 0)
            for (int m = 0; m < a.M; ++m) reinterpret_cast<u16*>(a.y)[(long)m * a.ldy + n] = f2bf(acc[m]);
    } else if constexpr (EPI == 1) {
        float other[MM];
#pragma unroll
        for (int m = 0; m < MM; ++m) other[m] = __shfl_xor(acc[m], LPR);
        if (valid && l16 == 0 && (wslot & 1) == 0)
            for (int m = 0; m < a.M; ++m) {
                const float g = bf2f(f2bf(acc[m])), u = bf2f(f2bf(other[m]));
                reinterpret_cast<u16*>(a.y)[(long)m * a.ldy + j] = f2bf(g * (1.f / (1.f + __expf(-g))) * u);
            }
    } else {
        float other[MM];
#pragma unroll
        for (int m = 0; m < MM; ++m) other[m] = __shfl_xor(acc[m], LPR);
        const int D = a.D, H = a.H, Hkv = a.Hkv;
        const int hh = n / D, d = n % D, p = a.pos[0];
        const bool rot = a.cosT != nullptr && hh < H + Hkv;
        float c = 1.f, s = 0.f;
        if (rot && valid) {
            c = a.cosT[(long)p * (D / 2) + d / 2];
            s = a.sinT[(long)p * (D / 2) + d / 2];
        }
        if (valid && l16 == 0)
            for (int m = 0; m < a.M; ++m) {
                const float me = bf2f(f2bf(acc[m])), pa = bf2f(f2bf(other[m]));
                float v = me;
                if (rot) v = (d & 1) ? pa * s + me * c : me * c - pa * s;
                const u16 o = f2bf(v);
                if (hh < H) reinterpret_cast<u16*>(a.y)[(long)m * a.ldy + n] = o;
                else if (p < a.Lmax) {
                    const bool isk = hh < H + Hkv;
                    const int hk = isk ? hh - H : hh - H - Hkv;
                    u16* cache = reinterpret_cast<u16*>(isk ? a.kc : a.vc);
                    cache[(((long)m * Hkv + hk) * a.Lmax + p) * D + d] = o;
                }
            }
    }
}

// ---------------------------------------------------------------------------------------------------------
// MFMA variant (2 <= M <= 16 rows): the per-row VALU dot products above cost ~8 converts + 8 FMAs per weight
// element and row, so at batch 8 they, not the weight stream, set the time.  Here a workgroup owns 16 weight
// rows and its 4 waves split K in quarters; each wave runs v_mfma_f32_16x16x32_bf16 with A = 16 W rows x 32 k
// (lane l: row l & 15, k = 8 (l >> 4) .. +7 -- one 16-byte load) and B = h^T (k x token; lane l: token l & 15,
// rows >= M are zero fragments), i.e. C[n][m] = y[m][n].  The four partial 16x16 tiles are summed through LDS
// and every epilogue (plain / SwiGLU / QKV + RoPE + cache write) runs on that tile; the SwiGLU workgroup takes
// 8 W1 rows and the matching 8 W3 rows.  Input rows sit in LDS with a 16-byte pad per row (the B reads of 16
// tokens at one k would otherwise hit the same banks).
constexpr int MF_PF = 8;  // k-steps (32 each) of W in flight per wave

template <int EPI>
__global__ void __launch_bounds__(256) gemv_mfma_kernel(const GemvArgs a) {
    extern __shared__ __attribute__((aligned(16))) u16 hs[];  // [M][K + 8] input rows, then float red[4][16][17]
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const int K = a.K, ldh = K + 8, nks = K / 32;
    // ---- this lane's A row (weight row) and the workgroup's row block
    const int r16 = lane & 15, kq = lane >> 4;
    int n, j0 = 0;
    bool valid;
    if constexpr (EPI == 1) {  // rows 0..7: W1 rows j0.., rows 8..15: the matching W3 rows F + j0..
        const int F = a.N / 2;
        j0 = blockIdx.x * 8;
        const int j = j0 + (r16 & 7);
        valid = j < F;
        n = r16 < 8 ? j : F + j;
    } else {
        n = blockIdx.x * 16 + r16;
        valid = n < a.N;
    }
    const u16* wr = reinterpret_cast<const u16*>(a.W) + (long)(valid ? n : 0) * a.ldw + 8 * kq;
    // wave wv owns k-steps [ks0, ks1) (K split in quarters)
    const int per = (nks + 3) / 4, ks0 = min(nks, wv * per), ks1 = min(nks, ks0 + per);
    u16x8 wp[MF_PF];
#pragma unroll
    for (int u = 0; u < MF_PF; ++u) {
        const int ks = ks0 + u;
        wp[u] = (valid && ks < ks1) ? wload(wr + 32 * ks) : u16x8{};
    }
    gemv_prologue_rows(a, hs, ldh, tid);
    __syncthreads();
    // ---- MFMA main loop
    const bool tok = r16 < a.M;  // B column (token) of this lane
    const u16* hb = hs + (long)r16 * ldh + 8 * kq;
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int u = 0; u < MF_PF; ++u) {
        const int ks = ks0 + u;
        if (ks >= ks1) break;
        const u16x8 bv = tok ? *reinterpret_cast<const u16x8*>(hb + 32 * ks) : u16x8{};
        acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, wp[u]),
                                                      __builtin_bit_cast(bf16x8, bv), acc, 0, 0, 0);
    }
    for (int ks = ks0 + MF_PF; ks < ks1; ks += 4) {
        u16x8 w4[4];
#pragma unroll
        for (int u = 0; u < 4; ++u)
            w4[u] = (valid && ks + u < ks1) ? wload(wr + 32 * (ks + u)) : u16x8{};
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            if (ks + u >= ks1) break;
            const u16x8 bv = tok ? *reinterpret_cast<const u16x8*>(hb + 32 * (ks + u)) : u16x8{};
            acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, w4[u]),
                                                          __builtin_bit_cast(bf16x8, bv), acc, 0, 0, 0);
        }
    }
    // ---- sum the 4 waves' partial tiles: C[row = 4 kq + i][col = r16]
    float* red = reinterpret_cast<float*>(hs + (long)a.M * ldh);  // [4][16][17]
#pragma unroll
    for (int i = 0; i < 4; ++i) red[(wv * 16 + 4 * kq + i) * 17 + r16] = acc[i];
    __syncthreads();
    const int r = tid >> 4, m = tid & 15;  // output tile element (weight row r, token m)
    float c = 0.f, cp = 0.f;
#pragma unroll
    for (int w = 0; w < 4; ++w) c += red[(w * 16 + r) * 17 + m];
    if constexpr (EPI != 0) {
        const int rp = EPI == 1 ? (r + 8) & 15 : r ^ 1;  // SwiGLU partner (W3 row) / RoPE pair partner
#pragma unroll
        for (int w = 0; w < 4; ++w) cp += red[(w * 16 + rp) * 17 + m];
    }
    if (m >= a.M) return;
    if constexpr (EPI == 0) {
        const int nn = blockIdx.x * 16 + r;
        if (nn < a.N) reinterpret_cast<u16*>(a.y)[(long)m * a.ldy + nn] = f2bf(c);
    } else if constexpr (EPI == 1) {
        const int j = j0 + r;
        if (r < 8 && j < a.N / 2) {
            const float g = bf2f(f2bf(c)), u = bf2f(f2bf(cp));
            reinterpret_cast<u16*>(a.y)[(long)m * a.ldy + j] = f2bf(g * (1.f / (1.f + __expf(-g))) * u);
        }
    } else {
        const int nn = blockIdx.x * 16 + r;
        if (nn >= a.N) return;
        const int D = a.D, H = a.H, Hkv = a.Hkv;
        const int hh = nn / D, d = nn % D, p = a.pos[0];
        const float me = bf2f(f2bf(c)), pa = bf2f(f2bf(cp));
        float v = me;
        if (a.cosT != nullptr && hh < H + Hkv) {
            const float cs = a.cosT[(long)p * (D / 2) + d / 2], sn = a.sinT[(long)p * (D / 2) + d / 2];
            v = (d & 1) ? pa * sn + me * cs : me * cs - pa * sn;
        }
        const u16 o = f2bf(v);
        if (hh < H) reinterpret_cast<u16*>(a.y)[(long)m * a.ldy + nn] = o;
        else if (p < a.Lmax) {
            const bool isk = hh < H + Hkv;
            const int hk = isk ? hh - H : hh - H - Hkv;
            u16* cache = reinterpret_cast<u16*>(isk ? a.kc : a.vc);
            cache[(((long)m * Hkv + hk) * a.Lmax + p) * D + d] = o;
        }
    }
}

}  // namespace gv
}  // namespace bpe

using namespace bpe::gv;

size_t gemv_lds_bytes(int M, int K) {
    const int MM = M <= 1 ? 1 : M <= 2 ? 2 : M <= 4 ? 4 : 8;
    return (size_t)MM * K * 2;
}

static size_t gemv_mfma_lds_bytes(int M, int K) { return (size_t)M * (K + 8) * 2 + 4 * 16 * 17 * 4; }

static bool mfma_fits(int M, int K) { return M <= 16 && K % 32 == 0 && gemv_mfma_lds_bytes(M, K) <= 160 * 1024; }

// M <= 8 on either kernel; 9..16 rows only on the MFMA one (its B operand has 16 token columns)
bool gemv_ok(int M, int K) {
    if (M < 1 || K % 8 != 0) return false;
    if (M > 8) return mfma_fits(M, K);
    return gemv_lds_bytes(M, K) <= 160 * 1024 || mfma_fits(M, K);
}

template <int MM, int EPI>
static void launch_mm(const GemvArgs& a, int grid, size_t lds, hipStream_t s) {
    if (lds > 64 * 1024)
        hipFuncSetAttribute(reinterpret_cast<const void*>(&gemv_kernel<MM, EPI>),
                            hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    gemv_kernel<MM, EPI><<<grid, 256, lds, s>>>(a);
}

template <int EPI>
static void launch_epi(const GemvArgs& a, int grid, size_t lds, hipStream_t s) {
    if (a.M <= 1) launch_mm<1, EPI>(a, grid, lds, s);
    else if (a.M <= 2) launch_mm<2, EPI>(a, grid, lds, s);
    else if (a.M <= 4) launch_mm<4, EPI>(a, grid, lds, s);
    else launch_mm<8, EPI>(a, grid, lds, s);
}

// decode rows from which the MFMA variant runs (BPE_GEMV_MFMA_MIN_M, default 2)
static int mfma_min_m() {
    static const int v = [] {
        const char* e = getenv("BPE_GEMV_MFMA_MIN_M");
        return e ? atoi(e) : 2;
    }();
    return v;
}

template <int EPI>
static void launch_mfma(const GemvArgs& a, int grid, hipStream_t s) {
    const size_t lds = gemv_mfma_lds_bytes(a.M, a.K);
    if (lds > 64 * 1024)
        hipFuncSetAttribute(reinterpret_cast<const void*>(&gemv_mfma_kernel<EPI>),
                            hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    gemv_mfma_kernel<EPI><<<grid, 256, lds, s>>>(a);
}

void launch_gemv(const GemvArgs& a, int epi, hipStream_t s) {
    if ((a.M >= mfma_min_m() || a.M > 8 || gemv_lds_bytes(a.M, a.K) > 160 * 1024) && mfma_fits(a.M, a.K)) {
        if (epi == 1) launch_mfma<1>(a, (a.N / 2 + 7) / 8, s);
        else if (epi == 2) launch_mfma<2>(a, (a.N + 15) / 16, s);
        else launch_mfma<0>(a, (a.N + 15) / 16, s);
        return;
    }
    const size_t lds = gemv_lds_bytes(a.M, a.K);
    if (epi == 1) launch_epi<1>(a, (a.N / 2 + 7) / 8, lds, s);
    else if (epi == 2) launch_epi<2>(a, (a.N + 15) / 16, lds, s);
    else launch_epi<0>(a, (a.N + 15) / 16, lds, s);
}
