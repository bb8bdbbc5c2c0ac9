// KV-cache decode attention and KV-cache append, gfx950.  Serving path of the framework: the reference has no
// inference engine (SURVEY §1 "absent layers"); generation with a KV cache reuses the training model's weights
// (`models/generation.py`).
//
//   q [B, H, D] (RoPE already applied), cache K / V [B, Hkv, Lmax, D] (roped K), valid length L = *pos + 1:
//   out[b, h] = softmax(q . K[b, h / G, :L]^T * scale) . V[b, h / G, :L]          (G = H / Hkv)
// (T > 1 new tokens per sequence -- chunked prefill into a filled cache, speculative verification -- is the same
// with one query row per (token, head) and token t limited to L = *pos + t + 1.)
//
// The position lives in device memory (int32), so one decode step -- append + attention for every layer -- is
// shape-static and is captured once into a HIP graph (the host never passes the growing length).
//
// Memory-bound (one pass over K and V per token), so the design is about bandwidth, not MFMA (guide
// Appendix B "Attention decode": K/V straight to VGPRs): the key range is split into chunks of CH keys, one
// workgroup per (batch, kv head, chunk) handles all G query heads of that kv head, so K and V are read once
// for the G heads.
//   1. scores: thread t owns key t of the chunk, streams its K row (16-byte loads) and dots it with the G query
//      rows (fp32, broadcast from LDS);
//   2. per head: block max / sum of exp over the chunk (fp32);
//   3. o[g][d] = sum_t p[g][t] V[t][d]: thread = (key partition, 8-wide d vector), 16-byte V loads; partitions
//      are reduced inside the wave with lane shuffles, then across the 4 waves through LDS;
//   4. the partial (o, m, l) of every (b, h, chunk) goes to fp32 scratch; a combine kernel merges the chunks
//      (flash-decoding) and writes bf16.  Chunks past the valid length write m = -inf and are skipped.  The
//      small-batch decode step skips the combine launch: the output projection's prologue merges the partials
//      (decode_gemv.hip, GemvArgs::part).
// All of a chunk's K and V loads are issued at kernel entry (register-resident, <= 128 VGPRs at D = 128).
#include "common.h"
#include "kernels.h"

namespace bpe {
namespace dec {

constexpr int CH = 256;  // keys per chunk (= threads per workgroup)

// MR (query rows per workgroup, >= G * T) is a template parameter: the per-row registers (m, l, o accumulators)
// must be statically indexed (guide §5.4 rule 20: runtime-indexed register arrays go to scratch).  Row r is
// new token t = r / G of the sequence and query head g = r % G of the kv head; with T new tokens at positions
// p0 .. p0 + T - 1 (p0 = *pos, already in the cache), token t attends keys [0, p0 + t] (causal within the chunk).
template <int D, int MR>
__global__ void __launch_bounds__(256) decode_attn_kernel(const __bf16* __restrict__ q, const __bf16* __restrict__ Kc,
                                                          const __bf16* __restrict__ Vc, float* __restrict__ part,
                                                          const int* __restrict__ pos, int H, int Hkv, int Lmax,
                                                          int nsplit, float scale, int T) {
    constexpr int DV = D / 8;     // 16-byte vectors per row
    constexpr int KP = 256 / DV;  // key partitions of the P.V step
    __shared__ float qs[MR][D];
    __shared__ float ps[MR][CH];
    __shared__ float red[2][4];
    __shared__ float ob[4][MR][D];
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const int bk = blockIdx.x / nsplit, split = blockIdx.x % nsplit;  // bk = b * Hkv + hk
    const int b = bk / Hkv, hk = bk % Hkv;
    const int G = H / Hkv, R = G * T;
    const int p0 = pos[0];
    const int L = min(p0 + T, Lmax);  // keys any row of this workgroup may see
    const int s0 = split * CH;
    // partial slot of row r: part[(((b * T + t) * H + h) * nsplit + split) * (D + 2)]
    auto prow = [&](int r) {
        return part + ((((long)b * T + r / G) * H + hk * G + r % G) * nsplit + split) * (D + 2);
    };
    if (s0 >= L) {  // uniform per workgroup: an empty chunk contributes nothing
        if (tid < R) {
            float* pr = prow(tid);
            pr[D] = -INFINITY;
            pr[D + 1] = 0.f;
        }
        return;
    }
    const int n = min(CH, L - s0);
    const long kvbase = ((long)bk * Lmax + s0) * D;
    // every K and V load of the chunk is issued up front (latency-bound at small batch: the q staging, the
    // score reductions and the softmax run while they are in flight)
    const bool ok = tid < n;
    u16x8 kr[DV];
    {
        const u16x8* kp = reinterpret_cast<const u16x8*>(Kc + kvbase + (long)tid * D);
#pragma unroll
        for (int v = 0; v < DV; ++v) kr[v] = ok ? kp[v] : u16x8{};
    }
    const int dv = tid % DV, kp = tid / DV;
    u16x8 vr[CH / KP];
#pragma unroll
    for (int j = 0; j < CH / KP; ++j) {
        const int t = kp + KP * j;
        vr[j] = t < n ? *reinterpret_cast<const u16x8*>(Vc + kvbase + (long)t * D + dv * 8) : u16x8{};
    }
    // query rows -> LDS (fp32, pre-scaled); rows >= R are zero
    for (int e = tid; e < MR * D; e += 256) {
        const int r = e / D, d = e % D;
        qs[r][d] = r < R ? bf2f(reinterpret_cast<const u16*>(q)[((((long)b * T + r / G) * H) + hk * G + r % G) * D + d]) *
                               scale
                         : 0.f;
    }
    __syncthreads();
    // 1. scores (key s0 + tid is visible to row r iff it is <= p0 + r / G)
    {
        float s[MR];
#pragma unroll
        for (int r = 0; r < MR; ++r) s[r] = 0.f;
        if (ok) {
#pragma unroll
            for (int v = 0; v < DV; ++v) {
                const u16x8 t = kr[v];
#pragma unroll
                for (int j = 0; j < 8; ++j) {
                    const float kx = bf2f(t[j]);
#pragma unroll
                    for (int r = 0; r < MR; ++r) s[r] += qs[r][8 * v + j] * kx;
                }
            }
        }
        const int key = s0 + tid;
#pragma unroll
        for (int r = 0; r < MR; ++r) ps[r][tid] = (ok && key <= p0 + r / G) ? s[r] : -INFINITY;
    }
    __syncthreads();
    // 2. per-row max / exp / sum over the chunk (a row with no visible key here: m = -inf, p = 0)
    float mg[MR], lg[MR];
#pragma unroll
    for (int r = 0; r < MR; ++r) {
        float m = wave_max(ps[r][tid]);
        if (lane == 0) red[0][wv] = m;
        __syncthreads();
        m = fmaxf(fmaxf(red[0][0], red[0][1]), fmaxf(red[0][2], red[0][3]));
        const float p = (tid < n && m != -INFINITY) ? __expf(ps[r][tid] - m) : 0.f;
        ps[r][tid] = p;
        float sm = wave_sum(p);
        if (lane == 0) red[1][wv] = sm;
        __syncthreads();
        mg[r] = m;
        lg[r] = red[1][0] + red[1][1] + red[1][2] + red[1][3];
        __syncthreads();  // red[] reused by the next row
    }
    // 3. o[r][d] = sum_t p[r][t] V[t][d]; thread = (key partition kp, vector dv)
    float acc[MR][8];
#pragma unroll
    for (int r = 0; r < MR; ++r)
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[r][j] = 0.f;
#pragma unroll
    for (int jj = 0; jj < CH / KP; ++jj) {
        const int t = kp + KP * jj;
        if (t >= n) break;
        const u16x8 vv = vr[jj];
#pragma unroll
        for (int r = 0; r < MR; ++r) {
            const float p = ps[r][t];
#pragma unroll
            for (int j = 0; j < 8; ++j) acc[r][j] += p * bf2f(vv[j]);
        }
    }
    // lanes that share dv differ by multiples of DV: butterfly over the wave's key partitions
#pragma unroll
    for (int off = DV; off < 64; off <<= 1)
#pragma unroll
        for (int r = 0; r < MR; ++r)
#pragma unroll
            for (int j = 0; j < 8; ++j) acc[r][j] += __shfl_xor(acc[r][j], off);
    if (lane < DV) {
#pragma unroll
        for (int r = 0; r < MR; ++r)
#pragma unroll
            for (int j = 0; j < 8; ++j) ob[wv][r][dv * 8 + j] = acc[r][j];
    }
    __syncthreads();
    // 4. partial results per row: {o[D], m, l}
    for (int e = tid; e < R * D; e += 256) {
        const int r = e / D, dd = e % D;
        prow(r)[dd] = ob[0][r][dd] + ob[1][r][dd] + ob[2][r][dd] + ob[3][r][dd];
    }
    if (tid < R) {  // the row statistics (registers, identical in every thread)
        float m = mg[0], l = lg[0];
#pragma unroll
        for (int r = 1; r < MR; ++r)
            if (tid == r) { m = mg[r]; l = lg[r]; }
        float* pr = prow(tid);
        pr[D] = m;
        pr[D + 1] = l;
    }
}

template <int D>
__global__ void __launch_bounds__(D) decode_combine_kernel(const float* __restrict__ part, __bf16* __restrict__ out,
                                                           int nsplit) {
    const long bh = blockIdx.x;
    const int d = threadIdx.x;
    const float* p = part + bh * nsplit * (D + 2);
    float M = -INFINITY;
    for (int s = 0; s < nsplit; ++s) M = fmaxf(M, p[s * (D + 2) + D]);
    float Lsum = 0.f, o = 0.f;
    for (int s = 0; s < nsplit; ++s) {
        const float m = p[s * (D + 2) + D];
        if (m == -INFINITY) continue;
        const float c = __expf(m - M);
        Lsum += c * p[s * (D + 2) + D + 1];
        o += c * p[s * (D + 2) + d];
    }
    reinterpret_cast<u16*>(out)[bh * D + d] = f2bf(Lsum > 0.f ? o / Lsum : 0.f);
}

// KV-cache append: fused-QKV rows [B*T, (H + 2*Hkv)*D] of T new tokens per sequence at positions
// *pos .. *pos+T-1 -> RoPE'd q [B*T, H*D] and roped K / plain V written into the caches [B, Hkv, Lmax, D].
// One thread per 16-byte vector (8 bf16); the rotation pairs (2i, 2i+1) never straddle a vector.
__global__ void __launch_bounds__(256) kv_append_kernel(const __bf16* __restrict__ qkv, long ld,
                                                        __bf16* __restrict__ qo, __bf16* __restrict__ Kc,
                                                        __bf16* __restrict__ Vc, const float* __restrict__ cosT,
                                                        const float* __restrict__ sinT, const int* __restrict__ pos,
                                                        int T, int H, int Hkv, int D, int Lmax, long total) {
    const int dv = D / 8, W = (H + 2 * Hkv) * dv;
    const int p0 = pos[0];
    for (long idx = blockIdx.x * 256L + threadIdx.x; idx < total; idx += (long)gridDim.x * 256) {
        const long r = idx / W;
        const int c = (int)(idx % W), hh = c / dv, d0 = (c % dv) * 8;
        const int b = (int)(r / T), p = p0 + (int)(r % T);
        if (p >= Lmax) continue;  // cache full: nothing is written past the end
        u16x8 x = *reinterpret_cast<const u16x8*>(qkv + r * ld + (long)hh * D + d0);
        if (hh < H + Hkv && cosT != nullptr) {
            const float* cs = cosT + (long)p * (D / 2) + d0 / 2;
            const float* sn = sinT + (long)p * (D / 2) + d0 / 2;
#pragma unroll
            for (int j = 0; j < 8; j += 2) {
                const float x1 = bf2f(x[j]), x2 = bf2f(x[j + 1]), cc = cs[j / 2], ss = sn[j / 2];
                x[j] = f2bf(x1 * cc - x2 * ss);
                x[j + 1] = f2bf(x1 * ss + x2 * cc);
            }
        }
        __bf16* dst;
        if (hh < H) dst = qo + r * (long)H * D + (long)hh * D + d0;
        else if (hh < H + Hkv) dst = Kc + (((long)b * Hkv + (hh - H)) * Lmax + p) * D + d0;
        else dst = Vc + (((long)b * Hkv + (hh - H - Hkv)) * Lmax + p) * D + d0;
        *reinterpret_cast<u16x8*>(dst) = x;
    }
}

}  // namespace dec
}  // namespace bpe

using namespace bpe::dec;

int decode_attn_splits(int Lmax) { return (Lmax + CH - 1) / CH; }

// T new tokens per sequence: the G * T query rows of a kv head share one workgroup (at most 8)
bool decode_attn_ok(int H, int Hkv, int D, int T) {
    const int G = Hkv > 0 ? H / Hkv : 0;
    return (D == 64 || D == 128) && Hkv > 0 && H % Hkv == 0 && T >= 1 && G >= 1 && G * T <= 8;
}

template <int D>
static void launch_d(const void* q, const void* k, const void* v, float* part, void* out, const int* pos, int B,
                     int T, int H, int Hkv, int Lmax, float scale, hipStream_t s) {
    const int ns = decode_attn_splits(Lmax);
    const int grid = B * Hkv * ns;
    const int R = (H / Hkv) * T;
#define DEC(MR)                                                                                                   \
    decode_attn_kernel<D, MR><<<grid, 256, 0, s>>>((const __bf16*)q, (const __bf16*)k, (const __bf16*)v, part, pos, \
                                                   H, Hkv, Lmax, ns, scale, T)
    if (R <= 1) DEC(1);
    else if (R <= 2) DEC(2);
    else if (R <= 4) DEC(4);
    else DEC(8);
#undef DEC
    if (out != nullptr) decode_combine_kernel<D><<<B * T * H, D, 0, s>>>(part, (__bf16*)out, ns);
}

void launch_decode_attn(const void* q, const void* k, const void* v, float* part, void* out, const int* pos, int B,
                        int T, int H, int Hkv, int D, int Lmax, float scale, hipStream_t s) {
    if (D == 64) launch_d<64>(q, k, v, part, out, pos, B, T, H, Hkv, Lmax, scale, s);
    else launch_d<128>(q, k, v, part, out, pos, B, T, H, Hkv, Lmax, scale, s);
}

void launch_kv_append(const void* qkv, long ld, void* qo, void* Kc, void* Vc, const float* cosT, const float* sinT,
                      const int* pos, int B, int T, int H, int Hkv, int D, int Lmax, hipStream_t s) {
    const long total = (long)B * T * (H + 2 * Hkv) * (D / 8);
    const long want = (total + 255) / 256;
    const int grid = (int)(want < 8192 ? want : 8192);
    kv_append_kernel<<<grid, 256, 0, s>>>((const __bf16*)qkv, ld, (__bf16*)qo, (__bf16*)Kc, (__bf16*)Vc, cosT, sinT,
                                          pos, T, H, Hkv, D, Lmax, total);
}
