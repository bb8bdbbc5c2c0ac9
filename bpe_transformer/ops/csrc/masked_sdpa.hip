// Generic masked scaled-dot-product attention, gfx950 (MI355X): the full reference contract K7
// (`/root/reference/tests/adapters.py:92-110`): softmax(Q K^T * scale + (mask ? 0 : -inf)) V with an arbitrary
// boolean mask (True = attend) broadcast over any leading dims, fp32 or bf16 operands, fp32 math throughout.
//
// This is the contract path (arbitrary masks, any sequence lengths, head dims up to 128), not the training path:
// the model's causal attention runs the MFMA flash kernels (flash_attn_fwd_v4.hip / flash_attn_bwd_split.hip),
// whose bf16 operands could not meet the contract's fp32 tolerance (atol 1e-6, `tests/test_model.py:57-74`).
//
// Structure: one workgroup = 4 waves = 4 query rows of one (batch, head); key / value tiles of 64 rows are staged
// in LDS as fp32 by all 256 threads (K rows padded to D + 1 floats, so the 64 lanes reading one column of 64
// different rows hit 64 different banks).  Per tile, lane j owns key j: its score is a D-long fp32 FMA chain against
// the wave's query row (an LDS broadcast); the online softmax keeps the running max / sum in registers (one wave
// max and one wave sum per tile); then lane j owns output columns j and j + 64 and adds sum_k p_k V[k][j] over the
// tile's keys (P broadcast from LDS, V rows read conflict-free).  A row whose every key is masked produces NaN, as
// softmax over all -inf does.
#include "common.h"
#include "kernels.h"

namespace bpe {
namespace msdpa {

constexpr int KT = 64, NW = 4, DMAX = 128;

template <typename T>
__device__ __forceinline__ float ld(const T* p);
template <>
__device__ __forceinline__ float ld<float>(const float* p) { return *p; }
template <>
__device__ __forceinline__ float ld<u16>(const u16* p) { return bf2f(*p); }
template <typename T>
__device__ __forceinline__ T cvt(float x);
template <>
__device__ __forceinline__ float cvt<float>(float x) { return x; }
template <>
__device__ __forceinline__ u16 cvt<u16>(float x) { return f2bf(x); }

template <typename T>
__global__ void __launch_bounds__(NW * 64)
masked_sdpa_kernel(const T* __restrict__ Q, const T* __restrict__ K, const T* __restrict__ V,
                   const uint8_t* __restrict__ Mk, long msb, long msq, long msk, T* __restrict__ O, int Sq, int Sk,
                   int D, int Dv, float scale) {
    __shared__ float Ks[KT * (DMAX + 1)];
    __shared__ float Vs[KT * DMAX];
    __shared__ float qs[NW][DMAX];
    __shared__ float ps[NW][KT];
    const int tid = threadIdx.x, w = tid >> 6, l = tid & 63;
    const long bh = blockIdx.y;
    const int q = blockIdx.x * NW + w;
    const bool active = q < Sq;  // every thread stays for the barriers
    const T* qp = Q + (bh * Sq + (active ? q : 0)) * D;
    for (int d = l; d < D; d += 64) qs[w][d] = ld(qp + d);
    const uint8_t* mrow = Mk != nullptr ? Mk + bh * msb + (long)(active ? q : 0) * msq : nullptr;
    const int DK = D + 1;
    float m_run = -INFINITY, l_run = 0.f, o0 = 0.f, o1 = 0.f;
    for (int k0 = 0; k0 < Sk; k0 += KT) {
        __syncthreads();  // the previous tile's K / V / P are no longer read
        const int nk = min(KT, Sk - k0);
        for (int e = tid; e < nk * D; e += NW * 64) {
            const int r = e / D, c = e - r * D;
            Ks[r * DK + c] = ld(K + (bh * Sk + k0 + r) * D + c);
        }
        for (int e = tid; e < nk * Dv; e += NW * 64) {
            const int r = e / Dv, c = e - r * Dv;
            Vs[r * DMAX + c] = ld(V + (bh * Sk + k0 + r) * Dv + c);
        }
        __syncthreads();
        if (active) {
            float s = -INFINITY;
            if (l < nk && (mrow == nullptr || mrow[(long)(k0 + l) * msk] != 0)) {
                float acc = 0.f;
                const float* kr = Ks + l * DK;
                for (int d = 0; d < D; ++d) acc = fmaf(qs[w][d], kr[d], acc);
                s = acc * scale;
            }
            const float m_new = fmaxf(m_run, wave_max(s));
            // nothing unmasked yet (m_new = -inf): P = 0, nothing to rescale
            const float p = s == -INFINITY ? 0.f : expf(s - m_new);
            const float alpha = m_run == -INFINITY ? (m_new == -INFINITY ? 1.f : 0.f) : expf(m_run - m_new);
            m_run = m_new;
            l_run = l_run * alpha + wave_sum(p);
            ps[w][l] = p;
            o0 *= alpha;
            o1 *= alpha;
            // the wave's P row is read by all its lanes: a wave's LDS operations complete in issue order, so its
            // own later reads see these writes (no workgroup barrier: the other waves use their own rows)
            __builtin_amdgcn_wave_barrier();
            for (int j = 0; j < nk; ++j) {
                const float pj = ps[w][j];
                if (l < Dv) o0 = fmaf(pj, Vs[j * DMAX + l], o0);
                if (l + 64 < Dv) o1 = fmaf(pj, Vs[j * DMAX + l + 64], o1);
            }
        }
    }
    if (active) {
        const float inv = l_run > 0.f ? 1.f / l_run : __builtin_nanf("");
        T* op = O + (bh * Sq + q) * Dv;
        if (l < Dv) op[l] = cvt<T>(o0 * inv);
        if (l + 64 < Dv) op[l + 64] = cvt<T>(o1 * inv);
    }
}

}  // namespace msdpa
}  // namespace bpe

void launch_masked_sdpa(int dtype, const void* q, const void* k, const void* v, const uint8_t* mask, long msb,
                        long msq, long msk, void* o, int BH, int Sq, int Sk, int D, int Dv, float scale,
                        hipStream_t s) {
    using namespace bpe::msdpa;
    const dim3 grid((Sq + NW - 1) / NW, BH);
    if (dtype == 0)
        masked_sdpa_kernel<float><<<grid, NW * 64, 0, s>>>((const float*)q, (const float*)k, (const float*)v, mask,
                                                           msb, msq, msk, (float*)o, Sq, Sk, D, Dv, scale);
    else
        masked_sdpa_kernel<u16><<<grid, NW * 64, 0, s>>>((const u16*)q, (const u16*)k, (const u16*)v, mask, msb, msq,
                                                         msk, (u16*)o, Sq, Sk, D, Dv, scale);
}
