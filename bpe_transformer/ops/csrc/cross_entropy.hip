// Fused softmax cross-entropy forward + gradient for gfx950.
//
// Parity target: reference contract K13, `tests/adapters.py:440-455`
// (mean over rows of logsumexp(x) - x[target]; stable for x1000 logits,
// `tests/test_nn_utils.py:53`).
//
// Large rows (see ce_fwd_bwd_reg_kernel for the default): one 256-thread block per row.  Pass 1 streams the row once with 16-byte
// vector loads, keeping a per-lane online (max, sum-exp) pair; the block
// merges them.  Pass 2 re-reads the row (L2-resident: a 50k-vocab bf16 row is
// 100 KB) and writes dlogits = (softmax - onehot) * scale IN PLACE over the
// logits, so the LM head never needs a second full-size buffer and the
// backward is just two GEMMs.  `scale` (1 / number of valid targets) comes
// from device memory, so no host sync is needed.  Rows may start at any
// 2-byte-aligned address (vocab 50257 is odd): a scalar head reaches 16-byte
// alignment, then the vector body, then a scalar tail.
#include "common.h"
#include "kernels.h"

namespace bpe {

__device__ __forceinline__ void online_merge(float& m, float& s, float m2, float s2) {
    const float mn = fmaxf(m, m2);
    if (mn == -INFINITY) return;
    s = s * __expf(m - mn) + s2 * __expf(m2 - mn);
    m = mn;
}

template <typename T>
__global__ void __launch_bounds__(256) ce_fwd_bwd_kernel(T* __restrict__ logits, long ld,
                                                         const int64_t* __restrict__ targets, float* __restrict__ loss,
                                                         float* __restrict__ lse_out, const float* __restrict__ nvalid,
                                                         int V, long ignore_index, int write_grad) {
    constexpr int VN = Vec<T>::N;
    __shared__ float red_m[4], red_s[4];
    const long row = blockIdx.x;
    T* x = logits + row * ld;
    const int tid = threadIdx.x;
    // alignment split
    const uintptr_t addr = reinterpret_cast<uintptr_t>(x);
    int head = (int)(((16 - (addr & 15)) & 15) / sizeof(T));
    if (head > V) head = V;
    const int nv = (V - head) / VN;
    const int body_end = head + nv * VN;

    float m = -INFINITY, s = 0.f;
    if (tid < head) { m = ld1<T>(x + tid); s = 1.f; }
    for (int i = tid; i < nv; i += 256) {
        Vec<T> a;
        a.load(x + head + i * VN);
        float vm = a.v[0];
#pragma unroll
        for (int j = 1; j < VN; ++j) vm = fmaxf(vm, a.v[j]);
        float vs = 0.f;
#pragma unroll
        for (int j = 0; j < VN; ++j) vs += __expf(a.v[j] - vm);
        online_merge(m, s, vm, vs);
    }
    for (int i = body_end + tid; i < V; i += 256) online_merge(m, s, ld1<T>(x + i), 1.f);
    // wave merge
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        const float m2 = __shfl_xor(m, o, 64), s2 = __shfl_xor(s, o, 64);
        online_merge(m, s, m2, s2);
    }
    if ((tid & 63) == 0) { red_m[tid >> 6] = m; red_s[tid >> 6] = s; }
    __syncthreads();
    m = red_m[0]; s = red_s[0];
#pragma unroll
    for (int w = 1; w < 4; ++w) online_merge(m, s, red_m[w], red_s[w]);
    const float lse = m + __logf(s);

    const long t = targets[row];
    const bool valid = (t != ignore_index);
    if (tid == 0) {
        float l = 0.f;
        if (valid) l = lse - ld1<T>(x + t);
        loss[row] = l;
        if (lse_out) lse_out[row] = lse;
    }
    if (!write_grad) return;
    __syncthreads();  // everyone has read x[t] (tid 0) before it is overwritten
    const float sc = valid ? 1.f / fmaxf(*nvalid, 1.f) : 0.f;
    if (tid < head) {
        const float p = __expf(ld1<T>(x + tid) - lse);
        st1<T>(x + tid, (p - (tid == t ? 1.f : 0.f)) * sc);
    }
    for (int i = tid; i < nv; i += 256) {
        const int base = head + i * VN;
        Vec<T> a;
        a.load(x + base);
#pragma unroll
        for (int j = 0; j < VN; ++j) a.v[j] = (__expf(a.v[j] - lse) - ((long)(base + j) == t ? 1.f : 0.f)) * sc;
        a.store(x + base);
    }
    for (int i = body_end + tid; i < V; i += 256) {
        const float p = __expf(ld1<T>(x + i) - lse);
        st1<T>(x + i, (p - (i == t ? 1.f : 0.f)) * sc);
    }
}

// Register-resident variant (the default when a row fits: V <= 512 threads x MAXV vectors): one 512-thread
// block per row loads the row ONCE into registers (16-byte vectors, <= MAXV per thread), then block max ->
// block sum of exp(x - max) -> writes (softmax - onehot) * scale from the registers.  One HBM read and one
// write per element (the two-pass kernel above re-reads the row, which at 8 blocks/CU x 100 KB rows falls
// out of L2), and no online (max, sum) merges.
template <typename T> struct RawVec;
template <> struct RawVec<__bf16> { typedef u16x8 type; };
template <> struct RawVec<float> { typedef f32x4 type; };

template <typename T>
__device__ __forceinline__ float raw_get(const typename RawVec<T>::type& r, int j);
template <> __device__ __forceinline__ float raw_get<__bf16>(const u16x8& r, int j) { return bf2f(r[j]); }
template <> __device__ __forceinline__ float raw_get<float>(const f32x4& r, int j) { return r[j]; }
template <typename T>
__device__ __forceinline__ void raw_set(typename RawVec<T>::type& r, int j, float v);
template <> __device__ __forceinline__ void raw_set<__bf16>(u16x8& r, int j, float v) { r[j] = f2bf(v); }
template <> __device__ __forceinline__ void raw_set<float>(f32x4& r, int j, float v) { r[j] = v; }

template <typename T, int MAXV>
__global__ void __launch_bounds__(512) ce_fwd_bwd_reg_kernel(T* __restrict__ logits, long ld,
                                                             const int64_t* __restrict__ targets,
                                                             float* __restrict__ loss, float* __restrict__ lse_out,
                                                             const float* __restrict__ nvalid, int V,
                                                             long ignore_index, int write_grad) {
    constexpr int VN = Vec<T>::N, NTH = 512;
    typedef typename RawVec<T>::type R;
    __shared__ float red[2][8];
    const long row = blockIdx.x;
    T* x = logits + row * ld;
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const uintptr_t addr = reinterpret_cast<uintptr_t>(x);
    int head = (int)(((16 - (addr & 15)) & 15) / sizeof(T));
    if (head > V) head = V;
    const int nv = (V - head) / VN;
    const int body_end = head + nv * VN;
    const int ntail = V - body_end;
    const long t = targets[row];
    const bool valid = (t != ignore_index);

    R r[MAXV];
#pragma unroll
    for (int k = 0; k < MAXV; ++k) {
        const int i = tid + k * NTH;
        if (i < nv) r[k] = __builtin_nontemporal_load(reinterpret_cast<const R*>(x + head + (long)i * VN));
    }
    // one scalar per thread covers the unaligned head (< VN elements) and the tail (< VN elements)
    const int si = tid < head ? tid : (tid >= 64 && tid - 64 < ntail ? body_end + tid - 64 : -1);
    const float sx = si >= 0 ? ld1<T>(x + si) : -INFINITY;
    const float xt = (tid == 0 && valid) ? ld1<T>(x + t) : 0.f;

    float m = sx;
#pragma unroll
    for (int k = 0; k < MAXV; ++k)
        if (tid + k * NTH < nv) {
#pragma unroll
            for (int j = 0; j < VN; ++j) m = fmaxf(m, raw_get<T>(r[k], j));
        }
    m = wave_max(m);
    if (lane == 0) red[0][wv] = m;
    __syncthreads();
    m = red[0][0];
#pragma unroll
    for (int w = 1; w < NTH / 64; ++w) m = fmaxf(m, red[0][w]);
    float sm = si >= 0 ? __expf(sx - m) : 0.f;
#pragma unroll
    for (int k = 0; k < MAXV; ++k)
        if (tid + k * NTH < nv) {
#pragma unroll
            for (int j = 0; j < VN; ++j) sm += __expf(raw_get<T>(r[k], j) - m);
        }
    sm = wave_sum(sm);
    if (lane == 0) red[1][wv] = sm;
    __syncthreads();
    sm = 0.f;
#pragma unroll
    for (int w = 0; w < NTH / 64; ++w) sm += red[1][w];
    const float lse = m + __logf(sm);
    if (tid == 0) {
        loss[row] = valid ? lse - xt : 0.f;
        if (lse_out) lse_out[row] = lse;
    }
    if (!write_grad) return;
    const float sc = valid ? 1.f / fmaxf(*nvalid, 1.f) : 0.f;
    if (si >= 0) st1<T>(x + si, (__expf(sx - lse) - (si == t ? 1.f : 0.f)) * sc);
#pragma unroll
    for (int k = 0; k < MAXV; ++k) {
        const int i = tid + k * NTH;
        if (i < nv) {
            const int base = head + i * VN;
            Vec<T> o;
#pragma unroll
            for (int j = 0; j < VN; ++j) o.v[j] = (__expf(raw_get<T>(r[k], j) - lse) - ((long)(base + j) == t ? 1.f : 0.f)) * sc;
            // streamed once in, once out: non-temporal on both sides (the row is not re-read by this kernel)
            R ov;
#pragma unroll
            for (int j = 0; j < VN; ++j) raw_set<T>(ov, j, o.v[j]);
            __builtin_nontemporal_store(ov, reinterpret_cast<R*>(x + base));
        }
    }
}

}  // namespace bpe

using namespace bpe;

void launch_ce_fwd_bwd(int dtype, void* logits, long ld, const int64_t* targets, float* loss, float* lse,
                       const float* nvalid, int M, int V, long ignore_index, int write_grad, hipStream_t s) {
    if (M == 0) return;
    constexpr int MAXV = 16;
    const int vn = dtype == DT_BF16 ? 8 : 4;
    if ((V + vn) / vn <= 512 * MAXV) {  // row fits in registers (V <= 65528 bf16 / 32760 fp32)
        if (dtype == DT_BF16)
            ce_fwd_bwd_reg_kernel<__bf16, MAXV><<<M, 512, 0, s>>>((__bf16*)logits, ld, targets, loss, lse, nvalid, V,
                                                                  ignore_index, write_grad);
        else
            ce_fwd_bwd_reg_kernel<float, MAXV><<<M, 512, 0, s>>>((float*)logits, ld, targets, loss, lse, nvalid, V,
                                                                 ignore_index, write_grad);
        return;
    }
    if (dtype == DT_BF16)
        ce_fwd_bwd_kernel<__bf16><<<M, 256, 0, s>>>((__bf16*)logits, ld, targets, loss, lse, nvalid, V, ignore_index,
                                                    write_grad);
    else
        ce_fwd_bwd_kernel<float><<<M, 256, 0, s>>>((float*)logits, ld, targets, loss, lse, nvalid, V, ignore_index,
                                                   write_grad);
}
