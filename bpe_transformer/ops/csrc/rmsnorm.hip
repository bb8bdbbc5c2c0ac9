// RMSNorm forward / backward for gfx950.
//
// Parity target: reference contract K4, `tests/adapters.py:364-384`
// (y = x / sqrt(mean(x^2) + eps) * g, statistics in fp32).
//
// Layout: x is [M, N] row-major, one wave64 per row, 16-byte vector accesses
// (8 bf16 or 4 fp32 per lane).  The backward writes dx directly and produces
// the weight gradient deterministically: each wave keeps its lane's column
// partial sums in registers across a grid-stride sweep of rows, the 4 waves of
// a block combine through LDS, and a second tiny kernel sums the per-block
// partials in a fixed order (no float atomics, bitwise reproducible).
#include "common.h"
#include "kernels.h"

namespace bpe {

template <typename T>
__global__ void __launch_bounds__(256) rmsnorm_fwd_kernel(const T* __restrict__ x, const T* __restrict__ w,
                                                          T* __restrict__ y, float* __restrict__ rstd_out,
                                                          int M, int N, float eps) {
    constexpr int V = Vec<T>::N;
    const int lane = threadIdx.x & 63;
    const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (row >= M) return;
    const T* xr = x + (size_t)row * N;
    T* yr = y + (size_t)row * N;
    const int nvec = N / V;
    float ss = 0.f;
    for (int i = lane; i < nvec; i += 64) {
        Vec<T> a;
        a.load(xr + i * V);
#pragma unroll
        for (int j = 0; j < V; ++j) ss += a.v[j] * a.v[j];
    }
    ss = wave_sum(ss);
    const float r = rsqrtf(ss / (float)N + eps);
    if (lane == 0 && rstd_out) rstd_out[row] = r;
    for (int i = lane; i < nvec; i += 64) {
        Vec<T> a, g;
        a.load(xr + i * V);
        g.load(w + i * V);
#pragma unroll
        for (int j = 0; j < V; ++j) a.v[j] = a.v[j] * r * g.v[j];
        a.store(yr + i * V);
    }
}

template <typename T> struct RawV;
template <> struct RawV<__bf16> {
    typedef u16x8 type;
    static __device__ __forceinline__ float get(const u16x8& r, int j) { return bf2f(r[j]); }
};
template <> struct RawV<float> {
    typedef f32x4 type;
    static __device__ __forceinline__ float get(const f32x4& r, int j) { return r[j]; }
};

// Residual add fused into the norm: s = x + d (rounded to T: the residual stream is stored in T), y = RMSNorm(s).
// Replaces "addmm(x, o, W^T)" (a full copy of x into the GEMM output, then a beta = 1 GEMM) + rmsnorm with a
// plain GEMM and one pass here.  C > 0: the lane's C chunks of s stay in registers for the second sweep (no
// read-after-write of the just-stored sum); C == 0: any width, the second sweep re-reads s (L2-resident).
template <typename T, int C>
__global__ void __launch_bounds__(256) add_rmsnorm_fwd_kernel(const T* __restrict__ x, const T* __restrict__ d,
                                                              const T* __restrict__ w, T* __restrict__ sum,
                                                              T* __restrict__ y, float* __restrict__ rstd_out, int M,
                                                              int N, float eps) {
    constexpr int V = Vec<T>::N;
    const int lane = threadIdx.x & 63;
    const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (row >= M) return;
    const size_t off = (size_t)row * N;
    const int nvec = N / V;
    float ss = 0.f;
    if constexpr (C > 0) {
        Vec<T> keep[C];
#pragma unroll
        for (int c = 0; c < C; ++c) {
            const int i = c * 64 + lane;
            if (i < nvec) {
                Vec<T> a, b;
                a.load(x + off + i * V);
                b.load(d + off + i * V);
#pragma unroll
                for (int j = 0; j < V; ++j) {
                    float v = a.v[j] + b.v[j];
                    if constexpr (sizeof(T) == 2) v = bf2f(f2bf(v));  // statistics of the stored (rounded) sum
                    a.v[j] = v;
                    ss += v * v;
                }
                a.store(sum + off + i * V);
                keep[c] = a;
            }
        }
        ss = wave_sum(ss);
        const float r = rsqrtf(ss / (float)N + eps);
        if (lane == 0 && rstd_out) rstd_out[row] = r;
#pragma unroll
        for (int c = 0; c < C; ++c) {
            const int i = c * 64 + lane;
            if (i < nvec) {
                Vec<T> g;
                g.load(w + i * V);
#pragma unroll
                for (int j = 0; j < V; ++j) keep[c].v[j] = keep[c].v[j] * r * g.v[j];
                keep[c].store(y + off + i * V);
            }
        }
        return;
    }
    for (int i = lane; i < nvec; i += 64) {
        Vec<T> a, b;
        a.load(x + off + i * V);
        b.load(d + off + i * V);
#pragma unroll
        for (int j = 0; j < V; ++j) {
            float v = a.v[j] + b.v[j];
            if constexpr (sizeof(T) == 2) v = bf2f(f2bf(v));
            a.v[j] = v;
            ss += v * v;
        }
        a.store(sum + off + i * V);
    }
    ss = wave_sum(ss);
    const float r = rsqrtf(ss / (float)N + eps);
    if (lane == 0 && rstd_out) rstd_out[row] = r;
    for (int i = lane; i < nvec; i += 64) {
        Vec<T> a, g;
        a.load(sum + off + i * V);
        g.load(w + i * V);
#pragma unroll
        for (int j = 0; j < V; ++j) a.v[j] = a.v[j] * r * g.v[j];
        a.store(y + off + i * V);
    }
}

// C = number of 16-byte column chunks each lane owns (ceil(N / V / 64)).  Activations go through the
// streaming (non-temporal) accessors: 140.3 -> 138.3 us at 131072 x 768, where each tensor is ~200 MB.  The
// forward kernels, and the wide kernel below at Llama's 67 MB tensors (which fit the 256 MB Infinity Cache),
// measured slower with them (docs/performance.md).
template <typename T, int C>
__global__ void __launch_bounds__(256) rmsnorm_bwd_kernel(const T* __restrict__ dy, const T* __restrict__ x,
                                                          const T* __restrict__ w,
                                                          const float* __restrict__ rstd, T* __restrict__ dx,
                                                          float* __restrict__ dw_partial,
                                                          const T* __restrict__ dres, int M, int N) {
    constexpr int V = Vec<T>::N;
    extern __shared__ __attribute__((aligned(16))) float lds[];  // [4][N]
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const int nvec = N / V;
    float dwacc[C][V];
    float wv[C][V];
#pragma unroll
    for (int c = 0; c < C; ++c) {
        const int i = c * 64 + lane;
#pragma unroll
        for (int j = 0; j < V; ++j) { dwacc[c][j] = 0.f; wv[c][j] = 0.f; }
        if (i < nvec) {
            Vec<T> g;
            g.load(w + i * V);
#pragma unroll
            for (int j = 0; j < V; ++j) wv[c][j] = g.v[j];
        }
    }
    // Rows are software-pipelined: the next row's x / dy / dres (raw 16-byte vectors) and rstd are loaded
    // while this row is reduced and written, and dres comes with the first loads instead of after the
    // reduction -- each wave keeps one row of loads in flight behind its compute.
    typedef typename RawV<T>::type R;
    const R zero{};
    R xa[C], ga[C], ra[C];
    float rcur = 0.f;
    auto load_row = [&](int row, R* xo, R* go, R* ro, float& rr) {
        rr = rstd[row];
#pragma unroll
        for (int c = 0; c < C; ++c) {
            const int i = c * 64 + lane;
            const bool ok = i < nvec;
            xo[c] = ok ? ld_stream(reinterpret_cast<const R*>(x + (size_t)row * N + i * V)) : zero;
            go[c] = ok ? ld_stream(reinterpret_cast<const R*>(dy + (size_t)row * N + i * V)) : zero;
            ro[c] = (ok && dres) ? ld_stream(reinterpret_cast<const R*>(dres + (size_t)row * N + i * V)) : zero;
        }
    };
    const int stride = gridDim.x * 4;
    int row = blockIdx.x * 4 + wid;
    if (row < M) load_row(row, xa, ga, ra, rcur);
    for (; row < M; row += stride) {
        R xb[C], gb[C], rb[C];
        float rnext = 0.f;
        if (row + stride < M) load_row(row + stride, xb, gb, rb, rnext);
        const float r = rcur;
        // x_hat and dy are re-expanded from the raw vectors in both passes (register budget: 4 waves / SIMD)
        float dot = 0.f;
#pragma unroll
        for (int c = 0; c < C; ++c)
#pragma unroll
            for (int j = 0; j < V; ++j)
                dot += RawV<T>::get(ga[c], j) * wv[c][j] * (RawV<T>::get(xa[c], j) * r);
        dot = wave_sum(dot) / (float)N;
        T* dxr = dx + (size_t)row * N;
#pragma unroll
        for (int c = 0; c < C; ++c) {
            const int i = c * 64 + lane;
            if (i < nvec) {
                Vec<T> o;
#pragma unroll
                for (int j = 0; j < V; ++j) {
                    const float xh = RawV<T>::get(xa[c], j) * r, g = RawV<T>::get(ga[c], j);
                    // fused residual-branch gradient: dx += dres (ra is zero without dres)
                    o.v[j] = r * (g * wv[c][j] - xh * dot) + RawV<T>::get(ra[c], j);
                    dwacc[c][j] += g * xh;
                }
                o.store_s(dxr + i * V);
            }
        }
#pragma unroll
        for (int c = 0; c < C; ++c) {
            xa[c] = xb[c];
            ga[c] = gb[c];
            ra[c] = rb[c];
        }
        rcur = rnext;
    }
    // combine the 4 waves of this block through LDS, then one partial row per block
#pragma unroll
    for (int c = 0; c < C; ++c) {
        const int i = c * 64 + lane;
        if (i < nvec) {
#pragma unroll
            for (int j = 0; j < V; ++j) lds[wid * N + i * V + j] = dwacc[c][j];
        }
    }
    __syncthreads();
    for (int col = threadIdx.x; col < N; col += 256) {
        float s = lds[col] + lds[N + col] + lds[2 * N + col] + lds[3 * N + col];
        dw_partial[(size_t)blockIdx.x * N + col] = s;
    }
}

// Half-wave rows (N / V a multiple of 32 and at most 128, e.g. d_model 768 in bf16: 96 vectors): each 32-lane half
// of a wave owns one row, lane vectors (lane & 31) + 32 c.  At N = 768 the one-wave-per-row kernel above leaves half
// of its lanes idle in its second chunk; here every lane holds 3 vectors per tensor and a wave has two rows' loads in
// flight (plus the next two prefetched).  Same arithmetic per element; the row dot product is summed over 32 lanes.
template <typename T, int C>
__global__ void __launch_bounds__(256) rmsnorm_bwd_hw_kernel(const T* __restrict__ dy, const T* __restrict__ x,
                                                             const T* __restrict__ w,
                                                             const float* __restrict__ rstd, T* __restrict__ dx,
                                                             float* __restrict__ dw_partial,
                                                             const T* __restrict__ dres, int M, int N) {
    constexpr int V = Vec<T>::N;
    extern __shared__ __attribute__((aligned(16))) float lds[];  // [4][N]
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, hl = lane & 31, half = lane >> 5;
    float dwacc[C][V], wv[C][V];
#pragma unroll
    for (int c = 0; c < C; ++c) {
        Vec<T> g;
        g.load(w + (c * 32 + hl) * V);
#pragma unroll
        for (int j = 0; j < V; ++j) { dwacc[c][j] = 0.f; wv[c][j] = g.v[j]; }
    }
    typedef typename RawV<T>::type R;
    R xa[C], ga[C], ra[C];
    float rcur = 0.f;
    auto load_row = [&](int row, R* xo, R* go, R* ro, float& rr) {
        rr = rstd[row];
#pragma unroll
        for (int c = 0; c < C; ++c) {
            const size_t off = (size_t)row * N + (c * 32 + hl) * V;
            xo[c] = ld_stream(reinterpret_cast<const R*>(x + off));
            go[c] = ld_stream(reinterpret_cast<const R*>(dy + off));
            ro[c] = dres ? ld_stream(reinterpret_cast<const R*>(dres + off)) : R{};
        }
    };
    // rows 2 (4 b + w) + half, stride 8 gridDim.x; M is even whenever this kernel runs (rows come in pairs)
    const int stride = gridDim.x * 8;
    int row = (blockIdx.x * 4 + wid) * 2 + half;
    if (row < M) load_row(row, xa, ga, ra, rcur);
    for (; row < M; row += stride) {
        R xb[C], gb[C], rb[C];
        float rnext = 0.f;
        if (row + stride < M) load_row(row + stride, xb, gb, rb, rnext);
        const float r = rcur;
        float dot = 0.f;
#pragma unroll
        for (int c = 0; c < C; ++c)
#pragma unroll
            for (int j = 0; j < V; ++j)
                dot += RawV<T>::get(ga[c], j) * wv[c][j] * (RawV<T>::get(xa[c], j) * r);
#pragma unroll
        for (int o = 16; o > 0; o >>= 1) dot += __shfl_xor(dot, o, 64);  // within the 32-lane half
        dot /= (float)N;
        T* dxr = dx + (size_t)row * N;
#pragma unroll
        for (int c = 0; c < C; ++c) {
            Vec<T> o;
#pragma unroll
            for (int j = 0; j < V; ++j) {
                const float xh = RawV<T>::get(xa[c], j) * r, g = RawV<T>::get(ga[c], j);
                o.v[j] = r * (g * wv[c][j] - xh * dot) + RawV<T>::get(ra[c], j);
                dwacc[c][j] += g * xh;
            }
            o.store_s(dxr + (c * 32 + hl) * V);
        }
#pragma unroll
        for (int c = 0; c < C; ++c) {
            xa[c] = xb[c];
            ga[c] = gb[c];
            ra[c] = rb[c];
        }
        rcur = rnext;
    }
    // both halves of a wave accumulated the same columns: add them, then the 4 waves through LDS
#pragma unroll
    for (int c = 0; c < C; ++c)
#pragma unroll
        for (int j = 0; j < V; ++j) dwacc[c][j] += __shfl_xor(dwacc[c][j], 32, 64);
    if (half == 0) {
#pragma unroll
        for (int c = 0; c < C; ++c)
#pragma unroll
            for (int j = 0; j < V; ++j) lds[wid * N + (c * 32 + hl) * V + j] = dwacc[c][j];
    }
    __syncthreads();
    for (int col = threadIdx.x; col < N; col += 256) {
        float s = lds[col] + lds[N + col] + lds[2 * N + col] + lds[3 * N + col];
        dw_partial[(size_t)blockIdx.x * N + col] = s;
    }
}

// Wide rows (N / V >= 256, e.g. d_model 2048 in bf16): the 4 waves of a block share each row -- thread t owns
// vectors t + 256 c -- and the block processes RPI rows at a time, so every thread keeps only C2 (usually 1)
// vectors per row in registers.  The one-wave-per-row kernel above needs C = 4 chunks per lane there (182
// VGPRs, 2 waves per SIMD, one row's loads in flight per wave: ~1.5 TB/s); this one runs at high occupancy
// with RPI rows of loads in flight per thread.  Per-row dot products: wave sums, then the 4 waves through LDS.
template <typename T, int C2, int RPI>
__global__ void __launch_bounds__(256) rmsnorm_bwd_wide_kernel(const T* __restrict__ dy, const T* __restrict__ x,
                                                               const T* __restrict__ w,
                                                               const float* __restrict__ rstd, T* __restrict__ dx,
                                                               float* __restrict__ dw_partial,
                                                               const T* __restrict__ dres, int M, int N) {
    constexpr int V = Vec<T>::N;
    typedef typename RawV<T>::type R;  // rows stay in registers as raw 16-byte vectors (few VGPRs)
    __shared__ float red[2][RPI][4];
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int nvec = N / V;
    float dwacc[C2][V], wv[C2][V];
#pragma unroll
    for (int c = 0; c < C2; ++c) {
        const int i = tid + 256 * c;
#pragma unroll
        for (int j = 0; j < V; ++j) { dwacc[c][j] = 0.f; wv[c][j] = 0.f; }
        if (i < nvec) {
            Vec<T> g;
            g.load(w + i * V);
#pragma unroll
            for (int j = 0; j < V; ++j) wv[c][j] = g.v[j];
        }
    }
    int par = 0;
    for (int r0 = blockIdx.x * RPI; r0 < M; r0 += gridDim.x * RPI, par ^= 1) {
        R xr[RPI][C2], gr[RPI][C2];
        float dot[RPI], rr[RPI];
#pragma unroll
        for (int k = 0; k < RPI; ++k) {
            const int row = r0 + k;
            const bool ok = row < M;
            rr[k] = ok ? rstd[row] : 0.f;
#pragma unroll
            for (int c = 0; c < C2; ++c) {
                const int i = tid + 256 * c;
                if (ok && i < nvec) {
                    xr[k][c] = *reinterpret_cast<const R*>(x + (size_t)row * N + i * V);
                    gr[k][c] = *reinterpret_cast<const R*>(dy + (size_t)row * N + i * V);
                } else {
                    xr[k][c] = R{};
                    gr[k][c] = R{};
                }
            }
        }
#pragma unroll
        for (int k = 0; k < RPI; ++k) {
            dot[k] = 0.f;
#pragma unroll
            for (int c = 0; c < C2; ++c)
#pragma unroll
                for (int j = 0; j < V; ++j)
                    dot[k] += RawV<T>::get(gr[k][c], j) * wv[c][j] * (RawV<T>::get(xr[k][c], j) * rr[k]);
            dot[k] = wave_sum(dot[k]);
            if (lane == 0) red[par][k][wid] = dot[k];
        }
        __syncthreads();  // double-buffered red[]: one barrier per row group
#pragma unroll
        for (int k = 0; k < RPI; ++k) {
            const int row = r0 + k;
            const float dk = (red[par][k][0] + red[par][k][1] + red[par][k][2] + red[par][k][3]) / (float)N;
            if (row >= M) continue;
#pragma unroll
            for (int c = 0; c < C2; ++c) {
                const int i = tid + 256 * c;
                if (i < nvec) {
                    Vec<T> o;
#pragma unroll
                    for (int j = 0; j < V; ++j) {
                        const float xh = RawV<T>::get(xr[k][c], j) * rr[k], g = RawV<T>::get(gr[k][c], j);
                        o.v[j] = rr[k] * (g * wv[c][j] - xh * dk);
                        dwacc[c][j] += g * xh;
                    }
                    if (dres) {
                        Vec<T> q;
                        q.load(dres + (size_t)row * N + i * V);
#pragma unroll
                        for (int j = 0; j < V; ++j) o.v[j] += q.v[j];
                    }
                    o.store(dx + (size_t)row * N + i * V);
                }
            }
        }
    }
#pragma unroll
    for (int c = 0; c < C2; ++c) {
        const int i = tid + 256 * c;
        if (i < nvec) {
#pragma unroll
            for (int j = 0; j < V; ++j) dw_partial[(size_t)blockIdx.x * N + i * V + j] = dwacc[c][j];
        }
    }
}

// Column sum of the per-block partials [rows, N] -> dw [N]: 16 waves per block,
// lane = column (coalesced 256-B rows), waves split the rows, fixed-order LDS
// combine (deterministic).  ACC: out += the sum (the parameter's flat gradient slot; bf16 or fp32), instead of a
// fresh dw and a separate add kernel.
template <typename T, bool ACC = false>
__global__ void __launch_bounds__(1024) colsum_kernel(const float* __restrict__ partial, T* __restrict__ out,
                                                      int rows, int N) {
    __shared__ float red[16][64];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int col = blockIdx.x * 64 + lane;
    float s = 0.f;
    if (col < N) {
#pragma unroll 8
        for (int r = w; r < rows; r += 16) s += partial[(size_t)r * N + col];
    }
    red[w][lane] = s;
    __syncthreads();
    if (w == 0 && col < N) {
        float t = 0.f;
#pragma unroll
        for (int i = 0; i < 16; ++i) t += red[i][lane];
        if constexpr (ACC) t += ld1<T>(out + col);
        st1<T>(out + col, t);
    }
}

}  // namespace bpe

using namespace bpe;

void launch_rmsnorm_fwd(int dtype, const void* x, const void* w, void* y, float* rstd, int M, int N, float eps,
                        hipStream_t s) {
    dim3 grid((M + 3) / 4), block(256);
    if (dtype == DT_BF16)
        rmsnorm_fwd_kernel<__bf16><<<grid, block, 0, s>>>((const __bf16*)x, (const __bf16*)w, (__bf16*)y, rstd,
                                                          M, N, eps);
    else
        rmsnorm_fwd_kernel<float><<<grid, block, 0, s>>>((const float*)x, (const float*)w, (float*)y, rstd, M, N,
                                                         eps);
}

// 1: the half-wave-row backward where the row width allows (a variant build with 0 keeps the one-wave-per-row kernel)
#ifndef BPE_RMS_BWD_HW
#define BPE_RMS_BWD_HW 1
#endif

// returns the grid it launched (the partial rows colsum_kernel then sums; at most the grid it was given)
template <typename T>
static int rms_bwd_dispatch(const T* dy, const T* x, const T* w, const float* rstd, T* dx, float* partial,
                            const T* dres, int grid, int M, int N, hipStream_t s) {
    constexpr int V = Vec<T>::N;
    if (N / V >= 256 && (N / V) % 256 == 0 && N / V <= 1024) {
        switch (N / V / 256) {
            case 1: rmsnorm_bwd_wide_kernel<T, 1, 2><<<grid, 256, 0, s>>>(dy, x, w, rstd, dx, partial, dres, M, N); break;
            case 2: rmsnorm_bwd_wide_kernel<T, 2, 1><<<grid, 256, 0, s>>>(dy, x, w, rstd, dx, partial, dres, M, N); break;
            case 3: rmsnorm_bwd_wide_kernel<T, 3, 1><<<grid, 256, 0, s>>>(dy, x, w, rstd, dx, partial, dres, M, N); break;
            default: rmsnorm_bwd_wide_kernel<T, 4, 1><<<grid, 256, 0, s>>>(dy, x, w, rstd, dx, partial, dres, M, N); break;
        }
        return grid;
    }
    const size_t lds = (size_t)4 * N * sizeof(float);
    if (BPE_RMS_BWD_HW && M % 2 == 0 && (N / V) % 32 == 0 && N / V >= 64 && N / V <= 128) {
        grid = grid < 512 ? grid : 512;  // one resident round: 2 workgroups per CU at 184 VGPRs (C = 3)
        switch (N / V / 32) {
            case 2: rmsnorm_bwd_hw_kernel<T, 2><<<grid, 256, lds, s>>>(dy, x, w, rstd, dx, partial, dres, M, N); break;
            case 3: rmsnorm_bwd_hw_kernel<T, 3><<<grid, 256, lds, s>>>(dy, x, w, rstd, dx, partial, dres, M, N); break;
            default: rmsnorm_bwd_hw_kernel<T, 4><<<grid, 256, lds, s>>>(dy, x, w, rstd, dx, partial, dres, M, N); break;
        }
        return grid;
    }
    const int chunks = (N / V + 63) / 64;
#define RMS_CASE(CC)                                                                                    \
    if (chunks <= CC) {                                                                                 \
        rmsnorm_bwd_kernel<T, CC><<<grid, 256, lds, s>>>(dy, x, w, rstd, dx, partial, dres, M, N);      \
        return grid;                                                                                    \
    }
    RMS_CASE(1) RMS_CASE(2) RMS_CASE(4) RMS_CASE(8)
#undef RMS_CASE
    return grid;
}

void launch_add_rmsnorm_fwd(int dtype, const void* x, const void* d, const void* w, void* sum, void* y, float* rstd,
                            int M, int N, float eps, hipStream_t s) {
    const int grid = (M + 3) / 4;
#define ADD_RMS(TT, CC)                                                                                        \
    add_rmsnorm_fwd_kernel<TT, CC><<<grid, 256, 0, s>>>((const TT*)x, (const TT*)d, (const TT*)w, (TT*)sum,   \
                                                        (TT*)y, rstd, M, N, eps)
    if (dtype == DT_BF16) {
        const int chunks = (N / 8 + 63) / 64;
        if (chunks <= 1) ADD_RMS(__bf16, 1);
        else if (chunks <= 2) ADD_RMS(__bf16, 2);
        else if (chunks <= 4) ADD_RMS(__bf16, 4);
        else ADD_RMS(__bf16, 0);
    } else {
        ADD_RMS(float, 0);
    }
#undef ADD_RMS
}

// one resident round: the narrow kernel holds 3 workgroups per CU (156 VGPRs at C = 2), 256 CUs
#ifndef BPE_RMS_BWD_GRID
#define BPE_RMS_BWD_GRID 768
#endif
int rmsnorm_bwd_grid(int M) {
    int g = (M + 3) / 4;
    return g < BPE_RMS_BWD_GRID ? g : BPE_RMS_BWD_GRID;
}

// dw_mode: 0 = write dw (the activation dtype), 1 / 2 = accumulate into a bf16 / fp32 gradient slot at dw
void launch_rmsnorm_bwd(int dtype, const void* dy, const void* x, const void* w, const float* rstd, void* dx,
                        float* partial, void* dw, const void* dres, int M, int N, hipStream_t s, int dw_mode) {
    const int grid = rmsnorm_bwd_grid(M);  // the partial buffer's rows (the kernel may use fewer)
    int g;
    if (dtype == DT_BF16)
        g = rms_bwd_dispatch<__bf16>((const __bf16*)dy, (const __bf16*)x, (const __bf16*)w, rstd, (__bf16*)dx,
                                     partial, (const __bf16*)dres, grid, M, N, s);
    else
        g = rms_bwd_dispatch<float>((const float*)dy, (const float*)x, (const float*)w, rstd, (float*)dx, partial,
                                    (const float*)dres, grid, M, N, s);
    const int cb = (N + 63) / 64;
    if (dw_mode == 1)
        colsum_kernel<__bf16, true><<<cb, 1024, 0, s>>>(partial, (__bf16*)dw, g, N);
    else if (dw_mode == 2)
        colsum_kernel<float, true><<<cb, 1024, 0, s>>>(partial, (float*)dw, g, N);
    else if (dtype == DT_BF16)
        colsum_kernel<__bf16><<<cb, 1024, 0, s>>>(partial, (__bf16*)dw, g, N);
    else
        colsum_kernel<float><<<cb, 1024, 0, s>>>(partial, (float*)dw, g, N);
}
