// Shared device helpers for the gfx950 (CDNA4, MI355X) kernels.
//
// Conventions used by every kernel in this directory:
//   * wave64: lane = threadIdx.x & 63, reductions span 64 lanes.
//   * bf16 values move as raw 16-bit words (u16) in 16-byte vectors
//     (8 x bf16 per lane per load) -- hipcc does not auto-vectorise bf16.
//   * all statistics / accumulations are fp32.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define BPE_WAVE 64

typedef unsigned short u16;
typedef u16 u16x8 __attribute__((ext_vector_type(8)));
typedef u16 u16x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

namespace bpe {

__device__ __forceinline__ float bf2f(u16 h) { return __uint_as_float(((unsigned)h) << 16); }
// Round-to-nearest-even; hipcc lowers the __bf16 cast to v_cvt_pk_bf16_f32 on gfx950
// (keeps NaN a NaN, unlike the integer-rounding trick).
__device__ __forceinline__ u16 f2bf(float f) { return __builtin_bit_cast(u16, (__bf16)f); }

// sigmoid(x) = 1 / (1 + 2^(-x log2 e)) with the hardware v_exp_f32 / v_rcp_f32 (1 ulp): a plain `1.f / (...)`
// compiles to the IEEE division sequence (v_div_scale x2, v_rcp, 4 fma, v_div_fmas, v_div_fixup) -- ~10 VALU
// per element in the SwiGLU kernels, whose outputs are rounded to bf16 anyway.  Saturates to 0 / 1 (exp2 -> inf
// gives rcp(inf) = 0), NaN stays NaN.
__device__ __forceinline__ float fast_sigmoid(float x) {
    return __builtin_amdgcn_rcpf(1.f + __builtin_amdgcn_exp2f(x * -1.4426950408889634f));
}

// Two elements at once: the arithmetic on the packed fp32 VALU (v_pk_mul_f32 / v_pk_add_f32 / v_pk_fma_f32, two
// lanes' worth per instruction), the transcendentals per element -- the same operations and rounding as
// fast_sigmoid, for epilogues that run no MFMAs beside them (explicit vectors: files built without the SLP
// vectorizer still get the packed forms).
typedef float f32x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ f32x2 fast_sigmoid2(f32x2 x) {
    const f32x2 t = x * -1.4426950408889634f;
    const f32x2 e = 1.f + f32x2{__builtin_amdgcn_exp2f(t.x), __builtin_amdgcn_exp2f(t.y)};
    return f32x2{__builtin_amdgcn_rcpf(e.x), __builtin_amdgcn_rcpf(e.y)};
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
    return v;
}

// ---- streaming (non-temporal) vector access ---------------------------------
// Activations that a memory-bound kernel reads or writes exactly once (hundreds of MB per tensor, never cached
// usefully) go through these: the nt hint keeps them from displacing reusable lines.  Measured on the
// softmax-CE kernel: 5.1 -> 5.5 TB/s (docs/performance.md).  -DBPE_STREAM_NT=0 builds the plain form (A/B).
#ifndef BPE_STREAM_NT
#define BPE_STREAM_NT 1
#endif
template <typename V> __device__ __forceinline__ V ld_stream(const V* p) {
#if BPE_STREAM_NT
    return __builtin_nontemporal_load(p);
#else
    return *p;
#endif
}
template <typename V> __device__ __forceinline__ void st_stream(V* p, V v) {
#if BPE_STREAM_NT
    __builtin_nontemporal_store(v, p);
#else
    *p = v;
#endif
}

// ---- typed 16-byte vector load/store, converting to/from fp32 -------------
// T = float (4 elems / 16 B) or __bf16 (8 elems / 16 B).
template <typename T> struct Vec;
template <> struct Vec<float> {
    static constexpr int N = 4;
    float v[4];
    __device__ __forceinline__ void load(const float* p) {
        f32x4 t = *reinterpret_cast<const f32x4*>(p);
        v[0] = t[0]; v[1] = t[1]; v[2] = t[2]; v[3] = t[3];
    }
    __device__ __forceinline__ void load_s(const float* p) {  // streaming (see ld_stream)
        f32x4 t = ld_stream(reinterpret_cast<const f32x4*>(p));
        v[0] = t[0]; v[1] = t[1]; v[2] = t[2]; v[3] = t[3];
    }
    __device__ __forceinline__ void store_s(float* p) const { st_stream(reinterpret_cast<f32x4*>(p), f32x4{v[0], v[1], v[2], v[3]}); }
    __device__ __forceinline__ void store(float* p) const {
        f32x4 t = {v[0], v[1], v[2], v[3]};
        *reinterpret_cast<f32x4*>(p) = t;
    }
};
template <> struct Vec<__bf16> {
    static constexpr int N = 8;
    float v[8];
    __device__ __forceinline__ void load(const __bf16* p) {
        u16x8 t = *reinterpret_cast<const u16x8*>(p);
#pragma unroll
        for (int i = 0; i < 8; ++i) v[i] = bf2f(t[i]);
    }
    __device__ __forceinline__ void store(__bf16* p) const {
        u16x8 t;
#pragma unroll
        for (int i = 0; i < 8; ++i) t[i] = f2bf(v[i]);
        *reinterpret_cast<u16x8*>(p) = t;
    }
    __device__ __forceinline__ void load_s(const __bf16* p) {  // streaming (see ld_stream)
        u16x8 t = ld_stream(reinterpret_cast<const u16x8*>(p));
#pragma unroll
        for (int i = 0; i < 8; ++i) v[i] = bf2f(t[i]);
    }
    __device__ __forceinline__ void store_s(__bf16* p) const {
        u16x8 t;
#pragma unroll
        for (int i = 0; i < 8; ++i) t[i] = f2bf(v[i]);
        st_stream(reinterpret_cast<u16x8*>(p), t);
    }
};

template <typename T> __device__ __forceinline__ float ld1(const T* p);
template <> __device__ __forceinline__ float ld1<float>(const float* p) { return *p; }
template <> __device__ __forceinline__ float ld1<__bf16>(const __bf16* p) {
    return bf2f(*reinterpret_cast<const u16*>(p));
}
template <typename T> __device__ __forceinline__ void st1(T* p, float v);
template <> __device__ __forceinline__ void st1<float>(float* p, float v) { *p = v; }
template <> __device__ __forceinline__ void st1<__bf16>(__bf16* p, float v) {
    *reinterpret_cast<u16*>(p) = f2bf(v);
}

// Block-wide sum for blockDim.x <= 1024 (multiple of 64). `red` needs 16 floats.
__device__ __forceinline__ float block_sum(float v, float* red) {
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = blockDim.x >> 6;
    v = wave_sum(v);
    __syncthreads();
    if (lane == 0) red[wid] = v;
    __syncthreads();
    float r = 0.f;
    for (int i = 0; i < nw; ++i) r += red[i];
    return r;
}
__device__ __forceinline__ float block_max(float v, float* red) {
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = blockDim.x >> 6;
    v = wave_max(v);
    __syncthreads();
    if (lane == 0) red[wid] = v;
    __syncthreads();
    float r = -INFINITY;
    for (int i = 0; i < nw; ++i) r = fmaxf(r, red[i]);
    return r;
}

// Grid size for memory-bound grid-stride kernels: enough blocks to fill 256 CUs
// several times over, capped so per-launch overhead stays low (guide G11).
__host__ __forceinline__ int stream_grid(size_t work_items, int block, int cap = 2048) {
    size_t g = (work_items + block - 1) / block;
    if (g < 1) g = 1;
    if (g > (size_t)cap) g = cap;
    return (int)g;
}

constexpr float FP8_E4M3_MAX = 448.f;     // OCP e4m3fn: activations / weights
constexpr float FP8_E5M2_MAX = 57344.f;   // OCP e5m2: gradients (wider range, 2 mantissa bits)

// FMT 0 = e4m3fn (v_cvt_pk_fp8_f32), 1 = e5m2 (v_cvt_pk_bf8_f32); saturating: clamp before the convert
template <int FMT>
__device__ __forceinline__ unsigned pack4_fp8(float a, float b, float c, float d) {
    constexpr float M = FMT == 0 ? FP8_E4M3_MAX : FP8_E5M2_MAX;
    a = fminf(fmaxf(a, -M), M);
    b = fminf(fmaxf(b, -M), M);
    c = fminf(fmaxf(c, -M), M);
    d = fminf(fmaxf(d, -M), M);
    int w;
    if constexpr (FMT == 0) {
        w = __builtin_amdgcn_cvt_pk_fp8_f32(a, b, 0, false);  // bytes 0,1
        w = __builtin_amdgcn_cvt_pk_fp8_f32(c, d, w, true);   // bytes 2,3
    } else {
        w = __builtin_amdgcn_cvt_pk_bf8_f32(a, b, 0, false);
        w = __builtin_amdgcn_cvt_pk_bf8_f32(c, d, w, true);
    }
    return (unsigned)w;
}

}  // namespace bpe
