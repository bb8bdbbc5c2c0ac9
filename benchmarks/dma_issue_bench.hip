// What an LDS-DMA piece costs the wave that issues it between its own MFMAs (gfx950).
//
// The 4-wave GEMM experiment of round 5 (docs/performance.md, "one wave per SIMD") measured its main loop 1.4-2x
// faster without the in-loop LDS-DMA, and no faster when the DMA was issued but never waited for: the cost is in
// issuing the pieces, not in waiting for them.  This microbenchmark isolates it: one workgroup of 4 waves per CU
// (one wave per SIMD), a loop of 64 independent mfma_f32_16x16x32_bf16 per iteration with P loads interleaved
// (one per 64 / P MFMAs), timed per variant:
//   0  no loads
//   1  buffer_load_dwordx4 ... lds, M0 rewritten per piece (distinct 1 KiB LDS destinations)
//   2  the same, every piece to one LDS destination (M0 written once)
//   3  global_load_dwordx4 into VGPRs (consumed once per iteration: no LDS)
//   4  global_load_lds_dwordx4 (64-bit VGPR addresses), M0 rewritten per piece
// Sources: a 1 MiB buffer re-read (L2-resident) or a 1 GiB one streamed (HBM).
//
//   hipcc --offload-arch=gfx950 -O3 -o /tmp/dma_issue_bench benchmarks/dma_issue_bench.hip && /tmp/dma_issue_bench
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) void lds_void;
typedef __attribute__((address_space(1))) void gbl_void;

constexpr int ITERS = 512;

template <int V, int P>
__global__ void __launch_bounds__(256, 1) probe(const char* __restrict__ src, unsigned long long span, float* out) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    // w wave-uniform for the compiler too: a buffer resource built from a VGPR value compiles to a waterfall loop
    const int tid = threadIdx.x, l = tid & 63, w = __builtin_amdgcn_readfirstlane(tid >> 6);
    f32x4 acc[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) acc[i] = f32x4{0.f, 0.f, 0.f, 0.f};
    bf16x8 a, b;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        a[j] = (__bf16)(0.001f * (l + j));
        b[j] = (__bf16)(0.002f * (l - j));
    }
    const unsigned long long base = ((unsigned long long)blockIdx.x * 4 + w) * 65536ull;
    u32x4 sink = {0, 0, 0, 0};
#if defined(__HIP_DEVICE_COMPILE__)
    for (int it = 0; it < ITERS; ++it) {
        const unsigned long long off = (base + (unsigned long long)it * P * 1024ull) % span;
        const char* p = src + off;
        const auto rsrc = __builtin_amdgcn_make_buffer_rsrc((void*)p, 0, 0x7fffffff, 0x00020000);
#pragma unroll
        for (int q = 0; q < 4; ++q) {
#pragma unroll
            for (int i = 0; i < 16; ++i) acc[i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, acc[i], 0, 0, 0);
#pragma unroll
            for (int j = 0; j < P / 4; ++j) {
                const int piece = q * (P / 4) + j;
                if constexpr (V == 1)
                    __builtin_amdgcn_raw_ptr_buffer_load_lds(rsrc, (lds_void*)(smem + (w * 16 + piece) * 1024), 16,
                                                             (unsigned)(piece * 1024 + 16 * l), 0, 0, 0);
                if constexpr (V == 2)
                    __builtin_amdgcn_raw_ptr_buffer_load_lds(rsrc, (lds_void*)(smem + w * 1024), 16,
                                                             (unsigned)(piece * 1024 + 16 * l), 0, 0, 0);
                if constexpr (V == 3)
                    sink ^= *reinterpret_cast<const u32x4*>(p + piece * 1024 + 16 * l);
                if constexpr (V == 4)
                    __builtin_amdgcn_global_load_lds((gbl_void*)(p + piece * 1024 + 16 * l),
                                                     (lds_void*)(smem + (w * 16 + piece) * 1024), 16, 0, 0);
            }
        }
        __builtin_amdgcn_sched_barrier(0);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#endif
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < 16; ++i) s += acc[i][0] + acc[i][1] + acc[i][2] + acc[i][3];
    s += (float)(sink[0] ^ sink[1] ^ sink[2] ^ sink[3]);
    if (s == 12345.f) out[tid] = s;
}

template <int V, int P>
static float run(const char* src, unsigned long long span, float* out, int reps) {
    auto* k = &probe<V, P>;
    (void)hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, 65536);
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    k<<<256, 256, 65536>>>(src, span, out);
    (void)hipEventRecord(e0);
    for (int r = 0; r < reps; ++r) k<<<256, 256, 65536>>>(src, span, out);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms = 0.f;
    (void)hipEventElapsedTime(&ms, e0, e1);
    return ms / reps;
}

int main() {
    const unsigned long long big = 1ull << 30, small = 1ull << 20;
    char* src = nullptr;
    float* out = nullptr;
    if (hipMalloc(&src, big) != hipSuccess || hipMalloc(&out, 4096) != hipSuccess) return 1;
    (void)hipMemset(src, 1, big);
    const int reps = 20;
    // MFMA time per iteration: 64 x 16 cycles; report microseconds per launch and the implied cycles per load beyond
    // the MFMA-only loop at an assumed 2.0 GHz (the clock under MFMA load is lower: compare variants, not absolutes)
    for (int pass = 0; pass < 2; ++pass) {
        const unsigned long long span = pass ? big : small;
        const char* tag = pass ? "HBM 1 GiB" : "L2 1 MiB";
        const float t0 = run<0, 4>(src, span, out, reps);
        printf("{\"src\": \"%s\", \"variant\": 0, \"loads_per_64_mfma\": 0, \"us\": %.2f}\n", tag, 1000 * t0);
#define ROW(VV, PP)                                                                                                \
    {                                                                                                              \
        const float t = run<VV, PP>(src, span, out, reps);                                                         \
        printf("{\"src\": \"%s\", \"variant\": %d, \"loads_per_64_mfma\": %d, \"us\": %.2f, \"extra_cycles_per_load\": " \
               "%.1f}\n",                                                                                          \
               tag, VV, PP, 1000 * t, (t - t0) * 1e-3 * 2.0e9 / (ITERS * PP));                                     \
    }
        ROW(1, 4) ROW(1, 8) ROW(1, 16) ROW(2, 8) ROW(2, 16) ROW(3, 8) ROW(3, 16) ROW(4, 8) ROW(4, 16)
#undef ROW
    }
    return 0;
}
