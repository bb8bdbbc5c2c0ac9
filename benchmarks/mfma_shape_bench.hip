// MFMA geometry microbenchmark for gfx950: v_mfma_f32_16x16x32_bf16 against v_mfma_f32_32x32x16_bf16 on random
// operands re-read from LDS, the ping-pong GEMM's regime (review round 5, item 4: "build the 32x32x16 geometry").
//
// Each wave owns a 64 x 64 output block (16 f32x4 accumulators of 16x16 or 4 f32x16 of 32x32: 64 accumulator
// registers either way) and per k-step of 32 reads its A (64 rows) and B (64 columns) fragments from a 32 KiB LDS
// image with ds_read_b128, then issues the MFMAs of the block: 16 x 16x16x32 or 8 x 32x32x16 (the same 262 144
// FLOP).  8 waves per workgroup (2 per SIMD), one workgroup per CU, 256 workgroups, random bf16 operands (the chip's
// clock under load depends on the data: MI355X_MICROARCH "DVFS give-back").  Reports TF/s and the in-kernel clock
// (s_memtime / s_memrealtime x 100 MHz, median over workgroups) for each shape, interleaved.
//
//   hipcc --offload-arch=gfx950 -O3 -o benchmarks/.bin/mfma_shape_bench benchmarks/mfma_shape_bench.hip
//   benchmarks/.bin/mfma_shape_bench [iters]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

#define CHECK(x)                                                                            \
    do {                                                                                    \
        hipError_t e_ = (x);                                                                \
        if (e_ != hipSuccess) {                                                             \
            fprintf(stderr, "%s failed: %s\n", #x, hipGetErrorString(e_));                  \
            exit(1);                                                                        \
        }                                                                                   \
    } while (0)

constexpr int NT = 512;

__device__ __forceinline__ bf16x8 lds_frag(const char* smem, int off) {
    return *reinterpret_cast<const bf16x8*>(smem + off);
}

// SHAPE 16: 4 x 4 blocks of 16x16 per wave, one 16x16x32 MFMA each per k-step; SHAPE 32: 2 x 2 blocks of 32x32,
// two 32x32x16 MFMAs each per k-step (k = 32)
template <int SHAPE>
__global__ void __launch_bounds__(NT, 1) mfma_loop(const __bf16* __restrict__ src, float* __restrict__ out,
                                                   long long* __restrict__ clk, int iters) {
    __shared__ __attribute__((aligned(16))) char smem[32768];
    const int tid = threadIdx.x, l = tid & 63, w = tid >> 6;
    // fill the LDS image with this workgroup's slice of the random operands
    for (int i = tid; i < 32768 / 16; i += NT)
        reinterpret_cast<bf16x8*>(smem)[i] = reinterpret_cast<const bf16x8*>(src)[(blockIdx.x * 2048 + i) % (1 << 20)];
    __syncthreads();
    const long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
    // per-lane fragment offsets: 16-byte chunks spread over the image so that the reads are conflict-free
    const int base = ((w * 64 + l) * 16) % 16384;
    float sink = 0.f;
    if constexpr (SHAPE == 16) {
        f32x4 acc[4][4];
        for (int i = 0; i < 4; ++i)
            for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
        for (int it = 0; it < iters; ++it) {
            bf16x8 a[4], b[4];
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int o = (base + 1024 * i + ((it & 3) << 12)) & 16383;  // varies per k-step: reads stay in the loop
                a[i] = lds_frag(smem, o);
                b[i] = lds_frag(smem, 16384 + o);
            }
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i], b[j], acc[i][j], 0, 0, 0);
        }
        for (int i = 0; i < 4; ++i)
            for (int j = 0; j < 4; ++j) sink += acc[i][j][0] + acc[i][j][3];
    } else {
        f32x16 acc[2][2];
        for (int i = 0; i < 2; ++i)
            for (int j = 0; j < 2; ++j)
                for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
        for (int it = 0; it < iters; ++it) {
            bf16x8 a[2][2], b[2][2];  // [block][k half]: 32 rows x 16 k per fragment, two per k-step of 32
#pragma unroll
            for (int i = 0; i < 2; ++i)
#pragma unroll
                for (int h = 0; h < 2; ++h) {
                    const int o = (base + 1024 * (2 * i + h) + ((it & 3) << 12)) & 16383;
                    a[i][h] = lds_frag(smem, o);
                    b[i][h] = lds_frag(smem, 16384 + o);
                }
#pragma unroll
            for (int h = 0; h < 2; ++h)
#pragma unroll
                for (int i = 0; i < 2; ++i)
#pragma unroll
                    for (int j = 0; j < 2; ++j)
                        acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[i][h], b[j][h], acc[i][j], 0, 0, 0);
        }
        for (int i = 0; i < 2; ++i)
            for (int j = 0; j < 2; ++j) sink += acc[i][j][0] + acc[i][j][15];
    }
    const long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
    out[blockIdx.x * NT + tid] = sink;
    if (tid == 0) {
        clk[2 * blockIdx.x] = t1 - t0;
        clk[2 * blockIdx.x + 1] = r1 - r0;
    }
}

int main(int argc, char** argv) {
    const int iters = argc > 1 ? atoi(argv[1]) : 20000;
    const int nwg = 256;
    std::vector<unsigned short> h(1 << 23);
    unsigned s = 12345;
    for (auto& x : h) {  // random bf16 in about [-1, 1): sign, exponent 120..127, random mantissa
        s = s * 1664525u + 1013904223u;
        x = (unsigned short)(((s >> 31) << 15) | ((120 + ((s >> 20) & 7)) << 7) | ((s >> 8) & 127));
    }
    __bf16* src;
    float* out;
    long long* clk;
    CHECK(hipMalloc(&src, h.size() * 2));
    CHECK(hipMalloc(&out, nwg * NT * sizeof(float)));
    CHECK(hipMalloc(&clk, nwg * 2 * sizeof(long long)));
    CHECK(hipMemcpy(src, h.data(), h.size() * 2, hipMemcpyHostToDevice));
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    const double flop = 2.0 * 64 * 64 * 32 * 8 * (double)iters * nwg;  // per wave 64 x 64 x 32 per k-step, 8 waves
    for (int round = 0; round < 3; ++round) {
        for (int shape : {16, 32}) {
            auto launch = [&]() {
                if (shape == 16) mfma_loop<16><<<nwg, NT>>>(src, out, clk, iters);
                else mfma_loop<32><<<nwg, NT>>>(src, out, clk, iters);
            };
            launch();  // warm (and clock ramp)
            CHECK(hipDeviceSynchronize());
            CHECK(hipEventRecord(e0));
            for (int r = 0; r < 5; ++r) launch();
            CHECK(hipEventRecord(e1));
            CHECK(hipEventSynchronize(e1));
            float ms = 0.f;
            CHECK(hipEventElapsedTime(&ms, e0, e1));
            std::vector<long long> c(nwg * 2);
            CHECK(hipMemcpy(c.data(), clk, c.size() * sizeof(long long), hipMemcpyDeviceToHost));
            std::vector<double> mhz(nwg);
            for (int i = 0; i < nwg; ++i) mhz[i] = (double)c[2 * i] / (double)c[2 * i + 1] * 100.0;
            std::nth_element(mhz.begin(), mhz.begin() + nwg / 2, mhz.end());
            const double cyc_per_kstep = (double)c[0] / iters;
            printf("{\"round\": %d, \"mfma\": \"%s\", \"ms\": %.3f, \"tflops\": %.1f, \"clock_mhz\": %.0f, "
                   "\"cycles_per_kstep\": %.1f, \"mfma_floor_cycles\": 512}\n",
                   round, shape == 16 ? "16x16x32" : "32x32x16", ms / 5, flop / (ms / 5 * 1e-3) / 1e12, mhz[nwg / 2],
                   cyc_per_kstep);
            fflush(stdout);
        }
    }
    return 0;
}
