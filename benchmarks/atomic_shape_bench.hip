// Float-atomic throughput by access shape per wave-instruction (gfx950), for sizing the attention-backward dQ
// accumulation (flash_attn_bwd.hip adds 64 x 64 fp32 tiles into a [rows][H*D] buffer).
//
//   hipcc -O3 --offload-arch=gfx950 benchmarks/atomic_shape_bench.hip -o build/atomic_shape_bench
//   ./build/atomic_shape_bench
//
// Every workgroup (256 threads) adds one 64-row x 64-float tile (16 KiB) into a buffer with a row stride of
// 768 floats (GPT-2: H*D), tiles spread over 400 MB.  Shapes (lanes of one instruction):
//   s4x64  : 4 rows x 16 floats (64 B segments)  -- a 16x16 MFMA accumulator as it stands
//   s2x128 : 2 rows x 32 floats (128 B segments) -- a 32x32 MFMA accumulator as it stands
//   s1x256 : 1 row  x 64 floats (256 B)
// plus plain 4-byte stores of the 2x128 shape and 16-byte stores (4 rows x 256 B) for comparison.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

constexpr int LD = 768;  // floats per row
constexpr int TILE_ROWS = 64, TILE_COLS = 64;

template <int SHAPE>
__global__ void __launch_bounds__(256) atomics(float* buf, long ntile_rows, int ntile_cols) {
    const int tile = blockIdx.x;
    const long r0 = (long)(tile / ntile_cols) * TILE_ROWS % ntile_rows;
    const int c0 = (tile % ntile_cols) * TILE_COLS;
    const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
    float* base = buf + r0 * LD + c0;
    // each wave covers 16 rows of the tile (4096 floats = 16 instructions of 64 lanes)
#pragma unroll
    for (int k = 0; k < 16; ++k) {
        int row, col;
        if (SHAPE == 0) {  // 4 rows x 16
            row = 16 * w + 4 * (k >> 2) + (l >> 4);
            col = 16 * (k & 3) + (l & 15);
        } else if (SHAPE == 1) {  // 2 rows x 32
            row = 16 * w + 2 * (k >> 1) + (l >> 5);
            col = 32 * (k & 1) + (l & 31);
        } else {  // 1 row x 64
            row = 16 * w + k;
            col = l;
        }
        if (SHAPE < 3)
            atomicAdd(base + (long)row * LD + col, 1.0f);
        else
            base[(long)row * LD + col] = 1.0f;  // plain 4-byte stores, 2 x 128 B shape
    }
}

__global__ void __launch_bounds__(256) stores16(float* buf, long ntile_rows, int ntile_cols) {
    const int tile = blockIdx.x;
    const long r0 = (long)(tile / ntile_cols) * TILE_ROWS % ntile_rows;
    const int c0 = (tile % ntile_cols) * TILE_COLS;
    const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
    float* base = buf + r0 * LD + c0;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const int row = 16 * w + 4 * k + (l >> 4);
        const int col = 4 * (l & 15);
        *reinterpret_cast<float4*>(base + (long)row * LD + col) = float4{1.f, 1.f, 1.f, 1.f};
    }
}

int main() {
    const long rows = 131072;  // 400 MB buffer
    const int ntc = LD / TILE_COLS;
    const long ntiles = rows / TILE_ROWS * ntc * 2;  // each element added twice over the launch
    float* buf;
    if (hipMalloc(&buf, rows * LD * sizeof(float)) != hipSuccess) return 1;
    (void)hipMemset(buf, 0, rows * LD * sizeof(float));
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    const double bytes = (double)ntiles * TILE_ROWS * TILE_COLS * 4;
    const char* names[] = {"atomic 4x64B", "atomic 2x128B", "atomic 1x256B", "store4 2x128B", "store16 4x256B"};
    for (int rep = 0; rep < 3; ++rep) {
        for (int s = 0; s < 5; ++s) {
            auto run = [&] {
                switch (s) {
                    case 0: atomics<0><<<ntiles, 256>>>(buf, rows, ntc); break;
                    case 1: atomics<1><<<ntiles, 256>>>(buf, rows, ntc); break;
                    case 2: atomics<2><<<ntiles, 256>>>(buf, rows, ntc); break;
                    case 3: atomics<3><<<ntiles, 256>>>(buf, rows, ntc); break;
                    default: stores16<<<ntiles, 256>>>(buf, rows, ntc); break;
                }
            };
            run();
            (void)hipEventRecord(a);
            for (int i = 0; i < 5; ++i) run();
            (void)hipEventRecord(b);
            (void)hipEventSynchronize(b);
            float ms = 0;
            (void)hipEventElapsedTime(&ms, a, b);
            ms /= 5;
            printf("%-16s %8.3f ms  %6.2f TB/s\n", names[s], ms, bytes / ms / 1e9);
        }
    }
    (void)hipFree(buf);
    return 0;
}
