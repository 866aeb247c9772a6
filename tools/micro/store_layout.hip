// Microbenchmark: does the per-CU epilogue store throughput depend on how many
// cache lines one wave-instruction touches? Each block writes T tiles of 256x256
// bf16 (row stride ld) with 16-B stores per lane in one of two lane layouts:
//   A: 16 rows x 64 B per instruction (the v4 GEMM epilogue after permlane16)
//   B:  8 rows x 128 B per instruction (full 128-B lines)
// Also the matching loads (aux read). hipcc -O3 --offload-arch=gfx950 -o store_layout store_layout.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#include <cstdlib>
typedef unsigned int v4u __attribute__((ext_vector_type(4)));

template <int LAYOUT, bool LOAD>
__global__ void __launch_bounds__(512) k(unsigned short* C, int M, int N, int tiles_per_block, int ld, v4u* sink) {
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 2, wn = wave & 3;
  const int gn = N / 256, gm = M / 256;
  v4u acc = {0, 0, 0, 0};
  for (int t = 0; t < tiles_per_block; ++t) {
    const int tile = (blockIdx.x * tiles_per_block + t) % (gm * gn);
    const int m0 = (tile / gn) * 256 + 128 * wm, n0 = (tile % gn) * 256 + 64 * wn;
    // the wave's block: 128 rows x 64 cols = 8 row-blocks of 16 x 64
#pragma unroll
    for (int rb = 0; rb < 8; ++rb) {
      if (LAYOUT == 0) {
#pragma unroll
        for (int q = 0; q < 2; ++q) {
          const int row = m0 + 16 * rb + (lane & 15);
          const int g = lane >> 4;
          const int col = n0 + 32 * q + 16 * (g & 1) + 8 * (g >> 1);
          v4u* p = (v4u*)(C + (size_t)row * ld + col);
          if (LOAD) acc += *p; else *p = v4u{(unsigned)row, (unsigned)col, 1u, 2u};
        }
      } else {
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const int row = m0 + 16 * rb + 8 * h + (lane >> 3);
          const int col = n0 + 8 * (lane & 7);
          v4u* p = (v4u*)(C + (size_t)row * ld + col);
          if (LOAD) acc += *p; else *p = v4u{(unsigned)row, (unsigned)col, 1u, 2u};
        }
      }
    }
  }
  if (LOAD && acc[0] == 12345u) sink[0] = acc;
}

int main(int argc, char** argv) {
  const int M = 50432, N = 2048, ld = N;
  unsigned short* C;
  v4u* sink;
  hipMalloc(&C, (size_t)M * ld * 2);
  hipMalloc(&sink, 64);
  hipMemset(C, 0, (size_t)M * ld * 2);
  const int tiles = (M / 256) * (N / 256);
  const int G = argc > 1 ? atoi(argv[1]) : 256, tpb = (tiles + 255) / 256;
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  auto run = [&](auto kern, const char* name) {
    for (int i = 0; i < 3; ++i) hipLaunchKernelGGL(kern, dim3(G), dim3(512), 0, 0, C, M, N, tpb, ld, sink);
    hipEventRecord(e0);
    const int reps = 20;
    for (int i = 0; i < reps; ++i) hipLaunchKernelGGL(kern, dim3(G), dim3(512), 0, 0, C, M, N, tpb, ld, sink);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    const double us = ms * 1000.0 / reps;
    const double bytes = (double)G * tpb * 256 * 256 * 2;
    printf("%-28s %8.1f us  %7.2f TB/s  %6.1f B/cyc/CU @2.1GHz\n", name, us, bytes / us / 1e6,
           bytes / (us * 1e-6) / 256 / 2.1e9);
  };
  run(k<0, false>, "store 16 rows x 64 B");
  run(k<1, false>, "store  8 rows x 128 B");
  run(k<0, true>, "load  16 rows x 64 B");
  run(k<1, true>, "load   8 rows x 128 B");
  return 0;
}
