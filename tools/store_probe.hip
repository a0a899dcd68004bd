// Store-pattern probe (dev tool, GPU): write a [M x N] bf16 matrix tile by tile (128 x 128 tiles, 256
// threads) in (a) the GEMM epilogue's accumulator order — a wave instruction covers 16 rows x four
// 16-B pieces 32 B apart — and (b) whole rows — a wave instruction covers 4 rows x 256 contiguous B.
//   hipcc --offload-arch=gfx950 -O3 tools/store_probe.hip -o tools/store_probe && tools/store_probe
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

__global__ void __launch_bounds__(256) st_epi(uint4* c, int n_cols, int tiles_n) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, wm = wave >> 1, wn = wave & 1;
  const int tm = blockIdx.x / tiles_n, tn = blockIdx.x % tiles_n;
  const int g = lane >> 4, rho = lane & 15;
  const uint4 v = make_uint4(blockIdx.x, threadIdx.x, 1u, 2u);
  for (int i = 0; i < 4; ++i)
    for (int h = 0; h < 2; ++h) {
      const long long row = (long long)tm * 128 + wm * 64 + i * 16 + rho;
      const int col = tn * 128 + wn * 64 + 16 * g + 8 * h;   // bf16 elements
      c[(row * n_cols + col) / 8] = v;
    }
}

__global__ void __launch_bounds__(256) st_rows(uint4* c, int n_cols, int tiles_n) {
  const int tm = blockIdx.x / tiles_n, tn = blockIdx.x % tiles_n;
  const uint4 v = make_uint4(blockIdx.x, threadIdx.x, 1u, 2u);
  for (int q = threadIdx.x; q < 128 * 16; q += 256) {   // 16 chunks of 16 B per 128-col row
    const long long row = (long long)tm * 128 + q / 16;
    const int col = tn * 128 + (q % 16) * 8;
    c[(row * n_cols + col) / 8] = v;
  }
}

// the same store orders with the GEMM's residency: 64 KB of LDS per workgroup (two per CU, 8 waves)
template <int MODE>
__global__ void __launch_bounds__(256) st_lds64(uint4* c, int n_cols, int tiles_n) {
  __shared__ uint4 pad[4096];   // 64 KB: occupancy only
  if (threadIdx.x == 1023) pad[threadIdx.x] = make_uint4(0, 0, 0, 0);   // never true: keeps the array
  if (MODE == 0) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, wm = wave >> 1, wn = wave & 1;
    const int tm = blockIdx.x / tiles_n, tn = blockIdx.x % tiles_n;
    const int g = lane >> 4, rho = lane & 15;
    const uint4 v = make_uint4(blockIdx.x, threadIdx.x, 1u, 2u);
    for (int i = 0; i < 4; ++i)
      for (int h = 0; h < 2; ++h) {
        const long long row = (long long)tm * 128 + wm * 64 + i * 16 + rho;
        const int col = tn * 128 + wn * 64 + 16 * g + 8 * h;
        c[(row * n_cols + col) / 8] = v;
      }
  } else {
    const int tm = blockIdx.x / tiles_n, tn = blockIdx.x % tiles_n;
    const uint4 v = make_uint4(blockIdx.x, threadIdx.x, 1u, 2u);
    for (int q = threadIdx.x; q < 128 * 16; q += 256) {
      const long long row = (long long)tm * 128 + q / 16;
      const int col = tn * 128 + (q % 16) * 8;
      c[(row * n_cols + col) / 8] = v;
    }
  }
}

int main() {
  const int M = 282240, N = 512;
  uint4* c;
  hipMalloc(&c, (size_t)M * N * 2);
  const int tiles_n = N / 128, tiles = (M / 128) * tiles_n;
  hipEvent_t e0, e1;
  hipEventCreate(&e0); hipEventCreate(&e1);
  const char* names[4] = {"epilogue order (16 rows x 4x16B)", "whole rows (4 rows x 256B)",
                          "epilogue order, 2 WG/CU (64 KB LDS)", "whole rows, 2 WG/CU (64 KB LDS)"};
  auto run = [&](int k) {
    if (k == 0) st_epi<<<tiles, 256>>>(c, N, tiles_n);
    else if (k == 1) st_rows<<<tiles, 256>>>(c, N, tiles_n);
    else if (k == 2) st_lds64<0><<<tiles, 256>>>(c, N, tiles_n);
    else st_lds64<1><<<tiles, 256>>>(c, N, tiles_n);
  };
  for (int k = 0; k < 4; ++k) {
    for (int w = 0; w < 3; ++w) run(k);
    hipEventRecord(e0);
    for (int it = 0; it < 20; ++it) run(k);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    const double us = ms * 1e3 / 20, bytes = (double)M * N * 2;
    printf("%-38s %8.1f us  %7.0f GB/s\n", names[k], us, bytes / us / 1e3);
  }
  hipFree(c);
  return 0;
}
