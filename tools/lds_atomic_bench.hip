// LDS atomic throughput probe (dev tool, GPU): the window-attention backward bins dS by relative
// position; this times 16 adds per lane per iteration into a 1024-entry LDS array with the address
// pattern of that binning (32 consecutive bins per half-wave, second half shifted by 4) for
// f32 / u32 / u64 atomics and a plain (racy) store baseline.
//   hipcc --offload-arch=gfx950 -O3 tools/lds_atomic_bench.hip -o /tmp/lds_atomic_bench
#include <hip/hip_runtime.h>
#include <cstdio>

template <int MODE>
__global__ void __launch_bounds__(320, 2) probe(float* out, int iters) {
  __shared__ float binsf[5][1024];
  __shared__ unsigned long long binsl[5][512];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  for (int i = threadIdx.x; i < 5 * 1024; i += 320) (&binsf[0][0])[i] = 0.f;
  for (int i = threadIdx.x; i < 5 * 512; i += 320) (&binsl[0][0])[i] = 0;
  __syncthreads();
  const int base = 400 - (lane & 31) + 4 * (lane >> 5);
  float v = 1.0f + lane * 1e-3f;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int b = base + ((r & 3) + 8 * (r >> 2)) * 3 + (it & 7);
      if (MODE == 0) atomicAdd(&binsf[w][b], v);
      if (MODE == 1) atomicAdd(reinterpret_cast<unsigned*>(&binsf[w][b]), (unsigned)(v * 1024.f));
      if (MODE == 2) atomicAdd(&binsl[w][b & 511], (unsigned long long)(v * 1048576.f));
      if (MODE == 3) binsf[w][b] = v;
    }
    v += 1e-3f;
  }
  __syncthreads();
  if (threadIdx.x == 0) out[blockIdx.x] = binsf[0][400] + (float)binsl[0][400];
}

template <int MODE>
float run(float* d, int blocks, int iters) {
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  probe<MODE><<<blocks, 320>>>(d, iters);
  hipEventRecord(a);
  probe<MODE><<<blocks, 320>>>(d, iters);
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms = 0.f;
  hipEventElapsedTime(&ms, a, b);
  return ms;
}

int main() {
  float* d;
  const int blocks = 1920, iters = 25;   // stage-3 launch: 1920 (window, head) x 5 tiles x 5 steps
  hipMalloc(&d, blocks * sizeof(float));
  const char* names[] = {"ds_add_f32", "ds_add_u32", "ds_add_u64", "ds_write_b32 (no atomic)"};
  float t[4] = {run<0>(d, blocks, iters), run<1>(d, blocks, iters), run<2>(d, blocks, iters), run<3>(d, blocks, iters)};
  for (int m = 0; m < 4; ++m) {
    const double instr = (double)blocks * 5 * iters * 16;   // wave-level LDS instructions
    printf("%-26s %8.1f us  %6.1f cycles per wave instruction per CU (2.4 GHz, 256 CUs)\n", names[m], t[m] * 1e3,
           t[m] * 1e-3 * 2.4e9 * 256 / instr);
  }
  hipFree(d);
  return 0;
}
