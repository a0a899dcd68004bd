// Device-scope hand-off latency probe (dev tool, GPU): the cost of one grid-wide exchange between
// resident workgroups, the unit the persistent decoder step (csrc/decoder_step.hip) pays several
// times per layer.  G workgroups of 256 threads (one per CU, G <= 256, all resident) run R rounds:
//   0 barrier    lane 0: one agent-scope atomic add on a shared counter, then poll it (s_sleep 1)
//                until it reaches (r + 1) G; the workgroup meets in an LDS barrier
//   1 hop        1 KB of 16-B write-through (sc1) stores, vmcnt(0), barrier, the atomic add; poll;
//                then 16-B sc1 loads of the NEXT workgroup's 1 KB (the decoder's publish / gather)
//   2 hop-spin   as 1, polling without s_sleep
//   3 tagged     no counter: every 16-B piece carries the round number in .w; each lane polls its
//                piece of the next workgroup's block until the tag matches (flag-in-payload)
//   4 tagged-12  as 3, each workgroup reads the blocks of the 12 workgroups after it (the decoder's
//                12-head gathers)
// Polls are bounded (2^22 iterations): a broken protocol ends the launch instead of hanging it.
// Prints the median / max over workgroups of microseconds per round (s_memrealtime, 100 MHz).
//   hipcc --offload-arch=gfx950 -O3 tools/hop_probe.hip -o tools/hop_probe && tools/hop_probe [G] [R]
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <cstdint>
#include <cstdlib>
#include <vector>

typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc_of(const void* p) {
  const uint64_t a = reinterpret_cast<uintptr_t>(p);
  const uint64_t u = (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)a) |
                     ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)(a >> 32)) << 32);
  return __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<void*>(u), (short)0, 0x7FFFFFFF, 0x00020000);
}
__device__ __forceinline__ u32x4 ld_sc1(const unsigned* base, int off) {
  return __builtin_amdgcn_raw_buffer_load_b128(rsrc_of(base), off * 4, 0, 16);
}
__device__ __forceinline__ void st_sc1(unsigned* base, int off, u32x4 v) {
  __builtin_amdgcn_raw_buffer_store_b128(v, rsrc_of(base), off * 4, 0, 16);
}

constexpr long long MAXIT = 1 << 22;

template <int MODE>
__global__ void __launch_bounds__(256) hop_kernel(unsigned* ctr, unsigned* blocks, int rounds, unsigned long long* t,
                                                  unsigned* sink, unsigned* fail) {
  __shared__ unsigned ok;
  const int G = gridDim.x, g = blockIdx.x, tid = threadIdx.x;
  unsigned acc = 0;
  __syncthreads();
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  for (int r = 0; r < rounds; ++r) {
    if (MODE == 1 || MODE == 2) {
      if (tid < 64) st_sc1(blocks, (g * 64 + tid) * 4, u32x4{(unsigned)r, (unsigned)g, 0u, (unsigned)r});
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    if (MODE <= 2) {
      __syncthreads();
      if (tid == 0) {
        __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const unsigned target = (unsigned)(r + 1) * G;
        long long it = 0;
        while (__hip_atomic_load(ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target && ++it < MAXIT)
          if (MODE != 2) __builtin_amdgcn_s_sleep(1);
        ok = it < MAXIT;
      }
      __syncthreads();
      if (!ok) { if (tid == 0) atomicAdd(fail, 1u); return; }
      if ((MODE == 1 || MODE == 2) && tid < 64) {
        const u32x4 v = ld_sc1(blocks, (((g + 1) % G) * 64 + tid) * 4);
        acc += v.x + v.w;
      }
    } else {
      // tagged: the payload is the flag
      const int nsrc = MODE == 3 ? 1 : 12;
      if (tid < 64) {
        // this round's block (double-buffered by round parity: a fast reader never sees a block
        // overwritten for round r + 1 before it read round r)
        unsigned* mine = blocks + (size_t)(r & 1) * G * 256;
        st_sc1(mine, (g * 64 + tid) * 4, u32x4{(unsigned)r + 1, (unsigned)g, 0u, (unsigned)r + 1});
      }
      bool good = true;
      if (tid < 64 * nsrc) {
        const int s = tid / 64, lane = tid & 63;
        const unsigned* src = blocks + (size_t)(r & 1) * G * 256;
        const int off = (((g + 1 + s) % G) * 64 + lane) * 4;
        long long it = 0;
        u32x4 v = ld_sc1(src, off);
        while (v.w < (unsigned)r + 1 && ++it < MAXIT) {
          __builtin_amdgcn_s_sleep(1);
          v = ld_sc1(src, off);
        }
        good = it < MAXIT;
        acc += v.x;
      }
      if (!good) atomicAdd(fail, 1u);
      __syncthreads();
    }
  }
  __syncthreads();
  const unsigned long long t1 = __builtin_amdgcn_s_memrealtime();
  if (tid == 0) t[g] = t1 - t0;
  if (acc == 0xdeadbeefu) sink[0] = acc;
}

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); return 1; } } while (0)

template <int MODE>
int run(const char* name, int G, int R) {
  unsigned *ctr, *blocks, *sink, *fail;
  unsigned long long* t;
  CK(hipMalloc(&ctr, 4)); CK(hipMalloc(&blocks, (size_t)2 * G * 256 * 4)); CK(hipMalloc(&sink, 4));
  CK(hipMalloc(&fail, 4)); CK(hipMalloc(&t, G * 8));
  std::vector<double> us;
  for (int rep = 0; rep < 3; ++rep) {
    CK(hipMemset(ctr, 0, 4)); CK(hipMemset(blocks, 0, (size_t)2 * G * 256 * 4)); CK(hipMemset(fail, 0, 4));
    hipLaunchKernelGGL(hop_kernel<MODE>, dim3(G), dim3(256), 0, 0, ctr, blocks, R, t, sink, fail);
    CK(hipDeviceSynchronize());
  }
  std::vector<unsigned long long> h(G);
  unsigned f = 0;
  CK(hipMemcpy(h.data(), t, G * 8, hipMemcpyDeviceToHost));
  CK(hipMemcpy(&f, fail, 4, hipMemcpyDeviceToHost));
  for (int i = 0; i < G; ++i) us.push_back(h[i] / 100.0 / R);
  std::sort(us.begin(), us.end());
  printf("%-10s G=%3d R=%5d  us/round median %6.3f  max %6.3f  %s\n", name, G, R, us[G / 2], us[G - 1], f ? "POLL TIMEOUTS" : "");
  CK(hipFree(ctr)); CK(hipFree(blocks)); CK(hipFree(sink)); CK(hipFree(fail)); CK(hipFree(t));
  return 0;
}

int main(int argc, char** argv) {
  const int G = argc > 1 ? atoi(argv[1]) : 120, R = argc > 2 ? atoi(argv[2]) : 2000;
  if (G < 13 || G > 256) { printf("G in [13, 256]\n"); return 1; }
  int rc = 0;
  rc |= run<0>("barrier", G, R);
  rc |= run<1>("hop", G, R);
  rc |= run<2>("hop-spin", G, R);
  rc |= run<3>("tagged", G, R);
  rc |= run<4>("tagged-12", G, R);
  return rc;
}
