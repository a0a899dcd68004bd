// Residency census (dev tool, GPU): how many workgroups of a given shape (threads, static LDS, VGPRs
// per lane) the MI355X keeps alive on one CU at once.  Each workgroup records its CU (HW_ID / XCC_ID)
// and its start / end time (s_memrealtime) around a ~20 us spin; the host reports the largest number
// of overlapping lifetimes on any CU.
//   hipcc --offload-arch=gfx950 -O3 -o tools/occupancy_probe tools/occupancy_probe.hip && tools/occupancy_probe
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <map>
#include <vector>

template <int NT, int LDSB, int VG>
__global__ void __launch_bounds__(NT) probe(unsigned long long* rec) {
  __shared__ unsigned char pad[LDSB > 0 ? LDSB : 4];
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  if (threadIdx.x == 0) {
    rec[blockIdx.x * 4 + 0] = t0;
    rec[blockIdx.x * 4 + 2] = __builtin_amdgcn_s_getreg(4 | (31 << 11));
    rec[blockIdx.x * 4 + 3] = __builtin_amdgcn_s_getreg(20 | (31 << 11));
  }
  pad[threadIdx.x % (LDSB > 0 ? LDSB : 4)] = 1;
  if constexpr (VG == 168) asm volatile("v_mov_b32 v167, 0" ::: "v167");
  if constexpr (VG == 64) asm volatile("v_mov_b32 v63, 0" ::: "v63");
  if constexpr (VG == 96) asm volatile("v_mov_b32 v95, 0" ::: "v95");
  if constexpr (VG == 128) asm volatile("v_mov_b32 v127, 0" ::: "v127");
  if constexpr (VG == 256) asm volatile("v_mov_b32 v255, 0" ::: "v255");
  while (__builtin_amdgcn_s_memrealtime() - t0 < 2000) __builtin_amdgcn_s_sleep(2);   // 20 us
  __syncthreads();
  if (threadIdx.x == 0) rec[blockIdx.x * 4 + 1] = __builtin_amdgcn_s_memrealtime();
  if (pad[(threadIdx.x + 1) % (LDSB > 0 ? LDSB : 4)] == 7) rec[0] = 0;
}

template <int NT, int LDSB, int VG>
void run(const char* name) {
  const int nwg = 2048;
  unsigned long long* d;
  hipMalloc(&d, nwg * 4 * sizeof(unsigned long long));
  hipLaunchKernelGGL((probe<NT, LDSB, VG>), dim3(nwg), dim3(NT), 0, 0, d);
  hipDeviceSynchronize();
  hipLaunchKernelGGL((probe<NT, LDSB, VG>), dim3(nwg), dim3(NT), 0, 0, d);
  hipDeviceSynchronize();
  std::vector<unsigned long long> h(nwg * 4);
  hipMemcpy(h.data(), d, h.size() * 8, hipMemcpyDeviceToHost);
  hipFree(d);
  std::map<unsigned, std::vector<std::pair<unsigned long long, int>>> ev;
  for (int i = 0; i < nwg; ++i) {
    const unsigned hw = (unsigned)h[i * 4 + 2], xcc = (unsigned)h[i * 4 + 3] & 0xF;
    const unsigned cu = ((hw >> 8) & 0xF) | (((hw >> 12) & 1) << 4) | (((hw >> 13) & 7) << 5) | (xcc << 8);
    ev[cu].push_back({h[i * 4 + 0], 1});
    ev[cu].push_back({h[i * 4 + 1], -1});
  }
  int best = 0;
  for (auto& kv : ev) {
    std::sort(kv.second.begin(), kv.second.end(), [](auto a, auto b) { return a.first != b.first ? a.first < b.first : a.second < b.second; });
    int cur = 0;
    for (auto& e : kv.second) best = std::max(best, cur += e.second);
  }
  printf("%-34s CUs %3zu  max workgroups alive per CU %d\n", name, ev.size(), best);
}

int main() {
  run<320, 0, 64>("320 thr, no LDS, 64 VGPR");
  run<320, 0, 96>("320 thr, no LDS, 96 VGPR");
  run<320, 0, 128>("320 thr, no LDS, 128 VGPR");
  run<320, 0, 168>("320 thr, no LDS, 168 VGPR");
  run<192, 0, 128>("192 thr, no LDS, 128 VGPR");
  run<192, 0, 168>("192 thr, no LDS, 168 VGPR");
  run<384, 0, 128>("384 thr, no LDS, 128 VGPR");
  run<384, 0, 168>("384 thr, no LDS, 168 VGPR");
  run<448, 0, 168>("448 thr, no LDS, 168 VGPR");
  run<640, 0, 128>("640 thr, no LDS, 128 VGPR");
  run<640, 0, 168>("640 thr, no LDS, 168 VGPR");
  run<640, 57256, 168>("640 thr, 57256 B LDS, 168 VGPR");
  run<256, 0, 64>("256 thr, no LDS, 64 VGPR");
  return 0;
}
