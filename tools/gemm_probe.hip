// GEMM design probe (dev tool, GPU): a persistent 256x256-tile bf16 GEMM, one 4-wave workgroup per
// CU, 128x128 per wave on v_mfma_f32_32x32x16_bf16, BK = 32, a 4-stage LDS-DMA ring (three K tiles
// in flight).  C[M][N] (bf16) = A[M][K] . B[N][K]^T.  Checks one shape against a naive kernel, then
// times the step's forward shapes.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/gemm_probe.hip -o /tmp/gemm_probe && /tmp/gemm_probe
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <cmath>
#include <vector>

typedef __bf16 bf16;
typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) __bf16 bf16x4;
typedef __attribute__((ext_vector_type(16))) float f32x16;

#define CHK(x)                                                                 \
  do {                                                                         \
    hipError_t e = (x);                                                        \
    if (e != hipSuccess) {                                                     \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); \
      exit(1);                                                                 \
    }                                                                          \
  } while (0)

constexpr int TM = 256, TN = 256, BK = 32, NS = 4, NT = 256;
constexpr int ROWB = BK * 2;                 // 64 B per staged row
constexpr int STG = (TM + TN) * ROWB;        // 32 KB per stage
constexpr int PIECES = (TM + TN) / 16;       // 1-KB DMA pieces per stage (32)
constexpr int PPW = PIECES / 4;              // per wave (8)

__device__ __forceinline__ int swz(int r) { return ((r >> 1) ^ (r >> 2)) & 3; }
__device__ __forceinline__ int opnd(int row, int c) { return row * ROWB + ((c ^ swz(row)) << 4); }

__device__ __forceinline__ void glds_s(const void* sbase, uint32_t voff, uint32_t lds_dst) {
  unsigned keep;
  const uint64_t a = reinterpret_cast<uintptr_t>(sbase);
  const uint64_t su = (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)a) |
                      ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)(a >> 32)) << 32);
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, %2\n\ts_mov_b32 m0, %0"
               : "=&s"(keep) : "v"(voff), "s"(su), "s"(__builtin_amdgcn_readfirstlane(lds_dst)) : "memory");
}
__device__ __forceinline__ uint32_t lds_addr(const void* p) {
  return (uint32_t)(uintptr_t)((__attribute__((address_space(3))) const void*)p);
}

__global__ void __launch_bounds__(NT, 1) gemm256(const bf16* __restrict__ A, const bf16* __restrict__ B, bf16* __restrict__ C,
                                               int M, int N, int K, int store, int reps = 0) {
  __shared__ __attribute__((aligned(16))) char lds[NS * STG];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int wave_u = __builtin_amdgcn_readfirstlane(wave);
  const int wm = wave >> 1, wn = wave & 1;
  const int tiles_m = (M + TM - 1) / TM, tiles_n = (N + TN - 1) / TN, ntiles = tiles_m * tiles_n;
  const int nk = K / BK;
  const uint32_t lbase = lds_addr(lds);
  // reps > 0: every workgroup computes tile (blockIdx.x % ntiles) `reps` times (L2-resident operands)
  const int tend = reps > 0 ? reps : ntiles;
  for (int tt = blockIdx.x; tt < (reps > 0 ? (int)gridDim.x * reps : tend); tt += gridDim.x) {
    const int t = reps > 0 ? blockIdx.x % ntiles : tt;
    // grouped order: 8 tile-rows per group, column-major inside (A panels reused across a group)
    const int GROUP = 8;
    const int gsz = GROUP * tiles_n;
    const int g = t / gsz, gr = t % gsz;
    const int rows_g = min(GROUP, tiles_m - g * GROUP);
    const int tm = g * GROUP + gr % rows_g, tn = gr / rows_g;
    const int m0 = tm * TM, n0 = tn * TN;
    uint32_t voff[PPW];
#pragma unroll
    for (int q = 0; q < PPW; ++q) {
      const int e = wave + 4 * q;                      // q < 4: A pieces, else B
      const int r = 16 * (e & 15) + (lane >> 2);      // row inside the operand tile
      const int img_row = (q < 4 ? 0 : TM) + r;
      const int c = (lane & 3) ^ swz(img_row);
      const int gr2 = q < 4 ? min(m0 + r, M - 1) : min(n0 + r, N - 1);
      voff[q] = (uint32_t)(((long long)gr2 * K + c * 8) * 2);
    }
    auto issue = [&](int kt, int st) {
#pragma unroll
      for (int q = 0; q < PPW; ++q)
        glds_s(reinterpret_cast<const char*>(q < 4 ? A : B) + kt * BK * 2, voff[q],
               lbase + (uint32_t)(st * STG) + (uint32_t)((wave_u + 4 * q) * 1024));
    };
    f32x16 acc[4][4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = f32x16{};
#pragma unroll
    for (int s = 0; s < NS - 1; ++s)
      if (s < nk) issue(s, s);
    for (int kt = 0; kt < nk; ++kt) {
      const int ahead = min(nk - 1 - kt, NS - 2);
      if (ahead >= 2) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * PPW) : "memory");
      else if (ahead == 1) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(PPW) : "memory");
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      __builtin_amdgcn_sched_barrier(0);
      if (kt + NS - 1 < nk) issue(kt + NS - 1, (kt + NS - 1) % NS);
      const char* st = lds + (kt % NS) * STG;
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        bf16x8 af[4], bfr[4];
#pragma unroll
        for (int i = 0; i < 4; ++i)
          af[i] = *reinterpret_cast<const bf16x8*>(st + opnd(wm * 128 + i * 32 + (lane & 31), 2 * ks + (lane >> 5)));
#pragma unroll
        for (int j = 0; j < 4; ++j)
          bfr[j] = *reinterpret_cast<const bf16x8*>(st + opnd(TM + wn * 128 + j * 32 + (lane & 31), 2 * ks + (lane >> 5)));
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(bfr[j], af[i], acc[i][j], 0, 0, 0);
      }
      __builtin_amdgcn_sched_barrier(0);
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    // C^T blocks: lane holds row m = m0 + wm*128 + i*32 + (lane&31), columns n = ... + 8(r/4) + 4hh + r%4
    if (store) {
      const int hh = lane >> 5;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int m = m0 + wm * 128 + i * 32 + (lane & 31);
        if (m >= M) continue;
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
          for (int g4 = 0; g4 < 4; ++g4) {
            const int n = n0 + wn * 128 + j * 32 + 8 * g4 + 4 * hh;
            if (n + 4 <= N) {
              bf16x4 v;
              v[0] = (bf16)acc[i][j][4 * g4]; v[1] = (bf16)acc[i][j][4 * g4 + 1];
              v[2] = (bf16)acc[i][j][4 * g4 + 2]; v[3] = (bf16)acc[i][j][4 * g4 + 3];
              *reinterpret_cast<bf16x4*>(C + (long long)m * N + n) = v;
            }
          }
      }
    }
  }
}


// Variant R: register-staged operand loads (global_load_dwordx4 -> VGPR -> ds_write_b128), BK = 64,
// two LDS stages [256 rows][64 k] per operand (128 B rows, 16-B chunk c at c ^ (row & 7)), one tile in
// registers in flight while the other two live in LDS.
constexpr int RBK = 64, RROWB = 128, RSTG = (TM + TN) * RROWB;   // 64 KB per stage
__device__ __forceinline__ int ropnd(int row, int c) { return row * RROWB + ((c ^ (row & 7)) << 4); }

__global__ void __launch_bounds__(NT, 1) gemm256r(const bf16* __restrict__ A, const bf16* __restrict__ B, bf16* __restrict__ C,
                                                int M, int N, int K, int store) {
  __shared__ __attribute__((aligned(16))) char lds[2 * RSTG];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, tid = threadIdx.x;
  const int wm = wave >> 1, wn = wave & 1;
  const int tiles_m = (M + TM - 1) / TM, tiles_n = (N + TN - 1) / TN, ntiles = tiles_m * tiles_n;
  const int nk = K / RBK;
  for (int t = blockIdx.x; t < ntiles; t += gridDim.x) {
    const int GROUP = 8;
    const int gsz = GROUP * tiles_n;
    const int g = t / gsz, gr = t % gsz;
    const int rows_g = min(GROUP, tiles_m - g * GROUP);
    const int tm = g * GROUP + gr % rows_g, tn = gr / rows_g;
    const int m0 = tm * TM, n0 = tn * TN;
    // thread tid loads 16 chunks per K tile: chunk i -> operand row (tid >> 3) + 32 i (rows 0..255 A,
    // 256..511 B), 16-B column tid & 7; the LDS slot of chunk i is dst0 + i * 32 rows
    uint32_t off[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int row = (tid >> 3) + 32 * i;
      const int gr2 = row < TM ? min(m0 + row, M - 1) : min(n0 + row - TM, N - 1);
      off[i] = (uint32_t)((long long)gr2 * K + (tid & 7) * 8);
    }
    const int dst0 = ropnd(tid >> 3, tid & 7);
    uint4 stage_regs[16];
    auto gload = [&](int kt) {
#pragma unroll
      for (int i = 0; i < 16; ++i) stage_regs[i] = *reinterpret_cast<const uint4*>((i < 8 ? A : B) + off[i] + kt * RBK);
    };
    auto swrite = [&](int st) {
#pragma unroll
      for (int i = 0; i < 16; ++i) *reinterpret_cast<uint4*>(lds + st * RSTG + dst0 + i * 32 * RROWB) = stage_regs[i];
    };
    f32x16 acc[4][4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = f32x16{};
    gload(0);
    swrite(0);
    if (nk > 1) gload(1);
    __syncthreads();
    for (int kt = 0; kt < nk; ++kt) {
      const char* st = lds + (kt & 1) * RSTG;
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) {
        bf16x8 af[4], bfr[4];
#pragma unroll
        for (int i = 0; i < 4; ++i)
          af[i] = *reinterpret_cast<const bf16x8*>(st + ropnd(wm * 128 + i * 32 + (lane & 31), 2 * ks + (lane >> 5)));
#pragma unroll
        for (int j = 0; j < 4; ++j)
          bfr[j] = *reinterpret_cast<const bf16x8*>(st + ropnd(TM + wn * 128 + j * 32 + (lane & 31), 2 * ks + (lane >> 5)));
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(bfr[j], af[i], acc[i][j], 0, 0, 0);
      }
      if (kt + 1 < nk) {
        swrite((kt + 1) & 1);            // stage (kt+1)&1 was consumed in iteration kt-1 (barrier since)
        if (kt + 2 < nk) gload(kt + 2);
      }
      __syncthreads();
    }
    if (store) {
      const int hh = lane >> 5;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int m = m0 + wm * 128 + i * 32 + (lane & 31);
        if (m >= M) continue;
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
          for (int g4 = 0; g4 < 4; ++g4) {
            const int n = n0 + wn * 128 + j * 32 + 8 * g4 + 4 * hh;
            if (n + 4 <= N) {
              bf16x4 v;
              v[0] = (bf16)acc[i][j][4 * g4]; v[1] = (bf16)acc[i][j][4 * g4 + 1];
              v[2] = (bf16)acc[i][j][4 * g4 + 2]; v[3] = (bf16)acc[i][j][4 * g4 + 3];
              *reinterpret_cast<bf16x4*>(C + (long long)m * N + n) = v;
            }
          }
      }
    }
  }
}

__global__ void ref_gemm(const bf16* A, const bf16* B, float* C, int M, int N, int K) {
  const int m = blockIdx.y, n = blockIdx.x * blockDim.x + threadIdx.x;
  if (n >= N) return;
  float s = 0.f;
  for (int k = 0; k < K; ++k) s += (float)A[(long long)m * K + k] * (float)B[(long long)n * K + k];
  C[(long long)m * N + n] = s;
}

__global__ void fill(bf16* x, long long n, unsigned seed) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  unsigned h = (unsigned)(i * 2654435761u) ^ seed;
  h ^= h >> 15; h *= 0x2c1b3c6dU; h ^= h >> 12;
  x[i] = (bf16)(((float)(h & 0xFFFF) / 65536.f - 0.5f));
}

int main() {
  int cus = 256;
  struct Shape { int m, n, k; };
  std::vector<Shape> shapes = {{4096, 4096, 4096}, {17640, 2048, 512}, {17640, 1536, 512}, {17640, 512, 2048},
                               {17640, 512, 512}, {282240, 512, 128}, {282240, 128, 512}, {17640, 2048, 4096}};
  // correctness on a ragged shape
  {
    const int M = 300, N = 520, K = 96;
    bf16 *A, *B, *C;
    float* R;
    CHK(hipMalloc(&A, (size_t)M * K * 2)); CHK(hipMalloc(&B, (size_t)N * K * 2));
    CHK(hipMalloc(&C, (size_t)M * N * 2)); CHK(hipMalloc(&R, (size_t)M * N * 4));
    fill<<<(M * K + 255) / 256, 256>>>(A, (long long)M * K, 1);
    fill<<<(N * K + 255) / 256, 256>>>(B, (long long)N * K, 2);
    gemm256<<<cus, NT>>>(A, B, C, M, N, K, 1);
    ref_gemm<<<dim3((N + 255) / 256, M), 256>>>(A, B, R, M, N, K);
    CHK(hipDeviceSynchronize());
    std::vector<uint16_t> hc((size_t)M * N);
    std::vector<float> hr((size_t)M * N);
    CHK(hipMemcpy(hc.data(), C, hc.size() * 2, hipMemcpyDeviceToHost));
    CHK(hipMemcpy(hr.data(), R, hr.size() * 4, hipMemcpyDeviceToHost));
    double err = 0, mx = 0;
    for (int m = 0; m < M; ++m)
      for (int n = 0; n < N - N % 4; ++n) {
        uint32_t u = (uint32_t)hc[(size_t)m * N + n] << 16;
        float v;
        std::memcpy(&v, &u, 4);
        err = fmax(err, fabs(v - hr[(size_t)m * N + n]));
        mx = fmax(mx, fabs(hr[(size_t)m * N + n]));
      }
    printf("check %dx%dx%d: max err %.3e (max |ref| %.3e)\n", M, N, K, err, mx);
    CHK(hipFree(A)); CHK(hipFree(B)); CHK(hipFree(C)); CHK(hipFree(R));
  }
  {
    // L2-resident operands: 256 workgroups recompute the same 4 tiles (K = 4096), 4 times each
    const int M = 512, N = 512, K = 4096;
    bf16 *A, *B, *C;
    CHK(hipMalloc(&A, (size_t)M * K * 2)); CHK(hipMalloc(&B, (size_t)N * K * 2)); CHK(hipMalloc(&C, (size_t)M * N * 2));
    fill<<<(M * K + 255) / 256, 256>>>(A, (long long)M * K, 1);
    fill<<<(N * K + 255) / 256, 256>>>(B, (long long)N * K, 2);
    hipEvent_t e0, e1;
    CHK(hipEventCreate(&e0)); CHK(hipEventCreate(&e1));
    for (int w = 0; w < 3; ++w) gemm256<<<cus, NT>>>(A, B, C, M, N, K, 0, 4);
    CHK(hipEventRecord(e0));
    for (int w = 0; w < 10; ++w) gemm256<<<cus, NT>>>(A, B, C, M, N, K, 0, 4);
    CHK(hipEventRecord(e1));
    CHK(hipEventSynchronize(e1));
    float ms;
    CHK(hipEventElapsedTime(&ms, e0, e1));
    const double us = ms * 100.0;
    const double fl = 2.0 * 256 * 256 * K * cus * 4;
    printf("L2-resident: %.1f us  %.1f TF/s (%.3f)  DMA %.1f GB/s per CU\n", us, fl / us * 1e-6, fl / us * 1e-6 / 2500,
           (double)(256 + 256) * K * 2 * 4 / us * 1e-3);
    CHK(hipFree(A)); CHK(hipFree(B)); CHK(hipFree(C));
  }
  for (auto s : shapes) {
    bf16 *A, *B, *C;
    CHK(hipMalloc(&A, (size_t)s.m * s.k * 2)); CHK(hipMalloc(&B, (size_t)s.n * s.k * 2));
    CHK(hipMalloc(&C, (size_t)s.m * s.n * 2));
    fill<<<(unsigned)(((long long)s.m * s.k + 255) / 256), 256>>>(A, (long long)s.m * s.k, 1);
    fill<<<(unsigned)(((long long)s.n * s.k + 255) / 256), 256>>>(B, (long long)s.n * s.k, 2);
    const int tiles = ((s.m + TM - 1) / TM) * ((s.n + TN - 1) / TN);
    const int grid = tiles < cus ? tiles : cus;
    hipEvent_t e0, e1;
    CHK(hipEventCreate(&e0)); CHK(hipEventCreate(&e1));
    for (int st = 0; st < 4; ++st) {
      auto run = [&]() {
        if (st < 2) gemm256<<<grid, NT>>>(A, B, C, s.m, s.n, s.k, st);
        else gemm256r<<<grid, NT>>>(A, B, C, s.m, s.n, s.k, st - 2);
      };
      for (int w = 0; w < 3; ++w) run();
      const int it = 20;
      CHK(hipEventRecord(e0));
      for (int w = 0; w < it; ++w) run();
      CHK(hipEventRecord(e1));
      CHK(hipEventSynchronize(e1));
      float ms;
      CHK(hipEventElapsedTime(&ms, e0, e1));
      const double us = ms * 1000.0 / it;
      const double tf = 2.0 * s.m * s.n * s.k / us * 1e-6;
      printf("%s %6d x %5d x %5d store=%d: %8.1f us %7.1f TF/s (%.3f of 2.5 PF)  tiles %d\n", st < 2 ? "dma" : "reg", s.m, s.n, s.k, st % 2, us, tf,
             tf / 2500.0, tiles);
    }
    CHK(hipFree(A)); CHK(hipFree(B)); CHK(hipFree(C));
  }
  return 0;
}
