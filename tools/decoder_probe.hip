// Decoder GEMV latency probe (dev tool, GPU): a chain of 36 dependent M = 10 linears (the recurrent
// decoder's 12 layers x 3 steps shape: f32 activations, fp16 weights [N][K], f32 accumulate), each
// launch reading the previous launch's output, captured in a HIP graph and replayed.  Reports the
// per-launch time of several kernel designs, with the weights hot (L2/MALL) and cold (a 1 GB sweep
// between replays), plus an empty-kernel chain for the launch-boundary floor.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/decoder_probe.hip -o /tmp/decoder_probe && /tmp/decoder_probe
#include <hip/hip_fp16.h>
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CHK(x)                                                                 \
  do {                                                                         \
    hipError_t e = (x);                                                        \
    if (e != hipSuccess) {                                                     \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); \
      exit(1);                                                                 \
    }                                                                          \
  } while (0)

typedef _Float16 f16;
typedef __attribute__((ext_vector_type(4))) float f32x4;

constexpr int M = 10;

__global__ void k_empty(const float* a, float* y) {
  if (threadIdx.x == 0 && blockIdx.x == 0 && a == nullptr) y[0] = 0.f;
}

// every workgroup reads the whole A block (M x K f32) and writes its 16 output columns
__global__ void __launch_bounds__(256) k_touch(const float* __restrict__ a, float* __restrict__ y, int N, int K) {
  __shared__ float red[4];
  float s = 0.f;
  for (int e = threadIdx.x * 4; e < M * K; e += 256 * 4) {
    const float4 v = *reinterpret_cast<const float4*>(a + e);
    s += v.x + v.y + v.z + v.w;
  }
  for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x < 16 * M) {
    const int m = threadIdx.x / 16, n = blockIdx.x * 16 + threadIdx.x % 16;
    y[m * N + n] = (red[0] + red[1] + red[2] + red[3]) * 1e-6f;
  }
}

// the product design (gemm_f32.hip skinny_kernel, KS = 1): 16 columns per workgroup, W waves split
// K, each lane issues all its loads of a 16*TS-deep trip up front, v_mfma_f32_16x16x4_f32, LDS
// reduction of the W partial tiles, bias epilogue
template <int W, int TS>
__global__ void __launch_bounds__(W * 64) k_skinny(const float* __restrict__ a, const f16* __restrict__ b,
                                                   const float* __restrict__ bias, float* __restrict__ y, int N, int K) {
  __shared__ float red[W][16][17];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int col = lane & 15, grp = lane >> 4;
  const int n0 = blockIdx.x * 16;
  const int kchunk = K / W;
  const int kb = wave * kchunk, ke = kb + kchunk;
  const float bv0 = bias[n0 + (threadIdx.x & 15)];
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  for (int k = kb; k < ke; k += 16 * TS) {
    float4 bq[TS], aq[TS];
#pragma unroll
    for (int u = 0; u < TS; ++u) {
      const int kk = k + 16 * u + 4 * grp;
      const bool ok = kk < ke;
      const uint2 w = ok ? *reinterpret_cast<const uint2*>(b + (long long)(n0 + col) * K + kk) : make_uint2(0, 0);
      const auto lo = [](unsigned x) { return (float)__builtin_bit_cast(f16, (unsigned short)(x & 0xFFFFu)); };
      const auto hi = [](unsigned x) { return (float)__builtin_bit_cast(f16, (unsigned short)(x >> 16)); };
      bq[u] = make_float4(lo(w.x), hi(w.x), lo(w.y), hi(w.y));
      aq[u] = (ok && col < M) ? *reinterpret_cast<const float4*>(a + col * K + kk) : make_float4(0.f, 0.f, 0.f, 0.f);
    }
#pragma unroll
    for (int u = 0; u < TS; ++u) {
      acc = __builtin_amdgcn_mfma_f32_16x16x4f32(aq[u].x, bq[u].x, acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_16x16x4f32(aq[u].y, bq[u].y, acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_16x16x4f32(aq[u].z, bq[u].z, acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_16x16x4f32(aq[u].w, bq[u].w, acc, 0, 0, 0);
    }
  }
#pragma unroll
  for (int r = 0; r < 4; ++r) red[wave][grp * 4 + r][col] = acc[r];
  __syncthreads();
  if (threadIdx.x < 256) {
    const int ml = threadIdx.x >> 4, nl = threadIdx.x & 15;
    if (ml < M) {
      float x = 0.f;
#pragma unroll
      for (int w = 0; w < W; ++w) x += red[w][ml][nl];
      y[ml * N + n0 + nl] = x + bv0;
    }
  }
}

// VALU design: one wave per 4 output columns, lanes split K in 8-element (16-B fp16) chunks, A read
// straight from global (L2) as float4 pairs, per-lane partial dot products for 10 rows x 4 columns,
// then a butterfly over the 64 lanes; no LDS, no barrier.  4 waves per workgroup = 16 columns.
template <int KMAX>
__global__ void __launch_bounds__(256) k_gemv(const float* __restrict__ a, const f16* __restrict__ b, const float* __restrict__ bias,
                                              float* __restrict__ y, int N, int K) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int n0 = blockIdx.x * 16 + wave * 4;
  constexpr int CH = KMAX / 8 / 64;   // chunks per lane (K = 768 -> 1.5: use KMAX multiple of 512)
  float acc[M][4];
#pragma unroll
  for (int m = 0; m < M; ++m)
#pragma unroll
    for (int c = 0; c < 4; ++c) acc[m][c] = 0.f;
#pragma unroll
  for (int i = 0; i < CH; ++i) {
    const int k = (lane + 64 * i) * 8;
    if (k < K) {
      uint4 w[4];
#pragma unroll
      for (int c = 0; c < 4; ++c) w[c] = *reinterpret_cast<const uint4*>(b + (long long)(n0 + c) * K + k);
      float4 av[M][2];
#pragma unroll
      for (int m = 0; m < M; ++m) {
        av[m][0] = *reinterpret_cast<const float4*>(a + m * K + k);
        av[m][1] = *reinterpret_cast<const float4*>(a + m * K + k + 4);
      }
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        const unsigned wu[4] = {w[c].x, w[c].y, w[c].z, w[c].w};
        float wf[8];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          wf[2 * e] = (float)__builtin_bit_cast(f16, (unsigned short)(wu[e] & 0xFFFFu));
          wf[2 * e + 1] = (float)__builtin_bit_cast(f16, (unsigned short)(wu[e] >> 16));
        }
#pragma unroll
        for (int m = 0; m < M; ++m) {
          acc[m][c] += av[m][0].x * wf[0] + av[m][0].y * wf[1] + av[m][0].z * wf[2] + av[m][0].w * wf[3] +
                       av[m][1].x * wf[4] + av[m][1].y * wf[5] + av[m][1].z * wf[6] + av[m][1].w * wf[7];
        }
      }
    }
  }
#pragma unroll
  for (int m = 0; m < M; ++m)
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      float v = acc[m][c];
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
      acc[m][c] = v;
    }
  if (lane < 4 * M) {
    const int m = lane >> 2, c = lane & 3;
    float v = 0.f;
#pragma unroll
    for (int mm = 0; mm < M; ++mm)
#pragma unroll
      for (int cc = 0; cc < 4; ++cc)
        if (mm == m && cc == c) v = acc[mm][cc];
    y[m * N + n0 + c] = v + bias[n0 + c];
  }
}

__global__ void k_sweep(float4* p, long long n) {
  for (long long i = blockIdx.x * 256LL + threadIdx.x; i < n; i += (long long)gridDim.x * 256) p[i] = make_float4(1.f, 2.f, 3.f, 4.f);
}

int main() {
  const int N = 768, K = 768, NL = 36;
  std::vector<f16*> ws(NL);
  float *a0, *a1, *bias, *ref, *sweep;
  const long long nsweep = 1LL << 26;   // 1 GB of float4
  CHK(hipMalloc(&sweep, nsweep * 16));
  for (int l = 0; l < NL; ++l) {
    CHK(hipMalloc(&ws[l], (size_t)N * K * 2));
    std::vector<f16> h((size_t)N * K);
    for (size_t i = 0; i < h.size(); ++i) h[i] = (f16)(((int)((i * 2654435761u + l * 97) % 2001) - 1000) * (1.0f / 1000.f / 27.7f));
    CHK(hipMemcpy(ws[l], h.data(), h.size() * 2, hipMemcpyHostToDevice));
  }
  CHK(hipMalloc(&a0, M * K * 4));
  CHK(hipMalloc(&a1, M * K * 4));
  CHK(hipMalloc(&ref, M * N * 4));
  CHK(hipMalloc(&bias, N * 4));
  CHK(hipMemset(bias, 0, N * 4));
  std::vector<float> ha(M * K);
  for (int i = 0; i < M * K; ++i) ha[i] = std::sin(0.37f * i);
  hipStream_t s;
  CHK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));

  // correctness of the variants on one launch against k_skinny<8, 8>
  auto check = [&](const char* name, auto launch) {
    CHK(hipMemcpy(a0, ha.data(), M * K * 4, hipMemcpyHostToDevice));
    k_skinny<8, 8><<<N / 16, 512, 0, s>>>(a0, ws[0], bias, ref, N, K);
    launch(a0, ws[0], a1);
    CHK(hipStreamSynchronize(s));
    std::vector<float> r(M * N), o(M * N);
    CHK(hipMemcpy(r.data(), ref, M * N * 4, hipMemcpyDeviceToHost));
    CHK(hipMemcpy(o.data(), a1, M * N * 4, hipMemcpyDeviceToHost));
    double md = 0, mr = 0;
    for (int i = 0; i < M * N; ++i) { md = fmax(md, fabs(r[i] - o[i])); mr = fmax(mr, fabs(r[i])); }
    printf("check %-28s max|d| %.3e (max|ref| %.3e)\n", name, md, mr);
  };
  auto timeit = [&](const char* name, auto launch) {
    CHK(hipMemcpy(a0, ha.data(), M * K * 4, hipMemcpyHostToDevice));
    hipGraph_t g;
    hipGraphExec_t ge;
    CHK(hipStreamBeginCapture(s, hipStreamCaptureModeGlobal));
    for (int l = 0; l < NL; ++l) launch(l & 1 ? a1 : a0, ws[l], l & 1 ? a0 : a1);
    CHK(hipStreamEndCapture(s, &g));
    CHK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
    hipEvent_t e0, e1;
    CHK(hipEventCreate(&e0));
    CHK(hipEventCreate(&e1));
    for (int cold = 0; cold < 2; ++cold) {
      float tot = 0.f;
      const int reps = 20;
      for (int r = 0; r < reps + 2; ++r) {
        if (cold) k_sweep<<<2048, 256, 0, s>>>(reinterpret_cast<float4*>(sweep), nsweep);
        CHK(hipEventRecord(e0, s));
        CHK(hipGraphLaunch(ge, s));
        CHK(hipEventRecord(e1, s));
        CHK(hipEventSynchronize(e1));
        float ms;
        CHK(hipEventElapsedTime(&ms, e0, e1));
        if (r >= 2) tot += ms;
      }
      printf("%-30s %s  %.2f us per launch\n", name, cold ? "cold" : "hot ", tot / reps / NL * 1e3);
    }
    CHK(hipGraphExecDestroy(ge));
    CHK(hipGraphDestroy(g));
  };

  check("skinny<4,8>", [&](float* a, f16* w, float* y) { k_skinny<4, 8><<<N / 16, 256, 0, s>>>(a, w, bias, y, N, K); });
  check("gemv<1024>", [&](float* a, f16* w, float* y) { k_gemv<1024><<<N / 16, 256, 0, s>>>(a, w, bias, y, N, K); });

  timeit("empty 48x512", [&](float* a, f16* w, float* y) { k_empty<<<48, 512, 0, s>>>(a, y); });
  timeit("empty 48x256", [&](float* a, f16* w, float* y) { k_empty<<<48, 256, 0, s>>>(a, y); });
  timeit("touch 48x256", [&](float* a, f16* w, float* y) { k_touch<<<48, 256, 0, s>>>(a, y, N, K); });
  timeit("skinny<8,8> 48x512", [&](float* a, f16* w, float* y) { k_skinny<8, 8><<<N / 16, 512, 0, s>>>(a, w, bias, y, N, K); });
  timeit("skinny<4,8> 48x256", [&](float* a, f16* w, float* y) { k_skinny<4, 8><<<N / 16, 256, 0, s>>>(a, w, bias, y, N, K); });
  timeit("skinny<16,8> 48x1024", [&](float* a, f16* w, float* y) { k_skinny<16, 8><<<N / 16, 1024, 0, s>>>(a, w, bias, y, N, K); });
  timeit("gemv<1024> 48x256", [&](float* a, f16* w, float* y) { k_gemv<1024><<<N / 16, 256, 0, s>>>(a, w, bias, y, N, K); });
  return 0;
}
