// Exact-f32 GEMM on the f32-input MFMA (v_mfma_f32_16x16x4_f32, 64 FLOP/clk/SIMD = the f32 VALU
// peak): used when the B operand is f32 — the recurrent decoder's query-side linears, whose M is
// the number of summary tokens (B or 5B <= 64 rows).  Those GEMMs are weight-bandwidth bound, so
// reading the f32 master weights directly costs 2x the bytes of a bf16 shadow but removes the
// dominant rounding error of the recurrence (36 sequential layer-steps).
// Same operand layouts / epilogues / split-K contract as lrce_gemm's bf16 path.
// Tile 64x64x32, 256 threads = 4 waves (2x2), 32x32 per wave = 2x2 MFMA blocks of 16x16.
#include "common.h"
#include "lrce_capi.h"

namespace {

constexpr int BM = 64, BN = 64, BK = 32, NT = 256, LD = BK + 1;

struct GemmF32P {
  const float* a;
  const float* b;
  void* c;
  long long lda, ldb, ldc;
  int m, n, k, k_chunk, split_k;
  int a_kmajor, b_kmajor;
  int flags;
  const float* bias;
  const void* aux;
  long long ld_aux;
  bf16* aux_out;
  long long ld_aux_out;
  const int* a_map;
  const int* c_map;
  float alpha;
  const float* row_scale;
  int rows_per_scale;
  const float* a_row_scale;
  int a_rows_per_scale;
  int tiles_n;
};

// stage a 64 (rows) x 32 (k) tile of an operand into LDS as [row][k] (padded)
__device__ __forceinline__ void stage(float (*lds)[LD], const float* base, long long ld, bool kmajor, int rows_total, int kend,
                                      int row0, int k0, const int* map, const float* rsc, int rps) {
  const int tid = threadIdx.x;
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int c = tid + NT * i;  // 512 float4 chunks
    if (kmajor) {
      const int r = c >> 3, kk = (c & 7) * 4;
      const int gr = row0 + r, gk = k0 + kk;
      float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
      if (gr < rows_total && gk < kend) {
        const long long rr = map ? (long long)map[gr] : (long long)gr;
        v = *reinterpret_cast<const float4*>(base + rr * ld + gk);
        if (rsc) { const float f = rsc[gr / rps]; v.x *= f; v.y *= f; v.z *= f; v.w *= f; }
      }
      lds[r][kk] = v.x; lds[r][kk + 1] = v.y; lds[r][kk + 2] = v.z; lds[r][kk + 3] = v.w;
    } else {
      const int kk = c >> 4, r = (c & 15) * 4;
      const int gr = row0 + r, gk = k0 + kk;
      float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
      if (gk < kend && gr < rows_total) {
        const long long kr = map ? (long long)map[gk] : (long long)gk;
        v = *reinterpret_cast<const float4*>(base + kr * ld + gr);
        if (rsc) { const float f = rsc[gk / rps]; v.x *= f; v.y *= f; v.z *= f; v.w *= f; }
      }
      lds[r][kk] = v.x; lds[r + 1][kk] = v.y; lds[r + 2][kk] = v.z; lds[r + 3][kk] = v.w;
    }
  }
}

__global__ void __launch_bounds__(NT) gemm_f32_kernel(GemmF32P p) {
  __shared__ float As[BM][LD];
  __shared__ float Bs[BN][LD];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const int tile = blockIdx.x;
  const int tn = tile % p.tiles_n, tm = tile / p.tiles_n;
  const int m0 = tm * BM, n0 = tn * BN;
  const int sk = blockIdx.y;
  const int kb = sk * p.k_chunk, ke = min(p.k, kb + p.k_chunk);
  f32x4 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  for (int k0 = kb; k0 < ke; k0 += BK) {
    stage(As, p.a, p.lda, p.a_kmajor, p.m, ke, m0, k0, p.a_map, p.a_row_scale, p.a_rows_per_scale);
    stage(Bs, p.b, p.ldb, p.b_kmajor, p.n, ke, n0, k0, nullptr, nullptr, 1);
    __syncthreads();
#pragma unroll
    for (int kk = 0; kk < BK; kk += 4) {
      float av[2], bv[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) av[i] = As[wm * 32 + i * 16 + (lane & 15)][kk + (lane >> 4)];
#pragma unroll
      for (int j = 0; j < 2; ++j) bv[j] = Bs[wn * 32 + j * 16 + (lane & 15)][kk + (lane >> 4)];
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[i], bv[j], acc[i][j], 0, 0, 0);
    }
    __syncthreads();
  }
  const int fl = p.flags;
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int n = n0 + wn * 32 + j * 16 + (lane & 15);
    if (n >= p.n) continue;
    const float bias = ((fl & LRCE_EPI_BIAS) && sk == 0) ? p.bias[n] : 0.f;
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = m0 + wm * 32 + i * 16 + (lane >> 4) * 4 + r;
        if (m >= p.m) continue;
        const long long row = p.c_map ? (long long)p.c_map[m] : (long long)m;
        float v = acc[i][j][r] * p.alpha + bias;
        if (fl & LRCE_EPI_GELU) {
          if (fl & LRCE_EPI_AUX_OUT) p.aux_out[row * p.ld_aux_out + n] = f2bf(v);
          v = gelu_f(v);
        }
        if (fl & LRCE_EPI_DGELU) v *= gelu_grad_f(bf2f(static_cast<const bf16*>(p.aux)[row * p.ld_aux + n]));
        if (p.row_scale) v *= p.row_scale[m / p.rows_per_scale];
        if ((fl & LRCE_EPI_RESID) && sk == 0) v += static_cast<const float*>(p.aux)[row * p.ld_aux + n];
        if (fl & LRCE_EPI_ATOMIC) atomicAdd(static_cast<float*>(p.c) + row * p.ldc + n, v);
        else if (fl & LRCE_EPI_ACCUM) static_cast<float*>(p.c)[row * p.ldc + n] += v;
        else if (fl & LRCE_EPI_OUT_F32) {
          static_cast<float*>(p.c)[row * p.ldc + n] = v;
          if (fl & LRCE_EPI_OUT_BOTH) p.aux_out[row * p.ld_aux_out + n] = f2bf(v);
        } else static_cast<bf16*>(p.c)[row * p.ldc + n] = f2bf(v);
      }
  }
}

}  // namespace

int lrce_gemm_f32(const LrceGemmDesc* d, void* stream) {
  if (!d->a_f32) return lrce_fail(LRCE_E_ARG, "gemm(f32 B): A must be f32 too");
  if (d->batch != 1) return lrce_fail(LRCE_E_ARG, "gemm(f32 B): batch must be 1");
  if (d->a_kmajor ? (d->k % 4) : (d->m % 4)) return lrce_fail(LRCE_E_ARG, "gemm(f32): A contiguous dim %% 4 != 0");
  if (d->b_kmajor ? (d->k % 4) : (d->n % 4)) return lrce_fail(LRCE_E_ARG, "gemm(f32): B contiguous dim %% 4 != 0");
  if ((d->lda % 4) || (d->ldb % 4)) return lrce_fail(LRCE_E_ARG, "gemm(f32): lda/ldb %% 4 != 0");
  GemmF32P p;
  p.a = static_cast<const float*>(d->a); p.b = static_cast<const float*>(d->b); p.c = d->c;
  p.lda = d->lda; p.ldb = d->ldb; p.ldc = d->ldc;
  p.m = d->m; p.n = d->n; p.k = d->k;
  p.a_kmajor = d->a_kmajor; p.b_kmajor = d->b_kmajor;
  p.flags = d->flags; p.bias = d->bias; p.aux = d->aux; p.ld_aux = d->ld_aux;
  p.aux_out = static_cast<bf16*>(d->aux_out); p.ld_aux_out = d->ld_aux_out;
  p.a_map = d->a_map; p.c_map = d->c_map; p.alpha = d->alpha;
  p.row_scale = d->row_scale; p.rows_per_scale = d->rows_per_scale > 0 ? d->rows_per_scale : 1;
  p.a_row_scale = d->a_row_scale; p.a_rows_per_scale = d->a_rows_per_scale > 0 ? d->a_rows_per_scale : 1;
  const int tiles_m = (d->m + BM - 1) / BM;
  p.tiles_n = (d->n + BN - 1) / BN;
  int split = d->split_k > 1 ? d->split_k : 1;
  if (split > 1 && !(d->flags & LRCE_EPI_ATOMIC)) return lrce_fail(LRCE_E_ARG, "gemm(f32): split_k needs ATOMIC");
  int chunk = (d->k + split - 1) / split;
  chunk = (chunk + BK - 1) / BK * BK;
  p.k_chunk = chunk;
  p.split_k = split;
  dim3 grid(tiles_m * p.tiles_n, split);
  gemm_f32_kernel<<<grid, NT, 0, static_cast<hipStream_t>(stream)>>>(p);
  return lrce_check_launch("gemm_f32");
}
