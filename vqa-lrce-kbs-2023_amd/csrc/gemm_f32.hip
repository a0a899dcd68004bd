// Exact-f32 GEMM on the f32-input MFMA (v_mfma_f32_16x16x4_f32, 64 FLOP/clk/SIMD = the f32 VALU
// peak): used when the B operand is f32 — the recurrent decoder's query-side linears, whose M is
// the number of summary tokens (B or 5B <= 64 rows).  Those GEMMs are weight-bandwidth bound, so
// reading the f32 master weights directly costs 2x the bytes of a bf16 shadow but removes the
// dominant rounding error of the recurrence (36 sequential layer-steps).
// Same operand layouts / epilogues / split-K contract as lrce_gemm's bf16 path.
// Tile 64x64x32, 256 threads = 4 waves (2x2), 32x32 per wave = 2x2 MFMA blocks of 16x16.
#include <algorithm>
#include <cstdlib>

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
        if (row < 0) continue;   // c_map -1: padded position, no output row
        float v = acc[i][j][r] * p.alpha + bias;
        if (fl & LRCE_EPI_GELU) {
          if (fl & LRCE_EPI_AUX_OUT) {
            if (fl & LRCE_EPI_AUX_F32) reinterpret_cast<float*>(p.aux_out)[row * p.ld_aux_out + n] = v;
            else p.aux_out[row * p.ld_aux_out + n] = f2bf(v);
          }
          v = gelu_f(v);
        }
        if (fl & LRCE_EPI_DGELU)
          v *= gelu_grad_f((fl & LRCE_EPI_AUX_F32) ? static_cast<const float*>(p.aux)[row * p.ld_aux + n]
                                                   : bf2f(static_cast<const bf16*>(p.aux)[row * p.ld_aux + n]));
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


// ---------------------------------------------------------------------------------------------
// Skinny-M exact-f32 kernels (M <= 64: the decoder's B or 5B summary-token rows).  The tiled kernel
// above puts a 64x64 tile per block, i.e. only N/64 blocks for these shapes; here a block owns 16
// output columns for ALL rows and its 4 waves split the reduction, so a 768-wide linear is 48
// blocks that each stream a 16-row slab of the weight once (float4 / 64-B row segments), and the
// 4 partial 16x16 tiles are combined through LDS before the fused epilogue.

constexpr int SK_NT = 256;

struct SkinnyP {
  const float* a;
  const void* b;        // f32, or IEEE fp16 (BH: the decoder's fp16 weight shadow, f32 compute)
  void* c;
  long long lda, ldb, ldc;
  int m, n, k;
  int flags;
  const float* bias;
  const void* aux;
  long long ld_aux;
  bf16* aux_out;
  long long ld_aux_out;
  float alpha;
  const float* row_scale;
  int rows_per_scale;
  int scale_cols;
  float scale_val;
  float* bias_grad;
  float drop_p;
  int drop_group;
  uint64_t drop_seed;
  const uint64_t* rng_off;
};

// The epilogue's global operands of one output element (bias, dGELU pre-activation, residual, the
// accumulated C), loaded at kernel start so they ride the same memory round trip as the weights
// instead of a second one after the reduction.
struct SkPre {
  float bias, dg, res, acc;
};

// four consecutive-k elements of B(n, k..k+3) as f32: B_KM -> B[n][k..k+3] (one 16-B f32 / 8-B fp16
// load), else B[k..k+3][n] (strided); BH: B holds IEEE fp16 (converted exactly to f32)
template <bool B_KM, bool BH>
__device__ __forceinline__ float4 ld_b4(const void* b, long long ldb, int n, int k) {
  if constexpr (BH) {
    const f16* bp = static_cast<const f16*>(b);
    if constexpr (B_KM) {
      const uint2 u = *reinterpret_cast<const uint2*>(bp + (long long)n * ldb + k);
      const auto lo = [](unsigned x) { return (float)__builtin_bit_cast(f16, (unsigned short)(x & 0xFFFFu)); };
      const auto hi = [](unsigned x) { return (float)__builtin_bit_cast(f16, (unsigned short)(x >> 16)); };
      return make_float4(lo(u.x), hi(u.x), lo(u.y), hi(u.y));
    } else {
      const f16* q = bp + (long long)k * ldb + n;
      return make_float4((float)q[0], (float)q[ldb], (float)q[2 * ldb], (float)q[3 * ldb]);
    }
  } else {
    const float* bp = static_cast<const float*>(b);
    if constexpr (B_KM) return *reinterpret_cast<const float4*>(bp + (long long)n * ldb + k);
    else {
      const float* q = bp + (long long)k * ldb + n;
      return make_float4(q[0], q[ldb], q[2 * ldb], q[3 * ldb]);
    }
  }
}

__device__ __forceinline__ SkPre sk_prefetch(const SkinnyP& p, int m, int n) {
  SkPre e{0.f, 1.f, 0.f, 0.f};
  if (m >= p.m || n >= p.n) return e;
  const int fl = p.flags;
  const long long row = m;
  if (fl & LRCE_EPI_BIAS) e.bias = p.bias[n];
  if (fl & LRCE_EPI_DGELU)
    e.dg = (fl & LRCE_EPI_AUX_F32) ? static_cast<const float*>(p.aux)[row * p.ld_aux + n]
                                   : bf2f(static_cast<const bf16*>(p.aux)[row * p.ld_aux + n]);
  if (fl & LRCE_EPI_RESID) e.res = static_cast<const float*>(p.aux)[row * p.ld_aux + n];
  if (fl & (LRCE_EPI_ATOMIC | LRCE_EPI_ACCUM)) e.acc = static_cast<const float*>(p.c)[row * p.ldc + n];
  return e;
}

__device__ __forceinline__ void sk_epilogue(const SkinnyP& p, float x, int m, int n, const SkPre& e) {
  const int fl = p.flags;
  const long long row = m;
  x = x * p.alpha + e.bias;
  x *= (n < p.scale_cols) ? p.scale_val : 1.f;
  if (fl & LRCE_EPI_GELU) {
    if (fl & LRCE_EPI_AUX_OUT) {
      if (fl & LRCE_EPI_AUX_F32) reinterpret_cast<float*>(p.aux_out)[row * p.ld_aux_out + n] = x;
      else p.aux_out[row * p.ld_aux_out + n] = f2bf(x);
    }
    x = gelu_f(x);
  }
  if (fl & LRCE_EPI_DGELU) x *= gelu_grad_f(e.dg);
  if (p.row_scale) x *= p.row_scale[m / p.rows_per_scale];
  if (p.drop_p > 0.f)   // same mask as lrce_dropout on the contiguous [m][n] result
    x = lrce_uniform(lrce_seed(p.drop_seed, p.rng_off), ((long long)m * p.n + n) / p.drop_group) >= p.drop_p
            ? x / (1.0f - p.drop_p) : 0.f;
  x += e.res;
  if (fl & (LRCE_EPI_ATOMIC | LRCE_EPI_ACCUM)) {
    static_cast<float*>(p.c)[row * p.ldc + n] = e.acc + x;   // one owner per element: a plain RMW suffices
  } else if (fl & LRCE_EPI_OUT_F32) {
    static_cast<float*>(p.c)[row * p.ldc + n] = x;
    if (fl & LRCE_EPI_OUT_BOTH) p.aux_out[row * p.ld_aux_out + n] = f2bf(x);
  } else {
    static_cast<bf16*>(p.c)[row * p.ldc + n] = f2bf(x);
  }
}

// C[m][n] = sum_k A[m][k] * B(k, n); B_KM: B stored [n][k] (forward, W), else [k][n] (dX = dY W).
// 8 waves split the reduction; each wave issues all loads of a trip of TS k-steps (16 deep) before
// its MFMAs, so a whole 768-deep reduction is one memory round trip per wave.
// (8 waves: a 16-wave variant measured slower on the 3072-deep decoder linear2, 18.8 vs ~9 us)
// Split-K (gridDim.y = KS > 1): workgroup (tile, ks) reduces k in [ks*kspan, (ks+1)*kspan), stores
// its 16 x 16*MT partial to `part`, and the LAST workgroup of the tile to arrive (device-scope
// counter, reset by that workgroup: graph-replay safe) sums the KS partials in ks order and runs
// the epilogue — so nonlinear epilogues (GELU, dGELU, residual) still see the full sum, and the
// result does not depend on arrival order.  Narrow-N decoder linears (N = 768 -> 48 tiles) get
// 3-4x the workgroups, deep ones (K = 3072) a quarter of the reduction per workgroup.
template <int MT, bool B_KM, int SK_WAVES, bool BH>
__global__ void __launch_bounds__(SK_WAVES * 64) skinny_kernel(SkinnyP p, float* __restrict__ part,
                                                               unsigned* __restrict__ counters, int kspan) {
  constexpr int TS = MT <= 2 ? 8 : 4;
  constexpr int NPART = SK_WAVES * 64 / 256;   // 256-thread groups finishing the m-tiles
  __shared__ float red[SK_WAVES][MT][16][17];
  __shared__ unsigned last_flag;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int col = lane & 15, grp = lane >> 4;
  const int n0 = blockIdx.x * 16;
  const int n = n0 + col;
  const bool n_ok = n < p.n;
  const int nc = n_ok ? n : 0;
  const int ks = blockIdx.y, KS = gridDim.y;
  const int kbase = ks * kspan, kend = min(p.k, kbase + kspan);
  int kchunk = (kend - kbase + SK_WAVES - 1) / SK_WAVES;
  kchunk = (kchunk + 15) & ~15;
  const int kb = kbase + wave * kchunk, ke = min(kend, kb + kchunk);
  const int ml = (threadIdx.x >> 4) & 15, nl = threadIdx.x & 15, grp256 = threadIdx.x >> 8;
  SkPre pre[MT];
#pragma unroll
  for (int t = 0; t < MT; ++t)
    pre[t] = (t % NPART == grp256) ? sk_prefetch(p, t * 16 + ml, n0 + nl) : SkPre{0.f, 1.f, 0.f, 0.f};
  f32x4 acc[MT];
#pragma unroll
  for (int t = 0; t < MT; ++t) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
  for (int k = kb; k < ke; k += 16 * TS) {
    float4 bv[TS], av[TS][MT];
#pragma unroll
    for (int u = 0; u < TS; ++u) {
      const int kk = k + 16 * u + 4 * grp;
      const bool k_ok = kk < ke;           // k % 4 == 0: a float4 is all in or all out
      const int kc = k_ok ? kk : 0;
      bv[u] = ld_b4<B_KM, BH>(p.b, p.ldb, nc, kc);
      if (!(k_ok && n_ok)) bv[u] = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
      for (int t = 0; t < MT; ++t) {
        const int m = t * 16 + col;
        const bool ok = k_ok && m < p.m;
        av[u][t] = *reinterpret_cast<const float4*>(p.a + (long long)(ok ? m : 0) * p.lda + kc);
        if (!ok) av[u][t] = make_float4(0.f, 0.f, 0.f, 0.f);
      }
    }
#pragma unroll
    for (int u = 0; u < TS; ++u)
#pragma unroll
      for (int t = 0; t < MT; ++t) {
        acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[u][t].x, bv[u].x, acc[t], 0, 0, 0);
        acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[u][t].y, bv[u].y, acc[t], 0, 0, 0);
        acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[u][t].z, bv[u].z, acc[t], 0, 0, 0);
        acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[u][t].w, bv[u].w, acc[t], 0, 0, 0);
      }
  }
#pragma unroll
  for (int t = 0; t < MT; ++t)
#pragma unroll
    for (int r = 0; r < 4; ++r) red[wave][t][grp * 4 + r][col] = acc[t][r];
  __syncthreads();
  if (KS == 1) {
#pragma unroll
    for (int t = 0; t < MT; ++t) {
      if (t % NPART != grp256) continue;   // 256-thread group g finishes m-tiles t = g (mod NPART)
      const int m = t * 16 + ml, nn = n0 + nl;
      if (m < p.m && nn < p.n) {
        float x = 0.f;
#pragma unroll
        for (int w = 0; w < SK_WAVES; ++w) x += red[w][t][ml][nl];
        sk_epilogue(p, x, m, nn, pre[t]);
      }
    }
    return;
  }
  // split-K: partial tile -> part[tile][ks][t][16][16]; the last arriver reduces + epilogue
  float* mine = part + ((long long)blockIdx.x * KS + ks) * (MT * 256);
#pragma unroll
  for (int t = 0; t < MT; ++t) {
    if (t % NPART != grp256) continue;
    float x = 0.f;
#pragma unroll
    for (int w = 0; w < SK_WAVES; ++w) x += red[w][t][ml][nl];
    // Hand-off protocol (MI355X_MICROARCH.md "Valid forms", first row of the sc1 hand-off table, in
    // place of a release/acquire pair): every partial is an agent-scope relaxed store (global_store
    // ... sc1, write-through past this XCD's L2), every storing wave drains it with s_waitcnt
    // vmcnt(0), a workgroup barrier follows, then ONE lane's agent-scope atomic add signals; the
    // block whose add returns KS-1 reduces, reading EVERY partial with agent-scope relaxed loads
    // (global_load ... sc1, L2 bypass) after the barrier that publishes last_flag.  All four
    // conditions of that row hold, so no buffer_wbl2 / buffer_inv (~1.7 us each per launch on these
    // latency-bound decoder linears) is needed.  tests/test_ops_gpu.py
    // test_gemm_f32_splitk_repeatable re-runs the split launches and checks every output word.
    __hip_atomic_store(mine + t * 256 + ml * 16 + nl, x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0)
    last_flag = __hip_atomic_fetch_add(&counters[blockIdx.x], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) ==
                (unsigned)(KS - 1);
  __syncthreads();
  if (!last_flag) return;
#pragma unroll
  for (int t = 0; t < MT; ++t) {
    if (t % NPART != grp256) continue;
    const int m = t * 16 + ml, nn = n0 + nl;
    float x = 0.f;
    float* src = part + (long long)blockIdx.x * KS * (MT * 256) + t * 256 + ml * 16 + nl;
    for (int j = 0; j < KS; ++j) x += __hip_atomic_load(src + j * (MT * 256), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (m < p.m && nn < p.n) sk_epilogue(p, x, m, nn, pre[t]);
  }
  if (threadIdx.x == 0)   // ready for the next launch / graph replay
    __hip_atomic_store(&counters[blockIdx.x], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// C[m][n] (+)= alpha * sum_{r < R} A[r][m] * B[r][n] with R <= 256 (dW of a skinny linear):
// one thread per 4 consecutive columns, the R-term outer-product sum in registers, one RMW.  The
// C read is issued first and the A/B rows are fetched 8 reduction steps per batch, so a thread has
// ~17 loads in flight instead of one dependent round trip per step.
__global__ void __launch_bounds__(256) outer_kernel(SkinnyP p) {
  constexpr int U = 8;
  const long long q = (long long)blockIdx.x * 256 + threadIdx.x;
  const int nq = p.n >> 2;
  if (q >= (long long)p.m * nq) return;
  const int m = (int)(q / nq), n = (int)(q % nq) * 4;
  float4* cp = reinterpret_cast<float4*>(static_cast<float*>(p.c) + (long long)m * p.ldc + n);
  const bool acc_c = p.flags & (LRCE_EPI_ATOMIC | LRCE_EPI_ACCUM);
  const float4 o = acc_c ? *cp : make_float4(0.f, 0.f, 0.f, 0.f);
  float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
  float asum = 0.f;
  const float* ap = p.a + m;
  const float* bp = static_cast<const float*>(p.b) + n;
  int r = 0;
  for (; r + U <= p.k; r += U) {
    float av[U];
    float4 bv[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      av[u] = ap[(long long)(r + u) * p.lda];
      bv[u] = *reinterpret_cast<const float4*>(bp + (long long)(r + u) * p.ldb);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      asum += av[u];
      acc.x = fmaf(av[u], bv[u].x, acc.x); acc.y = fmaf(av[u], bv[u].y, acc.y);
      acc.z = fmaf(av[u], bv[u].z, acc.z); acc.w = fmaf(av[u], bv[u].w, acc.w);
    }
  }
  for (; r < p.k; ++r) {
    const float av = ap[(long long)r * p.lda];
    asum += av;
    const float4 bv = *reinterpret_cast<const float4*>(bp + (long long)r * p.ldb);
    acc.x = fmaf(av, bv.x, acc.x); acc.y = fmaf(av, bv.y, acc.y); acc.z = fmaf(av, bv.z, acc.z); acc.w = fmaf(av, bv.w, acc.w);
  }
  acc.x = fmaf(acc.x, p.alpha, o.x); acc.y = fmaf(acc.y, p.alpha, o.y);
  acc.z = fmaf(acc.z, p.alpha, o.z); acc.w = fmaf(acc.w, p.alpha, o.w);
  *cp = acc;
  if ((p.flags & LRCE_EPI_BIAS_GRAD) && n == 0) p.bias_grad[m] += p.alpha * asum;   // db (one owner per m)
}

// The same outer-product sum with an MR x 4 block of C per thread (MR consecutive rows m, 4 columns
// n): per reduction step one A vector (MR rows) and one B float4 feed 4 MR FMAs, so the X rows,
// which every output row shares, are pulled from L2 MR times less often than by outer_kernel (one
// float4 of B per 4 outputs: at 3072 x 768 x R=30 that re-read, not the 9.4 MB read-modify-write of
// C, set the time).  Workgroup = 16 x 16 threads over a (16 MR) x 64 tile; lanes run along n, so a
// wave instruction touches MR x 4 rows of 256 contiguous bytes.  All U steps of a batch are issued
// before any is consumed.
template <int MR>
__global__ void __launch_bounds__(256) outer_tile_kernel(SkinnyP p) {
  constexpr int U = 8;
  const int tn = threadIdx.x & 15, tm = threadIdx.x >> 4;
  const int n = blockIdx.x * 64 + tn * 4;
  const int m = (blockIdx.y * 16 + tm) * MR;
  if (n >= p.n || m >= p.m) return;
  const bool acc_c = p.flags & (LRCE_EPI_ATOMIC | LRCE_EPI_ACCUM);
  float* cbase = static_cast<float*>(p.c) + (long long)m * p.ldc + n;
  float4 o[MR];
#pragma unroll
  for (int i = 0; i < MR; ++i)
    o[i] = acc_c ? *reinterpret_cast<const float4*>(cbase + (long long)i * p.ldc) : make_float4(0.f, 0.f, 0.f, 0.f);
  float4 acc[MR];
  float asum[MR];
#pragma unroll
  for (int i = 0; i < MR; ++i) { acc[i] = make_float4(0.f, 0.f, 0.f, 0.f); asum[i] = 0.f; }
  const float* ap = p.a + m;
  const float* bp = static_cast<const float*>(p.b) + n;
  auto lda_vec = [&](int r, float (&av)[MR]) {
    if constexpr (MR == 4) {
      const float4 t = *reinterpret_cast<const float4*>(ap + (long long)r * p.lda);
      av[0] = t.x; av[1] = t.y; av[2] = t.z; av[3] = t.w;
    } else {
      const float2 t = *reinterpret_cast<const float2*>(ap + (long long)r * p.lda);
      av[0] = t.x; av[1] = t.y;
    }
  };
  auto step = [&](const float (&av)[MR], const float4& bv) {
#pragma unroll
    for (int i = 0; i < MR; ++i) {
      asum[i] += av[i];
      acc[i].x = fmaf(av[i], bv.x, acc[i].x); acc[i].y = fmaf(av[i], bv.y, acc[i].y);
      acc[i].z = fmaf(av[i], bv.z, acc[i].z); acc[i].w = fmaf(av[i], bv.w, acc[i].w);
    }
  };
  int r = 0;
  for (; r + U <= p.k; r += U) {
    float av[U][MR];
    float4 bv[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      lda_vec(r + u, av[u]);
      bv[u] = *reinterpret_cast<const float4*>(bp + (long long)(r + u) * p.ldb);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) step(av[u], bv[u]);
  }
  for (; r < p.k; ++r) {
    float av[MR];
    lda_vec(r, av);
    step(av, *reinterpret_cast<const float4*>(bp + (long long)r * p.ldb));
  }
#pragma unroll
  for (int i = 0; i < MR; ++i) {
    if (m + i >= p.m) break;
    float4 w;
    w.x = fmaf(acc[i].x, p.alpha, o[i].x); w.y = fmaf(acc[i].y, p.alpha, o[i].y);
    w.z = fmaf(acc[i].z, p.alpha, o[i].z); w.w = fmaf(acc[i].w, p.alpha, o[i].w);
    *reinterpret_cast<float4*>(cbase + (long long)i * p.ldc) = w;
    if ((p.flags & LRCE_EPI_BIAS_GRAD) && n == 0) p.bias_grad[m + i] += p.alpha * asum[i];   // db (one owner per m)
  }
}

// ---------------------------------------------------------------------------------------------
// Skinny exact-f32 linear with a LayerNorm prologue on A (lrce_gemm_ln).  The recurrent decoder's
// post-norm LayerNorms (nn.TransformerDecoderLayer norm1..3, fusionv3.py:8-17) are folded into the
// GEMM that consumes their output: every workgroup reads whole A rows anyway (K = the LN width), so
// it computes the row statistics itself (two-pass mean / variance, 8-wave LDS reduction) and
// normalises in registers before its MFMAs; one launch instead of LayerNorm + GEMM.
//   PRO = 1 (forward):  A = x (pre-norm), the GEMM consumes y = (x - mean) rstd gamma + beta; mean /
//                       rstd [m] written by workgroup 0, y materialised (optional) by column slices.
//   PRO = 2 (backward): A = dy (gradient of the LN output), x = pre-norm rows, mean / rstd read:
//                       dx = rstd (g - mean(g) - xh mean(g xh)), g = dy gamma, xh = (x - mean) rstd;
//                       dgamma += colsum(dy xh), dbeta += colsum(dy); the GEMM consumes
//                       dropout_bwd(dx) (the forward dropout in front of the LN's residual add);
//                       dx and the dropped dx materialised (optional).
// Column slices of 16 are owned by workgroup (k / 16) % grid: the owner writes the materialised
// values and the gamma / beta gradient of its slice (one writer per element, no atomics).
// K = 8 waves x 16 x nu (nu <= 8): the whole row of A sits in the workgroup's registers.
struct LnP {
  const float* gamma;
  const float* beta;
  float eps;
  const float* x;
  long long ld_x;
  float* mean;
  float* rstd;
  float* y_out;
  long long ld_y;
  float* y2_out;
  long long ld_y2;
  float* dgamma;
  float* dbeta;
  float drop_p;
  int drop_group;
  uint64_t drop_seed;
};

constexpr int LN_W = 8, LN_US = 8;

template <int MT, bool B_KM, int PRO, bool BH>
__global__ void __launch_bounds__(LN_W * 64) skinny_ln_kernel(SkinnyP p, LnP q) {
  __shared__ float red[LN_W][MT][16][17];
  __shared__ float rsum[2][LN_W][MT * 16];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int col = lane & 15, grp = lane >> 4;
  const int n0 = blockIdx.x * 16;
  const int n = n0 + col;
  const bool n_ok = n < p.n;
  const int nc = n_ok ? n : 0;
  const int kw = p.k / LN_W, nu = kw >> 4;
  const int kb = wave * kw;
  const float inv_k = 1.0f / (float)p.k;
  const int ml = (threadIdx.x >> 4) & 15, nl = threadIdx.x & 15, grp256 = threadIdx.x >> 8;
  SkPre pre[MT];
#pragma unroll
  for (int t = 0; t < MT; ++t)
    pre[t] = (t % 2 == grp256) ? sk_prefetch(p, t * 16 + ml, n0 + nl) : SkPre{0.f, 1.f, 0.f, 0.f};
  // every global load up front: the weight slab, the A rows, gamma / beta, (PRO 2) x rows + stats
  float4 bv[LN_US], av[LN_US][MT], gv[LN_US], ev[LN_US];
  float4 xv[PRO == 2 ? LN_US : 1][MT];
  float mu[MT], rs[MT];
#pragma unroll
  for (int u = 0; u < LN_US; ++u) {
    if (u >= nu) break;
    const int k = kb + 16 * u + 4 * grp;
    bv[u] = ld_b4<B_KM, BH>(p.b, p.ldb, nc, k);
    if (!n_ok) bv[u] = make_float4(0.f, 0.f, 0.f, 0.f);
    gv[u] = *reinterpret_cast<const float4*>(q.gamma + k);
    if (PRO == 1) ev[u] = *reinterpret_cast<const float4*>(q.beta + k);
#pragma unroll
    for (int t = 0; t < MT; ++t) {
      const int m = t * 16 + col;
      const bool ok = m < p.m;
      av[u][t] = ok ? *reinterpret_cast<const float4*>(p.a + (long long)m * p.lda + k) : make_float4(0.f, 0.f, 0.f, 0.f);
      if (PRO == 2)
        xv[u][t] = ok ? *reinterpret_cast<const float4*>(q.x + (long long)m * q.ld_x + k) : make_float4(0.f, 0.f, 0.f, 0.f);
    }
  }
  if (PRO == 2) {
#pragma unroll
    for (int t = 0; t < MT; ++t) {
      const int m = min(t * 16 + col, p.m - 1);
      mu[t] = q.mean[m];
      rs[t] = q.rstd[m];
    }
  }
  // sum of (s1, s2) over the row: in-lane over the wave's k, across the 4 k-groups, across waves
  auto row_reduce = [&](float (&s1)[MT], float (&s2)[MT], bool two) {
#pragma unroll
    for (int t = 0; t < MT; ++t) {
      s1[t] += __shfl_xor(s1[t], 16, 64);
      s1[t] += __shfl_xor(s1[t], 32, 64);
      if (two) {
        s2[t] += __shfl_xor(s2[t], 16, 64);
        s2[t] += __shfl_xor(s2[t], 32, 64);
      }
      if (grp == 0) {
        rsum[0][wave][t * 16 + col] = s1[t];
        if (two) rsum[1][wave][t * 16 + col] = s2[t];
      }
    }
    __syncthreads();
#pragma unroll
    for (int t = 0; t < MT; ++t) {
      float a = 0.f, b = 0.f;
#pragma unroll
      for (int w = 0; w < LN_W; ++w) {
        a += rsum[0][w][t * 16 + col];
        if (two) b += rsum[1][w][t * 16 + col];
      }
      s1[t] = a;
      s2[t] = b;
    }
    __syncthreads();
  };
  const int slice0 = kb >> 4;   // this wave's first 16-column slice
  auto owns = [&](int u) { return (slice0 + u) % (int)gridDim.x == (int)blockIdx.x; };
  if (PRO == 1) {
    float s1[MT], s2[MT];
#pragma unroll
    for (int t = 0; t < MT; ++t) {
      s1[t] = 0.f;
      s2[t] = 0.f;
#pragma unroll
      for (int u = 0; u < LN_US; ++u) {
        if (u >= nu) break;
        s1[t] += (av[u][t].x + av[u][t].y) + (av[u][t].z + av[u][t].w);
      }
    }
    row_reduce(s1, s2, false);
#pragma unroll
    for (int t = 0; t < MT; ++t) {
      mu[t] = s1[t] * inv_k;
      s1[t] = 0.f;
#pragma unroll
      for (int u = 0; u < LN_US; ++u) {
        if (u >= nu) break;
        const float4 d = make_float4(av[u][t].x - mu[t], av[u][t].y - mu[t], av[u][t].z - mu[t], av[u][t].w - mu[t]);
        s1[t] += (d.x * d.x + d.y * d.y) + (d.z * d.z + d.w * d.w);
      }
    }
    row_reduce(s1, s2, false);
#pragma unroll
    for (int t = 0; t < MT; ++t) {
      rs[t] = rsqrtf(s1[t] * inv_k + q.eps);
      const int m = t * 16 + col;
      if (blockIdx.x == 0 && wave == 0 && grp == 0 && m < p.m) {
        if (q.mean) q.mean[m] = mu[t];
        if (q.rstd) q.rstd[m] = rs[t];
      }
    }
#pragma unroll
    for (int u = 0; u < LN_US; ++u) {
      if (u >= nu) break;
      const bool own = q.y_out && owns(u);
#pragma unroll
      for (int t = 0; t < MT; ++t) {
        float4& a = av[u][t];
        a.x = (a.x - mu[t]) * rs[t] * gv[u].x + ev[u].x;
        a.y = (a.y - mu[t]) * rs[t] * gv[u].y + ev[u].y;
        a.z = (a.z - mu[t]) * rs[t] * gv[u].z + ev[u].z;
        a.w = (a.w - mu[t]) * rs[t] * gv[u].w + ev[u].w;
        const int m = t * 16 + col;
        if (own && m < p.m) *reinterpret_cast<float4*>(q.y_out + (long long)m * q.ld_y + kb + 16 * u + 4 * grp) = a;
        if (m >= p.m) a = make_float4(0.f, 0.f, 0.f, 0.f);
      }
    }
  }
  if (PRO == 2) {
    float s1[MT], s2[MT];
#pragma unroll
    for (int t = 0; t < MT; ++t) {
      s1[t] = 0.f;
      s2[t] = 0.f;
#pragma unroll
      for (int u = 0; u < LN_US; ++u) {
        if (u >= nu) break;
        // xv <- xh, and the gamma / beta gradient terms of the owned slice before dy is replaced
        float4& x = xv[u][t];
        x = make_float4((x.x - mu[t]) * rs[t], (x.y - mu[t]) * rs[t], (x.z - mu[t]) * rs[t], (x.w - mu[t]) * rs[t]);
        const float4 g = make_float4(av[u][t].x * gv[u].x, av[u][t].y * gv[u].y, av[u][t].z * gv[u].z, av[u][t].w * gv[u].w);
        s1[t] += (g.x + g.y) + (g.z + g.w);
        s2[t] += (g.x * x.x + g.y * x.y) + (g.z * x.z + g.w * x.w);
      }
    }
    // dgamma / dbeta of the owned slice: column sums over the rows (16 lanes x MT tiles)
#pragma unroll
    for (int u = 0; u < LN_US; ++u) {
      if (u >= nu) break;
      if (!(q.dgamma && owns(u))) continue;
      float4 dg = make_float4(0.f, 0.f, 0.f, 0.f), db = dg;
#pragma unroll
      for (int t = 0; t < MT; ++t) {   // rows >= m hold dy = 0
        const float4 d = av[u][t], x = xv[u][t];
        dg.x += d.x * x.x; dg.y += d.y * x.y; dg.z += d.z * x.z; dg.w += d.w * x.w;
        db.x += d.x; db.y += d.y; db.z += d.z; db.w += d.w;
      }
#pragma unroll
      for (int o = 1; o < 16; o <<= 1) {
        dg.x += __shfl_xor(dg.x, o, 64); dg.y += __shfl_xor(dg.y, o, 64);
        dg.z += __shfl_xor(dg.z, o, 64); dg.w += __shfl_xor(dg.w, o, 64);
        db.x += __shfl_xor(db.x, o, 64); db.y += __shfl_xor(db.y, o, 64);
        db.z += __shfl_xor(db.z, o, 64); db.w += __shfl_xor(db.w, o, 64);
      }
      if (col == 0) {
        const int k = kb + 16 * u + 4 * grp;
        float4* pg = reinterpret_cast<float4*>(q.dgamma + k);
        float4* pb = reinterpret_cast<float4*>(q.dbeta + k);
        float4 og = *pg, ob = *pb;
        og.x += dg.x; og.y += dg.y; og.z += dg.z; og.w += dg.w;
        ob.x += db.x; ob.y += db.y; ob.z += db.z; ob.w += db.w;
        *pg = og;
        *pb = ob;
      }
    }
    row_reduce(s1, s2, true);
    const uint64_t seed = lrce_seed(q.drop_seed, p.rng_off);
    const float keep_div = 1.0f - q.drop_p;   // x / (1 - p): the bits of lrce_dropout_bwd
#pragma unroll
    for (int u = 0; u < LN_US; ++u) {
      if (u >= nu) break;
      const bool own = owns(u);
      const int k = kb + 16 * u + 4 * grp;
#pragma unroll
      for (int t = 0; t < MT; ++t) {
        const float mg = s1[t] * inv_k, mgx = s2[t] * inv_k;
        const int m = t * 16 + col;
        float4& a = av[u][t];
        const float4 x = xv[u][t];
        a = make_float4(rs[t] * (a.x * gv[u].x - mg - x.x * mgx), rs[t] * (a.y * gv[u].y - mg - x.y * mgx),
                        rs[t] * (a.z * gv[u].z - mg - x.z * mgx), rs[t] * (a.w * gv[u].w - mg - x.w * mgx));
        if (m >= p.m) a = make_float4(0.f, 0.f, 0.f, 0.f);
        if (own && q.y_out && m < p.m) *reinterpret_cast<float4*>(q.y_out + (long long)m * q.ld_y + k) = a;
        if (q.drop_p > 0.f) {
          const long long e = (long long)m * p.k + k;   // k % 4 == 0, K % 4 == 0: one hash per float4
          float4 uu;
          if (q.drop_group == 1) uu = lrce_uniform4(seed, (uint64_t)e >> 2);
          else uu = make_float4(lrce_uniform(seed, (e + 0) / q.drop_group), lrce_uniform(seed, (e + 1) / q.drop_group),
                                lrce_uniform(seed, (e + 2) / q.drop_group), lrce_uniform(seed, (e + 3) / q.drop_group));
          a.x = uu.x >= q.drop_p ? a.x / keep_div : 0.f;
          a.y = uu.y >= q.drop_p ? a.y / keep_div : 0.f;
          a.z = uu.z >= q.drop_p ? a.z / keep_div : 0.f;
          a.w = uu.w >= q.drop_p ? a.w / keep_div : 0.f;
        }
        if (own && q.y2_out && m < p.m) *reinterpret_cast<float4*>(q.y2_out + (long long)m * q.ld_y2 + k) = a;
      }
    }
  }
  f32x4 acc[MT];
#pragma unroll
  for (int t = 0; t < MT; ++t) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int u = 0; u < LN_US; ++u) {
    if (u >= nu) break;
#pragma unroll
    for (int t = 0; t < MT; ++t) {
      acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[u][t].x, bv[u].x, acc[t], 0, 0, 0);
      acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[u][t].y, bv[u].y, acc[t], 0, 0, 0);
      acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[u][t].z, bv[u].z, acc[t], 0, 0, 0);
      acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[u][t].w, bv[u].w, acc[t], 0, 0, 0);
    }
  }
#pragma unroll
  for (int t = 0; t < MT; ++t)
#pragma unroll
    for (int r = 0; r < 4; ++r) red[wave][t][grp * 4 + r][col] = acc[t][r];
  __syncthreads();
#pragma unroll
  for (int t = 0; t < MT; ++t) {
    if (t % 2 != grp256) continue;
    const int m = t * 16 + ml, nn = n0 + nl;
    if (m < p.m && nn < p.n) {
      float x = 0.f;
#pragma unroll
      for (int w = 0; w < LN_W; ++w) x += red[w][t][ml][nl];
      sk_epilogue(p, x, m, nn, pre[t]);
    }
  }
}

}  // namespace

namespace {
// Per-device split-K scratch of the skinny kernel: partial tiles + zero-initialised arrival
// counters (self-resetting).  Allocated once, outside stream capture; one stream per device uses it
// at a time (kernels on one stream serialise), so reuse across launches is race-free.
struct SkinnySplitWs {
  float* part = nullptr;
  unsigned* counters = nullptr;
  long long part_elems = 0;
  int n_counters = 0;
};
constexpr long long SK_PART_ELEMS = 192LL * 4 * 4 * 256;   // tiles x KS x MT x 256 (max shapes routed here)
constexpr int SK_COUNTERS = 4096;

SkinnySplitWs* skinny_split_ws(hipStream_t st, int tiles, int ks, int mt) {
  static SkinnySplitWs per_dev[64];
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return nullptr;
  SkinnySplitWs& w = per_dev[dev];
  if (!w.part) {
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    if (hipStreamIsCapturing(st, &cs) != hipSuccess || cs != hipStreamCaptureStatusNone) return nullptr;
    if (hipMalloc(&w.part, SK_PART_ELEMS * sizeof(float)) != hipSuccess) { w.part = nullptr; return nullptr; }
    if (hipMalloc(&w.counters, SK_COUNTERS * sizeof(unsigned)) != hipSuccess ||
        hipMemset(w.counters, 0, SK_COUNTERS * sizeof(unsigned)) != hipSuccess ||
        hipDeviceSynchronize() != hipSuccess) {
      (void)hipFree(w.part);
      w.part = nullptr;
      return nullptr;
    }
    w.part_elems = SK_PART_ELEMS;
    w.n_counters = SK_COUNTERS;
  }
  if ((long long)tiles * ks * mt * 256 > w.part_elems || tiles > w.n_counters) return nullptr;
  return &w;
}
}  // namespace

// the dW shape the outer-product kernel takes: A M-major, B N-major, reduction <= 256 rows
bool lrce_gemm_f32_outer_ok(const LrceGemmDesc* d) {
  return d->b_f32 == 1 && d->a_f32 && !d->a_kmajor && !d->b_kmajor && d->k <= 256 && (d->n % 4) == 0 && (d->ldc % 4) == 0 &&
         (d->ldb % 4) == 0 && d->batch == 1 && !d->a_map && !d->c_map && !d->a_row_scale && d->split_k <= 1 &&
         (d->flags & ~(LRCE_EPI_ATOMIC | LRCE_EPI_ACCUM | LRCE_EPI_OUT_F32 | LRCE_EPI_BIAS_GRAD)) == 0 &&
         (d->flags & (LRCE_EPI_ATOMIC | LRCE_EPI_ACCUM | LRCE_EPI_OUT_F32)) && !d->row_scale && d->scale_cols == 0 &&
         (reinterpret_cast<uintptr_t>(d->c) & 15) == 0 && (reinterpret_cast<uintptr_t>(d->b) & 15) == 0;
}

int lrce_gemm_f32(const LrceGemmDesc* d, void* stream) {
  if (!d->a_f32) return lrce_fail(LRCE_E_ARG, "gemm(f32 B): A must be f32 too");
  if (d->batch != 1) return lrce_fail(LRCE_E_ARG, "gemm(f32 B): batch must be 1");
  const bool bh = d->b_f32 == 2;   // fp16 B (weights), f32 A and compute: skinny path only
  if (d->a_kmajor ? (d->k % 4) : (d->m % 4)) return lrce_fail(LRCE_E_ARG, "gemm(f32): A contiguous dim %% 4 != 0");
  if (d->b_kmajor ? (d->k % 4) : (d->n % 4)) return lrce_fail(LRCE_E_ARG, "gemm(f32): B contiguous dim %% 4 != 0");
  if ((d->lda % 4) || (d->ldb % 4)) return lrce_fail(LRCE_E_ARG, "gemm(f32): lda/ldb %% 4 != 0");
  const bool plain = !d->a_map && !d->c_map && !d->a_row_scale && d->split_k <= 1;
  hipStream_t st = static_cast<hipStream_t>(stream);
  if (plain) {
    SkinnyP q;
    q.a = static_cast<const float*>(d->a); q.b = d->b; q.c = d->c;
    q.lda = d->lda; q.ldb = d->ldb; q.ldc = d->ldc;
    q.m = d->m; q.n = d->n; q.k = d->k; q.flags = d->flags; q.bias = d->bias;
    q.aux = d->aux; q.ld_aux = d->ld_aux; q.aux_out = static_cast<bf16*>(d->aux_out); q.ld_aux_out = d->ld_aux_out;
    q.alpha = d->alpha; q.row_scale = d->row_scale; q.rows_per_scale = d->rows_per_scale > 0 ? d->rows_per_scale : 1;
    q.scale_cols = d->scale_cols; q.scale_val = d->scale_val;
    q.bias_grad = const_cast<float*>(d->bias);
    q.drop_p = d->drop_p; q.drop_group = d->drop_group > 0 ? d->drop_group : 1; q.drop_seed = d->drop_seed;
    q.rng_off = lrce_rng_offset();
    const bool outer_ok = !bh && lrce_gemm_f32_outer_ok(d) && d->drop_p <= 0.f;
    if (outer_ok) {
      // MR x 4 per thread when the A rows allow vector loads: 4 while that still gives >= 512
      // workgroups, else 2 (a 768 x 768 dW: 288 workgroups)
      const bool avec = (reinterpret_cast<uintptr_t>(d->a) & 15) == 0 && d->lda % 4 == 0;
      const long long tiles64 = (long long)((d->n + 63) / 64) * ((d->m + 63) / 64);
      if (avec && d->m % 4 == 0 && tiles64 >= 512) {
        outer_tile_kernel<4><<<dim3((unsigned)((d->n + 63) / 64), (unsigned)((d->m + 63) / 64)), 256, 0, st>>>(q);
      } else if (avec && d->m % 2 == 0) {
        outer_tile_kernel<2><<<dim3((unsigned)((d->n + 63) / 64), (unsigned)((d->m + 31) / 32)), 256, 0, st>>>(q);
      } else {
        const long long work = (long long)d->m * (d->n / 4);
        outer_kernel<<<(unsigned)((work + 255) / 256), 256, 0, st>>>(q);
      }
      return lrce_check_launch("gemm_f32(outer)");
    }
    if (d->flags & LRCE_EPI_BIAS_GRAD) return lrce_fail(LRCE_E_ARG, "gemm(f32): internal: bias grad on a fused path");
    if (d->a_kmajor && d->m <= 64 && (reinterpret_cast<uintptr_t>(d->a) & 15) == 0 &&
        (!d->b_kmajor || (reinterpret_cast<uintptr_t>(d->b) & (bh ? 7 : 15)) == 0)) {
      const int mt = (d->m + 15) / 16;
      const int tiles = (d->n + 15) / 16;
      // split K for deep reductions (K >= 2048: the decoder FFN linear2 / linear1-dX) while the grid is under
      // ~192 workgroups (A/B on the full step: splitting the K = 768 linears too cost 0.4 %, K >= 2048 gained 1.4 %)
      int ks = 1;
      SkinnySplitWs* ws = nullptr;
      if (tiles < 192 && d->k >= 2048) {
        ks = std::min(std::min(4, d->k / 256), std::max(1, 192 / tiles));
        if (ks > 1 && !(ws = skinny_split_ws(st, tiles, ks, mt))) ks = 1;
      }
      int kspan = (d->k + ks - 1) / ks;
      kspan = (kspan + 15) & ~15;
      dim3 grid(tiles, ks);
      float* part = ws ? ws->part : nullptr;
      unsigned* ctr = ws ? ws->counters : nullptr;
#define LRCE_SK(MT)                                                                                       \
  if (bh) {                                                                                               \
    if (d->b_kmajor) skinny_kernel<MT, true, 8, true><<<grid, 8 * 64, 0, st>>>(q, part, ctr, kspan);      \
    else skinny_kernel<MT, false, 8, true><<<grid, 8 * 64, 0, st>>>(q, part, ctr, kspan);                 \
  } else {                                                                                                \
    if (d->b_kmajor) skinny_kernel<MT, true, 8, false><<<grid, 8 * 64, 0, st>>>(q, part, ctr, kspan);     \
    else skinny_kernel<MT, false, 8, false><<<grid, 8 * 64, 0, st>>>(q, part, ctr, kspan);                \
  }
      switch (mt) {
        case 1: LRCE_SK(1) break;
        case 2: LRCE_SK(2) break;
        case 3: LRCE_SK(3) break;
        default: LRCE_SK(4) break;
      }
#undef LRCE_SK
      return lrce_check_launch("gemm_f32(skinny)");
    }
  }
  if (d->drop_p > 0.f) return lrce_fail(LRCE_E_ARG, "gemm(f32): fused dropout needs the skinny path (K-major A, M <= 64)");
  if (bh) return lrce_fail(LRCE_E_ARG, "gemm(f32): fp16 B needs the skinny path (K-major 16-B aligned A, M <= 64)");
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

int lrce_gemm_ln(const LrceGemmDesc* d, const LrceLnPrologue* pro, void* stream) {
  if (!d || !pro) return lrce_fail(LRCE_E_ARG, "gemm_ln: null descriptor");
  if (pro->mode != 1 && pro->mode != 2) return lrce_fail(LRCE_E_ARG, "gemm_ln: mode %d", pro->mode);
  const bool bh = d->b_f32 == 2;
  if (!d->b_f32 || !d->a_f32 || !d->a_kmajor || d->batch != 1 || d->a_map || d->c_map || d->a_row_scale ||
      d->split_k > 1 || d->row_scale || (d->flags & (LRCE_EPI_ATOMIC | LRCE_EPI_BIAS_GRAD)))
    return lrce_fail(LRCE_E_ARG, "gemm_ln: f32 K-major A, f32 B, no maps / split / atomics");
  if (d->m < 1 || d->m > 64) return lrce_fail(LRCE_E_ARG, "gemm_ln: m=%d outside [1, 64]", d->m);
  if (d->k % (LN_W * 16) || d->k > LN_W * 16 * LN_US) return lrce_fail(LRCE_E_ARG, "gemm_ln: k=%d (multiple of 128, <= 1024)", d->k);
  if ((d->lda % 4) || (d->ldb % 4) || (reinterpret_cast<uintptr_t>(d->a) & 15) ||
      (reinterpret_cast<uintptr_t>(d->b) & (bh ? 7 : 15)))
    return lrce_fail(LRCE_E_ARG, "gemm_ln: A / B need 16-B (fp16 B: 8-B) alignment");
  if (!pro->gamma || (pro->mode == 1 && !pro->beta)) return lrce_fail(LRCE_E_ARG, "gemm_ln: gamma / beta");
  if (pro->mode == 2 && (!pro->x || !pro->mean || !pro->rstd || (pro->ld_x % 4) || (!pro->dgamma != !pro->dbeta)))
    return lrce_fail(LRCE_E_ARG, "gemm_ln: backward needs x (ld %% 4 == 0), mean, rstd; dgamma with dbeta");
  if ((pro->y_out && (pro->ld_y % 4)) || (pro->y2_out && (pro->ld_y2 % 4)))
    return lrce_fail(LRCE_E_ARG, "gemm_ln: materialised outputs need ld %% 4 == 0");
  const int tiles = (d->n + 15) / 16;
  SkinnyP q;
  q.a = static_cast<const float*>(d->a); q.b = d->b; q.c = d->c;
  q.lda = d->lda; q.ldb = d->ldb; q.ldc = d->ldc;
  q.m = d->m; q.n = d->n; q.k = d->k; q.flags = d->flags; q.bias = d->bias;
  q.aux = d->aux; q.ld_aux = d->ld_aux; q.aux_out = static_cast<bf16*>(d->aux_out); q.ld_aux_out = d->ld_aux_out;
  q.alpha = d->alpha; q.row_scale = nullptr; q.rows_per_scale = 1;
  q.scale_cols = d->scale_cols; q.scale_val = d->scale_val; q.bias_grad = nullptr;
  q.drop_p = d->drop_p; q.drop_group = d->drop_group > 0 ? d->drop_group : 1; q.drop_seed = d->drop_seed;
  q.rng_off = lrce_rng_offset();
  LnP l;
  l.gamma = pro->gamma; l.beta = pro->beta; l.eps = pro->eps; l.x = pro->x; l.ld_x = pro->ld_x;
  l.mean = pro->mean; l.rstd = pro->rstd; l.y_out = pro->y_out; l.ld_y = pro->ld_y; l.y2_out = pro->y2_out;
  l.ld_y2 = pro->ld_y2; l.dgamma = pro->dgamma; l.dbeta = pro->dbeta; l.drop_p = pro->drop_p;
  l.drop_group = pro->drop_group > 0 ? pro->drop_group : 1; l.drop_seed = pro->drop_seed;
  const int mt = (d->m + 15) / 16;
  hipStream_t st = static_cast<hipStream_t>(stream);
#define LRCE_SKLN(MT, PRO)                                                                         \
  if (bh) {                                                                                        \
    if (d->b_kmajor) skinny_ln_kernel<MT, true, PRO, true><<<tiles, LN_W * 64, 0, st>>>(q, l);     \
    else skinny_ln_kernel<MT, false, PRO, true><<<tiles, LN_W * 64, 0, st>>>(q, l);                \
  } else {                                                                                         \
    if (d->b_kmajor) skinny_ln_kernel<MT, true, PRO, false><<<tiles, LN_W * 64, 0, st>>>(q, l);    \
    else skinny_ln_kernel<MT, false, PRO, false><<<tiles, LN_W * 64, 0, st>>>(q, l);               \
  }
#define LRCE_SKLN_MT(PRO)                    \
  switch (mt) {                              \
    case 1: LRCE_SKLN(1, PRO) break;         \
    case 2: LRCE_SKLN(2, PRO) break;         \
    case 3: LRCE_SKLN(3, PRO) break;         \
    default: LRCE_SKLN(4, PRO) break;        \
  }
  if (pro->mode == 1) { LRCE_SKLN_MT(1) }
  else { LRCE_SKLN_MT(2) }
#undef LRCE_SKLN_MT
#undef LRCE_SKLN
  return lrce_check_launch("gemm_ln");
}
