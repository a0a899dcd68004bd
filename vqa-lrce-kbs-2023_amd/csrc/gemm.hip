// LDS-tiled bf16 MFMA GEMM for gfx950 with layout-flexible operands and fused epilogues.
//
// One kernel serves every linear layer of the LRCE path, forward and backward:
//   forward  Y = X W^T          A K-major (tokens x in),  B K-major (W [out][in])
//   dX       dX = dY W          A K-major (dY),           B N-major (W read as [k=out][n=in])
//   dW       dW = dY^T X        A M-major (dY, k=token),  B N-major (X, k=token)
// Tile 128x128x64, 256 threads (4 waves as 2x2, 64x64 per wave = 4x4 v_mfma_f32_16x16x32_bf16).
// Operands are staged global->registers->LDS (double buffered, one barrier per K tile).
// K-major tiles live in LDS as [row][64] with 16-B chunks XOR-swizzled by (row>>1)&7 and are
// read with ds_read_b128; M/N-major tiles live as [k][128] with 8-B units XOR-swizzled by a 3-bit
// function of k and are read with ds_read_b64_tr_b16 (hardware transpose), so no operand is
// ever transposed through HBM.
#include "common.h"
#include "lrce_capi.h"

namespace {

constexpr int BM = 128, BN = 128, BK = 64, NT = 256;

struct GemmP {
  const void* a;
  const bf16* b;
  void* c;
  long long lda, ldb, ldc, sa, sb, sc;
  int m, n, k, batch, split_k, k_chunk;
  int flags;
  const float* bias;
  const void* aux;
  long long ld_aux;
  bf16* aux_out;
  long long ld_aux_out;
  const int* a_map;
  const int* c_map;
  float alpha;
  int scale_cols;
  float scale_val;
  const float* row_scale;
  int rows_per_scale;
  const float* a_row_scale;
  int a_rows_per_scale;
  int tiles_m, tiles_n;
};

// ---- LDS addressing --------------------------------------------------------------------------
// K-major image: [128 rows][64 k] bf16, 128 B per row, 16-B chunk kc stored at kc ^ ((row>>1)&7).
__device__ __forceinline__ int km_off(int row, int kc) { return row * BK + ((kc ^ ((row >> 1) & 7)) << 3); }
// M-major image: [64 k][128 m] bf16, 256 B per row, 8-B unit u stored at u ^ (s(k)<<2).
__device__ __forceinline__ int mm_swz(int k) { return ((k & 3) | (((k >> 3) & 1) << 2)) << 2; }
__device__ __forceinline__ int mm_off(int k, int unit) { return k * 128 + ((unit ^ mm_swz(k)) << 2); }

// ---- global -> register staging ---------------------------------------------------------------
struct Stage {
  uint4 v[4];
};

template <bool KMAJ, bool F32>
__device__ __forceinline__ void load_tile(Stage& st, const void* base, long long ld, int rows_total, int kdim,
                                          int row0, int k0, const int* map, const float* rsc = nullptr, int rps = 1) {
  const int tid = threadIdx.x;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int c = tid + NT * i;
    int r, kk;  // r: index along the non-K dim inside the tile; kk: along K
    if (KMAJ) { r = c >> 3; kk = (c & 7) << 3; }
    else { kk = c >> 4; r = (c & 15) << 3; }
    const int gr = row0 + r, gk = k0 + kk;
    uint4 val = make_uint4(0, 0, 0, 0);
    bool ok = KMAJ ? (gr < rows_total && gk < kdim) : (gk < kdim && gr < rows_total);
    if (ok) {
      long long off;
      if (KMAJ) {
        const long long rr = map ? (long long)map[gr] : (long long)gr;
        off = rr * ld + gk;
      } else {
        const long long kr = map ? (long long)map[gk] : (long long)gk;
        off = kr * ld + gr;
      }
      if (F32) {
        const float4* p = reinterpret_cast<const float4*>(static_cast<const float*>(base) + off);
        float4 x0 = p[0], x1 = p[1];
        if (rsc) {
          if (KMAJ) {
            const float f = rsc[gr / rps];
            x0.x *= f; x0.y *= f; x0.z *= f; x0.w *= f; x1.x *= f; x1.y *= f; x1.z *= f; x1.w *= f;
          } else {
            const float f = rsc[gk / rps];
            x0.x *= f; x0.y *= f; x0.z *= f; x0.w *= f; x1.x *= f; x1.y *= f; x1.z *= f; x1.w *= f;
          }
        }
        bf16x8 t;
        t[0] = f2bf(x0.x); t[1] = f2bf(x0.y); t[2] = f2bf(x0.z); t[3] = f2bf(x0.w);
        t[4] = f2bf(x1.x); t[5] = f2bf(x1.y); t[6] = f2bf(x1.z); t[7] = f2bf(x1.w);
        val = *reinterpret_cast<uint4*>(&t);
      } else {
        val = *reinterpret_cast<const uint4*>(static_cast<const bf16*>(base) + off);
      }
    }
    st.v[i] = val;
  }
}

template <bool KMAJ>
__device__ __forceinline__ void store_tile(const Stage& st, bf16* lds) {
  const int tid = threadIdx.x;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int c = tid + NT * i;
    int off;
    if (KMAJ) off = km_off(c >> 3, c & 7);
    else off = mm_off(c >> 4, (c & 15) << 1);
    *reinterpret_cast<uint4*>(lds + off) = st.v[i];
  }
}

// Fragment of a 16(rows) x 32(k) operand block for v_mfma_f32_16x16x32_bf16:
// lane l holds [row = r0 + (l&15)][k = ks*32 + 8*(l>>4) + j], j = 0..7.
template <bool KMAJ>
__device__ __forceinline__ bf16x8 read_frag(const bf16* lds, int r0, int ks, int lane) {
  if (KMAJ) {
    const int row = r0 + (lane & 15);
    const int kc = ks * 4 + (lane >> 4);
    return *reinterpret_cast<const bf16x8*>(lds + km_off(row, kc));
  } else {
    const int g = lane >> 4, i = lane & 15, q = i >> 2, p = i & 3;
    const int unit = (r0 >> 2) + p;
    bf16x8 out;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int k = ks * 32 + 8 * g + 4 * h + q;
      const LRCE_LDS s16x4* src = (const LRCE_LDS s16x4*)(lds + mm_off(k, unit));
      s16x4 v = __builtin_amdgcn_ds_read_tr16_b64_v4i16(const_cast<LRCE_LDS s16x4*>(src));
      bf16x4 bv = *reinterpret_cast<bf16x4*>(&v);
      out[4 * h + 0] = bv[0]; out[4 * h + 1] = bv[1]; out[4 * h + 2] = bv[2]; out[4 * h + 3] = bv[3];
    }
    return out;
  }
}

template <bool A_KM, bool B_KM, bool A_F32>
__global__ void __launch_bounds__(NT, 2) gemm_kernel(GemmP p) {
  __shared__ __attribute__((aligned(16))) bf16 lds[2][2][BM * BK];  // [buf][A/B]
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int wm = wave >> 1, wn = wave & 1;

  const int tiles = p.tiles_m * p.tiles_n;
  const int z = blockIdx.y;  // batch * split
  const int bz = z / p.split_k, sk = z % p.split_k;
  const int lin = xcd_remap(blockIdx.x, tiles);
  const int tn = lin % p.tiles_n, tm = lin / p.tiles_n;
  const int m0 = tm * BM, n0 = tn * BN;

  const char* abase = static_cast<const char*>(p.a) + (long long)bz * p.sa * (A_F32 ? 4 : 2);
  const bf16* bbase = p.b + (long long)bz * p.sb;

  const int kb = sk * p.k_chunk;
  const int ke = min(p.k, kb + p.k_chunk);
  const int nk = (ke - kb + BK - 1) / BK;

  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  Stage sa, sb;
  if (nk > 0) {
    load_tile<A_KM, A_F32>(sa, abase, p.lda, p.m, ke, m0, kb, p.a_map, p.a_row_scale, p.a_rows_per_scale);
    load_tile<B_KM, false>(sb, bbase, p.ldb, p.n, ke, n0, kb, nullptr);
    store_tile<A_KM>(sa, lds[0][0]);
    store_tile<B_KM>(sb, lds[0][1]);
  }
  __syncthreads();

  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    const bool more = kt + 1 < nk;
    if (more) {
      load_tile<A_KM, A_F32>(sa, abase, p.lda, p.m, ke, m0, kb + (kt + 1) * BK, p.a_map, p.a_row_scale, p.a_rows_per_scale);
      load_tile<B_KM, false>(sb, bbase, p.ldb, p.n, ke, n0, kb + (kt + 1) * BK, nullptr);
    }
    const bf16* la = lds[cur][0];
    const bf16* lb = lds[cur][1];
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      bf16x8 af[4], bfr[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) af[i] = read_frag<A_KM>(la, wm * 64 + i * 16, ks, lane);
#pragma unroll
      for (int j = 0; j < 4; ++j) bfr[j] = read_frag<B_KM>(lb, wn * 64 + j * 16, ks, lane);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    }
    if (more) {
      store_tile<A_KM>(sa, lds[cur ^ 1][0]);
      store_tile<B_KM>(sb, lds[cur ^ 1][1]);
    }
    __syncthreads();
  }

  // ---- epilogue: lane holds rows (lane>>4)*4 + r, column lane&15 of each 16x16 tile
  const int fl = p.flags;
  char* cbase = static_cast<char*>(p.c) + (long long)bz * p.sc * ((fl & (LRCE_EPI_OUT_F32 | LRCE_EPI_ATOMIC | LRCE_EPI_ACCUM)) ? 4 : 2);
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int n = n0 + wn * 64 + j * 16 + (lane & 15);
    if (n >= p.n) continue;
    float bias = ((fl & LRCE_EPI_BIAS) && sk == 0) ? p.bias[n] : 0.f;
    const float csc = (n < p.scale_cols) ? p.scale_val : 1.f;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = m0 + wm * 64 + i * 16 + (lane >> 4) * 4 + r;
        if (m >= p.m) continue;
        const long long row = p.c_map ? (long long)p.c_map[m] : (long long)m;
        float v = acc[i][j][r] * p.alpha + bias;
        v *= csc;
        if (fl & LRCE_EPI_GELU) {
          if (fl & LRCE_EPI_AUX_OUT) p.aux_out[row * p.ld_aux_out + n] = f2bf(v);
          v = gelu_f(v);
        }
        if (fl & LRCE_EPI_DGELU) v *= gelu_grad_f(bf2f(static_cast<const bf16*>(p.aux)[row * p.ld_aux + n]));
        if (p.row_scale) v *= p.row_scale[m / p.rows_per_scale];
        if ((fl & LRCE_EPI_RESID) && sk == 0) v += static_cast<const float*>(p.aux)[row * p.ld_aux + n];
        if (fl & LRCE_EPI_ATOMIC) {
          atomicAdd(reinterpret_cast<float*>(cbase) + row * p.ldc + n, v);
        } else if (fl & LRCE_EPI_ACCUM) {
          reinterpret_cast<float*>(cbase)[row * p.ldc + n] += v;
        } else if (fl & LRCE_EPI_OUT_F32) {
          reinterpret_cast<float*>(cbase)[row * p.ldc + n] = v;
          if (fl & LRCE_EPI_OUT_BOTH) p.aux_out[row * p.ld_aux_out + n] = f2bf(v);
        } else {
          reinterpret_cast<bf16*>(cbase)[row * p.ldc + n] = f2bf(v);
        }
      }
    }
  }
}

}  // namespace

int lrce_gemm_f32(const LrceGemmDesc* d, void* stream);

extern "C" int lrce_gemm(const LrceGemmDesc* d, void* stream) {
  if (!d || !d->a || !d->b || !d->c) return lrce_fail(LRCE_E_ARG, "gemm: null pointer");
  if (d->m <= 0 || d->n <= 0 || d->k <= 0 || d->batch <= 0) return lrce_fail(LRCE_E_ARG, "gemm: empty shape");
  if ((d->flags & (LRCE_EPI_DGELU | LRCE_EPI_RESID)) && !d->aux) return lrce_fail(LRCE_E_ARG, "gemm: aux missing");
  if ((d->flags & (LRCE_EPI_AUX_OUT | LRCE_EPI_OUT_BOTH)) && !d->aux_out) return lrce_fail(LRCE_E_ARG, "gemm: aux_out missing");
  if ((d->flags & LRCE_EPI_BIAS) && !d->bias) return lrce_fail(LRCE_E_ARG, "gemm: bias missing");
  if (d->b_f32) return lrce_gemm_f32(d, stream);
  // vector loads need the contiguous dim of every operand to be a multiple of 8 elements
  if (d->a_kmajor ? (d->k % 8) : (d->m % 8)) return lrce_fail(LRCE_E_ARG, "gemm: A contiguous dim %% 8 != 0");
  if (d->b_kmajor ? (d->k % 8) : (d->n % 8)) return lrce_fail(LRCE_E_ARG, "gemm: B contiguous dim %% 8 != 0");
  if ((d->lda % 8) || (d->ldb % 8)) return lrce_fail(LRCE_E_ARG, "gemm: lda/ldb %% 8 != 0");
  const int split = d->split_k > 1 ? d->split_k : 1;
  if (split > 1 && !(d->flags & LRCE_EPI_ATOMIC)) return lrce_fail(LRCE_E_ARG, "gemm: split_k needs ATOMIC");
  if ((d->flags & (LRCE_EPI_GELU | LRCE_EPI_AUX_OUT)) == LRCE_EPI_AUX_OUT) return lrce_fail(LRCE_E_ARG, "gemm: AUX_OUT needs GELU");
  if ((d->flags & (LRCE_EPI_DGELU | LRCE_EPI_RESID)) && !d->aux) return lrce_fail(LRCE_E_ARG, "gemm: aux missing");
  if ((d->flags & (LRCE_EPI_AUX_OUT | LRCE_EPI_OUT_BOTH)) && !d->aux_out) return lrce_fail(LRCE_E_ARG, "gemm: aux_out missing");
  if ((d->flags & LRCE_EPI_BIAS) && !d->bias) return lrce_fail(LRCE_E_ARG, "gemm: bias missing");
  if (d->a_f32 && !d->a_kmajor && d->a_map == nullptr && (d->lda % 4)) return lrce_fail(LRCE_E_ARG, "gemm: f32 A lda");

  GemmP p;
  p.a = d->a; p.b = static_cast<const bf16*>(d->b); p.c = d->c;
  p.lda = d->lda; p.ldb = d->ldb; p.ldc = d->ldc;
  p.sa = d->stride_a; p.sb = d->stride_b; p.sc = d->stride_c;
  p.m = d->m; p.n = d->n; p.k = d->k; p.batch = d->batch; p.split_k = split;
  int chunk = (d->k + split - 1) / split;
  chunk = (chunk + BK - 1) / BK * BK;
  p.k_chunk = chunk;
  p.flags = d->flags;
  p.bias = d->bias; p.aux = d->aux; p.ld_aux = d->ld_aux;
  p.aux_out = static_cast<bf16*>(d->aux_out); p.ld_aux_out = d->ld_aux_out;
  p.a_map = d->a_map; p.c_map = d->c_map;
  p.alpha = d->alpha; p.scale_cols = d->scale_cols; p.scale_val = d->scale_val;
  p.row_scale = d->row_scale; p.rows_per_scale = d->rows_per_scale > 0 ? d->rows_per_scale : 1;
  p.a_row_scale = d->a_row_scale; p.a_rows_per_scale = d->a_rows_per_scale > 0 ? d->a_rows_per_scale : 1;
  if (p.a_row_scale && !d->a_f32) return lrce_fail(LRCE_E_ARG, "gemm: a_row_scale needs f32 A");
  p.tiles_m = (d->m + BM - 1) / BM; p.tiles_n = (d->n + BN - 1) / BN;
  dim3 grid(p.tiles_m * p.tiles_n, d->batch * split);
  hipStream_t s = static_cast<hipStream_t>(stream);
  const int key = (d->a_kmajor ? 4 : 0) | (d->b_kmajor ? 2 : 0) | (d->a_f32 ? 1 : 0);
  switch (key) {
    case 6: gemm_kernel<true, true, false><<<grid, NT, 0, s>>>(p); break;
    case 7: gemm_kernel<true, true, true><<<grid, NT, 0, s>>>(p); break;
    case 4: gemm_kernel<true, false, false><<<grid, NT, 0, s>>>(p); break;
    case 5: gemm_kernel<true, false, true><<<grid, NT, 0, s>>>(p); break;
    case 0: gemm_kernel<false, false, false><<<grid, NT, 0, s>>>(p); break;
    case 1: gemm_kernel<false, false, true><<<grid, NT, 0, s>>>(p); break;
    case 2: gemm_kernel<false, true, false><<<grid, NT, 0, s>>>(p); break;
    case 3: gemm_kernel<false, true, true><<<grid, NT, 0, s>>>(p); break;
  }
  return lrce_check_launch("gemm");
}
