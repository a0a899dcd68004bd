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
// Epilogue: each wave stages its 64x64 fp32 tile through LDS (two padded 32-row halves) and applies
// bias / GELU / dGELU / row scale / residual / output conversion on 8 consecutive columns per lane,
// so every global access of the epilogue is a 16-B vector (scalar fallback for ragged / unaligned
// edges).  All operand loads are unconditional (out-of-range lanes read a clamped in-bounds address
// and are zeroed by a select), which keeps the global loads of a K-tile batched.
#include <cstdlib>
#include <type_traits>
#include <vector>

#include "common.h"
#include "lrce_capi.h"

namespace {

constexpr int BM = 128, BN = 128, BK = 64, NT = 256;

struct GemmP {
  const void* a;
  const bf16* b;
  void* c;
  long long lda, ldb, ldc, sa, sb, sc;
  long long sbias;   // batch stride of the bias (elements; 0: one bias for every batch)
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
  int vec;  // 1: c/aux/aux_out/bias rows are 16-B aligned and n % 8 == 0 (vector epilogue)
  float* ws; // split-K slabs [split][m][n] (plain stores, reduced by splitk_reduce_kernel), or null
  int f16;   // 16-bit tensors are IEEE fp16 (LrceGemmDesc.f16)
  int group_m;   // tile raster: groups of group_m tile rows, column-major inside a group (1 = row-major)
  const float* alpha_dev;   // non-null: alpha read from device memory (a gradient scale computed on the GPU)
  long long salpha;         // batch stride of alpha_dev (floats)
  unsigned long long* trace;   // phase timestamps (builds with -DLRCE_GEMM_TRACE only; lrce_gemm_set_trace)
  // nn.Dropout in the epilogue (after bias / GELU / row scale, before the RESID add): the mask of
  // lrce_dropout over the contiguous [m][n] result (element m * n + col), drop_group 1
  float drop_p;
  uint64_t drop_seed;
  const uint64_t* rng_off;
};

// Grouped weight-gradient launch (lrce_gemm_grouped; lrce_gemm_ptr_batched is its one-shape case):
// entry e reads A / B from its own pointers, writes C / the bias gradient at f32 element offsets from
// p.c / p.bias, has its own shape (one of GSH per launch) and epilogue flags, and owns workgroups
// [start[e], start[e+1]) of a 1-D grid.  A Swin stage's four linears x blocks then run as ONE launch:
// no tail round per shape, and with the grid XCD-remapped as a whole each XCD walks whole entries in
// order, so its L2 reads an entry's dY / X panels once instead of every XCD reading a share of each.
constexpr int GPT = 80, GSH = 8;
struct GemmShape {
  int m, n, lda, ldb, ldc, tiles_m, tiles_n;
  int split, k_chunk;   // K slices of each entry of this shape (slice s: its own C / bias slab)
};
struct GemmPT : GemmP {
  int ng;                 // entries
  GemmShape sh[GSH];
  int start[GPT + 1];     // first workgroup of each entry; start[ng] = the grid
  int meta[GPT];          // shape index | epilogue flags << 8
  int coff[GPT];          // C offset from p.c (f32 elements)
  int boff[GPT];          // bias-gradient offset from p.bias (f32 elements), -1: none
  int aoff[GPT];          // device alpha offset from p.alpha_dev (floats), -1: the launch's alpha
  const void* ta[GPT];
  const bf16* tb[GPT];
};
static_assert(sizeof(GemmPT) <= 3840, "grouped GEMM tables must fit the kernel-argument block");
template <bool PT>
using GemmArg = typename std::conditional<PT, GemmPT, GemmP>::type;

// Debug phase marks of gemm_glds_kernel (tools/gemm_trace.py): wave 0 of every workgroup stores
// s_memrealtime (100 MHz) at mark i into trace[blockIdx.x * 8 + i]; slot 6/7 = HW_ID / XCC_ID.
#ifdef LRCE_GEMM_TRACE
#define GT_MARK(I)                                                                                   \
  do {                                                                                               \
    if (p.trace && threadIdx.x == 0 && blockIdx.y == 0)                                              \
      p.trace[(long long)blockIdx.x * 8 + (I)] = __builtin_amdgcn_s_memrealtime();                   \
  } while (0)
#else
#define GT_MARK(I) do {} while (0)
#endif
static unsigned long long* g_gemm_trace = nullptr;

__device__ __forceinline__ float alpha_of(const GemmP& p) { return p.alpha_dev ? *p.alpha_dev : p.alpha; }

// Tile (tm, tn) of linear index lin (already XCD-remapped: each XCD owns a contiguous lin range).
// Grouped order: a group is group_m tile rows x all tile columns, walked column by column, so the
// 8-32 consecutive tiles one XCD holds at a time form a group_m-tall block: its L2 serves each A panel
// to the block's columns and each B panel to its rows (row-major order gave an XCD one A panel and
// 8+ B panels, every B panel then fetched once per XCD that holds its column).
__device__ __forceinline__ void tile_of(const GemmP& p, int lin, int& tm, int& tn) {
  const int gm = p.group_m;
  const int per = gm * p.tiles_n;
  const int g = lin / per, rem = lin - g * per;
  const int m0 = g * gm;
  const int gsz = min(gm, p.tiles_m - m0);
  tm = m0 + rem % gsz;
  tn = rem / gsz;
}

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
    const bool ok = gr < rows_total && gk < kdim;
    const int grc = ok ? gr : 0, gkc = ok ? gk : 0;  // (0,0) is always in range: m, n, k > 0
    long long off;
    if (KMAJ) {
      const long long rr = map ? (long long)map[grc] : (long long)grc;
      off = rr * ld + gkc;
    } else {
      const long long kr = map ? (long long)map[gkc] : (long long)gkc;
      off = kr * ld + grc;
    }
    uint4 val;
    if (F32) {
      const float4* q = reinterpret_cast<const float4*>(static_cast<const float*>(base) + off);
      float4 x0 = q[0], x1 = q[1];
      if (rsc) {
        const float f = rsc[(KMAJ ? grc : gkc) / rps];
        x0.x *= f; x0.y *= f; x0.z *= f; x0.w *= f; x1.x *= f; x1.y *= f; x1.z *= f; x1.w *= f;
      }
      bf16x8 t;
      t[0] = f2bf(x0.x); t[1] = f2bf(x0.y); t[2] = f2bf(x0.z); t[3] = f2bf(x0.w);
      t[4] = f2bf(x1.x); t[5] = f2bf(x1.y); t[6] = f2bf(x1.z); t[7] = f2bf(x1.w);
      val = *reinterpret_cast<uint4*>(&t);
    } else {
      val = *reinterpret_cast<const uint4*>(static_cast<const bf16*>(base) + off);
    }
    if (!ok) val = make_uint4(0, 0, 0, 0);
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

constexpr int EP = 68;  // padded fp32 row of the epilogue staging tile (conflict-free writes)

__device__ __forceinline__ void wave_lds_fence() {
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  __builtin_amdgcn_wave_barrier();
}

// Fused epilogue for one element (row = c_map-resolved output row).
template <bool DROP = false>
__device__ __forceinline__ void epilogue1(const GemmP& p, float x, long long row, int m, int nn, bool first, float rs,
                                          char* cbase) {
  const int fl = p.flags;
  x = x * alpha_of(p) + (((fl & LRCE_EPI_BIAS) && first) ? p.bias[nn] : 0.f);
  x *= (nn < p.scale_cols) ? p.scale_val : 1.f;
  if (fl & LRCE_EPI_GELU) {
    if (fl & LRCE_EPI_AUX_OUT) p.aux_out[row * p.ld_aux_out + nn] = to16r(x, p.f16);
    x = gelu_f(x);
  }
  if (fl & LRCE_EPI_DGELU) x *= gelu_grad_f(from16r(static_cast<const bf16*>(p.aux)[row * p.ld_aux + nn], p.f16));
  x *= rs;
  if (DROP)
    x = lrce_uniform(lrce_seed(p.drop_seed, p.rng_off), (unsigned long long)m * p.n + nn) >= p.drop_p ? x / (1.0f - p.drop_p) : 0.f;
  if ((fl & LRCE_EPI_RESID) && first) x += static_cast<const float*>(p.aux)[row * p.ld_aux + nn];
  if (fl & LRCE_EPI_ATOMIC) {
    __hip_atomic_fetch_add(reinterpret_cast<float*>(cbase) + row * p.ldc + nn, x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  } else if (fl & LRCE_EPI_ACCUM) {
    reinterpret_cast<float*>(cbase)[row * p.ldc + nn] += x;
  } else if (fl & LRCE_EPI_OUT_F32) {
    reinterpret_cast<float*>(cbase)[row * p.ldc + nn] = x;
    if (fl & LRCE_EPI_OUT_BOTH) p.aux_out[row * p.ld_aux_out + nn] = to16r(x, p.f16);
  } else {
    reinterpret_cast<bf16*>(cbase)[row * p.ldc + nn] = to16r(x, p.f16);
  }
}

// Fused epilogue for 8 consecutive columns n..n+7 of output row m (see LrceGemmDesc flags).  The
// 16-bit format is a template parameter and every optional factor sits behind a wave-uniform branch
// (alpha, the q-scale columns — host guarantees scale_cols % 8 == 0 on the vector path — and the row
// scale), so a plain epilogue is a conversion and a 16-B store per 8 outputs.
// Epilogue operands loaded ahead of the epilogue's first store (gemm_glds_kernel): vmcnt counts loads
// and stores in one in-order counter, so a load issued after a store can only be waited for together
// with that store — per 8-column chunk that was a full store round trip (6.7-13 us of epilogue per
// workgroup in tools/gemm_trace.py).  `have` = 0: epilogue8 loads them itself (the legacy kernel).
struct EpiPf {
  int have;
  float al;              // alpha_of(p)
  long long row;         // c_map-resolved output row (-1: none)
  float rs;              // row scale (1 if none)
  const float4* bias;    // 2 float4 of bias for this chunk, or null
};

template <bool F16, bool DROP = false>
__device__ __forceinline__ void epilogue8(const GemmP& p, float v[8], int m, int n, int sk, char* cbase,
                                          const bf16x8* dg_pf = nullptr, const float4* rs_pf = nullptr,
                                          const EpiPf* pf = nullptr, const float4* acc_pf = nullptr) {
  if (m >= p.m || n >= p.n) return;
  const int fl = p.flags;
  const long long row = pf ? pf->row : (p.c_map ? (long long)p.c_map[m] : (long long)m);
  if (row < 0) return;   // c_map -1: a padded window position (no output row)
  const bool first = sk == 0;
  if (p.vec && n + 8 <= p.n) {
    const float al = pf ? pf->al : alpha_of(p);
    if (al != 1.f) {
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] *= al;
    }
    if ((fl & LRCE_EPI_BIAS) && first) {
      const float4 b0 = pf ? pf->bias[0] : *reinterpret_cast<const float4*>(p.bias + n);
      const float4 b1 = pf ? pf->bias[1] : *reinterpret_cast<const float4*>(p.bias + n + 4);
      v[0] += b0.x; v[1] += b0.y; v[2] += b0.z; v[3] += b0.w; v[4] += b1.x; v[5] += b1.y; v[6] += b1.z; v[7] += b1.w;
    }
    if (n < p.scale_cols) {
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] *= p.scale_val;
    }
    if (fl & LRCE_EPI_GELU) {
      if (fl & LRCE_EPI_AUX_OUT) {
        bf16x8 pre;
#pragma unroll
        for (int e = 0; e < 8; ++e) pre[e] = to16<F16>(v[e]);
        *reinterpret_cast<bf16x8*>(p.aux_out + row * p.ld_aux_out + n) = pre;
      }
#pragma unroll
      for (int e = 0; e < 8; e += 2) {
        const f32x2v g = gelu2(f32x2v{v[e], v[e + 1]});
        v[e] = g.x;
        v[e + 1] = g.y;
      }
    }
    if (fl & LRCE_EPI_DGELU) {
      const bf16x8 pre = dg_pf ? *dg_pf : *reinterpret_cast<const bf16x8*>(static_cast<const bf16*>(p.aux) + row * p.ld_aux + n);
#pragma unroll
      for (int e = 0; e < 8; e += 2) {
        const f32x2v g = gelu_grad2(f32x2v{from16<F16>(pre[e]), from16<F16>(pre[e + 1])});
        v[e] *= g.x;
        v[e + 1] *= g.y;
      }
    }
    if (p.row_scale) {
      const float rs = pf ? pf->rs : p.row_scale[m / p.rows_per_scale];
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] *= rs;
    }
    if (DROP) {   // lrce_dropout's bits: v / (1 - p) where kept (n % 8 == 0 on this path)
      const uint64_t sd = lrce_seed(p.drop_seed, p.rng_off);
      const unsigned long long i4 = ((unsigned long long)m * p.n + n) >> 2;
      const float4 u0 = lrce_uniform4(sd, i4), u1 = lrce_uniform4(sd, i4 + 1);
      const float u[8] = {u0.x, u0.y, u0.z, u0.w, u1.x, u1.y, u1.z, u1.w};
      const float kd = 1.0f - p.drop_p;
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] = u[e] >= p.drop_p ? v[e] / kd : 0.f;
    }
    if ((fl & LRCE_EPI_RESID) && first) {
      const float* ap = static_cast<const float*>(p.aux) + row * p.ld_aux + n;
      const float4 r0 = rs_pf ? rs_pf[0] : *reinterpret_cast<const float4*>(ap);
      const float4 r1 = rs_pf ? rs_pf[1] : *reinterpret_cast<const float4*>(ap + 4);
      v[0] += r0.x; v[1] += r0.y; v[2] += r0.z; v[3] += r0.w; v[4] += r1.x; v[5] += r1.y; v[6] += r1.z; v[7] += r1.w;
    }
    if (fl & LRCE_EPI_ATOMIC) {
      float* cp = reinterpret_cast<float*>(cbase) + row * p.ldc + n;
#pragma unroll
      for (int e = 0; e < 8; ++e) __hip_atomic_fetch_add(cp + e, v[e], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    } else if (fl & (LRCE_EPI_ACCUM | LRCE_EPI_OUT_F32)) {
      float4* cp = reinterpret_cast<float4*>(reinterpret_cast<float*>(cbase) + row * p.ldc + n);
      float4 o0 = make_float4(v[0], v[1], v[2], v[3]), o1 = make_float4(v[4], v[5], v[6], v[7]);
      if (fl & LRCE_EPI_ACCUM) {
        const float4 c0 = acc_pf ? acc_pf[0] : cp[0], c1 = acc_pf ? acc_pf[1] : cp[1];
        o0.x += c0.x; o0.y += c0.y; o0.z += c0.z; o0.w += c0.w; o1.x += c1.x; o1.y += c1.y; o1.z += c1.z; o1.w += c1.w;
      }
      cp[0] = o0; cp[1] = o1;
      if ((fl & LRCE_EPI_OUT_BOTH) && !(fl & LRCE_EPI_ACCUM)) {
        bf16x8 o;
#pragma unroll
        for (int e = 0; e < 8; ++e) o[e] = to16<F16>(v[e]);
        *reinterpret_cast<bf16x8*>(p.aux_out + row * p.ld_aux_out + n) = o;
      }
    } else {
      bf16x8 o;
#pragma unroll
      for (int e = 0; e < 8; ++e) o[e] = to16<F16>(v[e]);
      *reinterpret_cast<bf16x8*>(reinterpret_cast<bf16*>(cbase) + row * p.ldc + n) = o;
    }
    return;
  }
  const float rs = p.row_scale ? p.row_scale[m / p.rows_per_scale] : 1.f;
  // ragged / unaligned edge: element by element
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    if (n + e >= p.n) break;
    epilogue1<DROP>(p, v[e], row, m, n + e, first, rs, cbase);
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
  p.bias += (long long)bz * p.sbias;
  if (p.alpha_dev) p.alpha_dev += (long long)bz * p.salpha;
  const int lin = xcd_remap(blockIdx.x, tiles);
  int tm, tn;
  tile_of(p, lin, tm, tn);
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

  // ---- epilogue through LDS (the K loop ended with a barrier: every wave is done with the tiles)
  char* cbase = static_cast<char*>(p.c) +
                (long long)bz * p.sc * ((p.flags & (LRCE_EPI_OUT_F32 | LRCE_EPI_ATOMIC | LRCE_EPI_ACCUM)) ? 4 : 2);
  float* E = reinterpret_cast<float*>(&lds[0][0][0]) + wave * (32 * EP);
  const int cc = (lane & 7) * 8;
  auto half = [&](auto hc) {
    constexpr int h = decltype(hc)::value;
#pragma unroll
    for (int ii = 0; ii < 2; ++ii)
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r)
          E[(ii * 16 + (lane >> 4) * 4 + r) * EP + j * 16 + (lane & 15)] = acc[2 * h + ii][j][r];
    wave_lds_fence();
    if (p.flags & LRCE_EPI_ATOMIC) {
      // split-K partial sums: one row per instruction, 64 consecutive columns (coalesced atomics)
      const int n = n0 + wn * 64 + lane;
      if (n < p.n) {
        for (int rr = 0; rr < 32; ++rr) {
          const int m = m0 + wm * 64 + h * 32 + rr;
          if (m >= p.m) break;
          const long long row = p.c_map ? (long long)p.c_map[m] : (long long)m;
          if (row < 0) continue;
          const float rs = p.row_scale ? p.row_scale[m / p.rows_per_scale] : 1.f;
          epilogue1(p, E[rr * EP + lane], row, m, n, sk == 0, rs, cbase);
        }
      }
    } else {
#pragma unroll
      for (int it = 0; it < 4; ++it) {
        const int rr = it * 8 + (lane >> 3);
        const float4 x0 = *reinterpret_cast<const float4*>(E + rr * EP + cc);
        const float4 x1 = *reinterpret_cast<const float4*>(E + rr * EP + cc + 4);
        float v[8] = {x0.x, x0.y, x0.z, x0.w, x1.x, x1.y, x1.z, x1.w};
        epilogue8<false>(p, v, m0 + wm * 64 + h * 32 + rr, n0 + wn * 64 + cc, sk, cbase);   // f16 is LDS-DMA only
      }
    }
    wave_lds_fence();
  };
  half(std::integral_constant<int, 0>{});
  half(std::integral_constant<int, 1>{});
}


// ---------------------------------------------------------------------------------------------
// bf16 x bf16 path with LDS-DMA staging (global_load_lds_dwordx4): operand tiles go HBM/L2 -> LDS
// without passing through VGPRs, two LDS stages, the next K tile in flight while the current one
// is consumed (counted vmcnt + raw s_barrier, cdna_hip_programming.md §5 "Pipelining across
// barriers").  The LDS images are swizzled as above; glds writes lane-linearly, so each lane fetches
// the global chunk that the swizzle places at its linear position.
// Tile TBM x TBN (128x128 for large problems, 64x64 when the 128-tile grid would not fill the chip),
// 4 waves as 2x2, each (TBM/2)x(TBN/2).  The MFMA operands are swapped (B fragment first) so the
// accumulator holds C^T blocks; a permlane transpose then gives each lane 8 or 16 contiguous output
// columns of one row for 16-B vector epilogues.  A K tail (< 64) is staged through registers.

// M-major LDS image [64 k][R] bf16 (R = 128 or 64 elements per k row), 8-B units XOR-swizzled by an
// even (16-B-chunk granular, for the DMA) function of k.
template <int R>
__device__ __forceinline__ int mm_swz_r(int k) { return ((k & 3) | (((k >> 3) & 1) << 2)) << (R == 128 ? 2 : 1); }
template <int R>
__device__ __forceinline__ int mm_off_r(int k, int unit) { return k * R + ((unit ^ mm_swz_r<R>(k)) << 2); }

template <bool KMAJ, int R>
__device__ __forceinline__ bf16x8 read_frag_r(const bf16* lds, int r0, int ks, int lane) {
  if (KMAJ) {
    const int row = r0 + (lane & 15);
    const int kc = ks * 4 + (lane >> 4);
    return *reinterpret_cast<const bf16x8*>(lds + km_off(row, kc));
  } else {
    const int g = lane >> 4, i = lane & 15, q = i >> 2, pp = i & 3;
    const int unit = (r0 >> 2) + pp;
    bf16x8 out;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int k = ks * 32 + 8 * g + 4 * h + q;
      const LRCE_LDS s16x4* src = (const LRCE_LDS s16x4*)(lds + mm_off_r<R>(k, unit));
      s16x4 v = __builtin_amdgcn_ds_read_tr16_b64_v4i16(const_cast<LRCE_LDS s16x4*>(src));
      bf16x4 bv = *reinterpret_cast<bf16x4*>(&v);
      out[4 * h + 0] = bv[0]; out[4 * h + 1] = bv[1]; out[4 * h + 2] = bv[2]; out[4 * h + 3] = bv[3];
    }
    return out;
  }
}

// register-staged load of an R x 64 operand tile (the K tail), zero outside [rows_total) x [kdim)
template <bool KMAJ, int R>
__device__ __forceinline__ void tail_tile(bf16* lds, const bf16* base, long long ld, int rows_total, int kdim, int row0,
                                          int k0, const int* map) {
  constexpr int NI = R / 32;  // 16-B pieces per thread
  uint4 v[NI];
  const int tid = threadIdx.x;
#pragma unroll
  for (int i = 0; i < NI; ++i) {
    const int c = tid + NT * i;
    int r, kk;
    if (KMAJ) { r = c >> 3; kk = (c & 7) << 3; }
    else { kk = c / (R / 8); r = (c % (R / 8)) << 3; }
    const int gr = row0 + r, gk = k0 + kk;
    const bool ok = gr < rows_total && gk < kdim;
    const int grc = ok ? gr : 0, gkc = ok ? gk : 0;
    long long off;
    if (KMAJ) off = (map ? (long long)map[grc] : (long long)grc) * ld + gkc;
    else off = (long long)gkc * ld + grc;
    uint4 val = *reinterpret_cast<const uint4*>(base + off);
    if (!ok) val = make_uint4(0, 0, 0, 0);
    v[i] = val;
  }
#pragma unroll
  for (int i = 0; i < NI; ++i) {
    const int c = tid + NT * i;
    const int off = KMAJ ? km_off(c >> 3, c & 7) : mm_off_r<R>(c / (R / 8), (c % (R / 8)) << 1);
    *reinterpret_cast<uint4*>(lds + off) = v[i];
  }
}

__device__ __forceinline__ void glds16(const void* src, bf16* lds_dst) {
  __builtin_amdgcn_global_load_lds(src, (LRCE_LDS void*)lds_dst, 16, 0, 0);
}

// LDS-DMA with a wave-uniform 64-bit base in SGPRs and a 32-bit per-lane byte offset (the saddr
// form), M0 = the wave's 1-KB LDS destination.  Written as asm so the per-K-tile address update is
// ONE scalar add (a builtin takes a per-lane 64-bit pointer: 2 VALU adds + copies per instruction
// per tile) and so hipcc does not drain vmcnt(0) before every LDS read while a DMA is in flight;
// completion is ordered by the main loop's explicit vmcnt waits + s_barrier.
__device__ __forceinline__ void glds16_s(const void* sbase, uint32_t voff, uint32_t lds_dst) {
  unsigned keep;
  const uint64_t a = reinterpret_cast<uintptr_t>(sbase);
  // (readfirstlane returns int: go through uint32_t, or the low word would sign-extend)
  const uint64_t su = (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)a) |
                      ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)(a >> 32)) << 32);
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, %2\n\ts_mov_b32 m0, %0"
               : "=&s"(keep) : "v"(voff), "s"(su), "s"(__builtin_amdgcn_readfirstlane(lds_dst)) : "memory");
}
__device__ __forceinline__ uint32_t lds_addr(const void* p) { return (uint32_t)(uintptr_t)((LRCE_LDS const void*)p); }

// Per-lane source offsets of the R/32 glds instructions a wave issues per operand tile (1 KB each).
// K-major tile [R rows][64 k]: instruction i covers rows 8i..8i+7.
// M-major tile [64 k][R]: instruction i covers the 1024 / 2R k rows starting at i * 1024 / 2R.
// The offsets are loop-invariant; only the uniform base advances (glds_ok bounds them to 31 bits).
template <bool KMAJ, int R>
struct GldsOperand {
  static constexpr int NI = R / 32;
  const char* base;      // wave-uniform
  uint32_t off[NI];      // bytes from base
  uint32_t step;         // bytes per K tile

  __device__ __forceinline__ void init(const bf16* b, long long ld, int rows_total, int row0, int k0, int wave, int lane) {
    base = reinterpret_cast<const char*>(b);
#pragma unroll
    for (int q = 0; q < NI; ++q) {
      const int ins = wave + 4 * q;
      long long e;
      if (KMAJ) {
        const int r = ins * 8 + (lane >> 3), pos = lane & 7;
        const int kc = pos ^ ((r >> 1) & 7);
        int gr = row0 + r;
        gr = gr < rows_total ? gr : rows_total - 1;    // rows past the edge: any valid row (never stored)
        e = (long long)gr * ld + k0 + kc * 8;
      } else {
        constexpr int CPR = R / 8;                      // 16-B chunks per k row
        const int kr = ins * (64 / CPR) + lane / CPR, pos = lane % CPR;
        const int c = pos ^ (mm_swz_r<R>(kr) >> 1);
        int gm = row0 + c * 8;
        gm = gm < rows_total ? gm : 0;
        e = (long long)(k0 + kr) * ld + gm;
      }
      off[q] = (uint32_t)(e * 2);
    }
    step = (uint32_t)(KMAJ ? BK * 2 : (long long)BK * ld * 2);
  }
  __device__ __forceinline__ void issue(uint32_t tile, int wave_u) {
#pragma unroll
    for (int q = 0; q < NI; ++q) glds16_s(base, off[q], tile + (uint32_t)(wave_u + 4 * q) * 1024u);
  }
  __device__ __forceinline__ void advance() { base += step; }
};

// short-K epilogue-operand prefetch (gemm_glds_kernel): K tiles up to which it is done, and the
// register slots (accumulator row blocks) it may hold — the f32 residual only up to 4 row blocks
constexpr int PF_KT = 8;
constexpr int pf_dg_slots(int im) { return im; }
constexpr int pf_rs_slots(int im) { return im <= 4 ? im : 1; }

// DROP: the fused-dropout epilogue (a separate instantiation: the branch in every kernel measured
// 14-17 % slower tall-tile GEMMs through changed code generation)
template <int TBM, int TBN, bool A_KM, bool B_KM, bool F16 = false, int NS = 2, bool DROP = false, bool PT = false>
__global__ void __launch_bounds__(NT, 2) gemm_glds_kernel(const GemmArg<PT> pa) {
  // the shared fields as a local copy (registers); the grouped tables are read from the unmodified
  // argument (a dynamically indexed copy of the whole struct would live in scratch)
  GemmP p = pa;
  constexpr int WM = TBM / 2, WN = TBN / 2;      // per-wave tile
  constexpr int IM = WM / 16, JN = WN / 16;      // 16x16 accumulator blocks per wave
  constexpr int A_EL = TBM * BK, B_EL = TBN * BK;
  __shared__ __attribute__((aligned(16))) bf16 lds[NS * (A_EL + B_EL)];  // [stage][A | B]
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const int z = blockIdx.y;
  const int bz = z / p.split_k, sk = z % p.split_k;
  int lin;
  int kslice = sk;   // this workgroup's K slice
  const bf16* abase;
  const bf16* bbase;
  if constexpr (PT) {
    // grouped: the entry owning this workgroup (binary search of the start table), its shape / flags
    const int g = xcd_remap(blockIdx.x, pa.start[pa.ng]);
    int lo = 0, hi = pa.ng - 1;
    while (lo < hi) {
      const int mid = (lo + hi + 1) >> 1;
      if (pa.start[mid] <= g) lo = mid;
      else hi = mid - 1;
    }
    const int meta = pa.meta[lo];
    const GemmShape sh = pa.sh[meta & (GSH - 1)];
    p.m = sh.m; p.n = sh.n; p.lda = sh.lda; p.ldb = sh.ldb; p.ldc = sh.ldc;
    p.tiles_m = sh.tiles_m; p.tiles_n = sh.tiles_n;
    p.flags = meta >> 8;
    p.bias = pa.boff[lo] >= 0 ? p.bias + pa.boff[lo] : nullptr;
    p.alpha_dev = pa.aoff[lo] >= 0 ? p.alpha_dev + pa.aoff[lo] : nullptr;
    p.c = static_cast<float*>(p.c) + pa.coff[lo];
    abase = static_cast<const bf16*>(pa.ta[lo]);
    bbase = pa.tb[lo];
    lin = g - pa.start[lo];
    if (sh.split > 1) {   // slice-major: slice s stores its partial into slab s of C and of the bias
      const int tiles = sh.tiles_m * sh.tiles_n;
      kslice = lin / tiles;
      lin -= kslice * tiles;
      p.k_chunk = sh.k_chunk;
      p.c = static_cast<float*>(p.c) + (long long)kslice * sh.m * sh.ldc;
      if (p.bias) p.bias += (long long)kslice * sh.m;
    }
  } else {
    p.bias += (long long)bz * p.sbias;
    if (p.alpha_dev) p.alpha_dev += (long long)bz * p.salpha;
    lin = xcd_remap(blockIdx.x, p.tiles_m * p.tiles_n);
    abase = static_cast<const bf16*>(p.a) + (long long)bz * p.sa;
    bbase = p.b + (long long)bz * p.sb;
  }
  int tm, tn;
  tile_of(p, lin, tm, tn);
  const int m0 = tm * TBM, n0 = tn * TBN;
  GT_MARK(0);
#ifdef LRCE_GEMM_TRACE
  if (p.trace && threadIdx.x == 0 && blockIdx.y == 0) {
    p.trace[(long long)blockIdx.x * 8 + 6] = __builtin_amdgcn_s_getreg(4 | (31 << 11));
    p.trace[(long long)blockIdx.x * 8 + 7] = __builtin_amdgcn_s_getreg(20 | (31 << 11));
  }
#endif
  const int kb = kslice * p.k_chunk;
  const int ke = min(p.k, kb + p.k_chunk);
  const int nfull = ke > kb ? (ke - kb) / BK : 0;
  const bool tail = ke > kb + nfull * BK;
  bf16* const sa0 = lds;
  bf16* const sb0 = lds + A_EL;
  constexpr int STG = A_EL + B_EL;

  f32x4 acc[IM][JN];
#pragma unroll
  for (int i = 0; i < IM; ++i)
#pragma unroll
    for (int j = 0; j < JN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // bias gradient (dW GEMMs, A = dY^T): the waves of the first column tile also multiply A by a
  // ones operand, i.e. sum_k A(m, k) falls out of the MFMA pipe (IM extra MFMAs per IM*JN)
  const bool bias_block = !A_KM && (p.flags & LRCE_EPI_BIAS_GRAD) && tn == 0 && wn == 0;
  f32x4 accb[IM];
#pragma unroll
  for (int i = 0; i < IM; ++i) accb[i] = f32x4{0.f, 0.f, 0.f, 0.f};
  bf16x8 ones;
#pragma unroll
  for (int e = 0; e < 8; ++e) ones[e] = to16<F16>(1.0f);

  auto compute = [&](const bf16* la, const bf16* lb) {
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      bf16x8 af[IM], bfr[JN];
#pragma unroll
      for (int i = 0; i < IM; ++i) af[i] = read_frag_r<A_KM, TBM>(la, wm * WM + i * 16, ks, lane);
#pragma unroll
      for (int j = 0; j < JN; ++j) bfr[j] = read_frag_r<B_KM, TBN>(lb, wn * WN + j * 16, ks, lane);
#pragma unroll
      for (int i = 0; i < IM; ++i)
#pragma unroll
        for (int j = 0; j < JN; ++j) acc[i][j] = mfma16x16x32<F16>(bfr[j], af[i], acc[i][j]);
      if (bias_block) {
#pragma unroll
        for (int i = 0; i < IM; ++i) accb[i] = mfma16x16x32<F16>(ones, af[i], accb[i]);
      }
    }
  };

  // Short K (<= PF_KT full tiles): the epilogue's global operands (the dGELU pre-activation, the f32
  // residual) are loaded BEFORE the operand tiles, so they ride the tiles' memory round trip instead
  // of adding one after the MFMAs (at K = 128 the kernel is a chain of such round trips).  Issued
  // first, they also complete before the tiles' counted vmcnt waits pass (loads retire in order).
  constexpr int NH = JN / 2;
  const int ncol = n0 + wn * WN + (JN * 4) * (lane >> 4);
  const bool pf_dg = (p.flags & LRCE_EPI_DGELU) && p.vec && nfull <= PF_KT && !p.ws && !(p.flags & LRCE_EPI_ATOMIC);
  const bool pf_rs = IM <= 4 && (p.flags & LRCE_EPI_RESID) && sk == 0 && p.vec && nfull <= PF_KT && !p.ws &&
                     !(p.flags & LRCE_EPI_ATOMIC);
  bf16x8 dgp[pf_dg_slots(IM)][NH];
  float4 rsp[pf_rs_slots(IM)][NH][2];
  if (pf_dg || pf_rs) {
#pragma unroll
    for (int i = 0; i < IM; ++i) {
      const int m = m0 + wm * WM + i * 16 + (lane & 15);
      const long long row = m < p.m ? (p.c_map ? (long long)p.c_map[m] : (long long)m) : -1;
#pragma unroll
      for (int h = 0; h < NH; ++h) {
        const int n = ncol + 8 * h;
        const bool ok = row >= 0 && n + 8 <= p.n;
        if (pf_dg && i < pf_dg_slots(IM)) {
          const bf16* src = static_cast<const bf16*>(p.aux) + (ok ? row * p.ld_aux + n : 0);
          dgp[i][h] = *reinterpret_cast<const bf16x8*>(src);
        }
        if (pf_rs && i < pf_rs_slots(IM)) {
          const float* src = static_cast<const float*>(p.aux) + (ok ? row * p.ld_aux + n : 0);
          rsp[i][h][0] = *reinterpret_cast<const float4*>(src);
          rsp[i][h][1] = *reinterpret_cast<const float4*>(src + 4);
        }
      }
    }
  }
  if (nfull > 0 && nfull <= NS) {
    // every K tile has a stage of its own: issue them all now, then consume in order (one
    // round trip for the whole K instead of one per stage turnover)
    constexpr int INFLIGHT = (TBM + TBN) / 32;
    GldsOperand<A_KM, TBM> ga;
    GldsOperand<B_KM, TBN> gb;
    const int wave_u = __builtin_amdgcn_readfirstlane(wave);
    const uint32_t la0 = lds_addr(sa0), lb0 = lds_addr(sb0);
    ga.init(abase, p.lda, p.m, m0, kb, wave, lane);
    gb.init(bbase, p.ldb, p.n, n0, kb, wave, lane);
#pragma unroll
    for (int i = 0; i < NS; ++i)
      if (i < nfull) {
        if (i) { ga.advance(); gb.advance(); }
        ga.issue(la0 + (uint32_t)(i * STG * 2), wave_u);
        gb.issue(lb0 + (uint32_t)(i * STG * 2), wave_u);
      }
    for (int kt = 0; kt < nfull; ++kt) {
      const int ahead = nfull - 1 - kt;   // tiles issued after tile kt
      if (NS >= 4 && ahead >= 3) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(3 * INFLIGHT) : "memory");
      else if (NS >= 3 && ahead == 2) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * INFLIGHT) : "memory");
      else if (ahead == 1) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(INFLIGHT) : "memory");
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      __builtin_amdgcn_sched_barrier(0);
      if (kt == 0) GT_MARK(1);
      compute(sa0 + kt * STG, sb0 + kt * STG);
      __builtin_amdgcn_sched_barrier(0);
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();   // every wave is done with every stage (tail / LDS epilogue reuse)
    __builtin_amdgcn_sched_barrier(0);
  } else if (nfull > 0) {
    // NS-stage ring, one barrier per K tile: at the top of iteration kt this wave waits for its part
    // of tile kt (tiles kt+1 .. kt+NS-2 stay in flight), the barrier makes every wave's part visible
    // AND proves every wave finished tile kt-1, whose stage then receives tile kt+NS-1.
    constexpr int INFLIGHT = (TBM + TBN) / 32;   // glds per wave per K tile
    GldsOperand<A_KM, TBM> ga;
    GldsOperand<B_KM, TBN> gb;
    const int wave_u = __builtin_amdgcn_readfirstlane(wave);
    const uint32_t la0 = lds_addr(sa0), lb0 = lds_addr(sb0);
    ga.init(abase, p.lda, p.m, m0, kb, wave, lane);
    gb.init(bbase, p.ldb, p.n, n0, kb, wave, lane);
    ga.issue(la0, wave_u);
    gb.issue(lb0, wave_u);
#pragma unroll
    for (int i = 1; i < NS - 1; ++i)
      if (i < nfull) {
        ga.advance(); gb.advance();
        ga.issue(la0 + (uint32_t)(i * STG * 2), wave_u);
        gb.issue(lb0 + (uint32_t)(i * STG * 2), wave_u);
      }
    int cur = 0;
    for (int kt = 0; kt < nfull; ++kt) {
      const int ahead = min(NS - 2, nfull - 1 - kt);   // tiles issued after tile kt
      if constexpr (NS >= 4) {
        if (ahead >= 2) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * INFLIGHT) : "memory");
        else if (ahead == 1) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(INFLIGHT) : "memory");
        else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      } else if constexpr (NS == 3) {
        if (ahead >= 1) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(INFLIGHT) : "memory");
        else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      } else {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
      __builtin_amdgcn_s_barrier();
      __builtin_amdgcn_sched_barrier(0);
      if (kt == 0) GT_MARK(1);
      if (kt + NS - 1 < nfull) {
        const int nxt = cur == 0 ? NS - 1 : cur - 1;   // (kt + NS - 1) % NS
        ga.advance(); gb.advance();
        ga.issue(la0 + (uint32_t)(nxt * STG * 2), wave_u);
        gb.issue(lb0 + (uint32_t)(nxt * STG * 2), wave_u);
      }
      compute(sa0 + cur * STG, sb0 + cur * STG);
      __builtin_amdgcn_sched_barrier(0);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // this wave's reads of stage `cur` are done
      cur = cur + 1 == NS ? 0 : cur + 1;
    }
    __builtin_amdgcn_s_barrier();   // every wave is done with every stage (tail / LDS epilogue reuse)
    __builtin_amdgcn_sched_barrier(0);
  }
  if (tail) {
    const int k0 = kb + nfull * BK;
    const int st = nfull % NS;
    tail_tile<A_KM, TBM>(sa0 + st * STG, abase, p.lda, p.m, ke, m0, k0, p.a_map);
    tail_tile<B_KM, TBN>(sb0 + st * STG, bbase, p.ldb, p.n, ke, n0, k0, nullptr);
    __syncthreads();
    compute(sa0 + st * STG, sb0 + st * STG);
    __syncthreads();
  }

  GT_MARK(2);
  if (bias_block && (lane >> 4) == 0) {   // accb row 0 of each C^T block: sum_k A(m, k), m = lane&15
    float* db = const_cast<float*>(p.bias);
#pragma unroll
    for (int i = 0; i < IM; ++i) {
      const int m = m0 + wm * WM + i * 16 + (lane & 15);
      if (m < p.m) __hip_atomic_fetch_add(db + m, alpha_of(p) * accb[i][0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
  char* const cbase = static_cast<char*>(p.c) +   // (grouped: already the entry's C, bz = 0)
                      (long long)bz * p.sc * ((p.flags & (LRCE_EPI_OUT_F32 | LRCE_EPI_ATOMIC | LRCE_EPI_ACCUM)) ? 4 : 2);
  if ((p.flags & LRCE_EPI_ATOMIC) && !p.ws) {
    // split-K partials: stage 32-row slabs through LDS (free now) so each atomic instruction covers
    // consecutive columns of a row.  acc[i][j][r] = C[m = i*16 + (lane&15)][n = j*16 + 4*(lane>>4) + r]
    constexpr int EPW = WN + 4;
    float* E = reinterpret_cast<float*>(lds) + wave * (32 * EPW);
    static_for<IM / 2>([&](auto hc) {
      constexpr int h = decltype(hc)::value;
#pragma unroll
      for (int ii = 0; ii < 2; ++ii)
#pragma unroll
        for (int j = 0; j < JN; ++j)
#pragma unroll
          for (int r = 0; r < 4; ++r)
            E[(ii * 16 + (lane & 15)) * EPW + j * 16 + 4 * (lane >> 4) + r] = acc[2 * h + ii][j][r];
      wave_lds_fence();
      const int col = lane % WN;
      const int n = n0 + wn * WN + col;
      if (n < p.n) {
        for (int rr = lane / WN; rr < 32; rr += 64 / WN) {
          const int m = m0 + wm * WM + h * 32 + rr;
          if (m >= p.m) break;
          const long long row = p.c_map ? (long long)p.c_map[m] : (long long)m;
          if (row < 0) continue;
          const float rs = p.row_scale ? p.row_scale[m / p.rows_per_scale] : 1.f;
          epilogue1(p, E[rr * EPW + col], row, m, n, sk == 0, rs, cbase);
        }
      }
      wave_lds_fence();
    });
    return;
  }
  // Transpose the (lane group g, block j) arrangement of 4-column pieces across the four 16-lane
  // groups with permlane32/16 swaps (cdna_hip_programming.md T21).  JN = 4: lane (g, rho) holds
  // columns 16j + 4g + r of row rho before and 16g + 4j + r after (16 contiguous columns);
  // JN = 2: columns 16j + 4g + r before, 8g + 4j + r after (8 contiguous).  The epilogue then
  // reads/writes 16-B vectors (bias, residual, GELU pre-activation, output).
  auto transpose = [&](auto ic, uint32_t (&u)[JN][4]) {
    constexpr int i = decltype(ic)::value;
#pragma unroll
    for (int j = 0; j < JN; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) u[j][r] = __float_as_uint(acc[i][j][r]);
    if constexpr (JN == 4) {
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const auto s32 = __builtin_amdgcn_permlane32_swap(u[j][r], u[j + 2][r], false, false);
          u[j][r] = s32[0];
          u[j + 2][r] = s32[1];
        }
#pragma unroll
      for (int j = 0; j < 4; j += 2)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const auto s16 = __builtin_amdgcn_permlane16_swap(u[j][r], u[j + 1][r], false, false);
          u[j][r] = s16[0];
          u[j + 1][r] = s16[1];
        }
    } else {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const auto s32 = __builtin_amdgcn_permlane32_swap(u[0][r], u[1][r], false, false);
        const auto s16 = __builtin_amdgcn_permlane16_swap(s32[0], s32[1], false, false);
        u[0][r] = s16[0];
        u[1][r] = s16[1];
      }
    }
  };
  if (p.ws) {
    // split-K slab: this slice's alpha * partial tile, plain stores (reduced by splitk_reduce_kernel)
    float* slab = p.ws + (long long)sk * p.m * p.n;
    const bool vec4 = (p.n & 3) == 0;
    const float al = alpha_of(p);
    static_for<IM>([&](auto ic) {
      uint32_t u[JN][4];
      transpose(ic, u);
      const int m = m0 + wm * WM + decltype(ic)::value * 16 + (lane & 15);
      if (m < p.m) {
        float* row = slab + (long long)m * p.n;
#pragma unroll
        for (int j = 0; j < JN; ++j) {
          const int n = ncol + 4 * j;
          const float4 v = make_float4(__uint_as_float(u[j][0]) * al, __uint_as_float(u[j][1]) * al,
                                       __uint_as_float(u[j][2]) * al, __uint_as_float(u[j][3]) * al);
          if (vec4 && n + 4 <= p.n) {
            *reinterpret_cast<float4*>(row + n) = v;
          } else {
            if (n < p.n) row[n] = v.x;
            if (n + 1 < p.n) row[n + 1] = v.y;
            if (n + 2 < p.n) row[n + 2] = v.z;
            if (n + 3 < p.n) row[n + 3] = v.w;
          }
        }
      }
    });
    return;
  }
  // every global operand of the epilogue is loaded here, before its first store (EpiPf)
  const float al_pf = alpha_of(p);
  float4 bias_pf[NH][2];
  const bool have_bias = (p.flags & LRCE_EPI_BIAS) && sk == 0 && p.vec;
#pragma unroll
  for (int h = 0; h < NH; ++h) {
    const int n = ncol + 8 * h;
    const bool ok = have_bias && n + 8 <= p.n;
    bias_pf[h][0] = ok ? *reinterpret_cast<const float4*>(p.bias + n) : make_float4(0.f, 0.f, 0.f, 0.f);
    bias_pf[h][1] = ok ? *reinterpret_cast<const float4*>(p.bias + n + 4) : make_float4(0.f, 0.f, 0.f, 0.f);
  }
  long long row_pf[IM];
  float rsc_pf[IM];
#pragma unroll
  for (int i = 0; i < IM; ++i) {
    const int m = m0 + wm * WM + i * 16 + (lane & 15);
    row_pf[i] = m < p.m ? (p.c_map ? (long long)p.c_map[m] : (long long)m) : -1;
    rsc_pf[i] = (p.row_scale && m < p.m) ? p.row_scale[m / p.rows_per_scale] : 1.f;
  }
  // the dGELU pre-activation of a deeper K (not prefetched before the K loop): all of it now
  const bool late_dg = (p.flags & LRCE_EPI_DGELU) && p.vec && !pf_dg && !p.ws && !(p.flags & LRCE_EPI_ATOMIC);
  if (late_dg) {
#pragma unroll
    for (int i = 0; i < pf_dg_slots(IM); ++i)
#pragma unroll
      for (int h = 0; h < NH; ++h) {
        const int n = ncol + 8 * h;
        const bool ok = row_pf[i] >= 0 && n + 8 <= p.n;
        dgp[i][h] = *reinterpret_cast<const bf16x8*>(static_cast<const bf16*>(p.aux) + (ok ? row_pf[i] * p.ld_aux + n : 0));
      }
  }
  // the f32 residual / accumulated C (read-modify-write) of RC row blocks at a time: one memory round
  // trip per RC row blocks behind the stores already issued, instead of one per 8-column chunk
  constexpr int RC = IM >= 5 ? 1 : 2;
  const bool late_rs = (p.flags & LRCE_EPI_RESID) && sk == 0 && p.vec && !pf_rs && !p.ws && !(p.flags & LRCE_EPI_ATOMIC);
  const bool late_acc = (p.flags & LRCE_EPI_ACCUM) && !(p.flags & LRCE_EPI_RESID) && p.vec && !p.ws &&
                        !(p.flags & LRCE_EPI_ATOMIC);
  static_for<(IM + RC - 1) / RC>([&](auto cc) {
    constexpr int c0 = decltype(cc)::value * RC;
    float4 xq[RC][NH][2];
    if (late_rs || late_acc) {
#pragma unroll
      for (int ii = 0; ii < RC; ++ii) {
        if (c0 + ii >= IM) break;
#pragma unroll
        for (int h = 0; h < NH; ++h) {
          const int n = ncol + 8 * h;
          const long long rw = row_pf[c0 + ii < IM ? c0 + ii : 0];
          const bool ok = rw >= 0 && n + 8 <= p.n;
          const float* src = late_rs ? static_cast<const float*>(p.aux) + (ok ? rw * p.ld_aux + n : 0)
                                     : reinterpret_cast<const float*>(cbase) + (ok ? rw * p.ldc + n : 0);
          xq[ii][h][0] = *reinterpret_cast<const float4*>(src);
          xq[ii][h][1] = *reinterpret_cast<const float4*>(src + 4);
        }
      }
    }
    static_for<RC>([&](auto iic) {
      constexpr int i = c0 + decltype(iic)::value;
      if constexpr (i < IM) {
        uint32_t u[JN][4];
        transpose(std::integral_constant<int, i>{}, u);
        const int m = m0 + wm * WM + i * 16 + (lane & 15);
#pragma unroll
        for (int h = 0; h < JN / 2; ++h) {
          float v[8];
#pragma unroll
          for (int e = 0; e < 8; ++e) v[e] = __uint_as_float(u[2 * h + (e >> 2)][e & 3]);
          const bf16x8* dg = ((pf_dg || late_dg) && i < pf_dg_slots(IM)) ? &dgp[i < pf_dg_slots(IM) ? i : 0][h] : nullptr;
          const float4* rs = (pf_rs && i < pf_rs_slots(IM)) ? rsp[i < pf_rs_slots(IM) ? i : 0][h]
                             : late_rs ? xq[decltype(iic)::value][h] : nullptr;
          const float4* ac = late_acc ? xq[decltype(iic)::value][h] : nullptr;
          const EpiPf pf{1, al_pf, row_pf[i], rsc_pf[i], have_bias ? bias_pf[h] : nullptr};
          epilogue8<F16, DROP>(p, v, m, ncol + 8 * h, sk, cbase, dg, rs, &pf, ac);
        }
      }
    });
  });
  GT_MARK(3);   // epilogue math done, stores issued
#ifdef LRCE_GEMM_TRACE
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // the stores have left this wave
#endif
  GT_MARK(4);
}

// C[m][n] += sum_s ws[s][m][n]  (n % 4 == 0, ldc % 4 == 0)
__global__ void splitk_reduce_kernel(const float* __restrict__ ws, int split, int m, int n, float* __restrict__ c, long long ldc) {
  const long long mn = (long long)m * n;
  const long long e = ((long long)blockIdx.x * blockDim.x + threadIdx.x) * 4;
  if (e >= mn) return;
  float4 s = *reinterpret_cast<const float4*>(ws + e);
  for (int k = 1; k < split; ++k) {
    const float4 t = *reinterpret_cast<const float4*>(ws + k * mn + e);
    s.x += t.x; s.y += t.y; s.z += t.z; s.w += t.w;
  }
  float4* cp = reinterpret_cast<float4*>(c + (e / n) * ldc + (e % n));
  float4 o = *cp;
  o.x += s.x; o.y += s.y; o.z += s.z; o.w += s.w;
  *cp = o;
}

// Split-K of a linear with a bias / dropout / residual epilogue (the 320-row BERT output projections,
// K = 3072): out[m][n] = resid[m][n] + drop(sum_s ws[s][m][n] + bias[n]) (f32 out, n % 4 == 0), the
// dropout mask of lrce_dropout over the contiguous [m][n] result (element m * n + col, drop_group 1).
__global__ void splitk_reduce_epi_kernel(const float* __restrict__ ws, int split, int m, int n, const float* __restrict__ bias,
                                         const float* __restrict__ resid, long long ld_res, float p, uint64_t seed,
                                         const uint64_t* __restrict__ off, float* __restrict__ c, long long ldc) {
  const long long mn = (long long)m * n;
  const long long e = ((long long)blockIdx.x * blockDim.x + threadIdx.x) * 4;
  if (e >= mn) return;
  float4 s = *reinterpret_cast<const float4*>(ws + e);
  for (int k = 1; k < split; ++k) {
    const float4 t = *reinterpret_cast<const float4*>(ws + k * mn + e);
    s.x += t.x; s.y += t.y; s.z += t.z; s.w += t.w;
  }
  const long long r = e / n, col = e % n;
  if (bias) {
    const float4 b = *reinterpret_cast<const float4*>(bias + col);
    s.x += b.x; s.y += b.y; s.z += b.z; s.w += b.w;
  }
  if (p > 0.f) {
    const float4 u = lrce_uniform4(lrce_seed(seed, off), (unsigned long long)e >> 2);
    const float kd = 1.0f - p;
    s.x = u.x >= p ? s.x / kd : 0.f; s.y = u.y >= p ? s.y / kd : 0.f;
    s.z = u.z >= p ? s.z / kd : 0.f; s.w = u.w >= p ? s.w / kd : 0.f;
  }
  if (resid) {
    const float4 q = *reinterpret_cast<const float4*>(resid + r * ld_res + col);
    s.x += q.x; s.y += q.y; s.z += q.z; s.w += q.w;
  }
  *reinterpret_cast<float4*>(c + r * ldc + col) = s;
}

// Deep splits (small weight gradients over many rows: 100+ slices of a 384 x 128 tile) would leave
// the one-thread-per-float4 reduce above with a few waves each walking every slab serially; here a
// block is 64 float4 columns x 4 slice groups, each thread keeps 4 slab loads in flight, and the
// groups meet in LDS.
// slab reads: each slab element is read exactly once (a non-temporal hint measured no faster)
__device__ __forceinline__ float4 ld_slab(const float* q) { return *reinterpret_cast<const float4*>(q); }

__global__ void __launch_bounds__(256) splitk_reduce_deep_kernel(const float* __restrict__ ws, int split, int m, int n,
                                                                 float* __restrict__ c, long long ldc) {
  const long long mn = (long long)m * n;
  const int lane = threadIdx.x & 63, g = threadIdx.x >> 6;
  const long long e = ((long long)blockIdx.x * 64 + lane) * 4;
  float4 s = make_float4(0.f, 0.f, 0.f, 0.f);
  auto add = [&](const float4& t) { s.x += t.x; s.y += t.y; s.z += t.z; s.w += t.w; };
  if (e < mn) {
    int k = g;
    for (; k + 12 < split; k += 16) {
      const float4 t0 = ld_slab(ws + k * mn + e);
      const float4 t1 = ld_slab(ws + (k + 4) * mn + e);
      const float4 t2 = ld_slab(ws + (k + 8) * mn + e);
      const float4 t3 = ld_slab(ws + (k + 12) * mn + e);
      add(t0); add(t1); add(t2); add(t3);
    }
    for (; k < split; k += 4) add(ld_slab(ws + k * mn + e));
  }
  __shared__ float4 red[4][64];
  red[g][lane] = s;
  __syncthreads();
  if (g == 0 && e < mn) {
    const float4 a = red[1][lane], b = red[2][lane], d = red[3][lane];
    float4* cp = reinterpret_cast<float4*>(c + (e / n) * ldc + (e % n));
    float4 o = *cp;
    o.x += s.x + a.x + b.x + d.x; o.y += s.y + a.y + b.y + d.y;
    o.z += s.z + a.z + b.z + d.z; o.w += s.w + a.w + b.w + d.w;
    *cp = o;
  }
}

}  // namespace

int lrce_gemm_f32(const LrceGemmDesc* d, void* stream);

extern "C" int lrce_colsum(const void* x, int x_f32, const int32_t* row_map, int64_t ld, int m, int n, const float* row_scale,
                           int rows_per_scale, float* out, void* stream);

static int gemm_dispatch(const LrceGemmDesc* d, void* stream);
static bool glds_ok(const LrceGemmDesc* d);
bool lrce_gemm_f32_outer_ok(const LrceGemmDesc* d);

extern "C" int lrce_gemm(const LrceGemmDesc* d, void* stream) {
  if (d && d->drop_p > 0.f && !d->b_f32 &&
      (!glds_ok(d) || d->drop_group > 1 || (d->split_k > 1 && !d->workspace) || d->batch != 1 || d->c_map ||
       (d->flags & (LRCE_EPI_ATOMIC | LRCE_EPI_ACCUM | LRCE_EPI_BIAS_GRAD))))
    return lrce_fail(LRCE_E_ARG, "gemm: fused dropout needs the exact-f32 skinny path or the 16-bit LDS-DMA path "
                                 "(drop_group 1, one K slice, batch 1, no c_map / accumulate)");
  if (!d || !d->a || !d->b || !d->c) return lrce_fail(LRCE_E_ARG, "gemm: null pointer");
  if (d->f16 && (d->a_f32 || d->b_f32)) return lrce_fail(LRCE_E_ARG, "gemm: f16 operands cannot be combined with f32 A/B");
  if (!(d->flags & LRCE_EPI_BIAS_GRAD)) return gemm_dispatch(d, stream);
  // bias gradient of a weight-gradient GEMM: db[m] += sum_k A(m, k)
  if (d->a_kmajor || !d->bias) return lrce_fail(LRCE_E_ARG, "gemm: BIAS_GRAD needs M-major A and bias");
  if (d->flags & LRCE_EPI_BIAS) return lrce_fail(LRCE_E_ARG, "gemm: BIAS and BIAS_GRAD are exclusive");
  // batched (BERT's query / key / value weight gradients): LDS-DMA path, one K slice, a bias per batch
  if (d->batch != 1 && (d->b_f32 || !glds_ok(d) || d->split_k > 1 || d->stride_bias <= 0))
    return lrce_fail(LRCE_E_ARG, "gemm: batched BIAS_GRAD needs the 16-bit LDS-DMA path, split_k 1 and stride_bias > 0");
  const bool fused = d->b_f32 ? lrce_gemm_f32_outer_ok(d) : glds_ok(d);
  if (fused) return gemm_dispatch(d, stream);   // the skinny outer-product kernel sums A as it goes
  LrceGemmDesc g = *d;
  g.flags &= ~LRCE_EPI_BIAS_GRAD;
  g.bias = nullptr;
  if (int rc = gemm_dispatch(&g, stream)) return rc;
  if (d->alpha != 1.0f || d->alpha_dev) return lrce_fail(LRCE_E_ARG, "gemm: BIAS_GRAD with alpha != 1 off the fused paths");
  return lrce_colsum(d->a, d->a_f32, d->a_map, d->lda, d->k, d->m, d->a_row_scale, d->a_rows_per_scale,
                     const_cast<float*>(d->bias), stream);
}

// LDS-DMA path: bf16 operands with 16-B aligned rows; K-major A may carry a row map
// (no row map: the DMA addresses are 32-bit byte offsets from the operand base, bounded here)
static bool glds_ok(const LrceGemmDesc* d) {
  auto al16 = [](const void* q) { return (reinterpret_cast<uintptr_t>(q) & 15) == 0; };
  const long long ext_a = d->a_kmajor ? (long long)d->m * d->lda + d->k : (long long)d->k * d->lda + d->m;
  const long long ext_b = d->b_kmajor ? (long long)d->n * d->ldb + d->k : (long long)d->k * d->ldb + d->n;
  return !d->a_f32 && !d->b_f32 && al16(d->a) && al16(d->b) && (d->stride_a % 8 == 0) && (d->stride_b % 8 == 0) &&
         (d->lda % 8 == 0) && (d->ldb % 8 == 0) && !d->a_map && ext_a * 2 < (1LL << 31) && ext_b * 2 < (1LL << 31);
}

static int gemm_dispatch(const LrceGemmDesc* d, void* stream) {
  if (d->m <= 0 || d->n <= 0 || d->k <= 0 || d->batch <= 0) return lrce_fail(LRCE_E_ARG, "gemm: empty shape");
  if ((d->flags & LRCE_EPI_AUX_F32) && !d->b_f32)
    return lrce_fail(LRCE_E_ARG, "gemm: AUX_F32 (f32 pre-activation) is an exact-f32 path flag");
  if ((d->flags & (LRCE_EPI_DGELU | LRCE_EPI_RESID)) && !d->aux) return lrce_fail(LRCE_E_ARG, "gemm: aux missing");
  if ((d->flags & (LRCE_EPI_AUX_OUT | LRCE_EPI_OUT_BOTH)) && !d->aux_out) return lrce_fail(LRCE_E_ARG, "gemm: aux_out missing");
  if ((d->flags & LRCE_EPI_BIAS) && !d->bias) return lrce_fail(LRCE_E_ARG, "gemm: bias missing");
  if (d->b_f32) {
    if (d->alpha_dev) return lrce_fail(LRCE_E_ARG, "gemm: alpha_dev is not supported on the f32 / fp16-weight skinny path");
    return lrce_gemm_f32(d, stream);
  }
  // vector loads need the contiguous dim of every operand to be a multiple of 8 elements
  if (d->a_kmajor ? (d->k % 8) : (d->m % 8)) return lrce_fail(LRCE_E_ARG, "gemm: A contiguous dim %% 8 != 0");
  if (d->b_kmajor ? (d->k % 8) : (d->n % 8)) return lrce_fail(LRCE_E_ARG, "gemm: B contiguous dim %% 8 != 0");
  if ((d->lda % 8) || (d->ldb % 8)) return lrce_fail(LRCE_E_ARG, "gemm: lda/ldb %% 8 != 0");
  const int split = d->split_k > 1 ? d->split_k : 1;
  // split-K with an epilogue (bias / residual / f32 out / dropout): f32 slabs + splitk_reduce_epi_kernel
  const bool epi_split = split > 1 && !(d->flags & LRCE_EPI_ATOMIC) && d->workspace &&
                         (d->flags & ~(LRCE_EPI_BIAS | LRCE_EPI_RESID | LRCE_EPI_OUT_F32)) == 0 && (d->flags & LRCE_EPI_OUT_F32) &&
                         d->batch == 1 && !d->c_map && !d->row_scale && d->scale_cols == 0 && d->n % 4 == 0 &&
                         d->ldc % 4 == 0 && (!d->aux || d->ld_aux % 4 == 0) && d->drop_group <= 1 &&
                         d->workspace_elems >= (int64_t)split * d->m * d->n;
  if (split > 1 && !(d->flags & (LRCE_EPI_ATOMIC | LRCE_EPI_SLABS)) && !epi_split)
    return lrce_fail(LRCE_E_ARG, "gemm: split_k needs ATOMIC, SLABS, or a workspace and only BIAS / RESID / OUT_F32 epilogues");
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
  p.sbias = d->batch > 1 ? d->stride_bias : 0;
  p.aux_out = static_cast<bf16*>(d->aux_out); p.ld_aux_out = d->ld_aux_out;
  p.a_map = d->a_map; p.c_map = d->c_map;
  p.alpha = d->alpha; p.alpha_dev = d->alpha_dev; p.salpha = d->batch > 1 ? d->stride_alpha : 0; p.scale_cols = d->scale_cols; p.scale_val = d->scale_val;
  p.trace = g_gemm_trace;
  p.row_scale = d->row_scale; p.rows_per_scale = d->rows_per_scale > 0 ? d->rows_per_scale : 1;
  p.a_row_scale = d->a_row_scale; p.a_rows_per_scale = d->a_rows_per_scale > 0 ? d->a_rows_per_scale : 1;
  if (p.a_row_scale && !d->a_f32) return lrce_fail(LRCE_E_ARG, "gemm: a_row_scale needs f32 A");
  p.tiles_m = (d->m + BM - 1) / BM; p.tiles_n = (d->n + BN - 1) / BN;
  // grouped raster for the weight gradients (M-major A: split-K over tokens, 4-16 x 4-16 tiles per split,
  // 512x2048x17640 64.9 -> 58.0 us); the token-major forward / dX shapes measured 1-3 % better row-major
  p.group_m = d->a_kmajor ? 1 : 4;
  auto al16 = [](const void* q) { return (reinterpret_cast<uintptr_t>(q) & 15) == 0; };
  const bool out32 = d->flags & (LRCE_EPI_OUT_F32 | LRCE_EPI_ATOMIC | LRCE_EPI_ACCUM);
  p.vec = (d->n % 8 == 0) && (d->ldc % 8 == 0) && al16(d->c) && (d->stride_c % 8 == 0) && (d->scale_cols % 8 == 0) &&
          (!d->bias || (al16(d->bias) && p.sbias % 4 == 0)) && (!d->aux || (al16(d->aux) && d->ld_aux % 8 == 0)) &&
          (!d->aux_out || (al16(d->aux_out) && d->ld_aux_out % 8 == 0));
  (void)out32;
  p.ws = nullptr;
  p.f16 = d->f16 ? 1 : 0;
  p.drop_p = d->drop_p > 0.f ? d->drop_p : 0.f;
  p.drop_seed = d->drop_seed;
  p.rng_off = p.drop_p > 0.f ? lrce_rng_offset() : nullptr;
  if (p.f16 && !glds_ok(d))
    return lrce_fail(LRCE_E_ARG, "gemm: f16 needs 16-B aligned bf16-layout operands (LDS-DMA path)");
  // slabs only (LRCE_EPI_SLABS): the split slices' partials for a consumer kernel, no reduce launch
  const bool slabs_only = (d->flags & LRCE_EPI_SLABS) != 0;
  if (slabs_only && (split < 2 || !d->workspace || d->workspace_elems < (int64_t)split * d->m * d->n || d->batch != 1 ||
                     (d->flags & ~LRCE_EPI_SLABS) || d->c_map || d->row_scale || d->n % 4 || !glds_ok(d)))
    return lrce_fail(LRCE_E_ARG, "gemm: LRCE_EPI_SLABS needs split_k > 1, a workspace of split*m*n, the LDS-DMA path and no other epilogue");
  const bool use_ws = slabs_only || (epi_split || (d->workspace && split > 1 && (d->flags & ~(LRCE_EPI_ATOMIC | LRCE_EPI_BIAS_GRAD)) == 0 &&
                                     (d->flags & LRCE_EPI_ATOMIC) && d->batch == 1 && !d->c_map && !d->row_scale &&
                                     d->scale_cols == 0 && d->n % 4 == 0 && d->ldc % 4 == 0 &&
                                     d->workspace_elems >= (int64_t)split * d->m * d->n)) &&
                      (reinterpret_cast<uintptr_t>(d->c) & 15) == 0 && glds_ok(d);
  if (epi_split && !use_ws) return lrce_fail(LRCE_E_ARG, "gemm: split-K epilogue needs the 16-bit LDS-DMA path and a 16-B aligned C");
  if (epi_split) p.drop_p = 0.f;   // the reduce launch applies bias / dropout / residual
  if (use_ws) p.ws = d->workspace;
  dim3 grid(p.tiles_m * p.tiles_n, d->batch * split);
  hipStream_t s = static_cast<hipStream_t>(stream);
  if (glds_ok(d)) {
    // 128x128 tiles when they give every CU work; 64x64 otherwise (small-M / small-N problems)
    const int t128 = p.tiles_m * p.tiles_n * d->batch * split;
    // (fused dropout: 64x64 tiles only — the one instantiation family that carries that epilogue)
    const bool small = t128 < 256 || p.drop_p > 0.f;
    // Taller tiles (K-major A only): 160 or 192 rows x 128 do 1.25x / 1.5x the work of a 128x128
    // tile, so they win when the 128-row tile count overshoots a round of the 2-blocks-per-CU grid.
    // Pick the height minimising rounds x rows (e.g. M 17 640, N 512: 552 -> 444 tiles in ONE round
    // at 160 rows; N 2048: 3 rounds of 192-row tiles beat 4 of 160 and 5 of 128).
    int tall_m = 0;
    if (!small && d->a_kmajor) {
      const int slots = 2 * 256;
      const bool atomic_rows = (d->flags & LRCE_EPI_ATOMIC) && !p.ws;   // its LDS-slab epilogue wants an even row-block count
      long long best = (long long)((t128 + slots - 1) / slots) * 128;
      for (int h : {160, 192}) {
        if (h == 160 && atomic_rows) continue;
        const long long th = (long long)((d->m + h - 1) / h) * p.tiles_n * d->batch * split;
        const long long cost = (th + slots - 1) / slots * h;
        if (cost < best) { best = cost; tall_m = h; }
      }
    }
    if (small) {
      p.tiles_m = (d->m + 63) / 64; p.tiles_n = (d->n + 63) / 64;
      grid = dim3(p.tiles_m * p.tiles_n, d->batch * split);
    } else if (tall_m) {
      p.tiles_m = (d->m + tall_m - 1) / tall_m;
      grid = dim3(p.tiles_m * p.tiles_n, d->batch * split);
    }
    const int gk = (d->a_kmajor ? 2 : 0) | (d->b_kmajor ? 1 : 0) | (small ? 4 : 0) | (tall_m == 192 ? 8 : 0) |
                   (tall_m == 160 ? 16 : 0) | (p.f16 ? 32 : 0);
    auto launch = [&](auto nsc) {
      constexpr int S = decltype(nsc)::value;
      switch (gk) {
        case 32 + 11: gemm_glds_kernel<192, 128, true, true, true, S><<<grid, NT, 0, s>>>(p); break;
        case 32 + 19: gemm_glds_kernel<160, 128, true, true, true, S><<<grid, NT, 0, s>>>(p); break;
        case 32 + 3: gemm_glds_kernel<128, 128, true, true, true, S><<<grid, NT, 0, s>>>(p); break;
        case 32 + 7: gemm_glds_kernel<64, 64, true, true, true, S><<<grid, NT, 0, s>>>(p); break;
        // fp16 backward (BERT, scaled gradients): dX = dY W (B N-major) and dW = dY^T X (both M/N-major)
        case 32 + 10: gemm_glds_kernel<192, 128, true, false, true, S><<<grid, NT, 0, s>>>(p); break;
        case 32 + 18: gemm_glds_kernel<160, 128, true, false, true, S><<<grid, NT, 0, s>>>(p); break;
        case 32 + 2: gemm_glds_kernel<128, 128, true, false, true, S><<<grid, NT, 0, s>>>(p); break;
        case 32 + 6: gemm_glds_kernel<64, 64, true, false, true, S><<<grid, NT, 0, s>>>(p); break;
        case 32 + 0: gemm_glds_kernel<128, 128, false, false, true, S><<<grid, NT, 0, s>>>(p); break;
        case 32 + 4: gemm_glds_kernel<64, 64, false, false, true, S><<<grid, NT, 0, s>>>(p); break;
        default: return lrce_fail(LRCE_E_ARG, "gemm: no LDS-DMA kernel for operand layout key %d", gk);
        case 11: gemm_glds_kernel<192, 128, true, true, false, S><<<grid, NT, 0, s>>>(p); break;
        case 10: gemm_glds_kernel<192, 128, true, false, false, S><<<grid, NT, 0, s>>>(p); break;
        case 19: gemm_glds_kernel<160, 128, true, true, false, S><<<grid, NT, 0, s>>>(p); break;
        case 18: gemm_glds_kernel<160, 128, true, false, false, S><<<grid, NT, 0, s>>>(p); break;
        case 3: gemm_glds_kernel<128, 128, true, true, false, S><<<grid, NT, 0, s>>>(p); break;
        case 2: gemm_glds_kernel<128, 128, true, false, false, S><<<grid, NT, 0, s>>>(p); break;
        case 1: gemm_glds_kernel<128, 128, false, true, false, S><<<grid, NT, 0, s>>>(p); break;
        case 0: gemm_glds_kernel<128, 128, false, false, false, S><<<grid, NT, 0, s>>>(p); break;
        case 7: gemm_glds_kernel<64, 64, true, true, false, S><<<grid, NT, 0, s>>>(p); break;
        case 6: gemm_glds_kernel<64, 64, true, false, false, S><<<grid, NT, 0, s>>>(p); break;
        case 5: gemm_glds_kernel<64, 64, false, true, false, S><<<grid, NT, 0, s>>>(p); break;
        case 4: gemm_glds_kernel<64, 64, false, false, false, S><<<grid, NT, 0, s>>>(p); break;
      }
      return (int)LRCE_OK;
    };
    // two stages: a third (one resident workgroup per CU) measured 1.3-1.5x slower on every step shape.
    // 64x64 tiles (small problems: few workgroups, each latency-bound on its operand stream) take a
    // 4-stage ring in the same 64 KB of LDS as two 128x128 stages, so three K tiles are in flight
    // per workgroup instead of one
    auto launch_small = [&](auto nsc) {
      constexpr int S = decltype(nsc)::value;
      if (p.drop_p > 0.f) {
        switch (gk) {
          case 32 + 7: gemm_glds_kernel<64, 64, true, true, true, S, true><<<grid, NT, 0, s>>>(p); break;
          case 7: gemm_glds_kernel<64, 64, true, true, false, S, true><<<grid, NT, 0, s>>>(p); break;
          default: return lrce_fail(LRCE_E_ARG, "gemm: fused dropout needs K-major A and B (key %d)", gk);
        }
        return (int)LRCE_OK;
      }
      switch (gk) {
        case 32 + 7: gemm_glds_kernel<64, 64, true, true, true, S><<<grid, NT, 0, s>>>(p); break;
        case 32 + 6: gemm_glds_kernel<64, 64, true, false, true, S><<<grid, NT, 0, s>>>(p); break;
        case 32 + 4: gemm_glds_kernel<64, 64, false, false, true, S><<<grid, NT, 0, s>>>(p); break;
        case 7: gemm_glds_kernel<64, 64, true, true, false, S><<<grid, NT, 0, s>>>(p); break;
        case 6: gemm_glds_kernel<64, 64, true, false, false, S><<<grid, NT, 0, s>>>(p); break;
        case 5: gemm_glds_kernel<64, 64, false, true, false, S><<<grid, NT, 0, s>>>(p); break;
        case 4: gemm_glds_kernel<64, 64, false, false, false, S><<<grid, NT, 0, s>>>(p); break;
        default: return lrce_fail(LRCE_E_ARG, "gemm: no LDS-DMA kernel for operand layout key %d", gk);
      }
      return (int)LRCE_OK;
    };
    if (small) {
      if (int rc = launch_small(std::integral_constant<int, 4>{})) return rc;
    } else if (int rc = launch(std::integral_constant<int, 2>{})) {
      return rc;
    }
    if (slabs_only) {
      // the consumer reduces
    } else if (p.ws && epi_split) {
      const long long q4 = (long long)d->m * d->n / 4;
      splitk_reduce_epi_kernel<<<(unsigned)((q4 + 255) / 256), 256, 0, s>>>(
          p.ws, split, d->m, d->n, (d->flags & LRCE_EPI_BIAS) ? d->bias : nullptr,
          (d->flags & LRCE_EPI_RESID) ? static_cast<const float*>(d->aux) : nullptr, d->ld_aux, d->drop_p > 0.f ? d->drop_p : 0.f,
          d->drop_seed, d->drop_p > 0.f ? lrce_rng_offset() : nullptr, static_cast<float*>(d->c), d->ldc);
    } else if (p.ws) {
      const long long q4 = (long long)d->m * d->n / 4;
      if (split >= 8)
        splitk_reduce_deep_kernel<<<(unsigned)((q4 + 63) / 64), 256, 0, s>>>(
            p.ws, split, d->m, d->n, static_cast<float*>(d->c), d->ldc);
      else
        splitk_reduce_kernel<<<(unsigned)((q4 + 255) / 256), 256, 0, s>>>(p.ws, split, d->m, d->n, static_cast<float*>(d->c), d->ldc);
    }
    return lrce_check_launch("gemm(glds)");
  }
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

// Weight gradients of n linears in grouped launches: dW_e (=|+=) sum_k dY_e[k][m] X_e[k][n] (A M-major =
// dY_e, B N-major = X_e, C_e f32), db_e[m] += sum_k dY_e[k][m] for entries with BIAS_GRAD.  One K slice
// per tile (no split-K slabs, no reduce launch): the entries' summed tile count fills the chip.  All
// entries share K (the token count) and alpha; up to GPT entries / GSH distinct shapes per launch.
extern "C" int lrce_gemm_grouped(const LrceGemmItem* it, int n, int k, float alpha, void* stream) {
  if (n < 0 || (n > 0 && !it) || k <= 0) return lrce_fail(LRCE_E_ARG, "gemm_grouped: n=%d k=%d", n, k);
  auto al16 = [](const void* q) { return (reinterpret_cast<uintptr_t>(q) & 15) == 0; };
  for (int i = 0; i < n; ++i) {
    const LrceGemmItem& e = it[i];
    const int cf = e.flags & (LRCE_EPI_ACCUM | LRCE_EPI_OUT_F32);
    const bool bg = e.flags & LRCE_EPI_BIAS_GRAD;
    if ((e.flags & ~(LRCE_EPI_ACCUM | LRCE_EPI_OUT_F32 | LRCE_EPI_BIAS_GRAD)) ||
        (cf != LRCE_EPI_ACCUM && cf != LRCE_EPI_OUT_F32) || (bg && !e.bias))
      return lrce_fail(LRCE_E_ARG, "gemm_grouped: entry %d flags %d (ACCUM or OUT_F32 [| BIAS_GRAD with a bias])", i, e.flags);
    if (e.m <= 0 || e.n <= 0 || e.m % 8 || e.n % 8 || e.lda < e.m || e.ldb < e.n || e.ldc < e.n || e.lda % 8 ||
        e.ldb % 8 || e.ldc % 8)
      return lrce_fail(LRCE_E_ARG, "gemm_grouped: entry %d m=%d n=%d lda=%d ldb=%d ldc=%d", i, e.m, e.n, e.lda, e.ldb, e.ldc);
    if (e.split > 1 && (cf != LRCE_EPI_OUT_F32 || e.k_chunk <= 0 || e.k_chunk % BK || (long long)(e.split - 1) * e.k_chunk >= k ||
                        (long long)e.split * e.k_chunk < k))
      return lrce_fail(LRCE_E_ARG, "gemm_grouped: entry %d split %d x k_chunk %d over k=%d (slabs are stored: OUT_F32)", i,
                       e.split, e.k_chunk, k);
    if (e.split < 0 || e.split > 4096) return lrce_fail(LRCE_E_ARG, "gemm_grouped: entry %d split %d", i, e.split);
    if (((long long)k * e.lda + e.m) * 2 >= (1LL << 31) || ((long long)k * e.ldb + e.n) * 2 >= (1LL << 31))
      return lrce_fail(LRCE_E_ARG, "gemm_grouped: entry %d operand extent over 2 GB", i);
    if (!e.a || !e.b || !e.c || !al16(e.a) || !al16(e.b) || !al16(e.c) || (bg && !al16(e.bias)) ||
        (reinterpret_cast<uintptr_t>(e.alpha_dev) & 3) || (e.f16 != 0 && e.f16 != 1))
      return lrce_fail(LRCE_E_ARG, "gemm_grouped: entry %d null, misaligned or f16=%d", i, e.f16);
  }
  hipStream_t s = static_cast<hipStream_t>(stream);
  constexpr long long SPAN = (1LL << 31) - 1;   // f32 elements an offset from the chunk's base may reach
  int i = 0;
  while (i < n) {
    // one launch: entries i .. j-1, as many as fit the tables and keep C / bias within an int offset
    GemmPT p{};
    p.k = k; p.split_k = 1; p.batch = 1;
    p.k_chunk = (k + BK - 1) / BK * BK;
    p.alpha = alpha; p.scale_val = 1.f; p.rows_per_scale = 1; p.a_rows_per_scale = 1;
    p.group_m = 4;
    p.vec = 1;
    p.trace = g_gemm_trace;
    uintptr_t clo = ~(uintptr_t)0, chi = 0, blo = ~(uintptr_t)0, bhi = 0, alo = ~(uintptr_t)0, ahi = 0;
    int nsh = 0, j = i, tiles = 0;
    const int f16 = it[i].f16;
    for (; j < n && j - i < GPT; ++j) {
      const LrceGemmItem& e = it[j];
      if (e.f16 != f16) break;   // one operand format per launch
      int si = 0;
      const int sp = e.split > 1 ? e.split : 1, kc = e.split > 1 ? e.k_chunk : 0;
      while (si < nsh && !(p.sh[si].m == e.m && p.sh[si].n == e.n && p.sh[si].lda == e.lda && p.sh[si].ldb == e.ldb &&
                           p.sh[si].ldc == e.ldc && p.sh[si].split == sp && p.sh[si].k_chunk == kc))
        ++si;
      if (si == nsh && nsh == GSH) break;
      const uintptr_t c0 = reinterpret_cast<uintptr_t>(e.c);
      const uintptr_t c1 = c0 + ((uintptr_t)(sp - 1) * e.m * e.ldc + (uintptr_t)(e.m - 1) * e.ldc + e.n) * 4;
      const uintptr_t nclo = c0 < clo ? c0 : clo, nchi = c1 > chi ? c1 : chi;
      if ((long long)((nchi - nclo) / 4) > SPAN) break;
      uintptr_t nblo = blo, nbhi = bhi;
      if (e.flags & LRCE_EPI_BIAS_GRAD) {
        const uintptr_t b0 = reinterpret_cast<uintptr_t>(e.bias), b1 = b0 + (uintptr_t)sp * e.m * 4;
        nblo = b0 < blo ? b0 : blo; nbhi = b1 > bhi ? b1 : bhi;
        if ((long long)((nbhi - nblo) / 4) > SPAN) break;
      }
      uintptr_t nalo = alo, nahi = ahi;
      if (e.alpha_dev) {
        const uintptr_t a0 = reinterpret_cast<uintptr_t>(e.alpha_dev), a1 = a0 + 4;
        nalo = a0 < alo ? a0 : alo; nahi = a1 > ahi ? a1 : ahi;
        if ((long long)((nahi - nalo) / 4) > SPAN) break;
      }
      const int tm = (e.m + BM - 1) / BM, tn = (e.n + BN - 1) / BN;
      if ((long long)tiles + (long long)tm * tn * sp >= (1LL << 31)) break;
      if (si == nsh) p.sh[nsh++] = GemmShape{e.m, e.n, e.lda, e.ldb, e.ldc, tm, tn, sp, kc};
      clo = nclo; chi = nchi; blo = nblo; bhi = nbhi; alo = nalo; ahi = nahi;
      p.start[j - i] = tiles;
      tiles += tm * tn * sp;
      p.meta[j - i] = si | (e.flags << 8);
      p.ta[j - i] = e.a;
      p.tb[j - i] = static_cast<const bf16*>(e.b);
    }
    p.ng = j - i;
    p.start[p.ng] = tiles;
    p.c = reinterpret_cast<void*>(clo);
    p.bias = bhi ? reinterpret_cast<const float*>(blo) : nullptr;
    p.alpha_dev = ahi ? reinterpret_cast<const float*>(alo) : nullptr;
    p.f16 = f16;
    for (int q = 0; q < p.ng; ++q) {
      const LrceGemmItem& e = it[i + q];
      p.coff[q] = (int)((reinterpret_cast<uintptr_t>(e.c) - clo) / 4);
      p.boff[q] = (e.flags & LRCE_EPI_BIAS_GRAD) ? (int)((reinterpret_cast<uintptr_t>(e.bias) - blo) / 4) : -1;
      p.aoff[q] = e.alpha_dev ? (int)((reinterpret_cast<uintptr_t>(e.alpha_dev) - alo) / 4) : -1;
    }
    p.a = p.ta[0]; p.b = p.tb[0];
    p.m = p.sh[0].m; p.n = p.sh[0].n; p.tiles_m = p.sh[0].tiles_m; p.tiles_n = p.sh[0].tiles_n;
    if (f16) gemm_glds_kernel<128, 128, false, false, true, 2, false, true><<<dim3(tiles, 1), NT, 0, s>>>(p);
    else gemm_glds_kernel<128, 128, false, false, false, 2, false, true><<<dim3(tiles, 1), NT, 0, s>>>(p);
    i = j;
  }
  return lrce_check_launch("gemm_grouped");
}

// n same-shape weight gradients (d: shape / leading dims / flags ACCUM or OUT_F32 [| BIAS_GRAD]; its
// a / b / c / bias / batch / strides are ignored): lrce_gemm_grouped with one shape.
extern "C" int lrce_gemm_ptr_batched(const LrceGemmDesc* d, const void* const* a, const void* const* b, void* const* c,
                                     const float* const* bias, int n, void* stream) {
  if (!d || n < 0 || (n > 0 && (!a || !b || !c))) return lrce_fail(LRCE_E_ARG, "gemm_ptr_batched: null argument");
  if (n == 0) return LRCE_OK;
  const bool bg = d->flags & LRCE_EPI_BIAS_GRAD;
  if (d->a_kmajor || d->b_kmajor || d->a_f32 || d->b_f32 || d->f16 || d->a_map || d->c_map || d->split_k > 1 ||
      d->alpha_dev || d->row_scale || d->a_row_scale || d->scale_cols || d->drop_p > 0.f || (bg && !bias) ||
      d->lda > INT32_MAX || d->ldb > INT32_MAX || d->ldc > INT32_MAX)
    return lrce_fail(LRCE_E_ARG, "gemm_ptr_batched: bf16 weight gradients only (M-major dY, N-major X, ACCUM or OUT_F32 [| BIAS_GRAD])");
  std::vector<LrceGemmItem> items(n);
  for (int i = 0; i < n; ++i)
    items[i] = LrceGemmItem{a[i], b[i], static_cast<float*>(c[i]), bg ? const_cast<float*>(bias[i]) : nullptr,
                            nullptr, d->m, d->n, (int32_t)d->lda, (int32_t)d->ldb, (int32_t)d->ldc, d->flags, 0, 1, 0};
  return lrce_gemm_grouped(items.data(), n, d->k, d->alpha, stream);
}

// dst_i (=|+=) sum_s slabs_i[s][0..n_i) in slice order (the grouped launch's split-K weight gradients):
// one grid over every item's float4s, the item found by a scan of the start table.
constexpr int SLAB_ITEMS = 32;
struct SlabSumArgs {
  int items;
  long long start[SLAB_ITEMS + 1];   // first float4 of each item
  const float* src[SLAB_ITEMS];
  float* dst[SLAB_ITEMS];
  long long n[SLAB_ITEMS];
  int split[SLAB_ITEMS];
  int accum[SLAB_ITEMS];
};
__global__ void __launch_bounds__(256) slab_sum_kernel(const SlabSumArgs a) {
  const long long total = a.start[a.items];
  for (long long q = (long long)blockIdx.x * 256 + threadIdx.x; q < total; q += (long long)gridDim.x * 256) {
    int it = 0;
    while (it + 1 < a.items && a.start[it + 1] <= q) ++it;
    const long long i = (q - a.start[it]) * 4;
    const float* src = a.src[it] + i;
    const long long n = a.n[it];
    float4 acc = ld_slab(src);
    for (int sl = 1; sl < a.split[it]; ++sl) {
      const float4 v = ld_slab(src + sl * n);
      acc.x += v.x; acc.y += v.y; acc.z += v.z; acc.w += v.w;
    }
    float4* d = reinterpret_cast<float4*>(a.dst[it] + i);
    if (a.accum[it]) {
      const float4 o = *d;
      acc.x += o.x; acc.y += o.y; acc.z += o.z; acc.w += o.w;
    }
    *d = acc;
  }
}

extern "C" int lrce_slab_sum_grouped(const LrceSlabSum* items, int n, void* stream) {
  if (n < 0 || (n > 0 && !items)) return lrce_fail(LRCE_E_ARG, "slab_sum_grouped: n=%d", n);
  for (int i = 0; i < n; ++i) {
    const LrceSlabSum& e = items[i];
    if (!e.slabs || !e.dst || e.n <= 0 || e.n % 4 || e.split < 1 || (reinterpret_cast<uintptr_t>(e.slabs) & 15) ||
        (reinterpret_cast<uintptr_t>(e.dst) & 15))
      return lrce_fail(LRCE_E_ARG, "slab_sum_grouped: item %d (n %% 4 == 0, 16-B aligned, split >= 1)", i);
  }
  hipStream_t s = static_cast<hipStream_t>(stream);
  for (int i0 = 0; i0 < n; i0 += SLAB_ITEMS) {
    SlabSumArgs a{};
    a.items = n - i0 < SLAB_ITEMS ? n - i0 : SLAB_ITEMS;
    long long tot = 0;
    for (int j = 0; j < a.items; ++j) {
      const LrceSlabSum& e = items[i0 + j];
      a.start[j] = tot;
      tot += e.n / 4;
      a.src[j] = e.slabs; a.dst[j] = e.dst; a.n[j] = e.n; a.split[j] = e.split; a.accum[j] = e.accumulate != 0;
    }
    a.start[a.items] = tot;
    const long long blocks = (tot + 255) / 256;
    slab_sum_kernel<<<(int)(blocks < 2048 ? blocks : 2048), 256, 0, s>>>(a);
  }
  return lrce_check_launch("slab_sum_grouped");
}

// debug: phase timestamps of gemm_glds_kernel into buf (device, >= 8 per workgroup), NULL = off; the
// marks exist only in a -DLRCE_GEMM_TRACE build (tools/gemm_trace.py)
extern "C" int lrce_gemm_set_trace(uint64_t* buf) {
  g_gemm_trace = reinterpret_cast<unsigned long long*>(buf);
  return LRCE_OK;
}
