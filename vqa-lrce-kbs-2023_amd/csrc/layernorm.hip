// LayerNorm forward/backward, one wave per row, with fused row gather/scatter.
//
// The gather (in_map, nseg segments per row) fuses three reference data movements into the LN
// read: torch.roll + window_partition before the attention (video_swin_ori.py:262,268), the 2x2
// PatchMerging concat (:333-337), and identity for plain LNs.  HBM-bound: one read of x, one write
// of y, 8 B of stats per row.
// A missing source (in_map entry < 0) means zero padding: inside a multi-segment row (PatchMerging,
// which pads BEFORE its norm, :328-331) the segment reads as zeros; a whole missing row of a
// one-segment gather is a window position past the volume (the block pads AFTER norm1, :253-258):
// its output row is zero and it takes no part in the backward.
#include <cstdlib>
#include <type_traits>

#include "common.h"
#include "lrce_capi.h"
#include <cstdlib>

namespace {

constexpr int MAXC = 8;  // float4 chunks per lane -> cols <= 2048
constexpr int LN_RED_CTRS = 64;   // ln_bwd_reduce column blocks: (2 * 2048) / 64
constexpr int LN_RED_ROWS = 128;  // partial rows per ln_bwd_reduce block
constexpr int LN_RED_MAXY = 16;   // 2048 blocks / LN_RED_ROWS

template <typename T>
__device__ __forceinline__ float4 ld4(const T* p);
template <>
__device__ __forceinline__ float4 ld4<float>(const float* p) { return *reinterpret_cast<const float4*>(p); }
template <>
__device__ __forceinline__ float4 ld4<bf16>(const bf16* p) {
  const bf16x4 v = *reinterpret_cast<const bf16x4*>(p);
  return make_float4(bf2f(v[0]), bf2f(v[1]), bf2f(v[2]), bf2f(v[3]));
}
template <typename T>
__device__ __forceinline__ void st4(T* p, float4 v);
template <>
__device__ __forceinline__ void st4<float>(float* p, float4 v) { *reinterpret_cast<float4*>(p) = v; }
template <>
__device__ __forceinline__ void st4<bf16>(bf16* p, float4 v) {
  bf16x4 o;
  o[0] = f2bf(v.x); o[1] = f2bf(v.y); o[2] = f2bf(v.z); o[3] = f2bf(v.w);
  *reinterpret_cast<bf16x4*>(p) = o;
}

__device__ __forceinline__ void st4_16(bf16* p, float4 v, bool f16) {
  bf16x4 o;
  o[0] = to16r(v.x, f16); o[1] = to16r(v.y, f16); o[2] = to16r(v.z, f16); o[3] = to16r(v.w, f16);
  *reinterpret_cast<bf16x4*>(p) = o;
}

// address of the 4-chunk c (element 4c) of LN row r inside x
__device__ __forceinline__ long long src_off(const int* in_map, int nseg, int seg, int r, int c, int& valid) {
  const int e = c * 4;
  if (!in_map) { valid = 1; return (long long)r * (seg * nseg) + e; }
  const int s = e / seg;
  const int src = in_map[(long long)r * nseg + s];
  valid = src >= 0;
  return (long long)src * seg + (e - s * seg);
}

// Reductions over the LPR lanes that share one row (LPR = 64: whole wave; 32: half wave).
template <int LPR>
__device__ __forceinline__ float row_sum(float v) {
#pragma unroll
  for (int o = LPR / 2; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// CH float4 chunks per lane, LPR lanes per row (rows of <= 128 columns use half a wave each).
template <typename TX, typename TY, int CH, int LPR>
__global__ void __launch_bounds__(256) ln_fwd(const TX* x, const int* in_map, int nseg, const float* w, const float* b,
                                              float eps, TY* y, bf16* y2, const int* out_map, float* mean_o, float* rstd_o,
                                              int rows, int cols, int y2_f16) {
  constexpr int RPW = 64 / LPR;
  const int lane = threadIdx.x & 63, sl = lane % LPR;
  const int r = (blockIdx.x * 4 + (threadIdx.x >> 6)) * RPW + lane / LPR;
  if (r >= rows) return;
  const int nch = cols >> 2, seg = cols / nseg;
  if (in_map && nseg == 1 && in_map[r] < 0) {   // padded window position: zero row
    const long long orow = out_map ? (long long)out_map[r] : (long long)r;
#pragma unroll
    for (int t = 0; t < CH; ++t) {
      const int c = sl + LPR * t;
      if (c < nch) {
        st4<TY>(y + orow * cols + 4 * c, make_float4(0.f, 0.f, 0.f, 0.f));
        if (y2) st4_16(y2 + orow * cols + 4 * c, make_float4(0.f, 0.f, 0.f, 0.f), y2_f16 != 0);
      }
    }
    if (sl == 0) {
      if (mean_o) mean_o[r] = 0.f;
      if (rstd_o) rstd_o[r] = 0.f;
    }
    return;
  }
  float4 v[CH], ww[CH], bb[CH];
  float s = 0.f;
#pragma unroll
  for (int t = 0; t < CH; ++t) {   // gamma / beta issued with the row (one memory round trip, not two)
    const int c = sl + LPR * t;
    if (c < nch) {
      ww[t] = *reinterpret_cast<const float4*>(w + 4 * c);
      bb[t] = *reinterpret_cast<const float4*>(b + 4 * c);
    }
  }
#pragma unroll
  for (int t = 0; t < CH; ++t) {
    const int c = sl + LPR * t;
    v[t] = make_float4(0.f, 0.f, 0.f, 0.f);
    if (c < nch) {
      int ok;
      const long long o = src_off(in_map, nseg, seg, r, c, ok);
      if (ok) v[t] = ld4<TX>(x + o);
      s += v[t].x + v[t].y + v[t].z + v[t].w;
    }
  }
  const float mean = row_sum<LPR>(s) / cols;
  float q = 0.f;
#pragma unroll
  for (int t = 0; t < CH; ++t) {
    const int c = sl + LPR * t;
    if (c < nch) {
      const float a = v[t].x - mean, b2 = v[t].y - mean, c2 = v[t].z - mean, d = v[t].w - mean;
      q += a * a + b2 * b2 + c2 * c2 + d * d;
    }
  }
  const float rstd = rsqrtf(row_sum<LPR>(q) / cols + eps);
  const long long orow = out_map ? (long long)out_map[r] : (long long)r;
#pragma unroll
  for (int t = 0; t < CH; ++t) {
    const int c = sl + LPR * t;
    if (c < nch) {
      float4 o;
      o.x = (v[t].x - mean) * rstd * ww[t].x + bb[t].x;
      o.y = (v[t].y - mean) * rstd * ww[t].y + bb[t].y;
      o.z = (v[t].z - mean) * rstd * ww[t].z + bb[t].z;
      o.w = (v[t].w - mean) * rstd * ww[t].w + bb[t].w;
      st4<TY>(y + orow * cols + 4 * c, o);
      if (y2) st4_16(y2 + orow * cols + 4 * c, o, y2_f16 != 0);
    }
  }
  if (sl == 0) {
    if (mean_o) mean_o[r] = mean;
    if (rstd_o) rstd_o[r] = rstd;
  }
}

// Scaled fp16 copy of the LN input gradient (F16S: the BERT backward, text.py): dx16[r][c] =
// fp16(keep ? dx * S / (1 - p) : 0) with S = f16s->scale[0] (a delayed per-tensor gradient scale,
// lrce_grad_scale_update), the mask of lrce_dropout over the contiguous [rows][cols] tensor, and
// max|dx| folded into f16s->scale word 2 for the next step's scale.  A kept element whose scaled value
// rounds past the fp16 range (|dx S / (1 - p)| >= 65520: an infinite operand for the GEMMs that follow)
// sets word 3, the slot's found-inf flag (lrce_adamw_step's skip slots; lrce_grad_scale_update clears it).
struct F16Scaled {
  float* scale;          // [S, 1/S, amax bits (next step), found-inf]
  float p;
  uint64_t seed;
  const uint64_t* off;
};

// NT: non-temporal loads of x / dres and stores of dx (each touched once here; dx is next read by a
// LayerNorm backward a whole block later)
typedef float lnf4 __attribute__((ext_vector_type(4)));
template <bool NT>
__device__ __forceinline__ float4 ld4f(const float* p) {
  if constexpr (NT) {
    const lnf4 t = __builtin_nontemporal_load(reinterpret_cast<const lnf4*>(p));
    return make_float4(t.x, t.y, t.z, t.w);
  } else {
    return *reinterpret_cast<const float4*>(p);
  }
}
template <bool NT, typename TX>
__device__ __forceinline__ float4 ld4x(const TX* p) {
  if constexpr (NT && std::is_same<TX, float>::value) return ld4f<true>(reinterpret_cast<const float*>(p));
  else return ld4<TX>(p);
}

template <typename TD, typename TX, int CH, int LPR, bool F16S = false, bool NT = false>
__global__ void __launch_bounds__(256) ln_bwd(const TD* dy, const int* dy_map, const TX* x, const int* in_map, int nseg,
                                              const float* mean_i, const float* rstd_i, const float* w, float* dx,
                                              const float* dres, float* dw, float* db, int rows, int cols, bf16* dx16,
                                              const int* dx16_map, const float* dsc, int dsc_rps, float* part,
                                              F16Scaled fs = F16Scaled{}) {
  constexpr int RPW = 64 / LPR;
  __shared__ float red[2][4][4 * CH * LPR + 4];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, sl = lane % LPR;
  const int nch = cols >> 2, seg = cols / nseg;
  float4 aw[CH], ab[CH];  // dw/db partials of this lane's columns
#pragma unroll
  for (int t = 0; t < CH; ++t) { aw[t] = make_float4(0.f, 0.f, 0.f, 0.f); ab[t] = aw[t]; }
  // The raw operands of the NEXT row of this wave (x, dy, dres, stats) are fetched before the
  // current row is reduced and written, so a wave keeps one row of loads in flight (large inputs
  // run >= 8 rows per wave: without it each row is a full memory round trip).
  const int stride = gridDim.x * 4 * RPW;
  const float4 z4 = make_float4(0.f, 0.f, 0.f, 0.f);
  // rows of a one-segment gather whose source is missing are padding (no output, no dw / db); the
  // flag comes from the gather's own source lookup, so it does not delay the row's other loads
  auto fetch = [&](int rb, float4 (&xv)[CH], float4 (&dv)[CH], float4 (&rv)[CH], float& mu, float& rs, bool& pad) {
    const int r = rb + lane / LPR;
    const bool live = r < rows;
    pad = false;
    mu = live ? mean_i[r] : 0.f;
    rs = live ? rstd_i[r] : 0.f;
    const long long dyr = !live ? 0 : (dy_map ? (long long)dy_map[r] : (long long)r);
#pragma unroll
    for (int t = 0; t < CH; ++t) {
      const int c = sl + LPR * t;
      xv[t] = z4; dv[t] = z4; rv[t] = z4;
      if (live && c < nch) {
        int ok;
        const long long o = src_off(in_map, nseg, seg, r, c, ok);
        if (ok) {
          xv[t] = ld4x<NT, TX>(x + o);
          if (dres) rv[t] = ld4f<NT>(dres + o);
        } else if (nseg == 1) {
          pad = true;
        }
        dv[t] = ld4<TD>(dy + dyr * cols + 4 * c);
      }
    }
  };
  int r0 = (blockIdx.x * 4 + wave) * RPW;
  float4 wcol[CH];   // gamma of this lane's columns: loaded once, with the first row
#pragma unroll
  for (int t = 0; t < CH; ++t) {
    const int c = sl + LPR * t;
    wcol[t] = c < nch ? *reinterpret_cast<const float4*>(w + 4 * c) : z4;
  }
  float4 xcur[CH], dcur[CH], rcur[CH];
  float mcur = 0.f, scur = 0.f;
  bool pcur = false;
  float amax = 0.f;                                    // F16S: max |dx| of this wave's rows
  bool ovf = false;                                    // F16S: a kept element overflowed fp16
  const float s16 = F16S ? fs.scale[0] / (fs.p > 0.f ? 1.0f - fs.p : 1.0f) : 0.f;
  const uint64_t dseed = F16S && fs.p > 0.f ? lrce_seed(fs.seed, fs.off) : 0ull;
  if (r0 < rows) fetch(r0, xcur, dcur, rcur, mcur, scur, pcur);
  for (; r0 < rows; r0 += stride) {
    float4 xnx[CH], dnx[CH], rnx[CH];
    float mnx = 0.f, snx = 0.f;
    bool pnx = false;
    const bool more = r0 + stride < rows;
    if (more) fetch(r0 + stride, xnx, dnx, rnx, mnx, snx, pnx);
    const int r = r0 + lane / LPR;
    const bool live = r < rows && !pcur;
    const float mean = mcur, rstd = scur;
    float4 xh[CH], g[CH];
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int t = 0; t < CH; ++t) {
      const int c = sl + LPR * t;
      xh[t] = make_float4(0.f, 0.f, 0.f, 0.f);
      g[t] = xh[t];
      if (live && c < nch) {
        const float4 xv = xcur[t];
        xh[t] = make_float4((xv.x - mean) * rstd, (xv.y - mean) * rstd, (xv.z - mean) * rstd, (xv.w - mean) * rstd);
        const float4 d = dcur[t];
        const float4 ww = wcol[t];
        g[t] = make_float4(d.x * ww.x, d.y * ww.y, d.z * ww.z, d.w * ww.w);
        s1 += g[t].x + g[t].y + g[t].z + g[t].w;
        s2 += g[t].x * xh[t].x + g[t].y * xh[t].y + g[t].z * xh[t].z + g[t].w * xh[t].w;
        aw[t].x += d.x * xh[t].x; aw[t].y += d.y * xh[t].y; aw[t].z += d.z * xh[t].z; aw[t].w += d.w * xh[t].w;
        ab[t].x += d.x; ab[t].y += d.y; ab[t].z += d.z; ab[t].w += d.w;
      }
    }
    const float c1 = row_sum<LPR>(s1) / cols, c2 = row_sum<LPR>(s2) / cols;
#pragma unroll
    for (int t = 0; t < CH; ++t) {
      const int c = sl + LPR * t;
      if (live && c < nch) {
        int ok;
        const long long o = src_off(in_map, nseg, seg, r, c, ok);
        if (!ok) continue;
        float4 out;
        out.x = rstd * (g[t].x - c1 - xh[t].x * c2);
        out.y = rstd * (g[t].y - c1 - xh[t].y * c2);
        out.z = rstd * (g[t].z - c1 - xh[t].z * c2);
        out.w = rstd * (g[t].w - c1 - xh[t].w * c2);
        if (dres) {
          const float4 rr = rcur[t];
          out.x += rr.x; out.y += rr.y; out.z += rr.z; out.w += rr.w;
        }
        if (dx) {
          if constexpr (NT) __builtin_nontemporal_store(lnf4{out.x, out.y, out.z, out.w}, reinterpret_cast<lnf4*>(dx + o));
          else *reinterpret_cast<float4*>(dx + o) = out;
        }
        if constexpr (F16S) {   // (identity maps on this path: the host checks)
          const float a4[4] = {out.x, out.y, out.z, out.w};
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const float ae = fabsf(a4[e]);
            amax = (ae > amax || ae != ae) ? ae : amax;   // NaN sticks (lrce_grad_scale)
          }
          float4 u = make_float4(1.f, 1.f, 1.f, 1.f);
          if (fs.p > 0.f) u = lrce_uniform4(dseed, ((unsigned long long)r * cols + 4 * c) >> 2);
          typedef __attribute__((ext_vector_type(4))) _Float16 h4;
          h4 hv;
          const float o4[4] = {u.x >= fs.p ? out.x * s16 : 0.f, u.y >= fs.p ? out.y * s16 : 0.f,
                               u.z >= fs.p ? out.z * s16 : 0.f, u.w >= fs.p ? out.w * s16 : 0.f};
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            hv[e] = (f16)o4[e];
            ovf |= !(fabsf(o4[e]) < 65520.f);   // rounds to fp16 inf (or is NaN)
          }
          *reinterpret_cast<h4*>(dx16 + (long long)r * cols + 4 * c) = hv;
        } else if (dx16) {   // bf16 copy (optionally row-scaled / row-permuted) for the next GEMMs' A operand
          const float f = dsc ? dsc[r / dsc_rps] : 1.f;
          const long long orow = dx16_map ? (long long)dx16_map[r] : (long long)r;
          st4<bf16>(dx16 + orow * cols + 4 * c, make_float4(out.x * f, out.y * f, out.z * f, out.w * f));
        }
      }
    }
    if (more) {
#pragma unroll
      for (int t = 0; t < CH; ++t) { xcur[t] = xnx[t]; dcur[t] = dnx[t]; rcur[t] = rnx[t]; }
      mcur = mnx;
      scur = snx;
      pcur = pnx;
    }
  }
  if constexpr (F16S) {   // the next step's scale: one agent-scope max per wave (|x| bits order like values)
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      const float t = __shfl_xor(amax, o, 64);
      amax = (t > amax || t != t) ? t : amax;
    }
    if (lane == 0 && amax != 0.f)
      __hip_atomic_fetch_max(reinterpret_cast<unsigned*>(fs.scale + 2), __float_as_uint(amax), __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_AGENT);
    if (__ballot(ovf) != 0ull && lane == 0)
      __hip_atomic_store(reinterpret_cast<unsigned*>(fs.scale + 3), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  if (!dw && !db) return;
  if (LPR == 32) {  // fold the two half-wave row slots onto lanes 0..31
#pragma unroll
    for (int t = 0; t < CH; ++t) {
      aw[t].x += __shfl_xor(aw[t].x, 32, 64); aw[t].y += __shfl_xor(aw[t].y, 32, 64);
      aw[t].z += __shfl_xor(aw[t].z, 32, 64); aw[t].w += __shfl_xor(aw[t].w, 32, 64);
      ab[t].x += __shfl_xor(ab[t].x, 32, 64); ab[t].y += __shfl_xor(ab[t].y, 32, 64);
      ab[t].z += __shfl_xor(ab[t].z, 32, 64); ab[t].w += __shfl_xor(ab[t].w, 32, 64);
    }
  }
  if (lane < LPR) {
#pragma unroll
    for (int t = 0; t < CH; ++t) {
      const int e = 4 * (sl + LPR * t);
      red[0][wave][e] = aw[t].x; red[0][wave][e + 1] = aw[t].y; red[0][wave][e + 2] = aw[t].z; red[0][wave][e + 3] = aw[t].w;
      red[1][wave][e] = ab[t].x; red[1][wave][e + 1] = ab[t].y; red[1][wave][e + 2] = ab[t].z; red[1][wave][e + 3] = ab[t].w;
    }
  }
  __syncthreads();
  float* pb = part ? part + (long long)blockIdx.x * 2 * cols : nullptr;
  for (int e = threadIdx.x; e < cols; e += 256) {
    const float sw = red[0][0][e] + red[0][1][e] + red[0][2][e] + red[0][3][e];
    const float sb = red[1][0][e] + red[1][1][e] + red[1][2][e] + red[1][3][e];
    if (pb) {            // per-block partials, summed in block order by ln_bwd_reduce
      pb[e] = sw;
      pb[cols + e] = sb;
    } else if (gridDim.x == 1) {   // the only block: one writer per element (deterministic)
      if (dw) dw[e] += sw;
      if (db) db[e] += sb;
    } else {             // no workspace: same-address atomics (order-dependent rounding)
      if (dw) atomicAdd(dw + e, sw);
      if (db) atomicAdd(db + e, sb);
    }
  }
  // arrival counters of ln_bwd_reduce (after the partials: the next launch reads them zeroed)
  if (part && blockIdx.x == 0 && threadIdx.x < LN_RED_CTRS)
    reinterpret_cast<unsigned*>(part + ((long long)gridDim.x + (gridDim.x + LN_RED_ROWS - 1) / LN_RED_ROWS) * 2 * cols)[threadIdx.x] = 0u;
}

// split-K reduce + bias + dropout + residual + LayerNorm forward, one wave per row (lrce_splitk_reduce_ln);
// the same per-element math as splitk_reduce_epi_kernel (gemm.hip) and ln_fwd above
template <int CH>
__global__ void __launch_bounds__(256) splitk_reduce_ln_kernel(const float* __restrict__ ws, int split, int rows, int cols,
                                                               const float* __restrict__ bias, const float* __restrict__ resid,
                                                               long long ld_res, float p, uint64_t seed,
                                                               const uint64_t* __restrict__ off, float* __restrict__ pre,
                                                               const float* __restrict__ w, const float* __restrict__ b,
                                                               float eps, float* __restrict__ y, bf16* __restrict__ y16,
                                                               int y16_f16, float* __restrict__ mean_o,
                                                               float* __restrict__ rstd_o) {
  const int lane = threadIdx.x & 63;
  const int r = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (r >= rows) return;
  const long long mn = (long long)rows * cols;
  float4 v[CH], ww[CH], bb[CH];
#pragma unroll
  for (int t = 0; t < CH; ++t) {
    const int col = 4 * (lane + 64 * t);
    const long long e = (long long)r * cols + col;
    float4 s4 = *reinterpret_cast<const float4*>(ws + e);
    for (int k = 1; k < split; ++k) {
      const float4 q = *reinterpret_cast<const float4*>(ws + k * mn + e);
      s4.x += q.x; s4.y += q.y; s4.z += q.z; s4.w += q.w;
    }
    ww[t] = *reinterpret_cast<const float4*>(w + col);
    bb[t] = *reinterpret_cast<const float4*>(b + col);
    if (bias) {
      const float4 q = *reinterpret_cast<const float4*>(bias + col);
      s4.x += q.x; s4.y += q.y; s4.z += q.z; s4.w += q.w;
    }
    if (p > 0.f) {
      const float4 u = lrce_uniform4(lrce_seed(seed, off), (unsigned long long)e >> 2);
      const float kd = 1.0f - p;
      s4.x = u.x >= p ? s4.x / kd : 0.f; s4.y = u.y >= p ? s4.y / kd : 0.f;
      s4.z = u.z >= p ? s4.z / kd : 0.f; s4.w = u.w >= p ? s4.w / kd : 0.f;
    }
    if (resid) {
      const float4 q = *reinterpret_cast<const float4*>(resid + r * ld_res + col);
      s4.x += q.x; s4.y += q.y; s4.z += q.z; s4.w += q.w;
    }
    v[t] = s4;
    if (pre) *reinterpret_cast<float4*>(pre + e) = s4;
  }
  float s = 0.f;
#pragma unroll
  for (int t = 0; t < CH; ++t) s += v[t].x + v[t].y + v[t].z + v[t].w;
  const float mean = row_sum<64>(s) / cols;
  float q = 0.f;
#pragma unroll
  for (int t = 0; t < CH; ++t) {
    const float a = v[t].x - mean, b2 = v[t].y - mean, c2 = v[t].z - mean, d = v[t].w - mean;
    q += a * a + b2 * b2 + c2 * c2 + d * d;
  }
  const float rstd = rsqrtf(row_sum<64>(q) / cols + eps);
#pragma unroll
  for (int t = 0; t < CH; ++t) {
    const int col = 4 * (lane + 64 * t);
    float4 o;
    o.x = (v[t].x - mean) * rstd * ww[t].x + bb[t].x;
    o.y = (v[t].y - mean) * rstd * ww[t].y + bb[t].y;
    o.z = (v[t].z - mean) * rstd * ww[t].z + bb[t].z;
    o.w = (v[t].w - mean) * rstd * ww[t].w + bb[t].w;
    *reinterpret_cast<float4*>(y + (long long)r * cols + col) = o;
    if (y16) st4_16(y16 + (long long)r * cols + col, o, y16_f16 != 0);
  }
  if (lane == 0) {
    if (mean_o) mean_o[r] = mean;
    if (rstd_o) rstd_o[r] = rstd;
  }
}

// dw[e] += sum_b part[b][e], db[e] += sum_b part[b][cols + e], deterministically: block (x, y) sums
// LN_RED_ROWS partial rows of 64 columns (32 per wave, 8 loads in flight) into chunk row y; the last
// of the column block's ny (<= 16) blocks to arrive (agent-scope stores / counter, as the skinny
// split-K of gemm_f32.hip) adds the ny chunk rows in order — one writer per element, a fixed order.
// The hand-off is MI355X_MICROARCH.md's first-row sc1 form (relaxed agent-scope stores drained by
// vmcnt(0), a barrier, one agent atomic add, agent-scope relaxed loads in the last arriver): measured
// gfx950 behaviour, not a C++ memory-model release/acquire pair (see decoder.hip publish_partial).
__device__ __forceinline__ void ln_reduce_body(const float* __restrict__ part, int nb, int cols, float* dw, float* db,
                                               float* chunk, unsigned* counters, int bx, int by, int ny) {
  __shared__ float red[4][64];
  __shared__ unsigned last;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int e = bx * 64 + lane;
  float t = 0.f;
#pragma unroll
  for (int q = 0; q < LN_RED_ROWS / 32; ++q) {
    const int b0 = by * LN_RED_ROWS + q * 32 + wave * 8;
    float v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) v[u] = (e < 2 * cols && b0 + u < nb) ? part[(long long)(b0 + u) * 2 * cols + e] : 0.f;
#pragma unroll
    for (int u = 0; u < 8; ++u) t += v[u];
  }
  red[wave][lane] = t;
  __syncthreads();
  if (wave == 0 && e < 2 * cols)
    __hip_atomic_store(chunk + (long long)by * 2 * cols + e, (red[0][lane] + red[1][lane]) + (red[2][lane] + red[3][lane]),
                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0)
    last = __hip_atomic_fetch_add(&counters[bx], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == (unsigned)(ny - 1);
  __syncthreads();
  if (!last || wave != 0 || e >= 2 * cols) return;
  float cv[LN_RED_MAXY];
#pragma unroll
  for (int y = 0; y < LN_RED_MAXY; ++y)
    cv[y] = y < ny ? __hip_atomic_load(chunk + (long long)y * 2 * cols + e, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0.f;
  float s = 0.f;
#pragma unroll
  for (int y = 0; y < LN_RED_MAXY; ++y) s += cv[y];
  float* dst = e < cols ? (dw ? dw + e : nullptr) : (db ? db + (e - cols) : nullptr);
  if (dst) *dst += s;
}
__global__ void __launch_bounds__(256) ln_bwd_reduce(const float* __restrict__ part, int nb, int cols, float* dw, float* db,
                                                     float* chunk, unsigned* counters) {
  ln_reduce_body(part, nb, cols, dw, db, chunk, counters, blockIdx.x, blockIdx.y, gridDim.y);
}

// Many LayerNorms' deferred reductions in one launch (lrce_layernorm_grad_reduce): blockIdx.z picks the
// item, (x, y) as ln_bwd_reduce over that item's partials; blocks past an item's grid return at once.
struct LnRedItem {
  const float* part;
  float* dw;
  float* db;
  int nb, cols;
};
constexpr int LN_RED_BATCH = 40;
struct LnRedBatch {
  LnRedItem it[LN_RED_BATCH];
};
__global__ void __launch_bounds__(256) ln_bwd_reduce_batched(LnRedBatch b) {
  const LnRedItem& it = b.it[blockIdx.z];
  const int ny = (it.nb + LN_RED_ROWS - 1) / LN_RED_ROWS;
  if ((int)blockIdx.x * 64 >= 2 * it.cols || (int)blockIdx.y >= ny) return;   // uniform over the block
  float* chunk = const_cast<float*>(it.part) + (long long)it.nb * 2 * it.cols;
  unsigned* ctr = reinterpret_cast<unsigned*>(chunk + (long long)ny * 2 * it.cols);
  ln_reduce_body(it.part, it.nb, it.cols, it.dw, it.db, chunk, ctr, blockIdx.x, blockIdx.y, ny);
}

// rows per wave of ln_bwd: small inputs (the decoder / BERT rows) one row per wave (latency-bound:
// as many waves as rows); larger ones 4-8 with the next row prefetched.  (A chip-capacity grid —
// one row per wave up to 2-8 resident blocks per CU — measured 5-25 % slower on the 15 680 x 512 and
// 3 920 x 1024 shapes, 4 % faster on 62 720 rows: more blocks mean more dw / db partials to reduce;
// tools/ln_bench.py.)  Without a partials workspace every
// block adds its dw/db into the SAME 2 x cols addresses, so blocks are capped.
int ln_bwd_blocks(int rows, int lpr, bool ws, int cols) {
  const int rpb = 4 * (64 / lpr);                 // rows per block per pass
  // measured per row width (tools/ln_bench.py sweep, round 4): rows of <= 512 columns stream best
  // on a capped chip-wide grid — 1024 blocks at <= 256 columns, 768 at 512 (250 880 x 128: 116.5 ->
  // 112.6 us, 62 720 x 512: 123 -> 108 us) — wider rows with 4-8 rows per wave
  const int nch = cols / 4;
  if (ws && rows > 8192 && nch <= 128) {
    const int nb1 = (rows + rpb - 1) / rpb, cap = nch <= 64 ? 1024 : 768;
    return nb1 > cap ? cap : nb1;
  }
  const int per_wave = ws ? (rows <= 2048 ? 1 : rows <= 8192 ? 4 : 8) : (rows <= 8192 ? 1 : 8);
  const int nb = (rows + rpb * per_wave - 1) / (rpb * per_wave);
  return nb < 1 ? 1 : (nb > 2048 ? 2048 : nb);
}
int ln_bwd_lpr(int cols) { return cols / 4 <= 32 ? 32 : 64; }

}  // namespace

extern "C" int lrce_layernorm_fwd(const void* x, int x_f32, const int32_t* in_map, int nseg, const float* w,
                                  const float* b, float eps, void* y, int y_f32, uint16_t* y2, const int32_t* out_map,
                                  float* mean, float* rstd, int rows, int cols, int copy_f16, void* stream) {
  if (!x || !y || !w || !b) return lrce_fail(LRCE_E_ARG, "layernorm_fwd: null pointer");
  if (nseg < 1) nseg = 1;
  if (cols % 4 || (cols / nseg) % 4 || cols % nseg || cols > 64 * 4 * MAXC)
    return lrce_fail(LRCE_E_ARG, "layernorm_fwd: cols=%d nseg=%d unsupported", cols, nseg);
  if (rows <= 0) return LRCE_OK;
  hipStream_t s = static_cast<hipStream_t>(stream);
  const int nch = cols / 4;
#define LNF3(TX, TY, CH, LPR)                                                                                          \
  ln_fwd<TX, TY, CH, LPR><<<(rows + 4 * (64 / LPR) - 1) / (4 * (64 / LPR)), 256, 0, s>>>(                              \
      static_cast<const TX*>(x), in_map, nseg, w, b, eps, static_cast<TY*>(y), reinterpret_cast<bf16*>(y2), out_map, mean, \
      rstd, rows, cols, copy_f16)
#define LNF(TX, TY)                                   \
  if (nch <= 32) LNF3(TX, TY, 1, 32);                 \
  else if (nch <= 64) LNF3(TX, TY, 1, 64);            \
  else if (nch <= 128) LNF3(TX, TY, 2, 64);           \
  else if (nch <= 192) LNF3(TX, TY, 3, 64);           \
  else if (nch <= 256) LNF3(TX, TY, 4, 64);           \
  else LNF3(TX, TY, 8, 64);
  if (x_f32 && y_f32) { LNF(float, float) }
  else if (x_f32) { LNF(float, bf16) }
  else if (y_f32) { LNF(bf16, float) }
  else { LNF(bf16, bf16) }
#undef LNF
#undef LNF3
  return lrce_check_launch("layernorm_fwd");
}

static int layernorm_bwd_impl(const void* dy, int dy_f32, const int32_t* dy_map, const void* x, int x_f32,
                              const int32_t* in_map, int nseg, const float* mean, const float* rstd, const float* w,
                              float* dx, const float* dres, float* dw, float* db, int rows, int cols, uint16_t* dx_bf16,
                              const int32_t* dx_bf16_map, const float* dx_scale, int dx_scale_rps, float* workspace,
                              int64_t workspace_elems, void* stream, int* defer_nb) {
  if (defer_nb) *defer_nb = 0;
  if (!dy || !x || !mean || !rstd || !w || (!dx && !dx_bf16)) return lrce_fail(LRCE_E_ARG, "layernorm_bwd: null pointer");
  if (dx_scale_rps < 1) dx_scale_rps = 1;
  if (nseg < 1) nseg = 1;
  if (cols % 4 || (cols / nseg) % 4 || cols % nseg || cols > 64 * 4 * MAXC)
    return lrce_fail(LRCE_E_ARG, "layernorm_bwd: cols=%d nseg=%d unsupported", cols, nseg);
  if (rows <= 0) return LRCE_OK;
  hipStream_t s = static_cast<hipStream_t>(stream);
  const int nch = cols / 4;
  const int lpr = ln_bwd_lpr(cols);
  const bool want = dw || db;
  const int nb_ws = ln_bwd_blocks(rows, lpr, true, cols);
  const int ny = (nb_ws + LN_RED_ROWS - 1) / LN_RED_ROWS;
  // dw / db partials per block + a deterministic reduce launch; a one-block problem (rows <= 4-8, the
  // decoder's rows) or no workspace: one block adds its sums directly
  float* part = want && nb_ws > 1 && workspace && workspace_elems >= (int64_t)(nb_ws + ny) * 2 * cols + LN_RED_CTRS
                    ? workspace : nullptr;
  const int nb = (part || !want) ? nb_ws : ln_bwd_blocks(rows, lpr, false, cols);
  // non-temporal x / dres / dx on the large shapes only (tools/ln_bench.py: 250 880 x 128 and 62 720 x 512
  // 113 -> 98 / 94 us; at <= 16 M elements the hint costs up to 15 %)
  const bool nt = (long long)rows * cols >= (24LL << 20);
#define LNB3(TD, TX, CH, LPR)                                                                                          \
  (nt ? ln_bwd<TD, TX, CH, LPR, false, true> : ln_bwd<TD, TX, CH, LPR>)<<<nb, 256, 0, s>>>(                         \
      static_cast<const TD*>(dy), dy_map, static_cast<const TX*>(x), in_map, nseg, mean, rstd, w, dx, dres, dw, db, rows, \
      cols, reinterpret_cast<bf16*>(dx_bf16), dx_bf16_map, dx_scale, dx_scale_rps, part, F16Scaled{})
#define LNB(TD, TX)                                   \
  if (nch <= 32) LNB3(TD, TX, 1, 32);                 \
  else if (nch <= 64) LNB3(TD, TX, 1, 64);            \
  else if (nch <= 128) LNB3(TD, TX, 2, 64);           \
  else if (nch <= 192) LNB3(TD, TX, 3, 64);           \
  else if (nch <= 256) LNB3(TD, TX, 4, 64);           \
  else LNB3(TD, TX, 8, 64);
  if (dy_f32 && x_f32) { LNB(float, float) }
  else if (dy_f32) { LNB(float, bf16) }
  else if (x_f32) { LNB(bf16, float) }
  else { LNB(bf16, bf16) }
#undef LNB
#undef LNB3
  if (part && defer_nb) *defer_nb = nb;   // the caller reduces later (lrce_layernorm_grad_reduce)
  else if (part)
    ln_bwd_reduce<<<dim3((2 * cols + 63) / 64, ny), 256, 0, s>>>(
        part, nb, cols, dw, db, part + (long long)nb * 2 * cols, reinterpret_cast<unsigned*>(part + (long long)(nb + ny) * 2 * cols));
  return lrce_check_launch("layernorm_bwd");
}

extern "C" int lrce_layernorm_bwd(const void* dy, int dy_f32, const int32_t* dy_map, const void* x, int x_f32,
                                  const int32_t* in_map, int nseg, const float* mean, const float* rstd, const float* w,
                                  float* dx, const float* dres, float* dw, float* db, int rows, int cols, uint16_t* dx_bf16,
                                  const int32_t* dx_bf16_map, const float* dx_scale, int dx_scale_rps, float* workspace,
                                  int64_t workspace_elems, void* stream) {
  return layernorm_bwd_impl(dy, dy_f32, dy_map, x, x_f32, in_map, nseg, mean, rstd, w, dx, dres, dw, db, rows, cols, dx_bf16,
                            dx_bf16_map, dx_scale, dx_scale_rps, workspace, workspace_elems, stream, nullptr);
}

extern "C" int lrce_layernorm_bwd_deferred(const void* dy, int dy_f32, const int32_t* dy_map, const void* x, int x_f32,
                                           const int32_t* in_map, int nseg, const float* mean, const float* rstd,
                                           const float* w, float* dx, const float* dres, float* dw, float* db, int rows,
                                           int cols, uint16_t* dx_bf16, const int32_t* dx_bf16_map, const float* dx_scale,
                                           int dx_scale_rps, float* workspace, int64_t workspace_elems, int* nb_out,
                                           void* stream) {
  if (!nb_out) return lrce_fail(LRCE_E_ARG, "layernorm_bwd_deferred: null nb_out");
  return layernorm_bwd_impl(dy, dy_f32, dy_map, x, x_f32, in_map, nseg, mean, rstd, w, dx, dres, dw, db, rows, cols, dx_bf16,
                            dx_bf16_map, dx_scale, dx_scale_rps, workspace, workspace_elems, stream, nb_out);
}

extern "C" int lrce_layernorm_grad_reduce(const float* const* parts, const int32_t* nbs, const int32_t* cols,
                                          float* const* dw, float* const* db, int n, void* stream) {
  if (n < 0 || (n > 0 && (!parts || !nbs || !cols || !dw || !db))) return lrce_fail(LRCE_E_ARG, "layernorm_grad_reduce: args");
  hipStream_t s = static_cast<hipStream_t>(stream);
  for (int i0 = 0; i0 < n; i0 += LN_RED_BATCH) {
    LnRedBatch b{};
    const int m = n - i0 < LN_RED_BATCH ? n - i0 : LN_RED_BATCH;
    int gx = 1, gy = 1;
    for (int j = 0; j < m; ++j) {
      const int i = i0 + j;
      if (!parts[i] || nbs[i] < 2 || nbs[i] > LN_RED_MAXY * LN_RED_ROWS || cols[i] < 4 || cols[i] % 4 || (!dw[i] && !db[i]))
        return lrce_fail(LRCE_E_ARG, "layernorm_grad_reduce: item %d (nb=%d cols=%d)", i, nbs[i], cols[i]);
      b.it[j] = LnRedItem{parts[i], dw[i], db[i], nbs[i], cols[i]};
      const int bx = (2 * cols[i] + 63) / 64, by = (nbs[i] + LN_RED_ROWS - 1) / LN_RED_ROWS;
      gx = bx > gx ? bx : gx;
      gy = by > gy ? by : gy;
    }
    ln_bwd_reduce_batched<<<dim3(gx, gy, m), 256, 0, s>>>(b);
  }
  return lrce_check_launch("layernorm_grad_reduce");
}

// lrce_layernorm_bwd + the scaled fp16 operand of the next GEMM in one pass (the BERT backward):
// dx (f32, optional) and dx_f16 = fp16(S * dropout_bwd(dx)), S = scale[0]; max|dx| -> scale word 2
// (lrce_grad_scale_update turns it into the next step's S).  Identity maps, no residual, f32 dy / x.
static int layernorm_bwd_f16s_impl(const float* dy, const float* x, const float* mean, const float* rstd, const float* w,
                                   float* dx, float* dw, float* db, int rows, int cols, uint16_t* dx_f16, float* scale,
                                   float p, uint64_t seed, float* workspace, int64_t workspace_elems, void* stream,
                                   int* defer_nb) {
  if (defer_nb) *defer_nb = 0;
  if (!dy || !x || !mean || !rstd || !w || !dx_f16 || !scale) return lrce_fail(LRCE_E_ARG, "layernorm_bwd_f16s: null pointer");
  if (cols % 4 || cols > 64 * 4 * MAXC || cols / 4 <= 32) return lrce_fail(LRCE_E_ARG, "layernorm_bwd_f16s: cols=%d", cols);
  if (rows <= 0) return LRCE_OK;
  hipStream_t s = static_cast<hipStream_t>(stream);
  const int nch = cols / 4;
  const bool want = dw || db;
  const int nb_ws = ln_bwd_blocks(rows, 64, true, cols);
  const int ny = (nb_ws + LN_RED_ROWS - 1) / LN_RED_ROWS;
  float* part = want && nb_ws > 1 && workspace && workspace_elems >= (int64_t)(nb_ws + ny) * 2 * cols + LN_RED_CTRS
                    ? workspace : nullptr;
  const int nb = (part || !want) ? nb_ws : ln_bwd_blocks(rows, 64, false, cols);
  const F16Scaled fs{scale, p > 0.f ? p : 0.f, seed, p > 0.f ? lrce_rng_offset() : nullptr};
  bf16* o16 = reinterpret_cast<bf16*>(dx_f16);
#define LNBS(CH)                                                                                                    \
  ln_bwd<float, float, CH, 64, true><<<nb, 256, 0, s>>>(dy, nullptr, x, nullptr, 1, mean, rstd, w, dx, nullptr, dw, db, \
                                                        rows, cols, o16, nullptr, nullptr, 1, part, fs)
  if (nch <= 64) LNBS(1);
  else if (nch <= 128) LNBS(2);
  else if (nch <= 192) LNBS(3);
  else if (nch <= 256) LNBS(4);
  else LNBS(8);
#undef LNBS
  if (part && defer_nb) *defer_nb = nb;
  else if (part)
    ln_bwd_reduce<<<dim3((2 * cols + 63) / 64, ny), 256, 0, s>>>(
        part, nb, cols, dw, db, part + (long long)nb * 2 * cols, reinterpret_cast<unsigned*>(part + (long long)(nb + ny) * 2 * cols));
  return lrce_check_launch("layernorm_bwd_f16s");
}

extern "C" int lrce_layernorm_bwd_f16s(const float* dy, const float* x, const float* mean, const float* rstd, const float* w,
                                       float* dx, float* dw, float* db, int rows, int cols, uint16_t* dx_f16, float* scale,
                                       float p, uint64_t seed, float* workspace, int64_t workspace_elems, void* stream) {
  return layernorm_bwd_f16s_impl(dy, x, mean, rstd, w, dx, dw, db, rows, cols, dx_f16, scale, p, seed, workspace,
                                 workspace_elems, stream, nullptr);
}

extern "C" int lrce_layernorm_bwd_f16s_deferred(const float* dy, const float* x, const float* mean, const float* rstd,
                                                const float* w, float* dx, float* dw, float* db, int rows, int cols,
                                                uint16_t* dx_f16, float* scale, float p, uint64_t seed, float* workspace,
                                                int64_t workspace_elems, int* nb_out, void* stream) {
  if (!nb_out) return lrce_fail(LRCE_E_ARG, "layernorm_bwd_f16s_deferred: null nb_out");
  return layernorm_bwd_f16s_impl(dy, x, mean, rstd, w, dx, dw, db, rows, cols, dx_f16, scale, p, seed, workspace,
                                 workspace_elems, stream, nb_out);
}

extern "C" int64_t lrce_layernorm_bwd_workspace(int rows, int cols) {
  if (rows <= 0 || cols <= 0) return 0;
  const int nb = ln_bwd_blocks(rows, ln_bwd_lpr(cols), true, cols);
  return nb > 1 ? (int64_t)(nb + (nb + LN_RED_ROWS - 1) / LN_RED_ROWS) * 2 * cols + LN_RED_CTRS : 0;
}

extern "C" int lrce_splitk_reduce_ln(const float* ws, int split, int rows, int cols, const float* bias, const float* resid,
                                     int64_t ld_res, float p, uint64_t seed, float* pre, const float* gamma,
                                     const float* beta, float eps, float* y, uint16_t* y16, int y16_f16, float* mean,
                                     float* rstd, void* stream) {
  if (!ws || !gamma || !beta || !y) return lrce_fail(LRCE_E_ARG, "splitk_reduce_ln: null pointer");
  if (split < 1 || rows < 0 || cols % 256 || cols < 256 || cols > 1024 || (resid && ld_res % 4))
    return lrce_fail(LRCE_E_ARG, "splitk_reduce_ln: split=%d cols=%d ld_res=%lld", split, cols, (long long)ld_res);
  if (rows == 0) return LRCE_OK;
  hipStream_t s = static_cast<hipStream_t>(stream);
  const uint64_t* off = p > 0.f ? lrce_rng_offset() : nullptr;
  const dim3 grid((unsigned)((rows + 3) / 4));
  bf16* o16 = reinterpret_cast<bf16*>(y16);
#define LRCE_SRL(CH) splitk_reduce_ln_kernel<CH><<<grid, 256, 0, s>>>(ws, split, rows, cols, bias, resid, ld_res, p, seed, off, \
                                                                      pre, gamma, beta, eps, y, o16, y16_f16, mean, rstd)
  switch (cols / 256) {
    case 1: LRCE_SRL(1); break;
    case 2: LRCE_SRL(2); break;
    case 3: LRCE_SRL(3); break;
    default: LRCE_SRL(4); break;
  }
#undef LRCE_SRL
  return lrce_check_launch("splitk_reduce_ln");
}
