// LayerNorm forward/backward, one wave per row, with fused row gather/scatter.
//
// The gather (in_map, nseg segments per row) fuses three reference data movements into the LN
// read: torch.roll + window_partition before the attention (video_swin_ori.py:262,268), the 2x2
// PatchMerging concat (:333-337), and identity for plain LNs.  HBM-bound: one read of x, one write
// of y, 8 B of stats per row.
#include "common.h"
#include "lrce_capi.h"

namespace {

constexpr int MAXC = 8;  // float4 chunks per lane -> cols <= 2048

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

// address of the 4-chunk c (element 4c) of LN row r inside x
__device__ __forceinline__ long long src_off(const int* in_map, int nseg, int seg, int r, int c, int& valid) {
  const int e = c * 4;
  if (!in_map) { valid = 1; return (long long)r * (seg * nseg) + e; }
  const int s = e / seg;
  const int src = in_map[(long long)r * nseg + s];
  valid = src >= 0;
  return (long long)src * seg + (e - s * seg);
}

template <typename TX, typename TY>
__global__ void __launch_bounds__(256) ln_fwd(const TX* x, const int* in_map, int nseg, const float* w, const float* b,
                                              float eps, TY* y, bf16* y2, const int* out_map, float* mean_o, float* rstd_o,
                                              int rows, int cols) {
  const int lane = threadIdx.x & 63;
  const int r = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (r >= rows) return;
  const int nch = cols >> 2, seg = cols / nseg;
  float4 v[MAXC];
  float s = 0.f;
#pragma unroll
  for (int t = 0; t < MAXC; ++t) {
    const int c = lane + 64 * t;
    if (c < nch) {
      int ok;
      const long long o = src_off(in_map, nseg, seg, r, c, ok);
      v[t] = ok ? ld4<TX>(x + o) : make_float4(0.f, 0.f, 0.f, 0.f);
      s += v[t].x + v[t].y + v[t].z + v[t].w;
    }
  }
  const float mean = wave_sum(s) / cols;
  float q = 0.f;
#pragma unroll
  for (int t = 0; t < MAXC; ++t) {
    const int c = lane + 64 * t;
    if (c < nch) {
      const float a = v[t].x - mean, b2 = v[t].y - mean, c2 = v[t].z - mean, d = v[t].w - mean;
      q += a * a + b2 * b2 + c2 * c2 + d * d;
    }
  }
  const float rstd = rsqrtf(wave_sum(q) / cols + eps);
  const long long orow = out_map ? (long long)out_map[r] : (long long)r;
#pragma unroll
  for (int t = 0; t < MAXC; ++t) {
    const int c = lane + 64 * t;
    if (c < nch) {
      const float4 ww = *reinterpret_cast<const float4*>(w + 4 * c);
      const float4 bb = *reinterpret_cast<const float4*>(b + 4 * c);
      float4 o;
      o.x = (v[t].x - mean) * rstd * ww.x + bb.x;
      o.y = (v[t].y - mean) * rstd * ww.y + bb.y;
      o.z = (v[t].z - mean) * rstd * ww.z + bb.z;
      o.w = (v[t].w - mean) * rstd * ww.w + bb.w;
      st4<TY>(y + orow * cols + 4 * c, o);
      if (y2) st4<bf16>(y2 + orow * cols + 4 * c, o);
    }
  }
  if (lane == 0) {
    if (mean_o) mean_o[r] = mean;
    if (rstd_o) rstd_o[r] = rstd;
  }
}

template <typename TD, typename TX>
__global__ void __launch_bounds__(256) ln_bwd(const TD* dy, const int* dy_map, const TX* x, const int* in_map, int nseg,
                                              const float* mean_i, const float* rstd_i, const float* w, float* dx,
                                              const float* dres, float* dw, float* db, int rows, int cols) {
  __shared__ float red[2][4][1024 + 4];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int nch = cols >> 2, seg = cols / nseg;
  float4 aw[MAXC], ab[MAXC];  // dw/db partials for up to 8 chunks per lane (cols<=2048)
#pragma unroll
  for (int t = 0; t < 8; ++t) { aw[t] = make_float4(0.f, 0.f, 0.f, 0.f); ab[t] = aw[t]; }
  for (int r = blockIdx.x * 4 + wave; r < rows; r += gridDim.x * 4) {
    const float mean = mean_i[r], rstd = rstd_i[r];
    const long long dyr = dy_map ? (long long)dy_map[r] : (long long)r;
    float4 xh[8], g[8];
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int t = 0; t < 8; ++t) {
      const int c = lane + 64 * t;
      if (c < nch) {
        int ok;
        const long long o = src_off(in_map, nseg, seg, r, c, ok);
        float4 xv = ok ? ld4<TX>(x + o) : make_float4(0.f, 0.f, 0.f, 0.f);
        xh[t] = make_float4((xv.x - mean) * rstd, (xv.y - mean) * rstd, (xv.z - mean) * rstd, (xv.w - mean) * rstd);
        const float4 d = ld4<TD>(dy + dyr * cols + 4 * c);
        const float4 ww = *reinterpret_cast<const float4*>(w + 4 * c);
        g[t] = make_float4(d.x * ww.x, d.y * ww.y, d.z * ww.z, d.w * ww.w);
        s1 += g[t].x + g[t].y + g[t].z + g[t].w;
        s2 += g[t].x * xh[t].x + g[t].y * xh[t].y + g[t].z * xh[t].z + g[t].w * xh[t].w;
        aw[t].x += d.x * xh[t].x; aw[t].y += d.y * xh[t].y; aw[t].z += d.z * xh[t].z; aw[t].w += d.w * xh[t].w;
        ab[t].x += d.x; ab[t].y += d.y; ab[t].z += d.z; ab[t].w += d.w;
      }
    }
    const float c1 = wave_sum(s1) / cols, c2 = wave_sum(s2) / cols;
#pragma unroll
    for (int t = 0; t < 8; ++t) {
      const int c = lane + 64 * t;
      if (c < nch) {
        int ok;
        const long long o = src_off(in_map, nseg, seg, r, c, ok);
        if (!ok) continue;
        float4 out;
        out.x = rstd * (g[t].x - c1 - xh[t].x * c2);
        out.y = rstd * (g[t].y - c1 - xh[t].y * c2);
        out.z = rstd * (g[t].z - c1 - xh[t].z * c2);
        out.w = rstd * (g[t].w - c1 - xh[t].w * c2);
        if (dres) {
          const float4 rr = *reinterpret_cast<const float4*>(dres + o);
          out.x += rr.x; out.y += rr.y; out.z += rr.z; out.w += rr.w;
        }
        *reinterpret_cast<float4*>(dx + o) = out;
      }
    }
  }
  if (!dw && !db) return;
  // reduce the 4 waves' partials through LDS in 1024-column slabs, then one atomic per column
  for (int base = 0; base < cols; base += 1024) {
#pragma unroll
    for (int t = 0; t < 8; ++t) {
      const int c = lane + 64 * t;
      const int e = 4 * c - base;
      if (c < nch && e >= 0 && e < 1024) {
        red[0][wave][e] = aw[t].x; red[0][wave][e + 1] = aw[t].y; red[0][wave][e + 2] = aw[t].z; red[0][wave][e + 3] = aw[t].w;
        red[1][wave][e] = ab[t].x; red[1][wave][e + 1] = ab[t].y; red[1][wave][e + 2] = ab[t].z; red[1][wave][e + 3] = ab[t].w;
      }
    }
    __syncthreads();
    for (int e = threadIdx.x; e < 1024 && base + e < cols; e += 256) {
      const float sw = red[0][0][e] + red[0][1][e] + red[0][2][e] + red[0][3][e];
      const float sb = red[1][0][e] + red[1][1][e] + red[1][2][e] + red[1][3][e];
      if (dw) atomicAdd(dw + base + e, sw);
      if (db) atomicAdd(db + base + e, sb);
    }
    __syncthreads();
  }
}

}  // namespace

extern "C" int lrce_layernorm_fwd(const void* x, int x_f32, const int32_t* in_map, int nseg, const float* w,
                                  const float* b, float eps, void* y, int y_f32, uint16_t* y2, const int32_t* out_map,
                                  float* mean, float* rstd, int rows, int cols, void* stream) {
  if (!x || !y || !w || !b) return lrce_fail(LRCE_E_ARG, "layernorm_fwd: null pointer");
  if (nseg < 1) nseg = 1;
  if (cols % 4 || (cols / nseg) % 4 || cols % nseg || cols > 64 * 4 * MAXC)
    return lrce_fail(LRCE_E_ARG, "layernorm_fwd: cols=%d nseg=%d unsupported", cols, nseg);
  if (rows <= 0) return LRCE_OK;
  dim3 grid((rows + 3) / 4);
  hipStream_t s = static_cast<hipStream_t>(stream);
#define LNF(TX, TY) ln_fwd<TX, TY><<<grid, 256, 0, s>>>(static_cast<const TX*>(x), in_map, nseg, w, b, eps, static_cast<TY*>(y), reinterpret_cast<bf16*>(y2), out_map, mean, rstd, rows, cols)
  if (x_f32 && y_f32) LNF(float, float);
  else if (x_f32) LNF(float, bf16);
  else if (y_f32) LNF(bf16, float);
  else LNF(bf16, bf16);
#undef LNF
  return lrce_check_launch("layernorm_fwd");
}

extern "C" int lrce_layernorm_bwd(const void* dy, int dy_f32, const int32_t* dy_map, const void* x, int x_f32,
                                  const int32_t* in_map, int nseg, const float* mean, const float* rstd, const float* w,
                                  float* dx, const float* dres, float* dw, float* db, int rows, int cols, void* stream) {
  if (!dy || !x || !mean || !rstd || !w || !dx) return lrce_fail(LRCE_E_ARG, "layernorm_bwd: null pointer");
  if (nseg < 1) nseg = 1;
  if (cols % 4 || (cols / nseg) % 4 || cols % nseg || cols > 64 * 4 * MAXC)
    return lrce_fail(LRCE_E_ARG, "layernorm_bwd: cols=%d nseg=%d unsupported", cols, nseg);
  if (rows <= 0) return LRCE_OK;
  int nblk = (rows + 3) / 4;
  if (nblk > 1024) nblk = 1024;
  hipStream_t s = static_cast<hipStream_t>(stream);
#define LNB(TD, TX) ln_bwd<TD, TX><<<nblk, 256, 0, s>>>(static_cast<const TD*>(dy), dy_map, static_cast<const TX*>(x), in_map, nseg, mean, rstd, w, dx, dres, dw, db, rows, cols)
  if (dy_f32 && x_f32) LNB(float, float);
  else if (dy_f32) LNB(float, bf16);
  else if (x_f32) LNB(bf16, float);
  else LNB(bf16, bf16);
#undef LNB
  return lrce_check_launch("layernorm_bwd");
}
