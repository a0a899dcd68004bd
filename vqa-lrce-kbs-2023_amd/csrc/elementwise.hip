// Memory-bound helpers on the LRCE path: patch im2col (+ImageNet normalise +T padding), bias
// column sums, casts, dropout, and the embedding sums of BERT / LRCE positional embeddings.
// All vectorised 16 B per lane where the layout allows; HBM-bound by construction.
#include <algorithm>

#include "common.h"
#include "lrce_capi.h"

namespace {

// ---------------------------------------------------------------- patch im2col
// clip n, frame t, channel c at clips[n*s_clip + t*s_t + c*s_c + y*W + x] (f32) ->
// patches bf16 [(n*Dp + d)*Hp*Wp + h*Wp + w][96], column = c*32 + kt*16 + kh*4 + kw (the conv3d
// weight [128][3][2][4][4] flattened).  Normalize (video.py:35, if `normalize`) precedes the zero
// padding of T to a multiple of 2 (video_swin_ori.py:472-473): padded frames are exactly 0.
// One workgroup per strip (n, d, h) of Wp consecutive tokens: the strip's 24 source row segments
// (c, kt, kh: 4 W floats each) are read as whole rows — consecutive threads, consecutive 16 B — and
// transposed through LDS (token pitch 208 B: the 8-B writes of 16 consecutive tokens hit distinct
// banks) into the strip's Wp x 192 B of output, written as contiguous 16-B pieces.  (A wave per token
// with 24 active lanes, each reading 16 B of a different row: 81 us for the bs-10 step's 282 240
// tokens, 1.8 TB/s.)
constexpr int I2C_PITCH = 104;   // bf16 per token row in LDS (96 + 8: 208 B)
__global__ void __launch_bounds__(256) im2col_kernel(const float* __restrict__ clips, bf16* __restrict__ out, int T, int H,
                                                     int W, long long s_clip, long long s_t, long long s_c, int normalize) {
  extern __shared__ __attribute__((aligned(16))) char i2c_lds[];
  bf16* tile = reinterpret_cast<bf16*>(i2c_lds);
  const int Dp = (T + 1) / 2, Hp = H / 4, Wp = W / 4;
  const int strip = blockIdx.x;
  const int h = strip % Hp, d = (strip / Hp) % Dp;
  const long long n = strip / (Hp * Dp);
  for (int i = threadIdx.x; i < 24 * Wp; i += blockDim.x) {
    const int r = i / Wp, w = i - r * Wp;   // r = (c, kt, kh): column block r*4 .. r*4+3
    const int c = r >> 3, kt = (r >> 2) & 1, kh = r & 3;
    const int frame = 2 * d + kt;
    bf16x4 o;
    if (frame < T) {
      float mean = 0.f, istd = 1.f;
      if (normalize) {
        mean = c == 0 ? 0.485f : (c == 1 ? 0.456f : 0.406f);
        istd = c == 0 ? 1.0f / 0.229f : (c == 1 ? 1.0f / 0.224f : 1.0f / 0.225f);
      }
      const float4 v = *reinterpret_cast<const float4*>(clips + n * s_clip + frame * s_t + c * s_c + (long long)(4 * h + kh) * W + 4 * w);
      o[0] = f2bf((v.x - mean) * istd); o[1] = f2bf((v.y - mean) * istd);
      o[2] = f2bf((v.z - mean) * istd); o[3] = f2bf((v.w - mean) * istd);
    } else {
      o[0] = o[1] = o[2] = o[3] = f2bf(0.f);
    }
    *reinterpret_cast<bf16x4*>(tile + w * I2C_PITCH + r * 4) = o;
  }
  __syncthreads();
  uint4* dst = reinterpret_cast<uint4*>(out + (long long)strip * Wp * 96);
  for (int i = threadIdx.x; i < Wp * 12; i += blockDim.x) {
    const int w = i / 12, part = i - w * 12;
    dst[i] = *reinterpret_cast<const uint4*>(tile + w * I2C_PITCH + part * 8);
  }
}

// ---------------------------------------------------------------- column sums
// block: 256 threads = 64 lanes x V consecutive columns x 4 row groups; grid.x over column blocks,
// grid.y over row chunks; V = 4 (16-B f32 / 8-B bf16 loads) when rows are aligned.
template <typename T, int V>
__global__ void colsum_kernel(const T* __restrict__ x, const int* __restrict__ map, long long ld, int m, int n,
                              const float* __restrict__ rsc, int rps, float* __restrict__ out) {
  const int col = (blockIdx.x * 64 + (threadIdx.x & 63)) * V;
  const int rg = threadIdx.x >> 6;
  const int rows_per = (m + gridDim.y - 1) / gridDim.y;
  const int r0 = blockIdx.y * rows_per, r1 = min(m, r0 + rows_per);
  float s[V];
#pragma unroll
  for (int i = 0; i < V; ++i) s[i] = 0.f;
  if (col < n) {
    for (int r = r0 + rg; r < r1; r += 4) {
      const long long rr = map ? (long long)map[r] : (long long)r;
      const float f = rsc ? rsc[r / rps] : 1.0f;
      const T* src = x + rr * ld + col;
      if constexpr (V == 4) {
        if constexpr (sizeof(T) == 4) {
          const float4 v = *reinterpret_cast<const float4*>(src);
          s[0] += v.x * f; s[1] += v.y * f; s[2] += v.z * f; s[3] += v.w * f;
        } else {
          const bf16x4 v = *reinterpret_cast<const bf16x4*>(src);
          s[0] += bf2f(v[0]) * f; s[1] += bf2f(v[1]) * f; s[2] += bf2f(v[2]) * f; s[3] += bf2f(v[3]) * f;
        }
      } else {
        s[0] += (float)src[0] * f;
      }
    }
  }
  __shared__ float red[4][64 * V];
#pragma unroll
  for (int i = 0; i < V; ++i) red[rg][(threadIdx.x & 63) * V + i] = s[i];
  __syncthreads();
  if (rg == 0) {
#pragma unroll
    for (int i = 0; i < V; ++i) {
      const int c = (threadIdx.x & 63) * V + i;
      if (col + i < n) atomicAdd(out + col + i, red[0][c] + red[1][c] + red[2][c] + red[3][c]);
    }
  }
}

__global__ void cast_kernel(const float* __restrict__ x, bf16* __restrict__ y, long long n) {
  const long long i = ((long long)blockIdx.x * blockDim.x + threadIdx.x) * 4;
  if (i + 3 < n) {
    const float4 v = *reinterpret_cast<const float4*>(x + i);
    bf16x4 o;
    o[0] = f2bf(v.x); o[1] = f2bf(v.y); o[2] = f2bf(v.z); o[3] = f2bf(v.w);
    *reinterpret_cast<bf16x4*>(y + i) = o;
  } else {
    for (long long j = i; j < n; ++j) y[j] = f2bf(x[j]);
  }
}

__global__ void cast_f16_kernel(const float* __restrict__ x, bf16* __restrict__ y, long long n) {
  const long long i = ((long long)blockIdx.x * blockDim.x + threadIdx.x) * 4;
  if (i + 3 < n) {
    const float4 v = *reinterpret_cast<const float4*>(x + i);
    bf16x4 o;
    o[0] = to16<true>(v.x); o[1] = to16<true>(v.y); o[2] = to16<true>(v.z); o[3] = to16<true>(v.w);
    *reinterpret_cast<bf16x4*>(y + i) = o;
  } else {
    for (long long j = i; j < n; ++j) y[j] = to16<true>(x[j]);
  }
}

// fp16 -> bf16, 8 elements per thread (16-B loads / stores)
__global__ void f16_bf16_kernel(const bf16* __restrict__ x, bf16* __restrict__ y, long long n) {
  const long long i = ((long long)blockIdx.x * blockDim.x + threadIdx.x) * 8;
  if (i + 7 < n) {
    const bf16x8 v = *reinterpret_cast<const bf16x8*>(x + i);
    bf16x8 o;
#pragma unroll
    for (int e = 0; e < 8; ++e) o[e] = f2bf(from16<true>(v[e]));
    *reinterpret_cast<bf16x8*>(y + i) = o;
  } else {
    for (long long j = i; j < n; ++j) y[j] = f2bf(from16<true>(x[j]));
  }
}

// W64: more than 2^32 float4s (64-bit row arithmetic); otherwise the row of float4 i is a 32-bit
// division instead of the 64-bit software routine (tools/im2col_bench.py: 15 680 x 512 9.4 -> 8.6 us,
// 3 920 x 1024 9.2 -> 6.7 us)
template <bool W64>
__global__ void scale_cast_kernel(const float* __restrict__ x, long long n4, int cols4, const float* __restrict__ rsc, int rps,
                                  bf16* __restrict__ y) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n4) return;
  const long long e = i * 4;
  float f = 1.f;
  if (rsc) {
    const unsigned row = W64 ? (unsigned)(i / cols4) : (unsigned)i / (unsigned)cols4;
    f = rsc[row / (unsigned)rps];
  }
  const float4 v = *reinterpret_cast<const float4*>(x + e);
  bf16x4 o;
  o[0] = f2bf(v.x * f); o[1] = f2bf(v.y * f); o[2] = f2bf(v.z * f); o[3] = f2bf(v.w * f);
  *reinterpret_cast<bf16x4*>(y + e) = o;
}

__global__ void dropout_kernel(const float* __restrict__ x, const float* __restrict__ res, float* __restrict__ y,
                               bf16* __restrict__ yb, long long n, float p, uint64_t seed, long long group,
                               const uint64_t* __restrict__ off) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  float v = x[i];
  if (p > 0.f) v = (lrce_uniform(lrce_seed(seed, off), i / group) >= p) ? v / (1.0f - p) : 0.f;
  if (res) v += res[i];
  y[i] = v;
  if (yb) yb[i] = f2bf(v);
}

__global__ void dropout_bwd_kernel(const float* __restrict__ dy, float* __restrict__ dx, bf16* __restrict__ dx16, long long n,
                                   float p, uint64_t seed, long long group, const uint64_t* __restrict__ off) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  float v = dy[i];
  if (p > 0.f) v = (lrce_uniform(lrce_seed(seed, off), i / group) >= p) ? v / (1.0f - p) : 0.f;
  if (dx) dx[i] = v;
  if (dx16) dx16[i] = f2bf(v);
}

// GradScaler restated per tensor for the fp16 backward (agent_oe.py:40-42): max|x| over the grid
// (NaN-propagating), then the last block to arrive turns it into a power-of-two scale.  The arrival
// words live in scale[2..3] (agent-scope atomics on both sides; the last block resets them).
__global__ void __launch_bounds__(256) grad_scale_kernel(const float* __restrict__ x, long long n4, float* scale) {
  unsigned* words = reinterpret_cast<unsigned*>(scale + 2);
  __shared__ float red[4];
  float m = 0.f;
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < n4; i += (long long)gridDim.x * 256) {
    const float4 v = reinterpret_cast<const float4*>(x)[i];
    const float a[4] = {fabsf(v.x), fabsf(v.y), fabsf(v.z), fabsf(v.w)};
#pragma unroll
    for (int e = 0; e < 4; ++e) m = (a[e] > m || a[e] != a[e]) ? a[e] : m;   // NaN sticks
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float t = __shfl_xor(m, o, 64);
    m = (t > m || t != t) ? t : m;
  }
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = m;
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int w = 1; w < 4; ++w) m = (red[w] > m || red[w] != red[w]) ? red[w] : m;
    // |x| bit patterns order like the values (NaN above +inf)
    __hip_atomic_fetch_max(&words[0], __float_as_uint(m), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (__hip_atomic_fetch_add(&words[1], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == gridDim.x - 1) {
      const unsigned bits = __hip_atomic_fetch_max(&words[0], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const int e = (int)((bits >> 23) & 0xFF) - 127;          // floor(log2(max|x|)) for a normal max
      float s = 1.f;
      if (bits != 0 && e < 128 && e > -127) s = ldexpf(1.f, min(100, max(-100, 7 - e)));
      scale[0] = s;
      scale[1] = 1.f / s;
      __hip_atomic_store(&words[0], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(&words[1], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

// Delayed per-tensor scales (lrce_layernorm_bwd_f16s): slot i's max |x| of the last step (word 2,
// accumulated by the fused LN backward) becomes its scale S = 2^(7 - floor(log2 max)) and 1/S, and the
// word is cleared for this step, as is the found-inf flag (word 3, read by the last step's optimizer
// update); a slot with no recorded max keeps its scale.  One thread per slot.
__global__ void grad_scale_update_kernel(float* __restrict__ scale, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  float* sc = scale + 4 * i;
  unsigned* words = reinterpret_cast<unsigned*>(sc + 2);
  const unsigned bits = words[0];
  words[1] = 0u;
  if (bits == 0u) return;
  const int e = (int)((bits >> 23) & 0xFF) - 127;
  float s = 1.f;
  if (e < 128 && e > -127) s = ldexpf(1.f, min(100, max(-100, 7 - e)));
  else if (e >= 128) s = fmaxf(sc[0] * 0.5f, ldexpf(1.f, -100));   // inf / NaN max: back off (GradScaler)
  sc[0] = s;
  sc[1] = 1.f / s;
  words[0] = 0u;
}

__global__ void dropout_bwd_f16_kernel(const float* __restrict__ dy, f16* __restrict__ dx, long long n, float p, uint64_t seed,
                                       long long group, const uint64_t* __restrict__ off, const float* __restrict__ scale) {
  const long long i = ((long long)blockIdx.x * blockDim.x + threadIdx.x) * 4;
  if (i >= n) return;
  const float s = scale[0] / (p > 0.f ? 1.0f - p : 1.0f);
  const float4 v = *reinterpret_cast<const float4*>(dy + i);
  float o[4] = {v.x * s, v.y * s, v.z * s, v.w * s};
  if (p > 0.f) {
    const uint64_t sd = lrce_seed(seed, off);
#pragma unroll
    for (int e = 0; e < 4; ++e) o[e] = lrce_uniform(sd, (i + e) / group) >= p ? o[e] : 0.f;
  }
  typedef __attribute__((ext_vector_type(4))) _Float16 f16x4;
  f16x4 h;
#pragma unroll
  for (int e = 0; e < 4; ++e) h[e] = (f16)o[e];
  *reinterpret_cast<f16x4*>(dx + i) = h;
}

// ---------------------------------------------------------------- embeddings
// BERT: out[r][c] = word[ids[r]][c] + pos[r % L][c] + type[types[r]][c]
__global__ void bert_embed_kernel(const long long* __restrict__ ids, const long long* __restrict__ types, const float* __restrict__ word,
                                  const float* __restrict__ pos, const float* __restrict__ typ, float* __restrict__ out, int rows, int L,
                                  int C) {
  const long long e = ((long long)blockIdx.x * blockDim.x + threadIdx.x) * 4;
  if (e >= (long long)rows * C) return;
  const int r = e / C, c = e % C;
  const float4 a = *reinterpret_cast<const float4*>(word + ids[r] * C + c);
  const float4 b = *reinterpret_cast<const float4*>(pos + (long long)(r % L) * C + c);
  const float4 t = *reinterpret_cast<const float4*>(typ + types[r] * C + c);
  *reinterpret_cast<float4*>(out + e) = make_float4(a.x + b.x + t.x, a.y + b.y + t.y, a.z + b.z + t.z, a.w + b.w + t.w);
}
__global__ void bert_embed_bwd_kernel(const float* __restrict__ d, const long long* __restrict__ ids, const long long* __restrict__ types,
                                      float* __restrict__ dword, float* __restrict__ dpos, float* __restrict__ dtyp, int rows, int L, int C,
                                      long long pad_id) {
  const long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= (long long)rows * C) return;
  const int r = e / C, c = e % C;
  const float g = d[e];
  if (ids[r] != pad_id) atomicAdd(dword + ids[r] * C + c, g);  // nn.Embedding(padding_idx): no grad
  atomicAdd(dpos + (long long)(r % L) * C + c, g);
  atomicAdd(dtyp + types[r] * C + c, g);
}

// LRCE VideoPosEmbed (embedding.py:47-63) before its LayerNorm:
// out[b,s,t,p,c] = (p == 0 ? cls[c] : x[b,s,t,p-1,c]) + pos[p,c] + len[t,c] + clip[s,c]
__global__ void video_pos_kernel(const float* __restrict__ x, const float* __restrict__ cls, const float* __restrict__ pos,
                                 const float* __restrict__ len, const float* __restrict__ clip, float* __restrict__ out, int B, int S,
                                 int Tg, int P, int C) {
  const long long e = ((long long)blockIdx.x * blockDim.x + threadIdx.x) * 4;
  const long long total = (long long)B * S * Tg * (P + 1) * C;
  if (e >= total) return;
  long long t = e / C;
  const int c = e % C;
  const int p = t % (P + 1); t /= (P + 1);
  const int tg = t % Tg; t /= Tg;
  const int s = t % S;
  const long long bst = t * Tg + tg;  // (b*S + s)*Tg + tg
  float4 v = p == 0 ? *reinterpret_cast<const float4*>(cls + c)
                    : *reinterpret_cast<const float4*>(x + (bst * P + (p - 1)) * C + c);
  const float4 a = *reinterpret_cast<const float4*>(pos + (long long)p * C + c);
  const float4 l = *reinterpret_cast<const float4*>(len + (long long)tg * C + c);
  const float4 k = *reinterpret_cast<const float4*>(clip + (long long)s * C + c);
  *reinterpret_cast<float4*>(out + e) = make_float4(v.x + a.x + l.x + k.x, v.y + a.y + l.y + k.y, v.z + a.z + l.z + k.z, v.w + a.w + l.w + k.w);
}
// Backward of the above: one block per (clip s, frame group tg) x VP_PPB positions p, one lane per
// float4 column.  The B rows of a (s, tg, p) are loaded 8 at a time (independent loads in flight),
// summed in registers and copied out to dx (f32) and / or dx16 (bf16: the projection GEMMs' operand);
// the table gradients take the per-lane partial sums by atomics (dpos / dcls: S*Tg adds per element,
// dlen / dclip: one per block).
constexpr int VP_PPB = 2;
__global__ void __launch_bounds__(256) video_pos_bwd_kernel(const float* __restrict__ d, float* __restrict__ dx, bf16* __restrict__ dx16,
                                                            float* __restrict__ dcls, float* __restrict__ dpos, float* __restrict__ dlen,
                                                            float* __restrict__ dclip, int B, int S, int Tg, int P, int C) {
  const int s = blockIdx.x / Tg, tg = blockIdx.x % Tg;
  const int p0 = blockIdx.y * VP_PPB;
  const float4 z4 = make_float4(0.f, 0.f, 0.f, 0.f);
  auto add4 = [](float4& a, const float4& b) { a.x += b.x; a.y += b.y; a.z += b.z; a.w += b.w; };
  auto atom4 = [](float* dst, const float4& v) {
    atomicAdd(dst, v.x); atomicAdd(dst + 1, v.y); atomicAdd(dst + 2, v.z); atomicAdd(dst + 3, v.w);
  };
  for (int c = 4 * threadIdx.x; c < C; c += 4 * blockDim.x) {
    float4 acc = z4;
    for (int p = p0; p < p0 + VP_PPB && p <= P; ++p) {
      float4 sp = z4;
      for (int b0 = 0; b0 < B; b0 += 8) {
        float4 g[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          const long long bst = ((long long)(b0 + u) * S + s) * Tg + tg;
          g[u] = b0 + u < B ? *reinterpret_cast<const float4*>(d + (bst * (P + 1) + p) * C + c) : z4;
        }
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          if (b0 + u >= B) break;
          add4(sp, g[u]);
          if (p > 0) {
            const long long o = ((((long long)(b0 + u) * S + s) * Tg + tg) * P + (p - 1)) * C + c;
            if (dx) *reinterpret_cast<float4*>(dx + o) = g[u];
            if (dx16) {
              bf16x4 h;
              h[0] = f2bf(g[u].x); h[1] = f2bf(g[u].y); h[2] = f2bf(g[u].z); h[3] = f2bf(g[u].w);
              *reinterpret_cast<bf16x4*>(dx16 + o) = h;
            }
          }
        }
      }
      atom4(dpos + (long long)p * C + c, sp);
      if (p == 0) atom4(dcls + c, sp);
      add4(acc, sp);
    }
    atom4(dlen + (long long)tg * C + c, acc);
    atom4(dclip + (long long)s * C + c, acc);
  }
}

// TextPosEmbed (embedding.py:17-23): out[b,l,c] = (l == 0 ? cls[c] : x[b,l-1,c]) + pos[l,c]
__global__ void text_pos_kernel(const float* __restrict__ x, const float* __restrict__ cls, const float* __restrict__ pos,
                                float* __restrict__ out, int B, int L, int C) {
  const long long e = ((long long)blockIdx.x * blockDim.x + threadIdx.x) * 4;
  if (e >= (long long)B * (L + 1) * C) return;
  const long long r = e / C;
  const int c = e % C, l = r % (L + 1), b = r / (L + 1);
  float4 v = l == 0 ? *reinterpret_cast<const float4*>(cls + c) : *reinterpret_cast<const float4*>(x + ((long long)b * L + l - 1) * C + c);
  const float4 a = *reinterpret_cast<const float4*>(pos + (long long)l * C + c);
  *reinterpret_cast<float4*>(out + e) = make_float4(v.x + a.x, v.y + a.y, v.z + a.z, v.w + a.w);
}
__global__ void text_pos_bwd_kernel(const float* __restrict__ d, float* __restrict__ dx, float* __restrict__ dcls, float* __restrict__ dpos,
                                    int B, int L, int C) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  const int l = blockIdx.y;
  if (c >= C) return;
  float s = 0.f;
  for (int b = 0; b < B; ++b) {
    const float g = d[((long long)b * (L + 1) + l) * C + c];
    s += g;
    if (l > 0) dx[((long long)b * L + l - 1) * C + c] = g;
  }
  dpos[(long long)l * C + c] += s;
  if (l == 0) dcls[c] += s;
}

}  // namespace

extern "C" int lrce_patch_im2col(const float* clips, int n_clips, int T, int H, int W, int64_t s_clip, int64_t s_t,
                                 int64_t s_c, int normalize, uint16_t* patches, void* stream) {
  if (!clips || !patches) return lrce_fail(LRCE_E_ARG, "patch_im2col: null pointer");
  if (H % 4 || W % 4 || T < 1 || n_clips < 1) return lrce_fail(LRCE_E_ARG, "patch_im2col: H,W must be multiples of 4");
  if ((reinterpret_cast<uintptr_t>(clips) | reinterpret_cast<uintptr_t>(patches)) & 15 || s_clip % 4 || s_t % 4 || s_c % 4)
    return lrce_fail(LRCE_E_ARG, "patch_im2col: clips / patches must be 16-B aligned with strides of whole float4");
  const long long strips = (long long)n_clips * ((T + 1) / 2) * (H / 4);
  const size_t lds = (size_t)(W / 4) * I2C_PITCH * 2;
  if (lds > 64 * 1024) return lrce_fail(LRCE_E_ARG, "patch_im2col: W=%d too wide for one strip in LDS", W);
  im2col_kernel<<<(unsigned)strips, 256, lds, static_cast<hipStream_t>(stream)>>>(clips, reinterpret_cast<bf16*>(patches), T, H, W,
                                                                                 s_clip, s_t, s_c, normalize);
  return lrce_check_launch("patch_im2col");
}

extern "C" int lrce_colsum(const void* x, int x_f32, const int32_t* row_map, int64_t ld, int m, int n, const float* row_scale,
                           int rows_per_scale, float* out, void* stream) {
  if (rows_per_scale < 1) rows_per_scale = 1;
  if (!x || !out) return lrce_fail(LRCE_E_ARG, "colsum: null pointer");
  if (m <= 0 || n <= 0) return LRCE_OK;
  const bool vec = (n % 4 == 0) && (ld % 4 == 0) && ((reinterpret_cast<uintptr_t>(x) & (x_f32 ? 15 : 7)) == 0);
  const int V = vec ? 4 : 1;
  const int cblocks = (n + 64 * V - 1) / (64 * V);
  int chunks = (m + 63) / 64;                       // >= 16 rows per row group
  chunks = std::max(1, std::min(chunks, (1024 + cblocks - 1) / cblocks));
  dim3 grid(cblocks, chunks);
  hipStream_t s = static_cast<hipStream_t>(stream);
  if (x_f32) {
    if (vec) colsum_kernel<float, 4><<<grid, 256, 0, s>>>(static_cast<const float*>(x), row_map, ld, m, n, row_scale, rows_per_scale, out);
    else colsum_kernel<float, 1><<<grid, 256, 0, s>>>(static_cast<const float*>(x), row_map, ld, m, n, row_scale, rows_per_scale, out);
  } else {
    if (vec) colsum_kernel<bf16, 4><<<grid, 256, 0, s>>>(static_cast<const bf16*>(x), row_map, ld, m, n, row_scale, rows_per_scale, out);
    else colsum_kernel<bf16, 1><<<grid, 256, 0, s>>>(static_cast<const bf16*>(x), row_map, ld, m, n, row_scale, rows_per_scale, out);
  }
  return lrce_check_launch("colsum");
}

extern "C" int lrce_scale_cast_bf16(const float* x, int64_t rows, int cols, const float* row_scale, int rows_per_scale,
                                    uint16_t* y, void* stream) {
  if (!x || !y) return lrce_fail(LRCE_E_ARG, "scale_cast_bf16: null pointer");
  if (cols % 4) return lrce_fail(LRCE_E_ARG, "scale_cast_bf16: cols %% 4 != 0");
  if (rows_per_scale < 1) rows_per_scale = 1;
  const long long n4 = rows * (long long)cols / 4;
  if (n4 <= 0) return LRCE_OK;
  const auto kern = n4 >= (1LL << 32) ? scale_cast_kernel<true> : scale_cast_kernel<false>;
  kern<<<(unsigned)((n4 + 255) / 256), 256, 0, static_cast<hipStream_t>(stream)>>>(x, n4, cols / 4, row_scale, rows_per_scale,
                                                                                   reinterpret_cast<bf16*>(y));
  return lrce_check_launch("scale_cast_bf16");
}

// dst[i] = bf16(sum_r src[r * len + i]) with the sum in f32, r in ascending order (deterministic):
// the reduce step of the data-parallel gradient exchange (all-to-all of bf16 shards, this sum, then an
// all-gather), so the cross-rank sum is f32 with one bf16 rounding of the result.  8 elements / thread.
__global__ void sum_shards_kernel(const bf16* __restrict__ src, int nshard, long long len, bf16* __restrict__ dst) {
  const long long i = ((long long)blockIdx.x * blockDim.x + threadIdx.x) * 8;
  if (i >= len) return;
  float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  for (int r = 0; r < nshard; ++r) {
    const bf16x8 v = *reinterpret_cast<const bf16x8*>(src + (long long)r * len + i);
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[j] += bf2f(v[j]);
  }
  bf16x8 o;
#pragma unroll
  for (int j = 0; j < 8; ++j) o[j] = f2bf(acc[j]);
  *reinterpret_cast<bf16x8*>(dst + i) = o;
}

extern "C" int lrce_sum_shards_bf16(const uint16_t* src, int nshard, int64_t len, uint16_t* dst, void* stream) {
  if (!src || !dst) return lrce_fail(LRCE_E_ARG, "sum_shards_bf16: null pointer");
  if (nshard < 1 || len % 8 || ((reinterpret_cast<uintptr_t>(src) | reinterpret_cast<uintptr_t>(dst)) & 15))
    return lrce_fail(LRCE_E_ARG, "sum_shards_bf16: nshard=%d, len %% 8 == 0 and 16-B aligned buffers needed", nshard);
  if (len <= 0) return LRCE_OK;
  const long long thr = len / 8;
  sum_shards_kernel<<<(unsigned)((thr + 255) / 256), 256, 0, static_cast<hipStream_t>(stream)>>>(
      reinterpret_cast<const bf16*>(src), nshard, len, reinterpret_cast<bf16*>(dst));
  return lrce_check_launch("sum_shards_bf16");
}

extern "C" int lrce_cast_bf16(const float* x, uint16_t* y, int64_t n, void* stream) {
  if (!x || !y) return lrce_fail(LRCE_E_ARG, "cast_bf16: null pointer");
  if (n <= 0) return LRCE_OK;
  const long long thr = (n + 3) / 4;
  cast_kernel<<<(thr + 255) / 256, 256, 0, static_cast<hipStream_t>(stream)>>>(x, reinterpret_cast<bf16*>(y), n);
  return lrce_check_launch("cast_bf16");
}

extern "C" int lrce_cast_f16(const float* x, uint16_t* y, int64_t n, void* stream) {
  if (!x || !y) return lrce_fail(LRCE_E_ARG, "cast_f16: null pointer");
  if (n <= 0) return LRCE_OK;
  const long long thr = (n + 3) / 4;
  cast_f16_kernel<<<(thr + 255) / 256, 256, 0, static_cast<hipStream_t>(stream)>>>(x, reinterpret_cast<bf16*>(y), n);
  return lrce_check_launch("cast_f16");
}

extern "C" int lrce_cast_f16_bf16(const uint16_t* x, uint16_t* y, int64_t n, void* stream) {
  if (!x || !y) return lrce_fail(LRCE_E_ARG, "cast_f16_bf16: null pointer");
  if ((reinterpret_cast<uintptr_t>(x) | reinterpret_cast<uintptr_t>(y)) & 15)
    return lrce_fail(LRCE_E_ARG, "cast_f16_bf16: buffers must be 16-B aligned");
  if (n <= 0) return LRCE_OK;
  const long long thr = (n + 7) / 8;
  f16_bf16_kernel<<<(thr + 255) / 256, 256, 0, static_cast<hipStream_t>(stream)>>>(reinterpret_cast<const bf16*>(x),
                                                                                  reinterpret_cast<bf16*>(y), n);
  return lrce_check_launch("cast_f16_bf16");
}

extern "C" int lrce_dropout(const float* x, const float* res, float* y, uint16_t* y_bf16, int64_t n, float p, uint64_t seed,
                            int64_t group, void* stream) {
  if (!x || !y) return lrce_fail(LRCE_E_ARG, "dropout: null pointer");
  if (n <= 0) return LRCE_OK;
  if (group < 1) group = 1;
  dropout_kernel<<<(n + 255) / 256, 256, 0, static_cast<hipStream_t>(stream)>>>(x, res, y, reinterpret_cast<bf16*>(y_bf16), n, p,
                                                                               seed, group, lrce_rng_offset());
  return lrce_check_launch("dropout");
}

extern "C" int lrce_dropout_bwd(const float* dy, float* dx, uint16_t* dx_bf16, int64_t n, float p, uint64_t seed, int64_t group,
                                void* stream) {
  if (!dy || (!dx && !dx_bf16)) return lrce_fail(LRCE_E_ARG, "dropout_bwd: null pointer");
  if (n <= 0) return LRCE_OK;
  if (group < 1) group = 1;
  dropout_bwd_kernel<<<(n + 255) / 256, 256, 0, static_cast<hipStream_t>(stream)>>>(
      dy, dx, reinterpret_cast<bf16*>(dx_bf16), n, p, seed, group, lrce_rng_offset());
  return lrce_check_launch("dropout_bwd");
}

extern "C" int lrce_grad_scale(const float* x, int64_t n, float* scale, void* stream) {
  if (!x || !scale) return lrce_fail(LRCE_E_ARG, "grad_scale: null pointer");
  if ((n & 3) || (reinterpret_cast<uintptr_t>(x) & 15)) return lrce_fail(LRCE_E_ARG, "grad_scale: n %% 4 != 0 or x not 16-B aligned");
  const long long n4 = n / 4;
  const unsigned blocks = (unsigned)std::max<long long>(1, std::min<long long>(256, (n4 + 2047) / 2048));
  grad_scale_kernel<<<blocks, 256, 0, static_cast<hipStream_t>(stream)>>>(x, n4, scale);
  return lrce_check_launch("grad_scale");
}

extern "C" int lrce_grad_scale_update(float* scale, int n_slots, void* stream) {
  if (!scale || n_slots < 0) return lrce_fail(LRCE_E_ARG, "grad_scale_update: bad arguments");
  if (n_slots == 0) return LRCE_OK;
  grad_scale_update_kernel<<<(n_slots + 255) / 256, 256, 0, static_cast<hipStream_t>(stream)>>>(scale, n_slots);
  return lrce_check_launch("grad_scale_update");
}

extern "C" int lrce_dropout_bwd_f16(const float* dy, uint16_t* dx_f16, int64_t n, float p, uint64_t seed, int64_t group,
                                    const float* scale, void* stream) {
  if (!dy || !dx_f16 || !scale) return lrce_fail(LRCE_E_ARG, "dropout_bwd_f16: null pointer");
  if ((n & 3) || ((reinterpret_cast<uintptr_t>(dy) | reinterpret_cast<uintptr_t>(dx_f16)) & 7))
    return lrce_fail(LRCE_E_ARG, "dropout_bwd_f16: n %% 4 != 0 or unaligned buffers");
  if (n <= 0) return LRCE_OK;
  if (group < 1) group = 1;
  const long long thr = n / 4;
  dropout_bwd_f16_kernel<<<(unsigned)((thr + 255) / 256), 256, 0, static_cast<hipStream_t>(stream)>>>(
      dy, reinterpret_cast<f16*>(dx_f16), n, p, seed, group, lrce_rng_offset(), scale);
  return lrce_check_launch("dropout_bwd_f16");
}

extern "C" int lrce_bert_embed_fwd(const int64_t* ids, const int64_t* types, const float* word, const float* pos, const float* typ,
                                   float* out, int rows, int L, int C, void* stream) {
  if (!ids || !types || !word || !pos || !typ || !out || C % 4) return lrce_fail(LRCE_E_ARG, "bert_embed_fwd: bad args");
  const long long thr = (long long)rows * C / 4;
  bert_embed_kernel<<<(thr + 255) / 256, 256, 0, static_cast<hipStream_t>(stream)>>>(
      reinterpret_cast<const long long*>(ids), reinterpret_cast<const long long*>(types), word, pos, typ, out, rows, L, C);
  return lrce_check_launch("bert_embed_fwd");
}

extern "C" int lrce_bert_embed_bwd(const float* dout, const int64_t* ids, const int64_t* types, float* dword, float* dpos, float* dtyp,
                                   int rows, int L, int C, int64_t pad_id, void* stream) {
  if (!dout || !ids || !types || !dword || !dpos || !dtyp) return lrce_fail(LRCE_E_ARG, "bert_embed_bwd: null pointer");
  const long long n = (long long)rows * C;
  bert_embed_bwd_kernel<<<(n + 255) / 256, 256, 0, static_cast<hipStream_t>(stream)>>>(
      dout, reinterpret_cast<const long long*>(ids), reinterpret_cast<const long long*>(types), dword, dpos, dtyp, rows, L, C, pad_id);
  return lrce_check_launch("bert_embed_bwd");
}

extern "C" int lrce_video_posembed_fwd(const float* x, const float* cls, const float* pos, const float* len, const float* clip, float* out,
                                       int B, int S, int Tg, int P, int C, void* stream) {
  if (!x || !cls || !pos || !len || !clip || !out || C % 4) return lrce_fail(LRCE_E_ARG, "video_posembed_fwd: bad args");
  const long long thr = (long long)B * S * Tg * (P + 1) * C / 4;
  video_pos_kernel<<<(thr + 255) / 256, 256, 0, static_cast<hipStream_t>(stream)>>>(x, cls, pos, len, clip, out, B, S, Tg, P, C);
  return lrce_check_launch("video_posembed_fwd");
}

extern "C" int lrce_video_posembed_bwd(const float* dout, float* dx, uint16_t* dx_bf16, float* dcls, float* dpos, float* dlen,
                                       float* dclip, int B, int S, int Tg, int P, int C, void* stream) {
  if (!dout || (!dx && !dx_bf16) || !dcls || !dpos || !dlen || !dclip) return lrce_fail(LRCE_E_ARG, "video_posembed_bwd: null pointer");
  if (C % 4 || B < 1 || S < 1 || Tg < 1 || P < 0) return lrce_fail(LRCE_E_ARG, "video_posembed_bwd: bad shape");
  const int threads = std::min(256, (C / 4 + 63) / 64 * 64);
  dim3 grid(S * Tg, (P + 1 + VP_PPB - 1) / VP_PPB);
  video_pos_bwd_kernel<<<grid, threads, 0, static_cast<hipStream_t>(stream)>>>(dout, dx, reinterpret_cast<bf16*>(dx_bf16), dcls, dpos,
                                                                               dlen, dclip, B, S, Tg, P, C);
  return lrce_check_launch("video_posembed_bwd");
}

extern "C" int lrce_text_posembed_fwd(const float* x, const float* cls, const float* pos, float* out, int B, int L, int C, void* stream) {
  if (!x || !cls || !pos || !out || C % 4) return lrce_fail(LRCE_E_ARG, "text_posembed_fwd: bad args");
  const long long thr = (long long)B * (L + 1) * C / 4;
  text_pos_kernel<<<(thr + 255) / 256, 256, 0, static_cast<hipStream_t>(stream)>>>(x, cls, pos, out, B, L, C);
  return lrce_check_launch("text_posembed_fwd");
}

extern "C" int lrce_text_posembed_bwd(const float* dout, float* dx, float* dcls, float* dpos, int B, int L, int C, void* stream) {
  if (!dout || !dx || !dcls || !dpos) return lrce_fail(LRCE_E_ARG, "text_posembed_bwd: null pointer");
  dim3 grid((C + 255) / 256, L + 1);
  text_pos_bwd_kernel<<<grid, 256, 0, static_cast<hipStream_t>(stream)>>>(dout, dx, dcls, dpos, B, L, C);
  return lrce_check_launch("text_posembed_bwd");
}
