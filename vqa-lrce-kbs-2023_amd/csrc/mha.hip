// Small masked multi-head attention, head_dim 64:
//  * BERT self-attention (L = 30..40 tokens, 12 heads; HF BertSelfAttention via text.py:12-17);
//  * the LRCE decoder cross-attention: one summary-token query against the step's memory
//    [video clip tokens (150) ; question tokens (L+1)] (nn.MultiheadAttention inside
//    nn.TransformerDecoderLayer, fusionv3.py:8-17,44-49).
// The keys come from up to two segments so the memory is never concatenated in HBM: the text
// segment's K/V are projected ONCE and reused by every recurrent step, and the video segment can be
// shared by `bdiv` consecutive batch rows (the 5 answer choices of the MC head, fusionv3.py:259).
// Attention-probability dropout (train mode) is applied in-kernel from a counter hash, identically
// in the backward.  Problems are tiny and latency-bound: one workgroup per (batch row, head), K/V in
// LDS, f32 VALU math; the projections around it run on MFMA in lrce_gemm.
#include "common.h"
#include "lrce_capi.h"

namespace {

constexpr int D = 64;
constexpr int MAXK = 192;

__device__ __forceinline__ void wave_lds_fence_m() {
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  __builtin_amdgcn_wave_barrier();
}

struct MhaP {
  LrceMhaDesc d;
  const uint64_t* off;  // device RNG offset (lrce_set_rng_offset)
};

__device__ __forceinline__ const bf16* key_row(const LrceMhaDesc& d, const uint16_t* p1, const uint16_t* p2, int b, int j, int h) {
  if (j < d.lk1) return reinterpret_cast<const bf16*>(p1) + (long long)(b / d.kv1_bdiv) * d.stride_kv1_b + (long long)j * d.ld_kv1 + h * D;
  return reinterpret_cast<const bf16*>(p2) + (long long)(b / d.kv2_bdiv) * d.stride_kv2_b + (long long)(j - d.lk1) * d.ld_kv2 + h * D;
}

__device__ __forceinline__ float ld_io(const LrceMhaDesc& d, const void* p, long long i) {
  return d.f32_io ? static_cast<const float*>(p)[i] : bf2f(static_cast<const bf16*>(p)[i]);
}

__device__ __forceinline__ float drop_factor(const LrceMhaDesc& d, const uint64_t* off, int b, int h, int i, int j, int Lk) {
  if (d.drop_p <= 0.f) return 1.f;
  const uint64_t idx = (((uint64_t)b * d.H + h) * d.Lq + i) * (uint64_t)Lk + j;
  return lrce_uniform(lrce_seed(d.seed, off), idx) >= d.drop_p ? 1.0f / (1.0f - d.drop_p) : 0.f;
}

__global__ void __launch_bounds__(256) mha_fwd_kernel(MhaP P) {
  const LrceMhaDesc& d = P.d;
  __shared__ float ks[MAXK][D + 1];
  __shared__ float vs[MAXK][D];
  __shared__ float ps[4][MAXK];
  const int b = blockIdx.x / d.H, h = blockIdx.x % d.H;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int Lk = d.lk1 + d.lk2;
  for (int e = threadIdx.x; e < Lk * D; e += 256) {
    const int j = e / D, dd = e % D;
    ks[j][dd] = bf2f(key_row(d, d.k1, d.k2, b, j, h)[dd]);
    vs[j][dd] = bf2f(key_row(d, d.v1, d.v2, b, j, h)[dd]);
  }
  __syncthreads();
  for (int i = wave; i < d.Lq; i += 4) {
    const float qd = ld_io(d, d.q, ((long long)b * d.Lq + i) * d.ld_q + h * D + lane) * d.scale;
    float sc[MAXK / 64];
#pragma unroll
    for (int t = 0; t < MAXK / 64; ++t) sc[t] = 0.f;
    for (int dd = 0; dd < D; ++dd) {
      const float qv = __shfl(qd, dd, 64);
#pragma unroll
      for (int t = 0; t < MAXK / 64; ++t) {
        const int j = lane + 64 * t;
        if (j < Lk) sc[t] += qv * ks[j][dd];
      }
    }
    // masked / padded keys are excluded explicitly (no infinities: hipcc may assume finite math)
    float m = -1.0e30f;
    bool keep[MAXK / 64];
#pragma unroll
    for (int t = 0; t < MAXK / 64; ++t) {
      const int j = lane + 64 * t;
      keep[t] = j < Lk && (!d.key_mask || d.key_mask[(long long)b * Lk + j] != 0);
      if (keep[t]) m = fmaxf(m, sc[t]);
    }
    m = wave_max(m);
    float s = 0.f;
#pragma unroll
    for (int t = 0; t < MAXK / 64; ++t) {
      const int j = lane + 64 * t;
      const float p = keep[t] ? __expf(sc[t] - m) : 0.f;
      if (j < Lk) ps[wave][j] = p * drop_factor(d, P.off, b, h, i, j, Lk);
      s += p;
    }
    s = wave_sum(s);
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
    float o = 0.f;
    for (int j = 0; j < Lk; ++j) o += ps[wave][j] * vs[j][lane];
    const long long oi = ((long long)b * d.Lq + i) * d.ld_o + h * D + lane;
    if (d.f32_io) reinterpret_cast<float*>(d.out)[oi] = o / s;
    else reinterpret_cast<bf16*>(d.out)[oi] = f2bf(o / s);
    if (lane == 0) d.lse[((long long)b * d.H + h) * d.Lq + i] = m + __logf(s);
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
  }
}

__global__ void __launch_bounds__(256) mha_bwd_kernel(MhaP P) {
  const LrceMhaDesc& d = P.d;
  __shared__ bf16 ks[MAXK][D + 2];
  __shared__ bf16 vs[MAXK][D + 2];
  __shared__ float dks[MAXK][D];
  __shared__ float dvs[MAXK][D];
  __shared__ float ps[4][MAXK];
  __shared__ float dss[4][MAXK];
  const int b = blockIdx.x / d.H, h = blockIdx.x % d.H;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int Lk = d.lk1 + d.lk2;
  for (int e = threadIdx.x; e < Lk * D; e += 256) {
    const int j = e / D, dd = e % D;
    ks[j][dd] = key_row(d, d.k1, d.k2, b, j, h)[dd];
    vs[j][dd] = key_row(d, d.v1, d.v2, b, j, h)[dd];
    dks[j][dd] = 0.f;
    dvs[j][dd] = 0.f;
  }
  __syncthreads();
  for (int i = wave; i < d.Lq; i += 4) {
    const long long row = (long long)b * d.Lq + i;
    const float qd = ld_io(d, d.q, row * d.ld_q + h * D + lane);
    const float dod = ld_io(d, d.dout, row * d.ld_o + h * D + lane);
    const float od = ld_io(d, d.out, row * d.ld_o + h * D + lane);
    const float delta = wave_sum(dod * od);
    const float l = d.lse[((long long)b * d.H + h) * d.Lq + i];
    float sc[MAXK / 64], dp[MAXK / 64];
#pragma unroll
    for (int t = 0; t < MAXK / 64; ++t) { sc[t] = 0.f; dp[t] = 0.f; }
    for (int dd = 0; dd < D; ++dd) {
      const float qv = __shfl(qd, dd, 64) * d.scale;
      const float gv = __shfl(dod, dd, 64);
#pragma unroll
      for (int t = 0; t < MAXK / 64; ++t) {
        const int j = lane + 64 * t;
        if (j < Lk) { sc[t] += qv * bf2f(ks[j][dd]); dp[t] += gv * bf2f(vs[j][dd]); }
      }
    }
#pragma unroll
    for (int t = 0; t < MAXK / 64; ++t) {
      const int j = lane + 64 * t;
      if (j < Lk) {
        const bool keep = !d.key_mask || d.key_mask[(long long)b * Lk + j] != 0;
        const float p = keep ? __expf(sc[t] - l) : 0.f;
        const float f = drop_factor(d, P.off, b, h, i, j, Lk);
        ps[wave][j] = p * f;                 // dV uses the dropped probabilities
        dss[wave][j] = p * (f * dp[t] - delta);
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
    float g = 0.f;
    for (int j = 0; j < Lk; ++j) {
      const float ds = dss[wave][j];
      g += ds * bf2f(ks[j][lane]);
      atomicAdd(&dks[j][lane], ds * qd * d.scale);
      atomicAdd(&dvs[j][lane], ps[wave][j] * dod);
    }
    d.dq[row * d.ld_dq + h * D + lane] = g * d.scale;
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
  }
  __syncthreads();
  for (int e = threadIdx.x; e < Lk * D; e += 256) {
    const int j = e / D, dd = e % D;
    if (j < d.lk1) {
      const long long o = (long long)(b / d.kv1_bdiv) * d.stride_dkv1_b + (long long)j * d.ld_dkv1 + h * D + dd;
      atomicAdd(d.dk1 + o, dks[j][dd]);
      atomicAdd(d.dv1 + o, dvs[j][dd]);
    } else {
      const long long o = (long long)(b / d.kv2_bdiv) * d.stride_dkv2_b + (long long)(j - d.lk1) * d.ld_dkv2 + h * D + dd;
      atomicAdd(d.dk2 + o, dks[j][dd]);
      atomicAdd(d.dv2 + o, dvs[j][dd]);
    }
  }
}

// ---- single-query path (the recurrent decoder: Lq = 1, fusionv3.py:44-49) --------------------
// One workgroup (4 waves) per (batch row, head).  Scores / probabilities: thread t owns key t
// (its key row as 8 x 16 B in registers, q broadcast from LDS); block-wide max / sum through LDS.
// Output, dQ, dK, dV: lane = head dim, wave w takes keys w, w+4, ...  The forward issues every
// global load of the problem (key rows, the wave's V columns) before the first dependent
// instruction: one memory round trip plus the LDS reductions.  (The backward keeps 16-key batches:
// holding all 48 keys' K / dK / dV words per lane cost it 2x, 256 VGPRs and AGPR spills.)
// dK/dV rows are updated with plain read-modify-writes when this
// workgroup is their only writer (bdiv == 1: the question segment accumulates over the recurrent
// steps, which are separate launches), with atomics when bdiv answer choices share a video row.
constexpr int KW = MAXK / 4;   // keys per wave

__device__ __forceinline__ float dot_regs64(const bf16x8 (&kr)[8], const float* qs) {
  float acc = 0.f;
#pragma unroll
  for (int c = 0; c < 8; ++c) {
    const float4 q0 = *reinterpret_cast<const float4*>(qs + 8 * c);
    const float4 q1 = *reinterpret_cast<const float4*>(qs + 8 * c + 4);
    acc += bf2f(kr[c][0]) * q0.x + bf2f(kr[c][1]) * q0.y + bf2f(kr[c][2]) * q0.z + bf2f(kr[c][3]) * q0.w +
           bf2f(kr[c][4]) * q1.x + bf2f(kr[c][5]) * q1.y + bf2f(kr[c][6]) * q1.z + bf2f(kr[c][7]) * q1.w;
  }
  return acc;
}

__device__ __forceinline__ float dot_row64(const bf16* row, const float* qs) {
  float acc = 0.f;
#pragma unroll
  for (int c = 0; c < 8; ++c) {
    const bf16x8 kv = *reinterpret_cast<const bf16x8*>(row + 8 * c);
    const float4 q0 = *reinterpret_cast<const float4*>(qs + 8 * c);
    const float4 q1 = *reinterpret_cast<const float4*>(qs + 8 * c + 4);
    acc += bf2f(kv[0]) * q0.x + bf2f(kv[1]) * q0.y + bf2f(kv[2]) * q0.z + bf2f(kv[3]) * q0.w +
           bf2f(kv[4]) * q1.x + bf2f(kv[5]) * q1.y + bf2f(kv[6]) * q1.z + bf2f(kv[7]) * q1.w;
  }
  return acc;
}

__device__ __forceinline__ void load_row64(bf16x8 (&r)[8], const bf16* row) {
#pragma unroll
  for (int c = 0; c < 8; ++c) r[c] = *reinterpret_cast<const bf16x8*>(row + 8 * c);
}

__device__ __forceinline__ float block_max(float v, float* red) {
  v = wave_max(v);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
  __syncthreads();
  const float r = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
  __syncthreads();
  return r;
}
__device__ __forceinline__ float block_sum(float v, float* red) {
  v = wave_sum(v);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
  __syncthreads();
  const float r = (red[0] + red[1]) + (red[2] + red[3]);
  __syncthreads();
  return r;
}

__global__ void __launch_bounds__(256) mha1_fwd_kernel(MhaP P) {
  const LrceMhaDesc& d = P.d;
  __shared__ __attribute__((aligned(16))) float qs[D];
  __shared__ float ps[MAXK + 64];
  __shared__ float part[4][D];
  __shared__ float red[4];
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int b = blockIdx.x / d.H, h = blockIdx.x % d.H;
  const int Lk = d.lk1 + d.lk2;
  const bool live = t < Lk;
  bf16x8 kr[8];
  load_row64(kr, key_row(d, d.k1, d.k2, b, live ? t : 0, h));
  float vv[KW];
#pragma unroll
  for (int u = 0; u < KW; ++u) vv[u] = bf2f(key_row(d, d.v1, d.v2, b, min(wave + 4 * u, Lk - 1), h)[lane]);
  const bool keep = live && (!d.key_mask || d.key_mask[(long long)b * Lk + t] != 0);
  if (t < D) qs[t] = ld_io(d, d.q, (long long)b * d.ld_q + h * D + t) * d.scale;
  __syncthreads();
  const float sc = live ? dot_regs64(kr, qs) : 0.f;
  const float m = block_max(keep ? sc : -1.0e30f, red);
  const float pe = keep ? __expf(sc - m) : 0.f;
  const float s = block_sum(pe, red);
  ps[t] = live ? pe * drop_factor(d, P.off, b, h, 0, t, Lk) : 0.f;   // ps[j >= Lk] = 0
  __syncthreads();
  float o0 = 0.f, o1 = 0.f;
#pragma unroll
  for (int u = 0; u < KW; u += 2) {
    o0 += ps[wave + 4 * u] * vv[u];
    o1 += ps[wave + 4 * u + 4] * vv[u + 1];
  }
  part[wave][lane] = o0 + o1;
  __syncthreads();
  if (wave == 0) {
    const float o = (part[0][lane] + part[1][lane]) + (part[2][lane] + part[3][lane]);
    const long long oi = (long long)b * d.ld_o + h * D + lane;
    if (d.f32_io) reinterpret_cast<float*>(d.out)[oi] = o / s;
    else reinterpret_cast<bf16*>(d.out)[oi] = f2bf(o / s);
    if (lane == 0) d.lse[(long long)b * d.H + h] = m + __logf(s);
  }
}

__global__ void __launch_bounds__(256) mha1_bwd_kernel(MhaP P) {
  const LrceMhaDesc& d = P.d;
  __shared__ __attribute__((aligned(16))) float qs[D];
  __shared__ __attribute__((aligned(16))) float gs[D];
  __shared__ float ps[MAXK + 64];
  __shared__ float dss[MAXK + 64];
  __shared__ float part[4][D];
  __shared__ float red[4];
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int b = blockIdx.x / d.H, h = blockIdx.x % d.H;
  const int Lk = d.lk1 + d.lk2;
  float dod = 0.f, od = 0.f;
  if (t < D) {
    qs[t] = ld_io(d, d.q, (long long)b * d.ld_q + h * D + t) * d.scale;
    dod = ld_io(d, d.dout, (long long)b * d.ld_o + h * D + t);
    od = ld_io(d, d.out, (long long)b * d.ld_o + h * D + t);
    gs[t] = dod;
  }
  const float delta = block_sum(dod * od, red);   // also orders the qs / gs writes
  const float l = d.lse[(long long)b * d.H + h];
  const bool live = t < Lk;
  float pf = 0.f, ds = 0.f;
  if (live) {
    const float sc = dot_row64(key_row(d, d.k1, d.k2, b, t, h), qs);
    const float dp = dot_row64(key_row(d, d.v1, d.v2, b, t, h), gs);
    const bool keep = !d.key_mask || d.key_mask[(long long)b * Lk + t] != 0;
    const float p = keep ? __expf(sc - l) : 0.f;
    const float f = drop_factor(d, P.off, b, h, 0, t, Lk);
    pf = p * f;                       // dV uses the dropped probabilities
    ds = p * (f * dp - delta);
  }
  ps[t] = pf;
  dss[t] = ds;
  __syncthreads();
  const float q = qs[lane], g = gs[lane];
  float dq0 = 0.f, dq1 = 0.f;
  const bool at1 = d.kv1_bdiv > 1, at2 = d.kv2_bdiv > 1;
  // Keys in batches of UB per wave: every K-row load and dK/dV read of a batch is issued before its
  // first store, so the read-modify-writes overlap instead of forming one serial memory round trip
  // per key (single writer per row); rows shared by bdiv > 1 rows use no-return atomics.
  constexpr int UB = 16;
  for (int j0 = wave; j0 < Lk; j0 += 4 * UB) {
    float kv[UB], okk[UB], ovv[UB];
    float* pk[UB];
    float* pv[UB];
    bool at[UB];
#pragma unroll
    for (int u = 0; u < UB; ++u) {
      const int j = min(j0 + 4 * u, Lk - 1);
      kv[u] = bf2f(key_row(d, d.k1, d.k2, b, j, h)[lane]);
      if (j < d.lk1) {
        const long long o = (long long)(b / d.kv1_bdiv) * d.stride_dkv1_b + (long long)j * d.ld_dkv1 + h * D + lane;
        pk[u] = d.dk1 + o; pv[u] = d.dv1 + o; at[u] = at1;
      } else {
        const long long o = (long long)(b / d.kv2_bdiv) * d.stride_dkv2_b + (long long)(j - d.lk1) * d.ld_dkv2 + h * D + lane;
        pk[u] = d.dk2 + o; pv[u] = d.dv2 + o; at[u] = at2;
      }
      const bool fresh = d.dkv1_store && j < d.lk1;   // stored, not accumulated
      okk[u] = (at[u] || fresh) ? 0.f : *pk[u];
      ovv[u] = (at[u] || fresh) ? 0.f : *pv[u];
    }
#pragma unroll
    for (int u = 0; u < UB; ++u) {
      const int j = j0 + 4 * u;
      if (j < Lk) {
        const float dsj = dss[j], pj = ps[j];
        if (u & 1) dq1 += dsj * kv[u];
        else dq0 += dsj * kv[u];
        if (at[u]) {
          __hip_atomic_fetch_add(pk[u], dsj * q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          __hip_atomic_fetch_add(pv[u], pj * g, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        } else {
          *pk[u] = okk[u] + dsj * q;
          *pv[u] = ovv[u] + pj * g;
        }
      }
    }
  }
  part[wave][lane] = dq0 + dq1;
  __syncthreads();
  if (wave == 0)
    d.dq[(long long)b * d.ld_dq + h * D + lane] =
        ((part[0][lane] + part[1][lane]) + (part[2][lane] + part[3][lane])) * d.scale;
}

// ---- short self-attention on MFMA (BERT: Lq = Lk = L <= 64, one key segment) ---------------------
// One wave per (batch row, head); L padded to NTL x 32.  v_mfma_f32_32x32x16_bf16 throughout, the
// layout recipe of window_attn.hip: the forward computes S^T = K Q^T so a lane owns one query
// column (in-lane softmax + one cross-half exchange) and the probabilities feed O^T = V^T P^T from
// registers; the backward recomputes S = Q K^T per 32x32 tile, dV = P^T dO and dK = dS^T Q from
// registers, dQ = dS K through a 2 KB LDS transpose of dS.  Scores are scaled in f32 (HF order:
// (q.k) * d^-1/2, then the key mask, softmax, dropout on the probabilities).
constexpr float LOG2E_F = 1.4426950408889634f;

__device__ __forceinline__ int crow32(int reg, int h) { return (reg & 3) + 8 * (reg >> 2) + 4 * h; }

// transposed reads of a [rows][64] bf16 LDS image, columns col0 .. col0 + 31 (see window_attn.hip)
__device__ __forceinline__ bf16x8 tr_perm64(const bf16* img, int r_base, int col0, int lane) {
  const int g = lane >> 4, i = lane & 15, q = i >> 2, p = i & 3;
  const int hh = g >> 1, cb = col0 + 16 * (g & 1);
  bf16x8 out;
#pragma unroll
  for (int h2 = 0; h2 < 2; ++h2) {
    const int row = r_base + 8 * h2 + 4 * hh + q;
    const LRCE_LDS s16x4* src = (const LRCE_LDS s16x4*)(img + row * D + cb + 4 * p);
    s16x4 v = __builtin_amdgcn_ds_read_tr16_b64_v4i16(const_cast<LRCE_LDS s16x4*>(src));
    bf16x4 b = *reinterpret_cast<bf16x4*>(&v);
    out[4 * h2 + 0] = b[0]; out[4 * h2 + 1] = b[1]; out[4 * h2 + 2] = b[2]; out[4 * h2 + 3] = b[3];
  }
  return out;
}
template <int STRIDE>
__device__ __forceinline__ bf16x8 tr_nat(const bf16* img, int r_base, int col0, int lane) {
  const int g = lane >> 4, i = lane & 15, q = i >> 2, p = i & 3;
  const int hh = g >> 1, cb = col0 + 16 * (g & 1);
  bf16x8 out;
#pragma unroll
  for (int h2 = 0; h2 < 2; ++h2) {
    const int row = r_base + 8 * hh + 4 * h2 + q;
    const LRCE_LDS s16x4* src = (const LRCE_LDS s16x4*)(img + row * STRIDE + cb + 4 * p);
    s16x4 v = __builtin_amdgcn_ds_read_tr16_b64_v4i16(const_cast<LRCE_LDS s16x4*>(src));
    bf16x4 b = *reinterpret_cast<bf16x4*>(&v);
    out[4 * h2 + 0] = b[0]; out[4 * h2 + 1] = b[1]; out[4 * h2 + 2] = b[2]; out[4 * h2 + 3] = b[3];
  }
  return out;
}
__device__ __forceinline__ bf16x8 pack8f(const f32x16& a, int s) {
  bf16x8 o;
#pragma unroll
  for (int j = 0; j < 8; ++j) o[j] = f2bf(a[8 * s + j]);
  return o;
}
template <bool F16>
__device__ __forceinline__ bf16x8 pack8t(const f32x16& a, int s) {
  bf16x8 o;
#pragma unroll
  for (int j = 0; j < 8; ++j) o[j] = to16<F16>(a[8 * s + j]);
  return o;
}
__device__ __forceinline__ bf16x8 ldrow16(const bf16* p) { return *reinterpret_cast<const bf16x8*>(p); }

// rows [0, LP) x 64 of a head slice into an LDS image (rows >= n zero)
template <int LP>
__device__ __forceinline__ void stage64(bf16* img, const bf16* src, long long ld, int n, int lane) {
#pragma unroll
  for (int t = 0; t < LP / 8; ++t) {
    const int c = lane + 64 * t;
    const int row = c >> 3, part = c & 7;
    uint4 v = make_uint4(0, 0, 0, 0);
    if (row < n) v = *reinterpret_cast<const uint4*>(src + row * ld + part * 8);
    *reinterpret_cast<uint4*>(img + row * D + part * 8) = v;
  }
}

template <int NTL, bool F16>
__global__ void __launch_bounds__(256) mhaL_fwd_kernel(MhaP P) {
  constexpr int LP = 32 * NTL;
  const LrceMhaDesc& d = P.d;
  __shared__ __attribute__((aligned(16))) bf16 vimg_all[4][LP * D];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int bh = blockIdx.x * 4 + wave;
  if (bh >= d.B * d.H) return;
  const int b = bh / d.H, h = bh % d.H;
  const int L = d.lk1;
  const bf16* qb = reinterpret_cast<const bf16*>(d.q) + (long long)b * L * d.ld_q + h * D;
  const bf16* kb = reinterpret_cast<const bf16*>(d.k1) + (long long)b * d.stride_kv1_b + h * D;
  const bf16* vb = reinterpret_cast<const bf16*>(d.v1) + (long long)b * d.stride_kv1_b + h * D;
  bf16* vimg = vimg_all[wave];
  stage64<LP>(vimg, vb, d.ld_kv1, L, lane);
  const int hh = lane >> 5, r32 = lane & 31;
  bf16x8 kf[NTL][4];
#pragma unroll
  for (int kt = 0; kt < NTL; ++kt) {
    const int key = kt * 32 + r32;
#pragma unroll
    for (int s = 0; s < 4; ++s) kf[kt][s] = key < L ? ldrow16(kb + key * d.ld_kv1 + 16 * s + 8 * hh) : bf16x8{};
  }
  const int* km = d.key_mask ? d.key_mask + (long long)b * L : nullptr;
  bool kok[NTL][16];
#pragma unroll
  for (int kt = 0; kt < NTL; ++kt)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int key = kt * 32 + crow32(r, hh);
      kok[kt][r] = key < L && (!km || km[key] != 0);
    }
  wave_lds_fence_m();
  const float c2 = d.scale * LOG2E_F;
#pragma unroll
  for (int qt = 0; qt < NTL; ++qt) {
    const int qi = qt * 32 + r32;
    bf16x8 qf[4];
#pragma unroll
    for (int s = 0; s < 4; ++s) qf[s] = qi < L ? ldrow16(qb + qi * d.ld_q + 16 * s + 8 * hh) : bf16x8{};
    f32x16 acc[NTL];
#pragma unroll
    for (int kt = 0; kt < NTL; ++kt) {
      acc[kt] = f32x16{};
#pragma unroll
      for (int s = 0; s < 4; ++s) acc[kt] = mfma32x32x16<F16>(kf[kt][s], qf[s], acc[kt]);
    }
    float m = -1.0e30f;
#pragma unroll
    for (int kt = 0; kt < NTL; ++kt)
#pragma unroll
      for (int r = 0; r < 16; ++r) m = kok[kt][r] ? fmaxf(m, acc[kt][r]) : m;
    m = fmaxf(m, __shfl_xor(m, 32, 64));
    float sum = 0.f;
#pragma unroll
    for (int kt = 0; kt < NTL; ++kt)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        float p = kok[kt][r] ? __builtin_amdgcn_exp2f((acc[kt][r] - m) * c2) : 0.f;
        sum += p;
        if (d.drop_p > 0.f) p *= drop_factor(d, P.off, b, h, qi, kt * 32 + crow32(r, hh), L);
        acc[kt][r] = p;
      }
    sum += __shfl_xor(sum, 32, 64);
    f32x16 o[2] = {f32x16{}, f32x16{}};
#pragma unroll
    for (int kt = 0; kt < NTL; ++kt)
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        const bf16x8 pb = pack8t<F16>(acc[kt], s);
#pragma unroll
        for (int dt = 0; dt < 2; ++dt) o[dt] = mfma32x32x16<F16>(tr_perm64(vimg, kt * 32 + 16 * s, 32 * dt, lane), pb, o[dt]);
      }
    if (qi < L) {
      const float inv = 1.0f / sum;
      bf16* dst = reinterpret_cast<bf16*>(d.out) + ((long long)b * L + qi) * d.ld_o + h * D + 4 * hh;
#pragma unroll
      for (int dt = 0; dt < 2; ++dt)
#pragma unroll
        for (int rr = 0; rr < 4; ++rr) {
          bf16x4 v;
#pragma unroll
          for (int e = 0; e < 4; ++e) v[e] = to16<F16>(o[dt][4 * rr + e] * inv);
          *reinterpret_cast<bf16x4*>(dst + 32 * dt + 8 * rr) = v;
        }
      if (hh == 0) d.lse[((long long)b * d.H + h) * L + qi] = m * d.scale + __logf(sum);
    }
  }
}

template <int LP>
struct MhaLBwdLds {
  bf16 q[LP * D];
  bf16 k[LP * D];
  bf16 dout[LP * D];
  bf16 t[32 * 32];
  float lse2[LP];
  float delta[LP];
};

template <int NTL, bool F16>
__global__ void __launch_bounds__(128) mhaL_bwd_kernel(MhaP P) {
  constexpr int LP = 32 * NTL;
  const LrceMhaDesc& d = P.d;
  __shared__ __attribute__((aligned(16))) MhaLBwdLds<LP> S_all[2];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int bh = blockIdx.x * 2 + wave;
  if (bh >= d.B * d.H) return;
  MhaLBwdLds<LP>& S = S_all[wave];
  const int b = bh / d.H, h = bh % d.H;
  const int L = d.lk1;
  const bf16* qb = reinterpret_cast<const bf16*>(d.q) + (long long)b * L * d.ld_q + h * D;
  const bf16* kb = reinterpret_cast<const bf16*>(d.k1) + (long long)b * d.stride_kv1_b + h * D;
  const bf16* vb = reinterpret_cast<const bf16*>(d.v1) + (long long)b * d.stride_kv1_b + h * D;
  const bf16* ob = reinterpret_cast<const bf16*>(d.out) + (long long)b * L * d.ld_o + h * D;
  const bf16* gb = reinterpret_cast<const bf16*>(d.dout) + (long long)b * L * d.ld_o + h * D;
  stage64<LP>(S.q, qb, d.ld_q, L, lane);
  stage64<LP>(S.k, kb, d.ld_kv1, L, lane);
  stage64<LP>(S.dout, gb, d.ld_o, L, lane);
  (void)ob;
  wave_lds_fence_m();
  const int hh = lane >> 5, r32 = lane & 31;
  const int* km = d.key_mask ? d.key_mask + (long long)b * L : nullptr;
  const float c2 = d.scale * LOG2E_F;
  // Pass 1: this kernel's own softmax statistics.  Its lse and O need not match the scores
  // recomputed here (a bf16 backward of the fp16 forward; or the forward's dropout-free rounding), and a normalisation that does not sum
  // to one over the recomputed scores (or delta = dO.O from another P) leaves sum_j dS_ij != 0,
  // which swamps the small true dS of near-uniform attention rows.  So: per query row, max and sum
  // of the recomputed scores (whole row: L <= 64 keys) and delta_i = sum_j P_ij f_ij dP_ij from the
  // same P and dP — the row sums of dS are then zero up to f32 rounding.  Scores / dP transposed
  // (key rows, query on the lane) so the row reductions stay in registers + one cross-half swap.
#pragma unroll
  for (int qt = 0; qt < NTL; ++qt) {
    const int qi = qt * 32 + r32;
    f32x16 st[NTL], dpt[NTL];
#pragma unroll
    for (int kt = 0; kt < NTL; ++kt) {
      st[kt] = dpt[kt] = f32x16{};
      const int key = kt * 32 + r32;
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        const bf16x8 qa = *reinterpret_cast<const bf16x8*>(S.q + qi * D + 16 * s + 8 * hh);
        const bf16x8 ga = *reinterpret_cast<const bf16x8*>(S.dout + qi * D + 16 * s + 8 * hh);
        const bf16x8 kk = *reinterpret_cast<const bf16x8*>(S.k + key * D + 16 * s + 8 * hh);
        const bf16x8 vv = key < L ? ldrow16(vb + key * d.ld_kv1 + 16 * s + 8 * hh) : bf16x8{};
        st[kt] = mfma32x32x16<F16>(kk, qa, st[kt]);
        dpt[kt] = mfma32x32x16<F16>(vv, ga, dpt[kt]);
      }
    }
    float m = -1.0e30f;
#pragma unroll
    for (int kt = 0; kt < NTL; ++kt)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int key = kt * 32 + crow32(r, hh);
        if (key < L && (!km || km[key] != 0)) m = fmaxf(m, st[kt][r]);
      }
    m = fmaxf(m, __shfl_xor(m, 32, 64));
    float sum = 0.f, dl = 0.f;
#pragma unroll
    for (int kt = 0; kt < NTL; ++kt)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int key = kt * 32 + crow32(r, hh);
        if (key < L && (!km || km[key] != 0)) {
          const float p = __builtin_amdgcn_exp2f((st[kt][r] - m) * c2);
          const float f = d.drop_p > 0.f ? drop_factor(d, P.off, b, h, qi, key, L) : 1.f;
          sum += p;
          dl += p * f * dpt[kt][r];
        }
      }
    sum += __shfl_xor(sum, 32, 64);
    dl += __shfl_xor(dl, 32, 64);
    if (hh == 0) {
      S.lse2[qi] = sum > 0.f ? m * c2 + __log2f(sum) : 0.f;
      S.delta[qi] = sum > 0.f ? dl / sum : 0.f;
    }
  }
  wave_lds_fence_m();
  f32x16 dq[NTL][2];
#pragma unroll
  for (int qt = 0; qt < NTL; ++qt) dq[qt][0] = dq[qt][1] = f32x16{};
#pragma unroll
  for (int kt = 0; kt < NTL; ++kt) {
    const int key = kt * 32 + r32;
    const bool kok = key < L && (!km || km[key] != 0);
    bf16x8 kf[4], vf[4];
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      kf[s] = key < L ? ldrow16(kb + key * d.ld_kv1 + 16 * s + 8 * hh) : bf16x8{};
      vf[s] = key < L ? ldrow16(vb + key * d.ld_kv1 + 16 * s + 8 * hh) : bf16x8{};
    }
    f32x16 dv[2] = {f32x16{}, f32x16{}}, dk[2] = {f32x16{}, f32x16{}};
#pragma unroll
    for (int qt = 0; qt < NTL; ++qt) {
      f32x16 sacc = f32x16{}, dp = f32x16{};
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        const bf16x8 qa = *reinterpret_cast<const bf16x8*>(S.q + (qt * 32 + r32) * D + 16 * s + 8 * hh);
        const bf16x8 ga = *reinterpret_cast<const bf16x8*>(S.dout + (qt * 32 + r32) * D + 16 * s + 8 * hh);
        sacc = mfma32x32x16<F16>(qa, kf[s], sacc);
        dp = mfma32x32x16<F16>(ga, vf[s], dp);
      }
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int qi = qt * 32 + crow32(r, hh);
        const float p = (kok && qi < L) ? __builtin_amdgcn_exp2f(sacc[r] * c2 - S.lse2[qi]) : 0.f;
        const float f = d.drop_p > 0.f ? drop_factor(d, P.off, b, h, qi, key, L) : 1.f;
        sacc[r] = p * f;                        // dV uses the dropped probabilities
        dp[r] = p * (f * dp[r] - S.delta[qi]);  // dS (w.r.t. the scaled scores)
      }
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        const bf16x8 pa = pack8t<F16>(sacc, s), da = pack8t<F16>(dp, s);
#pragma unroll
        for (int dt = 0; dt < 2; ++dt) {
          dv[dt] = mfma32x32x16<F16>(pa, tr_perm64(S.dout, qt * 32 + 16 * s, 32 * dt, lane), dv[dt]);
          dk[dt] = mfma32x32x16<F16>(da, tr_perm64(S.q, qt * 32 + 16 * s, 32 * dt, lane), dk[dt]);
        }
      }
      // dS^T -> LDS T[key][query], then dQ[qt] += dS K
#pragma unroll
      for (int rr = 0; rr < 4; ++rr) {
        bf16x4 v;
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] = to16<F16>(dp[4 * rr + e]);
        *reinterpret_cast<bf16x4*>(S.t + r32 * 32 + 8 * rr + 4 * hh) = v;
      }
      wave_lds_fence_m();
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        const bf16x8 a = tr_nat<32>(S.t, 16 * s, 0, lane);
#pragma unroll
        for (int dt = 0; dt < 2; ++dt)
          dq[qt][dt] = mfma32x32x16<F16>(a, tr_nat<D>(S.k, kt * 32 + 16 * s, 32 * dt, lane), dq[qt][dt]);
      }
      wave_lds_fence_m();
    }
    // dK, dV rows of this key tile (this wave is their only writer): rows crow, column d = r32
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int kk = kt * 32 + crow32(r, hh);
      if (kk < L) {
        const long long o = (long long)b * d.stride_dkv1_b + (long long)kk * d.ld_dkv1 + h * D + r32;
#pragma unroll
        for (int dt = 0; dt < 2; ++dt) {
          if (d.grad16) {   // (host: grad16 implies dkv1_store)
            reinterpret_cast<f16*>(d.dk1)[o + 32 * dt] = f2h(dk[dt][r] * d.scale);
            reinterpret_cast<f16*>(d.dv1)[o + 32 * dt] = f2h(dv[dt][r]);
          } else if (d.dkv1_store) {
            d.dk1[o + 32 * dt] = dk[dt][r] * d.scale;
            d.dv1[o + 32 * dt] = dv[dt][r];
          } else {
            d.dk1[o + 32 * dt] += dk[dt][r] * d.scale;
            d.dv1[o + 32 * dt] += dv[dt][r];
          }
        }
      }
    }
  }
#pragma unroll
  for (int qt = 0; qt < NTL; ++qt)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int qi = qt * 32 + crow32(r, hh);
      if (qi < L) {
        const long long o = ((long long)b * L + qi) * d.ld_dq + h * D + r32;
        if (d.grad16) {
          f16* dst = reinterpret_cast<f16*>(d.dq) + o;
          dst[0] = f2h(dq[qt][0][r] * d.scale);
          dst[32] = f2h(dq[qt][1][r] * d.scale);
        } else {
          float* dst = d.dq + o;
          dst[0] = dq[qt][0][r] * d.scale;
          dst[32] = dq[qt][1][r] * d.scale;
        }
      }
    }
}

// key/value rows readable as 16-B vectors (single-query path)
bool aligned_rows(const LrceMhaDesc* d) {
  auto al = [](const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; };
  bool ok = al(d->k1) && al(d->v1) && d->ld_kv1 % 8 == 0 && d->stride_kv1_b % 8 == 0;
  if (d->lk2 > 0) ok = ok && al(d->k2) && al(d->v2) && d->ld_kv2 % 8 == 0 && d->stride_kv2_b % 8 == 0;
  return ok;
}

// BERT-shaped self-attention: one key segment, Lq = Lk <= 64, bf16 io, 16-B aligned rows
bool short_self(const LrceMhaDesc* d) {
  auto al = [](const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; };
  return d->lk2 == 0 && d->Lq == d->lk1 && d->Lq <= 64 && d->kv1_bdiv == 1 && !d->f32_io && aligned_rows(d) &&
         al(d->q) && d->ld_q % 8 == 0 && al(d->out) && d->ld_o % 8 == 0 && (!d->dout || al(d->dout)) &&
         d->stride_kv1_b == (long long)d->lk1 * d->ld_kv1;
}

int check(const LrceMhaDesc* d, bool bwd) {
  if (!d || !d->q || !d->k1 || !d->v1 || !d->out || !d->lse) return lrce_fail(LRCE_E_ARG, "mha: null pointer");
  if (d->d != D) return lrce_fail(LRCE_E_ARG, "mha: head dim %d unsupported (64)", d->d);
  if (d->lk2 > 0 && (!d->k2 || !d->v2)) return lrce_fail(LRCE_E_ARG, "mha: second key segment missing");
  const int Lk = d->lk1 + d->lk2;
  if (d->lk1 < 1 || Lk > MAXK || d->Lq < 1 || d->B < 1 || d->H < 1) return lrce_fail(LRCE_E_ARG, "mha: Lk=%d unsupported", Lk);
  if (d->kv1_bdiv < 1 || (d->lk2 > 0 && d->kv2_bdiv < 1)) return lrce_fail(LRCE_E_ARG, "mha: bdiv < 1");
  if (bwd && (!d->dout || !d->dq || !d->dk1 || !d->dv1 || (d->lk2 > 0 && (!d->dk2 || !d->dv2))))
    return lrce_fail(LRCE_E_ARG, "mha_bwd: null gradient pointer");
  return LRCE_OK;
}

}  // namespace

extern "C" int lrce_mha_fwd(const LrceMhaDesc* d, void* stream) {
  if (int rc = check(d, false)) return rc;
  MhaP p{*d, lrce_rng_offset()};
  if (short_self(d)) {
    const unsigned nb = (d->B * d->H + 3) / 4;
    hipStream_t st = static_cast<hipStream_t>(stream);
    if (d->f16) {
      if (d->Lq <= 32) mhaL_fwd_kernel<1, true><<<nb, 256, 0, st>>>(p);
      else mhaL_fwd_kernel<2, true><<<nb, 256, 0, st>>>(p);
    } else {
      if (d->Lq <= 32) mhaL_fwd_kernel<1, false><<<nb, 256, 0, st>>>(p);
      else mhaL_fwd_kernel<2, false><<<nb, 256, 0, st>>>(p);
    }
    return lrce_check_launch("mha_fwd(mfma)");
  }
  if (d->f16) return lrce_fail(LRCE_E_ARG, "mha_fwd: f16 io only on the short self-attention path (Lq = Lk <= 64)");
  if (d->Lq == 1 && aligned_rows(d)) {
    mha1_fwd_kernel<<<d->B * d->H, 256, 0, static_cast<hipStream_t>(stream)>>>(p);
    return lrce_check_launch("mha_fwd");
  }
  mha_fwd_kernel<<<d->B * d->H, 256, 0, static_cast<hipStream_t>(stream)>>>(p);
  return lrce_check_launch("mha_fwd");
}

extern "C" int lrce_mha_bwd(const LrceMhaDesc* d, void* stream) {
  if (int rc = check(d, true)) return rc;
  if (d->f16 && !short_self(d)) return lrce_fail(LRCE_E_ARG, "mha_bwd: f16 io only on the short self-attention path (Lq = Lk <= 64)");
  if (d->grad16 && (!short_self(d) || !d->dkv1_store))
    return lrce_fail(LRCE_E_ARG, "mha_bwd: fp16 gradients need the short self-attention path with dkv1_store");
  if (d->dkv1_store && !short_self(d) && (d->Lq != 1 || d->kv1_bdiv != 1 || !aligned_rows(d)))
    return lrce_fail(LRCE_E_ARG, "mha_bwd: dkv1_store needs the short self-attention path or the single-query path with kv1_bdiv == 1");
  MhaP p{*d, lrce_rng_offset()};
  if (short_self(d)) {
    const unsigned nb = (d->B * d->H + 1) / 2;
    hipStream_t st = static_cast<hipStream_t>(stream);
    if (d->f16) {
      if (d->Lq <= 32) mhaL_bwd_kernel<1, true><<<nb, 128, 0, st>>>(p);
      else mhaL_bwd_kernel<2, true><<<nb, 128, 0, st>>>(p);
    } else {
      if (d->Lq <= 32) mhaL_bwd_kernel<1, false><<<nb, 128, 0, st>>>(p);
      else mhaL_bwd_kernel<2, false><<<nb, 128, 0, st>>>(p);
    }
    return lrce_check_launch("mha_bwd(mfma)");
  }
  if (d->Lq == 1 && aligned_rows(d)) {
    mha1_bwd_kernel<<<d->B * d->H, 256, 0, static_cast<hipStream_t>(stream)>>>(p);
    return lrce_check_launch("mha_bwd");
  }
  mha_bwd_kernel<<<d->B * d->H, 256, 0, static_cast<hipStream_t>(stream)>>>(p);
  return lrce_check_launch("mha_bwd");
}
