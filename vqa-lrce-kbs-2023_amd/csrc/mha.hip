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
// (reads key row t as 8 x 16 B, q broadcast from LDS); block-wide max / sum through LDS.  Output,
// dQ, dK, dV: lane = head dim, the 4 waves split the keys, rows read / written coalesced (128 B).
// dK/dV rows are updated with plain read-modify-writes when this workgroup is their only writer
// (bdiv == 1: the question segment accumulates over the recurrent steps, which are separate
// launches), with atomics when bdiv answer choices share a video memory row.
constexpr int KT = MAXK / 64;

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
  if (t < D) qs[t] = ld_io(d, d.q, (long long)b * d.ld_q + h * D + t) * d.scale;
  __syncthreads();
  const bool live = t < Lk;
  const bool keep = live && (!d.key_mask || d.key_mask[(long long)b * Lk + t] != 0);
  const float sc = live ? dot_row64(key_row(d, d.k1, d.k2, b, t, h), qs) : 0.f;
  const float m = block_max(keep ? sc : -1.0e30f, red);
  const float pe = keep ? __expf(sc - m) : 0.f;
  const float s = block_sum(pe, red);
  ps[t] = live ? pe * drop_factor(d, P.off, b, h, 0, t, Lk) : 0.f;
  __syncthreads();
  // o[lane] = sum_j ps[j] V[j][lane]; wave w takes keys w, w+4, ...
  float o0 = 0.f, o1 = 0.f;
  int j = wave;
  for (; j + 4 < Lk; j += 8) {
    o0 += ps[j] * bf2f(key_row(d, d.v1, d.v2, b, j, h)[lane]);
    o1 += ps[j + 4] * bf2f(key_row(d, d.v1, d.v2, b, j + 4, h)[lane]);
  }
  if (j < Lk) o0 += ps[j] * bf2f(key_row(d, d.v1, d.v2, b, j, h)[lane]);
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

__device__ __forceinline__ void rmw_add(float* p, float v, bool atomic) {
  if (atomic) __hip_atomic_fetch_add(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  else *p += v;
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
  for (int j = wave; j < Lk; j += 4) {
    const float dsj = dss[j], pj = ps[j];
    const bf16* kr = key_row(d, d.k1, d.k2, b, j, h);
    if (j & 4) dq1 += dsj * bf2f(kr[lane]);
    else dq0 += dsj * bf2f(kr[lane]);
    if (j < d.lk1) {
      const long long o = (long long)(b / d.kv1_bdiv) * d.stride_dkv1_b + (long long)j * d.ld_dkv1 + h * D + lane;
      rmw_add(d.dk1 + o, dsj * q, at1);
      rmw_add(d.dv1 + o, pj * g, at1);
    } else {
      const long long o = (long long)(b / d.kv2_bdiv) * d.stride_dkv2_b + (long long)(j - d.lk1) * d.ld_dkv2 + h * D + lane;
      rmw_add(d.dk2 + o, dsj * q, at2);
      rmw_add(d.dv2 + o, pj * g, at2);
    }
  }
  part[wave][lane] = dq0 + dq1;
  __syncthreads();
  if (wave == 0)
    d.dq[(long long)b * d.ld_dq + h * D + lane] =
        ((part[0][lane] + part[1][lane]) + (part[2][lane] + part[3][lane])) * d.scale;
}

// key/value rows readable as 16-B vectors (single-query path)
bool aligned_rows(const LrceMhaDesc* d) {
  auto al = [](const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; };
  bool ok = al(d->k1) && al(d->v1) && d->ld_kv1 % 8 == 0 && d->stride_kv1_b % 8 == 0;
  if (d->lk2 > 0) ok = ok && al(d->k2) && al(d->v2) && d->ld_kv2 % 8 == 0 && d->stride_kv2_b % 8 == 0;
  return ok;
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
  if (d->Lq == 1 && aligned_rows(d)) {
    mha1_fwd_kernel<<<d->B * d->H, 256, 0, static_cast<hipStream_t>(stream)>>>(p);
    return lrce_check_launch("mha_fwd");
  }
  mha_fwd_kernel<<<d->B * d->H, 256, 0, static_cast<hipStream_t>(stream)>>>(p);
  return lrce_check_launch("mha_fwd");
}

extern "C" int lrce_mha_bwd(const LrceMhaDesc* d, void* stream) {
  if (int rc = check(d, true)) return rc;
  MhaP p{*d, lrce_rng_offset()};
  if (d->Lq == 1 && aligned_rows(d)) {
    mha1_bwd_kernel<<<d->B * d->H, 256, 0, static_cast<hipStream_t>(stream)>>>(p);
    return lrce_check_launch("mha_bwd");
  }
  mha_bwd_kernel<<<d->B * d->H, 256, 0, static_cast<hipStream_t>(stream)>>>(p);
  return lrce_check_launch("mha_bwd");
}
