// Small masked multi-head attention, head_dim 64: BERT self-attention (L = 30..40, 12 heads;
// HF BertSelfAttention as called from text.py:12-17) and the LRCE decoder cross-attention
// (one summary-token query against 183/191 memory keys; nn.MultiheadAttention inside
// nn.TransformerDecoderLayer, fusionv3.py:8-17,44-49).  These problems are tiny (<= 192 keys,
// <= 64 queries per (batch, head)) and latency-bound, so one workgroup owns a (batch, head),
// keeps K/V in LDS and computes in f32 on the VALU: the GEMM-shaped projections around it run
// on MFMA in lrce_gemm.
#include "common.h"
#include "lrce_capi.h"

namespace {

constexpr int D = 64;
constexpr int MAXK = 192;

__global__ void __launch_bounds__(256) mha_fwd_kernel(const bf16* __restrict__ q, long long ldq, const bf16* __restrict__ k,
                                                      const bf16* __restrict__ v, long long ldkv, long long skv,
                                                      const int* __restrict__ kmask, bf16* __restrict__ out, long long ldo,
                                                      float* __restrict__ lse, int B, int H, int Lq, int Lk, float scale) {
  __shared__ float ks[MAXK][D + 1];
  __shared__ float vs[MAXK][D];
  __shared__ float ps[4][MAXK];
  const int b = blockIdx.x / H, h = blockIdx.x % H;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const bf16* kb = k + b * skv + h * D;
  const bf16* vb = v + b * skv + h * D;
  for (int e = threadIdx.x; e < Lk * D; e += 256) {
    const int j = e / D, dd = e % D;
    ks[j][dd] = bf2f(kb[j * ldkv + dd]);
    vs[j][dd] = bf2f(vb[j * ldkv + dd]);
  }
  __syncthreads();
  for (int i = wave; i < Lq; i += 4) {
    const bf16* qr = q + ((long long)b * Lq + i) * ldq + h * D;
    const float qd = bf2f(qr[lane]) * scale;
    // scores: each lane accumulates q . k_j for keys j = lane + 64t; q broadcast through shuffles
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
    // masked / padded keys: excluded explicitly (no infinities: -1e30 sentinel, keep flags)
    float m = -1.0e30f;
    bool keep[MAXK / 64];
#pragma unroll
    for (int t = 0; t < MAXK / 64; ++t) {
      const int j = lane + 64 * t;
      keep[t] = j < Lk && (!kmask || kmask[(long long)b * Lk + j] != 0);
      if (keep[t]) m = fmaxf(m, sc[t]);
    }
    m = wave_max(m);
    float s = 0.f;
#pragma unroll
    for (int t = 0; t < MAXK / 64; ++t) {
      const int j = lane + 64 * t;
      const float p = keep[t] ? __expf(sc[t] - m) : 0.f;
      if (j < Lk) ps[wave][j] = p;
      s += p;
    }
    s = wave_sum(s);
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
    float o = 0.f;
    for (int j = 0; j < Lk; ++j) o += ps[wave][j] * vs[j][lane];
    out[((long long)b * Lq + i) * ldo + h * D + lane] = f2bf(o / s);
    if (lane == 0) lse[((long long)b * H + h) * Lq + i] = m + __logf(s);
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
  }
}

__global__ void __launch_bounds__(256) mha_bwd_kernel(const bf16* __restrict__ q, long long ldq, const bf16* __restrict__ k,
                                                      const bf16* __restrict__ v, long long ldkv, long long skv,
                                                      const int* __restrict__ kmask, const bf16* __restrict__ outp, long long ldo,
                                                      const bf16* __restrict__ dout, const float* __restrict__ lse,
                                                      float* __restrict__ dq, long long lddq, float* __restrict__ dk,
                                                      float* __restrict__ dv, long long lddkv, long long sdkv, int B, int H, int Lq,
                                                      int Lk, float scale) {
  __shared__ bf16 ks[MAXK][D + 2];
  __shared__ bf16 vs[MAXK][D + 2];
  __shared__ float dks[MAXK][D];
  __shared__ float dvs[MAXK][D];
  __shared__ float ps[4][MAXK];
  __shared__ float dss[4][MAXK];
  const int b = blockIdx.x / H, h = blockIdx.x % H;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const bf16* kb = k + b * skv + h * D;
  const bf16* vb = v + b * skv + h * D;
  for (int e = threadIdx.x; e < Lk * D; e += 256) {
    const int j = e / D, dd = e % D;
    ks[j][dd] = kb[j * ldkv + dd];
    vs[j][dd] = vb[j * ldkv + dd];
    dks[j][dd] = 0.f;
    dvs[j][dd] = 0.f;
  }
  __syncthreads();
  for (int i = wave; i < Lq; i += 4) {
    const long long row = (long long)b * Lq + i;
    const float qd = bf2f(q[row * ldq + h * D + lane]);
    const float dod = bf2f(dout[row * ldo + h * D + lane]);
    const float od = bf2f(outp[row * ldo + h * D + lane]);
    const float delta = wave_sum(dod * od);
    const float l = lse[((long long)b * H + h) * Lq + i];
    float sc[MAXK / 64], dp[MAXK / 64];
#pragma unroll
    for (int t = 0; t < MAXK / 64; ++t) { sc[t] = 0.f; dp[t] = 0.f; }
    for (int dd = 0; dd < D; ++dd) {
      const float qv = __shfl(qd, dd, 64) * scale;
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
        const bool keep = !kmask || kmask[(long long)b * Lk + j] != 0;
        const float p = keep ? __expf(sc[t] - l) : 0.f;
        ps[wave][j] = p;
        dss[wave][j] = p * (dp[t] - delta);
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
    float g = 0.f;
    for (int j = 0; j < Lk; ++j) {
      const float ds = dss[wave][j];
      g += ds * bf2f(ks[j][lane]);
      atomicAdd(&dks[j][lane], ds * qd * scale);
      atomicAdd(&dvs[j][lane], ps[wave][j] * dod);
    }
    dq[row * lddq + h * D + lane] = g * scale;
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
  }
  __syncthreads();
  for (int e = threadIdx.x; e < Lk * D; e += 256) {
    const int j = e / D, dd = e % D;
    dk[b * sdkv + j * lddkv + h * D + dd] = dks[j][dd];
    dv[b * sdkv + j * lddkv + h * D + dd] = dvs[j][dd];
  }
}

}  // namespace

extern "C" int lrce_mha_fwd(const uint16_t* q, int64_t ld_q, const uint16_t* k, const uint16_t* v, int64_t ld_kv,
                            int64_t stride_kv_b, const int32_t* key_mask, uint16_t* out, int64_t ld_o, float* lse, int B, int H,
                            int Lq, int Lk, int d, float scale, void* stream) {
  if (!q || !k || !v || !out || !lse) return lrce_fail(LRCE_E_ARG, "mha_fwd: null pointer");
  if (d != D || Lk < 1 || Lk > MAXK || Lq < 1) return lrce_fail(LRCE_E_ARG, "mha_fwd: d=%d Lk=%d unsupported", d, Lk);
  mha_fwd_kernel<<<B * H, 256, 0, static_cast<hipStream_t>(stream)>>>(
      reinterpret_cast<const bf16*>(q), ld_q, reinterpret_cast<const bf16*>(k), reinterpret_cast<const bf16*>(v), ld_kv,
      stride_kv_b, key_mask, reinterpret_cast<bf16*>(out), ld_o, lse, B, H, Lq, Lk, scale);
  return lrce_check_launch("mha_fwd");
}

extern "C" int lrce_mha_bwd(const uint16_t* q, int64_t ld_q, const uint16_t* k, const uint16_t* v, int64_t ld_kv,
                            int64_t stride_kv_b, const int32_t* key_mask, const uint16_t* out, int64_t ld_o, const uint16_t* dout,
                            const float* lse, float* dq, int64_t ld_dq, float* dk, float* dv, int64_t ld_dkv,
                            int64_t stride_dkv_b, int B, int H, int Lq, int Lk, int d, float scale, void* stream) {
  if (!q || !k || !v || !out || !dout || !lse || !dq || !dk || !dv) return lrce_fail(LRCE_E_ARG, "mha_bwd: null pointer");
  if (d != D || Lk < 1 || Lk > MAXK || Lq < 1) return lrce_fail(LRCE_E_ARG, "mha_bwd: d=%d Lk=%d unsupported", d, Lk);
  mha_bwd_kernel<<<B * H, 256, 0, static_cast<hipStream_t>(stream)>>>(
      reinterpret_cast<const bf16*>(q), ld_q, reinterpret_cast<const bf16*>(k), reinterpret_cast<const bf16*>(v), ld_kv,
      stride_kv_b, key_mask, reinterpret_cast<const bf16*>(out), ld_o, reinterpret_cast<const bf16*>(dout), lse, dq, ld_dq, dk, dv,
      ld_dkv, stride_dkv_b, B, H, Lq, Lk, scale);
  return lrce_check_launch("mha_bwd");
}
