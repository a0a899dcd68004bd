// Fused optimizer step over the flat parameter buffer: the caller side of the LRCE training step
// (AdamW with 3 learning-rate groups, agent_base.py:27-44, plus the L2-norm regulariser
// reg * sum_t ||p_t||_2, agent_base.py:103-108, whose gradient reg * p_t / ||p_t|| is folded in
// here instead of being back-propagated through 783 norm kernels).  Parameters are laid out so
// that every tensor starts at a multiple of 1024 elements; chunk c (1024 elements) belongs to one
// tensor (chunk_tensor[c]).  One pass reads p, g, m, v and writes p, m, v and the bf16 shadow
// copy the forward kernels consume: 4+4+4+4 + 4+4+4+2 = 30 B per parameter, HBM-bound.
#include <cstdlib>

#include "common.h"
#include "lrce_capi.h"

namespace {

// Per-tensor squared norms are reduced DETERMINISTICALLY: each 1024-element chunk's sum is stored
// (plain store, chunk_sq[c]), then segsum_kernel adds the chunks of every tensor in a fixed order.
// (Float atomics would make ||p|| — and through the L2 term reg * p / ||p|| every update — differ in
// the last bits from run to run and from rank to rank: data-parallel replicas would drift apart.)
__global__ void __launch_bounds__(256) sumsq_kernel(const float* __restrict__ p, const int* __restrict__ chunk_tensor, int n_chunks,
                                                    float* __restrict__ sumsq, float* __restrict__ chunk_sq) {
  const int c = blockIdx.x;
  if (c >= n_chunks) return;
  const float4 v = reinterpret_cast<const float4*>(p + (long long)c * 1024)[threadIdx.x];
  float s = v.x * v.x + v.y * v.y + v.z * v.z + v.w * v.w;
  s = wave_sum(s);
  __shared__ float red[4];
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) {
    const float t = (red[0] + red[1]) + (red[2] + red[3]);
    if (chunk_sq) chunk_sq[c] = t;
    else atomicAdd(sumsq + chunk_tensor[c], t);
  }
}

// out[t] = sum of chunk_sq over tensor t's chunks [off[t], off[t+1]), fixed order (one block per tensor)
__global__ void __launch_bounds__(256) segsum_kernel(const float* __restrict__ chunk_sq, const int* __restrict__ off,
                                                     int n_tensors, float* __restrict__ out) {
  const int t = blockIdx.x;
  if (t >= n_tensors) return;
  const int c0 = off[t], c1 = off[t + 1];
  float s = 0.f;
  for (int c = c0 + (int)threadIdx.x; c < c1; c += 256) s += chunk_sq[c];
  __shared__ float red[256];
  red[threadIdx.x] = s;
  __syncthreads();
#pragma unroll
  for (int w = 128; w > 0; w >>= 1) {
    if ((int)threadIdx.x < w) red[threadIdx.x] += red[threadIdx.x + w];
    __syncthreads();
  }
  if (threadIdx.x == 0) out[t] = red[0];
}

// One WAVE per 1024-element chunk (16 parameters per lane as 4 coalesced float4 rows), ADAMW_CPW
// consecutive chunks per wave, 4 waves per workgroup: the per-chunk scalars (tensor, lr, norm) are
// wave-uniform loads, every lane has 16 loads of p / g / m / v in flight, and the chunk's sum of
// squares (the next step's L2 norm, reduced deterministically by segsum_kernel) is one wave_sum —
// no workgroup barrier anywhere.  The bias corrections are computed from the device step
// (exp2 of t * log2(beta)), so the launch replays unchanged from a HIP graph.
constexpr int ADAMW_CPW = 2;

// NT: non-temporal loads / stores (every operand is touched once per step); CPW: chunks per wave
typedef float f32x4n __attribute__((ext_vector_type(4)));
template <bool NT>
__device__ __forceinline__ float4 ld_s(const float* q) {
  if constexpr (NT) {
    const f32x4n t = __builtin_nontemporal_load(reinterpret_cast<const f32x4n*>(q));
    return make_float4(t.x, t.y, t.z, t.w);
  } else {
    return *reinterpret_cast<const float4*>(q);
  }
}
template <bool NT>
__device__ __forceinline__ void st_s(float* q, float4 v) {
  if constexpr (NT) __builtin_nontemporal_store(f32x4n{v.x, v.y, v.z, v.w}, reinterpret_cast<f32x4n*>(q));
  else *reinterpret_cast<float4*>(q) = v;
}

template <bool NT, int CPW>
__global__ void __launch_bounds__(256) adamw_kernel(float* __restrict__ p, const float* __restrict__ g, float* __restrict__ m,
                                                    float* __restrict__ v, const int* __restrict__ chunk_tensor,
                                                    const float* __restrict__ tensor_lr, const float* __restrict__ sumsq,
                                                    bf16* __restrict__ pb, int n_chunks, float b1, float b2, float eps, float wd,
                                                    float gscale, float reg, float bc1, float bc2, const float* __restrict__ step_dev,
                                                    float* __restrict__ sumsq_next, bf16* __restrict__ ph, long long h_lo,
                                                    long long h_hi, const bf16* __restrict__ g16,
                                                    float* __restrict__ chunk_sq, const float* __restrict__ skip_slots,
                                                    int n_skip, long long skip_c0, long long skip_c1) {
  const int lane = threadIdx.x & 63;
  const int wave_id = blockIdx.x * 4 + (threadIdx.x >> 6);
  // found-inf: chunks [skip_c0, skip_c1) keep their parameters and moments when any of the n_skip
  // gradient-scale slots [S, 1/S, amax, flag] raised its flag (an fp16 gradient operand overflowed,
  // lrce_layernorm_bwd_f16s) — GradScaler's skipped step for the group those operands feed
  bool found_inf = false;
  if (skip_slots && wave_id * CPW < skip_c1 && (wave_id + 1) * CPW > skip_c0)
    found_inf = __ballot(lane < n_skip && skip_slots[4 * lane + 3] != 0.f) != 0ull;
  if (step_dev) {
    const float t = *step_dev;
    bc1 = 1.0f - exp2f(t * __log2f(b1));
    bc2 = 1.0f - exp2f(t * __log2f(b2));
  }
  const float isb2 = rsqrtf(bc2);
  for (int k = 0; k < CPW; ++k) {
    const int c = wave_id * CPW + k;
    if (c >= n_chunks) break;
    const int t = chunk_tensor[c];
    const float lr = tensor_lr[t];
    const float ss = sumsq ? sumsq[t] : 0.f;
    const float rc = (reg != 0.f && ss > 0.f) ? reg * rsqrtf(ss) : 0.f;
    const float step = lr / bc1, decay = 1.0f - lr * wd;
    const long long base = (long long)c * 1024 + lane * 4;
    const bool skip = found_inf && c >= skip_c0 && c < skip_c1;
    float4 pp[4], gg[4], mm[4], vv[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const long long i = base + r * 256;
      pp[r] = ld_s<NT>(p + i);
      if (g16) {   // bf16 gradient (the all-reduced bf16 buckets of lrce/distributed.py)
        const bf16x4 h = *reinterpret_cast<const bf16x4*>(g16 + i);
        gg[r] = make_float4(bf2f(h[0]), bf2f(h[1]), bf2f(h[2]), bf2f(h[3]));
      } else {
        gg[r] = ld_s<NT>(g + i);
      }
      mm[r] = ld_s<NT>(m + i);
      vv[r] = ld_s<NT>(v + i);
    }
    float q = 0.f;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const long long i = base + r * 256;
      float* pa = &pp[r].x; const float* ga = &gg[r].x; float* ma = &mm[r].x; float* va = &vv[r].x;
      bf16x4 ob;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const float gr = ga[j] * gscale + rc * pa[j];
        // a non-finite gradient element (an fp16 gradient operand that overflowed) leaves its parameter
        // and moments as they are, instead of poisoning them for every later step; the reference's
        // GradScaler skips the whole step in that case (agent_oe.py:40-42)
        const bool fin = __builtin_isfinite(gr) && !skip;
        const float mn = b1 * ma[j] + (1.0f - b1) * gr;
        const float vn = b2 * va[j] + (1.0f - b2) * gr * gr;
        const float np = pa[j] * decay - step * mn / (sqrtf(vn) * isb2 + eps);
        ma[j] = fin ? mn : ma[j];
        va[j] = fin ? vn : va[j];
        pa[j] = fin ? np : pa[j];
        ob[j] = f2bf(pa[j]);
      }
      st_s<NT>(p + i, pp[r]);
      st_s<NT>(m + i, mm[r]);
      st_s<NT>(v + i, vv[r]);
      if (pb) *reinterpret_cast<bf16x4*>(pb + i) = ob;
      if (ph && i >= h_lo && i < h_hi) {   // fp16 shadow of the BERT range (chunk-uniform branch)
        bf16x4 oh;
        oh[0] = to16<true>(pp[r].x); oh[1] = to16<true>(pp[r].y); oh[2] = to16<true>(pp[r].z); oh[3] = to16<true>(pp[r].w);
        *reinterpret_cast<bf16x4*>(ph + (i - h_lo)) = oh;
      }
      q += pp[r].x * pp[r].x + pp[r].y * pp[r].y + pp[r].z * pp[r].z + pp[r].w * pp[r].w;
    }
    if (sumsq_next) {
      q = wave_sum(q);
      if (lane == 0) {
        if (chunk_sq) chunk_sq[c] = q;
        else atomicAdd(sumsq_next + t, q);
      }
    }
  }
}

}  // namespace

extern "C" int lrce_l2norm_multi(const float* p, const int32_t* chunk_tensor, int n_chunks, float* sumsq, int n_tensors,
                                 const int32_t* tensor_chunk_off, float* chunk_sq, void* stream) {
  if (!p || !chunk_tensor || !sumsq) return lrce_fail(LRCE_E_ARG, "l2norm_multi: null pointer");
  if (!tensor_chunk_off != !chunk_sq) return lrce_fail(LRCE_E_ARG, "l2norm_multi: tensor_chunk_off and chunk_sq go together");
  hipStream_t s = static_cast<hipStream_t>(stream);
  if (!chunk_sq) (void)hipMemsetAsync(sumsq, 0, sizeof(float) * n_tensors, s);
  if (n_chunks > 0) sumsq_kernel<<<n_chunks, 256, 0, s>>>(p, chunk_tensor, n_chunks, sumsq, chunk_sq);
  if (chunk_sq && n_tensors > 0) segsum_kernel<<<n_tensors, 256, 0, s>>>(chunk_sq, tensor_chunk_off, n_tensors, sumsq);
  return lrce_check_launch("l2norm_multi");
}

extern "C" int lrce_adamw_step(float* p, const float* g, float* m, float* v, const int32_t* chunk_tensor, const float* tensor_lr,
                               const float* sumsq, uint16_t* p_bf16, int n_chunks, float beta1, float beta2, float eps,
                               float weight_decay, float grad_scale, float reg, float bc1, float bc2, const float* step,
                               float* sumsq_next, uint16_t* p_f16, int64_t f16_lo, int64_t f16_hi, const uint16_t* g_bf16,
                               const int32_t* tensor_chunk_off, float* chunk_sq, int n_tensors, const float* skip_slots,
                               int n_skip_slots, int64_t skip_c0, int64_t skip_c1, void* stream) {
  if (tensor_chunk_off && !chunk_sq) return lrce_fail(LRCE_E_ARG, "adamw_step: tensor_chunk_off needs chunk_sq");
  if (skip_slots && (n_skip_slots < 1 || n_skip_slots > 64 || skip_c0 < 0 || skip_c1 < skip_c0))
    return lrce_fail(LRCE_E_ARG, "adamw_step: skip slots n=%d range [%lld, %lld)", n_skip_slots, (long long)skip_c0,
                     (long long)skip_c1);
  if (!p || (!g && !g_bf16) || !m || !v || !chunk_tensor || !tensor_lr) return lrce_fail(LRCE_E_ARG, "adamw_step: null pointer");
  // the f16 range is relative to p (it may start before this call's first chunk: a sub-range update)
  if (p_f16 && (f16_lo % 1024 || f16_hi % 1024 || f16_hi < f16_lo))
    return lrce_fail(LRCE_E_ARG, "adamw_step: f16 shadow range [%lld, %lld) not chunk aligned", (long long)f16_lo, (long long)f16_hi);
  if (n_chunks > 0) {
    // one chunk per wave with non-temporal loads / stores: every operand is touched once per step, so
    // the streaming hint keeps them from evicting L2 lines for nothing, and one chunk per wave doubles
    // the waves in flight (110 M parameters: 630 -> 515 us, 5.2 -> 6.4 TB/s against two chunks per
    // wave with plain accesses)
    const int cpw = 1;
    const dim3 grid((n_chunks + 4 * cpw - 1) / (4 * cpw));
    hipStream_t s = static_cast<hipStream_t>(stream);
    auto launch = [&](auto kern) {
      kern<<<grid, 256, 0, s>>>(p, g, m, v, chunk_tensor, tensor_lr, sumsq, reinterpret_cast<bf16*>(p_bf16), n_chunks, beta1,
                                beta2, eps, weight_decay, grad_scale, reg, bc1, bc2, step, sumsq_next,
                                reinterpret_cast<bf16*>(p_f16), f16_lo, f16_hi, reinterpret_cast<const bf16*>(g_bf16),
                                sumsq_next ? chunk_sq : nullptr, skip_slots, n_skip_slots, skip_c0, skip_c1);
    };
    launch(adamw_kernel<true, 1>);
  }
  if (sumsq_next && chunk_sq && tensor_chunk_off && n_tensors > 0)
    segsum_kernel<<<n_tensors, 256, 0, static_cast<hipStream_t>(stream)>>>(chunk_sq, tensor_chunk_off, n_tensors, sumsq_next);
  return lrce_check_launch("adamw_step");
}
