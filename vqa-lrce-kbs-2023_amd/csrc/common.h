// Shared device helpers for the LRCE gfx950 kernels.  CDNA4 only (wave64, MFMA bf16).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>

typedef __bf16 bf16;
typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) __bf16 bf16x4;
typedef __attribute__((ext_vector_type(2))) __bf16 bf16x2;
typedef __attribute__((ext_vector_type(4))) short s16x4;
typedef __attribute__((ext_vector_type(4))) float f32x4;
typedef __attribute__((ext_vector_type(2))) float f32x2;
typedef __attribute__((ext_vector_type(16))) float f32x16;

#define LRCE_LDS __attribute__((address_space(3)))

__device__ __forceinline__ float bf2f(bf16 x) { return (float)x; }
__device__ __forceinline__ bf16 f2bf(float x) { return (bf16)x; }

__device__ __forceinline__ float bfbits2f(unsigned short u) { return __uint_as_float(((unsigned)u) << 16); }

// IEEE fp16: the BERT forward operands (the reference runs under fp16 autocast, agent_oe.py:28).
// 16-bit operands travel as bf16x8 bit patterns; these reinterpret them for the f16 MFMA forms.
typedef _Float16 f16;
typedef __attribute__((ext_vector_type(8))) _Float16 f16x8;
__device__ __forceinline__ float h2f(f16 x) { return (float)x; }
__device__ __forceinline__ f16 f2h(float x) { return (f16)x; }
// one 16-bit storage element from f32 (bf16 or f16 encoding) and back
template <bool F16>
__device__ __forceinline__ bf16 to16(float x) {
  if constexpr (F16) return __builtin_bit_cast(bf16, f2h(x));
  else return f2bf(x);
}
template <bool F16>
__device__ __forceinline__ float from16(bf16 x) {
  if constexpr (F16) return h2f(__builtin_bit_cast(f16, x));
  else return bf2f(x);
}
__device__ __forceinline__ bf16 to16r(float x, bool f16) { return f16 ? to16<true>(x) : to16<false>(x); }
__device__ __forceinline__ float from16r(bf16 x, bool f16) { return f16 ? from16<true>(x) : from16<false>(x); }

// 32x32x16 / 16x16x32 MFMA on 16-bit operands of either encoding
template <bool F16>
__device__ __forceinline__ f32x16 mfma32x32x16(bf16x8 a, bf16x8 b, f32x16 c) {
  if constexpr (F16)
    return __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(f16x8, a), __builtin_bit_cast(f16x8, b), c, 0, 0, 0);
  else
    return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}
template <bool F16>
__device__ __forceinline__ f32x4 mfma16x16x32(bf16x8 a, bf16x8 b, f32x4 c) {
  if constexpr (F16)
    return __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(f16x8, a), __builtin_bit_cast(f16x8, b), c, 0, 0, 0);
  else
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

// GELU, erf form (torch F.gelu default, approximate='none'), and its derivative.
// Phi(x) = 0.5 erfc(-x/sqrt2) from Abramowitz-Stegun 7.1.26 (|err(erf)| <= 1.5e-7): one rcp, one exp2,
// five FMAs — libm erff is a two-range polynomial with branches and dominated the GELU-epilogue GEMMs.
// The tail is evaluated as 0.5 * erfc(|z|) directly (no 1 - erf cancellation); the derivative reuses
// exp(-x^2/2) as the normal pdf.  Max abs error vs the exact form: 6e-7 (value), 2.5e-7 (derivative).
// z = |x|/sqrt2 and the 1/2 are folded into the constants (t = 1 / (1 + 0.3275911 z), the polynomial
// coefficients halved, exp(-z^2) = exp2(x^2 * -log2(e)/2)), and every step is an explicit fma / mul,
// so the scalar form and the packed pair form below (v_pk_fma_f32 / v_pk_mul_f32: half the VALU
// issue of the polynomial in the GEMM epilogues, which the GELU math dominates) give identical bits.
constexpr float GELU_T = 0.23164189f;          // 0.3275911 / sqrt(2)
constexpr float GELU_E = -0.72134752044448170f; // -log2(e) / 2
constexpr float GELU_B1 = 0.127414796f, GELU_B2 = -0.142248368f, GELU_B3 = 0.7107068705f, GELU_B4 = -0.7265760135f,
                GELU_B5 = 0.5307027145f;        // A&S 7.1.26 a1..a5, halved
constexpr float GELU_PDF = 0.39894228040143268f;   // 1 / sqrt(2 pi)
__device__ __forceinline__ float gelu_q(float x, float* e_out) {
  const float t = __builtin_amdgcn_rcpf(__builtin_fmaf(fabsf(x), GELU_T, 1.0f));
  const float e = __builtin_amdgcn_exp2f((x * x) * GELU_E);
  *e_out = e;
  float p = __builtin_fmaf(GELU_B5, t, GELU_B4);
  p = __builtin_fmaf(p, t, GELU_B3);
  p = __builtin_fmaf(p, t, GELU_B2);
  p = __builtin_fmaf(p, t, GELU_B1);
  const float pt = p * t;
  const float hi = __builtin_fmaf(-pt, e, 1.0f), lo = pt * e;   // 1 - q, q = 0.5 erfc(|x|/sqrt2)
  return x >= 0.f ? hi : lo;                                    // Phi(x)
}
__device__ __forceinline__ float gelu_f(float x) {
  float e;
  return x * gelu_q(x, &e);
}
__device__ __forceinline__ float gelu_grad_f(float x) {
  float e;
  const float phi = gelu_q(x, &e);
  return __builtin_fmaf(x * GELU_PDF, e, phi);
}
// the same on a pair (ext vector: the compiler issues the packed FP32 forms)
typedef float f32x2v __attribute__((ext_vector_type(2)));
__device__ __forceinline__ f32x2v gelu_q2(f32x2v x, f32x2v& e) {
  const f32x2v ax = __builtin_elementwise_abs(x);
  const f32x2v d = __builtin_elementwise_fma(ax, (f32x2v)(GELU_T), (f32x2v)(1.0f));
  f32x2v t;
  t.x = __builtin_amdgcn_rcpf(d.x);
  t.y = __builtin_amdgcn_rcpf(d.y);
  const f32x2v ee = (x * x) * (f32x2v)(GELU_E);
  e.x = __builtin_amdgcn_exp2f(ee.x);
  e.y = __builtin_amdgcn_exp2f(ee.y);
  f32x2v p = __builtin_elementwise_fma((f32x2v)(GELU_B5), t, (f32x2v)(GELU_B4));
  p = __builtin_elementwise_fma(p, t, (f32x2v)(GELU_B3));
  p = __builtin_elementwise_fma(p, t, (f32x2v)(GELU_B2));
  p = __builtin_elementwise_fma(p, t, (f32x2v)(GELU_B1));
  const f32x2v pt = p * t;
  const f32x2v hi = __builtin_elementwise_fma(-pt, e, (f32x2v)(1.0f)), lo = pt * e;
  f32x2v phi;
  phi.x = x.x >= 0.f ? hi.x : lo.x;
  phi.y = x.y >= 0.f ? hi.y : lo.y;
  return phi;
}
__device__ __forceinline__ f32x2v gelu2(f32x2v x) {
  f32x2v e;
  return x * gelu_q2(x, e);
}
__device__ __forceinline__ f32x2v gelu_grad2(f32x2v x) {
  f32x2v e;
  const f32x2v phi = gelu_q2(x, e);
  return __builtin_elementwise_fma(x * (f32x2v)(GELU_PDF), e, phi);
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// Bijective XCD-aware remap of a linear workgroup id (cdna_hip_programming.md §5 "XCD swizzle must
// be bijective"): blocks that the dispatcher deals to one XCD (id % 8 equal) get a contiguous range.
__device__ __forceinline__ int xcd_remap(int id, int nwg) {
  const int q = nwg >> 3, r = nwg & 7, x = id & 7;
  return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + (id >> 3);
}

// 64-bit counter-based hash -> uniform floats in [0,1): dropout / DropPath masks.  One hash serves
// four consecutive indices (16 bits each: keep-probability granularity 2^-16), so a thread handling
// a float4 of consecutive elements pays one hash instead of four (lrce_uniform4); every site draws
// element idx's value the same way, so forward and backward masks agree wherever they are computed.
__device__ __forceinline__ uint64_t lrce_hash64(uint64_t x) {
  x ^= x >> 33; x *= 0xff51afd7ed558ccdULL; x ^= x >> 33; x *= 0xc4ceb9fe1a85ec53ULL; x ^= x >> 33;
  return x;
}
__device__ __forceinline__ float lrce_uniform(uint64_t seed, uint64_t idx) {
  const uint64_t h = lrce_hash64(seed * 0x9E3779B97F4A7C15ULL + (idx >> 2));
  return (float)((h >> (16 * (idx & 3))) & 0xFFFFu) * (1.0f / 65536.0f);
}
// the uniforms of indices 4*idx4 .. 4*idx4 + 3
__device__ __forceinline__ float4 lrce_uniform4(uint64_t seed, uint64_t idx4) {
  const uint64_t h = lrce_hash64(seed * 0x9E3779B97F4A7C15ULL + idx4);
  const float s = 1.0f / 65536.0f;
  return make_float4((float)(h & 0xFFFFu) * s, (float)((h >> 16) & 0xFFFFu) * s, (float)((h >> 32) & 0xFFFFu) * s,
                     (float)((h >> 48) & 0xFFFFu) * s);
}
__device__ __forceinline__ uint64_t lrce_seed(uint64_t seed, const uint64_t* off) { return off ? seed + *off : seed; }

// compile-time loop: f(integral_constant<int, I>) for I = 0..N-1 (keeps accumulator indices static)
template <int I, int N, typename F>
__device__ __forceinline__ void static_for_impl(F&& f) {
  if constexpr (I < N) {
    f(std::integral_constant<int, I>{});
    static_for_impl<I + 1, N>(f);
  }
}
template <int N, typename F>
__device__ __forceinline__ void static_for(F&& f) { static_for_impl<0, N>(f); }
