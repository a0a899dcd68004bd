// Device helpers shared by the recurrent-decoder kernels (decoder.hip: per-block launches;
// decoder_step.hip: the persistent recurrent step).  Internal linkage: included by each .hip.
#pragma once
#include "common.h"

namespace {

constexpr int E = 768, H = 12, D = 64, NT = 256, MAXK = 192;

constexpr int WROWS = 16;            // rows of a head's 64-row weight slice per wave
constexpr int NRI = 24;              // 16-B register loads per lane for 16 rows x 768 (fp16)
constexpr int MAXTXT = 48;           // text-segment keys (question tokens + 1)
constexpr int TXI = (MAXTXT * 8 + NT - 1) / NT;   // text (key, 8-dim chunk) items per thread

// Debug phase timestamps (lrce_dec_set_trace; NULL in production): wave 0 of every workgroup stores
// s_memrealtime (100 MHz) at the marks of kernel k into p.trace[(k * 1024 + wg) * 16 + i] (the pointer
// rides in the kernel arguments: a scalar load, no vector-memory wait).
#define DEC_MARK(K, I)                                                                                     \
  do {                                                                                                   \
    if (p.trace && threadIdx.x == 0 && blockIdx.x < 1024)                                                \
      p.trace[((K) * 1024 + blockIdx.x) * 16 + (I)] = __builtin_amdgcn_s_memrealtime();                  \
  } while (0)

__device__ __forceinline__ void dec_glds(const void* sbase, uint32_t voff, uint32_t lds_dst) {
  unsigned keep;
  const uint64_t a = reinterpret_cast<uintptr_t>(sbase);
  const uint64_t su = (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)a) |
                      ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)(a >> 32)) << 32);
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, %2\n\ts_mov_b32 m0, %0"
               : "=&s"(keep) : "v"(voff), "s"(su), "s"(__builtin_amdgcn_readfirstlane(lds_dst)) : "memory");
}
__device__ __forceinline__ uint32_t dec_lds_addr(const void* p) { return (uint32_t)(uintptr_t)((LRCE_LDS const void*)p); }
// the same with a per-lane 64-bit source address (rows from two key segments in one instruction)
__device__ __forceinline__ void dec_glds_p(const void* src, uint32_t lds_dst) {
  unsigned keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
               : "=&s"(keep) : "v"(src), "s"(__builtin_amdgcn_readfirstlane(lds_dst)) : "memory");
}

// Workgroup barrier for LDS hand-offs only: __syncthreads() would also drain vmcnt(0), i.e. wait for
// every bulk load and LDS-DMA still in flight (the weight slices), serialising the loads with the
// LayerNorm / reduction phases they are meant to overlap.  Global-memory ordering is explicit where
// needed (s_waitcnt vmcnt(0) before reading DMA'd LDS, and in publish_partial).
__device__ __forceinline__ void lds_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

// Keep a loaded value in registers: hipcc may otherwise re-load a read-only operand at its later
// uses (to save VGPRs), and such a re-load behind the bulk loads waits for all of them.
__device__ __forceinline__ void pin(float4& v) { asm volatile("" : "+v"(v.x), "+v"(v.y), "+v"(v.z), "+v"(v.w)); }
// the device RNG offset (lrce_rng_offset), read once at kernel start
__device__ __forceinline__ uint64_t rng_off_now(const uint64_t* off) {
  uint64_t o = off ? *off : 0ull;
  asm volatile("" : "+v"(o));
  return o;
}

// cross-lane moves inside a row of 16 lanes (DPP: a VALU operand modifier, no LDS round trip)
template <int CTRL>
__device__ __forceinline__ float dpp_f(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), CTRL, 0xF, 0xF, false));
}
__device__ __forceinline__ float sum4(float v) {   // every lane: the sum of its aligned group of 4
  v += dpp_f<0xB1>(v);    // quad_perm [1,0,3,2]
  v += dpp_f<0x4E>(v);    // quad_perm [2,3,0,1]
  return v;
}
__device__ __forceinline__ float sum8(float v) {   // ... of 8
  v = sum4(v);
  v += dpp_f<0x141>(v);   // row_half_mirror: the other quad of the 8
  return v;
}

__device__ __forceinline__ void unpack8bf(const uint4 u, float (&f)[8]) {
  const unsigned w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    f[2 * e] = bfbits2f((unsigned short)(w[e] & 0xFFFFu));
    f[2 * e + 1] = bfbits2f((unsigned short)(w[e] >> 16));
  }
}

__device__ __forceinline__ void unpack8(const uint4 u, float (&f)[8]) {
  const unsigned w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    f[2 * e] = (float)__builtin_bit_cast(f16, (unsigned short)(w[e] & 0xFFFFu));
    f[2 * e + 1] = (float)__builtin_bit_cast(f16, (unsigned short)(w[e] >> 16));
  }
}

// The [768][64] slice W[:, h*64 .. h*64+63] of a row-major [768][768] fp16 matrix -> LDS image
// [n][64] (128-B rows), 8 rows per 1-KB DMA instruction, 24 per wave.  Issued at kernel start.
// 16-B chunk k of row n sits in slot k ^ (n & 7) (slice_at): a thread per row reading chunk k of 8
// consecutive rows then hits 8 different bank groups instead of one.
__device__ __forceinline__ void slice_dma(const f16* w, int h, void* lds, int wave, int lane) {
  const uint32_t base = dec_lds_addr(lds);
#pragma unroll 4
  for (int i = 0; i < 24; ++i) {
    const int ins = wave * 24 + i;
    const int row = ins * 8 + (lane >> 3);
    dec_glds(w, (uint32_t)((row * E + h * D + ((lane & 7) ^ (row & 7)) * 8) * 2), base + (uint32_t)ins * 1024u);
  }
}
__device__ __forceinline__ const f16* slice_at(const f16* S, int n, int k) { return S + n * D + ((k ^ (n & 7)) << 3); }

// Rows r0 .. r0+15 of a row-major [.][768] fp16 matrix into registers, 24 x 16 B per lane:
// ins r (< 16): row r0 + r, 8-element chunk `lane` (elements 8*lane .. 8*lane+7);
// ins 16 + s:   row r0 + 2s + (lane >= 32), chunk 64 + (lane & 31).
__device__ __forceinline__ void rows_load(const f16* w, int r0, int lane, uint4 (&reg)[NRI]) {
#pragma unroll
  for (int r = 0; r < 16; ++r) reg[r] = *reinterpret_cast<const uint4*>(w + (long long)(r0 + r) * E + lane * 8);
#pragma unroll
  for (int s = 0; s < 8; ++s)
    reg[16 + s] = *reinterpret_cast<const uint4*>(w + (long long)(r0 + 2 * s + (lane >> 5)) * E + (64 + (lane & 31)) * 8);
}

__device__ __forceinline__ float dot8(const float (&a)[8], const float* x) {
  const float4 x0 = *reinterpret_cast<const float4*>(x), x1 = *reinterpret_cast<const float4*>(x + 4);
  return ((a[0] * x0.x + a[1] * x0.y) + (a[2] * x0.z + a[3] * x0.w)) + ((a[4] * x1.x + a[5] * x1.y) + (a[6] * x1.z + a[7] * x1.w));
}

// out[r] = W[r0 + r] . x for the wave's 16 rows (x in LDS, 768 f32); result written to o[16] in LDS
// through a [16][64] partial image (each lane's per-row dot, then 4 lanes per row).
__device__ __forceinline__ void rows_gemv(const uint4 (&reg)[NRI], const float* x, float* pp, float* o, int lane) {
  float u[16];
  float wf[8];
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    unpack8(reg[r], wf);
    u[r] = dot8(wf, x + lane * 8);
  }
#pragma unroll
  for (int s = 0; s < 8; ++s) {
    unpack8(reg[16 + s], wf);
    const float v = dot8(wf, x + (64 + (lane & 31)) * 8);
    if (lane < 32) u[2 * s] += v;
    else u[2 * s + 1] += v;
  }
#pragma unroll
  for (int r = 0; r < 16; ++r) pp[r * 64 + lane] = u[r];
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  const int r = lane >> 2, q = lane & 3;
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < 16; ++i) s += pp[r * 64 + q * 16 + i];
  s = sum4(s);
  if (q == 0) o[r] = s;
}

// acc[768] (LDS, per wave) = sum_r v[r] W[r0 + r][:] for the wave's 16 rows (the transposed product
// W^T v of a dX): lane l owns columns 8l..8l+7 and 512 + 8(l&31).. (the latter split by lane half)
__device__ __forceinline__ void rows_gemv_t(const uint4 (&reg)[NRI], const float* v, float* acc, int lane) {
  float a[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f}, c[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  float wf[8];
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    unpack8(reg[r], wf);
    const float vr = v[r];
#pragma unroll
    for (int e = 0; e < 8; ++e) a[e] = fmaf(vr, wf[e], a[e]);
  }
#pragma unroll
  for (int s = 0; s < 8; ++s) {
    unpack8(reg[16 + s], wf);
    const float vr = v[2 * s + (lane >> 5)];
#pragma unroll
    for (int e = 0; e < 8; ++e) c[e] = fmaf(vr, wf[e], c[e]);
  }
#pragma unroll
  for (int e = 0; e < 8; ++e) c[e] += __shfl_xor(c[e], 32, 64);
  *reinterpret_cast<float4*>(acc + lane * 8) = make_float4(a[0], a[1], a[2], a[3]);
  *reinterpret_cast<float4*>(acc + lane * 8 + 4) = make_float4(a[4], a[5], a[6], a[7]);
  if (lane < 32) {
    *reinterpret_cast<float4*>(acc + 512 + lane * 8) = make_float4(c[0], c[1], c[2], c[3]);
    *reinterpret_cast<float4*>(acc + 512 + lane * 8 + 4) = make_float4(c[4], c[5], c[6], c[7]);
  }
}

// out[n] = sum_d S[n][d] v[d] over the LDS head slice S [768][64] (fp16): thread t owns rows t,
// t + 256, t + 512 and walks each whole row (8 x 16-B reads, swizzled slots), v (64 f32, LDS
// broadcast reads) in registers — no cross-lane reduction.  (Lane-per-chunk with an 8-lane DPP sum
// per row measured 2.5 us per launch for this phase: a dependent reduction chain per 8 rows.)
__device__ __forceinline__ void slice_gemv(const f16* S, const float* v, float* out, int t) {
  float vv[D];
#pragma unroll
  for (int e = 0; e < D; e += 4) {
    const float4 q = *reinterpret_cast<const float4*>(v + e);
    vv[e] = q.x; vv[e + 1] = q.y; vv[e + 2] = q.z; vv[e + 3] = q.w;
  }
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    const int n = t + 256 * i;
    float a0 = 0.f, a1 = 0.f;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      float wf[8];
      unpack8(*reinterpret_cast<const uint4*>(slice_at(S, n, k)), wf);
      a0 = fmaf(wf[0], vv[8 * k], a0); a1 = fmaf(wf[1], vv[8 * k + 1], a1);
      a0 = fmaf(wf[2], vv[8 * k + 2], a0); a1 = fmaf(wf[3], vv[8 * k + 3], a1);
      a0 = fmaf(wf[4], vv[8 * k + 4], a0); a1 = fmaf(wf[5], vv[8 * k + 5], a1);
      a0 = fmaf(wf[6], vv[8 * k + 6], a0); a1 = fmaf(wf[7], vv[8 * k + 7], a1);
    }
    out[n] = a0 + a1;
  }
}

// out[d] (d < 64) = sum_n S[n][d] u[n] (u: 768 in LDS); per-wave partials into red[wave][64]
__device__ __forceinline__ void slice_gemv_t(const f16* S, const float* u, float* red, int wave, int lane) {
  const int g = lane >> 3, c = lane & 7;
  float a[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll 4
  for (int i = 0; i < 24; ++i) {
    const int n = wave * 192 + i * 8 + g;
    float wf[8];
    unpack8(*reinterpret_cast<const uint4*>(slice_at(S, n, c)), wf);
    const float un = u[n];
#pragma unroll
    for (int e = 0; e < 8; ++e) a[e] = fmaf(un, wf[e], a[e]);
  }
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    a[e] += dpp_f<0x128>(a[e]);   // row_ror:8 (lanes g, g^1 of a row)
    a[e] += __shfl_xor(a[e], 16, 64);
    a[e] += __shfl_xor(a[e], 32, 64);
  }
  if (g == 0) {
#pragma unroll
    for (int e = 0; e < 8; ++e) red[wave * 64 + c * 8 + e] = a[e];
  }
}

__device__ __forceinline__ float block_sum4(float v, float* red2, int lane, int wave) {
  v = wave_sum(v);
  if (lane == 0) red2[wave] = v;
  lds_barrier();
  const float r = (red2[0] + red2[1]) + (red2[2] + red2[3]);
  lds_barrier();
  return r;
}
__device__ __forceinline__ float block_max4(float v, float* red2, int lane, int wave) {
  v = wave_max(v);
  if (lane == 0) red2[wave] = v;
  lds_barrier();
  const float r = fmaxf(fmaxf(red2[0], red2[1]), fmaxf(red2[2], red2[3]));
  lds_barrier();
  return r;
}

// LayerNorm forward of one 768 row held as float4 by threads t < 192 (two-pass statistics, the
// order of lrce_gemm_ln mode 1): y = (x - mu) rstd g + b into ys (LDS).  s1_local: this thread's
// (x.x + x.y) + (x.z + x.w) (0 past the row), computed by the caller before it issues its bulk loads
// (the compiler's in-order vmcnt waits would otherwise hold the statistics until they land).
__device__ __forceinline__ float row_sum_local(float4 x, int t) { return t < E / 4 ? (x.x + x.y) + (x.z + x.w) : 0.f; }
__device__ __forceinline__ void ln_row_fwd(float4 x, float s1_local, float4 gg, float4 be, float eps, float* ys,
                                           float* red2, int t, int lane, int wave, float& mu, float& rs) {
  const bool live = t < E / 4;
  const float s1 = block_sum4(s1_local, red2, lane, wave);
  mu = s1 * (1.0f / E);
  float4 d = make_float4(x.x - mu, x.y - mu, x.z - mu, x.w - mu);
  const float s2 = block_sum4(live ? (d.x * d.x + d.y * d.y) + (d.z * d.z + d.w * d.w) : 0.f, red2, lane, wave);
  rs = rsqrtf(s2 * (1.0f / E) + eps);
  if (live) {
    *reinterpret_cast<float4*>(ys + 4 * t) =
        make_float4(d.x * rs * gg.x + be.x, d.y * rs * gg.y + be.y, d.z * rs * gg.z + be.z, d.w * rs * gg.w + be.w);
  }
}

// LayerNorm backward of one row: dy (float4, t < 192), x, mean, rstd, gamma -> dx (float4), the
// formula of lrce_gemm_ln mode 2: dx = rstd (g - mean(g) - xh mean(g xh)), g = dy gamma.  Local
// part (g, xh and this thread's two sums) first, the block reductions after the caller's bulk loads.
struct LnBwdLocal {
  float4 g, xh;
  float s1, s2;
};
__device__ __forceinline__ LnBwdLocal ln_row_bwd_local(float4 dy, float4 x, float4 gm, float mu, float rs, int t) {
  LnBwdLocal l;
  l.g = make_float4(0.f, 0.f, 0.f, 0.f);
  l.xh = l.g;
  if (t < E / 4) {
    l.g = make_float4(dy.x * gm.x, dy.y * gm.y, dy.z * gm.z, dy.w * gm.w);
    l.xh = make_float4((x.x - mu) * rs, (x.y - mu) * rs, (x.z - mu) * rs, (x.w - mu) * rs);
  }
  l.s1 = (l.g.x + l.g.y) + (l.g.z + l.g.w);
  l.s2 = (l.g.x * l.xh.x + l.g.y * l.xh.y) + (l.g.z * l.xh.z + l.g.w * l.xh.w);
  return l;
}
__device__ __forceinline__ float4 ln_row_bwd(const LnBwdLocal& l, float rs, float* red2, int lane, int wave) {
  const float s1 = block_sum4(l.s1, red2, lane, wave);
  const float s2 = block_sum4(l.s2, red2, lane, wave);
  const float mg = s1 * (1.0f / E), mgx = s2 * (1.0f / E);
  const float4 g = l.g, xh = l.xh;
  return make_float4(rs * (g.x - mg - xh.x * mgx), rs * (g.y - mg - xh.y * mgx), rs * (g.z - mg - xh.z * mgx),
                     rs * (g.w - mg - xh.w * mgx));
}

__device__ __forceinline__ float drop1(float v, float p, uint64_t seed, long long idx) {
  return lrce_uniform(seed, (uint64_t)idx) >= p ? v / (1.0f - p) : 0.f;
}

// publish this head's partial row (768 f32) and return true in the last of the 12 heads to arrive.
// Hand-off protocol: MI355X_MICROARCH.md "Valid forms", first row of the sc1 hand-off table (the
// same as gemm_f32.hip's skinny split-K), in place of a release/acquire pair — every partial is an
// agent-scope relaxed store (global_store ... sc1: written through past this XCD's L2), every storing
// wave drains it with s_waitcnt vmcnt(0), a workgroup barrier follows, ONE lane's agent-scope atomic
// add signals, the workgroup whose add returns H-1 is told by that value, and it reads EVERY partial
// with agent-scope relaxed loads (global_load ... sc1, no L1/L2 reuse) after the barrier that
// publishes last_flag.  All four conditions of that row hold, so no buffer_wbl2 / buffer_inv (~1.7 us
// each, on a ~10-20 us latency-bound launch) is needed.  This is measured gfx950 behaviour, not a
// C++ memory-model guarantee: a port to another target must switch to __ATOMIC_RELEASE on the add
// plus an agent acquire fence in the last arriver.
__device__ __forceinline__ bool publish_partial(const float* part_lds, float* slab, unsigned* ctr, int b, int h, int t,
                                                unsigned* last_flag) {
  float* mine = slab + ((long long)b * H + h) * E;
#pragma unroll
  for (int i = 0; i < 3; ++i) __hip_atomic_store(mine + t + 256 * i, part_lds[t + 256 * i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (t == 0) *last_flag = __hip_atomic_fetch_add(&ctr[b], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == (unsigned)(H - 1);
  __syncthreads();
  return *last_flag != 0;
}
// the 12 partials of element n of row b, summed in head order
__device__ __forceinline__ float gather_partials(const float* slab, int b, int n) {
  float s = 0.f;
  const float* src = slab + (long long)b * H * E + n;
#pragma unroll
  for (int j = 0; j < H; ++j) s += __hip_atomic_load(src + j * E, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  return s;
}

struct KvP {
  const bf16* k1;   // video segment: row (b / bdiv1) * stride1 + j * ld (K at +0, V at +v_off)
  long long stride1, ld1;
  int bdiv1, lk1;
  const bf16* k2;   // text segment (NULL: none)
  long long stride2, ld2;
  int bdiv2, lk2;
  long long v_off;  // V = K + v_off (elements)
};
// the memory rows of one (b, h): two uniform segment bases (scalar registers), then a per-lane select
// — a per-lane choice between the parameter struct's fields would make hipcc fetch them with vector
// loads and drain vmcnt(0) (every bulk load in flight) before each use
// K / V images in LDS: row j (64 bf16 = 8 chunks of 16 B) with chunk c stored at chunk c ^ (j & 7),
// so a wave reading one 16-B chunk of 64 different rows spreads over every bank (the rows are 128 B
// apart: unswizzled, all 64 lanes hit the same two bank groups)
__device__ __forceinline__ int kv_swz(int j, int c) { return j * D + ((c ^ (j & 7)) << 3); }
__device__ __forceinline__ float kv_at(const bf16* img, int j, int d) { return bf2f(img[kv_swz(j, d >> 3) + (d & 7)]); }

struct KvRows {
  const bf16* base1;
  const bf16* base2;
  long long ld1, ld2;
  int lk1;
};
__device__ __forceinline__ KvRows kv_rows(const KvP& kv, int b, int h) {
  KvRows r;
  r.base1 = kv.k1 + (long long)(b / kv.bdiv1) * kv.stride1 + h * D;
  r.base2 = kv.k2 ? kv.k2 + (long long)(b / kv.bdiv2) * kv.stride2 + h * D : r.base1;
  r.ld1 = kv.ld1;
  r.ld2 = kv.ld2;
  r.lk1 = kv.lk1;
  return r;
}
__device__ __forceinline__ const bf16* kv_row(const KvRows& r, int j) {
  return j < r.lk1 ? r.base1 + (long long)j * r.ld1 : r.base2 + (long long)(j - r.lk1) * r.ld2;
}

}  // namespace
