// Recurrent LRCE decoder, per-head fused attention blocks (nn.TransformerDecoderLayer, post-norm,
// 768 wide, 12 heads x 64, one query token per batch row: fusionv3.py:8-17,44-49) on gfx950.
//
// The recurrent step is a chain of M = B (10..45) row linears: every launch boundary on it costs a
// dependent round trip (~2 us measured, tools/decoder_probe.hip) on top of the ~1.9 us launch, and the
// GPU is otherwise idle there.  Both attention blocks of a layer factor by head, so each becomes ONE
// launch of B x 12 workgroups, workgroup (b, h) doing the head's share of every linear:
//
//   self-attention (one key: softmax == 1, so out_proj(drop_head(v_proj(x0)))):
//     x0 = [LN3 of the previous layer](x_in)                  (row b, recomputed by every head)
//     v_h = W_v[h] x0 + b_v[h]    (64 x 768 slice, weight rows in registers)
//     sad_h = drop_head(v_h)      (mask per (b, h): the group-64 dropout of lrce_dropout)
//     part_h = W_o[:, h] sad_h    (768 x 64 slice, staged in LDS by LDS-DMA at kernel start)
//     x1p = x0 + drop(sum_h part_h + b_o)          (the last of the 12 heads to arrive sums in h order)
//   cross-attention:
//     x1 = LN1(x1p); q_h = W_q[h] x1 + b_q[h]; ctx_h = attn(q_h, memory K/V of head h) (dropout on P)
//     x2p = x1 + drop(sum_h W_oc[:, h] ctx_h + b_oc)
// and the backward of each block is one launch the same way (LN backward of the block's output
// gradient recomputed per head; dctx_h / dsav_h from the W_o slice; mha backward; the dX partials
// W_q[h]^T dq_h / W_v[h]^T dsav_h summed by the last head).  The FFN keeps its two lrce_gemm_ln /
// lrce_gemm launches (its 3072-wide hidden layer does not factor by head).
//
// Cross-workgroup hand-off: MI355X_MICROARCH.md "splitk-seam" / the skinny split-K of gemm_f32.hip:
// partial rows by agent-scope relaxed stores, s_waitcnt vmcnt(0), barrier, one agent-scope atomic add
// per workgroup on a per-row counter; the workgroup whose add returns 11 reads the 12 partials with
// agent-scope loads in head order (deterministic) and resets the counter (graph-replay safe).
// Weights are the decoder's IEEE fp16 shadow (the reference's fp16 autocast), arithmetic f32.
// Dropout masks are the ones the unfused path draws (lrce_dropout hash over the same [B][768] index,
// mha dropout over ((b*12 + h) * Lk + j)), so forward and backward agree with each other and with it.
#include "common.h"
#include "decoder_util.h"
#include "lrce_capi.h"

namespace {
unsigned long long* g_dec_trace_host = nullptr;

// ------------------------------------------------------------------ self-attention block forward
struct SaFwdP {
  int B;
  const float* x_in;              // [B][768]: s or the previous layer's pre-norm x3p
  const float* ln_g;              // previous layer's norm3 (NULL: x0 = x_in)
  const float* ln_b;
  float eps;
  float* x0_out;                  // LN output (when ln_g), [B][768]
  float* mean_out;
  float* rstd_out;
  const f16* wv;                  // W_v rows [768][768] (in_proj rows 2E..3E)
  const float* bv;
  const f16* wo;                  // out_proj [768][768]
  const float* bo;
  float* sad;                     // [B][768] dropped v (the out_proj's input, for its weight gradient)
  float* x1p;                     // [B][768]
  float p;
  uint64_t seed;                  // layer seed: head mask seed, out dropout seed + 1
  const uint64_t* rng_off;
  float* slab;
  unsigned* ctr;
  unsigned long long* trace;
};

struct SaFwdLds {
  f16 wo[E * D];                  // 96 KB
  float x0[E];
  float pp[4][16 * 64];
  alignas(16) float v[D];
  float part[E];
  float red2[4];
  unsigned last;
};

__global__ void __launch_bounds__(NT, 1) dec_sa_fwd_kernel(SaFwdP p) {
  __shared__ __attribute__((aligned(16))) SaFwdLds L;
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int b = blockIdx.x / H, h = blockIdx.x % H;
  DEC_MARK(0, 0);
  // everything that depends on nothing: the row, the W_v rows, the W_o slice (DMA)
  float4 xr = make_float4(0.f, 0.f, 0.f, 0.f), gg = xr, be = xr;
  if (t < E / 4) {
    xr = *reinterpret_cast<const float4*>(p.x_in + (long long)b * E + 4 * t);
    if (p.ln_g) {
      gg = *reinterpret_cast<const float4*>(p.ln_g + 4 * t);
      be = *reinterpret_cast<const float4*>(p.ln_b + 4 * t);
    }
  }
  // the row first (its statistics start right away: the asm pins the sum, and so the wait for the
  // row, here), then the bulk loads: W_v rows into registers, the W_o slice by DMA (last: the
  // compiler's in-order vmcnt waits do not count the DMAs)
  const uint64_t roff = rng_off_now(p.rng_off);
  pin(xr);
  pin(gg);
  pin(be);
  const float s1l = row_sum_local(xr, t);
  asm volatile("" ::"v"(s1l));
  __builtin_amdgcn_sched_barrier(0);
  uint4 wr[NRI];
  rows_load(p.wv, h * D + wave * WROWS, lane, wr);
  const float bvv = t < D ? p.bv[h * D + t] : 0.f;
  slice_dma(p.wo, h, L.wo, wave, lane);
  __builtin_amdgcn_sched_barrier(0);
  if (p.ln_g) {
    float mu, rs;
    ln_row_fwd(xr, s1l, gg, be, p.eps, L.x0, L.red2, t, lane, wave, mu, rs);
    if (h == 0) {
      if (t < E / 4) *reinterpret_cast<float4*>(p.x0_out + (long long)b * E + 4 * t) = *reinterpret_cast<const float4*>(L.x0 + 4 * t);
      if (t == 0) {
        p.mean_out[b] = mu;
        p.rstd_out[b] = rs;
      }
    }
  } else if (t < E / 4) {
    *reinterpret_cast<float4*>(L.x0 + 4 * t) = xr;
  }
  lds_barrier();
  DEC_MARK(0, 1);
  // v = W_v[h] x0 + b_v ; head dropout
  rows_gemv(wr, L.x0, L.pp[wave], L.v + wave * WROWS, lane);
  lds_barrier();
  DEC_MARK(0, 2);
  const uint64_t seed0 = p.seed + roff;
  if (t < D) {
    float v = L.v[t] + bvv;
    if (p.p > 0.f) v = drop1(v, p.p, seed0, ((long long)b * E + h * D + t) / D);
    L.v[t] = v;
    p.sad[(long long)b * E + h * D + t] = v;
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // this wave's slice DMA has landed
  lds_barrier();                                    // ... and every wave's; L.v complete
  DEC_MARK(0, 3);
  slice_gemv(L.wo, L.v, L.part, t);
  lds_barrier();
  DEC_MARK(0, 4);
  const bool last_sa = publish_partial(L.part, p.slab, p.ctr, b, h, t, &L.last);
  DEC_MARK(0, 5);
  if (!last_sa) return;
  const uint64_t seed1 = p.seed + 1 + roff;
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    const int n = t + 256 * i;
    float y = gather_partials(p.slab, b, n) + p.bo[n];
    if (p.p > 0.f) y = drop1(y, p.p, seed1, (long long)b * E + n);
    p.x1p[(long long)b * E + n] = L.x0[n] + y;
  }
  if (t == 0) __hip_atomic_store(&p.ctr[b], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  DEC_MARK(0, 6);
}

// ------------------------------------------------------------------ cross-attention block forward
struct CaFwdP {
  int B;
  const float* x1p;               // [B][768]
  const float* g1;                // norm1
  const float* b1;
  float eps;
  float* x1_out;                  // [B][768] (h == 0)
  float* mean_out;
  float* rstd_out;
  const f16* wq;                  // in_proj rows 0..E
  const float* bq;
  KvP kv;
  float* q_out;                   // [B][768] f32 (the backward's q)
  float* ctx_out;                 // [B][768]
  float* lse_out;                 // [B][12]
  const f16* wo;                  // out_proj [768][768]
  const float* bo;
  float* x2p;                     // [B][768]
  float p;
  uint64_t seed;                  // attention dropout seed (seed + 2 of the layer); out dropout seed + 1
  const uint64_t* rng_off;
  float* slab;
  unsigned* ctr;
  unsigned long long* trace;
};

struct CaFwdLds {
  f16 wo[E * D];
  bf16 vimg[MAXK * D];            // V rows of the head (24 KB)
  float x1[E];
  float pp[4][16 * 64];
  float q[D];
  float ps[MAXK + 64];
  float opart[4][D];
  alignas(16) float ctx[D];
  float part[E];
  float red2[4];
  unsigned last;
};

__global__ void __launch_bounds__(NT, 1) dec_ca_fwd_kernel(CaFwdP p) {
  __shared__ __attribute__((aligned(16))) CaFwdLds L;
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int b = blockIdx.x / H, h = blockIdx.x % H;
  const int Lk = p.kv.lk1 + p.kv.lk2;
  DEC_MARK(1, 0);
  float4 xr = make_float4(0.f, 0.f, 0.f, 0.f), gg = xr, be = xr;
  if (t < E / 4) {
    xr = *reinterpret_cast<const float4*>(p.x1p + (long long)b * E + 4 * t);
    gg = *reinterpret_cast<const float4*>(p.g1 + 4 * t);
    be = *reinterpret_cast<const float4*>(p.b1 + 4 * t);
  }
  const uint64_t roff = rng_off_now(p.rng_off);
  pin(xr);
  pin(gg);
  pin(be);
  const float s1l = row_sum_local(xr, t);
  asm volatile("" ::"v"(s1l));
  __builtin_amdgcn_sched_barrier(0);
  DEC_MARK(1, 9);
  // key row of thread t (registers; needed first, after q), the W_q rows, then the DMAs: the head's V
  // rows (LDS, 8 rows per instruction) and the W_o slice
  const bool live = t < Lk;
  const KvRows kvr = kv_rows(p.kv, b, h);
  uint4 kr[8];
  {
    const bf16* kp = kv_row(kvr, live ? t : 0);
#pragma unroll
    for (int c = 0; c < 8; ++c) kr[c] = *reinterpret_cast<const uint4*>(kp + 8 * c);
  }
  uint4 wr[NRI];
  rows_load(p.wq, h * D + wave * WROWS, lane, wr);
  const float bqv = t < D ? p.bq[h * D + t] : 0.f;
  __builtin_amdgcn_sched_barrier(0);
  DEC_MARK(1, 10);
  // LN1 while those land; the DMAs (needed last) are issued after it: a wave holds at most 63
  // vector-memory operations in flight, and issuing all of them first stalled the LN behind them
  float mu, rs;
  ln_row_fwd(xr, s1l, gg, be, p.eps, L.x1, L.red2, t, lane, wave, mu, rs);
  __builtin_amdgcn_sched_barrier(0);
  {
    const uint32_t vb = dec_lds_addr(L.vimg);
    for (int ins = wave; ins * 8 < Lk; ins += 4) {
      const int r = ins * 8 + (lane >> 3), j = min(r, Lk - 1);
      const bf16* vp = kv_row(kvr, j) + p.kv.v_off + (((lane & 7) ^ (r & 7)) << 3);
      dec_glds_p(vp, vb + (uint32_t)ins * 1024u);
    }
  }
  slice_dma(p.wo, h, L.wo, wave, lane);
  __builtin_amdgcn_sched_barrier(0);
  if (h == 0) {
    if (t < E / 4) *reinterpret_cast<float4*>(p.x1_out + (long long)b * E + 4 * t) = *reinterpret_cast<const float4*>(L.x1 + 4 * t);
    if (t == 0) {
      p.mean_out[b] = mu;
      p.rstd_out[b] = rs;
    }
  }
  lds_barrier();
  DEC_MARK(1, 1);
  rows_gemv(wr, L.x1, L.pp[wave], L.q + wave * WROWS, lane);
  lds_barrier();
  DEC_MARK(1, 2);
  if (t < D) {
    const float q = L.q[t] + bqv;
    p.q_out[(long long)b * E + h * D + t] = q;
    L.q[t] = q * 0.125f;   // head_dim^-0.5
  }
  lds_barrier();
  // scores, softmax (natural log), dropout on the probabilities
  float sc = 0.f;
  if (live) {
#pragma unroll
    for (int c = 0; c < 8; ++c) {
      const unsigned w4[4] = {kr[c].x, kr[c].y, kr[c].z, kr[c].w};
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        sc += bfbits2f((unsigned short)(w4[e] & 0xFFFFu)) * L.q[8 * c + 2 * e];
        sc += bfbits2f((unsigned short)(w4[e] >> 16)) * L.q[8 * c + 2 * e + 1];
      }
    }
  }
  const float m = block_max4(live ? sc : -1.0e30f, L.red2, lane, wave);
  const float pe = live ? __expf(sc - m) : 0.f;
  const float s = block_sum4(pe, L.red2, lane, wave);
  const uint64_t seed2 = p.seed + roff;
  float pf = pe;
  if (live && p.p > 0.f) pf = drop1(pe, p.p, seed2, ((long long)b * H + h) * Lk + t);
  L.ps[t] = live ? pf : 0.f;
  DEC_MARK(1, 3);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // V rows and the W_o slice have landed
  lds_barrier();
  DEC_MARK(1, 4);
  // ctx = sum_j p_j V_j / s: thread (key group kg = t / 8 of 32, 8-dim chunk c = t % 8) sums keys
  // j = kg, kg + 32, ... with 16-B row reads, then the 8 key groups of a wave (DPP / shuffles) and the
  // 4 waves (LDS)
  {
    const int c = t & 7, kg = t >> 3;
    float a[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll 2
    for (int j = kg; j < Lk; j += 32) {
      float vf[8];
      unpack8bf(*reinterpret_cast<const uint4*>(L.vimg + kv_swz(j, c)), vf);
      const float pj = L.ps[j];
#pragma unroll
      for (int e = 0; e < 8; ++e) a[e] = fmaf(pj, vf[e], a[e]);
    }
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      a[e] += dpp_f<0x128>(a[e]);   // row_ror:8 -> key groups g, g^1
      a[e] += __shfl_xor(a[e], 16, 64);
      a[e] += __shfl_xor(a[e], 32, 64);
    }
    if (lane < 8) {
#pragma unroll
      for (int e = 0; e < 8; ++e) L.opart[wave][c * 8 + e] = a[e];
    }
  }
  lds_barrier();
  if (t < D) {
    const float c = ((L.opart[0][t] + L.opart[1][t]) + (L.opart[2][t] + L.opart[3][t])) / s;
    L.ctx[t] = c;
    p.ctx_out[(long long)b * E + h * D + t] = c;
    if (t == 0) p.lse_out[(long long)b * H + h] = m + __logf(s);
  }
  lds_barrier();
  DEC_MARK(1, 5);
  slice_gemv(L.wo, L.ctx, L.part, t);
  lds_barrier();
  DEC_MARK(1, 6);
  const bool last_ca = publish_partial(L.part, p.slab, p.ctr, b, h, t, &L.last);
  DEC_MARK(1, 7);
  if (!last_ca) return;
  const uint64_t seed3 = p.seed + 1 + roff;
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    const int n = t + 256 * i;
    float y = gather_partials(p.slab, b, n) + p.bo[n];
    if (p.p > 0.f) y = drop1(y, p.p, seed3, (long long)b * E + n);
    p.x2p[(long long)b * E + n] = L.x1[n] + y;
  }
  if (t == 0) __hip_atomic_store(&p.ctr[b], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  DEC_MARK(1, 8);
}

// ------------------------------------------------------------------ cross-attention block backward
struct CaBwdP {
  int B;
  const float* dx2;               // [B][768] gradient of x2 = LN2(x2p)
  const float* x2p;
  const float* mean2;
  const float* rstd2;
  const float* g2;
  float* dcao_out;                // [B][768] dropout_bwd(dx2p): the out_proj's output gradient (h == 0)
  const f16* wo;                  // out_proj [768][768]
  KvP kv;
  const float* q;                 // [B][768] (unscaled)
  const float* ctx;               // [B][768]
  const float* lse;               // [B][12]
  float* dq_out;                  // [B][768]
  float* dk1;                     // video dK (dV at + dv_off): row (b/bdiv1)*dstride1 + j*dld1
  long long dstride1, dld1;
  int dkv1_atomic;                // rows shared by bdiv1 > 1 query rows: atomics, else stores
  float* dk2;                     // text dK, accumulated (one writer per row), or stored (dk2_store)
  int dk2_store;
  bf16* dk1_16;                   // non-null: the video rows' dK / dV stored as bf16 here instead of dk1
  long long dstride2, dld2;
  long long dv_off;
  const f16* wq;                  // in_proj rows 0..E
  float* dx1_out;                 // [B][768] = dx2p + W_q^T dq
  float p;
  uint64_t seed;                  // layer seed + 2 (attention dropout); + 1 = the out dropout (seed + 3)
  const uint64_t* rng_off;
  float* slab;
  unsigned* ctr;
  unsigned long long* trace;
};

struct CaBwdLds {
  f16 wo[E * D];
  union {
    bf16 kimg[MAXK * D];          // K rows of the head (dead once dq / dK / dV are done)
    float acc[4][E];              // then: per-wave dX partials
  };
  bf16 vimg[MAXK * D];
  float dx2p[E];
  float dcao[E];
  float red64[4][D];
  float dctx[D];
  float q[D];
  float dq[D];
  float ps[MAXK + 64];
  float dss[MAXK + 64];
  float red2[4];
  unsigned last;
};

__global__ void __launch_bounds__(NT, 1) dec_ca_bwd_kernel(CaBwdP p) {
  __shared__ __attribute__((aligned(16))) CaBwdLds L;
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int b = blockIdx.x / H, h = blockIdx.x % H;
  const int Lk = p.kv.lk1 + p.kv.lk2;
  DEC_MARK(2, 0);
  float4 dy = make_float4(0.f, 0.f, 0.f, 0.f), xr = dy, gm = dy;
  if (t < E / 4) {
    dy = *reinterpret_cast<const float4*>(p.dx2 + (long long)b * E + 4 * t);
    xr = *reinterpret_cast<const float4*>(p.x2p + (long long)b * E + 4 * t);
    gm = *reinterpret_cast<const float4*>(p.g2 + 4 * t);
  }
  const float mu = p.mean2[b], rs = p.rstd2[b];
  const uint64_t roff = rng_off_now(p.rng_off);
  LnBwdLocal lnl = ln_row_bwd_local(dy, xr, gm, mu, rs, t);
  pin(lnl.g);
  pin(lnl.xh);
  asm volatile("" : "+v"(lnl.s1), "+v"(lnl.s2));
  __builtin_amdgcn_sched_barrier(0);
  DEC_MARK(2, 9);
  uint4 wr[NRI];
  rows_load(p.wq, h * D + wave * WROWS, lane, wr);
  float qd = 0.f, od = 0.f;
  if (t < D) {
    qd = p.q[(long long)b * E + h * D + t];
    od = p.ctx[(long long)b * E + h * D + t];
  }
  const float lse = p.lse[(long long)b * H + h];
  const KvRows kvr = kv_rows(p.kv, b, h);
  // the text rows' running dK / dV (accumulated over the recurrent steps), read now as (key, 8-dim
  // chunk) items and added at the end
  const long long tbase = (long long)(b / p.kv.bdiv2) * p.dstride2 + h * D;
  float4 told[TXI][4];
#pragma unroll
  for (int i = 0; i < TXI; ++i) {
    const int e = t + 256 * i, tj = e >> 3, c = e & 7;
    told[i][0] = told[i][1] = told[i][2] = told[i][3] = make_float4(0.f, 0.f, 0.f, 0.f);
    if (tj < p.kv.lk2 && !p.dk2_store) {
      const float* src = p.dk2 + tbase + (long long)tj * p.dld2 + c * 8;
      told[i][0] = *reinterpret_cast<const float4*>(src);
      told[i][1] = *reinterpret_cast<const float4*>(src + 4);
      told[i][2] = *reinterpret_cast<const float4*>(src + p.dv_off);
      told[i][3] = *reinterpret_cast<const float4*>(src + p.dv_off + 4);
    }
  }
  __builtin_amdgcn_sched_barrier(0);
  DEC_MARK(2, 10);
  // LN2 backward while those land; the DMAs (needed after it) are issued next: a wave holds at most
  // 63 vector-memory operations in flight
  const float4 dx = ln_row_bwd(lnl, rs, L.red2, lane, wave);
  __builtin_amdgcn_sched_barrier(0);
  DEC_MARK(2, 11);
  {
    const uint32_t kb = dec_lds_addr(L.kimg), vb = dec_lds_addr(L.vimg);
    for (int ins = wave; ins * 8 < Lk; ins += 4) {
      const int r = ins * 8 + (lane >> 3), j = min(r, Lk - 1);
      const bf16* kp = kv_row(kvr, j) + (((lane & 7) ^ (r & 7)) << 3);
      dec_glds_p(kp, kb + (uint32_t)ins * 1024u);
      dec_glds_p(kp + p.kv.v_off, vb + (uint32_t)ins * 1024u);
    }
  }
  slice_dma(p.wo, h, L.wo, wave, lane);
  __builtin_amdgcn_sched_barrier(0);
  // the out dropout's backward (seed + 3 of the layer = p.seed + 1)
  const uint64_t seed3 = p.seed + 1 + roff;
  if (t < E / 4) {
    *reinterpret_cast<float4*>(L.dx2p + 4 * t) = dx;
    float4 d = dx;
    if (p.p > 0.f) {
      const long long e = (long long)b * E + 4 * t;
      d = make_float4(drop1(dx.x, p.p, seed3, e), drop1(dx.y, p.p, seed3, e + 1), drop1(dx.z, p.p, seed3, e + 2),
                      drop1(dx.w, p.p, seed3, e + 3));
    }
    *reinterpret_cast<float4*>(L.dcao + 4 * t) = d;
    if (h == 0) *reinterpret_cast<float4*>(p.dcao_out + (long long)b * E + 4 * t) = d;
  }
  if (t < D) L.q[t] = qd * 0.125f;
  DEC_MARK(2, 1);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  lds_barrier();
  DEC_MARK(2, 2);
  // dctx = W_o[:, h]^T dcao
  slice_gemv_t(L.wo, L.dcao, &L.red64[0][0], wave, lane);
  lds_barrier();
  DEC_MARK(2, 3);
  float dod = 0.f;
  if (t < D) {
    dod = (L.red64[0][t] + L.red64[1][t]) + (L.red64[2][t] + L.red64[3][t]);
    L.dctx[t] = dod;
  }
  const float delta = block_sum4(dod * od, L.red2, lane, wave);   // also publishes L.q / L.dctx
  // per key: P, dropout factor, dP, dS
  const bool live = t < Lk;
  float pf = 0.f, ds = 0.f;
  if (live) {
    float sc = 0.f, dp = 0.f;
#pragma unroll
    for (int c = 0; c < 8; ++c) {
      const uint4 ku = *reinterpret_cast<const uint4*>(L.kimg + kv_swz(t, c));
      const uint4 vu = *reinterpret_cast<const uint4*>(L.vimg + kv_swz(t, c));
      const unsigned k4[4] = {ku.x, ku.y, ku.z, ku.w}, v4[4] = {vu.x, vu.y, vu.z, vu.w};
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        sc += bfbits2f((unsigned short)(k4[e] & 0xFFFFu)) * L.q[8 * c + 2 * e] +
              bfbits2f((unsigned short)(k4[e] >> 16)) * L.q[8 * c + 2 * e + 1];
        dp += bfbits2f((unsigned short)(v4[e] & 0xFFFFu)) * L.dctx[8 * c + 2 * e] +
              bfbits2f((unsigned short)(v4[e] >> 16)) * L.dctx[8 * c + 2 * e + 1];
      }
    }
    const float pr = __expf(sc - lse);
    float f = 1.f;
    if (p.p > 0.f) f = lrce_uniform(p.seed + roff, (uint64_t)(((long long)b * H + h) * Lk + t)) >= p.p
                           ? 1.0f / (1.0f - p.p) : 0.f;
    pf = pr * f;
    ds = pr * (f * dp - delta);
  }
  L.ps[t] = pf;
  L.dss[t] = ds;
  lds_barrier();
  DEC_MARK(2, 4);
  // dq: lane = head dim, wave w sums keys j = w, w + 4, ...
  {
    float dq0 = 0.f, dq1 = 0.f;
    int j = wave;
    for (; j + 4 < Lk; j += 8) {
      dq0 += L.dss[j] * kv_at(L.kimg, j, lane);
      dq1 += L.dss[j + 4] * kv_at(L.kimg, j + 4, lane);
    }
    if (j < Lk) dq0 += L.dss[j] * kv_at(L.kimg, j, lane);
    L.red64[wave][lane] = dq0 + dq1;
  }
  // dK = dS q~, dV = (P * dropout) dO as (key, 8-dim chunk) items: 16-B stores (video rows: one writer,
  // stored; shared by bdiv1 > 1 MC choices: atomics), text rows: the prefetched sums + this step's
  {
    const long long vbase = (long long)(b / p.kv.bdiv1) * p.dstride1 + h * D;
    for (int e = t; e < p.kv.lk1 * 8; e += 256) {
      const int j = e >> 3, c = e & 7;
      const float dsj = L.dss[j], pj = L.ps[j];
      float kv8[16];
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        kv8[i] = dsj * L.q[c * 8 + i];
        kv8[8 + i] = pj * L.dctx[c * 8 + i];
      }
      if (p.dk1_16) {   // bf16 directly: the memory-side GEMMs' operand (same rounding as a later cast)
        bf16* d16 = p.dk1_16 + vbase + (long long)j * p.dld1 + c * 8;
        bf16x8 k16, v16;
#pragma unroll
        for (int i = 0; i < 8; ++i) { k16[i] = f2bf(kv8[i]); v16[i] = f2bf(kv8[8 + i]); }
        *reinterpret_cast<bf16x8*>(d16) = k16;
        *reinterpret_cast<bf16x8*>(d16 + p.dv_off) = v16;
        continue;
      }
      float* dst = p.dk1 + vbase + (long long)j * p.dld1 + c * 8;
      if (p.dkv1_atomic) {
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          __hip_atomic_fetch_add(dst + i, kv8[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          __hip_atomic_fetch_add(dst + p.dv_off + i, kv8[8 + i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
      } else {
        *reinterpret_cast<float4*>(dst) = make_float4(kv8[0], kv8[1], kv8[2], kv8[3]);
        *reinterpret_cast<float4*>(dst + 4) = make_float4(kv8[4], kv8[5], kv8[6], kv8[7]);
        *reinterpret_cast<float4*>(dst + p.dv_off) = make_float4(kv8[8], kv8[9], kv8[10], kv8[11]);
        *reinterpret_cast<float4*>(dst + p.dv_off + 4) = make_float4(kv8[12], kv8[13], kv8[14], kv8[15]);
      }
    }
#pragma unroll
    for (int i = 0; i < TXI; ++i) {
      const int e = t + 256 * i, tj = e >> 3, c = e & 7;
      if (tj < p.kv.lk2) {
        const int j = p.kv.lk1 + tj;
        const float dsj = L.dss[j], pj = L.ps[j];
        const float* qv = L.q + c * 8;
        const float* gv = L.dctx + c * 8;
        float* dst = p.dk2 + tbase + (long long)tj * p.dld2 + c * 8;
        const float4 a0 = told[i][0], a1 = told[i][1], a2 = told[i][2], a3 = told[i][3];
        *reinterpret_cast<float4*>(dst) =
            make_float4(a0.x + dsj * qv[0], a0.y + dsj * qv[1], a0.z + dsj * qv[2], a0.w + dsj * qv[3]);
        *reinterpret_cast<float4*>(dst + 4) =
            make_float4(a1.x + dsj * qv[4], a1.y + dsj * qv[5], a1.z + dsj * qv[6], a1.w + dsj * qv[7]);
        *reinterpret_cast<float4*>(dst + p.dv_off) =
            make_float4(a2.x + pj * gv[0], a2.y + pj * gv[1], a2.z + pj * gv[2], a2.w + pj * gv[3]);
        *reinterpret_cast<float4*>(dst + p.dv_off + 4) =
            make_float4(a3.x + pj * gv[4], a3.y + pj * gv[5], a3.z + pj * gv[6], a3.w + pj * gv[7]);
      }
    }
  }
  lds_barrier();
  if (t < D) {
    const float dq = ((L.red64[0][t] + L.red64[1][t]) + (L.red64[2][t] + L.red64[3][t])) * 0.125f;
    L.dq[t] = dq;
    p.dq_out[(long long)b * E + h * D + t] = dq;
  }
  lds_barrier();
  DEC_MARK(2, 5);
  // dx1 partial = W_q[h]^T dq
  rows_gemv_t(wr, L.dq + wave * WROWS, L.acc[wave], lane);
  lds_barrier();
  float* part = &L.acc[0][0];
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    const int n = t + 256 * i;
    part[n] = (L.acc[0][n] + L.acc[1][n]) + (L.acc[2][n] + L.acc[3][n]);
  }
  lds_barrier();
  DEC_MARK(2, 6);
  const bool last_cb = publish_partial(part, p.slab, p.ctr, b, h, t, &L.last);
  DEC_MARK(2, 7);
  if (!last_cb) return;
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    const int n = t + 256 * i;
    p.dx1_out[(long long)b * E + n] = L.dx2p[n] + gather_partials(p.slab, b, n);
  }
  if (t == 0) __hip_atomic_store(&p.ctr[b], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  DEC_MARK(2, 8);
}

// ------------------------------------------------------------------ self-attention block backward
struct SaBwdP {
  int B;
  const float* dx1;               // [B][768] gradient of x1 = LN1(x1p)
  const float* x1p;
  const float* mean1;
  const float* rstd1;
  const float* g1;
  float* dsao_out;                // [B][768] out_proj output gradient (h == 0)
  const f16* wo;                  // out_proj
  float* dsav_out;                // [B][768] v_proj output gradient (after the head mask)
  const f16* wv;                  // in_proj rows 2E..3E
  float* dx0_out;                 // [B][768] = dx1p + W_v^T dsav
  float p;
  uint64_t seed;                  // layer seed (head mask); + 1 = out dropout
  const uint64_t* rng_off;
  float* slab;
  unsigned* ctr;
  unsigned long long* trace;
};

struct SaBwdLds {
  f16 wo[E * D];
  float dx1p[E];
  float dsao[E];
  float red64[4][D];
  float dsav[D];
  float acc[4][E];
  float red2[4];
  unsigned last;
};

__global__ void __launch_bounds__(NT, 1) dec_sa_bwd_kernel(SaBwdP p) {
  __shared__ __attribute__((aligned(16))) SaBwdLds L;
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int b = blockIdx.x / H, h = blockIdx.x % H;
  DEC_MARK(3, 0);
  float4 dy = make_float4(0.f, 0.f, 0.f, 0.f), xr = dy, gm = dy;
  if (t < E / 4) {
    dy = *reinterpret_cast<const float4*>(p.dx1 + (long long)b * E + 4 * t);
    xr = *reinterpret_cast<const float4*>(p.x1p + (long long)b * E + 4 * t);
    gm = *reinterpret_cast<const float4*>(p.g1 + 4 * t);
  }
  const float mu = p.mean1[b], rs = p.rstd1[b];
  const uint64_t roff = rng_off_now(p.rng_off);
  LnBwdLocal lnl = ln_row_bwd_local(dy, xr, gm, mu, rs, t);
  pin(lnl.g);
  pin(lnl.xh);
  asm volatile("" : "+v"(lnl.s1), "+v"(lnl.s2));
  __builtin_amdgcn_sched_barrier(0);
  uint4 wr[NRI];
  rows_load(p.wv, h * D + wave * WROWS, lane, wr);
  slice_dma(p.wo, h, L.wo, wave, lane);
  __builtin_amdgcn_sched_barrier(0);
  const float4 dx = ln_row_bwd(lnl, rs, L.red2, lane, wave);
  const uint64_t seed1 = p.seed + 1 + roff;
  if (t < E / 4) {
    *reinterpret_cast<float4*>(L.dx1p + 4 * t) = dx;
    float4 d = dx;
    if (p.p > 0.f) {
      const long long e = (long long)b * E + 4 * t;
      d = make_float4(drop1(dx.x, p.p, seed1, e), drop1(dx.y, p.p, seed1, e + 1), drop1(dx.z, p.p, seed1, e + 2),
                      drop1(dx.w, p.p, seed1, e + 3));
    }
    *reinterpret_cast<float4*>(L.dsao + 4 * t) = d;
    if (h == 0) *reinterpret_cast<float4*>(p.dsao_out + (long long)b * E + 4 * t) = d;
  }
  DEC_MARK(3, 1);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  lds_barrier();
  DEC_MARK(3, 2);
  slice_gemv_t(L.wo, L.dsao, &L.red64[0][0], wave, lane);
  lds_barrier();
  if (t < D) {
    float v = (L.red64[0][t] + L.red64[1][t]) + (L.red64[2][t] + L.red64[3][t]);
    if (p.p > 0.f) v = drop1(v, p.p, p.seed + roff, ((long long)b * E + h * D + t) / D);
    L.dsav[t] = v;
    p.dsav_out[(long long)b * E + h * D + t] = v;
  }
  lds_barrier();
  rows_gemv_t(wr, L.dsav + wave * WROWS, L.acc[wave], lane);
  lds_barrier();
  float* part = &L.acc[0][0];
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    const int n = t + 256 * i;
    part[n] = (L.acc[0][n] + L.acc[1][n]) + (L.acc[2][n] + L.acc[3][n]);
  }
  lds_barrier();
  DEC_MARK(3, 3);
  const bool last_sb = publish_partial(part, p.slab, p.ctr, b, h, t, &L.last);
  DEC_MARK(3, 4);
  if (!last_sb) return;
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    const int n = t + 256 * i;
    p.dx0_out[(long long)b * E + n] = L.dx1p[n] + gather_partials(p.slab, b, n);
  }
  if (t == 0) __hip_atomic_store(&p.ctr[b], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  DEC_MARK(3, 5);
}

// ------------------------------------------------------------------ deferred LayerNorm parameter grads
// dgamma[c] += sum_r dy[r][c] (x[r][c] - mean[r]) rstd[r],  dbeta[c] += sum_r dy[r][c]  over the R = S*B
// rows of every recurrent step (one owner per column, rows in order: deterministic).  blockIdx.y picks
// one of up to 3 LayerNorms; a NULL dgamma or dbeta (frozen parameter) is skipped.
struct LnGradP {
  const float* dy[3];
  const float* x[3];
  const float* mean[3];
  const float* rstd[3];
  float* dgamma[3];
  float* dbeta[3];
  int rows;
};
// Workgroup (column block of 64, LayerNorm k): wave w sums rows w, w+4, ... of its lane's column with
// 8 rows of loads in flight, then the four wave sums are added in a fixed order (deterministic).
// (One thread per column looping over all S x B rows made the launch a chain of dependent round
// trips: 15.7 us for 3 x 256 threads.)
__global__ void __launch_bounds__(256) dec_ln_grads_kernel(LnGradP p) {
  constexpr int U = 8;
  __shared__ float red[2][4][64];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + lane, k = blockIdx.y;
  if (!p.dy[k]) return;   // uniform over the workgroup
  const float* dy = p.dy[k] + c;
  const float* x = p.x[k] + c;
  float sg = 0.f, sb = 0.f;
  int r = wave;
  for (; r + 4 * (U - 1) < p.rows; r += 4 * U) {
    float d[U], xv[U], mu[U], rs[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int rr = r + 4 * u;
      d[u] = dy[(long long)rr * E];
      xv[u] = x[(long long)rr * E];
      mu[u] = p.mean[k][rr];
      rs[u] = p.rstd[k][rr];
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      sg += d[u] * (xv[u] - mu[u]) * rs[u];
      sb += d[u];
    }
  }
  for (; r < p.rows; r += 4) {
    const float d = dy[(long long)r * E];
    sg += d * (x[(long long)r * E] - p.mean[k][r]) * p.rstd[k][r];
    sb += d;
  }
  red[0][wave][lane] = sg;
  red[1][wave][lane] = sb;
  __syncthreads();
  if (wave == 0) {
    const float g = (red[0][0][lane] + red[0][1][lane]) + (red[0][2][lane] + red[0][3][lane]);
    const float b = (red[1][0][lane] + red[1][1][lane]) + (red[1][2][lane] + red[1][3][lane]);
    if (p.dgamma[k]) p.dgamma[k][c] += g;
    if (p.dbeta[k]) p.dbeta[k][c] += b;
  }
}

template <typename P>
int launch(void (*kern)(P), const P& prm, int B, hipStream_t st, const char* what) {
  kern<<<(unsigned)(B * H), NT, 0, st>>>(prm);
  return lrce_check_launch(what);
}

bool al16(const void* q) { return (reinterpret_cast<uintptr_t>(q) & 15) == 0; }

}  // namespace

extern "C" int64_t lrce_dec_slab_elems(int B) { return (int64_t)B * H * E; }

extern "C" int lrce_dec_sa_fwd(const LrceDecSa* a, void* stream) {
  if (!a || !a->x_in || !a->wv || !a->bv || !a->wo || !a->bo || !a->sad || !a->x1p || !a->slab || !a->counters)
    return lrce_fail(LRCE_E_ARG, "dec_sa_fwd: null pointer");
  if (a->B < 1 || a->B > LRCE_DEC_MAX_ROWS) return lrce_fail(LRCE_E_ARG, "dec_sa_fwd: B=%d outside [1, %d]", a->B, LRCE_DEC_MAX_ROWS);
  if (a->ln_gamma && (!a->ln_beta || !a->x0_out || !a->mean_out || !a->rstd_out))
    return lrce_fail(LRCE_E_ARG, "dec_sa_fwd: the input LayerNorm needs beta, x0_out, mean_out, rstd_out");
  if (!al16(a->x_in) || !al16(a->wv) || !al16(a->wo) || (a->x0_out && !al16(a->x0_out)) || !al16(a->x1p))
    return lrce_fail(LRCE_E_ARG, "dec_sa_fwd: rows and weights need 16-B alignment");
  SaFwdP p;
  p.B = a->B; p.x_in = a->x_in; p.ln_g = a->ln_gamma; p.ln_b = a->ln_beta; p.eps = a->eps;
  p.x0_out = a->x0_out; p.mean_out = a->mean_out; p.rstd_out = a->rstd_out;
  p.wv = reinterpret_cast<const f16*>(a->wv); p.bv = a->bv; p.wo = reinterpret_cast<const f16*>(a->wo); p.bo = a->bo;
  p.sad = a->sad; p.x1p = a->x1p; p.p = a->drop_p; p.seed = a->seed; p.rng_off = lrce_rng_offset();
  p.slab = a->slab; p.ctr = a->counters; p.trace = g_dec_trace_host;
  return launch(dec_sa_fwd_kernel, p, a->B, static_cast<hipStream_t>(stream), "dec_sa_fwd");
}

static int kv_check(const LrceDecKv& kv, const char* what) {
  if (!kv.k1 || kv.lk1 < 1 || kv.bdiv1 < 1 || (kv.lk2 > 0 && (!kv.k2 || kv.bdiv2 < 1)) || kv.lk1 + kv.lk2 > MAXK ||
      kv.lk2 > MAXTXT)
    return lrce_fail(LRCE_E_ARG, "%s: memory segments (lk1=%d, lk2=%d <= %d, max %d keys)", what, kv.lk1, kv.lk2, MAXTXT, MAXK);
  if (!al16(kv.k1) || (kv.k2 && !al16(kv.k2)) || (kv.ld1 % 8) || (kv.stride1 % 8) || (kv.lk2 > 0 && ((kv.ld2 % 8) || (kv.stride2 % 8))) ||
      (kv.v_off % 8))
    return lrce_fail(LRCE_E_ARG, "%s: K/V rows need 16-B alignment", what);
  return LRCE_OK;
}
static KvP kv_conv(const LrceDecKv& a) {
  KvP k;
  k.k1 = reinterpret_cast<const bf16*>(a.k1); k.stride1 = a.stride1; k.ld1 = a.ld1; k.bdiv1 = a.bdiv1; k.lk1 = a.lk1;
  k.k2 = reinterpret_cast<const bf16*>(a.k2); k.stride2 = a.stride2; k.ld2 = a.ld2; k.bdiv2 = a.bdiv2 > 0 ? a.bdiv2 : 1;
  k.lk2 = a.lk2 > 0 ? a.lk2 : 0; k.v_off = a.v_off;
  return k;
}

extern "C" int lrce_dec_ca_fwd(const LrceDecCa* a, void* stream) {
  if (!a || !a->x1p || !a->g1 || !a->b1 || !a->x1_out || !a->mean_out || !a->rstd_out || !a->wq || !a->bq || !a->q_out ||
      !a->ctx_out || !a->lse_out || !a->wo || !a->bo || !a->x2p || !a->slab || !a->counters)
    return lrce_fail(LRCE_E_ARG, "dec_ca_fwd: null pointer");
  if (a->B < 1 || a->B > LRCE_DEC_MAX_ROWS) return lrce_fail(LRCE_E_ARG, "dec_ca_fwd: B=%d", a->B);
  if (int rc = kv_check(a->kv, "dec_ca_fwd")) return rc;
  if (!al16(a->x1p) || !al16(a->x1_out) || !al16(a->wq) || !al16(a->wo)) return lrce_fail(LRCE_E_ARG, "dec_ca_fwd: 16-B alignment");
  CaFwdP p;
  p.B = a->B; p.x1p = a->x1p; p.g1 = a->g1; p.b1 = a->b1; p.eps = a->eps; p.x1_out = a->x1_out;
  p.mean_out = a->mean_out; p.rstd_out = a->rstd_out; p.wq = reinterpret_cast<const f16*>(a->wq); p.bq = a->bq;
  p.kv = kv_conv(a->kv); p.q_out = a->q_out; p.ctx_out = a->ctx_out; p.lse_out = a->lse_out;
  p.wo = reinterpret_cast<const f16*>(a->wo); p.bo = a->bo; p.x2p = a->x2p; p.p = a->drop_p; p.seed = a->seed;
  p.rng_off = lrce_rng_offset(); p.slab = a->slab; p.ctr = a->counters; p.trace = g_dec_trace_host;
  return launch(dec_ca_fwd_kernel, p, a->B, static_cast<hipStream_t>(stream), "dec_ca_fwd");
}

extern "C" int lrce_dec_ca_bwd(const LrceDecCaBwd* a, void* stream) {
  if (!a || !a->dx2 || !a->x2p || !a->mean2 || !a->rstd2 || !a->g2 || !a->dcao_out || !a->wo || !a->q || !a->ctx || !a->lse ||
      !a->dq_out || (!a->dk1 && !a->dk1_bf16) || !a->wq || !a->dx1_out || !a->slab || !a->counters)
    return lrce_fail(LRCE_E_ARG, "dec_ca_bwd: null pointer");
  if (a->dk1_bf16 && (a->kv.bdiv1 > 1 || (reinterpret_cast<uintptr_t>(a->dk1_bf16) & 15) || a->dstride1 % 8 ||
                      a->dld1 % 8 || a->dv_off % 8))
    return lrce_fail(LRCE_E_ARG, "dec_ca_bwd: bf16 dK/dV needs one writer per row (bdiv1 == 1) and 16-B aligned rows");
  if (a->B < 1 || a->B > LRCE_DEC_MAX_ROWS) return lrce_fail(LRCE_E_ARG, "dec_ca_bwd: B=%d", a->B);
  if (int rc = kv_check(a->kv, "dec_ca_bwd")) return rc;
  if (a->kv.lk2 > 0 && !a->dk2) return lrce_fail(LRCE_E_ARG, "dec_ca_bwd: text segment without dk2");
  if (!al16(a->dx2) || !al16(a->x2p) || !al16(a->wq) || !al16(a->wo) || !al16(a->dcao_out))
    return lrce_fail(LRCE_E_ARG, "dec_ca_bwd: 16-B alignment");
  CaBwdP p;
  p.B = a->B; p.dx2 = a->dx2; p.x2p = a->x2p; p.mean2 = a->mean2; p.rstd2 = a->rstd2; p.g2 = a->g2;
  p.dcao_out = a->dcao_out; p.wo = reinterpret_cast<const f16*>(a->wo); p.kv = kv_conv(a->kv); p.q = a->q; p.ctx = a->ctx;
  p.lse = a->lse; p.dq_out = a->dq_out; p.dk1 = a->dk1; p.dstride1 = a->dstride1; p.dld1 = a->dld1;
  p.dkv1_atomic = a->kv.bdiv1 > 1; p.dk2 = a->dk2; p.dk2_store = a->dk2_store; p.dk1_16 = reinterpret_cast<bf16*>(a->dk1_bf16); p.dstride2 = a->dstride2; p.dld2 = a->dld2; p.dv_off = a->dv_off;
  p.wq = reinterpret_cast<const f16*>(a->wq); p.dx1_out = a->dx1_out; p.p = a->drop_p; p.seed = a->seed;
  p.rng_off = lrce_rng_offset(); p.slab = a->slab; p.ctr = a->counters; p.trace = g_dec_trace_host;
  return launch(dec_ca_bwd_kernel, p, a->B, static_cast<hipStream_t>(stream), "dec_ca_bwd");
}

extern "C" int lrce_dec_sa_bwd(const LrceDecSaBwd* a, void* stream) {
  if (!a || !a->dx1 || !a->x1p || !a->mean1 || !a->rstd1 || !a->g1 || !a->dsao_out || !a->wo || !a->dsav_out || !a->wv ||
      !a->dx0_out || !a->slab || !a->counters)
    return lrce_fail(LRCE_E_ARG, "dec_sa_bwd: null pointer");
  if (a->B < 1 || a->B > LRCE_DEC_MAX_ROWS) return lrce_fail(LRCE_E_ARG, "dec_sa_bwd: B=%d", a->B);
  if (!al16(a->dx1) || !al16(a->x1p) || !al16(a->wv) || !al16(a->wo) || !al16(a->dsao_out))
    return lrce_fail(LRCE_E_ARG, "dec_sa_bwd: 16-B alignment");
  SaBwdP p;
  p.B = a->B; p.dx1 = a->dx1; p.x1p = a->x1p; p.mean1 = a->mean1; p.rstd1 = a->rstd1; p.g1 = a->g1;
  p.dsao_out = a->dsao_out; p.wo = reinterpret_cast<const f16*>(a->wo); p.dsav_out = a->dsav_out;
  p.wv = reinterpret_cast<const f16*>(a->wv); p.dx0_out = a->dx0_out; p.p = a->drop_p; p.seed = a->seed;
  p.rng_off = lrce_rng_offset(); p.slab = a->slab; p.ctr = a->counters; p.trace = g_dec_trace_host;
  return launch(dec_sa_bwd_kernel, p, a->B, static_cast<hipStream_t>(stream), "dec_sa_bwd");
}

extern "C" int lrce_dec_ln_grads(const float* const* dy, const float* const* x, const float* const* mean,
                                 const float* const* rstd, float* const* dgamma, float* const* dbeta, int n_ln, int rows,
                                 void* stream) {
  if (n_ln < 1 || n_ln > 3 || rows < 1) return lrce_fail(LRCE_E_ARG, "dec_ln_grads: n_ln=%d rows=%d", n_ln, rows);
  LnGradP p{};
  for (int k = 0; k < n_ln; ++k) {
    if (!dy[k] || !x[k] || !mean[k] || !rstd[k] || (!dgamma[k] && !dbeta[k]))
      return lrce_fail(LRCE_E_ARG, "dec_ln_grads: null pointer (one of dgamma / dbeta may be NULL, not both)");
    p.dy[k] = dy[k]; p.x[k] = x[k]; p.mean[k] = mean[k]; p.rstd[k] = rstd[k]; p.dgamma[k] = dgamma[k]; p.dbeta[k] = dbeta[k];
  }
  p.rows = rows;
  dec_ln_grads_kernel<<<dim3(E / 64, n_ln), 256, 0, static_cast<hipStream_t>(stream)>>>(p);
  return lrce_check_launch("dec_ln_grads");
}

// debug: phase timestamps of the fused decoder kernels into buf (device, >= 4 * 1024 * 16 uint64), NULL = off
extern "C" int lrce_dec_set_trace(uint64_t* buf) {
  g_dec_trace_host = reinterpret_cast<unsigned long long*>(buf);
  return LRCE_OK;
}
