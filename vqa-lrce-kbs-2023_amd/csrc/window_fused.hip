// Fused QKV projection + 3D shifted-window attention forward for Video Swin
// (WindowAttention3D.forward, video_swin_ori.py:158-189: qkv Linear -> q scale -> QK^T -> + rel-pos
// bias (+ shift mask) -> softmax -> PV) on gfx950.
//
// One workgroup = one window (n <= 160 tokens, 147 = 3x7x7) x a PAIR of heads, 8 waves, 66 KB of
// LDS, so two workgroups share a CU: while one streams its GEMM operands the other runs its
// attention (the phases of one workgroup are serial; two resident workgroups overlap them).
//  1. GEMM  [160 tokens x C] . [C x 192]^T  (the q, k, v rows of W_qkv for the 2 heads), BK = 32,
//     both operands K-major, staged L2 -> LDS by LDS-DMA (global_load_lds_dwordx4, 1 KB = 16 rows x
//     64 B per wave instruction, source-side XOR swizzle chunk ^ ((row >> 1) & 3): conflict-free
//     ds_read_b128 fragment reads), a ring of three stages: two K tiles in flight while one is
//     consumed (one in flight left the GEMM bound by the L2 -> LDS latency); v_mfma_f32_16x16x32_bf16,
//     wave grid 2 (tokens) x 4 (columns), 80 x 48 per wave.
//  2. Epilogue: + bias, q * head_dim^-0.5 * log2(e), bf16, into per-head LDS images [160][32]
//     (the GEMM stages are free by then); the first attention unit's bias tile loads are already in
//     flight.  The qkv rows the backward reads are then stored FROM the images, 16 B per lane, whole
//     128-B row segments (q | k | v of the head pair are contiguous in each part).
//  3. Attention per (head, 32-query tile) unit, 10 units over the 8 waves: S^T = K Q^T started from
//     the pre-combined bias + mask tile (fp16, log2 domain) one key tile at a time with an online
//     softmax (running max / sum, O rescaled: 16 S registers live instead of 80), O^T = V^T P^T with P^T
//     from the accumulators; O parked in the unit's own (consumed) Q rows, then stored as whole
//     128-B row segments with 16-B lanes; the row log-sum-exp.
// Windows are visited in mask-pattern order (win_order): the workgroups the dispatcher deals to one
// XCD then share few patterns, so their bias tiles (plus W_qkv and the window's x rows, re-read by
// every head pair) stay in that XCD's 4 MB L2.
// This is the kernel bench.py's roofline reports: with the QKV projection in it the intensity of
// what it reads (the window's LN1 rows, the W_qkv slice, the bias tiles) passes the bf16 ridge at
// C >= 512 (stages 3-4).
#include "common.h"
#include "lrce_capi.h"

namespace {

constexpr int HD = 32;          // head dim
constexpr int HB = 2;           // heads per workgroup
constexpr int TQ = 32;          // attention tile edge
constexpr int NTILE = 5;        // 160 / 32
constexpr int NPAD = 160;
constexpr int NW = 8;           // waves
constexpr int BK = 32;          // GEMM K tile
constexpr int ROWB = BK * 2;    // bytes per staged operand row
constexpr int AROWS = NPAD;     // token rows of the A image
constexpr int BROWS = 3 * HB * HD;                 // 192 weight rows: q | k | v of the 2 heads
constexpr int STG = (AROWS + BROWS) * ROWB;        // bytes per GEMM stage (22 KB)
constexpr int APIECES = AROWS / 16, PIECES = (AROWS + BROWS) / 16;   // 1-KB LDS-DMA pieces (10, 22)
constexpr int PPW = (PIECES + NW - 1) / NW;        // pieces per wave, at most (3)
constexpr int NS = 3;                              // GEMM ring stages (two K tiles in flight)
constexpr int IMG = NPAD * HD;                     // bf16 elements of one head image
constexpr int IMG_BYTES = 3 * HB * IMG * 2;        // 60 KB: the head images (alias the GEMM ring)
constexpr int LDS_BYTES = NS * STG > IMG_BYTES ? NS * STG : IMG_BYTES;   // 66 KB: two workgroups per CU
constexpr int TILE_ELEMS = 64 * 16;
constexpr int PH_ELEMS = NTILE * NTILE * TILE_ELEMS;
static_assert(PIECES <= NW * PPW && PIECES > NW * (PPW - 1), "piece split");

// K-major operand image: byte offset of (row, 16-B chunk c) — rows of 64 B, chunk c ^ ((row >> 1) & 3)
__device__ __forceinline__ int opnd(int row, int c) { return row * ROWB + ((c ^ ((row >> 1) & 3)) << 4); }
// per-head attention images [160][32] bf16: Q and K chunk-swizzled for conflict-free row reads, V plain
__device__ __forceinline__ int qk_off(int row, int d) { return row * HD + ((((d >> 3) ^ ((row >> 2) & 3))) << 3) + (d & 7); }
__device__ __forceinline__ int crow(int reg, int h) { return (reg & 3) + 8 * (reg >> 2) + 4 * h; }

__device__ __forceinline__ void glds_s(const void* sbase, uint32_t voff, uint32_t lds_dst) {
  unsigned keep;
  const uint64_t a = reinterpret_cast<uintptr_t>(sbase);
  const uint64_t su = (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)a) |
                      ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)(a >> 32)) << 32);
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, %2\n\ts_mov_b32 m0, %0"
               : "=&s"(keep) : "v"(voff), "s"(su), "s"(__builtin_amdgcn_readfirstlane(lds_dst)) : "memory");
}
__device__ __forceinline__ uint32_t lds_addr(const void* p) { return (uint32_t)(uintptr_t)((LRCE_LDS const void*)p); }

// Workgroup barrier for LDS hand-offs only: __syncthreads() also drains vmcnt(0), i.e. waits for the
// attention's bias-tile loads and the qkv / O row stores still in flight.
__device__ __forceinline__ void lds_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

// element j = img[r_base + 8*(j>>2) + 4*hh + (j&3)][lane & 31] of a plain [rows][32] image: the
// A operand of O^T = V^T P^T in the accumulators' permuted key order (window_attn.hip)
__device__ __forceinline__ bf16x8 tr_read_perm(const bf16* img, int r_base, int lane) {
  const int g = lane >> 4, i = lane & 15, q = i >> 2, p = i & 3;
  const int hh = g >> 1, cb = 16 * (g & 1);
  bf16x8 out;
#pragma unroll
  for (int h2 = 0; h2 < 2; ++h2) {
    const int row = r_base + 8 * h2 + 4 * hh + q;
    const LRCE_LDS s16x4* src = (const LRCE_LDS s16x4*)(img + row * 32 + cb + 4 * p);
    s16x4 v = __builtin_amdgcn_ds_read_tr16_b64_v4i16(const_cast<LRCE_LDS s16x4*>(src));
    bf16x4 b = *reinterpret_cast<bf16x4*>(&v);
    out[4 * h2 + 0] = b[0]; out[4 * h2 + 1] = b[1]; out[4 * h2 + 2] = b[2]; out[4 * h2 + 3] = b[3];
  }
  return out;
}
__device__ __forceinline__ bf16x8 pack8(const f32x16& a, int s) {
  bf16x8 o;
#pragma unroll
  for (int j = 0; j < 8; ++j) o[j] = f2bf(a[8 * s + j]);
  return o;
}

struct FusedP {
  const bf16* x;        // LN1 output, window-ordered rows [n_win * n][C]
  const bf16* w;        // W_qkv [3C][C]
  const float* b;       // b_qkv [3C]
  const uint2* biasf;   // pre-combined bias + mask tiles, fp16 (lrce_wattn_bias_build, forward layout)
  const int* win_pat;   // window -> mask pattern (NULL: pattern 0)
  const int* win_order; // visiting order of the windows (NULL: identity)
  bf16* qkv;            // [n_win * n][3C] (q pre-scaled), for the backward
  bf16* out;            // [n_win * n][C]
  float* lse;           // [n_win][nH][160], log2 domain
  float qscale;         // head_dim^-0.5 * log2(e)
  int n_win, n, nH, C;
  unsigned long long* trace;   // phase timestamps (builds with -DLRCE_WATTN_TRACE only; lrce_wattn_set_trace)
};

// debug phase marks: thread 0 of each workgroup stamps s_memrealtime (100 MHz) into trace[wg * 16 + i]
#ifdef LRCE_WATTN_TRACE
#define WF_MARK(I) \
  if (p.trace && threadIdx.x == 0) p.trace[(long long)blockIdx.x * 16 + (I)] = __builtin_amdgcn_s_memrealtime();
#else
#define WF_MARK(I)
#endif

// the 20 fp16x4 bias loads of one attention unit: bias row of query tile qt, key tiles 0..4
__device__ __forceinline__ void bias_load(const FusedP& p, int pat, int h, int qt, int lane, uint2 (&bv)[NTILE][4]) {
  const uint2* src = p.biasf + ((long long)(pat * p.nH + h) * PH_ELEMS + (long long)qt * NTILE * TILE_ELEMS) / 4 + lane;
#pragma unroll
  for (int kt = 0; kt < NTILE; ++kt)
#pragma unroll
    for (int v = 0; v < 4; ++v) bv[kt][v] = src[kt * (TILE_ELEMS / 4) + 64 * v];
}
__device__ __forceinline__ float h16lo(unsigned u) { return (float)__builtin_bit_cast(f16, (unsigned short)(u & 0xFFFFu)); }
__device__ __forceinline__ float h16hi(unsigned u) { return (float)__builtin_bit_cast(f16, (unsigned short)(u >> 16)); }

__global__ void __launch_bounds__(NW * 64, 4) wattn_qkv_fwd_kernel(FusedP p) {
  __shared__ __attribute__((aligned(16))) char lds_raw[LDS_BYTES];   // GEMM stages; later the head images
  bf16* lds = reinterpret_cast<bf16*>(lds_raw);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int ngrp = p.nH / HB;
  const int lin = xcd_remap(blockIdx.x, gridDim.x);   // a window's head pairs on one XCD (shared x rows)
  const int hg = lin % ngrp, slot = lin / ngrp;
  const int w = p.win_order ? p.win_order[slot] : slot;
  const int C = p.C, n = p.n;
  const long long ld3 = 3LL * C;
  const bf16* xwin = p.x + (long long)w * n * C;
  const int pat = p.win_pat ? p.win_pat[w] : 0;
  WF_MARK(0)
#ifdef LRCE_WATTN_TRACE
  if (p.trace && threadIdx.x == 0) {   // placement: HW_ID (cu / sh / se) and XCC_ID
    p.trace[(long long)blockIdx.x * 16 + 10] = __builtin_amdgcn_s_getreg(4 | (31 << 11));
    p.trace[(long long)blockIdx.x * 16 + 11] = __builtin_amdgcn_s_getreg(20 | (31 << 11));
  }
#endif

  // ---- 1. GEMM: acc[i][j][r] = Y[tok = wm*80 + i*16 + (lane&15)][col = wn*48 + j*16 + 4*(lane>>4) + r]
  const int wm = wave >> 2, wn = wave & 3;
  constexpr int IM = 5, JN = 3;
  // the qkv bias of this lane's epilogue columns, loaded first: issued after the attention's bias-tile
  // loads it would wait behind them (in-order vmcnt) — 3.3 us of epilogue per workgroup in the trace
  float4 bqkv[JN];
#pragma unroll
  for (int j = 0; j < JN; ++j) {
    const int col = wn * 48 + j * 16 + 4 * (lane >> 4);
    bqkv[j] = *reinterpret_cast<const float4*>(p.b + (col / (HB * HD)) * C + hg * (HB * HD) + (col % (HB * HD)));
  }
  f32x4 acc[IM][JN];
#pragma unroll
  for (int i = 0; i < IM; ++i)
#pragma unroll
    for (int j = 0; j < JN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // DMA pieces of this wave: piece e = wave + NW * q (q < PPW, e < PIECES); e < APIECES: token rows
  // 16e..16e+15, else weight rows; lane i fills image row 16e + i/4, stored chunk i%4
  const int wave_u = __builtin_amdgcn_readfirstlane(wave);
  const int mine = wave_u + NW * (PPW - 1) < PIECES ? PPW : PPW - 1;
  const void* sbase[PPW];
  uint32_t voff[PPW], ldoff[PPW];
#pragma unroll
  for (int q = 0; q < PPW; ++q) {
    const int e = wave_u + NW * q < PIECES ? wave_u + NW * q : 0;
    const int r = 16 * e + (lane >> 2);                // image row
    const int c = (lane & 3) ^ ((r >> 1) & 3);         // logical 16-B chunk this lane fetches
    if (e < APIECES) {
      const int tok = r < n ? r : n - 1;               // padded rows: any valid row (never stored)
      sbase[q] = xwin;
      voff[q] = (uint32_t)(((long long)tok * C + c * 8) * 2);
    } else {
      const int wr = r - AROWS;                        // 0..191: part (q|k|v), head of the pair, dim
      const int wrow = (wr / (HB * HD)) * C + hg * (HB * HD) + (wr % (HB * HD));
      sbase[q] = p.w;
      voff[q] = (uint32_t)(((long long)wrow * C + c * 8) * 2);
    }
    ldoff[q] = (uint32_t)(e * 1024);
  }
  const uint32_t lbase = lds_addr(lds_raw);
  auto issue = [&](int kt, int stage) {
#pragma unroll
    for (int q = 0; q < PPW; ++q)
      if (q < mine)
        glds_s(static_cast<const char*>(sbase[q]) + kt * BK * 2, voff[q], lbase + (uint32_t)(stage * STG) + ldoff[q]);
  };
  auto compute = [&](const char* stage) {
    bf16x8 af[IM], bfr[JN];
#pragma unroll
    for (int i = 0; i < IM; ++i)
      af[i] = *reinterpret_cast<const bf16x8*>(stage + opnd(wm * 80 + i * 16 + (lane & 15), lane >> 4));
#pragma unroll
    for (int j = 0; j < JN; ++j)
      bfr[j] = *reinterpret_cast<const bf16x8*>(stage + opnd(AROWS + wn * 48 + j * 16 + (lane & 15), lane >> 4));
#pragma unroll
    for (int i = 0; i < IM; ++i)
#pragma unroll
      for (int j = 0; j < JN; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bfr[j], af[i], acc[i][j], 0, 0, 0);
  };
  // ring of NS stages, one barrier per K tile: wait for this wave's pieces of tile kt, barrier (every
  // wave's pieces landed, every wave done with tile kt-1 whose stage the next issue refills), issue
  // tile kt+NS-1, compute tile kt — NS-1 tiles in flight behind the one being consumed
  const int nk = C / BK;
#pragma unroll
  for (int t = 0; t < NS - 1; ++t)
    if (t < nk) issue(t, t);
  for (int kt = 0; kt < nk; ++kt) {
    const int ahead = min(nk - 1 - kt, NS - 2);        // tiles issued after kt and not yet waited for
    if (mine == PPW) {
      if (ahead >= 1) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(PPW) : "memory");
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    } else {
      if (ahead >= 1) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(PPW - 1) : "memory");
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // this wave's reads of tile kt-1 are done
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    if (kt + NS - 1 < nk) issue(kt + NS - 1, (kt + NS - 1) % NS);
    compute(lds_raw + (kt % NS) * STG);
    __builtin_amdgcn_sched_barrier(0);
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();                                      // ring free: the images alias it
  __builtin_amdgcn_sched_barrier(0);
  WF_MARK(1)

  const int hh = lane >> 5, r32 = lane & 31;
  uint2 bv[NTILE][4];
  {
    const int u = wave;
    bias_load(p, pat, hg * HB + u / NTILE, u % NTILE, lane, bv);
  }

  // ---- 2. epilogue: bias, q scale, bf16 -> per-head images img(part, head) = lds + (part*HB + head)*IMG
#pragma unroll
  for (int j = 0; j < JN; ++j) {
    const int col = wn * 48 + j * 16 + 4 * (lane >> 4);   // 4 consecutive columns, one head
    const int part = col / (HB * HD), hl = (col % (HB * HD)) / HD, d = col % HD;
    const float4 bb = bqkv[j];
    const float sc = part == 0 ? p.qscale : 1.0f;
    bf16* img = lds + (part * HB + hl) * IMG;
#pragma unroll
    for (int i = 0; i < IM; ++i) {
      const int tok = wm * 80 + i * 16 + (lane & 15);
      bf16x4 v;
      v[0] = f2bf((acc[i][j][0] + bb.x) * sc); v[1] = f2bf((acc[i][j][1] + bb.y) * sc);
      v[2] = f2bf((acc[i][j][2] + bb.z) * sc); v[3] = f2bf((acc[i][j][3] + bb.w) * sc);
      const int off = part == 2 ? tok * HD + d : qk_off(tok, d);
      *reinterpret_cast<bf16x4*>(img + off) = v;
    }
  }
  lds_barrier();
  WF_MARK(2)
  // qkv rows for the backward: per token and part, the head pair's 64 columns = 128 contiguous bytes
  for (int it = threadIdx.x; it < n * 3 * 8; it += NW * 64) {
    const int c8 = it & 7, tp = it >> 3;
    const int part = tp % 3, tok = tp / 3;
    const int hl = c8 >> 2, c4 = c8 & 3;
    const bf16* img = lds + (part * HB + hl) * IMG;
    const int off = part == 2 ? tok * HD + c4 * 8 : qk_off(tok, c4 * 8);
    const uint4 v = *reinterpret_cast<const uint4*>(img + off);
    *reinterpret_cast<uint4*>(p.qkv + ((long long)w * n + tok) * ld3 + part * C + hg * (HB * HD) + c8 * 8) = v;
  }
  lds_barrier();   // the Q rows are read by the stores above before a unit parks its O in them
  WF_MARK(3)

  // ---- 3. attention: unit u = (head hl, query tile qt), u = wave, wave + 8 (< 10)
  for (int u = wave; u < HB * NTILE; u += NW) {
    const int hl = u / NTILE, qt = u % NTILE;
    const int h = hg * HB + hl;
    if (u != wave) bias_load(p, pat, h, qt, lane, bv);
    bf16* qimg = lds + (0 * HB + hl) * IMG;
    const bf16* kimg = lds + (1 * HB + hl) * IMG;
    const bf16* vimg = lds + (2 * HB + hl) * IMG;
    const int qi = qt * TQ + r32;
    bf16x8 qf[2];
#pragma unroll
    for (int s = 0; s < 2; ++s) qf[s] = *reinterpret_cast<const bf16x8*>(qimg + qk_off(qi, 16 * s + 8 * hh));
    // S^T = K Q~^T + bias one key tile at a time (rows = keys, query on the lane), online softmax:
    // running max m (shared by the two lane halves), running sum, O^T rescaled when m grows
    float m = -1.0e30f, sum = 0.f;
    f32x16 o = {};
#pragma unroll
    for (int kt = 0; kt < NTILE; ++kt) {
      f32x16 sc;
#pragma unroll
      for (int v = 0; v < 4; ++v) {
        sc[4 * v] = h16lo(bv[kt][v].x); sc[4 * v + 1] = h16hi(bv[kt][v].x);
        sc[4 * v + 2] = h16lo(bv[kt][v].y); sc[4 * v + 3] = h16hi(bv[kt][v].y);
      }
      const int key = kt * TQ + r32;
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        const bf16x8 kf = *reinterpret_cast<const bf16x8*>(kimg + qk_off(key, 16 * s + 8 * hh));
        sc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(kf, qf[s], sc, 0, 0, 0);
      }
      float mt = sc[0];
#pragma unroll
      for (int r = 1; r < 16; ++r) mt = fmaxf(mt, sc[r]);
      mt = fmaxf(mt, __shfl_xor(mt, 32, 64));
      const float mn = fmaxf(m, mt);
      const float corr = __builtin_amdgcn_exp2f(m - mn);
      m = mn;
      sum *= corr;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        o[r] *= corr;
        sc[r] = __builtin_amdgcn_exp2f(sc[r] - m);
        sum += sc[r];
      }
      o = __builtin_amdgcn_mfma_f32_32x32x16_bf16(tr_read_perm(vimg, kt * TQ, lane), pack8(sc, 0), o, 0, 0, 0);
      o = __builtin_amdgcn_mfma_f32_32x32x16_bf16(tr_read_perm(vimg, kt * TQ + 16, lane), pack8(sc, 1), o, 0, 0, 0);
    }
    sum += __shfl_xor(sum, 32, 64);
    // O^T: rows = head dims 8 rr + 4 hh + e, query qi on the lane -> park in this unit's Q rows
    const float inv = 1.0f / sum;
#pragma unroll
    for (int rr = 0; rr < 4; ++rr) {
      bf16x4 v;
      v[0] = f2bf(o[4 * rr] * inv); v[1] = f2bf(o[4 * rr + 1] * inv);
      v[2] = f2bf(o[4 * rr + 2] * inv); v[3] = f2bf(o[4 * rr + 3] * inv);
      *reinterpret_cast<bf16x4*>(qimg + qk_off(qi, 8 * rr + 4 * hh)) = v;
    }
    if (hh == 0 && qi < n) p.lse[((long long)w * p.nH + h) * NPAD + qi] = m + __log2f(sum);
  }
  lds_barrier();
  WF_MARK(4)
  // O rows: per token the head pair's 64 columns = 128 contiguous bytes
  for (int it = threadIdx.x; it < n * 8; it += NW * 64) {
    const int c8 = it & 7, tok = it >> 3;
    const int hl = c8 >> 2, c4 = c8 & 3;
    const uint4 v = *reinterpret_cast<const uint4*>(lds + hl * IMG + qk_off(tok, c4 * 8));
    *reinterpret_cast<uint4*>(p.out + ((long long)w * n + tok) * C + hg * (HB * HD) + c8 * 8) = v;
  }
#ifdef LRCE_WATTN_TRACE
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  WF_MARK(5)
#endif
}

}  // namespace

extern unsigned long long* g_wattn_trace;   // window_attn.hip, lrce_wattn_set_trace

extern "C" int lrce_wattn_qkv_fwd(const uint16_t* x, const uint16_t* w_qkv, const float* b_qkv, float qscale,
                                  const uint16_t* bias_fwd16, const int32_t* win_pat, const int32_t* win_order,
                                  uint16_t* qkv, uint16_t* out, float* lse, int n_win, int n, int nH, void* stream) {
  if (!x || !w_qkv || !b_qkv || !bias_fwd16 || !qkv || !out || !lse) return lrce_fail(LRCE_E_ARG, "wattn_qkv_fwd: null pointer");
  if (n <= 4 * TQ || n > NPAD) return lrce_fail(LRCE_E_ARG, "wattn_qkv_fwd: n=%d outside (128,160]", n);
  if (nH < HB || nH % HB) return lrce_fail(LRCE_E_ARG, "wattn_qkv_fwd: nH=%d not a multiple of %d", nH, HB);
  const int C = nH * HD;
  auto al16 = [](const void* q) { return (reinterpret_cast<uintptr_t>(q) & 15) == 0; };
  if (!al16(x) || !al16(w_qkv) || !al16(b_qkv) || !al16(qkv) || !al16(out) || !al16(bias_fwd16))
    return lrce_fail(LRCE_E_ARG, "wattn_qkv_fwd: operands must be 16-B aligned");
  // 32-bit DMA offsets: the window's rows and the weight matrix must stay below 2 GB
  if ((long long)n * C * 2 >= (1LL << 31) || 3LL * C * C * 2 >= (1LL << 31)) return lrce_fail(LRCE_E_ARG, "wattn_qkv_fwd: too large");
  if (n_win <= 0) return LRCE_OK;
  FusedP p;
  p.x = reinterpret_cast<const bf16*>(x);
  p.w = reinterpret_cast<const bf16*>(w_qkv);
  p.b = b_qkv;
  p.biasf = reinterpret_cast<const uint2*>(bias_fwd16);
  p.win_pat = win_pat;
  p.win_order = win_order;
  p.qkv = reinterpret_cast<bf16*>(qkv);
  p.out = reinterpret_cast<bf16*>(out);
  p.lse = lse;
  p.qscale = qscale;
  p.n_win = n_win; p.n = n; p.nH = nH; p.C = C;
  p.trace = g_wattn_trace;
  wattn_qkv_fwd_kernel<<<(unsigned)(n_win * (nH / HB)), NW * 64, 0, static_cast<hipStream_t>(stream)>>>(p);
  return lrce_check_launch("wattn_qkv_fwd");
}
