// Fused QKV projection + 3D shifted-window attention forward for Video Swin
// (WindowAttention3D.forward, video_swin_ori.py:158-189: qkv Linear -> q scale -> QK^T -> + rel-pos
// bias (+ shift mask) -> softmax -> PV) on gfx950.
//
// One workgroup = one window (n <= 160 tokens, 147 = 3x7x7) x a group of HB = 4 heads, 8 waves:
//  1. GEMM  [160 tokens x C] . [C x 384]^T  (the q, k, v rows of W_qkv for the 4 heads), BK = 64,
//     both operands K-major, staged HBM/L2 -> LDS by LDS-DMA (global_load_lds_dwordx4, source-side
//     XOR swizzle), two stages, the next K tile in flight while the current one is consumed;
//     v_mfma_f32_16x16x32_bf16, wave grid 2 (tokens) x 4 (columns), 80 x 96 per wave.
//  2. Epilogue: + bias, q * head_dim^-0.5 * log2(e); the bf16 q / k / v rows are stored to HBM (the
//     backward reads them) AND kept in LDS as per-head images (the GEMM stages are free by then).
//  3. Attention per (head, 32-query tile) unit, 20 units over the 8 waves: S^T = K Q^T started from
//     the pre-combined bias + mask tile (log2 domain), in-lane softmax, O^T = V^T P^T with P^T from
//     the accumulators (wattn_fwd3's recipe), 8-B stores of O rows and the row log-sum-exp.
// The attention core alone is HBM-bound (73.5 flop/B, below the 312 flop/B ridge); with the QKV
// projection in the same kernel the intensity of what the kernel reads from HBM (the window's LN1
// rows, the weights from L2) passes the ridge: this is the kernel bench.py's roofline reports.
#include "common.h"
#include "lrce_capi.h"

namespace {

constexpr int HD = 32;          // head dim
constexpr int HB = 4;           // heads per workgroup
constexpr int TQ = 32;          // attention tile edge
constexpr int NTILE = 5;        // 160 / 32
constexpr int NPAD = 160;
constexpr int BKF = 64;         // GEMM K tile
constexpr int AROWS = 192;      // A tile rows in LDS (160 used; 24 DMA pieces so 72 pieces / 8 waves)
constexpr int BROWS = 3 * HB * HD;   // 384 weight rows: q | k | v of the 4 heads
constexpr int A_EL = AROWS * BKF, B_EL = BROWS * BKF, STG = A_EL + B_EL;   // bf16 elements per stage
constexpr int PIECES = (AROWS + BROWS) / 8;   // 1-KB LDS-DMA pieces per stage (72)
constexpr int PPW = PIECES / 8;               // per wave (9)
constexpr int TILE_ELEMS = 64 * 16;
constexpr int PH_ELEMS = NTILE * NTILE * TILE_ELEMS;
constexpr float NEG_BIG = -1.0e30f;
static_assert(PIECES % 8 == 0, "DMA pieces must split over 8 waves");

// K-major LDS image [rows][64] bf16, 16-B chunk kc stored at kc ^ ((row >> 1) & 7) (as gemm.hip)
__device__ __forceinline__ int km(int row, int kc) { return row * BKF + ((kc ^ ((row >> 1) & 7)) << 3); }
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
  const float* biasf;   // pre-combined bias + mask tiles (lrce_wattn_bias_build, forward layout)
  const int* win_pat;   // window -> mask pattern (NULL: pattern 0)
  bf16* qkv;            // [n_win * n][3C] (q pre-scaled), for the backward
  bf16* out;            // [n_win * n][C]
  float* lse;           // [n_win][nH][160], log2 domain
  float qscale;         // head_dim^-0.5 * log2(e)
  int n_win, n, nH, C;
};

__global__ void __launch_bounds__(512, 2) wattn_qkv_fwd_kernel(FusedP p) {
  __shared__ __attribute__((aligned(16))) bf16 lds[2 * STG];   // GEMM stages; later the q/k/v head images
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int ngrp = p.nH / HB;
  const int lin = xcd_remap(blockIdx.x, gridDim.x);   // a window's head groups on one XCD (shared x rows)
  const int hg = lin % ngrp, w = lin / ngrp;
  const int C = p.C, n = p.n;
  const long long ld3 = 3LL * C;
  const bf16* xwin = p.x + (long long)w * n * C;

  // ---- 1. GEMM: acc[i][j][r] = Y[tok = wm*80 + i*16 + (lane&15)][col = wn*96 + j*16 + 4*(lane>>4) + r]
  const int wm = wave >> 2, wn = wave & 3;
  constexpr int IM = 5, JN = 6;
  f32x4 acc[IM][JN];
#pragma unroll
  for (int i = 0; i < IM; ++i)
#pragma unroll
    for (int j = 0; j < JN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // DMA pieces of this wave: piece e = wave * PPW + q; e < 24: A rows 8e..8e+7, else B rows 8(e-24)..
  const int wave_u = __builtin_amdgcn_readfirstlane(wave);
  const void* sbase[PPW];
  uint32_t voff[PPW], ldoff[PPW];
#pragma unroll
  for (int q = 0; q < PPW; ++q) {
    const int e = wave_u * PPW + q;
    const int rl = lane >> 3, pos = lane & 7;
    if (e < AROWS / 8) {
      const int r = e * 8 + rl;
      const int kc = pos ^ ((r >> 1) & 7);
      const int tok = r < n ? r : n - 1;              // padded rows: any valid row (never stored)
      sbase[q] = xwin;
      voff[q] = (uint32_t)(((long long)tok * C + kc * 8) * 2);
      ldoff[q] = (uint32_t)(e * 1024);
    } else {
      const int r = (e - AROWS / 8) * 8 + rl;           // 0..383: part (q|k|v), head, dim
      const int kc = pos ^ ((r >> 1) & 7);
      const int wrow = (r / (HB * HD)) * C + hg * (HB * HD) + (r % (HB * HD));
      sbase[q] = p.w;
      voff[q] = (uint32_t)(((long long)wrow * C + kc * 8) * 2);
      ldoff[q] = (uint32_t)((A_EL + (e - AROWS / 8) * 512) * 2);
    }
  }
  const uint32_t lbase = lds_addr(lds);
  auto issue = [&](int kt, int stage) {
#pragma unroll
    for (int q = 0; q < PPW; ++q)
      glds_s(static_cast<const char*>(sbase[q]) + kt * BKF * 2, voff[q], lbase + (uint32_t)(stage * STG * 2) + ldoff[q]);
  };
  auto compute = [&](const bf16* la, const bf16* lb) {
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      bf16x8 af[IM], bfr[JN];
#pragma unroll
      for (int i = 0; i < IM; ++i)
        af[i] = *reinterpret_cast<const bf16x8*>(la + km(wm * 80 + i * 16 + (lane & 15), ks * 4 + (lane >> 4)));
#pragma unroll
      for (int j = 0; j < JN; ++j)
        bfr[j] = *reinterpret_cast<const bf16x8*>(lb + km(wn * 96 + j * 16 + (lane & 15), ks * 4 + (lane >> 4)));
#pragma unroll
      for (int i = 0; i < IM; ++i)
#pragma unroll
        for (int j = 0; j < JN; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bfr[j], af[i], acc[i][j], 0, 0, 0);
    }
  };
  const int nk = C / BKF;
  issue(0, 0);
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    if (kt + 1 < nk) {
      issue(kt + 1, cur ^ 1);
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(PPW) : "memory");   // tile kt landed (this wave's part)
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __builtin_amdgcn_s_barrier();                                    // ... and every other wave's
    __builtin_amdgcn_sched_barrier(0);
    compute(lds + cur * STG, lds + cur * STG + A_EL);
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();                                    // stage `cur` free
    __builtin_amdgcn_sched_barrier(0);
  }

  // ---- 2. epilogue: bias, q scale, bf16; qkv rows to HBM; per-head images into LDS
  // images: img(part, head) = lds + (part * HB + head) * NPAD * HD
#pragma unroll
  for (int j = 0; j < JN; ++j) {
    const int col = wn * 96 + j * 16 + 4 * (lane >> 4);   // 4 consecutive columns, one head
    const int part = col / (HB * HD), hl = (col % (HB * HD)) / HD, d = col % HD;
    const int gcol = part * C + hg * (HB * HD) + (col % (HB * HD));
    const float4 bb = *reinterpret_cast<const float4*>(p.b + gcol);
    const float sc = part == 0 ? p.qscale : 1.0f;
    bf16* img = lds + (part * HB + hl) * NPAD * HD;
#pragma unroll
    for (int i = 0; i < IM; ++i) {
      const int tok = wm * 80 + i * 16 + (lane & 15);
      bf16x4 v;
      v[0] = f2bf((acc[i][j][0] + bb.x) * sc); v[1] = f2bf((acc[i][j][1] + bb.y) * sc);
      v[2] = f2bf((acc[i][j][2] + bb.z) * sc); v[3] = f2bf((acc[i][j][3] + bb.w) * sc);
      if (tok < n) *reinterpret_cast<bf16x4*>(p.qkv + ((long long)w * n + tok) * ld3 + gcol) = v;
      const int off = part == 2 ? tok * HD + d : qk_off(tok, d);
      *reinterpret_cast<bf16x4*>(img + off) = v;
    }
  }
  __syncthreads();

  // ---- 3. attention: unit u = (head hl, query tile qt), u = wave, wave + 8, wave + 16 (< 20)
  const int hh = lane >> 5, r32 = lane & 31;
  const int pat = p.win_pat ? p.win_pat[w] : 0;
  for (int u = wave; u < HB * NTILE; u += 8) {
    const int hl = u / NTILE, qt = u % NTILE;
    if (qt * TQ >= n) continue;
    const int h = hg * HB + hl;
    const bf16* qimg = lds + (0 * HB + hl) * NPAD * HD;
    const bf16* kimg = lds + (1 * HB + hl) * NPAD * HD;
    const bf16* vimg = lds + (2 * HB + hl) * NPAD * HD;
    f32x16 sacc[NTILE];
    {
      const float4* src = reinterpret_cast<const float4*>(p.biasf + (long long)(pat * p.nH + h) * PH_ELEMS +
                                                          (long long)qt * NTILE * TILE_ELEMS) + lane;
#pragma unroll
      for (int kt = 0; kt < NTILE; ++kt)
#pragma unroll
        for (int v = 0; v < 4; ++v) {
          const float4 b = src[kt * (TILE_ELEMS / 4) + 64 * v];
          sacc[kt][4 * v] = b.x; sacc[kt][4 * v + 1] = b.y; sacc[kt][4 * v + 2] = b.z; sacc[kt][4 * v + 3] = b.w;
        }
    }
    const int qi = qt * TQ + r32;
    bf16x8 qf[2];
#pragma unroll
    for (int s = 0; s < 2; ++s) qf[s] = *reinterpret_cast<const bf16x8*>(qimg + qk_off(qi, 16 * s + 8 * hh));
    // S^T = K Q~^T + bias: rows = keys, query on the lane
#pragma unroll
    for (int kt = 0; kt < NTILE; ++kt) {
      const int key = kt * TQ + r32;
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        const bf16x8 kf = *reinterpret_cast<const bf16x8*>(kimg + qk_off(key, 16 * s + 8 * hh));
        sacc[kt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(kf, qf[s], sacc[kt], 0, 0, 0);
      }
    }
    float m = NEG_BIG;
#pragma unroll
    for (int kt = 0; kt < NTILE; ++kt)
#pragma unroll
      for (int r = 0; r < 16; ++r) m = fmaxf(m, sacc[kt][r]);
    m = fmaxf(m, __shfl_xor(m, 32, 64));
    float sum = 0.f;
#pragma unroll
    for (int kt = 0; kt < NTILE; ++kt)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const float e = __builtin_amdgcn_exp2f(sacc[kt][r] - m);
        sacc[kt][r] = e;
        sum += e;
      }
    sum += __shfl_xor(sum, 32, 64);
    f32x16 o0 = {}, o1 = {};
#pragma unroll
    for (int kt = 0; kt < NTILE; ++kt) {
      o0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(tr_read_perm(vimg, kt * TQ, lane), pack8(sacc[kt], 0), o0, 0, 0, 0);
      o1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(tr_read_perm(vimg, kt * TQ + 16, lane), pack8(sacc[kt], 1), o1, 0, 0, 0);
    }
    if (qi < n) {
      const f32x16 o = o0 + o1;
      const float inv = 1.0f / sum;
      bf16* dst = p.out + ((long long)w * n + qi) * C + h * HD + 4 * hh;
#pragma unroll
      for (int rr = 0; rr < 4; ++rr) {
        bf16x4 v;
        v[0] = f2bf(o[4 * rr] * inv); v[1] = f2bf(o[4 * rr + 1] * inv);
        v[2] = f2bf(o[4 * rr + 2] * inv); v[3] = f2bf(o[4 * rr + 3] * inv);
        *reinterpret_cast<bf16x4*>(dst + 8 * rr) = v;
      }
      if (hh == 0) p.lse[((long long)w * p.nH + h) * NPAD + qi] = m + __log2f(sum);
    }
  }
}

}  // namespace

extern "C" int lrce_wattn_qkv_fwd(const uint16_t* x, const uint16_t* w_qkv, const float* b_qkv, float qscale,
                                  const float* bias_fwd, const int32_t* win_pat, uint16_t* qkv, uint16_t* out, float* lse,
                                  int n_win, int n, int nH, void* stream) {
  if (!x || !w_qkv || !b_qkv || !bias_fwd || !qkv || !out || !lse) return lrce_fail(LRCE_E_ARG, "wattn_qkv_fwd: null pointer");
  if (n <= 4 * TQ || n > NPAD) return lrce_fail(LRCE_E_ARG, "wattn_qkv_fwd: n=%d outside (128,160]", n);
  if (nH < HB || nH % HB) return lrce_fail(LRCE_E_ARG, "wattn_qkv_fwd: nH=%d not a multiple of %d", nH, HB);
  const int C = nH * HD;
  if (C % BKF) return lrce_fail(LRCE_E_ARG, "wattn_qkv_fwd: C=%d not a multiple of %d", C, BKF);
  auto al16 = [](const void* q) { return (reinterpret_cast<uintptr_t>(q) & 15) == 0; };
  if (!al16(x) || !al16(w_qkv) || !al16(b_qkv) || !al16(qkv) || !al16(out))
    return lrce_fail(LRCE_E_ARG, "wattn_qkv_fwd: operands must be 16-B aligned");
  // 32-bit DMA offsets: the window's rows and the weight matrix must stay below 2 GB
  if ((long long)n * C * 2 >= (1LL << 31) || 3LL * C * C * 2 >= (1LL << 31)) return lrce_fail(LRCE_E_ARG, "wattn_qkv_fwd: too large");
  if (n_win <= 0) return LRCE_OK;
  FusedP p;
  p.x = reinterpret_cast<const bf16*>(x);
  p.w = reinterpret_cast<const bf16*>(w_qkv);
  p.b = b_qkv;
  p.biasf = bias_fwd;
  p.win_pat = win_pat;
  p.qkv = reinterpret_cast<bf16*>(qkv);
  p.out = reinterpret_cast<bf16*>(out);
  p.lse = lse;
  p.qscale = qscale;
  p.n_win = n_win; p.n = n; p.nH = nH; p.C = C;
  wattn_qkv_fwd_kernel<<<(unsigned)(n_win * (nH / HB)), 512, 0, static_cast<hipStream_t>(stream)>>>(p);
  return lrce_check_launch("wattn_qkv_fwd");
}
