// Fused 3D shifted-window attention for Video Swin (WindowAttention3D.forward,
// video_swin_ori.py:158-189) on gfx950.
//
// Problems are (window, head) pairs: n <= 160 tokens (147 = 3x7x7 padded to 5 tiles of 32), head_dim
// 32.  All products use v_mfma_f32_32x32x16_bf16.
//
// Forward (wattn_fwd3): S^T = K Q^T so each lane owns one query column and 80 key rows: the softmax
// row reductions are in-lane plus one cross-half exchange, and the probabilities are already the B
// operand of O^T = V^T P^T (cdna_hip_programming.md §3 "accumulator tile as the next MFMA's
// operand").  The relative-position bias, the shift mask (-100) and the key padding (-1e30) are
// pre-combined per (mask pattern, head), pre-multiplied by log2(e) and stored in the exact per-lane
// accumulator order, so the MFMA chain starts from the bias: no VALU for scale/bias/mask.  q is
// pre-scaled by head_dim^-0.5 * log2(e) in the QKV GEMM epilogue, so p = exp2(s - max).
//
// Backward: one kernel per (window, head) with the bias-table gradient binned in LDS (wattn_bwd_kernel).
#include <cstdlib>
#include <type_traits>

#include "common.h"
#include "lrce_capi.h"

namespace {

constexpr int TQ = 32;        // tile edge
constexpr int NTILE = 5;      // 160 / 32
constexpr int NPAD = 160;
constexpr int HD = 32;        // head dim
constexpr int TILE_ELEMS = 64 * 16;
constexpr int PH_ELEMS = NTILE * NTILE * TILE_ELEMS;  // per (pattern, head)
constexpr float LOG2E = 1.4426950408889634f;
constexpr float NEG_BIG = -1.0e30f;

// row index (inside a 32x32 C tile) held in register `reg` by lane half `h`
__device__ __forceinline__ int crow(int reg, int h) { return (reg & 3) + 8 * (reg >> 2) + 4 * h; }

__device__ __forceinline__ bf16x8 ld_row16(const bf16* p) { return *reinterpret_cast<const bf16x8*>(p); }

// transposed read of an LDS image [rows][32] bf16 (64-B rows): returns 8 elements
// element j = img[r_base + 8*(j>>2) + 4*hh + (j&3)][c = 16*((lane>>4)&1) + (lane&15)],
// i.e. the operand fragment whose k index follows the permuted accumulator order.
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
// tr_read_perm of a 32 x 32 tile stored with its 8-B chunks XOR-swizzled by (row >> 2) & 7 (each
// lane's 8-B load is the same data, so the transposed result is unchanged; the swizzle spreads the
// producer's row-strided stores over all banks)
__device__ __forceinline__ int swz8(int row, int chunk) { return row * 32 + 4 * (chunk ^ ((row >> 2) & 7)); }
__device__ __forceinline__ bf16x8 tr_read_perm_swz(const bf16* img, int r_base, int lane) {
  const int g = lane >> 4, i = lane & 15, q = i >> 2, p = i & 3;
  const int hh = g >> 1, cb = 4 * (g & 1);
  bf16x8 out;
#pragma unroll
  for (int h2 = 0; h2 < 2; ++h2) {
    const int row = r_base + 8 * h2 + 4 * hh + q;
    const LRCE_LDS s16x4* src = (const LRCE_LDS s16x4*)(img + swz8(row, cb + p));
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

// ------------------------------------------------------------------------------ bias tiles
// forward tiles f32 (bf) or fp16 (bfh: the fused QKV + attention forward), backward tiles f32 (bb) or
// fp16 (bbh) — fp16 halves the bytes every (window, head) reads; padded keys at -30000 (exp2 -> 0 all
// the same).  The forward and backward of one layer use the same rounding, so the probabilities the
// backward recomputes are the forward's.
__global__ void bias_build_kernel(const float* table, const int64_t* index, int ld, int n, int nH,
                                  const int* region, int n_pat, float* bf, f16* bfh, float* bb, f16* bbh) {
  const long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  const long long total = (long long)n_pat * nH * PH_ELEMS;
  if (e >= total) return;
  const int reg = e & 15, lane = (e >> 4) & 63;
  const int et = e % TILE_ELEMS;                                   // forward tiles: [u][lane][4]
  const int lane_f = (et >> 2) & 63, reg_f = 4 * (et >> 8) + (et & 3);
  const int tile = (e / TILE_ELEMS) % (NTILE * NTILE);
  const int ph = e / PH_ELEMS;
  const int h = ph % nH, pat = ph / nH;
  const int qt = tile / NTILE, kt = tile % NTILE;
  const int* rg = region ? region + pat * n : nullptr;
  auto val = [&](int i, int j) -> float {
    if (j >= n) return NEG_BIG;
    if (i >= n) return 0.f;
    float v = table[index[(long long)i * ld + j] * nH + h];
    if (rg && rg[i] != rg[j]) v += -100.0f;
    return v * LOG2E;
  };
  // forward: S^T tile (rows = keys, cols = queries)
  const float vf = val(qt * TQ + (lane_f & 31), kt * TQ + crow(reg_f, lane_f >> 5));
  if (bfh) bfh[e] = f2h(vf < -30000.f ? -30000.f : vf);
  else bf[e] = vf;
  const int hh = lane >> 5, col = lane & 31;
  // backward: S tile (rows = queries, cols = keys)
  const float vb = val(qt * TQ + crow(reg, hh), kt * TQ + col);
  if (bbh) bbh[e] = f2h(vb < -30000.f ? -30000.f : vb);
  else bb[e] = vb;
}

// K rows XOR-swizzled by 16-B chunk (conflict-free row reads of the grouped forward's Q tiles)
__device__ __forceinline__ int kswz(int row, int chunk) { return row * HD + ((chunk ^ ((row >> 2) & 3)) << 3); }

// ------------------------------------------------------------------------------ forward, grouped
// Four windows of ONE (mask pattern, head) per workgroup, one wave each: the 20 KB bias row of the
// current query tile is staged ONCE per workgroup in LDS (LDS-DMA, prefetched one query tile
// ahead) instead of being re-read from L2 by every window, and every operand of the loop body comes
// from LDS or registers filled a tile ahead (V and the next Q tile by LDS-DMA), so no wave stalls on
// a global load inside the loop.  Windows are grouped by pattern on the host (win_list, -1 = empty
// slot; grp_pat = the group's pattern); unshifted stages use the identity grouping.
constexpr int GW = 4;                         // windows (waves) per workgroup
constexpr int BIAS_ROW = NTILE * TILE_ELEMS;  // floats of one query tile's bias row (20 KB)

struct Fwd3Lds {
  float bias[BIAS_ROW];
  bf16 v[GW][NPAD * HD];
  bf16 q[GW][2][TQ * HD];
};

__device__ __forceinline__ void glds16w(const void* src, void* lds_dst) {
  __builtin_amdgcn_global_load_lds(src, (LRCE_LDS void*)lds_dst, 16, 0, 0);
}
// The same LDS-DMA hidden from hipcc's wait bookkeeping (cdna_hip_programming.md §5.7): a builtin DMA
// in flight makes hipcc drain vmcnt(0) before every later LDS read, which would serialize the
// prefetch with the PV reads of V.  Completion is ordered by the loop's own vmcnt(0) + s_barrier.
__device__ __forceinline__ uint32_t lds_u32(const void* p) { return (uint32_t)(uintptr_t)((LRCE_LDS const void*)p); }
__device__ __forceinline__ void glds16_asm(const void* src, uint32_t lds_dst) {
  unsigned keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
               : "=&s"(keep) : "v"(src), "s"(lds_dst) : "memory");
}

__global__ void __launch_bounds__(256, 2) wattn_fwd3_kernel(const bf16* __restrict__ qkv, const float* __restrict__ biasf,
                                                            const int* __restrict__ win_list, const int* __restrict__ grp_pat,
                                                            bf16* __restrict__ out, float* __restrict__ lse, int n_win, int n,
                                                            int nH) {
  __shared__ __attribute__((aligned(16))) Fwd3Lds S;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int lin = xcd_remap(blockIdx.x, gridDim.x);   // a group's heads run on one XCD (shared qkv lines)
  const int h = lin % nH, g = lin / nH;
  const int wraw = win_list ? win_list[g * GW + wave] : g * GW + wave;
  const bool valid = wraw >= 0 && wraw < n_win;
  const int w = valid ? wraw : 0;
  const int pat = grp_pat ? grp_pat[g] : 0;
  const int C = nH * HD;
  const long long ld = 3LL * C;
  const bf16* base = qkv + (long long)w * n * ld;
  const float* bias_ph = biasf + (long long)(pat * nH + h) * PH_ELEMS;
  const int hh = lane >> 5, r32 = lane & 31;

  // LDS-DMA issue helpers (lane-linear destinations, 1 KB per wave-instruction); ASM: hidden from hipcc.
  // Per-lane source offsets are loop-invariant 32-bit element offsets; only the query-tile term
  // (a multiple of the row stride) changes per tile, so the loop body does one add per address.
  const int wv = __builtin_amdgcn_readfirstlane(wave);
  const float* bias_lane = bias_ph + wv * 5 * 256 + lane * 4;
  int qoff[2], qoff_last[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int row = i * 16 + (lane >> 2), pos = lane & 3;
    const int c = pos ^ ((row >> 2) & 3);
    qoff[i] = row * (int)ld + h * HD + c * 8;                                   // tiles 0..3: never clamped
    qoff_last[i] = min((NTILE - 1) * TQ + row, n - 1) * (int)ld + h * HD + c * 8;   // tile 4: rows >= n clamped
  }
  auto issue_bias = [&](int qt, auto asm_c) {   // 20 x 1 KB, 5 per wave
    const float* src = bias_lane + qt * BIAS_ROW;
#pragma unroll
    for (int i = 0; i < 5; ++i) {
      const int ins = wv * 5 + i;
      if constexpr (decltype(asm_c)::value) glds16_asm(src + i * 256, lds_u32(S.bias + ins * 256));
      else glds16w(src + i * 256, S.bias + ins * 256);
    }
  };
  auto issue_q = [&](int qt, auto asm_c) {      // 32 rows x 64 B = 2 x 1 KB, chunks XOR-swizzled by row (kswz)
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const bf16* src = base + (qt == NTILE - 1 ? qoff_last[i] : qt * TQ * (int)ld + qoff[i]);
      if constexpr (decltype(asm_c)::value) glds16_asm(src, lds_u32(&S.q[wv][qt & 1][i * 512]));
      else glds16w(src, &S.q[wv][qt & 1][i * 512]);
    }
  };
  constexpr std::false_type BUILTIN{};
  constexpr std::true_type ASM{};

  // prologue: bias row 0 (whole workgroup), this wave's V image and Q tile 0, K fragments
  issue_bias(0, BUILTIN);
  if (valid) {
#pragma unroll
    for (int i = 0; i < NPAD / 16; ++i) {       // V rows 16i .. 16i+15, rows >= n clamped (never weighted)
      const int tok = min(i * 16 + (lane >> 2), n - 1);
      glds16w(base + tok * ld + 2 * C + h * HD + (lane & 3) * 8, &S.v[wave][i * 512]);
    }
    issue_q(0, BUILTIN);
  }
  bf16x8 kf[NTILE][2];
#pragma unroll
  for (int kt = 0; kt < NTILE; ++kt) {
    const int key = kt * TQ + r32;
#pragma unroll
    for (int s = 0; s < 2; ++s) kf[kt][s] = (valid && key < n) ? ld_row16(base + key * ld + C + h * HD + 16 * s + 8 * hh) : bf16x8{};
  }

  // The output rows of tile qt are stored one iteration late (right after the next tile's wait), so
  // the vmcnt(0) that waits for the next tile's DMA never also waits on this tile's fresh stores.
  bf16x4 pend[4];
  float pend_lse = 0.f;
  int pend_qi = NPAD;   // >= n: nothing pending
  auto flush = [&]() {
    if (valid && pend_qi < n) {
      bf16* dst = out + ((long long)w * n + pend_qi) * C + h * HD + 4 * hh;
#pragma unroll
      for (int rr = 0; rr < 4; ++rr) *reinterpret_cast<bf16x4*>(dst + 8 * rr) = pend[rr];
      if (hh == 0) lse[((long long)w * nH + h) * NPAD + pend_qi] = pend_lse;
    }
  };
  for (int qt = 0; qt < NTILE; ++qt) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // this wave's DMA for tile qt (and tile qt-2's stores)
    __builtin_amdgcn_s_barrier();                        // ... and every other wave's part of the bias row
    flush();
    f32x16 acc[NTILE];
    {
      const float4* src = reinterpret_cast<const float4*>(S.bias) + lane;
#pragma unroll
      for (int kt = 0; kt < NTILE; ++kt)
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const float4 b = src[kt * (TILE_ELEMS / 4) + 64 * u];
          acc[kt][4 * u] = b.x; acc[kt][4 * u + 1] = b.y; acc[kt][4 * u + 2] = b.z; acc[kt][4 * u + 3] = b.w;
        }
    }
    bf16x8 qf[2];
#pragma unroll
    for (int s = 0; s < 2; ++s) qf[s] = *reinterpret_cast<const bf16x8*>(&S.q[wave][qt & 1][kswz(r32, 2 * s + hh)]);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();                        // bias row consumed by every wave: refill it
    if (qt + 1 < NTILE) {
      issue_bias(qt + 1, ASM);
      if (valid) issue_q(qt + 1, ASM);
    }
    if (valid) {
      const int qi = qt * TQ + r32;
#pragma unroll
      for (int kt = 0; kt < NTILE; ++kt) {
        acc[kt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(kf[kt][0], qf[0], acc[kt], 0, 0, 0);
        acc[kt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(kf[kt][1], qf[1], acc[kt], 0, 0, 0);
      }
      // softmax over keys.  Row max: 4 independent v_max3 chains + the cross-half exchange.  When
      // every row max of the wave lies in [-64, 64] (always, short of pathological logits) the
      // exponent needs no shift: exp2(s) / sum exp2(s) == exp2(s - m) / sum exp2(s - m), and f32
      // exp2 of [-inf, 64] neither overflows nor loses a row to underflow.
      float mp[4] = {NEG_BIG, NEG_BIG, NEG_BIG, NEG_BIG};
#pragma unroll
      for (int kt = 0; kt < NTILE; ++kt)
#pragma unroll
        for (int r = 0; r < 16; ++r) mp[r & 3] = fmaxf(mp[r & 3], acc[kt][r]);
      float m = fmaxf(fmaxf(mp[0], mp[1]), fmaxf(mp[2], mp[3]));
      m = fmaxf(m, __shfl_xor(m, 32, 64));
      if (__all(m <= 64.f && m >= -64.f)) m = 0.f;
      f32x2 sp[2] = {f32x2{0.f, 0.f}, f32x2{0.f, 0.f}};
      const f32x2 mm = {m, m};
#pragma unroll
      for (int kt = 0; kt < NTILE; ++kt)
#pragma unroll
        for (int r = 0; r < 16; r += 2) {
          const f32x2 d = f32x2{acc[kt][r], acc[kt][r + 1]} - mm;   // packed subtract / sum: one op per pair
          const f32x2 p = {__builtin_amdgcn_exp2f(d[0]), __builtin_amdgcn_exp2f(d[1])};
          acc[kt][r] = p[0];
          acc[kt][r + 1] = p[1];
          sp[(r >> 1) & 1] += p;
        }
      float sum = (sp[0][0] + sp[0][1]) + (sp[1][0] + sp[1][1]);
      sum += __shfl_xor(sum, 32, 64);
      f32x16 o0 = {}, o1 = {};   // two independent accumulation chains, summed once
      const bf16* vimg = S.v[wave];
#pragma unroll
      for (int kt = 0; kt < NTILE; ++kt) {
        o0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(tr_read_perm(vimg, kt * TQ, lane), pack8(acc[kt], 0), o0, 0, 0, 0);
        o1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(tr_read_perm(vimg, kt * TQ + 16, lane), pack8(acc[kt], 1), o1, 0, 0, 0);
      }
      const f32x16 o = o0 + o1;
      const float inv = 1.0f / sum;
#pragma unroll
      for (int rr = 0; rr < 4; ++rr) {
        pend[rr][0] = f2bf(o[4 * rr] * inv); pend[rr][1] = f2bf(o[4 * rr + 1] * inv);
        pend[rr][2] = f2bf(o[4 * rr + 2] * inv); pend[rr][3] = f2bf(o[4 * rr + 3] * inv);
      }
      pend_lse = m + __log2f(sum);
      pend_qi = qi;
    }
  }
  flush();
}

// ------------------------------------------------------------------------------ backward
// One workgroup per (window, head), five waves; wave t owns key tile t (dK, dV) AND query tile t (dQ).
// Step s = 0..4: wave t computes the tile (qt = t+s mod 5, kt = t) once, in the dK/dV orientation
//   S = Q~ K^T + bias (rows = queries, key on the lane), dP = dO V^T, P = exp2(S - lse),
//   dS = P (dP - delta);  dV^T += dO^T P, dK^T += Q~^T dS  (P / dS straight from the accumulators as
//   B operands, dO / Q~ by transposed LDS reads: results have the key on the lane -> 8-B stores).
// dQ needs the same dS transposed: each wave parks its dS tile (bf16, key-major [key][query]) in an
// LDS slot, one barrier, and wave t reads the tile (t, t-s mod 5) that wave t-s wrote this step as the
// B operand of dQ^T += K^T dS^T (both operands by ds_read_tr16 in the accumulator's permuted key
// order).  Slots are double-buffered by step parity: one barrier per step, dQ summed in a fixed order.
// So every product is computed once (S, dP, dV, dK, dQ: 10 MFMAs per tile) and every operand byte is
// read from HBM once per (window, head).
// Relative-position-bias gradient: the table row of (query i, key j) is a linear function of the
// token codes, code(i) - code(j) + off (video_swin_ori.py:133-148 with window (wd, wh, ww)), so dS is
// binned in LDS by that difference and each (window, head) writes n_bins floats (3.4 KB at 3x7x7)
// instead of its 160^2 dS image.  The bins are fixed-point int32 (ds_add_u32): integer adds make the
// sum independent of wave timing (an LDS integer add is a few cycles per wave instruction against
// ~230 for ds_add_f32, tools/lds_atomic_bench.hip).  The fixed point is scaled per (window, head) by
// 2^s from a bound on |dS| (|dS_ij| = P_ij |dP_ij - delta_i| <= 2 max|dP| <= 2 max_i |dO_i| max_j |V_j|,
// so |dS| 2^s < 2^22 and a bin of <= 160 terms stays below 2^30): the quantum follows the gradient's
// magnitude (an absolute quantum lost batch-mean-sized gradients) and is 2^-22 of the bound — finer
// than the bf16 dS the dQ / dK products use.  Conversion: one f32 fma onto 1.5 * 2^23 leaves
// round(dS 2^s) in the low mantissa bits; the add takes the fma's bit pattern as it is and the
// epilogue subtracts 0x4B400000 times the bin's (closed-form) number of adds, modulo 2^32 (the f64 /
// int64 form of round 2 spent ~7 VALU per element on the conversion and twice the LDS atomic bandwidth).
// lrce_wattn_dbias sums the windows in a fixed order and scatters bins to table rows.
// Bank-spread bin order: in LDS a relative position (dt, dh, dw) lives at dt A + dh B + dw with B = ww
// (mod 32), A = wh ww (mod 32) and A, B large enough to keep the map injective (3x7x7: B = 39,
// A = 497, 2469 slots), so the token code t A + h B + w is congruent to the token index mod 32: the
// 32 lanes of a half (one query, 32 consecutive keys) add to 32 distinct banks.  The natural radix
// (2ww-1, 2wh-1) put key rows 7 words apart in 13-word strides — 32 keys spanned ~56 words, so lanes
// 32 words apart collided (45 % of the LDS cycles were bank conflicts).  The bins leave in natural
// order (the relative-position index the dbias pass and lrce_wattn_dbias's bin_row use).
// Workgroup barrier for LDS hand-offs only: __syncthreads() would also drain vmcnt(0), i.e. wait for
// the bias-tile loads of later steps and the dK / dV / dQ stores in flight.
__device__ __forceinline__ void lds_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

constexpr int BW = 5;        // waves per backward workgroup (= tiles of 32 rows)
constexpr int NBMAX = 1024;  // relative-position bins per (window, head) written out (natural order)
constexpr int NBL = 2560;    // LDS bins per head in the bank-spread order (bin_spread)
constexpr int WCH = 32;      // window chunks of the deterministic bias-gradient reduction

struct BwdLds {
  bf16 q[NPAD * HD];
  bf16 dout[NPAD * HD];
  bf16 k[NPAD * HD];
  bf16 ds[2][BW][TQ * TQ];
  unsigned bins[NBL];      // 2^s fixed point (two's complement int32), bank-spread order
  float4 qinfo[NPAD];   // per query: lse, delta, token code (as bits), -
  float nmax[BW][2];    // per wave: max |dO_q|^2, max |V_q|^2 over its rows (the bins' scale)
};

// HPW heads per workgroup (2 when nH is even): the hardware keeps only ONE 5-wave workgroup per CU at
// this kernel's ~160 VGPRs (tools/occupancy_probe.hip: 320-thread workgroups at 136-168 VGPRs are
// admitted one per CU, 256-thread ones three), so pairing two heads' independent 5-wave halves in one
// workgroup doubles the waves per CU.
template <bool BH, int HPW>
__global__ void __launch_bounds__(BW * 64 * HPW, 3) wattn_bwd_kernel(const bf16* __restrict__ qkv, const bf16* __restrict__ outp,
                                                              const bf16* __restrict__ dout, const float* __restrict__ lse_g,
                                                              const void* __restrict__ biasb, const int* __restrict__ win_pat,
                                                              bf16* __restrict__ dqkv, float* __restrict__ dbias_part, int n_win,
                                                              int n, int nH, int wh, int ww, int nb, int boff, int ba, int bb,
                                                              float qscale, unsigned long long* __restrict__ trace) {
  __shared__ __attribute__((aligned(16))) BwdLds LL[HPW];
  // debug phase timestamps, compiled in only with -DLRCE_WATTN_TRACE (tools/wattn_trace.py builds that
  // variant: the marks cost registers this kernel does not have to spare): thread 0 of each workgroup
#ifdef LRCE_WATTN_TRACE
#define WB_MARK(I)                                                                    \
  if (trace && threadIdx.x == 0) trace[(long long)blockIdx.x * 16 + (I)] = __builtin_amdgcn_s_memrealtime();
  WB_MARK(0)
  if (trace && threadIdx.x == 0) {   // placement: HW_ID (cu / sh / se) and XCC_ID
    trace[(long long)blockIdx.x * 16 + 10] = __builtin_amdgcn_s_getreg(4 | (31 << 11));
    trace[(long long)blockIdx.x * 16 + 11] = __builtin_amdgcn_s_getreg(20 | (31 << 11));
  }
#else
#define WB_MARK(I)
#endif
  const int hs = HPW == 1 ? 0 : __builtin_amdgcn_readfirstlane((int)threadIdx.x / (BW * 64));   // head of the workgroup
  const int lt = (int)threadIdx.x - hs * BW * 64;   // thread index within that head's half
  BwdLds& L = LL[hs];
  const int lane = lt & 63, t = lt >> 6;
  // logical order (head pair, window, head of the pair): the two heads sharing 128-B qkv / dO lines
  // run in one workgroup (HPW = 2) or next to each other, and one XCD's contiguous range covers few
  // heads (their bias tiles stay in that XCD's L2)
  const int lin = xcd_remap(blockIdx.x, gridDim.x);
  int h, w;
  if constexpr (HPW == 2) {
    h = (lin / n_win) * 2 + hs;
    w = lin % n_win;
  } else {
    const int hp = (nH & 1) ? 1 : 2;
    h = (lin / hp / n_win) * hp + lin % hp;
    w = (lin / hp) % n_win;
  }
  const int C = nH * HD;
  const long long ld = 3LL * C;
  const bf16* base = qkv + (long long)w * n * ld;
  const bf16* obase = outp + (long long)w * n * C + h * HD;
  const bf16* dobase = dout + (long long)w * n * C + h * HD;
  const int hh = lane >> 5, r32 = lane & 31;
  const int key = t * TQ + r32;
  // Q~, K and dO images [160][32] (rows >= n zero): 3 x 640 16-B chunks over 320 threads
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int c = lt + BW * 64 * i;
    const int row = c >> 2, part = c & 3;
    uint4 qv = make_uint4(0, 0, 0, 0), kv = make_uint4(0, 0, 0, 0), dv = make_uint4(0, 0, 0, 0);
    if (row < n) {
      qv = *reinterpret_cast<const uint4*>(base + row * ld + h * HD + part * 8);
      kv = *reinterpret_cast<const uint4*>(base + row * ld + C + h * HD + part * 8);
      dv = *reinterpret_cast<const uint4*>(dobase + (long long)row * C + part * 8);
    }
    *reinterpret_cast<uint4*>(L.q + row * HD + part * 8) = qv;
    *reinterpret_cast<uint4*>(L.k + row * HD + part * 8) = kv;
    *reinterpret_cast<uint4*>(L.dout + row * HD + part * 8) = dv;
  }
  // V fragments of this wave's key tile (B operand of dP = dO V^T), straight to registers
  bf16x8 vf[2];
#pragma unroll
  for (int s = 0; s < 2; ++s) vf[s] = key < n ? ld_row16(base + key * ld + 2 * C + h * HD + 16 * s + 8 * hh) : bf16x8{};
  // delta[q] = dO[q] . O[q], lse[q] (0 past n: padded queries contribute nothing), token codes;
  // |dO_q|^2 and |V_q|^2 for the bins' scale
  float dn2 = 0.f, vn2 = 0.f;
  if (lt < NPAD) {
    const int q = lt;
    float d = 0.f, l = 0.f;
    int code = 0;
    if (q < n) {
#pragma unroll
      for (int part = 0; part < 4; ++part) {
        const bf16x8 a = ld_row16(obase + (long long)q * C + part * 8);
        const bf16x8 b = ld_row16(dobase + (long long)q * C + part * 8);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          d += bf2f(a[j]) * bf2f(b[j]);
          dn2 += bf2f(b[j]) * bf2f(b[j]);
        }
      }
      l = lse_g[((long long)w * nH + h) * NPAD + q];
      code = (q / (wh * ww)) * ba + ((q / ww) % wh) * bb + q % ww;   // bank-spread token code
    }
    L.qinfo[q] = make_float4(l, d, __int_as_float(code), 0.f);
  }
  // |V_key|^2 from the wave's own V fragments (lanes l and l + 32 hold the two halves of a key row)
#pragma unroll
  for (int s = 0; s < 2; ++s)
#pragma unroll
    for (int j = 0; j < 8; ++j) vn2 += bf2f(vf[s][j]) * bf2f(vf[s][j]);
  vn2 += __shfl_xor(vn2, 32, 64);
  dn2 = wave_max(dn2);
  vn2 = wave_max(vn2);
  if (lane == 0) {
    L.nmax[t][0] = dn2;
    L.nmax[t][1] = vn2;
  }
  for (int i = lt; i < NBL; i += BW * 64) L.bins[i] = 0u;
  __syncthreads();
  WB_MARK(1)
  // bins' scale 2^s: |dS| <= 2 max|dO| max|V| = bound < 2^e -> |dS| 2^s < 2^22 with s = 22 - e
  float bscale, binv;
  {
    float m0 = 0.f, m1 = 0.f;
#pragma unroll
    for (int i = 0; i < BW; ++i) {
      m0 = fmaxf(m0, L.nmax[i][0]);
      m1 = fmaxf(m1, L.nmax[i][1]);
    }
    int e = 0;
    (void)frexpf(2.0f * sqrtf(m0) * sqrtf(m1) * 1.0001f, &e);   // margin for the norms' own rounding
    const int sh = max(-126, min(126, 22 - e));   // (clamp: both powers stay normal f32)
    bscale = ldexpf(1.0f, sh);
    binv = ldexpf(1.0f, -sh);
  }
  bf16x8 kf[2];
#pragma unroll
  for (int s = 0; s < 2; ++s) kf[s] = *reinterpret_cast<const bf16x8*>(L.k + key * HD + 16 * s + 8 * hh);
  const int pat = win_pat ? win_pat[w] : 0;
  const long long bofs = (long long)(pat * nH + h) * PH_ELEMS + lane * 16;   // this lane's 16 values per tile
  const bool key_live = key < n;
  const int kbin = boff - (key_live ? __float_as_int(L.qinfo[key].z) : 0);
  const bool want_bins = dbias_part != nullptr;
  f32x16 dkT = {}, dvT = {}, dqT = {};
#pragma unroll 1
  for (int s = 0; s < NTILE; ++s) {
    const int qt = t + s < NTILE ? t + s : t + s - NTILE;
    f32x16 sacc;
    if constexpr (BH) {
      const uint4* src = reinterpret_cast<const uint4*>(static_cast<const f16*>(biasb) + bofs + (qt * NTILE + t) * TILE_ELEMS);
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const uint4 b = src[u];
        const unsigned w4[4] = {b.x, b.y, b.z, b.w};
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          sacc[8 * u + 2 * e] = (float)__builtin_bit_cast(f16, (unsigned short)(w4[e] & 0xFFFFu));
          sacc[8 * u + 2 * e + 1] = (float)__builtin_bit_cast(f16, (unsigned short)(w4[e] >> 16));
        }
      }
    } else {
      const float4* src = reinterpret_cast<const float4*>(static_cast<const float*>(biasb) + bofs + (qt * NTILE + t) * TILE_ELEMS);
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const float4 b = src[u];
        sacc[4 * u] = b.x; sacc[4 * u + 1] = b.y; sacc[4 * u + 2] = b.z; sacc[4 * u + 3] = b.w;
      }
    }
    f32x16 dp = {};
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2) {
      const bf16x8 qa = *reinterpret_cast<const bf16x8*>(L.q + (qt * TQ + r32) * HD + 16 * s2 + 8 * hh);
      const bf16x8 da = *reinterpret_cast<const bf16x8*>(L.dout + (qt * TQ + r32) * HD + 16 * s2 + 8 * hh);
      sacc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(qa, kf[s2], sacc, 0, 0, 0);
      dp = __builtin_amdgcn_mfma_f32_32x32x16_bf16(da, vf[s2], dp, 0, 0, 0);
    }
    // P and dS (natural-log scale); rows = queries crow(r, hh), key on the lane
    float4 qi4[16];
#pragma unroll
    for (int r = 0; r < 16; ++r) qi4[r] = L.qinfo[qt * TQ + crow(r, hh)];
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const float p = __builtin_amdgcn_exp2f(sacc[r] - qi4[r].x);
      sacc[r] = p;
      dp[r] = p * (dp[r] - qi4[r].y);
    }
    // bias-table gradient: dS is exactly 0 for padded queries (zero dO rows, delta 0; their code 0 keeps
    // the bin inside the array) and padded keys (P = 0); the padded keys' lanes are masked off (they
    // would all add to one word)
    if (want_bins && key_live) {
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        // round(dS * 2^s) to int32: the fma result lies in [2^23, 2^24) (ulp 1) for |dS 2^s| < 2^22
        // the add carries the bias 0x4B400000 of the fma trick; the epilogue subtracts it once per add
        const float m = __builtin_fmaf(dp[r], bscale, 0x1.8p23f);
        atomicAdd(&L.bins[__float_as_int(qi4[r].z) + kbin], (unsigned)__float_as_int(m));
      }
    }
    // dV^T += dO^T P ; dK^T += Q~^T dS  (the accumulators as B operands, permuted k order)
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2) {
      dvT = __builtin_amdgcn_mfma_f32_32x32x16_bf16(tr_read_perm(L.dout, qt * TQ + 16 * s2, lane), pack8(sacc, s2), dvT, 0, 0, 0);
      dkT = __builtin_amdgcn_mfma_f32_32x32x16_bf16(tr_read_perm(L.q, qt * TQ + 16 * s2, lane), pack8(dp, s2), dkT, 0, 0, 0);
    }
    // park dS key-major: slot[key][query] (8-B chunks swizzled), register r = 4g + e holds query
    // 8g + 4hh + e = chunk 2g + hh
    bf16* slot = L.ds[s & 1][t];
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      bf16x4 v;
#pragma unroll
      for (int e = 0; e < 4; ++e) v[e] = f2bf(dp[4 * g + e]);
      *reinterpret_cast<bf16x4*>(slot + swz8(r32, 2 * g + hh)) = v;
    }
    lds_barrier();
    WB_MARK(2 + s)
    // dQ^T(t) += K(kt2)^T dS(t, kt2)^T with the tile wave kt2 = t - s parked this step
    const int kt2 = t - s >= 0 ? t - s : t - s + NTILE;
    const bf16* src = L.ds[s & 1][kt2];
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2)
      dqT = __builtin_amdgcn_mfma_f32_32x32x16_bf16(tr_read_perm(L.k, kt2 * TQ + 16 * s2, lane), tr_read_perm_swz(src, 16 * s2, lane),
                                                    dqT, 0, 0, 0);
  }
  // dK^T / dV^T: rows = head dims crow(r, hh), key on the lane -> 4 x 8-B stores per row piece
  if (key_live) {
    const float kscale = 1.0f / LOG2E;   // q~ = q d^-1/2 log2(e): dK = dS^T q d^-1/2 = dS^T q~ / log2(e)
    bf16* row = dqkv + ((long long)w * n + key) * ld + h * HD + 4 * hh;
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      bf16x4 a, b;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        a[e] = f2bf(dkT[4 * g + e] * kscale);
        b[e] = f2bf(dvT[4 * g + e]);
      }
      *reinterpret_cast<bf16x4*>(row + C + 8 * g) = a;
      *reinterpret_cast<bf16x4*>(row + 2 * C + 8 * g) = b;
    }
  }
  // dQ^T: rows = head dims, query t*32 + r32 on the lane
  const int q = t * TQ + r32;
  if (q < n) {
    bf16* row = dqkv + ((long long)w * n + q) * ld + h * HD + 4 * hh;
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      bf16x4 a;
#pragma unroll
      for (int e = 0; e < 4; ++e) a[e] = f2bf(dqT[4 * g + e] * qscale);
      *reinterpret_cast<bf16x4*>(row + 8 * g) = a;
    }
  }
  WB_MARK(7)
  if (!want_bins) return;
  lds_barrier();   // every wave's bin adds are done (the row stores above stay in flight)
  float* dst = dbias_part + ((long long)w * nH + h) * nb;
  const int nw2 = 2 * ww - 1, nh2 = 2 * wh - 1, wd = n / (wh * ww);
  for (int b = lt; b < nb; b += BW * 64) {   // natural bin b = ((dt + wd-1) nh2 + dh + wh-1) nw2 + dw + ww-1
    const int dw = b % nw2 - (ww - 1), r = b / nw2;
    const int dh = r % nh2 - (wh - 1), dt = r / nh2 - (wd - 1);
    // adds into this slot: the (query, key) pairs at that relative position, plus one per padded query
    // (code 0) for the relative positions of -(a key's position) — each carried the 0x4B400000 bias
    const unsigned cnt = (unsigned)((wd - abs(dt)) * (wh - abs(dh)) * (ww - abs(dw)) +
                                    ((dt <= 0 && dh <= 0 && dw <= 0) ? NPAD - n : 0));
    dst[b] = (float)(int)(L.bins[dt * ba + dh * bb + dw + boff] - cnt * 0x4B400000u) * binv;
  }
  WB_MARK(8)
#undef WB_MARK
}

// Bias-table gradient from the per-(window, head) bin rows, no atomics: (1) WCH chunks of windows
// summed per (head, bin) into the scratch tail, (2) the chunks summed in order and added to the table
// row of that bin (bin_row: -1 = no (query, key) pair uses the bin) — one writer per entry.
__global__ void dbias_chunk_kernel(const float* __restrict__ part, int n_win, int hb, float* __restrict__ red) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= hb) return;
  const int per = (n_win + WCH - 1) / WCH;
  const int w0 = blockIdx.y * per, w1 = min(n_win, w0 + per);
  float s = 0.f;
  for (int w = w0; w < w1; ++w) s += part[(long long)w * hb + e];
  red[(long long)blockIdx.y * hb + e] = s;
}

__global__ void dbias_scatter_kernel(const float* __restrict__ red, int hb, int nb, int nH, const int* __restrict__ bin_row,
                                     float* __restrict__ tgrad) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= hb) return;
  const int h = e / nb, row = bin_row[e % nb];
  if (row < 0) return;
  float s = 0.f;
#pragma unroll 8
  for (int c = 0; c < WCH; ++c) s += red[(long long)c * hb + e];
  tgrad[(long long)row * nH + h] += s;
}

// Several blocks' bias-table gradients in two launches (lrce_wattn_dbias_batched): blockIdx.z picks
// the block (its bins, bin map, table gradient); the same two passes as above.
struct DbItem {
  float* part;
  const int* bin_row;
  float* tgrad;
  int n_win, nH, nb;
};
constexpr int DB_BATCH = 24;
struct DbBatch {
  DbItem it[DB_BATCH];
};
__global__ void dbias_chunk_batched(DbBatch b) {
  const DbItem& it = b.it[blockIdx.z];
  const int hb = it.nH * it.nb;
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= hb) return;
  const int per = (it.n_win + WCH - 1) / WCH;
  const int w0 = blockIdx.y * per, w1 = min(it.n_win, w0 + per);
  float s = 0.f;
  for (int w = w0; w < w1; ++w) s += it.part[(long long)w * hb + e];
  it.part[(long long)it.n_win * hb + (long long)blockIdx.y * hb + e] = s;
}
__global__ void dbias_scatter_batched(DbBatch b) {
  const DbItem& it = b.it[blockIdx.z];
  const int hb = it.nH * it.nb;
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= hb) return;
  const int h = e / it.nb, row = it.bin_row[e % it.nb];
  if (row < 0) return;
  const float* red = it.part + (long long)it.n_win * hb;
  float s = 0.f;
#pragma unroll 8
  for (int c = 0; c < WCH; ++c) s += red[(long long)c * hb + e];
  it.tgrad[(long long)row * it.nH + h] += s;
}

}  // namespace

static unsigned long long* g_wb_trace = nullptr;   // lrce_wattn_set_trace
unsigned long long* g_wattn_trace = nullptr;      // the same buffer, read by lrce_wattn_qkv_fwd (window_fused.hip)

extern "C" int64_t lrce_wattn_bias_elems(int n_pat, int nH) { return (int64_t)n_pat * nH * PH_ELEMS; }
// bias-gradient scratch (f32): one bin row per (window, head) + the WCH chunk sums
extern "C" int64_t lrce_wattn_dbias_part_elems(int n_win, int nH, int n_bins) {
  return (int64_t)(n_win + WCH) * nH * n_bins;
}

extern "C" int lrce_wattn_bias_build(const float* table, const int64_t* index, int index_ld, int n, int nH,
                                     const int32_t* region, int n_pat, void* bias_fwd, int fwd_f16, void* bias_bwd,
                                     int bwd_f16, void* stream) {
  if (!table || !index || !bias_fwd || !bias_bwd) return lrce_fail(LRCE_E_ARG, "wattn_bias_build: null pointer");
  if (n <= 0 || n > NPAD || n_pat < 1 || nH < 1) return lrce_fail(LRCE_E_ARG, "wattn_bias_build: n=%d", n);
  const long long total = (long long)n_pat * nH * PH_ELEMS;
  bias_build_kernel<<<(total + 255) / 256, 256, 0, static_cast<hipStream_t>(stream)>>>(
      table, index, index_ld, n, nH, region, n_pat, fwd_f16 ? nullptr : static_cast<float*>(bias_fwd),
      fwd_f16 ? static_cast<f16*>(bias_fwd) : nullptr, bwd_f16 ? nullptr : static_cast<float*>(bias_bwd),
      bwd_f16 ? static_cast<f16*>(bias_bwd) : nullptr);
  return lrce_check_launch("wattn_bias_build");
}

extern "C" int lrce_wattn_fwd_grouped(const uint16_t* qkv, const float* bias_fwd, const int32_t* win_list,
                                      const int32_t* grp_pat, int n_groups, uint16_t* out, float* lse, int n_win, int n,
                                      int nH, void* stream) {
  if (!qkv || !bias_fwd || !out || !lse) return lrce_fail(LRCE_E_ARG, "wattn_fwd_grouped: null pointer");
  if (n <= 4 * TQ || n > NPAD) return lrce_fail(LRCE_E_ARG, "wattn_fwd_grouped: n=%d outside (128,160]", n);
  if (!win_list && n_groups * GW < n_win) return lrce_fail(LRCE_E_ARG, "wattn_fwd_grouped: %d groups < %d windows", n_groups, n_win);
  if (n_win <= 0 || n_groups <= 0) return LRCE_OK;
  wattn_fwd3_kernel<<<(unsigned)(n_groups * nH), 256, 0, static_cast<hipStream_t>(stream)>>>(
      reinterpret_cast<const bf16*>(qkv), bias_fwd, win_list, grp_pat, reinterpret_cast<bf16*>(out), lse, n_win, n, nH);
  return lrce_check_launch("wattn_fwd_grouped");
}

extern "C" int lrce_wattn_bwd(const uint16_t* qkv, const uint16_t* out, const uint16_t* dout, const float* lse,
                              const void* bias_bwd, int bias_f16, const int32_t* win_pat, uint16_t* dqkv, float* dbias_part,
                              int n_win, int n, int nH, int wh, int ww, void* stream) {
  if (!qkv || !out || !dout || !lse || !bias_bwd || !dqkv) return lrce_fail(LRCE_E_ARG, "wattn_bwd: null pointer");
  if (n <= 4 * TQ || n > NPAD) return lrce_fail(LRCE_E_ARG, "wattn_bwd: n=%d outside (128,160]", n);
  if (wh < 1 || ww < 1 || n % (wh * ww)) return lrce_fail(LRCE_E_ARG, "wattn_bwd: n=%d is not a wd x %d x %d window", n, wh, ww);
  const int wd = n / (wh * ww);
  const int nb = (2 * wd - 1) * (2 * wh - 1) * (2 * ww - 1);
  if (nb > NBMAX) return lrce_fail(LRCE_E_ARG, "wattn_bwd: %d relative-position bins > %d", nb, NBMAX);
  if (n_win <= 0) return LRCE_OK;
  // bank-spread LDS bin order (see the kernel's comment): B = ww, A = wh ww (mod 32), injective
  int bb = 2 * ww - 1;
  while ((bb - ww) % 32) ++bb;
  int ba = 2 * ((wh - 1) * bb + (ww - 1)) + 1;
  while ((ba - wh * ww) % 32) ++ba;
  const int boff = (wd - 1) * ba + (wh - 1) * bb + (ww - 1);
  if (2 * boff + 1 > NBL) return lrce_fail(LRCE_E_ARG, "wattn_bwd: %d bank-spread bins > %d", 2 * boff + 1, NBL);
  const int hpw = (nH & 1) ? 1 : 2;   // two heads per workgroup (one head each measured slower)
  const auto kern = bias_f16 ? (hpw == 2 ? wattn_bwd_kernel<true, 2> : wattn_bwd_kernel<true, 1>)
                             : (hpw == 2 ? wattn_bwd_kernel<false, 2> : wattn_bwd_kernel<false, 1>);
  kern<<<(unsigned)(n_win * nH / hpw), BW * 64 * hpw, 0, static_cast<hipStream_t>(stream)>>>(
      reinterpret_cast<const bf16*>(qkv), reinterpret_cast<const bf16*>(out), reinterpret_cast<const bf16*>(dout), lse, bias_bwd,
      win_pat, reinterpret_cast<bf16*>(dqkv), dbias_part, n_win, n, nH, wh, ww, nb, boff, ba, bb, 1.0f / sqrtf((float)HD),
      g_wb_trace);
  return lrce_check_launch("wattn_bwd");
}

// debug: phase timestamps of wattn_bwd into buf (device, >= workgroups * 16 uint64), NULL = off; recorded
// only by a build with -DLRCE_WATTN_TRACE
extern "C" int lrce_wattn_set_trace(uint64_t* buf) {
  g_wb_trace = reinterpret_cast<unsigned long long*>(buf);
  g_wattn_trace = g_wb_trace;
  return LRCE_OK;
}

extern "C" int lrce_wattn_dbias(float* dbias_part, int n_win, int nH, int n_bins, const int32_t* bin_row, float* table_grad,
                                void* stream) {
  if (!dbias_part || !bin_row || !table_grad) return lrce_fail(LRCE_E_ARG, "wattn_dbias: null pointer");
  if (n_win <= 0 || nH <= 0 || n_bins <= 0 || n_bins > NBMAX)
    return lrce_fail(LRCE_E_ARG, "wattn_dbias: n_win=%d nH=%d n_bins=%d", n_win, nH, n_bins);
  const int hb = nH * n_bins;
  float* red = dbias_part + (long long)n_win * hb;
  hipStream_t st = static_cast<hipStream_t>(stream);
  dbias_chunk_kernel<<<dim3((unsigned)((hb + 255) / 256), WCH), 256, 0, st>>>(dbias_part, n_win, hb, red);
  dbias_scatter_kernel<<<(unsigned)((hb + 255) / 256), 256, 0, st>>>(red, hb, n_bins, nH, bin_row, table_grad);
  return lrce_check_launch("wattn_dbias");
}

extern "C" int lrce_wattn_dbias_batched(float* const* dbias_part, const int32_t* n_win, const int32_t* nH, const int32_t* n_bins,
                                        const int32_t* const* bin_row, float* const* table_grad, int n, void* stream) {
  if (n < 0 || (n > 0 && (!dbias_part || !n_win || !nH || !n_bins || !bin_row || !table_grad)))
    return lrce_fail(LRCE_E_ARG, "wattn_dbias_batched: args");
  hipStream_t st = static_cast<hipStream_t>(stream);
  for (int i0 = 0; i0 < n; i0 += DB_BATCH) {
    DbBatch b{};
    const int m = n - i0 < DB_BATCH ? n - i0 : DB_BATCH;
    int gx = 1;
    for (int j = 0; j < m; ++j) {
      const int i = i0 + j;
      if (!dbias_part[i] || !bin_row[i] || !table_grad[i] || n_win[i] <= 0 || nH[i] <= 0 || n_bins[i] <= 0 || n_bins[i] > NBMAX)
        return lrce_fail(LRCE_E_ARG, "wattn_dbias_batched: item %d (n_win=%d nH=%d n_bins=%d)", i, n_win[i], nH[i], n_bins[i]);
      b.it[j] = DbItem{dbias_part[i], bin_row[i], table_grad[i], n_win[i], nH[i], n_bins[i]};
      const int bx = (nH[i] * n_bins[i] + 255) / 256;
      gx = bx > gx ? bx : gx;
    }
    dbias_chunk_batched<<<dim3((unsigned)gx, WCH, (unsigned)m), 256, 0, st>>>(b);
    dbias_scatter_batched<<<dim3((unsigned)gx, 1, (unsigned)m), 256, 0, st>>>(b);
  }
  return lrce_check_launch("wattn_dbias_batched");
}
