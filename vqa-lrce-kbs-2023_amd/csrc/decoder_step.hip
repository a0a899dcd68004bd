// The recurrent LRCE decoder step as ONE persistent launch per recurrent step and direction
// (FusionTransformer.forward's clip loop, fusionv3.py:43-49, over the 12 nn.TransformerDecoderLayer of
// fusionv3.py:8-17: d_model 768, 12 heads x 64, FFN 3072 GELU, post-norm, eps 1e-12) on gfx950.
//
// Why: the step is a chain of M = B (10..64) row linears — 36 layer-steps, each four dependent
// launches of ~10-17 us on the per-block path (decoder.hip + the skinny FFN GEMMs), the chip mostly
// idle.  Here 12 x R workgroups (R = min(B, 10) row groups, one per CU: the LDS image of a weight
// slice keeps one per CU) stay resident for the whole step and hand rows to each other inside the
// launch, so nothing waits for a kernel boundary and every phase issues its weight loads BEFORE it
// waits for its input rows (the weights do not depend on them).
//
// Per layer l (forward):
//   A  (head h, row b):  [x3p_{l-1} = x2_{l-1} + drop(sum_j P_j + b2) for columns h*64..h*64+63 (the FFN
//                        partials of the previous layer, summed in slice order)] -> x0 = LN3_{l-1}(x3p)
//                        -> v_h -> head dropout -> W_o[:, h] v_h partial -> the last of the 12 heads of
//                        row b sums them: x1p = x0 + drop(. + b_o)              (as dec_sa_fwd)
//   B  (head h, row b):  x1 = LN1(x1p) -> q_h -> attention over the step's memory keys -> W_oc[:, h] ctx_h
//                        partial -> last head: x2p = x1 + drop(. + b_oc)         (as dec_ca_fwd)
//   C  (FFN slice j of 32 hidden units, ALL rows): x2 = LN2(x2p) -> pre = W1[j] x2 + b1 -> gd =
//                        drop(GELU(pre)) -> P_j = W2[:, j] gd (partial of linear2, written to a slab)
// then the step tail: x3 = LN3(x3p_11), tsum = x3 + s, s' = drop(LN_f(tsum)).  The backward mirrors it:
//   tail: du = drop'(ds), dt = LN_f'(du) = d x3 of layer 11;  per layer (11 .. 0):
//   FB (FFN slice j, all rows): dx3p = LN3'(dx3), df = drop'(dx3p), dgp_j = drop'(W2[:, j]^T df) gelu'(pre),
//                        Q_j = W1[j]^T dgp_j (partial of dx2)
//   CB (head h, row b):  dx2 = dx3p + sum_j Q_j (columns h*64..) -> LN2' -> ... (as dec_ca_bwd) -> dx1
//   SB (head h, row b):  LN1' -> ... (as dec_sa_bwd) -> dx0 = d x3 of layer l-1 (or, l = 0, ds_in of the
//                        previous step: dx0 + dt).
//
// Hand-offs: the payload is the flag.  Every hand-off buffer holds a sentinel bit pattern (0xFFFFFFFF,
// a NaN no arithmetic here produces: converted fp16 / bf16 NaNs and the hardware's canonical NaN all
// differ) until its producer stores the value with a 16-B write-through (sc1) store; a consumer reads
// the 16-B piece with an sc1 load and re-reads it (s_sleep between polls) while any of its four dwords
// is still the sentinel — dword stores are single-copy atomic, so no torn value is ever accepted.  No
// arrival counter, no drain before a signal: one store and one load per hand-off instead of store,
// drain, atomic, poll and load (tools/hop_probe.hip on the box: 0.93 us per 12-producer exchange
// against 4.35 us for the counter protocol, whose 120 atomics on one word alone serialise to 1.96 us).
// Buffers are re-armed in two ways:
//  * the head partial slabs and the FFN slice partials have ONE reader per piece, which stores the
//    sentinel back after reading it (and drains those stores before its next hand-off: the next write
//    of the piece is causally after that);
//  * the row mailboxes (many readers) are per layer, in two sets used by alternate launches: a launch
//    uses set (epoch & 1) and re-arms the other set, which the previous launch used; the epoch word
//    advances when the last workgroup finishes.
// Polls are bounded: after 0.5 s a wait records its code in status[0] and raises a sticky abort word,
// and every later wait gives up at once (the launch ends with garbage and the host raises; never a
// hang); lrce_dec_step_reset then re-arms the workspace.  Bytes written by earlier launches (weights,
// K/V, the forward's saved activations) are read with plain loads.  Every cross-workgroup sum is taken
// in a fixed order: deterministic.
//
// Residency: all 12 R workgroups must be resident at once (they wait for each other).  R <= 10 keeps
// the grid at <= 120 workgroups of one per CU, so even two such launches (two processes sharing a
// GPU) fit on the 256 CUs together.
#include "common.h"
#include "decoder_util.h"
#include "lrce_capi.h"

namespace {

constexpr int FF = 3072, FS = 32, NF = FF / FS, RMAX = 10, MAXB = LRCE_DEC_MAX_ROWS, RCH = 16;
constexpr int XP = 100, XROW = 8 * XP + 4;   // padded LDS row of 768: 8 parts of 96 (+4), rows 804 apart (MFMA row reads)
constexpr int NLMAX = LRCE_DEC_LAYERS;
// counter block (uint32): the finishing count, the sticky abort word, the launch epoch, the row count of
// the last launch (the rows of the mailbox set it used)
constexpr int C_DONE = 0, C_ABORT = 1, C_EPOCH = 2, C_LASTB = 3, CTR_WORDS = 16;
// workspace (f32, all sentinel between launches): two per-head partial slabs [MAXB][12][768], the FFN
// slice partials [NF][MAXB][768], then the row mailboxes: 2 sets x NKIND kinds x NLMAX layers x
// [MAXB][768].  Kinds, forward: x3p, x1p, x2p, x2 (LN2 output); backward: d x3 (the FFN block's
// input gradient), dx3p, dx2 (LN2 input gradient), dx1, dt (layer 0 only)
constexpr long long WS_SLAB = (long long)MAXB * H * E;
constexpr long long WS_P = (long long)NF * MAXB * E;
constexpr int NKIND = 5;
enum { K_X3P = 0, K_X1P = 1, K_X2P = 2, K_X2 = 3 };
enum { K_DLN3 = 0, K_DRES = 1, K_DLN2 = 2, K_DLN1 = 3, K_DT = 4 };
constexpr long long MB_KIND = (long long)NLMAX * MAXB * E;
constexpr long long WS_MB = 2LL * NKIND * MB_KIND;
constexpr long long WS_ELEMS = 2 * WS_SLAB + WS_P + WS_MB;
constexpr unsigned SENT = 0xFFFFFFFFu;

// ---- arena layout (shared with the host through lrce_dec_step_field)
constexpr int NFWD = 18, NBWD = 9;
__host__ __device__ constexpr int fwd_width(int f) {
  return f <= 8 ? E : f <= 10 ? FF : f == 11 ? H : 1;   // x0 sad x1p x1 q ctx x2p x2 x3p | pre gd | lse | m1 r1 m2 r2 m3 r3
}
__host__ __device__ constexpr int bwd_width(int f) { return f == 1 ? FF : E; }   // df dgp dcao dq dsao dsav dln1 dln2 dln3
__host__ __device__ inline long long field_off(int kind, int f, int l, int B, int S) {
  const int nf = kind ? NBWD : NFWD;
  long long pre = 0, tot = 0;
  for (int i = 0; i < nf; ++i) {
    const int w = kind ? bwd_width(i) : fwd_width(i);
    if (i < f) pre += w;
    tot += w;
  }
  const long long block = ((long long)S * B * tot + 63) / 64 * 64;
  return (long long)l * block + (long long)S * B * pre;
}
enum { F_X0 = 0, F_SAD, F_X1P, F_X1, F_Q, F_CTX, F_X2P, F_X2, F_X3P, F_PRE, F_GD, F_LSE, F_M1, F_R1, F_M2, F_R2, F_M3, F_R3 };
enum { G_DF = 0, G_DGP, G_DCAO, G_DQ, G_DSAO, G_DSAV, G_DLN1, G_DLN2, G_DLN3 };

struct Ar {   // one arena field at (layer, step): row b at base + b * width
  float* base;
  int w;
  __device__ float* row(int b) const { return base + (long long)b * w; }
};
__device__ __forceinline__ Ar fwd_field(const LrceDecStep& p, int f, int l, int step) {
  return Ar{p.acts + field_off(0, f, l, p.B, p.S) + (long long)step * p.B * fwd_width(f), fwd_width(f)};
}
__device__ __forceinline__ Ar bwd_field(const LrceDecStep& p, int f, int l, int step) {
  return Ar{p.grads + field_off(1, f, l, p.B, p.S) + (long long)step * p.B * bwd_width(f), bwd_width(f)};
}

// ---- write-through hand-off accesses: 16-B buffer loads / stores with the sc1 bit.  The buffer
// descriptor must be wave-uniform (SGPRs): a per-lane pointer would make hipcc loop over the lanes
// (a waterfall of 64 descriptor builds per access), so every call takes a uniform base (forced with
// readfirstlane) and a per-lane element offset.
__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc_of(const void* p) {
  const uint64_t a = reinterpret_cast<uintptr_t>(p);
  const uint64_t u = (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)a) |
                     ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)(a >> 32)) << 32);
  return __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<void*>(u), (short)0, 0x7FFFFFFF, 0x00020000);
}
__device__ __forceinline__ float4 ld4_sc1(const float* base, long long off) {   // 16 B, sc1 (L1 bypass): a handed-off row
  const auto v = __builtin_amdgcn_raw_buffer_load_b128(rsrc_of(base), (int)(off * 4), 0, 16);
  return __builtin_bit_cast(float4, v);
}
__device__ __forceinline__ void st4_sc1(float* base, long long off, float4 v) {   // 16 B, sc1 (write-through)
  __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(__attribute__((ext_vector_type(4))) unsigned, v),
                                         rsrc_of(base), (int)(off * 4), 0, 16);
}
__device__ __forceinline__ float ld_sc1(const float* p) { return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }
__device__ __forceinline__ void st_sc1(float* p, float v) { __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }
__device__ __forceinline__ float4 add4(float4 a, float4 b) { return make_float4(a.x + b.x, a.y + b.y, a.z + b.z, a.w + b.w); }
__device__ __forceinline__ float4 lds4(const float* p) { return *reinterpret_cast<const float4*>(p); }
// y / (1 - p) where the element's uniform >= p, else 0: the mask of lrce_dropout over [rows][768] for elements e .. e+3
__device__ __forceinline__ float4 drop4(float4 y, float p, uint64_t seed, long long e) {
  if (p <= 0.f) return y;
  const float4 u = lrce_uniform4(seed, (uint64_t)e >> 2);
  const float k = 1.0f - p;
  return make_float4(u.x >= p ? y.x / k : 0.f, u.y >= p ? y.y / k : 0.f, u.z >= p ? y.z / k : 0.f, u.w >= p ? y.w / k : 0.f);
}

__device__ __forceinline__ bool unset4(float4 v) {
  return __float_as_uint(v.x) == SENT || __float_as_uint(v.y) == SENT || __float_as_uint(v.z) == SENT ||
         __float_as_uint(v.w) == SENT;
}
__device__ __forceinline__ float4 sent4() {
  const float f = __uint_as_float(SENT);
  return make_float4(f, f, f, f);
}
// A handed-off 16-B piece: re-read (s_sleep between polls) while any dword is still the sentinel.
// Bounded: every 64 polls the sticky abort word is checked; after SPIN_MAX polls (~0.5 s: each poll is
// a memory round trip) the wait gives up through wait_fail (raises the abort word, records the code).
constexpr unsigned SPIN_MAX = 1u << 20;
__device__ __attribute__((noinline)) void wait_fail(unsigned* ctrs, unsigned* status, unsigned code) {
  __hip_atomic_store(ctrs + C_ABORT, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  unsigned zero = 0;
  __hip_atomic_compare_exchange_strong(status, &zero, code, __ATOMIC_RELAXED, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ float4 ld4_wait(const float* base, long long off, const LrceDecStep& p, unsigned code) {
  float4 v = ld4_sc1(base, off);
  unsigned it = 0;
  while (unset4(v)) {
    __builtin_amdgcn_s_sleep(1);
    v = ld4_sc1(base, off);
    if ((++it & 63u) == 0 &&
        (it >= SPIN_MAX || __hip_atomic_load(p.counters + C_ABORT, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))) {
      if (it >= SPIN_MAX) wait_fail(p.counters, p.status, code);
      break;
    }
  }
  return v;
}

// this head's partial row (LDS part[768], 16-B aligned) -> slab[b][h] (write-through)
__device__ __forceinline__ void publish(const float* part, float* slab, int b, int h) {
  const int t = threadIdx.x;
  if (t < E / 4) st4_sc1(slab, ((long long)b * H + h) * E + 4 * t, lds4(part + 4 * t));
}
// columns h*64 .. h*64+63 of row b summed over the 12 heads' partials in head order (thread q < 16
// returns columns 4q .. 4q+3): thread (j, q) waits for its piece of head j, stores the sentinel back
// (this workgroup is the piece's only reader) and the sum runs through red.  The re-arming stores are
// drained before the caller's next hand-off (s_waitcnt vmcnt(0) in the caller's path).
__device__ float4 gather_cols(float* slab, int b, int h, float4 (&red)[16][16], const LrceDecStep& p, unsigned code) {
  const int t = threadIdx.x;
  if (t < H * 16) {
    const int j = t >> 4, q = t & 15;
    const long long off = ((long long)b * H + j) * E + h * D + 4 * q;
    red[j][q] = ld4_wait(slab, off, p, code);
    st4_sc1(slab, off, sent4());
  }
  lds_barrier();
  float4 s = make_float4(0.f, 0.f, 0.f, 0.f);
  if (t < 16) {
    s = red[0][t];
#pragma unroll
    for (int j = 1; j < H; ++j) s = add4(s, red[j][t]);
  }
  lds_barrier();
  return s;
}

// threadIdx.x through an empty asm: lane-derived values computed from it inside a loop body stay in
// that body (the compiler cannot hoist them out of the layer loop and keep them live, or spill them,
// across every phase)
__device__ __forceinline__ int opaque_tid() {
  int v = threadIdx.x;
  asm volatile("" : "+v"(v));
  return v;
}
// the thread index a shared helper uses: opaque in the backward kernel (O = true: its per-lane
// offsets are recomputed in each phase instead of hoisted and spilled), plain in the forward (which
// does not spill and measured faster with the hoisted form)
template <bool O>
__device__ __forceinline__ int tid_() { return O ? opaque_tid() : (int)threadIdx.x; }

// the row mailboxes of one set: kind k, layer l, row b at mb(...) + b * E
__device__ __forceinline__ float* mb_of(const LrceDecStep& p, unsigned set, int kind, int l) {
  return p.ws + 2 * WS_SLAB + WS_P + ((long long)(set * NKIND + kind) * NLMAX + l) * MAXB * E;
}
// the launch's epoch (read by every workgroup before any finishes) and the re-arming of the other set,
// which the previous launch used (it has ended): the rows it wrote — its row count, which may differ
// from this launch's — of every kind and layer, sentinel stores
__device__ unsigned launch_begin(const LrceDecStep& p) {
  const unsigned ep = __hip_atomic_load(p.counters + C_EPOCH, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const unsigned pb = __hip_atomic_load(p.counters + C_LASTB, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const unsigned other = (ep + 1) & 1u;
  const long long per = (long long)(pb < (unsigned)MAXB ? pb : (unsigned)MAXB) * (E / 4);   // float4 pieces of one (kind, layer)
  const long long tot = (long long)NKIND * NLMAX * per;
  for (long long i = (long long)blockIdx.x * NT + opaque_tid(); i < tot; i += (long long)gridDim.x * NT) {
    const long long kl = i / per, e = i % per;
    st4_sc1(mb_of(p, other, (int)(kl / NLMAX), (int)(kl % NLMAX)), 4 * e, sent4());
  }
  return ep & 1u;
}

// the last workgroup to finish zeroes the finishing count and advances the epoch (the next launch
// then uses the other mailbox set)
__device__ void finish(const LrceDecStep& p, unsigned* last_word) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (opaque_tid() == 0)
    *last_word = __hip_atomic_fetch_add(p.counters + C_DONE, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == gridDim.x - 1;
  __syncthreads();
  if (!*last_word || opaque_tid() != 0) return;
  __hip_atomic_store(p.counters + C_DONE, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __hip_atomic_store(p.counters + C_LASTB, (unsigned)p.B, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __hip_atomic_fetch_add(p.counters + C_EPOCH, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Debug phase timestamps (lrce_dec_step_set_trace; NULL in production): thread 0 of workgroup w stores
// s_memrealtime (100 MHz) at mark i of layer l into trace[((dir * 128 + w) * 16 + l) * 8 + i].
unsigned long long* g_step_trace = nullptr;
// sub-phase marks inside the FFN slices of layer 1 (slot 14 of the layer index)
#define SUB_MARK(DIR, I)                                                                                  \
  do {                                                                                                    \
    if (trace && l == 1 && opaque_tid() == 0)                                                              \
      trace[(((DIR) * 128 + blockIdx.x) * 16 + 14) * 8 + (I)] = __builtin_amdgcn_s_memrealtime();         \
  } while (0)
#define STEP_MARK_P(DIR, L, I) do { } while (0)
#define STEP_MARK(DIR, L, I)                                                                              \
  do {                                                                                                    \
    if (trace && opaque_tid() == 0)                                                                        \
      trace[(((DIR) * 128 + blockIdx.x) * 16 + (L)) * 8 + (I)] = __builtin_amdgcn_s_memrealtime();       \
  } while (0)
__device__ __forceinline__ uint64_t layer_seed(const LrceDecStep& p, int l) {
  return p.seed + 64ull * (uint64_t)(p.step * p.n_layers + l);
}
__device__ __forceinline__ uint64_t tail_seed(const LrceDecStep& p) { return p.seed + 7ull + 64000ull * (uint64_t)(p.step + 1); }

__device__ __forceinline__ KvP kv_of(const LrceDecStep& p, int l) {
  KvP k;
  k.k1 = reinterpret_cast<const bf16*>(p.kv_video) + l * p.kv_video_lstride + (long long)p.step * 150 * 2 * E;
  k.stride1 = (long long)p.S * 150 * 2 * E;
  k.ld1 = 2 * E;
  k.bdiv1 = p.nmc;
  k.lk1 = 150;
  k.k2 = p.lt ? reinterpret_cast<const bf16*>(p.kv_text) + l * p.kv_text_lstride : nullptr;
  k.stride2 = (long long)p.lt * 2 * E;
  k.ld2 = 2 * E;
  k.bdiv2 = 1;
  k.lk2 = p.lt;
  k.v_off = E;
  return k;
}

// ------------------------------------------------------------------------------------ LDS images
struct SaL {                      // self-attention block (forward and backward)
  f16 wo[E * D];
  alignas(16) float x0[E];
  float pp[4][16 * 64];
  alignas(16) float v[D];
  alignas(16) float part[E];
  alignas(16) float dx1p[E];
  float dsao[E];
  float red64[4][D];
  alignas(16) float acc[4][E];
  float red2[4];
  unsigned last;
};
struct CaL {                      // cross-attention block: forward and backward images share the tail
  f16 wo[E * D];
  bf16 vimg[MAXK * D];
  union {
    struct {                      // forward
      alignas(16) float x1[E];
      float pp[4][16 * 64];
      float q[D];
      float ps[MAXK + 64];
      float opart[4][D];
      alignas(16) float ctx[D];
      alignas(16) float part[E];
    } f;
    struct {                      // backward
      union {
        bf16 kimg[MAXK * D];
        alignas(16) float acc[4][E];
      };
      alignas(16) float dx2p[E];
      float dcao[E];
      float red64[4][D];
      float dctx[D];
      float dq[D];
      float q[D];
      float ps[MAXK + 64];
      float dss[MAXK + 64];
    } b;
  };
  float red2[4];
  unsigned last;
};
struct FfL {                      // FFN slices over all rows (MFMA: the rows are the 16 M lanes)
  alignas(16) float x[RCH * XROW];   // the chunk's input rows (padded), then the output partial tile
  alignas(16) float hb[RCH][FS + 4]; // the hidden slice (forward: dropped GELU; backward: dgp)
  float kacc[2][16][16];          // the second K half of the hidden-slice product
  f16 w2s[E * FS];                // backward: the W2 column slice [768][32]
  f16 w1s[FS * E];                // backward: the W1 row slice [32][768]
  float preb[RCH][FS];            // backward: the saved pre-activations of the chunk's rows
  float rsc[RCH], rinv[RCH];      // backward: per-row power-of-two scale of the f16-split MFMA operands
};
struct RedL {                     // the FFN-partial reduce (outside the union: the next phase's weight
  float4 red[16][16];             // slices stream into the union while it runs)
};
union StepLds {
  SaL sa;
  CaL ca;
  FfL ff;
};

// ---------------------------------------------------------------------------- FFN partial reduce
// columns h*64 .. h*64+63 of row b: out = base + epi(sum_j P[j][b][..]) over the NF slices in slice order
// (16 groups of 6, then the groups in order); fwd: base = x2, epi = drop(. + b2, seed); bwd: base =
// dx3p, epi = identity.  P pieces are waited for and re-armed (this workgroup is their only reader),
// base is a mailbox row (waited for); out goes to the mailbox row (sc1) and to the arena row `keep`.
// Ends with the re-arming stores drained (before this workgroup's next hand-off).
template <bool O>
__device__ void slice_reduce(float* P, int b, int h, const float* bias, float drop_p, uint64_t seed, const float* base_row,
                             float* out_row, float* keep, RedL& L, const LrceDecStep& p, unsigned code) {
  const int t = tid_<O>(), q = t & 15, g = t >> 4;
  const int col = h * D + 4 * q;
  float4 s = make_float4(0.f, 0.f, 0.f, 0.f);
  float4 v[NF / 16];
#pragma unroll
  for (int i = 0; i < NF / 16; ++i) v[i] = ld4_sc1(P, ((long long)(g + 16 * i) * MAXB + b) * E + col);
#pragma unroll
  for (int i = 0; i < NF / 16; ++i) {
    const long long off = ((long long)(g + 16 * i) * MAXB + b) * E + col;
    if (unset4(v[i])) v[i] = ld4_wait(P, off, p, code);
    st4_sc1(P, off, sent4());
  }
#pragma unroll
  for (int i = 0; i < NF / 16; ++i) { s.x += v[i].x; s.y += v[i].y; s.z += v[i].z; s.w += v[i].w; }
  L.red[g][q] = s;
  lds_barrier();
  if (t < 16) {
    float4 a = L.red[0][q];
#pragma unroll
    for (int i = 1; i < 16; ++i) { const float4 r = L.red[i][q]; a.x += r.x; a.y += r.y; a.z += r.z; a.w += r.w; }
    if (bias) {
      const float4 bb = *reinterpret_cast<const float4*>(bias + col);
      a = make_float4(a.x + bb.x, a.y + bb.y, a.z + bb.z, a.w + bb.w);
      if (drop_p > 0.f) {
        const long long e = (long long)b * E + col;
        const float4 u = lrce_uniform4(seed, (uint64_t)e >> 2);
        const float k = 1.0f - drop_p;
        a.x = u.x >= drop_p ? a.x / k : 0.f; a.y = u.y >= drop_p ? a.y / k : 0.f;
        a.z = u.z >= drop_p ? a.z / k : 0.f; a.w = u.w >= drop_p ? a.w / k : 0.f;
      }
    }
    const float4 r = ld4_wait(base_row, col, p, code + 0x1000);
    const float4 o = make_float4(r.x + a.x, r.y + a.y, r.z + a.z, r.w + a.w);
    st4_sc1(out_row, col, o);
    *reinterpret_cast<float4*>(keep + col) = o;
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  lds_barrier();
}

// W rows h*64 .. h*64+63 of a row-major [768][768] fp16 matrix -> LDS [64][768] (96 KB contiguous: 24
// LDS-DMA instructions of 1 KB per wave)
__device__ __forceinline__ void rows_dma(const f16* w, int h, void* lds, int wave, int lane) {
  const uint32_t base = dec_lds_addr(lds);
#pragma unroll 4
  for (int i = 0; i < 24; ++i) {
    const int ins = wave * 24 + i;
    dec_glds(w, (uint32_t)(h * D * E * 2 + ins * 1024 + lane * 16), base + (uint32_t)ins * 1024u);
  }
}
// part[4t .. 4t+3] (t < 192) = sum_r v[r] W[r][4t .. 4t+3] over the 64 LDS rows (the transposed product W^T v of
// a backward dX partial: each thread sums all 64 rows of its 4 columns, no cross-wave reduction)
__device__ __forceinline__ void rows_t_lds(const f16* Wl, const float* v, float* part) {
  const int t = opaque_tid();
  if (t >= E / 4) return;
  float4 a = make_float4(0.f, 0.f, 0.f, 0.f), c = a;
#pragma unroll 8
  for (int r = 0; r < D; r += 2) {
    const uint2 u0 = *reinterpret_cast<const uint2*>(Wl + r * E + 4 * t);
    const uint2 u1 = *reinterpret_cast<const uint2*>(Wl + (r + 1) * E + 4 * t);
    const float v0 = v[r], v1 = v[r + 1];
    const float4 w0 = make_float4((float)__builtin_bit_cast(f16, (unsigned short)(u0.x & 0xFFFFu)), (float)__builtin_bit_cast(f16, (unsigned short)(u0.x >> 16)),
                                  (float)__builtin_bit_cast(f16, (unsigned short)(u0.y & 0xFFFFu)), (float)__builtin_bit_cast(f16, (unsigned short)(u0.y >> 16)));
    const float4 w1 = make_float4((float)__builtin_bit_cast(f16, (unsigned short)(u1.x & 0xFFFFu)), (float)__builtin_bit_cast(f16, (unsigned short)(u1.x >> 16)),
                                  (float)__builtin_bit_cast(f16, (unsigned short)(u1.y & 0xFFFFu)), (float)__builtin_bit_cast(f16, (unsigned short)(u1.y >> 16)));
    a.x = fmaf(v0, w0.x, a.x); a.y = fmaf(v0, w0.y, a.y); a.z = fmaf(v0, w0.z, a.z); a.w = fmaf(v0, w0.w, a.w);
    c.x = fmaf(v1, w1.x, c.x); c.y = fmaf(v1, w1.y, c.y); c.z = fmaf(v1, w1.z, c.z); c.w = fmaf(v1, w1.w, c.w);
  }
  *reinterpret_cast<float4*>(part + 4 * t) = make_float4(a.x + c.x, a.y + c.y, a.z + c.z, a.w + c.w);
}

// ------------------------------------------------------------------- forward: self-attention row
// x0 (LDS) is ready; v_h -> head dropout -> partial (published) -> this workgroup's 64 columns of row b:
// x1p = x0 + drop(sum of the 12 partials + b_o), into the x1p mailbox (and the arena).  wr: W_v[h] rows
// (registers), L.wo: the W_o slice (DMA'd; waited for here)
__device__ void sa_fwd_row(const LrceDecStep& p, int l, int b, int h, const f16* wv, float bvv, SaL& L,
                           uint64_t seed0, uint64_t seed1, bool wait_dma, RedL& RD, float* mbx1) {
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const LrceDecLayerW& W = p.layer[l];
  {
    uint4 wr[NRI];   // W_v[h] rows, loaded at use: held across the row's waits they cost spills
    rows_load(wv, h * D + wave * WROWS, lane, wr);
    rows_gemv(wr, L.x0, L.pp[wave], L.v + wave * WROWS, lane);
  }
  lds_barrier();
  if (t < D) {
    float v = L.v[t] + bvv;
    if (p.drop_p > 0.f) v = drop1(v, p.drop_p, seed0, ((long long)b * E + h * D + t) / D);
    L.v[t] = v;
    fwd_field(p, F_SAD, l, p.step).row(b)[h * D + t] = v;
  }
  if (wait_dma) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  lds_barrier();
  slice_gemv(L.wo, L.v, L.part, t);
  lds_barrier();
  publish(L.part, p.ws, b, h);
  const float4 sm = gather_cols(p.ws, b, h, RD.red, p, 0x200 + l);
  if (t < 16) {
    const int c = h * D + 4 * t;
    const float4 y = drop4(add4(sm, lds4(W.bo + c)), p.drop_p, seed1, (long long)b * E + c);
    const float4 o = add4(lds4(L.x0 + c), y);
    st4_sc1(mbx1 + (long long)b * E, c, o);
    *reinterpret_cast<float4*>(fwd_field(p, F_X1P, l, p.step).row(b) + c) = o;
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // the re-arming stores, before the next hand-off
}

// ------------------------------------------------------------------ forward: cross-attention row
// what a cross-attention row needs that nothing in this launch writes: the key row of thread t
// (registers) and the head's V rows (LDS DMA) — issued before the row's wait
__device__ void ca_fwd_prefetch(const LrceDecStep& p, int l, int b, int h, CaL& L, uint4 (&kr)[8]) {
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const KvP kv = kv_of(p, l);
  const int Lk = kv.lk1 + kv.lk2;
  const KvRows kvr = kv_rows(kv, b, h);
  {
    const bf16* kp = kv_row(kvr, t < Lk ? t : 0);
#pragma unroll
    for (int c = 0; c < 8; ++c) kr[c] = *reinterpret_cast<const uint4*>(kp + 8 * c);
  }
  const uint32_t vb = dec_lds_addr(L.vimg);
  for (int ins = wave; ins * 8 < Lk; ins += 4) {
    const int r = ins * 8 + (lane >> 3), j = min(r, Lk - 1);
    const bf16* vp = kv_row(kvr, j) + kv.v_off + (((lane & 7) ^ (r & 7)) << 3);
    dec_glds_p(vp, vb + (uint32_t)ins * 1024u);
  }
}

__device__ void ca_fwd_row(const LrceDecStep& p, int l, int b, int h, const f16* wq, float bqv, CaL& L,
                           uint64_t seed2, uint64_t seed3, const uint4 (&kr)[8], RedL& RD, const float* mbx1, float* mbx2) {
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const LrceDecLayerW& W = p.layer[l];
  const KvP kv = kv_of(p, l);
  const int Lk = kv.lk1 + kv.lk2;
  float4 xr = make_float4(0.f, 0.f, 0.f, 0.f), gg = xr, be = xr;
  if (t < E / 4) {
    gg = *reinterpret_cast<const float4*>(W.g1 + 4 * t);
    be = *reinterpret_cast<const float4*>(W.be1 + 4 * t);
    xr = ld4_wait(mbx1 + (long long)b * E, 4 * t, p, 0x300 + l);
  }
  const float s1l = row_sum_local(xr, t);
  const bool live = t < Lk;
  float mu, rs;
  ln_row_fwd(xr, s1l, gg, be, p.eps, L.f.x1, L.red2, t, lane, wave, mu, rs);
  if (h == 0) {
    if (t < E / 4) *reinterpret_cast<float4*>(fwd_field(p, F_X1, l, p.step).row(b) + 4 * t) = *reinterpret_cast<const float4*>(L.f.x1 + 4 * t);
    if (t == 0) {
      fwd_field(p, F_M1, l, p.step).row(b)[0] = mu;
      fwd_field(p, F_R1, l, p.step).row(b)[0] = rs;
    }
  }
  lds_barrier();
  {
    uint4 wr[NRI];
    rows_load(wq, h * D + wave * WROWS, lane, wr);
    rows_gemv(wr, L.f.x1, L.f.pp[wave], L.f.q + wave * WROWS, lane);
  }
  lds_barrier();
  if (t < D) {
    const float q = L.f.q[t] + bqv;
    fwd_field(p, F_Q, l, p.step).row(b)[h * D + t] = q;
    L.f.q[t] = q * 0.125f;
  }
  lds_barrier();
  float sc = 0.f;
  if (live) {
#pragma unroll
    for (int c = 0; c < 8; ++c) {
      const unsigned w4[4] = {kr[c].x, kr[c].y, kr[c].z, kr[c].w};
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        sc += bfbits2f((unsigned short)(w4[e] & 0xFFFFu)) * L.f.q[8 * c + 2 * e];
        sc += bfbits2f((unsigned short)(w4[e] >> 16)) * L.f.q[8 * c + 2 * e + 1];
      }
    }
  }
  const float m = block_max4(live ? sc : -1.0e30f, L.red2, lane, wave);
  const float pe = live ? __expf(sc - m) : 0.f;
  const float s = block_sum4(pe, L.red2, lane, wave);
  float pf = pe;
  if (live && p.drop_p > 0.f) pf = drop1(pe, p.drop_p, seed2, ((long long)b * H + h) * Lk + t);
  L.f.ps[t] = live ? pf : 0.f;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // V rows (and, first row, the W_oc slice) have landed
  lds_barrier();
  {
    const int c = t & 7, kg = t >> 3;
    float a[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll 2
    for (int j = kg; j < Lk; j += 32) {
      float vf[8];
      unpack8bf(*reinterpret_cast<const uint4*>(L.vimg + kv_swz(j, c)), vf);
      const float pj = L.f.ps[j];
#pragma unroll
      for (int e = 0; e < 8; ++e) a[e] = fmaf(pj, vf[e], a[e]);
    }
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      a[e] += dpp_f<0x128>(a[e]);
      a[e] += __shfl_xor(a[e], 16, 64);
      a[e] += __shfl_xor(a[e], 32, 64);
    }
    if (lane < 8) {
#pragma unroll
      for (int e = 0; e < 8; ++e) L.f.opart[wave][c * 8 + e] = a[e];
    }
  }
  lds_barrier();
  if (t < D) {
    const float c = ((L.f.opart[0][t] + L.f.opart[1][t]) + (L.f.opart[2][t] + L.f.opart[3][t])) / s;
    L.f.ctx[t] = c;
    fwd_field(p, F_CTX, l, p.step).row(b)[h * D + t] = c;
    if (t == 0) fwd_field(p, F_LSE, l, p.step).row(b)[h] = m + __logf(s);
  }
  lds_barrier();
  slice_gemv(L.wo, L.f.ctx, L.f.part, t);
  lds_barrier();
  publish(L.f.part, p.ws + WS_SLAB, b, h);
  const float4 sm = gather_cols(p.ws + WS_SLAB, b, h, RD.red, p, 0x400 + l);
  if (t < 16) {
    const int c = h * D + 4 * t;
    const float4 y = drop4(add4(sm, lds4(W.boc + c)), p.drop_p, seed3, (long long)b * E + c);
    const float4 o = add4(lds4(L.f.x1 + c), y);
    st4_sc1(mbx2 + (long long)b * E, c, o);
    *reinterpret_cast<float4*>(fwd_field(p, F_X2P, l, p.step).row(b) + c) = o;
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // the re-arming stores, before the next hand-off
}

// ------------------------------------------------------------------------ FFN: rows into LDS
// rows c0 .. c0+nr-1 of a [B][768] row mailbox into the padded image L.x: all 12 loads per thread in
// flight at once, then the pieces not yet written are waited for
template <bool O>
__device__ __forceinline__ void rows_to_lds(const float* src, int c0, int nr, FfL& L, const LrceDecStep& p, unsigned code) {
  constexpr int PER = RCH * (E / 4) / NT;
  float4 v[PER];
#pragma unroll
  for (int q = 0; q < PER; ++q) {
    const int i = tid_<O>() + q * NT, rr = i / (E / 4), k = (i % (E / 4)) * 4;
    v[q] = rr < nr ? ld4_sc1(src, (long long)(c0 + rr) * E + k) : make_float4(0.f, 0.f, 0.f, 0.f);
  }
#pragma unroll
  for (int q = 0; q < PER; ++q) {
    const int i = tid_<O>() + q * NT, rr = i / (E / 4), k = (i % (E / 4)) * 4;
    if (rr < nr && unset4(v[q])) v[q] = ld4_wait(src, (long long)(c0 + rr) * E + k, p, code);
    *reinterpret_cast<float4*>(L.x + rr * XROW + (k / 96) * XP + (k % 96)) = v[q];
  }
}
// element k of padded row rr
__device__ __forceinline__ float* xat(FfL& L, int rr, int k) { return L.x + rr * XROW + (k / 96) * XP + (k % 96); }

// wave-per-row LayerNorm (forward) of the image rows in place; lane owns k = 12 lane .. 12 lane + 11
// full-wave sum without LDS round trips (a __shfl_xor butterfly is six dependent ds_bpermute): DPP within
// 16-lane rows, then the four row sums by v_readlane
__device__ __forceinline__ float wave_sum_dpp(float v) {
  v += dpp_f<0xB1>(v);    // quad_perm [1,0,3,2]
  v += dpp_f<0x4E>(v);    // quad_perm [2,3,0,1]
  v += dpp_f<0x141>(v);   // row_half_mirror
  v += dpp_f<0x140>(v);   // row_mirror: every lane holds its 16-lane row's sum
  // the four row sums through the scalar unit (uniform result, in row order)
  const float r0 = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), 0));
  const float r1 = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), 16));
  const float r2 = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), 32));
  const float r3 = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), 48));
  return (r0 + r1) + (r2 + r3);
}
__device__ __forceinline__ float wave_max_dpp(float v) {   // v >= 0
  v = fmaxf(v, dpp_f<0xB1>(v));
  v = fmaxf(v, dpp_f<0x4E>(v));
  v = fmaxf(v, dpp_f<0x141>(v));
  v = fmaxf(v, dpp_f<0x140>(v));
  const float r0 = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), 0));
  const float r1 = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), 16));
  const float r2 = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), 32));
  const float r3 = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), 48));
  return fmaxf(fmaxf(r0, r1), fmaxf(r2, r3));
}
// the four rows of a wave reduced together (independent chains: their latencies overlap)
__device__ __forceinline__ void wave_sum_x4(float (&v)[4]) {
#pragma unroll
  for (int q = 0; q < 4; ++q) v[q] = wave_sum_dpp(v[q]);
}

// wave-per-row LayerNorm (forward) of the image rows in place, the wave's rows rr = wave + 4 q (q < 4)
// processed together; lane owns k = 12 lane .. 12 lane + 11
__device__ void ln_rows_fwd(FfL& L, int nr, const float* g, const float* be, float eps, float* mean_out, float* rstd_out,
                            float* y_rows /* sc1-stored mailbox copy or NULL */, float* y_keep /* arena copy */, int c0) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  float4 v[4][3];
  float s1[4], s2[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const float* xp = xat(L, wave + 4 * q, 12 * lane);   // rows >= nr are zero
#pragma unroll
    for (int i = 0; i < 3; ++i) v[q][i] = *reinterpret_cast<const float4*>(xp + 4 * i);
    s1[q] = 0.f;
#pragma unroll
    for (int i = 0; i < 3; ++i) s1[q] += (v[q][i].x + v[q][i].y) + (v[q][i].z + v[q][i].w);
  }
  wave_sum_x4(s1);
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const float mu = s1[q] * (1.0f / E);
    s2[q] = 0.f;
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      const float4 d = make_float4(v[q][i].x - mu, v[q][i].y - mu, v[q][i].z - mu, v[q][i].w - mu);
      s2[q] += (d.x * d.x + d.y * d.y) + (d.z * d.z + d.w * d.w);
    }
  }
  wave_sum_x4(s2);
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int rr = wave + 4 * q;
    if (rr >= nr) break;
    const float mu = s1[q] * (1.0f / E), rs = rsqrtf(s2[q] * (1.0f / E) + eps);
    float* xp = xat(L, rr, 12 * lane);
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      const int k = 12 * lane + 4 * i;
      const float4 gg = *reinterpret_cast<const float4*>(g + k), bb = *reinterpret_cast<const float4*>(be + k);
      const float4 y = make_float4((v[q][i].x - mu) * rs * gg.x + bb.x, (v[q][i].y - mu) * rs * gg.y + bb.y,
                                   (v[q][i].z - mu) * rs * gg.z + bb.z, (v[q][i].w - mu) * rs * gg.w + bb.w);
      *reinterpret_cast<float4*>(xp + 4 * i) = y;
      if (y_rows) {
        st4_sc1(y_rows, (long long)(c0 + rr) * E + k, y);
        *reinterpret_cast<float4*>(y_keep + (long long)(c0 + rr) * E + k) = y;
      }
    }
    if (lane == 0 && mean_out) {
      mean_out[c0 + rr] = mu;
      rstd_out[c0 + rr] = rs;
    }
  }
}

// --------------------------------------------------------------------------- forward: FFN slice j
// 16 k of an f32 x fp16 product on the f16 MFMA: a split into hi = f16(a) and lo = f16(a - hi)
// (a = hi + lo to ~22 bits: the products of fp16 weights with either part are exact in f32), two
// v_mfma_f32_16x16x16_f16 (K = 16, 8 passes each) in place of four f32 16x16x4 (32 passes each) and
// the weight conversions.  A(i = lane & 15, k0 + 4 (lane >> 4) + e), C row 4 (lane >> 4) + r, column
// lane & 15.  b: four fp16 of B(k0 + 4 (lane >> 4) + e, j).  For operands of order one
// (LayerNorm outputs, GELU activations): no scaling needed for the f16 range.
typedef __attribute__((ext_vector_type(4))) _Float16 f16x4v;
__device__ __forceinline__ f32x4 mfma_sp(float4 a, uint2 b, f32x4 c) {
  const f16x4v hi = {(f16)a.x, (f16)a.y, (f16)a.z, (f16)a.w};
  const f16x4v lo = {(f16)(a.x - (float)hi[0]), (f16)(a.y - (float)hi[1]), (f16)(a.z - (float)hi[2]), (f16)(a.w - (float)hi[3])};
  const f16x4v bb = __builtin_bit_cast(f16x4v, b);
  c = __builtin_amdgcn_mfma_f32_16x16x16f16(hi, bb, c, 0, 0, 0);
  return __builtin_amdgcn_mfma_f32_16x16x16f16(lo, bb, c, 0, 0, 0);
}

// C tiles of one wave (12 column tiles of 16 over the 768 outputs, rows = the chunk's 16 rows) -> the
// padded image, then the chunk's live rows -> dst (write-through 16-B stores)
template <bool O>
__device__ __forceinline__ void tiles_out(FfL& L, const f32x4 (&acc)[12], float* dst, int c0, int nr) {
  const int lane = tid_<O>() & 63, wave = tid_<O>() >> 6, col = lane & 15, kq = lane >> 4;
#pragma unroll
  for (int tt = 0; tt < 12; ++tt)
#pragma unroll
    for (int r = 0; r < 4; ++r) *xat(L, 4 * kq + r, (wave * 12 + tt) * 16 + col) = acc[tt][r];
  lds_barrier();
  constexpr int PER = RCH * (E / 4) / NT;
#pragma unroll
  for (int q = 0; q < PER; ++q) {
    const int i = tid_<O>() + q * NT, rr = i / (E / 4), k = (i % (E / 4)) * 4;
    if (rr < nr) st4_sc1(dst, (long long)(c0 + rr) * E + k, *reinterpret_cast<const float4*>(xat(L, rr, k)));
  }
}

// the FFN slice's weights into LDS by DMA: W2[:, j*32 .. +32] -> [768][32] (row n = 4 chunks of 16 B) and
// W1[j*32 .. +32][:] -> [32][768] (row c = 96 chunks); 12 + 12 instructions of 1 KB per wave.  The MFMA
// B fragments are read from these images right before each use (nothing held in registers across a wait).
__device__ __forceinline__ void ffn_slices_dma(const f16* w1, const f16* w2, int j, FfL& L, int wave, int lane) {
  const uint32_t b2 = dec_lds_addr(L.w2s), b1 = dec_lds_addr(L.w1s);
#pragma unroll
  for (int i = 0; i < 12; ++i) {
    const int ins = wave * 12 + i;
    const int n = ins * 16 + (lane >> 2);
    dec_glds(w2, (uint32_t)(((long long)n * FF + j * FS + (lane & 3) * 8) * 2), b2 + (uint32_t)ins * 1024u);
    const int chunk = ins * 64 + lane;
    dec_glds(w1, (uint32_t)(((long long)(j * FS + chunk / 96) * E + (chunk % 96) * 8) * 2), b1 + (uint32_t)ins * 1024u);
  }
}

// Forward FFN slice j (32 hidden units) over all rows, 16 rows per chunk as the MFMA M dimension:
// linear1 (wave = 16 hidden units x half of K, the halves added through LDS) -> + b1 -> pre, GELU,
// dropout -> gd; linear2 partial (wave = 12 of the 48 output tiles, K = 32) -> P_j.  The weight slices
// are issued before the rows are waited for (mbx2: the layer's x2p mailbox, mbxn: its x2 mailbox).
__device__ void ffn_fwd_slice(const LrceDecStep& p, int l, int j, FfL& L, uint64_t seed4, const float* mbx2, float* mbxn,
                              unsigned long long* trace) {
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6, col = lane & 15, kq = lane >> 4;
  const int ct = wave & 1, kh = wave >> 1;
  const LrceDecLayerW& W = p.layer[l];
  const f16* w1 = reinterpret_cast<const f16*>(W.w1);
  const f16* w2 = reinterpret_cast<const f16*>(W.w2);
  ffn_slices_dma(w1, w2, j, L, wave, lane);
  const float b1v = W.b1[j * FS + ct * 16 + col];
  SUB_MARK(0, 0);
  SUB_MARK(0, 1);
  Ar pre = fwd_field(p, F_PRE, l, p.step), gd = fwd_field(p, F_GD, l, p.step);
  float* Pj = p.ws + 2 * WS_SLAB + (long long)j * MAXB * E;
  const bool owner = j == 0;   // slice 0's workgroup materialises x2 (read back by the next layer's reducers) and its stats
  for (int c0 = 0; c0 < p.B; c0 += RCH) {
    const int nr = min(RCH, p.B - c0);
    lds_barrier();   // the previous chunk's image is consumed
    rows_to_lds<false>(mbx2, c0, nr, L, p, 0x500 + l);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // (first chunk) the weight slices have landed too
    lds_barrier();
    SUB_MARK(0, 2);
    ln_rows_fwd(L, nr, W.g2, W.be2, p.eps, owner ? fwd_field(p, F_M2, l, p.step).base : nullptr,
                owner ? fwd_field(p, F_R2, l, p.step).base : nullptr, owner ? mbxn : nullptr, fwd_field(p, F_X2, l, p.step).base, c0);
    lds_barrier();
    SUB_MARK(0, 3);
    // linear1 slice
    f32x4 acc4[4] = {{0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}};
#pragma unroll
    for (int s = 0; s < 24; ++s)   // four independent accumulation chains
      acc4[s & 3] = mfma_sp(*reinterpret_cast<const float4*>(xat(L, col, kh * 384 + 16 * s + 4 * kq)),
                            *reinterpret_cast<const uint2*>(L.w1s + (ct * 16 + col) * E + kh * 384 + 16 * s + 4 * kq), acc4[s & 3]);
    f32x4 acc;
#pragma unroll
    for (int r = 0; r < 4; ++r) acc[r] = (acc4[0][r] + acc4[1][r]) + (acc4[2][r] + acc4[3][r]);
    if (kh) {
#pragma unroll
      for (int r = 0; r < 4; ++r) L.kacc[ct][4 * kq + r][col] = acc[r];
    }
    lds_barrier();
    if (!kh) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int rr = 4 * kq + r, b = c0 + rr, cc = ct * 16 + col, cg = j * FS + cc;
        float g = 0.f;
        if (rr < nr) {
          const float hv = acc[r] + L.kacc[ct][rr][col] + b1v;
          pre.row(b)[cg] = hv;
          g = gelu_f(hv);
          if (p.drop_p > 0.f) g = drop1(g, p.drop_p, seed4, (long long)b * FF + cg);
          gd.row(b)[cg] = g;
        }
        L.hb[rr][cc] = g;
      }
    }
    lds_barrier();
    SUB_MARK(0, 4);
    // linear2 partial: 12 output tiles per wave, K = the 32 hidden units
    f32x4 o[12];
#pragma unroll
    for (int tt = 0; tt < 12; ++tt) o[tt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const float4 a = *reinterpret_cast<const float4*>(&L.hb[col][16 * q + 4 * kq]);
#pragma unroll
      for (int tt = 0; tt < 12; ++tt)
        o[tt] = mfma_sp(a, *reinterpret_cast<const uint2*>(L.w2s + ((wave * 12 + tt) * 16 + col) * FS + 16 * q + 4 * kq), o[tt]);
    }
    SUB_MARK(0, 5);
    tiles_out<false>(L, o, Pj, c0, nr);
    SUB_MARK(0, 6);
  }
}

// ------------------------------------------------------------------------------- forward kernel
__global__ void __launch_bounds__(NT, 1) dec_step_fwd_kernel(LrceDecStep p, const uint64_t* rng_off, unsigned long long* trace) {
  __shared__ __attribute__((aligned(16))) StepLds U;
  __shared__ __attribute__((aligned(16))) RedL RD;
  __shared__ unsigned ok_word;
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int G = gridDim.x, R = G / H;
  const int h = blockIdx.x % H, r = blockIdx.x / H;
  const uint64_t roff = rng_off_now(rng_off);
  const int L_ = p.n_layers;
  const unsigned set = launch_begin(p);
  for (int l = 0; l < L_; ++l) {
    const LrceDecLayerW& W = p.layer[l];
    const uint64_t sl = layer_seed(p, l) + roff;
    // ---- A: self-attention block (after reducing the previous layer's FFN partials)
    STEP_MARK(0, l, 0);
    SaL& S = U.sa;
    lds_barrier();
    slice_dma(reinterpret_cast<const f16*>(W.wo), h, S.wo, wave, lane);
    if (l > 0) {
      STEP_MARK(0, l, 1);
      const LrceDecLayerW& Wp = p.layer[l - 1];
      for (int b = r; b < p.B; b += R)
        slice_reduce<false>(p.ws + 2 * WS_SLAB, b, h, Wp.b2, p.drop_p, layer_seed(p, l - 1) + 5 + roff,
                     mb_of(p, set, K_X2, l - 1) + (long long)b * E, mb_of(p, set, K_X3P, l - 1) + (long long)b * E,
                     fwd_field(p, F_X3P, l - 1, p.step).row(b), RD, p, 0x100 + l);
    }
    // W_v rows into registers after the reduce (held across it they cost spills)
    const float bvv = t < D ? W.bv[h * D + t] : 0.f;
    bool first = true;
    for (int b = r; b < p.B; b += R) {
      if (l > 0) {
        const LrceDecLayerW& Wp = p.layer[l - 1];
        float4 xr = make_float4(0.f, 0.f, 0.f, 0.f), gg = xr, be = xr;
        if (t < E / 4) {
          gg = *reinterpret_cast<const float4*>(Wp.g3 + 4 * t);
          be = *reinterpret_cast<const float4*>(Wp.be3 + 4 * t);
          xr = ld4_wait(mb_of(p, set, K_X3P, l - 1) + (long long)b * E, 4 * t, p, 0x600 + l);
        }
        if (first) STEP_MARK(0, l, 2);
        float mu, rs;
        ln_row_fwd(xr, row_sum_local(xr, t), gg, be, p.eps, S.x0, S.red2, t, lane, wave, mu, rs);
        if (h == 0) {
          if (t < E / 4)
            *reinterpret_cast<float4*>(fwd_field(p, F_X0, l, p.step).row(b) + 4 * t) = *reinterpret_cast<const float4*>(S.x0 + 4 * t);
          if (t == 0) {
            fwd_field(p, F_M3, l - 1, p.step).row(b)[0] = mu;
            fwd_field(p, F_R3, l - 1, p.step).row(b)[0] = rs;
          }
        }
      } else if (t < E / 4) {
        *reinterpret_cast<float4*>(S.x0 + 4 * t) = *reinterpret_cast<const float4*>(fwd_field(p, F_X0, 0, p.step).row(b) + 4 * t);
      }
      lds_barrier();
      sa_fwd_row(p, l, b, h, reinterpret_cast<const f16*>(W.wv), bvv, S, sl, sl + 1, first, RD, mb_of(p, set, K_X1P, l));
      first = false;
      lds_barrier();
    }
    STEP_MARK(0, l, 3);
    // ---- B: cross-attention block
    CaL& C = U.ca;
    lds_barrier();
    const float bqv = t < D ? W.bq[h * D + t] : 0.f;
    slice_dma(reinterpret_cast<const f16*>(W.woc), h, C.wo, wave, lane);
    first = true;
    for (int b = r; b < p.B; b += R) {
      uint4 kr[8];
      ca_fwd_prefetch(p, l, b, h, C, kr);
      if (first) STEP_MARK(0, l, 4);
      ca_fwd_row(p, l, b, h, reinterpret_cast<const f16*>(W.wq), bqv, C, sl + 2, sl + 3, kr, RD, mb_of(p, set, K_X1P, l), mb_of(p, set, K_X2P, l));
      first = false;
      lds_barrier();
    }
    STEP_MARK(0, l, 5);
    // ---- C: FFN slices over all rows
    for (int j = blockIdx.x; j < NF; j += G) {
      ffn_fwd_slice(p, l, j, U.ff, sl + 4, mb_of(p, set, K_X2P, l), mb_of(p, set, K_X2, l), trace);
      SUB_MARK(0, 7);
    }
    STEP_MARK(0, l, 7);
  }
  // ---- step tail: x3p of the last layer, then (head 0) x3 = LN3, tsum = x3 + s, s' = drop(LN_f(tsum))
  const int Ll = L_ - 1;
  STEP_MARK(0, L_, 1);
  for (int b = r; b < p.B; b += R)
    slice_reduce<false>(p.ws + 2 * WS_SLAB, b, h, p.layer[Ll].b2, p.drop_p, layer_seed(p, Ll) + 5 + roff,
                 mb_of(p, set, K_X2, Ll) + (long long)b * E, mb_of(p, set, K_X3P, Ll) + (long long)b * E,
                 fwd_field(p, F_X3P, Ll, p.step).row(b), RD, p, 0x700);
  if (h == 0) {
    SaL& S = U.sa;
    const uint64_t st = tail_seed(p) + roff;
    for (int b = r; b < p.B; b += R) {
      float4 xr = make_float4(0.f, 0.f, 0.f, 0.f), gg = xr, be = xr;
      if (t < E / 4) {
        gg = *reinterpret_cast<const float4*>(p.layer[Ll].g3 + 4 * t);
        be = *reinterpret_cast<const float4*>(p.layer[Ll].be3 + 4 * t);
        xr = ld4_wait(mb_of(p, set, K_X3P, Ll) + (long long)b * E, 4 * t, p, 0x800);
      }
      float mu, rs;
      ln_row_fwd(xr, row_sum_local(xr, t), gg, be, p.eps, S.x0, S.red2, t, lane, wave, mu, rs);
      if (t == 0) {
        fwd_field(p, F_M3, Ll, p.step).row(b)[0] = mu;
        fwd_field(p, F_R3, Ll, p.step).row(b)[0] = rs;
      }
      lds_barrier();
      float4 ts = make_float4(0.f, 0.f, 0.f, 0.f);
      if (t < E / 4) {
        const float4 sv = *reinterpret_cast<const float4*>(fwd_field(p, F_X0, 0, p.step).row(b) + 4 * t);
        const float4 x3 = *reinterpret_cast<const float4*>(S.x0 + 4 * t);
        ts = make_float4(x3.x + sv.x, x3.y + sv.y, x3.z + sv.z, x3.w + sv.w);
        *reinterpret_cast<float4*>(fwd_field(p, F_X0, L_, p.step).row(b) + 4 * t) = ts;   // tsum
        gg = *reinterpret_cast<const float4*>(p.gf + 4 * t);
        be = *reinterpret_cast<const float4*>(p.bf + 4 * t);
      }
      lds_barrier();
      ln_row_fwd(ts, row_sum_local(ts, t), gg, be, p.eps, S.part, S.red2, t, lane, wave, mu, rs);
      if (t == 0) {
        fwd_field(p, F_M1, L_, p.step).row(b)[0] = mu;
        fwd_field(p, F_R1, L_, p.step).row(b)[0] = rs;
      }
      lds_barrier();
      float* dst = p.step + 1 < p.S ? fwd_field(p, F_X0, 0, p.step + 1).row(b) : p.s_out + (long long)b * E;
#pragma unroll
      for (int i = 0; i < 3; ++i) {
        const int n = t + 256 * i;
        float v = S.part[n];
        if (p.drop_p > 0.f) v = drop1(v, p.drop_p, st, (long long)b * E + n);
        dst[n] = v;
      }
      lds_barrier();
    }
  }
  STEP_MARK(0, L_, 7);
  finish(p, &ok_word);
}

// =============================================================================== backward
// ---------------------------------------------------------------- backward: FFN slice j, all rows
__device__ void ffn_bwd_slice(const LrceDecStep& p, int l, int j, FfL& L, uint64_t seed4, uint64_t seed5, const float* mbd3,
                              float* dres, unsigned long long* trace) {
  const int t = opaque_tid(), lane = t & 63, wave = t >> 6, col = lane & 15, kq = lane >> 4;
  const int ct = wave & 1, kh = wave >> 1;
  const LrceDecLayerW& W = p.layer[l];
  const f16* w1 = reinterpret_cast<const f16*>(W.w1);
  const f16* w2 = reinterpret_cast<const f16*>(W.w2);
  const Ar df = bwd_field(p, G_DF, l, p.step), dgp = bwd_field(p, G_DGP, l, p.step);
  const Ar x3p = fwd_field(p, F_X3P, l, p.step), m3 = fwd_field(p, F_M3, l, p.step), r3 = fwd_field(p, F_R3, l, p.step);
  const Ar pre = fwd_field(p, F_PRE, l, p.step);
  float* Qj = p.ws + 2 * WS_SLAB + (long long)j * MAXB * E;
  const bool owner = j == 0;
  // the saved pre-activations of a chunk's rows (written by the forward launch): loaded into registers
  // BEFORE the weight-slice DMA (vmcnt is in order: a load issued after the DMA could only be consumed
  // once the whole 96 KB had landed), parked in LDS once the chunk's rows arrived
  constexpr int PPT = RCH * FS / NT;   // 2 per thread
  float pv[PPT];
  auto pre_load = [&](int c0, int nr) {
#pragma unroll
    for (int q = 0; q < PPT; ++q) {
      const int i = t + q * NT;
      pv[q] = i < nr * FS ? pre.row(c0 + i / FS)[j * FS + i % FS] : 0.f;
    }
  };
  auto pre_park = [&]() {
#pragma unroll
    for (int q = 0; q < PPT; ++q) {
      const int i = t + q * NT;
      L.preb[i / FS][i % FS] = pv[q];
    }
  };
  // likewise the LayerNorm-3 operands of the wave's four rows (x3p, mean, rstd, gamma)
  float4 xq[4][3], gq[3];
  float muq[4], rsq[4];
  auto ln_load = [&](int c0, int nr) {
    const int lane_ = t & 63;
#pragma unroll
    for (int i = 0; i < 3; ++i) gq[i] = *reinterpret_cast<const float4*>(W.g3 + 12 * lane_ + 4 * i);
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int b = c0 + min(wave + 4 * q, nr - 1);
      muq[q] = m3.row(b)[0];
      rsq[q] = r3.row(b)[0];
#pragma unroll
      for (int i = 0; i < 3; ++i) xq[q][i] = *reinterpret_cast<const float4*>(x3p.row(b) + 12 * lane_ + 4 * i);
    }
  };
  pre_load(0, min(RCH, p.B));
  ln_load(0, min(RCH, p.B));
  ffn_slices_dma(w1, w2, j, L, wave, lane);
  SUB_MARK(1, 0);
  SUB_MARK(1, 1);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // the slices and prefetches have landed (read after the next barrier)
  lds_barrier();
  auto pack4 = [](const f16* p0, int stride) {   // four fp16 down a column of an LDS image
    const unsigned a = __builtin_bit_cast(unsigned short, p0[0]), b = __builtin_bit_cast(unsigned short, p0[stride]);
    const unsigned c = __builtin_bit_cast(unsigned short, p0[2 * stride]), d = __builtin_bit_cast(unsigned short, p0[3 * stride]);
    return make_uint2(a | (b << 16), c | (d << 16));
  };
  SUB_MARK(1, 2);
  for (int c0 = 0; c0 < p.B; c0 += RCH) {
    const int nr = min(RCH, p.B - c0);
    lds_barrier();
    if (c0 > 0) {
      pre_load(c0, nr);
      ln_load(c0, nr);
    }
    rows_to_lds<true>(mbd3, c0, nr, L, p, 0x900 + l);
    pre_park();
    lds_barrier();
    SUB_MARK(1, 3);
    // LayerNorm-3 backward per row (the wave's four rows together), then the out-dropout backward -> df
    // in the image
    {
      float4 g[4][3], xh[4][3];
      float s1[4], s2[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int rr = wave + 4 * q;
        const float mu = muq[q], rs = rsq[q];
        const float* xp = xat(L, rr, 12 * lane);
        s1[q] = s2[q] = 0.f;
#pragma unroll
        for (int i = 0; i < 3; ++i) {
          const float4 dy = *reinterpret_cast<const float4*>(xp + 4 * i);   // zero for rows >= nr
          const float4 gm = gq[i];
          const float4 x = xq[q][i];
          g[q][i] = make_float4(dy.x * gm.x, dy.y * gm.y, dy.z * gm.z, dy.w * gm.w);
          xh[q][i] = make_float4((x.x - mu) * rs, (x.y - mu) * rs, (x.z - mu) * rs, (x.w - mu) * rs);
          s1[q] += (g[q][i].x + g[q][i].y) + (g[q][i].z + g[q][i].w);
          s2[q] += (g[q][i].x * xh[q][i].x + g[q][i].y * xh[q][i].y) + (g[q][i].z * xh[q][i].z + g[q][i].w * xh[q][i].w);
        }
      }
      wave_sum_x4(s1);
      wave_sum_x4(s2);
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int rr = wave + 4 * q;
        if (rr >= nr) break;
        const int b = c0 + rr;
        const float rs = rsq[q], mg = s1[q] * (1.0f / E), mgx = s2[q] * (1.0f / E);
        float* xp = xat(L, rr, 12 * lane);
#pragma unroll
        for (int i = 0; i < 3; ++i) {
          const int k = 12 * lane + 4 * i;
          float4 d = make_float4(rs * (g[q][i].x - mg - xh[q][i].x * mgx), rs * (g[q][i].y - mg - xh[q][i].y * mgx),
                                 rs * (g[q][i].z - mg - xh[q][i].z * mgx), rs * (g[q][i].w - mg - xh[q][i].w * mgx));
          if (owner) st4_sc1(dres, (long long)b * E + k, d);
          d = drop4(d, p.drop_p, seed5, (long long)b * E + k);
          *reinterpret_cast<float4*>(xp + 4 * i) = d;
          if (owner) *reinterpret_cast<float4*>(df.row(b) + k) = d;
          g[q][i] = d;   // (for the row maximum below)
        }
      }
      // per-row power-of-two scale 2^(7 - e), e = exponent of the row's max |df|: the f16-split operands
      // of this chunk (df, then dgp) sit in [2^7, 2^8) at most, far from the f16 range's ends (exact:
      // the products and the later unscaling are by powers of two)
      float mx[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        mx[q] = 0.f;
        if (wave + 4 * q < nr) {
#pragma unroll
          for (int i = 0; i < 3; ++i)
            mx[q] = fmaxf(mx[q], fmaxf(fmaxf(fabsf(g[q][i].x), fabsf(g[q][i].y)), fmaxf(fabsf(g[q][i].z), fabsf(g[q][i].w))));
        }
      }
#pragma unroll
      for (int q = 0; q < 4; ++q) mx[q] = wave_max_dpp(mx[q]);
      if (lane == 0) {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int rr = wave + 4 * q;
          const int e = mx[q] > 0.f ? ilogbf(mx[q]) : 0;
          L.rsc[rr] = ldexpf(1.0f, 7 - e);
          L.rinv[rr] = ldexpf(1.0f, e - 7);
        }
      }
    }
    lds_barrier();
    SUB_MARK(1, 4);
    // dgp = drop'(W2[:, slice]^T df) gelu'(pre)
    f32x4 acc4[4] = {{0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}};
#pragma unroll
    for (int s = 0; s < 24; ++s) {
      const float sa = L.rsc[col];
      float4 a = *reinterpret_cast<const float4*>(xat(L, col, kh * 384 + 16 * s + 4 * kq));
      a = make_float4(a.x * sa, a.y * sa, a.z * sa, a.w * sa);
      acc4[s & 3] = mfma_sp(a, pack4(L.w2s + (kh * 384 + 16 * s + 4 * kq) * FS + ct * 16 + col, FS), acc4[s & 3]);
    }
    f32x4 acc;
#pragma unroll
    for (int r = 0; r < 4; ++r) acc[r] = (acc4[0][r] + acc4[1][r]) + (acc4[2][r] + acc4[3][r]);
    if (kh) {
#pragma unroll
      for (int r = 0; r < 4; ++r) L.kacc[ct][4 * kq + r][col] = acc[r];
    }
    lds_barrier();
    if (!kh) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int rr = 4 * kq + r, b = c0 + rr, cc = ct * 16 + col, cg = j * FS + cc;
        float d = 0.f;
        if (rr < nr) {
          d = acc[r] + L.kacc[ct][rr][col];   // scaled by rsc[rr]
          if (p.drop_p > 0.f) d = drop1(d, p.drop_p, seed4, (long long)b * FF + cg);
          d *= gelu_grad_f(L.preb[rr][cc]);
          dgp.row(b)[cg] = d * L.rinv[rr];
        }
        L.hb[rr][cc] = d;   // kept scaled for Q_j
      }
    }
    lds_barrier();
    // Q_j = W1[slice]^T dgp: 12 column tiles per wave, K = the 32 hidden units
    f32x4 o[12];
#pragma unroll
    for (int tt = 0; tt < 12; ++tt) o[tt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const float4 a = *reinterpret_cast<const float4*>(&L.hb[col][16 * q + 4 * kq]);
#pragma unroll
      for (int tt = 0; tt < 12; ++tt)
        o[tt] = mfma_sp(a, pack4(L.w1s + (16 * q + 4 * kq) * E + (wave * 12 + tt) * 16 + col, E), o[tt]);
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) {   // unscale row 4 kq + r
      const float u = L.rinv[4 * kq + r];
#pragma unroll
      for (int tt = 0; tt < 12; ++tt) o[tt][r] *= u;
    }
    SUB_MARK(1, 5);
    tiles_out<true>(L, o, Qj, c0, nr);
    SUB_MARK(1, 6);
  }
}

// ------------------------------------------------------------ backward: cross-attention row b
// dx2 (handed-off row) -> LN2' -> dcao -> dctx -> attention backward (dq, memory dK / dV) -> the last
// head writes dx1 = dx2p + sum_h W_q[h]^T dq_h and raises the row flag
// what a cross-attention backward row needs that this launch does not write (the forward's rows and
// statistics, the question rows' running dK / dV, the head's K / V images by DMA): issued before the
// row's wait
struct CaBwdPre {
  float4 xr, gm;
  float mu, rs, qd, od, lse;
};
__device__ void ca_bwd_prefetch(const LrceDecStep& p, int l, int b, int h, CaL& L, CaBwdPre& q) {
  const int t = opaque_tid(), lane = t & 63, wave = t >> 6;
  const LrceDecLayerW& W = p.layer[l];
  const KvP kv = kv_of(p, l);
  const int Lk = kv.lk1 + kv.lk2;
  q.xr = q.gm = make_float4(0.f, 0.f, 0.f, 0.f);
  if (t < E / 4) {
    q.xr = *reinterpret_cast<const float4*>(fwd_field(p, F_X2P, l, p.step).row(b) + 4 * t);
    q.gm = *reinterpret_cast<const float4*>(W.g2 + 4 * t);
  }
  q.mu = fwd_field(p, F_M2, l, p.step).row(b)[0];
  q.rs = fwd_field(p, F_R2, l, p.step).row(b)[0];
  q.qd = q.od = 0.f;
  if (t < D) {
    q.qd = fwd_field(p, F_Q, l, p.step).row(b)[h * D + t];
    q.od = fwd_field(p, F_CTX, l, p.step).row(b)[h * D + t];
  }
  q.lse = fwd_field(p, F_LSE, l, p.step).row(b)[h];
  const KvRows kvr = kv_rows(kv, b, h);
  const uint32_t kb = dec_lds_addr(L.b.kimg), vb = dec_lds_addr(L.vimg);
  for (int ins = wave; ins * 8 < Lk; ins += 4) {
    const int r = ins * 8 + (lane >> 3), j = min(r, Lk - 1);
    const bf16* kp = kv_row(kvr, j) + (((lane & 7) ^ (r & 7)) << 3);
    dec_glds_p(kp, kb + (uint32_t)ins * 1024u);
    dec_glds_p(kp + kv.v_off, vb + (uint32_t)ins * 1024u);
  }
}

__device__ void ca_bwd_row(const LrceDecStep& p, int l, int b, int h, CaL& L, uint64_t seed2, uint64_t seed3,
                           const CaBwdPre& q, RedL& RD, const float* mbd2, float* mbd1) {
  const int t = opaque_tid(), lane = t & 63, wave = t >> 6;
  const KvP kv = kv_of(p, l);
  const int Lk = kv.lk1 + kv.lk2;
  float4 dy = make_float4(0.f, 0.f, 0.f, 0.f);
  if (t < E / 4) dy = ld4_wait(mbd2 + (long long)b * E, 4 * t, p, 0xB00 + l);
  const float rs = q.rs, qd = q.qd, od = q.od, lse = q.lse;
  LnBwdLocal lnl = ln_row_bwd_local(dy, q.xr, q.gm, q.mu, rs, t);
  const float* dk2r = p.lt ? p.dkv_text + l * p.dkv_text_lstride : nullptr;
  float* dk2 = const_cast<float*>(dk2r);
  const long long tbase = (long long)b * p.lt * 2 * E + h * D;
  const float4 dx = ln_row_bwd(lnl, rs, L.red2, lane, wave);
  if (t < E / 4) {
    *reinterpret_cast<float4*>(L.b.dx2p + 4 * t) = dx;
    float4 d = dx;
    if (p.drop_p > 0.f) {
      const long long e = (long long)b * E + 4 * t;
      d = make_float4(drop1(dx.x, p.drop_p, seed3, e), drop1(dx.y, p.drop_p, seed3, e + 1), drop1(dx.z, p.drop_p, seed3, e + 2),
                      drop1(dx.w, p.drop_p, seed3, e + 3));
    }
    *reinterpret_cast<float4*>(L.b.dcao + 4 * t) = d;
    if (h == 0) *reinterpret_cast<float4*>(bwd_field(p, G_DCAO, l, p.step).row(b) + 4 * t) = d;
  }
  if (t < D) L.b.q[t] = qd * 0.125f;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // K / V rows (and, first row, the W_oc slice) have landed
  lds_barrier();
  slice_gemv_t(L.wo, L.b.dcao, &L.b.red64[0][0], wave, lane);
  lds_barrier();
  // the W_oc slice is consumed: stream W_q[h] rows into its place for the dX partial at the end
  rows_dma(reinterpret_cast<const f16*>(p.layer[l].wq), h, L.wo, wave, lane);
  float dod = 0.f;
  if (t < D) {
    dod = (L.b.red64[0][t] + L.b.red64[1][t]) + (L.b.red64[2][t] + L.b.red64[3][t]);
    L.b.dctx[t] = dod;
  }
  const float delta = block_sum4(dod * od, L.red2, lane, wave);
  const bool live = t < Lk;
  float pf = 0.f, ds = 0.f;
  if (live) {
    float sc = 0.f, dp = 0.f;
#pragma unroll
    for (int c = 0; c < 8; ++c) {
      const uint4 ku = *reinterpret_cast<const uint4*>(L.b.kimg + kv_swz(t, c));
      const uint4 vu = *reinterpret_cast<const uint4*>(L.vimg + kv_swz(t, c));
      const unsigned k4[4] = {ku.x, ku.y, ku.z, ku.w}, v4[4] = {vu.x, vu.y, vu.z, vu.w};
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        sc += bfbits2f((unsigned short)(k4[e] & 0xFFFFu)) * L.b.q[8 * c + 2 * e] +
              bfbits2f((unsigned short)(k4[e] >> 16)) * L.b.q[8 * c + 2 * e + 1];
        dp += bfbits2f((unsigned short)(v4[e] & 0xFFFFu)) * L.b.dctx[8 * c + 2 * e] +
              bfbits2f((unsigned short)(v4[e] >> 16)) * L.b.dctx[8 * c + 2 * e + 1];
      }
    }
    const float pr = __expf(sc - lse);
    float f = 1.f;
    if (p.drop_p > 0.f) f = lrce_uniform(seed2, (uint64_t)(((long long)b * H + h) * Lk + t)) >= p.drop_p ? 1.0f / (1.0f - p.drop_p) : 0.f;
    pf = pr * f;
    ds = pr * (f * dp - delta);
  }
  L.b.ps[t] = pf;
  L.b.dss[t] = ds;
  lds_barrier();
  {
    float dq0 = 0.f, dq1 = 0.f;
    int j = wave;
    for (; j + 4 < Lk; j += 8) {
      dq0 += L.b.dss[j] * kv_at(L.b.kimg, j, lane);
      dq1 += L.b.dss[j + 4] * kv_at(L.b.kimg, j + 4, lane);
    }
    if (j < Lk) dq0 += L.b.dss[j] * kv_at(L.b.kimg, j, lane);
    L.b.red64[wave][lane] = dq0 + dq1;
  }
  // the question rows' running dK / dV (stored by the first backward step, S - 1, added to after it):
  // loaded here, ahead of the video rows' loop that hides their latency
  float4 told[TXI][4];
  {
    const bool dk2_store = p.step == p.S - 1;
#pragma unroll
    for (int i = 0; i < TXI; ++i) {
      const int e = t + 256 * i, tj = e >> 3, c = e & 7;
      told[i][0] = told[i][1] = told[i][2] = told[i][3] = make_float4(0.f, 0.f, 0.f, 0.f);
      if (tj < kv.lk2 && !dk2_store) {
        const float* src = dk2 + tbase + (long long)tj * 2 * E + c * 8;
        told[i][0] = *reinterpret_cast<const float4*>(src);
        told[i][1] = *reinterpret_cast<const float4*>(src + 4);
        told[i][2] = *reinterpret_cast<const float4*>(src + E);
        told[i][3] = *reinterpret_cast<const float4*>(src + E + 4);
      }
    }
  }
  {
    const long long lvs = l * p.dkv_video_lstride;
    const long long vbase = (long long)(b / kv.bdiv1) * kv.stride1 + (long long)p.step * 150 * 2 * E + h * D;
    for (int e = t; e < kv.lk1 * 8; e += 256) {
      const int j = e >> 3, c = e & 7;
      const float dsj = L.b.dss[j], pj = L.b.ps[j];
      float kv8[16];
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        kv8[i] = dsj * L.b.q[c * 8 + i];
        kv8[8 + i] = pj * L.b.dctx[c * 8 + i];
      }
      const long long o = lvs + vbase + (long long)j * 2 * E + c * 8;
      if (p.dkv_video16) {
        bf16* d16 = reinterpret_cast<bf16*>(p.dkv_video16) + o;
        bf16x8 k16, v16;
#pragma unroll
        for (int i = 0; i < 8; ++i) { k16[i] = f2bf(kv8[i]); v16[i] = f2bf(kv8[8 + i]); }
        *reinterpret_cast<bf16x8*>(d16) = k16;
        *reinterpret_cast<bf16x8*>(d16 + E) = v16;
      } else {
        float* dst = p.dkv_video32 + o;
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          __hip_atomic_fetch_add(dst + i, kv8[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          __hip_atomic_fetch_add(dst + E + i, kv8[8 + i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
      }
    }
#pragma unroll
    for (int i = 0; i < TXI; ++i) {
      const int e = t + 256 * i, tj = e >> 3, c = e & 7;
      if (tj < kv.lk2) {
        const int j = kv.lk1 + tj;
        const float dsj = L.b.dss[j], pj = L.b.ps[j];
        const float* qv = L.b.q + c * 8;
        const float* gv = L.b.dctx + c * 8;
        float* dst = dk2 + tbase + (long long)tj * 2 * E + c * 8;
        const float4 a0 = told[i][0], a1 = told[i][1], a2 = told[i][2], a3 = told[i][3];
        *reinterpret_cast<float4*>(dst) = make_float4(a0.x + dsj * qv[0], a0.y + dsj * qv[1], a0.z + dsj * qv[2], a0.w + dsj * qv[3]);
        *reinterpret_cast<float4*>(dst + 4) = make_float4(a1.x + dsj * qv[4], a1.y + dsj * qv[5], a1.z + dsj * qv[6], a1.w + dsj * qv[7]);
        *reinterpret_cast<float4*>(dst + E) = make_float4(a2.x + pj * gv[0], a2.y + pj * gv[1], a2.z + pj * gv[2], a2.w + pj * gv[3]);
        *reinterpret_cast<float4*>(dst + E + 4) = make_float4(a3.x + pj * gv[4], a3.y + pj * gv[5], a3.z + pj * gv[6], a3.w + pj * gv[7]);
      }
    }
  }
  lds_barrier();
  if (t < D) {
    const float dq = ((L.b.red64[0][t] + L.b.red64[1][t]) + (L.b.red64[2][t] + L.b.red64[3][t])) * 0.125f;
    L.b.dq[t] = dq;
    bwd_field(p, G_DQ, l, p.step).row(b)[h * D + t] = dq;
  }
  lds_barrier();
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // the W_q rows have landed
  lds_barrier();
  float* part = &L.b.acc[0][0];
  rows_t_lds(L.wo, L.b.dq, part);
  publish(part, p.ws, b, h);
  const float4 sm = gather_cols(p.ws, b, h, RD.red, p, 0xC00 + l);
  if (t < 16) {
    const int c = h * D + 4 * t;
    const float4 o = add4(lds4(L.b.dx2p + c), sm);
    st4_sc1(mbd1 + (long long)b * E, c, o);
    *reinterpret_cast<float4*>(bwd_field(p, G_DLN1, l, p.step).row(b) + c) = o;
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // the re-arming stores, before the next hand-off
}

// ------------------------------------------------------------- backward: self-attention row b
// dx1 (handed-off row) -> LN1' -> dsao -> dsav_h -> the last head writes dx0 = dx1p + sum_h W_v[h]^T dsav_h:
// d x3 of layer l-1 (handed off), or (l = 0) the step input's gradient dx0 + dt.
__device__ void sa_bwd_row(const LrceDecStep& p, int l, int b, int h, SaL& L, uint64_t seed0, uint64_t seed1, RedL& RD,
                           const float* mbd1, float* mbd3, const float* mbdt) {
  const int t = opaque_tid(), lane = t & 63, wave = t >> 6;
  const LrceDecLayerW& W = p.layer[l];
  float4 dy = make_float4(0.f, 0.f, 0.f, 0.f), xr = dy, gm = dy;
  const float mu = fwd_field(p, F_M1, l, p.step).row(b)[0], rs = fwd_field(p, F_R1, l, p.step).row(b)[0];
  if (t < E / 4) {
    xr = *reinterpret_cast<const float4*>(fwd_field(p, F_X1P, l, p.step).row(b) + 4 * t);
    gm = *reinterpret_cast<const float4*>(W.g1 + 4 * t);
    dy = ld4_wait(mbd1 + (long long)b * E, 4 * t, p, 0xD00 + l);
  }
  LnBwdLocal lnl = ln_row_bwd_local(dy, xr, gm, mu, rs, t);
  const float4 dx = ln_row_bwd(lnl, rs, L.red2, lane, wave);
  if (t < E / 4) {
    *reinterpret_cast<float4*>(L.dx1p + 4 * t) = dx;
    float4 d = dx;
    if (p.drop_p > 0.f) {
      const long long e = (long long)b * E + 4 * t;
      d = make_float4(drop1(dx.x, p.drop_p, seed1, e), drop1(dx.y, p.drop_p, seed1, e + 1), drop1(dx.z, p.drop_p, seed1, e + 2),
                      drop1(dx.w, p.drop_p, seed1, e + 3));
    }
    *reinterpret_cast<float4*>(L.dsao + 4 * t) = d;
    if (h == 0) *reinterpret_cast<float4*>(bwd_field(p, G_DSAO, l, p.step).row(b) + 4 * t) = d;
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  lds_barrier();
  slice_gemv_t(L.wo, L.dsao, &L.red64[0][0], wave, lane);
  lds_barrier();
  rows_dma(reinterpret_cast<const f16*>(p.layer[l].wv), h, L.wo, wave, lane);   // W_v[h] rows in place of the W_o slice
  if (t < D) {
    float v = (L.red64[0][t] + L.red64[1][t]) + (L.red64[2][t] + L.red64[3][t]);
    if (p.drop_p > 0.f) v = drop1(v, p.drop_p, seed0, ((long long)b * E + h * D + t) / D);
    L.v[t] = v;
    bwd_field(p, G_DSAV, l, p.step).row(b)[h * D + t] = v;
  }
  lds_barrier();
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  lds_barrier();
  float* part = &L.acc[0][0];
  rows_t_lds(L.wo, L.v, part);
  publish(part, p.ws + WS_SLAB, b, h);
  const float4 sm = gather_cols(p.ws + WS_SLAB, b, h, RD.red, p, 0xE00 + l);
  if (t < 16) {
    const int c = h * D + 4 * t;
    if (l > 0) {
      const float4 o = add4(lds4(L.dx1p + c), sm);
      st4_sc1(mbd3 + (long long)b * E, c, o);
      *reinterpret_cast<float4*>(bwd_field(p, G_DLN3, l - 1, p.step).row(b) + c) = o;
    } else {
      const float4 dt = ld4_wait(mbdt + (long long)b * E, c, p, 0xF00);
      *reinterpret_cast<float4*>(p.ds_out + (long long)b * E + c) = add4(add4(lds4(L.dx1p + c), sm), dt);
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // the re-arming stores, before the next hand-off
}

__global__ void __launch_bounds__(NT, 1) dec_step_bwd_kernel(LrceDecStep p, const uint64_t* rng_off, unsigned long long* trace) {
  __shared__ __attribute__((aligned(16))) StepLds U;
  __shared__ __attribute__((aligned(16))) RedL RD;
  __shared__ unsigned ok_word;
  const int t = opaque_tid(), lane = t & 63, wave = t >> 6;
  const int G = gridDim.x, R = G / H;
  const int h = blockIdx.x % H, r = blockIdx.x / H;
  const uint64_t roff = rng_off_now(rng_off);
  const int L_ = p.n_layers;
  const unsigned set = launch_begin(p);
  // ---- tail: du = drop'(ds), dt = LN_f'(du) -> d x3 of the last layer
  STEP_MARK(1, L_, 0);
  if (h == 0) {
    SaL& S = U.sa;
    const uint64_t st = tail_seed(p) + roff;
    for (int b = r; b < p.B; b += R) {
      float4 dy = make_float4(0.f, 0.f, 0.f, 0.f), xr = dy, gm = dy;
      if (t < E / 4) {
        dy = *reinterpret_cast<const float4*>(p.ds_in + (long long)b * E + 4 * t);
        if (p.drop_p > 0.f) {
          const long long e = (long long)b * E + 4 * t;
          dy = make_float4(drop1(dy.x, p.drop_p, st, e), drop1(dy.y, p.drop_p, st, e + 1), drop1(dy.z, p.drop_p, st, e + 2),
                           drop1(dy.w, p.drop_p, st, e + 3));
        }
        *reinterpret_cast<float4*>(bwd_field(p, G_DF, L_, p.step).row(b) + 4 * t) = dy;   // du (fusion LN's gamma / beta)
        xr = *reinterpret_cast<const float4*>(fwd_field(p, F_X0, L_, p.step).row(b) + 4 * t);   // tsum
        gm = *reinterpret_cast<const float4*>(p.gf + 4 * t);
      }
      const float mu = fwd_field(p, F_M1, L_, p.step).row(b)[0], rs = fwd_field(p, F_R1, L_, p.step).row(b)[0];
      LnBwdLocal lnl = ln_row_bwd_local(dy, xr, gm, mu, rs, t);
      const float4 dx = ln_row_bwd(lnl, rs, S.red2, lane, wave);
      if (t < E / 4) {
        *reinterpret_cast<float4*>(bwd_field(p, G_DCAO, L_, p.step).row(b) + 4 * t) = dx;   // dt
        *reinterpret_cast<float4*>(bwd_field(p, G_DLN3, L_ - 1, p.step).row(b) + 4 * t) = dx;
        st4_sc1(mb_of(p, set, K_DT, 0) + (long long)b * E, 4 * t, dx);         // read by layer 0's last step
        st4_sc1(mb_of(p, set, K_DLN3, L_ - 1) + (long long)b * E, 4 * t, dx);
      }
    }
  }
  for (int l = L_ - 1; l >= 0; --l) {
    const LrceDecLayerW& W = p.layer[l];
    const uint64_t sl = layer_seed(p, l) + roff;
    // ---- FB: FFN slices over all rows
    STEP_MARK(1, l, 0);
    for (int j = blockIdx.x; j < NF; j += G) {
      ffn_bwd_slice(p, l, j, U.ff, sl + 4, sl + 5, mb_of(p, set, K_DLN3, l), mb_of(p, set, K_DRES, l), trace);
      SUB_MARK(1, 7);
    }
    // ---- CB: dx2 slices, then the cross-attention block backward per row; the weight slices and the
    // first row's saved operands / K / V images are issued before the FFN slices are waited for
    CaL& C = U.ca;
    lds_barrier();
    slice_dma(reinterpret_cast<const f16*>(W.woc), h, C.wo, wave, lane);
    STEP_MARK(1, l, 2);
    STEP_MARK(1, l, 3);
    for (int b = r; b < p.B; b += R)
      slice_reduce<true>(p.ws + 2 * WS_SLAB, b, h, nullptr, 0.f, 0, mb_of(p, set, K_DRES, l) + (long long)b * E,
                   mb_of(p, set, K_DLN2, l) + (long long)b * E, bwd_field(p, G_DLN2, l, p.step).row(b), RD, p, 0xA00 + l);
    // the row's saved operands and K / V images after the reduce (held across it they cost spills)
    CaBwdPre pre;
    bool first = true;
    for (int b = r; b < p.B; b += R) {
      if (!first)   // the previous row left W_q rows in the slice's place
        slice_dma(reinterpret_cast<const f16*>(W.woc), h, C.wo, wave, lane);
      ca_bwd_prefetch(p, l, b, h, C, pre);
      if (first) STEP_MARK(1, l, 4);
      first = false;
      ca_bwd_row(p, l, b, h, C, sl + 2, sl + 3, pre, RD, mb_of(p, set, K_DLN2, l), mb_of(p, set, K_DLN1, l));
      lds_barrier();
    }
    STEP_MARK(1, l, 5);
    // ---- SB: self-attention block backward per row
    SaL& S = U.sa;
    first = true;
    for (int b = r; b < p.B; b += R) {
      lds_barrier();
      slice_dma(reinterpret_cast<const f16*>(W.wo), h, S.wo, wave, lane);
      if (first) STEP_MARK(1, l, 6);
      first = false;
      sa_bwd_row(p, l, b, h, S, sl, sl + 1, RD, mb_of(p, set, K_DLN1, l), l > 0 ? mb_of(p, set, K_DLN3, l - 1) : nullptr,
                 mb_of(p, set, K_DT, 0));
      lds_barrier();
    }
    STEP_MARK(1, l, 7);
  }
  finish(p, &ok_word);
}

int grid_for(int B) { return H * (B < RMAX ? B : RMAX); }

int check(const LrceDecStep* a, bool bwd) {
  if (!a || !a->acts || !a->ws || !a->counters || !a->status || !a->kv_video || !a->gf || !a->bf)
    return lrce_fail(LRCE_E_ARG, "dec_step: null pointer");
  if (a->B < 1 || a->B > MAXB) return lrce_fail(LRCE_E_ARG, "dec_step: B=%d outside [1, %d]", a->B, MAXB);
  if (a->n_layers < 1 || a->n_layers > NLMAX || a->S < 1 || a->step < 0 || a->step >= a->S || a->nmc < 1 || a->B % a->nmc)
    return lrce_fail(LRCE_E_ARG, "dec_step: n_layers=%d S=%d step=%d nmc=%d", a->n_layers, a->S, a->step, a->nmc);
  if (a->lt < 0 || a->lt > MAXTXT || 150 + a->lt > MAXK || (a->lt > 0 && !a->kv_text))
    return lrce_fail(LRCE_E_ARG, "dec_step: lt=%d (<= %d question keys)", a->lt, MAXTXT);
  if (!bwd && a->step == a->S - 1 && !a->s_out) return lrce_fail(LRCE_E_ARG, "dec_step: the last step needs s_out");
  if (bwd && (!a->grads || !a->ds_in || !a->ds_out || (!a->dkv_video16 && !a->dkv_video32) || (a->lt > 0 && !a->dkv_text)))
    return lrce_fail(LRCE_E_ARG, "dec_step backward: grads / ds_in / ds_out / dK dV buffers");
  if (bwd && a->dkv_video16 && a->nmc != 1) return lrce_fail(LRCE_E_ARG, "dec_step backward: bf16 video dK/dV needs nmc == 1");
  for (int l = 0; l < a->n_layers; ++l) {
    const LrceDecLayerW& w = a->layer[l];
    const void* ps[] = {w.wv, w.bv, w.wo, w.bo, w.g1, w.be1, w.wq, w.bq, w.woc, w.boc, w.g2, w.be2, w.w1, w.b1, w.w2, w.b2, w.g3, w.be3};
    for (const void* q : ps)
      if (!q || (reinterpret_cast<uintptr_t>(q) & 15)) return lrce_fail(LRCE_E_ARG, "dec_step: layer %d parameter null or not 16-B aligned", l);
  }
  if ((reinterpret_cast<uintptr_t>(a->acts) & 15) || (a->grads && (reinterpret_cast<uintptr_t>(a->grads) & 15)) ||
      (reinterpret_cast<uintptr_t>(a->ws) & 15) || (reinterpret_cast<uintptr_t>(a->kv_video) & 15) ||
      (a->kv_text && (reinterpret_cast<uintptr_t>(a->kv_text) & 15)))
    return lrce_fail(LRCE_E_ARG, "dec_step: arenas / K/V need 16-B alignment");
  return LRCE_OK;
}

}  // namespace

extern "C" int64_t lrce_dec_step_field(int kind, int field, int layer, int B, int S, int n_layers) {
  if (kind < 0 || kind > 1 || B < 1 || S < 1 || n_layers < 1 || n_layers > NLMAX) return -1;
  if (field == -1) return field_off(kind, 0, n_layers + 1, B, S);   // total: n_layers + the tail block
  if (field < 0 || field >= (kind ? NBWD : NFWD) || layer < 0 || layer > n_layers) return -1;
  return field_off(kind, field, layer, B, S);
}
extern "C" int64_t lrce_dec_step_ws_elems(void) { return WS_ELEMS; }
extern "C" int64_t lrce_dec_step_counter_words(void) { return CTR_WORDS; }
extern "C" int lrce_dec_step_grid(int B) { return grid_for(B); }

extern "C" int lrce_dec_step_fwd(const LrceDecStep* a, void* stream) {
  if (int rc = check(a, false)) return rc;
  dec_step_fwd_kernel<<<grid_for(a->B), NT, 0, static_cast<hipStream_t>(stream)>>>(*a, lrce_rng_offset(), g_step_trace);
  return lrce_check_launch("dec_step_fwd");
}

extern "C" int lrce_dec_step_bwd(const LrceDecStep* a, void* stream) {
  if (int rc = check(a, true)) return rc;
  dec_step_bwd_kernel<<<grid_for(a->B), NT, 0, static_cast<hipStream_t>(stream)>>>(*a, lrce_rng_offset(), g_step_trace);
  return lrce_check_launch("dec_step_bwd");
}

extern "C" int lrce_dec_step_set_trace(uint64_t* buf) {
  g_step_trace = reinterpret_cast<unsigned long long*>(buf);
  return LRCE_OK;
}

extern "C" int lrce_dec_step_reset(float* ws, uint32_t* counters, uint32_t* status, void* stream) {
  if (!ws || !counters || !status) return lrce_fail(LRCE_E_ARG, "dec_step_reset: null pointer");
  hipStream_t st = static_cast<hipStream_t>(stream);
  if (hipMemsetAsync(ws, 0xFF, WS_ELEMS * sizeof(float), st) != hipSuccess ||
      hipMemsetAsync(counters, 0, CTR_WORDS * sizeof(uint32_t), st) != hipSuccess ||
      hipMemsetAsync(status, 0, 4 * sizeof(uint32_t), st) != hipSuccess)
    return lrce_fail(LRCE_E_LAUNCH, "dec_step_reset: memset failed");
  return LRCE_OK;
}
