// Clip assembly on the device (the step before the hot path: reference e2e_dataset.py:60-116).
//
// The reference decodes every frame on the host, resizes each with torchvision
// Resize((224, 224)) on a PIL image (= Pillow's antialiased BILINEAR resample), converts with
// ToTensor (/255, CHW), then picks frames for the temporal scales.  Here decoded RGB frames are
// handed over once as uint8 [T][H][W][3]; one kernel gathers the selected frames and resamples them
// straight into the (clips, 3, 224, 224) float layout the patch-embed im2col reads.
//
// Resampling restates Pillow's Resample.c (precompute_coeffs + normalize_coeffs_8bpc +
// ImagingResampleHorizontal/Vertical_8bpc) bit for bit:
//   scale = in / out, filterscale = max(scale, 1), support = filterscale (bilinear support 1);
//   output i: center = (i + 0.5) * scale, taps x in [int(center - support + 0.5), int(center + support
//   + 0.5)) clamped to the image, w = tri((x - center + 0.5) / filterscale), normalised in double, then
//   fixed point with 22 fraction bits (round half away from zero);
//   horizontal pass first (sum + 2^21) >> 22 clipped to [0, 255], then the vertical pass on those
//   8-bit values likewise.  A pass whose size does not change is skipped (as Pillow does).
// Each thread recomputes its taps in double (same IEEE operations as Pillow), so no coefficient
// tables travel; every vertical tap recomputes its horizontal 8-bit intermediate (<= 5 x 5 taps for
// the downscales of MSVD / MSRVTT / TGIF frames to 224).
#include "common.h"
#include "lrce_capi.h"

namespace {

constexpr int PREC = 22;        // PRECISION_BITS = 32 - 8 - 2
constexpr int MAX_TAPS = 24;    // 2 * ceil(in / out) + 1 taps: downscales up to 11x per axis (1920 -> 224 is 8.6x)

struct Taps {
  int lo, n;
  int k[MAX_TAPS];
};

__device__ __forceinline__ double tri(double x) {
  x = fabs(x);
  return x < 1.0 ? 1.0 - x : 0.0;
}

__device__ void taps(int in_size, int out_size, int i, Taps& t) {
  const double scale = (double)in_size / out_size;
  const double fs = scale < 1.0 ? 1.0 : scale;
  const double support = fs;
  const double center = (i + 0.5) * scale;
  const double ss = 1.0 / fs;
  int xmin = (int)(center - support + 0.5);
  if (xmin < 0) xmin = 0;
  int xmax = (int)(center + support + 0.5);
  if (xmax > in_size) xmax = in_size;
  xmax -= xmin;
  if (xmax > MAX_TAPS) xmax = MAX_TAPS;   // (guarded on the host: never reached)
  double ww = 0.0;   // Pillow sums the weights in tap order, then divides each by the sum
  for (int x = 0; x < xmax; ++x) ww += tri((x + xmin - center + 0.5) * ss);
  for (int x = 0; x < xmax; ++x) {
    const double w = tri((x + xmin - center + 0.5) * ss);
    const double k = ww != 0.0 ? w / ww : w;
    t.k[x] = k < 0 ? (int)(-0.5 + k * (1 << PREC)) : (int)(0.5 + k * (1 << PREC));
  }
  t.lo = xmin;
  t.n = xmax;
}

__device__ __forceinline__ int clip8(int v) {
  v >>= PREC;
  return v < 0 ? 0 : (v > 255 ? 255 : v);
}

// one thread per (output clip-frame, y, x); the three channels share the taps
__global__ void frames_resize_kernel(const uint8_t* __restrict__ frames, int H, int W, const int* __restrict__ idx, int n_out,
                                     int OH, int OW, float* __restrict__ out) {
  const long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  const long long per = (long long)OH * OW;
  if (e >= (long long)n_out * per) return;
  const int f = (int)(e / per);
  const int yx = (int)(e - (long long)f * per);
  const int y = yx / OW, x = yx - (yx / OW) * OW;
  const uint8_t* img = frames + (long long)idx[f] * H * W * 3;
  const bool need_h = OW != W, need_v = OH != H;
  Taps tx, ty;
  if (need_h) taps(W, OW, x, tx);
  else { tx.lo = x; tx.n = 1; tx.k[0] = 1 << PREC; }
  if (need_v) taps(H, OH, y, ty);
  else { ty.lo = y; ty.n = 1; ty.k[0] = 1 << PREC; }
  int acc[3] = {1 << (PREC - 1), 1 << (PREC - 1), 1 << (PREC - 1)};
  for (int j = 0; j < ty.n; ++j) {
    const uint8_t* row = img + (long long)(ty.lo + j) * W * 3;
    int mid[3];
    if (need_h) {
      int s[3] = {1 << (PREC - 1), 1 << (PREC - 1), 1 << (PREC - 1)};
      for (int i = 0; i < tx.n; ++i) {
        const uint8_t* p = row + (tx.lo + i) * 3;
        s[0] += p[0] * tx.k[i]; s[1] += p[1] * tx.k[i]; s[2] += p[2] * tx.k[i];
      }
      mid[0] = clip8(s[0]); mid[1] = clip8(s[1]); mid[2] = clip8(s[2]);
    } else {
      const uint8_t* p = row + x * 3;
      mid[0] = p[0]; mid[1] = p[1]; mid[2] = p[2];
    }
    if (need_v) {
      acc[0] += mid[0] * ty.k[j]; acc[1] += mid[1] * ty.k[j]; acc[2] += mid[2] * ty.k[j];
    } else {
      acc[0] = mid[0]; acc[1] = mid[1]; acc[2] = mid[2];
    }
  }
  float* o = out + (long long)f * 3 * per + yx;
#pragma unroll
  for (int c = 0; c < 3; ++c) {
    const int v = need_v ? clip8(acc[c]) : acc[c];
    o[c * per] = (float)v / 255.0f;   // ToTensor
  }
}

}  // namespace

extern "C" int lrce_frames_resize(const uint8_t* frames, int n_frames, int H, int W, const int32_t* frame_idx, int n_out,
                                  int out_h, int out_w, float* out, void* stream) {
  if (!frames || !frame_idx || !out) return lrce_fail(LRCE_E_ARG, "frames_resize: null pointer");
  if (n_frames <= 0 || H <= 0 || W <= 0 || out_h <= 0 || out_w <= 0 || n_out < 0)
    return lrce_fail(LRCE_E_ARG, "frames_resize: bad sizes T=%d H=%d W=%d -> %dx%d", n_frames, H, W, out_h, out_w);
  // taps per axis: 2 * ceil(support) + 1 with support = max(in / out, 1)
  const int th = 2 * ((H + out_h - 1) / out_h) + 2, tw = 2 * ((W + out_w - 1) / out_w) + 2;
  if (th > MAX_TAPS || tw > MAX_TAPS) return lrce_fail(LRCE_E_ARG, "frames_resize: downscale %dx%d -> %dx%d too large", H, W, out_h, out_w);
  if (n_out == 0) return LRCE_OK;
  const long long total = (long long)n_out * out_h * out_w;
  frames_resize_kernel<<<(unsigned)((total + 255) / 256), 256, 0, static_cast<hipStream_t>(stream)>>>(
      frames, H, W, frame_idx, n_out, out_h, out_w, out);
  return lrce_check_launch("frames_resize");
}
