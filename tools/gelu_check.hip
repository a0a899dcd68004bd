// GELU helper check (dev tool, GPU): the packed-pair and scalar erf-GELU / derivative of csrc/common.h against
// double-precision erfc on [-12, 12]; they must agree bit for bit with each other.
//   hipcc --offload-arch=gfx950 -O3 -I vqa-lrce-kbs-2023_amd/csrc tools/gelu_check.hip -o tools/gelu_check
#include "common.h"
#include <cstdio>
#include <cmath>
__global__ void k(const float* x, float* a, float* b, float* c, float* d, int n) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (2 * i + 1 >= n) return;
  f32x2v g = gelu2(f32x2v{x[2 * i], x[2 * i + 1]}), gg = gelu_grad2(f32x2v{x[2 * i], x[2 * i + 1]});
  a[2 * i] = g.x; a[2 * i + 1] = g.y;
  b[2 * i] = gelu_f(x[2 * i]); b[2 * i + 1] = gelu_f(x[2 * i + 1]);
  c[2 * i] = gg.x; c[2 * i + 1] = gg.y;
  d[2 * i] = gelu_grad_f(x[2 * i]); d[2 * i + 1] = gelu_grad_f(x[2 * i + 1]);
}
int main() {
  const int n = 1 << 20;
  float *x, *a, *b, *c, *d;
  hipMallocManaged(&x, n * 4); hipMallocManaged(&a, n * 4); hipMallocManaged(&b, n * 4); hipMallocManaged(&c, n * 4); hipMallocManaged(&d, n * 4);
  for (int i = 0; i < n; ++i) x[i] = -12.f + 24.f * i / n;
  k<<<n / 512, 256>>>(x, a, b, c, d, n);
  hipDeviceSynchronize();
  double me = 0, mg = 0; int diff = 0;
  for (int i = 0; i < n; ++i) {
    double xx = x[i], ref = 0.5 * xx * erfc(-xx / sqrt(2.0)), refg = 0.5 * erfc(-xx / sqrt(2.0)) + xx * exp(-xx * xx / 2) / sqrt(2 * M_PI);
    me = fmax(me, fabs(a[i] - ref)); mg = fmax(mg, fabs(c[i] - refg));
    if (a[i] != b[i] || c[i] != d[i]) ++diff;
  }
  printf("max abs err gelu %.3g grad %.3g; pair vs scalar mismatches %d\n", me, mg, diff);
  return 0;
}
