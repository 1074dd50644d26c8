// pk_selftest.hip -- checks the packed-f32 (VOP3P op_sel / neg) complex helpers of
// sonido-sonar_amd/csrc/pk_complex.h against scalar arithmetic on the GPU.
//   hipcc -O3 --offload-arch=gfx950 -I sonido-sonar_amd/csrc tools/pk_selftest.hip -o tools/pk_selftest
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <vector>

#include "pk_complex.h"

using namespace sonar::pk;

constexpr int kOps = 18;

__global__ void pk_kernel(const float2* a, const float2* b, float2* out, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const cf x = cf{a[i].x, a[i].y}, y = cf{b[i].x, b[i].y};
  cf r[kOps];
  r[0] = cadd(x, y);
  r[1] = csub(x, y);
  r[2] = cadd_mi(x, y);
  r[3] = csub_mi(x, y);
  r[4] = cmul(x, y);
  r[5] = swapadd(x);
  r[6] = fma_k(x, y);
  r[7] = fnma_k(x, y);
  r[8] = fma_k_mi(x, y);
  r[9] = fnma_k_mi(x, y);
  r[10] = negi(x);
  r[11] = mul_k(x);
  r[12] = mul_k_mi(x);
  r[13] = pw2(x, y);
  r[14] = fma_bx(x, y, r[0]);
  r[15] = fma_by(x, y, r[1]);
  r[16] = mul_bx(x, y);
  r[17] = mul_by(x, y);
  for (int k = 0; k < kOps; k++) out[i * kOps + k] = make_float2(r[k].x, r[k].y);
}

int main() {
  const int n = 4096;
  std::vector<float2> a(n), b(n), o(n * kOps);
  unsigned s = 1;
  auto rnd = [&]() { s = s * 1664525u + 1013904223u; return ((s >> 8) / 16777216.0f) * 2.f - 1.f; };
  for (int i = 0; i < n; i++) { a[i] = make_float2(rnd(), rnd()); b[i] = make_float2(rnd(), rnd()); }
  float2 *da, *db, *dout;
  if (hipMalloc(&da, n * 8) || hipMalloc(&db, n * 8) || hipMalloc(&dout, n * kOps * 8)) return 2;
  hipMemcpy(da, a.data(), n * 8, hipMemcpyHostToDevice);
  hipMemcpy(db, b.data(), n * 8, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(pk_kernel, dim3(n / 256), dim3(256), 0, 0, da, db, dout, n);
  if (hipMemcpy(o.data(), dout, n * kOps * 8, hipMemcpyDeviceToHost) != hipSuccess) return 2;
  const double k = 0.70710678118654752440;
  const char* names[kOps] = {"cadd", "csub", "cadd_mi", "csub_mi", "cmul", "swapadd", "fma_k", "fnma_k",
                             "fma_k_mi", "fnma_k_mi", "negi", "mul_k", "mul_k_mi", "pw2", "fma_bx", "fma_by",
                             "mul_bx", "mul_by"};
  double worst[kOps] = {0};
  for (int i = 0; i < n; i++) {
    const double ax = a[i].x, ay = a[i].y, bx = b[i].x, by = b[i].y;
    const double e[kOps][2] = {
        {ax + bx, ay + by}, {ax - bx, ay - by}, {ax + by, ay - bx}, {ax - by, ay + bx},
        {ax * bx - ay * by, ax * by + ay * bx}, {ax + ay, ay - ax},
        {bx + k * ax, by + k * ay}, {bx - k * ax, by - k * ay},
        {bx + k * ay, by - k * ax}, {bx - k * ay, by + k * ax},
        {ay, -ax}, {k * ax, k * ay}, {k * ay, -k * ax},
        {(ax + bx) * (ax + bx) + (ay - by) * (ay - by), (ax - bx) * (ax - bx) + (ay + by) * (ay + by)},
        {ax * bx + (ax + bx), ax * by + (ay + by)}, {ay * bx + (ax - bx), ay * by + (ay - by)},
        {ax * bx, ay * bx}, {ax * by, ay * by}};
    for (int q = 0; q < kOps; q++)
      for (int c = 0; c < 2; c++) {
        const double g = c ? o[i * kOps + q].y : o[i * kOps + q].x;
        const double d = std::fabs(g - e[q][c]);
        if (!(d <= worst[q])) worst[q] = d;
      }
  }
  int bad = 0;
  for (int q = 0; q < kOps; q++) {
    const bool ok = worst[q] < 1e-5;
    bad += !ok;
    printf("%-10s max abs err %.3g %s\n", names[q], worst[q], ok ? "ok" : "FAIL");
  }
  printf(bad ? "PK SELFTEST FAILED\n" : "PK SELFTEST OK\n");
  return bad ? 1 : 0;
}
