// fp_probe.hip -- checks that float64 sqrt / div / mul / add on gfx950 are
// correctly rounded (bit-identical to the host), the premise of the
// bit-exact NCC / DTW / YIN parity claims.
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <random>
#include <vector>
__global__ void probe(const double* a, const double* b, double* o, int n) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  o[4 * i + 0] = sqrt(a[i]);
  o[4 * i + 1] = __ddiv_rn(a[i], b[i]);
  o[4 * i + 2] = __dsqrt_rn(a[i]);
  o[4 * i + 3] = __builtin_amdgcn_sqrt(a[i]);
}
int main() {
  const int n = 1 << 22;
  std::vector<double> a(n), b(n), o(4 * (size_t)n);
  std::mt19937_64 g(1);
  std::uniform_real_distribution<double> u(0, 1);
  for (int i = 0; i < n; i++) { a[i] = std::ldexp(u(g), (int)(g() % 80) - 40); b[i] = std::ldexp(u(g) + 0.5, (int)(g() % 20) - 10); }
  double *da, *db, *dout;
  hipMalloc(&da, n * 8); hipMalloc(&db, n * 8); hipMalloc(&dout, 32 * (size_t)n);
  hipMemcpy(da, a.data(), n * 8, hipMemcpyHostToDevice); hipMemcpy(db, b.data(), n * 8, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(probe, dim3((n + 255) / 256), dim3(256), 0, 0, da, db, dout, n);
  hipMemcpy(o.data(), dout, 32 * (size_t)n, hipMemcpyDeviceToHost);
  long bad[4] = {0, 0, 0, 0};
  for (int i = 0; i < n; i++) {
    double r[4] = {std::sqrt(a[i]), a[i] / b[i], std::sqrt(a[i]), std::sqrt(a[i])};
    for (int k = 0; k < 4; k++) if (std::memcmp(&r[k], &o[4 * (size_t)i + k], 8)) bad[k]++;
  }
  std::printf("mismatches of %d: sqrt=%ld ddiv_rn=%ld dsqrt_rn=%ld amdgcn_sqrt=%ld\n", n, bad[0], bad[1], bad[2], bad[3]);
  return 0;
}
