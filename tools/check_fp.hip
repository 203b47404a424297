// Checks device float primitives against the host (IEEE round-to-nearest).
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <random>
#include <vector>

__global__ void k(const float* a, const float* b, int n, float* o_sqrt, float* o_div, float* o_dd,
                  float* o_round, float* o_plain_div, float* o_plain_sqrt) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  o_sqrt[i] = __fsqrt_rn(a[i]);
  o_div[i] = __fdiv_rn(a[i], b[i]);
  o_dd[i] = static_cast<float>(static_cast<double>(a[i]) / 3.14159265358979323846);
  o_round[i] = roundf(a[i] - 0.5f);
  o_plain_div[i] = a[i] / b[i];
  o_plain_sqrt[i] = sqrtf(a[i]);
}

int main() {
  const int n = 1 << 22;
  std::mt19937 g(3);
  std::uniform_real_distribution<float> U(1e-4f, 100.f);
  std::vector<float> a(n), b(n);
  for (int i = 0; i < n; ++i) { a[i] = U(g); b[i] = U(g); }
  float *da, *db, *o[6];
  hipMalloc(&da, 4 * n); hipMalloc(&db, 4 * n);
  for (auto& p : o) hipMalloc(&p, 4 * n);
  hipMemcpy(da, a.data(), 4 * n, hipMemcpyHostToDevice);
  hipMemcpy(db, b.data(), 4 * n, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(k, dim3(n / 256), dim3(256), 0, 0, da, db, n, o[0], o[1], o[2], o[3], o[4], o[5]);
  std::vector<float> r[6];
  for (int j = 0; j < 6; ++j) { r[j].resize(n); hipMemcpy(r[j].data(), o[j], 4 * n, hipMemcpyDeviceToHost); }
  int bad[6] = {0};
  for (int i = 0; i < n; ++i) {
    if (r[0][i] != std::sqrt(a[i])) ++bad[0];
    if (r[1][i] != a[i] / b[i]) ++bad[1];
    if (r[2][i] != static_cast<float>(static_cast<double>(a[i]) / M_PI)) ++bad[2];
    if (r[3][i] != std::round(a[i] - 0.5f)) ++bad[3];
    if (r[4][i] != a[i] / b[i]) ++bad[4];
    if (r[5][i] != std::sqrt(a[i])) ++bad[5];
  }
  printf("mismatches of %d: fsqrt_rn %d fdiv_rn %d ddiv %d roundf %d plain_div %d sqrtf %d\n", n,
         bad[0], bad[1], bad[2], bad[3], bad[4], bad[5]);
  return 0;
}
