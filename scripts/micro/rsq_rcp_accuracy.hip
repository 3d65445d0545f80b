// Accuracy of the gfx950 f64 approximation instructions (measurement only):
// v_rsq_f64 and v_rcp_f64 on their own and after one Newton step, against
// the host's long-double evaluation, over s in [1, 4) (k_cloud's ray norms:
// s = x^2 + y^2 + 1) and d in [2^-20, 2) (plane denominators).  Prints the
// largest relative errors in units of 2^-53.
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <vector>

constexpr int kN = 1 << 22;

__global__ void k(const double* s, const double* d, double* o) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= kN) return;
  const double y = __builtin_amdgcn_rsq(s[i]);
  // one Newton step for 1/sqrt(s): y (1.5 - 0.5 s y^2)
  const double h = 0.5 * s[i];
  const double e = __builtin_fma(-h * y, y, 0.5);
  const double y1 = __builtin_fma(y, e, y);
  const double r = __builtin_amdgcn_rcp(d[i]);
  const double f = __builtin_fma(-d[i], r, 1.0);
  const double r1 = __builtin_fma(r, f, r);
  o[4 * i] = y;
  o[4 * i + 1] = y1;
  o[4 * i + 2] = r;
  o[4 * i + 3] = r1;
}

int main() {
  std::vector<double> s(kN), d(kN), o(4 * static_cast<size_t>(kN));
  uint64_t st = 88172645463325252ull;
  auto rnd = [&]() { st ^= st << 13; st ^= st >> 7; st ^= st << 17; return (st >> 11) * 0x1.0p-53; };
  for (int i = 0; i < kN; ++i) {
    s[i] = 1.0 + 3.0 * rnd();
    d[i] = ldexp(1.0 + rnd(), -static_cast<int>(rnd() * 21.0));
  }
  double *ds, *dd, *dO;
  if (hipMalloc(&ds, 8 * kN) || hipMalloc(&dd, 8 * kN) || hipMalloc(&dO, 32 * kN)) return 1;
  hipMemcpy(ds, s.data(), 8 * kN, hipMemcpyHostToDevice);
  hipMemcpy(dd, d.data(), 8 * kN, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(k, dim3(kN / 256), dim3(256), 0, 0, ds, dd, dO);
  hipMemcpy(o.data(), dO, 32 * static_cast<size_t>(kN), hipMemcpyDeviceToHost);
  double m[4] = {0, 0, 0, 0};
  for (int i = 0; i < kN; ++i) {
    const long double rs = 1.0L / sqrtl(static_cast<long double>(s[i]));
    const long double rc = 1.0L / static_cast<long double>(d[i]);
    const long double e[4] = {fabsl(o[4 * i] - rs) / rs, fabsl(o[4 * i + 1] - rs) / rs, fabsl(o[4 * i + 2] - rc) / rc,
                              fabsl(o[4 * i + 3] - rc) / rc};
    for (int k2 = 0; k2 < 4; ++k2) m[k2] = fmax(m[k2], static_cast<double>(e[k2] * 0x1.0p53L));
  }
  printf("{\"n\": %d, \"max_rel_err_units_2^-53\": {\"rsq\": %.3f, \"rsq_nr1\": %.3f, \"rcp\": %.3f, \"rcp_nr1\": %.3f}}\n",
         kN, m[0], m[1], m[2], m[3]);
  return 0;
}
