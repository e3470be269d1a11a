// probe_rsq.hip — accuracy of the hardware v_rsq_f64 (no Newton step) on
// gfx950 against a correctly rounded 1/sqrt computed in long double on the
// host.  Inputs: random mantissas over exponents 2^-60 .. 2^60.
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>

__global__ void rsq(const double *x, double *y, double *z, int n) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const double v = x[i];
  const double r = __builtin_amdgcn_rsq(v);  // v_rsq_f64
  y[i] = r;
  // one Newton step: r (1.5 - 0.5 v r^2)
  const double h = __builtin_fma(-v * r, r, 1.0);
  z[i] = __builtin_fma(r * 0.5, h, r);
}

int main() {
  const int n = 1 << 22;
  std::vector<double> x(n), y(n), z(n);
  std::mt19937_64 g(7);
  std::uniform_real_distribution<double> u(1.0, 2.0);
  std::uniform_int_distribution<int> e(-60, 60);
  for (int i = 0; i < n; ++i) x[i] = std::ldexp(u(g), e(g));
  double *dx, *dy, *dz;
  hipMalloc(&dx, n * 8);
  hipMalloc(&dy, n * 8);
  hipMalloc(&dz, n * 8);
  hipMemcpy(dx, x.data(), n * 8, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(rsq, dim3(n / 256), dim3(256), 0, 0, dx, dy, dz, n);
  hipMemcpy(y.data(), dy, n * 8, hipMemcpyDeviceToHost);
  hipMemcpy(z.data(), dz, n * 8, hipMemcpyDeviceToHost);
  double m0 = 0, m1 = 0, s0 = 0;
  for (int i = 0; i < n; ++i) {
    const long double t = 1.0L / std::sqrt((long double)x[i]);
    const double e0 = (double)std::fabs((y[i] - t) / t), e1 = (double)std::fabs((z[i] - t) / t);
    m0 = std::max(m0, e0);
    m1 = std::max(m1, e1);
    s0 += e0;
  }
  std::printf("v_rsq_f64 max rel err %.3e (%.2f ulp-ish), mean %.3e; with one Newton step %.3e\n",
              m0, m0 / 1.1102230246251565e-16, s0 / n, m1);
  return 0;
}
