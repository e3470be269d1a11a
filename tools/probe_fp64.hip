// probe_fp64.hip — measures on the MI355X: accuracy of v_rsq_f64 (raw and
// with one Newton step) and the issue cost of FP64 VALU ops, to size the
// direct-sum kernel's per-pair instruction budget.
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s\n", hipGetErrorString(e)); exit(1);} } while (0)

__global__ void rsq_kernel(const double* in, double* raw, double* nr, int n) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  double x = in[i];
  double y = __builtin_amdgcn_rsq(x);
  raw[i] = y;
  double e = __builtin_fma(-x * y, y, 1.0);
  nr[i] = __builtin_fma(0.5 * y, e, y);
}

// chains of independent ops per lane; OP: 0 fma, 1 rsq, 2 mul, 3 rsq_f32 via cvt
template <int OP>
__global__ void tput(double* out, int iters, double seed) {
  double a0 = seed + threadIdx.x * 1e-9, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3;
  double a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
  for (int i = 0; i < iters; ++i) {
#define STEP(a) if (OP == 0) a = __builtin_fma(a, 0.999999, 1e-7); \
                else if (OP == 1) a = __builtin_amdgcn_rsq(a) + 1.0; \
                else if (OP == 2) a = a * 1.0000001; \
                else a = (double)__builtin_amdgcn_rsqf((float)a) + 1.0;
    STEP(a0) STEP(a1) STEP(a2) STEP(a3) STEP(a4) STEP(a5) STEP(a6) STEP(a7)
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7;
}

int main() {
  const int n = 1 << 22;
  std::vector<double> h(n), raw(n), nr(n);
  std::mt19937_64 g(1);
  std::uniform_real_distribution<double> u(-30.0, 30.0);
  for (int i = 0; i < n; ++i) h[i] = std::pow(10.0, u(g)) * (1.0 + 1e-3 * (i % 7));
  h[0] = 2.2250738585072014e-308; h[1] = 1.0; h[2] = 4.0; h[3] = 1e300;
  double *d_in, *d_raw, *d_nr;
  CK(hipMalloc(&d_in, n * 8)); CK(hipMalloc(&d_raw, n * 8)); CK(hipMalloc(&d_nr, n * 8));
  CK(hipMemcpy(d_in, h.data(), n * 8, hipMemcpyHostToDevice));
  rsq_kernel<<<n / 256, 256>>>(d_in, d_raw, d_nr, n);
  CK(hipMemcpy(raw.data(), d_raw, n * 8, hipMemcpyDeviceToHost));
  CK(hipMemcpy(nr.data(), d_nr, n * 8, hipMemcpyDeviceToHost));
  double eraw = 0, enr = 0;
  for (int i = 0; i < n; ++i) {
    long double ref = 1.0L / sqrtl((long double)h[i]);
    double r1 = (double)fabsl((raw[i] - ref) / ref), r2 = (double)fabsl((nr[i] - ref) / ref);
    if (r1 > eraw) eraw = r1;
    if (r2 > enr) enr = r2;
  }
  printf("rsq_f64 raw max rel err %.3e ; with 1 NR %.3e ; rsq(tiny)=%.6e\n", eraw, enr, raw[0]);

  hipDeviceProp_t p; CK(hipGetDeviceProperties(&p, 0));
  int cus = p.multiProcessorCount;
  double* d_out; CK(hipMalloc(&d_out, 1 << 26));
  const int iters = 20000;
  const char* names[] = {"v_fma_f64", "v_rsq_f64(+add)", "v_mul_f64", "cvt+rsq_f32+cvt(+add)"};
  for (int op = 0; op < 4; ++op) {
    hipEvent_t a, b; CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
    dim3 grid(cus * 8), blk(256);
    for (int rep = 0; rep < 2; ++rep) {
      CK(hipEventRecord(a));
      if (op == 0) tput<0><<<grid, blk>>>(d_out, iters, 1.5);
      if (op == 1) tput<1><<<grid, blk>>>(d_out, iters, 1.5);
      if (op == 2) tput<2><<<grid, blk>>>(d_out, iters, 1.5);
      if (op == 3) tput<3><<<grid, blk>>>(d_out, iters, 1.5);
      CK(hipEventRecord(b)); CK(hipEventSynchronize(b));
    }
    float ms; CK(hipEventElapsedTime(&ms, a, b));
    double lane_ops = (double)grid.x * blk.x * iters * 8;
    double ops_per_s = lane_ops / (ms * 1e-3);
    // cycles per wave64 instruction per SIMD at the nominal 2.4 GHz
    double cyc = (cus * 4.0 * 2.4e9) / (ops_per_s / 64.0);
    printf("%-24s %8.3f ms  %.3e lane-ops/s  ~%.2f cyc/wave-instr/SIMD @2.4GHz\n", names[op], ms,
           ops_per_s, cyc);
  }
  printf("device %s CUs %d clock %d kHz\n", p.name, cus, p.clockRate);
  return 0;
}
