// probe_mfma.hip — does FP64 MFMA (v_mfma_f64_16x16x4_f64) issue on a pipe
// separate from the FP64 VALU on gfx950?  Measures three loops on the whole
// chip: VALU v_fma_f64 only, MFMA only, and both interleaved in every wave
// (independent chains).  If the mixed loop finishes in about max() rather
// than sum() of the two, MFMA throughput is additional to the VALU's.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s\n", hipGetErrorString(e)); exit(1);} } while (0)

typedef double v4d __attribute__((ext_vector_type(4)));

template <int MODE>  // 0 valu, 1 mfma, 2 both
__global__ void __launch_bounds__(256) probe(double *out, int iters, double seed) {
  double a0 = seed + threadIdx.x * 1e-9, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3;
  double a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
  v4d c0 = {a0, a1, a2, a3}, c1 = {a4, a5, a6, a7}, c2 = c0 + 1.0, c3 = c1 + 1.0;
  const double x = 1.0 + threadIdx.x * 1e-12, y = 0.999999;
  for (int i = 0; i < iters; ++i) {
    if (MODE != 1) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        a0 = __builtin_fma(a0, y, 1e-7); a1 = __builtin_fma(a1, y, 1e-7);
        a2 = __builtin_fma(a2, y, 1e-7); a3 = __builtin_fma(a3, y, 1e-7);
        a4 = __builtin_fma(a4, y, 1e-7); a5 = __builtin_fma(a5, y, 1e-7);
        a6 = __builtin_fma(a6, y, 1e-7); a7 = __builtin_fma(a7, y, 1e-7);
      }
    }
    if (MODE != 0) {
      c0 = __builtin_amdgcn_mfma_f64_16x16x4f64(x, y, c0, 0, 0, 0);
      c1 = __builtin_amdgcn_mfma_f64_16x16x4f64(x, y, c1, 0, 0, 0);
      c2 = __builtin_amdgcn_mfma_f64_16x16x4f64(x, y, c2, 0, 0, 0);
      c3 = __builtin_amdgcn_mfma_f64_16x16x4f64(x, y, c3, 0, 0, 0);
    }
  }
  double s = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7;
  s += c0[0] + c1[1] + c2[2] + c3[3] + c0[3] + c1[2] + c2[1] + c3[0];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

int main() {
  hipDeviceProp_t p;
  CK(hipGetDeviceProperties(&p, 0));
  const int cus = p.multiProcessorCount;
  const int blocks = cus * 8, threads = 256, iters = 20000;
  double *out;
  CK(hipMalloc(&out, sizeof(double) * blocks * threads));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const char *names[3] = {"valu fma_f64 x32/iter", "mfma_f64_16x16x4 x4/iter", "both"};
  for (int mode = 0; mode < 3; ++mode) {
    for (int rep = 0; rep < 2; ++rep) {
      CK(hipEventRecord(e0));
      if (mode == 0) hipLaunchKernelGGL(probe<0>, dim3(blocks), dim3(threads), 0, 0, out, iters, 1.0);
      if (mode == 1) hipLaunchKernelGGL(probe<1>, dim3(blocks), dim3(threads), 0, 0, out, iters, 1.0);
      if (mode == 2) hipLaunchKernelGGL(probe<2>, dim3(blocks), dim3(threads), 0, 0, out, iters, 1.0);
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      if (rep == 1) {
        const double waves = (double)blocks * threads / 64.0;
        const double valu_flops = (mode != 1) ? waves * 64 * 32.0 * 2 * iters : 0.0;
        const double mfma_flops = (mode != 0) ? waves * 4.0 * 2048.0 * iters : 0.0;
        printf("%-26s %8.3f ms  valu %.1f TF  mfma %.1f TF  total %.1f TF\n", names[mode], ms,
               valu_flops / ms / 1e9, mfma_flops / ms / 1e9, (valu_flops + mfma_flops) / ms / 1e9);
      }
    }
  }
  printf("device %s CUs %d\n", p.gcnArchName, cus);
  return 0;
}
