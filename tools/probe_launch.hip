// probe_launch.hip — the per-kernel floor of a dependent launch chain on
// the MI355X: K back-to-back launches on one stream, timed with events
// (best of 5), for an empty kernel, a kernel that stores one word per
// block, and a 1 MiB streaming write per launch.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)

__global__ void k_empty() {}
__global__ void k_word(unsigned *p) { if (threadIdx.x == 0) p[blockIdx.x] = blockIdx.x; }
__global__ void k_stream(double *p, int n) {
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) p[i] = i;
}

int main() {
  unsigned *w;
  double *d;
  CK(hipMalloc(&w, 1 << 20));
  CK(hipMalloc(&d, 1 << 20));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  const int K = 200;
  auto run = [&](const char *name, auto launch) {
    float best = 1e30f;
    for (int r = 0; r < 6; ++r) {
      CK(hipEventRecord(a));
      for (int k = 0; k < K; ++k) launch();
      CK(hipEventRecord(b));
      CK(hipEventSynchronize(b));
      float ms;
      CK(hipEventElapsedTime(&ms, a, b));
      if (r) best = ms < best ? ms : best;
    }
    printf("%-28s %7.2f us per launch\n", name, best * 1e3 / K);
  };
  run("empty 1 block", [&] { hipLaunchKernelGGL(k_empty, dim3(1), dim3(64), 0, 0); });
  run("empty 1024 blocks", [&] { hipLaunchKernelGGL(k_empty, dim3(1024), dim3(256), 0, 0); });
  run("one word per block, 256", [&] { hipLaunchKernelGGL(k_word, dim3(256), dim3(256), 0, 0, w); });
  run("1 MiB write, 256 blocks", [&] { hipLaunchKernelGGL(k_stream, dim3(256), dim3(256), 0, 0, d, 1 << 17); });
  return 0;
}
