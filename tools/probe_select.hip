// probe_select.hip — what bounds the profile selection pass on the MI355X?
// 64M AoS particles, the first 60 % in the selected family, ~all inside the
// sphere.  Times (hipEvents, best of 5):
//   read    : positions + masses of the family read, x computed, one sum per block
//   compact : read + order-free compaction (block offset by one atomic) of x, w, idx
//   write   : the compacted outputs' bytes written contiguously, nothing read
// and prints the effective GB/s of each, to compare with select_onepass
// (same bytes plus the ordered look-back).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)

constexpr int TPB = 256, IPT = 16, TILE = TPB * IPT;

__device__ __forceinline__ uint32_t rank_below(uint64_t m) {
  return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}

template <int MODE>  // 0 read, 1 compact
__global__ void __launch_bounds__(TPB) sel(const double *__restrict__ pos, const double *__restrict__ mass,
                                           int64_t n, int64_t fam_hi, double r2, unsigned long long *ctr,
                                           double *xo, double *wo, int *io, double *sums) {
  const int w = threadIdx.x >> 6;
  const uint32_t lane = threadIdx.x & 63;
  const int64_t wbase = (int64_t)blockIdx.x * TILE + (int64_t)w * (TILE / 4);
  double px[IPT], py[IPT], pz[IPT], xv[IPT], mv[IPT];
  uint32_t inb = 0, keepb = 0, c = 0;
#pragma unroll
  for (int k = 0; k < IPT; ++k) {
    const int64_t i = wbase + k * 64 + lane;
    const bool in = i < n && i < fam_hi;
    inb |= (uint32_t)in << k;
    const double *q = pos + 3 * (in ? i : 0);
    px[k] = q[0]; py[k] = q[1]; pz[k] = q[2];
  }
#pragma unroll
  for (int k = 0; k < IPT; ++k) {
    const double d2 = (px[k] * px[k] + py[k] * py[k]) + pz[k] * pz[k];
    const bool keep = ((inb >> k) & 1u) && d2 < r2;
    keepb |= (uint32_t)keep << k;
    xv[k] = __builtin_sqrt(d2);
    c += __popcll(__ballot(keep));
  }
#pragma unroll
  for (int k = 0; k < IPT; ++k) mv[k] = mass[((keepb >> k) & 1u) ? wbase + k * 64 + lane : 0];
  if (MODE == 0) {
    double s = 0;
#pragma unroll
    for (int k = 0; k < IPT; ++k) s += ((keepb >> k) & 1u) ? xv[k] + mv[k] : 0.0;
    for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
    if (lane == 0) sums[blockIdx.x * 4 + w] = s;
    return;
  }
  __shared__ uint32_t wc[4];
  __shared__ unsigned long long base;
  if (lane == 0) wc[w] = c;
  __syncthreads();
  if (threadIdx.x == 0) base = atomicAdd(ctr, (unsigned long long)(wc[0] + wc[1] + wc[2] + wc[3]));
  __syncthreads();
  uint64_t run = base;
  for (int ww = 0; ww < w; ++ww) run += wc[ww];
#pragma unroll
  for (int k = 0; k < IPT; ++k) {
    const bool keep = (keepb >> k) & 1u;
    const uint64_t b = __ballot(keep);
    if (keep) {
      const uint64_t o = run + rank_below(b);
      xo[o] = xv[k];
      wo[o] = mv[k];
      io[o] = (int)(wbase + k * 64 + lane);
    }
    run += __popcll(b);
  }
}

__global__ void __launch_bounds__(TPB) wr(int64_t m, double *xo, double *wo, int *io) {
  for (int64_t i = (int64_t)blockIdx.x * TPB + threadIdx.x; i < m; i += (int64_t)gridDim.x * TPB) {
    xo[i] = (double)i;
    wo[i] = 1.0;
    io[i] = (int)i;
  }
}

int main() {
  const int64_t n = 64000000, fam = n * 6 / 10;
  std::vector<double> hp(3 * n), hm(n, 1.0 / n);
  uint64_t s = 12345;
  auto rnd = [&]() { s = s * 6364136223846793005ull + 1442695040888963407ull; return ((s >> 11) * 0x1.0p-53) * 2 - 1; };
  for (int64_t i = 0; i < 3 * n; ++i) hp[i] = rnd();
  double *pos, *mass, *xo, *wo, *sums;
  int *io;
  unsigned long long *ctr;
  CK(hipMalloc(&pos, 24 * n)); CK(hipMalloc(&mass, 8 * n));
  CK(hipMalloc(&xo, 8 * n)); CK(hipMalloc(&wo, 8 * n)); CK(hipMalloc(&io, 4 * n));
  CK(hipMalloc(&sums, 8 * (n / TILE + 1) * 4)); CK(hipMalloc(&ctr, 8));
  CK(hipMemcpy(pos, hp.data(), 24 * n, hipMemcpyHostToDevice));
  CK(hipMemcpy(mass, hm.data(), 8 * n, hipMemcpyHostToDevice));
  const int nt = (int)((n + TILE - 1) / TILE);
  const double r2 = 2.9;  // keeps ~all of the cube (corner regions excluded)
  hipEvent_t a, b;
  CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
  unsigned long long kept = 0;
  auto timeit = [&](const char *name, auto launch, double bytes) {
    float best = 1e30f;
    for (int r = 0; r < 6; ++r) {
      CK(hipMemset(ctr, 0, 8));
      CK(hipEventRecord(a));
      launch();
      CK(hipEventRecord(b));
      CK(hipEventSynchronize(b));
      float ms;
      CK(hipEventElapsedTime(&ms, a, b));
      if (r) best = ms < best ? ms : best;
    }
    printf("%-8s %8.1f us  %7.0f GB/s  (%.0f MB)\n", name, best * 1e3, bytes / (best * 1e-3) / 1e9, bytes / 1e6);
  };
  timeit("compact", [&] { hipLaunchKernelGGL(sel<1>, dim3(nt), dim3(TPB), 0, 0, pos, mass, n, fam, r2, ctr, xo, wo, io, sums); }, 0);
  CK(hipMemcpy(&kept, ctr, 8, hipMemcpyDeviceToHost));
  const double rd = 24.0 * fam + 8.0 * kept, wb = 20.0 * kept;
  printf("kept %llu of %lld family\n", kept, (long long)fam);
  timeit("read", [&] { hipLaunchKernelGGL(sel<0>, dim3(nt), dim3(TPB), 0, 0, pos, mass, n, fam, r2, ctr, xo, wo, io, sums); }, rd);
  timeit("compact", [&] { hipLaunchKernelGGL(sel<1>, dim3(nt), dim3(TPB), 0, 0, pos, mass, n, fam, r2, ctr, xo, wo, io, sums); }, rd + wb);
  timeit("write", [&] { hipLaunchKernelGGL(wr, dim3(4096), dim3(TPB), 0, 0, (int64_t)kept, xo, wo, io); }, wb);
  return 0;
}
