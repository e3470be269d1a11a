// probe_stream.hip — the data movement of the tiled selection (select_tiles)
// alone: n AoS f64 positions (24 B each) read, one f64 per particle written
// in particle order, at the 64M bench point's family span (38.4M particles).
// Variants (hipEvents, best of 6 after a warm-up):
//   rd3    : three 8-byte loads per particle (lane stride 24 B), r^2 summed per block
//   rd3w   : rd3 + sqrt(r^2) stored by particle slot (select_tiles' pattern)
//   rd4    : the same bytes as 16-byte coalesced loads, r^2 from an LDS transpose, summed
//   rd4w   : rd4 + sqrt(r^2) stored by slot
//   rd3nt  : rd3w with nt stores
//   rd2p(w): lane pairs — a lane's two consecutive particles as three 16-byte
//            loads, their two x as one 16-byte nt store
//   copy4  : float4 copy of the position bytes (reference rate)
// usage: probe_stream [n]
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)

constexpr int BT = 512, PPL = 8, TILE = BT * PPL;  // 4096 particles per block

template <bool WR>
__global__ void __launch_bounds__(BT) rd3(const double *__restrict__ pos, int64_t n, double *__restrict__ xo,
                                          double *__restrict__ sums) {
  const int64_t b0 = (int64_t)blockIdx.x * TILE + (threadIdx.x >> 6) * (TILE / (BT / 64));
  const uint32_t lane = threadIdx.x & 63;
  double px[PPL], py[PPL], pz[PPL];
#pragma unroll
  for (int k = 0; k < PPL; ++k) {
    const int64_t i = b0 + k * 64 + lane;
    const double *q = pos + 3 * (i < n ? i : 0);
    px[k] = q[0]; py[k] = q[1]; pz[k] = q[2];
  }
  double s = 0;
#pragma unroll
  for (int k = 0; k < PPL; ++k) {
    const int64_t i = b0 + k * 64 + lane;
    const double r2 = (px[k] * px[k] + py[k] * py[k]) + pz[k] * pz[k];
    if (WR) {
      if (i < n) xo[i] = __builtin_sqrt(r2);
    } else {
      s += r2;
    }
  }
  if (!WR) {
    for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
    if (lane == 0) sums[blockIdx.x * (BT / 64) + (threadIdx.x >> 6)] = s;
  }
}

// 16-B loads: a wave's 512 particles = 12 KB = 768 x 16 B = 12 loads per lane,
// staged through LDS (per-wave 12 KB region), then read back per particle
template <bool WR>
__global__ void __launch_bounds__(BT) rd4(const double *__restrict__ pos, int64_t n, double *__restrict__ xo,
                                          double *__restrict__ sums) {
  __shared__ double4 lds[BT / 64][TILE / (BT / 64) * 3 / 4];  // 8 waves x 384 double4 (12 KB each)
  const int w = threadIdx.x >> 6;
  const uint32_t lane = threadIdx.x & 63;
  const int64_t b0 = (int64_t)blockIdx.x * TILE + w * (TILE / (BT / 64));  // first particle of the wave
  const double2 *src = (const double2 *)(pos + 3 * b0);
  const int64_t lim2 = (3 * n - 3 * b0) / 2;  // double2 units available
  double2 v[12];
#pragma unroll
  for (int k = 0; k < 12; ++k) {
    const int64_t j = k * 64 + lane;
    v[k] = src[j < lim2 ? j : 0];
  }
  double2 *l2 = (double2 *)lds[w];
#pragma unroll
  for (int k = 0; k < 12; ++k) l2[k * 64 + lane] = v[k];
  __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0)
  __builtin_amdgcn_wave_barrier();
  const double *l1 = (const double *)lds[w];
  double s = 0;
#pragma unroll
  for (int k = 0; k < PPL; ++k) {
    const int p = k * 64 + lane;
    const double x = l1[3 * p], y = l1[3 * p + 1], z = l1[3 * p + 2];
    const double r2 = (x * x + y * y) + z * z;
    const int64_t i = b0 + p;
    if (WR) {
      if (i < n) xo[i] = __builtin_sqrt(r2);
    } else {
      s += r2;
    }
  }
  if (!WR) {
    for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
    if (lane == 0) sums[blockIdx.x * (BT / 64) + w] = s;
  }
}

// lane-pair layout: lane l of a wave's 128-particle group holds particles
// 2l and 2l + 1 (48 contiguous bytes: three 16-byte loads) and stores their
// two x as one 16-byte store
template <bool WR>
__global__ void __launch_bounds__(BT) rd2p(const double *__restrict__ pos, int64_t n,
                                           double *__restrict__ xo, double *__restrict__ sums) {
  const int64_t b0 = (int64_t)blockIdx.x * TILE + (threadIdx.x >> 6) * (TILE / (BT / 64));
  const uint32_t lane = threadIdx.x & 63;
  constexpr int G = PPL / 2;  // 128-particle groups per wave slice
  double2 q[G][3];
#pragma unroll
  for (int k = 0; k < G; ++k) {
    const int64_t i = b0 + k * 128 + 2 * lane;
    const double2 *src = (const double2 *)(pos + 3 * (i + 1 < n ? i : 0));
    q[k][0] = src[0];
    q[k][1] = src[1];
    q[k][2] = src[2];
  }
  double s = 0;
#pragma unroll
  for (int k = 0; k < G; ++k) {
    const double x0 = q[k][0].x, y0 = q[k][0].y, z0 = q[k][1].x;
    const double x1 = q[k][1].y, y1 = q[k][2].x, z1 = q[k][2].y;
    const double r0 = (x0 * x0 + y0 * y0) + z0 * z0, r1 = (x1 * x1 + y1 * y1) + z1 * z1;
    const int64_t i = b0 + k * 128 + 2 * lane;
    if (WR) {
      typedef double d2v __attribute__((ext_vector_type(2)));
      d2v o;
      o.x = __builtin_sqrt(r0);
      o.y = __builtin_sqrt(r1);
      if (i + 1 < n) __builtin_nontemporal_store(o, (d2v *)(xo + i));
    } else {
      s += r0 + r1;
    }
  }
  if (!WR) {
    for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
    if (lane == 0) sums[blockIdx.x * (BT / 64) + (threadIdx.x >> 6)] = s;
  }
}

// rd3w with nt stores (select_tiles' store flavour)
__global__ void __launch_bounds__(BT) rd3nt(const double *__restrict__ pos, int64_t n, double *__restrict__ xo) {
  const int64_t b0 = (int64_t)blockIdx.x * TILE + (threadIdx.x >> 6) * (TILE / (BT / 64));
  const uint32_t lane = threadIdx.x & 63;
  double px[PPL], py[PPL], pz[PPL];
#pragma unroll
  for (int k = 0; k < PPL; ++k) {
    const int64_t i = b0 + k * 64 + lane;
    const double *q = pos + 3 * (i < n ? i : 0);
    px[k] = q[0]; py[k] = q[1]; pz[k] = q[2];
  }
#pragma unroll
  for (int k = 0; k < PPL; ++k) {
    const int64_t i = b0 + k * 64 + lane;
    const double r2 = (px[k] * px[k] + py[k] * py[k]) + pz[k] * pz[k];
    if (i < n) __builtin_nontemporal_store(__builtin_sqrt(r2), xo + i);
  }
}

__global__ void __launch_bounds__(256) copy4(const double4 *__restrict__ a, double4 *__restrict__ b, int64_t m) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < m; i += (int64_t)gridDim.x * 256) b[i] = a[i];
}

int main(int argc, char **argv) {
  const int64_t n = argc > 1 ? atoll(argv[1]) : 38400000;
  std::vector<double> hp(3 * n);
  uint64_t s = 12345;
  auto rnd = [&]() { s = s * 6364136223846793005ull + 1442695040888963407ull; return ((s >> 11) * 0x1.0p-53) * 2 - 1; };
  for (int64_t i = 0; i < 3 * n; ++i) hp[i] = rnd();
  double *pos, *xo, *sums, *cp;
  const int nt = (int)((n + TILE - 1) / TILE);
  CK(hipMalloc(&pos, 24 * n + 64)); CK(hipMalloc(&xo, 8 * n)); CK(hipMalloc(&cp, 24 * n + 64));
  CK(hipMalloc(&sums, 8 * (size_t)nt * (BT / 64)));
  CK(hipMemcpy(pos, hp.data(), 24 * n, hipMemcpyHostToDevice));
  hipEvent_t a, b;
  CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
  auto timeit = [&](const char *name, auto launch, double bytes) {
    float best = 1e30f;
    for (int r = 0; r < 7; ++r) {
      CK(hipEventRecord(a));
      launch();
      CK(hipEventRecord(b));
      CK(hipEventSynchronize(b));
      float ms;
      CK(hipEventElapsedTime(&ms, a, b));
      if (r) best = ms < best ? ms : best;
    }
    printf("%-6s %8.1f us  %7.0f GB/s  (%.0f MB)\n", name, best * 1e3, bytes / (best * 1e-3) / 1e9, bytes / 1e6);
  };
  const double R = 24.0 * n, W = 8.0 * n;
  printf("n = %lld particles, %d tiles of %d\n", (long long)n, nt, TILE);
  timeit("rd3", [&] { hipLaunchKernelGGL(rd3<false>, dim3(nt), dim3(BT), 0, 0, pos, n, xo, sums); }, R);
  timeit("rd3w", [&] { hipLaunchKernelGGL(rd3<true>, dim3(nt), dim3(BT), 0, 0, pos, n, xo, sums); }, R + W);
  timeit("rd4", [&] { hipLaunchKernelGGL(rd4<false>, dim3(nt), dim3(BT), 0, 0, pos, n, xo, sums); }, R);
  timeit("rd4w", [&] { hipLaunchKernelGGL(rd4<true>, dim3(nt), dim3(BT), 0, 0, pos, n, xo, sums); }, R + W);
  timeit("rd3nt", [&] { hipLaunchKernelGGL(rd3nt, dim3(nt), dim3(BT), 0, 0, pos, n, xo); }, R + W);
  timeit("rd2p", [&] { hipLaunchKernelGGL(rd2p<false>, dim3(nt), dim3(BT), 0, 0, pos, n, xo, sums); }, R);
  timeit("rd2pw", [&] { hipLaunchKernelGGL(rd2p<true>, dim3(nt), dim3(BT), 0, 0, pos, n, xo, sums); }, R + W);
  timeit("copy4", [&] { hipLaunchKernelGGL(copy4, dim3(4096), dim3(256), 0, 0, (const double4 *)pos, (double4 *)cp, (int64_t)(3 * n / 4)); }, 2 * R);
  return 0;
}
