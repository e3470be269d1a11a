// Probe: do same-address lanes of ONE returning LDS atomic (ds_add_rtn_u32)
// get their old values in ascending lane order on gfx950?  For every wave
// instruction the returned value of lane l must equal the count of equal
// addresses in lanes < l (plus the counter before).  Counts mismatches over
// many random digit patterns, address strides and wave counts.
// build: hipcc --offload-arch=gfx950 -O3 tools/probe_ldsorder.hip -o tools/probe_ldsorder
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

__device__ __forceinline__ uint32_t lane_id() {
  return __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u));
}
__device__ __forceinline__ uint32_t rank_below(uint64_t m) {
  return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}
__device__ __forceinline__ uint64_t peers8(uint32_t d) {
  uint64_t m = ~0ull;
  for (int b = 0; b < 9; ++b) {
    uint64_t bal = __ballot((d >> b) & 1u);
    m &= ((d >> b) & 1u) ? bal : ~bal;
  }
  return m;
}

__global__ void __launch_bounds__(256) probe(int K, int stride, int iters, unsigned long long *bad,
                                             unsigned long long *tot) {
  __shared__ uint32_t cnt[4][512 * 4];
  const int w = threadIdx.x >> 6;
  const uint32_t lane = lane_id();
  uint32_t x = 2654435761u * (blockIdx.x * 256 + threadIdx.x + 1) ^ (K * 97 + stride);
  unsigned long long nb = 0, nt = 0;
  for (int it = 0; it < iters; ++it) {
    for (int i = lane; i < 512 * 4; i += 64) cnt[w][i] = 0;
    __builtin_amdgcn_s_waitcnt(0);
    x ^= x << 13; x ^= x >> 17; x ^= x << 5;
    const uint32_t d = (x >> 8) % (uint32_t)K;
    const uint32_t r = atomicAdd(&cnt[w][d * stride], 1u);
    const uint64_t m = peers8(d);
    nb += (r != rank_below(m)) ? 1 : 0;
    nt += 1;
  }
  atomicAdd(bad, nb);
  atomicAdd(tot, nt);
}

int main() {
  unsigned long long *d;
  hipMalloc(&d, 16);
  int Ks[] = {1, 2, 3, 5, 8, 16, 33, 64, 129, 256, 511};
  int strides[] = {1, 2, 3, 4};
  unsigned long long allbad = 0;
  for (int K : Ks)
    for (int s : strides) {
      hipMemset(d, 0, 16);
      hipLaunchKernelGGL(probe, dim3(2048), dim3(256), 0, 0, K, s, 64, d, d + 1);
      unsigned long long h[2];
      hipMemcpy(h, d, 16, hipMemcpyDeviceToHost);
      printf("K=%3d stride=%d: %llu mismatches of %llu lane results\n", K, s, h[0], h[1]);
      allbad += h[0];
    }
  printf("TOTAL mismatches %llu\n", allbad);
  return allbad ? 1 : 0;
}
// Result (round 3): this standalone probe saw no exception in 1.5e9 lane
// results, but the same check inside libpbx (varying address counts and
// strides within one launch) found 307 out-of-lane-order returns in 12.6M:
// the order is NOT guaranteed, and the CSR / radix ranks keep peer masks.
