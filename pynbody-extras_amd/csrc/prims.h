// prims.h — device primitives shared by the profile and octree engines:
// wave-ballot ranks, block/tile exclusive scans of u32, and one stable LSD
// radix pass (8-bit digit) over u32/u64 keys with optional int32 values.
//
// One tile = 256 threads x 16 items = 4096 elements.  A radix pass is:
// per-tile digit histogram -> exclusive scan over [digit][tile] -> stable
// scatter whose in-tile ranks come from 64-lane "peer masks" of equal
// digits (the scatter preserves input order within a digit, so a sequence
// of passes is a stable sort).
#pragma once

#include <algorithm>

#include "pbx_common.h"

namespace pbx {
namespace prim {

constexpr int TPB = 256;
constexpr int NWAVE = TPB / 64;
constexpr int IPT = 16;
constexpr int TILE = TPB * IPT;
constexpr int RADIX = 256;

// Order-preserving u64 key of a double in numpy's sort order: NaN last
// (all NaNs equal), -0.0 == +0.0.
__host__ __device__ inline uint64_t dkey(double v) {
  if (v != v) return ~0ull;
  if (v == 0.0) v = 0.0;
  uint64_t b = __builtin_bit_cast(uint64_t, v);
  return (b >> 63) ? ~b : (b | 0x8000000000000000ull);
}

__host__ __device__ inline double dkey_inv(uint64_t k) {
  uint64_t b = (k >> 63) ? (k & 0x7fffffffffffffffull) : ~k;
  return __builtin_bit_cast(double, b);
}

__device__ __forceinline__ uint32_t lane_id() {
  return __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u));
}

// In-launch hand-off loads / stores (relaxed agent-scope atomics: global
// load / store ... sc1): a word stored sc1 by its producer — whose wave
// drains vmcnt(0) before it signals — and loaded sc1 by its consumer needs
// no release / acquire fence (a fence writes back the whole XCD L2).  Used
// by radial_mono's grid barriers and the octree payload up-sweep.
template <typename T>
__device__ __forceinline__ T ld_sc1(const T *p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
template <typename T>
__device__ __forceinline__ void st_sc1(T *p, T v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ double ld_sc1d(const double *p) {
  return __builtin_bit_cast(double, ld_sc1((const uint64_t *)p));
}
__device__ __forceinline__ void st_sc1d(double *p, double v) {
  st_sc1((uint64_t *)p, __builtin_bit_cast(uint64_t, v));
}

// a zero the compiler cannot see through (a VGPR): added to a wave-uniform
// index it makes the load a vector load, counted in order by vmcnt (a
// scalar load's result is waited for with lgkmcnt(0), together with every
// LDS access in flight)
__device__ __forceinline__ uint32_t vgpr_zero() {
  uint32_t z;
  asm volatile("v_mov_b32 %0, 0" : "=v"(z));
  return z;
}

// number of set bits of m in lanes below this lane
__device__ __forceinline__ uint32_t rank_below(uint64_t m) {
  return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32),
                                   __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}

// lanes (of `valid`) whose 8-bit digit equals this lane's: per bit, the
// lane's bit as 0 / -1 (one v_bfe_i32), the ballot of it, and the two mask
// halves ANDed with XNOR(ballot, bit) — 6 VALU per bit (the select form
// `bit ? bal : ~bal` compiled to ~15)
__device__ __forceinline__ uint64_t peers8(uint32_t d, uint64_t valid) {
  uint32_t lo = (uint32_t)valid, hi = (uint32_t)(valid >> 32);
#pragma unroll
  for (int b = 0; b < 8; ++b) {
    const uint32_t sp = (uint32_t)__builtin_amdgcn_sbfe((int)d, b, 1);  // 0 or 0xffffffff
    const uint64_t bal = __ballot(sp != 0u);
    lo &= ~((uint32_t)bal ^ sp);
    hi &= ~((uint32_t)(bal >> 32) ^ sp);
  }
  return ((uint64_t)hi << 32) | lo;
}

// Stable wave-local ranks from LDS instead of ballots (peers8 costs ~85 VALU
// per item and made the CSR / radix scatters VALU-bound): for item k every
// valid lane ORs its lane bit into its half-wave's 32-bit half of its
// digit's 64-bit word of this wave's pmask row (ds_or_b32: OR commutes, the
// lanes' order inside the instruction does not matter), reads the whole word
// back (= its peers), reads the digit's
// running count run[d], and the group writes count + popcount back and
// clears the word.  One wave's LDS instructions execute in issue order, so
// each read sees all of item k's ORs and none of item k + 1's.  Relaxed
// wavefront-scope atomics keep the accesses as ds_ instructions in program
// order (volatile ones became FLAT accesses, not ordered against ds_or).
// lp[k] = the item's rank among the wave's earlier items of its digit;
// run[d] ends as the wave's count of digit d.  pmask (RADIX words) must be
// zero on entry and is zero on exit.
template <int IPT>
__device__ __forceinline__ void wave_ranks_lds(const uint32_t (&dig)[IPT], const bool (&ok)[IPT],
                                               uint32_t *run, uint64_t *pmask,
                                               uint32_t (&lp)[IPT]) {
#pragma unroll
  for (int k = 0; k < IPT; ++k) {
    uint32_t l = 0;
    if (ok[k]) {
      const uint32_t d = dig[k];
      // a 32-bit peer word per half-wave: 4-byte ORs and clears (half the
      // LDS bytes of one 64-bit word per wave; csr_slots 91 -> 86 us at
      // 64M, same-box A/B/A/B, profiles/r5/r5a)
      uint32_t *pw = (uint32_t *)&pmask[d];
      const uint32_t h = lane_id() >> 5;
      __hip_atomic_fetch_or(pw + h, 1u << (lane_id() & 31u), __ATOMIC_RELAXED,
                            __HIP_MEMORY_SCOPE_WAVEFRONT);
      const uint64_t m = __hip_atomic_load(&pmask[d], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
      const uint32_t base = __hip_atomic_load(&run[d], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
      __hip_atomic_store(&run[d], base + (uint32_t)__popcll(m), __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_WAVEFRONT);
      __hip_atomic_store(pw + h, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
      l = base + rank_below(m);
    }
    lp[k] = l;
  }
}

// bin = searchsorted(edges, x, 'left') - 1, x == e[0] -> 0, then
// x == e[nb] -> nb-1, invalid (out of range) -> nb (bins.py:368-379).
// Branchless lower bound over the nb+1 edges: the trip count depends on nb
// only (uniform), so a wave's searches never diverge.  "e[k] < v" is
// monotone in k for sorted edges (a NaN edge, sorted last by numpy, compares
// false like +inf), so this is the first k with !(e[k] < v) exactly as the
// classic bisection finds it.
// NaN x: numpy orders NaN after every number and equal to a NaN edge, so
// searchsorted returns the first NaN edge (nb + 1 when there is none, then
// the particle is dropped): with NaN edges — equaln over x holding NaN and
// no window, bins.py:734-744 — NaN particles land in the bin below the first
// NaN edge, as np.digitize(right=True) puts them (checked against the
// reference's _assign_particles).
template <class E>
__device__ __forceinline__ uint32_t bin_of(double v, E e, int nb) {
  int base = 0, len = nb + 1;
  while (len > 1) {
    const int half = len >> 1;
    base = (e[base + half] < v) ? base + half : base;
    len -= half;
  }
  const int lo = base + (e[base] < v ? 1 : 0);  // first k with e[k] >= v
  int b = lo - 1;
  if (v == e[0]) b = 0;
  if (v == e[nb]) b = nb - 1;
  if (v != v) {  // rare: first NaN edge (NaN edges are the tail of the sorted edges)
    int j = nb + 1;
    if (e[nb] != e[nb]) {
      int l = 0, h = nb;  // first k with e[k] NaN, e[nb] is
      while (l < h) {
        const int m = (l + h) >> 1;
        if (e[m] != e[m]) h = m; else l = m + 1;
      }
      j = l;
    }
    b = j - 1;
  }
  return (b < 0 || b >= nb) ? (uint32_t)nb : (uint32_t)b;
}

// exclusive scan of one u32 per thread over the block
__device__ inline uint32_t block_excl_scan(uint32_t v, uint32_t *lds_wave, uint32_t *total) {
  const uint32_t lane = lane_id();
  const int w = threadIdx.x >> 6;
  uint32_t x = v;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    uint32_t y = __shfl_up(x, o, 64);
    if (lane >= (uint32_t)o) x += y;
  }
  if (lane == 63) lds_wave[w] = x;
  __syncthreads();
  uint32_t off = 0, tot = 0;
#pragma unroll
  for (int k = 0; k < NWAVE; ++k) {
    uint32_t s = lds_wave[k];
    off += (k < w) ? s : 0u;
    tot += s;
  }
  __syncthreads();
  if (total) *total = tot;
  return off + x - v;
}

namespace {

// per-tile sums of `in` (len elements)
__global__ void __launch_bounds__(TPB) scan_tile_sums(const uint32_t *__restrict__ in, int64_t len,
                                                      uint32_t *__restrict__ sums) {
  __shared__ uint32_t wsum[NWAVE];
  int64_t base = (int64_t)blockIdx.x * TILE + (int64_t)threadIdx.x * IPT;
  uint32_t s = 0;
#pragma unroll
  for (int k = 0; k < IPT; ++k) s += (base + k < len) ? in[base + k] : 0u;
  uint32_t tot;
  block_excl_scan(s, wsum, &tot);
  if (threadIdx.x == 0) sums[blockIdx.x] = tot;
}

// exclusive scan of `in` into `out` (in place allowed), adding tile_off[tile]
__global__ void __launch_bounds__(TPB) scan_tiles(const uint32_t *in, int64_t len,
                                                  const uint32_t *__restrict__ tile_off,
                                                  uint32_t *out) {
  __shared__ uint32_t wsum[NWAVE];
  int64_t base = (int64_t)blockIdx.x * TILE + (int64_t)threadIdx.x * IPT;
  uint32_t v[IPT];
  uint32_t s = 0;
#pragma unroll
  for (int k = 0; k < IPT; ++k) {
    v[k] = (base + k < len) ? in[base + k] : 0u;
    s += v[k];
  }
  uint32_t run = block_excl_scan(s, wsum, nullptr) + (tile_off ? tile_off[blockIdx.x] : 0u);
#pragma unroll
  for (int k = 0; k < IPT; ++k) {
    if (base + k < len) out[base + k] = run;
    run += v[k];
  }
}

// Single-pass exclusive scan in place (decoupled look-back).  Status word of
// a tile: epoch (30 bits) | flag (2: 1 = tile sum, 2 = inclusive prefix) |
// value (32); words of an earlier call carry another epoch and read as "not
// ready", so the status array is zeroed only when it is (re)allocated.  The
// look-back is wave 0's: lane l inspects tile (hi - l).
// Tile order: with ticket = 1 tiles are claimed in dispatch order by a
// ticket (one same-address atomic per block, issued before the block's
// loads — at 1184 tiles, the 256M profile's [bin][tile] table, they
// serialised into most of the kernel's time), and the block drawing the last
// ticket re-arms the counter.  With ticket = 0 (the host's choice when the
// whole grid fits the device at once) tile = workgroup id.  Progress then
// rests on each XCD dispatching its workgroups in id order: a running tile's
// predecessors on its own XCD were dispatched before it, and those on other
// XCDs come before any later id there, so no tile waits for one that our own
// waiting tiles keep from being dispatched; kernels of other streams or
// processes can only delay a predecessor until they release its XCD.
// Watchdog: a look-back still waiting after 2^24 sleeps (~10 s; only a
// foreign kernel holding an XCD that long) gives up and sets ctr[1]; the
// scan's result is then incomplete, and the pipelines that read it check
// that word (scan_watchdog) at their next host read-back and fail loudly.
constexpr uint64_t kScAgg = 1ull << 32, kScPre = 2ull << 32;
__global__ void __launch_bounds__(TPB)
    scan_onepass(uint32_t *a, int64_t len, uint64_t *__restrict__ status,
                 unsigned long long *__restrict__ ctr, uint32_t epoch, int ticket) {
  __shared__ uint32_t wsum[NWAVE];
  __shared__ uint32_t s_tile, s_excl;
  uint32_t tile = blockIdx.x;
  if (ticket) {
    if (threadIdx.x == 0) {
      const uint32_t t = (uint32_t)atomicAdd(&ctr[0], 1ull);
      if (t == gridDim.x - 1) atomicExch(&ctr[0], 0ull);  // every ticket is out
      s_tile = t;
    }
    __syncthreads();
    tile = s_tile;
  }
  const int64_t base = (int64_t)tile * TILE + (int64_t)threadIdx.x * IPT;
  uint32_t v[IPT];
  uint32_t sum = 0;
  const bool full = base + IPT <= len && (((uintptr_t)a & 15u) == 0);  // four 16-B loads
  if (full) {
#pragma unroll
    for (int k = 0; k < IPT / 4; ++k) {
      const uint4 q = ((const uint4 *)(a + base))[k];
      v[4 * k] = q.x;
      v[4 * k + 1] = q.y;
      v[4 * k + 2] = q.z;
      v[4 * k + 3] = q.w;
    }
  } else {
#pragma unroll
    for (int k = 0; k < IPT; ++k) v[k] = (base + k < len) ? a[base + k] : 0u;
  }
#pragma unroll
  for (int k = 0; k < IPT; ++k) sum += v[k];
  uint32_t tot;
  const uint32_t in_tile = block_excl_scan(sum, wsum, &tot);
  const uint64_t tag = (uint64_t)epoch << 34;
  if (threadIdx.x < 64) {
    const uint32_t lane = threadIdx.x;
    if (lane == 0)
      __hip_atomic_store(&status[tile], tag | (tile == 0 ? kScPre : kScAgg) | tot, __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_AGENT);
    uint32_t excl = 0, spins = 0;
    for (int64_t hi = (int64_t)tile - 1; tile != 0 && hi >= 0;) {
      const int64_t q = hi - (int64_t)lane;
      uint64_t st = q >= 0 ? __hip_atomic_load(&status[q], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                           : (tag | kScPre);  // before tile 0: an inclusive prefix of 0
      const bool mine = (st >> 34) == epoch;
      const uint32_t fl = mine ? (uint32_t)(st >> 32) & 3u : 0u;
      const uint64_t pre = __ballot(fl == 2);
      const uint64_t notready = __ballot(fl == 0);
      const uint64_t need = pre ? (((pre & -pre) << 1) - 1) : ~0ull;  // lanes up to the nearest prefix
      if (notready & need) {
        if (++spins > (1u << 24)) {  // watchdog (see above): ctr[1], checked by the caller
          if (lane == 0) atomicOr(&ctr[1], 1ull);
          break;
        }
        __builtin_amdgcn_s_sleep(1);
        continue;
      }
      uint32_t val = ((need >> lane) & 1ull) ? (uint32_t)st : 0u;
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) val += __shfl_xor(val, o, 64);
      excl += val;
      if (pre) break;
      hi -= 64;
    }
    if (lane == 0) {
      if (tile != 0)
        __hip_atomic_store(&status[tile], tag | kScPre | (uint32_t)(excl + tot), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
      s_excl = excl;
    }
  }
  __syncthreads();
  uint32_t run = s_excl + in_tile;
  uint32_t o[IPT];
#pragma unroll
  for (int k = 0; k < IPT; ++k) {
    o[k] = run;
    run += v[k];
  }
  if (full) {
#pragma unroll
    for (int k = 0; k < IPT / 4; ++k)
      ((uint4 *)(a + base))[k] = make_uint4(o[4 * k], o[4 * k + 1], o[4 * k + 2], o[4 * k + 3]);
  } else {
#pragma unroll
    for (int k = 0; k < IPT; ++k)
      if (base + k < len) a[base + k] = o[k];
  }
}

}  // namespace

template <typename K>
__global__ void __launch_bounds__(TPB) radix_hist(const K *__restrict__ keys, int64_t n, int shift,
                                                  uint32_t *__restrict__ hist, uint32_t ntiles,
                                                  const int64_t *__restrict__ n_dev) {
  __shared__ uint32_t cnt[RADIX];
  if (n_dev) n = *n_dev;  // device-resident length (<= the n the grid was sized for)
  cnt[threadIdx.x] = 0;
  __syncthreads();
  const int64_t base = (int64_t)blockIdx.x * TILE;
  K kv[IPT];  // every load of the tile in flight first (index 0 past n)
#pragma unroll
  for (int k = 0; k < IPT; ++k) {
    const int64_t i = base + k * TPB + threadIdx.x;
    kv[k] = keys[i < n ? i : 0];
  }
#pragma unroll
  for (int k = 0; k < IPT; ++k) {
    const int64_t i = base + k * TPB + threadIdx.x;
    if (i < n) atomicAdd(&cnt[(uint32_t)(kv[k] >> shift) & 255u], 1u);
  }
  __syncthreads();
  hist[(int64_t)threadIdx.x * ntiles + blockIdx.x] = cnt[threadIdx.x];
}

enum ValMode { VAL_NONE = 0, VAL_IOTA = 1, VAL_ARRAY = 2 };

// Stable scatter of one radix pass.  Element order inside a tile is
// (wave, iteration, lane) == index order, so ranks from per-wave running
// counters keep the sort stable.  The tile is first sorted by digit in LDS
// and then written out run by run: consecutive threads store consecutive
// addresses of one digit's output run (a direct scatter would store 64
// lanes into up to 64 different runs).  kout may be null (values only).
template <typename K, int VM>
__global__ void __launch_bounds__(TPB)
    radix_scatter(const K *__restrict__ kin, const int32_t *__restrict__ vin, int64_t n, int shift,
                  const uint32_t *__restrict__ offs, uint32_t ntiles, K *__restrict__ kout,
                  int32_t *__restrict__ vout, const int64_t *__restrict__ n_dev) {
  __shared__ uint32_t run[NWAVE][RADIX];
  if (n_dev) n = *n_dev;  // device-resident length (<= the n the grid was sized for)
  __shared__ uint32_t dstart[RADIX];  // tile-local start of each digit
  __shared__ uint32_t gofs[RADIX];    // global start of each digit's run of this tile
  __shared__ uint32_t wsum[NWAVE];
  __shared__ __attribute__((aligned(16))) K sk[TILE];
  __shared__ int32_t sv[VM == VAL_NONE ? 1 : TILE];
  static_assert(sizeof(K) * TILE >= sizeof(uint64_t) * NWAVE * RADIX, "pmask fits in sk");
  uint64_t *pmask = (uint64_t *)sk;  // phase 1 only: [NWAVE][RADIX] peer words
  const int w = threadIdx.x >> 6;
  const uint32_t lane = lane_id();
  for (int d = threadIdx.x; d < NWAVE * RADIX; d += TPB) {
    (&run[0][0])[d] = 0;
    pmask[d] = 0ull;
  }
  __syncthreads();
  const int64_t tbase = (int64_t)blockIdx.x * TILE;
  const int64_t wbase = tbase + (int64_t)w * (TILE / NWAVE);
  K key[IPT];
  int32_t val[VM == VAL_ARRAY ? IPT : 1];
  uint32_t lp[IPT];  // rank among this wave's earlier elements of the same digit
#pragma unroll
  for (int k = 0; k < IPT; ++k) {  // every load of the tile in flight first
    const int64_t i = wbase + k * 64 + lane;
    key[k] = i < n ? kin[i] : (K)0;
    if (VM == VAL_ARRAY) val[k] = vin[i < n ? i : 0];
  }
  // phase 1: per-wave digit counts; each element keeps its wave-local rank
  // (items in (k, lane) order = index order), so phase 2 needs no ballots.
  // One leader per (k, digit) adds its peer count with a returning LDS
  // atomic; a wave's LDS operations execute in issue order, so the 16
  // atomics go out back to back and each returns the count of that digit
  // in the wave's earlier items (no round trip per k).
  {
    uint32_t dg[IPT];
    bool okk[IPT];
#pragma unroll
    for (int k = 0; k < IPT; ++k) {
      okk[k] = wbase + k * 64 + lane < n;
      dg[k] = (uint32_t)(key[k] >> shift) & 255u;
    }
    wave_ranks_lds<IPT>(dg, okk, &run[w][0], pmask + w * RADIX, lp);
  }
  __syncthreads();
  // tile-local digit starts, per-wave starts inside them, global run starts
  {
    const int d = threadIdx.x;  // TPB == RADIX
    uint32_t tot = 0;
#pragma unroll
    for (int ww = 0; ww < NWAVE; ++ww) tot += run[ww][d];
    const uint32_t st = block_excl_scan(tot, wsum, nullptr);
    dstart[d] = st;
    gofs[d] = offs[(int64_t)d * ntiles + blockIdx.x];
    uint32_t acc = st;
#pragma unroll
    for (int ww = 0; ww < NWAVE; ++ww) {
      uint32_t c = run[ww][d];
      run[ww][d] = acc;
      acc += c;
    }
  }
  __syncthreads();
  // phase 2: tile-local positions -> LDS
#pragma unroll
  for (int k = 0; k < IPT; ++k) {
    const int64_t i = wbase + k * 64 + lane;
    if (i < n) {
      const uint32_t d = (uint32_t)(key[k] >> shift) & 255u;
      const uint32_t pos = run[w][d] + lp[k];
      sk[pos] = key[k];
      if (VM == VAL_IOTA) sv[pos] = (int32_t)i;
      if (VM == VAL_ARRAY) sv[pos] = val[k];
    }
  }
  __syncthreads();
  // phase 3: runs out, coalesced
  const int tn = (int)((n - tbase) < TILE ? (n - tbase) : TILE);
  for (int j = threadIdx.x; j < tn; j += TPB) {
    const K kk = sk[j];
    const uint32_t d = (uint32_t)(kk >> shift) & 255u;
    const uint32_t p = gofs[d] + ((uint32_t)j - dstart[d]);
    if (kout) kout[p] = kk;
    if (VM != VAL_NONE) vout[p] = sv[j];
  }
}

// ------------------------------------------------------------------ host
// A grow-only device allocation owned by one engine object; its blocks come
// from (and go back to) the device's allocation cache (dev_alloc).
struct Buf {
  void *p = nullptr;
  size_t bytes = 0;
  uint32_t epoch = 0;  // scan workspaces: the current call's status tag
  int dev = 0;
  void *get(size_t need) {
    if (need <= bytes) return p;
    release();
    p = dev_alloc(need, &bytes, &dev);
    return p;
  }
  template <typename T> T *as() const { return (T *)p; }
  void release() {
    if (p) dev_release(p, bytes, dev);
    p = nullptr;
    bytes = 0;
  }
};

// Pinned host staging (hipHostMalloc), grown on demand: D2H copies into it
// stay asynchronous, so a batch of readbacks costs one stream sync.
// mapped = true: coherent host memory a kernel stores its (small) results
// into directly (dev = its device address) — no copy on the stream.
struct HostBuf {
  void *p = nullptr, *dev = nullptr;
  size_t bytes = 0;
  bool mapped = false;
  void *get(size_t need) {
    if (need <= bytes) return p;
    if (p) (void)hipHostFree(p);
    p = dev = nullptr;
    bytes = 0;
    size_t want = need < 4096 ? 4096 : need;
    PBX_HIP(hipHostMalloc(&p, want,
                          mapped ? (hipHostMallocMapped | hipHostMallocCoherent) : hipHostMallocDefault));
    if (mapped) {
      // The completion-tag protocols that write here (fused_pack, radial_mono)
      // rely on the mapping being coherent (fine-grained: the device does not
      // cache it, so a store is performed at the fabric once its vmcnt
      // drains, and the tag is the last posted write): check, fail loudly.
      unsigned int fl = 0;
      PBX_HIP(hipHostGetFlags(&fl, p));
      if (!(fl & hipHostMallocCoherent) || !(fl & hipHostMallocMapped)) {
        (void)hipHostFree(p);
        p = nullptr;
        fail(PBX_ERR_RUNTIME, "mapped results buffer is not coherent host memory (flags 0x%x)", fl);
      }
      PBX_HIP(hipHostGetDevicePointer(&dev, p, 0));
    }
    bytes = want;
    return p;
  }
  void release() {
    if (p) (void)hipHostFree(p);
    p = dev = nullptr;
    bytes = 0;
  }
};

static inline uint32_t ntiles_of(int64_t n) { return (uint32_t)((n + TILE - 1) / TILE); }

// The sticky watchdog word of a scan workspace (scan_onepass ctr[1]):
// non-zero once a look-back gave up; cleared by the reader that reports it.
static inline unsigned long long *scan_watchdog(Buf &ws) { return (unsigned long long *)ws.p + 1; }

// Exclusive scan of len u32 in place, any length: one launch (scan_onepass).
// `ws` holds [ticket counter, watchdog][status word per tile]; its host-side
// epoch tags this call's status words.
static inline void scan_u32(Buf &ws, hipStream_t st, uint32_t *a, int64_t len) {
  if (len <= 0) return;
  const int64_t nt = (len + TILE - 1) / TILE;
  if (nt >= ((int64_t)1 << 31)) fail(PBX_ERR_VALUE, "scan too long");
  const size_t need = sizeof(uint64_t) * (size_t)(2 + nt);
  if (ws.bytes < need || ++ws.epoch >= (1u << 30)) {
    if (ws.bytes < need) {
      ws.release();
      ws.get(need + need / 2);
    }
    PBX_HIP(hipMemsetAsync(ws.p, 0, ws.bytes, st));
    ws.epoch = 1;
  }
  uint64_t *w = (uint64_t *)ws.p;
  static const int64_t resident = [] {  // blocks resident at once on this device
    int dev = 0, cus = 0, per = 0;
    PBX_HIP(hipGetDevice(&dev));
    PBX_HIP(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
    PBX_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(
        &per, reinterpret_cast<const void *>(&scan_onepass), TPB, 0));
    return (int64_t)cus * per;
  }();
  // tickets only when the grid is not resident at once (a resident grid
  // waits only for running tiles: tile = workgroup id, no ticket atomic)
  const int ticket = nt > resident ? 1 : 0;
  hipLaunchKernelGGL(scan_onepass, dim3((unsigned)nt), dim3(TPB), 0, st, a, len, w + 2,
                     (unsigned long long *)w, ws.epoch, ticket);
  PBX_HIP(hipGetLastError());
}

// one stable radix pass: kin -> kout (+ values)
template <typename K>
// (prehist: hist_buf already holds this pass's [digit][tile] counts)
static void radix_pass(Buf &hist_buf, Buf &tsum, hipStream_t st, const K *kin, const int32_t *vin,
                       int vm, int64_t n, int shift, K *kout, int32_t *vout, bool prehist = false,
                       const int64_t *n_dev = nullptr) {
  uint32_t nt = ntiles_of(n);
  uint32_t *hist = (uint32_t *)hist_buf.get(sizeof(uint32_t) * (size_t)nt * RADIX);
  if (!prehist)
    hipLaunchKernelGGL(radix_hist<K>, dim3(nt), dim3(TPB), 0, st, kin, n, shift, hist, nt, n_dev);
  scan_u32(tsum, st, hist, (int64_t)nt * RADIX);
  if (vm == VAL_NONE)
    hipLaunchKernelGGL((radix_scatter<K, VAL_NONE>), dim3(nt), dim3(TPB), 0, st, kin, vin, n,
                       shift, hist, nt, kout, vout, n_dev);
  else if (vm == VAL_IOTA)
    hipLaunchKernelGGL((radix_scatter<K, VAL_IOTA>), dim3(nt), dim3(TPB), 0, st, kin, vin, n,
                       shift, hist, nt, kout, vout, n_dev);
  else
    hipLaunchKernelGGL((radix_scatter<K, VAL_ARRAY>), dim3(nt), dim3(TPB), 0, st, kin, vin, n,
                       shift, hist, nt, kout, vout, n_dev);
  PBX_HIP(hipGetLastError());
}

}  // namespace prim
}  // namespace pbx
