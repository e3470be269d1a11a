// profile.hip — radial-profile binning and per-bin reduction on gfx950.
//
// Replaces the numpy hot spots of pynbodyext.profiles (SURVEY.md §8a
// a12-a19):
//   * Sphere & FamilyFilter mask + r = sqrt((x*x+y*y)+z*z) + sub-snapshot
//     (filters/filt.py:42-86, core/calculate/context.py:622-641)  -> select
//   * equaln edges = exact order statistics of the kept x
//     (profiles/bins.py:720-746)                                   -> sort
//   * bin = digitize(x, edges, right=True) - 1 with the extrema fix-ups and
//     stable per-bin index lists (bins.py:346-395)                 -> assign/CSR
//   * per-bin sums behind Mean/Sum/Sum_w/RMS/Dispersion/Abs_*
//     (profiles/proarray.py:272-334, 632-860)                      -> moments
//
// All state of one profile lives in HBM behind an opaque handle; only the
// O(nbins) results and, on request, the CSR travel back to the host.
//
// Building blocks (one tile = 256 threads x 16 items = 4096 elements):
//   * stable LSD radix pass (8-bit digits): per-tile digit histogram,
//     global exclusive scan over [digit][tile], stable scatter whose
//     in-tile ranks come from wave ballots (the 64-lane "peer mask" of
//     equal digits) -> the CSR is exactly numpy's stable argsort grouping.
//   * stream compaction with the same ballot ranks (order preserving).
//   * per-bin sums accumulated with LDS ds_add_f64 per tile, then a
//     fixed-order reduction over tiles.
#include <cstdlib>
#include <cstring>
#include <type_traits>
#include <vector>

#include "prims.h"


namespace pbx {
namespace prof {

using namespace prim;

constexpr int NMOM = 7;          // Σw, Σfw, Σf²w, Σf, Σf², Σ|f|w, Σ|f|
constexpr int MAX_FAM = 16;
constexpr int LDS_EDGES = 4096;  // edges held in LDS up to this many
constexpr int LDS_MOM_BINS = 800;



// ----------------------------------------------------------------- select
struct SelectParams {
  int use_sphere;
  int ndim;  // 3 -> r, 2 -> rxy
  int nfam;  // 0 -> no family filter
  int64_t base;  // first particle of the tiles (the families' span; 0 without families)
  int mass_f32;  // masses are float (else double)
  int tiled;     // lazy + tiled: x of tile t at xo[t * TILE ..], no look-back
  int sphere_origin;  // the Sphere is centred at (0, 0, 0) (and ndim == 3): its test IS r^2 < R^2
  double cx, cy, cz, r2max;
  int64_t fam_lo[MAX_FAM];
  int64_t fam_hi[MAX_FAM];
};

// family membership of particle i (contiguous slices; no slices = all)
__device__ __forceinline__ bool in_family(int64_t i, const SelectParams &p) {
  if (p.nfam == 0) return true;
  bool in = false;
  for (int f = 0; f < p.nfam; ++f) in |= (i >= p.fam_lo[f]) & (i < p.fam_hi[f]);
  return in;
}

// mask and x of one particle from its loaded position (no FMA contraction:
// numpy evaluates these as separate multiplies and adds; sqrt is correctly
// rounded).  float positions (T = float) follow numpy's dtype rules for a
// float32 snapshot: the Sphere distance mixes the float64 centre in, so it
// is evaluated in double on the exactly widened coordinates; r / rxy of the
// float32 array stay float32 arithmetic (its float32 values are stored
// widened, exactly).
template <typename T>
__device__ __forceinline__ bool select_xyz(T px, T py, T pz, const SelectParams &p, double &x) {
#pragma clang fp contract(off)
  if constexpr (std::is_same<T, double>::value) {
    // a Sphere at the origin: dx = x - 0.0 is x exactly (NaN and -0.0
    // included), so ((dx*dx + dy*dy) + dz*dz) is r^2 itself — one sum of
    // squares for both the test and r
    if (p.sphere_origin) {
      const double r2 = (px * px + py * py) + pz * pz;
      x = __builtin_sqrt(r2);
      return r2 < p.r2max;
    }
  }
  bool keep = true;
  if (p.use_sphere) {
    double dx = (double)px - p.cx, dy = (double)py - p.cy, dz = (double)pz - p.cz;
    keep = ((dx * dx + dy * dy) + dz * dz) < p.r2max;
  }
  const T r2 = (p.ndim == 2) ? (px * px + py * py) : ((px * px + py * py) + pz * pz);
  if constexpr (std::is_same<T, float>::value) x = (double)__builtin_sqrtf(r2);
  else x = __builtin_sqrt(r2);
  return keep;
}

__device__ __forceinline__ double load_mass(const void *mass, int64_t i, int f32) {
  return f32 ? (double)((const float *)mass)[i] : ((const double *)mass)[i];
}

// One pass: mask + x of a tile, then the tile's output offset by a
// decoupled look-back over its predecessors' published counts, then the
// order-preserving write of x, weight and original index; also the key
// min / max of the kept x (NaN-aware: NaN keys are the maximum key).
// Tiles are numbered in the order blocks start (atomic ticket), so every
// predecessor a block waits for is already running and publishes its
// count before it looks back itself: the chain always drains.  The status
// words are relaxed device-scope atomics: the counts they carry are the
// only thing another block reads (a release would write back the XCD's
// whole L2 — the tile outputs — per tile).  status[t]
// = flag (bits 62-63: 1 count of tile t, 2 inclusive prefix through t) |
// value; ctrl[0] = ticket, ctrl[1] = watchdog flag (bounded spin).
constexpr int MM_SLOTS = 8;  // key min / max slot pairs of the selection
constexpr uint64_t kStAgg = 1ull << 62, kStPre = 2ull << 62, kStVal = (1ull << 62) - 1;

// BT threads per block, one 4096-element tile each: 256 (16 items per
// lane) on big inputs; 1024 (4 per lane) when there are few tiles, so a
// small input still puts 16 waves on each CU.
// LAZY: no weights / original indices are written; instead one keep word
// per 64 particles (kw, the wave ballots: word j of tile t covers particles
// base + 64 * (64 t + j) ...) and the tile's output offset (toff[t]), from
// which the weights and indices are materialised only when needed
// (sel_materialize) and the assignment reads the masses directly.
template <int BT, bool LAZY, typename T>
__global__ void __launch_bounds__(BT)
    select_onepass(const T *__restrict__ pos, const void *__restrict__ mass, int64_t n,
                   SelectParams p, uint64_t *__restrict__ status, uint32_t *__restrict__ ctrl,
                   double *__restrict__ xo, double *__restrict__ wo, int32_t *__restrict__ io,
                   unsigned long long *__restrict__ minmax, uint64_t *__restrict__ kw,
                   uint32_t *__restrict__ toff, uint16_t *__restrict__ kpre) {
  constexpr int NW = BT / 64, SI = TILE / BT;  // waves, items per lane
  __shared__ uint32_t wcnt[NW];
  __shared__ unsigned long long wmin[NW], wmax[NW];
  __shared__ uint32_t s_tile, s_excl;
  // the ticket (a returning device atomic before any load can be issued)
  // orders the look-back; a tiled selection has none: block = tile
  if (threadIdx.x == 0) s_tile = (LAZY && p.tiled) ? blockIdx.x : atomicAdd(&ctrl[0], 1u);
  __syncthreads();
  const uint32_t tile = s_tile;
  const int w = threadIdx.x >> 6;
  const uint32_t lane = lane_id();
  const int64_t wbase = p.base + (int64_t)tile * TILE + (int64_t)w * (TILE / NW);
  double xv[SI];
  uint32_t keepbits = 0, c = 0;
  unsigned long long kmin = ~0ull, kmax = 0ull;
  // all SI positions in flight at once (particles outside the range or the
  // family slices read particle 0: no branch around the loads, no extra lines)
  T px[SI], py[SI], pz[SI];
  uint32_t inbits = 0;
#pragma unroll
  for (int k = 0; k < SI; ++k) {
    const int64_t i = wbase + k * 64 + lane;
    const bool in = (i < n) && in_family(i, p);
    inbits |= (uint32_t)in << k;
    const T *q = pos + 3 * (in ? i : 0);
    px[k] = q[0];
    py[k] = q[1];
    pz[k] = q[2];
  }
#pragma unroll
  for (int k = 0; k < SI; ++k) {
    bool keep = ((inbits >> k) & 1u) && select_xyz(px[k], py[k], pz[k], p, xv[k]);
    keepbits |= (uint32_t)keep << k;
    c += (uint32_t)__popcll(__ballot(keep));
    if (keep) {
      unsigned long long kk = dkey(xv[k]);
      kmin = kk < kmin ? kk : kmin;
      kmax = kk > kmax ? kk : kmax;
    }
  }
  // the kept particles' weights: loads issued now, consumed after the look-back
  double mv[SI];
  if (!LAZY && wo) {
#pragma unroll
    for (int k = 0; k < SI; ++k) {
      const int64_t i = wbase + k * 64 + lane;
      mv[k] = mass ? load_mass(mass, ((keepbits >> k) & 1u) ? i : 0, p.mass_f32) : 1.0;
    }
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    unsigned long long a = __shfl_xor(kmin, o, 64);
    unsigned long long b = __shfl_xor(kmax, o, 64);
    kmin = a < kmin ? a : kmin;
    kmax = b > kmax ? b : kmax;
  }
  if (lane == 0) {
    wcnt[w] = c;
    wmin[w] = kmin;
    wmax[w] = kmax;
  }
  __syncthreads();
  if (w == 0) {  // wave 0: publish this tile's count, then look back 64 tiles at a time
    uint32_t tot = 0;
    unsigned long long a = wmin[0], b = wmax[0];
    for (int ww = 0; ww < NW; ++ww) {
      tot += wcnt[ww];
      a = wmin[ww] < a ? wmin[ww] : a;
      b = wmax[ww] > b ? wmax[ww] : b;
    }
    if (lane == 0) {
      // complemented min: zero-filled start; MM_SLOTS slot pairs (by tile)
      // so that no single L2 address takes every block's atomics
      unsigned long long *mmq = minmax + 2 * (tile % MM_SLOTS);
      if (a != ~0ull) atomicMax(&mmq[0], ~a);
      if (b != 0ull) atomicMax(&mmq[1], b);
      __hip_atomic_store(&status[tile], (tile == 0 ? kStPre : kStAgg) | (uint64_t)tot,
                         __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    uint64_t excl = 0;
    uint32_t spins = 0;
    // lane l inspects tile (hi - l): lane 0 is the nearest predecessor;
    // tiles before 0 read as an inclusive prefix of 0
    for (int64_t hi = (int64_t)tile - 1; tile != 0 && !p.tiled && hi >= -1;) {
      const int64_t q = hi - (int64_t)lane;
      const uint64_t s = q >= 0 ? __hip_atomic_load(&status[q], __ATOMIC_RELAXED,
                                                    __HIP_MEMORY_SCOPE_AGENT)
                                : kStPre;
      const uint64_t pre = __ballot((s >> 62) == 2);
      const uint64_t notready = __ballot((s >> 62) == 0);
      const uint64_t need = pre ? (((pre & -pre) << 1) - 1) : ~0ull;  // lanes up to the nearest prefix
      if (notready & need) {  // a predecessor is still counting
        if (++spins > (1u << 24)) {
          if (lane == 0) atomicOr(&ctrl[1], 1u);
          break;
        }
        __builtin_amdgcn_s_sleep(1);
        continue;
      }
      uint64_t v = ((need >> lane) & 1ull) ? (s & kStVal) : 0ull;
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
      excl += v;
      if (pre) break;
      hi -= 64;
    }
    if (lane == 0) {
      if (tile != 0 && !p.tiled)
        __hip_atomic_store(&status[tile], kStPre | (excl + tot), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
      s_excl = (uint32_t)excl;
      if (LAZY && !p.tiled) toff[tile] = (uint32_t)excl;
    }
  }
  __syncthreads();
  uint32_t run = s_excl;
  for (int ww = 0; ww < w; ++ww) run += wcnt[ww];
  // tiled: x in particle-slot layout, the kept particle of slot j of tile t
  // at xo[t * TILE + j] (no in-tile compaction: the readers' addresses do
  // not wait for the keep words)
  const bool slots = LAZY && p.tiled;
  if (slots) xo += (int64_t)tile * TILE + (int64_t)w * (TILE / NW);
#pragma unroll
  for (int k = 0; k < SI; ++k) {
    bool keep = (keepbits >> k) & 1u;
    uint64_t b = __ballot(keep);
    if (LAZY && lane == 0) {  // keep word + its in-tile prefix (kept particles before it)
      kw[(int64_t)tile * (TILE / 64) + w * SI + k] = b;
      kpre[(int64_t)tile * (TILE / 64) + w * SI + k] = (uint16_t)(run - s_excl);
    }
    if (keep) {
      int64_t i = wbase + k * 64 + lane;
      uint32_t pos_out = slots ? (uint32_t)(k * 64) + lane : run + rank_below(b);
      xo[pos_out] = xv[k];
      if (!LAZY) {
        if (wo) wo[pos_out] = mv[k];
        io[pos_out] = (int32_t)i;
      }
    }
    run += (uint32_t)__popcll(b);
  }
}

// Positions of a lazy selection's tile (TPB threads, the select layout:
// item (wave w, k, lane) = particle base + 64 (64 t + 16 w + k) + lane):
// the tile's 64 keep words into LDS with the kept count before each word.
__device__ __forceinline__ void sel_tile_words(const uint64_t *__restrict__ kw,
                                               const uint32_t *__restrict__ toff, uint32_t t,
                                               uint64_t *wrd, uint32_t *wpre) {
  if (threadIdx.x < 64) {
    const uint64_t word = kw[(int64_t)t * 64 + threadIdx.x];
    const uint32_t c = (uint32_t)__popcll(word);
    uint32_t x = c;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const uint32_t y = __shfl_up(x, o, 64);
      if (threadIdx.x >= (uint32_t)o) x += y;
    }
    wrd[threadIdx.x] = word;
    wpre[threadIdx.x] = toff[t] + x - c;
  }
}

// Tiled lazy selection (large inputs): the select kernel skips the
// decoupled look-back and writes each tile's kept x into the tile's own
// TILE slots; block 0 of fused_hist0 then turns the tiles' published
// counts into the exclusive tile offsets (toff) and the kept count.
// (At 64M the look-back held every select block until its predecessors'
// prefixes arrived: 309 -> 211 us of select without it.)
constexpr int TS_TPB = 1024;
constexpr int TS_PT = 16;  // tiles per thread per round (one round up to 16384 tiles = 64M slots)
// (a block of TS_TPB threads; returns the total in every thread)
__device__ uint32_t tile_scan_block(const uint64_t *__restrict__ status, uint32_t nt,
                                    uint32_t *__restrict__ toff, uint32_t *wsum) {
  const uint32_t lane = lane_id();
  const int wv = threadIdx.x >> 6;
  uint32_t carry = 0;
  for (uint32_t r0 = 0; r0 < nt; r0 += TS_TPB * TS_PT) {
    // thread t owns tiles r0 + t * TS_PT .. + TS_PT - 1: all loads in flight together
    const uint32_t t0 = r0 + threadIdx.x * TS_PT;
    uint32_t c[TS_PT], tot = 0;
#pragma unroll
    for (int k = 0; k < TS_PT; ++k) c[k] = t0 + k < nt ? (uint32_t)(status[t0 + k] & kStVal) : 0u;
#pragma unroll
    for (int k = 0; k < TS_PT; ++k) tot += c[k];
    uint32_t x = tot;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const uint32_t y = __shfl_up(x, o, 64);
      if (lane >= (uint32_t)o) x += y;
    }
    if (lane == 63) wsum[wv] = x;
    __syncthreads();
    uint32_t ex = carry + x - tot, all = carry;
    for (int k = 0; k < TS_TPB / 64; ++k) {
      if (k < wv) ex += wsum[k];
      all += wsum[k];
    }
#pragma unroll
    for (int k = 0; k < TS_PT; ++k) {
      if (t0 + k < nt) toff[t0 + k] = ex;
      ex += c[k];
    }
    carry = all;
    __syncthreads();
  }
  return carry;
}

// a tiled selection's per-slot values (x, or assign_gather's byte bins)
// compacted to selection order (for the consumers that index by selection
// index): slot 64 j + lane of tile t -> wpre[j] + its rank in word j
template <typename T, typename U>
__global__ void __launch_bounds__(TPB)
    tile_compact(const T *__restrict__ vt, const uint64_t *__restrict__ kw,
                 const uint32_t *__restrict__ toff, U *__restrict__ vc) {
  __shared__ uint64_t wrd[64];
  __shared__ uint32_t wpre[64];
  const uint32_t t = blockIdx.x;
  sel_tile_words(kw, toff, t, wrd, wpre);
  __syncthreads();
  const int w = threadIdx.x >> 6;
  const uint32_t lane = lane_id();
#pragma unroll 4
  for (int k = 0; k < 16; ++k) {
    const int j = w * 16 + k;
    const uint64_t word = wrd[j];
    if ((word >> lane) & 1ull) vc[wpre[j] + rank_below(word)] = (U)vt[(int64_t)t * TILE + 64 * j + lane];
  }
}

// weights and original indices of a lazy selection, materialised on demand
__global__ void __launch_bounds__(TPB)
    sel_materialize(const uint64_t *__restrict__ kw, const uint32_t *__restrict__ toff,
                    int64_t base, const double *__restrict__ mass, double *__restrict__ wo,
                    int32_t *__restrict__ io) {
  __shared__ uint64_t wrd[64];
  __shared__ uint32_t wpre[64];
  const uint32_t t = blockIdx.x;
  sel_tile_words(kw, toff, t, wrd, wpre);
  __syncthreads();
  const int w = threadIdx.x >> 6;
  const uint32_t lane = lane_id();
#pragma unroll 4
  for (int k = 0; k < 16; ++k) {
    const int j = w * 16 + k;
    const uint64_t word = wrd[j];
    if ((word >> lane) & 1ull) {
      const uint32_t pos = wpre[j] + rank_below(word);
      const int64_t i = base + 64 * ((int64_t)t * 64 + j) + lane;
      if (wo) wo[pos] = mass ? mass[i] : 1.0;
      if (io) io[pos] = (int32_t)i;
    }
  }
}

// min / max key of an x array (generic path): grid-stride, block reduce,
// one atomic pair per block
__global__ void __launch_bounds__(TPB) minmax_keys(const double *__restrict__ x, int64_t n,
                                                   unsigned long long *__restrict__ minmax) {
  __shared__ unsigned long long smin[NWAVE], smax[NWAVE];
  unsigned long long kmin = ~0ull, kmax = 0ull;
  for (int64_t i = (int64_t)blockIdx.x * TPB + threadIdx.x; i < n; i += (int64_t)gridDim.x * TPB) {
    unsigned long long k = dkey(x[i]);
    kmin = k < kmin ? k : kmin;
    kmax = k > kmax ? k : kmax;
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    unsigned long long a = __shfl_xor(kmin, o, 64);
    unsigned long long b = __shfl_xor(kmax, o, 64);
    kmin = a < kmin ? a : kmin;
    kmax = b > kmax ? b : kmax;
  }
  const int w = threadIdx.x >> 6;
  if (lane_id() == 0) {
    smin[w] = kmin;
    smax[w] = kmax;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int k = 1; k < NWAVE; ++k) {
      kmin = smin[k] < kmin ? smin[k] : kmin;
      kmax = smax[k] > kmax ? smax[k] : kmax;
    }
    if (kmin != ~0ull) atomicMin(&minmax[0], kmin);
    if (kmax != 0ull) atomicMax(&minmax[1], kmax);
  }
}

__global__ void __launch_bounds__(TPB) make_keys(const double *__restrict__ x, int64_t n,
                                                 uint64_t *__restrict__ keys) {
  for (int64_t i = (int64_t)blockIdx.x * TPB + threadIdx.x; i < n; i += (int64_t)gridDim.x * TPB)
    keys[i] = dkey(x[i]);
}

// In a sorted key array: out[0] = first key >= a, out[1] = first key > b,
// out[2] = first NaN key (lanes 0..2 each do one binary search).
__global__ void count_bounds(const uint64_t *__restrict__ keys, int64_t n, uint64_t a, uint64_t b,
                             int64_t *__restrict__ out) {
  const int t = threadIdx.x;
  if (blockIdx.x != 0 || t > 2) return;
  const uint64_t probe = (t == 0) ? a : (t == 1 ? b : ~0ull);
  const bool strict = (t == 1);  // first key > probe, else first key >= probe
  int64_t lo = 0, hi = n;
  while (lo < hi) {
    int64_t mid = (lo + hi) >> 1;
    bool left = strict ? (keys[mid] <= probe) : (keys[mid] < probe);
    if (left) lo = mid + 1; else hi = mid;
  }
  out[t] = lo;
}

__global__ void gather_keys(const uint64_t *__restrict__ keys, const int64_t *__restrict__ ranks,
                            int64_t m, double *__restrict__ out) {
  int64_t t = (int64_t)blockIdx.x * TPB + threadIdx.x;
  if (t < m) out[t] = dkey_inv(keys[ranks[t]]);
}

// ------------------------------------------------ equaln by radix select
// The nbins+1 order statistics of the window keys, found together by an MSD
// radix select on the bits of (key - base).  Level 0 takes the top 14 bits
// with a privatised LDS histogram per block (rows reduced afterwards); each
// rank then picks its digit from the prefix sums and narrows its residual
// rank.  Level 1 reads x once more, keeps only keys whose level-0 digit some
// rank chose (an LDS bitmap test, then a search of the sorted active groups)
// and appends them to a compact list; deeper levels work on that list only,
// compacting again as they go.  No sort, no host round trip until the edges
// are done.
#ifndef PBX_MS0_BITS
#define PBX_MS0_BITS 14
#endif
constexpr int MS0_BITS = PBX_MS0_BITS;
constexpr int MS0_DIG = 1 << MS0_BITS;
constexpr int MS0_TPB = 1024;
constexpr int MS_BITS = 12;
constexpr int MS_DIG = 1 << MS_BITS;
constexpr int MS_MAXQ = 1025;  // nbins <= 1024 (more bins: the radix-sort path)
constexpr int MS_MAXL = 8;

struct MsRank {
  uint64_t prefix;  // digits chosen so far
  int64_t rr;       // rank inside the current prefix group
  int32_t group;    // index of the group (sorted unique prefixes)
  int32_t pad;
};

// level 0: one 2^w0-bin histogram per block in LDS, written out as a row
__global__ void __launch_bounds__(MS0_TPB)
    msel_hist0(const double *__restrict__ x, int64_t n, uint64_t ka, uint64_t kb, uint64_t base,
               int s, uint32_t *__restrict__ rows) {
  __shared__ uint32_t lh[MS0_DIG];
  for (int i = threadIdx.x; i < MS0_DIG; i += MS0_TPB) lh[i] = 0;
  __syncthreads();
  // window keys satisfy base <= k <= base + span < base + 2^B, so the digit
  // (k - base) >> s is below 2^w0 without masking
  constexpr int U = 8;  // loads in flight per thread
  for (int64_t i0 = (int64_t)blockIdx.x * MS0_TPB * U; i0 < n; i0 += (int64_t)gridDim.x * MS0_TPB * U) {
    double v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t i = i0 + u * MS0_TPB + threadIdx.x;
      v[u] = i < n ? x[i] : 0.0;
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t i = i0 + u * MS0_TPB + threadIdx.x;
      const uint64_t k = dkey(v[u]);
      if (i < n && k >= ka && k <= kb) atomicAdd(&lh[(uint32_t)((k - base) >> s)], 1u);
    }
  }
  __syncthreads();
  uint32_t *row = rows + (int64_t)blockIdx.x * MS0_DIG;
  for (int i = threadIdx.x; i < MS0_DIG; i += MS0_TPB) row[i] = lh[i];
}

// column sums of the level-0 rows; blockIdx.y takes every gridDim.y-th row
// (H is zero on entry)
__global__ void __launch_bounds__(TPB)
    msel_reduce0(const uint32_t *__restrict__ rows, int nrows, uint32_t *__restrict__ H) {
  const int d = blockIdx.x * TPB + threadIdx.x;
  uint32_t s = 0;
  for (int r = blockIdx.y; r < nrows; r += gridDim.y) s += rows[(int64_t)r * MS0_DIG + d];
  if (s) atomicAdd(&H[d], s);
}

// H from the level-0 rows: select_tiles' u16 rows (two counts per word)
// when the call kept the hinted geometry (ctl->hint), else fused_hist0's
// u32 rows.  Block = 64 digits (32 words) of H, which it stores whole (no
// atomics, no zeroed H needed).  u16 rows: thread t loads 16 bytes (4 words,
// 8 digits) of rows t / 8, t / 8 + 128, ..., four rows in flight; u32 rows:
// one digit of rows t / 64, t / 64 + 16, ...; the row groups' partial sums
// are added through LDS.  (The u16 sums as 4-byte words, one row in flight
// per thread, inside fused_hist0: 16 us at 64M, load latency bound; as
// atomics from 1024 blocks of 256 threads: 7 us.)  Block 0 also zeroes
// `zero` (the selection's tail words, whose last reader was fused_hist0)
// for the next tiled call.
constexpr int R0_DIG = 64;  // digits per msel_reduce0h block
__global__ void __launch_bounds__(MS0_TPB)
    msel_reduce0h(const uint32_t *__restrict__ rows, int nrows, const uint32_t *__restrict__ rows16,
                  int nrows16, const int32_t *__restrict__ hint, uint32_t *__restrict__ H,
                  uint64_t *__restrict__ zero, int nzero) {
  if (blockIdx.x == 0 && (int)threadIdx.x < nzero) zero[threadIdx.x] = 0ull;
  __shared__ int32_t shint;  // one load per block (not one per wave)
  __shared__ uint32_t part[MS0_TPB * 8];
  if (threadIdx.x == 0) shint = *hint;
  __syncthreads();
  const int d0 = blockIdx.x * R0_DIG;
  if (shint && rows16) {
    constexpr int RG = MS0_TPB / 8, U = 4, NW = MS0_DIG / 2;
    const int c = threadIdx.x & 7, rg = threadIdx.x >> 3;
    uint32_t s[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    const uint32_t *base = rows16 + d0 / 2 + 4 * c;
    for (int r0 = rg; r0 < nrows16; r0 += RG * U) {
      uint4 v[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int r = r0 + u * RG;
        v[u] = r < nrows16 ? *(const uint4 *)(base + (int64_t)r * NW) : make_uint4(0, 0, 0, 0);
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        s[0] += v[u].x & 0xffffu;
        s[1] += v[u].x >> 16;
        s[2] += v[u].y & 0xffffu;
        s[3] += v[u].y >> 16;
        s[4] += v[u].z & 0xffffu;
        s[5] += v[u].z >> 16;
        s[6] += v[u].w & 0xffffu;
        s[7] += v[u].w >> 16;
      }
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) part[rg * R0_DIG + 8 * c + j] = s[j];
    __syncthreads();
    {  // digit t % 64, row groups 8 (t / 64) .. + 7
      const int k = threadIdx.x & 63, p = threadIdx.x >> 6;
      uint32_t a = 0;
#pragma unroll
      for (int j = 0; j < RG / 16; ++j) a += part[(p * (RG / 16) + j) * R0_DIG + k];
      __syncthreads();
      part[threadIdx.x] = a;
    }
  } else {
    constexpr int RG = MS0_TPB / R0_DIG, U = 8;
    const int k = threadIdx.x & 63, rg = threadIdx.x >> 6;
    uint32_t a = 0;
    for (int r0 = rg; r0 < nrows; r0 += RG * U) {
      uint32_t v[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int r = r0 + u * RG;
        v[u] = r < nrows ? rows[(int64_t)r * MS0_DIG + d0 + k] : 0u;
      }
#pragma unroll
      for (int u = 0; u < U; ++u) a += v[u];
    }
    part[threadIdx.x] = a;
  }
  __syncthreads();
  if (threadIdx.x < R0_DIG) {  // 16 partials per digit
    uint32_t a = 0;
#pragma unroll
    for (int p = 0; p < MS0_TPB / 64; ++p) a += part[p * 64 + threadIdx.x];
    H[d0 + threadIdx.x] = a;
  }
}

// levels >= 1: keys whose prefix is an active group add to that group's
// digit row and are kept for the next level (when there is one).  Every
// wave owns a fixed region of the key list (cap keys) and keeps its members
// there, compacted in place from level to level, with its count in
// wcnt[wave]: no shared counter at all (one global counter took ~20k
// same-address atomics and serialised the pass).  Level 1 reads x
// grid-stride; later levels read each wave's own region.
constexpr int MS_U = 8;  // keys per lane per step
constexpr int MS_STEP = TPB * MS_U;

template <bool FROM_X>
__global__ void __launch_bounds__(TPB)
    msel_filter(const double *__restrict__ x, int64_t n, uint64_t ka, uint64_t kb, uint64_t base,
                uint64_t *list, const uint32_t *__restrict__ wcnt_in, int64_t cap, int s, int w,
                const uint64_t *__restrict__ groups, const int32_t *__restrict__ ng_ptr,
                uint32_t *__restrict__ H, int keep, uint32_t *__restrict__ wcnt_out) {
  __shared__ uint64_t gs[FROM_X ? 1 : MS_MAXQ];
  // level 1: group index of every level-0 digit (0xffff: no rank chose it)
  __shared__ uint16_t gidx[FROM_X ? MS0_DIG : 1];
  const int ng = *ng_ptr;
  if (FROM_X) {
    for (int i = threadIdx.x; i < MS0_DIG / 2; i += TPB) ((uint32_t *)gidx)[i] = ~0u;
    __syncthreads();
    for (int i = threadIdx.x; i < ng; i += TPB) gidx[(uint32_t)groups[i]] = (uint16_t)i;
  } else {
    for (int i = threadIdx.x; i < ng; i += TPB) gs[i] = groups[i];
  }
  __syncthreads();
  const uint32_t lane = lane_id();
  const int64_t wave = (int64_t)blockIdx.x * NWAVE + (threadIdx.x >> 6);
  uint64_t *region = list + wave * cap;
  // level 1: x[it + u*TPB + threadIdx.x] for it = blockIdx*MS_STEP + k*stride;
  // later: region[it + u*64 + lane] for it = 0, 512, ... < wcnt_in[wave]
  const int64_t beg = FROM_X ? (int64_t)blockIdx.x * MS_STEP : 0;
  const int64_t end = FROM_X ? n : (int64_t)wcnt_in[wave];
  const int64_t stride = FROM_X ? (int64_t)gridDim.x * MS_STEP : 64 * MS_U;
  const uint64_t dmask = (1ull << w) - 1;
  uint32_t wcount = 0;  // wave-uniform
  auto idx_of = [&](int64_t it, int u) -> int64_t {
    return FROM_X ? it + u * TPB + threadIdx.x : it + u * 64 + lane;
  };
  // software-pipelined: the next step's loads are in flight while this
  // step's keys are processed
  auto load_step = [&](int64_t it, uint64_t (&r)[MS_U]) {
#pragma unroll
    for (int u = 0; u < MS_U; ++u) {
      const int64_t i = idx_of(it, u);
      r[u] = i < end ? (FROM_X ? __builtin_bit_cast(uint64_t, x[i]) : region[i]) : 0ull;
    }
  };
  uint64_t nxt[MS_U];
  load_step(beg, nxt);
  for (int64_t it = beg; it < end; it += stride) {
    uint64_t raw[MS_U];
    uint32_t hidx[MS_U];
#pragma unroll
    for (int u = 0; u < MS_U; ++u) raw[u] = nxt[u];
    load_step(it + stride, nxt);
    // phase 1: every key's group (all LDS lookups of the step in flight
    // together); phase 2: ballots, the kept keys, histogram slots
    int ga[MS_U];
    uint64_t offs[MS_U];
#pragma unroll
    for (int u = 0; u < MS_U; ++u) {
      const int64_t i = idx_of(it, u);
      int a = 0xffff;
      uint64_t off = 0;
      if (i < end) {
        if (FROM_X) {  // one LDS lookup: no per-key search on the full pass
          const uint64_t k = dkey(__builtin_bit_cast(double, raw[u]));
          off = k - base;
          if (k >= ka && k <= kb) a = gidx[(uint32_t)(off >> (s + w))];
        } else {  // few keys: search the sorted active groups
          off = raw[u];
          const uint64_t pref = off >> (s + w);
          int lo = 0, b = ng;
          while (lo < b) {
            const int mid = (lo + b) >> 1;
            if (gs[mid] < pref) lo = mid + 1; else b = mid;
          }
          if (lo < ng && gs[lo] == pref) a = lo;
        }
      }
      ga[u] = a;
      offs[u] = off;
    }
    // (in place is safe: keys kept so far sit below every key already read)
#pragma unroll
    for (int u = 0; u < MS_U; ++u) {
      const bool mem = ga[u] != 0xffff;
      hidx[u] = mem ? (uint32_t)ga[u] * MS_DIG + (uint32_t)((offs[u] >> s) & dmask) : ~0u;
      if (keep) {
        const uint64_t bal = __ballot(mem);
        if (mem) region[wcount + rank_below(bal)] = offs[u];
        wcount += (uint32_t)__popcll(bal);
      }
    }
#pragma unroll
    for (int u = 0; u < MS_U; ++u)
      if (hidx[u] != ~0u) atomicAdd(&H[hidx[u]], 1u);
  }
  if (keep && lane == 0) wcnt_out[wave] = wcount;
}

// one block per active group: prefix sums of its DIG-bin histogram (the row
// is zeroed for the next level), then every rank of the group picks its
// digit
template <int DIG>
__global__ void __launch_bounds__(TPB)
    msel_resolve(uint32_t *__restrict__ H, const int32_t *__restrict__ ng_ptr,
                 MsRank *__restrict__ R, int nq, int first, int64_t nbins, int w,
                 int64_t *__restrict__ m_out) {
  constexpr int PT = DIG / TPB;
  const int g = blockIdx.x;
  const int ng = first ? 1 : *ng_ptr;
  if (g >= ng) return;
  __shared__ uint32_t incl[DIG];
  __shared__ uint32_t wsum[NWAVE];
  uint32_t *row = H + (int64_t)g * DIG;
  uint32_t v[PT];
  uint32_t tot = 0;
#pragma unroll
  for (int k = 0; k < PT; ++k) {
    v[k] = row[threadIdx.x * PT + k];
    tot += v[k];
  }
  uint32_t run = block_excl_scan(tot, wsum, nullptr);
#pragma unroll
  for (int k = 0; k < PT; ++k) {
    run += v[k];
    incl[threadIdx.x * PT + k] = run;
    row[threadIdx.x * PT + k] = 0;
  }
  __syncthreads();
  if (first) {  // the window size m and the reference's ranks (bins.py:738-744)
    const int64_t m = (int64_t)incl[DIG - 1];
    if (threadIdx.x == 0) *m_out = m;
    for (int q = threadIdx.x; q < nq; q += TPB) {
      int64_t r = 0;
      if (m >= 2) r = (q == nq - 1) ? m - 1 : (int64_t)((double)(q * m) / (double)nbins);
      R[q].prefix = 0;
      R[q].rr = r;
      R[q].group = 0;
    }
    __syncthreads();
  }
  const int top = (1 << w) - 1;
  for (int q = threadIdx.x; q < nq; q += TPB) {
    if (R[q].group != g) continue;
    const int64_t rr = R[q].rr;
    int a = 0, b = top;  // first digit whose inclusive count exceeds rr
    while (a < b) {
      const int mid = (a + b) >> 1;
      if ((int64_t)incl[mid] <= rr) a = mid + 1; else b = mid;
    }
    R[q].rr = rr - (a ? (int64_t)incl[a - 1] : 0);
    R[q].prefix = (R[q].prefix << w) | (uint64_t)a;
  }
}

// the active groups of the next level.  The ranks are non-decreasing in q,
// so are the values they select and so are the chosen prefixes: the sorted
// unique prefixes are the run starts, numbered by a scan (one block)
__global__ void __launch_bounds__(1024)
    msel_groups(MsRank *__restrict__ R, int nq, uint64_t *__restrict__ groups,
                int32_t *__restrict__ ng_out) {
  __shared__ uint32_t wtot[16];
  const int q0 = 2 * threadIdx.x;  // two ranks per thread covers nq <= 2048
  uint32_t f[2];
  uint64_t p[2];
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const int q = q0 + k;
    p[k] = q < nq ? R[q].prefix : 0;
    f[k] = (q < nq && (q == 0 || R[q - 1].prefix != p[k])) ? 1u : 0u;
  }
  const uint32_t v = f[0] + f[1], lane = lane_id();
  const int wv = threadIdx.x >> 6;
  uint32_t xs = v;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t y = __shfl_up(xs, o, 64);
    if (lane >= (uint32_t)o) xs += y;
  }
  if (lane == 63) wtot[wv] = xs;
  __syncthreads();
  uint32_t off = 0, tot = 0;
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    off += (k < wv) ? wtot[k] : 0u;
    tot += wtot[k];
  }
  uint32_t c = off + xs - v;  // groups started before q0
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const int q = q0 + k;
    if (q >= nq) break;
    if (f[k]) groups[c] = p[k];
    c += f[k];
    R[q].group = (int32_t)c - 1;
  }
  if (threadIdx.x == 0) *ng_out = (int32_t)tot;
}

__global__ void msel_edges(const MsRank *__restrict__ R, int nq, uint64_t base,
                           double *__restrict__ out) {
  const int q = blockIdx.x * TPB + threadIdx.x;
  if (q < nq) out[q] = dkey_inv(base + R[q].prefix);
}

// x[i], x[i + 1] with one 16-byte load when both exist (i even: aligned)
__device__ __forceinline__ void load_pair(const double *__restrict__ x, int64_t i, int64_t n,
                                          double *v) {
  if (i + 1 < n) {
    const double2 q = *(const double2 *)(x + i);
    v[0] = q.x;
    v[1] = q.y;
  } else {
    v[0] = i < n ? x[i] : 0.0;
    v[1] = 0.0;
  }
}

// ------------------------------------- one-sync equaln (select -> sums)
// pbx_profile_radial_equaln: selection, equaln edges, assignment, CSR and
// per-bin sums back to back on the stream with ONE host round trip at the
// end.  Everything the host used to read between the stages (kept count,
// key range, level digits) stays in a device control block, and the kernels
// after the selection take their length from it (their grids are sized for
// the input length).  equaln = level-0 radix select (top <= 14 bits of
// key - base, as msel) + gather of the chosen level-0 buckets' keys into
// per-group segments + one block per group that radix-selects the
// remaining bits of each of its ranks (segment staged in LDS when small).  Same ranks and keys as the
// multi-level msel path, so the same edges.
struct FusedCtl {
  int64_t n;       // kept particles
  int64_t m;       // equaln window size
  uint64_t lo;     // key base of the window
  int32_t s0;      // bits below the level-0 digit
  int32_t w0;      // level-0 digit width
  int32_t err;     // 1: look-back incomplete, 2: empty window / no keys
  int32_t ng;      // chosen level-0 buckets (groups)
  int64_t total;   // keys gathered into the group segments
  uint64_t kmin, kmax;
  int32_t hint;    // 1: the level-0 geometry (lo, s0, w0) is the previous call's, its
                   // histogram was built by select_tiles (no re-read of x)
  int32_t spec;    // SPEC_MATCH: this call's level-0 ranks equal the stored bin table's;
                   // SPEC_HIT: select_tiles binned with that table (no assignment pass)
};
constexpr int32_t SPEC_MATCH = 1, SPEC_HIT = 2, SPEC_NOX = 4, SPEC_EDGE = 8;

// Level-0 digit geometry of a handle's previous tiled call (select_tiles
// counts this call's keys with it while they are still in registers; the
// call keeps it iff every window key fell inside it).  Two slots per
// handle, by call parity: a call reads one and writes the other.
struct SelHint {
  uint64_t lo;
  int32_t s, w;
  int32_t valid;
  int32_t sampled;  // a first call's geometry from a sample of the keys (sample_hint), not kept
};
constexpr int AS_MAXM = 8;
struct FusedStats {
  int nm;
  int f[AS_MAXM];
  int w[AS_MAXM];
  int col[AS_MAXM];
  int op[AS_MAXM];  // MO_* when the slot's monomial has a dedicated form, else MO_GEN
};
struct AgRec {  // a deferred key: key - window base, weight, particle slot, tile | group << 24
  uint64_t off;
  double w;
  uint32_t pos, tg;
};
constexpr uint32_t AG_TBITS = 24;  // tiles < 2^24 (profiles hold < 2^31 particles); groups < 256

// the common monomials in their own (uniform-branch) loops: the generic
// form selects a(f), f, ww per element (~14 VALU), these are 0-2 VALU.
// Each is the value monomial() computes for that slot, bit for bit (the
// products are the same products; x*1.0 is exact)
enum : int { MO_GEN = 0, MO_W = 1, MO_X = 2, MO_XW = 3, MO_XXW = 4, MO_XX = 5, MO_WW = 6 };

// monomial value of column `col` (the expression moments_kernel sums):
// a(f) in {1, f, f*f, |f|} times b in {1, ww}; x*1.0 is exact, so this is
// bit-identical to the per-column expressions
__device__ __forceinline__ double monomial(int col, double f, double ww) {
  const int am = (col == 0) ? 0 : (col == 1 || col == 3) ? 1 : (col == 2 || col == 4) ? 2 : 3;
  const bool wb = (col == 0 || col == 1 || col == 2 || col == 5);
  const double a = am == 0 ? 1.0 : am == 1 ? f : am == 2 ? f * f : __builtin_fabs(f);
  return wb ? a * ww : a;
}

// aq[bk[k]] += monomial of slot (op, col, fq, wq) for the K elements whose bin
// is < nb (LDS atomics)
template <int K>
__device__ __forceinline__ void mom_add(double *aq, int op, int col, int fq, int wq,
                                        const uint32_t *bk, const double *xv, const double *wv,
                                        uint32_t nb) {
#define PBX_MOM_LOOP(EXPR)                                     \
  _Pragma("unroll") for (int k = 0; k < K; ++k) if (bk[k] < nb) \
      atomicAdd(&aq[bk[k]], (EXPR));                           \
  return;
  switch (op) {
    case MO_W: PBX_MOM_LOOP(wv[k])
    case MO_X: PBX_MOM_LOOP(xv[k])
    case MO_XW: PBX_MOM_LOOP(xv[k] * wv[k])
    case MO_XXW: PBX_MOM_LOOP((xv[k] * xv[k]) * wv[k])
    case MO_XX: PBX_MOM_LOOP(xv[k] * xv[k])
    case MO_WW: PBX_MOM_LOOP(wv[k] * wv[k])
    default:
      PBX_MOM_LOOP(monomial(col, fq == 0 ? xv[k] : wv[k], wq == 0 ? xv[k] : wv[k]))
  }
#undef PBX_MOM_LOOP
}

// bin_of(v, e, nb) for a v whose lower bound lies in [qa, qb]
__device__ __forceinline__ uint32_t bin_of_in(double v, const double *e, int nb, int qa, int qb) {
  if (v != v) return bin_of(v, e, nb);  // rare: the first NaN edge
  int l = qa, h = qb;  // first k in [qa, qb) with !(e[k] < v), qb if none
  while (l < h) {
    const int m = (l + h) >> 1;
    if (e[m] < v) l = m + 1;
    else h = m;
  }
  const int lo = l;
  int b = lo - 1;
  if (v == e[0]) b = 0;
  if (v == e[nb]) b = nb - 1;
  return (b < 0 || b >= nb) ? (uint32_t)nb : (uint32_t)b;
}

// Speculative assignment (tiled one-rank calls).  The bin of a key whose
// level-0 digit holds no edge depends only on the digit: bin = #{ranks q
// with digit_q < digit} - 1 (assign_gather's table).  So when this call's
// level-0 digit of every rank q equals the previous full call's (same
// geometry, same nq), that call's digit -> bin table bins this call's keys
// exactly, and select_tiles can bin every key while x is still in registers
// (byte bins, per-bin sums, and the keys of edge-holding digits into a
// deferred list) — the assignment pass that re-reads x and the masses is
// skipped.  fused_resolve compares the digits (SPEC_MATCH) once the level-0
// histogram is known; on a mismatch assign_gather runs as before and stores
// the new table.  The table: written by assign_gather's block 0 (which has
// no tiles of its own), read by the next call's select_tiles and
// fused_resolve (before that call's assign_gather may rewrite it).
struct SpecTab {
  uint64_t lo;             // level-0 geometry the digits are taken in
  int32_t s0, w0;
  int32_t nb, nq, ng, valid;
  uint32_t qd[MS_MAXQ];    // level-0 digit of each rank q
  uint8_t bin[MS0_DIG];    // digit -> bin (nb: outside the edges); SPEC_DEFER: the digit holds edges
  // the edges of the last call with these digits (fix_deferred) and the
  // groups (gdig: assign_gather, gq: fix_deferred), for the edge speculation
  uint32_t gdig[MS_MAXQ];  // the edge-holding digits, ascending
  uint32_t gq[MS_MAXQ + 1];  // group g's ranks gq[g] .. gq[g + 1]
  double edges[MS_MAXQ];
  int32_t edges_valid;
  int32_t enc;  // 1 (nb <= 128): an edge-holding digit's byte is 128 + its group (255: group
                // >= 127, found by search); 0: SPEC_DEFER for all of them
};
constexpr uint8_t SPEC_DEFER = 0xff;
constexpr int SPEC_MAXB = 254;   // bins (and groups <= nq = nb + 1 < 256) a byte table holds
constexpr int SPEC_MACC = 256;   // per-bin sums (nm * nb doubles) select_tiles keeps in LDS
constexpr int SPEC_LIST = 4;     // deferred-list capacity: 1 / SPEC_LIST of a block's slots
struct SpecArgs {
  const SpecTab *tab;      // null: no speculation (select_tiles<FAM, false>)
  const double *mass;      // f64 masses by particle (null: unit weights)
  uint8_t *bins;           // byte bins by particle slot (assign_gather's bins8)
  uint32_t *th;            // [bin][tile] counts of the CSR pass (deferred keys: fix_deferred adds)
  double *slab;            // per select block: nm * nb sums
  AgRec *rec;              // deferred lists: select block j's at rbase[j]
  uint32_t *rbase, *rn;    // per select block: list start, length
  uint32_t *flag;          // bit 0: a block could not bin (table / hint geometry differ, a
                           // list overflowed): the call takes the assignment pass;
                           // bit 1: the blocks binned and stored no x (SPEC_NOX);
                           // bit 2: edge speculation (every key binned with the table's edges)
  uint32_t *lteq;          // edge speculation: per rank q, window keys of its digit < / == edge q
  FusedStats fs;
  int nb;
  int edge;                // 1: the edge speculation (the host saw the last call's edges repeat)
};

// select_tiles blocks per assign_gather block (tile sub-ranges): 3 x 255
// blocks of 8 waves at <= 80 VGPRs (6 waves per SIMD) are all resident at once
#ifndef PBX_SH_K
#define PBX_SH_K 3
#endif
constexpr int SH_K = PBX_SH_K;
// the full assignment (assign_tiles) runs one workgroup per select block
// (+ block 0, which writes the bin table): its segment offsets come from the
// select blocks' own level-0 rows (fused_resolve)
__host__ __device__ constexpr uint32_t at_blocks(int g0) { return 1u + (uint32_t)SH_K * (uint32_t)(g0 - 1); }


// the inputs x is recomputed from when a speculating selection stored none (xsrc_tiles)
struct XSrc {
  const double *pos;  // the selection's positions (null: x was stored)
  int64_t n_hi;       // particles [sp.base, n_hi) are tiled
  SelectParams sp;
  double *x;          // x by slot
  const uint64_t *kw;
};

// The step's control record from the selection's status words: kept count
// (inclusive prefix of the last tile), key range (min over the slot pairs),
// the equaln window's key base and level-0 digit geometry.  Every block of
// fused_hist0 derives it (a few scalar loads); block 0 publishes it.
struct FusedSetup {
  const uint64_t *stat;
  uint32_t nt;
  int64_t n_in;
  uint64_t ka, kb;
  int empty_bounds;
  int tiled;  // tiled selection: x of tile t at x[t * TILE ..], its count in stat[t]
  uint32_t *toff;  // tiled: the tile offsets block 0 writes
  uint32_t *zero;  // words block 0 zeroes for later kernels (fused_resolve's per-block counts)
  int nzero;
  int dist;  // one rank of several: the key range (mm slots) is global, no keys here is no error
  const uint64_t *kw;  // tiled: the selection's keep words (slot i holds a key iff its bit is set)
  const SelHint *hint;   // tiled, one rank: the geometry select_tiles counted with (or null)
  const uint32_t *hflag; // select_tiles: a window key fell outside the hint (or null)
  SelHint *hint_out;     // fused_hist0 block 0: this call's own geometry, for the next call
  const uint32_t *btot;  // tiled: select_tiles' block totals (SH_K (gridDim - 1) blocks)
  const uint32_t *sflag; // tiled, speculating: select_tiles' flags (bit 1: no x stored)
  XSrc xs;               // ... and what x is recomputed from then
};

// Element range of fused_hist0 / fused_gather: the kept x [0, n), or with
// a tiled selection the tiles' particle slots [0, nt * TILE), slot i holding
// a key iff bit i % 64 of keep word i / 64 is set.  One block step covers
// EL_STEP slots = two whole tiles.
constexpr int EL_U = 4;  // 16-byte loads per lane per step (two keys each)
constexpr int64_t EL_STEP = (int64_t)MS0_TPB * 2 * EL_U;
static_assert(EL_STEP == 2 * TILE, "a step is two tiles");
struct ElRange {
  const uint64_t *kw;  // tiled: the selection's keep words
  uint32_t nt;
  int64_t n;    // kept keys
  int64_t lim;  // slots
};
__device__ __forceinline__ ElRange el_range(const uint64_t *kw, uint32_t nt, int64_t n) {
  return kw ? ElRange{kw, nt, n, (int64_t)nt * TILE} : ElRange{nullptr, 0u, n, n};
}

__device__ FusedCtl fused_ctl(const FusedSetup &f) {
  FusedCtl c{};
  const uint32_t *ctrl = (const uint32_t *)(f.stat + f.nt);
  const unsigned long long *mm = (const unsigned long long *)(f.stat + f.nt + 1);
  if (f.tiled) {  // the kept count comes from fused_hist0's block 0 (tile_scan_block)
    c.n = -1;
    if (ctrl[1]) c.err |= 1;
  } else if (f.n_in > 0) {  // the last tile's inclusive prefix
    const uint64_t last = f.stat[f.nt - 1];
    if (ctrl[1] || (last >> 62) != 2) c.err |= 1;
    c.n = (int64_t)(last & kStVal);
  }
  c.kmin = ~0ull;
  c.kmax = 0ull;
  for (int q = 0; q < MM_SLOTS; ++q) {
    c.kmin = ~mm[2 * q] < c.kmin ? ~mm[2 * q] : c.kmin;
    c.kmax = mm[2 * q + 1] > c.kmax ? mm[2 * q + 1] : c.kmax;
  }
  const uint64_t lo = f.ka > c.kmin ? f.ka : c.kmin;
  const uint64_t hi = f.kb < c.kmax ? f.kb : c.kmax;
  if ((c.n == 0 && !f.dist) || f.empty_bounds || lo > hi) {
    c.err |= 2;
    c.w0 = 1;
  } else {
    const uint64_t span = hi - lo;
    const int B = span ? 64 - __builtin_clzll(span) : 1;
    c.w0 = B < MS0_BITS ? B : MS0_BITS;
    c.s0 = B - c.w0;
    c.lo = lo;
  }
  return c;
}

// fused_ctl, then the hinted geometry when select_tiles counted every
// window key with it (the digits of any base <= the window's lowest key and
// any width covering its highest key rank the keys the same: same edges)
__device__ FusedCtl fused_ctl_eff(const FusedSetup &f) {
  FusedCtl c = fused_ctl(f);
  if (f.hint && !f.dist && !(c.err & 2)) {
    const SelHint h = *f.hint;
    if (h.valid && !*f.hflag) {
      c.lo = h.lo;
      c.s0 = h.s;
      c.w0 = h.w;
      c.hint = 1;
    }
  }
  return c;
}

// Tiled lazy selection (large inputs), persistent: block j takes the
// j % SH_K-th part of the tile range assign_gather block 1 + j / SH_K walks
// (tile_range); each of its 8 waves streams its 512-particle slice of every
// tile with no block barrier in the loop: mask + x (8 particles per lane,
// all loads in flight), x stored in particle-slot layout, the keep words,
// each word's prefix INSIDE ITS WAVE SLICE (kpre) and the slice's count
// (wcnt[t][w]).  At the end one barrier: the block's tiles' offsets
// relative to the block (toff; fused_hist0 adds the block's base from the
// block totals btot), the key range.
// With a valid hint (the previous tiled call's level-0 geometry) the block
// also counts every window key's level-0 digit in LDS (two u16 counts per
// word: at most SH_TMAX tiles = 61440 keys per block) while x is still in
// registers, and stores its row — fused_hist0 then need not read x again; a
// window key outside the hint's range sets *hflag and the call falls back.
constexpr int SH_BT = 512;
constexpr int SH_NW = SH_BT / 64;  // wave slices per tile
constexpr uint32_t SH_TMAX = 15;   // tiles per block for the u16 digit counts
constexpr uint32_t SH_MAXT = 64;   // tiles per block for the block-local offsets (LDS)
constexpr uint32_t SH_RSUB_MAX = 8;  // u16 count rows per block (flushed every SH_TMAX tiles)
// FAM: several family slices (membership tested per particle); else every
// particle of the span [base, n) is a member (no family, or one slice: the
// span is that slice) and the 16 slice bounds stay out of the registers.
// SPEC: the speculative assignment (SpecArgs above) — with a stored table
// whose geometry is the hint's, every kept key is also binned here: byte bin
// by slot, per-bin sums in LDS (one slab row per block), the keys of
// edge-holding digits into the block's deferred list.
template <bool FAM, bool SPEC>
__global__ void __launch_bounds__(SH_BT) __attribute__((amdgpu_waves_per_eu(4)))
    select_tiles(const double *__restrict__ pos, int64_t n, SelectParams p, uint32_t nt,
                 uint32_t G0, double *__restrict__ xo, uint64_t *__restrict__ kw,
                 uint16_t *__restrict__ kpre, uint32_t *__restrict__ wcnt,
                 uint32_t *__restrict__ toff, uint32_t *__restrict__ btot,
                 unsigned long long *__restrict__ minmax, const SelHint *__restrict__ hint,
                 uint64_t ka, uint64_t kb, uint32_t *__restrict__ rows16, uint32_t rsub,
                 uint32_t *__restrict__ hflag, SpecArgs sa) {
  constexpr int SI = TILE / SH_BT;
  __shared__ uint32_t lh[MS0_DIG / 2];
  __shared__ uint32_t tcnt[SH_MAXT][SH_NW];
  __shared__ unsigned long long wmin[SH_NW], wmax[SH_NW];
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint32_t lane = lane_id();
  // this block's tiles: part j % SH_K of assign block 1 + j / SH_K's range
  const uint32_t ab = blockIdx.x / SH_K, sub = blockIdx.x % SH_K;
  const uint32_t ta0 = (uint32_t)((uint64_t)nt * ab / (G0 - 1));
  const uint32_t tb0 = (uint32_t)((uint64_t)nt * (ab + 1) / (G0 - 1));
  const uint32_t ta = ta0 + (uint32_t)((uint64_t)(tb0 - ta0) * sub / SH_K);
  const uint32_t tb = ta0 + (uint32_t)((uint64_t)(tb0 - ta0) * (sub + 1) / SH_K);
  // the hint: one load per block, through LDS (not one per wave from all
  // the grid's waves at once: the same-line hot spot fused_hist0 had)
  __shared__ SelHint shh;
  __shared__ uint8_t sdt[SPEC ? MS0_DIG : 1];      // the table's digit -> bin
  __shared__ double sacc[SPEC ? SPEC_MACC + 1 : 1];  // per-bin sums (+ a trash slot)
  // per-(tile, bin) counts of the current SH_TMAX tiles (flushed with the u16 rows)
  __shared__ uint32_t tcs[SPEC ? SH_TMAX * ((SPEC_MAXB + 2) | 1) : 1];  // (+ a trash slot)
  __shared__ uint32_t sdk;                         // deferred keys listed
  __shared__ int s_spec, s_edge, s_enc;
  // edge speculation: the table's edges (and their keys), groups, and per
  // rank the window keys of its digit below / equal to its edge
  __shared__ double sedg[SPEC ? SPEC_MAXB + 1 : 1];
  __shared__ uint64_t sek[SPEC ? SPEC_MAXB + 1 : 1];
  __shared__ uint32_t sgq[SPEC ? SPEC_MAXB + 2 : 1], sgd[SPEC ? SPEC_MAXB + 1 : 1];
  __shared__ uint32_t slt[SPEC ? 2 * (SPEC_MAXB + 1) : 1];
  if (threadIdx.x == 0) {
    SelHint t{};
    if (hint) t = *hint;
    shh = t;
    if (SPEC) {
      const SpecTab *tb = sa.tab;
      s_spec = tb->valid && t.valid && tb->lo == t.lo && tb->s0 == t.s && tb->w0 == t.w &&
               tb->nb == sa.nb;
      s_edge = s_spec && sa.edge && tb->edges_valid;
      s_enc = tb->enc;
      sdk = 0;
    }
  }
  __syncthreads();
  const SelHint h = shh;
  // rsub rows per block: the u16 counts are flushed to the next row every
  // SH_TMAX tiles (families above ~47M particles)
  const bool hv = h.valid && rows16 && tb - ta <= SH_TMAX * rsub;
  const uint64_t hlo = h.lo;
  const int hsh = h.s;
  // highest key the hint's digits cover: lo + 2^(s + w) - 1 (saturating)
  const int hb = h.s + h.w;
  const uint64_t hspan = hb >= 64 ? ~0ull : ((1ull << hb) - 1);
  const uint64_t hhi = hlo + hspan < hlo ? ~0ull : hlo + hspan;
  const bool spec = SPEC && hv && s_spec;
  const int nb = SPEC ? sa.nb : 0;
  const int macc = SPEC ? sa.fs.nm * nb : 0;
  uint32_t mfl = 0;  // SPEC: per monomial q, factors x, x, w, w present (bits 4q ..)
  int mmode = 0;     // SPEC: 1 = {Σw, Σx·w}, 2 = {Σw} (dedicated adds), else the factor loop
  if constexpr (SPEC) {
#pragma unroll
    for (int q = 0; q < AS_MAXM; ++q) {  // unrolled: fs's fields are kernel-argument scalars
      if (q >= sa.fs.nm) break;
      const int op = sa.fs.op[q];
      const uint32_t f = ((op == MO_X || op == MO_XW || op == MO_XXW || op == MO_XX) ? 1u : 0u) |
                         ((op == MO_XXW || op == MO_XX) ? 2u : 0u) |
                         ((op == MO_W || op == MO_XW || op == MO_XXW || op == MO_WW) ? 4u : 0u) |
                         ((op == MO_WW) ? 8u : 0u);
      mfl |= f << (4 * q);
    }
    mmode = (sa.fs.nm == 2 && mfl == 0x54u) ? 1 : (sa.fs.nm == 1 && mfl == 0x4u) ? 2 : 0;
  }
  const int nrs = (nb + 2) | 1;  // bins 0 .. nb, the trash slot nb + 1; odd
  // the block's deferred list: 1 / SPEC_LIST of its slots (an overflow fails the speculation)
  const uint64_t lbase = (uint64_t)ta * TILE / SPEC_LIST;
  const uint32_t lcap = (uint32_t)((uint64_t)(tb - ta) * TILE / SPEC_LIST);
  if (SPEC) {
    if (spec) {
      if (blockIdx.x == 0 && threadIdx.x == 0) atomicOr(sa.flag, s_edge ? 6u : 2u);  // NOX, EDGE
      if (s_edge) {
        const int nq = nb + 1, ng = sa.tab->ng;
        for (int q = threadIdx.x; q < nq; q += SH_BT) {
          const double e = sa.tab->edges[q];
          sedg[q] = e;
          sek[q] = dkey(e);
          slt[2 * q] = slt[2 * q + 1] = 0;
        }
        for (int g = threadIdx.x; g <= ng; g += SH_BT) {
          sgq[g] = sa.tab->gq[g];
          if (g < ng) sgd[g] = sa.tab->gdig[g];
        }
      }
      const uint4 *src = (const uint4 *)sa.tab->bin;
      for (int i = threadIdx.x; i < MS0_DIG / 16; i += SH_BT) ((uint4 *)sdt)[i] = src[i];
      for (int i = threadIdx.x; i < macc; i += SH_BT) sacc[i] = 0.0;
      for (int i = threadIdx.x; i < SH_TMAX * nrs; i += SH_BT) tcs[i] = 0;
    } else if (threadIdx.x == 0) {
      atomicOr(sa.flag, 1u);
    }
  }
  if (hv) {
    for (int i = threadIdx.x; i < MS0_DIG / 2; i += SH_BT) lh[i] = 0;
    __syncthreads();
  }
  unsigned long long kmin = ~0ull, kmax = 0ull;
  bool oob = false;
  // a wave's slice of a tile in two halves of SH_HALF particles per lane,
  // software-pipelined: the next half's positions are loaded while this
  // half is selected (ping-pong registers; every load unconditional — past
  // the range the last tile again — so the vmcnt waits stay exact).  (All
  // blocks start together: without the overlap each wave's loads and math
  // alternated in lockstep with its neighbours', 283 us at 64M.)
  constexpr int SH_HALF = SI / 2;
  struct Half {
    double x[SH_HALF], y[SH_HALF], z[SH_HALF];
    double m[SPEC ? SH_HALF : 1];  // SPEC: the masses (loaded with the positions)
    uint32_t in;
  };
  auto ld = [&](uint32_t tile, int h, Half &H, auto sp) {  // sp: the speculating loop (masses)
    const int64_t wbase = p.base + (int64_t)tile * TILE + (int64_t)w * (TILE / SH_NW) + h * SH_HALF * 64;
    H.in = 0;
#pragma unroll
    for (int k = 0; k < SH_HALF; ++k) {
      const int64_t i = wbase + k * 64 + lane;
      const bool in = (i < n) && (!FAM || in_family(i, p));
      H.in |= (uint32_t)in << k;
      const double *q = pos + 3 * (in ? i : 0);
      H.x[k] = q[0];
      H.y[k] = q[1];
      H.z[k] = q[2];
      if constexpr (SPEC && decltype(sp)::value) H.m[k] = sa.mass ? sa.mass[in ? i : 0] : 1.0;
    }
  };
  uint32_t run = 0;
  // SPEC, speculating: the selection of a half (as sel below, without the x
  // stores), then the bins of its kept keys — the table lookups of the
  // half's four keys issued together, one LDS wait — then their bytes,
  // per-tile counts, sums and deferred list entries
  auto sel_spec = [&](uint32_t tile, int h, const Half &H) {
    if constexpr (SPEC) {
      const int64_t wj = (int64_t)tile * (TILE / 64) + w * SI + h * SH_HALF;
      const uint32_t slot0 = tile * (uint32_t)TILE + (uint32_t)w * (TILE / SH_NW) + h * SH_HALF * 64 + lane;
      double xk[SH_HALF];
      uint64_t kk[SH_HALF];
      uint32_t kb4 = 0, in4 = 0;  // kept / kept and in the hinted window, per key
#pragma unroll
      for (int k = 0; k < SH_HALF; ++k) {
        double xv = 0.0;
        const bool keep = ((H.in >> k) & 1u) && select_xyz(H.x[k], H.y[k], H.z[k], p, xv);
        const uint64_t bal = __ballot(keep);
        if (lane == 0) {
          kw[wj + k] = bal;
          kpre[wj + k] = (uint16_t)run;
        }
        run += (uint32_t)__popcll(bal);
        xk[k] = xv;
        kk[k] = dkey(xv);
        kb4 |= (uint32_t)keep << k;
        if (keep) {
          kmin = kk[k] < kmin ? kk[k] : kmin;
          kmax = kk[k] > kmax ? kk[k] : kmax;
          if (kk[k] >= ka && kk[k] <= kb) {
            if (kk[k] >= hlo && kk[k] <= hhi) {
              const uint32_t d = (uint32_t)((kk[k] - hlo) >> hsh);
              atomicAdd(&lh[d >> 1], 1u << (16 * (d & 1)));
              in4 |= 1u << k;
            } else {
              oob = true;
            }
          }
        }
      }
      uint32_t c8[SH_HALF];
#pragma unroll
      for (int k = 0; k < SH_HALF; ++k)
        c8[k] = ((in4 >> k) & 1u) ? (uint32_t)sdt[(uint32_t)((kk[k] - hlo) >> hsh)] : (uint32_t)nb;
      uint32_t *trow = tcs + ((tile - ta) % SH_TMAX) * nrs;
      const uint32_t gmin = s_enc ? 128u : (uint32_t)SPEC_DEFER;  // bytes >= gmin: edge-holding digit
      // a kept key's common effects — its byte, its tile's count of its bin,
      // its bin's sums; a lane without one counts in the trash slots with
      // the same instructions (no branch per key: the divergent regions,
      // their exec-mask bookkeeping and the code copies they need had made
      // this the kernel's largest cost after the loads)
      auto common = [&](bool on, bool every, uint32_t code, double xv, double mv, uint32_t slot) {
        // every: the byte of every lane's slot (the readers take the kept
        // slots' only; a deferred key's is stored later by fix_deferred)
        if (every || on) sa.bins[slot] = (uint8_t)code;
        atomicAdd(&trow[on ? code : (uint32_t)nb + 1u], 1u);
        const bool sum = on && code < (uint32_t)nb;
        if (mmode == 1) {  // Σw, Σx·w (mass / mean profiles)
          atomicAdd(&sacc[sum ? code : (uint32_t)SPEC_MACC], mv);
          atomicAdd(&sacc[sum ? (uint32_t)nb + code : (uint32_t)SPEC_MACC], xv * mv);
        } else if (mmode == 2) {  // Σw
          atomicAdd(&sacc[sum ? code : (uint32_t)SPEC_MACC], mv);
        } else if (macc) {
          // the dedicated monomials only (the host checks): (a1 a2)(b1 b2)
          // with a = x or 1, b = w or 1 — mom_add's products (x * 1.0 is
          // exact); monomial q's factors are bits 4q .. 4q + 3 of mfl
#pragma unroll 1
          for (int q = 0; q < sa.fs.nm; ++q) {
            const uint32_t f = mfl >> (4 * q);
            const double a = ((f & 1u) ? xv : 1.0) * ((f & 2u) ? xv : 1.0);
            const double b = ((f & 4u) ? mv : 1.0) * ((f & 8u) ? mv : 1.0);
            atomicAdd(&sacc[sum ? (uint32_t)q * nb + code : (uint32_t)SPEC_MACC], a * b);
          }
        }
      };
      // rare: kept window keys of an edge-holding digit
      uint32_t rare = 0;
#pragma unroll
      for (int k = 0; k < SH_HALF; ++k) rare |= (((in4 >> k) & 1u) && c8[k] >= gmin) ? 1u << k : 0u;
#pragma unroll
      for (int k = 0; k < SH_HALF; ++k)  // (kept outside the window: c8 = nb, the dropped bin)
        common(((kb4 & ~rare) >> k) & 1u, true, c8[k], xk[k], H.m[k], slot0 + 64u * k);
      if (__ballot(rare != 0u)) {  // (wave-uniform, rare) one key per lane and round
        const bool edge = s_edge != 0;
        uint32_t todo = rare;
        while (__ballot(todo != 0u)) {  // at most SH_HALF rounds
          const int k = todo ? __builtin_ctz(todo) : 0;
          double xv = xk[0], mv = H.m[0];
          uint64_t kv = kk[0];
          uint32_t cv = c8[0];
#pragma unroll
          for (int u = 1; u < SH_HALF; ++u) {
            xv = k == u ? xk[u] : xv;
            mv = k == u ? H.m[u] : mv;
            kv = k == u ? kk[u] : kv;
            cv = k == u ? c8[u] : cv;
          }
          const uint32_t slot = slot0 + 64u * (uint32_t)k;
          const bool act = todo != 0u;
          bool def = act;
          if (edge && act) {
            // the bin among its group's edges (the table's), and per edge the
            // keys below / equal to it (the edges are checked against this
            // call's ranks by fused_resolve)
            int g;
            if (cv != SPEC_DEFER) {
              g = (int)cv - 128;  // (the byte carries the group)
            } else {  // search the group by its digit
              const uint32_t dd = (uint32_t)((kv - hlo) >> hsh);
              int lo = 0, hi = sa.tab->ng - 1;
              while (lo < hi) {
                const int mid = (lo + hi) >> 1;
                if (sgd[mid] < dd) lo = mid + 1; else hi = mid;
              }
              g = lo;
            }
            const int qa = (int)sgq[g], qb = (int)sgq[g + 1];
            cv = bin_of_in(xv, sedg, nb, qa, qb);
            for (int q = qa; q < qb; ++q) {
              if (kv < sek[q]) atomicAdd(&slt[2 * q], 1u);
              else if (kv == sek[q]) atomicAdd(&slt[2 * q + 1], 1u);
            }
            def = false;
          }
          if (edge) common(act, false, cv, xv, mv, slot);
          const uint64_t bd = __ballot(def);
          if (bd) {  // keys of edge-holding digits, into the block's list
            uint32_t b0 = 0;
            if (lane == 0) b0 = atomicAdd(&sdk, (uint32_t)__popcll(bd));
            b0 = __shfl(b0, 0, 64);
            if (def) {
              const uint32_t idx = b0 + rank_below(bd);
              // (the group: filled in by assign_gather from the key — a global
              // table lookup here stalled almost every wave step)
              if (idx < lcap) sa.rec[lbase + idx] = AgRec{kv - hlo, mv, slot, tile};
            }
          }
          todo &= todo - 1u;
        }
      }
    }
  };
  auto sel = [&](uint32_t tile, int h, const Half &H) {
    double *xt = xo + (int64_t)tile * TILE + (int64_t)w * (TILE / SH_NW) + h * SH_HALF * 64;
    const int64_t wj = (int64_t)tile * (TILE / 64) + w * SI + h * SH_HALF;
#pragma unroll
    for (int k = 0; k < SH_HALF; ++k) {
      double xv = 0.0;
      const bool keep = ((H.in >> k) & 1u) && select_xyz(H.x[k], H.y[k], H.z[k], p, xv);
      const uint64_t bal = __ballot(keep);
      // (the wave's 8 words stored from lanes 0..7 once per tile instead:
      // 265 vs 268 us at 64M, no gain, round 6 — and one store per half
      // from lane k: csr_slots +19 us; both dropped)
      if (lane == 0) {
        kw[wj + k] = bal;
        kpre[wj + k] = (uint16_t)run;  // kept particles before the word in this wave's slice
      }
      run += (uint32_t)__popcll(bal);
      // every slot's x stored (the readers mask by the keep bits): whole
      // lines, 277 -> 264 us at 64M (same box; measured against kept-only
      // stores once fused_hist0's timing was stable, see fused_hist0); as
      // streaming (nt) stores: select 280 -> 274 us and assign_gather's
      // re-read of x 202 -> 191 us at 64M (same box A/B/A/B)
      __builtin_nontemporal_store(xv, xt + k * 64 + lane);
      if (keep) {
        const uint64_t kk = dkey(xv);
        kmin = kk < kmin ? kk : kmin;
        kmax = kk > kmax ? kk : kmax;
        if (hv && kk >= ka && kk <= kb) {
          if (kk >= hlo && kk <= hhi) {
            const uint32_t d = (uint32_t)((kk - hlo) >> hsh);
            atomicAdd(&lh[d >> 1], 1u << (16 * (d & 1)));
          } else {
            oob = true;
          }
        }
      }
    }
  };
  // SPEC: tiles [t0, t1) of the current SH_TMAX group are complete (after a
  // block barrier): their [bin][tile] counts out, the LDS counts zeroed
  auto flush_tc = [&](uint32_t t0, uint32_t t1) {
    if constexpr (SPEC) {
      const int ntl = (int)(t1 - t0), nr = nb + 1;
      for (int k = threadIdx.x; k < ntl * nr; k += SH_BT) {
        const int b = k / ntl, tl = k - b * ntl;
        uint32_t &c = tcs[((t0 - ta + tl) % SH_TMAX) * nrs + b];
        sa.th[(int64_t)b * nt + t0 + tl] = c;
        c = 0;
      }
    }
  };
  // end of a tile: the wave's count; every SH_TMAX tiles the u16 digit rows
  auto tile_end = [&](uint32_t tile) {
    if (lane == 0) {
      wcnt[(int64_t)tile * SH_NW + w] = run;
      if (tile - ta < SH_MAXT) tcnt[tile - ta][w] = run;
    }
    if (hv && (tile - ta) % SH_TMAX == SH_TMAX - 1 && tile + 1 < tb) {  // (block-uniform)
      __syncthreads();  // every wave's counts of this row's tiles are in
      if (spec) flush_tc(tile + 1 - SH_TMAX, tile + 1);
      uint32_t *row = rows16 + ((int64_t)blockIdx.x * rsub + (tile - ta) / SH_TMAX) * (MS0_DIG / 2);
      for (int i = threadIdx.x; i < MS0_DIG / 2; i += SH_BT) {
        row[i] = lh[i];
        lh[i] = 0;
      }
      __syncthreads();
    }
  };
  // the tile loop, once per kind of block: speculating or not (one loop
  // choosing per half had both bodies' registers live: spills)
  auto tiles = [&](auto sp) {
    Half A, B;
    if (ta < tb) ld(ta, 0, A, sp);
    for (uint32_t tile = ta; tile < tb; ++tile) {
      ld(tile, 1, B, sp);
      run = 0;
      if constexpr (decltype(sp)::value) sel_spec(tile, 0, A); else sel(tile, 0, A);
      ld(tile + 1 < tb ? tile + 1 : tile, 0, A, sp);
      if constexpr (decltype(sp)::value) sel_spec(tile, 1, B); else sel(tile, 1, B);
      tile_end(tile);
    }
  };
  if (SPEC && spec) tiles(std::integral_constant<bool, SPEC>{});
  else tiles(std::false_type{});
  // (three half buffers with two halves in flight, at the same 2 blocks per
  // CU: 273 -> 275 us — the loads in flight are not what bounds it: dropped)
  // the block's key range: one atomic pair per block
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const unsigned long long a = __shfl_xor(kmin, o, 64);
    const unsigned long long b = __shfl_xor(kmax, o, 64);
    kmin = a < kmin ? a : kmin;
    kmax = b > kmax ? b : kmax;
  }
  if (lane == 0) {
    wmin[w] = kmin;
    wmax[w] = kmax;
  }
  const uint64_t anyoob = __ballot(oob);
  if (anyoob && lane == 0) atomicOr(hflag, 1u);
  __syncthreads();
  if (SPEC && spec) {  // the block's sums row and list, its last tiles' counts
    if (tb > ta) flush_tc(ta + ((tb - ta - 1) / SH_TMAX) * SH_TMAX, tb);
    if (s_edge)
      for (int i = threadIdx.x; i < 2 * (nb + 1); i += SH_BT)
        if (slt[i]) atomicAdd(&sa.lteq[i], slt[i]);
    for (int i = threadIdx.x; i < macc; i += SH_BT) sa.slab[(int64_t)blockIdx.x * macc + i] = sacc[i];
    if (threadIdx.x == 0) {
      const uint32_t c = sdk;
      sa.rbase[blockIdx.x] = (uint32_t)lbase;
      sa.rn[blockIdx.x] = c < lcap ? c : lcap;
      if (c > lcap) atomicOr(sa.flag, 1u);
    }
  }
  if (w == 0) {
    // block-local exclusive tile offsets (lane = tile, 64 at a time) and the block total
    uint32_t carry = 0;
    for (uint32_t t0 = ta; t0 < tb; t0 += 64) {
      const uint32_t t = t0 + lane;
      uint32_t c = 0;
      if (t < tb) {
        if (t - ta < SH_MAXT) {
#pragma unroll
          for (int ww = 0; ww < SH_NW; ++ww) c += tcnt[t - ta][ww];
        } else {
#pragma unroll
          for (int ww = 0; ww < SH_NW; ++ww) c += wcnt[(int64_t)t * SH_NW + ww];
        }
      }
      uint32_t x = c;
#pragma unroll
      for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = __shfl_up(x, o, 64);
        if (lane >= (uint32_t)o) x += y;
      }
      if (t < tb) toff[t] = carry + x - c;
      carry += __shfl(x, 63, 64);
    }
    if (lane == 0) {
      btot[blockIdx.x] = carry;
      unsigned long long a = ~0ull, b = 0ull;
      for (int ww = 0; ww < SH_NW; ++ww) {
        a = wmin[ww] < a ? wmin[ww] : a;
        b = wmax[ww] > b ? wmax[ww] : b;
      }
      unsigned long long *mmq = minmax + 2 * (blockIdx.x % MM_SLOTS);
      if (a != ~0ull) atomicMax(&mmq[0], ~a);
      if (b != 0ull) atomicMax(&mmq[1], b);
    }
  }
  if (hv) {  // this block's last row, and zero rows after it (coalesced words)
    const uint32_t last = tb > ta ? (tb - ta - 1) / SH_TMAX : 0u;
    for (uint32_t r = last; r < rsub; ++r) {
      uint32_t *row = rows16 + ((int64_t)blockIdx.x * rsub + r) * (MS0_DIG / 2);
      for (int i = threadIdx.x; i < MS0_DIG / 2; i += SH_BT) row[i] = r == last ? lh[i] : 0u;
    }
  } else if (hint && h.valid && threadIdx.x == 0) {
    // more tiles than the block's rsub rows of u16 counts hold: fall back to
    // the re-read of x (the host sizes rsub for the span, up to SH_RSUB_MAX)
    atomicOr(hflag, 1u);
  }
}

// A first tiled call has no previous geometry for its level-0 histogram, so
// fused_hist0 would read x a second time.  sample_hint gives it one: the
// kept window keys of S (<= 32768) evenly spaced particles of the span, their range
// widened below by 2^-6 in value and above by 2^5 (a power-law tail) or up
// to the Sphere's bound (|c| + R: no key beyond it), clipped to the window.
// The sampled minimum of S of N particles in an r^3 core (Plummer) is the
// whole set's times (N/S)^(1/3) E^(1/3), E the ratio of two unit
// exponentials: it stays within 2^6 but for a fraction 1 / (1 + 2^18 S/N)
// of the sets (0.4 % at 38M; an r^2 core escapes more often).  A key
// outside it escapes the hint as any other's would (select_tiles sets
// hflag): the call re-reads x, the results are the same.  The last block
// writes the hint and re-arms the scratch (mm2 = [~min, max], done).
constexpr int SMP_BT = 256, SMP_PER = 4;  // samples per thread, their loads in flight together
template <bool FAM>
__global__ void __launch_bounds__(SMP_BT)
    sample_hint(const double *__restrict__ pos, int64_t n, SelectParams p, int64_t span,
                uint32_t S, uint64_t ka, uint64_t kb, uint64_t kub,
                unsigned long long *__restrict__ mm2, unsigned *__restrict__ done,
                SelHint *__restrict__ out) {
  __shared__ unsigned long long wmin[SMP_BT / 64], wmax[SMP_BT / 64];
  __shared__ int s_last;
  unsigned long long kmin = ~0ull, kmax = 0ull;
  double px[SMP_PER], py[SMP_PER], pz[SMP_PER];
  bool in[SMP_PER];
#pragma unroll
  for (int u = 0; u < SMP_PER; ++u) {
    const uint32_t j = (blockIdx.x * SMP_PER + u) * SMP_BT + threadIdx.x;
    const int64_t i = p.base + (int64_t)(((uint64_t)j * (uint64_t)span) / S);
    in[u] = j < S && i < n && (!FAM || in_family(i, p));
    const double *q = pos + 3 * (in[u] ? i : 0);
    px[u] = q[0];
    py[u] = q[1];
    pz[u] = q[2];
  }
#pragma unroll
  for (int u = 0; u < SMP_PER; ++u) {
    double xv = 0.0;
    if (in[u] && select_xyz(px[u], py[u], pz[u], p, xv)) {
      const uint64_t k = dkey(xv);
      if (k >= ka && k <= kb) {
        kmin = k < kmin ? k : kmin;
        kmax = k > kmax ? k : kmax;
      }
    }
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const unsigned long long a = __shfl_xor(kmin, o, 64), b = __shfl_xor(kmax, o, 64);
    kmin = a < kmin ? a : kmin;
    kmax = b > kmax ? b : kmax;
  }
  const int w = threadIdx.x >> 6;
  if (lane_id() == 0) {
    wmin[w] = kmin;
    wmax[w] = kmax;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int q = 1; q < SMP_BT / 64; ++q) {
      kmin = wmin[q] < kmin ? wmin[q] : kmin;
      kmax = wmax[q] > kmax ? wmax[q] : kmax;
    }
    if (kmin != ~0ull) atomicMax(&mm2[0], ~kmin);
    if (kmax != 0ull) atomicMax(&mm2[1], kmax);
    __threadfence();
    s_last = atomicAdd(done, 1u) + 1 == gridDim.x;
  }
  __syncthreads();
  if (!s_last || threadIdx.x != 0) return;
  __threadfence();
  const unsigned long long a = ~__hip_atomic_load(&mm2[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const unsigned long long b = __hip_atomic_load(&mm2[1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  mm2[0] = 0ull;
  mm2[1] = 0ull;
  *done = 0u;
  SelHint h{};
  if (b >= a && a != ~0ull) {
    // keys of non-negative doubles: one binary order of magnitude = 1 << 52
    constexpr uint64_t OCT = 1ull << 52, KZERO = 0x8000000000000000ull;  // dkey(+0.0)
    uint64_t lo = a >= KZERO + 6 * OCT ? a - 6 * OCT : (a >= KZERO ? KZERO : a);
    uint64_t hi = kub ? kub : (b + 5 * OCT < b ? ~0ull : b + 5 * OCT);
    lo = lo > ka ? lo : ka;
    hi = hi < kb ? hi : kb;
    if (hi >= lo) {
      const uint64_t sp = hi - lo;
      const int B = sp ? 64 - __builtin_clzll(sp) : 1;
      h.w = B < MS0_BITS ? B : MS0_BITS;
      h.s = B - h.w;
      h.lo = lo;
      h.valid = 1;
      h.sampled = 1;
    }
  }
  *out = h;
}

// A speculating select_tiles stores no x (SPEC_NOX): a hit never reads it.
// When a call does need it after all — a key escaped the level-0 hint
// (fused_hist0 counts x again) or the digits missed the table (assign_gather
// bins x) — each block of those kernels first recomputes x for its own
// tiles from the positions (the kept slots, by the keep words; select_xyz:
// the same value select_tiles computed); after a hit the host marks x
// missing and ensure_x rebuilds it the same way (xsrc_kernel) for a later
// consumer.
__device__ void xsrc_tiles(const XSrc &xs, uint32_t ta, uint32_t tb) {
  constexpr int U = 4;  // slots per thread in flight
  const int bt = blockDim.x;
  const int64_t s0 = (int64_t)ta * TILE, s1 = (int64_t)tb * TILE;
  for (int64_t a = s0 + threadIdx.x; a < s1; a += (int64_t)bt * U) {
    double px[U], py[U], pz[U];
    bool kp[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t sl = a + (int64_t)u * bt;
      kp[u] = sl < s1 && ((xs.kw[sl >> 6] >> (sl & 63)) & 1ull);
      const double *q = xs.pos + 3 * (kp[u] ? xs.sp.base + sl : 0);
      px[u] = q[0];
      py[u] = q[1];
      pz[u] = q[2];
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      double xv = 0.0;
      if (kp[u] && select_xyz(px[u], py[u], pz[u], xs.sp, xv)) xs.x[a + (int64_t)u * bt] = xv;
    }
  }
}
__global__ void __launch_bounds__(TPB) xsrc_kernel(XSrc xs, uint32_t nt, uint32_t tiles_per_block) {
  const uint32_t ta = blockIdx.x * tiles_per_block;
  xsrc_tiles(xs, ta, min(nt, ta + tiles_per_block));
}

// fused_hist0 blocks >= 1 (tiled): the global tile offsets, select_tiles'
// block-local ones plus each select block's base (the sum of the block
// totals before it); block 0: the kept count
__device__ void tile_offsets_fix(const uint32_t *__restrict__ btot, uint32_t nt, uint32_t *toff,
                                 uint32_t *red) {
  const uint32_t G0 = gridDim.x;
  if (blockIdx.x == 0 || G0 < 2) return;
  const uint32_t ab = blockIdx.x - 1;  // select blocks ab SH_K .. + SH_K - 1
  const uint32_t j0 = ab * SH_K;
  uint32_t v = 0;
  for (uint32_t j = threadIdx.x; j < j0; j += blockDim.x) v += btot[j];
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  if (lane_id() == 0) red[threadIdx.x >> 6] = v;
  __syncthreads();
  uint32_t base = 0;
  for (int q = 0; q < (int)(blockDim.x >> 6); ++q) base += red[q];
  const uint32_t ta0 = (uint32_t)((uint64_t)nt * ab / (G0 - 1));
  const uint32_t tb0 = (uint32_t)((uint64_t)nt * (ab + 1) / (G0 - 1));
  for (uint32_t sb = 0; sb < (uint32_t)SH_K; ++sb) {
    const uint32_t ta = ta0 + (uint32_t)((uint64_t)(tb0 - ta0) * sb / SH_K);
    const uint32_t tb = ta0 + (uint32_t)((uint64_t)(tb0 - ta0) * (sb + 1) / SH_K);
    for (uint32_t t = ta + threadIdx.x; t < tb; t += blockDim.x) toff[t] += base;
    base += btot[j0 + sb];
  }
}

// every key slot of this block (grid-stride by EL_STEP): f(x value, valid).
// (Issuing the next step's loads before this step's keys are processed made
// fused_gather slower at 64M, 71 -> 91 us: kept single-step.)
// With a tiled selection block 0 runs the tile scan instead (fused_hist0)
// and blocks 1.. each take a contiguous range of tiles (tile_range), two
// per step: assign_gather walks the same ranges, so a block's gathered keys
// are exactly those it counted here.
__device__ __forceinline__ void tile_range(uint32_t nt, uint32_t &ta, uint32_t &tb) {
  const uint32_t b0 = gridDim.x > 1 ? 1u : 0u;
  if (blockIdx.x < b0) {
    ta = tb = 0;
    return;
  }
  const uint64_t G = gridDim.x - b0, b = blockIdx.x - b0;
  ta = (uint32_t)((uint64_t)nt * b / G);
  tb = (uint32_t)((uint64_t)nt * (b + 1) / G);
}

template <class F>
__device__ __forceinline__ void el_for_each(const double *__restrict__ x, const ElRange &er,
                                            int64_t lim, F &&f) {
  constexpr int U = EL_U;
  if (er.kw) {
    uint32_t ta, tb;
    tile_range(er.nt, ta, tb);
    if (lim == 0 || ta >= tb) return;
    // unconditional 16-B loads of slot pairs with their keep words (a lone
    // last tile re-reads itself for its missing partner: no branch around a
    // load), the next step's in flight while this one is processed
    // (ping-pong, no register copies)
    auto ld = [&](uint32_t t, double *v, uint64_t *kv) {
      const int64_t i0 = (int64_t)t * TILE;
      const int64_t end = (int64_t)(t + 1 < tb ? t + 2 : t + 1) * TILE;
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int64_t i = i0 + 2 * (u * MS0_TPB + threadIdx.x);
        const int64_t ii = i < end ? i : i - TILE;
        const double2 q = *(const double2 *)(x + ii);
        v[2 * u] = q.x;
        v[2 * u + 1] = q.y;
        kv[u] = er.kw[ii >> 6];
      }
    };
    auto use = [&](uint32_t t, const double *v, const uint64_t *kv) {
      const bool two = t + 1 < tb;
#pragma unroll
      for (int u = 0; u < 2 * U; ++u) {
        const int64_t j = 2 * ((u >> 1) * MS0_TPB + threadIdx.x) + (u & 1);
        f(v[u], (j < TILE || two) && ((kv[u >> 1] >> (j & 63)) & 1ull));
      }
    };
    double va[2 * U], vb[2 * U];
    uint64_t ka[U], kb[U];
    // unconditional loads (past the range: the first tile again), so the
    // same loads are in flight on every path and the vmcnt waits stay exact
    auto cl = [&](uint32_t t) { return t < tb ? t : ta; };
    ld(ta, va, ka);
    for (uint32_t t = ta; t < tb; t += 4) {
      ld(cl(t + 2), vb, kb);
      use(t, va, ka);
      if (t + 2 >= tb) break;
      ld(cl(t + 4), va, ka);
      use(t + 2, vb, kb);
    }
    return;
  }
  for (int64_t i0 = (int64_t)blockIdx.x * EL_STEP; i0 < lim; i0 += (int64_t)gridDim.x * EL_STEP) {
    double v[2 * U];
#pragma unroll
    for (int u = 0; u < U; ++u) load_pair(x, i0 + 2 * (u * MS0_TPB + threadIdx.x), lim, v + 2 * u);
#pragma unroll
    for (int u = 0; u < 2 * U; ++u) {
      const int64_t i = i0 + 2 * ((u >> 1) * MS0_TPB + threadIdx.x) + (u & 1);
      f(v[u], i < er.n);
    }
  }
}

static_assert(MS0_TPB == TS_TPB, "fused_hist0's block 0 runs the tile scan");

// level-0 histogram rows (msel_hist0 with the base / shift / length from ctl)
__global__ void __launch_bounds__(MS0_TPB)
    fused_hist0(const double *__restrict__ x, FusedSetup fsu, FusedCtl *__restrict__ ctl_out,
                unsigned long long *__restrict__ counts, int nb, uint32_t *__restrict__ rows) {
  __shared__ uint32_t lh[MS0_DIG];
  // the control record derived once per block and broadcast through LDS
  // (in every wave, its ~20 scalar loads of the same few lines from all 4096
  // waves; bimodal 19 / 31 us per process at 64M)
  __shared__ FusedCtl sctl;
  if (threadIdx.x == 0) sctl = fused_ctl_eff(fsu);
  __syncthreads();
  const FusedCtl ctl = sctl;
  if (blockIdx.x == 0 && threadIdx.x == 0 && fsu.hint_out) {
    // this call's window key range widened by 1/64 of its span on each side
    // (a similar next call still fits), as a level-0 geometry for the next call
    const FusedCtl nat = fused_ctl(fsu);
    SelHint h{};
    if (!(nat.err & 2)) {
      const uint64_t hi = fsu.kb < nat.kmax ? fsu.kb : nat.kmax;
      const uint64_t m = (hi - nat.lo) >> 6;
      const uint64_t lo2 = nat.lo >= m ? nat.lo - m : 0ull;
      const uint64_t hi2 = hi + m < hi ? ~0ull : hi + m;
      const uint64_t span = hi2 - lo2;
      const int B = span ? 64 - __builtin_clzll(span) : 1;
      h.w = B < MS0_BITS ? B : MS0_BITS;
      h.s = B - h.w;
      h.lo = lo2;
      h.valid = 1;
      // this call kept the hinted geometry (every window key inside it): when
      // the fresh one has the same digit width, keep it — the level-0 digits
      // (and the stored bin table's, SpecTab) stay comparable from call to
      // call of a slowly changing snapshot
      if (ctl.hint && !fsu.hint->sampled && fsu.hint->s == h.s && fsu.hint->w == h.w) h = *fsu.hint;
    }
    *fsu.hint_out = h;
  }
  __shared__ uint32_t red[MS0_TPB / 64];
  if (blockIdx.x == 0) {  // the step's shared state: control record, zeroed counts / H
    if (fsu.tiled) {  // tiled selection: the kept count = the sum of select_tiles' block totals
      const uint32_t G1 = SH_K * (gridDim.x - 1);
      uint32_t v = 0;
      for (uint32_t j = threadIdx.x; j < G1; j += MS0_TPB) v += fsu.btot[j];
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
      if (lane_id() == 0) red[threadIdx.x >> 6] = v;
      __syncthreads();
      if (threadIdx.x == 0) {
        uint32_t total = 0;
        for (int q = 0; q < MS0_TPB / 64; ++q) total += red[q];
        FusedCtl c = ctl;
        c.n = total;
        *ctl_out = c;
      }
    } else if (threadIdx.x == 0) {
      *ctl_out = ctl;
    }
    for (int k = threadIdx.x; k <= nb; k += MS0_TPB) counts[k] = 0;  // for assign_bins
    for (int k = threadIdx.x; k < fsu.nzero; k += MS0_TPB) fsu.zero[k] = 0;
  }
  if (fsu.tiled) tile_offsets_fix(fsu.btot, fsu.nt, fsu.toff, red);  // (blocks >= 1)
  if (ctl.hint) return;  // select_tiles counted the keys (msel_reduce0h sums its rows)
  __shared__ int s_nox;
  if (threadIdx.x == 0) s_nox = (fsu.tiled && fsu.sflag && (*fsu.sflag & 2u)) ? 1 : 0;
  __syncthreads();
  if (s_nox) {  // a speculating selection stored no x and a key escaped the hint: x of this block's tiles
    uint32_t ta, tb;
    tile_range(fsu.nt, ta, tb);
    xsrc_tiles(fsu.xs, ta, tb);
    __threadfence();
    __syncthreads();
  }
  for (int i = threadIdx.x; i < MS0_DIG; i += MS0_TPB) lh[i] = 0;
  __syncthreads();
  const uint64_t ka = fsu.ka, kb = fsu.kb;
  const ElRange er = el_range(fsu.tiled ? fsu.kw : nullptr, fsu.nt, (ctl.err & 2) ? 0 : ctl.n);
  const int64_t lim = (ctl.err & 2) ? 0 : er.lim;
  const uint64_t base = ctl.lo;
  const int s = ctl.s0;
  el_for_each(x, er, lim, [&](double xv, bool ok) {
    const uint64_t k = dkey(xv);
    if (ok && k >= ka && k <= kb) atomicAdd(&lh[(uint32_t)((k - base) >> s)], 1u);
  });
  __syncthreads();
  uint32_t *row = rows + (int64_t)blockIdx.x * MS0_DIG;
  for (int i = threadIdx.x; i < MS0_DIG; i += MS0_TPB) row[i] = lh[i];
}

// Level-0 resolve + groups and the per-block segment offsets, one launch of
// nq blocks x 1024 (was fused_resolve0 + fused_boff): EVERY block scans H
// (64 KB, L2-resident) and derives the window size m, each rank's level-0
// digit and residual rank (bins.py:738-744 ranks), the distinct chosen
// digits in rank order (= ascending) — the groups — with their key counts
// and segment offsets, identically; block 0 publishes them (R, gdig, goff,
// gq, ctl->ng / m / total), and block g then gives group g its per-block
// offsets: block b of fused_hist0 / select_tiles counted rows[b][digit of g]
// keys of group g, so its keys go to goff[g] + the exclusive sum over
// earlier blocks.  H is left as it is (the next call's msel_reduce0h
// overwrites every word).
constexpr int FR_TPB = 1024;
__global__ void __launch_bounds__(FR_TPB)
    fused_resolve(const uint32_t *__restrict__ H, FusedCtl *__restrict__ ctl, int64_t nbins, int nq,
                  MsRank *__restrict__ R, uint32_t *__restrict__ gdig, uint32_t *__restrict__ goff,
                  uint32_t *__restrict__ gq, const uint32_t *__restrict__ rows, int g0,
                  uint32_t *__restrict__ boff, uint32_t *__restrict__ bcnt,
                  uint32_t *__restrict__ lc, const uint32_t *__restrict__ rows16, uint32_t rsub,
                  const SpecTab *__restrict__ tab, uint32_t *__restrict__ sflag, int nb,
                  uint32_t *__restrict__ lteq) {
  constexpr int PT = MS0_DIG / FR_TPB;
  __shared__ uint32_t incl[MS0_DIG];
  __shared__ uint32_t wsum[FR_TPB / 64];
  __shared__ uint32_t qdig[MS_MAXQ];
  __shared__ uint32_t gstart[MS_MAXQ + 1];
  __shared__ uint32_t gd[MS_MAXQ], go[MS_MAXQ + 1];
  __shared__ int sng, s_err, s_w0, s_hint, s_spec, s_eok;
  __shared__ uint32_t s_flag;
  const int tid = threadIdx.x;
  const uint32_t lane = lane_id();
  const int wv = tid >> 6;
  const bool pub = blockIdx.x == 0;  // the block that publishes the shared results
  if (tid == 0) {  // the control record's fields: one load per block
    s_err = ctl->err;
    s_w0 = ctl->w0;
    s_hint = ctl->hint;
    // the stored bin table (SpecTab) applies iff this call's geometry and
    // every rank's level-0 digit are its own (compared below, in every
    // block: an edge hit needs no per-block offsets)
    s_spec = 0;
    if (tab && tab->valid && !(s_err & 2) && tab->nb == nb && tab->nq == nq &&
        tab->lo == ctl->lo && tab->s0 == ctl->s0 && tab->w0 == s_w0)
      s_spec = 1;
    s_eok = 1;  // (edge speculation: every edge at its rank, below)
    s_flag = sflag ? *sflag : 0u;  // (reset by fused_finish, after every reader)
  }
  for (int k = tid; k < MS0_DIG; k += FR_TPB) incl[k] = H[k];  // coalesced, via LDS
  __syncthreads();
  uint32_t v[PT], tot = 0;
#pragma unroll
  for (int k = 0; k < PT; ++k) {
    v[k] = incl[tid * PT + k];
    tot += v[k];
  }
  __syncthreads();
  // block exclusive scan of the per-thread totals (16 waves)
  uint32_t xs = tot;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t y = __shfl_up(xs, o, 64);
    if (lane >= (uint32_t)o) xs += y;
  }
  if (lane == 63) wsum[wv] = xs;
  __syncthreads();
  uint32_t run = xs - tot;
  for (int k = 0; k < wv; ++k) run += wsum[k];
#pragma unroll
  for (int k = 0; k < PT; ++k) {
    run += v[k];
    incl[tid * PT + k] = run;
  }
  __syncthreads();
  const int64_t m = (s_err & 2) ? 0 : (int64_t)incl[MS0_DIG - 1];
  const int top = (1 << s_w0) - 1;
  for (int q = tid; q < nq; q += FR_TPB) {
    int64_t r = 0;
    if (m >= 2) r = (q == nq - 1) ? m - 1 : (int64_t)((double)(q * m) / (double)nbins);
    int a = 0, b = top;  // first digit whose inclusive count exceeds r
    while (a < b) {
      const int mid = (a + b) >> 1;
      if ((int64_t)incl[mid] <= r) a = mid + 1; else b = mid;
    }
    if (pub) {
      R[q].prefix = (uint64_t)a;
      R[q].rr = r - (a ? (int64_t)incl[a - 1] : 0);
    }
    qdig[q] = (uint32_t)a;
    if (s_spec && tab->qd[q] != (uint32_t)a) s_spec = 0;  // (benign race: all write 0)
    if (lteq) {  // the table's edge q is this call's iff rank r is among its equals
      const int64_t rr = r - (a ? (int64_t)incl[a - 1] : 0);
      const uint32_t lt = lteq[2 * q], eq = lteq[2 * q + 1];
      if (!((int64_t)lt <= rr && rr < (int64_t)lt + (int64_t)eq)) s_eok = 0;
    }
  }
  __syncthreads();
  // a hit: select_tiles binned every key with the table (no block gave up);
  // an edge-speculating call (it listed no deferred keys) only when its
  // edges hold too — otherwise the assignment runs
  const uint32_t f = s_flag;
  const bool hit = s_spec && sflag && !(f & 1u) && (!(f & 4u) || s_eok);
  const bool edge_hit = hit && (f & 4u);
  if (pub && tid == 0)
    ctl->spec = (s_spec ? SPEC_MATCH : 0) | (hit ? SPEC_HIT : 0) | ((f & 2u) ? SPEC_NOX : 0) |
                (edge_hit ? SPEC_EDGE : 0);
  // groups: run starts of the (non-decreasing) digits; one wave numbers them
  if (wv == 0) {
    uint32_t ng = 0;
    for (int q0 = 0; q0 < nq; q0 += 64) {
      const int q = q0 + (int)lane;
      const bool st = q < nq && (q == 0 || qdig[q - 1] != qdig[q]);
      const uint64_t bal = __ballot(st);
      if (st) gstart[ng + rank_below(bal)] = (uint32_t)q;
      ng += (uint32_t)__popcll(bal);
    }
    if (lane == 0) {
      gstart[ng] = (uint32_t)nq;
      sng = (int)ng;
      if (pub) {
        ctl->ng = (int32_t)ng;
        ctl->m = m;
      }
    }
  }
  __syncthreads();
  const int ng = sng;
  // group g: digit, count, segment offset (prefix over groups: one wave)
  if (wv == 0) {
    uint32_t base = 0;
    for (int gg0 = 0; gg0 < ng; gg0 += 64) {
      const int g = gg0 + (int)lane;
      uint32_t c = 0, d = 0;
      if (g < ng) {
        d = qdig[gstart[g]];
        c = incl[d] - (d ? incl[d - 1] : 0u);
        gd[g] = d;
        if (pub) gdig[g] = d;
      }
      uint32_t ys = c;
#pragma unroll
      for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = __shfl_up(ys, o, 64);
        if (lane >= (uint32_t)o) ys += y;
      }
      if (g < ng) {
        go[g] = base + ys - c;
        if (pub) goff[g] = base + ys - c;
      }
      base += __shfl(ys, 63, 64);
    }
    if (lane == 0) {
      go[ng] = base;
      if (pub) {
        goff[ng] = base;
        ctl->total = base;
      }
    }
  }
  if (pub) {
    for (int g = tid; g <= ng; g += FR_TPB) gq[g] = gstart[g];  // each group's ranks
    for (int q = tid; q < nq; q += FR_TPB) {  // every rank's group: last start <= q
      int a = 0, b = ng - 1;
      while (a < b) {
        const int mid = (a + b + 1) >> 1;
        if ((int)gstart[mid] <= q) a = mid; else b = mid - 1;
      }
      R[q].group = a;
    }
  }
  __syncthreads();
  // this block's group: the segment offsets of the assignment's workgroups
  // (one thread each; an edge hit gathers no keys).  Hinted: one workgroup
  // per select block, b = 1 + select block (its rsub u16 rows count its
  // keys); else one per level-0 block of fused_hist0 (its row), b < g0.
  // Either way the workgroups' slices of a group follow in index order, so
  // the select blocks of level-0 block ab hold one contiguous run.
  const int g = blockIdx.x;
  if ((s_err & 2) || g >= ng || edge_hit) return;
  const uint32_t d = gd[g];
  uint32_t c = 0;
  const int b = tid;  // nblk <= FR_TPB
  const int nblk = s_hint ? at_blocks(g0) : g0;
  if (s_hint) {
    if (b >= 1 && b < nblk)
      for (uint32_t j = 0; j < rsub; ++j)  // the select block's rsub rows
        c += (rows16[((int64_t)(b - 1) * rsub + j) * (MS0_DIG / 2) + (d >> 1)] >> (16 * (d & 1))) &
             0xffffu;
  } else if (b < g0) {
    c = rows[(int64_t)b * MS0_DIG + d];
  }
  // exclusive scan of c over the block's 16 waves (block_excl_scan is 4-wave)
  uint32_t xc = c;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t y = __shfl_up(xc, o, 64);
    if (lane >= (uint32_t)o) xc += y;
  }
  if (lane == 63) wsum[wv] = xc;
  __syncthreads();
  uint32_t ex = xc - c, btot = 0;
  for (int k = 0; k < FR_TPB / 64; ++k) {
    ex += k < wv ? wsum[k] : 0u;
    btot += wsum[k];
  }
  if (b < nblk) boff[(int64_t)b * MS_MAXQ + g] = go[g] + ex;
  if (bcnt && b < nblk && c) atomicAdd(&bcnt[b], c);  // keys workgroup b gathers, all groups
  if (lc && b == 0) lc[g] = btot;  // distributed: this rank's keys of group g
}

// Distributed equaln: every rank's keys of group g occupy one slice of the
// GLOBAL segment (goff from the summed histogram), ranks in order: rank r's
// slice starts after the keys of ranks < r (lc_all[r'][g], all-reduced), so
// the ranks' gathers fill disjoint slots of one zeroed array and a SUM
// all-reduce of it is the all-gather of every group's keys.
__global__ void __launch_bounds__(TPB)
    dist_rank_offsets(const FusedCtl *__restrict__ ctl, const uint32_t *__restrict__ lc_all,
                      int rank, int g0, uint32_t *__restrict__ boff) {
  const int g = blockIdx.x;
  if ((ctl->err & 2) || g >= ctl->ng) return;
  uint32_t before = 0;
  for (int r = 0; r < rank; ++r) before += lc_all[(int64_t)r * MS_MAXQ + g];
  for (int b = threadIdx.x; b < g0; b += TPB) boff[(int64_t)b * MS_MAXQ + g] += before;
}

// Distributed: this rank's {kept count, look-back failure} for one i64 sum
// all-reduce, so a selection that failed on ANY rank fails on every rank at
// the same point (before the later collectives), not just on its own.
__global__ void dist_status(const FusedCtl *__restrict__ ctl, int64_t *__restrict__ out) {
  out[0] = ctl->n;
  out[1] = ctl->err & 1;
}

// keys of the chosen level-0 buckets -> their group's segment (key - base).
// Same grid and element order as fused_hist0, so block b owns exactly the
// slots fused_resolve gave it; inside the block an LDS counter per group hands
// them out (no global atomics: the keys of one group are few and were
// contended on a handful of addresses).
__global__ void __launch_bounds__(MS0_TPB)
    fused_gather(const double *__restrict__ x, uint64_t ka, uint64_t kb,
                 const FusedCtl *__restrict__ ctl, const uint32_t *__restrict__ gdig,
                 const uint32_t *__restrict__ boff, uint64_t *__restrict__ seg,
                 const uint64_t *__restrict__ tkw, uint32_t nt) {
  __shared__ uint16_t gidx[MS0_DIG];
  __shared__ uint32_t slot[MS_MAXQ];
  if (ctl->err & 2) return;
  const int64_t n = ctl->n;
  const int ng = ctl->ng;
  const uint64_t base = ctl->lo;
  const int s = ctl->s0;
  for (int i = threadIdx.x; i < MS0_DIG / 2; i += MS0_TPB) ((uint32_t *)gidx)[i] = ~0u;
  __syncthreads();
  for (int i = threadIdx.x; i < ng; i += MS0_TPB) {
    gidx[gdig[i]] = (uint16_t)i;
    slot[i] = boff[(int64_t)blockIdx.x * MS_MAXQ + i];
  }
  __syncthreads();
  const ElRange er = el_range(tkw, nt, n);
  const int64_t lim = er.lim;
  el_for_each(x, er, lim, [&](double xv, bool ok) {
    const uint64_t key = dkey(xv);
    if (ok && key >= ka && key <= kb) {
      const uint64_t off = key - base;
      const uint32_t g = gidx[(uint32_t)(off >> s)];
      if (g != 0xffffu) seg[atomicAdd(&slot[g], 1u)] = off;
    }
  });
}

// Per-bin sums fused into the assignment pass (the one-sync equaln path):
// the distinct per-element values ("monomials") the requested statistics'
// columns sum — e.g. Sum of the mass and the weights column of a
// mass-weighted Mean are the same Σw, accumulated once.  Monomial q is
// column col[q] of pbx_profile_moments_cols for field f[q] (0 = x, 1 =
// weights) and weights w[q] (0 = x, 1 = weights, -1 = none); block sums in
// LDS, one slab row (nm x nb) per block.

// One block (FR_TPB threads) per group: for each of its ranks, an MSD radix
// select (FS_BITS-bit digits, LDS histogram, parallel scan) over the group's
// keys below the level-0 digit; the segment is staged in LDS when it fits
// (<= FS_LDS keys), else every pass re-reads it from global memory.
constexpr int FS_BITS = 11;
constexpr int FS_DIG = 1 << FS_BITS;
constexpr int FS_LDS = 16384;  // group keys staged in LDS (128 KB: a 64M call's groups, ~10-20k keys, fit)
constexpr uint32_t FS_CAND = 256;  // finish_group: keys gathered for the direct rank

// keys of sk[0, S) below / equal to k: 8 keys per step from four 16-B LDS
// reads (broadcast: every lane reads the same address), counts split over
// two chains
__device__ __forceinline__ void count_rank(const uint64_t *sk, int S, uint64_t k, uint32_t &less,
                                           uint32_t &eq) {
  uint32_t l0 = 0, l1 = 0, e0 = 0, e1 = 0;
  int j = 0;
  for (; j + 8 <= S; j += 8) {
    const ulonglong2 a = *(const ulonglong2 *)(sk + j), b = *(const ulonglong2 *)(sk + j + 2);
    const ulonglong2 c = *(const ulonglong2 *)(sk + j + 4), d = *(const ulonglong2 *)(sk + j + 6);
    l0 += (a.x < k) + (a.y < k) + (b.x < k) + (b.y < k);
    l1 += (c.x < k) + (c.y < k) + (d.x < k) + (d.y < k);
    e0 += (a.x == k) + (a.y == k) + (b.x == k) + (b.y == k);
    e1 += (c.x == k) + (c.y == k) + (d.x == k) + (d.y == k);
  }
  for (; j < S; ++j) {
    const uint64_t kj = sk[j];
    l0 += kj < k ? 1u : 0u;
    e0 += kj == k ? 1u : 0u;
  }
  less = l0 + l1;
  eq = e0 + e1;
}

template <bool IN_LDS, bool SC1 = false>  // SC1: keys handed over in-launch (radial_mono)
__device__ void finish_group(const uint64_t *__restrict__ keys, int64_t S, uint64_t pref0, int s,
                             int64_t rr, uint32_t *hist, uint32_t *wsum, uint64_t *pick,
                             uint64_t &out) {
  const int tid = threadIdx.x;
  const uint32_t lane = lane_id();
  const int wv = tid >> 6;
  uint64_t pref = pref0;
  int sh = s;
  while (sh > 0) {
    const int wd = sh >= FS_BITS ? FS_BITS : sh;
    sh -= wd;
    const uint64_t hmask = ~((1ull << (sh + wd)) - 1);  // bits above this digit
    const uint32_t dm = (1u << wd) - 1;
    for (int d = tid; d < FS_DIG; d += FR_TPB) hist[d] = 0;
    __syncthreads();
    // FS_U keys per thread in flight (a group of ~20k keys re-read from
    // global memory was one latency per 1024 keys per pass)
    constexpr int FS_U = IN_LDS ? 1 : 8;
    for (int64_t i0 = 0; i0 < S; i0 += (int64_t)FR_TPB * FS_U) {
      uint64_t kv[FS_U];
#pragma unroll
      for (int u = 0; u < FS_U; ++u) {
        const int64_t i = i0 + (int64_t)u * FR_TPB + tid;
        const int64_t ic = i < S ? i : 0;  // unconditional loads
        kv[u] = SC1 ? __hip_atomic_load(&keys[ic], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                    : keys[ic];
      }
#pragma unroll
      for (int u = 0; u < FS_U; ++u) {
        const int64_t i = i0 + (int64_t)u * FR_TPB + tid;
        if (i < S && (kv[u] & hmask) == pref) atomicAdd(&hist[(uint32_t)(kv[u] >> sh) & dm], 1u);
      }
    }
    __syncthreads();
    // inclusive scan of 2 digits per thread; the thread whose digits hold rank rr picks
    const uint32_t c0 = hist[2 * tid], c1 = hist[2 * tid + 1];
    uint32_t xs = c0 + c1;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const uint32_t y = __shfl_up(xs, o, 64);
      if (lane >= (uint32_t)o) xs += y;
    }
    if (lane == 63) wsum[wv] = xs;
    __syncthreads();
    uint32_t ex = xs - (c0 + c1);
    for (int k = 0; k < wv; ++k) ex += wsum[k];
    if ((int64_t)ex <= rr && rr < (int64_t)(ex + c0)) {
      pick[0] = (uint64_t)(2 * tid);
      pick[1] = ex;
    } else if ((int64_t)(ex + c0) <= rr && rr < (int64_t)(ex + c0 + c1)) {
      pick[0] = (uint64_t)(2 * tid + 1);
      pick[1] = ex + c0;
    }
    __syncthreads();
    pref |= pick[0] << sh;
    rr -= (int64_t)pick[1];
    const uint32_t left = hist[(uint32_t)pick[0]];  // keys with the new prefix (block-uniform)
    __syncthreads();
    if (sh > 0 && left <= FS_CAND) {
      // few keys share the prefix (one 11-bit pass below a level-0 digit of
      // ~2k keys leaves ~1): gather them into LDS and take the rr-th by
      // counting, instead of the remaining radix passes (same key: the
      // rr-th smallest of the keys with this prefix, ties included)
      const uint64_t m2 = ~((1ull << sh) - 1);
      uint64_t *cand = (uint64_t *)hist;
      if (tid == 0) pick[1] = 0ull;
      __syncthreads();
      constexpr int FS_U = IN_LDS ? 1 : 8;
      for (int64_t i0 = 0; i0 < S; i0 += (int64_t)FR_TPB * FS_U) {
        uint64_t kv[FS_U];
#pragma unroll
        for (int u = 0; u < FS_U; ++u) {
          const int64_t i = i0 + (int64_t)u * FR_TPB + tid;
          const int64_t ic = i < S ? i : 0;
          kv[u] = SC1 ? __hip_atomic_load(&keys[ic], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                      : keys[ic];
        }
#pragma unroll
        for (int u = 0; u < FS_U; ++u) {
          const int64_t i = i0 + (int64_t)u * FR_TPB + tid;
          if (i < S && (kv[u] & m2) == pref)
            cand[atomicAdd((unsigned long long *)&pick[1], 1ull)] = kv[u];
        }
      }
      __syncthreads();
      const int nc = (int)pick[1];  // == left
      if (tid < nc) {
        const uint64_t k = cand[tid];
        uint32_t less = 0, eq = 0;
        for (int j = 0; j < nc; ++j) {
          const uint64_t kj = cand[j];
          less += kj < k ? 1u : 0u;
          eq += kj == k ? 1u : 0u;
        }
        if ((int64_t)less <= rr && rr < (int64_t)(less + eq)) pick[0] = k;  // ties: same value
      }
      __syncthreads();
      out = pick[0];
      __syncthreads();  // (pick / hist are reused by the caller's next rank)
      return;
    }
  }
  out = pref;
}

__global__ void __launch_bounds__(FR_TPB)
    fused_finish(const FusedCtl *__restrict__ ctl, const MsRank *__restrict__ R,
                 const uint32_t *__restrict__ gq, const uint32_t *__restrict__ goff,
                 const uint64_t *__restrict__ seg, double *__restrict__ edges,
                 const SpecTab *__restrict__ tab, int nq, uint32_t *__restrict__ sflag,
                 uint32_t *__restrict__ lteq) {
  __shared__ __attribute__((aligned(16))) uint64_t sk[FS_LDS];
  __shared__ __attribute__((aligned(16))) uint32_t hist[FS_DIG];  // (u64 candidates, finish_group)
  __shared__ uint32_t wsum[FR_TPB / 64];
  __shared__ uint64_t pick[2];
  static_assert(FS_DIG == 2 * FR_TPB, "two digits per thread");
  const int g = blockIdx.x;
  const int tid = threadIdx.x;
  __shared__ uint64_t c_lo;  // the control record's fields and the group's
  __shared__ int c_s, c_run; // segment: one load per block, through LDS
  __shared__ uint32_t c_o0, c_o1;
  __shared__ int c_edge;
  if (tid == 0) {
    c_edge = (ctl->spec & SPEC_EDGE) ? 1 : 0;
    c_run = !(ctl->err & 2) && g < ctl->ng && !c_edge;
    c_lo = ctl->lo;
    c_s = ctl->s0;
    c_o0 = c_run ? goff[g] : 0u;
    c_o1 = c_run ? goff[g + 1] : 0u;
  }
  // the speculation's flag and edge counts, read by fused_hist0 / fused_resolve:
  // zeroed for the next speculating call
  if (g == 0) {
    if (sflag && tid == 0) *sflag = 0u;
    if (lteq)
      for (int i = tid; i < 2 * nq; i += FR_TPB) lteq[i] = 0u;
  }
  __syncthreads();
  if (c_edge) {  // the edge speculation held: the table's edges are this call's
    if (g == 0)
      for (int q = tid; q < nq; q += FR_TPB) edges[q] = tab->edges[q];
    return;
  }
  if (!c_run) return;
  const uint64_t base = c_lo;
  const int s = c_s;
  const int64_t o = c_o0, S = (int64_t)c_o1 - o;
  const bool in_lds = S <= FS_LDS;
  if (in_lds) {  // (FS_SU loads per thread in flight: a group of ~10-20k keys was ~15 dependent trips)
    constexpr int FS_SU = 8;
    for (int64_t i0 = tid; i0 < S; i0 += (int64_t)FR_TPB * FS_SU) {
      uint64_t v[FS_SU];
#pragma unroll
      for (int u = 0; u < FS_SU; ++u) {
        const int64_t i = i0 + (int64_t)u * FR_TPB;
        v[u] = seg[o + (i < S ? i : 0)];
      }
#pragma unroll
      for (int u = 0; u < FS_SU; ++u) {
        const int64_t i = i0 + (int64_t)u * FR_TPB;
        if (i < S) sk[i] = v[u];
      }
    }
    __syncthreads();
  }
  if (S <= FR_TPB) {  // small group: each key's rank by counting (one key per thread)
    const uint64_t k = tid < S ? sk[tid] : ~0ull;
    uint32_t less = 0, eq = 0;
    count_rank(sk, (int)S, k, less, eq);
    for (int q = (int)gq[g]; q < (int)gq[g + 1]; ++q) {
      const int64_t rr = R[q].rr;
      if (tid < S && (int64_t)less <= rr && rr < (int64_t)(less + eq))
        edges[q] = dkey_inv(base + k);  // tied threads write the same value
    }
    return;
  }
  for (int q = (int)gq[g]; q < (int)gq[g + 1]; ++q) {  // this group's ranks
    uint64_t key;
    if (in_lds)
      finish_group<true>(sk, S, (uint64_t)R[q].prefix << s, s, R[q].rr, hist, wsum, pick, key);
    else
      finish_group<false>(seg + o, S, (uint64_t)R[q].prefix << s, s, R[q].rr, hist, wsum, pick,
                          key);
    if (tid == 0) edges[q] = dkey_inv(base + key);
  }
}

// the step's results in one contiguous block (mapped host memory for one rank, else one D2H copy):
// [ctl][edges nq][counts nb][monomial sums nm x nb].  Blocks [0, nhead)
// copy the head; block nhead + j sums column j of the assign slab (`rows`
// block rows, then the rows2 rows of slab2, fixed order: thread
// t takes rows t, t + TPB, ... in turn, then a fixed LDS tree) — the slab
// reduction and the packing in one launch.
// offs (optional): the CSR pass's scanned [bin][tile] histogram (ntiles
// columns); the bin counts are then its row-start differences, and are
// also stored to `counts` (assign_bins skipped its global count atomics).
constexpr int SLAB_G = 64;  // partial groups of the general (moments) path
// done (optional): `out` is coherent mapped host memory; every block adds
// one to *done once its stores have landed, and the block that brings it to
// done_target stores done_target at out[tagpos] (radial_mono's mono_done
// protocol): the host polls that word instead of a copy + stream sync.
struct PackArgs {
  const FusedCtl *ctl;
  const double *edges;
  int nq;
  unsigned long long *counts;
  int nb;
  const double *slab;
  int64_t rows;
  int nsum;
  double *out;
  const uint32_t *offs;
  uint32_t ntiles;
  int nhead;
  const double *slab2;
  int64_t rows2;
  uint64_t *done;
  uint64_t done_target;
  int tagpos;
  const unsigned long long *scan_wd;
  double *stage;  // done != null: the pack in device memory (sc1), copied out by the last block
};

// The completion-tag hand-off into coherent mapped host memory (fused_pack,
// csr_slots' pack blocks, radial_mono): each block stores its part of the
// pack into a DEVICE staging copy with sc1 stores and drains them (vmcnt)
// before a relaxed agent-scope count — the hand-off form of
// MI355X_MICROARCH.md's table, no L2 write-back per block; the block whose
// count completes the target loads the whole stage with sc1 loads, writes it
// to the host pack, drains, then issues the one system-scope fence and the
// tag.  Only that block writes host memory, so its fence orders every pack
// word before the tag.  (Round 4 let every block write the host pack
// directly and fenced only in the last block: with no ordering between
// different blocks' posted writes and the tag, a pack whose blocks ran
// beside heavy HBM traffic — the pack riding in csr_slots — was read with
// words missing.)  Returns in the last block only after the tag.
__device__ void pack_complete(uint64_t *done, uint64_t target, const double *stage, double *out,
                              int ntot, int tagpos, uint64_t tag) {
  __shared__ int s_last;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this block's sc1 stage stores performed
  __syncthreads();
  if (threadIdx.x == 0) {
    const uint64_t old = __hip_atomic_fetch_add(done, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    s_last = old + 1 == target;
  }
  __syncthreads();
  if (!s_last) return;
  for (int i = threadIdx.x; i < ntot; i += blockDim.x) out[i] = ld_sc1d(&stage[i]);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    __threadfence_system();
    __hip_atomic_store((uint64_t *)(out + tagpos), tag, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

// pack block pb of the a.nhead + a.nsum blocks (red: TPB doubles of LDS)
__device__ void pack_block(const PackArgs &a, int pb, double *red) {
  constexpr int NC = (int)(sizeof(FusedCtl) / sizeof(double));
  constexpr int ERRW = (int)(offsetof(FusedCtl, err) / sizeof(double));  // the word holding err
  const int nq = a.nq, nb = a.nb;
  // mapped: the staging copy (sc1), else the device pack itself (copied by the host)
  auto put = [&](int i, double v) {
    if (a.done) st_sc1d(&a.stage[i], v);
    else a.out[i] = v;
  };
  if (pb >= a.nhead) {
    const int j = pb - a.nhead;
    double v = 0.0;
    for (int64_t r = threadIdx.x; r < a.rows; r += TPB) v += a.slab[r * a.nsum + j];
    // fix_deferred's rows (none written on an edge hit)
    const int64_t rows2 = (a.ctl->spec & SPEC_EDGE) ? 0 : a.rows2;
    for (int64_t r = threadIdx.x; r < rows2; r += TPB) v += a.slab2[r * a.nsum + j];
    red[threadIdx.x] = v;
    __syncthreads();
#pragma unroll
    for (int h = TPB / 2; h > 0; h >>= 1) {
      if ((int)threadIdx.x < h) red[threadIdx.x] += red[threadIdx.x + h];
      __syncthreads();
    }
    if (threadIdx.x == 0) put(NC + nq + nb + j, red[0]);
  } else {
    const int t = pb * TPB + threadIdx.x;
    if (t < NC) {
      double v = ((const double *)a.ctl)[t];
      if (t == ERRW && a.scan_wd && *a.scan_wd) {  // a scan of this step gave up: err bit 4
        const uint64_t b = __builtin_bit_cast(uint64_t, v) |
                           ((uint64_t)4u << (8 * (offsetof(FusedCtl, err) % sizeof(double))));
        v = __builtin_bit_cast(double, b);
      }
      put(t, v);
    } else if (t < NC + nq) {
      put(t, a.edges[t - NC]);
    } else if (t < NC + nq + nb) {
      const int b = t - NC - nq;
      unsigned long long c;
      if (a.offs) {
        c = (unsigned long long)(a.offs[(int64_t)(b + 1) * a.ntiles] - a.offs[(int64_t)b * a.ntiles]);
        a.counts[b] = c;
      } else {
        c = a.counts[b];
      }
      put(t, __builtin_bit_cast(double, c));
    }
  }
  if (a.done) pack_complete(a.done, a.done_target, a.stage, a.out, a.tagpos, a.tagpos, a.done_target);
}

__global__ void __launch_bounds__(TPB) fused_pack(PackArgs a) {
  __shared__ double red[TPB];
  pack_block(a, (int)blockIdx.x, red);
}

// ----------------------------------------------------------------- assign
// bin_of (prims.h): bins.py:368-379 bin assignment

// One block takes `tpbk` (<= AS_TILES) consecutive 4096-element tiles:
// AS_TILES on big inputs (LDS init and the tile_hist rows amortised), fewer
// when that would leave the chip with too few blocks.  Per-tile bin
// counts double as the CSR pass's radix histogram ([digit][tile], one
// 8-bit pass) when nb < RADIX: tile_hist is then written, 8 consecutive
// tiles per digit row at once (one 32-B segment instead of 8 scattered
// words); else tile_hist is null.  Block totals go to `counts` with one
// contiguous atomic per bin.
constexpr int AS_TILES = 8;

// LDSE: the edges sit in LDS (nb + 1 <= LDS_EDGES); else they are read from
// global memory (L2-resident).  Loads of tile t+1 (x and weights) are in
// flight while tile t is binned.
// BT threads per block: 256, or 1024 when every block takes one tile of a
// small input (more waves per CU for the same tiles)
template <bool MOM, bool LDSE, bool WL, int BT>
__global__ void __launch_bounds__(BT)
    assign_bins(const double *__restrict__ x, int64_t n, const double *__restrict__ edges, int nb,
                uint32_t *__restrict__ bins, unsigned long long *__restrict__ counts,
                uint32_t *__restrict__ tile_hist, uint32_t ntiles, uint32_t tpbk,
                const int64_t *__restrict__ n_dev, const double *__restrict__ wsel, FusedStats fs,
                double *__restrict__ slab) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  __shared__ uint32_t th[AS_TILES][RADIX];
  if (n_dev) n = *n_dev;  // device-resident length (<= the n the grid was sized for)
  const int macc = MOM ? fs.nm * nb : 0;
  double *acc = (double *)smem;  // MOM: the block's sums
  double *e = acc + macc;
  uint32_t *cnt = (uint32_t *)(e + (LDSE ? nb + 1 : 0));
  if (MOM)
    for (int k = threadIdx.x; k < macc; k += BT) acc[k] = 0.0;
  if (LDSE)
    for (int k = threadIdx.x; k <= nb; k += BT) e[k] = edges[k];
  for (int k = threadIdx.x; k <= nb; k += BT) cnt[k] = 0;
  for (int k = threadIdx.x; k < AS_TILES * RADIX; k += BT) (&th[0][0])[k] = 0;
  __syncthreads();
  const uint32_t t0 = blockIdx.x * tpbk;
  const uint32_t t1 = min(ntiles, t0 + tpbk);
  constexpr bool wload = MOM && WL;  // weights loaded (else 1.0)
  // half tiles of AS_IPT x BT elements; software-pipelined: the next half
  // tile's loads (x and weights) fly while this one is binned (indices past
  // n read element 0: unconditional loads, no branches)
  constexpr int AS_IPT = TILE / BT / 2, HALF = AS_IPT * BT;
  const uint32_t s0 = 2 * t0, s1 = 2 * t1;
  double nv[AS_IPT], nw[AS_IPT];
#pragma unroll
  for (int k = 0; k < AS_IPT; ++k) {
    const int64_t i = (int64_t)s0 * HALF + k * BT + threadIdx.x;
    const int64_t j = (s0 < s1 && i < n) ? i : 0;
    nv[k] = x[j];
    if (wload) nw[k] = wsel[j];
  }
  for (uint32_t sh = s0; sh < s1; ++sh) {
    const int64_t base = (int64_t)sh * HALF;
    uint32_t *hrow = tile_hist ? th[(sh >> 1) - t0] : cnt;
    double v[AS_IPT], wv[AS_IPT];
#pragma unroll
    for (int k = 0; k < AS_IPT; ++k) {
      v[k] = nv[k];
      wv[k] = wload ? nw[k] : 1.0;
      const int64_t i = base + HALF + k * BT + threadIdx.x;
      const int64_t j = (sh + 1 < s1 && i < n) ? i : 0;
      nv[k] = x[j];
      if (wload) nw[k] = wsel[j];
    }
    uint32_t b[AS_IPT];  // the searches interleave; LDS atomics after
#pragma unroll
    for (int k = 0; k < AS_IPT; ++k) {
      const int64_t i = base + k * BT + threadIdx.x;
      b[k] = (i < n) ? (LDSE ? bin_of(v[k], e, nb) : bin_of(v[k], edges, nb)) : (uint32_t)nb + 1;
    }
#pragma unroll
    for (int k = 0; k < AS_IPT; ++k)
      if (b[k] <= (uint32_t)nb) atomicAdd(&hrow[b[k]], 1u);
#pragma unroll
    for (int k = 0; k < AS_IPT; ++k) {
      const int64_t i = base + k * BT + threadIdx.x;
      if (i < n) bins[i] = b[k];
    }
    if (MOM) {
#pragma unroll
      for (int q = 0; q < AS_MAXM; ++q) {  // unrolled: fs's fields are kernel-argument scalars
        if (q >= fs.nm) break;
        const int col = fs.col[q], fq = fs.f[q], wq = fs.w[q];
        double *aq = acc + (int64_t)q * nb;
        mom_add<AS_IPT>(aq, fs.op[q], col, fq, wq, b, v, wv, (uint32_t)nb);
      }
    }
  }
  __syncthreads();
  if (MOM) {
    double *dst = slab + (int64_t)blockIdx.x * macc;
    for (int k = threadIdx.x; k < macc; k += BT) dst[k] = acc[k];
  }
  if (tile_hist) {  // RADIX > nb: thread d < RADIX owns digit d
    const int d = threadIdx.x;
    if (d < RADIX) {
      uint32_t tot = 0;
      for (uint32_t t = t0; t < t1; ++t) {
        const uint32_t c = th[t - t0][d];
        tile_hist[(int64_t)d * ntiles + t] = c;
        tot += c;
      }
      if (d <= nb) cnt[d] = tot;
    }
    __syncthreads();
  }
  if (counts)  // (null: the caller derives the counts from the scanned tile_hist)
    for (int k = threadIdx.x; k < nb; k += BT)
      if (cnt[k]) atomicAdd(&counts[k], (unsigned long long)cnt[k]);
}

template <bool MOM>
static void launch_assign(uint32_t blocks, size_t lds, hipStream_t st, const double *x, int64_t n,
                          const double *edges, int nb, uint32_t *bins,
                          unsigned long long *counts, uint32_t *tile_hist, uint32_t ntiles,
                          uint32_t tpbk, const int64_t *n_dev, const double *wsel,
                          const FusedStats &fs, double *slab) {
  const bool wl = MOM && wsel;
  const bool wide = tpbk == 1 && ntiles < 1024;  // few tiles: 1024-thread blocks
  auto go = [&](auto kern, int bt) {
    hipLaunchKernelGGL(kern, dim3(blocks), dim3(bt), lds, st, x, n, edges, nb, bins, counts,
                       tile_hist, ntiles, tpbk, n_dev, wsel, fs, slab);
  };
  if (wide) {
    if ((nb + 1) <= LDS_EDGES) {
      if (wl) go(assign_bins<MOM, true, true, 1024>, 1024);
      else go(assign_bins<MOM, true, false, 1024>, 1024);
    } else {
      if (wl) go(assign_bins<MOM, false, true, 1024>, 1024);
      else go(assign_bins<MOM, false, false, 1024>, 1024);
    }
  } else if ((nb + 1) <= LDS_EDGES) {
    if (wl) go(assign_bins<MOM, true, true, TPB>, TPB);
    else go(assign_bins<MOM, true, false, TPB>, TPB);
  } else {
    if (wl) go(assign_bins<MOM, false, true, TPB>, TPB);
    else go(assign_bins<MOM, false, false, TPB>, TPB);
  }
}

// ------------------------------------- assignment over a lazy selection
// The one-sync radial path (pbx_profile_radial_equaln) keeps the selection
// lazy: x compacted, one keep word per 64 particles and each tile's output
// offset.  Assignment and the CSR pass then walk the SELECTION's tiles
// (4096 particles of the families' span each): a lane finds its kept
// particles' compacted positions from the keep words, reads x there and the
// caller's masses at the particle itself (coalesced), so no weight / index
// array is written or read.  Per-tile bin counts ([bin][tile], bins < 256)
// are the CSR pass's histogram; the per-bin sums go to one slab row per
// block (fixed-order final sum in fused_pack).
template <bool MOM, bool LDSE, int BT>
__global__ void __launch_bounds__(BT)
    assign_sel(const double *__restrict__ x, const uint64_t *__restrict__ kw,
               const uint32_t *__restrict__ toff, int64_t base, uint32_t ntiles, uint32_t tpbk,
               const double *__restrict__ mass, const double *__restrict__ edges, int nb,
               uint32_t *__restrict__ bins, uint32_t *__restrict__ tile_hist, FusedStats fs,
               double *__restrict__ slab, int xtiled) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  __shared__ uint32_t th[AS_TILES][RADIX];
  const int macc = MOM ? fs.nm * nb : 0;
  double *acc = (double *)smem;
  double *e = acc + macc;
  constexpr int NW = BT / 64;
  if (MOM)
    for (int k = threadIdx.x; k < macc; k += BT) acc[k] = 0.0;
  if (LDSE)
    for (int k = threadIdx.x; k <= nb; k += BT) e[k] = edges[k];
  for (int k = threadIdx.x; k < AS_TILES * RADIX; k += BT) (&th[0][0])[k] = 0;
  __syncthreads();
  const uint32_t t0 = blockIdx.x * tpbk;
  const uint32_t t1 = min(ntiles, t0 + tpbk);
  const int w = threadIdx.x >> 6;
  const uint32_t lane = lane_id();
  const bool wneed = MOM && mass;
#ifndef PBX_AS_CH
#define PBX_AS_CH 4
#endif
  constexpr int CH = PBX_AS_CH;  // words (64-particle groups) per chunk: CH items per lane
  // every wave streams whole tiles on its own (no block barrier per tile):
  // the tile's 64 keep words, one per lane, scanned across the wave; chunk
  // c + 1's loads are in flight while chunk c is binned
  // G waves share a tile (all of the block's when it has a single tile:
  // small inputs still put every wave to work), each taking (64 / CH) / G
  // consecutive chunks
  const int G = (t1 - t0 <= 1) ? NW : 1;
  const int c0 = (w % G) * ((64 / CH) / G), c1 = c0 + (64 / CH) / G;
  for (uint32_t t = t0 + w / G; t < t1; t += NW / G) {
    const uint64_t word = kw[(int64_t)t * 64 + lane];
    const uint32_t cw = (uint32_t)__popcll(word);
    uint32_t incl = cw;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const uint32_t y = __shfl_up(incl, o, 64);
      if (lane >= (uint32_t)o) incl += y;
    }
    const uint32_t pre = toff[t] + incl - cw;
    // x of a tiled selection sits in the tile's particle slots
    const double *xt = xtiled ? x + (int64_t)t * TILE : x;
    const int64_t dflt = xtiled ? 0 : (int64_t)toff[t];
    const int64_t pbase = base + (int64_t)t * TILE + lane;
    uint32_t *hrow = th[t - t0];
    double nv[CH], nw[CH];
    uint32_t npos[CH], nkeep = 0;
    auto load = [&](int c, double *v, double *wv, uint32_t *pos, uint32_t &keep) {
      keep = 0;
#pragma unroll
      for (int kk = 0; kk < CH; ++kk) {
        const int j = c * CH + kk;
        const uint64_t wj = __shfl(word, j, 64);
        const uint32_t pj = (uint32_t)__shfl((int)pre, j, 64);
        const bool kp = (wj >> lane) & 1ull;
        keep |= (uint32_t)kp << kk;
        pos[kk] = pj + rank_below(wj);
        v[kk] = xtiled ? xt[64 * j + lane] : xt[kp ? pos[kk] : dflt];  // unconditional loads
        const double mv = (wneed ? mass : xt)[(kp && wneed) ? pbase + 64 * j : (wneed ? base : dflt)];
        wv[kk] = wneed ? mv : 1.0;
      }
    };
    load(c0, nv, nw, npos, nkeep);
#pragma unroll 1
    for (int c = c0; c < c1; ++c) {
      double v[CH], wv[CH];
      uint32_t pos[CH], keep = nkeep;
#pragma unroll
      for (int kk = 0; kk < CH; ++kk) {
        v[kk] = nv[kk];
        wv[kk] = nw[kk];
        pos[kk] = npos[kk];
      }
      if (c + 1 < c1) load(c + 1, nv, nw, npos, nkeep);
      uint32_t b[CH];
#pragma unroll
      for (int kk = 0; kk < CH; ++kk)
        b[kk] = ((keep >> kk) & 1u) ? (LDSE ? bin_of(v[kk], e, nb) : bin_of(v[kk], edges, nb))
                                    : (uint32_t)nb + 1;
#pragma unroll
      for (int kk = 0; kk < CH; ++kk)
        if (b[kk] <= (uint32_t)nb) atomicAdd(&hrow[b[kk]], 1u);
#pragma unroll
      for (int kk = 0; kk < CH; ++kk)
        if ((keep >> kk) & 1u) bins[pos[kk]] = b[kk];
      if (MOM) {
#pragma unroll
        for (int q = 0; q < AS_MAXM; ++q) {  // unrolled: fs's fields are kernel-argument scalars
          if (q >= fs.nm) break;
          const int col = fs.col[q], fq = fs.f[q], wq = fs.w[q];
          double *aq = acc + (int64_t)q * nb;
          mom_add<CH>(aq, fs.op[q], col, fq, wq, b, v, wv, (uint32_t)nb);
        }
      }
    }
  }
  __syncthreads();
  if (MOM) {
    double *dst = slab + (int64_t)blockIdx.x * macc;
    for (int k = threadIdx.x; k < macc; k += BT) dst[k] = acc[k];
  }
  const int d = threadIdx.x;  // thread d < RADIX owns digit d
  if (d < RADIX)
    for (uint32_t t = t0; t < t1; ++t) tile_hist[(int64_t)d * ntiles + t] = th[t - t0][d];
}

// ------------------------------ assignment fused with the level-0 gather
// Tiled (large) selections: after the level-0 resolve ONE more read of x
// both gathers the keys of the chosen level-0 buckets (fused_gather's job)
// and assigns every other kept particle.  The edges' level-0 digits are
// known (R[q].prefix, non-decreasing in q), so a key whose digit holds no
// edge lies strictly between the edges of smaller and of larger digits: its
// bin is #{q : digit_q < digit} - 1 (bins.py:368-379, searchsorted - 1;
// neither extremum can equal it; < 0 or >= nb -> invalid), a per-digit
// table (lut).  A key in a digit that does hold edges (a group's) goes to
// the group's segment (for fused_finish) and, with its weight and position,
// to this block's list of deferred keys (fix_deferred bins them once the
// edges are known, block by block, so its writes stay inside the block's
// own tiles).  NaN keys are binned like the others (bin_of's NaN rule: the
// bin below the first NaN edge, else dropped).  Blocks walk fused_hist0's tile
// ranges (tile_range), so block b fills exactly the segment slots fused_resolve
// gave it, and its list lies at the exclusive sum of the earlier blocks'
// gathered counts (bcnt).  Bins are bytes (nb < 256; invalid = nb).
// Per-tile counts for the CSR pass ([bin][tile], nb + 1 rows) stay in LDS
// for up to AG_TR tiles and leave as contiguous row pieces; per-bin sums:
// one slab row per block.
struct GatherOut {
  uint64_t *seg;          // key - window base, by segment slot
  AgRec *rec;             // deferred keys, block by block
  const uint32_t *bcnt;   // per block: keys gathered (fused_resolve)
  uint32_t *rbase, *rn;   // per block: list start, deferred keys written
};

// exclusive sum of v[0 .. k) over a block (k <= blockDim.x)
__device__ __forceinline__ uint32_t block_prefix(const uint32_t *__restrict__ v, int k,
                                                 uint32_t *red) {
  uint32_t x = (int)threadIdx.x < k ? v[threadIdx.x] : 0u;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) x += __shfl_xor(x, o, 64);
  if (lane_id() == 0) red[threadIdx.x >> 6] = x;
  __syncthreads();
  uint32_t t = 0;
  for (int w = 0; w < (int)(blockDim.x >> 6); ++w) t += red[w];
  return t;
}

// The speculative assignment's hand-over (select_tiles<FAM, true>): on a hit
// (ctl->spec & SPEC_HIT) assign_hit only moves the select blocks' deferred
// keys into their groups' segments and sums their slab rows; on a miss
// assign_tiles assigns as below and (block 0) stores the table for the next
// call.  The host launches both in a speculating call; each returns at once
// unless the call is its case.
constexpr int AG_HU = 4;  // assign_hit: records per thread in flight
struct SpecIO {
  SpecTab *tab;            // written by block 0 of a full assignment
  AgRec *srec;             // select blocks' deferred lists (their groups filled in) ...
  const uint32_t *srbase, *srn;
  const double *sslab;     // ... and per-bin sums (SH_K rows per assign block)
};

// assign_tiles' decomposition: with the level-0 hint (select_tiles counted
// the digits, rows per select block) workgroup 1 + j walks select block j's
// tiles (part j % SH_K of level-0 block 1 + j / SH_K's range, tile_range)
// with the segment offsets fused_resolve gave it; without (fused_hist0 read
// x, rows per level-0 block) workgroup 1 + SH_K (ab - 1) walks level-0 block
// ab's whole range and the others return (the rare path: a key escaped the
// hint).  Block 0 writes the table.  Slot counters and the deferred list's
// count in LDS, like the whole-block kernel it replaced.
constexpr int AT_BT = 512;
constexpr int AT_H = SH_K;
constexpr int AT_TR = 16;                // tiles whose [tile][bin] counts stay in LDS
constexpr int AT_SL = TILE / AT_BT;      // slots per lane of a tile (8)
constexpr int AT_HS = AT_SL / 2;         // ... taken in two halves
static_assert(AT_SL == 8 && TILE / 64 == 64, "a wave takes 8 keep words of a tile");

template <bool MOM>
__global__ void __launch_bounds__(MS0_TPB)
    assign_hit(const FusedCtl *__restrict__ ctl, const uint32_t *__restrict__ gdig,
               const uint32_t *__restrict__ boff, int nb, FusedStats fs, double *__restrict__ slab,
               GatherOut go, SpecIO sio) {
  __shared__ uint16_t dtab[MS0_DIG];
  __shared__ uint32_t sslot[RADIX];
  __shared__ int c_ng, c_s, c_hit;
  const int tid = threadIdx.x;
  if (tid == 0) {
    c_hit = (ctl->spec & SPEC_HIT) ? 1 : 0;
    c_ng = (ctl->err & 2) ? 0 : ctl->ng;
    c_s = ctl->s0;
  }
  __syncthreads();
  if (!c_hit) return;
  const int ng = c_ng;
  const int macc = MOM ? fs.nm * nb : 0;
  // (a hit is hinted: the offsets are per select block, the level-0 block's
  // SH_K select blocks' slices one contiguous run from its first one's)
  const int64_t ob = blockIdx.x >= 1 ? 1 + (int64_t)SH_K * (blockIdx.x - 1) : 0;
  for (int g = tid; g < ng; g += MS0_TPB) sslot[g] = boff[ob * MS_MAXQ + g];
  // digit -> group of the edge-holding digits (the records carry key - lo)
  for (int g = tid; g < ng; g += MS0_TPB) dtab[gdig[g]] = (uint16_t)g;
  __syncthreads();
  const int s = c_s;
  if (blockIdx.x >= 1) {  // the SH_K lists as one index range, AG_HU records in flight
    uint32_t lb[SH_K], le[SH_K], tot = 0;
#pragma unroll
    for (int l = 0; l < SH_K; ++l) {
      const uint32_t j = SH_K * (blockIdx.x - 1) + l;
      lb[l] = sio.srbase[j] - tot;  // record of list l at index i: lb[l] + i
      tot += sio.srn[j];
      le[l] = tot;
    }
    for (uint32_t i0 = 0; i0 < tot; i0 += MS0_TPB * AG_HU) {
      AgRec *rp[AG_HU];
      uint64_t off[AG_HU];
#pragma unroll
      for (int u = 0; u < AG_HU; ++u) {
        const uint32_t i = i0 + u * MS0_TPB + tid;
        const uint32_t ii = i < tot ? i : 0u;
        uint32_t base = lb[SH_K - 1];
#pragma unroll
        for (int l = SH_K - 2; l >= 0; --l) base = ii < le[l] ? lb[l] : base;
        rp[u] = sio.srec + base + ii;
        off[u] = rp[u]->off;
      }
#pragma unroll
      for (int u = 0; u < AG_HU; ++u) {
        if (i0 + u * MS0_TPB + tid >= tot) break;
        const uint32_t g = dtab[(uint32_t)(off[u] >> s)];
        go.seg[atomicAdd(&sslot[g], 1u)] = off[u];
        rp[u]->tg |= g << AG_TBITS;  // (fix_deferred reads the group)
      }
    }
  }
  if (MOM) {  // this block's row: its SH_K select blocks' sums; assign_tiles' extra rows zero
    double *dst = slab + (int64_t)blockIdx.x * macc;
    for (int k = tid; k < macc; k += MS0_TPB) {
      double v = 0.0;
      if (blockIdx.x >= 1)
        for (uint32_t j = SH_K * (blockIdx.x - 1); j < SH_K * blockIdx.x; ++j)
          v += sio.sslab[(int64_t)j * macc + k];
      dst[k] = v;
    }
    if (blockIdx.x >= 1) {
      double *ex = slab + ((int64_t)gridDim.x + (int64_t)(blockIdx.x - 1) * (AT_H - 1)) * macc;
      for (int k = tid; k < (AT_H - 1) * macc; k += MS0_TPB) ex[k] = 0.0;
    }
  }
}

// The full assignment of a tiled selection (see the section comment above):
// every kept slot's x, mass and keep bit once, each key's bin from a byte
// per level-0 digit (the SpecTab encoding: bin, or for an edge-holding digit
// 128 + group when nb <= 128, else 0xff and the group searched), the [tile]
// [bin] counts of the CSR pass and the per-bin sums in LDS, the keys of
// edge-holding digits into their group's segment and the assign block's
// deferred list.  512-thread workgroups, four per assign block (<= 64 VGPRs,
// ~27 KB of LDS at 128 bins: 8 waves per SIMD) — the previous kernel ran one
// 1024-thread workgroup per assign block at 124 VGPRs (4 waves per SIMD,
// 43 % of wave time parked on waits).  MM: the sums' form — 1 {Σw, Σx·w},
// 2 {Σw} as dedicated adds, 0 any monomials (monomial(): the same values).
template <bool MOM, int MM>
__global__ void __launch_bounds__(AT_BT) __attribute__((amdgpu_waves_per_eu(8)))
    assign_tiles(const double *__restrict__ x, const uint64_t *__restrict__ kw, int64_t base,
                 int64_t span, uint32_t nt, const double *__restrict__ mass, const FusedCtl *__restrict__ ctl,
                 uint64_t ka, uint64_t kb, const MsRank *__restrict__ R, int nq,
                 const uint32_t *__restrict__ gdig, uint32_t *__restrict__ boff, int nb,
                 uint8_t *__restrict__ bins, uint32_t *__restrict__ tile_hist, FusedStats fs,
                 double *__restrict__ slab, GatherOut go, SpecTab *__restrict__ tab, int g0) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  __shared__ uint8_t dtab[MS0_DIG];
  __shared__ uint32_t sgd[RADIX];  // the edge-holding digits (groups), ascending
  __shared__ uint32_t qd[RADIX];
  __shared__ uint32_t red[AT_BT / 64];
  __shared__ uint32_t sslot[RADIX];  // this workgroup's next slot in each group's segment
  __shared__ uint32_t dk;            // deferred keys listed
  __shared__ uint64_t c_lo;
  __shared__ int c_ng, c_s, c_win, c_w0, c_hit, c_hint;
  const int tid = threadIdx.x;
  if (tid == 0) {  // the control record: one load per block, broadcast through LDS
    const bool w0 = !(ctl->err & 2);
    c_hit = (ctl->spec & SPEC_HIT) ? 1 : 0;
    c_hint = ctl->hint ? 1 : 0;
    c_win = w0;
    c_ng = w0 ? ctl->ng : 0;
    c_lo = ctl->lo;
    c_s = ctl->s0;
    c_w0 = ctl->w0;
    dk = 0;
  }
  __syncthreads();
  if (c_hit) return;  // (assign_hit)
  const bool hinted = c_hint != 0;
  // without the hint one workgroup per level-0 block works (see above); the
  // others leave zero sums (the pack adds every workgroup's row)
  if (!hinted && blockIdx.x >= 1 && (blockIdx.x - 1u) % SH_K != 0u) {
    if (MOM)
      for (int k = tid; k < fs.nm * nb; k += AT_BT) slab[(int64_t)blockIdx.x * fs.nm * nb + k] = 0.0;
    return;
  }
  const int ng = c_ng, macc = MOM ? fs.nm * nb : 0;
  const int nr = nb + 1, nrs = nr | 1;  // th row stride odd
  double *acc = (double *)smem;
  uint32_t *th = (uint32_t *)(acc + macc);  // [tile][bin]
  const int enc = nb <= 128 ? 1 : 0;
  const uint32_t gmin = enc ? 128u : (uint32_t)SPEC_DEFER;  // bytes >= gmin: edge-holding digit
  for (int q = tid; q < nq; q += AT_BT) qd[q] = (uint32_t)R[q].prefix;
  for (int g = tid; g < ng; g += AT_BT) sgd[g] = gdig[g];
  for (int k = tid; k < macc; k += AT_BT) acc[k] = 0.0;
  for (int k = tid; k < nrs * AT_TR; k += AT_BT) th[k] = 0;
  __syncthreads();
  for (int d = tid; d < MS0_DIG; d += AT_BT) {  // #{q : digit_q < d} - 1, lower bound
    int a = 0, len = nq;
    while (len > 0) {
      const int hh = len >> 1;
      if (qd[a + hh] < (uint32_t)d) {
        a += hh + 1;
        len -= hh + 1;
      } else {
        len = hh;
      }
    }
    const int b = a - 1;
    const int e = (b < 0 || b >= nb) ? nb : b;  // (no window key has such a digit)
    dtab[d] = (uint8_t)(enc ? (e < 128 ? e : 0) : e);
  }
  __syncthreads();
  for (int g = tid; g < ng; g += AT_BT)
    dtab[sgd[g]] = enc ? (g < 127 ? (uint8_t)(128 + g) : SPEC_DEFER) : SPEC_DEFER;
  __syncthreads();
  const uint64_t lo = c_lo;
  const int s = c_s;
  if (blockIdx.x == 0) {  // (no tiles) the table for the next call's speculation
    if (tab) {
      SpecTab *T = tab;
      const bool ok = c_win && nb <= SPEC_MAXB && ng < 256;
      for (int d = tid; d < MS0_DIG / 16; d += AT_BT) ((uint4 *)T->bin)[d] = ((const uint4 *)dtab)[d];
      for (int q = tid; q < nq; q += AT_BT) T->qd[q] = qd[q];
      for (int g = tid; g < ng; g += AT_BT) T->gdig[g] = sgd[g];
      if (tid == 0) {
        T->enc = enc;
        T->edges_valid = 0;  // (fix_deferred stores this call's edges)
        T->lo = lo;
        T->s0 = s;
        T->w0 = c_w0;
        T->nb = nb;
        T->nq = nq;
        T->ng = ng;
        T->valid = ok ? 1 : 0;
      }
    }
    if (MOM)
      for (int k = tid; k < macc; k += AT_BT) slab[k] = 0.0;
    return;
  }
  // this workgroup's tiles: select block j's (part h of level-0 block ab's
  // range, tile_range over g0 blocks), or without the hint block ab's all;
  // bi: the index of its offsets, key count and list (fused_resolve's)
  const uint32_t ab = 1u + (blockIdx.x - 1u) / SH_K, h = (blockIdx.x - 1u) % SH_K;
  const uint64_t G = (uint64_t)(g0 - 1);
  const uint32_t ta0 = (uint32_t)((uint64_t)nt * (ab - 1) / G), tb0 = (uint32_t)((uint64_t)nt * ab / G);
  const uint32_t ta = hinted ? ta0 + (uint32_t)((uint64_t)(tb0 - ta0) * h / SH_K) : ta0;
  const uint32_t tb = hinted ? ta0 + (uint32_t)((uint64_t)(tb0 - ta0) * (h + 1) / SH_K) : tb0;
  const uint32_t bi = hinted ? blockIdx.x : ab;
  for (int g = tid; g < ng; g += AT_BT) sslot[g] = boff[(int64_t)bi * MS_MAXQ + g];
  // the list starts after the earlier workgroups' gathered keys
  uint32_t pre = 0;
  for (uint32_t i = (uint32_t)tid; i < bi; i += AT_BT) pre += go.bcnt[i];
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) pre += __shfl_xor(pre, o, 64);
  if (lane_id() == 0) red[tid >> 6] = pre;
  __syncthreads();
  uint32_t rb = 0;
  for (int q = 0; q < AT_BT / 64; ++q) rb += red[q];
  if (tid == 0) go.rbase[bi] = rb;
  const bool win = c_win;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const uint32_t lane = lane_id();
  const bool wneed = mass != nullptr;
  const double *mp = wneed ? mass + base : x;  // (the masses of the selection's span)
  for (uint32_t r0 = ta; r0 < tb; r0 += AT_TR) {
    const uint32_t r1 = min(tb, r0 + (uint32_t)AT_TR);
    for (uint32_t t = r0; t < r1; ++t) {
      const uint32_t tl = t - r0;
#pragma unroll
      for (int hf = 0; hf < 2; ++hf) {  // the wave's 8 keep words in two halves of 4
      const int64_t s0 = (int64_t)t * TILE + (int64_t)w * (64 * AT_SL) + hf * (64 * AT_HS);
      // the half's 4 keep words (uniform: scalar loads), 4 slots per lane
      const uint64_t *kwp = kw + (s0 >> 6);
      uint64_t kk[AT_HS];
      double xv[AT_HS], mv[AT_HS];
      // (only the span's last slots lie past its masses: the clamp for that
      // half alone, a uniform test, not a 64-bit select per slot)
      const bool past = s0 + 64 * AT_HS > span;
#pragma unroll
      for (int k = 0; k < AT_HS; ++k) {
        kk[k] = kwp[k];
        const int64_t sl = s0 + 64 * k + lane;
        xv[k] = __builtin_nontemporal_load(x + sl);
        if (wneed) mv[k] = __builtin_nontemporal_load(mp + (past ? (sl < span ? sl : span - 1) : sl));
        else mv[k] = 1.0;
      }
      uint32_t c[AT_HS];
      uint64_t key[AT_HS];
      uint32_t kp8 = 0, inw8 = 0;
#pragma unroll
      for (int k = 0; k < AT_HS; ++k) {  // every lookup issued before any is used
        const bool kp = (kk[k] >> lane) & 1ull;
        key[k] = dkey(xv[k]);
        const bool inw = kp && win && key[k] >= ka && key[k] <= kb;
        kp8 |= (uint32_t)kp << k;
        inw8 |= (uint32_t)inw << k;
        c[k] = dtab[inw ? (uint32_t)((key[k] - lo) >> s) : 0u];
      }
      uint32_t defm = 0;
#pragma unroll
      for (int k = 0; k < AT_HS; ++k) {
        if (!((kp8 >> k) & 1u)) continue;
        const bool inw = (inw8 >> k) & 1u;
        if (inw && c[k] >= gmin) {
          defm |= 1u << k;
          continue;
        }
        const uint32_t bk = inw ? c[k] : (uint32_t)nb;  // outside the window: dropped
        bins[s0 + 64 * k + lane] = (uint8_t)bk;
        atomicAdd(&th[tl * nrs + bk], 1u);
        if (MOM && bk < (uint32_t)nb) {
          if (MM == 1) {
            atomicAdd(&acc[bk], mv[k]);
            atomicAdd(&acc[nb + bk], xv[k] * mv[k]);
          } else if (MM == 2) {
            atomicAdd(&acc[bk], mv[k]);
          } else {
#pragma unroll
            for (int q = 0; q < AS_MAXM; ++q) {  // unrolled: fs's fields are kernel-argument scalars
              if (q >= fs.nm) break;
              const double f = fs.f[q] == 0 ? xv[k] : mv[k];
              const double ww = fs.w[q] == 0 ? xv[k] : mv[k];
              atomicAdd(&acc[q * nb + bk], monomial(fs.col[q], f, ww));
            }
          }
        }
      }
      if (__ballot(defm != 0u)) {  // the keys of edge-holding digits (~3 % of them)
        // the half's list slots with ONE LDS atomic, and every key's segment
        // slot issued before any is used: two LDS round trips per half, not
        // two per key word (a wave half almost always holds one such key)
        uint64_t bd[AT_HS];
        uint32_t before[AT_HS], tot = 0;
#pragma unroll
        for (int k = 0; k < AT_HS; ++k) {
          bd[k] = __ballot((defm >> k) & 1u);
          before[k] = tot;
          tot += (uint32_t)__popcll(bd[k]);
        }
        uint32_t li0 = 0;
        if (lane == 0) li0 = atomicAdd(&dk, tot);
        uint32_t g[AT_HS], sl[AT_HS];
#pragma unroll
        for (int k = 0; k < AT_HS; ++k) {
          g[k] = 0;
          sl[k] = 0;
          if ((defm >> k) & 1u) {
            if (c[k] != SPEC_DEFER) {
              g[k] = c[k] - 128u;
            } else {  // search the group by its digit
              const uint32_t dd = (uint32_t)((key[k] - lo) >> s);
              int l = 0, hh = ng - 1;
              while (l < hh) {
                const int mid = (l + hh) >> 1;
                if (sgd[mid] < dd) l = mid + 1; else hh = mid;
              }
              g[k] = (uint32_t)l;
            }
            sl[k] = atomicAdd(&sslot[g[k]], 1u);
          }
        }
        li0 = __shfl(li0, 0, 64);
#pragma unroll
        for (int k = 0; k < AT_HS; ++k) {
          if ((defm >> k) & 1u) {
            const uint64_t off = key[k] - lo;
            go.seg[sl[k]] = off;
            const uint32_t slot = (uint32_t)(s0 + 64 * k) + lane;
            go.rec[rb + li0 + before[k] + rank_below(bd[k])] =
                AgRec{off, mv[k], slot, t | (g[k] << AG_TBITS)};
          }
        }
      }
      }
    }
    __syncthreads();
    const int nrt = (int)(r1 - r0);
    for (int k = tid; k < nr * nrt; k += AT_BT) {
      const int b = k / nrt, tl = k - b * nrt;
      tile_hist[(int64_t)b * nt + r0 + tl] = th[tl * nrs + b];
    }
    __syncthreads();
    for (int k = tid; k < nrs * AT_TR; k += AT_BT) th[k] = 0;
    __syncthreads();
  }
  if (tid == 0) go.rn[bi] = dk;
  if (MOM) {
    double *dst = slab + (int64_t)blockIdx.x * macc;
    for (int k = tid; k < macc; k += AT_BT) dst[k] = acc[k];
  }
}

// A speculating selection stored no x and its call missed with the level-0
// hint held (fused_hist0 did not rebuild it): x of every tile, from the
// positions, before assign_tiles reads it (every block returns at once
// otherwise)
__global__ void __launch_bounds__(TPB)
    xsrc_miss(const FusedCtl *__restrict__ ctl, XSrc xs, uint32_t nt, uint32_t tiles_per_block) {
  __shared__ int c_x;
  if (threadIdx.x == 0)
    c_x = ((ctl->spec & SPEC_NOX) && !(ctl->spec & SPEC_HIT) && ctl->hint) ? 1 : 0;
  __syncthreads();
  if (!c_x) return;
  const uint32_t ta = blockIdx.x * tiles_per_block;
  xsrc_tiles(xs, ta, min(nt, ta + tiles_per_block));
}

// The deferred keys' bins once fused_finish has the edges (the ~1-3 % of
// the kept particles whose level-0 digit holds an edge): block b takes
// assign_gather block b's list, so its byte stores and [bin][tile] counts
// stay inside that block's tiles.  A key of group g lies above every edge of
// an earlier group and below every edge of a later one, so its lower bound
// is searched among the group's own ranks gq[g] .. gq[g + 1] only (usually
// one or two edges, not an 8-step dependent LDS chain over all of them).
// The [tile][bin] counts are kept in LDS for a window of the block's tiles
// at a time (a pass over the list per window: one pass up to FD_LDSW / (nb + 1)
// tiles, i.e. up to ~1G particles at 129 bins) — global atomics on scattered
// (bin, tile) words ran at ~0.1 of LDS speed (256M: 203 us).
// (A block's list mixes all groups, so a wave's keys spread over many bins:
// plain LDS atomics; a per-distinct-bin wave reduction — dependent
// ds_bpermute chains — took 316 us at 64M.)
constexpr int FD_U = 4;          // keys per thread in flight
constexpr int FD_LDSW = 28672;   // LDS words for the block's [tile][bin] counts (112 KB)

template <bool MOM>
__global__ void __launch_bounds__(MS0_TPB)
    fix_deferred(const FusedCtl *__restrict__ ctl, const AgRec *__restrict__ rec,
                 const uint32_t *__restrict__ rbase, const uint32_t *__restrict__ rn,
                 const double *__restrict__ edges, const uint32_t *__restrict__ gq, int nb,
                 uint8_t *__restrict__ bins, uint32_t *__restrict__ tile_hist, uint32_t nt,
                 FusedStats fs, double *__restrict__ slab, SpecIO sio) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  __shared__ uint32_t gql[MS_MAXQ + 1];  // the groups' first ranks (gq), ng + 1 of them
  const int macc = MOM ? fs.nm * nb : 0;
  double *acc = (double *)smem;
  double *e = acc + macc;
  uint32_t *tc = (uint32_t *)(e + nb + 1);  // [window tile][bin]
  const int tid = threadIdx.x;
  const int nrs = (nb + 1) | 1;
  uint32_t ta, tb;
  tile_range(nt, ta, tb);
  const uint32_t wt = (uint32_t)(FD_LDSW / nrs);  // tiles per window
  __shared__ uint64_t c_lo;  // the control record's fields, one load per block
  __shared__ int c_ng, c_hit, c_edge, c_hint;  // (c_ng -1: no window)
  if (tid == 0) {
    const bool ok = !(ctl->err & 2);
    c_ng = ok ? ctl->ng : -1;
    c_lo = ctl->lo;
    c_hit = (ctl->spec & SPEC_HIT) ? 1 : 0;
    c_edge = (ctl->spec & SPEC_EDGE) ? 1 : 0;
    c_hint = ctl->hint ? 1 : 0;
  }
  __syncthreads();
  // an edge hit: no deferred keys, and the table keeps its edges (the pack
  // reads no fix_deferred sums either)
  if (c_edge) return;
  for (int k = tid; k < macc; k += MS0_TPB) acc[k] = 0.0;
  for (int k = tid; k <= nb; k += MS0_TPB) e[k] = edges[k];
  __syncthreads();
  const bool ok_all = c_ng >= 0;
  for (int k = tid; k <= c_ng; k += MS0_TPB) gql[k] = gq[k];
  const uint64_t lo = c_lo;
  if (blockIdx.x == 0 && sio.tab && ok_all) {
    // the table now holds this call's digits: its edges and groups with it
    // (the next call's edge speculation)
    SpecTab *T = sio.tab;
    __shared__ int s_fin;
    if (tid == 0) s_fin = 1;
    __syncthreads();
    for (int q = tid; q <= nb; q += MS0_TPB) {
      const double v = edges[q];
      T->edges[q] = v;
      if (!(v - v == 0.0)) s_fin = 0;  // (NaN / inf edges: no edge speculation)
    }
    for (int k = tid; k <= c_ng; k += MS0_TPB) T->gq[k] = gq[k];
    __syncthreads();
    if (tid == 0) T->edges_valid = s_fin;
  }
  // this block's deferred keys (keys of its own tiles): on a speculation hit
  // the lists of its SH_K select blocks; else assign_tiles' lists — one per
  // select block with the level-0 hint, one for the block without
  const bool hit = c_hit != 0;
  const int nl = blockIdx.x == 0 ? 0 : (hit || c_hint) ? SH_K : 1;
  int64_t lb[SH_K], lc[SH_K];
  int64_t cnt_all = 0;
#pragma unroll
  for (int l = 0; l < SH_K; ++l) {
    lb[l] = 0;
    lc[l] = 0;
    if (l < nl && ok_all) {
      const uint32_t j = hit ? SH_K * (blockIdx.x - 1) + l
                             : (c_hint ? 1 + SH_K * (blockIdx.x - 1) + l : blockIdx.x);
      lb[l] = hit ? sio.srbase[j] : rbase[j];
      lc[l] = hit ? sio.srn[j] : rn[j];
      cnt_all += lc[l];
    }
  }
  const AgRec *lr = hit ? sio.srec : rec;
  for (uint32_t w0 = ta; w0 < tb || (w0 == ta && cnt_all); w0 += wt) {  // (block-uniform)
    const uint32_t w1 = min(tb, w0 + wt);
    for (int k = tid; k < (int)(w1 - w0) * nrs; k += MS0_TPB) tc[k] = 0;
    __syncthreads();
    const bool first = w0 == ta;  // bytes and sums on the first pass only
    for (int l = 0; l < nl; ++l) {
      const int64_t r0 = lb[l], cnt = lc[l];
      for (int64_t i0 = 0; i0 < cnt; i0 += (int64_t)MS0_TPB * FD_U) {
        AgRec r[FD_U];
#pragma unroll
        for (int u = 0; u < FD_U; ++u) {
          const int64_t i = i0 + u * MS0_TPB + tid;
          r[u] = lr[r0 + (i < cnt ? i : 0)];  // unconditional loads
        }
#pragma unroll
        for (int u = 0; u < FD_U; ++u) {
          const int64_t i = i0 + u * MS0_TPB + tid;
          const double v = dkey_inv(lo + r[u].off);
          const bool ok = i < cnt;
          const uint32_t t = r[u].tg & ((1u << AG_TBITS) - 1), g = r[u].tg >> AG_TBITS;
          const uint32_t b = ok ? bin_of_in(v, e, nb, (int)gql[g], (int)gql[g + 1]) : (uint32_t)nb;
          if (ok) {
            if (first) bins[r[u].pos] = (uint8_t)b;
            if (t >= w0 && t < w1) atomicAdd(&tc[(t - w0) * nrs + b], 1u);
          }
          if (MOM && first && ok && b < (uint32_t)nb)
#pragma unroll
            for (int q = 0; q < AS_MAXM; ++q) {  // unrolled: fs's fields are kernel-argument scalars
              if (q >= fs.nm) break;
              const double f = fs.f[q] == 0 ? v : r[u].w;
              const double ww = fs.w[q] == 0 ? v : r[u].w;
              atomicAdd(&acc[q * nb + b], monomial(fs.col[q], f, ww));
            }
        }
      }
    }
    __syncthreads();
    for (int k = tid; k < (int)(w1 - w0) * (nb + 1); k += MS0_TPB) {  // the block owns these columns
      const int b = k / (int)(w1 - w0), tl = k - b * (int)(w1 - w0);
      const uint32_t c = tc[tl * nrs + b];
      if (c) tile_hist[(int64_t)b * nt + w0 + tl] += c;
    }
    if (w1 >= tb) break;
    __syncthreads();
  }
  if (MOM) {
    __syncthreads();
    double *dst = slab + (int64_t)blockIdx.x * macc;
    for (int k2 = tid; k2 < macc; k2 += MS0_TPB) dst[k2] = acc[k2];
  }
}

// Stable CSR scatter over a lazy selection's tiles: radix_scatter's scheme
// (per-wave peer ranks, tile sorted by bin in LDS, runs written out
// coalesced) with the elements = the tile's kept particles in particle
// order, key = bin, value = compacted position.  offs = the exclusive scan
// of assign_sel's [bin][tile] counts (nrows rows: the digits that occur).
// A tile's kept particles are the contiguous compacted positions
// [toff[t], toff[t + 1]) in particle order, so the pass walks those
// positions directly (element e = w * 1024 + k * 64 + lane: (wave,
// iteration, lane) = position order); the tile's offsets are loaded first,
// beside the bins.  LDS holds the digit (byte) and the in-tile position
// (u16) of each element.
template <typename BT>  // bins: uint32_t, or bytes (assign_gather)
__global__ void __launch_bounds__(TPB)
    csr_sel(const uint32_t *__restrict__ toff, const int64_t *__restrict__ n_dev,
            const BT *__restrict__ bins, const uint32_t *__restrict__ offs, uint32_t ntiles,
            int32_t *__restrict__ perm, uint32_t nrows) {
  __shared__ uint32_t run[NWAVE][RADIX];
  __shared__ uint32_t dstart[RADIX];
  __shared__ uint32_t gofs[RADIX];
  __shared__ uint32_t wsum[NWAVE];
  __shared__ uint8_t sk[TILE];
  __shared__ __attribute__((aligned(16))) uint16_t sv[TILE];  // (first: the ranks' peer words)
  uint64_t *pmask = (uint64_t *)sv;
  const int w = threadIdx.x >> 6;
  const uint32_t lane = lane_id();
  const uint32_t t = blockIdx.x;
  const uint32_t o = toff[t];
  const uint32_t tn = (t + 1 < ntiles ? toff[t + 1] : (uint32_t)*n_dev) - o;
  const int d0 = threadIdx.x;  // TPB == RADIX
  const uint32_t go = (uint32_t)d0 < nrows ? offs[(int64_t)d0 * ntiles + t] : 0u;
  for (int d = threadIdx.x; d < NWAVE * RADIX; d += TPB) {
    (&run[0][0])[d] = 0;
    pmask[d] = 0ull;
  }
  uint32_t key[16];
  uint64_t okm[16];
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    const uint32_t e = (uint32_t)(w * 1024 + k * 64) + lane;
    const bool ok = e < tn;
    okm[k] = __ballot(ok);
    key[k] = (uint32_t)bins[o + (ok ? e : 0u)];  // unconditional (o: this tile's or the next's first)
  }
  __syncthreads();
  uint32_t lp[16];
  {
    uint32_t dg[16];
    bool okk[16];
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      okk[k] = (okm[k] >> lane) & 1ull;
      dg[k] = key[k] & 255u;
    }
    wave_ranks_lds<16>(dg, okk, &run[w][0], pmask + w * RADIX, lp);
  }
  __syncthreads();
  {
    uint32_t tot = 0;
#pragma unroll
    for (int ww = 0; ww < NWAVE; ++ww) tot += run[ww][d0];
    const uint32_t st = block_excl_scan(tot, wsum, nullptr);
    dstart[d0] = st;
    gofs[d0] = go;
    uint32_t a = st;
#pragma unroll
    for (int ww = 0; ww < NWAVE; ++ww) {
      const uint32_t c = run[ww][d0];
      run[ww][d0] = a;
      a += c;
    }
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    if ((okm[k] >> lane) & 1ull) {
      const uint32_t dgt = key[k] & 255u;
      const uint32_t q = run[w][dgt] + lp[k];
      sk[q] = (uint8_t)dgt;
      sv[q] = (uint16_t)(w * 1024 + k * 64 + lane);
    }
  }
  __syncthreads();
  for (int j = threadIdx.x; j < (int)tn; j += TPB) {
    const uint32_t dgt = sk[j];
    perm[gofs[dgt] + ((uint32_t)j - dstart[dgt])] = (int32_t)(o + sv[j]);
  }
}

// Stable CSR scatter over a tiled selection's particle slots (assign_gather
// bytes): csr_sel's scheme with element e = slot (wave, iteration, lane) =
// particle order, valid iff its keep bit is set (keep words loaded up front
// into SGPRs: every load address is known at launch), value = the selection
// index toff[t] + kpre + rank in the word.  Wave-local stable ranks from LDS
// (prims.h wave_ranks_lds: ~12 VALU + 5 LDS instructions per 64 slots
// instead of peers8's ~85 VALU, which made this pass VALU-bound, 105.5 ->
// 90.6 us at 64M), the tile sorted by bin in LDS and written out run by run
// (coalesced; storing each element at its CSR position directly was 194 vs
// 128 us).  Tiles are XCD-contiguous (xcd_swizzle: a (bin, tile) run's
// output lines shared with the next tile's run, and the [bin][tile] offset
// words 16 tiles share, stay in one L2).
// pack / npk: the step's results pack (fused_pack's work, PackArgs) rides in
// the first npk blocks, before their tile — one launch less per step.
__global__ void __launch_bounds__(TPB)
    csr_slots(const uint32_t *__restrict__ toff, const uint64_t *__restrict__ kw,
              const uint16_t *__restrict__ kpre, const uint32_t *__restrict__ wcnt,
              const uint8_t *__restrict__ bins, const uint32_t *__restrict__ offs,
              uint32_t ntiles, int32_t *__restrict__ perm, uint32_t nrows, PackArgs pack,
              int npk) {
  __shared__ uint32_t run[NWAVE][RADIX];
  __shared__ uint32_t delta[RADIX];  // a digit's run: global offset - its start in the sorted tile
  __shared__ uint32_t wsum[NWAVE];
  // the tile sorted by bin, one word per element: digit << 16 | in-tile
  // position (one LDS write per element when sorting, one read when writing
  // out — a byte array and a u16 array took two of each, and the out pass
  // read the digit's offset and start separately: ~48 fewer LDS
  // instructions per thread); during the ranking the [NWAVE][RADIX] peer
  // words, before both the pack's reduction buffer (TPB doubles)
  __shared__ __attribute__((aligned(16))) uint32_t sw[TILE];
  static_assert(sizeof(uint32_t) * TILE >= sizeof(uint64_t) * NWAVE * RADIX, "pmask aliases sw");
  static_assert(sizeof(uint32_t) * TILE >= sizeof(double) * TPB, "the pack's buffer fits sw");
  uint64_t *pmask = (uint64_t *)sw;
  if ((int)blockIdx.x < npk) {
    pack_block(pack, (int)blockIdx.x, (double *)sw);
    __syncthreads();
  }
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);  // keep words: scalar loads
  const uint32_t lane = lane_id();
  const uint32_t t = xcd_swizzle(blockIdx.x, gridDim.x);
  const int d0 = threadIdx.x;  // TPB == RADIX
  const uint32_t dr = (uint32_t)d0 < nrows ? (uint32_t)d0 : nrows - 1;  // no branch around the load
  const uint32_t go0 = offs[(int64_t)dr * ntiles + t];
  const uint32_t go = (uint32_t)d0 < nrows ? go0 : 0u;
  const uint8_t *bt = bins + (int64_t)t * TILE + w * 1024 + lane;
  const uint64_t *kwt = kw + (int64_t)t * 64 + w * 16;
  const uint16_t *kpt = kpre + (int64_t)t * 64 + w * 16;
  const uint32_t o = toff[t];
  // kpre counts inside select_tiles' 512-particle wave slices: this wave's
  // 16 words are slices 2w, 2w + 1
  static_assert(SH_NW == 2 * NWAVE, "two select slices per CSR wave");
  const uint32_t *wct = wcnt + (int64_t)t * SH_NW;
  uint32_t sbase0 = 0, tn = 0;
#pragma unroll
  for (int q = 0; q < SH_NW; ++q) {
    const uint32_t c = wct[q];
    sbase0 += q < 2 * w ? c : 0u;
    tn += c;
  }
  const uint32_t sbase1 = sbase0 + wct[2 * w];
  uint64_t wds[16];  // the wave's keep words, loaded before any store
  uint32_t key[16];
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    const uint64_t v = kwt[k];
    wds[k] = ((uint64_t)__builtin_amdgcn_readfirstlane((uint32_t)(v >> 32)) << 32) |
             (uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)v);
    key[k] = bt[k * 64];  // unconditional: every slot exists
  }
  for (int d = threadIdx.x; d < NWAVE * RADIX; d += TPB) {
    (&run[0][0])[d] = 0;
    pmask[d] = 0ull;
  }
  __syncthreads();
  uint32_t lp[16];
  {
    uint32_t dg[16];
    bool okk[16];
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      okk[k] = (wds[k] >> lane) & 1ull;
      dg[k] = key[k] & 255u;
    }
    wave_ranks_lds<16>(dg, okk, &run[w][0], pmask + w * RADIX, lp);
  }
  __syncthreads();
  {
    uint32_t tot = 0;
#pragma unroll
    for (int ww = 0; ww < NWAVE; ++ww) tot += run[ww][d0];
    const uint32_t st = block_excl_scan(tot, wsum, nullptr);
    delta[d0] = go - st;  // (mod 2^32: + the sorted position is the CSR position)
    uint32_t a = st;  // tile-local sorted position
#pragma unroll
    for (int ww = 0; ww < NWAVE; ++ww) {
      const uint32_t c = run[ww][d0];
      run[ww][d0] = a;
      a += c;
    }
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    const uint64_t wd = wds[k];
    if ((wd >> lane) & 1ull) {
      const uint32_t dgt = key[k] & 255u;
      const uint32_t q = run[w][dgt] + lp[k];
      const uint32_t v = (k < 8 ? sbase0 : sbase1) + (uint32_t)kpt[k] + rank_below(wd);
      sw[q] = (dgt << 16) | v;  // (v < TILE)
    }
  }
  __syncthreads();
  for (int j = threadIdx.x; j < (int)tn; j += TPB) {
    const uint32_t e = sw[j];
    perm[delta[e >> 16] + (uint32_t)j] = (int32_t)(o + (e & 0xffffu));
  }
}

// ---------------------------- one-launch radial equaln (small selections)
// A selection of at most one tile per CU (<= MONO_MAXT tiles of 4096
// particles: ~1M) runs the whole pbx_profile_radial_equaln step as ONE
// persistent launch: block t = selection tile t (select_onepass<1024>'s
// layout, 4 particles per lane), every block resident, five grid barriers.
// A tile's particles stay in registers from the selection to the CSR
// scatter (x, mass, compacted position): the kept x is written once and
// never re-read, and the 11 dependent launches of the multi-kernel path
// (each ~5 us at this size) become phases of one.  Results are those of
// the multi-kernel path (same rank rules, same selection code, same
// stable CSR order); the per-bin sums differ by float-add order only.
//   1 select: mask, x, keep words; the tile's count and key range -> rec[t]
//   2 every block: totals, key range, window geometry (fused_ctl's rules),
//     this tile's offset; compacted x; level-0 histogram of the tile's
//     window keys in LDS, its non-zero bins added to H
//   3 every block: scan of H, each rank's level-0 digit and residual rank
//     (fused_resolve's rules), the groups; the tile's keys of chosen
//     buckets -> the group segments (one global atomic per tile and group)
//   4 block g (and g + grid, ...): group g's ranks (fused_finish) -> edges
//   5 bins (bin_of), per-bin monomial sums in LDS (one slab row per tile),
//     the tile's bin counts -> th[bin][tile], in-tile CSR ranks (csr_sel)
//   6 every block: its CSR offsets from the th table, perm scatter; block 0
//     packs ctl / edges / counts; slab columns summed in fixed order
constexpr int MONO_BT = 1024;
constexpr int MONO_NW = MONO_BT / 64;
constexpr int MONO_SI = TILE / MONO_BT;  // particles per lane
constexpr uint32_t MONO_MAXT = 256;
// level-0 digits of the one-launch path (13 bits: the histogram flush and
// H scan got 5.5 us faster, the finish of the twice larger groups 10 us
// slower at 1M)
constexpr int MONO_BITS = 14;
constexpr int MONO_DIG = 1 << MONO_BITS;
static_assert(MONO_DIG <= MS0_DIG, "the LDS arrays are MS0_DIG long");
constexpr int BAR_LINE = 16;             // u64 words per 128-B line
// lines 0-7 group counters, 8 top counter, 9 generation, 10 completions,
// 11 the call (gen0 + 1) in which a window key fell outside the hint
constexpr size_t BAR_WORDS = (size_t)BAR_LINE * 12;

// Hand-off loads / stores of the one-launch path: sc1 (relaxed agent-scope
// atomics: global_load / global_store ... sc1), so no fence is needed at a
// barrier — the measured-valid form of MI355X_MICROARCH.md's hand-off table
// (every handed-off word stored sc1 by its producer and loaded sc1 by every
// consumer; the producer waves drain vmcnt(0) before the arrival).  An
// agent-scope release writes back the whole XCD L2 (~2-6 us per wave that
// issues it): with one per wave per phase the first version spent ~40 us
// per phase in fences.
// (ld_sc1 / st_sc1 / ld_sc1d / st_sc1d: prims.h)

// Grid barrier of a co-resident grid, XCD-hierarchical: a block arrives on
// the counter of its group (block % 8, the dispatcher's XCD round robin:
// a speed hint only), the last block of a group on the top counter, and the
// last group publishes generation `gen`.  Counters are monotonic across
// calls: the host carries the generation and zeroes them when the grid size
// changes or a call failed.  Every wave drains its stores (vmcnt(0)) before
// the block's arrival; the data handed over a barrier is stored and loaded
// sc1 (ld_sc1 / st_sc1).  Bounded spin: false when the generation did not
// come (the host discards the call).
__device__ bool grid_sync(uint64_t *bar, uint64_t gen, uint32_t nblk, int *ok) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    const uint32_t g = blockIdx.x % 8, ngrp = nblk < 8 ? nblk : 8;
    const uint64_t gs = nblk / 8 + (g < nblk % 8 ? 1 : 0);
    const uint64_t old = __hip_atomic_fetch_add(bar + BAR_LINE * g, 1ull, __ATOMIC_RELAXED,
                                                __HIP_MEMORY_SCOPE_AGENT);
    if (old + 1 == gen * gs) {
      const uint64_t o2 = __hip_atomic_fetch_add(bar + BAR_LINE * 8, 1ull, __ATOMIC_RELAXED,
                                                 __HIP_MEMORY_SCOPE_AGENT);
      if (o2 + 1 == gen * ngrp) st_sc1(bar + BAR_LINE * 9, gen);
    }
    uint32_t spins = 0;
    while (ld_sc1(bar + BAR_LINE * 9) < gen) {
      if (++spins > (1u << 22)) {
        *ok = 0;
        break;
      }
      __builtin_amdgcn_s_sleep(1);
    }
  }
  __syncthreads();
  return *ok != 0;
}

// A grid_sync arrival without the wait: keeps the counters at the
// generation the host carries when a call skips a barrier it does not need
// (every block skips it: the decision is grid-uniform).
__device__ void grid_arrive(uint64_t *bar, uint64_t gen, uint32_t nblk) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    const uint32_t g = blockIdx.x % 8, ngrp = nblk < 8 ? nblk : 8;
    const uint64_t gs = nblk / 8 + (g < nblk % 8 ? 1 : 0);
    const uint64_t old = __hip_atomic_fetch_add(bar + BAR_LINE * g, 1ull, __ATOMIC_RELAXED,
                                                __HIP_MEMORY_SCOPE_AGENT);
    if (old + 1 == gen * gs) {
      const uint64_t o2 = __hip_atomic_fetch_add(bar + BAR_LINE * 8, 1ull, __ATOMIC_RELAXED,
                                                 __HIP_MEMORY_SCOPE_AGENT);
      if (o2 + 1 == gen * ngrp) st_sc1(bar + BAR_LINE * 9, gen);
    }
  }
}

struct MonoRec {  // a tile's selection result (phase 1)
  uint64_t cnt, kmin, kmax, pad;
};

struct MonoArgs {
  const double *pos;
  const double *mass;  // null: unit weights
  int64_t n_hi;        // particles [sp.base, n_hi) are tiled
  SelectParams sp;
  uint64_t ka, kb;     // equaln window keys (bins.py:734-737)
  int empty_bounds;
  int nb, nq;
  int64_t nbins;
  FusedStats fs;
  MonoRec *rec;
  uint32_t *H;      // level-0 histogram counted in phase 1 with the hint's geometry (MS0_DIG)
  uint32_t *H2;     // ... or in phase 2 with this call's own (both zero on entry and exit)
  const SelHint *hin;  // the previous call's level-0 geometry (null: none)
  SelHint *hout;       // this call's, for the next call
  uint32_t *gcnt;   // per-group segment fill (MS_MAXQ)
  uint64_t *seg;    // group segments (keys - lo)
  double *x;        // compacted kept x
  uint64_t *kw;
  uint32_t *toff;
  uint32_t *bins;
  int32_t *perm;
  double *edges;
  uint32_t *th;     // [RADIX][nt] bin counts per tile
  double *slab;     // [nt][nm * nb] per-tile monomial sums
  unsigned long long *counts;
  double *pack;     // [ctl][edges nq][counts nb][sums nm x nb][tag] (mapped host memory)
  double *stage;    // the same in device memory (sc1 stores; pack_complete copies it out)
  uint64_t *bar;
  uint64_t gen0;         // barrier generations gen0 + 1, + 2, ... (the call reports how many
                         // it used: FusedCtl::spec >> 8); tag of this call
  // edge speculation: the previous call's edges (rewritten by every call) and
  // per edge the window keys below (by upper bound) / equal, summed over the
  // blocks (zero on entry and exit); eg: speculate (the host saw them repeat)
  double *pedges;
  uint32_t *eU, *eE;
  int eg;
  uint64_t done_target;  // the completion counter's value once every block is done
  uint64_t *trace;       // PBX_MONO_TRACE diagnostic: 8 wall-clock stamps per block, or null
};

// End of a block's part of the call (pack_complete): the block whose
// completion brings the (monotonic) counter to its target copies the staged
// pack to the host pack and writes the tag.  A call in which a block gave up
// at a barrier never reaches the target: no tag, and the host discards the
// call.  The host may read the pack as soon as it sees the tag (radial_mono_run
// spins on it).  (A system-scope fence in EVERY block — an L2 write-back each
// — cost the kernel 65 -> 73 us at 1M, round 3: only the last block fences.)
__device__ void mono_done(const MonoArgs &a, int tagpos) {
  pack_complete(a.bar + BAR_LINE * 10, a.done_target, a.stage, a.pack, tagpos, tagpos, a.gen0);
}

#define MONO_STAMP(k)                                                       \
  do {                                                                      \
    if (a.trace && threadIdx.x == 0) a.trace[blockIdx.x * 8 + (k)] = wall_clock64(); \
  } while (0)
__global__ void __launch_bounds__(MONO_BT) radial_mono(MonoArgs a) {
  static_assert(MONO_SI == 4 && MONO_NW == 16, "4 particles per lane, 16 waves");
  MONO_STAMP(0);
  __shared__ __attribute__((aligned(16))) uint32_t L0[MONO_DIG];  // hist / scan; keys; th partials
  __shared__ __attribute__((aligned(16))) uint16_t L1[MONO_DIG];  // digit -> group; finish hist; runs + sums
  __shared__ int64_t q_rr[RADIX];
  __shared__ uint32_t q_dig[RADIX];
  __shared__ uint32_t g_start[RADIX + 1], g_off[RADIX + 1], g_lcnt[RADIX], g_base[RADIX];
  __shared__ double e_lds[RADIX];
  __shared__ uint32_t wcnt[MONO_NW], wsum[MONO_NW];
  __shared__ unsigned long long wmin[MONO_NW], wmax[MONO_NW];
  __shared__ uint32_t s_gofs[RADIX];
  __shared__ uint64_t pick[2];
  __shared__ FusedCtl s_ctl;
  __shared__ uint32_t s_toff;
  __shared__ int s_ok;
  const uint32_t t = blockIdx.x, nt = gridDim.x;
  const int tid = threadIdx.x, w = tid >> 6;
  const uint32_t lane = lane_id();
  const int nb = a.nb, nq = a.nq;
  __shared__ SelHint s_hint;
  __shared__ int s_hinted, s_edge;
  __shared__ uint64_t ek_l[RADIX];             // edge speculation: the previous edges' keys,
  __shared__ uint32_t eUl[RADIX + 1], eEl[RADIX];  // this block's keys by upper bound / equal
  if (tid == 0) {
    s_ok = 1;
    SelHint h{};
    if (a.hin) h = *a.hin;  // (one load per block)
    s_hint = h;
    s_edge = 0;
  }
  if (a.eg)
    for (int i = tid; i <= nq; i += MONO_BT) {
      if (i < nq) {
        ek_l[i] = dkey(a.pedges[i]);
        eEl[i] = 0;
      }
      eUl[i] = 0;
    }
  for (int i = tid; i < MONO_DIG; i += MONO_BT) L0[i] = 0;
  if (t == 0)  // zeroed here, used after barrier 1
    for (int i = tid; i < RADIX; i += MONO_BT) st_sc1(&a.gcnt[i], 0u);
  __syncthreads();
  // the previous call's level-0 geometry: this call's window keys are counted
  // with it while x is in registers (phase 1, into H); if every window key of
  // the call falls inside it (no block sets the bar's line 11), the digits of
  // that geometry rank the keys exactly as this call's own would (any base <=
  // the lowest window key and any width covering the highest: same groups,
  // same edges) and phase 2's count and barrier are skipped
  const SelHint hint = s_hint;
  // (an edge-speculating call counts no hinted level 0: a hit needs none, a
  // miss counts this call's own in phase 2)
  const bool hv = hint.valid != 0 && !a.eg;
  const int hb = hint.s + hint.w;
  const uint64_t hspan = hb >= 64 ? ~0ull : ((1ull << hb) - 1);
  const uint64_t hhi = hint.lo + hspan < hint.lo ? ~0ull : hint.lo + hspan;
  // ---- 1: selection (select_onepass) -------------------------------------
  const int64_t wbase = a.sp.base + (int64_t)t * TILE + (int64_t)w * (TILE / MONO_NW);
  double xv[MONO_SI], mv[MONO_SI];
  uint64_t bal[MONO_SI];
  uint32_t keepbits = 0;
  unsigned long long kmin = ~0ull, kmax = 0ull;
  {
    double px[MONO_SI], py[MONO_SI], pz[MONO_SI];
    uint32_t inbits = 0;
#pragma unroll
    for (int k = 0; k < MONO_SI; ++k) {
      const int64_t i = wbase + k * 64 + lane;
      const bool in = (i < a.n_hi) && in_family(i, a.sp);
      inbits |= (uint32_t)in << k;
      const double *q = a.pos + 3 * (in ? i : 0);
      px[k] = q[0];
      py[k] = q[1];
      pz[k] = q[2];
    }
    bool esc = false;
#pragma unroll
    for (int k = 0; k < MONO_SI; ++k) {
      const bool keep = ((inbits >> k) & 1u) && select_xyz(px[k], py[k], pz[k], a.sp, xv[k]);
      keepbits |= (uint32_t)keep << k;
      bal[k] = __ballot(keep);
      if (keep) {
        const unsigned long long kk = dkey(xv[k]);
        kmin = kk < kmin ? kk : kmin;
        kmax = kk > kmax ? kk : kmax;
        if (hv && kk >= a.ka && kk <= a.kb) {
          if (kk >= hint.lo && kk <= hhi) atomicAdd(&L0[(uint32_t)((kk - hint.lo) >> hint.s)], 1u);
          else esc = true;
        }
        if (a.eg && kk >= a.ka && kk <= a.kb) {  // edge speculation: upper bound among the edges
          int lo = 0, hi = nq;
          while (lo < hi) {
            const int mid = (lo + hi) >> 1;
            if (ek_l[mid] <= kk) lo = mid + 1; else hi = mid;
          }
          atomicAdd(&eUl[lo], 1u);
          if (lo > 0 && ek_l[lo - 1] == kk) atomicAdd(&eEl[lo - 1], 1u);
        }
      }
    }
    if (__ballot(esc) && lane == 0) st_sc1(a.bar + BAR_LINE * 11, a.gen0 + 1);
#pragma unroll
    for (int k = 0; k < MONO_SI; ++k) {
      const int64_t i = wbase + k * 64 + lane;
      mv[k] = (a.mass && ((keepbits >> k) & 1u)) ? a.mass[i] : 1.0;
    }
  }
  uint32_t c = 0;
#pragma unroll
  for (int k = 0; k < MONO_SI; ++k) {
    c += (uint32_t)__popcll(bal[k]);
    if (lane == 0) a.kw[(int64_t)t * (TILE / 64) + w * MONO_SI + k] = bal[k];
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const unsigned long long p = __shfl_xor(kmin, o, 64), q = __shfl_xor(kmax, o, 64);
    kmin = p < kmin ? p : kmin;
    kmax = q > kmax ? q : kmax;
  }
  if (lane == 0) {
    wcnt[w] = c;
    wmin[w] = kmin;
    wmax[w] = kmax;
  }
  __syncthreads();
  if (hv)  // the hinted counts -> H (complete at barrier 1)
    for (int i = tid; i < MONO_DIG; i += MONO_BT) {
      const uint32_t v = L0[i];
      if (v) atomicAdd(&a.H[i], v);
    }
  if (a.eg)  // ... and the edge counts
    for (int i = tid; i <= nq; i += MONO_BT) {
      if (eUl[i]) atomicAdd(&a.eU[i], eUl[i]);
      if (i < nq && eEl[i]) atomicAdd(&a.eE[i], eEl[i]);
    }
  if (tid == 0) {
    MonoRec r{0, ~0ull, 0ull, 0};
    for (int k = 0; k < MONO_NW; ++k) {
      r.cnt += wcnt[k];
      r.kmin = wmin[k] < r.kmin ? wmin[k] : r.kmin;
      r.kmax = wmax[k] > r.kmax ? wmax[k] : r.kmax;
    }
    st_sc1(&a.rec[t].cnt, r.cnt);
    st_sc1(&a.rec[t].kmin, r.kmin);
    st_sc1(&a.rec[t].kmax, r.kmax);
  }
  uint64_t gn = a.gen0 + 1;  // the barrier generation (sequential: skipped barriers take none)
  if (!grid_sync(a.bar, gn, nt, &s_ok)) return;
  MONO_STAMP(1);
  int64_t m_edge = 0;
  if (a.eg) {
    // the previous edges are this call's iff every rank r_q lies among the
    // keys equal to edge q: #keys < e_q <= r_q < #keys <= e_q (#keys < e_q =
    // the keys whose upper bound is <= q; equal ones counted at the last of
    // equal edges); every block decides the same from the same sums
    uint32_t u = 0;
    if (tid <= nq) u = ld_sc1(&a.eU[tid]);
    if (tid < nq) eEl[tid] = ld_sc1(&a.eE[tid]);
    uint32_t xs = u;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const uint32_t y = __shfl_up(xs, o, 64);
      if (lane >= (uint32_t)o) xs += y;
    }
    if (lane == 63) wsum[w] = xs;
    __syncthreads();
    uint32_t incl = xs;
    for (int k = 0; k < w; ++k) incl += wsum[k];
    if (tid <= nq) eUl[tid] = incl;  // keys with upper bound <= tid = keys < e_tid
    if (tid == 0) s_edge = 1;
    __syncthreads();
    const int64_t m = (int64_t)eUl[nq];  // every window key
    m_edge = m;
    if (tid < nq) {
      int j = tid;  // the last edge equal to this one
      while (j + 1 < nq && ek_l[j + 1] == ek_l[tid]) ++j;
      // #keys < e_q = the keys whose upper bound is <= q (eUl: inclusive prefix)
      const int64_t below = (int64_t)eUl[tid], eq = (int64_t)eEl[j];
      const int64_t r = (tid == nq - 1) ? m - 1 : (int64_t)((double)(tid * m) / (double)a.nbins);
      if (m < 2 || !(below <= r && r < below + eq)) s_edge = 0;
    }
    __syncthreads();
  }

  // ---- 2: totals, this tile's offset, compacted x, level-0 histogram -----
  {
    uint32_t cc = 0;
    unsigned long long mn = ~0ull, mx = 0ull;
    if ((uint32_t)tid < nt) {
      cc = (uint32_t)ld_sc1(&a.rec[tid].cnt);
      mn = ld_sc1(&a.rec[tid].kmin);
      mx = ld_sc1(&a.rec[tid].kmax);
    }
    uint32_t xs = cc;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const uint32_t y = __shfl_up(xs, o, 64);
      if (lane >= (uint32_t)o) xs += y;
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      const unsigned long long p = __shfl_xor(mn, o, 64), q = __shfl_xor(mx, o, 64);
      mn = p < mn ? p : mn;
      mx = q > mx ? q : mx;
    }
    if (lane == 63) wsum[w] = xs;
    if (lane == 0) {
      wmin[w] = mn;
      wmax[w] = mx;
    }
    __syncthreads();
    uint32_t ex = xs - cc;
    for (int k = 0; k < w; ++k) ex += wsum[k];
    if ((uint32_t)tid == t) s_toff = ex;
    if (tid == 0) {
      FusedCtl cl{};
      uint64_t tot = 0;
      cl.kmin = ~0ull;
      cl.kmax = 0ull;
      for (int k = 0; k < MONO_NW; ++k) {
        tot += wsum[k];
        cl.kmin = wmin[k] < cl.kmin ? wmin[k] : cl.kmin;
        cl.kmax = wmax[k] > cl.kmax ? wmax[k] : cl.kmax;
      }
      cl.n = (int64_t)tot;
      const uint64_t lo = a.ka > cl.kmin ? a.ka : cl.kmin;
      const uint64_t hi = a.kb < cl.kmax ? a.kb : cl.kmax;
      SelHint ho{};
      if (cl.n == 0 || a.empty_bounds || lo > hi) {
        cl.err |= 2;
        cl.w0 = 1;
      } else {
        const uint64_t span = hi - lo;
        const int B = span ? 64 - __builtin_clzll(span) : 1;
        cl.w0 = B < MONO_BITS ? B : MONO_BITS;
        cl.s0 = B - cl.w0;
        cl.lo = lo;
        // the next call's hint: this call's digit width with the base moved
        // down by half the room the width leaves above the window, when that
        // room is at least 1/32 of the span (a similar next call still fits
        // with digits as fine as its own); else the window widened by 1/64
        // of its span each side (one more key bit: digits twice as wide,
        // groups twice as large — the finish took +5 us at 1M that way)
        const uint64_t cap = B >= 64 ? ~0ull : ((1ull << B) - 1);
        const uint64_t room = cap - span;
        if (room >= (span >> 5)) {
          const uint64_t mg = room >> 1;
          ho.w = cl.w0;
          ho.s = cl.s0;
          ho.lo = lo >= mg ? lo - mg : 0ull;
        } else {
          const uint64_t mg = span >> 6;
          const uint64_t lo2 = lo >= mg ? lo - mg : 0ull;
          const uint64_t hi2 = hi + mg < hi ? ~0ull : hi + mg;
          const uint64_t sp2 = hi2 - lo2;
          const int B2 = sp2 ? 64 - __builtin_clzll(sp2) : 1;
          ho.w = B2 < MONO_BITS ? B2 : MONO_BITS;
          ho.s = B2 - ho.w;
          ho.lo = lo2;
        }
        ho.valid = 1;
      }
      if (t == 0 && a.hout) *a.hout = ho;
      const bool hinted = hv && !(cl.err & 2) && ld_sc1(a.bar + BAR_LINE * 11) != a.gen0 + 1;
      if (hinted) {
        cl.lo = hint.lo;
        cl.s0 = hint.s;
        cl.w0 = hint.w;
        cl.hint = 1;
      }
      if (s_edge && !(cl.err & 2)) {  // the previous edges hold: no order statistics to find
        cl.m = m_edge;
        cl.spec = SPEC_EDGE;
      } else {
        s_edge = 0;
      }
      s_hinted = hinted ? 1 : 0;
      s_ctl = cl;
    }
  }
  __syncthreads();
  const FusedCtl ctl0 = s_ctl;
  const bool ok2 = !(ctl0.err & 2);
  uint32_t pos[MONO_SI];
  {
    uint32_t run = s_toff;
    for (int k = 0; k < w; ++k) run += wcnt[k];
#pragma unroll
    for (int k = 0; k < MONO_SI; ++k) {
      pos[k] = run + rank_below(bal[k]);
      if ((keepbits >> k) & 1u) a.x[pos[k]] = xv[k];
      run += (uint32_t)__popcll(bal[k]);
    }
    if (tid == 0) a.toff[t] = s_toff;
  }
  const bool hinted = s_hinted != 0;
  const bool edge = s_edge != 0;
  if (edge) {  // nothing reads the level-0 histogram: zeroed for the next call, slice by slice
    const uint32_t per = (MONO_DIG + nt - 1) / nt, h0 = t * per;
    for (uint32_t i = h0 + tid; i < min<uint32_t>(h0 + per, MONO_DIG); i += MONO_BT)
      if (hv) a.H[i] = 0u;
  } else if (hinted) {  // H is complete: no second count, no barrier
  } else {
    if (hv) {  // (phase 1 counted into L0 with the hint's geometry)
      for (int i = tid; i < MONO_DIG; i += MONO_BT) L0[i] = 0;
      __syncthreads();
    }
    if (ok2) {
#pragma unroll
      for (int k = 0; k < MONO_SI; ++k) {
        const uint64_t key = dkey(xv[k]);
        if (((keepbits >> k) & 1u) && key >= a.ka && key <= a.kb)
          atomicAdd(&L0[(uint32_t)((key - ctl0.lo) >> ctl0.s0)], 1u);
      }
    }
    __syncthreads();
    if (ok2)
      for (int i = tid; i < MONO_DIG; i += MONO_BT) {
        const uint32_t v = L0[i];
        if (v) atomicAdd(&a.H2[i], v);
      }
    if (!grid_sync(a.bar, ++gn, nt, &s_ok)) return;
  }
  const uint32_t *Hs = hinted ? a.H : a.H2;
  MONO_STAMP(2);

  // ---- 3: ranks -> level-0 digits and groups; keys -> group segments -----
  // (an edge hit skips phases 3 and 4 and their barriers)
  int ng = 0;
  if (ok2 && !edge) {
    constexpr int PT = MONO_DIG / MONO_BT;
    static_assert(PT % 4 == 0, "16-B LDS reads");
    // H in with lane-consecutive sc1 loads (a thread's PT consecutive words
    // loaded directly put a wave's 64 lanes 4 KB apart: ~64 L2 requests
    // per load), through LDS to each thread's PT consecutive digits
    {
      uint32_t h[PT];
#pragma unroll
      for (int k = 0; k < PT; ++k) h[k] = ld_sc1(&Hs[k * MONO_BT + tid]);
#pragma unroll
      for (int k = 0; k < PT; ++k) L0[k * MONO_BT + tid] = h[k];
    }
    __syncthreads();
    uint32_t v[PT], tot = 0;
#pragma unroll
    for (int k = 0; k < PT; k += 4) {
      const uint4 q = *(const uint4 *)&L0[tid * PT + k];
      v[k] = q.x;
      v[k + 1] = q.y;
      v[k + 2] = q.z;
      v[k + 3] = q.w;
    }
#pragma unroll
    for (int k = 0; k < PT; ++k) tot += v[k];
    uint32_t xs = tot;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const uint32_t y = __shfl_up(xs, o, 64);
      if (lane >= (uint32_t)o) xs += y;
    }
    if (lane == 63) wsum[w] = xs;
    __syncthreads();
    uint32_t run = xs - tot;
    for (int k = 0; k < w; ++k) run += wsum[k];
#pragma unroll
    for (int k = 0; k < PT; ++k) {
      run += v[k];
      L0[tid * PT + k] = run;  // inclusive counts
    }
    for (int i = tid; i < MONO_DIG / 2; i += MONO_BT) ((uint32_t *)L1)[i] = ~0u;
    __syncthreads();
    MONO_STAMP(7);
    const int64_t m = (int64_t)L0[MONO_DIG - 1];
    const int top = (1 << ctl0.w0) - 1;
    for (int q = tid; q < nq; q += MONO_BT) {
      int64_t r = 0;
      if (m >= 2) r = (q == nq - 1) ? m - 1 : (int64_t)((double)(q * m) / (double)a.nbins);
      int lo = 0, hi = top;  // first digit whose inclusive count exceeds r
      while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if ((int64_t)L0[mid] <= r) lo = mid + 1; else hi = mid;
      }
      q_dig[q] = (uint32_t)lo;
      q_rr[q] = r - (lo ? (int64_t)L0[lo - 1] : 0);
    }
    __syncthreads();
    if (w == 0) {  // groups = run starts of the non-decreasing digits; sizes, offsets
      uint32_t cnt = 0;
      for (int q0 = 0; q0 < nq; q0 += 64) {
        const int q = q0 + (int)lane;
        const bool st = q < nq && (q == 0 || q_dig[q - 1] != q_dig[q]);
        const uint64_t b = __ballot(st);
        if (st) g_start[cnt + rank_below(b)] = (uint32_t)q;
        cnt += (uint32_t)__popcll(b);
      }
      if (lane == 0) g_start[cnt] = (uint32_t)nq;
      uint32_t base = 0;
      for (uint32_t g0 = 0; g0 < cnt; g0 += 64) {
        const uint32_t g = g0 + lane;
        uint32_t sz = 0;
        if (g < cnt) {
          const uint32_t d = q_dig[g_start[g]];
          sz = L0[d] - (d ? L0[d - 1] : 0u);
          L1[d] = (uint16_t)g;
          g_lcnt[g] = 0;
        }
        uint32_t ys = sz;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
          const uint32_t y = __shfl_up(ys, o, 64);
          if (lane >= (uint32_t)o) ys += y;
        }
        if (g < cnt) g_off[g] = base + ys - sz;
        base += __shfl(ys, 63, 64);
      }
      if (lane == 0) {
        g_off[cnt] = base;
        s_ctl.m = m;
        s_ctl.ng = (int32_t)cnt;
        s_ctl.total = base;
      }
    }
    __syncthreads();
    ng = s_ctl.ng;
    // this tile's keys of chosen buckets: LDS slots per group, then one
    // global atomic per non-empty group for the tile's place in its segment
    uint32_t gg[MONO_SI], ls[MONO_SI];
#pragma unroll
    for (int k = 0; k < MONO_SI; ++k) {
      gg[k] = 0xffffu;
      const uint64_t key = dkey(xv[k]);
      if (((keepbits >> k) & 1u) && key >= a.ka && key <= a.kb)
        gg[k] = L1[(uint32_t)((key - ctl0.lo) >> ctl0.s0)];
      ls[k] = gg[k] != 0xffffu ? atomicAdd(&g_lcnt[gg[k]], 1u) : 0u;
    }
    __syncthreads();
    if (tid < ng && g_lcnt[tid]) g_base[tid] = atomicAdd(&a.gcnt[tid], g_lcnt[tid]);
    __syncthreads();
#pragma unroll
    for (int k = 0; k < MONO_SI; ++k)
      if (gg[k] != 0xffffu)
        st_sc1(&a.seg[g_off[gg[k]] + g_base[gg[k]] + ls[k]], dkey(xv[k]) - ctl0.lo);
  }
  if (!edge) {
    if (!grid_sync(a.bar, ++gn, nt, &s_ok)) return;
    MONO_STAMP(3);
    // H / H2 read for the last time: zeroed for the next call, slice by slice
    const uint32_t per = (MONO_DIG + nt - 1) / nt, h0 = t * per;
    for (uint32_t i = h0 + tid; i < min<uint32_t>(h0 + per, MONO_DIG); i += MONO_BT) {
      if (hv) a.H[i] = 0u;
      if (!hinted) a.H2[i] = 0u;
    }
  }

  // ---- 4: each group's ranks (fused_finish) -> edges ---------------------
  if (ok2 && !edge) {
    uint64_t *sk = (uint64_t *)L0;
    uint32_t *hist = (uint32_t *)L1;
    const uint64_t lo = ctl0.lo;
    const int s = ctl0.s0;
    for (int g = (int)t; g < ng; g += (int)nt) {
      const int64_t o = g_off[g], S = (int64_t)g_off[g + 1] - o;
      const bool in_lds = S <= (int64_t)(sizeof(L0) / 8);  // (L0 holds 8192 u64 keys)
      if (in_lds)
        for (int64_t i = tid; i < S; i += MONO_BT) sk[i] = ld_sc1(&a.seg[o + i]);
      __syncthreads();
      if (S <= MONO_BT) {  // small group: each key's rank by counting
        const uint64_t k = tid < S ? sk[tid] : ~0ull;
        uint32_t less = 0, eq = 0;
        count_rank(sk, (int)S, k, less, eq);
        for (int q = (int)g_start[g]; q < (int)g_start[g + 1]; ++q) {
          const int64_t rr = q_rr[q];
          if (tid < S && (int64_t)less <= rr && rr < (int64_t)(less + eq))
            st_sc1d(&a.edges[q], dkey_inv(lo + k));  // tied threads write the same value
        }
      } else {
        for (int q = (int)g_start[g]; q < (int)g_start[g + 1]; ++q) {
          uint64_t key;
          const uint64_t pref0 = (uint64_t)q_dig[q] << s;
          if (in_lds) finish_group<true>(sk, S, pref0, s, q_rr[q], hist, wsum, pick, key);
          else finish_group<false, true>(a.seg + o, S, pref0, s, q_rr[q], hist, wsum, pick, key);
          if (tid == 0) st_sc1d(&a.edges[q], dkey_inv(lo + key));
        }
      }
      __syncthreads();
    }
  }
  if (!edge) {
    if (!grid_sync(a.bar, ++gn, nt, &s_ok)) return;
    MONO_STAMP(4);
  }
  if (!ok2) {  // nothing to bin: the control record tells the host
    // every block takes this branch (ctl0 is the same in all of them); one
    // more barrier: every block has read the edge sums (a.eU) before block 0
    // zeroes them
    if (tid == 0) s_ctl.spec = (int32_t)((gn + 1 - a.gen0) << 8);  // the barriers used
    if (!grid_sync(a.bar, ++gn, nt, &s_ok)) return;
    if (t == 0 && a.eg)
      for (int i = tid; i <= nq; i += MONO_BT) {
        a.eU[i] = 0u;
        if (i < nq) a.eE[i] = 0u;
      }
    constexpr int NC = (int)(sizeof(FusedCtl) / sizeof(double));
    if (t == 0 && tid < NC) st_sc1d(&a.stage[tid], ((const double *)&s_ctl)[tid]);
    mono_done(a, NC + nq + nb + a.fs.nm * nb);
    return;
  }

  // ---- 5: bins, per-bin sums, the tile's counts and in-tile CSR ranks ----
  uint32_t *runs = (uint32_t *)L1;                         // [MONO_NW][RADIX]
  double *acc = (double *)((char *)L1 + sizeof(uint32_t) * MONO_NW * RADIX);
  const int nm = a.fs.nm, macc = nm * nb;
  for (int i = tid; i < nq; i += MONO_BT) e_lds[i] = ld_sc1d(edge ? &a.pedges[i] : &a.edges[i]);
  // the ranks' peer words (prims.h wave_ranks_lds) in L0: free between the
  // finish (phase 4) and the CSR offsets (phase 6)
  uint64_t *pmask = (uint64_t *)L0;
  static_assert(sizeof(uint32_t) * MONO_DIG >= sizeof(uint64_t) * MONO_NW * RADIX, "pmask in L0");
  for (int i = tid; i < MONO_NW * RADIX; i += MONO_BT) {
    runs[i] = 0;
    pmask[i] = 0ull;
  }
  for (int i = tid; i < macc; i += MONO_BT) acc[i] = 0.0;
  __syncthreads();
  uint32_t bk[MONO_SI], lp[MONO_SI];
  {
#pragma unroll
    for (int k = 0; k < MONO_SI; ++k) {
      const bool kp = (keepbits >> k) & 1u;
      bk[k] = kp ? bin_of(xv[k], e_lds, nb) : (uint32_t)nb + 1;
      if (kp) a.bins[pos[k]] = bk[k];
    }
#pragma unroll
    for (int q = 0; q < AS_MAXM; ++q) {  // unrolled: the fields are kernel-argument scalars
      if (q >= nm) break;
      mom_add<MONO_SI>(acc + q * nb, a.fs.op[q], a.fs.col[q], a.fs.f[q], a.fs.w[q], bk, xv, mv,
                       (uint32_t)nb);
    }
    // element order (wave, k, lane) = particle order
    uint32_t dg[MONO_SI];
    bool okk[MONO_SI];
#pragma unroll
    for (int k = 0; k < MONO_SI; ++k) {
      okk[k] = (keepbits >> k) & 1u;
      dg[k] = bk[k] & 255u;
    }
    wave_ranks_lds<MONO_SI>(dg, okk, runs + w * RADIX, pmask + w * RADIX, lp);
  }
  __syncthreads();
  if (tid < RADIX) {  // the tile's count of bin d; runs -> offsets over the waves
    uint32_t s = 0;
    for (int k = 0; k < MONO_NW; ++k) {
      const uint32_t v = runs[k * RADIX + tid];
      runs[k * RADIX + tid] = s;
      s += v;
    }
    st_sc1(&a.th[(int64_t)tid * nt + t], s);
  }
  for (int i = tid; i < macc; i += MONO_BT) st_sc1d(&a.slab[(int64_t)t * macc + i], acc[i]);
  if (tid == 0) s_ctl.spec = (edge ? SPEC_EDGE : 0) | (int32_t)((gn + 1 - a.gen0) << 8);
  if (!grid_sync(a.bar, ++gn, nt, &s_ok)) return;
  MONO_STAMP(5);
  if (t == 0) {  // (every block read the edge sums and the previous edges before barrier 1 / here)
    for (int i = tid; i < nq; i += MONO_BT) {
      a.pedges[i] = e_lds[i];  // the next call's speculation
      a.edges[i] = e_lds[i];
    }
    if (a.eg)
      for (int i = tid; i <= nq; i += MONO_BT) {
        a.eU[i] = 0u;
        if (i < nq) a.eE[i] = 0u;
      }
  }

  // ---- 6: CSR offsets, perm, counts, packed results ----------------------
  {
    // bin d: its count in the tiles before t and in all tiles.  Wave w reads
    // rows d = w, w + 16, ... of the [bin][tile] table coalesced (lane = tile,
    // nt <= 256: 4 loads per lane and row), six rows (24 loads) in flight;
    // only the nb + 1 rows a bin can occupy (nb: invalid), the rest are 0
    uint32_t *pb = L0, *pa = L0 + RADIX;
    static_assert(MONO_MAXT <= 256, "4 tiles per lane and row");
    constexpr int RR = 6;
    const int nr = nb + 1;
    for (int d = nr + tid; d < RADIX; d += MONO_BT) pa[d] = pb[d] = 0u;
    for (int d0 = w; d0 < nr; d0 += RR * MONO_NW) {
      uint32_t v[RR][4];
#pragma unroll
      for (int r = 0; r < RR; ++r)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const uint32_t u = lane + 64 * j;
          v[r][j] = (u < nt && d0 + r * MONO_NW < nr)
                        ? ld_sc1(&a.th[(int64_t)(d0 + r * MONO_NW) * nt + u]) : 0u;
        }
#pragma unroll
      for (int r = 0; r < RR; ++r) {
        if (d0 + r * MONO_NW >= nr) continue;  // (uniform)
        uint32_t al = 0, be = 0;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          al += v[r][j];
          be += (lane + 64 * j) < t ? v[r][j] : 0u;
        }
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) {
          al += __shfl_xor(al, o, 64);
          be += __shfl_xor(be, o, 64);
        }
        if (lane == 0) {
          pa[d0 + r * MONO_NW] = al;
          pb[d0 + r * MONO_NW] = be;
        }
      }
    }
    __syncthreads();
    const int d = tid & (RADIX - 1);
    // bins d < RADIX on waves 0-3: total, tiles-before-t count, bin start
    uint32_t bl = 0, tot = 0, xs = 0;
    if (tid < RADIX) {
      bl = pb[d];
      tot = pa[d];
      xs = tot;
#pragma unroll
      for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = __shfl_up(xs, o, 64);
        if (lane >= (uint32_t)o) xs += y;
      }
      if (lane == 63) wsum[w] = xs;
    }
    __syncthreads();
    if (tid < RADIX) {
      uint32_t ex = 0;
      for (int k = 0; k < w; ++k) ex += wsum[k];
      if (t == 0 && d < nb) {
        a.counts[d] = tot;
        constexpr int NC = (int)(sizeof(FusedCtl) / sizeof(double));
        st_sc1d(&a.stage[NC + nq + d], __builtin_bit_cast(double, (unsigned long long)tot));
      }
      s_gofs[d] = ex + xs - tot + bl;  // bin start + this bin's keys in tiles before t
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < MONO_SI; ++k)
      if ((keepbits >> k) & 1u) {
        const uint32_t dgt = bk[k] & 255u;
        a.perm[s_gofs[dgt] + runs[w * RADIX + dgt] + lp[k]] = (int32_t)pos[k];
      }
  }
  constexpr int NC = (int)(sizeof(FusedCtl) / sizeof(double));
  if (t == 0) {
    if (tid < NC) st_sc1d(&a.stage[tid], ((const double *)&s_ctl)[tid]);
    for (int i = tid; i < nq; i += MONO_BT) st_sc1d(&a.stage[NC + i], e_lds[i]);
  }
  // per-bin sums: column j summed over the tiles in a fixed order by one
  // wave; columns spread over the blocks first (its 4 loads per lane are 64
  // lines apart: a few columns per CU, not 16 on each of the first CUs)
  const int nsum = macc;
  for (int j = (int)t + w * (int)nt; j < nsum; j += (int)nt * MONO_NW) {
    double v[4];  // nt <= 256: four rows per lane, loads in flight together
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const uint32_t r = lane + 64 * k;
      v[k] = r < nt ? ld_sc1d(&a.slab[(int64_t)r * macc + j]) : 0.0;
    }
    double s = ((v[0] + v[1]) + v[2]) + v[3];
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
    if (lane == 0) st_sc1d(&a.stage[NC + nq + nb + j], s);
  }
  MONO_STAMP(6);
  mono_done(a, NC + nq + nb + nsum);
}

// ----------------------------------------------------------------- moments
// LDS: accumulators in LDS (nb <= LDS_MOM_BINS), one slab row per block;
// else straight to global_acc.  Templated so the LDS path indexes the
// __shared__ array itself (ds_add_f64): through a pointer that may be either,
// every atomic would be a flat atomic.
template <int WMODE, bool LDS>  // WMODE 0: no weights, 1: weights
__global__ void __launch_bounds__(TPB)
    moments_kernel(const uint32_t *__restrict__ bins, const double *__restrict__ f,
                   const double *__restrict__ wt, int64_t n, int nb, uint32_t cols,
                   double *__restrict__ slab, double *__restrict__ global_acc) {
  extern __shared__ double acc_lds[];
  if (LDS) {
    for (int k = threadIdx.x; k < nb * NMOM; k += TPB) acc_lds[k] = 0.0;
    __syncthreads();
  }
  auto add = [&](int64_t idx, double v) {
    if (LDS) atomicAdd(&acc_lds[idx], v);
    else atomicAdd(&global_acc[idx], v);
  };
  // grid-stride over tiles: at most gridDim.x slabs to reduce afterwards
  for (int64_t base = (int64_t)blockIdx.x * TILE; base < n; base += (int64_t)gridDim.x * TILE) {
    uint32_t bv[IPT];  // the tile's loads first, then the LDS accumulation
    double fv[IPT], wv[IPT];
#pragma unroll
    for (int k = 0; k < IPT; ++k) {
      const int64_t i = base + k * TPB + threadIdx.x;
      const bool ok = i < n;
      bv[k] = ok ? bins[i] : (uint32_t)nb;
      fv[k] = ok ? f[i] : 0.0;
      wv[k] = (WMODE && ok) ? wt[i] : 1.0;
    }
#pragma unroll
    for (int k = 0; k < IPT; ++k) {
      if (bv[k] >= (uint32_t)nb) continue;
      const double v = fv[k], a = __builtin_fabs(v), ww = wv[k];
      const int64_t t = (int64_t)bv[k] * NMOM;
      // only the requested columns (cols is uniform: scalar branches)
      if (WMODE) {
        if (cols & 1u) add(t + 0, ww);
        if (cols & 2u) add(t + 1, v * ww);
        if (cols & 4u) add(t + 2, (v * v) * ww);
        if (cols & 32u) add(t + 5, a * ww);
      }
      if (cols & 8u) add(t + 3, v);
      if (cols & 16u) add(t + 4, v * v);
      if (cols & 64u) add(t + 6, a);
    }
  }
  if (LDS) {
    __syncthreads();
    double *dst = slab + (int64_t)blockIdx.x * nb * NMOM;
    for (int k = threadIdx.x; k < nb * NMOM; k += TPB) dst[k] = acc_lds[k];
  }
}

// Sum slab[row][len] over rows in a fixed order (deterministic): first
// SLAB_G partials, partial g = rows g, g+SLAB_G, ... in turn; then the
// partials in g order.
__global__ void __launch_bounds__(TPB) reduce_slab_part(const double *__restrict__ slab,
                                                        int64_t rows, int64_t len,
                                                        double *__restrict__ part) {
  const int64_t col = (int64_t)blockIdx.x * TPB + threadIdx.x;
  const int g = blockIdx.y;
  if (col >= len) return;
  double s = 0.0;
  for (int64_t r = g; r < rows; r += SLAB_G) s += slab[r * len + col];
  part[(int64_t)g * len + col] = s;
}

__global__ void __launch_bounds__(TPB) reduce_slab_final(const double *__restrict__ part,
                                                         int64_t len, double *__restrict__ out) {
  const int64_t col = (int64_t)blockIdx.x * TPB + threadIdx.x;
  if (col >= len) return;
  double s = 0.0;
#pragma unroll 8
  for (int g = 0; g < SLAB_G; ++g) s += part[(int64_t)g * len + col];
  out[col] = s;
}

__global__ void gather_by_idx(const double *__restrict__ src, const int32_t *__restrict__ idx,
                              int64_t n, double *__restrict__ dst) {
  int64_t t = (int64_t)blockIdx.x * TPB + threadIdx.x;
  if (t < n) dst[t] = src[idx[t]];
}

__global__ void widen_perm(const int32_t *__restrict__ p, int64_t n, int64_t *__restrict__ out) {
  int64_t t = (int64_t)blockIdx.x * TPB + threadIdx.x;
  if (t < n) out[t] = p[t];
}

// ---------------------------------------------- per-bin order statistics
// Percentile / Median / Abs_pXX (proarray.py:689-722): per bin, argsort the
// field, cumsum the weights in that order (or linspace(0, 1, m) without
// weights), normalise, np.interp(p/100, cdf, sorted field).
//
// Segmented sort: every element of the binned space is sorted by (bin id,
// value key) with stable LSD radix passes (value key first, then bin id);
// ties keep index order (numpy's argsort is not stable: tied values are
// equal, only the summation order of tied weights can differ).  Dropped
// elements (bin id nb) land behind the last bin.

// value keys of f (|f| for abs_*), NaN last like np.argsort
__global__ void pct_keys(const double *__restrict__ f, int64_t n, int absval,
                         uint64_t *__restrict__ keys) {
  const int64_t t = (int64_t)blockIdx.x * TPB + threadIdx.x;
  if (t >= n) return;
  double v = f[t];
  if (absval) v = fabs(v);
  keys[t] = dkey(v);
}

__global__ void gather_bin_ids(const uint32_t *__restrict__ bins, const int32_t *__restrict__ e,
                               int64_t n, uint32_t *__restrict__ out) {
  const int64_t t = (int64_t)blockIdx.x * TPB + threadIdx.x;
  if (t < n) out[t] = bins[e[t]];
}

// offsets[b] = Σ counts[< b] (nb + 1 entries), one block
__global__ void __launch_bounds__(1024) counts_to_offsets(const uint64_t *__restrict__ counts,
                                                          int64_t nb, int64_t *__restrict__ off) {
  __shared__ int64_t part[1024];
  const int t = threadIdx.x;
  const int64_t per = (nb + 1023) / 1024;
  const int64_t a = std::min<int64_t>(nb, t * per), b = std::min<int64_t>(nb, a + per);
  int64_t s = 0;
  for (int64_t k = a; k < b; ++k) s += (int64_t)counts[k];
  part[t] = s;
  __syncthreads();
  if (t == 0) {
    int64_t run = 0;
    for (int k = 0; k < 1024; ++k) {
      const int64_t v = part[k];
      part[k] = run;
      run += v;
    }
  }
  __syncthreads();
  s = part[t];
  for (int64_t k = a; k < b; ++k) {
    off[k] = s;
    s += (int64_t)counts[k];
  }
  if (t == 1023) off[nb] = s;
}

// numpy's binary_search_with_guess (numpy/_core/src/multiarray/
// compiled_base.c), literally: the index it returns for NaN-containing or
// non-monotone xp (negative weights) depends on the probe sequence.
template <typename XP>
__device__ int64_t np_bsearch_guess(double key, const XP &xp, int64_t len, int64_t guess) {
  constexpr int64_t LIKELY_IN_CACHE_SIZE = 8;
  int64_t imin = 0, imax = len;
  if (key > xp(len - 1)) return len;
  if (key < xp(0)) return -1;
  if (len <= 4) {
    int64_t i = 1;
    for (; i < len && key >= xp(i); ++i) {
    }
    return i - 1;
  }
  if (guess > len - 3) guess = len - 3;
  if (guess < 1) guess = 1;
  if (key < xp(guess)) {
    if (key < xp(guess - 1)) {
      imax = guess - 1;
      if (guess > LIKELY_IN_CACHE_SIZE && key >= xp(guess - LIKELY_IN_CACHE_SIZE))
        imin = guess - LIKELY_IN_CACHE_SIZE;
    } else {
      return guess - 1;
    }
  } else {
    if (key < xp(guess + 1)) return guess;
    if (key < xp(guess + 2)) return guess + 1;
    imin = guess + 2;
    if (guess < len - LIKELY_IN_CACHE_SIZE - 1 && key < xp(guess + LIKELY_IN_CACHE_SIZE))
      imax = guess + LIKELY_IN_CACHE_SIZE;
  }
  while (imin < imax) {
    const int64_t imid = imin + ((imax - imin) >> 1);
    if (key >= xp(imid)) imin = imid + 1;
    else imax = imid;
  }
  return imin - 1;
}

// np.interp(x, xp, fp) for one scalar x (arr_interp, default left/right)
template <typename XP, typename FP>
__device__ double np_interp1(double x, const XP &xp, const FP &fp, int64_t len) {
#pragma clang fp contract(off)
  const double lval = fp(0), rval = fp(len - 1);
  if (len == 1) {
    const double xv = xp(0);
    return (x < xv) ? lval : ((x > xv) ? rval : fp(0));
  }
  if (x != x) return x;
  const int64_t j = np_bsearch_guess(x, xp, len, 0);
  if (j == -1) return lval;
  if (j == len) return rval;
  if (j == len - 1) return fp(j);
  const double xj = xp(j);
  if (xj == x) return fp(j);
  const double xj1 = xp(j + 1), fj = fp(j), fj1 = fp(j + 1);
  const double slope = (fj1 - fj) / (xj1 - xj);
  double r = slope * (x - xj) + fj;
  if (r != r) {
    r = slope * (x - xj1) + fj1;
    if (r != r && fj == fj1) r = fj;
  }
  return r;
}

constexpr int PCT_CH = 2048;  // weights per LDS chunk of the sequential cumsum

// One block per bin.  e: element ids sorted by (bin, value); off: bin
// offsets into e; q: the nq fractions p/100.  Weighted: the cumulative sum
// runs on ONE lane in the reference's order (np.cumsum is sequential, so
// this reproduces its rounding), staged through LDS; cdf scratch holds it.
__global__ void __launch_bounds__(TPB)
pct_bins(const int32_t *__restrict__ e, const int64_t *__restrict__ off,
         const double *__restrict__ f, const double *__restrict__ w, int absval,
         const double *__restrict__ q, int nq, double *__restrict__ cdf,
         double *__restrict__ out) {
#pragma clang fp contract(off)
  __shared__ double ws[PCT_CH];
  __shared__ double cs[PCT_CH];
  const int b = blockIdx.x;
  const int64_t o = off[b], m = off[b + 1] - o;
  const int tid = threadIdx.x;
  if (m == 0) {
    for (int k = tid; k < nq; k += TPB) out[(int64_t)b * nq + k] = __builtin_nan("");
    return;
  }
  if (w && m >= 2) {
    double c = 0.0;
    for (int64_t base = 0; base < m; base += PCT_CH) {
      const int len = (int)std::min<int64_t>(PCT_CH, m - base);
      for (int i = tid; i < len; i += TPB) ws[i] = w[e[o + base + i]];
      __syncthreads();
      if (tid == 0) {
        int i = 0;
        if (base == 0) {
          c = ws[0];
          cs[0] = c;
          i = 1;
        }
        for (; i + 8 <= len; i += 8) {
          double v[8];
#pragma unroll
          for (int j = 0; j < 8; ++j) v[j] = ws[i + j];
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            c = c + v[j];
            cs[i + j] = c;
          }
        }
        for (; i < len; ++i) {
          c = c + ws[i];
          cs[i] = c;
        }
      }
      __syncthreads();
      for (int i = tid; i < len; i += TPB) cdf[o + base + i] = cs[i];
      __syncthreads();
    }
  }
  auto fp = [&](int64_t k) -> double {
    const double v = f[e[o + k]];
    return absval ? fabs(v) : v;
  };
  for (int k = tid; k < nq; k += TPB) {
    const double x = q[k];
    double r;
    if (w && m >= 2) {
      const double c0 = cdf[o];
      const double d = cdf[o + m - 1] - c0;
      auto xp = [&](int64_t i) -> double { return (cdf[o + i] - c0) / d; };
      r = np_interp1(x, xp, fp, m);
    } else if (m >= 2) {
      // np.linspace(0, 1, m): k * (1 / (m - 1)), last element exactly 1
      const double step = 1.0 / (double)(m - 1);
      auto xp = [&](int64_t i) -> double { return i == m - 1 ? 1.0 : (double)i * step; };
      r = np_interp1(x, xp, fp, m);
    } else {
      r = fp(0);  // one element: the single-point np.interp
    }
    out[(int64_t)b * nq + k] = r;
  }
}

// ----------------------------------------------------------------- handle
struct MselState {  // radix select in progress (equaln)
  bool active = false;
  int nq = 0, B = 0, L = 0, next = 0;
  int wd[MS_MAXL] = {};
  int64_t nbins = 0;
  uint64_t ka = 0, kb = 0, lo = 0;
};

struct Profile {
  int device = -1;
  int64_t n = 0;          // elements in the binned space
  int64_t nb = -1;        // bins of the last assignment
  int64_t n_valid = 0;
  bool has_w = false;
  bool has_idx = false;
  bool csr_ready = false;
  bool csrh_ready = false;  // csrh = the CSR pass histogram, from assign_bins
  bool mm_valid = false;   // mm = min / max key of x, cached on the host
  uint64_t mm[2] = {0, 0};
  MselState ms;
  Buf msH, msR, msG, msNg, msM, msRows, msL0, msL1, msCnt, csrh, slabp, selst, accs;
  prim::HostBuf pin;  // pinned readback staging (async D2H, one sync)
  Buf x, w, idx, bins, perm, keys0, keys1, vtmp, hist, tsum, edges, counts, minmax, slab, acc,
      field, weight, ranks, bounds;
  Buf pk0, pk1, pv0, pv1, pbk, pcdf, poff, pq, pout;  // order statistics
  Buf fctl, fseg, fgrp, fslab, fpack, frec, fblk, bins8;  // one-sync equaln path
  bool bins_in8 = false;  // the last assignment's bins are bytes in bins8 (ensure_bins32)
  // lazy selection (select_launch): keep words, tile offsets, staged masses
  Buf kw, toff, mstage, xc, kpre;
  // tiled radial calls: level-0 geometry hints (two SelHint slots, by call
  // parity) and select_tiles' digit rows
  Buf shint, shs, srows, swc, sbt;  // (shs: sample_hint scratch) + select_tiles' per-(tile, wave) counts and block totals
  // speculative assignment: the stored bin table, select_tiles' deferred
  // lists, their [start, length] per select block, per-block sums
  Buf stab, srec, sspec, sslab, sflag;
  bool spec_next = false;  // the last tiled call's ranks matched the table: speculate
  // a speculating call launched select_tiles<_, true> and has not finished
  // (an error between it and fused_finish, which clears them, can leave the
  // speculation flag word and the per-edge counts set): the next speculating
  // call zeroes them first
  bool spec_dirty = false;
  // pbx_profile_set_source_stable: the caller's device positions stay alive
  // and unchanged until the next selection on this handle, so a speculating
  // call may keep no copy of x (ensure_x rebuilds it from them); without it
  // only handle-owned (staged host) positions let a call speculate
  bool src_stable = false;
  bool edge_next = false;  // ... and its edges were the call's before it: speculate on edges too
  std::vector<double> last_edges;  // the last tiled call's edges
  Buf slteq;               // edge speculation: per rank, keys below / equal to its edge
  int64_t n_edge_hit = 0;
  bool x_missing = false;  // the last selection stored no x (a speculation hit): ensure_x rebuilds it
  XSrc xsrc{};             // ... from these positions / parameters
  Buf posst;               // lazy selections of host arrays: the staged positions (kept for xsrc)
  int64_t n_spec = 0, n_spec_hit = 0;  // tiled calls that speculated, of them hits
  uint64_t n_tiled = 0;
  bool lazy = false, w_ready = false, idx_ready = false;
  bool x_tiled = false;  // x holds a tiled selection (tile t at x[t * TILE ..]): ensure_x
  int64_t sel_base = 0, sel_span = 0;
  uint32_t sel_nt = 0;
  uint32_t sel_rsub = 1;  // select_tiles' u16 level-0 rows per block (hinted calls)
  // selst's tail words [ctrl][key min / max slots][hint flag] at this address
  // are zero: the previous tiled call's msel_reduce0h cleared them after
  // their last reader (fused_hist0), so select_launch skips the fill
  const uint64_t *sel_tail_zero = nullptr;
  const double *sel_mass = nullptr;
  // one-launch radial path (radial_mono): tile records + group fill, grid
  // barrier words; barrier generation / completion count carried across calls
  Buf mono, bar, mono_trace;
  Buf mH, mhint;  // radial_mono: its two level-0 histograms, its level-0 hint slots
  int64_t n_mhint = 0, n_mono_hinted = 0, n_mono_edge = 0;
  Buf mpedges, meue;  // radial_mono's edge speculation: the last edges, the per-edge sums
  bool medge_next = false;
  int medge_nq = 0;
  std::vector<double> mono_last_edges;
  Buf dscal, dlc;  // distributed radial_equaln: global scalars, per-rank group counts
  uint64_t bar_gen = 0, bar_done = 0;
  uint32_t bar_n = 0;  // grid size the barrier words were counted for (0: reset)
  prim::HostBuf mpin{nullptr, nullptr, 0, true};  // radial_mono's / fused_pack's results pack (mapped host)
  Buf pstage;              // the results pack staged in device memory (pack_complete)
  Buf pdone;               // fused_pack's completion counter (monotonic) ...
  uint64_t pack_done = 0;  // ... and its value after the last call
  // path counters (pbx_profile_path_stats): one-launch calls, of them
  // discarded (re-run by the multi-kernel path), multi-kernel calls
  int64_t n_mono = 0, n_mono_discard = 0, n_multi = 0;
  // tiled multi-kernel calls, of them with the level-0 histogram from
  // select_tiles (the hinted geometry held: no re-read of x)
  int64_t n_tiled_calls = 0, n_hinted = 0;
  bool hint_off = false;  // pbx_profile_set_level0_hint(handle, 0): every tiled call re-reads x
};

static void ensure_x(Profile &P, hipStream_t st);

// bins as uint32 by selection index for the consumers that read them
// (assign_gather leaves bytes by particle slot)
static void ensure_bins32(Profile &P, hipStream_t st) {
  if (!P.bins_in8) return;
  if (P.n > 0 && P.sel_nt) {
    uint32_t *b = (uint32_t *)P.bins.get(sizeof(uint32_t) * (size_t)P.n);
    hipLaunchKernelGGL((tile_compact<uint8_t, uint32_t>), dim3(P.sel_nt), dim3(TPB), 0, st,
                       (const uint8_t *)P.bins8.p, (const uint64_t *)P.kw.p,
                       (const uint32_t *)P.toff.p, b);
    PBX_HIP(hipGetLastError());
  }
  P.bins_in8 = false;
}

// exclusive scan of len u32 in place
static void scan_u32(Profile &P, hipStream_t st, uint32_t *a, int64_t len) {
  prim::scan_u32(P.tsum, st, a, len);
}

// one stable radix pass: kin -> kout (+ values)
template <typename K>
static void radix_pass(Profile &P, hipStream_t st, const K *kin, const int32_t *vin, int vm,
                       int64_t n, int shift, K *kout, int32_t *vout) {
  prim::radix_pass<K>(P.hist, P.tsum, st, kin, vin, vm, n, shift, kout, vout);
}

static void check_n(int64_t n) {
  if (n < 0) fail(PBX_ERR_VALUE, "negative length");
  if (n >= (int64_t)1 << 31) fail(PBX_ERR_VALUE, "profiles are limited to < 2^31 particles");
}

// min / max key of the current x (cached: the fused selection produces it
// for free; otherwise one grid-stride reduction)
static void minmax_of(Profile &P, hipStream_t st, uint64_t out[2]) {
  if (!P.mm_valid) {
    unsigned long long *mm = (unsigned long long *)P.minmax.get(16);
    unsigned long long h[2] = {~0ull, 0ull};
    PBX_HIP(hipMemcpyAsync(mm, h, 16, hipMemcpyHostToDevice, st));
    if (P.n) {
      unsigned grid = (unsigned)std::min<int64_t>(1024, (P.n + TPB - 1) / TPB);
      ensure_x(P, st);
      hipLaunchKernelGGL(minmax_keys, dim3(grid), dim3(TPB), 0, st, (const double *)P.x.p, P.n, mm);
      PBX_HIP(hipGetLastError());
    }
    PBX_HIP(hipMemcpyAsync(h, mm, 16, hipMemcpyDeviceToHost, st));
    PBX_HIP(hipStreamSynchronize(st));
    P.mm[0] = h[0];
    P.mm[1] = h[1];
    P.mm_valid = true;
  }
  out[0] = P.mm[0];
  out[1] = P.mm[1];
}

// equaln edges by multi-rank radix select (see msel_* kernels).  Window and
// rank semantics are those of the sort path: sorted_x[sorted_x >= bin_min],
// then [sorted_x <= bin_max] (bins.py:734-737; NaN fails both and a NaN
// bound keeps nothing; without bounds NaN sorts last and stays), then
// edges = s[0], s[int(i*m/nb)], s[m-1] (bins.py:738-744).
//
// Staged so the per-level digit histograms can be summed over ranks
// (distributed equaln): begin (global key range) -> per
// level: hist (this rank's keys) [+ all-reduce of the histogram] -> resolve
// (identical on every rank) -> edges.  Single GPU: the same stages back to
// back (equaln_select).
static void msel_begin(Profile &P, int64_t nbins, int has_min, double bin_min, int has_max,
                       double bin_max, uint64_t kmin, uint64_t kmax) {
  MselState &S = P.ms;
  S = MselState();
  S.nbins = nbins;
  S.nq = (int)nbins + 1;
  bool empty = false;
  uint64_t ka = 0ull, kb = ~0ull;
  if (has_min || has_max) {
    kb = ~0ull - 1;  // NaN keys never pass a comparison
    if (has_min) {
      if (bin_min != bin_min) empty = true;
      else ka = dkey(bin_min);
    }
    if (has_max) {
      if (bin_max != bin_max) empty = true;
      else kb = std::min<uint64_t>(kb, dkey(bin_max));
    }
  }
  const uint64_t lo = std::max<uint64_t>(ka, kmin);
  const uint64_t hi = std::min<uint64_t>(kb, kmax);
  if (empty || lo > hi) fail(PBX_ERR_VALUE, "index 0 is out of bounds for axis 0 with size 0");
  const uint64_t span = hi - lo;
  S.B = span ? 64 - __builtin_clzll(span) : 1;
  S.L = 1;
  S.wd[0] = std::min(S.B, MS0_BITS);
  for (int rem = S.B - S.wd[0]; rem > 0; rem -= MS_BITS) S.wd[S.L++] = std::min(rem, MS_BITS);
  S.ka = ka;
  S.kb = kb;
  S.lo = lo;
  S.next = 0;
  S.active = true;
}

static size_t msel_hbytes(const MselState &S) {
  return sizeof(uint32_t) * std::max<size_t>((size_t)S.nq * MS_DIG, MS0_DIG);
}

// this rank's digit histogram of `level` into H; returns the u32 count that
// a distributed caller sums over ranks
static int64_t msel_hist(Profile &P, hipStream_t st, int level) {
  MselState &S = P.ms;
  if (!S.active || level != S.next || level >= S.L)
    fail(PBX_ERR_VALUE, "radix select: level %d out of order", level);
  const int64_t n = P.n;
  const int nq = S.nq;
  const unsigned grid = (unsigned)std::min<int64_t>(2048, std::max<int64_t>(1, (n + TPB - 1) / TPB));
  uint32_t *H = (uint32_t *)P.msH.get(msel_hbytes(S));
  uint64_t *G = (uint64_t *)P.msG.get(sizeof(uint64_t) * (size_t)nq);
  int32_t *ng = (int32_t *)P.msNg.get(16);
  int s = S.B;
  for (int l = 0; l <= level; ++l) s -= S.wd[l];
  if (level == 0) {
    PBX_HIP(hipMemsetAsync(H, 0, msel_hbytes(S), st));
    const int g0 = (int)std::min<int64_t>(256, std::max<int64_t>(1, n / (MS0_TPB * 16)));
    uint32_t *rows = (uint32_t *)P.msRows.get(sizeof(uint32_t) * (size_t)g0 * MS0_DIG);
    if (n) {
      ensure_x(P, st);
      hipLaunchKernelGGL(msel_hist0, dim3(g0), dim3(MS0_TPB), 0, st, (const double *)P.x.p, n,
                         S.ka, S.kb, S.lo, s, rows);
      hipLaunchKernelGGL(msel_reduce0, dim3(MS0_DIG / TPB, 8), dim3(TPB), 0, st, rows, g0, H);
    }
    PBX_HIP(hipGetLastError());
    return MS0_DIG;
  }
  // per-wave key regions (msel_filter): the level-1 grid-stride pass gives
  // each wave at most steps * 64 * MS_U keys
  const int64_t steps = (n + (int64_t)grid * MS_STEP - 1) / ((int64_t)grid * MS_STEP);
  const int64_t cap = std::max<int64_t>(1, steps) * 64 * MS_U;
  const int64_t nw = (int64_t)grid * NWAVE;
  uint64_t *list = (uint64_t *)P.msL0.get(sizeof(uint64_t) * (size_t)(nw * cap));
  uint32_t *wc = (uint32_t *)P.msL1.get(sizeof(uint32_t) * (size_t)(nw * MS_MAXL));
  const int keep = level + 1 < S.L ? 1 : 0;
  ensure_x(P, st);
  if (level == 1)
    hipLaunchKernelGGL(msel_filter<true>, dim3(grid), dim3(TPB), 0, st, (const double *)P.x.p, n,
                       S.ka, S.kb, S.lo, list, (const uint32_t *)nullptr, cap, s, S.wd[level], G,
                       ng, H, keep, wc + nw * level);
  else
    hipLaunchKernelGGL(msel_filter<false>, dim3(grid), dim3(TPB), 0, st, (const double *)nullptr,
                       n, S.ka, S.kb, S.lo, list, (const uint32_t *)(wc + nw * (level - 1)), cap,
                       s, S.wd[level], G, ng, H, keep, wc + nw * level);
  PBX_HIP(hipGetLastError());
  return (int64_t)nq * MS_DIG;
}

// digits of `level` from the (summed) histogram; then the next level's groups
static void msel_resolve_level(Profile &P, hipStream_t st, int level) {
  MselState &S = P.ms;
  if (!S.active || level != S.next) fail(PBX_ERR_VALUE, "radix select: level %d out of order", level);
  const int nq = S.nq;
  uint32_t *H = (uint32_t *)P.msH.p;
  MsRank *R = (MsRank *)P.msR.get(sizeof(MsRank) * (size_t)nq);
  uint64_t *G = (uint64_t *)P.msG.get(sizeof(uint64_t) * (size_t)nq);
  int32_t *ng = (int32_t *)P.msNg.get(16);
  int64_t *m_dev = (int64_t *)P.msM.get(16);
  if (level == 0)
    hipLaunchKernelGGL(msel_resolve<MS0_DIG>, dim3(1), dim3(TPB), 0, st, H, ng, R, nq, 1,
                       S.nbins, S.wd[0], m_dev);
  else
    hipLaunchKernelGGL(msel_resolve<MS_DIG>, dim3(nq), dim3(TPB), 0, st, H, ng, R, nq, 0,
                       S.nbins, S.wd[level], m_dev);
  if (level + 1 < S.L) hipLaunchKernelGGL(msel_groups, dim3(1), dim3(1024), 0, st, R, nq, G, ng);
  PBX_HIP(hipGetLastError());
  S.next = level + 1;
}

static void msel_edges_out(Profile &P, hipStream_t st, double *h_edges, int64_t *n_edges) {
  MselState &S = P.ms;
  if (!S.active || S.next != S.L) fail(PBX_ERR_VALUE, "radix select: %d of %d levels resolved", S.next, S.L);
  const int nq = S.nq;
  double *de = (double *)P.edges.get(sizeof(double) * (size_t)nq);
  hipLaunchKernelGGL(msel_edges, dim3(ceil_div(nq, TPB)), dim3(TPB), 0, st,
                     (const MsRank *)P.msR.p, nq, S.lo, de);
  PBX_HIP(hipGetLastError());
  int64_t m = 0;
  PBX_HIP(hipMemcpyAsync(&m, P.msM.p, 8, hipMemcpyDeviceToHost, st));
  PBX_HIP(hipMemcpyAsync(h_edges, de, sizeof(double) * nq, hipMemcpyDeviceToHost, st));
  PBX_HIP(hipStreamSynchronize(st));
  S.active = false;
  if (m == 0) fail(PBX_ERR_VALUE, "index 0 is out of bounds for axis 0 with size 0");
  *n_edges = (m < 2) ? 2 : nq;
}

static void equaln_select(Profile &P, hipStream_t st, int64_t nbins, int has_min, double bin_min,
                          int has_max, double bin_max, double *h_edges, int64_t *n_edges) {
  uint64_t mm[2];
  minmax_of(P, st, mm);
  msel_begin(P, nbins, has_min, bin_min, has_max, bin_max, mm[0], mm[1]);
  for (int l = 0; l < P.ms.L; ++l) {
    msel_hist(P, st, l);
    msel_resolve_level(P, st, l);
  }
  msel_edges_out(P, st, h_edges, n_edges);
}

// ---- device-side stages shared by the entry points ----------------------
// bin ids + per-bin counts (P.counts, device) for nb bins of device edges
static void assign_device(Profile &P, hipStream_t st, const double *de, int64_t nb) {
  if (nb >= (int64_t)1 << 24) fail(PBX_ERR_VALUE, "too many bins");
  const int64_t n = P.n;
  unsigned long long *cnt = (unsigned long long *)P.counts.get(sizeof(uint64_t) * (size_t)(nb + 1));
  PBX_HIP(hipMemsetAsync(cnt, 0, sizeof(uint64_t) * (nb + 1), st));
  uint32_t *bins = (uint32_t *)P.bins.get(sizeof(uint32_t) * (size_t)(n ? n : 1));
  P.csrh_ready = false;
  P.bins_in8 = false;
  if (n) {
    size_t lds = ((nb + 1) <= LDS_EDGES ? sizeof(double) * (nb + 1) : 0) +
                 sizeof(uint32_t) * (nb + 1);
    if (lds > 150 * 1024) fail(PBX_ERR_VALUE, "too many bins for the device histogram (%lld)", (long long)nb);
    const uint32_t nt = ntiles_of(n);
    uint32_t *th = (nb < RADIX) ? (uint32_t *)P.csrh.get(sizeof(uint32_t) * (size_t)nt * RADIX)
                                : nullptr;
    // >= ~1024 blocks where the input allows it
    const uint32_t tpbk = std::min<uint32_t>(AS_TILES, std::max<uint32_t>(1, nt / 1024));
    ensure_x(P, st);
    launch_assign<false>(ceil_div(nt, tpbk), lds, st, (const double *)P.x.p, n, de, (int)nb, bins,
                         cnt, th, nt, tpbk, nullptr, nullptr, FusedStats{}, nullptr);
    P.csrh_ready = th != nullptr;
    PBX_HIP(hipGetLastError());
  }
  P.nb = nb;
  P.csr_ready = false;
}

// stable counting sort of the bin ids (nb = dropped) carrying indices -> P.perm
static void csr_device(Profile &P, hipStream_t st) {
  const int64_t n = P.n, nb = P.nb;
  if (P.csr_ready || !n) return;
  ensure_bins32(P, st);
  int bits = 0;
  while (((int64_t)1 << bits) <= nb) ++bits;
  uint32_t *ka = (uint32_t *)P.keys0.get(sizeof(uint32_t) * (size_t)n);
  uint32_t *kb = (uint32_t *)P.keys1.get(sizeof(uint32_t) * (size_t)n);
  int32_t *va = (int32_t *)P.perm.get(sizeof(int32_t) * (size_t)n);
  int32_t *vb = (int32_t *)P.vtmp.get(sizeof(int32_t) * (size_t)n);
  const uint32_t *kin = (const uint32_t *)P.bins.p;
  bool first = true;
  for (int shift = 0; shift < bits; shift += 8) {
    const bool last = shift + 8 >= bits;  // the sorted bin ids themselves are not needed
    if (first && P.csrh_ready) {  // bins < 256: assign_bins counted the only pass
      prim::radix_pass<uint32_t>(P.csrh, P.tsum, st, kin, nullptr, VAL_IOTA, n, shift,
                                 last ? nullptr : ka, va, true);
      P.csrh_ready = false;  // scanned in place: now offsets
      first = false;
    } else if (first) {
      radix_pass<uint32_t>(P, st, kin, nullptr, VAL_IOTA, n, shift, last ? nullptr : ka, va);
      first = false;
    } else {
      radix_pass<uint32_t>(P, st, ka, va, VAL_ARRAY, n, shift, last ? nullptr : kb, vb);
      std::swap(ka, kb);
      std::swap(va, vb);
    }
  }
  if ((void *)va != P.perm.p)
    PBX_HIP(hipMemcpyAsync(P.perm.p, va, sizeof(int32_t) * n, hipMemcpyDeviceToDevice, st));
  P.csr_ready = true;
}

// Launch the fused selection (mask + x + compaction + key range) of n
// particles into P.x / P.w / P.idx; the kept count and key range stay on
// the device (status words / selst).  Only the families' span is tiled.
// lazy: P.w / P.idx are not written (keep words + tile offsets instead, see
// select_onepass); the masses are then read from `mass` (the caller's device
// array, or a handle-owned staged copy) when the weights are needed.
// Returns the tile count.
struct SelPrep {  // a selection's parameters and output buffers (select_prep)
  SelectParams sp;
  int64_t hi = 0, span = 0;
  uint32_t nt = 0;
  const void *d_pos = nullptr, *d_mass = nullptr;
  double *xo = nullptr;
  uint64_t *kw = nullptr;
  uint32_t *toff = nullptr;
  uint16_t *kpre = nullptr;
};

// parameters, host staging and output buffers of a selection (no launch)
static SelPrep select_prep(Profile &P, hipStream_t st, const void *pos, const void *mass,
                           int64_t n, int on_device, int use_sphere, const double *sphere,
                           const int64_t *fam, int nfam, int ndim, bool lazy, int pos_f32,
                           int mass_f32, bool tiled) {
  check_n(n);
  if (ndim != 2 && ndim != 3) fail(PBX_ERR_VALUE, "ndim must be either 2 or 3");
  if (nfam < 0 || nfam > MAX_FAM) fail(PBX_ERR_VALUE, "at most %d family ranges", MAX_FAM);
  SelectParams sp{};
  sp.use_sphere = use_sphere;
  sp.ndim = ndim;
  sp.nfam = nfam;
  if (use_sphere) {
    sp.cx = sphere[0];
    sp.cy = sphere[1];
    sp.cz = sphere[2];
    sp.r2max = sphere[3];
    // (+0.0 or -0.0 centre: x - c == x for every x)
    sp.sphere_origin = ndim == 3 && sphere[0] == 0.0 && sphere[1] == 0.0 && sphere[2] == 0.0;
  }
  int64_t lo = 0, hi = n;  // the span holding every family member
  if (nfam > 0) {
    lo = n;
    hi = 0;
    for (int f = 0; f < nfam; ++f) {
      sp.fam_lo[f] = fam[2 * f];
      sp.fam_hi[f] = fam[2 * f + 1];
      const int64_t a = std::max<int64_t>(0, fam[2 * f]), b = std::min<int64_t>(n, fam[2 * f + 1]);
      if (b > a) {
        lo = std::min(lo, a);
        hi = std::max(hi, b);
      }
    }
    if (hi <= lo) lo = hi = 0;
  }
  sp.base = lo;
  const int64_t span = hi - lo;
  if (lazy && (pos_f32 || mass_f32)) fail(PBX_ERR_VALUE, "the lazy selection takes float64 arrays");
  sp.mass_f32 = mass_f32;
  const size_t ps = pos_f32 ? sizeof(float) : sizeof(double);
  const size_t ms = mass_f32 ? sizeof(float) : sizeof(double);
  const void *d_pos = pos, *d_mass = mass;
  P.x_missing = false;
  if (!on_device && n) {
    // Only the families' span [lo, hi) is read: only it crosses PCIe, at its
    // own offset in an n-sized buffer (the kernels index particles
    // absolutely), through pinned chunks (h2d_staged).
    // (lazy: kept for the selection's lifetime — a speculating tiled call may
    // have to recompute x from them later, ensure_x)
    Device &dv = current_device();
    char *tp = (char *)(lazy ? P.posst : P.keys0).get(ps * 3 * (size_t)n);
    if (span) h2d_staged(dv, tp + ps * 3 * (size_t)lo, (const char *)pos + ps * 3 * (size_t)lo,
                         ps * 3 * (size_t)span, st);
    d_pos = tp;
    if (mass) {
      Buf &mb = lazy ? P.mstage : P.keys1;  // lazy: kept for the selection's lifetime
      char *tm2 = (char *)mb.get(ms * (size_t)n);
      if (span) h2d_staged(dv, tm2 + ms * (size_t)lo, (const char *)mass + ms * (size_t)lo,
                           ms * (size_t)span, st);
      d_mass = tm2;
    }
  }
  const uint32_t nt = ntiles_of(span);
  // large lazy selections: tiled output, no look-back (tile offsets: fused_hist0)
  tiled = tiled && lazy && nt >= 1024;
  sp.tiled = tiled ? 1 : 0;
  const int64_t xlen = tiled ? (int64_t)nt * TILE : span;
  SelPrep r;
  r.xo = (double *)P.x.get(sizeof(double) * (size_t)(xlen ? xlen : 1));
  if (lazy) {
    r.kw = (uint64_t *)P.kw.get(sizeof(uint64_t) * (TILE / 64) * (size_t)std::max<uint32_t>(nt, 1));
    r.toff = (uint32_t *)P.toff.get(sizeof(uint32_t) * (size_t)std::max<uint32_t>(nt, 1));
    r.kpre = (uint16_t *)P.kpre.get(sizeof(uint16_t) * (TILE / 64) * (size_t)std::max<uint32_t>(nt, 1));
  }
  r.sp = sp;
  r.hi = hi;
  r.span = span;
  r.nt = nt;
  r.d_pos = d_pos;
  r.d_mass = d_mass;
  P.lazy = lazy;
  P.x_tiled = tiled && span;
  P.sel_base = lo;
  P.sel_span = span;
  P.sel_nt = nt;
  P.sel_mass = lazy ? (const double *)d_mass : nullptr;
  return r;
}

// grid of the fused level-0 kernels (fused_hist0, assign_gather, ...) over n_sel particles
static int fused_grid(int64_t n_sel) {
  return (int)std::min<int64_t>(256, std::max<int64_t>(1, n_sel / (MS0_TPB * 16)));
}

struct TileHist {  // select_tiles' hinted level-0 histogram (null hint: none)
  const SelHint *hint = nullptr;
  bool cold = false;  // the hint slot holds no geometry yet (a first call): sample one
  uint64_t ka = 0, kb = ~0ull;
  // the speculative assignment (tab non-null: wanted); select_launch fills
  // the rest and sets `spec` when it launched select_tiles<FAM, true>, and
  // `xs`: what x is recomputed from when that kernel stored none
  SpecArgs sa{};
  bool spec = false;
  XSrc xs{};
};

static uint32_t select_launch(Profile &P, hipStream_t st, const void *pos, const void *mass,
                              int64_t n, int on_device, int use_sphere, const double *sphere,
                              const int64_t *fam, int nfam, int ndim, bool lazy = false,
                              int pos_f32 = 0, int mass_f32 = 0, bool tiled = false,
                              TileHist *th = nullptr) {
  const SelPrep r = select_prep(P, st, pos, mass, n, on_device, use_sphere, sphere, fam, nfam, ndim,
                                lazy, pos_f32, mass_f32, tiled);
  const SelectParams &sp = r.sp;
  const uint32_t nt = r.nt;
  const int64_t hi = r.hi, span = r.span;
  const void *d_pos = r.d_pos, *d_mass = r.d_mass;
  // per-tile look-back status words + ticket / watchdog (selection scratch)
  // [stat nt][ctrl: ticket, watchdog][MM_SLOTS x (~min key, max key)][hint flag]: one zero fill
  const size_t nst = (size_t)nt + 1 + 2 * MM_SLOTS + 1;
  const size_t sbytes0 = P.selst.bytes;
  uint64_t *stat = (uint64_t *)P.selst.get(sizeof(uint64_t) * nst);
  // the persistent tiled selection reads none of the per-tile status words:
  // only the tail needs zeros, and it already holds them when the previous
  // tiled call cleared it at this address (same buffer, same nt)
  const bool persist = span && !pos_f32 && nt >= 1024 && lazy && P.x_tiled;
  const bool tail_zero = persist && P.selst.bytes == sbytes0 &&
                         P.sel_tail_zero == stat + nt;
  P.sel_tail_zero = nullptr;
  uint32_t *ctrl = (uint32_t *)(stat + nt);
  double *xo = r.xo;
  double *wo = nullptr;
  int32_t *io = nullptr;
  uint64_t *kw = r.kw;
  uint32_t *toff = r.toff;
  if (!lazy) {
    wo = (double *)P.w.get(sizeof(double) * (size_t)(span ? span : 1));
    io = (int32_t *)P.idx.get(sizeof(int32_t) * (size_t)(span ? span : 1));
  }
  unsigned long long *mm = (unsigned long long *)(stat + nt + 1);
  if (!persist) PBX_HIP(hipMemsetAsync(stat, 0, sizeof(uint64_t) * nst, st));
  else if (!tail_zero) PBX_HIP(hipMemsetAsync(stat + nt, 0, sizeof(uint64_t) * (nst - nt), st));
  if (span) {
    auto go = [&](auto kern, int bt, auto tp) {
      using T = decltype(tp);
      hipLaunchKernelGGL(kern, dim3(nt), dim3(bt), 0, st, (const T *)d_pos, d_mass, hi, sp, stat,
                         ctrl, xo, wo, io, mm, kw, toff, r.kpre);
    };
    if (pos_f32) {  // float32 snapshots: eager only
      if (nt < 1024) go(select_onepass<1024, false, float>, 1024, 0.0f);
      else go(select_onepass<TPB, false, float>, TPB, 0.0f);
    } else if (nt < 1024) {
      if (lazy) go(select_onepass<1024, true, double>, 1024, 0.0);
      else go(select_onepass<1024, false, double>, 1024, 0.0);
    } else {
      // 512-thread tiles (8 particles per lane, 64 VGPRs: 8 waves per SIMD):
      // 244 -> 233 us at 64M against 256 threads (16 per lane, 136 VGPRs, 3 waves)
      if (lazy && P.x_tiled) {  // persistent tiles (+ the hinted level-0 histogram)
        const int G0 = fused_grid(span);
        const unsigned G1 = (unsigned)(SH_K * (G0 - 1));
        // tiles of the largest select block (tile_range of the assign block, split SH_K ways)
        const uint64_t tab = ((uint64_t)nt + (G0 - 1) - 1) / (G0 - 1);
        const uint64_t tsel = (tab + SH_K - 1) / SH_K + 1;
        const uint32_t rsub = (uint32_t)std::max<uint64_t>(
            1, std::min<uint64_t>(SH_RSUB_MAX, (tsel + SH_TMAX - 1) / SH_TMAX));
        P.sel_rsub = rsub;
        uint32_t *rows16 = nullptr;
        if (th && th->hint)
          rows16 = (uint32_t *)P.srows.get(sizeof(uint32_t) * (size_t)G1 * rsub * (MS0_DIG / 2));
        uint32_t *wc = (uint32_t *)P.swc.get(sizeof(uint32_t) * (size_t)nt * SH_NW);
        uint32_t *bt = (uint32_t *)P.sbt.get(sizeof(uint32_t) * (size_t)G1);
        SpecArgs sa{};
        const bool spec = th && th->sa.tab && rows16;
        if (spec) {  // select_tiles bins with the stored table too
          sa = th->sa;
          sa.mass = (const double *)d_mass;
          sa.bins = (uint8_t *)P.bins8.get((size_t)nt * TILE);
          sa.th = (uint32_t *)P.csrh.get(sizeof(uint32_t) * (size_t)nt * (sa.nb + 1));
          sa.slab = (double *)P.sslab.get(sizeof(double) * (size_t)G1 * std::max(1, sa.fs.nm * sa.nb));
          sa.rec = (AgRec *)P.srec.get(sizeof(AgRec) * ((size_t)nt * TILE / SPEC_LIST + 1));
          sa.rbase = (uint32_t *)P.sspec.get(sizeof(uint32_t) * 2 * (size_t)G1);
          sa.rn = sa.rbase + G1;
          // (zeroed once; fused_resolve resets it after reading it)
          if (!P.sflag.p) {
            P.sflag.get(sizeof(uint32_t));
            PBX_HIP(hipMemsetAsync(P.sflag.p, 0, sizeof(uint32_t), st));
          }
          sa.flag = (uint32_t *)P.sflag.p;
          th->sa = sa;
        }
        if (th) {
          th->spec = spec;
          th->xs = XSrc{spec ? (const double *)d_pos : nullptr, hi, sp, xo, kw};
        }
        if (spec) {  // (x missing until the call's pack says it missed: x rebuilt)
          P.x_missing = true;
          P.xsrc = th->xs;
        }
        if (th && th->hint && th->cold && rows16) {  // a first call: a sampled geometry
          if (!P.shs.p) {
            P.shs.get(sizeof(uint64_t) * 3);
            PBX_HIP(hipMemsetAsync(P.shs.p, 0, sizeof(uint64_t) * 3, st));
          }
          const uint32_t S = (uint32_t)std::min<int64_t>(32768, std::max<int64_t>(1, span / 64));
          uint64_t kub = 0;  // the Sphere's bound on every kept x (|c| + R, a few ulps up)
          if (sp.use_sphere || sp.sphere_origin) {
            const double c = std::sqrt(sp.cx * sp.cx + sp.cy * sp.cy + sp.cz * sp.cz);
            const double ub = (c + std::sqrt(sp.r2max)) * (1.0 + 1e-12);
            if (std::isfinite(ub)) kub = dkey(ub);
          }
          unsigned long long *smm = (unsigned long long *)P.shs.p;
          auto sk = sp.nfam > 1 ? sample_hint<true> : sample_hint<false>;
          hipLaunchKernelGGL(sk, dim3(ceil_div(S, SMP_BT * SMP_PER)), dim3(SMP_BT), 0, st, (const double *)d_pos,
                             hi, sp, span, S, th->ka, th->kb, kub, smm, (unsigned *)(smm + 2),
                             (SelHint *)th->hint);
        }
        auto kern = spec ? (sp.nfam > 1 ? select_tiles<true, true> : select_tiles<false, true>)
                         : (sp.nfam > 1 ? select_tiles<true, false> : select_tiles<false, false>);
        hipLaunchKernelGGL(kern, dim3(G1),
                           dim3(SH_BT), 0, st, (const double *)d_pos, hi,
                           sp, nt, (uint32_t)G0, xo, kw, r.kpre, wc, toff, bt, mm,
                           th ? th->hint : nullptr, th ? th->ka : 0ull, th ? th->kb : ~0ull, rows16, rsub,
                           (uint32_t *)(mm + 2 * MM_SLOTS), sa);
      } else if (lazy) go(select_onepass<512, true, double>, 512, 0.0);
      else go(select_onepass<512, false, double>, 512, 0.0);
    }
    PBX_HIP(hipGetLastError());
  }
  return nt;
}

// materialise a lazy selection's weights / original indices
static void ensure_w(Profile &P, hipStream_t st) {
  if (!P.lazy || P.w_ready) return;
  double *wo = (double *)P.w.get(sizeof(double) * (size_t)std::max<int64_t>(P.n, 1));
  if (P.sel_nt)
    hipLaunchKernelGGL(sel_materialize, dim3(P.sel_nt), dim3(TPB), 0, st, (const uint64_t *)P.kw.p,
                       (const uint32_t *)P.toff.p, P.sel_base, P.sel_mass, wo, (int32_t *)nullptr);
  PBX_HIP(hipGetLastError());
  P.w_ready = true;
}

static void ensure_idx(Profile &P, hipStream_t st) {
  if (!P.lazy || P.idx_ready) return;
  int32_t *io = (int32_t *)P.idx.get(sizeof(int32_t) * (size_t)std::max<int64_t>(P.n, 1));
  if (P.sel_nt)
    hipLaunchKernelGGL(sel_materialize, dim3(P.sel_nt), dim3(TPB), 0, st, (const uint64_t *)P.kw.p,
                       (const uint32_t *)P.toff.p, P.sel_base, (const double *)nullptr,
                       (double *)nullptr, io);
  PBX_HIP(hipGetLastError());
  P.idx_ready = true;
}

// compact a tiled selection's x (consumers that index x by selection index)
static void ensure_x(Profile &P, hipStream_t st) {
  if (P.x_missing) {  // a speculation hit stored no x: recompute it from the positions
    const uint32_t tpb = 4;
    XSrc xs = P.xsrc;
    xs.x = (double *)P.x.p;
    xs.kw = (const uint64_t *)P.kw.p;
    if (P.sel_nt)
      hipLaunchKernelGGL(xsrc_kernel, dim3(ceil_div(P.sel_nt, tpb)), dim3(TPB), 0, st, xs,
                         P.sel_nt, tpb);
    PBX_HIP(hipGetLastError());
    P.x_missing = false;
  }
  if (!P.x_tiled) return;
  double *xc = (double *)P.xc.get(sizeof(double) * (size_t)std::max<int64_t>(P.n, 1));
  if (P.sel_nt && P.n)
    hipLaunchKernelGGL((tile_compact<double, double>), dim3(P.sel_nt), dim3(TPB), 0, st,
                       (const double *)P.x.p, (const uint64_t *)P.kw.p, (const uint32_t *)P.toff.p,
                       xc);
  PBX_HIP(hipGetLastError());
  std::swap(P.x, P.xc);
  P.x_tiled = false;
}

// the handle's state after a selection of `kept` particles (key range in P.mm)
static void select_commit(Profile &P, int64_t kept) {
  P.w_ready = P.idx_ready = !P.lazy;
  P.mm_valid = true;
  P.n = kept;
  P.has_w = true;
  P.has_idx = true;
  P.csr_ready = false;
  P.csrh_ready = false;
  P.ms.active = false;
  P.nb = -1;
}

// device pointer of a per-element source: 0 = x, 1 = selection weights,
// 2 = host array of n doubles (staged), 3 = device array per ORIGINAL particle
static const double *resolve_src(Profile &P, hipStream_t st, int which, const double *hp,
                                 Buf &stage) {
  const int64_t n = P.n;
  if (which == 0) {
    ensure_x(P, st);
    return (const double *)P.x.p;
  }
  if (which == 1) {
    if (!P.has_w) fail(PBX_ERR_VALUE, "profile has no selection weights");
    ensure_w(P, st);
    return (const double *)P.w.p;
  }
  if (which == 2) {
    if (!hp && n) fail(PBX_ERR_VALUE, "host array is NULL");
    double *dp = (double *)stage.get(sizeof(double) * (size_t)(n ? n : 1));
    if (n) h2d_staged(current_device(), dp, hp, sizeof(double) * n, st);  // (pinned chunks)
    return dp;
  }
  if (which == 3) {  // device array per ORIGINAL particle (e.g. a tree potential)
    if (!hp && n) fail(PBX_ERR_VALUE, "device array is NULL");
    if (!P.has_idx) return hp;
    ensure_idx(P, st);
    double *dp = (double *)stage.get(sizeof(double) * (size_t)(n ? n : 1));
    if (n)
      hipLaunchKernelGGL(gather_by_idx, dim3(ceil_div(n, TPB)), dim3(TPB), 0, st, hp,
                         (const int32_t *)P.idx.p, n, dp);
    return dp;
  }
  fail(PBX_ERR_VALUE, "bad source selector %d", which);
}

// per-bin sums of the requested columns into acc (nb x NMOM doubles, device)
static void moments_device(Profile &P, hipStream_t st, int f_src, const double *h_f, Buf &fstage,
                           int w_src, const double *h_w, Buf &wstage, uint32_t cols,
                           double *acc) {
  const int64_t n = P.n, nb = P.nb;
  auto src = [&](int which, const double *hp, Buf &stage) -> const double * {
    return resolve_src(P, st, which, hp, stage);
  };
  const double *f = src(f_src, h_f, fstage);
  const double *w = (w_src < 0) ? nullptr : src(w_src, h_w, wstage);
  const int64_t len = nb * NMOM;
  PBX_HIP(hipMemsetAsync(acc, 0, sizeof(double) * len, st));
  ensure_bins32(P, st);
  if (n && nb > 0) {
    // <= 1024 blocks (4 per CU) stride over the tiles
    uint32_t nt = std::min<uint32_t>(ntiles_of(n), 1024u);
    const bool in_lds = nb <= LDS_MOM_BINS;
    double *slab = in_lds ? (double *)P.slab.get(sizeof(double) * (size_t)nt * len) : nullptr;
    size_t lds = in_lds ? sizeof(double) * (size_t)len : 0;
    auto launch = [&](auto wm, auto lds_t) {
      hipLaunchKernelGGL((moments_kernel<decltype(wm)::value, decltype(lds_t)::value>), dim3(nt),
                         dim3(TPB), lds, st, (const uint32_t *)P.bins.p, f, w, n, (int)nb, cols,
                         slab, acc);
    };
    using W1 = std::integral_constant<int, 1>;
    using W0 = std::integral_constant<int, 0>;
    if (w && in_lds) launch(W1{}, std::true_type{});
    else if (w) launch(W1{}, std::false_type{});
    else if (in_lds) launch(W0{}, std::true_type{});
    else launch(W0{}, std::false_type{});
    PBX_HIP(hipGetLastError());
    if (in_lds) {
      double *part = (double *)P.slabp.get(sizeof(double) * (size_t)SLAB_G * len);
      hipLaunchKernelGGL(reduce_slab_part, dim3(ceil_div(len, TPB), SLAB_G), dim3(TPB), 0, st,
                         slab, (int64_t)nt, len, part);
      hipLaunchKernelGGL(reduce_slab_final, dim3(ceil_div(len, TPB)), dim3(TPB), 0, st, part,
                         len, acc);
      PBX_HIP(hipGetLastError());
    }
  }
}

// per-bin percentiles of a field (Percentile.__call__ per bin,
// proarray.py:700-722) into out (nb x nq doubles, device)
static void percentiles_device(Profile &P, hipStream_t st, int f_src, const double *h_f,
                               int w_src, const double *h_w, int absval, int nq,
                               const double *h_q, double *out) {
  const int64_t n = P.n, nb = P.nb;
  const double *f = resolve_src(P, st, f_src, h_f, P.field);
  const double *w = (w_src < 0) ? nullptr : resolve_src(P, st, w_src, h_w, P.weight);
  double *dq = (double *)P.pq.get(sizeof(double) * (size_t)nq);
  PBX_HIP(hipMemcpyAsync(dq, h_q, sizeof(double) * nq, hipMemcpyHostToDevice, st));
  int64_t *off = (int64_t *)P.poff.get(sizeof(int64_t) * (size_t)(nb + 1));
  hipLaunchKernelGGL(counts_to_offsets, dim3(1), dim3(1024), 0, st, (const uint64_t *)P.counts.p,
                     nb, off);
  int32_t *e = nullptr;
  if (n) {
    uint64_t *ka = (uint64_t *)P.pk0.get(sizeof(uint64_t) * (size_t)n);
    uint64_t *kb = (uint64_t *)P.pk1.get(sizeof(uint64_t) * (size_t)n);
    int32_t *va = (int32_t *)P.pv0.get(sizeof(int32_t) * (size_t)n);
    int32_t *vb = (int32_t *)P.pv1.get(sizeof(int32_t) * (size_t)n);
    hipLaunchKernelGGL(pct_keys, dim3(ceil_div(n, TPB)), dim3(TPB), 0, st, f, n, absval, ka);
    // value key, 8 bits at a time (stable; first pass seeds the element ids)
    for (int shift = 0; shift < 64; shift += 8) {
      const bool last = shift + 8 >= 64;
      radix_pass<uint64_t>(P, st, ka, shift == 0 ? nullptr : va, shift == 0 ? VAL_IOTA : VAL_ARRAY,
                           n, shift, last ? nullptr : kb, vb);
      std::swap(ka, kb);
      std::swap(va, vb);
    }
    // then the bin id (stable: value order kept inside each bin)
    uint32_t *ba = (uint32_t *)P.pbk.get(sizeof(uint32_t) * 2 * (size_t)n);
    uint32_t *bb = ba + n;
    ensure_bins32(P, st);
    hipLaunchKernelGGL(gather_bin_ids, dim3(ceil_div(n, TPB)), dim3(TPB), 0, st,
                       (const uint32_t *)P.bins.p, va, n, ba);
    int bits = 0;
    while (((int64_t)1 << bits) <= nb) ++bits;
    for (int shift = 0; shift < bits; shift += 8) {
      const bool last = shift + 8 >= bits;
      radix_pass<uint32_t>(P, st, ba, va, VAL_ARRAY, n, shift, last ? nullptr : bb, vb);
      std::swap(ba, bb);
      std::swap(va, vb);
    }
    e = va;
  }
  if (nb > 0) {
    double *cdf = (double *)P.pcdf.get(sizeof(double) * (size_t)(n ? n : 1));
    hipLaunchKernelGGL(pct_bins, dim3((unsigned)nb), dim3(TPB), 0, st, (const int32_t *)e, off, f,
                       w, absval, (const double *)dq, nq, cdf, out);
    PBX_HIP(hipGetLastError());
  }
}

// ---- one-launch radial path (radial_mono) -------------------------------
// Completion of a call whose last kernel stores a tag into mapped host
// memory (radial_mono, fused_pack): the tag is polled (a stream sync wakes
// the host several microseconds after the kernel ends); the stream is
// queried now and then, so a call that ends without its tag (a discarded
// radial_mono, a fault) ends the wait too.  Returns whether the tag arrived.
// (The spin beats a stream sync by 1-2 us of wall time per call.)
static bool wait_tag(hipStream_t st, const double *word, uint64_t want) {
  volatile const uint64_t *tag = (volatile const uint64_t *)word;
  for (uint32_t k = 1; *tag == ~0ull; ++k) {
    if ((k & 1023u) == 0) {
      const hipError_t q = hipStreamQuery(st);
      if (q == hipSuccess) break;
      if (q != hipErrorNotReady) PBX_HIP(q);
    }
    __builtin_ia32_pause();
  }
  if (*tag != want) PBX_HIP(hipStreamSynchronize(st));
  const bool ok = *tag == want;
  __atomic_thread_fence(__ATOMIC_ACQUIRE);  // the pack's words are read after the tag
  return ok;
}

// Tiles (= blocks) the one-launch path may use on a device: every block must
// be resident at once, one 1024-thread block per CU (0: never)
static uint32_t mono_max_tiles(int dev) {
  static std::mutex mu;
  static std::vector<int> cache;
  std::lock_guard<std::mutex> lk(mu);
  if ((int)cache.size() <= dev) cache.resize((size_t)dev + 1, -1);
  if (cache[(size_t)dev] < 0) {
    int cus = 0, per = 0;
    PBX_HIP(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
    PBX_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(
        &per, reinterpret_cast<const void *>(&radial_mono), MONO_BT, 0));
    cache[(size_t)dev] = per >= 1 ? std::min<int>(cus, (int)MONO_MAXT) : 0;
  }
  return (uint32_t)cache[(size_t)dev];
}

// the families' span of n particles (select_prep's rule)
static int64_t family_span(int64_t n, const int64_t *fam, int nfam) {
  if (nfam <= 0) return n;
  int64_t lo = n, hi = 0;
  for (int f = 0; f < nfam; ++f) {
    const int64_t a = std::max<int64_t>(0, fam[2 * f]), b = std::min<int64_t>(n, fam[2 * f + 1]);
    if (b > a) {
      lo = std::min(lo, a);
      hi = std::max(hi, b);
    }
  }
  return hi > lo ? hi - lo : 0;
}

// Runs the step as one launch when the selection fits (<= one tile per CU,
// bins < 256, the fused sums in LDS); returns the pinned results pack
// ([ctl][edges][counts][sums], the fused_pack layout) after ONE sync, or
// null when the path does not apply or the call was discarded (a block gave
// up at a barrier: the barrier words are reset and the caller runs the
// multi-kernel path, which recomputes everything).
static double *radial_mono_run(Profile &P, hipStream_t st, const void *pos, const void *mass,
                               int64_t n, int on_device, int use_sphere, const double *sphere,
                               const int64_t *fam, int nfam, int ndim, int64_t nbins, uint64_t ka,
                               uint64_t kb, bool empty_bounds, const FusedStats &fs, int *nsum) {
  check_n(n);
  const int nb = (int)nbins, nq = nb + 1, macc = fs.nm * nb;
  if (nb >= RADIX || ndim < 2 || ndim > 3 || nfam < 0 || nfam > MAX_FAM) return nullptr;
  if (sizeof(double) * (size_t)macc + sizeof(uint32_t) * MONO_NW * RADIX > sizeof(uint16_t) * MONO_DIG)
    return nullptr;
  const uint32_t nt = ntiles_of(family_span(n, fam, nfam));
  if (nt == 0 || nt > mono_max_tiles(P.device)) return nullptr;
  const SelPrep r = select_prep(P, st, pos, mass, n, on_device, use_sphere, sphere, fam, nfam, ndim,
                                /*lazy=*/true, 0, 0, /*tiled=*/false);
  const int64_t ns = std::max<int64_t>(r.span, 1);
  MonoArgs a{};
  a.pos = (const double *)r.d_pos;
  a.mass = (const double *)r.d_mass;
  a.n_hi = r.hi;
  a.sp = r.sp;
  a.ka = ka;
  a.kb = kb;
  a.empty_bounds = empty_bounds ? 1 : 0;
  a.nb = nb;
  a.nq = nq;
  a.nbins = nbins;
  a.fs = fs;
  char *scr = (char *)P.mono.get(sizeof(MonoRec) * MONO_MAXT + sizeof(uint32_t) * RADIX);
  a.rec = (MonoRec *)scr;
  a.gcnt = (uint32_t *)(scr + sizeof(MonoRec) * MONO_MAXT);
  const bool fresh_h = !P.mH.p;
  a.H = (uint32_t *)P.mH.get(sizeof(uint32_t) * 2 * MS0_DIG);
  a.H2 = a.H + MS0_DIG;
  if (!P.mhint.p) {
    P.mhint.get(2 * sizeof(SelHint));
    PBX_HIP(hipMemsetAsync(P.mhint.p, 0, 2 * sizeof(SelHint), st));
  }
  SelHint *mh = (SelHint *)P.mhint.p;
  a.hin = P.hint_off ? nullptr : mh + (P.n_mhint & 1);
  a.hout = mh + ((P.n_mhint + 1) & 1);
  a.seg = (uint64_t *)P.fseg.get(sizeof(uint64_t) * (size_t)ns);
  a.x = r.xo;
  a.kw = r.kw;
  a.toff = r.toff;
  a.bins = (uint32_t *)P.bins.get(sizeof(uint32_t) * (size_t)ns);
  P.bins_in8 = false;
  a.perm = (int32_t *)P.perm.get(sizeof(int32_t) * (size_t)ns);
  a.edges = (double *)P.edges.get(sizeof(double) * (size_t)nq);
  a.th = (uint32_t *)P.csrh.get(sizeof(uint32_t) * RADIX * (size_t)nt);
  a.slab = macc ? (double *)P.fslab.get(sizeof(double) * (size_t)nt * macc) : nullptr;
  a.counts = (unsigned long long *)P.counts.get(sizeof(uint64_t) * (size_t)(nb + 1));
  constexpr int NC = (int)(sizeof(FusedCtl) / sizeof(double));
  const int ntot = NC + nq + nb + macc;
  // the pack lands in mapped host memory: the kernel's stores are the
  // readback (no copy on the stream), the host reads it after the sync
  double *hp = (double *)P.mpin.get(sizeof(double) * (size_t)(ntot + 1));
  a.pack = (double *)P.mpin.dev;
  a.stage = (double *)P.pstage.get(sizeof(double) * (size_t)ntot);
  hp[ntot] = __builtin_bit_cast(double, ~0ull);
  if (P.bar_n != nt || !P.bar.p || fresh_h) {  // counters are counted for one grid size
    P.bar.get(sizeof(uint64_t) * BAR_WORDS);
    PBX_HIP(hipMemsetAsync(P.bar.p, 0, sizeof(uint64_t) * BAR_WORDS, st));
    // (after a discarded call H / H2 may hold counts: both zero on entry)
    PBX_HIP(hipMemsetAsync(a.H, 0, sizeof(uint32_t) * 2 * MS0_DIG, st));
    P.bar_gen = P.bar_done = 0;
    P.bar_n = nt;
  }
  a.bar = (uint64_t *)P.bar.p;
  static const bool trace_env = [] {
    const char *v = std::getenv("PBX_MONO_TRACE");
    return v && v[0] == '1';
  }();
  a.trace = trace_env ? (uint64_t *)P.mono_trace.get(sizeof(uint64_t) * 8 * nt) : nullptr;
  a.gen0 = P.bar_gen;
  a.done_target = P.bar_done + nt;
  // edge speculation: the previous call's edges (every call leaves its own in
  // P.mpedges) and the per-edge sums (zero on entry and exit); tried when the
  // last two one-launch calls' edges were identical
  if (!P.mpedges.p) {
    P.mpedges.get(sizeof(double) * RADIX);
    PBX_HIP(hipMemsetAsync(P.mpedges.p, 0, sizeof(double) * RADIX, st));
    P.meue.get(sizeof(uint32_t) * (2 * RADIX + 1));
    PBX_HIP(hipMemsetAsync(P.meue.p, 0, sizeof(uint32_t) * (2 * RADIX + 1), st));
  }
  a.pedges = (double *)P.mpedges.p;
  a.eU = (uint32_t *)P.meue.p;
  a.eE = a.eU + RADIX + 1;
  a.eg = (P.medge_next && nq == P.medge_nq) ? 1 : 0;
  hipLaunchKernelGGL(radial_mono, dim3(nt), dim3(MONO_BT), 0, st, a);
  PBX_HIP(hipGetLastError());
  P.bar_done += nt;
  ++P.n_mono;
  ++P.n_mhint;
  if (!wait_tag(st, hp + ntot, a.gen0)) {
    P.bar_n = 0;  // discarded: zero the barrier words before the next call
    P.medge_next = false;
    ++P.n_mono_discard;
    if (P.mpedges.p) {  // (the edge sums may hold counts)
      PBX_HIP(hipMemsetAsync(P.meue.p, 0, sizeof(uint32_t) * (2 * RADIX + 1), st));
    }
    return nullptr;
  }
  {  // the barriers the call used (skipped phases take none); edges for the next call
    const FusedCtl *hc = (const FusedCtl *)hp;
    P.bar_gen += (uint64_t)((hc->spec >> 8) & 0xff);
    if (hc->spec & SPEC_EDGE) ++P.n_mono_edge;
    const double *he = hp + NC;
    P.medge_next = (int)P.mono_last_edges.size() == nq &&
                   std::memcmp(P.mono_last_edges.data(), he, sizeof(double) * nq) == 0;
    P.mono_last_edges.assign(he, he + nq);
    P.medge_nq = nq;
  }
  if (a.trace) {  // per phase: min / max over blocks of the stamp, relative to the earliest start
    std::vector<uint64_t> tr((size_t)8 * nt);
    PBX_HIP(hipMemcpy(tr.data(), a.trace, sizeof(uint64_t) * 8 * nt, hipMemcpyDeviceToHost));
    uint64_t t0 = ~0ull;
    for (uint32_t b = 0; b < nt; ++b) t0 = std::min(t0, tr[(size_t)b * 8]);
    std::fprintf(stderr, "[mono] nt=%u", nt);
    for (int k = 0; k < 8; ++k) {
      uint64_t lo = ~0ull, hi = 0;
      for (uint32_t b = 0; b < nt; ++b) {
        lo = std::min(lo, tr[(size_t)b * 8 + k] - t0);
        hi = std::max(hi, tr[(size_t)b * 8 + k] - t0);
      }
      std::fprintf(stderr, " p%d %.2f-%.2fus", k, lo / 100.0, hi / 100.0);
    }
    std::fprintf(stderr, "\n");
  }
  P.csrh_ready = false;
  if (((const FusedCtl *)hp)->hint) ++P.n_mono_hinted;
  *nsum = macc;
  return hp;
}

static Profile &as_profile(void *h) {
  if (!h) fail(PBX_ERR_VALUE, "null profile handle");
  Profile *p = (Profile *)h;
  int dev = current_device().id;
  if (p->device != dev) fail(PBX_ERR_VALUE, "profile belongs to device %d", p->device);
  return *p;
}

}  // namespace prof
}  // namespace pbx

using namespace pbx;
using namespace pbx::prof;

extern "C" {

int pbx_profile_create(void **handle) {
  return guard([&] {
    Device &d = current_device();
    Profile *p = new Profile();
    p->device = d.id;
    *handle = p;
  });
}

int pbx_profile_destroy(void *handle) {
  return guard([&] {
    if (!handle) return;
    Profile *p = (Profile *)handle;
    current_device();
    Buf *all[] = {&p->x, &p->w, &p->idx, &p->bins, &p->perm, &p->keys0, &p->keys1, &p->vtmp,
                  &p->hist, &p->tsum, &p->edges, &p->counts, &p->minmax, &p->slab, &p->acc,
                  &p->field, &p->weight, &p->ranks, &p->bounds, &p->msH, &p->msR, &p->msG,
                  &p->msNg, &p->msM, &p->msRows, &p->msL0, &p->msL1, &p->msCnt, &p->csrh, &p->slabp, &p->selst, &p->accs,
                  &p->pk0, &p->pk1, &p->pv0, &p->pv1, &p->pbk, &p->pcdf, &p->poff, &p->pq, &p->pout,
                  &p->fctl, &p->fseg, &p->fgrp, &p->fslab, &p->fpack, &p->frec, &p->fblk,
                  &p->bins8, &p->kw, &p->toff, &p->mstage, &p->xc, &p->kpre, &p->shint, &p->shs, &p->srows,
                  &p->swc, &p->sbt, &p->mono, &p->bar,
                  &p->mono_trace, &p->dscal, &p->dlc, &p->pdone, &p->pstage, &p->mH,
                  &p->mhint, &p->stab, &p->srec, &p->sspec, &p->sslab, &p->sflag, &p->posst,
                  &p->slteq, &p->mpedges, &p->meue};
    for (Buf *b : all) b->release();
    p->pin.release();
    p->mpin.release();
    delete p;
  });
}

int pbx_profile_level0_stats(void *handle, int64_t *out) {
  return guard([&] {
    Profile &P = as_profile(handle);
    if (!out) fail(PBX_ERR_VALUE, "null output");
    out[0] = P.n_tiled_calls;
    out[1] = P.n_hinted;
  });
}

int pbx_profile_spec_stats(void *handle, int64_t *out) {
  return guard([&] {
    Profile &P = as_profile(handle);
    if (!out) fail(PBX_ERR_VALUE, "null output");
    out[0] = P.n_spec;
    out[1] = P.n_spec_hit;
    out[2] = P.n_edge_hit;
  });
}

int pbx_profile_set_source_stable(void *handle, int stable) {
  return guard([&] {
    Profile &P = as_profile(handle);
    P.src_stable = stable != 0;
  });
}

int pbx_profile_set_level0_hint(void *handle, int enabled) {
  return guard([&] {
    Profile &P = as_profile(handle);
    if (enabled == 2) {  // forget the earlier calls: the next call is a first call
      Device &d = current_device();
      std::lock_guard<std::mutex> lk(d.mu);
      P.hint_off = false;
      P.n_tiled = 0;
      P.n_mhint = 0;
      P.spec_next = P.edge_next = P.medge_next = false;
      P.last_edges.clear();
      P.mono_last_edges.clear();
      if (P.shint.p) PBX_HIP(hipMemsetAsync(P.shint.p, 0, P.shint.bytes, d.stream));
      if (P.mhint.p) PBX_HIP(hipMemsetAsync(P.mhint.p, 0, P.mhint.bytes, d.stream));
      return;
    }
    P.hint_off = enabled == 0;
  });
}

int pbx_profile_mono_stats(void *handle, int64_t *out) {
  return guard([&] {
    Profile &P = as_profile(handle);
    if (!out) fail(PBX_ERR_VALUE, "null output");
    out[0] = P.n_mono;
    out[1] = P.n_mono_hinted;
    out[2] = P.n_mono_edge;
  });
}

int pbx_profile_path_stats(void *handle, int64_t *out) {
  return guard([&] {
    Profile &P = as_profile(handle);
    if (!out) fail(PBX_ERR_VALUE, "null output");
    out[0] = P.n_mono;
    out[1] = P.n_mono_discard;
    out[2] = P.n_multi;
  });
}

int pbx_profile_set_x(void *handle, const double *h_x, int64_t n) {
  return guard([&] {
    Profile &P = as_profile(handle);
    check_n(n);
    Device &d = current_device();
    std::lock_guard<std::mutex> lk(d.mu);
    double *x = (double *)P.x.get(sizeof(double) * (size_t)(n ? n : 1));
    if (n) h2d_staged(d, x, h_x, sizeof(double) * n, d.stream);  // (through pinned chunks)
    P.n = n;
    P.has_w = false;
    P.has_idx = false;
    P.lazy = false;
    P.x_tiled = false;
    P.x_missing = false;
    P.csr_ready = false;
    P.csrh_ready = false;
    P.ms.active = false;
    P.mm_valid = false;
    P.nb = -1;
  });
}

int pbx_profile_select(void *handle, const double *pos, const double *mass, int64_t n,
                       int on_device, int use_sphere, const double *sphere, const int64_t *fam,
                       int nfam, int ndim, int64_t *n_kept) {
  return pbx_profile_select_typed(handle, pos, PBX_F64, mass, PBX_F64, n, on_device, use_sphere,
                                  sphere, fam, nfam, ndim, n_kept);
}

int pbx_profile_select_typed(void *handle, const void *pos, int pos_dtype, const void *mass,
                             int mass_dtype, int64_t n, int on_device, int use_sphere,
                             const double *sphere, const int64_t *fam, int nfam, int ndim,
                             int64_t *n_kept) {
  return guard([&] {
    Profile &P = as_profile(handle);
    if ((pos_dtype != PBX_F64 && pos_dtype != PBX_F32) ||
        (mass_dtype != PBX_F64 && mass_dtype != PBX_F32))
      fail(PBX_ERR_VALUE, "dtype must be PBX_F64 or PBX_F32");
    Device &d = current_device();
    std::lock_guard<std::mutex> lk(d.mu);
    hipStream_t st = d.stream;
    ScopedTimer tm("pbx.profile.select");
    const uint32_t nt = select_launch(P, st, pos, mass, n, on_device, use_sphere, sphere, fam,
                                      nfam, ndim, false, pos_dtype == PBX_F32,
                                      mass_dtype == PBX_F32);
    int64_t kept = 0;
    if (nt) {
      uint64_t *stat = (uint64_t *)P.selst.p;
      const size_t nh = 2 + 2 * MM_SLOTS;
      uint64_t *h = (uint64_t *)P.pin.get(sizeof(uint64_t) * nh);
      PBX_HIP(hipMemcpyAsync(h, stat + nt - 1, sizeof(uint64_t) * nh, hipMemcpyDeviceToHost, st));
      PBX_HIP(hipStreamSynchronize(st));
      const uint64_t last = h[0];
      if ((h[1] >> 32) || (last >> 62) != 2) fail(PBX_ERR_RUNTIME, "selection look-back did not complete");
      kept = (int64_t)(last & kStVal);
      P.mm[0] = ~0ull;
      P.mm[1] = 0ull;
      for (int q = 0; q < MM_SLOTS; ++q) {
        P.mm[0] = std::min<uint64_t>(P.mm[0], ~h[2 + 2 * q]);
        P.mm[1] = std::max<uint64_t>(P.mm[1], h[3 + 2 * q]);
      }
    }
    select_commit(P, kept);
    *n_kept = kept;
  });
}

int pbx_profile_get_selection(void *handle, int64_t *h_idx, double *h_x, double *h_w) {
  return guard([&] {
    Profile &P = as_profile(handle);
    Device &d = current_device();
    std::lock_guard<std::mutex> lk(d.mu);
    hipStream_t st = d.stream;
    if (!P.has_idx) fail(PBX_ERR_VALUE, "profile has no selection");
    const int64_t n = P.n;
    if (n == 0) return;
    if (h_idx) ensure_idx(P, st);
    if (h_w) ensure_w(P, st);
    // (int32 across PCIe, widened by the host threads; small ones on the device)
    if (h_idx && !d2h_staged_widen(d, h_idx, (const int32_t *)P.idx.p, n, st)) {
      int64_t *tmp = (int64_t *)P.vtmp.get(sizeof(int64_t) * (size_t)n);
      hipLaunchKernelGGL(widen_perm, dim3(ceil_div(n, TPB)), dim3(TPB), 0, st,
                         (const int32_t *)P.idx.p, n, tmp);
      d2h_staged(d, h_idx, tmp, sizeof(int64_t) * n, st);
    }
    if (h_x) {
      ensure_x(P, st);
      d2h_staged(d, h_x, P.x.p, sizeof(double) * n, st);
    }
    if (h_w && P.has_w) d2h_staged(d, h_w, P.w.p, sizeof(double) * n, st);
    PBX_HIP(hipStreamSynchronize(st));
  });
}

// np.min / np.max of x (NaN propagates to both, like numpy)
int pbx_profile_minmax(void *handle, double *mn, double *mx) {
  return guard([&] {
    Profile &P = as_profile(handle);
    Device &d = current_device();
    std::lock_guard<std::mutex> lk(d.mu);
    hipStream_t st = d.stream;
    if (P.n == 0) fail(PBX_ERR_VALUE, "zero-size array to reduction operation minimum which has no identity");
    uint64_t h[2];
    minmax_of(P, st, h);
    double lo = dkey_inv(h[0]), hi = dkey_inv(h[1]);
    if (hi != hi) lo = hi;  // any NaN -> both NaN
    *mn = lo;
    *mx = hi;
  });
}

// ---- distributed equaln: the radix select in stages ----
int pbx_profile_key_range(void *handle, uint64_t *kmin, uint64_t *kmax) {
  return guard([&] {
    Profile &P = as_profile(handle);
    Device &d = current_device();
    std::lock_guard<std::mutex> lk(d.mu);
    uint64_t h[2] = {~0ull, 0ull};
    if (P.n) minmax_of(P, d.stream, h);
    *kmin = h[0];
    *kmax = h[1];
  });
}

int pbx_profile_msel_begin(void *handle, int64_t nbins, int has_min, double bin_min, int has_max,
                           double bin_max, uint64_t kmin, uint64_t kmax, int *levels) {
  return guard([&] {
    Profile &P = as_profile(handle);
    if (nbins < 1) fail(PBX_ERR_VALUE, "nbins must be >= 1");
    if (nbins + 1 > MS_MAXQ) fail(PBX_ERR_VALUE, "distributed equaln supports nbins <= %d", MS_MAXQ - 1);
    msel_begin(P, nbins, has_min, bin_min, has_max, bin_max, kmin, kmax);
    *levels = P.ms.L;
  });
}

int pbx_profile_msel_hist(void *handle, int level, uint32_t **d_hist, int64_t *count) {
  return guard([&] {
    Profile &P = as_profile(handle);
    Device &d = current_device();
    std::lock_guard<std::mutex> lk(d.mu);
    *count = msel_hist(P, d.stream, level);
    *d_hist = (uint32_t *)P.msH.p;
  });
}

int pbx_profile_msel_resolve(void *handle, int level) {
  return guard([&] {
    Profile &P = as_profile(handle);
    Device &d = current_device();
    std::lock_guard<std::mutex> lk(d.mu);
    msel_resolve_level(P, d.stream, level);
  });
}

int pbx_profile_msel_edges(void *handle, double *h_edges, int64_t *n_edges) {
  return guard([&] {
    Profile &P = as_profile(handle);
    Device &d = current_device();
    std::lock_guard<std::mutex> lk(d.mu);
    msel_edges_out(P, d.stream, h_edges, n_edges);
  });
}

// equaln edges (bins.py:720-746): order statistics of the x values inside
// [bin_min, bin_max]; returns the number of edges written (nbins+1, or 2
// for the degenerate < 2 case; 0 with status VALUE for empty input).
int pbx_profile_edges_equaln(void *handle, int64_t nbins, int has_min, double bin_min,
                             int has_max, double bin_max, double *h_edges, int64_t *n_edges) {
  return guard([&] {
    Profile &P = as_profile(handle);
    if (nbins < 1) fail(PBX_ERR_VALUE, "nbins must be >= 1");
    Device &d = current_device();
    std::lock_guard<std::mutex> lk(d.mu);
    hipStream_t st = d.stream;
    ScopedTimer tm("pbx.profile.equaln");
    const int64_t n = P.n;
    if (n == 0) fail(PBX_ERR_VALUE, "Cannot create bins: input array is empty");
    if (nbins + 1 <= MS_MAXQ) {  // (more bins: the radix-sort path below)
      equaln_select(P, st, nbins, has_min, bin_min, has_max, bin_max, h_edges, n_edges);
      return;
    }
    uint64_t *k0 = (uint64_t *)P.keys0.get(sizeof(uint64_t) * (size_t)n);
    uint64_t *k1 = (uint64_t *)P.keys1.get(sizeof(uint64_t) * (size_t)n);
    unsigned grid = (unsigned)std::min<int64_t>(4096, (n + TPB - 1) / TPB);
    ensure_x(P, st);
    hipLaunchKernelGGL(make_keys, dim3(grid), dim3(TPB), 0, st, (const double *)P.x.p, n, k0);
    PBX_HIP(hipGetLastError());
    // only the bits where min and max keys differ need sorting
    uint64_t h[2];
    minmax_of(P, st, h);
    uint64_t diff = h[0] ^ h[1];
    int hb = diff ? 63 - __builtin_clzll(diff) : -1;
    uint64_t *a = k0, *b = k1;
    for (int shift = 0; shift <= hb; shift += 8) {
      radix_pass<uint64_t>(P, st, a, nullptr, VAL_NONE, n, shift, b, nullptr);
      std::swap(a, b);
    }
    // clip window [lo, hi) of the sorted keys: sorted_x[sorted_x >= bin_min]
    // then [sorted_x <= bin_max] (bins.py:734-737).  A NaN x fails both
    // comparisons and NaN keys sort last; a NaN bound keeps nothing.
    int64_t lo = 0, hi = n;
    if (has_min || has_max) {
      uint64_t ka = has_min ? dkey(bin_min) : 0ull;
      uint64_t kb = has_max ? dkey(bin_max) : ~0ull;
      int64_t *bd = (int64_t *)P.bounds.get(32);
      hipLaunchKernelGGL(count_bounds, dim3(1), dim3(64), 0, st, a, n, ka, kb, bd);
      PBX_HIP(hipGetLastError());
      int64_t b3[3];
      PBX_HIP(hipMemcpyAsync(b3, bd, 24, hipMemcpyDeviceToHost, st));
      PBX_HIP(hipStreamSynchronize(st));
      hi = b3[2];  // drop the NaN block
      if (has_min) lo = (bin_min != bin_min) ? hi : b3[0];
      if (has_max) hi = (bin_max != bin_max) ? lo : std::min<int64_t>(hi, b3[1]);
      if (hi < lo) hi = lo;
    }
    const int64_t m = hi - lo;
    std::vector<int64_t> ranks;
    if (m < 2) {
      if (m == 0) fail(PBX_ERR_VALUE, "index 0 is out of bounds for axis 0 with size 0");
      ranks = {lo, lo};
    } else {
      ranks.push_back(lo);
      for (int64_t i = 1; i < nbins; ++i)
        ranks.push_back(lo + (int64_t)((double)(i * m) / (double)nbins));
      ranks.push_back(lo + m - 1);
    }
    const int64_t ne = (int64_t)ranks.size();
    int64_t *dr = (int64_t *)P.ranks.get(sizeof(int64_t) * (size_t)ne);
    double *de = (double *)P.edges.get(sizeof(double) * (size_t)ne);
    PBX_HIP(hipMemcpyAsync(dr, ranks.data(), sizeof(int64_t) * ne, hipMemcpyHostToDevice, st));
    hipLaunchKernelGGL(gather_keys, dim3(ceil_div(ne, TPB)), dim3(TPB), 0, st, a, dr, ne, de);
    PBX_HIP(hipGetLastError());
    PBX_HIP(hipMemcpyAsync(h_edges, de, sizeof(double) * ne, hipMemcpyDeviceToHost, st));
    PBX_HIP(hipStreamSynchronize(st));
    *n_edges = ne;
  });
}

// bins + per-bin counts for explicit edges (ascending); builds the bin ids
// the CSR and moments use.  counts: nb int64 (host).
int pbx_profile_assign(void *handle, const double *h_edges, int64_t n_edges, int64_t *h_counts,
                       int64_t *n_valid) {
  return guard([&] {
    Profile &P = as_profile(handle);
    if (n_edges < 2) fail(PBX_ERR_VALUE, "Explicit bin_edges must be a 1D array of length >= 2");
    Device &d = current_device();
    std::lock_guard<std::mutex> lk(d.mu);
    hipStream_t st = d.stream;
    ScopedTimer tm("pbx.profile.assign");
    double *de = (double *)P.edges.get(sizeof(double) * (size_t)n_edges);
    PBX_HIP(hipMemcpyAsync(de, h_edges, sizeof(double) * n_edges, hipMemcpyHostToDevice, st));
    assign_device(P, st, de, n_edges - 1);
    PBX_HIP(hipMemcpyAsync(h_counts, P.counts.p, sizeof(int64_t) * (n_edges - 1),
                           hipMemcpyDeviceToHost, st));
    PBX_HIP(hipStreamSynchronize(st));
    int64_t s = 0;
    for (int64_t k = 0; k < n_edges - 1; ++k) s += h_counts[k];
    P.n_valid = s;
    *n_valid = s;
  });
}

// CSR of the last assignment: perm (n_valid int64, ascending indices inside
// each bin = the reference's binind lists concatenated) and offsets (nb+1).
// Either output may be NULL (then the CSR stays on the device only).
int pbx_profile_csr(void *handle, int64_t *h_perm, int64_t *h_offsets) {
  return guard([&] {
    Profile &P = as_profile(handle);
    if (P.nb < 0) fail(PBX_ERR_VALUE, "call pbx_profile_assign first");
    Device &d = current_device();
    std::lock_guard<std::mutex> lk(d.mu);
    hipStream_t st = d.stream;
    ScopedTimer tm("pbx.profile.csr");
    const int64_t nb = P.nb;
    csr_device(P, st);
    if (h_offsets) {
      std::vector<int64_t> c((size_t)nb);
      PBX_HIP(hipMemcpyAsync(c.data(), P.counts.p, sizeof(int64_t) * nb, hipMemcpyDeviceToHost, st));
      PBX_HIP(hipStreamSynchronize(st));
      h_offsets[0] = 0;
      for (int64_t k = 0; k < nb; ++k) h_offsets[k + 1] = h_offsets[k] + c[(size_t)k];
    }
    if (h_perm && P.n_valid && !d2h_staged_widen(d, h_perm, (const int32_t *)P.perm.p, P.n_valid, st)) {
      int64_t *tmp = (int64_t *)P.field.get(sizeof(int64_t) * (size_t)P.n_valid);
      hipLaunchKernelGGL(widen_perm, dim3(ceil_div(P.n_valid, TPB)), dim3(TPB), 0, st,
                         (const int32_t *)P.perm.p, P.n_valid, tmp);
      PBX_HIP(hipMemcpyAsync(h_perm, tmp, sizeof(int64_t) * P.n_valid, hipMemcpyDeviceToHost, st));
    }
    PBX_HIP(hipStreamSynchronize(st));
  });
}

// Per-bin sums of the last assignment:
//   out[bin*7 + k], k = Σw, Σf·w, Σf²·w, Σf, Σf², Σ|f|·w, Σ|f|
// f_src / w_src: 0 = the profile's x, 1 = its weights (selection mass),
// 2 = a host array of n doubles (h_f / h_w); w_src -1 = unweighted (the
// weighted columns are then left 0).
int pbx_profile_moments(void *handle, int f_src, const double *h_f, int w_src, const double *h_w,
                        double *h_out) {
  return pbx_profile_moments_cols(handle, f_src, h_f, w_src, h_w, 0x7fu, h_out);
}

// the same, accumulating only the columns in `cols` (bit k = column k; the
// others are returned as 0): e.g. Sum needs Σf only, a weighted Mean Σw
// and Σf·w (pynbodyext.profiles.proarray derives the set per statistic)
int pbx_profile_moments_cols(void *handle, int f_src, const double *h_f, int w_src,
                             const double *h_w, uint32_t cols, double *h_out) {
  return guard([&] {
    Profile &P = as_profile(handle);
    if (P.nb < 0) fail(PBX_ERR_VALUE, "call pbx_profile_assign first");
    Device &d = current_device();
    std::lock_guard<std::mutex> lk(d.mu);
    hipStream_t st = d.stream;
    ScopedTimer tm("pbx.profile.moments");
    const int64_t len = P.nb * NMOM;
    double *acc = (double *)P.acc.get(sizeof(double) * (size_t)std::max<int64_t>(len, 1));
    moments_device(P, st, f_src, h_f, P.field, w_src, h_w, P.weight, cols, acc);
    PBX_HIP(hipMemcpyAsync(h_out, acc, sizeof(double) * len, hipMemcpyDeviceToHost, st));
    PBX_HIP(hipStreamSynchronize(st));
  });
}

// One radial-profile pass after pbx_profile_select, with a single host
// round trip: equaln edges (radix select, kept on the device), assignment
// with those edges, the CSR (optional) and the per-bin sums of n_stats
// (field, weight, columns) requests, then one batch of copies back.
int pbx_profile_binned_equaln(void *handle, int64_t nbins, int has_min, double bin_min,
                              int has_max, double bin_max, int build_csr, int n_stats,
                              const int *f_src, const int *w_src, const uint32_t *cols,
                              double *h_edges, int64_t *n_edges, int64_t *h_counts,
                              int64_t *n_valid, double *h_moments) {
  return guard([&] {
    Profile &P = as_profile(handle);
    if (nbins < 1) fail(PBX_ERR_VALUE, "nbins must be >= 1");
    if (nbins + 1 > MS_MAXQ) fail(PBX_ERR_VALUE, "the fused path supports nbins <= %d", MS_MAXQ - 1);
    if (n_stats < 0 || n_stats > 16) fail(PBX_ERR_VALUE, "at most 16 statistics");
    for (int k = 0; k < n_stats; ++k)
      if (f_src[k] < 0 || f_src[k] > 1 || w_src[k] < -1 || w_src[k] > 1)
        fail(PBX_ERR_VALUE, "the fused path takes the profile's x / weights only");
    Device &d = current_device();
    std::lock_guard<std::mutex> lk(d.mu);
    hipStream_t st = d.stream;
    ScopedTimer tm("pbx.profile.binned_equaln");
    if (P.n == 0) fail(PBX_ERR_VALUE, "Cannot create bins: input array is empty");
    uint64_t mm[2];
    minmax_of(P, st, mm);
    msel_begin(P, nbins, has_min, bin_min, has_max, bin_max, mm[0], mm[1]);
    for (int l = 0; l < P.ms.L; ++l) {
      msel_hist(P, st, l);
      msel_resolve_level(P, st, l);
    }
    const int nq = P.ms.nq;
    double *de = (double *)P.edges.get(sizeof(double) * (size_t)nq);
    hipLaunchKernelGGL(msel_edges, dim3(ceil_div(nq, TPB)), dim3(TPB), 0, st,
                       (const MsRank *)P.msR.p, nq, P.ms.lo, de);
    PBX_HIP(hipGetLastError());
    P.ms.active = false;
    // speculate m >= 2 (nbins bins): everything stays on the device
    assign_device(P, st, de, nbins);
    if (build_csr) csr_device(P, st);
    const int64_t len = nbins * NMOM;
    double *accs = (double *)P.accs.get(sizeof(double) * (size_t)std::max<int64_t>(1, n_stats * len));
    for (int k = 0; k < n_stats; ++k)
      moments_device(P, st, f_src[k], nullptr, P.field, w_src[k], nullptr, P.weight, cols[k],
                     accs + k * len);
    // async readbacks into pinned staging, one sync
    char *hp = (char *)P.pin.get(8 * (1 + nq + nbins + n_stats * len));
    int64_t *hm = (int64_t *)hp;
    double *he = (double *)(hm + 1);
    int64_t *hc = (int64_t *)(he + nq);
    double *hmo = (double *)(hc + nbins);
    PBX_HIP(hipMemcpyAsync(hm, P.msM.p, 8, hipMemcpyDeviceToHost, st));
    PBX_HIP(hipMemcpyAsync(he, de, sizeof(double) * nq, hipMemcpyDeviceToHost, st));
    PBX_HIP(hipMemcpyAsync(hc, P.counts.p, sizeof(int64_t) * nbins, hipMemcpyDeviceToHost, st));
    if (n_stats)
      PBX_HIP(hipMemcpyAsync(hmo, accs, sizeof(double) * n_stats * len, hipMemcpyDeviceToHost, st));
    PBX_HIP(hipStreamSynchronize(st));
    const int64_t m = *hm;
    std::memcpy(h_edges, he, sizeof(double) * nq);
    std::memcpy(h_counts, hc, sizeof(int64_t) * nbins);
    if (n_stats) std::memcpy(h_moments, hmo, sizeof(double) * n_stats * len);
    if (m == 0) fail(PBX_ERR_VALUE, "index 0 is out of bounds for axis 0 with size 0");
    if (m < 2) {  // the reference's degenerate [s0, s0]: one bin, redo with 2 edges
      h_edges[1] = h_edges[0];
      double *de = (double *)P.edges.get(sizeof(double) * 2);
      PBX_HIP(hipMemcpyAsync(de, h_edges, sizeof(double) * 2, hipMemcpyHostToDevice, st));
      assign_device(P, st, de, 1);
      if (build_csr) csr_device(P, st);
      for (int k = 0; k < n_stats; ++k)
        moments_device(P, st, f_src[k], nullptr, P.field, w_src[k], nullptr, P.weight, cols[k],
                       accs + k * NMOM);
      PBX_HIP(hipMemcpyAsync(h_counts, P.counts.p, sizeof(int64_t), hipMemcpyDeviceToHost, st));
      if (n_stats)
        PBX_HIP(hipMemcpyAsync(h_moments, accs, sizeof(double) * n_stats * NMOM,
                               hipMemcpyDeviceToHost, st));
      PBX_HIP(hipStreamSynchronize(st));
      *n_edges = 2;
    } else {
      *n_edges = nq;
    }
    const int64_t nb = *n_edges - 1;
    int64_t s = 0;
    for (int64_t k = 0; k < nb; ++k) s += h_counts[k];
    P.n_valid = s;
    *n_valid = s;
  });
}

// Per-bin percentiles (Percentile / Median / Abs_pXX, proarray.py:689-722)
// of the last assignment: h_out[bin*nq + k] = np.interp(q[k], cdf_bin,
// sorted field_bin), cdf = normalised cumsum of the weights in value order
// (w_src -1: np.linspace(0, 1, m)); empty bins NaN.  f_src / w_src as in
// pbx_profile_moments (3 = device array per original particle); absval:
// statistic of |f|.  q[k] = p/100.
int pbx_profile_percentiles(void *handle, int f_src, const double *h_f, int w_src,
                            const double *h_w, int absval, int nq, const double *q,
                            double *h_out) {
  return guard([&] {
    Profile &P = as_profile(handle);
    if (P.nb < 0) fail(PBX_ERR_VALUE, "call pbx_profile_assign first");
    if (nq < 1 || nq > 4096) fail(PBX_ERR_VALUE, "1 to 4096 percentiles per call");
    if (f_src < 0 || f_src > 3 || w_src < -1 || w_src > 3) fail(PBX_ERR_VALUE, "bad source selector");
    Device &d = current_device();
    std::lock_guard<std::mutex> lk(d.mu);
    hipStream_t st = d.stream;
    ScopedTimer tm("pbx.profile.percentiles");
    const int64_t nb = P.nb;
    double *out = (double *)P.pout.get(sizeof(double) * (size_t)std::max<int64_t>(1, nb * nq));
    percentiles_device(P, st, f_src, h_f, w_src, h_w, absval, nq, q, out);
    if (nb > 0)
      PBX_HIP(hipMemcpyAsync(h_out, out, sizeof(double) * nb * nq, hipMemcpyDeviceToHost, st));
    PBX_HIP(hipStreamSynchronize(st));
  });
}

// Selection + equaln radial profile with ONE host round trip
// (RadialProfileBuilder equaln path: filters/filt.py:42-86 mask and r,
// bins.py:720-746 edges, :346-395 assignment, proarray sums).  Same results
// and errors as pbx_profile_select followed by pbx_profile_binned_equaln;
// the distinct sums of the requested statistics (<= AS_MAXM) are
// accumulated inside the assignment pass (more: separate moment passes).
//
// comm (pbx_profile_radial_equaln_comm): this rank's particles of a profile
// sharded over the communicator's ranks.  The same kernels
// with four device all-reduces between them and one extra host read-back:
// the selection's key-range slots (max) -> global window geometry; the
// level-0 digit histogram (sum) -> every rank resolves the same digits and
// groups; each rank gathers its keys of the chosen digits into its own
// slice of the GLOBAL group segments (dist_rank_offsets) and a sum
// all-reduce of the zeroed segment array all-gathers them -> every rank
// finishes the same edges; the packed counts and per-bin sums (sum).  The
// ctl read-back after the resolve sizes the segment array on the host.
static int radial_equaln_entry(void *comm, void *handle, const double *pos, const double *mass,
                               int64_t n, int on_device, int use_sphere, const double *sphere,
                               const int64_t *fam, int nfam, int ndim, int64_t nbins, int has_min,
                               double bin_min, int has_max, double bin_max, int build_csr,
                               int n_stats, const int *f_src, const int *w_src,
                               const uint32_t *cols, int64_t *n_kept, double *h_edges,
                               int64_t *n_edges, int64_t *h_counts, int64_t *n_valid,
                               double *h_moments, int64_t *h_counts_local) {
  return guard([&] {
    Profile &P = as_profile(handle);
    const bool dist = comm != nullptr;
    const CommRanks cr = dist ? comm_ranks(comm) : CommRanks{1, 0};
    if (nbins < 1) fail(PBX_ERR_VALUE, "nbins must be >= 1");
    if (nbins + 1 > MS_MAXQ) fail(PBX_ERR_VALUE, "the fused path supports nbins <= %d", MS_MAXQ - 1);
    if (n_stats < 0 || n_stats > 16) fail(PBX_ERR_VALUE, "at most 16 statistics");
    for (int k = 0; k < n_stats; ++k)
      if (f_src[k] < 0 || f_src[k] > 1 || w_src[k] < -1 || w_src[k] > 1)
        fail(PBX_ERR_VALUE, "the fused path takes the profile's x / weights only");
    Device &d = current_device();
    std::unique_lock<std::mutex> lk(d.mu);  // (released inside comm_allreduce's host wait)
    hipStream_t st = d.stream;
    ScopedTimer tm("pbx.profile.radial_equaln");
    // bins < 256: the lazy selection + tile-walking assignment / CSR passes
    const bool lazy = nbins < RADIX;
    const int nq = (int)nbins + 1;
    // the window of bins.py:734-737 as key bounds (msel_begin)
    bool empty_bounds = false;
    uint64_t ka = 0ull, kb = ~0ull;
    if (has_min || has_max) {
      kb = ~0ull - 1;
      if (has_min) {
        if (bin_min != bin_min) empty_bounds = true;
        else ka = dkey(bin_min);
      }
      if (has_max) {
        if (bin_max != bin_max) empty_bounds = true;
        else kb = std::min<uint64_t>(kb, dkey(bin_max));
      }
    }
    const int64_t nb = nbins;
    // distinct monomials of the requested columns (x^a w^b |x|^c |w|^d);
    // mono[k][c] = its slot, -1 = column not accumulated (0)
    FusedStats fs{};
    fs.nm = 0;
    const int64_t len = nb * NMOM;
    double *accs = (double *)P.accs.get(sizeof(double) * (size_t)std::max<int64_t>(1, n_stats * len));
    std::vector<int> mono((size_t)n_stats * NMOM, -1);
    std::vector<uint32_t> mkey;
    bool fuse = n_stats > 0;
    for (int k = 0; k < n_stats && fuse; ++k)
      for (int c = 0; c < NMOM; ++c) {
        if (!((cols[k] >> c) & 1u)) continue;
        const bool wc = (c == 0 || c == 1 || c == 2 || c == 5);
        if (wc && w_src[k] < 0) continue;  // unweighted: the weighted columns stay 0
        uint32_t e[4] = {0, 0, 0, 0};       // powers of x, w, |x|, |w|
        const int fp = (c == 2 || c == 4) ? 2 : (c == 0 ? 0 : 1);
        const bool fa = (c == 5 || c == 6);
        e[(fa ? 2 : 0) + f_src[k]] += fp;
        if (wc) e[w_src[k]] += 1;
        const uint32_t key = e[0] | e[1] << 4 | e[2] << 8 | e[3] << 12;
        int slot = -1;
        for (size_t j = 0; j < mkey.size(); ++j)
          if (mkey[j] == key) slot = (int)j;
        if (slot < 0) {
          if (fs.nm == AS_MAXM || (int64_t)(fs.nm + 1) * nb > 2 * LDS_MOM_BINS * NMOM) {
            fuse = false;
            break;
          }
          slot = fs.nm++;
          mkey.push_back(key);
          fs.f[slot] = f_src[k];
          fs.w[slot] = w_src[k];
          fs.col[slot] = c;
          fs.op[slot] = key == 0x010u ? MO_W : key == 0x001u ? MO_X : key == 0x011u ? MO_XW
                      : key == 0x012u ? MO_XXW : key == 0x002u ? MO_XX : key == 0x020u ? MO_WW
                      : MO_GEN;
        }
        mono[(size_t)k * NMOM + c] = slot;
      }
    if (!fuse) fs.nm = 0;
    constexpr int NC = (int)(sizeof(FusedCtl) / sizeof(double));
    static_assert(sizeof(FusedCtl) % sizeof(double) == 0, "FusedCtl packs as doubles");
    // small selections: the whole step as one persistent launch (radial_mono)
    double *hp = nullptr;
    bool tiled_call = false;  // the multi-kernel path over a tiled selection
    int nsum = 0;
    int64_t n_global = 0;  // dist: kept particles over all ranks
    if (lazy && !dist)
      hp = radial_mono_run(P, st, pos, mass, n, on_device, use_sphere, sphere, fam, nfam, ndim,
                           nbins, ka, kb, empty_bounds, fs, &nsum);
    if (!hp) {  // the multi-kernel path
      ++P.n_multi;
      // one rank, lazy: the level-0 histogram of a tiled selection is built by
      // select_tiles with the previous tiled call's geometry (slot n_tiled & 1;
      // fused_hist0 writes this call's into the other slot)
      SelHint *hints = nullptr;
      if (!dist && lazy && !P.hint_off) {
        if (!P.shint.p) {
          P.shint.get(2 * sizeof(SelHint));
          PBX_HIP(hipMemsetAsync(P.shint.p, 0, 2 * sizeof(SelHint), st));
        }
        hints = (SelHint *)P.shint.p;
      }
      TileHist thist;
      thist.hint = hints ? hints + (P.n_tiled & 1) : nullptr;
      thist.cold = hints && P.n_tiled == 0;  // (no earlier tiled call left a geometry)
      thist.ka = ka;
      thist.kb = empty_bounds ? 0ull : kb;
      // the speculative assignment: when the last tiled call's level-0 ranks
      // matched the stored table (a repeated or similar call), select_tiles
      // bins with it (checked by fused_resolve; a miss takes assign_tiles).
      // It stores no x, which is then rebuilt from the positions on demand:
      // only from positions the handle owns (staged host arrays) or that the
      // caller declared stable
      bool spec_ops = true;  // select_tiles' sums take the dedicated monomials only
      for (int q = 0; q < fs.nm; ++q) spec_ops = spec_ops && fs.op[q] != MO_GEN;
      if (hints && P.spec_next && P.stab.p && nb <= SPEC_MAXB && fs.nm * nb <= SPEC_MACC &&
          spec_ops && (!on_device || P.src_stable)) {
        thist.sa.tab = (const SpecTab *)P.stab.p;
        thist.sa.fs = fs;
        thist.sa.nb = (int)nb;
        thist.sa.edge = P.edge_next ? 1 : 0;
        if (thist.sa.edge && !P.slteq.p) {  // (zero before the first use; fused_resolve re-zeroes)
          P.slteq.get(sizeof(uint32_t) * 2 * MS_MAXQ);
          PBX_HIP(hipMemsetAsync(P.slteq.p, 0, sizeof(uint32_t) * 2 * MS_MAXQ, st));
        }
        thist.sa.lteq = (uint32_t *)P.slteq.p;
        if (P.spec_dirty) {
          if (P.sflag.p) PBX_HIP(hipMemsetAsync(P.sflag.p, 0, sizeof(uint32_t), st));
          if (P.slteq.p) PBX_HIP(hipMemsetAsync(P.slteq.p, 0, sizeof(uint32_t) * 2 * MS_MAXQ, st));
          P.spec_dirty = false;
        }
      }
      const uint32_t nt = select_launch(P, st, pos, mass, n, on_device, use_sphere, sphere, fam,
                                        nfam, ndim, lazy, 0, 0, /*tiled=*/true, &thist);
      if (thist.spec) {
        ++P.n_spec;
        P.spec_dirty = true;  // (until the call's results arrive)
      }
      const bool hinted = hints && P.x_tiled;
      tiled_call = P.x_tiled;
      if (hinted) ++P.n_tiled;  // (the next tiled call reads the slot this one writes)
      if (dist)  // global key range: every min / max slot pair (~min, max) max-reduced
        comm_allreduce(comm, (uint64_t *)P.selst.p + nt + 1, (uint64_t *)P.selst.p + nt + 1,
                       2 * MM_SLOTS, 2, 2, st, lk);
      const int64_t n_sel = nt ? P.sel_span : 0;  // tiled particles (the families' span)
      const bool tiled = P.x_tiled;  // x by tile (large inputs): tile offsets from fused_hist0
      uint64_t *stat = (uint64_t *)P.selst.p;
      FusedCtl *ctl = (FusedCtl *)P.fctl.get(sizeof(FusedCtl));
      unsigned long long *cnt = (unsigned long long *)P.counts.get(sizeof(uint64_t) * (size_t)(nb + 1));
      uint32_t *H = (uint32_t *)P.msH.get(sizeof(uint32_t) * MS0_DIG);
      const int64_t *n_dev = &ctl->n;
      const double *x = (const double *)P.x.p;
      // level 0 (rows -> H), resolve + groups, per-block offsets, gather,
      // per-group finish -> edges
      const int g0 = fused_grid(n_sel);
      uint32_t *rows = (uint32_t *)P.msRows.get(sizeof(uint32_t) * (size_t)g0 * MS0_DIG);
      // tiled selections: assignment fused with the gather (assign_tiles),
      // the deferred keys binned block by block by fix_deferred; the three
      // per-block words [bcnt | rbase | rn] zeroed by fused_hist0
      const bool agath = tiled && lazy && n_sel;
      if (agath && g0 < 2) fail(PBX_ERR_RUNTIME, "tiled selection with one level-0 block");
      // [bcnt | rbase | rn] per assignment workgroup (at_blocks: one per select block + 1)
      const uint32_t nab = agath ? at_blocks(g0) : 0u;
      uint32_t *bcnt = agath ? (uint32_t *)P.fblk.get(sizeof(uint32_t) * 3 * (size_t)nab) : nullptr;
      const uint32_t *hflag = (const uint32_t *)(stat + nt + 1 + 2 * MM_SLOTS);
      const FusedSetup fsu{(const uint64_t *)stat, nt, n_sel, ka, kb, (int)empty_bounds, (int)tiled,
                           (uint32_t *)P.toff.p, bcnt, agath ? 3 * (int)nab : 0, (int)dist,
                           (const uint64_t *)P.kw.p,
                           hinted ? hints + ((P.n_tiled - 1) & 1) : nullptr, hflag,
                           hinted ? hints + (P.n_tiled & 1) : nullptr, (const uint32_t *)P.sbt.p,
                           thist.spec ? (const uint32_t *)thist.sa.flag : nullptr, thist.xs};
      hipLaunchKernelGGL(fused_hist0, dim3(g0), dim3(MS0_TPB), 0, st, x, fsu, ctl, cnt, (int)nb,
                         rows);
      hipLaunchKernelGGL(msel_reduce0h, dim3(MS0_DIG / R0_DIG), dim3(MS0_TPB), 0, st,
                         (const uint32_t *)rows, g0, hinted ? (const uint32_t *)P.srows.p : nullptr,
                         hinted ? SH_K * (g0 - 1) * (int)P.sel_rsub : 0, (const int32_t *)&ctl->hint, H,
                         stat + nt, 2 + 2 * MM_SLOTS);
      PBX_HIP(hipGetLastError());
      P.sel_tail_zero = stat + nt;  // (select_launch: no fill before the next tiled call)
      int64_t *gsc = nullptr;  // dist: [global kept count][ctl copy]
      uint32_t *lc_all = nullptr;
      if (dist) {
        gsc = (int64_t *)P.dscal.get(sizeof(int64_t) * 4 + sizeof(FusedCtl));
        lc_all = (uint32_t *)P.dlc.get(sizeof(uint32_t) * (size_t)cr.nranks * MS_MAXQ);
        PBX_HIP(hipMemsetAsync(lc_all, 0, sizeof(uint32_t) * (size_t)cr.nranks * MS_MAXQ, st));
        // [global kept count, ranks whose look-back failed]
        hipLaunchKernelGGL(dist_status, dim3(1), dim3(1), 0, st, (const FusedCtl *)ctl, gsc + 2);
        comm_allreduce(comm, gsc + 2, gsc, 2, 1, 0, st, lk);
        comm_allreduce(comm, H, H, MS0_DIG, 3, 0, st, lk);
      }
      MsRank *R = (MsRank *)P.msR.get(sizeof(MsRank) * (size_t)nq);
      // [gdig | goff | gq | boff: a row per assignment workgroup (g0 or nab rows)]
      uint32_t *gdig = (uint32_t *)P.fgrp.get(sizeof(uint32_t) * (3 + (size_t)std::max<uint32_t>(g0, nab)) *
                                              (MS_MAXQ + 1));
      uint32_t *goff = gdig + (MS_MAXQ + 1), *gq = goff + (MS_MAXQ + 1);
      uint32_t *boff = gq + (MS_MAXQ + 1);
      // the stored bin table (one rank, tiled assignment): allocated zeroed (invalid)
      SpecTab *stab = nullptr;
      if (agath && !dist) {
        if (!P.stab.p) {
          P.stab.get(sizeof(SpecTab));
          PBX_HIP(hipMemsetAsync(P.stab.p, 0, sizeof(SpecTab), st));
        }
        stab = (SpecTab *)P.stab.p;
      }
      hipLaunchKernelGGL(fused_resolve, dim3(nq), dim3(FR_TPB), 0, st, (const uint32_t *)H, ctl,
                         nbins, nq, R, gdig, goff, gq, (const uint32_t *)rows, g0, boff, bcnt,
                         dist ? lc_all + (size_t)cr.rank * MS_MAXQ : nullptr,
                         (const uint32_t *)P.srows.p, P.sel_rsub, (const SpecTab *)stab,
                         thist.spec ? thist.sa.flag : nullptr, (int)nb,
                         (thist.spec && thist.sa.edge) ? thist.sa.lteq : nullptr);
      int64_t seg_total = 0;  // dist: keys in all ranks' group segments
      if (dist) {
        comm_allreduce(comm, lc_all, lc_all, (int64_t)cr.nranks * MS_MAXQ, 3, 0, st, lk);
        hipLaunchKernelGGL(dist_rank_offsets, dim3(nq), dim3(TPB), 0, st, (const FusedCtl *)ctl,
                           (const uint32_t *)lc_all, cr.rank, g0, boff);
        PBX_HIP(hipGetLastError());
        // the one extra read-back: the global segment length (and kept count)
        FusedCtl *hc = (FusedCtl *)P.pin.get(sizeof(FusedCtl) + 16);
        int64_t *hn = (int64_t *)(hc + 1);
        PBX_HIP(hipMemcpyAsync(hc, ctl, sizeof(FusedCtl), hipMemcpyDeviceToHost, st));
        PBX_HIP(hipMemcpyAsync(hn, gsc, 2 * sizeof(int64_t), hipMemcpyDeviceToHost, st));
        PBX_HIP(hipStreamSynchronize(st));
        n_global = hn[0];
        if (hn[1])  // (every rank sees the same sum: all fail here, no rank left in a collective)
          fail(PBX_ERR_RUNTIME, "selection look-back did not complete (%lld of %d ranks)",
               (long long)hn[1], cr.nranks);
        seg_total = (hc->err & 2) ? 0 : hc->total;
        if (n_global >= (int64_t)1 << 32)  // (every rank sees the same count: all fail here)
          fail(PBX_ERR_VALUE, "distributed equaln over %lld particles: the u32 digit "
               "histograms hold at most 2**32 - 1", (long long)n_global);
      }
      uint64_t *seg = (uint64_t *)P.fseg.get(
          sizeof(uint64_t) * (size_t)std::max<int64_t>(1, std::max<int64_t>(n_sel, seg_total)));
      if (seg_total) PBX_HIP(hipMemsetAsync(seg, 0, sizeof(uint64_t) * (size_t)seg_total, st));
      double *de = (double *)P.edges.get(sizeof(double) * (size_t)nq);
      uint32_t *bins = (uint32_t *)P.bins.get(sizeof(uint32_t) * (size_t)(n_sel ? n_sel : 1));
      P.bins_in8 = agath;
      double *maccs = nullptr, *maccs2 = nullptr;
      P.csrh_ready = false;
      uint32_t ablocks = 0;
      const uint32_t *cnt_offs = nullptr;  // scanned CSR histogram the counts come from
      bool csr_pack = false;  // tiled: csr_slots launched with the pack
      uint32_t *th = nullptr;
      uint8_t *bins8 = nullptr;
      GatherOut go{};
      SpecIO sio{};
      if (agath) {
        const int nr = (int)nb + 1;
        const int64_t macc = (int64_t)fs.nm * nb;
        th = (uint32_t *)P.csrh.get(sizeof(uint32_t) * (size_t)nt * nr);
        bins8 = (uint8_t *)P.bins8.get((size_t)nt * TILE);  // by particle slot
        // (nab: assign_tiles' workgroups = its slab rows)
        double *slab = fs.nm ? (double *)P.fslab.get(sizeof(double) * (size_t)(nab + g0) * macc) : nullptr;
        go = GatherOut{seg, (AgRec *)P.frec.get(sizeof(AgRec) * (size_t)n_sel), bcnt, bcnt + nab,
                       bcnt + 2 * nab};
        sio = SpecIO{stab, thist.spec ? thist.sa.rec : nullptr,
                     thist.spec ? (const uint32_t *)thist.sa.rbase : nullptr,
                     thist.spec ? (const uint32_t *)thist.sa.rn : nullptr,
                     thist.spec ? (const double *)thist.sa.slab : nullptr};
        if (thist.spec) {
          // a speculating call: the hit's hand-over (assign_hit), and x from the
          // positions for a miss whose selection stored none (xsrc_miss); each
          // returns at once unless the call is its case
          constexpr uint32_t xpb = 4;
          hipLaunchKernelGGL(xsrc_miss, dim3(ceil_div(nt, xpb)), dim3(TPB), 0, st, (const FusedCtl *)ctl,
                             thist.xs, nt, xpb);
          if (fs.nm)
            hipLaunchKernelGGL(assign_hit<true>, dim3(g0), dim3(MS0_TPB), 0, st, (const FusedCtl *)ctl,
                               (const uint32_t *)gdig, (const uint32_t *)boff, (int)nb, fs, slab, go, sio);
          else
            hipLaunchKernelGGL(assign_hit<false>, dim3(g0), dim3(MS0_TPB), 0, st, (const FusedCtl *)ctl,
                               (const uint32_t *)gdig, (const uint32_t *)boff, (int)nb, fs, slab, go, sio);
        }
        // the sums' form: {Σw, Σx·w} / {Σw} as dedicated adds, else any monomials
        const int mm = (fs.nm == 2 && fs.op[0] == MO_W && fs.op[1] == MO_XW) ? 1
                       : (fs.nm == 1 && fs.op[0] == MO_W) ? 2 : 0;
        const size_t lds = sizeof(double) * (size_t)macc + sizeof(uint32_t) * (size_t)(nr | 1) * AT_TR;
        auto at = [&](auto kern) {
          hipLaunchKernelGGL(kern, dim3(nab), dim3(AT_BT), lds, st, x, (const uint64_t *)P.kw.p,
                             P.sel_base, P.sel_span, nt, P.sel_mass, (const FusedCtl *)ctl, ka, kb,
                             (const MsRank *)R, nq, (const uint32_t *)gdig, boff, (int)nb, bins8, th, fs,
                             slab, go, stab, g0);
        };
        if (!fs.nm) at(assign_tiles<false, 0>);
        else if (mm == 1) at(assign_tiles<true, 1>);
        else if (mm == 2) at(assign_tiles<true, 2>);
        else at(assign_tiles<true, 0>);
        PBX_HIP(hipGetLastError());
        ablocks = nab;
        if (fs.nm) {
          maccs = slab;
          maccs2 = slab + (size_t)nab * macc;
        }
      } else {
        hipLaunchKernelGGL(fused_gather, dim3(g0), dim3(MS0_TPB), 0, st, x, ka, kb,
                           (const FusedCtl *)ctl, (const uint32_t *)gdig, (const uint32_t *)boff,
                           seg, tiled ? (const uint64_t *)P.kw.p : nullptr, nt);
      }
      if (dist)  // every rank's group keys, each in its own slice: the all-gather
        comm_allreduce(comm, seg, seg, seg_total, 2, 0, st, lk);
      hipLaunchKernelGGL(fused_finish, dim3(nq), dim3(FR_TPB), 0, st, (const FusedCtl *)ctl,
                         (const MsRank *)R, (const uint32_t *)gq, (const uint32_t *)goff,
                         (const uint64_t *)seg, de, (const SpecTab *)stab, nq,
                         thist.spec ? thist.sa.flag : nullptr,
                         (thist.spec && thist.sa.edge) ? thist.sa.lteq : nullptr);
      PBX_HIP(hipGetLastError());
      // assignment (+ the statistics' distinct sums) with the device edges
      if (agath) {
        const uint32_t nr = (uint32_t)nb + 1;
        const size_t lds = sizeof(double) * ((size_t)fs.nm * nb + nb + 1) + sizeof(uint32_t) * FD_LDSW;
        auto fd = [&](auto kern) {
          hipLaunchKernelGGL(kern, dim3(g0), dim3(MS0_TPB), lds, st, (const FusedCtl *)ctl,
                             (const AgRec *)go.rec, (const uint32_t *)go.rbase,
                             (const uint32_t *)go.rn, (const double *)de, (const uint32_t *)gq,
                             (int)nb, bins8, th, nt, fs, maccs2, sio);
        };
        if (fs.nm) fd(fix_deferred<true>);
        else fd(fix_deferred<false>);
        PBX_HIP(hipGetLastError());
        // (a row-wise scan — one block per bin row, its base from row totals
        // summed by assign_gather / fix_deferred — took 15-16 us against this
        // one-pass look-back scan's 11 us at 64M: dropped)
        scan_u32(P, st, th, (int64_t)nt * nr);
        cnt_offs = th;
        // the CSR pass (csr_slots) is launched with the results pack below
        // (its first blocks carry the pack)
        csr_pack = build_csr;
      } else if (n_sel && lazy) {
        // tile-walking assignment over the lazy selection + its CSR pass
        const int64_t macc = (int64_t)fs.nm * nb;
        const bool ldse = (nb + 1) <= LDS_EDGES;
        const size_t lds = sizeof(double) * (size_t)macc + (ldse ? sizeof(double) * (nb + 1) : 0);
        uint32_t *th = (uint32_t *)P.csrh.get(sizeof(uint32_t) * (size_t)nt * RADIX);
        const uint32_t tpbk = std::min<uint32_t>(AS_TILES, std::max<uint32_t>(1, nt / 1024));
        ablocks = ceil_div(nt, tpbk);
        double *slab = fs.nm ? (double *)P.fslab.get(sizeof(double) * (size_t)ablocks * macc) : nullptr;
        const uint64_t *kwp = (const uint64_t *)P.kw.p;
        const uint32_t *tof = (const uint32_t *)P.toff.p;
        // few tiles: one tile per 1024-thread block, every wave a piece of it
        const bool wide = tpbk == 1 && nt < 1024;
        auto go = [&](auto kern, int bt) {
          hipLaunchKernelGGL(kern, dim3(ablocks), dim3(bt), lds, st, x, kwp, tof, P.sel_base, nt,
                             tpbk, P.sel_mass, (const double *)de, (int)nb, bins, th, fs, slab,
                             tiled ? 1 : 0);
        };
        if (wide) {
          if (fs.nm) {
            if (ldse) go(assign_sel<true, true, 1024>, 1024);
            else go(assign_sel<true, false, 1024>, 1024);
          } else {
            if (ldse) go(assign_sel<false, true, 1024>, 1024);
            else go(assign_sel<false, false, 1024>, 1024);
          }
        } else if (fs.nm) {
          if (ldse) go(assign_sel<true, true, TPB>, TPB);
          else go(assign_sel<true, false, TPB>, TPB);
        } else {
          if (ldse) go(assign_sel<false, true, TPB>, TPB);
          else go(assign_sel<false, false, TPB>, TPB);
        }
        PBX_HIP(hipGetLastError());
        if (fs.nm) maccs = slab;
        // the counts are row-start differences of the scanned [bin][tile] table
        scan_u32(P, st, th, (int64_t)nt * RADIX);
        cnt_offs = th;
        if (build_csr) {
          int32_t *perm = (int32_t *)P.perm.get(sizeof(int32_t) * (size_t)n_sel);
          hipLaunchKernelGGL(csr_sel<uint32_t>, dim3(nt), dim3(TPB), 0, st, tof, n_dev, (const uint32_t *)bins,
                             (const uint32_t *)th, nt, perm, (uint32_t)RADIX);
          PBX_HIP(hipGetLastError());
        }
      } else if (n_sel) {
        const int64_t macc = (int64_t)fs.nm * nb;
        size_t lds = sizeof(double) * (size_t)macc +
                     ((nb + 1) <= LDS_EDGES ? sizeof(double) * (nb + 1) : 0) +
                     sizeof(uint32_t) * (nb + 1);
        if (lds > 150 * 1024) fail(PBX_ERR_VALUE, "too many bins for the device histogram (%lld)", (long long)nb);
        uint32_t *th = (nb < RADIX) ? (uint32_t *)P.csrh.get(sizeof(uint32_t) * (size_t)nt * RADIX)
                                    : nullptr;
        const uint32_t tpbk = std::min<uint32_t>(AS_TILES, std::max<uint32_t>(1, nt / 1024));
        ablocks = ceil_div(nt, tpbk);
        double *slab = fs.nm ? (double *)P.fslab.get(sizeof(double) * (size_t)ablocks * macc) : nullptr;
        // with the CSR pass, the bin counts are differences of its scanned
        // [bin][tile] histogram: no global count atomics in assign_bins
        if (th && build_csr) cnt_offs = th;
        unsigned long long *acnt = cnt_offs ? nullptr : cnt;
        if (fs.nm)
          launch_assign<true>(ablocks, lds, st, x, n_sel, (const double *)de, (int)nb, bins, acnt, th,
                              nt, tpbk, n_dev, (const double *)P.w.p, fs, slab);
        else
          launch_assign<false>(ablocks, lds, st, x, n_sel, (const double *)de, (int)nb, bins, acnt, th,
                               nt, tpbk, n_dev, nullptr, fs, nullptr);
        PBX_HIP(hipGetLastError());
        P.csrh_ready = th != nullptr;
        if (fs.nm) maccs = slab;  // its rows are summed inside fused_pack
        if (build_csr) {  // stable counting sort of the bin ids, device length
          int bits = 0;
          while (((int64_t)1 << bits) <= nb) ++bits;
          uint32_t *ka2 = (uint32_t *)P.keys0.get(sizeof(uint32_t) * (size_t)n_sel);
          uint32_t *kb2 = (uint32_t *)P.keys1.get(sizeof(uint32_t) * (size_t)n_sel);
          int32_t *va = (int32_t *)P.perm.get(sizeof(int32_t) * (size_t)n_sel);
          int32_t *vb = (int32_t *)P.vtmp.get(sizeof(int32_t) * (size_t)n_sel);
          const uint32_t *kin = bins;
          bool first = true;
          for (int shift = 0; shift < bits; shift += 8) {
            const bool last = shift + 8 >= bits;
            if (first) {
              prim::radix_pass<uint32_t>(P.csrh_ready ? P.csrh : P.hist, P.tsum, st, kin, nullptr,
                                         VAL_IOTA, n_sel, shift, last ? nullptr : ka2, va, P.csrh_ready,
                                         n_dev);
              first = false;
            } else {
              prim::radix_pass<uint32_t>(P.hist, P.tsum, st, ka2, va, VAL_ARRAY, n_sel, shift,
                                         last ? nullptr : kb2, vb, false, n_dev);
              std::swap(ka2, kb2);
              std::swap(va, vb);
            }
          }
          P.csrh_ready = false;
          if ((void *)va != P.perm.p)
            PBX_HIP(hipMemcpyAsync(P.perm.p, va, sizeof(int32_t) * n_sel, hipMemcpyDeviceToDevice, st));
        }
      }
      // the results packed into one block: mapped host memory + tag (one rank), or a device block, one copy, one sync (dist)
      // (dist: every rank packs the fused sums' columns, zeros without
      // particles, so the all-reduced regions have the same length)
      nsum = (maccs || (dist && fs.nm)) ? fs.nm * (int)nb : 0;
      if (!maccs) ablocks = 0;
      const int ntot = NC + nq + (int)nb + nsum;
      const int nloc = dist ? (int)nb : 0;  // dist: this rank's counts after the global ones
      double *dpk = (double *)P.fpack.get(sizeof(double) * (size_t)(ntot + nloc));
      const int nhead = (int)ceil_div(NC + nq + (int)nb, TPB);
      const uint32_t npk = (uint32_t)(nhead + nsum);
      // one rank: the pack lands in mapped host memory with a completion tag
      // (no D2H copy, no stream sync); dist: all-reduced on the device, copied
      const bool mapped = !dist;
      uint64_t *pdone = nullptr;
      if (mapped) {
        if (!P.pdone.p) {
          P.pdone.get(sizeof(uint64_t));
          PBX_HIP(hipMemsetAsync(P.pdone.p, 0, sizeof(uint64_t), st));
          P.pack_done = 0;
        }
        pdone = (uint64_t *)P.pdone.p;
        hp = (double *)P.mpin.get(sizeof(double) * (size_t)(ntot + 1));
        hp[ntot] = __builtin_bit_cast(double, ~0ull);
        dpk = (double *)P.mpin.dev;
      }
      const PackArgs pk{(const FusedCtl *)ctl, (const double *)de, nq, cnt, (int)nb,
                        (const double *)maccs, (int64_t)ablocks, nsum, dpk, cnt_offs, nt, nhead,
                        (const double *)maccs2, maccs2 ? (int64_t)g0 : 0, pdone,
                        P.pack_done + npk, ntot,
                        P.tsum.p ? (const unsigned long long *)prim::scan_watchdog(P.tsum) : nullptr,
                        mapped ? (double *)P.pstage.get(sizeof(double) * (size_t)ntot) : nullptr};
      auto csr = [&](int np) {
        hipLaunchKernelGGL(csr_slots, dim3(nt), dim3(TPB), 0, st, (const uint32_t *)P.toff.p,
                           (const uint64_t *)P.kw.p, (const uint16_t *)P.kpre.p,
                           (const uint32_t *)P.swc.p, (const uint8_t *)bins8, (const uint32_t *)th,
                           nt, (int32_t *)P.perm.get(sizeof(int32_t) * (size_t)n_sel),
                           (uint32_t)nb + 1, pk, np);
      };
      if (csr_pack && npk <= nt) {  // the pack rides in csr_slots' first npk blocks
        csr((int)npk);
      } else {
        if (csr_pack) csr(0);
        hipLaunchKernelGGL(fused_pack, dim3(npk), dim3(TPB), 0, st, pk);
      }
      PBX_HIP(hipGetLastError());
      if (mapped) {
        P.pack_done += npk;
        if (!wait_tag(st, hp + ntot, P.pack_done))
          fail(PBX_ERR_RUNTIME, "the results pack of a radial profile call did not complete");
      } else {
        if (dist) {
          PBX_HIP(hipMemcpyAsync(dpk + ntot, dpk + NC + nq, sizeof(double) * nb,
                                 hipMemcpyDeviceToDevice, st));
          comm_allreduce(comm, dpk + NC + nq, dpk + NC + nq, nb, 2, 0, st, lk);   // counts (u64)
          comm_allreduce(comm, dpk + NC + nq + nb, dpk + NC + nq + nb, nsum, 0, 0, st, lk);  // sums
        }
        hp = (double *)P.pin.get(sizeof(double) * (size_t)(ntot + nloc));
        PBX_HIP(hipMemcpyAsync(hp, dpk, sizeof(double) * (ntot + nloc), hipMemcpyDeviceToHost, st));
        PBX_HIP(hipStreamSynchronize(st));
      }
    }
    const FusedCtl *hc = (const FusedCtl *)hp;
    const double *he = hp + NC;
    const int64_t *hcn = (const int64_t *)(he + nq);
    const double *hmo = (const double *)(hcn + nb);
    const FusedCtl c = *hc;
    if (c.err & 1) fail(PBX_ERR_RUNTIME, "selection look-back did not complete");
    if (c.err & 4) {  // (the watchdog word is sticky: cleared as it is reported)
      PBX_HIP(hipMemsetAsync(prim::scan_watchdog(P.tsum), 0, sizeof(uint64_t), st));
      fail(PBX_ERR_RUNTIME, "a device scan of the profile step did not complete (look-back watchdog)");
    }
    if (tiled_call) {
      ++P.n_tiled_calls;
      if (c.hint) ++P.n_hinted;
      if (c.spec & SPEC_HIT) ++P.n_spec_hit;
      if (c.spec & SPEC_EDGE) ++P.n_edge_hit;
      P.spec_next = !dist && (c.spec & SPEC_MATCH);
      // edge speculation next: this call's digits matched and its edges are
      // the previous call's, bit for bit
      const bool same = (int64_t)P.last_edges.size() == nq &&
                        std::memcmp(P.last_edges.data(), he, sizeof(double) * nq) == 0;
      P.edge_next = P.spec_next && same;
      P.last_edges.assign(he, he + nq);
      // a hit stored no x (ensure_x rebuilds it on demand); a miss rebuilt it
      P.x_missing = (c.spec & SPEC_NOX) && (c.spec & SPEC_HIT);
      P.spec_dirty = false;  // fused_finish cleared the flag word and the edge counts
    }
    P.mm[0] = c.kmin;
    P.mm[1] = c.kmax;
    select_commit(P, c.n);
    if (dist) P.mm_valid = false;  // the pack's key range is the global one
    *n_kept = c.n;
    if ((dist ? n_global : c.n) == 0) fail(PBX_ERR_VALUE, "Cannot create bins: input array is empty");
    const int64_t m = c.m;
    int64_t sv_local = 0;  // dist: this rank's particles in bins
    if ((c.err & 2) || m == 0) fail(PBX_ERR_VALUE, "index 0 is out of bounds for axis 0 with size 0");
    std::memcpy(h_edges, he, sizeof(double) * nq);
    if (m < 2) {  // the reference's degenerate [s0, s0]: one bin, stepwise
      h_edges[1] = h_edges[0];
      double *de = (double *)P.edges.get(sizeof(double) * 2);
      PBX_HIP(hipMemcpyAsync(de, h_edges, sizeof(double) * 2, hipMemcpyHostToDevice, st));
      assign_device(P, st, de, 1);
      if (build_csr) csr_device(P, st);
      for (int k = 0; k < n_stats; ++k)
        moments_device(P, st, f_src[k], nullptr, P.field, w_src[k], nullptr, P.weight, cols[k],
                       accs + k * NMOM);
      if (dist) {
        PBX_HIP(hipMemcpyAsync(&sv_local, P.counts.p, sizeof(int64_t), hipMemcpyDeviceToHost, st));
        PBX_HIP(hipStreamSynchronize(st));
        int64_t *gc = (int64_t *)P.dscal.get(sizeof(int64_t) * 4 + sizeof(FusedCtl));
        PBX_HIP(hipMemcpyAsync(gc, P.counts.p, sizeof(int64_t), hipMemcpyDeviceToDevice, st));
        comm_allreduce(comm, gc, gc, 1, 1, 0, st, lk);
        comm_allreduce(comm, accs, accs, (int64_t)n_stats * NMOM, 0, 0, st, lk);
        PBX_HIP(hipMemcpyAsync(h_counts, gc, sizeof(int64_t), hipMemcpyDeviceToHost, st));
      } else {
        PBX_HIP(hipMemcpyAsync(h_counts, P.counts.p, sizeof(int64_t), hipMemcpyDeviceToHost, st));
      }
      if (n_stats)
        PBX_HIP(hipMemcpyAsync(h_moments, accs, sizeof(double) * n_stats * NMOM,
                               hipMemcpyDeviceToHost, st));
      PBX_HIP(hipStreamSynchronize(st));
      *n_edges = 2;
    } else {
      P.nb = nb;
      P.csr_ready = build_csr != 0;
      std::memcpy(h_counts, hcn, sizeof(int64_t) * nb);
      if (dist) {  // this rank's counts follow the packed (global) results
        const int64_t *hl = (const int64_t *)(hp + NC + nq + nb + nsum);
        for (int64_t b2 = 0; b2 < nb; ++b2) sv_local += hl[b2];
        if (h_counts_local) std::memcpy(h_counts_local, hl, sizeof(int64_t) * nb);
      }
      if (fs.nm) {  // expand the monomial sums into [stat][bin][column]
        for (int k = 0; k < n_stats; ++k)
          for (int64_t b2 = 0; b2 < nb; ++b2)
            for (int c = 0; c < NMOM; ++c) {
              const int slot = mono[(size_t)k * NMOM + c];
              h_moments[(k * nb + b2) * NMOM + c] = slot < 0 ? 0.0 : hmo[slot * nb + b2];
            }
      } else if (n_stats) {  // too many distinct sums to fuse: separate passes
        for (int k = 0; k < n_stats; ++k)
          moments_device(P, st, f_src[k], nullptr, P.field, w_src[k], nullptr, P.weight, cols[k],
                         accs + k * len);
        if (dist) comm_allreduce(comm, accs, accs, (int64_t)n_stats * len, 0, 0, st, lk);
        PBX_HIP(hipMemcpyAsync(h_moments, accs, sizeof(double) * n_stats * len,
                               hipMemcpyDeviceToHost, st));
        PBX_HIP(hipStreamSynchronize(st));
      }
      *n_edges = nq;
    }
    const int64_t nbo = *n_edges - 1;
    int64_t sv = 0;
    for (int64_t k = 0; k < nbo; ++k) sv += h_counts[k];
    if (dist) {
      sv = sv_local;
      if (h_counts_local && nbo == 1 && m < 2) h_counts_local[0] = sv_local;
    }
    P.n_valid = sv;
    *n_valid = sv;
  });
}

int pbx_profile_radial_equaln(void *handle, const double *pos, const double *mass, int64_t n,
                              int on_device, int use_sphere, const double *sphere,
                              const int64_t *fam, int nfam, int ndim, int64_t nbins, int has_min,
                              double bin_min, int has_max, double bin_max, int build_csr,
                              int n_stats, const int *f_src, const int *w_src,
                              const uint32_t *cols, int64_t *n_kept, double *h_edges,
                              int64_t *n_edges, int64_t *h_counts, int64_t *n_valid,
                              double *h_moments) {
  return radial_equaln_entry(nullptr, handle, pos, mass, n, on_device, use_sphere, sphere, fam, nfam,
                             ndim, nbins, has_min, bin_min, has_max, bin_max, build_csr, n_stats,
                             f_src, w_src, cols, n_kept, h_edges, n_edges, h_counts, n_valid,
                             h_moments, nullptr);
}

int pbx_profile_radial_equaln_comm(void *comm, void *handle, const double *pos, const double *mass,
                                   int64_t n, int on_device, int use_sphere, const double *sphere,
                                   const int64_t *fam, int nfam, int ndim, int64_t nbins,
                                   int has_min, double bin_min, int has_max, double bin_max,
                                   int build_csr, int n_stats, const int *f_src, const int *w_src,
                                   const uint32_t *cols, int64_t *n_kept, double *h_edges,
                                   int64_t *n_edges, int64_t *h_counts, int64_t *h_counts_local,
                                   int64_t *n_valid, double *h_moments) {
  if (!comm) return guard([&] { fail(PBX_ERR_VALUE, "null communicator"); });
  return radial_equaln_entry(comm, handle, pos, mass, n, on_device, use_sphere, sphere, fam, nfam,
                             ndim, nbins, has_min, bin_min, has_max, bin_max, build_csr, n_stats,
                             f_src, w_src, cols, n_kept, h_edges, n_edges, h_counts, n_valid,
                             h_moments, h_counts_local);
}

}  // extern "C"
