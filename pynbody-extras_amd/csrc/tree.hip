// tree.hip — Barnes–Hut octree gravity on gfx950: device build, payloads
// and a wave-coherent stackless walk.
//
// Replaces crates/gravity/src/tree.rs (Octree, Tree3D) and the multipole
// machinery of crates/gravity/src/multipole.rs behind the C ABI of
// include/pbx.h (the PyO3 class it replaces is
// crates/pynbodyext-rust/src/gravity.rs:114-445).
//
// Parity contract (DESIGN.md "octree"): the device tree is the reference's
// tree — same cubic root box (tree.rs:628-654), same `>=`-centre octant
// rule and child centres c +- half/2 (tree.rs:804-845), same split rule
// count > leaf_capacity (tree.rs:847-864), leaf particle lists in ascending
// index order, same BH payload summation order (tree.rs:866-932), same
// opening test size2 < theta^2 (|com - t|^2 + tiny) with the mul_add of
// tree.rs:1117 and the h_max guard (tree.rs:56-71), and each target visits
// the nodes of the reference's DFS in the same order.  Acceptance
// decisions are therefore identical to the reference; only the arithmetic
// inside an accepted interaction (v_rsq_f64 + Newton, FMA, recurrence for
// the derivative tensor, binomial M2M) differs, at the 1e-15 level.
//
// Build (all on the device):
//   1. bounding box (ordered-key atomics), root centre/half on the host
//      with the reference's expressions;
//   2. per particle, its octant path through the reference's node centres
//      (centre updates are the same sequential additions as tree.rs:834-838)
//      packed 21 levels per u64 word;
//   3. stable LSD radix sort of the paths (stable => equal paths stay in
//      index order);
//   4. level-synchronous split: every node that must split finds its
//      children's ranges by binary search on the next digit; children are
//      allocated contiguously (breadth-first ids) and threaded with
//      first/next links like tree.rs:736-776;
//   5. leaf lists re-sorted by original index (the Rust Vec order), then
//      particles are packed as 32-byte records {x, y, z, m} in leaf order;
//   6. payloads bottom-up level by level: mass/COM, h_max, P2M at the COM
//      for leaves and M2M (binomial translation) for internal nodes.
//
// Walk: one target per lane, 64 spatially adjacent targets per wave.  The
// wave walks the UNION of its lanes' walks: a wave-uniform node index w
// (node records and leaf particles are scalar loads), each lane keeps the
// next node of ITS OWN reference walk in p and is active at w iff p == w.
// After an internal node the wave descends iff some active lane opened it.
// Every lane therefore sees exactly its own sequence of nodes, in the
// reference's order, and makes the reference's decision at each of them.
#include <algorithm>
#include <cstdlib>
#include <utility>
#include <cstring>
#include <vector>

#include "prims.h"

namespace pbx {
namespace tree {

using namespace prim;

static constexpr double kR2Tiny = 2.2250738585072014e-308;  // tree.rs:36
constexpr int LPW = 21;                                      // octree levels per key word
constexpr int MAX_WORDS = 53;  // 1113 levels: half underflows to 0 before that
constexpr int WALK_TPB = 256;  // walk kernels' launch bound (the grids use one wave per block)

// --------------------------------------------------------------- moments
// Cartesian slots in graded order (the field order of MultipoleMoment,
// multipole.rs:11-74): slot s <-> (l, m, n), l + m + n <= 5.
struct Slot3 {
  int l, m, n;
};
constexpr Slot3 kSlots[56] = {
    {0, 0, 0}, {1, 0, 0}, {0, 1, 0}, {0, 0, 1}, {2, 0, 0}, {0, 2, 0}, {0, 0, 2}, {1, 1, 0},
    {1, 0, 1}, {0, 1, 1}, {3, 0, 0}, {0, 3, 0}, {0, 0, 3}, {2, 1, 0}, {2, 0, 1}, {1, 2, 0},
    {1, 0, 2}, {0, 2, 1}, {0, 1, 2}, {1, 1, 1}, {4, 0, 0}, {0, 4, 0}, {0, 0, 4}, {3, 1, 0},
    {3, 0, 1}, {1, 3, 0}, {1, 0, 3}, {0, 3, 1}, {0, 1, 3}, {2, 2, 0}, {2, 0, 2}, {0, 2, 2},
    {2, 1, 1}, {1, 2, 1}, {1, 1, 2}, {5, 0, 0}, {0, 5, 0}, {0, 0, 5}, {4, 1, 0}, {4, 0, 1},
    {1, 4, 0}, {1, 0, 4}, {0, 4, 1}, {0, 1, 4}, {3, 2, 0}, {3, 0, 2}, {2, 3, 0}, {2, 0, 3},
    {0, 3, 2}, {0, 2, 3}, {2, 2, 1}, {2, 1, 2}, {1, 2, 2}, {3, 1, 1}, {1, 3, 1}, {1, 1, 3}};

__host__ __device__ constexpr int ncoef(int order) {
  return (order + 1) * (order + 2) * (order + 3) / 6;
}

__host__ __device__ constexpr int slot_of(int l, int m, int n) {
  for (int s = 0; s < 56; ++s)
    if (kSlots[s].l == l && kSlots[s].m == m && kSlots[s].n == n) return s;
  return -1;
}


// slot index as a guaranteed constant expression
template <int L, int M, int N> constexpr int kSlot = slot_of(L, M, N);

__device__ __forceinline__ double rsqrt_nr(double x) {
  double y = __builtin_amdgcn_rsq(x);
  double e = __builtin_fma(-x * y, y, 1.0);
  return __builtin_fma(0.5 * y, e, y);
}

// 1/sqrt(x) of the walk: RAW (fast mode, pbx_set_precise(0)) is v_rsq_f64
// as is (~5e-8 relative), else one Newton step (~1e-16)
template <bool RAW> __device__ __forceinline__ double rsq_walk(double x) {
  return RAW ? __builtin_amdgcn_rsq(x) : rsqrt_nr(x);
}

// Derivative tensor D[s] = d^(l+m+n)/dx^l dy^m dz^n of 1/|R| at R = (x, y, z)
// up to order P, from the recurrence obtained by differentiating
// r^2 dphi/dx + x phi = 0 (Leibniz):
//   r^2 D(l,m,n) = -(2l-1) x D(l-1,m,n) - (l-1)^2 D(l-2,m,n)
//                  - 2m y D(l,m-1,n) - m(m-1) D(l,m-2,n)
//                  - 2n z D(l,m,n-1) - n(n-1) D(l,m,n-2),   l >= 1
// (and the same with the roles of the axes exchanged when l = 0).
// compile-time loop: f(std::integral_constant<int, 0..N-1>) in order
template <class F, int... S>
__device__ __forceinline__ void static_for_impl(F &&f, std::integer_sequence<int, S...>) {
  (f(std::integral_constant<int, S>{}), ...);
}
template <int N, class F> __device__ __forceinline__ void static_for(F &&f) {
  static_for_impl(f, std::make_integer_sequence<int, N>{});
}

template <int P>
__device__ __forceinline__ void derivs(double x, double y, double z, double inv_r,
                                       double (&D)[ncoef(P)]) {
  const double q = inv_r * inv_r;  // 1/r^2
  D[0] = inv_r;
  static_for<ncoef(P)>([&](auto sc) {
    constexpr int s = decltype(sc)::value;
    if constexpr (s > 0) {
      constexpr int l = kSlots[s].l, m = kSlots[s].m, n = kSlots[s].n;
      constexpr int a = l > 0 ? 0 : (m > 0 ? 1 : 2);  // recurse along axis a
      double acc = 0.0;
      if constexpr (l > 0) {
        acc = __builtin_fma((a == 0 ? 2.0 * l - 1.0 : 2.0 * l) * x, D[kSlot<l - 1, m, n>], acc);
        if constexpr (l > 1)
          acc = __builtin_fma(a == 0 ? (l - 1.0) * (l - 1.0) : l * (l - 1.0),
                              D[kSlot<l - 2, m, n>], acc);
      }
      if constexpr (m > 0) {
        acc = __builtin_fma((a == 1 ? 2.0 * m - 1.0 : 2.0 * m) * y, D[kSlot<l, m - 1, n>], acc);
        if constexpr (m > 1)
          acc = __builtin_fma(a == 1 ? (m - 1.0) * (m - 1.0) : m * (m - 1.0),
                              D[kSlot<l, m - 2, n>], acc);
      }
      if constexpr (n > 0) {
        acc = __builtin_fma((a == 2 ? 2.0 * n - 1.0 : 2.0 * n) * z, D[kSlot<l, m, n - 1>], acc);
        if constexpr (n > 1)
          acc = __builtin_fma(a == 2 ? (n - 1.0) * (n - 1.0) : n * (n - 1.0),
                              D[kSlot<l, m, n - 2>], acc);
      }
      D[s] = -acc * q;
    }
  });
}

// phi and a from moments M (about the node COM) and D at R = COM - target,
// with the reference's term selection (multipole.rs:1352-1528): phi drops
// the dipole (M about the COM), a_i = -sum_{|s|<=P-1} M[s] D[s + e_i].
template <int P, int WANT>
__device__ __forceinline__ void eval_multipole(const double *__restrict__ M,
                                               const double (&D)[ncoef(P)], double &ph,
                                               double &ax, double &ay, double &az) {
  if (WANT & PBX_WANT_POT) {
    double sum = 0.0;
    static_for<ncoef(P)>([&](auto kc) {
      constexpr int k = decltype(kc)::value;
      if constexpr (k == 0 || k > 3) sum = __builtin_fma(M[k], D[k], sum);
    });
    ph -= sum;
  }
  if (WANT & PBX_WANT_ACC) {
    constexpr int PA = P >= 2 ? P - 1 : 0;
    double gx = 0.0, gy = 0.0, gz = 0.0;
    static_for<ncoef(PA)>([&](auto kc) {
      constexpr int k = decltype(kc)::value;
      constexpr int l = kSlots[k].l, m = kSlots[k].m, n = kSlots[k].n;
      const double mk = M[k];
      gx = __builtin_fma(mk, D[kSlot<l + 1, m, n>], gx);
      gy = __builtin_fma(mk, D[kSlot<l, m + 1, n>], gy);
      gz = __builtin_fma(mk, D[kSlot<l, m, n + 1>], gz);
    });
    ax -= gx;
    ay -= gy;
    az -= gz;
  }
}

// ---------------------------------------------------------- softening
// kernel.rs:41-82 (Plummer 0, W2 spline 1); r is sqrt(r^2 + tiny).
__device__ __forceinline__ double w2_pot(double u) {
  double u2 = u * u;
  if (u < 0.5) {
    double u4 = u2 * u2;
    return (16.0 / 3.0) * u2 - (48.0 / 5.0) * u4 + (32.0 / 5.0) * (u4 * u) - 14.0 / 5.0;
  }
  if (u < 1.0) {
    double u3 = u2 * u, u4 = u2 * u2;
    return (1.0 / 15.0) / u + (32.0 / 3.0) * u2 - 16.0 * u3 + (48.0 / 5.0) * u4 -
           (32.0 / 15.0) * (u4 * u) - 16.0 / 5.0;
  }
  return -1.0 / u;
}

__device__ __forceinline__ double w2_der(double u) {
  double u2 = u * u, u3 = u2 * u, u4 = u2 * u2;
  if (u < 0.5) return (32.0 / 3.0) * u - (192.0 / 5.0) * u3 + 32.0 * u4;
  if (u < 1.0)
    return -(1.0 / 15.0) / u2 + (64.0 / 3.0) * u - 48.0 * u2 + (192.0 / 5.0) * u3 -
           (32.0 / 3.0) * u4;
  return 1.0 / u2;
}

__device__ __forceinline__ double kern_pot(int kind, double r, double h) {
  if (r == 0.0) return 0.0;
  if (kind == 0) return -1.0 / __builtin_sqrt(r * r + h * h);
  if (h <= 0.0) return -1.0 / r;
  return w2_pot(r / h) / h;
}

__device__ __forceinline__ double kern_acc(int kind, double r, double h) {
  if (r == 0.0) return 0.0;
  if (kind == 0) {
    double s2 = r * r + h * h;
    return 1.0 / (__builtin_sqrt(s2) * s2);
  }
  if (h <= 0.0) return 1.0 / (r * r * r);
  return w2_der(r / h) / (h * h) / r;
}

// squared distance with the reference's mul_add nesting (tree.rs:139,1117)
__device__ __forceinline__ double dist2_fma(double dx, double dy, double dz) {
#pragma clang fp contract(off)
  return __builtin_fma(dx, dx, __builtin_fma(dy, dy, dz * dz));
}

// dist2_fma(dx, dy, dz) + R2_TINY with the addition folded into the first
// multiply (one FP64 instruction less).  The same double except when dz^2
// is within ~2^52 R2_TINY of zero (separations below ~1e-146) or its exact
// value is a rounding tie (then one ulp): used by the fast walk (FAST =
// RAW, whose rsq is ~5e-8 anyway); the precise walk keeps the reference's
// sequence.
template <bool FAST>
__device__ __forceinline__ double dist2_tiny(double dx, double dy, double dz) {
#pragma clang fp contract(off)
  if constexpr (FAST) return __builtin_fma(dx, dx, __builtin_fma(dy, dy, __builtin_fma(dz, dz, kR2Tiny)));
  else return dist2_fma(dx, dy, dz) + kR2Tiny;
}

// ------------------------------------------------------------------ build
// bounding box: ordered keys of min x,y,z and max x,y,z (NaN ignored like
// the `<` / `>` updates of tree.rs:631-640).  The positions are read as one
// flat array of 3n doubles, lane-contiguous, four loads in flight per
// thread; the grid holds a multiple of 3 threads, so every element a thread
// sees lies on the same axis (its index mod 3).
__global__ void __launch_bounds__(TPB) bbox_kernel(const double *__restrict__ pos, int64_t n,
                                                   unsigned long long *__restrict__ out) {
  __shared__ unsigned long long red[6][NWAVE];
  const int64_t T = (int64_t)gridDim.x * TPB;  // a multiple of 3
  const int64_t t = (int64_t)blockIdx.x * TPB + threadIdx.x, m = 3 * n;
  unsigned long long mn = ~0ull, mx = 0ull;
  auto take = [&](double v) {
    if (v != v) return;
    const unsigned long long k = dkey(v);
    mn = k < mn ? k : mn;
    mx = k > mx ? k : mx;
  };
  int64_t j = t;
  for (; j + 3 * T < m; j += 4 * T) {
    double v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) v[u] = pos[j + u * T];
#pragma unroll
    for (int u = 0; u < 4; ++u) take(v[u]);
  }
  for (; j < m; j += T) take(pos[j]);
  const int ax = (int)(t % 3);
  const int w = threadIdx.x >> 6;
#pragma unroll
  for (int d = 0; d < 3; ++d) {
    unsigned long long lo = ax == d ? mn : ~0ull, hi = ax == d ? mx : 0ull;
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) {
      const unsigned long long a = __shfl_xor(lo, o, 64), b = __shfl_xor(hi, o, 64);
      lo = a < lo ? a : lo;
      hi = b > hi ? b : hi;
    }
    if ((threadIdx.x & 63) == 0) {
      red[d][w] = lo;
      red[3 + d][w] = hi;
    }
  }
  __syncthreads();
  if (threadIdx.x < 3) {
    int d = threadIdx.x;
    unsigned long long a = red[d][0], b = red[3 + d][0];
    for (int k = 1; k < NWAVE; ++k) {
      a = red[d][k] < a ? red[d][k] : a;
      b = red[3 + d][k] > b ? red[3 + d][k] : b;
    }
    atomicMin(&out[d], a);
    atomicMax(&out[3 + d], b);
  }
}

// Octant path of every particle through the reference's node centres,
// LPW levels per word (level 0 in the top bits of word 0).
__global__ void __launch_bounds__(TPB)
    path_keys(const double *__restrict__ pos, int64_t n, double cx0, double cy0, double cz0,
              double half0, int nwords, uint64_t *__restrict__ keys,
              const double *__restrict__ mass, double4 *__restrict__ rec0) {
#pragma clang fp contract(off)
  int64_t i = (int64_t)blockIdx.x * TPB + threadIdx.x;
  if (i >= n) return;
  const double x = pos[3 * i], y = pos[3 * i + 1], z = pos[3 * i + 2];
  // {x, y, z, m} in original order while the positions are in registers:
  // pack_records then gathers one 32-byte record per particle
  if (rec0) rec0[i] = make_double4(x, y, z, mass ? mass[i] : 1.0);
  double cx = cx0, cy = cy0, cz = cz0, h = half0;
  for (int w = 0; w < nwords; ++w) {
    uint64_t word = 0;
    for (int l = 0; l < LPW; ++l) {
      uint32_t o = (x >= cx ? 1u : 0u) | (y >= cy ? 2u : 0u) | (z >= cz ? 4u : 0u);
      word = (word << 3) | o;
      double off = h / 2.0;
      cx += (o & 1u) ? off : -off;
      cy += (o & 2u) ? off : -off;
      cz += (o & 4u) ? off : -off;
      h = off;
    }
    keys[(int64_t)w * n + i] = word;
  }
}

__global__ void gather_u64(const uint64_t *__restrict__ src, const int32_t *__restrict__ perm,
                           int64_t n, uint64_t *__restrict__ dst) {
  int64_t i = (int64_t)blockIdx.x * TPB + threadIdx.x;
  if (i < n) dst[i] = perm ? src[perm[i]] : src[i];
}

__global__ void __launch_bounds__(TPB) key_or_and(const uint64_t *__restrict__ k, int64_t n,
                                                  unsigned long long *__restrict__ out) {
  __shared__ unsigned long long so[NWAVE], sa[NWAVE];
  unsigned long long o = 0, a = ~0ull;
  for (int64_t i = (int64_t)blockIdx.x * TPB + threadIdx.x; i < n; i += (int64_t)gridDim.x * TPB) {
    o |= k[i];
    a &= k[i];
  }
#pragma unroll
  for (int s = 32; s >= 1; s >>= 1) {
    o |= __shfl_xor(o, s, 64);
    a &= __shfl_xor(a, s, 64);
  }
  if ((threadIdx.x & 63) == 0) {
    so[threadIdx.x >> 6] = o;
    sa[threadIdx.x >> 6] = a;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int w = 1; w < NWAVE; ++w) {
      o |= so[w];
      a &= sa[w];
    }
    atomicOr(&out[0], o);
    atomicAnd(&out[1], a);
  }
}

struct BuildView {
  const uint64_t *keys;  // sorted paths, nwords x n
  const int32_t *perm;   // sorted -> original
  const double *pos;     // original order
  int64_t n;
  int nwords;
  int64_t cap;           // leaf capacity
  int32_t *nstart, *ncount, *nfirst, *nnext, *nchild;
  double4 *ncen;         // centre xyz + half
};

__device__ __forceinline__ uint32_t digit_at(const BuildView &v, int64_t i, int d) {
  const uint64_t k = v.keys[(int64_t)(d / LPW) * v.n + i];
  return (uint32_t)(k >> (3 * (LPW - 1 - d % LPW))) & 7u;
}

// A node with more than leaf_capacity particles that all sit on one point
// never separates (tree.rs:847-864 recurses forever); it stays a leaf here.
__device__ bool all_identical(const BuildView &v, int64_t a, int64_t b) {
  for (int w = 0; w < v.nwords; ++w)
    if (v.keys[(int64_t)w * v.n + a] != v.keys[(int64_t)w * v.n + b - 1]) return false;
  const int64_t p0 = v.perm[a];
  const uint64_t *q0 = (const uint64_t *)(v.pos + 3 * p0);
  for (int64_t i = a + 1; i < b; ++i) {
    const uint64_t *q = (const uint64_t *)(v.pos + 3 * (int64_t)v.perm[i]);
    if (q[0] != q0[0] || q[1] != q0[1] || q[2] != q0[2]) return false;
  }
  return true;
}

__global__ void root_init(BuildView v, double cx, double cy, double cz, double half,
                          int32_t *__restrict__ frontier, uint32_t *__restrict__ nfront) {
  v.nstart[0] = 0;
  v.ncount[0] = (int32_t)v.n;
  v.nfirst[0] = -1;
  v.nnext[0] = -1;
  v.nchild[0] = 0;
  v.ncen[0] = make_double4(cx, cy, cz, half);
  bool split = v.n > v.cap && half != 0.0 && !all_identical(v, 0, v.n);
  if (split) frontier[0] = 0;
  *nfront = split ? 1u : 0u;
}

// children ranges of every frontier node: lb[f*9 + o] = first particle with
// digit >= o at level d (digits are sorted inside a node's range)
// 8 lanes per frontier node: lane o finds the first index of the node's
// (path-sorted) range with digit >= o by its own binary search (the eight
// searches of a node run side by side instead of one after another);
// lb[f][0..7] = those starts, lb[f][8] = end, cnt[f] = non-empty octants.
// Also zeroes the scan sentinel cnt[F] and the child flags (8F + 1 words,
// the most children the level can create) for split_make.
__global__ void split_count(BuildView v, const int32_t *__restrict__ frontier, int64_t F, int d,
                            int32_t *__restrict__ lb, uint32_t *__restrict__ cnt,
                            uint32_t *__restrict__ flags) {
  const int64_t t = (int64_t)blockIdx.x * TPB + threadIdx.x;
  const int64_t f = t >> 3;
  const uint32_t o = (uint32_t)(t & 7);
  const bool ok = f < F;
  if (t <= 8 * F) flags[t] = 0u;
  if (t == 0) cnt[F] = 0u;
  int64_t s = 0, e = 0;
  if (ok) {
    const int32_t node = frontier[f];
    s = v.nstart[node];
    e = s + v.ncount[node];
  }
  int64_t a = s, b = e;  // first index in [s, e) with digit >= o
  while (a < b) {
    const int64_t mid = (a + b) >> 1;
    if (digit_at(v, mid, d) < o) a = mid + 1;
    else b = mid;
  }
  // start of the next octant (lane o + 1; the end for o = 7), same 8-lane group
  const int64_t an = __shfl_down(a, 1, 8);
  const int64_t nxt = o == 7 ? e : an;
  const uint64_t nonempty = __ballot(ok && nxt > a);
  if (!ok) return;
  lb[f * 9 + o] = (int32_t)a;
  if (o == 7) lb[f * 9 + 8] = (int32_t)e;
  if (o == 0) cnt[f] = (uint32_t)__popcll((nonempty >> (threadIdx.x & 56)) & 0xffull);
}

// create the children of every frontier node (ids base + exclusive scan);
// flag the ones that must split at the next level
__global__ void split_make(BuildView v, const int32_t *__restrict__ frontier, int64_t F,
                           const int32_t *__restrict__ lb, const uint32_t *__restrict__ cbase,
                           int32_t level_base, uint32_t *__restrict__ flags) {
#pragma clang fp contract(off)
  int64_t f = (int64_t)blockIdx.x * TPB + threadIdx.x;
  if (f >= F) return;
  const int32_t node = frontier[f];
  const double4 pc = v.ncen[node];
  const double off = pc.w / 2.0;  // tree.rs:835
  int32_t k = level_base + (int32_t)cbase[f];
  int last = -1, nkid = 0;
  for (int o = 0; o < 8; ++o)
    if (lb[f * 9 + o + 1] > lb[f * 9 + o]) {
      last = o;
      ++nkid;
    }
  v.nfirst[node] = k;
  v.nchild[node] = nkid;
  const int32_t parent_next = v.nnext[node];
  for (int o = 0; o < 8; ++o) {
    const int32_t a = lb[f * 9 + o], b = lb[f * 9 + o + 1];
    if (b <= a) continue;
    const int32_t c = k++;
    double4 cc;
    cc.x = pc.x + ((o & 1) ? off : -off);
    cc.y = pc.y + ((o & 2) ? off : -off);
    cc.z = pc.z + ((o & 4) ? off : -off);
    cc.w = off;
    v.ncen[c] = cc;
    v.nstart[c] = a;
    v.ncount[c] = b - a;
    v.nfirst[c] = -1;
    v.nchild[c] = 0;
    v.nnext[c] = (o == last) ? parent_next : c + 1;
    bool split = (int64_t)(b - a) > v.cap && off != 0.0 && !all_identical(v, a, b);
    flags[c - level_base] = split ? 1u : 0u;
  }
}

// the next frontier; C (children made this level) is the scanned child
// count total cnt[F]; (C, next frontier size) go to sizes[0..1] for the
// level's single host read-back
__global__ void compact_frontier(const uint32_t *__restrict__ scanned,
                                 const uint32_t *__restrict__ cnt, int64_t F, int32_t level_base,
                                 int32_t *__restrict__ out, uint32_t *__restrict__ sizes) {
  const int64_t C = cnt[F];
  const int64_t c = (int64_t)blockIdx.x * TPB + threadIdx.x;
  if (c == 0) {
    sizes[0] = (uint32_t)C;
    sizes[1] = scanned[C];
  }
  if (c >= C) return;
  if (scanned[c + 1] != scanned[c]) out[scanned[c]] = level_base + (int32_t)c;
}

// leaf lists in ascending original index (the Rust Vec order of
// tree.rs:815-828), then the records of every particle in leaf order
__global__ void leaf_sort(const int32_t *__restrict__ nchild, const int32_t *__restrict__ nstart,
                          const int32_t *__restrict__ ncount, int64_t nn,
                          int32_t *__restrict__ perm) {
  int64_t k = (int64_t)blockIdx.x * TPB + threadIdx.x;
  if (k >= nn || nchild[k] != 0) return;
  const int32_t s = nstart[k], c = ncount[k];
  if (c <= 8) {  // in registers: a fixed sorting network (odd-even merge, 19
                 // compare-exchanges) — not an insertion sort whose every
                 // step is a dependent global read (~28 of them in a full leaf)
    constexpr int32_t PAD = 0x7fffffff;  // (original indices are < 2^31 - 1)
    int32_t v[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) v[q] = q < c ? perm[s + q] : PAD;
    auto cx = [&](int a, int b) {
      const int32_t lo = v[a] < v[b] ? v[a] : v[b], hi = v[a] < v[b] ? v[b] : v[a];
      v[a] = lo;
      v[b] = hi;
    };
    cx(0, 1); cx(2, 3); cx(4, 5); cx(6, 7);
    cx(0, 2); cx(1, 3); cx(4, 6); cx(5, 7);
    cx(1, 2); cx(5, 6);
    cx(0, 4); cx(1, 5); cx(2, 6); cx(3, 7);
    cx(2, 4); cx(3, 5);
    cx(1, 2); cx(3, 4); cx(5, 6);
#pragma unroll
    for (int q = 0; q < 8; ++q)
      if (q < c) perm[s + q] = v[q];
    return;
  }
  for (int32_t i = s + 1; i < s + c; ++i) {
    int32_t v = perm[i];
    int32_t j = i - 1;
    while (j >= s && perm[j] > v) {
      perm[j + 1] = perm[j];
      --j;
    }
    perm[j + 1] = v;
  }
}

__global__ void pack_records(const double4 *__restrict__ rec0, const int32_t *__restrict__ perm,
                             int64_t n, double4 *__restrict__ rec) {
  int64_t i = (int64_t)blockIdx.x * TPB + threadIdx.x;
  if (i < n) rec[i] = rec0[perm[i]];
}

__global__ void interleave_records(const double *__restrict__ pos, const double *__restrict__ mass,
                                   int64_t n, double4 *__restrict__ rec0) {
  int64_t i = (int64_t)blockIdx.x * TPB + threadIdx.x;
  if (i < n) rec0[i] = make_double4(pos[3 * i], pos[3 * i + 1], pos[3 * i + 2], mass ? mass[i] : 1.0);
}

__global__ void gather_f64(const double *__restrict__ src, const int32_t *__restrict__ perm,
                           int64_t n, double *__restrict__ dst) {
  int64_t i = (int64_t)blockIdx.x * TPB + threadIdx.x;
  if (i < n) dst[i] = src[perm[i]];
}

// P2M of one particle at (x, y, z) relative to the expansion centre:
// M[l,m,n] += mass x^l y^m z^n / (l! m! n!)
template <int P>
__device__ __forceinline__ void p2m_add(double (&M)[ncoef(P)], double m, double x, double y,
                                        double z) {
  double px[P + 1], py[P + 1], pz[P + 1];
  px[0] = m;
  py[0] = 1.0;
  pz[0] = 1.0;
  static_for<P>([&](auto ac) {
    constexpr int a = decltype(ac)::value + 1;
    px[a] = px[a - 1] * x * (1.0 / a);
    py[a] = py[a - 1] * y * (1.0 / a);
    pz[a] = pz[a - 1] * z * (1.0 / a);
  });
  static_for<ncoef(P)>([&](auto sc) {
    constexpr int s = decltype(sc)::value;
    M[s] += px[kSlots[s].l] * (py[kSlots[s].m] * pz[kSlots[s].n]);
  });
}

// M2M: moments C about the child COM shifted by t = parent COM - child COM
// (multipole.rs:1536-1595 in binomial form):
//   M[l,m,n] += sum_{i<=l, j<=m, k<=n} C[i,j,k] (-t)^(l-i,m-j,n-k) / (l-i)!(m-j)!(n-k)!
template <int P>
__device__ __forceinline__ void m2m_add(double (&M)[ncoef(P)], const double *__restrict__ C,
                                        int64_t cs, double tx, double ty, double tz) {
  double ex[P + 1], ey[P + 1], ez[P + 1];
  ex[0] = ey[0] = ez[0] = 1.0;
  static_for<P>([&](auto ac) {
    constexpr int a = decltype(ac)::value + 1;
    ex[a] = ex[a - 1] * (-tx) * (1.0 / a);
    ey[a] = ey[a - 1] * (-ty) * (1.0 / a);
    ez[a] = ez[a - 1] * (-tz) * (1.0 / a);
  });
  double c[ncoef(P)];
  static_for<ncoef(P)>([&](auto sc) { c[decltype(sc)::value] = C[decltype(sc)::value * cs]; });
  static_for<ncoef(P)>([&](auto sc) {
    constexpr int s = decltype(sc)::value;
    constexpr int l = kSlots[s].l, m = kSlots[s].m, n = kSlots[s].n;
    double acc = 0.0;
    static_for<l + 1>([&](auto ic) {
      constexpr int i = decltype(ic)::value;
      static_for<m + 1>([&](auto jc) {
        constexpr int j = decltype(jc)::value;
        static_for<n + 1>([&](auto kc) {
          constexpr int k = decltype(kc)::value;
          acc = __builtin_fma(c[kSlot<i, j, k>], ex[l - i] * (ey[m - j] * ez[n - k]), acc);
        });
      });
    });
    M[s] += acc;
  });
}

// One record per node in DFS preorder, read by a wave with a single burst of
// scalar loads:  [cx cy cz mass | size2 hmax | next first | leaf_start count]
// (64 B) followed by the node's evaluation coefficients (orders 2-3: the
// detraced Q', K'; orders 4-5: raw moments).
template <int P> __host__ __device__ constexpr int rec_stride() {
  return P <= 1 ? 8 : (P == 2 ? 16 : (P == 3 ? 24 : (P == 4 ? 48 : 64)));
}

template <int P>
__device__ __forceinline__ void detraced_coef(const double *M, double *C) {
  const double sxx = 2.0 * M[4], syy = 2.0 * M[5], szz = 2.0 * M[6];
  const double tr3 = (sxx + syy + szz) * (1.0 / 3.0);
  C[0] = 1.5 * (sxx - tr3);
  C[1] = 1.5 * (syy - tr3);
  C[2] = 1.5 * (szz - tr3);
  C[3] = 1.5 * M[7];  // xy
  C[4] = 1.5 * M[8];  // xz
  C[5] = 1.5 * M[9];  // yz
  if constexpr (P == 3) {
    // S_ijk = l! m! n! M_lmn
    const double sxxx = 6.0 * M[10], syyy = 6.0 * M[11], szzz = 6.0 * M[12];
    const double sxxy = 2.0 * M[13], sxxz = 2.0 * M[14], sxyy = 2.0 * M[15];
    const double sxzz = 2.0 * M[16], syyz = 2.0 * M[17], syzz = 2.0 * M[18];
    const double sxyz = M[19];
    const double tx = sxxx + sxyy + sxzz, ty = sxxy + syyy + syzz, tz = sxxz + syyz + szzz;
    // T[S3]_ijk = S_ijk - (d_ij t_k + d_ik t_j + d_jk t_i) / 5
    const double oxxx = sxxx - 0.6 * tx, oyyy = syyy - 0.6 * ty, ozzz = szzz - 0.6 * tz;
    const double oxxy = sxxy - 0.2 * ty, oxxz = sxxz - 0.2 * tz, oxyy = sxyy - 0.2 * tx;
    const double oxzz = sxzz - 0.2 * tx, oyyz = syyz - 0.2 * tz, oyzz = syzz - 0.2 * ty;
    C[6] = 2.5 * oxxx;         // x^3
    C[7] = 2.5 * 3.0 * oxxy;   // x^2 y
    C[8] = 2.5 * 3.0 * oxxz;   // x^2 z
    C[9] = 2.5 * 3.0 * oxyy;   // x y^2
    C[10] = 2.5 * 6.0 * sxyz;  // x y z
    C[11] = 2.5 * 3.0 * oxzz;  // x z^2
    C[12] = 2.5 * oyyy;        // y^3
    C[13] = 2.5 * 3.0 * oyyz;  // y^2 z
    C[14] = 2.5 * 3.0 * oyzz;  // y z^2
    C[15] = 2.5 * ozzz;        // z^3
  }
}

struct PayloadView {
  const int32_t *nstart, *ncount, *nfirst, *nchild;
  const double4 *rec;
  const double *soft;  // sorted softenings or null
  double4 *com;        // com xyz + mass
  double *hmax;        // or null
  double *mom;         // ncoef(P) per node (P >= 2) or null; coefficient q of node k at q * nn + k
  // the node's walk record, written here too (DFS preorder pre[k])
  const int32_t *pre, *size;
  const double4 *ncen;
  int64_t nn;
  double *walk;
  const uint8_t *leaf_dfs;  // per DFS id: no children (walk-record flags), or null
};

// Bottom-up payload pass (tree.rs:866-1067) in two parts:
//  * payload_leaves: every leaf at once (leaves depend on nothing; 85 % of
//    the nodes at 4M) — mass / COM over its records in index order, h_max,
//    P2M at the COM, one lane per leaf;
//  * payload_internal, one launch per level, bottom up: EIGHT lanes per
//    internal node, lane q on child q.  Every lane sums the children's mass
//    and COM in octant order exactly as the reference (contraction off:
//    bit-identical), then lane q shifts child q's moments to the node's COM
//    (M2M) and the eight shifted moments are added by a fixed butterfly.
//    One lane per node made each node ~11 dependent memory round trips
//    (links, child COMs, then each child's 20 moments in turn) at 2 waves
//    per SIMD: the levels were latency-bound (SQ counters,
//    profiles/r3/payload_split_rejected/); with a lane per child the
//    children's moments arrive in one round trip and a level has 8x the
//    waves to hide it.
// Moments are coefficient-major (q * nn + k) and the walk records (DFS
// preorder) leave in record-contiguous pieces.
constexpr int PL_TPB = 256;

// Walk-record flags: bits of the record's leaf-count word (dword 15) saying
// whether the node the wave steps to next — `next`, or `first` when some
// lane opens — is a leaf.  A leaf step reads only the record's first
// 64-byte chunk, so the walk then issues one scalar load for it instead of
// the record's NCH.  The flags come from the structure (no children), known
// before any payload: an empty internal node (walked as a leaf) is simply
// not flagged and loads its whole record.
constexpr uint32_t WF_NEXT_LEAF = 1u << 30, WF_FIRST_LEAF = 1u << 29;
constexpr uint32_t WF_COUNT = WF_FIRST_LEAF - 1u;

// leaf_dfs[pre[k]] = node k has no children
__global__ void leaf_dfs_kernel(const int32_t *__restrict__ nchild, const int32_t *__restrict__ pre,
                                int64_t nn, uint8_t *__restrict__ leaf_dfs) {
  const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (k < nn) leaf_dfs[pre[k]] = nchild[k] == 0 ? 1 : 0;
}

// the node's walk record: [cx cy cz mass | size2 hmax | next first |
// leaf_start count + flags] and the evaluation coefficients
template <int P>
__device__ __forceinline__ void walk_record(const PayloadView &v, int32_t k, int32_t pk, int32_t nc,
                                            double cx, double cy, double cz, double mass, double hm,
                                            const double *M, double *r) {
#pragma clang fp contract(off)
  r[0] = cx;
  r[1] = cy;
  r[2] = cz;
  r[3] = mass;
  const double sz = v.ncen[k].w * 2.0;  // tree.rs:794-798
  r[4] = sz * sz;
  r[5] = v.hmax ? hm : 0.0;
  // DFS preorder ids: first child = k + 1, next_branch = k + subtree size
  // (the same threading as tree.rs:736-776, renumbered)
  const int64_t after = (int64_t)pk + v.size[k];
  const bool leaf = nc == 0;
  int32_t ir[4];
  ir[0] = after < v.nn ? (int32_t)after : -1;
  ir[1] = leaf ? -1 : pk + 1;
  ir[2] = leaf ? v.nstart[k] : 0;
  ir[3] = leaf ? v.ncount[k] : 0;
  // an empty node (mass 0, tree.rs:1087-1090: skipped) walks as a leaf of no
  // records: no descent, no pairs, the same next — one sign test in the
  // walk decides leaf / internal
  if (mass == 0.0) {
    ir[1] = -1;
    ir[2] = 0;
    ir[3] = 0;
  }
  if (v.leaf_dfs) {
    if (ir[0] >= 0 && v.leaf_dfs[ir[0]]) ir[3] |= (int32_t)WF_NEXT_LEAF;
    if (ir[1] >= 0 && v.leaf_dfs[ir[1]]) ir[3] |= (int32_t)WF_FIRST_LEAF;
  }
  r[6] = __builtin_bit_cast(double, (uint64_t)(uint32_t)ir[0] | ((uint64_t)(uint32_t)ir[1] << 32));
  r[7] = __builtin_bit_cast(double, (uint64_t)(uint32_t)ir[2] | ((uint64_t)(uint32_t)ir[3] << 32));
  if constexpr (P == 2 || P == 3) {
    detraced_coef<P>(M, r + 8);
  } else if constexpr (P >= 4) {
#pragma unroll
    for (int q = 0; q < ncoef(P); ++q) r[8 + q] = M[q];
  }
}

template <int P>
__global__ void __launch_bounds__(PL_TPB) payload_leaves(PayloadView v) {
  constexpr int RS = rec_stride<P>();
  constexpr int HW = (RS + 1) / 2;  // record words per transposition half
  constexpr int HP = HW + 1;        // LDS row stride (odd)
  __shared__ double rs[(PL_TPB / 64) * 64 * HP];
  const int64_t k64 = (int64_t)blockIdx.x * PL_TPB + threadIdx.x;
  const bool in = k64 < v.nn;
  const int32_t k = in ? (int32_t)k64 : 0;
  // the node's fields all at once (no branch between their loads)
  const int32_t nch = in ? v.nchild[k] : 1;
  const int32_t s0 = v.nstart[k], c0 = v.ncount[k], pk0 = v.pre[k];
  const bool live = in && nch == 0;
  const int32_t s = s0, c = live ? c0 : 0, pk = live ? pk0 : -1;
  double mass = 0.0, cx = 0.0, cy = 0.0, cz = 0.0, hm = 0.0;
  constexpr int PL = 8;  // leaves of up to PL records: all of them in flight at once
  double4 rr[PL];
  const bool small = c <= PL;
  if (small) {
#pragma unroll
    for (int q = 0; q < PL; ++q) rr[q] = v.rec[q < c ? s + q : s];
  }
  {
#pragma clang fp contract(off)
    if (small) {
#pragma unroll
      for (int q = 0; q < PL; ++q) {
        if (q >= c) break;
        mass += rr[q].w;
        cx += rr[q].x * rr[q].w;
        cy += rr[q].y * rr[q].w;
        cz += rr[q].z * rr[q].w;
      }
    } else {
      for (int32_t j = s; j < s + c; ++j) {
        const double4 r = v.rec[j];
        mass += r.w;
        cx += r.x * r.w;
        cy += r.y * r.w;
        cz += r.z * r.w;
      }
    }
    if (mass > 0.0) {
      cx /= mass;
      cy /= mass;
      cz /= mass;
    }
  }
  if (v.hmax)
    for (int32_t j = s; j < s + c; ++j) hm = __builtin_fmax(hm, __builtin_fmax(v.soft[j], 0.0));
  double M[P >= 2 ? ncoef(P) : 1];
  static_for<(P >= 2 ? ncoef(P) : 1)>([&](auto qc) { M[decltype(qc)::value] = 0.0; });
  if constexpr (P >= 2) {
    if (mass != 0.0) {
      if (small) {
#pragma unroll
        for (int q = 0; q < PL; ++q) {
          if (q >= c) break;
          p2m_add<P>(M, rr[q].w, rr[q].x - cx, rr[q].y - cy, rr[q].z - cz);
        }
      } else {
        for (int32_t j = s; j < s + c; ++j) {
          const double4 r = v.rec[j];
          p2m_add<P>(M, r.w, r.x - cx, r.y - cy, r.z - cz);
        }
      }
    }
    if (live)
      static_for<ncoef(P)>([&](auto qc) {
        v.mom[(int64_t)decltype(qc)::value * v.nn + k] = M[decltype(qc)::value];
      });
  }
  if (live) {
    v.com[k] = make_double4(cx, cy, cz, mass);
    if (v.hmax) v.hmax[k] = hm;
  }
  double r[2 * HW];
  r[2 * HW - 1] = 0.0;
  if (live) walk_record<P>(v, k, pk, 0, cx, cy, cz, mass, hm, M, r);
  // the records leave through this wave's LDS rows, half a record at a
  // time: consecutive lanes store consecutive words of one record (no block
  // barrier: a wave's LDS operations complete in order)
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  double *wr = rs + w * 64 * HP;
#pragma unroll
  for (int h = 0; h < 2; ++h) {
#pragma unroll
    for (int j = 0; j < HW; ++j) wr[lane * HP + j] = r[h * HW + j];
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    for (int idx = lane; idx < 64 * HW; idx += 64) {
      const int i = idx / HW, j = idx - i * HW;
      const int32_t pi = __shfl(pk, i, 64);
      if (pi >= 0 && h * HW + j < RS) v.walk[(int64_t)pi * RS + h * HW + j] = wr[i * HP + j];
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  }
}

// the internal nodes, breadth-first (so level by level): flag, scan, list
__global__ void internal_flags(const int32_t *__restrict__ nchild, int64_t nn,
                               uint32_t *__restrict__ flag) {
  const int64_t k = (int64_t)blockIdx.x * TPB + threadIdx.x;
  if (k <= nn) flag[k] = (k < nn && nchild[k] > 0) ? 1u : 0u;
}
__global__ void internal_list(const int32_t *__restrict__ nchild, const uint32_t *__restrict__ scan,
                              int64_t nn, int32_t *__restrict__ list) {
  const int64_t k = (int64_t)blockIdx.x * TPB + threadIdx.x;
  if (k < nn && nchild[k] > 0) list[scan[k]] = (int32_t)k;
}

constexpr int PI_G = 8;  // lanes per internal node: one per child slot
template <int P>
__global__ void __launch_bounds__(PL_TPB)
    payload_internal(PayloadView v, const int32_t *__restrict__ ilist,
                     const uint32_t *__restrict__ iscan, int32_t a, int32_t b, int64_t lo_h,
                     int64_t hi_h) {
  constexpr int RS = rec_stride<P>();
  constexpr int NM = P >= 2 ? ncoef(P) : 1;
  // the level's run of the internal list: from the host when the build
  // counted it (lo_h >= 0), else from the scan
  const uint32_t lo = lo_h >= 0 ? (uint32_t)lo_h : iscan[a];
  const uint32_t hi = lo_h >= 0 ? (uint32_t)hi_h : iscan[b];
  const uint32_t g0 = lo + blockIdx.x * (PL_TPB / PI_G);
  if (g0 >= hi) return;  // (uniform: the grid is an upper bound)
  const int q = (int)(threadIdx.x & (PI_G - 1));
  const uint32_t g = g0 + threadIdx.x / PI_G;
  const bool live = g < hi;
  const int32_t k = live ? ilist[g] : 0;
  const int32_t nc = live ? v.nchild[k] : 0, f = live ? v.nfirst[k] : 0;
  const int32_t pk = live ? v.pre[k] : 0;
  const int64_t nn = v.nn;
  // mass / COM over the children in octant order, on every lane alike
  double4 cq[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) cq[j] = v.com[j < nc ? f + j : f];
  double mass = 0.0, cx = 0.0, cy = 0.0, cz = 0.0, hm = 0.0;
  {
#pragma clang fp contract(off)
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      if (j >= nc) break;
      const double4 c4 = cq[j];
      if (c4.w == 0.0) continue;
      mass += c4.w;
      cx += c4.x * c4.w;
      cy += c4.y * c4.w;
      cz += c4.z * c4.w;
    }
    if (mass > 0.0) {
      cx /= mass;
      cy /= mass;
      cz /= mass;
    }
  }
  if (v.hmax) {  // the children's h_max (lane q: child q), max over the group
    hm = q < nc ? v.hmax[f + q] : 0.0;
#pragma unroll
    for (int o = 1; o < PI_G; o <<= 1) hm = __builtin_fmax(hm, __shfl_xor(hm, o, 64));
  }
  double M[NM];
  static_for<NM>([&](auto qc) { M[decltype(qc)::value] = 0.0; });
  if constexpr (P >= 2) {
    // child q's moments shifted to this node's COM
    const double4 mine = v.com[q < nc ? f + q : f];  // (a load: a select chain over cq spills)
    if (live && q < nc && mass != 0.0 && mine.w != 0.0)
      m2m_add<P>(M, v.mom + (f + q), nn, cx - mine.x, cy - mine.y, cz - mine.z);
    // the eight children's shifts, added by a fixed butterfly
#pragma unroll
    for (int o = 1; o < PI_G; o <<= 1)
      static_for<NM>([&](auto qc) {
        constexpr int t = decltype(qc)::value;
        M[t] += __shfl_xor(M[t], o, 64);
      });
  }
  if (!live) return;
  if constexpr (P >= 2)
    static_for<NM>([&](auto qc) {
      constexpr int t = decltype(qc)::value;
      if (t % PI_G == q) v.mom[(int64_t)t * nn + k] = M[t];
    });
  if (q == 0) {
    v.com[k] = make_double4(cx, cy, cz, mass);
    if (v.hmax) v.hmax[k] = hm;
  }
  double r[RS];
  walk_record<P>(v, k, pk, nc, cx, cy, cz, mass, hm, M, r);
#pragma unroll
  for (int j = 0; j < RS; ++j)
    if (j % PI_G == q) v.walk[(int64_t)pk * RS + j] = r[j];
}

// Detraced evaluation coefficients (orders 2 and 3).  With raw moments
// M_lmn = sum m x^l y^m z^n / (l! m! n!) and S^(n) = sum m x^(n-fold), the
// order-n part of the reference's sum_k M_k D_k(R) is
//   (1/n!) S^(n) : grad^n (1/r) = (1/n!) (-1)^n (2n-1)!! r^-(2n+1) T[S^(n)] : R^n
// because grad^n (1/r) is the detraced tensor (-1)^n (2n-1)!! T[R^n] / r^(2n+1)
// and T is an orthogonal projection.  Per node we store
//   Q' = 3/2 T[S2]           (xx, yy, zz, xy, xz, yz)
//   K' = 5/2 T[S3] with each component times its multinomial weight
//        (x^3, x^2y, x^2z, xy^2, xyz, xz^2, y^3, y^2z, yz^2, z^3)
// so phi = -M/r - q2'/r^5 + q3'/r^7 with q2' = R.Q'.R and q3' = K'(R).
__host__ __device__ constexpr int ncoef_fast(int P) { return P == 3 ? 16 : (P == 2 ? 6 : 0); }

// ------------------------------------------------------------------- walk
// One record per node in DFS preorder, read by a wave with a single burst of
// scalar loads:  [cx cy cz mass | size2 hmax | next first | leaf_start count]
// (64 B) followed by the node's evaluation coefficients (orders 2-3: the
// detraced Q', K'; orders 4-5: raw moments).
// (rec_stride: defined with the payload, which writes the walk records)

// subtree sizes, one level bottom-up
__global__ void subtree_size(const int32_t *__restrict__ nfirst, const int32_t *__restrict__ nchild,
                             int32_t a, int32_t b, int32_t *__restrict__ size) {
  int32_t k = a + (int32_t)(blockIdx.x * TPB + threadIdx.x);
  if (k >= b) return;
  int32_t s = 1;
  const int32_t f = nfirst[k], nc = nchild[k];
  for (int32_t c = f; c < f + nc; ++c) s += size[c];
  size[k] = s;
}

// DFS preorder ids of the children of one level's nodes, top-down
__global__ void preorder_ids(const int32_t *__restrict__ nfirst, const int32_t *__restrict__ nchild,
                             const int32_t *__restrict__ size, int32_t a, int32_t b,
                             int32_t *__restrict__ pre) {
  int32_t k = a + (int32_t)(blockIdx.x * TPB + threadIdx.x);
  if (k >= b) return;
  int32_t run = pre[k] + 1;
  const int32_t f = nfirst[k], nc = nchild[k];
  for (int32_t c = f; c < f + nc; ++c) {
    pre[c] = run;
    run += size[c];
  }
}

struct WalkParams {
  const double *walk;       // node records in DFS preorder, rec_stride<P>() doubles each
  const double4 *rec;       // sources in leaf order (+ 4 zero records of padding)
  const double *soft;       // sorted softenings (softenings set) or null
  const double *tgt;        // (m, 3) query points; null => targets are the sources
  const int32_t *perm;      // leaf order -> original index (self mode)
  int64_t m;                // number of targets
  int64_t first;            // self mode: targets are leaf-order particles first .. first+m-1
  int compact;              // self mode: 1 -> outputs at t (leaf order), 0 -> original index
  int32_t *cost;            // optional per-target cost (cost_kind)
  int cost_kind;            // 0: interactions (nodes + leaf pairs); 1: the wave's work
  double theta2;
  double sep;               // multipole_min_separation_factor (kernel.rs:20-37)
  int kernel;
  int has_hmax;
  double *pot, *acc;
  unsigned long long *counters;  // [accepted nodes, leaf pairs, fault, wave steps, active lanes]
  int64_t max_steps;             // > number of nodes
  unsigned int *fault;           // set when a wave exceeds max_steps
  unsigned xcd_chunk;            // blocks per XCD chunk (0: launch order)
  unsigned long long *trace;     // diagnostic (PBX_WALK_TRACE): per block start, end, steps
};

typedef uint32_t u32x16 __attribute__((ext_vector_type(16)));

// 64-byte scalar chunk -> the i-th double / int of it (i compile-time)
__device__ __forceinline__ double chunk_d(const u32x16 &c, int i) {
  return __builtin_bit_cast(double, (uint64_t)c[2 * i] | ((uint64_t)c[2 * i + 1] << 32));
}
__device__ __forceinline__ int32_t chunk_i(const u32x16 &c, int i) { return (int32_t)c[i]; }

// the chunks of one node record (or of 4 leaf records) with all scalar
// loads in flight together: one memory round trip (the compiler would sink
// the coefficient loads into the accept branch and serialise them)
template <int NCH>
__device__ __forceinline__ void load_chunks(const double *ptr, u32x16 (&c)[NCH]) {
  // the address is wave-uniform; make sure it sits in SGPRs
  const uint64_t a = (uint64_t)ptr;
  // (readfirstlane returns a signed int: go through uint32_t so the low
  // word is zero-extended, not sign-extended)
  const uint32_t hi = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(a >> 32));
  const uint32_t lo = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)a);
  const double *base = (const double *)(((uint64_t)hi << 32) | (uint64_t)lo);
  if constexpr (NCH == 1) {
    asm volatile("s_load_dwordx16 %0, %1, 0x0\n\ts_waitcnt lgkmcnt(0)"
                 : "=&s"(c[0]) : "s"(base) : "memory");
  } else if constexpr (NCH == 2) {
    asm volatile("s_load_dwordx16 %0, %2, 0x0\n\ts_load_dwordx16 %1, %2, 0x40\n\t"
                 "s_waitcnt lgkmcnt(0)"
                 : "=&s"(c[0]), "=&s"(c[1]) : "s"(base) : "memory");
  } else {
    static_assert(NCH == 3, "node records are 1-3 chunks");
    asm volatile("s_load_dwordx16 %0, %3, 0x0\n\ts_load_dwordx16 %1, %3, 0x40\n\t"
                 "s_load_dwordx16 %2, %3, 0x80\n\ts_waitcnt lgkmcnt(0)"
                 : "=&s"(c[0]), "=&s"(c[1]), "=&s"(c[2]) : "s"(base) : "memory");
  }
}

// load_chunks for a walk step: the chunks past the first only when the
// node is not known to be a leaf (leaf = 1).  One asm block with its own
// branch, so the chunk registers are the same on both paths (as two C++
// paths the chunks became phis of undefined values: ~200 SGPR spills)
template <int NCH>
__device__ __forceinline__ void load_chunks_node(const double *ptr, u32x16 (&c)[NCH], uint32_t leaf) {
  if constexpr (NCH == 1) {
    load_chunks<1>(ptr, c);
  } else {
    const uint64_t a = (uint64_t)ptr;
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(a >> 32));
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)a);
    const double *base = (const double *)(((uint64_t)hi << 32) | (uint64_t)lo);
    const uint32_t lf = (uint32_t)__builtin_amdgcn_readfirstlane((int)leaf);
    if constexpr (NCH == 2) {
      asm volatile("s_load_dwordx16 %0, %2, 0x0\n\ts_bitcmp1_b32 %3, 0\n\t"
                   "s_cbranch_scc1 1f\n\ts_load_dwordx16 %1, %2, 0x40\n1:\n\t"
                   "s_waitcnt lgkmcnt(0)"
                   : "=&s"(c[0]), "=&s"(c[1]) : "s"(base), "s"(lf) : "memory", "scc");
    } else {
      static_assert(NCH == 3, "node records are 1-3 chunks");
      asm volatile("s_load_dwordx16 %0, %3, 0x0\n\ts_bitcmp1_b32 %4, 0\n\t"
                   "s_cbranch_scc1 1f\n\ts_load_dwordx16 %1, %3, 0x40\n\t"
                   "s_load_dwordx16 %2, %3, 0x80\n1:\n\ts_waitcnt lgkmcnt(0)"
                   : "=&s"(c[0]), "=&s"(c[1]), "=&s"(c[2]) : "s"(base), "s"(lf) : "memory", "scc");
    }
  }
}

// one source pair of a leaf (tree.rs:98-417), self pair neutralised
template <int WANT, bool SOFT, bool RAW>
__device__ __forceinline__ void leaf_pair(const WalkParams &wp, double sx, double sy, double sz,
                                          double sm, double sh, bool me, double tx, double ty,
                                          double tz, double th, double &ph, double &ax,
                                          double &ay, double &az) {
  double dx = sx - tx, dy = sy - ty, dz = sz - tz;
  const double m = me ? 0.0 : sm;
  dx = me ? 1.0 : dx;
  if constexpr (!SOFT) {  // (the unsoftened pair: r^2 + R2_TINY in one chain)
    const double y = rsq_walk<RAW>(dist2_tiny<RAW>(dx, dy, dz));
    if (WANT & PBX_WANT_POT) ph = __builtin_fma(-m, y, ph);
    if (WANT & PBX_WANT_ACC) {
      const double g = m * (y * y * y);
      ax = __builtin_fma(g, dx, ax);
      ay = __builtin_fma(g, dy, ay);
      az = __builtin_fma(g, dz, az);
    }
    return;
  }
  const double r2 = dist2_fma(dx, dy, dz);
  double h = 0.0;
  if (SOFT) h = wp.soft ? __builtin_fmax(__builtin_fmax(sh, 0.0), th) : th;
  if (!SOFT || h <= 0.0 || (wp.kernel == 1 && r2 >= h * h)) {
    const double y = rsq_walk<RAW>(r2 + kR2Tiny);
    if (WANT & PBX_WANT_POT) ph = __builtin_fma(-m, y, ph);
    if (WANT & PBX_WANT_ACC) {
      const double g = m * (y * y * y);
      ax = __builtin_fma(g, dx, ax);
      ay = __builtin_fma(g, dy, ay);
      az = __builtin_fma(g, dz, az);
    }
  } else {
    const double rr = __builtin_sqrt(r2 + kR2Tiny);
    if (WANT & PBX_WANT_POT) ph = __builtin_fma(m, kern_pot(wp.kernel, rr, h), ph);
    if (WANT & PBX_WANT_ACC) {
      const double g = m * kern_acc(wp.kernel, rr, h);
      ax = __builtin_fma(g, dx, ax);
      ay = __builtin_fma(g, dy, ay);
      az = __builtin_fma(g, dz, az);
    }
  }
}

// the pairs of one leaf [s, e) for this lane's target, ascending index
// order (tree.rs:1093-1110); SELF: the leaf may hold the target itself
template <int WANT, bool SOFT, bool RAW, bool SELF>
__device__ __forceinline__ void leaf_sum(const WalkParams &wp, int32_t s, int32_t e, int32_t self,
                                         double tx, double ty, double tz, double th, double &ph,
                                         double &ax, double &ay, double &az) {
  for (int32_t j = s; j < e; j += 4) {  // 4 records (128 B) per round trip
    u32x16 r[2];
    load_chunks<2>((const double *)(wp.rec + j), r);
    double4 hs = make_double4(0.0, 0.0, 0.0, 0.0);
    if (SOFT && wp.soft) hs = *(const double4 *)(wp.soft + j);
    const double hv[4] = {hs.x, hs.y, hs.z, hs.w};
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      if (j + q < e)
        leaf_pair<WANT, SOFT, RAW>(wp, chunk_d(r[q / 2], 4 * (q & 1)),
                                   chunk_d(r[q / 2], 4 * (q & 1) + 1),
                                   chunk_d(r[q / 2], 4 * (q & 1) + 2),
                                   chunk_d(r[q / 2], 4 * (q & 1) + 3), hv[q],
                                   SELF && j + q == self, tx, ty, tz, th, ph, ax, ay, az);
    }
  }
}

// SOFT: h_max guard and/or softened leaf sums are live.  The walk hides
// its scalar-load latency with other waves: orders <= 3 without softening
// are held to 7 waves per SIMD (~100 SGPRs would leave room for only 6; at
// 8 the 64-VGPR budget spilled to scratch inside the accept path and parked
// ~30 SGPRs in VGPR lanes — 110 v_readlane; at 7: 88 SGPRs, 65 VGPRs, no
// scratch, 20 v_readlane, walk 44.5 -> 44.2 ms same-box A/B).
// LCOST: per-lane interaction counts are wanted (cost kind 0 with a cost
// array); otherwise their per-step VALU updates are compiled out
// W8: 8 waves per SIMD (the order-3 force + potential walks without
// softening: 56 VGPRs, ~78 SGPRs, 36 B of scratch outside the loop; the
// 4M walk 31.1-31.2 -> 30.4-30.5 ms against 7 waves, profiles/r5/r5z6/)
// CNT: the walk statistics (interaction counts, SIMD-efficiency counters:
// pbx_octree_info) are accumulated; a walk whose caller turned them off
// (pbx_octree_set_walk_counters) runs without their ~7 scalar operations per
// wave step — the same decisions and sums, only the instrumentation is gone.
template <int P, int WANT, bool SOFT, bool RAW, bool LCOST = true, bool W8 = false,
          bool CNT = true>
__global__ void __launch_bounds__(WALK_TPB)
    __attribute__((amdgpu_waves_per_eu(W8 ? 8 : ((P <= 3 && !SOFT) ? 7 : 1), W8 ? 8 : 7)))
    walk_kernel(WalkParams wp) {
  constexpr int RS = rec_stride<P>();
  constexpr int NCH = (P == 2 || P == 3) ? RS / 8 : 1;  // chunks loaded eagerly
  const unsigned long long t_start = wp.trace ? (unsigned long long)wall_clock64() : 0ull;  // (100 MHz)
  const unsigned lb = wp.xcd_chunk ? xcd_chunk_swizzle(blockIdx.x, wp.xcd_chunk) : blockIdx.x;
  const bool lane0 = (threadIdx.x & 63) == 0;
  const int64_t t = (int64_t)lb * blockDim.x + threadIdx.x;
  const bool valid = t < wp.m;
  const bool self_mode = wp.tgt == nullptr;
  double tx = 0.0, ty = 0.0, tz = 0.0, th = 0.0;
  int32_t self32 = -1;  // this target's own record (self mode)
  if (valid) {
    if (self_mode) {
      const int64_t ts = wp.first + t;
      const double4 r = wp.rec[ts];
      tx = r.x;
      ty = r.y;
      tz = r.z;
      self32 = (int32_t)ts;
      if (SOFT && wp.soft) th = __builtin_fmax(wp.soft[ts], 0.0);
    } else {
      tx = wp.tgt[3 * t];
      ty = wp.tgt[3 * t + 1];
      tz = wp.tgt[3 * t + 2];
    }
  }
  const bool has_th = SOFT && self_mode && wp.soft != nullptr;
  double ph = 0.0, ax = 0.0, ay = 0.0, az = 0.0;
  int32_t cost = 0;  // this lane's accepted nodes + leaf pairs
  // wave-uniform counters (ballot popcounts, kept in SGPRs)
  // (32-bit: a wave's counts stay below 2^32 — at most 64 lanes x 2^31
  // pairs would not, so n_pp is added to 64 bits per leaf; one scalar add
  // per counter instead of an add / add-with-carry pair)
  uint32_t n_node = 0, n_active = 0, leaf_steps = 0, leaf_active = 0, open_steps = 0;
  unsigned long long n_pp = 0;
  int32_t p = valid ? 0 : -2;  // this lane's next node in its own walk
  int32_t w = 0;               // the wave's node (uniform)
  // wave steps left before the guard against corrupted links trips, minus
  // one: the loop runs while (w | budget) >= 0 — one scalar OR and compare
  // for both exits (steps = max_steps - 1 - budget afterwards)
  uint32_t leaf_rounds = 0;    // 4-record leaf rounds (cost_kind 1)
  // One path through the body, no `continue`: every exit of a divergent
  // region merges into the same accumulator registers, and p takes one
  // select at the bottom (a body with three early exits to the latch made
  // the register allocator copy the accumulators and counters through
  // phi registers: ~20 v_mov_b64 per wave step, as many VALU issues as the
  // opening test itself).
  const uint32_t max_steps = (uint32_t)wp.max_steps;
  int32_t budget = (int32_t)max_steps - 1;  // (max_steps < 2^31: nodes + 16)
  // theta^2 in a VGPR pair: left a kernel argument, it was reloaded from the
  // kernarg segment every step (a scalar load and its wait; SGPRs are full)
  const uint64_t th2b = __builtin_bit_cast(uint64_t, wp.theta2);
  const double theta2 = __builtin_bit_cast(
      double, ((uint64_t)((uint32_t)(th2b >> 32) | vgpr_zero()) << 32) |
                  (uint64_t)((uint32_t)th2b | vgpr_zero()));
  while ((w | budget) >= 0) {  // corrupted links: stop instead of hanging
    --budget;
    w = __builtin_amdgcn_readfirstlane(w);  // uniform: keep it (and the address math) scalar
    // bit 30 of w: the node is a leaf (walk-record flags; set only below)
    const uint32_t wleaf = ((uint32_t)w >> 30) & 1u;
    w &= 0x3fffffff;
    u32x16 c[NCH];
    load_chunks_node<NCH>(wp.walk + (int64_t)w * RS, c, wleaf);
    const double mass = chunk_d(c[0], 3);
    const int32_t next = chunk_i(c[0], 12), first = chunk_i(c[0], 13);
    const uint32_t wflags = (uint32_t)chunk_i(c[0], 15);
    uint32_t nleaf = wflags & WF_NEXT_LEAF;  // (bit 30: the flag of w below as it is)
    const bool act = (p == w);
    const unsigned na = CNT ? (unsigned)__popcll(__ballot(act)) : 0u;
    if (CNT) n_active += na;  // SIMD efficiency counter
    uint64_t bo = 0ull;  // the lanes that open this node
    // this lane's next node (a leaf: next) — act ? next : p as an unsigned
    // max (see the opening test below: p >= next(w) unless p = w)
    int32_t pn = (int32_t)__builtin_elementwise_max((uint32_t)p, (uint32_t)next);
    int32_t nw = next;
    // tree.rs:1087-1090: empty nodes are skipped — their records say "leaf
    // of no records" (walk_record), so the sign of `first` alone decides.
    // Two independent uniform ifs, not an if / else chain (the chain made a
    // flow block through which the internal path's values were copied)
    if (first >= 0) {
    {  // the test runs on every lane (some lane is always active at w, so an
       // `if (act)` would never skip it; as a branch it doubled the phis)
      const double dx = chunk_d(c[0], 0) - tx, dy = chunk_d(c[0], 1) - ty,
                   dz = chunk_d(c[0], 2) - tz;
      const double dist2 = dist2_tiny<RAW>(dx, dy, dz);  // tree.rs:1117
      bool soft_ok = true;
      if (SOFT && wp.has_hmax) {  // node_soft_ok, tree.rs:56-71
        double h = __builtin_fmax(chunk_d(c[0], 5), 0.0);
        if (has_th) h = __builtin_fmax(h, th);
        if (h > 0.0) {
          const double ch = wp.sep * h;
          soft_ok = dist2 > ch * ch;
        }
      }
      // (the fast unsoftened walk: size2 / theta^2 pre-divided into the
      // record's h_max slot per theta — open_scale — one multiply less per
      // step; it can differ from size2 < theta^2 dist2 only within an ulp)
      const bool accept = act && soft_ok &&
                          ((RAW && !SOFT) ? chunk_d(c[0], 5) < dist2
                                          : chunk_d(c[0], 4) < theta2 * dist2);
      // this lane's next node, and the lanes that open w as the ballot of ONE
      // compare (pn == first holds exactly for the lanes that opened w: a lane
      // not at w cannot have its next node inside w's subtree) — a ballot of
      // the bool `open` is rebuilt from a VGPR copy (v_cndmask + v_cmp)
      // (act ? ... : p as an unsigned max: a lane not at w has its next node
      // past w's subtree, p >= next(w) > first = w + 1, or -1 / -2 (done /
      // no target) — the largest unsigned values; a lane at w has p = w <
      // first.  One v_max with `first` as a scalar operand instead of a
      // select whose two scalar operands both had to be copied to VGPRs)
      pn = accept ? next : (int32_t)__builtin_elementwise_max((uint32_t)p, (uint32_t)first);
      bo = __ballot(pn == first);
      if (LCOST) cost += accept ? 1 : 0;
      if (accept) {
        if constexpr (P == 0) {  // monopole without multipoles (tree.rs:1126-1129, 1284-1291)
          const double y = rsq_walk<RAW>(RAW ? dist2 : dist2 + kR2Tiny);  // (see inv_r)
          if (WANT & PBX_WANT_POT) ph = __builtin_fma(-mass, y, ph);
          if (WANT & PBX_WANT_ACC) {
            const double g = mass * (y * y * y);
            ax = __builtin_fma(g, dx, ax);
            ay = __builtin_fma(g, dy, ay);
            az = __builtin_fma(g, dz, az);
          }
        } else {
          // derivative builders add eps2 = R2_TINY and R2_TINY again
          // (multipole.rs:594, tree.rs:1429); the fast walk's second add is
          // dropped: dist2 (>= R2_TINY) + R2_TINY is dist2 itself unless the
          // node lies within ~1e-146 of the target
          const double inv_r = rsq_walk<RAW>(RAW ? dist2 : dist2 + kR2Tiny);
          if constexpr (P == 1) {  // stored as O0: monopole with the D1 tensor (multipole.rs:272)
            double D[4];
            derivs<1>(dx, dy, dz, inv_r, D);
            if (WANT & PBX_WANT_POT) ph = __builtin_fma(-mass, D[0], ph);
            if (WANT & PBX_WANT_ACC) {
              ax = __builtin_fma(-mass, D[1], ax);
              ay = __builtin_fma(-mass, D[2], ay);
              az = __builtin_fma(-mass, D[3], az);
            }
          } else if constexpr (P == 2 || P == 3) {
            // detraced evaluation (see pack_coef): u = 1/r,
            //   phi = -M u - u^5 q2' + u^7 q3',  q2' = R.Q'.R, q3' = K'(R)
            //   a   = (M u^3 + 5 q2' u^7) R - 2 u^5 Q'.R
            auto C = [&](int i) { return chunk_d(c[1 + (i >> 3)], i & 7); };
            const double u = inv_r, u2 = u * u, u3 = u2 * u, u5 = u3 * u2;
            const double qx = __builtin_fma(C(0), dx, __builtin_fma(C(3), dy, C(4) * dz));
            const double qy = __builtin_fma(C(3), dx, __builtin_fma(C(1), dy, C(5) * dz));
            const double qz = __builtin_fma(C(4), dx, __builtin_fma(C(5), dy, C(2) * dz));
            const double q2 = __builtin_fma(dx, qx, __builtin_fma(dy, qy, dz * qz));
            if (WANT & PBX_WANT_POT) {
              // (the fast walk accumulates the terms into ph one by one: one
              // add less; the precise walk sums the node's terms first, as
              // the reference does)
              double tp = RAW ? __builtin_fma(-u5, q2, __builtin_fma(-mass, u, ph))
                              : __builtin_fma(-u5, q2, -mass * u);
              if constexpr (P == 3) {
                const double zz = dz * dz;
                const double A = __builtin_fma(C(6), dx, __builtin_fma(C(7), dy, C(8) * dz));
                const double B = __builtin_fma(C(9), dy, C(10) * dz);
                const double X = __builtin_fma(dx, A, __builtin_fma(dy, B, C(11) * zz));
                const double G = __builtin_fma(C(12), dy, C(13) * dz);
                const double Y = __builtin_fma(dy, G, C(14) * zz);
                const double q3 = __builtin_fma(dx, X, __builtin_fma(dy, Y, (C(15) * dz) * zz));
                tp = __builtin_fma(u5 * u2, q3, tp);
              }
              ph = RAW ? tp : ph + tp;
            }
            if (WANT & PBX_WANT_ACC) {
              // the order-P force uses moments up to P-1 (multipole.rs:1408-1528):
              // order 2 -> monopole (+ the dipole, zero about the COM)
              double cc = mass * u3, sq = 0.0;
              if constexpr (P == 3) {
                cc = __builtin_fma(5.0 * q2, u5 * u2, cc);
                sq = -2.0 * u5;
              }
              ax = __builtin_fma(cc, dx, __builtin_fma(sq, qx, ax));
              ay = __builtin_fma(cc, dy, __builtin_fma(sq, qy, ay));
              az = __builtin_fma(cc, dz, __builtin_fma(sq, qz, az));
            }
          } else {
            double D[ncoef(P)];
            derivs<P>(dx, dy, dz, inv_r, D);
            eval_multipole<P, WANT>(wp.walk + (int64_t)w * RS + 8, D, ph, ax, ay, az);
          }
        }
      }
    }
    const unsigned no = CNT ? (unsigned)__popcll(bo) : (bo != 0ull ? 1u : 0u);
    if (CNT) {
      n_node += na - no;  // active lanes accept or open
      open_steps += no ? 1u : 0u;
    }
    nw = no ? first : next;
    nleaf = no ? ((wflags & WF_FIRST_LEAF) << 1) : nleaf;
    }
    if (first < 0) {  // leaf: direct sum in ascending index order
      const int32_t s = chunk_i(c[0], 14), e = s + (int32_t)(wflags & WF_COUNT);
      if (CNT) {
        ++leaf_steps;
        leaf_active += na;
        n_pp += (unsigned long long)na * (unsigned long long)(e - s);
      }
      if (CNT || wp.cost_kind) leaf_rounds += (uint32_t)(e - s + 3) >> 2;
      if (act) {
        if (LCOST) cost += e - s;
        // only a target's own leaf needs the self-pair mask (an int compare
        // and four selects per pair): every other leaf takes the plain loop.
        // Per-lane (exec-masked) ifs, not one uniform if / else on the ballot:
        // two alternative loops merged their accumulators through 8 v_mov_b64
        // per leaf step; each lane still runs exactly one loop, in index order
        // (VALU 1.52e10 -> 1.46e10, walk 29.70 -> 29.20 ms, profiles/r6/r7d/)
        const bool own = (uint32_t)(self32 - s) < (uint32_t)(e - s);
        if (!own)
          leaf_sum<WANT, SOFT, RAW, false>(wp, s, e, -1, tx, ty, tz, th, ph, ax, ay, az);
        if (own)
          leaf_sum<WANT, SOFT, RAW, true>(wp, s, e, self32, tx, ty, tz, th, ph, ax, ay, az);
      }
    }
    p = pn;
    // (nleaf is set only for a real node: nw >= 0)
    static_assert(WF_NEXT_LEAF == 0x40000000u && WF_FIRST_LEAF << 1 == WF_NEXT_LEAF, "w's leaf bit");
    w = nw | (int32_t)nleaf;
  }
  const uint32_t steps = (uint32_t)((int32_t)max_steps - 1 - budget);
  if (w >= 0 && lane0) atomicOr(wp.fault, 1u);
  if (wp.trace && lane0) {
    const int64_t wv = (int64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
    wp.trace[3 * wv] = t_start;
    wp.trace[3 * wv + 1] = (unsigned long long)wall_clock64();
    wp.trace[3 * wv + 2] = (unsigned long long)steps;
  }
  if (CNT && wp.counters) {
    if (lane0) {
      atomicAdd(&wp.counters[0], (unsigned long long)n_node);
      atomicAdd(&wp.counters[1], n_pp);
      atomicAdd(&wp.counters[3], (unsigned long long)steps);
      atomicAdd(&wp.counters[4], (unsigned long long)n_active);
      atomicAdd(&wp.counters[5], (unsigned long long)leaf_steps);
      atomicAdd(&wp.counters[6], (unsigned long long)leaf_active);
      atomicAdd(&wp.counters[7], (unsigned long long)open_steps);
    }
  }
  const int32_t wcost = (int32_t)(steps + leaf_rounds);
  if (!valid) return;
  const int64_t o = (self_mode && !wp.compact) ? (int64_t)wp.perm[wp.first + t] : t;
  if (wp.cost) wp.cost[t] = wp.cost_kind ? wcost : cost;
  if (WANT & PBX_WANT_POT) wp.pot[o] = ph;
  if (WANT & PBX_WANT_ACC) {
    wp.acc[3 * o] = ax;
    wp.acc[3 * o + 1] = ay;
    wp.acc[3 * o + 2] = az;
  }
}

__global__ void leaf_particles_kernel(const double4 *__restrict__ rec, const int32_t *__restrict__ perm,
                                      int64_t first, int64_t count, double *__restrict__ pos,
                                      double *__restrict__ mass, int64_t *__restrict__ idx) {
  int64_t t = (int64_t)blockIdx.x * TPB + threadIdx.x;
  if (t >= count) return;
  const double4 r = rec[first + t];
  if (pos) {
    pos[3 * t] = r.x;
    pos[3 * t + 1] = r.y;
    pos[3 * t + 2] = r.z;
  }
  if (mass) mass[t] = r.w;
  if (idx) idx[t] = perm[first + t];
}

// ------------------------------------------ parallel structure (sorted paths)
// The level-synchronous split (split_count / split_make, one host read-back
// per level) rebuilt from the sorted octant paths in a fixed number of
// launches.  With the paths sorted, the particles of any node form one run
// of a common path prefix, and a node at level d exists iff its parent's
// run holds more than leaf_capacity particles (tree.rs:847-864).  For
// particle i let m(i) = the deepest level whose run containing i still has
// > cap particles: some window of cap + 1 consecutive sorted particles
// around i shares that prefix, so m(i) = max over the windows [k, k + cap]
// that contain i of lcp(path k, path k + cap).  i's leaf sits at level
// L(i) = m(i) + 1, and the nodes that START at i are the levels
// fd(i) .. L(i), fd(i) = 1 + lcp(path i - 1, path i) (fd(0) = 0).  Their
// DFS preorder ids are S(i) + d - fd(i) with S the exclusive scan of the
// per-particle node counts (the shallower node of a shared start comes
// first); a stable sort of the nodes by level gives the breadth-first ids
// of split_make (children contiguous, in octant order); every other field
// (range end, subtree size, threaded next, first child, centre replayed
// with the same additions as split_make, parent's child count) follows
// from these.  Inputs the rule cannot decide (a run of > cap particles on
// one full path: identical points, or deeper than the key words) fall back
// to the level-synchronous builder.
constexpr int BP_MAX_LEVEL = 200;

// common leading octant digits of sorted paths a and b (multi-word)
__device__ __forceinline__ int path_lcp(const uint64_t *__restrict__ keys, int64_t n, int nw,
                                        int64_t a, int64_t b) {
  for (int w = 0; w < nw; ++w) {
    const uint64_t x = keys[(int64_t)w * n + a] ^ keys[(int64_t)w * n + b];
    if (x) return w * LPW + (__builtin_clzll(x) - 1) / 3;  // bit 63 is never used
  }
  return nw * LPW;
}

// lcp of every window [k, k + cap] of cap + 1 consecutive sorted paths
// (u8; 255 where the window does not exist) and of each path with its
// predecessor
__global__ void __launch_bounds__(TPB)
    bp_lcp(const uint64_t *__restrict__ keys, int64_t n, int nw, int64_t cap,
           uint8_t *__restrict__ eq, uint8_t *__restrict__ win) {
  const int64_t k = (int64_t)blockIdx.x * TPB + threadIdx.x;
  if (k >= n) return;
  const int e = k ? path_lcp(keys, n, nw, k - 1, k) : 0;
  eq[k] = (uint8_t)(e < 254 ? e : 254);
  int l = 255;
  if (k + cap < n) {
    l = path_lcp(keys, n, nw, k, k + cap);
    l = l < 254 ? l : 254;
  }
  win[k] = (uint8_t)l;
}

// Range ends without path compares.  For sorted paths, path_lcp(i, j) =
// min(eq[i+1 .. j]), so a node's range end is the first j > i with eq[j] < d
// and its parent's start the last q <= i with eq[q] < d - 1.  eq_mins keeps
// the minimum of every 64-byte line of eq (b1) and of every 64 lines (b2);
// a search reads one line per level (eq, b1, b2, b1, eq: five dependent
// 64-byte reads at most, plus a walk over b2 for the few nodes near the
// root) instead of galloping plus bisection over the paths (~2 log2 of the
// range dependent key loads: ~44 for the root at 4M).
constexpr int EQ_LINE = 64;
__global__ void __launch_bounds__(64)
    eq_mins(const uint8_t *__restrict__ eq, int64_t n, uint8_t *__restrict__ b1,
            uint8_t *__restrict__ b2) {
  const int64_t b = (int64_t)blockIdx.x * 64 + threadIdx.x;  // line of eq
  const int64_t nb1 = (n + EQ_LINE - 1) / EQ_LINE;
  uint32_t m = 255;
  if (b < nb1) {
    const int64_t j1 = (b + 1) * EQ_LINE < n ? (b + 1) * EQ_LINE : n;
    for (int64_t j = b * EQ_LINE; j < j1; ++j) m = m < eq[j] ? m : eq[j];
    b1[b] = (uint8_t)m;
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const uint32_t y = (uint32_t)__shfl_xor((int)m, o, 64);
    m = m < y ? m : y;
  }
  if (threadIdx.x == 0) b2[blockIdx.x] = (uint8_t)m;
}

// the bytes of w below t (t <= 128), as their high bits: per byte
// (x | 0x80) - t cannot borrow, and its high bit is clear iff x < t for x < 128
__device__ __forceinline__ uint64_t bytes_lt(uint64_t w, uint64_t tt) {
  constexpr uint64_t H = 0x8080808080808080ull;
  return ~((w | H) - tt) & ~w & H;
}
// byte positions [lo, hi) of word k of a line (0 <= lo, hi <= 64)
__device__ __forceinline__ uint64_t line_word_mask(int k, int lo, int hi) {
  const int a = lo - 8 * k, b = hi - 8 * k;
  const uint64_t up = b >= 8 ? ~0ull : (b <= 0 ? 0ull : (~0ull >> (64 - 8 * b)));
  const uint64_t dn = a <= 0 ? ~0ull : (a >= 8 ? 0ull : (~0ull << (8 * a)));
  return up & dn;
}
// the first (FWD) or last position j in [lo, hi) of the 64-byte line p
// (16-byte aligned) whose byte is < t, or -1
template <bool FWD>
__device__ __forceinline__ int line_find_lt(const uint8_t *__restrict__ p, int lo, int hi,
                                            uint64_t tt) {
  const uint4 *q = (const uint4 *)p;
  uint64_t w[8];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const uint4 v = q[k];
    w[2 * k] = (uint64_t)v.x | ((uint64_t)v.y << 32);
    w[2 * k + 1] = (uint64_t)v.z | ((uint64_t)v.w << 32);
  }
  int r = -1;
#pragma unroll
  for (int kk = 0; kk < 8; ++kk) {
    const int k = FWD ? kk : 7 - kk;
    const uint64_t f = bytes_lt(w[k], tt) & line_word_mask(k, lo, hi);
    if (r < 0 && f)
      r = 8 * k + (FWD ? __builtin_ctzll(f) : 63 - __builtin_clzll(f)) / 8;
  }
  return r;
}
// first j in [j0, n) with eq[j] < t (t <= 128), or n
__device__ int64_t eq_next_lt(const uint8_t *__restrict__ eq, const uint8_t *__restrict__ b1,
                              const uint8_t *__restrict__ b2, int64_t n, int64_t j0, int t) {
  if (j0 >= n) return n;
  const uint64_t tt = 0x0101010101010101ull * (uint64_t)t;
  const int64_t nb1 = (n + EQ_LINE - 1) / EQ_LINE, nb2 = (nb1 + EQ_LINE - 1) / EQ_LINE;
  auto lim = [](int64_t a, int64_t base) { return (int)(a - base < EQ_LINE ? a - base : EQ_LINE); };
  int64_t b = j0 / EQ_LINE;
  int r = line_find_lt<true>(eq + EQ_LINE * b, (int)(j0 - EQ_LINE * b), lim(n, EQ_LINE * b), tt);
  if (r >= 0) return EQ_LINE * b + r;
  int64_t c = b / EQ_LINE;  // the later lines of b's group of 64
  r = line_find_lt<true>(b1 + EQ_LINE * c, (int)(b + 1 - EQ_LINE * c), lim(nb1, EQ_LINE * c), tt);
  if (r < 0) {  // the later groups
    int64_t g = c + 1, found = -1;
    while (g < nb2) {
      const int64_t L = g / EQ_LINE;
      const int rr = line_find_lt<true>(b2 + EQ_LINE * L, (int)(g - EQ_LINE * L), lim(nb2, EQ_LINE * L), tt);
      if (rr >= 0) {
        found = EQ_LINE * L + rr;
        break;
      }
      g = EQ_LINE * (L + 1);
    }
    if (found < 0) return n;
    c = found;
    r = line_find_lt<true>(b1 + EQ_LINE * c, 0, lim(nb1, EQ_LINE * c), tt);
  }
  b = EQ_LINE * c + r;
  return EQ_LINE * b + line_find_lt<true>(eq + EQ_LINE * b, 0, lim(n, EQ_LINE * b), tt);
}
// last q in [0, i] with eq[q] < t (t <= 128), or -1
__device__ int64_t eq_prev_lt(const uint8_t *__restrict__ eq, const uint8_t *__restrict__ b1,
                              const uint8_t *__restrict__ b2, int64_t n, int64_t i, int t) {
  if (i < 0) return -1;
  const uint64_t tt = 0x0101010101010101ull * (uint64_t)t;
  const int64_t nb1 = (n + EQ_LINE - 1) / EQ_LINE;
  auto lim = [](int64_t a, int64_t base) { return (int)(a - base < EQ_LINE ? a - base : EQ_LINE); };
  int64_t b = i / EQ_LINE;
  int r = line_find_lt<false>(eq + EQ_LINE * b, 0, (int)(i - EQ_LINE * b + 1), tt);
  if (r >= 0) return EQ_LINE * b + r;
  int64_t c = b / EQ_LINE;  // the earlier lines of b's group
  r = line_find_lt<false>(b1 + EQ_LINE * c, 0, (int)(b - EQ_LINE * c), tt);
  if (r < 0) {  // the earlier groups
    int64_t g = c - 1, found = -1;
    while (g >= 0) {
      const int64_t L = g / EQ_LINE;
      const int rr = line_find_lt<false>(b2 + EQ_LINE * L, 0, (int)(g - EQ_LINE * L + 1), tt);
      if (rr >= 0) {
        found = EQ_LINE * L + rr;
        break;
      }
      g = EQ_LINE * L - 1;
    }
    if (found < 0) return -1;
    c = found;
    r = line_find_lt<false>(b1 + EQ_LINE * c, 0, lim(nb1, EQ_LINE * c), tt);
  }
  b = EQ_LINE * c + r;
  return EQ_LINE * b + line_find_lt<false>(eq + EQ_LINE * b, 0, lim(n, EQ_LINE * b), tt);
}

// fd(i), L(i) and the node count of every sorted position; level
// histogram (LDS per block, one global add per level and block: the grid
// is bounded, so those adds stay few — every block adds to the same words)
constexpr int BP_DEPTH_BLOCKS = 1024;
__global__ void __launch_bounds__(TPB)
    bp_depth(const uint8_t *__restrict__ eq, const uint8_t *__restrict__ win, int64_t n, int D,
             int64_t cap, uint8_t *__restrict__ fd, uint8_t *__restrict__ lv,
             uint32_t *__restrict__ cnt, unsigned int *__restrict__ flag) {
  __shared__ unsigned int h[BP_MAX_LEVEL + 1], hin[BP_MAX_LEVEL + 1];
  __shared__ uint8_t sw[TPB + 64];  // the windows [i - cap, i] of the chunk, cap <= 64
  for (int d = threadIdx.x; d <= BP_MAX_LEVEL; d += TPB) h[d] = hin[d] = 0u;
  bool over = false;
  for (int64_t base = (int64_t)blockIdx.x * TPB; base < n; base += (int64_t)gridDim.x * TPB) {
    __syncthreads();  // the previous chunk's windows are read
    for (int j = threadIdx.x; j < TPB + cap; j += TPB) {
      const int64_t k = base - cap + j;
      sw[j] = (k >= 0 && k < n) ? win[k] : (uint8_t)255;
    }
    __syncthreads();
    const int64_t i = base + threadIdx.x;
    const bool ok = i < n;
    int f = 1, L = 0;
    if (ok) {  // D: levels whose prefix runs are contiguous (sorted)
      f = i ? eq[i] + 1 : 0;
      f = f < 255 ? f : 255;
      int m = -1;
      for (int j = 0; j <= cap; ++j) {
        const int l = sw[threadIdx.x + j];
        if (l != 255) m = l > m ? l : m;
      }
      over |= (m >= D || m + 1 > BP_MAX_LEVEL);  // undecidable: fall back
      L = m + 1 < BP_MAX_LEVEL ? m + 1 : BP_MAX_LEVEL;
      fd[i] = (uint8_t)f;
      lv[i] = (uint8_t)L;
      cnt[i] = (uint32_t)(L >= f ? L - f + 1 : 0);
    }
    // nodes per level and of them internal ones (all but the deepest node
    // starting at i): ballots per level and wave, over the levels at which
    // some lane of the wave starts a node (sorted paths: most start only
    // their leaf, so [wave min f, wave max L] is a few levels, not 0 .. L)
    int dmax = ok ? L : -1;
    int dmin = (ok && f <= L) ? f : BP_MAX_LEVEL + 1;
    for (int o = 32; o > 0; o >>= 1) {
      const int y = __shfl_xor(dmax, o, 64);
      dmax = y > dmax ? y : dmax;
      const int z = __shfl_xor(dmin, o, 64);
      dmin = z < dmin ? z : dmin;
    }
    for (int d = dmin; d <= dmax; ++d) {
      const uint32_t c = (uint32_t)__popcll(__ballot(ok && f <= d && d <= L));
      const uint32_t ci = (uint32_t)__popcll(__ballot(ok && f <= d && d < L));
      if ((threadIdx.x & 63) == 0 && c) atomicAdd(&h[d], c);
      if ((threadIdx.x & 63) == 0 && ci) atomicAdd(&hin[d], ci);
    }
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) cnt[n] = 0u;  // scan sentinel: S[n] = nodes
  if (__ballot(over) && (threadIdx.x & 63) == 0) atomicOr(flag, 1u);
  __syncthreads();
  for (int d = threadIdx.x; d <= BP_MAX_LEVEL; d += TPB) {
    if (h[d]) atomicAdd(&flag[1 + d], h[d]);
    if (hin[d]) atomicAdd(&flag[2 + BP_MAX_LEVEL + d], hin[d]);
  }
}

// every node in preorder: its level and start
__global__ void __launch_bounds__(TPB)
    bp_nodes_pre(const uint8_t *__restrict__ fd, const uint8_t *__restrict__ lv,
                 const uint32_t *__restrict__ S, int64_t n, uint32_t *__restrict__ level,
                 int32_t *__restrict__ start) {
  const int64_t i = (int64_t)blockIdx.x * TPB + threadIdx.x;
  if (i >= n) return;
  const int f = fd[i], L = lv[i];
  uint32_t pre = S[i];
  for (int d = f; d <= L; ++d, ++pre) {
    level[pre] = (uint32_t)d;
    start[pre] = (int32_t)i;
  }
}

__global__ void bp_inverse(const int32_t *__restrict__ b2p, int64_t nn, int32_t *__restrict__ p2b) {
  const int64_t k = (int64_t)blockIdx.x * TPB + threadIdx.x;
  if (k < nn) p2b[b2p[k]] = (int32_t)k;
}

// every node: range, centre, links, subtree size (in its breadth-first
// slot); its parent's child count
__global__ void __launch_bounds__(TPB)
    bp_nodes_bfs(const uint64_t *__restrict__ keys, int64_t n, int nw, const uint8_t *__restrict__ eq,
                 const uint8_t *__restrict__ eb1, const uint8_t *__restrict__ eb2,
                 const uint8_t *__restrict__ fd,
                 const uint8_t *__restrict__ lv, const uint32_t *__restrict__ S,
                 const uint32_t *__restrict__ level, const int32_t *__restrict__ start,
                 const int32_t *__restrict__ b2p, const int32_t *__restrict__ p2b, int64_t nn,
                 double4 root, BuildView v, int32_t *__restrict__ size) {
#pragma clang fp contract(off)
  // threads take the nodes in breadth-first order, so the six per-node
  // outputs are coalesced stores (in preorder they were scattered 4-byte
  // writes, a cache line each); a level's nodes are in preorder order, so
  // their start / level / path reads stay close together
  const int64_t k = (int64_t)blockIdx.x * TPB + threadIdx.x;
  if (k >= nn) return;
  const int32_t pre = b2p[k];
  const int64_t i = start[pre];
  const int d = (int)level[pre];
  const int f = fd[i];
  // range end: the first later path whose level-d prefix differs (eq of
  // that path < d): the next 16 eq bytes first (leaves and the levels
  // above them), then galloping over the paths
  int64_t lo = i + 1, hi = n;
  {
    uint8_t e[16];
#pragma unroll
    for (int q = 0; q < 16; ++q) e[q] = (i + 1 + q < n) ? eq[i + 1 + q] : (uint8_t)0;
    int q0 = 16;
#pragma unroll
    for (int q = 15; q >= 0; --q)
      if ((int)e[q] < d) q0 = q;
    if (q0 < 16 || i + 17 >= n) hi = lo = (i + 1 + q0 < n) ? i + 1 + q0 : n;
    else lo = i + 17;
  }
  if (lo < hi && eb1 && d <= 128) {  // the first eq < d at or after lo (eq_next_lt)
    lo = hi = eq_next_lt(eq, eb1, eb2, n, lo, d);
  }
  for (int64_t step = 1; lo < hi;) {
    const int64_t probe = lo + step - 1 < hi ? lo + step - 1 : hi - 1;
    if (path_lcp(keys, n, nw, i, probe) >= d) {
      lo = probe + 1;
      step <<= 1;
    } else {
      hi = probe;
      break;
    }
  }
  while (lo < hi) {
    const int64_t mid = (lo + hi) >> 1;
    if (path_lcp(keys, n, nw, i, mid) >= d) lo = mid + 1;
    else hi = mid;
  }
  const int64_t end = lo;
  const int32_t sz = (int32_t)((S[end] - S[i]) - (uint32_t)(d - f));
  v.nstart[k] = (int32_t)i;
  v.ncount[k] = (int32_t)(end - i);
  v.nfirst[k] = (d == (int)lv[i]) ? -1 : p2b[pre + 1];
  v.nnext[k] = (pre + sz < nn) ? p2b[pre + sz] : -1;
  size[k] = sz;
  // centre: the path's digits from the root, split_make's additions
  double cx = root.x, cy = root.y, cz = root.z, h = root.w;
  uint64_t word = 0;
  for (int l = 0; l < d; ++l) {
    if (l % LPW == 0) word = keys[(int64_t)(l / LPW) * n + i];
    const uint32_t o = (uint32_t)(word >> (3 * (LPW - 1 - l % LPW))) & 7u;
    const double off = h / 2.0;
    cx = cx + ((o & 1u) ? off : -off);
    cy = cy + ((o & 2u) ? off : -off);
    cz = cz + ((o & 4u) ? off : -off);
    h = off;
  }
  v.ncen[k] = make_double4(cx, cy, cz, h);
  if (d > 0) {
    int32_t ppre;
    if (f <= d - 1) {
      ppre = pre - 1;  // the parent starts at i too
    } else {  // the parent's start: the first path sharing the level-(d-1) prefix
      int64_t a = 0, b = i;
      {  // the 16 eq bytes up to i first: b = the last p <= i with eq(p) < d - 1
        uint8_t e[16];
#pragma unroll
        for (int q = 0; q < 16; ++q) e[q] = (i - q > 0) ? eq[i - q] : (uint8_t)0;
        int q0 = 16;
#pragma unroll
        for (int q = 15; q >= 0; --q)
          if ((int)e[q] < d - 1) q0 = q;
        if (q0 < 16) a = b = (i - q0 > 0) ? i - q0 : 0;
        else b = i - 16;
      }
      if (a < b && eb1 && d - 1 <= 128) {  // the last eq < d - 1 at or before b (eq_prev_lt)
        const int64_t q = eq_prev_lt(eq, eb1, eb2, n, b, d - 1);
        a = b = q > 0 ? q : 0;
      }
      for (int64_t step = 1; a < b;) {  // galloping back
        const int64_t probe = b - step > a ? b - step : a;
        if (path_lcp(keys, n, nw, probe, i) >= d - 1) {
          b = probe;
          step <<= 1;
        } else {
          a = probe + 1;
          break;
        }
      }
      while (a < b) {
        const int64_t mid = (a + b) >> 1;
        if (path_lcp(keys, n, nw, mid, i) >= d - 1) b = mid;
        else a = mid + 1;
      }
      ppre = (int32_t)(S[a] + (uint32_t)(d - 1 - fd[a]));
    }
    atomicAdd(&v.nchild[p2b[ppre]], 1);
  }
}

// ------------------------------------------------- cost-balanced target ranges
// Multi-GPU walks split the leaf-ordered targets into contiguous ranges of
// about equal cost (interactions per target).  The costs of one walk are
// carried to the next step in ORIGINAL particle order (the leaf order of the
// next build may differ), so no extra walk is needed to balance a step.
constexpr int BAL_TPB = 1024;
constexpr int BAL_PER = 4;
constexpr int BAL_CHUNK = BAL_TPB * BAL_PER;  // targets per block-sum entry

__global__ void cost_to_orig(const int32_t *__restrict__ cost_leaf, const int32_t *__restrict__ perm,
                             int64_t n, int32_t *__restrict__ cost_orig) {
  int64_t i = (int64_t)blockIdx.x * TPB + threadIdx.x;
  if (i < n) cost_orig[perm[i]] = cost_leaf[i];
}

__device__ __forceinline__ int64_t bal_cost(const int32_t *cost_orig, const int32_t *perm, int64_t i,
                                            int64_t n) {
  // balanced_ranges (parallel.py) counts every target as at least 1
  return i < n ? (int64_t)max(cost_orig[perm[i]], 1) : 0;
}

// per chunk of BAL_CHUNK leaf positions: sum of max(cost, 1)
__global__ __launch_bounds__(BAL_TPB) void bal_chunk_sums(const int32_t *__restrict__ cost_orig,
                                                          const int32_t *__restrict__ perm, int64_t n,
                                                          int64_t *__restrict__ sums) {
  __shared__ int64_t part[BAL_TPB / 64];
  const int64_t base = (int64_t)blockIdx.x * BAL_CHUNK;
  int64_t s = 0;
#pragma unroll
  for (int k = 0; k < BAL_PER; ++k) s += bal_cost(cost_orig, perm, base + k * BAL_TPB + threadIdx.x, n);
  for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o);
  if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) {
    int64_t t = 0;
    for (int w = 0; w < BAL_TPB / 64; ++w) t += part[w];
    sums[blockIdx.x] = t;
  }
}

// inclusive block scan of one int64 per thread (BAL_TPB threads)
__device__ int64_t bal_block_scan(int64_t v, int64_t *lds, int64_t *total) {
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  for (int o = 1; o < 64; o <<= 1) {
    int64_t u = __shfl_up(v, o);
    if (lane >= o) v += u;
  }
  if (lane == 63) lds[wv] = v;
  __syncthreads();
  if (threadIdx.x == 0) {
    int64_t run = 0;
    for (int w = 0; w < BAL_TPB / 64; ++w) {
      const int64_t x = lds[w];
      lds[w] = run;
      run += x;
    }
    lds[BAL_TPB / 64] = run;
  }
  __syncthreads();
  v += lds[wv];
  *total = lds[BAL_TPB / 64];
  __syncthreads();
  return v;
}

// One block: cuts[r] = 1 + first leaf position whose inclusive cost prefix
// reaches total * r / world (the same float comparison as balanced_ranges:
// searchsorted(cum, total * r / world, 'left') + 1), made monotone, <= n.
__global__ __launch_bounds__(BAL_TPB) void bal_cuts(const int32_t *__restrict__ cost_orig,
                                                    const int32_t *__restrict__ perm, int64_t n,
                                                    const int64_t *__restrict__ sums, int64_t nchunks,
                                                    int world, int64_t *__restrict__ cuts) {
  __shared__ int64_t lds[BAL_TPB / 64 + 1];
  __shared__ int64_t found;
  // pass 1: the grand total
  int64_t total = 0;
  for (int64_t b0 = 0; b0 < nchunks; b0 += BAL_TPB) {
    int64_t t;
    bal_block_scan(b0 + threadIdx.x < nchunks ? sums[b0 + threadIdx.x] : 0, lds, &t);
    total += t;
  }
  int64_t prev = 0;
  if (threadIdx.x == 0) cuts[0] = 0;
  for (int r = 1; r < world; ++r) {
    const double target = (double)total * (double)r / (double)world;
    // the chunk holding the crossing: scan the chunk sums again
    if (threadIdx.x == 0) found = -1;
    __syncthreads();
    int64_t run = 0, chunk = -1, before = 0;
    for (int64_t b0 = 0; b0 < nchunks; b0 += BAL_TPB) {
      const int64_t b = b0 + threadIdx.x;
      const int64_t v = b < nchunks ? sums[b] : 0;
      int64_t t;
      const int64_t inc = run + bal_block_scan(v, lds, &t);
      if (b < nchunks && (double)inc >= target && (double)(inc - v) < target) found = b;
      __syncthreads();
      if (found >= 0) {
        chunk = found;
        break;
      }
      run += t;
    }
    int64_t cut = n;  // target beyond the total (rounding): everything
    if (chunk >= 0) {
      // prefix before the chunk
      for (int64_t b0 = 0; b0 < chunk; b0 += BAL_TPB) {
        const int64_t b = b0 + threadIdx.x;
        int64_t t;
        bal_block_scan(b < chunk ? sums[b] : 0, lds, &t);
        before += t;
      }
      // inside the chunk: BAL_PER consecutive leaf positions per thread
      const int64_t base = chunk * BAL_CHUNK + (int64_t)threadIdx.x * BAL_PER;
      int64_t c[BAL_PER], s = 0;
#pragma unroll
      for (int k = 0; k < BAL_PER; ++k) {
        c[k] = bal_cost(cost_orig, perm, base + k, n);
        s += c[k];
      }
      int64_t t;
      int64_t inc = before + bal_block_scan(s, lds, &t) - s;
      if (threadIdx.x == 0) found = -1;
      __syncthreads();
      int64_t mine = -1;
#pragma unroll
      for (int k = 0; k < BAL_PER; ++k) {
        inc += c[k];
        if (mine < 0 && base + k < n && (double)inc >= target) mine = base + k;
      }
      if (mine >= 0) atomicMin((unsigned long long *)&found, (unsigned long long)mine);
      __syncthreads();
      if (found >= 0 && found != -1) cut = found + 1;
    }
    cut = cut < prev ? prev : (cut > n ? n : cut);
    prev = cut;
    if (threadIdx.x == 0) cuts[r] = cut;
    __syncthreads();
  }
  if (threadIdx.x == 0) cuts[world] = n;
}

// ------------------------------------------------------------------- host
struct Octree {
  int device = -1;
  int64_t n = 0;
  int64_t leaf_capacity = 32;
  int order = 0;   // multipole_order as given
  int kernel = 0;  // 0 Plummer, 1 spline
  bool user_mass = false;
  bool soft_set = false;
  bool has_bh = false;
  bool has_hmax = false;
  // theta^2 the walk records' h_max slot holds size2 / theta^2 for (the
  // fast unsoftened walks' opening test; -1: not scaled since the payload)
  double open_theta2 = -1.0;
  int nwords = 1;
  double root[4] = {0, 0, 0, 0};
  int64_t nn = 0, cap = 0;
  std::vector<int32_t> lvl;  // first node id of every level (+ end)
  std::vector<int32_t> lvl_int;  // internal nodes per level (parallel build; else empty)
  Buf pos, mass, soft;       // original order (device copies)
  Buf perm, rec, soft_s;     // leaf order
  Buf trace;                 // PBX_WALK_TRACE diagnostic
  Buf nstart, ncount, nfirst, nnext, nchild, ncen, pre, size;
  Buf com, hmax, mom, coef, walk, leaf_dfs;
  Buf keys, ktmp0, ktmp1, vtmp, hist, tsum, front0, front1, lb, cnt, flags, small, counters;
  Buf bal;                   // cost-balanced ranges: chunk sums + cuts
  Buf iscan, ilist, iws;     // payload: internal-node flags / scan, list, scan state
  int cost_kind = 0;                   // d_cost contents (WalkParams::cost_kind)
  bool walk_counts = true;             // pbx_octree_set_walk_counters
  Buf bp_fl, bp_eq, bp_s, bp_ctl, bp_level, bp_start, bp_p2b;  // parallel structure build
  Buf bp_emin;  // eq's line / group minima (eq_mins)
  Buf rec0;                  // {x, y, z, m} in original order (path_keys)
  bool rec0_valid = false;   // rec0 holds the current masses
  prim::HostBuf rm_pin;      // radial_moments readback staging
  ~Octree() {
    Buf *bufs[] = {&pos, &mass, &soft, &perm, &rec, &soft_s, &nstart, &ncount, &nfirst, &nnext,
                   &nchild, &ncen, &pre, &size, &com, &hmax, &mom, &coef, &walk, &leaf_dfs, &keys, &ktmp0,
                   &ktmp1, &vtmp, &hist, &tsum, &front0, &front1, &lb, &cnt, &flags, &small,
                   &counters, &trace, &bal, &iscan, &ilist, &iws, &bp_fl, &bp_eq, &bp_emin, &bp_s, &rec0, &bp_ctl, &bp_level, &bp_start,
                   &bp_p2b};
    for (Buf *b : bufs) b->release();
    rm_pin.release();
  }
  // accepted nodes, leaf pairs, fault flag, wave steps, active-lane steps
  // + leaf wave steps, their active lanes, descending wave steps
  unsigned long long last_counts[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  int moment_order() const { return order < 5 ? order : 5; }
};

static inline unsigned nblk(int64_t n) { return (unsigned)((n + TPB - 1) / TPB); }

// grow a node array to `ncap` elements of `esize` bytes keeping `keep` elements
static void grow_keep(Buf &b, size_t esize, int64_t ncap, int64_t keep, hipStream_t st) {
  size_t need = esize * (size_t)ncap;
  if (need <= b.bytes) return;
  size_t got = 0;
  int dev = 0;
  void *np = dev_alloc(need, &got, &dev);
  if (keep > 0 && b.p) PBX_HIP(hipMemcpyAsync(np, b.p, esize * (size_t)keep, hipMemcpyDeviceToDevice, st));
  b.release();  // (the copy is queued before any later owner's work on st)
  b.p = np;
  b.bytes = got;
  b.dev = dev;
}

static void ensure_nodes(Octree &T, int64_t need, hipStream_t st) {
  if (need <= T.cap) return;
  int64_t c = std::max<int64_t>(need, T.cap * 2);
  grow_keep(T.nstart, 4, c, T.nn, st);
  grow_keep(T.ncount, 4, c, T.nn, st);
  grow_keep(T.nfirst, 4, c, T.nn, st);
  grow_keep(T.nnext, 4, c, T.nn, st);
  grow_keep(T.nchild, 4, c, T.nn, st);
  grow_keep(T.ncen, sizeof(double4), c, T.nn, st);
  T.cap = c;
}

static uint32_t read_u32(const void *dptr, hipStream_t st) {
  uint32_t v = 0;
  PBX_HIP(hipMemcpyAsync(&v, dptr, 4, hipMemcpyDeviceToHost, st));
  PBX_HIP(hipStreamSynchronize(st));
  return v;
}

// sort perm by the multi-word paths (LSD over words, last word first).
// min_shift > 0 (one path word): only the bytes from bit min_shift up are
// sorted, with no read-back of the varying bits — the runs of a common
// prefix are then contiguous down to level (62 - min_shift) / 3 only,
// which split_parallel checks (levels deeper than that need the full sort).
static void sort_paths(Octree &T, hipStream_t st, int min_shift = 0) {
  const int64_t n = T.n;
  uint64_t *keys = T.keys.as<uint64_t>();
  uint64_t *k0 = (uint64_t *)T.ktmp0.get(8 * (size_t)n);
  uint64_t *k1 = (uint64_t *)T.ktmp1.get(8 * (size_t)n);
  int32_t *v0 = T.perm.as<int32_t>();
  int32_t *v1 = (int32_t *)T.vtmp.get(4 * (size_t)n);
  unsigned long long *oa = (unsigned long long *)T.small.get(64);
  bool have_perm = false;
  const bool partial = min_shift > 0 && T.nwords == 1;
  for (int w = T.nwords - 1; w >= 0; --w) {
    uint64_t vary = ~0ull;
    if (!partial) {  // bits that vary across all paths of this word
      unsigned long long h[2] = {0ull, ~0ull};
      PBX_HIP(hipMemcpyAsync(oa, h, 16, hipMemcpyHostToDevice, st));
      hipLaunchKernelGGL(key_or_and, dim3(std::min<unsigned>(1024, nblk(n))), dim3(TPB), 0, st,
                         keys + (int64_t)w * n, n, oa);
      PBX_HIP(hipMemcpyAsync(h, oa, 16, hipMemcpyDeviceToHost, st));
      PBX_HIP(hipStreamSynchronize(st));
      vary = h[0] ^ h[1];
      if (!vary) continue;
    }
    hipLaunchKernelGGL(gather_u64, dim3(nblk(n)), dim3(TPB), 0, st, keys + (int64_t)w * n,
                       have_perm ? v0 : (const int32_t *)nullptr, n, k0);
    for (int shift = partial ? min_shift : 0; shift < 64; shift += 8) {
      if (!((vary >> shift) & 0xffull)) continue;
      radix_pass<uint64_t>(T.hist, T.tsum, st, k0, v0, have_perm ? VAL_ARRAY : VAL_IOTA, n,
                           shift, k1, v1);
      std::swap(k0, k1);
      std::swap(v0, v1);
      have_perm = true;
    }
  }
  if (!have_perm) {  // every path equal: identity order
    std::vector<int32_t> iota(n);
    for (int64_t i = 0; i < n; ++i) iota[i] = (int32_t)i;
    PBX_HIP(hipMemcpyAsync(v0, iota.data(), 4 * (size_t)n, hipMemcpyHostToDevice, st));
    PBX_HIP(hipStreamSynchronize(st));
  }
  if (v0 != T.perm.as<int32_t>()) {
    // result landed in the scratch buffer: swap the allocations
    std::swap(T.perm, T.vtmp);
  }
  // sorted paths (structure pass reads them in leaf order): one word that
  // went through a pass is sorted already in k0
  if (T.nwords == 1 && have_perm) {
    Buf &b = (k0 == T.ktmp0.as<uint64_t>()) ? T.ktmp0 : T.ktmp1;
    std::swap(T.keys, b);
    return;
  }
  uint64_t *sorted = (uint64_t *)T.ktmp1.get(8 * (size_t)n * T.nwords);
  for (int w = 0; w < T.nwords; ++w)
    hipLaunchKernelGGL(gather_u64, dim3(nblk(n)), dim3(TPB), 0, st, keys + (int64_t)w * n,
                       T.perm.as<int32_t>(), n, sorted + (int64_t)w * n);
  PBX_HIP(hipGetLastError());
  std::swap(T.keys, T.ktmp1);
}

// The whole structure from the sorted paths (bp_* kernels), one host
// read-back; also the DFS preorder ids and subtree sizes (T.pre, T.size).
// Returns false where the rule cannot decide (see bp_depth) or the leaf
// capacity makes the windows long: the level-synchronous split then runs.
static bool split_parallel(Octree &T, hipStream_t st, int sorted_levels) {
  const int64_t n = T.n;
  if (n <= 0 || T.leaf_capacity > 64 || !(T.root[3] > 1e-290) || n >= ((int64_t)1 << 31) - 1)
    return false;
  const uint64_t *keys = T.keys.as<uint64_t>();
  uint8_t *fd = (uint8_t *)T.bp_fl.get(2 * (size_t)n + 16);
  uint8_t *lv = fd + n;
  uint32_t *S = (uint32_t *)T.bp_s.get(4 * (size_t)(n + 1));
  // [undecidable flag][nodes per level][internal nodes per level][nodes]
  const size_t nctl = 3 + 2 * (size_t)BP_MAX_LEVEL + 1;
  unsigned int *ctl = (unsigned int *)T.bp_ctl.get(4 * nctl);
  PBX_HIP(hipMemsetAsync(ctl, 0, 4 * nctl, st));
  // (+128: eq_next_lt / eq_prev_lt read eq's last line whole)
  uint8_t *eq = (uint8_t *)T.bp_eq.get(2 * (size_t)n + 128), *win = eq + n;
  hipLaunchKernelGGL(bp_lcp, dim3(nblk(n)), dim3(TPB), 0, st, keys, n, T.nwords, T.leaf_capacity,
                     eq, win);
  hipLaunchKernelGGL(bp_depth, dim3(std::min<unsigned>(BP_DEPTH_BLOCKS, nblk(n))), dim3(TPB), 0,
                     st, (const uint8_t *)eq,
                     (const uint8_t *)win, n, sorted_levels, T.leaf_capacity, fd, lv, S, ctl);
  scan_u32(T.tsum, st, S, n + 1);
  PBX_HIP(hipMemcpyAsync(ctl + (nctl - 1), S + n, 4, hipMemcpyDeviceToDevice, st));  // nn
  std::vector<unsigned int> h(nctl);
  unsigned long long wd = 0;  // the scan's look-back watchdog (prims.h), read in the same batch
  PBX_HIP(hipMemcpyAsync(h.data(), ctl, 4 * nctl, hipMemcpyDeviceToHost, st));
  PBX_HIP(hipMemcpyAsync(&wd, prim::scan_watchdog(T.tsum), sizeof(wd), hipMemcpyDeviceToHost, st));
  PBX_HIP(hipStreamSynchronize(st));
  if (wd) {
    PBX_HIP(hipMemsetAsync(prim::scan_watchdog(T.tsum), 0, sizeof(wd), st));
    fail(PBX_ERR_RUNTIME, "a device scan of the octree build did not complete (look-back watchdog)");
  }
  if (h[0]) return false;
  const int64_t nn = h[nctl - 1];
  // levels: nodes per level -> breadth-first id ranges
  T.lvl.assign(1, 0);
  T.lvl_int.clear();
  int64_t tot = 0;
  for (int d = 0; d <= BP_MAX_LEVEL && tot < nn; ++d) {
    tot += h[1 + d];
    T.lvl.push_back((int32_t)tot);
    T.lvl_int.push_back((int32_t)h[2 + BP_MAX_LEVEL + d]);
  }
  if (tot != nn || nn < 1) fail(PBX_ERR_RUNTIME, "parallel octree build: %lld nodes by level, %lld in all",
                                (long long)tot, (long long)nn);
  T.nn = 0;
  ensure_nodes(T, nn, st);
  uint32_t *level = (uint32_t *)T.bp_level.get(4 * (size_t)nn);
  int32_t *startp = (int32_t *)T.bp_start.get(4 * (size_t)nn);
  hipLaunchKernelGGL(bp_nodes_pre, dim3(nblk(n)), dim3(TPB), 0, st, (const uint8_t *)fd,
                     (const uint8_t *)lv, (const uint32_t *)S, n, level, startp);
  // breadth-first order = preorder stably sorted by level
  int32_t *b2p = (int32_t *)T.pre.get(4 * (size_t)nn);
  radix_pass<uint32_t>(T.hist, T.tsum, st, level, nullptr, VAL_IOTA, nn, 0, nullptr, b2p);
  int32_t *p2b = (int32_t *)T.bp_p2b.get(4 * (size_t)nn);
  hipLaunchKernelGGL(bp_inverse, dim3(nblk(nn)), dim3(TPB), 0, st, (const int32_t *)b2p, nn, p2b);
  PBX_HIP(hipMemsetAsync(T.nchild.p, 0, 4 * (size_t)nn, st));
  BuildView v;
  v.keys = keys;
  v.perm = T.perm.as<int32_t>();
  v.pos = T.pos.as<double>();
  v.n = n;
  v.nwords = T.nwords;
  v.cap = T.leaf_capacity;
  v.nstart = T.nstart.as<int32_t>();
  v.ncount = T.ncount.as<int32_t>();
  v.nfirst = T.nfirst.as<int32_t>();
  v.nnext = T.nnext.as<int32_t>();
  v.nchild = T.nchild.as<int32_t>();
  v.ncen = T.ncen.as<double4>();
  int32_t *size = (int32_t *)T.size.get(4 * (size_t)nn);
  const int64_t nb1 = (n + EQ_LINE - 1) / EQ_LINE, nb2 = (nb1 + EQ_LINE - 1) / EQ_LINE;
  const size_t l1 = (size_t)nb2 * EQ_LINE, l2 = ((size_t)nb2 + EQ_LINE - 1) / EQ_LINE * EQ_LINE;
  uint8_t *eb1 = (uint8_t *)T.bp_emin.get(l1 + l2 + 64), *eb2 = eb1 + l1;
  hipLaunchKernelGGL(eq_mins, dim3((unsigned)nb2), dim3(64), 0, st, (const uint8_t *)eq, n, eb1, eb2);
  hipLaunchKernelGGL(bp_nodes_bfs, dim3(nblk(nn)), dim3(TPB), 0, st, keys, n, T.nwords,
                     (const uint8_t *)eq, (const uint8_t *)eb1, (const uint8_t *)eb2, (const uint8_t *)fd, (const uint8_t *)lv, (const uint32_t *)S,
                     (const uint32_t *)level, (const int32_t *)startp, (const int32_t *)b2p,
                     (const int32_t *)p2b, nn,
                     make_double4(T.root[0], T.root[1], T.root[2], T.root[3]), v, size);
  PBX_HIP(hipGetLastError());
  T.nn = nn;
  return true;
}

// levels of the tree; returns false when the paths are too short
static bool split_levels(Octree &T, hipStream_t st) {
  const int64_t n = T.n;
  T.nn = 0;
  ensure_nodes(T, std::max<int64_t>(64, n / 2 + 64), st);
  BuildView v;
  v.keys = T.keys.as<uint64_t>();
  v.perm = T.perm.as<int32_t>();
  v.pos = T.pos.as<double>();
  v.n = n;
  v.nwords = T.nwords;
  v.cap = T.leaf_capacity;
  auto bind = [&] {
    v.nstart = T.nstart.as<int32_t>();
    v.ncount = T.ncount.as<int32_t>();
    v.nfirst = T.nfirst.as<int32_t>();
    v.nnext = T.nnext.as<int32_t>();
    v.nchild = T.nchild.as<int32_t>();
    v.ncen = T.ncen.as<double4>();
  };
  bind();
  int32_t *fr = (int32_t *)T.front0.get(4 * 64);
  uint32_t *sm = (uint32_t *)T.small.get(64);
  hipLaunchKernelGGL(root_init, dim3(1), dim3(1), 0, st, v, T.root[0], T.root[1], T.root[2],
                     T.root[3], fr, sm);
  int64_t F = read_u32(sm, st);
  T.nn = 1;
  T.lvl.assign({0, 1});
  T.lvl_int.clear();
  int d = 0;
  while (F > 0) {
    if (d >= LPW * T.nwords) return false;
    int32_t *front = T.front0.as<int32_t>();
    // one host read-back per level: the node arrays, flags and next frontier
    // are sized for the most children the level can make (8F); the actual
    // count C and next frontier size come back together at the end
    const int64_t Cmax = 8 * F;
    if (T.nn + Cmax >= ((int64_t)1 << 31))
      fail(PBX_ERR_VALUE, "octree too large (%lld nodes)", (long long)(T.nn + Cmax));
    int32_t *lb = (int32_t *)T.lb.get(4 * 9 * (size_t)F);
    uint32_t *cnt = (uint32_t *)T.cnt.get(4 * (size_t)(F + 1));
    uint32_t *flags = (uint32_t *)T.flags.get(4 * (size_t)(Cmax + 1));
    ensure_nodes(T, T.nn + Cmax, st);
    bind();
    hipLaunchKernelGGL(split_count, dim3(nblk(Cmax + 1)), dim3(TPB), 0, st, v, front, F, d, lb,
                       cnt, flags);
    scan_u32(T.tsum, st, cnt, F + 1);
    hipLaunchKernelGGL(split_make, dim3(nblk(F)), dim3(TPB), 0, st, v, front, F, lb, cnt,
                       (int32_t)T.nn, flags);
    scan_u32(T.tsum, st, flags, Cmax + 1);
    int32_t *front2 = (int32_t *)T.front1.get(4 * (size_t)std::max<int64_t>(Cmax, 1));
    uint32_t *sizes = (uint32_t *)T.small.get(64);
    hipLaunchKernelGGL(compact_frontier, dim3(nblk(Cmax)), dim3(TPB), 0, st, flags, cnt, F,
                       (int32_t)T.nn, front2, sizes);
    PBX_HIP(hipGetLastError());
    uint32_t hs[2];
    PBX_HIP(hipMemcpyAsync(hs, sizes, 8, hipMemcpyDeviceToHost, st));
    PBX_HIP(hipStreamSynchronize(st));
    const int64_t C = hs[0], F2 = hs[1];
    T.nn += C;
    T.lvl.push_back((int32_t)T.nn);
    std::swap(T.front0, T.front1);
    F = F2;
    ++d;
  }
  return true;
}

// subtree sizes (bottom-up) and DFS preorder ids (top-down) of every node
static void preorder(Octree &T, hipStream_t st) {
  int32_t *size = (int32_t *)T.size.get(4 * (size_t)std::max<int64_t>(T.nn, 1));
  int32_t *pre = (int32_t *)T.pre.get(4 * (size_t)std::max<int64_t>(T.nn, 1));
  const int L = (int)T.lvl.size() - 1;
  for (int l = L - 1; l >= 0; --l) {
    const int32_t a = T.lvl[l], b = T.lvl[l + 1];
    hipLaunchKernelGGL(subtree_size, dim3(nblk(b - a)), dim3(TPB), 0, st, T.nfirst.as<int32_t>(),
                       T.nchild.as<int32_t>(), a, b, size);
  }
  PBX_HIP(hipMemsetAsync(pre, 0, 4, st));
  for (int l = 0; l < L; ++l) {
    const int32_t a = T.lvl[l], b = T.lvl[l + 1];
    hipLaunchKernelGGL(preorder_ids, dim3(nblk(b - a)), dim3(TPB), 0, st, T.nfirst.as<int32_t>(),
                       T.nchild.as<int32_t>(), size, a, b, pre);
  }
  PBX_HIP(hipGetLastError());
}

static void build_structure(Octree &T, hipStream_t st) {
  ScopedTimer tm("octree.build_structure");
  const int64_t n = T.n;
  // root box (tree.rs:628-654)
  double mn[3], mx[3];
  {
    unsigned long long *bb = (unsigned long long *)T.small.get(64);
    unsigned long long h[6] = {~0ull, ~0ull, ~0ull, 0ull, 0ull, 0ull};
    PBX_HIP(hipMemcpyAsync(bb, h, 48, hipMemcpyHostToDevice, st));
    if (n > 0)
      hipLaunchKernelGGL(bbox_kernel,  // 3k blocks (TPB = 256): 3 | threads
                         dim3(3 * std::min<unsigned>(256, (nblk(3 * n) + 2) / 3)), dim3(TPB), 0,
                         st, T.pos.as<double>(), n, bb);
    PBX_HIP(hipMemcpyAsync(h, bb, 48, hipMemcpyDeviceToHost, st));
    PBX_HIP(hipStreamSynchronize(st));
    for (int d = 0; d < 3; ++d) {
      // no finite value seen: the reference's +inf / -inf initial bounds
      mn[d] = h[d] == ~0ull ? INFINITY : dkey_inv(h[d]);
      mx[d] = h[3 + d] == 0ull ? -INFINITY : dkey_inv(h[3 + d]);
    }
  }
  {
#pragma clang fp contract(off)
    for (int d = 0; d < 3; ++d) T.root[d] = (mn[d] + mx[d]) / 2.0;
    double half = 0.0;
    for (int d = 0; d < 3; ++d) half = std::fmax(half, (mx[d] - mn[d]) / 2.0);
    if (half == 0.0) half = 1e-6;
    T.root[3] = half;
  }
  T.perm.get(4 * (size_t)std::max<int64_t>(n, 1));
  if (n == 0) {
    T.nn = 0;
    ensure_nodes(T, 64, st);
    int32_t z[2] = {0, 0};
    int32_t neg = -1;
    PBX_HIP(hipMemcpyAsync(T.nstart.p, &z[0], 4, hipMemcpyHostToDevice, st));
    PBX_HIP(hipMemcpyAsync(T.ncount.p, &z[1], 4, hipMemcpyHostToDevice, st));
    PBX_HIP(hipMemcpyAsync(T.nfirst.p, &neg, 4, hipMemcpyHostToDevice, st));
    PBX_HIP(hipMemcpyAsync(T.nnext.p, &neg, 4, hipMemcpyHostToDevice, st));
    PBX_HIP(hipMemcpyAsync(T.nchild.p, &z[0], 4, hipMemcpyHostToDevice, st));
    double4 c = make_double4(T.root[0], T.root[1], T.root[2], T.root[3]);
    PBX_HIP(hipMemcpyAsync(T.ncen.p, &c, sizeof(c), hipMemcpyHostToDevice, st));
    PBX_HIP(hipStreamSynchronize(st));
    T.nn = 1;
    T.lvl.assign({0, 1});
    T.lvl_int.clear();
    T.rec.get(64);
    preorder(T, st);
    return;
  }
  bool parallel = false;
  for (T.nwords = 1;; ++T.nwords) {
    if (T.nwords > MAX_WORDS) fail(PBX_ERR_RUNTIME, "octree deeper than %d levels", LPW * MAX_WORDS);
    auto make_keys = [&] {
      uint64_t *keys = (uint64_t *)T.keys.get(8 * (size_t)n * T.nwords);
      double4 *rec0 = (double4 *)T.rec0.get(sizeof(double4) * (size_t)n);
      hipLaunchKernelGGL(path_keys, dim3(nblk(n)), dim3(TPB), 0, st, T.pos.as<double>(), n,
                         T.root[0], T.root[1], T.root[2], T.root[3], T.nwords, keys,
                         T.user_mass ? T.mass.as<double>() : (const double *)nullptr, rec0);
      T.rec0_valid = true;
      PBX_HIP(hipGetLastError());
    };
    make_keys();
    if (T.nwords == 1) {  // the top 6 bytes first: levels 0..14 (enough for most trees)
      sort_paths(T, st, 16);
      if (split_parallel(T, st, 15)) {
        parallel = true;
        break;
      }
      make_keys();  // the sort replaced the keys: start over with the full sort
    }
    sort_paths(T, st);
    if (split_parallel(T, st, LPW * T.nwords)) {
      parallel = true;
      break;
    }
    if (split_levels(T, st)) break;
  }
  hipLaunchKernelGGL(leaf_sort, dim3(nblk(T.nn)), dim3(TPB), 0, st, T.nchild.as<int32_t>(),
                     T.nstart.as<int32_t>(), T.ncount.as<int32_t>(), T.nn, T.perm.as<int32_t>());
  PBX_HIP(hipGetLastError());
  if (!parallel) preorder(T, st);  // (the parallel build made pre / size already)
}

// softenings in leaf order (+ 4 zero pad entries, read 4 at a time)
static void gather_softenings(Octree &T, hipStream_t st) {
  double *d = (double *)T.soft_s.get(8 * (size_t)(T.n + 4));
  PBX_HIP(hipMemsetAsync(d + T.n, 0, 32, st));
  hipLaunchKernelGGL(gather_f64, dim3(nblk(T.n)), dim3(TPB), 0, st, T.soft.as<double>(),
                     T.perm.as<int32_t>(), T.n, d);
}

static void pack_particles(Octree &T, hipStream_t st) {
  const int64_t n = T.n;
  // 4 zero records of padding: the walk reads leaves 4 records at a time
  double4 *rec = (double4 *)T.rec.get(sizeof(double4) * (size_t)(n + 4));
  PBX_HIP(hipMemsetAsync(rec + n, 0, sizeof(double4) * 4, st));
  if (n > 0) {
    double4 *rec0 = (double4 *)T.rec0.get(sizeof(double4) * (size_t)n);
    if (!T.rec0_valid)  // masses changed since the build (build_mass)
      hipLaunchKernelGGL(interleave_records, dim3(nblk(n)), dim3(TPB), 0, st, T.pos.as<double>(),
                         T.user_mass ? T.mass.as<double>() : (const double *)nullptr, n, rec0);
    T.rec0_valid = true;
    // (one record per thread: a 4-records-per-thread variant with all
    // gathers in flight measured the same, 98.6 vs 100.6 us at 4M — the
    // random 32-byte reads are line-bound, not latency-bound)
    hipLaunchKernelGGL(pack_records, dim3(nblk(n)), dim3(TPB), 0, st, (const double4 *)rec0,
                       T.perm.as<int32_t>(), n, rec);
    if (T.soft_set) gather_softenings(T, st);
  }
  PBX_HIP(hipGetLastError());
}

template <int P>
static void run_payload(Octree &T, hipStream_t st, PayloadView v) {
  const int64_t nn = T.nn;
  if (nn <= 0) return;
  hipLaunchKernelGGL(payload_leaves<P>, dim3((unsigned)((nn + PL_TPB - 1) / PL_TPB)), dim3(PL_TPB),
                     0, st, v);
  // the internal nodes as one breadth-first list (flag, scan, scatter)
  uint32_t *iscan = (uint32_t *)T.iscan.get(sizeof(uint32_t) * (size_t)(nn + 1));
  int32_t *ilist = (int32_t *)T.ilist.get(sizeof(int32_t) * (size_t)nn);
  hipLaunchKernelGGL(internal_flags, dim3(nblk(nn + 1)), dim3(TPB), 0, st, v.nchild, nn, iscan);
  prim::scan_u32(T.iws, st, iscan, nn + 1);
  hipLaunchKernelGGL(internal_list, dim3(nblk(nn)), dim3(TPB), 0, st, v.nchild, iscan, nn, ilist);
  const int nl = (int)T.lvl.size() - 1;
  const bool counted = (int64_t)T.lvl_int.size() == nl;
  std::vector<int64_t> ibase(nl + 1, 0);  // first list slot of each level (counted builds)
  for (int L = 0; counted && L < nl; ++L) ibase[L + 1] = ibase[L] + T.lvl_int[L];
  for (int L = nl - 2; L >= 0; --L) {
    const int32_t a = T.lvl[L], b = T.lvl[L + 1];
    // internal nodes of level L: counted by the parallel build, else at
    // most its nodes and at most the next level's
    const int64_t ub = counted ? T.lvl_int[L]
                       : std::min<int64_t>(b - a, T.lvl[L + 2] - T.lvl[L + 1]);
    if (ub > 0)
      hipLaunchKernelGGL(payload_internal<P>,
                         dim3((unsigned)((ub * PI_G + PL_TPB - 1) / PL_TPB)), dim3(PL_TPB), 0, st,
                         v, (const int32_t *)ilist, (const uint32_t *)iscan, a, b,
                         counted ? ibase[L] : (int64_t)-1, counted ? ibase[L + 1] : (int64_t)-1);
  }
  PBX_HIP(hipGetLastError());
}

// build_mass_payload (tree.rs:968-1012)
static void build_payload(Octree &T, hipStream_t st) {
  ScopedTimer tm("octree.build_mass_payload");
  pack_particles(T, st);
  T.has_hmax = T.soft_set;
  PayloadView v;
  v.nstart = T.nstart.as<int32_t>();
  v.ncount = T.ncount.as<int32_t>();
  v.nfirst = T.nfirst.as<int32_t>();
  v.nchild = T.nchild.as<int32_t>();
  v.rec = T.rec.as<double4>();
  v.soft = T.soft_set ? T.soft_s.as<double>() : nullptr;
  v.com = (double4 *)T.com.get(sizeof(double4) * (size_t)T.nn);
  v.hmax = T.has_hmax ? (double *)T.hmax.get(8 * (size_t)T.nn) : nullptr;
  const int P = T.moment_order();
  v.mom = P >= 2 ? (double *)T.mom.get(8 * (size_t)T.nn * ncoef(P)) : nullptr;
  v.pre = T.pre.as<int32_t>();
  v.size = T.size.as<int32_t>();
  v.ncen = T.ncen.as<double4>();
  v.nn = T.nn;
  auto walk_buf = [&](int stride) { return (double *)T.walk.get(8 * (size_t)T.nn * stride); };
  // walk-record leaf flags share the count word: counts stay below WF_FIRST_LEAF
  v.leaf_dfs = nullptr;
  if (T.nn > 0 && T.n < (int64_t)WF_FIRST_LEAF && T.nn < (int64_t)WF_NEXT_LEAF) {
    uint8_t *ld = (uint8_t *)T.leaf_dfs.get((size_t)T.nn);
    hipLaunchKernelGGL(leaf_dfs_kernel, dim3((unsigned)((T.nn + 255) / 256)), dim3(256), 0, st,
                       (const int32_t *)v.nchild, v.pre, (int64_t)T.nn, ld);
    v.leaf_dfs = ld;
  }
  switch (P) {
    case 0:
    case 1:
      v.walk = walk_buf(rec_stride<0>());
      run_payload<0>(T, st, v);
      break;
    case 2:
      v.walk = walk_buf(rec_stride<2>());
      run_payload<2>(T, st, v);
      break;
    case 3:
      v.walk = walk_buf(rec_stride<3>());
      run_payload<3>(T, st, v);
      break;
    case 4:
      v.walk = walk_buf(rec_stride<4>());
      run_payload<4>(T, st, v);
      break;
    default:
      v.walk = walk_buf(rec_stride<5>());
      run_payload<5>(T, st, v);
      break;
  }
  PBX_HIP(hipGetLastError());
  T.has_bh = true;
  T.open_theta2 = -1.0;
}

// the fast unsoftened walk's opening sizes: size2 / theta^2 into the h_max
// slot (field 5, unused without softening) of every walk record
__global__ void open_scale(double *__restrict__ walk, int64_t nn, int rs, double theta2) {
  const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (k < nn) walk[k * rs + 5] = walk[k * rs + 4] / theta2;
}

// Walk grids: one wave (64 targets) per block, blocks handed out to the XCDs
// in chunks of WALK_XCD_CHUNK consecutive blocks (xcd_chunk_swizzle: the
// waves of neighbouring targets, which walk much the same nodes, share an
// XCD's L2).  Chunks of 16 / 32 / 64 / 128 / 256 blocks: 34.14 / 34.06 /
// 33.95 / 33.67 / 33.76 ms at 4M (profiles/r3/walk_xcd_sweep/), 64 and 256
// re-measured slower again at 8 waves per SIMD (round 5).  Round 6, the
// 4M walk at HEAD (profiles/r6/r7o/, r7p/, three runs each): 128 / 256 /
// 512 28.86 / 28.83 / 28.82 ms (within the noise), 384 / 768 / 1024
// 29.45 / 30.31 / 29.98 ms.
#ifndef PBX_WALK_XCD_CHUNK
#define PBX_WALK_XCD_CHUNK 128
#endif
constexpr unsigned WALK_XCD_CHUNK = PBX_WALK_XCD_CHUNK;
constexpr unsigned WALK_BT = 64;

template <int P, int WANT>
static void launch_walk_pw(WalkParams wp, bool soft, hipStream_t st) {
  unsigned grid = (unsigned)((wp.m + WALK_BT - 1) / WALK_BT);
  wp.xcd_chunk = WALK_XCD_CHUNK;
  {  // whole rounds of kNumXcd chunks (a bijection); the extra blocks find no targets
    const unsigned round = kNumXcd * wp.xcd_chunk;
    grid = (grid + round - 1) / round * round;
  }
  const bool raw = !precise_mode();
  const bool lcost = wp.cost && !wp.cost_kind;  // per-lane counts wanted
  const bool cnt = wp.counters != nullptr;  // (walk() clears it only where a CNT=false variant exists)
  // order 3, potential + acceleration, no softening, no per-lane counts: 8 waves per SIMD
  constexpr bool w8 = P == 3 && WANT == (PBX_WANT_POT | PBX_WANT_ACC);
  if (!cnt) {  // ... fast mode, the statistics off (walk())
    if constexpr (w8)
      hipLaunchKernelGGL((walk_kernel<P, WANT, false, true, false, true, false>), dim3(grid),
                         dim3(WALK_BT), 0, st, wp);
    return;
  }
  if (soft && raw)
    hipLaunchKernelGGL((walk_kernel<P, WANT, true, true>), dim3(grid), dim3(WALK_BT), 0, st, wp);
  else if (soft)
    hipLaunchKernelGGL((walk_kernel<P, WANT, true, false>), dim3(grid), dim3(WALK_BT), 0, st, wp);
  else if (raw && lcost)
    hipLaunchKernelGGL((walk_kernel<P, WANT, false, true, true>), dim3(grid), dim3(WALK_BT), 0, st, wp);
  else if (raw && w8)
    hipLaunchKernelGGL((walk_kernel<P, WANT, false, true, false, true>), dim3(grid), dim3(WALK_BT), 0,
                       st, wp);
  else if (raw)
    hipLaunchKernelGGL((walk_kernel<P, WANT, false, true, false>), dim3(grid), dim3(WALK_BT), 0, st, wp);
  else if (lcost)
    hipLaunchKernelGGL((walk_kernel<P, WANT, false, false, true>), dim3(grid), dim3(WALK_BT), 0, st, wp);
  else if (w8)  // precise, 8 waves per SIMD
    hipLaunchKernelGGL((walk_kernel<P, WANT, false, false, false, true>), dim3(grid), dim3(WALK_BT), 0,
                       st, wp);
  else
    hipLaunchKernelGGL((walk_kernel<P, WANT, false, false, false>), dim3(grid), dim3(WALK_BT), 0, st, wp);
}

template <int P>
static void launch_walk_p(const WalkParams &wp, int want, bool soft, hipStream_t st) {
  if (want == PBX_WANT_POT) launch_walk_pw<P, PBX_WANT_POT>(wp, soft, st);
  else if (want == PBX_WANT_ACC) launch_walk_pw<P, PBX_WANT_ACC>(wp, soft, st);
  else launch_walk_pw<P, PBX_WANT_POT | PBX_WANT_ACC>(wp, soft, st);
}

// walk for m targets (tgt == null: all particles, skip_self) into device
// outputs in original / query order
static void walk(Octree &T, double theta, int want, const double *d_tgt, int64_t m, double *d_pot,
                 double *d_acc, hipStream_t st, int64_t first = 0, int compact = 0,
                 int32_t *d_cost = nullptr) {
  unsigned long long *ctr = (unsigned long long *)T.counters.get(64);
  PBX_HIP(hipMemsetAsync(ctr, 0, 64, st));
  if (m == 0) return;
  WalkParams wp;
  wp.walk = T.walk.as<double>();
  wp.rec = T.rec.as<double4>();
  wp.tgt = d_tgt;

  wp.soft = T.soft_set ? T.soft_s.as<double>() : nullptr;
  wp.perm = T.perm.as<int32_t>();
  wp.m = m;
  wp.first = first;
  wp.compact = compact;
  wp.cost = d_cost;
  {
#pragma clang fp contract(off)
    wp.theta2 = theta * theta;  // tree.rs:1428
  }
  wp.sep = T.kernel == 0 ? 2.8 : 1.0;
  wp.kernel = T.kernel;
  wp.has_hmax = T.has_hmax ? 1 : 0;
  wp.pot = d_pot;
  wp.acc = d_acc;
  // the walk statistics, unless the caller turned them off for a walk that
  // has a CNT=false variant (order 3, pot + acc, no softening, fast mode,
  // no per-lane interaction counts)
  const bool nocnt = !T.walk_counts && T.moment_order() == 3 && !(T.has_hmax || T.soft_set) &&
                     want == (PBX_WANT_POT | PBX_WANT_ACC) && !precise_mode() &&
                     !(d_cost && T.cost_kind == 0);
  wp.counters = nocnt ? nullptr : ctr;
  wp.max_steps = T.nn + 16;
  wp.fault = (unsigned int *)(ctr + 2);
  wp.cost_kind = T.cost_kind;
  wp.trace = nullptr;
  const char *trace_path = std::getenv("PBX_WALK_TRACE");  // diagnostic only
  unsigned tgrid = 0;
  if (trace_path) {
    tgrid = (unsigned)((m + WALK_BT - 1) / WALK_BT);  // one trace record per wave (block)
    const unsigned c = WALK_XCD_CHUNK;
    tgrid = (tgrid + kNumXcd * c - 1) / (kNumXcd * c) * (kNumXcd * c);
    wp.trace = (unsigned long long *)T.trace.get(24 * (size_t)tgrid);
  }
  // softened leaves need softenings; the guard needs h_max; at query points
  // there is no target softening (tree.rs:1516,1547)
  const bool soft = T.has_hmax || T.soft_set;
  if (!soft && !precise_mode() && T.nn > 0 && T.open_theta2 != wp.theta2) {
    const int rs = T.moment_order() <= 1 ? rec_stride<0>() : T.moment_order() == 2 ? rec_stride<2>()
                   : T.moment_order() == 3 ? rec_stride<3>() : T.moment_order() == 4 ? rec_stride<4>()
                                                             : rec_stride<5>();
    hipLaunchKernelGGL(open_scale, dim3((unsigned)((T.nn + 255) / 256)), dim3(256), 0, st,
                       T.walk.as<double>(), (int64_t)T.nn, rs, wp.theta2);
    T.open_theta2 = wp.theta2;
  }
  if (T.n == 0) {
    if (d_pot) PBX_HIP(hipMemsetAsync(d_pot, 0, 8 * (size_t)m, st));
    if (d_acc) PBX_HIP(hipMemsetAsync(d_acc, 0, 24 * (size_t)m, st));
    return;
  }
  switch (T.moment_order()) {
    case 0: launch_walk_p<0>(wp, want, soft, st); break;
    case 1: launch_walk_p<1>(wp, want, soft, st); break;
    case 2: launch_walk_p<2>(wp, want, soft, st); break;
    case 3: launch_walk_p<3>(wp, want, soft, st); break;
    case 4: launch_walk_p<4>(wp, want, soft, st); break;
    default: launch_walk_p<5>(wp, want, soft, st); break;
  }
  PBX_HIP(hipGetLastError());
  if (trace_path) {  // append (start, end, steps) per block, launch order
    std::vector<unsigned long long> h(3 * (size_t)tgrid);
    PBX_HIP(hipMemcpyAsync(h.data(), wp.trace, 24 * (size_t)tgrid, hipMemcpyDeviceToHost, st));
    PBX_HIP(hipStreamSynchronize(st));
    if (FILE *f = std::fopen(trace_path, "ab")) {
      std::fwrite(h.data(), 8, h.size(), f);
      std::fclose(f);
    }
  }
}

static Octree &as_tree(pbx_octree *h) {
  if (!h) fail(PBX_ERR_VALUE, "null octree handle");
  Octree *t = (Octree *)h;
  if (t->device != current_device().id) fail(PBX_ERR_VALUE, "octree belongs to device %d", t->device);
  return *t;
}

static void upload(Buf &b, const double *src, int64_t count, int on_device, hipStream_t st) {
  double *d = (double *)b.get(8 * (size_t)std::max<int64_t>(count, 1));
  if (count > 0)
    PBX_HIP(hipMemcpyAsync(d, src, 8 * (size_t)count,
                           on_device ? hipMemcpyDeviceToDevice : hipMemcpyHostToDevice, st));
}

// Octree::new on (new) particles (gravity.rs:123-226): copies, structure,
// mass payload iff masses; HBM buffers are grow-only and reused
static void init_tree(Octree &T, const double *pos, int64_t n, const double *masses,
                      const double *softenings, int on_device, hipStream_t st) {
  T.n = n;
  T.has_bh = T.has_hmax = false;
  T.user_mass = T.soft_set = false;
  upload(T.pos, pos, 3 * n, on_device, st);
  if (masses) {
    upload(T.mass, masses, n, on_device, st);
    T.user_mass = true;
  }
  if (softenings) {
    upload(T.soft, softenings, n, on_device, st);
    T.soft_set = true;
  }
  build_structure(T, st);
  if (masses) build_payload(T, st);  // gravity.rs:210-220
  PBX_HIP(hipStreamSynchronize(st));
}

static const char *method_name(int want, bool at_points) {
  if (at_points) return want == PBX_WANT_POT ? "potentials_at_points" : "accelerations_at_points";
  return want == PBX_WANT_POT ? "compute_potentials" : "compute_accelerations";
}

// ---------------------------------------- radial profile of walk outputs
// The 3-D radial profile of a per-target field (the potential of config 5)
// over a range of the leaf-ordered targets, straight from the tree's
// records: RadialProfile(ndim=3) with explicit edges — r = sqrt((x*x+y*y)+z*z)
// (the selection's expression, no FMA), bins.py:346-395 assignment (bin_of),
// and the seven per-bin columns of pbx_profile_moments with f = the field,
// w = the mass (proarray.py:272-334 statistics read them) + the bin counts.
// It replaces select + assign + gather + moments (and their host syncs).
// Every thread takes RM_PT consecutive targets — neighbours in leaf order,
// mostly one bin — and adds a run's sums to LDS when the bin changes, so
// the LDS atomics are few and rarely contended; one slab row per block and
// a fixed-order sum over the rows (radial_moments_reduce).
constexpr int RM_PT = 8;
constexpr int RM_CHUNK = TPB * RM_PT;
constexpr int RM_MAXB = 1024;
__global__ void __launch_bounds__(TPB)
    radial_moments_kernel(const double4 *__restrict__ rec, const double *__restrict__ f,
                          int64_t first, int64_t count, const double *__restrict__ edges, int nb,
                          double *__restrict__ slab, uint32_t *__restrict__ cslab,
                          int e_lds) {
  extern __shared__ __attribute__((aligned(16))) double rm_sm[];
  // edges in LDS when everything fits the 64 KB a workgroup may allocate
  // (nb <= 963); above that they are read from global memory (L1/L2-hot)
  const double *e = e_lds ? rm_sm : edges;
  double *acc = rm_sm + (e_lds ? nb + 1 : 0);
  uint32_t *cnt = (uint32_t *)(acc + 7 * (int64_t)nb);
  if (e_lds)
    for (int k = threadIdx.x; k <= nb; k += TPB) rm_sm[k] = edges[k];
  for (int k = threadIdx.x; k < 7 * nb; k += TPB) acc[k] = 0.0;
  for (int k = threadIdx.x; k < nb; k += TPB) cnt[k] = 0u;
  __syncthreads();
  for (int64_t c0 = (int64_t)blockIdx.x * RM_CHUNK; c0 < count; c0 += (int64_t)gridDim.x * RM_CHUNK) {
    const int64_t i0 = c0 + (int64_t)threadIdx.x * RM_PT;
    double4 q[RM_PT];
    double v[RM_PT];
#pragma unroll
    for (int k = 0; k < RM_PT; ++k) {  // all loads in flight before use
      const int64_t i = i0 + k < count ? i0 + k : 0;
      q[k] = rec[first + i];
      v[k] = f[i];
    }
    uint32_t cur = (uint32_t)nb, c = 0;
    double s[7] = {0, 0, 0, 0, 0, 0, 0};
    auto flush = [&]() {
      if (cur < (uint32_t)nb && c) {
#pragma unroll
        for (int j = 0; j < 7; ++j) atomicAdd(&acc[cur * 7 + j], s[j]);
        atomicAdd(&cnt[cur], c);
      }
#pragma unroll
      for (int j = 0; j < 7; ++j) s[j] = 0.0;
      c = 0;
    };
#pragma unroll
    for (int k = 0; k < RM_PT; ++k) {
      if (i0 + k >= count) break;
      double r;
      {
#pragma clang fp contract(off)
        r = __builtin_sqrt((q[k].x * q[k].x + q[k].y * q[k].y) + q[k].z * q[k].z);
      }
      const uint32_t b = bin_of(r, e, nb);
      if (b != cur) {
        flush();
        cur = b;
      }
      if (b < (uint32_t)nb) {
#pragma clang fp contract(off)
        const double x = v[k], w = q[k].w, a = __builtin_fabs(x);
        s[0] += w;
        s[1] += x * w;
        s[2] += (x * x) * w;
        s[3] += x;
        s[4] += x * x;
        s[5] += a * w;
        s[6] += a;
        ++c;
      }
    }
    flush();
  }
  __syncthreads();
  double *dst = slab + (int64_t)blockIdx.x * 7 * nb;
  for (int k = threadIdx.x; k < 7 * nb; k += TPB) dst[k] = acc[k];
  uint32_t *cd = cslab + (int64_t)blockIdx.x * nb;
  for (int k = threadIdx.x; k < nb; k += TPB) cd[k] = cnt[k];
}

// out = [counts nb (u64)][moments nb x 7]: column j summed over the rows in
// a fixed order: RR_G row groups (group g: rows g, g + RR_G, ...) summed
// by one thread each, coalesced over RR_C columns, then the group partials
// in group order (LDS).  (One thread per column over all rows took 130 us
// at 4M: ~2k dependent rows per thread.)
constexpr int RR_C = 32, RR_G = 32;
__global__ void __launch_bounds__(RR_C * RR_G)
    radial_moments_reduce(const double *__restrict__ slab, const uint32_t *__restrict__ cslab,
                          int rows, int nb, double *__restrict__ out) {
  __shared__ double ps[RR_G][RR_C + 1];
  __shared__ unsigned long long pc[RR_G][RR_C + 1];
  const int c = threadIdx.x % RR_C, g = threadIdx.x / RR_C;
  const int j = blockIdx.x * RR_C + c;
  double sum = 0.0;
  unsigned long long cnt = 0;
  if (j < nb) {
    for (int r = g; r < rows; r += RR_G) cnt += cslab[(int64_t)r * nb + j];
  } else if (j < 8 * nb) {
    const int k = j - nb;
    for (int r = g; r < rows; r += RR_G) sum += slab[(int64_t)r * 7 * nb + k];
  }
  ps[g][c] = sum;
  pc[g][c] = cnt;
  __syncthreads();
  if (g == 0 && j < 8 * nb) {
    if (j < nb) {
      unsigned long long t = 0;
      for (int q = 0; q < RR_G; ++q) t += pc[q][c];
      out[j] = __builtin_bit_cast(double, t);
    } else {
      double t = 0.0;
      for (int q = 0; q < RR_G; ++q) t += ps[q][c];
      out[j] = t;
    }
  }
}

}  // namespace tree
}  // namespace pbx

using namespace pbx;
using namespace pbx::tree;

extern "C" {

int pbx_octree_create(const double *pos, int64_t n, const double *masses,
                      const double *softenings, int64_t leaf_capacity, int multipole_order,
                      int kernel, int on_device, pbx_octree **out) {
  return guard([&] {
    if (!out) fail(PBX_ERR_VALUE, "null output handle");
    *out = nullptr;
    if (n < 0) fail(PBX_ERR_VALUE, "negative particle count");
    if (n >= ((int64_t)1 << 31) - 1) fail(PBX_ERR_VALUE, "octrees are limited to < 2^31 particles");
    if (n > 0 && !pos) fail(PBX_ERR_VALUE, "positions must not be null");
    if (kernel != 0 && kernel != 1) fail(PBX_ERR_VALUE, "kernel must be 0 (Plummer) or 1 (CubicSplineW2)");
    if (multipole_order < 0 || multipole_order > 255) fail(PBX_ERR_VALUE, "multipole_order must fit in u8");
    Device &dev = current_device();
    std::lock_guard<std::mutex> lk(dev.mu);
    Octree *T = new Octree();
    try {
      T->device = dev.id;
      T->leaf_capacity = leaf_capacity < 1 ? 1 : leaf_capacity;  // tree.rs:701
      T->order = multipole_order;
      T->kernel = kernel;
      init_tree(*T, pos, n, masses, softenings, on_device, dev.stream);
    } catch (...) {
      delete T;
      throw;
    }
    *out = (pbx_octree *)T;
  });
}

int pbx_octree_rebuild(pbx_octree *t, const double *pos, int64_t n, const double *masses,
                       const double *softenings, int on_device) {
  return guard([&] {
    Octree &T = as_tree(t);
    if (n < 0) fail(PBX_ERR_VALUE, "negative particle count");
    if (n >= ((int64_t)1 << 31) - 1) fail(PBX_ERR_VALUE, "octrees are limited to < 2^31 particles");
    if (n > 0 && !pos) fail(PBX_ERR_VALUE, "positions must not be null");
    Device &dev = current_device();
    std::lock_guard<std::mutex> lk(dev.mu);
    init_tree(T, pos, n, masses, softenings, on_device, dev.stream);
  });
}

int pbx_octree_destroy(pbx_octree *t) {
  return guard([&] { delete (Octree *)t; });
}

int pbx_octree_build_mass(pbx_octree *t, const double *masses, int on_device) {
  return guard([&] {
    Octree &T = as_tree(t);
    Device &dev = current_device();
    std::lock_guard<std::mutex> lk(dev.mu);
    if (masses) {
      upload(T.mass, masses, T.n, on_device, dev.stream);
      T.user_mass = true;
      T.rec0_valid = false;
    }
    build_payload(T, dev.stream);
    PBX_HIP(hipStreamSynchronize(dev.stream));
  });
}

int pbx_octree_set_softenings(pbx_octree *t, const double *softenings, int on_device) {
  return guard([&] {
    Octree &T = as_tree(t);
    Device &dev = current_device();
    std::lock_guard<std::mutex> lk(dev.mu);
    if (softenings) {
      upload(T.soft, softenings, T.n, on_device, dev.stream);
      T.soft_set = true;
      if (T.n > 0) gather_softenings(T, dev.stream);
    } else {
      T.soft_set = false;  // h_max keeps its build-time value (tree.rs:777-782)
    }
    PBX_HIP(hipStreamSynchronize(dev.stream));
  });
}

int pbx_octree_set_kernel(pbx_octree *t, int kernel) {
  return guard([&] {
    Octree &T = as_tree(t);
    if (kernel != 0 && kernel != 1) fail(PBX_ERR_VALUE, "kernel must be 0 (Plummer) or 1 (CubicSplineW2)");
    T.kernel = kernel;
  });
}

int pbx_octree_compute(pbx_octree *t, double theta, int want, double *pot, double *acc,
                       int on_device) {
  return guard([&] {
    Octree &T = as_tree(t);
    if (want < 1 || want > 3) fail(PBX_ERR_VALUE, "want must be 1, 2 or 3");
    if (!T.has_bh)
      fail(PBX_ERR_VALUE, "mass payload not built; call build_mass() before %s",
           method_name(want, false));
    Device &dev = current_device();
    std::lock_guard<std::mutex> lk(dev.mu);
    hipStream_t st = dev.stream;
    ScopedTimer tm("octree.compute");
    const int64_t n = T.n;
    double *dp = nullptr, *da = nullptr;
    if (on_device) {
      dp = (want & PBX_WANT_POT) ? pot : nullptr;
      da = (want & PBX_WANT_ACC) ? acc : nullptr;
    } else {
      if (want & PBX_WANT_POT) dp = (double *)dev.slot(kSlotPot).ensure(8 * (size_t)std::max<int64_t>(n, 1));
      if (want & PBX_WANT_ACC) da = (double *)dev.slot(kSlotAcc).ensure(24 * (size_t)std::max<int64_t>(n, 1));
    }
    walk(T, theta, want, nullptr, n, dp, da, st);
    PBX_HIP(hipMemcpyAsync(T.last_counts, T.counters.p, 64, hipMemcpyDeviceToHost, st));
    if (!on_device) {
      if (dp && n) PBX_HIP(hipMemcpyAsync(pot, dp, 8 * (size_t)n, hipMemcpyDeviceToHost, st));
      if (da && n) PBX_HIP(hipMemcpyAsync(acc, da, 24 * (size_t)n, hipMemcpyDeviceToHost, st));
    }
    PBX_HIP(hipStreamSynchronize(st));
    if (T.last_counts[2] & 0xffffffffull) fail(PBX_ERR_RUNTIME, "octree walk exceeded its step bound");
  });
}

int pbx_octree_at_points(pbx_octree *t, const double *points, int64_t m, double theta, int want,
                         double *pot, double *acc, int on_device) {
  return guard([&] {
    Octree &T = as_tree(t);
    if (want < 1 || want > 3) fail(PBX_ERR_VALUE, "want must be 1, 2 or 3");
    if (!T.has_bh)
      fail(PBX_ERR_VALUE, "mass payload not built; call build_mass() before %s",
           method_name(want, true));
    if (m < 0) fail(PBX_ERR_VALUE, "negative point count");
    if (m >= ((int64_t)1 << 31)) fail(PBX_ERR_VALUE, "too many query points");
    if (m > 0 && !points) fail(PBX_ERR_VALUE, "points must not be null");
    Device &dev = current_device();
    std::lock_guard<std::mutex> lk(dev.mu);
    hipStream_t st = dev.stream;
    const double *dt = points;
    double *dp = nullptr, *da = nullptr;
    if (on_device) {
      dp = (want & PBX_WANT_POT) ? pot : nullptr;
      da = (want & PBX_WANT_ACC) ? acc : nullptr;
    } else {
      double *tb = (double *)dev.slot(kSlotTgt).ensure(24 * (size_t)std::max<int64_t>(m, 1));
      if (m) PBX_HIP(hipMemcpyAsync(tb, points, 24 * (size_t)m, hipMemcpyHostToDevice, st));
      dt = tb;
      if (want & PBX_WANT_POT) dp = (double *)dev.slot(kSlotPot).ensure(8 * (size_t)std::max<int64_t>(m, 1));
      if (want & PBX_WANT_ACC) da = (double *)dev.slot(kSlotAcc).ensure(24 * (size_t)std::max<int64_t>(m, 1));
    }
    // at points there is no target softening and no self skip
    walk(T, theta, want, dt, m, dp, da, st);
    PBX_HIP(hipMemcpyAsync(T.last_counts, T.counters.p, 64, hipMemcpyDeviceToHost, st));
    if (!on_device) {
      if (dp && m) PBX_HIP(hipMemcpyAsync(pot, dp, 8 * (size_t)m, hipMemcpyDeviceToHost, st));
      if (da && m) PBX_HIP(hipMemcpyAsync(acc, da, 24 * (size_t)m, hipMemcpyDeviceToHost, st));
    }
    PBX_HIP(hipStreamSynchronize(st));
    if (T.last_counts[2] & 0xffffffffull) fail(PBX_ERR_RUNTIME, "octree walk exceeded its step bound");
  });
}

int pbx_octree_compute_range(pbx_octree *t, double theta, int want, int64_t first, int64_t count,
                             int compact, double *d_pot, double *d_acc, int32_t *d_cost) {
  return guard([&] {
    Octree &T = as_tree(t);
    if (want < 1 || want > 3) fail(PBX_ERR_VALUE, "want must be 1, 2 or 3");
    if (!T.has_bh)
      fail(PBX_ERR_VALUE, "mass payload not built; call build_mass() before %s",
           method_name(want, false));
    if (first < 0 || count < 0 || first + count > T.n)
      fail(PBX_ERR_VALUE, "target range [%lld, %lld) outside [0, %lld)", (long long)first,
           (long long)(first + count), (long long)T.n);
    Device &dev = current_device();
    std::lock_guard<std::mutex> lk(dev.mu);
    hipStream_t st = dev.stream;
    ScopedTimer tm("octree.compute_range");
    walk(T, theta, want, nullptr, count, (want & PBX_WANT_POT) ? d_pot : nullptr,
         (want & PBX_WANT_ACC) ? d_acc : nullptr, st, first, compact, d_cost);
    PBX_HIP(hipMemcpyAsync(T.last_counts, T.counters.p, 64, hipMemcpyDeviceToHost, st));
    PBX_HIP(hipStreamSynchronize(st));
    if (T.last_counts[2] & 0xffffffffull) fail(PBX_ERR_RUNTIME, "octree walk exceeded its step bound");
  });
}

int pbx_octree_leaf_particles(pbx_octree *t, int64_t first, int64_t count, double *d_pos,
                              double *d_mass, int64_t *d_idx) {
  return guard([&] {
    Octree &T = as_tree(t);
    if (first < 0 || count < 0 || first + count > T.n) fail(PBX_ERR_VALUE, "range outside the tree");
    if (!T.has_bh) fail(PBX_ERR_VALUE, "mass payload not built; call build_mass() first");
    Device &dev = current_device();
    std::lock_guard<std::mutex> lk(dev.mu);
    if (count > 0)
      hipLaunchKernelGGL(leaf_particles_kernel, dim3(nblk(count)), dim3(TPB), 0, dev.stream,
                         T.rec.as<double4>(), T.perm.as<int32_t>(), first, count, d_pos, d_mass,
                         d_idx);
    PBX_HIP(hipGetLastError());
    PBX_HIP(hipStreamSynchronize(dev.stream));
  });
}

// select + assign + moments of a leaf-order range, fused: the device result
// [nbins int64 counts | nbins x 7 doubles] in the device's staging slot
static const double *radial_moments_run(Octree &T, int64_t first, int64_t count, const double *d_f,
                                        const double *h_edges, int64_t nbins, Device &dev) {
  if (first < 0 || count < 0 || first + count > T.n) fail(PBX_ERR_VALUE, "range outside the tree");
  if (!T.has_bh) fail(PBX_ERR_VALUE, "mass payload not built; call build_mass() first");
  if (nbins < 1 || nbins > RM_MAXB) fail(PBX_ERR_VALUE, "nbins must be in [1, %d]", RM_MAXB);
  for (int64_t k = 0; k < nbins; ++k)
    if (!(h_edges[k] <= h_edges[k + 1]))
      fail(PBX_ERR_VALUE, "bin edges must be increasing");
  hipStream_t st = dev.stream;
  const int nb = (int)nbins;
  const int rows = (int)std::max<int64_t>(1, std::min<int64_t>(512, (count + RM_CHUNK - 1) / RM_CHUNK));
  const size_t eb = sizeof(double) * (size_t)(nb + 1);
  const size_t sb = sizeof(double) * 7 * (size_t)nb * rows, cb = sizeof(uint32_t) * (size_t)nb * rows;
  const size_t ob = sizeof(double) * 8 * (size_t)nb;
  char *w = (char *)dev.slot(kSlotProf7).ensure(eb + sb + cb + ob + 64);
  double *de = (double *)w;
  double *slab = (double *)(w + ((eb + 15) & ~(size_t)15));
  uint32_t *cslab = (uint32_t *)((char *)slab + sb);
  double *out = (double *)(((uintptr_t)((char *)cslab + cb) + 15) & ~(uintptr_t)15);
  PBX_HIP(hipMemcpyAsync(de, h_edges, eb, hipMemcpyHostToDevice, st));
  const size_t lds_acc = sizeof(double) * 7 * nb + sizeof(uint32_t) * nb;
  const int e_lds = eb + lds_acc <= 65536 ? 1 : 0;
  const size_t lds = (e_lds ? eb : 0) + lds_acc;  // <= 61,440 B at RM_MAXB
  hipLaunchKernelGGL(radial_moments_kernel, dim3(rows), dim3(TPB), lds, st, T.rec.as<double4>(),
                     d_f, first, count, (const double *)de, nb, slab, cslab, e_lds);
  hipLaunchKernelGGL(radial_moments_reduce, dim3((unsigned)((8 * (int64_t)nb + RR_C - 1) / RR_C)),
                     dim3(RR_C * RR_G), 0, st,
                     (const double *)slab, (const uint32_t *)cslab, rows, nb, out);
  PBX_HIP(hipGetLastError());
  return out;
}

int pbx_octree_radial_moments(pbx_octree *t, int64_t first, int64_t count, const double *d_f,
                              const double *h_edges, int64_t nbins, int64_t *h_counts,
                              double *h_moments) {
  return guard([&] {
    Octree &T = as_tree(t);
    Device &dev = current_device();
    std::lock_guard<std::mutex> lk(dev.mu);
    ScopedTimer tm("octree.radial_moments");
    const double *out = radial_moments_run(T, first, count, d_f, h_edges, nbins, dev);
    const size_t ob = sizeof(double) * 8 * (size_t)nbins;
    double *hp = (double *)T.rm_pin.get(ob);
    PBX_HIP(hipMemcpyAsync(hp, out, ob, hipMemcpyDeviceToHost, dev.stream));
    PBX_HIP(hipStreamSynchronize(dev.stream));
    std::memcpy(h_counts, hp, sizeof(int64_t) * nbins);
    std::memcpy(h_moments, hp + nbins, sizeof(double) * 7 * nbins);
  });
}

int pbx_octree_radial_moments_device(pbx_octree *t, int64_t first, int64_t count,
                                     const double *d_f, const double *h_edges, int64_t nbins,
                                     void *d_out) {
  return guard([&] {
    Octree &T = as_tree(t);
    if (!d_out) fail(PBX_ERR_VALUE, "null output");
    Device &dev = current_device();
    std::lock_guard<std::mutex> lk(dev.mu);
    ScopedTimer tm("octree.radial_moments");
    const double *out = radial_moments_run(T, first, count, d_f, h_edges, nbins, dev);
    PBX_HIP(hipMemcpyAsync(d_out, out, sizeof(double) * 8 * (size_t)nbins,
                           hipMemcpyDeviceToDevice, dev.stream));
  });
}

int pbx_octree_cost_to_orig(pbx_octree *t, const int32_t *d_cost_leaf, int32_t *d_cost_orig) {
  return guard([&] {
    Octree &T = as_tree(t);
    if (T.n > 0 && (!d_cost_leaf || !d_cost_orig)) fail(PBX_ERR_VALUE, "null cost array");
    Device &dev = current_device();
    std::lock_guard<std::mutex> lk(dev.mu);
    if (T.n > 0)
      hipLaunchKernelGGL(cost_to_orig, dim3(nblk(T.n)), dim3(TPB), 0, dev.stream, d_cost_leaf,
                         T.perm.as<int32_t>(), T.n, d_cost_orig);
    PBX_HIP(hipGetLastError());
  });
}

int pbx_octree_set_walk_counters(pbx_octree *t, int enabled) {
  return guard([&] {
    Octree &T = as_tree(t);
    T.walk_counts = enabled != 0;
  });
}

int pbx_octree_set_cost_kind(pbx_octree *t, int kind) {
  return guard([&] {
    Octree &T = as_tree(t);
    if (kind != 0 && kind != 1) fail(PBX_ERR_VALUE, "cost kind must be 0 or 1");
    T.cost_kind = kind;
  });
}

int pbx_octree_balance(pbx_octree *t, const int32_t *d_cost_orig, int world, int64_t *cuts) {
  return guard([&] {
    Octree &T = as_tree(t);
    if (world < 1 || world > 4096) fail(PBX_ERR_VALUE, "world must be in [1, 4096]");
    if (!cuts) fail(PBX_ERR_VALUE, "null cuts");
    if (T.n > 0 && !d_cost_orig) fail(PBX_ERR_VALUE, "null cost array");
    Device &dev = current_device();
    std::lock_guard<std::mutex> lk(dev.mu);
    hipStream_t st = dev.stream;
    const int64_t nchunks = (T.n + BAL_CHUNK - 1) / BAL_CHUNK;
    int64_t *sums = (int64_t *)T.bal.get(8 * (size_t)(nchunks + world + 1));
    int64_t *dcuts = sums + nchunks;
    if (nchunks > 0)
      hipLaunchKernelGGL(bal_chunk_sums, dim3((unsigned)nchunks), dim3(BAL_TPB), 0, st, d_cost_orig,
                         T.perm.as<int32_t>(), T.n, sums);
    hipLaunchKernelGGL(bal_cuts, dim3(1), dim3(BAL_TPB), 0, st, d_cost_orig, T.perm.as<int32_t>(),
                       T.n, sums, nchunks, world, dcuts);
    PBX_HIP(hipGetLastError());
    PBX_HIP(hipMemcpyAsync(cuts, dcuts, 8 * (size_t)(world + 1), hipMemcpyDeviceToHost, st));
    PBX_HIP(hipStreamSynchronize(st));
  });
}

int pbx_octree_info(pbx_octree *t, int64_t *out) {
  return guard([&] {
    Octree &T = as_tree(t);
    if (!out) fail(PBX_ERR_VALUE, "null output");
    out[0] = T.n;
    out[1] = T.nn;
    out[2] = (int64_t)T.lvl.size() - 1;  // levels (root = 1)
    out[3] = T.has_bh;
    out[4] = T.has_hmax;
    out[5] = (int64_t)T.last_counts[0];
    out[6] = (int64_t)T.last_counts[1];
    out[7] = T.nwords;
    out[8] = (int64_t)T.last_counts[3];
    out[9] = (int64_t)T.last_counts[4];
    out[10] = (int64_t)T.last_counts[5];
    out[11] = (int64_t)T.last_counts[6];
    out[12] = (int64_t)T.last_counts[7];
  });
}

int pbx_octree_export(pbx_octree *t, double *center, double *com, double *hmax, int64_t *links,
                      int64_t *leaf, int64_t *perm, double *moments) {
  return guard([&] {
    Octree &T = as_tree(t);
    Device &dev = current_device();
    std::lock_guard<std::mutex> lk(dev.mu);
    hipStream_t st = dev.stream;
    const int64_t nn = T.nn, n = T.n;
    auto dl = [&](void *dst, const void *src, size_t bytes) {
      if (dst && bytes) PBX_HIP(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, st));
    };
    dl(center, T.ncen.p, sizeof(double4) * nn);
    if (com) {
      if (!T.has_bh) fail(PBX_ERR_VALUE, "mass payload not built");
      dl(com, T.com.p, sizeof(double4) * nn);
    }
    if (hmax && T.has_hmax) dl(hmax, T.hmax.p, 8 * nn);
    std::vector<int32_t> a(nn), b(nn), c(nn), s(nn), k(nn);
    if (links || leaf) {
      dl(a.data(), T.nfirst.p, 4 * nn);
      dl(b.data(), T.nnext.p, 4 * nn);
      dl(c.data(), T.nchild.p, 4 * nn);
      dl(s.data(), T.nstart.p, 4 * nn);
      dl(k.data(), T.ncount.p, 4 * nn);
    }
    std::vector<int32_t> pm(n);
    if (perm) dl(pm.data(), T.perm.p, 4 * n);
    std::vector<double> momq;  // coefficient-major on the device
    if (moments && T.has_bh && T.moment_order() >= 2) {
      momq.resize((size_t)nn * ncoef(T.moment_order()));
      dl(momq.data(), T.mom.p, 8 * momq.size());
    }
    PBX_HIP(hipStreamSynchronize(st));
    if (!momq.empty()) {
      const int nq = ncoef(T.moment_order());
      for (int64_t i = 0; i < nn; ++i)
        for (int q = 0; q < nq; ++q) moments[i * nq + q] = momq[(size_t)q * nn + i];
    }
    for (int64_t i = 0; i < nn; ++i) {
      if (links) {
        links[3 * i] = c[i] ? a[i] : -1;
        links[3 * i + 1] = b[i];
        links[3 * i + 2] = c[i];
      }
      if (leaf) {
        leaf[2 * i] = s[i];
        leaf[2 * i + 1] = k[i];
      }
    }
    if (perm)
      for (int64_t i = 0; i < n; ++i) perm[i] = pm[i];
  });
}

}  // extern "C"
