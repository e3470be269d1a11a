// direct.hip — O(N^2) direct-summation gravity for gfx950.
//
// Replaces crates/gravity/src/direct.rs:115-658 (all eight direct-sum entry
// points) and the softening kernels of crates/gravity/src/kernel.rs:41-128,
// behind the C ABI of include/pbx.h (the PyO3 layer it replaces is
// crates/pynbodyext-rust/src/gravity.rs:448-709).
//
// Design (see DESIGN.md "direct-sum kernel"):
//  * Sources live in HBM as 32-byte records {x, y, z, m}.  Every lane of a
//    wave walks the SAME source index j, so each record is a wave-uniform
//    load that the compiler issues as a scalar (s_load) fetch through the
//    scalar cache: no LDS, no barriers, and the record's doubles feed the
//    FP64 VALU as SGPR operands.
//  * Each lane owns T targets (registers), so one scalar record feeds
//    64*T pair interactions.  The path is FP64-VALU bound; HBM traffic is
//    32 B per source per wave pass, served from L2 / Infinity Cache.
//  * 1/sqrt(s2) is v_rsq_f64 (about 2^-23 relative) refined by one
//    Newton-Raphson step to ~1e-16, then cubed for the force.
//  * The source range can be split over blockIdx.y (partial sums reduced in
//    a fixed order by a second kernel) so small target sets still fill the
//    256 CUs.
//  * Self-interaction (all-particles form) is excluded only on the
//    "diagonal" source window of each block, so the main loop carries no
//    per-pair compare.
#include <cstdlib>
#include <cstring>

#include "pbx_common.h"

namespace pbx {

// f64::MIN_POSITIVE, the additive guard of direct.rs:7.
static constexpr double kR2Tiny = 2.2250738585072014e-308;
static constexpr int kBlock = 256;

__device__ __forceinline__ double rsqrt_nr(double x) {
  double y = __builtin_amdgcn_rsq(x);
  double e = __builtin_fma(-x * y, y, 1.0);
  return __builtin_fma(0.5 * y, e, y);
}

// Springel W2 kernel and derivative (kernel.rs:85-128), u in [0, 1).
__device__ __forceinline__ double w2_inner(double u) {
  double u2 = u * u;
  if (u < 0.5) {
    double u4 = u2 * u2;
    double u5 = u4 * u;
    return (16.0 / 3.0) * u2 - (48.0 / 5.0) * u4 + (32.0 / 5.0) * u5 - 14.0 / 5.0;
  }
  double inv_u = 1.0 / u;
  double u3 = u2 * u;
  double u4 = u2 * u2;
  double u5 = u4 * u;
  return (1.0 / 15.0) * inv_u + (32.0 / 3.0) * u2 - 16.0 * u3 + (48.0 / 5.0) * u4 -
         (32.0 / 15.0) * u5 - 16.0 / 5.0;
}

__device__ __forceinline__ double w2p_inner(double u) {
  double u2 = u * u;
  double u3 = u2 * u;
  double u4 = u2 * u2;
  if (u < 0.5) return (32.0 / 3.0) * u - (192.0 / 5.0) * u3 + 32.0 * u4;
  return -(1.0 / 15.0) * (1.0 / u2) + (64.0 / 3.0) * u - 48.0 * u2 + (192.0 / 5.0) * u3 -
         (32.0 / 3.0) * u4;
}

// One source interaction for one target.  KERN: -1 Newtonian, 0 Plummer,
// 1 spline.
//
// Scaled accumulation: with y0 = v_rsq_f64(s) and w = y0 * (3 - s*y0^2)
// (= 2*y1, y1 the Newton-refined 1/sqrt(s)), the kernel accumulates
//     ph += m*w        (= -2 * m * phi_unit)
//     a  += m*w^3 * d  (=  8 * m * g * d)
// and the epilogue multiplies by -1/2 and 1/8 (exact powers of two).  This
// shares m*w between potential and force and costs 10 FP64 ops after the
// rsq instead of 11.  Only overflow moves: m*w^3 overflows for r below
// ~1e-103 (the reference's m/r^3 a factor 8 later), i.e. for particles
// that are already coincident to ~1e-103.
template <int KERN, int WANT>
__device__ __forceinline__ void pair(double dx, double dy, double dz, double m, double h,
                                     double &ph, double &ax, double &ay, double &az) {
  // s2 = r^2 + R2_TINY (direct.rs:174,305; kernel variants use r = sqrt(s2))
  double s2 = __builtin_fma(dx, dx, __builtin_fma(dy, dy, __builtin_fma(dz, dz, kR2Tiny)));
  // Plummer: 1/sqrt(r^2 + h^2), 1/(r^2+h^2)^(3/2)  (kernel.rs:46,67-70)
  const double s = (KERN == 0) ? __builtin_fma(h, h, s2) : s2;
  const double y0 = __builtin_amdgcn_rsq(s);
  const double w = y0 * __builtin_fma(-s, y0 * y0, 3.0);
  double mw = m * w;
  double g8 = mw * (w * w);
  if (KERN == 1) {
    // spline (kernel.rs:47-54,71-80): inside the support replace the
    // Newtonian values, expressed in the same scaled units
    double r = s2 * (0.5 * w);
    if (h > 0.0 && r < h) {
      double hinv = 1.0 / h;
      double u = r * hinv;
      mw = -2.0 * m * (w2_inner(u) * hinv);
      g8 = 8.0 * m * (w2p_inner(u) * (hinv * hinv) / r);
    }
  }
  if (WANT & PBX_WANT_POT) ph += mw;
  if (WANT & PBX_WANT_ACC) {
    ax = __builtin_fma(g8, dx, ax);
    ay = __builtin_fma(g8, dy, ay);
    az = __builtin_fma(g8, dz, az);
  }
}

template <int KERN, int WANT, bool CHECK, int T>
__device__ __forceinline__ void sweep(const double4 *__restrict__ src,
                                      const double *__restrict__ src_h, bool has_h,
                                      int64_t j0, int64_t j1, const double (&xi)[T],
                                      const double (&yi)[T], const double (&zi)[T],
                                      const double (&hi)[T], const int64_t (&me)[T],
                                      double (&ph)[T], double (&ax)[T], double (&ay)[T],
                                      double (&az)[T]) {
#pragma unroll 4
  for (int64_t j = j0; j < j1; ++j) {
    const double4 s = src[j];
    double hj = 0.0;
    if (KERN >= 0) hj = has_h ? src_h[j] : 0.0;
#pragma unroll
    for (int k = 0; k < T; ++k) {
      double dx = s.x - xi[k];
      double dy = s.y - yi[k];
      double dz = s.z - zi[k];
      double m = s.w;
      if (CHECK) {
        // the self pair contributes nothing: zero mass and a unit distance
        // keep 0 * inf out of the force
        bool self = (j == me[k]);
        m = self ? 0.0 : m;
        dx = self ? 1.0 : dx;
      }
      double h = 0.0;
      if (KERN >= 0) h = __builtin_fmax(hi[k], hj);
      pair<KERN, WANT>(dx, dy, dz, m, h, ph[k], ax[k], ay[k], az[k]);
    }
  }
}

// Grid: x = target tiles of kBlock*T, y = source splits of `chunk` sources.
// Output: when out_split_stride == 0 the final arrays, else partial slabs
// indexed [blockIdx.y][target].
template <int KERN, int WANT, bool SELF, int T>
__global__ void __launch_bounds__(kBlock)
    direct_kernel(const double4 *__restrict__ src, const double *__restrict__ src_h,
                  int has_h, int64_t n_src, int64_t chunk, const double *__restrict__ tgt,
                  const double *__restrict__ tgt_h, int64_t n_tgt, int64_t self_offset,
                  double *__restrict__ pot_out, double *__restrict__ acc_out,
                  int64_t out_split_stride) {
  const int64_t tbase = (int64_t)blockIdx.x * (kBlock * T);
  const int64_t js = (int64_t)blockIdx.y * chunk;
  const int64_t je = (js + chunk < n_src) ? js + chunk : n_src;

  double xi[T], yi[T], zi[T], hi[T], ph[T], ax[T], ay[T], az[T];
  int64_t me[T];
#pragma unroll
  for (int k = 0; k < T; ++k) {
    int64_t t = tbase + k * kBlock + threadIdx.x;
    int64_t tc = t < n_tgt ? t : n_tgt - 1;
    xi[k] = tgt[3 * tc + 0];
    yi[k] = tgt[3 * tc + 1];
    zi[k] = tgt[3 * tc + 2];
    hi[k] = (SELF && KERN >= 0 && has_h) ? tgt_h[tc] : 0.0;
    me[k] = SELF ? self_offset + t : -1;
    ph[k] = ax[k] = ay[k] = az[k] = 0.0;
  }

  const bool hh = has_h != 0;
  if (SELF) {
    int64_t d0 = self_offset + tbase;
    int64_t d1 = d0 + kBlock * T;
    d0 = d0 < js ? js : (d0 > je ? je : d0);
    d1 = d1 < js ? js : (d1 > je ? je : d1);
    sweep<KERN, WANT, false, T>(src, src_h, hh, js, d0, xi, yi, zi, hi, me, ph, ax, ay, az);
    sweep<KERN, WANT, true, T>(src, src_h, hh, d0, d1, xi, yi, zi, hi, me, ph, ax, ay, az);
    sweep<KERN, WANT, false, T>(src, src_h, hh, d1, je, xi, yi, zi, hi, me, ph, ax, ay, az);
  } else {
    sweep<KERN, WANT, false, T>(src, src_h, hh, js, je, xi, yi, zi, hi, me, ph, ax, ay, az);
  }

  const int64_t soff = (int64_t)blockIdx.y * out_split_stride;
#pragma unroll
  for (int k = 0; k < T; ++k) {
    int64_t t = tbase + k * kBlock + threadIdx.x;
    if (t < n_tgt) {
      // undo the scaled accumulation of pair(): exact powers of two
      if (WANT & PBX_WANT_POT) pot_out[soff + t] = -0.5 * ph[k];
      if (WANT & PBX_WANT_ACC) {
        double *a = acc_out + 3 * (soff + t);
        a[0] = 0.125 * ax[k];
        a[1] = 0.125 * ay[k];
        a[2] = 0.125 * az[k];
      }
    }
  }
}

// Sum the source-split partial slabs in split order (deterministic).
template <int WANT>
__global__ void __launch_bounds__(kBlock)
    reduce_splits(const double *__restrict__ pot_part, const double *__restrict__ acc_part,
                  int nsplit, int64_t n_tgt, double *__restrict__ pot,
                  double *__restrict__ acc) {
  int64_t t = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if (t >= n_tgt) return;
  if (WANT & PBX_WANT_POT) {
    double s = 0.0;
    for (int k = 0; k < nsplit; ++k) s += pot_part[(int64_t)k * n_tgt + t];
    pot[t] = s;
  }
  if (WANT & PBX_WANT_ACC) {
    double sx = 0.0, sy = 0.0, sz = 0.0;
    for (int k = 0; k < nsplit; ++k) {
      const double *a = acc_part + 3 * ((int64_t)k * n_tgt + t);
      sx += a[0];
      sy += a[1];
      sz += a[2];
    }
    acc[3 * t + 0] = sx;
    acc[3 * t + 1] = sy;
    acc[3 * t + 2] = sz;
  }
}

__global__ void __launch_bounds__(kBlock)
    pack_sources_kernel(const double *__restrict__ pos, const double *__restrict__ mass,
                        int64_t n, double4 *__restrict__ rec) {
  int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if (i >= n) return;
  rec[i] = make_double4(pos[3 * i + 0], pos[3 * i + 1], pos[3 * i + 2],
                        mass ? mass[i] : 1.0);
}

// Targets per lane: 4 (measured +2 % over 2, +6 % over 1).
constexpr int kTargetsPerLane = 4;

template <int KERN, int WANT, bool SELF>
static void launch_variant(hipStream_t st, dim3 grid, const double4 *src, const double *src_h,
                           int has_h, int64_t n_src, int64_t chunk, const double *tgt,
                           const double *tgt_h, int64_t n_tgt, int64_t self_offset,
                           double *pot, double *acc, int64_t stride) {
  hipLaunchKernelGGL((direct_kernel<KERN, WANT, SELF, kTargetsPerLane>), grid, dim3(kBlock), 0,
                     st, src, src_h, has_h, n_src, chunk, tgt, tgt_h, n_tgt, self_offset, pot, acc,
                     stride);
}

template <int KERN, int WANT>
static void launch_self(bool self, hipStream_t st, dim3 grid, const double4 *src,
                        const double *src_h, int has_h, int64_t n_src, int64_t chunk,
                        const double *tgt, const double *tgt_h, int64_t n_tgt,
                        int64_t self_offset, double *pot, double *acc, int64_t stride) {
  if (self)
    launch_variant<KERN, WANT, true>(st, grid, src, src_h, has_h, n_src, chunk, tgt, tgt_h,
                                     n_tgt, self_offset, pot, acc, stride);
  else
    launch_variant<KERN, WANT, false>(st, grid, src, src_h, has_h, n_src, chunk, tgt, tgt_h,
                                      n_tgt, self_offset, pot, acc, stride);
}

template <int KERN>
static void launch_want(int want, bool self, hipStream_t st, dim3 grid, const double4 *src,
                        const double *src_h, int has_h, int64_t n_src, int64_t chunk,
                        const double *tgt, const double *tgt_h, int64_t n_tgt,
                        int64_t self_offset, double *pot, double *acc, int64_t stride) {
  switch (want) {
    case 1:
      launch_self<KERN, 1>(self, st, grid, src, src_h, has_h, n_src, chunk, tgt, tgt_h, n_tgt,
                           self_offset, pot, acc, stride);
      break;
    case 2:
      launch_self<KERN, 2>(self, st, grid, src, src_h, has_h, n_src, chunk, tgt, tgt_h, n_tgt,
                           self_offset, pot, acc, stride);
      break;
    default:
      launch_self<KERN, 3>(self, st, grid, src, src_h, has_h, n_src, chunk, tgt, tgt_h, n_tgt,
                           self_offset, pot, acc, stride);
      break;
  }
}

// direct_sym.hip
int64_t sym_padded(int64_t n);
int64_t sym_unit_count(int64_t n);
void sym_accumulate(Device &d, double4 *rec, int64_t n, int64_t u0, int64_t u1, int want,
                    double *acc4, DevBuf &unit_buf);
void sym_finish(Device &d, const double *acc4, int64_t lo, int64_t hi, int want, double *pot,
                double *acc);

// All-particles Newtonian sums of at least this many particles evaluate each
// unordered pair once (direct_sym.hip).
static constexpr int64_t kSymMinN = 8192;

// Launch the direct sum on device-resident data (all pointers device).
void direct_device(Device &d, const double *src, const double *src_h, int64_t n_src,
                   const double *tgt, const double *tgt_h, int64_t n_tgt, int64_t self_offset,
                   int kernel, int want, double *pot, double *acc) {
  if (n_tgt <= 0) return;
  hipStream_t st = d.stream;
  if (kernel == PBX_KERNEL_NONE && self_offset == 0 && n_tgt == n_src && n_src >= kSymMinN) {
    const int64_t npad = sym_padded(n_src);
    double4 *rec = (double4 *)d.slot(kSlotSymRec).ensure(sizeof(double4) * npad);
    double *acc4 = (double *)d.slot(kSlotSymAcc).ensure(sizeof(double) * 4 * npad);
    PBX_HIP(hipMemcpyAsync(rec, src, sizeof(double4) * n_src, hipMemcpyDeviceToDevice, st));
    PBX_HIP(hipMemsetAsync(acc4, 0, sizeof(double) * 4 * npad, st));
    sym_accumulate(d, rec, n_src, 0, sym_unit_count(n_src), want, acc4, d.slot(kSlotSymUnits));
    sym_finish(d, acc4, 0, n_src, want, pot, acc);
    return;
  }
  if (n_src <= 0) {
    if (want & PBX_WANT_POT) PBX_HIP(hipMemsetAsync(pot, 0, sizeof(double) * n_tgt, st));
    if (want & PBX_WANT_ACC) PBX_HIP(hipMemsetAsync(acc, 0, sizeof(double) * 3 * n_tgt, st));
    return;
  }
  const int64_t per_block = (int64_t)kBlock * kTargetsPerLane;
  const int64_t bx = (n_tgt + per_block - 1) / per_block;
  // Aim for >= 2048 blocks (8 per CU) but keep >= 4096 sources per split.
  int64_t nsplit = (2048 + bx - 1) / bx;
  int64_t max_split = (n_src + 4095) / 4096;
  if (nsplit > max_split) nsplit = max_split;
  if (nsplit > 64) nsplit = 64;
  if (nsplit < 1) nsplit = 1;
  const int64_t chunk = (n_src + nsplit - 1) / nsplit;
  nsplit = (n_src + chunk - 1) / chunk;
  if (bx > 0x7fffffff) fail(PBX_ERR_VALUE, "too many targets (%lld)", (long long)n_tgt);
  dim3 grid((unsigned)bx, (unsigned)nsplit);
  const bool self = self_offset >= 0;
  const int has_h = src_h != nullptr;

  double *pot_k = pot, *acc_k = acc;
  int64_t stride = 0;
  if (nsplit > 1) {
    size_t per = 0;
    if (want & PBX_WANT_POT) per += 1;
    if (want & PBX_WANT_ACC) per += 3;
    double *part = (double *)d.slot(kSlotPart).ensure(sizeof(double) * per * nsplit * n_tgt);
    pot_k = (want & PBX_WANT_POT) ? part : nullptr;
    acc_k = (want & PBX_WANT_ACC) ? part + ((want & PBX_WANT_POT) ? nsplit * n_tgt : 0)
                                  : nullptr;
    stride = n_tgt;
  }
  const double4 *src4 = (const double4 *)src;
  switch (kernel) {
    case PBX_KERNEL_NONE:
      launch_want<-1>(want, self, st, grid, src4, src_h, has_h, n_src, chunk, tgt, tgt_h,
                      n_tgt, self_offset, pot_k, acc_k, stride);
      break;
    case PBX_KERNEL_PLUMMER:
      launch_want<0>(want, self, st, grid, src4, src_h, has_h, n_src, chunk, tgt, tgt_h,
                     n_tgt, self_offset, pot_k, acc_k, stride);
      break;
    case PBX_KERNEL_SPLINE:
      launch_want<1>(want, self, st, grid, src4, src_h, has_h, n_src, chunk, tgt, tgt_h,
                     n_tgt, self_offset, pot_k, acc_k, stride);
      break;
    default:
      fail(PBX_ERR_VALUE, "kernel must be 0 (Plummer) or 1 (CubicSplineW2)");
  }
  PBX_HIP(hipGetLastError());
  if (nsplit > 1) {
    dim3 rg(ceil_div(n_tgt, kBlock));
    switch (want) {
      case 1:
        hipLaunchKernelGGL(reduce_splits<1>, rg, dim3(kBlock), 0, st, pot_k, acc_k,
                           (int)nsplit, n_tgt, pot, acc);
        break;
      case 2:
        hipLaunchKernelGGL(reduce_splits<2>, rg, dim3(kBlock), 0, st, pot_k, acc_k,
                           (int)nsplit, n_tgt, pot, acc);
        break;
      default:
        hipLaunchKernelGGL(reduce_splits<3>, rg, dim3(kBlock), 0, st, pot_k, acc_k,
                           (int)nsplit, n_tgt, pot, acc);
        break;
    }
    PBX_HIP(hipGetLastError());
  }
}

void pack_sources_device(Device &d, const double *pos, const double *mass, int64_t n,
                         double *rec) {
  if (n <= 0) return;
  hipLaunchKernelGGL(pack_sources_kernel, dim3(ceil_div(n, kBlock)), dim3(kBlock), 0, d.stream,
                     pos, mass, n, (double4 *)rec);
  PBX_HIP(hipGetLastError());
}

static void check_kernel(int kernel, const double *soft) {
  if (kernel != PBX_KERNEL_NONE && kernel != PBX_KERNEL_PLUMMER && kernel != PBX_KERNEL_SPLINE)
    fail(PBX_ERR_VALUE, "kernel must be 0 (Plummer) or 1 (CubicSplineW2)");
  if (kernel == PBX_KERNEL_NONE && soft != nullptr)
    fail(PBX_ERR_VALUE,
         "softenings require an explicit kernel; pass kernel=0/1 (or omit softenings)");
}

// Host-array entry: copy in, pack, run, copy out.
static void direct_host(const double *h_pos, int64_t n, const double *h_tgt, int64_t m,
                        const double *h_mass, const double *h_soft, int kernel, int want,
                        double *h_out) {
  if (n < 0 || m < 0) fail(PBX_ERR_VALUE, "negative particle count");
  check_kernel(kernel, h_soft);
  const bool self = (h_tgt == nullptr);
  const int64_t n_tgt = self ? n : m;
  if (n_tgt == 0) return;
  Device &d = current_device();
  std::lock_guard<std::mutex> lk(d.mu);
  hipStream_t st = d.stream;
  size_t out_elems = (want == PBX_WANT_POT ? 1 : 3) * (size_t)n_tgt;
  if (n == 0) {
    std::memset(h_out, 0, sizeof(double) * out_elems);
    return;
  }
  ScopedTimer total("pbx.direct.total");
  double *d_pos = (double *)d.slot(kSlotPos).ensure(sizeof(double) * 3 * n);
  double *d_mass = h_mass ? (double *)d.slot(kSlotMass).ensure(sizeof(double) * n) : nullptr;
  double *d_src = (double *)d.slot(kSlotSrc).ensure(sizeof(double) * 4 * n);
  const bool use_h = h_soft != nullptr && kernel != PBX_KERNEL_NONE;
  double *d_src_h = use_h ? (double *)d.slot(kSlotSrcH).ensure(sizeof(double) * n) : nullptr;
  double *d_tgt = self ? d_pos : (double *)d.slot(kSlotTgt).ensure(sizeof(double) * 3 * m);
  double *d_out = (double *)d.slot(want == PBX_WANT_POT ? kSlotPot : kSlotAcc)
                      .ensure(sizeof(double) * out_elems);
  {
    ScopedTimer t("pbx.direct.h2d");
    PBX_HIP(hipMemcpyAsync(d_pos, h_pos, sizeof(double) * 3 * n, hipMemcpyHostToDevice, st));
    if (h_mass)
      PBX_HIP(hipMemcpyAsync(d_mass, h_mass, sizeof(double) * n, hipMemcpyHostToDevice, st));
    if (use_h)
      PBX_HIP(hipMemcpyAsync(d_src_h, h_soft, sizeof(double) * n, hipMemcpyHostToDevice, st));
    if (!self)
      PBX_HIP(hipMemcpyAsync(d_tgt, h_tgt, sizeof(double) * 3 * m, hipMemcpyHostToDevice, st));
    if (timing_enabled()) PBX_HIP(hipStreamSynchronize(st));
  }
  {
    ScopedTimer t("pbx.direct.compute");
    pack_sources_device(d, d_pos, d_mass, n, d_src);
    direct_device(d, d_src, d_src_h, n, d_tgt, self ? d_src_h : nullptr, n_tgt,
                  self ? 0 : -1, kernel, want, want == PBX_WANT_POT ? d_out : nullptr,
                  want == PBX_WANT_ACC ? d_out : nullptr);
    if (timing_enabled()) PBX_HIP(hipStreamSynchronize(st));
  }
  {
    ScopedTimer t("pbx.direct.d2h");
    PBX_HIP(hipMemcpyAsync(h_out, d_out, sizeof(double) * out_elems, hipMemcpyDeviceToHost, st));
    PBX_HIP(hipStreamSynchronize(st));
  }
}

}  // namespace pbx

using namespace pbx;

extern "C" {

int pbx_direct_accelerations(const double *h_pos, int64_t n, const double *h_masses,
                             const double *h_softenings, int kernel, double *h_acc) {
  return guard([&] {
    direct_host(h_pos, n, nullptr, 0, h_masses, h_softenings, kernel, PBX_WANT_ACC, h_acc);
  });
}

int pbx_direct_potentials(const double *h_pos, int64_t n, const double *h_masses,
                          const double *h_softenings, int kernel, double *h_pot) {
  return guard([&] {
    direct_host(h_pos, n, nullptr, 0, h_masses, h_softenings, kernel, PBX_WANT_POT, h_pot);
  });
}

int pbx_direct_accelerations_at_points(const double *h_pos, int64_t n, const double *h_targets,
                                       int64_t m, const double *h_masses,
                                       const double *h_softenings, int kernel, double *h_acc) {
  return guard([&] {
    if (m > 0 && !h_targets) fail(PBX_ERR_VALUE, "targets must be (N,3) float64 array");
    direct_host(h_pos, n, h_targets ? h_targets : h_pos, m, h_masses, h_softenings, kernel,
                PBX_WANT_ACC, h_acc);
  });
}

int pbx_direct_potentials_at_points(const double *h_pos, int64_t n, const double *h_targets,
                                    int64_t m, const double *h_masses,
                                    const double *h_softenings, int kernel, double *h_pot) {
  return guard([&] {
    if (m > 0 && !h_targets) fail(PBX_ERR_VALUE, "targets must be (N,3) float64 array");
    direct_host(h_pos, n, h_targets ? h_targets : h_pos, m, h_masses, h_softenings, kernel,
                PBX_WANT_POT, h_pot);
  });
}

int pbx_pack_sources(const double *d_pos, const double *d_mass, int64_t n, double *d_records) {
  return guard([&] {
    if (n < 0) fail(PBX_ERR_VALUE, "negative particle count");
    Device &d = current_device();
    pack_sources_device(d, d_pos, d_mass, n, d_records);
  });
}

int pbx_direct_dev(const double *d_src, const double *d_src_h, int64_t n_src,
                   const double *d_tgt, const double *d_tgt_h, int64_t n_tgt,
                   int64_t self_offset, int kernel, int want, double *d_pot, double *d_acc) {
  return guard([&] {
    if (n_src < 0 || n_tgt < 0) fail(PBX_ERR_VALUE, "negative particle count");
    if (want < 1 || want > 3) fail(PBX_ERR_VALUE, "want must be 1 (pot), 2 (acc) or 3");
    if ((want & PBX_WANT_POT) && !d_pot && n_tgt) fail(PBX_ERR_VALUE, "d_pot is NULL");
    if ((want & PBX_WANT_ACC) && !d_acc && n_tgt) fail(PBX_ERR_VALUE, "d_acc is NULL");
    if (kernel != PBX_KERNEL_NONE && kernel != PBX_KERNEL_PLUMMER && kernel != PBX_KERNEL_SPLINE)
      fail(PBX_ERR_VALUE, "kernel must be 0 (Plummer) or 1 (CubicSplineW2)");
    if (self_offset >= 0 && self_offset + n_tgt > n_src)
      fail(PBX_ERR_VALUE, "self_offset + n_tgt exceeds n_src");
    if (self_offset >= 0 && kernel != PBX_KERNEL_NONE && d_src_h && !d_tgt_h)
      fail(PBX_ERR_VALUE, "all-particles softened form needs d_tgt_h");
    Device &d = current_device();
    std::lock_guard<std::mutex> lk(d.mu);
    direct_device(d, d_src, kernel == PBX_KERNEL_NONE ? nullptr : d_src_h, n_src, d_tgt,
                  d_tgt_h, n_tgt, self_offset, kernel, want, d_pot, d_acc);
  });
}

}  // extern "C"
