// direct_sym.hip — all-particles Newtonian direct sum with every UNORDERED
// pair evaluated once (Newton's third law) on gfx950.
//
// Same result as direct.rs:115-185 / :255-313 (potential and acceleration
// of every particle from all others, self pair skipped), for the bench /
// multi-GPU path and the host entry points at N >= kSymMinN.  The per-pair
// arithmetic is the scaled form of direct.hip (w = 2/r refined from
// v_rsq_f64; potential and force accumulate m w and m w^3 d; the epilogue
// multiplies by -1/2 and 1/8) and is shared by both particles of a pair:
// 21 FP64 instructions + 1 rsq per unordered pair instead of 2 x (16 + 1).
// Fast mode (the default, pbx_set_precise(0)) skips the Newton step: w is
// v_rsq_f64 itself (1/r to ~5e-8 relative, measured), 18 FP64 instructions
// per pair, results within ~1e-7 of the reference (contract: 1e-5).
//
// Decomposition: particles padded to a multiple of 4 x 64 kT (pads: zero
// mass, far away, distinct).  I-block = 64 kT targets of one wave (kT per
// lane), J-chunk = 64 kS sources.  A workgroup (4 waves) owns a superblock
// of 4 consecutive I-blocks and walks a range of J-chunks; for each J-chunk a
// wave evaluates the I-block x J-chunk pairs with its targets in registers
// while the
// chunk's sources — and their accumulators — rotate one lane per step around
// the wave (by DPP wave_rol:1 on the VALU; the LDS crossbar, ds_bpermute,
// is the alternative PBX_SYM_DPP_MASK selects): after 64 steps every source
// met every target, so neither side needs a cross-lane reduction.  Chunk
// j past block b: both sides accumulate; b's own chunks: target side only (each
// ordered pair exactly once, self pair masked); chunks before b: skipped (done by the
// other block).  The source side of the 4 waves is summed in LDS and added
// to a per-particle accumulator with coalesced f64 atomics; the target side
// is added once per work unit.  Atomic bytes ~ 16 N^2 / 1024 (3 % of the
// runtime at 1M).  Float atomics make the last bits depend on arrival order.
#include <algorithm>
#include <type_traits>
#include <vector>

#include "pbx_common.h"

namespace pbx {
namespace sym {

static constexpr double kR2Tiny = 2.2250738585072014e-308;  // direct.rs:7
constexpr int kWaves = 4;
// 12 targets x 2 source slots per lane (254 VGPRs, no scratch: 2 waves per
// SIMD): a slot's rotation serves 12 pairs — 20.0 VALU issues per unordered
// pair; 8 x 4 took 20.5, 10 x 2 20.2, 6 x 2 (158 VGPRs, 3 waves) 21.0 —
// same box 337.4 / 332.0 / 338.5 against 331.1 ms (profiles/r6/r6y/)
#ifndef PBX_SYM_KT
#define PBX_SYM_KT 12
#endif
#ifndef PBX_SYM_KS
#define PBX_SYM_KS 2
#endif
constexpr int kT = PBX_SYM_KT;         // targets per lane
constexpr int kS = PBX_SYM_KS;         // source slots per lane
constexpr int kBlk = 64 * kT;          // targets per I-block (one wave)
constexpr int kChunk = 64 * kS;        // sources per J-chunk
constexpr int kJPerI = kBlk / kChunk;  // J-chunks per I-block
constexpr int kSuper = kWaves * kBlk;  // particles per superblock (workgroup)
static_assert(kJPerI * kChunk == kBlk, "an I-block is a whole number of J-chunks");

struct Unit {
  int32_t sb;  // superblock
  int32_t j0;  // first J-chunk
  int32_t j1;  // one past the last J-chunk
  int32_t pad;
};

__device__ __forceinline__ double rot(double v, int addr) {
  const uint64_t b = __builtin_bit_cast(uint64_t, v);
  const int lo = __builtin_amdgcn_ds_bpermute(addr, (int)(uint32_t)b);
  const int hi = __builtin_amdgcn_ds_bpermute(addr, (int)(uint32_t)(b >> 32));
  return __builtin_bit_cast(double, ((uint64_t)(uint32_t)hi << 32) | (uint64_t)(uint32_t)lo);
}

// the same rotation on the VALU: DPP wave_rol:1 (lane l takes lane l + 1's
// value, lane 63 lane 0's), no LDS operation / lgkmcnt slot
__device__ __forceinline__ double rot_dpp(double v) {
  const uint64_t b = __builtin_bit_cast(uint64_t, v);
  // (old = the source itself: every lane receives a value, and the
  // rotated word may then reuse the source's register — no v_mov of 0 and
  // no copy back into the loop-carried register)
  const int l0 = (int)(uint32_t)b, h0 = (int)(uint32_t)(b >> 32);
  const int lo = __builtin_amdgcn_update_dpp(l0, l0, 0x134, 0xF, 0xF, false);
  const int hi = __builtin_amdgcn_update_dpp(h0, h0, 0x134, 0xF, 0xF, false);
  return __builtin_bit_cast(double, ((uint64_t)(uint32_t)hi << 32) | (uint64_t)(uint32_t)lo);
}
// Which of a slot's eight rotated values go through DPP (bits: sx sy sz sm
// sp sa sb sc) instead of the LDS crossbar.  A slot's 16 ds_bpermute per
// step exceed the 15 LDS operations a wave may have in flight (lgkmcnt):
// the waves waited on LDS 22 % of their cycles (SQ_WAIT_INST_LDS).  Moving
// some rotations to the VALU (v_mov_b32_dpp wave_rol:1) trades VALU issue
// for LDS slots.  Same-box A/B at 1M (`profiles/r3/sym_dpp_ab/`): all LDS
// 376-377 ms; with the DPP result written in place (old = source) sx, sy
// 348, the four source values 339, those and sp, sa 333-343 (the best on
// two boxes), everything 334; before in-place DPP every rotated word cost
// a v_mov of 0 and a copy back (sx, sy: 358 ms).  Round 6, 12 pairs per
// slot rotation (profiles/r6/r6z/): everything on DPP 328.8-329.0 ms,
// 0x3F 331.0-331.7, 0x0F 333.6-334.5, all on the crossbar 340.0-340.6.
#ifndef PBX_SYM_DPP_MASK
#define PBX_SYM_DPP_MASK 0xFF
#endif

// One J-chunk for one wave.  SYMM: both sides; else chunk DOFF of the
// wave's own I-block (target side only, self pair masked at rotation 0:
// source slot ks of that chunk is target kt = DOFF * kS + ks).
template <int WANT, bool SYMM, bool RAW, int DOFF = 0>
__device__ __forceinline__ void chunk(const double4 *__restrict__ rec, int64_t jbase, int lane,
                                      const double (&tx)[kT], const double (&ty)[kT],
                                      const double (&tz)[kT], const double (&tm)[kT],
                                      double (&tp)[kT], double (&ta)[kT], double (&tb)[kT],
                                      double (&tc)[kT], double (&sp)[kS], double (&sa)[kS],
                                      double (&sb)[kS], double (&sc)[kS]) {
  double sx[kS], sy[kS], sz[kS], sm[kS];
#pragma unroll
  for (int k = 0; k < kS; ++k) {
    const double4 r = rec[jbase + k * 64 + lane];
    sx[k] = r.x;
    sy[k] = r.y;
    sz[k] = r.z;
    sm[k] = r.w;
    sp[k] = sa[k] = sb[k] = sc[k] = 0.0;
  }
  const int addr = ((lane + 1) & 63) << 2;  // rotate: take the next lane's sources
  for (int r = 0; r < 64; ++r) {
#pragma unroll
    for (int ks = 0; ks < kS; ++ks) {
#pragma unroll
      for (int kt = 0; kt < kT; ++kt) {
        double dx = sx[ks] - tx[kt], dy = sy[ks] - ty[kt], dz = sz[ks] - tz[kt];
        double ms = sm[ks];
        if (!SYMM && kt == DOFF * kS + ks) {
          const bool self = (r == 0);
          ms = self ? 0.0 : ms;
          dx = self ? 1.0 : dx;
        }
        const double s2 =
            __builtin_fma(dx, dx, __builtin_fma(dy, dy, __builtin_fma(dz, dz, kR2Tiny)));
        const double y0 = __builtin_amdgcn_rsq(s2);
        // precise: one Newton step, w = 2/r (~1e-16); fast: w = v_rsq_f64 =
        // 1/r to ~5e-8 relative (3 FP64 instructions fewer per pair)
        const double w = RAW ? y0 : y0 * __builtin_fma(-s2, y0 * y0, 3.0);
        const double q = w * (w * w);  // w^3
        if (WANT & PBX_WANT_POT) tp[kt] = __builtin_fma(ms, w, tp[kt]);
        if (WANT & PBX_WANT_ACC) {
          const double g = ms * q;
          ta[kt] = __builtin_fma(g, dx, ta[kt]);
          tb[kt] = __builtin_fma(g, dy, tb[kt]);
          tc[kt] = __builtin_fma(g, dz, tc[kt]);
        }
        if (SYMM) {
          if (WANT & PBX_WANT_POT) sp[ks] = __builtin_fma(tm[kt], w, sp[ks]);
          if (WANT & PBX_WANT_ACC) {
            const double g = tm[kt] * q;
            sa[ks] = __builtin_fma(-g, dx, sa[ks]);
            sb[ks] = __builtin_fma(-g, dy, sb[ks]);
            sc[ks] = __builtin_fma(-g, dz, sc[ks]);
          }
        }
      }
      // pass this slot on as soon as its pairs are done: the LDS-crossbar
      // round trip overlaps the next slot's arithmetic
      auto rt = [&](double x, int bit) {
        return ((PBX_SYM_DPP_MASK >> bit) & 1) ? rot_dpp(x) : rot(x, addr);
      };
      sx[ks] = rt(sx[ks], 0);
      sy[ks] = rt(sy[ks], 1);
      sz[ks] = rt(sz[ks], 2);
      sm[ks] = rt(sm[ks], 3);
      if (SYMM) {
        if (WANT & PBX_WANT_POT) sp[ks] = rt(sp[ks], 4);
        if (WANT & PBX_WANT_ACC) {
          sa[ks] = rt(sa[ks], 5);
          sb[ks] = rt(sb[ks], 6);
          sc[ks] = rt(sc[ks], 7);
        }
      }
    }
  }
}

// chunk d of the wave's own I-block (d < kJPerI, a compile-time DOFF each)
template <int WANT, bool RAW, int D>
__device__ __forceinline__ void own_chunk(int d, const double4 *__restrict__ rec, int64_t jbase,
                                          int lane, const double (&tx)[kT], const double (&ty)[kT],
                                          const double (&tz)[kT], const double (&tm)[kT],
                                          double (&tp)[kT], double (&ta)[kT], double (&tb)[kT],
                                          double (&tc)[kT], double (&sp)[kS], double (&sa)[kS],
                                          double (&sb)[kS], double (&sc)[kS]) {
  if (d == D)
    chunk<WANT, false, RAW, D>(rec, jbase, lane, tx, ty, tz, tm, tp, ta, tb, tc, sp, sa, sb, sc);
  else if constexpr (D + 1 < kJPerI)
    own_chunk<WANT, RAW, D + 1>(d, rec, jbase, lane, tx, ty, tz, tm, tp, ta, tb, tc, sp, sa, sb, sc);
}

template <int WANT, bool RAW>
__global__ void __launch_bounds__(kWaves * 64)
    sym_kernel(const double4 *__restrict__ rec, const Unit *__restrict__ units,
               double *__restrict__ acc4) {
  __shared__ double jl[kWaves][4][kChunk];  // source-side partials of one chunk, per wave
  const Unit u = units[blockIdx.x];
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int64_t iblk = (int64_t)u.sb * kWaves + w;
  double tx[kT], ty[kT], tz[kT], tm[kT], tp[kT], ta[kT], tb[kT], tc[kT];
#pragma unroll
  for (int k = 0; k < kT; ++k) {
    const double4 r = rec[iblk * kBlk + k * 64 + lane];
    tx[k] = r.x;
    ty[k] = r.y;
    tz[k] = r.z;
    tm[k] = r.w;
    tp[k] = ta[k] = tb[k] = tc[k] = 0.0;
  }
  const int64_t jdiag = iblk * kJPerI;  // this wave's first own chunk
  for (int32_t j = u.j0; j < u.j1; ++j) {
    double sp[kS], sa[kS], sb[kS], sc[kS];
#pragma unroll
    for (int k = 0; k < kS; ++k) sp[k] = sa[k] = sb[k] = sc[k] = 0.0;
    if (j >= jdiag + kJPerI)
      chunk<WANT, true, RAW>(rec, (int64_t)j * kChunk, lane, tx, ty, tz, tm, tp, ta, tb, tc, sp, sa,
                             sb, sc);
    else if (j >= jdiag)  // one of the wave's own chunks (target side, self pair masked)
      own_chunk<WANT, RAW, 0>((int)(j - jdiag), rec, (int64_t)j * kChunk, lane, tx, ty, tz, tm, tp,
                              ta, tb, tc, sp, sa, sb, sc);
#pragma unroll
    for (int k = 0; k < kS; ++k) {
      jl[w][0][k * 64 + lane] = sp[k];
      jl[w][1][k * 64 + lane] = sa[k];
      jl[w][2][k * 64 + lane] = sb[k];
      jl[w][3][k * 64 + lane] = sc[k];
    }
    __syncthreads();
    // chunk j has source-side partials only past the superblock's first I-block
    if ((int64_t)j >= ((int64_t)u.sb * kWaves + 1) * kJPerI) {
      double *dst = acc4 + (int64_t)j * kChunk * 4;
      static_assert(kWaves * 64 * kS == kChunk * 4, "kS (source, quantity) words per thread");
#pragma unroll
      for (int i = 0; i < kS; ++i) {
        const int idx = threadIdx.x + i * kWaves * 64;  // 0 .. 1023 = (source, quantity)
        const int s = idx >> 2, q = idx & 3;
        const double v = jl[0][q][s] + jl[1][q][s] + jl[2][q][s] + jl[3][q][s];
        if (v != 0.0) atomicAdd(dst + idx, v);
      }
    }
    __syncthreads();
  }
#pragma unroll
  for (int k = 0; k < kT; ++k) {
    double *dst = acc4 + (iblk * kBlk + k * 64 + lane) * 4;
    if (WANT & PBX_WANT_POT) atomicAdd(dst + 0, tp[k]);
    if (WANT & PBX_WANT_ACC) {
      atomicAdd(dst + 1, ta[k]);
      atomicAdd(dst + 2, tb[k]);
      atomicAdd(dst + 3, tc[k]);
    }
  }
}

// records of n particles + pads up to npad (zero mass, far apart)
__global__ void pad_records(double4 *__restrict__ rec, int64_t n, int64_t npad) {
  int64_t i = n + (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= npad) return;
  const double far = 1e30 * (double)(i - n + 1);
  rec[i] = make_double4(far, -far, 2.0 * far, 0.0);
}

// undo the scaled accumulation: particles [lo, hi) -> outputs
__global__ void finish_kernel(const double *__restrict__ acc4, int64_t lo, int64_t hi, int want,
                              int raw, double *__restrict__ pot, double *__restrict__ acc) {
  int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (lo + t >= hi) return;
  const double *a = acc4 + (lo + t) * 4;
  const double kp = raw ? -1.0 : -0.5, ka = raw ? 1.0 : 0.125;  // undo the w scale
  if (want & PBX_WANT_POT) pot[t] = kp * a[0];
  if (want & PBX_WANT_ACC) {
    acc[3 * t + 0] = ka * a[1];
    acc[3 * t + 1] = ka * a[2];
    acc[3 * t + 2] = ka * a[3];
  }
}

}  // namespace sym

// ------------------------------------------------------------------ host
int64_t sym_padded(int64_t n) {
  return (n + sym::kSuper - 1) / sym::kSuper * sym::kSuper;
}

// Work units over the upper triangle of (superblock, J-chunk): superblock sb
// covers chunks [kWaves kJPerI sb, nchunks) split into pieces of at most
// kChunksPerUnit.
#ifndef PBX_SYM_CHUNKS_PER_UNIT
#define PBX_SYM_CHUNKS_PER_UNIT 32
#endif
static std::vector<sym::Unit> sym_units(int64_t npad) {
  constexpr int kChunksPerUnit = PBX_SYM_CHUNKS_PER_UNIT;
  const int32_t nch = (int32_t)(npad / sym::kChunk);
  const int32_t nsb = (int32_t)(npad / sym::kSuper);
  std::vector<sym::Unit> u;
  for (int32_t sb = 0; sb < nsb; ++sb)
    for (int32_t j = sb * sym::kWaves * sym::kJPerI; j < nch; j += kChunksPerUnit)
      u.push_back({sb, j, std::min(nch, j + kChunksPerUnit), 0});
  return u;
}

int64_t sym_unit_count(int64_t n) { return (int64_t)sym_units(sym_padded(n)).size(); }



// Units [u0, u1) of the (padded) record array into acc4 (npad x 4, caller
// zeroes it).  rec must hold npad records; pads are written here.
void sym_accumulate(Device &d, double4 *rec, int64_t n, int64_t u0, int64_t u1, int want,
                    double *acc4, DevBuf &unit_buf) {
  const int64_t npad = sym_padded(n);
  hipStream_t st = d.stream;
  if (npad > n)
    hipLaunchKernelGGL(sym::pad_records, dim3(ceil_div(npad - n, 256)), dim3(256), 0, st, rec, n,
                       npad);
  std::vector<sym::Unit> all = sym_units(npad);
  u0 = std::max<int64_t>(0, u0);
  u1 = std::min<int64_t>((int64_t)all.size(), u1);
  if (u1 <= u0) return;
  // heaviest units first: fuller pieces start the grid, the diagonal pieces fill the tail
  std::vector<sym::Unit> mine(all.begin() + u0, all.begin() + u1);
  std::stable_sort(mine.begin(), mine.end(), [](const sym::Unit &a, const sym::Unit &b) {
    return (a.j1 - a.j0) > (b.j1 - b.j0);
  });
  sym::Unit *du = (sym::Unit *)unit_buf.ensure(sizeof(sym::Unit) * mine.size());
  PBX_HIP(hipMemcpyAsync(du, mine.data(), sizeof(sym::Unit) * mine.size(), hipMemcpyHostToDevice,
                         st));
  const dim3 grid((unsigned)mine.size()), block(sym::kWaves * 64);
  auto launch = [&](auto raw) {
    constexpr bool R = decltype(raw)::value;
    if (want == PBX_WANT_POT)
      hipLaunchKernelGGL((sym::sym_kernel<PBX_WANT_POT, R>), grid, block, 0, st, rec, du, acc4);
    else if (want == PBX_WANT_ACC)
      hipLaunchKernelGGL((sym::sym_kernel<PBX_WANT_ACC, R>), grid, block, 0, st, rec, du, acc4);
    else
      hipLaunchKernelGGL((sym::sym_kernel<PBX_WANT_POT | PBX_WANT_ACC, R>), grid, block, 0, st,
                         rec, du, acc4);
  };
  if (precise_mode())
    launch(std::false_type{});
  else
    launch(std::true_type{});
  PBX_HIP(hipGetLastError());
  // the unit table must outlive the launch before the host buffer goes away
  PBX_HIP(hipStreamSynchronize(st));
}

void sym_finish(Device &d, const double *acc4, int64_t lo, int64_t hi, int want, double *pot,
                double *acc) {
  if (hi <= lo) return;
  hipLaunchKernelGGL(sym::finish_kernel, dim3(ceil_div(hi - lo, 256)), dim3(256), 0, d.stream,
                     acc4, lo, hi, want, precise_mode() ? 0 : 1, pot, acc);
  PBX_HIP(hipGetLastError());
}

}  // namespace pbx

using namespace pbx;

extern "C" {

int pbx_direct_sym_plan(int64_t n, int64_t *npad, int64_t *n_units, int64_t *h_weights) {
  return guard([&] {
    if (n < 0) fail(PBX_ERR_VALUE, "negative particle count");
    const int64_t np = sym_padded(n);
    std::vector<sym::Unit> u = sym_units(np);
    if (npad) *npad = np;
    if (n_units) *n_units = (int64_t)u.size();
    if (h_weights)
      for (size_t i = 0; i < u.size(); ++i) h_weights[i] = u[i].j1 - u[i].j0;
  });
}

int pbx_direct_sym_accumulate(const double *d_src, int64_t n, int64_t u0, int64_t u1, int want,
                              double *d_acc4) {
  return guard([&] {
    if (n < 0) fail(PBX_ERR_VALUE, "negative particle count");
    if (want < 1 || want > 3) fail(PBX_ERR_VALUE, "want must be 1 (pot), 2 (acc) or 3");
    if (n == 0) return;
    Device &d = current_device();
    std::lock_guard<std::mutex> lk(d.mu);
    const int64_t npad = sym_padded(n);
    double4 *rec = (double4 *)d.slot(kSlotSymRec).ensure(sizeof(double4) * npad);
    PBX_HIP(hipMemcpyAsync(rec, d_src, sizeof(double4) * n, hipMemcpyDeviceToDevice, d.stream));
    sym_accumulate(d, rec, n, u0, u1, want, d_acc4, d.slot(kSlotSymUnits));
  });
}

int pbx_direct_sym_finish(const double *d_acc4, int64_t lo, int64_t hi, int want, double *d_pot,
                          double *d_acc) {
  return guard([&] {
    if (lo < 0 || hi < lo) fail(PBX_ERR_VALUE, "bad particle range");
    Device &d = current_device();
    std::lock_guard<std::mutex> lk(d.mu);
    sym_finish(d, d_acc4, lo, hi, want, d_pot, d_acc);
    PBX_HIP(hipStreamSynchronize(d.stream));
  });
}

}  // extern "C"
