/*
 * pbx.h — C ABI of libpbx.so, the MI355X-native (gfx950, HIP) engine behind
 * the pynbodyext gravity and radial-profile hot path.
 *
 * Every entry point takes plain pointers and sizes (no framework types) and
 * returns an int status:
 *     PBX_OK          0  success
 *     PBX_ERR_VALUE   1  bad argument          -> Python ValueError
 *     PBX_ERR_RUNTIME 2  HIP / RCCL failure     -> Python RuntimeError
 *     PBX_ERR_NODEV   3  no usable gfx950 GPU   -> Python RuntimeError
 * and the message of the last failure on the calling thread is returned by
 * pbx_last_error().  Nothing here falls back to a CPU path: a missing GPU is
 * an error.
 *
 * The functions below replace the reference's PyO3 boundary module
 * `pynbodyext._rust` (crates/pynbodyext-rust/src/lib.rs:10-27) and the numpy
 * seams of pynbodyext.profiles (profiles/bins.py:346-395,
 * profiles/proarray.py:272-334).  Each block cites the reference interface
 * it replaces.  Host ("h_") pointers are pageable host memory owned by the
 * caller; device ("d_") pointers are HBM allocations (pbx_malloc) and are
 * only used by the device-resident API (bench, multi-GPU).
 */
#ifndef PBX_H
#define PBX_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define PBX_OK 0
#define PBX_ERR_VALUE 1
#define PBX_ERR_RUNTIME 2
#define PBX_ERR_NODEV 3

/* Softening kernel codes: the reference's Option<u8> kernel argument
 * (crates/pynbodyext-rust/src/gravity.rs:67-82).  PBX_KERNEL_NONE is the
 * Newtonian path taken when kernel is None (direct.rs:115-368). */
#define PBX_KERNEL_NONE (-1)
#define PBX_KERNEL_PLUMMER 0
#define PBX_KERNEL_SPLINE 1

/* want bitmask for the fused direct-sum entry */
#define PBX_WANT_POT 1
#define PBX_WANT_ACC 2

/* element types of pbx_profile_select_typed */
#define PBX_F64 0
#define PBX_F32 1

/* ------------------------------------------------------------------ */
/* runtime                                                             */
/* ------------------------------------------------------------------ */
const char *pbx_last_error(void);
int pbx_version(void);                   /* returns e.g. 100 for 0.1.0 */
int pbx_device_count(int *count);
int pbx_set_device(int device);          /* per calling thread */
int pbx_get_device(int *device);
/* Direct-sum precision (process-wide).  precise=1: every 1/sqrt is
 * v_rsq_f64 + one Newton step (~1e-16 relative, the reference's IEEE
 * 1.0/sqrt to rounding).  precise=0 (default; env PBX_PRECISE=1 flips it):
 * the all-particles Newtonian symmetric kernel (n >= 8192) uses v_rsq_f64
 * unrefined, ~5e-8 relative per pair, results within ~1e-7 of the reference
 * (contract 1e-5; direct.rs:165-180 / :296-308 replaced).  No equivalent in
 * the PyO3 module (gravity.rs:448-709). */
int pbx_set_precise(int on);
int pbx_get_precise(int *on);
int pbx_device_synchronize(void);
int pbx_device_name(char *buf, int buflen);

int pbx_malloc(void **d_ptr, size_t bytes);
int pbx_free(void *d_ptr);
int pbx_memcpy_htod(void *d_dst, const void *h_src, size_t bytes);
/* Host -> device copy rates of `bytes` (best of 3 after a warm-up, GB/s):
 * from pinned host memory (one DMA) and from pageable memory through the
 * library's pinned chunks (what a profile call on host arrays uses).  No
 * reference counterpart: the bench's bound for the user-facing profile. */
int pbx_measure_h2d(int64_t bytes, double *pinned_gbs, double *staged_gbs);
/* The current device's cache of engine buffers (profile / octree handles
 * take freed blocks instead of hipMalloc): out[0] cached bytes, out[1]
 * cached blocks, out[2] allocations served from the cache, out[3]
 * allocations that called hipMalloc.  pbx_device_pool_trim frees every
 * cached block (memory back to the device for other users).  No reference
 * counterpart (runtime). */
int pbx_device_pool_stats(int64_t *out);
int pbx_device_pool_trim(void);
int pbx_memcpy_dtoh(void *h_dst, const void *d_src, size_t bytes);
int pbx_memcpy_dtod(void *d_dst, const void *d_src, size_t bytes);
int pbx_memset(void *d_ptr, int value, size_t bytes);

/* Library-owned stream of the current device (all pbx kernels run on it)
 * and HIP events on that stream, so callers can time kernels live. */
int pbx_stream(void **stream);
int pbx_event_create(void **event);
int pbx_event_destroy(void *event);
int pbx_event_record(void *event);
int pbx_event_elapsed_ms(void *start, void *stop, float *ms);
int pbx_stream_synchronize(void);

/* ------------------------------------------------------------------ */
/* gravity: direct summation, host-array boundary                      */
/* ------------------------------------------------------------------ */
/* Replace the four PyO3 pyfunctions of crates/pynbodyext-rust/src/gravity.rs:
 *   direct_accelerations_py            (:448-512)
 *   direct_accelerations_at_points_py  (:514-583)
 *   direct_potentials_py               (:585-644)
 *   direct_potentials_at_points_py     (:646-709)
 * which call crates/gravity/src/direct.rs:115-658.
 * h_pos: n x 3 doubles, C order.  h_masses / h_softenings: n doubles or NULL
 * (NULL masses = unit masses, direct.rs:121-128).  kernel: PBX_KERNEL_*;
 * softenings with PBX_KERNEL_NONE is a PBX_ERR_VALUE with the reference's
 * message (gravity.rs:480-484).  Outputs are caller-allocated:
 * h_acc n x 3, h_pot n. */
int pbx_direct_accelerations(const double *h_pos, int64_t n,
                             const double *h_masses, const double *h_softenings,
                             int kernel, double *h_acc);
int pbx_direct_potentials(const double *h_pos, int64_t n,
                          const double *h_masses, const double *h_softenings,
                          int kernel, double *h_pot);
int pbx_direct_accelerations_at_points(const double *h_pos, int64_t n,
                                       const double *h_targets, int64_t m,
                                       const double *h_masses,
                                       const double *h_softenings, int kernel,
                                       double *h_acc);
int pbx_direct_potentials_at_points(const double *h_pos, int64_t n,
                                    const double *h_targets, int64_t m,
                                    const double *h_masses,
                                    const double *h_softenings, int kernel,
                                    double *h_pot);

/* ------------------------------------------------------------------ */
/* gravity: direct summation, device-resident API (bench / multi-GPU)  */
/* ------------------------------------------------------------------ */
/* Pack device arrays pos (n x 3) and mass (n, or NULL = unit masses) into
 * the 32-byte source records {x, y, z, m} the direct-sum kernel streams. */
int pbx_pack_sources(const double *d_pos, const double *d_mass, int64_t n,
                     double *d_records);
/* Fused direct sum over device-resident records.
 *   d_src      : n_src x 4 records {x,y,z,m}
 *   d_src_h    : n_src softenings or NULL (only read when kernel >= 0)
 *   d_tgt      : n_tgt x 3 target positions
 *   d_tgt_h    : n_tgt target softenings or NULL (all-particles softened
 *                form h = max(h_i, h_j), direct.rs:402,426)
 *   self_offset: >= 0 -> target t is source (self_offset + t) and that pair
 *                is skipped (all-particles form); -1 -> at-points form, no skip
 *   want       : PBX_WANT_POT | PBX_WANT_ACC
 *   d_pot      : n_tgt doubles, d_acc: n_tgt x 3 doubles (either may be NULL
 *                when not wanted) */
int pbx_direct_dev(const double *d_src, const double *d_src_h, int64_t n_src,
                   const double *d_tgt, const double *d_tgt_h, int64_t n_tgt,
                   int64_t self_offset, int kernel, int want, double *d_pot,
                   double *d_acc);

/* All-particles Newtonian direct sum with each unordered pair evaluated
 * once (Newton's third law; pbx_direct_dev and the host entry points use it
 * by themselves for n >= 8192), split into work units so that ranks can
 * share one solve: every rank runs its units into a per-particle
 * accumulator d_acc4 (npad x 4 doubles, zeroed by the caller), the ranks sum
 * the accumulators (pbx_comm_allreduce_f64), and each rank converts its own
 * particles [lo, hi) into potentials / accelerations.  h_weights (optional,
 * n_units) = relative cost of each unit, for balancing. */
int pbx_direct_sym_plan(int64_t n, int64_t *npad, int64_t *n_units, int64_t *h_weights);
int pbx_direct_sym_accumulate(const double *d_src, int64_t n, int64_t u0, int64_t u1, int want,
                              double *d_acc4);
int pbx_direct_sym_finish(const double *d_acc4, int64_t lo, int64_t hi, int want, double *d_pot,
                          double *d_acc);

/* ------------------------------------------------------------------ */
/* gravity: Barnes-Hut octree                                          */
/* ------------------------------------------------------------------ */
/* Replaces the PyO3 class `Octree` (crates/pynbodyext-rust/src/gravity.rs:
 * 114-445) over crates/gravity/src/tree.rs + multipole.rs.  The tree lives
 * in HBM behind an opaque handle; it reproduces the reference octree node
 * for node (root box, octants, split rule, payload order), so the opening
 * decisions of every target equal the reference's.
 * pos/masses/softenings/points/outputs are host arrays when on_device == 0,
 * device arrays when on_device == 1.  kernel: PBX_KERNEL_PLUMMER or
 * PBX_KERNEL_SPLINE (the PyO3 layer maps None to Plummer, gravity.rs:77-82).
 * want: PBX_WANT_POT | PBX_WANT_ACC. */
typedef struct pbx_octree pbx_octree;
/* Octree::new (gravity.rs:123-226): structure; mass payload iff masses */
int pbx_octree_create(const double *pos, int64_t n, const double *masses,
                      const double *softenings, int64_t leaf_capacity,
                      int multipole_order, int kernel, int on_device,
                      pbx_octree **out);
int pbx_octree_destroy(pbx_octree *tree);
/* Octree::new semantics on new particles (same leaf_capacity / order /
 * kernel), reusing the handle's HBM buffers (a time step of a simulation,
 * the next snapshot); mass payload iff masses */
int pbx_octree_rebuild(pbx_octree *tree, const double *pos, int64_t n, const double *masses,
                       const double *softenings, int on_device);
/* build_mass(masses=None) (gravity.rs:228-239): NULL keeps current masses */
int pbx_octree_build_mass(pbx_octree *tree, const double *masses, int on_device);
/* set_softenings (gravity.rs:241-258; h_max is not rebuilt, tree.rs:777) */
int pbx_octree_set_softenings(pbx_octree *tree, const double *softenings, int on_device);
/* set_kernel (gravity.rs:260-265) */
int pbx_octree_set_kernel(pbx_octree *tree, int kernel);
/* compute_potentials / compute_accelerations (gravity.rs:267-346,
 * tree.rs:1415-1496): every particle, self pair skipped, outputs in the
 * caller's particle order (pot n, acc n x 3) */
int pbx_octree_compute(pbx_octree *tree, double theta, int want, double *pot,
                       double *acc, int on_device);
/* potentials_at_points / accelerations_at_points (gravity.rs:348-445,
 * tree.rs:1498-1558): m query points (m x 3), no self skip */
int pbx_octree_at_points(pbx_octree *tree, const double *points, int64_t m,
                         double theta, int want, double *pot, double *acc,
                         int on_device);
/* One rank's shard of compute_*: the targets are the particles
 * [first, first + count) of the tree's leaf (DFS) order, self pairs skipped.
 * compact = 0: outputs at the particles' original indices (full-length
 * device arrays); compact = 1: count entries in leaf order.  d_cost
 * (optional, count int32): accepted nodes + leaf pairs per target, to
 * balance the next split.  Device pointers only. */
int pbx_octree_compute_range(pbx_octree *tree, double theta, int want, int64_t first,
                             int64_t count, int compact, double *d_pot, double *d_acc,
                             int32_t *d_cost);
/* positions (count x 3), masses and original indices (int64) of the leaf-order
 * particles [first, first + count), into device buffers (any may be NULL) */
int pbx_octree_leaf_particles(pbx_octree *tree, int64_t first, int64_t count, double *d_pos,
                              double *d_mass, int64_t *d_idx);
/* 3-D radial profile of a per-target field over the leaf-order targets
 * [first, first + count): d_f (device, count doubles in leaf order, e.g. the
 * potential of compute_range with compact = 1), nbins + 1 increasing host
 * edges; r = sqrt((x*x + y*y) + z*z) of the tree's own positions, bin as
 * BinsSet._assign_particles (bins.py:346-395).  Outputs (host): counts[nbins]
 * and moments[nbins][7] = {Σw, Σf·w, Σf²·w, Σf, Σf², Σ|f|·w, Σ|f|} with w =
 * the mass (pbx_profile_moments' columns, proarray.py:272-334).  Replaces
 * the select / assign / moments round trips of a tree's potential profile. */
int pbx_octree_radial_moments(pbx_octree *tree, int64_t first, int64_t count, const double *d_f,
                              const double *h_edges, int64_t nbins, int64_t *h_counts,
                              double *h_moments);
/* The same into DEVICE memory, no sync: d_out = nbins int64 counts followed
 * by nbins x 7 doubles (row-major), e.g. for an in-place all-reduce of the
 * ranks' partial profiles before one read-back. */
int pbx_octree_radial_moments_device(pbx_octree *tree, int64_t first, int64_t count,
                                     const double *d_f, const double *h_edges, int64_t nbins,
                                     void *d_out);
/* Multi-GPU load balance without an extra walk (the reference has one
 * process; its rayon pool splits targets dynamically, tree.rs:1443-1556):
 * cost_to_orig scatters per-target costs held in leaf order (n int32, e.g.
 * the d_cost of every rank's compute_range, all-gathered) to original
 * particle order; balance reads such costs through the CURRENT build's leaf
 * order and writes to host cuts[world + 1] the contiguous leaf-order ranges
 * [cuts[r], cuts[r+1]) of about equal summed max(cost, 1) — the split of
 * pynbodyext.parallel.balanced_ranges.  Device pointers; balance syncs. */
int pbx_octree_cost_to_orig(pbx_octree *tree, const int32_t *d_cost_leaf, int32_t *d_cost_orig);
int pbx_octree_balance(pbx_octree *tree, const int32_t *d_cost_orig, int world, int64_t *cuts);
/* What d_cost of compute_range holds: kind 0 (default) the target's accepted
 * nodes + leaf pairs; kind 1 its wave's work (the wave's node steps + its
 * 4-record leaf rounds, the same for the 64 targets of one wave), which is
 * what a walk's time follows — ShardedTree balances on it. */
int pbx_octree_set_cost_kind(pbx_octree *tree, int kind);
/* Walk statistics on (1, default) or off (0) for this tree's later walks of
 * order 3 with potential + acceleration, no softening, in fast mode (no
 * reference counterpart: instrumentation).  Off, pbx_octree_info reports zero
 * interaction and step counts for those walks; decisions and values are
 * unchanged. */
int pbx_octree_set_walk_counters(pbx_octree *tree, int enabled);
/* out[13] = {n, nodes, levels, has_mass_payload, has_hmax,
 *            accepted node interactions and leaf pairs of the last walk,
 *            path words, wave steps and active-lane steps of the last walk
 *            (SIMD efficiency = active / (64 * steps)), leaf wave steps,
 *            their active lanes, wave steps that descended} */
int pbx_octree_info(pbx_octree *tree, int64_t *out);
/* Node arrays for parity tests (any pointer may be NULL), node ids in the
 * device's breadth-first numbering:
 *   center nodes x 4 {cx, cy, cz, half}; com nodes x 4 {x, y, z, mass};
 *   hmax nodes; links nodes x 3 {first (-1 for a leaf), next, n_children};
 *   leaf nodes x 2 {start, count} into perm; perm n (leaf order -> index);
 *   moments nodes x ncoef(order) (order >= 2). */
int pbx_octree_export(pbx_octree *tree, double *center, double *com, double *hmax,
                      int64_t *links, int64_t *leaf, int64_t *perm, double *moments);

/* ------------------------------------------------------------------ */
/* radial profiles: binning + per-bin reduction                        */
/* ------------------------------------------------------------------ */
/* One opaque handle per profile holds the binned quantity x (and, after a
 * fused selection, the selection weights and original indices) in HBM.
 * Replaces, in pynbodyext/profiles:
 *   BinsSet._assign_particles        bins.py:346-395  (assign + csr)
 *   equal_number_bins_algorithm      bins.py:720-746  (edges_equaln)
 *   np.min / np.max in lin / log     bins.py:689-718  (minmax)
 *   ProfileArray._compute sums       proarray.py:272-334 (moments)
 * and the filter scope feeding it (Sphere & FamilyFilter + sim["r"],
 * filters/filt.py:42-86, profiles/spatial_profile.py:30-35) (select). */
int pbx_profile_create(void **handle);
int pbx_profile_destroy(void *handle);
/* x = host array of n doubles (the generic BinsSet path) */
int pbx_profile_set_x(void *handle, const double *h_x, int64_t n);
/* Fused selection: keep particle i when (no family ranges given, or
 * fam[2f] <= i < fam[2f+1] for some f < nfam) and (use_sphere == 0, or
 * ((x-cx)^2+(y-cy)^2)+(z-cz)^2 < sphere[3]) with sphere = {cx,cy,cz,R^2};
 * x = sqrt((x*x+y*y)+z*z) (ndim 3) or sqrt(x*x+y*y) (ndim 2), weights =
 * mass (or 1), kept in index order.  pos/mass are host (on_device = 0) or
 * device pointers (on_device = 1). */
int pbx_profile_select(void *handle, const double *pos, const double *mass, int64_t n,
                       int on_device, int use_sphere, const double *sphere,
                       const int64_t *fam, int nfam, int ndim, int64_t *n_kept);
/* The same for float32 snapshots without a host up-cast (pos_dtype /
 * mass_dtype PBX_F64 or PBX_F32).  numpy's dtype rules for a float32 pos
 * array: the Sphere distance against the float64 centre is evaluated in
 * double on the exactly widened coordinates; x = sim["r"] / sim["rxy"] of the
 * float32 array is float32 arithmetic ((x*x+y*y)+z*z, correctly rounded
 * sqrtf) and is held widened (exactly) as double; masses are widened. */
int pbx_profile_select_typed(void *handle, const void *pos, int pos_dtype, const void *mass,
                             int mass_dtype, int64_t n, int on_device, int use_sphere,
                             const double *sphere, const int64_t *fam, int nfam, int ndim,
                             int64_t *n_kept);
/* original indices (int64), x and weights of the selection (any may be NULL) */
int pbx_profile_get_selection(void *handle, int64_t *h_idx, double *h_x, double *h_w);
int pbx_profile_minmax(void *handle, double *mn, double *mx);
/* equaln edges into h_edges (capacity nbins + 1); *n_edges = nbins + 1, or
 * 2 for the reference's degenerate "< 2 values" case */
int pbx_profile_edges_equaln(void *handle, int64_t nbins, int has_min, double bin_min,
                             int has_max, double bin_max, double *h_edges,
                             int64_t *n_edges);
/* Distributed equaln (no reference counterpart — the
 * reference is single-process): the radix select of
 * pbx_profile_edges_equaln in stages.  Every rank: key_range (local
 * order-preserving u64 keys of x; (~0, 0) when empty) -> min/max over ranks
 * -> msel_begin(global range, same bounds on every rank; returns the level
 * count L) -> for level 0..L-1: msel_hist (this rank's digit histogram,
 * *count u32 at *d_hist on the device) -> sum *d_hist over ranks in place
 * (pbx_comm_allreduce, dtype u32) -> msel_resolve -> msel_edges (identical
 * on every rank; same results and errors as pbx_profile_edges_equaln on the
 * concatenated x).  nbins <= 1024. */
int pbx_profile_key_range(void *profile, uint64_t *kmin, uint64_t *kmax);
int pbx_profile_msel_begin(void *profile, int64_t nbins, int has_min, double bin_min, int has_max,
                           double bin_max, uint64_t kmin, uint64_t kmax, int *levels);
int pbx_profile_msel_hist(void *profile, int level, uint32_t **d_hist, int64_t *count);
int pbx_profile_msel_resolve(void *profile, int level);
int pbx_profile_msel_edges(void *profile, double *h_edges, int64_t *n_edges);
/* bin ids + counts (nb = n_edges - 1 int64) for ascending edges */
int pbx_profile_assign(void *handle, const double *h_edges, int64_t n_edges,
                       int64_t *h_counts, int64_t *n_valid);
/* CSR of the assignment (perm: n_valid int64, offsets: nb+1); NULL = skip */
int pbx_profile_csr(void *handle, int64_t *h_perm, int64_t *h_offsets);
/* per-bin sums h_out[nb][7] = {Σw, Σf·w, Σf²·w, Σf, Σf², Σ|f|·w, Σ|f|};
 * f_src / w_src: 0 = x, 1 = selection weights, 2 = host array (h_f / h_w,
 * n doubles in selection order), 3 = device array indexed by ORIGINAL
 * particle (gathered through the selection, e.g. a tree potential left in
 * HBM by pbx_octree_compute); w_src = -1: unweighted */
int pbx_profile_moments(void *handle, int f_src, const double *h_f, int w_src,
                        const double *h_w, double *h_out);
/* the same for the columns whose bit is set in cols (bit k = column k of
 * h_out; the others are 0): each statistic reads only some of the sums
 * (proarray.py:632-860 — Sum: Σf; weighted Mean: Σw, Σf·w; ...) */
int pbx_profile_moments_cols(void *handle, int f_src, const double *h_f, int w_src,
                             const double *h_w, uint32_t cols, double *h_out);
/* One equaln radial-profile pass after pbx_profile_select with a single host
 * round trip (bins.py:720-746 edges, :346-395 assignment, the CSR when
 * build_csr, and per-bin sums of n_stats <= 16 requests (f_src / w_src in
 * {0 x, 1 weights} / -1, column mask cols[k]) as h_moments[k][nb][7]).
 * Same results and errors as pbx_profile_edges_equaln + pbx_profile_assign
 * (+ pbx_profile_csr) + pbx_profile_moments_cols; *n_edges = nbins + 1 or 2
 * (the reference's degenerate case, then nb = 1).  nbins <= 1024. */
int pbx_profile_binned_equaln(void *handle, int64_t nbins, int has_min, double bin_min,
                              int has_max, double bin_max, int build_csr, int n_stats,
                              const int *f_src, const int *w_src, const uint32_t *cols,
                              double *h_edges, int64_t *n_edges, int64_t *h_counts,
                              int64_t *n_valid, double *h_moments);
/* pbx_profile_select + pbx_profile_binned_equaln with ONE host round trip
 * (the RadialProfileBuilder equaln path end to end: filters/filt.py:42-86,
 * bins.py:720-746 / :346-395, proarray.py:272-334 sums).  Same arguments,
 * results and errors as the two calls in sequence; *n_kept as
 * pbx_profile_select (also set when the binning then fails).
 * Lifetime: with on_device = 1 the selection is lazy — the weights of the
 * kept particles are read from the caller's `mass` device array by the
 * first later call on this handle that needs them (pbx_profile_moments*,
 * pbx_profile_get_selection with h_w, weighted percentiles) and held by the
 * handle from then on, so that array must stay allocated and unchanged
 * until that call (or the next selection).  The same holds for `pos`: a
 * repeated large (tiled) call that bins with the stored table
 * (pbx_profile_spec_stats) keeps no copy of x, and the first later call that
 * reads x (pbx_profile_get_selection with h_x, statistics or percentiles of
 * x, pbx_profile_edges_equaln / assign on this selection) recomputes it from
 * `pos`.  Host inputs (on_device = 0) are staged into the handle. */
int pbx_profile_radial_equaln(void *handle, const double *pos, const double *mass, int64_t n,
                              int on_device, int use_sphere, const double *sphere,
                              const int64_t *fam, int nfam, int ndim, int64_t nbins, int has_min,
                              double bin_min, int has_max, double bin_max, int build_csr,
                              int n_stats, const int *f_src, const int *w_src,
                              const uint32_t *cols, int64_t *n_kept, double *h_edges,
                              int64_t *n_edges, int64_t *h_counts, int64_t *n_valid,
                              double *h_moments);
/* pbx_profile_radial_equaln for one rank of a profile whose particles are
 * sharded over the ranks of `comm` (the reference is
 * single-process): pos / mass are this rank's particles, the edges are the
 * equaln order statistics of ALL ranks' kept x (identical on every rank),
 * h_counts / h_moments the global per-bin counts and sums, h_counts_local
 * (nbins, may be NULL) this rank's counts; *n_kept / *n_valid and the CSR
 * left in the handle are this rank's.  Every rank calls it with the same
 * nbins, window and statistics.  Device all-reduces between the kernels,
 * two host read-backs per call. */
int pbx_profile_radial_equaln_comm(void *comm, void *handle, const double *pos, const double *mass,
                                   int64_t n, int on_device, int use_sphere, const double *sphere,
                                   const int64_t *fam, int nfam, int ndim, int64_t nbins,
                                   int has_min, double bin_min, int has_max, double bin_max,
                                   int build_csr, int n_stats, const int *f_src, const int *w_src,
                                   const uint32_t *cols, int64_t *n_kept, double *h_edges,
                                   int64_t *n_edges, int64_t *h_counts, int64_t *h_counts_local,
                                   int64_t *n_valid, double *h_moments);
/* Telemetry of pbx_profile_radial_equaln on this handle (no reference
 * counterpart): out[3] = {calls run as the one-launch persistent kernel,
 * of those the calls discarded at a grid barrier and re-run by the
 * multi-kernel path (a silent ~2x slowdown if non-zero), calls that took
 * the multi-kernel path}. */
int pbx_profile_path_stats(void *handle, int64_t *out);
/* Telemetry of the one-launch calls (no reference counterpart): out[3] =
 * {one-launch calls, of those the calls whose level-0 digit histogram was
 * counted during the selection with the previous one-launch call's geometry
 * (every window key inside it: one grid barrier and the second count
 * skipped; the edges are the same either way), and the calls that found the
 * previous call's edges at their ranks (tried when the last two calls' edges
 * were identical: each edge's keys below / equal counted during the
 * selection; a hit skips the order-statistic phases and their barriers)}.
 * PBX_MONO_EDGE=0 disables the edge speculation. */
int pbx_profile_mono_stats(void *handle, int64_t *out);
/* Telemetry of the tiled (>= 1024 selection tiles) multi-kernel calls of
 * pbx_profile_radial_equaln on this handle (no reference counterpart):
 * out[2] = {tiled calls, of those the calls whose level-0 digit histogram
 * was counted by the selection kernel with the previous tiled call's digit
 * geometry (every window key inside it), so x was not read a second time}. */
int pbx_profile_level0_stats(void *handle, int64_t *out);
/* Telemetry of the speculative assignment of the tiled calls (no reference
 * counterpart): out[3] = {calls whose selection kernel also binned every key
 * with the bin table stored by an earlier call (launched when the previous
 * tiled call's level-0 digits of every rank matched that table), of those the
 * calls whose own digits matched it too, so the assignment pass (a second
 * read of x and the masses) was skipped, and of those the calls that also
 * binned the keys of edge-holding digits with the previous call's edges
 * (launched when the last two calls' edges were identical) and found every
 * edge at its rank: no deferred keys and no order-statistic finish}.  A
 * miss re-runs the assignment; results are identical either way.
 * A speculating call stores no x: it is rebuilt from the positions when a
 * later call reads it, so with on-device inputs the speculation runs only
 * after pbx_profile_set_source_stable(handle, 1) (host inputs are staged
 * into the handle and always qualify). */
int pbx_profile_spec_stats(void *handle, int64_t *out);
/* stable = 1: the caller's DEVICE positions (and masses) given to this
 * handle's radial_equaln calls stay alive and unchanged until the next
 * selection on the handle — a speculating call may then keep no copy of x
 * and rebuild it from them for a later reader (selection(x), statistics or
 * percentiles of x).  0 (default): on-device calls do not speculate, x is
 * stored (no lifetime contract on the positions beyond the call).  No
 * reference counterpart (numpy has no such hazard). */
int pbx_profile_set_source_stable(void *handle, int stable);
/* enabled = 0: this handle's tiled calls never use a level-0 digit
 * geometry they did not derive themselves (every call re-reads x for its
 * level-0 histogram); 1 (default): use the previous call's when it holds,
 * and on a first call one from a sample of the keys (sample_hint); 2:
 * forget the earlier calls (geometries, speculation state) — the next call
 * runs as a handle's first.  Results are identical in every mode. */
int pbx_profile_set_level0_hint(void *handle, int enabled);
/* Per-bin percentiles of the last assignment — replaces the per-bin loop of
 * ProfileArray._compute for Percentile / Median / Abs_pXX
 * (proarray.py:272-334 + :689-722): h_out[bin*nq + k] = np.interp(q[k],
 * cdf, sorted field) with cdf = (cumsum(w[order]) - c0) / (c_last - c0)
 * (np.cumsum order and rounding) or np.linspace(0, 1, m) when w_src = -1;
 * empty bins NaN.  f_src / w_src as above; absval: statistic of |f|;
 * q[k] = p/100, 1 <= nq <= 4096. */
int pbx_profile_percentiles(void *handle, int f_src, const double *h_f, int w_src,
                            const double *h_w, int absval, int nq, const double *q,
                            double *h_out);

/* ------------------------------------------------------------------ */
/* multi-GPU: RCCL communicator (one process per GPU, over xGMI)       */
/* ------------------------------------------------------------------ */
/* No reference counterpart: the reference is single-process (rayon
 * threads).  North-star multi-GPU design: targets are
 * sharded across ranks, source records are all-gathered, profile partials
 * are all-reduced.  The unique id (pbx_comm_unique_id_size() bytes) is
 * created on rank 0 and distributed by the caller's control plane. */
int pbx_comm_unique_id_size(void);
int pbx_comm_unique_id(unsigned char *buf, int buflen);
int pbx_comm_init(void **comm, int nranks, int rank, const unsigned char *uid);
int pbx_comm_destroy(void *comm);
/* In-place all-gather-v of byte segments: segment r is
 * [displs[r], displs[r]+counts[r]) of d_buf, this rank's already in place. */
int pbx_comm_allgatherv(void *comm, void *d_buf, const int64_t *counts,
                        const int64_t *displs);
int pbx_comm_allreduce_f64(void *comm, const double *d_send, double *d_recv,
                           int64_t count);
/* generic: dtype 0 f64, 1 i64, 2 u64, 3 u32; op 0 sum, 1 min, 2 max */
int pbx_comm_allreduce(void *comm, const void *d_send, void *d_recv, int64_t count, int dtype,
                       int op);
int pbx_comm_allreduce_i64(void *comm, const int64_t *d_send, int64_t *d_recv,
                           int64_t count);
/* all-reduce of a small HOST array in place (dtype / op as above) through
 * the communicator's persistent device + pinned staging: no allocation per
 * call, one stream sync (the profile partials of ShardedProfile) */
int pbx_comm_allreduce_host(void *comm, void *h_buf, int64_t count, int dtype, int op);
/* Control plane on the same communicator: device barrier (returns after
 * every rank reached it and the stream drained) and max over ranks of a
 * host double. */
int pbx_comm_barrier(void *comm);
int pbx_comm_max_f64(void *comm, double value, double *out);

/* A communicator whose collectives go through a caller-supplied HOST
 * transport instead of RCCL (no reference counterpart).  Every collective
 * of the library — the pbx_comm_* calls above and the all-reduces inside
 * pbx_profile_radial_equaln_comm — stages its device bytes through pinned
 * host memory (D2H, stream sync), calls `fn`, and copies the result back.
 * fn(ctx, kind, h_buf, count, dtype, op, counts, displs) returns 0 on
 * success:
 *   kind PBX_COLL_ALLREDUCE: reduce `count` elements of `dtype` (codes as
 *     pbx_comm_allreduce) with `op` over the ranks, in place in h_buf;
 *   kind PBX_COLL_ALLGATHERV: h_buf holds the whole byte buffer with this
 *     rank's segment [displs[rank], +counts[rank]) in place; fill in the
 *     others (count = nranks).
 * While fn runs, a library call that issued the collective has released
 * the device lock, so the ranks of one process may be threads sharing one
 * device (the one-GPU multi-rank tests) — or processes on a host transport
 * (MPI, shared memory) where RCCL is unavailable. */
#define PBX_COLL_ALLREDUCE 0
#define PBX_COLL_ALLGATHERV 1
typedef int (*pbx_host_collective_fn)(void *ctx, int kind, void *h_buf, int64_t count, int dtype,
                                      int op, const int64_t *counts, const int64_t *displs);
int pbx_comm_init_host(void **comm, int nranks, int rank, pbx_host_collective_fn fn, void *ctx);

#ifdef __cplusplus
}
#endif
#endif /* PBX_H */
