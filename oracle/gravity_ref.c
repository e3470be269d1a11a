/*
 * gravity_ref.c — ORACLE (test infrastructure only; never shipped, never the
 * measured path).  Only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg may load it.
 *
 * A plain-C restatement of the reference's direct-summation gravity:
 *   crates/gravity/src/kernel.rs:1-128   softening kernels
 *   crates/gravity/src/direct.rs:115-658 the eight direct-sum functions
 * It repeats the Rust arithmetic operation for operation: Rust does not
 * contract a*b+c into an FMA, so this file must be compiled with
 * -ffp-contract=off (see oracle/Makefile); (a*b)*c groupings, the
 * ascending-j summation order, the N<512 symmetric pair loops and the
 * per-target loops of the N>=512 branches are all kept.  With those flags
 * the results are bitwise what the Rust code computes on x86-64 (IEEE
 * double, correctly rounded sqrt and divide).
 *
 * Parity status: the Rust crate cannot be built in this image (no cargo /
 * rustc), and the reference holds no golden vectors for this path, so this
 * restatement is pinned by the reference's own property tests re-run on it
 * (crates/gravity/tests/gravity_tests.rs, single_node.rs) and by analytic
 * known-answer tests (tests/test_oracle_gravity.py).  Absolute parity with
 * the Rust binary itself is "unpinned" beyond those properties.
 *
 * The per-target loops are parallelised with OpenMP like the reference's
 * rayon par_iter (each target's sum is still sequential in j, so the result
 * does not depend on the thread count).
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define R2_TINY 2.2250738585072014e-308 /* f64::MIN_POSITIVE, direct.rs:7 */

enum { K_PLUMMER = 0, K_SPLINE = 1 };

/* kernel.rs:85-106 */
static double w2(double u) {
  if (u < 0.5) {
    double u2 = u * u;
    double u4 = u2 * u2;
    double u5 = u4 * u;
    return (16.0 / 3.0) * u2 - (48.0 / 5.0) * u4 + (32.0 / 5.0) * u5 - 14.0 / 5.0;
  } else if (u < 1.0) {
    double inv_u = 1.0 / u;
    double u2 = u * u;
    double u3 = u2 * u;
    double u4 = u2 * u2;
    double u5 = u4 * u;
    return (1.0 / 15.0) * inv_u + (32.0 / 3.0) * u2 - 16.0 * u3 + (48.0 / 5.0) * u4 -
           (32.0 / 15.0) * u5 - 16.0 / 5.0;
  }
  return -1.0 / u;
}

/* kernel.rs:108-128 */
static double w2_prime(double u) {
  if (u < 0.5) {
    double u2 = u * u;
    double u3 = u2 * u;
    double u4 = u2 * u2;
    return (32.0 / 3.0) * u - (192.0 / 5.0) * u3 + 32.0 * u4;
  } else if (u < 1.0) {
    double u2 = u * u;
    double u3 = u2 * u;
    double u4 = u2 * u2;
    return -(1.0 / 15.0) * (1.0 / u2) + (64.0 / 3.0) * u - 48.0 * u2 + (192.0 / 5.0) * u3 -
           (32.0 / 3.0) * u4;
  }
  return 1.0 / (u * u);
}

/* kernel.rs:41-56 */
double pbxref_kernel_potential(int kind, double r, double h) {
  if (r == 0.0) return 0.0;
  if (kind == K_PLUMMER) return -1.0 / sqrt(r * r + h * h);
  if (h <= 0.0) return -1.0 / r;
  double h_inv = 1.0 / h;
  double u = r * h_inv;
  return w2(u) * h_inv;
}

/* kernel.rs:62-82 */
double pbxref_kernel_accel_factor(int kind, double r, double h) {
  if (r == 0.0) return 0.0;
  if (kind == K_PLUMMER) {
    double s2 = r * r + h * h;
    return 1.0 / (sqrt(s2) * s2);
  }
  if (h <= 0.0) return 1.0 / (r * r * r);
  double h_inv = 1.0 / h;
  double u = r * h_inv;
  return w2_prime(u) * (h_inv * h_inv) / r;
}

/* kernel.rs:20-37 */
int pbxref_multipole_soft_ok(int kind, double r, double h) {
  if (h <= 0.0) return 1;
  double c = (kind == K_PLUMMER) ? 2.8 : 1.0;
  return r > c * h;
}

/* Rust f64::max: NaN-ignoring, like C fmax. */
static inline double rmax(double a, double b) { return fmax(a, b); }

static inline double mass_of(const double *m, int64_t j) { return m ? m[j] : 1.0; }
static inline double soft_of(const double *h, int64_t j) { return h ? h[j] : 0.0; }

/* direct.rs:115-185 */
void pbxref_direct_accelerations(const double *pos, int64_t n, const double *mass,
                                 double *acc) {
  memset(acc, 0, sizeof(double) * 3 * (size_t)n);
  if (n == 0) return;
  if (n < 512) {
    for (int64_t i = 0; i < n; ++i) {
      const double *pi = pos + 3 * i;
      double mi = mass_of(mass, i);
      for (int64_t j = i + 1; j < n; ++j) {
        const double *pj = pos + 3 * j;
        double dx = pj[0] - pi[0], dy = pj[1] - pi[1], dz = pj[2] - pi[2];
        double r2 = dx * dx + dy * dy + dz * dz;
        double s2 = r2 + R2_TINY;
        double invr3 = 1.0 / (sqrt(s2) * s2);
        double mj = mass_of(mass, j);
        acc[3 * i + 0] += mj * dx * invr3;
        acc[3 * i + 1] += mj * dy * invr3;
        acc[3 * i + 2] += mj * dz * invr3;
        acc[3 * j + 0] -= mi * dx * invr3;
        acc[3 * j + 1] -= mi * dy * invr3;
        acc[3 * j + 2] -= mi * dz * invr3;
      }
    }
    return;
  }
#pragma omp parallel for schedule(static)
  for (int64_t i = 0; i < n; ++i) {
    const double *pi = pos + 3 * i;
    double ax = 0.0, ay = 0.0, az = 0.0;
    for (int64_t j = 0; j < n; ++j) {
      if (j == i) continue;
      const double *pj = pos + 3 * j;
      double dx = pj[0] - pi[0], dy = pj[1] - pi[1], dz = pj[2] - pi[2];
      double r2 = dx * dx + dy * dy + dz * dz;
      double s2 = r2 + R2_TINY;
      double invr3 = 1.0 / (sqrt(s2) * s2);
      double mj = mass_of(mass, j);
      ax += mj * dx * invr3;
      ay += mj * dy * invr3;
      az += mj * dz * invr3;
    }
    acc[3 * i + 0] = ax;
    acc[3 * i + 1] = ay;
    acc[3 * i + 2] = az;
  }
}

/* direct.rs:187-251 (both branches are the same per-target loop) */
void pbxref_direct_accelerations_at_points(const double *pos, int64_t n, const double *mass,
                                           const double *tgt, int64_t m, double *acc) {
  memset(acc, 0, sizeof(double) * 3 * (size_t)m);
  if (m == 0 || n == 0) return;
#pragma omp parallel for schedule(static) if (m >= 512)
  for (int64_t i = 0; i < m; ++i) {
    const double *pi = tgt + 3 * i;
    double ax = 0.0, ay = 0.0, az = 0.0;
    for (int64_t j = 0; j < n; ++j) {
      const double *pj = pos + 3 * j;
      double dx = pj[0] - pi[0], dy = pj[1] - pi[1], dz = pj[2] - pi[2];
      double r2 = dx * dx + dy * dy + dz * dz;
      double s2 = r2 + R2_TINY;
      double invr3 = 1.0 / (sqrt(s2) * s2);
      double mm = mass_of(mass, j);
      ax += mm * dx * invr3;
      ay += mm * dy * invr3;
      az += mm * dz * invr3;
    }
    acc[3 * i + 0] = ax;
    acc[3 * i + 1] = ay;
    acc[3 * i + 2] = az;
  }
}

/* direct.rs:255-313 */
void pbxref_direct_potentials(const double *pos, int64_t n, const double *mass, double *pot) {
  memset(pot, 0, sizeof(double) * (size_t)n);
  if (n == 0) return;
  if (n < 512) {
    for (int64_t i = 0; i < n; ++i) {
      const double *pi = pos + 3 * i;
      double mi = mass_of(mass, i);
      for (int64_t j = i + 1; j < n; ++j) {
        const double *pj = pos + 3 * j;
        double dx = pj[0] - pi[0], dy = pj[1] - pi[1], dz = pj[2] - pi[2];
        double r2 = dx * dx + dy * dy + dz * dz;
        double invr = 1.0 / sqrt(r2 + R2_TINY);
        double mj = mass_of(mass, j);
        double phi_pair = -invr;
        pot[i] += phi_pair * mj;
        pot[j] += phi_pair * mi;
      }
    }
    return;
  }
#pragma omp parallel for schedule(static)
  for (int64_t i = 0; i < n; ++i) {
    const double *pi = pos + 3 * i;
    double phi = 0.0;
    for (int64_t j = 0; j < n; ++j) {
      if (j == i) continue;
      const double *pj = pos + 3 * j;
      double dx = pj[0] - pi[0], dy = pj[1] - pi[1], dz = pj[2] - pi[2];
      double r2 = dx * dx + dy * dy + dz * dz;
      double invr = 1.0 / sqrt(r2 + R2_TINY);
      double mj = mass_of(mass, j);
      phi += -mj * invr;
    }
    pot[i] = phi;
  }
}

/* direct.rs:315-368 */
void pbxref_direct_potentials_at_points(const double *pos, int64_t n, const double *mass,
                                        const double *tgt, int64_t m, double *pot) {
  memset(pot, 0, sizeof(double) * (size_t)m);
  if (m == 0 || n == 0) return;
#pragma omp parallel for schedule(static) if (m >= 512)
  for (int64_t i = 0; i < m; ++i) {
    const double *pi = tgt + 3 * i;
    double phi = 0.0;
    for (int64_t j = 0; j < n; ++j) {
      const double *pj = pos + 3 * j;
      double dx = pj[0] - pi[0], dy = pj[1] - pi[1], dz = pj[2] - pi[2];
      double r2 = dx * dx + dy * dy + dz * dz;
      double invr = 1.0 / sqrt(r2 + R2_TINY);
      double mm = mass_of(mass, j);
      phi += -mm * invr;
    }
    pot[i] = phi;
  }
}

/* direct.rs:370-441 */
void pbxref_direct_potentials_kernel(const double *pos, int64_t n, const double *mass,
                                     const double *soft, int kind, double *pot) {
  memset(pot, 0, sizeof(double) * (size_t)n);
  if (n == 0) return;
  if (n < 512) {
    for (int64_t i = 0; i < n; ++i) {
      const double *pi = pos + 3 * i;
      double mi = mass_of(mass, i);
      double hi = soft_of(soft, i);
      for (int64_t j = i + 1; j < n; ++j) {
        const double *pj = pos + 3 * j;
        double mj = mass_of(mass, j);
        double hj = soft_of(soft, j);
        double h = rmax(hi, hj);
        double dx = pj[0] - pi[0], dy = pj[1] - pi[1], dz = pj[2] - pi[2];
        double r2 = dx * dx + dy * dy + dz * dz;
        double r = sqrt(r2 + R2_TINY);
        double phi_pair = pbxref_kernel_potential(kind, r, h);
        pot[i] += mj * phi_pair;
        pot[j] += mi * phi_pair;
      }
    }
    return;
  }
#pragma omp parallel for schedule(static)
  for (int64_t i = 0; i < n; ++i) {
    const double *pi = pos + 3 * i;
    double hi = soft_of(soft, i);
    double phi = 0.0;
    for (int64_t j = 0; j < n; ++j) {
      if (j == i) continue;
      const double *pj = pos + 3 * j;
      double hj = soft_of(soft, j);
      double h = rmax(hi, hj);
      double dx = pj[0] - pi[0], dy = pj[1] - pi[1], dz = pj[2] - pi[2];
      double r2 = dx * dx + dy * dy + dz * dz;
      double r = sqrt(r2 + R2_TINY);
      double phi_ij = pbxref_kernel_potential(kind, r, h);
      phi += mass_of(mass, j) * phi_ij;
    }
    pot[i] = phi;
  }
}

/* direct.rs:443-524 */
void pbxref_direct_accelerations_kernel(const double *pos, int64_t n, const double *mass,
                                        const double *soft, int kind, double *acc) {
  memset(acc, 0, sizeof(double) * 3 * (size_t)n);
  if (n == 0) return;
  if (n < 512) {
    for (int64_t i = 0; i < n; ++i) {
      const double *pi = pos + 3 * i;
      double mi = mass_of(mass, i);
      double hi = soft_of(soft, i);
      for (int64_t j = i + 1; j < n; ++j) {
        const double *pj = pos + 3 * j;
        double mj = mass_of(mass, j);
        double hj = soft_of(soft, j);
        double h = rmax(hi, hj);
        double dx = pj[0] - pi[0], dy = pj[1] - pi[1], dz = pj[2] - pi[2];
        double r2 = dx * dx + dy * dy + dz * dz;
        double r = sqrt(r2 + R2_TINY);
        double g = pbxref_kernel_accel_factor(kind, r, h);
        acc[3 * i + 0] += mj * dx * g;
        acc[3 * i + 1] += mj * dy * g;
        acc[3 * i + 2] += mj * dz * g;
        acc[3 * j + 0] -= mi * dx * g;
        acc[3 * j + 1] -= mi * dy * g;
        acc[3 * j + 2] -= mi * dz * g;
      }
    }
    return;
  }
#pragma omp parallel for schedule(static)
  for (int64_t i = 0; i < n; ++i) {
    const double *pi = pos + 3 * i;
    double hi = soft_of(soft, i);
    double ax = 0.0, ay = 0.0, az = 0.0;
    for (int64_t j = 0; j < n; ++j) {
      if (j == i) continue;
      const double *pj = pos + 3 * j;
      double hj = soft_of(soft, j);
      double h = rmax(hi, hj);
      double dx = pj[0] - pi[0], dy = pj[1] - pi[1], dz = pj[2] - pi[2];
      double r2 = dx * dx + dy * dy + dz * dz;
      double r = sqrt(r2 + R2_TINY);
      double g = pbxref_kernel_accel_factor(kind, r, h);
      double mj = mass_of(mass, j);
      ax += mj * dx * g;
      ay += mj * dy * g;
      az += mj * dz * g;
    }
    acc[3 * i + 0] = ax;
    acc[3 * i + 1] = ay;
    acc[3 * i + 2] = az;
  }
}

/* direct.rs:526-585 */
void pbxref_direct_potentials_kernel_at_points(const double *pos, int64_t n,
                                               const double *mass, const double *soft,
                                               const double *tgt, int64_t m, int kind,
                                               double *pot) {
  memset(pot, 0, sizeof(double) * (size_t)m);
  if (m == 0 || n == 0) return;
#pragma omp parallel for schedule(static) if (m >= 512)
  for (int64_t i = 0; i < m; ++i) {
    const double *pi = tgt + 3 * i;
    double phi = 0.0;
    for (int64_t j = 0; j < n; ++j) {
      const double *pj = pos + 3 * j;
      double dx = pj[0] - pi[0], dy = pj[1] - pi[1], dz = pj[2] - pi[2];
      double r2 = dx * dx + dy * dy + dz * dz;
      double r = sqrt(r2 + R2_TINY);
      double hj = soft_of(soft, j);
      double h = rmax(hj, 0.0);
      phi += mass_of(mass, j) * pbxref_kernel_potential(kind, r, h);
    }
    pot[i] = phi;
  }
}

/* direct.rs:587-658 */
void pbxref_direct_accelerations_kernel_at_points(const double *pos, int64_t n,
                                                  const double *mass, const double *soft,
                                                  const double *tgt, int64_t m, int kind,
                                                  double *acc) {
  memset(acc, 0, sizeof(double) * 3 * (size_t)m);
  if (m == 0 || n == 0) return;
#pragma omp parallel for schedule(static) if (m >= 512)
  for (int64_t i = 0; i < m; ++i) {
    const double *pi = tgt + 3 * i;
    double ax = 0.0, ay = 0.0, az = 0.0;
    for (int64_t j = 0; j < n; ++j) {
      const double *pj = pos + 3 * j;
      double dx = pj[0] - pi[0], dy = pj[1] - pi[1], dz = pj[2] - pi[2];
      double r2 = dx * dx + dy * dy + dz * dz;
      double r = sqrt(r2 + R2_TINY);
      double hj = soft_of(soft, j);
      double h = rmax(hj, 0.0);
      double g = pbxref_kernel_accel_factor(kind, r, h);
      double mj = mass_of(mass, j);
      ax += mj * dx * g;
      ay += mj * dy * g;
      az += mj * dz * g;
    }
    acc[3 * i + 0] = ax;
    acc[3 * i + 1] = ay;
    acc[3 * i + 2] = az;
  }
}

/* Subset helper for the CPU baseline / large-N parity: potentials and
 * accelerations of the all-particles form for a LIST of target indices
 * (same per-target loop as the N>=512 branches of direct.rs:160-182,
 * 293-310).  Each target's sum is identical to what the full call returns
 * for that index when n >= 512. */
void pbxref_direct_subset(const double *pos, int64_t n, const double *mass,
                          const int64_t *idx, int64_t k, double *pot, double *acc) {
#pragma omp parallel for schedule(dynamic, 16)
  for (int64_t t = 0; t < k; ++t) {
    int64_t i = idx[t];
    const double *pi = pos + 3 * i;
    double phi = 0.0, ax = 0.0, ay = 0.0, az = 0.0;
    for (int64_t j = 0; j < n; ++j) {
      if (j == i) continue;
      const double *pj = pos + 3 * j;
      double dx = pj[0] - pi[0], dy = pj[1] - pi[1], dz = pj[2] - pi[2];
      double r2 = dx * dx + dy * dy + dz * dz;
      double s2 = r2 + R2_TINY;
      double mj = mass_of(mass, j);
      double invr = 1.0 / sqrt(s2);           /* direct.rs:305 */
      phi += -mj * invr;
      double invr3 = 1.0 / (sqrt(s2) * s2);   /* direct.rs:175 */
      ax += mj * dx * invr3;
      ay += mj * dy * invr3;
      az += mj * dz * invr3;
    }
    if (pot) pot[t] = phi;
    if (acc) {
      acc[3 * t + 0] = ax;
      acc[3 * t + 1] = ay;
      acc[3 * t + 2] = az;
    }
  }
}

int pbxref_num_threads(void) {
#ifdef _OPENMP
  extern int omp_get_max_threads(void);
  return omp_get_max_threads();
#else
  return 1;
#endif
}

void pbxref_set_num_threads(int n) {
#ifdef _OPENMP
  extern void omp_set_num_threads(int);
  omp_set_num_threads(n);
#else
  (void)n;
#endif
}
