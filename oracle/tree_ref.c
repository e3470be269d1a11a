/*
 * tree_ref.c — ORACLE (test infrastructure only; never shipped, never the
 * measured path).  Only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg may load it.
 *
 * A plain-C restatement of the reference's Barnes–Hut octree:
 *   crates/gravity/src/tree.rs:34-71      R2_TINY, inv_r helpers, node_soft_ok
 *   crates/gravity/src/tree.rs:98-417     leaf potential / acceleration sums
 *   crates/gravity/src/tree.rs:628-864    bbox, from_owned, links, subdivide
 *   crates/gravity/src/tree.rs:866-1067   BH / h_max / multipole payloads
 *   crates/gravity/src/tree.rs:1069-1391  stackless traversals (+ :419-543)
 *   crates/gravity/src/tree.rs:1393-1559  Tree3D (build, compute_*, *_at_points)
 *   crates/gravity/src/multipole.rs:82-252     P2M (from_points_const)
 *   crates/gravity/src/multipole.rs:584-856, 1216-1349  derivative tensors
 *   crates/gravity/src/multipole.rs:397-580, 858-1025, 1352-1528  evaluators
 *   crates/gravity/src/multipole.rs:1536-1595  M2M (translate_multipole)
 *
 * Node numbering, child order, payload summation order, traversal order and
 * every arithmetic expression follow the Rust code (mul_add -> fma, all other
 * a*b+c unfused: compile with -ffp-contract=off, see oracle/Makefile).  The
 * compact per-order moment/derivative structs of multipole.rs compute the
 * same expressions as the full ones truncated at that order, so one 56-slot
 * layout (the MultipoleMoment field order, multipole.rs:11-74) is used here.
 * x.powi(k) is restated as the binary-exponentiation product LLVM emits
 * (powi3 = x*(x*x), powi4 = (x*x)*(x*x), powi5 = x*((x*x)*(x*x))).
 *
 * Divergence (documented in DESIGN.md): the reference recurses forever when
 * more than leaf_capacity particles share one position (tree.rs:847-864 has
 * no depth cap).  Here such a node stops splitting when all of its particles
 * are bitwise-identical or its half size underflows to 0 — the product build
 * uses the same rule.
 *
 * Parity status: the Rust crate cannot be built in this image (no cargo /
 * rustc) and the reference holds no golden vectors for the tree, so this
 * restatement is pinned by the reference's own property tests re-run on it
 * (crates/gravity/tests/gravity_tests.rs, single_node.rs,
 * translate_multipole.rs — tests/test_oracle_tree.py) plus known-answer
 * tests; absolute parity with the Rust binary is "unpinned" beyond those.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define R2_TINY 2.2250738585072014e-308 /* f64::MIN_POSITIVE, tree.rs:36 */
#define NONE ((int64_t)-1)              /* usize::MAX */
#define NMOM 56

enum { K_PLUMMER = 0, K_SPLINE = 1 };

/* from gravity_ref.c (kernel.rs:41-82) */
double pbxref_kernel_potential(int kind, double r, double h);
double pbxref_kernel_accel_factor(int kind, double r, double h);

/* MultipoleMoment / PotentialDerivatives field order (multipole.rs:11-74,
 * 1157-1214). */
enum {
  I000, I100, I010, I001,
  I200, I020, I002, I110, I101, I011,
  I300, I030, I003, I210, I201, I120, I102, I021, I012, I111,
  I400, I040, I004, I310, I301, I130, I103, I031, I013, I220, I202, I022, I211, I121, I112,
  I500, I050, I005, I410, I401, I140, I104, I041, I014, I320, I302, I230, I203, I032, I023,
  I221, I212, I122, I311, I131, I113
};

static const int IDX_LMN[NMOM][3] = {
  {0,0,0},{1,0,0},{0,1,0},{0,0,1},
  {2,0,0},{0,2,0},{0,0,2},{1,1,0},{1,0,1},{0,1,1},
  {3,0,0},{0,3,0},{0,0,3},{2,1,0},{2,0,1},{1,2,0},{1,0,2},{0,2,1},{0,1,2},{1,1,1},
  {4,0,0},{0,4,0},{0,0,4},{3,1,0},{3,0,1},{1,3,0},{1,0,3},{0,3,1},{0,1,3},{2,2,0},{2,0,2},
  {0,2,2},{2,1,1},{1,2,1},{1,1,2},
  {5,0,0},{0,5,0},{0,0,5},{4,1,0},{4,0,1},{1,4,0},{1,0,4},{0,4,1},{0,1,4},{3,2,0},{3,0,2},
  {2,3,0},{2,0,3},{0,3,2},{0,2,3},{2,2,1},{2,1,2},{1,2,2},{3,1,1},{1,3,1},{1,1,3}
};

static int slot_of(int l, int m, int n) {
  for (int s = 0; s < NMOM; ++s)
    if (IDX_LMN[s][0] == l && IDX_LMN[s][1] == m && IDX_LMN[s][2] == n) return s;
  return -1;
}

static inline double powi(double x, int k) { /* LLVM ExpandPowI / __powidf2 */
  double r = 1.0;
  int first = 1;
  while (k) {
    if (k & 1) {
      r = first ? x : r * x;
      first = 0;
    }
    k >>= 1;
    if (k) x = x * x;
  }
  return r;
}

/* ------------------------------------------------------------------ */
/* multipole.rs:82-170  from_points_const<O>                           */
/* ------------------------------------------------------------------ */
void pbxref_multipole_from_points(const double *pos, const double *mass, const int64_t *idx,
                                  int64_t nidx, const double *center, int order, double *m) {
  memset(m, 0, sizeof(double) * NMOM);
  int O = order < 5 ? order : 5;
  for (int64_t t = 0; t < nidx; ++t) {
    int64_t pi = idx[t];
    double ms = mass ? mass[pi] : 1.0;
    double x = pos[3 * pi + 0] - center[0];
    double y = pos[3 * pi + 1] - center[1];
    double z = pos[3 * pi + 2] - center[2];
    m[I000] += ms;
    if (O >= 1) {
      m[I100] += ms * x;
      m[I010] += ms * y;
      m[I001] += ms * z;
    }
    if (O >= 2) {
      m[I200] += 0.5 * ms * x * x;
      m[I020] += 0.5 * ms * y * y;
      m[I002] += 0.5 * ms * z * z;
      m[I110] += ms * x * y;
      m[I101] += ms * x * z;
      m[I011] += ms * y * z;
    }
    if (O >= 3) {
      m[I300] += (1.0 / 6.0) * ms * powi(x, 3);
      m[I030] += (1.0 / 6.0) * ms * powi(y, 3);
      m[I003] += (1.0 / 6.0) * ms * powi(z, 3);
      m[I210] += 0.5 * ms * x * x * y;
      m[I201] += 0.5 * ms * x * x * z;
      m[I120] += 0.5 * ms * y * y * x;
      m[I102] += 0.5 * ms * x * z * z;
      m[I021] += 0.5 * ms * y * y * z;
      m[I012] += 0.5 * ms * y * z * z;
      m[I111] += ms * x * y * z;
    }
    if (O >= 4) {
      m[I400] += (1.0 / 24.0) * ms * powi(x, 4);
      m[I040] += (1.0 / 24.0) * ms * powi(y, 4);
      m[I004] += (1.0 / 24.0) * ms * powi(z, 4);
      m[I310] += (1.0 / 6.0) * ms * powi(x, 3) * y;
      m[I301] += (1.0 / 6.0) * ms * powi(x, 3) * z;
      m[I130] += (1.0 / 6.0) * ms * powi(y, 3) * x;
      m[I103] += (1.0 / 6.0) * ms * x * powi(z, 3);
      m[I031] += (1.0 / 6.0) * ms * powi(y, 3) * z;
      m[I013] += (1.0 / 6.0) * ms * y * powi(z, 3);
      m[I220] += 0.25 * ms * x * x * y * y;
      m[I202] += 0.25 * ms * x * x * z * z;
      m[I022] += 0.25 * ms * y * y * z * z;
      m[I211] += 0.5 * ms * x * x * y * z;
      m[I121] += 0.5 * ms * y * y * x * z;
      m[I112] += 0.5 * ms * z * z * x * y;
    }
    if (O >= 5) {
      m[I500] += (1.0 / 120.0) * ms * powi(x, 5);
      m[I050] += (1.0 / 120.0) * ms * powi(y, 5);
      m[I005] += (1.0 / 120.0) * ms * powi(z, 5);
      m[I410] += (1.0 / 24.0) * ms * powi(x, 4) * y;
      m[I401] += (1.0 / 24.0) * ms * powi(x, 4) * z;
      m[I140] += (1.0 / 24.0) * ms * powi(y, 4) * x;
      m[I104] += (1.0 / 24.0) * ms * powi(z, 4) * x;
      m[I041] += (1.0 / 24.0) * ms * powi(y, 4) * z;
      m[I014] += (1.0 / 24.0) * ms * powi(z, 4) * y;
      m[I320] += (1.0 / 12.0) * ms * powi(x, 3) * powi(y, 2);
      m[I302] += (1.0 / 12.0) * ms * powi(x, 3) * powi(z, 2);
      m[I230] += (1.0 / 12.0) * ms * powi(x, 2) * powi(y, 3);
      m[I203] += (1.0 / 12.0) * ms * powi(x, 2) * powi(z, 3);
      m[I032] += (1.0 / 12.0) * ms * powi(y, 3) * powi(z, 2);
      m[I023] += (1.0 / 12.0) * ms * powi(y, 2) * powi(z, 3);
      m[I221] += 0.25 * ms * x * x * y * y * z;
      m[I212] += 0.25 * ms * x * x * z * z * y;
      m[I122] += 0.25 * ms * y * y * z * z * x;
      m[I311] += (1.0 / 6.0) * ms * powi(x, 3) * y * z;
      m[I131] += (1.0 / 6.0) * ms * powi(y, 3) * x * z;
      m[I113] += (1.0 / 6.0) * ms * powi(z, 3) * x * y;
    }
  }
}

/* multipole.rs:1536-1595  translate_multipole (M2M) */
static const double FACT[6] = {1.0, 1.0, 2.0, 6.0, 24.0, 120.0};

void pbxref_translate_multipole(const double *mc, const double *shift, int order, double *out) {
  int o = order < 5 ? order : 5;
  memset(out, 0, sizeof(double) * NMOM);
  for (int l = 0; l <= o; ++l)
    for (int mm = 0; mm <= o; ++mm)
      for (int n = 0; n <= o; ++n) {
        if (l + mm + n > o) continue;
        double sum = 0.0;
        for (int i = 0; i <= l; ++i)
          for (int j = 0; j <= mm; ++j)
            for (int k = 0; k <= n; ++k) {
              int s = slot_of(i, j, k);
              double base = s >= 0 ? mc[s] : 0.0;
              if (base == 0.0) continue;
              int dl = l - i, dm = mm - j, dn = n - k;
              double pw;
              if (dl + dm + dn == 0) {
                pw = 1.0;
              } else {
                double sx = dl > 0 ? powi(shift[0], dl) : 1.0;
                double sy = dm > 0 ? powi(shift[1], dm) : 1.0;
                double sz = dn > 0 ? powi(shift[2], dn) : 1.0;
                pw = sx * sy * sz;
              }
              double sign = ((dl + dm + dn) % 2 == 0) ? 1.0 : -1.0;
              double coeff = sign * pw / (FACT[dl] * FACT[dm] * FACT[dn]);
              sum += coeff * base;
            }
        int s = slot_of(l, mm, n);
        if (s >= 0) out[s] = sum;
      }
}

/* multipole.rs:1216-1349  PotentialDerivatives::new (the compact
 * PotentialDerivatives1/2/3 of :593-771 evaluate the same expressions). */
void pbxref_potential_derivatives(double dx, double dy, double dz, double eps2, int order,
                                  double *d) {
  memset(d, 0, sizeof(double) * NMOM);
  int max = order < 5 ? order : 5;
  double r2 = dx * dx + dy * dy + dz * dz + eps2 + R2_TINY;
  double r = sqrt(r2);
  double r_inv = 1.0 / r;
  double dt_1 = r_inv;
  double dt_2 = -dt_1 * r_inv;
  double dt_3 = -3.0 * dt_2 * r_inv;
  double dt_4 = -5.0 * dt_3 * r_inv;
  double dt_5 = -7.0 * dt_4 * r_inv;
  double dt_6 = -9.0 * dt_5 * r_inv;
  double rx_r = dx * r_inv, ry_r = dy * r_inv, rz_r = dz * r_inv;
  double rx_r2 = rx_r * rx_r, ry_r2 = ry_r * ry_r, rz_r2 = rz_r * rz_r;
  double rx_r3 = rx_r2 * rx_r, ry_r3 = ry_r2 * ry_r, rz_r3 = rz_r2 * rz_r;
  double rx_r4 = rx_r3 * rx_r, ry_r4 = ry_r3 * ry_r, rz_r4 = rz_r3 * rz_r;
  double rx_r5 = rx_r4 * rx_r, ry_r5 = ry_r4 * ry_r, rz_r5 = rz_r4 * rz_r;
  d[I000] = dt_1;
  if (max == 0) return;
  d[I100] = dt_2 * rx_r;
  d[I010] = dt_2 * ry_r;
  d[I001] = dt_2 * rz_r;
  if (max == 1) return;
  dt_2 *= r_inv;
  d[I200] = dt_3 * rx_r2 + dt_2;
  d[I020] = dt_3 * ry_r2 + dt_2;
  d[I002] = dt_3 * rz_r2 + dt_2;
  d[I110] = dt_3 * rx_r * ry_r;
  d[I101] = dt_3 * rx_r * rz_r;
  d[I011] = dt_3 * ry_r * rz_r;
  if (max == 2) return;
  dt_3 *= r_inv;
  d[I300] = dt_4 * rx_r3 + 3.0 * dt_3 * rx_r;
  d[I030] = dt_4 * ry_r3 + 3.0 * dt_3 * ry_r;
  d[I003] = dt_4 * rz_r3 + 3.0 * dt_3 * rz_r;
  d[I210] = dt_4 * rx_r2 * ry_r + dt_3 * ry_r;
  d[I201] = dt_4 * rx_r2 * rz_r + dt_3 * rz_r;
  d[I120] = dt_4 * ry_r2 * rx_r + dt_3 * rx_r;
  d[I102] = dt_4 * rz_r2 * rx_r + dt_3 * rx_r;
  d[I021] = dt_4 * ry_r2 * rz_r + dt_3 * rz_r;
  d[I012] = dt_4 * rz_r2 * ry_r + dt_3 * ry_r;
  d[I111] = dt_4 * rx_r * ry_r * rz_r;
  if (max == 3) return;
  dt_3 *= r_inv;
  dt_4 *= r_inv;
  d[I400] = dt_5 * rx_r4 + 6.0 * dt_4 * rx_r2 + 3.0 * dt_3;
  d[I040] = dt_5 * ry_r4 + 6.0 * dt_4 * ry_r2 + 3.0 * dt_3;
  d[I004] = dt_5 * rz_r4 + 6.0 * dt_4 * rz_r2 + 3.0 * dt_3;
  d[I310] = dt_5 * rx_r3 * ry_r + 3.0 * dt_4 * rx_r * ry_r;
  d[I301] = dt_5 * rx_r3 * rz_r + 3.0 * dt_4 * rx_r * rz_r;
  d[I130] = dt_5 * ry_r3 * rx_r + 3.0 * dt_4 * ry_r * rx_r;
  d[I103] = dt_5 * rz_r3 * rx_r + 3.0 * dt_4 * rx_r * rz_r;
  d[I031] = dt_5 * ry_r3 * rz_r + 3.0 * dt_4 * rz_r * ry_r;
  d[I013] = dt_5 * rz_r3 * ry_r + 3.0 * dt_4 * rz_r * ry_r;
  d[I220] = dt_5 * rx_r2 * ry_r2 + dt_4 * (rx_r2 + ry_r2) + dt_3;
  d[I202] = dt_5 * rx_r2 * rz_r2 + dt_4 * (rx_r2 + rz_r2) + dt_3;
  d[I022] = dt_5 * ry_r2 * rz_r2 + dt_4 * (ry_r2 + rz_r2) + dt_3;
  d[I211] = dt_5 * rx_r2 * ry_r * rz_r + dt_4 * ry_r * rz_r;
  d[I121] = dt_5 * ry_r2 * rx_r * rz_r + dt_4 * rx_r * rz_r;
  d[I112] = dt_5 * rz_r2 * rx_r * ry_r + dt_4 * rx_r * ry_r;
  if (max == 4) return;
  dt_4 *= r_inv;
  dt_5 *= r_inv;
  d[I500] = dt_6 * rx_r5 + 10.0 * dt_5 * rx_r3 + 15.0 * dt_4 * rx_r;
  d[I050] = dt_6 * ry_r5 + 10.0 * dt_5 * ry_r3 + 15.0 * dt_4 * ry_r;
  d[I005] = dt_6 * rz_r5 + 10.0 * dt_5 * rz_r3 + 15.0 * dt_4 * rz_r;
  d[I410] = dt_6 * rx_r4 * ry_r + 6.0 * dt_5 * rx_r2 * ry_r + 3.0 * dt_4 * ry_r;
  d[I401] = dt_6 * rx_r4 * rz_r + 6.0 * dt_5 * rx_r2 * rz_r + 3.0 * dt_4 * rz_r;
  d[I140] = dt_6 * ry_r4 * rx_r + 6.0 * dt_5 * ry_r2 * rx_r + 3.0 * dt_4 * rx_r;
  d[I041] = dt_6 * ry_r4 * rz_r + 6.0 * dt_5 * ry_r2 * rz_r + 3.0 * dt_4 * rz_r;
  d[I104] = dt_6 * rz_r4 * rx_r + 6.0 * dt_5 * rz_r2 * rx_r + 3.0 * dt_4 * rx_r;
  d[I014] = dt_6 * rz_r4 * ry_r + 6.0 * dt_5 * rz_r2 * ry_r + 3.0 * dt_4 * ry_r;
  d[I320] = dt_6 * rx_r3 * ry_r2 + dt_5 * rx_r3 + 3.0 * dt_5 * rx_r * ry_r2 + 3.0 * dt_4 * rx_r;
  d[I302] = dt_6 * rx_r3 * rz_r2 + dt_5 * rx_r3 + 3.0 * dt_5 * rx_r * rz_r2 + 3.0 * dt_4 * rx_r;
  d[I230] = dt_6 * ry_r3 * rx_r2 + dt_5 * ry_r3 + 3.0 * dt_5 * ry_r * rx_r2 + 3.0 * dt_4 * ry_r;
  d[I032] = dt_6 * ry_r3 * rz_r2 + dt_5 * ry_r3 + 3.0 * dt_5 * ry_r * rz_r2 + 3.0 * dt_4 * ry_r;
  d[I203] = dt_6 * rz_r3 * rx_r2 + dt_5 * rz_r3 + 3.0 * dt_5 * rz_r * rx_r2 + 3.0 * dt_4 * rz_r;
  d[I023] = dt_6 * rz_r3 * ry_r2 + dt_5 * rz_r3 + 3.0 * dt_5 * rz_r * ry_r2 + 3.0 * dt_4 * rz_r;
  d[I311] = dt_6 * rx_r3 * ry_r * rz_r + 3.0 * dt_5 * rx_r * ry_r * rz_r;
  d[I131] = dt_6 * ry_r3 * rx_r * rz_r + 3.0 * dt_5 * rx_r * ry_r * rz_r;
  d[I113] = dt_6 * rz_r3 * rx_r * ry_r + 3.0 * dt_5 * rx_r * ry_r * rz_r;
  d[I122] = dt_6 * rx_r * ry_r2 * rz_r2 + dt_5 * rx_r * ry_r2 + dt_5 * rx_r * rz_r2 + dt_4 * rx_r;
  d[I212] = dt_6 * ry_r * rx_r2 * rz_r2 + dt_5 * ry_r * rx_r2 + dt_5 * ry_r * rz_r2 + dt_4 * ry_r;
  d[I221] = dt_6 * rz_r * rx_r2 * ry_r2 + dt_5 * rz_r * rx_r2 + dt_5 * rz_r * ry_r2 + dt_4 * rz_r;
}

/* multipole.rs:1352-1405 (and the o0..o4 specialisations :397-459, 858-917) */
double pbxref_gravity_potential_multipole(const double *m, const double *d, int order) {
  int o = order < 5 ? order : 5;
  if (o <= 1) return -m[I000] * d[I000];
  double phi = -m[I000] * d[I000];
  phi -= m[I200] * d[I200] + m[I020] * d[I020] + m[I002] * d[I002];
  phi -= m[I110] * d[I110] + m[I101] * d[I101] + m[I011] * d[I011];
  if (o == 2) return phi;
  phi -= m[I300] * d[I300] + m[I030] * d[I030] + m[I003] * d[I003];
  phi -= m[I210] * d[I210] + m[I201] * d[I201] + m[I120] * d[I120];
  phi -= m[I102] * d[I102] + m[I021] * d[I021] + m[I012] * d[I012];
  phi -= m[I111] * d[I111];
  if (o == 3) return phi;
  phi -= m[I400] * d[I400] + m[I040] * d[I040] + m[I004] * d[I004];
  phi -= m[I310] * d[I310] + m[I301] * d[I301] + m[I130] * d[I130];
  phi -= m[I103] * d[I103] + m[I031] * d[I031] + m[I013] * d[I013];
  phi -= m[I220] * d[I220] + m[I202] * d[I202] + m[I022] * d[I022];
  phi -= m[I211] * d[I211] + m[I121] * d[I121] + m[I112] * d[I112];
  if (o == 4) return phi;
  phi -= m[I500] * d[I500] + m[I050] * d[I050] + m[I005] * d[I005];
  phi -= m[I410] * d[I410] + m[I401] * d[I401] + m[I140] * d[I140];
  phi -= m[I104] * d[I104] + m[I041] * d[I041] + m[I014] * d[I014];
  phi -= m[I320] * d[I320] + m[I302] * d[I302] + m[I230] * d[I230];
  phi -= m[I203] * d[I203] + m[I032] * d[I032] + m[I023] * d[I023];
  phi -= m[I221] * d[I221] + m[I212] * d[I212] + m[I122] * d[I122];
  phi -= m[I311] * d[I311] + m[I131] * d[I131] + m[I113] * d[I113];
  return phi;
}

/* multipole.rs:1408-1528 (and :466-575, 919-1025) */
void pbxref_gravity_accel_multipole(const double *m, const double *d, int order, double *a) {
  int o = order < 5 ? order : 5;
  double ax = -m[I000] * d[I100];
  double ay = -m[I000] * d[I010];
  double az = -m[I000] * d[I001];
  if (o >= 2) {
    ax -= m[I100] * d[I200] + m[I010] * d[I110] + m[I001] * d[I101];
    ay -= m[I100] * d[I110] + m[I010] * d[I020] + m[I001] * d[I011];
    az -= m[I100] * d[I101] + m[I010] * d[I011] + m[I001] * d[I002];
  }
  if (o >= 3) {
    ax -= m[I200] * d[I300] + m[I020] * d[I120] + m[I002] * d[I102];
    ax -= m[I110] * d[I210] + m[I101] * d[I201] + m[I011] * d[I111];
    ay -= m[I200] * d[I210] + m[I020] * d[I030] + m[I002] * d[I012];
    ay -= m[I110] * d[I120] + m[I101] * d[I111] + m[I011] * d[I021];
    az -= m[I200] * d[I201] + m[I020] * d[I021] + m[I002] * d[I003];
    az -= m[I110] * d[I111] + m[I101] * d[I102] + m[I011] * d[I012];
  }
  if (o >= 4) {
    ax -= m[I003] * d[I103] + m[I012] * d[I112] + m[I021] * d[I121] + m[I030] * d[I130] +
          m[I102] * d[I202] + m[I111] * d[I211] + m[I120] * d[I220] + m[I201] * d[I301] +
          m[I210] * d[I310] + m[I300] * d[I400];
    ay -= m[I003] * d[I013] + m[I012] * d[I022] + m[I021] * d[I031] + m[I030] * d[I040] +
          m[I102] * d[I112] + m[I111] * d[I121] + m[I120] * d[I130] + m[I201] * d[I211] +
          m[I210] * d[I220] + m[I300] * d[I310];
    az -= m[I003] * d[I004] + m[I012] * d[I013] + m[I021] * d[I022] + m[I030] * d[I031] +
          m[I102] * d[I103] + m[I111] * d[I112] + m[I120] * d[I121] + m[I201] * d[I202] +
          m[I210] * d[I211] + m[I300] * d[I301];
  }
  if (o >= 5) {
    ax -= m[I004] * d[I104] + m[I013] * d[I113] + m[I022] * d[I122] + m[I031] * d[I131] +
          m[I040] * d[I140] + m[I103] * d[I203] + m[I112] * d[I212] + m[I121] * d[I221] +
          m[I130] * d[I230] + m[I202] * d[I302] + m[I211] * d[I311] + m[I220] * d[I320] +
          m[I301] * d[I401] + m[I310] * d[I410] + m[I400] * d[I500];
    ay -= m[I004] * d[I014] + m[I013] * d[I023] + m[I022] * d[I032] + m[I031] * d[I041] +
          m[I040] * d[I050] + m[I103] * d[I113] + m[I112] * d[I122] + m[I121] * d[I131] +
          m[I130] * d[I140] + m[I202] * d[I212] + m[I211] * d[I221] + m[I220] * d[I230] +
          m[I301] * d[I311] + m[I310] * d[I320] + m[I400] * d[I410];
    az -= m[I004] * d[I005] + m[I013] * d[I014] + m[I022] * d[I023] + m[I031] * d[I032] +
          m[I040] * d[I041] + m[I103] * d[I104] + m[I112] * d[I113] + m[I121] * d[I122] +
          m[I130] * d[I131] + m[I202] * d[I203] + m[I211] * d[I212] + m[I220] * d[I221] +
          m[I301] * d[I302] + m[I310] * d[I311] + m[I400] * d[I401];
  }
  a[0] = ax;
  a[1] = ay;
  a[2] = az;
}

/* ------------------------------------------------------------------ */
/* Octree (tree.rs:573-612)                                            */
/* ------------------------------------------------------------------ */
typedef struct {
  int64_t n;
  double *pos;   /* (n,3) owned copy */
  double *mass;  /* nullable */
  double *soft;  /* nullable */
  int64_t leaf_capacity;
  int order;     /* multipole_order as given (u8) */
  int kernel;
  /* nodes */
  int64_t nn, cap;
  double *center, *half, *size2;
  int64_t *children; /* 8 per node, NONE if absent; children[0..8]=NONE & !internal = leaf */
  unsigned char *internal;
  int64_t *ind_off, *ind_len; /* leaf particle lists, slices of perm */
  int64_t *perm;              /* leaf lists concatenated in creation order */
  int64_t perm_len;
  int64_t *first, *next;
  /* payloads */
  int has_bh;
  double *com, *bmass; /* (nn,3), (nn) */
  double *hmax;        /* nullable */
  double *mom;         /* (nn,56) nullable */
} pbxref_tree;

static void grow_nodes(pbxref_tree *t) {
  if (t->nn < t->cap) return;
  int64_t c = t->cap ? 2 * t->cap : 64;
  t->center = realloc(t->center, sizeof(double) * 3 * c);
  t->half = realloc(t->half, sizeof(double) * c);
  t->size2 = realloc(t->size2, sizeof(double) * c);
  t->children = realloc(t->children, sizeof(int64_t) * 8 * c);
  t->internal = realloc(t->internal, c);
  t->ind_off = realloc(t->ind_off, sizeof(int64_t) * c);
  t->ind_len = realloc(t->ind_len, sizeof(int64_t) * c);
  t->cap = c;
}

/* make_node (tree.rs:792-802); indices live in a scratch list passed around */
static int64_t push_node(pbxref_tree *t, const double *c, double half) {
  grow_nodes(t);
  int64_t k = t->nn++;
  double s = half * 2.0;
  t->center[3 * k + 0] = c[0];
  t->center[3 * k + 1] = c[1];
  t->center[3 * k + 2] = c[2];
  t->half[k] = half;
  t->size2[k] = s * s;
  for (int o = 0; o < 8; ++o) t->children[8 * k + o] = NONE;
  t->internal[k] = 0;
  t->ind_off[k] = -1;
  t->ind_len[k] = 0;
  return k;
}

static int all_identical(const pbxref_tree *t, const int64_t *ind, int64_t cnt) {
  for (int64_t i = 1; i < cnt; ++i)
    if (memcmp(t->pos + 3 * ind[0], t->pos + 3 * ind[i], 3 * sizeof(double)) != 0) return 0;
  return 1;
}

/* build_recursive + subdivide_node (tree.rs:804-864).  `ind` is this
 * node's index list (ascending bucket order, as the Rust Vec<usize>). */
static void build_rec(pbxref_tree *t, int64_t k, int64_t *ind, int64_t cnt) {
  if (cnt <= t->leaf_capacity || all_identical(t, ind, cnt) || t->half[k] == 0.0) {
    /* leaf: record its list in perm */
    t->ind_off[k] = t->perm_len;
    t->ind_len[k] = cnt;
    memcpy(t->perm + t->perm_len, ind, sizeof(int64_t) * cnt);
    t->perm_len += cnt;
    return;
  }
  double c[3] = {t->center[3 * k], t->center[3 * k + 1], t->center[3 * k + 2]};
  double half = t->half[k];
  int64_t bcount[8] = {0};
  unsigned char *oct = malloc(cnt ? cnt : 1);
  for (int64_t i = 0; i < cnt; ++i) {
    const double *p = t->pos + 3 * ind[i];
    int o = 0;
    if (p[0] >= c[0]) o |= 1;
    if (p[1] >= c[1]) o |= 2;
    if (p[2] >= c[2]) o |= 4;
    oct[i] = (unsigned char)o;
    bcount[o]++;
  }
  int64_t *buckets[8];
  int64_t fill[8] = {0};
  for (int o = 0; o < 8; ++o) buckets[o] = bcount[o] ? malloc(sizeof(int64_t) * bcount[o]) : NULL;
  for (int64_t i = 0; i < cnt; ++i) buckets[oct[i]][fill[oct[i]]++] = ind[i];
  free(oct);
  t->internal[k] = 1;
  int64_t kids[8];
  for (int o = 0; o < 8; ++o) {
    kids[o] = NONE;
    if (!bcount[o]) continue;
    double cc[3] = {c[0], c[1], c[2]};
    double offset = half / 2.0;
    cc[0] += (o & 1) ? offset : -offset;
    cc[1] += (o & 2) ? offset : -offset;
    cc[2] += (o & 4) ? offset : -offset;
    kids[o] = push_node(t, cc, offset);
  }
  for (int o = 0; o < 8; ++o) t->children[8 * k + o] = kids[o];
  for (int o = 0; o < 8; ++o) {
    if (kids[o] == NONE) continue;
    build_rec(t, kids[o], buckets[o], bcount[o]);
    free(buckets[o]);
  }
}

/* build_treewalk_links (tree.rs:736-776) */
static void links_rec(pbxref_tree *t, int64_t k) {
  if (!t->internal[k]) return;
  int64_t last = NONE;
  for (int o = 0; o < 8; ++o) {
    int64_t c = t->children[8 * k + o];
    if (c == NONE) continue;
    if (t->first[k] == NONE) t->first[k] = c;
    if (last != NONE) t->next[last] = c;
    last = c;
  }
  if (last != NONE) t->next[last] = t->next[k];
  for (int o = 0; o < 8; ++o) {
    int64_t c = t->children[8 * k + o];
    if (c == NONE) continue;
    if (t->internal[c]) links_rec(t, c);
  }
}

static double *dup(const double *a, int64_t n) {
  if (!a) return NULL;
  double *b = malloc(sizeof(double) * (n ? n : 1));
  memcpy(b, a, sizeof(double) * n);
  return b;
}

/* Octree::from_owned (tree.rs:658-734) incl. bbox_of_points (:628-654) */
pbxref_tree *pbxref_tree_new(const double *pos, int64_t n, const double *mass,
                             const double *soft, int64_t leaf_capacity, int order, int kernel) {
  pbxref_tree *t = calloc(1, sizeof(pbxref_tree));
  t->n = n;
  t->pos = dup(pos, 3 * n);
  t->mass = dup(mass, n);
  t->soft = dup(soft, n);
  t->leaf_capacity = leaf_capacity < 1 ? 1 : leaf_capacity;
  t->order = order;
  t->kernel = kernel;
  double minp[3] = {INFINITY, INFINITY, INFINITY};
  double maxp[3] = {-INFINITY, -INFINITY, -INFINITY};
  for (int64_t i = 0; i < n; ++i)
    for (int d = 0; d < 3; ++d) {
      double v = pos[3 * i + d];
      if (v < minp[d]) minp[d] = v;
      if (v > maxp[d]) maxp[d] = v;
    }
  double center[3] = {(minp[0] + maxp[0]) / 2.0, (minp[1] + maxp[1]) / 2.0,
                      (minp[2] + maxp[2]) / 2.0};
  double half = 0.0;
  for (int d = 0; d < 3; ++d) half = fmax(half, (maxp[d] - minp[d]) / 2.0);
  if (half == 0.0) half = 1e-6;
  t->perm = malloc(sizeof(int64_t) * (n ? n : 1));
  int64_t *ind = malloc(sizeof(int64_t) * (n ? n : 1));
  for (int64_t i = 0; i < n; ++i) ind[i] = i;
  push_node(t, center, half);
  build_rec(t, 0, ind, n);
  free(ind);
  t->first = malloc(sizeof(int64_t) * t->nn);
  t->next = malloc(sizeof(int64_t) * t->nn);
  for (int64_t k = 0; k < t->nn; ++k) t->first[k] = t->next[k] = NONE;
  t->next[0] = NONE;
  links_rec(t, 0);
  return t;
}

void pbxref_tree_free(pbxref_tree *t) {
  if (!t) return;
  free(t->pos); free(t->mass); free(t->soft);
  free(t->center); free(t->half); free(t->size2); free(t->children); free(t->internal);
  free(t->ind_off); free(t->ind_len); free(t->perm); free(t->first); free(t->next);
  free(t->com); free(t->bmass); free(t->hmax); free(t->mom);
  free(t);
}

/* build_mass_payload (tree.rs:968-1012) = BH (:866-932) + h_max (:941-965)
 * + multipoles (:1014-1067) */
void pbxref_tree_build_mass_payload(pbxref_tree *t) {
  int64_t nn = t->nn;
  free(t->com); free(t->bmass); free(t->hmax); free(t->mom);
  t->com = calloc(3 * nn, sizeof(double));
  t->bmass = calloc(nn, sizeof(double));
  t->hmax = NULL;
  t->mom = NULL;
  for (int64_t k = nn - 1; k >= 0; --k) {
    double mass = 0.0, com[3] = {0.0, 0.0, 0.0};
    if (!t->internal[k]) {
      const int64_t *ind = t->perm + t->ind_off[k];
      int64_t cnt = t->ind_len[k];
      if (cnt > 0) {
        for (int64_t i = 0; i < cnt; ++i) {
          const double *p = t->pos + 3 * ind[i];
          if (t->mass) {
            double m = t->mass[ind[i]];
            mass += m;
            com[0] += p[0] * m;
            com[1] += p[1] * m;
            com[2] += p[2] * m;
          } else {
            mass += 1.0;
            com[0] += p[0];
            com[1] += p[1];
            com[2] += p[2];
          }
        }
        if (mass > 0.0) {
          com[0] /= mass;
          com[1] /= mass;
          com[2] /= mass;
        }
      }
    } else {
      for (int o = 0; o < 8; ++o) {
        int64_t c = t->children[8 * k + o];
        if (c == NONE) continue;
        double cm = t->bmass[c];
        if (cm == 0.0) continue;
        mass += cm;
        com[0] += t->com[3 * c + 0] * cm;
        com[1] += t->com[3 * c + 1] * cm;
        com[2] += t->com[3 * c + 2] * cm;
      }
      if (mass > 0.0) {
        com[0] /= mass;
        com[1] /= mass;
        com[2] /= mass;
      }
    }
    t->bmass[k] = mass;
    t->com[3 * k + 0] = com[0];
    t->com[3 * k + 1] = com[1];
    t->com[3 * k + 2] = com[2];
  }
  t->has_bh = 1;
  if (t->soft) {
    t->hmax = calloc(nn, sizeof(double));
    for (int64_t k = nn - 1; k >= 0; --k) {
      double m = 0.0;
      if (!t->internal[k]) {
        const int64_t *ind = t->perm + t->ind_off[k];
        for (int64_t i = 0; i < t->ind_len[k]; ++i) m = fmax(m, fmax(t->soft[ind[i]], 0.0));
      } else {
        for (int o = 0; o < 8; ++o) {
          int64_t c = t->children[8 * k + o];
          if (c != NONE) m = fmax(m, t->hmax[c]);
        }
      }
      t->hmax[k] = m;
    }
  }
  if (t->order > 0) {
    int order = t->order < 5 ? t->order : 5;
    t->mom = calloc((size_t)nn * NMOM, sizeof(double));
    double tr[NMOM];
    for (int64_t k = nn - 1; k >= 0; --k) {
      if (t->bmass[k] == 0.0) continue;
      double *mk = t->mom + (size_t)k * NMOM;
      const double *cen = t->com + 3 * k;
      if (!t->internal[k]) {
        if (t->ind_len[k] == 0) continue;
        pbxref_multipole_from_points(t->pos, t->mass, t->perm + t->ind_off[k], t->ind_len[k],
                                     cen, order, mk);
      } else {
        for (int o = 0; o < 8; ++o) {
          int64_t c = t->children[8 * k + o];
          if (c == NONE || t->bmass[c] == 0.0) continue;
          double shift[3] = {cen[0] - t->com[3 * c + 0], cen[1] - t->com[3 * c + 1],
                             cen[2] - t->com[3 * c + 2]};
          pbxref_translate_multipole(t->mom + (size_t)c * NMOM, shift, order, tr);
          for (int s = 0; s < NMOM; ++s) mk[s] += tr[s];
        }
      }
    }
  }
}

/* set_masses + build (PyO3 build_mass, gravity.rs:228-239) */
void pbxref_tree_build_mass(pbxref_tree *t, const double *mass) {
  if (mass) {
    free(t->mass);
    t->mass = dup(mass, t->n);
  }
  pbxref_tree_build_mass_payload(t);
}

void pbxref_tree_set_softenings(pbxref_tree *t, const double *soft) {
  free(t->soft);
  t->soft = dup(soft, t->n);
}

void pbxref_tree_set_kernel(pbxref_tree *t, int kernel) { t->kernel = kernel; }
int pbxref_tree_has_bh(const pbxref_tree *t) { return t->has_bh; }
int64_t pbxref_tree_num_nodes(const pbxref_tree *t) { return t->nn; }

/* ------------------------------------------------------------------ */
/* traversal (tree.rs:34-71, 98-417, 1069-1391)                        */
/* ------------------------------------------------------------------ */
static inline double inv_r_from_r2(double r2) {
  double s2 = r2 + R2_TINY;
  return 1.0 / sqrt(s2);
}

static inline double inv_r3_from_r2(double r2) {
  double s2 = r2 + R2_TINY;
  double inv_r = 1.0 / sqrt(s2);
  double inv_r2 = inv_r * inv_r;
  return inv_r2 * inv_r;
}

static inline int node_soft_ok(const pbxref_tree *t, int64_t k, double dist2, int has_th,
                               double th) {
  if (!t->hmax) return 1;
  double h = fmax(t->hmax[k], 0.0);
  if (has_th) h = fmax(h, fmax(th, 0.0));
  if (h <= 0.0) return 1;
  double c = t->kernel == K_PLUMMER ? 2.8 : 1.0;
  double ch = c * h;
  return dist2 > ch * ch;
}

/* leaf_potential_sum (tree.rs:98-277) */
static void leaf_pot(const pbxref_tree *t, int64_t k, const double *tg, int64_t skip,
                     int has_th, double th, double *out) {
  const int64_t *ind = t->perm + t->ind_off[k];
  int64_t cnt = t->ind_len[k];
  double tx = tg[0], ty = tg[1], tz = tg[2];
  double target_h = fmax(has_th ? th : 0.0, 0.0);
  int use_soft = t->soft != NULL || target_h > 0.0;
  const double *P = t->pos;
  if (use_soft && t->mass && !t->soft) { /* constant-target-h fast path :122-170 */
    double h = target_h;
    if (h <= 0.0) {
      /* falls through to the general logic below */
    } else if (t->kernel == K_SPLINE) {
      double hh = h * h;
      for (int64_t i = 0; i < cnt; ++i) {
        int64_t pi = ind[i];
        if (pi == skip) continue;
        double ddx = P[3 * pi] - tx, ddy = P[3 * pi + 1] - ty, ddz = P[3 * pi + 2] - tz;
        double r2 = fma(ddx, ddx, fma(ddy, ddy, ddz * ddz));
        double m = t->mass[pi];
        if (r2 >= hh) {
          *out += -m * inv_r_from_r2(r2);
        } else {
          double r = sqrt(r2 + R2_TINY);
          *out += m * pbxref_kernel_potential(t->kernel, r, h);
        }
      }
      return;
    } else {
      for (int64_t i = 0; i < cnt; ++i) {
        int64_t pi = ind[i];
        if (pi == skip) continue;
        double ddx = P[3 * pi] - tx, ddy = P[3 * pi + 1] - ty, ddz = P[3 * pi + 2] - tz;
        double r2 = fma(ddx, ddx, fma(ddy, ddy, ddz * ddz));
        double r = sqrt(r2 + R2_TINY);
        *out += t->mass[pi] * pbxref_kernel_potential(t->kernel, r, h);
      }
      return;
    }
  }
  if (!use_soft) {
    for (int64_t i = 0; i < cnt; ++i) {
      int64_t pi = ind[i];
      if (pi == skip) continue;
      double ddx = P[3 * pi] - tx, ddy = P[3 * pi + 1] - ty, ddz = P[3 * pi + 2] - tz;
      double r2 = fma(ddx, ddx, fma(ddy, ddy, ddz * ddz));
      double inv_r = inv_r_from_r2(r2);
      if (t->mass)
        *out += -t->mass[pi] * inv_r;
      else
        *out += -inv_r;
    }
    return;
  }
  int spline = t->kernel == K_SPLINE;
  for (int64_t i = 0; i < cnt; ++i) {
    int64_t pi = ind[i];
    if (pi == skip) continue;
    double ddx = P[3 * pi] - tx, ddy = P[3 * pi + 1] - ty, ddz = P[3 * pi + 2] - tz;
    double r2 = fma(ddx, ddx, fma(ddy, ddy, ddz * ddz));
    double m = t->mass ? t->mass[pi] : 1.0;
    double h;
    if (t->soft) {
      double hi = fmax(t->soft[pi], 0.0);
      h = fmax(hi, target_h);
    } else {
      h = target_h;
    }
    if (h <= 0.0 || (spline && r2 >= h * h)) {
      *out += -m * inv_r_from_r2(r2);
    } else {
      double r = sqrt(r2 + R2_TINY);
      *out += m * pbxref_kernel_potential(t->kernel, r, h);
    }
  }
}

/* leaf_acceleration_sum (tree.rs:280-417) */
static void leaf_acc(const pbxref_tree *t, int64_t k, const double *tg, int64_t skip,
                     int has_th, double th, double *out) {
  const int64_t *ind = t->perm + t->ind_off[k];
  int64_t cnt = t->ind_len[k];
  double tx = tg[0], ty = tg[1], tz = tg[2];
  double target_h = fmax(has_th ? th : 0.0, 0.0);
  int use_soft = t->soft != NULL || target_h > 0.0;
  const double *P = t->pos;
  if (!use_soft) {
    for (int64_t i = 0; i < cnt; ++i) {
      int64_t pi = ind[i];
      if (pi == skip) continue;
      double ddx = P[3 * pi] - tx, ddy = P[3 * pi + 1] - ty, ddz = P[3 * pi + 2] - tz;
      double r2 = fma(ddx, ddx, fma(ddy, ddy, ddz * ddz));
      double inv_r3 = inv_r3_from_r2(r2);
      if (t->mass) {
        double m = t->mass[pi];
        out[0] += m * ddx * inv_r3;
        out[1] += m * ddy * inv_r3;
        out[2] += m * ddz * inv_r3;
      } else {
        out[0] += ddx * inv_r3;
        out[1] += ddy * inv_r3;
        out[2] += ddz * inv_r3;
      }
    }
    return;
  }
  int spline = t->kernel == K_SPLINE;
  for (int64_t i = 0; i < cnt; ++i) {
    int64_t pi = ind[i];
    if (pi == skip) continue;
    double ddx = P[3 * pi] - tx, ddy = P[3 * pi + 1] - ty, ddz = P[3 * pi + 2] - tz;
    double r2 = fma(ddx, ddx, fma(ddy, ddy, ddz * ddz));
    double m = t->mass ? t->mass[pi] : 1.0;
    double h;
    if (t->soft) {
      double hi = fmax(t->soft[pi], 0.0);
      h = fmax(hi, target_h);
    } else {
      h = target_h;
    }
    if (h <= 0.0 || (spline && r2 >= h * h)) {
      double inv_r3 = inv_r3_from_r2(r2);
      out[0] += m * ddx * inv_r3;
      out[1] += m * ddy * inv_r3;
      out[2] += m * ddz * inv_r3;
    } else {
      double r = sqrt(r2 + R2_TINY);
      double g = pbxref_kernel_accel_factor(t->kernel, r, h);
      out[0] += m * ddx * g;
      out[1] += m * ddy * g;
      out[2] += m * ddz * g;
    }
  }
}

/* One target: potential_traversal_cached_{no_,with_}multipoles
 * (tree.rs:1069-1206) and acceleration_traversal_cached_* (:1228-1370).
 * want: 1 = potential, 2 = acceleration.  Returns the number of accepted
 * nodes + leaf particles visited in *work (for interaction counting). */
static void walk(const pbxref_tree *t, double theta2, const double *tg, int64_t skip, int has_th,
                 double th, int want, double *pot, double *acc, int64_t *n_node,
                 int64_t *n_pp) {
  int softening_enabled = t->hmax != NULL || has_th;
  int use_mp = t->mom != NULL;
  int order = t->order < 5 ? t->order : 5;
  double tx = tg[0], ty = tg[1], tz = tg[2];
  double d[NMOM], a[3];
  int64_t k = 0;
  while (k != NONE) {
    if (t->bmass[k] == 0.0) {
      k = t->next[k];
      continue;
    }
    if (!t->internal[k]) {
      if (want & 1) leaf_pot(t, k, tg, skip, has_th, th, pot);
      if (want & 2) leaf_acc(t, k, tg, skip, has_th, th, acc);
      if (n_pp) *n_pp += t->ind_len[k];
      k = t->next[k];
      continue;
    }
    const double *com = t->com + 3 * k;
    double dx = com[0] - tx, dy = com[1] - ty, dz = com[2] - tz;
    double dist2 = fma(dx, dx, fma(dy, dy, dz * dz)) + R2_TINY;
    int soft_ok = softening_enabled ? node_soft_ok(t, k, dist2, has_th, th) : 1;
    if (soft_ok && t->size2[k] < theta2 * dist2) {
      if (!use_mp) {
        double inv_r = inv_r_from_r2(dist2);
        if (want & 1) *pot += -t->bmass[k] * inv_r;
        if (want & 2) {
          double inv_r2 = inv_r * inv_r;
          double inv_r3 = inv_r2 * inv_r;
          acc[0] += t->bmass[k] * dx * inv_r3;
          acc[1] += t->bmass[k] * dy * inv_r3;
          acc[2] += t->bmass[k] * dz * inv_r3;
        }
      } else {
        /* order 1 is stored as O0 (multipole.rs:272) */
        int eo = order <= 1 ? 0 : order;
        pbxref_potential_derivatives(dx, dy, dz, R2_TINY, eo == 0 ? 1 : eo, d);
        const double *m = t->mom + (size_t)k * NMOM;
        if (want & 1) *pot += pbxref_gravity_potential_multipole(m, d, eo);
        if (want & 2) {
          pbxref_gravity_accel_multipole(m, d, eo, a);
          acc[0] += a[0];
          acc[1] += a[1];
          acc[2] += a[2];
        }
      }
      if (n_node) *n_node += 1;
      k = t->next[k];
    } else {
      k = t->first[k];
    }
  }
}

/* Tree3D::compute_potentials / compute_accelerations (tree.rs:1415-1496):
 * skip_self = i, target_h = softenings[i] when softenings are set. */
void pbxref_tree_compute(const pbxref_tree *t, double theta, int want, double *pot,
                         double *acc) {
  double theta2 = theta * theta;
#pragma omp parallel for schedule(dynamic, 64)
  for (int64_t i = 0; i < t->n; ++i) {
    double p = 0.0, a[3] = {0.0, 0.0, 0.0};
    int has_th = t->soft != NULL;
    double th = has_th ? t->soft[i] : 0.0;
    walk(t, theta2, t->pos + 3 * i, i, has_th, th, want, &p, a, NULL, NULL);
    if (want & 1) pot[i] = p;
    if (want & 2) {
      acc[3 * i + 0] = a[0];
      acc[3 * i + 1] = a[1];
      acc[3 * i + 2] = a[2];
    }
  }
}

/* Same walk for a list of target indices (CPU baseline / large-N parity on
 * a subset; each target's result equals the full call's). */
void pbxref_tree_compute_subset(const pbxref_tree *t, double theta, int want,
                                const int64_t *idx, int64_t k, double *pot, double *acc,
                                int64_t *n_node, int64_t *n_pp) {
  double theta2 = theta * theta;
#pragma omp parallel for schedule(dynamic, 16)
  for (int64_t s = 0; s < k; ++s) {
    int64_t i = idx[s];
    double p = 0.0, a[3] = {0.0, 0.0, 0.0};
    int has_th = t->soft != NULL;
    double th = has_th ? t->soft[i] : 0.0;
    int64_t nn = 0, np = 0;
    walk(t, theta2, t->pos + 3 * i, i, has_th, th, want, &p, a, &nn, &np);
    if (pot) pot[s] = p;
    if (acc) {
      acc[3 * s + 0] = a[0];
      acc[3 * s + 1] = a[1];
      acc[3 * s + 2] = a[2];
    }
    if (n_node) n_node[s] = nn;
    if (n_pp) n_pp[s] = np;
  }
}

/* Tree3D::{accelerations,potentials}_at_points (tree.rs:1498-1558):
 * skip_self = None, target_h = None. */
void pbxref_tree_at_points(const pbxref_tree *t, const double *pts, int64_t m, double theta,
                           int want, double *pot, double *acc) {
  double theta2 = theta * theta;
#pragma omp parallel for schedule(dynamic, 64)
  for (int64_t i = 0; i < m; ++i) {
    double p = 0.0, a[3] = {0.0, 0.0, 0.0};
    walk(t, theta2, pts + 3 * i, NONE, 0, 0.0, want, &p, a, NULL, NULL);
    if (want & 1) pot[i] = p;
    if (want & 2) {
      acc[3 * i + 0] = a[0];
      acc[3 * i + 1] = a[1];
      acc[3 * i + 2] = a[2];
    }
  }
}

/* ------------------------------------------------------------------ */
/* export (for geometry / payload parity checks)                        */
/* ------------------------------------------------------------------ */
void pbxref_tree_export(const pbxref_tree *t, double *center, double *half, double *size2,
                        int64_t *first, int64_t *next, int64_t *leaf_off, int64_t *leaf_len,
                        double *com, double *mass, double *hmax, double *mom, int64_t *perm) {
  int64_t nn = t->nn;
  if (center) memcpy(center, t->center, sizeof(double) * 3 * nn);
  if (half) memcpy(half, t->half, sizeof(double) * nn);
  if (size2) memcpy(size2, t->size2, sizeof(double) * nn);
  if (first) memcpy(first, t->first, sizeof(int64_t) * nn);
  if (next) memcpy(next, t->next, sizeof(int64_t) * nn);
  for (int64_t k = 0; k < nn; ++k) {
    if (leaf_off) leaf_off[k] = t->internal[k] ? -1 : t->ind_off[k];
    if (leaf_len) leaf_len[k] = t->internal[k] ? 0 : t->ind_len[k];
  }
  if (com && t->com) memcpy(com, t->com, sizeof(double) * 3 * nn);
  if (mass && t->bmass) memcpy(mass, t->bmass, sizeof(double) * nn);
  if (hmax && t->hmax) memcpy(hmax, t->hmax, sizeof(double) * nn);
  if (mom && t->mom) memcpy(mom, t->mom, sizeof(double) * NMOM * nn);
  if (perm) memcpy(perm, t->perm, sizeof(int64_t) * t->perm_len);
}

int pbxref_tree_has_hmax(const pbxref_tree *t) { return t->hmax != NULL; }
int pbxref_tree_has_moments(const pbxref_tree *t) { return t->mom != NULL; }
