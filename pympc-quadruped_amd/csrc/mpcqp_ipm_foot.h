// mpcqp_ipm_foot.h -- per-foot-step algebra of the interior-point class
// (mpcqp_ipm.h), host- and device-callable so tests/ can check it on the CPU.
#pragma once
#include <math.h>

#ifndef __HIPCC__
#define __host__
#define __device__
#endif

// 3x3 inverse by the adjugate (symmetric positive definite arguments)
__host__ __device__ inline void inv3(const double (&a)[9], double (&o)[9]) {
  const double c00 = a[4] * a[8] - a[5] * a[7], c01 = a[5] * a[6] - a[3] * a[8], c02 = a[3] * a[7] - a[4] * a[6];
  const double det = a[0] * c00 + a[1] * c01 + a[2] * c02;
  const double id = 1.0 / det;
  o[0] = c00 * id;
  o[3] = c01 * id;
  o[6] = c02 * id;
  o[1] = (a[2] * a[7] - a[1] * a[8]) * id;
  o[4] = (a[0] * a[8] - a[2] * a[6]) * id;
  o[7] = (a[1] * a[6] - a[0] * a[7]) * id;
  o[2] = (a[1] * a[5] - a[2] * a[4]) * id;
  o[5] = (a[2] * a[3] - a[0] * a[5]) * id;
  o[8] = (a[0] * a[4] - a[1] * a[3]) * id;
}

// Multipliers of one foot-step: the largest min_r lambda_r over the linearly
// independent nq-subsets of the active rows `am` (bit r = row r) with
// g = sum lambda_r a_r (Caratheodory: g is in the cone of the active rows iff some such
// subset has lambda >= 0).  best = -inf when no subset reproduces g; drop = the row of
// the best subset's most negative multiplier when best < -tol.
__host__ __device__ inline void ipm_cone_multipliers(const double (&rw)[6][3], int am, int nq, const double (&g)[3],
                                                     double tol, double& best, int& drop) {
  best = -INFINITY;
  drop = -1;
  for (int r1 = 0; r1 < 6; ++r1) {
    if (!((am >> r1) & 1)) continue;
    for (int r2 = nq >= 2 ? r1 + 1 : 6; r2 < 6 || nq < 2; ++r2) {
      if (nq >= 2 && !((am >> r2) & 1)) continue;
      for (int r3 = nq >= 3 ? r2 + 1 : 6; r3 < 6 || nq < 3; ++r3) {
        if (nq >= 3 && !((am >> r3) & 1)) continue;
        // rows of the subset (unused slots: zero rows, identity Gram entries)
        const double* a1 = rw[r1];
        const double* a2 = nq >= 2 ? rw[r2] : nullptr;
        const double* a3 = nq >= 3 ? rw[r3] : nullptr;
        double gm[9] = {1.0, 0.0, 0.0, 0.0, 1.0, 0.0, 0.0, 0.0, 1.0}, gi[9];
        double b1 = a1[0] * g[0] + a1[1] * g[1] + a1[2] * g[2], b2 = 0.0, b3 = 0.0;
        gm[0] = a1[0] * a1[0] + a1[1] * a1[1] + a1[2] * a1[2];
        if (a2) {
          b2 = a2[0] * g[0] + a2[1] * g[1] + a2[2] * g[2];
          gm[1] = gm[3] = a1[0] * a2[0] + a1[1] * a2[1] + a1[2] * a2[2];
          gm[4] = a2[0] * a2[0] + a2[1] * a2[1] + a2[2] * a2[2];
        }
        if (a3) {
          b3 = a3[0] * g[0] + a3[1] * g[1] + a3[2] * g[2];
          gm[2] = gm[6] = a1[0] * a3[0] + a1[1] * a3[1] + a1[2] * a3[2];
          gm[5] = gm[7] = a2[0] * a3[0] + a2[1] * a3[1] + a2[2] * a3[2];
          gm[8] = a3[0] * a3[0] + a3[1] * a3[1] + a3[2] * a3[2];
        }
        const double det = gm[0] * (gm[4] * gm[8] - gm[5] * gm[7]) - gm[1] * (gm[3] * gm[8] - gm[5] * gm[6]) +
                           gm[2] * (gm[3] * gm[7] - gm[4] * gm[6]);
        if (fabs(det) > 1e-10) {
          inv3(gm, gi);
          const double l1 = gi[0] * b1 + gi[1] * b2 + gi[2] * b3;
          const double l2 = gi[3] * b1 + gi[4] * b2 + gi[5] * b3;
          const double l3 = gi[6] * b1 + gi[7] * b2 + gi[8] * b3;
          double res = 0.0;
          for (int x = 0; x < 3; ++x) {
            double v = g[x] - l1 * a1[x];
            if (a2) v -= l2 * a2[x];
            if (a3) v -= l3 * a3[x];
            res = fmax(res, fabs(v));
          }
          if (res <= tol) {
            double mn = l1;
            int am_r = r1;
            if (a2 && l2 < mn) { mn = l2; am_r = r2; }
            if (a3 && l3 < mn) { mn = l3; am_r = r3; }
            if (mn > best) {
              best = mn;
              drop = mn < -tol ? am_r : -1;
            }
          }
        }
        if (nq < 3) break;
      }
      if (nq < 2) break;
    }
  }
}


// Null space of a foot-step's active cone rows `am` (bit r = row r, rows[6][3]) for
// the polish: Gram-Schmidt in the order 5, 0, 1, 2, 3, 4 (row 5, -n.f >= -ub, is the
// only one with a non-zero right-hand side h5), dependent rows skipped.  Outputs the
// projector pj = I - sum q q^T onto the null space, the minimum-norm particular
// solution fp of the independent active rows (a_r . fp = h_r), and the weight
// W = pj (pj Rh pj + I - pj)^-1 pj of the reduced stage problem (rh: the leg's 3
// diagonal input weights).  Returns the rank (0..3).
__host__ __device__ inline int ipm_foot_nullspace(const double (&rw)[6][3], int am, double h5, const double (&rh)[3],
                                                  double (&pj)[9], double (&fp)[3], double (&W)[9]) {
  double q0[3] = {0.0, 0.0, 0.0}, q1[3] = {0.0, 0.0, 0.0}, q2[3] = {0.0, 0.0, 0.0};
  double c0 = 0.0, c1 = 0.0, c2 = 0.0;   // L c = h over the independent rows (forward substitution)
  int nq = 0;
  for (int o = 0; o < 6; ++o) {
    const int r = o == 0 ? 5 : o - 1;
    if (!((am >> r) & 1) || nq == 3) continue;
    double v[3] = {rw[r][0], rw[r][1], rw[r][2]};
    const double n0 = sqrt(v[0] * v[0] + v[1] * v[1] + v[2] * v[2]);
    const double hr = r == 5 ? h5 : 0.0;
    double l0 = 0.0, l1 = 0.0;
    if (nq >= 1) {
      l0 = q0[0] * v[0] + q0[1] * v[1] + q0[2] * v[2];
      for (int x = 0; x < 3; ++x) v[x] -= l0 * q0[x];
    }
    if (nq >= 2) {
      l1 = q1[0] * v[0] + q1[1] * v[1] + q1[2] * v[2];
      for (int x = 0; x < 3; ++x) v[x] -= l1 * q1[x];
    }
    const double nv = sqrt(v[0] * v[0] + v[1] * v[1] + v[2] * v[2]);
    if (!(nv > 1e-9 * n0)) continue;   // dependent on the rows already taken
    if (nq == 0) {
      for (int x = 0; x < 3; ++x) q0[x] = v[x] / nv;
      c0 = hr / nv;
    } else if (nq == 1) {
      for (int x = 0; x < 3; ++x) q1[x] = v[x] / nv;
      c1 = (hr - l0 * c0) / nv;
    } else {
      for (int x = 0; x < 3; ++x) q2[x] = v[x] / nv;
      c2 = (hr - l0 * c0 - l1 * c1) / nv;
    }
    ++nq;
  }
  for (int x = 0; x < 3; ++x) {
    fp[x] = c0 * q0[x] + c1 * q1[x] + c2 * q2[x];
    for (int y = 0; y < 3; ++y)
      pj[3 * x + y] = ((x == y) ? 1.0 : 0.0) - q0[x] * q0[y] - q1[x] * q1[y] - q2[x] * q2[y];
  }
  double a[9], o[9], t[9];
  for (int x = 0; x < 3; ++x)
    for (int y = 0; y < 3; ++y) {
      double v = ((x == y) ? 1.0 : 0.0) - pj[3 * x + y];
      for (int z = 0; z < 3; ++z) v += pj[3 * x + z] * rh[z] * pj[3 * z + y];
      a[3 * x + y] = v;
    }
  inv3(a, o);
  for (int x = 0; x < 3; ++x)
    for (int y = 0; y < 3; ++y) t[3 * x + y] = o[3 * x] * pj[y] + o[3 * x + 1] * pj[3 + y] + o[3 * x + 2] * pj[6 + y];
  for (int x = 0; x < 3; ++x)
    for (int y = 0; y < 3; ++y)
      W[3 * x + y] = pj[3 * x] * t[y] + pj[3 * x + 1] * t[3 + y] + pj[3 * x + 2] * t[6 + y];
  return nq;
}

// Interior-point weight of a foot-step: W = (diag(rh) + sum_r d_r a_r a_r^T)^-1 over the
// rows in `live` (bit r).
__host__ __device__ inline void ipm_foot_weight(const double (&rw)[6][3], int live, const double (&d)[6],
                                                const double (&rh)[3], double (&W)[9]) {
  double a[9];
  for (int x = 0; x < 3; ++x)
    for (int y = 0; y < 3; ++y) {
      double v = (x == y) ? rh[x] : 0.0;
      for (int r = 0; r < 6; ++r)
        if ((live >> r) & 1) v += d[r] * rw[r][x] * rw[r][y];
      a[3 * x + y] = v;
    }
  inv3(a, W);
}

// ipm_foot_nullspace with the leg's full 3 x 3 block of the input weights (row-major;
// mpcqp_set_weights): W = pj (pj Rh pj + I - pj)^-1 pj.
__host__ __device__ inline int ipm_foot_nullspace(const double (&rw)[6][3], int am, double h5, const double (&rh)[9],
                                                  double (&pj)[9], double (&fp)[3], double (&W)[9]) {
  double q0[3] = {0.0, 0.0, 0.0}, q1[3] = {0.0, 0.0, 0.0}, q2[3] = {0.0, 0.0, 0.0};
  double c0 = 0.0, c1 = 0.0, c2 = 0.0;   // L c = h over the independent rows (forward substitution)
  int nq = 0;
  for (int o = 0; o < 6; ++o) {
    const int r = o == 0 ? 5 : o - 1;
    if (!((am >> r) & 1) || nq == 3) continue;
    double v[3] = {rw[r][0], rw[r][1], rw[r][2]};
    const double n0 = sqrt(v[0] * v[0] + v[1] * v[1] + v[2] * v[2]);
    const double hr = r == 5 ? h5 : 0.0;
    double l0 = 0.0, l1 = 0.0;
    if (nq >= 1) {
      l0 = q0[0] * v[0] + q0[1] * v[1] + q0[2] * v[2];
      for (int x = 0; x < 3; ++x) v[x] -= l0 * q0[x];
    }
    if (nq >= 2) {
      l1 = q1[0] * v[0] + q1[1] * v[1] + q1[2] * v[2];
      for (int x = 0; x < 3; ++x) v[x] -= l1 * q1[x];
    }
    const double nv = sqrt(v[0] * v[0] + v[1] * v[1] + v[2] * v[2]);
    if (!(nv > 1e-9 * n0)) continue;   // dependent on the rows already taken
    if (nq == 0) {
      for (int x = 0; x < 3; ++x) q0[x] = v[x] / nv;
      c0 = hr / nv;
    } else if (nq == 1) {
      for (int x = 0; x < 3; ++x) q1[x] = v[x] / nv;
      c1 = (hr - l0 * c0) / nv;
    } else {
      for (int x = 0; x < 3; ++x) q2[x] = v[x] / nv;
      c2 = (hr - l0 * c0 - l1 * c1) / nv;
    }
    ++nq;
  }
  for (int x = 0; x < 3; ++x) {
    fp[x] = c0 * q0[x] + c1 * q1[x] + c2 * q2[x];
    for (int y = 0; y < 3; ++y)
      pj[3 * x + y] = ((x == y) ? 1.0 : 0.0) - q0[x] * q0[y] - q1[x] * q1[y] - q2[x] * q2[y];
  }
  double a[9], o[9], t[9];
  for (int x = 0; x < 3; ++x)
    for (int y = 0; y < 3; ++y) {
      double v = ((x == y) ? 1.0 : 0.0) - pj[3 * x + y];
      for (int z = 0; z < 3; ++z)
        for (int w = 0; w < 3; ++w) v += pj[3 * x + z] * rh[3 * z + w] * pj[3 * w + y];
      a[3 * x + y] = v;
    }
  inv3(a, o);
  for (int x = 0; x < 3; ++x)
    for (int y = 0; y < 3; ++y) t[3 * x + y] = o[3 * x] * pj[y] + o[3 * x + 1] * pj[3 + y] + o[3 * x + 2] * pj[6 + y];
  for (int x = 0; x < 3; ++x)
    for (int y = 0; y < 3; ++y)
      W[3 * x + y] = pj[3 * x] * t[y] + pj[3 * x + 1] * t[3 + y] + pj[3 * x + 2] * t[6 + y];
  return nq;
}

// The same with the leg's full 3 x 3 block of the input weights (row-major; mpcqp_set_weights).
__host__ __device__ inline void ipm_foot_weight(const double (&rw)[6][3], int live, const double (&d)[6],
                                                const double (&rh)[9], double (&W)[9]) {
  double a[9];
  for (int x = 0; x < 3; ++x)
    for (int y = 0; y < 3; ++y) {
      double v = rh[3 * x + y];
      for (int r = 0; r < 6; ++r)
        if ((live >> r) & 1) v += d[r] * rw[r][x] * rw[r][y];
      a[3 * x + y] = v;
    }
  inv3(a, W);
}

// G^T D G of a foot-step: sum_r d_r a_r a_r^T over the rows in `live` (bit r) -- the block a
// cross-leg R's stage weight adds on the foot's leg before the stage inversion (mpcqp_ipm.h).
__host__ __device__ inline void ipm_foot_gdg(const double (&rw)[6][3], int live, const double (&d)[6], double (&o)[9]) {
  for (int x = 0; x < 3; ++x)
    for (int y = 0; y < 3; ++y) {
      double v = 0.0;
      for (int r = 0; r < 6; ++r)
        if ((live >> r) & 1) v += d[r] * rw[r][x] * rw[r][y];
      o[3 * x + y] = v;
    }
}
