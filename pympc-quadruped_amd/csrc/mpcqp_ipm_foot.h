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

