// Diagnostic: class 64's MFMA sweep (mpcqp_sweep_mfma.h) against a host float64
// single-pivot sweep on random SPD matrices of several sizes and conditionings, and
// (when tools/ubench/realH.bin / realR.bin exist: 16 padded 64 x 64 stance-reduced
// Hessians and numpy's -H^-1, float64) on real config-2 Hessians.
#include "../../pympc-quadruped_amd/csrc/mpcqp.hip"
#include "mpcqp_sweep_mfma.h"

#include <stdio.h>
#include <stdlib.h>

namespace {
__global__ __launch_bounds__(128) void k_sweep(const double* H, int n, double* out) {
  __shared__ double buf[4096];
  const int tid = threadIdx.x, tr = tid >> 3, tc = tid & 7;
  double W[4][8], Ws[4][8];
  for (int r = 0; r < 4; ++r)
    for (int c = 0; c < 8; ++c) W[r][c] = H[(4 * tr + r) * 64 + 8 * tc + c];
  sweep_mfma64(W, Ws, buf, n, tid);
  for (int r = 0; r < 4; ++r)
    for (int c = 0; c < 8; ++c) out[(4 * tr + r) * 64 + 8 * tc + c] = Ws[r][c];
}
}  // namespace

int main() {
  static double H[4096], R[4096], O[4096];
  double *dH, *dO;
  (void)hipMalloc(&dH, sizeof(H));
  (void)hipMalloc(&dO, sizeof(O));
  srand(7);
  for (int n : {60, 57, 64, 12, 5}) {
    for (int cond = 0; cond < 2; ++cond) {
      // H = X X^T + scale, identity padding beyond n
      static double X[64 * 64];
      for (int i = 0; i < 64 * 64; ++i) X[i] = (rand() / (double)RAND_MAX - 0.5) * (cond ? ((i % 7) ? 1.0 : 1e3) : 1.0);
      for (int i = 0; i < 64; ++i)
        for (int j = 0; j < 64; ++j) {
          double s = 0.0;
          if (i < n && j < n)
            for (int k = 0; k < 64; ++k) s += X[i * 64 + k] * X[j * 64 + k];
          H[i * 64 + j] = (i < n && j < n) ? s + (i == j ? 1.0 : 0.0) : (i == j ? 1.0 : 0.0);
        }
      // host single-pivot sweep (the reference result, -H^-1 on the first n)
      for (int i = 0; i < 4096; ++i) R[i] = H[i];
      for (int K = 0; K < n; ++K) {
        const double d = R[K * 64 + K];
        double z[64];
        for (int i = 0; i < 64; ++i) z[i] = R[i * 64 + K];
        for (int i = 0; i < 64; ++i)
          for (int j = 0; j < 64; ++j) R[i * 64 + j] -= z[i] * z[j] / d;
        for (int i = 0; i < 64; ++i) {
          R[i * 64 + K] = z[i] / d;
          R[K * 64 + i] = z[i] / d;
        }
        R[K * 64 + K] = -1.0 / d;
      }
      (void)hipMemcpy(dH, H, sizeof(H), hipMemcpyHostToDevice);
      hipLaunchKernelGGL(k_sweep, dim3(1), dim3(128), 0, 0, dH, n, dO);
      (void)hipMemcpy(O, dO, sizeof(O), hipMemcpyDeviceToHost);
      double emax = 0.0, rmax = 0.0, pmax = 0.0;
      int wi = 0, wj = 0;
      for (int i = 0; i < 64; ++i)
        for (int j = 0; j < 64; ++j) {
          const double e = fabs(O[i * 64 + j] - R[i * 64 + j]);
          if (i < n && j < n) {
            if (e > emax) {
              emax = e;
              wi = i;
              wj = j;
            }
            rmax = fmax(rmax, fabs(R[i * 64 + j]));
          } else {
            pmax = fmax(pmax, e);
          }
        }
      printf("n %2d cond-skew %d: max |mfma - host| / max|host| = %.2e at (%d, %d); padding max diff %.2e\n", n, cond,
             emax / rmax, wi, wj, pmax);
    }
  }
  // real Hessians (16 config-2 robots, n = 60) against numpy's inverse
  FILE* fh = fopen("tools/ubench/realH.bin", "rb");
  FILE* fr = fopen("tools/ubench/realR.bin", "rb");
  if (fh && fr) {
    for (int b = 0; b < 16; ++b) {
      if (fread(H, 8, 4096, fh) != 4096 || fread(R, 8, 4096, fr) != 4096) break;
      (void)hipMemcpy(dH, H, sizeof(H), hipMemcpyHostToDevice);
      hipLaunchKernelGGL(k_sweep, dim3(1), dim3(128), 0, 0, dH, 60, dO);
      (void)hipMemcpy(O, dO, sizeof(O), hipMemcpyDeviceToHost);
      double emax = 0.0, rmax = 0.0;
      for (int i = 0; i < 60; ++i)
        for (int j = 0; j < 60; ++j) {
          emax = fmax(emax, fabs(O[i * 64 + j] - R[i * 64 + j]));
          rmax = fmax(rmax, fabs(R[i * 64 + j]));
        }
      printf("real robot %2d: max |mfma - numpy inv| / max = %.2e\n", b, emax / rmax);
    }
  }
  return 0;
}
