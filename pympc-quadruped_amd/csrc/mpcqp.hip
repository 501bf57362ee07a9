// mpcqp.hip -- MI355X (gfx950) batched convex-MPC QP engine: kernels + C ABI.
//
// One workgroup (256 threads = 4 wave64) per robot.  Per robot, fused in one
// launch, nothing but the inputs and u0/U/status leaves the CU:
//
//   1. model      A_c, B_c exactly as the reference rounds them to float32
//                 (mpc.py:173-192), then the exact discretisation: M^3 = 0
//                 for M = [[A_c,B_c],[0,0]], so expm(M dt) = I + M dt + M^2 dt^2/2
//                 (replaces scipy expm, mpc.py:194-208), in float64.
//   2. condense   A_d = I + Nm with Nm^3 = 0, so A^k B_d = X0 + k X1 + C(k,2) X2
//                 (X0 = B_d, X1 = Nm X0, X2 = Nm X1).  The condensed Hessian
//                 H = 2(Su^T Qbar Su + Rbar) (mpc.py:232) restricted to the
//                 stance variables is then  2 sum_pq T_pq(j_a,j_b) Y_pq[c_a][c_b]
//                 with Y_pq = X_p^T Q X_q (12x12) and scalar Toeplitz weights
//                 T_pq; g (mpc.py:233) likewise.  All float64.
//   3. swing      swing-leg GRFs are exactly 0 (ub: fz <= 0, cone rows: mu fz >=
//                 |fx|,|fy| >= 0), so only n = 3 * #stance variables remain.
//   4. W = H^-1   symmetric sweep (Gauss-Jordan on SPD) in LDS, float64.
//   5. solve      Goldfarb-Idnani dual active-set method in range-space form
//                 (W known, explicit inverse of the active-set Gram matrix
//                 M_AA = A_A W A_A^T updated by bordering / downdating), exact
//                 up to float64 rounding; then one refinement step and a KKT
//                 check of every constraint row.
//
// The QP is the Drake branch of _solve_mpc (mpc.py:277-286):
//   min 1/2 U^T H U + g^T U  s.t.  lb <= C U <= ub, C = kron(I_4N, cone) (mpc.py:239-246)
// generalised to a per-robot cone normal n (n = e_z reproduces mpc.py exactly).

#include <hip/hip_runtime.h>

#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include <new>
#include <string>

#include "mpcqp.h"

namespace {

constexpr int kThreads = 256;
constexpr int NX = 13;   // state dimension (mpc.py:26)
constexpr int NU = 12;   // input dimension (mpc.py:28)
constexpr int kMaxN = 20;  // horizon supported by the LDS-resident formulation scratch

struct KParams {
  int N;
  int max_iter;
  double dt;
  double q[NX];
  double r[NU];
};

__device__ __forceinline__ double f32r(double v) { return (double)(float)v; }

// Toeplitz weight polynomials: A^k = I + k Nm + C(k,2) Nm^2
__device__ __forceinline__ double cpoly(int p, int k) {
  return p == 0 ? 1.0 : (p == 1 ? (double)k : 0.5 * (double)k * (double)(k - 1));
}

// T table index for (d, m): d in [0,N), m in [1, N-d]
__device__ __forceinline__ int tidx(int N, int d, int m) { return d * N - (d * (d - 1)) / 2 + (m - 1); }

template <int NMAX>
struct Shared {
  static constexpr int LD = NMAX + 1;       // odd leading dimension: conflict-free ds_read_b64
  static constexpr int MMAX = 2 * NMAX;     // 6 rows per 3 variables
  static constexpr int SMAX = NMAX / 3;     // stance foot-steps
  double W[NMAX * LD];                      // H, then H^-1
  double Minv[NMAX * LD];                   // (M_AA)^-1; formulation scratch before the solve
  double g[NMAX], w[NMAX], v[NMAX], z[NMAX], x[NMAX];
  double s[MMAX], zs[MMAX];
  double u[NMAX], mp[NMAX], r[NMAX];
  int act[NMAX];
  int foot_t[SMAX], foot_leg[SMAX];
  double foot_ub[SMAX];
  int stance_of[4 * MPCQP_MAX_HORIZON];
  double rows[6][3];                        // cone rows a_r (same for every foot of the robot)
  double x0[NX];
  double y1[NX], y2[NX];
  double red_val[4];
  int red_idx[4];
  int S, n, m, q, flag;
  int p;
  double tstep;
  int lidx, add;
};

// wave-level argmin (value, index) across 64 lanes; ties -> lowest index
__device__ __forceinline__ void wave_argmin(double& v, int& i) {
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) {
    double ov = __shfl_xor(v, off);
    int oi = __shfl_xor(i, off);
    if (ov < v || (ov == v && oi < i)) { v = ov; i = oi; }
  }
}

template <int NMAX>
__global__ __launch_bounds__(kThreads) void mpcqp_kernel(KParams P, int B, int n_lo, int is_top,
                                                         const float* __restrict__ x0g,
                                                         const float* __restrict__ xrefg,
                                                         const float* __restrict__ contactg,
                                                         const float* __restrict__ feetg,
                                                         const float* __restrict__ robotg,
                                                         float* __restrict__ u0g, float* __restrict__ Ug,
                                                         int* __restrict__ statusg, int* __restrict__ itersg) {
  using SM = Shared<NMAX>;
  constexpr int LD = SM::LD;
  __shared__ SM sm;
  const int b = blockIdx.x;
  const int tid = threadIdx.x;
  const int N = P.N;
  if (b >= B) return;

  // ---------------------------------------------------------------- inputs
  const float* cb = contactg + (size_t)b * N * 4;
  if (tid == 0) {
    int S = 0;
    for (int k = 0; k < 4 * N; ++k) {
      float c = cb[k];
      if (c > 0.f) {
        sm.stance_of[k] = S;
        if (S < SM::SMAX) {
          sm.foot_t[S] = k / 4;
          sm.foot_leg[S] = k % 4;
        }
        ++S;
      } else {
        sm.stance_of[k] = -1;
      }
    }
    sm.S = S;
    sm.n = 3 * S;
    sm.m = 6 * S;
  }
  __syncthreads();
  const int S = sm.S, n = sm.n, m = sm.m;
  // capacity dispatch: robots with n <= n_lo belong to a smaller instance
  if (n <= n_lo && n_lo > 0) return;
  if (n > NMAX) {
    if (is_top) {
      if (tid < 12) u0g[(size_t)b * 12 + tid] = 0.f;
      if (Ug)
        for (int k = tid; k < N * 12; k += kThreads) Ug[(size_t)b * N * 12 + k] = 0.f;
      if (tid == 0) {
        if (statusg) statusg[b] = MPCQP_STATUS_TOO_LARGE;
        if (itersg) itersg[b] = 0;
      }
    }
    return;
  }

  const float* rb = robotg + (size_t)b * MPCQP_ROBOT_STRIDE;
  const float* xb = x0g + (size_t)b * NX;
  const float* xrb = xrefg + (size_t)b * N * NX;
  const float* fb = feetg + (size_t)b * 12;

  // non-finite guard (reference would propagate NaN through Drake)
  if (tid == 0) sm.flag = 0;
  __syncthreads();
  {
    int bad = 0;
    for (int k = tid; k < N * NX; k += kThreads) bad |= !isfinite(xrb[k]);
    if (tid < NX) bad |= !isfinite(xb[tid]);
    if (tid < 12) bad |= !isfinite(fb[tid]);
    if (tid < 12) bad |= !isfinite(rb[tid]);
    if (bad) sm.flag = 1;
  }
  __syncthreads();
  if (sm.flag) {
    if (tid < 12) u0g[(size_t)b * 12 + tid] = 0.f;
    if (Ug)
      for (int k = tid; k < N * 12; k += kThreads) Ug[(size_t)b * N * 12 + k] = 0.f;
    if (tid == 0) {
      if (statusg) statusg[b] = MPCQP_STATUS_NONFINITE;
      if (itersg) itersg[b] = 0;
    }
    return;
  }

  // Formulation scratch lives in the (not yet used) Minv region, in doubles:
  //   [0,169) A_c  [169,338) Nm  [338,494) B_c      -- model / discretisation
  //   [0,13N) e    [13N,49N) zp                     -- gradient
  //   [0,1296) Y   [1296,1296+9N(N+1)/2) T          -- Hessian
  //   [3186,3654) X0 | X1 | X2                      -- alive until Y is built
  static_assert(NMAX * (NMAX + 1) >= 3186 + 3 * NX * NU, "scratch does not fit");
  double* const scr = sm.Minv;
  double* const Acm = scr;
  double* const Nmm = scr + NX * NX;
  double* const Bcm = scr + 2 * NX * NX;
  double* const Xb = scr + 3186;  // X_p at Xb + p * NX * NU
  if (tid < NX) sm.x0[tid] = (double)xb[tid];
  for (int k = tid; k < NX * NX; k += kThreads) Acm[k] = 0.0;
  __syncthreads();

  // ------------------------------------------------ 1. model (mpc.py:173-192)
  // Reference dtype path: Rz float32 from float64 cos/sin; I_w = Rz I Rz^T in
  // float32; inv(I_w) float32; inv(I_w) @ skew(r) in float64 rounded to float32;
  // I/m float32.  Emulated as float64 arithmetic rounded where the reference stores.
  if (tid == 0) {
    const double yaw = (double)xb[2];
    const double c = f32r(cos(yaw)), s = f32r(sin(yaw));
    const double Rz[3][3] = {{c, -s, 0.0}, {s, c, 0.0}, {0.0, 0.0, 1.0}};
    const double Ib[3][3] = {{rb[1], rb[2], rb[3]}, {rb[2], rb[4], rb[5]}, {rb[3], rb[5], rb[6]}};
    double T1[3][3], Iw[3][3], Ii[3][3];
    for (int i = 0; i < 3; ++i)
      for (int j = 0; j < 3; ++j) {
        double a = 0.0;
        for (int k = 0; k < 3; ++k) a += Rz[i][k] * Ib[k][j];
        T1[i][j] = f32r(a);
      }
    for (int i = 0; i < 3; ++i)
      for (int j = 0; j < 3; ++j) {
        double a = 0.0;
        for (int k = 0; k < 3; ++k) a += T1[i][k] * Rz[j][k];
        Iw[i][j] = f32r(a);
      }
    // 3x3 inverse by adjugate (float64), stored float32 like np.linalg.inv on float32
    const double c00 = Iw[1][1] * Iw[2][2] - Iw[1][2] * Iw[2][1];
    const double c01 = Iw[1][2] * Iw[2][0] - Iw[1][0] * Iw[2][2];
    const double c02 = Iw[1][0] * Iw[2][1] - Iw[1][1] * Iw[2][0];
    const double det = Iw[0][0] * c00 + Iw[0][1] * c01 + Iw[0][2] * c02;
    const double id = 1.0 / det;
    Ii[0][0] = c00 * id;
    Ii[1][0] = c01 * id;
    Ii[2][0] = c02 * id;
    Ii[0][1] = (Iw[0][2] * Iw[2][1] - Iw[0][1] * Iw[2][2]) * id;
    Ii[1][1] = (Iw[0][0] * Iw[2][2] - Iw[0][2] * Iw[2][0]) * id;
    Ii[2][1] = (Iw[0][1] * Iw[2][0] - Iw[0][0] * Iw[2][1]) * id;
    Ii[0][2] = (Iw[0][1] * Iw[1][2] - Iw[0][2] * Iw[1][1]) * id;
    Ii[1][2] = (Iw[0][2] * Iw[1][0] - Iw[0][0] * Iw[1][2]) * id;
    Ii[2][2] = (Iw[0][0] * Iw[1][1] - Iw[0][1] * Iw[1][0]) * id;
    for (int i = 0; i < 3; ++i)
      for (int j = 0; j < 3; ++j) Ii[i][j] = f32r(Ii[i][j]);
    // A_c (mpc.py:184-186)
    for (int i = 0; i < 3; ++i)
      for (int j = 0; j < 3; ++j) Acm[i * NX + 6 + j] = Rz[j][i];
    for (int i = 0; i < 3; ++i) Acm[(3 + i) * NX + 9 + i] = 1.0;
    Acm[11 * NX + 12] = 1.0;
    // B_c into tmp as 13x12 (mpc.py:188-190)
    double* Bc = Bcm;
    for (int k = 0; k < NX * NU; ++k) Bc[k] = 0.0;
    const double minv = f32r(1.0 / (double)rb[0]);
    for (int leg = 0; leg < 4; ++leg) {
      const double rx = fb[3 * leg], ry = fb[3 * leg + 1], rz = fb[3 * leg + 2];
      const double sk[3][3] = {{0.0, -rz, ry}, {rz, 0.0, -rx}, {-ry, rx, 0.0}};
      for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) {
          double a = 0.0;
          for (int k = 0; k < 3; ++k) a += Ii[i][k] * sk[k][j];
          Bc[(6 + i) * NU + 3 * leg + j] = f32r(a);
        }
      for (int i = 0; i < 3; ++i) Bc[(9 + i) * NU + 3 * leg + i] = minv;
    }
    // friction-cone rows in the (t1, t2, n) frame (mpc.py:239-245 for n = e_z)
    double nx = rb[9], ny = rb[10], nz = rb[11];
    const double nn = sqrt(nx * nx + ny * ny + nz * nz);
    if (!(nn > 0.0)) { nx = 0.0; ny = 0.0; nz = 1.0; } else { nx /= nn; ny /= nn; nz /= nn; }
    double t1x = 1.0 - nx * nx, t1y = -nx * ny, t1z = -nx * nz;
    const double tn = sqrt(t1x * t1x + t1y * t1y + t1z * t1z);
    t1x /= tn; t1y /= tn; t1z /= tn;
    const double t2x = ny * t1z - nz * t1y, t2y = nz * t1x - nx * t1z, t2z = nx * t1y - ny * t1x;
    const double mu = rb[7];
    const double rws[6][3] = {{t1x + mu * nx, t1y + mu * ny, t1z + mu * nz},
                              {-t1x + mu * nx, -t1y + mu * ny, -t1z + mu * nz},
                              {t2x + mu * nx, t2y + mu * ny, t2z + mu * nz},
                              {-t2x + mu * nx, -t2y + mu * ny, -t2z + mu * nz},
                              {nx, ny, nz},
                              {-nx, -ny, -nz}};
    for (int r = 0; r < 6; ++r)
      for (int j = 0; j < 3; ++j) sm.rows[r][j] = rws[r][j];
  }
  if (tid < S && tid < SM::SMAX) {
    const float c = cb[sm.foot_t[tid] * 4 + sm.foot_leg[tid]];
    sm.foot_ub[tid] = (double)c * (double)rb[8];   // ub = contact * fz_max (mpc.py:257)
  }
  __syncthreads();

  // -------------------------------- 2. exact discretisation (mpc.py:194-208)
  const double dt = P.dt;
  // Nm = A_c dt + A_c^2 dt^2/2 ;  B_d = B_c dt + A_c B_c dt^2/2
  for (int k = tid; k < NX * NX; k += kThreads) {
    const int i = k / NX, j = k % NX;
    double a2 = 0.0;
    for (int l = 0; l < NX; ++l) a2 += Acm[i * NX + l] * Acm[l * NX + j];
    Nmm[k] = Acm[k] * dt + a2 * (0.5 * dt * dt);
  }
  for (int k = tid; k < NX * NU; k += kThreads) {
    const int i = k / NU, j = k % NU;
    double ab = 0.0;
    for (int l = 0; l < NX; ++l) ab += Acm[i * NX + l] * Bcm[l * NU + j];
    Xb[0 * NX * NU + k] = Bcm[k] * dt + ab * (0.5 * dt * dt);
  }
  __syncthreads();
  for (int k = tid; k < NX * NU; k += kThreads) {
    const int i = k / NU, j = k % NU;
    double a = 0.0;
    for (int l = 0; l < NX; ++l) a += Nmm[i * NX + l] * Xb[0 * NX * NU + l * NU + j];
    Xb[1 * NX * NU + k] = a;
  }
  if (tid < NX) {
    double a = 0.0;
    for (int l = 0; l < NX; ++l) a += Nmm[tid * NX + l] * sm.x0[l];
    sm.y1[tid] = a;
  }
  __syncthreads();
  for (int k = tid; k < NX * NU; k += kThreads) {
    const int i = k / NU, j = k % NU;
    double a = 0.0;
    for (int l = 0; l < NX; ++l) a += Nmm[i * NX + l] * Xb[1 * NX * NU + l * NU + j];
    Xb[2 * NX * NU + k] = a;
  }
  if (tid < NX) {
    double a = 0.0;
    for (int l = 0; l < NX; ++l) a += Nmm[tid * NX + l] * sm.y1[l];
    sm.y2[tid] = a;
  }
  __syncthreads();

  // ---------------------------------------- 3. condensed cost (mpc.py:211-235)
  double* const e = scr;
  double* const zp = scr + N * NX;
  double* const Y = scr;
  double* const T = scr + 9 * NU * NU;
  const int nT = N * (N + 1) / 2;
  // e_t = A^{t+1} x0 - xref_t   (Sx @ xt - Xref, mpc.py:233)
  for (int k = tid; k < N * NX; k += kThreads) {
    const int t = k / NX, sIdx = k % NX;
    const double kk = (double)(t + 1);
    e[k] = sm.x0[sIdx] + kk * sm.y1[sIdx] + 0.5 * kk * (kk - 1.0) * sm.y2[sIdx] - (double)xrb[k];
  }
  __syncthreads();
  // zp[p][t][c] = sum_s X_p[s][c] Q_s e_t[s]
  for (int k = tid; k < 3 * N * NU; k += kThreads) {
    const int p = k / (N * NU), rem = k % (N * NU), t = rem / NU, c = rem % NU;
    double a = 0.0;
    for (int sIdx = 0; sIdx < NX; ++sIdx) a += Xb[p * NX * NU + sIdx * NU + c] * P.q[sIdx] * e[t * NX + sIdx];
    zp[k] = a;
  }
  __syncthreads();
  // g[a] = 2 sum_p sum_{t >= j_a} c_p(t - j_a) zp[p][t][c_a]
  for (int a = tid; a < n; a += kThreads) {
    const int sf = a / 3, ax = a % 3;
    const int ja = sm.foot_t[sf], ca = 3 * sm.foot_leg[sf] + ax;
    double acc = 0.0;
    for (int t = ja; t < N; ++t)
      for (int p = 0; p < 3; ++p) acc += cpoly(p, t - ja) * zp[(p * N + t) * NU + ca];
    sm.g[a] = 2.0 * acc;
  }
  __syncthreads();
  // Y_pq[c][c'] = sum_s Q_s X_p[s][c] X_q[s][c']   (overwrites e / zp)
  for (int k = tid; k < 9 * NU * NU; k += kThreads) {
    const int pq = k / (NU * NU), cc = k % (NU * NU);
    const int p = pq / 3, q = pq % 3, c = cc / NU, c2 = cc % NU;
    double a = 0.0;
    for (int sIdx = 0; sIdx < NX; ++sIdx) a += P.q[sIdx] * Xb[p * NX * NU + sIdx * NU + c] * Xb[q * NX * NU + sIdx * NU + c2];
    Y[k] = a;
  }
  // T_pq(d, m) = sum_{s<m} c_p(s+d) c_q(s)  (prefix sums over m)
  for (int k = tid; k < 9 * N; k += kThreads) {
    const int pq = k / N, d = k % N;
    const int p = pq / 3, q = pq % 3;
    double acc = 0.0;
    for (int mm = 1; mm <= N - d; ++mm) {
      const int sIdx = mm - 1;
      acc += cpoly(p, sIdx + d) * cpoly(q, sIdx);
      T[pq * nT + tidx(N, d, mm)] = acc;
    }
  }
  __syncthreads();
  // H[a][b] = 2 sum_pq Tv Y_pq[c_a][c_b] + 2 R delta   (stance rows/cols only)
  for (int k = tid; k < n * n; k += kThreads) {
    const int a = k / n, bb = k % n;
    if (bb > a) continue;
    const int sa = a / 3, sb = bb / 3;
    const int ja = sm.foot_t[sa], jb = sm.foot_t[sb];
    const int ca = 3 * sm.foot_leg[sa] + a % 3, cb2 = 3 * sm.foot_leg[sb] + bb % 3;
    double acc = 0.0;
    if (ja <= jb) {
      const int ti = tidx(N, jb - ja, N - jb);
      for (int p = 0; p < 3; ++p)
        for (int q = 0; q < 3; ++q) acc += T[(p * 3 + q) * nT + ti] * Y[(p * 3 + q) * NU * NU + ca * NU + cb2];
    } else {
      const int ti = tidx(N, ja - jb, N - ja);
      for (int p = 0; p < 3; ++p)
        for (int q = 0; q < 3; ++q) acc += T[(q * 3 + p) * nT + ti] * Y[(p * 3 + q) * NU * NU + ca * NU + cb2];
    }
    double h = 2.0 * acc;
    if (a == bb) h += 2.0 * P.r[ca];
    sm.W[a * LD + bb] = h;
    sm.W[bb * LD + a] = h;
  }
  __syncthreads();

  // ------------------------------------------ 4. W = H^-1 (symmetric sweep)
  for (int k = 0; k < n; ++k) {
    for (int i = tid; i < n; i += kThreads) sm.z[i] = sm.W[i * LD + k];
    __syncthreads();
    const double inv = 1.0 / sm.z[k];
    for (int idx = tid; idx < n * n; idx += kThreads) {
      const int i = idx / n, j = idx % n;
      if (i == k || j == k) continue;
      sm.W[i * LD + j] -= sm.z[i] * sm.z[j] * inv;
    }
    for (int i = tid; i < n; i += kThreads) {
      if (i == k) sm.W[k * LD + k] = -inv;
      else {
        const double val = sm.z[i] * inv;
        sm.W[i * LD + k] = val;
        sm.W[k * LD + i] = val;
      }
    }
    __syncthreads();
  }
  for (int idx = tid; idx < n * n; idx += kThreads) {
    const int i = idx / n, j = idx % n;
    sm.W[i * LD + j] = -sm.W[i * LD + j];
  }
  __syncthreads();

  // unconstrained minimiser x = -W g ; constraint values s = A x - b
  for (int i = tid; i < n; i += kThreads) {
    double a = 0.0;
    for (int j = 0; j < n; ++j) a += sm.W[i * LD + j] * sm.g[j];
    sm.x[i] = -a;
  }
  __syncthreads();
  for (int i = tid; i < m; i += kThreads) {
    const int f = i / 6, rr = i % 6;
    const double val = sm.rows[rr][0] * sm.x[3 * f] + sm.rows[rr][1] * sm.x[3 * f + 1] + sm.rows[rr][2] * sm.x[3 * f + 2];
    sm.s[i] = (rr == 5) ? val + sm.foot_ub[f] : val;
  }
  if (tid == 0) sm.q = 0;
  __syncthreads();

  // ---------------------------- 5. Goldfarb-Idnani dual active set (range space)
  const int max_iter = P.max_iter > 0 ? P.max_iter : 8 * NMAX + 64;
  const double tol = 1e-9;
  int it = 0;
  int status = MPCQP_STATUS_OK;
  while (true) {
    // most violated constraint
    if (tid < 64) {
      double bv = INFINITY;
      int bi = 0x7fffffff;
      for (int i = tid; i < m; i += 64) {
        const double sv = sm.s[i];
        if (sv < bv) { bv = sv; bi = i; }
      }
      wave_argmin(bv, bi);
      if (tid == 0) {
        sm.p = bi;
        sm.red_val[0] = bv;
      }
    }
    __syncthreads();
    if (!(sm.red_val[0] < -tol)) break;
    const int p = sm.p;
    const int fp = p / 6, rp = p % 6;
    // w = W a_p
    for (int i = tid; i < n; i += kThreads)
      sm.w[i] = sm.W[i * LD + 3 * fp] * sm.rows[rp][0] + sm.W[i * LD + 3 * fp + 1] * sm.rows[rp][1] +
                sm.W[i * LD + 3 * fp + 2] * sm.rows[rp][2];
    double up = 0.0;  // multiplier of p (tracked by every thread identically)
    __syncthreads();
    bool added = false;
    while (!added) {
      if (++it > max_iter) { status = MPCQP_STATUS_MAX_ITER; break; }
      const int q = sm.q;
      // mp_j = a_j . w(foot_j)
      for (int j = tid; j < q; j += kThreads) {
        const int cj = sm.act[j], fj = cj / 6, rj = cj % 6;
        sm.mp[j] = sm.rows[rj][0] * sm.w[3 * fj] + sm.rows[rj][1] * sm.w[3 * fj + 1] + sm.rows[rj][2] * sm.w[3 * fj + 2];
      }
      for (int i = tid; i < n; i += kThreads) sm.v[i] = 0.0;
      __syncthreads();
      // r = Minv mp
      for (int j = tid; j < q; j += kThreads) {
        double a = 0.0;
        for (int l = 0; l < q; ++l) a += sm.Minv[j * LD + l] * sm.mp[l];
        sm.r[j] = a;
      }
      __syncthreads();
      // v = a_p - sum_j r_j a_j   (scatter onto foot variables)
      if (tid == 0) {
        for (int c = 0; c < 3; ++c) sm.v[3 * fp + c] += sm.rows[rp][c];
        for (int j = 0; j < q; ++j) {
          const int cj = sm.act[j], fj = cj / 6, rj = cj % 6;
          for (int c = 0; c < 3; ++c) sm.v[3 * fj + c] -= sm.r[j] * sm.rows[rj][c];
        }
      }
      __syncthreads();
      // z = W v   (primal step direction)
      for (int i = tid; i < n; i += kThreads) {
        double a = 0.0;
        for (int j = 0; j < n; ++j) a += sm.W[i * LD + j] * sm.v[j];
        sm.z[i] = a;
      }
      __syncthreads();
      for (int i = tid; i < m; i += kThreads) {
        const int f = i / 6, rr = i % 6;
        sm.zs[i] = sm.rows[rr][0] * sm.z[3 * f] + sm.rows[rr][1] * sm.z[3 * f + 1] + sm.rows[rr][2] * sm.z[3 * f + 2];
      }
      __syncthreads();
      // step lengths (wave 0)
      if (tid < 64) {
        double bv = INFINITY;
        int bi = 0x7fffffff;
        for (int j = tid; j < q; j += 64) {
          const double rj = sm.r[j];
          if (rj > 0.0) {
            const double ratio = sm.u[j] / rj;
            if (ratio < bv) { bv = ratio; bi = j; }
          }
        }
        wave_argmin(bv, bi);
        if (tid == 0) {
          const double t1 = bv;
          const double zsp = sm.zs[p];
          const double ap_w = sm.rows[rp][0] * sm.w[3 * fp] + sm.rows[rp][1] * sm.w[3 * fp + 1] + sm.rows[rp][2] * sm.w[3 * fp + 2];
          double t2 = INFINITY;
          if (zsp > 1e-12 * ap_w) t2 = -sm.s[p] / zsp;
          double t = t1 < t2 ? t1 : t2;
          int add = (t2 <= t1) ? 1 : 0;
          if (!(t < INFINITY)) { add = -1; t = 0.0; }
          sm.tstep = t;
          sm.add = add;
          sm.lidx = bi;
        }
      }
      __syncthreads();
      const int add = sm.add;
      if (add < 0) { status = MPCQP_STATUS_INFEASIBLE; break; }
      const double t = sm.tstep;
      // apply step: u_A -= t r, u_p += t, s += t zs
      for (int j = tid; j < q; j += kThreads) sm.u[j] -= t * sm.r[j];
      for (int i = tid; i < m; i += kThreads) sm.s[i] += t * sm.zs[i];
      up += t;
      __syncthreads();
      if (add) {
        // bordered update of Minv with sigma = zs_p (Schur complement)
        const double sig = sm.zs[p];
        const double is = 1.0 / sig;
        for (int idx = tid; idx < q * q; idx += kThreads) {
          const int i = idx / q, j = idx % q;
          sm.Minv[i * LD + j] += sm.r[i] * sm.r[j] * is;
        }
        for (int i = tid; i < q; i += kThreads) {
          sm.Minv[i * LD + q] = -sm.r[i] * is;
          sm.Minv[q * LD + i] = -sm.r[i] * is;
        }
        if (tid == 0) {
          sm.Minv[q * LD + q] = is;
          sm.act[q] = p;
          sm.u[q] = up;
          sm.s[p] = 0.0;
          sm.q = q + 1;
        }
        __syncthreads();
        added = true;
      } else {
        // drop l: Minv' = Minv - Minv[:,l] Minv[l,:] / Minv[l][l], then move last into l
        const int l = sm.lidx;
        const double ill = 1.0 / sm.Minv[l * LD + l];
        for (int i = tid; i < q; i += kThreads) sm.v[i] = sm.Minv[i * LD + l];
        __syncthreads();
        for (int idx = tid; idx < q * q; idx += kThreads) {
          const int i = idx / q, j = idx % q;
          sm.Minv[i * LD + j] -= sm.v[i] * sm.v[j] * ill;
        }
        __syncthreads();
        const int last = q - 1;
        if (l != last) {
          for (int i = tid; i < q; i += kThreads) {
            sm.Minv[i * LD + l] = sm.Minv[i * LD + last];
          }
          __syncthreads();
          for (int i = tid; i < q; i += kThreads) {
            sm.Minv[l * LD + i] = sm.Minv[last * LD + i];
          }
          if (tid == 0) {
            sm.act[l] = sm.act[last];
            sm.u[l] = sm.u[last];
          }
        }
        if (tid == 0) sm.q = last;
        __syncthreads();
      }
    }
    if (status != MPCQP_STATUS_OK) break;
  }
  __syncthreads();

  // ------------------------------- 6. refinement, final x, KKT verification
  {
    const int q = sm.q;
    for (int pass = 0; pass < 2; ++pass) {
      // x = -W g + W A_A^T u
      for (int i = tid; i < n; i += kThreads) sm.v[i] = -sm.g[i];
      __syncthreads();
      if (tid == 0) {
        for (int j = 0; j < q; ++j) {
          const int cj = sm.act[j], fj = cj / 6, rj = cj % 6;
          for (int c = 0; c < 3; ++c) sm.v[3 * fj + c] += sm.u[j] * sm.rows[rj][c];
        }
      }
      __syncthreads();
      for (int i = tid; i < n; i += kThreads) {
        double a = 0.0;
        for (int j = 0; j < n; ++j) a += sm.W[i * LD + j] * sm.v[j];
        sm.x[i] = a;
      }
      __syncthreads();
      if (pass == 1) break;
      // residual of the active rows, correct multipliers: u -= Minv (A_A x - b_A)
      for (int j = tid; j < q; j += kThreads) {
        const int cj = sm.act[j], fj = cj / 6, rj = cj % 6;
        double val = sm.rows[rj][0] * sm.x[3 * fj] + sm.rows[rj][1] * sm.x[3 * fj + 1] + sm.rows[rj][2] * sm.x[3 * fj + 2];
        if (rj == 5) val += sm.foot_ub[fj];
        sm.mp[j] = val;
      }
      __syncthreads();
      for (int j = tid; j < q; j += kThreads) {
        double a = 0.0;
        for (int l = 0; l < q; ++l) a += sm.Minv[j * LD + l] * sm.mp[l];
        sm.r[j] = a;
      }
      __syncthreads();
      for (int j = tid; j < q; j += kThreads) sm.u[j] -= sm.r[j];
      __syncthreads();
    }
    // verify primal feasibility of every row and dual feasibility
    if (tid == 0) sm.flag = 0;
    __syncthreads();
    int bad = 0;
    for (int i = tid; i < m; i += kThreads) {
      const int f = i / 6, rr = i % 6;
      double val = sm.rows[rr][0] * sm.x[3 * f] + sm.rows[rr][1] * sm.x[3 * f + 1] + sm.rows[rr][2] * sm.x[3 * f + 2];
      if (rr == 5) val += sm.foot_ub[f];
      if (val < -1e-6 || !isfinite(val)) bad = 1;
    }
    for (int j = tid; j < q; j += kThreads)
      if (sm.u[j] < -1e-9) bad = 1;
    if (bad) sm.flag = 1;
    __syncthreads();
    if (status == MPCQP_STATUS_OK && sm.flag) status = MPCQP_STATUS_MAX_ITER;
  }

  // ---------------------------------------------------------------- output
  for (int k = tid; k < 12; k += kThreads) {
    const int leg = k / 3, ax = k % 3;
    const int sidx = sm.stance_of[leg];
    u0g[(size_t)b * 12 + k] = sidx >= 0 ? (float)sm.x[3 * sidx + ax] : 0.f;
  }
  if (Ug) {
    for (int k = tid; k < N * 12; k += kThreads) {
      const int fs = k / 3, ax = k % 3;
      const int sidx = sm.stance_of[fs];
      Ug[(size_t)b * N * 12 + k] = sidx >= 0 ? (float)sm.x[3 * sidx + ax] : 0.f;
    }
  }
  if (tid == 0) {
    if (statusg) statusg[b] = status;
    if (itersg) itersg[b] = it;
  }
}

}  // namespace

// ============================================================== C ABI
struct mpcqp_ctx {
  mpcqp_params params;
  int device;
  int stance_hint;
  std::string err;
};

static int set_err(mpcqp_ctx* ctx, int code, const std::string& msg) {
  if (ctx) ctx->err = msg;
  return code;
}

extern "C" {

int32_t mpcqp_abi_version(void) { return MPCQP_ABI_VERSION; }

void mpcqp_default_params(mpcqp_params* p, int32_t horizon) {
  if (!p) return;
  static const double q[13] = {5., 5., 10., 10., 10., 50., 0.01, 0.01, 0.2, 0.2, 0.2, 0.2, 0.};
  memset(p, 0, sizeof(*p));
  p->horizon = horizon;
  p->max_iter = 0;
  p->dt = 0.05;
  for (int i = 0; i < 13; ++i) p->q_diag[i] = q[i];
  for (int i = 0; i < 12; ++i) p->r_diag[i] = 1e-5;
}

int mpcqp_create(const mpcqp_params* p, int32_t device, mpcqp_ctx** out) {
  if (!p || !out) return MPCQP_ERR_ARG;
  *out = nullptr;
  if (p->horizon < 1 || p->horizon > kMaxN) return MPCQP_ERR_ARG;
  if (!(p->dt > 0.0)) return MPCQP_ERR_ARG;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || device < 0 || device >= ndev) return MPCQP_ERR_HIP;
  mpcqp_ctx* ctx = new (std::nothrow) mpcqp_ctx();
  if (!ctx) return MPCQP_ERR_ALLOC;
  ctx->params = *p;
  ctx->device = device;
  ctx->stance_hint = 0;
  *out = ctx;
  return MPCQP_OK;
}

int mpcqp_set_stance_hint(mpcqp_ctx* ctx, int32_t max_stance) {
  if (!ctx || max_stance < 0) return MPCQP_ERR_ARG;
  ctx->stance_hint = max_stance;
  return MPCQP_OK;
}

int mpcqp_solve(mpcqp_ctx* ctx, int32_t batch, const float* x0, const float* xref, const float* contact,
                const float* feet, const float* robot, float* u0, float* U, int32_t* status, int32_t* iters,
                void* stream) {
  if (!ctx) return MPCQP_ERR_ARG;
  if (batch < 0) return set_err(ctx, MPCQP_ERR_ARG, "batch < 0");
  if (batch == 0) return MPCQP_OK;
  if (!x0 || !xref || !contact || !feet || !robot || !u0)
    return set_err(ctx, MPCQP_ERR_ARG, "null input/output pointer");
  if (hipSetDevice(ctx->device) != hipSuccess) return set_err(ctx, MPCQP_ERR_HIP, "hipSetDevice failed");
  KParams kp;
  kp.N = ctx->params.horizon;
  kp.max_iter = ctx->params.max_iter;
  kp.dt = ctx->params.dt;
  for (int i = 0; i < NX; ++i) kp.q[i] = ctx->params.q_diag[i];
  for (int i = 0; i < NU; ++i) kp.r[i] = ctx->params.r_diag[i];
  hipStream_t st = (hipStream_t)stream;
  // capacity class 64 (the only class of this build): n = 3 * #stance <= 64
  hipLaunchKernelGGL((mpcqp_kernel<64>), dim3(batch), dim3(kThreads), 0, st, kp, (int)batch, 0, 1, x0, xref,
                     contact, feet, robot, u0, U, (int*)status, (int*)iters);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return set_err(ctx, MPCQP_ERR_HIP, std::string("launch: ") + hipGetErrorString(e));
  return MPCQP_OK;
}

int mpcqp_destroy(mpcqp_ctx* ctx) {
  delete ctx;
  return MPCQP_OK;
}

const char* mpcqp_last_error(const mpcqp_ctx* ctx) { return ctx ? ctx->err.c_str() : "null context"; }

}  // extern "C"
