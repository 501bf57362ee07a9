// cpu_mpc.cpp -- compiled CPU restatement of the reference's per-tick MPC
// formulate + solve (TEST INFRASTRUCTURE / CPU BASELINE ONLY: loaded by tests/ and by
// bench.py's cpu_baseline leg, never by the product path).
//
// Per robot it follows ModelPredictiveController._solve_mpc (/root/reference/linear_mpc/
// mpc.py:262-290) step by step, in the reference's own representation:
//   * A_c, B_c (mpc.py:173-192) with the reference's float32 storage;
//   * discretisation (mpc.py:194-208): expm of [[A_c, B_c], [0, 0]] h, evaluated exactly
//     as I + M h + M^2 h^2 / 2 (M^3 = 0), stored float32 like scipy's f32 expm result;
//   * condensing (mpc.py:211-230): float32 powers A^k and the dense block-Toeplitz Su
//     (13N x 12N), Sx (13N x 13);
//   * H = 2 (Su^T Qbar Su + Rbar), g = 2 Su^T Qbar (Sx x0 - xref) (mpc.py:232-233): dense,
//     float64 (Qbar is float64 in the reference);
//   * cone rows (mpc.py:237-260), generalised to a per-robot surface normal;
//   * the Drake-branch QP (mpc.py:277-286) by a float64 Goldfarb-Idnani dual active set
//     (Cholesky of H, J = L^-T with Householder adds / Givens drops) on the stance
//     variables (swing GRFs are exactly 0: ub gives fz <= 0 and the cone mu fz >= |ft|).
// Formulation and solve are timed separately.  OpenMP over robots.
#include <math.h>
#include <omp.h>
#include <stdint.h>
#include <string.h>

#include <chrono>
#include <vector>

namespace {

constexpr int NX = 13, NU = 12;

inline float f32(double v) { return (float)v; }

struct Robot {
  const float* x0;      // 13
  const float* xref;    // N * 13
  const float* contact; // N * 4
  const float* feet;    // 12
  const float* rec;     // 16: mass, ixx, ixy, ixz, iyy, iyz, izz, mu, fz_max, nx, ny, nz
};

// ---------------------------------------------------------------- formulation
// H (n x n, n = 12N, row-major) and g (n), float64
void formulate(const Robot& r, int N, double h, const double* q, const double* rw, std::vector<double>& H,
               std::vector<double>& g) {
  const int n = NU * N, m = NX * N;
  // mpc.py:178-182: R_z float32, I_w = R_z I_B R_z^T in float32, inv in float32
  const double yaw = r.x0[2];
  const float c = f32(cos(yaw)), s = f32(sin(yaw));
  const float Rz[3][3] = {{c, -s, 0.f}, {s, c, 0.f}, {0.f, 0.f, 1.f}};
  const float IB[3][3] = {{r.rec[1], r.rec[2], r.rec[3]}, {r.rec[2], r.rec[4], r.rec[5]}, {r.rec[3], r.rec[5], r.rec[6]}};
  float T[3][3], Iw[3][3], Ii[3][3];
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) T[i][j] = Rz[i][0] * IB[0][j] + Rz[i][1] * IB[1][j] + Rz[i][2] * IB[2][j];
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) Iw[i][j] = T[i][0] * Rz[j][0] + T[i][1] * Rz[j][1] + T[i][2] * Rz[j][2];
  {
    const double det = (double)Iw[0][0] * (Iw[1][1] * Iw[2][2] - Iw[1][2] * Iw[2][1]) -
                       (double)Iw[0][1] * (Iw[1][0] * Iw[2][2] - Iw[1][2] * Iw[2][0]) +
                       (double)Iw[0][2] * (Iw[1][0] * Iw[2][1] - Iw[1][1] * Iw[2][0]);
    for (int i = 0; i < 3; ++i)
      for (int j = 0; j < 3; ++j) {
        const int r1 = (j + 1) % 3, r2 = (j + 2) % 3, c1 = (i + 1) % 3, c2 = (i + 2) % 3;
        Ii[i][j] = f32(((double)Iw[r1][c1] * Iw[r2][c2] - (double)Iw[r1][c2] * Iw[r2][c1]) / det);
      }
  }
  float Ac[NX][NX] = {}, Bc[NX][NU] = {};
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) Ac[i][6 + j] = Rz[j][i];   // R_z^T (mpc.py:184)
  for (int i = 0; i < 3; ++i) Ac[3 + i][9 + i] = 1.f;
  Ac[11][12] = 1.f;
  const float minv = f32(1.0 / (double)r.rec[0]);
  for (int leg = 0; leg < 4; ++leg) {
    const double rx = r.feet[3 * leg], ry = r.feet[3 * leg + 1], rz = r.feet[3 * leg + 2];
    const double sk[3][3] = {{0, -rz, ry}, {rz, 0, -rx}, {-ry, rx, 0}};   // vec2so3 (float64)
    for (int i = 0; i < 3; ++i)
      for (int j = 0; j < 3; ++j)
        Bc[6 + i][3 * leg + j] = f32(Ii[i][0] * sk[0][j] + Ii[i][1] * sk[1][j] + Ii[i][2] * sk[2][j]);
    for (int i = 0; i < 3; ++i) Bc[9 + i][3 * leg + i] = minv;
  }
  // exact discretisation, stored float32
  float Ad[NX][NX], Bd[NX][NU];
  for (int i = 0; i < NX; ++i)
    for (int j = 0; j < NX; ++j) {
      double a2 = 0.0;
      for (int k = 0; k < NX; ++k) a2 += (double)Ac[i][k] * Ac[k][j];
      Ad[i][j] = f32((i == j ? 1.0 : 0.0) + Ac[i][j] * h + 0.5 * h * h * a2);
    }
  for (int i = 0; i < NX; ++i)
    for (int j = 0; j < NU; ++j) {
      double ab = 0.0;
      for (int k = 0; k < NX; ++k) ab += (double)Ac[i][k] * Bc[k][j];
      Bd[i][j] = f32(Bc[i][j] * h + 0.5 * h * h * ab);
    }
  // float32 powers A^0..A^N and blocks A^k Bd (mpc.py:213-230)
  // per-thread scratch reused across robots (large per-robot allocations would go to
  // mmap / munmap and serialise the threads)
  thread_local std::vector<float> P, AB;
  thread_local std::vector<double> Ts, e;
  P.assign((size_t)(N + 1) * NX * NX, 0.f);
  AB.assign((size_t)N * NX * NU, 0.f);
  for (int i = 0; i < NX; ++i)
    for (int j = 0; j < NX; ++j) P[i * NX + j] = i == j ? 1.f : 0.f;
  for (int k = 1; k <= N; ++k)
    for (int i = 0; i < NX; ++i)
      for (int j = 0; j < NX; ++j) {
        float v = 0.f;
        for (int t = 0; t < NX; ++t) v += P[(size_t)(k - 1) * NX * NX + i * NX + t] * Ad[t][j];
        P[(size_t)k * NX * NX + i * NX + j] = v;
      }
  for (int k = 0; k < N; ++k)
    for (int i = 0; i < NX; ++i)
      for (int j = 0; j < NU; ++j) {
        float v = 0.f;
        for (int t = 0; t < NX; ++t) v += P[(size_t)k * NX * NX + i * NX + t] * Bd[t][j];
        AB[(size_t)k * NX * NU + i * NU + j] = v;
      }
  // dense Su (m x n) float32, scaled rows Ts = sqrt(q) Su in float64 for H = 2 (Ts^T Ts + Rbar)
  Ts.assign((size_t)m * n, 0.0);
  for (int i = 0; i < N; ++i)
    for (int j = 0; j <= i; ++j)
      for (int a = 0; a < NX; ++a) {
        const double sq = sqrt(q[a]);
        for (int bcol = 0; bcol < NU; ++bcol)
          Ts[(size_t)(NX * i + a) * n + NU * j + bcol] = sq * (double)AB[(size_t)(i - j) * NX * NU + a * NU + bcol];
      }
  H.assign((size_t)n * n, 0.0);
  for (int row = 0; row < m; ++row) {
    const double* t = &Ts[(size_t)row * n];
    for (int a = 0; a < n; ++a) {
      const double ta = t[a];
      if (ta == 0.0) continue;
      double* Ha = &H[(size_t)a * n];
      for (int b = a; b < n; ++b) Ha[b] += ta * t[b];
    }
  }
  for (int a = 0; a < n; ++a) {
    H[(size_t)a * n + a] = 2.0 * (H[(size_t)a * n + a] + rw[a % NU]);
    for (int b = a + 1; b < n; ++b) {
      H[(size_t)a * n + b] *= 2.0;
      H[(size_t)b * n + a] = H[(size_t)a * n + b];
    }
  }
  // g = 2 Su^T Qbar (Sx x0 - xref): Sx x0 and the difference in float32 (mpc.py:233)
  e.assign(m, 0.0);
  for (int i = 0; i < N; ++i)
    for (int a = 0; a < NX; ++a) {
      float v = 0.f;
      for (int t = 0; t < NX; ++t) v += P[(size_t)(i + 1) * NX * NX + a * NX + t] * r.x0[t];
      e[NX * i + a] = (double)(v - r.xref[NX * i + a]) * sqrt(q[a]);   // Ts row scale
    }
  g.assign(n, 0.0);
  for (int row = 0; row < m; ++row) {
    const double* t = &Ts[(size_t)row * n];
    const double ev = e[row];
    for (int a = 0; a < n; ++a) g[a] += 2.0 * t[a] * ev;
  }
}

// ---------------------------------------------------------------- solve
// Goldfarb-Idnani on min 1/2 x^T G x + a^T x  s.t.  C_i . x >= b_i (dense, float64)
struct GI {
  int n;
  std::vector<double> J, R, z, d, r, u, x;
  std::vector<int> act;
  // rows i: C_i . x = sum_k coef[3 i + k] x[col0[i] + k] (a cone row touches one foot-step)
  int solve(const std::vector<double>& G0, const std::vector<double>& a, const std::vector<int>& col0,
            const std::vector<double>& coef, const std::vector<double>& b, int mrows, int max_iter) {
    thread_local std::vector<double> L;
    L = G0;
    // Cholesky G = L L^T (lower, in place)
    for (int j = 0; j < n; ++j) {
      double s = L[(size_t)j * n + j];
      for (int k = 0; k < j; ++k) s -= L[(size_t)j * n + k] * L[(size_t)j * n + k];
      const double djj = sqrt(s);
      L[(size_t)j * n + j] = djj;
      for (int i = j + 1; i < n; ++i) {
        double t = L[(size_t)i * n + j];
        for (int k = 0; k < j; ++k) t -= L[(size_t)i * n + k] * L[(size_t)j * n + k];
        L[(size_t)i * n + j] = t / djj;
      }
    }
    // J = L^-T (upper triangular): solve L^T J = I column by column
    J.assign((size_t)n * n, 0.0);
    for (int col = 0; col < n; ++col)
      for (int i = n - 1; i >= 0; --i) {
        double v = (i == col) ? 1.0 : 0.0;
        for (int k = i + 1; k < n; ++k) v -= L[(size_t)k * n + i] * J[(size_t)k * n + col];
        J[(size_t)i * n + col] = v / L[(size_t)i * n + i];
      }
    // unconstrained minimiser x = -G^-1 a = -J J^T a
    x.assign(n, 0.0);
    {
      std::vector<double> t(n, 0.0);
      for (int k = 0; k < n; ++k)
        for (int i = 0; i < n; ++i) t[k] += J[(size_t)i * n + k] * a[i];
      for (int i = 0; i < n; ++i) {
        double v = 0.0;
        for (int k = 0; k < n; ++k) v += J[(size_t)i * n + k] * t[k];
        x[i] = -v;
      }
    }
    R.assign((size_t)n * n, 0.0);
    u.clear();
    act.clear();
    d.assign(n, 0.0);
    z.assign(n, 0.0);
    int it = 0;
    double bscale = 1.0;
    for (int i = 0; i < mrows; ++i) bscale = fmax(bscale, 1.0 + fabs(b[i]));
    const double tol = 1e-11 * bscale;
    while (true) {
      int p = -1;
      double smin = -tol;
      for (int i = 0; i < mrows; ++i) {
        const double* cf = &coef[3 * i];
        const double s = cf[0] * x[col0[i]] + cf[1] * x[col0[i] + 1] + cf[2] * x[col0[i] + 2] - b[i];
        if (s < smin) {
          smin = s;
          p = i;
        }
      }
      if (p < 0) return it;
      const int c0 = col0[p];
      const double* cp = &coef[3 * p];
      double up = 0.0;
      while (true) {
        if (++it > max_iter) return -it;
        const int q = (int)act.size();
        for (int k = 0; k < n; ++k)
          d[k] = J[(size_t)c0 * n + k] * cp[0] + J[(size_t)(c0 + 1) * n + k] * cp[1] + J[(size_t)(c0 + 2) * n + k] * cp[2];
        for (int i = 0; i < n; ++i) {
          double v = 0.0;
          for (int k = q; k < n; ++k) v += J[(size_t)i * n + k] * d[k];
          z[i] = v;
        }
        r.assign(q, 0.0);
        for (int i = q - 1; i >= 0; --i) {
          double v = d[i];
          for (int k = i + 1; k < q; ++k) v -= R[(size_t)i * n + k] * r[k];
          r[i] = v / R[(size_t)i * n + i];
        }
        double t1 = INFINITY;
        int l = -1;
        for (int j = 0; j < q; ++j)
          if (r[j] > 0.0 && u[j] / r[j] < t1) {
            t1 = u[j] / r[j];
            l = j;
          }
        double dn = 0.0;
        for (int i = 0; i < n; ++i) dn += d[i] * d[i];
        const double zn = cp[0] * z[c0] + cp[1] * z[c0 + 1] + cp[2] * z[c0 + 2];
        const double sp = cp[0] * x[c0] + cp[1] * x[c0 + 1] + cp[2] * x[c0 + 2] - b[p];
        const double t2 = zn > 1e-14 * fmax(dn, 1e-300) ? -sp / zn : INFINITY;
        const double t = fmin(t1, t2);
        if (!isfinite(t)) return -it;
        if (isfinite(t2))
          for (int i = 0; i < n; ++i) x[i] += t * z[i];
        for (int j = 0; j < q; ++j) u[j] -= t * r[j];
        up += t;
        if (isfinite(t2) && t == t2) {
          add(q);
          act.push_back(p);
          u.push_back(up);
          break;
        }
        drop(l);
      }
    }
  }
  void add(int q) {
    // Householder on d[q:] ; R[:q, q] = d[:q], R[q, q] = -sign alpha
    double alpha = 0.0;
    for (int k = q; k < n; ++k) alpha += d[k] * d[k];
    alpha = sqrt(alpha);
    double rqq = d[q];
    if (q < n - 1 && alpha > 0.0) {
      const double sign = d[q] >= 0.0 ? 1.0 : -1.0;
      std::vector<double> v(d.begin() + q, d.end());
      v[0] += sign * alpha;
      double vv = 0.0;
      for (double w : v) vv += w * w;
      if (vv > 0.0)
        for (int i = 0; i < n; ++i) {
          double s = 0.0;
          for (int k = q; k < n; ++k) s += J[(size_t)i * n + k] * v[k - q];
          s *= 2.0 / vv;
          for (int k = q; k < n; ++k) J[(size_t)i * n + k] -= s * v[k - q];
        }
      rqq = -sign * alpha;
    }
    for (int i = 0; i < q; ++i) R[(size_t)i * n + q] = d[i];
    R[(size_t)q * n + q] = rqq;
  }
  void drop(int l) {
    const int q = (int)act.size();
    // remove column l of R (q x q upper), restore triangularity by Givens on rows l..q-1
    for (int j = l; j < q - 1; ++j)
      for (int i = 0; i < q; ++i) R[(size_t)i * n + j] = R[(size_t)i * n + j + 1];
    for (int i = 0; i < q; ++i) R[(size_t)i * n + q - 1] = 0.0;
    for (int j = l; j < q - 1; ++j) {
      const double a_ = R[(size_t)j * n + j], b_ = R[(size_t)(j + 1) * n + j];
      const double hh = hypot(a_, b_);
      if (hh == 0.0) continue;
      const double cc = a_ / hh, ss = b_ / hh;
      for (int k = 0; k < q - 1; ++k) {
        const double r1 = R[(size_t)j * n + k], r2 = R[(size_t)(j + 1) * n + k];
        R[(size_t)j * n + k] = cc * r1 + ss * r2;
        R[(size_t)(j + 1) * n + k] = -ss * r1 + cc * r2;
      }
      for (int i = 0; i < n; ++i) {
        const double j1 = J[(size_t)i * n + j], j2 = J[(size_t)i * n + j + 1];
        J[(size_t)i * n + j] = cc * j1 + ss * j2;
        J[(size_t)i * n + j + 1] = -ss * j1 + cc * j2;
      }
    }
    for (int k = 0; k < n; ++k) R[(size_t)(q - 1) * n + k] = 0.0;
    for (int i = 0; i < q; ++i)
      if (i >= q - 1)
        for (int k = 0; k < n; ++k) R[(size_t)i * n + k] = 0.0;
    act.erase(act.begin() + l);
    u.erase(u.begin() + l);
  }
};

// one robot: formulate, eliminate swing variables, solve; U (12N) out
int solve_robot(const Robot& r, int N, double h, const double* q, const double* rw, double* U, double& tf,
                double& ts) {
  using clk = std::chrono::steady_clock;
  const auto t0 = clk::now();
  thread_local std::vector<double> H, g;
  formulate(r, N, h, q, rw, H, g);
  // cone rows (mpc.py:239-245 for n = e_z; per-robot normal otherwise)
  double nx = r.rec[9], ny = r.rec[10], nz = r.rec[11];
  const double nn = sqrt(nx * nx + ny * ny + nz * nz);
  if (!(nn > 0.0)) {
    nx = 0.0;
    ny = 0.0;
    nz = 1.0;
  } else {
    nx /= nn;
    ny /= nn;
    nz /= nn;
  }
  double t1x = 1.0 - nx * nx, t1y = -nx * ny, t1z = -nx * nz;
  const double tn = sqrt(t1x * t1x + t1y * t1y + t1z * t1z);
  t1x /= tn;
  t1y /= tn;
  t1z /= tn;
  const double t2x = ny * t1z - nz * t1y, t2y = nz * t1x - nx * t1z, t2z = nx * t1y - ny * t1x;
  const double mu = r.rec[7], fzmax = r.rec[8];
  const double rows[6][3] = {{t1x + mu * nx, t1y + mu * ny, t1z + mu * nz},
                             {-t1x + mu * nx, -t1y + mu * ny, -t1z + mu * nz},
                             {t2x + mu * nx, t2y + mu * ny, t2z + mu * nz},
                             {-t2x + mu * nx, -t2y + mu * ny, -t2z + mu * nz},
                             {nx, ny, nz},
                             {-nx, -ny, -nz}};
  thread_local std::vector<int> idx;
  thread_local std::vector<double> ubs;
  idx.clear();
  ubs.clear();
  for (int k = 0; k < 4 * N; ++k)
    if (r.contact[k] > 0.f) {
      idx.push_back(k);
      ubs.push_back((double)r.contact[k] * fzmax);
    }
  const int S = (int)idx.size(), n = 3 * S, m = 6 * S;
  thread_local std::vector<double> Hr, gr, coef, b;
  thread_local std::vector<int> col0;
  Hr.assign((size_t)n * n, 0.0);
  gr.assign(n, 0.0);
  coef.assign((size_t)3 * m, 0.0);
  b.assign(m, 0.0);
  col0.assign(m, 0);
  for (int a = 0; a < n; ++a) {
    const int fa = 3 * idx[a / 3] + a % 3;
    gr[a] = g[fa];
    for (int c = 0; c < n; ++c) Hr[(size_t)a * n + c] = H[(size_t)fa * (NU * N) + 3 * idx[c / 3] + c % 3];
  }
  for (int j = 0; j < S; ++j)
    for (int rr = 0; rr < 6; ++rr) {
      col0[6 * j + rr] = 3 * j;
      for (int k = 0; k < 3; ++k) coef[3 * (6 * j + rr) + k] = rows[rr][k];
      b[6 * j + rr] = rr == 5 ? -ubs[j] : 0.0;
    }
  const auto t1 = clk::now();
  int it = 0;
  for (int k = 0; k < NU * N; ++k) U[k] = 0.0;
  if (n > 0) {
    thread_local GI gi;
    gi.n = n;
    it = gi.solve(Hr, gr, col0, coef, b, m, 100000);
    for (int a = 0; a < n; ++a) U[3 * idx[a / 3] + a % 3] = gi.x[a];
  }
  const auto t2 = clk::now();
  tf += std::chrono::duration<double>(t1 - t0).count();
  ts += std::chrono::duration<double>(t2 - t1).count();
  return it;
}

}  // namespace

extern "C" {

// B robots (layouts of include/mpcqp.h), horizon N, model step dt, diagonal weights q[13],
// r[12]; U [B][N][12] float64 out; iters [B] (negative: iteration cap / failure).
// t_form / t_solve: summed thread seconds.  threads <= 0: OpenMP default.
int mpc_cpu_solve_batch(int B, int N, const float* x0, const float* xref, const float* contact, const float* feet,
                        const float* robot, double dt, const double* q, const double* r, double* U, int* iters,
                        double* t_form, double* t_solve, int threads) {
  double tf = 0.0, ts = 0.0;
  if (threads > 0) omp_set_num_threads(threads);
#pragma omp parallel for schedule(dynamic, 1) reduction(+ : tf, ts)
  for (int bb = 0; bb < B; ++bb) {
    Robot rb{x0 + (size_t)bb * NX, xref + (size_t)bb * N * NX, contact + (size_t)bb * N * 4, feet + (size_t)bb * 12,
             robot + (size_t)bb * 16};
    const int it = solve_robot(rb, N, dt, q, r, U + (size_t)bb * N * NU, tf, ts);
    if (iters) iters[bb] = it;
  }
  if (t_form) *t_form = tf;
  if (t_solve) *t_solve = ts;
  return 0;
}

}  // extern "C"
