// mpcqp_ipm.h -- the large capacity class: robots with more than 126 stance
// variables (standing and near-standing schedules at N = 16 / 20, n up to 240),
// one wave per robot (included by mpcqp.hip inside its anonymous namespace).
//
// The dense classes keep the n x n reduced inverse Hessian in registers; at
// n = 240 it no longer fits one CU.  This class never forms H: it solves the
// same QP (mpc.py:211-286) on the uncondensed horizon,
//
//   min 1/2 sum_k x_{k+1}^T Qh x_{k+1} + qh_k^T x_{k+1} + 1/2 u_k^T Rh u_k
//   s.t. x_{k+1} = A_d x_k + B_d u_k,   cone rows a_r . f_j >= h_r per stance foot-step,
//
// (Qh = 2 diag q, Rh = 2 diag r, qh_k = -Qh xref_k: exactly 1/2 U^T H U + g^T U + const,
// H = 2(Su^T Qbar Su + Rbar), so the optimum is the Drake-branch QP's) by
//   * a Mehrotra predictor-corrector interior point whose Newton systems
//     (H + G^T D G) d = rhs are solved by a Riccati recursion over the N stages,
//     in information form: E_k = B W_k B^T (W_k = per-leg 3x3 (Rh + G^T D G)^-1),
//     S_k = (I + P_{k+1} E_k)^-1 P_{k+1} (Gauss-Jordan on [I + P E | P]),
//     P_k = Qh + A^T S_k A.  (The textbook P - P B (R + B^T P B)^-1 B^T P loses ~4
//     digits: B_d has a 6-dimensional null space -- internal forces between feet --
//     where only Rh = 2e-5 acts.)  The constant gravity state x[12] never moves in a
//     Newton direction, so the recursions run on the 12-dimensional state.
//   * an active-set polish: once mu is small, the rows with lambda > s define an
//     equality-constrained QP, solved exactly on each foot's null space (Gram-Schmidt
//     of its active rows; the same Riccati with B_leg W_j B_leg^T, W_j = P_j (P_j Rh P_j
//     + I - P_j)^-1 P_j) plus two Newton refinements, then verified: stationarity on
//     the null spaces, primal feasibility of every row and multipliers >= 0 (the
//     gradient in the cone of the foot's active rows, Caratheodory subsets).  A failed
//     check corrects the set (violated rows in, the most negative multiplier out) up
//     to IPM_NCORR times; the IPM continues otherwise.
// A verified polish is the exact optimum (status OK); tools/ipm_proto.py is the NumPy
// model of every step (64 golden / synthetic cases, worst error 1.3e-6).

#include "mpcqp_ipm_foot.h"

constexpr int IPM_MAX_IT = 60;
constexpr int IPM_NCORR = 8;
constexpr int IPM_NREF = 2;
constexpr double IPM_TAU = 0.995;
constexpr double IPM_POLISH_MU = 1e-7;
constexpr double IPM_MU_FLOOR = 1e-13;
constexpr double IPM_STAT_TOL = 1e-10;
constexpr int IPM_FPL = 2;   // stance foot-steps per lane (4 kMaxN <= 128)

struct alignas(16) IpmShared {
  union {
    struct {
      Form f;
      FormY fy;
    } fa;                          // formulation scratch (dead once Bm / x0 / xr are copied)
    double S[kMaxN][144];          // Riccati S_k (12 x 12, row-major)
  };
  RobotMeta mt;
  double Bm[12][12];               // B_d rows 0..11 (row 12 is 0)
  double nmr[3][3];                // h R_z^T: A_d[r][6 + c] (r < 3)
  double x0[16];
  double xr[kMaxN][NX];            // xref, float64
  double qh[16];                   // 2 q
  double rh[NU];                   // 2 r
  double W[4 * kMaxN][9];          // per stance foot-step 3x3 weight
  double E[144];
  double M[12][24];                // Gauss-Jordan [I + P E | P]
  double P[144];
  double U[kMaxN][NU];             // iterate (swing entries 0)
  double dU[kMaxN][NU];
  double rhs[kMaxN][NU];
  double gr[kMaxN][NU];
  double Y[kMaxN][NU];
  double By[kMaxN][NU];
  double Us[kMaxN][NU];            // the IPM iterate while a polish overwrites U
  double X[kMaxN + 1][16];
  double v0[16], v1[16], v2[16], vn[2][16];
};

__device__ __forceinline__ double wave_sum_d(double v) {
  v += dpp_d<DPP_XOR1>(v);
  v += dpp_d<DPP_XOR2>(v);
  v += dpp_d<DPP_HMIRROR>(v);
  v += dpp_d<DPP_MIRROR>(v);
  {
    const double t = dpp_m<DPP_BCAST15, 0xA>(v);
    v = (((threadIdx.x & 63) >> 4) & 1) ? v + t : v;   // rows 1, 3 += lane 15 of rows 0, 2
  }
  {
    const double t = dpp_m<DPP_BCAST31, 0xC>(v);
    v = ((threadIdx.x & 63) >> 5) ? v + t : v;          // rows 2, 3 += lane 31
  }
  return readlane_d(v, 63);
}
__device__ __forceinline__ double wave_min_all(double v) { return wave_min(v); }
__device__ __forceinline__ double wave_max_all(double v) { return wave_max_d(v); }


// One robot with n > 126 stance variables.  Called by a 64-thread workgroup.
__device__ void solve_robot_ipm(const KParams& KP, int b, IpmShared& sm, const float* __restrict__ x0g,
                                const float* __restrict__ xrefg, const float* __restrict__ contactg,
                                const float* __restrict__ feetg, const float* __restrict__ robotg,
                                float* __restrict__ u0g, float* __restrict__ Ug, int* __restrict__ statusg,
                                int* __restrict__ itersg) {
  constexpr int NT = LANES;
  const int lane = threadIdx.x;
  const int N = KP.N;
  const double h = KP.dt;

  // ------------------------------------------------ formulation (mpcqp_form.h)
  Form& smf = sm.fa.f;
  if (!form_stage<NT>(smf, N, b, lane, x0g, xrefg, contactg, feetg, robotg)) {
    write_empty_t<NT>(b, lane, N, MPCQP_STATUS_NONFINITE, u0g, Ug, statusg, itersg);
    return;
  }
  form_stance(smf, sm.mt, N, lane);
  fsync<NT>();
  const int S = uni(sm.mt.S);
  form_model<NT>(KP, smf, sm.fa.fy, sm.mt, N, lane);
  fsync<NT>();
  {
    const double minv = smf.minv;
    for (int e = lane; e < 144; e += NT) {
      const int i = e / 12, c = e % 12;
      double v = 0.0;
      if (i < 3) v = smf.G[i][c] * (0.5 * h * h);
      else if (i < 6) v = (c % 3 == i - 3) ? 0.5 * h * h * minv : 0.0;
      else if (i < 9) v = smf.K[i - 6][c] * h;
      else v = (c % 3 == i - 9) ? h * minv : 0.0;
      sm.Bm[i][c] = v;
    }
    if (lane < 9) {
      const int r = lane / 3, c = lane % 3;   // (R_z^T)[r][c] = R_z[c][r]
      const double co = smf.rz[0], si = smf.rz[1];
      const double rzcr = c == 2 ? (r == 2 ? 1.0 : 0.0) : (r == 2 ? 0.0 : (c == r ? co : (c == 0 ? -si : si)));
      sm.nmr[r][c] = h * rzcr;
    }
    if (lane < NX) {
      sm.x0[lane] = (double)smf.in[IN_X0 + lane];
      sm.qh[lane] = 2.0 * KP.q[lane];
    }
    if (lane < NU) sm.rh[lane] = 2.0 * KP.r[lane];
    for (int e = lane; e < N * NX; e += NT) sm.xr[e / NX][e % NX] = (double)smf.in[IN_XREF + e];
    for (int e = lane; e < N * NU; e += NT) sm.U[e / NU][e % NU] = 0.0;
  }
  fsync<NT>();   // the formulation scratch (union with S) is dead from here on

  // ------------------------------------------------ per-lane foot-steps
  const bool implied = sm.mt.fz0_implied != 0;
  int jt[IPM_FPL], jl[IPM_FPL];
  bool own[IPM_FPL];
  double hb[IPM_FPL];   // h of row 5: -ub
#pragma unroll
  for (int q = 0; q < IPM_FPL; ++q) {
    const int j = lane + LANES * q;
    own[q] = j < S;
    jt[q] = own[q] ? sm.mt.foot_t[j] : 0;
    jl[q] = own[q] ? sm.mt.foot_leg[j] : 0;
    hb[q] = own[q] ? -sm.mt.ub[j] : 0.0;
  }
  auto live = [&](int r) -> bool { return r != 4 || !implied; };
  auto arow = [&](int r, int k) -> double { return sm.mt.rows[r][k]; };
  auto hrow = [&](int q, int r) -> double { return r == 5 ? hb[q] : 0.0; };
  const int R = implied ? 5 : 6;
  const double m_tot = (double)(S * R);

  // ------------------------------------------------ stage recursions
  // Nm = A_d - I on the 13-state: rows 0..2 <- h R_z^T x[6..8]; rows 3..5 <- h x[9..11]
  // (+ h^2/2 x[12] on row 5); row 11 <- h x[12]
  auto gradient = [&]() {   // sm.gr = H U + g on stance coordinates (forward sim + adjoint)
    if (lane < NX) sm.X[0][lane] = sm.x0[lane];
    fsync<NT>();
    for (int k = 0; k < N; ++k) {
      if (lane < NX) {
        const double* x = sm.X[k];
        double v = x[lane];
        if (lane < 3) v += sm.nmr[lane][0] * x[6] + sm.nmr[lane][1] * x[7] + sm.nmr[lane][2] * x[8];
        else if (lane < 6) v += h * x[lane + 6] + (lane == 5 ? 0.5 * h * h * x[12] : 0.0);
        else if (lane == 11) v += h * x[12];
        if (lane < 12) {
#pragma unroll
          for (int c = 0; c < NU; ++c) v = fma(sm.Bm[lane][c], sm.U[k][c], v);
        }
        sm.X[k + 1][lane] = v;
      }
      fsync<NT>();
    }
    for (int k = N - 1; k >= 0; --k) {
      double* nu = sm.vn[k & 1];
      const double* np = sm.vn[(k + 1) & 1];
      if (lane < NX) {
        double v = sm.qh[lane] * (sm.X[k + 1][lane] - sm.xr[k][lane]);
        if (k < N - 1) {
          double a = np[lane];
          if (lane >= 6 && lane < 9)
            a += sm.nmr[0][lane - 6] * np[0] + sm.nmr[1][lane - 6] * np[1] + sm.nmr[2][lane - 6] * np[2];
          else if (lane >= 9 && lane < 12) a += h * np[lane - 6];
          else if (lane == 12) a += 0.5 * h * h * np[5] + h * np[11];
          v += a;
        }
        nu[lane] = v;
      }
      fsync<NT>();
      if (lane < NU) {
        const bool st = sm.mt.stance_of[4 * k + lane / 3] >= 0;
        double g = sm.rh[lane] * sm.U[k][lane];
#pragma unroll
        for (int i = 0; i < 12; ++i) g = fma(sm.Bm[i][lane], nu[i], g);
        sm.gr[k][lane] = st ? g : 0.0;
      }
    }
    fsync<NT>();
  };

  // (A^T v)[i] on the 12-state, v in LDS
  auto at_apply = [&](const double* v, int i) -> double {
    double a = v[i];
    if (i >= 6 && i < 9) a += sm.nmr[0][i - 6] * v[0] + sm.nmr[1][i - 6] * v[1] + sm.nmr[2][i - 6] * v[2];
    else if (i >= 9) a += h * v[i - 6];
    return a;
  };
  // (A v)[i] on the 12-state
  auto a_apply = [&](const double* v, int i) -> double {
    double a = v[i];
    if (i < 3) a += sm.nmr[i][0] * v[6] + sm.nmr[i][1] * v[7] + sm.nmr[i][2] * v[8];
    else if (i < 6) a += h * v[i + 6];
    return a;
  };

  // Riccati factorisation with the per-foot-step weights sm.W: S_k for every stage
  auto factor = [&]() {
    for (int e = lane; e < 144; e += NT) sm.P[e] = (e / 12 == e % 12) ? sm.qh[e / 12] : 0.0;
    fsync<NT>();
    for (int k = N - 1; k >= 0; --k) {
      // E_k = sum_legs B_leg W B_leg^T
      for (int e = lane; e < 144; e += NT) {
        const int i = e / 12, m = e % 12;
        double v = 0.0;
#pragma unroll
        for (int l = 0; l < 4; ++l) {
          const int j = sm.mt.stance_of[4 * k + l];
          if (j >= 0) {
            const double* w = sm.W[j];
            const double* bi = &sm.Bm[i][3 * l];
            const double* bm = &sm.Bm[m][3 * l];
#pragma unroll
            for (int a = 0; a < 3; ++a) v = fma(bi[a], w[3 * a] * bm[0] + w[3 * a + 1] * bm[1] + w[3 * a + 2] * bm[2], v);
          }
        }
        sm.E[e] = v;
      }
      fsync<NT>();
      // [I + P E | P]
      double tv[3];
#pragma unroll
      for (int t = 0; t < 3; ++t) {
        const int e = lane + NT * t;
        tv[t] = 0.0;
        if (e < 144) {
          const int i = e / 12, j = e % 12;
          double v = (i == j) ? 1.0 : 0.0;
#pragma unroll
          for (int m = 0; m < 12; ++m) v = fma(sm.P[12 * i + m], sm.E[12 * m + j], v);
          tv[t] = v;
        }
      }
#pragma unroll
      for (int t = 0; t < 3; ++t) {
        const int e = lane + NT * t;
        if (e < 144) {
          sm.M[e / 12][e % 12] = tv[t];
          sm.M[e / 12][12 + e % 12] = sm.P[e];
        }
      }
      fsync<NT>();
      // Gauss-Jordan: right half becomes (I + P E)^-1 P
      for (int kk = 0; kk < 12; ++kk) {
        const double ip = 1.0 / sm.M[kk][kk];
        double nv[5];
#pragma unroll
        for (int t = 0; t < 5; ++t) {
          const int e = lane + NT * t;
          const int i = e / 24, j = e % 24;
          nv[t] = 0.0;
          if (e < 288 && j > kk) {
            const double rowv = sm.M[kk][j] * ip;
            nv[t] = (i == kk) ? rowv : fma(-sm.M[i][kk], rowv, sm.M[i][j]);
          }
        }
#pragma unroll
        for (int t = 0; t < 5; ++t) {
          const int e = lane + NT * t;
          const int i = e / 24, j = e % 24;
          if (e < 288 && j > kk) sm.M[i][j] = nv[t];
        }
        fsync<NT>();
      }
      for (int e = lane; e < 144; e += NT) {
        const int i = e / 12, j = e % 12;
        sm.S[k][e] = 0.5 * (sm.M[i][12 + j] + sm.M[j][12 + i]);
      }
      fsync<NT>();
      if (k > 0) {
        // P_k = Qh + A^T S_k A  (A = I + Nm on the 12-state)
        const double* Sk = sm.S[k];
        for (int e = lane; e < 144; e += NT) {
          const int i = e / 12, j = e % 12;
          // (S A)[m][j] for the rows m that column i of Nm touches, and S[i][.] A[.][j]
          auto sa = [&](int m) -> double {   // (S_k A)[m][j]
            double v = Sk[12 * m + j];
            if (j >= 6 && j < 9) v += Sk[12 * m + 0] * sm.nmr[0][j - 6] + Sk[12 * m + 1] * sm.nmr[1][j - 6] +
                                      Sk[12 * m + 2] * sm.nmr[2][j - 6];
            else if (j >= 9) v += h * Sk[12 * m + j - 6];
            return v;
          };
          double v = sa(i);
          if (i >= 6 && i < 9) v += sm.nmr[0][i - 6] * sa(0) + sm.nmr[1][i - 6] * sa(1) + sm.nmr[2][i - 6] * sa(2);
          else if (i >= 9) v += h * sa(i - 6);
          if (i == j) v += sm.qh[i];
          sm.P[e] = v;
        }
        fsync<NT>();
      }
    }
  };

  // (H + G^T D G) d = rhs restricted to the foot-steps' subspaces (sm.rhs -> sm.dU)
  auto lsolve = [&]() {
    if (lane < 12) sm.v0[lane] = 0.0;
    fsync<NT>();
    for (int k = N - 1; k >= 0; --k) {
      if (lane < NU) {
        const int j = sm.mt.stance_of[4 * k + lane / 3];
        double z = 0.0;
        if (j >= 0) {
          z = -sm.rhs[k][lane];
#pragma unroll
          for (int i = 0; i < 12; ++i) z = fma(sm.Bm[i][lane], sm.v0[i], z);
        }
        sm.v1[lane] = z;
      }
      fsync<NT>();
      if (lane < NU) {
        const int l = lane / 3, a = lane % 3;
        const int j = sm.mt.stance_of[4 * k + l];
        double y = 0.0;
        if (j >= 0) {
          const double* w = sm.W[j] + 3 * a;
          y = w[0] * sm.v1[3 * l] + w[1] * sm.v1[3 * l + 1] + w[2] * sm.v1[3 * l + 2];
        }
        sm.Y[k][lane] = y;
      }
      fsync<NT>();
      if (lane < 12) {
        double v = 0.0;
#pragma unroll
        for (int c = 0; c < NU; ++c) v = fma(sm.Bm[lane][c], sm.Y[k][c], v);
        sm.By[k][lane] = v;
      }
      fsync<NT>();
      if (k > 0) {
        if (lane < 12) {
          double t = sm.v0[lane];
#pragma unroll
          for (int m = 0; m < 12; ++m) t = fma(-sm.S[k][12 * lane + m], sm.By[k][m], t);
          sm.v2[lane] = t;
        }
        fsync<NT>();
        if (lane < 12) sm.v0[lane] = at_apply(sm.v2, lane);
        fsync<NT>();
      }
    }
    if (lane < 12) sm.v0[lane] = 0.0;   // dx
    fsync<NT>();
    for (int k = 0; k < N; ++k) {
      if (lane < 12) sm.v1[lane] = sm.By[k][lane] - a_apply(sm.v0, lane);
      fsync<NT>();
      if (lane < 12) {
        double w = 0.0;
#pragma unroll
        for (int m = 0; m < 12; ++m) w = fma(sm.S[k][12 * lane + m], sm.v1[m], w);
        sm.v2[lane] = w;
      }
      fsync<NT>();
      if (lane < NU) {
        double z = 0.0;
#pragma unroll
        for (int i = 0; i < 12; ++i) z = fma(sm.Bm[i][lane], sm.v2[i], z);
        sm.v1[lane] = z;
      }
      fsync<NT>();
      if (lane < NU) {
        const int l = lane / 3, a = lane % 3;
        const int j = sm.mt.stance_of[4 * k + l];
        double d = 0.0;
        if (j >= 0) {
          const double* w = sm.W[j] + 3 * a;
          d = w[0] * sm.v1[3 * l] + w[1] * sm.v1[3 * l + 1] + w[2] * sm.v1[3 * l + 2] - sm.Y[k][lane];
        }
        sm.dU[k][lane] = d;
      }
      fsync<NT>();
      if (lane < 12) {
        double v = a_apply(sm.v0, lane);
#pragma unroll
        for (int c = 0; c < NU; ++c) v = fma(sm.Bm[lane][c], sm.dU[k][c], v);
        sm.v2[lane] = v;
      }
      fsync<NT>();
      if (lane < 12) sm.v0[lane] = sm.v2[lane];
      fsync<NT>();
    }
  };

  // per-foot-step helpers
  auto fvec = [&](const double (*A)[NU], int q, double (&o)[3]) {
    const double* p = &A[jt[q]][3 * jl[q]];
    o[0] = p[0];
    o[1] = p[1];
    o[2] = p[2];
  };
  auto adot = [&](int r, const double (&v)[3]) -> double {
    return arow(r, 0) * v[0] + arow(r, 1) * v[1] + arow(r, 2) * v[2];
  };
  // W_j = (Rh_leg + sum_r d_r a_r a_r^T)^-1
  auto set_w_ipm = [&](int q, const double (&d)[6]) {
    double a[9];
#pragma unroll
    for (int x = 0; x < 3; ++x)
#pragma unroll
      for (int y = 0; y < 3; ++y) {
        double v = (x == y) ? sm.rh[3 * jl[q] + x] : 0.0;
#pragma unroll
        for (int r = 0; r < 6; ++r)
          if (live(r)) v = fma(d[r] * arow(r, x), arow(r, y), v);
        a[3 * x + y] = v;
      }
    double o[9];
    inv3(a, o);
    double* w = sm.W[lane + LANES * q];
#pragma unroll
    for (int e = 0; e < 9; ++e) w[e] = o[e];
  };

  double s[IPM_FPL][6], lam[IPM_FPL][6];
  int status = MPCQP_STATUS_MAX_ITER;
  int nfact = 0;
#ifdef MPCQP_IPM_DEBUG
  // diagnostic build: 8 floats per IPM iteration written to U (the solution is not)
  int dbg_n = 0;
  auto dbg = [&](double v) {
    if (lane == 0 && Ug && dbg_n < N * NU) Ug[(size_t)b * N * NU + dbg_n] = (float)v;
    ++dbg_n;
  };
  double dbg_p[5] = {0.0, 0.0, 0.0, 0.0, 0.0};
#endif

  // scales: gradient at U = 0 and the largest bound
  gradient();
  double gmax = 0.0, hmax = 0.0;
#pragma unroll
  for (int q = 0; q < IPM_FPL; ++q) {
    if (!own[q]) continue;
    double g[3];
    fvec(sm.gr, q, g);
    gmax = fmax(gmax, fmax(fabs(g[0]), fmax(fabs(g[1]), fabs(g[2]))));
    hmax = fmax(hmax, fabs(hb[q]));
  }
  const double gscale = 1.0 + sgpr_d(wave_max_all(gmax));
  const double hscale = 1.0 + sgpr_d(wave_max_all(hmax));
  const double tol_g = 1e-9 * gscale, tol_h = 1e-9 * hscale;

  // ---- start: minimiser under a mild barrier weight, slacks shifted into the interior
  {
#pragma unroll
    for (int q = 0; q < IPM_FPL; ++q)
      if (own[q]) {
        double d[6];
#pragma unroll
        for (int r = 0; r < 6; ++r) d[r] = 1e-2;
        set_w_ipm(q, d);
      }
    for (int e = lane; e < N * NU; e += NT) sm.rhs[e / NU][e % NU] = -sm.gr[e / NU][e % NU];
    fsync<NT>();
    factor();
    ++nfact;
    lsolve();
    for (int e = lane; e < N * NU; e += NT) sm.U[e / NU][e % NU] = sm.dU[e / NU][e % NU];
    fsync<NT>();
#pragma unroll
    for (int q = 0; q < IPM_FPL; ++q) {
      double f[3];
      fvec(sm.U, q, f);
#pragma unroll
      for (int r = 0; r < 6; ++r) {
        s[q][r] = own[q] && live(r) ? fmax(adot(r, f) - hrow(q, r), 1.0) : 1.0;
        lam[q][r] = own[q] && live(r) ? 1.0 : 0.0;
      }
    }
  }

  // ---- active-set polish on the rows `act`; true when verified (sm.U = the optimum)
  int act[IPM_FPL];
  auto polish = [&]() -> bool {
    double pj[IPM_FPL][9];
    unsigned int nq_of[IPM_FPL];
#pragma unroll
    for (int q = 0; q < IPM_FPL; ++q) {
      pj[q][0] = 1.0; pj[q][1] = 0.0; pj[q][2] = 0.0;
      pj[q][3] = 0.0; pj[q][4] = 1.0; pj[q][5] = 0.0;
      pj[q][6] = 0.0; pj[q][7] = 0.0; pj[q][8] = 1.0;
      nq_of[q] = 0;
      if (!own[q]) continue;
      // Gram-Schmidt of the active rows (row 5 first: the only one with h != 0)
      double qv[3][3], L[3][3], fp[3] = {0.0, 0.0, 0.0}, c[3] = {0.0, 0.0, 0.0};
      int nq = 0;
      for (int o = 0; o < 6; ++o) {
        const int r = o == 0 ? 5 : o - 1;
        if (!((act[q] >> r) & 1) || !live(r) || nq == 3) continue;
        double v[3] = {arow(r, 0), arow(r, 1), arow(r, 2)};
        const double n0 = sqrt(v[0] * v[0] + v[1] * v[1] + v[2] * v[2]);
        double coef[3] = {0.0, 0.0, 0.0};
        for (int i = 0; i < nq; ++i) {
          coef[i] = qv[i][0] * v[0] + qv[i][1] * v[1] + qv[i][2] * v[2];
          v[0] -= coef[i] * qv[i][0];
          v[1] -= coef[i] * qv[i][1];
          v[2] -= coef[i] * qv[i][2];
        }
        const double nv = sqrt(v[0] * v[0] + v[1] * v[1] + v[2] * v[2]);
        if (!(nv > 1e-9 * n0)) continue;   // dependent on the rows taken
        for (int i = 0; i < nq; ++i) L[nq][i] = coef[i];
        L[nq][nq] = nv;
        qv[nq][0] = v[0] / nv;
        qv[nq][1] = v[1] / nv;
        qv[nq][2] = v[2] / nv;
        // forward substitution of L c = h over the independent rows
        double hv = hrow(q, r);
        for (int i = 0; i < nq; ++i) hv -= L[nq][i] * c[i];
        c[nq] = hv / nv;
        ++nq;
      }
      for (int i = 0; i < nq; ++i)
        for (int x = 0; x < 3; ++x) fp[x] += c[i] * qv[i][x];
      for (int x = 0; x < 3; ++x)
        for (int y = 0; y < 3; ++y) {
          double v = (x == y) ? 1.0 : 0.0;
          for (int i = 0; i < nq; ++i) v -= qv[i][x] * qv[i][y];
          pj[q][3 * x + y] = v;
        }
      nq_of[q] = nq;
      // W = P_j (P_j Rh P_j + I - P_j)^-1 P_j
      double a[9], o[9];
#pragma unroll
      for (int x = 0; x < 3; ++x)
#pragma unroll
        for (int y = 0; y < 3; ++y) {
          double v = -pj[q][3 * x + y] + ((x == y) ? 1.0 : 0.0);
#pragma unroll
          for (int z = 0; z < 3; ++z) v = fma(pj[q][3 * x + z] * sm.rh[3 * jl[q] + z], pj[q][3 * z + y], v);
          a[3 * x + y] = v;
        }
      inv3(a, o);
      double t[9];
#pragma unroll
      for (int x = 0; x < 3; ++x)
#pragma unroll
        for (int y = 0; y < 3; ++y)
          t[3 * x + y] = o[3 * x] * pj[q][y] + o[3 * x + 1] * pj[q][3 + y] + o[3 * x + 2] * pj[q][6 + y];
      double* w = sm.W[lane + LANES * q];
#pragma unroll
      for (int x = 0; x < 3; ++x)
#pragma unroll
        for (int y = 0; y < 3; ++y)
          w[3 * x + y] = pj[q][3 * x] * t[y] + pj[q][3 * x + 1] * t[3 + y] + pj[q][3 * x + 2] * t[6 + y];
      double* u = &sm.U[jt[q]][3 * jl[q]];
      u[0] = fp[0];
      u[1] = fp[1];
      u[2] = fp[2];
    }
    fsync<NT>();
    factor();
    ++nfact;
    for (int rf = 0; rf < IPM_NREF; ++rf) {
      gradient();
      for (int e = lane; e < N * NU; e += NT) sm.rhs[e / NU][e % NU] = 0.0;
      fsync<NT>();
#pragma unroll
      for (int q = 0; q < IPM_FPL; ++q)
        if (own[q]) {
          double g[3];
          fvec(sm.gr, q, g);
          double* r = &sm.rhs[jt[q]][3 * jl[q]];
#pragma unroll
          for (int x = 0; x < 3; ++x) r[x] = -(pj[q][3 * x] * g[0] + pj[q][3 * x + 1] * g[1] + pj[q][3 * x + 2] * g[2]);
        }
      fsync<NT>();
      lsolve();
#pragma unroll
      for (int q = 0; q < IPM_FPL; ++q)
        if (own[q]) {
          double d[3];
          fvec(sm.dU, q, d);
          double* u = &sm.U[jt[q]][3 * jl[q]];
          u[0] += d[0];
          u[1] += d[1];
          u[2] += d[2];
        }
      fsync<NT>();
    }
    gradient();
    double stat = 0.0, smin = INFINITY, lminw = INFINITY;
#ifdef MPCQP_IPM_DEBUG
    double dbg_code = 0.0, dbg_r = 0.0;
#endif
#pragma unroll
    for (int q = 0; q < IPM_FPL; ++q) {
      if (!own[q]) continue;
      double g[3], f[3];
      fvec(sm.gr, q, g);
      fvec(sm.U, q, f);
#pragma unroll
      for (int x = 0; x < 3; ++x)
        stat = fmax(stat, fabs(pj[q][3 * x] * g[0] + pj[q][3 * x + 1] * g[1] + pj[q][3 * x + 2] * g[2]));
      int viol = 0;
#pragma unroll
      for (int r = 0; r < 6; ++r)
        if (live(r)) {
          const double sl = adot(r, f) - hrow(q, r);
          smin = fmin(smin, sl);
          if (sl < -tol_h) viol |= 1 << r;
        }
      // multipliers: g = sum lambda_r a_r over an independent subset of the active rows
      const int am = act[q] & (implied ? 0x2F : 0x3F);
      const int nq = (int)nq_of[q];
      double best = nq == 0 ? INFINITY : -INFINITY;
      int drop = -1;
#ifdef MPCQP_IPM_DEBUG
      double dbg_res = INFINITY;
      int dbg_ndet = 0;
#endif
      if (nq > 0) {
        double rw[6][3];
#pragma unroll
        for (int r = 0; r < 6; ++r)
#pragma unroll
          for (int x = 0; x < 3; ++x) rw[r][x] = arow(r, x);
        ipm_cone_multipliers(rw, am, nq, g, tol_g, best, drop);
      }
#ifdef MPCQP_IPM_DEBUG
      if (best == -INFINITY && dbg_code == 0.0) {
        dbg_code = am * 1000 + nq * 100 + dbg_ndet + 0.5;
        dbg_r = fmax(fabs(g[0]), fmax(fabs(g[1]), fabs(g[2])));
      }
#endif
      lminw = fmin(lminw, best);
      act[q] = (act[q] | viol) & ~(drop >= 0 ? (1 << drop) : 0);
    }
    stat = wave_max_all(stat);
    smin = wave_min_all(smin);
    lminw = wave_min_all(lminw);
#ifdef MPCQP_IPM_DEBUG
    dbg_p[0] = stat / gscale;
    dbg_p[1] = smin;
    dbg_p[2] = lminw;
    dbg_p[3] = wave_max_all(dbg_code);
    dbg_p[4] = wave_max_all(dbg_code > 0.0 ? dbg_r : 0.0);
#endif
    return stat < IPM_STAT_TOL * gscale && smin > -tol_h && lminw > -tol_g;
  };

  // ------------------------------------------------ interior point
  int it = 0;
  bool done = false;
  while (!done && it < IPM_MAX_IT) {
    ++it;
    gradient();
    double rd[IPM_FPL][3], rp[IPM_FPL][6];
    double sl = 0.0;
#pragma unroll
    for (int q = 0; q < IPM_FPL; ++q) {
      double g[3], f[3];
      fvec(sm.gr, q, g);
      fvec(sm.U, q, f);
#pragma unroll
      for (int x = 0; x < 3; ++x) {
        double v = g[x];
#pragma unroll
        for (int r = 0; r < 6; ++r) v = fma(-lam[q][r], arow(r, x), v);
        rd[q][x] = own[q] ? v : 0.0;
      }
#pragma unroll
      for (int r = 0; r < 6; ++r) {
        const bool on = own[q] && live(r);
        rp[q][r] = on ? adot(r, f) - hrow(q, r) - s[q][r] : 0.0;
        sl += on ? s[q][r] * lam[q][r] : 0.0;
      }
    }
    const double mu = sgpr_d(wave_sum_d(sl)) / m_tot;
#ifdef MPCQP_IPM_DEBUG
    {
      double rdm = 0.0, rpm = 0.0;
#pragma unroll
      for (int q = 0; q < IPM_FPL; ++q) {
#pragma unroll
        for (int x = 0; x < 3; ++x) rdm = fmax(rdm, fabs(rd[q][x]));
#pragma unroll
        for (int r = 0; r < 6; ++r) rpm = fmax(rpm, fabs(rp[q][r]));
      }
      rdm = wave_max_all(rdm);
      rpm = wave_max_all(rpm);
      dbg((double)it);
      dbg(mu);
      dbg(rdm);
      dbg(rpm);
      dbg(dbg_p[0]);
      dbg(dbg_p[1]);
      dbg(dbg_p[2]);
      dbg(dbg_p[3]);
      dbg(dbg_p[4]);
    }
#endif
    if (mu < IPM_POLISH_MU * gscale * hscale) {
#pragma unroll
      for (int q = 0; q < IPM_FPL; ++q) {
        act[q] = 0;
#pragma unroll
        for (int r = 0; r < 6; ++r)
          if (own[q] && live(r) && lam[q][r] > s[q][r]) act[q] |= 1 << r;
      }
      // U is overwritten by the polish: keep the IPM iterate
      for (int e = lane; e < N * NU; e += NT) sm.Us[e / NU][e % NU] = sm.U[e / NU][e % NU];
      fsync<NT>();
      for (int corr = 0; corr <= IPM_NCORR; ++corr) {
        int before[IPM_FPL];
#pragma unroll
        for (int q = 0; q < IPM_FPL; ++q) before[q] = act[q];
        if (polish()) {
          done = true;
          status = MPCQP_STATUS_OK;
          break;
        }
        int same = 1;
#pragma unroll
        for (int q = 0; q < IPM_FPL; ++q) same &= before[q] == act[q];
        if (__all(same)) break;
      }
      if (done) break;
      for (int e = lane; e < N * NU; e += NT) sm.U[e / NU][e % NU] = sm.Us[e / NU][e % NU];
      fsync<NT>();
    }
    double D[IPM_FPL][6];
#pragma unroll
    for (int q = 0; q < IPM_FPL; ++q) {
#pragma unroll
      for (int r = 0; r < 6; ++r) D[q][r] = own[q] && live(r) ? lam[q][r] / s[q][r] : 0.0;
      if (own[q]) set_w_ipm(q, D[q]);
    }
    fsync<NT>();
    factor();
    ++nfact;
    // Newton direction for the complementarity target rc (per row); ds, dl out
    double ds[IPM_FPL][6], dl[IPM_FPL][6];
    auto newton = [&](const double (&rc)[IPM_FPL][6]) {
      for (int e = lane; e < N * NU; e += NT) sm.rhs[e / NU][e % NU] = 0.0;
      fsync<NT>();
#pragma unroll
      for (int q = 0; q < IPM_FPL; ++q)
        if (own[q]) {
          double* rr = &sm.rhs[jt[q]][3 * jl[q]];
#pragma unroll
          for (int x = 0; x < 3; ++x) {
            double v = -rd[q][x];
#pragma unroll
            for (int r = 0; r < 6; ++r)
              if (live(r)) v = fma(arow(r, x), rc[q][r] / s[q][r] - D[q][r] * rp[q][r], v);
            rr[x] = v;
          }
        }
      fsync<NT>();
      lsolve();
#pragma unroll
      for (int q = 0; q < IPM_FPL; ++q) {
        double d[3];
        fvec(sm.dU, q, d);
#pragma unroll
        for (int r = 0; r < 6; ++r) {
          const bool on = own[q] && live(r);
          ds[q][r] = on ? adot(r, d) + rp[q][r] : 0.0;
          dl[q][r] = on ? (rc[q][r] - lam[q][r] * ds[q][r]) / s[q][r] : 0.0;
        }
      }
    };
    auto max_steps = [&](double& ap, double& ad) {
      double a1 = 1.0, a2 = 1.0;
#pragma unroll
      for (int q = 0; q < IPM_FPL; ++q)
#pragma unroll
        for (int r = 0; r < 6; ++r) {
          if (ds[q][r] < 0.0) a1 = fmin(a1, -s[q][r] / ds[q][r]);
          if (dl[q][r] < 0.0) a2 = fmin(a2, -lam[q][r] / dl[q][r]);
        }
      ap = sgpr_d(wave_min_all(a1));
      ad = sgpr_d(wave_min_all(a2));
    };
    double rc[IPM_FPL][6];
#pragma unroll
    for (int q = 0; q < IPM_FPL; ++q)
#pragma unroll
      for (int r = 0; r < 6; ++r) rc[q][r] = -s[q][r] * lam[q][r];
    newton(rc);
    double ap, ad;
    max_steps(ap, ad);
    double sa = 0.0;
#pragma unroll
    for (int q = 0; q < IPM_FPL; ++q)
#pragma unroll
      for (int r = 0; r < 6; ++r)
        if (own[q] && live(r)) sa += (s[q][r] + ap * ds[q][r]) * (lam[q][r] + ad * dl[q][r]);
    const double mu_aff = sgpr_d(wave_sum_d(sa)) / m_tot;
    const double sig = mu_aff / mu;
    const double target = fmax(sig * sig * sig * mu, IPM_MU_FLOOR * gscale * hscale);
#pragma unroll
    for (int q = 0; q < IPM_FPL; ++q)
#pragma unroll
      for (int r = 0; r < 6; ++r) rc[q][r] = -s[q][r] * lam[q][r] - ds[q][r] * dl[q][r] + target;
    newton(rc);
    max_steps(ap, ad);
    ap = fmin(1.0, IPM_TAU * ap);
    ad = fmin(1.0, IPM_TAU * ad);
#pragma unroll
    for (int q = 0; q < IPM_FPL; ++q) {
      if (own[q]) {
        double d[3];
        fvec(sm.dU, q, d);
        double* u = &sm.U[jt[q]][3 * jl[q]];
        u[0] += ap * d[0];
        u[1] += ap * d[1];
        u[2] += ap * d[2];
      }
#pragma unroll
      for (int r = 0; r < 6; ++r)
        if (own[q] && live(r)) {
          s[q][r] += ap * ds[q][r];
          lam[q][r] += ad * dl[q][r];
        }
    }
    fsync<NT>();
  }

  // ------------------------------------------------ output (U: the polished optimum or the last iterate)
  bool finite = true;
  for (int e = lane; e < N * NU; e += NT) finite &= isfinite(sm.U[e / NU][e % NU]);
  if (__any(!finite)) status = MPCQP_STATUS_NONFINITE;
  if (lane < 12) u0g[(size_t)b * 12 + lane] = (float)sm.U[0][lane];
#ifdef MPCQP_IPM_DEBUG
  Ug = nullptr;
#endif
  if (Ug)
    for (int e = lane; e < N * NU; e += NT) Ug[(size_t)b * N * NU + e] = (float)sm.U[e / NU][e % NU];
  if (lane == 0) {
    if (statusg) statusg[b] = status;
    if (itersg) itersg[b] = nfact;
  }
}
