// mpcqp_form.h -- per-robot QP formulation shared by both capacity classes
// (included by mpcqp.hip inside its anonymous namespace).
//
// Restates ModelPredictiveController._solve_mpc's formulation (mpc.py:173-260)
// for one robot with NT threads, in closed form:
//
//   * model (mpc.py:173-192): R_z, I_w = R_z I_B R_z^T, inv(I_w), inv(I_w)[r]x
//     and I/m with the reference's float32 rounding; everything after is float64.
//   * discretisation (mpc.py:194-208): M = [[A_c, B_c], [0, 0]] has M^3 = 0, so
//     A_d = I + A_c h + A_c^2 h^2/2 and B_d = B_c h + A_c B_c h^2/2 exactly.  With
//     K = inv(I_w)[r]x (3x12), G = R_z^T K and S = [I I I I]:
//        X0 = B_d     = [G h^2/2 ; S h^2/(2m) ; K h ; S h/m ; 0]
//        X1 = Nm X0   = [G h^2   ; S h^2/m    ; 0   ; 0     ; 0]   (Nm = A_d - I)
//        Nm X1 = 0, so the horizon blocks are A^k B_d = X0 + k X1.
//   * condensing (mpc.py:211-233): with diagonal Q, X0^T Q X1 = 2 Ya and
//     X1^T Q X1 = 4 Ya, X0^T Q X0 = Ya + Yb, where
//        Ya = h^4/4 (G^T Q_th G + S^T Q_p S / m^2),  Yb = h^2 (K^T Q_w K + S^T Q_v S / m^2),
//     so block (ja, jb) of H = 2(Su^T Qbar Su + Rbar) is
//        2 [ m Yb + Ta Ya ] (+ 2R on the diagonal),  m = N - max(ja, jb),
//        Ta = sum_{t >= max} (1 + 2(t - ja))(1 + 2(t - jb)) = m(4m^2 - 1)/3 + 2|ja - jb| m^2,
//     and g = 2 Su^T Qbar (Sx x0 - Xref) reduces to suffix sums over the horizon of
//     Q e_t and t Q e_t, e_t = A^{t+1} x0 - xref_t = x0 + (t+1) n1 + C(t+1, 2) n2 - xref_t
//     with n1 = Nm x0, n2 = Nm^2 x0 = h^2 x0[12] e_5.
//   * full (non-diagonal) Q / R (mpc.py:49-52 builds kron(I_N, Q) from any matrix): with
//     Y00 = X0^T Q X0, Y01 = X0^T Q X1, Y11 = X1^T Q X1 the block is
//        2 [ m Y00 + Sb Y01 + Sa Y01^T + T Y11 ] (+ 2 R on the same-step blocks),
//     Sa = sum_t (t - ja), Sb = sum_t (t - jb), T = sum_t (t - ja)(t - jb) over t = max..N-1
//     (exact integers); g keeps its form with E0 / E1 = Q times the suffix sums of e_t, t e_t.
//     The diagonal case (Y00 = Ya + Yb, Y01 = 2 Ya, Y11 = 4 Ya) keeps the two-term path.
//   * friction cone (mpc.py:237-260): 6 one-sided rows per stance foot-step
//     (4 pyramid rows, fz >= 0, fz <= contact * fz_max), generalised to a per-robot
//     surface normal (normal = e_z reproduces mpc.py:239-245 exactly).
// Swing foot-steps are eliminated exactly (their GRFs are 0: ub gives fz <= 0 and
// the cone gives mu fz >= |fx|, |fy| >= 0), leaving n = 3 * #stance variables.

// Transient formulation scratch (dead once H and g are built), sized for horizons N <= NM
// (the dense classes: kDenseN; the interior-point class: its own stage count)
template <int NM>
struct alignas(16) FormT {
  static constexpr int IN_XREF = IN_CONTACT + 4 * NM, IN_END = IN_XREF + NX * NM;
  float in[IN_END];              // staged inputs (x0, feet, robot record, contact, xref)
  double K[3][NU];               // inv(I_w)[r_leg]x, float32-rounded (B_c rows 6:9)
  double G[3][NU];               // R_z^T K                            (A_c B_c rows 0:3)
  double E0[NM][16];             // sum_{t >= j} q_s e_t[s]
  double E1[NM][8];              // sum_{t >= j} t q_s e_t[s]  (s < 6)
  double ii[9];                  // 3x3 work (world inertia, its inverse)
  double rz[2];                  // float32(cos yaw), float32(sin yaw)
  double minv;                   // float32(1/m)
  double q[16];                  // state weights (staged: indexed per lane below)
  // full Q only (KParams::wfull): Q, the raw suffix sums of e_t and t e_t, X0 / X1 and Q X0 / Q X1
  double qf[NX * NX];
  double es[2][NM][NX];
  double X[2][NX][NU];
  double QX[2][NX][NU];
};
using Form = FormT<kDenseN>;

// Hessian blocks {Ya, Yb}[c1][c2]: kept for the whole solve (H entries are
// re-derived from it when a constraint is dropped)
struct alignas(16) FormY {
  d2 Y[NU * NU];
  double rd2[NU];   // 2 R_ii (input weights; kernel arguments indexed per lane would be memory loads)
  // full Q / R only: Y00, Y01, Y11 and 2 R (12 x 12, row-major)
  double Yf[3][NU * NU];
  double rf2[NU * NU];
};

// Per-robot data every class keeps for the solve (horizons N <= NM).
template <int NM>
struct alignas(16) RobotMetaT {
  double rows[6][3];             // one-sided cone rows a_r (a_r . f >= b_r)
  double ub[4 * NM];             // contact * fz_max per stance foot-step (mpc.py:257)
  int foot_t[4 * NM];            // stance foot-step -> horizon step
  int foot_leg[4 * NM];          // stance foot-step -> leg
  int stance_of[4 * NM];         // (step, leg) -> stance foot-step or -1
  int S;
  int fz0_implied;               // mu > 0: the n.f >= 0 row is the half-sum of rows 0 and 1
};
using RobotMeta = RobotMetaT<kDenseN>;

template <int NT>
__device__ __forceinline__ void fsync() {
  if constexpr (NT == LANES) {
    // one wave: the LDS executes a wave's DS instructions in issue order
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
    __builtin_amdgcn_wave_barrier();
  } else {
    __syncthreads();
  }
}

template <int NT>
__device__ __forceinline__ bool fany(bool v) {
  if constexpr (NT == LANES) return __any(v);
  else return __syncthreads_or(v) != 0;
}

// Stage the robot's inputs in LDS; false if any is non-finite (status NONFINITE).
template <int NT, class F>
__device__ __forceinline__ bool form_stage(F& f, int N, int b, int tid, const float* __restrict__ x0g,
                                           const float* __restrict__ xrefg, const float* __restrict__ contactg,
                                           const float* __restrict__ feetg, const float* __restrict__ robotg) {
  // The robot's five input slices, staged into LDS with 16-byte loads: each slice is
  // covered by the 16-byte-aligned chunks that hold it (a chunk never crosses a page,
  // so the few bytes of the neighbouring robots it also holds are always readable),
  // and a lane stores the chunk's floats that fall inside the slice.
  float* const in = f.in;
  // slices: x0, feet, robot record, contact, xref (no runtime-indexed private
  // arrays below: those would live in scratch)
  const float* const p0 = x0g + (size_t)b * NX;
  const float* const p1 = feetg + (size_t)b * 12;
  const float* const p2 = robotg + (size_t)b * MPCQP_ROBOT_STRIDE;
  const float* const p3 = contactg + (size_t)b * N * 4;
  const float* const p4 = xrefg + (size_t)b * N * NX;
  auto nchunks = [](const float* q, int len) -> int {
    const uintptr_t a = (uintptr_t)q;
    return (int)(((a + 4 * (uintptr_t)len + 15) >> 4) - (a >> 4));
  };
  const int c1 = nchunks(p0, NX), c2 = c1 + nchunks(p1, 12), c3 = c2 + nchunks(p2, MPCQP_ROBOT_STRIDE),
            c4 = c3 + nchunks(p3, 4 * N), c5 = c4 + nchunks(p4, NX * N);
  int bad = 0;
  for (int c = tid; c < c5; c += NT) {
    const int i = (c >= c1) + (c >= c2) + (c >= c3) + (c >= c4);
    const float* const q = i == 0 ? p0 : i == 1 ? p1 : i == 2 ? p2 : i == 3 ? p3 : p4;
    const int cb = i == 0 ? 0 : i == 1 ? c1 : i == 2 ? c2 : i == 3 ? c3 : c4;
    const int len = i == 0 ? NX : i == 1 ? 12 : i == 2 ? 12 : i == 3 ? 4 * N : NX * N;   // robot: 12 fields read
    const int dst = i == 0 ? IN_X0 : i == 1 ? IN_FEET : i == 2 ? IN_ROBOT : i == 3 ? IN_CONTACT : F::IN_XREF;
    const uintptr_t base = ((uintptr_t)q & ~(uintptr_t)15) + 16 * (uintptr_t)(c - cb);
    const float4 v = *reinterpret_cast<const float4*>(base);
    const int e = (int)(((intptr_t)base - (intptr_t)q) >> 2);   // slice index of v.x (may be < 0)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const float w = j == 0 ? v.x : j == 1 ? v.y : j == 2 ? v.z : v.w;
      const int k = e + j;
      if (k >= 0 && k < len) {
        in[dst + k] = w;
        bad |= i != 3 && !isfinite(w);   // contact is not checked
      }
    }
  }
  return !fany<NT>(bad != 0);
}

// Stance list from the gait table (one wave: lanes cover 4N <= 128 entries).
// Returns S (wave-uniform).  Writes meta.{foot_t, foot_leg, ub, stance_of, S}.
template <class F, class MT>
__device__ __forceinline__ int form_stance(const F& f, MT& mt, int N, int lane) {
  const unsigned long long lt_mask = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
  const int nk = 4 * N;
  const float c0 = lane < nk ? f.in[IN_CONTACT + lane] : 0.f;
  const float c1 = lane + LANES < nk ? f.in[IN_CONTACT + lane + LANES] : 0.f;
  const bool f0 = c0 > 0.f, f1 = c1 > 0.f;   // contact > 0: stance (ub = contact * fz_max > 0)
  const unsigned long long m0 = __ballot(f0), m1 = __ballot(f1);
  const int S0 = __popcll(m0);
  const int S = uni(S0 + __popcll(m1));
  const int i0 = __popcll(m0 & lt_mask), i1 = S0 + __popcll(m1 & lt_mask);
  const double fzmax = (double)f.in[IN_ROBOT + 8];
  if (lane < nk) mt.stance_of[lane] = f0 ? i0 : -1;
  if (lane + LANES < nk) mt.stance_of[lane + LANES] = f1 ? i1 : -1;
  if (f0) {
    mt.foot_t[i0] = lane / 4;
    mt.foot_leg[i0] = lane % 4;
    mt.ub[i0] = (double)c0 * fzmax;
  }
  if (f1) {
    mt.foot_t[i1] = (lane + LANES) / 4;
    mt.foot_leg[i1] = (lane + LANES) % 4;
    mt.ub[i1] = (double)c1 * fzmax;
  }
  if (lane == 0) mt.S = S;
  return S;
}

// e_t's state component sc at horizon step t (0-based: e_t = A^{t+1} x0 - xref_t)
template <class F>
__device__ __forceinline__ double form_e(const F& f, int sc, int t, double h) {
  const float* xin = f.in + IN_X0;
  auto rz = [&](int a, int bb) -> double {
    return a == 2 ? (bb == 2 ? 1.0 : 0.0) : (bb == 2 ? 0.0 : (a == bb ? f.rz[0] : (a == 0 ? -f.rz[1] : f.rz[1])));
  };
  double x0s = (double)xin[sc], n1 = 0.0, n2 = 0.0;
  const double g12 = (double)xin[12];
  if (sc < 3) n1 = h * (rz(0, sc) * (double)xin[6] + rz(1, sc) * (double)xin[7] + rz(2, sc) * (double)xin[8]);
  else if (sc < 6) n1 = h * (double)xin[6 + sc] + (sc == 5 ? 0.5 * h * h * g12 : 0.0);
  else if (sc == 11) n1 = h * g12;
  if (sc == 5) n2 = h * h * g12;
  const double k = (double)(t + 1);
  return x0s + k * n1 + 0.5 * k * (k - 1.0) * n2 - (double)f.in[F::IN_XREF + t * NX + sc];
}

// Full (non-diagonal) Q / R (KParams::wfull): E0 / E1 = Q times the suffix sums of e_t and
// t e_t, and the closed-form blocks Y00 = X0^T Q X0, Y01 = X0^T Q X1, Y11 = X1^T Q X1 with X0
// = B_d, X1 = Nm B_d written out (K, G, minv are in LDS: called after their barrier).
template <int NT, class F>
__device__ __forceinline__ void form_model_full(const KParams& P, F& f, FormY& fy, int N, int tid) {
  const double h = P.dt;
  fsync<NT>();   // K, G (written just before by threads < 36) are read below
  for (int e = tid; e < NX * NX; e += NT) f.qf[e] = P.wfull[e];
  for (int e = tid; e < NU * NU; e += NT) fy.rf2[e] = 2.0 * P.wfull[NX * NX + e];
  // X0 (rows: G h^2/2, S h^2/(2m), K h, S h/m, 0) and X1 = Nm X0 (G h^2, S h^2/m, 0, 0, 0)
  for (int e = tid; e < NX * NU; e += NT) {
    const int i = e / NU, c = e % NU;
    double x0v = 0.0, x1v = 0.0;
    if (i < 3) {
      x0v = f.G[i][c] * (0.5 * h * h);
      x1v = f.G[i][c] * (h * h);
    } else if (i < 6) {
      const double on = (c % 3 == i - 3) ? f.minv : 0.0;
      x0v = on * (0.5 * h * h);
      x1v = on * (h * h);
    } else if (i < 9) {
      x0v = f.K[i - 6][c] * h;
    } else if (i < 12) {
      x0v = (c % 3 == i - 9) ? f.minv * h : 0.0;
    }
    f.X[0][i][c] = x0v;
    f.X[1][i][c] = x1v;
  }
  // raw suffix sums of e_t and t e_t, thread = state component
  if (tid < NX) {
    double s0 = 0.0, s1 = 0.0;
    for (int t = N - 1; t >= 0; --t) {
      const double e = form_e(f, tid, t, h);
      s0 += e;
      s1 = fma((double)t, e, s1);
      f.es[0][t][tid] = s0;
      f.es[1][t][tid] = s1;
    }
  }
  fsync<NT>();
  for (int e = tid; e < 2 * NX * NU; e += NT) {   // Q X0, Q X1
    const int w = e / (NX * NU), i = (e / NU) % NX, c = e % NU;
    double a = 0.0;
#pragma unroll
    for (int j = 0; j < NX; ++j) a = fma(f.qf[i * NX + j], f.X[w][j][c], a);
    f.QX[w][i][c] = a;
  }
  for (int e = tid; e < N * NX; e += NT) {   // E0 = Q es0, E1 = Q es1 (components < 6)
    const int t = e / NX, sc = e % NX;
    double a0 = 0.0, a1 = 0.0;
#pragma unroll
    for (int j = 0; j < NX; ++j) {
      a0 = fma(f.qf[sc * NX + j], f.es[0][t][j], a0);
      a1 = fma(f.qf[sc * NX + j], f.es[1][t][j], a1);
    }
    f.E0[t][sc] = a0;
    if (sc < 6) f.E1[t][sc] = a1;
  }
  fsync<NT>();
  for (int e = tid; e < 3 * NU * NU; e += NT) {   // Y00 = X0^T Q X0, Y01 = X0^T Q X1, Y11 = X1^T Q X1
    const int w = e / (NU * NU), c1 = (e / NU) % NU, c2 = e % NU;
    const int xa = w == 2 ? 1 : 0, qb = w == 0 ? 0 : 1;
    double a = 0.0;
#pragma unroll
    for (int i = 0; i < NX; ++i) a = fma(f.X[xa][i][c1], f.QX[qb][i][c2], a);
    fy.Yf[w][c1 * NU + c2] = a;
  }
}

// Model (float32-faithful), cone rows, Ya/Yb, horizon suffix sums.  All NT threads.
template <int NT, class F, class MT>
__device__ __forceinline__ void form_model(const KParams& P, F& f, FormY& fy, MT& mt, int N, int tid) {
  const float* const rbs = f.in + IN_ROBOT;
  const double h = P.dt;
  // ---- R_z, I_w = float32(float32(R_z I_B) R_z^T), inverse (mpc.py:178-182)
  const double yaw = (double)f.in[IN_X0 + 2];
  const double c = f32r(cos(yaw)), s = f32r(sin(yaw));
  auto rz = [&](int a, int bb) -> double {   // R_z[a][bb] (kinematics rot_z, float32 entries)
    return a == 2 ? (bb == 2 ? 1.0 : 0.0) : (bb == 2 ? 0.0 : (a == bb ? c : (a == 0 ? -s : s)));
  };
  {
    const int i = tid / 3, j = tid % 3;
    auto ib = [&](int a, int bb) -> double {
      const int lo = a < bb ? a : bb, hi = a < bb ? bb : a;
      const int idx = lo == 0 ? hi : (lo == 1 ? 2 + hi : 5);   // ixx ixy ixz iyy iyz izz
      return (double)rbs[1 + idx];
    };
    if (tid < 9) f.ii[tid] = f32r(rz(i, 0) * ib(0, j) + rz(i, 1) * ib(1, j) + rz(i, 2) * ib(2, j));
    if (tid < NX) f.q[tid] = P.q[tid];
    if (tid == 0) {
      f.rz[0] = c;
      f.rz[1] = s;
      f.minv = f32r(1.0 / (double)rbs[0]);   // I / m in float32 (mpc.py:190)
    }
    fsync<NT>();
    double iw = 0.0;
    if (tid < 9) iw = f32r(f.ii[3 * i] * rz(j, 0) + f.ii[3 * i + 1] * rz(j, 1) + f.ii[3 * i + 2] * rz(j, 2));
    fsync<NT>();
    if (tid < 9) f.ii[tid] = iw;
    fsync<NT>();
    if (tid < 9) {   // 3x3 inverse by adjugate (float64), stored float32 like np.linalg.inv
      const double* I = f.ii;
      const int r1 = (j + 1) % 3, r2 = (j + 2) % 3, c1 = (i + 1) % 3, c2 = (i + 2) % 3;
      const double cof = I[r1 * 3 + c1] * I[r2 * 3 + c2] - I[r1 * 3 + c2] * I[r2 * 3 + c1];   // adj(I)[i][j]
      const double det = I[0] * (I[4] * I[8] - I[5] * I[7]) - I[1] * (I[3] * I[8] - I[5] * I[6]) +
                         I[2] * (I[3] * I[7] - I[4] * I[6]);
      iw = f32r(cof / det);
    }
    fsync<NT>();
    if (tid < 9) f.ii[tid] = iw;
  }
  // ---- friction-cone rows in the (t1, t2, n) frame (mpc.py:239-245 for n = e_z)
  if (tid >= 64 - 18 && tid < 64) {
    const int k18 = tid - (64 - 18);
    double nx = rbs[9], ny = rbs[10], nz = rbs[11];
    const double nn = sqrt(nx * nx + ny * ny + nz * nz);
    if (!(nn > 0.0)) {
      nx = 0.0; ny = 0.0; nz = 1.0;
    } else {
      nx /= nn; ny /= nn; nz /= nn;
    }
    double t1x = 1.0 - nx * nx, t1y = -nx * ny, t1z = -nx * nz;
    const double tn = sqrt(t1x * t1x + t1y * t1y + t1z * t1z);
    t1x /= tn; t1y /= tn; t1z /= tn;
    const double t2x = ny * t1z - nz * t1y, t2y = nz * t1x - nx * t1z, t2z = nx * t1y - ny * t1x;
    const double mu = rbs[7];
    const int rr = k18 / 3, k = k18 % 3;
    const double nk = k == 0 ? nx : (k == 1 ? ny : nz);
    const double t1k = k == 0 ? t1x : (k == 1 ? t1y : t1z);
    const double t2k = k == 0 ? t2x : (k == 1 ? t2y : t2z);
    const double val = rr == 0 ? t1k + mu * nk
                     : rr == 1 ? -t1k + mu * nk
                     : rr == 2 ? t2k + mu * nk
                     : rr == 3 ? -t2k + mu * nk
                     : rr == 4 ? nk : -nk;
    mt.rows[rr][k] = val;
    if (k18 == 0) mt.fz0_implied = mu > 0.0;
  }
  fsync<NT>();
  // ---- K = float32(inv(I_w) [r]x) (mpc.py:188-189) and G = R_z^T K; thread (i, col)
  if (tid < 36) {
    const int i = tid / NU, col = tid % NU, leg = col / 3, j = col % 3;
    const float* fb = f.in + IN_FEET;
    const double rx = fb[3 * leg], ry = fb[3 * leg + 1], rzz = fb[3 * leg + 2];
    const double sk0 = (j == 0) ? 0.0 : (j == 1 ? -rzz : ry);   // column j of [r]x
    const double sk1 = (j == 0) ? rzz : (j == 1 ? 0.0 : -rx);
    const double sk2 = (j == 0) ? -ry : (j == 1 ? rx : 0.0);
    double kk[3];
#pragma unroll
    for (int a = 0; a < 3; ++a) kk[a] = f32r(f.ii[3 * a] * sk0 + f.ii[3 * a + 1] * sk1 + f.ii[3 * a + 2] * sk2);
    f.K[i][col] = kk[i];
    f.G[i][col] = rz(0, i) * kk[0] + rz(1, i) * kk[1] + rz(2, i) * kk[2];
  }
  // ---- horizon suffix sums of Q e_t and t Q e_t; thread s (state component)
  if (tid < NU) fy.rd2[tid] = 2.0 * P.r[tid];
  if (P.wfull) {
    form_model_full<NT>(P, f, fy, N, tid);
    return;
  }
  if (tid >= 64 - 16 && tid < 64 - 16 + NX) {
    const int sc = tid - (64 - 16);
    const float* xin = f.in + IN_X0;
    const double q = f.q[sc];
    // n1 = Nm x0, n2 = Nm^2 x0 (closed form of the 13x13 products)
    double x0s = (double)xin[sc], n1 = 0.0, n2 = 0.0;
    const double g12 = (double)xin[12];
    if (sc < 3) n1 = h * (rz(0, sc) * (double)xin[6] + rz(1, sc) * (double)xin[7] + rz(2, sc) * (double)xin[8]);
    else if (sc < 6) n1 = h * (double)xin[6 + sc] + (sc == 5 ? 0.5 * h * h * g12 : 0.0);
    else if (sc == 11) n1 = h * g12;
    if (sc == 5) n2 = h * h * g12;
    double e0 = 0.0, e1 = 0.0;
    for (int t = N - 1; t >= 0; --t) {
      const double k = (double)(t + 1);
      const double e = x0s + k * n1 + 0.5 * k * (k - 1.0) * n2 - (double)f.in[F::IN_XREF + t * NX + sc];
      e0 = fma(q, e, e0);
      e1 = fma((double)t * q, e, e1);
      f.E0[t][sc] = e0;
      if (sc < 6) f.E1[t][sc] = e1;
    }
  }
  fsync<NT>();
  // ---- Ya, Yb (12 x 12 each)
  {
    const double minv2 = f.minv * f.minv;
    const double ca = 0.25 * h * h * h * h, cb = h * h;
    for (int k = tid; k < NU * NU; k += NT) {
      const int c1 = k / NU, c2 = k % NU;
      double ya = 0.0, yb = 0.0;
#pragma unroll
      for (int i = 0; i < 3; ++i) {
        ya = fma(f.G[i][c1] * f.q[i], f.G[i][c2], ya);
        yb = fma(f.K[i][c1] * f.q[6 + i], f.K[i][c2], yb);
      }
      if (c1 % 3 == c2 % 3) {
        ya = fma(f.q[3 + c1 % 3], minv2, ya);
        yb = fma(f.q[9 + c1 % 3], minv2, yb);
      }
      fy.Y[k] = d2{ca * ya, cb * yb};
    }
  }
}

// g[a] for the stance variable a < n held by this thread (mpc.py:233)
template <class F, class MT>
__device__ __forceinline__ double form_g(const KParams& P, const F& f, const MT& mt, int a) {
  const double h = P.dt;
  const int sf = a / 3, ax = a % 3;
  const int j = mt.foot_t[sf], cc = 3 * mt.foot_leg[sf] + ax;
  const double* E0 = f.E0[j];
  const double* E1 = f.E1[j];
  const double al0 = f.G[0][cc] * E0[0] + f.G[1][cc] * E0[1] + f.G[2][cc] * E0[2] + E0[3 + ax] * f.minv;
  const double al1 = f.G[0][cc] * E1[0] + f.G[1][cc] * E1[1] + f.G[2][cc] * E1[2] + E1[3 + ax] * f.minv;
  const double be0 = f.K[0][cc] * E0[6] + f.K[1][cc] * E0[7] + f.K[2][cc] * E0[8] + E0[9 + ax] * f.minv;
  return 2.0 * (0.5 * h * h * ((double)(1 - 2 * j) * al0 + 2.0 * al1) + h * be0);
}

// H[a][b] for full Q / R (header comment), the same-step R block included
__device__ __forceinline__ double form_h_full(const FormY& fy, int N, int ja, int ca, int jb, int cb) {
  const int mx = ja > jb ? ja : jb;
  const int m = N - mx, da = mx - ja, db = mx - jb;   // N <= 20: every product fits an int
  const int s1 = (m * (m - 1)) >> 1;
  const double sa = (double)(s1 + m * da), sb = (double)(s1 + m * db);
  const double tt = (double)(((m - 1) * m * (2 * m - 1)) / 6 + (da + db) * s1 + m * da * db);
  double v = (double)m * fy.Yf[0][ca * NU + cb];
  v = fma(sb, fy.Yf[1][ca * NU + cb], v);
  v = fma(sa, fy.Yf[1][cb * NU + ca], v);
  v = fma(tt, fy.Yf[2][ca * NU + cb], v);
  const double rv = fy.rf2[ca * NU + cb];   // unconditional: a guarded load splits the block
  return fma(2.0, v, ja == jb ? rv : 0.0);
}

// H[a][b] from the foot-steps' horizon steps (ja, jb) and input columns (ca, cb)
// form_h with (Ta, m) of the step pair looked up (the same arithmetic, bitwise)
__device__ __forceinline__ double form_h_tab(const FormY& fy, d2 tm, int ca, int cb) {
  const d2 y = fy.Y[ca * NU + cb];
  return 2.0 * fma(tm[1], y[1], tm[0] * y[0]);
}
__device__ __forceinline__ double form_h(const FormY& fy, int N, int ja, int ca, int jb, int cb) {
  const int mx = ja > jb ? ja : jb;
  const int d = ja > jb ? ja - jb : jb - ja;
  const int m = N - mx;
  const int ta = (m * (4 * m * m - 1)) / 3 + 2 * d * m * m;   // exact integer
  const d2 y = fy.Y[ca * NU + cb];
  return 2.0 * fma((double)m, y[1], (double)ta * y[0]);
}
