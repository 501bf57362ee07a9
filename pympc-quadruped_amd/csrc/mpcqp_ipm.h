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
//     S_k = (I + P_{k+1} E_k)^-1 P_{k+1}, P_k = Qh + A^T S_k A -- evaluated on B_d's
//     6-dimensional range in the basis T = I - Nm / 2 (a 6-pivot Gauss-Jordan per stage,
//     factor() below).  (The textbook P - P B (R + B^T P B)^-1 B^T P loses ~4
//     digits: B_d has a 6-dimensional null space -- internal forces between feet --
//     where only Rh = 2e-5 acts.)  The constant gravity state x[12] never moves in a
//     Newton direction, so the recursions run on the 12-dimensional state.
//   * an active-set polish: once mu is small, the rows the last step moved towards
//     activity (Tapia's indicator lambda+ / lambda > s+ / s) define an
//     equality-constrained QP, solved exactly on each foot's null space (Gram-Schmidt
//     of its active rows; the same Riccati with B_leg W_j B_leg^T, W_j = P_j (P_j Rh P_j
//     + I - P_j)^-1 P_j) plus two Newton refinements, then verified: stationarity on
//     the null spaces, primal feasibility of every row and multipliers >= 0 (the
//     gradient in the cone of the foot's active rows, Caratheodory subsets).  A failed
//     check corrects the set (violated rows in, the most negative multiplier out) up
//     to IPM_NCORR times (IPM_NCORR_IPM from an interior-point iterate); the IPM continues
//     otherwise.
// A verified polish is the exact optimum (status OK); tools/ipm_proto.py is the NumPy
// model of every step (64 golden / synthetic cases, worst error 1.3e-6).

#include "mpcqp_ipm_foot.h"

constexpr int IPM_MAX_IT = 60;
constexpr int IPM_NCORR = 8;       // set corrections of a warm start's polish
// ... and of a polish from an interior-point iterate: a set that needs more is far off, and one
// more IPM iteration (one factorisation) costs less than the corrections (one each): round 6,
// tools/ipm_proto.py NCORR=2 -- the slowest standing robots 22 -> 16 factorisations, the
// golden / synthetic cases unchanged (mean 10.95, max 13)
constexpr int IPM_NCORR_IPM = 2;
constexpr int IPM_NREF = 2;
// fraction to the boundary (round 6: 0.995 -> 0.98 -- the slowest standing robots' long runs
// of short steps end sooner: fleet factorisations mean 10.86 -> 10.32, max 19 -> 15, 0.79 ->
// 0.935 M QP/s; 0.99 0.90 M, 0.97 0.93 M; tools/ipm_proto.py TAU: 64 cases all verified)
constexpr double IPM_TAU = 0.98;
// polish once mu < this * scale (tools/ipm_ab.sh: 1e-7 -> 3e-9 cut the slowest of 256 standing
// robots from 31 to 18 factorisations; round 6, with the Tapia polish set, 3e-9 -> 5e-10: a
// first polish that verifies more often, standing fleet 0.724 -> 0.753 M QP/s though the mean
// factorisations rise 10.64 -> 10.86; 1e-8 / 3e-8 slower, profiles/r6_ipm/polish_mu.txt)
constexpr double IPM_POLISH_MU = 5e-10;
constexpr double IPM_MU_FLOOR = 1e-13;
constexpr double IPM_STAT_TOL = 1e-10;
constexpr int IPM_FPL = 2;             // stance foot-steps per lane (4 kMaxN <= 128)

// per stance foot-step interior-point state (row slots 0..5)
template <int NF>
struct IpmFootLds {
  double fs[NF][6], fl[NF][6], frp[NF][6], frd[NF][4];
  union {
    struct {
      double fds[NF][6], fdl[NF][6];   // Newton directions of s and lambda
    };
    double fpj[NF][9];             // polish: null-space projector per foot-step
  };
  int fact[NF];                    // polish: active rows per foot-step
  int fprev[NF];                   // polish: the rows of the previous try
};
struct IpmFootNone {};
// the same for the one foot-step of a lane (registers)
struct IpmFootReg {
  double fs[6], fl[6], frp[6], frd[4], fds[6], fdl[6], fpj[9];
  int fact, fprev;
};

// LDS of one robot, sized for horizons N <= NM.  NM = 16 (the reference's default horizon):
// MG (throughput layout) 40 KB with diagonal weights -- four robots per CU, one wave per
// SIMD --, 43 KB with full ones (three); without MG (latency layout, M_k in LDS) 52 KB,
// three per CU; NM = 20 / 32 one robot per CU.  The Riccati S_k always live in a
// per-workgroup global scratch slot (read only by lsolve's batched phases); with MG at NM = 16
// the slot also holds M_k and its transpose (read row by row in lsolve's two recursions, the
// next stage's row loaded under the current stage's work) and the saved IPM iterate.  The
// formulation scratch shares its space with the per-stage temporaries (and M_k when it is
// in LDS), which are first written after it is dead.
struct IpmEmpty {};
template <int NM>
struct IpmMLds {
  alignas(16) double M[NM][144];   // M_k = A^T (I - S_k E_k): lsolve's stage maps (row-major)
};
template <int NM>
struct IpmUsLds {
  alignas(16) double Us[NM][NU];   // the IPM iterate while a polish overwrites U
};
struct IpmWFull {
  double qf[NX][NX];               // Qh = 2 Q (full)
  double rf[NU][NU];               // Rh = 2 R (leg blocks used)
};
template <int NM, bool FULL, bool MG>
struct alignas(16) IpmSharedT {
  static constexpr int IPM_NF = 4 * NM;
  static constexpr bool kMG = MG && NM <= 16;   // M_k, M_k^T and the saved iterate in the global slot
  union {
    struct {
      FormT<NM> f;
      FormY fy;
    } fa;                          // formulation scratch (dead once Bm / x0 / xr are copied)
    struct {
      [[no_unique_address]] std::conditional_t<kMG, IpmEmpty, IpmMLds<NM>> mk;
      union {
        struct {                       // gradient() temporaries
          alignas(16) double X[NM + 1][16];
          alignas(16) double BU[NM][NU];   // B_d U_k
          alignas(16) double nuh[NM][NU];  // adjoint nu_k (rows 0..11)
        };
        struct {                       // lsolve() temporaries
          alignas(16) double Y[NM][NU];
          alignas(16) double By[NM][NU];
          alignas(16) double la[NM][NU], lb[NM][NU], lc[NM][NU];   // per-stage vectors
          alignas(16) double ph[NM][NU];   // p_{k+1}, the backward recursion's input at stage k
          alignas(16) double dxh[NM][NU];  // dx_k
        };
      };
    };
  };
  RobotMetaT<NM> mt;
  alignas(16) double Bm[12][12];   // B_d rows 0..11 (row 12 is 0)
  alignas(16) double BmT[12][12];  // its transpose
  alignas(16) double TT[12][12];   // factor scratch: (I + P E)^T, then S_k^T
  double nmr[3][3];                // h R_z^T: A_d[r][6 + c] (r < 3)
  double x0[16];
  double xr[NM][NX];               // xref, float64
  double qh[16];                   // 2 q
  double rh[NU];                   // 2 r
  [[no_unique_address]] std::conditional_t<FULL, IpmWFull, IpmEmpty> wf;   // full weights only
  double W[IPM_NF][9];             // per stance foot-step 3x3 weight of the Newton system
  alignas(16) double QT[144];      // T^-T Qh T^-1, the factorisation's stage cost (12 x 12)
  alignas(16) double U[NM][NU];    // iterate (swing entries 0)
  alignas(16) double dU[NM][NU];
  alignas(16) double rhs[NM][NU];
  alignas(16) double gr[NM][NU];
  [[no_unique_address]] std::conditional_t<kMG, IpmEmpty, IpmUsLds<NM>> us;
  // per stance foot-step interior-point state in LDS when a lane owns more than one
  // foot-step (NM > 16); with at most 64 foot-steps each lane keeps its one in registers
  std::conditional_t<(IPM_NF > LANES), IpmFootLds<IPM_NF>, IpmFootNone> ft;
};
static_assert(sizeof(IpmSharedT<16, false, true>) <= 160 * 1024 / 4, "N <= 16, diagonal weights: four robots per CU");
static_assert(sizeof(IpmSharedT<16, true, true>) <= 160 * 1024 / 3, "N <= 16, full weights: three robots per CU");
static_assert(sizeof(IpmSharedT<16, true, false>) <= 160 * 1024 / 3, "N <= 16, M_k in LDS: three robots per CU");
// One robot's global slot (doubles): S_k, then -- used by the four-per-CU layout at NM = 16
// only -- M_k, M_k^T and the saved iterate.  A cross-leg R (XR) keeps its 12 x 12 stage weights
// W_k at offset W: the latency layouts it runs in hold M_k in LDS, so at NM = 16 they take M's
// place.  The stride depends on the stage count alone, so one pool per context (sized for its
// horizon) serves every layout.
template <int NM>
struct IpmSlot {
  static constexpr int M = NM * 144, MT = 2 * NM * 144, US = 3 * NM * 144, W = NM * 144;
  static constexpr int SIZE = NM <= 16 ? 3 * NM * 144 + NM * NU : 2 * NM * 144;
};
// the slot stride of the layouts a context of horizon N launches (host and device)
__host__ __device__ constexpr int ipm_slot_doubles(int N) {
  return N <= 16 ? IpmSlot<16>::SIZE : N <= kDenseN ? IpmSlot<kDenseN>::SIZE : IpmSlot<kMaxN>::SIZE;
}

// 12 consecutive doubles of a 16-B aligned LDS vector, 16 B per read
__device__ __forceinline__ void ld12(double (&v)[12], const double* p) {
  const d2* q = reinterpret_cast<const d2*>(p);
#pragma unroll
  for (int i = 0; i < 6; ++i) {
    const d2 x = q[i];
    v[2 * i] = x[0];
    v[2 * i + 1] = x[1];
  }
}
__device__ __forceinline__ void st12(double* p, const double (&v)[12]) {
  d2* q = reinterpret_cast<d2*>(p);
#pragma unroll
  for (int i = 0; i < 6; ++i) q[i] = d2{v[2 * i], v[2 * i + 1]};
}
// the same from global memory (the Riccati S_k scratch slot)
__device__ __forceinline__ void ld12g(double (&v)[12], const double* __restrict__ p) {
  const d2* q = reinterpret_cast<const d2*>(p);
#pragma unroll
  for (int i = 0; i < 6; ++i) {
    const d2 x = q[i];
    v[2 * i] = x[0];
    v[2 * i + 1] = x[1];
  }
}
__device__ __forceinline__ double dot12(const double (&a)[12], const double (&b)[12]) {
  double s0 = a[0] * b[0], s1 = a[1] * b[1], s2 = a[2] * b[2];
#pragma unroll
  for (int i = 3; i < 12; i += 3) {
    s0 = fma(a[i], b[i], s0);
    s1 = fma(a[i + 1], b[i + 1], s1);
    s2 = fma(a[i + 2], b[i + 2], s2);
  }
  return (s0 + s1) + s2;
}

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

// One robot with more than 128 stance variables.  Called by a 64-thread workgroup.
// XR: the weights' R couples different legs (mpcqp_set_weights; FULL and the latency layout):
// the stage weights W_k are then whole 12 x 12 matrices (stage_weights below) instead of the
// foot-steps' 3 x 3 blocks.
template <bool FULL, int NM, bool MG, bool XR = false>
__device__ __forceinline__ void solve_robot_ipm(const KParams& KP, int b, IpmSharedT<NM, FULL, MG>& sm, double* __restrict__ Sg,
                                                const float* __restrict__ x0g, const float* __restrict__ xrefg,
                                                const float* __restrict__ contactg, const float* __restrict__ feetg,
                                                const float* __restrict__ robotg, float* __restrict__ u0g,
                                                float* __restrict__ Ug, int* __restrict__ statusg,
                                                int* __restrict__ itersg) {
  constexpr int NT = LANES;
  const int lane = threadIdx.x;
  const int N = KP.N;
  const double h = KP.dt;

  // ------------------------------------------------ formulation (mpcqp_form.h)
  auto& smf = sm.fa.f;
  if (!form_stage<NT>(smf, N, b, lane, x0g, xrefg, contactg, feetg, robotg)) {
    write_empty_t<NT>(b, lane, N, MPCQP_STATUS_NONFINITE, u0g, Ug, statusg, itersg);
    return;
  }
  form_stance(smf, sm.mt, N, lane);
  fsync<NT>();
  const int S = uni(sm.mt.S);
  if (S == 0) {   // no stance foot-step (a caller's promise broken by a flight schedule): U = 0
    write_empty_t<NT>(b, lane, N, MPCQP_STATUS_OK, u0g, Ug, statusg, itersg);
    return;
  }
  static_assert(!XR || (FULL && !MG), "a cross-leg R runs in the full-weight latency layouts");
  if constexpr (FULL && !XR) {   // the host routes a cross-leg R to the XR instantiation: a guard
    bool cross = false;
    for (int e = lane; e < NU * NU; e += NT)
      cross |= (e / NU) / 3 != (e % NU) / 3 && KP.wfull[NX * NX + e] != 0.0;
    if (__any(cross)) {
      write_empty_t<NT>(b, lane, N, MPCQP_STATUS_UNSUPPORTED, u0g, Ug, statusg, itersg);
      return;
    }
  }
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
      sm.BmT[c][i] = v;
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
    if constexpr (FULL) {
      for (int e = lane; e < NX * NX; e += NT) sm.wf.qf[e / NX][e % NX] = 2.0 * KP.wfull[e];
      for (int e = lane; e < NU * NU; e += NT) sm.wf.rf[e / NU][e % NU] = 2.0 * KP.wfull[NX * NX + e];
    }
    for (int e = lane; e < N * NX; e += NT) sm.xr[e / NX][e % NX] = (double)smf.in[FormT<NM>::IN_XREF + e];
    for (int e = lane; e < N * NU; e += NT) sm.U[e / NU][e % NU] = 0.0;
  }
  fsync<NT>();   // the formulation scratch (union with S) is dead from here on

  // ------------------------------------------------ per-lane foot-steps
  const int liv = sm.mt.fz0_implied != 0 ? 0x2F : 0x3F;   // live rows: n.f >= 0 is implied when mu > 0
  const int R = sm.mt.fz0_implied != 0 ? 5 : 6;
  const double m_tot = (double)(S * R);
  double rw[6][3];   // cone rows (wave-uniform)
#pragma unroll
  for (int r = 0; r < 6; ++r)
#pragma unroll
    for (int x = 0; x < 3; ++x) rw[r][x] = sgpr_d(sm.mt.rows[r][x]);
  auto adot = [&](int r, const double (&v)[3]) -> double {
    return rw[r][0] * v[0] + rw[r][1] * v[1] + rw[r][2] * v[2];
  };
  auto foot = [&](int j, const double (*A)[NU], double (&o)[3]) {   // stance foot-step j of an N x 12 array
    const double* p = &A[sm.mt.foot_t[j]][3 * sm.mt.foot_leg[j]];
    o[0] = p[0];
    o[1] = p[1];
    o[2] = p[2];
  };
  auto foot_ptr = [&](int j, double (*A)[NU]) -> double* { return &A[sm.mt.foot_t[j]][3 * sm.mt.foot_leg[j]]; };
  // the lane's stance foot-step state: registers when a lane owns at most one foot-step
  // (every loop below runs j = lane, lane + 64, ...: then only j = lane), else LDS
  constexpr bool kRegFoot = 4 * NM <= LANES;
  IpmFootReg fr;
  auto FS = [&](int j) -> double (&)[6] { if constexpr (kRegFoot) return fr.fs; else return sm.ft.fs[j]; };
  auto FL = [&](int j) -> double (&)[6] { if constexpr (kRegFoot) return fr.fl; else return sm.ft.fl[j]; };
  auto FRP = [&](int j) -> double (&)[6] { if constexpr (kRegFoot) return fr.frp; else return sm.ft.frp[j]; };
  auto FRD = [&](int j) -> double (&)[4] { if constexpr (kRegFoot) return fr.frd; else return sm.ft.frd[j]; };
  auto FDS = [&](int j) -> double (&)[6] { if constexpr (kRegFoot) return fr.fds; else return sm.ft.fds[j]; };
  auto FDL = [&](int j) -> double (&)[6] { if constexpr (kRegFoot) return fr.fdl; else return sm.ft.fdl[j]; };
  auto FPJ = [&](int j) -> double (&)[9] { if constexpr (kRegFoot) return fr.fpj; else return sm.ft.fpj[j]; };
  auto FACT = [&](int j) -> int& { if constexpr (kRegFoot) return fr.fact; else return sm.ft.fact[j]; };
  auto FPREV = [&](int j) -> int& { if constexpr (kRegFoot) return fr.fprev; else return sm.ft.fprev[j]; };
  constexpr int kRh = FULL ? 9 : 3;   // the leg's 3 x 3 block of Rh, or its diagonal
  auto legrh = [&](int j, double (&o)[kRh]) {
    const int l = sm.mt.foot_leg[j];
    if constexpr (FULL) {
#pragma unroll
      for (int x = 0; x < 3; ++x)
#pragma unroll
        for (int y = 0; y < 3; ++y) o[3 * x + y] = sm.wf.rf[3 * l + x][3 * l + y];
    } else {
      o[0] = sm.rh[3 * l];
      o[1] = sm.rh[3 * l + 1];
      o[2] = sm.rh[3 * l + 2];
    }
  };

#ifdef MPCQP_IPM_DEBUG
  unsigned long long cyc[8] = {0, 0, 0, 0, 0, 0, 0, 0}, cyc_t0 = __builtin_amdgcn_s_memtime();
#define IPM_T0() const unsigned long long t0_ = __builtin_amdgcn_s_memtime()
#define IPM_T1(i) cyc[i] += __builtin_amdgcn_s_memtime() - t0_
#define IPM_TS(v)                                                   \
  __builtin_amdgcn_sched_barrier(0);                                \
  const unsigned long long v = __builtin_amdgcn_s_memtime();        \
  __builtin_amdgcn_sched_barrier(0)
#define IPM_TA(i, a, bb) cyc[i] += (bb) - (a)
#else
#define IPM_TS(v) do {} while (0)
#define IPM_TA(i, a, bb) do {} while (0)
#define IPM_T0() do {} while (0)
#define IPM_T1(i) do {} while (0)
#endif
  // ------------------------------------------------ stage recursions (one wave).  Nm =
  // A_d - I on the 13-state: rows 0..2 <- h R_z^T x[6..8]; rows 3..5 <- h x[9..11]
  // (+ h^2/2 x[12] on row 5); row 11 <- h x[12].  Every recursion over the stages runs in
  // registers, lane i holding entry i of the stage vector; its only cross-lane traffic is
  // readlane of the entries the stage map mixes in.  Everything that does not depend on
  // the recursion (B_d U_k, the stage gradients, the per-stage matvecs of lsolve) is
  // computed for all N stages at once in LDS phases: N x 12 entries over the 64 lanes,
  // operands loaded as whole 12-vectors (6 x 16-B LDS reads issued back to back).
  //
  // Lane coefficients of Nm (lane = state row i): (Nm x)_i = sum_s fc[s] x_{6+s}, s = 0..6;
  // (Nm^T nu)_i = sum_s bc[s] nu_{src(s)}, src = 0, 1, 2, 3, 4, 5, 11.
  double fc[7], bc[7];
  {
    const double h2 = 0.5 * h * h;
    const int r3 = lane < 3 ? lane : 0, c3 = (lane >= 6 && lane < 9) ? lane - 6 : 0;
#pragma unroll
    for (int c = 0; c < 3; ++c) {
      fc[c] = lane < 3 ? sm.nmr[r3][c] : 0.0;
      bc[c] = (lane >= 6 && lane < 9) ? sm.nmr[c][c3] : 0.0;
    }
#pragma unroll
    for (int s = 3; s < 6; ++s) {
      fc[s] = lane == s ? h : 0.0;       // rows 3..5 <- h x_{row + 6}
      bc[s] = lane == s + 6 ? h : 0.0;   // rows 9..11 <- h nu_{row - 6}
    }
    fc[6] = lane == 5 ? h2 : (lane == 11 ? h : 0.0);
    bc[5] = lane == 11 ? h : (lane == 12 ? h2 : 0.0);
    bc[6] = lane == 12 ? h : 0.0;
  }
  auto mix7 = [](const double (&cf)[7], const double (&s)[7], double add) -> double {
    const double a0 = fma(cf[0], s[0], cf[1] * s[1]);
    const double a1 = fma(cf[2], s[2], cf[3] * s[3]);
    const double a2 = fma(cf[4], s[4], cf[5] * s[5]);
    const double a3 = fma(cf[6], s[6], add);
    return (a0 + a1) + (a2 + a3);
  };

  const int lr = lane >> 4, lc = lane & 15;
  const int lcc = lc < 12 ? lc : 0;
  double Nmb[2], Bop[3], bx[3][3];   // Nm[4q+lr][lc]; B_d[lc][4q+lr]; B_d[lc][3 leg(4q+lr) + a]
#pragma unroll
  for (int q = 0; q < 3; ++q) {
    const int c = 4 * q + lr;
    const bool ok = c < 12 && lc < 12;
    const int cc = ok ? c : 0;
    if (q < 2) {
      double nv = 0.0;
      if (c < 3 && lc >= 6 && lc < 9) nv = sm.nmr[cc][lc - 6];
      else if (c >= 3 && c < 6 && lc == c + 6) nv = h;
      Nmb[q] = nv;
    }
    Bop[q] = ok ? sm.Bm[lcc][cc] : 0.0;
#pragma unroll
    for (int a2 = 0; a2 < 3; ++a2) bx[q][a2] = ok ? sm.Bm[lcc][3 * (cc / 3) + a2] : 0.0;
  }
  auto diag4 = [&](double d) -> d4 {   // d I (12 x 12) in result layout
    d4 v;
#pragma unroll
    for (int i = 0; i < 4; ++i) v[i] = (lr + 4 * i == lc && lc < 12) ? d : 0.0;
    return v;
  };
  auto qhat4 = [&]() -> d4 {   // Qh's 12 x 12 moving-state block in result layout
    d4 v;
    if constexpr (FULL) {
#pragma unroll
      for (int i = 0; i < 4; ++i) v[i] = (lr + 4 * i < 12 && lc < 12) ? sm.wf.qf[lr + 4 * i][lc] : 0.0;
    } else {
      v = diag4(sm.qh[lcc]);
    }
    return v;
  };
  auto mfma = [](double a, double b, d4 c) -> d4 { return __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0); };
  // dst_k = src_k M^T for every stage k < N, M = B_d (bop = Bop) or B_d^T (bop = BmT's operands):
  // the N x 12 by 12 x 12 product on the f64 matrix cores, 16 stages per tile -- per K-chunk one
  // 8-byte LDS read and one v_mfma_f64_16x16x4_f64 per lane, in place of two whole 12-vector reads
  // per output entry (the batched phases' LDS traffic bounds the class at four robots per CU)
  auto stage_gemm = [&](double (*dst)[NU], const double (*src)[NU], const double (&bop)[3]) {
    for (int t = 0; t < N; t += 16) {
      d4 D = diag4(0.0);
      const int ka = t + lc;
#pragma unroll
      for (int q = 0; q < 3; ++q) {
        const int j = 4 * q + lr;
        D = mfma(ka < N && j < 12 ? src[ka][j] : 0.0, bop[q], D);
      }
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int k = t + lr + 4 * i;
        if (k < N && lc < 12) dst[k][lc] = D[i];
      }
    }
    fsync<NT>();
  };
  // B_d^T's B operands: B_d[4q + lr][lc] (BmT is B_d^T, row lc)
  auto bt_ops = [&](double (&bt)[3]) {
#pragma unroll
    for (int q = 0; q < 3; ++q) {
      const int c = 4 * q + lr;
      bt[q] = c < 12 && lc < 12 ? sm.BmT[lc][c] : 0.0;
    }
  };

  // sm.gr = H U + g on stance coordinates: forward simulation + adjoint recursion
  auto gradient = [&]() {
    IPM_T0();
    stage_gemm(sm.BU, sm.U, Bop);   // B_d U_k, every stage
    // x_{k+1} = x_k + Nm x_k + B_d u_k (lane 12, the gravity state, stays constant)
    double x = lane < NX ? sm.x0[lane] : 0.0;
    if (lane < NX) sm.X[0][lane] = x;
    for (int k = 0; k < N; ++k) {
      const double bu = sm.BU[k][lane < NU ? lane : 0];
      double s[7];
#pragma unroll
      for (int t = 0; t < 7; ++t) s[t] = readlane_d(x, 6 + t);
      x += mix7(fc, s, lane < NU ? bu : 0.0);
      if (lane < NX) sm.X[k + 1][lane] = x;   // read back by the same lane below
    }
    // nu_k = Qh (x_{k+1} - xref_k) + (I + Nm^T) nu_{k+1}
    double nu = 0.0;
    const int li = lane < NX ? lane : 0;
    for (int k = N - 1; k >= 0; --k) {
      double v = 0.0;
      if constexpr (FULL) {
        if (lane < NX) {
#pragma unroll
          for (int j = 0; j < NX; ++j) v = fma(sm.wf.qf[li][j], sm.X[k + 1][j] - sm.xr[k][j], v);
        }
      } else {
        v = lane < NX ? sm.qh[li] * (sm.X[k + 1][li] - sm.xr[k][li]) : 0.0;
      }
      if (k < N - 1) {
        double s[7];
#pragma unroll
        for (int t = 0; t < 6; ++t) s[t] = readlane_d(nu, t);
        s[6] = readlane_d(nu, 11);
        v += nu + mix7(bc, s, 0.0);
      }
      nu = v;
      if (lane < NU) sm.nuh[k][lane] = nu;
    }
    fsync<NT>();
    {
      double bt[3];
      bt_ops(bt);
      stage_gemm(sm.BU, sm.nuh, bt);   // B_d^T nu_k, every stage (B_d U_k is dead)
    }
    for (int e = lane; e < N * NU; e += NT) {   // stage gradients R u_k + B_d^T nu_k
      const int k = e / NU, c = e % NU;
      double ru;
      if constexpr (XR) {   // the whole row of Rh (swing entries of U are 0)
        double r12[12], u12[12];
        ld12(r12, sm.wf.rf[c]);
        ld12(u12, sm.U[k]);
        ru = dot12(r12, u12);
      } else if constexpr (FULL) {
        const int c3 = 3 * (c / 3);   // Rh's leg block (no cross-leg couplings in this instantiation)
        ru = fma(sm.wf.rf[c][c3 + 2], sm.U[k][c3 + 2], fma(sm.wf.rf[c][c3 + 1], sm.U[k][c3 + 1], sm.wf.rf[c][c3] * sm.U[k][c3]));
      } else {
        ru = sm.rh[c] * sm.U[k][c];
      }
      const double g = ru + sm.BU[k][c];
      sm.gr[k][c] = sm.mt.stance_of[4 * k + c / 3] >= 0 ? g : 0.0;
    }
    fsync<NT>();
    IPM_T1(0);
  };

  // Riccati factorisation with the per-foot-step weights sm.W: S_k and M_k for every
  // stage, the 12 x 12 stage products on the f64 matrix cores.  v_mfma_f64_16x16x4f64
  // (tools/ubench/mfma_f64_check.hip; lr = lane >> 4, lc = lane & 15): the A operand of
  // K-chunk q is A[lc][4q + lr], the B operand B[4q + lr][lc], result register i
  // D[lr + 4i][lc] -- so result register q of a matrix IS its B operand of chunk q, and
  // its A operand when the matrix is symmetric; the recursion P -> T -> S -> P stays in
  // registers (12 x 12 padded to 16 x 16) except for the Gauss-Jordan sweep.  Per stage:
  //   E = B_d blockdiag(W_k) B_d^T   (blockdiag(W_k) B_d^T formed on the VALU in B-operand form)
  //   T = I + P E;  S = T^-1 P by Gauss-Jordan on [T | P] (lane j < 12 holds column j of T,
  //       lane 12 + j column j of P; pivot column by readlane), symmetrised
  //   P <- Qh + A^T S A;  M_k = A^T (I - S E)     (A = I + Nm; Nm has rows 0..5 only, so
  //       a product with Nm or Nm^T is 2 K-chunks)
  // (information form; the textbook P - P B (R + B^T P B)^-1 B^T P loses ~4 digits here).
  // The critical path per stage is S -> P -> T -> sweep; E of the next stage and M of the
  // previous one are issued before the sweep, so the matrix cores run them under it.
  auto stage_e = [&](int k) -> d4 {   // E_k
    d4 Er = diag4(0.0);
    if constexpr (XR) {   // (W_k B_d^T)[c][lc] = W_k row c . B_d row lc (W_k: 0 on swing rows)
      double brow[12];
      ld12(brow, sm.Bm[lcc]);
#pragma unroll
      for (int q = 0; q < 3; ++q) {
        const int c = 4 * q + lr;
        double x = 0.0;
        if (c < 12 && lc < 12) {
          double wr[12];
          ld12g(wr, Sg + IpmSlot<NM>::W + k * 144 + 12 * c);
          x = dot12(wr, brow);
        }
        Er = mfma(Bop[q], x, Er);
      }
      return Er;
    }
#pragma unroll
    for (int q = 0; q < 3; ++q) {
      const int c = 4 * q + lr;
      double x = 0.0;
      if (c < 12 && lc < 12) {
        const int j = sm.mt.stance_of[4 * k + c / 3];
        if (j >= 0) {
          const double* w = sm.W[j] + 3 * (c % 3);
          x = w[0] * bx[q][0] + w[1] * bx[q][1] + w[2] * bx[q][2];
        }
      }
      Er = mfma(Bop[q], x, Er);
    }
    return Er;
  };
  // The factorisation runs in the basis x~ = T x, T = I - Nm / 2 (12-state: Nm maps rows 6..11
  // into rows 0..5, so Nm^2 = 0 and T^-1 = I + Nm / 2).  There B_d = T^-1 [0; B6] (B6 = B_d's
  // rows 6..11: rows 0..5 of B_d are (h^2 / 2) R_z^T K and h^2 / 2m, i.e. Nm / 2 of rows 6..11 --
  // the midpoint rule), T A_d T^-1 = A_d, the stage cost is Qt = T^-T Qh T^-1, and
  // E~_k = diag(0, C_k) with C_k = E_k[6:12, 6:12] = B6 W_k B6^T.  Riccati on P~ = T^-T P T^-1:
  //   K = P~[6:12, 6:12], V = P~[6:12, :], G = (I + C K)^-1, Y = G C = (C^-1 + K)^-1 (6 x 6),
  //   S~ = (I + P~ E~)^-1 P~ = P~ - V^T Y V,   P~_k = Qt + A^T S~ A   (Woodbury),
  // one Gauss-Jordan on [I + C K | C | I] -- 6 pivots over 18 lanes, 6-entry pivot columns --
  // in place of [I + P E | P] (12 pivots over 24 lanes, 12-entry columns: 4x the v_readlane
  // broadcasts).  lsolve's operators, in the original basis:
  //   S L = T^T V^T G            (S_k B = (S L) B6: its only use of S_k),
  //   M_k = A^T (I - S E) = (I + Nm^T / 2) (I - V^T Y [0 I]) (I + Nm^T / 2).
  // S L and M_k are never formed from S: where E is large S is small in E's range and
  // P~ - V^T Y V cancels there (absolute error eps |P|, then multiplied by E), while V^T G and
  // V^T Y carry no such cancellation (tools/ipm_proto.py FACTOR=range: identical iteration counts
  // on its 64 + 32 cases; S L taken from S fails a sparse N = 32 case).
  auto nm12 = [&](int i, int j) -> double {   // Nm[i][j] on the 12-state
    if (i < 3 && j >= 6 && j < 9) return sm.nmr[i][j - 6];
    if (i >= 3 && i < 6 && j == i + 6) return h;
    return 0.0;
  };
  double NbT[3], IpB[3];   // Nm[lc][4q + lr] (B operands of Nm^T); (I + Nm^T / 2)[4q + lr][lc]
#pragma unroll
  for (int q = 0; q < 3; ++q) {
    const int c = 4 * q + lr;
    const bool ok = c < 12 && lc < 12;
    NbT[q] = ok ? nm12(lc, c) : 0.0;
    IpB[q] = ok ? (c == lc ? 1.0 : 0.0) + 0.5 * nm12(lc, c) : 0.0;
  }
  {   // Qt = (I + Nm^T / 2) Qh (I + Nm / 2) -> sm.QT (once per robot)
    const d4 Qr = qhat4();
    d4 R = Qr;   // Qh (I + Nm / 2)
#pragma unroll
    for (int q = 0; q < 2; ++q) R = mfma(Qr[q], 0.5 * Nmb[q], R);
    d4 Q = R;
#pragma unroll
    for (int q = 0; q < 2; ++q) Q = mfma(0.5 * Nmb[q], R[q], Q);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int r = lr + 4 * i;
      if (r < 12 && lc < 12) sm.QT[12 * r + lc] = Q[i];
    }
    fsync<NT>();
  }
  auto qt4 = [&]() -> d4 {   // Qt in result layout
    d4 v;
#pragma unroll
    for (int i = 0; i < 4; ++i) v[i] = (lr + 4 * i < 12 && lc < 12) ? sm.QT[12 * (lr + 4 * i) + lc] : 0.0;
    return v;
  };
  auto blk6 = [&](const d4& X, bool cols) -> d4 {   // rows 6..11 of X (and columns 6..11 when cols)
    d4 c;
#pragma unroll
    for (int i = 0; i < 4; ++i) c[i] = (lr + 4 * i >= 6 && (!cols || lc >= 6)) ? X[i] : 0.0;
    return c;
  };
  constexpr bool kMG = IpmSharedT<NM, FULL, MG>::kMG;
  // M_k = (I + Nm^T / 2) X (I + Nm^T / 2), X = I - V^T Y [0 I] -> M[k] (and M^T).  Zr = (Y V)'s
  // result registers: X^T = I - Y V, so its result registers are X's A operands
  auto stage_m = [&](int k, const d4& Zr) {
    d4 R1 = diag4(0.0);   // X (I + Nm^T / 2)
#pragma unroll
    for (int q = 0; q < 3; ++q) R1 = mfma(((lr + 4 * q == lc && lc < 12) ? 1.0 : 0.0) - Zr[q], IpB[q], R1);
    d4 Mr = R1;
#pragma unroll
    for (int q = 0; q < 2; ++q) Mr = mfma(0.5 * Nmb[q], R1[q], Mr);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int r = lr + 4 * i;
      if (r < 12 && lc < 12) {
        if constexpr (kMG) {
          Sg[IpmSlot<NM>::M + k * 144 + 12 * r + lc] = Mr[i];
          Sg[IpmSlot<NM>::MT + k * 144 + 12 * lc + r] = Mr[i];
        } else {
          sm.mk.M[k][12 * r + lc] = Mr[i];
        }
      }
    }
  };

  // Riccati factorisation: per stage k the global slot's 144 doubles hold S~_k [0; I] = V^T G
  // (12 x 6, row-major) and its transpose (6 x 12), from which lsolve takes every product with
  // S_k (S_k L = T^T V^T G); M_k as stage_m stores it
  auto factor = [&]() {
    IPM_T0();
    d4 Pr = qt4();   // P~_{k+1}
    d4 Cr = blk6(stage_e(N - 1), true), Zp = diag4(0.0);
    const int jc = lane < 18 ? lane : 0;
    for (int k = N - 1; k >= 0; --k) {
      IPM_TS(ta);
      const d4 Kr = blk6(Pr, true);
      d4 Mr = diag4(1.0);   // I + C K
#pragma unroll
      for (int q = 1; q < 3; ++q) Mr = mfma(Cr[q], Kr[q], Mr);
      // column c < 6 of I + C K at TT[c], column c of C at TT[6 + c] (rows 6..11 -> 0..5)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int r = lr + 4 * i;
        if (r >= 6 && r < 12 && lc >= 6 && lc < 12) {
          sm.TT[lc - 6][r - 6] = Mr[i];
          sm.TT[lc][r - 6] = Cr[i];
        }
      }
      fsync<NT>();
      IPM_TS(tb);
      double col[6];   // lanes 0..5: I + C K, 6..11: C, 12..17: I
      if (lane < 12) {
        const d2* q = reinterpret_cast<const d2*>(sm.TT[jc]);
#pragma unroll
        for (int i = 0; i < 3; ++i) {
          const d2 x = q[i];
          col[2 * i] = x[0];
          col[2 * i + 1] = x[1];
        }
      } else {
#pragma unroll
        for (int i = 0; i < 6; ++i) col[i] = jc - 12 == i ? 1.0 : 0.0;
      }
      // under the sweep: M of the previous stage, C of the next
      if (k < N - 1) stage_m(k + 1, Zp);
      const d4 Cn = k > 0 ? blk6(stage_e(k - 1), true) : diag4(0.0);
#pragma unroll
      for (int kk = 0; kk < 6; ++kk) {
        double pc[6];
#pragma unroll
        for (int i = 0; i < 6; ++i) pc[i] = readlane_d(col[i], kk);
        const double ip = rcp_nr(pc[kk]);
        const double rowv = col[kk] * ip;
#pragma unroll
        for (int i = 0; i < 6; ++i) col[i] = (i == kk) ? rowv : fma(-pc[i], rowv, col[i]);
      }
      IPM_TS(tc);
      if (lane >= 6 && lane < 18) {   // Y's columns over C's (TT[6 + c]), G's over I + C K's (TT[c])
        d2* q = reinterpret_cast<d2*>(sm.TT[lane < 12 ? jc : jc - 12]);
#pragma unroll
        for (int i = 0; i < 3; ++i) q[i] = d2{col[2 * i], col[2 * i + 1]};
      }
      fsync<NT>();
      IPM_TS(td);
      IPM_TA(4, ta, tb);
      IPM_TA(5, tb, tc);
      IPM_TA(6, tc, td);
      d4 Yr, Gr;   // (Y + Y^T) / 2 and G in the block [6:12, 6:12]
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int r = lr + 4 * i;
        const bool in = r >= 6 && r < 12 && lc >= 6 && lc < 12;
        const int r6 = in ? r - 6 : 0, c6 = in ? lc - 6 : 0;
        Yr[i] = in ? 0.5 * (sm.TT[6 + c6][r6] + sm.TT[6 + r6][c6]) : 0.0;
        Gr[i] = in ? sm.TT[c6][r6] : 0.0;
      }
      const d4 Vr = blk6(Pr, false);
      d4 Zr = diag4(0.0);   // Y V
#pragma unroll
      for (int q = 1; q < 3; ++q) Zr = mfma(Yr[q], Vr[q], Zr);
      if (k > 0) {   // P~_k = Qt + A^T S~ A, S~ = P~ - V^T Y V
        d4 Sr = Pr;
#pragma unroll
        for (int q = 1; q < 3; ++q) Sr = mfma(-Vr[q], Zr[q], Sr);
        d4 SA = Sr;
#pragma unroll
        for (int q = 0; q < 2; ++q) SA = mfma(Sr[q], Nmb[q], SA);
        Pr = qt4();
#pragma unroll
        for (int i = 0; i < 4; ++i) Pr[i] += SA[i];
#pragma unroll
        for (int q = 0; q < 2; ++q) Pr = mfma(Nmb[q], SA[q], Pr);
      }
      d4 SLr = diag4(0.0);   // S~ [0; I] = V^T G (columns 6..11); lsolve applies S L = T^T of it
#pragma unroll
      for (int q = 1; q < 3; ++q) SLr = mfma(Vr[q], Gr[q], SLr);
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int r = lr + 4 * i;
        if (r < 12 && lc >= 6 && lc < 12) {
          Sg[k * 144 + 6 * r + lc - 6] = SLr[i];
          Sg[k * 144 + 72 + 12 * (lc - 6) + r] = SLr[i];
        }
      }
      Zp = Zr;
      Cr = Cn;
      IPM_TS(te);
      IPM_TA(7, td, te);
    }
    stage_m(0, Zp);
    fsync<NT>();   // S_k L, M_k for lsolve
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "workgroup");   // the global stores (S_k L, M_k), before lsolve reads them
    IPM_T1(1);
  };

  // (H + G^T D G) d = rhs restricted to the foot-steps' subspaces: sm.rhs -> sm.dU
  // The Riccati sweep in affine form (factor's M_k = A^T (I - S_k E_k), E_k = B W_k B^T):
  //   backward  Y_k = W_k (B^T p_{k+1} - rhs_k),  p_k = A^T (p_{k+1} - S_k B Y_k)
  //                                              = M_k p_{k+1} + A^T S_k B W_k rhs_k,
  //   forward   d_k = W_k B^T S_k (B Y_k - A dx_k) - Y_k,  dx_{k+1} = A dx_k + B d_k
  //                                              = M_k^T dx_k + B (W_k B^T S_k B Y_k - Y_k),
  // so each recursion is one 12 x 12 matvec per stage (12 lanes, readlane of the vector)
  // and every other product runs for all stages at once.
  auto bmat = [&](double (*dst)[NU], double (*src)[NU]) { stage_gemm(dst, src, Bop); };   // dst_k = B_d src_k
  // W_k (z_k - sub_k) restricted to entry c (leg l = c / 3), z_k = B_d^T x_k precomputed for every
  // stage by stage_gemm; 0 for a swing leg
  auto wz = [&](int k, int c, const double (*z)[NU], const double* sub) -> double {
    if constexpr (XR) {   // W_k row c . (z_k - sub)
      double wr[12], zv[12];
      ld12g(wr, Sg + IpmSlot<NM>::W + k * 144 + 12 * c);
      ld12(zv, z[k]);
      if (sub) {
        double sv[12];
        ld12(sv, sub);
#pragma unroll
        for (int i = 0; i < 12; ++i) zv[i] -= sv[i];
      }
      return dot12(wr, zv);
    }
    const int l = c / 3, a = c % 3;
    const int j = sm.mt.stance_of[4 * k + l];
    if (j < 0) return 0.0;
    const double z0 = z[k][3 * l] - (sub ? sub[3 * l] : 0.0);
    const double z1 = z[k][3 * l + 1] - (sub ? sub[3 * l + 1] : 0.0);
    const double z2 = z[k][3 * l + 2] - (sub ? sub[3 * l + 2] : 0.0);
    const double* wj = sm.W[j] + 3 * a;
    return wj[0] * z0 + wj[1] * z1 + wj[2] * z2;
  };
  double btop[3];   // B_d^T's operands for the lsolve phases
  bt_ops(btop);
  // t_k = S~_k [0; I] (src_k rows 6..11) for src_k = B_d y in B_d's range, every stage, so that
  // S_k src_k = T^T t_k; range: rows 0..5 of t_k set to 0 (then B_d^T T^T t_k = B_d^T dst_k,
  // T B_d = [0; B6])
  auto smat = [&](double (*dst)[NU], double (*src)[NU], bool range) {
    for (int e = lane; e < N * NU; e += NT) {
      const int k = e / NU, i = e % NU;
      const d2* sr = reinterpret_cast<const d2*>(Sg + k * 144 + 6 * i);
      const d2* v = reinterpret_cast<const d2*>(src[k] + 6);
      const d2 s0 = sr[0], s1 = sr[1], s2 = sr[2], v0 = v[0], v1 = v[1], v2 = v[2];
      const double t = fma(s0[0], v0[0], fma(s1[0], v1[0], s2[0] * v2[0])) + fma(s0[1], v0[1], fma(s1[1], v1[1], s2[1] * v2[1]));
      dst[k][i] = range && i < 6 ? 0.0 : t;
    }
    fsync<NT>();
  };
  const int l12 = lane < NU ? lane : 0;

  auto lsolve = [&]() {
    IPM_T0();
    for (int e = lane; e < N * NU; e += NT) {   // la_k = W_k rhs_k
      const int k = e / NU, c = e % NU, l = c / 3, a = c % 3;
      const int j = sm.mt.stance_of[4 * k + l];
      double v = 0.0;
      if constexpr (XR) {
        v = wz(k, c, sm.rhs, nullptr);
      } else if (j >= 0) {
        const double* wj = sm.W[j] + 3 * a;
        v = wj[0] * sm.rhs[k][3 * l] + wj[1] * sm.rhs[k][3 * l + 1] + wj[2] * sm.rhs[k][3 * l + 2];
      }
      sm.la[k][c] = v;
    }
    fsync<NT>();
    bmat(sm.lb, sm.la);   // B W rhs
    smat(sm.la, sm.lb, false);   // t: S B W rhs = T^T t
    for (int e = lane; e < N * NU; e += NT) {   // lc_k = A^T S B W rhs = A^T T^T t = (I + Nm / 2)^T t
      const int k = e / NU, i = e % NU;
      double v = sm.la[k][i];
      if (i >= 6 && i < 9) v += 0.5 * (sm.nmr[0][i - 6] * sm.la[k][0] + sm.nmr[1][i - 6] * sm.la[k][1] + sm.nmr[2][i - 6] * sm.la[k][2]);
      else if (i >= 9) v += 0.5 * h * sm.la[k][i - 6];
      sm.lc[k][i] = v;
    }
    fsync<NT>();
    // backward recursion: lane i < 12 holds p_i
    double p = 0.0;
    if constexpr (kMG) {   // row l12 of M_k from the global slot, the next stage's issued ahead
      double mn[12];
      if (N > 1) ld12g(mn, Sg + IpmSlot<NM>::M + (N - 1) * 144 + 12 * l12);
      for (int k = N - 1; k >= 0; --k) {
        if (lane < NU) sm.ph[k][lane] = p;
        if (k > 0) {
          double mr[12], r[12];
#pragma unroll
          for (int j = 0; j < 12; ++j) mr[j] = mn[j];
          if (k > 1) ld12g(mn, Sg + IpmSlot<NM>::M + (k - 1) * 144 + 12 * l12);
          const double ck = sm.lc[k][l12];
#pragma unroll
          for (int j = 0; j < 12; ++j) r[j] = readlane_d(p, j);
          p = lane < NU ? dot12(mr, r) + ck : 0.0;
        }
      }
    } else {
      for (int k = N - 1; k >= 0; --k) {
        if (lane < NU) sm.ph[k][lane] = p;
        if (k > 0) {
          double mr[12], r[12];
          ld12(mr, sm.mk.M[k] + 12 * l12);
          const double ck = sm.lc[k][l12];
#pragma unroll
          for (int j = 0; j < 12; ++j) r[j] = readlane_d(p, j);
          p = lane < NU ? dot12(mr, r) + ck : 0.0;
        }
      }
    }
    fsync<NT>();
    stage_gemm(sm.la, sm.ph, btop);   // B^T p_{k+1} (la is dead until S B Y below)
    for (int e = lane; e < N * NU; e += NT) {   // Y_k = W_k (B^T p_{k+1} - rhs_k)
      const int k = e / NU, c = e % NU;
      sm.Y[k][c] = wz(k, c, sm.la, sm.rhs[k]);
    }
    fsync<NT>();
    bmat(sm.By, sm.Y);    // B Y
    smat(sm.la, sm.By, true);   // [0; t rows 6..11]: B^T of it = B^T S B Y
    stage_gemm(sm.lc, sm.la, btop);   // B^T S B Y (lc is dead until B lb below)
    for (int e = lane; e < N * NU; e += NT) {   // lb_k = W_k B^T S_k B Y_k - Y_k
      const int k = e / NU, c = e % NU;
      sm.lb[k][c] = wz(k, c, sm.lc, nullptr) - sm.Y[k][c];
    }
    fsync<NT>();
    bmat(sm.lc, sm.lb);   // B lb
    // forward recursion: lane i < 12 holds dx_i; dx_{k+1} = M_k^T dx_k + lc_k
    double dx = 0.0;
    if constexpr (kMG) {   // column l12 of M_k = row l12 of the stored transpose, issued ahead
      double mn[12];
      if (N > 1) ld12g(mn, Sg + IpmSlot<NM>::MT + 12 * l12);
      for (int k = 0; k < N; ++k) {
        if (lane < NU) sm.dxh[k][lane] = dx;
        if (k < N - 1) {
          double mc[12], r[12];
#pragma unroll
          for (int j = 0; j < 12; ++j) mc[j] = mn[j];
          if (k < N - 2) ld12g(mn, Sg + IpmSlot<NM>::MT + (k + 1) * 144 + 12 * l12);
          const double ek = sm.lc[k][l12];
#pragma unroll
          for (int j = 0; j < 12; ++j) r[j] = readlane_d(dx, j);
          dx = lane < NU ? dot12(mc, r) + ek : 0.0;
        }
      }
    } else {
      for (int k = 0; k < N; ++k) {
        if (lane < NU) sm.dxh[k][lane] = dx;
        if (k < N - 1) {
          double mc[12], r[12];
#pragma unroll
          for (int j = 0; j < 12; ++j) mc[j] = sm.mk.M[k][12 * j + l12];
          const double ek = sm.lc[k][l12];
#pragma unroll
          for (int j = 0; j < 12; ++j) r[j] = readlane_d(dx, j);
          dx = lane < NU ? dot12(mc, r) + ek : 0.0;
        }
      }
    }
    fsync<NT>();
    for (int e = lane; e < N * NU; e += NT) {   // la_k = L^T S_k (B Y_k - A dx_k) = (V^T G)^T T (...) at rows 6..11, 0 above
      const int k = e / NU, i = e % NU;
      double v = 0.0;
      if (i >= 6) {
        double dxv[12], by[12], sr[12];
        ld12(dxv, sm.dxh[k]);
        ld12(by, sm.By[k]);
        ld12g(sr, Sg + k * 144 + 72 + 12 * (i - 6));   // row i - 6 of (V^T G)^T
#pragma unroll
        for (int m = 0; m < 12; ++m) {   // A dx on the 12-state
          double a = dxv[m];
          if (m < 3) a += sm.nmr[m][0] * dxv[6] + sm.nmr[m][1] * dxv[7] + sm.nmr[m][2] * dxv[8];
          else if (m < 6) a += h * dxv[m + 6];
          by[m] -= a;
        }
#pragma unroll
        for (int m = 0; m < 6; ++m)   // T (B Y - A dx): (S L)^T v = (V^T G)^T T v
          by[m] -= 0.5 * (m < 3 ? sm.nmr[m][0] * by[6] + sm.nmr[m][1] * by[7] + sm.nmr[m][2] * by[8] : h * by[m + 6]);
        v = dot12(sr, by);
      }
      sm.la[k][i] = v;
    }
    fsync<NT>();
    stage_gemm(sm.lb, sm.la, btop);   // B^T S_k (...) = B6^T la_k[6:12] (lb is dead after B lb)
    for (int e = lane; e < N * NU; e += NT) {   // d_k = W_k B^T la_k - Y_k
      const int k = e / NU, c = e % NU;
      sm.dU[k][c] = wz(k, c, sm.lb, nullptr) - sm.Y[k][c];
    }
    fsync<NT>();
    IPM_T1(2);
  };

  // XR: the stage weights W_k (IpmSlot::W, 12 x 12 row-major) over the stage's stance entries
  // (swing rows / columns 0), from the foot-steps' blocks in sm.W[j]: the interior point's
  // G_j^T D_j G_j, W_k = (Rh + blockdiag G_j^T D_j G_j)^-1, or the polish's null-space projectors
  // P_j, W_k = P (P Rh P + I - P)^-1 P with P = blockdiag P_j -- the per-foot-step weights of the
  // leg-block instantiations with Rh's cross-leg blocks kept.  One stage at a time, Gauss-Jordan
  // on [A | I] or [A | P] (A SPD, no pivoting): lane c < 12 holds column c of A, lane 12 + c
  // column c of the right-hand side; the pivot column by readlane, as in factor().
  auto stage_weights = [&](bool pol) {
    if constexpr (XR) {
      const int jc = lane < 12 ? lane : (lane < 24 ? lane - 12 : 0);
      const int lj = jc / 3, cj = jc % 3;
      const bool rhs = lane >= 12;
      for (int k = 0; k < N; ++k) {
        const int fc = lane < 24 ? sm.mt.stance_of[4 * k + lj] : -1;   // this lane's column foot-step
        int fl[4];   // each leg's foot-step at stage k (-1: swing), wave-uniform
#pragma unroll
        for (int l = 0; l < 4; ++l) fl[l] = uni(sm.mt.stance_of[4 * k + l]);
        double pcol[3] = {0.0, 0.0, 0.0};   // column cj of P_fc (polish)
        if (pol && fc >= 0) {
#pragma unroll
          for (int a = 0; a < 3; ++a) pcol[a] = sm.W[fc][3 * a + cj];
        }
        double t[12];   // polish: (Rh P)[m][jc]
#pragma unroll
        for (int m = 0; m < 12; ++m) {
          const double* r = &sm.wf.rf[m][3 * lj];
          t[m] = pol ? fma(r[2], pcol[2], fma(r[1], pcol[1], r[0] * pcol[0])) : 0.0;
        }
        double col[12];
#pragma unroll
        for (int i = 0; i < 12; ++i) {
          const int li = i / 3, ai = i % 3;
          const int fi = fl[li];
          double v;
          if (rhs) {   // e_jc, or column jc of P
            v = pol ? (li == lj ? pcol[ai] : 0.0) : (i == jc ? 1.0 : 0.0);
          } else if (fi < 0 || fc < 0) {   // a swing leg's rows / columns: the identity
            v = i == jc ? 1.0 : 0.0;
          } else if (!pol) {   // Rh + G^T D G on the leg's block
            v = sm.wf.rf[i][jc] + (li == lj ? sm.W[fc][3 * ai + cj] : 0.0);
          } else {   // P Rh P + I - P
            const double* pi = sm.W[fi] + 3 * ai;   // row ai of P_fi
            v = fma(pi[2], t[3 * li + 2], fma(pi[1], t[3 * li + 1], pi[0] * t[3 * li]));
            if (li == lj) v += (i == jc ? 1.0 : 0.0) - pcol[ai];
          }
          col[i] = v;
        }
#pragma unroll
        for (int kk = 0; kk < 12; ++kk) {
          double pc[12];
#pragma unroll
          for (int i = 0; i < 12; ++i) pc[i] = readlane_d(col[i], kk);
          const double ip = rcp_nr(pc[kk]);
          const double rowv = col[kk] * ip;
#pragma unroll
          for (int i = 0; i < 12; ++i) col[i] = (i == kk) ? rowv : fma(-pc[i], rowv, col[i]);
        }
        if (rhs && lane < 24) {   // column jc of W_k: A^-1 (stance block), or P A^-1 P
#pragma unroll
          for (int i = 0; i < 12; ++i) {
            const int li = i / 3, ai = i % 3;
            const int fi = fl[li];
            double w = 0.0;
            if (fi >= 0 && fc >= 0) {
              if (pol) {
                const double* pi = sm.W[fi] + 3 * ai;
                w = fma(pi[2], col[3 * li + 2], fma(pi[1], col[3 * li + 1], pi[0] * col[3 * li]));
              } else {
                w = col[i];
              }
            }
            Sg[IpmSlot<NM>::W + k * 144 + 12 * i + jc] = w;
          }
        }
      }
      __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "workgroup");   // the W_k stores, before stage_e / wz read them
      fsync<NT>();
    }
  };

  int status = MPCQP_STATUS_MAX_ITER;
  int nfact = 0;
#ifdef MPCQP_IPM_DEBUG
  // diagnostic build: 8 floats per IPM iteration written to U (the solution is not)
  int dbg_n = 0;
  auto dbg = [&](double v) {
    if (lane == 0 && Ug && dbg_n < N * NU) Ug[(size_t)b * N * NU + dbg_n] = (float)v;
    ++dbg_n;
  };
  double dbg_p[3] = {0.0, 0.0, 0.0};
#endif

  // scales: gradient at U = 0 and the largest bound
  gradient();
  double gmax = 0.0, hmax = 0.0;
  for (int j = lane; j < S; j += NT) {
    double g[3];
    foot(j, sm.gr, g);
    gmax = fmax(gmax, fmax(fabs(g[0]), fmax(fabs(g[1]), fabs(g[2]))));
    hmax = fmax(hmax, sm.mt.ub[j]);
  }
  const double gscale = 1.0 + sgpr_d(wave_max_d(gmax));
  const double hscale = 1.0 + sgpr_d(wave_max_d(hmax));
  const double tol_g = 1e-9 * gscale, tol_h = 1e-9 * hscale;

  // ---- active-set polish on the rows FACT; true when verified (sm.U = the optimum)
  auto polish = [&]() -> bool {
    for (int j = lane; j < S; j += NT) {
      double rh[kRh], pj[9], fp[3], wv[9];
      legrh(j, rh);
      ipm_foot_nullspace(rw, FACT(j) & liv, -sm.mt.ub[j], rh, pj, fp, wv);
#pragma unroll
      for (int e = 0; e < 9; ++e) {
        sm.W[j][e] = XR ? pj[e] : wv[e];   // XR: the projector, for stage_weights
        FPJ(j)[e] = pj[e];
      }
      double* u = foot_ptr(j, sm.U);
      u[0] = fp[0];
      u[1] = fp[1];
      u[2] = fp[2];
    }
    fsync<NT>();
    stage_weights(true);
    factor();
    ++nfact;
    bool have_gr = false;   // sm.gr is the gradient at the final U (a refinement found it stationary)
    for (int rf = 0; rf < IPM_NREF; ++rf) {
      gradient();
      for (int e = lane; e < N * NU; e += NT) sm.rhs[e / NU][e % NU] = 0.0;
      fsync<NT>();
      double st = 0.0;
      for (int j = lane; j < S; j += NT) {
        double g[3];
        foot(j, sm.gr, g);
        const double (&pj)[9] = FPJ(j);
        double* r = foot_ptr(j, sm.rhs);
#pragma unroll
        for (int x = 0; x < 3; ++x) {
          r[x] = -(pj[3 * x] * g[0] + pj[3 * x + 1] * g[1] + pj[3 * x + 2] * g[2]);
          st = fmax(st, fabs(r[x]));
        }
      }
      fsync<NT>();
      // a later refinement of an already stationary iterate changes nothing the check can see:
      // the check takes this gradient (round 6: one Newton solve and one gradient fewer per
      // standing robot, tools/ipm_proto.py ADAPT_REF=1)
      if (rf > 0 && sgpr_d(wave_max_d(st)) < IPM_STAT_TOL * gscale) {
        have_gr = true;
        break;
      }
      lsolve();
      for (int j = lane; j < S; j += NT) {
        double d[3];
        foot(j, sm.dU, d);
        double* u = foot_ptr(j, sm.U);
        u[0] += d[0];
        u[1] += d[1];
        u[2] += d[2];
      }
      fsync<NT>();
    }
    if (!have_gr) gradient();
    double stat = 0.0, smin = INFINITY, lminw = INFINITY;
    for (int j = lane; j < S; j += NT) {
      double g[3], f[3];
      foot(j, sm.gr, g);
      foot(j, sm.U, f);
      const double (&pj)[9] = FPJ(j);
#pragma unroll
      for (int x = 0; x < 3; ++x) stat = fmax(stat, fabs(pj[3 * x] * g[0] + pj[3 * x + 1] * g[1] + pj[3 * x + 2] * g[2]));
      int viol = 0;
      const double h5 = -sm.mt.ub[j];
#pragma unroll
      for (int r = 0; r < 6; ++r)
        if ((liv >> r) & 1) {
          const double sl = adot(r, f) - (r == 5 ? h5 : 0.0);
          smin = fmin(smin, sl);
          if (sl < -tol_h) viol |= 1 << r;
        }
      const int am = FACT(j) & liv;
      double best = INFINITY;
      int drop = -1;
      if (am) {
        double pjl[9], fpd[3], wd[9], rh[kRh];
        legrh(j, rh);
        const int nq = ipm_foot_nullspace(rw, am, h5, rh, pjl, fpd, wd);
        ipm_cone_multipliers(rw, am, nq, g, tol_g, best, drop);
      }
      lminw = fmin(lminw, best);
      FACT(j) = (FACT(j) | viol) & ~(drop >= 0 ? (1 << drop) : 0);
    }
    stat = wave_max_d(stat);
    smin = wave_min(smin);
    lminw = wave_min(lminw);
    fsync<NT>();
#ifdef MPCQP_IPM_DEBUG
    dbg_p[0] = stat / gscale;
    dbg_p[1] = smin;
    dbg_p[2] = lminw;
#endif
    return stat < IPM_STAT_TOL * gscale && smin > -tol_h && lminw > -tol_g;
  };
  // polish, then correct the set (violated rows in, the most negative multiplier out)
  // until it verifies, stops changing or ncorr corrections are spent
  auto polish_corrected = [&](int ncorr) -> bool {
    for (int corr = 0; corr <= ncorr; ++corr) {
      int changed = 0;
      for (int j = lane; j < S; j += NT) FPREV(j) = FACT(j);
      fsync<NT>();
      if (polish()) return true;
      for (int j = lane; j < S; j += NT) changed |= FACT(j) != FPREV(j);
      if (!__any(changed)) break;
    }
    return false;
  };

  bool done = false;
  // ---- warm start (mpcqp_set_warm_start): the rows this robot's last verified solve had
  // active at the same (stage, leg); the cold start below when they do not verify
  unsigned char* const wmem = KP.warm && b < KP.warm_cap ? KP.warm + (size_t)b * MPCQP_WARM_BYTES : nullptr;
  if (wmem) {
    int known = 0;
    for (int j = lane; j < S; j += NT) {
      const int v = wmem[4 * sm.mt.foot_t[j] + sm.mt.foot_leg[j]];
      FACT(j) = v & liv;
      known |= v & 0x80;
    }
    if (__any(known)) {
      if (polish_corrected(IPM_NCORR)) {
        done = true;
        status = MPCQP_STATUS_OK;
      } else {   // back to U = 0 and its gradient for the cold start
        for (int e = lane; e < N * NU; e += NT) sm.U[e / NU][e % NU] = 0.0;
        fsync<NT>();
        gradient();
      }
    }
  }

  // ---- start: minimiser under a mild barrier weight, slacks shifted into the interior
  if (!done) {
    for (int j = lane; j < S; j += NT) {
      double d[6], rh[kRh], wv[9];
#pragma unroll
      for (int r = 0; r < 6; ++r) d[r] = 1e-2;
      legrh(j, rh);
      if constexpr (XR) ipm_foot_gdg(rw, liv, d, wv);   // the leg's block of the stage weight
      else ipm_foot_weight(rw, liv, d, rh, wv);
#pragma unroll
      for (int e = 0; e < 9; ++e) sm.W[j][e] = wv[e];
    }
    for (int e = lane; e < N * NU; e += NT) sm.rhs[e / NU][e % NU] = -sm.gr[e / NU][e % NU];
    fsync<NT>();
    stage_weights(false);
    factor();
    ++nfact;
    lsolve();
    for (int e = lane; e < N * NU; e += NT) sm.U[e / NU][e % NU] = sm.dU[e / NU][e % NU];
    fsync<NT>();
    for (int j = lane; j < S; j += NT) {
      double f[3];
      foot(j, sm.U, f);
      const double h5 = -sm.mt.ub[j];
#pragma unroll
      for (int r = 0; r < 6; ++r) {
        const bool on = (liv >> r) & 1;
        FS(j)[r] = on ? fmax(adot(r, f) - (r == 5 ? h5 : 0.0), 1.0) : 1.0;
        FL(j)[r] = on ? 1.0 : 0.0;
      }
    }
    fsync<NT>();
  }

  // ------------------------------------------------ interior point
  int it = 0;
  double ap_last = 0.0, ad_last = 0.0;   // the last step's lengths (FDS / FDL hold its direction); 0: none yet
  // sm.gr after a step: g + ap H dU, H dU = rhs - G^T D G dU per foot-step (the Newton system
  // (H + G^T D G) dU = rhs), in place of a forward simulation and adjoint per iteration
  // (round 6, tools/ipm_proto.py INCR_GRAD=1: same iterations on its 64 cases, gradients per
  // golden N = 16 robot 13.1 -> 4.4); any polish recomputes it from scratch
  bool gr_valid = false;
  while (!done && it < IPM_MAX_IT) {
    ++it;
    if (!gr_valid) gradient();
    gr_valid = false;
    // residuals rd = g - G^T lam, rp = G f - h - s; mu
    double sl = 0.0;
    for (int j = lane; j < S; j += NT) {
      double g[3], f[3];
      foot(j, sm.gr, g);
      foot(j, sm.U, f);
      const double h5 = -sm.mt.ub[j];
#pragma unroll
      for (int x = 0; x < 3; ++x) {
        double v = g[x];
#pragma unroll
        for (int r = 0; r < 6; ++r) v = fma(-FL(j)[r], rw[r][x], v);
        FRD(j)[x] = v;
      }
#pragma unroll
      for (int r = 0; r < 6; ++r) {
        const bool on = (liv >> r) & 1;
        FRP(j)[r] = on ? adot(r, f) - (r == 5 ? h5 : 0.0) - FS(j)[r] : 0.0;
        sl += on ? FS(j)[r] * FL(j)[r] : 0.0;
      }
    }
    const double mu = sgpr_d(wave_sum_d(sl)) / m_tot;
#ifdef MPCQP_IPM_DEBUG
    dbg((double)it);
    dbg(mu);
    dbg(dbg_p[0]);
    dbg(dbg_p[1]);
    dbg(dbg_p[2]);
    dbg((double)nfact);
    dbg(gscale);
    dbg(hscale);
#endif
    bool polished = false;   // a failed polish left sm.gr at its own iterate
    if (mu < IPM_POLISH_MU * gscale * hscale) {
      polished = true;
      for (int j = lane; j < S; j += NT) {
        int a = 0;
#pragma unroll
        for (int r = 0; r < 6; ++r)
          if ((liv >> r) & 1) {
            // the rows whose slack the last step shrank by a larger factor than their
            // multiplier (Tapia's indicator: lam+ / lam > s+ / s; lam > s before any step) --
            // lam > s misses the weakly active rows, whose lam is still below s at this mu
            // (tools/ipm_proto.py POLISH_RULE=tapia: 13.1 -> 10.6 factorisations per robot)
            const double s1 = FS(j)[r], l1 = FL(j)[r];
            const double s0 = s1 - ap_last * FDS(j)[r], l0 = l1 - ad_last * FDL(j)[r];
            if (ap_last > 0.0 ? l1 * s0 > s1 * l0 : l1 > s1) a |= 1 << r;
          }
        FACT(j) = a;
      }
      // U is overwritten by the polish: keep the IPM iterate
      for (int e = lane; e < N * NU; e += NT) {
        if constexpr (kMG) Sg[IpmSlot<NM>::US + e] = sm.U[e / NU][e % NU];
        else sm.us.Us[e / NU][e % NU] = sm.U[e / NU][e % NU];
      }
      fsync<NT>();
      if (polish_corrected(IPM_NCORR_IPM)) {
        done = true;
        status = MPCQP_STATUS_OK;
        break;
      }
      for (int e = lane; e < N * NU; e += NT) {
        if constexpr (kMG) sm.U[e / NU][e % NU] = Sg[IpmSlot<NM>::US + e];
        else sm.U[e / NU][e % NU] = sm.us.Us[e / NU][e % NU];
      }
      fsync<NT>();
    }
    for (int j = lane; j < S; j += NT) {
      double d[6], rh[kRh], wv[9];
#pragma unroll
      for (int r = 0; r < 6; ++r) d[r] = ((liv >> r) & 1) ? FL(j)[r] / FS(j)[r] : 0.0;
      legrh(j, rh);
      if constexpr (XR) ipm_foot_gdg(rw, liv, d, wv);
      else ipm_foot_weight(rw, liv, d, rh, wv);
#pragma unroll
      for (int e = 0; e < 9; ++e) sm.W[j][e] = wv[e];
    }
    fsync<NT>();
    stage_weights(false);
    factor();
    ++nfact;
    // Newton direction for the complementarity target: predictor (sig = 0, corr = false)
    // or corrector (target mu, the affine ds dl second-order term)
    auto newton = [&](bool corr, double target) {
      for (int e = lane; e < N * NU; e += NT) sm.rhs[e / NU][e % NU] = 0.0;
      fsync<NT>();
      for (int j = lane; j < S; j += NT) {
        double* rr = foot_ptr(j, sm.rhs);
#pragma unroll
        for (int x = 0; x < 3; ++x) {
          double v = -FRD(j)[x];
#pragma unroll
          for (int r = 0; r < 6; ++r)
            if ((liv >> r) & 1) {
              const double s_ = FS(j)[r], l_ = FL(j)[r];
              const double rc = -s_ * l_ + (corr ? target - FDS(j)[r] * FDL(j)[r] : 0.0);
              v = fma(rw[r][x], rc / s_ - (l_ / s_) * FRP(j)[r], v);
            }
          rr[x] = v;
        }
      }
      fsync<NT>();
      lsolve();
      double a1 = 1.0, a2 = 1.0;
      for (int j = lane; j < S; j += NT) {
        double d[3];
        foot(j, sm.dU, d);
#pragma unroll
        for (int r = 0; r < 6; ++r)
          if ((liv >> r) & 1) {
            const double s_ = FS(j)[r], l_ = FL(j)[r];
            const double rc = -s_ * l_ + (corr ? target - FDS(j)[r] * FDL(j)[r] : 0.0);
            const double ds = adot(r, d) + FRP(j)[r];
            const double dl = (rc - l_ * ds) / s_;
            FDS(j)[r] = ds;
            FDL(j)[r] = dl;
            if (ds < 0.0) a1 = fmin(a1, -s_ / ds);
            if (dl < 0.0) a2 = fmin(a2, -l_ / dl);
          }
      }
      return d2{sgpr_d(wave_min(a1)), sgpr_d(wave_min(a2))};
    };
    d2 al = newton(false, 0.0);
    double sa = 0.0;
    for (int j = lane; j < S; j += NT)
#pragma unroll
      for (int r = 0; r < 6; ++r)
        if ((liv >> r) & 1) sa += (FS(j)[r] + al[0] * FDS(j)[r]) * (FL(j)[r] + al[1] * FDL(j)[r]);
    const double mu_aff = sgpr_d(wave_sum_d(sa)) / m_tot;
    const double sig = mu_aff / mu;
    const double target = fmax(sig * sig * sig * mu, IPM_MU_FLOOR * gscale * hscale);
    fsync<NT>();
    al = newton(true, target);
    const double ap = fmin(1.0, IPM_TAU * al[0]), ad = fmin(1.0, IPM_TAU * al[1]);
    ap_last = ap;
    ad_last = ad;
    for (int j = lane; j < S; j += NT) {
      double d[3], rr[3];
      foot(j, sm.dU, d);
      foot(j, sm.rhs, rr);   // the corrector's right-hand side
      double* u = foot_ptr(j, sm.U);
      u[0] += ap * d[0];
      u[1] += ap * d[1];
      u[2] += ap * d[2];
      double* g = foot_ptr(j, sm.gr);
      double hd[3] = {rr[0], rr[1], rr[2]};   // H d = rhs - G^T D G d (D of this iteration)
#pragma unroll
      for (int r = 0; r < 6; ++r)
        if ((liv >> r) & 1) {
          const double w = FL(j)[r] / FS(j)[r] * adot(r, d);
          hd[0] = fma(-w, rw[r][0], hd[0]);
          hd[1] = fma(-w, rw[r][1], hd[1]);
          hd[2] = fma(-w, rw[r][2], hd[2]);
          FS(j)[r] += ap * FDS(j)[r];
          FL(j)[r] += ad * FDL(j)[r];
        }
      if (!polished) {
        g[0] = fma(ap, hd[0], g[0]);
        g[1] = fma(ap, hd[1], g[1]);
        g[2] = fma(ap, hd[2], g[2]);
      }
    }
    fsync<NT>();
    gr_valid = !polished;
  }

  // ------------------------------------------------ output (the polished optimum or the last iterate)
  bool finite = true;
  for (int e = lane; e < N * NU; e += NT) finite &= isfinite(sm.U[e / NU][e % NU]);
  if (__any(!finite)) status = MPCQP_STATUS_NONFINITE;
  if (lane < 12) u0g[(size_t)b * 12 + lane] = (float)sm.U[0][lane];
  if (wmem) {   // remember the verified set (0x80 | rows; swing foot-steps 0x80), or nothing
    const bool ok = status == MPCQP_STATUS_OK;
    unsigned char* const wb = reinterpret_cast<unsigned char*>(&sm.rhs[0][0]);   // free from here on
    for (int e = lane; e < MPCQP_WARM_BYTES; e += NT) wb[e] = ok && e < 4 * N ? 0x80 : 0;
    fsync<NT>();
    if (ok)
      for (int j = lane; j < S; j += NT) wb[4 * sm.mt.foot_t[j] + sm.mt.foot_leg[j]] = (unsigned char)(0x80 | (FACT(j) & liv));
    fsync<NT>();
    for (int e = lane; e < MPCQP_WARM_BYTES; e += NT) wmem[e] = wb[e];
  }
#ifdef MPCQP_IPM_DEBUG
  {   // the last 8 slots: cycles in gradient / factor / lsolve / total, factor T / GJ / S store / sym
    const unsigned long long tot = __builtin_amdgcn_s_memtime() - cyc_t0;
    if (lane == 0 && Ug) {
      float* dst = Ug + (size_t)b * N * NU + N * NU - 8;
      dst[0] = (float)cyc[0];
      dst[1] = (float)cyc[1];
      dst[2] = (float)cyc[2];
      dst[3] = (float)tot;
      dst[4] = (float)cyc[4];
      dst[5] = (float)cyc[5];
      dst[6] = (float)cyc[6];
      dst[7] = (float)cyc[7];
    }
  }
  Ug = nullptr;
#endif
  if (Ug)
    for (int e = lane; e < N * NU; e += NT) Ug[(size_t)b * N * NU + e] = (float)sm.U[e / NU][e % NU];
  if (lane == 0) {
    if (statusg) statusg[b] = status;
    if (itersg) itersg[b] = nfact;
  }
}
