// mpcqp.hip -- MI355X (gfx950) batched convex-MPC QP engine: kernel + C ABI.
//
// ONE WAVE (64 lanes) PER ROBOT, wave-synchronous; 4 robots per CU (LDS < 40 KB),
// so a 1024-robot batch is one wave of blocks on the 256 CUs.
//
// Register / LDS layout
//   W = H^-1 (64x64 f64) lives in VGPRs as 8x8 tiles: lane l = (tr, tc) =
//   (l >> 3, l & 7) holds W[8tr + r][8tc + c].  A sweep pivot then needs 16
//   broadcast values per lane (one LDS round trip), and a matvec ends in a DPP
//   reduce-scatter that leaves y[l] in lane l.
//   Lane i is also "variable i" (stance GRF component i), "slot i" of the active
//   set and holds constraint rows i and i+64.  (M_AA)^-1 is in LDS, row j at j*LDM.
//
// Per robot, fused in one launch (nothing but inputs and outputs touches HBM):
//   1. model      A_c, B_c as the reference rounds them to float32
//                 (mpc.py:173-192); exact discretisation: M^3 = 0 for
//                 M = [[A_c,B_c],[0,0]], so expm(M dt) = I + M dt + M^2 dt^2/2
//                 (replaces scipy expm, mpc.py:194-208); float64 from here on.
//   2. condense   A_d = I + Nm, Nm^3 = 0  =>  A^k B_d = X0 + k X1 + C(k,2) X2.
//                 Y = [X0 X1 X2]^T Q [X0 X1 X2] (36x36) on the f64 MFMA;
//                 H = 2(Su^T Qbar Su + Rbar) (mpc.py:232) restricted to stance
//                 variables = 2 sum_pq T_pq(j_a,j_b) Y_pq[c_a][c_b] + 2R with scalar
//                 Toeplitz weights T_pq; g likewise (mpc.py:233).
//   3. swing      swing GRFs are exactly 0 (ub: fz <= 0; cone rows: mu fz >=
//                 |fx|,|fy| >= 0), so n = 3 * #stance variables remain.
//   4. W = H^-1   symmetric sweep over the register tiles.
//   5. solve      Goldfarb-Idnani dual active set in range-space form with an
//                 explicit, bordered/downdated (M_AA)^-1; exact up to float64
//                 rounding; one multiplier refinement; KKT check of every row.
//
// QP = Drake branch of _solve_mpc (mpc.py:277-286):
//   min 1/2 U^T H U + g^T U  s.t.  lb <= C U <= ub,  C = kron(I_4N, cone) (mpc.py:239-260)
// generalised to a per-robot cone normal (normal = e_z reproduces mpc.py exactly).

#include <hip/hip_runtime.h>

#include <math.h>
#include <stdint.h>
#include <string.h>

#include <new>
#include <string>
#include <utility>

#include "mpcqp.h"

namespace {

constexpr int NX = 13;      // state dimension (mpc.py:26)
constexpr int NU = 12;      // input dimension (mpc.py:28)
constexpr int NV = 64;      // variables per robot = lanes
constexpr int LANES = 64;
constexpr int SMAX = NV / 3;            // 21 stance foot-steps
constexpr int kMaxN = 20;               // LDS scratch is sized for N <= 20
constexpr int kNT = kMaxN * (kMaxN + 1) / 2;
constexpr int NY = 36;                  // columns of [X0 X1 X2]
// formulation scratch offsets (doubles) inside Shared::scr
constexpr int OFF_AC = 0, OFF_NM = NX * NX, OFF_BC = 2 * NX * NX;   // model phase
constexpr int OFF_Y = 0, OFF_T = 9 * NU * NU;                        // Hessian phase
constexpr int OFF_X = OFF_T + 9 * kNT;                               // X0|X1|X2 ([p][s][c]), alive until Y
constexpr int SCR0 = OFF_X + 3 * NX * NU;                            // 3654 doubles
constexpr int LDM = LANES + 2;                                       // (M_AA)^-1 row stride (16-B rows)
constexpr int SCR = LANES * LDM;                                     // 4224 doubles
// staged inputs (floats) in the scratch tail
constexpr int IN_X0 = 0, IN_FEET = 13, IN_ROBOT = 25, IN_CONTACT = 44, IN_XREF = 44 + 4 * kMaxN;
constexpr int IN_END = IN_XREF + NX * kMaxN;
static_assert(SCR0 * 2 + IN_END <= SCR * 2, "staged inputs do not fit");
constexpr int PV = LANES + 4;
constexpr int NL_CAP = 126;             // variables of the large class (mpcqp_large.h)           // padded broadcast vector: element i at pv(i)

// i -> i + 2*(i/32): the 8 column segments {8tc..8tc+7} land on distinct bank groups
__host__ __device__ constexpr int pv(int i) { return i + 2 * (i >> 5); }

typedef double d2 __attribute__((ext_vector_type(2)));
typedef double d4 __attribute__((ext_vector_type(4)));

struct KParams {
  int N;
  int max_iter;
  double dt;
  double q[NX];
  double r[NU];
};

struct alignas(16) Shared {
  double scr[SCR];      // formulation scratch + staged inputs; then (M_AA)^-1, row j at j*LDM
  double vb[PV];        // matvec right-hand side (padded)
  double zc[2][PV];     // sweep pivot column, double-buffered (padded)
  double wv[LANES];     // w = W a_p          (gathers)
  double zv[LANES];     // z / x              (gathers)
  double rv[LANES];     // per-slot vector    (gathers)
  double gv[LANES];     // g
  double rows[6][3];    // cone rows a_r, shared by every foot of the robot
  double ii[9];         // inverse world inertia (float32-rounded)
  double x0[NX], y1[NX], y2[NX];
  double qd[NX], rd[NU];   // cost weights (kernel arguments indexed at run time would be memory loads)
  double ub[SMAX + 1];
  int foot_t[SMAX + 1], foot_leg[SMAX + 1];
  int stance_of[4 * kMaxN];
  int S;
};

// Diagnostic build only (-DMPCQP_STAMPS): per-phase s_memtime stamps written to U
// (U must then hold >= 16 floats per robot); the shipped kernel executes no stamp.
#ifdef MPCQP_STAMPS
#define STAMP(i)                                \
  do {                                          \
    __builtin_amdgcn_sched_barrier(0);          \
    stamps_[i] = __builtin_amdgcn_s_memtime();  \
    __builtin_amdgcn_sched_barrier(0);          \
  } while (0)
#else
#define STAMP(i) \
  do {           \
  } while (0)
#endif

#define MPCQP_FENCE() __builtin_amdgcn_sched_barrier(0)

// one wave per workgroup: LDS write -> read visibility needs the writes to
// land (lgkmcnt) and the compiler not to move memory operations across
#define WSYNC() __syncthreads()

__device__ __forceinline__ double f32r(double v) { return (double)(float)v; }

__device__ __forceinline__ int uni(int x) { return __builtin_amdgcn_readfirstlane(x); }

__device__ __forceinline__ double readlane_d(double v, int lane) {
  const long long b = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_readlane((int)(b & 0xffffffffll), lane);
  const int hi = __builtin_amdgcn_readlane((int)(b >> 32), lane);
  return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}

__device__ __forceinline__ double cpoly(int p, int k) {
  return p == 0 ? 1.0 : (p == 1 ? (double)k : 0.5 * (double)k * (double)(k - 1));
}

// Compile-time loop: f(std::integral_constant<int, I>{}) for I = 0..N-1.  Used where a
// register array is indexed, so no index can stay a runtime value (a runtime index
// demotes the whole array to scratch).
template <typename F, int... Is>
__device__ __forceinline__ void static_for_impl(F&& f, std::integer_sequence<int, Is...>) {
  (f(std::integral_constant<int, Is>{}), ...);
}
template <int N, typename F>
__device__ __forceinline__ void static_for(F&& f) {
  static_for_impl(f, std::make_integer_sequence<int, N>{});
}

// T table index for (d, m): d in [0,N), m in [1, N-d]
__device__ __forceinline__ int tidx(int N, int d, int m) { return d * N - (d * (d - 1)) / 2 + (m - 1); }

template <int CTRL>
__device__ __forceinline__ double dpp_d(double v) {
  const long long bits = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_update_dpp((int)bits, (int)bits, CTRL, 0xF, 0xF, false);
  const int hi = __builtin_amdgcn_update_dpp((int)(bits >> 32), (int)(bits >> 32), CTRL, 0xF, 0xF, false);
  return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}
constexpr int DPP_XOR1 = 0xB1;      // quad_perm [1,0,3,2]
constexpr int DPP_XOR2 = 0x4E;      // quad_perm [2,3,0,1]
constexpr int DPP_HMIRROR = 0x141;  // row_half_mirror: i <-> 7-i within 8 lanes
constexpr int DPP_MIRROR = 0x140;   // row_mirror: i <-> 15-i within 16 lanes

// Cross-lane min on the VALU (DPP inside 16-lane rows, then readlane of the rows)
__device__ __forceinline__ double wave_min(double v) {
  v = fmin(v, dpp_d<DPP_XOR1>(v));
  v = fmin(v, dpp_d<DPP_XOR2>(v));
  v = fmin(v, dpp_d<DPP_HMIRROR>(v));
  v = fmin(v, dpp_d<DPP_MIRROR>(v));
  return fmin(fmin(readlane_d(v, 0), readlane_d(v, 16)), fmin(readlane_d(v, 32), readlane_d(v, 48)));
}

// argmin over rows {lane} (a) and {lane + 64} (b): lowest index attaining the min
__device__ __forceinline__ int wave_argmin2(double a, double b, double& vmin) {
  vmin = wave_min(fmin(a, b));
  const unsigned long long ma = __ballot(a == vmin), mb = __ballot(b == vmin);
  return uni(ma ? __builtin_ctzll(ma) : (mb ? 64 + __builtin_ctzll(mb) : 0x7fffffff));
}

// 8 consecutive padded doubles starting at element 8k (16-B aligned)
__device__ __forceinline__ void ld8(double (&v)[8], const double* base, int k) {
  const d2* p = reinterpret_cast<const d2*>(base + pv(8 * k));
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const d2 x = p[i];
    v[2 * i] = x[0];
    v[2 * i + 1] = x[1];
  }
}

__device__ __forceinline__ void st8(double* base, int k, const double (&v)[8]) {
  d2* p = reinterpret_cast<d2*>(base + pv(8 * k));
#pragma unroll
  for (int i = 0; i < 4; ++i) p[i] = d2{v[2 * i], v[2 * i + 1]};
}

// y = W v for the tile layout.  v is read from LDS (padded); returns y[lane].
// 64 FMAs into 8 row partials, then a reduce-scatter over the 8 lanes of the
// tile row: half-mirror (keep rows 0-3 / 4-7), xor 2, xor 1 -> lane l owns row l.
__device__ __forceinline__ double tile_matvec(const double (&W)[8][8], const double* v, int tr, int tc,
                                              int lane) {
  double vs[8];
  ld8(vs, v, tc);
  MPCQP_FENCE();
  double acc[8];
#pragma unroll
  for (int r = 0; r < 8; ++r) {
    double a = 0.0;
#pragma unroll
    for (int c = 0; c < 8; ++c) a = fma(W[r][c], vs[c], a);
    acc[r] = a;
  }
  const bool hi4 = (lane & 4) != 0;
  double k4[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const double send = hi4 ? acc[k] : acc[4 + k];
    const double keep = hi4 ? acc[4 + k] : acc[k];
    k4[k] = keep + dpp_d<DPP_HMIRROR>(send);
  }
  const bool hi2 = (lane & 2) != 0;
  double k2[2];
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const double send = hi2 ? k4[k] : k4[2 + k];
    const double keep = hi2 ? k4[2 + k] : k4[k];
    k2[k] = keep + dpp_d<DPP_XOR2>(send);
  }
  const bool hi1 = (lane & 1) != 0;
  const double send = hi1 ? k2[0] : k2[1];
  const double keep = hi1 ? k2[1] : k2[0];
  (void)tr;
  return keep + dpp_d<DPP_XOR1>(send);
}

// One pivot K = 8 KT + KC of the symmetric sweep; KC compile-time so W stays in
// VGPRs, KT a runtime loop index so the code (8 pivots) stays in the I-cache.
// W_ij -= z_i z_j / d (i,j != K), W_iK = z_i/d, W_KK = -1/d; the pivot row uses
// W_Kj = z_j (symmetry): W_Kj + (1/d - 1) z_j = z_j/d.  Ends at -H^-1.
// Rows/columns >= n are identity padding: z = 0 there, they never change.
template <int KC>
__device__ __forceinline__ void sweep_pivot(double (&W)[8][8], Shared& sm, int tr, int tc, int KT, int n) {
  const int K = 8 * KT + KC;
  if (K < n) {   // wave-uniform
    double* const zc = sm.zc[KC & 1];
    if (tc == KT) {
      double col[8];
#pragma unroll
      for (int r = 0; r < 8; ++r) col[r] = W[r][KC];
      st8(zc, tr, col);
    }
    WSYNC();
    double zr[8], zi[8];
    ld8(zr, zc, tc);
    ld8(zi, zc, tr);
    const double d = zc[pv(K)];
    MPCQP_FENCE();
    const double inv = 1.0 / d;
    double beta[8];
#pragma unroll
    for (int r = 0; r < 8; ++r) beta[r] = -zi[r] * inv;
    if (tr == KT) beta[KC] = inv - 1.0;
#pragma unroll
    for (int r = 0; r < 8; ++r)
#pragma unroll
      for (int c = 0; c < 8; ++c) W[r][c] = fma(beta[r], zr[c], W[r][c]);
    if (tc == KT) {
#pragma unroll
      for (int r = 0; r < 8; ++r) W[r][KC] = zi[r] * inv;
      if (tr == KT) W[KC][KC] = -inv;
    }
  }
}

__device__ __forceinline__ void sweep_all(double (&W)[8][8], Shared& sm, int tr, int tc, int n) {
#pragma unroll 1
  for (int KT = 0; 8 * KT < n; ++KT) {
    static_for<8>([&](auto C) { sweep_pivot<decltype(C)::value>(W, sm, tr, tc, KT, n); });
  }
}

// y_lane = sum_{k < 8*nch} M[lane][k] vec[k]   (row of M in LDS, vec broadcast), b128 loads
__device__ __forceinline__ double lds_matvec(const double* Mrow, const double* vec, int nch) {
  double a0 = 0.0, a1 = 0.0, a2 = 0.0, a3 = 0.0;
  const d2* mp = reinterpret_cast<const d2*>(Mrow);
  const d2* vp = reinterpret_cast<const d2*>(vec);
  for (int c = 0; c < nch; ++c) {
    d2 m[4], v[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      m[i] = mp[4 * c + i];
      v[i] = vp[4 * c + i];
    }
    MPCQP_FENCE();
#pragma unroll
    for (int i = 0; i < 4; i += 2) {
      a0 = fma(m[i][0], v[i][0], a0);
      a1 = fma(m[i][1], v[i][1], a1);
      a2 = fma(m[i + 1][0], v[i + 1][0], a2);
      a3 = fma(m[i + 1][1], v[i + 1][1], a3);
    }
    MPCQP_FENCE();
  }
  return (a0 + a1) + (a2 + a3);
}

// M[lane][k] += c * vec[k] for k < 8*nch
__device__ __forceinline__ void lds_rank1(double* Mrow, double c, const double* vec, int nch) {
  d2* mp = reinterpret_cast<d2*>(Mrow);
  const d2* vp = reinterpret_cast<const d2*>(vec);
  for (int ch = 0; ch < nch; ++ch) {
    d2 m[4], v[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      m[i] = mp[4 * ch + i];
      v[i] = vp[4 * ch + i];
    }
    MPCQP_FENCE();
#pragma unroll
    for (int i = 0; i < 4; ++i) mp[4 * ch + i] = d2{fma(c, v[i][0], m[i][0]), fma(c, v[i][1], m[i][1])};
    MPCQP_FENCE();
  }
}

__device__ __forceinline__ void write_empty(int b, int lane, int N, int code, float* u0g, float* Ug,
                                            int* statusg, int* itersg) {
  if (lane < 12) u0g[(size_t)b * 12 + lane] = 0.f;
  if (Ug)
    for (int k = lane; k < N * 12; k += LANES) Ug[(size_t)b * N * 12 + k] = 0.f;
  if (lane == 0) {
    if (statusg) statusg[b] = code;
    if (itersg) itersg[b] = 0;
  }
}

__global__ __launch_bounds__(LANES) __attribute__((amdgpu_waves_per_eu(1, 2))) void mpcqp_kernel(
    KParams P, int B, const float* __restrict__ x0g, const float* __restrict__ xrefg,
    const float* __restrict__ contactg, const float* __restrict__ feetg, const float* __restrict__ robotg,
    float* __restrict__ u0g, float* __restrict__ Ug, int* __restrict__ statusg, int* __restrict__ itersg,
    int* __restrict__ queue) {
  __shared__ Shared sm;
  const int b = blockIdx.x;
  const int lane = threadIdx.x;
#ifdef MPCQP_STAMPS
  unsigned long long stamps_[7];
#endif
  const int N = P.N;
  if (b >= B) return;
  const int tr = lane >> 3, tc = lane & 7;
  STAMP(0);

  // ------------------------------------------ stage every input in LDS at once
  float* const in = (float*)(sm.scr + SCR0);
  {
    const float* xb = x0g + (size_t)b * NX;
    const float* fb = feetg + (size_t)b * 12;
    const float* rb = robotg + (size_t)b * MPCQP_ROBOT_STRIDE;
    const float* cb = contactg + (size_t)b * N * 4;
    const float* xrb = xrefg + (size_t)b * N * NX;
    if (lane < NX) in[IN_X0 + lane] = xb[lane];
    else if (lane < NX + 12) in[IN_FEET + lane - NX] = fb[lane - NX];
    else if (lane < NX + 12 + MPCQP_ROBOT_STRIDE) in[IN_ROBOT + lane - NX - 12] = rb[lane - NX - 12];
    for (int k = lane; k < 4 * N; k += LANES) in[IN_CONTACT + k] = cb[k];
    for (int k = lane; k < NX * N; k += LANES) in[IN_XREF + k] = xrb[k];
  }
  WSYNC();
  {
    int bad = 0;
    for (int k = lane; k < NX * N; k += LANES) bad |= !isfinite(in[IN_XREF + k]);
    if (lane < NX + 12 + 12) bad |= !isfinite(in[lane]);   // x0, feet, robot[0:12]
    if (__any(bad)) {
      write_empty(b, lane, N, MPCQP_STATUS_NONFINITE, u0g, Ug, statusg, itersg);
      return;
    }
  }
  const float* const rbs = in + IN_ROBOT;

  // ------------------------------------------------ stance list (gait table)
  int S;
  {
    const unsigned long long lt_mask = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
    const int nk = 4 * N;
    const float c0 = lane < nk ? in[IN_CONTACT + lane] : 0.f;
    const float c1 = lane + LANES < nk ? in[IN_CONTACT + lane + LANES] : 0.f;
    const bool f0 = c0 > 0.f, f1 = c1 > 0.f;
    const unsigned long long m0 = __ballot(f0), m1 = __ballot(f1);
    const int S0 = __popcll(m0);
    S = uni(S0 + __popcll(m1));
    const int i0 = __popcll(m0 & lt_mask), i1 = S0 + __popcll(m1 & lt_mask);
    const double fzmax = (double)rbs[8];
    if (lane < nk) sm.stance_of[lane] = f0 ? i0 : -1;
    if (lane + LANES < nk) sm.stance_of[lane + LANES] = f1 ? i1 : -1;
    if (f0 && i0 < SMAX) {
      sm.foot_t[i0] = lane / 4;
      sm.foot_leg[i0] = lane % 4;
      sm.ub[i0] = (double)c0 * fzmax;   // ub = contact * fz_max (mpc.py:257)
    }
    if (f1 && i1 < SMAX) {
      sm.foot_t[i1] = (lane + LANES) / 4;
      sm.foot_leg[i1] = (lane + LANES) % 4;
      sm.ub[i1] = (double)c1 * fzmax;
    }
  }
  const int n = 3 * S, m = 6 * S;
  if (n > NV) {
    if (queue && n <= NL_CAP) {   // the 8-wave class (mpcqp_kernel_large) takes it
      if (lane == 0) queue[4 + atomicAdd(&queue[0], 1)] = b;
      return;
    }
    write_empty(b, lane, N, MPCQP_STATUS_TOO_LARGE, u0g, Ug, statusg, itersg);
    return;
  }

  double* const scr = sm.scr;
  double* const Ac = scr + OFF_AC;
  double* const Nm = scr + OFF_NM;
  double* const Bc = scr + OFF_BC;
  double* const X = scr + OFF_X;   // X_p[s][c] at X + p*NX*NU + s*NU + c
  for (int k = lane; k < NX * NX + NX * NU; k += LANES) (k < NX * NX ? Ac[k] : Bc[k - NX * NX]) = 0.0;
  if (lane < NX) sm.x0[lane] = (double)in[IN_X0 + lane];
  if (lane < NX) sm.qd[lane] = P.q[lane];
  if (lane < NU) sm.rd[lane] = P.r[lane];

  // ------------------------------------------------ 1. model (mpc.py:173-192)
  // Reference dtypes: Rz float32 of float64 cos/sin; I_w = Rz I Rz^T float32;
  // inv(I_w) float32; inv(I_w) @ skew(r) float64 rounded to float32; I/m float32.
  {
    const double yaw = (double)in[IN_X0 + 2];
    const double c = f32r(cos(yaw)), s = f32r(sin(yaw));
    // lane k < 9: entry (i, j) of T1 = Rz I_B, then of I_w = T1 Rz^T (float32 each)
    const int i = lane / 3, j = lane % 3;
    auto rz = [&](int a, int bb) -> double {
      return a == 2 ? (bb == 2 ? 1.0 : 0.0) : (bb == 2 ? 0.0 : (a == bb ? c : (a == 0 ? -s : s)));
    };
    auto ib = [&](int a, int bb) -> double {
      const int lo = a < bb ? a : bb, hi = a < bb ? bb : a;
      const int idx = lo == 0 ? hi : (lo == 1 ? 2 + hi : 5);   // ixx ixy ixz iyy iyz izz
      return (double)rbs[1 + idx];
    };
    double t1 = 0.0, iw = 0.0;
    if (lane < 9) {
      t1 = f32r(rz(i, 0) * ib(0, j) + rz(i, 1) * ib(1, j) + rz(i, 2) * ib(2, j));
      sm.ii[lane] = t1;
    }
    WSYNC();
    if (lane < 9) iw = f32r(sm.ii[3 * i] * rz(j, 0) + sm.ii[3 * i + 1] * rz(j, 1) + sm.ii[3 * i + 2] * rz(j, 2));
    WSYNC();
    if (lane < 9) sm.ii[lane] = iw;
    WSYNC();
    if (lane < 9) {   // 3x3 inverse by adjugate (float64), stored float32 like np.linalg.inv
      const double* I = sm.ii;
      const int r1 = (j + 1) % 3, r2 = (j + 2) % 3, c1 = (i + 1) % 3, c2 = (i + 2) % 3;
      const double cof = I[r1 * 3 + c1] * I[r2 * 3 + c2] - I[r1 * 3 + c2] * I[r2 * 3 + c1];   // adj(I)[i][j]
      const double det = I[0] * (I[4] * I[8] - I[5] * I[7]) - I[1] * (I[3] * I[8] - I[5] * I[6]) +
                         I[2] * (I[3] * I[7] - I[4] * I[6]);
      iw = f32r(cof / det);
    }
    WSYNC();
    if (lane < 9) sm.ii[lane] = iw;
    // A_c (mpc.py:184-186)
    if (lane < 9) Ac[i * NX + 6 + j] = rz(j, i);       // A_c[0:3,6:9] = Rz^T
    if (lane < 3) Ac[(3 + lane) * NX + 9 + lane] = 1.0;   // A_c[3:6,9:12] = I
    if (lane == 0) Ac[11 * NX + 12] = 1.0;               // A_c[11,12] = 1
    // friction-cone rows in the (t1, t2, n) frame (mpc.py:239-245 for n = e_z)
    if (lane < 18) {
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
      const int rr = lane / 3, k = lane % 3;
      const double nk = k == 0 ? nx : (k == 1 ? ny : nz);
      const double t1k = k == 0 ? t1x : (k == 1 ? t1y : t1z);
      const double t2k = k == 0 ? t2x : (k == 1 ? t2y : t2z);
      const double val = rr == 0 ? t1k + mu * nk
                       : rr == 1 ? -t1k + mu * nk
                       : rr == 2 ? t2k + mu * nk
                       : rr == 3 ? -t2k + mu * nk
                       : rr == 4 ? nk : -nk;
      sm.rows[rr][k] = val;
    }
  }
  WSYNC();
  // B_c (mpc.py:188-190): lanes 0..35 the skew blocks, 36..47 the 1/m diagonal
  if (lane < 36) {
    const int leg = lane / 9, i = (lane % 9) / 3, j = lane % 3;
    const float* fb = in + IN_FEET;
    const double rx = fb[3 * leg], ry = fb[3 * leg + 1], rz = fb[3 * leg + 2];
    const double sk0 = (j == 0) ? 0.0 : (j == 1 ? -rz : ry);   // column j of [r]x
    const double sk1 = (j == 0) ? rz : (j == 1 ? 0.0 : -rx);
    const double sk2 = (j == 0) ? -ry : (j == 1 ? rx : 0.0);
    Bc[(6 + i) * NU + 3 * leg + j] = f32r(sm.ii[3 * i] * sk0 + sm.ii[3 * i + 1] * sk1 + sm.ii[3 * i + 2] * sk2);
  } else if (lane < 48) {
    const int leg = (lane - 36) / 3, i = (lane - 36) % 3;
    Bc[(9 + i) * NU + 3 * leg + i] = f32r(1.0 / (double)rbs[0]);
  }
  WSYNC();

  // -------------------------------- 2. exact discretisation (mpc.py:194-208)
  const double dt = P.dt, hdt2 = 0.5 * P.dt * P.dt;
  for (int k = lane; k < NX * NX + NX * NU; k += LANES) {
    if (k < NX * NX) {   // Nm = A_c dt + A_c^2 dt^2/2
      const int i = k / NX, j = k % NX;
      double a2 = 0.0;
      for (int l = 0; l < NX; ++l) a2 = fma(Ac[i * NX + l], Ac[l * NX + j], a2);
      Nm[k] = Ac[k] * dt + a2 * hdt2;
    } else {             // X0 = B_d = B_c dt + A_c B_c dt^2/2
      const int kk = k - NX * NX, i = kk / NU, j = kk % NU;
      double ab = 0.0;
      for (int l = 0; l < NX; ++l) ab = fma(Ac[i * NX + l], Bc[l * NU + j], ab);
      X[kk] = Bc[kk] * dt + ab * hdt2;
    }
  }
  WSYNC();
  for (int pw = 1; pw < 3; ++pw) {   // X_pw = Nm X_{pw-1};  y_pw = Nm y_{pw-1}  (y0 = x0)
    for (int k = lane; k < NX * NU + NX; k += LANES) {
      if (k < NX * NU) {
        const int i = k / NU, j = k % NU;
        double a = 0.0;
        for (int l = 0; l < NX; ++l) a = fma(Nm[i * NX + l], X[(pw - 1) * NX * NU + l * NU + j], a);
        X[pw * NX * NU + k] = a;
      } else {
        const int i = k - NX * NU;
        const double* yp = (pw == 1) ? sm.x0 : sm.y1;
        double a = 0.0;
        for (int l = 0; l < NX; ++l) a = fma(Nm[i * NX + l], yp[l], a);
        ((pw == 1) ? sm.y1 : sm.y2)[i] = a;
      }
    }
    WSYNC();
  }
  STAMP(1);

  // -------------------------------------- 3. condensed cost (mpc.py:211-235)
  {
    double* const e = scr;            // e_t = A^{t+1} x0 - xref_t   (Sx x0 - Xref)
    double* const zp = scr + N * NX;  // zp[p][t][c] = sum_s X_p[s][c] Q_s e_t[s]
    for (int k = lane; k < N * NX; k += LANES) {
      const int t = k / NX, s = k % NX;
      const double kk = (double)(t + 1);
      e[k] = sm.x0[s] + kk * sm.y1[s] + 0.5 * kk * (kk - 1.0) * sm.y2[s] - (double)in[IN_XREF + k];
    }
    WSYNC();
    for (int k = lane; k < 3 * N * NU; k += LANES) {
      const int p = k / (N * NU), rem = k % (N * NU), t = rem / NU, c = rem % NU;
      double a = 0.0;
      for (int s = 0; s < NX; ++s) a = fma(X[p * NX * NU + s * NU + c], P.q[s] * e[t * NX + s], a);
      zp[k] = a;
    }
    WSYNC();
    double gl = 0.0;   // g[a] = 2 sum_p sum_{t >= j_a} c_p(t - j_a) zp[p][t][c_a]
    if (lane < n) {
      const int sf = lane / 3;
      const int ja = sm.foot_t[sf], ca = 3 * sm.foot_leg[sf] + lane % 3;
      for (int t = ja; t < N; ++t) {
        const int k = t - ja;
        gl += zp[t * NU + ca] + (double)k * zp[(N + t) * NU + ca] +
              0.5 * (double)k * (double)(k - 1) * zp[(2 * N + t) * NU + ca];
      }
      gl *= 2.0;
    }
    sm.gv[lane] = gl;
    WSYNC();
  }
  double* const Y = scr + OFF_Y;
  double* const T = scr + OFF_T;
  const int nT = N * (N + 1) / 2;
  {
    // Y = Xc^T diag(Q) Xc with Xc = [X0 X1 X2] (13 x 36), on the f64 MFMA:
    // v_mfma_f64_16x16x4 -- A[i][k] in lane (i + 16k), B[k][j] in lane (j + 16k),
    // D[row][col] with col = lane & 15, row = (lane >> 4) + 4 reg.  Upper tiles
    // (I <= J) only; each result is written to Y_pq[c][c2] and its transpose.
    const int li = lane & 15, lk = lane >> 4;
#pragma unroll
    for (int I = 0; I < 3; ++I) {
#pragma unroll
      for (int J = I; J < 3; ++J) {
        d4 acc = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
        for (int ks = 0; ks < 4; ++ks) {
          const int s = 4 * ks + lk;
          const int ja = 16 * I + li, jb = 16 * J + li;
          double a = 0.0, bq = 0.0;
          if (s < NX && ja < NY) a = X[(ja / NU) * NX * NU + s * NU + ja % NU];
          if (s < NX && jb < NY) bq = sm.qd[s] * X[(jb / NU) * NX * NU + s * NU + jb % NU];
          acc = __builtin_amdgcn_mfma_f64_16x16x4f64(a, bq, acc, 0, 0, 0);
        }
#pragma unroll
        for (int rg = 0; rg < 4; ++rg) {
          const int j1 = 16 * I + lk + 4 * rg, j2 = 16 * J + li;
          if (j1 < NY && j2 < NY) {
            const int p = j1 / NU, c = j1 % NU, q = j2 / NU, c2 = j2 % NU;
            Y[(3 * p + q) * NU * NU + c * NU + c2] = acc[rg];
            Y[(3 * q + p) * NU * NU + c2 * NU + c] = acc[rg];
          }
        }
      }
    }
  }
  for (int k = lane; k < 9 * N; k += LANES) {   // T_pq(d, m) = sum_{s<m} c_p(s+d) c_q(s)
    const int pq = k / N, d = k % N;
    const int p = pq / 3, q = pq % 3;
    double acc = 0.0;
    for (int mm = 1; mm <= N - d; ++mm) {
      acc += cpoly(p, mm - 1 + d) * cpoly(q, mm - 1);
      T[pq * nT + tidx(N, d, mm)] = acc;
    }
  }
  WSYNC();
  STAMP(2);

  // H tile (rows 8tr.., cols 8tc..) into registers; rows/cols >= n are identity padding
  double W[8][8];
  {
    // one runtime loop over the tile rows (compact code: the H build runs once per
    // robot, so its instructions would otherwise stream through the I-cache once)
    int cj[8], cc[8];
    static_for<8>([&](auto C) {
      constexpr int c = decltype(C)::value;
      const int col = 8 * tc + c;
      const int sb = col < n ? col / 3 : 0;
      cj[c] = sm.foot_t[sb];
      cc[c] = 3 * sm.foot_leg[sb] + col % 3;
    });
#pragma unroll
    for (int r = 0; r < 8; ++r)
#pragma unroll
      for (int c = 0; c < 8; ++c) W[r][c] = 0.0;
#pragma unroll 1
    for (int r = 0; r < 8; ++r) {
      const int row = 8 * tr + r;
      const bool rowv = row < n;
      const int sa = rowv ? row / 3 : 0;
      const int ja = sm.foot_t[sa];
      const int ca = 3 * sm.foot_leg[sa] + row % 3;
      const double r2 = 2.0 * sm.rd[rowv ? ca : 0];
      double h[8];
      static_for<8>([&](auto Cc) {
        constexpr int c = decltype(Cc)::value;
        const int col = 8 * tc + c;
        const bool le = ja <= cj[c];
        const int ti = le ? tidx(N, cj[c] - ja, N - cj[c]) : tidx(N, ja - cj[c], N - ja);
        double acc = 0.0;
#pragma unroll
        for (int pq = 0; pq < 9; ++pq) {
          const int p = pq / 3, q = pq % 3;
          acc = fma(T[(le ? pq : q * 3 + p) * nT + ti], Y[pq * NU * NU + ca * NU + cc[c]], acc);
        }
        const double hv = 2.0 * acc + (row == col ? r2 : 0.0);
        h[c] = (rowv && col < n) ? hv : (row == col ? 1.0 : 0.0);
      });
      static_for<8>([&](auto Rr) {
        constexpr int rr = decltype(Rr)::value;
#pragma unroll
        for (int c = 0; c < 8; ++c) W[rr][c] = (rr == r) ? h[c] : W[rr][c];
      });
    }
  }
  STAMP(3);

  // ------------------------------------------------ 4. W = H^-1 (symmetric sweep)
  sweep_all(W, sm, tr, tc, n);
#pragma unroll
  for (int r = 0; r < 8; ++r)
#pragma unroll
    for (int c = 0; c < 8; ++c) W[r][c] = -W[r][c];
  STAMP(4);

  // Per-lane constraint bookkeeping, kept as indices (cone coefficients re-read
  // from LDS):  constraint lanes: rows c = lane, lane + 64 ;  variable lanes: i ->
  // foot i/3, axis i%3, slot of each of the foot's 6 rows ;  slot lanes: the row
  // held in slot j.
  const bool clo_ok = lane < m, chi_ok = lane + LANES < m;
  const int clo = clo_ok ? lane : 0, chi = chi_ok ? lane + LANES : 0;
  const int vf = lane / 3, vax = lane % 3;
  const bool vok = lane < n;
  int fslot[6];
#pragma unroll
  for (int rr = 0; rr < 6; ++rr) fslot[rr] = -1;
  int sl_c = 0;
  auto cdot = [&](const double* v, int c, bool bound) -> double {   // a_c . v(foot c) (+ bound term)
    const int f = c / 6, rr = c % 6;
    double d = sm.rows[rr][0] * v[3 * f] + sm.rows[rr][1] * v[3 * f + 1] + sm.rows[rr][2] * v[3 * f + 2];
    if (bound && rr == 5) d += sm.ub[f];   // s_c = a_c . x + contact * fz_max on row 5
    return d;
  };

  // unconstrained minimiser x = -W g ; constraint values s = A x - b
  sm.vb[pv(lane)] = sm.gv[lane];
  WSYNC();
  sm.zv[lane] = -tile_matvec(W, sm.vb, tr, tc, lane);
  WSYNC();
  double s_lo = clo_ok ? cdot(sm.zv, clo, true) : INFINITY;
  double s_hi = chi_ok ? cdot(sm.zv, chi, true) : INFINITY;

  // ------------------------- 5. Goldfarb-Idnani dual active set (range space)
  // (M_AA)^-1 over active-set slots in LDS (scratch is dead now); free rows/cols are 0
  double* const Mrow = scr + lane * LDM;
  {
    d2* mr = reinterpret_cast<d2*>(Mrow);
#pragma unroll
    for (int k = 0; k < LANES / 2; ++k) mr[k] = d2{0.0, 0.0};
  }
  double u = 0.0;               // multiplier of slot `lane`
  unsigned long long occ = 0;   // occupied slots (wave-uniform)
  const int max_iter = P.max_iter > 0 ? P.max_iter : 8 * NV + 64;
  const double tol = 1e-9;
  int it = 0;
  int status = MPCQP_STATUS_OK;
  WSYNC();
  while (true) {
    double bv;
    const int p = wave_argmin2(s_lo, s_hi, bv);   // most violated row
    if (!(bv < -tol)) break;
    const int fp = p / 6, rp = p % 6;
    const double ap_l = (vok && vf == fp) ? sm.rows[rp][vax] : 0.0;   // a_p on variable lanes
    sm.vb[pv(lane)] = ap_l;
    WSYNC();
    const double wl = tile_matvec(W, sm.vb, tr, tc, lane);   // w = W a_p
    sm.wv[lane] = wl;
    WSYNC();
    const double apw = cdot(sm.wv, p, false);
    double up = 0.0;
    bool added = false;
    while (!added) {
      if (++it > max_iter) {
        status = MPCQP_STATUS_MAX_ITER;
        break;
      }
      const bool mine = (occ >> lane) & 1ull;
      const int nch = uni((64 - __clzll(occ) + 1 + 7) / 8);   // 8-slot chunks in use (+ next free)
      // mp_j = a_{A_j} . w(foot_j) ;  r = Minv mp
      sm.rv[lane] = mine ? cdot(sm.wv, sl_c, false) : 0.0;
      WSYNC();
      double r = lds_matvec(Mrow, sm.rv, nch);
      if (!mine) r = 0.0;
      WSYNC();
      sm.rv[lane] = r;
      WSYNC();
      // v = a_p - sum_j r_j a_{A_j} on the variable lanes (per-foot slot cache)
      double vl = ap_l;
#pragma unroll
      for (int rr = 0; rr < 6; ++rr)
        if (fslot[rr] >= 0) vl -= sm.rv[fslot[rr]] * sm.rows[rr][vax];
      sm.vb[pv(lane)] = vok ? vl : 0.0;
      WSYNC();
      sm.zv[lane] = tile_matvec(W, sm.vb, tr, tc, lane);   // primal direction z = W v
      WSYNC();
      const double zs_lo = clo_ok ? cdot(sm.zv, clo, false) : 0.0;
      const double zs_hi = chi_ok ? cdot(sm.zv, chi, false) : 0.0;
      // dual step bound t1 (smallest u_j / r_j over r_j > 0), primal step t2
      double t1;
      const int l = wave_argmin2((mine && r > 0.0) ? u / r : INFINITY, INFINITY, t1);
      const double zsp = readlane_d(p < LANES ? zs_lo : zs_hi, p & (LANES - 1));
      const double sp = readlane_d(p < LANES ? s_lo : s_hi, p & (LANES - 1));
      double t2 = INFINITY;
      if (zsp > 1e-12 * apw) t2 = -sp / zsp;
      const bool add = t2 <= t1;
      const double tstep = add ? t2 : t1;
      if (!(tstep < INFINITY)) {
        status = MPCQP_STATUS_INFEASIBLE;
        break;
      }
      if (mine) u -= tstep * r;
      s_lo += tstep * zs_lo;
      s_hi += tstep * zs_hi;
      up += tstep;
      if (add) {
        // border (M_AA)^-1 with slot q: sigma = zs_p (Schur complement)
        const int q = uni(__builtin_ctzll(~occ));
        const double is = 1.0 / zsp;
        const double ci = (lane == q) ? -is : r * is;   // row q was zero: becomes -r^T / sigma
        lds_rank1(Mrow, ci, sm.rv, nch);
        Mrow[q] = (lane == q) ? is : -r * is;           // column q (own row: no cross-lane hazard)
        if (lane == q) {
          u = up;
          sl_c = p;
        }
        if (lane == (p & (LANES - 1))) {
          if (p < LANES) s_lo = 0.0;
          else s_hi = 0.0;
        }
        if (vf == fp) {
#pragma unroll
          for (int rr = 0; rr < 6; ++rr)
            if (rr == rp) fslot[rr] = q;
        }
        occ |= 1ull << q;
        added = true;
      } else {
        // drop slot l: Minv -= Minv[:,l] Minv[l,:] / Minv[l][l], clear row/col l
        const double col = Mrow[l];
        sm.vb[lane] = col;   // column l == row l (symmetry), unpadded here
        WSYNC();
        const double ill = 1.0 / sm.vb[l];
        lds_rank1(Mrow, -col * ill, sm.vb, nch);
        Mrow[l] = 0.0;     // column l
        WSYNC();
        scr[l * LDM + lane] = 0.0;   // row l
        const int cdrop = uni(__builtin_amdgcn_readlane(sl_c, l));
        if (vf == cdrop / 6) {
#pragma unroll
          for (int rr = 0; rr < 6; ++rr)
            if (rr == cdrop % 6) fslot[rr] = -1;
        }
        if (lane == l) u = 0.0;
        occ &= ~(1ull << l);
      }
      WSYNC();
    }
    if (status != MPCQP_STATUS_OK) break;
  }
  WSYNC();
  STAMP(5);

  // ------------------------------- 6. refinement, final x, KKT verification
  for (int pass = 0; pass < 2; ++pass) {
    // x = W (A_A^T u - g)
    const bool mine = (occ >> lane) & 1ull;
    sm.rv[lane] = mine ? u : 0.0;
    WSYNC();
    double vl = -sm.gv[lane];
#pragma unroll
    for (int rr = 0; rr < 6; ++rr)
      if (fslot[rr] >= 0) vl += sm.rv[fslot[rr]] * sm.rows[rr][vax];
    sm.vb[pv(lane)] = vok ? vl : 0.0;
    WSYNC();
    sm.zv[lane] = tile_matvec(W, sm.vb, tr, tc, lane);
    WSYNC();
    if (pass == 1) break;
    // u -= Minv (A_A x - b_A): pull the active rows back onto their bounds
    sm.rv[lane] = mine ? cdot(sm.zv, sl_c, true) : 0.0;
    WSYNC();
    const double du = lds_matvec(Mrow, sm.rv, LANES / 8);
    if (mine) u -= du;
    WSYNC();
  }
  {
    const double vlo = cdot(sm.zv, clo, true);
    const double vhi = cdot(sm.zv, chi, true);
    int bad = (clo_ok && (vlo < -1e-6 || !isfinite(vlo))) || (chi_ok && (vhi < -1e-6 || !isfinite(vhi)));
    if ((occ >> lane) & 1ull) bad |= (u < -1e-9);
    if (__any(bad) && status == MPCQP_STATUS_OK) status = MPCQP_STATUS_MAX_ITER;
  }
  STAMP(6);

  // ---------------------------------------------------------------- output
#ifdef MPCQP_STAMPS
  // stamps are held in SGPRs until here so the diagnostic build keeps the
  // shipped kernel's register allocation
  if (lane == 0 && Ug) {
    unsigned long long* dst = (unsigned long long*)(Ug + (size_t)b * N * 12);
    for (int i = 0; i < 7; ++i) dst[i] = stamps_[i];
  }
  Ug = nullptr;
#endif
  if (lane < 12) {
    const int sidx = sm.stance_of[lane / 3];
    u0g[(size_t)b * 12 + lane] = sidx >= 0 ? (float)sm.zv[3 * sidx + lane % 3] : 0.f;
  }
  if (Ug) {
    for (int k = lane; k < N * 12; k += LANES) {
      const int sidx = sm.stance_of[k / 3];
      Ug[(size_t)b * N * 12 + k] = sidx >= 0 ? (float)sm.zv[3 * sidx + k % 3] : 0.f;
    }
  }
  if (lane == 0) {
    if (statusg) statusg[b] = status;
    if (itersg) itersg[b] = it;
  }
}

#include "mpcqp_large.h"
static_assert(NL - 2 == NL_CAP, "large-class capacity");

}  // namespace

// ============================================================== C ABI
struct mpcqp_ctx {
  mpcqp_params params;
  int device;
  int stance_hint;
  int ncu;
  int qcap;           // robots the device queue can hold
  int* queue;         // [count, next, exited, pad, robots...] for the large class
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
  ctx->queue = nullptr;
  ctx->qcap = 0;
  ctx->ncu = 0;
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, device) == hipSuccess) ctx->ncu = prop.multiProcessorCount;
  if (ctx->ncu <= 0) ctx->ncu = 256;
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
  // robots with more than 64 stance variables are queued for the 8-wave class,
  // unless the caller promised (stance hint) that none exceeds one wave
  const bool large = !(ctx->stance_hint > 0 && 3 * ctx->stance_hint <= NV);
  if (large && batch > ctx->qcap) {
    if (ctx->queue) (void)hipFree(ctx->queue);
    ctx->queue = nullptr;
    ctx->qcap = 0;
    if (hipMalloc(&ctx->queue, sizeof(int) * (4 + (size_t)batch)) != hipSuccess)
      return set_err(ctx, MPCQP_ERR_ALLOC, "queue allocation failed");
    if (hipMemset(ctx->queue, 0, sizeof(int) * 4) != hipSuccess)
      return set_err(ctx, MPCQP_ERR_HIP, "queue init failed");
    ctx->qcap = batch;
  }
  int* q = large ? ctx->queue : nullptr;
  hipLaunchKernelGGL(mpcqp_kernel, dim3(batch), dim3(LANES), 0, st, kp, (int)batch, x0, xref, contact, feet,
                     robot, u0, U, (int*)status, (int*)iters, q);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return set_err(ctx, MPCQP_ERR_HIP, std::string("launch: ") + hipGetErrorString(e));
  if (large) {
    hipLaunchKernelGGL(mpcqp_kernel_large, dim3(batch), dim3(LT), 0, st, kp, x0, xref, contact, feet, robot, u0, U,
                       (int*)status, (int*)iters, q);
    e = hipGetLastError();
    if (e != hipSuccess) return set_err(ctx, MPCQP_ERR_HIP, std::string("launch (large): ") + hipGetErrorString(e));
  }
  return MPCQP_OK;
}

int mpcqp_destroy(mpcqp_ctx* ctx) {
  if (ctx && ctx->queue) (void)hipFree(ctx->queue);
  delete ctx;
  return MPCQP_OK;
}

const char* mpcqp_last_error(const mpcqp_ctx* ctx) { return ctx ? ctx->err.c_str() : "null context"; }

}  // extern "C"
