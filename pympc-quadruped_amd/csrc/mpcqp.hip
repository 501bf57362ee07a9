// mpcqp.hip -- MI355X (gfx950) batched convex-MPC QP engine: kernel + C ABI.
//
// ONE WAVE (64 lanes) PER ROBOT, wave-synchronous, register-resident:
//   lane i  <->  free variable i (a stance GRF component), n <= 64
//   lane l  <->  constraint rows l and l+64, m = 6 * #stance <= 126
//   lane j  <->  active-set slot j
// Per lane: row i of W = H^-1 (64 f64) and row j of M_AA^-1 (64 f64) in VGPRs.
// LDS (~38 KB) holds only formulation scratch and the broadcast vectors, so
// four robots share a CU and a 1024-robot batch runs in one wave of blocks.
//
// Per robot, fused in one launch (nothing but inputs and outputs touches HBM):
//   1. model      A_c, B_c as the reference rounds them to float32
//                 (mpc.py:173-192); exact discretisation: M^3 = 0 for
//                 M = [[A_c,B_c],[0,0]], so expm(M dt) = I + M dt + M^2 dt^2/2
//                 (replaces scipy expm, mpc.py:194-208); float64 from here on.
//   2. condense   A_d = I + Nm, Nm^3 = 0  =>  A^k B_d = X0 + k X1 + C(k,2) X2.
//                 H = 2(Su^T Qbar Su + Rbar) (mpc.py:232) restricted to stance
//                 variables = 2 sum_pq T_pq(j_a,j_b) Y_pq[c_a][c_b] + 2R,
//                 Y_pq = X_p^T Q X_q, T_pq scalar Toeplitz weights; g likewise
//                 (mpc.py:233).
//   3. swing      swing GRFs are exactly 0 (ub: fz <= 0; cone rows: mu fz >=
//                 |fx|,|fy| >= 0), so n = 3 * #stance variables remain.
//   4. W = H^-1   symmetric sweep, register-resident.
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
constexpr int MC = 2 * LANES;           // constraint slots (6 * SMAX = 126 used)
constexpr int kMaxN = 20;               // LDS scratch is sized for N <= 20
constexpr int kNT = kMaxN * (kMaxN + 1) / 2;
// formulation scratch offsets (doubles) inside Shared::scr
constexpr int OFF_AC = 0, OFF_NM = NX * NX, OFF_BC = 2 * NX * NX;   // model phase
constexpr int OFF_II = 2 * NX * NX + NX * NU;                        // 3x3 inverse inertia
constexpr int OFF_Y = 0, OFF_T = 9 * NU * NU;                        // Hessian phase
constexpr int OFF_X = OFF_T + 9 * kNT;                               // X0|X1|X2, alive to the end
constexpr int SCR0 = OFF_X + 3 * NX * NU;                            // 3654 doubles
constexpr int LDM = LANES + 2;                                       // Minv row stride: 16-B rows, b128 conflict-free
constexpr int SCR = (SCR0 > LANES * LDM) ? SCR0 : LANES * LDM;       // scratch, then (M_AA)^-1

struct KParams {
  int N;
  int max_iter;
  double dt;
  double q[NX];
  double r[NU];
};

struct Shared {
  double scr[SCR];    // formulation scratch; after H is in registers: (M_AA)^-1, row j at j*LDM
  double vb[LANES];   // broadcast vector for matvecs
  double wv[LANES];   // w = W a_p        (gathers by constraint lanes)
  double zv[LANES];   // z / x            (gathers by constraint lanes)
  double rv[LANES];   // r per slot       (gathers by variable lanes)
  double gv[LANES];   // g
  int foot_t[SMAX + 1], foot_leg[SMAX + 1];
  double foot_ub[SMAX + 1];
  int stance_of[4 * kMaxN];
  double rows[6][3];  // cone rows a_r, shared by every foot of the robot
  double x0[NX], y1[NX], y2[NX];
};

// Diagnostic build only (-DMPCQP_STAMPS): per-phase s_memtime stamps written to U
// (U must then hold >= 16 floats per robot); the shipped kernel executes no stamp.
#ifdef MPCQP_STAMPS
#define STAMP(i)                                                                          \
  do {                                                                                    \
    __builtin_amdgcn_sched_barrier(0);                                                    \
    const unsigned long long _t = __builtin_amdgcn_s_memtime();                           \
    if (lane == 0 && Ug) ((unsigned long long*)(Ug + (size_t)b * N * 12))[i] = _t;       \
    __builtin_amdgcn_sched_barrier(0);                                                    \
  } while (0)
#else
#define STAMP(i) \
  do {           \
  } while (0)
#endif

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

// T table index for (d, m): d in [0,N), m in [1, N-d]
__device__ __forceinline__ int tidx(int N, int d, int m) { return d * N - (d * (d - 1)) / 2 + (m - 1); }

// Cross-lane min on the VALU: DPP butterflies inside each 16-lane row (xor 1,
// xor 2, half-row mirror, row mirror), then the four row results via readlane.
// No LDS round trip (ds_bpermute) on the active-set critical path.
template <int CTRL>
__device__ __forceinline__ double dpp_d(double v) {
  const long long bits = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_update_dpp((int)bits, (int)bits, CTRL, 0xF, 0xF, false);
  const int hi = __builtin_amdgcn_update_dpp((int)(bits >> 32), (int)(bits >> 32), CTRL, 0xF, 0xF, false);
  return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}

__device__ __forceinline__ double wave_min(double v) {
  v = fmin(v, dpp_d<0xB1>(v));    // quad_perm [1,0,3,2]
  v = fmin(v, dpp_d<0x4E>(v));    // quad_perm [2,3,0,1]
  v = fmin(v, dpp_d<0x141>(v));   // row_half_mirror
  v = fmin(v, dpp_d<0x140>(v));   // row_mirror
  return fmin(fmin(readlane_d(v, 0), readlane_d(v, 16)), fmin(readlane_d(v, 32), readlane_d(v, 48)));
}

// argmin over rows {lane} (a) and {lane + 64} (b): (value, lowest index), wave-uniform
__device__ __forceinline__ int wave_argmin2(double a, double b, double& vmin) {
  vmin = wave_min(fmin(a, b));
  const unsigned long long ma = __ballot(a == vmin), mb = __ballot(b == vmin);
  return uni(ma ? __builtin_ctzll(ma) : (mb ? 64 + __builtin_ctzll(mb) : 0x7fffffff));
}

#define MPCQP_R8(M, b) M(b + 0) M(b + 1) M(b + 2) M(b + 3) M(b + 4) M(b + 5) M(b + 6) M(b + 7)
#define MPCQP_R64(M) \
  MPCQP_R8(M, 0) MPCQP_R8(M, 8) MPCQP_R8(M, 16) MPCQP_R8(M, 24) MPCQP_R8(M, 32) MPCQP_R8(M, 40) MPCQP_R8(M, 48) MPCQP_R8(M, 56)

// LDS traffic is software-pipelined in chunks of CH doubles: every load of a
// chunk is issued (sched_barrier fences) before the FMAs that consume the
// previous chunk, so a wave alone on its SIMD pays one LDS latency per chunk
// instead of one per load.
constexpr int CH = 8;
#define MPCQP_FENCE() __builtin_amdgcn_sched_barrier(0)

// y_lane = sum_j A[lane][j] * vec[j]   (A in VGPRs, vec broadcast from LDS)
__device__ __forceinline__ double matvec(const double (&A)[LANES], const double* vec) {
  double a0 = 0.0, a1 = 0.0, a2 = 0.0, a3 = 0.0;
#pragma unroll
  for (int c = 0; c < LANES; c += CH) {
    double v[CH];
#pragma unroll
    for (int i = 0; i < CH; ++i) v[i] = vec[c + i];
    MPCQP_FENCE();
#pragma unroll
    for (int i = 0; i < CH; i += 4) {
      a0 = fma(A[c + i], v[i], a0);
      a1 = fma(A[c + i + 1], v[i + 1], a1);
      a2 = fma(A[c + i + 2], v[i + 2], a2);
      a3 = fma(A[c + i + 3], v[i + 3], a3);
    }
    MPCQP_FENCE();
  }
  return (a0 + a1) + (a2 + a3);
}

// y_lane = sum_{k < 16*nch} M[lane][k] vec[k]   (row of M in LDS, vec broadcast)
__device__ __forceinline__ double lds_matvec(const double* Mrow, const double* vec, int nch) {
  double a0 = 0.0, a1 = 0.0, a2 = 0.0, a3 = 0.0;
  for (int c = 0; c < nch; ++c) {
    double mv[CH], vv[CH];
#pragma unroll
    for (int i = 0; i < CH; ++i) {
      mv[i] = Mrow[c * CH + i];
      vv[i] = vec[c * CH + i];
    }
    MPCQP_FENCE();
#pragma unroll
    for (int i = 0; i < CH; i += 4) {
      a0 = fma(mv[i], vv[i], a0);
      a1 = fma(mv[i + 1], vv[i + 1], a1);
      a2 = fma(mv[i + 2], vv[i + 2], a2);
      a3 = fma(mv[i + 3], vv[i + 3], a3);
    }
    MPCQP_FENCE();
  }
  return (a0 + a1) + (a2 + a3);
}

// M[lane][k] += c * vec[k] for k < 16*nch
__device__ __forceinline__ void lds_rank1(double* Mrow, double c, const double* vec, int nch) {
  for (int ch = 0; ch < nch; ++ch) {
    double mv[CH], vv[CH];
#pragma unroll
    for (int i = 0; i < CH; ++i) {
      mv[i] = Mrow[ch * CH + i];
      vv[i] = vec[ch * CH + i];
    }
    MPCQP_FENCE();
#pragma unroll
    for (int i = 0; i < CH; ++i) Mrow[ch * CH + i] = fma(c, vv[i], mv[i]);
    MPCQP_FENCE();
  }
}

// One pivot of the symmetric sweep, pivot index K a compile-time constant so that
// W stays in VGPRs (a runtime pivot index would demote W to scratch).
// W_ij -= z_i z_j / d (i,j != K), W_iK = z_i/d, W_KK = -1/d; the pivot row uses
// W_Kj = z_j (symmetry): W_Kj + (1/d - 1) z_j = z_j/d.  Ends at -H^-1.
template <int K>
__device__ __forceinline__ void sweep_step(double (&W)[LANES], double* vb, int lane, int n) {
  if (K < n) {   // wave-uniform; padded pivots are skipped (identity rows, decoupled)
    const double zk = W[K];
    vb[lane] = zk;
    __syncthreads();
    const double d = vb[K];
    const double inv = 1.0 / d;
    const double beta = (lane == K) ? (inv - 1.0) : -zk * inv;
#pragma unroll
    for (int c = 0; c < LANES; c += CH) {
      double v[CH];
#pragma unroll
      for (int i = 0; i < CH; ++i) v[i] = vb[c + i];
      MPCQP_FENCE();
#pragma unroll
      for (int i = 0; i < CH; ++i)
        if (c + i != K) W[c + i] = fma(beta, v[i], W[c + i]);
      MPCQP_FENCE();
    }
    W[K] = (lane == K) ? -inv : zk * inv;
    __syncthreads();
  }
}

template <int... Ks>
__device__ __forceinline__ void sweep_all(double (&W)[LANES], double* vb, int lane, int n,
                                          std::integer_sequence<int, Ks...>) {
  (sweep_step<Ks>(W, vb, lane, n), ...);
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

__global__ __launch_bounds__(LANES) __attribute__((amdgpu_waves_per_eu(1, 2))) void mpcqp_wave_kernel(
    KParams P, int B, const float* __restrict__ x0g, const float* __restrict__ xrefg,
    const float* __restrict__ contactg, const float* __restrict__ feetg, const float* __restrict__ robotg,
    float* __restrict__ u0g, float* __restrict__ Ug, int* __restrict__ statusg, int* __restrict__ itersg) {
  __shared__ Shared sm;
  const int b = blockIdx.x;
  const int lane = threadIdx.x;
  const int N = P.N;
  if (b >= B) return;
  const unsigned long long lt_mask = (lane == 0) ? 0ull : (~0ull >> (64 - lane));

  const float* cb = contactg + (size_t)b * N * 4;
  const float* rb = robotg + (size_t)b * MPCQP_ROBOT_STRIDE;
  const float* xb = x0g + (size_t)b * NX;
  const float* xrb = xrefg + (size_t)b * N * NX;
  const float* fb = feetg + (size_t)b * 12;

  STAMP(0);
  // ------------------------------------------------ stance list (gait table)
  const int nk = 4 * N;
  const float c0 = lane < nk ? cb[lane] : 0.f;
  const float c1 = lane + LANES < nk ? cb[lane + LANES] : 0.f;
  const bool f0 = c0 > 0.f, f1 = c1 > 0.f;
  const unsigned long long m0 = __ballot(f0), m1 = __ballot(f1);
  const int S0 = __popcll(m0);
  const int S = uni(S0 + __popcll(m1));
  const int n = 3 * S, m = 6 * S;
  const double fzmax = (double)rb[8];
  {
    const int i0 = __popcll(m0 & lt_mask), i1 = S0 + __popcll(m1 & lt_mask);
    if (lane < nk) sm.stance_of[lane] = f0 ? i0 : -1;
    if (lane + LANES < nk) sm.stance_of[lane + LANES] = f1 ? i1 : -1;
    if (f0 && i0 < SMAX) {
      sm.foot_t[i0] = lane / 4;
      sm.foot_leg[i0] = lane % 4;
      sm.foot_ub[i0] = (double)c0 * fzmax;   // ub = contact * fz_max (mpc.py:257)
    }
    if (f1 && i1 < SMAX) {
      sm.foot_t[i1] = (lane + LANES) / 4;
      sm.foot_leg[i1] = (lane + LANES) % 4;
      sm.foot_ub[i1] = (double)c1 * fzmax;
    }
  }
  if (n > NV) {
    write_empty(b, lane, N, MPCQP_STATUS_TOO_LARGE, u0g, Ug, statusg, itersg);
    return;
  }
  {
    int bad = 0;
    for (int k = lane; k < N * NX; k += LANES) bad |= !isfinite(xrb[k]);
    if (lane < NX) bad |= !isfinite(xb[lane]);
    if (lane < 12) bad |= !isfinite(fb[lane]) | !isfinite(rb[lane]);
    if (__any(bad)) {
      write_empty(b, lane, N, MPCQP_STATUS_NONFINITE, u0g, Ug, statusg, itersg);
      return;
    }
  }

  double* const scr = sm.scr;
  double* const Ac = scr + OFF_AC;
  double* const Nm = scr + OFF_NM;
  double* const Bc = scr + OFF_BC;
  double* const Ii = scr + OFF_II;
  double* const X = scr + OFF_X;   // X_p at X + p * NX * NU
  for (int k = lane; k < NX * NX; k += LANES) Ac[k] = 0.0;
  for (int k = lane; k < NX * NU; k += LANES) Bc[k] = 0.0;
  if (lane < NX) sm.x0[lane] = (double)xb[lane];
  __syncthreads();

  // ------------------------------------------------ 1. model (mpc.py:173-192)
  // Reference dtypes: Rz float32 of float64 cos/sin; I_w = Rz I Rz^T float32;
  // inv(I_w) float32; inv(I_w) @ skew(r) float64 rounded to float32; I/m float32.
  if (lane == 0) {
    const double yaw = (double)xb[2];
    const double c = f32r(cos(yaw)), s = f32r(sin(yaw));
    const double Rz[3][3] = {{c, -s, 0.0}, {s, c, 0.0}, {0.0, 0.0, 1.0}};
    const double Ib[3][3] = {{rb[1], rb[2], rb[3]}, {rb[2], rb[4], rb[5]}, {rb[3], rb[5], rb[6]}};
    double T1[3][3], Iw[3][3];
    for (int i = 0; i < 3; ++i)
      for (int j = 0; j < 3; ++j) T1[i][j] = f32r(Rz[i][0] * Ib[0][j] + Rz[i][1] * Ib[1][j] + Rz[i][2] * Ib[2][j]);
    for (int i = 0; i < 3; ++i)
      for (int j = 0; j < 3; ++j) Iw[i][j] = f32r(T1[i][0] * Rz[j][0] + T1[i][1] * Rz[j][1] + T1[i][2] * Rz[j][2]);
    const double a00 = Iw[1][1] * Iw[2][2] - Iw[1][2] * Iw[2][1];
    const double a10 = Iw[1][2] * Iw[2][0] - Iw[1][0] * Iw[2][2];
    const double a20 = Iw[1][0] * Iw[2][1] - Iw[1][1] * Iw[2][0];
    const double id = 1.0 / (Iw[0][0] * a00 + Iw[0][1] * a10 + Iw[0][2] * a20);
    Ii[0] = f32r(a00 * id);
    Ii[1] = f32r((Iw[0][2] * Iw[2][1] - Iw[0][1] * Iw[2][2]) * id);
    Ii[2] = f32r((Iw[0][1] * Iw[1][2] - Iw[0][2] * Iw[1][1]) * id);
    Ii[3] = f32r(a10 * id);
    Ii[4] = f32r((Iw[0][0] * Iw[2][2] - Iw[0][2] * Iw[2][0]) * id);
    Ii[5] = f32r((Iw[0][2] * Iw[1][0] - Iw[0][0] * Iw[1][2]) * id);
    Ii[6] = f32r(a20 * id);
    Ii[7] = f32r((Iw[0][1] * Iw[2][0] - Iw[0][0] * Iw[2][1]) * id);
    Ii[8] = f32r((Iw[0][0] * Iw[1][1] - Iw[0][1] * Iw[1][0]) * id);
    for (int i = 0; i < 3; ++i)
      for (int j = 0; j < 3; ++j) Ac[i * NX + 6 + j] = Rz[j][i];   // A_c[0:3,6:9] = Rz^T
    for (int i = 0; i < 3; ++i) Ac[(3 + i) * NX + 9 + i] = 1.0;     // A_c[3:6,9:12] = I
    Ac[11 * NX + 12] = 1.0;                                          // A_c[11,12] = 1
    // friction-cone rows in the (t1, t2, n) frame (mpc.py:239-245 for n = e_z)
    double nx = rb[9], ny = rb[10], nz = rb[11];
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
    const double mu = rb[7];
    const double rw[6][3] = {{t1x + mu * nx, t1y + mu * ny, t1z + mu * nz},
                             {-t1x + mu * nx, -t1y + mu * ny, -t1z + mu * nz},
                             {t2x + mu * nx, t2y + mu * ny, t2z + mu * nz},
                             {-t2x + mu * nx, -t2y + mu * ny, -t2z + mu * nz},
                             {nx, ny, nz},
                             {-nx, -ny, -nz}};
    for (int r = 0; r < 6; ++r)
      for (int j = 0; j < 3; ++j) sm.rows[r][j] = rw[r][j];
  }
  __syncthreads();
  // B_c (mpc.py:188-190): lanes 0..35 the skew blocks, 36..47 the 1/m diagonal
  if (lane < 36) {
    const int leg = lane / 9, i = (lane % 9) / 3, j = lane % 3;
    const double rx = fb[3 * leg], ry = fb[3 * leg + 1], rz = fb[3 * leg + 2];
    // column j of skew(r) = [r]x
    const double sk0 = (j == 0) ? 0.0 : (j == 1 ? -rz : ry);
    const double sk1 = (j == 0) ? rz : (j == 1 ? 0.0 : -rx);
    const double sk2 = (j == 0) ? -ry : (j == 1 ? rx : 0.0);
    Bc[(6 + i) * NU + 3 * leg + j] = f32r(Ii[3 * i] * sk0 + Ii[3 * i + 1] * sk1 + Ii[3 * i + 2] * sk2);
  } else if (lane < 48) {
    const int leg = (lane - 36) / 3, i = (lane - 36) % 3;
    Bc[(9 + i) * NU + 3 * leg + i] = f32r(1.0 / (double)rb[0]);
  }
  __syncthreads();

  // -------------------------------- 2. exact discretisation (mpc.py:194-208)
  const double dt = P.dt, hdt2 = 0.5 * P.dt * P.dt;
  for (int k = lane; k < NX * NX; k += LANES) {   // Nm = A_c dt + A_c^2 dt^2/2
    const int i = k / NX, j = k % NX;
    double a2 = 0.0;
    for (int l = 0; l < NX; ++l) a2 = fma(Ac[i * NX + l], Ac[l * NX + j], a2);
    Nm[k] = Ac[k] * dt + a2 * hdt2;
  }
  for (int k = lane; k < NX * NU; k += LANES) {   // B_d = B_c dt + A_c B_c dt^2/2
    const int i = k / NU, j = k % NU;
    double ab = 0.0;
    for (int l = 0; l < NX; ++l) ab = fma(Ac[i * NX + l], Bc[l * NU + j], ab);
    X[k] = Bc[k] * dt + ab * hdt2;
  }
  __syncthreads();
  for (int k = lane; k < NX * NU; k += LANES) {   // X1 = Nm X0
    const int i = k / NU, j = k % NU;
    double a = 0.0;
    for (int l = 0; l < NX; ++l) a = fma(Nm[i * NX + l], X[l * NU + j], a);
    X[NX * NU + k] = a;
  }
  if (lane < NX) {
    double a = 0.0;
    for (int l = 0; l < NX; ++l) a = fma(Nm[lane * NX + l], sm.x0[l], a);
    sm.y1[lane] = a;
  }
  __syncthreads();
  for (int k = lane; k < NX * NU; k += LANES) {   // X2 = Nm X1
    const int i = k / NU, j = k % NU;
    double a = 0.0;
    for (int l = 0; l < NX; ++l) a = fma(Nm[i * NX + l], X[NX * NU + l * NU + j], a);
    X[2 * NX * NU + k] = a;
  }
  if (lane < NX) {
    double a = 0.0;
    for (int l = 0; l < NX; ++l) a = fma(Nm[lane * NX + l], sm.y1[l], a);
    sm.y2[lane] = a;
  }
  __syncthreads();

  STAMP(1);
  // -------------------------------------- 3. condensed cost (mpc.py:211-235)
  {
    double* const e = scr;            // e_t = A^{t+1} x0 - xref_t   (Sx x0 - Xref)
    double* const zp = scr + N * NX;  // zp[p][t][c] = sum_s X_p[s][c] Q_s e_t[s]
    for (int k = lane; k < N * NX; k += LANES) {
      const int t = k / NX, s = k % NX;
      const double kk = (double)(t + 1);
      e[k] = sm.x0[s] + kk * sm.y1[s] + 0.5 * kk * (kk - 1.0) * sm.y2[s] - (double)xrb[k];
    }
    __syncthreads();
    for (int k = lane; k < 3 * N * NU; k += LANES) {
      const int p = k / (N * NU), rem = k % (N * NU), t = rem / NU, c = rem % NU;
      double a = 0.0;
      for (int s = 0; s < NX; ++s) a = fma(X[p * NX * NU + s * NU + c], P.q[s] * e[t * NX + s], a);
      zp[k] = a;
    }
    __syncthreads();
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
    __syncthreads();
  }
  double* const Y = scr + OFF_Y;
  double* const T = scr + OFF_T;
  const int nT = N * (N + 1) / 2;
  for (int k = lane; k < 9 * NU * NU; k += LANES) {   // Y_pq = X_p^T Q X_q
    const int pq = k / (NU * NU), cc = k % (NU * NU);
    const int p = pq / 3, q = pq % 3, c = cc / NU, c2 = cc % NU;
    double a = 0.0;
    for (int s = 0; s < NX; ++s) a = fma(P.q[s] * X[p * NX * NU + s * NU + c], X[q * NX * NU + s * NU + c2], a);
    Y[k] = a;
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
  __syncthreads();

  STAMP(2);
  // H row `lane` into registers; rows/cols >= n are the identity (padding)
  double W[LANES];
  {
    const bool act_row = lane < n;
    const int sa = act_row ? lane / 3 : 0;
    const int ja = sm.foot_t[sa];
    const int ca = 3 * sm.foot_leg[sa] + lane % 3;
    const double r2 = 2.0 * P.r[act_row ? ca : 0];
#pragma unroll
    for (int sb = 0; sb < SMAX; ++sb) {
      if (3 * sb < n) {   // wave-uniform
        const int jb = sm.foot_t[sb], lb = sm.foot_leg[sb];
        const bool le = ja <= jb;
        const int ti = le ? tidx(N, jb - ja, N - jb) : tidx(N, ja - jb, N - ja);
        double tv[9];
#pragma unroll
        for (int p = 0; p < 3; ++p)
#pragma unroll
          for (int q = 0; q < 3; ++q) tv[p * 3 + q] = T[(le ? p * 3 + q : q * 3 + p) * nT + ti];
#pragma unroll
        for (int be = 0; be < 3; ++be) {
          const int bcol = 3 * sb + be;
          const int cbv = 3 * lb + be;
          double acc = 0.0;
#pragma unroll
          for (int pq = 0; pq < 9; ++pq) acc = fma(tv[pq], Y[pq * NU * NU + ca * NU + cbv], acc);
          const double h = 2.0 * acc + (lane == bcol ? r2 : 0.0);
          W[bcol] = act_row ? h : (lane == bcol ? 1.0 : 0.0);
        }
      } else {
#pragma unroll
        for (int be = 0; be < 3; ++be) W[3 * sb + be] = (lane == 3 * sb + be) ? 1.0 : 0.0;
      }
    }
    W[63] = (lane == 63) ? 1.0 : 0.0;
  }
  __syncthreads();

  STAMP(3);
  // ------------------------------------------------ 4. W = H^-1 (symmetric sweep)
  sweep_all(W, sm.vb, lane, n, std::make_integer_sequence<int, LANES>{});
#pragma unroll
  for (int j = 0; j < LANES; ++j) W[j] = -W[j];

  STAMP(4);
  // Per-lane register caches of the constraint data (no dependent LDS lookups
  // inside the active-set loop):
  //   constraint lanes: rows c = lane, lane + 64 -> foot, row vector a_c, bound term
  //   variable lanes:   i -> foot i/3, column (i%3) of the 6 cone rows, slot of each row
  //   slot lanes:       j -> foot, row vector, bound term of the constraint in slot j
  auto crow = [&](int c, int& f, double& a0, double& a1, double& a2, double& bt) {
    const int cc = c < m ? c : 0;
    f = cc / 6;
    const int rr = cc % 6;
    a0 = sm.rows[rr][0];
    a1 = sm.rows[rr][1];
    a2 = sm.rows[rr][2];
    bt = (rr == 5) ? sm.foot_ub[f] : 0.0;   // s_c = a_c . x + bt  (b = -contact*fz_max on row 5)
  };
  int clo_f, chi_f;
  double clo_a0, clo_a1, clo_a2, clo_b, chi_a0, chi_a1, chi_a2, chi_b;
  crow(lane, clo_f, clo_a0, clo_a1, clo_a2, clo_b);
  crow(lane + LANES, chi_f, chi_a0, chi_a1, chi_a2, chi_b);
  const bool clo_ok = lane < m, chi_ok = lane + LANES < m;
  const int vf = lane / 3, vax = lane % 3;
  const bool vok = lane < n;
  double acol[6];
  int fslot[6];
#pragma unroll
  for (int rr = 0; rr < 6; ++rr) {
    acol[rr] = sm.rows[rr][vax];
    fslot[rr] = -1;
  }
  int sl_c = 0, sl_f = 0;
  double sl_a0 = 0.0, sl_a1 = 0.0, sl_a2 = 0.0, sl_b = 0.0;

  // unconstrained minimiser x = -W g ; constraint values s = A x - b
  const double xu = -matvec(W, sm.gv);
  sm.zv[lane] = xu;
  __syncthreads();
  double s_lo = clo_ok ? clo_a0 * sm.zv[3 * clo_f] + clo_a1 * sm.zv[3 * clo_f + 1] + clo_a2 * sm.zv[3 * clo_f + 2] + clo_b
                       : INFINITY;
  double s_hi = chi_ok ? chi_a0 * sm.zv[3 * chi_f] + chi_a1 * sm.zv[3 * chi_f + 1] + chi_a2 * sm.zv[3 * chi_f + 2] + chi_b
                       : INFINITY;

  // ------------------------- 5. Goldfarb-Idnani dual active set (range space)
  // (M_AA)^-1 over active-set slots in LDS (scratch is dead now); free rows/cols are 0
  double* const Mrow = scr + lane * LDM;
  __syncthreads();
  for (int k = 0; k < LANES; k += 2) {
    Mrow[k] = 0.0;
    Mrow[k + 1] = 0.0;
  }
  double u = 0.0;               // multiplier of slot `lane`
  unsigned long long occ = 0;   // occupied slots (wave-uniform)
  const int max_iter = P.max_iter > 0 ? P.max_iter : 8 * NV + 64;
  const double tol = 1e-9;
  int it = 0;
  int status = MPCQP_STATUS_OK;
  __syncthreads();
  while (true) {
    // most violated row
    double bv;
    const int p = wave_argmin2(s_lo, s_hi, bv);
    if (!(bv < -tol)) break;
    const int fp = p / 6, rp = p % 6;
    const double ap0 = sm.rows[rp][0], ap1 = sm.rows[rp][1], ap2 = sm.rows[rp][2];
    double acol_p = 0.0;   // a_p[vax] for this variable lane
#pragma unroll
    for (int rr = 0; rr < 6; ++rr) acol_p = (rr == rp) ? acol[rr] : acol_p;
    const double ap_l = (vok && vf == fp) ? acol_p : 0.0;
    // w = W a_p  (a_p lives on the 3 variables of foot fp)
    sm.vb[lane] = ap_l;
    __syncthreads();
    const double wl = matvec(W, sm.vb);
    sm.wv[lane] = wl;
    const double apw = ap0 * readlane_d(wl, 3 * fp) + ap1 * readlane_d(wl, 3 * fp + 1) + ap2 * readlane_d(wl, 3 * fp + 2);
    double up = 0.0;
    bool added = false;
    __syncthreads();
    while (!added) {
      if (++it > max_iter) {
        status = MPCQP_STATUS_MAX_ITER;
        break;
      }
      const bool mine = (occ >> lane) & 1ull;
      // mp_j = a_{A_j} . w(foot_j)  ->  vb ;  r = Minv mp
      const double mpj =
          mine ? sl_a0 * sm.wv[3 * sl_f] + sl_a1 * sm.wv[3 * sl_f + 1] + sl_a2 * sm.wv[3 * sl_f + 2] : 0.0;
      sm.vb[lane] = mpj;
      __syncthreads();
      const int nch = uni((64 - __clzll(occ) + 1 + CH - 1) / CH);   // slot chunks in use (+ next free)
      double r = lds_matvec(Mrow, sm.vb, nch);
      if (!mine) r = 0.0;
      sm.rv[lane] = r;
      __syncthreads();
      // v = a_p - sum_j r_j a_{A_j}  on the variable lanes (per-foot slot cache)
      double vl = ap_l;
#pragma unroll
      for (int rr = 0; rr < 6; ++rr)
        if (fslot[rr] >= 0) vl -= sm.rv[fslot[rr]] * acol[rr];
      sm.vb[lane] = vok ? vl : 0.0;
      __syncthreads();
      const double zl = matvec(W, sm.vb);   // primal direction z = W v
      sm.zv[lane] = zl;
      __syncthreads();
      const double zs_lo = clo_ok ? clo_a0 * sm.zv[3 * clo_f] + clo_a1 * sm.zv[3 * clo_f + 1] + clo_a2 * sm.zv[3 * clo_f + 2] : 0.0;
      const double zs_hi = chi_ok ? chi_a0 * sm.zv[3 * chi_f] + chi_a1 * sm.zv[3 * chi_f + 1] + chi_a2 * sm.zv[3 * chi_f + 2] : 0.0;
      // dual step bound t1 (smallest u_j / r_j over r_j > 0), primal step t2
      double t1;
      const int l = wave_argmin2((mine && r > 0.0) ? u / r : INFINITY, INFINITY, t1);
      const double zsp = readlane_d(p < LANES ? zs_lo : zs_hi, p & (LANES - 1));
      const double sp = readlane_d(p < LANES ? s_lo : s_hi, p & (LANES - 1));
      double t2 = INFINITY;
      if (zsp > 1e-12 * apw) t2 = -sp / zsp;
      const bool add = t2 <= t1;
      const double t = add ? t2 : t1;
      if (!(t < INFINITY)) {
        status = MPCQP_STATUS_INFEASIBLE;
        break;
      }
      if (mine) u -= t * r;
      s_lo += t * zs_lo;
      s_hi += t * zs_hi;
      up += t;
      if (add) {
        // border (M_AA)^-1 with slot q: sigma = zs_p (Schur complement)
        const int q = uni(__builtin_ctzll(~occ));
        const double is = 1.0 / zsp;
        const double ci = (lane == q) ? -is : r * is;   // row q was zero: becomes -r^T / sigma
        lds_rank1(Mrow, ci, sm.rv, nch);
        __syncthreads();
        Mrow[q] = (lane == q) ? is : -r * is;
        if (lane == q) {
          u = up;
          sl_c = p;
          sl_f = fp;
          sl_a0 = ap0;
          sl_a1 = ap1;
          sl_a2 = ap2;
          sl_b = (rp == 5) ? sm.foot_ub[fp] : 0.0;
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
        sm.vb[lane] = col;
        __syncthreads();
        const double ill = 1.0 / sm.vb[l];
        lds_rank1(Mrow, -col * ill, sm.vb, nch);
        __syncthreads();
        Mrow[l] = 0.0;                 // column l
        scr[l * LDM + lane] = 0.0;     // row l
        const int cdrop = uni(__builtin_amdgcn_readlane(sl_c, l));
        if (vf == cdrop / 6) {
#pragma unroll
          for (int rr = 0; rr < 6; ++rr)
            if (rr == cdrop % 6) fslot[rr] = -1;
        }
        if (lane == l) u = 0.0;
        occ &= ~(1ull << l);
      }
      __syncthreads();
    }
    if (status != MPCQP_STATUS_OK) break;
  }
  __syncthreads();

  STAMP(5);
  // ------------------------------- 6. refinement, final x, KKT verification
  double x = 0.0;
  for (int pass = 0; pass < 2; ++pass) {
    // x = W (A_A^T u - g)
    sm.rv[lane] = ((occ >> lane) & 1ull) ? u : 0.0;
    __syncthreads();
    double vl = -sm.gv[lane];
#pragma unroll
    for (int rr = 0; rr < 6; ++rr)
      if (fslot[rr] >= 0) vl += sm.rv[fslot[rr]] * acol[rr];
    sm.vb[lane] = vok ? vl : 0.0;
    __syncthreads();
    x = matvec(W, sm.vb);
    sm.zv[lane] = x;
    __syncthreads();
    if (pass == 1) break;
    // u -= Minv (A_A x - b_A): pull the active rows back onto their bounds
    const bool mine = (occ >> lane) & 1ull;
    const double res =
        mine ? sl_a0 * sm.zv[3 * sl_f] + sl_a1 * sm.zv[3 * sl_f + 1] + sl_a2 * sm.zv[3 * sl_f + 2] + sl_b : 0.0;
    sm.vb[lane] = res;
    __syncthreads();
    const double du = lds_matvec(Mrow, sm.vb, LANES / CH);
    if (mine) u -= du;
    __syncthreads();
  }
  {
    const double vlo = clo_a0 * sm.zv[3 * clo_f] + clo_a1 * sm.zv[3 * clo_f + 1] + clo_a2 * sm.zv[3 * clo_f + 2] + clo_b;
    const double vhi = chi_a0 * sm.zv[3 * chi_f] + chi_a1 * sm.zv[3 * chi_f + 1] + chi_a2 * sm.zv[3 * chi_f + 2] + chi_b;
    int bad = (clo_ok && (vlo < -1e-6 || !isfinite(vlo))) || (chi_ok && (vhi < -1e-6 || !isfinite(vhi)));
    if ((occ >> lane) & 1ull) bad |= (u < -1e-9);
    if (__any(bad) && status == MPCQP_STATUS_OK) status = MPCQP_STATUS_MAX_ITER;
  }

  STAMP(6);
  // ---------------------------------------------------------------- output
#ifdef MPCQP_STAMPS
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
  hipLaunchKernelGGL(mpcqp_wave_kernel, dim3(batch), dim3(LANES), 0, st, kp, (int)batch, x0, xref, contact, feet,
                     robot, u0, U, (int*)status, (int*)iters);
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
