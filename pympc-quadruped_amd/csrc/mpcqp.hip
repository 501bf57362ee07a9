// mpcqp.hip -- MI355X (gfx950) batched convex-MPC QP engine: kernels + C ABI.
//
// Replaces, for a batch of independent robots, the per-tick formulate-and-solve of
// ModelPredictiveController._solve_mpc (/root/reference/linear_mpc/mpc.py:262-290):
// model (mpc.py:173-192), discretisation (:194-208), condensing and H/g (:211-235),
// friction-cone rows (:237-260) and the Drake-branch QP (:277-286)
//
//   min 1/2 U^T H U + g^T U   s.t.  lb <= C U <= ub,   C = kron(I_4N, cone)
//
// generalised to a per-robot cone normal (normal = e_z reproduces mpc.py exactly).
//
// ONE WORKGROUP PER ROBOT, nothing but the inputs and outputs touches HBM:
//   class NV =  64: 2 waves, n = 3 * #stance <= 64   (mpcqp_kernel_64)
//   class NV =  96: 6 waves, 4 x 6 tiles, n <= 96   (mpcqp_kernel_96, fed by a
//                   device queue the first class fills)
//   class NV = 128: 8 waves, n <= 126                (mpcqp_kernel_128, fed by a
//                   device queue the first class fills)
//   large class:    1 wave, n up to 12 N = 240       (mpcqp_kernel_ipm: Riccati-factored
//                   interior point + exact active-set polish, mpcqp_ipm.h)
// Formulation in closed form (mpcqp_form.h); H^-1 by a symmetric sweep over
// register tiles; Goldfarb-Idnani dual active set in projected form with the
// reduced inverse Hessian and the multiplier map in registers (mpcqp_solve.h).

#include <hip/hip_runtime.h>

#include <math.h>
#include <stdint.h>

#include <cmath>
#include <string.h>

#include <new>
#include <string>
#include <type_traits>
#include <utility>
#include <vector>

#include "mpcqp.h"

namespace {

constexpr int NX = 13;      // state dimension (mpc.py:26)
constexpr int NU = 12;      // input dimension (mpc.py:28)
constexpr int LANES = 64;
constexpr int kMaxN = MPCQP_MAX_HORIZON;   // the longest horizon mpcqp_create accepts (include/mpcqp.h)
constexpr int kDenseN = 20;   // the dense classes' LDS layouts hold N <= 20; longer horizons go to
                              // the interior-point class, sized for N <= kMaxN
static_assert(kMaxN >= kDenseN && 4 * kMaxN <= 2 * LANES, "stance lists cover 4 N <= 128 entries");
static_assert(MPCQP_WARM_BYTES == 4 * kMaxN, "warm-start memory: one byte per (stage, leg)");
// staged inputs (floats)
constexpr int IN_X0 = 0, IN_FEET = 13, IN_ROBOT = 25, IN_CONTACT = 44;   // + FormT<NM>::IN_XREF

typedef double d2 __attribute__((ext_vector_type(2)));
typedef double d4 __attribute__((ext_vector_type(4)));   // v_mfma_f64_16x16x4 accumulators (mpcqp_ipm.h)

struct KParams {
  int N;
  int max_iter;
  double dt;
  double q[NX];
  double r[NU];
  const double* wfull;   // device: full Q (13 x 13) then R (12 x 12), row-major; nullptr = diagonal q, r
  unsigned char* warm;   // device: per-robot warm-start memory (mpcqp_set_warm_start), or nullptr
  int warm_cap;          // robots with memory
};

// Diagnostic build only (-DMPCQP_STAMPS): per-phase s_memtime stamps and per-section
// cycle accumulators of the active-set loop, written to U (>= 32 floats per robot);
// the shipped kernel executes no stamp.
#ifdef MPCQP_STAMPS
#define STAMP(i)                                \
  do {                                          \
    __builtin_amdgcn_sched_barrier(0);          \
    stamps_[i] = __builtin_amdgcn_s_memtime();  \
    __builtin_amdgcn_sched_barrier(0);          \
  } while (0)
// section accumulators live one per lane (lane k holds section k): a uniform
// compare, no runtime-indexed private array (that would go to scratch, and the
// next barrier's vmcnt wait would absorb the scratch latency)
#define SEC(k)                                                   \
  do {                                                           \
    __builtin_amdgcn_sched_barrier(0);                           \
    const unsigned long long t_ = __builtin_amdgcn_s_memtime();  \
    if (lane == seccur_) secacc_ += t_ - seclast_;               \
    seclast_ = t_;                                               \
    seccur_ = (k);                                               \
    __builtin_amdgcn_sched_barrier(0);                           \
  } while (0)
#define CNT(k) (secacc_ += (lane == (k)) ? 1ull : 0ull)
#ifndef MPCQP_SOLO_LDS
// stamps builds only (tools/solo_stamps.py): extra dynamic LDS per class-64 workgroup, so that one
// robot holds a CU alone -- each robot's solo latency against its four robots per CU
#define MPCQP_SOLO_LDS 0
#endif
constexpr unsigned kDiagLds = MPCQP_SOLO_LDS;
constexpr int kStampU64 = 256;   // stamp slots per robot (the stamps build's U buffer: 512 floats per robot)
static_assert(32 + 24 * 8 <= kStampU64, "eight waves' section accumulators");
#else
constexpr unsigned kDiagLds = 0;
#define CNT(k) \
  do {         \
  } while (0)
#define STAMP(i) \
  do {           \
  } while (0)
#define SEC(k) \
  do {         \
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

// wave-uniform double kept in SGPRs (frees the VGPR pair a uniform VALU result
// would otherwise occupy for its whole live range)
__device__ __forceinline__ double sgpr_d(double v) {
  const long long b = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_readfirstlane((int)(b & 0xffffffffll));
  const int hi = __builtin_amdgcn_readfirstlane((int)(b >> 32));
  return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}

// Compile-time loop: f(std::integral_constant<int, I>{}) for I = 0..N-1 (register
// arrays indexed by I stay in registers).
template <typename F, int... Is>
__device__ __forceinline__ void static_for_impl(F&& f, std::integer_sequence<int, Is...>) {
  (f(std::integral_constant<int, Is>{}), ...);
}
template <int N, typename F>
__device__ __forceinline__ void static_for(F&& f) {
  static_for_impl(f, std::make_integer_sequence<int, N>{});
}

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

// v_min_f64 / v_max_f64 without the NaN canonicalisation fmin/fmax carry (no
// operand here is NaN: +inf marks "no candidate")
__device__ __forceinline__ double vmin(double a, double b) {
  double r;
  asm("v_min_f64 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
  return r;
}
__device__ __forceinline__ double vmax(double a, double b) {
  double r;
  asm("v_max_f64 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
  return r;
}

template <int CTRL, int ROWMASK>
__device__ __forceinline__ double dpp_m(double v) {   // rows outside ROWMASK keep v
  const long long bits = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_update_dpp((int)bits, (int)bits, CTRL, ROWMASK, 0xF, false);
  const int hi = __builtin_amdgcn_update_dpp((int)(bits >> 32), (int)(bits >> 32), CTRL, ROWMASK, 0xF, false);
  return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}
constexpr int DPP_BCAST15 = 0x142;  // row_bcast:15 -- lane 15 of each row to the next row
constexpr int DPP_BCAST31 = 0x143;  // row_bcast:31 -- lane 31 to rows 2 and 3

// Cross-lane min / max over the wave: butterfly inside 16-lane rows, then the
// row_bcast chain leaves the result in lane 63
__device__ __forceinline__ double wave_min(double v) {
  v = vmin(v, dpp_d<DPP_XOR1>(v));
  v = vmin(v, dpp_d<DPP_XOR2>(v));
  v = vmin(v, dpp_d<DPP_HMIRROR>(v));
  v = vmin(v, dpp_d<DPP_MIRROR>(v));
  v = vmin(v, dpp_m<DPP_BCAST15, 0xA>(v));
  v = vmin(v, dpp_m<DPP_BCAST31, 0xC>(v));
  return readlane_d(v, 63);
}
__device__ __forceinline__ double wave_max_d(double v) {
  v = vmax(v, dpp_d<DPP_XOR1>(v));
  v = vmax(v, dpp_d<DPP_XOR2>(v));
  v = vmax(v, dpp_d<DPP_HMIRROR>(v));
  v = vmax(v, dpp_d<DPP_MIRROR>(v));
  v = vmax(v, dpp_m<DPP_BCAST15, 0xA>(v));
  v = vmax(v, dpp_m<DPP_BCAST31, 0xC>(v));
  return readlane_d(v, 63);
}

// 1/d: hardware reciprocal estimate refined by two Newton steps (~1 ulp; d is a
// normal, well-scaled pivot / curvature, never 0, inf or denormal here)
__device__ __forceinline__ double rcp_nr(double d) {
  double y = __builtin_amdgcn_rcp(d);
  double e = fma(-d, y, 1.0);
  y = fma(y, e, y);
  e = fma(-d, y, 1.0);
  return fma(y, e, y);
}
// a / b with one residual correction of the quotient
__device__ __forceinline__ double div_nr(double a, double b) {
  const double y = rcp_nr(b);
  const double q = a * y;
  return fma(fma(-b, q, a), y, q);
}

// 8 / 4 consecutive doubles starting at element 8k / 4k (16-B aligned LDS vectors)
__device__ __forceinline__ void ld8(double (&v)[8], const double* base, int k) {
  const d2* p = reinterpret_cast<const d2*>(base + 8 * k);
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const d2 x = p[i];
    v[2 * i] = x[0];
    v[2 * i + 1] = x[1];
  }
}
__device__ __forceinline__ void st8(double* base, int k, const double (&v)[8]) {
  d2* p = reinterpret_cast<d2*>(base + 8 * k);
#pragma unroll
  for (int i = 0; i < 4; ++i) p[i] = d2{v[2 * i], v[2 * i + 1]};
}
// TW consecutive doubles starting at element TW k (TW even; 16-B aligned LDS vectors)
template <int TW>
__device__ __forceinline__ void ldt(double (&v)[TW], const double* base, int k) {
  const d2* p = reinterpret_cast<const d2*>(base + TW * k);
#pragma unroll
  for (int i = 0; i < TW / 2; ++i) {
    const d2 x = p[i];
    v[2 * i] = x[0];
    v[2 * i + 1] = x[1];
  }
}
template <int TW>
__device__ __forceinline__ void stt(double* base, int k, const double (&v)[TW]) {
  d2* p = reinterpret_cast<d2*>(base + TW * k);
#pragma unroll
  for (int i = 0; i < TW / 2; ++i) p[i] = d2{v[2 * i], v[2 * i + 1]};
}
// TW consecutive doubles starting at element TS k (TS >= TW: a padded tile-column stride)
template <int TW, int TS>
__device__ __forceinline__ void lds_t(double (&v)[TW], const double* base, int k) {
  const d2* p = reinterpret_cast<const d2*>(base + TS * k);
#pragma unroll
  for (int i = 0; i < TW / 2; ++i) {
    const d2 x = p[i];
    v[2 * i] = x[0];
    v[2 * i + 1] = x[1];
  }
}
// 4 consecutive doubles at p (16-B aligned)
__device__ __forceinline__ void ld4s(double (&v)[4], const double* p) {
  const d2 a = reinterpret_cast<const d2*>(p)[0], b = reinterpret_cast<const d2*>(p)[1];
  v[0] = a[0]; v[1] = a[1]; v[2] = b[0]; v[3] = b[1];
}
__device__ __forceinline__ void st4s(double* p, const double (&v)[4]) {
  reinterpret_cast<d2*>(p)[0] = d2{v[0], v[1]};
  reinterpret_cast<d2*>(p)[1] = d2{v[2], v[3]};
}
__device__ __forceinline__ void ld4(double (&v)[4], const double* base, int k) {
  const d2* p = reinterpret_cast<const d2*>(base + 4 * k);
  const d2 a = p[0], b = p[1];
  v[0] = a[0]; v[1] = a[1]; v[2] = b[0]; v[3] = b[1];
}
__device__ __forceinline__ void st4(double* base, int k, const double (&v)[4]) {
  d2* p = reinterpret_cast<d2*>(base + 4 * k);
  p[0] = d2{v[0], v[1]};
  p[1] = d2{v[2], v[3]};
}

// ---- wave argmin with an f32 pre-selection.  Round-to-nearest f64 -> f32 is
// monotone, so the f64 minimum's f32 image is the f32 minimum: a unique f32
// minimum IS the exact answer; f32 ties fall back to the f64 reduction.  The
// f32 reduction is one DPP-encoded v_min_f32 per stage.
// The six stages are one asm statement: each DPP read of the previous stage's VGPR needs
// two wait states (s_nop 1), and separate statements made hipcc pad every boundary again.
__device__ __forceinline__ float wave_min_f32(float v) {
  asm volatile(
      "s_nop 1\n\t"
      "v_min_f32_dpp %0, %0, %0 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n\t"
      "s_nop 1\n\t"
      "v_min_f32_dpp %0, %0, %0 quad_perm:[2,3,0,1] row_mask:0xf bank_mask:0xf\n\t"
      "s_nop 1\n\t"
      "v_min_f32_dpp %0, %0, %0 row_half_mirror row_mask:0xf bank_mask:0xf\n\t"
      "s_nop 1\n\t"
      "v_min_f32_dpp %0, %0, %0 row_mirror row_mask:0xf bank_mask:0xf\n\t"
      "s_nop 1\n\t"
      "v_min_f32_dpp %0, %0, %0 row_bcast:15 row_mask:0xa bank_mask:0xf\n\t"
      "s_nop 1\n\t"
      "v_min_f32_dpp %0, %0, %0 row_bcast:31 row_mask:0xc bank_mask:0xf"
      : "+v"(v));
  return __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), 63));
}
// lowest lane holding the wave minimum of v (+inf = no candidate); vmin_out = that minimum
__device__ __forceinline__ int wave_argmin_d(double v, double& vmin_out) {
  const float f = (float)v;
  const float fm = wave_min_f32(f);
  const unsigned long long cand = __ballot(f == fm);
  int l;
  if (__popcll(cand) == 1) {
    l = uni(__builtin_ctzll(cand));
    vmin_out = readlane_d(v, l);
  } else if (fm == INFINITY && __ballot(v < INFINITY) == 0ull) {
    // no candidate in any lane (e.g. no active slot blocks the step): the common
    // all-+inf tie needs no f64 reduction
    l = 0;
    vmin_out = INFINITY;
  } else {
    const double vv = (f == fm) ? v : INFINITY;
    const double m = wave_min(vv);
    l = uni(__builtin_ctzll(__ballot(vv == m)));
    vmin_out = m;
  }
  return l;
}

// lowest lane holding the f32-rounded wave minimum of v; vmin_out = v in that lane.
// Not the exact f64 argmin on f32 ties -- for choices where any deterministic
// near-minimal lane will do (every wave computes the same lane).
__device__ __forceinline__ int wave_argmin_f32(double v, double& vmin_out) {
  const float f = (float)v;
  const float fm = wave_min_f32(f);
  const int l = uni(__builtin_ctzll(__ballot(f == fm)));
  vmin_out = readlane_d(v, l);
  return l;
}

#include "mpcqp_form.h"
#include "mpcqp_combo_asm.h"
#include "mpcqp_solve.h"
#include "mpcqp_ipm.h"
#include "mpcqp_plan.h"

// Workgroups are dealt round-robin over the 8 XCDs (block bid runs on XCD bid % 8,
// MI355X_MICROARCH.md "Workgroup dispatch"; speed only, never correctness).  Block bid
// solves robot xcd_robot(bid, B): each XCD takes one contiguous range of robots, so
// neighbouring robots -- whose input records and u0 / status / iters entries share
// cache lines -- meet in one L2 and their lines are fetched and written back once.
// A bijection of [0, B) for every B.
__device__ __forceinline__ int xcd_robot(int bid, int B) {
  const int x = bid & 7, i = bid >> 3, q = B >> 3, r = B & 7;
  return x * q + (x < r ? x : r) + i;
}

// ---- Dispatch order (ABI 6, mpcqp_set_order).  A robot's active set -- and so its solve
// time -- grows with the horizontal velocity correction its cone forces must supply: on the
// benchmark batches |v0 - vref_0| has correlation 0.87 (config 2) / 0.85 (config 4) with the
// iteration count (tools/order_sim.py).  mpcqp_order_kernel sorts each dispatch segment by
// that key, largest first, so that in a batch that queues on the CUs (configs 3 to 5) the longest
// robots start first and the launch ends near its mean load instead of behind a late long
// robot (configs 3 / 4 / 5 +7.7 / +6.2 / +3.7 %, profiles/r5_combo/ab_order.txt).  Only the
// robot -> workgroup map changes: every robot's solve is bitwise the same.
constexpr int kOrderMax = 8192;   // class 64: robots per XCD range the order kernel takes (8 per thread)
constexpr int kOrderSeg = 1024;   // classes 96 / 128: robots per interleaved segment (one per thread)
constexpr int kOrderMin = 64;     // smaller batches keep their order (nothing to balance)
constexpr int kOrderBuckets = 256;

__device__ __forceinline__ float order_key(const float* __restrict__ x0g, const float* __restrict__ xrefg, int N,
                                           int r) {
  const float ex = x0g[(size_t)r * NX + 9] - xrefg[(size_t)r * N * NX + 9];
  const float ey = x0g[(size_t)r * NX + 10] - xrefg[(size_t)r * N * NX + 10];
  const float k = ex * ex + ey * ey;
  return k >= 0.0f && k <= 3.0e38f ? k : 0.0f;   // NaN / inf: no preference
}

// One 1024-thread workgroup per segment, a counting sort into 256 key buckets, largest first
// (the order within a bucket is the atomics' order: it is a schedule, not a result).  A segment
// is the robots start + stride j (j < len), and rank r goes to position start + stride r:
//   mode 0: the 8 contiguous XCD ranges of class 64 (xcd_robot: the robots of blocks x, x + 8,
//           ...), so a sorted range keeps its robots on their XCD's L2;
//   mode 1: ceil(B / 1024) interleaved segments (stride = their count) for classes 96 / 128
//           taking the batch directly: position s + S r holds segment s's r-th heaviest robot,
//           so the workgroups dispatched first get the heaviest robots of every segment.
// Buckets: sqrt(key / max key) in 256 steps (|v0 - vref_0| relative to the batch's largest).
__global__ __launch_bounds__(1024) void mpcqp_order_kernel(int B, int N, const float* __restrict__ x0g,
                                                           const float* __restrict__ xrefg, int* __restrict__ perm,
                                                           int mode) {
  __shared__ int hist[kOrderBuckets], cursor[kOrderBuckets];
  __shared__ unsigned kmax_bits;
  __shared__ int wsum[kOrderBuckets / LANES];
  const int seg = blockIdx.x, tid = threadIdx.x, lane = tid & (LANES - 1);
  int start, stride, len;
  if (mode == 0) {
    const int q = B >> 3, r = B & 7;
    start = seg * q + (seg < r ? seg : r);
    stride = 1;
    len = q + (seg < r ? 1 : 0);
  } else {
    const int S = (B + kOrderSeg - 1) / kOrderSeg;
    start = seg;
    stride = S;
    len = (B - seg + S - 1) / S;
  }
  constexpr int KPT = kOrderMax / 1024;   // keys per thread
  float key[KPT];
  float kmx = 0.0f;
#pragma unroll
  for (int t = 0; t < KPT; ++t) {
    const int j = tid + 1024 * t;
    key[t] = j < len ? order_key(x0g, xrefg, N, start + stride * j) : 0.0f;
    kmx = fmaxf(kmx, key[t]);
  }
  if (tid < kOrderBuckets) hist[tid] = cursor[tid] = 0;
  if (tid == 0) kmax_bits = 0u;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) kmx = fmaxf(kmx, __shfl_xor(kmx, o));
  __syncthreads();
  if (lane == 0) atomicMax(&kmax_bits, __float_as_uint(kmx));   // non-negative floats order as bits
  __syncthreads();
  const float inv = kmax_bits ? 1.0f / __uint_as_float(kmax_bits) : 0.0f;
  int bk[KPT];
#pragma unroll
  for (int t = 0; t < KPT; ++t) {
    const int j = tid + 1024 * t;
    const int b = min(kOrderBuckets - 1, (int)((float)kOrderBuckets * sqrtf(key[t] * inv)));
    bk[t] = kOrderBuckets - 1 - b;   // descending: the largest keys first
    if (j < len) atomicAdd(&hist[bk[t]], 1);
  }
  __syncthreads();
  // exclusive scan of the 256 bucket counts (4 waves)
  if (tid < kOrderBuckets) {
    const int v = hist[tid];
    int x = v;
#pragma unroll
    for (int o = 1; o < LANES; o <<= 1) {
      const int y = __shfl_up(x, o);
      if (lane >= o) x += y;
    }
    if (lane == LANES - 1) wsum[tid >> 6] = x;
    hist[tid] = x - v;   // exclusive within the wave
  }
  __syncthreads();
  if (tid < kOrderBuckets) {
    int off = 0;
    for (int w = 0; w < (tid >> 6); ++w) off += wsum[w];
    hist[tid] += off;
  }
  __syncthreads();
#pragma unroll
  for (int t = 0; t < KPT; ++t) {
    const int j = tid + 1024 * t;
    if (j < len) {
      const int pos = hist[bk[t]] + atomicAdd(&cursor[bk[t]], 1);
      perm[start + stride * pos] = start + stride * j;
    }
  }
}

// class 64's capacity (stance variables)
constexpr int kCap64 = 64;
// interior-point class: global S_k slots per CU.  Every layout takes more than a fifth of a
// CU's LDS, so at most kIpmPerCU of its (one-wave) workgroups are resident on a CU at once
// and a claim finds a free slot without waiting (ipm_claim_slot).
constexpr int kIpmPerCU = 4;
template <int NM, bool FULL, bool MG>
constexpr bool ipm_within_slots() {
  return sizeof(IpmSharedT<NM, FULL, MG>) > 160 * 1024 / (kIpmPerCU + 1);
}
static_assert(ipm_within_slots<16, false, true>() && ipm_within_slots<16, true, true>() &&
                  ipm_within_slots<16, false, false>() && ipm_within_slots<16, true, false>() &&
                  ipm_within_slots<kDenseN, false, false>() && ipm_within_slots<kDenseN, true, false>() &&
                  ipm_within_slots<kMaxN, false, false>() && ipm_within_slots<kMaxN, true, false>(),
              "an interior-point layout fits more workgroups on a CU than kIpmPerCU slots");

// Class NV = 64: one 2-wave workgroup per robot of the batch.  Robots with more
// than 64 stance variables are appended to `queue` (when given) for class 96, those
// with more than 96 to `queue_big` (when given) for class 128.
template <bool FULL>
__global__ __launch_bounds__(Cfg<64>::NT) __attribute__((amdgpu_waves_per_eu(2, Cfg<64>::NW))) void mpcqp_kernel_64(
    KParams P, int B, const float* __restrict__ x0g, const float* __restrict__ xrefg,
    const float* __restrict__ contactg, const float* __restrict__ feetg, const float* __restrict__ robotg,
    float* __restrict__ u0g, float* __restrict__ Ug, int* __restrict__ statusg, int* __restrict__ itersg,
    int* __restrict__ queue, int* __restrict__ queue_big, int* __restrict__ queue_ipm, const int* __restrict__ perm) {
  if ((int)blockIdx.x >= B) return;
  int b = xcd_robot(blockIdx.x, B);
  if (perm) b = uni(perm[b]);   // the dispatch order (mpcqp_order_kernel, mode 0)
  __shared__ SharedT<64> sm;
  solve_robot<64, FULL>(P, b, sm, x0g, xrefg, contactg, feetg, robotg, u0g, Ug, statusg, itersg, queue, queue_big,
                  queue_ipm);
}

// Class NV = 96: one 6-wave workgroup (4 x 6 register tiles) per robot queued by
// class 64 (64 < n <= 96: the N = 16 trot / pace / bound schedules); robots with more
// stance variables go on to class 128 through `qout`.  Same launch / reset protocol
// as class 128 below.
template <bool FULL>
__global__ __launch_bounds__(Cfg<96>::NT) __attribute__((amdgpu_waves_per_eu((Cfg<96>::NW + 3) / 4, (Cfg<96>::NW + 3) / 4))) void mpcqp_kernel_96(
    KParams P, const float* __restrict__ x0g, const float* __restrict__ xrefg,
    const float* __restrict__ contactg, const float* __restrict__ feetg, const float* __restrict__ robotg,
    float* __restrict__ u0g, float* __restrict__ Ug, int* __restrict__ statusg, int* __restrict__ itersg,
    int* __restrict__ queue, int* __restrict__ qout, int* __restrict__ q_ipm, int direct_B,
    const int* __restrict__ perm) {
  __shared__ SharedT<96> sm;
  const int tid = threadIdx.x;
  const int k = blockIdx.x;
  if (direct_B > 0) {   // the caller's stance range rules class 64 out: robot = workgroup (or perm[k])
    if (k < direct_B)
      solve_robot<96, FULL>(P, perm ? uni(perm[k]) : k, sm, x0g, xrefg, contactg, feetg, robotg, u0g, Ug, statusg,
                            itersg, qout, nullptr, q_ipm);
    return;
  }
  const int cnt = uni(__hip_atomic_load(&queue[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
  if (k < cnt) {
    const int b = uni(queue[4 + k]);
    solve_robot<96, FULL>(P, b, sm, x0g, xrefg, contactg, feetg, robotg, u0g, Ug, statusg, itersg, qout, nullptr, q_ipm);
    // only the cnt workers count themselves (no contended atomic from the idle rest)
    if (tid == 0 && atomicAdd(&queue[2], 1) == cnt - 1) {
      atomicExch(&queue[0], 0);
      atomicExch(&queue[2], 0);
    }
  }
}

// Class NV = 128: one 8-wave workgroup per queued robot.  The launch has one
// workgroup per robot of the batch (the host cannot know the queue length without a
// sync); the ones beyond the queue count exit at once.  The last queued robot's
// workgroup to finish resets the counters for the next launch (queue[0] = count, queue[2] = finished
// workgroups, queue[4..] = robot indices).  Workloads that fit class 64 skip this
// launch via mpcqp_set_stance_hint.
template <bool FULL>
__global__ __launch_bounds__(Cfg<128>::NT) void mpcqp_kernel_128(
    KParams P, const float* __restrict__ x0g, const float* __restrict__ xrefg,
    const float* __restrict__ contactg, const float* __restrict__ feetg, const float* __restrict__ robotg,
    float* __restrict__ u0g, float* __restrict__ Ug, int* __restrict__ statusg, int* __restrict__ itersg,
    int* __restrict__ queue, int* __restrict__ q_ipm, int direct_B, const int* __restrict__ perm) {
  __shared__ SharedT<128> sm;
  const int tid = threadIdx.x;
  const int k = blockIdx.x;
  if (direct_B > 0) {
    if (k < direct_B)
      solve_robot<128, FULL>(P, perm ? uni(perm[k]) : k, sm, x0g, xrefg, contactg, feetg, robotg, u0g, Ug, statusg,
                             itersg, q_ipm, nullptr, q_ipm);
    return;
  }
  const int cnt = uni(__hip_atomic_load(&queue[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
  if (k < cnt) {
    const int b = uni(queue[4 + k]);
    solve_robot<128, FULL>(P, b, sm, x0g, xrefg, contactg, feetg, robotg, u0g, Ug, statusg, itersg, q_ipm, nullptr, q_ipm);
    // only the cnt workers count themselves (no contended atomic from the idle rest)
    if (tid == 0 && atomicAdd(&queue[2], 1) == cnt - 1) {
      atomicExch(&queue[0], 0);
      atomicExch(&queue[2], 0);
    }
  }
}

// Riccati-factored interior point + active-set polish (mpcqp_ipm.h).  Same launch / reset
// protocol as class 128.  FULL: non-diagonal weights (mpcqp_set_weights).
// A free slot of the interior-point class's global S_k scratch: one bit per slot in `bits`
// (nw words), claimed with atomicOr, released with atomicAnd.  The search terminates: a slot
// holder never waits for anything before it releases its slot, and there are at least as
// many slots as workgroups of the class can be resident at once (kIpmPerCU per CU, every
// layout LDS-bound to at most that: the static_assert above), so a free one exists whenever
// a workgroup searches.  Called by one lane.
__device__ __forceinline__ int ipm_claim_slot(unsigned* bits, int nw, int start) {
  for (int i = 0;; ++i) {
    if (i >= nw) __builtin_amdgcn_s_sleep(2);   // a full sweep found none: back off (never expected)
    const int w = (start + i) % nw;
    unsigned m = ~__hip_atomic_load(&bits[w], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    while (m) {
      const int bit = __builtin_ctz(m);
      const unsigned old = atomicOr(&bits[w], 1u << bit);
      if (!(old & (1u << bit))) return 32 * w + bit;
      m &= ~old & ~(1u << bit);
    }
  }
}

// Large class (n > 128, and every robot at N > 20): one wave per robot; its Riccati S_k in
// a global slot claimed for the robot's solve (sbits: slot bitmap, nsw words)
// One wave per SIMD at most (LDS bounds a CU to 3 or 4 of these workgroups): the wave may take
// the whole 512-register file, so values beyond the 256 arch VGPRs live in AGPRs, not scratch
// XR: an R with cross-leg couplings (full-weight latency layouts only)
template <bool FULL, int NM, bool MG = false, bool XR = false>
__global__ __launch_bounds__(LANES) __attribute__((amdgpu_waves_per_eu(1, 1))) void mpcqp_kernel_ipm(
    KParams P, const float* __restrict__ x0g, const float* __restrict__ xrefg,
    const float* __restrict__ contactg, const float* __restrict__ feetg, const float* __restrict__ robotg,
    float* __restrict__ u0g, float* __restrict__ Ug, int* __restrict__ statusg, int* __restrict__ itersg,
    int* __restrict__ queue, int direct_B, double* __restrict__ sscratch, unsigned* __restrict__ sbits,
    int nsw) {
  __shared__ IpmSharedT<NM, FULL, MG> sm;
  const int tid = threadIdx.x;
  const int k = blockIdx.x;
  // direct_B > 0: the caller's stance range (or N > 20) rules the dense classes out, robot = k
  const bool direct = direct_B > 0;
  const int cnt = direct ? direct_B : uni(__hip_atomic_load(&queue[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
  if (k >= cnt) return;   // idle workgroups touch no counter
  const int b = direct ? k : uni(queue[4 + k]);
  int slot = 0;
  if (tid == 0) slot = ipm_claim_slot(sbits, nsw, k % nsw);
  slot = __builtin_amdgcn_readlane(slot, 0);
  solve_robot_ipm<FULL, NM, MG, XR>(P, b, sm, sscratch + (size_t)slot * IpmSlot<NM>::SIZE, x0g, xrefg, contactg, feetg, robotg, u0g,
                            Ug, statusg, itersg);
  if (tid == 0) {
    atomicAnd(&sbits[slot >> 5], ~(1u << (slot & 31)));   // the solve's S_k reads are done
    // only the queued robots count themselves; the last one resets the queue
    if (!direct && atomicAdd(&queue[2], 1) == cnt - 1) {
      atomicExch(&queue[0], 0);
      atomicExch(&queue[2], 0);
    }
  }
}

}  // namespace

// ============================================================== C ABI
// Device queues of one stream: three queues of [count, next, finished, pad, robots...
// (cap)] -- class 64 -> class 96, -> class 128, -> the interior-point class.  Calls on
// one stream are ordered, so the count / reset protocol of the queued kernels is
// safe; calls on different streams of one context use different queue sets.
struct QueueSet {
  hipStream_t stream;
  int cap;
  int* buf;
  unsigned long long used;   // last use (LRU eviction beyond kMaxQueueSets streams)
  // the interior-point class runs on a side stream forked from `stream` after the first
  // (routing) class and joined back at the end of the call (created on first use)
  hipStream_t side;
  hipEvent_t ev_fork, ev_join;
  hipEvent_t ev_done;   // recorded on `stream` after each call's last launch (eviction waits on it)
};

// Releases a queue set's device resources (the caller has synchronised the device).
static void release_set(QueueSet& q) {
  if (q.buf) (void)hipFree(q.buf);
  if (q.ev_fork) (void)hipEventDestroy(q.ev_fork);
  if (q.ev_join) (void)hipEventDestroy(q.ev_join);
  if (q.ev_done) (void)hipEventDestroy(q.ev_done);
  q.ev_done = nullptr;
  if (q.side) (void)hipStreamDestroy(q.side);
  q.buf = nullptr;
  q.ev_fork = q.ev_join = nullptr;
  q.side = nullptr;
}

struct mpcqp_ctx {
  mpcqp_params params;
  int device;
  int stance_hint;   // max stance foot-steps per robot promised by the caller (0: none)
  int stance_min;    // min stance foot-steps per robot promised by the caller
  int order;         // dispatch order (mpcqp_set_order): 1 = predicted-cost order, 0 = batch order
  int ncu;
  std::vector<QueueSet> queues;
  unsigned long long use_clock;
  // the interior-point class's global slots (Riccati S_k; at N <= 16 also M_k, M_k^T and the
  // saved iterate): kIpmPerCU per CU, one pool for every stream of the context (the slots in
  // use never exceed the class's resident workgroups, whichever launches they belong to),
  // ipm_slot_doubles(horizon) each, then the slot bitmap; allocated on first use
  double* sscratch;
  int sslots;
  double* wdev;       // full Q (13 x 13) then R (12 x 12) on the device (mpcqp_set_weights); nullptr: diagonal
  bool xr;            // R couples different legs: the interior-point class's XR instantiations
  double q_full[13 * 13];   // the current weights as whole matrices (host copies: a NULL argument
  double r_full[12 * 12];   // of mpcqp_set_weights keeps that matrix, off-diagonal entries included)
  std::vector<double*> retired;   // earlier full-weight buffers (in-flight solves may read them)
  unsigned char* warm;   // warm-start memory (caller-owned device buffer), mpcqp_set_warm_start
  int warm_cap;
  double dt_control;  // planner constants (mpcqp_set_planner)
  double gravity;
  double max_pos_error;
  std::string err;
};

static int set_err(mpcqp_ctx* ctx, int code, const std::string& msg) {
  if (ctx) ctx->err = msg;
  return code;
}

// Makes the context's device current for one ABI call and restores the caller's.
struct DeviceScope {
  int prev = -1;
  bool ok = false;
  explicit DeviceScope(int dev) {
    if (hipGetDevice(&prev) != hipSuccess) prev = -1;
    ok = hipSetDevice(dev) == hipSuccess;
  }
  ~DeviceScope() {
    if (prev >= 0) (void)hipSetDevice(prev);
  }
};

// At most this many streams keep a queue set; a new stream beyond them takes over the
// least recently used set with its buffers, once the event recorded after that set's last
// call has completed (its stream may still run launches that use it, and may already have
// been destroyed by the caller: the event outlives it).  No device-wide synchronisation.
constexpr int kMaxQueueSets = 8;
// Full-weight buffers retired by mpcqp_set_weights before one device-wide release.
constexpr size_t kMaxRetired = 64;

// The queue set of `st`, holding at least `batch` robots per queue (grown on demand;
// the old buffer is freed once the stream's earlier launches are done).
static QueueSet* stream_queues(mpcqp_ctx* ctx, hipStream_t st, int batch, int* err, int* cap) {
  *err = MPCQP_OK;
  QueueSet* qs = nullptr;
  for (auto& q : ctx->queues)
    if (q.stream == st) qs = &q;
  if (qs) qs->used = ++ctx->use_clock;
  if (qs && qs->cap >= batch) {
    *cap = qs->cap;
    return qs;
  }
  if (!qs && (int)ctx->queues.size() >= kMaxQueueSets) {
    QueueSet* lru = &ctx->queues[0];
    for (auto& q : ctx->queues)
      if (q.used < lru->used) lru = &q;
    // ev_done is recorded after every call that launched anything on the set, on its error
    // paths too; without one, wait for the whole device
    const hipError_t se = lru->ev_done ? hipEventSynchronize(lru->ev_done) : hipDeviceSynchronize();
    if (se != hipSuccess) {
      *err = set_err(ctx, MPCQP_ERR_HIP, "queue eviction: sync failed");
      return nullptr;
    }
    // every launch that used the set is done: its queues are back at rest (each kernel
    // resets its header) -- the new stream reuses them as they are
    lru->stream = st;
    lru->used = ++ctx->use_clock;
    qs = lru;
  }
  if (!qs) {
    hipEvent_t ev = nullptr;
    if (hipEventCreateWithFlags(&ev, hipEventDisableTiming) != hipSuccess) {
      *err = set_err(ctx, MPCQP_ERR_HIP, "queue event creation failed");
      return nullptr;
    }
    ctx->queues.push_back(QueueSet{st, 0, nullptr, ++ctx->use_clock, nullptr, nullptr, nullptr, ev});
    qs = &ctx->queues.back();
  }
  if (qs->buf) {
    if (hipStreamSynchronize(st) != hipSuccess) {
      *err = set_err(ctx, MPCQP_ERR_HIP, "queue growth: stream sync failed");
      return nullptr;
    }
    (void)hipFree(qs->buf);
    qs->buf = nullptr;
    qs->cap = 0;
  }
  // three queues of 4 + batch ints, then the dispatch order (mpcqp_order_kernel) of batch ints
  const size_t bytes = sizeof(int) * (3 * (4 + (size_t)batch) + (size_t)batch);
  if (hipMalloc(&qs->buf, bytes) != hipSuccess) {
    qs->buf = nullptr;
    *err = set_err(ctx, MPCQP_ERR_ALLOC, "queue allocation failed");
    return nullptr;
  }
  if (hipMemsetAsync(qs->buf, 0, bytes, st) != hipSuccess) {
    *err = set_err(ctx, MPCQP_ERR_HIP, "queue init failed");
    return nullptr;
  }
  qs->cap = batch;
  *cap = batch;
  return qs;
}

// The side stream and fork / join events of a queue set (created on first use).
static bool side_stream(QueueSet* qs) {
  if (!qs->side && hipStreamCreateWithFlags(&qs->side, hipStreamNonBlocking) != hipSuccess) {
    qs->side = nullptr;
    return false;
  }
  if (!qs->ev_fork && hipEventCreateWithFlags(&qs->ev_fork, hipEventDisableTiming) != hipSuccess) {
    qs->ev_fork = nullptr;
    return false;
  }
  if (!qs->ev_join && hipEventCreateWithFlags(&qs->ev_join, hipEventDisableTiming) != hipSuccess) {
    qs->ev_join = nullptr;
    return false;
  }
  return true;
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
  ctx->stance_min = 0;
  ctx->order = 1;
  ctx->ncu = 0;
  ctx->use_clock = 0;
  ctx->sscratch = nullptr;
  ctx->sslots = 0;
  ctx->wdev = nullptr;
  ctx->xr = false;
  ctx->warm = nullptr;
  ctx->warm_cap = 0;
  for (int i = 0; i < 13 * 13; ++i) ctx->q_full[i] = (i % 14 == 0) ? p->q_diag[i / 14] : 0.0;
  for (int i = 0; i < 12 * 12; ++i) ctx->r_full[i] = (i % 13 == 0) ? p->r_diag[i / 13] : 0.0;
  ctx->dt_control = 0.001;    // linear_mpc_configs.py:6
  ctx->gravity = 9.81;        // linear_mpc_configs.py:13
  ctx->max_pos_error = 0.1;   // mpc.py:121
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, device) == hipSuccess) ctx->ncu = prop.multiProcessorCount;
  if (ctx->ncu <= 0) ctx->ncu = 256;
  *out = ctx;
  return MPCQP_OK;
}

int mpcqp_set_warm_start(mpcqp_ctx* ctx, void* memory, int32_t capacity) {
  if (!ctx) return MPCQP_ERR_ARG;
  if (capacity < 0 || (capacity > 0 && !memory))
    return set_err(ctx, MPCQP_ERR_ARG, "warm start: capacity < 0, or no memory for capacity > 0");
  ctx->warm = capacity > 0 ? static_cast<unsigned char*>(memory) : nullptr;
  ctx->warm_cap = capacity > 0 ? capacity : 0;
  return MPCQP_OK;
}

int mpcqp_set_order(mpcqp_ctx* ctx, int32_t mode) {
  if (!ctx) return MPCQP_ERR_ARG;
  if (mode != 0 && mode != 1) return set_err(ctx, MPCQP_ERR_ARG, "order: mode must be 0 or 1");
  ctx->order = mode;
  return MPCQP_OK;
}

int mpcqp_set_stance_hint(mpcqp_ctx* ctx, int32_t max_stance) {
  return mpcqp_set_stance_range(ctx, 0, max_stance);
}

int mpcqp_set_stance_range(mpcqp_ctx* ctx, int32_t min_stance, int32_t max_stance) {
  if (!ctx) return MPCQP_ERR_ARG;
  if (min_stance < 0 || max_stance < 0 || (max_stance > 0 && min_stance > max_stance))
    return set_err(ctx, MPCQP_ERR_ARG, "stance range: min > max or negative");
  // a schedule has at most 4 N stance foot-steps: a larger minimum would route the whole
  // batch past every class mpcqp_solve launches (and leave the outputs unwritten)
  if (min_stance > 4 * ctx->params.horizon)
    return set_err(ctx, MPCQP_ERR_ARG, "stance range: min_stance > 4 * horizon");
  ctx->stance_min = min_stance;
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
  DeviceScope dev(ctx->device);
  if (!dev.ok) return set_err(ctx, MPCQP_ERR_HIP, "hipSetDevice failed");
  KParams kp;
  kp.N = ctx->params.horizon;
  kp.max_iter = ctx->params.max_iter;
  kp.dt = ctx->params.dt;
  for (int i = 0; i < NX; ++i) kp.q[i] = ctx->params.q_diag[i];
  for (int i = 0; i < NU; ++i) kp.r[i] = ctx->params.r_diag[i];
  kp.wfull = ctx->wdev;
  kp.warm = ctx->warm;
  kp.warm_cap = ctx->warm_cap;
  const bool full = ctx->wdev != nullptr;   // the dense classes' full-weight instantiations
  hipStream_t st = (hipStream_t)stream;
  // A robot has n = 3 * #stance <= 12 N variables.  Robots with more than 64 are queued
  // for class 96, more than 96 for class 128, more than 128 for the interior-point
  // class -- each queued launch skipped when no robot can need it (horizon, or the
  // caller's stance range).  When the range rules out the smaller classes, the first
  // class that can be needed takes the batch directly (one workgroup per robot) and
  // routes the larger robots on.
  const int nmax_h = 12 * kp.N;
  const int nmax = ctx->stance_hint > 0 && 3 * ctx->stance_hint < nmax_h ? 3 * ctx->stance_hint : nmax_h;
  const int nmin = 3 * ctx->stance_min;
  // horizons beyond the dense classes' LDS layouts (N > kDenseN): the interior-point class
  // takes the whole batch directly, whatever the stance counts
  const bool ipm_only = kp.N > kDenseN;
  const bool large = ipm_only || nmax > kCap64, huge = !ipm_only && nmax > 96, giant = ipm_only || nmax > 128;
  // the first class launched: 0 = class 64, 1 = 96, 2 = 128, 3 = interior point
  // When the interior-point class may be needed beside the dense ones, class 64 routes the
  // batch (a formulation-stage pass, microseconds) so the interior-point launch forks onto
  // its side stream at once -- a dense class taking the batch directly would route its
  // standing robots only as its own workgroups run, and the fork would wait for all of it.
  const int first = ipm_only || nmin > 128 ? 3 : giant ? 0 : nmin > 96 ? 2 : nmin > kCap64 ? 1 : 0;
  // the dispatch order (mpcqp_order_kernel) of the first class's launch: class 64 sorts its 8 XCD
  // ranges (each <= kOrderMax robots), classes 96 / 128 taking the batch directly sort interleaved
  // segments of <= kOrderSeg; the interior-point class and small batches keep the batch order
  // -- only when the batch queues on the CUs: a batch the chip holds at once (config 2: 1024
  // robots = 4 per CU) gains nothing from its order (the heaviest robots' CU-mates are lighter
  // either way, measured) and would pay the sort launch (config 2 -1.5 %, profiles/r5_combo/)
  const int resident = (first == 0 ? 4 : 1) * ctx->ncu;   // class 64: 4 workgroups per CU; 96 / 128: 1
  const bool use_order = ctx->order && batch >= kOrderMin && batch > resident && first < 3 &&
                         (first > 0 || batch <= 8 * kOrderMax);
  int* q = nullptr;
  QueueSet* qs = nullptr;
  int cap = 0;
  if (large || use_order) {
    int qerr = MPCQP_OK;
    qs = stream_queues(ctx, st, batch, &qerr, &cap);
    if (!qs) return qerr;
    q = qs->buf;
  }
  const size_t sstride = (size_t)ipm_slot_doubles(kp.N);   // doubles per slot
  if (giant && !ctx->sscratch) {   // the interior-point class's global slots (first use)
    const int slots = 32 * ((kIpmPerCU * ctx->ncu + 31) / 32);
    const size_t sbytes = sizeof(double) * sstride * (size_t)slots;
    if (hipMalloc(&ctx->sscratch, sbytes + slots / 8) != hipSuccess) {
      ctx->sscratch = nullptr;
      return set_err(ctx, MPCQP_ERR_ALLOC, "interior-point scratch allocation failed");
    }
    // the slot bitmap after the slots: all free (every solve releases its slot); cleared on this
    // stream and waited for, so a launch on any stream of the context finds it cleared
    if (hipMemsetAsync((char*)ctx->sscratch + sbytes, 0, slots / 8, st) != hipSuccess ||
        hipStreamSynchronize(st) != hipSuccess) {
      (void)hipFree(ctx->sscratch);
      ctx->sscratch = nullptr;
      return set_err(ctx, MPCQP_ERR_HIP, "interior-point scratch init failed");
    }
    ctx->sslots = slots;
  }
  // the interior-point class (one wave per robot, latency-bound) on a side stream as soon
  // as the first class has routed its robots, beside classes 96 / 128 instead of behind
  // them; the caller's stream waits for it at the end of the call
  const bool fork = giant && first < 3 && side_stream(qs);
  bool ipm_done = false;
  auto launch_ipm = [&](hipStream_t s) -> hipError_t {
    // the LDS layout for the horizon: N <= 16 (the reference's default) three robots per CU,
    // N <= 20 one, longer horizons (up to kMaxN) one
    // N <= 16: the throughput layout (four robots per CU, M_k in the global slot) when the
    // class takes a batch larger than three robots per CU can hold at once; otherwise -- a
    // single drop-in robot, or robots queued from a mixed batch, whose latency is the
    // launch's tail -- the latency layout (M_k in LDS, three per CU)
    // A cross-leg R (ctx->xr) takes the XR instantiations: 12 x 12 stage weights, latency layouts.
    const bool thru = first == 3 && batch > 3 * ctx->ncu;
    auto kern = ctx->xr ? (kp.N <= 16 ? mpcqp_kernel_ipm<true, 16, false, true>
                           : kp.N <= kDenseN ? mpcqp_kernel_ipm<true, kDenseN, false, true>
                                             : mpcqp_kernel_ipm<true, kMaxN, false, true>)
                : kp.N <= 16 ? (thru ? (full ? mpcqp_kernel_ipm<true, 16, true> : mpcqp_kernel_ipm<false, 16, true>)
                                     : (full ? mpcqp_kernel_ipm<true, 16> : mpcqp_kernel_ipm<false, 16>))
                : kp.N <= kDenseN ? (full ? mpcqp_kernel_ipm<true, kDenseN> : mpcqp_kernel_ipm<false, kDenseN>)
                                  : (full ? mpcqp_kernel_ipm<true, kMaxN> : mpcqp_kernel_ipm<false, kMaxN>);
    // one workgroup per robot of the batch (the queued ones beyond the count exit at once)
    unsigned* sbits = (unsigned*)(ctx->sscratch + sstride * ctx->sslots);
    hipLaunchKernelGGL(kern, dim3(batch), dim3(LANES), 0, s, kp, x0, xref, contact, feet, robot, u0, U,
                       (int*)status, (int*)iters, q + 2 * (4 + (size_t)cap), first == 3 ? (int)batch : 0,
                       ctx->sscratch, sbits, ctx->sslots / 32);
    ipm_done = true;
    return hipGetLastError();
  };
  auto fork_ipm = [&]() -> int {
    if (!fork || ipm_done) return MPCQP_OK;
    if (hipEventRecord(qs->ev_fork, st) != hipSuccess || hipStreamWaitEvent(qs->side, qs->ev_fork, 0) != hipSuccess)
      return set_err(ctx, MPCQP_ERR_HIP, "interior-point fork failed");
    const hipError_t le = launch_ipm(qs->side);
    if (le != hipSuccess) return set_err(ctx, MPCQP_ERR_HIP, std::string("launch (ipm): ") + hipGetErrorString(le));
    if (hipEventRecord(qs->ev_join, qs->side) != hipSuccess) return set_err(ctx, MPCQP_ERR_HIP, "join record failed");
    return MPCQP_OK;
  };
  const size_t qstride = 4 + (size_t)cap;   // the set's layout: three queues of 4 + cap ints, the order
  int* q1 = large ? q : nullptr;
  int* perm = use_order ? q + 3 * qstride : nullptr;
  int* q2 = huge ? q + qstride : nullptr;
  int* q3 = giant ? q + 2 * qstride : nullptr;
  hipError_t e = hipSuccess;
  int fe = MPCQP_OK;
  // an error after a launch still marks the queue set's last use: eviction waits on ev_done
  auto failed = [&](int code) -> int {
    if (fork && ipm_done) (void)hipStreamWaitEvent(st, qs->ev_join, 0);   // the side stream's launch too
    if (qs) (void)hipEventRecord(qs->ev_done, st);
    return code;
  };
  if (use_order) {
    const int segs = first == 0 ? 8 : (int)((batch + kOrderSeg - 1) / kOrderSeg);
    hipLaunchKernelGGL(mpcqp_order_kernel, dim3(segs), dim3(1024), 0, st, (int)batch, kp.N, x0, xref, perm,
                       first == 0 ? 0 : 1);
    e = hipGetLastError();
    if (e != hipSuccess) return failed(set_err(ctx, MPCQP_ERR_HIP, std::string("launch (order): ") + hipGetErrorString(e)));
  }
  if (first == 0) {
    hipLaunchKernelGGL(full ? mpcqp_kernel_64<true> : mpcqp_kernel_64<false>, dim3(batch), dim3(Cfg<64>::NT),
                       kDiagLds, st, kp, (int)batch, x0, xref, contact,
                       feet, robot, u0, U, (int*)status, (int*)iters, q1, q2, q3, perm);
    e = hipGetLastError();
    if (e != hipSuccess) return failed(set_err(ctx, MPCQP_ERR_HIP, std::string("launch: ") + hipGetErrorString(e)));
    if ((fe = fork_ipm()) != MPCQP_OK) return failed(fe);
  }
  if (large && first <= 1) {
    hipLaunchKernelGGL(full ? mpcqp_kernel_96<true> : mpcqp_kernel_96<false>, dim3(batch), dim3(Cfg<96>::NT), 0, st, kp, x0, xref, contact, feet, robot,
                       u0, U, (int*)status, (int*)iters, q1, q2, q3, first == 1 ? (int)batch : 0,
                       first == 1 ? perm : nullptr);
    e = hipGetLastError();
    if (e != hipSuccess) return failed(set_err(ctx, MPCQP_ERR_HIP, std::string("launch (96): ") + hipGetErrorString(e)));
    if ((fe = fork_ipm()) != MPCQP_OK) return failed(fe);
  }
  if (huge && first <= 2) {
    hipLaunchKernelGGL(full ? mpcqp_kernel_128<true> : mpcqp_kernel_128<false>, dim3(batch), dim3(Cfg<128>::NT), 0, st, kp, x0, xref, contact, feet, robot,
                       u0, U, (int*)status, (int*)iters, q2, q3, first == 2 ? (int)batch : 0,
                       first == 2 ? perm : nullptr);
    e = hipGetLastError();
    if (e != hipSuccess) return failed(set_err(ctx, MPCQP_ERR_HIP, std::string("launch (128): ") + hipGetErrorString(e)));
    if ((fe = fork_ipm()) != MPCQP_OK) return failed(fe);
  }
  if (giant && !ipm_done) {   // the interior-point class takes the batch directly (or no side stream)
    e = launch_ipm(st);
    if (e != hipSuccess) return failed(set_err(ctx, MPCQP_ERR_HIP, std::string("launch (ipm): ") + hipGetErrorString(e)));
  } else if (fork && hipStreamWaitEvent(st, qs->ev_join, 0) != hipSuccess) {
    return failed(set_err(ctx, MPCQP_ERR_HIP, "interior-point join failed"));
  }
  if (qs && hipEventRecord(qs->ev_done, st) != hipSuccess) return set_err(ctx, MPCQP_ERR_HIP, "queue event record failed");
  return MPCQP_OK;
}

int mpcqp_set_weights(mpcqp_ctx* ctx, const double* Q, const double* R) {
  if (!ctx) return MPCQP_ERR_ARG;
  double q[NX * NX], r[NU * NU];
  memcpy(q, Q ? Q : ctx->q_full, sizeof(q));   // NULL keeps the current matrix
  memcpy(r, R ? R : ctx->r_full, sizeof(r));
  // symmetric and finite (the reference's kron(I_N, Q) enters H = 2 Su^T Qbar Su; an
  // asymmetric Q would make H asymmetric, which no QP solver of the reference accepts)
  double qmax = 0.0, rmax = 0.0;
  bool finite = true;   // per entry: fmax drops a NaN operand
  for (int i = 0; i < NX * NX; ++i) {
    finite = finite && std::isfinite(q[i]);
    qmax = fmax(qmax, fabs(q[i]));
  }
  for (int i = 0; i < NU * NU; ++i) {
    finite = finite && std::isfinite(r[i]);
    rmax = fmax(rmax, fabs(r[i]));
  }
  if (!finite) return set_err(ctx, MPCQP_ERR_ARG, "weights: non-finite entry");
  bool diag = true, cross = false;
  for (int i = 0; i < NX; ++i)
    for (int j = 0; j < NX; ++j) {
      if (fabs(q[i * NX + j] - q[j * NX + i]) > 1e-12 * qmax) return set_err(ctx, MPCQP_ERR_ARG, "weights: Q not symmetric");
      if (i != j && q[i * NX + j] != 0.0) diag = false;
    }
  for (int i = 0; i < NU; ++i)
    for (int j = 0; j < NU; ++j) {
      if (fabs(r[i * NU + j] - r[j * NU + i]) > 1e-12 * rmax) return set_err(ctx, MPCQP_ERR_ARG, "weights: R not symmetric");
      if (i != j && r[i * NU + j] != 0.0) diag = false;
      if (i / 3 != j / 3 && r[i * NU + j] != 0.0) cross = true;
    }
  DeviceScope dev(ctx->device);
  if (!dev.ok) return set_err(ctx, MPCQP_ERR_HIP, "hipSetDevice failed");
  // Device work first, into a fresh buffer; the context changes only once it all succeeded
  // (a failed allocation or upload leaves the previous weights in force).
  double* nb = nullptr;
  if (!diag) {
    if (hipMalloc(&nb, sizeof(double) * (NX * NX + NU * NU)) != hipSuccess)
      return set_err(ctx, MPCQP_ERR_ALLOC, "weights: allocation failed");
    double host[NX * NX + NU * NU];
    memcpy(host, q, sizeof(q));
    memcpy(host + NX * NX, r, sizeof(r));
    if (hipMemcpy(nb, host, sizeof(host), hipMemcpyHostToDevice) != hipSuccess) {
      (void)hipFree(nb);
      return set_err(ctx, MPCQP_ERR_HIP, "weights: upload failed");
    }
  }
  // launches on any stream (non-blocking ones included) may still read the previous
  // buffer: it is retired, not freed (2.5 KB each), and released at mpcqp_destroy -- or,
  // past kMaxRetired changes, all at once after a device synchronisation
  if (ctx->wdev) {
    if (ctx->retired.size() >= kMaxRetired) {
      if (hipDeviceSynchronize() != hipSuccess) {
        if (nb) (void)hipFree(nb);
        return set_err(ctx, MPCQP_ERR_HIP, "weights: device sync failed");
      }
      for (double* o : ctx->retired) (void)hipFree(o);
      ctx->retired.clear();
    }
    ctx->retired.push_back(ctx->wdev);
  }
  ctx->wdev = nb;   // nullptr: the diagonal fast path (the weights live in the kernel arguments)
  ctx->xr = cross;
  memcpy(ctx->q_full, q, sizeof(q));
  memcpy(ctx->r_full, r, sizeof(r));
  for (int i = 0; i < NX; ++i) ctx->params.q_diag[i] = q[i * (NX + 1)];
  for (int i = 0; i < NU; ++i) ctx->params.r_diag[i] = r[i * (NU + 1)];
  return MPCQP_OK;
}

int mpcqp_set_planner(mpcqp_ctx* ctx, double dt_control, double gravity, double max_pos_error) {
  if (!ctx || !(dt_control >= 0.0) || !(max_pos_error >= 0.0)) return MPCQP_ERR_ARG;
  ctx->dt_control = dt_control;
  ctx->gravity = gravity;
  ctx->max_pos_error = max_pos_error;
  return MPCQP_OK;
}

static int launch_plan(mpcqp_ctx* ctx, int32_t batch, int32_t flags, int root_layout, const float* quat,
                       const float* pos, const float* omega, const float* vel, const float* rot,
                       const double* vel_body_des, const double* yaw_rate_des, const int32_t* gait,
                       const int32_t* iteration, const float* height_des, double* plan_state, float* x0,
                       float* xref, float* contact, void* stream) {
  if (!ctx) return MPCQP_ERR_ARG;
  if (batch < 0) return set_err(ctx, MPCQP_ERR_ARG, "batch < 0");
  if (batch == 0) return MPCQP_OK;
  if (!quat || (!root_layout && (!pos || !omega || !vel)) || !vel_body_des || !yaw_rate_des || !plan_state ||
      !x0)
    return set_err(ctx, MPCQP_ERR_ARG, "null planner input/output pointer");
  if (flags & ~(MPCQP_PLAN_REFERENCE | MPCQP_PLAN_NO_INTEGRATE))
    return set_err(ctx, MPCQP_ERR_ARG, "unknown planner flags");
  const int mpc_tick = (flags & MPCQP_PLAN_REFERENCE) ? 1 : 0;
  if (mpc_tick && (!height_des || !xref))
    return set_err(ctx, MPCQP_ERR_ARG, "null height/xref pointer on an MPC tick");
  if (mpc_tick && gait && (!iteration || !contact))
    return set_err(ctx, MPCQP_ERR_ARG, "gait given without iteration/contact");
  DeviceScope dev(ctx->device);
  if (!dev.ok) return set_err(ctx, MPCQP_ERR_HIP, "hipSetDevice failed");
  PlanParams pp;
  pp.N = ctx->params.horizon;
  pp.mpc_tick = mpc_tick;
  pp.root_layout = root_layout;
  pp.integrate = (flags & MPCQP_PLAN_NO_INTEGRATE) ? 0 : 1;
  pp.dt = ctx->params.dt;
  pp.dt_control = ctx->dt_control;
  pp.gravity = ctx->gravity;
  pp.max_pos_error = ctx->max_pos_error;
  hipLaunchKernelGGL(mpcqp_plan_kernel, dim3((batch + kPlanRobots - 1) / kPlanRobots), dim3(kPlanThreads), 0,
                     (hipStream_t)stream, pp, (int)batch, quat, pos, omega, vel, rot, vel_body_des, yaw_rate_des,
                     gait, iteration, height_des, plan_state, x0, xref, contact);
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) return set_err(ctx, MPCQP_ERR_HIP, std::string("plan launch: ") + hipGetErrorString(e));
  return MPCQP_OK;
}

int mpcqp_plan(mpcqp_ctx* ctx, int32_t batch, int32_t flags, const float* quat, const float* pos,
               const float* omega, const float* vel, const float* rot, const double* vel_body_des,
               const double* yaw_rate_des, const int32_t* gait, const int32_t* iteration,
               const float* height_des, double* plan_state, float* x0, float* xref, float* contact,
               void* stream) {
  return launch_plan(ctx, batch, flags, 0, quat, pos, omega, vel, rot, vel_body_des, yaw_rate_des, gait,
                     iteration, height_des, plan_state, x0, xref, contact, stream);
}

int mpcqp_plan_root_states(mpcqp_ctx* ctx, int32_t batch, int32_t flags, const float* root_states,
                           const double* vel_body_des, const double* yaw_rate_des, const int32_t* gait,
                           const int32_t* iteration, const float* height_des, double* plan_state, float* x0,
                           float* xref, float* contact, void* stream) {
  return launch_plan(ctx, batch, flags, 1, root_states, nullptr, nullptr, nullptr, nullptr, vel_body_des,
                     yaw_rate_des, gait, iteration, height_des, plan_state, x0, xref, contact, stream);
}

int mpcqp_stance_torques(mpcqp_ctx* ctx, int32_t batch, const float* jac, const float* contact,
                         int32_t contact_stride, const float* u0, float* tau, void* stream) {
  if (!ctx) return MPCQP_ERR_ARG;
  if (batch < 0 || contact_stride < 4) return set_err(ctx, MPCQP_ERR_ARG, "batch < 0 or contact_stride < 4");
  if (batch == 0) return MPCQP_OK;
  if (!jac || !contact || !u0 || !tau) return set_err(ctx, MPCQP_ERR_ARG, "null torque pointer");
  DeviceScope dev(ctx->device);
  if (!dev.ok) return set_err(ctx, MPCQP_ERR_HIP, "hipSetDevice failed");
  const int threads = (int)batch * 12;
  hipLaunchKernelGGL(mpcqp_stance_torque_kernel, dim3((threads + 255) / 256), dim3(256), 0, (hipStream_t)stream,
                     (int)batch, jac, contact, (int)contact_stride, u0, tau);
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) return set_err(ctx, MPCQP_ERR_HIP, std::string("torque launch: ") + hipGetErrorString(e));
  return MPCQP_OK;
}

int mpcqp_destroy(mpcqp_ctx* ctx) {
  if (ctx) {
    DeviceScope dev(ctx->device);
    // hipFree synchronises the device before releasing the memory: no per-stream sync
    // (a recorded stream may already have been destroyed by the caller)
    for (auto& q : ctx->queues) release_set(q);
    if (ctx->sscratch) (void)hipFree(ctx->sscratch);
    if (ctx->wdev) (void)hipFree(ctx->wdev);
    for (double* o : ctx->retired) (void)hipFree(o);
  }
  delete ctx;
  return MPCQP_OK;
}

const char* mpcqp_last_error(const mpcqp_ctx* ctx) { return ctx ? ctx->err.c_str() : "null context"; }

}  // extern "C"
