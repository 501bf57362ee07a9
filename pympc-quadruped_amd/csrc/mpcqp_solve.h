// mpcqp_solve.h -- one robot's formulate + solve by one workgroup (included by
// mpcqp.hip inside its anonymous namespace).
//
// Capacity class NV (stance variables n = 3 * #stance <= NV):
//   NV =  64: 2 waves (128 threads) per robot -- every trot/pace/bound schedule at N <= 10
//   NV =  96: 6 waves (384 threads) per robot -- N = 16 schedules (n <= 96)
//   NV = 128: 8 waves (512 threads) per robot -- N = 20 schedules, standing at N <= 10
// Register tiles: lane t = (tr, tc) = (t / TCN, t % TCN) holds rows 4tr..4tr+3 and
// columns TW tc..TW tc+TW-1 of each NV x NV matrix (TW = 8: 32 doubles per matrix
// per lane; class 96 uses TW = 6 -- 24 doubles, and a foot-step's 3 columns never
// straddle two tiles).
//
// Solver: Goldfarb-Idnani dual active set (Math. Prog. 27, 1983) on
//   min 1/2 x^T H x + g^T x   s.t.  a_c . x >= b_c  (6 one-sided cone rows per foot-step)
// in "projected" form.  With W = H^-1 and the active rows A:
//   P = W - (A W)^T (A W A^T)^-1 (A W)     (n x n, reduced inverse Hessian)
//   R = (A W A^T)^-1 A W                   (slots x n)
// the primal / dual step directions for a violated row p are z = P a_p and
// r = R a_p; a_p touches the 3 variables of one foot-step, so both are
// combinations of 3 register columns (no matrix-vector product per iteration).
// Adding p into free slot q:   P -= z z^T / s,   R -= (r - e_q) z^T / s   (s = a_p . z)
// Dropping slot l (eta = Minv_ll, y = Minv[:, l] = R H R_l^T):
//                              P += R_l^T R_l / eta,   R -= y R_l / eta,  R_l = 0.
// Scalar state (constraint values s, x, multipliers u, the active-slot mask) is
// kept redundantly by every wave, so one iteration needs ONE workgroup barrier
// (the z / r exchange) and every wave reaches the same decisions.

template <int NV>
struct Cfg {
  // tile width: 4 x TW register tiles
  static constexpr int TW = NV == 96 ? 6 : 8;
  static constexpr int NW = NV * NV / (4 * TW * LANES);   // waves per robot
  static constexpr int NT = NW * LANES;
  static constexpr int TCN = NV / TW;         // tile columns (lanes per tile row)
  static constexpr int RPW = 256 / TCN;       // tile rows (slots / variables) per wave
  static constexpr int CPL = NV / 32;         // constraint rows per lane (m = 6S <= 2NV)
  static constexpr int VPL = (NV + LANES - 1) / LANES;   // variables / slots per lane
  static constexpr int VEC = VPL * LANES;     // LDS vector length (entries >= NV are padding)
  // The sweep's pivot columns: each tile column's TW-double slice at a stride of TS doubles.
  // ds_read_b128 serves a wave in four 16-lane groups that each hold every tile column (class
  // 128) or every one twice (class 64); at a 64-B stride the slices fold onto 4 (2) of the
  // 256-B bank row's 16 slots, a 4-way (2-way) conflict.  80 B puts the 16 (8) slices on
  // distinct slots; class 96's 48-B stride already does.
  static constexpr int TS = TW == 8 ? 10 : TW;
  static constexpr int SVEC = TW == 8 ? TCN * TS : VEC;   // class 96: the unpadded vectors
  static_assert(NW * LANES * 4 * TW == NV * NV, "4 x TW tiles");
  static_assert(TCN == 8 || TCN == 16, "tile rows are reduced over 8 or 16 lanes");
};

// Every class keeps a copy of H (its register tiles, lane-interleaved) in LDS for
// the drop path, in the space of the formulation scratch, which is dead once H is
// built: 32 KB for class 64 (4 robots still share a CU's 160 KB), 72 / 128 KB for
// classes 96 / 128, which hold one robot per CU anyway (VGPR-bound).
template <int NV>
struct FormArea {
  Form f;
  FormY fy;
  d2 mt_tab[kDenseN * kDenseN];   // (Ta, m) of every foot-step step pair (ja, jb) for the diagonal-Q H build
};
template <int NV>
struct alignas(16) SharedT {
  static constexpr bool kPair = NV <= 96;   // pair steps in classes 64 / 96 (class 128: no VGPRs to spare)
  union {
    FormArea<NV> fa;
    double ht[NV * NV];   // elements (e, e + 1) of thread t (e even) as one 16-B pair at ht[e * NT + 2 t]
  };
  RobotMeta mt;
  union {
    struct {
      alignas(16) double zc[2][Cfg<NV>::VEC];   // sweep pivot column (double-buffered); in the loop:
                                      // z2 = P a_p2 of a pair step (double-buffered)
      alignas(16) double vz[2][Cfg<NV>::VEC];   // z = P a_p (double-buffered by iteration)
    };
    double wb[4 * Cfg<NV>::VEC];   // between sweep and loop: W's 3x3 foot-step blocks (9 S <= 4 NV)
    // the sweep's pivot columns, tile-column stride TS: two (class 64, single pivots) or two
    // pairs (classes 96 / 128), double-buffered
    alignas(16) double swz[(NV >= 96 ? 4 : 2) * Cfg<NV>::SVEC];
  };
  alignas(16) double vr[2][Cfg<NV>::VEC];   // r = R a_p (slot-indexed)
  union {
    struct {
      alignas(16) double vx[Cfg<NV>::VEC];  // x (before and after the loop)
      alignas(16) double gv[Cfg<NV>::VEC];  // g (before the loop)
    };
    alignas(16) double vr2[2][Cfg<NV>::VEC];   // in the loop: r2 = R a_p2 of a pair step
  };
  alignas(16) double rl[Cfg<NV>::VEC];      // drop path: R_l, H R_l^T, R H R_l^T
  // class 128: z = P a_p again in the sweep's strided layout (double-buffered by iteration), for the
  // add pass's tile-column reads (unpadded, class 128's 16 tile columns fold 4-way on the banks)
  alignas(16) double zp[NV == 128 ? 2 * Cfg<NV>::SVEC : 2];
  alignas(16) double tv[Cfg<NV>::VEC];
  alignas(16) double yv[Cfg<NV>::VEC];
  double wmax[Cfg<NV>::NW];
  int choice;   // classes 64 / 96 (split choice): wave 1's published {pass tag, p2 + 1, p + 1}
};
// the formulation scratch must not grow the H copy's union (class 64: 4 robots per CU)
static_assert(sizeof(FormArea<64>) <= sizeof(double) * 64 * 64, "formulation scratch exceeds the H copy");
static_assert(sizeof(SharedT<64>) <= 160 * 1024 / 4, "class 64 holds four robots per CU");

constexpr int DPP_SHL1 = 0x101;   // row_shl:1 -- lane i reads lane i + 1 (same 16-lane row)
constexpr int DPP_ROR8 = 0x128;   // row_ror:8 -- lane i <-> i ^ 8 inside 16 lanes

__device__ __forceinline__ double dpp_shl1(double v) {
  const long long bits = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_update_dpp(0, (int)bits, DPP_SHL1, 0xF, 0xF, true);
  const int hi = __builtin_amdgcn_update_dpp(0, (int)(bits >> 32), DPP_SHL1, 0xF, 0xF, true);
  return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}
// Sum 4 row partials over the TCN lanes of a tile row.  Lane keeps row
// 4tr + 2 bit2(lane) + bit1(lane) (see trow / twriter).
template <int TCN>
__device__ __forceinline__ double tile_reduce(const double (&acc)[4], int lane) {
  const bool hi4 = (lane & 4) != 0;
  double k2[2];
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const double send = hi4 ? acc[k] : acc[2 + k];
    const double keep = hi4 ? acc[2 + k] : acc[k];
    k2[k] = keep + dpp_d<DPP_HMIRROR>(send);
  }
  const bool hi2 = (lane & 2) != 0;
  const double send = hi2 ? k2[0] : k2[1];
  const double keep = hi2 ? k2[1] : k2[0];
  double y = keep + dpp_d<DPP_XOR2>(send);
  y += dpp_d<DPP_XOR1>(y);
  if constexpr (TCN == 16) y += dpp_d<DPP_ROR8>(y);
  return y;
}
template <int TCN>
__device__ __forceinline__ int trow(int tr, int lane) {
  return 4 * tr + 2 * ((lane >> 2) & 1) + ((lane >> 1) & 1);
}
template <int TCN>
__device__ __forceinline__ bool twriter(int lane) {
  return TCN == 16 ? (lane & 9) == 0 : (lane & 1) == 0;
}

// y = M v, v in LDS; returns row trow<TCN>(tr, lane)'s value
template <int TCN, int TW>
__device__ __forceinline__ double tile_matvec4(const double (&M)[4][TW], const double* v, int tc, int lane) {
  double vs[TW];
  ldt<TW>(vs, v, tc);
  double acc[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    double a = 0.0, b2 = 0.0;
#pragma unroll
    for (int c = 0; c < TW; c += 2) {
      a = fma(M[r][c], vs[c], a);
      b2 = fma(M[r][c + 1], vs[c + 1], b2);
    }
    acc[r] = a + b2;
  }
  return tile_reduce<TCN>(acc, lane);
}

// z / r column combination out[r] = a0 M[r][C0] + a1 M[r][C0 + 1] + a2 M[r][C0 + 2] with uniform
// coefficients (class 96: a foot-step never straddles two tile columns, whose lanes alone store
// the result); the R half only where the wave's slot rows hold an active constraint (rlive)
template <int C0, int TW>
__device__ __forceinline__ void colcombo_u(const double (&Pm)[4][TW], const double (&Rm)[4][TW], double a0, double a1,
                                           double a2, bool rlive, double (&zq)[4], double (&rq)[4]) {
#pragma unroll
  for (int r = 0; r < 4; ++r) zq[r] = fma(a2, Pm[r][C0 + 2], fma(a1, Pm[r][C0 + 1], a0 * Pm[r][C0]));
  if (rlive) {
#pragma unroll
    for (int r = 0; r < 4; ++r) rq[r] = fma(a2, Rm[r][C0 + 2], fma(a1, Rm[r][C0 + 1], a0 * Rm[r][C0]));
  } else {
#pragma unroll
    for (int r = 0; r < 4; ++r) rq[r] = 0.0;
  }
}

template <int NT>
__device__ __forceinline__ void write_empty_t(int b, int tid, int N, int code, float* u0g, float* Ug, int* statusg,
                                              int* itersg) {
  if (tid < 12) u0g[(size_t)b * 12 + tid] = 0.f;
  if (Ug)
    for (int k = tid; k < N * 12; k += NT) Ug[(size_t)b * N * 12 + k] = 0.f;
  if (tid == 0) {
    if (statusg) statusg[b] = code;
    if (itersg) itersg[b] = 0;
  }
}

// One robot.  A robot exceeding NV is appended to `queue` (when given) for the
// next capacity class -- or to `queue_big` / `queue_ipm` for the ones after, when
// it exceeds those too -- otherwise reported MPCQP_STATUS_TOO_LARGE.
template <int NV, bool FULL>
__device__ __forceinline__ void solve_robot(const KParams& P, int b, SharedT<NV>& sm, const float* __restrict__ x0g,
                                            const float* __restrict__ xrefg, const float* __restrict__ contactg,
                                            const float* __restrict__ feetg, const float* __restrict__ robotg,
                                            float* __restrict__ u0g, float* __restrict__ Ug, int* __restrict__ statusg,
                                            int* __restrict__ itersg, int* __restrict__ queue,
                                            int* __restrict__ queue_big = nullptr,
                                            int* __restrict__ queue_ipm = nullptr) {
  using C = Cfg<NV>;
  constexpr int NT = C::NT, TCN = C::TCN, CPL = C::CPL, VPL = C::VPL, RPW = C::RPW, TW = C::TW;
  const int tid = threadIdx.x;
  const int lane = tid & (LANES - 1), wave = uni(tid >> 6);
  const int tr = tid / TCN, tc = tid % TCN;
  const int N = P.N;
#ifdef MPCQP_STAMPS
  unsigned long long stamps_[7];
  unsigned long long secacc_ = 0, seclast_ = 0;
  int seccur_ = 7;
#endif
  STAMP(0);
#ifdef MPCQP_STAMPS
  const unsigned long long rt0_ = __builtin_amdgcn_s_memrealtime();   // 100 MHz, chip-wide
#endif

  // ------------------------------------------------ inputs, stance list
  Form& smf = sm.fa.f;
  FormY& smfy = sm.fa.fy;
  if (!form_stage<NT>(smf, N, b, tid, x0g, xrefg, contactg, feetg, robotg)) {
    write_empty_t<NT>(b, tid, N, MPCQP_STATUS_NONFINITE, u0g, Ug, statusg, itersg);
    return;
  }
  if (wave == 0) form_stance(smf, sm.mt, N, lane);
  fsync<NT>();
  const int S = uni(sm.mt.S);
  const int n = 3 * S, m = 6 * S;
  if (n > NV) {
    // the next capacity class takes it: `queue`, `queue_big` (when given) for a robot
    // beyond class 96 as well, `queue_ipm` (when given) for one beyond class 128
    int* qn = queue;
    if (queue_big && n > 96) qn = queue_big;
    if (queue_ipm && n > 128) qn = queue_ipm;
    if (qn) {
      if (tid == 0) qn[4 + atomicAdd(&qn[0], 1)] = b;
      return;
    }
    write_empty_t<NT>(b, tid, N, MPCQP_STATUS_TOO_LARGE, u0g, Ug, statusg, itersg);
    return;
  }

  // ------------------------------------------------ formulation (mpcqp_form.h)
  form_model<NT>(P, smf, smfy, sm.mt, N, tid);
  if constexpr (!FULL) {
    // the H build's integer block weights, once per step pair instead of once per entry
    for (int e = tid; e < N * N; e += NT) {
      const int ja = e / N, jb = e - ja * N;
      const int mx = ja > jb ? ja : jb;
      const int d = ja > jb ? ja - jb : jb - ja;
      const int m = N - mx;
      const int ta = (m * (4 * m * m - 1)) / 3 + 2 * d * m * m;   // exact integer
      sm.fa.mt_tab[e] = d2{(double)ta, (double)m};
    }
  }
  fsync<NT>();
  if (tid < NV) sm.gv[tid] = tid < n ? form_g(P, smf, sm.mt, tid) : 0.0;
  STAMP(1);

  // row `r` of the lane's H tile (identity padding beyond n); cj / cc: the tile
  // columns' foot-step horizon step and input column
  auto hcols = [&](int (&cj)[TW], int (&cc)[TW]) {
#pragma unroll
    for (int c = 0; c < TW; ++c) {
      const int col = TW * tc + c;
      const int sb = col < n ? col / 3 : 0;
      cj[c] = sm.mt.foot_t[sb];
      cc[c] = 3 * sm.mt.foot_leg[sb] + col % 3;
    }
  };
  // FULL: non-diagonal Q / R (form_h_full, the same-step R block included); the kernels
  // are instantiated once per weight kind, so each keeps a single register assignment
  auto hrow = [&](int r, const int (&cj)[TW], const int (&cc)[TW], double (&h)[TW]) {
    const int row = 4 * tr + r;
    const int sa = row < n ? row / 3 : 0;
    const int ja = sm.mt.foot_t[sa];
    const int car = 3 * sm.mt.foot_leg[sa] + row % 3;
    const double r2 = smfy.rd2[row < n ? car : 0];
#pragma unroll
    for (int c = 0; c < TW; ++c) {
      const int col = TW * tc + c;
      double hv;
      if constexpr (FULL) hv = form_h_full(smfy, N, ja, car, cj[c], cc[c]);
      else hv = form_h_tab(smfy, sm.fa.mt_tab[ja * N + cj[c]], car, cc[c]) + (row == col ? r2 : 0.0);
      h[c] = (row < n && col < n) ? hv : (row == col ? 1.0 : 0.0);
    }
  };
  double W[4][TW];
  {
    int cj[TW], cc[TW];
    hcols(cj, cc);
#pragma unroll
    for (int r = 0; r < 4; ++r) hrow(r, cj, cc, W[r]);   // unrolled: rows land in their registers
  }
  fsync<NT>();   // every lane is done reading the formulation scratch H overwrites
#pragma unroll
  for (int r = 0; r < 4; ++r)
#pragma unroll
    for (int c = 0; c < TW; c += 2)   // column pairs, lane-interleaved: 16-B accesses
      reinterpret_cast<d2*>(sm.ht)[((TW * r + c) >> 1) * NT + tid] = d2{W[r][c], W[r][c + 1]};
  STAMP(2);

  // ------------------------------------------------ W = H^-1 (symmetric sweep)
  // element 4 tr (the lane's tile row) of a pivot column in the strided layout
  const int i4s = C::TS * (tr >> 1) + 4 * (tr & 1);   // TW = 8
  if constexpr (NV >= 96) {
  // Classes 96 / 128 (one robot per CU, latency-bound; 6- / 8-wave barriers):
  // pivot PAIRS {K, K + 1} (K even: one tile column, one 4-row group; K + 1 = n is
  // the decoupled identity padding when n is odd).  With Z = W[:, {K, K+1}] and its
  // pivot block D, the block sweep W_ij -= (Z D^-1)_i . Z_j, W_iK = (Z D^-1)_i,
  // W_KK = -D^-1 is ONE rank-2 pass: coefficient rows -(Z D^-1)_i (pivot rows:
  // (D^-1 - I)_a, turning rows K into D^-1 Z^T), the pair's columns entering with
  // D - I in place of D (turning columns K into Z D^-1), then -2 on the pivot
  // diagonal.  Half the barriers and pivot-column round trips of single pivots;
  // class 64 (four robots per CU, issue-bound when they sweep together) keeps
  // single pivots, which issue fewer instructions.  The pair's two columns are
  // double-buffered by pair parity in the zc / vz space.
#pragma unroll 1
  for (int KT = 0; TW * KT < n; ++KT) {
    static_for<TW / 2>([&](auto KPc) {
      constexpr int KC = 2 * decltype(KPc)::value;
      const int K = TW * KT + KC;
      const int KR = TW == 8 ? 2 * KT + (KC >> 2) : K >> 2;
      const int KRR = TW == 8 ? (KC & 3) : (K & 3);   // 0 or 2
      if (K < n) {
        // class 96 keeps its unpadded vectors (zc / vz) and their addressing as it was
        double* const z0 = (TW == 8 ? sm.swz : sm.zc[0]) + ((K >> 1) & 1) * (2 * C::SVEC);
        double* const z1 = z0 + C::SVEC;
        const int ks = TW == 8 ? C::TS * KT + KC : K;   // element K in the strided layout
        const int i4 = TW == 8 ? i4s : 4 * tr;
        if (tc == KT) {
          d2* q0 = reinterpret_cast<d2*>(z0 + i4);
          q0[0] = d2{W[0][KC], W[1][KC]};
          q0[1] = d2{W[2][KC], W[3][KC]};
          d2* q1 = reinterpret_cast<d2*>(z1 + i4);
          q1[0] = d2{W[0][KC + 1], W[1][KC + 1]};
          q1[1] = d2{W[2][KC + 1], W[3][KC + 1]};
        }
        fsync<NT>();
        double zr0[TW], zr1[TW], zi0[4], zi1[4];
        lds_t<TW, C::TS>(zr0, z0, tc);
        lds_t<TW, C::TS>(zr1, z1, tc);
        if constexpr (TW == 8) {
          ld4s(zi0, z0 + i4s);
          ld4s(zi1, z1 + i4s);
        } else {
          ld4(zi0, z0, tr);
          ld4(zi1, z1, tr);
        }
        const double d00 = z0[ks], d01 = z0[ks + 1], d11 = z1[ks + 1];
        const double idet = rcp_nr(fma(d00, d11, -d01 * d01));
        const double e00 = d11 * idet, e01 = -d01 * idet, e11 = d00 * idet;   // D^-1
        double c0[4], c1[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          c0[r] = -fma(zi0[r], e00, zi1[r] * e01);
          c1[r] = -fma(zi0[r], e01, zi1[r] * e11);
        }
        if constexpr (TW == 8) {
          if (tr == KR) {
            c0[KRR] = e00 - 1.0;
            c1[KRR] = e01;
            c0[KRR + 1] = e01;
            c1[KRR + 1] = e11 - 1.0;
          }
        } else {
#pragma unroll
          for (int r = 0; r < 4; r += 2) {
            const bool at = tr == KR && r == KRR;
            c0[r] = at ? e00 - 1.0 : c0[r];
            c1[r] = at ? e01 : c1[r];
            c0[r + 1] = at ? e01 : c0[r + 1];
            c1[r + 1] = at ? e11 - 1.0 : c1[r + 1];
          }
        }
        if (tc == KT) {   // the pair's columns enter with D - I
          zr0[KC] -= 1.0;
          zr1[KC + 1] -= 1.0;
        }
#pragma unroll
        for (int r = 0; r < 4; ++r)
#pragma unroll
          for (int c = 0; c < TW; ++c) W[r][c] = fma(c1[r], zr1[c], fma(c0[r], zr0[c], W[r][c]));
        if constexpr (TW == 8) {
          if (tc == KT && tr == KR) {
            W[KRR][KC] -= 2.0;
            W[KRR + 1][KC + 1] -= 2.0;
          }
        } else {
#pragma unroll
          for (int r = 0; r < 4; r += 2) {
            const bool at = tc == KT && tr == KR && r == KRR;
            W[r][KC] -= at ? 2.0 : 0.0;
            W[r + 1][KC + 1] -= at ? 2.0 : 0.0;
          }
        }
      }
    });
  }
  } else {
  // pivot K = 8 KT + KC: W_ij -= z_i z_j / d, W_iK = z_i / d, W_KK = -1/d (ends at
  // -H^-1; padding rows/columns >= n never change).  One generic rank-1 pass (the
  // pivot row's coefficient made inv - 1 turns row K into z_j / d, the pivot column's
  // entry of row K made d - 1 turns column K into z_i / d), then the diagonal.  KC compile-time
  // (register column), KT a runtime loop so the code stays in the instruction cache.
#pragma unroll 1
  for (int KT = 0; TW * KT < n; ++KT) {
    static_for<TW>([&](auto KCc) {
      constexpr int KC = decltype(KCc)::value;
      const int K = TW * KT + KC;
      // pivot row K: tile row KR, register row KRR (compile-time when TW = 8)
      const int KR = TW == 8 ? 2 * KT + (KC >> 2) : K >> 2;
      const int KRR = TW == 8 ? (KC & 3) : (K & 3);
      if (K < n) {
        double* const zc = sm.swz + (KC & 1) * C::SVEC;
        if (tc == KT) {
          d2* pz = reinterpret_cast<d2*>(zc + i4s);
          pz[0] = d2{W[0][KC], W[1][KC]};
          pz[1] = d2{W[2][KC], W[3][KC]};
        }
        fsync<NT>();
        double zr[TW], zi[4];
        lds_t<TW, C::TS>(zr, zc, tc);
        ld4s(zi, zc + i4s);
        const double dK = zc[C::TS * KT + KC];
        const double inv = rcp_nr(dK);
        double beta[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) beta[r] = -zi[r] * inv;
        if constexpr (TW == 8) {
          if (tr == KR) beta[KC & 3] = inv - 1.0;
        } else {
#pragma unroll
          for (int r = 0; r < 4; ++r) beta[r] = (tr == KR && r == KRR) ? inv - 1.0 : beta[r];
        }
        // column K rides along in the same pass: with its row-K entry taken as d - 1,
        // W_iK + beta_i (d - 1) = z_i - z_i (d - 1) / d = z_i / d, and the pivot
        // entry becomes d + (1/d - 1)(d - 1) = 2 - 1/d (-> -1/d below)
        if (tc == KT) zr[KC] = dK - 1.0;
#pragma unroll
        for (int r = 0; r < 4; ++r)
#pragma unroll
          for (int c = 0; c < TW; ++c) W[r][c] = fma(beta[r], zr[c], W[r][c]);
        if constexpr (TW == 8) {
          W[KC & 3][KC] += (tc == KT && tr == KR) ? -2.0 : 0.0;
        } else {
#pragma unroll
          for (int r = 0; r < 4; ++r) W[r][KC] += (tc == KT && tr == KR && r == KRR) ? -2.0 : 0.0;
        }
      }
    });
  }
  }
  // P = -(sweep result) = H^-1 ; largest diagonal entry (dependency threshold scale)
  double wd = 0.0;
#pragma unroll
  for (int r = 0; r < 4; ++r)
#pragma unroll
    for (int c = 0; c < TW; ++c) W[r][c] = -W[r][c];
  if constexpr (TW == 8) {
    if (tc == (tr >> 1)) {
      // diagonal entries: column r (even tile row) or 4 + r (odd); blended
      // arithmetically -- a select between the two would index the tile at run time
      const double odd = (double)(tr & 1);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const double dv = fma(odd, W[r][4 + r], (1.0 - odd) * W[r][r]);
        if (4 * tr + r < n) wd = fmax(wd, dv);
      }
    }
  } else {
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
      for (int c = 0; c < TW; ++c)
        if (4 * tr + r == TW * tc + c && 4 * tr + r < n) wd = fmax(wd, W[r][c]);
  }
  wd = wave_max_d(wd);
  if (lane == 0) sm.wmax[wave] = wd;
  // the foot-steps' 3x3 diagonal blocks of W, for the rows' dual-curvature scales below
  fsync<NT>();   // every lane is done reading the last pivot column (wb aliases zc)
#pragma unroll
  for (int r = 0; r < 4; ++r)
#pragma unroll
    for (int c = 0; c < TW; ++c) {
      const int row = 4 * tr + r, col = TW * tc + c;
      if (row < n && col < n && row / 3 == col / 3) sm.wb[9 * (row / 3) + 3 * (row % 3) + col % 3] = W[r][c];
    }
  STAMP(3);

  // unconstrained minimiser x = -W g
  {
    const double y = tile_matvec4<TCN, TW>(W, sm.gv, tc, lane);
    if (twriter<TCN>(lane)) sm.vx[trow<TCN>(tr, lane)] = -y;
  }
  fsync<NT>();
  double wscale = sm.wmax[0];
#pragma unroll
  for (int w = 1; w < C::NW; ++w) wscale = fmax(wscale, sm.wmax[w]);
  wscale = sgpr_d(wscale);
  const float qfloor = fmaxf((float)(1e-9 * wscale), 1e-30f);   // rows dependent on the active set

  // ---- per-lane constraint rows c = lane + 64k (redundant in every wave): the
  // row's foot-step variables start at cz, its cone coefficients at sm.mt.rows[crt]
  // (re-read from LDS: registers hold the two tiles); s = a_c . x - b_c.
  // Row choice: the violated row with the most negative s_c / sqrt(a_c^T P a_c), P the
  // current projected inverse Hessian -- the row whose full step raises the dual
  // objective most (s_c^2 / (2 a_c^T P a_c)); tools/gi_sim.py: the slowest robot of a
  // config-2 batch needs 8-17 % fewer passes than with the initial metric W.  q_c =
  // a_c^T P a_c is kept per row by the rank-1/2 updates of P: an add subtracts
  // (a_c . z)^2 / (a_p . z) (a_c . z = zs_c is computed for every row anyway), a pair
  // [zs, zs2] S^-1 [zs, zs2]^T, a drop adds (a_c . R_l)^2 / eta.  q_c is held in f32
  // (one VGPR per row, as the f32 key it scales): the choice is a heuristic, and any
  // choice reaches the same optimum.  With mu > 0 the n.f >= 0 row is implied by the
  // two opposite t1 rows and never enters (s = +inf): it only adds degenerate steps at
  // the cone apex.
  int cz[CPL], crt[CPL];
  double s[CPL];
  // class 128 keeps the initial metric: the per-pass updates cost more than the passes they
  // save (config 5 -1 %); class 96 uses the current one since its choosing wave updates q_c
  // in the early-choice block (config 4 +1.5 %; before the early choice -3 %)
  constexpr bool kCurKey = NV <= 96;
  float qm[CPL];   // a_c^T P a_c (f32, classes 64 / 96; class 128: 1 / sqrt(a_c^T W a_c)): scales the f32 row key
  auto cdot = [&](const double* v, int k) -> double {
    const double* a = sm.mt.rows[crt[k]];
    const double* vf = v + cz[k];
    return a[0] * vf[0] + a[1] * vf[1] + a[2] * vf[2];
  };
  auto cbound = [&](int k) -> double {   // -b_c: ub on the fz <= ub row (mpc.py:257)
    return crt[k] == 5 ? sm.mt.ub[cz[k] / 3] : 0.0;
  };
#pragma unroll
  for (int k = 0; k < CPL; ++k) {
    const int c = lane + LANES * k;
    const bool ok = c < m;
    cz[k] = ok ? 3 * (c / 6) : 0;
    crt[k] = ok ? c % 6 : 0;
    const bool live = ok && !(crt[k] == 4 && sm.mt.fz0_implied);
    s[k] = live ? cdot(sm.vx, k) + cbound(k) : INFINITY;
    const double* a = sm.mt.rows[crt[k]];
    const double* w = sm.wb + 3 * cz[k];
    double q = 0.0;
#pragma unroll
    for (int i = 0; i < 3; ++i) q = fma(a[i], fma(w[3 * i], a[0], fma(w[3 * i + 1], a[1], w[3 * i + 2] * a[2])), q);
    if constexpr (kCurKey) qm[k] = ok && q > 0.0 ? (float)q : 1.0f;
    else qm[k] = ok && q > 0.0 ? (float)__builtin_amdgcn_rsq(q) : 1.0f;
  }
  double x[VPL], u[VPL];
#pragma unroll
  for (int k = 0; k < VPL; ++k) {
    x[k] = sm.vx[lane + LANES * k];
    u[k] = 0.0;
  }
  if (tid == 0) sm.choice = 0;   // no pass tag yet (split choice)
  // the cone rows' coefficients (lanes 0..17: row r's a_i at 3 r + i) and dependency
  // thresholds 1e-12 |a_r|^2 wscale (lanes 18..23) in one register, read by v_readlane into
  // SGPRs when a row is chosen (an LDS load + readfirstlane chain otherwise)
  constexpr bool kRowTab = NV <= 96;   // class 128: no VGPRs to spare (an 8-byte spill)
  constexpr bool kZp = NV == 128;      // z's strided copy (SharedT::zp)
  double rowtab = 0.0;
  if (!kRowTab) {
  } else if (lane < 18) rowtab = sm.mt.rows[lane / 3][lane % 3];
  else if (lane < 24) {
    const double* a = sm.mt.rows[lane - 18];
    rowtab = 1e-12 * (a[0] * a[0] + a[1] * a[1] + a[2] * a[2]) * wscale;
  }
  fsync<NT>();   // wb, vx and gv are dead: the loop reuses zc / vz / vr2
  unsigned long long occ[VPL];
#pragma unroll
  for (int k = 0; k < VPL; ++k) occ[k] = 0ull;
  double Rm[4][TW];
#pragma unroll
  for (int r = 0; r < 4; ++r)
#pragma unroll
    for (int c = 0; c < TW; ++c) Rm[r][c] = 0.0;
  auto slots_live = [&](int lo) -> bool {   // any occupied slot in [lo, lo + RPW)
    const unsigned long long w = occ[lo >> 6] >> (lo & 63);
    return (RPW >= 64 ? w : (w & ((1ull << RPW) - 1))) != 0ull;
  };

  // ------------------------- Goldfarb-Idnani dual active set, projected form
  // One flat loop (one loop-carried copy of the register tiles): each pass takes
  // one step for the pending violated row p (choosing the most violated row when
  // none is pending); the step either adds p or drops a blocking slot.
  const int max_iter = P.max_iter > 0 ? P.max_iter : 8 * NV + 64;
  const double tol = 1e-9;
  int it = 0;
  int status = MPCQP_STATUS_OK;
  int p = -1;                       // pending violated row (uniform)
  int v0 = 0, tcA = 0, c0 = 0;      // its foot-step's first variable, tile column, register column
  double a0 = 0.0, a1 = 0.0, a2 = 0.0, thr = 0.0, sp = 0.0, up = 0.0;
  // the next rows p (and its pair candidate p2): the most violated row in the dual metric
  // (f32-rounded keys, lowest lane on ties), then the best row of any other foot-step;
  // with the split choice (classes 64 and 96) wave 1 publishes {p, p2} in one pass-tagged
  // LDS word the other waves read (class 96: its six waves sit 2-2-1-1 on the SIMDs, so
  // five fewer argmins free the shared SIMDs' issue: config 4 +1.2 %, bitwise identical)
  // (class 128 would spill: 138 VGPRs with the split choice)
  constexpr bool kSplit = NV <= 96;
  // early choice: the choosing wave (wave 1 of the split choice; the only wave of the one-wave
  // class 64) chooses the next rows before a pass's rank updates, which then overlap it
  // (class 96 with the split choice: config 4 +4.7 %, bitwise identical)
  constexpr bool kEarly = kSplit;
  constexpr int kChooser = 1;
  auto choose = [&](int tag_it, int& pc, int& pc2) {
    pc = -1;
    pc2 = -1;
    if constexpr (kCurKey) {   // the keys in f32 throughout: the argmin is an f32 selection anyway
      float keyf[CPL];
#pragma unroll
      for (int k = 0; k < CPL; ++k)
        keyf[k] = s[k] < -tol ? (float)s[k] * __builtin_amdgcn_rsqf(fmaxf(qm[k], qfloor)) : INFINITY;
      float bv = keyf[0];
      int bk = 0;
#pragma unroll
      for (int k = 1; k < CPL; ++k) {
        bk = keyf[k] < bv ? k : bk;
        bv = fminf(bv, keyf[k]);
      }
      const float fm = wave_min_f32(bv);
      if (fm < INFINITY) {
        const int pl = uni(__builtin_ctzll(__ballot(bv == fm)));
        pc = pl + LANES * uni(__builtin_amdgcn_readlane(bk, pl));
        if constexpr (SharedT<NV>::kPair) {
          const int vc = 3 * (pc / 6);
          float bw = INFINITY;
          int bk2 = 0;
#pragma unroll
          for (int k = 0; k < CPL; ++k) {
            const float kk = cz[k] == vc ? INFINITY : keyf[k];
            bk2 = kk < bw ? k : bk2;
            bw = fminf(bw, kk);
          }
          const float fm2 = wave_min_f32(bw);
          if (fm2 < INFINITY) {
            const int ql = uni(__builtin_ctzll(__ballot(bw == fm2)));
            pc2 = ql + LANES * uni(__builtin_amdgcn_readlane(bk2, ql));
          }
        }
      }
      if constexpr (kSplit) {
        if (lane == 0)
          __hip_atomic_store(&sm.choice, (((tag_it + 1) & 0xffff) << 16) | ((pc2 + 1) << 8) | (pc + 1),
                             __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      }
      return;
    }
    // class 128: f64 keys in the initial metric (qm = 1 / sqrt(a_c^T W a_c))
    double key[CPL];
#pragma unroll
    for (int k = 0; k < CPL; ++k) key[k] = s[k] < -tol ? s[k] * (double)qm[k] : INFINITY;
    double bv = key[0];
    int bk = 0;
#pragma unroll
    for (int k = 1; k < CPL; ++k) {
      bk = key[k] < bv ? k : bk;
      bv = vmin(bv, key[k]);
    }
    double kmn;
    const int pl = wave_argmin_f32(bv, kmn);
    if (kmn < INFINITY) {
      pc = pl + LANES * uni(__builtin_amdgcn_readlane(bk, pl));
      if constexpr (SharedT<NV>::kPair) {
        const int vc = 3 * (pc / 6);
        double bw = INFINITY;
        int bk2 = 0;
#pragma unroll
        for (int k = 0; k < CPL; ++k) {
          const double kk = cz[k] == vc ? INFINITY : key[k];
          bk2 = kk < bw ? k : bk2;
          bw = vmin(bw, kk);
        }
        double kmn2;
        const int ql = wave_argmin_f32(bw, kmn2);
        if (kmn2 < INFINITY) pc2 = ql + LANES * uni(__builtin_amdgcn_readlane(bk2, ql));
      }
    }
    if constexpr (kSplit) {
      if (lane == 0)
        // relaxed workgroup-scope atomics, not volatile: a volatile access keeps the
        // generic address space (a FLAT load / store with a vmcnt wait); these stay DS ops
        __hip_atomic_store(&sm.choice, (((tag_it + 1) & 0xffff) << 16) | ((pc2 + 1) << 8) | (pc + 1),
                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    }
  };
  bool early = false;   // kEarly: wave 1 already holds (and has published) the next choice
  int epc = -1, epc2 = -1;
  SEC(0);
  while (true) {
    // pair candidate p2 (another foot-step's most violated row), set on a fresh choice
    int p2 = -1, tcA2 = 0, c02 = 0;
    double b0 = 0.0, b1 = 0.0, b2 = 0.0, thr2 = 0.0, sp2 = 0.0;
    if (p < 0) {
      // the next row p (and its pair candidate p2): the most violated row in the dual
      // metric (f32-rounded keys, lowest lane on ties), then the best row of any other
      // foot-step.  Classes 64 / 96 (split choice): wave 1 -- whose slot rows of R
      // are idle while <= 32 slots are active -- chooses and publishes {p, p2} in one
      // pass-tagged LDS word, which wave 0 reads after its R update instead of
      // repeating both argmins (every decision is identical in both waves, so both
      // reach every choice point and every exit together).
      int pc = -1, pc2 = -1;
      if (!kSplit || wave == 1) {
        if (kEarly && early) {   // chosen (and published) at the end of the previous pass
          pc = epc;
          pc2 = epc2;
          early = false;
        } else {
          choose(it, pc, pc2);
        }
      } else {
        const int tag = (it + 1) & 0xffff;
        int w;
        do {
          w = uni(__hip_atomic_load(&sm.choice, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP));
        } while ((w >> 16) != tag);
        pc = (w & 0xff) - 1;
        pc2 = ((w >> 8) & 0xff) - 1;
      }
      if (pc < 0) break;
      p = pc;
      const int pl = p & (LANES - 1), kp = p / LANES;
      double sv = s[0];
#pragma unroll
      for (int k = 1; k < CPL; ++k) sv = (k == kp) ? s[k] : sv;
      const double vmn = readlane_d(sv, pl);
      CNT(4);
      const int rp = p % 6;
      if constexpr (kRowTab) {
        a0 = readlane_d(rowtab, 3 * rp);
        a1 = readlane_d(rowtab, 3 * rp + 1);
        a2 = readlane_d(rowtab, 3 * rp + 2);
        thr = readlane_d(rowtab, 18 + rp);
      } else {
        a0 = sgpr_d(sm.mt.rows[rp][0]);
        a1 = sgpr_d(sm.mt.rows[rp][1]);
        a2 = sgpr_d(sm.mt.rows[rp][2]);
        thr = sgpr_d(1e-12 * (a0 * a0 + a1 * a1 + a2 * a2) * wscale);
      }
      v0 = 3 * (p / 6);
      tcA = (int)((unsigned)v0 / TW);   // v0 >= 0: shifts for TW = 8
      c0 = (int)((unsigned)v0 % TW);
      sp = sgpr_d(vmn);   // s_p, tracked like s[] (identical arithmetic)
      up = 0.0;
      SEC(8);
      if (pc2 >= 0) {
        const int ql = pc2 & (LANES - 1), kq = pc2 / LANES;
        double sv2 = s[0];
#pragma unroll
        for (int k = 1; k < CPL; ++k) sv2 = (k == kq) ? s[k] : sv2;
        sp2 = sgpr_d(readlane_d(sv2, ql));
        p2 = pc2;
        const int rq = p2 % 6;
        if constexpr (kRowTab) {
          b0 = readlane_d(rowtab, 3 * rq);
          b1 = readlane_d(rowtab, 3 * rq + 1);
          b2 = readlane_d(rowtab, 3 * rq + 2);
          thr2 = readlane_d(rowtab, 18 + rq);
        } else {
          b0 = sgpr_d(sm.mt.rows[rq][0]);
          b1 = sgpr_d(sm.mt.rows[rq][1]);
          b2 = sgpr_d(sm.mt.rows[rq][2]);
          thr2 = sgpr_d(1e-12 * (b0 * b0 + b1 * b1 + b2 * b2) * wscale);
        }
        const int w0 = 3 * (p2 / 6);
        tcA2 = (int)((unsigned)w0 / TW);   // w0 >= 0: shifts for TW = 8
        c02 = (int)((unsigned)w0 % TW);
      }
    }
    if (++it > max_iter) {
      status = MPCQP_STATUS_MAX_ITER;
      break;
    }
    SEC(1);
    // z = P a_p, r = R a_p: rows 4tr..4tr+3 in the lanes of tile column tcA
    // (R rows of slots no wave member holds active are zero: skipped)
    const bool rlive = slots_live(RPW * wave);
    // rows 4tr..4tr+3 of P a and R a for a row a of the foot-step at variable
    // 8 tA + cA, stored by the lanes of tile column tA
    auto combo_store = [&](int cA, int tA, double e0, double e1, double e2, double* dz, double* dr) {
      double zq[4], rq[4];
      if constexpr (TW == 6) {   // foot-steps start at register column 0 or 3: never straddle,
        // so the uniform (SGPR) coefficients need no per-lane mask: only tile column tA stores
        if (cA == 0) colcombo_u<0, TW>(W, Rm, e0, e1, e2, rlive, zq, rq);
        else colcombo_u<3, TW>(W, Rm, e0, e1, e2, rlive, zq, rq);
      } else {   // TW = 8: classes 64 and 128
        // one computed jump into straight-line cases (mpcqp_combo_asm.h); R's half
        // unconditionally (rows of no active slot are zero; a second, P-only table for those
        // waves measured 0.6 % slower).  A foot-step inside one tile column (c0 <= 5) takes
        // the SGPR coefficients unmasked -- only that tile column's lanes store; a straddling
        // one masks them by the tile column each of its three columns lies in and adds the
        // next lane's partial.
        if (__builtin_expect(cA + 2 >= TW, 0)) {
          const int t1 = tA + (cA == 7 ? 1 : 0), t2 = tA + (cA >= 6 ? 1 : 0);
          combo_asm64(W, Rm, cA, tc == tA ? e0 : 0.0, tc == t1 ? e1 : 0.0, tc == t2 ? e2 : 0.0, zq, rq);
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            zq[r] += dpp_shl1(zq[r]);
            rq[r] += dpp_shl1(rq[r]);
          }
        } else {
          combo_asm64_s(W, Rm, cA, e0, e1, e2, zq, rq);
        }
      }
      if (tc == tA) {
        st4(dz, tr, zq);
        st4(dr, tr, rq);
        // class 128: z also in the sweep's strided layout (tile-column stride TS), for the add
        // pass's conflict-free tile-column reads (cdot and the per-lane reads keep the plain one)
        if constexpr (kZp) st4s(sm.zp + (it & 1) * C::SVEC + i4s, zq);
      }
    };
    const int buf = it & 1;
    double* const vz = sm.vz[buf];
    double* const vr = sm.vr[buf];
    double* const vz2 = sm.zc[buf];
    double* const vzp = sm.zp + buf * C::SVEC;   // kZp: z in the strided layout
    double* const vr2 = sm.vr2[buf];
    combo_store(c0, tcA, a0, a1, a2, vz, vr);
    if (p2 >= 0) combo_store(c02, tcA2, b0, b1, b2, vz2, vr2);
    SEC(9);
    fsync<NT>();
    SEC(2);
    // constraint-row steps zs = A z, slot directions r, variable steps
    double zs[CPL];
#pragma unroll
    for (int k = 0; k < CPL; ++k) zs[k] = cdot(vz, k);
    double zsp = zs[0];
#pragma unroll
    for (int k = 1; k < CPL; ++k) zsp = (k == (p >> 6)) ? zs[k] : zsp;
    zsp = readlane_d(zsp, p & 63);   // lane p computed a_p . z exactly as zs
    SEC(10);

    // ---- pair step: add p and p2 together when the equality-constrained solution
    // on A + {p, p2} keeps every multiplier positive.  With Z = [z, z2] and the 2x2
    // S = [a_p a_p2]^T Z, t = -S^-1 (s_p, s_p2): x += Z t, u_A -= [r r2] t,
    // u_{p,p2} = t, P -= Z S^-1 Z^T, R -= ([r r2] - E) S^-1 Z^T.  (x, A + {p, p2}) is
    // then a valid dual active-set iterate (KKT of the sub-problem, u >= 0), so the
    // method's convergence argument is unchanged; otherwise p takes the usual step.
    if (p2 >= 0) {
      CNT(3);
      // the slot directions r, r2 first: their loads overlap the 2 x 2 solve below, which no
      // longer branches (tp, tq, id are used only when ok, as before)
      double rs1[VPL], rs2[VPL];
#pragma unroll
      for (int k = 0; k < VPL; ++k) {
        rs1[k] = vr[lane + LANES * k];
        rs2[k] = vr2[lane + LANES * k];
      }
      double zs2[CPL];
#pragma unroll
      for (int k = 0; k < CPL; ++k) zs2[k] = cdot(vz2, k);
      double v12 = zs2[0], v22 = zs2[0];
#pragma unroll
      for (int k = 1; k < CPL; ++k) {
        v12 = (k == (p >> 6)) ? zs2[k] : v12;
        v22 = (k == (p2 >> 6)) ? zs2[k] : v22;
      }
      const double s12 = sgpr_d(readlane_d(v12, p & 63));    // a_p . z2
      const double s22 = sgpr_d(readlane_d(v22, p2 & 63));   // a_p2 . z2
      const double det = zsp * s22 - s12 * s12;
      const double id = rcp_nr(det);
      const double tp = sgpr_d((s12 * sp2 - s22 * sp) * id);
      const double tq = sgpr_d((s12 * sp - zsp * sp2) * id);
      const bool ok = zsp > thr && s22 > thr2 && det > thr2 * zsp && tp > 0.0 && tq > 0.0;
      int bad = 0;
#pragma unroll
      for (int k = 0; k < VPL; ++k) {
        const bool mine = (occ[k] >> lane) & 1ull;
        bad |= mine && fma(-tq, rs2[k], fma(-tp, rs1[k], u[k])) < 0.0;
      }
      if (ok && !__any(bad)) {
        SEC(16);
#pragma unroll
        for (int k = 0; k < VPL; ++k) {
          const double zx1 = vz[lane + LANES * k], zx2 = vz2[lane + LANES * k];
          x[k] = fma(tq, zx2, fma(tp, zx1, x[k]));
          const bool mine = (occ[k] >> lane) & 1ull;
          u[k] = mine ? fma(-tq, rs2[k], fma(-tp, rs1[k], u[k])) : u[k];
        }
#pragma unroll
        for (int k = 0; k < CPL; ++k) {
          const int c = lane + LANES * k;
          s[k] = (c == p || c == p2) ? 0.0 : fma(tq, zs2[k], fma(tp, zs[k], s[k]));
        }
        // slots qa < qb: the first two free ones
        int qa = 0, qb = 0;
        {
          unsigned long long f0 = ~occ[0];
          if constexpr (VPL == 1) {
            qa = __builtin_ctzll(f0);
            qb = __builtin_ctzll(f0 & (f0 - 1));
          } else {
            const unsigned long long f1 = ~occ[1];
            qa = f0 ? __builtin_ctzll(f0) : LANES + __builtin_ctzll(f1);
            const unsigned long long g0 = f0 & (f0 - 1);
            qb = g0 ? __builtin_ctzll(g0) : LANES + __builtin_ctzll(f0 ? f1 : (f1 & (f1 - 1)));
          }
        }
#pragma unroll
        for (int k = 0; k < VPL; ++k) {
          const int sl = lane + LANES * k;
          u[k] = sl == qa ? tp : (sl == qb ? tq : u[k]);
        }
        occ[qa >> 6] |= 1ull << (qa & 63);
        occ[qb >> 6] |= 1ull << (qb & 63);
        // class 64: R's row coefficients -(al, be) once per slot lane (both waves write the
        // same values), read back by tile row below -- instead of per tile row, with two
        // LDS loads and two selects each (tv / yv are written only on drop passes, after
        // the next pass's barrier)
        constexpr bool kSlotCoef = NV == 64;
        const double i11 = s22 * id, i12 = -s12 * id, i22 = zsp * id;
        if constexpr (kSlotCoef) {
          const double e1 = rs1[0] - (lane == qa ? 1.0 : 0.0);
          const double e2 = rs2[0] - (lane == qb ? 1.0 : 0.0);
          sm.tv[lane] = -fma(i11, e1, i12 * e2);
          sm.yv[lane] = -fma(i12, e1, i22 * e2);
        }
        // rank-2 updates: row coefficients (al, be) = S^-1 (row's pair), then
        // M[r][c] -= al cz1[c] + be cz2[c]
        // q_c, the row metric, is read only by the choosing wave (wave 1 with the split choice)
        auto qm_pair = [&]() {
          if constexpr (kCurKey)
#pragma unroll
            for (int k = 0; k < CPL; ++k)
              qm[k] = (float)((double)qm[k] - fma(i11 * zs[k], zs[k], fma(2.0 * i12 * zs[k], zs2[k], i22 * zs2[k] * zs2[k])));
        };
        ++it;   // a pair step counts as the two additions it makes
        if constexpr (kEarly) {
          if (wave == kChooser) {   // the row values are final for this pass: choose now, before the FMAs
            qm_pair();
            choose(it, epc, epc2);
            early = true;
          }
        } else {
          qm_pair();
        }
        SEC(17);
        double cz1[TW], cz2[TW], z41[4], z42[4];
        ldt<TW>(cz1, vz, tc);
        ldt<TW>(cz2, vz2, tc);
        ld4(z41, vz, tr);
        ld4(z42, vz2, tr);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const double al = fma(i11, z41[r], i12 * z42[r]);
          const double be = fma(i12, z41[r], i22 * z42[r]);
#pragma unroll
          for (int c = 0; c < TW; ++c) W[r][c] = fma(-be, cz2[c], fma(-al, cz1[c], W[r][c]));
        }
        SEC(18);
        if (rlive || slots_live(RPW * wave)) {
          // r / r2 entries read per row (not as two 4-vectors): the shorter live
          // ranges keep the kernel spill-free (a 4-byte VGPR spill here otherwise,
          // written back as ~266 KiB of scratch per config-2 launch)
          if constexpr (kSlotCoef) {
            fsync<LANES>();   // this wave's tv / yv stores are done
            double nal[4], nbe[4];
            ld4(nal, sm.tv, tr);
            ld4(nbe, sm.yv, tr);
#pragma unroll
            for (int r = 0; r < 4; ++r)
#pragma unroll
              for (int c = 0; c < TW; ++c) Rm[r][c] = fma(nbe[r], cz2[c], fma(nal[r], cz1[c], Rm[r][c]));
          } else {
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int sl = 4 * tr + r;
            const double e1 = vr[sl] - (sl == qa ? 1.0 : 0.0);
            const double e2 = vr2[sl] - (sl == qb ? 1.0 : 0.0);
            const double al = fma(i11, e1, i12 * e2);
            const double be = fma(i12, e1, i22 * e2);
#pragma unroll
            for (int c = 0; c < TW; ++c) Rm[r][c] = fma(-be, cz2[c], fma(-al, cz1[c], Rm[r][c]));
          }
          }
        }
        p = -1;
        CNT(15);
        SEC(0);
        continue;
      }
    }
    SEC(11);
    // 1 / (a_p . z) and the primal step t2 = -s_p / (a_p . z), issued ahead of the ratio test,
    // which does not feed them: their division chain overlaps its loads and divisions, and the
    // add reuses the reciprocal (the operations of rcp_nr(zsp) and div_nr(-sp, zsp))
    const double is = rcp_nr(zsp);
    double t2 = INFINITY;
    if (zsp > thr) {
      const double q = -sp * is;
      t2 = fma(fma(-zsp, q, -sp), is, q);
    }
    double rs[VPL], zx[VPL];
    double rbest = INFINITY;
    int lk = 0;
#pragma unroll
    for (int k = 0; k < VPL; ++k) {
      rs[k] = vr[lane + LANES * k];
      zx[k] = vz[lane + LANES * k];
      const bool mine = (occ[k] >> lane) & 1ull;
      const double ratio = (mine && rs[k] > 0.0) ? div_nr(u[k], rs[k]) : INFINITY;
      lk = ratio < rbest ? k : lk;
      rbest = vmin(rbest, ratio);
    }
    // dual step bound t1 (blocking slot l), primal step t2
    double t1;
    const int ll = wave_argmin_d(rbest, t1);
    const int l = ll + LANES * uni(__builtin_amdgcn_readlane(lk, ll));
    SEC(12);
    const bool add = t2 <= t1;
    const double tstep = add ? t2 : t1;
    if (!(tstep < INFINITY)) {
      status = MPCQP_STATUS_INFEASIBLE;
      break;
    }
#pragma unroll
    for (int k = 0; k < VPL; ++k) {
      x[k] = fma(tstep, zx[k], x[k]);
      const bool mine = (occ[k] >> lane) & 1ull;
      u[k] = mine ? fma(-tstep, rs[k], u[k]) : u[k];
    }
#pragma unroll
    for (int k = 0; k < CPL; ++k) s[k] = fma(tstep, zs[k], s[k]);
    sp = sgpr_d(fma(tstep, zsp, sp));
    up = sgpr_d(up + tstep);
    SEC(add ? 5 : 6);
    // rank-1 updates  W += aW cv^T,  R += aR cv^T  (rows by the lane's tile row)
    double aW[4], aR[4], cv[TW];
    int zrow = -1;   // R row to clear (drop)
    double iedrop = 0.0;   // 1 / eta of a drop
    if (add) {
      // slot q (first free); P -= z z^T / sigma ; R -= (r - e_q) z^T / sigma
      int q = 0;
#pragma unroll
      for (int k = VPL - 1; k >= 0; --k)
        if (~occ[k]) q = LANES * k + __builtin_ctzll(~occ[k]);
      double zr4[4], rr4[4];
      constexpr bool kSlotCoef1 = NV == 64;
      if constexpr (kSlotCoef1) {   // R's row coefficient once per slot lane (as the pair step's)
        sm.tv[lane] = ((lane == q) ? 1.0 - rs[0] : -rs[0]) * is;
        fsync<LANES>();
      }
      if constexpr (kZp) {
        ld4s(zr4, vzp + i4s);
        lds_t<TW, C::TS>(cv, vzp, tc);
      } else {
        ld4(zr4, vz, tr);
        ldt<TW>(cv, vz, tc);
      }
      ld4(rr4, kSlotCoef1 ? sm.tv : vr, tr);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        aW[r] = -zr4[r] * is;
        if constexpr (kSlotCoef1) aR[r] = rr4[r];
        else aR[r] = ((4 * tr + r == q) ? 1.0 - rr4[r] : -rr4[r]) * is;
      }
#pragma unroll
      for (int k = 0; k < VPL; ++k) u[k] = (lane + LANES * k == q) ? up : u[k];
      occ[q >> 6] |= 1ull << (q & 63);
#pragma unroll
      for (int k = 0; k < CPL; ++k) s[k] = (lane + LANES * k == p) ? 0.0 : s[k];
      p = -1;
      if constexpr (kEarly) {
        if (wave == kChooser) {   // the row values are final for this pass: choose before the FMAs
          if constexpr (kCurKey)   // q_c is read only by the choosing wave
#pragma unroll
            for (int k = 0; k < CPL; ++k) qm[k] = (float)fma(-zs[k] * zs[k], is, (double)qm[k]);
          choose(it, epc, epc2);
          early = true;
        }
      }
    } else {
      // drop slot l: eta = Minv_ll, y = Minv[:, l] = R (H R_l^T)
      const int lt = l >> 2, lr = l & 3;
      if (tr == lt) {   // lr is wave-uniform: one scalar dispatch, then whole-row stores
        switch (lr) {
          case 0: stt<TW>(sm.rl, tc, Rm[0]); break;
          case 1: stt<TW>(sm.rl, tc, Rm[1]); break;
          case 2: stt<TW>(sm.rl, tc, Rm[2]); break;
          default: stt<TW>(sm.rl, tc, Rm[3]); break;
        }
      }
      fsync<NT>();
      ldt<TW>(cv, sm.rl, tc);
      {
        double acc[4] = {0.0, 0.0, 0.0, 0.0};
        // the lane's H tile, from LDS
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          double a = 0.0, a2 = 0.0;
#pragma unroll
          for (int c = 0; c < TW; c += 2) {
            const d2 hp = reinterpret_cast<const d2*>(sm.ht)[((TW * r + c) >> 1) * NT + tid];
            a = fma(hp[0], cv[c], a);
            a2 = fma(hp[1], cv[c + 1], a2);
          }
          acc[r] = a + a2;
        }
        const double tvv = tile_reduce<TCN>(acc, lane);
        if (twriter<TCN>(lane)) sm.tv[trow<TCN>(tr, lane)] = tvv;
      }
      fsync<NT>();
      {
        const double yvv = tile_matvec4<TCN, TW>(Rm, sm.tv, tc, lane);
        if (twriter<TCN>(lane)) sm.yv[trow<TCN>(tr, lane)] = yvv;
      }
      fsync<NT>();
      const double ie = rcp_nr(sm.yv[l]);
      iedrop = ie;
      double rl4[4], yv4[4];
      ld4(rl4, sm.rl, tr);
      ld4(yv4, sm.yv, tr);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        aW[r] = rl4[r] * ie;     // P += R_l^T R_l / eta
        // R -= y R_l / eta; row l itself takes exactly -1 (y_l = eta): fma(-1, R_l, R_l) clears
        // it exactly, with no separate zeroing pass
        aR[r] = 4 * tr + r == l ? -1.0 : -yv4[r] * ie;
      }
      zrow = l;
      CNT(14);
#pragma unroll
      for (int k = 0; k < VPL; ++k) u[k] = (lane + LANES * k == l) ? 0.0 : u[k];
      occ[l >> 6] &= ~(1ull << (l & 63));
    }
    SEC(13);
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
      for (int c = 0; c < TW; ++c) W[r][c] = fma(aW[r], cv[c], W[r][c]);
    if (rlive || slots_live(RPW * wave)) {   // this wave's slot rows, before or after the step
#pragma unroll
      for (int r = 0; r < 4; ++r)
#pragma unroll
        for (int c = 0; c < TW; ++c) Rm[r][c] = fma(aR[r], cv[c], Rm[r][c]);
    }
    if (zrow >= 0) {
      if (kCurKey && (!kSplit || wave == 1)) {   // q_c is read only by the choosing wave
#pragma unroll
        for (int k = 0; k < CPL; ++k) {   // q_c += (a_c . R_l)^2 / eta (sm.rl holds R_l until the next drop)
          const double ar = cdot(sm.rl, k);
          qm[k] = (float)fma(ar * ar, iedrop, (double)qm[k]);
        }
      }
      fsync<NT>();   // the drop buffers are rewritten by the next drop
    }
    SEC(0);
  }
  SEC(7);
  STAMP(4);

  // ------------------------------- final x, KKT verification, output
  fsync<NT>();   // vx aliases the loop's vr2: every wave is done reading it
  if (wave == 0) {
#pragma unroll
    for (int k = 0; k < VPL; ++k) sm.vx[lane + LANES * k] = x[k];
  }
  fsync<NT>();
  {
    int bad = 0;
#pragma unroll
    for (int k = 0; k < CPL; ++k) {
      if (lane + LANES * k < m) {
        const double v = cdot(sm.vx, k) + cbound(k);
        bad |= (v < -1e-6) || !isfinite(v);
      }
    }
#pragma unroll
    for (int k = 0; k < VPL; ++k)
      if ((occ[k] >> lane) & 1ull) bad |= (u[k] < -1e-9);
    if (__any(bad) && status == MPCQP_STATUS_OK) status = MPCQP_STATUS_MAX_ITER;
  }
  STAMP(5);
  STAMP(6);

#ifdef MPCQP_STAMPS
  // stamps build: U is a diagnostic buffer of kStampU64 u64 per robot (tools/phase_stamps.py):
  // [0, 7) phase stamps, 7 / 8 chip-wide start / end (s_memrealtime), [16, 24) each wave's HW_ID,
  // [32 + 24 w, 56 + 24 w) wave w's section accumulators and event counters (lane k: section k)
  if (Ug) {
    unsigned long long* dst = (unsigned long long*)Ug + (size_t)b * kStampU64;
    if (tid == 0) {
      for (int i = 0; i < 7; ++i) dst[i] = stamps_[i];
      dst[7] = rt0_;
      dst[8] = __builtin_amdgcn_s_memrealtime();
    }
    if (lane < 24) dst[32 + 24 * wave + lane] = secacc_;
    if (lane == 0)   // SIMD, CU, SE; XCC_ID; workgroup id
      dst[16 + wave] = (unsigned)__builtin_amdgcn_s_getreg((31 << 11) | 4) |
                       ((unsigned long long)(__builtin_amdgcn_s_getreg((3 << 11) | 20) & 15) << 32) |
                       ((unsigned long long)blockIdx.x << 40);
  }
  Ug = nullptr;
#endif
  if (wave == 0) {
    if (lane < 12) {
      const int sidx = sm.mt.stance_of[lane / 3];
      u0g[(size_t)b * 12 + lane] = sidx >= 0 ? (float)sm.vx[3 * sidx + lane % 3] : 0.f;
    }
    if (Ug) {
      for (int k = lane; k < N * 12; k += LANES) {
        const int sidx = sm.mt.stance_of[k / 3];
        Ug[(size_t)b * N * 12 + k] = sidx >= 0 ? (float)sm.vx[3 * sidx + k % 3] : 0.f;
      }
    }
    if (lane == 0) {
      if (statusg) statusg[b] = status;
      if (itersg) itersg[b] = it;
    }
  }
}

