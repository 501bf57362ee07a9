// mpcqp_bm.h -- class 64 (n = 3 * #stance <= 63) as a brain / muscle pair of waves
// (included by mpcqp.hip inside its anonymous namespace, after mpcqp_solve.h).
//
// The same Goldfarb-Idnani dual active set in projected form as mpcqp_solve.h
// (P = reduced inverse Hessian, R = multiplier map, pair steps, rows keyed in the
// current metric a^T P a), with the work of a pass split by role instead of
// repeated in both waves:
//
//   muscle (wave 0): P as 8 x 8 register tiles (lane (tr, tc) holds rows 8 tr..8 tr+7,
//                    columns 8 tc..8 tc+7) and x; forms the step directions
//                    z = P a_p (z2 = P a_p2) and applies the rank updates of P;
//   brain  (wave 1): R with one slot per lane (R row in registers), the multipliers,
//                    the constraint values s, the row metric, and every decision
//                    (row choice, pair test, ratio test, add / drop).
//
// A pass is two workgroup barriers: A (the brain's command is published) and B (the
// step directions are in LDS).  Each side applies the previous step's rank update ONE
// PASS LATE -- the muscle after barrier B, while the brain decides; the brain between
// A and B, while the muscle forms z -- and the directions of a pass are formed from the
// lagging matrices plus a correction for that pending update, whose coefficients the
// brain knows from the previous pass (tools/bm_sim.py: the lagged loop reproduces the
// eager one to 1e-14):
//   add (sigma, z, r, slot q):  P a = P_old a - z (a.z)/sigma,
//                               R a = R_old a - (r - e_q)(a.z)/sigma
//   pair (S^-1, z, z2, r, r2):  [c1 c2] = S^-1 [a.z, a.z2]:  P a = P_old a - c1 z - c2 z2,
//                               R a = R_old a - c1 (r - e_qa) - c2 (r2 - e_qb)
//   drop (eta, R_l, y):         c = (R_l . a)/eta:  P a = P_old a + c R_l,  R a = R_old a - c y
// So the rank-1 / rank-2 FMAs of both matrices run beside the other wave's critical
// chain instead of on it.  A drop adds one helper round: the muscle forms t = H R_l^T
// (H's copy in LDS), the brain y = R t (= column l of (A W A^T)^-1).

constexpr int BM_SOLVE = 0, BM_HRL = 1, BM_EXIT = 2;
constexpr int BM_NONE = 0, BM_ADD = 1, BM_PAIR = 2, BM_DROP = 3;

struct BmCmd {
  int op;                // BM_SOLVE / BM_HRL / BM_EXIT
  int v0, v02;           // first variable of p's / p2's foot-step (v02 = -1: no pair candidate)
  int pend;              // pending update the muscle applies after barrier B (BM_NONE / ADD / PAIR / DROP)
  int zbuf;              // vz / vz2 parity of the pending update's z, z2
  int dbuf;              // rl parity of the pending (or HRL) drop
  int buf;               // vz / vz2 parity of this pass's z, z2
  int pad;
  double a[3], b[3];     // cone rows of p, p2
  double cp[2], cq[2];   // the pending update's correction coefficients for p's / p2's direction
  double k[3];           // pending P update: 1/sigma | S^-1 (i11, i12, i22) | 1/eta
  double tx[2];          // pending x step: t | (tp, tq)
};

struct alignas(16) SharedBM {
  union {
    FormArea<64> fa;      // formulation scratch (dead once H is built)
    d2 ht[32][64];        // H copy in the muscle's tile layout: pair k = (8 r + c) / 2 of lane L at ht[k][L]
  };
  RobotMeta mt;
  union {
    alignas(16) double zc[2][64];   // the sweep's pivot column (double-buffered)
    struct {
      alignas(16) double tv[64];    // loop: t = H R_l^T (drop helper round)
      alignas(16) double vx[64];    // x before and after the loop
    };
  };
  union {
    struct {
      alignas(16) double vz[2][64];    // z = P a_p  (pass parity)
      alignas(16) double vz2[2][64];   // z2 = P a_p2 (pass parity)
      alignas(16) double rl[2][64];    // R_l of a drop (drop parity)
    };
    struct {
      alignas(16) double gv[64];       // before the loop: g
      alignas(16) double gpad[64];
      alignas(16) double wb[192];      // before the loop: W's 3x3 foot-step blocks (9 S <= 189)
    };
  };
  double wmax;
  BmCmd cmd;
};
static_assert(sizeof(SharedBM) <= 40960, "four class-64 robots share a CU's 160 KB of LDS");

// rows 8 tr..8 tr+7 of M a for the foot-step row a at variable 8 tcA + C0 (lanes of tile
// column tcA; a foot-step that straddles into tile column tcA + 1 is summed over DPP)
template <int C0>
__device__ __forceinline__ void bm_combo_c(const double (&M)[8][8], int tc, int tcA, double a0, double a1, double a2,
                                           double (&zq)[8]) {
  const double al0 = (tc == tcA + (C0 + 0) / 8) ? a0 : 0.0;
  const double al1 = (tc == tcA + (C0 + 1) / 8) ? a1 : 0.0;
  const double al2 = (tc == tcA + (C0 + 2) / 8) ? a2 : 0.0;
  constexpr int c0 = C0 % 8, c1 = (C0 + 1) % 8, c2 = (C0 + 2) % 8;
#pragma unroll
  for (int r = 0; r < 8; ++r) zq[r] = fma(al2, M[r][c2], fma(al1, M[r][c1], al0 * M[r][c0]));
  if constexpr (C0 + 2 >= 8) {
#pragma unroll
    for (int r = 0; r < 8; ++r) zq[r] += dpp_shl1(zq[r]);
  }
}
__device__ __forceinline__ void bm_combo(const double (&M)[8][8], int tc, int v0, double a0, double a1, double a2,
                                         double (&zq)[8]) {
  const int tcA = v0 >> 3;
  switch (v0 & 7) {
    case 0: bm_combo_c<0>(M, tc, tcA, a0, a1, a2, zq); break;
    case 1: bm_combo_c<1>(M, tc, tcA, a0, a1, a2, zq); break;
    case 2: bm_combo_c<2>(M, tc, tcA, a0, a1, a2, zq); break;
    case 3: bm_combo_c<3>(M, tc, tcA, a0, a1, a2, zq); break;
    case 4: bm_combo_c<4>(M, tc, tcA, a0, a1, a2, zq); break;
    case 5: bm_combo_c<5>(M, tc, tcA, a0, a1, a2, zq); break;
    case 6: bm_combo_c<6>(M, tc, tcA, a0, a1, a2, zq); break;
    default: bm_combo_c<7>(M, tc, tcA, a0, a1, a2, zq); break;
  }
}

// Sum 8 row partials over the 8 lanes of a tile row; lane tc keeps row tc.
__device__ __forceinline__ double bm_reduce8(const double (&acc)[8], int lane) {
  const bool h4 = (lane & 4) != 0;
  double k4[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const double send = h4 ? acc[i] : acc[4 + i];
    const double keep = h4 ? acc[4 + i] : acc[i];
    k4[i] = keep + dpp_d<DPP_HMIRROR>(send);
  }
  const bool h2 = (lane & 2) != 0;
  double k2[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const double send = h2 ? k4[i] : k4[2 + i];
    const double keep = h2 ? k4[2 + i] : k4[i];
    k2[i] = keep + dpp_d<DPP_XOR2>(send);
  }
  const bool h1 = (lane & 1) != 0;
  const double send = h1 ? k2[0] : k2[1];
  const double keep = h1 ? k2[1] : k2[0];
  return keep + dpp_d<DPP_XOR1>(send);
}

// a . R[3 f .. 3 f + 2] for the lane's R row, f wave-uniform (a binary search over
// compile-time foot-steps: the row stays in registers)
template <int LO, int HI>
__device__ __forceinline__ double bm_rsel(const double (&Rr)[64], int f, double a0, double a1, double a2) {
  if constexpr (LO == HI) {
    double v = fma(a2, Rr[3 * LO + 2], fma(a1, Rr[3 * LO + 1], a0 * Rr[3 * LO]));
    // a leaf-specific no-op keeps the leaves distinct: merged, their loads would become
    // one runtime-indexed load and push the whole row out of registers into scratch
    asm volatile("; bm_rsel leaf %1" : "+v"(v) : "i"(LO));
    return v;
  } else {
    constexpr int MID = (LO + HI) / 2;
    if (f <= MID) return bm_rsel<LO, MID>(Rr, f, a0, a1, a2);
    return bm_rsel<MID + 1, HI>(Rr, f, a0, a1, a2);
  }
}

__device__ __forceinline__ void solve_robot_bm(const KParams& P, int b, SharedBM& sm, const float* __restrict__ x0g,
                                               const float* __restrict__ xrefg, const float* __restrict__ contactg,
                                               const float* __restrict__ feetg, const float* __restrict__ robotg,
                                               float* __restrict__ u0g, float* __restrict__ Ug,
                                               int* __restrict__ statusg, int* __restrict__ itersg,
                                               int* __restrict__ queue, int* __restrict__ queue_big,
                                               int* __restrict__ queue_ipm) {
  constexpr int NT = 128, CPL = 2;
  const int tid = threadIdx.x;
  const int lane = tid & (LANES - 1), wave = uni(tid >> 6);
  const int tr = lane >> 3, tc = lane & 7;   // the muscle's tile of P
  const int N = P.N;
#ifdef MPCQP_STAMPS
  unsigned long long stamps_[7] = {0, 0, 0, 0, 0, 0, 0};
  unsigned long long secacc_ = 0, seclast_ = __builtin_amdgcn_s_memtime();
  int seccur_ = 15;
#endif
  STAMP(0);

  // ------------------------------------------------ inputs, stance list, routing
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
  if (n > 64) {
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
  fsync<NT>();
  if (tid < 64) sm.gv[tid] = tid < n ? form_g(P, smf, sm.mt, tid) : 0.0;
  STAMP(1);
  // H in the muscle's tile layout: thread t builds rows 4 h..4 h+3 (h = t / 64) of lane
  // (t % 64)'s 8 x 8 tile (identity padding beyond n), held in registers until every
  // thread is done reading the formulation scratch H's copy overwrites
  {
    const int L = tid & 63, h = tid >> 6;
    const int ltr = L >> 3, ltc = L & 7;
    int cj[8], cc[8];
#pragma unroll
    for (int c = 0; c < 8; ++c) {
      const int col = 8 * ltc + c;
      const int sb = col < n ? col / 3 : 0;
      cj[c] = sm.mt.foot_t[sb];
      cc[c] = 3 * sm.mt.foot_leg[sb] + col % 3;
    }
    double hv[4][8];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int row = 8 * ltr + 4 * h + r;
      const int sa = row < n ? row / 3 : 0;
      const int ja = sm.mt.foot_t[sa];
      const int car = 3 * sm.mt.foot_leg[sa] + row % 3;
      const double r2 = smfy.rd2[row < n ? car : 0];
#pragma unroll
      for (int c = 0; c < 8; ++c) {
        const int col = 8 * ltc + c;
        const double v = form_h(smfy, N, ja, car, cj[c], cc[c]) + (row == col ? r2 : 0.0);
        hv[r][c] = (row < n && col < n) ? v : (row == col ? 1.0 : 0.0);
      }
    }
    fsync<NT>();
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
      for (int c = 0; c < 8; c += 2) sm.ht[(8 * (4 * h + r) + c) >> 1][L] = d2{hv[r][c], hv[r][c + 1]};
  }
  fsync<NT>();
  STAMP(2);

  if (wave == 0) {
    // ============================================================ muscle: H^-1
    double Pm[8][8];
#pragma unroll
    for (int r = 0; r < 8; ++r)
#pragma unroll
      for (int c = 0; c < 8; c += 2) {
        const d2 v = sm.ht[(8 * r + c) >> 1][lane];
        Pm[r][c] = -v[0];   // the sweep of -H ends at -(-H)^-1 = H^-1
        Pm[r][c + 1] = -v[1];
      }
    // Symmetric sweep of -H, one pivot K = 8 KT + KC at a time (one wave: the pivot
    // column's LDS round trip needs no barrier).  W_ij -= z_i z_j / d, W_iK = z_i / d,
    // W_KK = -1/d (ends at -(-H)^-1 = H^-1, no negation pass that would double the tile's
    // live registers): the pivot row's coefficient made 1/d - 1 turns row K into z_j / d,
    // the pivot column's row-K entry made d - 1 turns column K into z_i / d, then -2 on
    // the pivot (as mpcqp_solve.h's class-64 sweep).
#pragma unroll 1
    for (int KT = 0; 8 * KT < n; ++KT) {
      static_for<8>([&](auto KCc) {
        constexpr int KC = decltype(KCc)::value;
        const int K = 8 * KT + KC;
        if (K < n) {
          double* const zcol = sm.zc[KC & 1];
          if (tc == KT) {
            d2* pz = reinterpret_cast<d2*>(zcol + 8 * tr);
#pragma unroll
            for (int i = 0; i < 4; ++i) pz[i] = d2{Pm[2 * i][KC], Pm[2 * i + 1][KC]};
          }
          fsync<LANES>();
          double zr[8], zi[8];
          ld8(zr, zcol, tc);
          ld8(zi, zcol, tr);
          const double dK = zcol[K];
          const double inv = rcp_nr(dK);
          double beta[8];
#pragma unroll
          for (int r = 0; r < 8; ++r) beta[r] = -zi[r] * inv;
          if (tr == KT) beta[KC] = inv - 1.0;
          if (tc == KT) zr[KC] = dK - 1.0;
#pragma unroll
          for (int r = 0; r < 8; ++r)
#pragma unroll
            for (int c = 0; c < 8; ++c) Pm[r][c] = fma(beta[r], zr[c], Pm[r][c]);
          Pm[KC][KC] += (tc == KT && tr == KT) ? -2.0 : 0.0;
        }
      });
    }
    // P = H^-1; largest diagonal entry; W's 3x3 foot-step blocks; x = -W g
    double wd = 0.0;
    if (tr == tc) {
#pragma unroll
      for (int r = 0; r < 8; ++r)
        if (8 * tr + r < n) wd = fmax(wd, Pm[r][r]);
    }
    wd = wave_max_d(wd);
    if (lane == 0) sm.wmax = wd;
#pragma unroll
    for (int r = 0; r < 8; ++r)
#pragma unroll
      for (int c = 0; c < 8; ++c) {
        const int row = 8 * tr + r, col = 8 * tc + c;
        if (row < n && col < n && row / 3 == col / 3) sm.wb[9 * (row / 3) + 3 * (row % 3) + col % 3] = Pm[r][c];
      }
    {
      double gc[8], acc[8];
      ld8(gc, sm.gv, tc);
#pragma unroll
      for (int r = 0; r < 8; ++r) {
        double a = 0.0, a2 = 0.0;
#pragma unroll
        for (int c = 0; c < 8; c += 2) {
          a = fma(Pm[r][c], gc[c], a);
          a2 = fma(Pm[r][c + 1], gc[c + 1], a2);
        }
        acc[r] = a + a2;
      }
      sm.vx[8 * tr + tc] = -bm_reduce8(acc, lane);
    }
    fsync<NT>();   // (1) W's blocks, x, wmax published
    fsync<NT>();   // (2) the brain has read them

    // ============================================================ muscle: the loop
    // One latch: every round reads the command after barrier A, does its A -> B part
    // (directions, or t = H R_l^T in a drop's helper round), and after barrier B applies
    // the pending update (the brain's HRL command carries none) -- so the tile has a
    // single loop-carried register assignment.
    int pend = BM_NONE, zbuf = 0, dbuf = 0;
    double k0 = 0.0, k1 = 0.0, k2 = 0.0, tx0 = 0.0, tx1 = 0.0;
    SEC(0);
    while (true) {
      fsync<NT>();   // A
      SEC(1);
      const int op = uni(sm.cmd.op);
      pend = uni(sm.cmd.pend);
      zbuf = uni(sm.cmd.zbuf);
      dbuf = uni(sm.cmd.dbuf);
      tx0 = sgpr_d(sm.cmd.tx[0]);
      tx1 = sgpr_d(sm.cmd.tx[1]);
      if (op == BM_EXIT) break;
      k0 = sgpr_d(sm.cmd.k[0]);
      k1 = sgpr_d(sm.cmd.k[1]);
      k2 = sgpr_d(sm.cmd.k[2]);
      if (op == BM_HRL) {
        // t = H R_l^T from H's copy: lane rows 8 tr.., columns 8 tc..
        double rc[8], acc[8];
        ld8(rc, sm.rl[dbuf], tc);
        static_for<8>([&](auto rr) {
          constexpr int r = decltype(rr)::value;
          double a = 0.0, a2 = 0.0;
#pragma unroll
          for (int c = 0; c < 8; c += 2) {
            const d2 hh = sm.ht[(8 * r + c) >> 1][lane];
            a = fma(hh[0], rc[c], a);
            a2 = fma(hh[1], rc[c + 1], a2);
          }
          acc[r] = a + a2;
          __builtin_amdgcn_sched_barrier(0);   // one tile row of H in flight (P holds 128 VGPRs)
        });
        sm.tv[8 * tr + tc] = bm_reduce8(acc, lane);
      } else {
        // ---- directions for p (and p2) from the lagging P plus the pending correction
        const int v0 = uni(sm.cmd.v0), v02 = uni(sm.cmd.v02);
        const int buf = uni(sm.cmd.buf);
        const double a0 = sgpr_d(sm.cmd.a[0]), a1 = sgpr_d(sm.cmd.a[1]), a2 = sgpr_d(sm.cmd.a[2]);
        const double cp0 = sgpr_d(sm.cmd.cp[0]), cp1 = sgpr_d(sm.cmd.cp[1]);
        // the pending update's row vectors (rows 8 tr..): z / z2 (add, pair), R_l (drop)
        double ur[8], ur2[8];
        ld8(ur, pend == BM_DROP ? sm.rl[dbuf] : sm.vz[zbuf], tr);
        ld8(ur2, sm.vz2[zbuf], tr);
        // direction = P_old a + e1 ur + e2 ur2: add (-c, 0), pair (-c1, -c2), drop (+c, 0)
        const double e1 = pend == BM_DROP ? cp0 : (pend == BM_NONE ? 0.0 : -cp0);
        const double e2 = pend == BM_PAIR ? -cp1 : 0.0;
        {
          double zq[8];
          bm_combo(Pm, tc, v0, a0, a1, a2, zq);
#pragma unroll
          for (int r = 0; r < 8; ++r) zq[r] = fma(e2, pend == BM_PAIR ? ur2[r] : 0.0, fma(e1, ur[r], zq[r]));
          if (tc == (v0 >> 3)) st8(sm.vz[buf], tr, zq);
        }
        if (v02 >= 0) {
          const double b0 = sgpr_d(sm.cmd.b[0]), b1 = sgpr_d(sm.cmd.b[1]), b2 = sgpr_d(sm.cmd.b[2]);
          const double cq0 = sgpr_d(sm.cmd.cq[0]), cq1 = sgpr_d(sm.cmd.cq[1]);
          const double f1 = pend == BM_DROP ? cq0 : (pend == BM_NONE ? 0.0 : -cq0);
          const double f2 = pend == BM_PAIR ? -cq1 : 0.0;
          double zq[8];
          bm_combo(Pm, tc, v02, b0, b1, b2, zq);
#pragma unroll
          for (int r = 0; r < 8; ++r) zq[r] = fma(f2, pend == BM_PAIR ? ur2[r] : 0.0, fma(f1, ur[r], zq[r]));
          if (tc == (v02 >> 3)) st8(sm.vz2[buf], tr, zq);
        }
      }
      SEC(2);
      fsync<NT>();   // B
      SEC(3);
      // ---- the pending update of P and x (beside the brain's decisions), as two rank-1
      // sweeps P += co1 uc1^T + co2 uc2^T (coefficients 0 where the kind has no such
      // term); x lives in LDS (vx), rows 8 tr.. updated by the lanes of tile column 0
      if (pend != BM_NONE) {
        const bool dr = pend == BM_DROP, pr = pend == BM_PAIR;
        const double* v1 = dr ? sm.rl[dbuf] : sm.vz[zbuf];
        double r1[8], r2[8], co[8], uc[8];
        ld8(r1, v1, tr);
        ld8(r2, sm.vz2[zbuf], tr);
        ld8(uc, v1, tc);
        // add: -z/sigma; pair: -(i11 z + i12 z2); drop: R_l/eta
        const double s1 = dr ? k0 : -k0, s2 = pr ? -k1 : 0.0;
#pragma unroll
        for (int r = 0; r < 8; ++r) {
          co[r] = fma(s1, r1[r], s2 * (pr ? r2[r] : 0.0));
#pragma unroll
          for (int c = 0; c < 8; ++c) Pm[r][c] = fma(co[r], uc[c], Pm[r][c]);
        }
        ld8(uc, sm.vz2[zbuf], tc);
        const double t1 = pr ? -k1 : 0.0, t2 = pr ? -k2 : 0.0;
#pragma unroll
        for (int r = 0; r < 8; ++r) {
          co[r] = pr ? fma(t1, r1[r], t2 * r2[r]) : 0.0;
#pragma unroll
          for (int c = 0; c < 8; ++c) Pm[r][c] = fma(co[r], pr ? uc[c] : 0.0, Pm[r][c]);
        }
        if (tc == 0) {
          double xr[8], zr[8];
          ld8(xr, sm.vx, tr);
          ld8(zr, sm.vz[zbuf], tr);
#pragma unroll
          for (int r = 0; r < 8; ++r) xr[r] = fma(pr ? tx1 : 0.0, pr ? r2[r] : 0.0, fma(tx0, zr[r], xr[r]));
          st8(sm.vx, tr, xr);
        }
      }
    }
    // ---- exit: the last pending x step
    if (tc == 0 && pend != BM_NONE) {
      double xr[8], zr[8];
      ld8(xr, sm.vx, tr);
      ld8(zr, sm.vz[zbuf], tr);
#pragma unroll
      for (int r = 0; r < 8; ++r) xr[r] = fma(tx0, zr[r], xr[r]);
      if (pend == BM_PAIR) {
        ld8(zr, sm.vz2[zbuf], tr);
#pragma unroll
        for (int r = 0; r < 8; ++r) xr[r] = fma(tx1, zr[r], xr[r]);
      }
      st8(sm.vx, tr, xr);
    }
    SEC(0);
    fsync<NT>();   // C
#ifdef MPCQP_STAMPS
    if (lane < 16 && Ug && 40 < N * 6) reinterpret_cast<unsigned long long*>(Ug + (size_t)b * N * 12)[24 + lane] = secacc_;
#endif
    return;   // the brain writes the outputs
  }

  // ============================================================ brain (wave 1)
  fsync<NT>();   // (1)
  STAMP(3);
  const double wscale = sgpr_d(sm.wmax);
  const float qfloor = fmaxf((float)(1e-9 * wscale), 1e-30f);
  const int fz0i = uni(sm.mt.fz0_implied);
  int cz[CPL], crt[CPL];
  double s[CPL], zs[CPL], zs2[CPL];
  float qm[CPL];
  auto cdot = [&](const double* v, int k) -> double {
    const double* a = sm.mt.rows[crt[k]];
    const double* vf = v + cz[k];
    return a[0] * vf[0] + a[1] * vf[1] + a[2] * vf[2];
  };
  auto cbound = [&](int k) -> double { return crt[k] == 5 ? sm.mt.ub[cz[k] / 3] : 0.0; };
#pragma unroll
  for (int k = 0; k < CPL; ++k) {
    const int c = lane + LANES * k;
    const bool ok = c < m;
    cz[k] = ok ? 3 * (c / 6) : 0;
    crt[k] = ok ? c % 6 : 0;
    const bool live = ok && !(crt[k] == 4 && fz0i);
    s[k] = live ? cdot(sm.vx, k) + cbound(k) : INFINITY;
    const double* a = sm.mt.rows[crt[k]];
    const double* w = sm.wb + 3 * cz[k];
    double q = 0.0;
#pragma unroll
    for (int i = 0; i < 3; ++i) q = fma(a[i], fma(w[3 * i], a[0], fma(w[3 * i + 1], a[1], w[3 * i + 2] * a[2])), q);
    qm[k] = ok && q > 0.0 ? (float)q : 1.0f;
    zs[k] = 0.0;
    zs2[k] = 0.0;
  }
  fsync<NT>();   // (2) wb / gv are dead: the loop reuses their space
  STAMP(4);

  double Rr[64];
  static_for<64>([&](auto jj) { Rr[decltype(jj)::value] = 0.0; });
  double u = 0.0;
  unsigned long long occ = 0ull;   // wave-uniform slot mask
  // this pass's directions at the lane's slot, and the pending update's (brain side)
  double rc = 0.0, r2c = 0.0, rp = 0.0, rp2 = 0.0, yp = 0.0;
  int pend = BM_NONE, pq = 0, pq2 = 0, pl = 0, zbuf = 0, dbuf = 0;
  double pk0 = 0.0, pk1 = 0.0, pk2 = 0.0, ptx0 = 0.0, ptx1 = 0.0;
  bool hrl = false;   // a drop waits for its helper round
  int dl = 0, dpar = 0;
  double dt = 0.0;
  const int max_iter = P.max_iter > 0 ? P.max_iter : 8 * 64 + 64;
  const double tol = 1e-9;
  int it = 0, buf = 0;
  int status = MPCQP_STATUS_OK;
  int p = -1, p2 = -1;
  double a0 = 0.0, a1 = 0.0, a2 = 0.0, thr = 0.0, sp = 0.0, up = 0.0;
  double b0 = 0.0, b1 = 0.0, b2 = 0.0, thr2 = 0.0, sp2 = 0.0;
  int fp = 0, fq = 0;   // foot-steps of p, p2
  bool exiting = false;

  // correction coefficients of the pending update for the direction of row c (foot-step f, row e)
  auto corr = [&](int c, int f, double e0, double e1, double e2, double& c0, double& c1) __attribute__((always_inline)) {
    c0 = 0.0;
    c1 = 0.0;
    if (pend == BM_ADD) {
      const double zc = readlane_d((c >> 6) ? zs[1] : zs[0], c & 63);
      c0 = sgpr_d(zc * pk0);
    } else if (pend == BM_PAIR) {
      const double zc = readlane_d((c >> 6) ? zs[1] : zs[0], c & 63);
      const double zc2 = readlane_d((c >> 6) ? zs2[1] : zs2[0], c & 63);
      c0 = sgpr_d(fma(pk0, zc, pk1 * zc2));
      c1 = sgpr_d(fma(pk1, zc, pk2 * zc2));
    } else if (pend == BM_DROP) {
      const double v = bm_rsel<0, 20>(Rr, uni(f), e0, e1, e2);
      c0 = sgpr_d(readlane_d(v, pl) * pk0);
    }
  };
  // this pass's r at the lane's slot from the lagging R plus the pending correction
  auto rdir = [&](int f, double e0, double e1, double e2, double c0, double c1) __attribute__((always_inline)) -> double {
    double v = bm_rsel<0, 20>(Rr, uni(f), e0, e1, e2);
    if (pend == BM_ADD) {
      v = fma(-c0, rp - (lane == pq ? 1.0 : 0.0), v);
    } else if (pend == BM_PAIR) {
      v = fma(-c1, rp2 - (lane == pq2 ? 1.0 : 0.0), fma(-c0, rp - (lane == pq ? 1.0 : 0.0), v));
    } else if (pend == BM_DROP) {
      v = lane == pl ? 0.0 : fma(-c0, yp, v);
    }
    return v;
  };

  // One latch (as the muscle's): the command, barrier A, the A -> B part (r, r2 and the
  // pending update of R), barrier B, the B -> A part (a SOLVE pass's decisions or a drop
  // helper round's y) -- R keeps a single loop-carried register assignment.
  SEC(0);
  while (true) {
    // the brain's control state is wave-uniform: readfirstlane keeps it in SGPRs (the
    // divergence analysis cannot prove it through the loop's phis, and a "divergent"
    // pend / p would turn every branch below into an exec-masked one)
    pend = uni(pend);
    p = uni(p);
    zbuf = uni(zbuf);
    dbuf = uni(dbuf);
    buf = uni(buf);
    dpar = uni(dpar);
    pq = uni(pq);
    pq2 = uni(pq2);
    pl = uni(pl);
    dl = uni(dl);
    it = uni(it);
    fp = uni(fp);
    hrl = uni((int)hrl) != 0;
    exiting = uni((int)exiting) != 0;
    sp = sgpr_d(sp);
    up = sgpr_d(up);
    pk0 = sgpr_d(pk0);
    pk1 = sgpr_d(pk1);
    pk2 = sgpr_d(pk2);
    ptx0 = sgpr_d(ptx0);
    ptx1 = sgpr_d(ptx1);
    dt = sgpr_d(dt);
    a0 = sgpr_d(a0);
    a1 = sgpr_d(a1);
    a2 = sgpr_d(a2);
    thr = sgpr_d(thr);
    int op;
    double cp0 = 0.0, cp1 = 0.0, cq0 = 0.0, cq1 = 0.0;
    if (hrl) {
      op = BM_HRL;
      if (lane == 0) {
        sm.cmd.op = BM_HRL;
        sm.cmd.pend = BM_NONE;   // the pending update was applied by both sides this pass
        sm.cmd.dbuf = dpar;
        sm.cmd.zbuf = zbuf;
        sm.cmd.tx[0] = 0.0;
        sm.cmd.tx[1] = 0.0;
      }
    } else {
      p2 = -1;
      if (p < 0) {
        // the most violated row in the current metric (f32 keys, lowest lane on ties),
        // then the best row of any other foot-step (the pair candidate)
        double key[CPL];
#pragma unroll
        for (int k = 0; k < CPL; ++k)
          key[k] = s[k] < -tol ? s[k] * (double)__builtin_amdgcn_rsqf(fmaxf(qm[k], qfloor)) : INFINITY;
        double bv = key[0];
        int bk = 0;
#pragma unroll
        for (int k = 1; k < CPL; ++k) {
          bk = key[k] < bv ? k : bk;
          bv = vmin(bv, key[k]);
        }
        double kmn;
        const int pl0 = wave_argmin_f32(bv, kmn);
        if (!(kmn < INFINITY)) {
          exiting = true;
        } else {
          p = pl0 + LANES * uni(__builtin_amdgcn_readlane(bk, pl0));
          const int vc = 3 * (p / 6);
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
          if (kmn2 < INFINITY) p2 = ql + LANES * uni(__builtin_amdgcn_readlane(bk2, ql));
          sp = sgpr_d(readlane_d((p >> 6) ? s[1] : s[0], p & 63));
          up = 0.0;
          const int rp_ = p % 6;
          a0 = sgpr_d(sm.mt.rows[rp_][0]);
          a1 = sgpr_d(sm.mt.rows[rp_][1]);
          a2 = sgpr_d(sm.mt.rows[rp_][2]);
          thr = sgpr_d(1e-12 * (a0 * a0 + a1 * a1 + a2 * a2) * wscale);
          fp = p / 6;
          if (p2 >= 0) {
            sp2 = sgpr_d(readlane_d((p2 >> 6) ? s[1] : s[0], p2 & 63));
            const int rq = p2 % 6;
            b0 = sgpr_d(sm.mt.rows[rq][0]);
            b1 = sgpr_d(sm.mt.rows[rq][1]);
            b2 = sgpr_d(sm.mt.rows[rq][2]);
            thr2 = sgpr_d(1e-12 * (b0 * b0 + b1 * b1 + b2 * b2) * wscale);
            fq = p2 / 6;
          }
        }
      }
      if (!exiting && ++it > max_iter) {
        status = MPCQP_STATUS_MAX_ITER;
        exiting = true;
      }
      if (exiting) {
        op = BM_EXIT;
        if (lane == 0) {
          sm.cmd.op = BM_EXIT;
          sm.cmd.pend = pend;
          sm.cmd.zbuf = zbuf;
          sm.cmd.tx[0] = ptx0;
          sm.cmd.tx[1] = ptx1;
        }
      } else {
        op = BM_SOLVE;
        corr(p, fp, a0, a1, a2, cp0, cp1);
        if (p2 >= 0) corr(p2, fq, b0, b1, b2, cq0, cq1);
        if (lane == 0) {
          sm.cmd.op = BM_SOLVE;
          sm.cmd.v0 = 3 * fp;
          sm.cmd.v02 = p2 >= 0 ? 3 * fq : -1;
          sm.cmd.pend = pend;
          sm.cmd.zbuf = zbuf;
          sm.cmd.dbuf = dbuf;
          sm.cmd.buf = buf;
          sm.cmd.a[0] = a0;
          sm.cmd.a[1] = a1;
          sm.cmd.a[2] = a2;
          sm.cmd.b[0] = b0;
          sm.cmd.b[1] = b1;
          sm.cmd.b[2] = b2;
          sm.cmd.cp[0] = cp0;
          sm.cmd.cp[1] = cp1;
          sm.cmd.cq[0] = cq0;
          sm.cmd.cq[1] = cq1;
          sm.cmd.k[0] = pk0;
          sm.cmd.k[1] = pk1;
          sm.cmd.k[2] = pk2;
          sm.cmd.tx[0] = ptx0;
          sm.cmd.tx[1] = ptx1;
        }
      }
    }
    op = uni(op);
    p2 = uni(p2);
    fq = uni(fq);
    SEC(1);
    CNT(op == BM_HRL ? 11 : 10);
    fsync<NT>();   // A
    SEC(2);
    if (op == BM_EXIT) break;
    // ---------------------------------------------------------------- A -> B
    if (op == BM_SOLVE) {
      rc = rdir(fp, a0, a1, a2, cp0, cp1);
      r2c = p2 >= 0 ? rdir(fq, b0, b1, b2, cq0, cq1) : 0.0;
    }
    // the pending update of R as one sweep R_row -= al v1 (- be v2 for a pair); a drop's
    // row l takes al = 1 against its own bitwise copy in rl: exactly 0
    if (pend != BM_NONE) {
      double al, be = 0.0;
      if (pend == BM_ADD) {
        al = (rp - (lane == pq ? 1.0 : 0.0)) * pk0;
      } else if (pend == BM_PAIR) {
        const double e1 = rp - (lane == pq ? 1.0 : 0.0), e2 = rp2 - (lane == pq2 ? 1.0 : 0.0);
        al = fma(pk0, e1, pk1 * e2);
        be = fma(pk1, e1, pk2 * e2);
      } else {
        al = lane == pl ? 1.0 : yp * pk0;
      }
      const double* v1 = pend == BM_DROP ? sm.rl[dbuf] : sm.vz[zbuf];
      static_for<32>([&](auto jj) {
        constexpr int j = 2 * decltype(jj)::value;
        const d2 zz = *reinterpret_cast<const d2*>(v1 + j);
        Rr[j] = fma(-al, zz[0], Rr[j]);
        Rr[j + 1] = fma(-al, zz[1], Rr[j + 1]);
        if constexpr ((j & 7) == 6) __builtin_amdgcn_sched_barrier(0);   // 8 columns in flight
      });
      if (pend == BM_PAIR) {
        const double* v2 = sm.vz2[zbuf];
        static_for<32>([&](auto jj) {
          constexpr int j = 2 * decltype(jj)::value;
          const d2 zz = *reinterpret_cast<const d2*>(v2 + j);
          Rr[j] = fma(-be, zz[0], Rr[j]);
          Rr[j + 1] = fma(-be, zz[1], Rr[j + 1]);
          if constexpr ((j & 7) == 6) __builtin_amdgcn_sched_barrier(0);
        });
      }
    }
    pend = BM_NONE;
    SEC(3);
    fsync<NT>();   // B
    SEC(op == BM_HRL ? 5 : 4);
    // ---------------------------------------------------------------- B -> A
    if (op == BM_HRL) {
      double y = 0.0, y2 = 0.0;
      static_for<32>([&](auto jj) {
        constexpr int j = 2 * decltype(jj)::value;
        const d2 tt = *reinterpret_cast<const d2*>(sm.tv + j);
        y = fma(Rr[j], tt[0], y);
        y2 = fma(Rr[j + 1], tt[1], y2);
        if constexpr ((j & 7) == 6) __builtin_amdgcn_sched_barrier(0);
      });
      y += y2;
      const double eta = readlane_d(y, dl);
      const double ie = sgpr_d(rcp_nr(eta));
#pragma unroll
      for (int k = 0; k < CPL; ++k) {   // q_c += (a_c . R_l)^2 / eta
        const double ar = cdot(sm.rl[dpar], k);
        qm[k] = (float)fma(ar * ar, ie, (double)qm[k]);
      }
      u = lane == dl ? 0.0 : u;
      occ &= ~(1ull << dl);
      pend = BM_DROP;
      pk0 = ie;
      pk1 = 0.0;
      pk2 = 0.0;
      ptx0 = dt;
      ptx1 = 0.0;
      pl = dl;
      yp = y;
      dbuf = dpar;
      dpar ^= 1;
      hrl = false;
    } else {
      const double* zv = sm.vz[buf];
#pragma unroll
      for (int k = 0; k < CPL; ++k) zs[k] = cdot(zv, k);
      const double zsp = readlane_d((p >> 6) ? zs[1] : zs[0], p & 63);
      const bool mine = (occ >> lane) & 1ull;
      bool paired = false;
      if (p2 >= 0) {
        const double* zv2 = sm.vz2[buf];
#pragma unroll
        for (int k = 0; k < CPL; ++k) zs2[k] = cdot(zv2, k);
        const double s12 = sgpr_d(readlane_d((p >> 6) ? zs2[1] : zs2[0], p & 63));    // a_p . z2
        const double s22 = sgpr_d(readlane_d((p2 >> 6) ? zs2[1] : zs2[0], p2 & 63));  // a_p2 . z2
        const double det = zsp * s22 - s12 * s12;
        bool ok = zsp > thr && s22 > thr2 && det > thr2 * zsp;
        double tp = 0.0, tq = 0.0, id = 0.0;
        if (ok) {
          id = rcp_nr(det);
          tp = sgpr_d((s12 * sp2 - s22 * sp) * id);
          tq = sgpr_d((s12 * sp - zsp * sp2) * id);
          ok = tp > 0.0 && tq > 0.0;
        }
        if (ok) {
          const double un = fma(-tq, r2c, fma(-tp, rc, u));
          ok = !__any(mine && un < 0.0);
          if (ok) {
            u = mine ? un : u;
#pragma unroll
            for (int k = 0; k < CPL; ++k) {
              const int c = lane + LANES * k;
              s[k] = (c == p || c == p2) ? 0.0 : fma(tq, zs2[k], fma(tp, zs[k], s[k]));
            }
            const unsigned long long f0 = ~occ;
            const int qa = __builtin_ctzll(f0);
            const int qb = __builtin_ctzll(f0 & (f0 - 1));
            u = lane == qa ? tp : (lane == qb ? tq : u);
            occ |= (1ull << qa) | (1ull << qb);
            const double i11 = s22 * id, i12 = -s12 * id, i22 = zsp * id;
#pragma unroll
            for (int k = 0; k < CPL; ++k)
              qm[k] = (float)((double)qm[k] - fma(i11 * zs[k], zs[k], fma(2.0 * i12 * zs[k], zs2[k], i22 * zs2[k] * zs2[k])));
            pend = BM_PAIR;
            pk0 = sgpr_d(i11);
            pk1 = sgpr_d(i12);
            pk2 = sgpr_d(i22);
            ptx0 = tp;
            ptx1 = tq;
            pq = qa;
            pq2 = qb;
            rp = rc;
            rp2 = r2c;
            zbuf = buf;
            p = -1;
            ++it;   // a pair step counts as the two additions it makes
            paired = true;
          }
        }
      }
      if (!paired) {
        // dual step bound t1 (blocking slot l), primal step t2
        const double ratio = (mine && rc > 0.0) ? div_nr(u, rc) : INFINITY;
        double t1;
        const int l = wave_argmin_d(ratio, t1);
        double t2 = INFINITY;
        if (zsp > thr) t2 = div_nr(-sp, zsp);
        const bool add = t2 <= t1;
        const double tstep = add ? t2 : t1;
        if (!(tstep < INFINITY)) {
          status = MPCQP_STATUS_INFEASIBLE;
          exiting = true;   // no pending step: the command carries the previous one (none)
        } else {
          u = mine ? fma(-tstep, rc, u) : u;
#pragma unroll
          for (int k = 0; k < CPL; ++k) s[k] = fma(tstep, zs[k], s[k]);
          sp = sgpr_d(fma(tstep, zsp, sp));
          up = sgpr_d(up + tstep);
          if (add) {
            const int q = __builtin_ctzll(~occ);
            const double is = rcp_nr(zsp);
#pragma unroll
            for (int k = 0; k < CPL; ++k) qm[k] = (float)fma(-zs[k] * zs[k], is, (double)qm[k]);
            u = lane == q ? up : u;
            occ |= 1ull << q;
#pragma unroll
            for (int k = 0; k < CPL; ++k) s[k] = (lane + LANES * k == p) ? 0.0 : s[k];
            pend = BM_ADD;
            pk0 = sgpr_d(is);
            ptx0 = tstep;
            ptx1 = 0.0;
            pq = q;
            rp = rc;
            zbuf = buf;
            p = -1;
          } else {
            // drop slot l: R_l to LDS, y = R H R_l^T after the helper round
            if (lane == l) {
              d2* dst = reinterpret_cast<d2*>(sm.rl[dpar]);
              static_for<32>([&](auto jj) {
                constexpr int j = 2 * decltype(jj)::value;
                dst[j >> 1] = d2{Rr[j], Rr[j + 1]};
              });
            }
            hrl = true;
            dl = l;
            dt = tstep;
            zbuf = buf;   // the drop pass's x step runs along this pass's z
          }
        }
      }
      buf ^= 1;
    }
    SEC(0);
  }
  SEC(6);
  STAMP(5);

  // ------------------------------- final x, KKT verification, output
  fsync<NT>();   // C: x in vx
  STAMP(6);
#ifdef MPCQP_STAMPS
  if (Ug && 40 < N * 6) {
    unsigned long long* dst = reinterpret_cast<unsigned long long*>(Ug + (size_t)b * N * 12);
    if (lane < 7) {
      unsigned long long v = stamps_[0];
#pragma unroll
      for (int i = 1; i < 7; ++i) v = lane == i ? stamps_[i] : v;
      dst[lane] = v;
    }
    if (lane < 16) dst[8 + lane] = secacc_;
  }
  Ug = nullptr;
#endif
  {
    int bad = 0;
#pragma unroll
    for (int k = 0; k < CPL; ++k) {
      if (lane + LANES * k < m) {
        const double v = cdot(sm.vx, k) + cbound(k);
        bad |= (v < -1e-6) || !isfinite(v);
      }
    }
    if ((occ >> lane) & 1ull) bad |= (u < -1e-9);
    if (__any(bad) && status == MPCQP_STATUS_OK) status = MPCQP_STATUS_MAX_ITER;
  }
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
