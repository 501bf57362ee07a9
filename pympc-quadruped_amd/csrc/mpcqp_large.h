// mpcqp_large.h -- the large capacity class of the engine (included by mpcqp.hip,
// inside its anonymous namespace; uses its constants and helpers).
//
// Robots whose stance variables do not fit one wave (n = 3 * #stance > 64: horizon
// 16/20 trot/pace/bound, standing at N <= 10) are queued by mpcqp_kernel and solved
// here by ONE WORKGROUP OF 8 WAVES PER ROBOT (512 lanes) over a device work queue.  Same algorithm as the wave kernel:
// float32-faithful model, exact discretisation, Toeplitz-condensed H/g over the
// stance variables, W = H^-1 by symmetric sweep, Goldfarb-Idnani dual active set
// with an explicit (M_AA)^-1, refinement and KKT check.
//
// Register layout: both W = H^-1 (n <= 126, padded to 128) and (M_AA)^-1 (128
// slots) live in VGPRs as 4x8 tiles: lane t = (tr, tc) = (t >> 4, t & 15) holds
// rows 4tr..4tr+3, columns 8tc..8tc+7 (32 doubles each matrix).  A matvec is 32
// FMAs per lane plus a 16-lane DPP reduction (no LDS), then one LDS write and a
// workgroup barrier to redistribute the result.  Lane t is also constraint row t
// (m = 6 * #stance <= 252), variable t and slot t.

constexpr int LW = 8;                  // waves per robot
constexpr int LT = LW * LANES;         // 512 threads
constexpr int NL = 128;                // variable / active-slot capacity (tiles)
constexpr int SL = 42;                 // stance foot-steps: n = 3 * 42 = 126 <= NL
constexpr int ML = 6 * SL;             // 252 constraint rows
constexpr int PL = NL + 8;             // padded vector (pv(127) = 133)
constexpr int DPP_ROR8 = 0x128;        // row_ror:8 -> lane i <-> i ^ 8 inside 16 lanes

struct alignas(16) LShared {
  static_assert(PL % 2 == 0, "16-B vector rows");
  // formulation
  double Ac[NX * NX], Nm[NX * NX], Bc[NX * NU];
  double X[3 * NX * NU];               // X_p[s][c]
  double e[kMaxN * NX];                // A^{t+1} x0 - xref_t
  double zp[3 * kMaxN * NU];           // sum_s X_p[s][c] Q_s e_t[s]
  double Y[9 * NU * NU];               // Y_pq[c][c2]
  double T[9 * kNT];                   // Toeplitz weights
  double x0[NX], y1[NX], y2[NX];
  double qd[NX], rd[NU];               // cost weights
  double ii[9];
  double rows[6][3];
  double ub[SL + 1];
  // solve -- every vector read with ds_read_b128 is 16-B aligned (an unaligned
  // b128 access is replayed at ~64 cycles per wave-instruction)
  alignas(16) double vb[PL];           // matvec right-hand side (padded)
  alignas(16) double zc[2][PL];        // sweep pivot column, double-buffered
  alignas(16) double rr[PL];           // r = Minv mp (padded, slot-indexed)
  alignas(16) double cv[PL];           // dropped column of Minv (padded)
  alignas(16) double rv[PL];
  alignas(16) double wv[NL];
  alignas(16) double zv[NL];
  alignas(16) double gv[NL];
  double redv[2][LW];                  // per-wave argmin partials (double-buffered)
  int redi[2][LW];
  double bc_zs, bc_s;                  // zs_p, s_p broadcast
  int foot_t[SL + 1], foot_leg[SL + 1];
  int stance_of[4 * kMaxN];
  int S;
  float in[IN_END];
};

// y = M v on the 4x8 tiles; v padded in LDS.  Returns the sum for row 4tr + R with
// R = 2 bit2(lane) + bit1(lane), valid in every lane (4 copies per row).
__device__ __forceinline__ double ltile_matvec(const double (&M)[4][8], const double* v, int tc, int lane) {
  double vs[8];
  ld8(vs, v, tc);
  MPCQP_FENCE();
  double acc[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    double a = 0.0, b2 = 0.0;
#pragma unroll
    for (int c = 0; c < 8; c += 2) {
      a = fma(M[r][c], vs[c], a);
      b2 = fma(M[r][c + 1], vs[c + 1], b2);
    }
    acc[r] = a + b2;
  }
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
  y += dpp_d<DPP_ROR8>(y);
  return y;
}

// row index of the value ltile_matvec leaves in this lane, and whether the lane
// is the one copy that writes it out
__device__ __forceinline__ int lrow(int tr, int lane) { return 4 * tr + 2 * ((lane >> 2) & 1) + ((lane >> 1) & 1); }
__device__ __forceinline__ bool lwriter(int lane) { return (lane & 9) == 0; }

// 4 consecutive padded doubles at element 4k (16-B aligned; never straddles a pad)
__device__ __forceinline__ void ld4(double (&v)[4], const double* base, int k) {
  const d2* p = reinterpret_cast<const d2*>(base + pv(4 * k));
  const d2 a = p[0], b = p[1];
  v[0] = a[0]; v[1] = a[1]; v[2] = b[0]; v[3] = b[1];
}

// Workgroup argmin: lowest index attaining the minimum of v over all lanes
// (idx increasing with the thread id).  Contains one barrier.
__device__ __forceinline__ int lwg_argmin(double v, int idx, LShared& sm, int wave, int lane, int& buf,
                                          double& vmin) {
  const double wm = wave_min(v);
  const unsigned long long msk = __ballot(v == wm);
  const int wi = msk ? __builtin_amdgcn_readlane(idx, __builtin_ctzll(msk)) : 0x7fffffff;
  if (lane == 0) {
    sm.redv[buf][wave] = wm;
    sm.redi[buf][wave] = wi;
  }
  __syncthreads();
  double best = sm.redv[buf][0];
  int bi = sm.redi[buf][0];
#pragma unroll
  for (int k = 1; k < LW; ++k) {
    const double x = sm.redv[buf][k];
    const int j = sm.redi[buf][k];
    if (x < best || (x == best && j < bi)) {
      best = x;
      bi = j;
    }
  }
  buf ^= 1;
  vmin = best;
  return uni(bi);
}

// One pivot K = 8 KT + KC of the symmetric sweep over the 4x8 tiles (see
// sweep_step).  KC is compile-time (register column), KT a runtime loop index:
// the sweep's code is 8 pivots long, so it stays in the instruction cache.
template <int KC>
__device__ __forceinline__ void lsweep_pivot(double (&W)[4][8], LShared& sm, int tr, int tc, int KT, int n) {
  const int K = 8 * KT + KC;
  if (K < n) {
    constexpr int KRR = KC & 3;
    const int KR = 2 * KT + (KC >> 2);
    double* const zc = sm.zc[KC & 1];
    if (tc == KT) {
      d2* p = reinterpret_cast<d2*>(zc + pv(4 * tr));
      p[0] = d2{W[0][KC], W[1][KC]};
      p[1] = d2{W[2][KC], W[3][KC]};
    }
    __syncthreads();
    double zr[8], zi[4];
    ld8(zr, zc, tc);
    ld4(zi, zc, tr);
    const double d = zc[pv(K)];
    MPCQP_FENCE();
    const double inv = 1.0 / d;
    double beta[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) beta[r] = -zi[r] * inv;
    if (tr == KR) beta[KRR] = inv - 1.0;
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
      for (int c = 0; c < 8; ++c) W[r][c] = fma(beta[r], zr[c], W[r][c]);
    if (tc == KT) {
#pragma unroll
      for (int r = 0; r < 4; ++r) W[r][KC] = zi[r] * inv;
      if (tr == KR) W[KRR][KC] = -inv;
    }
  }
}

__device__ __forceinline__ void lsweep_all(double (&W)[4][8], LShared& sm, int tr, int tc, int n,
                                           unsigned long long* dbg) {
#pragma unroll 1
  for (int KT = 0; 8 * KT < n; ++KT) {
#ifdef MPCQP_STAMPS
    if (dbg && threadIdx.x == 0) dbg[KT] = __builtin_amdgcn_s_memtime();
#endif
    static_for<8>([&](auto C) { lsweep_pivot<decltype(C)::value>(W, sm, tr, tc, KT, n); });
  }
}

__device__ __forceinline__ void lwrite_empty(int b, int tid, int N, int code, float* u0g, float* Ug, int* statusg,
                                             int* itersg) {
  if (tid < 12) u0g[(size_t)b * 12 + tid] = 0.f;
  if (Ug)
    for (int k = tid; k < N * 12; k += LT) Ug[(size_t)b * N * 12 + k] = 0.f;
  if (tid == 0) {
    if (statusg) statusg[b] = code;
    if (itersg) itersg[b] = 0;
  }
}

// ---------------------------------------------------------------- one robot
__device__ __forceinline__ void lsolve_robot(const KParams& P, int b, LShared& sm, const float* __restrict__ x0g,
                                             const float* __restrict__ xrefg, const float* __restrict__ contactg,
                                             const float* __restrict__ feetg, const float* __restrict__ robotg,
                                             float* __restrict__ u0g, float* __restrict__ Ug,
                                             int* __restrict__ statusg, int* __restrict__ itersg) {
  const int tid = threadIdx.x;
  const int lane = tid & (LANES - 1), wave = tid >> 6;
  const int tr = tid >> 4, tc = tid & 15;
  const int N = P.N;
  float* const in = sm.in;
#ifdef MPCQP_STAMPS
  unsigned long long stamps_[7];
#endif
  STAMP(0);

  // ------------------------------------------------------------ stage inputs
  {
    const float* xb = x0g + (size_t)b * NX;
    const float* fb = feetg + (size_t)b * 12;
    const float* rb = robotg + (size_t)b * MPCQP_ROBOT_STRIDE;
    const float* cb = contactg + (size_t)b * N * 4;
    const float* xrb = xrefg + (size_t)b * N * NX;
    if (tid < NX) in[IN_X0 + tid] = xb[tid];
    else if (tid < NX + 12) in[IN_FEET + tid - NX] = fb[tid - NX];
    else if (tid < NX + 12 + MPCQP_ROBOT_STRIDE) in[IN_ROBOT + tid - NX - 12] = rb[tid - NX - 12];
    if (tid < 4 * N) in[IN_CONTACT + tid] = cb[tid];
    if (tid < NX * N) in[IN_XREF + tid] = xrb[tid];
  }
  __syncthreads();
  {
    int bad = 0;
    if (tid < NX * N) bad |= !isfinite(in[IN_XREF + tid]);
    if (tid < NX + 12 + 12) bad |= !isfinite(in[tid]);
    if (__syncthreads_or(bad)) {
      lwrite_empty(b, tid, N, MPCQP_STATUS_NONFINITE, u0g, Ug, statusg, itersg);
      return;
    }
  }
  const float* const rbs = in + IN_ROBOT;

  // ------------------------------------------------ stance list (wave 0)
  if (wave == 0) {
    const unsigned long long lt_mask = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
    const int nk = 4 * N;
    const float c0 = lane < nk ? in[IN_CONTACT + lane] : 0.f;
    const float c1 = lane + LANES < nk ? in[IN_CONTACT + lane + LANES] : 0.f;
    const bool f0 = c0 > 0.f, f1 = c1 > 0.f;
    const unsigned long long m0 = __ballot(f0), m1 = __ballot(f1);
    const int S0 = __popcll(m0);
    const int i0 = __popcll(m0 & lt_mask), i1 = S0 + __popcll(m1 & lt_mask);
    const double fzmax = (double)rbs[8];
    if (lane < nk) sm.stance_of[lane] = f0 ? i0 : -1;
    if (lane + LANES < nk) sm.stance_of[lane + LANES] = f1 ? i1 : -1;
    if (f0 && i0 < SL) {
      sm.foot_t[i0] = lane / 4;
      sm.foot_leg[i0] = lane % 4;
      sm.ub[i0] = (double)c0 * fzmax;
    }
    if (f1 && i1 < SL) {
      sm.foot_t[i1] = (lane + LANES) / 4;
      sm.foot_leg[i1] = (lane + LANES) % 4;
      sm.ub[i1] = (double)c1 * fzmax;
    }
    if (lane == 0) sm.S = S0 + __popcll(m1);
  }
  __syncthreads();
  const int S = uni(sm.S);
  const int n = 3 * S, m = 6 * S;
  if (n > NL - 2) {
    lwrite_empty(b, tid, N, MPCQP_STATUS_TOO_LARGE, u0g, Ug, statusg, itersg);
    return;
  }

  // ------------------------------------------------ 1. model (mpc.py:173-192)
  double* const Ac = sm.Ac;
  double* const Bc = sm.Bc;
  for (int k = tid; k < NX * NX + NX * NU; k += LT) (k < NX * NX ? Ac[k] : Bc[k - NX * NX]) = 0.0;
  if (tid < NX) sm.x0[tid] = (double)in[IN_X0 + tid];
  if (tid < NX) sm.qd[tid] = P.q[tid];
  if (tid < NU) sm.rd[tid] = P.r[tid];
  {
    const double yaw = (double)in[IN_X0 + 2];
    const double c = f32r(cos(yaw)), s = f32r(sin(yaw));
    const int i = tid / 3, j = tid % 3;
    auto rz = [&](int a, int bb) -> double {
      return a == 2 ? (bb == 2 ? 1.0 : 0.0) : (bb == 2 ? 0.0 : (a == bb ? c : (a == 0 ? -s : s)));
    };
    auto ib = [&](int a, int bb) -> double {
      const int lo = a < bb ? a : bb, hi = a < bb ? bb : a;
      const int idx = lo == 0 ? hi : (lo == 1 ? 2 + hi : 5);
      return (double)rbs[1 + idx];
    };
    double iw = 0.0;
    if (tid < 9) sm.ii[tid] = f32r(rz(i, 0) * ib(0, j) + rz(i, 1) * ib(1, j) + rz(i, 2) * ib(2, j));
    __syncthreads();
    if (tid < 9) iw = f32r(sm.ii[3 * i] * rz(j, 0) + sm.ii[3 * i + 1] * rz(j, 1) + sm.ii[3 * i + 2] * rz(j, 2));
    __syncthreads();
    if (tid < 9) sm.ii[tid] = iw;
    __syncthreads();
    if (tid < 9) {
      const double* I = sm.ii;
      const int r1 = (j + 1) % 3, r2 = (j + 2) % 3, c1 = (i + 1) % 3, c2 = (i + 2) % 3;
      const double cof = I[r1 * 3 + c1] * I[r2 * 3 + c2] - I[r1 * 3 + c2] * I[r2 * 3 + c1];
      const double det = I[0] * (I[4] * I[8] - I[5] * I[7]) - I[1] * (I[3] * I[8] - I[5] * I[6]) +
                         I[2] * (I[3] * I[7] - I[4] * I[6]);
      iw = f32r(cof / det);
    }
    __syncthreads();
    if (tid < 9) sm.ii[tid] = iw;
    if (tid < 9) Ac[i * NX + 6 + j] = rz(j, i);
    if (tid < 3) Ac[(3 + tid) * NX + 9 + tid] = 1.0;
    if (tid == 0) Ac[11 * NX + 12] = 1.0;
    if (tid >= 64 && tid < 64 + 18) {   // cone rows (another wave)
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
      const int rr = (tid - 64) / 3, k = (tid - 64) % 3;
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
  __syncthreads();
  if (tid < 36) {
    const int leg = tid / 9, i = (tid % 9) / 3, j = tid % 3;
    const float* fb = in + IN_FEET;
    const double rx = fb[3 * leg], ry = fb[3 * leg + 1], rz = fb[3 * leg + 2];
    const double sk0 = (j == 0) ? 0.0 : (j == 1 ? -rz : ry);
    const double sk1 = (j == 0) ? rz : (j == 1 ? 0.0 : -rx);
    const double sk2 = (j == 0) ? -ry : (j == 1 ? rx : 0.0);
    Bc[(6 + i) * NU + 3 * leg + j] = f32r(sm.ii[3 * i] * sk0 + sm.ii[3 * i + 1] * sk1 + sm.ii[3 * i + 2] * sk2);
  } else if (tid < 48) {
    const int leg = (tid - 36) / 3, i = (tid - 36) % 3;
    Bc[(9 + i) * NU + 3 * leg + i] = f32r(1.0 / (double)rbs[0]);
  }
  __syncthreads();

  // -------------------------------- 2. exact discretisation (mpc.py:194-208)
  double* const Nm = sm.Nm;
  double* const X = sm.X;
  const double dt = P.dt, hdt2 = 0.5 * P.dt * P.dt;
  if (tid < NX * NX + NX * NU) {
    const int k = tid;
    if (k < NX * NX) {
      const int i = k / NX, j = k % NX;
      double a2 = 0.0;
      for (int l = 0; l < NX; ++l) a2 = fma(Ac[i * NX + l], Ac[l * NX + j], a2);
      Nm[k] = Ac[k] * dt + a2 * hdt2;
    } else {
      const int kk = k - NX * NX, i = kk / NU, j = kk % NU;
      double ab = 0.0;
      for (int l = 0; l < NX; ++l) ab = fma(Ac[i * NX + l], Bc[l * NU + j], ab);
      X[kk] = Bc[kk] * dt + ab * hdt2;
    }
  }
  __syncthreads();
  for (int pw = 1; pw < 3; ++pw) {
    if (tid < NX * NU + NX) {
      const int k = tid;
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
    __syncthreads();
  }

  STAMP(1);

  // -------------------------------------- 3. condensed cost (mpc.py:211-235)
  if (tid < N * NX) {
    const int t = tid / NX, s = tid % NX;
    const double kk = (double)(t + 1);
    sm.e[tid] = sm.x0[s] + kk * sm.y1[s] + 0.5 * kk * (kk - 1.0) * sm.y2[s] - (double)in[IN_XREF + tid];
  }
  __syncthreads();
  for (int k = tid; k < 3 * N * NU; k += LT) {
    const int p = k / (N * NU), rem = k % (N * NU), t = rem / NU, c = rem % NU;
    double a = 0.0;
    for (int s = 0; s < NX; ++s) a = fma(X[p * NX * NU + s * NU + c], P.q[s] * sm.e[t * NX + s], a);
    sm.zp[k] = a;
  }
  // Y = Xc^T diag(Q) Xc on the f64 MFMA, one upper tile pair per wave (waves 0-5)
  if (wave < 6) {
    const int I = wave < 3 ? 0 : (wave < 5 ? 1 : 2);
    const int J = wave < 3 ? wave : (wave < 5 ? wave - 2 : 2);
    const int li = lane & 15, lk = lane >> 4;
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
        sm.Y[(3 * p + q) * NU * NU + c * NU + c2] = acc[rg];
        sm.Y[(3 * q + p) * NU * NU + c2 * NU + c] = acc[rg];
      }
    }
  }
  const int nT = N * (N + 1) / 2;
  for (int k = tid - 384; k >= 0 && k < 9 * N; k += LT - 384) {   // T_pq(d, m) = sum_{s<m} c_p(s+d) c_q(s)  (waves 6-7)
    const int pq = k / N, d = k % N;
    const int p = pq / 3, q = pq % 3;
    double acc = 0.0;
    for (int mm = 1; mm <= N - d; ++mm) {
      acc += cpoly(p, mm - 1 + d) * cpoly(q, mm - 1);
      sm.T[pq * nT + tidx(N, d, mm)] = acc;
    }
  }
  __syncthreads();
  {
    double gl = 0.0;   // g[a] = 2 sum_p sum_{t >= j_a} c_p(t - j_a) zp[p][t][c_a]
    if (tid < n) {
      const int sf = tid / 3;
      const int ja = sm.foot_t[sf], ca = 3 * sm.foot_leg[sf] + tid % 3;
      for (int t = ja; t < N; ++t) {
        const int k = t - ja;
        gl += sm.zp[t * NU + ca] + (double)k * sm.zp[(N + t) * NU + ca] +
              0.5 * (double)k * (double)(k - 1) * sm.zp[(2 * N + t) * NU + ca];
      }
      gl *= 2.0;
    }
    if (tid < NL) sm.gv[tid] = gl;
  }

  __syncthreads();
  STAMP(2);
  // H tile (rows 4tr.., cols 8tc..) into registers; identity padding beyond n
  double W[4][8];
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
    for (int r = 0; r < 4; ++r)
#pragma unroll
      for (int c = 0; c < 8; ++c) W[r][c] = 0.0;
#pragma unroll 1
    for (int r = 0; r < 4; ++r) {
      const int row = 4 * tr + r;
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
          acc = fma(sm.T[(le ? pq : q * 3 + p) * nT + ti], sm.Y[pq * NU * NU + ca * NU + cc[c]], acc);
        }
        const double hv = 2.0 * acc + (row == col ? r2 : 0.0);
        h[c] = (rowv && col < n) ? hv : (row == col ? 1.0 : 0.0);
      });
      static_for<4>([&](auto Rr) {
        constexpr int rr = decltype(Rr)::value;
#pragma unroll
        for (int c = 0; c < 8; ++c) W[rr][c] = (rr == r) ? h[c] : W[rr][c];
      });
    }
  }

  STAMP(3);
  // ------------------------------------------------ 4. W = H^-1 (symmetric sweep)
  lsweep_all(W, sm, tr, tc, n, Ug ? (unsigned long long*)(Ug + (size_t)b * N * 12) + 8 : nullptr);
#pragma unroll
  for (int r = 0; r < 4; ++r)
#pragma unroll
    for (int c = 0; c < 8; ++c) W[r][c] = -W[r][c];
  STAMP(4);

  // constraint lane tid (row c = tid), variable lane tid, slot lane tid
  const bool cok = tid < m;
  const int vf = tid / 3, vax = tid % 3;
  const bool vok = tid < n;
  const bool sok = tid < NL;
  int fslot[6];
#pragma unroll
  for (int rr = 0; rr < 6; ++rr) fslot[rr] = -1;
  int sl_c = 0;
  auto cdot = [&](const double* v, int c, bool bound) -> double {   // a_c . v(foot c) (+ bound term)
    const int f = c / 6, rr = c % 6;
    double d = sm.rows[rr][0] * v[3 * f] + sm.rows[rr][1] * v[3 * f + 1] + sm.rows[rr][2] * v[3 * f + 2];
    if (bound && rr == 5) d += sm.ub[f];
    return d;
  };
  const int wr = lrow(tr, lane);
  const bool wrt = lwriter(lane);

  // unconstrained minimiser x = -W g ; constraint values s = A x - b
  if (sok) sm.vb[pv(tid)] = sm.gv[tid];
  __syncthreads();
  {
    const double y = ltile_matvec(W, sm.vb, tc, lane);
    if (wrt) sm.zv[wr] = -y;
  }
  __syncthreads();
  double s = cok ? cdot(sm.zv, tid, true) : INFINITY;

  // ------------------------- 5. Goldfarb-Idnani dual active set (range space)
  double Mi[4][8];
#pragma unroll
  for (int r = 0; r < 4; ++r)
#pragma unroll
    for (int c = 0; c < 8; ++c) Mi[r][c] = 0.0;
  double u = 0.0;
  unsigned long long occ0 = 0, occ1 = 0;   // occupied slots 0-63, 64-127 (uniform)
  const int max_iter = P.max_iter > 0 ? P.max_iter : 8 * NL + 64;
  const double tol = 1e-9;
  int it = 0;
  int status = MPCQP_STATUS_OK;
  int rbuf = 0;
  while (true) {
    double bv;
    const int p = lwg_argmin(s, tid, sm, wave, lane, rbuf, bv);   // most violated row
    if (!(bv < -tol)) break;
    const int fp = p / 6, rp = p % 6;
    const double ap_l = (vok && vf == fp) ? sm.rows[rp][vax] : 0.0;
    if (sok) sm.vb[pv(tid)] = ap_l;
    __syncthreads();
    {
      const double y = ltile_matvec(W, sm.vb, tc, lane);   // w = W a_p
      if (wrt) sm.wv[wr] = y;
    }
    __syncthreads();
    const double apw = cdot(sm.wv, p, false);
    double up = 0.0;
    bool added = false;
    while (!added) {
      if (++it > max_iter) {
        status = MPCQP_STATUS_MAX_ITER;
        break;
      }
      const bool mine = sok && (((tid < 64 ? occ0 : occ1) >> (tid & 63)) & 1ull);
      if (sok) sm.rv[pv(tid)] = mine ? cdot(sm.wv, sl_c, false) : 0.0;
      __syncthreads();
      {
        const double y = ltile_matvec(Mi, sm.rv, tc, lane);   // r = Minv mp
        if (wrt) sm.rr[pv(wr)] = y;
      }
      __syncthreads();
      const double r_s = sok ? sm.rr[pv(tid)] : 0.0;
      double vl = ap_l;
#pragma unroll
      for (int rr = 0; rr < 6; ++rr)
        if (fslot[rr] >= 0) vl -= sm.rr[pv(fslot[rr])] * sm.rows[rr][vax];
      if (sok) sm.vb[pv(tid)] = vok ? vl : 0.0;
      __syncthreads();
      {
        const double y = ltile_matvec(W, sm.vb, tc, lane);   // z = W v
        if (wrt) sm.zv[wr] = y;
      }
      __syncthreads();
      const double zs = cok ? cdot(sm.zv, tid, false) : 0.0;
      if (tid == p) {
        sm.bc_zs = zs;
        sm.bc_s = s;
      }
      double t1;
      const int l = lwg_argmin((mine && r_s > 0.0) ? u / r_s : INFINITY, tid, sm, wave, lane, rbuf, t1);
      const double zsp = sm.bc_zs, sp = sm.bc_s;
      double t2 = INFINITY;
      if (zsp > 1e-12 * apw) t2 = -sp / zsp;
      const bool add = t2 <= t1;
      const double tstep = add ? t2 : t1;
      if (!(tstep < INFINITY)) {
        status = MPCQP_STATUS_INFEASIBLE;
        break;
      }
      if (mine) u -= tstep * r_s;
      if (cok) s += tstep * zs;
      up += tstep;
      if (add) {
        // (M_AA)^-1 += e e^T / sigma with e = r - e_q (borders slot q)
        const int q = occ0 != ~0ull ? __builtin_ctzll(~occ0) : 64 + __builtin_ctzll(~occ1);
        const double is = 1.0 / zsp;
        double er[4], ec[8];
        ld4(er, sm.rr, tr);
        ld8(ec, sm.rr, tc);
        MPCQP_FENCE();
#pragma unroll
        for (int r = 0; r < 4; ++r) er[r] = (4 * tr + r == q) ? -is : er[r] * is;
#pragma unroll
        for (int c = 0; c < 8; ++c) ec[c] = (8 * tc + c == q) ? -1.0 : ec[c];
#pragma unroll
        for (int r = 0; r < 4; ++r)
#pragma unroll
          for (int c = 0; c < 8; ++c) Mi[r][c] = fma(er[r], ec[c], Mi[r][c]);
        if (tid == q) {
          u = up;
          sl_c = p;
        }
        if (tid == p) s = 0.0;
        if (vok && vf == fp) {
#pragma unroll
          for (int rr = 0; rr < 6; ++rr)
            if (rr == rp) fslot[rr] = q;
        }
        if (q < 64) occ0 |= 1ull << q;
        else occ1 |= 1ull << (q - 64);
        added = true;
      } else {
        // drop slot l: Minv -= Minv[:,l] Minv[l,:] / Minv[l][l]; row/col l -> 0
        const int lt = l >> 3, lc = l & 7;
        if (tc == lt) {
          double col[4];
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            double v = 0.0;
            static_for<8>([&](auto C) {
              constexpr int c = decltype(C)::value;
              v = (c == lc) ? Mi[r][c] : v;
            });
            col[r] = v;
          }
          d2* pp = reinterpret_cast<d2*>(sm.cv + pv(4 * tr));
          pp[0] = d2{col[0], col[1]};
          pp[1] = d2{col[2], col[3]};
        }
        __syncthreads();
        double cr[4], ccv[8];
        ld4(cr, sm.cv, tr);
        ld8(ccv, sm.cv, tc);
        const double cll = sm.cv[pv(l)];
        MPCQP_FENCE();
        const double f = -1.0 / cll;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const bool rl = (4 * tr + r == l);
#pragma unroll
          for (int c = 0; c < 8; ++c) {
            const double nv = fma(cr[r] * f, ccv[c], Mi[r][c]);
            Mi[r][c] = (rl || 8 * tc + c == l) ? 0.0 : nv;
          }
        }
        if (vok) {
#pragma unroll
          for (int rr = 0; rr < 6; ++rr)
            if (fslot[rr] == l) fslot[rr] = -1;
        }
        if (tid == l) u = 0.0;
        if (l < 64) occ0 &= ~(1ull << l);
        else occ1 &= ~(1ull << (l - 64));
      }
    }
    if (status != MPCQP_STATUS_OK) break;
  }
  __syncthreads();
  STAMP(5);

  // ------------------------------- 6. refinement, final x, KKT verification
  for (int pass = 0; pass < 2; ++pass) {
    const bool mine = sok && (((tid < 64 ? occ0 : occ1) >> (tid & 63)) & 1ull);
    if (sok) sm.rv[pv(tid)] = mine ? u : 0.0;
    __syncthreads();
    double vl = -sm.gv[tid < NL ? tid : 0];
#pragma unroll
    for (int rr = 0; rr < 6; ++rr)
      if (fslot[rr] >= 0) vl += sm.rv[pv(fslot[rr])] * sm.rows[rr][vax];
    __syncthreads();
    if (sok) sm.vb[pv(tid)] = vok ? vl : 0.0;
    __syncthreads();
    {
      const double y = ltile_matvec(W, sm.vb, tc, lane);
      if (wrt) sm.zv[wr] = y;
    }
    __syncthreads();
    if (pass == 1) break;
    if (sok) sm.rv[pv(tid)] = mine ? cdot(sm.zv, sl_c, true) : 0.0;
    __syncthreads();
    {
      const double y = ltile_matvec(Mi, sm.rv, tc, lane);
      if (wrt) sm.rr[pv(wr)] = y;
    }
    __syncthreads();
    if (mine) u -= sm.rr[pv(tid)];
    __syncthreads();
  }
  {
    const double v = cok ? cdot(sm.zv, tid, true) : 0.0;
    int bad = cok && (v < -1e-6 || !isfinite(v));
    const bool mine = sok && (((tid < 64 ? occ0 : occ1) >> (tid & 63)) & 1ull);
    if (mine) bad |= (u < -1e-9);
    if (__syncthreads_or(bad) && status == MPCQP_STATUS_OK) status = MPCQP_STATUS_MAX_ITER;
  }
  STAMP(6);

  // ---------------------------------------------------------------- output
#ifdef MPCQP_STAMPS
  if (tid == 0 && Ug) {
    unsigned long long* dst = (unsigned long long*)(Ug + (size_t)b * N * 12);
    for (int i = 0; i < 7; ++i) dst[i] = stamps_[i];
  }
  Ug = nullptr;
#endif
  if (tid < 12) {
    const int sidx = sm.stance_of[tid / 3];
    u0g[(size_t)b * 12 + tid] = sidx >= 0 ? (float)sm.zv[3 * sidx + tid % 3] : 0.f;
  }
  if (Ug) {
    for (int k = tid; k < N * 12; k += LT) {
      const int sidx = sm.stance_of[k / 3];
      Ug[(size_t)b * N * 12 + k] = sidx >= 0 ? (float)sm.zv[3 * sidx + k % 3] : 0.f;
    }
  }
  if (tid == 0) {
    if (statusg) statusg[b] = status;
    if (itersg) itersg[b] = it;
  }
}

// One workgroup per queued robot: the wave kernel filled queue[0] = count,
// queue[4..] = robot indices; the launch has one workgroup per robot of the batch
// and the ones beyond the count exit at once.  The last workgroup to finish resets
// the counters for the next launch (queue[2] counts finished workgroups).
__global__ __launch_bounds__(LT) void mpcqp_kernel_large(
    KParams P, const float* __restrict__ x0g, const float* __restrict__ xrefg,
    const float* __restrict__ contactg, const float* __restrict__ feetg, const float* __restrict__ robotg,
    float* __restrict__ u0g, float* __restrict__ Ug, int* __restrict__ statusg, int* __restrict__ itersg,
    int* __restrict__ queue) {
  __shared__ LShared sm;
  const int tid = threadIdx.x;
  const int k = blockIdx.x;
  const int cnt = uni(__hip_atomic_load(&queue[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
  if (k < cnt) {
    const int b = uni(queue[4 + k]);
    lsolve_robot(P, b, sm, x0g, xrefg, contactg, feetg, robotg, u0g, Ug, statusg, itersg);
  }
  if (tid == 0) {
    if (atomicAdd(&queue[2], 1) == (int)gridDim.x - 1) {
      atomicExch(&queue[0], 0);
      atomicExch(&queue[2], 0);
    }
  }
}
