// mpcqp_sweep_mfma.h -- class 64's H^-1 sweep on the f64 matrix cores (included by
// mpcqp.hip inside its anonymous namespace, before mpcqp_solve.h).
//
// The symmetric sweep of mpcqp_solve.h, blocked by 4 pivots K = {4k .. 4k+3}.  Each
// single-pivot sweep there is one rank-1 update beta zeta^T of the whole matrix plus
// -2 on its pivot's diagonal entry, and the four rank-1 vectors of a block depend only
// on the block's 4 panel columns; so the panel rows run the four pivots' recurrence
// (one lane per row; the same arithmetic as four single pivots -- an explicit inverse
// of the 4 x 4 pivot block instead loses ~2 digits on these Hessians and costs the
// active set extra iterations), publish their rank-1 entries through LDS, and the
// four rank-1 terms become ONE rank-4
// update W += A B, A = [beta_0 .. beta_3], B = [zeta_0 .. zeta_3]^T.  A rank-4 update
// of a 16 x 16 block is one
// v_mfma_f64_16x16x4_f64 (C/D: lane l, register i holds row (l >> 4) + 4 i, column
// l & 15; A: lane l holds A[l & 15][l >> 4]; B: lane l holds B[l >> 4][l & 15] --
// tools/ubench/mfma_f64_check.hip checks these maps with exact data), so the sweep's
// FMAs leave the VALU for the matrix cores: 8 MFMAs per wave per 4 pivots instead of
// 128 v_fma_f64, and two barriers per 4 pivots instead of 4.  The four robots of a CU
// sweep at the same time; their VALU work (pivot blocks, coefficients) then overlaps
// the other robots' MFMAs.
//
// Layout: the sweep runs on an MFMA-layout copy of the matrix (wave w holds rows
// 32 w .. 32 w + 31 as 2 x 4 blocks of 16 x 16 = 8 d4 registers per lane); the
// solver's 4 x 8 register tiles are converted in and out through the H copy's LDS
// (free during the sweep: H itself stays in the caller's registers and is stored as
// the drop path's copy afterwards).

// d4: the ext_vector_type(4) double typedef of mpcqp.hip

// On entry W holds H in the 4 x 8 tile layout (lane (tr, tc) = (tid / 8, tid % 8):
// rows 4 tr .. 4 tr + 3, columns 8 tc .. 8 tc + 7).  On exit Wout holds the sweep
// result -H^-1 in the same layout and `buf` (>= 64 * 64 doubles of LDS) is free.
// n <= 64 real variables; indices >= n are the identity padding (decoupled).
__device__ __forceinline__ void sweep_mfma64(const double (&W)[4][8], double (&Wout)[4][8], double* __restrict__ buf,
                                             int n, int tid) {
  constexpr int NT = 128;
  const int lane = tid & 63, wave = tid >> 6;
  const int tr = tid >> 3, tc = tid & 7;
  const int lr = lane >> 4, lc = lane & 15;
  // ---- 4 x 8 tiles -> row-major image -> MFMA layout
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    d2* p = reinterpret_cast<d2*>(buf + (4 * tr + r) * 64 + 8 * tc);
#pragma unroll
    for (int q = 0; q < 4; ++q) p[q] = d2{W[r][2 * q], W[r][2 * q + 1]};
  }
  fsync<NT>();
  d4 M[8];   // block (bi, bj) = M[4 bi + bj]: rows 32 wave + 16 bi + lr + 4 i, column 16 bj + lc
#pragma unroll
  for (int bi = 0; bi < 2; ++bi)
#pragma unroll
    for (int bj = 0; bj < 4; ++bj)
#pragma unroll
      for (int i = 0; i < 4; ++i) M[4 * bi + bj][i] = buf[(32 * wave + 16 * bi + lr + 4 * i) * 64 + 16 * bj + lc];
  fsync<NT>();   // the image is dead: buf holds the pivot columns from here on
  // ---- blocked sweep: BJ = the pivots' 16-column group, SUB = their 4-column block
  static_for<4>([&](auto BJc) {
    constexpr int BJ = decltype(BJc)::value;
    static_for<4>([&](auto SUBc) {
      constexpr int SUB = decltype(SUBc)::value;
      constexpr int K = 16 * BJ + 4 * SUB;
      if (K < n) {
        double* const z = buf + ((K >> 2) & 1) * 256;   // Z row-major [64][4], double-buffered
        // publish Z: the lanes holding columns K .. K+3 (block column BJ)
        const int kk = lc - 4 * SUB;
        if (kk >= 0 && kk < 4) {
#pragma unroll
          for (int bi = 0; bi < 2; ++bi)
#pragma unroll
            for (int i = 0; i < 4; ++i) z[(32 * wave + 16 * bi + lr + 4 * i) * 4 + kk] = M[4 * bi + BJ][i];
        }
        fsync<NT>();
        // The four single-pivot sweeps' rank-1 vectors, exactly as mpcqp_solve.h forms
        // them one pivot at a time: sweep k adds beta_k zeta_k^T with
        //   beta_k[i] = -w_i / d_k  (pivot row K+k: 1/d_k - 1),
        //   zeta_k[j] = w_j         (pivot column K+k: d_k - 1),
        // w = column K+k after sweeps 0..k-1.  Every panel row runs that recurrence on
        // its 4 panel entries; the pivot rows' part (d_k, the zeta_k entries of columns
        // K..K+3) is uniform.  The four rank-1 terms then go into one rank-4 MFMA.
        double P4[4][4];
#pragma unroll
        for (int a = 0; a < 4; ++a) {
          const d2* p = reinterpret_cast<const d2*>(z + (K + a) * 4);
          const d2 u = p[0], v = p[1];
          P4[a][0] = u[0];
          P4[a][1] = u[1];
          P4[a][2] = v[0];
          P4[a][3] = v[1];
        }
        double dd[4], inv[4], zk[4][4];   // zk[a][k] = zeta_k at column K + a
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          dd[k] = P4[k][k];
          inv[k] = rcp_nr(dd[k]);
          double be[4];
#pragma unroll
          for (int a = 0; a < 4; ++a) {
            be[a] = a == k ? inv[k] - 1.0 : -P4[a][k] * inv[k];
            zk[a][k] = a == k ? dd[k] - 1.0 : P4[a][k];
          }
#pragma unroll
          for (int a = 0; a < 4; ++a)
#pragma unroll
            for (int k2 = k + 1; k2 < 4; ++k2) P4[a][k2] = fma(be[a], zk[k2][k], P4[a][k2]);
        }
        // panel row r = 32 wave + lane (lanes < 32): its 4 entries through the four
        // pivots' recurrence -> beta_k[r], zeta_k[r], published for every lane's operands
        double* const ab = buf + 512;   // [64][8]: beta_0..3, zeta_0..3 of each panel row
        if (lane < 32) {
          const int r = 32 * wave + lane;
          const d2* p = reinterpret_cast<const d2*>(z + r * 4);
          const d2 u = p[0], v = p[1];
          double q[4] = {u[0], u[1], v[0], v[1]};
          double be[4], ze[4];
#pragma unroll
          for (int k = 0; k < 4; ++k) {
            const bool piv = r == K + k;
            be[k] = piv ? inv[k] - 1.0 : -q[k] * inv[k];
            ze[k] = piv ? dd[k] - 1.0 : q[k];
#pragma unroll
            for (int k2 = k + 1; k2 < 4; ++k2) q[k2] = fma(be[k], zk[k2][k], q[k2]);
          }
          d2* o = reinterpret_cast<d2*>(ab + r * 8);
          o[0] = d2{be[0], be[1]};
          o[1] = d2{be[2], be[3]};
          o[2] = d2{ze[0], ze[1]};
          o[3] = d2{ze[2], ze[3]};
        }
        fsync<NT>();
        // A operands: row 32 wave + 16 bi + lc, pivot lr; B operands: column 16 bj + lc
        double A[2], Bv[4];
#pragma unroll
        for (int bi = 0; bi < 2; ++bi) A[bi] = ab[(32 * wave + 16 * bi + lc) * 8 + lr];
#pragma unroll
        for (int bj = 0; bj < 4; ++bj) Bv[bj] = ab[(16 * bj + lc) * 8 + 4 + lr];
#pragma unroll
        for (int bi = 0; bi < 2; ++bi)
#pragma unroll
          for (int bj = 0; bj < 4; ++bj)
            M[4 * bi + bj] = __builtin_amdgcn_mfma_f64_16x16x4f64(A[bi], Bv[bj], M[4 * bi + bj], 0, 0, 0);
        // pivot diagonal: 2 - D^-1 -> -D^-1
#pragma unroll
        for (int bi = 0; bi < 2; ++bi)
          if (2 * wave + bi == BJ) M[4 * bi + BJ][SUB] += (lc == 4 * SUB + lr) ? -2.0 : 0.0;
      }
    });
  });
  // ---- MFMA layout -> row-major image -> 4 x 8 tiles
  fsync<NT>();   // every lane is done reading the last pivot block
#pragma unroll
  for (int bi = 0; bi < 2; ++bi)
#pragma unroll
    for (int bj = 0; bj < 4; ++bj)
#pragma unroll
      for (int i = 0; i < 4; ++i) buf[(32 * wave + 16 * bi + lr + 4 * i) * 64 + 16 * bj + lc] = M[4 * bi + bj][i];
  fsync<NT>();
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const d2* p = reinterpret_cast<const d2*>(buf + (4 * tr + r) * 64 + 8 * tc);
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const d2 v = p[q];
      Wout[r][2 * q] = v[0];
      Wout[r][2 * q + 1] = v[1];
    }
  }
  fsync<NT>();   // buf is free again (the caller stores H there)
}
