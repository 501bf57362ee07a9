// Diagnostic: the large-class sweep in isolation (8 waves, 4x8 tiles), s_memtime-timed,
// plus stripped variants to locate the cost.
#include "../../pympc-quadruped_amd/csrc/mpcqp.hip"
#include <stdio.h>

namespace {
template <int KC, int V>
__device__ __forceinline__ void piv(double (&W)[4][8], LShared& sm, int tr, int tc, int KT, int n) {
  const int K = 8 * KT + KC;
  if (K < n) {
    constexpr int KRR = KC & 3;
    const int KR = 2 * KT + (KC >> 2);
    double* const zc = sm.zc[KC & 1];
    if (V != 3 && tc == KT) {
      d2* p = reinterpret_cast<d2*>(zc + pv(4 * tr));
      p[0] = d2{W[0][KC], W[1][KC]};
      p[1] = d2{W[2][KC], W[3][KC]};
    }
    __syncthreads();
    double zr[8], zi[4];
    if (V == 3) {
      for (int c = 0; c < 8; ++c) zr[c] = W[0][c] * 1e-3;
      for (int r = 0; r < 4; ++r) zi[r] = W[r][1] * 1e-3;
    } else {
      ld8(zr, zc, tc);
      ld4(zi, zc, tr);
    }
    const double d = V == 3 ? 2.0 + W[0][0] : zc[pv(K)];
    MPCQP_FENCE();
    const double inv = V == 1 ? d : 1.0 / d;
    double beta[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) beta[r] = -zi[r] * inv;
    if (tr == KR) beta[KRR] = inv - 1.0;
    if (V != 2) {
#pragma unroll
      for (int r = 0; r < 4; ++r)
#pragma unroll
        for (int c = 0; c < 8; ++c) W[r][c] = fma(beta[r], zr[c], W[r][c]);
    } else {
      W[0][0] += beta[0] * zr[0] + beta[1] * zr[1] + beta[2] + beta[3] * zr[7];
    }
    if (tc == KT) {
#pragma unroll
      for (int r = 0; r < 4; ++r) W[r][KC] = zi[r] * inv;
      if (tr == KR) W[KRR][KC] = -inv;
    }
  }
}

template <int V>
__global__ __launch_bounds__(LT) void sweep_v(double* out, int n, unsigned long long* cyc) {
  __shared__ LShared sm;
  const int tid = threadIdx.x, tr = tid >> 4, tc = tid & 15;
  double W[4][8];
#pragma unroll
  for (int r = 0; r < 4; ++r)
#pragma unroll
    for (int c = 0; c < 8; ++c) {
      const int row = 4 * tr + r, col = 8 * tc + c;
      W[r][c] = row == col ? 4.0 + 0.01 * row : 1.0 / (1.0 + row + col);
    }
  __syncthreads();
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  if (V == 0) {
    lsweep_all(W, sm, tr, tc, n, nullptr);
  } else {
#pragma unroll 1
    for (int KT = 0; 8 * KT < n; ++KT) {
      static_for<8>([&](auto C) { piv<decltype(C)::value, V>(W, sm, tr, tc, KT, n); });
    }
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  double s = 0;
#pragma unroll
  for (int r = 0; r < 4; ++r)
#pragma unroll
    for (int c = 0; c < 8; ++c) s += W[r][c];
  out[blockIdx.x * LT + tid] = s;
  if (tid == 0) cyc[blockIdx.x] = t1 - t0;
}
}  // namespace

int main() {
  double* d; unsigned long long* c;
  hipMalloc(&d, 256 * LT * 8); hipMalloc(&c, 256 * 8);
  unsigned long long h[1];
  const char* names[] = {"full", "no divide", "no rank-1 FMAs", "no LDS traffic (barrier only)", "full, 4 waves"};
  auto run = [&](int v, void (*k)(double*, int, unsigned long long*), int threads) {
    hipLaunchKernelGGL(k, dim3(256), dim3(threads), 0, 0, d, 96, c);
    hipLaunchKernelGGL(k, dim3(256), dim3(threads), 0, 0, d, 96, c);
    hipDeviceSynchronize();
    hipMemcpy(h, c, 8, hipMemcpyDeviceToHost);
    printf("sweep n=96 %-32s: %.0f cycles per pivot\n", names[v], h[0] / 96.0);
  };
  run(0, sweep_v<0>, LT);
  run(1, sweep_v<1>, LT);
  run(2, sweep_v<2>, LT);
  run(3, sweep_v<3>, LT);
  return 0;
}
