// Microbenchmark (diagnostic only): f64 FMA issue cost by operand sources.  The dense
// classes' rank updates W[r][c] += a[r] z[c] read three VGPR pairs per FMA; fma_bench.hip
// measured FMAs with one VGPR operand.  Cycles per wave FMA instruction (s_memtime, median
// over waves) at 1 and 2 waves per SIMD.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <algorithm>
#include <vector>

template <int MODE>
__global__ __launch_bounds__(512) void k(double* out, int iters, unsigned long long* cyc, double as, double bs) {
  const int t = threadIdx.x;
  double W[4][8], a[4], z[8];
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    a[r] = 1e-3 * (t + r);
#pragma unroll
    for (int c = 0; c < 8; ++c) W[r][c] = t + r + c;
  }
#pragma unroll
  for (int c = 0; c < 8; ++c) z[c] = 1e-3 * (t - c);
  const double av = 1e-3 * t;
  __syncthreads();
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
      for (int c = 0; c < 8; ++c) {
        if (MODE == 0) W[r][c] = __builtin_fma(W[r][c], as, bs);            // 1 VGPR pair
        if (MODE == 1) W[r][c] = __builtin_fma(z[c], as, W[r][c]);          // 2 VGPR pairs + SGPR
        if (MODE == 2) W[r][c] = __builtin_fma(z[c], av, W[r][c]);          // 3 VGPR pairs (one shared)
        if (MODE == 3) W[r][c] = __builtin_fma(a[r], z[c], W[r][c]);        // rank-1 tile (the sweep)
        if (MODE == 4) W[r][c] = __builtin_fma(a[r], z[c], __builtin_fma(a[3 - r], z[7 - c], W[r][c]));  // rank-2
      }
    __builtin_amdgcn_sched_barrier(0);
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  double s = 0;
#pragma unroll
  for (int r = 0; r < 4; ++r)
#pragma unroll
    for (int c = 0; c < 8; ++c) s += W[r][c];
  out[blockIdx.x * blockDim.x + t] = s;
  if (t % 64 == 0) cyc[blockIdx.x * 8 + t / 64] = t1 - t0;
}

template <int MODE>
static void run(const char* name, int waves, int blocks) {
  double* out;
  unsigned long long* cyc;
  hipMalloc(&out, sizeof(double) * blocks * 512);
  hipMalloc(&cyc, sizeof(unsigned long long) * blocks * 8);
  hipMemset(cyc, 0, sizeof(unsigned long long) * blocks * 8);
  const int iters = 2000;
  for (int rep = 0; rep < 2; ++rep)
    hipLaunchKernelGGL(k<MODE>, dim3(blocks), dim3(64 * waves), 0, 0, out, iters, cyc, 0.999, 1e-3);
  hipDeviceSynchronize();
  std::vector<unsigned long long> h(blocks * 8);
  hipMemcpy(h.data(), cyc, sizeof(unsigned long long) * blocks * 8, hipMemcpyDeviceToHost);
  std::vector<unsigned long long> v;
  for (auto x : h)
    if (x) v.push_back(x);
  std::sort(v.begin(), v.end());
  const double nf = MODE == 4 ? 64.0 : 32.0;
  printf("%-34s waves/SIMD %d: %6.2f cycles per wave FMA\n", name, waves / 4, (double)v[v.size() / 2] / (iters * nf));
  hipFree(out);
  hipFree(cyc);
}

int main() {
  for (int w : {4, 8}) {   // one block per CU (256 blocks): 4 waves = 1 per SIMD, 8 = 2
    run<0>("fma(W, s, s)      1 VGPR", w, 256);
    run<1>("fma(z, s, W)      2 VGPR", w, 256);
    run<2>("fma(z, v, W)      3 VGPR", w, 256);
    run<3>("fma(a[r], z[c], W) rank-1 tile", w, 256);
    run<4>("rank-2 tile", w, 256);
  }
  return 0;
}
