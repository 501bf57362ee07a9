// Diagnostic: the cost of the class-64 combo dispatch (a uniform 8-way switch on the
// foot-step's register column, two of them per pass) against straight-line code.
//   V0: switch(c) over 8 compile-time column combos (the kernel's colcombo dispatch)
//   V1: the same arithmetic at a fixed column (no branches)
//   V2: a branch-free select of the coefficient per column (8 columns x 4 rows)
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <algorithm>
#include <vector>

template <int C0>
__device__ __forceinline__ void combo(const double (&W)[4][8], double a0, double a1, double a2, double (&z)[4]) {
  constexpr int c0 = C0 % 8, c1 = (C0 + 1) % 8, c2 = (C0 + 2) % 8;
  for (int r = 0; r < 4; ++r) z[r] = fma(a2, W[r][c2], fma(a1, W[r][c1], a0 * W[r][c0]));
}

template <int V>
__global__ __launch_bounds__(64) void bench(int cmode, int iters, double* out, unsigned long long* cyc) {
  const int lane = threadIdx.x;
  double W[4][8];
  for (int r = 0; r < 4; ++r)
    for (int c = 0; c < 8; ++c) W[r][c] = 1.0 + 0.01 * (r * 8 + c + lane);
  double acc[4] = {0, 0, 0, 0};
  unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < iters; ++it) {
    const int cA = __builtin_amdgcn_readfirstlane(cmode ? 3 : ((it * 5 + (it >> 2)) & 7));
    const double a0 = 0.5 + it * 1e-6, a1 = 0.25, a2 = 0.125;
    double z[4];
    if constexpr (V == 0) {
      switch (cA) {
        case 0: combo<0>(W, a0, a1, a2, z); break;
        case 1: combo<1>(W, a0, a1, a2, z); break;
        case 2: combo<2>(W, a0, a1, a2, z); break;
        case 3: combo<3>(W, a0, a1, a2, z); break;
        case 4: combo<4>(W, a0, a1, a2, z); break;
        case 5: combo<5>(W, a0, a1, a2, z); break;
        case 6: combo<6>(W, a0, a1, a2, z); break;
        default: combo<7>(W, a0, a1, a2, z); break;
      }
    } else if constexpr (V == 1) {
      combo<3>(W, a0 + cA, a1, a2, z);
    } else if constexpr (V == 3) {
      // uniform runtime column index into register vectors (VGPR index mode)
      typedef double d8 __attribute__((ext_vector_type(8)));
      for (int r = 0; r < 4; ++r) {
        d8 w;
        for (int c = 0; c < 8; ++c) w[c] = W[r][c];
        z[r] = fma(a2, w[(cA + 2) & 7], fma(a1, w[(cA + 1) & 7], a0 * w[cA]));
      }
    } else {
      double al[8];
      for (int c = 0; c < 8; ++c) {
        const int d = c - cA;
        al[c] = d == 0 ? a0 : d == 1 ? a1 : d == 2 ? a2 : 0.0;
      }
      for (int r = 0; r < 4; ++r) {
        double s = 0.0;
        for (int c = 0; c < 8; ++c) s = fma(al[c], W[r][c], s);
        z[r] = s;
      }
    }
    for (int r = 0; r < 4; ++r) {
      acc[r] += z[r];
      W[r][r] += 1e-9 * z[r];   // keep W live and changing
    }
  }
  unsigned long long t1 = __builtin_amdgcn_s_memtime();
  out[blockIdx.x * 64 + lane] = acc[0] + acc[1] + acc[2] + acc[3];
  if (lane == 0) cyc[blockIdx.x] = t1 - t0;
}

template <int V>
void run(int cmode, const char* name) {
  const int B = 256, iters = 4096;
  double* out;
  unsigned long long* cyc;
  (void)hipMalloc(&out, B * 64 * sizeof(double));
  (void)hipMalloc(&cyc, B * sizeof(unsigned long long));
  for (int rep = 0; rep < 3; ++rep) hipLaunchKernelGGL(bench<V>, dim3(B), dim3(64), 0, 0, cmode, iters, out, cyc);
  (void)hipDeviceSynchronize();
  std::vector<unsigned long long> h(B);
  (void)hipMemcpy(h.data(), cyc, B * sizeof(unsigned long long), hipMemcpyDeviceToHost);
  std::sort(h.begin(), h.end());
  printf("%-40s %6.1f cycles per combo (median over %d waves)\n", name, (double)h[B / 2] / iters, B);
  (void)hipFree(out);
  (void)hipFree(cyc);
}

int main() {
  run<0>(0, "V0 8-way switch (kernel dispatch)");
  run<1>(0, "V1 fixed column, no branch");
  run<2>(0, "V2 branch-free 8-column selects");
  run<3>(0, "V3 uniform index into register vector");
  run<0>(1, "V0 switch, constant column");
  return 0;
}
