// Diagnostic: class 64's two-wave H^-1 sweep (4 x 8 full tiles, one barrier per pivot, the
// kernel's code) against a two-wave sweep of the 120 lower 4 x 4 tiles (n <= 60, half the
// FMAs per lane), s_memtime-timed per workgroup, four workgroups per CU as in config 2.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <algorithm>
#include <vector>

typedef double d2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ double rcp_nr(double d) {
  double y = __builtin_amdgcn_rcp(d);
  double e = fma(-d, y, 1.0);
  y = fma(y, e, y);
  e = fma(-d, y, 1.0);
  return fma(y, e, y);
}
template <typename F, int... Is>
__device__ __forceinline__ void sfor(F&& f, std::integer_sequence<int, Is...>) {
  (f(std::integral_constant<int, Is>{}), ...);
}
__device__ __forceinline__ double hval(int i, int j, int n, int b) {
  return (i < n && j < n) ? (i == j ? n + 1.0 : 1.0 / (1.0 + (i > j ? i - j : j - i))) + 1e-3 * b : (i == j ? 1.0 : 0.0);
}

// V = 0: full 4 x 8 tiles (tr, tc) = (tid / 8, tid % 8), the kernel's single-pivot pass
// V = 1: lower 4 x 4 tiles, lane L = br (br + 1) / 2 + bc (L < 120)
template <int V>
__global__ __launch_bounds__(128) __attribute__((amdgpu_waves_per_eu(2, 2))) void sweep(int n, double* out,
                                                                                     unsigned long long* cyc) {
  __shared__ __attribute__((aligned(16))) double zc[2][64];
  const int tid = threadIdx.x;
  if (tid < 64) { zc[0][tid] = 0.0; zc[1][tid] = 0.0; }
  __syncthreads();
  double acc = 0.0;
  unsigned long long t0 = __builtin_amdgcn_s_memtime();
  if constexpr (V == 0) {
    const int tr = tid >> 3, tc = tid & 7;
    double W[4][8];
    for (int r = 0; r < 4; ++r)
      for (int c = 0; c < 8; ++c) W[r][c] = hval(4 * tr + r, 8 * tc + c, n, blockIdx.x);
#pragma unroll 1
    for (int KT = 0; 8 * KT < n; ++KT) {
      sfor([&](auto KCc) {
        constexpr int KC = decltype(KCc)::value;
        const int K = 8 * KT + KC;
        const int KR = 2 * KT + (KC >> 2);
        if (K < n) {
          double* const z = zc[KC & 1];
          if (tc == KT) {
            d2* p = reinterpret_cast<d2*>(z + 4 * tr);
            p[0] = d2{W[0][KC], W[1][KC]};
            p[1] = d2{W[2][KC], W[3][KC]};
          }
          __syncthreads();
          double zr[8], zi[4];
          const d2* p = reinterpret_cast<const d2*>(z + 8 * tc);
          for (int i = 0; i < 4; ++i) { const d2 x = p[i]; zr[2 * i] = x[0]; zr[2 * i + 1] = x[1]; }
          const d2* q = reinterpret_cast<const d2*>(z + 4 * tr);
          const d2 a = q[0], bb = q[1];
          zi[0] = a[0]; zi[1] = a[1]; zi[2] = bb[0]; zi[3] = bb[1];
          const double dK = z[K];
          const double inv = rcp_nr(dK);
          double beta[4];
          for (int r = 0; r < 4; ++r) beta[r] = -zi[r] * inv;
          if (tr == KR) beta[KC & 3] = inv - 1.0;
          if (tc == KT) zr[KC] = dK - 1.0;
          for (int r = 0; r < 4; ++r)
            for (int c = 0; c < 8; ++c) W[r][c] = fma(beta[r], zr[c], W[r][c]);
          W[KC & 3][KC] += (tc == KT && tr == KR) ? -2.0 : 0.0;
        }
      }, std::make_integer_sequence<int, 8>{});
    }
    for (int r = 0; r < 4; ++r)
      for (int c = 0; c < 8; ++c)
        if (4 * tr + r == 8 * tc + c) acc += W[r][c];
  } else {
    int br = 0;
    for (int bb = 1; bb < 15; ++bb) br = (bb * (bb + 1)) / 2 <= tid ? bb : br;
    const bool live = tid < 120;
    const int bc = live ? tid - (br * (br + 1)) / 2 : 0;
    if (!live) br = 15;   // idle lanes: a row block no pivot touches
    double W[4][4];
    for (int r = 0; r < 4; ++r)
      for (int c = 0; c < 4; ++c) W[r][c] = hval(4 * br + r, 4 * bc + c, n, blockIdx.x);
#pragma unroll 1
    for (int KB = 0; 4 * KB < n; ++KB) {
      sfor([&](auto KIc) {
        constexpr int KI = decltype(KIc)::value;
        const int K = 4 * KB + KI;
        if (K < n) {
          double* const z = zc[KI & 1];
          if (live && br == KB) {   // row K: columns 4 bc .. 4 bc + 3
            d2* p = reinterpret_cast<d2*>(z + 4 * bc);
            p[0] = d2{W[KI][0], W[KI][1]};
            p[1] = d2{W[KI][2], W[KI][3]};
          }
          __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
          if (live && bc == KB) {   // column K: rows 4 br .. 4 br + 3 (after the row stores)
            d2* p = reinterpret_cast<d2*>(z + 4 * br);
            p[0] = d2{W[0][KI], W[1][KI]};
            p[1] = d2{W[2][KI], W[3][KI]};
          }
          __syncthreads();
          double zr[4], zi[4];
          const d2* p = reinterpret_cast<const d2*>(z + 4 * bc);
          const d2 a0 = p[0], a1 = p[1];
          zr[0] = a0[0]; zr[1] = a0[1]; zr[2] = a1[0]; zr[3] = a1[1];
          const d2* q = reinterpret_cast<const d2*>(z + 4 * br);
          const d2 c0 = q[0], c1 = q[1];
          zi[0] = c0[0]; zi[1] = c0[1]; zi[2] = c1[0]; zi[3] = c1[1];
          const double dK = z[K];
          const double inv = rcp_nr(dK);
          double beta[4];
          for (int r = 0; r < 4; ++r) beta[r] = -zi[r] * inv;
          if (br == KB) beta[KI] = inv - 1.0;
          if (bc == KB) zr[KI] = dK - 1.0;
          for (int r = 0; r < 4; ++r)
            for (int c = 0; c < 4; ++c) W[r][c] = fma(beta[r], zr[c], W[r][c]);
          W[KI][KI] += (bc == KB && br == KB) ? -2.0 : 0.0;
        }
      }, std::make_integer_sequence<int, 4>{});
    }
    for (int r = 0; r < 4; ++r)
      for (int c = 0; c < 4; ++c)
        if (live && 4 * br + r == 4 * bc + c) acc += W[r][c];
  }
  unsigned long long t1 = __builtin_amdgcn_s_memtime();
  // trace of the (negated) inverse, summed over the workgroup, for a cross-check
  __shared__ double red[128];
  red[tid] = acc;
  __syncthreads();
  if (tid == 0) {
    double s = 0.0;
    for (int i = 0; i < 128; ++i) s += red[i];
    out[blockIdx.x] = s;
    cyc[blockIdx.x] = t1 - t0;
  }
}

template <int V>
void run(int B, int n, const char* name) {
  double* out;
  unsigned long long* cyc;
  (void)hipMalloc(&out, B * sizeof(double));
  (void)hipMalloc(&cyc, B * sizeof(unsigned long long));
  for (int rep = 0; rep < 5; ++rep) hipLaunchKernelGGL(sweep<V>, dim3(B), dim3(128), 0, 0, n, out, cyc);
  (void)hipDeviceSynchronize();
  std::vector<unsigned long long> h(B);
  std::vector<double> o(B);
  (void)hipMemcpy(h.data(), cyc, B * sizeof(unsigned long long), hipMemcpyDeviceToHost);
  (void)hipMemcpy(o.data(), out, B * sizeof(double), hipMemcpyDeviceToHost);
  std::sort(h.begin(), h.end());
  printf("%-34s B=%5d n=%d  median %7llu cycles (%5.0f / pivot)  max %7llu  trace[0] %.15e\n", name, B, n, h[B / 2],
         (double)h[B / 2] / n, h[B - 1], o[0]);
  (void)hipFree(out);
  (void)hipFree(cyc);
}

int main() {
  for (int B : {256, 1024}) {
    run<0>(B, 60, "full 4x8 tiles (kernel)");
    run<1>(B, 60, "lower 4x4 tiles (120 lanes)");
  }
  return 0;
}
