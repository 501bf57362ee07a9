// Diagnostic: the class-64 one-wave lower-tile sweep (mpcqp_solve.h, kSym) in isolation,
// s_memtime-timed per workgroup, with stripped variants to locate the cost per pivot:
//   V0 full, V1 no FMAs, V2 no LDS pivot column (register stand-in), V3 no reciprocal,
//   V4 full but with a wave-level s_barrier-free fence removed (plain program order)
// Workgroups of 128 threads (wave 1 idles as in the kernel), 4 per CU.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <vector>
#include <algorithm>

typedef double d2 __attribute__((ext_vector_type(2)));
constexpr int LANES = 64;

__device__ __forceinline__ int lt_idx(int br, int bc) {
  const int m = br >> 1;
  return ((br & 1) ? (m + 1) * (m + 1) : m * (m + 1)) + bc;
}
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

template <int V>
__global__ __launch_bounds__(128) __attribute__((amdgpu_waves_per_eu(2, 2))) void symsweep(int n, double* out,
                                                                                        unsigned long long* cyc) {
  __shared__ double ht[2048];
  __shared__ __attribute__((aligned(16))) double zc[64];
  __shared__ __attribute__((aligned(16))) double zc2[64];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  // synthetic SPD H: diag n + 1, off-diagonal 1 / (1 + |i - j|)
  for (int e = tid; e < 2048; e += 128) {
    const int L = e & 63, el = e >> 6, r = el >> 3, c = el & 7;
    int br = 0;
    for (int bb = 1; bb < 15; ++bb) br = lt_idx(bb, 0) <= L ? bb : br;
    const int bc = L - lt_idx(br, 0);
    const int i = 4 * br + r, j = 8 * bc + c;
    double h = (i < n && j < n) ? (i == j ? n + 1.0 : 1.0 / (1.0 + (i > j ? i - j : j - i))) : (i == j ? 1.0 : 0.0);
    ht[e] = h + 1e-3 * blockIdx.x;
  }
  __syncthreads();
  unsigned long long t0 = __builtin_amdgcn_s_memtime();
  double acc = 0.0;
  if (wave == 0) {
    int br = 0;
    for (int bb = 1; bb < 15; ++bb) br = lt_idx(bb, 0) <= lane ? bb : br;
    const int bc = lane - lt_idx(br, 0);
    double W[4][8];
    for (int r = 0; r < 4; ++r)
      for (int c = 0; c < 8; ++c) W[r][c] = ht[(8 * r + c) * 64 + lane];
    if (lane < 4) zc[60 + lane] = 0.0;
    if constexpr (V == 6) {
      // pipelined: pivot K + 1's row and column are updated first and published before the
      // rest of pivot K's FMAs, which then overlap the LDS round trip
      auto publish = [&](auto KCn, int KTn) {
        constexpr int KC = decltype(KCn)::value;
        constexpr int KRR = KC & 3;
        const int KR = 2 * KTn + (KC >> 2);
        if (br == KR) {
          d2* p = reinterpret_cast<d2*>(zc + 8 * bc);
          for (int i = 0; i < 4; ++i) p[i] = d2{W[KRR][2 * i], W[KRR][2 * i + 1]};
        }
        if (bc == KTn) {
          d2* pz = reinterpret_cast<d2*>(zc + 4 * br);
          pz[0] = d2{W[0][KC], W[1][KC]};
          pz[1] = d2{W[2][KC], W[3][KC]};
        }
        __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
        __builtin_amdgcn_wave_barrier();
      };
      publish(std::integral_constant<int, 0>{}, 0);
#pragma unroll 1
      for (int KT = 0; 8 * KT < n; ++KT) {
        sfor([&](auto KCc) {
          constexpr int KC = decltype(KCc)::value;
          constexpr int KRR = KC & 3;
          constexpr int NC = (KC + 1) & 7, NR = (KC + 1) & 3;
          const int K = 8 * KT + KC;
          const int KR = 2 * KT + (KC >> 2);
          if (K < n) {
            double zr[8], zi[4];
            const d2* p = reinterpret_cast<const d2*>(zc + 8 * bc);
            for (int i = 0; i < 4; ++i) { const d2 x = p[i]; zr[2 * i] = x[0]; zr[2 * i + 1] = x[1]; }
            const d2* q = reinterpret_cast<const d2*>(zc + 4 * br);
            const d2 a = q[0], b = q[1];
            zi[0] = a[0]; zi[1] = a[1]; zi[2] = b[0]; zi[3] = b[1];
            const double dK = zc[K];
            const double inv = rcp_nr(dK);
            double beta[4];
            for (int r = 0; r < 4; ++r) beta[r] = -zi[r] * inv;
            if (br == KR) beta[KRR] = inv - 1.0;
            if (bc == KT) zr[KC] = dK - 1.0;
            // pivot K + 1's row NR and column NC first
            for (int c = 0; c < 8; ++c) W[NR][c] = fma(beta[NR], zr[c], W[NR][c]);
            for (int r = 0; r < 4; ++r)
              if (r != NR) W[r][NC] = fma(beta[r], zr[NC], W[r][NC]);
            if constexpr (NR == KRR || NC == KC) {
            }
            __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
            __builtin_amdgcn_wave_barrier();
            if (K + 1 < n) publish(std::integral_constant<int, NC>{}, KC == 7 ? KT + 1 : KT);
            for (int r = 0; r < 4; ++r)
              for (int c = 0; c < 8; ++c)
                if (r != NR && c != NC) W[r][c] = fma(beta[r], zr[c], W[r][c]);
            W[KRR][KC] += (bc == KT && br == KR) ? -2.0 : 0.0;
          }
        }, std::make_integer_sequence<int, 8>{});
      }
    } else if constexpr (V == 5) {
      double* const z0 = zc;
      double* const z1 = zc2;
      if (lane < 4) { z0[60 + lane] = 0.0; z1[60 + lane] = 0.0; }
#pragma unroll 1
      for (int KT = 0; 8 * KT < n; ++KT) {
        sfor([&](auto KPc) {
          constexpr int KC = 2 * decltype(KPc)::value;
          constexpr int KRR = KC & 3;   // 0 or 2
          const int K = 8 * KT + KC;
          const int KR = 2 * KT + (KC >> 2);
          if (K < n) {
            if (br == KR) {
              d2* p = reinterpret_cast<d2*>(z0 + 8 * bc);
              d2* q = reinterpret_cast<d2*>(z1 + 8 * bc);
              for (int i = 0; i < 4; ++i) {
                p[i] = d2{W[KRR][2 * i], W[KRR][2 * i + 1]};
                q[i] = d2{W[KRR + 1][2 * i], W[KRR + 1][2 * i + 1]};
              }
            }
            if (bc == KT) {
              d2* p = reinterpret_cast<d2*>(z0 + 4 * br);
              d2* q = reinterpret_cast<d2*>(z1 + 4 * br);
              p[0] = d2{W[0][KC], W[1][KC]};
              p[1] = d2{W[2][KC], W[3][KC]};
              q[0] = d2{W[0][KC + 1], W[1][KC + 1]};
              q[1] = d2{W[2][KC + 1], W[3][KC + 1]};
            }
            __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
            __builtin_amdgcn_wave_barrier();
            double zr0[8], zr1[8], zi0[4], zi1[4];
            {
              const d2* p = reinterpret_cast<const d2*>(z0 + 8 * bc);
              const d2* q = reinterpret_cast<const d2*>(z1 + 8 * bc);
              for (int i = 0; i < 4; ++i) {
                const d2 x = p[i], y = q[i];
                zr0[2 * i] = x[0]; zr0[2 * i + 1] = x[1];
                zr1[2 * i] = y[0]; zr1[2 * i + 1] = y[1];
              }
              const d2* a = reinterpret_cast<const d2*>(z0 + 4 * br);
              const d2* b = reinterpret_cast<const d2*>(z1 + 4 * br);
              const d2 a0 = a[0], a1 = a[1], b0 = b[0], b1 = b[1];
              zi0[0] = a0[0]; zi0[1] = a0[1]; zi0[2] = a1[0]; zi0[3] = a1[1];
              zi1[0] = b0[0]; zi1[1] = b0[1]; zi1[2] = b1[0]; zi1[3] = b1[1];
            }
            const double d00 = z0[K], d01 = z0[K + 1], d11 = z1[K + 1];
            const double idet = rcp_nr(fma(d00, d11, -d01 * d01));
            const double e00 = d11 * idet, e01 = -d01 * idet, e11 = d00 * idet;
            double c0[4], c1[4];
            for (int r = 0; r < 4; ++r) {
              c0[r] = -fma(zi0[r], e00, zi1[r] * e01);
              c1[r] = -fma(zi0[r], e01, zi1[r] * e11);
            }
            if (br == KR) {
              c0[KRR] = e00 - 1.0;
              c1[KRR] = e01;
              c0[KRR + 1] = e01;
              c1[KRR + 1] = e11 - 1.0;
            }
            if (bc == KT) {
              zr0[KC] -= 1.0;
              zr1[KC + 1] -= 1.0;
            }
            for (int r = 0; r < 4; ++r)
              for (int c = 0; c < 8; ++c) W[r][c] = fma(c1[r], zr1[c], fma(c0[r], zr0[c], W[r][c]));
            if (bc == KT && br == KR) {
              W[KRR][KC] -= 2.0;
              W[KRR + 1][KC + 1] -= 2.0;
            }
            __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
            __builtin_amdgcn_wave_barrier();
          }
        }, std::make_integer_sequence<int, 4>{});
      }
    } else
#pragma unroll 1
    for (int KT = 0; 8 * KT < n; ++KT) {
      sfor([&](auto KCc) {
        constexpr int KC = decltype(KCc)::value;
        constexpr int KRR = KC & 3;
        const int K = 8 * KT + KC;
        const int KR = 2 * KT + (KC >> 2);
        if (K < n) {
          double zr[8], zi[4];
          double dK;
          if constexpr (V == 2) {
            for (int c = 0; c < 8; ++c) zr[c] = W[KRR][c] * 1e-3;
            for (int r = 0; r < 4; ++r) zi[r] = W[r][KC] * 1e-3;
            dK = 2.0 + W[0][0] * 1e-3;
          } else {
            if (br == KR) {
              d2* p = reinterpret_cast<d2*>(zc + 8 * bc);
              for (int i = 0; i < 4; ++i) p[i] = d2{W[KRR][2 * i], W[KRR][2 * i + 1]};
            }
            if (bc == KT) {
              d2* pz = reinterpret_cast<d2*>(zc + 4 * br);
              pz[0] = d2{W[0][KC], W[1][KC]};
              pz[1] = d2{W[2][KC], W[3][KC]};
            }
            if constexpr (V != 4) {
              __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
              __builtin_amdgcn_wave_barrier();
            }
            const d2* p = reinterpret_cast<const d2*>(zc + 8 * bc);
            for (int i = 0; i < 4; ++i) { const d2 x = p[i]; zr[2 * i] = x[0]; zr[2 * i + 1] = x[1]; }
            const d2* q = reinterpret_cast<const d2*>(zc + 4 * br);
            const d2 a = q[0], b = q[1];
            zi[0] = a[0]; zi[1] = a[1]; zi[2] = b[0]; zi[3] = b[1];
            dK = zc[K];
          }
          const double inv = V == 3 ? dK : rcp_nr(dK);
          double beta[4];
          for (int r = 0; r < 4; ++r) beta[r] = -zi[r] * inv;
          if (br == KR) beta[KRR] = inv - 1.0;
          if (bc == KT) zr[KC] = dK - 1.0;
          if constexpr (V != 1) {
            for (int r = 0; r < 4; ++r)
              for (int c = 0; c < 8; ++c) W[r][c] = fma(beta[r], zr[c], W[r][c]);
          } else {
            W[KRR][KC] += beta[0] * zr[1];
          }
          W[KRR][KC] += (bc == KT && br == KR) ? -2.0 : 0.0;
          if constexpr (V != 4) {
            __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
            __builtin_amdgcn_wave_barrier();
          }
        }
      }, std::make_integer_sequence<int, 8>{});
    }
    if constexpr (V == 5) {   // pivot pairs {K, K + 1}: one rank-2 pass per pair
      // (W was swept by the single-pivot loop above only when V != 5)
    }
    for (int r = 0; r < 4; ++r)
      for (int c = 0; c < 8; ++c) acc += W[r][c];
  }
  unsigned long long t1 = __builtin_amdgcn_s_memtime();
  __syncthreads();
  if (tid == 0) cyc[blockIdx.x] = t1 - t0;
  if (wave == 0) out[blockIdx.x * 64 + lane] = acc;
}

template <int V>
void run(int B, int n, const char* name) {
  double* out;
  unsigned long long* cyc;
  hipMalloc(&out, B * 64 * sizeof(double));
  hipMalloc(&cyc, B * sizeof(unsigned long long));
  for (int rep = 0; rep < 3; ++rep) hipLaunchKernelGGL(symsweep<V>, dim3(B), dim3(128), 0, 0, n, out, cyc);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  hipEventRecord(e0);
  for (int rep = 0; rep < 20; ++rep) hipLaunchKernelGGL(symsweep<V>, dim3(B), dim3(128), 0, 0, n, out, cyc);
  hipEventRecord(e1);
  hipDeviceSynchronize();
  float ms;
  hipEventElapsedTime(&ms, e0, e1);
  std::vector<unsigned long long> h(B);
  hipMemcpy(h.data(), cyc, B * sizeof(unsigned long long), hipMemcpyDeviceToHost);
  std::sort(h.begin(), h.end());
  printf("%-28s B=%5d n=%d  median %7llu cycles (%5.0f / pivot)  max %7llu  kernel %.1f us\n", name, B, n, h[B / 2],
         (double)h[B / 2] / n, h[B - 1], ms / 20 * 1e3);
  std::vector<double> o(B * 64);
  hipMemcpy(o.data(), out, B * 64 * sizeof(double), hipMemcpyDeviceToHost);
  printf("    checksum %.15e\n", o[0] + o[64 * (B - 1) + 5]);
  hipFree(out);
  hipFree(cyc);
}

int main() {
  for (int B : {256, 1024}) {
    run<0>(B, 60, "V0 full");
    run<1>(B, 60, "V1 no FMAs");
    run<2>(B, 60, "V2 no LDS pivot column");
    run<3>(B, 60, "V3 no reciprocal");
    run<4>(B, 60, "V4 no wave fences");
    run<5>(B, 60, "V5 pivot pairs");
    run<6>(B, 60, "V6 pipelined publish");
  }
  return 0;
}
