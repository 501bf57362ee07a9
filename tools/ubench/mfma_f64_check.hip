// Diagnostic: operand / result lane maps of v_mfma_f64_16x16x4_f64 on gfx950, checked
// with exact integer data against a host product, plus its issue cost (s_memtime).
//   A (16x4): lane l holds A[l & 15][l >> 4];  B (4x16): lane l holds B[l >> 4][l & 15]
//   C/D (16x16): lane l, register i holds D[(l >> 4) + 4 i][l & 15]
#include <hip/hip_runtime.h>
#include <stdio.h>

typedef double d4 __attribute__((ext_vector_type(4)));

__global__ void k_map(const double* A, const double* B, const double* C, double* D) {
  const int l = threadIdx.x;
  const double a = A[(l & 15) * 4 + (l >> 4)];
  const double b = B[(l >> 4) * 16 + (l & 15)];
  d4 c;
  for (int i = 0; i < 4; ++i) c[i] = C[((l >> 4) + 4 * i) * 16 + (l & 15)];
  d4 d = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0);
  for (int i = 0; i < 4; ++i) D[((l >> 4) + 4 * i) * 16 + (l & 15)] = d[i];
}

__global__ void k_rate(double* out, int iters, unsigned long long* cyc) {
  const int l = threadIdx.x;
  double a = 1.0 + l * 1e-3, b = 0.5;
  d4 c[8];
  for (int j = 0; j < 8; ++j)
    for (int i = 0; i < 4; ++i) c[j][i] = j + i;
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < iters; ++it)
#pragma unroll
    for (int j = 0; j < 8; ++j) c[j] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c[j], 0, 0, 0);
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  double s = 0;
  for (int j = 0; j < 8; ++j) s += c[j][0] + c[j][1] + c[j][2] + c[j][3];
  out[blockIdx.x * 64 + l] = s;
  if (l == 0) cyc[blockIdx.x] = t1 - t0;
}

int main() {
  double hA[64], hB[64], hC[256], hD[256], ref[256];
  for (int i = 0; i < 64; ++i) {
    hA[i] = (i * 7) % 11 - 5;
    hB[i] = (i * 5) % 13 - 6;
  }
  for (int i = 0; i < 256; ++i) hC[i] = (i * 3) % 17 - 8;
  for (int r = 0; r < 16; ++r)
    for (int c = 0; c < 16; ++c) {
      double s = hC[r * 16 + c];
      for (int k = 0; k < 4; ++k) s += hA[r * 4 + k] * hB[k * 16 + c];
      ref[r * 16 + c] = s;
    }
  double *dA, *dB, *dC, *dD;
  (void)hipMalloc(&dA, 512);
  (void)hipMalloc(&dB, 512);
  (void)hipMalloc(&dC, 2048);
  (void)hipMalloc(&dD, 2048);
  (void)hipMemcpy(dA, hA, 512, hipMemcpyHostToDevice);
  (void)hipMemcpy(dB, hB, 512, hipMemcpyHostToDevice);
  (void)hipMemcpy(dC, hC, 2048, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(k_map, dim3(1), dim3(64), 0, 0, dA, dB, dC, dD);
  (void)hipMemcpy(hD, dD, 2048, hipMemcpyDeviceToHost);
  int bad = 0;
  for (int i = 0; i < 256; ++i) bad += hD[i] != ref[i];
  printf("mfma_f64_16x16x4 lane maps: %s (%d of 256 entries differ)\n", bad ? "MISMATCH" : "exact", bad);
  double* out;
  unsigned long long* cyc;
  (void)hipMalloc(&out, 64 * 8 * 1024);
  (void)hipMalloc(&cyc, 8 * 1024);
  for (int blocks : {256, 1024, 2048}) {
    hipLaunchKernelGGL(k_rate, dim3(blocks), dim3(64), 0, 0, out, 1000, cyc);
    hipLaunchKernelGGL(k_rate, dim3(blocks), dim3(64), 0, 0, out, 1000, cyc);
    unsigned long long h[2048];
    (void)hipMemcpy(h, cyc, 8 * blocks, hipMemcpyDeviceToHost);
    unsigned long long s = 0;
    for (int i = 0; i < blocks; ++i) s += h[i];
    printf("blocks %4d (waves/SIMD %.2f): %.1f cycles per MFMA per wave (8 independent accumulators)\n", blocks,
           blocks / 1024.0, (double)s / blocks / (1000.0 * 8));
  }
  return 0;
}
