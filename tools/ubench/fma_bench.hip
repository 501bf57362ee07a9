// Microbenchmark (diagnostic only): issue cost of f64 / f32 FMAs for one wave per
// SIMD vs several, with independent accumulators (throughput) and one dependent
// chain (latency).  s_memtime cycles per instruction, median over blocks.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <algorithm>
#include <vector>

template <typename T, int ACC>
__global__ __launch_bounds__(256) void fma_k(T* out, int iters, unsigned long long* cyc, T a, T b) {
  T acc[ACC];
#pragma unroll
  for (int i = 0; i < ACC; ++i) acc[i] = (T)(threadIdx.x + i);
  __syncthreads();
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int r = 0; r < 8; ++r)
#pragma unroll
      for (int i = 0; i < ACC; ++i) acc[i] = __builtin_fma(acc[i], a, b);
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  T s = 0;
#pragma unroll
  for (int i = 0; i < ACC; ++i) s += acc[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
  if (threadIdx.x % 64 == 0) cyc[blockIdx.x * 4 + threadIdx.x / 64] = t1 - t0;
}

template <typename T, int ACC>
static void run(const char* name, int waves_per_block, int blocks) {
  T* out;
  unsigned long long* cyc;
  hipMalloc(&out, sizeof(T) * blocks * 256);
  hipMalloc(&cyc, sizeof(unsigned long long) * blocks * 4);
  hipMemset(cyc, 0, sizeof(unsigned long long) * blocks * 4);
  const int iters = 2000;
  for (int rep = 0; rep < 2; ++rep)
    hipLaunchKernelGGL((fma_k<T, ACC>), dim3(blocks), dim3(64 * waves_per_block), 0, 0, out, iters, cyc, (T)0.999,
                       (T)1e-3);
  hipDeviceSynchronize();
  std::vector<unsigned long long> h(blocks * 4);
  hipMemcpy(h.data(), cyc, sizeof(unsigned long long) * blocks * 4, hipMemcpyDeviceToHost);
  std::vector<unsigned long long> v;
  for (auto x : h)
    if (x) v.push_back(x);
  std::sort(v.begin(), v.end());
  const double per = (double)v[v.size() / 2] / ((double)iters * 8 * ACC);
  printf("%-10s acc %2d  waves/block %d blocks %5d: %6.2f cycles per wave instruction\n", name, ACC, waves_per_block,
         blocks, per);
  hipFree(out);
  hipFree(cyc);
}

int main() {
  // 256 CUs x 4 SIMDs: 256 blocks of 4 waves -> 1 wave / SIMD; 512 -> 2; 1024 -> 4
  for (int blocks : {256, 512, 1024}) {
    run<double, 8>("f64 fma", 4, blocks);
    run<double, 1>("f64 fma", 4, blocks);
    run<float, 8>("f32 fma", 4, blocks);
  }
  return 0;
}
