// Microbenchmarks (diagnostic only): one wave per CU, s_memtime-timed.
#include <hip/hip_runtime.h>
#include <stdio.h>

__global__ void fma_indep(double* out, int iters, unsigned long long* cyc) {
  double a[16];
  for (int i = 0; i < 16; ++i) a[i] = threadIdx.x * 1e-3 + i;
  const double b = 1.0000001, c = 1e-9;
  unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < 16; ++i) a[i] = fma(a[i], b, c);
  }
  unsigned long long t1 = __builtin_amdgcn_s_memtime();
  double s = 0; for (int i = 0; i < 16; ++i) s += a[i];
  out[threadIdx.x] = s;
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

__global__ void fma32_indep(float* out, int iters, unsigned long long* cyc) {
  float a[16];
  for (int i = 0; i < 16; ++i) a[i] = threadIdx.x * 1e-3f + i;
  const float b = 1.0000001f, c = 1e-9f;
  unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < 16; ++i) a[i] = fmaf(a[i], b, c);
  }
  unsigned long long t1 = __builtin_amdgcn_s_memtime();
  float s = 0; for (int i = 0; i < 16; ++i) s += a[i];
  out[threadIdx.x] = s;
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

__global__ void lds_chain(double* out, int iters, unsigned long long* cyc) {
  __shared__ double buf[256];
  buf[threadIdx.x] = threadIdx.x;
  __syncthreads();
  int idx = 0;
  double acc = 0;
  unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < iters; ++it) {
    double v = buf[idx];             // broadcast read, dependent chain
    idx = ((int)v + 1) & 63;
    acc += v;
  }
  unsigned long long t1 = __builtin_amdgcn_s_memtime();
  out[threadIdx.x] = acc;
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

__global__ void lds_b128_burst(double* out, int iters, unsigned long long* cyc) {
  __shared__ double buf[64];
  buf[threadIdx.x] = threadIdx.x;
  __syncthreads();
  double acc = 0;
  unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < iters; ++it) {
    double v[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) v[i] = buf[(i + it) & 63];   // broadcast reads
#pragma unroll
    for (int i = 0; i < 16; ++i) acc += v[i];
    __builtin_amdgcn_s_waitcnt(0);
  }
  unsigned long long t1 = __builtin_amdgcn_s_memtime();
  out[threadIdx.x] = acc;
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

__global__ void memtime_vs_realtime(unsigned long long* o) {
  unsigned long long a = __builtin_amdgcn_s_memtime(), r = __builtin_amdgcn_s_memrealtime();
  double x = threadIdx.x;
  for (int i = 0; i < 2000000; ++i) x = fma(x, 1.0000001, 1e-9);
  unsigned long long b = __builtin_amdgcn_s_memtime(), r2 = __builtin_amdgcn_s_memrealtime();
  if (threadIdx.x == 0) { o[0] = b - a; o[1] = r2 - r; o[2] = (unsigned long long)x; }
}

typedef double d4 __attribute__((ext_vector_type(4)));
__global__ void mfma_f64(double* out, int iters, unsigned long long* cyc) {
  d4 acc0 = {0, 0, 0, 0}, acc1 = acc0, acc2 = acc0, acc3 = acc0;
  double a = threadIdx.x * 1e-3, b = 1.0 + threadIdx.x * 1e-4;
  unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < iters; ++it) {
    acc0 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc0, 0, 0, 0);
    acc1 = __builtin_amdgcn_mfma_f64_16x16x4f64(b, a, acc1, 0, 0, 0);
    acc2 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, a, acc2, 0, 0, 0);
    acc3 = __builtin_amdgcn_mfma_f64_16x16x4f64(b, b, acc3, 0, 0, 0);
  }
  unsigned long long t1 = __builtin_amdgcn_s_memtime();
  out[threadIdx.x] = acc0[0] + acc1[1] + acc2[2] + acc3[3];
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

__global__ void lds_b128_bcast(double* out, int iters, unsigned long long* cyc) {
  __shared__ double buf[128];
  buf[threadIdx.x] = threadIdx.x; buf[threadIdx.x + 64] = threadIdx.x;
  __syncthreads();
  double acc = 0;
  typedef double d2 __attribute__((ext_vector_type(2)));
  const d2* p = (const d2*)buf;
  unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < iters; ++it) {
    d2 v[16];
    const int o = it & 31;
#pragma unroll
    for (int i = 0; i < 16; ++i) v[i] = p[(o + i) & 63];
#pragma unroll
    for (int i = 0; i < 16; ++i) acc += v[i][0] + v[i][1];
  }
  unsigned long long t1 = __builtin_amdgcn_s_memtime();
  out[threadIdx.x] = acc;
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

// LDS write -> workgroup barrier -> LDS read of another wave's value, per iteration
__global__ void bar_lds(double* out, int iters, unsigned long long* cyc) {
  __shared__ double buf[1024];
  const int t = threadIdx.x, nt = blockDim.x;
  double v = t;
  unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < iters; ++it) {
    buf[(it & 1) * 512 + t] = v;
    __syncthreads();
    v += buf[(it & 1) * 512 + (t + 64) % nt] * 1e-9;
  }
  unsigned long long t1 = __builtin_amdgcn_s_memtime();
  out[t] = v;
  if (t == 0) cyc[blockIdx.x] = t1 - t0;
}

// 32 independent f64 FMAs per iteration with a barrier every iteration
__global__ void bar_fma(double* out, int iters, unsigned long long* cyc) {
  double a[32];
  for (int i = 0; i < 32; ++i) a[i] = threadIdx.x * 1e-3 + i;
  const double b = 1.0000001, c = 1e-9;
  unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < 32; ++i) a[i] = fma(a[i], b, c);
    __syncthreads();
  }
  unsigned long long t1 = __builtin_amdgcn_s_memtime();
  double s = 0; for (int i = 0; i < 32; ++i) s += a[i];
  out[threadIdx.x] = s;
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

int main() {
  double* d; float* f; unsigned long long* c;
  hipMalloc(&d, 1 << 20); hipMalloc(&f, 1 << 20); hipMalloc(&c, 1 << 16);
  unsigned long long h[4];
  const int iters = 10000;
  auto run = [&](const char* name, void (*k)(double*, int, unsigned long long*), int grid, double ops_per_iter) {
    hipLaunchKernelGGL(k, dim3(grid), dim3(64), 0, 0, d, iters, c);
    hipLaunchKernelGGL(k, dim3(grid), dim3(64), 0, 0, d, iters, c);
    hipDeviceSynchronize();
    hipMemcpy(h, c, 8, hipMemcpyDeviceToHost);
    printf("%-24s grid %4d: %.2f cycles per op\n", name, grid, (double)h[0] / (iters * ops_per_iter));
  };
  run("v_fma_f64 (16 indep)", fma_indep, 1, 16);
  run("v_fma_f64 (16 indep)", fma_indep, 1024, 16);
  hipLaunchKernelGGL(fma32_indep, dim3(1), dim3(64), 0, 0, f, iters, c);
  hipDeviceSynchronize(); hipMemcpy(h, c, 8, hipMemcpyDeviceToHost);
  printf("%-24s grid %4d: %.2f cycles per op\n", "v_fma_f32 (16 indep)", 1, (double)h[0] / (iters * 16));
  run("ds_read_b64 dep chain", lds_chain, 1, 1);
  run("mfma_f64_16x16x4 (4 acc)", mfma_f64, 1, 4);
  run("mfma_f64_16x16x4 (4 acc)", mfma_f64, 1024, 4);
  run("16x ds_read_b128 bcast", lds_b128_bcast, 1, 16);
  run("16x ds_read bcast+wait", lds_b128_burst, 1, 1);
  for (int nt = 64; nt <= 512; nt *= 2) {
    for (int g : {1, 256}) {
      hipLaunchKernelGGL(bar_lds, dim3(g), dim3(nt), 0, 0, d, 2000, c);
      hipLaunchKernelGGL(bar_lds, dim3(g), dim3(nt), 0, 0, d, 2000, c);
      hipDeviceSynchronize(); hipMemcpy(h, c, 8, hipMemcpyDeviceToHost);
      printf("write+barrier+read   %3d thr grid %3d: %.1f cycles/iter\n", nt, g, (double)h[0] / 2000);
      hipLaunchKernelGGL(bar_fma, dim3(g), dim3(nt), 0, 0, d, 2000, c);
      hipLaunchKernelGGL(bar_fma, dim3(g), dim3(nt), 0, 0, d, 2000, c);
      hipDeviceSynchronize(); hipMemcpy(h, c, 8, hipMemcpyDeviceToHost);
      printf("32 fma_f64 + barrier %3d thr grid %3d: %.1f cycles/iter\n", nt, g, (double)h[0] / 2000);
    }
  }
  hipLaunchKernelGGL(memtime_vs_realtime, dim3(1), dim3(64), 0, 0, c);
  hipDeviceSynchronize(); hipMemcpy(h, c, 16, hipMemcpyDeviceToHost);
  printf("s_memtime ticks %llu vs realtime(100MHz) %llu -> %.3f GHz\n", h[0], h[1], h[0] / (h[1] / 100e6) / 1e9);
  return 0;
}
