// Microbenchmark (diagnostic only): cost of one LDS exchange step between the waves of
// a workgroup -- write a value, synchronise, read another wave's value -- for 1, 2 and
// 4 waves, with __syncthreads() and with the wave-only fence; plus the f64 wave argmin
// chain and a readlane broadcast.  s_memtime cycles per step, median over blocks.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <algorithm>
#include <vector>

template <int NT, bool BAR>
__global__ __launch_bounds__(NT) void exch(double* out, int iters, unsigned long long* cyc) {
  __shared__ double buf[2][NT];
  const int t = threadIdx.x;
  double v = t;
  buf[0][t] = v;
  __syncthreads();
  unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < iters; ++it) {
    const int b = it & 1;
    v = buf[b][(t + 67 * (it + 1)) % NT] + 1.0;   // another wave's entry
    buf[b ^ 1][t] = v;
    if (BAR) {
      __syncthreads();
    } else {
      __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
      __builtin_amdgcn_wave_barrier();
    }
  }
  unsigned long long t1 = __builtin_amdgcn_s_memtime();
  out[blockIdx.x * NT + t] = v;
  if (t == 0) cyc[blockIdx.x] = t1 - t0;
}

template <typename K>
static void run(const char* name, K kern, int nt, int blocks) {
  double* out;
  unsigned long long* cyc;
  hipMalloc(&out, sizeof(double) * blocks * 1024);
  hipMalloc(&cyc, sizeof(unsigned long long) * blocks);
  const int iters = 2000;
  hipLaunchKernelGGL(kern, dim3(blocks), dim3(nt), 0, 0, out, iters, cyc);
  hipLaunchKernelGGL(kern, dim3(blocks), dim3(nt), 0, 0, out, iters, cyc);
  hipDeviceSynchronize();
  std::vector<unsigned long long> h(blocks);
  hipMemcpy(h.data(), cyc, sizeof(unsigned long long) * blocks, hipMemcpyDeviceToHost);
  std::sort(h.begin(), h.end());
  printf("%-34s blocks %4d: %7.1f cycles/step (median)\n", name, blocks, (double)h[blocks / 2] / iters);
  hipFree(out);
  hipFree(cyc);
}

int main() {
  for (int blocks : {256, 1024}) {
    run("1 wave, wave fence", exch<64, false>, 64, blocks);
    run("1 wave, __syncthreads", exch<64, true>, 64, blocks);
    run("2 waves, __syncthreads", exch<128, true>, 128, blocks);
    run("4 waves, __syncthreads", exch<256, true>, 256, blocks);
    run("8 waves, __syncthreads", exch<512, true>, 512, blocks);
  }
  return 0;
}
