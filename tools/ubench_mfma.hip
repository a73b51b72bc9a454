// Microbenchmark: issue rate of v_mfma_f32_16x16x4_f32 from registers only (no memory), with T
// independent accumulators per wave, 1 wave per SIMD (256-thread workgroups, one per CU) -- the
// ceiling the forward's MLP K loop is measured against.
//   hipcc --offload-arch=gfx950 -O3 tools/ubench_mfma.hip -o tools/ubench_mfma && ./tools/ubench_mfma
#include <hip/hip_runtime.h>
#include <stdio.h>

typedef float f32x4 __attribute__((ext_vector_type(4)));

template <int T>
__global__ void __launch_bounds__(512) mfma_loop(float* out, int iters, uint64_t* cyc) {
  f32x4 acc[T];
#pragma unroll
  for (int j = 0; j < T; ++j) acc[j] = f32x4{0.f, 0.f, 0.f, 0.f};
  float a = threadIdx.x * 1e-3f, b = blockIdx.x * 1e-3f;
  const uint64_t t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int j = 0; j < T; ++j) acc[j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, acc[j], 0, 0, 0);
  }
  const uint64_t t1 = __builtin_amdgcn_s_memtime();
  float s = 0.f;
#pragma unroll
  for (int j = 0; j < T; ++j) s += acc[j][0] + acc[j][1] + acc[j][2] + acc[j][3];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

template <int T>
void run(float* out, uint64_t* cyc, int iters, int nth = 256) {
  hipLaunchKernelGGL(mfma_loop<T>, dim3(256), dim3(nth), 0, 0, out, iters, cyc);
  hipDeviceSynchronize();
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  hipEventRecord(e0);
  hipLaunchKernelGGL(mfma_loop<T>, dim3(256), dim3(nth), 0, 0, out, iters, cyc);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms;
  hipEventElapsedTime(&ms, e0, e1);
  uint64_t c[256];
  hipMemcpy(c, cyc, sizeof c, hipMemcpyDeviceToHost);
  double mean = 0;
  for (int i = 0; i < 256; ++i) mean += c[i] / 256.0;
  const double n = (double)iters * T;
  const double tflops = 256.0 * (nth / 64) * n * 2048 / (ms * 1e-3) / 1e12;
  printf("waves/CU=%d T=%d: %.2f cycles/MFMA (s_memtime), %.1f TFLOP/s, clock %.2f GHz\n", nth / 64, T, mean / n, tflops,
         mean / (ms * 1e-3) / 1e9);
}

int main() {
  float* out;
  uint64_t* cyc;
  hipMalloc(&out, 256 * 512 * sizeof(float));
  hipMalloc(&cyc, 256 * sizeof(uint64_t));
  run<4>(out, cyc, 20000);
  run<6>(out, cyc, 20000);
  run<7>(out, cyc, 20000);
  run<8>(out, cyc, 20000);
  run<6>(out, cyc, 20000, 512);
  run<8>(out, cyc, 20000, 512);
  return 0;
}
