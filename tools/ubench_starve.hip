// Microbenchmark: how fast does a wave progress beside waves that saturate its SIMD's matrix pipe?
// One 768-thread workgroup per CU: waves 0-7 ("MLP", two per SIMD) issue back-to-back independent
// v_mfma_f32_16x16x4_f32 (12 accumulators, like the MLP K loop) while waves 8-11 ("helper", one per SIMD) time
// one of: a chain of dependent MFMAs, a chain of dependent VALU FMAs, a chain of dependent LDS reads; with the MLP
// waves idle, busy, one per SIMD busy, busy with an s_sleep after every 12 MFMAs, and with the helper at priority 3.
// DESIGN.md §3.7 / §4.5 (profiles/r05/ubench_starve.log).
//   hipcc --offload-arch=gfx950 -O3 tools/ubench_starve.hip -o /tmp/ubench_starve && /tmp/ubench_starve
#include <hip/hip_runtime.h>
#include <stdio.h>

typedef float f32x4 __attribute__((ext_vector_type(4)));

__global__ void __launch_bounds__(768) starve(float* out, int mlp_iters, int chain, int kind, int mode,
                                             int prio, int helpers_first, uint64_t* cyc) {
  __shared__ int lds[1024];
  const int tid = threadIdx.x, lane = tid & 63;
  // helpers_first: the helpers are waves 0-3 (the oldest on their SIMDs), the MLP waves 4-11
  const int w = tid >> 6, wave = helpers_first ? (w < 4 ? w + 8 : w - 4) : w;
  for (int i = tid; i < 1024; i += 768) lds[i] = (i + 1) & 1023;
  __syncthreads();
  float a = lane * 1e-3f, b = blockIdx.x * 1e-3f;
  if (wave < 8) {
    f32x4 acc[12];
#pragma unroll
    for (int j = 0; j < 12; ++j) acc[j] = f32x4{0.f, 0.f, 0.f, 0.f};
    // mode 1: back to back; mode 2: one MLP wave per SIMD (waves 4-7 idle); mode 3: s_sleep 1 after every 12 MFMAs
    const int n = (mode == 0 || (mode == 2 && wave >= 4)) ? 0 : mlp_iters;
    const uint64_t m0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < n; ++i) {
#pragma unroll
      for (int j = 0; j < 12; ++j) acc[j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, acc[j], 0, 0, 0);
      if (mode == 3) __builtin_amdgcn_s_sleep(1);
    }
    const uint64_t m1 = __builtin_amdgcn_s_memtime();
    if (lane == 0 && wave == 0) cyc[1024 + blockIdx.x] = m1 - m0;  // (role 0: the first MLP wave)
    float s = 0.f;
#pragma unroll
    for (int j = 0; j < 12; ++j) s += acc[j][0];
    out[blockIdx.x * 768 + tid] = s;
  } else {
    // let the MLP waves get going first
    __builtin_amdgcn_s_sleep(20);
    if (prio) __builtin_amdgcn_s_setprio(3);
    const uint64_t t0 = __builtin_amdgcn_s_memtime();
    float s = 0.f;
    if (kind == 0) {
      f32x4 acc = f32x4{0.f, 0.f, 0.f, 0.f};
      for (int i = 0; i < chain; ++i) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, acc, 0, 0, 0);
      s = acc[0];
    } else if (kind == 1) {
      float x = a;
      for (int i = 0; i < chain; ++i) x = fmaf(x, 1.0001f, b);
      s = x;
    } else {
      int p = lane;
      for (int i = 0; i < chain; ++i) p = lds[p];
      s = (float)p;
    }
    const uint64_t t1 = __builtin_amdgcn_s_memtime();
    out[blockIdx.x * 768 + tid] = s;
    if (lane == 0) cyc[blockIdx.x * 4 + (wave - 8)] = t1 - t0;
  }
}

int main() {
  float* out;
  uint64_t* cyc;
  hipMalloc(&out, 256 * 768 * sizeof(float));
  hipMalloc(&cyc, 256 * 5 * sizeof(uint64_t));
  const char* kinds[3] = {"dependent MFMA", "dependent VALU fma", "dependent LDS read"};
  const int chains[3] = {200, 2000, 500};
  for (int kind = 0; kind < 3; ++kind) {
    const char* modes[6] = {"idle", "busy", "busy, one MLP wave per SIMD", "busy, s_sleep 1 per 12 MFMAs",
                            "busy, helper at priority 3", "busy, helpers the oldest waves"};
    for (int mode = 0; mode < 6; ++mode) {
      for (int rep = 0; rep < 2; ++rep)
        hipLaunchKernelGGL(starve, dim3(256), dim3(768), 0, 0, out, 4000, chains[kind], kind, mode >= 4 ? 1 : mode,
                           mode == 4, mode == 5, cyc);
      hipDeviceSynchronize();
      uint64_t c[1280];
      hipMemcpy(c, cyc, sizeof c, hipMemcpyDeviceToHost);
      double mean = 0, mlp = 0;
      for (int i = 0; i < 1024; ++i) mean += c[i] / 1024.0;
      for (int i = 0; i < 256; ++i) mlp += c[1024 + i] / 256.0;
      printf("%-20s MLP waves %-30s: %8.1f cycles per chain step; MLP wave 0: %.1f cycles per MFMA\n", kinds[kind],
             modes[mode], mean / chains[kind], mode == 0 ? 0.0 : mlp / (4000.0 * 12));
    }
  }
  return 0;
}
