// ubench_mlp.hip -- the forward's MLP K loop in isolation: 16x16x4 f32 MFMAs over a weight stream
// from L2 ([tile][chunk][64 lanes] float4, every workgroup reading the same bytes) and activation
// fragments from LDS.  Variants: register sets in flight (prefetch distance NS-1 chunks), K split
// over KS waves per SIMD (8 waves per workgroup at KS = 2), loads on / off, waves-per-EU budget.
// Random weights.  3 layers x 25 chunks x 4*TPW tiles per launch, 16 rows per workgroup.
//   hipcc --offload-arch=gfx950 -O3 tools/ubench_mlp.hip -o tools/ubench_mlp && ./tools/ubench_mlp
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

typedef float f32x4 __attribute__((ext_vector_type(4)));
#define CHECK(x) do { hipError_t err_ = (x); if (err_ != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(err_), __LINE__); exit(1); } } while (0)

template <int TPW, int KS, int NS, bool LOADS, int WPE>
__global__ void __launch_bounds__(256 * KS) __attribute__((amdgpu_waves_per_eu(WPE)))
kern(const f32x4* __restrict__ w, int NT_, int NC, int layers, float* out) {
  __shared__ f32x4 actl[32 * 64];
  __shared__ f32x4 red[KS > 1 ? 4 * TPW * 64 : 1];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, g = wave & 3, kh = wave >> 2;
  for (int i = threadIdx.x; i < 32 * 64; i += 256 * KS) actl[i] = f32x4{1e-3f * i, 0.5f, 1.f, -2.f};
  __syncthreads();
  f32x4 acc[TPW];
  float keep = 0.f;
  for (int L = 0; L < layers; ++L) {
#pragma unroll
    for (int j = 0; j < TPW; ++j) acc[j] = f32x4{0, 0, 0, 0};
    int soff[TPW];
#pragma unroll
    for (int j = 0; j < TPW; ++j) {
      int t = g + 4 * j;
      t = t < NT_ ? t : NT_ - 1;
      soff[j] = __builtin_amdgcn_readfirstlane(t * NC * 1024);
    }
    const __amdgpu_buffer_rsrc_t rsrc =
        __builtin_amdgcn_make_buffer_rsrc((void*)(w + (size_t)L * NT_ * NC * 64), (short)0, NT_ * NC * 1024, 0x00020000);
    const int n = (NC - kh + KS - 1) / KS;
    auto chunk = [n, kh](int i) { return kh + KS * (i < n ? i : n - 1); };
    f32x4 b[NS][TPW];
    f32x4 a[NS];
    auto LOAD = [&](f32x4 (&bb)[TPW], int c) {
      if constexpr (LOADS) {
#pragma unroll
        for (int j = 0; j < TPW; ++j)
          bb[j] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rsrc, lane * 16, soff[j] + c * 1024, 0));
      } else {
#pragma unroll
        for (int j = 0; j < TPW; ++j) bb[j] = f32x4{0.01f * j, 0.02f, 0.03f, (float)c};
      }
    };
#pragma unroll
    for (int s = 0; s < NS - 1; ++s) {
      LOAD(b[s], chunk(s));
      a[s] = actl[(chunk(s) & 31) * 64 + lane];
    }
    for (int i0 = 0; i0 < n; i0 += NS) {
#pragma unroll
      for (int u = 0; u < NS; ++u) {
        const int i = i0 + u;
        if (i < n) {
          constexpr int dummy = 0;
          (void)dummy;
          const int z = (u + NS - 1) % NS;
          a[z] = actl[(chunk(i + NS - 1) & 31) * 64 + lane];
          LOAD(b[z], chunk(i + NS - 1));
#pragma unroll
          for (int s = 0; s < 4; ++s)
#pragma unroll
            for (int j = 0; j < TPW; ++j) acc[j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[u][s], b[u][j][s], acc[j], 0, 0, 0);
          __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
          for (int q = 0; q < TPW; ++q) {
            __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);
            __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);
          }
          __builtin_amdgcn_sched_group_barrier(0x008, 2 * TPW, 0);
          __builtin_amdgcn_sched_barrier(0);
        }
      }
    }
    if constexpr (KS == 2) {
      if (kh == 1) {
#pragma unroll
        for (int j = 0; j < TPW; ++j) red[(g * TPW + j) * 64 + lane] = acc[j];
      }
      __syncthreads();
      if (kh == 0) {
#pragma unroll
        for (int j = 0; j < TPW; ++j) acc[j] += red[(g * TPW + j) * 64 + lane];
      }
    }
#pragma unroll
    for (int j = 0; j < TPW; ++j) keep += acc[j][0] + acc[j][1] + acc[j][2] + acc[j][3];
    __syncthreads();
  }
  if (keep == 12345.678f) out[threadIdx.x] = keep;
}

template <int TPW, int KS, int NS, bool LOADS, int WPE>
void run(const char* name, const f32x4* w, int grid, float* out, hipStream_t* st, int nst) {
  const int NT_ = 4 * TPW, NC = 25, layers = 3;
  auto k = kern<TPW, KS, NS, LOADS, WPE>;
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  for (int r = 0; r < 3; ++r) hipLaunchKernelGGL(k, dim3(grid), dim3(256 * KS), 0, st[0], w, NT_, NC, layers, out);
  CHECK(hipDeviceSynchronize());
  const int reps = 100;
  CHECK(hipEventRecord(e0, 0));
  for (int s = 0; s < nst; ++s) CHECK(hipStreamWaitEvent(st[s], e0, 0));
  for (int r = 0; r < reps; ++r) hipLaunchKernelGGL(k, dim3(grid), dim3(256 * KS), 0, st[r % nst], w, NT_, NC, layers, out);
  for (int s = 0; s < nst; ++s) {
    hipEvent_t ev;
    CHECK(hipEventCreate(&ev));
    CHECK(hipEventRecord(ev, st[s]));
    CHECK(hipStreamWaitEvent(0, ev, 0));
  }
  CHECK(hipEventRecord(e1, 0));
  CHECK(hipEventSynchronize(e1));
  float ms;
  CHECK(hipEventElapsedTime(&ms, e0, e1));
  const double us = ms * 1e3 / reps;
  const double mfma = (double)layers * NC * TPW * 4 * 4 * grid;
  printf("%-46s grid %4d streams %d: %7.2f us/launch %6.1f TFLOP/s %6.2f us per 4096 rows\n", name, grid, nst, us,
         mfma * 2048 / (us * 1e6), us * 4096.0 / (16.0 * grid));
}

int main() {
  const size_t n = (size_t)3 * 32 * 25 * 64;
  f32x4* w;
  float* out;
  CHECK(hipMalloc(&w, n * sizeof(f32x4)));
  CHECK(hipMalloc(&out, 4096 * sizeof(float)));
  float* h = (float*)malloc(n * sizeof(f32x4));
  srand(1);
  for (size_t i = 0; i < n * 4; ++i) h[i] = (rand() / (float)RAND_MAX - 0.5f) * 0.1f;
  CHECK(hipMemcpy(w, h, n * sizeof(f32x4), hipMemcpyHostToDevice));
  hipStream_t st[4];
  for (int s = 0; s < 4; ++s) CHECK(hipStreamCreate(&st[s]));
  run<6, 1, 3, true, 2>("KS1 NS3 loads (forward today)", w, 256, out, st, 1);
  run<6, 1, 3, false, 2>("KS1 NS3 no loads", w, 256, out, st, 1);
  run<6, 1, 4, true, 2>("KS1 NS4 loads", w, 256, out, st, 1);
  run<6, 1, 5, true, 2>("KS1 NS5 loads", w, 256, out, st, 1);
  run<6, 1, 6, true, 1>("KS1 NS6 loads wpe1", w, 256, out, st, 1);
  run<6, 2, 3, true, 4>("KS2 NS3 loads wpe4", w, 256, out, st, 1);
  run<6, 2, 3, true, 4>("KS2 NS3 loads wpe4", w, 256, out, st, 2);
  run<6, 2, 2, true, 4>("KS2 NS2 loads wpe4", w, 256, out, st, 2);
  run<6, 1, 3, true, 2>("KS1 NS3 loads", w, 256, out, st, 2);
  run<6, 1, 4, true, 2>("KS1 NS4 loads", w, 256, out, st, 2);
  return 0;
}
