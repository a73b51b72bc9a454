// ubench_m32.hip -- MLP weight stream + f32 MFMA with MT row tiles (16 samples each) per workgroup.
// MT = 2 uses every weight fragment for two 16-row tiles (half the L2 -> CU bytes per FLOP).
// Random weights (the chip's clock under MFMA load depends on the data), 3 layers of 25x25 chunks,
// three register sets in flight like the forward's K loop.  Prints TFLOP/s for several grids.
//   hipcc --offload-arch=gfx950 -O3 tools/ubench_m32.hip -o tools/ubench_m32 && ./tools/ubench_m32
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

typedef float f32x4 __attribute__((ext_vector_type(4)));
#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

template <int TPW, int MT, int NW = 4, bool LD = true, bool AL = true, int NS = 3, bool REAL = false, int IL = 0>
__global__ void __launch_bounds__(64 * NW) __attribute__((amdgpu_waves_per_eu(NW == 16 ? 8 : NW / 2)))
kern(const f32x4* __restrict__ w, int NT_, int NC, int layers, float* out, unsigned* cu_ids) {
  __shared__ f32x4 actl[MT][REAL ? 1 : 32 * 64];
  extern __shared__ float lds_pad[];
  if (cu_ids && threadIdx.x == 0) {
    const unsigned hw = __builtin_amdgcn_s_getreg(4 | (31 << 11));    // HW_REG_HW_ID
    const unsigned xcc = __builtin_amdgcn_s_getreg(20 | (31 << 11));  // HW_REG_XCC_ID
    cu_ids[blockIdx.x] = ((xcc & 0xF) << 8) | ((hw >> 8) & 0xFF);
    lds_pad[0] = 0.f;
  }
  __shared__ float tile[2][16 * 404];
  for (int i = threadIdx.x; i < 2 * 16 * 404; i += 64 * NW) (&tile[0][0])[i] = 1e-3f * (i & 255);
  const int lane = threadIdx.x & 63, g = threadIdx.x >> 6;
  if constexpr (!REAL)
    for (int i = threadIdx.x; i < MT * 32 * 64; i += 64 * NW) (&actl[0][0])[i] = f32x4{1e-3f * i, 0.5f, 1.f, -2.f};
  __syncthreads();
  f32x4 acc[MT][TPW];
#pragma unroll
  for (int m = 0; m < MT; ++m)
#pragma unroll
    for (int j = 0; j < TPW; ++j) acc[m][j] = f32x4{0, 0, 0, 0};
  for (int L = 0; L < layers; ++L) {
    int soff[TPW];
#pragma unroll
    for (int j = 0; j < TPW; ++j) {
      int t = g + NW * j;
      t = t < NT_ ? t : NT_ - 1;
      soff[j] = __builtin_amdgcn_readfirstlane(t * NC * 1024);
    }
    const __amdgpu_buffer_rsrc_t rsrc =
        __builtin_amdgcn_make_buffer_rsrc((void*)(w + (size_t)L * NT_ * NC * 64), (short)0, NT_ * NC * 1024, 0x00020000);
    const int n = NC;
    auto chunk = [n](int i) { return i < n ? i : n - 1; };
    auto LOAD = [&](f32x4 (&b)[TPW], int c) {
#pragma unroll
      for (int j = 0; j < TPW; ++j) {
        if constexpr (LD)
          b[j] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rsrc, lane * 16, soff[j] + c * 1024, 0));
        else
          b[j] = f32x4{0.01f * j, 0.02f * lane, 0.03f, 0.04f};
      }
    };
    f32x4 b0[TPW], b1[TPW], b2[TPW], b3[TPW];
    f32x4 a0[MT], a1[MT], a2[MT], a3[MT];
    LOAD(b0, chunk(0));
    LOAD(b1, chunk(1));
#pragma unroll
    for (int m = 0; m < MT; ++m) {
      a0[m] = REAL ? *reinterpret_cast<const f32x4*>(&tile[0][(lane & 15) * 404 + 4 * (lane >> 4)]) : actl[m][(chunk(0) & 31) * 64 + lane];
      a1[m] = REAL ? *reinterpret_cast<const f32x4*>(&tile[0][(lane & 15) * 404 + 4 * (lane >> 4) + 16]) : actl[m][(chunk(1) & 31) * 64 + lane];
    }
#define STEP(X, AX, Z, AZ, i)                                                        \
  {                                                                                  \
    _Pragma("unroll") for (int m = 0; m < MT; ++m) AZ[m] = !AL ? AX[m] : (REAL ? *reinterpret_cast<const f32x4*>(&tile[L & 1][(lane & 15) * 404 + 4 * (lane >> 4) + 16 * chunk((i) + NS - 1)]) : actl[m][(chunk((i) + NS - 1) & 31) * 64 + lane]); \
    LOAD(Z, chunk((i) + NS - 1));                                                       \
    _Pragma("unroll") for (int s = 0; s < 4; ++s)                                    \
    _Pragma("unroll") for (int m = 0; m < MT; ++m)                                   \
    _Pragma("unroll") for (int j = 0; j < TPW; ++j)                                  \
      acc[m][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(AX[m][s], X[j][s], acc[m][j], 0, 0, 0); \
    if constexpr (IL == 0) {                                                         \
      __builtin_amdgcn_sched_group_barrier(0x100, MT, 0);                            \
      for (int q = 0; q < TPW; ++q) {                                                \
        __builtin_amdgcn_sched_group_barrier(0x008, 2 * MT, 0);                      \
        __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);                           \
      }                                                                              \
      __builtin_amdgcn_sched_group_barrier(0x008, 2 * MT * TPW, 0);                  \
    } else if constexpr (IL == 1) {                                                  \
      __builtin_amdgcn_sched_group_barrier(0x100, MT, 0);                            \
      for (int q = 0; q < TPW; ++q) {                                                \
        __builtin_amdgcn_sched_group_barrier(0x008, 4 * MT, 0);                      \
        __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);                           \
      }                                                                              \
      __builtin_amdgcn_sched_group_barrier(0x008, 2 * MT * TPW, 0);                  \
    } else if constexpr (IL == 2) {                                                  \
      __builtin_amdgcn_sched_group_barrier(0x100, MT, 0);                            \
      __builtin_amdgcn_sched_group_barrier(0x020, TPW, 0);                           \
      __builtin_amdgcn_sched_group_barrier(0x008, 4 * MT * TPW, 0);                  \
    } else {                                                                         \
      __builtin_amdgcn_sched_group_barrier(0x008, 2 * MT, 0);                        \
      __builtin_amdgcn_sched_group_barrier(0x100, MT, 0);                            \
      for (int q = 0; q < TPW; ++q) {                                                \
        __builtin_amdgcn_sched_group_barrier(0x008, 1 * MT, 0);                      \
        __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);                           \
      }                                                                              \
      __builtin_amdgcn_sched_group_barrier(0x008, 2 * MT * TPW, 0);                  \
    }                                                                                \
    __builtin_amdgcn_sched_barrier(0);                                               \
  }
    int i = 0;
    if constexpr (NS == 3) {
      for (; i + 3 <= n; i += 3) {
        STEP(b0, a0, b2, a2, i);
        STEP(b1, a1, b0, a0, i + 1);
        STEP(b2, a2, b1, a1, i + 2);
      }
      if (i < n) STEP(b0, a0, b2, a2, i);
      if (i + 1 < n) STEP(b1, a1, b0, a0, i + 1);
    } else {
      LOAD(b2, chunk(2));
#pragma unroll
      for (int m = 0; m < MT; ++m) a2[m] = actl[m][(chunk(2) & 31) * 64 + lane];
      for (; i + 4 <= n; i += 4) {
        STEP(b0, a0, b3, a3, i);
        STEP(b1, a1, b0, a0, i + 1);
        STEP(b2, a2, b1, a1, i + 2);
        STEP(b3, a3, b2, a2, i + 3);
      }
      if (i < n) STEP(b0, a0, b3, a3, i);
      if (i + 1 < n) STEP(b1, a1, b0, a0, i + 1);
      if (i + 2 < n) STEP(b2, a2, b1, a1, i + 2);
    }
#undef STEP
    if constexpr (REAL) {
      // epilogue like the forward's: bias + ReLU, outputs to the other tile, barrier
#pragma unroll
      for (int j = 0; j < TPW; ++j) {
        const int n = (g + NW * j) * 16 + (lane & 15);
#pragma unroll
        for (int m = 0; m < MT; ++m) {
#pragma unroll
          for (int r = 0; r < 4; ++r) tile[(L + 1) & 1][((lane >> 4) * 4 + r) * 404 + n] = fmaxf(acc[m][j][r] + 0.01f, 0.f);
          acc[m][j] = f32x4{0, 0, 0, 0};
        }
      }
    }
    __syncthreads();
  }
  float s = 0.f;
#pragma unroll
  for (int m = 0; m < MT; ++m)
#pragma unroll
    for (int j = 0; j < TPW; ++j) s += acc[m][j][0] + acc[m][j][1] + acc[m][j][2] + acc[m][j][3];
  if (s == 12345.678f) out[threadIdx.x] = s;
}

template <int TPW, int MT, int NW = 4, bool LD = true, bool AL = true, int NS = 3, bool REAL = false, int IL = 0>
void run(const char* name, const f32x4* w, int grid, float* out, hipStream_t* st, int nst, size_t pad = 0,
         unsigned* cu = nullptr) {
  const int NT_ = NW * TPW, NC = 25, layers = 3;
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  if (pad) CHECK(hipFuncSetAttribute(reinterpret_cast<const void*>(kern<TPW, MT, NW, LD, AL, NS, REAL, IL>),
                                     hipFuncAttributeMaxDynamicSharedMemorySize, (int)pad));
  for (int r = 0; r < 3; ++r) hipLaunchKernelGGL((kern<TPW, MT, NW, LD, AL, NS, REAL, IL>), dim3(grid), dim3(64 * NW), pad, st[0], w, NT_, NC, layers, out, nullptr);
  if (cu) {  // placement of one launch on an idle GPU: distinct CUs used
    CHECK(hipDeviceSynchronize());
    hipLaunchKernelGGL((kern<TPW, MT, NW, LD, AL, NS, REAL, IL>), dim3(grid), dim3(64 * NW), pad, st[0], w, NT_, NC, layers, out, cu);
    CHECK(hipDeviceSynchronize());
    unsigned h[4096];
    CHECK(hipMemcpy(h, cu, grid * sizeof(unsigned), hipMemcpyDeviceToHost));
    int distinct = 0, maxper = 0;
    for (int i = 0; i < grid; ++i) {
      int c = 0, first = 1;
      for (int j = 0; j < grid; ++j) { if (h[j] == h[i]) { ++c; if (j < i) first = 0; } }
      distinct += first; maxper = c > maxper ? c : maxper;
    }
    printf("  placement of one launch (grid %d, pad %zu): %d distinct CUs, at most %d WGs on one CU\n", grid, pad, distinct, maxper);
  }
  CHECK(hipDeviceSynchronize());
  const int reps = 100;
  CHECK(hipEventRecord(e0, 0));
  for (int r = 0; r < reps; ++r)
    hipLaunchKernelGGL((kern<TPW, MT, NW, LD, AL, NS, REAL, IL>), dim3(grid), dim3(64 * NW), pad, st[r % nst], w, NT_, NC, layers, out, nullptr);
  for (int k = 0; k < nst; ++k) {
    hipEvent_t ev;
    CHECK(hipEventCreate(&ev));
    CHECK(hipEventRecord(ev, st[k]));
    CHECK(hipStreamWaitEvent(0, ev, 0));
  }
  CHECK(hipEventRecord(e1, 0));
  CHECK(hipEventSynchronize(e1));
  float ms;
  CHECK(hipEventElapsedTime(&ms, e0, e1));
  const double us = ms * 1e3 / reps;
  const double mfma = (double)layers * NC * TPW * NW * 4 * MT * grid;
  const double samples = 16.0 * MT * grid;
  printf("%-40s grid %4d streams %d: %7.2f us/launch  %6.1f TFLOP/s  %6.2f us per 4096 samples\n", name, grid, nst, us,
         mfma * 2048 / (us * 1e6), us * 4096.0 / samples);
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
  for (int k = 0; k < 4; ++k) CHECK(hipStreamCreate(&st[k]));
  unsigned* cu;
  CHECK(hipMalloc(&cu, 4096 * sizeof(unsigned)));
  run<3, 1, 8, true, true, 3, true, 0>("warm-up", w, 256, out, st, 2);
  // streams with CU masks: A / B halves of the chip, as interleaved bits (even / odd CU ids) or as low / high ids
  hipStream_t ms[2][4];
  for (int mode = 0; mode < 2; ++mode)
    for (int k = 0; k < 4; ++k) {
      uint32_t mask[8];
      for (int i = 0; i < 8; ++i) {
        if (mode == 0) mask[i] = (k & 1) ? 0xAAAAAAAAu : 0x55555555u;
        else mask[i] = ((i < 4) == ((k & 1) == 0)) ? 0xFFFFFFFFu : 0u;
      }
      CHECK(hipExtStreamCreateWithCUMask(&ms[mode][k], 8, mask));
    }
  for (int rep = 0; rep < 2; ++rep) {
    run<3, 1, 8, true, true, 3, true, 0>("MT1 TPW3 8w real (forward today)", w, 256, out, st, 2);
    run<3, 2, 8, true, true, 3, true, 0>("MT2 grid 256, 2 streams (ceiling)", w, 256, out, st, 2);
    run<3, 2, 8, true, true, 3, true, 0>("MT2 grid 128, 4 streams", w, 128, out, st, 4);
    run<3, 2, 8, true, true, 3, true, 0>("MT2 grid 128, 4 masked streams even/odd", w, 128, out, ms[0], 4, 0, cu);
    run<3, 2, 8, true, true, 3, true, 0>("MT2 grid 128, 4 masked streams lo/hi", w, 128, out, ms[1], 4, 0, cu);
    run<3, 2, 8, true, true, 3, true, 0>("MT2 grid 128, 2 masked streams even/odd", w, 128, out, ms[0], 2);
    run<3, 1, 8, true, true, 3, true, 0>("MT1 grid 256, 4 masked streams even/odd", w, 256, out, ms[0], 4);
  }
  return 0;
}
