// ubench_stream.hip -- how fast can one workgroup per CU stream the packed MLP weights from L2?
// Mirrors the fused forward's weight stream: 1.9 MiB of [tile][chunk][64 lanes] float4 per
// workgroup, every workgroup reading the same bytes (so the XCD L2 serves them), TPW tiles per
// wave, three register sets in flight.  Variants: plain vs nt loads, 4 vs 8 waves per CU, with or
// without the 16x16x4 f32 MFMAs the real loop issues.  Prints GB/s per CU and TFLOP/s.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

typedef float f32x4 __attribute__((ext_vector_type(4)));
#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

template <int TPW, bool NT>
__device__ __forceinline__ void load_set(f32x4 (&b)[TPW], const f32x4* const (&wp)[TPW], int c) {
#pragma unroll
  for (int j = 0; j < TPW; ++j) {
    if constexpr (NT) b[j] = __builtin_nontemporal_load(wp[j] + (size_t)c * 64);
    else b[j] = wp[j][(size_t)c * 64];
  }
}

template <int TPW>
__device__ __forceinline__ void load_set_buf(f32x4 (&b)[TPW], __amdgpu_buffer_rsrc_t rsrc, const int (&soff)[TPW], int voff) {
#pragma unroll
  for (int j = 0; j < TPW; ++j) {
    auto v = __builtin_amdgcn_raw_buffer_load_b128(rsrc, voff, soff[j], 0);
    b[j] = __builtin_bit_cast(f32x4, v);
  }
}

template <int TPW, bool MFMA>
__device__ __forceinline__ void use(f32x4 (&acc)[TPW], const f32x4& a, const f32x4 (&b)[TPW]) {
#pragma unroll
  for (int j = 0; j < TPW; ++j) {
    if constexpr (MFMA) {
      acc[j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a.x, b[j].x, acc[j], 0, 0, 0);
      acc[j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a.y, b[j].y, acc[j], 0, 0, 0);
      acc[j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a.z, b[j].z, acc[j], 0, 0, 0);
      acc[j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a.w, b[j].w, acc[j], 0, 0, 0);
    } else {
      acc[j] += b[j];
    }
  }
}

// waves = 4*KS; wave w streams tiles of group (w & 3), chunks (w >> 2) + KS*i
template <int TPW, int KS, bool NT, bool MFMA, bool BUF = false, bool IL = false, int MODE = 0>
__global__ void __launch_bounds__(256 * KS) stream(const f32x4* __restrict__ w, int NT_, int NC, int layers, float* out) {
  __shared__ f32x4 actl[64 * 32];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, g = wave & 3, kh = wave >> 2;
  for (int i = threadIdx.x; i < 64 * 32; i += 256 * KS) actl[i] = f32x4{1e-3f * i, 0.f, 1.f, 2.f};
  __syncthreads();
  f32x4 acc[TPW];
#pragma unroll
  for (int j = 0; j < TPW; ++j) acc[j] = f32x4{0, 0, 0, 0};
  for (int L = 0; L < layers; ++L) {
    const f32x4* wp[TPW];
    int soff[TPW];
#pragma unroll
    for (int j = 0; j < TPW; ++j) {
      int t = g + 4 * j;
      t = t < NT_ ? t : NT_ - 1;
      wp[j] = w + ((size_t)L * NT_ * NC + (size_t)t * NC) * 64 + lane;
      soff[j] = __builtin_amdgcn_readfirstlane(t * NC * 1024);
    }
    const __amdgpu_buffer_rsrc_t rsrc =
        __builtin_amdgcn_make_buffer_rsrc((void*)(w + (size_t)L * NT_ * NC * 64), (short)0, NT_ * NC * 1024, 0x00020000);
    const int n = (NC - kh + KS - 1) / KS;
    auto chunk = [n, kh](int i) { return kh + KS * (i < n ? i : n - 1); };
    auto LOAD = [&](f32x4 (&b)[TPW], int c) {
      if constexpr (BUF) load_set_buf<TPW>(b, rsrc, soff, lane * 16 + c * 1024);
      else load_set<TPW, NT>(b, wp, c);
    };
    f32x4 b0[TPW], b1[TPW], b2[TPW];
    LOAD(b0, chunk(0));
    LOAD(b1, chunk(1));
    f32x4 a = actl[(chunk(0) & 31) * 64 + lane];
#define STEP(X, Z, i)                                                 \
  {                                                                   \
    f32x4 an = a;                                                     \
    if constexpr (MODE == 0) a = actl[(chunk(i) & 31) * 64 + lane];   \
    if constexpr (MODE == 1) an = actl[(chunk((i) + 1) & 31) * 64 + lane]; \
    if constexpr (MODE != 2) LOAD(Z, chunk((i) + 2));                 \
    if constexpr (!IL) __builtin_amdgcn_sched_barrier(0);             \
    use<TPW, MFMA>(acc, a, X);                                        \
    if constexpr (IL && MODE != 2) {                                  \
      for (int q = 0; q < TPW; ++q) {                                 \
        __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);            \
        __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);            \
      }                                                               \
      __builtin_amdgcn_sched_group_barrier(0x008, 2 * TPW, 0);        \
    }                                                                 \
    __builtin_amdgcn_sched_barrier(0);                                \
    if constexpr (MODE == 1) a = an;                                  \
  }
    int i = 0;
    for (; i + 3 <= n; i += 3) {
      STEP(b0, b2, i);
      STEP(b1, b0, i + 1);
      STEP(b2, b1, i + 2);
    }
    if (i < n) STEP(b0, b2, i);
    if (i + 1 < n) STEP(b1, b0, i + 1);
#undef STEP
  }
  float s = 0.f;
#pragma unroll
  for (int j = 0; j < TPW; ++j) s += acc[j][0] + acc[j][1] + acc[j][2] + acc[j][3];
  if (s == 12345.678f) out[threadIdx.x] = s;  // keep the work live
}

template <int TPW, int KS, bool NT, bool MFMA, bool BUF = false, bool IL = false, int MODE = 0>
void run(const char* name, const f32x4* w, int NT_, int NC, int layers, int grid, float* out) {
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  for (int r = 0; r < 3; ++r) hipLaunchKernelGGL((stream<TPW, KS, NT, MFMA, BUF, IL, MODE>), dim3(grid), dim3(256 * KS), 0, 0, w, NT_, NC, layers, out);
  CHECK(hipDeviceSynchronize());
  const int reps = 50;
  CHECK(hipEventRecord(e0));
  for (int r = 0; r < reps; ++r) hipLaunchKernelGGL((stream<TPW, KS, NT, MFMA, BUF, IL, MODE>), dim3(grid), dim3(256 * KS), 0, 0, w, NT_, NC, layers, out);
  CHECK(hipEventRecord(e1));
  CHECK(hipEventSynchronize(e1));
  float ms;
  CHECK(hipEventElapsedTime(&ms, e0, e1));
  const double us = ms * 1e3 / reps;
  const double bytes_per_wg = (double)layers * (4 * TPW) * NC * 1024.0;  // slots incl. clamped duplicates
  const double mfma = (double)layers * NC * TPW * 4 * 4 * grid;        // 16x16x4 instructions
  printf("%-34s %7.2f us  %6.1f GB/s/CU  %6.1f TFLOP/s\n", name, us, bytes_per_wg / (us * 1e3),
         MFMA ? mfma * 2048 / (us * 1e6) : 0.0);
}

int main() {
  const int NT_ = 25, NC = 25, layers = 3, grid = 256;
  const size_t n = (size_t)layers * NT_ * NC * 64;
  f32x4* w;
  float* out;
  CHECK(hipMalloc(&w, n * sizeof(f32x4)));
  CHECK(hipMalloc(&out, 4096 * sizeof(float)));
  CHECK(hipMemset(w, 0, n * sizeof(f32x4)));
  run<7, 1, false, true, true, true, 0>("buf+il  a-at-use", w, NT_, NC, layers, grid, out);
  run<7, 1, false, true, true, true, 1>("buf+il  a-prefetched", w, NT_, NC, layers, grid, out);
  run<7, 1, false, true, false, false, 2>("mfma only (ceiling) 4w", w, NT_, NC, layers, grid, out);
  run<7, 2, false, true, false, false, 2>("mfma only (ceiling) 8w", w, NT_, NC, layers, grid, out);
  run<7, 2, false, true, true, true, 1>("buf+il  a-prefetched 8 waves", w, NT_, NC, layers, grid, out);
  run<4, 1, false, true, true, true, 1>("buf+il  a-prefetched TPW4", w, NT_, NC, layers, grid, out);
  run<8, 1, false, true, true, true, 1>("buf+il  a-prefetched TPW8", w, 32, NC, layers, grid, out);
  return 0;
}
