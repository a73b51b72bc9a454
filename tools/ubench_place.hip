// ubench_place.hip -- placement of 32-sample forward tiles: a forward-shaped workgroup (a gather
// prologue of dependent Xi -> row loads into LDS, then a 3 x 25-chunk f32-MFMA MLP with the
// weight stream and bias/ReLU epilogue of the forward) with MT row tiles of 16 samples, one batch of
// 4096 samples per launch, launches round-robin over S streams.  The dynamic-LDS pad sets how many
// workgroups fit per CU.  Prints microseconds per 4096 samples.
//   hipcc --offload-arch=gfx950 -O3 tools/ubench_place.hip -o tools/ubench_place && ./tools/ubench_place
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

typedef float f32x4 __attribute__((ext_vector_type(4)));
#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

constexpr int SA = 404;

template <int TPW, int MT, int NW>
__global__ void __launch_bounds__(64 * NW) __attribute__((amdgpu_waves_per_eu(NW / 4 * 2)))
kern(const f32x4* __restrict__ w, const long* __restrict__ xi, const float* __restrict__ table, long nrows, float* out) {
  extern __shared__ __attribute__((aligned(16))) float tile[];  // [MT*16][SA], in place across layers
  const int lane = threadIdx.x & 63, g = threadIdx.x >> 6;
  constexpr int BM = 16 * MT, NTH = 64 * NW;
  // gather: BM samples x 26 rows of 40 B, all loads in flight before the LDS stores
  constexpr int RPT = (BM * 26 + NTH - 1) / NTH;
  long key[RPT];
#pragma unroll
  for (int k = 0; k < RPT; ++k) {
    const int r = threadIdx.x + k * NTH;
    key[k] = r < BM * 26 ? xi[((long)blockIdx.x * BM + r % BM) * 26 + r / BM] : 0;
  }
  float v[RPT][10];
#pragma unroll
  for (int k = 0; k < RPT; ++k)
#pragma unroll
    for (int d = 0; d < 10; ++d) v[k][d] = table[(key[k] % nrows) * 10 + d];
#pragma unroll
  for (int k = 0; k < RPT; ++k) {
    const int r = threadIdx.x + k * NTH;
    if (r < BM * 26)
#pragma unroll
      for (int d = 0; d < 10; ++d) tile[(r % BM) * SA + (r / BM) * 10 + d] = v[k][d];
  }
  for (int i = threadIdx.x; i < BM * 140; i += NTH) tile[(i / 140) * SA + 260 + i % 140] = 0.01f;
  __syncthreads();
  float dsum = 0.f;
  for (int L = 0; L < 3; ++L) {
    f32x4 acc[MT][TPW];
#pragma unroll
    for (int m = 0; m < MT; ++m)
#pragma unroll
      for (int j = 0; j < TPW; ++j) acc[m][j] = f32x4{0, 0, 0, 0};
    const int NT_ = NW * TPW, NC = 25;
    int soff[TPW];
#pragma unroll
    for (int j = 0; j < TPW; ++j) soff[j] = __builtin_amdgcn_readfirstlane((g + NW * j) * NC * 1024);
    const __amdgpu_buffer_rsrc_t rsrc =
        __builtin_amdgcn_make_buffer_rsrc((void*)(w + (size_t)L * NT_ * NC * 64), (short)0, NT_ * NC * 1024, 0x00020000);
    const int n = NC;
    auto chunk = [n](int i) { return i < n ? i : n - 1; };
    auto LOAD = [&](f32x4 (&b)[TPW], int c) {
#pragma unroll
      for (int j = 0; j < TPW; ++j)
        b[j] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rsrc, lane * 16, soff[j] + c * 1024, 0));
    };
    auto ALOAD = [&](f32x4 (&a)[MT], int c) {
#pragma unroll
      for (int m = 0; m < MT; ++m)
        a[m] = *reinterpret_cast<const f32x4*>(&tile[(m * 16 + (lane & 15)) * SA + 4 * (lane >> 4) + 16 * c]);
    };
    f32x4 b0[TPW], b1[TPW], b2[TPW];
    f32x4 a0[MT], a1[MT], a2[MT];
    LOAD(b0, chunk(0));
    LOAD(b1, chunk(1));
    ALOAD(a0, chunk(0));
    ALOAD(a1, chunk(1));
#define STEP(X, AX, Z, AZ, i)                                                        \
  {                                                                                  \
    ALOAD(AZ, chunk((i) + 2));                                                       \
    LOAD(Z, chunk((i) + 2));                                                         \
    _Pragma("unroll") for (int s = 0; s < 4; ++s)                                    \
    _Pragma("unroll") for (int m = 0; m < MT; ++m)                                   \
    _Pragma("unroll") for (int j = 0; j < TPW; ++j)                                  \
      acc[m][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(AX[m][s], X[j][s], acc[m][j], 0, 0, 0); \
    __builtin_amdgcn_sched_group_barrier(0x100, MT, 0);                              \
    for (int q = 0; q < TPW; ++q) {                                                  \
      __builtin_amdgcn_sched_group_barrier(0x008, 2 * MT, 0);                        \
      __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);                             \
    }                                                                                \
    __builtin_amdgcn_sched_group_barrier(0x008, 2 * MT * TPW, 0);                    \
    __builtin_amdgcn_sched_barrier(0);                                               \
  }
    int i = 0;
    for (; i + 3 <= n; i += 3) {
      STEP(b0, a0, b2, a2, i);
      STEP(b1, a1, b0, a0, i + 1);
      STEP(b2, a2, b1, a1, i + 2);
    }
    if (i < n) STEP(b0, a0, b2, a2, i);
    if (i + 1 < n) STEP(b1, a1, b0, a0, i + 1);
#undef STEP
    __syncthreads();  // every wave done reading the tile: the outputs overwrite it in place
#pragma unroll
    for (int m = 0; m < MT; ++m)
#pragma unroll
      for (int j = 0; j < TPW; ++j) {
        const int nn = (g + NW * j) * 16 + (lane & 15);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float x = fmaxf(acc[m][j][r] + 0.01f, 0.f);
          if (L < 2) tile[(m * 16 + (lane >> 4) * 4 + r) * SA + nn] = x;
          else dsum += x;
        }
      }
    __syncthreads();
  }
  if (dsum == 12345.678f) out[threadIdx.x] = dsum;
}

template <int TPW, int MT, int NW>
void run(const char* name, const f32x4* w, const long* xi, const float* table, long nrows, size_t lds, float* out,
         hipStream_t* st, int nst) {
  auto k = kern<TPW, MT, NW>;
  CHECK(hipFuncSetAttribute(reinterpret_cast<const void*>(k), hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  const int grid = 4096 / (16 * MT);
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  for (int r = 0; r < 400; ++r) hipLaunchKernelGGL(k, dim3(grid), dim3(64 * NW), lds, st[r % nst], w, xi, table, nrows, out);
  CHECK(hipDeviceSynchronize());
  const int reps = 400;
  CHECK(hipEventRecord(e0, 0));
  for (int k2 = 0; k2 < nst; ++k2) CHECK(hipStreamWaitEvent(st[k2], e0, 0));
  for (int r = 0; r < reps; ++r) hipLaunchKernelGGL(k, dim3(grid), dim3(64 * NW), lds, st[r % nst], w, xi, table, nrows, out);
  for (int k2 = 0; k2 < nst; ++k2) {
    hipEvent_t ev;
    CHECK(hipEventCreate(&ev));
    CHECK(hipEventRecord(ev, st[k2]));
    CHECK(hipStreamWaitEvent(0, ev, 0));
  }
  CHECK(hipEventRecord(e1, 0));
  CHECK(hipEventSynchronize(e1));
  float ms;
  CHECK(hipEventElapsedTime(&ms, e0, e1));
  const double us = ms * 1e3 / reps;
  printf("%-34s lds %6zu streams %d: %7.2f us per 4096 samples  %6.1f TFLOP/s (3x400x400 MLP)\n", name, lds, nst, us,
         4096.0 * 3 * 2 * 400 * 400 / (us * 1e6));
}

int main() {
  const size_t n = (size_t)3 * 32 * 25 * 64;
  f32x4* w;
  float* out;
  long* xi;
  float* table;
  const long nrows = 1326042;
  CHECK(hipMalloc(&w, n * sizeof(f32x4)));
  CHECK(hipMalloc(&out, 4096 * sizeof(float)));
  CHECK(hipMalloc(&xi, 8 * 4096 * 26 * sizeof(long)));
  CHECK(hipMalloc(&table, nrows * 10 * sizeof(float)));
  float* h = (float*)malloc(n * sizeof(f32x4));
  srand(1);
  for (size_t i = 0; i < n * 4; ++i) h[i] = (rand() / (float)RAND_MAX - 0.5f) * 0.1f;
  CHECK(hipMemcpy(w, h, n * sizeof(f32x4), hipMemcpyHostToDevice));
  long* hx = (long*)malloc(4096 * 26 * sizeof(long));
  for (int i = 0; i < 4096 * 26; ++i) hx[i] = ((long)rand() * 7919 + rand()) % nrows;
  CHECK(hipMemcpy(xi, hx, 4096 * 26 * sizeof(long), hipMemcpyHostToDevice));
  CHECK(hipMemset(table, 0, nrows * 10 * sizeof(float)));
  hipStream_t st[4];
  for (int k = 0; k < 4; ++k) CHECK(hipStreamCreate(&st[k]));
  const size_t t16 = 16 * SA * 4, t32 = 32 * SA * 4;
  for (int rep = 0; rep < 2; ++rep) {
    run<3, 1, 8>("MT1 8w (16-sample tiles)", w, xi, table, nrows, t16 + 10000, out, st, 2);
    run<3, 1, 8>("MT1 8w (16-sample tiles)", w, xi, table, nrows, t16 + 10000, out, st, 3);
    run<3, 2, 8>("MT2 8w 1/CU", w, xi, table, nrows, 100000, out, st, 1);
    run<3, 2, 8>("MT2 8w 1/CU", w, xi, table, nrows, 100000, out, st, 2);
    run<3, 2, 8>("MT2 8w 1/CU", w, xi, table, nrows, 100000, out, st, 3);
    run<3, 2, 8>("MT2 8w 1/CU", w, xi, table, nrows, 100000, out, st, 4);
    run<3, 2, 8>("MT2 8w 2/CU", w, xi, table, nrows, t32 + 10000, out, st, 2);
    run<3, 2, 8>("MT2 8w 2/CU", w, xi, table, nrows, t32 + 10000, out, st, 3);
    run<3, 2, 8>("MT2 8w 2/CU", w, xi, table, nrows, t32 + 10000, out, st, 4);
  }
  return 0;
}
