// ubench_fwd2.hip -- which structural choice of the forward's MLP phase costs what.  A forward-shaped
// workgroup (16 samples: dependent Xi -> 26 row loads into LDS, then 3 MLP layers 400 wide on the real
// K loop of csrc/dfwfm_device.h), one batch of 4096 per launch, launches round-robin over S streams.
//   TAIL   : 0 = 24 output tiles (3 per wave), 1 = 25 tiles, the 25th split by K over the 8 waves (real)
//   TWOBUF : 0 = one activation tile, overwritten in place (barrier, epilogue, barrier, then the next
//            layer's loads); 1 = two tiles, next layer's weights preloaded before the barrier (real)
// Prints microseconds per 4096 samples and TFLOP/s counted for the real 400-wide MLP.
//   hipcc --offload-arch=gfx950 -O3 -I xsdeepfwfm_deprecated_amd/csrc tools/ubench_fwd2.hip -o tools/ubench_fwd2
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#include "dfwfm_device.h"

using namespace dfwfm;
#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

constexpr int SA = 404, NC = 25, NG = 8, TPW = 3;

template <bool TAIL, bool TWOBUF>
__global__ void __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(4)))
kern(const float4* __restrict__ w, int wbytes, const long* __restrict__ xi, const float* __restrict__ table, long nrows,
     float* out) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  float* bufX = smem;
  float* bufY = smem + 16 * SA;
  float* tailr = smem + (TWOBUF ? 32 : 16) * SA;
  const int tid = threadIdx.x, lane = tid & 63;
  const int g = __builtin_amdgcn_readfirstlane(tid >> 6);
  constexpr int NT = TAIL ? 25 : 24, TT = 24;
  constexpr int RPT = (16 * 26 + 511) / 512;
  long key[RPT];
#pragma unroll
  for (int k = 0; k < RPT; ++k) {
    const int r = tid + k * 512;
    key[k] = r < 16 * 26 ? xi[((long)blockIdx.x * 16 + (r & 15)) * 26 + (r >> 4)] : 0;
  }
  float v[RPT][10];
#pragma unroll
  for (int k = 0; k < RPT; ++k)
#pragma unroll
    for (int d = 0; d < 10; ++d) v[k][d] = table[(key[k] % nrows) * 10 + d];
  const __amdgpu_buffer_rsrc_t wr = __builtin_amdgcn_make_buffer_rsrc(const_cast<float4*>(w), (short)0, wbytes, 0x00020000);
  LayerStream<TPW, 1, NG> ls;
  TailStream<NG> ts;
  f32x4 wb0[TPW], wb1[TPW], wb2[TPW], tw[TailStream<NG>::C];
  ls.init(wr, 0, NC, NT, g, 0);
  ls.preload(wb0, wb1, lane * 16);
  if (TAIL) {
    ts.init(0, NC, TT, g);
    ts.load(wr, tw, lane * 16);
  }
#pragma unroll
  for (int k = 0; k < RPT; ++k) {
    const int r = tid + k * 512;
    if (r < 16 * 26)
#pragma unroll
      for (int d = 0; d < 10; ++d) bufX[(r & 15) * SA + (r >> 4) * 10 + d] = v[k][d];
  }
  for (int i = tid; i < 16 * 140; i += 512) bufX[(i / 140) * SA + 260 + i % 140] = 0.01f;
  __syncthreads();
  float dsum = 0.f;
  int loff = 0;
  for (int L = 0; L < 3; ++L) {
    const float* in = (TWOBUF && (L & 1)) ? bufY : bufX;
    float* o = TWOBUF ? ((L & 1) ? bufX : bufY) : bufX;
    if (!TWOBUF && L > 0) {
      ls.init(wr, loff, NC, NT, g, 0);
      ls.preload(wb0, wb1, lane * 16);
      if (TAIL) {
        ts.init(loff, NC, TT, g);
        ts.load(wr, tw, lane * 16);
      }
    }
    if (TAIL) reinterpret_cast<f32x4*>(tailr)[g * 64 + lane] = ts.mma(in, SA, tw, lane);
    f32x4 acc[TPW];
    mlp_k_loop<TPW, 1, NG>(acc, in, SA, ls, wb0, wb1, wb2, lane);
    if (!TWOBUF) __syncthreads();
#pragma unroll
    for (int j = 0; j < TPW; ++j) {
      const int n = (g + NG * j) * 16 + (lane & 15);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float x = relu_keep_nan(acc[j][r] + 0.01f);
        if (L < 2) o[((lane >> 4) * 4 + r) * SA + n] = x;
        else dsum += x;
      }
    }
    loff += NT * NC * 64;
    if (TWOBUF && L < 2) {
      ls.init(wr, loff, NC, NT, g, 0);
      ls.preload(wb0, wb1, lane * 16);
      if (TAIL) {
        ts.init(loff, NC, TT, g);
        ts.load(wr, tw, lane * 16);
      }
    }
    __syncthreads();
    if (TAIL) {
      if (g < 4) {
        const int n = TT * 16 + (lane & 15);
        const int rr = (lane >> 4) * 4 + g;
        float s = tailr[lane * 4 + g];
#pragma unroll
        for (int q = 1; q < NG; ++q) s += tailr[q * 256 + lane * 4 + g];
        const float x = relu_keep_nan(s + 0.01f);
        if (L < 2) o[rr * SA + n] = x;
        else dsum += x;
      }
      if (L < 2) __syncthreads();
    }
  }
  if (dsum == 12345.678f) out[tid] = dsum;
}

template <bool TAIL, bool TWOBUF>
void run(const char* name, const float4* w, int wbytes, const long* xi, const float* table, long nrows, float* out,
         hipStream_t* st, int nst) {
  auto k = kern<TAIL, TWOBUF>;
  const size_t lds = ((TWOBUF ? 32 : 16) * SA + 8 * 256) * 4 + (size_t)(getenv("PAD") ? atoi(getenv("PAD")) : 0);
  CHECK(hipFuncSetAttribute(reinterpret_cast<const void*>(k), hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  for (int r = 0; r < 600; ++r) hipLaunchKernelGGL(k, dim3(256), dim3(512), lds, st[r % nst], w, wbytes, xi + (r % 4) * 4096 * 26, table, nrows, out);
  CHECK(hipDeviceSynchronize());
  const int reps = 1000;
  CHECK(hipEventRecord(e0, 0));
  for (int k2 = 0; k2 < nst; ++k2) CHECK(hipStreamWaitEvent(st[k2], e0, 0));
  for (int r = 0; r < reps; ++r) hipLaunchKernelGGL(k, dim3(256), dim3(512), lds, st[r % nst], w, wbytes, xi + (r % 4) * 4096 * 26, table, nrows, out);
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
  printf("%-28s lds %6zu streams %d: %7.2f us per 4096  %6.1f TFLOP/s (400-wide)\n", name, lds, nst, us,
         4096.0 * 2 * (390 * 400 + 2 * 400 * 400 + 400) / (us * 1e6));
}

int main() {
  const size_t n = (size_t)3 * 25 * 25 * 64;
  float4* w;
  float* out;
  long* xi;
  float* table;
  const long nrows = 1326042;
  CHECK(hipMalloc(&w, n * sizeof(float4)));
  CHECK(hipMalloc(&out, 4096 * sizeof(float)));
  CHECK(hipMalloc(&xi, 4 * 4096 * 26 * sizeof(long)));
  CHECK(hipMalloc(&table, nrows * 10 * sizeof(float)));
  float* h = (float*)malloc(n * sizeof(float4));
  srand(1);
  for (size_t i = 0; i < n * 4; ++i) h[i] = (rand() / (float)RAND_MAX - 0.5f) * 0.1f;
  CHECK(hipMemcpy(w, h, n * sizeof(float4), hipMemcpyHostToDevice));
  long* hx = (long*)malloc(4 * 4096 * 26 * sizeof(long));
  for (int i = 0; i < 4 * 4096 * 26; ++i) hx[i] = ((long)rand() * 7919 + rand()) % nrows;
  CHECK(hipMemcpy(xi, hx, 4 * 4096 * 26 * sizeof(long), hipMemcpyHostToDevice));
  float* ht = (float*)malloc(nrows * 10 * sizeof(float));
  for (long i = 0; i < nrows * 10; ++i) ht[i] = (rand() / (float)RAND_MAX - 0.5f) * 0.02f;
  CHECK(hipMemcpy(table, ht, nrows * 10 * sizeof(float), hipMemcpyHostToDevice));
  hipStream_t st[4];
  for (int k = 0; k < 4; ++k) CHECK(hipStreamCreate(&st[k]));
  const int wb = (int)(n * sizeof(float4));
  for (int rep = 0; rep < 2; ++rep) {
    for (int s = 2; s <= 3; ++s) {
      run<false, false>("24 tiles, in place", w, wb, xi, table, nrows, out, st, s);
      run<false, true>("24 tiles, two buffers", w, wb, xi, table, nrows, out, st, s);
      run<true, false>("25 (tail), in place", w, wb, xi, table, nrows, out, st, s);
      run<true, true>("25 (tail), two buffers", w, wb, xi, table, nrows, out, st, s);
    }
  }
  return 0;
}
