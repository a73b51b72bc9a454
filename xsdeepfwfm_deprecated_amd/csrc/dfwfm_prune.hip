// dfwfm_prune.hip -- magnitude pruning of the training loop on the device (reference
// model/DeepFMs.py:647-673 with binary_search_threshold, :807-823).
//
// The reference finds each threshold by bisection on (0, 100): up to 101 rounds of
// `(abs(param) < mid).sum().item()` -- a full pass over the tensor and a host sync per round.  Here:
//   1. magnitudes -> uint32 keys (non-negative floats order like their bit patterns),
//   2. one radix sort (hipcub),
//   3. one thread replays the reference's bisection exactly (same doubles, same 101-round cap, the
//      comparison `|x| < mid` done in f32 as torch does for a float32 tensor and a Python float),
//      counting each round by a binary search on the sorted keys,
//   4. the mask is applied in place reading the threshold from device memory.
// No host synchronisation; thresholds stay on the device.
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>
#include <stdint.h>

#include "dfwfm_internal.h"

namespace dfwfm {

// magnitudes of every source element -> keys[off + i]; R sources use |(W[k][l] + W[l][k]) / 2|
__global__ void prune_keys_kernel(const PruneList L, uint32_t* __restrict__ keys) {
  const int s = blockIdx.y;
  if (s >= L.n) return;
  const PruneSrc src = L.s[s];
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < src.numel; i += (int64_t)gridDim.x * blockDim.x) {
    float v;
    if (src.sym_f > 0) {
      const int64_t k = i / src.sym_f, l = i - k * src.sym_f;
      v = __fmul_rn(0.5f, __fadd_rn(src.p[i], src.p[l * src.sym_f + k]));  // 0.5 * (W + W.t())
    } else {
      v = src.p[i];
    }
    keys[src.offset + i] = __float_as_uint(fabsf(v));
  }
}

// number of sorted keys strictly below the key of x (x >= 0)
__device__ __forceinline__ int64_t count_below(const uint32_t* __restrict__ sorted, int64_t n, float x) {
  const uint32_t key = __float_as_uint(x);
  int64_t lo = 0, hi = n;
  while (lo < hi) {
    const int64_t mid = (lo + hi) >> 1;
    if (sorted[mid] < key) lo = mid + 1;
    else hi = mid;
  }
  return lo;
}

// the reference's binary_search_threshold, verbatim in double, counts exact
__global__ void prune_bisect_kernel(const uint32_t* __restrict__ sorted, int64_t n, double total, double target,
                                    double* __restrict__ thr) {
  double l = 0.0, r = 1e2, mid = 0.0;
  int cnt = 0;
  while (l < r) {
    cnt += 1;
    mid = (l + r) / 2;
    const double items = (double)count_below(sorted, n, (float)mid);  // (abs(param) < mid) in f32
    const double rate = items / total;
    if (fabs(rate - target) < 0.0001) break;
    if (rate > target) r = mid;
    else l = mid;
    if (cnt > 100) break;
  }
  *thr = mid;
}

// param[i] = 0 where |param[i]| < thr (f32 compare)
__global__ void prune_apply_kernel(float* __restrict__ p, int64_t numel, const double* __restrict__ thr) {
  const float t = (float)*thr;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < numel; i += (int64_t)gridDim.x * blockDim.x)
    if (fabsf(p[i]) < t) p[i] = 0.f;
}

// R: the mask comes from |(W + W^T)/2| of the UNMODIFIED W, so the whole matrix goes through LDS first
// (one workgroup; F <= 64)
__global__ void prune_apply_sym_kernel(float* __restrict__ w, int F, const double* __restrict__ thr) {
  __shared__ float s[64 * 64];
  const float t = (float)*thr;
  for (int i = threadIdx.x; i < F * F; i += blockDim.x) s[i] = w[i];
  __syncthreads();
  for (int i = threadIdx.x; i < F * F; i += blockDim.x) {
    const int k = i / F, l = i - k * F;
    const float v = __fmul_rn(0.5f, __fadd_rn(s[i], s[l * F + k]));
    if (fabsf(v) < t) w[i] = 0.f;
  }
}

size_t prune_workspace_bytes(int64_t n) {
  size_t temp = 0;
  (void)hipcub::DeviceRadixSort::SortKeys(nullptr, temp, (const uint32_t*)nullptr, (uint32_t*)nullptr, (int)n, 0, 31);
  const size_t keys = ((size_t)n * sizeof(uint32_t) + 255) & ~(size_t)255;
  return 2 * keys + ((temp + 255) & ~(size_t)255);
}

hipError_t launch_prune_threshold(const PruneList& L, double target, double* d_thr, void* ws, size_t ws_bytes,
                                  hipStream_t s) {
  int64_t total = 0, maxn = 0;
  for (int i = 0; i < L.n; ++i) {
    total += L.s[i].numel;
    maxn = L.s[i].numel > maxn ? L.s[i].numel : maxn;
  }
  if (L.n <= 0 || L.n > kMaxPruneSrc || total <= 0 || total > 0x7fffffff) return hipErrorInvalidValue;
  if (ws_bytes < prune_workspace_bytes(total)) return hipErrorInvalidValue;
  char* base = reinterpret_cast<char*>(ws);
  const size_t keys = ((size_t)total * sizeof(uint32_t) + 255) & ~(size_t)255;
  uint32_t* k_in = reinterpret_cast<uint32_t*>(base);
  uint32_t* k_out = reinterpret_cast<uint32_t*>(base + keys);
  void* temp = base + 2 * keys;
  size_t temp_bytes = ws_bytes - 2 * keys;
  const unsigned gx = (unsigned)((maxn + 255) / 256 < 2048 ? (maxn + 255) / 256 : 2048);
  hipLaunchKernelGGL(prune_keys_kernel, dim3(gx, L.n), dim3(256), 0, s, L, k_in);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  e = hipcub::DeviceRadixSort::SortKeys(temp, temp_bytes, k_in, k_out, (int)total, 0, 31, s);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(prune_bisect_kernel, dim3(1), dim3(1), 0, s, k_out, total, (double)total, target, d_thr);
  return hipGetLastError();
}

hipError_t launch_prune_apply(float* p, int64_t numel, int sym_f, const double* d_thr, hipStream_t s) {
  if (numel <= 0) return hipSuccess;
  if (sym_f > 0) {
    if (sym_f > 64 || (int64_t)sym_f * sym_f != numel) return hipErrorInvalidValue;
    hipLaunchKernelGGL(prune_apply_sym_kernel, dim3(1), dim3(256), 0, s, p, sym_f, d_thr);
  } else {
    const unsigned g = (unsigned)((numel + 255) / 256 < 4096 ? (numel + 255) / 256 : 4096);
    hipLaunchKernelGGL(prune_apply_kernel, dim3(g), dim3(256), 0, s, p, numel, d_thr);
  }
  return hipGetLastError();
}

}  // namespace dfwfm
