// dfwfm_metrics.hip -- the evaluation metrics of eval_by_batch on the device (reference
// model/DeepFMs.py:777-800: sklearn roc_auc_score, precision_recall_curve + auc, log_loss, RCE, CTR).
//
// pred = sigmoid(logit) in f32 (torch.sigmoid), widened to double as the reference's y_pred.  One
// descending radix sort of (pred, label); the distinct predictions form tie groups (run-length
// encode + per-group positive counts); exclusive scans give each group's rank start and positives
// above it.  Then, per group g with n_g samples, p_g positives, P_above positives ranked higher:
//   ROC AUC   = sum_g (n_g - p_g) * (P_above + p_g / 2) / (P * N)     (Mann-Whitney with ties = the
//               trapezoid under sklearn's ROC, which has one point per distinct threshold)
//   PR AUC    = trapezoid over sklearn's PR curve: (recall 0, precision 1), then one point per
//               distinct threshold from the highest: recall = TP/P, precision = TP/(TP+FP)
//   log_loss  = mean of -[y log q + (1-y) log(1-q)], q = [1-p, p] renormalised, clipped to
//               [eps, 1-eps] (double eps), as sklearn 1.7
//   RCE       = (1 - log_loss / log_loss(constant CTR)) * 100
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>
#include <math.h>
#include <stdint.h>

#include "dfwfm_internal.h"

namespace dfwfm {

namespace {

constexpr double kEps = 2.220446049250313e-16;  // np.finfo(np.float64).eps

__device__ __forceinline__ double clipped_ll(double p, int y) {
  // sklearn: y_pred = [1 - p, p] / row sum, clipped; loss = -xlogy(onehot, y_pred)
  double a = 1.0 - p, b = p;
  const double s = a + b;
  a /= s;
  b /= s;
  a = fmin(fmax(a, kEps), 1.0 - kEps);
  b = fmin(fmax(b, kEps), 1.0 - kEps);
  return y ? -log(b) : -log(a);
}

__device__ __forceinline__ double block_sum(double v, double* sh) {
  for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o);
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) sh[w] = v;
  __syncthreads();
  double t = 0.0;
  if (threadIdx.x == 0)
    for (int i = 0; i < (int)(blockDim.x >> 6); ++i) t += sh[i];
  __syncthreads();
  return t;
}

// keys = bits of sigmoid(z) (non-negative floats order like their bits), vals = label; log-loss and
// positive-count partial sums
__global__ void __launch_bounds__(256) metrics_prep_kernel(const float* __restrict__ z, const float* __restrict__ y,
                                                           int64_t n, uint32_t* __restrict__ keys,
                                                           int32_t* __restrict__ vals, double* __restrict__ acc) {
  __shared__ double sh[4];
  double ll = 0.0, pos = 0.0;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    const float p = 1.f / (1.f + expf(-z[i]));
    const int lab = y[i] > 0.5f ? 1 : 0;
    keys[i] = __float_as_uint(p);
    vals[i] = lab;
    ll += clipped_ll((double)p, lab);
    pos += lab;
  }
  ll = block_sum(ll, sh);
  pos = block_sum(pos, sh);
  if (threadIdx.x == 0) {
    atomicAdd(acc + 0, ll);
    atomicAdd(acc + 1, pos);
  }
}

// per tie group (descending prediction): ROC and PR contributions
__global__ void __launch_bounds__(256) metrics_groups_kernel(const int32_t* __restrict__ cnt,
                                                             const int32_t* __restrict__ gpos,
                                                             const int64_t* __restrict__ start,
                                                             const int64_t* __restrict__ pos_above,
                                                             const int32_t* __restrict__ n_groups,
                                                             double* __restrict__ acc) {
  __shared__ double sh[4];
  const int64_t G = *n_groups;
  const double P = acc[1];  // positives, summed by metrics_prep_kernel
  double roc = 0.0, pr = 0.0;
  for (int64_t g = (int64_t)blockIdx.x * 256 + threadIdx.x; g < G; g += (int64_t)gridDim.x * 256) {
    const double ng = cnt[g], pg = gpos[g], pa = (double)pos_above[g], st = (double)start[g];
    roc += (ng - pg) * (pa + 0.5 * pg);
    const double r0 = P > 0 ? pa / P : 1.0, r1 = P > 0 ? (pa + pg) / P : 1.0;
    const double p0 = g == 0 ? 1.0 : pa / st;
    const double p1 = (pa + pg) / (st + ng);
    pr += (r1 - r0) * (p0 + p1) * 0.5;
  }
  roc = block_sum(roc, sh);
  pr = block_sum(pr, sh);
  if (threadIdx.x == 0) {
    atomicAdd(acc + 2, roc);
    atomicAdd(acc + 3, pr);
  }
}

// out = {auc, prauc, log_loss, rce, ctr, positives, n, groups}
__global__ void metrics_final_kernel(const double* __restrict__ acc, const int32_t* __restrict__ n_groups, int64_t n,
                                     double* __restrict__ out) {
  const double P = acc[1], N = (double)n - P;
  const double ll = acc[0] / (double)n;
  const double c = P / (double)n;
  double straw = 0.0;  // log_loss(gt, [ctr] * n): the same per-row formula, closed form
  if (P > 0) straw += P * clipped_ll(c, 1);
  if (N > 0) straw += N * clipped_ll(c, 0);
  straw /= (double)n;
  out[0] = (P > 0 && N > 0) ? acc[2] / (P * N) : nan("");
  out[1] = acc[3];
  out[2] = ll;
  out[3] = (1.0 - ll / straw) * 100.0;
  out[4] = c;
  out[5] = P;
  out[6] = (double)n;
  out[7] = (double)*n_groups;
}

size_t align256(size_t x) { return (x + 255) & ~(size_t)255; }

struct MetricsWs {
  uint32_t *k0, *k1;
  int32_t *v0, *v1;
  uint32_t* ukeys;
  int32_t *cnt, *gpos, *ngroups, *ngroups2;
  int64_t *start, *pos_above, *cnt64, *gpos64;
  double* acc;
  void* temp;
  size_t temp_bytes;
  size_t total;
};

size_t cub_temp_bytes(int n) {
  size_t a = 0, b = 0, c = 0, d = 0;
  (void)hipcub::DeviceRadixSort::SortPairsDescending(nullptr, a, (const uint32_t*)nullptr, (uint32_t*)nullptr,
                                                      (const int32_t*)nullptr, (int32_t*)nullptr, n, 0, 32);
  (void)hipcub::DeviceRunLengthEncode::Encode(nullptr, b, (const uint32_t*)nullptr, (uint32_t*)nullptr,
                                              (int32_t*)nullptr, (int32_t*)nullptr, n);
  (void)hipcub::DeviceReduce::ReduceByKey(nullptr, c, (const uint32_t*)nullptr, (uint32_t*)nullptr,
                                          (const int32_t*)nullptr, (int32_t*)nullptr, (int32_t*)nullptr,
                                          hipcub::Sum(), n);
  (void)hipcub::DeviceScan::ExclusiveSum(nullptr, d, (const int64_t*)nullptr, (int64_t*)nullptr, n);
  size_t m = a > b ? a : b;
  m = m > c ? m : c;
  return m > d ? m : d;
}

MetricsWs carve(void* base, int64_t n) {
  MetricsWs w;
  char* p = reinterpret_cast<char*>(base);
  size_t o = 0;
  auto take = [&](size_t bytes) {
    void* r = p + o;
    o += align256(bytes);
    return r;
  };
  w.k0 = (uint32_t*)take(n * 4);
  w.k1 = (uint32_t*)take(n * 4);
  w.v0 = (int32_t*)take(n * 4);
  w.v1 = (int32_t*)take(n * 4);
  w.ukeys = (uint32_t*)take(n * 4);
  w.cnt = (int32_t*)take(n * 4);
  w.gpos = (int32_t*)take(n * 4);
  w.cnt64 = (int64_t*)take(n * 8);
  w.gpos64 = (int64_t*)take(n * 8);
  w.start = (int64_t*)take(n * 8);
  w.pos_above = (int64_t*)take(n * 8);
  w.ngroups = (int32_t*)take(4);
  w.ngroups2 = (int32_t*)take(4);
  w.acc = (double*)take(8 * 8);
  w.temp_bytes = cub_temp_bytes((int)n);
  w.temp = take(w.temp_bytes);
  w.total = o;
  return w;
}

__global__ void widen_kernel(const int32_t* __restrict__ a, const int32_t* __restrict__ b, int64_t* __restrict__ a64,
                             int64_t* __restrict__ b64, const int32_t* __restrict__ n_groups) {
  const int64_t G = *n_groups;
  for (int64_t g = (int64_t)blockIdx.x * 256 + threadIdx.x; g < G; g += (int64_t)gridDim.x * 256) {
    a64[g] = a[g];
    b64[g] = b[g];
  }
}

}  // namespace

size_t metrics_workspace_bytes(int64_t n) {
  if (n <= 0) n = 1;
  return carve(nullptr, n).total + 256;
}

// out: 8 doubles (device)
hipError_t launch_metrics(const float* z, const float* y, int64_t n, double* out, void* ws, size_t ws_bytes,
                          hipStream_t s) {
  if (n <= 0 || n > 0x7fffffff) return hipErrorInvalidValue;
  if (ws_bytes < metrics_workspace_bytes(n)) return hipErrorInvalidValue;
  void* base = reinterpret_cast<void*>((reinterpret_cast<uintptr_t>(ws) + 255) & ~(uintptr_t)255);
  MetricsWs w = carve(base, n);
  hipError_t e = hipMemsetAsync(w.acc, 0, 8 * sizeof(double), s);
  if (e != hipSuccess) return e;
  const unsigned grid = (unsigned)((n + 255) / 256 < 2048 ? (n + 255) / 256 : 2048);
  hipLaunchKernelGGL(metrics_prep_kernel, dim3(grid), dim3(256), 0, s, z, y, n, w.k0, w.v0, w.acc);
  if ((e = hipGetLastError()) != hipSuccess) return e;
  const int N = (int)n;
  size_t tb = w.temp_bytes;
  e = hipcub::DeviceRadixSort::SortPairsDescending(w.temp, tb, w.k0, w.k1, w.v0, w.v1, N, 0, 32, s);
  if (e != hipSuccess) return e;
  tb = w.temp_bytes;
  e = hipcub::DeviceRunLengthEncode::Encode(w.temp, tb, w.k1, w.ukeys, w.cnt, w.ngroups, N, s);
  if (e != hipSuccess) return e;
  tb = w.temp_bytes;
  e = hipcub::DeviceReduce::ReduceByKey(w.temp, tb, w.k1, w.ukeys, w.v1, w.gpos, w.ngroups2, hipcub::Sum(), N, s);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(widen_kernel, dim3(grid), dim3(256), 0, s, w.cnt, w.gpos, w.cnt64, w.gpos64, w.ngroups);
  if ((e = hipGetLastError()) != hipSuccess) return e;
  // scans over n entries (groups past the run count hold garbage and are never read)
  tb = w.temp_bytes;
  e = hipcub::DeviceScan::ExclusiveSum(w.temp, tb, w.cnt64, w.start, N, s);
  if (e != hipSuccess) return e;
  tb = w.temp_bytes;
  e = hipcub::DeviceScan::ExclusiveSum(w.temp, tb, w.gpos64, w.pos_above, N, s);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(metrics_groups_kernel, dim3(grid), dim3(256), 0, s, w.cnt, w.gpos, w.start, w.pos_above,
                     w.ngroups, w.acc);
  if ((e = hipGetLastError()) != hipSuccess) return e;
  hipLaunchKernelGGL(metrics_final_kernel, dim3(1), dim3(1), 0, s, w.acc, w.ngroups, n, out);
  return hipGetLastError();
}

}  // namespace dfwfm
