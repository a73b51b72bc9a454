// dfwfm_metrics.hip -- the evaluation metrics of eval_by_batch on the device (reference
// model/DeepFMs.py:777-800: sklearn roc_auc_score, precision_recall_curve + auc, log_loss, RCE, CTR).
//
// pred = sigmoid(logit) in f32 (torch.sigmoid), widened to double as the reference's y_pred.  The (pred, label)
// pairs are ranked by a hand-written LSD radix sort (four stable 8-bit passes: per-tile digit histograms, one
// exclusive scan over (digit, tile), a stable scatter whose in-wave ranks come from ballots); the distinct
// predictions form tie groups: a scan of the labels gives the positives ranked above every position, a scan of the
// group-start flags lists where each group starts.  Then, per group g with n_g samples, p_g positives, P_above
// positives ranked higher:
//   ROC AUC   = sum_g (n_g - p_g) * (P_above + p_g / 2) / (P * N)     (Mann-Whitney with ties = the
//               trapezoid under sklearn's ROC, which has one point per distinct threshold)
//   PR AUC    = trapezoid over sklearn's PR curve: (recall 0, precision 1), then one point per
//               distinct threshold from the highest: recall = TP/P, precision = TP/(TP+FP)
//   log_loss  = mean of -[y log q + (1-y) log(1-q)], q = [1-p, p] renormalised, clipped to
//               [eps, 1-eps] (double eps), as sklearn 1.7
//   RCE       = (1 - log_loss / log_loss(constant CTR)) * 100
// Every sum is formed per tile and the tiles are added in tile order (no float atomics): the same bits each run.
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

#include "dfwfm_internal.h"

namespace dfwfm {

namespace {

constexpr double kEps = 2.220446049250313e-16;  // np.finfo(np.float64).eps
constexpr int kT = 256;                         // threads per workgroup
constexpr int kIPT = 16;                        // items per thread
constexpr int kTile = kT * kIPT;                // items per tile (workgroup)

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

// workgroup sum in a fixed order (lanes by a butterfly, then the four waves in wave order); thread 0 holds it
template <typename T>
__device__ __forceinline__ T block_sum(T v, T* sh) {
  for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o);
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) sh[w] = v;
  __syncthreads();
  T t = 0;
  if (threadIdx.x == 0)
    for (int i = 0; i < kT / 64; ++i) t += sh[i];
  __syncthreads();
  return t;
}

// keys = ~bits of sigmoid(z) (non-negative floats order like their bits; complemented: ascending = descending
// prediction), vals = label; per tile: log-loss and positive count
__global__ void __launch_bounds__(kT) metrics_prep_kernel(const float* __restrict__ z, const float* __restrict__ y,
                                                          int64_t n, uint32_t* __restrict__ keys,
                                                          int32_t* __restrict__ vals, double* __restrict__ part) {
  __shared__ double sh[4];
  double ll = 0.0, pos = 0.0;
  const int64_t i0 = (int64_t)blockIdx.x * kTile;
  for (int r = 0; r < kIPT; ++r) {
    const int64_t i = i0 + r * kT + threadIdx.x;
    if (i < n) {
      const float p = 1.f / (1.f + expf(-z[i]));
      const int lab = y[i] > 0.5f ? 1 : 0;
      keys[i] = ~__float_as_uint(p);
      vals[i] = lab;
      ll += clipped_ll((double)p, lab);
      pos += lab;
    }
  }
  ll = block_sum(ll, sh);
  pos = block_sum(pos, sh);
  if (threadIdx.x == 0) {
    part[2 * blockIdx.x] = ll;
    part[2 * blockIdx.x + 1] = pos;
  }
}

// ---- exclusive scans (int64 out) over n items of a source: tile sums, one workgroup scanning the tile sums, then
// each tile's own scan plus its offset
struct ScanSrc {
  const int32_t* a;      // mode 0: the int32 items
  const uint32_t* keys;  // mode 1: item i = 1 where a tie group starts (i == 0 or keys[i] != keys[i - 1])
  int mode;
};
__device__ __forceinline__ int32_t scan_item(const ScanSrc& s, int64_t i) {
  if (s.mode == 0) return s.a[i];
  return (i == 0 || s.keys[i] != s.keys[i - 1]) ? 1 : 0;
}

__global__ void __launch_bounds__(kT) scan_tiles_kernel(ScanSrc src, int64_t n, int64_t* __restrict__ tsum) {
  __shared__ int64_t sh[4];
  const int64_t i0 = (int64_t)blockIdx.x * kTile + (int64_t)threadIdx.x * kIPT;
  int64_t v = 0;
#pragma unroll
  for (int q = 0; q < kIPT; ++q)
    if (i0 + q < n) v += scan_item(src, i0 + q);
  v = block_sum(v, sh);
  if (threadIdx.x == 0) tsum[blockIdx.x] = v;
}

// one workgroup: tsum[0, nt) -> exclusive prefix in place, the total into *total
__global__ void __launch_bounds__(1024) scan_top_kernel(int64_t* __restrict__ tsum, int64_t nt,
                                                        int64_t* __restrict__ total) {
  __shared__ int64_t th[1024];
  const int tid = threadIdx.x;
  const int64_t per = (nt + 1023) / 1024;
  const int64_t lo = tid * per, hi = lo + per < nt ? lo + per : nt;
  int64_t s = 0;
  for (int64_t i = lo; i < hi; ++i) s += tsum[i];
  th[tid] = s;
  __syncthreads();
  for (int o = 1; o < 1024; o <<= 1) {  // inclusive Hillis-Steele over the threads' sums
    const int64_t x = tid >= o ? th[tid - o] : 0;
    __syncthreads();
    th[tid] += x;
    __syncthreads();
  }
  int64_t run = tid > 0 ? th[tid - 1] : 0;
  for (int64_t i = lo; i < hi; ++i) {
    const int64_t x = tsum[i];
    tsum[i] = run;
    run += x;
  }
  if (tid == 1023) *total = th[1023];
}

// the tile's exclusive scan (thread = kIPT consecutive items) + its offset: mode 0 writes out[i]; mode 1 (group
// starts) writes the position of every group start at its group index: gstart[prefix] = i
__global__ void __launch_bounds__(kT) scan_down_kernel(ScanSrc src, int64_t n, const int64_t* __restrict__ tsum,
                                                       int64_t* __restrict__ out) {
  __shared__ int64_t th[kT];
  const int tid = threadIdx.x;
  const int64_t i0 = (int64_t)blockIdx.x * kTile + (int64_t)tid * kIPT;
  int32_t x[kIPT];
  int64_t s = 0;
#pragma unroll
  for (int q = 0; q < kIPT; ++q) {
    x[q] = i0 + q < n ? scan_item(src, i0 + q) : 0;
    s += x[q];
  }
  th[tid] = s;
  __syncthreads();
  for (int o = 1; o < kT; o <<= 1) {
    const int64_t y = tid >= o ? th[tid - o] : 0;
    __syncthreads();
    th[tid] += y;
    __syncthreads();
  }
  int64_t run = tsum[blockIdx.x] + (tid > 0 ? th[tid - 1] : 0);
#pragma unroll
  for (int q = 0; q < kIPT; ++q) {
    if (i0 + q < n) {
      if (src.mode == 0) out[i0 + q] = run;
      else if (x[q]) out[run] = i0 + q;
    }
    run += x[q];
  }
}

// ---- radix sort pass (8 bits at `shift`): per-tile digit counts, digit-major [256][tiles]
__global__ void __launch_bounds__(kT) radix_hist_kernel(const uint32_t* __restrict__ keys, int64_t n, int shift,
                                                        int32_t* __restrict__ counts, int64_t ntiles) {
  __shared__ int32_t h[256];
  h[threadIdx.x] = 0;
  __syncthreads();
  const int64_t i0 = (int64_t)blockIdx.x * kTile;
  for (int r = 0; r < kIPT; ++r) {
    const int64_t i = i0 + r * kT + threadIdx.x;
    if (i < n) atomicAdd(&h[(keys[i] >> shift) & 255], 1);  // integer counts: order-free
  }
  __syncthreads();
  counts[(int64_t)threadIdx.x * ntiles + blockIdx.x] = h[threadIdx.x];
}

// stable scatter: the tile's items in index order (round r = items [r*256, r*256+256) of the tile, one per thread in
// thread order); an item's place = the digit's offset for this tile (scanned counts) + items of the same digit in
// earlier rounds + in earlier waves of this round + in earlier lanes of its wave (ballots over the digit's 8 bits)
__global__ void __launch_bounds__(kT) radix_scatter_kernel(const uint32_t* __restrict__ kin,
                                                           const int32_t* __restrict__ vin, int64_t n, int shift,
                                                           const int64_t* __restrict__ offs, int64_t ntiles,
                                                           uint32_t* __restrict__ kout, int32_t* __restrict__ vout) {
  __shared__ int64_t base[256];
  __shared__ int32_t run[256];
  __shared__ int32_t wcnt[4][256];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  base[tid] = offs[(int64_t)tid * ntiles + blockIdx.x];
  run[tid] = 0;
#pragma unroll
  for (int w = 0; w < 4; ++w) wcnt[w][tid] = 0;
  const uint64_t lt = lane ? (~0ull >> (64 - lane)) : 0ull;  // lanes below this one
  const int64_t i0 = (int64_t)blockIdx.x * kTile;
  __syncthreads();
  for (int r = 0; r < kIPT; ++r) {
    const int64_t i = i0 + r * kT + tid;
    const bool valid = i < n;
    const uint32_t k = valid ? kin[i] : 0u;
    const int32_t v = valid ? vin[i] : 0;
    const int d = (int)((k >> shift) & 255);
    uint64_t same = __ballot(valid);
#pragma unroll
    for (int b = 0; b < 8; ++b) {
      const uint64_t bb = __ballot((d >> b) & 1);
      same &= ((d >> b) & 1) ? bb : ~bb;
    }
    const int rank = __popcll(same & lt);
    if (valid && rank == 0) wcnt[wave][d] = __popcll(same);
    __syncthreads();
    if (valid) {
      int off = run[d] + rank;
      for (int w = 0; w < wave; ++w) off += wcnt[w][d];
      const int64_t pos = base[d] + off;
      kout[pos] = k;
      vout[pos] = v;
    }
    __syncthreads();
    run[tid] += ((wcnt[0][tid] + wcnt[1][tid]) + wcnt[2][tid]) + wcnt[3][tid];
#pragma unroll
    for (int w = 0; w < 4; ++w) wcnt[w][tid] = 0;
    __syncthreads();
  }
}

// per tie group (descending prediction): ROC and PR contributions, per tile of groups
__global__ void __launch_bounds__(kT) metrics_groups_kernel(const int64_t* __restrict__ gstart,
                                                            const int64_t* __restrict__ cpos,
                                                            const int64_t* __restrict__ n_groups, int64_t n,
                                                            const int64_t* __restrict__ pos_total,
                                                            double* __restrict__ part) {
  __shared__ double sh[4];
  const int64_t G = *n_groups;
  const double P = (double)*pos_total;
  double roc = 0.0, pr = 0.0;
  const int64_t g0 = (int64_t)blockIdx.x * kTile;
  for (int r = 0; r < kIPT; ++r) {
    const int64_t g = g0 + r * kT + threadIdx.x;
    if (g < G) {
      const int64_t s = gstart[g], e = g + 1 < G ? gstart[g + 1] : n;
      const double pa = (double)cpos[s], pe = e < n ? (double)cpos[e] : P;
      const double ng = (double)(e - s), pg = pe - pa, st = (double)s;
      roc += (ng - pg) * (pa + 0.5 * pg);
      const double r0 = P > 0 ? pa / P : 1.0, r1 = P > 0 ? pe / P : 1.0;
      const double p0 = g == 0 ? 1.0 : pa / st;
      const double p1 = pe / (st + ng);
      pr += (r1 - r0) * (p0 + p1) * 0.5;
    }
  }
  roc = block_sum(roc, sh);
  pr = block_sum(pr, sh);
  if (threadIdx.x == 0) {
    part[2 * blockIdx.x] = roc;
    part[2 * blockIdx.x + 1] = pr;
  }
}

// out = {auc, prauc, log_loss, rce, ctr, positives, n, groups}: the tiles' partial sums added in tile order
__global__ void __launch_bounds__(kT) metrics_final_kernel(const double* __restrict__ prep, int64_t nprep,
                                                           const double* __restrict__ grp,
                                                           const int64_t* __restrict__ n_groups, int64_t n,
                                                           double* __restrict__ out) {
  __shared__ double sh[4][kT];
  const int tid = threadIdx.x;
  const int64_t ng = (*n_groups + kTile - 1) / kTile;
  // thread t sums tiles t, t + 256, ... in order; then thread 0 adds the 256 thread sums in order
  double a[4] = {0.0, 0.0, 0.0, 0.0};
  for (int64_t b = tid; b < nprep; b += kT) {
    a[0] += prep[2 * b];
    a[1] += prep[2 * b + 1];
  }
  for (int64_t b = tid; b < ng; b += kT) {
    a[2] += grp[2 * b];
    a[3] += grp[2 * b + 1];
  }
#pragma unroll
  for (int q = 0; q < 4; ++q) sh[q][tid] = a[q];
  __syncthreads();
  if (tid != 0) return;
  double t[4] = {0.0, 0.0, 0.0, 0.0};
  for (int i = 0; i < kT; ++i)
#pragma unroll
    for (int q = 0; q < 4; ++q) t[q] += sh[q][i];
  const double P = t[1], N = (double)n - P;
  const double ll = t[0] / (double)n;
  const double c = P / (double)n;
  double straw = 0.0;  // log_loss(gt, [ctr] * n): the same per-row formula, closed form
  if (P > 0) straw += P * clipped_ll(c, 1);
  if (N > 0) straw += N * clipped_ll(c, 0);
  straw /= (double)n;
  out[0] = (P > 0 && N > 0) ? t[2] / (P * N) : nan("");
  out[1] = t[3];
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
  int32_t* counts;     // [256][tiles] digit counts of a radix pass
  int64_t* offs;       // their exclusive scan
  int64_t* cpos;       // positives ranked above each position
  int64_t* gstart;     // start of each tie group
  int64_t* tsum;       // scan tile sums (the largest scan: 256 x tiles items)
  int64_t* scal;       // [0] scan total (scratch), [1] positives, [2] groups
  double* prep;        // per tile: log-loss, positives
  double* grp;         // per tile of groups: roc, pr
  size_t total;
};

int64_t tiles_of(int64_t n) { return (n + kTile - 1) / kTile; }

MetricsWs carve(void* base, int64_t n) {
  MetricsWs w;
  char* p = reinterpret_cast<char*>(base);
  size_t o = 0;
  auto take = [&](size_t bytes) {
    void* r = p + o;
    o += align256(bytes);
    return r;
  };
  const int64_t nt = tiles_of(n);
  w.k0 = (uint32_t*)take(n * 4);
  w.k1 = (uint32_t*)take(n * 4);
  w.v0 = (int32_t*)take(n * 4);
  w.v1 = (int32_t*)take(n * 4);
  w.counts = (int32_t*)take(256 * nt * 4);
  w.offs = (int64_t*)take(256 * nt * 8);
  w.cpos = (int64_t*)take(n * 8);
  w.gstart = (int64_t*)take(n * 8);
  w.tsum = (int64_t*)take(tiles_of(256 * nt) * 8);
  w.scal = (int64_t*)take(4 * 8);
  w.prep = (double*)take(2 * nt * 8);
  w.grp = (double*)take(2 * nt * 8);
  w.total = o;
  return w;
}

hipError_t exclusive_scan(const ScanSrc& src, int64_t n, int64_t* tsum, int64_t* total, int64_t* out, hipStream_t s) {
  const int64_t nt = tiles_of(n);
  hipLaunchKernelGGL(scan_tiles_kernel, dim3((unsigned)nt), dim3(kT), 0, s, src, n, tsum);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(scan_top_kernel, dim3(1), dim3(1024), 0, s, tsum, nt, total);
  if ((e = hipGetLastError()) != hipSuccess) return e;
  hipLaunchKernelGGL(scan_down_kernel, dim3((unsigned)nt), dim3(kT), 0, s, src, n, tsum, out);
  return hipGetLastError();
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
  const int64_t nt = tiles_of(n);
  hipLaunchKernelGGL(metrics_prep_kernel, dim3((unsigned)nt), dim3(kT), 0, s, z, y, n, w.k0, w.v0, w.prep);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  // four stable 8-bit passes, k0 -> k1 -> k0 -> k1 -> k0
  uint32_t* kin = w.k0;
  uint32_t* kout = w.k1;
  int32_t* vin = w.v0;
  int32_t* vout = w.v1;
  for (int shift = 0; shift < 32; shift += 8) {
    hipLaunchKernelGGL(radix_hist_kernel, dim3((unsigned)nt), dim3(kT), 0, s, kin, n, shift, w.counts, nt);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    if ((e = exclusive_scan(ScanSrc{w.counts, nullptr, 0}, 256 * nt, w.tsum, w.scal, w.offs, s)) != hipSuccess)
      return e;
    hipLaunchKernelGGL(radix_scatter_kernel, dim3((unsigned)nt), dim3(kT), 0, s, kin, vin, n, shift, w.offs, nt,
                       kout, vout);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    uint32_t* tk = kin;
    kin = kout;
    kout = tk;
    int32_t* tv = vin;
    vin = vout;
    vout = tv;
  }
  // kin / vin: sorted by descending prediction.  Positives above each position, and the tie groups' starts
  if ((e = exclusive_scan(ScanSrc{vin, nullptr, 0}, n, w.tsum, w.scal + 1, w.cpos, s)) != hipSuccess) return e;
  if ((e = exclusive_scan(ScanSrc{nullptr, kin, 1}, n, w.tsum, w.scal + 2, w.gstart, s)) != hipSuccess) return e;
  hipLaunchKernelGGL(metrics_groups_kernel, dim3((unsigned)nt), dim3(kT), 0, s, w.gstart, w.cpos, w.scal + 2, n,
                     w.scal + 1, w.grp);
  if ((e = hipGetLastError()) != hipSuccess) return e;
  hipLaunchKernelGGL(metrics_final_kernel, dim3(1), dim3(kT), 0, s, w.prep, nt, w.grp, w.scal + 2, n, out);
  return hipGetLastError();
}

}  // namespace dfwfm
