// dfwfm_prune.hip -- magnitude pruning of the training loop on the device (reference
// model/DeepFMs.py:647-673 with binary_search_threshold, :807-823).
//
// The reference finds each threshold by bisection on (0, 100): up to 101 rounds of
// `(abs(param) < mid).sum().item()` -- a full pass over the tensor and a host sync per round.  Here the same
// bisection is resolved kSelDepth rounds per pass over the magnitudes, with no sort and no host sync:
//   * the next kSelDepth rounds can only ask for the 2^kSelDepth - 1 mids of the bisection tree below the current
//     (l, r); listed in order they ascend (left subtree < mid < right subtree), so
//   * one pass places every |x| among those candidate thresholds (a 12-step binary lift over the candidate keys in
//     LDS) and histograms the positions -- count(|x| < c_j) is the histogram's prefix sum at j,
//   * one workgroup then replays the reference's rounds down the tree (same doubles, same break tests, the compare
//     `|x| < mid` in f32 as torch does for a float32 tensor and a Python float) and lists the next tree's candidates.
// Every count is exact, so the thresholds are the reference's bit for bit.  A pass is two launches (count; reduce +
// walk, the walk by the reduce grid's last workgroup); the host enqueues the 9 passes the 101-round cap can need, and
// passes after the bisection has ended return at once.  The mask is applied in place reading the threshold from
// device memory.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "dfwfm_internal.h"

namespace dfwfm {

constexpr int kSelDepth = 12;                            // bisection rounds resolved per pass
constexpr int kSelBins = 1 << kSelDepth;                 // histogram positions 0..kSelCand
constexpr int kSelCand = kSelBins - 1;                   // candidate thresholds per pass (4095)
constexpr int kSelPasses = (101 + kSelDepth - 1) / kSelDepth;  // the reference's cap: at most 101 rounds
constexpr int kSelThreads = 256;
constexpr int kSelMaxWG = 256;

struct SelState {
  double l, r, mid;
  int32_t cnt, done;
  uint32_t ticket, pad_;
};

struct SelWs {
  SelState* st;
  uint32_t* cand;     // [kSelCand] candidate keys (f32 bits of (float)mid), ascending
  uint32_t* hist;     // [kSelBins] summed histogram
  uint32_t* part;     // [nwg][kSelBins] per-workgroup histograms
};

static int sel_nwg(int64_t n) {
  const int64_t w = (n + 8191) / 8192;
  return (int)(w < 1 ? 1 : (w > kSelMaxWG ? kSelMaxWG : w));
}

static size_t align256(size_t b) { return (b + 255) & ~(size_t)255; }

static SelWs sel_ws(void* ws, int nwg) {
  char* b = reinterpret_cast<char*>(ws);
  SelWs w;
  w.st = reinterpret_cast<SelState*>(b);
  b += align256(sizeof(SelState));
  w.cand = reinterpret_cast<uint32_t*>(b);
  b += align256(sizeof(uint32_t) * kSelCand);
  w.hist = reinterpret_cast<uint32_t*>(b);
  b += align256(sizeof(uint32_t) * kSelBins);
  w.part = reinterpret_cast<uint32_t*>(b);
  (void)nwg;
  return w;
}

size_t prune_workspace_bytes(int64_t n) {
  return align256(sizeof(SelState)) + align256(sizeof(uint32_t) * kSelCand) + align256(sizeof(uint32_t) * kSelBins) +
         align256(sizeof(uint32_t) * kSelBins * (size_t)sel_nwg(n));
}

// the mid of the bisection-tree node with in-order index i (1..kSelCand) below (l, r): the path from the root
// repeats the reference's updates (count above target -> r = mid: left; else l = mid: right)
__device__ __forceinline__ double tree_mid(double l, double r, int i) {
  int lo = 0, hi = kSelBins;
  for (;;) {
    const int m = (lo + hi) >> 1;
    const double mid = (l + r) / 2;
    if (i == m) return mid;
    if (i < m) { hi = m; r = mid; }
    else { lo = m; l = mid; }
  }
}

__device__ void list_candidates(const SelState& s, uint32_t* __restrict__ cand) {
  for (int i = threadIdx.x; i < kSelCand; i += blockDim.x)
    cand[i] = __float_as_uint((float)tree_mid(s.l, s.r, i + 1));
}

__global__ void select_start_kernel(SelWs w) {
  __shared__ SelState s;
  if (threadIdx.x == 0) {
    s.l = 0.0;
    s.r = 1e2;
    s.mid = 0.0;
    s.cnt = 0;
    s.done = 0;
    s.ticket = 0;
    s.pad_ = 0;
    *w.st = s;
  }
  __syncthreads();
  list_candidates(s, w.cand);
}

__device__ __forceinline__ float src_value(const PruneSrc& src, int64_t i) {
  if (src.sym_f > 0) {
    const int64_t k = i / src.sym_f, l = i - k * src.sym_f;
    return __fmul_rn(0.5f, __fadd_rn(src.p[i], src.p[l * src.sym_f + k]));  // 0.5 * (W + W.t())
  }
  return src.p[i];
}

// every magnitude's position among the candidates (the number of candidate keys <= its key; non-negative floats
// order like their bit patterns, and a NaN's key is above every candidate, so it is never counted below a
// threshold, as `abs(nan) < mid` is false) -> this workgroup's histogram
__global__ __launch_bounds__(kSelThreads) void select_count_kernel(const PruneList L, SelWs w) {
  if (w.st->done) return;
  __shared__ uint32_t cand[kSelCand + 1];
  __shared__ uint32_t hist[kSelBins];
  for (int i = threadIdx.x; i < kSelCand; i += kSelThreads) cand[i] = w.cand[i];
  for (int i = threadIdx.x; i < kSelBins; i += kSelThreads) hist[i] = 0;
  __syncthreads();
  const int lane = threadIdx.x & 63;
  const int64_t stride = (int64_t)gridDim.x * kSelThreads;
  for (int s = 0; s < L.n; ++s) {
    const PruneSrc src = L.s[s];
    for (int64_t base = (int64_t)blockIdx.x * kSelThreads + threadIdx.x; base - threadIdx.x < src.numel;
         base += 4 * stride) {
      float v[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int64_t i = base + u * stride;
        v[u] = i < src.numel ? src_value(src, i) : 0.f;
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const bool valid = base + u * stride < src.numel;
        const uint32_t key = __float_as_uint(fabsf(v[u]));
        int p = 0;
#pragma unroll
        for (int step = kSelBins >> 1; step > 0; step >>= 1)
          if (cand[p + step - 1] <= key) p += step;
        // most magnitudes fall into a few positions (below or above the whole candidate range): the wave adds the
        // two commonest positions with one LDS atomic each, the rest per lane
        bool pending = valid;
#pragma unroll
        for (int round = 0; round < 2; ++round) {
          const uint64_t act = __ballot(pending);
          if (act == 0) break;
          const int leader = __ffsll((unsigned long long)act) - 1;
          const int lp = __shfl(p, leader);
          const bool same = pending && p == lp;
          const uint64_t sm = __ballot(same);
          if (lane == leader) atomicAdd(&hist[lp], (uint32_t)__popcll(sm));
          pending = pending && !same;
        }
        if (pending) atomicAdd(&hist[p], 1u);
      }
    }
  }
  __syncthreads();
  uint32_t* out = w.part + (size_t)blockIdx.x * kSelBins;
  for (int i = threadIdx.x; i < kSelBins; i += kSelThreads) out[i] = hist[i];
}

// sum the workgroups' histograms; the last workgroup to finish scans the sum, replays up to kSelDepth rounds of the
// reference's bisection down the candidate tree, and lists the next candidates (or writes the threshold)
__global__ __launch_bounds__(kSelThreads) void select_walk_kernel(SelWs w, int nwg, double total, double target,
                                                                  double* __restrict__ thr) {
  if (w.st->done) return;
  const int c = blockIdx.x * kSelThreads + threadIdx.x;  // gridDim.x * kSelThreads == kSelBins
  uint32_t sum = 0;
  for (int g = 0; g < nwg; ++g) sum += w.part[(size_t)g * kSelBins + c];
  w.hist[c] = sum;
  __threadfence();
  __shared__ uint32_t last;
  __syncthreads();
  if (threadIdx.x == 0) last = atomicAdd(&w.st->ticket, 1u) == gridDim.x - 1;
  __syncthreads();
  if (!last) return;
  __threadfence();
  // inclusive scan of the kSelBins sums: 16 per thread, then the 256 thread totals
  __shared__ uint32_t scan[kSelBins];
  __shared__ uint32_t tot[kSelThreads];
  __shared__ SelState s;
  constexpr int per = kSelBins / kSelThreads;
  uint32_t run = 0;
  for (int j = 0; j < per; ++j) {
    run += __atomic_load_n(&w.hist[threadIdx.x * per + j], __ATOMIC_RELAXED);
    scan[threadIdx.x * per + j] = run;
  }
  tot[threadIdx.x] = run;
  __syncthreads();
  if (threadIdx.x == 0) {
    uint32_t acc = 0;
    for (int t = 0; t < kSelThreads; ++t) {
      const uint32_t x = tot[t];
      tot[t] = acc;
      acc += x;
    }
  }
  __syncthreads();
  for (int j = 0; j < per; ++j) scan[threadIdx.x * per + j] += tot[threadIdx.x];
  __syncthreads();
  if (threadIdx.x == 0) {
    s = *w.st;
    int lo = 0, hi = kSelBins;
    bool done = false;
    for (int d = 0; d < kSelDepth; ++d) {  // binary_search_threshold, one round per tree level
      if (!(s.l < s.r)) { done = true; break; }
      s.cnt += 1;
      const int m = (lo + hi) >> 1;
      s.mid = (s.l + s.r) / 2;
      const double items = (double)scan[m - 1];  // count(|x| < (float)mid): positions 0 .. m-1
      const double rate = items / total;
      if (fabs(rate - target) < 0.0001) { done = true; break; }
      if (rate > target) { s.r = s.mid; hi = m; }
      else { s.l = s.mid; lo = m; }
      if (s.cnt > 100) { done = true; break; }
    }
    s.done = done ? 1 : 0;
    s.ticket = 0;
    if (done) *thr = s.mid;
    *w.st = s;
  }
  __syncthreads();
  if (!s.done) list_candidates(s, w.cand);
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

hipError_t launch_prune_threshold(const PruneList& L, double target, double* d_thr, void* ws, size_t ws_bytes,
                                  hipStream_t s) {
  int64_t total = 0;
  for (int i = 0; i < L.n; ++i) total += L.s[i].numel;
  if (L.n <= 0 || L.n > kMaxPruneSrc || total <= 0 || total > 0x7fffffff) return hipErrorInvalidValue;
  if (ws_bytes < prune_workspace_bytes(total)) return hipErrorInvalidValue;
  const int nwg = sel_nwg(total);
  const SelWs w = sel_ws(ws, nwg);
  hipLaunchKernelGGL(select_start_kernel, dim3(1), dim3(1024), 0, s, w);
  hipError_t e = hipGetLastError();
  for (int pass = 0; pass < kSelPasses && e == hipSuccess; ++pass) {
    hipLaunchKernelGGL(select_count_kernel, dim3(nwg), dim3(kSelThreads), 0, s, L, w);
    hipLaunchKernelGGL(select_walk_kernel, dim3(kSelBins / kSelThreads), dim3(kSelThreads), 0, s, w, nwg,
                       (double)total, target, d_thr);
    e = hipGetLastError();
  }
  return e;
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
