// dfwfm_sparse.hip -- touched-row gradients of the categorical tables, for the data-parallel exchange.
//
// The reference's tables produce DENSE gradients (nn.Embedding(sparse=False), model/DeepFMs.py:199-210)
// and Adam's coupled L2 then touches every row (:553-556), so the reference's data-parallel equivalent
// all-reduces every table (58 MB at Criteo-39).  Only the rows a batch touched carry a data gradient: a
// rank can hand over (row, summed gradient) pairs instead, every rank adds all ranks' pairs into its local
// dense buffer, and the dense L2 + Adam step then runs locally on identical gradients.
//
// Deterministic by construction -- the replicas must stay bit-identical:
//   1. keys  (task << 32 | row) for every (table task, sample), value = sample index;
//   2. one stable radix sort (hipcub) -> equal rows adjacent, samples ascending within a row;
//   3. heads + inclusive scan -> entry index of every sorted position, entry starts;
//   4. segmented sums in a fixed order: 64-position blocks of the sorted order each sum their part of every
//      segment serially (thread per (block, column)); a segment that crosses blocks gets its block partials
//      added in block order by a second pass.  No atomics: the same inputs give the same bits;
//   5. the receiver adds the entry lists of rank 0, 1, ... in that order (one launch per list, destinations
//      unique within a list): plain read-add-write.
// dfwfm_sparse_grads_local (below) forms the same lists from the rank's dense local gradients instead (claim + copy,
// no sort): what the data-parallel training step uses.
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>
#include <stdint.h>

#include "dfwfm_internal.h"

namespace dfwfm {

constexpr int kSegBlock = 64;  // sorted positions per block of the segmented sum

__global__ void __launch_bounds__(256) sparse_keys_kernel(const SparseArgs a, uint64_t* __restrict__ keys,
                                                          uint32_t* __restrict__ vals) {
  const int k = blockIdx.y;
  const int64_t b = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (k >= a.ntasks || b >= a.batch) return;
  const SparseTask T = a.t[k];
  const FieldDev fd = a.fields[T.field];
  int64_t idx = a.xi[b * a.xi_stride + (T.field - a.num)];
  if (idx < 0 || idx >= fd.n) idx = 0;  // the forward clamped (and flagged) it the same way
  int64_t row = idx;
  if (T.kind == 1) row = idx / T.c;
  else if (T.kind == 2) row = idx % T.c;
  const int64_t i = (int64_t)k * a.batch + b;
  keys[i] = ((uint64_t)k << 32) | (uint64_t)(uint32_t)row;
  vals[i] = (uint32_t)b;
}

__global__ void __launch_bounds__(256) sparse_heads_kernel(const uint64_t* __restrict__ keys, int64_t n,
                                                           int32_t* __restrict__ head) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i < n) head[i] = (i == 0 || keys[i] != keys[i - 1]) ? 1 : 0;
}

// pos = inclusive scan of heads: entry of position i = pos[i] - 1; starts[e] = first position of entry e
__global__ void __launch_bounds__(256) sparse_starts_kernel(const int32_t* __restrict__ head,
                                                            const int32_t* __restrict__ pos, int64_t n,
                                                            int32_t* __restrict__ starts, int32_t* __restrict__ count) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  if (head[i]) starts[pos[i] - 1] = (int32_t)i;
  if (i == n - 1) {
    *count = pos[i];
    starts[pos[i]] = (int32_t)n;
  }
}

__device__ __forceinline__ float sparse_value(const SparseArgs& a, const SparseTask& T, int64_t b, int d) {
  const int f = T.field;
  float v = a.src == 1 ? a.dlogit[b] * (a.lw ? a.lw[f] : 1.f) : a.sv_de[b * (int64_t)a.F * a.D + f * a.D + d];
  if (T.other) {
    int64_t idx = a.xi[b * a.xi_stride + (f - a.num)];
    if (idx < 0 || idx >= a.fields[f].n) idx = 0;
    const int64_t part = T.kind == 1 ? idx % T.c : idx / T.c;  // the partner row of a QR "mult" field
    v *= T.other[part * a.w + d];
  }
  return v;
}

// pass A: thread per (64-position block, column).  Sums each segment's positions inside the block in order;
// a segment ending inside the block writes its in-block sum to its entry's row (final unless the segment began
// in an earlier block); a segment running past the block end leaves the partial in carry[block].
__global__ void __launch_bounds__(256) sparse_block_sum_kernel(const SparseArgs a, const uint64_t* __restrict__ keys,
                                                               const uint32_t* __restrict__ vals,
                                                               const int32_t* __restrict__ pos, int64_t n,
                                                               float* __restrict__ carry, int64_t* __restrict__ out_dest,
                                                               float* __restrict__ out_rows) {
  const int w = a.w;
  const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int64_t blk = t / w;
  const int d = (int)(t - blk * w);
  const int64_t p0 = blk * kSegBlock;
  if (p0 >= n) return;
  const int64_t p1 = p0 + kSegBlock < n ? p0 + kSegBlock : n;
  float acc = 0.f;
  uint64_t key = keys[p0];
  for (int64_t p = p0; p < p1; ++p) {
    const SparseTask& T = a.t[(int)(key >> 32)];
    acc += sparse_value(a, T, vals[p], d);
    const uint64_t next = p + 1 < n ? keys[p + 1] : ~0ull;
    if (next != key) {  // last position of this segment
      const int64_t e = pos[p] - 1;
      out_rows[e * w + d] = acc;
      if (d == 0) out_dest[e] = T.dest + (int64_t)(uint32_t)key * w;
      acc = 0.f;
    } else if (p + 1 == p1) {
      carry[blk * w + d] = acc;  // the segment continues in the next block
    }
    key = next;
  }
}

// pass B: thread per (entry, column); entries whose segment spans blocks c1 < c2 become
// ((carry[c1] + carry[c1+1]) + ... + carry[c2-1]) + (their part in block c2)
__global__ void __launch_bounds__(256) sparse_carry_kernel(const SparseArgs a, const int32_t* __restrict__ starts,
                                                           const int32_t* __restrict__ count,
                                                           const float* __restrict__ carry, int64_t cap,
                                                           float* __restrict__ out_rows) {
  const int w = a.w;
  const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int64_t e = t / w;
  const int d = (int)(t - e * w);
  if (e >= cap || e >= *count) return;
  const int64_t c1 = starts[e] / kSegBlock, c2 = (starts[e + 1] - 1) / kSegBlock;
  if (c1 == c2) return;
  float s = carry[c1 * w + d];
  for (int64_t c = c1 + 1; c < c2; ++c) s += carry[c * w + d];
  out_rows[e * w + d] = s + out_rows[e * w + d];
}

// receiver: grad[dest[e] + j] += rows[e * w + j] for the list's entries (destinations unique in a list)
__global__ void __launch_bounds__(256) sparse_apply_kernel(float* __restrict__ grad, int w,
                                                           const int64_t* __restrict__ dest,
                                                           const float* __restrict__ rows,
                                                           const int32_t* __restrict__ count, int64_t cap) {
  const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int64_t e = t / w;
  const int j = (int)(t - e * w);
  if (e >= cap || e >= *count) return;
  float* g = grad + dest[e] + j;
  *g = *g + rows[e * w + j];
}

// ---- touched-row lists from the rank's own dense table gradients (dfwfm_sparse_grads_local) ----------------------
// The backward scatters the rank's categorical-table gradients into a local dense buffer (as the single-GPU step does
// into its gradient buffer); the lists are then the touched rows of that buffer, deduplicated without atomics: every
// (table, sample) writes its sample index into its row's stamp (plain stores, some sample wins), then the sample
// whose index the stamp holds appends the row (only rows touched in this call are ever read back, so stale stamps
// of other rows never matter and the stamps need no reset); every appended row is copied out and cleared (the buffer
// is zero again for the next step).  Entries come in no particular order and their sums in atomic order -- harmless
// for the replicas: every rank applies the SAME bytes of every rank's list, in rank order, and destinations are
// unique within a list.
__device__ __forceinline__ int64_t local_row_off(const SparseArgs& a, int k, int64_t b) {
  const SparseTask T = a.t[k];
  const FieldDev fd = a.fields[T.field];
  int64_t idx = a.xi[b * a.xi_stride + (T.field - a.num)];
  if (idx < 0 || idx >= fd.n) idx = 0;  // the forward and the scatter clamped it the same way
  int64_t row = idx;
  if (T.kind == 1) row = idx / T.c;
  else if (T.kind == 2) row = idx % T.c;
  return T.dest + row * a.w;
}

__global__ void __launch_bounds__(256) local_mark_kernel(const SparseArgs a, int32_t* __restrict__ stamp,
                                                         int32_t* __restrict__ count) {
  const int k = blockIdx.y;
  const int64_t b = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (k == 0 && b == 0) *count = 0;
  if (k < a.ntasks && b < a.batch) stamp[local_row_off(a, k, b)] = (int32_t)b;
}

constexpr int kClaimThreads = 1024;  // one list-counter atomic per 1024 (table, sample) pairs

__global__ void __launch_bounds__(kClaimThreads) local_claim_kernel(const SparseArgs a,
                                                                    const int32_t* __restrict__ stamp,
                                                                    int64_t* __restrict__ out_dest,
                                                                    int32_t* __restrict__ count) {
  __shared__ int32_t wave_n[kClaimThreads / 64];
  __shared__ int32_t wg_base;
  const int k = blockIdx.y;
  const int64_t b = (int64_t)blockIdx.x * kClaimThreads + threadIdx.x;
  bool claim = false;
  int64_t off = 0;
  if (k < a.ntasks && b < a.batch) {
    off = local_row_off(a, k, b);
    claim = stamp[off] == (int32_t)b;
  }
  // slots: a prefix over the workgroup's waves, one counter atomic per workgroup
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const uint64_t mask = __ballot(claim);
  if (lane == 0) wave_n[wave] = (int32_t)__popcll(mask);
  __syncthreads();
  if (threadIdx.x == 0) {
    int32_t tot = 0;
    for (int w = 0; w < kClaimThreads / 64; ++w) {
      const int32_t n = wave_n[w];
      wave_n[w] = tot;
      tot += n;
    }
    wg_base = tot ? atomicAdd(count, tot) : 0;
  }
  __syncthreads();
  if (claim) out_dest[wg_base + wave_n[wave] + __popcll(mask & ((1ull << lane) - 1))] = off;
}

__global__ void __launch_bounds__(256) local_gather_kernel(float* __restrict__ local, int w,
                                                           const int64_t* __restrict__ dest, const int32_t* __restrict__ count,
                                                           int64_t cap, float* __restrict__ rows) {
  const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int64_t e = t / w;
  const int j = (int)(t - e * w);
  if (e >= cap || e >= *count) return;
  float* src = local + dest[e] + j;
  rows[e * w + j] = *src;
  *src = 0.f;
}

hipError_t launch_sparse_local(const SparseArgs& a, float* local, int32_t* stamp, int64_t cap, int64_t* out_dest,
                               float* out_rows, int32_t* out_count, hipStream_t s) {
  const int64_t n = (int64_t)a.ntasks * a.batch;
  if (n == 0) return hipMemsetAsync(out_count, 0, sizeof(int32_t), s);
  hipLaunchKernelGGL(local_mark_kernel, dim3((unsigned)((a.batch + 255) / 256), a.ntasks), dim3(256), 0, s, a, stamp,
                     out_count);
  hipLaunchKernelGGL(local_claim_kernel, dim3((unsigned)((a.batch + kClaimThreads - 1) / kClaimThreads), a.ntasks),
                     dim3(kClaimThreads), 0, s, a, stamp, out_dest, out_count);
  if (cap > 0)
    hipLaunchKernelGGL(local_gather_kernel, dim3((unsigned)((cap * a.w + 255) / 256)), dim3(256), 0, s, local, a.w,
                       out_dest, out_count, cap, out_rows);
  return hipGetLastError();
}

// ---- workspace carve-up -----------------------------------------------------------------------------
namespace {
struct SparseWs {
  uint64_t *k0, *k1;
  uint32_t *v0, *v1;
  int32_t *head, *pos, *starts;
  float* carry;
  void* cub;
  size_t cub_bytes, total;
};

size_t al256(size_t x) { return (x + 255) & ~(size_t)255; }

SparseWs carve(void* base, int64_t n, int w, int end_bit) {
  SparseWs s;
  size_t sort_b = 0, scan_b = 0;
  (void)hipcub::DeviceRadixSort::SortPairs(nullptr, sort_b, (const uint64_t*)nullptr, (uint64_t*)nullptr,
                                           (const uint32_t*)nullptr, (uint32_t*)nullptr, (int)n, 0, end_bit);
  (void)hipcub::DeviceScan::InclusiveSum(nullptr, scan_b, (const int32_t*)nullptr, (int32_t*)nullptr, (int)n);
  s.cub_bytes = sort_b > scan_b ? sort_b : scan_b;
  const int64_t nblk = (n + kSegBlock - 1) / kSegBlock;
  char* p = static_cast<char*>(base);
  size_t o = 0;
  auto take = [&](size_t bytes) { char* r = p ? p + o : nullptr; o += al256(bytes); return r; };
  s.k0 = (uint64_t*)take(8 * n);
  s.k1 = (uint64_t*)take(8 * n);
  s.v0 = (uint32_t*)take(4 * n);
  s.v1 = (uint32_t*)take(4 * n);
  s.head = (int32_t*)take(4 * n);
  s.pos = (int32_t*)take(4 * n);
  s.starts = (int32_t*)take(4 * (n + 1));
  s.carry = (float*)take(4 * (size_t)nblk * w);
  s.cub = take(s.cub_bytes);
  s.total = o;
  return s;
}

int task_bits(int ntasks) {
  int b = 1;
  while ((1 << b) < ntasks) ++b;
  return b;
}
}  // namespace

size_t sparse_workspace_bytes(int64_t n, int w, int ntasks) {
  return carve(nullptr, n, w, 32 + task_bits(ntasks)).total;
}

hipError_t launch_sparse_grads(const SparseArgs& a, int64_t* out_dest, float* out_rows, int32_t* out_count, void* ws,
                               size_t ws_bytes, hipStream_t s) {
  const int64_t n = (int64_t)a.ntasks * a.batch;
  const int end_bit = 32 + task_bits(a.ntasks);
  SparseWs W = carve(ws, n, a.w, end_bit);
  if (W.total > ws_bytes) return hipErrorInvalidValue;
  if (n == 0) return hipMemsetAsync(out_count, 0, sizeof(int32_t), s);
  const unsigned gb = (unsigned)((a.batch + 255) / 256);
  hipLaunchKernelGGL(sparse_keys_kernel, dim3(gb, a.ntasks), dim3(256), 0, s, a, W.k0, W.v0);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  size_t cb = W.cub_bytes;
  e = hipcub::DeviceRadixSort::SortPairs(W.cub, cb, W.k0, W.k1, W.v0, W.v1, (int)n, 0, end_bit, s);
  if (e != hipSuccess) return e;
  const unsigned gn = (unsigned)((n + 255) / 256);
  hipLaunchKernelGGL(sparse_heads_kernel, dim3(gn), dim3(256), 0, s, W.k1, n, W.head);
  cb = W.cub_bytes;
  e = hipcub::DeviceScan::InclusiveSum(W.cub, cb, W.head, W.pos, (int)n, s);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(sparse_starts_kernel, dim3(gn), dim3(256), 0, s, W.head, W.pos, n, W.starts, out_count);
  const int64_t nblk = (n + kSegBlock - 1) / kSegBlock;
  hipLaunchKernelGGL(sparse_block_sum_kernel, dim3((unsigned)((nblk * a.w + 255) / 256)), dim3(256), 0, s, a, W.k1,
                     W.v1, W.pos, n, W.carry, out_dest, out_rows);
  hipLaunchKernelGGL(sparse_carry_kernel, dim3((unsigned)((n * a.w + 255) / 256)), dim3(256), 0, s, a, W.starts,
                     out_count, W.carry, n, out_rows);
  return hipGetLastError();
}

hipError_t launch_sparse_apply(float* grad, int w, const int64_t* dest, const float* rows, const int32_t* count,
                               int64_t cap, hipStream_t s) {
  if (cap <= 0) return hipSuccess;
  hipLaunchKernelGGL(sparse_apply_kernel, dim3((unsigned)((cap * w + 255) / 256)), dim3(256), 0, s, grad, w, dest,
                     rows, count, cap);
  return hipGetLastError();
}

}  // namespace dfwfm
