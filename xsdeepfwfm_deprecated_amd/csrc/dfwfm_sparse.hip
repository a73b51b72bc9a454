// dfwfm_sparse.hip -- touched-row gradients of the categorical tables, for the data-parallel exchange.
//
// The reference's tables produce DENSE gradients (nn.Embedding(sparse=False), model/DeepFMs.py:199-210)
// and Adam's coupled L2 then touches every row (:553-556), so the reference's data-parallel equivalent
// all-reduces every table (58 MB at Criteo-39).  Only the rows a batch touched carry a data gradient: a
// rank can hand over (row, summed gradient) pairs instead, every rank adds all ranks' pairs into its local
// dense buffer, and the dense L2 + Adam step then runs locally on identical gradients.
//
// dfwfm_sparse_grads_local forms each rank's list from its own dense table gradients (mark, claim, copy; no sort);
// the receiver adds the lists of rank 0, 1, ... in that order (one launch per list, destinations unique within a
// list): plain read-add-write, the same bytes in the same order on every rank, so the replicas stay bit-identical.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "dfwfm_internal.h"

namespace dfwfm {

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
                                                                    int64_t* __restrict__ out_dest, int64_t cap,
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
  // the capacity (dfwfm_sparse_grads_size: sum over tables of min(batch, rows)) bounds the distinct rows; the guard
  // keeps a list write inside the buffer whatever the caller passed (the count may then exceed cap; every reader
  // stops at min(count, cap))
  const int64_t slot = (int64_t)wg_base + wave_n[wave] + __popcll(mask & ((1ull << lane) - 1));
  if (claim && slot < cap) out_dest[slot] = off;
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
                     dim3(kClaimThreads), 0, s, a, stamp, out_dest, cap, out_count);
  if (cap > 0)
    hipLaunchKernelGGL(local_gather_kernel, dim3((unsigned)((cap * a.w + 255) / 256)), dim3(256), 0, s, local, a.w,
                       out_dest, out_count, cap, out_rows);
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
