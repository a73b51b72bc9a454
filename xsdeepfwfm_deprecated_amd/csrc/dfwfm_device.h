// dfwfm_device.h -- device helpers shared by the forward and training kernels.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "dfwfm_internal.h"

namespace dfwfm {

typedef float f32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ float relu_keep_nan(float v) { return v < 0.f ? 0.f : v; }

// Diagnostic phase stamps (p.stamps != nullptr only in DFWFM_DIAG stamps= runs; in production the
// branch is never taken): wave 0 lane 0 records the shader clock at phase boundaries.
__device__ __forceinline__ void stamp(uint64_t* st, int slot, int tid) {
  if (st != nullptr && tid == 0) st[(size_t)blockIdx.x * kStampSlots + slot] = __builtin_amdgcn_s_memtime();
}

// the batch and first row of this workgroup's tile (ROWS samples per workgroup), and that batch's inputs and logits:
// the batch set of dfwfm_forward_batches (p.nb > 1), else the one batch of the launch
struct TileRef {
  const int64_t* xi;
  const float* xv;
  float* out;
  int64_t b0;
};
template <int ROWS>
__device__ __forceinline__ TileRef tile_ref(const FwdArgs& p) {
  if (p.nb > 1) {
    const int bi = (int)blockIdx.x / p.tiles;  // wave-uniform
    return TileRef{p.set_xi[bi], p.set_xv[bi], p.set_out[bi], (int64_t)((int)blockIdx.x - bi * p.tiles) * ROWS};
  }
  return TileRef{p.xi, p.xv, p.out, (int64_t)blockIdx.x * ROWS};
}

// one DPP-moved copy of v (the move rides on the VALU; a __shfl_xor is an LDS-crossbar round trip)
template <int CTRL>
__device__ __forceinline__ float dpp_f(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), CTRL, 0xF, 0xF, false));
}

// sum over the 16 lanes of an aligned 16-lane group (a DPP row), every lane gets the total: row_ror:8,
// row_ror:4, then quad_perm [2,3,0,1] and [1,0,3,2].  Each step adds the partner of lane i ^ 8, ^ 4, ^ 2, ^ 1
// (a rotation by 8 is i ^ 8; after it every value is symmetric under ^ 8, so a rotation by 4 adds i ^ 4's).
__device__ __forceinline__ float sum16(float v) {
  v += dpp_f<0x128>(v);
  v += dpp_f<0x124>(v);
  v += dpp_f<0x4E>(v);
  v += dpp_f<0xB1>(v);
  return v;
}

// constant-rate (100 MHz) clock, comparable across XCDs: workgroup start/end spread
__device__ __forceinline__ void stamp_rt(uint64_t* st, int slot, int tid) {
  if (st != nullptr && tid == 0) st[(size_t)blockIdx.x * kStampSlots + slot] = __builtin_amdgcn_s_memrealtime();
}

// workgroup start (slot 14) / end (slot 15) on the 100 MHz clock; the end word carries the XCC and
// the CU / SH / SE bits of HW_ID in bits 48-59, for a cross-launch timeline (tools/timeline.py)
__device__ __forceinline__ void stamp_start_rt(uint64_t* st, int tid) { stamp_rt(st, 14, tid); }
__device__ __forceinline__ void stamp_end_rt(uint64_t* st, int tid) {
  if (st != nullptr && tid == 0) {
    const uint32_t hw = __builtin_amdgcn_s_getreg(4 | (31 << 11));    // HW_REG_HW_ID
    const uint32_t xcc = __builtin_amdgcn_s_getreg(20 | (31 << 11));  // HW_REG_XCC_ID
    const uint64_t id = (uint64_t)(((xcc & 0xF) << 8) | ((hw >> 8) & 0xFF));
    st[(size_t)blockIdx.x * kStampSlots + 15] = __builtin_amdgcn_s_memrealtime() | (id << 48);
  }
}

template <int D>
__device__ __forceinline__ void load_row(float (&v)[D], const float* __restrict__ src) {
  if constexpr (D % 4 == 0) {
#pragma unroll
    for (int d = 0; d < D; d += 4) {
      const float4 x = *reinterpret_cast<const float4*>(src + d);
      v[d] = x.x; v[d + 1] = x.y; v[d + 2] = x.z; v[d + 3] = x.w;
    }
  } else if constexpr (D % 2 == 0) {
#pragma unroll
    for (int d = 0; d < D; d += 2) {
      const float2 x = *reinterpret_cast<const float2*>(src + d);
      v[d] = x.x; v[d + 1] = x.y;
    }
  } else {
#pragma unroll
    for (int d = 0; d < D; ++d) v[d] = src[d];
  }
}

template <int D>
__device__ __forceinline__ void store_row(float* dst, const float (&v)[D]) {
  if constexpr (D % 4 == 0) {
#pragma unroll
    for (int d = 0; d < D; d += 4) *reinterpret_cast<float4*>(dst + d) = make_float4(v[d], v[d + 1], v[d + 2], v[d + 3]);
  } else if constexpr (D % 2 == 0) {
#pragma unroll
    for (int d = 0; d < D; d += 2) *reinterpret_cast<float2*>(dst + d) = make_float2(v[d], v[d + 1]);
  } else {
#pragma unroll
    for (int d = 0; d < D; ++d) dst[d] = v[d];
  }
}

// one row of the tables' serving copy (dfwfm_model_pack_tables): D floats of second order, then the first-order
// weight, from a 16-byte aligned row: ceil((D + 1) / 4) dwordx4 loads
template <int D>
__device__ __forceinline__ void load_row_fo(float (&v)[D], float& fo, const float* __restrict__ src) {
  constexpr int NQ = (D + 4) / 4;
  f32x4 x[NQ];
#pragma unroll
  for (int q = 0; q < NQ; ++q) x[q] = reinterpret_cast<const f32x4*>(src)[q];
#pragma unroll
  for (int d = 0; d < D; ++d) v[d] = x[d / 4][d % 4];
  fo = x[D / 4][D % 4];
}

// row combine modes: 0 = a * scale (numerical / plain, scale 1), 1 = a * b (QR mult), 2 = a + b (QR add)
__device__ __forceinline__ float combine(int mode, float a, float b, float scale) {
  return mode == 1 ? a * b : (mode == 2 ? a + b : a * scale);
}

// ---------------------------------------------------------------------------
// phase M: one MLP layer for the workgroup's 16 rows, one wave's share.
//   act : LDS [16][SA] input activations (K zero-padded to NC*16)
//   wl  : packed weights of this layer, [NT][NC][64 lanes] float4
//   the wave group g (0..3) owns output tiles g, g+4, ... (TPW of them; tiles
//   past NT are clamped duplicates whose results are discarded); it walks K
//   chunks c0, c0+KS, ...
// Fragment algebra (16x16x4 f32): in sub-step s of chunk c lane l supplies
//   A = act[l&15][16c + 4(l>>4) + s],  B = W[n0 + (l&15)][16c + 4(l>>4) + s].
// ---------------------------------------------------------------------------
// WA: the weights are the A operand and the activations B, so the accumulator comes out transposed:
// lane l holds neurons 4(l>>4) + r of row l&15 -- four consecutive outputs of one sample, stored as one
// 16-byte LDS write (same products, same k order: bit-identical sums)
template <bool WA>
__device__ __forceinline__ f32x4 mfma_wa(float a, float w, f32x4 c) {
  return WA ? __builtin_amdgcn_mfma_f32_16x16x4f32(w, a, c, 0, 0, 0) : __builtin_amdgcn_mfma_f32_16x16x4f32(a, w, c, 0, 0, 0);
}

template <int TPW, bool WA = false>
__device__ __forceinline__ void mfma_chunk(f32x4 (&acc)[TPW], const float4& a, const f32x4 (&b)[TPW]) {
  // sub-step-major: consecutive MFMAs hit different accumulators (16x16x4 f32 has a 40-cycle
  // dependent latency against a 32-cycle issue interval)
#pragma unroll
  for (int j = 0; j < TPW; ++j) acc[j] = mfma_wa<WA>(a.x, b[j].x, acc[j]);
#pragma unroll
  for (int j = 0; j < TPW; ++j) acc[j] = mfma_wa<WA>(a.y, b[j].y, acc[j]);
#pragma unroll
  for (int j = 0; j < TPW; ++j) acc[j] = mfma_wa<WA>(a.z, b[j].z, acc[j]);
#pragma unroll
  for (int j = 0; j < TPW; ++j) acc[j] = mfma_wa<WA>(a.w, b[j].w, acc[j]);
}

// One layer's weight stream for one wave: output tiles g, g+4, ... (clamped to NT-1) and K chunks
// c0, c0+KS, ... of the packed [NT][NC][64] float4 layout.  Loads are buffer loads: the per-tile
// base and the chunk offset are scalar (SALU), the only vector operand is lane*16 -- flat loads
// spent a 64-bit VALU add per load in front of the MFMAs.
template <int TPW, int KS, int NG = 4>
struct LayerStream {
  __amdgpu_buffer_rsrc_t rsrc;
  int sbase[TPW];  // byte offset of each owned tile's [NC][64] block (wave-uniform)
  int n, c0;
  __device__ __forceinline__ void init(__amdgpu_buffer_rsrc_t r, int layer_off, int NC, int NT, int g, int c0_) {
    rsrc = r;
#pragma unroll
    for (int j = 0; j < TPW; ++j) {
      int t = g + NG * j;
      t = t < NT ? t : NT - 1;
      sbase[j] = __builtin_amdgcn_readfirstlane((layer_off + t * NC * 64) * 16);
    }
    c0 = c0_;
    n = c0 < NC ? (NC - c0 + KS - 1) / KS : 0;
  }
  __device__ __forceinline__ int chunk(int i) const { return c0 + KS * (i < n ? i : n - 1); }
  __device__ __forceinline__ void load(f32x4 (&b)[TPW], int c, int voff) const {
#pragma unroll
    for (int j = 0; j < TPW; ++j)
      b[j] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rsrc, voff, sbase[j] + c * 1024, 0));
  }
  // the first two chunks, issued ahead of time (before the previous phase's epilogue / barrier)
  __device__ __forceinline__ void preload(f32x4 (&b0)[TPW], f32x4 (&b1)[TPW], int voff) const {
    if (n == 0) return;
    load(b0, chunk(0), voff);
    load(b1, chunk(1), voff);
  }
};

// The split tail tile: when the layer has 4*TPW + 1 output tiles, tile T = 4*TPW is shared by the
// four waves, wave g taking K chunks [NC*g/4, NC*(g+1)/4) of it, so every SIMD carries 6.25 tiles
// instead of one carrying 7.  All of a wave's tail fragments are loaded with the layer's preload
// (kTailC <= 8 chunks per wave, NC <= 32) and consumed after the main K loop.
template <int NG = 4>
struct TailStream {
  static constexpr int C = kTailC * 4 / NG;  // K chunks per wave at most (layer widths <= 512)
  int sbase, c_lo, cnt;
  __device__ __forceinline__ void init(int layer_off, int NC, int T, int g) {
    sbase = __builtin_amdgcn_readfirstlane((layer_off + T * NC * 64) * 16);
    c_lo = (NC * g) / NG;
    cnt = (NC * (g + 1)) / NG - c_lo;
  }
  __device__ __forceinline__ void load(__amdgpu_buffer_rsrc_t r, f32x4 (&tw)[C], int voff) const {
#pragma unroll
    for (int u = 0; u < C; ++u)
      if (u < cnt)
        tw[u] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(r, voff, sbase + (c_lo + u) * 1024, 0));
  }
  // this wave's partial product of the tail tile (two accumulators: no back-to-back dependent MFMAs)
  template <bool WA = false>
  __device__ __forceinline__ f32x4 mma(const float* __restrict__ act, int SA, const f32x4 (&tw)[C], int lane) const {
    const float* arow = act + (lane & 15) * SA + 4 * (lane >> 4);
    f32x4 a0 = f32x4{0.f, 0.f, 0.f, 0.f}, a1 = a0;
#pragma unroll
    for (int u = 0; u < C; ++u) {
      if (u < cnt) {
        const float4 a = *reinterpret_cast<const float4*>(arow + 16 * (c_lo + u));
        f32x4& c = (u & 1) ? a1 : a0;
        c = mfma_wa<WA>(a.x, tw[u].x, c);
        c = mfma_wa<WA>(a.y, tw[u].y, c);
        c = mfma_wa<WA>(a.z, tw[u].z, c);
        c = mfma_wa<WA>(a.w, tw[u].w, c);
      }
    }
    return a0 + a1;
  }
  // mlp_k_loop_s form: fragments [u0, u0 + TPW) of this wave's share go into a weight register set the
  // K loop has just freed (its drain steps), and are multiplied after its last step
  template <int TPW>
  __device__ __forceinline__ void load_set(__amdgpu_buffer_rsrc_t r, f32x4 (&b)[TPW], int u0, int voff) const {
#pragma unroll
    for (int j = 0; j < TPW; ++j)
      if (u0 + j < cnt)
        b[j] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(r, voff, sbase + (c_lo + u0 + j) * 1024, 0));
  }
  template <int TPW, bool WA>
  __device__ __forceinline__ void mma_set(const float* __restrict__ arow, const f32x4 (&b)[TPW], int u0, f32x4& c0,
                                          f32x4& c1) const {
#pragma unroll
    for (int j = 0; j < TPW; ++j) {
      const int u = u0 + j;
      if (u < cnt) {
        const float4 a = *reinterpret_cast<const float4*>(arow + 16 * (c_lo + u));
        f32x4& c = (u & 1) ? c1 : c0;
        c = mfma_wa<WA>(a.x, b[j].x, c);
        c = mfma_wa<WA>(a.y, b[j].y, c);
        c = mfma_wa<WA>(a.z, b[j].z, c);
        c = mfma_wa<WA>(a.w, b[j].w, c);
      }
    }
  }
};

// K loop of one layer, entered with chunks 0 and 1 already in b0 / b1.  Weight fragments rotate
// through three register sets, each refilled two chunks ahead of its MFMAs (the loop is unrolled
// by 3 so no set is ever copied: a copy makes hipcc wait for the load it copies).  The activation
// fragments rotate with them (three float4, read from LDS two chunks ahead): with only two, every
// other step's read targeted the register its own MFMAs were still reading, so it issued behind
// them and the next step's first MFMA waited out the LDS latency.  Within a step the LDS read goes
// first, then the refill loads interleave with the MFMAs (sched_group_barrier: 2 MFMA, 1 load,
// ...), and a sched_barrier closes the step so hipcc cannot sink them to their use.
// SEEDED: acc arrives holding the initial values (e.g. the bias), else it starts from zero
template <int TPW, int KS, int NG = 4, bool WA = false, bool SEEDED = false>
__device__ __forceinline__ void mlp_k_loop(f32x4 (&acc)[TPW], const float* __restrict__ act, int SA,
                                           const LayerStream<TPW, KS, NG>& ls, f32x4 (&b0)[TPW],
                                           f32x4 (&b1)[TPW], f32x4 (&b2)[TPW], int lane) {
  if constexpr (!SEEDED) {
#pragma unroll
    for (int j = 0; j < TPW; ++j) acc[j] = f32x4{0.f, 0.f, 0.f, 0.f};
  }
  const int n = ls.n;
  if (n == 0) return;
  const int voff = lane * 16;
  const float* arow = act + (lane & 15) * SA + 4 * (lane >> 4);
  float4 a0 = *reinterpret_cast<const float4*>(arow + 16 * ls.chunk(0));
  float4 a1 = *reinterpret_cast<const float4*>(arow + 16 * ls.chunk(1));
  float4 a2;
#define DFWFM_MFMA_STEP(X, AX)                                                         \
  mfma_chunk<TPW, WA>(acc, AX, X);                                                     \
  __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);                                   \
  for (int q = 0; q < TPW; ++q) {                                                      \
    __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);                                 \
    __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);                                 \
  }                                                                                    \
  __builtin_amdgcn_sched_group_barrier(0x008, 2 * TPW, 0);                             \
  __builtin_amdgcn_sched_barrier(0);
  // a step that refills the set it frees with chunk i + 2
#define DFWFM_STEP(X, AX, Z, AZ, i)                                                    \
  {                                                                                    \
    AZ = *reinterpret_cast<const float4*>(arow + 16 * ls.chunk((i) + 2));              \
    ls.load(Z, ls.chunk((i) + 2), voff);                                               \
    DFWFM_MFMA_STEP(X, AX)                                                             \
  }
  // a drain step (no chunk left to fetch): no load at all -- a load of a chunk nobody consumes keeps a
  // register busy past the loop and the epilogue then waits for it, i.e. for the next layer's preload
#define DFWFM_STEP_N(X, AX) \
  { DFWFM_MFMA_STEP(X, AX) }
  int i = 0;
  for (; i + 5 <= n; i += 3) {  // steady state: steps i..i+2 fetch chunks i+2..i+4 < n
    DFWFM_STEP(b0, a0, b2, a2, i);
    DFWFM_STEP(b1, a1, b0, a0, i + 1);
    DFWFM_STEP(b2, a2, b1, a1, i + 2);
  }
  const int r = n - i;  // 1..4 steps left; step j fetches chunk i + j + 2 only while that is < n
  if (r == 1) {
    DFWFM_STEP_N(b0, a0);
  } else if (r == 2) {
    DFWFM_STEP_N(b0, a0);
    DFWFM_STEP_N(b1, a1);
  } else if (r == 3) {
    DFWFM_STEP(b0, a0, b2, a2, i);
    DFWFM_STEP_N(b1, a1);
    DFWFM_STEP_N(b2, a2);
  } else {
    DFWFM_STEP(b0, a0, b2, a2, i);
    DFWFM_STEP(b1, a1, b0, a0, i + 1);
    DFWFM_STEP_N(b2, a2);
    DFWFM_STEP_N(b0, a0);
  }
#undef DFWFM_STEP_N
#undef DFWFM_STEP
#undef DFWFM_MFMA_STEP
}

// mlp_k_loop with the chunk count NS fixed at compile time (every step unrolled, so each step's register
// sets are static) and the wave's share of the split tail tile riding on the same sets: the two drain steps
// (which fetch no chunk) fetch its fragments into the sets just freed, multiplied after the last step into
// tpart.  Nothing of the tail is held across the layer boundary (preloaded tail fragments spilled, and a
// spill store after the next layer's preload waits for all of it).  Needs 2 * TPW >= the wave's tail share.
template <int TPW, int NG, int NS, bool WA>
__device__ __forceinline__ void mlp_k_loop_s(f32x4 (&acc)[TPW], const float* __restrict__ act, int SA,
                                             const LayerStream<TPW, 1, NG>& ls, f32x4 (&b0)[TPW],
                                             f32x4 (&b1)[TPW], f32x4 (&b2)[TPW], int lane,
                                             const TailStream<NG>& ts, f32x4& tpart) {
  static_assert(NS >= 3, "static K loop: at least 3 chunks");
  const int voff = lane * 16;
  const float* arow = act + (lane & 15) * SA + 4 * (lane >> 4);
  float4 a0 = *reinterpret_cast<const float4*>(arow);
  float4 a1 = *reinterpret_cast<const float4*>(arow + 16);
  float4 a2;
#pragma unroll
  for (int i = 0; i < NS; ++i) {
    f32x4 (&X)[TPW] = (i % 3 == 0) ? b0 : ((i % 3 == 1) ? b1 : b2);
    f32x4 (&Z)[TPW] = (i % 3 == 0) ? b2 : ((i % 3 == 1) ? b0 : b1);
    float4& AX = (i % 3 == 0) ? a0 : ((i % 3 == 1) ? a1 : a2);
    float4& AZ = (i % 3 == 0) ? a2 : ((i % 3 == 1) ? a0 : a1);
    if (i + 2 < NS) {
      AZ = *reinterpret_cast<const float4*>(arow + 16 * (i + 2));
      ls.load(Z, ls.c0 + i + 2, voff);
    } else {
      ts.template load_set<TPW>(ls.rsrc, Z, i + 2 == NS ? 0 : TPW, voff);
    }
    mfma_chunk<TPW, WA>(acc, AX, X);
    __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
    for (int q = 0; q < TPW; ++q) {
      __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);
      __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);
    }
    __builtin_amdgcn_sched_group_barrier(0x008, 2 * TPW, 0);
    __builtin_amdgcn_sched_barrier(0);
  }
  f32x4 c0 = f32x4{0.f, 0.f, 0.f, 0.f}, c1 = c0;
  ts.template mma_set<TPW, WA>(arow, NS % 3 == 0 ? b0 : (NS % 3 == 1 ? b1 : b2), 0, c0, c1);
  ts.template mma_set<TPW, WA>(arow, (NS + 1) % 3 == 0 ? b0 : ((NS + 1) % 3 == 1 ? b1 : b2), TPW, c0, c1);
  tpart = c0 + c1;
}


// Counter-based dropout mask (deep tower; reference nn.Dropout(0.5), model/DeepFMs.py:260-282):
// keep element (layer, row, col) of a step iff the top 24 bits of a murmur3-finalised key
// (seed ^ row*K1 ^ col*K2 ^ layer*K3) / 2^24 >= p.  The same function regenerates the mask in the
// backward; oracle/torch_port.dropout_masks restates it.
__device__ __forceinline__ uint32_t mix32(uint32_t x) {
  x ^= x >> 16;
  x *= 0x85EBCA6BU;
  x ^= x >> 13;
  x *= 0xC2B2AE35U;
  x ^= x >> 16;
  return x;
}
__device__ __forceinline__ bool dropout_keep(uint32_t seed, int layer, int64_t row, int col, float p) {
  const uint32_t h =
      mix32(seed ^ ((uint32_t)row * 0x9E3779B9U) ^ ((uint32_t)col * 0x7FEB352DU) ^ ((uint32_t)layer * 0x846CA68BU));
  return (float)(h >> 8) * (1.0f / 16777216.0f) >= p;
}

// Copy rows [0, nrows) x 4*cols4 floats of an LDS tile (row stride lds_stride) to global rows of stride
// gstride (both multiples of 4 floats, 16-byte aligned bases): one float4 per lane per step.
__device__ __forceinline__ void store_tile(float* __restrict__ g, int64_t gstride, const float* __restrict__ lds,
                                           int lds_stride, int nrows, int cols4, int tid, int nth) {
  const int n = nrows * cols4;
  for (int i = tid; i < n; i += nth) {
    const int b = i / cols4;
    const int c = (i - b * cols4) * 4;
    *reinterpret_cast<float4*>(g + b * gstride + c) = *reinterpret_cast<const float4*>(lds + b * lds_stride + c);
  }
}

// Copy rows [0, nrows) x 4*cols4 floats of a global tile (row stride gstride floats) into an LDS tile
// (row stride lds_stride), zero-filling rows [nrows, kBM) and columns [4*cols4, 4*pad4): KPT float4 per
// thread in flight, every load issued before any LDS store (a load-then-store loop waits out one
// round trip per iteration).  16-byte aligned bases and strides.
template <int KPT>
__device__ __forceinline__ void load_tile(float* __restrict__ lds, int lds_stride, const float* __restrict__ g,
                                          int64_t gstride, int nrows, int cols4, int pad4, int tid, int nth) {
  const int n = kBM * pad4;
  f32x4 v[KPT];
#pragma unroll
  for (int k = 0; k < KPT; ++k) {
    const int i = tid + k * nth;
    const int b = i / pad4;
    const int c = i - b * pad4;
    v[k] = f32x4{0.f, 0.f, 0.f, 0.f};
    if (i < n && b < nrows && c < cols4) v[k] = reinterpret_cast<const f32x4*>(g + b * gstride)[c];
  }
#pragma unroll
  for (int k = 0; k < KPT; ++k) {
    const int i = tid + k * nth;
    const int b = i / pad4;
    if (i < n) reinterpret_cast<f32x4*>(lds + b * lds_stride)[i - b * pad4] = v[k];
  }
  for (int i = tid + KPT * nth; i < n; i += nth) {  // wider tiles
    const int b = i / pad4;
    const int c = i - b * pad4;
    reinterpret_cast<f32x4*>(lds + b * lds_stride)[c] =
        (b < nrows && c < cols4) ? reinterpret_cast<const f32x4*>(g + b * gstride)[c] : f32x4{0.f, 0.f, 0.f, 0.f};
  }
}

// Staged copies (load everything first, store later): stage_load reads items tid + k * nth (k < KPT) of n into
// registers through get(i); stage_store writes them through put(i, v) and copies any items past KPT * nth
// directly.  Several arrays' stage_loads issued back to back cost one round trip.
template <int KPT, class T, class Get>
__device__ __forceinline__ void stage_load(T (&v)[KPT], int n, int tid, int nth, Get get) {
#pragma unroll
  for (int k = 0; k < KPT; ++k) {
    const int i = tid + k * nth;
    v[k] = i < n ? get(i) : T{};
  }
}
template <int KPT, class T, class Get, class Put>
__device__ __forceinline__ void stage_store(const T (&v)[KPT], int n, int tid, int nth, Get get, Put put) {
#pragma unroll
  for (int k = 0; k < KPT; ++k) {
    const int i = tid + k * nth;
    if (i < n) put(i, v[k]);
  }
  for (int i = tid + KPT * nth; i < n; i += nth) put(i, get(i));
}

// load_tile split in two (the same tile, the same zero fill): tile_load issues the loads, tile_store writes LDS
template <int KPT>
__device__ __forceinline__ void tile_load(f32x4 (&v)[KPT], const float* __restrict__ g, int64_t gstride, int nrows,
                                          int cols4, int pad4, int tid, int nth) {
  const int n = kBM * pad4;
#pragma unroll
  for (int k = 0; k < KPT; ++k) {
    const int i = tid + k * nth;
    const int b = i / pad4;
    const int c = i - b * pad4;
    v[k] = f32x4{0.f, 0.f, 0.f, 0.f};
    if (i < n && b < nrows && c < cols4) v[k] = reinterpret_cast<const f32x4*>(g + b * gstride)[c];
  }
}
template <int KPT>
__device__ __forceinline__ void tile_store(float* __restrict__ lds, int lds_stride, const f32x4 (&v)[KPT],
                                           const float* __restrict__ g, int64_t gstride, int nrows, int cols4,
                                           int pad4, int tid, int nth) {
  const int n = kBM * pad4;
#pragma unroll
  for (int k = 0; k < KPT; ++k) {
    const int i = tid + k * nth;
    const int b = i / pad4;
    if (i < n) reinterpret_cast<f32x4*>(lds + b * lds_stride)[i - b * pad4] = v[k];
  }
  for (int i = tid + KPT * nth; i < n; i += nth) {  // wider tiles
    const int b = i / pad4;
    const int c = i - b * pad4;
    reinterpret_cast<f32x4*>(lds + b * lds_stride)[c] =
        (b < nrows && c < cols4) ? reinterpret_cast<const f32x4*>(g + b * gstride)[c] : f32x4{0.f, 0.f, 0.f, 0.f};
  }
}

// Dropout seed of a step: the host's seed, or -- for graph-replayed steps -- that seed mixed with a
// device step counter (read at kernel time, so every replay draws fresh masks).
__device__ __forceinline__ uint32_t step_seed(uint32_t base, const int64_t* src) {
  if (src == nullptr) return base;
  const uint32_t step = (uint32_t)*src;
  return base ^ mix32(step * 0x9E3779B9U + 0x7F4A7C15U);
}

}  // namespace dfwfm
