// dfwfm_kernels.hip -- CDNA4 (gfx950) kernels for the DeepFwFM forward.
//
// One fused launch computes the whole forward of reference
// model/DeepFMs.py:285-469 for a tile of BM = 16 samples:
//
//   phase G  gather: 26 categorical rows (plain nn.Embedding / EmbeddingBag,
//            or QR quotient x remainder, model/QREmbeddingBag.py:156-174) and
//            13 numerical rows v_f[0] * Xv (model/DeepFMs.py:297-299,334) into
//            an LDS tile E[16][F*D] -- this IS deep_emb (field-major `cat`,
//            model/DeepFMs.py:398) and the `stack` of :337;
//   phase S  shallow part from LDS: first order (per-field tables :304, or
//            fwlw :338-347) projected by lw (:445-450) or summed, and the
//            FwFM second order sum_{k<l} r_kl <E_k, E_l> (:352-367) over a
//            compact list of non-zero symmetric pairs (pruned R => fewer pairs);
//   phase M  the h_depth x N ReLU MLP (:412-428) on f32 MFMA
//            (v_mfma_f32_16x16x4_f32, exact f32 fma chain): activations stay
//            in LDS, weights stream from L2 in a pre-packed fragment order
//            (one 1 KiB dwordx4 load per wave per 16-deep K chunk per tile),
//            bias+ReLU fused into the epilogue, net_1_fc fused into the last
//            layer's epilogue;
//   combine  total = ((first + second) + deep) + bias   (:458 order).
//
// Nothing of the reference's [39,39,B,10] outer-product intermediates exists.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "dfwfm_internal.h"

namespace dfwfm {

typedef float f32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ float relu_keep_nan(float v) { return v < 0.f ? 0.f : v; }

// ---------------------------------------------------------------------------
// phase G helpers
// ---------------------------------------------------------------------------
template <int D>
__device__ __forceinline__ void copy_row(float* __restrict__ dst, const float* __restrict__ src) {
  if constexpr (D % 4 == 0) {
#pragma unroll
    for (int d = 0; d < D; d += 4) *reinterpret_cast<float4*>(dst + d) = *reinterpret_cast<const float4*>(src + d);
  } else if constexpr (D % 2 == 0) {
#pragma unroll
    for (int d = 0; d < D; d += 2) *reinterpret_cast<float2*>(dst + d) = *reinterpret_cast<const float2*>(src + d);
  } else {
#pragma unroll
    for (int d = 0; d < D; ++d) dst[d] = src[d];
  }
}

template <int D>
__device__ __forceinline__ void combine_rows(float* __restrict__ dst, const float* __restrict__ q,
                                             const float* __restrict__ r, int op) {
  float a[D], b[D];
  if constexpr (D % 2 == 0) {
#pragma unroll
    for (int d = 0; d < D; d += 2) {
      float2 x = *reinterpret_cast<const float2*>(q + d);
      float2 y = *reinterpret_cast<const float2*>(r + d);
      a[d] = x.x; a[d + 1] = x.y; b[d] = y.x; b[d + 1] = y.y;
    }
  } else {
#pragma unroll
    for (int d = 0; d < D; ++d) { a[d] = q[d]; b[d] = r[d]; }
  }
  // QREmbeddingBag: embed_q * embed_r ('mult') or embed_q + embed_r ('add')
#pragma unroll
  for (int d = 0; d < D; ++d) dst[d] = (op == 0) ? a[d] * b[d] : a[d] + b[d];
}

// ---------------------------------------------------------------------------
// phase M: one MLP layer for the workgroup's 16 rows.
//   act   : LDS [16][SA] input activations (K padded with zeros to NC*16)
//   wl    : packed weights of this layer, [NT][NC][64 lanes] float4
//   wave w owns output tiles w, w+4, ... (TPW of them; tiles past NT are
//   clamped duplicates whose results are discarded -- they ride on a SIMD
//   that would otherwise idle at the layer barrier).
// Fragment algebra (16x16x4 f32): in sub-step s of chunk c lane l supplies
//   A = act[l&15][16c + 4(l>>4) + s],  B = W[n0 + (l&15)][16c + 4(l>>4) + s],
// so one ds_read_b128 (A) and one dwordx4 per tile (B) feed 4 MFMAs.
// ---------------------------------------------------------------------------
template <int TPW>
__device__ __forceinline__ void mlp_layer(const float* __restrict__ act, int SA, int NC,
                                          const float4* __restrict__ wl, int NT, int N,
                                          const float* __restrict__ bias, float* __restrict__ out_act,
                                          int SO, const float* __restrict__ fc, float (&dpart)[4],
                                          bool last, int wave, int lane) {
  const float4* wp[TPW];
#pragma unroll
  for (int j = 0; j < TPW; ++j) {
    int t = wave + 4 * j;
    t = t < NT ? t : NT - 1;
    wp[j] = wl + (size_t)t * NC * 64 + lane;
  }
  f32x4 acc[TPW];
#pragma unroll
  for (int j = 0; j < TPW; ++j) acc[j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const float* arow = act + (lane & 15) * SA + 4 * (lane >> 4);

  // two chunks of weight fragments in flight ahead of the MFMAs
  float4 b0[TPW], b1[TPW];
  const int c1 = NC > 1 ? 1 : 0;
#pragma unroll
  for (int j = 0; j < TPW; ++j) b0[j] = wp[j][0];
#pragma unroll
  for (int j = 0; j < TPW; ++j) b1[j] = wp[j][(size_t)c1 * 64];

  for (int c = 0; c < NC; ++c) {
    const float4 a = *reinterpret_cast<const float4*>(arow + 16 * c);
    int cn = c + 2;
    cn = cn < NC ? cn : NC - 1;  // clamped: the tail re-loads a resident chunk, never branches
    float4 b2[TPW];
#pragma unroll
    for (int j = 0; j < TPW; ++j) b2[j] = wp[j][(size_t)cn * 64];
#pragma unroll
    for (int j = 0; j < TPW; ++j) {
      acc[j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a.x, b0[j].x, acc[j], 0, 0, 0);
      acc[j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a.y, b0[j].y, acc[j], 0, 0, 0);
      acc[j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a.z, b0[j].z, acc[j], 0, 0, 0);
      acc[j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a.w, b0[j].w, acc[j], 0, 0, 0);
    }
#pragma unroll
    for (int j = 0; j < TPW; ++j) { b0[j] = b1[j]; b1[j] = b2[j]; }
  }

  // epilogue: C/D layout col = lane&15, row = (lane>>4)*4 + r
  const int row0 = (lane >> 4) * 4;
#pragma unroll
  for (int j = 0; j < TPW; ++j) {
    const int t = wave + 4 * j;
    if (t < NT) {
      const int n = t * 16 + (lane & 15);
      const bool valid = n < N;
      const float bn = valid ? bias[n] : 0.f;
      if (!last) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float v = valid ? relu_keep_nan(acc[j][r] + bn) : 0.f;
          out_act[(row0 + r) * SO + n] = v;
        }
      } else {
        const float w = valid ? fc[n] : 0.f;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float v = valid ? relu_keep_nan(acc[j][r] + bn) : 0.f;
          dpart[r] = fmaf(v, w, dpart[r]);
        }
      }
    }
  }
}

// ---------------------------------------------------------------------------
// the fused forward kernel
// ---------------------------------------------------------------------------
template <int D, int TPW>
__global__ void __launch_bounds__(kWG) fwd_kernel(FwdArgs p) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int F = p.F;
  const int num = p.num;
  const int SX = p.SX;
  const int SY = p.SY;
  const bool deep = (p.flags & kHasDeep) != 0;

  float* bufX = smem;                                   // [BM][SX]  E tile / even-layer input
  float* bufY = bufX + kBM * SX;                        // [BM][SY]  odd-layer input (deep only)
  float* fo = bufY + (deep ? kBM * SY : 0);             // [BM][F]   first order per field
  float* part2 = fo + kBM * F;                          // [BM][D]   second order per dim
  float* dsum = part2 + kBM * D;                        // [4][BM]   deep partial per wave
  float* fs = dsum + 4 * kBM;                           // [BM]      first + second

  const int64_t b0 = (int64_t)blockIdx.x * kBM;
  const int ncat = F - num;
  const int kpad0 = p.NC0 * 16;
  const bool fo_tables = (p.flags & kFoTables) != 0;

  // ---- phase G: gather E (and table first order) into LDS -----------------
  for (int r = tid; r < kBM * F; r += kWG) {
    const int b = r / F;
    const int f = r - b * F;
    const int64_t gb = b0 + b;
    float* dst = bufX + b * SX + f * D;
    float fo_v = 0.f;
    if (gb >= p.batch) {
#pragma unroll
      for (int d = 0; d < D; ++d) dst[d] = 0.f;
    } else {
      const FieldDev fd = p.fields[f];
      if (f < num) {
        const float x = p.xv[gb * p.xv_stride + f];
#pragma unroll
        for (int d = 0; d < D; ++d) dst[d] = fd.emb2[d] * x;
        if (fo_tables) fo_v = fd.emb1[0] * x;
      } else {
        int64_t idx = p.xi[gb * p.xi_stride + (f - num)];
        if (idx < 0 || idx >= fd.n) {
          atomicOr(p.err, DFWFM_FLAG_INDEX_OUT_OF_RANGE);
          idx = 0;
        }
        if (fd.c == 0) {
          copy_row<D>(dst, fd.emb2 + idx * D);
          if (fo_tables) fo_v = fd.emb1[idx];
        } else {
          const int64_t q = idx / fd.c;
          const int64_t rr = idx - q * fd.c;
          combine_rows<D>(dst, fd.emb2 + q * D, fd.emb2_r + rr * D, fd.op);
          if (fo_tables) {
            const float x = fd.emb1[q], y = fd.emb1_r[rr];
            fo_v = (fd.op == 0) ? x * y : x + y;
          }
        }
      }
    }
    fo[b * F + f] = fo_v;
  }
  // zero the K padding of the E tile (layer-0 reads NC0*16 columns)
  for (int r = tid; r < kBM * (kpad0 - F * D); r += kWG) {
    const int w = kpad0 - F * D;
    const int b = r / w;
    bufX[b * SX + F * D + (r - b * w)] = 0.f;
  }
  __syncthreads();

  // ---- phase S: shallow part ----------------------------------------------
  if (p.flags & kFoFwlw) {
    // fm_first_order[b, f] = sum_d E[b, f, d] * Wfl[f, d]  (einsum 'ijk,ik->ijk' then 'ijk->ji')
    for (int r = tid; r < kBM * F; r += kWG) {
      const int b = r / F;
      const int f = r - b * F;
      const float* e = bufX + b * SX + f * D;
      const float* w = p.fwlw + f * D;
      float s = 0.f;
#pragma unroll
      for (int d = 0; d < D; ++d) s += e[d] * w[d];
      fo[r] = s;
    }
  }
  if (p.flags & kHasSecond) {
    // second[b, d] = sum over pairs k<l with r_kl != 0 of (E_k[d] * E_l[d]) * r_kl
    const int np = *p.npairs;
    for (int r = tid; r < kBM * D; r += kWG) {
      const int b = r / D;
      const int d = r - b * D;
      const float* e = bufX + b * SX + d;
      float acc = 0.f;
      for (int q = 0; q < np; ++q) {
        const Pair pr = p.pairs[q];
        acc = fmaf(e[pr.k * D] * e[pr.l * D], pr.r, acc);
      }
      part2[r] = acc;
    }
  }
  __syncthreads();
  if (tid < kBM) {
    float first = 0.f;
    if (p.flags & kFoLw) {
      for (int f = 0; f < F; ++f) first = fmaf(fo[tid * F + f], p.lw[f], first);
    } else {
      for (int f = 0; f < F; ++f) first += fo[tid * F + f];
    }
    float second = 0.f;
    if (p.flags & kHasSecond) {
#pragma unroll
      for (int d = 0; d < D; ++d) second += part2[tid * D + d];
    }
    fs[tid] = first + second;
  }

  if (!deep) {
    __syncthreads();
    if (tid < kBM && b0 + tid < p.batch) {
      float t = fs[tid];
      if (p.bias) t += p.bias[0];
      p.out[b0 + tid] = t;
    }
    return;
  }

  // ---- phase M: MLP on MFMA -------------------------------------------------
  float dpart[4] = {0.f, 0.f, 0.f, 0.f};
  const float4* wl = p.wpack;
  for (int h = 0; h < p.H; ++h) {
    const bool even = (h & 1) == 0;
    const float* in = even ? bufX : bufY;
    const int SA = even ? SX : SY;
    float* out = even ? bufY : bufX;
    const int SO = even ? SY : SX;
    const int NC = h == 0 ? p.NC0 : p.NT;
    const bool last = h == p.H - 1;
    mlp_layer<TPW>(in, SA, NC, wl, p.NT, p.N, p.mlp_b + (size_t)h * p.NT * 16, out, SO, p.fc, dpart,
                   last, wave, lane);
    wl += (size_t)p.NT * NC * 64;
    __syncthreads();
  }

  // deep[b] = sum_n h_last[b, n] * fc[n]: reduce the 16 lanes sharing (lane>>4), then the 4 waves
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    float v = dpart[r];
    v += __shfl_xor(v, 8);
    v += __shfl_xor(v, 4);
    v += __shfl_xor(v, 2);
    v += __shfl_xor(v, 1);
    dpart[r] = v;
  }
  if ((lane & 15) == 0) {
#pragma unroll
    for (int r = 0; r < 4; ++r) dsum[wave * kBM + (lane >> 4) * 4 + r] = dpart[r];
  }
  __syncthreads();
  if (tid < kBM && b0 + tid < p.batch) {
    const float deepv = ((dsum[tid] + dsum[kBM + tid]) + dsum[2 * kBM + tid]) + dsum[3 * kBM + tid];
    float t = fs[tid] + deepv;
    if (p.bias) t += p.bias[0];
    p.out[b0 + tid] = t;
  }
}

// ---------------------------------------------------------------------------
// dense-parameter packing (run on weight updates, not per forward)
// ---------------------------------------------------------------------------

// W [N][K] row-major (nn.Linear.weight) -> [NT][NC][64][4] fragment order
__global__ void pack_linear_kernel(const float* __restrict__ w, int N, int K, int NT, int NC,
                                   float4* __restrict__ out) {
  const int64_t total = (int64_t)NT * NC * 64;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int lane = (int)(i & 63);
    const int64_t tc = i >> 6;
    const int c = (int)(tc % NC);
    const int t = (int)(tc / NC);
    const int n = t * 16 + (lane & 15);
    const int k0 = 16 * c + 4 * (lane >> 4);
    float v[4];
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      const int k = k0 + s;
      v[s] = (n < N && k < K) ? w[(int64_t)n * K + k] : 0.f;
    }
    out[i] = make_float4(v[0], v[1], v[2], v[3]);
  }
}

// dst[i] = i < n ? src[i] : 0 for i < npad (src may be null => zeros)
__global__ void pad_copy_kernel(const float* __restrict__ src, int n, int npad, float* __restrict__ dst) {
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < npad; i += gridDim.x * blockDim.x)
    dst[i] = (src && i < n) ? src[i] : 0.f;
}

// Compact list of the non-zero upper-triangle entries of R_sym = (R^T + R) * 0.5
// (model/DeepFMs.py:363-364), in (k, l) order.  mode 1 = FM (all ones).
// One workgroup of 1024 threads; ballot + LDS prefix keeps the order stable.
__global__ void __launch_bounds__(1024) build_pairs_kernel(const float* __restrict__ R, int F, int mode,
                                                           Pair* __restrict__ pairs,
                                                           int32_t* __restrict__ npairs) {
  __shared__ int wave_cnt[16];
  __shared__ int base_s;
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  if (tid == 0) base_s = 0;
  __syncthreads();
  const int total = F * F;
  for (int start = 0; start < total; start += 1024) {
    const int i = start + tid;
    int k = 0, l = 0;
    float r = 0.f;
    bool keep = false;
    if (i < total) {
      k = i / F;
      l = i - k * F;
      if (l > k) {
        r = (mode == 1) ? 1.f : (R[l * F + k] + R[k * F + l]) * 0.5f;
        keep = r != 0.f;
      }
    }
    const unsigned long long m = __ballot(keep);
    const int before = __popcll(m & ((1ull << lane) - 1ull));
    if (lane == 0) wave_cnt[wave] = __popcll(m);
    __syncthreads();
    int off = base_s;
    for (int w = 0; w < wave; ++w) off += wave_cnt[w];
    if (keep) {
      Pair pr;
      pr.k = (int16_t)k;
      pr.l = (int16_t)l;
      pr.r = r;
      pairs[off + before] = pr;
    }
    __syncthreads();
    if (tid == 0) {
      int s = 0;
      for (int w = 0; w < 16; ++w) s += wave_cnt[w];
      base_s += s;
    }
    __syncthreads();
  }
  if (tid == 0) *npairs = base_s;
}

// ---------------------------------------------------------------------------
// launchers
// ---------------------------------------------------------------------------
template <int D, int TPW>
static hipError_t launch_fwd_t(const FwdArgs& a, size_t lds, hipStream_t s) {
  auto k = fwd_kernel<D, TPW>;
  if (lds > 65536) {
    hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(k),
                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return e;
  }
  const unsigned grid = (unsigned)((a.batch + kBM - 1) / kBM);
  hipLaunchKernelGGL(k, dim3(grid), dim3(kWG), lds, s, a);
  return hipGetLastError();
}

template <int D>
static hipError_t launch_fwd_d(const FwdArgs& a, int tpw, size_t lds, hipStream_t s) {
  switch (tpw) {
    case 1: return launch_fwd_t<D, 1>(a, lds, s);
    case 2: return launch_fwd_t<D, 2>(a, lds, s);
    case 3: return launch_fwd_t<D, 3>(a, lds, s);
    case 4: return launch_fwd_t<D, 4>(a, lds, s);
    case 5: return launch_fwd_t<D, 5>(a, lds, s);
    case 6: return launch_fwd_t<D, 6>(a, lds, s);
    case 7: return launch_fwd_t<D, 7>(a, lds, s);
    case 8: return launch_fwd_t<D, 8>(a, lds, s);
    default: return hipErrorInvalidValue;
  }
}

bool supported_embedding_size(int D) {
  return D == 4 || D == 8 || D == 10 || D == 16 || D == 32;
}

hipError_t launch_forward(const FwdArgs& a, int D, int tpw, size_t lds, hipStream_t s) {
  switch (D) {
    case 4: return launch_fwd_d<4>(a, tpw, lds, s);
    case 8: return launch_fwd_d<8>(a, tpw, lds, s);
    case 10: return launch_fwd_d<10>(a, tpw, lds, s);
    case 16: return launch_fwd_d<16>(a, tpw, lds, s);
    case 32: return launch_fwd_d<32>(a, tpw, lds, s);
    default: return hipErrorInvalidValue;
  }
}

hipError_t launch_pack_linear(const float* w, int N, int K, int NT, int NC, float4* out, hipStream_t s) {
  const int64_t total = (int64_t)NT * NC * 64;
  const unsigned grid = (unsigned)((total + 255) / 256 < 4096 ? (total + 255) / 256 : 4096);
  hipLaunchKernelGGL(pack_linear_kernel, dim3(grid), dim3(256), 0, s, w, N, K, NT, NC, out);
  return hipGetLastError();
}

hipError_t launch_pad_copy(const float* src, int n, int npad, float* dst, hipStream_t s) {
  if (npad <= 0) return hipSuccess;
  const unsigned grid = (unsigned)((npad + 255) / 256 < 1024 ? (npad + 255) / 256 : 1024);
  hipLaunchKernelGGL(pad_copy_kernel, dim3(grid), dim3(256), 0, s, src, n, npad, dst);
  return hipGetLastError();
}

hipError_t launch_build_pairs(const float* R, int F, int mode, Pair* pairs, int32_t* npairs, hipStream_t s) {
  hipLaunchKernelGGL(build_pairs_kernel, dim3(1), dim3(1024), 0, s, R, F, mode, pairs, npairs);
  return hipGetLastError();
}

}  // namespace dfwfm
