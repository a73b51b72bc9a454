// dfwfm_spmlp.hip -- the deep tower over magnitude-pruned weights (BASELINE configs[3]: every
// net_1_linear_*.weight 90 % zero after the reference's masks, model/DeepFMs.py:647-673).
//
// The reference keeps the pruned forward dense (utils/util.py:49-51 discards to_sparse()), and so does
// fwd_kernel: at 10 % density no 16x4 weight block of an MFMA operand is all zero (0.9^64), so the
// matrix cores cannot skip anything.  This path instead runs the MLP on the vector ALUs over the
// nonzeros only:
//
//   ell_build_kernel   per layer, each neuron's nonzero (k, w) pairs compacted in k order (one wave per
//                      row, ballot + mbcnt), padded with (0, 0) to a multiple of kEllPad; run once per
//                      weight update (dfwfm_model_build_sparse_mlp), not per forward;
//   sparse_mlp_kernel  64 samples per workgroup (lane = sample), the E tile of the gather launch
//                      (fwd_kernel PART = 1) transposed into LDS as x[k][64]; eight waves own neurons
//                      n = wave + 8i, each neuron's pairs come in as scalar loads (wave-uniform), and a
//                      pair costs one LDS read of x[k][lane] plus one FMA -- 47.6 k FMAs per sample at
//                      Criteo-39 / 90 % instead of the dense 476 k; a layer's outputs stay in registers
//                      until every wave has finished reading x, then overwrite it in place; net_1_fc and
//                      the combine ((first + second) + deep) + bias are fused into the last layer.
//
// The sums run in k order from the bias (a different association from the dense MFMA chain; parity is
// the 1e-5 logit bar, tests/test_gpu_sparse.py).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "dfwfm_internal.h"

namespace dfwfm {

namespace {
constexpr int kSpS = 64;  // samples per workgroup (lane = sample)
constexpr int kSpW = 8;   // waves per workgroup
}  // namespace

__global__ void __launch_bounds__(64) ell_build_kernel(const EllArgs a) {
  const int row = blockIdx.x;
  const int l = row / a.N;
  const int n = row - l * a.N;
  const int lane = threadIdx.x;
  const int K = a.K[l];
  const float* w = a.w[l] + (int64_t)n * K;
  int2* e = a.ell + a.off[l] + (int64_t)n * a.W[l];
  int c = 0;
  for (int k0 = 0; k0 < K; k0 += 64) {
    const int k = k0 + lane;
    const float v = k < K ? w[k] : 0.f;
    const bool nz = v != 0.f;  // NaN is kept, +-0 dropped
    const uint64_t mask = __builtin_amdgcn_ballot_w64(nz);
    const int pos = c + (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(mask >> 32),
                                                       __builtin_amdgcn_mbcnt_lo((uint32_t)mask, 0));
    if (nz) e[pos] = make_int2(k, __float_as_int(v));
    c += __builtin_popcountll(mask);
  }
  const int cp = (c + kEllPad - 1) / kEllPad * kEllPad;
  for (int j = c + lane; j < cp; j += 64) e[j] = make_int2(0, 0);
  if (lane == 0) {
    a.cnt[l * a.N + n] = cp;
    atomicMax(&a.stat[0], c);
    atomicAdd(&a.stat[1], c);
  }
}

template <int NPW>
__global__ void __launch_bounds__(64 * kSpW) sparse_mlp_kernel(const SpMlpArgs p) {
  extern __shared__ __attribute__((aligned(16))) float x[];  // [max(K0p, N)][64], then red [kSpW][64]
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int64_t b0 = (int64_t)blockIdx.x * kSpS;
  const int nrows = (int)((p.batch - b0) < kSpS ? (p.batch - b0) : kSpS);
  const int N = p.N;
  const int XK = p.K0p > N ? p.K0p : N;
  float* red = x + XK * kSpS;

  // E tile (the gather launch's [B][K0p] rows, zero padded past F*D) -> x[k][b]: lane = sample, each wave
  // a set of 16-byte column chunks; every load in flight before the LDS stores (conflict-free: consecutive
  // lanes write consecutive words)
  {
    constexpr int kCh = 16;  // chunks per wave per pass
    const int nch = p.K0p >> 2;
    const float* src = p.part_e + (b0 + (lane < nrows ? lane : 0)) * p.part_stride;
    for (int c0 = wave; c0 < nch; c0 += kSpW * kCh) {
      float4 v[kCh];
#pragma unroll
      for (int u = 0; u < kCh; ++u) {
        const int c = c0 + u * kSpW;
        v[u] = c < nch ? *reinterpret_cast<const float4*>(src + 4 * c) : make_float4(0.f, 0.f, 0.f, 0.f);
      }
#pragma unroll
      for (int u = 0; u < kCh; ++u) {
        const int c = c0 + u * kSpW;
        if (c < nch) {
          const bool live = lane < nrows;
          x[(4 * c + 0) * kSpS + lane] = live ? v[u].x : 0.f;
          x[(4 * c + 1) * kSpS + lane] = live ? v[u].y : 0.f;
          x[(4 * c + 2) * kSpS + lane] = live ? v[u].z : 0.f;
          x[(4 * c + 3) * kSpS + lane] = live ? v[u].w : 0.f;
        }
      }
    }
  }
  __syncthreads();

  float dpart = 0.f;
  for (int h = 0; h < p.H; ++h) {
    const int2* ell = p.ell + p.off[h];
    const int W = p.W[h];
    const int* cnt = p.cnt + h * N;
    const float* bh = p.mlp_b + h * p.NT * 16;
    const bool last = h == p.H - 1;
    float acc[NPW];
#pragma unroll
    for (int i = 0; i < NPW; ++i) {
      const int n = wave + kSpW * i;
      acc[i] = 0.f;
      if (n < N) {
        float a = bh[n];
        const int2* e = ell + (int64_t)n * W;
        const int c = cnt[n];
        for (int j = 0; j < c; j += kEllPad) {
          int2 q[kEllPad];
#pragma unroll
          for (int u = 0; u < kEllPad; ++u) q[u] = e[j + u];
#pragma unroll
          for (int u = 0; u < kEllPad; ++u) a = fmaf(__int_as_float(q[u].y), x[q[u].x * kSpS + lane], a);
        }
        const float r = a < 0.f ? 0.f : a;  // ReLU (NaN kept, as relu_keep_nan)
        acc[i] = r;
        if (last) dpart = fmaf(r, p.fc[n], dpart);
      }
    }
    if (!last) {
      __syncthreads();  // every wave has finished reading this layer's input
#pragma unroll
      for (int i = 0; i < NPW; ++i) {
        const int n = wave + kSpW * i;
        if (n < N) x[n * kSpS + lane] = acc[i];
      }
      __syncthreads();
    }
  }
  red[wave * kSpS + lane] = dpart;
  __syncthreads();
  if (wave == 0 && lane < nrows) {
    float deep = red[lane];
#pragma unroll
    for (int w = 1; w < kSpW; ++w) deep += red[w * kSpS + lane];
    p.out[b0 + lane] = (p.part_fs[b0 + lane] + deep) + p.bias[0];
  }
}

hipError_t launch_ell_build(const EllArgs& a, int rows, hipStream_t s) {
  if (rows <= 0) return hipSuccess;
  hipLaunchKernelGGL(ell_build_kernel, dim3(rows), dim3(64), 0, s, a);
  return hipGetLastError();
}

size_t sparse_mlp_lds_bytes(int K0p, int N) {
  const int XK = K0p > N ? K0p : N;
  return sizeof(float) * ((size_t)XK * kSpS + kSpW * kSpS);
}

template <int NPW>
static hipError_t launch_sp_t(const SpMlpArgs& a, hipStream_t s) {
  const size_t lds = sparse_mlp_lds_bytes(a.K0p, a.N);
  auto k = sparse_mlp_kernel<NPW>;
  hipError_t e = ensure_lds_limit(reinterpret_cast<const void*>(k), lds);
  if (e != hipSuccess) return e;
  const unsigned grid = (unsigned)((a.batch + kSpS - 1) / kSpS);
  hipLaunchKernelGGL(k, dim3(grid), dim3(64 * kSpW), lds, s, a);
  return hipGetLastError();
}

hipError_t launch_sparse_mlp(const SpMlpArgs& a, hipStream_t s) {
  const int npw = (a.N + kSpW - 1) / kSpW;
  if (npw <= 16) return launch_sp_t<16>(a, s);
  if (npw <= 32) return launch_sp_t<32>(a, s);
  if (npw <= 48) return launch_sp_t<48>(a, s);
  if (npw <= 64) return launch_sp_t<64>(a, s);
  return hipErrorInvalidValue;
}

}  // namespace dfwfm
