// dfwfm_spmlp.hip -- the deep tower over magnitude-pruned weights (BASELINE configs[3]: every
// net_1_linear_*.weight 90 % zero after the reference's masks, model/DeepFMs.py:647-673).
//
// The reference keeps the pruned forward dense (utils/util.py:49-51 discards to_sparse()), and so does
// fwd_kernel: at 10 % density no 16x4 weight block of an MFMA operand is all zero (0.9^64), so the
// matrix cores cannot skip anything.  This path instead runs the MLP on the vector ALUs over the
// nonzeros only:
//
//   ell_build_kernel   per layer and group of four neurons, each neuron's nonzero (k, w) pairs compacted
//                      in k order (one wave per group, ballot + mbcnt), interleaved [entry][neuron] and
//                      padded with (0, 0) to the group's longest row; run once per weight update
//                      (dfwfm_model_build_sparse_mlp), not per forward;
//   sparse_mlp_kernel  64 samples per workgroup (lane = sample), the E tile of the gather launch
//                      (fwd_kernel PART = 1) transposed into LDS as x[k][64]; eight waves own neuron
//                      groups g = wave + 8i, a group's entries staged through the wave's LDS slot (loaded
//                      one unit ahead, read back as broadcasts: 32 pairs per step, all LDS reads in flight
//                      before the FMAs), and a
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
constexpr int kSpS = 64;   // samples per workgroup (lane = sample)
constexpr int kSpW = 8;    // waves per workgroup
constexpr int kSpCap = 64;  // ELL entries (of four neurons) a wave stages in LDS at once
}  // namespace

// one wave per group of four neurons 4g..4g+3: each row's nonzeros compacted in k order (ballot + mbcnt),
// written interleaved [entry j][neuron u] into the group's fixed slot, the shorter rows padded with
// (0, 0) up to the group's longest row rounded to kEllPad
__global__ void __launch_bounds__(64) ell_build_kernel(const EllArgs a) {
  const int G = (a.N + 3) / 4;
  const int row = blockIdx.x;
  const int l = row / G;
  const int g = row - l * G;
  const int lane = threadIdx.x;
  const int K = a.K[l];
  int2* e = a.ell + a.off[l] + (int64_t)g * a.W[l] * 4;
  int cnt[4];  // wave-uniform (popcounts of ballots)
  int cmax = 0, total = 0;
  for (int u = 0; u < 4; ++u) {
    const int n = 4 * g + u;
    int c = 0;
    if (n < a.N) {
      const float* w = a.w[l] + (int64_t)n * K;
      for (int k0 = 0; k0 < K; k0 += 64) {
        const int k = k0 + lane;
        const float v = k < K ? w[k] : 0.f;
        const bool nz = v != 0.f;  // NaN is kept, +-0 dropped
        const uint64_t mask = __builtin_amdgcn_ballot_w64(nz);
        const int pos = c + (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(mask >> 32),
                                                           __builtin_amdgcn_mbcnt_lo((uint32_t)mask, 0));
        if (nz) {
          int* slot = reinterpret_cast<int*>(e) + (pos * 2 + (u >> 1)) * 4 + (u & 1);
          slot[0] = k;
          slot[2] = __float_as_int(v);
        }
        c += __builtin_popcountll(mask);
      }
      if (lane == 0) a.cnt[l * a.N + n] = c;
    }
    cnt[u] = c;
    cmax = c > cmax ? c : cmax;
    total += c;
  }
  const int cp = (cmax + kEllPad - 1) / kEllPad * kEllPad;
  // pad every row of the group from its own count up to cp
  for (int u = 0; u < 4; ++u)
    for (int j = cnt[u] + lane; j < cp; j += 64) {
      int* slot = reinterpret_cast<int*>(e) + (j * 2 + (u >> 1)) * 4 + (u & 1);
      slot[0] = 0;
      slot[2] = 0;
    }
  if (lane == 0) {
    a.gcnt[l * G + g] = cp;
    atomicMax(&a.stat[0], cmax);
    atomicAdd(&a.stat[1], total);
  }
}

// NGW: neuron groups (of four) per wave, >= ceil(ceil(N/4) / kSpW)
template <int NGW>
__global__ void __launch_bounds__(64 * kSpW) __attribute__((amdgpu_waves_per_eu(2)))
sparse_mlp_kernel(const SpMlpArgs p) {
  extern __shared__ __attribute__((aligned(16))) float x[];  // [max(K0p, N)][64], then red [kSpW][64]
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int64_t b0 = (int64_t)blockIdx.x * kSpS;
  const int nrows = (int)((p.batch - b0) < kSpS ? (p.batch - b0) : kSpS);
  const int N = p.N;
  const int G = (N + 3) / 4;
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
  // each wave's ELL entries come through its own LDS slot: a unit (group g, entries [j0, j0 + n), n <= kSpCap)
  // is loaded into registers (every lane 16 bytes, coalesced) while the previous unit is processed, then stored to
  // the slot, where the walk reads it with broadcast LDS reads -- no global-memory round trip inside the walk
  const int cap = p.ecap;  // entries per unit (<= kSpCap)
  int4* eslot = reinterpret_cast<int4*>(red + kSpW * kSpS) + wave * (2 * cap);
  constexpr int kRegs = 2 * kSpCap / 64;  // int4 per lane per unit (at most)
  for (int h = 0; h < p.H; ++h) {
    const int4* ell = reinterpret_cast<const int4*>(p.ell + p.off[h]);
    const int64_t W2 = (int64_t)p.W[h] * 2;  // int4 per group slot (W entries x 4 neurons x 8 bytes)
    const int* gcnt = p.gcnt + h * G;
    const float* bh = p.mlp_b + h * p.NT * 16;
    const bool last = h == p.H - 1;
    float acc[NGW][4];
#pragma unroll
    for (int i = 0; i < NGW; ++i)
#pragma unroll
      for (int u = 0; u < 4; ++u) acc[i][u] = 0.f;
    // units of this wave: groups g = wave + kSpW i, each in chunks of kSpCap entries
    int ui = 0, uj = 0;  // next unit to load: group index i, first entry
    auto unit_n = [&](int i, int j) -> int {
      const int g = wave + kSpW * i;
      if (i >= NGW || g >= G) return -1;
      const int c = gcnt[g];
      return c - j < cap ? c - j : cap;
    };
    int4 rq[kRegs];
    auto load_unit = [&](int i, int j, int n) {
      const int4* src = ell + (int64_t)(wave + kSpW * i) * W2 + 2 * j;
#pragma unroll
      for (int r = 0; r < kRegs; ++r) {
        const int q = lane + 64 * r;
        if (q < 2 * n) rq[r] = src[q];
      }
    };
    int cur_n = unit_n(0, 0);
    if (cur_n >= 0) load_unit(0, 0, cur_n);
    int ci = 0, cj = 0;  // unit being processed
    typedef float f32x2 __attribute__((ext_vector_type(2)));
    f32x2 a01 = {0.f, 0.f}, a23 = {0.f, 0.f};
    if (cur_n >= 0) {
      const int g0 = wave;
      a01 = f32x2{bh[4 * g0], bh[4 * g0 + 1]};  // padded biases: zero past N
      a23 = f32x2{bh[4 * g0 + 2], bh[4 * g0 + 3]};
    }
    while (cur_n >= 0) {
      // the unit's entries -> this wave's slot (the previous unit's broadcast reads retired in order)
#pragma unroll
      for (int r = 0; r < kRegs; ++r) {
        const int q = lane + 64 * r;
        if (q < 2 * cur_n) eslot[q] = rq[r];
      }
      // the following unit's loads go out now
      int ni = ci, nj = cj + cur_n;
      int nn = nj < gcnt[wave + kSpW * ci] ? unit_n(ni, nj) : -1;
      if (nn < 0) {
        ni = ci + 1;
        nj = 0;
        nn = unit_n(ni, 0);
      }
      if (nn >= 0) load_unit(ni, nj, nn);
      // walk: eight entries (32 pairs) per step, every LDS read of the step in flight before its FMAs
      for (int j = 0; j < cur_n; j += 8) {
        int4 q[16];
#pragma unroll
        for (int t = 0; t < 16; ++t) q[t] = eslot[2 * j + t];
        f32x2 xv[16];
#pragma unroll
        for (int t = 0; t < 16; ++t) xv[t] = f32x2{x[q[t].x * kSpS + lane], x[q[t].y * kSpS + lane]};
#pragma unroll
        for (int t = 0; t < 16; ++t) {
          const f32x2 w = {__int_as_float(q[t].z), __int_as_float(q[t].w)};
          if (t & 1) a23 = __builtin_elementwise_fma(w, xv[t], a23);
          else a01 = __builtin_elementwise_fma(w, xv[t], a01);
        }
      }
      if (ni != ci) {
        // group done: ReLU, the last layer's net_1_fc, the register copy for the in-place overwrite
        const int g = wave + kSpW * ci;
        const float av[4] = {a01.x, a01.y, a23.x, a23.y};
#pragma unroll
        for (int i = 0; i < NGW; ++i)
          if (i == ci) {
#pragma unroll
            for (int u = 0; u < 4; ++u) {
              const int n = 4 * g + u;
              const float r = av[u] < 0.f ? 0.f : av[u];  // ReLU (NaN kept, as relu_keep_nan)
              acc[i][u] = n < N ? r : 0.f;
              if (last && n < N) dpart = fmaf(r, p.fc[n], dpart);
            }
          }
        if (nn >= 0) {
          const int g2 = wave + kSpW * ni;
          a01 = f32x2{bh[4 * g2], bh[4 * g2 + 1]};
          a23 = f32x2{bh[4 * g2 + 2], bh[4 * g2 + 3]};
        }
      }
      ci = ni;
      cj = nj;
      cur_n = nn;
    }
    if (!last) {
      __syncthreads();  // every wave has finished reading this layer's input
#pragma unroll
      for (int i = 0; i < NGW; ++i) {
        const int g = wave + kSpW * i;
#pragma unroll
        for (int u = 0; u < 4; ++u)
          if (g < G && 4 * g + u < N) x[(4 * g + u) * kSpS + lane] = acc[i][u];
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

hipError_t launch_ell_build(const EllArgs& a, int rows, hipStream_t s) {  // rows = H * ceil(N/4) groups
  if (rows <= 0) return hipSuccess;
  hipLaunchKernelGGL(ell_build_kernel, dim3(rows), dim3(64), 0, s, a);
  return hipGetLastError();
}

// ELL entries per staging unit: kSpCap, or what the LDS left by the x tile holds (multiple of 8; 0: no room)
static int sparse_mlp_cap(int K0p, int N) {
  const int XK = K0p > N ? K0p : N;
  const int64_t base = (int64_t)sizeof(float) * ((int64_t)XK * kSpS + kSpW * kSpS);
  const int64_t room = (160 * 1024 - base) / (int64_t)(sizeof(int4) * 2 * kSpW);
  const int64_t cap = room < kSpCap ? room / 8 * 8 : kSpCap;
  return cap > 0 ? (int)cap : 0;
}

size_t sparse_mlp_lds_bytes(int K0p, int N) {
  const int XK = K0p > N ? K0p : N;
  const int cap = sparse_mlp_cap(K0p, N);
  if (cap == 0) return (size_t)-1;  // does not fit
  return sizeof(float) * ((size_t)XK * kSpS + kSpW * kSpS) + sizeof(int4) * 2 * (size_t)cap * kSpW;
}

template <int NGW>
static hipError_t launch_sp_t(SpMlpArgs a, hipStream_t s) {
  a.ecap = sparse_mlp_cap(a.K0p, a.N);
  if (a.ecap == 0) return hipErrorInvalidValue;
  const size_t lds = sparse_mlp_lds_bytes(a.K0p, a.N);
  auto k = sparse_mlp_kernel<NGW>;
  hipError_t e = ensure_lds_limit(reinterpret_cast<const void*>(k), lds);
  if (e != hipSuccess) return e;
  const unsigned grid = (unsigned)((a.batch + kSpS - 1) / kSpS);
  hipLaunchKernelGGL(k, dim3(grid), dim3(64 * kSpW), lds, s, a);
  return hipGetLastError();
}

hipError_t launch_sparse_mlp(const SpMlpArgs& a, hipStream_t s) {
  const int ngw = ((a.N + 3) / 4 + kSpW - 1) / kSpW;
  if (ngw <= 4) return launch_sp_t<4>(a, s);
  if (ngw <= 8) return launch_sp_t<8>(a, s);
  if (ngw <= 12) return launch_sp_t<12>(a, s);
  if (ngw <= 16) return launch_sp_t<16>(a, s);
  return hipErrorInvalidValue;
}

}  // namespace dfwfm
