// dfwfm_fwfm.hip -- the MLP-free forward (use_deep = 0: BASELINE configs[0]'s model, reference
// model/DeepFMs.py:300-367 + the combine :458) with one lane per (sample, pair of embedding columns).
//
// fwd_kernel's MLP-free form computes the FwFM from a per-sample Gram on f32 MFMA: 16 x 16 tiles over 39 fields and
// K = 10 padded to 12 do 2.5x the useful products, and the E tile, the Gram fragments and the barriers around them
// bound a CU to three to five 16-sample workgroups.  Here a wave owns 12 samples, five lanes per sample, lane j holding
// columns (2j, 2j+1) of every field's embedding row in registers (78 VGPRs at Criteo-39):
//   second[b] = sum_d sum_{k<l} U[k][l] e[k][d] e[l][d],  U = strictly upper (R + R^T) / 2 (FM: ones),
// as t_k = sum_{l>k} U[k][l] x_l, acc += x_k . t_k per lane -- exactly the 741 x 10 useful FMAs, U wave-uniform:
// staged through 6 KB of LDS into 25 registers spread over the wave and taken entry by entry with v_readlane (scalar
// loads of it missed the scalar cache on every first touch of a CU; LDS reads in the loop waited every few FMAs).  Every wave runs alone, so a CU holds as many
// waves as registers allow and one wave's dependent gather (index -> row) overlaps the others' FMAs.  Each field's row is one 8-byte load
// per lane (five lanes read the 40-byte row), the index / Xv of a field is loaded once per sample and passed to the
// sample's other lanes by a cross-lane read, and the table first order of field f is read by lane f % 5.
// The five lanes' partial sums are added by cross-lane reads; out[b] = (first + second) + bias as the reference.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>

#include "dfwfm_device.h"
#include "dfwfm_internal.h"

namespace dfwfm {

namespace {

template <int F, int NUM, int D>
struct LaneShape {
  static constexpr int LPS = D / 2;          // lanes per sample
  static constexpr int SPW = 64 / LPS;       // samples per wave
  static constexpr int NCAT = F - NUM;
  static constexpr int PI = (NCAT + LPS - 1) / LPS;  // categorical indices loaded per lane
  static constexpr int PV = (NUM + LPS - 1) / LPS;   // Xv values loaded per lane
};

}  // namespace

// WPE4: capped at 128 registers (four waves per SIMD, a few spilled) instead of ~166 (three); A/B DFWFM_LANE_WPE=4
template <int F, int NUM, int D, bool WPE4>
__global__ void __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(WPE4 ? 4 : 1))) fwfm_lane_kernel(FwdArgs p) {
  using S = LaneShape<F, NUM, D>;
  constexpr int LPS = S::LPS, SPW = S::SPW;
  static_assert(D % 2 == 0 && SPW * LPS <= 64, "lane layout");
  typedef float f2 __attribute__((ext_vector_type(2)));
  const int lane = threadIdx.x;
  const int s = lane / LPS;          // sample of this lane (SPW: an idle lane)
  const int j = lane - s * LPS;      // its column pair
  const int base = s * LPS;          // the sample's first lane
  const TileRef tr = tile_ref<SPW>(p);
  const int64_t b = tr.b0 + s;
  const bool live = s < SPW && b < p.batch;
  const int flags = p.flags;
  typedef const __attribute__((address_space(4))) float* cf_t;
  // the field descriptors in ONE round trip: lane f < F loads field f's table bases and row count, the loops below
  // take them with v_readlane (scalar loads of them, one field at a time, put a cold scalar-cache miss in front of
  // every row load: 23 us for a lone batch)
  uint32_t d_e2lo = 0, d_e2hi = 0, d_e1lo = 0, d_e1hi = 0, d_nlo = 0, d_nhi = 0;
  const float d_lw = ((flags & kFoLw) && lane < F) ? p.lw[lane] : 0.f;  // lw[f] the same way
  if (lane < F) {
    const FieldDev fdl = p.fields[lane];
    const uint64_t e2 = reinterpret_cast<uint64_t>(fdl.emb2), e1 = reinterpret_cast<uint64_t>(fdl.emb1);
    d_e2lo = (uint32_t)e2; d_e2hi = (uint32_t)(e2 >> 32);
    d_e1lo = (uint32_t)e1; d_e1hi = (uint32_t)(e1 >> 32);
    d_nlo = (uint32_t)fdl.n; d_nhi = (uint32_t)((uint64_t)fdl.n >> 32);
  }
  auto ptr_of = [](uint32_t lo, uint32_t hi, int f) {
    return reinterpret_cast<const float*>(((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)hi, f) << 32) |
                                          (uint32_t)__builtin_amdgcn_readlane((int)lo, f));
  };

  constexpr int FP = (F + 3) & ~3;
  __shared__ float4 us[F * FP / 4];
  if (flags & kHasSecond) {  // U [F][FP] -> LDS, behind which the index loads go out
    const float4* ug = reinterpret_cast<const float4*>(p.utri);
    for (int i = lane; i < F * FP / 4; i += 64) us[i] = ug[i];
  }

  // ---- indices and Xv: lane j loads the entries of columns j, j + LPS, ... of its sample -----------------------
  int64_t kv[S::PI];
  float xvv[S::PV];
#pragma unroll
  for (int q = 0; q < S::PI; ++q) {
    const int c = j + q * LPS;
    kv[q] = (live && c < S::NCAT) ? tr.xi[b * p.xi_stride + c] : 0;
  }
  int32_t idx[S::PI];
#pragma unroll
  for (int q = 0; q < S::PI; ++q) {
    const int c = j + q * LPS;
    // field NUM + c's row count from the lane that loaded its descriptor (c differs by lane: a cross-lane read)
    const int src = NUM + (c < S::NCAT ? c : 0);
    const int64_t n = (int64_t)(((uint64_t)(uint32_t)__shfl((int)d_nhi, src) << 32) | (uint32_t)__shfl((int)d_nlo, src));
    int64_t v = kv[q];
    if (live && c < S::NCAT && (v < 0 || v >= n)) {
      atomicOr(p.err, DFWFM_FLAG_INDEX_OUT_OF_RANGE);
      v = 0;
    }
    idx[q] = (int32_t)v;
  }
#pragma unroll
  for (int q = 0; q < S::PV; ++q) {
    const int c = j + q * LPS;
    xvv[q] = (live && c < NUM) ? tr.xv[b * p.xv_stride + c] : 0.f;
  }

  // ---- the rows: field f's columns (2j, 2j + 1); the table first order of field f by lane f % LPS -------------
  const bool need_e = (flags & kNeedE) != 0;
  const bool fo_tab = (flags & kFoTables) != 0;
  const bool lw = (flags & kFoLw) != 0;
  f2 x[F];
  // the first order's terms (numerical weights times Xv up to 63) cancel to a logit of ~1e2 in the FwFM-only models:
  // the lane's sum carries its rounding errors along (two-sum), which keeps the logits inside the north-star bar of
  // the reference's own fp32 result (golden fwfm_nolw: 1.15e-5 plain, 7.6e-6 compensated, the reference 6.3e-6)
  float first = 0.f, fcomp = 0.f;
  auto add_first = [&](float v) {
    const float s = first + v;
    const float bb = s - first;
    fcomp += (first - (s - bb)) + (v - bb);
    first = s;
  };
#pragma unroll
  for (int f = 0; f < F; ++f) {
    const float* e2 = ptr_of(d_e2lo, d_e2hi, f);
    const float* e1 = ptr_of(d_e1lo, d_e1hi, f);
    x[f] = f2{0.f, 0.f};
    float fo = 0.f;
    if (f < NUM) {
      const float xv = __shfl(xvv[f / LPS], base + f % LPS);
      if (live && need_e) {
        const f2 w = *reinterpret_cast<const f2*>(e2 + 2 * j);
        x[f] = f2{w.x * xv, w.y * xv};
      }
      if (live && fo_tab && j == f % LPS) fo = e1[0] * xv;
    } else {
      const int64_t r = __shfl(idx[(f - NUM) / LPS], base + (f - NUM) % LPS);
      if (live && need_e) x[f] = *reinterpret_cast<const f2*>(e2 + r * D + 2 * j);
      if (live && fo_tab && j == f % LPS) fo = e1[r];
    }
    if (fo_tab && j == f % LPS) add_first(lw ? fo * __shfl(d_lw, f) : fo);
  }

  // ---- fwlw first order: sum_d fwlw[f][d] e[f][d] over this lane's d (lw-projected when use_lw) -------------------
  if (flags & kFoFwlw) {
#pragma unroll
    for (int f = 0; f < F; ++f) {
      const f2 w = *reinterpret_cast<const f2*>(p.fwlw + f * D + 2 * j);
      const float v = fmaf(x[f].y, w.y, x[f].x * w.x);
      add_first(lw ? v * __shfl(d_lw, f) : v);
    }
  }
  first += fcomp;

  __syncthreads();  // the wave's U stores are visible (the workgroup is this one wave)
  // ---- second order: sum_k x_k . (sum_{l>k} U[k][l] x_l), U in the wave's registers (UReg: readlane -> SGPR) -------
  float second = 0.f;
  if (flags & kHasSecond) {
    UReg<F> U;
    U.load(reinterpret_cast<const float*>(us), lane);
    float ax = 0.f, ay = 0.f;
#pragma unroll
    for (int k = 0; k < F - 1; ++k) {
      float tx = 0.f, ty = 0.f;
#pragma unroll
      for (int l = k + 1; l < F; ++l) {
        const float u = U.at(k, l);
        tx = fmaf(u, x[l].x, tx);
        ty = fmaf(u, x[l].y, ty);
      }
      ax = fmaf(x[k].x, tx, ax);
      ay = fmaf(x[k].y, ty, ay);
    }
    second = ax + ay;
  }

  // ---- the sample's LPS lanes -> lane base ---------------------------------------------------------------------
  float fsum = first, ssum = second;
#pragma unroll
  for (int o = 1; o < LPS; ++o) {
    fsum += __shfl(first, base + o);
    ssum += __shfl(second, base + o);
  }
  if (live && j == 0) tr.out[b] = (fsum + ssum) + ((cf_t)p.bias)[0];
}

// the shapes with a lane kernel: Criteo-39 (39 fields, 13 numerical, emb 10)
bool fwfm_lane_supported(int F, int num, int D) { return F == 39 && num == 13 && D == 10; }

int fwfm_lane_rows(int D) { return 64 / (D / 2); }

hipError_t launch_fwfm_lane(const FwdArgs& a, hipStream_t s) {
  if (!fwfm_lane_supported(a.F, a.num, 10)) return hipErrorInvalidValue;
  const char* w = getenv("DFWFM_LANE_WPE");
  auto k = (w && atoi(w) == 4) ? fwfm_lane_kernel<39, 13, 10, true> : fwfm_lane_kernel<39, 13, 10, false>;
  hipLaunchKernelGGL(k, dim3(fwd_grid(a, fwfm_lane_rows(10))), dim3(64), 0, s, a);
  return hipGetLastError();
}

}  // namespace dfwfm
