// dfwfm_shallow.hip -- the forward of a model without the deep tower (use_deep = 0: FwFM / FM / LR,
// reference model/DeepFMs.py:285-367 and the combine :455-469), the FwFM-only config of BASELINE
// configs[0].
//
// Without an MLP there is nothing to hide the gather's latency behind, so this kernel is built for a
// short critical path per 16-sample tile (one workgroup of eight waves per tile, 256 tiles per
// 4096-row batch -- one per CU, and further batches in flight share the CUs):
//
//   stage   field descriptors -> LDS; every lane's keys (Xi indices / Xv values) and the shallow
//           parameters (FwFM fragments, fwlw, lw, bias) in flight together;
//   gather  row slots (sample b, field f), f fastest, each row read by D/PW lanes with one PW-float
//           load each (PW = 4 when rows are 16-byte multiples, else 2): a wave load instruction covers
//           64/(D/PW) whole rows (12 rows of 40 B for D = 10) instead of one 8-byte piece of 64 rows,
//           so the vector L1 looks up each row's lines once per instruction rather than D/2 times.
//           Every round's loads are issued before any is consumed; QR rows read both operands;
//   shallow first order (tables, fwlw or numerical v*x) projected by lw or summed; FwFM / FM second
//           order on f32 MFMA as  second[b] = sum_{k,d} E[b,k,d] * (U E_b)[k,d],  U = strictly upper
//           (R + R^T)/2, in the same (row tile, column tile) pieces and step order as fwd_kernel, with
//           the next piece's operands read from LDS while the current piece's MFMAs run;
//   combine first + second + bias, stored by the lane that finishes the sample's sums.
//
// The arithmetic (products, sums and their order) is that of fwd_kernel's shallow phases, so the
// logits are bit-identical to the fused kernel's (tests/test_gpu_parity.py::
// test_shallow_kernel_is_bit_identical_to_fused).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>

#include "dfwfm_device.h"
#include "dfwfm_internal.h"

namespace dfwfm {

namespace {

typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));

template <int D>
struct RowSplit {
  static constexpr int PW = (D % 4 == 0) ? 4 : 2;  // floats per lane (every supported D is even)
  static constexpr int LPR = D / PW;                // lanes per row
  static constexpr int RPW = 64 / LPR;              // rows per wave per round
};

template <int PW>
struct PartVec;
template <>
struct PartVec<2> {
  using T = f32x2;
};
template <>
struct PartVec<4> {
  using T = f32x4;
};

// a load through a pointer known to be global memory: table pointers come from the LDS descriptors, and
// as generic pointers they would compile to flat loads (which also count against lgkmcnt, so every wait
// for a row would wait for the LDS traffic too)
template <typename T>
__device__ __forceinline__ T gload(const void* ptr) {
  return *(const __attribute__((address_space(1))) T*)(ptr);
}

constexpr int kSMax = (kMaxMT * 16) / 4;  // FwFM contraction steps for F <= 64

}  // namespace

// QR: some field is a QR embedding (kHasQR); FOT: first order from the per-field tables (kFoTables);
// NE: second-order embeddings are gathered (kNeedE; only a logistic-regression model has none)
template <int D, int NW, bool QR, bool FOT, bool NE>
__global__ void __launch_bounds__(64 * NW) __attribute__((amdgpu_waves_per_eu(4)))
shallow_kernel(FwdArgs p) {
  constexpr int kRoundChunk = NW == 4 ? 14 : 8;  // gather rounds in flight per lane (F = 39: one chunk)
  using RS = RowSplit<D>;
  constexpr int PW = RS::PW, LPR = RS::LPR, RPW = RS::RPW;
  using PV = typename PartVec<PW>::T;
  constexpr int NTH = 64 * NW;
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int F = p.F;
  const int num = p.num;
  const int SX = p.SX;
  const int flags = p.flags;
  const int Fp = r4(F);
  const LdsLayout L = lds_layout(F, D, p.MT, p.S, SX, 0, 1, 1, false, false);
  FieldDev* desc = reinterpret_cast<FieldDev*>(smem + L.desc);
  float* lw_s = smem + L.lw;
  float* fwlw_s = smem + L.fwlw;
  float* upk = smem + L.upk;
  float* bufX = smem + L.bufX;
  float* fo = smem + L.fo;
  float* part2 = smem + L.part2;

  const int64_t b0 = (int64_t)blockIdx.x * kBM;
  stamp(p.stamps, 0, tid);
  stamp_start_rt(p.stamps, tid);
  const int nrows = (int)((p.batch - b0) < kBM ? (p.batch - b0) : kBM);

  // this lane's row slots: round k covers slots [k*NW*RPW, (k+1)*NW*RPW), wave w rows w*RPW.., part pp
  const int rl = lane / LPR;       // row of the wave (rl < RPW: active)
  const int pp = lane - rl * LPR;  // part of the row
  const bool act = rl < RPW;
  const int nslots = kBM * F;
  const int nrounds = (nslots + NW * RPW - 1) / (NW * RPW);
  const int ncat = F - num;

  // ---- stage: descriptors and shallow parameters -> LDS (L2-resident, shared by every workgroup),
  // issued first; then the first chunk's keys, which stay in flight across those stores -------------
  {
    constexpr int kDescPT = (7 * 64 + NTH - 1) / NTH;
    constexpr int kUpkPT = (kMaxMT * 16 * 16 + NTH - 1) / NTH;
    constexpr int kFwlwPT = (64 * 32 + NTH - 1) / NTH;
    u32x2 dw[kDescPT];
#pragma unroll
    for (int k = 0; k < kDescPT; ++k) {
      const int i = tid + k * NTH;
      if (i < 7 * F) dw[k] = reinterpret_cast<const u32x2*>(p.fields)[i];
    }
    f32x4 uw[kUpkPT];
    const int n_upk = (flags & kHasSecond) ? p.MT * p.S * 16 : 0;
#pragma unroll
    for (int k = 0; k < kUpkPT; ++k) {
      const int i = tid + k * NTH;
      if (i < n_upk) uw[k] = reinterpret_cast<const f32x4*>(p.upack)[i];
    }
    float fw[kFwlwPT];
    const int n_fwlw = (flags & kFoFwlw) ? F * D : 0;
#pragma unroll
    for (int k = 0; k < kFwlwPT; ++k) {
      const int i = tid + k * NTH;
      if (i < n_fwlw) fw[k] = p.fwlw[i];
    }
    const float lwv = ((flags & kFoLw) && tid < F) ? p.lw[tid] : 0.f;
#pragma unroll
    for (int k = 0; k < kDescPT; ++k) {
      const int i = tid + k * NTH;
      if (i < 7 * F) reinterpret_cast<u32x2*>(desc)[i] = dw[k];
    }
#pragma unroll
    for (int k = 0; k < kUpkPT; ++k) {
      const int i = tid + k * NTH;
      if (i < n_upk) reinterpret_cast<f32x4*>(upk)[i] = uw[k];
    }
#pragma unroll
    for (int k = 0; k < kFwlwPT; ++k) {
      const int i = tid + k * NTH;
      if (i < n_fwlw) fwlw_s[i] = fw[k];
    }
    if ((flags & kFoLw) && tid < F) lw_s[tid] = lwv;
    // zero the E-tile columns past F*D that the FwFM contraction reads (4*S fields)
    const int w = p.W0 - F * D;
    for (int i = tid; i < kBM * w; i += NTH) {
      const int b = i / w;
      bufX[b * SX + F * D + (i - b * w)] = 0.f;
    }
  }

  // ---- gather, kRoundChunk rounds in flight at a time (one chunk while 16 * F <= 8 * NW * RPW) -----
  // Branch-free per round: lanes without a live slot read a valid element of the tile's first row /
  // field 0's row 0 and are masked at the store, so every round's loads stay in flight together.
  for (int c0 = 0; c0 < nrounds; c0 += kRoundChunk) {
    int64_t kx[kRoundChunk];
    float kv[kRoundChunk];
#pragma unroll
    for (int k = 0; k < kRoundChunk; ++k) {
      kx[k] = 0;
      kv[k] = 0.f;
    }
    if (ncat > 0) {
#pragma unroll
      for (int k = 0; k < kRoundChunk; ++k) {
        const int slot = (c0 + k) * NW * RPW + wave * RPW + rl;
        const int b = slot / F;
        const int f = slot - b * F;
        const bool cat = act & (slot < nslots) & (b < nrows) & (f >= num);  // slot < nslots: round < nrounds
        kx[k] = p.xi[(b0 + (cat ? b : 0)) * p.xi_stride + (cat ? f - num : 0)];
      }
    }
    if (num > 0) {
#pragma unroll
      for (int k = 0; k < kRoundChunk; ++k) {
        const int slot = (c0 + k) * NW * RPW + wave * RPW + rl;
        const int b = slot / F;
        const int f = slot - b * F;
        const bool nm = act & (slot < nslots) & (b < nrows) & (f < num);
        kv[k] = p.xv[(b0 + (nm ? b : 0)) * p.xv_stride + (nm ? f : 0)];
      }
    }
    if (c0 == 0) {
      __syncthreads();  // descriptors and parameters in LDS
      stamp(p.stamps, 1, tid);
    }
    // row addresses and loads, every round's issued before any is consumed (32-bit row arithmetic: the
    // host keeps tables below 2^31 rows on this path)
    PV va[kRoundChunk], vb[kRoundChunk];
    float fa[kRoundChunk], fb[kRoundChunk];
    bool bad = false;
#pragma unroll
    for (int k = 0; k < kRoundChunk; ++k) {
      const int slot = (c0 + k) * NW * RPW + wave * RPW + rl;
      const int b = slot / F;
      const int f = slot - b * F;
      const bool live = act & (slot < nslots) & (b < nrows);
      const bool cat = live & (f >= num);
      const FieldDev* fd = desc + (live ? f : 0);
      const int64_t n = fd->n;
      const int64_t idx = cat ? kx[k] : 0;
      const bool oob = cat & ((idx < 0) | (idx >= n));
      bad |= oob;
      const int ix = oob ? 0 : (int)idx;
      int q = ix, rr = 0;
      bool qr = false;
      if constexpr (QR) {
        const int c = (int)fd->c;
        qr = cat & (c > 0);
        const unsigned cu = qr ? (unsigned)c : 1u;
        q = (int)((unsigned)ix / cu);
        rr = ix - q * (int)cu;
      }
      if constexpr (NE) {
        const float* pa = fd->emb2 + (int64_t)q * D + pp * PW;
        va[k] = gload<PV>(pa);
        if constexpr (QR) vb[k] = gload<PV>(qr ? fd->emb2_r + (int64_t)rr * D + pp * PW : pa);
      }
      if constexpr (FOT) {
        const float* qa = fd->emb1 + q;
        fa[k] = gload<float>(qa);
        if constexpr (QR) fb[k] = gload<float>(qr ? fd->emb1_r + rr : qa);
      }
    }
    if (__builtin_amdgcn_ballot_w64(bad) != 0 && lane == 0) atomicOr(p.err, DFWFM_FLAG_INDEX_OUT_OF_RANGE);
#pragma unroll
    for (int k = 0; k < kRoundChunk; ++k) {
      const int slot = (c0 + k) * NW * RPW + wave * RPW + rl;
      if (act && slot < nslots) {
        const int b = slot / F;
        const int f = slot - b * F;
        const bool live = b < nrows;
        // row combine: numerical v * x, plain row, QR q * r (mult) or q + r (add)
        int mode = 0;
        float scale = 1.f;
        if (f < num) {
          scale = kv[k];
        } else if constexpr (QR) {
          const FieldDev* fd = desc + f;
          mode = fd->c > 0 ? (fd->op == 0 ? 1 : 2) : 0;
        }
        if constexpr (NE) {
          PV e;
#pragma unroll
          for (int j = 0; j < PW; ++j)
            e[j] = live ? combine(mode, va[k][j], QR ? vb[k][j] : 0.f, scale) : 0.f;
          *reinterpret_cast<PV*>(bufX + b * SX + f * D + pp * PW) = e;
        }
        if (pp == 0) {
          float x = 0.f;
          if constexpr (FOT) x = live ? combine(mode, fa[k], QR ? fb[k] : 0.f, scale) : 0.f;
          fo[b * Fp + f] = x;
        }
      }
    }
  }
  __syncthreads();
  stamp(p.stamps, 2, tid);

  // ---- shallow part -------------------------------------------------------------------------------
  if (flags & kFoFwlw) {
    // fm_first_order[b, f] = sum_d E[b, f, d] * Wfl[f, d]  (einsum 'ijk,ik->ijk' then 'ijk->ji')
    for (int r = tid; r < kBM * F; r += NTH) {
      const int f = r >> 4;
      const int b = r & 15;
      const float* e = bufX + b * SX + f * D;
      const float* w = fwlw_s + f * D;
      float s = 0.f;
#pragma unroll
      for (int d = 0; d < D; ++d) s += e[d] * w[d];
      fo[b * Fp + f] = s;
    }
  }
  stamp(p.stamps, 9, tid);
  if (flags & kHasSecond) {
    // pieces pc = (row tile m, column tile nt) in the host's balanced assignment (fw_list8 / fw_list4);
    // a piece accumulates U[16m.., 4s..] * E over its steps s = 4m .. S-1 in ascending order
    // (fwd_kernel's order); all of a piece's operands are read before its MFMAs, and the co-resident
    // wave of the SIMD fills the MFMA dependency gaps
    const int S = p.S;
    const uint8_t* plist = NW == 8 ? p.fw_list8 : p.fw_list4;
    const int p_lo = NW == 8 ? p.fw_off8[wave] : p.fw_off4[wave];
    const int p_hi = NW == 8 ? p.fw_off8[wave + 1] : p.fw_off4[wave + 1];
    for (int pi = p_lo; pi < p_hi; ++pi) {
      const int pc = plist[pi];
      const int m = pc / D;
      const int n = (pc - m * D) * 16 + (lane & 15);
      const int b = n / D;
      const float* ecol = bufX + b * SX + (n - b * D);  // E[b][l][d] = ecol[l * D]
      const float* ua = upk + m * S * 64 + lane;        // A fragment of step s: ua[s * 64]
      float av[kSMax], bv[kSMax];
#pragma unroll
      for (int s = 0; s < kSMax; ++s) {
        if (s >= 4 * m && s < S) {
          av[s] = ua[s * 64];
          bv[s] = ecol[(4 * s + (lane >> 4)) * D];
        }
      }
      f32x4 acc = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int s = 0; s < kSMax; ++s)
        if (s >= 4 * m && s < S) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(av[s], bv[s], acc, 0, 0, 0);
      if (pi == p_lo) stamp(p.stamps, 3, tid);  // diagnostics: first piece's MFMAs issued
      float v = 0.f;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int k = 16 * m + 4 * (lane >> 4) + r;
        const float e = ecol[(k < F ? k : 0) * D];
        v = fmaf(k < F ? e : 0.f, acc[r], v);
      }
      v += __shfl_xor(v, 16);
      v += __shfl_xor(v, 32);
      if (lane < 16) part2[pc * 16 + lane] = v;
      if (pi - p_lo < 4) stamp(p.stamps, 4 + pi - p_lo, tid);  // diagnostics: piece ends (slots 4-7)
    }
  }
  stamp(p.stamps, 10, tid);
  __syncthreads();
  stamp(p.stamps, 11, tid);
  if (wave < 4) {
    // first[b] (lw projection or plain sum) and second[b]: 16 lanes per sample, then a butterfly
    const int b = wave * 4 + (lane >> 4);
    const int q = lane & 15;
    float first = 0.f, second = 0.f;
    for (int f = q; f < F; f += 16) {
      const float x = fo[b * Fp + f];
      first = (flags & kFoLw) ? fmaf(x, lw_s[f], first) : first + x;
    }
    if (flags & kHasSecond) {
      for (int d = q; d < D; d += 16) {
        const int n = b * D + d;
        for (int m = 0; m < p.MT; ++m) second += part2[(m * D + (n >> 4)) * 16 + (n & 15)];
      }
    }
#pragma unroll
    for (int o = 8; o >= 1; o >>= 1) {
      first += __shfl_xor(first, o);
      second += __shfl_xor(second, o);
    }
    if (q == 0 && b < nrows) {
      const float fs = first + second;
      p.out[b0 + b] = fs + p.bias[0];
    }
  }
  stamp(p.stamps, 8, tid);
  stamp_end_rt(p.stamps, tid);
}

static int shallow_waves() {
  static const int nw = [] {
    const char* v = getenv("DFWFM_SHALLOW_NW");
    return (v && atoi(v) == 4) ? 4 : 8;
  }();
  return nw;
}

template <int D, bool QR, bool FOT, bool NE = true>
static hipError_t launch_shallow_t(const FwdArgs& a, size_t lds, hipStream_t s) {
  const int nw = shallow_waves();
  auto k = nw == 4 ? shallow_kernel<D, 4, QR, FOT, NE> : shallow_kernel<D, 8, QR, FOT, NE>;
  hipError_t e = ensure_lds_limit(reinterpret_cast<const void*>(k), lds);
  if (e != hipSuccess) return e;
  const unsigned grid = (unsigned)((a.batch + kBM - 1) / kBM);
  hipLaunchKernelGGL(k, dim3(grid), dim3(64 * nw), lds, s, a);
  return hipGetLastError();
}

template <int D>
static hipError_t launch_shallow_d(const FwdArgs& a, size_t lds, hipStream_t s) {
  const bool qr = (a.flags & kHasQR) != 0, fot = (a.flags & kFoTables) != 0;
  if (!(a.flags & kNeedE))  // logistic regression: first order from the tables only
    return qr ? launch_shallow_t<D, true, true, false>(a, lds, s) : launch_shallow_t<D, false, true, false>(a, lds, s);
  if (qr) return fot ? launch_shallow_t<D, true, true>(a, lds, s) : launch_shallow_t<D, true, false>(a, lds, s);
  return fot ? launch_shallow_t<D, false, true>(a, lds, s) : launch_shallow_t<D, false, false>(a, lds, s);
}

hipError_t launch_shallow(const FwdArgs& a, int D, size_t lds, hipStream_t s) {
  switch (D) {
    case 4: return launch_shallow_d<4>(a, lds, s);
    case 8: return launch_shallow_d<8>(a, lds, s);
    case 10: return launch_shallow_d<10>(a, lds, s);
    case 16: return launch_shallow_d<16>(a, lds, s);
    case 32: return launch_shallow_d<32>(a, lds, s);
    default: return hipErrorInvalidValue;
  }
}

}  // namespace dfwfm
