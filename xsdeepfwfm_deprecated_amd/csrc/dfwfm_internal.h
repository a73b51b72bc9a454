// dfwfm_internal.h -- types shared by the kernels and the C-ABI layer.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/dfwfm.h"

namespace dfwfm {

constexpr int kBM = 16;     // samples per workgroup = one 16-row MFMA tile
constexpr int kMaxTPW = 8;  // MLP output tiles per wave group => deep_nodes <= 4*8*16 = 512
constexpr int kMaxMT = 4;   // FwFM row tiles => field_size <= 64
constexpr int kStampSlots = 16;  // diagnostic phase stamps per workgroup

// flags
constexpr int kHasSecond = 1;  // FwFM / FM second order
constexpr int kHasDeep = 2;    // MLP
constexpr int kFoTables = 4;   // first order from fm_1st_embeddings
constexpr int kFoFwlw = 8;     // first order from fwfm_linear
constexpr int kFoLw = 16;      // project first order with fm_1st.weight
constexpr int kNeedE = 32;     // second-order / deep embeddings are gathered

// Device copy of dfwfm_field_tables (same field order and sizes); for QR fields
// n holds the accepted index bound ceil(n/c)*c.
struct FieldDev {
  const float* emb2;
  const float* emb2_r;
  const float* emb1;
  const float* emb1_r;
  int64_t n;
  int64_t c;
  int32_t op;
  int32_t reserved;
};
static_assert(sizeof(FieldDev) == sizeof(dfwfm_field_tables), "descriptor layout");
static_assert(sizeof(FieldDev) == 56, "descriptor is 7 x 8 bytes in LDS");

struct FwdArgs {
  const FieldDev* fields;
  const int64_t* xi;
  int64_t xi_stride;
  const float* xv;
  int64_t xv_stride;
  int64_t batch;
  float* out;
  int32_t* err;
  const float* upack;  // FwFM A-operand fragments [MT][S][64]: strictly-upper (R + R^T)/2
  const float* fwlw;   // [F*D]
  const float* lw;     // [F]
  const float* bias;   // [1]
  const float4* wpack; // MLP weights, per layer [NT][NC][64] float4
  int32_t wpack_bytes; // buffer-descriptor range of wpack
  const float* mlp_b;  // [H][NT*16]
  const float* fc;     // [NT*16]
  int32_t F, num, H, N;
  int32_t NT, NC0;     // MLP: output tiles, layer-0 K chunks
  int32_t MT, S;       // FwFM: row tiles ceil(F/16), K steps ceil(F/4)
  int32_t SX, SY;      // LDS row strides (floats) of the two activation tiles
  int32_t W0;          // E-tile columns that must be valid (zero padded past F*D)
  int32_t flags;
  uint64_t* stamps;    // diagnostics only: [grid][kStampSlots] shader-clock stamps, normally null
};

// LDS carve-up, in floats; every region starts 16-byte aligned.
struct LdsLayout {
  int desc, lw, fwlw, upk, bufX, bufY, red, fo, part2, dsum, fs, total;
};

__host__ __device__ inline int r4(int x) { return (x + 3) & ~3; }

__host__ __device__ inline LdsLayout lds_layout(int F, int D, int MT, int S, int SX, int SY, int TPW, int KS,
                                                bool deep) {
  LdsLayout L;
  int o = 0;
  L.desc = o;  o += r4(14 * F);
  L.lw = o;    o += r4(F);
  L.fwlw = o;  o += r4(F * D);
  L.upk = o;   o += MT * S * 64;
  L.bufX = o;  o += kBM * SX;
  L.bufY = o;  o += deep ? kBM * SY : 0;
  L.red = o;   o += (deep && KS == 2) ? 4 * TPW * 64 * 4 : 0;
  L.fo = o;    o += kBM * r4(F);
  L.part2 = o; o += r4(kBM * D);
  L.dsum = o;  o += 4 * kBM;
  L.fs = o;    o += kBM;
  L.total = r4(o);
  return L;
}

bool supported_embedding_size(int D);
hipError_t launch_forward(const FwdArgs& a, int D, int tpw, int ks, size_t lds, hipStream_t s);
hipError_t launch_pack_linear(const float* w, int N, int K, int NT, int NC, float4* out, hipStream_t s);
hipError_t launch_pad_copy(const float* src, int n, int npad, float* dst, hipStream_t s);
hipError_t launch_pack_fwfm(const float* R, int F, int mode, int MT, int S, float* out, hipStream_t s);

}  // namespace dfwfm
