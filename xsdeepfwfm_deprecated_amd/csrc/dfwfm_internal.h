// dfwfm_internal.h -- types shared by the kernels and the C-ABI layer.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/dfwfm.h"

namespace dfwfm {

constexpr int kBM = 16;   // samples per workgroup = one 16-row MFMA tile
constexpr int kWG = 256;  // 4 waves (one per SIMD)
constexpr int kMaxTPW = 8;  // output tiles per wave => deep_nodes <= 4*8*16 = 512

// flags
constexpr int kHasSecond = 1;  // FwFM / FM second order
constexpr int kHasDeep = 2;    // MLP
constexpr int kFoTables = 4;   // first order from fm_1st_embeddings
constexpr int kFoFwlw = 8;     // first order from fwfm_linear
constexpr int kFoLw = 16;      // project first order with fm_1st.weight

// Device copy of dfwfm_field_tables (same field order and sizes).
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

struct Pair {
  int16_t k, l;
  float r;
};

struct FwdArgs {
  const FieldDev* fields;
  const int64_t* xi;
  int64_t xi_stride;
  const float* xv;
  int64_t xv_stride;
  int64_t batch;
  float* out;
  int32_t* err;
  const Pair* pairs;
  const int32_t* npairs;
  const float* fwlw;
  const float* lw;
  const float* bias;
  const float4* wpack;
  const float* mlp_b;
  const float* fc;
  int32_t F, num, H, N;
  int32_t NT, NC0;
  int32_t SX, SY;
  int32_t flags;
};

bool supported_embedding_size(int D);
hipError_t launch_forward(const FwdArgs& a, int D, int tpw, size_t lds, hipStream_t s);
hipError_t launch_pack_linear(const float* w, int N, int K, int NT, int NC, float4* out, hipStream_t s);
hipError_t launch_pad_copy(const float* src, int n, int npad, float* dst, hipStream_t s);
hipError_t launch_build_pairs(const float* R, int F, int mode, Pair* pairs, int32_t* npairs, hipStream_t s);

}  // namespace dfwfm
