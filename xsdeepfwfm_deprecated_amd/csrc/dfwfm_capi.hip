// dfwfm_capi.hip -- the extern "C" boundary (include/dfwfm.h) over the kernels.
#include <hip/hip_runtime.h>
#include <mutex>
#include <stdint.h>
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <cmath>
#include <string>
#include <vector>

#include "dfwfm_internal.h"

using namespace dfwfm;

struct dfwfm_model {
  dfwfm_config cfg;
  int device;
  int F, D, num, H, N;
  int NT, NC0, SX, SY, TPW, MT, S, W0, KS;
  int TPWF, tail;  // forward: full tiles per wave, split-tail mode (NT == 4*TPWF + 1); TPW = ceil(NT/4)
  int flags;
  size_t lds_bytes;
  size_t lds_gather;   // split forward: LDS of the gather launch (no MLP buffers)
  int NG, TPWI, tailI; // inference forward: tile groups (waves, 4 or 8), tiles per wave, split tail
  int r32;             // 32-sample workgroups (fwd32_kernel) usable: 0 no, 1 when the stream's CUs are covered, 2 forced
  size_t lds_r32;
  size_t lds_ftrain;   // the training forward with helper waves (ftrain_kernel), 0: not this model's form
  void* cu_stream[8];  // streams whose CU counts are cached (hipExtStreamGetCUMask), round-robin replaced
  int cu_count[8], cu_n, cu_next;
  int dev_cus;         // CUs of the device (0 until the first stream_cu_count)
  size_t lds_inf;      // inference forward LDS (lds_bytes: the training forward's, NG = 4)
  // sparse deep tower (dfwfm_model_build_sparse_mlp): ELL of the pruned weights, used by dfwfm_forward_ws
  int sp;                          // enabled (cleared by set_dense: the ELL is then stale)
  const float* lin_w[kMaxH];       // the caller's weights from the last set_dense
  int2* d_ell;
  int32_t* d_cnt;                  // [H][N] + [H][ceil(N/4)] (row, group counts)
  int32_t* d_spstat;               // [2]
  int spW[kMaxH];
  int64_t spoff[kMaxH];
  double sp_density;               // nonzero fraction of the last build
  uint8_t fw_list4[kMaxPieces], fw_off4[5];  // FwFM pieces per wave, 4- and 8-wave launches (fw_schedule)
  uint8_t fw_list8[kMaxPieces], fw_off8[9];
  // device state (owned)
  FieldDev* d_fields;
  float* d_upack;  // FwFM A-operand fragments [MT][S][64]
  int2* d_pairs;   // build_fwfm_pairs: nonzero pairs of a pruned R (F (F - 1) / 2 capacity)
  float* d_pkrows;       // dfwfm_model_pack_tables: the serving rows of every categorical field
  size_t pkrows_floats;  // capacity
  const float** d_pk;    // [64] per-field row bases (device)
  int pkw;               // row stride in floats while the copy is in use, else 0
  int32_t npairs;
  int32_t* d_err;
  float4* d_wpack;
  size_t wpack_elems;
  float* d_mlp_b;  // [H][NT*16]
  float* d_fc;     // [NT*16]
  float* d_fwlw;   // [F*D]
  float* d_lw;     // [F]
  float* d_bias;   // [1]
  uint64_t* d_stamps;  // diagnostics (DFWFM_DIAG stamps=)
  size_t stamps_cap;   // workgroups the stamp buffer holds
  size_t stamps_ring;  // launches kept (DFWFM_DIAG ring=), each its own slice of the buffer
  size_t stamps_next;  // next slice
  // training
  float4* d_wtpack;    // transposed MLP packs for dX_{l-1} = G_l W_l
  size_t wtpack_elems;
  int wt_off[kMaxH + 1];
  float* d_rsk;        // symmetric off-diagonal (R+R^T)/2 fragments
  float* d_ws;         // activation workspace (E, fo, X_0..X_H, G_1..G_H)
  int64_t ws_batch;
  int64_t ws_gen;      // bumped on every (re)allocation of d_ws (graphs that baked its pointers are stale)
  float* sv_e;
  float* sv_fo;
  float* sv_x[kMaxH + 1];
  float* sv_g[kMaxH + 1];
  float* sv_de;
  int32_t* sv_keys;     // the training forward's clamped categorical indices, column-major (sorted scatter keys)
  int64_t keys_stride;
  bool t_keys;          // the last training forward wrote sv_keys
  float* sv_x0;           // X_0 after deep-tower dropout (without dropout X_0 is sv_e)
  float* red_part;        // per-16-row-tile partial sums of the shallow reductions
  float* dw_part;         // weight-gradient GEMM: per (block, split) slices (deterministic split-K, dwr_block)
  float* dw_bpart;
  int64_t dw_slices;      // blocks x splits the slices hold
  FieldDev h_fields[64];  // host copy of the field descriptors (scatter task planning)
  // the last dfwfm_train_forward, replayed by dfwfm_backward
  const int64_t* t_xi;
  int64_t t_xs;
  const float* t_xv;
  int64_t t_vs;
  int64_t t_batch;
  float t_drop;
  uint32_t t_seed;
  const int64_t* step_src;  // dfwfm_set_step_source
  bool trained;
  bool bwd_tables;  // the per-tile backward (sv_de) ran for the last dfwfm_train_forward
  bool bwd_fused_red;  // ... with the dense shallow reductions fused in (per-tile partials written)
  float* bwd_loss_sum; // ... and the loss gradient fused in too: the tiles' losses are partials, summed into this
  bool deterministic;  // dfwfm_set_deterministic: fixed-order table scatter and split-K sums
  bool tables_set;
  bool dense_set;
};

namespace {

thread_local std::string g_last_error;

int fail(int code, const char* fmt, ...) __attribute__((format(printf, 2, 3)));
int fail(int code, const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof buf, fmt, ap);
  va_end(ap);
  g_last_error = buf;
  return code;
}

int hip_fail(hipError_t e, const char* what) {
  return fail(DFWFM_ERR_HIP, "%s: %s", what, hipGetErrorString(e));
}

#define HIP_TRY(expr)                                  \
  do {                                                 \
    hipError_t e_ = (expr);                            \
    if (e_ != hipSuccess) return hip_fail(e_, #expr);  \
  } while (0)

template <typename T>
int dev_alloc(T** p, size_t count) {
  *p = nullptr;
  if (count == 0) count = 1;
  HIP_TRY(hipMalloc(reinterpret_cast<void**>(p), count * sizeof(T)));
  return DFWFM_OK;
}

void free_model(dfwfm_model* m) {
  if (!m) return;
  void* ptrs[] = {m->d_fields, m->d_upack, m->d_err,     m->d_wpack, m->d_mlp_b,   m->d_fc,  m->d_fwlw,
                  m->d_lw,     m->d_bias,  m->d_stamps,  m->d_wtpack, m->d_rsk,   m->d_ws,
                  m->d_ell,    m->d_cnt,   m->d_spstat, m->d_pairs, m->d_pkrows, m->d_pk};
  for (void* p : ptrs)
    if (p) (void)hipFree(p);
  delete m;
}

}  // namespace

// FwFM second-order pieces (row tile m, column tile nt; S - 4m MFMA steps each) balanced over `nw` waves:
// largest first, each to the least-loaded wave; a wave's list is in ascending piece order.  The pieces'
// results do not depend on the assignment, so 4- and 8-wave launches give identical logits.
static void fw_schedule(int MT, int D, int S, int nw, uint8_t* list, uint8_t* off) {
  int load[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  int owner[kMaxPieces];
  for (int m = 0; m < MT; ++m)  // sizes fall with m: row tile order is largest first
    for (int nt = 0; nt < D; ++nt) {
      int w = 0;
      for (int k = 1; k < nw; ++k)
        if (load[k] < load[w]) w = k;
      owner[m * D + nt] = w;
      load[w] += S - 4 * m;
    }
  int o = 0;
  for (int w = 0; w < nw; ++w) {
    off[w] = (uint8_t)o;
    for (int pc = 0; pc < MT * D; ++pc)
      if (owner[pc] == w) list[o++] = (uint8_t)pc;
  }
  off[nw] = (uint8_t)o;
}

extern "C" {

const char* dfwfm_last_error(void) { return g_last_error.c_str(); }
int dfwfm_abi_version(void) { return DFWFM_ABI_VERSION; }

int dfwfm_model_create(const dfwfm_config* cfg, dfwfm_model** out) {
  if (!cfg || !out) return fail(DFWFM_ERR_INVALID_ARG, "null argument");
  *out = nullptr;
  const dfwfm_config& c = *cfg;
  if (c.field_size <= 0 || c.field_size > 64)
    return fail(DFWFM_ERR_UNSUPPORTED, "field_size %d outside [1, 64]", c.field_size);
  if (c.numerical < 0 || c.numerical > c.field_size)
    return fail(DFWFM_ERR_INVALID_ARG, "numerical %d outside [0, field_size]", c.numerical);
  if (!supported_embedding_size(c.embedding_size))
    return fail(DFWFM_ERR_UNSUPPORTED, "embedding_size %d not in {4, 8, 10, 16, 32}", c.embedding_size);
  if ((c.use_fwfm != 0) + (c.use_fm != 0) + (c.use_logit != 0) > 1)
    return fail(DFWFM_ERR_INVALID_ARG, "only one of use_fwfm / use_fm / use_logit may be set");
  if (!c.use_fwfm && !c.use_fm && !c.use_logit)
    return fail(DFWFM_ERR_UNSUPPORTED,
                "a shallow part (fwfm, fm or logit) is required: the reference's deep-only "
                "forward reads a bias it never creates (model/DeepFMs.py:467)");
  if (c.use_logit && c.use_deep)
    return fail(DFWFM_ERR_UNSUPPORTED,
                "use_logit with use_deep: the reference's deep branch then indexes Xi with all "
                "field_size columns and fails (model/DeepFMs.py:402)");
  if (c.use_logit && c.use_fwlw)
    return fail(DFWFM_ERR_INVALID_ARG, "use_logit with use_fwlw has no first-order tables");
  const int F = c.field_size, D = c.embedding_size;
  int H = 0, N = 0, NT = 0, TPW = 0;
  if (c.use_deep) {
    H = c.h_depth;
    N = c.deep_nodes;
    if (H < 1 || H > 16) return fail(DFWFM_ERR_UNSUPPORTED, "h_depth %d outside [1, 16]", H);
    NT = (N + 15) / 16;
    TPW = (NT + 3) / 4;
    if (N < 1 || TPW > kMaxTPW)
      return fail(DFWFM_ERR_UNSUPPORTED, "deep_nodes %d outside [1, %d]", N, 64 * kMaxTPW);
  }

  dfwfm_model* m = new dfwfm_model();
  memset(m, 0, sizeof *m);
  m->cfg = c;
  m->deterministic = true;  // fixed-order gradient sums unless dfwfm_set_deterministic(m, 0)
  hipError_t e = hipGetDevice(&m->device);
  if (e != hipSuccess) {
    delete m;
    return hip_fail(e, "hipGetDevice");
  }
  m->F = F;
  m->D = D;
  m->num = c.numerical;
  m->H = H;
  m->N = N;
  m->NT = NT;
  m->TPW = TPW;
  m->NC0 = (F * D + 15) / 16;
  m->MT = (F + 15) / 16;
  m->S = (F + 3) / 4;
  fw_schedule(m->MT, D, m->S, 4, m->fw_list4, m->fw_off4);
  fw_schedule(m->MT, D, m->S, 8, m->fw_list8, m->fw_off8);
  // E-tile columns read by the MLP (NC0*16) and by the FwFM contraction (4*S fields)
  m->W0 = m->NC0 * 16 > 4 * m->S * D ? m->NC0 * 16 : 4 * m->S * D;
  const int kx = m->W0 > NT * 16 ? m->W0 : NT * 16;
  m->SX = r4(kx) + 4;
  m->SY = c.use_deep ? NT * 16 + 4 : 0;
  // one wave per SIMD (two per SIMD splitting K measured slower, removed in round 6)
  m->KS = 1;
  // 4k+1 output tiles (N = 400: 25): the last tile is split by K over the four waves instead of
  // giving one SIMD an extra whole tile
  m->TPWF = TPW;
  m->tail = 0;
  if (c.use_deep && m->KS == 1 && NT % 4 == 1 && NT >= 5 && m->NC0 >= 4 && m->NC0 <= 4 * kTailC &&
      NT <= 4 * kTailC) {
    m->TPWF = NT / 4;
    m->tail = 1;
  }
  const bool second = c.use_fwfm || c.use_fm;
  m->flags = (second ? kHasSecond : 0) | (c.use_deep ? kHasDeep : 0) |
             (c.use_fwlw ? kFoFwlw : kFoTables) | ((second && c.use_lw) ? kFoLw : 0) |
             ((second || c.use_deep) ? kNeedE : 0);
  const LdsLayout L = lds_layout(F, D, m->MT, m->S, m->SX, m->SY, m->TPWF > 0 ? m->TPWF : 1, m->KS,
                                 c.use_deep != 0, m->tail != 0);
  m->lds_bytes = sizeof(float) * (size_t)L.total;
  m->lds_gather = sizeof(float) * (size_t)lds_layout(F, D, m->MT, m->S, m->SX, m->SY, m->TPWF > 0 ? m->TPWF : 1,
                                                     1, false, false).total;
  // inference: eight tile groups (two waves per SIMD at <= 128 registers) when the layer fits them
  // (<= 32 output tiles); DFWFM_DIAG ng=4 selects the four-wave kernel the training forward uses
  m->NG = 4;
  m->TPWI = m->TPWF;
  m->tailI = m->tail;
  m->lds_inf = m->lds_bytes;
  if (!c.use_deep)  // the MLP-free forward runs on eight waves (fwd_kernel PART 3): its layout's per-wave slots
    m->lds_inf = sizeof(float) * (size_t)lds_layout(F, D, m->MT, m->S, m->SX, m->SY, 1, 1, false, false, 8).total;
  if (c.use_deep && m->KS == 1 && NT <= 32 && m->NC0 <= 32) {
    if (diag_opt("ng", 8) == 8) {  // (DFWFM_DIAG ng=4: the four-wave kernel, tests)
      m->NG = 8;
      m->tailI = (NT % 8 == 1 && NT >= 9 && m->NC0 >= 8) ? 1 : 0;
      m->TPWI = m->tailI ? NT / 8 : (NT + 7) / 8;
      m->lds_inf = sizeof(float) * (size_t)lds_layout(F, D, m->MT, m->S, m->SX, m->SY, m->TPWI, 1, true,
                                                      m->tailI != 0, 8).total;
    }
  }
  // 32-sample workgroups (fwd32_kernel: every weight fragment feeds both 16-row tiles) for the static 3x400 form,
  // chosen per launch when the batch's 32-sample workgroups still cover every CU the stream may use (a stream
  // masked to half of the chip, or a batch of >= 32 x CUs rows; else the 16-sample kernel keeps all CUs busy);
  // DFWFM_DIAG r32=0 never, r32=1 always (tests)
  {
    const int r32 = diag_opt("r32", -1);
    const int mode = r32 < 0 ? 1 : (r32 != 0 ? 2 : 0);
    m->r32 = (c.use_deep && fwd32_supported(F, D, H, NT, m->NC0, m->tailI, m->NG)) ? mode : 0;
    m->lds_r32 = m->r32 ? fwd32_lds_bytes(F, D, m->MT, m->S, m->SX) : 0;
    m->lds_ftrain = (c.use_deep && ftrain_supported(F, D, H, NT, m->NC0, m->tailI, m->NG))
                        ? ftrain_lds_bytes(F, D, m->MT, m->S, m->SX, m->SY) : 0;
    if (m->lds_ftrain > 160 * 1024) m->lds_ftrain = 0;
  }
  // (the split forward -- gather / shallow part and MLP as two launches -- measured slower than the fused launch
  // and was removed in round 6; dfwfm_forward_gather gives the gather its own launch for measurement)
  if (m->lds_bytes > 160 * 1024 || m->lds_inf > 160 * 1024) {
    free_model(m);
    return fail(DFWFM_ERR_UNSUPPORTED, "LDS tile of %zu bytes exceeds 160 KiB", m->lds_bytes);
  }

  int rc = DFWFM_OK;
  if ((rc = dev_alloc(&m->d_fields, F)) || (rc = dev_alloc(&m->d_upack, (size_t)m->MT * m->S * 64)) ||
      (rc = dev_alloc(&m->d_err, 1)) ||
      (rc = dev_alloc(&m->d_fwlw, (size_t)F * D)) || (rc = dev_alloc(&m->d_lw, F)) ||
      (rc = dev_alloc(&m->d_bias, 1))) {
    free_model(m);
    return rc;
  }
  if ((rc = dev_alloc(&m->d_rsk, (size_t)m->MT * m->S * 64))) {
    free_model(m);
    return rc;
  }
  if (c.use_deep) {
    m->wpack_elems = (size_t)NT * m->NC0 * 64 + (size_t)(H - 1) * NT * NT * 64;
    if (m->wpack_elems * sizeof(float4) >= (size_t)1 << 31) {
      free_model(m);
      return fail(DFWFM_ERR_UNSUPPORTED, "packed MLP weights exceed the 2 GiB buffer-descriptor range");
    }
    // transposed packs: layer 1 block [NC0 tiles][NT chunks], layers 2..H [NT][NT]; same total
    m->wtpack_elems = m->wpack_elems;
    m->wt_off[1] = 0;
    for (int l = 2; l <= H; ++l) m->wt_off[l] = m->wt_off[l - 1] + (l == 2 ? m->NC0 : NT) * NT * 64;
    if ((rc = dev_alloc(&m->d_wtpack, m->wtpack_elems)) || (rc = dev_alloc(&m->d_wpack, m->wpack_elems)) ||
        (rc = dev_alloc(&m->d_mlp_b, (size_t)H * NT * 16)) || (rc = dev_alloc(&m->d_fc, (size_t)NT * 16))) {
      free_model(m);
      return rc;
    }
  }
  e = hipMemset(m->d_err, 0, sizeof(int32_t));
  if (e == hipSuccess) e = hipMemset(m->d_upack, 0, sizeof(float) * (size_t)m->MT * m->S * 64);
  if (e != hipSuccess) {
    free_model(m);
    return hip_fail(e, "hipMemset");
  }
  *out = m;
  return DFWFM_OK;
}

void dfwfm_model_destroy(dfwfm_model* m) { free_model(m); }

int dfwfm_model_set_tables(dfwfm_model* m, const dfwfm_field_tables* t, int32_t n, void* stream) {
  if (!m || !t) return fail(DFWFM_ERR_INVALID_ARG, "null argument");
  if (n != m->F) return fail(DFWFM_ERR_INVALID_ARG, "%d tables for %d fields", n, m->F);
  const bool need_fo = (m->flags & kFoTables) != 0;
  const bool need_e = (m->flags & kNeedE) != 0;
  for (int f = 0; f < n; ++f) {
    const dfwfm_field_tables& x = t[f];
    if (need_e && !x.emb2) return fail(DFWFM_ERR_INVALID_ARG, "field %d: emb2 is null", f);
    if (need_fo && !x.emb1) return fail(DFWFM_ERR_INVALID_ARG, "field %d: emb1 is null", f);
    if (x.num_categories < 1) return fail(DFWFM_ERR_INVALID_ARG, "field %d: num_categories < 1", f);
    if (x.qr_collisions < 0) return fail(DFWFM_ERR_INVALID_ARG, "field %d: qr_collisions < 0", f);
    if (x.qr_collisions > 0) {
      if (f < m->num) return fail(DFWFM_ERR_INVALID_ARG, "field %d: numerical field cannot be QR", f);
      if ((need_e && !x.emb2_r) || (need_fo && !x.emb1_r))
        return fail(DFWFM_ERR_INVALID_ARG, "field %d: QR remainder table is null", f);
      if (x.qr_operation != 0 && x.qr_operation != 1)
        return fail(DFWFM_ERR_UNSUPPORTED, "field %d: QR operation %d (only mult=0, add=1)", f,
                    x.qr_operation);
    }
    const uintptr_t align = (m->D % 4 == 0) ? 16 : (m->D % 2 == 0 ? 8 : 4);
    if (((uintptr_t)x.emb2 % align) || (x.emb2_r && ((uintptr_t)x.emb2_r % align)))
      return fail(DFWFM_ERR_UNSUPPORTED, "field %d: table base not %zu-byte aligned", f, (size_t)align);
  }
  // Device copy; for a QR field the accepted index range is every i whose quotient row exists,
  // [0, ceil(n/c) * c) -- F.embedding_bag on weight_q only rejects i // c >= ceil(n/c).
  FieldDev host[64];
  memcpy(host, t, sizeof(dfwfm_field_tables) * n);
  for (int f = 0; f < n; ++f)
    if (host[f].c > 0) host[f].n = (host[f].n + host[f].c - 1) / host[f].c * host[f].c;
  memcpy(m->h_fields, host, sizeof(FieldDev) * n);
  m->pkw = 0;  // the serving copy was built from the old tables
  m->flags &= ~kHasQR;
  for (int f = 0; f < n; ++f)
    if (host[f].c > 0) m->flags |= kHasQR;
  HIP_TRY(hipMemcpyAsync(m->d_fields, host, sizeof(FieldDev) * n, hipMemcpyHostToDevice, (hipStream_t)stream));
  HIP_TRY(hipStreamSynchronize((hipStream_t)stream));  // `host` is a stack buffer
  m->tables_set = true;
  return DFWFM_OK;
}

static int set_dense_impl(dfwfm_model* m, const float* field_cov, const float* fwfm_lin, const float* fm_1st,
                          const float* bias, const float* const* lin_w, const float* const* lin_b,
                          const float* fc_w, float* zero, int64_t nzero, void* stream) {
  if (!m) return fail(DFWFM_ERR_INVALID_ARG, "null model");
  if (nzero < 0 || (nzero > 0 && (!zero || (nzero & 3) || (reinterpret_cast<uintptr_t>(zero) & 15))))
    return fail(DFWFM_ERR_INVALID_ARG, "zero range: 16-byte aligned, a multiple of 4 floats");
  hipStream_t s = (hipStream_t)stream;
  const dfwfm_config& c = m->cfg;
  if (c.use_fwfm && !field_cov) return fail(DFWFM_ERR_INVALID_ARG, "use_fwfm needs field_cov");
  if ((m->flags & kFoFwlw) && !fwfm_lin) return fail(DFWFM_ERR_INVALID_ARG, "use_fwlw needs fwfm_linear");
  if ((m->flags & kFoLw) && !fm_1st) return fail(DFWFM_ERR_INVALID_ARG, "use_lw needs fm_1st");
  if (!bias) return fail(DFWFM_ERR_INVALID_ARG, "bias is required");
  PackList L;
  memset(&L, 0, sizeof L);
  int blocks = 0;
  auto job = [&](int type, const float* src, void* dst, int64_t total, int a, int b, int d) {
    PackJob& j = L.j[L.n++];
    j.src = src;
    j.dst = reinterpret_cast<float*>(dst);
    j.total = total;
    j.type = type;
    j.a = a;
    j.b = b;
    j.d = d;
    j.block0 = blocks;
    blocks += (int)((total + 255) / 256);
  };
  // the zero range first (its blocks are the long ones), in float4 units of kPackZeroPT per thread
  if (nzero > 0) {
    const int64_t n4 = nzero / 4;
    if ((n4 + 256 * kPackZeroPT - 1) / (256 * kPackZeroPT) > 0x3fffffff) return fail(DFWFM_ERR_UNSUPPORTED, "zero range");
    PackJob& j = L.j[L.n++];
    j.src = nullptr;
    j.dst = zero;
    j.total = n4;
    j.type = kPackZero;
    j.a = j.b = j.d = 0;
    j.block0 = blocks;
    blocks += (int)((n4 + 256 * kPackZeroPT - 1) / (256 * kPackZeroPT));
  }
  if (c.use_fwfm || c.use_fm) {
    const int64_t tot = (int64_t)m->MT * m->S * 64;
    job(kPackFwfm, field_cov, m->d_upack, tot, m->F, c.use_fm ? 1 : 0, m->S);
    job(kPackFwfmSym, field_cov, m->d_rsk, tot, m->F, c.use_fm ? 1 : 0, m->S);
  }
  if (m->flags & kFoFwlw) job(kPackPad, fwfm_lin, m->d_fwlw, m->F * m->D, m->F * m->D, 0, 0);
  if (m->flags & kFoLw) job(kPackPad, fm_1st, m->d_lw, m->F, m->F, 0, 0);
  job(kPackPad, bias, m->d_bias, 1, 1, 0, 0);
  if (c.use_deep) {
    if (!lin_w || !lin_b || !fc_w) return fail(DFWFM_ERR_INVALID_ARG, "use_deep needs MLP weights");
    size_t off = 0;
    for (int h = 0; h < m->H; ++h) {
      if (!lin_w[h] || !lin_b[h]) return fail(DFWFM_ERR_INVALID_ARG, "layer %d weight/bias is null", h);
      const int K = h == 0 ? m->F * m->D : m->N;
      const int NC = h == 0 ? m->NC0 : m->NT;
      const int64_t tot = (int64_t)m->NT * NC * 64;
      job(kPackLinear, lin_w[h], m->d_wpack + off, tot, m->N, K, NC);
      job(kPackLinearT, lin_w[h], m->d_wtpack + m->wt_off[h + 1], tot, m->N, K, m->NT);
      job(kPackPad, lin_b[h], m->d_mlp_b + (size_t)h * m->NT * 16, m->NT * 16, m->N, 0, 0);
      off += (size_t)tot;
    }
    job(kPackPad, fc_w, m->d_fc, m->NT * 16, m->N, 0, 0);
  }
  hipError_t e = launch_pack_list(L, blocks, s);
  if (e != hipSuccess) return hip_fail(e, "pack launch");
  m->dense_set = true;
  m->sp = 0;  // new weights: the sparse tower's ELL is stale until rebuilt
  m->flags &= ~kPairs;  // and so is the FwFM pair list
  for (int h = 0; h < m->H; ++h) m->lin_w[h] = lin_w ? lin_w[h] : nullptr;
  return DFWFM_OK;
}

int dfwfm_model_set_dense(dfwfm_model* m, const float* field_cov, const float* fwfm_lin, const float* fm_1st,
                          const float* bias, const float* const* lin_w, const float* const* lin_b,
                          const float* fc_w, void* stream) {
  return set_dense_impl(m, field_cov, fwfm_lin, fm_1st, bias, lin_w, lin_b, fc_w, nullptr, 0, stream);
}

int dfwfm_model_set_dense_zero(dfwfm_model* m, const float* field_cov, const float* fwfm_lin, const float* fm_1st,
                               const float* bias, const float* const* lin_w, const float* const* lin_b,
                               const float* fc_w, float* zero, int64_t nzero, void* stream) {
  return set_dense_impl(m, field_cov, fwfm_lin, fm_1st, bias, lin_w, lin_b, fc_w, zero, nzero, stream);
}

}  // extern "C"

namespace {

int check_inputs(dfwfm_model* m, const int64_t* xi, int64_t xi_stride, const float* xv, int64_t xv_stride,
                 int64_t batch, const void* out) {
  if (batch < 0) return fail(DFWFM_ERR_INVALID_ARG, "negative batch");
  if (!m->tables_set || !m->dense_set)
    return fail(DFWFM_ERR_STATE, "set_tables and set_dense must precede forward");
  if (batch == 0) return DFWFM_OK;
  const int ncat = m->F - m->num;
  if (!out || (ncat > 0 && !xi) || (m->num > 0 && !xv))
    return fail(DFWFM_ERR_INVALID_ARG, "null input/output pointer");
  if (ncat > 0 && xi_stride < ncat) return fail(DFWFM_ERR_INVALID_ARG, "xi_stride < F - numerical");
  if (m->num > 0 && xv_stride < m->num) return fail(DFWFM_ERR_INVALID_ARG, "xv_stride < numerical");
  if ((batch + kBM - 1) / kBM > 0x7fffffff) return fail(DFWFM_ERR_UNSUPPORTED, "batch too large");
  return DFWFM_OK;
}

void fill_forward_args(const dfwfm_model* m, FwdArgs& a, const int64_t* xi, int64_t xi_stride, const float* xv,
                       int64_t xv_stride, int64_t batch, float* out) {
  memset(&a, 0, sizeof a);
  a.fields = m->d_fields;
  a.xi = xi;
  a.xi_stride = xi_stride;
  a.xv = xv;
  a.xv_stride = xv_stride;
  a.batch = batch;
  a.out = out;
  a.err = m->d_err;
  a.upack = m->d_upack;
  a.pk = m->pkw ? m->d_pk : nullptr;
  a.pkw = m->pkw;
  a.pairs = m->d_pairs;
  a.npairs = m->npairs;
  a.fwlw = m->d_fwlw;
  a.lw = m->d_lw;
  a.bias = m->d_bias;
  a.wpack = m->d_wpack;
  a.wpack_bytes = (int32_t)(m->wpack_elems * sizeof(float4));
  a.mlp_b = m->d_mlp_b;
  a.fc = m->d_fc;
  a.F = m->F;
  a.num = m->num;
  a.H = m->H;
  a.N = m->N;
  a.NT = m->NT;
  a.NC0 = m->NC0;
  a.MT = m->MT;
  a.S = m->S;
  a.W0 = m->W0;
  a.tail = m->tail;
  a.SX = m->SX;
  a.SY = m->SY;
  a.flags = m->flags;
  // the MLP-free forward's FwFM form: U'E pieces (default; batch sets 2.34 vs 2.59 us per batch at 2000 steps, 2.85-2.90
  // vs 3.05 at 20, profiles/r05/r05l_*; a lone batch on eight waves 7.7 vs 7.3 us) or per-sample Gram tiles
  // (the Gram form remains for MT > 3) -- the same form for a batch set and a lone batch, so a set's logits stay bit-identical
  // to each batch's own forward; pieces only while the U' fragments fit the eight-wave form's registers (MT <= 3)
  if (!m->cfg.use_deep && m->MT <= 3) a.flags |= kP3Pieces;
  // the static K loop (fwd_kernel NS = 25) when every layer is 25 chunks deep and 25 tiles wide
  a.ns = (m->NC0 == 25 && m->NT == 25) ? 25 : 0;
  memcpy(a.fw_list4, m->fw_list4, sizeof a.fw_list4);
  memcpy(a.fw_list8, m->fw_list8, sizeof a.fw_list8);
  memcpy(a.fw_off4, m->fw_off4, sizeof a.fw_off4);
  memcpy(a.fw_off8, m->fw_off8, sizeof a.fw_off8);
}

// The weight-gradient GEMM's grid for `batch` rows: 80 x 80 blocks per layer (per_split of them over all layers) in
// `splits` batch splits of `rows` rows.  One workgroup per CU at most (tools/ubench_dw, Criteo-39, B = 4096: 3 splits
// = 225 workgroups 42 us; 6 splits 47 us; past one round of workgroups 60+ us), each split over >= 128 rows.
// `cap` (optional) = the split count before the rows are rounded to whole k-step groups: it bounds `splits` for this
// batch AND for every smaller one (each term that sets it is non-decreasing in the batch), so slices sized from the
// cap of the workspace's batch serve every ragged batch after it.
int dw_plan(const dfwfm_model* m, int64_t batch, int* per_split, int64_t* splits, int64_t* rows,
            int64_t* cap = nullptr) {
  const int edge = kDwEdge, quantum = kDwRows;
  const int nnb = (m->N + edge - 1) / edge;
  int ps = 0;
  for (int l = 1; l <= m->H; ++l) ps += nnb * (((l == 1 ? m->F * m->D : m->N) + edge - 1) / edge);
  *per_split = ps;
  *splits = *rows = 0;
  if (cap) *cap = 0;
  if (ps == 0 || batch <= 0) return DFWFM_OK;
  int64_t sp = 256 / ps;
  const int64_t max_splits = (batch + 127) / 128;
  if (sp > max_splits) sp = max_splits;
  if (sp < 1) sp = 1;
  // a wave's raw-buffer range (a quarter of a split's rows x the widest row, in bytes) must fit 31 bits
  const int64_t wmax = r4(m->F * m->D) > m->N ? r4(m->F * m->D) : m->N;
  const int64_t rows_cap = ((0x7fffffffLL / (wmax * 4)) * 4 - 4 * quantum) / quantum * quantum;
  if (rows_cap < quantum) return fail(DFWFM_ERR_UNSUPPORTED, "MLP rows of %lld floats", (long long)wmax);
  if ((batch + sp - 1) / sp > rows_cap) sp = (batch + rows_cap - 1) / rows_cap;
  if (cap) *cap = sp;
  int64_t r = (batch + sp - 1) / sp;
  r = (r + quantum - 1) / quantum * quantum;  // whole k-step groups per wave
  *splits = (batch + r - 1) / r;
  *rows = r;
  return DFWFM_OK;
}

// Activation workspace for `batch` rows: E [B][F*D], fo [B][F], X_0 [B][r4(F*D)], X_h and G_h [B][N]; and the
// weight-gradient GEMM's split slices.
int ensure_workspace(dfwfm_model* m, int64_t batch) {
  if (batch <= m->ws_batch) return DFWFM_OK;
  const int64_t FD = (int64_t)m->F * m->D;
  const int64_t SE = r4((int)FD);
  const int64_t per_row = SE + FD + m->F + (m->H > 0 ? SE + 2 * (int64_t)m->H * m->N : 0);
  const int64_t keys_stride = (batch + 3) & ~(int64_t)3;  // the categorical keys, column-major
  const int64_t keys_words = (int64_t)(m->F - m->num) * keys_stride;
  const int64_t red_blocks = (batch + kBM - 1) / kBM;
  const int64_t red_floats = red_blocks * red_outputs(m->F, m->D, m->N, m->num);
  int per_split = 0;
  int64_t splits = 0, rows = 0, cap = 0;
  int rc = dw_plan(m, batch, &per_split, &splits, &rows, &cap);
  if (rc != DFWFM_OK) return rc;
  // sized from the cap, not from this batch's rounded split count: a smaller (ragged) batch can round to more splits
  const int64_t slices = cap > 1 ? (int64_t)per_split * cap : 0;
  const int64_t dw_floats = slices * (kDwEdge * kDwEdge + kDwEdge);  // the blocks' and the bias sums' slices
  if (m->d_ws) (void)hipFree(m->d_ws);
  m->d_ws = nullptr;
  m->ws_batch = 0;
  const size_t total = (size_t)(per_row * batch + red_floats + dw_floats + keys_words + 64);
  HIP_TRY(hipMalloc(reinterpret_cast<void**>(&m->d_ws), sizeof(float) * total));
  // every array starts 16-byte aligned: the row counts are multiples of 4 or the offsets are padded
  auto al = [](int64_t x) { return (x + 3) & ~(int64_t)3; };
  float* p = m->d_ws;
  m->dw_part = p;   p += slices * kDwEdge * kDwEdge;
  m->dw_bpart = p;  p += al(slices * kDwEdge);
  m->dw_slices = slices;
  m->sv_e = p;   p += al(SE * batch);
  m->sv_de = p;  p += al(FD * batch);
  m->red_part = p;  p += al(red_floats);
  m->sv_fo = p;  p += al((int64_t)m->F * batch);
  m->sv_keys = reinterpret_cast<int32_t*>(p);  p += keys_words;
  m->keys_stride = keys_stride;
  for (int h = 0; h <= kMaxH; ++h) m->sv_x[h] = m->sv_g[h] = nullptr;
  if (m->H > 0) {
    m->sv_x0 = p;  p += SE * batch;
    for (int h = 1; h <= m->H; ++h) {
      m->sv_x[h] = p;  p += (int64_t)m->N * batch;
      m->sv_g[h] = p;  p += (int64_t)m->N * batch;
    }
  }
  m->ws_batch = batch;
  m->ws_gen++;
  return DFWFM_OK;
}

// the sparse deep tower's forward workspace (dfwfm_forward_ws): the gather launch's E rows [B][NC0*16], then first + second [B]
size_t split_e_floats(const dfwfm_model* m, int64_t batch) { return (size_t)batch * m->NC0 * 16; }
size_t split_ws_bytes(const dfwfm_model* m, int64_t batch) {
  return sizeof(float) * (split_e_floats(m, batch) + (size_t)batch);
}

// diagnostics only: with DFWFM_DIAG stamps=<which> the launch records per-workgroup phase clocks
int diag_stamps_buffer(dfwfm_model* m, int64_t batch, int which, uint64_t** out) {
  *out = nullptr;
  if (diag_opt("stamps", 0) != which) return DFWFM_OK;
  const size_t grid = (size_t)((batch + kBM - 1) / kBM);
  // DFWFM_DIAG ring=R: R launches in a row (e.g. captured into graphs on several streams) each get
  // their own slice, for a cross-launch timeline (tools/timeline.py)
  const size_t ring = diag_opt("ring", 1) > 1 ? (size_t)diag_opt("ring", 1) : 1;
  if (grid > m->stamps_cap || ring != m->stamps_ring) {
    if (m->d_stamps) (void)hipFree(m->d_stamps);
    m->d_stamps = nullptr;
    m->stamps_cap = 0;
    HIP_TRY(hipMalloc(reinterpret_cast<void**>(&m->d_stamps), ring * grid * kStampSlots * sizeof(uint64_t)));
    m->stamps_cap = grid;
    m->stamps_ring = ring;
    m->stamps_next = 0;
  }
  *out = m->d_stamps + (m->stamps_next % ring) * m->stamps_cap * kStampSlots;
  m->stamps_next++;
  return DFWFM_OK;
}

// CUs a stream may use (its CU mask; cached per stream handle).  The cache is shared by every host thread that
// uses the model, so it is guarded; a handle the runtime reuses for a stream with another mask keeps the old count
// until replaced, which only changes which (bit-identical) forward kernel runs.
std::mutex g_cu_mu;

int stream_cu_count(dfwfm_model* m, void* stream) {
  std::lock_guard<std::mutex> lock(g_cu_mu);
  if (m->dev_cus == 0) {
    hipDeviceProp_t prop;
    m->dev_cus = hipGetDeviceProperties(&prop, m->device) == hipSuccess ? prop.multiProcessorCount : 256;
  }
  const int cached = m->cu_n < 8 ? m->cu_n : 8;
  for (int i = 0; i < cached; ++i)
    if (m->cu_stream[i] == stream) return m->cu_count[i];
  int n = 0;
  uint32_t mask[64] = {0};
  if (hipExtStreamGetCUMask((hipStream_t)stream, 64, mask) == hipSuccess) {
    for (int i = 0; i < 64; ++i) n += __builtin_popcount(mask[i]);
  } else {
    (void)hipGetLastError();
    hipDeviceProp_t prop;
    n = hipGetDeviceProperties(&prop, m->device) == hipSuccess ? prop.multiProcessorCount : 256;
  }
  const int slot = m->cu_n < 8 ? m->cu_n++ : (m->cu_next++ & 7);
  m->cu_stream[slot] = stream;
  m->cu_count[slot] = n > 0 ? n : 256;
  return m->cu_count[slot];
}

// fwd32 (32-sample workgroups) when its workgroups give every CU of the stream two of them (two per CU hide each
// other's gather and shallow phases); on a CU-masked stream (the caller runs several batches side by side, one
// stream per part of the chip) one per CU is enough.  Otherwise the 16-sample kernel: twice the workgroups for the
// same rows -- a lone 8192-row batch is 512 of them, two per CU, where fwd32 would leave each CU one.
bool use_fwd32(dfwfm_model* m, int64_t batch, void* stream) {
  if (m->r32 == 0) return false;
  if (m->r32 == 2) return true;
  const int cus = stream_cu_count(m, stream);
  const bool masked = cus < m->dev_cus;
  return (batch + 31) / 32 >= (masked ? 1 : 2) * (int64_t)cus;
}

}  // namespace

extern "C" {

int dfwfm_forward(dfwfm_model* m, const int64_t* xi, int64_t xi_stride, const float* xv, int64_t xv_stride,
                  int64_t batch, float* out, void* stream) {
  if (!m) return fail(DFWFM_ERR_INVALID_ARG, "null model");
  int rc = check_inputs(m, xi, xi_stride, xv, xv_stride, batch, out);
  if (rc != DFWFM_OK || batch == 0) return rc;
  FwdArgs a;
  fill_forward_args(m, a, xi, xi_stride, xv, xv_stride, batch, out);
  // diagnostics only (phase timing): DFWFM_DIAG drop_flags clears flag bits, results become invalid
  a.flags &= ~diag_opt("drop_flags", 0);
  // gather / shallow phases at raised wave priority: beside the other batch's MLP on the same CU they otherwise lose
  // the issue arbitration -- 33.71 -> 33.38 us per batch; the fwd32 epilogue priority and the deferred split-tile
  // barrier (set kernel only)
  a.flags |= kPrio | kPrioEpi | kDeferTail;
  // diagnostics only: DFWFM_DIAG stamps=1 records per-workgroup phase clocks (dfwfm_diag_stamps)
  if ((rc = diag_stamps_buffer(m, batch, 1, &a.stamps)) != DFWFM_OK) return rc;
  a.tail = m->tailI;
  const bool r32 = (a.flags & kHasDeep) && use_fwd32(m, batch, stream);
  hipError_t e = r32 ? launch_fwd32(a, m->D, m->lds_r32, (hipStream_t)stream)
                     : launch_forward(a, m->D, m->TPWI > 0 ? m->TPWI : 1, m->KS, m->NG, m->lds_inf, (hipStream_t)stream);
  if (e != hipSuccess) return hip_fail(e, "forward launch");
  return DFWFM_OK;
}

int dfwfm_forward_batches(dfwfm_model* m, int32_t nb, const int64_t* const* xi, int64_t xi_stride,
                          const float* const* xv, int64_t xv_stride, int64_t batch, float* const* out, void* stream) {
  if (!m) return fail(DFWFM_ERR_INVALID_ARG, "null model");
  if (nb < 0) return fail(DFWFM_ERR_INVALID_ARG, "negative batch count");
  if (nb == 0) return DFWFM_OK;
  if (!xi || !xv || !out) return fail(DFWFM_ERR_INVALID_ARG, "null pointer array");
  for (int32_t i = 0; i < nb; ++i) {
    const int rc = check_inputs(m, xi[i], xi_stride, xv[i], xv_stride, batch, out[i]);
    if (rc != DFWFM_OK) return rc;
  }
  if (batch == 0) return DFWFM_OK;
  if (nb == 1) {
    for (int32_t i = 0; i < nb; ++i) {
      const int rc = dfwfm_forward(m, xi[i], xi_stride, xv[i], xv_stride, batch, out[i], stream);
      if (rc != DFWFM_OK) return rc;
    }
    return DFWFM_OK;
  }
  if ((int64_t)nb * ((batch + kBM - 1) / kBM) > 0x7fffffff) return fail(DFWFM_ERR_UNSUPPORTED, "batch set too large");
  // the kernel for the first launch's rows (a set of up to kMaxSet batches); later launches of a larger set use it too
  const int64_t set_rows = (int64_t)(nb < kMaxSet ? nb : kMaxSet) * batch;
  const bool r32 = m->cfg.use_deep && use_fwd32(m, set_rows, stream);
  const int rows = r32 ? 32 : kBM;
  for (int32_t i0 = 0; i0 < nb; i0 += kMaxSet) {
    const int32_t n = nb - i0 < kMaxSet ? nb - i0 : kMaxSet;
    FwdArgs a;
    fill_forward_args(m, a, xi[i0], xi_stride, xv[i0], xv_stride, batch, out[i0]);
    // fwd32 schedule: raised priority in the MLP epilogues, the split tile's barrier inside the next K loop --
    // 30.33 -> 30.08 us per batch at 2000 steps, 31.3 -> 31.05 on a 20-batch set (r03be)
    a.flags |= kPrio | kPrioEpi | kDeferTail;
    a.tail = m->tailI;
    if (n > 1) {
      a.nb = n;
      a.tiles = (int32_t)((batch + rows - 1) / rows);
      for (int32_t j = 0; j < n; ++j) {
        a.set_xi[j] = xi[i0 + j];
        a.set_xv[j] = xv[i0 + j];
        a.set_out[j] = out[i0 + j];
      }
    }
    int rc = diag_stamps_buffer(m, (int64_t)n * a.tiles * rows, 1, &a.stamps);
    if (rc != DFWFM_OK) return rc;
    const hipError_t e = r32 ? launch_fwd32(a, m->D, m->lds_r32, (hipStream_t)stream)
                             : launch_forward(a, m->D, m->TPWI > 0 ? m->TPWI : 1, m->KS, m->NG, m->lds_inf,
                                              (hipStream_t)stream);
    if (e != hipSuccess) return hip_fail(e, "batch-set forward launch");
  }
  return DFWFM_OK;
}

int dfwfm_forward_workspace_bytes(dfwfm_model* m, int64_t batch, size_t* bytes) {
  if (!m || !bytes || batch < 0) return fail(DFWFM_ERR_INVALID_ARG, "null argument");
  *bytes = m->sp ? split_ws_bytes(m, batch) : 0;
  return DFWFM_OK;
}

int dfwfm_forward_ws(dfwfm_model* m, const int64_t* xi, int64_t xi_stride, const float* xv, int64_t xv_stride,
                     int64_t batch, float* out, void* workspace, size_t ws_bytes, void* stream) {
  if (!m) return fail(DFWFM_ERR_INVALID_ARG, "null model");
  if (!m->sp || !workspace) return dfwfm_forward(m, xi, xi_stride, xv, xv_stride, batch, out, stream);
  int rc = check_inputs(m, xi, xi_stride, xv, xv_stride, batch, out);
  if (rc != DFWFM_OK || batch == 0) return rc;
  if (ws_bytes < split_ws_bytes(m, batch))
    return fail(DFWFM_ERR_INVALID_ARG, "workspace of %zu bytes < %zu (dfwfm_forward_workspace_bytes)", ws_bytes,
                split_ws_bytes(m, batch));
  if (reinterpret_cast<uintptr_t>(workspace) % 16) return fail(DFWFM_ERR_INVALID_ARG, "workspace not 16-byte aligned");
  FwdArgs a;
  fill_forward_args(m, a, xi, xi_stride, xv, xv_stride, batch, out);
  a.part_stride = m->NC0 * 16;
  a.part_e = static_cast<float*>(workspace);
  a.part_fs = a.part_e + split_e_floats(m, batch);
  if ((rc = diag_stamps_buffer(m, batch, 1, &a.stamps)) != DFWFM_OK) return rc;
  a.tail = m->tailI;
  {
    // pruned deep tower: the gather launch, then the sparse MLP over the ELL (dfwfm_spmlp.hip)
    hipError_t e = launch_forward_gather(a, m->D, m->lds_gather, (hipStream_t)stream);
    if (e != hipSuccess) return hip_fail(e, "gather launch");
    SpMlpArgs sa;
    memset(&sa, 0, sizeof sa);
    sa.part_e = a.part_e;
    sa.part_fs = a.part_fs;
    sa.part_stride = a.part_stride;
    sa.K0p = a.part_stride;
    sa.ell = m->d_ell;
    sa.gcnt = m->d_cnt + m->H * m->N;
    for (int h = 0; h < m->H; ++h) {
      sa.W[h] = m->spW[h];
      sa.off[h] = m->spoff[h];
    }
    sa.mlp_b = m->d_mlp_b;
    sa.fc = m->d_fc;
    sa.bias = m->d_bias;
    sa.out = out;
    sa.batch = batch;
    sa.H = m->H;
    sa.N = m->N;
    sa.NT = m->NT;
    e = launch_sparse_mlp(sa, (hipStream_t)stream);
    if (e != hipSuccess) return hip_fail(e, "sparse MLP launch");
    return DFWFM_OK;
  }
}

int dfwfm_forward_gather(dfwfm_model* m, const int64_t* xi, int64_t xi_stride, const float* xv, int64_t xv_stride,
                         int64_t batch, float* deep_emb, int64_t deep_emb_stride, float* first_second, void* stream) {
  if (!m) return fail(DFWFM_ERR_INVALID_ARG, "null model");
  if (!m->cfg.use_deep) return fail(DFWFM_ERR_UNSUPPORTED, "forward_gather: the model has no deep tower");
  int rc = check_inputs(m, xi, xi_stride, xv, xv_stride, batch, first_second);
  if (rc != DFWFM_OK || batch == 0) return rc;
  if (!deep_emb || deep_emb_stride != (int64_t)m->NC0 * 16)
    return fail(DFWFM_ERR_INVALID_ARG, "deep_emb stride %lld, need %d", (long long)deep_emb_stride, m->NC0 * 16);
  if (reinterpret_cast<uintptr_t>(deep_emb) % 16) return fail(DFWFM_ERR_INVALID_ARG, "deep_emb not 16-byte aligned");
  // the MLP-free forward's kernel (fwd_kernel PART 3: the serving copy, the U'E FwFM pieces) storing the E tile and
  // first + second instead of the logit
  FwdArgs a;
  fill_forward_args(m, a, xi, xi_stride, xv, xv_stride, batch, nullptr);
  a.flags &= ~kHasDeep;
  if (m->MT <= 3) a.flags |= kP3Pieces;
  a.part_stride = m->NC0 * 16;
  a.part_e = deep_emb;
  a.part_fs = first_second;
  hipError_t e = launch_forward(a, m->D, 1, 1, 8, m->lds_inf, (hipStream_t)stream);
  if (e != hipSuccess) return hip_fail(e, "gather launch");
  return DFWFM_OK;
}

int dfwfm_model_pack_tables(dfwfm_model* m, int32_t enable, int32_t* enabled, void* stream) {
  if (!m || !enabled) return fail(DFWFM_ERR_INVALID_ARG, "null argument");
  *enabled = 0;
  m->pkw = 0;
  if (!enable) return DFWFM_OK;
  if (!m->tables_set) return fail(DFWFM_ERR_STATE, "set_tables must precede pack_tables");
  const int need = kHasSecond | kNeedE | kFoTables;
  if ((m->flags & need) != need || (m->flags & kHasQR) || m->F - m->num < 1) return DFWFM_OK;
  const int D = m->D;
  const int pkw = D + 1 <= 16 ? 16 : (D + 4) & ~3;
  PackTabList L;
  memset(&L, 0, sizeof L);
  L.D = D;
  L.pkw = pkw;
  size_t rows = 0;
  for (int f = m->num; f < m->F; ++f) rows += (size_t)m->h_fields[f].n;
  if (rows * pkw > m->pkrows_floats) {
    if (m->d_pkrows) (void)hipFree(m->d_pkrows);
    m->d_pkrows = nullptr;
    m->pkrows_floats = 0;
    HIP_TRY(hipMalloc(reinterpret_cast<void**>(&m->d_pkrows), rows * pkw * sizeof(float)));
    m->pkrows_floats = rows * pkw;
  }
  if (!m->d_pk) HIP_TRY(hipMalloc(reinterpret_cast<void**>(&m->d_pk), 64 * sizeof(float*)));
  const float* bases[64] = {};
  size_t off = 0;
  for (int f = m->num; f < m->F; ++f) {
    const int j = f - m->num;
    const int64_t n = m->h_fields[f].n;
    bases[f] = m->d_pkrows + off;
    L.emb2[j] = m->h_fields[f].emb2;
    L.emb1[j] = m->h_fields[f].emb1;
    L.dst[j] = m->d_pkrows + off;
    L.n[j] = n;
    const int64_t nb = (n + 255) / 256;
    if ((int64_t)L.blk0[j] + nb > 0x7fffffff) return fail(DFWFM_ERR_UNSUPPORTED, "tables too large to pack");
    L.blk0[j + 1] = L.blk0[j] + (int32_t)nb;
    off += (size_t)n * pkw;
  }
  L.nf = m->F - m->num;
  hipStream_t s = (hipStream_t)stream;
  HIP_TRY(hipMemcpyAsync(m->d_pk, bases, sizeof bases, hipMemcpyHostToDevice, s));
  HIP_TRY(hipStreamSynchronize(s));  // `bases` is a stack buffer (once per weight update)
  hipError_t e = launch_pack_tables(L, s);
  if (e != hipSuccess) return hip_fail(e, "pack tables launch");
  m->pkw = pkw;
  *enabled = 1;
  return DFWFM_OK;
}

int dfwfm_model_build_fwfm_pairs(dfwfm_model* m, int32_t max_pairs, int32_t* enabled, void* stream) {
  if (!m || !enabled) return fail(DFWFM_ERR_INVALID_ARG, "null argument");
  *enabled = 0;
  m->flags &= ~kPairs;
  if (!m->dense_set) return fail(DFWFM_ERR_STATE, "set_dense must precede build_fwfm_pairs");
  if (!(m->flags & kHasSecond) || max_pairs <= 0) return DFWFM_OK;
  hipStream_t s = (hipStream_t)stream;
  // the packed strictly-upper (R + R^T)/2 (FM: ones), as the forward reads it
  std::vector<float> pk((size_t)m->MT * m->S * 64);
  hipError_t e = hipMemcpyAsync(pk.data(), m->d_upack, pk.size() * sizeof(float), hipMemcpyDeviceToHost, s);
  if (e == hipSuccess) e = hipStreamSynchronize(s);
  if (e != hipSuccess) return hip_fail(e, "read FwFM pack");
  std::vector<int2> list;
  for (int k = 0; k < m->F; ++k)
    for (int l = k + 1; l < m->F; ++l) {
      const float w = pk[((size_t)(k >> 4) * m->S + (l >> 2)) * 64 + (k & 15) + 16 * (l & 3)];
      if (w != 0.f) {
        if ((int)list.size() >= max_pairs) return DFWFM_OK;  // denser than the pair path pays for
        int2 q;
        q.x = k | (l << 16);
        memcpy(&q.y, &w, sizeof w);
        list.push_back(q);
      }
    }
  if (!m->d_pairs) {
    const size_t cap = (size_t)m->F * (m->F - 1) / 2 + 1;
    e = hipMalloc(&m->d_pairs, cap * sizeof(int2));
    if (e != hipSuccess) return hip_fail(e, "pair list alloc");
  }
  if (!list.empty()) {
    e = hipMemcpyAsync(m->d_pairs, list.data(), list.size() * sizeof(int2), hipMemcpyHostToDevice, s);
    if (e == hipSuccess) e = hipStreamSynchronize(s);
    if (e != hipSuccess) return hip_fail(e, "pair list upload");
  }
  m->npairs = (int32_t)list.size();
  m->flags |= kPairs;
  *enabled = 1;
  return DFWFM_OK;
}

int dfwfm_model_build_sparse_mlp(dfwfm_model* m, double max_density, int32_t* enabled, void* stream) {
  if (!m || !enabled) return fail(DFWFM_ERR_INVALID_ARG, "null argument");
  *enabled = 0;
  m->sp = 0;
  if (!m->dense_set) return fail(DFWFM_ERR_STATE, "set_dense must precede build_sparse_mlp");
  if (m->H == 0 || max_density <= 0.0) return DFWFM_OK;
  for (int h = 0; h < m->H; ++h)
    if (!m->lin_w[h]) return fail(DFWFM_ERR_STATE, "layer %d weight unknown", h);
  if (sparse_mlp_lds_bytes(m->NC0 * 16, m->N) > 160 * 1024) return DFWFM_OK;  // tile does not fit: dense
  hipStream_t s = (hipStream_t)stream;
  EllArgs a;
  memset(&a, 0, sizeof a);
  int64_t total = 0, dense = 0;
  for (int h = 0; h < m->H; ++h) {
    const int K = h == 0 ? m->F * m->D : m->N;
    a.w[h] = m->lin_w[h];
    a.K[h] = K;
    a.W[h] = (K + kEllPad - 1) / kEllPad * kEllPad;
    a.off[h] = total;
    m->spW[h] = a.W[h];
    m->spoff[h] = total;
    total += (int64_t)((m->N + 3) / 4) * 4 * a.W[h];
    dense += (int64_t)m->N * K;
  }
  if (!m->d_ell) {
    HIP_TRY(hipMalloc(reinterpret_cast<void**>(&m->d_ell), sizeof(int2) * (size_t)total));
    HIP_TRY(hipMalloc(reinterpret_cast<void**>(&m->d_cnt), sizeof(int32_t) * (size_t)m->H * (m->N + (m->N + 3) / 4)));
    HIP_TRY(hipMalloc(reinterpret_cast<void**>(&m->d_spstat), sizeof(int32_t) * 2));
  }
  a.ell = m->d_ell;
  a.cnt = m->d_cnt;
  a.gcnt = m->d_cnt + m->H * m->N;
  a.stat = m->d_spstat;
  a.N = m->N;
  a.H = m->H;
  HIP_TRY(hipMemsetAsync(m->d_spstat, 0, sizeof(int32_t) * 2, s));
  hipError_t e = launch_ell_build(a, m->H * ((m->N + 3) / 4), s);
  if (e != hipSuccess) return hip_fail(e, "ELL build launch");
  int32_t st[2] = {0, 0};
  HIP_TRY(hipMemcpyAsync(st, m->d_spstat, sizeof st, hipMemcpyDeviceToHost, s));
  HIP_TRY(hipStreamSynchronize(s));
  m->sp_density = dense > 0 ? (double)st[1] / (double)dense : 1.0;
  m->sp = m->sp_density <= max_density ? 1 : 0;
  *enabled = m->sp;
  return DFWFM_OK;
}

int dfwfm_train_forward(dfwfm_model* m, const int64_t* xi, int64_t xi_stride, const float* xv, int64_t xv_stride,
                        int64_t batch, float* out, float dropout_p, uint32_t seed, void* stream) {
  if (!m) return fail(DFWFM_ERR_INVALID_ARG, "null model");
  m->trained = false;
  m->t_keys = false;
  m->bwd_tables = false;
  m->bwd_fused_red = false;
  m->bwd_loss_sum = nullptr;
  int rc = check_inputs(m, xi, xi_stride, xv, xv_stride, batch, out);
  if (rc != DFWFM_OK) return rc;
  if (!(dropout_p >= 0.f && dropout_p < 1.f)) return fail(DFWFM_ERR_INVALID_ARG, "dropout_p outside [0, 1)");
  if (m->H > 0 && m->N % 4 != 0)
    return fail(DFWFM_ERR_UNSUPPORTED, "training needs deep_nodes %% 4 == 0 (got %d)", m->N);
  if (m->KS != 1) return fail(DFWFM_ERR_UNSUPPORTED, "training runs with one K half per wave only");
  if (backward_lds_bytes(m->F, m->D, m->MT, m->S, m->SX, m->SY) > 160 * 1024)
    return fail(DFWFM_ERR_UNSUPPORTED, "backward LDS tile exceeds 160 KiB");
  if ((rc = ensure_workspace(m, batch)) != DFWFM_OK) return rc;
  m->t_xi = xi;
  m->t_xs = xi_stride;
  m->t_xv = xv;
  m->t_vs = xv_stride;
  m->t_batch = batch;
  m->t_drop = dropout_p;
  m->t_seed = seed;
  if (batch == 0) {
    m->trained = true;
    return DFWFM_OK;
  }
  FwdArgs a;
  fill_forward_args(m, a, xi, xi_stride, xv, xv_stride, batch, out);
  a.pk = nullptr;  // the training forward reads the tables the optimizer updates, never the serving copy
  a.pkw = 0;
  a.flags |= kTrain | ((m->H > 0 && dropout_p > 0.f) ? kDrop : 0);
  a.sv_e = m->sv_e;
  a.sv_fo = m->sv_fo;
  // without deep-tower dropout X_0 == E: one saved copy
  m->sv_x[0] = m->H > 0 ? ((dropout_p > 0.f) ? m->sv_x0 : m->sv_e) : nullptr;
  for (int h = 0; h <= m->H; ++h) a.sv_x[h] = m->sv_x[h];
  a.drop_p = dropout_p;
  a.drop_scale = 1.f / (1.f - dropout_p);
  a.seed = seed;
  a.seed_src = m->step_src;
  if ((rc = diag_stamps_buffer(m, batch, 1, &a.stamps)) != DFWFM_OK) return rc;
  // the eight-wave layout when the model has it (DFWFM_DIAG ng=4 keeps the four-wave kernel)
  a.tail = m->tailI;
  // the helper-wave form when the model has it (DFWFM_DIAG ftrain=0: fwd_kernel<TRAIN>, bit-identical, tests)
  const int dg = diag_opt("ft", 0);  // diagnostics only (results invalid)
  a.flags |= ((dg & 1) ? kFtDiagHwId : 0) | ((dg & 2) ? kFtDiagNoMlp : 0);
  const bool helpers = m->lds_ftrain > 0 && diag_opt("ftrain", 1) != 0;
  // the helper-wave forward also writes the categorical indices column-major for the sorted scatter
  a.sv_keys = helpers ? m->sv_keys : nullptr;
  a.keys_stride = m->keys_stride;
  m->t_keys = helpers;
  hipError_t e = helpers ? launch_ftrain(a, m->D, m->lds_ftrain, (hipStream_t)stream)
                         : launch_forward(a, m->D, m->TPWI > 0 ? m->TPWI : 1, 1, m->NG, m->lds_inf, (hipStream_t)stream);
  if (e != hipSuccess) return hip_fail(e, "train forward launch");
  m->trained = true;
  return DFWFM_OK;
}

struct BceFuse {
  const float* z;
  const float* y;
  float* loss_sum;
  float denom;
};

static int backward_impl(dfwfm_model* m, const float* dlogit, const dfwfm_grads* g, int phases, void* stream,
                         const BceFuse* bce = nullptr) {
  if (!m || !g) return fail(DFWFM_ERR_INVALID_ARG, "null argument");
  if (phases & ~(DFWFM_BWD_TABLES | DFWFM_BWD_MLP_WEIGHTS | DFWFM_BWD_TILES | DFWFM_BWD_SPREAD | DFWFM_BWD_REDUCE |
                 DFWFM_BWD_SCATTER))
    return fail(DFWFM_ERR_INVALID_ARG, "unknown phase bits");
  // DFWFM_BWD_TABLES = the per-tile backward (TILES) + the reductions (REDUCE) and the table scatter (SCATTER)
  if (phases & DFWFM_BWD_TABLES) phases |= DFWFM_BWD_TILES | DFWFM_BWD_SPREAD;
  if (phases & DFWFM_BWD_SPREAD) phases |= DFWFM_BWD_REDUCE | DFWFM_BWD_SCATTER;
  if (!m->trained) return fail(DFWFM_ERR_STATE, "dfwfm_backward needs a preceding dfwfm_train_forward");
  const int64_t batch = m->t_batch;
  if (batch == 0) return DFWFM_OK;
  if (!dlogit) return fail(DFWFM_ERR_INVALID_ARG, "null dlogit");
  hipStream_t s = (hipStream_t)stream;
  const int F = m->F, D = m->D, num = m->num, H = m->H;
  const bool drop = H > 0 && m->t_drop > 0.f;
  hipError_t e;
  if ((phases & (DFWFM_BWD_REDUCE | DFWFM_BWD_SCATTER)) && !(phases & DFWFM_BWD_TILES) && !m->bwd_tables &&
      (m->flags & kNeedE))
    return fail(DFWFM_ERR_STATE, "DFWFM_BWD_SPREAD needs the per-tile backward (DFWFM_BWD_TILES) first");
  bool fused_red = (phases & DFWFM_BWD_TILES) ? false : m->bwd_fused_red;

  // 1. per-tile backward: dE and the G chain (no atomics)
  if ((phases & DFWFM_BWD_TILES) && (m->flags & kNeedE)) {
    BwdArgs a;
    memset(&a, 0, sizeof a);
    a.batch = batch;
    a.dlogit = dlogit;
    if (bce) {
      a.bce_z = bce->z;
      a.bce_y = bce->y;
      a.bce_dl = const_cast<float*>(dlogit);
      a.loss_sum = bce->loss_sum;
      a.bce_denom = bce->denom;
    }
    a.sv_e = m->sv_e;
    for (int h = 0; h <= H; ++h) {
      a.sv_x[h] = m->sv_x[h];
      a.sv_g[h] = m->sv_g[h];
    }
    a.sv_de = m->sv_de;
    a.rsk = m->d_rsk;
    a.fwlw = m->d_fwlw;
    a.lw = m->d_lw;
    a.fc = m->d_fc;
    a.wtpack = m->d_wtpack;
    a.wtpack_bytes = (int32_t)(m->wtpack_elems * sizeof(float4));
    for (int l = 1; l <= H; ++l) a.wt_off[l] = m->wt_off[l];
    a.F = F;
    a.H = H;
    a.N = m->N;
    a.NT = m->NT;
    a.NC0 = m->NC0;
    a.MT = m->MT;
    a.S = m->S;
    a.SX = m->SX;
    a.SY = m->SY;
    a.W0 = m->W0;
    a.flags = m->flags | (drop ? kDrop : 0);
    // diagnostics only (backward phase costs): DFWFM_DIAG bwd= ORs in kDiagBwd* bits, results invalid
    a.flags |= diag_opt("bwd", 0) << 20;
    a.drop_p = m->t_drop;
    a.drop_scale = 1.f / (1.f - m->t_drop);
    a.seed = m->t_seed;
    a.seed_src = m->step_src;
    // the dense shallow reductions ride along (reduce_kernel's re-read of E / fo / X_H / dE is skipped)
    {
      a.part = m->red_part;
      a.sv_fo = m->sv_fo;
      a.xv = m->t_xv;
      a.xv_stride = m->t_vs;
      a.num = num;
      a.red = kRedOn | ((m->flags & kFoLw) && g->fm_1st ? kRedLw : 0) |
              ((m->flags & kFoFwlw) && g->fwfm_lin ? kRedFwlw : 0) | (m->cfg.use_fwfm && g->field_cov ? kRedR : 0) |
              (H > 0 && g->fc_w ? kRedFc : 0) | kRedNum2 | kRedNum1;
      fused_red = true;
    }
    // diagnostics only: DFWFM_DIAG stamps=2 records the backward's phase clocks instead of the forward's
    int src = diag_stamps_buffer(m, batch, 2, &a.stamps);
    if (src != DFWFM_OK) return src;
    const size_t lds = backward_lds_bytes(F, D, m->MT, m->S, m->SX, m->SY);
    // eight waves (the 8*TPW+1-th tile split by K, like the forward) unless DFWFM_DIAG ng=4
    const int NT = m->NT;
    const bool ng8 = H > 0 && NT <= 32 && diag_opt("ng", 8) != 4;
    const int tpw = ng8 ? (NT % 8 == 1 && NT >= 9 ? NT / 8 : (NT + 7) / 8) : (m->TPW > 0 ? m->TPW : 1);
    e = launch_backward(a, D, tpw > 0 ? tpw : 1, ng8 ? 8 : 4, lds, s);
    if (e != hipSuccess) return hip_fail(e, "backward launch");
    m->bwd_tables = true;
    m->bwd_fused_red = fused_red;
    m->bwd_loss_sum = (fused_red && bce) ? bce->loss_sum : nullptr;
  }

  // 2. dense shallow reductions: per 16-row tile, then summed over tiles.  When this call also runs the
  // weight-gradient GEMM, the final sums ride in its launch (launch_dw_reduce)
  RedArgs r;
  bool red_pending = false;
  if (phases & DFWFM_BWD_REDUCE) {
    memset(&r, 0, sizeof r);
    r.batch = batch;
    r.part = m->red_part;
    r.dlogit = dlogit;
    r.sv_e = m->sv_e;
    r.sv_fo = m->sv_fo;
    r.sv_de = (m->flags & kNeedE) ? m->sv_de : nullptr;
    r.x_h = H > 0 ? m->sv_x[H] : nullptr;
    r.xv = m->t_xv;
    r.xv_stride = m->t_vs;
    r.lw = (m->flags & kFoLw) ? m->d_lw : nullptr;
    r.g_bias = g->bias;
    r.g_lw = (m->flags & kFoLw) ? g->fm_1st : nullptr;
    r.g_fwlw = (m->flags & kFoFwlw) ? g->fwfm_lin : nullptr;
    r.g_R = m->cfg.use_fwfm ? g->field_cov : nullptr;
    r.g_fc = H > 0 ? g->fc_w : nullptr;
    for (int f = 0; f < num && g->fields; ++f) {
      r.g_num2[f] = (m->flags & kNeedE) ? g->fields[f].emb2 : nullptr;
      r.g_num1[f] = (m->flags & kFoTables) ? g->fields[f].emb1 : nullptr;
    }
    r.F = F;
    r.D = D;
    r.num = num;
    r.N = m->N;
    r.MT = m->MT;
    r.flags = m->flags;
    r.loss_sum = fused_red ? m->bwd_loss_sum : nullptr;
    red_pending = fused_red && (phases & DFWFM_BWD_MLP_WEIGHTS) && H > 0 && (g->lin_w || g->lin_b);
    if (!red_pending) {
      e = fused_red ? launch_reduce_final(r, s) : launch_reduce(r, s);
      if (e != hipSuccess) return hip_fail(e, "reduce launch");
    }
  }

  // 3. categorical tables: the atomic scatter (privatised LDS tasks for small tables, global atomics for large ones;
  // sums in arrival order) unless deterministic mode, which runs the sorted per-row-owner scatter (one task per field
  // and row kind, both table families)
  const bool atomic_scatter = !m->deterministic;
  if ((phases & DFWFM_BWD_SCATTER) && g->fields && !atomic_scatter) {
    SortScatterArgs sa;
    memset(&sa, 0, sizeof sa);
    int sblocks = 0;
    sa.D = D;
    sa.F = F;
    sa.num = num;
    sa.fields = m->d_fields;
    sa.xi = m->t_xi;
    sa.xi_stride = m->t_xs;
    sa.batch = batch;
    sa.sv_de = m->sv_de;
    sa.dlogit = dlogit;
    sa.lw = (m->flags & kFoLw) ? m->d_lw : nullptr;
    sa.keys = (m->t_keys && batch <= m->ws_batch) ? m->sv_keys : nullptr;
    sa.keys_stride = m->keys_stride;
    sa.diag = diag_opt("scatter", 0);  // diagnostics only: results invalid
    const bool need2 = (m->flags & kNeedE) != 0, need1 = (m->flags & kFoTables) != 0;
    auto add = [&](float* g2, float* g1, const float* o2, const float* o1, int64_t c, int f, int kind,
                   int64_t rows) -> int {
      if (!need2) g2 = nullptr;
      if (!need1) g1 = nullptr;
      if (!g2 && !g1) return DFWFM_OK;
      if (sa.ntasks == kSortScatterList) {
        hipError_t er = launch_sort_scatter(sa, sblocks, s);
        if (er != hipSuccess) return hip_fail(er, "scatter launch");
        sa.ntasks = 0;
        sa.key64 = 0;
        sblocks = 0;
      }
      SortScatterTask& t = sa.t[sa.ntasks++];
      // row buckets, one workgroup each: tables of at most 64 rows one row per bucket (no sort; a few hundred samples
      // each), larger ones eight buckets of ~B/8 samples (~540 keys at B = 4096: one 55-stage network over 1024
      // threads; 12 / 16 buckets measured slower, more workgroups than CUs)
      t.onerow = rows <= 64 ? 1 : 0;
      t.nbuck = (int16_t)(rows <= 64 ? (rows > 0 ? rows : 1) : 8);
      t.block0 = sblocks;
      t.pad8 = 0;
      sblocks += t.nbuck;
      if ((rows + t.nbuck - 1) / t.nbuck >= kSortKey32Rows) sa.key64 = 1;
      t.g2 = g2;
      t.g1 = g1;
      t.o2 = need2 ? o2 : nullptr;
      t.o1 = need1 ? o1 : nullptr;
      t.c = (int32_t)c;
      t.field = (int16_t)f;
      t.kind = (int8_t)kind;
      return DFWFM_OK;
    };
    int rc = DFWFM_OK;
    for (int f = num; f < F && rc == DFWFM_OK; ++f) {
      const FieldDev& fd = m->h_fields[f];
      const dfwfm_field_grads& fg = g->fields[f];
      if (fd.n > 0x7fffffffLL) return fail(DFWFM_ERR_UNSUPPORTED, "field %d: table of more than 2^31 rows", f);
      if (fd.c == 0) {
        rc = add(fg.emb2, fg.emb1, nullptr, nullptr, 0, f, 0, fd.n);
      } else {
        if (fd.c > 0x7fffffff) return fail(DFWFM_ERR_UNSUPPORTED, "field %d: QR collisions too large", f);
        const bool mult = fd.op == 0;
        rc = add(fg.emb2, fg.emb1, mult ? fd.emb2_r : nullptr, mult ? fd.emb1_r : nullptr, fd.c, f, 1,
                 (fd.n + fd.c - 1) / fd.c);
        if (rc == DFWFM_OK)
          rc = add(fg.emb2_r, fg.emb1_r, mult ? fd.emb2 : nullptr, mult ? fd.emb1 : nullptr, fd.c, f, 2, fd.c);
      }
    }
    if (rc != DFWFM_OK) return rc;
    // diagnostics only: DFWFM_DIAG stamps=3 records this (last) launch's phase clocks per workgroup
    if ((rc = diag_stamps_buffer(m, (int64_t)sblocks * kBM, 3, &sa.stamps)) != DFWFM_OK) return rc;
    e = launch_sort_scatter(sa, sblocks, s);
    if (e != hipSuccess) return hip_fail(e, "scatter launch");
  }
  if ((phases & DFWFM_BWD_SCATTER) && g->fields && atomic_scatter) {
    // privatised tasks (small tables: per-chunk LDS sums, one flush per touched row) and global-atomic tasks (large
    // tables), one launch for both kinds: the privatised tasks first in the grid
    ScatterArgs L;
    memset(&L, 0, sizeof L);
    L.D = D;
    L.F = F;
    L.num = num;
    L.fields = m->d_fields;
    L.xi = m->t_xi;
    L.xi_stride = m->t_xs;
    L.batch = batch;
    L.sv_de = m->sv_de;
    L.dlogit = dlogit;
    L.lw = (m->flags & kFoLw) ? m->d_lw : nullptr;
    // samples per workgroup: 128 measured best in the mixed launch (17.2 us against 18.2 at 256 and 18.8 at 64 at
    // Criteo-39, B = 4096, profiles/r05/sc_*): more workgroups spread the atomics, fewer flush the private rows less
    L.chunk = 128;
    const int64_t nb = (batch + L.chunk - 1) / L.chunk;
    ScatterTask pt[kScatterList], at[kScatterList];
    int np = 0, na = 0;
    auto flush = [&]() -> int {
      L.ntasks = 0;
      int64_t blocks = 0;
      for (int i = 0; i < np; ++i, blocks += nb) {
        L.t[L.ntasks] = pt[i];
        L.t[L.ntasks++].block0 = (int32_t)blocks;
      }
      for (int i = 0; i < na; ++i, blocks += nb) {
        L.t[L.ntasks] = at[i];
        L.t[L.ntasks++].block0 = (int32_t)blocks;
      }
      np = na = 0;
      if (L.ntasks == 0) return DFWFM_OK;
      if (blocks > 0x7fffffff) return fail(DFWFM_ERR_UNSUPPORTED, "scatter grid too large");
      hipError_t er = launch_scatter(L, (int)blocks, s);
      return er == hipSuccess ? DFWFM_OK : hip_fail(er, "scatter launch");
    };
    auto add = [&](float* gt, const float* other, int64_t c, int f, int kind, int src, int64_t rows) -> int {
      if (!gt || rows <= 0) return DFWFM_OK;
      if (rows > 0x7fffffff) return fail(DFWFM_ERR_UNSUPPORTED, "field %d: table of more than 2^31 rows", f);
      const int w = src == 0 ? D : 1;
      // tables up to kPrivRows rows (and kPrivFloats of LDS) accumulate privately; bigger ones spread
      // their atomics well enough (64 / 512 / 2000 rows measured slower)
      const bool is_priv = rows * (w + 1) <= kPrivFloats && rows <= kPrivRows;
      if (np + na == kScatterList || (int64_t)(np + na + 1) * nb > 0x7fffffff) {
        int rc = flush();
        if (rc != DFWFM_OK) return rc;
      }
      ScatterTask& t = is_priv ? pt[np++] : at[na++];
      t.g = gt;
      t.other = other;
      t.c = (int32_t)c;
      t.field = (int16_t)f;
      t.kind = (int8_t)(kind | (is_priv ? kScatterPriv : 0));
      t.src = (int8_t)src;
      t.rows = (int32_t)(rows < 0x7fffffff ? rows : 0x7fffffff);
      t.block0 = 0;
      return DFWFM_OK;
    };
    int rc = DFWFM_OK;
    for (int f = num; f < F && rc == DFWFM_OK; ++f) {
      const FieldDev& fd = m->h_fields[f];
      const dfwfm_field_grads& fg = g->fields[f];
      if (fd.c > 0 && fd.c > 0x7fffffff) return fail(DFWFM_ERR_UNSUPPORTED, "field %d: QR collisions too large", f);
      for (int src = 0; src < 2 && rc == DFWFM_OK; ++src) {
        if (src == 0 && !(m->flags & kNeedE)) continue;
        if (src == 1 && !(m->flags & kFoTables)) continue;
        float* gq = src == 0 ? fg.emb2 : fg.emb1;
        float* gr = src == 0 ? fg.emb2_r : fg.emb1_r;
        if (fd.c == 0) {
          rc = add(gq, nullptr, 0, f, 0, src, fd.n);
        } else {
          const bool mult = fd.op == 0;
          const float* tq = src == 0 ? fd.emb2 : fd.emb1;
          const float* tr = src == 0 ? fd.emb2_r : fd.emb1_r;
          // quotient rows: ceil(n / c) (weight_q's rows; an index past the last full group lands in the last row)
          rc = add(gq, mult ? tr : nullptr, fd.c, f, 1, src, (fd.n + fd.c - 1) / fd.c);
          if (rc == DFWFM_OK) rc = add(gr, mult ? tq : nullptr, fd.c, f, 2, src, fd.c);
        }
      }
    }
    if (rc == DFWFM_OK) rc = flush();
    if (rc != DFWFM_OK) return rc;
  }

  // 4. dW_l += G_l^T X_{l-1}, db_l += sum_b G_l
  if ((phases & DFWFM_BWD_MLP_WEIGHTS) && H > 0 && (g->lin_w || g->lin_b)) {
    DwArgs d;
    memset(&d, 0, sizeof d);
    d.H = H;
    d.N = m->N;
    const int edge = kDwEdge;
    d.nnb = (m->N + edge - 1) / edge;
    d.batch = batch;
    int per_split = 0;
    for (int l = 1; l <= H; ++l) {
      d.G[l] = m->sv_g[l];
      d.X[l] = m->sv_x[l - 1];
      d.gW[l] = g->lin_w ? g->lin_w[l - 1] : nullptr;
      d.gB[l] = g->lin_b ? g->lin_b[l - 1] : nullptr;
      d.K[l] = l == 1 ? F * D : m->N;
      d.ldx[l] = l == 1 ? r4(F * D) : m->N;
      d.nkb[l] = d.gW[l] ? (d.K[l] + edge - 1) / edge : (d.gB[l] ? 1 : 0);
      per_split += d.nnb * d.nkb[l];
    }
    if (per_split > 0) {
      // the split plan the workspace was sized for (over every layer's K blocks: per_split <= plan_blocks)
      int plan_blocks = 0;
      int64_t splits = 0, rows = 0;
      int rc = dw_plan(m, batch, &plan_blocks, &splits, &rows);
      if (rc != DFWFM_OK) return rc;
      // the slices are used only by the deterministic split-K sum; the float-atomic form never reads them
      if (m->deterministic && splits > 1 && (int64_t)per_split * splits > m->dw_slices)
        return fail(DFWFM_ERR_STATE, "weight-gradient split slices: %lld needed, %lld allocated", (long long)per_split * splits, (long long)m->dw_slices);
      d.splits = (int32_t)splits;
      d.rows_per_split = rows;
      d.part = m->deterministic ? m->dw_part : nullptr;  // split slices (deterministic) or float atomics
      d.bpart = m->deterministic ? m->dw_bpart : nullptr;
      d.blk0[1] = 0;
      for (int l = 1; l <= H; ++l) d.blk0[l + 1] = d.blk0[l] + d.nnb * d.nkb[l] * (int32_t)splits;
      e = red_pending ? launch_dw_reduce(d, d.blk0[H + 1], r, s) : launch_dw(d, d.blk0[H + 1], s);
      if (e != hipSuccess) return hip_fail(e, "dw launch");
      red_pending = false;
    }
  }
  if (red_pending) {
    e = launch_reduce_final(r, s);
    if (e != hipSuccess) return hip_fail(e, "reduce launch");
  }
  return DFWFM_OK;
}

int dfwfm_set_deterministic(dfwfm_model* m, int32_t on) {
  if (!m) return fail(DFWFM_ERR_INVALID_ARG, "null model");
  m->deterministic = on != 0;
  return DFWFM_OK;
}

int dfwfm_backward(dfwfm_model* m, const float* dlogit, const dfwfm_grads* g, void* stream) {
  return backward_impl(m, dlogit, g, DFWFM_BWD_TABLES | DFWFM_BWD_MLP_WEIGHTS, stream);
}

int dfwfm_backward_phases(dfwfm_model* m, const float* dlogit, const dfwfm_grads* g, int32_t phases, void* stream) {
  return backward_impl(m, dlogit, g, phases, stream);
}

int dfwfm_backward_phases_bce(dfwfm_model* m, const float* z, const float* y, double denom, float* dlogit,
                              float* loss_sum, const dfwfm_grads* g, int32_t phases, void* stream) {
  if (!m || !g) return fail(DFWFM_ERR_INVALID_ARG, "null argument");
  if (!(denom > 0.0)) return fail(DFWFM_ERR_INVALID_ARG, "denom must be > 0");
  if (!m->trained) return fail(DFWFM_ERR_STATE, "dfwfm_backward needs a preceding dfwfm_train_forward");
  const int64_t n = m->t_batch;
  if (n > 0 && (!z || !y || !dlogit)) return fail(DFWFM_ERR_INVALID_ARG, "null argument");
  const bool tiles = (phases & (DFWFM_BWD_TABLES | DFWFM_BWD_TILES)) != 0;
  if (!tiles || !(m->flags & kNeedE) || n == 0) {
    // no per-tile backward to carry it: the separate gradient launch
    hipError_t e = launch_bce_grad(z, y, n, (float)denom, dlogit, loss_sum, (hipStream_t)stream);
    if (e != hipSuccess) return hip_fail(e, "bce launch");
    return backward_impl(m, dlogit, g, phases, stream);
  }
  const BceFuse b{z, y, loss_sum, (float)denom};
  return backward_impl(m, dlogit, g, phases, stream, &b);
}

int dfwfm_adam_step(const dfwfm_adam_tensor* t, int32_t n, double lr, double beta1, double beta2, double eps,
                    double weight_decay, int64_t step, void* stream) {
  if (n > 0 && !t) return fail(DFWFM_ERR_INVALID_ARG, "null tensor list");
  if (n < 0) return fail(DFWFM_ERR_INVALID_ARG, "negative tensor count");
  if (step < 1) return fail(DFWFM_ERR_INVALID_ARG, "step must be >= 1");
  for (int i = 0; i < n; ++i)
    if (t[i].grad && t[i].numel > 0 && (!t[i].param || !t[i].exp_avg || !t[i].exp_avg_sq))
      return fail(DFWFM_ERR_INVALID_ARG, "adam tensor %d: null state pointer", i);
  // torch.optim.Adam: bias corrections and step size in double (Python floats), rounded to f32 per use
  const double bc1 = 1.0 - pow(beta1, (double)step);
  const double bc2 = 1.0 - pow(beta2, (double)step);
  const float step_size = (float)(lr / bc1), omb1 = (float)(1.0 - beta1), b2 = (float)beta2,
              omb2 = (float)(1.0 - beta2), epsf = (float)eps, wd = (float)weight_decay, bc2s = (float)sqrt(bc2);
  AdamList list;
  memset(&list, 0, sizeof list);
  int64_t blocks = 0;
  auto flush = [&]() -> int {
    if (list.n == 0) return DFWFM_OK;
    hipError_t e = launch_adam(list, (int)blocks, step_size, omb1, b2, omb2, epsf, wd, bc2s, (hipStream_t)stream);
    list.n = 0;
    blocks = 0;
    return e == hipSuccess ? DFWFM_OK : hip_fail(e, "adam launch");
  };
  for (int i = 0; i < n; ++i) {
    if (!t[i].grad || t[i].numel <= 0) continue;  // torch skips parameters without a grad
    const int64_t nb = (t[i].numel + kAdamBlock - 1) / kAdamBlock;
    if (nb > 0x7fffffff) return fail(DFWFM_ERR_UNSUPPORTED, "adam tensor %d too large", i);
    if (list.n == kAdamList || blocks + nb > 0x7fffffff) {
      int rc = flush();
      if (rc != DFWFM_OK) return rc;
    }
    AdamTensor& a = list.t[list.n];
    a.p = t[i].param;
    a.g = t[i].grad;
    a.m = t[i].exp_avg;
    a.v = t[i].exp_avg_sq;
    a.n = t[i].numel;
    list.block0[list.n++] = (int32_t)blocks;
    blocks += nb;
  }
  return flush();
}

}  // extern "C"

namespace {

// the sparse-gradient tasks of one table family: per categorical field its plain / quotient table, then its
// remainder table (QR); dest == NULL lists every table (capacity), else only those with an offset >= 0
int sparse_tasks(const dfwfm_model* m, int family, const dfwfm_sparse_dest* dest, SparseArgs* a) {
  int n = 0;
  const bool has = family == DFWFM_FAMILY_SECOND ? (m->flags & kNeedE) != 0 : (m->flags & kFoTables) != 0;
  if (!has) return 0;
  for (int f = m->num; f < m->F; ++f) {
    const FieldDev& fd = m->h_fields[f];
    for (int part = 0; part < (fd.c > 0 ? 2 : 1); ++part) {
      const int64_t off = dest ? (part == 0 ? dest[f].q : dest[f].r) : 0;
      if (off < 0) continue;
      if (a) {
        SparseTask& t = a->t[n];
        t.dest = off;
        t.field = (int16_t)f;
        t.c = (int32_t)fd.c;
        t.kind = (int8_t)(fd.c == 0 ? 0 : 1 + part);
      }
      ++n;
    }
  }
  return n;
}

// largest entry count of one family's touched-row list: a table contributes at most one entry per distinct row,
// so min(batch, its rows) -- plain tables n_f rows, QR quotient tables n_f / c (n_f rounded up to a multiple of
// c at set_tables), remainder tables c -- instead of batch per table (Criteo-39, B = 4096: 14 of 26 tables have
// fewer rows than the batch)
int64_t sparse_capacity(const dfwfm_model* m, int family, const dfwfm_sparse_dest* dest, int64_t batch) {
  const bool has = family == DFWFM_FAMILY_SECOND ? (m->flags & kNeedE) != 0 : (m->flags & kFoTables) != 0;
  if (!has) return 0;
  int64_t cap = 0;
  for (int f = m->num; f < m->F; ++f) {
    const FieldDev& fd = m->h_fields[f];
    for (int part = 0; part < (fd.c > 0 ? 2 : 1); ++part) {
      if (dest && (part == 0 ? dest[f].q : dest[f].r) < 0) continue;
      const int64_t rows = fd.c == 0 ? fd.n : (part == 0 ? fd.n / fd.c : (int64_t)fd.c);
      cap += rows < batch ? rows : batch;
    }
  }
  return cap;
}

}  // namespace

extern "C" {

int dfwfm_sparse_grads_size(dfwfm_model* m, int32_t family, int64_t batch, int64_t* capacity, int32_t* width,
                            int64_t* ws_bytes) {
  if (!m || !capacity || !width || !ws_bytes || batch < 0) return fail(DFWFM_ERR_INVALID_ARG, "null argument");
  if (family != DFWFM_FAMILY_SECOND && family != DFWFM_FAMILY_FIRST) return fail(DFWFM_ERR_INVALID_ARG, "bad family");
  if (!m->tables_set) return fail(DFWFM_ERR_STATE, "set_tables must precede dfwfm_sparse_grads_size");
  const int nt = sparse_tasks(m, family, nullptr, nullptr);
  *width = family == DFWFM_FAMILY_SECOND ? m->D : 1;
  if ((int64_t)nt * batch > 0x7fffffff) return fail(DFWFM_ERR_UNSUPPORTED, "more than 2^31 (table, sample) pairs");
  *capacity = sparse_capacity(m, family, nullptr, batch);
  *ws_bytes = 0;  // dfwfm_sparse_grads_local needs no workspace (kept in the signature: ABI version 2)
  return DFWFM_OK;
}

int dfwfm_sparse_grads_local(dfwfm_model* m, int32_t family, const dfwfm_sparse_dest* dest, int64_t capacity,
                             float* local, int32_t* stamp, int64_t local_floats, int64_t* out_dest, float* out_rows,
                             int32_t* out_count, void* stream) {
  if (!m || !dest || !out_count || !local || !stamp) return fail(DFWFM_ERR_INVALID_ARG, "null argument");
  if (family != DFWFM_FAMILY_SECOND && family != DFWFM_FAMILY_FIRST) return fail(DFWFM_ERR_INVALID_ARG, "bad family");
  if (!m->trained) return fail(DFWFM_ERR_STATE, "dfwfm_sparse_grads_local needs a preceding dfwfm_train_forward");
  SparseArgs a;
  memset(&a, 0, sizeof a);
  a.ntasks = sparse_tasks(m, family, dest, &a);
  a.D = m->D;
  a.F = m->F;
  a.num = m->num;
  a.w = family == DFWFM_FAMILY_SECOND ? m->D : 1;
  a.fields = m->d_fields;
  a.xi = m->t_xi;
  a.xi_stride = m->t_xs;
  a.batch = m->t_batch;
  const int64_t bound = sparse_capacity(m, family, dest, a.batch);
  if (bound > capacity)
    return fail(DFWFM_ERR_INVALID_ARG, "capacity %lld < %lld entries", (long long)capacity, (long long)bound);
  if (bound > 0 && (!out_dest || !out_rows)) return fail(DFWFM_ERR_INVALID_ARG, "null buffer");
  // every row a task can touch must lie inside the caller's local buffer (and its stamp array, as long)
  for (int k = 0; k < a.ntasks; ++k) {
    const SparseTask& T = a.t[k];
    const FieldDev& fd = m->h_fields[T.field];
    const int64_t rows = T.kind == 0 ? fd.n : (T.kind == 1 ? fd.n / fd.c : (int64_t)fd.c);
    if (T.dest < 0 || T.dest + rows * a.w > local_floats)
      return fail(DFWFM_ERR_INVALID_ARG, "table of field %d outside the local buffer", (int)T.field);
  }
  hipError_t e = launch_sparse_local(a, local, stamp, capacity, out_dest, out_rows, out_count, (hipStream_t)stream);
  return e == hipSuccess ? DFWFM_OK : hip_fail(e, "sparse grads (local)");
}

int dfwfm_sparse_grads_apply(float* grad, int32_t width, const int64_t* dest, const float* rows, const int32_t* count,
                             int64_t capacity, void* stream) {
  if (capacity < 0 || width < 1) return fail(DFWFM_ERR_INVALID_ARG, "bad size");
  if (capacity > 0 && (!grad || !dest || !rows || !count)) return fail(DFWFM_ERR_INVALID_ARG, "null argument");
  hipError_t e = launch_sparse_apply(grad, width, dest, rows, count, capacity, (hipStream_t)stream);
  return e == hipSuccess ? DFWFM_OK : hip_fail(e, "sparse apply");
}

int dfwfm_workspace_generation(const dfwfm_model* m, int64_t* gen) {
  if (!m || !gen) return fail(DFWFM_ERR_INVALID_ARG, "null argument");
  *gen = m->ws_gen;
  return DFWFM_OK;
}

int dfwfm_set_step_source(dfwfm_model* m, const int64_t* step_dev) {
  if (!m) return fail(DFWFM_ERR_INVALID_ARG, "null model");
  m->step_src = step_dev;
  return DFWFM_OK;
}

int dfwfm_adam_step_dev(const dfwfm_adam_tensor* t, int32_t n, double lr, double beta1, double beta2, double eps,
                        double weight_decay, void* state_dev, void* stream) {
  if ((n > 0 && !t) || !state_dev) return fail(DFWFM_ERR_INVALID_ARG, "null argument");
  if (n < 0) return fail(DFWFM_ERR_INVALID_ARG, "negative tensor count");
  static_assert(sizeof(AdamDevState) == DFWFM_ADAM_STATE_BYTES, "state block size");
  for (int i = 0; i < n; ++i)
    if (t[i].grad && t[i].numel > 0 && (!t[i].param || !t[i].exp_avg || !t[i].exp_avg_sq))
      return fail(DFWFM_ERR_INVALID_ARG, "adam tensor %d: null state pointer", i);
  AdamDevState* st = reinterpret_cast<AdamDevState*>(state_dev);
  const AdamHyper h{lr, beta1, beta2, eps, weight_decay};
  // the tensors' launches (<= kAdamList tensors each); the last one advances the device step counter (a list
  // without tensors still advances it: one empty workgroup)
  std::vector<int> keep;
  for (int i = 0; i < n; ++i)
    if (t[i].grad && t[i].numel > 0) keep.push_back(i);
  AdamList list;
  memset(&list, 0, sizeof list);
  int64_t blocks = 0;
  for (size_t k = 0; k <= keep.size(); ++k) {
    const bool last = k == keep.size();
    const int64_t nb = last ? 0 : (t[keep[k]].numel + kAdamBlock - 1) / kAdamBlock;
    if (nb > 0x7fffffff) return fail(DFWFM_ERR_UNSUPPORTED, "adam tensor %d too large", keep[k]);
    if (list.n > 0 && (last || list.n == kAdamList || blocks + nb > 0x7fffffff)) {
      hipError_t e = launch_adam_dev(list, (int)blocks, st, h, last, (hipStream_t)stream);
      if (e != hipSuccess) return hip_fail(e, "adam launch");
      list.n = 0;
      blocks = 0;
    }
    if (last) break;
    const dfwfm_adam_tensor& x = t[keep[k]];
    AdamTensor& a = list.t[list.n];
    a.p = x.param;
    a.g = x.grad;
    a.m = x.exp_avg;
    a.v = x.exp_avg_sq;
    a.n = x.numel;
    list.block0[list.n++] = (int32_t)blocks;
    blocks += nb;
  }
  if (keep.empty()) {
    hipError_t e = launch_adam_dev(list, 1, st, h, true, (hipStream_t)stream);
    if (e != hipSuccess) return hip_fail(e, "adam launch");
  }
  return DFWFM_OK;
}

int dfwfm_bce_grad(const float* z, const float* y, int64_t n, double denom, float* dz, float* loss_sum,
                   void* stream) {
  if (n < 0) return fail(DFWFM_ERR_INVALID_ARG, "negative count");
  if (n > 0 && (!z || !y || !dz)) return fail(DFWFM_ERR_INVALID_ARG, "null argument");
  if (!(denom > 0.0)) return fail(DFWFM_ERR_INVALID_ARG, "denom must be > 0");
  hipError_t e = launch_bce_grad(z, y, n, (float)denom, dz, loss_sum, (hipStream_t)stream);
  return e == hipSuccess ? DFWFM_OK : hip_fail(e, "bce launch");
}

int64_t dfwfm_prune_workspace_bytes(int64_t numel) {
  if (numel <= 0 || numel > 0x7fffffff) return 0;
  return (int64_t)prune_workspace_bytes(numel);
}

int dfwfm_prune_threshold(const dfwfm_prune_source* src, int32_t n, double target, double* thr_dev, void* ws,
                          int64_t ws_bytes, void* stream) {
  if (!src || n <= 0 || !thr_dev || !ws) return fail(DFWFM_ERR_INVALID_ARG, "null argument");
  if (n > kMaxPruneSrc) return fail(DFWFM_ERR_UNSUPPORTED, "more than %d pruning sources", kMaxPruneSrc);
  PruneList L;
  memset(&L, 0, sizeof L);
  int64_t off = 0;
  for (int i = 0; i < n; ++i) {
    if (!src[i].values || src[i].numel <= 0) return fail(DFWFM_ERR_INVALID_ARG, "source %d is empty", i);
    if (src[i].sym_f < 0 || src[i].sym_f > 64 || (src[i].sym_f > 0 && (int64_t)src[i].sym_f * src[i].sym_f != src[i].numel))
      return fail(DFWFM_ERR_INVALID_ARG, "source %d: sym_f %d does not match numel", i, src[i].sym_f);
    L.s[i].p = src[i].values;
    L.s[i].numel = src[i].numel;
    L.s[i].offset = off;
    L.s[i].sym_f = src[i].sym_f;
    off += src[i].numel;
  }
  L.n = n;
  if (off > 0x7fffffff) return fail(DFWFM_ERR_UNSUPPORTED, "more than 2^31 magnitudes");
  if (ws_bytes < (int64_t)prune_workspace_bytes(off))
    return fail(DFWFM_ERR_INVALID_ARG, "workspace of %lld bytes < %lld", (long long)ws_bytes,
                (long long)prune_workspace_bytes(off));
  hipError_t e = launch_prune_threshold(L, target, thr_dev, ws, (size_t)ws_bytes, (hipStream_t)stream);
  return e == hipSuccess ? DFWFM_OK : hip_fail(e, "prune threshold");
}

int dfwfm_prune_apply(float* values, int64_t numel, int32_t sym_f, const double* thr_dev, void* stream) {
  if (!values || !thr_dev || numel < 0) return fail(DFWFM_ERR_INVALID_ARG, "null argument");
  if (sym_f < 0 || sym_f > 64 || (sym_f > 0 && (int64_t)sym_f * sym_f != numel))
    return fail(DFWFM_ERR_INVALID_ARG, "sym_f %d does not match numel", sym_f);
  hipError_t e = launch_prune_apply(values, numel, sym_f, thr_dev, (hipStream_t)stream);
  return e == hipSuccess ? DFWFM_OK : hip_fail(e, "prune apply");
}

int64_t dfwfm_metrics_workspace_bytes(int64_t n) {
  if (n <= 0 || n > 0x7fffffff) return 0;
  return (int64_t)metrics_workspace_bytes(n);
}

int dfwfm_eval_metrics(const float* z, const float* y, int64_t n, double* out, void* ws, int64_t ws_bytes,
                       void* stream) {
  if (!z || !y || !out || !ws) return fail(DFWFM_ERR_INVALID_ARG, "null argument");
  if (n <= 0 || n > 0x7fffffff) return fail(DFWFM_ERR_UNSUPPORTED, "n = %lld outside [1, 2^31)", (long long)n);
  if (ws_bytes < (int64_t)metrics_workspace_bytes(n))
    return fail(DFWFM_ERR_INVALID_ARG, "workspace of %lld bytes < %lld", (long long)ws_bytes,
                (long long)metrics_workspace_bytes(n));
  hipError_t e = launch_metrics(z, y, n, out, ws, (size_t)ws_bytes, (hipStream_t)stream);
  return e == hipSuccess ? DFWFM_OK : hip_fail(e, "eval metrics");
}

int dfwfm_diag_stamps(dfwfm_model* m, uint64_t* host, int64_t n, void* stream) {
  if (!m || !host || n < 0) return fail(DFWFM_ERR_INVALID_ARG, "null argument");
  if (!m->d_stamps) return fail(DFWFM_ERR_STATE, "no stamps recorded (set DFWFM_DIAG=stamps=1)");
  const size_t cap = m->stamps_cap * kStampSlots * (m->stamps_ring ? m->stamps_ring : 1);
  const size_t cnt = (size_t)n < cap ? (size_t)n : cap;
  HIP_TRY(hipMemcpyAsync(host, m->d_stamps, cnt * sizeof(uint64_t), hipMemcpyDeviceToHost, (hipStream_t)stream));
  HIP_TRY(hipStreamSynchronize((hipStream_t)stream));
  return (int)(cnt / kStampSlots);
}

int dfwfm_read_error_flag(dfwfm_model* m, int32_t* flag, void* stream) {
  if (!m || !flag) return fail(DFWFM_ERR_INVALID_ARG, "null argument");
  hipStream_t s = (hipStream_t)stream;
  int32_t v = 0;
  HIP_TRY(hipMemcpyAsync(&v, m->d_err, sizeof v, hipMemcpyDeviceToHost, s));
  HIP_TRY(hipStreamSynchronize(s));
  if (v) HIP_TRY(hipMemsetAsync(m->d_err, 0, sizeof(int32_t), s));
  *flag = v;
  return DFWFM_OK;
}

}  // extern "C"
