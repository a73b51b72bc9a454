// dfwfm_capi.hip -- the extern "C" boundary (include/dfwfm.h) over the kernels.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <string>

#include "dfwfm_internal.h"

using namespace dfwfm;

struct dfwfm_model {
  dfwfm_config cfg;
  int device;
  int F, D, num, H, N;
  int NT, NC0, SX, SY, TPW, MT, S, W0, KS;
  int flags;
  size_t lds_bytes;
  // device state (owned)
  FieldDev* d_fields;
  float* d_upack;  // FwFM A-operand fragments [MT][S][64]
  int32_t* d_err;
  float4* d_wpack;
  size_t wpack_elems;
  float* d_mlp_b;  // [H][NT*16]
  float* d_fc;     // [NT*16]
  float* d_fwlw;   // [F*D]
  float* d_lw;     // [F]
  float* d_bias;   // [1]
  uint64_t* d_stamps;  // diagnostics (DFWFM_DIAG_STAMPS)
  size_t stamps_cap;   // workgroups the stamp buffer holds
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
  void* ptrs[] = {m->d_fields, m->d_upack, m->d_err, m->d_wpack, m->d_mlp_b,
                  m->d_fc,     m->d_fwlw,  m->d_lw,  m->d_bias,  m->d_stamps};
  for (void* p : ptrs)
    if (p) (void)hipFree(p);
  delete m;
}

}  // namespace

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
  // E-tile columns read by the MLP (NC0*16) and by the FwFM contraction (4*S fields)
  m->W0 = m->NC0 * 16 > 4 * m->S * D ? m->NC0 * 16 : 4 * m->S * D;
  const int kx = m->W0 > NT * 16 ? m->W0 : NT * 16;
  m->SX = r4(kx) + 4;
  m->SY = c.use_deep ? NT * 16 + 4 : 0;
  // one wave per SIMD; DFWFM_KSPLIT=2 runs two per SIMD splitting K (measured slower, kept for A/B)
  m->KS = 1;
  if (const char* ks = getenv("DFWFM_KSPLIT")) m->KS = atoi(ks) == 2 ? 2 : 1;
  const bool second = c.use_fwfm || c.use_fm;
  m->flags = (second ? kHasSecond : 0) | (c.use_deep ? kHasDeep : 0) |
             (c.use_fwlw ? kFoFwlw : kFoTables) | ((second && c.use_lw) ? kFoLw : 0) |
             ((second || c.use_deep) ? kNeedE : 0);
  const LdsLayout L = lds_layout(F, D, m->MT, m->S, m->SX, m->SY, TPW > 0 ? TPW : 1, m->KS, c.use_deep != 0);
  m->lds_bytes = sizeof(float) * (size_t)L.total;
  if (m->lds_bytes > 160 * 1024) {
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
  if (c.use_deep) {
    m->wpack_elems = (size_t)NT * m->NC0 * 64 + (size_t)(H - 1) * NT * NT * 64;
    if (m->wpack_elems * sizeof(float4) >= (size_t)1 << 31) {
      free_model(m);
      return fail(DFWFM_ERR_UNSUPPORTED, "packed MLP weights exceed the 2 GiB buffer-descriptor range");
    }
    if ((rc = dev_alloc(&m->d_wpack, m->wpack_elems)) ||
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
  HIP_TRY(hipMemcpyAsync(m->d_fields, host, sizeof(FieldDev) * n, hipMemcpyHostToDevice, (hipStream_t)stream));
  HIP_TRY(hipStreamSynchronize((hipStream_t)stream));  // `host` is a stack buffer
  m->tables_set = true;
  return DFWFM_OK;
}

int dfwfm_model_set_dense(dfwfm_model* m, const float* field_cov, const float* fwfm_lin, const float* fm_1st,
                          const float* bias, const float* const* lin_w, const float* const* lin_b,
                          const float* fc_w, void* stream) {
  if (!m) return fail(DFWFM_ERR_INVALID_ARG, "null model");
  hipStream_t s = (hipStream_t)stream;
  const dfwfm_config& c = m->cfg;
  if (c.use_fwfm && !field_cov) return fail(DFWFM_ERR_INVALID_ARG, "use_fwfm needs field_cov");
  if ((m->flags & kFoFwlw) && !fwfm_lin) return fail(DFWFM_ERR_INVALID_ARG, "use_fwlw needs fwfm_linear");
  if ((m->flags & kFoLw) && !fm_1st) return fail(DFWFM_ERR_INVALID_ARG, "use_lw needs fm_1st");
  if (!bias) return fail(DFWFM_ERR_INVALID_ARG, "bias is required");
  if (c.use_fwfm || c.use_fm) {
    hipError_t e = launch_pack_fwfm(field_cov, m->F, c.use_fm ? 1 : 0, m->MT, m->S, m->d_upack, s);
    if (e != hipSuccess) return hip_fail(e, "pack_fwfm");
  }
  hipError_t e = hipSuccess;
  if (m->flags & kFoFwlw) e = launch_pad_copy(fwfm_lin, m->F * m->D, m->F * m->D, m->d_fwlw, s);
  if (e == hipSuccess && (m->flags & kFoLw)) e = launch_pad_copy(fm_1st, m->F, m->F, m->d_lw, s);
  if (e == hipSuccess) e = launch_pad_copy(bias, 1, 1, m->d_bias, s);
  if (e != hipSuccess) return hip_fail(e, "pad_copy");
  if (c.use_deep) {
    if (!lin_w || !lin_b || !fc_w) return fail(DFWFM_ERR_INVALID_ARG, "use_deep needs MLP weights");
    float4* dst = m->d_wpack;
    for (int h = 0; h < m->H; ++h) {
      if (!lin_w[h] || !lin_b[h]) return fail(DFWFM_ERR_INVALID_ARG, "layer %d weight/bias is null", h);
      const int K = h == 0 ? m->F * m->D : m->N;
      const int NC = h == 0 ? m->NC0 : m->NT;
      e = launch_pack_linear(lin_w[h], m->N, K, m->NT, NC, dst, s);
      if (e == hipSuccess) e = launch_pad_copy(lin_b[h], m->N, m->NT * 16, m->d_mlp_b + (size_t)h * m->NT * 16, s);
      if (e != hipSuccess) return hip_fail(e, "pack_linear");
      dst += (size_t)m->NT * NC * 64;
    }
    e = launch_pad_copy(fc_w, m->N, m->NT * 16, m->d_fc, s);
    if (e != hipSuccess) return hip_fail(e, "pad_copy fc");
  }
  m->dense_set = true;
  return DFWFM_OK;
}

int dfwfm_forward(dfwfm_model* m, const int64_t* xi, int64_t xi_stride, const float* xv, int64_t xv_stride,
                  int64_t batch, float* out, void* stream) {
  if (!m) return fail(DFWFM_ERR_INVALID_ARG, "null model");
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

  FwdArgs a;
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
  a.SX = m->SX;
  a.SY = m->SY;
  a.flags = m->flags;
  // diagnostics only (phase timing): DFWFM_DIAG_DROP_FLAGS clears flag bits, results become invalid
  if (const char* drop = getenv("DFWFM_DIAG_DROP_FLAGS")) a.flags &= ~atoi(drop);
  // diagnostics only: DFWFM_DIAG_STAMPS=1 records per-workgroup phase clocks (dfwfm_diag_stamps)
  a.stamps = nullptr;
  if (getenv("DFWFM_DIAG_STAMPS")) {
    const size_t grid = (size_t)((batch + kBM - 1) / kBM);
    if (grid > m->stamps_cap) {
      if (m->d_stamps) (void)hipFree(m->d_stamps);
      m->d_stamps = nullptr;
      m->stamps_cap = 0;
      HIP_TRY(hipMalloc(reinterpret_cast<void**>(&m->d_stamps), grid * kStampSlots * sizeof(uint64_t)));
      m->stamps_cap = grid;
    }
    a.stamps = m->d_stamps;
  }
  hipError_t e = launch_forward(a, m->D, m->TPW > 0 ? m->TPW : 1, m->KS, m->lds_bytes, (hipStream_t)stream);
  if (e != hipSuccess) return hip_fail(e, "forward launch");
  return DFWFM_OK;
}

int dfwfm_diag_stamps(dfwfm_model* m, uint64_t* host, int64_t n, void* stream) {
  if (!m || !host || n < 0) return fail(DFWFM_ERR_INVALID_ARG, "null argument");
  if (!m->d_stamps) return fail(DFWFM_ERR_STATE, "no stamps recorded (set DFWFM_DIAG_STAMPS=1)");
  const size_t cap = m->stamps_cap * kStampSlots;
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
