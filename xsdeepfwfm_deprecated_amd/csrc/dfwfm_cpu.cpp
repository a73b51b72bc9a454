// dfwfm_cpu.cpp -- host (CPU) DeepFwFM forward and backward: the CPU kernel of torch.ops.dfwfm.forward
// (include/dfwfm_cpu.h).  For a module on the CPU -- the reference's -use_cuda 0 / -time_on_cuda 0 paths
// (main_all.py:42-63) and the thread sweep of run_benchmark (model/DeepFMs.py:982-1009).
//
// Per sample the same algebra as the HIP kernels (reference model/DeepFMs.py:285-469):
//   E_f     = v_f[0] * Xv_f (numerical) | v_f[idx] | Wq[idx / c] (*|+) Wr[idx % c] (QREmbeddingBag :156-174)
//   fo_f    = w1_f[...] (tables) | <E_f, Wfl_f> (fwlw);  first = sum_f fo_f (* lw_f)
//   second  = sum_{k<l} Rs[k,l] <E_k, E_l>,  Rs = (R + R^T) / 2 (FwFM) | 1 (FM)
//   deep    = fc . relu(W_H .. relu(W_1 E + b_1) .. + b_H)   (dropout in training: counter-hash masks)
//   logit   = (first + second) + deep + bias
// first and second are accumulated in double (one rounding to f32), the MLP is an AVX2 / FMA GEMM over
// blocks of samples.  Work runs on `threads` std::threads over sample blocks; every reduction is formed per
// block and summed in block order (or per field / output row in sample order), so results do not depend on
// the thread count.
#include "../../include/dfwfm_cpu.h"

#include <atomic>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

namespace {

thread_local std::string g_err;

int fail(int code, const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof buf, fmt, ap);
  va_end(ap);
  g_err = buf;
  return code;
}

typedef float v8f __attribute__((vector_size(32)));

inline v8f ld8(const float* p) {
  v8f v;
  memcpy(&v, p, sizeof v);
  return v;
}
inline void st8(float* p, v8f v) { memcpy(p, &v, sizeof v); }
inline float hsum(v8f v) {
  return ((v[0] + v[4]) + (v[1] + v[5])) + ((v[2] + v[6]) + (v[3] + v[7]));
}

// fn(task, slot) for task < n on up to `threads` threads (slot = the thread's index); tasks are handed out
// dynamically, so nothing may depend on which slot runs a task
template <class Fn>
void parallel_for(int64_t n, int threads, Fn fn) {
  if (n <= 0) return;
  int t = threads < 1 ? 1 : threads;
  if (t > n) t = (int)n;
  if (t == 1) {
    for (int64_t i = 0; i < n; ++i) fn(i, 0);
    return;
  }
  std::atomic<int64_t> next{0};
  auto worker = [&](int slot) {
    for (;;) {
      const int64_t i = next.fetch_add(1);
      if (i >= n) break;
      fn(i, slot);
    }
  };
  std::vector<std::thread> pool;
  pool.reserve(t - 1);
  for (int s = 1; s < t; ++s) pool.emplace_back(worker, s);
  worker(0);
  for (auto& th : pool) th.join();
}

// counter-hash dropout keep mask of the HIP kernels (csrc/dfwfm_device.h dropout_keep)
inline uint32_t mix32(uint32_t x) {
  x ^= x >> 16;
  x *= 0x85EBCA6BU;
  x ^= x >> 13;
  x *= 0xC2B2AE35U;
  x ^= x >> 16;
  return x;
}
inline bool keep(uint32_t seed, int layer, int64_t row, int col, float p) {
  const uint32_t h =
      mix32(seed ^ ((uint32_t)row * 0x9E3779B9U) ^ ((uint32_t)col * 0x7FEB352DU) ^ ((uint32_t)layer * 0x846CA68BU));
  return (float)(h >> 8) * (1.0f / 16777216.0f) >= p;
}

constexpr int kBlock = 32;  // samples per task

struct Model {
  const dfwfm_cpu_model* m;
  int F, num, D, FD, KP, H, N;
  bool second, fwfm, deep, needE, fo_tab, fwlw, lw;
  std::vector<float> Rs;  // [F][F] (R + R^T) / 2 (FM: ones), zero diagonal
  std::vector<int> K;     // input width of layer l
};

int prepare(const dfwfm_cpu_model* m, Model& P) {
  if (!m || !m->fields) return fail(DFWFM_ERR_INVALID_ARG, "null model");
  const dfwfm_config& c = m->cfg;
  P.m = m;
  P.F = c.field_size;
  P.num = c.numerical;
  P.D = c.embedding_size;
  if (P.F < 1 || P.F > 64 || P.num < 0 || P.num > P.F || P.D < 1 || P.D > 64)  // the HIP kernels' limits too
    return fail(DFWFM_ERR_INVALID_ARG, "bad config (F=%d numerical=%d D=%d)", P.F, P.num, P.D);
  if ((c.use_fwfm != 0) + (c.use_fm != 0) + (c.use_logit != 0) > 1)
    return fail(DFWFM_ERR_INVALID_ARG, "at most one of use_fwfm / use_fm / use_logit");
  P.FD = P.F * P.D;
  P.KP = (P.FD + 7) & ~7;
  P.second = c.use_fwfm || c.use_fm;
  P.fwfm = c.use_fwfm != 0;
  P.deep = c.use_deep != 0;
  P.needE = P.second || P.deep;
  P.fwlw = c.use_fwlw != 0;
  P.fo_tab = !P.fwlw;
  P.lw = P.second && c.use_lw;
  P.H = P.deep ? c.h_depth : 0;
  P.N = P.deep ? c.deep_nodes : 0;
  if (!P.second && !P.deep && !c.use_logit) return fail(DFWFM_ERR_INVALID_ARG, "no model part selected");
  if (P.fwfm && !m->field_cov) return fail(DFWFM_ERR_INVALID_ARG, "use_fwfm needs field_cov");
  if (P.fwlw && !m->fwfm_lin) return fail(DFWFM_ERR_INVALID_ARG, "use_fwlw needs fwfm_linear");
  if (P.fwlw && !P.needE) return fail(DFWFM_ERR_UNSUPPORTED, "use_fwlw without embeddings");
  if (P.lw && !m->fm_1st) return fail(DFWFM_ERR_INVALID_ARG, "use_lw needs fm_1st");
  if (P.deep) {
    if (P.H < 1 || P.N < 1 || !m->lin_w || !m->lin_b || !m->fc_w)
      return fail(DFWFM_ERR_INVALID_ARG, "use_deep needs h_depth >= 1 layers and net_1_fc");
    for (int l = 0; l < P.H; ++l)
      if (!m->lin_w[l] || !m->lin_b[l]) return fail(DFWFM_ERR_INVALID_ARG, "layer %d: null weight", l);
  }
  for (int f = 0; f < P.F; ++f) {
    const dfwfm_field_tables& t = m->fields[f];
    if (P.needE && !t.emb2) return fail(DFWFM_ERR_INVALID_ARG, "field %d: null second-order table", f);
    if (P.fo_tab && !t.emb1) return fail(DFWFM_ERR_INVALID_ARG, "field %d: null first-order table", f);
    if (t.qr_collisions > 0 && f >= P.num) {
      if ((P.needE && !t.emb2_r) || (P.fo_tab && !t.emb1_r))
        return fail(DFWFM_ERR_INVALID_ARG, "field %d: QR table without its remainder table", f);
      if (t.qr_operation != 0 && t.qr_operation != 1)
        return fail(DFWFM_ERR_UNSUPPORTED, "field %d: QR operation %d", f, t.qr_operation);
    }
  }
  P.Rs.assign((size_t)P.F * P.F, 0.f);
  if (P.second)
    for (int k = 0; k < P.F; ++k)
      for (int l = 0; l < P.F; ++l)
        if (k != l)
          P.Rs[(size_t)k * P.F + l] =
              P.fwfm ? (m->field_cov[(size_t)l * P.F + k] + m->field_cov[(size_t)k * P.F + l]) * 0.5f : 1.f;
  P.K.assign(P.H, P.N);
  if (P.H) P.K[0] = P.FD;
  return DFWFM_OK;
}

inline int64_t saved_floats(const Model& P) { return (int64_t)P.FD + P.F + (int64_t)P.H * P.N; }

// one field's lookup: the E row (D floats) and the first-order value, index clamped like the HIP kernels
inline void lookup(const Model& P, int f, const int64_t* xi_row, const float* xv_row, float* e, float* fo,
                   int32_t* bad) {
  const dfwfm_field_tables& t = P.m->fields[f];
  const int D = P.D;
  if (f < P.num) {
    const float x = xv_row[f];
    if (P.needE)
      for (int d = 0; d < D; ++d) e[d] = t.emb2[d] * x;
    *fo = P.fo_tab ? t.emb1[0] * x : 0.f;
    return;
  }
  int64_t idx = xi_row[f - P.num];
  const int64_t c = t.qr_collisions > 0 ? t.qr_collisions : 0;
  const int64_t bound = c ? (t.num_categories + c - 1) / c * c : t.num_categories;  // QR: weight_q rows * c
  if (idx < 0 || idx >= bound) {
    *bad = 1;
    idx = 0;
  }
  if (!c) {
    if (P.needE) memcpy(e, t.emb2 + idx * D, sizeof(float) * D);
    *fo = P.fo_tab ? t.emb1[idx] : 0.f;
    return;
  }
  const int64_t q = idx / c, r = idx - q * c;
  const bool mult = t.qr_operation == 0;
  if (P.needE) {
    const float* a = t.emb2 + q * D;
    const float* b = t.emb2_r + r * D;
    for (int d = 0; d < D; ++d) e[d] = mult ? a[d] * b[d] : a[d] + b[d];
  }
  *fo = P.fo_tab ? (mult ? t.emb1[q] * t.emb1_r[r] : t.emb1[q] + t.emb1_r[r]) : 0.f;
}

// Y[r][n] = bias[n] + sum_k X[r][k] W[n][k] for r < R, n < N (X rows zero-padded to a multiple of 8 past K)
void gemm_nt(int R, int N, int K, const float* X, int ldx, const float* W, const float* bias, float* Y, int ldy) {
  const int K8 = K & ~7;
  for (int n0 = 0; n0 < N; n0 += 2) {
    const int nn = N - n0 < 2 ? N - n0 : 2;
    const float* w0 = W + (size_t)n0 * K;
    const float* w1 = W + (size_t)(n0 + nn - 1) * K;
    for (int r0 = 0; r0 < R; r0 += 4) {
      const int rr = R - r0 < 4 ? R - r0 : 4;
      const float* x[4];
      for (int i = 0; i < 4; ++i) x[i] = X + (size_t)(r0 + (i < rr ? i : rr - 1)) * ldx;
      v8f a00 = {}, a01 = {}, a10 = {}, a11 = {}, a20 = {}, a21 = {}, a30 = {}, a31 = {};
      for (int k = 0; k < K8; k += 8) {
        const v8f b0 = ld8(w0 + k), b1 = ld8(w1 + k);
        const v8f x0 = ld8(x[0] + k), x1 = ld8(x[1] + k), x2 = ld8(x[2] + k), x3 = ld8(x[3] + k);
        a00 += x0 * b0; a01 += x0 * b1;
        a10 += x1 * b0; a11 += x1 * b1;
        a20 += x2 * b0; a21 += x2 * b1;
        a30 += x3 * b0; a31 += x3 * b1;
      }
      float s[4][2] = {{hsum(a00), hsum(a01)}, {hsum(a10), hsum(a11)}, {hsum(a20), hsum(a21)}, {hsum(a30), hsum(a31)}};
      for (int k = K8; k < K; ++k)
        for (int i = 0; i < 4; ++i) {
          s[i][0] += x[i][k] * w0[k];
          s[i][1] += x[i][k] * w1[k];
        }
      for (int i = 0; i < rr; ++i)
        for (int j = 0; j < nn; ++j) Y[(size_t)(r0 + i) * ldy + n0 + j] = bias[n0 + j] + s[i][j];
    }
  }
}

// y[0..K) += g * w[0..K)
inline void axpy(int K, float g, const float* w, float* y) {
  int k = 0;
  const v8f gv = {g, g, g, g, g, g, g, g};
  for (; k + 8 <= K; k += 8) st8(y + k, ld8(y + k) + gv * ld8(w + k));
  for (; k < K; ++k) y[k] += g * w[k];
}

// ---- forward -------------------------------------------------------------------------------------------
void forward_block(const Model& P, int64_t b0, int64_t nb, const int64_t* xi, int64_t xs, const float* xv,
                   int64_t vs, float* out, float* saved, float drop_p, uint32_t seed, int32_t* bad) {
  const int F = P.F, D = P.D, FD = P.FD, KP = P.KP, N = P.N;
  const int NP = (N + 7) & ~7;
  std::vector<float> E((size_t)kBlock * KP, 0.f), fo((size_t)kBlock * F);
  std::vector<float> A, Bf;
  const bool train = saved != nullptr;
  const bool drop = train && P.deep && drop_p > 0.f;
  const float scale = drop ? 1.f / (1.f - drop_p) : 1.f;
  double first[kBlock], second[kBlock];
  std::vector<double> ed((size_t)FD), acc((size_t)D);  // one sample's E in double, the FwFM row sum
  for (int64_t i = 0; i < nb; ++i) {
    const int64_t b = b0 + i;
    const int64_t* xr = xi + b * xs;
    const float* vr = xv + b * vs;
    float* e = E.data() + i * KP;
    float* o = fo.data() + i * F;
    for (int f = 0; f < F; ++f) lookup(P, f, xr, vr, e + f * D, o + f, bad);
    if (P.fwlw)
      for (int f = 0; f < F; ++f) {
        float s = 0.f;
        for (int d = 0; d < D; ++d) s += e[f * D + d] * P.m->fwfm_lin[f * D + d];
        o[f] = s;
      }
    double s1 = 0.0;
    for (int f = 0; f < F; ++f) s1 += P.lw ? (double)o[f] * (double)P.m->fm_1st[f] : (double)o[f];
    double s2 = 0.0;
    if (P.second) {
      // sum_k <E_k, sum_{l>k} Rs[k,l] E_l>, in double: the inner sum is a D-wide axpy (vectorises over d)
      for (int j = 0; j < FD; ++j) ed[j] = e[j];
      for (int k = 0; k + 1 < F; ++k) {
        const float* rk = P.Rs.data() + (size_t)k * F;
        for (int d = 0; d < D; ++d) acc[d] = 0.0;
        for (int l = k + 1; l < F; ++l) {
          const double r = rk[l];
          const double* el = ed.data() + (size_t)l * D;
          for (int d = 0; d < D; ++d) acc[d] += r * el[d];
        }
        const double* ek = ed.data() + (size_t)k * D;
        for (int d = 0; d < D; ++d) s2 += ek[d] * acc[d];
      }
    }
    first[i] = s1;
    second[i] = s2;
    if (train) {
      float* sv = saved + b * saved_floats(P);
      memcpy(sv, e, sizeof(float) * FD);
      memcpy(sv + FD, o, sizeof(float) * F);
    }
  }
  float deep[kBlock] = {};
  if (P.deep) {
    // A: this layer's input [kBlock][ldA], Bf: its output; X_0 = E (dropped in training)
    const int ld0 = KP > NP ? KP : NP;
    A.assign((size_t)kBlock * ld0, 0.f);
    Bf.assign((size_t)kBlock * ld0, 0.f);
    for (int64_t i = 0; i < nb; ++i)
      for (int k = 0; k < FD; ++k) {
        const float v = E[i * KP + k];
        A[i * ld0 + k] = drop ? (keep(seed, 0, b0 + i, k, drop_p) ? v * scale : 0.f) : v;
      }
    for (int l = 0; l < P.H; ++l) {
      gemm_nt((int)nb, N, P.K[l], A.data(), ld0, P.m->lin_w[l], P.m->lin_b[l], Bf.data(), ld0);
      for (int64_t i = 0; i < nb; ++i) {
        float* y = Bf.data() + i * ld0;
        for (int n = 0; n < N; ++n) {
          float v = y[n] > 0.f ? y[n] : 0.f;  // ReLU (NaN -> NaN is irrelevant here: finite inputs)
          if (drop) v = keep(seed, l + 1, b0 + i, n, drop_p) ? v * scale : 0.f;
          y[n] = v;
        }
        for (int n = N; n < ld0; ++n) y[n] = 0.f;
        if (train) memcpy(saved + (b0 + i) * saved_floats(P) + FD + F + (size_t)l * N, y, sizeof(float) * N);
      }
      A.swap(Bf);
    }
    for (int64_t i = 0; i < nb; ++i) {
      const float* h = A.data() + i * ld0;
      float s = 0.f;
      for (int n = 0; n < N; ++n) s += h[n] * P.m->fc_w[n];
      deep[i] = s;
    }
  }
  const float bias = P.m->bias ? P.m->bias[0] : 0.f;
  for (int64_t i = 0; i < nb; ++i) out[b0 + i] = ((float)(first[i] + second[i]) + deep[i]) + bias;
}

// ---- backward ------------------------------------------------------------------------------------------
// per-block partial sums of the small dense gradients: bias | lw[F] | fwlw[F*D] | R[F*F] | fc[N]
struct Partial {
  int F, D, N;
  int o_lw, o_fwlw, o_r, o_fc, size;
  void init(int F_, int D_, int N_) {
    F = F_, D = D_, N = N_;
    o_lw = 1;
    o_fwlw = o_lw + F;
    o_r = o_fwlw + F * D;
    o_fc = o_r + F * F;
    size = o_fc + N;
  }
};

}  // namespace

extern "C" {

int dfwfm_cpu_abi_version(void) { return DFWFM_CPU_ABI_VERSION; }

const char* dfwfm_cpu_last_error(void) { return g_err.c_str(); }

int64_t dfwfm_cpu_saved_floats(const dfwfm_config* c) {
  if (!c) return 0;
  const int64_t H = c->use_deep ? c->h_depth : 0, N = c->use_deep ? c->deep_nodes : 0;
  return (int64_t)c->field_size * c->embedding_size + c->field_size + H * N;
}

int dfwfm_cpu_forward(const dfwfm_cpu_model* m, const int64_t* xi, int64_t xi_stride, const float* xv,
                      int64_t xv_stride, int64_t batch, float* out, float* saved, float drop_p, uint32_t seed,
                      int32_t* err_flags, int32_t threads) {
  Model P;
  int rc = prepare(m, P);
  if (rc != DFWFM_OK) return rc;
  if (batch < 0) return fail(DFWFM_ERR_INVALID_ARG, "negative batch");
  if (batch == 0) return DFWFM_OK;
  if (!out || (P.F > P.num && !xi) || (P.num > 0 && !xv)) return fail(DFWFM_ERR_INVALID_ARG, "null input");
  if (drop_p < 0.f || drop_p >= 1.f) return fail(DFWFM_ERR_INVALID_ARG, "dropout p %f", (double)drop_p);
  const int64_t nblk = (batch + kBlock - 1) / kBlock;
  std::vector<int32_t> bad(nblk, 0);
  parallel_for(nblk, threads, [&](int64_t t, int) {
    const int64_t b0 = t * kBlock;
    const int64_t nb = batch - b0 < kBlock ? batch - b0 : kBlock;
    forward_block(P, b0, nb, xi, xi_stride, xv, xv_stride, out, saved, drop_p, seed, &bad[t]);
  });
  if (err_flags)
    for (int32_t v : bad)
      if (v) *err_flags |= DFWFM_FLAG_INDEX_OUT_OF_RANGE;
  return DFWFM_OK;
}

int dfwfm_cpu_backward(const dfwfm_cpu_model* m, const int64_t* xi, int64_t xs, const float* xv, int64_t vs,
                       int64_t batch, const float* dlogit, const float* saved, float drop_p, uint32_t seed,
                       const dfwfm_grads* g, int32_t threads) {
  Model P;
  int rc = prepare(m, P);
  if (rc != DFWFM_OK) return rc;
  if (!g) return fail(DFWFM_ERR_INVALID_ARG, "null grads");
  if (batch <= 0) return batch < 0 ? fail(DFWFM_ERR_INVALID_ARG, "negative batch") : DFWFM_OK;
  if (!dlogit || !saved) return fail(DFWFM_ERR_INVALID_ARG, "null dlogit / saved activations");
  const int F = P.F, D = P.D, FD = P.FD, N = P.N, H = P.H;
  const int64_t SV = saved_floats(P);
  const bool drop = P.deep && drop_p > 0.f;
  const float scale = drop ? 1.f / (1.f - drop_p) : 1.f;
  const int64_t nblk = (batch + kBlock - 1) / kBlock;
  Partial pl;
  pl.init(F, D, N);
  std::vector<float> part((size_t)nblk * pl.size, 0.f);
  std::vector<float> dE(P.needE ? (size_t)batch * FD : 0);
  std::vector<float> G((size_t)H * batch * N), A0(P.deep ? (size_t)batch * FD : 0);
  const int K0 = FD;

  // phase 1, per sample block: the deep chain (G_l saved for the weight gradients), dE, the dense partials
  parallel_for(nblk, threads, [&](int64_t t, int) {
    const int64_t b0 = t * kBlock;
    const int64_t nb = batch - b0 < kBlock ? batch - b0 : kBlock;
    float* pt = part.data() + (size_t)t * pl.size;
    std::vector<float> dA((size_t)kBlock * (K0 > N ? K0 : N)), dB((size_t)kBlock * (K0 > N ? K0 : N));
    const int ldd = K0 > N ? K0 : N;
    if (P.deep) {
      // dA_H = dlogit * fc; G_l = dA_{l+1} * (A_{l+1} > 0) * scale; dA_l = W_l^T G_l
      for (int64_t i = 0; i < nb; ++i) {
        const int64_t b = b0 + i;
        const float dl = dlogit[b];
        const float* aH = saved + b * SV + FD + F + (size_t)(H - 1) * N;
        float* dst = dA.data() + i * ldd;
        for (int n = 0; n < N; ++n) {
          dst[n] = dl * P.m->fc_w[n];
          pt[pl.o_fc + n] += dl * aH[n];
        }
      }
      for (int l = H - 1; l >= 0; --l) {
        const int Kl = P.K[l];
        const float* W = P.m->lin_w[l];
        for (int64_t i = 0; i < nb; ++i) {
          const int64_t b = b0 + i;
          const float* aout = saved + b * SV + FD + F + (size_t)l * N;  // A_{l+1}
          float* gl = G.data() + ((size_t)l * batch + b) * N;
          const float* da = dA.data() + i * ldd;
          for (int n = 0; n < N; ++n) gl[n] = aout[n] > 0.f ? da[n] * scale : 0.f;
          float* dx = dB.data() + i * ldd;
          memset(dx, 0, sizeof(float) * Kl);
          for (int n = 0; n < N; ++n)
            if (gl[n] != 0.f) axpy(Kl, gl[n], W + (size_t)n * Kl, dx);
        }
        dA.swap(dB);
      }
      // dA now holds dA_0 = dL/d(dropped E); A_0 for the layer-1 weight gradient
      for (int64_t i = 0; i < nb; ++i) {
        const int64_t b = b0 + i;
        const float* e = saved + b * SV;
        float* a0 = A0.data() + b * FD;
        float* de = dE.data() + b * FD;
        const float* da = dA.data() + i * ldd;
        for (int k = 0; k < FD; ++k) {
          const bool kp = !drop || keep(seed, 0, b, k, drop_p);
          a0[k] = kp ? e[k] * scale : 0.f;
          de[k] = kp ? da[k] * scale : 0.f;
        }
      }
    } else if (P.needE) {
      for (int64_t i = 0; i < nb; ++i) memset(dE.data() + (b0 + i) * FD, 0, sizeof(float) * FD);
    }
    // shallow terms
    for (int64_t i = 0; i < nb; ++i) {
      const int64_t b = b0 + i;
      const float dl = dlogit[b];
      const float* e = saved + b * SV;
      const float* fo = e + FD;
      float* de = P.needE ? dE.data() + b * FD : nullptr;
      pt[0] += dl;
      for (int f = 0; f < F; ++f) {
        const float lwf = P.lw ? P.m->fm_1st[f] : 1.f;
        if (P.lw) pt[pl.o_lw + f] += dl * fo[f];
        if (P.fwlw)
          for (int d = 0; d < D; ++d) {
            de[f * D + d] += dl * lwf * P.m->fwfm_lin[f * D + d];
            pt[pl.o_fwlw + f * D + d] += dl * lwf * e[f * D + d];
          }
      }
      if (P.second) {
        for (int k = 0; k < F; ++k) {
          const float* rk = P.Rs.data() + (size_t)k * F;
          float* dk = de + k * D;
          for (int l = 0; l < F; ++l) {
            if (l == k) continue;
            const float w = dl * rk[l];
            const float* el = e + l * D;
            for (int d = 0; d < D; ++d) dk[d] += w * el[d];
            if (P.fwfm && l > k) {
              float dot = 0.f;
              for (int d = 0; d < D; ++d) dot += e[k * D + d] * el[d];
              const float gr = 0.5f * dl * dot;  // d second / d R[k][l] = d / d R[l][k] = <E_k, E_l> / 2
              pt[pl.o_r + k * F + l] += gr;
              pt[pl.o_r + l * F + k] += gr;
            }
          }
        }
      }
    }
  });

  // the dense partials, in block order
  auto reduce_into = [&](float* dst, int off, int n) {
    if (!dst) return;
    for (int j = 0; j < n; ++j) {
      float s = 0.f;
      for (int64_t t = 0; t < nblk; ++t) s += part[(size_t)t * pl.size + off + j];
      dst[j] += s;
    }
  };
  reduce_into(g->bias, 0, 1);
  if (P.lw) reduce_into(g->fm_1st, pl.o_lw, F);
  if (P.fwlw) reduce_into(g->fwfm_lin, pl.o_fwlw, F * D);
  if (P.fwfm) reduce_into(g->field_cov, pl.o_r, F * F);
  if (P.deep) reduce_into(g->fc_w, pl.o_fc, N);

  // phase 2: weight gradients dW_l[n][k] += sum_b G_l[b][n] A_l[b][k] (8 output rows per task, samples in order)
  if (P.deep && g->lin_w) {
    const int nbn = (N + 7) / 8;
    parallel_for((int64_t)H * nbn, threads, [&](int64_t t, int) {
      const int l = (int)(t / nbn);
      const int n0 = (int)(t % nbn) * 8;
      const int n1 = n0 + 8 < N ? n0 + 8 : N;
      const int Kl = P.K[l];
      float* dW = g->lin_w[l];
      float* db = g->lin_b ? g->lin_b[l] : nullptr;
      for (int64_t b = 0; b < batch; ++b) {
        const float* a = l == 0 ? A0.data() + b * FD : saved + b * SV + FD + F + (size_t)(l - 1) * N;
        const float* gl = G.data() + ((size_t)l * batch + b) * N;
        for (int n = n0; n < n1; ++n) {
          const float gv = gl[n];
          if (gv == 0.f) continue;
          if (dW) axpy(Kl, gv, a, dW + (size_t)n * Kl);
          if (db) db[n] += gv;
        }
      }
    });
  }

  // phase 3: the tables, one task per field (samples in order: no races, fixed summation order)
  parallel_for(F, threads, [&](int64_t ft, int) {
    const int f = (int)ft;
    const dfwfm_field_tables& t = P.m->fields[f];
    const dfwfm_field_grads* fg = g->fields ? &g->fields[f] : nullptr;
    if (!fg) return;
    const float lwf = P.lw ? P.m->fm_1st[f] : 1.f;
    const int64_t c = (f >= P.num && t.qr_collisions > 0) ? t.qr_collisions : 0;
    const int64_t bound = c ? (t.num_categories + c - 1) / c * c : t.num_categories;
    for (int64_t b = 0; b < batch; ++b) {
      const float* de = P.needE ? dE.data() + b * FD + f * D : nullptr;
      const float dfo = dlogit[b] * lwf;
      if (f < P.num) {
        const float x = xv[b * vs + f];
        if (de && fg->emb2)
          for (int d = 0; d < D; ++d) fg->emb2[d] += de[d] * x;
        if (P.fo_tab && fg->emb1) fg->emb1[0] += dfo * x;
        continue;
      }
      int64_t idx = xi[b * xs + (f - P.num)];
      if (idx < 0 || idx >= bound) idx = 0;
      if (!c) {
        if (de && fg->emb2) axpy(D, 1.f, de, fg->emb2 + idx * D);
        if (P.fo_tab && fg->emb1) fg->emb1[idx] += dfo;
        continue;
      }
      const int64_t q = idx / c, r = idx - q * c;
      const bool mult = t.qr_operation == 0;
      if (de) {
        const float* wq = t.emb2 + q * D;
        const float* wr = t.emb2_r + r * D;
        for (int d = 0; d < D; ++d) {
          if (fg->emb2) fg->emb2[q * D + d] += mult ? de[d] * wr[d] : de[d];
          if (fg->emb2_r) fg->emb2_r[r * D + d] += mult ? de[d] * wq[d] : de[d];
        }
      }
      if (P.fo_tab) {
        if (fg->emb1) fg->emb1[q] += mult ? dfo * t.emb1_r[r] : dfo;
        if (fg->emb1_r) fg->emb1_r[r] += mult ? dfo * t.emb1[q] : dfo;
      }
    }
  });
  return DFWFM_OK;
}

}  // extern "C"
