/*
 * dfwfm_cpu.h -- C ABI of the host (CPU) DeepFwFM forward / backward (libdfwfm_cpu.so).
 *
 * The same hot path as include/dfwfm.h -- `DeepFMs.forward(Xi, Xv) -> logits` (reference
 * model/DeepFMs.py:285-469) and, for training, its backward (`loss.backward()`, :636) -- for a module that
 * lives on the CPU: the reference's `-use_cuda 0` / `-time_on_cuda 0` paths (main_all.py:42-63) and its
 * 1- / 4-thread timing sweep (model/DeepFMs.py:982-1009).  It is the CPU kernel of the custom operator
 * `torch.ops.dfwfm.forward` (dispatched by the tensors' device), never a fallback of the HIP path: a module
 * on a HIP device runs libdfwfm.so or raises.
 *
 * Written for the host, not translated from the reference's op sequence: one pass per sample block --
 * gather, first order, the FwFM second order as sum_{k<l} Rs[k,l] <E_k, E_l> over the upper triangle
 * (no [F, F, B, D] intermediates), the MLP as a register-blocked AVX2 / FMA GEMM -- on `threads` host
 * threads (torch.get_num_threads() of the caller).
 *
 * Host pointers only; the tables are the caller's parameters (dfwfm_field_tables with host pointers).
 * Status codes as dfwfm_status; never aborts; out-of-range indices are clamped to row 0 and reported in
 * *err_flags (DFWFM_FLAG_INDEX_OUT_OF_RANGE), like the HIP forward's sticky flag.
 */
#ifndef DFWFM_CPU_H
#define DFWFM_CPU_H

#include <stdint.h>

#include "dfwfm.h"

#ifdef __cplusplus
extern "C" {
#endif

#define DFWFM_CPU_ABI_VERSION 1

/* A model's parameters, by host pointer (the same tensors dfwfm_model_set_tables / _set_dense take). */
typedef struct {
  dfwfm_config cfg;
  const dfwfm_field_tables* fields;  /* cfg.field_size entries                                     */
  const float* field_cov;            /* [F, F] or NULL                                              */
  const float* fwfm_lin;             /* [F, D] or NULL                                              */
  const float* fm_1st;               /* [F] or NULL                                                 */
  const float* bias;                 /* [1] or NULL                                                 */
  const float* const* lin_w;         /* h_depth pointers, [N, K_h] each (use_deep)                 */
  const float* const* lin_b;         /* h_depth pointers, [N] each                                  */
  const float* fc_w;                 /* [N] (use_deep)                                              */
} dfwfm_cpu_model;

/* Floats per sample that a training forward saves for dfwfm_cpu_backward (E, first order, hidden outputs). */
int64_t dfwfm_cpu_saved_floats(const dfwfm_config* cfg);

/* logits[b], b < batch (replaces model/DeepFMs.py:285-469).  xi int64 [batch, F - numerical] (row stride
 * xi_stride), xv f32 [batch, >= numerical] (row stride xv_stride).  saved (or NULL): batch x
 * dfwfm_cpu_saved_floats floats written for the backward, and the deep tower's dropout (drop_p, seed: the
 * HIP kernels' counter-hash masks) applied -- a training forward.  *err_flags |= DFWFM_FLAG_INDEX_OUT_OF_RANGE
 * when an index is outside its table (the row is read as row 0). */
int dfwfm_cpu_forward(const dfwfm_cpu_model* m, const int64_t* xi, int64_t xi_stride, const float* xv,
                      int64_t xv_stride, int64_t batch, float* out, float* saved, float drop_p, uint32_t seed,
                      int32_t* err_flags, int32_t threads);

/* Gradients of sum_b dlogit[b] * logit[b] accumulated (+=) into `grads` (host pointers, NULL skips a tensor;
 * replaces loss.backward(), :636), from the activations a training forward saved on the same inputs. */
int dfwfm_cpu_backward(const dfwfm_cpu_model* m, const int64_t* xi, int64_t xi_stride, const float* xv,
                       int64_t xv_stride, int64_t batch, const float* dlogit, const float* saved, float drop_p,
                       uint32_t seed, const dfwfm_grads* grads, int32_t threads);

const char* dfwfm_cpu_last_error(void);
int dfwfm_cpu_abi_version(void);

#ifdef __cplusplus
}
#endif

#endif /* DFWFM_CPU_H */
