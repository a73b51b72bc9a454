/*
 * dfwfm.h -- C ABI of the MI355X-native DeepFwFM forward engine (libdfwfm.so).
 *
 * This is the drop-in boundary for the one hot path of the reference
 * (ShanningLiu/xsDeepFwFM_deprecated): `DeepFMs.forward(Xi, Xv) -> logits`
 * (reference model/DeepFMs.py:285-469) together with the per-field embedding
 * modules it calls (nn.Embedding / nn.EmbeddingBag, model/DeepFMs.py:201-210,
 * 1066-1091, and QREmbeddingBag, model/QREmbeddingBag.py:156-174).
 *
 * Plain C: device pointers, sizes, an opaque model handle, and the HIP stream
 * passed as `void*` (a hipStream_t; NULL = the default stream).  No torch
 * types cross this boundary.  All pointers named "device" must be HIP device
 * memory on the current device; nothing here synchronises the stream except
 * dfwfm_read_error_flag().
 *
 * Error behaviour: every entry point returns a dfwfm_status (0 = ok, negative
 * = error) and never aborts; dfwfm_last_error() gives a human-readable message
 * for the calling thread.  Out-of-range embedding indices (the reference
 * raises IndexError from nn.Embedding) cannot be reported synchronously by a
 * kernel: the forward clamps the read to row 0 so it never faults, and sets a
 * sticky device flag that dfwfm_read_error_flag() returns (and clears).
 */
#ifndef DFWFM_H
#define DFWFM_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define DFWFM_ABI_VERSION 4  /* 4: dfwfm_model_pack_tables / dfwfm_forward_gather added, the split forward of
                                dfwfm_forward_ws removed (its workspace now serves the sparse tower only); 3:
                                dfwfm_sparse_grads removed, dfwfm_model_set_dense_zero / dfwfm_backward_phases_bce added */

typedef enum {
  DFWFM_OK = 0,
  DFWFM_ERR_INVALID_ARG = -1,  /* null pointer, bad size, inconsistent config  */
  DFWFM_ERR_UNSUPPORTED = -2,  /* a shape the compiled kernels do not cover     */
  DFWFM_ERR_HIP = -3,          /* a HIP runtime call failed                    */
  DFWFM_ERR_STATE = -4,        /* forward before tables / dense weights are set */
} dfwfm_status;

/* Error flag bits written by the forward kernel (dfwfm_read_error_flag). */
#define DFWFM_FLAG_INDEX_OUT_OF_RANGE 1

/* Model configuration -- mirrors the DeepFMs constructor switches
 * (reference model/DeepFMs.py:81-89, utils/util.py:58-73).  Exactly one of
 * use_fwfm / use_fm / use_logit may be set (reference :159-161). */
typedef struct {
  int32_t field_size;      /* F: fields (39 for Criteo)                         */
  int32_t numerical;       /* leading numerical fields (13 for Criteo)          */
  int32_t embedding_size;  /* D (10)                                            */
  int32_t use_fwfm;        /* FwFM second order  sum_{k<l} r_kl <v_k, v_l>      */
  int32_t use_fm;          /* FM second order (r_kl = 1)                        */
  int32_t use_logit;       /* logistic regression: first order only            */
  int32_t use_deep;        /* 3x400 ReLU MLP on the concatenated embeddings     */
  int32_t use_lw;          /* first order projected by fm_1st.weight [1, F]     */
  int32_t use_fwlw;        /* first order from fwfm_linear.weight [F, D]        */
  int32_t h_depth;         /* hidden layers (3)                                 */
  int32_t deep_nodes;      /* hidden width (400)                                */
} dfwfm_config;

/* Per-field embedding tables (device pointers into the caller's parameters).
 *  - numerical field  (f < numerical): emb2 = v_f [1, D], emb1 = w1_f [1, 1]
 *  - plain categorical: emb2 = [n, D], emb1 = [n, 1]
 *  - QR categorical (qr_collisions > 0): emb2 = weight_q [ceil(n/c), D],
 *    emb2_r = weight_r [c, D]; likewise emb1 / emb1_r for the first-order
 *    QR bag (reference create_emb, model/DeepFMs.py:1066-1091).
 * emb1 / emb1_r are NULL when the first order comes from fwlw or is unused. */
typedef struct {
  const float* emb2;
  const float* emb2_r;
  const float* emb1;
  const float* emb1_r;
  int64_t num_categories;  /* n: valid indices are [0, n)                     */
  int64_t qr_collisions;   /* c; 0 = plain table                              */
  int32_t qr_operation;    /* 0 = "mult", 1 = "add" ("concat" unsupported)    */
  int32_t reserved;
} dfwfm_field_tables;

typedef struct dfwfm_model dfwfm_model;

/* Allocates the model's device-side state (packed dense weights, field
 * descriptors, error flag) on the current device. */
int dfwfm_model_create(const dfwfm_config* cfg, dfwfm_model** out);
void dfwfm_model_destroy(dfwfm_model* m);

/* Uploads the F per-field table descriptors.  Call again whenever a table is
 * re-allocated (e.g. after moving the module); in-place updates need no call. */
int dfwfm_model_set_tables(dfwfm_model* m, const dfwfm_field_tables* tables,
                           int32_t n_fields, void* stream);

/* Packs the dense parameters into the kernel layout, on `stream` (no sync).
 * Call again after any in-place update of these parameters.
 *   field_cov  [F, F]    field_cov.weight (R; symmetrised as (R + R^T)/2)  or NULL
 *   fwfm_lin   [F, D]    fwfm_linear.weight                                or NULL
 *   fm_1st     [F]       fm_1st.weight                                     or NULL
 *   bias       [1]       bias                                              or NULL
 *   lin_w[h]   [N, K_h]  net_1_linear_{h+1}.weight, K_0 = F*D, K_h = N      (use_deep)
 *   lin_b[h]   [N]       net_1_linear_{h+1}.bias                            (use_deep)
 *   fc_w       [N]       net_1_fc.weight                                    (use_deep)
 * lin_w / lin_b are host arrays of h_depth device pointers. */
int dfwfm_model_set_dense(dfwfm_model* m, const float* field_cov, const float* fwfm_lin,
                          const float* fm_1st, const float* bias,
                          const float* const* lin_w, const float* const* lin_b,
                          const float* fc_w, void* stream);
/* The same, and zero[0, nzero) (device floats, 16-byte aligned, nzero a multiple of 4) zeroed in the same launch:
 * a training step's gradient buffer, so the re-pack and the zeroing run side by side (one launch, not two). */
int dfwfm_model_set_dense_zero(dfwfm_model* m, const float* field_cov, const float* fwfm_lin,
                               const float* fm_1st, const float* bias,
                               const float* const* lin_w, const float* const* lin_b,
                               const float* fc_w, float* zero, int64_t nzero, void* stream);

/* The hot path: logits[b] for b in [0, batch).
 *   xi  int64 [batch, F - numerical] (row stride xi_stride elements): categorical indices
 *   xv  f32   [batch, >= numerical]  (row stride xv_stride elements): numerical values
 *   out f32   [batch]  pre-sigmoid logits (reference forward return value)
 * Replaces DeepFMs.forward, model/DeepFMs.py:285-469. */
int dfwfm_forward(dfwfm_model* m, const int64_t* xi, int64_t xi_stride, const float* xv,
                  int64_t xv_stride, int64_t batch, float* out, void* stream);

/* The forward of nb batches in ONE launch per (up to) 32 batches on `stream`: batch i reads xi[i] / xv[i]
 * (device pointers, `batch` rows each, the same strides) and writes its logits to out[i].  A serving queue's
 * batches in flight as one grid: the workgroups of all of them are dispatched as CU slots free up, so no batch
 * waits for a launch boundary and a short run has no per-launch drain.  Every batch's logits are bit-identical to
 * dfwfm_forward on that batch alone.  Replaces nb calls of the reference's forward (model/DeepFMs.py:285-469),
 * e.g. eval_by_batch's per-batch loop (:750-780) over resident batches. */
int dfwfm_forward_batches(dfwfm_model* m, int32_t nb, const int64_t* const* xi, int64_t xi_stride,
                          const float* const* xv, int64_t xv_stride, int64_t batch, float* const* out, void* stream);

/* The forward as two launches on `stream` -- the gather / shallow part (E tile and first + second
 * order to `workspace`), then the MLP and the combine -- so that two batches in flight on two
 * streams overlap their MLPs on every CU.  Same logits as dfwfm_forward, bit for bit.
 * dfwfm_forward_workspace_bytes reports the workspace a batch needs (0: this model runs the single
 * fused launch, e.g. no deep part, and dfwfm_forward_ws == dfwfm_forward).  The workspace is
 * caller-owned device memory, 16-byte aligned, in use until the launches complete on `stream`;
 * NULL also selects the fused launch.  Replaces the same reference call as dfwfm_forward
 * (model/DeepFMs.py:285-469). */
int dfwfm_forward_workspace_bytes(dfwfm_model* m, int64_t batch, size_t* bytes);
int dfwfm_forward_ws(dfwfm_model* m, const int64_t* xi, int64_t xi_stride, const float* xv,
                     int64_t xv_stride, int64_t batch, float* out, void* workspace, size_t ws_bytes,
                     void* stream);

/* The gather / shallow half of a deep model's forward alone (reference model/DeepFMs.py:300-367 and the deep_emb
 * `cat` of :398): the per-field embedding rows (numerical v_f * Xv, categorical nn.Embedding / QR rows) into
 * deep_emb [batch][deep_emb_stride] (zero padded past F * D) and first + second order into first_second[batch] --
 * the forward without its MLP (the MLP-free forward's kernel storing deep_emb), so that the gather has its own
 * duration and HBM rate (bench.py roofline_gather); first_second agrees with the fused forward's shallow part to
 * fp32 summation order.  deep_emb_stride must equal ceil(F * D / 16) * 16 (the MLP's K chunks).  Models without
 * a deep tower: DFWFM_ERR_UNSUPPORTED (their whole forward is this half). */
int dfwfm_forward_gather(dfwfm_model* m, const int64_t* xi, int64_t xi_stride, const float* xv, int64_t xv_stride,
                         int64_t batch, float* deep_emb, int64_t deep_emb_stride, float* first_second, void* stream);

/* Pruned deep tower (BASELINE configs[3]; reference masks model/DeepFMs.py:647-673, whose forward stays
 * dense): compacts every hidden layer's nonzero weights (the tensors of the last
 * dfwfm_model_set_dense) into a per-neuron (k, w) list on the device and, when the nonzero fraction
 * of the hidden layers is <= max_density, makes dfwfm_forward_ws run the gather launch followed by a
 * sparse MLP over those lists (dfwfm_forward_workspace_bytes then reports the gather workspace).
 * *enabled = 1 when the sparse path is on.  Synchronises `stream` (reads the nonzero count); call it
 * after a weight update, not per forward.  dfwfm_model_set_dense turns the path off again until the
 * next call; max_density <= 0 turns it off.  Logits agree with the dense forward to fp32 summation
 * order (1e-5 bar). */
int dfwfm_model_build_sparse_mlp(dfwfm_model* m, double max_density, int32_t* enabled, void* stream);

/* Pruned FwFM (R masked by |(R + R^T)/2|, reference model/DeepFMs.py:661-666; SURVEY a12: 73 of 741 pairs at
 * Criteo-39): lists the nonzero strictly-upper entries of (R + R^T)/2 from the last dfwfm_model_set_dense and,
 * when there are at most max_pairs, makes the forward without a deep tower (fwd_kernel PART 3) sum
 * second[b] = sum over the list of w_kl <E_bk, E_bl> instead of the dense per-sample Gram on MFMA.
 * *enabled = 1 when the pair path is on.  Synchronises `stream` (reads the packed R); call it after a weight
 * update, not per forward; dfwfm_model_set_dense turns the path off until the next call; max_pairs <= 0 turns
 * it off.  Logits agree with the dense forward to fp32 summation order (1e-5 bar). */
int dfwfm_model_build_fwfm_pairs(dfwfm_model* m, int32_t max_pairs, int32_t* enabled, void* stream);

/* Serving copy of the categorical tables for the inference forward (dfwfm_forward / _batches; not the training
 * forward, which reads the tables the optimizer updates): every row of
 * every categorical field's second-order table (emb2) with its first-order weight (emb1) appended, padded to a
 * 64-byte row (D + 1 <= 16 floats; else D + 1 rounded up to 4), so the gather reads ONE aligned row per (sample,
 * field) instead of a 40-B row plus a 4-B first-order word from another table (the separate 4-B reads cost the
 * gather alone +0.5 us per 4096 samples with Infinity-Cache-resident tables and +0.8-1.3 us HBM-resident,
 * tools/ubench_gather.hip).  The values are copied, so the logits are bit-identical with and without it.
 * enable = 1 (re)builds the copy from the tables of the last dfwfm_model_set_tables (stream-ordered, no sync) and
 * the inference forward reads it from then on; enable = 0 drops it.  It is a snapshot: rebuild it after any
 * in-place update of the tables (the Python engine does, from torch's version counters), and
 * dfwfm_model_set_tables drops it.  *enabled = 1 when the copy is in use (models with QR fields, no first-order
 * tables or no second order keep the plain tables: 0). */
int dfwfm_model_pack_tables(dfwfm_model* m, int32_t enable, int32_t* enabled, void* stream);

/* ---- training step (reference model/DeepFMs.py:553-637) ---------------------------------- */

/* Forward of a training step: as dfwfm_forward, and additionally keeps (in model-owned device
 * memory, grown on demand -- so the first call at a new batch size allocates) the activations
 * the backward needs.  dropout_p is the deep tower's dropout (reference nn.Dropout(0.5) on
 * deep_emb and after every hidden ReLU, :260-282; 0 = none); masks come from a counter hash of
 * (seed, layer, row, column), so the backward regenerates them. */
int dfwfm_train_forward(dfwfm_model* m, const int64_t* xi, int64_t xi_stride, const float* xv,
                        int64_t xv_stride, int64_t batch, float* out, float dropout_p, uint32_t seed,
                        void* stream);

/* Gradient buffers of one field's tables (device, dense, same shapes as the tables; any may be
 * NULL to skip it). */
typedef struct {
  float* emb2;
  float* emb2_r;
  float* emb1;
  float* emb1_r;
} dfwfm_field_grads;

/* Dense gradient buffers, accumulated into (+=), like autograd's .grad.  NULL skips a tensor. */
typedef struct {
  const dfwfm_field_grads* fields;  /* host array of field_size entries                     */
  float* field_cov;                 /* [F, F]                                                */
  float* fwfm_lin;                  /* [F, D]                                                */
  float* fm_1st;                    /* [F]                                                   */
  float* bias;                      /* [1]                                                   */
  float* const* lin_w;              /* host array of h_depth device pointers, [N, K_h] each  */
  float* const* lin_b;              /* host array of h_depth device pointers, [N] each       */
  float* fc_w;                      /* [N]                                                   */
} dfwfm_grads;

/* Backward of the last dfwfm_train_forward: dlogit [batch] = dLoss/dlogit (e.g. (sigmoid(z) - y)
 * / batch for the reference's BCE-with-logits mean, :634).  Replaces loss.backward() (:636). */
int dfwfm_backward(dfwfm_model* m, const float* dlogit, const dfwfm_grads* grads, void* stream);

/* Deterministic backward (ON by default since ABI 4's round-6 build; +2.6 % per Criteo-39 training step): every
 * gradient sum is formed in a fixed order -- the categorical tables' contributions sorted by (row, sample) and summed
 * by one owner per row, the weight-gradient GEMM's batch splits summed in split order -- so two runs of the same step
 * give the same bits (the reference's CPU step, model/DeepFMs.py:634-637, is reproducible).  Off (on = 0), both use
 * float atomics (sums in arrival order).  Affects the launches enqueued after the call. */
int dfwfm_set_deterministic(dfwfm_model* m, int32_t on);

/* The same backward in two parts, so that a data-parallel caller can start the all-reduce of every
 * gradient except the MLP weights' while those are still being formed (bucketed all-reduce
 * overlapped with the weight-gradient GEMM): DFWFM_BWD_TABLES = the per-tile backward, the shallow
 * reductions and the table scatter (every gradient but lin_w / lin_b); DFWFM_BWD_MLP_WEIGHTS =
 * dW_l and db_l (reads what the first part saved).  Same results as dfwfm_backward when both run,
 * in this order, on one stream. */
#define DFWFM_BWD_TABLES 1
#define DFWFM_BWD_MLP_WEIGHTS 2
/* DFWFM_BWD_TABLES in two halves: the per-tile backward (TILES: dE, the G chain, per-tile partials) and what
 * sums over the batch (SPREAD: the shallow reductions' final sums and the table scatter).  SPREAD and
 * DFWFM_BWD_MLP_WEIGHTS both only read what TILES saved, so they may run concurrently on two streams. */
#define DFWFM_BWD_TILES 4
#define DFWFM_BWD_SPREAD 8
/* The two halves of DFWFM_BWD_SPREAD on their own: the shallow reductions' final sums, the table scatter. */
#define DFWFM_BWD_REDUCE 16
#define DFWFM_BWD_SCATTER 32
int dfwfm_backward_phases(dfwfm_model* m, const float* dlogit, const dfwfm_grads* grads, int32_t phases,
                          void* stream);

/* One tensor of an Adam step (device pointers; grad NULL = tensor skipped, as torch does). */
typedef struct {
  float* param;
  const float* grad;
  float* exp_avg;
  float* exp_avg_sq;
  int64_t numel;
} dfwfm_adam_tensor;

/* torch.optim.Adam(lr, betas, eps, weight_decay) step number `step` (1-based) over n tensors
 * (replaces optimizer.step(), :637).  The hyper-parameters are doubles, like the Python floats torch
 * derives its scalars from (bias corrections in double, then rounded to f32 per use).  Tensors must
 * not alias.  Needs no model: the list travels in the kernel arguments (no host synchronisation). */
int dfwfm_adam_step(const dfwfm_adam_tensor* tensors, int32_t n, double lr, double beta1, double beta2,
                    double eps, double weight_decay, int64_t step, void* stream);

/* ---- graph-replayable training step -------------------------------------------------------
 * A training step whose every launch reads its per-step scalars from device memory can be captured
 * once into a HIP graph and replayed (no host work per step).  The per-step state is one
 * caller-allocated, zero-initialised device block of DFWFM_ADAM_STATE_BYTES: an int64 step counter,
 * the last step's Adam scalars and a completion counter (zero between steps). */
#define DFWFM_ADAM_STATE_BYTES 48

/* From now on the dropout masks of dfwfm_train_forward / dfwfm_backward mix the device step counter
 * at `step_dev` (an int64 in such a state block; NULL restores host-only seeds) into their seed,
 * read when the kernels run -- so a replayed step draws fresh masks. */
int dfwfm_set_step_source(dfwfm_model* m, const int64_t* step_dev);

/* The training activations live in model-owned memory that dfwfm_train_forward grows on demand (a
 * larger batch frees and re-allocates it).  A captured graph bakes those pointers in: the generation
 * counter changes on every re-allocation, so a caller replaying a graph compares it with the value at
 * capture time and re-captures when it differs. */
int dfwfm_workspace_generation(const dfwfm_model* m, int64_t* gen);

/* dfwfm_adam_step with the step counter and bias corrections on the device: every workgroup derives the
 * scalars of step (counter + 1) there (double, then f32) and updates its tensors; the last workgroup of the
 * call's last launch advances the counter (no separate scalar launch). */
int dfwfm_adam_step_dev(const dfwfm_adam_tensor* tensors, int32_t n, double lr, double beta1, double beta2,
                        double eps, double weight_decay, void* state_dev, void* stream);

/* Gradient of binary_cross_entropy_with_logits (reference criterion, model/DeepFMs.py:561, :634) with
 * the summed loss divided by `denom` (the batch for reduction='mean'): dlogit[i] = (sigmoid(z_i) - y_i)
 * / denom.  When loss_sum is non-NULL the per-sample losses are added to *loss_sum. */
int dfwfm_bce_grad(const float* logits, const float* labels, int64_t n, double denom, float* dlogit,
                   float* loss_sum, void* stream);

/* dfwfm_bce_grad fused into dfwfm_backward_phases: the per-tile backward (phases must include
 * DFWFM_BWD_TILES or DFWFM_BWD_TABLES) forms dlogit from the training forward's logits and the labels with
 * dfwfm_bce_grad's arithmetic (the same dlogit bits), writes it to `dlogit` for the later phases and adds the
 * per-sample losses to *loss_sum (when non-NULL); one launch fewer per step.  A model without embeddings (no
 * per-tile backward) runs dfwfm_bce_grad then dfwfm_backward_phases.
 * The loss is summed like the dense gradients: each 16-row tile's loss is a per-tile partial that the REDUCE phase
 * (DFWFM_BWD_REDUCE, part of DFWFM_BWD_SPREAD / DFWFM_BWD_TABLES) adds in tile order, so *loss_sum is formed when
 * that phase runs -- in this call, or in a later dfwfm_backward_phases call on the same training forward (the
 * TILES-then-SPREAD split).  A caller that runs DFWFM_BWD_TILES and never runs REDUCE gets no loss. */
int dfwfm_backward_phases_bce(dfwfm_model* m, const float* logits, const float* labels, double denom, float* dlogit,
                              float* loss_sum, const dfwfm_grads* grads, int32_t phases, void* stream);

/* ---- touched-row gradients of the categorical tables (data-parallel exchange) --------------------
 * The reference's tables have dense gradients (nn.Embedding(sparse=False), model/DeepFMs.py:199-210) and
 * its Adam applies coupled L2 to every row (:553-556), so the data-parallel form of its step all-reduces
 * every table.  Only the rows a batch touched carry a data gradient: each rank builds the list of
 * (destination, summed gradient row) of the rows its batch touched, the ranks exchange the lists, every rank
 * adds all lists into its own dense gradient buffer (rank 0's first, then rank 1's, ...) and runs the dense
 * L2 + Adam step.  The lists are deterministic (stable sort, fixed-order sums, no atomics), so the replicas
 * stay bit-identical.
 *
 * A family is the second-order tables (fm_2nd_embeddings, rows of width D) or the first-order tables
 * (fm_1st_embeddings, width 1) of the categorical fields.  dest[f] (host array of field_size entries) holds
 * the float offset, in the caller's flat gradient buffer, of field f's plain / quotient table gradient (q)
 * and of its QR remainder table gradient (r); -1 leaves a table out (numerical fields are never listed: the
 * backward's reductions form their gradients).  The backward must have run with DFWFM_BWD_TABLES for the
 * last dfwfm_train_forward, with the categorical fields' gradient pointers NULL (no dense scatter); dlogit is
 * the one that backward got. */
#define DFWFM_FAMILY_SECOND 0
#define DFWFM_FAMILY_FIRST 1
typedef struct {
  int64_t q;
  int64_t r;
} dfwfm_sparse_dest;

/* Entries a batch of `batch` rows can produce (capacity = sum over the family's tables of min(batch, the
 * table's rows): one entry per distinct touched row) and their row width; *ws_bytes is always 0 (no workspace). */
int dfwfm_sparse_grads_size(dfwfm_model* m, int32_t family, int64_t batch, int64_t* capacity, int32_t* width,
                            int64_t* ws_bytes);
/* The list of the last training step, formed from the rank's OWN dense gradients of these tables: out_dest[e]
 * (device int64) = float offset of entry e's row in the flat buffer, out_rows[e * width ...] its summed gradient,
 * *out_count (device int32) the number of entries.  The backward (DFWFM_BWD_TABLES) scattered the tables into
 * `local` (local_floats floats, the tables at the `dest` offsets, zero elsewhere); every touched row is claimed once
 * through `stamp` (local_floats int32 of scratch, any contents: each call writes the stamps of exactly the rows it
 * reads back), copied to out_rows and cleared in `local` (zero again afterwards).  Entries come unsorted
 * (destinations unique), sums in atomic order: the replicas of a data-parallel step stay identical because every
 * rank applies the same bytes of every list.  No sort, no workspace; stream-ordered, graph-capturable. */
int dfwfm_sparse_grads_local(dfwfm_model* m, int32_t family, const dfwfm_sparse_dest* dest, int64_t capacity,
                             float* local, int32_t* stamp, int64_t local_floats, int64_t* out_dest, float* out_rows,
                             int32_t* out_count, void* stream);
/* grad[dest[e] + j] += rows[e * width + j] for e < *count (one list; lists with shared destinations must be
 * applied one after the other, in a fixed order, for bit-identical results). */
int dfwfm_sparse_grads_apply(float* grad, int32_t width, const int64_t* dest, const float* rows, const int32_t* count,
                             int64_t capacity, void* stream);

/* ---- magnitude pruning (reference model/DeepFMs.py:647-673, binary_search_threshold :807-823) ----
 * The threshold whose fraction of |x| < threshold (compared in f32) hits `target`, found by the
 * reference's own bisection on (0, 100) -- same rounds, same result -- resolved 12 rounds per pass over
 * the magnitudes (each pass histograms them against the 4095 mids the next 12 rounds can ask for)
 * instead of up to 101 passes with a host sync each; no sort.  Runs on `stream`; the threshold is
 * written to device memory (`thr_dev`, one double) and never read back by the library. */
typedef struct {
  const float* values;  /* device                                                                  */
  int64_t numel;
  int32_t sym_f;        /* 0: |values|; F > 0: values is F x F and the magnitudes are |(W + W^T)/2| */
  int32_t reserved;
} dfwfm_prune_source;

/* Device workspace bytes dfwfm_prune_threshold needs for `numel` magnitudes in total. */
int64_t dfwfm_prune_workspace_bytes(int64_t numel);
/* Threshold over the concatenation of n sources (e.g. all second-order tables, :652-656). */
int dfwfm_prune_threshold(const dfwfm_prune_source* sources, int32_t n, double target, double* thr_dev,
                          void* workspace, int64_t workspace_bytes, void* stream);
/* values[i] = 0 where the magnitude (as in the source) < threshold; sym_f > 0 zeroes W[k][l] where
 * |(W[k][l] + W[l][k]) / 2| < threshold, computed from the unmodified matrix (:666-670). */
int dfwfm_prune_apply(float* values, int64_t numel, int32_t sym_f, const double* thr_dev, void* stream);

/* ---- evaluation metrics (reference eval_by_batch, model/DeepFMs.py:777-800) --------------------
 * From logits z and labels y (device, n each): pred = sigmoid(z) in f32; writes 8 doubles to out_dev:
 * {roc_auc_score(y, pred), auc(precision_recall_curve), log_loss, RCE, CTR, positives, n, distinct
 * predictions}, the sklearn 1.7 definitions (ties grouped, [1-p, p] renormalised and clipped to the
 * float64 eps).  AUC is NaN when only one class is present (sklearn raises). */
int64_t dfwfm_metrics_workspace_bytes(int64_t n);
int dfwfm_eval_metrics(const float* logits, const float* labels, int64_t n, double* out_dev, void* workspace,
                       int64_t workspace_bytes, void* stream);

/* Synchronises `stream`, returns the sticky error-flag word and clears it. */
int dfwfm_read_error_flag(dfwfm_model* m, int32_t* flag, void* stream);

/* Diagnostics. */
const char* dfwfm_last_error(void);
/* With DFWFM_DIAG=stamps=1 in the environment, each forward records 16 shader-clock stamps per
 * 16-sample workgroup at its phase boundaries; copies up to n of them (synchronising `stream`)
 * and returns the number of workgroups copied, or a negative status. */
int dfwfm_diag_stamps(dfwfm_model* m, uint64_t* host, int64_t n, void* stream);
int dfwfm_abi_version(void);

#ifdef __cplusplus
}
#endif
#endif /* DFWFM_H */
