// dfwfm_internal.h -- types shared by the kernels and the C-ABI layer.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include <mutex>
#include <unordered_map>

#include "../../include/dfwfm.h"

namespace dfwfm {

constexpr int kBM = 16;     // samples per workgroup = one 16-row MFMA tile
constexpr int kMaxTPW = 8;  // MLP output tiles per wave group => deep_nodes <= 4*8*16 = 512
constexpr int kMaxMT = 4;   // FwFM row tiles => field_size <= 64
constexpr int kStampSlots = 16;  // diagnostic phase stamps per workgroup
constexpr int kTailC = 8;        // split tail tile: K chunks per wave (layer widths <= 4*8*16 = 512)
constexpr int kMaxPieces = kMaxMT * 32;  // FwFM work pieces (row tile m, column tile nt): MT * D

// flags
constexpr int kHasSecond = 1;  // FwFM / FM second order
constexpr int kHasDeep = 2;    // MLP
constexpr int kFoTables = 4;   // first order from fm_1st_embeddings
constexpr int kFoFwlw = 8;     // first order from fwfm_linear
constexpr int kFoLw = 16;      // project first order with fm_1st.weight
constexpr int kNeedE = 32;     // second-order / deep embeddings are gathered
constexpr int kTrain = 64;     // save the activations the backward needs (FwdArgs::sv_*)
constexpr int kDrop = 128;     // dropout on the deep tower (train only)
constexpr int kPrio = 256;     // raise the wave priority for the phases before the MLP (always on)
constexpr int kHasQR = 512;    // some field is a QR embedding (set by set_tables)
constexpr int kPrioEpi = 2048; // fwd32: raise the wave priority in the MLP epilogues too (set kernel)
constexpr int kDeferTail = 4096; // fwd32: the split tile's barrier moved into the next K loop (set kernel)
constexpr int kPairs = 1024;   // FwFM over the nonzero pairs of a pruned R (build_fwfm_pairs; MLP-free forward)
constexpr int kP3Pieces = 8192; // MLP-free forward: FwFM as U' E pieces (11.25 MFMAs per sample) instead of per-sample
                                // Gram tiles (18); set when MT <= 3
// bwd_kernel diagnostics / A/B (DFWFM_DIAG bwd=<bits> sets them << 20; off the flag range the model itself uses):
// no G_l stores (results invalid), no mask loads (results invalid), the generic K loop instead of the static form
constexpr int kBwdNoGStore = 1 << 20, kBwdNoMask = 1 << 21, kBwdGeneric = 1 << 22;
// ftrain_kernel diagnostics (DFWFM_DIAG ft=<bits> sets them << 23, results invalid): each wave's HW_ID into the stamp
// slots instead of clocks; the MLP waves skip their K loops
constexpr int kFtDiagHwId = 1 << 23, kFtDiagNoMlp = 1 << 24;
constexpr int kMaxH = 16;      // hidden layers
constexpr int kMaxSet = 32;    // batches per launch of dfwfm_forward_batches (the set is a kernel argument)

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
  const float* const* pk;  // dfwfm_model_pack_tables: per field, rows of pkw floats (emb2 row, emb1 weight, zero
  int32_t pkw;             // pad) for the categorical fields; pkw = 0: the plain tables (PART 3 reads it)
  const float* upack;  // FwFM A-operand fragments [MT][S][64]: strictly-upper (R + R^T)/2
  const int2* pairs;   // kPairs: the nonzero strictly-upper entries of (R + R^T)/2, (k | l << 16, w bits), k-major
  int32_t npairs;
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
  int32_t tail;        // 1: NT == 4*TPW + 1 and tile 4*TPW is split by K over the four waves
  int32_t ns;          // 25: every layer has 25 K chunks and 25 output tiles (static K loop), else 0
  int32_t flags;
  uint64_t* stamps;    // diagnostics only: [grid][kStampSlots] shader-clock stamps, normally null
  // training (flags & kTrain): activations kept for the backward
  float* sv_e;              // [B][F*D] E before dropout
  float* sv_fo;             // [B][F]   first order per field
  float* sv_x[kMaxH + 1];   // X_0 [B][F*D] (deep_emb after dropout), X_h [B][N] (layer h output after
                            // ReLU and dropout), h = 1..H
  float drop_p;             // dropout probability of the deep tower (kDrop)
  float drop_scale;         // 1 / (1 - p)
  uint32_t seed;            // dropout hash seed of this step
  const int64_t* seed_src;  // device step counter mixed into the seed (graph replay), or null
  int32_t* sv_keys;         // training: [F - num][keys_stride] the categorical indices, clamped, column-major (the
                            // sorted scatter's keys), or null
  int64_t keys_stride;
  // gather launch (PART 1; the sparse deep tower reads them) or dfwfm_forward_gather (PART 3)
  float* part_e;            // [B][part_stride] E tile rows (W0 columns, zero padded past F*D)
  float* part_fs;           // [B] first + second order
  int32_t part_stride;      // floats per row (W0, a multiple of 4)
  // FwFM second order: the pieces (row tile m, column tile nt) -> pc = m * D + nt each wave runs, for 4- and
  // 8-wave launches: wave w takes fw_list{4,8}[fw_off{4,8}[w] .. fw_off{4,8}[w + 1]) (balanced on the host)
  uint8_t fw_list4[kMaxPieces];
  uint8_t fw_list8[kMaxPieces];
  uint8_t fw_off4[5];
  uint8_t fw_off8[9];
  // batch set (dfwfm_forward_batches): nb > 1 -> workgroup w runs tile w % tiles of batch w / tiles, whose inputs
  // and logits are set_xi / set_xv / set_out[w / tiles] (every batch `batch` rows, the strides above); nb <= 1:
  // one batch at xi / xv / out
  int32_t nb;
  int32_t tiles;            // workgroups per batch
  const int64_t* set_xi[kMaxSet];
  const float* set_xv[kMaxSet];
  float* set_out[kMaxSet];
};

// workgroups of a forward launch with `rows` samples per workgroup
inline unsigned fwd_grid(const FwdArgs& a, int rows) {
  const unsigned tiles = (unsigned)((a.batch + rows - 1) / rows);
  return a.nb > 1 ? (unsigned)a.nb * tiles : tiles;
}

// Test and diagnostics options, all in ONE environment variable: DFWFM_DIAG="key=value,key=value", read where
// they apply (product runs set none).  Keys: r32 (0 never / 1 always the 32-sample set kernel), ng (4: four-wave
// forward / backward), ftrain (0: fwd_kernel<TRAIN> instead of the helper-wave training forward), part3 (0: the
// generic kernel for MLP-free models), p3ng (4 / 8: MLP-free waves), stamps / ring / ft / bwd / scatter /
// drop_flags (phase stamps and phase-skip bits; results invalid).  dflt when the key is absent.
inline int diag_opt(const char* key, int dflt) {
  const char* s = getenv("DFWFM_DIAG");
  const size_t kl = strlen(key);
  while (s && *s) {
    if (!strncmp(s, key, kl) && s[kl] == '=') return atoi(s + kl + 1);
    s = strchr(s, ',');
    if (s) ++s;
  }
  return dflt;
}

// LDS carve-up, in floats; every region starts 16-byte aligned.
struct LdsLayout {
  int desc, lw, fwlw, upk, bufX, bufY, red, tailr, fo, part2, dsum, fs, total;
};

__host__ __device__ inline int r4(int x) { return (x + 3) & ~3; }

// p3: the MLP-free forward (fwd_kernel PART 3): FwFM fragments read from global memory (no upk), fwlw only when
// that first order is used, one FwFM sum per sample -- 30.7 KB at Criteo-39 (42.3 KB generic), so five
// workgroups share a CU
__host__ __device__ inline LdsLayout lds_layout(int F, int D, int MT, int S, int SX, int SY, int TPW, int KS,
                                                bool deep, bool tail, int NG = 4, bool p3 = false, bool fwlw = true) {
  LdsLayout L;
  int o = 0;
  L.desc = o;  o += r4(14 * F);
  L.lw = o;    o += r4(F);
  L.fwlw = o;  o += (p3 && !fwlw) ? 0 : r4(F * D);
  L.upk = o;   o += p3 ? 0 : MT * S * 64;
  L.bufX = o;  o += kBM * SX;
  L.bufY = o;  o += deep ? kBM * SY : 0;
  L.red = o;   o += (deep && KS == 2) ? 4 * TPW * 64 * 4 : 0;
  L.tailr = o; o += (deep && tail) ? NG * 64 * 4 + 4 * kBM : 0;  // partials + per-(wave, row) deep sums of the tail
  L.fo = o;    o += kBM * r4(F);
  L.part2 = o; o += p3 ? kBM * D : MT * D * 16;  // per FwFM piece, its 16 column sums (p3: per sample / column)
  L.dsum = o;  o += p3 ? 0 : NG * kBM;
  L.fs = o;    o += kBM;
  L.total = r4(o);
  return L;
}

// Backward, per 16-sample tile (no atomics): dE of the shallow terms and of the MLP input (the
// dX_{l-1} = G_l W_l chain on MFMA), G_l saved for the weight-gradient GEMM, dE saved for the
// reductions and the table scatter.
struct BwdArgs {
  int64_t batch;
  const float* dlogit;           // [B] dL/dlogit (read unless bce_z is set)
  // BCE fused in (dfwfm_backward_phases_bce): dlogit formed from the logits bce_z and labels bce_y as
  // bce_grad_kernel does, written to bce_dl, the per-sample losses added to *loss_sum (when non-null)
  const float* bce_z;
  const float* bce_y;
  float* bce_dl;
  float* loss_sum;
  float bce_denom;
  const float* sv_e;             // [B][F*D]
  const float* sv_x[kMaxH + 1];  // X_0 .. X_H
  float* sv_g[kMaxH + 1];        // G_1 .. G_H written here ([B][N], dL/dz of each layer)
  float* sv_de;                  // [B][F*D] dL/dE written here
  const float* rsk;              // [MT][S][64] symmetric off-diagonal (R + R^T)/2 fragments (FM: ones)
  const float* fwlw;             // [F*D]
  const float* lw;               // [F]
  const float* fc;               // [NT*16]
  const float4* wtpack;          // transposed MLP packs: layer l block [KT_l][NT][64] float4
  int32_t wtpack_bytes;
  int32_t wt_off[kMaxH + 1];     // float4 offset of layer l's block (l = 1..H)
  int32_t F, H, N;
  int32_t NT, NC0, MT, S;
  int32_t SX, SY, W0;
  int32_t flags;
  float drop_p, drop_scale;
  uint32_t seed;
  const int64_t* seed_src;       // as FwdArgs::seed_src
  uint64_t* stamps;              // diagnostics only (DFWFM_DIAG stamps=2): phase clocks per workgroup
  // the dense shallow reductions fused in (red != 0): the tile's partial sums to part[blockIdx.x] in
  // reduce_kernel's layout (red_outputs), from the E / X_H / dE tiles already in LDS; reduce_final_kernel
  // adds them.  red: kRed* bits of the gradients wanted
  float* part;
  const float* sv_fo;            // [B][F]
  const float* xv;               // numerical values
  int64_t xv_stride;
  int32_t num;
  int32_t red;
};
constexpr int kRedOn = 1, kRedLw = 2, kRedFwlw = 4, kRedR = 8, kRedFc = 16, kRedNum2 = 32, kRedNum1 = 64;

// Batch reductions of the dense shallow parameters, per 16-row tile then summed over tiles:
// bias, fm_1st (lw), fwfm_linear, field_cov (Gram on MFMA), net_1_fc, numerical-field tables.
struct RedArgs {
  int64_t batch;
  const float* dlogit;
  const float* sv_e;             // [B][F*D]
  const float* sv_fo;            // [B][F]
  const float* sv_de;            // [B][F*D]
  const float* x_h;              // [B][N] last hidden layer output (net_1_fc input) or null
  const float* xv;               // numerical values
  int64_t xv_stride;
  const float* lw;               // [F] (kFoLw)
  float* g_bias;
  float* g_lw;
  float* g_fwlw;
  float* g_R;
  float* g_fc;
  float* g_num2[64];             // numerical field f: d v_f [D]
  float* g_num1[64];             // numerical field f: d w1_f [1]
  float* part;                   // [ceil(B/16)][red_outputs] per-tile partial sums (no atomics)
  float* loss_sum;               // the per-tile BCE sums (last slot, the fused backward with the loss gradient) or null
  int32_t F, D, num, N, MT;
  int32_t flags;
};
// packed per-block outputs of the reduction: bias | lw[F] | fwlw[F*D] | R[F*F] | fc[N] | num2[num*D] | num1[num] |
// the tile's loss (summed into loss_sum in tile order, like the gradients: the same bits on every run)
__host__ __device__ inline int red_outputs(int F, int D, int N, int num) {
  return 1 + F + F * D + F * F + N + num * D + num + 1;
}

// Embedding-table scatter: one task per (categorical field, table) with dense grads.  Tables of at
// most kPrivRows*w floats accumulate in LDS inside one workgroup (no global contention: a field
// with 4 categories receives every sample); larger tables take global atomics, lane per element.
constexpr int kPrivFloats = 24 * 1024;  // LDS of a privatised task: rows * (w + 1) (sums + row flags)
constexpr int64_t kPrivRows = 128;       // row bound of a privatised task: measured best (step 0.380 -> 0.370 ms)
struct ScatterTask {
  float* g;             // grad of this table
  const float* other;   // QR mult: the partner table whose row multiplies the gradient (else null)
  int32_t c;            // QR collisions (kind 1, 2)
  int16_t field;        // model field index
  int8_t kind;          // 0 plain row idx, 1 quotient row idx / c, 2 remainder row idx % c; | kScatterPriv
  int8_t src;           // 0: dE[b, f, :] (row width D), 1: dfo[b, f] = dlogit * (lw[f] or 1) (width 1)
  int32_t rows;         // table rows
  int32_t block0;       // first workgroup of the task in its launch
};
static_assert(sizeof(ScatterTask) == 32, "scatter task layout");
constexpr int kScatterPriv = 64;  // ScatterTask::kind flag: a privatised (LDS-accumulated) task
constexpr int kScatterList = 96;  // tasks per launch: the list is a kernel argument (< 4 KiB)
struct ScatterArgs {
  ScatterTask t[kScatterList];
  int32_t ntasks;
  int32_t D, F, num;
  const FieldDev* fields;
  const int64_t* xi;
  int64_t xi_stride;
  int64_t batch;
  const float* sv_de;
  const float* dlogit;
  const float* lw;      // [F] or null (dfo = dlogit)
  int32_t chunk;        // samples per workgroup of a non-privatised task
};

// Deterministic table scatter (sort_scatter_kernel): one task per (categorical field, row kind) -- the rows a
// field's samples hit in its plain table, or its QR quotient / remainder table -- covering both table families
// (second order, width D; first order, width 1).  A workgroup sorts the batch's (row, sample) keys in LDS and sums
// every row's contributions in a fixed order, so the gradients are the same bits on every run.
constexpr int kSortSeg = 4096;      // samples sorted per pass (larger batches: passes in sample order)
constexpr int kSortCh = 16;         // sorted positions per chunk of the segmented sums
constexpr int kSortThreads = 1024;
struct SortScatterTask {
  float* g2;            // second-order table grad (width D) or null
  float* g1;            // first-order table grad (width 1) or null
  const float* o2;      // QR mult: the partner second-order table (its row multiplies the gradient) or null
  const float* o1;      // QR mult: the partner first-order table or null
  int32_t c;            // QR collisions (kind 1, 2)
  int16_t field;        // model field index
  int8_t kind;          // 0 plain row idx, 1 quotient row idx / c, 2 remainder row idx % c
  int8_t pad8;
  int32_t block0;       // the task's first workgroup
  int16_t nbuck;        // row buckets (row % nbuck), one workgroup each
  int16_t onerow;       // nbuck == rows: every bucket holds one row (no sort needed)
};
static_assert(sizeof(SortScatterTask) == 48, "sort scatter task layout");
constexpr int kSortScatterList = 64;  // tasks per launch (the list is a kernel argument, < 4 KiB)
struct SortScatterArgs {
  SortScatterTask t[kSortScatterList];
  int32_t ntasks;
  int32_t D, F, num;
  const FieldDev* fields;
  const int64_t* xi;
  int64_t xi_stride;
  int64_t batch;
  const float* sv_de;
  const float* dlogit;
  const float* lw;      // [F] or null (dfo = dlogit)
  const int32_t* keys;  // the training forward's clamped categorical indices [F - num][keys_stride] or null (xi)
  int64_t keys_stride;  // a multiple of 4
  int32_t key64;        // 1: some task's buckets reach 2^20 rows (64-bit sort keys)
  int32_t diag;         // diagnostics only (DFWFM_DIAG scatter=): 1 skip the sort, 2 skip the sums, 4 no row adds,
                        // 8 empty, 16 key loads only, 32 every position reads one sample
  uint64_t* stamps;     // diagnostics only (DFWFM_DIAG stamps=3): phase clocks per workgroup, normally null
};
// a task's sort keys are (row / nbuck) << 12 | sample in 32 bits when every bucket's rows stay under 2^20, else 64
constexpr int kSortKey32Rows = 1 << 20;
size_t sort_scatter_lds_bytes(int D);

// Touched-row gradients of one table family (dfwfm_sparse.hip): one task per categorical table.
struct SparseTask {
  const float* other;   // unused (kept for the 24-byte layout)
  int64_t dest;         // float offset of this table's gradient in the caller's flat buffer
  int32_t c;            // QR collisions (kind 1, 2)
  int16_t field;        // model field index
  int8_t kind;          // 0 plain row idx, 1 quotient row idx / c, 2 remainder row idx % c
  int8_t pad_;
};
static_assert(sizeof(SparseTask) == 24, "sparse task layout");
constexpr int kSparseTasks = 128;  // 2 tables x 64 fields; the list is a kernel argument (< 4 KiB)
struct SparseArgs {
  SparseTask t[kSparseTasks];
  int32_t ntasks;
  int32_t D, F, num;
  int32_t w;            // row width of the family: D (second-order tables) or 1 (first-order tables)
  const FieldDev* fields;
  const int64_t* xi;
  int64_t xi_stride;
  int64_t batch;
};
hipError_t launch_sparse_apply(float* grad, int w, const int64_t* dest, const float* rows, const int32_t* count,
                               int64_t cap, hipStream_t s);
hipError_t launch_sparse_local(const SparseArgs& a, float* local, int32_t* stamp, int64_t cap, int64_t* out_dest,
                               float* out_rows, int32_t* out_count, hipStream_t s);

// Sparse deep tower (dfwfm_spmlp.hip): per layer, neurons in groups of four; a group's slot holds its rows'
// nonzero (k, w bits) pairs in k order, interleaved [entry j][neuron u], padded with (0, 0) to the
// group's longest row rounded up to kEllPad; slot capacity W[l] entries per row.
constexpr int kEllPad = 8;
struct EllArgs {
  const float* w[kMaxH];   // nn.Linear weights [N][K_l], row-major (the caller's tensors)
  int32_t K[kMaxH];
  int32_t W[kMaxH];        // entries per row of layer l (>= K_l, multiple of kEllPad)
  int64_t off[kMaxH];      // first entry of layer l
  int2* ell;
  int32_t* cnt;            // [H][N] nonzeros per row
  int32_t* gcnt;           // [H][ceil(N/4)] padded entries per group
  int32_t* stat;           // [2]: max row count, total nonzeros (atomics; zeroed by the caller)
  int32_t N, H;
};
struct SpMlpArgs {
  const float* part_e;     // [B][part_stride] E rows of the gather launch (zero padded past F*D)
  const float* part_fs;    // [B] first + second order
  int32_t part_stride, K0p;  // K0p = columns of part_e the first layer may read (part_stride)
  const int2* ell;
  const int32_t* gcnt;     // [H][ceil(N/4)]
  int32_t W[kMaxH];
  int64_t off[kMaxH];
  const float* mlp_b;      // [H][NT*16] padded biases
  const float* fc;         // [NT*16]
  const float* bias;       // [1]
  float* out;
  int64_t batch;
  int32_t H, N, NT;
  int32_t ecap;            // ELL entries per LDS staging unit (set by the launcher)
};
hipError_t launch_ell_build(const EllArgs& a, int rows, hipStream_t s);
hipError_t launch_sparse_mlp(const SpMlpArgs& a, hipStream_t s);
size_t sparse_mlp_lds_bytes(int K0p, int N);

// dW_l += G_l^T X_{l-1} and db_l += sum_b G_l for every layer in one launch.
struct DwArgs {
  const float* G[kMaxH + 1];
  const float* X[kMaxH + 1];
  float* gW[kMaxH + 1];
  float* gB[kMaxH + 1];
  int32_t K[kMaxH + 1];          // input width of layer l
  int32_t ldx[kMaxH + 1];        // row stride of X_{l-1} (multiple of 4)
  int32_t blk0[kMaxH + 2];       // first workgroup of layer l (prefix over layers)
  int32_t nkb[kMaxH + 1];        // 80-wide K blocks of layer l
  int32_t H, N, nnb, splits;
  int64_t batch;
  int64_t rows_per_split;
  // deterministic split-K (splits > 1): per (block, split) slices of the 80 x 80 block and of db, added in split
  // order by dw_sum_kernel; see dwr_block
  float* part;
  float* bpart;
  int32_t xcd_gs;       // dwr_reduce_kernel: blocks per XCD-local group (0: blockIdx order), and the groups
  int32_t xcd_groups;
};

// One tensor of a fused Adam step.
struct AdamTensor {
  float* p;
  const float* g;
  float* m;
  float* v;
  int64_t n;
};
constexpr int kAdamBlock = 4096;  // elements per Adam work unit (16 per thread: four float4 of each array in flight)
constexpr int kAdamList = 91;    // tensors per Adam launch (the list is a kernel argument, < 4 KiB)
struct AdamList {
  AdamTensor t[kAdamList];
  int32_t block0[kAdamList];     // first workgroup of each tensor
  int32_t n;
};
static_assert(sizeof(AdamList) + 64 <= 4096, "Adam launch arguments over 4 KiB");

// Raises a kernel's dynamic-LDS limit when a launch needs more than previously granted.  Done once
// per kernel and size, not per launch, so launches recorded into a HIP graph make no attribute calls.
inline hipError_t ensure_lds_limit(const void* fn, size_t lds) {
  if (lds <= 65536) return hipSuccess;
  static std::mutex mu;
  static std::unordered_map<const void*, size_t> granted;
  std::lock_guard<std::mutex> g(mu);
  size_t& cur = granted[fn];
  if (lds <= cur) return hipSuccess;
  hipError_t e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  if (e == hipSuccess) cur = lds;
  return e;
}

// One packing job of set_dense (see pack_dense_kernel).
enum PackType : int32_t { kPackPad = 0, kPackLinear = 1, kPackLinearT = 2, kPackFwfm = 3, kPackFwfmSym = 4, kPackZero = 5 };
constexpr int kPackZeroPT = 16;  // kPackZero: float4 written per thread (a job element = kPackZeroPT float4)
struct PackJob {
  const float* src;
  float* dst;
  int64_t total;    // elements (float or float4) written
  int32_t type;
  int32_t a, b, d;  // pad: n (valid), -, -; linear: N, K, NC; fwfm: F, mode, S
  int32_t block0;
  int32_t pad_;
};
constexpr int kPackList = 56;  // 3 per hidden layer (kMaxH = 16) + 6; the list is a kernel argument (< 4 KiB)
struct PackList {
  PackJob j[kPackList];
  int32_t n;
};

// Pruning sources: magnitudes of p (sym_f > 0: of (W + W^T)/2 for an F x F matrix) at keys[offset..]
struct PruneSrc {
  const float* p;
  int64_t numel;
  int64_t offset;
  int32_t sym_f;
  int32_t pad_;
};
constexpr int kMaxPruneSrc = 96;  // the list is a kernel argument (< 4 KiB)
struct PruneList {
  PruneSrc s[kMaxPruneSrc];
  int32_t n;
};
size_t prune_workspace_bytes(int64_t n);
hipError_t launch_prune_threshold(const PruneList& L, double target, double* d_thr, void* ws, size_t ws_bytes,
                                  hipStream_t s);
hipError_t launch_prune_apply(float* p, int64_t numel, int sym_f, const double* d_thr, hipStream_t s);

size_t metrics_workspace_bytes(int64_t n);
hipError_t launch_metrics(const float* z, const float* y, int64_t n, double* out, void* ws, size_t ws_bytes,
                          hipStream_t s);

bool supported_embedding_size(int D);
hipError_t launch_forward(const FwdArgs& a, int D, int tpw, int ks, int ng, size_t lds, hipStream_t s);

// dfwfm_model_pack_tables: the categorical fields' (emb2 row | emb1 weight | zero pad) serving rows, one launch
constexpr int kPackTabList = 64;
struct PackTabList {
  const float* emb2[kPackTabList];
  const float* emb1[kPackTabList];
  float* dst[kPackTabList];
  int64_t n[kPackTabList];
  int32_t blk0[kPackTabList + 1];  // first workgroup of each field (256 rows per workgroup)
  int32_t nf, D, pkw;
};
hipError_t launch_pack_tables(const PackTabList& L, hipStream_t s);
// the gather + shallow part alone (-> a.part_e / a.part_fs): the sparse deep tower's first launch
hipError_t launch_forward_gather(const FwdArgs& a, int D, size_t lds1, hipStream_t s);
hipError_t launch_pack_list(const PackList& L, int total_blocks, hipStream_t s);
// the fused inference forward on 32-sample workgroups (dfwfm_fwd32.hip): both 16-row tiles per wave in the MLP;
// the static 3x400 form only (fwd32_supported), bit-identical logits to fwd_kernel's
bool fwd32_supported(int F, int D, int H, int NT, int NC0, int tailI, int NG);
size_t fwd32_lds_bytes(int F, int D, int MT, int S, int SX);
hipError_t launch_fwd32(const FwdArgs& a, int D, size_t lds, hipStream_t s);
// the training forward with helper waves (dfwfm_ftrain.hip): the static 3x400 form only (ftrain_supported); logits
// and saved activations bit-identical to fwd_kernel<TRAIN>'s
bool ftrain_supported(int F, int D, int H, int NT, int NC0, int tailI, int NG);
size_t ftrain_lds_bytes(int F, int D, int MT, int S, int SX, int SY);
hipError_t launch_ftrain(const FwdArgs& a, int D, size_t lds, hipStream_t s);
// per-embedding-size launchers, each compiled in its own translation unit (-DDFWFM_KD=<D>)
#define DFWFM_PER_D_CAT2(a, b) a##b
#define DFWFM_PER_D_CAT(a, b) DFWFM_PER_D_CAT2(a, b)
#define DFWFM_PER_D(name) DFWFM_PER_D_CAT(name, DFWFM_KD)
#define DFWFM_DECL_PER_D(D)                                                                                   \
  hipError_t launch_forward_d##D(const FwdArgs& a, int tpw, int ks, int ng, size_t lds, hipStream_t s);        \
  hipError_t launch_forward_gather_d##D(const FwdArgs& a, size_t lds1, hipStream_t s);                      \
  hipError_t launch_backward_d##D(const BwdArgs& a, int tpw, int ng, size_t lds, hipStream_t s);
DFWFM_DECL_PER_D(4)
DFWFM_DECL_PER_D(8)
DFWFM_DECL_PER_D(10)
DFWFM_DECL_PER_D(16)
DFWFM_DECL_PER_D(32)
hipError_t launch_backward(const BwdArgs& a, int D, int tpw, int ng, size_t lds, hipStream_t s);
size_t backward_lds_bytes(int F, int D, int MT, int S, int SX, int SY);
// the register-direct dwr_kernel: 80 x 80 blocks (nnb, nkb), batch splits of a multiple of kDwRows rows
hipError_t launch_dw(const DwArgs& a, int total_blocks, hipStream_t s);
// launch_dw with reduce_final's workgroups appended to the same grid (one launch for both)
hipError_t launch_dw_reduce(const DwArgs& a, int total_blocks, const RedArgs& r, hipStream_t s);
constexpr int kDwEdge = 80;
constexpr int kDwRows = 64;  // four waves x whole groups of four four-row k-steps
hipError_t launch_reduce(const RedArgs& a, hipStream_t s);  // both stages
hipError_t launch_reduce_final(const RedArgs& a, hipStream_t s);  // the second stage only (bwd_kernel red)
// privatised (kind | kScatterPriv) and global-atomic tasks in one launch
hipError_t launch_scatter(const ScatterArgs& a, int total_blocks, hipStream_t s);
hipError_t launch_sort_scatter(const SortScatterArgs& a, int total_blocks, hipStream_t s);
hipError_t launch_adam(const AdamList& list, int total_blocks, float step_size, float omb1, float b2, float omb2,
                       float eps, float wd, float bc2_sqrt, hipStream_t s);
// device-side step: state = {int64 step; float step_size, omb1, b2, omb2, eps, wd, bc2_sqrt}
struct AdamDevState {
  int64_t step;
  float step_size, omb1, b2, omb2, eps, wd, bc2_sqrt;  // the last step's scalars (diagnostics)
  int32_t ticket;                                       // workgroups done in the step's last launch
  int32_t pad[2];
};
constexpr int kAdamGrid = 2048;  // workgroups of a device-counter Adam launch (8 per CU), walking the blocks
struct AdamHyper {
  double lr, b1, b2, eps, wd;
};
// one launch of a device-counter Adam step: every workgroup derives the scalars of step (counter + 1); with `bump`
// (the step's last launch) the last workgroup to finish advances the counter
hipError_t launch_adam_dev(const AdamList& list, int total_blocks, AdamDevState* st, const AdamHyper& h, bool bump,
                           hipStream_t s);
hipError_t launch_bce_grad(const float* z, const float* y, int64_t n, float denom, float* dz, float* loss_sum,
                           hipStream_t s);

}  // namespace dfwfm
