// dfwfm_kernels.hip -- CDNA4 (gfx950) kernels for the DeepFwFM forward.
//
// One fused launch computes the whole forward of reference
// model/DeepFMs.py:285-469 for a tile of kBM = 16 samples:
//
//   phase 0  stage the 39 field descriptors, lw, fwlw and the FwFM operand
//            fragments in LDS; issue the tile's Xi / Xv loads;
//   phase G  gather: 26 categorical rows (plain nn.Embedding / EmbeddingBag,
//            or QR quotient (*|+) remainder, model/QREmbeddingBag.py:156-174)
//            and 13 numerical rows v_f[0] * Xv (model/DeepFMs.py:297-299,334)
//            into an LDS tile E[16][F*D] -- this IS deep_emb (the field-major
//            `cat` of :398) and the `stack` of :337; all of a thread's row
//            loads are issued before any is consumed;
//   phase S  first order (per-field tables :304, or fwlw :338-347) projected
//            by lw (:445-450) or summed; FwFM second order (:352-367) on f32
//            MFMA as  second[b] = sum_{k,d} E[b,k,d] * (U E_b)[k,d]  with U the
//            strictly upper triangle of (R + R^T)/2 -- no [39,39,B,10]
//            intermediates, and R's zero blocks skipped;
//   phase M  the h_depth x N ReLU MLP (:412-428) on f32 MFMA
//            (v_mfma_f32_16x16x4_f32, exact f32 fma chain): activations stay
//            in LDS, weights stream from L2 in a pre-packed fragment order
//            (one 1 KiB dwordx4 load per wave per 16-deep K chunk per output
//            tile), next chunk's loads pinned ahead of the current chunk's
//            MFMAs; with KS = 2 two waves per SIMD split K (even / odd chunks)
//            and reduce through LDS; bias+ReLU fused into the epilogue,
//            net_1_fc fused into the last layer's epilogue;
//   combine  total = ((first + second) + deep) + bias   (:458 order).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>

#include <type_traits>

#include "dfwfm_device.h"
#include "dfwfm_internal.h"

namespace dfwfm {

// ---------------------------------------------------------------------------
// the fused forward kernel
// ---------------------------------------------------------------------------
// TRAIN: the training-step variant (activations saved, dropout); compiled separately so the inference
// kernel carries none of it
#ifndef DFWFM_FWD_WPE
#define DFWFM_FWD_WPE 2  // register budget of two waves per SIMD (<= 256 per lane): a second batch's
                         // workgroup fits beside this one (stream-level overlap)
#endif
#ifndef DFWFM_P3_WPE
#define DFWFM_P3_WPE 6  // MLP-free forward on eight waves: six waves per SIMD (<= 80 registers): three workgroups per CU
#endif
#ifndef DFWFM_P3_DIRECT_DESC
#define DFWFM_P3_DIRECT_DESC 1  // MLP-free forward without QR: row descriptors from global, no staging barrier
#endif
#ifndef DFWFM_DIRECT_DESC_DEEP
#define DFWFM_DIRECT_DESC_DEEP 1  // the fused forward (static 3x400 form) without QR: the same direct descriptors
#endif
#ifndef DFWFM_P3_WPE4
#define DFWFM_P3_WPE4 5  // MLP-free forward on four waves: five waves per SIMD (<= 96 registers): five workgroups
                         // per CU (LDS 30.7 KB each at Criteo-39)
#endif
// PART: 0 = the whole forward in one launch; 1 = stage, gather and shallow part only, E tile and
// first + second to p.part_e / p.part_fs (the sparse deep tower's first launch); 3 = a model without deep tower
// (no MLP code, trimmed LDS, FwFM fragments read from global memory: 70 registers on eight waves; with
// p.part_e set, dfwfm_forward_gather: E tile and first + second out instead of the logit).  (PART 2, the MLP
// half of the split forward, was removed in round 6 with that forward.)
// NG: MLP output-tile groups = waves (4: one wave per SIMD, <= 256 registers; 8: two per SIMD, <= 128
// registers, so one workgroup issues MFMAs from two waves per SIMD while a second batch's workgroup
// on the same CU runs its gather; the training variant, one batch in flight, keeps 256 registers)
// NS: every layer has NS K chunks and NS output tiles (0: any) -- the K loop is then fully static and the
// split tail tile rides on its register sets (mlp_k_loop_s)
// QR: some field may be a QR embedding (false: the gather carries no second operand and loads its row descriptors
// directly -- PART 3, and PART 0's static form)
template <int D, int TPW, int KS, bool TRAIN, int PART, int NG, int NS, bool QR = true>
__global__ void __launch_bounds__(64 * NG * KS)
__attribute__((amdgpu_waves_per_eu(PART == 1 ? 3 : (PART == 3 ? (NG == 4 ? DFWFM_P3_WPE4 : DFWFM_P3_WPE)
                                                               : (NG == 8 ? (TRAIN ? 2 : 4) : DFWFM_FWD_WPE)))))
fwd_kernel(FwdArgs p) {
  static_assert(NG == 4 || (NG == 8 && KS == 1), "8 tile groups: no K split");
  constexpr int NTH = 64 * NG * KS;
  constexpr int NW = NG * KS;
  constexpr int RPT = (kBM * 64 + NTH - 1) / NTH;  // gather rows per thread (F <= 64)
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);  // provably wave-uniform (SGPR)
  const int F = p.F;
  const int num = p.num;
  const int SX = p.SX;
  const int SY = p.SY;
  const int flags = p.flags;
  const bool deep = PART != 1 && PART != 3 && (flags & kHasDeep) != 0;  // the MLP runs in this launch
  const int Fp = r4(F);
  const bool tail = KS == 1 && p.tail != 0;
  const LdsLayout L = lds_layout(F, D, p.MT, p.S, SX, SY, TPW, KS, deep, tail, NG, PART == 3,
                                 (flags & kFoFwlw) != 0);  // PART 1: no MLP buffers; PART 3: trimmed
  FieldDev* desc = reinterpret_cast<FieldDev*>(smem + L.desc);
  float* lw_s = smem + L.lw;
  float* fwlw_s = smem + L.fwlw;
  float* upk = smem + L.upk;
  float* bufX = smem + L.bufX;
  float* bufY = smem + L.bufY;
  f32x4* red = reinterpret_cast<f32x4*>(smem + L.red);
  float* tailr = smem + L.tailr;  // [4 waves][64 lanes][4] partial products of the tail tile
  float* fo = smem + L.fo;
  float* part2 = smem + L.part2;
  float* dsum = smem + L.dsum;
  float* fs = smem + L.fs;

  const TileRef tr = tile_ref<kBM>(p);  // batch set: this workgroup's batch
  const int64_t b0 = tr.b0;
  stamp(p.stamps, 0, tid);
  stamp_start_rt(p.stamps, tid);
  // gather / shallow phases at a raised priority: beside a co-resident workgroup's MLP they would otherwise
  // lose every issue arbitration (A/B switch, kPrio)
  if (flags & kPrio) __builtin_amdgcn_s_setprio(1);
  const int g = wave & (NG - 1);  // MLP output-tile group
  const int kh = wave / NG;       // MLP K half (KS == 2)

  LayerStream<TPW, KS, NG> ls;
  // weight fragments: three register sets, prefetch distance 2 chunks (a fourth set / distance 3
  // measured slower)
  f32x4 wb0[TPW], wb1[TPW], wb2[TPW];
#define DFWFM_PRELOAD(LS) (LS).preload(wb0, wb1, lane * 16)
#define DFWFM_KLOOP(ACC, IN, SA, LS) mlp_k_loop<TPW, KS, NG>(ACC, IN, SA, LS, wb0, wb1, wb2, lane)
  const __amdgpu_buffer_rsrc_t wrsrc = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<float4*>(p.wpack), (short)0, p.wpack_bytes, 0x00020000);
  // biases [H][NT*16] and net_1_fc [NT*16] (padded, so every tile's lanes are in range)
  const __amdgpu_buffer_rsrc_t brsrc = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<float*>(p.mlp_b), (short)0, p.H * p.NT * 16 * 4, 0x00020000);
  const __amdgpu_buffer_rsrc_t frsrc = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<float*>(p.fc), (short)0, p.NT * 16 * 4, 0x00020000);
  TailStream<NG> ts;
  // NS is the MLP's static K-chunk count, except in the MLP-free PART 3, where it is the FwFM row-tile count
  constexpr int NSK = PART == 3 ? 0 : NS;
  f32x4 tw[NSK ? 1 : TailStream<NG>::C];  // preloaded tail fragments (NSK == 0)
  constexpr int TT = NG * TPW;  // the tail tile (when p.tail)

  constexpr bool train = TRAIN;
  const int FD = F * D;
  const int SE = r4(FD);  // row stride of the saved E / X_0 tiles
  const int nrows = (int)((p.batch - b0) < kBM ? (p.batch - b0) : kBM);
  const bool drop0 = train && deep && (flags & kDrop) != 0;
  {
  // ---- phase 0: field descriptors -> LDS; this thread's Xi / Xv; shallow parameters in flight --
  // Every load is issued before any is consumed (a load-then-store loop waits one round trip per
  // iteration).  Only the descriptors and the tile's Xi / Xv gate the gather; the FwFM fragments,
  // lw and fwlw are stored to LDS after the gather's loads are out.
  constexpr int kDescPT = (7 * 64 + NTH - 1) / NTH;    // uint2 words of descriptors per thread
  constexpr int kUpkPT = (kMaxMT * 16 * 16 + NTH - 1) / NTH;  // float4 of FwFM fragments per thread
  constexpr int kFwlwPT = (64 * 32 + NTH - 1) / NTH;   // fwlw floats per thread
  // ext-vector element types throughout: HIP's uint2 / float4 are unions, which keeps these arrays out
  // of registers (scratch, and a vmcnt(0) at every spill point)
  typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
  // PART 3 without QR fields: each thread loads its rows' descriptor fields (table bases, row count) from
  // global memory with its keys -- no LDS staging and no barrier before the gather
  constexpr bool kDirectDesc = !QR && ((DFWFM_P3_DIRECT_DESC && PART == 3) || (DFWFM_DIRECT_DESC_DEEP && PART == 0));
  u32x2 dw[kDirectDesc ? 1 : kDescPT];
  const float* rd_emb2[kDirectDesc ? RPT : 1];
  const float* rd_emb1[kDirectDesc ? RPT : 1];
  int64_t rd_n[kDirectDesc ? RPT : 1];
  // the inference forward with the serving copy (dfwfm_model_pack_tables): a categorical row and its first-order
  // weight are ONE row of pkw floats
  constexpr bool kPackable = (PART == 3 || (PART == 0 && !TRAIN)) && !QR && kDirectDesc;
  bool pkrow[kPackable ? RPT : 1];
  if constexpr (kDirectDesc) {
#pragma unroll
    for (int k = 0; k < RPT; ++k) {
      const int f = (tid + k * NTH) >> 4;
      rd_emb2[k] = rd_emb1[k] = nullptr;
      rd_n[k] = 0;
      if constexpr (kPackable) pkrow[k] = p.pkw != 0 && f >= num && f < F;
      if (f < F) {
        rd_emb2[k] = (kPackable && pkrow[kPackable ? k : 0]) ? p.pk[f] : p.fields[f].emb2;
        rd_emb1[k] = p.fields[f].emb1;
        rd_n[k] = p.fields[f].n;
      }
    }
  } else {
#pragma unroll
    for (int k = 0; k < kDescPT; ++k) {
      const int i = tid + k * NTH;
      if (i < 7 * F) dw[k] = reinterpret_cast<const u32x2*>(p.fields)[i];
    }
  }
  int64_t key[RPT];  // gather row r -> field f = r / 16, sample b = r % 16: index or Xv bits
#pragma unroll
  for (int k = 0; k < RPT; ++k) {
    const int r = tid + k * NTH;
    const int f = r >> 4;
    const int64_t gb = b0 + (r & 15);
    key[k] = 0;
    if (f < F && gb < p.batch) {
      if (f < num)
        key[k] = __float_as_int(tr.xv[gb * p.xv_stride + f]);
      else
        key[k] = tr.xi[gb * p.xi_stride + (f - num)];
    }
  }
  f32x4 uw[kUpkPT];
  const int n_upk = (PART != 3 && (flags & kHasSecond)) ? p.MT * p.S * 16 : 0;  // PART 3 reads them from global
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
  if constexpr (!kDirectDesc) {
#pragma unroll
    for (int k = 0; k < kDescPT; ++k) {
      const int i = tid + k * NTH;
      if (i < 7 * F) reinterpret_cast<u32x2*>(desc)[i] = dw[k];
    }
    __syncthreads();
  }
  stamp(p.stamps, 1, tid);

  // PART 3: this lane's U' entries of every upper Gram tile (the same for every sample), loaded from the packed
  // A fragments in global memory (L2) behind the gather's row loads: lane holds
  // G[16m + 4(lane>>4) + r][16n + (lane&15)], and U'[k][l] sits in the pack at [(k/16) S + l/4][(k%16) + 16 (l%4)]
  constexpr int P3_MTC = NS > 0 ? NS : kMaxMT;  // row tiles (PART 3 instantiates NS = MT: no idle registers)
  constexpr int P3_NTL = PART == 3 ? P3_MTC * (P3_MTC + 1) / 2 : 1;  // upper tiles (m <= n)
  // the U'E pieces form (kP3Pieces) while its U' fragments fit the eight-wave form's 80 registers (MT <= 3; the host
  // asks for pieces only then, so a batch set and a lone batch take the same form: the same bits)
  constexpr bool kPieces = PART == 3 && P3_MTC <= 3;
  float uu[P3_NTL][4];
  auto load_uu = [&]() {
    if constexpr (PART == 3) {
      const float* up = p.upack;
      const int MT = p.MT, S = p.S;
#pragma unroll
      for (int m = 0, t = 0; m < P3_MTC; ++m)
#pragma unroll
        for (int n = m; n < P3_MTC; ++n, ++t) {
          const int l = 16 * n + (lane & 15);
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int k = 16 * m + 4 * (lane >> 4) + r;
            uu[t][r] = ((flags & kHasSecond) && n < MT && l < 4 * S)
                           ? up[((k >> 4) * S + (l >> 2)) * 64 + (k & 15) + 16 * (l & 3)] : 0.f;
          }
        }
    }
  };

  // ---- phase G: gather E rows and table first order --------------------------
  {
    const bool needE = (flags & kNeedE) != 0;
    const bool fo_tab = (flags & kFoTables) != 0;
    const float* pa[RPT];
    constexpr int RQ = QR ? RPT : 1;  // QR second operands
    const float* pb[RQ];
    const float* qa[RPT];
    const float* qb[RQ];
    float scale[RPT];
    int mode[RPT];
    bool live[RPT];
#pragma unroll
    for (int k = 0; k < RPT; ++k) {
      const int r = tid + k * NTH;
      const int f = r >> 4;
      live[k] = f < F && (b0 + (r & 15)) < p.batch;
      pa[k] = qa[k] = nullptr;
      if constexpr (QR) pb[k] = qb[k] = nullptr;
      scale[k] = 1.f;
      mode[k] = 0;
      if (kDirectDesc && live[k]) {
        if (f < num) {
          scale[k] = __int_as_float((int)key[k]);
          pa[k] = rd_emb2[kDirectDesc ? k : 0];
          qa[k] = rd_emb1[kDirectDesc ? k : 0];
        } else {
          int64_t idx = key[k];
          if (idx < 0 || idx >= rd_n[kDirectDesc ? k : 0]) {
            atomicOr(p.err, DFWFM_FLAG_INDEX_OUT_OF_RANGE);
            idx = 0;
          }
          if (kPackable && pkrow[kPackable ? k : 0]) {
            pa[k] = rd_emb2[kDirectDesc ? k : 0] + idx * p.pkw;
          } else {
            pa[k] = rd_emb2[kDirectDesc ? k : 0] + idx * D;
            if (fo_tab) qa[k] = rd_emb1[kDirectDesc ? k : 0] + idx;
          }
        }
      } else if (live[k]) {
        const FieldDev fd = desc[f];
        if (f < num) {
          scale[k] = __int_as_float((int)key[k]);
          pa[k] = fd.emb2;
          qa[k] = fd.emb1;
        } else {
          int64_t idx = key[k];
          if (idx < 0 || idx >= fd.n) {
            atomicOr(p.err, DFWFM_FLAG_INDEX_OUT_OF_RANGE);
            idx = 0;
          }
          if (!QR || fd.c == 0) {
            pa[k] = fd.emb2 + idx * D;
            if (fo_tab) qa[k] = fd.emb1 + idx;
          } else if constexpr (QR) {
            const int64_t q = idx / fd.c;
            const int64_t rr = idx - q * fd.c;
            mode[k] = fd.op == 0 ? 1 : 2;
            pa[k] = fd.emb2 + q * D;
            pb[k] = fd.emb2_r + rr * D;
            if (fo_tab) {
              qa[k] = fd.emb1 + q;
              qb[k] = fd.emb1_r + rr;
            }
          }
        }
      }
    }
    // all loads first (the second operand only for QR rows) ...
    float va[RPT][D], vb[RQ][D], fa[RPT], fb[RQ];
#pragma unroll
    for (int k = 0; k < RPT; ++k) {
      fa[k] = 0.f;
#pragma unroll
      for (int d = 0; d < D; ++d) va[k][d] = 0.f;
      if constexpr (QR) {
        fb[k] = 0.f;
#pragma unroll
        for (int d = 0; d < D; ++d) vb[k][d] = 0.f;
      }
      if (kPackable && live[k] && pkrow[kPackable ? k : 0]) {  // second and first order in one aligned row
        load_row_fo<D>(va[k], fa[k], pa[k]);
      } else {
        if (live[k] && needE) {
          load_row<D>(va[k], pa[k]);
          if constexpr (QR)
            if (mode[k] != 0) load_row<D>(vb[k], pb[k]);
        }
        if (live[k] && fo_tab) {
          fa[k] = *qa[k];
          if constexpr (QR)
            if (mode[k] != 0) fb[k] = *qb[k];
        }
      }
    }
    // layer-0 weights: the first two chunks go out behind the row loads (vmcnt retires in issue order, so
    // issuing them earlier would make every gather wait for 56 KB of weights) and land during the combine,
    // the shallow part and the barriers
    if (deep) {
      ls.init(wrsrc, 0, p.NC0, p.NT, g, kh);
      DFWFM_PRELOAD(ls);
    }
    if constexpr (!QR)  // PART 3: behind the row loads (vmcnt retires in order); QR: no room
      if (!(flags & kPairs) && !(kPieces && (flags & kP3Pieces))) load_uu();
    // ... the shallow parameters go to LDS while the row loads are in flight ...
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
    // zero the E-tile padding read by the MLP (NC0*16 columns) and the FwFM (S*4 fields)
    const int w = p.W0 - F * D;
    for (int i = tid; i < kBM * w; i += NTH) {
      const int b = i / w;
      bufX[b * SX + F * D + (i - b * w)] = 0.f;
    }
    // ... then combine and store
#pragma unroll
    for (int k = 0; k < RPT; ++k) {
      const int r = tid + k * NTH;
      const int f = r >> 4;
      const int b = r & 15;
      if (f < F) {
        if (needE) {
          float e[D];
#pragma unroll
          for (int d = 0; d < D; ++d) e[d] = live[k] ? combine(mode[k], va[k][d], QR ? vb[k][d] : 0.f, scale[k]) : 0.f;
          store_row<D>(bufX + b * SX + f * D, e);
        }
        fo[b * Fp + f] = live[k] ? combine(mode[k], fa[k], QR ? fb[k] : 0.f, scale[k]) : 0.f;
      }
    }
  }
  __syncthreads();
  stamp(p.stamps, 2, tid);
  if constexpr (PART == 1 || PART == 3) {
    // the E tile (W0 columns, zero padded past F*D) for the MLP launch, behind the shallow part (PART 3: only for
    // dfwfm_forward_gather, the deep model's gather half as the MLP-free kernel)
    if (PART == 1 || p.part_e)
      store_tile(p.part_e + b0 * p.part_stride, p.part_stride, bufX, SX, nrows, p.part_stride >> 2, tid, NTH);
  }
  if constexpr (train) {
    // E for the shallow backward.  Without deep-tower dropout E is also X_0 and is saved after
    // layer 1's K loop from the same LDS tile (stores issued behind that layer's weight stream)
    if (drop0 || !deep) store_tile(p.sv_e + b0 * SE, SE, bufX, SX, nrows, SE / 4, tid, NTH);
  }

  // ---- phase S: shallow part ----------------------------------------------
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
  if constexpr (PART == 3) {
    if ((flags & kHasSecond) && (flags & kPairs)) {
      // pruned R (dfwfm_model_build_fwfm_pairs): second[b] = sum over the nonzero pairs of w_kl <E_bk, E_bl>,
      // LPS lanes per sample taking every LPS-th pair (k-major list), then an LPS-lane butterfly
      constexpr int LPS = NTH / kBM;
      const int b = tid / LPS, j = tid % LPS;
      const float* eb = bufX + b * SX;
      float part = 0.f;
      for (int q = j; q < p.npairs; q += LPS) {
        const int2 pr = p.pairs[q];
        const float* ek = eb + (pr.x & 0xffff) * D;
        const float* el = eb + (pr.x >> 16) * D;
        float dot = 0.f;
#pragma unroll
        for (int d = 0; d < D; ++d) dot = fmaf(ek[d], el[d], dot);
        part = fmaf(__int_as_float(pr.y), dot, part);
      }
#pragma unroll
      for (int o = LPS / 2; o >= 1; o >>= 1) part += __shfl_xor(part, o);
      if (j == 0) part2[b] = part;
    } else if ((flags & kHasSecond) && kPieces && (flags & kP3Pieces)) {
      // MLP-free forward (four waves in batch sets, five workgroups per CU; eight for a lone batch), FwFM as pieces: Y = U' E (rows k: fields, MT tiles of 16; columns n = b*D + d of the 16
      // samples: D tiles of 16; contraction over l: S steps of 4, from step 4m on -- U' is strictly upper), column
      // tile nt owned by wave nt % NW for every row tile m; second[b] = sum_{k,d} E[b,k,d] Y[k, b*D + d].  180
      // MFMAs per 16 samples against the Gram's 288: the MFMA time, not only the latency, sets this kernel's rate in
      // batch sets (five workgroups per CU).  U' fragments (A operands) arrive with the row loads (uf).
      constexpr int MTC = P3_MTC;
      constexpr int SMAX = 4 * MTC;
      const int MT = p.MT, S = p.S;
      float uf[MTC][SMAX];
      {
        const float* up = p.upack;
#pragma unroll
        for (int m = 0; m < MTC; ++m)
#pragma unroll
          for (int s = 0; s < SMAX; ++s)
            uf[m][s] = (m < MT && s >= 4 * m && s < S) ? up[(m * S + s) * 64 + lane] : 0.f;
      }
      for (int nt = wave; nt < D; nt += NW) {
        const int n = nt * 16 + (lane & 15);
        const int b = n / D;
        const int d = n - b * D;
        const float* ecol = bufX + b * SX + d;  // E[b][l][d] = ecol[l * D]
        // the row tiles' chains side by side: step s's B operand (E column, one LDS read) feeds every row tile m
        // with 4m <= s, each into its own accumulator (two column tiles at a time measured slower: 14.2k vs 11.6k
        // cycles for the phase, profiles/r05/r05m_stP.log)
        f32x4 acc[MTC];
#pragma unroll
        for (int m = 0; m < MTC; ++m) acc[m] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int s0 = 0; s0 < SMAX; s0 += 4) {
          float bv[4];
#pragma unroll
          for (int u = 0; u < 4; ++u) {
            const int s = s0 + u;
            bv[u] = s < S ? ecol[(4 * s + (lane >> 4)) * D] : 0.f;
          }
#pragma unroll
          for (int u = 0; u < 4; ++u)
#pragma unroll
            for (int m = 0; m < MTC; ++m)
              if (4 * m <= s0 + u && s0 + u < S && m < MT)
                acc[m] = __builtin_amdgcn_mfma_f32_16x16x4f32(uf[m][s0 + u], bv[u], acc[m], 0, 0, 0);
        }
        float colv = 0.f;
#pragma unroll
        for (int m = 0; m < MTC; ++m) {
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int k = 16 * m + 4 * (lane >> 4) + r;
            colv = fmaf(k < F ? ecol[(k < F ? k : 0) * D] : 0.f, acc[m][r], colv);
          }
        }
        colv += __shfl_xor(colv, 16);
        colv += __shfl_xor(colv, 32);
        if (lane < 16) part2[n] = colv;  // column n's sum over k (row tiles in order)
      }
    } else if (flags & kHasSecond) {
      // MLP-free forward: second[b] = sum_{k<l} U'[k,l] <E_bk, E_bl> from the per-sample Gram G_b = E_b E_b^T
      // on MFMA (rows k, columns l, contraction over d: ceil(D/4) steps).  A sample's MT*ceil(D/4) operand
      // fragments serve as both A and B of its upper tiles (m <= n), so every chain is ceil(D/4) MFMAs deep
      // and a wave has 6 x 3 independent ones per sample at Criteo-39 -- the (row tile, column tile)
      // pieces' 10-deep chains of fwd_kernel's other forms left this phase latency-bound.  U' is the
      // strictly upper (R + R^T)/2 (FM: ones) read from the A-fragment pack in LDS.
      constexpr int SD = (D + 3) / 4;
      constexpr int MTC = P3_MTC;
      constexpr int NTL = P3_NTL;
      const int MT = p.MT;
      if constexpr (QR) load_uu();
      for (int b = wave; b < kBM; b += NW) {
        float ev[MTC][SD];
#pragma unroll
        for (int m = 0; m < MTC; ++m)
#pragma unroll
          for (int s = 0; s < SD; ++s) {
            const int k = 16 * m + (lane & 15);
            const int d = 4 * s + (lane >> 4);
            ev[m][s] = (m < MT && k < F && d < D) ? bufX[b * SX + k * D + d] : 0.f;
          }
        // every upper tile's chain issued step by step across the tiles (independent accumulators), then the
        // U'-weighted sum
        f32x4 acc[NTL];
#pragma unroll
        for (int t = 0; t < NTL; ++t) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int s = 0; s < SD; ++s)
#pragma unroll
          for (int m = 0, t = 0; m < MTC; ++m)
#pragma unroll
            for (int n = m; n < MTC; ++n, ++t)
              if (n < MT) acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(ev[m][s], ev[n][s], acc[t], 0, 0, 0);
        float part = 0.f;
#pragma unroll
        for (int t = 0; t < NTL; ++t)
#pragma unroll
          for (int r = 0; r < 4; ++r) part = fmaf(uu[t][r], acc[t][r], part);
#pragma unroll
        for (int o = 32; o >= 1; o >>= 1) part += __shfl_xor(part, o);
        if (lane == 0) part2[b] = part;
      }
    }
  } else if (flags & kHasSecond) {
    // Y = U * E_b on MFMA: rows k (fields, MT tiles of 16), columns n = b*D + d (D tiles of 16), contraction
    // over l (fields, S steps of 4).  second[b] = sum_{k,d} E[b,k,d] * Y[k, b*D+d].  The work is cut into
    // pieces pc = (row tile m, column tile nt) of S - 4m steps each (U's rows 16m.. vanish for l <= 16m); the
    // host balances the pieces over the waves (fw_list), and every piece leaves its 16 column sums in
    // part2[pc] -- so the result does not depend on the wave count.
    const int S = p.S;
    const uint8_t* plist = NW == 8 ? p.fw_list8 : p.fw_list4;
    const int p_lo = NW == 8 ? p.fw_off8[wave] : p.fw_off4[wave];
    const int p_hi = NW == 8 ? p.fw_off8[wave + 1] : p.fw_off4[wave + 1];
    for (int pi = p_lo; pi < p_hi; ++pi) {
      const int pc = plist[pi];
      const int m = pc / D;
      const int nt = pc - m * D;
      const int n = nt * 16 + (lane & 15);
      const int b = n / D;
      const float* ecol = bufX + b * SX + (n - b * D);  // E[b][l][d] = ecol[l * D]
      const float* ua = upk + m * S * 64 + lane;        // A fragment of step s: ua[s * 64]
      f32x4 acc = f32x4{0.f, 0.f, 0.f, 0.f};
      // steps in groups: every operand of a group is read from LDS before its MFMAs
      auto group = [&](int s0, auto U_) {
        constexpr int U = decltype(U_)::value;
        float av[U], bv[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
          av[u] = ua[(s0 + u) * 64];
          bv[u] = ecol[(4 * (s0 + u) + (lane >> 4)) * D];
        }
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int u = 0; u < U; ++u) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(av[u], bv[u], acc, 0, 0, 0);
      };
      int s0 = 4 * m;
      for (; s0 + 4 <= S; s0 += 4) group(s0, std::integral_constant<int, 4>{});
      const int rem = S - s0;
      if (rem == 3) group(s0, std::integral_constant<int, 3>{});
      else if (rem == 2) group(s0, std::integral_constant<int, 2>{});
      else if (rem == 1) group(s0, std::integral_constant<int, 1>{});
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
    }
  }
  // layer 0's tail fragments once the gather rows are dead (live across the gather, they spilled)
  if constexpr (NSK == 0) {
    if (deep && tail) {
      ts.init(0, p.NC0, TT, g);
      ts.load(wrsrc, tw, lane * 16);
    }
  }
  stamp(p.stamps, 10, tid);
  __syncthreads();
  stamp(p.stamps, 11, tid);
  if constexpr (train) {
    for (int i = tid; i < kBM * F; i += NTH) {
      const int b = i / F;
      if (b0 + b < p.batch) p.sv_fo[(b0 + b) * F + (i - b * F)] = fo[b * Fp + (i - b * F)];
    }
    if (drop0) {  // deep_emb dropout (net_1_linear_0_dropout, model/DeepFMs.py:411), in place
      const uint32_t dseed = step_seed(p.seed, p.seed_src);
      for (int i = tid; i < kBM * FD; i += NTH) {
        const int b = i / FD;
        const int c = i - b * FD;
        const float v = bufX[b * SX + c];
        bufX[b * SX + c] = dropout_keep(dseed, 0, b0 + b, c, p.drop_p) ? v * p.drop_scale : 0.f;
      }
    }
  }
  if (wave < 4) {
    // first[b] (lw projection or plain sum over fields) and second[b] (sum over d): 16 lanes per sample
    // each take every 16th term, then a 16-lane DPP sum.  Every LDS read is issued before the first add:
    // this runs while waves 4-7 already stream layer 1 through the LDS, and a chain of a dozen dependent
    // LDS round trips (loop-carried reads, __shfl_xor butterflies) took ~10k cycles there.
    const int b = wave * 4 + (lane >> 4);
    const int q = lane & 15;
    float first = 0.f, second = 0.f;
    for (int f0 = 0; f0 < F; f0 += 64) {
      float x[4], l[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int f = min(f0 + 16 * k + q, F - 1);
        x[k] = fo[b * Fp + f];
        l[k] = (flags & kFoLw) ? lw_s[f] : 1.f;
      }
#pragma unroll
      for (int k = 0; k < 4; ++k) first = f0 + 16 * k + q < F ? fmaf(x[k], l[k], first) : first;
    }
    if (flags & kHasSecond) {
      if constexpr (PART == 3) {
        if (kPieces && (flags & kP3Pieces) && !(flags & kPairs)) {
          for (int d = q; d < D; d += 16) second += part2[b * D + d];  // the sample's column sums
        } else {
          second = q == 0 ? part2[b] : 0.f;  // the sample's Gram sum
        }
      } else {
        const int MT = p.MT;
        for (int d = q; d < D; d += 16) {  // D = 32: two terms per lane
          const int n = b * D + d;
          const float* pp = part2 + (n >> 4) * 16 + (n & 15);  // part2[(m * D + (n >> 4)) * 16 + (n & 15)]
          float v[4];
#pragma unroll
          for (int m = 0; m < 4; ++m) v[m] = pp[min(m, MT - 1) * D * 16];
#pragma unroll
          for (int m = 0; m < 4; ++m) second += m < MT ? v[m] : 0.f;
          for (int m = 4; m < MT; ++m) second += pp[m * D * 16];
        }
      }
    }
    first = sum16(first);
    second = sum16(second);
    if (q == 0) fs[b] = first + second;
  }
  if (p.H < 4) stamp(p.stamps, 7, tid);  // diagnostics: the sums' end (slot 7 is a layer slot only past three layers)

  if (!deep) {
    __syncthreads();
    if (PART == 1 || (PART == 3 && p.part_fs)) {
      if (tid < kBM && b0 + tid < p.batch) p.part_fs[b0 + tid] = fs[tid];
    } else {
      if (tid < kBM && b0 + tid < p.batch) tr.out[b0 + tid] = fs[tid] + p.bias[0];
    }
    stamp(p.stamps, 8, tid);
    stamp_end_rt(p.stamps, tid);
    return;
  }
  }

  stamp(p.stamps, 3, tid);
  if (flags & kPrio) __builtin_amdgcn_s_setprio(0);
  if constexpr (train) __syncthreads();  // the dropped X_0 tile is complete before layer 1 reads it
  // ---- phase M: MLP on MFMA -------------------------------------------------
  // Weights are the MFMA A operand (mlp_k_loop WA): lane l holds neurons 4(l>>4) + r of sample row l&15, so
  // a tile's four outputs of a sample leave as one 16-byte LDS store.  The accumulators start from the bias.
  const bool drop = train && (flags & kDrop) != 0;
  const uint32_t hseed = drop ? step_seed(p.seed, p.seed_src) : 0u;
  // this wave's biases (four per tile, 16-byte buffer loads), fetched one layer ahead: they seed the
  // accumulators at the start of the K loop (so they are dead during it)
  auto load_bias = [&](f32x4 (&bq)[TPW], int h, int nq) {
#pragma unroll
    for (int j = 0; j < TPW; ++j) {
      int t = g + NG * j;
      t = t < p.NT ? t : p.NT - 1;
      // lane part nq*4 in a VGPR, the tile / layer part in the scalar offset (per-tile lane offsets were
      // hoisted out of the layer loop, spilled, and every reload waited for the whole preload)
      bq[j] = kh == 0 ? __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(
                            brsrc, nq * 4, __builtin_amdgcn_readfirstlane((h * p.NT + t) * 64), 0))
                      : f32x4{0.f, 0.f, 0.f, 0.f};
    }
  };
  f32x4 bq[TPW];
  load_bias(bq, 0, 4 * (lane >> 4));
  int layer_off = 0;  // float4 offset of layer h in wpack
  for (int h = 0; h < p.H; ++h) {
    // the lane-derived epilogue values are recomputed per layer: hoisted out of the loop they stay live across
    // it and spill, and a reload after the next layer's preload waits for the whole preload (vmcnt order)
    int lv = lane;
    asm volatile("" : "+v"(lv));
    const int rowl = lv & 15;
    const int nq = 4 * (lv >> 4);
    const bool even = (h & 1) == 0;
    const float* in = even ? bufX : bufY;
    const int SA = even ? SX : SY;
    float* outa = even ? bufY : bufX;
    const int SO = even ? SY : SX;
    const int NC = h == 0 ? p.NC0 : p.NT;
    const bool last = h == p.H - 1;
    // the tail tile's bias (one neuron per lane of waves 0..3), fetched before the K loop
    const int boff = __builtin_amdgcn_readfirstlane((h * p.NT + TT) * 64 + (g & 3) * 4);
    const int ntail = TT * 16 + nq + (g & 3);
    const float bn_t = tail ? __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(brsrc, nq * 4, boff, 0))
                            : 0.f;

    f32x4 acc[TPW];
#pragma unroll
    for (int j = 0; j < TPW; ++j) acc[j] = bq[j];  // the K loop accumulates onto the bias
    if constexpr (NSK > 0) {
      // the tail tile's share rides on the K loop's register sets
      if (tail) ts.init(layer_off, NC, TT, g);
      else ts.cnt = 0;
      f32x4 tp;
      mlp_k_loop_s<TPW, NG, NSK, true>(acc, in, SA, ls, wb0, wb1, wb2, lane, ts, tp);
      if (tail) reinterpret_cast<f32x4*>(tailr)[g * 64 + lane] = tp;
    } else {
      // the tail tile's share first: its fragments (loaded with the preload) are then dead during the K loop
      if (tail) reinterpret_cast<f32x4*>(tailr)[g * 64 + lane] = ts.template mma<true>(in, SA, tw, lane);
      mlp_k_loop<TPW, KS, NG, true, true>(acc, in, SA, ls, wb0, wb1, wb2, lane);
    }
    if (h == 0) stamp(p.stamps, 12, tid);
    if constexpr (KS == 2) {
      if (kh == 1) {
#pragma unroll
        for (int j = 0; j < TPW; ++j) red[(g * TPW + j) * 64 + lane] = acc[j];
      }
      __syncthreads();
      if (kh == 0) {
#pragma unroll
        for (int j = 0; j < TPW; ++j) acc[j] += red[(g * TPW + j) * 64 + lane];
      }
    }
    float dpart = 0.f;  // last layer: this lane's share of deep[row] (not live across layers)
    if (kh == 0) {
      float* orow = outa + rowl * SO + nq;  // + t*16 (wave-uniform) per tile
#pragma unroll
      for (int j = 0; j < TPW; ++j) {
        const int t = g + NG * j;  // wave-uniform
        if (t < p.NT) {
          float v[4];
          if (t * 16 + 16 <= p.N) {  // no padded neuron in this tile
#pragma unroll
            for (int r = 0; r < 4; ++r) v[r] = relu_keep_nan(acc[j][r]);
          } else {  // padded neurons stay exactly 0 (bias / fc pads are 0)
#pragma unroll
            for (int r = 0; r < 4; ++r) v[r] = nq + r < p.N - t * 16 ? relu_keep_nan(acc[j][r]) : 0.f;
          }
          if constexpr (train) {
            // dropout after the ReLU (net_1_linear_{h}_dropout, :416-426)
            if (drop) {
#pragma unroll
              for (int r = 0; r < 4; ++r)
                v[r] = dropout_keep(hseed, h + 1, b0 + rowl, t * 16 + nq + r, p.drop_p) ? v[r] * p.drop_scale : 0.f;
            }
          }
          // the tile goes to LDS also in the last layer of a training step, from where X_H is saved
          if (!last || train) *reinterpret_cast<f32x4*>(orow + t * 16) = f32x4{v[0], v[1], v[2], v[3]};
          if (last) {
            const f32x4 wf =
                __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(frsrc, nq * 4, t * 64, 0));
            dpart = fmaf(v[0], wf[0], dpart);
            dpart = fmaf(v[1], wf[1], dpart);
            dpart = fmaf(v[2], wf[2], dpart);
            dpart = fmaf(v[3], wf[3], dpart);
          }
        }
      }
    }
    if (last && kh == 0) {
      // deep[b] = sum_n h_last[b, n] * fc[n]: reduce the four lanes sharing the row, then (after the final
      // barrier) the NG groups
      dpart += __shfl_xor(dpart, 16);
      dpart += __shfl_xor(dpart, 32);
      if (lane < 16) dsum[g * kBM + rowl] = dpart;
    }
    // next layer's first chunks and biases go out now, ahead of the barrier -- but after the epilogue: once
    // they are issued, any wait on a vector-memory result (a spill reload) waits for them too
    layer_off += p.NT * NC * 64;
    if (!last) {
      ls.init(wrsrc, layer_off, p.NT, p.NT, g, kh);
      DFWFM_PRELOAD(ls);
      if constexpr (NSK == 0) {
        if (tail) {
          ts.init(layer_off, p.NT, TT, g);
          ts.load(wrsrc, tw, lane * 16);
        }
      }
      load_bias(bq, h + 1, nq);
    }
    if constexpr (train) {
      // this layer's input X_h for the backward, from LDS (intact until the next layer's epilogue):
      // behind the next layer's preload, so those loads do not wait for the stores (vmcnt is in order)
      // (measured: issued after the next layer's K loop instead, the training forward went 111.0k -> 113.4k cycles,
      // profiles/r04/r04l_st-train.log)
      if (h == 0)
        store_tile(p.sv_x[0] + b0 * SE, SE, in, SA, nrows, SE / 4, tid, NTH);
      else
        store_tile(p.sv_x[h] + b0 * p.N, p.N, in, SA, nrows, p.N / 4, tid, NTH);
    }
    if (h == 0) stamp(p.stamps, 13, tid);
    __syncthreads();
    if (tail) {
      // the tail tile: wave g < 4 finishes neuron TT*16 + nq + g of row rowl from the NG partial products
      if (g < 4) {
        float* orow_t = outa + rowl * SO + nq;
        const bool valid = ntail < p.N;
        const float* tp = tailr + lane * 4 + g;
        float sum = tp[0];
#pragma unroll
        for (int w = 1; w < NG; ++w) sum += tp[w * 256];
        float v = valid ? relu_keep_nan(sum + bn_t) : 0.f;
        if constexpr (train) {
          if (drop) v = dropout_keep(hseed, h + 1, b0 + rowl, ntail, p.drop_p) ? v * p.drop_scale : 0.f;
          if (last) orow_t[TT * 16 + g] = v;  // X_H is saved from LDS
        }
        if (!last) {
          orow_t[TT * 16 + g] = v;
        } else {
          // the tail's share of deep[b]: its four neurons of this wave, reduced over the lane groups, one slot
          // per (wave, row); added last in the final combine, so a row's logit does not depend on its slot
          const float wf_t = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(
                                 frsrc, nq * 4, __builtin_amdgcn_readfirstlane(TT * 64 + g * 4), 0));
          float c = v * wf_t;
          c += __shfl_xor(c, 16);
          c += __shfl_xor(c, 32);
          if (lane < 16) tailr[NG * 64 * 4 + g * kBM + rowl] = c;
        }
      }
      if (!last) __syncthreads();
    }
    stamp(p.stamps, 4 + (h < 3 ? h : 3), tid);
  }

  if constexpr (train) {
    // X_H (the last layer's output after ReLU / dropout) from LDS: the buffer the last layer wrote
    if (tail) __syncthreads();  // the tail tile's rows were written after the layer's barrier
    float* last_out = ((p.H - 1) & 1) == 0 ? bufY : bufX;
    const int SL = ((p.H - 1) & 1) == 0 ? SY : SX;
    store_tile(p.sv_x[p.H] + b0 * p.N, p.N, last_out, SL, nrows, p.N / 4, tid, NTH);
  }

  __syncthreads();
  if (tid < kBM && b0 + tid < p.batch) {
    float deepv = dsum[tid];
#pragma unroll
    for (int w = 1; w < NG; ++w) deepv += dsum[w * kBM + tid];
    if (tail) deepv += ((tailr[NG * 64 * 4 + tid] + tailr[NG * 64 * 4 + kBM + tid]) +
                        tailr[NG * 64 * 4 + 2 * kBM + tid]) + tailr[NG * 64 * 4 + 3 * kBM + tid];
    tr.out[b0 + tid] = (fs[tid] + deepv) + p.bias[0];
  }
  stamp(p.stamps, 8, tid);
  stamp_end_rt(p.stamps, tid);
}

#ifndef DFWFM_KD  // packing: the common translation unit only
// ---------------------------------------------------------------------------
// dense-parameter packing (run on weight updates, not per forward)
// ---------------------------------------------------------------------------

// ---------------------------------------------------------------------------
// Dense-parameter packing, one launch for every job of a set_dense (re-run after each optimizer step):
//   kPackPad       dst[i] = i < n ? src[i] : 0, i < npad
//   kPackLinear    W [N][K] (nn.Linear.weight) -> [NT][NC][64] float4 forward fragments:
//                  out[(t*NC + c)*64 + lane][s] = W[16t + (lane&15)][16c + 4(lane>>4) + s]
//   kPackLinearT   the backward's transposed fragments (outputs k, contraction n):
//                  out[(t*NC + c)*64 + lane][s] = W[16c + 4(lane>>4) + s][16t + (lane&15)]
//   kPackFwfm      FwFM A operand U[k][l] = (R[l][k] + R[k][l]) / 2 for l > k (model/DeepFMs.py:363-364;
//                  the diagonal is removed by :366-367); FM: 1 above the diagonal.  Fragment order
//                  out[(m*S + s)*64 + lane] = U[16m + (lane&15)][4s + (lane>>4)]
//   kPackFwfmSym   the backward's symmetric off-diagonal (R + R^T)/2 (FM: ones), same order
// ---------------------------------------------------------------------------
__device__ __forceinline__ void pack_elem(const PackJob& j, int64_t i) {
  switch (j.type) {
    case kPackPad:
      j.dst[i] = (j.src && i < j.a) ? j.src[i] : 0.f;
      break;
    case kPackLinear:
    case kPackLinearT: {
      const int N = j.a, K = j.b, NC = j.d;
      const int lane = (int)(i & 63);
      const int64_t tc = i >> 6;
      const int c = (int)(tc % NC);
      const int t = (int)(tc / NC);
      const bool tr = j.type == kPackLinearT;
      float v[4];
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        const int n = tr ? 16 * c + 4 * (lane >> 4) + s : t * 16 + (lane & 15);
        const int k = tr ? t * 16 + (lane & 15) : 16 * c + 4 * (lane >> 4) + s;
        v[s] = (n < N && k < K) ? j.src[(int64_t)n * K + k] : 0.f;
      }
      reinterpret_cast<float4*>(j.dst)[i] = make_float4(v[0], v[1], v[2], v[3]);
      break;
    }
    case kPackFwfm:
    case kPackFwfmSym: {
      const int F = j.a, mode = j.b, S = j.d;
      const int lane = (int)(i & 63);
      const int ms = (int)(i >> 6);
      const int s = ms % S;
      const int m = ms / S;
      const int k = 16 * m + (lane & 15);
      const int l = 4 * s + (lane >> 4);
      const bool keep = j.type == kPackFwfm ? l > k : l != k;
      float u = 0.f;
      if (k < F && l < F && keep) u = (mode == 1) ? 1.f : (j.src[l * F + k] + j.src[k * F + l]) * 0.5f;
      j.dst[i] = u;
      break;
    }
    default:
      break;
  }
}

__global__ void __launch_bounds__(256) pack_dense_kernel(const PackList L) {
  int lo = 0, hi = L.n - 1;
  const int bid = blockIdx.x;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (L.j[mid].block0 <= bid) lo = mid;
    else hi = mid - 1;
  }
  const PackJob& j = L.j[lo];
  if (j.type == kPackZero) {
    // a bulk zero (the training step's gradient buffer): 16-byte stores, the block's threads on consecutive float4
    float4* d = reinterpret_cast<float4*>(j.dst);
    const int64_t q0 = (int64_t)(bid - j.block0) * 256 * kPackZeroPT + threadIdx.x;
#pragma unroll
    for (int u = 0; u < kPackZeroPT; ++u)
      if (q0 + u * 256 < j.total) d[q0 + u * 256] = make_float4(0.f, 0.f, 0.f, 0.f);
    return;
  }
  const int64_t i = (int64_t)(bid - j.block0) * 256 + threadIdx.x;
  if (i < j.total) pack_elem(j, i);
}

#endif  // DFWFM_KD

// ---------------------------------------------------------------------------
// launchers
// ---------------------------------------------------------------------------
template <int D, int TPW, int KS, bool TRAIN, int PART = 0, int NG = 4>
static hipError_t launch_fwd_t(const FwdArgs& a, size_t lds, hipStream_t s) {
  // the static 25-chunk form (3x400 MLP over 39x10 embeddings: 25 tiles = 8 waves x 3 + the split 25th)
  constexpr bool S25 = NG == 8 && TPW == 3 && KS == 1 && PART != 1;
  // the static form without QR fields also loads its row descriptors directly (no staging barrier)
  constexpr bool S25D = S25 && PART == 0 && DFWFM_DIRECT_DESC_DEEP;
  auto k = (S25 && a.ns == 25) ? ((S25D && !(a.flags & kHasQR)) ? fwd_kernel<D, TPW, KS, TRAIN, PART, NG, S25 ? 25 : 0, false>
                                                               : fwd_kernel<D, TPW, KS, TRAIN, PART, NG, S25 ? 25 : 0>)
                               : fwd_kernel<D, TPW, KS, TRAIN, PART, NG, 0>;
  {
    hipError_t e = ensure_lds_limit(reinterpret_cast<const void*>(k), lds);
    if (e != hipSuccess) return e;
  }
  const unsigned grid = fwd_grid(a, kBM);
  hipLaunchKernelGGL(k, dim3(grid), dim3(64 * NG * KS), lds, s, a);
  return hipGetLastError();
}

template <int D, int KS, bool TRAIN>
static hipError_t launch_fwd_k(const FwdArgs& a, int tpw, size_t lds, hipStream_t s) {
  switch (tpw) {
    case 1: return launch_fwd_t<D, 1, KS, TRAIN>(a, lds, s);
    case 2: return launch_fwd_t<D, 2, KS, TRAIN>(a, lds, s);
    case 3: return launch_fwd_t<D, 3, KS, TRAIN>(a, lds, s);
    case 4: return launch_fwd_t<D, 4, KS, TRAIN>(a, lds, s);
    case 5: return launch_fwd_t<D, 5, KS, TRAIN>(a, lds, s);
    case 6: return launch_fwd_t<D, 6, KS, TRAIN>(a, lds, s);
    case 7: return launch_fwd_t<D, 7, KS, TRAIN>(a, lds, s);
    case 8: return launch_fwd_t<D, 8, KS, TRAIN>(a, lds, s);
    default: return hipErrorInvalidValue;
  }
}

// eight tile groups (inference): at most 32 output tiles, so at most 4 per wave
template <int D, int PART, bool TRAIN = false>
static hipError_t launch_fwd_8(const FwdArgs& a, int tpw, size_t lds, hipStream_t s) {
  switch (tpw) {
    case 1: return launch_fwd_t<D, 1, 1, TRAIN, PART, 8>(a, lds, s);
    case 2: return launch_fwd_t<D, 2, 1, TRAIN, PART, 8>(a, lds, s);
    case 3: return launch_fwd_t<D, 3, 1, TRAIN, PART, 8>(a, lds, s);
    case 4: return launch_fwd_t<D, 4, 1, TRAIN, PART, 8>(a, lds, s);
    default: return hipErrorInvalidValue;
  }
}

template <int D>
static hipError_t launch_fwd_d(const FwdArgs& a, int tpw, int ks, int ng, size_t lds, hipStream_t s) {
  // no deep tower: the MLP-free instantiation on eight waves (105 registers, no scratch): 4.92 us per batch
  // at three batches in flight against 5.19 for the generic four-wave one (DFWFM_DIAG part3=0) and 6.0 for a
  // four-wave MLP-free one (128 registers + spills)
  if (!(a.flags & (kHasDeep | kTrain)) && diag_opt("part3", 1) != 0) {
    // one instantiation per FwFM row-tile count (NS = MT): the Gram tiles' registers sized to the model.  Eight
    // waves (70 registers, three workgroups per CU: 3.55 us per batch at three batches in flight); four waves without
    // QR operands (94 registers, five workgroups per CU by the trimmed LDS: 3.74 us at three or six in flight,
    // profiles/r02/r02r_*); a model with a QR field always takes eight (four would spill the QR rows' second
    // operands).  DFWFM_DIAG p3ng=4 / 8 forces either (tests)
    const int png = diag_opt("p3ng", 0);
    const bool qr = (a.flags & kHasQR) != 0;
    // batch sets (a.nb > 1): four waves -- with the CU slots refilled across batch boundaries, five four-wave
    // workgroups per CU beat three eight-wave ones (2.52 vs 2.92 us per batch, profiles/r03/r03be_*)
    const bool w8 = qr || (png ? png != 4 : a.nb <= 1);
    auto pick = [&](auto ng_, auto qr_) {
      constexpr int NG = decltype(ng_)::value;
      constexpr bool Q = decltype(qr_)::value;
      return a.MT == 1 ? fwd_kernel<D, 1, 1, false, 3, NG, 1, Q>
           : a.MT == 2 ? fwd_kernel<D, 1, 1, false, 3, NG, 2, Q>
           : a.MT == 3 ? fwd_kernel<D, 1, 1, false, 3, NG, 3, Q> : fwd_kernel<D, 1, 1, false, 3, NG, 4, Q>;
    };
    using I4 = std::integral_constant<int, 4>;
    using I8 = std::integral_constant<int, 8>;
    using T = std::true_type;
    using Fl = std::false_type;
    auto k = qr ? pick(I8{}, T{}) : (w8 ? pick(I8{}, Fl{}) : pick(I4{}, Fl{}));
    const int ng = w8 ? 8 : 4;
    const size_t lds3 = sizeof(float) * (size_t)lds_layout(a.F, D, a.MT, a.S, a.SX, a.SY, 1, 1, false, false, ng,
                                                            true, (a.flags & kFoFwlw) != 0).total;
    hipError_t e = ensure_lds_limit(reinterpret_cast<const void*>(k), lds3);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k, dim3(fwd_grid(a, kBM)), dim3(64 * ng), lds3, s, a);
    return hipGetLastError();
  }
  if (a.flags & kTrain) return ng == 8 ? launch_fwd_8<D, 0, true>(a, tpw, lds, s) : launch_fwd_k<D, 1, true>(a, tpw, lds, s);
  if (ng == 8) return launch_fwd_8<D, 0>(a, tpw, lds, s);
  return launch_fwd_k<D, 1, false>(a, tpw, lds, s);  // (one K half per wave: the K split was removed in round 6)
}

#ifdef DFWFM_KD
// one translation unit per embedding size (parallel build): this one's launchers
hipError_t DFWFM_PER_D(launch_forward_d)(const FwdArgs& a, int tpw, int ks, int ng, size_t lds, hipStream_t s) {
  return launch_fwd_d<DFWFM_KD>(a, tpw, ks, ng, lds, s);
}
hipError_t DFWFM_PER_D(launch_forward_gather_d)(const FwdArgs& a, size_t lds1, hipStream_t s) {
  return launch_fwd_t<DFWFM_KD, 1, 1, false, 1, 4>(a, lds1, s);
}
#else
hipError_t launch_forward_gather(const FwdArgs& a, int D, size_t lds1, hipStream_t s) {
  switch (D) {
    case 4: return launch_forward_gather_d4(a, lds1, s);
    case 8: return launch_forward_gather_d8(a, lds1, s);
    case 10: return launch_forward_gather_d10(a, lds1, s);
    case 16: return launch_forward_gather_d16(a, lds1, s);
    case 32: return launch_forward_gather_d32(a, lds1, s);
    default: return hipErrorInvalidValue;
  }
}

bool supported_embedding_size(int D) { return D == 4 || D == 8 || D == 10 || D == 16 || D == 32; }

hipError_t launch_forward(const FwdArgs& a, int D, int tpw, int ks, int ng, size_t lds, hipStream_t s) {
  switch (D) {
    case 4: return launch_forward_d4(a, tpw, ks, ng, lds, s);
    case 8: return launch_forward_d8(a, tpw, ks, ng, lds, s);
    case 10: return launch_forward_d10(a, tpw, ks, ng, lds, s);
    case 16: return launch_forward_d16(a, tpw, ks, ng, lds, s);
    case 32: return launch_forward_d32(a, tpw, ks, ng, lds, s);
    default: return hipErrorInvalidValue;
  }
}

// dfwfm_model_pack_tables: thread = one row of one categorical field, written as pkw / 4 float4:
// [emb2 row (D floats) | emb1 weight | zeros]
__global__ void __launch_bounds__(256) pack_tables_kernel(const PackTabList L) {
  int j = 0;
  while (j + 1 < L.nf && (int)blockIdx.x >= L.blk0[j + 1]) ++j;  // this workgroup's field (wave-uniform)
  const int64_t r = (int64_t)((int)blockIdx.x - L.blk0[j]) * 256 + threadIdx.x;
  if (r >= L.n[j]) return;
  const float* e2 = L.emb2[j] + r * L.D;
  const float e1 = L.emb1[j][r];
  f32x4* dst = reinterpret_cast<f32x4*>(L.dst[j] + r * L.pkw);
  for (int q = 0; q < L.pkw / 4; ++q) {
    f32x4 v;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int e = 4 * q + i;
      v[i] = e < L.D ? e2[e] : (e == L.D ? e1 : 0.f);
    }
    dst[q] = v;
  }
}

hipError_t launch_pack_tables(const PackTabList& L, hipStream_t s) {
  if (L.nf <= 0 || L.blk0[L.nf] <= 0) return hipSuccess;
  hipLaunchKernelGGL(pack_tables_kernel, dim3(L.blk0[L.nf]), dim3(256), 0, s, L);
  return hipGetLastError();
}

hipError_t launch_pack_list(const PackList& L, int total_blocks, hipStream_t s) {
  if (total_blocks <= 0 || L.n <= 0) return hipSuccess;
  hipLaunchKernelGGL(pack_dense_kernel, dim3(total_blocks), dim3(256), 0, s, L);
  return hipGetLastError();
}
#endif  // DFWFM_KD

}  // namespace dfwfm
