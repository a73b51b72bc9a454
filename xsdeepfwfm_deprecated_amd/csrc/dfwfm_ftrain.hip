// dfwfm_ftrain.hip -- the training forward of the static 3x400 form, the shallow part off the MLP's critical path.
//
// The training step's forward (reference model/DeepFMs.py:285-469 in train mode: dropout after every deep
// layer and on the deep input) has one 16-sample workgroup per CU at B = 4096, so the MLP's MFMA time per CU is
// fixed (~60k cycles for Criteo-39's 390 -> 400 -> 400 -> 400) and everything that does not feed the MLP only adds
// to it: fwd_kernel<TRAIN> runs the shallow part (fwlw, the FwFM pieces, the first / second sums: ~17k cycles)
// and the copies of the saved activations (X_h, from LDS, behind each layer) between the MLP's K loops.  Here:
//
//   all 12 waves   keys, gather, E tile (and X_0 = dropout(E)) into LDS
//   waves 0-7      the MLP exactly as fwd_kernel's static form (mlp_k_loop_s, split 25th tile, dropout after the
//                  ReLU), two barriers per layer
//   waves 8-11     the FwFM pieces, fwlw first order, E / X_0 saves, the first + second sums, the first-order save
//                  and X_h -> workspace for h >= 1, spread over the MLP's layers and meeting the MLP waves at its
//                  barriers
//
// The helper waves are slow beside a saturated matrix pipe (their SIMD's two MLP waves win the issue: the FwFM
// chains ran ~30k cycles there against ~11k alone), so layer 1's window still waits ~8k cycles for them.
// E stays in its own LDS tile and the layers' outputs rotate through two more, so nothing the helpers read is
// overwritten before they are done.  Every value is formed by the same arithmetic in the same order as
// fwd_kernel<TRAIN>'s (same K order onto the bias, same split-tile partials, same pieces, same sums): the logits
// and every saved activation are bit-identical to it (tests/test_gpu_train.py).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>

#include "dfwfm_device.h"
#include "dfwfm_internal.h"

namespace dfwfm {

namespace {

constexpr int kNG = 8;   // MLP waves (output-tile groups), two per SIMD
constexpr int kNH = 4;   // helper waves, one per SIMD
constexpr int kTPW = 3;  // whole output tiles per MLP wave: 25 = 8 x 3 + the split 25th
constexpr int kNS = 25;  // K chunks of every layer (static K loop)
constexpr int kNTH = 64 * (kNG + kNH);
constexpr int kHTH = 64 * kNH;

struct LdsT {
  int desc, lw, fwlw, upk, bufE, bufX, bufY, bufZ, tailr, taild, fo, part2, dsum, fs, total;
};

__host__ __device__ inline LdsT ldst_layout(int F, int D, int MT, int S, int SX, int SY) {
  LdsT L;
  int o = 0;
  L.desc = o;  o += r4(14 * F);
  L.lw = o;    o += r4(F);
  L.fwlw = o;  o += r4(F * D);
  L.upk = o;   o += MT * S * 64;
  L.bufE = o;  o += kBM * SX;  // E (the helpers' operand)
  L.bufX = o;  o += kBM * SX;  // X_0 after dropout (kept to the end: the helpers save it during layer 3)
  L.bufY = o;  o += kBM * SY;  // the outputs of layers 1, 3, ...
  L.bufZ = o;  o += kBM * SY;  // the outputs of layers 2, 4, ...
  L.tailr = o; o += kNG * 64 * 4;
  L.taild = o; o += 4 * kBM;
  L.fo = o;    o += kBM * r4(F);
  L.part2 = o; o += MT * D * 16;
  L.dsum = o;  o += kNG * kBM;
  L.fs = o;    o += kBM;
  L.total = r4(o);
  return L;
}

}  // namespace

template <int D, bool QR>
__global__ void __launch_bounds__(kNTH) ftrain_kernel(FwdArgs p) {
  constexpr int RPT = (kBM * 48 + kNTH - 1) / kNTH;  // gather rows per thread: F <= 48
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int F = p.F;
  const int num = p.num;
  const int SX = p.SX;
  const int SY = p.SY;
  const int flags = p.flags;
  const int Fp = r4(F);
  const int FD = F * D;
  const int SE = r4(FD);
  const LdsT L = ldst_layout(F, D, p.MT, p.S, SX, SY);
  FieldDev* desc = reinterpret_cast<FieldDev*>(smem + L.desc);
  float* lw_s = smem + L.lw;
  float* fwlw_s = smem + L.fwlw;
  float* upk = smem + L.upk;
  float* bufE = smem + L.bufE;
  float* bufX = smem + L.bufX;
  float* bufY = smem + L.bufY;
  float* bufZ = smem + L.bufZ;
  float* tailr = smem + L.tailr;
  float* taild = smem + L.taild;
  float* fo = smem + L.fo;
  float* part2 = smem + L.part2;
  float* dsum = smem + L.dsum;
  float* fs = smem + L.fs;
  uint64_t* const stamps = (flags & kFtDiagHwId) ? nullptr : p.stamps;  // HW_ID mode: no clocks
  const TileRef tr = tile_ref<kBM>(p);
  const int64_t b0 = tr.b0;
  const int nrows = (int)((p.batch - b0) < kBM ? (p.batch - b0) : kBM);
  const bool drop = (flags & kDrop) != 0;  // the deep tower's dropout (input and every hidden layer)
  const uint32_t dseed = drop ? step_seed(p.seed, p.seed_src) : 0u;
  const int H = p.H;
  stamp(stamps, 0, tid);
  stamp_start_rt(stamps, tid);

  // diagnostics (kFtDiagHwId: each wave's HW_ID into stamp slot `wave` instead of clocks; kFtDiagNoMlp)
  if ((flags & kFtDiagHwId) && p.stamps != nullptr && lane == 0)
    p.stamps[(size_t)blockIdx.x * kStampSlots + wave] = __builtin_amdgcn_s_getreg(4 | (31 << 11));
  const bool mlpw = wave < kNG;  // wave-uniform
  const int g = wave;            // MLP output-tile group (waves 0-7)
  LayerStream<kTPW, 1, kNG> ls;
  f32x4 wb0[kTPW], wb1[kTPW], wb2[kTPW];
  const __amdgpu_buffer_rsrc_t wrsrc = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<float4*>(p.wpack), (short)0, p.wpack_bytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t brsrc = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<float*>(p.mlp_b), (short)0, p.H * p.NT * 16 * 4, 0x00020000);
  const __amdgpu_buffer_rsrc_t frsrc = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<float*>(p.fc), (short)0, p.NT * 16 * 4, 0x00020000);
  TailStream<kNG> ts;
  constexpr int TT = kNG * kTPW;  // the split tile

  // ---- phase 0: descriptors, keys, shallow parameters in flight --------------------------------------------------
  typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
  constexpr int kDescPT = (7 * 64 + kNTH - 1) / kNTH;
  constexpr int kUpkPT = (kMaxMT * 16 * 16 + kNTH - 1) / kNTH;
  constexpr int kFwlwPT = (64 * 32 + kNTH - 1) / kNTH;
  u32x2 dw[QR ? kDescPT : 1];
  const float* rd_emb2[QR ? 1 : RPT];
  const float* rd_emb1[QR ? 1 : RPT];
  int64_t rd_n[QR ? 1 : RPT];
  if constexpr (!QR) {
#pragma unroll
    for (int k = 0; k < RPT; ++k) {
      const int f = (tid + k * kNTH) >> 4;
      rd_emb2[k] = rd_emb1[k] = nullptr;
      rd_n[k] = 0;
      if (f < F) {
        rd_emb2[k] = p.fields[f].emb2;
        rd_emb1[k] = p.fields[f].emb1;
        rd_n[k] = p.fields[f].n;
      }
    }
  } else {
#pragma unroll
    for (int k = 0; k < kDescPT; ++k) {
      const int i = tid + k * kNTH;
      if (i < 7 * F) dw[k] = reinterpret_cast<const u32x2*>(p.fields)[i];
    }
  }
  int64_t key[RPT];  // gather row r -> field f = r / 16, sample b = r % 16: index or Xv bits
#pragma unroll
  for (int k = 0; k < RPT; ++k) {
    const int r = tid + k * kNTH;
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
  const int n_upk = (flags & kHasSecond) ? p.MT * p.S * 16 : 0;
#pragma unroll
  for (int k = 0; k < kUpkPT; ++k) {
    const int i = tid + k * kNTH;
    if (i < n_upk) uw[k] = reinterpret_cast<const f32x4*>(p.upack)[i];
  }
  float fw[kFwlwPT];
  const int n_fwlw = (flags & kFoFwlw) ? FD : 0;
#pragma unroll
  for (int k = 0; k < kFwlwPT; ++k) {
    const int i = tid + k * kNTH;
    if (i < n_fwlw) fw[k] = p.fwlw[i];
  }
  const float lwv = ((flags & kFoLw) && tid < F) ? p.lw[tid] : 0.f;
  if (p.sv_keys != nullptr) {  // the sorted scatter's keys: the clamped categorical indices, column-major
#pragma unroll
    for (int k = 0; k < RPT; ++k) {
      const int r = tid + k * kNTH;
      const int f = r >> 4;
      const int64_t gb = b0 + (r & 15);
      if (f >= num && f < F && gb < p.batch) {
        int64_t n;
        if constexpr (QR) n = p.fields[f].n;
        else n = rd_n[k];
        p.sv_keys[(int64_t)(f - num) * p.keys_stride + gb] = (key[k] < 0 || key[k] >= n) ? 0 : (int32_t)key[k];
      }
    }
  }
  if constexpr (QR) {
#pragma unroll
    for (int k = 0; k < kDescPT; ++k) {
      const int i = tid + k * kNTH;
      if (i < 7 * F) reinterpret_cast<u32x2*>(desc)[i] = dw[k];
    }
    __syncthreads();
  }
  stamp(stamps, 1, tid);

  // ---- phase G: gather; E (and X_0) to LDS and, from the registers, to the workspace -----------------------------
  {
    const bool fo_tab = (flags & kFoTables) != 0;
    const float* pa[RPT];
    constexpr int RQ = QR ? RPT : 1;
    const float* pb[RQ];
    const float* qa[RPT];
    const float* qb[RQ];
    float scale[RPT];
    int mode[RPT];
    bool live[RPT];
#pragma unroll
    for (int k = 0; k < RPT; ++k) {
      const int r = tid + k * kNTH;
      const int f = r >> 4;
      live[k] = f < F && (b0 + (r & 15)) < p.batch;
      pa[k] = qa[k] = nullptr;
      if constexpr (QR) pb[k] = qb[k] = nullptr;
      scale[k] = 1.f;
      mode[k] = 0;
      if (!live[k]) continue;
      if constexpr (!QR) {
        if (f < num) {
          scale[k] = __int_as_float((int)key[k]);
          pa[k] = rd_emb2[k];
          qa[k] = rd_emb1[k];
        } else {
          int64_t idx = key[k];
          if (idx < 0 || idx >= rd_n[k]) {
            atomicOr(p.err, DFWFM_FLAG_INDEX_OUT_OF_RANGE);
            idx = 0;
          }
          pa[k] = rd_emb2[k] + idx * D;
          if (fo_tab) qa[k] = rd_emb1[k] + idx;
        }
      } else {
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
          if (fd.c == 0) {
            pa[k] = fd.emb2 + idx * D;
            if (fo_tab) qa[k] = fd.emb1 + idx;
          } else {
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
      if (live[k]) {
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
    // layer-0 weights behind the row loads (vmcnt retires in issue order)
    if (mlpw) {
      ls.init(wrsrc, 0, p.NC0, p.NT, g, 0);
      ls.preload(wb0, wb1, lane * 16);
    }
    // the dropout keep bits of this thread's X_0 row while the row loads are in flight
    uint32_t keep[RPT];
#pragma unroll
    for (int k = 0; k < RPT; ++k) {
      keep[k] = 0;
      const int r = tid + k * kNTH;
      if (drop && live[k]) {
#pragma unroll
        for (int d = 0; d < D; ++d)
          keep[k] |= dropout_keep(dseed, 0, b0 + (r & 15), (r >> 4) * D + d, p.drop_p) ? (1u << d) : 0u;
      }
    }
    // the shallow parameters to LDS
#pragma unroll
    for (int k = 0; k < kUpkPT; ++k) {
      const int i = tid + k * kNTH;
      if (i < n_upk) reinterpret_cast<f32x4*>(upk)[i] = uw[k];
    }
#pragma unroll
    for (int k = 0; k < kFwlwPT; ++k) {
      const int i = tid + k * kNTH;
      if (i < n_fwlw) fwlw_s[i] = fw[k];
    }
    if ((flags & kFoLw) && tid < F) lw_s[tid] = lwv;
    // zero the tiles' padding the MLP (NC0*16 columns) and the FwFM (S*4 fields) read
    const int w = p.W0 - FD;
    for (int i = tid; i < kBM * w; i += kNTH) {
      const int b = i / w;
      bufE[b * SX + FD + (i - b * w)] = 0.f;
      if (drop) bufX[b * SX + FD + (i - b * w)] = 0.f;
    }
#pragma unroll
    for (int k = 0; k < RPT; ++k) {
      const int r = tid + k * kNTH;
      const int f = r >> 4;
      const int b = r & 15;
      if (f < F) {
        float e[D];
#pragma unroll
        for (int d = 0; d < D; ++d) e[d] = live[k] ? combine(mode[k], va[k][d], QR ? vb[k][d] : 0.f, scale[k]) : 0.f;
        store_row<D>(bufE + b * SX + f * D, e);
        fo[b * Fp + f] = live[k] ? combine(mode[k], fa[k], QR ? fb[k] : 0.f, scale[k]) : 0.f;
        if (drop) {
          float x[D];
#pragma unroll
          for (int d = 0; d < D; ++d) x[d] = ((keep[k] >> d) & 1u) ? e[d] * p.drop_scale : 0.f;
          store_row<D>(bufX + b * SX + f * D, x);
        }
      }
    }
  }
  __syncthreads();  // B1
  stamp(stamps, 2, tid);
  stamp(stamps, 3, tid);

  if (mlpw) {
    // ---- MLP waves: fwd_kernel's static form, layer by layer ---------------------------------------------------
    const float* x0 = drop ? bufX : bufE;
    auto load_bias = [&](f32x4 (&bq)[kTPW], int h, int nq) {
#pragma unroll
      for (int j = 0; j < kTPW; ++j) {
        int t = g + kNG * j;
        t = t < p.NT ? t : p.NT - 1;
        bq[j] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(
                                              brsrc, nq * 4, __builtin_amdgcn_readfirstlane((h * p.NT + t) * 64), 0));
      }
    };
    f32x4 bq[kTPW];
    load_bias(bq, 0, 4 * (lane >> 4));
    // E and X_0 (== E without dropout, zero padding columns included) to the workspace before layer 1's K loop:
    // memory instructions the MLP waves issue while the matrix pipes are still free, so the helper waves run their
    // FwFM pieces at full issue rate meanwhile (beside the K loop they crawl)
    store_tile(p.sv_e + b0 * SE, SE, bufE, SX, nrows, SE / 4, tid, 64 * kNG);
    if (drop) store_tile(p.sv_x[0] + b0 * SE, SE, bufX, SX, nrows, SE / 4, tid, 64 * kNG);
    int layer_off = 0;
    for (int h = 0; h < H; ++h) {
      int lv = lane;
      asm volatile("" : "+v"(lv));
      const int rowl = lv & 15;
      const int nq = 4 * (lv >> 4);
      // layer h writes bufY (h even) or bufZ (h odd) and reads X_0 (h = 0) or the previous layer's output
      const float* in = h == 0 ? x0 : ((h & 1) ? bufY : bufZ);
      const int SA = h == 0 ? SX : SY;
      float* outa = (h & 1) ? bufZ : bufY;
      const int SO = SY;
      const int NC = h == 0 ? p.NC0 : p.NT;
      const bool last = h == H - 1;
      const int boff = __builtin_amdgcn_readfirstlane((h * p.NT + TT) * 64 + (g & 3) * 4);
      const int ntail = TT * 16 + nq + (g & 3);
      const float bn_t = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(brsrc, nq * 4, boff, 0));

      f32x4 acc[kTPW];
#pragma unroll
      for (int j = 0; j < kTPW; ++j) acc[j] = bq[j];
      ts.init(layer_off, NC, TT, g);
      f32x4 tp;
      if (!(flags & kFtDiagNoMlp))
        mlp_k_loop_s<kTPW, kNG, kNS, true>(acc, in, SA, ls, wb0, wb1, wb2, lane, ts, tp);
      else
        tp = f32x4{0.f, 0.f, 0.f, 0.f};
      reinterpret_cast<f32x4*>(tailr)[g * 64 + lane] = tp;
      if (h == 0) stamp(stamps, 12, tid);
      float dpart = 0.f;
      float* orow = outa + rowl * SO + nq;
#pragma unroll
      for (int j = 0; j < kTPW; ++j) {
        const int t = g + kNG * j;
        if (t < p.NT) {
          float v[4];
          if (t * 16 + 16 <= p.N) {
#pragma unroll
            for (int r = 0; r < 4; ++r) v[r] = relu_keep_nan(acc[j][r]);
          } else {
#pragma unroll
            for (int r = 0; r < 4; ++r) v[r] = nq + r < p.N - t * 16 ? relu_keep_nan(acc[j][r]) : 0.f;
          }
          if (drop) {
#pragma unroll
            for (int r = 0; r < 4; ++r)
              v[r] = dropout_keep(dseed, h + 1, b0 + rowl, t * 16 + nq + r, p.drop_p) ? v[r] * p.drop_scale : 0.f;
          }
          *reinterpret_cast<f32x4*>(orow + t * 16) = f32x4{v[0], v[1], v[2], v[3]};
          if (last) {
            // X_H to the workspace from the registers (the helpers copy the hidden layers' outputs from LDS)
            if (b0 + rowl < p.batch)
              *reinterpret_cast<f32x4*>(p.sv_x[H] + (b0 + rowl) * p.N + t * 16 + nq) = f32x4{v[0], v[1], v[2], v[3]};
            const f32x4 wf =
                __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(frsrc, nq * 4, t * 64, 0));
            dpart = fmaf(v[0], wf[0], dpart);
            dpart = fmaf(v[1], wf[1], dpart);
            dpart = fmaf(v[2], wf[2], dpart);
            dpart = fmaf(v[3], wf[3], dpart);
          }
        }
      }
      if (last) {
        dpart += __shfl_xor(dpart, 16);
        dpart += __shfl_xor(dpart, 32);
        if (lane < 16) dsum[g * kBM + rowl] = dpart;
      }
      layer_off += p.NT * NC * 64;
      if (!last) {
        ls.init(wrsrc, layer_off, p.NT, p.NT, g, 0);
        ls.preload(wb0, wb1, lane * 16);
        load_bias(bq, h + 1, nq);
      }
      if (h == 0) stamp(stamps, 13, tid);
      __syncthreads();  // A_h
      if (g < 4) {
        // the split tile: wave g < 4 finishes neuron TT*16 + nq + g of row rowl from the eight partials
        const bool valid = ntail < p.N;
        const float* tpp = tailr + lane * 4 + g;
        float sum = tpp[0];
#pragma unroll
        for (int w = 1; w < kNG; ++w) sum += tpp[w * 256];
        float v = valid ? relu_keep_nan(sum + bn_t) : 0.f;
        if (drop) v = dropout_keep(dseed, h + 1, b0 + rowl, ntail, p.drop_p) ? v * p.drop_scale : 0.f;
        outa[rowl * SO + nq + TT * 16 + g] = v;
        if (last) {
          if (valid && b0 + rowl < p.batch) p.sv_x[H][(b0 + rowl) * p.N + ntail] = v;
          const float wf_t = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(
                                                           frsrc, nq * 4, __builtin_amdgcn_readfirstlane(TT * 64 + g * 4), 0));
          float c = v * wf_t;
          c += __shfl_xor(c, 16);
          c += __shfl_xor(c, 32);
          if (lane < 16) taild[g * kBM + rowl] = c;
        }
      }
      __syncthreads();  // B_h
      stamp(stamps, 4 + (h < 3 ? h : 3), tid);
    }
  } else {
    // ---- helper waves --------------------------------------------------------------------------------------------
    const int hw = wave - kNG;
    const int htid = tid - 64 * kNG;
    // diagnostics: the first helper lane's phase clocks (slots 9, 10, 11, 7)
    auto hstamp = [&](int slot) {
      if (stamps != nullptr && htid == 0) stamps[(size_t)blockIdx.x * kStampSlots + slot] = __builtin_amdgcn_s_memtime();
    };
    // The helpers' work in the MLP's windows (each ends at the barrier after that layer's K loop + epilogue):
    //   [B1, A_0)       the FwFM pieces, fwlw first order (E and X_0 leave from the MLP waves before their K loop)
    //   [B_0, A_1)      first + second sums, the first order, X_1 (layer 3 overwrites it after B_1)
    //   [B_{h-1}, A_h)  X_h, h >= 2
    // (X_H leaves from the MLP waves' registers.)  The pieces (m, nt) are fwd_kernel PART 0's chains and sums, each
    // piece in the same order, per column tile nt with its MT row tiles' chains side by side on one E read per step.
    // The helpers run at the top priority: beside the two MLP waves of their SIMD (a saturated matrix pipe) their
    // instructions issue slowly -- the pieces took ~30k cycles there against ~11k alone, and at priority 0 the sums
    // stretched ~10x.
    __builtin_amdgcn_s_setprio(3);
    auto pieces = [&]() {
      if (!(flags & kHasSecond)) return;
      constexpr int MTC = 3, SM = 12;  // F <= 48
      const int S = p.S, MT = p.MT;
      for (int nt = hw; nt < D; nt += kNH) {
        const int n = nt * 16 + (lane & 15);
        const int b = n / D;
        const float* ecol = bufE + b * SX + (n - b * D);  // E[b][l][d] = ecol[l * D]
        f32x4 acc[MTC];
#pragma unroll
        for (int m = 0; m < MTC; ++m) acc[m] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int s0 = 0; s0 < SM; s0 += 4) {
          if (s0 < S) {
            float bv[4], av[4][MTC];
#pragma unroll
            for (int u = 0; u < 4; ++u) {
              const int s = s0 + u;
              bv[u] = ecol[(4 * (s < S ? s : 0) + (lane >> 4)) * D];
#pragma unroll
              for (int m = 0; m < MTC; ++m)  // unused fragments read a valid slot (no predicated loads)
                av[u][m] = 4 * m <= s ? upk[((m < MT && s < S) ? m * S + s : 0) * 64 + lane] : 0.f;
            }
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int u = 0; u < 4; ++u)
#pragma unroll
              for (int m = 0; m < MTC; ++m)
                if (4 * m <= s0 + u && m < MT && s0 + u < S)
                  acc[m] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[u][m], bv[u], acc[m], 0, 0, 0);
          }
        }
#pragma unroll
        for (int m = 0; m < MTC; ++m) {
          if (m < MT) {
            float v = 0.f;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              const int k = 16 * m + 4 * (lane >> 4) + r;
              const float e = ecol[(k < F ? k : 0) * D];
              v = fmaf(k < F ? e : 0.f, acc[m][r], v);
            }
            v += __shfl_xor(v, 16);
            v += __shfl_xor(v, 32);
            if (lane < 16) part2[(m * D + nt) * 16 + lane] = v;
          }
        }
      }
    };
    auto sums_and_saves = [&]() {
      {
        // first[b] and second[b] (fwd_kernel's sums): 16 lanes per sample, four samples per wave
        const int b = hw * 4 + (lane >> 4);
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
          const int MT = p.MT;
          for (int d = q; d < D; d += 16) {
            const int n = b * D + d;
            const float* pp = part2 + (n >> 4) * 16 + (n & 15);
            float v[4];
#pragma unroll
            for (int m = 0; m < 4; ++m) v[m] = pp[min(m, MT - 1) * D * 16];
#pragma unroll
            for (int m = 0; m < 4; ++m) second += m < MT ? v[m] : 0.f;
            for (int m = 4; m < MT; ++m) second += pp[m * D * 16];
          }
        }
        first = sum16(first);
        second = sum16(second);
        if (q == 0) fs[b] = first + second;
      }
      // the first order per field
      for (int i = htid; i < kBM * F; i += kHTH) {
        const int b = i / F;
        if (b < nrows) p.sv_fo[(b0 + b) * F + (i - b * F)] = fo[b * Fp + (i - b * F)];
      }
    };
    pieces();
    hstamp(10);
    if (flags & kFoFwlw) {
      for (int r = htid; r < kBM * F; r += kHTH) {
        const int f = r >> 4;
        const int b = r & 15;
        const float* e = bufE + b * SX + f * D;
        const float* w = fwlw_s + f * D;
        float s = 0.f;
#pragma unroll
        for (int d = 0; d < D; ++d) s += e[d] * w[d];
        fo[b * Fp + f] = s;
      }
    }
    hstamp(9);
    __syncthreads();  // A_0
    __syncthreads();  // B_0
    for (int h = 1; h < H; ++h) {
      if (h == 1) sums_and_saves();
      // X_h (layer h - 1's output, complete at B_{h-1}; layer h + 1 overwrites it after B_h)
      store_tile(p.sv_x[h] + b0 * p.N, p.N, (h & 1) ? bufY : bufZ, SY, nrows, p.N / 4, htid, kHTH);
      if (h <= 2) hstamp(h == 1 ? 11 : 7);
      __syncthreads();  // A_h
      __syncthreads();  // B_h
    }
    if (H == 1) sums_and_saves();
  }
  __syncthreads();  // C: fs, dsum and the split tile's shares are complete
  if (tid < kBM && b0 + tid < p.batch) {
    float deepv = dsum[tid];
#pragma unroll
    for (int w = 1; w < kNG; ++w) deepv += dsum[w * kBM + tid];
    deepv += ((taild[tid] + taild[kBM + tid]) + taild[2 * kBM + tid]) + taild[3 * kBM + tid];
    tr.out[b0 + tid] = (fs[tid] + deepv) + p.bias[0];
  }
  stamp(stamps, 8, tid);
  stamp_end_rt(stamps, tid);
}

size_t ftrain_lds_bytes(int F, int D, int MT, int S, int SX, int SY) {
  return sizeof(float) * (size_t)ldst_layout(F, D, MT, S, SX, SY).total;
}

bool ftrain_supported(int F, int D, int H, int NT, int NC0, int tailI, int NG) {
  return D == 10 && F <= 48 && H >= 1 && NT == kNS && NC0 == kNS && tailI == 1 && NG == kNG;
}

hipError_t launch_ftrain(const FwdArgs& a, int D, size_t lds, hipStream_t s) {
  if (D != 10 || a.nb > 1) return hipErrorInvalidValue;
  auto k = (a.flags & kHasQR) ? ftrain_kernel<10, true> : ftrain_kernel<10, false>;
  hipError_t e = ensure_lds_limit(reinterpret_cast<const void*>(k), lds);
  if (e != hipSuccess) return e;
  const unsigned grid = (unsigned)((a.batch + kBM - 1) / kBM);
  hipLaunchKernelGGL(k, dim3(grid), dim3(kNTH), lds, s, a);
  return hipGetLastError();
}

}  // namespace dfwfm
