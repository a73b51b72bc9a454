// dfwfm_fwd32.hip -- the fused DeepFwFM forward on 32-sample workgroups (two 16-row MFMA tiles per wave).
//
// Same phases and the same arithmetic as fwd_kernel's static 3x400 form (dfwfm_kernels.hip, reference
// model/DeepFMs.py:285-469) -- gather, first order, FwFM second order on MFMA, the MLP on
// v_mfma_f32_16x16x4_f32 with the weights as the A operand, combine -- but every wave carries BOTH 16-row
// tiles of its workgroup through the MLP: each 1 KiB weight fragment it streams from L2 feeds 8 MFMAs instead
// of 4, so the L2 -> CU weight bytes per FLOP halve (tools/ubench_m32.hip: the K loop + epilogue at 0.93 of the
// f32 MFMA peak against 0.86 with 16-row tiles).  The activations live in ONE LDS tile updated in place (a
// barrier between a layer's K loop and its epilogue), and the shallow phase's scratch is reused for the MLP's
// split-tile partials, so a workgroup takes ~70 KB of LDS and two share a CU.
//
// Per sample the summation order equals fwd_kernel's (same K order onto the bias, same split-tail partials in
// wave order, same FwFM pieces per 16-row half, same sums): the logits are bit-identical to it.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "dfwfm_device.h"
#include "dfwfm_internal.h"

namespace dfwfm {

namespace {

constexpr int kRT = 2;           // 16-row tiles per workgroup
constexpr int kRows = 16 * kRT;  // samples per workgroup
constexpr int kNG = 8;           // waves (output-tile groups), two per SIMD
constexpr int kTPW = 3;          // whole output tiles per wave: 25 = 8 x 3 + the split 25th
constexpr int kNS = 25;          // K chunks of every layer (static K loop)
constexpr int kNTH = 64 * kNG;

// the activation tile (in place), the sums that live to the end, and a scratch region used first by the shallow
// phase (descriptors, lw, fwlw, FwFM fragments, first order, FwFM piece sums) and then by the MLP's split tile
struct Lds32 {
  int buf, fs, dsum, desc, lw, fwlw, upk, fo, part2, tailr, taild, total;
};

__host__ __device__ inline Lds32 lds32_layout(int F, int D, int MT, int S, int SX) {
  Lds32 L;
  int o = 0;
  L.buf = o;   o += kRows * SX;
  L.fs = o;    o += kRows;
  L.dsum = o;  o += kNG * kRows;
  int s = o;
  L.desc = s;  s += r4(14 * F);
  L.lw = s;    s += r4(F);
  L.fwlw = s;  s += r4(F * D);
  L.upk = s;   s += MT * S * 64;
  L.fo = s;    s += kRows * r4(F);
  L.part2 = s; s += kRT * MT * D * 16;
  int t = o;
  L.tailr = t; t += kNG * kRT * 64 * 4;  // [wave][row tile][lane][4] partial products of the split tile
  L.taild = t; t += 4 * kRows;           // [wave < 4][row] the split tile's share of deep[row]
  L.total = r4(s > t ? s : t);
  return L;
}

// one K chunk of both row tiles: weights the A operand (lane: four consecutive outputs of one sample)
template <int TPW, int RT>
__device__ __forceinline__ void mfma_chunk_rt(f32x4 (&acc)[RT][TPW], const float4 (&a)[RT], const f32x4 (&w)[TPW]) {
#pragma unroll
  for (int s = 0; s < 4; ++s)
#pragma unroll
    for (int rt = 0; rt < RT; ++rt)
#pragma unroll
      for (int j = 0; j < TPW; ++j) {
        const float av = s == 0 ? a[rt].x : (s == 1 ? a[rt].y : (s == 2 ? a[rt].z : a[rt].w));
        acc[rt][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(w[j][s], av, acc[rt][j], 0, 0, 0);
      }
}

// mlp_k_loop_s for RT row tiles: the NS-chunk static K loop with three rotating weight / activation register
// sets, refills two chunks ahead, and the wave's share of the split tile riding on the sets the last two steps
// free (multiplied after the loop into tp[rt])
template <int TPW, int RT, int NG, int NS>
__device__ __forceinline__ void k_loop_rt(f32x4 (&acc)[RT][TPW], const float* __restrict__ act, int SA,
                                          const LayerStream<TPW, 1, NG>& ls, f32x4 (&b0)[TPW], f32x4 (&b1)[TPW],
                                          f32x4 (&b2)[TPW], int lane, const TailStream<NG>& ts, f32x4 (&tp)[RT],
                                          bool mid_barrier) {
  const int voff = lane * 16;
  const float* arow = act + (lane & 15) * SA + 4 * (lane >> 4);
  float4 a0[RT], a1[RT], a2[RT];
#pragma unroll
  for (int rt = 0; rt < RT; ++rt) {
    a0[rt] = *reinterpret_cast<const float4*>(arow + rt * 16 * SA);
    a1[rt] = *reinterpret_cast<const float4*>(arow + rt * 16 * SA + 16);
  }
#pragma unroll
  for (int i = 0; i < NS; ++i) {
    f32x4 (&X)[TPW] = (i % 3 == 0) ? b0 : ((i % 3 == 1) ? b1 : b2);
    f32x4 (&Z)[TPW] = (i % 3 == 0) ? b2 : ((i % 3 == 1) ? b0 : b1);
    float4 (&AX)[RT] = (i % 3 == 0) ? a0 : ((i % 3 == 1) ? a1 : a2);
    float4 (&AZ)[RT] = (i % 3 == 0) ? a2 : ((i % 3 == 1) ? a0 : a1);
    if (i + 3 == NS && mid_barrier) __syncthreads();  // the previous layer's split tile (chunk NS - 1) is written
    if (i + 2 < NS) {
#pragma unroll
      for (int rt = 0; rt < RT; ++rt) AZ[rt] = *reinterpret_cast<const float4*>(arow + rt * 16 * SA + 16 * (i + 2));
      ls.load(Z, ls.c0 + i + 2, voff);
    } else {
      ts.template load_set<TPW>(ls.rsrc, Z, i + 2 == NS ? 0 : TPW, voff);
    }
    mfma_chunk_rt<TPW, RT>(acc, AX, X);
    __builtin_amdgcn_sched_group_barrier(0x100, RT, 0);
    for (int q = 0; q < TPW; ++q) {
      __builtin_amdgcn_sched_group_barrier(0x008, 2 * RT, 0);
      __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);
    }
    __builtin_amdgcn_sched_group_barrier(0x008, 2 * RT * TPW, 0);
    __builtin_amdgcn_sched_barrier(0);
  }
  // the split tile: fragments [0, TPW) in the set of step NS, [TPW, 2 TPW) in the set of step NS + 1; two
  // accumulators per row tile by chunk parity (no back-to-back dependent MFMAs), like TailStream::mma_set
  f32x4 c0[RT], c1[RT];
#pragma unroll
  for (int rt = 0; rt < RT; ++rt) c0[rt] = c1[rt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int half = 0; half < 2; ++half) {
    const f32x4 (&B)[TPW] = ((NS + half) % 3 == 0) ? b0 : (((NS + half) % 3 == 1) ? b1 : b2);
#pragma unroll
    for (int j = 0; j < TPW; ++j) {
      const int u = half * TPW + j;
      if (u < ts.cnt) {
#pragma unroll
        for (int rt = 0; rt < RT; ++rt) {
          const float4 a = *reinterpret_cast<const float4*>(arow + rt * 16 * SA + 16 * (ts.c_lo + u));
          f32x4& c = (u & 1) ? c1[rt] : c0[rt];
          c = __builtin_amdgcn_mfma_f32_16x16x4f32(B[j].x, a.x, c, 0, 0, 0);
          c = __builtin_amdgcn_mfma_f32_16x16x4f32(B[j].y, a.y, c, 0, 0, 0);
          c = __builtin_amdgcn_mfma_f32_16x16x4f32(B[j].z, a.z, c, 0, 0, 0);
          c = __builtin_amdgcn_mfma_f32_16x16x4f32(B[j].w, a.w, c, 0, 0, 0);
        }
      }
    }
  }
#pragma unroll
  for (int rt = 0; rt < RT; ++rt) tp[rt] = c0[rt] + c1[rt];
}

}  // namespace

// QR: some field may be a QR embedding (false: no second operand, row descriptors loaded directly with the keys)
template <int D, bool QR>
__global__ void __launch_bounds__(kNTH) __attribute__((amdgpu_waves_per_eu(4)))
fwd32_kernel(FwdArgs p) {
  constexpr int RPT = (kRows * 48 + kNTH - 1) / kNTH;  // gather rows per thread: F <= 48
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int F = p.F;
  const int num = p.num;
  const int SX = p.SX;
  const int flags = p.flags;
  const int Fp = r4(F);
  const Lds32 L = lds32_layout(F, D, p.MT, p.S, SX);
  float* buf = smem + L.buf;
  float* fs = smem + L.fs;
  float* dsum = smem + L.dsum;
  FieldDev* desc = reinterpret_cast<FieldDev*>(smem + L.desc);
  float* lw_s = smem + L.lw;
  float* fwlw_s = smem + L.fwlw;
  float* upk = smem + L.upk;
  float* fo = smem + L.fo;
  float* part2 = smem + L.part2;
  float* tailr = smem + L.tailr;
  float* taild = smem + L.taild;
  const TileRef tr = tile_ref<kRows>(p);  // batch set: this workgroup's batch
  const int64_t b0 = tr.b0;
  stamp(p.stamps, 0, tid);
  stamp_start_rt(p.stamps, tid);
  if (flags & kPrio) __builtin_amdgcn_s_setprio(1);
  const int g = wave;

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

  // ---- phase 0: descriptors (QR: staged in LDS; else loaded by each thread with its keys), keys, shallow
  // parameters in flight -------------------------------------------------------------------------------------
  typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
  constexpr int kDescPT = (7 * 64 + kNTH - 1) / kNTH;
  constexpr int kUpkPT = (kMaxMT * 16 * 16 + kNTH - 1) / kNTH;
  constexpr int kFwlwPT = (64 * 32 + kNTH - 1) / kNTH;
  u32x2 dw[QR ? kDescPT : 1];
  const float* rd_emb2[QR ? 1 : RPT];
  const float* rd_emb1[QR ? 1 : RPT];
  int64_t rd_n[QR ? 1 : RPT];
  // the tables' serving copy (dfwfm_model_pack_tables): a categorical row and its first-order weight in one row
  bool pkrow[QR ? 1 : RPT];
  if constexpr (!QR) {
#pragma unroll
    for (int k = 0; k < RPT; ++k) {
      const int f = (tid + k * kNTH) >> 5;
      rd_emb2[k] = rd_emb1[k] = nullptr;
      rd_n[k] = 0;
      pkrow[k] = p.pkw != 0 && f >= num && f < F;
      if (f < F) {
        rd_emb2[k] = pkrow[k] ? p.pk[f] : p.fields[f].emb2;
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
  int64_t key[RPT];  // gather row r -> field f = r / 32, sample b = r % 32: index or Xv bits
#pragma unroll
  for (int k = 0; k < RPT; ++k) {
    const int r = tid + k * kNTH;
    const int f = r >> 5;
    const int64_t gb = b0 + (r & 31);
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
  const int n_fwlw = (flags & kFoFwlw) ? F * D : 0;
#pragma unroll
  for (int k = 0; k < kFwlwPT; ++k) {
    const int i = tid + k * kNTH;
    if (i < n_fwlw) fw[k] = p.fwlw[i];
  }
  const float lwv = ((flags & kFoLw) && tid < F) ? p.lw[tid] : 0.f;
  if constexpr (QR) {
#pragma unroll
    for (int k = 0; k < kDescPT; ++k) {
      const int i = tid + k * kNTH;
      if (i < 7 * F) reinterpret_cast<u32x2*>(desc)[i] = dw[k];
    }
    __syncthreads();
  }
  stamp(p.stamps, 1, tid);

  // ---- phase G: gather the E rows (both 16-row tiles) and the table first order --------------------------------
  {
    const bool needE = (flags & kNeedE) != 0;
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
      const int f = r >> 5;
      live[k] = f < F && (b0 + (r & 31)) < p.batch;
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
          if (pkrow[k]) {
            pa[k] = rd_emb2[k] + idx * p.pkw;
          } else {
            pa[k] = rd_emb2[k] + idx * D;
            if (fo_tab) qa[k] = rd_emb1[k] + idx;
          }
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
      if (!QR && live[k] && pkrow[QR ? 0 : k]) {  // second and first order in one aligned row
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
    // layer-0 weights behind the row loads (vmcnt retires in issue order)
    ls.init(wrsrc, 0, p.NC0, p.NT, g, 0);
    ls.preload(wb0, wb1, lane * 16);
    // the shallow parameters to LDS while the row loads are in flight
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
    // zero the E-tile padding the MLP (NC0*16 columns) and the FwFM (S*4 fields) read
    const int w = p.W0 - F * D;
    for (int i = tid; i < kRows * w; i += kNTH) {
      const int b = i / w;
      buf[b * SX + F * D + (i - b * w)] = 0.f;
    }
#pragma unroll
    for (int k = 0; k < RPT; ++k) {
      const int r = tid + k * kNTH;
      const int f = r >> 5;
      const int b = r & 31;
      if (f < F) {
        if (needE) {
          float e[D];
#pragma unroll
          for (int d = 0; d < D; ++d) e[d] = live[k] ? combine(mode[k], va[k][d], QR ? vb[k][d] : 0.f, scale[k]) : 0.f;
          store_row<D>(buf + b * SX + f * D, e);
        }
        fo[b * Fp + f] = live[k] ? combine(mode[k], fa[k], QR ? fb[k] : 0.f, scale[k]) : 0.f;
      }
    }
  }
  __syncthreads();
  stamp(p.stamps, 2, tid);

  // ---- phase S: first order (fwlw) and the FwFM second order, per 16-row half as fwd_kernel's pieces -------
  if (flags & kFoFwlw) {
    for (int r = tid; r < kRows * F; r += kNTH) {
      const int f = r >> 5;
      const int b = r & 31;
      const float* e = buf + b * SX + f * D;
      const float* w = fwlw_s + f * D;
      float s = 0.f;
#pragma unroll
      for (int d = 0; d < D; ++d) s += e[d] * w[d];
      fo[b * Fp + f] = s;
    }
  }
  stamp(p.stamps, 9, tid);
  if (flags & kHasSecond) {
    // both 16-row halves of a piece at once: one U fragment read feeds two independent MFMA chains (each chain's
    // order is fwd_kernel's, so the sums are the same bits), which halves this phase's dependent latency
    const int S = p.S;
    const int MTD = p.MT * D;
    const int p_lo = p.fw_off8[wave], p_hi = p.fw_off8[wave + 1];
    for (int pi = p_lo; pi < p_hi; ++pi) {
      const int pc = p.fw_list8[pi];
      const int m = pc / D;
      const int nt = pc - m * D;
      const int n = nt * 16 + (lane & 15);
      const int b = n / D;
      const float* ecol0 = buf + b * SX + (n - b * D);  // E[b][l][d] = ecol0[l * D]; the second half 16 rows on
      const float* ecol1 = ecol0 + 16 * SX;
      const float* ua = upk + m * S * 64 + lane;
      f32x4 acc0 = f32x4{0.f, 0.f, 0.f, 0.f}, acc1 = acc0;
      auto group = [&](int s0, auto U_) {
        constexpr int U = decltype(U_)::value;
        float av[U], bv0[U], bv1[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const int l = (4 * (s0 + u) + (lane >> 4)) * D;
          av[u] = ua[(s0 + u) * 64];
          bv0[u] = ecol0[l];
          bv1[u] = ecol1[l];
        }
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int u = 0; u < U; ++u) {
          acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(av[u], bv0[u], acc0, 0, 0, 0);
          acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(av[u], bv1[u], acc1, 0, 0, 0);
        }
      };
      int s0 = 4 * m;
      for (; s0 + 4 <= S; s0 += 4) group(s0, std::integral_constant<int, 4>{});
      const int rem = S - s0;
      if (rem == 3) group(s0, std::integral_constant<int, 3>{});
      else if (rem == 2) group(s0, std::integral_constant<int, 2>{});
      else if (rem == 1) group(s0, std::integral_constant<int, 1>{});
      float v0 = 0.f, v1 = 0.f;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int k = 16 * m + 4 * (lane >> 4) + r;
        const int kk = (k < F ? k : 0) * D;
        v0 = fmaf(k < F ? ecol0[kk] : 0.f, acc0[r], v0);
        v1 = fmaf(k < F ? ecol1[kk] : 0.f, acc1[r], v1);
      }
      v0 += __shfl_xor(v0, 16);
      v1 += __shfl_xor(v1, 16);
      v0 += __shfl_xor(v0, 32);
      v1 += __shfl_xor(v1, 32);
      if (lane < 16) {
        part2[pc * 16 + lane] = v0;
        part2[(MTD + pc) * 16 + lane] = v1;
      }
    }
  }
  stamp(p.stamps, 10, tid);
  __syncthreads();
  stamp(p.stamps, 11, tid);
  {
    // first[b] (lw projection or plain sum) and second[b]: 16 lanes per sample, every 16th term, then a 16-lane
    // DPP sum -- eight waves x four samples = the 32 rows.  All LDS reads issue before the first add (no chain
    // of dependent LDS round trips, see fwd_kernel's sums).
    const int b = wave * 4 + (lane >> 4);
    const int h = b >> 4;
    const int bl = b & 15;
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
        const int n = bl * D + d;
        const float* pp = part2 + (h * MT * D + (n >> 4)) * 16 + (n & 15);  // + m * D * 16 for row tile m
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
  stamp(p.stamps, 3, tid);
  if (flags & kPrio) __builtin_amdgcn_s_setprio(0);

  // ---- phase M: the MLP on MFMA, both row tiles per wave, activations in place --------------------------------
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
  int layer_off = 0;
  for (int h = 0; h < p.H; ++h) {
    int lv = lane;
    asm volatile("" : "+v"(lv));
    const int rowl = lv & 15;
    const int nq = 4 * (lv >> 4);
    const int NC = h == 0 ? p.NC0 : p.NT;
    const bool last = h == p.H - 1;
    const int boff = __builtin_amdgcn_readfirstlane((h * p.NT + TT) * 64 + (g & 3) * 4);
    const int ntail = TT * 16 + nq + (g & 3);
    const float bn_t = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(brsrc, nq * 4, boff, 0));

    f32x4 acc[kRT][kTPW];
#pragma unroll
    for (int rt = 0; rt < kRT; ++rt)
#pragma unroll
      for (int j = 0; j < kTPW; ++j) acc[rt][j] = bq[j];
    ts.init(layer_off, NC, TT, g);
    f32x4 tp[kRT];
    // kDeferTail: the barrier after the split tile's reduction waits inside this K loop, right before chunk NS - 1
    // (the split tile's columns) is read -- until then the waves that did not reduce run their MFMAs
    k_loop_rt<kTPW, kRT, kNG, kNS>(acc, buf, SX, ls, wb0, wb1, wb2, lane, ts, tp, h > 0 && (flags & kDeferTail));
    if (flags & kPrioEpi) __builtin_amdgcn_s_setprio(1);
    if (h == 0) stamp(p.stamps, 12, tid);
    __syncthreads();  // every wave has read the layer's input: the tile may be overwritten
#pragma unroll
    for (int rt = 0; rt < kRT; ++rt) reinterpret_cast<f32x4*>(tailr)[(g * kRT + rt) * 64 + lane] = tp[rt];
    float dpart[kRT] = {0.f, 0.f};
#pragma unroll
    for (int rt = 0; rt < kRT; ++rt) {
      float* orow = buf + (rt * 16 + rowl) * SX + nq;
#pragma unroll
      for (int j = 0; j < kTPW; ++j) {
        const int t = g + kNG * j;
        float v[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] = relu_keep_nan(acc[rt][j][r]);
        if (!last) {
          *reinterpret_cast<f32x4*>(orow + t * 16) = f32x4{v[0], v[1], v[2], v[3]};
        } else {
          const f32x4 wf = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(frsrc, nq * 4, t * 64, 0));
          dpart[rt] = fmaf(v[0], wf[0], dpart[rt]);
          dpart[rt] = fmaf(v[1], wf[1], dpart[rt]);
          dpart[rt] = fmaf(v[2], wf[2], dpart[rt]);
          dpart[rt] = fmaf(v[3], wf[3], dpart[rt]);
        }
      }
    }
    if (last) {
#pragma unroll
      for (int rt = 0; rt < kRT; ++rt) {
        float d = dpart[rt];
        d += __shfl_xor(d, 16);
        d += __shfl_xor(d, 32);
        if (lane < 16) dsum[g * kRows + rt * 16 + rowl] = d;
      }
    }
    layer_off += p.NT * NC * 64;
    if (!last) {  // the next layer's first chunks and biases, ahead of the barrier (after the epilogue)
      ls.init(wrsrc, layer_off, p.NT, p.NT, g, 0);
      ls.preload(wb0, wb1, lane * 16);
      load_bias(bq, h + 1, nq);
    }
    if (h == 0) stamp(p.stamps, 13, tid);
    __syncthreads();
    // the split tile: wave g < 4 finishes neuron TT*16 + nq + g of both rows tiles' row rowl from the kNG partials
    if (g < 4) {
      const bool valid = ntail < p.N;
      float wf_t = 0.f;
      if (last)
        wf_t = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(
                                             frsrc, nq * 4, __builtin_amdgcn_readfirstlane(TT * 64 + g * 4), 0));
#pragma unroll
      for (int rt = 0; rt < kRT; ++rt) {
        const float* tpp = tailr + (rt * 64 + lane) * 4 + g;
        float sum = tpp[0];
#pragma unroll
        for (int w = 1; w < kNG; ++w) sum += tpp[w * kRT * 256];
        const float v = valid ? relu_keep_nan(sum + bn_t) : 0.f;
        if (!last) {
          buf[(rt * 16 + rowl) * SX + TT * 16 + nq + g] = v;
        } else {
          float c = v * wf_t;
          c += __shfl_xor(c, 16);
          c += __shfl_xor(c, 32);
          if (lane < 16) taild[g * kRows + rt * 16 + rowl] = c;
        }
      }
    }
    if (last || !(flags & kDeferTail)) __syncthreads();
    if (flags & kPrioEpi) __builtin_amdgcn_s_setprio(0);
    stamp(p.stamps, 4 + (h < 3 ? h : 3), tid);
  }

  if (tid < kRows && b0 + tid < p.batch) {
    float deepv = dsum[tid];
#pragma unroll
    for (int w = 1; w < kNG; ++w) deepv += dsum[w * kRows + tid];
    deepv += ((taild[tid] + taild[kRows + tid]) + taild[2 * kRows + tid]) + taild[3 * kRows + tid];
    tr.out[b0 + tid] = (fs[tid] + deepv) + p.bias[0];
  }
  stamp(p.stamps, 8, tid);
  stamp_end_rt(p.stamps, tid);
}

size_t fwd32_lds_bytes(int F, int D, int MT, int S, int SX) {
  return sizeof(float) * (size_t)lds32_layout(F, D, MT, S, SX).total;
}

bool fwd32_supported(int F, int D, int H, int NT, int NC0, int tailI, int NG) {
  return D == 10 && F <= 48 && H >= 1 && NT == kNS && NC0 == kNS && tailI == 1 && NG == kNG;
}

hipError_t launch_fwd32(const FwdArgs& a, int D, size_t lds, hipStream_t s) {
  if (D != 10) return hipErrorInvalidValue;
  auto k = (a.flags & kHasQR) ? fwd32_kernel<10, true> : fwd32_kernel<10, false>;
  hipError_t e = ensure_lds_limit(reinterpret_cast<const void*>(k), lds);
  if (e != hipSuccess) return e;
  const unsigned grid = fwd_grid(a, kRows);
  hipLaunchKernelGGL(k, dim3(grid), dim3(kNTH), lds, s, a);
  return hipGetLastError();
}

}  // namespace dfwfm
