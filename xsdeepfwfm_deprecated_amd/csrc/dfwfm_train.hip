// dfwfm_train.hip -- CDNA4 (gfx950) kernels of the DeepFwFM training step
// (reference model/DeepFMs.py:553-637: loss.backward() and Adam(weight_decay=l2).step()).
//
// Every gradient is a sum over the batch; the kernels are split by how that sum is formed, so that
// no address receives more than a few dozen atomic adds (256-way contended device atomics cost more
// than the rest of the step together):
//   bwd_kernel      per 16-sample tile, no atomics: dE of the FwFM term ((R+R^T)/2 * E on MFMA)
//                   and of fwlw, the MLP input-gradient chain dX_{l-1} = G_l W_l on MFMA (the
//                   forward's weight-streaming loop over transposed packs) with ReLU / dropout masks
//                   from the saved layer outputs; G_l and dE go to the workspace.
//   reduce_kernel   dense shallow grads over 64-row blocks: bias, fm_1st, fwfm_linear, field_cov (a
//                   dlogit-weighted Gram matrix on MFMA), net_1_fc, the numerical fields' tables.
//   scatter_kernel  dE / dfo into the categorical tables' dense grads (nn.Embedding(sparse=False)):
//                   small tables accumulate privately in LDS, large ones take global atomics.
//   dwr_kernel      dW_l += G_l^T X_{l-1} and db_l += sum G_l for all layers in one launch.
//   adam_kernel     torch.optim.Adam's update (coupled L2, bias correction) over a tensor list.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string.h>

#include "dfwfm_device.h"
#include "dfwfm_internal.h"

namespace dfwfm {

struct BwdLds {
  int lw, fwlw, rsk, bufE, bufD, bufA, dl, fc, tailr, fo, xv, gram, total;
};

__host__ __device__ inline BwdLds bwd_layout(int F, int D, int MT, int S, int SX, int SY) {
  BwdLds L;
  int o = 0;
  L.lw = o;    o += r4(F);
  L.fwlw = o;  o += r4(F * D);
  L.rsk = o;   o += MT * S * 64;
  L.bufE = o;  o += kBM * (SX > SY ? SX : SY);  // E tile; reused as the second G buffer
  L.bufD = o;  o += kBM * SX;                   // dE tile
  // G buffer; until P2 stores X_H into it, it holds the field_cov Gram's chains (P1 -> the reduction after it)
  L.bufA = o;  o += kBM * SY > 2 * MT * MT * 256 ? kBM * SY : 2 * MT * MT * 256;
  L.gram = L.bufA;
  L.dl = o;    o += kBM;
  L.fc = o;    o += SY;                       // net_1_fc (G_H = dlogit * fc * mask)
  L.tailr = o; o += 8 * 64 * 4;               // split-tail partial products (eight waves)
  L.fo = o;    o += kBM * r4(F);              // fused reductions: first order per field
  L.xv = o;    o += kBM * r4(F);              //                   numerical values (num <= F)
  L.total = r4(o);
  return L;
}

#ifndef DFWFM_KD
size_t backward_lds_bytes(int F, int D, int MT, int S, int SX, int SY) {
  return sizeof(float) * (size_t)bwd_layout(F, D, MT, S, SX, SY).total;
}
#endif

// NG: waves = output-tile groups of the MLP chain.  4: one wave per SIMD, TPW tiles each; 8: two
// per SIMD (256 registers, one workgroup per CU) with the 8*TPW+1-th tile of a layer split by K over
// the eight waves (tail), as in the forward.
template <int D, int TPW, int NG>
__global__ void __launch_bounds__(64 * NG) __attribute__((amdgpu_waves_per_eu(NG == 8 ? 2 : 1)))
bwd_kernel(BwdArgs p) {
  constexpr int NTH = 64 * NG;
  constexpr int NW = NG;
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int F = p.F, SX = p.SX, SY = p.SY, FD = F * D;
  const int flags = p.flags;
  const bool deep = (flags & kHasDeep) != 0;
  const bool second = (flags & kHasSecond) != 0;
  const bool fwlw = (flags & kFoFwlw) != 0;
  const bool lwp = (flags & kFoLw) != 0;
  const bool drop = (flags & kDrop) != 0;
  const BwdLds L = bwd_layout(F, D, p.MT, p.S, SX, SY);
  float* lw_s = smem + L.lw;
  float* fwlw_s = smem + L.fwlw;
  float* rsk = smem + L.rsk;
  float* bufE = smem + L.bufE;
  float* bufD = smem + L.bufD;
  float* bufA = smem + L.bufA;
  float* bufB = bufE;  // the E tile is dead once the shallow dE is formed
  float* dl = smem + L.dl;
  float* fc_s = smem + L.fc;
  float* tailr = smem + L.tailr;
  const int64_t b0 = (int64_t)blockIdx.x * kBM;
  const int row0 = (lane >> 4) * 4;
  const int nrows = (int)((p.batch - b0) < kBM ? (p.batch - b0) : kBM);

  // ---- P0: stage --------------------------------------------------------------
  // every global read of the phase is issued before the first LDS store (one round trip instead of one per staging
  // loop); X_H's reads go out too, but land in LDS (bufA, which P1 leaves alone) only after P1
  stamp(p.stamps, 0, tid);
  stamp_rt(p.stamps, 10, tid);
  const int red = p.red;
  float* fo_s = smem + L.fo;
  float* xv_s = smem + L.xv;
  const int num = p.num, Fp = r4(F);
  const int64_t b0f = b0 * F;
  const float* xvb = p.xv + b0 * p.xv_stride;
  auto get_lw = [&](int i) { return p.lw[i]; };
  auto get_fwlw = [&](int i) { return p.fwlw[i]; };
  auto get_fc = [&](int i) { return p.fc[i]; };
  const bool bce = p.bce_z != nullptr;
  auto get_dl = [&](int i) { return b0 + i < p.batch ? (bce ? p.bce_z : p.dlogit)[b0 + i] : 0.f; };
  auto get_y = [&](int i) { return b0 + i < p.batch ? p.bce_y[b0 + i] : 0.f; };
  auto get_fo = [&](int i) {
    const int b = i / F;
    return b < nrows ? p.sv_fo[b0f + i] : 0.f;
  };
  auto get_xv = [&](int i) {
    const int b = i / num;
    return b < nrows ? xvb[b * p.xv_stride + (i - b * num)] : 0.f;
  };
  auto get_rsk = [&](int i) { return reinterpret_cast<const f32x4*>(p.rsk)[i]; };
  const int n_lw = lwp ? F : 0, n_fwlw = fwlw ? FD : 0, n_rsk = second ? p.MT * p.S * 16 : 0;
  const int n_fo = (red & kRedLw) ? kBM * F : 0, n_xv = red ? kBM * num : 0, n_fc = deep ? p.NT * 16 : 0;
  float v_lw[1], v_fwlw[1], v_fc[1], v_dl[1], v_y[1], v_fo[2], v_xv[1];
  f32x4 v_rsk[1], v_e[4], v_x[4];
  stage_load<1>(v_lw, n_lw, tid, NTH, get_lw);
  stage_load<1>(v_fwlw, n_fwlw, tid, NTH, get_fwlw);
  stage_load<1>(v_rsk, n_rsk, tid, NTH, get_rsk);
  stage_load<1>(v_dl, kBM, tid, NTH, get_dl);
  stage_load<1>(v_y, bce ? kBM : 0, tid, NTH, get_y);
  stage_load<2>(v_fo, n_fo, tid, NTH, get_fo);
  stage_load<1>(v_xv, n_xv, tid, NTH, get_xv);
  stage_load<1>(v_fc, n_fc, tid, NTH, get_fc);
  // the E tile: rows of r4(F*D) floats (zero past F*D), zero-padded to W0 columns; X_H: N columns padded to NT*16
  const float* xh_g = deep ? p.sv_x[p.H] + b0 * p.N : nullptr;
  tile_load<4>(v_e, p.sv_e + b0 * r4(FD), r4(FD), second ? nrows : 0, r4(FD) / 4, p.W0 / 4, tid, NTH);
  if (deep) tile_load<4>(v_x, xh_g, p.N, nrows, p.N / 4, p.NT * 4, tid, NTH);
  stage_store<1>(v_lw, n_lw, tid, NTH, get_lw, [&](int i, float v) { lw_s[i] = v; });
  stage_store<1>(v_fwlw, n_fwlw, tid, NTH, get_fwlw, [&](int i, float v) { fwlw_s[i] = v; });
  stage_store<1>(v_rsk, n_rsk, tid, NTH, get_rsk, [&](int i, f32x4 v) { reinterpret_cast<f32x4*>(rsk)[i] = v; });
  if (bce && tid < kBM) {
    // binary_cross_entropy_with_logits and its gradient for this tile's rows: bce_grad_kernel's arithmetic
    const bool valid = b0 + tid < p.batch;
    const float x = v_dl[0], t = v_y[0];
    const float sg = 1.f / (1.f + expf(-x));
    v_dl[0] = valid ? __fdiv_rn(__fsub_rn(sg, t), p.bce_denom) : 0.f;
    float l = valid ? fmaxf(x, 0.f) - x * t + log1pf(expf(-fabsf(x))) : 0.f;
    if (valid) p.bce_dl[b0 + tid] = v_dl[0];
    l = sum16(l);
    // with the fused reductions the tile's loss is a partial like its gradients (reduce_final adds the tiles in
    // order); else an atomic add
    if (tid == 0 && red) p.part[(size_t)blockIdx.x * red_outputs(F, D, p.N, num) + red_outputs(F, D, p.N, num) - 1] = l;
    else if (tid == 0 && p.loss_sum) atomicAdd(p.loss_sum, l);
  }
  stage_store<1>(v_dl, kBM, tid, NTH, get_dl, [&](int i, float v) { dl[i] = v; });
  stage_store<2>(v_fo, n_fo, tid, NTH, get_fo, [&](int i, float v) {
    const int b = i / F;
    fo_s[b * Fp + (i - b * F)] = v;
  });
  stage_store<1>(v_xv, n_xv, tid, NTH, get_xv, [&](int i, float v) {
    const int b = i / num;
    xv_s[b * Fp + (i - b * num)] = v;
  });
  stage_store<1>(v_fc, n_fc, tid, NTH, get_fc, [&](int i, float v) { fc_s[i] = v; });
  tile_store<4>(bufE, SX, v_e, p.sv_e + b0 * r4(FD), r4(FD), second ? nrows : 0, r4(FD) / 4, p.W0 / 4, tid, NTH);
  float* rout = p.part + (size_t)blockIdx.x * red_outputs(F, D, p.N, num);  // fused reductions' partials
  for (int i = tid; i < kBM * (p.W0 / 4); i += NTH) {
    const int b = i / (p.W0 / 4);
    reinterpret_cast<f32x4*>(bufD + b * SX)[i - b * (p.W0 / 4)] = f32x4{0.f, 0.f, 0.f, 0.f};
  }
  __syncthreads();
  stamp(p.stamps, 1, tid);

  // ---- P1: dE of the shallow part and the field_cov Gram ---------------------------------
  // The work is dealt to the waves by cost, and every operand of a chain (or of a group of four steps) is read from
  // LDS before its MFMAs, with the wave-uniform decoding done once per chain:
  //  * field_cov's Gram (fused reduction): chain h of tile (mk, ml) takes the steps 4g + 2i + h (g < D, i < 2) --
  //    reduce_kernel's two accumulators -- i.e. (b, d) = divmod(16g + 8i + 4h + (lane >> 4), D): 2D MFMAs; the
  //    chains' sums go to LDS and are added after the barrier.  Chains round-robin from wave 0.
  //  * the FwFM dE pieces (m, nt): S dependent MFMAs each, round-robin from the last wave.
  {
    const int MT = p.MT, S = p.S;
    if (red & kRedR) {
      float* gram = smem + L.gram;
      // a wave's chains all have its parity h = wave & 1 (c = wave + NW k), so the (b, d) of every step -- its LDS
      // offset b SX + d and its dlogit -- are the same for all of them: formed once
      const int hq = 4 * (wave & 1) + (lane >> 4);
      int off[2 * D];
      float dlj[2 * D];
#pragma unroll
      for (int j = 0; j < 2 * D; ++j) {
        const int nn = 16 * (j >> 1) + 8 * (j & 1) + hq;
        const int b = nn / D;
        off[j] = b * SX + (nn - b * D);
        dlj[j] = dl[b];
      }
      for (int c = wave; c < 2 * MT * MT; c += NW) {
        const int t = c >> 1;
        const int mk = t / MT, ml = t - mk * MT;
        const int kA = 16 * mk + (lane & 15), lB = 16 * ml + (lane & 15);
        const bool va = kA < F, vb = lB < F;
        const float* ea = bufE + (va ? kA : 0) * D;
        const float* eb = bufE + (vb ? lB : 0) * D;
        float av[2 * D], bv[2 * D];
#pragma unroll
        for (int j = 0; j < 2 * D; ++j) {
          const float x = ea[off[j]];
          av[j] = va ? dlj[j] * x : 0.f;
          bv[j] = vb ? eb[off[j]] : 0.f;
        }
        f32x4 acc = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int j = 0; j < 2 * D; ++j) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(av[j], bv[j], acc, 0, 0, 0);
        reinterpret_cast<f32x4*>(gram)[c * 64 + lane] = acc;
      }
    }
    stamp(p.stamps, 12, tid);
    if (second) {
      // dE[b,k,d] = dlogit_b * sum_{l != k} Rs[k,l] E[b,l,d]  (+ dfo[b,k] * Wfl[k,d] with fwlw, :344-345)
      for (int it = NW - 1 - wave; it < MT * D; it += NW) {
        const int m = it / D, nt = it - m * D;
        const int n = nt * 16 + (lane & 15);
        const int b = n / D;
        const int d = n - b * D;
        const float* ecol = bufE + b * SX + d + (lane >> 4) * D;  // + 4 s D at step s
        const float* ua = rsk + m * S * 64 + lane;                 // + 64 s
        f32x4 acc = f32x4{0.f, 0.f, 0.f, 0.f};
        auto group = [&](int s0, auto U_) {
          constexpr int U = decltype(U_)::value;
          float av[U], bv[U];
#pragma unroll
          for (int u = 0; u < U; ++u) {
            av[u] = ua[(s0 + u) * 64];
            bv[u] = ecol[(s0 + u) * 4 * D];
          }
#pragma unroll
          for (int u = 0; u < U; ++u) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(av[u], bv[u], acc, 0, 0, 0);
        };
        int s0 = 0;
        for (; s0 + 8 <= S; s0 += 8) group(s0, std::integral_constant<int, 8>{});
        const int rem = S - s0;
        if (rem >= 4) {
          group(s0, std::integral_constant<int, 4>{});
          s0 += 4;
        }
        if (S - s0 == 3) group(s0, std::integral_constant<int, 3>{});
        else if (S - s0 == 2) group(s0, std::integral_constant<int, 2>{});
        else if (S - s0 == 1) group(s0, std::integral_constant<int, 1>{});
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int k = 16 * m + row0 + r;
          if (k < F) {
            float v = dl[b] * acc[r];
            if (fwlw) v = fmaf(lwp ? dl[b] * lw_s[k] : dl[b], fwlw_s[k * D + d], v);
            bufD[b * SX + k * D + d] = v;
          }
        }
      }
    }
  }
  stamp(p.stamps, 13, tid);
  // ---- R: the other dense shallow reductions over this tile (reduce_kernel's arithmetic, same order), from the
  // tiles in LDS: bias, fm_1st, fwfm_linear, the numerical fields' first order
  if (red) {
    float* o_lw = rout + 1;
    float* o_fw = o_lw + F;
    if (tid < kBM) {
      const float v = sum16(dl[tid]);
      if (tid == 0) rout[0] = v;
    }
    if (tid < F) {
      float sl = 0.f;
      if (red & kRedLw)
#pragma unroll
        for (int b = 0; b < kBM; ++b) sl = fmaf(dl[b], fo_s[b * Fp + tid], sl);
      o_lw[tid] = sl;
    }
    for (int i = tid; i < FD; i += NTH) {
      float sf = 0.f;
      if (red & kRedFwlw)
#pragma unroll
        for (int b = 0; b < kBM; ++b) sf = fmaf(dl[b], bufE[b * SX + i], sf);
      o_fw[i] = sf;
    }
    if (tid < num) {
      float sn = 0.f;
#pragma unroll
      for (int b = 0; b < kBM; ++b) sn = fmaf(dl[b], xv_s[b * Fp + tid], sn);
      float* o_n1 = o_fw + FD + F * F + p.N + num * D;
      o_n1[tid] = sn;
    }
  }
  __syncthreads();
  if (red) {
    // field_cov: d W[k,l] = 0.5 * sum_b dlogit_b <E_bk, E_bl>, k != l (:363-367) from the two chains of each tile
    float* o_R = rout + 1 + F + FD;
    if (red & kRedR) {
      const int MT = p.MT;
      const float* gram = smem + L.gram;
      for (int e = tid; e < MT * MT * 256; e += NTH) {
        const int t = e >> 8, ln = (e >> 2) & 63, r = e & 3;
        const int mk = t / MT, ml = t - mk * MT;
        const int k = 16 * mk + (ln >> 4) * 4 + r, lB = 16 * ml + (ln & 15);
        if (k < F && lB < F) o_R[k * F + lB] = k != lB ? 0.5f * (gram[(2 * t) * 256 + 4 * ln + r] +
                                                                 gram[(2 * t + 1) * 256 + 4 * ln + r])
                                                       : 0.f;
      }
    } else {
      for (int i = tid; i < F * F; i += NTH) o_R[i] = 0.f;
    }
  }
  stamp(p.stamps, 2, tid);

  // ---- P2: MLP backward (net_1_fc then net_1_linear_H .. 1, :412-428) ---------------
  if (deep) {
    const int H = p.H, N = p.N, NT = p.NT, NP = NT * 16;
    const float scale = drop ? p.drop_scale : 1.f;
    const uint32_t dseed = drop ? step_seed(p.seed, p.seed_src) : 0u;
    // G_H = dlogit * fc * (X_H > 0) * scale -> bufA (X_H read in P0, written to LDS now; G_H is stored to the
    // workspace at the top of layer H, behind its weight preload).  bufA held the field_cov Gram until now.
    if (red & kRedR) __syncthreads();
    tile_store<4>(bufA, SY, v_x, xh_g, p.N, nrows, p.N / 4, p.NT * 4, tid, NTH);
    __syncthreads();
    // column n per thread: the fused net_1_fc reduction (sum_b dlogit_b X_H[b, n], reduce_kernel's order)
    // reads the column before it is overwritten with G_H
    float* o_fc = rout + 1 + F + FD + F * F;
    for (int n = tid; n < NP; n += NTH) {
      float sc = 0.f;
#pragma unroll
      for (int b = 0; b < kBM; ++b) {
        const float x = bufA[b * SY + n];
        sc = fmaf(dl[b], x, sc);
        bufA[b * SY + n] = (n < N && x > 0.f) ? dl[b] * fc_s[n] * scale : 0.f;
      }
      if (red && n < N) o_fc[n] = (red & kRedFc) ? sc : 0.f;
    }
    __syncthreads();
    stamp(p.stamps, 3, tid);

    const __amdgpu_buffer_rsrc_t wrsrc = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<float4*>(p.wtpack), (short)0, p.wtpack_bytes, 0x00020000);
    LayerStream<TPW, 1, NG> ls;
    f32x4 wb0[TPW], wb1[TPW], wb2[TPW];
    TailStream<NG> ts;
    f32x4 tw[TailStream<NG>::C];
    const int g = wave;
    // the static form (Criteo's 400-wide layers: 25 chunks, 24 + 1 split tiles per layer, like the forward's
    // NS = 25 loop): the split tile's share rides on the K loop's register sets (no tail loads and MMA exposed
    // before the loop), and each layer's first chunks go out before the previous layer's barrier
    constexpr bool kStatForm = NG == 8 && TPW == 3;
    const bool stat = kStatForm && NT == 25 && p.NC0 == 25 && NT <= NG * TailStream<NG>::C &&
                      !(flags & kBwdGeneric);
    // the epilogue's ReLU / dropout mask sources X_{l-1} for this lane's outputs of the layer's first pass (tile
    // t0 + g + NG j, rows row0 + r) and of the split tile (row row0 + (g & 3)), loaded behind the layer's preload
    // and the G_l stores (measured: loaded ahead, before the preload, or from LDS bytes prefetched in P0, the
    // kernel was 4-14k cycles slower, profiles/r04/r04k_bwdstamps.log, r04l_bwdstamps.log)
    auto load_masks = [&](int l, int t0, float (&xm)[TPW][4], float& xt) {
      const int K = l == 1 ? FD : N;
      const int KT = l == 1 ? p.NC0 : NT;
      const bool ltail = NG == 8 && KT == NG * TPW + 1 && NT <= NG * TailStream<NG>::C;
      const int KTm = ltail ? KT - 1 : KT;
#pragma unroll
      for (int j = 0; j < TPW; ++j) {
        const int t = t0 + g + NG * j;
        const int k = t * 16 + (lane & 15);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int64_t row = b0 + row0 + r;
          xm[j][r] = (l > 1 && t < KTm && k < K && row < p.batch)
                         ? ((flags & kBwdNoMask) ? 1.f : p.sv_x[l - 1][row * N + k]) : 0.f;
        }
      }
      const int k = (KT - 1) * 16 + (lane & 15);
      const int64_t row = b0 + row0 + (g & 3);
      xt = (ltail && t0 == 0 && l > 1 && g < 4 && k < K && row < p.batch)
               ? ((flags & kBwdNoMask) ? 1.f : p.sv_x[l - 1][row * N + k]) : 0.f;
    };
    if (stat) {
      ls.init(wrsrc, p.wt_off[H], NT, NT - 1, g, 0);
      ls.preload(wb0, wb1, lane * 16);
    }
    for (int l = H; l >= 1; --l) {
      const bool fromA = ((H - l) & 1) == 0;
      const float* in = fromA ? bufA : bufB;
      float* outg = fromA ? bufB : bufA;
      const int K = l == 1 ? FD : N;
      const int KT = l == 1 ? p.NC0 : NT;
      // eight waves: the last tile of a layer with 8*TPW + 1 tiles is split by K over the waves
      const bool ltail = NG == 8 && KT == NG * TPW + 1 && NT <= NG * TailStream<NG>::C;
      const int KTm = ltail ? KT - 1 : KT;
      const int T = KT - 1;  // the tail tile
      float xt = 0.f;        // its ReLU mask source, row row0 + g
      // output tiles (the layer's inputs k) in passes of NG*TPW: layer 1 may have more tiles
      // (ceil(F*D/16)) than the hidden width the kernel's TPW was sized for
      for (int t0 = 0; t0 < KTm; t0 += NG * TPW) {
        if (!stat) {
          ls.init(wrsrc, p.wt_off[l] + t0 * NT * 64, NT, KTm - t0, g, 0);
          ls.preload(wb0, wb1, lane * 16);
          if (ltail && t0 == 0) {
            ts.init(p.wt_off[l], NT, T, g);
            ts.load(wrsrc, tw, lane * 16);
          }
        }
        // G_l (this layer's input tile) -> workspace for the weight-gradient GEMM: coalesced rows from LDS, behind
        // the preload (stores count in vmcnt too)
        if (t0 == 0 && !(flags & kBwdNoGStore)) store_tile(p.sv_g[l] + b0 * N, N, in, SY, nrows, N / 4, tid, NTH);
        float xm[TPW][4];
        {
          float xt0;
          load_masks(l, t0, xm, xt0);
          if (ltail && t0 == 0) xt = xt0;
        }
        // the tail's share first (generic form): its fragments are then dead during the K loop
        if (ltail && t0 == 0 && !stat) reinterpret_cast<f32x4*>(tailr)[g * 64 + lane] = ts.mma(in, SY, tw, lane);
        f32x4 acc[TPW];
        if constexpr (kStatForm) {
          if (stat) {
#pragma unroll
            for (int j = 0; j < TPW; ++j) acc[j] = f32x4{0.f, 0.f, 0.f, 0.f};
            ts.init(p.wt_off[l], NT, T, g);
            f32x4 tp;
            mlp_k_loop_s<TPW, NG, 25, false>(acc, in, SY, ls, wb0, wb1, wb2, lane, ts, tp);
            reinterpret_cast<f32x4*>(tailr)[g * 64 + lane] = tp;
          } else {
            mlp_k_loop<TPW, 1, NG>(acc, in, SY, ls, wb0, wb1, wb2, lane);
          }
        } else {
          mlp_k_loop<TPW, 1, NG>(acc, in, SY, ls, wb0, wb1, wb2, lane);
        }
#pragma unroll
        for (int j = 0; j < TPW; ++j) {
          const int t = t0 + g + NG * j;
          if (t >= KTm) continue;  // wave-uniform
          const int k = t * 16 + (lane & 15);
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int b = row0 + r;
            const int64_t row = b0 + b;
            if (l > 1) {
              outg[b * SY + k] = (k < K && xm[j][r] > 0.f) ? acc[j][r] * scale : 0.f;
            } else if (k < FD) {
              float gv = acc[j][r];
              if (drop) gv = dropout_keep(dseed, 0, row, k, p.drop_p) ? gv * scale : 0.f;
              // the final dE of this element: to LDS (the numerical fields' reduction) and to the workspace from here
              const float v = bufD[b * SX + k] + gv;
              bufD[b * SX + k] = v;
              if (row < p.batch) p.sv_de[row * FD + k] = v;
            }
          }
        }
        // the next layer's first chunks, ahead of the barrier (after the epilogue: any wait on a vector-memory
        // result after them would wait for them too)
        if (stat && l > 1) {
          ls.init(wrsrc, p.wt_off[l - 1], NT, NT - 1, g, 0);
          ls.preload(wb0, wb1, lane * 16);
        }
      }
      __syncthreads();
      if (ltail) {
        // wave g < 4 finishes row (lane>>4)*4 + g of the tail tile from the NG partial products
        if (g < 4) {
          const int k = T * 16 + (lane & 15);
          const int b = row0 + g;
          const float* tp = tailr + lane * 4 + g;
          float sum = tp[0];
#pragma unroll
          for (int w = 1; w < NG; ++w) sum += tp[w * 256];
          if (l > 1) {
            outg[b * SY + k] = (k < K && xt > 0.f) ? sum * scale : 0.f;
          } else if (k < FD) {
            float gv = sum;
            if (drop) gv = dropout_keep(dseed, 0, b0 + b, k, p.drop_p) ? gv * scale : 0.f;
            const float v = bufD[b * SX + k] + gv;
            bufD[b * SX + k] = v;
            if (b0 + b < p.batch) p.sv_de[(b0 + b) * FD + k] = v;
          }
        }
        __syncthreads();
      }
      stamp(p.stamps, 4 + (H - l < 3 ? H - l : 3), tid);
    }
  }
  stamp(p.stamps, 8, tid);

  // ---- P3: dE -> workspace (coalesced rows); with the MLP its layer-1 epilogue stored every element already (the
  // store pass after the last barrier took ~5.8k cycles) -------------------------------------------------------
  if (!deep) {
    for (int i = tid; i < kBM * FD; i += NTH) {
      const int b = i / FD;
      const int c = i - b * FD;
      if (b0 + b < p.batch) p.sv_de[(b0 + b) * FD + c] = bufD[b * SX + c];
    }
  }
  if (red) {
    // numerical fields' second-order tables: E_f = v_f * Xv_f (:297-299) -> sum_b dE[b, f, :] * Xv[b, f]
    float* o_n2 = rout + 1 + F + FD + F * F + p.N;
    for (int i = tid; i < num * D; i += NTH) {
      const int f = i / D;
      float s2 = 0.f;
      if (red & kRedNum2)
#pragma unroll
        for (int b = 0; b < kBM; ++b) s2 = fmaf(bufD[b * SX + i], xv_s[b * Fp + f], s2);
      o_n2[i] = s2;
    }
  }
  stamp(p.stamps, 9, tid);
  stamp_rt(p.stamps, 11, tid);
}

// ---------------------------------------------------------------------------
// Dense shallow gradients, one 16-row tile per workgroup: the tile's rows of E, fo and X_H are
// contiguous in the workspace, so they are staged with linear float4 loads (all in flight at once);
// each block writes its partial sums (no atomics) and reduce_final_kernel adds the blocks.
// ---------------------------------------------------------------------------
constexpr int kRedMaxFD = 2048;  // F*D (64 x 32)
constexpr int kRedMaxN = 512;

struct RedLds {
  int e, fo, xh, xv, de, total;
};
__host__ __device__ inline RedLds red_layout(int F, int D, int N, int num) {
  RedLds L;
  int o = 0;
  L.e = o;   o += kBM * r4(F * D);  // rows of stride r4(F*D), as in the workspace
  L.fo = o;  o += r4(kBM * F);
  L.xh = o;  o += r4(kBM * N);
  L.xv = o;  o += r4(kBM * (num > 0 ? num : 1));
  L.de = o;  o += r4(kBM * (num > 0 ? num * D : 1));
  L.total = r4(o);
  return L;
}

// copy n contiguous floats (16-byte aligned source and destination offsets) global -> LDS, zero-filling
// [n, ncap); U float4 per thread in flight
// stage_linear in two halves, so that several sources' loads are in flight together: stage_issue
// loads the first 256*U float4 into registers, stage_commit stores them and copies any remainder
#ifndef DFWFM_KD  // the non-templated kernels: the common translation unit only
template <int U>
__device__ __forceinline__ void stage_issue(f32x4 (&v)[U], const float* __restrict__ src, int n, int ncap, int tid) {
  const int n4 = ncap >> 2;
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int q = tid + u * 256;
    const int e = q * 4;
    v[u] = f32x4{0.f, 0.f, 0.f, 0.f};
    if (q < n4 && e + 3 < n) {
      v[u] = *reinterpret_cast<const f32x4*>(src + e);
    } else if (q < n4) {
      v[u].x = e < n ? src[e] : 0.f;
      v[u].y = e + 1 < n ? src[e + 1] : 0.f;
      v[u].z = e + 2 < n ? src[e + 2] : 0.f;
    }
  }
}

template <int U>
__device__ __forceinline__ void stage_commit(float* __restrict__ dst, const f32x4 (&v)[U], const float* __restrict__ src,
                                             int n, int ncap, int tid) {
  const int n4 = ncap >> 2;
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int q = tid + u * 256;
    if (q < n4) *reinterpret_cast<f32x4*>(dst + q * 4) = v[u];
  }
  for (int q = tid + 256 * U; q < n4; q += 256) {
    const int e = q * 4;
    f32x4 w = f32x4{0.f, 0.f, 0.f, 0.f};
    if (e + 3 < n) w = *reinterpret_cast<const f32x4*>(src + e);
    else {
      w.x = e < n ? src[e] : 0.f;
      w.y = e + 1 < n ? src[e + 1] : 0.f;
      w.z = e + 2 < n ? src[e + 2] : 0.f;
    }
    *reinterpret_cast<f32x4*>(dst + q * 4) = w;
  }
}

template <int U>
__device__ __forceinline__ void stage_linear(float* __restrict__ dst, const float* __restrict__ src, int n, int ncap,
                                             int tid) {
  const int n4 = ncap >> 2;
  for (int q0 = tid; q0 < n4; q0 += 256 * U) {
    float4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int q = q0 + u * 256;
      const int e = q * 4;
      if (q < n4 && e + 3 < n) {
        v[u] = *reinterpret_cast<const float4*>(src + e);
      } else {
        v[u].x = (q < n4 && e < n) ? src[e] : 0.f;
        v[u].y = (q < n4 && e + 1 < n) ? src[e + 1] : 0.f;
        v[u].z = (q < n4 && e + 2 < n) ? src[e + 2] : 0.f;
        v[u].w = 0.f;
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int q = q0 + u * 256;
      if (q < n4) *reinterpret_cast<float4*>(dst + q * 4) = v[u];
    }
  }
}

__global__ void __launch_bounds__(256) reduce_kernel(RedArgs a) {
  constexpr int NTH = 256;
  constexpr int KF = kRedMaxFD / NTH;  // per-thread E columns
  constexpr int KN = kRedMaxN / NTH;   // per-thread hidden units
  __shared__ float dl[kBM];
  extern __shared__ __attribute__((aligned(16))) float sm[];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int F = a.F, D = a.D, FD = F * D, num = a.num, N = a.N, numD = num * D;
  const int SE = r4(FD);  // row stride of the saved E
  const RedLds L = red_layout(F, D, N, num);
  float* es = sm + L.e;
  float* fos = sm + L.fo;
  float* xhs = sm + L.xh;
  float* xvs = sm + L.xv;
  float* des = sm + L.de;
  const int64_t rb = (int64_t)blockIdx.x * kBM;
  const int nt = (int)((a.batch - rb) < kBM ? (a.batch - rb) : kBM);
  const bool lwp = (a.flags & kFoLw) != 0;
  const bool need_e = a.g_fwlw || a.g_R;
  const bool need_num2 = numD > 0 && a.sv_de != nullptr;
  if (tid < kBM) dl[tid] = tid < nt ? a.dlogit[rb + tid] : 0.f;
  // every staging load is issued before any LDS store: one memory round trip instead of one per
  // source (the tiles are contiguous rows of the workspace)
  constexpr int UE = 8, UF = 2, UH = 8, UD = 9;
  f32x4 ve[UE], vf[UF], vh[UH];
  float vd[UD], vx = 0.f;
  if (need_e) stage_issue<UE>(ve, a.sv_e + rb * SE, nt * SE, kBM * SE, tid);
  if (a.g_lw) stage_issue<UF>(vf, a.sv_fo + rb * F, nt * F, r4(kBM * F), tid);
  if (a.g_fc) stage_issue<UH>(vh, a.x_h + rb * N, nt * N, r4(kBM * N), tid);
  if (num > 0 && tid < kBM * num) {
    const int b = tid / num, c = tid - b * num;
    vx = b < nt ? a.xv[(rb + b) * a.xv_stride + c] : 0.f;
  }
#pragma unroll
  for (int u = 0; u < UD; ++u) {
    const int i = tid + u * NTH;
    const int b = i / (numD > 0 ? numD : 1), c = i - b * numD;
    vd[u] = (need_num2 && i < kBM * numD && b < nt) ? a.sv_de[(rb + b) * FD + c] : 0.f;
  }
  if (need_e) stage_commit<UE>(es, ve, a.sv_e + rb * SE, nt * SE, kBM * SE, tid);
  if (a.g_lw) stage_commit<UF>(fos, vf, a.sv_fo + rb * F, nt * F, r4(kBM * F), tid);
  if (a.g_fc) stage_commit<UH>(xhs, vh, a.x_h + rb * N, nt * N, r4(kBM * N), tid);
  if (num > 0) {
    if (tid < kBM * num) xvs[tid] = vx;
    for (int i = tid + NTH; i < kBM * num; i += NTH) {  // num > 16
      const int b = i / num, c = i - b * num;
      xvs[i] = b < nt ? a.xv[(rb + b) * a.xv_stride + c] : 0.f;
    }
  }
  if (need_num2) {
#pragma unroll
    for (int u = 0; u < UD; ++u) {
      const int i = tid + u * NTH;
      if (i < kBM * numD) des[i] = vd[u];
    }
    for (int i = tid + UD * NTH; i < kBM * numD; i += NTH) {  // wider numerical parts
      const int b = i / numD, c = i - b * numD;
      des[i] = b < nt ? a.sv_de[(rb + b) * FD + c] : 0.f;
    }
  }
  __syncthreads();

  float* out = a.part + (size_t)blockIdx.x * red_outputs(F, D, N, num);
  float* o_lw = out + 1;
  float* o_fw = o_lw + F;
  float* o_R = o_fw + FD;
  float* o_fc = o_R + F * F;
  float* o_n2 = o_fc + N;
  float* o_n1 = o_n2 + numD;
  // bias (total_sum += self.bias, :458)
  if (tid < kBM) {
    const float v = sum16(dl[tid]);
    if (tid == 0) out[0] = v;
  }
  // fm_1st: first = fo . w_lw (:450)
  if (tid < F) {
    float s = 0.f;
    if (a.g_lw)
#pragma unroll
      for (int b = 0; b < kBM; ++b) s = fmaf(dl[b], fos[b * F + tid], s);
    o_lw[tid] = s;
  }
  // fwfm_linear: fo[b,f] = <E[b,f,:], Wfl[f,:]> (:344-345); dfo's lw[f] factor is applied by the final sum
#pragma unroll
  for (int j = 0; j < KF; ++j) {
    const int i = tid + j * NTH;
    if (i < FD) {
      float s = 0.f;
      if (a.g_fwlw)
#pragma unroll
        for (int b = 0; b < kBM; ++b) s = fmaf(dl[b], es[b * SE + i], s);
      o_fw[i] = s;
    }
  }
  // numerical fields: E_f = v_f * Xv_f, fo_f = w1_f * Xv_f (:297-299, :304, :334)
  for (int i = tid; i < numD; i += NTH) {
    const int f = i / D;
    float s = 0.f;
    if (need_num2)
#pragma unroll
      for (int b = 0; b < kBM; ++b) s = fmaf(des[b * numD + i], xvs[b * num + f], s);
    o_n2[i] = s;
  }
  if (tid < num) {
    float s = 0.f;
#pragma unroll
    for (int b = 0; b < kBM; ++b) s = fmaf(dl[b], xvs[b * num + tid], s);
    o_n1[tid] = s;
  }
  // net_1_fc: deep = X_H . w_fc (:428-436)
#pragma unroll
  for (int j = 0; j < KN; ++j) {
    const int n = tid + j * NTH;
    if (n < N) {
      float s = 0.f;
      if (a.g_fc)
#pragma unroll
        for (int b = 0; b < kBM; ++b) s = fmaf(dl[b], xhs[b * N + n], s);
      o_fc[n] = s;
    }
  }
  // field_cov: d W[k,l] = 0.5 * sum_b dlogit_b <E_bk, E_bl>, k != l (:363-367): a Gram matrix on MFMA,
  // contraction over (b, d)
  if (a.g_R) {
    const int MT = a.MT, ntile = MT * MT;
    const int steps = (kBM * D) / 4;
    for (int t = wave; t < ntile; t += 4) {
      const int mk = t / MT, ml = t - mk * MT;
      const int kA = 16 * mk + (lane & 15);
      const int lB = 16 * ml + (lane & 15);
      // two accumulators, each group's eight operands read from LDS before its four MFMAs (one
      // dependent chain over 40 steps exposed the MFMA and LDS latencies at every step)
      f32x4 acc0 = f32x4{0.f, 0.f, 0.f, 0.f}, acc1 = acc0;
      int s = 0;
      for (; s + 4 <= steps; s += 4) {
        float av[4], bv[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const int n = 4 * (s + u) + (lane >> 4);
          const int b = n / D;
          const int d = n - b * D;
          av[u] = kA < F ? dl[b] * es[b * SE + kA * D + d] : 0.f;
          bv[u] = lB < F ? es[b * SE + lB * D + d] : 0.f;
        }
        acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(av[0], bv[0], acc0, 0, 0, 0);
        acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(av[1], bv[1], acc1, 0, 0, 0);
        acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(av[2], bv[2], acc0, 0, 0, 0);
        acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(av[3], bv[3], acc1, 0, 0, 0);
      }
      for (; s < steps; ++s) {
        const int n = 4 * s + (lane >> 4);
        const int b = n / D;
        const int d = n - b * D;
        const float av = kA < F ? dl[b] * es[b * SE + kA * D + d] : 0.f;
        const float bv = lB < F ? es[b * SE + lB * D + d] : 0.f;
        acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(av, bv, acc0, 0, 0, 0);
      }
      const f32x4 acc = acc0 + acc1;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int k = 16 * mk + (lane >> 4) * 4 + r;
        if (k < F && lB < F) o_R[k * F + lB] = k != lB ? 0.5f * acc[r] : 0.f;
      }
    }
  }
}

// Sum of the per-block partials, added into the grads (accumulate, like autograd): 64 outputs per
// workgroup, each wave sums a quarter of the blocks in block order (32 loads in flight per lane: the sum is a
// chain of dependent L2 round trips otherwise -- 8 in flight made it 6 us alone and ~39 us beside the weight
// GEMM), then the four quarters are combined in a fixed order (deterministic).
// block `bx` of the final sums (64 outputs, the four waves each a quarter of the tiles)
__device__ __forceinline__ void reduce_final_block(const RedArgs& a, int nblk, int bx) {
  __shared__ float q4[4][64];
  const int F = a.F, D = a.D, N = a.N, num = a.num, FD = F * D, numD = num * D;
  const int P = red_outputs(F, D, N, num);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int o = bx * 64 + lane;
  const int per = (nblk + 3) / 4;
  const int b0 = wave * per, b1 = b0 + per < nblk ? b0 + per : nblk;
  float s = 0.f;
  if (o < P) {
    int b = b0;
    for (; b + 32 <= b1; b += 32) {
      float v[32];
#pragma unroll
      for (int u = 0; u < 32; ++u) v[u] = a.part[(size_t)(b + u) * P + o];
#pragma unroll
      for (int u = 0; u < 32; ++u) s += v[u];
    }
    for (; b + 8 <= b1; b += 8) {
      float v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) v[u] = a.part[(size_t)(b + u) * P + o];
#pragma unroll
      for (int u = 0; u < 8; ++u) s += v[u];
    }
    for (; b < b1; ++b) s += a.part[(size_t)b * P + o];
  }
  q4[wave][lane] = s;
  __syncthreads();
  if (wave != 0 || o >= P) return;
  s = ((q4[0][lane] + q4[1][lane]) + q4[2][lane]) + q4[3][lane];
  const bool lwp = (a.flags & kFoLw) != 0;
  float* dst = nullptr;
  float scale = 1.f;
  int i = o;
  if (i < 1) {
    dst = a.g_bias;
  } else if ((i -= 1) < F) {
    dst = a.g_lw ? a.g_lw + i : nullptr;
  } else if ((i -= F) < FD) {
    dst = a.g_fwlw ? a.g_fwlw + i : nullptr;
    if (lwp) scale = a.lw[i / D];
  } else if ((i -= FD) < F * F) {
    dst = a.g_R ? a.g_R + i : nullptr;
  } else if ((i -= F * F) < N) {
    dst = a.g_fc ? a.g_fc + i : nullptr;
  } else if ((i -= N) < numD) {
    dst = a.g_num2[i / D] ? a.g_num2[i / D] + i % D : nullptr;
  } else if ((i -= numD) < num) {
    dst = a.g_num1[i];
    if (lwp) scale = a.lw[i];
  } else {
    dst = a.loss_sum;  // the tiles' losses (only the fused backward with the loss gradient writes them)
  }
  if (dst) *dst += s * scale;
}

__global__ void __launch_bounds__(256) reduce_final_kernel(RedArgs a, int nblk) { reduce_final_block(a, nblk, blockIdx.x); }

// ---------------------------------------------------------------------------
// Categorical-table scatter (reference nn.Embedding / EmbeddingBag / QREmbeddingBag backward with
// dense grads).  Each workgroup takes a.chunk samples of one task.  PRIV (small tables): the chunk
// accumulates in an LDS copy of the table, then each touched row is added to the grad once (so an
// address sees at most one atomic per chunk even when every sample hits it); else one sample per
// lane with global atomics.
// ---------------------------------------------------------------------------
template <bool PRIV>
__device__ __forceinline__ void scatter_body(const ScatterArgs& a, const ScatterTask& T, int bid, float* acc,
                                             int32_t* srow, int32_t* spart) {
  // Lanes walk (sample, d) elements with d fastest, so one atomic wave-instruction adds ~6 rows of
  // 4*w contiguous bytes instead of 64 lanes hitting 64 different rows (~17x slower on gfx950,
  // MI355X_MICROARCH.md, float atomics).  Each sample's row / partner row is located once into LDS.
  const int tid = threadIdx.x;
  const FieldDev fd = a.fields[T.field];
  const int f = T.field, D = a.D, FD = a.F * D, w = T.src == 0 ? D : 1;
  const int col = f - a.num;
  const float lwf = a.lw ? a.lw[f] : 1.f;
  const int64_t s0 = (int64_t)(bid - T.block0) * a.chunk;
  const int ns = (int)((a.batch - s0) < a.chunk ? (a.batch - s0) : a.chunk);  // samples of this chunk
  // row of each sample in this task's table, and the partner-table row (QR)
  for (int sl = tid; sl < ns; sl += 256) {
    const int64_t b = s0 + sl;
    int64_t idx = a.xi[b * a.xi_stride + col];
    if (idx < 0 || idx >= fd.n) idx = 0;  // the forward clamped (and flagged) it the same way
    int64_t row = idx, part = 0;
    const int kind = T.kind & 3;
    if (kind == 1) {
      row = idx / T.c;
      part = idx - row * T.c;
    } else if (kind == 2) {
      part = idx / T.c;
      row = idx - part * T.c;
    }
    srow[sl] = (int32_t)row;
    spart[sl] = (int32_t)part;
  }
  auto value = [&](int64_t b, int part, int d) -> float {
    float v = T.src == 1 ? a.dlogit[b] * lwf : a.sv_de[b * FD + f * D + d];
    if (T.other) v *= T.other[T.src == 1 ? part : part * D + d];
    return v;
  };
  const int ne = ns * w;
  // elements in groups of SU per thread: all SU value loads are issued before the first atomic (an
  // atomic between two loads keeps the compiler from batching them: one memory round trip per element)
  // (measured: the first group's values issued with the keys' loads, 28.1 -> 29.7 us for the two launches)
  constexpr int SU = 8;
  if constexpr (PRIV) {
    int* flag = reinterpret_cast<int*>(acc + T.rows * w);
    const int n = T.rows * (w + 1);
    for (int i = tid; i < n; i += 256) acc[i] = 0.f;  // sums and row flags
    __syncthreads();
    for (int i0 = 0; i0 < ne; i0 += 256 * SU) {
      float v[SU];
      int at[SU];
#pragma unroll
      for (int u = 0; u < SU; ++u) {
        const int i = i0 + tid + 256 * u;
        at[u] = -1;
        v[u] = 0.f;
        if (i < ne) {
          const int sl = i / w;
          const int d = i - sl * w;
          const int row = srow[sl];
          at[u] = row * w + d;
          v[u] = value(s0 + sl, spart[sl], d);
          if (d == 0) flag[row] = 1;
        }
      }
#pragma unroll
      for (int u = 0; u < SU; ++u)
        if (at[u] >= 0) atomicAdd(&acc[at[u]], v[u]);
    }
    __syncthreads();
    // flush every touched row once, lane per element
    const int nf = T.rows * w;
    for (int i = tid; i < nf; i += 256) {
      const int row = i / w;
      if (flag[row]) atomicAdd(T.g + i, acc[i]);
    }
  } else {
    __syncthreads();
    for (int i0 = 0; i0 < ne; i0 += 256 * SU) {
      float v[SU];
      int64_t at[SU];
#pragma unroll
      for (int u = 0; u < SU; ++u) {
        const int i = i0 + tid + 256 * u;
        at[u] = -1;
        v[u] = 0.f;
        if (i < ne) {
          const int sl = i / w;
          const int d = i - sl * w;
          at[u] = (int64_t)srow[sl] * w + d;
          v[u] = value(s0 + sl, spart[sl], d);
        }
      }
#pragma unroll
      for (int u = 0; u < SU; ++u)
        if (at[u] >= 0) atomicAdd(T.g + at[u], v[u]);
    }
  }
}

// Both kinds of scatter tasks in one launch (privatised tasks first; they are independent of the global-atomic ones):
// the small tables' LDS accumulation runs beside the large tables' atomics instead of one launch after the other
__global__ void __launch_bounds__(256) scatter_kernel(ScatterArgs a) {
  extern __shared__ __attribute__((aligned(16))) float acc[];
  __shared__ int32_t srow[4 * 256];
  __shared__ int32_t spart[4 * 256];
  int lo = 0, hi = a.ntasks - 1;
  const int bid = blockIdx.x;
  while (lo < hi) {  // last task whose block0 <= bid
    const int mid = (lo + hi + 1) >> 1;
    if (a.t[mid].block0 <= bid) lo = mid;
    else hi = mid - 1;
  }
  const ScatterTask T = a.t[lo];
  if (T.kind & kScatterPriv) scatter_body<true>(a, T, bid, acc, srow, spart);
  else scatter_body<false>(a, T, bid, acc, srow, spart);
}

// ---------------------------------------------------------------------------
// Deterministic categorical-table scatter (deterministic mode, dfwfm_set_deterministic; the atomic scatter_kernel
// adds a row's contributions in arrival order, so two runs of the same step can differ in the last bits).  A task is
// one field and row kind, both table families at once; its rows are split into nbuck buckets (row % nbuck), one
// workgroup each, so every row has ONE owner workgroup.  Per pass over <= kSortSeg samples the owner:
//   1. reads the field's keys (the training forward's clamped indices, column-major: 32 contiguous bytes per
//      thread; xi when absent), keeps its bucket's samples in sample order (wave ballots, one barrier) as keys
//      (row / nbuck) << 12 | sample -- unique, so any correct sort gives the same order -- in 32 bits when the
//      bucket's rows stay under 2^20, with each sample's QR partner row; 2. bitonic sort in registers (partners inside
//      a row of 16 lanes by DPP, 16 apart by swizzle, 32 by the LDS crossbar, farther through LDS); 3. walks the
//      sorted positions in chunks of kSortCh: a work item (chunk, component) sums each run of equal rows in position
//      order; a run that starts and ends inside the chunk is added to its row at once, a run cut by the chunk's start /
//      end leaves its partial sum in LDS (lead / trail); 4. the chunk holding a cut run's head adds trail + the
//      following chunks' leads in chunk order.  Every row is added by exactly one thread per pass (passes follow each
//      other behind a barrier), in an order fixed by the sorted positions: the same bits on every run.
// ---------------------------------------------------------------------------
template <int NTH, typename K>
__device__ __forceinline__ void bitonic_sort_lds(K* key, int np, int tid) {
  for (int k = 2; k <= np; k <<= 1)
    for (int j = k >> 1; j > 0; j >>= 1) {
      for (int i = tid; i < (np >> 1); i += NTH) {
        const int lo = ((i & ~(j - 1)) << 1) | (i & (j - 1));
        const int hi = lo + j;
        const bool asc = (lo & k) == 0;
        const K x = key[lo], y = key[hi];
        if ((x > y) == asc) {
          key[lo] = y;
          key[hi] = x;
        }
      }
      __syncthreads();
    }
}

// the value of lane ^ M (M = 1 .. 32): DPP moves on the VALU inside a row of 16 lanes (quad permutes, rotations:
// row_ror:n reads lane (i - n) mod 16), a swizzle for 16, the LDS crossbar (bpermute) for 32
template <int M>
__device__ __forceinline__ uint32_t xor_lane(uint32_t v, int lane) {
  const int x = (int)v;
  if constexpr (M == 1) return (uint32_t)__builtin_amdgcn_mov_dpp(x, 0xB1, 0xF, 0xF, false);  // quad_perm [1,0,3,2]
  else if constexpr (M == 2) return (uint32_t)__builtin_amdgcn_mov_dpp(x, 0x4E, 0xF, 0xF, false);  // [2,3,0,1]
  else if constexpr (M == 4) {
    const int from_lo = __builtin_amdgcn_mov_dpp(x, 0x124, 0xF, 0xF, false);  // row_ror:4: lane i - 4
    const int from_hi = __builtin_amdgcn_mov_dpp(x, 0x12C, 0xF, 0xF, false);  // row_ror:12: lane i + 4
    return (uint32_t)((lane & 4) ? from_lo : from_hi);
  } else if constexpr (M == 8) return (uint32_t)__builtin_amdgcn_mov_dpp(x, 0x128, 0xF, 0xF, false);  // row_ror:8
  else if constexpr (M == 16) return (uint32_t)__builtin_amdgcn_ds_swizzle(x, 0x401F);  // bitmask mode, xor 16
  else return (uint32_t)__shfl_xor(x, M);
}
template <int M>
__device__ __forceinline__ uint64_t xor_lane(uint64_t v, int lane) {
  return ((uint64_t)xor_lane<M>((uint32_t)(v >> 32), lane) << 32) | xor_lane<M>((uint32_t)v, lane);
}

// one compare-exchange stage (merge size KK, partner distance J) of the network over NTH * E keys, each thread's E
// consecutive keys in registers: J < E inside the thread, E <= J < 64 E across the wave (lane ^ J / E), past a wave
// through LDS (two barriers)
template <int NTH, int E, int KK, int J, typename K>
__device__ __forceinline__ void bitonic_stage(K (&x)[E], K* key, int tid, int lane) {
  if constexpr (J < E) {
#pragma unroll
    for (int e = 0; e < E; ++e) {
      if ((e & J) == 0) {
        const bool asc = ((tid * E + e) & KK) == 0;
        const K lo = x[e], hi = x[e + J];
        if ((lo > hi) == asc) {
          x[e] = hi;
          x[e + J] = lo;
        }
      }
    }
  } else if constexpr (J < 64 * E) {
#pragma unroll
    for (int e = 0; e < E; ++e) {
      const int i = tid * E + e;
      const K y = xor_lane<J / E>(x[e], lane);
      const bool take_min = ((i & KK) == 0) == ((i & J) == 0);
      x[e] = take_min ? (y < x[e] ? y : x[e]) : (y > x[e] ? y : x[e]);
    }
  } else {
#pragma unroll
    for (int e = 0; e < E; ++e) key[tid * E + e] = x[e];
    __syncthreads();
#pragma unroll
    for (int e = 0; e < E; ++e) {
      const int i = tid * E + e;
      const K y = key[i ^ J];
      const bool take_min = ((i & KK) == 0) == ((i & J) == 0);
      x[e] = take_min ? (y < x[e] ? y : x[e]) : (y > x[e] ? y : x[e]);
    }
    __syncthreads();
  }
}
template <int NTH, int E, int KK, int J, typename K>
__device__ __forceinline__ void bitonic_net(K (&x)[E], K* key, int tid, int lane) {
  bitonic_stage<NTH, E, KK, J>(x, key, tid, lane);
  if constexpr (J > 1) bitonic_net<NTH, E, KK, J / 2>(x, key, tid, lane);
  else if constexpr (KK < NTH * E) bitonic_net<NTH, E, KK * 2, KK>(x, key, tid, lane);
}

// the whole network unrolled at compile time (every stage's partner move static): at np = 512 on 512 threads 6 of
// the 45 stages take a barrier
template <int NTH, int E, typename K>
__device__ __forceinline__ void bitonic_sort_reg(K* key, int tid) {
  K x[E];
#pragma unroll
  for (int e = 0; e < E; ++e) x[e] = key[tid * E + e];
  bitonic_net<NTH, E, 2, 1>(x, key, tid, tid & 63);
#pragma unroll
  for (int e = 0; e < E; ++e) key[tid * E + e] = x[e];
  __syncthreads();
}

// np keys (a power of two, 2 <= np <= kSortSeg) in LDS, sorted ascending in place.  (A rank sort -- each thread
// counting the keys below its own from 16-byte broadcast reads, two barriers -- measured 26k cycles against the
// network's 9k for ~540 keys on 1024 threads, profiles/r06/r06_rank.log.)
template <int NTH, typename K>
__device__ __forceinline__ void sort_keys(K* key, int np, int tid) {
  if (np <= NTH) {
    // pad to NTH keys (sentinels sort last), one per thread
    for (int i = np + tid; i < NTH; i += NTH) key[i] = ~(K)0;
    __syncthreads();
    bitonic_sort_reg<NTH, 1>(key, tid);
    return;
  }
  if constexpr (2 * NTH <= kSortSeg)
    if (np == 2 * NTH) return bitonic_sort_reg<NTH, 2>(key, tid);
  if constexpr (4 * NTH <= kSortSeg)
    if (np == 4 * NTH) return bitonic_sort_reg<NTH, 4>(key, tid);
  if constexpr (8 * NTH <= kSortSeg)
    if (np == 8 * NTH) return bitonic_sort_reg<NTH, 8>(key, tid);
  bitonic_sort_lds<NTH>(key, np, tid);
}

__host__ __device__ inline int sort_scatter_nch() { return kSortSeg / kSortCh; }

template <typename K>
__global__ void __launch_bounds__(kSortThreads) sort_scatter_kernel(SortScatterArgs a) {
  constexpr int NTH = kSortThreads;
  constexpr int CH = kSortCh;
  constexpr int SPT = kSortSeg / NTH;  // samples per thread when selecting the bucket's samples
  static_assert(SPT == 8 || SPT == 4, "one or two 16-byte key loads per thread");
  const int NCH = sort_scatter_nch();
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int D = a.D, FD = a.F * D, ncomp = D + 1;  // components: 0..D-1 second-order row, D first order
  K* key = reinterpret_cast<K*>(smem);
  int32_t* partv = reinterpret_cast<int32_t*>(smem + kSortSeg * 2);  // room for 64-bit keys
  int32_t* wtot_s = partv + kSortSeg;                                  // [NTH / 64] kept samples per wave
  float* lead = reinterpret_cast<float*>(wtot_s + NTH / 64);          // [NCH][ncomp]
  float* trail = lead + NCH * ncomp;
  uint8_t* cflag = reinterpret_cast<uint8_t*>(trail + NCH * ncomp);  // bit 0: first run continues from the
                                                                     // previous chunk, 1: last run continues into
                                                                     // the next, 2: one run
  // this workgroup's task and bucket
  int lo = 0, hi = a.ntasks - 1;
  const int bid = blockIdx.x;
  while (lo < hi) {  // last task whose block0 <= bid
    const int mid = (lo + hi + 1) >> 1;
    if (a.t[mid].block0 <= bid) lo = mid;
    else hi = mid - 1;
  }
  const SortScatterTask T = a.t[lo];
  const int bucket = bid - T.block0, nbuck = T.nbuck;
  stamp(a.stamps, 0, tid);
  if (a.stamps && tid == 0) a.stamps[(size_t)bid * kStampSlots + 8] = (uint64_t)lo;
  if (a.diag & 8) return;
  const FieldDev fd = a.fields[T.field];
  const int f = T.field, col = f - a.num;
  const float lwf = a.lw ? a.lw[f] : 1.f;
  for (int64_t s0 = 0; s0 < a.batch; s0 += kSortSeg) {
    const int ns = (int)((a.batch - s0) < kSortSeg ? (a.batch - s0) : kSortSeg);
    // 1. this bucket's samples of the pass, in sample order: thread t looks at samples [SPT t, SPT t + SPT)
    int64_t idxv[SPT];
    if (a.keys) {  // clamped by the training forward
      const int32_t* kc = a.keys + (int64_t)col * a.keys_stride + s0 + tid * SPT;
      if (tid * SPT + SPT <= ns) {
#pragma unroll
        for (int q = 0; q < SPT / 4; ++q) {
          const int4 k4 = reinterpret_cast<const int4*>(kc)[q];
          idxv[4 * q] = k4.x;
          idxv[4 * q + 1] = k4.y;
          idxv[4 * q + 2] = k4.z;
          idxv[4 * q + 3] = k4.w;
        }
      } else {
#pragma unroll
        for (int u = 0; u < SPT; ++u) idxv[u] = tid * SPT + u < ns ? kc[u] : -1;
      }
    } else {
#pragma unroll
      for (int u = 0; u < SPT; ++u) {
        const int i = tid * SPT + u;
        int64_t idx = -1;
        if (i < ns) {
          idx = a.xi[(s0 + i) * a.xi_stride + col];
          if (idx < 0 || idx >= fd.n) idx = 0;  // the forward clamped (and flagged) it the same way
        }
        idxv[u] = idx;
      }
    }
    K kk[SPT];
    int32_t pt[SPT];
    bool keep[SPT];
#pragma unroll
    for (int u = 0; u < SPT; ++u) {
      const int64_t idx = idxv[u];
      int64_t row = idx, part = 0;
      if (T.kind == 1) {
        row = idx / T.c;
        part = idx - row * T.c;
      } else if (T.kind == 2) {
        part = idx / T.c;
        row = idx - part * T.c;
      }
      keep[u] = idx >= 0 && (int)((uint32_t)row % (uint32_t)nbuck) == bucket;  // rows < 2^31
      kk[u] = ((K)((uint32_t)row / (uint32_t)nbuck) << 12) | (K)(tid * SPT + u);
      pt[u] = (int32_t)part;
    }
    if (a.diag & 16) {  // diagnostics: the key loads only
      if (keep[0] && kk[0] == (K)99999) wtot_s[0] = 1;
      return;
    }
    stamp(a.stamps, 1, tid);
    // positions in sample order: the kept samples of lower lanes (one ballot per slot u), then of lower waves
    int before = 0, wtot = 0;
#pragma unroll
    for (int u = 0; u < SPT; ++u) {
      const uint64_t bal = __ballot(keep[u]);
      before += (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(bal >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)bal, 0u));
      wtot += __popcll(bal);
    }
    if (lane == 0) wtot_s[wave] = wtot;
    __syncthreads();
    int pos = before, n = 0;
#pragma unroll
    for (int w = 0; w < NTH / 64; ++w) {
      const int c = wtot_s[w];
      pos += w < wave ? c : 0;
      n += c;
    }
#pragma unroll
    for (int u = 0; u < SPT; ++u) {
      if (keep[u]) {
        key[pos++] = kk[u];
        partv[tid * SPT + u] = pt[u];
      }
    }
    __syncthreads();
    stamp(a.stamps, 2, tid);
    if (a.stamps && tid == 0) a.stamps[(size_t)bid * kStampSlots + 9] = (uint64_t)n;
    if (n > 0) {
      int np = 2;
      while (np < n) np <<= 1;
      for (int i = n + tid; i < np; i += NTH) key[i] = ~(K)0;
      __syncthreads();
      // one row per bucket (small tables): the keys are already in order (sample order, one run)
      if (!(a.diag & 1) && !T.onerow) sort_keys<NTH>(key, np, tid);
      stamp(a.stamps, 3, tid);
      if (a.stamps) {  // diagnostics: count out-of-order neighbours (slot 10; 0 for a correct sort)
        __shared__ int s_bad;
        if (tid == 0) s_bad = 0;
        __syncthreads();
        for (int i = tid; i + 1 < n; i += NTH)
          if (key[i] > key[i + 1]) atomicAdd(&s_bad, 1);
        __syncthreads();
        if (tid == 0) a.stamps[(size_t)bid * kStampSlots + 10] = (uint64_t)s_bad;
      }
      const int nch = (n + CH - 1) / CH;
      for (int c = tid; c < nch; c += NTH) {
        const int p0 = c * CH, p1 = (p0 + CH < n ? p0 + CH : n) - 1;
        const K r0 = key[p0] >> 12, r1 = key[p1] >> 12;
        const bool cin = p0 > 0 && (key[p0 - 1] >> 12) == r0;
        const bool cout = p1 + 1 < n && (key[p1 + 1] >> 12) == r1;
        cflag[c] = (uint8_t)((cin ? 1 : 0) | (cout ? 2 : 0) | (r0 == r1 ? 4 : 0));
      }
      __syncthreads();
      stamp(a.stamps, 4, tid);
      // 3. runs inside each chunk.  Items: (chunk, d) of the second-order family with d fastest -- the lanes of one
      // chunk read one sample's 40-byte dE row per position and add one 40-byte table row per run: coalesced --
      // then one item per chunk for the first-order family
      const int n2 = (T.g2 && !(a.diag & 2)) ? nch * D : 0, n1 = (T.g1 && !(a.diag & 2)) ? nch : 0;
      const bool adds = !(a.diag & 4);
      auto item = [&](int it, int& c, int& j) {
        if (it < n2) {
          c = it / D;
          j = it - c * D;
        } else {
          c = it - n2;
          j = D;
        }
      };
      for (int it = tid; it < n2 + n1; it += NTH) {
        int c, j;
        item(it, c, j);
        const bool fam2 = j < D;
        float* g = fam2 ? T.g2 : T.g1;
        const int w = fam2 ? D : 1, jj = fam2 ? j : 0;
        const float* o = fam2 ? T.o2 : T.o1;
        const int p0 = c * CH, cnt = n - p0 < CH ? n - p0 : CH;
        const int fl = cflag[c];
        // every position's load issued before any is used (unguarded: positions past the batch read the chunk's last
        // key and are zeroed), so the chunk waits for one memory round trip, not one per position
        const float* src = fam2 ? a.sv_de + (int64_t)f * D + jj : a.dlogit;
        const int64_t sstride = fam2 ? FD : 1;
        const float scale = fam2 ? 1.f : lwf;
        float v[CH];
        uint32_t rq[CH];
        int sm[CH];
#pragma unroll
        for (int q = 0; q < CH; ++q) {
          const K k = key[p0 + (q < cnt ? q : cnt - 1)];
          sm[q] = (a.diag & 32) ? 0 : (int)(k & 4095);  // diagnostics: one sample's row
          rq[q] = q < cnt ? (uint32_t)(k >> 12) : 0xffffffffu;
        }
#pragma unroll
        for (int q = 0; q < CH; ++q) v[q] = src[(s0 + sm[q]) * sstride] * scale;
        if (o) {
#pragma unroll
          for (int q = 0; q < CH; ++q) v[q] *= o[(int64_t)partv[sm[q]] * w + jj];
        }
#pragma unroll
        for (int q = 0; q < CH; ++q) v[q] = q < cnt ? v[q] : 0.f;
        float sum = 0.f;
        uint32_t cur = rq[0];
        bool first = true;
        auto row_of = [&](uint32_t rl) { return (int64_t)rl * nbuck + bucket; };
#pragma unroll
        for (int q = 0; q < CH; ++q) {
          if (q < cnt) {
            if (rq[q] != cur) {  // a run ends inside the chunk
              if (first && (fl & 1)) lead[c * ncomp + j] = sum;
              else if (adds) atomicAdd(g + row_of(cur) * w + jj, sum);  // the row's only adder in this pass
              first = false;
              cur = rq[q];
              sum = 0.f;
            }
            sum += v[q];
          }
        }
        if (first && (fl & 1)) lead[c * ncomp + j] = sum;  // continues from the previous chunk (maybe into the next)
        else if (fl & 2) trail[c * ncomp + j] = sum;     // its head is here, its tail in the next chunk(s)
        else if (adds) atomicAdd(g + row_of(cur) * w + jj, sum);
      }
      // LDS-only barrier: the leads / trails are visible, the row adds stay in flight (phase 4 adds other rows)
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
      __builtin_amdgcn_s_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
      stamp(a.stamps, 5, tid);
      // 4. runs cut by chunk ends: the chunk with the head adds its trail and the following chunks' leads in order
      // (eight chunks' flags and leads read at a time: a long run's walk is not one LDS round trip per chunk)
      for (int it = tid; it < n2 + n1; it += NTH) {
        int c, j;
        item(it, c, j);
        const int fl = cflag[c];
        if (!(fl & 2) || (fl & 5) == 5) continue;  // no run leaves this chunk, or it is not headed here
        const bool fam2 = j < D;
        float* g = fam2 ? T.g2 : T.g1;
        float sum = trail[c * ncomp + j];
        int c2 = c + 1;
        bool done = false;
        while (!done) {
          uint8_t f8[8];
          float l8[8];
#pragma unroll
          for (int t = 0; t < 8; ++t) {
            const int cc = c2 + t < nch ? c2 + t : nch - 1;
            f8[t] = cflag[cc];
            l8[t] = lead[cc * ncomp + j];
          }
#pragma unroll
          for (int t = 0; t < 8; ++t) {
            if (!done) {
              sum += l8[t];
              done = (f8[t] & 6) != 6;  // the run ends in this chunk unless the whole chunk continues it
            }
          }
          c2 += 8;
        }
        const int p1 = c * CH + CH - 1;  // a chunk with a continuing last run is full
        const int64_t row = (int64_t)(uint32_t)(key[p1] >> 12) * nbuck + bucket;
        if (adds) atomicAdd(g + row * (fam2 ? D : 1) + (fam2 ? j : 0), sum);
      }
    }
    // the next pass's adds to the same rows come after these (this workgroup's own atomics, retired before the
    // barrier; no device-scope fence: nothing another workgroup reads); the last pass leaves them in flight
    if (s0 + kSortSeg < a.batch) {
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
      __syncthreads();
    }
  }
  stamp(a.stamps, 6, tid);
}

size_t sort_scatter_lds_bytes(int D) {
  const int NCH = sort_scatter_nch();
  return (size_t)kSortSeg * 12 + (size_t)(kSortThreads / 64) * 4 + (size_t)2 * NCH * (D + 1) * 4 + (size_t)NCH;
}

hipError_t launch_sort_scatter(const SortScatterArgs& a, int total_blocks, hipStream_t s) {
  if (a.ntasks <= 0 || a.batch <= 0 || total_blocks <= 0) return hipSuccess;
  const size_t lds = sort_scatter_lds_bytes(a.D);
  const void* fn = a.key64 ? reinterpret_cast<const void*>(sort_scatter_kernel<uint64_t>)
                           : reinterpret_cast<const void*>(sort_scatter_kernel<uint32_t>);
  hipError_t e = ensure_lds_limit(fn, lds);
  if (e != hipSuccess) return e;
  if (a.key64) hipLaunchKernelGGL(sort_scatter_kernel<uint64_t>, dim3(total_blocks), dim3(kSortThreads), lds, s, a);
  else hipLaunchKernelGGL(sort_scatter_kernel<uint32_t>, dim3(total_blocks), dim3(kSortThreads), lds, s, a);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------
// dW_l += G_l^T X_{l-1} with the MFMA operands loaded straight from global memory into registers (no LDS
// staging, no barrier in the K loop).  Workgroup = one 80 (n) x 80 (k) block of one layer over one batch split;
// its four waves each take a contiguous quarter of the split's rows and own the whole block: 5 x 5 16x16 MFMA
// tiles, 100 accumulators.  A k-step is four batch rows; for it a lane (m = lane & 15, row = lane >> 4) loads
// ONE float4 + ONE float of G and the same of X: tile t < 4 of the block maps its row / column m to n0 + 4m + t
// (the float4's element t), tile 4 to n0 + 64 + m -- so 16 lanes read 320 contiguous bytes of a row and every
// k-step is 4 loads for 25 MFMAs (round 2's LDS-staged 64 x 64 kernel: 8 staging loads, 8 LDS stores and 80 LDS
// reads per 64 MFMAs, 59.5 us against 42.1 for this one at Criteo-39, B = 4096; tools/ubench_dw).
// Loads run kDwrP k-steps ahead.  The four waves' blocks are summed through LDS in a fixed order ((w0 + w2) +
// (w1 + w3)) and added to dW with one coalesced atomic per element per workgroup; db_l = sum G_l rides on the
// k-block-0 workgroups, from the A operands they already hold.
// ---------------------------------------------------------------------------
constexpr int kDwrT = 80;       // block edge (5 MFMA tiles)
constexpr int kDwrLd = kDwrT;   // LDS row stride of the reduction blocks (52.5 KB: three workgroups per CU)
__device__ __forceinline__ int dwr_local(int t, int m) { return t < 4 ? 4 * m + t : 64 + m; }

// kDwrP: k-steps of loads in flight per wave; NW: waves per workgroup (each a contiguous 1/NW of the split's rows).
// Measured alike: kDwrP 4 / 6 / 8 (42.1 / 43.5 / 43.6 us) and eight waves per workgroup (43.7 us).
template <int kDwrP, int NW>
__device__ __forceinline__ void dwr_block(const DwArgs& a, int bid) {
  __shared__ __attribute__((aligned(16))) float red[2][kDwrT][kDwrLd];
  __shared__ float bred[NW][kDwrT];
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  int l = 1;
  while (l < a.H && bid >= a.blk0[l + 1]) ++l;
  bid -= a.blk0[l];
  const int per_layer_blocks = a.nnb * a.nkb[l];
  const int split = bid / per_layer_blocks;
  const int rem = bid - split * per_layer_blocks;
  const int nb = rem / a.nkb[l];
  const int kb = rem - nb * a.nkb[l];
  const int N = a.N, K = a.K[l], ldx = a.ldx[l];
  const int n0 = nb * kDwrT, k0 = kb * kDwrT;
  // this wave's rows: a contiguous 1/NW of the split (rows_per_split is a multiple of 16 NW)
  const int64_t q = a.rows_per_split / NW;
  const int64_t r_lo = (int64_t)split * a.rows_per_split + wave * q;
  int64_t r_hi = r_lo + q;
  if (r_hi > a.batch) r_hi = a.batch;
  const int nsteps = r_hi > r_lo ? (int)((r_hi - r_lo + 3) >> 2) : 0;
  const int m = lane & 15, kk = lane >> 4;
  // raw buffers over this wave's rows from column n0 / k0 on: rows past r_hi (another wave's) and everything past
  // the array read as 0; columns n >= N / k >= K of a valid row read the next row's values, which only reach
  // accumulators of outputs that are never stored
  const int64_t nrows = r_hi > r_lo ? r_hi - r_lo : 0;
  const int64_t g_bytes = nrows > 0 ? (nrows * N - n0) * 4 : 0;
  const int64_t x_bytes = nrows > 0 ? (nrows * ldx - k0) * 4 : 0;
  const __amdgpu_buffer_rsrc_t grs = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<float*>(a.G[l] + r_lo * N + n0), (short)0, (int)(g_bytes > 0 ? g_bytes : 0), 0x00020000);
  const __amdgpu_buffer_rsrc_t xrs = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<float*>(a.X[l] + r_lo * ldx + k0), (short)0, (int)(x_bytes > 0 ? x_bytes : 0), 0x00020000);
  const int gvo = (kk * N + 4 * m) * 4, xvo = (kk * ldx + 4 * m) * 4;  // this lane's float4 in a k-step
  const int gvo1 = (kk * N + 64 + m) * 4, xvo1 = (kk * ldx + 64 + m) * 4;  // and its float of tile 4
  const int gstep = 16 * N, xstep = 16 * ldx;                          // bytes per k-step (four rows)
  f32x4 ga[kDwrP], xa[kDwrP];
  float gb[kDwrP], xb[kDwrP];
#define DWR_LOAD(J, S)                                                                                  \
  do {                                                                                                  \
    const int go_ = (J) * gstep, xo_ = (J) * xstep;                                                     \
    ga[S] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(grs, gvo, go_, 0));         \
    gb[S] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(grs, gvo1, go_, 0));         \
    xa[S] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(xrs, xvo, xo_, 0));         \
    xb[S] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(xrs, xvo1, xo_, 0));         \
  } while (0)
  f32x4 acc[5][5];
#pragma unroll
  for (int i = 0; i < 5; ++i)
#pragma unroll
    for (int j = 0; j < 5; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  float bs0 = 0.f, bs1 = 0.f, bs2 = 0.f, bs3 = 0.f, bs4 = 0.f;
  // whole groups of kDwrP k-steps, every load unconditional: steps past the wave's rows read 0 (the buffer's
  // range), so the last group's prefetch and a ragged tail cost no branches and no register copies; a slot is
  // refilled right after the MFMAs that read it, kDwrP - 1 k-steps before it is needed
  const int nit = (nsteps + kDwrP - 1) / kDwrP;
#pragma unroll
  for (int s = 0; s < kDwrP; ++s) {
    DWR_LOAD(s, s);  // slot by slot, in the loop's order (so the loop's waits count the same loads)
    __builtin_amdgcn_sched_barrier(0);
  }
  for (int it = 0; it < nit; ++it) {
#pragma unroll
    for (int s = 0; s < kDwrP; ++s) {
      const float a0 = ga[s][0], a1 = ga[s][1], a2 = ga[s][2], a3 = ga[s][3], a4 = gb[s];
      const float b0 = xa[s][0], b1 = xa[s][1], b2 = xa[s][2], b3 = xa[s][3], b4 = xb[s];
      bs0 += a0; bs1 += a1; bs2 += a2; bs3 += a3; bs4 += a4;
#define DWR_ROW(TN, A)                                                                       \
  acc[TN][0] = __builtin_amdgcn_mfma_f32_16x16x4f32(A, b0, acc[TN][0], 0, 0, 0);             \
  acc[TN][1] = __builtin_amdgcn_mfma_f32_16x16x4f32(A, b1, acc[TN][1], 0, 0, 0);             \
  acc[TN][2] = __builtin_amdgcn_mfma_f32_16x16x4f32(A, b2, acc[TN][2], 0, 0, 0);             \
  acc[TN][3] = __builtin_amdgcn_mfma_f32_16x16x4f32(A, b3, acc[TN][3], 0, 0, 0);             \
  acc[TN][4] = __builtin_amdgcn_mfma_f32_16x16x4f32(A, b4, acc[TN][4], 0, 0, 0)
      DWR_ROW(0, a0);
      DWR_ROW(1, a1);
      DWR_ROW(2, a2);
      DWR_ROW(3, a3);
      DWR_ROW(4, a4);
#undef DWR_ROW
      __builtin_amdgcn_sched_barrier(0);  // the refill after every MFMA that reads the slot (no register copies)
      DWR_LOAD((it + 1) * kDwrP + s, s);
      __builtin_amdgcn_sched_barrier(0);  // and before the next slot's MFMAs (the scheduler sinks it to the loop end)
    }
  }
#undef DWR_LOAD
  float bs[5] = {bs0, bs1, bs2, bs3, bs4};

  // db_l: the block's column sums of G over the four rows of each lane group, then over the waves
  float* gB = kb == 0 ? a.gB[l] : nullptr;
  if (gB) {
#pragma unroll
    for (int t = 0; t < 5; ++t) {
      bs[t] += __shfl_xor(bs[t], 16);
      bs[t] += __shfl_xor(bs[t], 32);
    }
    if (kk == 0)
#pragma unroll
      for (int t = 0; t < 5; ++t) bred[wave][dwr_local(t, m)] = bs[t];
  }
  // the NW waves' blocks: waves 0 / 1 store, then waves 2 / 3, 4 / 5, ... add theirs in turn (a fixed order), and
  // every thread adds the two sums into dW row by row (coalesced atomics)
  float* gW = a.gW[l];
  for (int g = 0; g < NW / 2; ++g) {
    if (g > 0) __syncthreads();
    if (wave >> 1 == g) {
      float(&rb)[kDwrT][kDwrLd] = red[wave & 1];
#pragma unroll
      for (int tn = 0; tn < 5; ++tn)
#pragma unroll
        for (int tk = 0; tk < 5; ++tk)
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            float& r = rb[dwr_local(tn, 4 * kk + i)][dwr_local(tk, m)];
            r = g == 0 ? acc[tn][tk][i] : r + acc[tn][tk][i];
          }
    }
  }
  __syncthreads();
  // Split-K: with one split the block is added to dW (and db) directly -- one writer per element.  Otherwise by
  // default float atomics (the splits summed in arrival order: the last bits differ run to run); deterministic mode
  // (a.part set) writes every split's block to its own slice and the next launch (dw_sum_kernel) adds the slices in
  // split order -- the same bits on every run (a last-split ticket instead needs device-scope fences, whose L2
  // write-backs cost more than the launch).
  constexpr int BE = kDwrT * kDwrT;
  const int splits = a.splits;
  const int ublk = a.blk0[l] / splits + rem;  // the block's index over all layers, without the split
  float bsum = 0.f;
  if (gB && tid < kDwrT) {
    bsum = bred[0][tid];
#pragma unroll
    for (int w = 1; w < NW; ++w) bsum += bred[w][tid];
  }
  if (splits > 1 && !a.part) {
    // the default (fast) form: float atomics, one per element per split -- the sum of the splits in arrival order
    if (gB && tid < kDwrT && n0 + tid < N) atomicAdd(gB + n0 + tid, bsum);
    if (!gW) return;
    for (int e = tid; e < BE; e += 64 * NW) {  // consecutive lanes on consecutive k of a row: 256 contiguous bytes
      const int r = e / kDwrT, c = e - r * kDwrT;
      const int n = n0 + r, k = k0 + c;
      if (n < N && k < K) atomicAdd(gW + (int64_t)n * K + k, red[0][r][c] + red[1][r][c]);
    }
    return;
  }
  if (splits > 1) {
    // deterministic: this split's block and column sums to its slices; dw_sum_kernel adds them in split order
    float* mine = a.part + ((size_t)ublk * splits + split) * BE;
    for (int e = tid; e < BE; e += 64 * NW) {
      const int r = e / kDwrT, c = e - r * kDwrT;
      mine[e] = red[0][r][c] + red[1][r][c];
    }
    if (gB && tid < kDwrT) a.bpart[((size_t)ublk * splits + split) * kDwrT + tid] = bsum;
    return;
  }
  if (gB && tid < kDwrT && n0 + tid < N) gB[n0 + tid] += bsum;
  if (!gW) return;
  for (int e = tid; e < BE; e += 64 * NW) {
    const int r = e / kDwrT, c = e - r * kDwrT;
    const int n = n0 + r, k = k0 + c;
    if (n < N && k < K) gW[(int64_t)n * K + k] += red[0][r][c] + red[1][r][c];
  }
}

// XCD-local groups (workgroup p runs on XCD p % 8): a group of a.xcd_gs consecutive logical blocks that share operand
// slices goes to one XCD, so one block fetches a slice and the others read it from that XCD's L2.  Whole rounds of
// eight groups first (XCD x takes groups x, x + 8, ...), then the leftover groups' blocks round-robin over the XCDs;
// -1 for the physical slots past the last block (those workgroups exit)
__device__ __forceinline__ int dwr_logical(const DwArgs& a, int p) {
  if (a.xcd_gs <= 0) return p;
  const int x = p & 7, s = p >> 3;
  const int full = a.xcd_groups / 8 * 8, head = full / 8 * a.xcd_gs;
  if (s < head) return ((s / a.xcd_gs) * 8 + x) * a.xcd_gs + s % a.xcd_gs;
  const int e = (s - head) * 8 + x;
  return e < (a.xcd_groups - full) * a.xcd_gs ? full * a.xcd_gs + e : -1;
}

template <int kDwrP, int NW>
__global__ void __launch_bounds__(64 * NW) dwr_kernel(DwArgs a) {
  const int li = dwr_logical(a, blockIdx.x);
  if (li >= 0) dwr_block<kDwrP, NW>(a, li);
}

// the split slices of every weight / bias gradient element added in split order (the GEMM's second launch when it
// splits the batch): kDwSumParts workgroups per 80 x 80 block (16 of its rows each), its splits' slices contiguous --
// every slice read in flight before the adds (one thread per element walking the layers with integer divisions took
// 7.2 us at Criteo-39; one workgroup per block 13)
constexpr int kDwSumParts = 5;
__global__ void __launch_bounds__(256) dw_sum_kernel(DwArgs a) {
  constexpr int BE = kDwrT * kDwrT;
  constexpr int BP = BE / kDwSumParts;  // elements of this workgroup's part
  constexpr int PT = (BP + 255) / 256;
  static_assert(BE % kDwSumParts == 0, "block parts");
  const int splits = a.splits;
  const int ub = blockIdx.x / kDwSumParts, part = blockIdx.x - ub * kDwSumParts;
  int l = 1;
  while (l < a.H && ub >= a.blk0[l + 1] / splits) ++l;
  const int rem = ub - a.blk0[l] / splits;
  const int nb = rem / a.nkb[l], kb = rem - nb * a.nkb[l];
  const int n0 = nb * kDwrT, k0 = kb * kDwrT;
  const int tid = threadIdx.x;
  float* gW = a.gW[l];
  if (gW) {
    const int K = a.K[l];
    const float* sl = a.part + (size_t)ub * splits * BE + part * BP;
    float v[PT];
#pragma unroll
    for (int j = 0; j < PT; ++j) {
      const int e = tid + 256 * j;
      v[j] = e < BP ? sl[e] : 0.f;
    }
    for (int sp = 1; sp < splits; ++sp) {
      float w[PT];
#pragma unroll
      for (int j = 0; j < PT; ++j) {
        const int e = tid + 256 * j;
        w[j] = e < BP ? sl[(size_t)sp * BE + e] : 0.f;
      }
#pragma unroll
      for (int j = 0; j < PT; ++j) v[j] += w[j];
    }
#pragma unroll
    for (int j = 0; j < PT; ++j) {
      const int e = part * BP + tid + 256 * j;
      const int r = e / kDwrT, c = e - r * kDwrT;
      const int n = n0 + r, k = k0 + c;
      if (tid + 256 * j < BP && n < a.N && k < K) gW[(int64_t)n * K + k] += v[j];
    }
  }
  if (a.gB[l] && kb == 0 && part == 0 && tid < kDwrT && n0 + tid < a.N) {
    const float* bp = a.bpart + (size_t)ub * splits * kDwrT + tid;
    float v = bp[0];
    for (int sp = 1; sp < splits; ++sp) v += bp[(size_t)sp * kDwrT];
    a.gB[l][n0 + tid] += v;
  }
}

// The weight-gradient GEMM and the shallow reductions' final sums as ONE launch (the one-stream step): the GEMM is
// one round of workgroups that leaves CUs idle (225 for 256 CUs at Criteo-39), and the final sums' workgroups
// (39) run there instead of in a launch of their own after it
template <int kDwrP, int NW>
__global__ void __launch_bounds__(64 * NW) dwr_reduce_kernel(DwArgs a, RedArgs r, int nblk, int dw_blocks) {
  if ((int)blockIdx.x < dw_blocks) {
    const int li = dwr_logical(a, blockIdx.x);
    if (li >= 0) dwr_block<kDwrP, NW>(a, li);
  } else {
    reduce_final_block(r, nblk, (int)blockIdx.x - dw_blocks);
  }
}

// ---------------------------------------------------------------------------
// Adam (torch.optim.Adam, single-tensor form, torch/optim/adam.py _single_tensor_adam):
// g += wd * p; m = lerp(m, g, 1 - b1);
// v = v * b2 + (1 - b2) * g * g; p -= (lr / bc1) * m / (sqrt(v) / sqrt(bc2) + eps)
// ---------------------------------------------------------------------------
// one element of torch.optim.Adam: torch's CPU kernels' evaluation order -- fmadd where ATen's vector path
// uses one, every other product / sum rounded on its own
struct AdamCoef {
  float step_size, omb1, b2, omb2, eps, wd, bc2_sqrt;
};
__device__ __forceinline__ void adam_elem(const AdamCoef& c, float& p, float g, float& m, float& v) {
  if (c.wd != 0.f) g = fmaf(c.wd, p, g);                          // grad.add(param, alpha=wd): ATen's fmadd
  m = fmaf(c.omb1, __fsub_rn(g, m), m);                            // exp_avg.lerp_(grad, 1-b1): fmadd, w < 0.5
  v = __fmul_rn(v, c.b2);                                          // exp_avg_sq.mul_(b2)
  v = __fadd_rn(v, __fmul_rn(__fmul_rn(c.omb2, g), g));           //   .addcmul_(g, g, 1-b2)
  const float denom = __fadd_rn(__fdiv_rn(__fsqrt_rn(v), c.bc2_sqrt), c.eps);  // sqrt(v)/sqrt(bc2) + eps
  p = __fadd_rn(p, __fdiv_rn(__fmul_rn(-c.step_size, m), denom));  // addcdiv_(m, denom, -lr/bc1)
}

// a block's kAdamBlock (4096) elements: when the tensor's four arrays are 16-byte aligned thread t owns the four
// float4 [4t + 1024u, 4t + 1024u + 4), u < 4 -- all sixteen 16-byte loads issued before any update (bytes in flight
// for HBM), three 16-byte stores each -- else the lanes take consecutive elements
template <typename TList>
__device__ __forceinline__ void adam_block(const TList& list, const AdamCoef& c, int bid) {
  if (list.n <= 0) return;
  int lo = 0, hi = list.n - 1;
  while (lo < hi) {  // last tensor whose block0 <= bid
    const int mid = (lo + hi + 1) >> 1;
    if (list.block0[mid] <= bid) lo = mid;
    else hi = mid - 1;
  }
  const AdamTensor T = list.t[lo];
  const int64_t i0 = (int64_t)(bid - list.block0[lo]) * kAdamBlock;
  const bool vec = (((uintptr_t)T.p | (uintptr_t)T.g | (uintptr_t)T.m | (uintptr_t)T.v) & 15) == 0;
  if (!vec) {
    // unaligned arrays (a gradient view at an odd offset of the flat buffer): lane-consecutive elements
    for (int64_t j = i0 + threadIdx.x; j < i0 + kAdamBlock && j < T.n; j += 256) {
      float p = T.p[j], m = T.m[j], v = T.v[j];
      adam_elem(c, p, T.g[j], m, v);
      T.m[j] = m;
      T.v[j] = v;
      T.p[j] = p;
    }
    return;
  }
  constexpr int U = kAdamBlock / 1024;
  float4 p[U], g[U], m[U], v[U];
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int64_t i = i0 + 1024 * u + 4 * threadIdx.x;
    if (i + 3 < T.n) {
      p[u] = *reinterpret_cast<const float4*>(T.p + i);
      g[u] = *reinterpret_cast<const float4*>(T.g + i);
      m[u] = *reinterpret_cast<const float4*>(T.m + i);
      v[u] = *reinterpret_cast<const float4*>(T.v + i);
    }
  }
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int64_t i = i0 + 1024 * u + 4 * threadIdx.x;
    if (i + 3 < T.n) {
      adam_elem(c, p[u].x, g[u].x, m[u].x, v[u].x);
      adam_elem(c, p[u].y, g[u].y, m[u].y, v[u].y);
      adam_elem(c, p[u].z, g[u].z, m[u].z, v[u].z);
      adam_elem(c, p[u].w, g[u].w, m[u].w, v[u].w);
      *reinterpret_cast<float4*>(T.m + i) = m[u];
      *reinterpret_cast<float4*>(T.v + i) = v[u];
      *reinterpret_cast<float4*>(T.p + i) = p[u];
    } else {
      for (int k = 0; k < 4; ++k) {
        if (i + k >= T.n) break;
        float pp = T.p[i + k], mm = T.m[i + k], vv = T.v[i + k];
        adam_elem(c, pp, T.g[i + k], mm, vv);
        T.m[i + k] = mm;
        T.v[i + k] = vv;
        T.p[i + k] = pp;
      }
    }
  }
}

__global__ void __launch_bounds__(256) adam_kernel(const AdamList list, float step_size, float omb1, float b2,
                                                   float omb2, float eps, float wd, float bc2_sqrt) {
  adam_block(list, AdamCoef{step_size, omb1, b2, omb2, eps, wd, bc2_sqrt}, blockIdx.x);
}

// Graph-replayable Adam: every workgroup derives the step's scalars from the device counter + 1 (in double, as
// torch does from Python floats, then f32) -- no separate prep launch; in the step's last launch the last workgroup
// to finish (a ticket counter) advances the counter, after every workgroup of the step has read it.
__device__ __forceinline__ AdamCoef adam_coef(int64_t step, const AdamHyper& h) {
  const double bc1 = 1.0 - pow(h.b1, (double)step);
  const double bc2 = 1.0 - pow(h.b2, (double)step);
  return AdamCoef{(float)(h.lr / bc1), (float)(1.0 - h.b1), (float)h.b2, (float)(1.0 - h.b2), (float)h.eps,
                  (float)h.wd, (float)sqrt(bc2)};
}

// (a bounded grid walking the 1024-element blocks: one ticket atomic per workgroup, a few thousand at most -- one
// per block serialised on the counter's address)
template <typename TList>
__device__ __forceinline__ void adam_dev_part(const TList& list, AdamDevState* __restrict__ st, const AdamHyper& h,
                                              int bump, int nblocks, int wg, int nwg) {
  __shared__ AdamCoef sc;
  __shared__ int64_t s_step;
  if (threadIdx.x == 0) {
    s_step = st->step + 1;
    sc = adam_coef(s_step, h);
  }
  __syncthreads();
  for (int b = wg; b < nblocks; b += nwg) adam_block(list, sc, b);
  if (bump && threadIdx.x == 0 && atomicAdd(&st->ticket, 1) == nwg - 1) {
    const AdamCoef c = sc;
    st->step_size = c.step_size;
    st->omb1 = c.omb1;
    st->b2 = c.b2;
    st->omb2 = c.omb2;
    st->eps = c.eps;
    st->wd = c.wd;
    st->bc2_sqrt = c.bc2_sqrt;
    st->ticket = 0;
    st->step = s_step;
  }
}

__global__ void __launch_bounds__(256) adam_dev_kernel(const AdamList list, AdamDevState* __restrict__ st,
                                                       const AdamHyper h, int bump, int nblocks) {
  adam_dev_part(list, st, h, bump, nblocks, blockIdx.x, gridDim.x);
}

// dL/dz of BCE-with-logits with the loss normalised by `denom` (torch: (sigmoid(z) - y) * 1, then
// divided by numel for reduction='mean'); optionally the loss sum (stable form) into *loss_sum.
__global__ void __launch_bounds__(256) bce_grad_kernel(const float* __restrict__ z, const float* __restrict__ y,
                                                       int64_t n, float denom, float* __restrict__ dz,
                                                       float* __restrict__ loss_sum) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  float l = 0.f;
  if (i < n) {
    const float x = z[i], t = y[i];
    const float sg = 1.f / (1.f + expf(-x));
    dz[i] = __fdiv_rn(__fsub_rn(sg, t), denom);
    l = fmaxf(x, 0.f) - x * t + log1pf(expf(-fabsf(x)));
  }
  if (loss_sum) {
    for (int o = 32; o >= 1; o >>= 1) l += __shfl_xor(l, o);
    __shared__ float ws[4];
    if ((threadIdx.x & 63) == 0) ws[threadIdx.x >> 6] = l;
    __syncthreads();
    if (threadIdx.x == 0) atomicAdd(loss_sum, ((ws[0] + ws[1]) + ws[2]) + ws[3]);
  }
}

#endif  // DFWFM_KD

// ---------------------------------------------------------------------------
// launchers
// ---------------------------------------------------------------------------
template <int D, int TPW, int NG>
static hipError_t launch_bwd_t(const BwdArgs& a, size_t lds, hipStream_t s) {
  auto k = bwd_kernel<D, TPW, NG>;
  {
    hipError_t e = ensure_lds_limit(reinterpret_cast<const void*>(k), lds);
    if (e != hipSuccess) return e;
  }
  const unsigned grid = (unsigned)((a.batch + kBM - 1) / kBM);
  hipLaunchKernelGGL(k, dim3(grid), dim3(64 * NG), lds, s, a);
  return hipGetLastError();
}

template <int D>
static hipError_t launch_bwd_d(const BwdArgs& a, int tpw, int ng, size_t lds, hipStream_t s) {
  if (ng == 8) {
    switch (tpw) {
      case 1: return launch_bwd_t<D, 1, 8>(a, lds, s);
      case 2: return launch_bwd_t<D, 2, 8>(a, lds, s);
      case 3: return launch_bwd_t<D, 3, 8>(a, lds, s);
      case 4: return launch_bwd_t<D, 4, 8>(a, lds, s);
      default: return hipErrorInvalidValue;
    }
  }
  switch (tpw) {
    case 1: return launch_bwd_t<D, 1, 4>(a, lds, s);
    case 2: return launch_bwd_t<D, 2, 4>(a, lds, s);
    case 3: return launch_bwd_t<D, 3, 4>(a, lds, s);
    case 4: return launch_bwd_t<D, 4, 4>(a, lds, s);
    case 5: return launch_bwd_t<D, 5, 4>(a, lds, s);
    case 6: return launch_bwd_t<D, 6, 4>(a, lds, s);
    case 7: return launch_bwd_t<D, 7, 4>(a, lds, s);
    case 8: return launch_bwd_t<D, 8, 4>(a, lds, s);
    default: return hipErrorInvalidValue;
  }
}

#ifdef DFWFM_KD
// one translation unit per embedding size (parallel build): this one's backward launcher
hipError_t DFWFM_PER_D(launch_backward_d)(const BwdArgs& a, int tpw, int ng, size_t lds, hipStream_t s) {
  return launch_bwd_d<DFWFM_KD>(a, tpw, ng, lds, s);
}
#else
hipError_t launch_backward(const BwdArgs& a, int D, int tpw, int ng, size_t lds, hipStream_t s) {
  switch (D) {
    case 4: return launch_backward_d4(a, tpw, ng, lds, s);
    case 8: return launch_backward_d8(a, tpw, ng, lds, s);
    case 10: return launch_backward_d10(a, tpw, ng, lds, s);
    case 16: return launch_backward_d16(a, tpw, ng, lds, s);
    case 32: return launch_backward_d32(a, tpw, ng, lds, s);
    default: return hipErrorInvalidValue;
  }
}

hipError_t launch_reduce_final(const RedArgs& a, hipStream_t s) {
  const int nblk = (int)((a.batch + kBM - 1) / kBM);
  const int P = red_outputs(a.F, a.D, a.N, a.num);
  hipLaunchKernelGGL(reduce_final_kernel, dim3((P + 63) / 64), dim3(256), 0, s, a, nblk);
  return hipGetLastError();
}

hipError_t launch_reduce(const RedArgs& a, hipStream_t s) {
  if (a.batch <= 0) return hipSuccess;
  const unsigned grid = (unsigned)((a.batch + kBM - 1) / kBM);
  if (a.F * a.D > kRedMaxFD || a.N > kRedMaxN || a.num * a.D > 512) return hipErrorInvalidValue;
  const size_t lds = sizeof(float) * (size_t)red_layout(a.F, a.D, a.N, a.num).total;
  {
    hipError_t e = ensure_lds_limit(reinterpret_cast<const void*>(reduce_kernel), lds);
    if (e != hipSuccess) return e;
  }
  hipLaunchKernelGGL(reduce_kernel, dim3(grid), dim3(256), lds, s, a);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  const int P = red_outputs(a.F, a.D, a.N, a.num);
  hipLaunchKernelGGL(reduce_final_kernel, dim3((P + 63) / 64), dim3(256), 0, s, a, (int)grid);
  return hipGetLastError();
}

hipError_t launch_scatter(const ScatterArgs& a, int total_blocks, hipStream_t s) {
  if (total_blocks <= 0 || a.ntasks <= 0) return hipSuccess;
  // LDS for the largest privatised table of this launch only (not kPrivFloats): more workgroups per CU
  size_t floats = 0;
  for (int i = 0; i < a.ntasks; ++i) {
    if (!(a.t[i].kind & kScatterPriv)) continue;
    if (a.chunk > 4 * 256) return hipErrorInvalidValue;
    const size_t f = (size_t)a.t[i].rows * ((a.t[i].src == 0 ? a.D : 1) + 1);
    floats = f > floats ? f : floats;
  }
  if (floats > (size_t)kPrivFloats) return hipErrorInvalidValue;
  if (a.chunk > 256) return hipErrorInvalidValue;  // the srow / spart staging of a chunk
  const size_t lds = sizeof(float) * (floats > 0 ? floats : 1);
  hipError_t e = ensure_lds_limit(reinterpret_cast<const void*>(scatter_kernel), lds);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(scatter_kernel, dim3(total_blocks), dim3(256), lds, s, a);
  return hipGetLastError();
}

// the XCD-local grouping of the weight-gradient GEMM's blocks (dwr_logical) and the physical grid it needs: each
// (layer, split)'s nnb x nkb blocks share every G_l and X_{l-1} slice and fit one XCD's 32 CUs (DFWFM_DIAG dwr_xcd=1:
// the nkb blocks of one G_l slice per group, 0: blockIdx order)
static int dwr_xcd_plan(const DwArgs& a, int total_blocks, DwArgs& b) {
  b = a;
  b.xcd_gs = 0;
  b.xcd_groups = 0;
  bool uniform = a.H >= 1;
  for (int l = 2; l <= a.H; ++l) uniform = uniform && a.nkb[l] == a.nkb[1];
  const int mode = diag_opt("dwr_xcd", 2);
  if (!uniform || !mode || total_blocks % a.nkb[1] != 0) return total_blocks;
  const int sg = a.nnb * a.nkb[1];
  b.xcd_gs = (mode == 2 && sg <= 32) ? sg : a.nkb[1];
  b.xcd_groups = total_blocks / b.xcd_gs;
  const int full = b.xcd_groups / 8 * 8;
  return 8 * (full / 8 * b.xcd_gs + ((b.xcd_groups - full) * b.xcd_gs + 7) / 8);
}

static hipError_t launch_dw_sum(const DwArgs& a, hipStream_t s) {
  if (a.splits <= 1 || !a.part) return hipSuccess;
  const int blocks = a.blk0[a.H + 1] / a.splits;  // unsplit 80 x 80 blocks over every layer
  if (blocks <= 0) return hipSuccess;
  hipLaunchKernelGGL(dw_sum_kernel, dim3((unsigned)(blocks * kDwSumParts)), dim3(256), 0, s, a);
  return hipGetLastError();
}

hipError_t launch_dw(const DwArgs& a, int total_blocks, hipStream_t s) {
  if (total_blocks <= 0) return hipSuccess;
  // a wave's raw-buffer ranges and k-step offsets are 32-bit byte counts over its quarter of a split's rows
  const int64_t q = a.rows_per_split / 4 + 4;
  for (int l = 1; l <= a.H; ++l) {
    const int64_t w = a.ldx[l] > a.N ? a.ldx[l] : a.N;
    if (q * w * 4 >= 0x7fffffffLL) return hipErrorInvalidValue;
  }
  DwArgs b;
  const int phys = dwr_xcd_plan(a, total_blocks, b);
  hipLaunchKernelGGL((dwr_kernel<4, 4>), dim3(phys), dim3(256), 0, s, b);
  hipError_t e = hipGetLastError();
  return e != hipSuccess ? e : launch_dw_sum(b, s);
}

hipError_t launch_dw_reduce(const DwArgs& a, int total_blocks, const RedArgs& r, hipStream_t s) {
  if (total_blocks <= 0) return launch_reduce_final(r, s);
  const int64_t q = a.rows_per_split / 4 + 4;
  for (int l = 1; l <= a.H; ++l) {
    const int64_t w = a.ldx[l] > a.N ? a.ldx[l] : a.N;
    if (q * w * 4 >= 0x7fffffffLL) return hipErrorInvalidValue;
  }
  const int nblk = (int)((r.batch + kBM - 1) / kBM);
  const int P = red_outputs(r.F, r.D, r.N, r.num);
  const int rblocks = (P + 63) / 64;
  DwArgs b;
  const int phys = dwr_xcd_plan(a, total_blocks, b);
  hipLaunchKernelGGL((dwr_reduce_kernel<4, 4>), dim3(phys + rblocks), dim3(256), 0, s, b, r, nblk, phys);
  hipError_t e = hipGetLastError();
  return e != hipSuccess ? e : launch_dw_sum(b, s);
}

hipError_t launch_adam(const AdamList& list, int total_blocks, float step_size, float omb1, float b2, float omb2,
                       float eps, float wd, float bc2_sqrt, hipStream_t s) {
  if (total_blocks <= 0) return hipSuccess;
  hipLaunchKernelGGL(adam_kernel, dim3(total_blocks), dim3(256), 0, s, list, step_size, omb1, b2, omb2, eps, wd,
                     bc2_sqrt);
  return hipGetLastError();
}

hipError_t launch_adam_dev(const AdamList& list, int total_blocks, AdamDevState* st, const AdamHyper& h, bool bump,
                           hipStream_t s) {
  if (total_blocks <= 0) return hipSuccess;
  const int grid = total_blocks < kAdamGrid ? total_blocks : kAdamGrid;
  hipLaunchKernelGGL(adam_dev_kernel, dim3(grid), dim3(256), 0, s, list, st, h, bump ? 1 : 0, total_blocks);
  return hipGetLastError();
}

hipError_t launch_bce_grad(const float* z, const float* y, int64_t n, float denom, float* dz, float* loss_sum,
                           hipStream_t s) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(bce_grad_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, z, y, n, denom, dz,
                     loss_sum);
  return hipGetLastError();
}

#endif  // DFWFM_KD

}  // namespace dfwfm
