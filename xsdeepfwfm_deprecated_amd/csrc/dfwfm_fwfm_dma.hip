// dfwfm_fwfm_dma.hip -- the MLP-free forward (use_deep = 0, reference model/DeepFMs.py:300-367 + :445-458) over a
// batch set as ONE persistent launch whose embedding rows reach LDS by LDS-DMA (global_load_lds_dword), with the
// next tile's rows in flight while the current tile's FwFM runs.
//
// fwd_kernel's MLP-free instantiation (PART 3) is a chain per 16-sample tile -- keys -> rows -> FwFM -> sums -- and
// a CU overlaps only the five tiles it holds at once; every row it gathers passes through registers (a load, a wait,
// an LDS store), so a persistent form that kept the next tile's rows in flight ran out of registers (DESIGN.md
// §3.6).  Here the rows go straight from memory into the E tile: a workgroup walks tiles w, w + G, w + 2G, ... of
// the set and per tile
//   [A] waits for its own DMA (vmcnt) and meets the other waves (raw s_barrier: a __syncthreads fence would drain
//       the DMA it does not need yet),
//   [B] issues the Xi keys of the tile two ahead, forms the current tile's numerical fields (v_f[0] * Xv) and turns
//       the next tile's keys into row addresses (range-checked like nn.Embedding; out of range -> row 0 + flag),
//   [C] issues the next tile's 26 x 16 rows (ten lanes per 40-B row, one DMA per 64 dwords: rows need no
//       registers in flight), its first-order entries and its Xv, then runs the current tile's FwFM on MFMA,
//   [D] forms first + second and the logit.
// Every sum is fwd_kernel PART 3's (the U'E pieces of kP3Pieces, the 16-lane DPP sums, the (first + second) + bias
// order), so each batch's logits are bit-identical to its own dfwfm_forward (tests/test_gpu_batches.py).
//
// LDS (one workgroup's, two per CU): the E tile field-major, E[l][b][d] at (l * 16 + b) * D + d, so the categorical
// fields of all 16 samples are one contiguous run of 16 * C * D dwords (whole 64-dword DMA pieces) and a column
// n = b * D + d of the FwFM's B operand is E[l][n] -- stride 16 * D over the fields; fields F .. 4S - 1 are zero.
#include "dfwfm_internal.h"
#include "dfwfm_device.h"

namespace dfwfm {

namespace {

// one dword per lane, global -> LDS at lds_base + lane * 4 (lds_base wave-uniform; inactive lanes write nothing)
__device__ __forceinline__ void glds_dword(const void* g, float* lds_base) {
  __builtin_amdgcn_global_load_lds((__attribute__((address_space(1))) void*)g,
                                   (__attribute__((address_space(3))) void*)lds_base, 4, 0, 0);
}

__device__ __forceinline__ void wait_dma() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

// LDS writes / reads of this wave done, then the workgroup barrier; no vmcnt (DMA of the next tile stays in flight)
__device__ __forceinline__ void lds_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

// LDS carve-up in floats.  The DMA targets (three row tiles [C][16][D], three first-order tiles [C][16], three Xv
// tiles [16][num], two key tiles [16][C] int64) are rounded up to whole 64-dword pieces: every DMA runs with all 64
// lanes (the instruction count per wave is then known, which the counted vmcnt waits need), and the lanes past a
// region's end write into its rounding.  Keys go out one tile before the rows they address (three key tiles).  Then the numerical fields' E [num][16][D] (formed per tile), the validated
// row indices [C][16], the tables' bases [C] (second order, first order), the numerical fields' vectors [num][D] and
// the FwFM column sums [16 D].
constexpr int kDmaDepth = 2;               // rows are issued this many tiles ahead
constexpr int kDmaBufs = kDmaDepth + 1;    // row / first-order / Xv tiles in LDS

__host__ __device__ inline int r64(int x) { return (x + 63) & ~63; }

struct DmaLayout {
  int cat, ncat, fo, nfo, xv, nxv, keys, nkey, nume, ridx, base2, base1, vnum, part2, zero, total;
};

__host__ __device__ inline DmaLayout dma_layout(int F, int num, int D) {
  const int C = F - num;
  DmaLayout L;
  L.ncat = r64(C * kBM * D);
  L.nfo = r64(kBM * C);
  L.nxv = r64(kBM * num);
  L.nkey = r64(2 * kBM * C);
  int o = 0;
  L.cat = o;   o += kDmaBufs * L.ncat;
  L.fo = o;    o += kDmaBufs * L.nfo;
  L.xv = o;    o += kDmaBufs * L.nxv;
  L.keys = o;  o += kDmaBufs * L.nkey;
  L.nume = o;  o += r4(num * kBM * D);
  L.ridx = o;  o += r4(kBM * C);
  L.base2 = o; o += r4(2 * C);
  L.base1 = o; o += r4(2 * C);
  L.vnum = o;  o += r4(num * D);
  L.part2 = o; o += r4(kBM * D);
  L.zero = o;  o += 4;
  L.total = o;
  return L;
}

struct DmaTile {
  const int64_t* xi;
  const float* xv;
  float* out;
  int64_t b0;
  int nrows;
};

// the set's tiles w, w + G, w + 2G, ... as (batch, tile in batch), advanced without a division per step
struct TileCursor {
  int bi, tb;
  __device__ __forceinline__ void init(const FwdArgs& p, int t) {
    bi = p.nb > 1 ? t / p.tiles : 0;
    tb = t - bi * p.tiles;
  }
  __device__ __forceinline__ void step(const FwdArgs& p, int G) {
    tb += G;
    while (tb >= p.tiles) {
      tb -= p.tiles;
      ++bi;
    }
  }
  __device__ __forceinline__ DmaTile tile(const FwdArgs& p) const {
    DmaTile r;
    if (p.nb > 1) {
      r.xi = p.set_xi[bi];
      r.xv = p.set_xv[bi];
      r.out = p.set_out[bi];
    } else {
      r.xi = p.xi;
      r.xv = p.xv;
      r.out = p.out;
    }
    r.b0 = (int64_t)tb * kBM;
    const int64_t left = p.batch - r.b0;
    r.nrows = left < kBM ? (int)left : kBM;
    return r;
  }
};

// s_waitcnt vmcnt(n) for a wave-uniform n in [0, 63] (the immediate is an encoding field)
__device__ __forceinline__ void wait_vm(int n) {
  switch (n) {
#define DFWFM_VMW(k) case k: asm volatile("s_waitcnt vmcnt(" #k ")" ::: "memory"); break;
    DFWFM_VMW(0) DFWFM_VMW(1) DFWFM_VMW(2) DFWFM_VMW(3) DFWFM_VMW(4) DFWFM_VMW(5) DFWFM_VMW(6) DFWFM_VMW(7)
    DFWFM_VMW(8) DFWFM_VMW(9) DFWFM_VMW(10) DFWFM_VMW(11) DFWFM_VMW(12) DFWFM_VMW(13) DFWFM_VMW(14) DFWFM_VMW(15)
    DFWFM_VMW(16) DFWFM_VMW(17) DFWFM_VMW(18) DFWFM_VMW(19) DFWFM_VMW(20) DFWFM_VMW(21) DFWFM_VMW(22) DFWFM_VMW(23)
    DFWFM_VMW(24) DFWFM_VMW(25) DFWFM_VMW(26) DFWFM_VMW(27) DFWFM_VMW(28) DFWFM_VMW(29) DFWFM_VMW(30) DFWFM_VMW(31)
    DFWFM_VMW(32) DFWFM_VMW(33) DFWFM_VMW(34) DFWFM_VMW(35) DFWFM_VMW(36) DFWFM_VMW(37) DFWFM_VMW(38) DFWFM_VMW(39)
    DFWFM_VMW(40) DFWFM_VMW(41) DFWFM_VMW(42) DFWFM_VMW(43) DFWFM_VMW(44) DFWFM_VMW(45) DFWFM_VMW(46) DFWFM_VMW(47)
    DFWFM_VMW(48) DFWFM_VMW(49) DFWFM_VMW(50) DFWFM_VMW(51) DFWFM_VMW(52) DFWFM_VMW(53) DFWFM_VMW(54) DFWFM_VMW(55)
    DFWFM_VMW(56) DFWFM_VMW(57) DFWFM_VMW(58) DFWFM_VMW(59) DFWFM_VMW(60) DFWFM_VMW(61) DFWFM_VMW(62)
#undef DFWFM_VMW
    default: asm volatile("s_waitcnt vmcnt(63)" ::: "memory"); break;
  }
}

}  // namespace

// diagnostics only (timing of the phases; results invalid): skip the FwFM MFMAs / the row DMA
constexpr int kDmaDiagNoFwfm = 1 << 25, kDmaDiagNoRows = 1 << 26;

// D: embedding size; MTC: FwFM row tiles (ceil(F / 16) <= 3, the U'E pieces' U' fragments in registers); SL: the
// K steps of the last row tile (S = 4 (MTC - 1) + SL): every step and MFMA of the FwFM is known at compile time
template <int D, int MTC, int SL>
__global__ void __launch_bounds__(256) fwfm_dma_kernel(FwdArgs p, int ntiles) {
  constexpr int NTH = 256, NW = 4;
  constexpr int S = 4 * (MTC - 1) + SL;  // FwFM K steps of 4 fields
  constexpr int FS = kBM * D;            // E floats per field
  constexpr int RA = (kBM * 48 + NTH - 1) / NTH;  // row-index rows per thread (C <= 48)
  constexpr int KP = (2 * kBM * 48 + 63) / 64;     // key pieces per tile (C <= 48)
  constexpr int XP = (kBM * 64 + 63) / 64;         // Xv pieces per tile (num <= 64)
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int F = p.F, num = p.num, C = F - num;
  const int flags = p.flags;
  const DmaLayout L = dma_layout(F, num, D);
  float* const catbuf = smem + L.cat;
  float* const fobuf = smem + L.fo;
  float* const xvbuf = smem + L.xv;
  float* const keybuf = smem + L.keys;
  float* const nume = smem + L.nume;
  int32_t* const ridx = reinterpret_cast<int32_t*>(smem + L.ridx);
  const float** const base2 = reinterpret_cast<const float**>(smem + L.base2);
  const float** const base1 = reinterpret_cast<const float**>(smem + L.base1);
  float* const vnum = smem + L.vnum;
  float* const part2 = smem + L.part2;
  float* const zero = smem + L.zero;
  const int G = gridDim.x;
  const int w0 = blockIdx.x;
  const int nmine = w0 < ntiles ? (ntiles - w0 + G - 1) / G : 0;
  if (nmine == 0) return;

  // ---- loop invariants -------------------------------------------------------------------------------------
  for (int i = tid; i < num * D; i += NTH) {  // the numerical fields' vectors v_f (their tables have one row)
    const int f = i / D;
    vnum[i] = p.fields[f].emb2[i - f * D];
  }
  if (tid == 0) zero[0] = 0.f;
  for (int c = tid; c < C; c += NTH) {
    base2[c] = p.fields[num + c].emb2;
    base1[c] = p.fields[num + c].emb1;
  }
  // this thread's rows of the row-index stage: r = tid + k * NTH -> categorical field c = r / 16, sample r % 16
  int64_t rn[RA];
#pragma unroll
  for (int k = 0; k < RA; ++k) {
    const int c = (tid + k * NTH) >> 4;
    rn[k] = c < C ? p.fields[num + c].n : 0;
  }
  // the sums: sample b = 4 wave + lane / 16, lane q takes fields q, q + 16, q + 32, q + 48 (fwd_kernel's order)
  const int sb = wave * 4 + (lane >> 4);
  const int q = lane & 15;
  float lwv[4], num1[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int f = min(16 * k + q, F - 1);
    lwv[k] = (flags & kFoLw) ? p.lw[f] : 1.f;
    num1[k] = f < num ? p.fields[f].emb1[0] : 0.f;  // the numerical fields' first-order weight (one row)
  }
  const float bias = p.bias[0];
  // U' fragments (the FwFM's A operands, the same for every tile): uf[m][s] = U'[16m + lane % 16][4s + lane / 16]
  float uf[MTC][S];
#pragma unroll
  for (int m = 0; m < MTC; ++m)
#pragma unroll
    for (int s = 0; s < S; ++s) uf[m][s] = s >= 4 * m ? p.upack[(m * S + s) * 64 + lane] : 0.f;

  // ---- DMA: every instruction with all 64 lanes (lanes without a source of their own read a valid dummy) ------
  const int nrow_i = L.ncat / 64, nfo_i = L.nfo / 64;       // row and first-order pieces per tile
  const int nkey_i = L.nkey / 64, nxv_i = L.nxv / 64;       // key and Xv pieces per tile (wave 3)
  // this wave's row + first-order pieces per tile (pieces j = wave, wave + 4, ... of the rows, then of the firsts)
  const int nmine_rows = (nrow_i + NW - 1 - wave) / NW + (nfo_i + NW - 1 - wave) / NW;
  // the key / Xv pieces' (sample, word) per lane, once: sample << 16 | dword of the sample's row
  int kbw[KP], xbw[XP];
#pragma unroll
  for (int j = 0; j < KP; ++j) {
    const int i = j * 64 + lane, b = i / (2 * C);
    kbw[j] = (b << 16) | (i - b * 2 * C);
  }
#pragma unroll
  for (int j = 0; j < XP; ++j) {
    const int i = j * 64 + lane, b = num ? i / num : 0;
    xbw[j] = (b << 16) | (i - b * num);
  }
  // Xi keys of tile t (16 x C int64, 2 dwords each) -> key slot; Xv of tile t -> Xv slot (wave 3).  Samples past the
  // batch (and lanes past a piece's end) read sample 0's words
  auto issue_keys = [&](const DmaTile& t, float* kb) {
    const uint32_t* x0 = reinterpret_cast<const uint32_t*>(t.xi + t.b0 * p.xi_stride);
    const int64_t st = 2 * p.xi_stride;
#pragma unroll
    for (int j = 0; j < KP; ++j) {
      if (j >= nkey_i) break;
      const int b = kbw[j] >> 16;
      glds_dword(x0 + (b < t.nrows ? b : 0) * st + (kbw[j] & 0xffff), kb + j * 64);
    }
  };
  auto issue_xv = [&](const DmaTile& t, float* xb) {
    const float* x0 = t.xv + t.b0 * p.xv_stride;
#pragma unroll
    for (int j = 0; j < XP; ++j) {
      if (j >= nxv_i) break;
      const int b = xbw[j] >> 16;
      glds_dword(x0 + (b < t.nrows ? (b * p.xv_stride + (xbw[j] & 0xffff)) : 0), xb + j * 64);
    }
  };
  // the rows of the tile whose indices are in ridx: D dwords per row into its row tile, one dword of first order per
  // row (row r = c * 16 + b); four pieces at a time, every LDS read of a group before its DMAs
  auto issue_rows = [&](float* eb, float* fb) {
    const int nr = kBM * C;
    for (int j = wave; j < nrow_i; j += 4 * NW) {
      const float* src[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int i = (j + u * NW) * 64 + lane;
        int r = i / D;
        int e = i - r * D;
        if (r >= nr) r = e = 0;
        src[u] = base2[r >> 4] + (int64_t)ridx[r] * D + e;
      }
#pragma unroll
      for (int u = 0; u < 4; ++u)
        if (j + u * NW < nrow_i) glds_dword(src[u], eb + (j + u * NW) * 64);
    }
    for (int jf = wave; jf < nfo_i; jf += NW) {
      int i = jf * 64 + lane;
      if (i >= nr) i = 0;
      glds_dword(base1[i >> 4] + ridx[i], fb + jf * 64);
    }
  };
  // keys (landed in kb) -> validated row indices, range-checked like nn.Embedding (out of range: row 0 and the
  // sticky flag); samples past the batch read row 0
  auto row_indices = [&](const DmaTile& t, const float* kb) {
    const int64_t* keys = reinterpret_cast<const int64_t*>(kb);
#pragma unroll
    for (int k = 0; k < RA; ++k) {
      const int r = tid + k * NTH;
      if (r < kBM * C) {
        const int c = r >> 4, b = r & 15;
        int64_t idx = 0;
        if (b < t.nrows) {
          idx = keys[b * C + c];
          if (idx < 0 || idx >= rn[k]) {
            atomicOr(p.err, DFWFM_FLAG_INDEX_OUT_OF_RANGE);
            idx = 0;
          }
        }
        ridx[r] = (int32_t)idx;
      }
    }
  };
  // the numerical fields of the tile: E[l][b][d] = v_l[d] * Xv[b][l] (combine mode 0: a * scale); thread (l, b)
  auto numerical = [&](const float* xc) {
    for (int i = tid; i < num * kBM; i += NTH) {
      const int l = i >> 4, b = i & 15;
      const float x = xc[b * num + l];
      float e[D];
#pragma unroll
      for (int d = 0; d < D; ++d) e[d] = vnum[l * D + d] * x;
      store_row<D>(nume + i * D, e);
    }
  };
  // first + second and the logit of a tile whose FwFM column sums are in part2
  auto sums = [&](const DmaTile& t, const float* fc, const float* xc) -> int {
    float first = 0.f, second = 0.f;
    float x[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int f = min(16 * k + q, F - 1);
      x[k] = f < num ? num1[k] * xc[sb * num + f] : fc[(f - num) * kBM + sb];
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) first = 16 * k + q < F ? fmaf(x[k], lwv[k], first) : first;
    for (int d = q; d < D; d += 16) second += part2[sb * D + d];
    first = sum16(first);
    second = sum16(second);
    if (q == 0 && sb < t.nrows) t.out[t.b0 + sb] = (first + second) + bias;
    return 4 * wave < t.nrows;  // a store went out
  };
  const bool rows_on = !(flags & kDmaDiagNoRows);

  // ---- prologue: tiles 0 and 1's rows in flight, tile 2's keys landing --------------------------------------
  TileCursor cc, c2, c4;  // tiles it, it + 2, it + 4
  cc.init(p, w0);
  c2 = cc;
  c2.step(p, G);  // tile 1 for now
  c4 = c2;
  c4.step(p, G);  // tile 2 for now
  {
    const DmaTile t0 = cc.tile(p);
    DmaTile t1;
    if (nmine > 1) t1 = c2.tile(p);
    if (wave == NW - 1) {  // keys of tiles 0, 1, 2
      issue_keys(t0, keybuf);
      if (nmine > 1) issue_keys(t1, keybuf + L.nkey);
      if (nmine > 2) issue_keys(c4.tile(p), keybuf + 2 * L.nkey);
    }
    wait_vm(0);
    lds_barrier();
    row_indices(t0, keybuf);
    lds_barrier();
    if (rows_on) issue_rows(catbuf, fobuf);
    if (wave == NW - 1) issue_xv(t0, xvbuf);
    c4.step(p, G);  // tile 3
    if (nmine > 1) {
      lds_barrier();  // tile 0's row indices read
      row_indices(t1, keybuf + L.nkey);
      lds_barrier();
      if (wave == NW - 1 && nmine > 3) issue_keys(c4.tile(p), keybuf);  // tile 3's (tile 0's slot)
      if (rows_on) issue_rows(catbuf + L.ncat, fobuf + L.nfo);
      if (wave == NW - 1) issue_xv(t1, xvbuf + L.nxv);
    }
    c2.step(p, G);  // tile 2
    c4.step(p, G);  // tile 4
    // tile 0's rows and Xv landed (tile 3's keys and tile 1's rows and Xv may fly on)
    wait_vm((nmine > 1 && rows_on ? nmine_rows : 0) + (nmine > 1 && wave == NW - 1 ? nxv_i : 0) +
            (nmine > 3 && wave == NW - 1 ? nkey_i : 0));
    lds_barrier();
  }

  // Per iteration (tile it; on entry its rows / first order / Xv and tile it + 2's keys have landed, all waves):
  //   [B] keys of tile it + 4; tile it's numerical fields; tile it + 2's row indices; tile it - 1's sums
  //   [C] tile it + 2's rows / first order / Xv go out; tile it's FwFM; then wait for tile it + 1's DMA and tile
  //       it + 3's keys (both issued an iteration ago)
  DmaTile tprev = cc.tile(p);
  int stored = 0;  // a logit store is the most recent vm op of this wave
  for (int it = 0; it < nmine; ++it) {
    const int cur = it % kDmaBufs;
    const float* const ec = catbuf + cur * L.ncat;
    const DmaTile tc = cc.tile(p);
    // [B]
    const bool keys4 = wave == NW - 1 && it + 4 < nmine;
    if (keys4) issue_keys(c4.tile(p), keybuf + ((it + 4) % kDmaBufs) * L.nkey);
    numerical(xvbuf + cur * L.nxv);
    const bool ahead = it + kDmaDepth < nmine;
    DmaTile ta;
    if (ahead) {
      ta = c2.tile(p);
      row_indices(ta, keybuf + ((it + 2) % kDmaBufs) * L.nkey);
    }
    stored = 0;
    if (it > 0) {
      const int pv = (it - 1) % kDmaBufs;
      stored = sums(tprev, fobuf + pv * L.nfo, xvbuf + pv * L.nxv);
    }
    lds_barrier();
    // [C] the DMA of the tile kDmaDepth ahead, then this tile's FwFM (fwd_kernel PART 3, kP3Pieces): Y = U'E, column
    // n = b * D + d of wave nt % 4's column tiles, partial = sum_k E[k][n] Y[k][n]
    if (ahead) {
      const int nb = (it + kDmaDepth) % kDmaBufs;
      if (rows_on) issue_rows(catbuf + nb * L.ncat, fobuf + nb * L.nfo);
      if (wave == NW - 1) issue_xv(ta, xvbuf + nb * L.nxv);
    }
    for (int nt = wave; nt < D && !(flags & kDmaDiagNoFwfm); nt += NW) {
      const int n = nt * 16 + (lane & 15);
      // field l of column n: the numerical fields' E, the row tile's categorical fields, zero past F (one LDS
      // read from the selected address)
      auto eat = [&](int l) { return *(l < num ? nume + l * FS + n : (l < F ? ec + (l - num) * FS + n : zero)); };
      // every operand of the column tile read from LDS first (the B operands of the S steps and the E values the
      // column sum weights), then the row tiles' MFMA chains side by side
      float bv[S], ek[MTC][4];
#pragma unroll
      for (int s = 0; s < S; ++s) bv[s] = eat(4 * s + (lane >> 4));
#pragma unroll
      for (int m = 0; m < MTC; ++m)
#pragma unroll
        for (int r = 0; r < 4; ++r) ek[m][r] = eat(16 * m + 4 * (lane >> 4) + r);
      __builtin_amdgcn_sched_barrier(0);
      f32x4 acc[MTC];
#pragma unroll
      for (int m = 0; m < MTC; ++m) acc[m] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int s = 0; s < S; ++s)
#pragma unroll
        for (int m = 0; m < MTC; ++m)
          if (4 * m <= s) acc[m] = __builtin_amdgcn_mfma_f32_16x16x4f32(uf[m][s], bv[s], acc[m], 0, 0, 0);
      float colv = 0.f;
#pragma unroll
      for (int m = 0; m < MTC; ++m)
#pragma unroll
        for (int r = 0; r < 4; ++r) colv = fmaf(ek[m][r], acc[m][r], colv);
      colv += __shfl_xor(colv, 16);
      colv += __shfl_xor(colv, 32);
      if (lane < 16) part2[n] = colv;
    }
    // tile it + 1's rows / first order / Xv and tile it + 3's keys (issued last iteration) have landed; this
    // iteration's DMA (keys, rows, Xv) and the previous tile's logit store may fly on
    {
      const int infl = (keys4 ? nkey_i : 0) + stored + (ahead && rows_on ? nmine_rows : 0) +
                       (ahead && wave == NW - 1 ? nxv_i : 0);
      wait_vm(infl);
    }
    lds_barrier();
    tprev = tc;
    cc.step(p, G);
    c2.step(p, G);
    c4.step(p, G);
  }
  // the last tile's sums
  {
    const int pv = (nmine - 1) % kDmaBufs;
    sums(tprev, fobuf + pv * L.nfo, xvbuf + pv * L.nxv);
  }
}

template <int D, int MTC>
static auto pick_dma(int S) {
  const int sl = S - 4 * (MTC - 1);
  return sl == 1 ? fwfm_dma_kernel<D, MTC, 1> : sl == 2 ? fwfm_dma_kernel<D, MTC, 2>
       : sl == 3 ? fwfm_dma_kernel<D, MTC, 3> : fwfm_dma_kernel<D, MTC, 4>;
}

template <int D>
static hipError_t launch_dma_d(const FwdArgs& a, int ntiles, int grid, size_t lds, hipStream_t s) {
  auto k = a.MT == 1 ? pick_dma<D, 1>(a.S) : a.MT == 2 ? pick_dma<D, 2>(a.S) : pick_dma<D, 3>(a.S);
  hipError_t e = ensure_lds_limit(reinterpret_cast<const void*>(k), lds);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(k, dim3(grid), dim3(256), lds, s, a, ntiles);
  return hipGetLastError();
}

size_t fwfm_dma_lds_bytes(int F, int num, int D) { return sizeof(float) * (size_t)dma_layout(F, num, D).total; }

bool fwfm_dma_supported(const FwdArgs& a, int D) {
  const int need = kHasSecond | kNeedE | kFoTables | kP3Pieces;
  if ((a.flags & need) != need || (a.flags & (kHasDeep | kTrain | kHasQR | kPairs | kFoFwlw))) return false;
  if (a.MT < 1 || a.MT > 3 || a.F - a.num < 1 || a.F - a.num > 48) return false;
  if (!(D == 4 || D == 8 || D == 10 || D == 16)) return false;
  return fwfm_dma_lds_bytes(a.F, a.num, D) <= 80 * 1024;  // two workgroups per CU
}

// the persistent launch: two workgroups per CU (by LDS), each walking tiles w, w + G, ...
hipError_t launch_fwfm_dma(const FwdArgs& a, int D, hipStream_t s) {
  static int cus = 0;
  if (cus == 0) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) !=
                                                hipSuccess || cus <= 0)
      cus = 256;
  }
  const int tiles = (int)((a.batch + kBM - 1) / kBM);
  const int ntiles = a.nb > 1 ? a.nb * tiles : tiles;
  const int grid = ntiles < 2 * cus ? ntiles : 2 * cus;
  const size_t lds = fwfm_dma_lds_bytes(a.F, a.num, D);
  switch (D) {
    case 4: return launch_dma_d<4>(a, ntiles, grid, lds, s);
    case 8: return launch_dma_d<8>(a, ntiles, grid, lds, s);
    case 10: return launch_dma_d<10>(a, ntiles, grid, lds, s);
    case 16: return launch_dma_d<16>(a, ntiles, grid, lds, s);
    default: return hipErrorInvalidValue;
  }
}

}  // namespace dfwfm
