// ubench_gather.hip -- what does the FwFM-only forward's gather cost by itself?
// Criteo-39's categorical part: B = 4096 samples x 26 int64 indices into 26 tables of 10-float rows
// (53 MB in all, the real field sizes), uniform random indices.  Each 16-sample tile: load the tile's
// indices, gather its 416 rows into an LDS tile, barrier, one float per sample out (so nothing is dead).
// Variants of the row loads (per wave instruction):
//   0  one lane per row, 5 dwordx2 per row (fwd_kernel PART 3 today: 64 rows per instruction)
//   1  five lanes per row, one dwordx2 each (12 rows per instruction, 60 lanes busy)
//   2  ten lanes per row, one dword each (6 rows per instruction)
//   3  one lane per row, two 16-B aligned dwordx4 + one dwordx2 placed by the row's alignment (3 loads per row)
//   4  one lane per row of a PACKED copy: rows at a 16-float (64-B) stride, 64-B aligned -- every row one line,
//      two dwordx4 + one dwordx2
//   5  variant 0 plus the row's first-order weight from its own [n][1] table (one dword per row: the MLP-free
//      forward's real pattern with lw first order, fm_1st_embeddings)
//   6  one lane per row of a packed copy holding second AND first order: 12-float (48-B) rows, 16-B aligned,
//      three dwordx4 (the first-order weight at float 10)
//   7  the same at a 16-float (64-B) stride: every row one line
// argv: [NB batches in flight] [table scale K: every table K x as many rows, e.g. 8 -> 424 MB, HBM-resident]
// TILES: 16-sample tiles per workgroup (walked with the next tile's loads issued before this tile's
// LDS stores: TILES > 1 is the persistent form).  Reports microseconds per 4096-sample batch with
// NB batches in flight (one launch over NB batches, as NB streams would).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include <vector>

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

constexpr int F = 26, D = 10, BM = 16, NTH = 512;

struct Args {
  const float* const* tabs;  // [F] table bases
  const float* const* ptabs; // [F] packed (16-float stride) table bases
  const float* const* ftabs; // [F] first-order tables [n][1]
  const float* const* q12;   // [F] packed second + first order, 12-float stride
  const float* const* q16;   // [F] packed second + first order, 16-float stride
  const int64_t* xi;         // [NB*B][F]
  float* out;                // [NB*B]
  int64_t total;             // samples
};

template <int V>
__device__ __forceinline__ void tile_loads(const Args& a, int64_t b0, int tid, float2 (&v2)[8], float (&v1)[16]) {
  if constexpr (V == 0) {
    const int r = tid;  // row r: field r / 16, sample r % 16
    if (r < F * BM) {
      const int f = r >> 4;
      const int64_t idx = a.xi[(b0 + (r & 15)) * F + f];
      const float2* src = reinterpret_cast<const float2*>(a.tabs[f] + idx * D);
#pragma unroll
      for (int j = 0; j < 5; ++j) v2[j] = src[j];
    }
  } else if constexpr (V == 3) {  // one lane per row: two aligned dwordx4 + one dwordx2 (fwd_kernel's load_row_x4)
    const int r = tid;
    if (r < F * BM) {
      const int f = r >> 4;
      const int64_t idx = a.xi[(b0 + (r & 15)) * F + f];
      const float* src = a.tabs[f] + idx * D;
      const bool al = (reinterpret_cast<uintptr_t>(src) & 15) == 0;
      const float* q = al ? src : src + 2;
      const float* t = al ? src + 8 : src;
      const float4 x0 = reinterpret_cast<const float4*>(q)[0], x1 = reinterpret_cast<const float4*>(q)[1];
      const float2 c = *reinterpret_cast<const float2*>(t);
      v1[0] = al ? x0.x : c.x; v1[1] = al ? x0.y : c.y; v1[2] = al ? x0.z : x0.x; v1[3] = al ? x0.w : x0.y;
      v1[4] = al ? x1.x : x0.z; v1[5] = al ? x1.y : x0.w; v1[6] = al ? x1.z : x1.x; v1[7] = al ? x1.w : x1.y;
      v1[8] = al ? c.x : x1.z; v1[9] = al ? c.y : x1.w;
    }
  } else if constexpr (V == 4) {
    const int r = tid;
    if (r < F * BM) {
      const int f = r >> 4;
      const int64_t idx = a.xi[(b0 + (r & 15)) * F + f];
      const float* src = a.ptabs[f] + idx * 16;
      const float4 x0 = reinterpret_cast<const float4*>(src)[0], x1 = reinterpret_cast<const float4*>(src)[1];
      const float2 c = reinterpret_cast<const float2*>(src)[4];
      v1[0] = x0.x; v1[1] = x0.y; v1[2] = x0.z; v1[3] = x0.w;
      v1[4] = x1.x; v1[5] = x1.y; v1[6] = x1.z; v1[7] = x1.w;
      v1[8] = c.x; v1[9] = c.y;
    }
  } else if constexpr (V == 5) {
    const int r = tid;
    if (r < F * BM) {
      const int f = r >> 4;
      const int64_t idx = a.xi[(b0 + (r & 15)) * F + f];
      const float2* src = reinterpret_cast<const float2*>(a.tabs[f] + idx * D);
#pragma unroll
      for (int j = 0; j < 5; ++j) v2[j] = src[j];
      v1[10] = a.ftabs[f][idx];
    }
  } else if constexpr (V == 6 || V == 7) {
    const int r = tid;
    if (r < F * BM) {
      const int f = r >> 4;
      const int64_t idx = a.xi[(b0 + (r & 15)) * F + f];
      const float4* src = reinterpret_cast<const float4*>((V == 6 ? a.q12[f] + idx * 12 : a.q16[f] + idx * 16));
      const float4 x0 = src[0], x1 = src[1], x2 = src[2];
      v1[0] = x0.x; v1[1] = x0.y; v1[2] = x0.z; v1[3] = x0.w;
      v1[4] = x1.x; v1[5] = x1.y; v1[6] = x1.z; v1[7] = x1.w;
      v1[8] = x2.x; v1[9] = x2.y; v1[10] = x2.z;
    }
  } else if constexpr (V == 1) {
    const int w = tid >> 6, lane = tid & 63;
    const int rw = lane / 5, part = lane - rw * 5;  // 12 rows per wave per round
#pragma unroll
    for (int k = 0; k < 5; ++k) {  // 8 waves x 12 rows x 5 rounds = 480 >= 416
      const int r = (k * 8 + w) * 12 + rw;
      if (rw < 12 && r < F * BM) {
        const int f = r >> 4;
        const int64_t idx = a.xi[(b0 + (r & 15)) * F + f];
        v2[k] = reinterpret_cast<const float2*>(a.tabs[f] + idx * D)[part];
      }
    }
  } else {
    const int w = tid >> 6, lane = tid & 63;
    const int rw = lane / 10, part = lane - rw * 10;  // 6 rows per wave per round
#pragma unroll
    for (int k = 0; k < 9; ++k) {  // 8 x 6 x 9 = 432 >= 416
      const int r = (k * 8 + w) * 6 + rw;
      if (rw < 6 && r < F * BM) {
        const int f = r >> 4;
        const int64_t idx = a.xi[(b0 + (r & 15)) * F + f];
        v1[k] = (a.tabs[f] + idx * D)[part];
      }
    }
  }
}

template <int V>
__device__ __forceinline__ void tile_stores(float* E, int tid, const float2 (&v2)[8], const float (&v1)[16]) {
  if constexpr (V == 0 || V == 5) {
    const int r = tid;
    if (r < F * BM) {
      float2* dst = reinterpret_cast<float2*>(E + (r & 15) * (F * D + 2) + (r >> 4) * D);
#pragma unroll
      for (int j = 0; j < 5; ++j) dst[j] = v2[j];
      if constexpr (V == 5) E[BM * (F * D + 2) + r] = v1[10];
    }
  } else if constexpr (V == 3 || V == 4 || V == 6 || V == 7) {
    const int r = tid;
    if (r < F * BM) {
      float2* dst = reinterpret_cast<float2*>(E + (r & 15) * (F * D + 2) + (r >> 4) * D);
#pragma unroll
      for (int j = 0; j < 5; ++j) dst[j] = make_float2(v1[2 * j], v1[2 * j + 1]);
      if constexpr (V >= 6) E[BM * (F * D + 2) + r] = v1[10];
    }
  } else if constexpr (V == 1) {
    const int w = tid >> 6, lane = tid & 63;
    const int rw = lane / 5, part = lane - rw * 5;
#pragma unroll
    for (int k = 0; k < 5; ++k) {
      const int r = (k * 8 + w) * 12 + rw;
      if (rw < 12 && r < F * BM) reinterpret_cast<float2*>(E + (r & 15) * (F * D + 2) + (r >> 4) * D)[part] = v2[k];
    }
  } else {
    const int w = tid >> 6, lane = tid & 63;
    const int rw = lane / 10, part = lane - rw * 10;
#pragma unroll
    for (int k = 0; k < 9; ++k) {
      const int r = (k * 8 + w) * 6 + rw;
      if (rw < 6 && r < F * BM) (E + (r & 15) * (F * D + 2) + (r >> 4) * D)[part] = v1[k];
    }
  }
}

template <int V, int TILES>
__global__ void __launch_bounds__(NTH) gather_kernel(Args a) {
  __shared__ float E[BM * (F * D + 2) + F * BM];  // rows, then first order [F][BM]
  const int tid = threadIdx.x;
  float2 v2[8];
  float v1[16];
  for (int t = 0; t < TILES; ++t) {
    const int64_t b0 = ((int64_t)blockIdx.x * TILES + t) * BM;
    if (b0 >= a.total) break;
    tile_loads<V>(a, b0, tid, v2, v1);
    __syncthreads();  // the previous tile's sums are done with E
    tile_stores<V>(E, tid, v2, v1);
    __syncthreads();
    if (tid < 64 * 4) {  // 16 lanes per sample
      const int b = tid >> 4, q = tid & 15;
      float s = 0.f;
      for (int c = q; c < F * D; c += 16) s += E[b * (F * D + 2) + c];
      if (V >= 5) for (int f = q; f < F; f += 16) s += E[BM * (F * D + 2) + f * BM + b];
#pragma unroll
      for (int o = 8; o >= 1; o >>= 1) s += __shfl_xor(s, o);
      if (q == 0) a.out[b0 + b] = s;
    }
  }
}

// synth.CRITEO_FEATURE_SIZES (the 26 categorical fields bench.py's model uses: 1.33 M rows, 53 MB)
static const int64_t kSizes[F] = {1458, 556, 245197, 166166, 306, 20, 12055, 634, 4, 46330, 5229, 243454, 3177,
                                  27, 11745, 225322, 11, 4727, 2058, 5, 238640, 18, 16, 67856, 89, 50942};

int main(int argc, char** argv) {
  const int B = 4096;
  const int NB = argc > 1 ? atoi(argv[1]) : 3;
  const int K = argc > 2 ? atoi(argv[2]) : 1;
  const int reps = 200;
  std::vector<int64_t> n(kSizes, kSizes + F);
  for (auto& x : n) x *= K;
  int64_t rows = 0;
  for (int f = 0; f < F; ++f) rows += n[f];
  float* tab;
  CHECK(hipMalloc(&tab, rows * D * 4));
  CHECK(hipMemset(tab, 0, rows * D * 4));
  std::vector<const float*> hb(F);
  int64_t off = 0;
  for (int f = 0; f < F; ++f) { hb[f] = tab + off * D; off += n[f]; }
  const float** dtabs;
  CHECK(hipMalloc(&dtabs, F * sizeof(float*)));
  CHECK(hipMemcpy(dtabs, hb.data(), F * sizeof(float*), hipMemcpyHostToDevice));
  float* ptab;
  CHECK(hipMalloc(&ptab, rows * 16 * 4));
  CHECK(hipMemset(ptab, 0, rows * 16 * 4));
  std::vector<const float*> hp(F);
  off = 0;
  for (int f = 0; f < F; ++f) { hp[f] = ptab + off * 16; off += n[f]; }
  const float** dptabs;
  CHECK(hipMalloc(&dptabs, F * sizeof(float*)));
  CHECK(hipMemcpy(dptabs, hp.data(), F * sizeof(float*), hipMemcpyHostToDevice));
  // first-order tables and the packed second + first order copies
  auto table_set = [&](int stride) {
    float* t;
    CHECK(hipMalloc(&t, rows * stride * 4));
    CHECK(hipMemset(t, 0, rows * stride * 4));
    std::vector<const float*> h(F);
    int64_t o = 0;
    for (int f = 0; f < F; ++f) { h[f] = t + o * stride; o += n[f]; }
    const float** d;
    CHECK(hipMalloc(&d, F * sizeof(float*)));
    CHECK(hipMemcpy(d, h.data(), F * sizeof(float*), hipMemcpyHostToDevice));
    return d;
  };
  const float** dftabs = table_set(1);
  const float** dq12 = table_set(12);
  const float** dq16 = table_set(16);
  printf("tables x%d: %.0f MB of 40-B rows, %.0f MB packed\n", K, rows * D * 4 / 1e6, rows * 64 / 1e6);
  const int64_t total = (int64_t)NB * B;
  std::vector<int64_t> hx(total * F);
  uint64_t s = 88172645463325252ull;
  for (int64_t i = 0; i < total; ++i)
    for (int f = 0; f < F; ++f) { s ^= s << 13; s ^= s >> 7; s ^= s << 17; hx[i * F + f] = (int64_t)(s % (uint64_t)n[f]); }
  int64_t* dx;
  float* dout;
  CHECK(hipMalloc(&dx, hx.size() * 8));
  CHECK(hipMemcpy(dx, hx.data(), hx.size() * 8, hipMemcpyHostToDevice));
  CHECK(hipMalloc(&dout, total * 4));
  Args a{dtabs, dptabs, dftabs, dq12, dq16, dx, dout, total};
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  auto run = [&](auto kern, int tiles, const char* name) {
    const int grid = (int)((total / BM + tiles - 1) / tiles);
    for (int i = 0; i < 50; ++i) kern<<<grid, NTH>>>(a);
    CHECK(hipEventRecord(e0));
    for (int i = 0; i < reps; ++i) kern<<<grid, NTH>>>(a);
    CHECK(hipEventRecord(e1));
    CHECK(hipEventSynchronize(e1));
    float ms;
    CHECK(hipEventElapsedTime(&ms, e0, e1));
    const double us_batch = ms * 1e3 / reps / NB;
    const double alg = (double)B * (F * 8 + F * D * 4);  // indices + rows
    printf("%-28s NB=%d tiles/wg=%d grid=%6d: %.3f us per 4096-sample batch, %.2f TB/s of index+row bytes\n", name, NB,
           tiles, grid, us_batch, alg / (us_batch * 1e-6) / 1e12);
  };
  run(gather_kernel<0, 1>, 1, "lane per row (5 x dwordx2)");
  run(gather_kernel<5, 1>, 1, "+ first order, own tables");
  run(gather_kernel<6, 1>, 1, "2nd+1st packed 48-B (3 x4)");
  run(gather_kernel<7, 1>, 1, "2nd+1st packed 64-B (3 x4)");
  if (argc > 3) return 0;
  run(gather_kernel<4, 1>, 1, "packed 64-B rows (2 x4 + x2)");
  run(gather_kernel<3, 1>, 1, "lane per row (2 x4 + 1 x2)");
  run(gather_kernel<1, 1>, 1, "5 lanes per row (dwordx2)");
  run(gather_kernel<2, 1>, 1, "10 lanes per row (dword)");
  run(gather_kernel<0, 4>, 4, "lane per row, 4 tiles/wg");
  run(gather_kernel<1, 4>, 4, "5 lanes per row, 4 tiles/wg");
  return 0;
}
