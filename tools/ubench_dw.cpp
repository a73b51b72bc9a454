// Weight-gradient GEMM alone: dW_l += G_l^T X_{l-1}, db_l += sum G_l for the Criteo-39 3 x 400 MLP at B = 4096,
// through libdfwfm.so's own launcher (dfwfm::launch_dw), staged (LDS, 64 x 64) vs register-direct (80 x 80), by
// batch splits.  Reports us per launch, TFLOP/s and the largest difference between the two kernels' gradients.
//   hipcc --offload-arch=gfx950 -O2 -std=c++17 -I xsdeepfwfm_deprecated_amd/csrc -I include tools/ubench_dw.cpp \
//     -L xsdeepfwfm_deprecated_amd -ldfwfm -Wl,-rpath,'$ORIGIN/../xsdeepfwfm_deprecated_amd' -o tools/ubench_dw
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <vector>

#include "dfwfm_internal.h"

#define CHECK(x)                                                                   \
  do {                                                                             \
    hipError_t e_ = (x);                                                           \
    if (e_ != hipSuccess) {                                                        \
      printf("HIP %s @%d\n", hipGetErrorString(e_), __LINE__);                     \
      exit(1);                                                                     \
    }                                                                              \
  } while (0)

using namespace dfwfm;

static int setup(DwArgs& d, bool staged, int splits_req, int64_t batch, int H, int N, int K0,
                 float* const* G, float* const* X, float* const* gW, float* const* gB) {
  memset(&d, 0, sizeof d);
  const int edge = dw_block_edge(staged), quantum = dw_row_quantum(staged);
  d.H = H;
  d.N = N;
  d.nnb = (N + edge - 1) / edge;
  d.batch = batch;
  int per_split = 0;
  for (int l = 1; l <= H; ++l) {
    d.G[l] = G[l];
    d.X[l] = X[l];
    d.gW[l] = gW[l];
    d.gB[l] = gB[l];
    d.K[l] = l == 1 ? K0 : N;
    d.ldx[l] = l == 1 ? (K0 + 3) / 4 * 4 : N;
    d.nkb[l] = (d.K[l] + edge - 1) / edge;
    per_split += d.nnb * d.nkb[l];
  }
  int64_t splits = splits_req > 0 ? splits_req : (staged ? 768 : 512) / per_split;
  if (splits < 1) splits = 1;
  int64_t rows = (batch + splits - 1) / splits;
  rows = (rows + quantum - 1) / quantum * quantum;
  splits = (batch + rows - 1) / rows;
  d.splits = (int32_t)splits;
  d.rows_per_split = rows;
  d.blk0[1] = 0;
  for (int l = 1; l <= H; ++l) d.blk0[l + 1] = d.blk0[l] + d.nnb * d.nkb[l] * (int32_t)splits;
  return d.blk0[H + 1];
}

int main(int argc, char** argv) {
  const int64_t B = argc > 1 ? atoll(argv[1]) : 4096;
  const int iters = argc > 2 ? atoi(argv[2]) : 200;
  const int H = 3, N = 400, K0 = 390;
  const int ld0 = (K0 + 3) / 4 * 4;
  float *G[4] = {}, *X[4] = {}, *gW[2][4] = {}, *gB[2][4] = {};
  std::vector<float> h;
  unsigned s = 12345;
  auto rnd = [&]() { s = s * 1664525u + 1013904223u; return ((s >> 8) & 0xFFFF) / 65536.f - 0.5f; };
  for (int l = 1; l <= H; ++l) {
    const int K = l == 1 ? K0 : N, ldx = l == 1 ? ld0 : N;
    h.resize((size_t)B * N);
    for (auto& v : h) v = rnd();
    CHECK(hipMalloc(&G[l], h.size() * 4));
    CHECK(hipMemcpy(G[l], h.data(), h.size() * 4, hipMemcpyHostToDevice));
    h.resize((size_t)B * ldx);
    for (auto& v : h) v = rnd();
    CHECK(hipMalloc(&X[l], h.size() * 4));
    CHECK(hipMemcpy(X[l], h.data(), h.size() * 4, hipMemcpyHostToDevice));
    for (int k = 0; k < 2; ++k) {
      CHECK(hipMalloc(&gW[k][l], (size_t)N * K * 4));
      CHECK(hipMalloc(&gB[k][l], (size_t)N * 4));
    }
  }
  const double flops = 2.0 * B * ((double)N * K0 + 2.0 * N * N);
  hipStream_t st;
  CHECK(hipStreamCreate(&st));
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  // correctness: both kernels once from zero, compare
  for (int k = 0; k < 2; ++k) {
    for (int l = 1; l <= H; ++l) {
      const int K = l == 1 ? K0 : N;
      CHECK(hipMemset(gW[k][l], 0, (size_t)N * K * 4));
      CHECK(hipMemset(gB[k][l], 0, (size_t)N * 4));
    }
    DwArgs d;
    const int nb = setup(d, k == 1, 0, B, H, N, K0, G, X, gW[k], gB[k]);
    CHECK(launch_dw(d, nb, k == 1, st));
  }
  CHECK(hipStreamSynchronize(st));
  double maxd = 0, maxa = 0;
  for (int l = 1; l <= H; ++l) {
    const int K = l == 1 ? K0 : N;
    std::vector<float> a((size_t)N * K), b((size_t)N * K), ab(N), bb(N);
    CHECK(hipMemcpy(a.data(), gW[0][l], a.size() * 4, hipMemcpyDeviceToHost));
    CHECK(hipMemcpy(b.data(), gW[1][l], b.size() * 4, hipMemcpyDeviceToHost));
    CHECK(hipMemcpy(ab.data(), gB[0][l], N * 4, hipMemcpyDeviceToHost));
    CHECK(hipMemcpy(bb.data(), gB[1][l], N * 4, hipMemcpyDeviceToHost));
    for (size_t i = 0; i < a.size(); ++i) {
      maxd = fmax(maxd, fabs((double)a[i] - b[i]));
      maxa = fmax(maxa, fabs((double)b[i]));
    }
    for (int i = 0; i < N; ++i) maxd = fmax(maxd, fabs((double)ab[i] - bb[i]));
  }
  printf("check: max |dwr - staged| = %.3e (max |dW| %.3e)\n", maxd, maxa);
  const int split_list[] = {0, 2, 3, 4, 5, 6, 7, 8};
  const int pf_list[] = {4, 6, 48, 0};  // dwr prefetch depths (48: four, eight waves), then the staged kernel
  for (int pf : pf_list) {
    const int k = pf == 0 ? 1 : 0;
    for (int sp : split_list) {
      DwArgs d;
      const int nb = setup(d, k == 1, sp, B, H, N, K0, G, X, gW[k], gB[k]);
      d.pf = pf == 48 ? 4 : pf;
      d.nw = pf == 48 ? 8 : 4;
      for (int i = 0; i < 10; ++i) CHECK(launch_dw(d, nb, k == 1, st));
      CHECK(hipEventRecord(e0, st));
      for (int i = 0; i < iters; ++i) CHECK(launch_dw(d, nb, k == 1, st));
      CHECK(hipEventRecord(e1, st));
      CHECK(hipEventSynchronize(e1));
      float ms = 0;
      CHECK(hipEventElapsedTime(&ms, e0, e1));
      const double us = 1e3 * ms / iters;
      printf("%s pf %d splits %2d (req %2d) workgroups %4d: %7.2f us  %6.1f TFLOP/s\n", k ? "staged" : "dwr   ", pf,
             d.splits, sp, nb, us, flops / us * 1e-6);
    }
  }
  return 0;
}
