// Weight-gradient GEMM alone: dW_l += G_l^T X_{l-1}, db_l += sum G_l for the Criteo-39 3 x 400 MLP at B = 4096,
// through libdfwfm.so's own launcher (dfwfm::launch_dw, the register-direct 80 x 80 dwr_kernel), by batch splits.
// Reports us per launch, TFLOP/s, and the largest difference of one launch's gradients from a float64 host GEMM.
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

static int setup(DwArgs& d, int splits_req, int64_t batch, int H, int N, int K0, float* const* G, float* const* X,
                 float* const* gW, float* const* gB) {
  memset(&d, 0, sizeof d);
  d.H = H;
  d.N = N;
  d.nnb = (N + kDwEdge - 1) / kDwEdge;
  d.batch = batch;
  int per_split = 0;
  for (int l = 1; l <= H; ++l) {
    d.G[l] = G[l];
    d.X[l] = X[l];
    d.gW[l] = gW[l];
    d.gB[l] = gB[l];
    d.K[l] = l == 1 ? K0 : N;
    d.ldx[l] = l == 1 ? (K0 + 3) / 4 * 4 : N;
    d.nkb[l] = (d.K[l] + kDwEdge - 1) / kDwEdge;
    per_split += d.nnb * d.nkb[l];
  }
  int64_t splits = splits_req > 0 ? splits_req : 256 / per_split;
  if (splits < 1) splits = 1;
  int64_t rows = (batch + splits - 1) / splits;
  rows = (rows + kDwRows - 1) / kDwRows * kDwRows;
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
  float *G[4] = {}, *X[4] = {}, *gW[4] = {}, *gB[4] = {};
  std::vector<std::vector<float>> hG(4), hX(4);
  unsigned s = 12345;
  auto rnd = [&]() { s = s * 1664525u + 1013904223u; return ((s >> 8) & 0xFFFF) / 65536.f - 0.5f; };
  for (int l = 1; l <= H; ++l) {
    const int K = l == 1 ? K0 : N, ldx = l == 1 ? ld0 : N;
    hG[l].resize((size_t)B * N);
    for (auto& v : hG[l]) v = rnd();
    CHECK(hipMalloc(&G[l], hG[l].size() * 4));
    CHECK(hipMemcpy(G[l], hG[l].data(), hG[l].size() * 4, hipMemcpyHostToDevice));
    hX[l].resize((size_t)B * ldx);
    for (auto& v : hX[l]) v = rnd();
    CHECK(hipMalloc(&X[l], hX[l].size() * 4));
    CHECK(hipMemcpy(X[l], hX[l].data(), hX[l].size() * 4, hipMemcpyHostToDevice));
    CHECK(hipMalloc(&gW[l], (size_t)N * K * 4));
    CHECK(hipMalloc(&gB[l], (size_t)N * 4));
  }
  const double flops = 2.0 * B * ((double)N * K0 + 2.0 * N * N);
  hipStream_t st;
  CHECK(hipStreamCreate(&st));
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  // correctness: one launch from zero against a float64 host GEMM (a sample of rows n)
  for (int l = 1; l <= H; ++l) {
    const int K = l == 1 ? K0 : N;
    CHECK(hipMemset(gW[l], 0, (size_t)N * K * 4));
    CHECK(hipMemset(gB[l], 0, (size_t)N * 4));
  }
  {
    DwArgs d;
    const int nb = setup(d, 0, B, H, N, K0, G, X, gW, gB);
    CHECK(launch_dw(d, nb, st));
    CHECK(hipStreamSynchronize(st));
  }
  double maxrel = 0;
  for (int l = 1; l <= H; ++l) {
    const int K = l == 1 ? K0 : N, ldx = l == 1 ? ld0 : N;
    std::vector<float> w((size_t)N * K), b(N);
    CHECK(hipMemcpy(w.data(), gW[l], w.size() * 4, hipMemcpyDeviceToHost));
    CHECK(hipMemcpy(b.data(), gB[l], N * 4, hipMemcpyDeviceToHost));
    for (int n = 0; n < N; n += 37) {
      double bs = 0;
      for (int64_t r = 0; r < B; ++r) bs += hG[l][r * N + n];
      maxrel = fmax(maxrel, fabs(b[n] - bs) / (fabs(bs) + 1.0));
      for (int k = 0; k < K; ++k) {
        double acc = 0, mag = 0;
        for (int64_t r = 0; r < B; ++r) {
          acc += (double)hG[l][r * N + n] * hX[l][r * ldx + k];
          mag += fabs((double)hG[l][r * N + n] * hX[l][r * ldx + k]);
        }
        maxrel = fmax(maxrel, fabs(w[(size_t)n * K + k] - acc) / (mag + 1e-30));
      }
    }
  }
  printf("check: max |dW - float64| / sum |terms| = %.3e (sampled rows)\n", maxrel);
  const int split_list[] = {0, 2, 3, 4, 5, 6, 7, 8};
  for (int sp : split_list) {
    DwArgs d;
    const int nb = setup(d, sp, B, H, N, K0, G, X, gW, gB);
    for (int i = 0; i < 10; ++i) CHECK(launch_dw(d, nb, st));
    CHECK(hipEventRecord(e0, st));
    for (int i = 0; i < iters; ++i) CHECK(launch_dw(d, nb, st));
    CHECK(hipEventRecord(e1, st));
    CHECK(hipEventSynchronize(e1));
    float ms = 0;
    CHECK(hipEventElapsedTime(&ms, e0, e1));
    const double us = 1e3 * ms / iters;
    printf("dwr splits %2d (req %2d) workgroups %4d: %7.2f us  %6.1f TFLOP/s\n", d.splits, sp, nb, us, flops / us * 1e-6);
  }
  return 0;
}
