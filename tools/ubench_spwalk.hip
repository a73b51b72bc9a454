// ubench_spwalk.hip -- the floor of the sparse deep tower's pair walk (pruned config, BASELINE configs[3]).
// One workgroup per CU (grid 256), 64 samples per workgroup (lane = sample), x[k][64] in LDS (400 x 64 floats),
// eight waves; each wave walks PW (k, w) pairs accumulating into four running sums -- what sparse_mlp_kernel does
// per layer.  PW = 8400 per wave ~ 67 k pairs per workgroup: Criteo-39's three 400-wide layers at 90 % zero
// (40 nonzeros per row, padded to the group of four's longest row rounded to 8 -> ~48 entries per neuron).
// How a wave obtains each pair's (k, w):
//   A  computed from the loop counter (no list at all; a few VALU ops per pair): the LDS x-read + FMA floor
//   B  the list staged in LDS, read back as wave-uniform ds_read_b128 broadcasts (two pairs each) -- the kernel
//   C  the list in VGPRs, one entry per lane (one coalesced 512-B load per 64 pairs), v_readlane to SGPRs per pair
//   D  the list read with wave-uniform (scalar) loads from global memory
// Reports us per launch (= per workgroup) and per 4096-sample batch (64 workgroups; 256 in flight = 4 batches).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <vector>

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

constexpr int S = 64, NW = 8, K = 400, PW = 8400;

template <int V>
__global__ void __launch_bounds__(64 * NW) walk(const int2* __restrict__ list, float* __restrict__ out) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  float* x = lds;                                      // [K][64]
  int4* slot = reinterpret_cast<int4*>(lds + K * S);   // V == 1: per wave 64 entries (32 int4)
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  for (int i = threadIdx.x; i < K * S; i += 64 * NW) x[i] = (float)(i & 7) * 0.25f;
  __syncthreads();
  // every workgroup walks the SAME lists (one per wave), as every workgroup of the kernel walks the same weights
  const int2* L = list + (int64_t)wave * PW;
  float a0 = 0.f, a1 = 0.f, a2 = 0.f, a3 = 0.f;
  if constexpr (V == 0) {
    for (int j = 0; j < PW; j += 4) {
      const int k0 = (j * 37 + wave * 13) & 255, k1 = k0 + 131, k2 = (k0 + 57) & 255, k3 = k0 + 9;
      a0 = fmaf(0.5f, x[k0 * S + lane], a0);
      a1 = fmaf(0.5f, x[k1 * S + lane], a1);
      a2 = fmaf(0.5f, x[k2 * S + lane], a2);
      a3 = fmaf(0.5f, x[k3 * S + lane], a3);
    }
  } else if constexpr (V == 1) {
    int4* my = slot + wave * 32;
    for (int j0 = 0; j0 < PW; j0 += 64) {
      const int2 e = L[j0 + lane];          // 64 entries, stored as 32 int4 pairs of entries
      reinterpret_cast<int2*>(my)[lane] = e;
#pragma unroll 2
      for (int t = 0; t < 32; t += 8) {
        int4 q[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) q[u] = my[t + u];
        float xv[16];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          xv[2 * u] = x[q[u].x * S + lane];
          xv[2 * u + 1] = x[q[u].z * S + lane];
        }
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          const float w0 = __int_as_float(q[u].y), w1 = __int_as_float(q[u].w);
          if (u & 1) { a2 = fmaf(w0, xv[2 * u], a2); a3 = fmaf(w1, xv[2 * u + 1], a3); }
          else { a0 = fmaf(w0, xv[2 * u], a0); a1 = fmaf(w1, xv[2 * u + 1], a1); }
        }
      }
    }
  } else if constexpr (V == 2) {
    for (int j0 = 0; j0 < PW; j0 += 64) {
      const int2 e = L[j0 + lane];
#pragma unroll 16
      for (int t = 0; t < 64; t += 4) {
        float xv[4], w[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const int k = __builtin_amdgcn_readlane(e.x, t + u);
          w[u] = __int_as_float(__builtin_amdgcn_readlane(e.y, t + u));
          xv[u] = x[k * S + lane];
        }
        a0 = fmaf(w[0], xv[0], a0);
        a1 = fmaf(w[1], xv[1], a1);
        a2 = fmaf(w[2], xv[2], a2);
        a3 = fmaf(w[3], xv[3], a3);
      }
    }
  } else {
    for (int j = 0; j < PW; j += 8) {
      int2 q[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) q[u] = L[j + u];   // uniform address: scalar loads
      float xv[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) xv[u] = x[q[u].x * S + lane];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const float w = __int_as_float(q[u].y);
        if ((u & 3) == 0) a0 = fmaf(w, xv[u], a0);
        else if ((u & 3) == 1) a1 = fmaf(w, xv[u], a1);
        else if ((u & 3) == 2) a2 = fmaf(w, xv[u], a2);
        else a3 = fmaf(w, xv[u], a3);
      }
    }
  }
  out[((int64_t)blockIdx.x * NW + wave) * 64 + lane] = (a0 + a1) + (a2 + a3);
}

int main() {
  const int grid = 256;
  const int64_t n = (int64_t)NW * PW;
  std::vector<int2> h(n);
  uint64_t s = 88172645463325252ull;
  for (int64_t i = 0; i < n; ++i) {
    s ^= s << 13; s ^= s >> 7; s ^= s << 17;
    h[i].x = (int)(s % K);
    float w = 0.001f * (float)(s >> 40 & 1023);
    memcpy(&h[i].y, &w, 4);
  }
  int2* d;
  float* out;
  CHECK(hipMalloc(&d, n * sizeof(int2)));
  CHECK(hipMemcpy(d, h.data(), n * sizeof(int2), hipMemcpyHostToDevice));
  CHECK(hipMalloc(&out, (size_t)grid * NW * 64 * 4));
  const size_t lds = (size_t)K * S * 4 + NW * 32 * 16;
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  auto run = [&](auto kern, const char* name) {
    CHECK(hipFuncSetAttribute(reinterpret_cast<const void*>(kern), hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    for (int i = 0; i < 3; ++i) kern<<<grid, 64 * NW, lds>>>(d, out);
    CHECK(hipEventRecord(e0));
    const int reps = 10;
    for (int i = 0; i < reps; ++i) kern<<<grid, 64 * NW, lds>>>(d, out);
    CHECK(hipEventRecord(e1));
    CHECK(hipEventSynchronize(e1));
    float ms;
    CHECK(hipEventElapsedTime(&ms, e0, e1));
    const double us = ms * 1e3 / reps;
    printf("%-44s %8.1f us per launch (workgroup), %6.1f us per 4096-sample batch, %.2f CU-clk per pair-wave @2.4GHz\n",
           name, us, us / 4, us * 2400.0 / (NW * PW));
  };
  run(walk<0>, "A computed (k, w): LDS x read + FMA floor");
  run(walk<1>, "B LDS-staged list, b128 broadcasts");
  run(walk<2>, "C list in VGPRs, v_readlane per pair");
  run(walk<3>, "D wave-uniform global (scalar) loads");
  return 0;
}
