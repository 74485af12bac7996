// Microbenchmark (debug only): what bounds the lower-triangle Gram build at n = 4096?
// Variants over the same unit ranges as gram.hip's ardse_kernel: MODE 0 store-only (constant
// value), 1 compute-only (exp + distance, a checksum store per wave), 2 both, 3 both with the
// library's sqrt(beta)-prescaled distance (2 d ops per element instead of 3 d); lane = row,
// 512-B column segments, 64 x 64 tiles.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#include <cmath>
#include "../../gladsgp_amd/csrc/gram.hip"

template <int MODE>
__global__ __launch_bounds__(256) void k(const double* X, int n, double* out, int total, int rows2) {
  __shared__ double xs_all[4][64 * 8];
  const int lane = threadIdx.x & 63, w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  double* xs = xs_all[w];
  const long long nw = (long long)gridDim.x * 4, gw = (long long)blockIdx.x * 4 + w;
  int u = (int)(total * gw / nw);
  const int u1 = (int)(total * (gw + 1) / nw);
  double xa[8], bet[8], chk = 0.0;
  for (int q = 0; q < 8; ++q) bet[q] = 0.5 + q * 0.5;
  while (u < u1) {
    const int t = u >> 6, c0 = u & 63;
    const int len = min(64 - c0, u1 - u);
    int ti = (int)((sqrt(8.0 * t + 1.0) - 1.0) * 0.5);
    while (ti * (ti + 1) / 2 > t) --ti;
    while ((ti + 1) * (ti + 2) / 2 <= t) ++ti;
    const int tj = t - ti * (ti + 1) / 2;
    const int i = ti * 64 + lane;
    for (int q = 0; q < 8; ++q) xa[q] = X[i * 8 + q];
    __builtin_amdgcn_wave_barrier();
    for (int q = 0; q < 8; ++q) xs[lane * 8 + q] = X[(tj * 64 + lane) * 8 + q];
    __builtin_amdgcn_wave_barrier();
    double* o = out + i;
    for (int c = c0; c < c0 + len; ++c) {
      const int j = tj * 64 + c;
      double v = 1.0;
      if (MODE != 0) {
        const double* xb = xs + c * 8;
        double acc = 0.0;
#pragma unroll
        for (int q = 0; q < 8; ++q) {
          const double dt = xa[q] - xb[q];
          acc = MODE == 3 ? fma(dt, dt, acc) : fma(bet[q] * dt, dt, acc);
        }
        v = exp_neg(acc);
      }
      if (MODE == 1) chk += v;
      else if (j <= i) o[(long long)j * n] = v;
    }
    u += len;
  }
  if (MODE == 1 && chk == 12345.678) out[0] = chk;
}

int main() {
  const int n = 4096, TR = n / 64;
  const int total = TR * (TR + 1) / 2 * 64;
  std::vector<double> hX(n * 8);
  for (size_t q = 0; q < hX.size(); ++q) hX[q] = (q * 7919 % 1000) / 1000.0;
  double *X, *G;
  hipMalloc(&X, hX.size() * 8);
  hipMalloc(&G, (size_t)n * n * 8);
  hipMemcpy(X, hX.data(), hX.size() * 8, hipMemcpyHostToDevice);
  hipEvent_t a, b;
  hipEventCreate(&a); hipEventCreate(&b);
  for (int mode = 0; mode < 4; ++mode)
    for (int bpc : {2, 4, 7, 8}) {
      const int grid = 256 * bpc;
      auto run = [&] {
        if (mode == 0) hipLaunchKernelGGL(k<0>, dim3(grid), dim3(256), 0, 0, X, n, G, total, 0);
        if (mode == 1) hipLaunchKernelGGL(k<1>, dim3(grid), dim3(256), 0, 0, X, n, G, total, 0);
        if (mode == 2) hipLaunchKernelGGL(k<2>, dim3(grid), dim3(256), 0, 0, X, n, G, total, 0);
        if (mode == 3) hipLaunchKernelGGL(k<3>, dim3(grid), dim3(256), 0, 0, X, n, G, total, 0);
      };
      for (int r = 0; r < 3; ++r) run();
      hipEventRecord(a);
      for (int r = 0; r < 20; ++r) run();
      hipEventRecord(b);
      hipEventSynchronize(b);
      float ms; hipEventElapsedTime(&ms, a, b);
      printf("mode %d (%s) bpc %d: %.2f us/launch\n", mode,
             mode == 0 ? "store only" : mode == 1 ? "compute only" : mode == 2 ? "both"
             : "both, prescaled 2d distance", bpc, ms * 1e3 / 20);
    }
  // the library kernel itself (lower triangle, as gp_fit_predict / gp_loglik build it)
  double *beta, *sv, *dv;
  hipMalloc(&beta, 64); hipMalloc(&sv, 8); hipMalloc(&dv, 8);
  std::vector<double> hb(8);
  for (int q = 0; q < 8; ++q) hb[q] = 0.5 + q * 0.5;
  const double one = 1.0, dl = 1e-6;
  hipMemcpy(beta, hb.data(), 64, hipMemcpyHostToDevice);
  hipMemcpy(sv, &one, 8, hipMemcpyHostToDevice);
  hipMemcpy(dv, &dl, 8, hipMemcpyHostToDevice);
  for (int lower = 1; lower >= 0; --lower) {
    auto run = [&] { gpfit_ardse_launch(X, n, 8, X, n, 8, 8, beta, 8, sv, dv, G, n, (long long)n * n,
                                        n, n, 1, 0, lower != 0); };
    for (int r = 0; r < 3; ++r) run();
    hipEventRecord(a);
    for (int r = 0; r < 20; ++r) run();
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms; hipEventElapsedTime(&ms, a, b);
    printf("library ardse_kernel %s: %.2f us/launch\n", lower ? "lower" : "full", ms * 1e3 / 20);
  }
  return 0;
}
