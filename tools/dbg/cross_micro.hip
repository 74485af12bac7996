// Microbenchmark (debug only): what bounds the prediction's cross-covariance (predict.hip
// cross_kp_kernel)?  Same grid and k-major output layout as the library at the C4 chunk (32 GPs,
// n = 1024, 8192 test points: 268M elements, 2.15 GB written) and the C3 chunk (1 GP, n = 4096,
// 16384 points).  Variants:
//   cur       the library's kernel (copied)
//   nostore   the arithmetic alone (one checksum store per thread)
//   storeonly the stores alone (a constant)
//   tabexp    exp from a 64-entry 2^(j/64) table in LDS + a degree-5 polynomial (fewer fp64 ops;
//             not bit-identical: max relative difference to `cur` printed)
//   pair16    two test points per thread, 16-B stores
//   hipcc --offload-arch=gfx950 -O3 -o tools/dbg/cross_micro tools/dbg/cross_micro.hip
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <vector>
#include "../../gladsgp_amd/csrc/gpfit_common.h"

constexpr int D = 8;

__constant__ double c_tab[64];

template <int MODE>   // 0 cur, 1 nostore, 2 storeonly, 3 tabexp
__global__ __launch_bounds__(256) void cross_v(const double* __restrict__ X, int n,
                                               const double* __restrict__ Xs, int mv,
                                               const double* __restrict__ beta,
                                               double* __restrict__ Kt2, int mc, long long sK) {
  const int b = blockIdx.z;
  const int c = blockIdx.x * 256 + threadIdx.x;
  const int kp0 = blockIdx.y * 32;
  __shared__ double xk[64][D];
  __shared__ double bs[D];
  __shared__ double tab[64];
  const double* bb = beta + (long long)b * D;
  if (threadIdx.x < D) bs[threadIdx.x] = __builtin_sqrt(bb[threadIdx.x]);
  if (MODE == 3 && threadIdx.x < 64) tab[threadIdx.x] = c_tab[threadIdx.x];
  __syncthreads();
  for (int t = threadIdx.x; t < 64 * D; t += 256) {
    const int kk = t / D, dd = t % D, k = 2 * kp0 + kk;
    xk[kk][dd] = (k < n) ? X[(long long)k * D + dd] * bs[dd] : 0.0;
  }
  double xc[D];
#pragma unroll
  for (int dd = 0; dd < D; ++dd) xc[dd] = (c < mv) ? Xs[(long long)c * D + dd] * bs[dd] : 0.0;
  __syncthreads();
  if (c >= mc) return;
  double* o = Kt2 + (long long)b * sK;
  const bool col_ok = c < mv;
  double chk = 0.0;
#pragma unroll 2
  for (int kk = 0; kk < 32; ++kk) {
    const int k = 2 * (kp0 + kk);
    double v0 = 1.0, v1 = 1.0;
    if (MODE != 2) {
      double e0 = 0.0, e1 = 0.0;
#pragma unroll
      for (int dd = 0; dd < D; ++dd) {
        const double t0 = xk[2 * kk][dd] - xc[dd], t1 = xk[2 * kk + 1][dd] - xc[dd];
        e0 = fma(t0, t0, e0);
        e1 = fma(t1, t1, e1);
      }
      if (MODE == 3) {
        // exp(-e) = 2^(q >> 6) 2^((q & 63)/64) exp(r), q = rint(-e 64/ln2), |r| <= ln2/128
        auto ex = [&](double a) {
          const double x = -fmin(a, 1100.0);
          const double q = __builtin_rint(x * 0x1.71547652b82fep+6);
          double r = fma(q, -0x1.62e42fefa39efp-7, x);
          r = fma(q, -0x1.abc9e3b39803fp-62, r);
          double p = fma_sc(r, 0x1.1111111111111p-7, 0x1.5555555555555p-5);   // 1/120, 1/24
          p = fma_sc(p, r, 0x1.5555555555555p-3);                              // 1/6
          p = fma_sc(p, r, 0.5);
          p = fma(p, r, 1.0);
          p = p * r;                                                           // exp(r) - 1
          const int qi = (int)q;
          const double t = tab[qi & 63];
          return fma(a, 0.0, __builtin_ldexp(fma(t, p, t), qi >> 6));
        };
        v0 = ex(e0);
        v1 = ex(e1);
      } else {
        v0 = exp_neg(e0);
        v1 = exp_neg(e1);
      }
    }
    if (MODE == 1) {
      chk += v0 + v1;
    } else {
      o[(long long)k * mc + c] = (col_ok && k < n) ? v0 : 0.0;
      o[(long long)(k + 1) * mc + c] = (col_ok && k + 1 < n) ? v1 : 0.0;
    }
  }
  if (MODE == 1 && chk == 12345.678) o[c] = chk;
}

// two test points per thread (c, c + 1), 16-B stores
__global__ __launch_bounds__(256) void cross_pair(const double* __restrict__ X, int n,
                                                  const double* __restrict__ Xs, int mv,
                                                  const double* __restrict__ beta,
                                                  double* __restrict__ Kt2, int mc, long long sK) {
  const int b = blockIdx.z;
  const int c = 2 * (blockIdx.x * 256 + threadIdx.x);
  const int kp0 = blockIdx.y * 32;
  __shared__ double xk[64][D];
  __shared__ double bs[D];
  const double* bb = beta + (long long)b * D;
  if (threadIdx.x < D) bs[threadIdx.x] = __builtin_sqrt(bb[threadIdx.x]);
  __syncthreads();
  for (int t = threadIdx.x; t < 64 * D; t += 256) {
    const int kk = t / D, dd = t % D, k = 2 * kp0 + kk;
    xk[kk][dd] = (k < n) ? X[(long long)k * D + dd] * bs[dd] : 0.0;
  }
  double xa[D], xb[D];
#pragma unroll
  for (int dd = 0; dd < D; ++dd) {
    xa[dd] = (c < mv) ? Xs[(long long)c * D + dd] * bs[dd] : 0.0;
    xb[dd] = (c + 1 < mv) ? Xs[(long long)(c + 1) * D + dd] * bs[dd] : 0.0;
  }
  __syncthreads();
  if (c >= mc) return;
  double* o = Kt2 + (long long)b * sK;
#pragma unroll 2
  for (int kk = 0; kk < 64; ++kk) {
    const int k = 2 * kp0 + kk;
    double ea = 0.0, eb = 0.0;
#pragma unroll
    for (int dd = 0; dd < D; ++dd) {
      const double ta = xk[kk][dd] - xa[dd], tb = xk[kk][dd] - xb[dd];
      ea = fma(ta, ta, ea);
      eb = fma(tb, tb, eb);
    }
    const double va = exp_neg(ea), vb = exp_neg(eb);
    *reinterpret_cast<double2*>(o + (long long)k * mc + c) =
        make_double2((c < mv && k < n) ? va : 0.0, (c + 1 < mv && k < n) ? vb : 0.0);
  }
}

int main() {
  std::vector<double> ht(64);
  for (int j = 0; j < 64; ++j) ht[j] = std::exp2(j / 64.0);
  hipMemcpyToSymbol(HIP_SYMBOL(c_tab), ht.data(), 64 * 8);
  struct Cfg { int B, n, mc; const char* name; };
  for (Cfg cfg : {Cfg{32, 1024, 8192, "C4 chunk (32 x 1024 x 8192)"},
                  Cfg{1, 4096, 16384, "C3 chunk (1 x 4096 x 16384)"}}) {
    const int B = cfg.B, n = cfg.n, mc = cfg.mc;
    std::vector<double> hX((size_t)n * D), hXs((size_t)mc * D), hb((size_t)B * D);
    for (size_t q = 0; q < hX.size(); ++q) hX[q] = (q * 7919 % 1000) / 1000.0;
    for (size_t q = 0; q < hXs.size(); ++q) hXs[q] = (q * 104729 % 997) / 997.0;
    for (size_t q = 0; q < hb.size(); ++q) hb[q] = 0.5 + (q * 31 % 45) / 10.0;
    double *X, *Xs, *be, *K0, *K1;
    const long long sK = (long long)mc * n;
    hipMalloc(&X, hX.size() * 8);
    hipMalloc(&Xs, hXs.size() * 8);
    hipMalloc(&be, hb.size() * 8);
    hipMalloc(&K0, (size_t)B * sK * 8);
    hipMalloc(&K1, (size_t)B * sK * 8);
    hipMemcpy(X, hX.data(), hX.size() * 8, hipMemcpyHostToDevice);
    hipMemcpy(Xs, hXs.data(), hXs.size() * 8, hipMemcpyHostToDevice);
    hipMemcpy(be, hb.data(), hb.size() * 8, hipMemcpyHostToDevice);
    hipEvent_t a, e;
    hipEventCreate(&a); hipEventCreate(&e);
    const dim3 grid(mc / 256, n / 64, B), grid2(mc / 512, n / 64, B);
    auto time = [&](const char* nm, auto fn, double* out) {
      for (int r = 0; r < 3; ++r) fn(out);
      hipEventRecord(a);
      for (int r = 0; r < 10; ++r) fn(out);
      hipEventRecord(e);
      hipEventSynchronize(e);
      float ms;
      hipEventElapsedTime(&ms, a, e);
      ms /= 10;
      printf("  %-10s %8.1f us  %6.0f GB/s of %.2f GB written\n", nm, 1e3 * ms,
             8.0 * B * sK / (ms * 1e-3) / 1e9, 8.0 * B * sK / 1e9);
    };
    printf("%s\n", cfg.name);
    time("cur", [&](double* o) { hipLaunchKernelGGL(cross_v<0>, grid, dim3(256), 0, 0, X, n, Xs, mc, be, o, mc, sK); }, K0);
    time("nostore", [&](double* o) { hipLaunchKernelGGL(cross_v<1>, grid, dim3(256), 0, 0, X, n, Xs, mc, be, o, mc, sK); }, K1);
    time("storeonly", [&](double* o) { hipLaunchKernelGGL(cross_v<2>, grid, dim3(256), 0, 0, X, n, Xs, mc, be, o, mc, sK); }, K1);
    time("tabexp", [&](double* o) { hipLaunchKernelGGL(cross_v<3>, grid, dim3(256), 0, 0, X, n, Xs, mc, be, o, mc, sK); }, K1);
    {
      std::vector<double> h0((size_t)n * mc), h1((size_t)n * mc);
      hipMemcpy(h0.data(), K0, h0.size() * 8, hipMemcpyDeviceToHost);
      hipMemcpy(h1.data(), K1, h1.size() * 8, hipMemcpyDeviceToHost);
      double mx = 0;
      long long nd = 0;
      for (size_t q = 0; q < h0.size(); ++q) {
        if (h0[q] != h1[q]) ++nd;
        if (h0[q] > 1e-300) mx = fmax(mx, fabs(h1[q] - h0[q]) / h0[q]);
      }
      printf("  tabexp vs cur (problem 0): max rel diff %.3e (%.2f ulp), %lld of %zu differ\n", mx,
             mx / 2.220446049250313e-16, nd, h0.size());
    }
    time("pair16", [&](double* o) { hipLaunchKernelGGL(cross_pair, grid2, dim3(256), 0, 0, X, n, Xs, mc, be, o, mc, sK); }, K1);
    hipFree(X); hipFree(Xs); hipFree(be); hipFree(K0); hipFree(K1);
  }
  return 0;
}
