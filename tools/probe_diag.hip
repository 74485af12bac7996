// Timing probe for the Cholesky diagonal-block factor (diag_factor_inv): one block factors a
// 64x64 SPD tile `iters` times; s_memtime stamps inside the sweep (GPFIT_DIAG_PROBE) give the
// wave-0 sweep, wave-1 lag and epilogue cycle counts.  Build: see tools/gpu_probe_diag.sh.
#define GPFIT_DIAG_PROBE 1
#include "../gladsgp_amd/csrc/chol.hip"
#include <cstdio>
#include <cmath>
#include <vector>

namespace {
__global__ __launch_bounds__(256, 2) void probe_kernel(const double* A, double* out, int iters,
                                                    unsigned long long* st) {
  Smem& sm = g_sm;
  double lg = 0.0;
  unsigned long long acc[4] = {0, 0, 0, 0};
  for (int it = 0; it < iters; ++it) {
    for (int g = threadIdx.x; g < NB * NB; g += 256) sm.As[(g >> 6) * LP + (g & 63)] = A[g];
    __syncthreads();
#ifdef OLD
    diag_factor_inv(sm, sm.As, sm.Bs, NB, &lg);
#else
    diag_factor_inv(NB, &lg);
#endif
    __syncthreads();
#ifndef OLD
    if (threadIdx.x == 0) {
      acc[0] += gpfit_diag_probe[1] - gpfit_diag_probe[0];
      acc[1] += gpfit_diag_probe[2] - gpfit_diag_probe[0];
      acc[2] += gpfit_diag_probe[3] - gpfit_diag_probe[0];
    }
#endif
  }
  for (int g = threadIdx.x; g < NB * NB; g += 256) {
    out[g] = sm.As[(g >> 6) * LP + (g & 63)];
    out[NB * NB + g] = sm.Bs[(g >> 6) * LP + (g & 63)];
  }
  if (threadIdx.x == 0) {
    st[0] = acc[0]; st[1] = acc[1]; st[2] = acc[2];
    double* o = out + 2 * NB * NB;
    o[0] = lg;
  }
}
}  // namespace

int main() {
  const int n = NB;
  std::vector<double> A(n * n), out(2 * n * n + 1);
  for (int i = 0; i < n; ++i)
    for (int j = 0; j < n; ++j) A[i * n + j] = exp(-0.02 * (i - j) * (i - j)) + (i == j ? 0.5 : 0.0);
  double *dA, *dO;
  unsigned long long* dS;
  hipMalloc(&dA, n * n * 8);
  hipMalloc(&dO, out.size() * 8);
  hipMalloc(&dS, 64);
  hipMemcpy(dA, A.data(), n * n * 8, hipMemcpyHostToDevice);
  const int iters = 200;
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  hipLaunchKernelGGL(probe_kernel, dim3(1), dim3(256), 0, 0, dA, dO, 2, dS);
  hipEventRecord(e0);
  hipLaunchKernelGGL(probe_kernel, dim3(1), dim3(256), 0, 0, dA, dO, iters, dS);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms;
  hipEventElapsedTime(&ms, e0, e1);
  unsigned long long st[3];
  hipMemcpy(st, dS, 24, hipMemcpyDeviceToHost);
  hipMemcpy(out.data(), dO, out.size() * 8, hipMemcpyDeviceToHost);
  // check: L L^T = A and Linv L = I
  double e1m = 0, e2m = 0;
  for (int i = 0; i < n; ++i)
    for (int j = 0; j <= i; ++j) {
      double s = 0, t = 0;
      for (int k = 0; k < n; ++k) {
        s += out[i * n + k] * out[j * n + k];
        t += out[n * n + i * n + k] * out[k * n + j];
      }
      e1m = fmax(e1m, fabs(s - A[i * n + j]));
      e2m = fmax(e2m, fabs(t - (i == j ? 1.0 : 0.0)));
    }
  // cold: flush L2/MALL by writing a large buffer, then one factor per launch
  void* big;
  hipMalloc(&big, 1ull << 30);
  float cold = 0.f;
  for (int rep = 0; rep < 5; ++rep) {
    hipMemset(big, rep, 1ull << 30);
    hipEventRecord(e0);
    hipLaunchKernelGGL(probe_kernel, dim3(1), dim3(256), 0, 0, dA, dO, 1, dS);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float t;
    hipEventElapsedTime(&t, e0, e1);
    cold += t / 5;
  }
  float warm1 = 0.f;
  for (int rep = 0; rep < 5; ++rep) {
    hipEventRecord(e0);
    hipLaunchKernelGGL(probe_kernel, dim3(1), dim3(256), 0, 0, dA, dO, 1, dS);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float t;
    hipEventElapsedTime(&t, e0, e1);
    warm1 += t / 5;
  }
  printf("single launch: cold-L2 %.2f us, warm %.2f us\n", cold * 1e3, warm1 * 1e3);
  printf("per factor: %.2f us (event)  memtime ticks: w0 sweep %.0f  w1 done %.0f  end %.0f\n",
         ms * 1e3 / iters, (double)st[0] / iters, (double)st[1] / iters, (double)st[2] / iters);
  printf("max |LL^T - A| = %.3e   max |Linv L - I| = %.3e   logdet %.6f\n", e1m, e2m,
         out[2 * n * n]);
  return 0;
}
