// Timing + correctness probe for the Cholesky diagonal-block factor: gp_potrf_inv at n = 64 is
// exactly one chol_diag_kernel launch.  Run under rocprofv3 --kernel-trace for the kernel's
// duration (in-kernel s_memtime stamps were tried and distort the kernel's codegen).
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -mllvm -amdgpu-mfma-vgpr-form
//        -Xclang -target-feature -Xclang +enable-ds128 tools/probe_diag.hip
//        gladsgp_amd/csrc/profile.hip gladsgp_amd/csrc/gram.hip -o tools/probe_diag
#include "../gladsgp_amd/csrc/chol.hip"
#include <cstdio>
#include <cmath>
#include <vector>

// diag_factor_inv twice in one launch from the same tile: the first call runs on a cold
// instruction cache (as in every update launch), the second on a warm one (if it fits).
__global__ __launch_bounds__(256, 2) void diag_twice(const double* __restrict__ A,
                                                    unsigned long long* stamps) {
  Smem& sm = g_sm;
  for (int pass = 0; pass < 2; ++pass) {
    for (int g = threadIdx.x; g < NB * NB; g += 256) {
      const int row = g & (NB - 1), col = g >> 6;
      sm.As[row * LP + col] = A[row + col * NB];
    }
    __syncthreads();
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    double lg = 0.0;
    diag_factor_inv(NB, &lg);
    const unsigned long long t1 = __builtin_amdgcn_s_memrealtime();
    if (threadIdx.x == 0) { stamps[2 * pass] = t0; stamps[2 * pass + 1] = t1; }
    __syncthreads();
  }
}

int main() {
  const int n = NB;
  std::vector<double> A(n * n), L(n * n), X(n * n);
  for (int i = 0; i < n; ++i)
    for (int j = 0; j < n; ++j) A[i + j * n] = exp(-0.02 * (i - j) * (i - j)) + (i == j ? 0.5 : 0.0);
  double *dA, *dW, *dX, *dl;
  int* di;
  hipMalloc(&dA, n * n * 8);
  hipMalloc(&dW, n * n * 8);
  hipMalloc(&dX, 128 * 128 * 8);
  hipMalloc(&dl, 8);
  hipMalloc(&di, 4);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  const int reps = 20;
  double ev = 0;
  for (int r = 0; r < reps + 2; ++r) {
    hipMemcpy(dW, A.data(), n * n * 8, hipMemcpyHostToDevice);
    hipEventRecord(e0);
    gp_potrf_inv(dW, n, n, 0, dX, 128, 0, 1, di, dl, 0);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    if (r >= 2) ev += ms * 1e3 / reps;
  }
  hipMemcpy(L.data(), dW, n * n * 8, hipMemcpyDeviceToHost);
  std::vector<double> Xf(128 * 128);
  hipMemcpy(Xf.data(), dX, 128 * 128 * 8, hipMemcpyDeviceToHost);
  double e1m = 0, e2m = 0;
  for (int i = 0; i < n; ++i)
    for (int j = 0; j <= i; ++j) {
      double s = 0, t = 0;
      for (int k = 0; k <= j; ++k) s += L[i + k * n] * L[j + k * n];
      for (int k = j; k <= i; ++k) t += Xf[i + k * 128] * L[k + j * n];
      e1m = fmax(e1m, fabs(s - A[i + j * n]));
      e2m = fmax(e2m, fabs(t - (i == j ? 1.0 : 0.0)));
    }
  printf("potrf(64) call %.2f us (events, incl. the memsets)\n", ev);
  unsigned long long* dst;
  hipMalloc(&dst, 32);
  for (int r = 0; r < 3; ++r) {
    hipLaunchKernelGGL(diag_twice, dim3(1), dim3(256), 0, 0, dA, dst);
    hipDeviceSynchronize();
    unsigned long long h[4];
    hipMemcpy(h, dst, 32, hipMemcpyDeviceToHost);
    printf("diag_factor_inv: first call %.2f us, second call %.2f us\n", (h[1] - h[0]) / 100.0,
           (h[3] - h[2]) / 100.0);
  }
  printf("max |LL^T - A| = %.3e   max |Linv L - I| = %.3e\n", e1m, e2m);
  return 0;
}
