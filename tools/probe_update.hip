// Timing probe for one trailing-update launch of the n = 4096 factorisation (step k): the
// production kernel, its workers alone (block 0 skips the diagonal factor) and block 0 alone
// (tile + factor), each averaged over repetitions from the same input state.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -mllvm -amdgpu-mfma-vgpr-form
//        -Xclang -target-feature -Xclang +enable-ds128 tools/probe_update.hip
//        gladsgp_amd/csrc/profile.hip gladsgp_amd/csrc/gram.hip -o tools/probe_update
#include "../gladsgp_amd/csrc/chol.hip"
#include <cstdio>
#include <vector>
#include <algorithm>

int main(int argc, char** argv) {
  const int n = argc > 1 ? atoi(argv[1]) : 4096, N = n / NB;
  std::vector<double> A((size_t)n * n);
  for (int j = 0; j < n; ++j)
    for (int i = 0; i < n; ++i) A[i + (size_t)j * n] = exp(-0.0005 * (i - j) * (i - j)) + (i == j ? 1.0 : 0.0);
  double *dA, *dW, *dX, *dl;
  int* di;
  hipMalloc(&dA, (size_t)n * n * 8);
  hipMalloc(&dW, (size_t)n * n * 8);
  hipMalloc(&dX, (size_t)n * n * 8);
  hipMalloc(&dl, 8 * 2 * 4096);
  hipMalloc(&di, 4);
  hipMemcpy(dA, A.data(), (size_t)n * n * 8, hipMemcpyHostToDevice);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  for (int kf = 0; kf < 5; ++kf) {
    const int k = (N - 8) * kf / 4;
    const int T = N - k - 1, nt = T * (T + 1) / 2 + T * (k + 1);
    const int g = argc > 2 ? std::min(nt, atoi(argv[2])) : update_grid(nt, 1);
    double t[4] = {0, 0, 0, 0};
    const int reps = 10;
    for (int mode = 0; mode < 4; ++mode)
      for (int r = 0; r < reps + 1; ++r) {
        hipMemcpy(dW, dA, (size_t)n * n * 8, hipMemcpyDeviceToDevice);
        hipMemset(dX, 0, (size_t)n * n * 8);
        hipMemset(di, 0, 4);
        hipEventRecord(e0);
        if (mode == 0)
          hipLaunchKernelGGL(chol_update_kernel<0>, dim3(g, 1), dim3(256), 0, 0, dW, n, 0LL, dX, n, 0LL, n, k, T, di, dl);
        else if (mode == 1)
          hipLaunchKernelGGL(chol_update_kernel<1>, dim3(g, 1), dim3(256), 0, 0, dW, n, 0LL, dX, n, 0LL, n, k, T, di, dl);
        else if (mode == 2)
          hipLaunchKernelGGL(chol_update_kernel<2>, dim3(1, 1), dim3(256), 0, 0, dW, n, 0LL, dX, n, 0LL, n, k, T, di, dl);
        else
          hipLaunchKernelGGL(chol_update_kernel<6>, dim3(g, 1), dim3(256), 0, 0, dW, n, 0LL, dX, n, 0LL, n, k, T, di, dl);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms;
        hipEventElapsedTime(&ms, e0, e1);
        if (r) t[mode] += ms * 1e3 / reps;
      }
    printf("n=%d k=%2d tiles=%5d grid=%4d  full %6.1f  workers %6.1f  block0 %6.1f  "
           "empty %6.1f us (events)\n", n, k, nt, g, t[0], t[1], t[2], t[3]);
    // per-block start / end stamps of the workers (s_memrealtime, 100 MHz); pass 2 of 2
    for (int mm = 8; mm <= 9; ++mm) {
    hipMemcpy(dW, dA, (size_t)n * n * 8, hipMemcpyDeviceToDevice);
    if (mm == 8)
      hipLaunchKernelGGL(chol_update_kernel<8>, dim3(g, 1), dim3(256), 0, 0, dW, n, 0LL, dX, n, 0LL, n, k, T, di, dl);
    else
      hipLaunchKernelGGL(chol_update_kernel<9>, dim3(g, 1), dim3(256), 0, 0, dW, n, 0LL, dX, n, 0LL, n, k, T, di, dl);
    hipDeviceSynchronize();
    std::vector<double> st(2 * g);
    hipMemcpy(st.data(), dl, 16 * g, hipMemcpyDeviceToHost);
    double t0 = 1e300, t1 = 0, dmin = 1e300, dmax = 0, dsum = 0, smax = 0;
    for (int b = 1; b < g; ++b) t0 = std::min(t0, st[2 * b]);
    for (int b = 1; b < g; ++b) {
      const double d = (st[2 * b + 1] - st[2 * b]) / 100.0;   // us
      dmin = std::min(dmin, d); dmax = std::max(dmax, d); dsum += d;
      smax = std::max(smax, (st[2 * b] - t0) / 100.0);
      t1 = std::max(t1, st[2 * b + 1]);
    }
    printf("    workers%s: start spread %.1f us, duration min %.1f mean %.1f max %.1f us, span %.1f us\n",
           mm == 9 ? " (2nd pass)" : "", smax, dmin, dsum / (g - 1), dmax, (t1 - t0) / 100.0);
    }
  }
  return 0;
}
