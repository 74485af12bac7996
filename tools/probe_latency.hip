// Latency probe: per-iteration cycles (s_memtime) of the primitives on the diag critical path.
#include <hip/hip_runtime.h>
#include <cstdio>
#define CK(x) do{hipError_t e=(x); if(e!=hipSuccess){printf("HIP error %s line %d\n",hipGetErrorString(e),__LINE__); return 1;}}while(0)
__device__ __forceinline__ unsigned long long clk() { return __builtin_amdgcn_s_memtime(); }
__device__ __forceinline__ unsigned long long rclk() { return __builtin_amdgcn_s_memrealtime(); }

template <int MODE>
__global__ void probe(double* out, unsigned long long* cyc, int iters) {
  __shared__ double buf[2][256];
  double x = threadIdx.x * 1e-3 + 1.0;
  buf[0][threadIdx.x] = x; buf[1][threadIdx.x] = x;
  __syncthreads();
  unsigned long long t0 = clk(), r0 = rclk();
  for (int it = 0; it < iters; ++it) {
    if (MODE == 0) { __syncthreads(); }                                  // barrier only
    if (MODE == 1) { buf[it & 1][threadIdx.x] = x; __syncthreads(); x += buf[it & 1][(threadIdx.x + 1) & 255]; }  // lds write-barrier-read chain
    if (MODE == 2) { x = fma(x, 0.999999, 1e-7); }                        // dependent f64 fma
    if (MODE == 3) { double p = __builtin_amdgcn_rsq(x); x = x * p + 1.0; } // rsq chain
    if (MODE == 4) { x = sqrt(x) + 1.0; }                                 // full sqrt
    if (MODE == 5) { x = 1.0 / x + 1.0; }                                 // full div
  }
  unsigned long long t1 = clk(), r1 = rclk();
  if (threadIdx.x == 0) { cyc[blockIdx.x * 2] = t1 - t0; cyc[blockIdx.x * 2 + 1] = r1 - r0; }
  if (x == 12345.0) out[0] = x;
}

int main() {
  double* out; unsigned long long* cyc; CK(hipMalloc(&out, 8)); CK(hipMalloc(&cyc, 16 * 1024));
  const char* names[] = {"barrier(256thr)", "lds wr+barrier+rd", "dep f64 fma", "rsq chain", "sqrt()", "1/x"};
  int iters = 10000;
  for (int rep = 0; rep < 2; ++rep)
  for (int mode = 0; mode < 6; ++mode) {
    unsigned long long h[2];
    switch (mode) {
      case 0: probe<0><<<1, 256>>>(out, cyc, iters); break;
      case 1: probe<1><<<1, 256>>>(out, cyc, iters); break;
      case 2: probe<2><<<1, 256>>>(out, cyc, iters); break;
      case 3: probe<3><<<1, 256>>>(out, cyc, iters); break;
      case 4: probe<4><<<1, 256>>>(out, cyc, iters); break;
      case 5: probe<5><<<1, 256>>>(out, cyc, iters); break;
    }
    CK(hipDeviceSynchronize());
    CK(hipMemcpy(h, cyc, 16, hipMemcpyDeviceToHost));
    double ns = h[1] * 10.0 / iters;  // memrealtime = 100 MHz
    if (rep) printf("%-22s %8.1f cycles/iter  %7.1f ns/iter  (clock %.2f GHz)\n", names[mode], (double)h[0] / iters, ns, (double)h[0] / (h[1] * 10.0));
  }
  return 0;
}
