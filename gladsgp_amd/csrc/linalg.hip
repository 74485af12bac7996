// Small fp64 linear-algebra helpers on the fit side of the path:
//   gp_trmv : z = L^-1 w            (triangular gemv, HBM-bound: reads n^2/2 doubles)
//   gp_nll  : 1/2 ||L^-1 w||^2 + 1/2 log|A|   — the GP negative log-likelihood of GPmodule
//             (examples/02...ipynb:70-72, no 2pi term) and the per-PC quadratic form + logdet
//             of SEPIA's logLik (src/model.py:234-235 drives it through do_mcmc).
#include "gpfit_common.h"
#include "../../include/gpfit.h"

namespace {

// z_b[r] = sum_{k<=r, k<n} Linv_b[r,k] w_b[k] for r < rows.  1024 threads = 64 rows x 16
// k-slices: each wave reads 64 consecutive rows of one column (512 B, coalesced), the 16
// partial sums meet in LDS.  Reads the n^2/2 lower triangle once: HBM-bound.
constexpr int kTrmvSlices = 16;
__global__ __launch_bounds__(1024) void trmv_kernel(const double* __restrict__ Linv, int ld,
                                                    long long sL, const double* __restrict__ w,
                                                    int ldw, double* __restrict__ z, int ldz,
                                                    int rows, int n) {
  const int b = blockIdx.y;
  const int r = blockIdx.x * 64 + (threadIdx.x & 63);
  const int ks = threadIdx.x >> 6;
  const double* L = Linv + b * sL;
  const double* wb = w + (long long)b * ldw;
  double acc0 = 0.0, acc1 = 0.0;
  const int kend = min(blockIdx.x * 64 + 64, n);   // block-uniform bound; L is zero above r
  if (r < rows) {
    int k = ks;
    for (; k + kTrmvSlices < kend; k += 2 * kTrmvSlices) {
      acc0 = fma(L[r + (long long)k * ld], wb[k], acc0);
      acc1 = fma(L[r + (long long)(k + kTrmvSlices) * ld], wb[k + kTrmvSlices], acc1);
    }
    if (k < kend) acc0 = fma(L[r + (long long)k * ld], wb[k], acc0);
  }
  __shared__ double red[kTrmvSlices][64];
  red[ks][threadIdx.x & 63] = acc0 + acc1;
  __syncthreads();
  if (ks == 0 && r < rows) {
    const int t = threadIdx.x;
    double s = 0.0;
#pragma unroll
    for (int q = 0; q < kTrmvSlices; ++q) s += red[q][t];
    z[(long long)b * ldz + r] = s;
  }
}

__global__ __launch_bounds__(256) void nll_reduce_kernel(const double* __restrict__ z, int ldz,
                                                         int n,
                                                         const double* __restrict__ logdet,
                                                         double* __restrict__ nll) {
  const int b = blockIdx.x;
  const double* zb = z + (long long)b * ldz;
  double acc = 0.0;
  for (int r = threadIdx.x; r < n; r += 256) acc = fma(zb[r], zb[r], acc);
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) acc += __shfl_xor(acc, off, 64);
  __shared__ double red[4];
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = acc;
  __syncthreads();
  if (threadIdx.x == 0) nll[b] = 0.5 * ((red[0] + red[1]) + (red[2] + red[3])) + 0.5 * logdet[b];
}

}  // namespace

hipError_t gpfit_trmv_launch(const double* Linv, int ld, long long sL, const double* w,
                             int ldw, double* z, int ldz, int rows, int n, int batch,
                             hipStream_t st) {
  hipLaunchKernelGGL(trmv_kernel, dim3(gp_ceil_div(rows, 64), batch), dim3(1024), 0, st, Linv,
                     ld, sL, w, ldw, z, ldz, rows, n);
  return hipGetLastError();
}

extern "C" int gp_trmv(const double* Linv, int ldinv, long long strideInv, int n,
                       const double* w, int ldw, double* z, int ldz, int batch,
                       hipStream_t stream) {
  if (!Linv) return -1;
  if (ldinv < n || ldinv < 1) return -2;
  if (batch > 1 && strideInv < (long long)ldinv * n) return -3;
  if (n < 0) return -4;
  if (!w) return -5;
  if (ldw < n && batch > 1) return -6;
  if (!z) return -7;
  if (ldz < n && batch > 1) return -8;
  if (batch < 0) return -9;
  if (n == 0 || batch == 0) return 0;
  hipError_t e = gpfit_trmv_launch(Linv, ldinv, strideInv, w, ldw, z, ldz, n, n, batch, stream);
  return e == hipSuccess ? 0 : GPFIT_ERR_HIP - (int)e;
}

extern "C" int gp_nll(const double* Linv, int ldinv, long long strideInv, int n,
                      const double* w, int ldw, const double* logdet, double* nll,
                      double* work, int batch, hipStream_t stream) {
  if (!Linv) return -1;
  if (ldinv < n || ldinv < 1) return -2;
  if (batch > 1 && strideInv < (long long)ldinv * n) return -3;
  if (n < 0) return -4;
  if (!w) return -5;
  if (ldw < n && batch > 1) return -6;
  if (!logdet) return -7;
  if (!nll) return -8;
  if (!work) return -9;
  if (batch < 0) return -10;
  if (n == 0 || batch == 0) return 0;
  hipError_t e = gpfit_trmv_launch(Linv, ldinv, strideInv, w, ldw, work, n, n, n, batch, stream);
  if (e != hipSuccess) return GPFIT_ERR_HIP - (int)e;
  hipLaunchKernelGGL(nll_reduce_kernel, dim3(batch), dim3(256), 0, stream, work, n, n, logdet,
                     nll);
  e = hipGetLastError();
  return e == hipSuccess ? 0 : GPFIT_ERR_HIP - (int)e;
}
