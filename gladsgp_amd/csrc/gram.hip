// ARD squared-exponential Gram / cross-covariance build (HBM-write-bound).
//
// One kernel serves both (reference: examples/01...ipynb:135-141, SEPIA compute_cov_mat):
//   out[i + j*ldo] = s * exp(-sum_k beta_k (XA[i,k] - XB[j,k])^2) + delta*(i==j && diag)
// Rows i of the output are the fast (contiguous) index, so each wave stores 64 consecutive
// doubles (512 B) per column: fully coalesced column-major writes.  A block covers 256 rows x
// COLS columns; its row design vectors live in registers and the COLS column design vectors
// are staged once in LDS and read as wave-uniform broadcasts.
//
// Roofline: 8 B written per output element + 8 d B read per row/col vector (amortised);
// one f64 exp (~1.3 T exp/s chip-wide, probe_f64) per element — the store stream (≈6 TB/s =
// 0.75 T elements/s) is the bound.
#include "gpfit_common.h"
#include "gpfit_profile.h"
#include "../../include/gpfit.h"

namespace {

constexpr int kRows = 256;   // threads per block == rows per block
constexpr int kCols = 32;    // columns per block

template <int D>
__global__ __launch_bounds__(kRows) void ardse_kernel(
    const double* __restrict__ XA, int na, int ldxa,      // row points (output rows)
    const double* __restrict__ XB, int nb, int ldxb,      // column points (output columns)
    int d, const double* __restrict__ beta, int ldbeta,
    const double* __restrict__ s, const double* __restrict__ delta,
    double* __restrict__ out, int ldo, long long stride_o,
    int rows_out, int cols_out) {
  const int b = blockIdx.z;
  const int i = blockIdx.x * kRows + threadIdx.x;
  const int j0 = blockIdx.y * kCols;
  __shared__ double xb_s[kCols][D];
  __shared__ double beta_s[D];

  const double* bb = beta + (long long)b * ldbeta;
  if (threadIdx.x < D) beta_s[threadIdx.x] = (threadIdx.x < d) ? bb[threadIdx.x] : 0.0;
  for (int t = threadIdx.x; t < kCols * D; t += kRows) {
    int jj = t / D, k = t % D;
    int j = j0 + jj;
    xb_s[jj][k] = (j < nb && k < d) ? XB[(long long)j * ldxb + k] : 0.0;
  }
  double xa[D];
#pragma unroll
  for (int k = 0; k < D; ++k) xa[k] = (i < na && k < d) ? XA[(long long)i * ldxa + k] : 0.0;
  __syncthreads();

  const double sb = s[b];
  const double db = delta ? delta[b] : 0.0;
  double* o = out + (long long)b * stride_o;
  if (i >= rows_out) return;
  const bool row_ok = i < na;
#pragma unroll 4
  for (int jj = 0; jj < kCols; ++jj) {
    const int j = j0 + jj;
    if (j >= cols_out) break;
    double v = 0.0;
    if (row_ok && j < nb) {
      double acc = 0.0;
#pragma unroll
      for (int k = 0; k < D; ++k) {
        double t = xa[k] - xb_s[jj][k];
        acc = fma(beta_s[k] * t, t, acc);
      }
      v = sb * exp(-acc);
      if (delta && i == j) v += db;
    }
    o[i + (long long)j * ldo] = v;
  }
}

template <int D>
hipError_t launch_ardse(const double* XA, int na, int ldxa, const double* XB, int nb, int ldxb,
                        int d, const double* beta, int ldbeta, const double* s,
                        const double* delta, double* out, int ldo, long long stride_o,
                        int rows_out, int cols_out, int batch, hipStream_t st) {
  dim3 grid(gp_ceil_div(rows_out, kRows), gp_ceil_div(cols_out, kCols), batch);
  hipLaunchKernelGGL((ardse_kernel<D>), grid, dim3(kRows), 0, st, XA, na, ldxa, XB, nb, ldxb,
                     d, beta, ldbeta, s, delta, out, ldo, stride_o, rows_out, cols_out);
  return hipGetLastError();
}

}  // namespace

// Internal entry shared with predict.hip: rows_out/cols_out may exceed na/nb (zero padding).
hipError_t gpfit_ardse_launch(const double* XA, int na, int ldxa, const double* XB, int nb,
                              int ldxb, int d, const double* beta, int ldbeta,
                              const double* s, const double* delta, double* out, int ldo,
                              long long stride_o, int rows_out, int cols_out, int batch,
                              hipStream_t st) {
  if (d <= 8)
    return launch_ardse<8>(XA, na, ldxa, XB, nb, ldxb, d, beta, ldbeta, s, delta, out, ldo,
                           stride_o, rows_out, cols_out, batch, st);
  if (d <= 16)
    return launch_ardse<16>(XA, na, ldxa, XB, nb, ldxb, d, beta, ldbeta, s, delta, out, ldo,
                            stride_o, rows_out, cols_out, batch, st);
  return launch_ardse<32>(XA, na, ldxa, XB, nb, ldxb, d, beta, ldbeta, s, delta, out, ldo,
                          stride_o, rows_out, cols_out, batch, st);
}

extern "C" int gp_version(void) { return 100; }

extern "C" int gp_padded_n(int n) { return n <= 0 ? 0 : gp_ceil_div(n, GPFIT_TILE) * GPFIT_TILE; }

extern "C" int gp_gram_ardse(const double* X, int n, int d, int ldx, const double* beta,
                             int ldbeta, const double* s, const double* delta, double* G,
                             int ldg, long long strideG, int batch, hipStream_t stream) {
  if (!X) return -1;
  if (n < 0) return -2;
  if (d < 1 || d > GPFIT_MAX_DIM) return -3;
  if (ldx < d) return -4;
  if (!beta) return -5;
  if (ldbeta < d && batch > 1) return -6;
  if (!s) return -7;
  if (!delta) return -8;
  if (!G) return -9;
  if (ldg < n) return -10;
  if (batch > 1 && strideG < (long long)ldg * n) return -11;
  if (batch < 0) return -12;
  if (n == 0 || batch == 0) return 0;
  gpfit_prof_begin(GP_PROF_GRAM, stream);
  hipError_t e = gpfit_ardse_launch(X, n, ldx, X, n, ldx, d, beta, ldbeta, s, delta, G, ldg,
                                    strideG, n, n, batch, stream);
  gpfit_prof_end(GP_PROF_GRAM, stream);
  return e == hipSuccess ? 0 : GPFIT_ERR_HIP - (int)e;
}

extern "C" int gp_cross_ardse(const double* X, int n, int ldx, const double* Xs, int m,
                              int ldxs, int d, const double* beta, int ldbeta,
                              const double* s, double* Kt, int ldk, long long strideK,
                              int batch, hipStream_t stream) {
  if (!X) return -1;
  if (n < 0) return -2;
  if (ldx < d) return -3;
  if (!Xs) return -4;
  if (m < 0) return -5;
  if (ldxs < d) return -6;
  if (d < 1 || d > GPFIT_MAX_DIM) return -7;
  if (!beta) return -8;
  if (ldbeta < d && batch > 1) return -9;
  if (!s) return -10;
  if (!Kt) return -11;
  if (ldk < n) return -12;
  if (batch > 1 && strideK < (long long)ldk * m) return -13;
  if (batch < 0) return -14;
  if (n == 0 || m == 0 || batch == 0) return 0;
  hipError_t e = gpfit_ardse_launch(X, n, ldx, Xs, m, ldxs, d, beta, ldbeta, s, nullptr, Kt,
                                    ldk, strideK, n, m, batch, stream);
  return e == hipSuccess ? 0 : GPFIT_ERR_HIP - (int)e;
}
