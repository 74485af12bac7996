// ARD squared-exponential Gram / cross-covariance build (HBM-write-bound).
//
// One kernel serves both (reference: examples/01...ipynb:135-141, SEPIA compute_cov_mat):
//   out[i + j*ldo] = s * exp(-sum_k beta_k (XA[i,k] - XB[j,k])^2) + delta*(i==j && diag)
// A block of 4 waves owns a 64 x 64 output tile; lane = row, so each wave stores 64
// consecutive doubles (512 B) per column: fully coalesced column-major writes.  The row design
// vector lives in registers; each wave walks its 16 columns, whose design vectors are
// wave-uniform scalar loads.  A square Gram can be built lower-triangle only (the grid then
// enumerates the tiles on and below the diagonal), which is all the factorisation reads.
//
// Roofline: 8 B written per output element + 8 d B read per row/col vector (amortised);
// one f64 exp (~1.3 T exp/s chip-wide, probe_f64) per element — the store stream (≈6 TB/s =
// 0.75 T elements/s) is the bound.
#include "gpfit_common.h"
#include "gpfit_profile.h"
#include "gpfit_internal.h"
#include "../../include/gpfit.h"

namespace {

constexpr int kTile = 64;    // output tile kTile x kTile per block of 4 waves
constexpr int kWCols = 16;   // columns per wave (lane = row)

// Block (ti, tj) of the output; with `lower`, blockIdx.x enumerates the tiles tj <= ti only.
template <int D>
__global__ __launch_bounds__(256) void ardse_kernel(
    const double* __restrict__ XA, int na, int ldxa,      // row points (output rows)
    const double* __restrict__ XB, int nb, int ldxb,      // column points (output columns)
    int d, const double* __restrict__ beta, int ldbeta,
    const double* __restrict__ s, const double* __restrict__ delta,
    double* __restrict__ out, int ldo, long long stride_o,
    int rows_out, int cols_out, bool lower) {
  const int b = blockIdx.z;
  int ti, tj;
  if (lower) {
    const int t = blockIdx.x;
    ti = (int)((sqrt(8.0 * t + 1.0) - 1.0) * 0.5);
    while (ti * (ti + 1) / 2 > t) --ti;
    while ((ti + 1) * (ti + 2) / 2 <= t) ++ti;
    tj = t - ti * (ti + 1) / 2;
  } else {
    ti = blockIdx.x;
    tj = blockIdx.y;
  }
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int i = ti * kTile + lane;
  const int jw = tj * kTile + w * kWCols;          // this wave's first column (uniform)
  const double* bb = beta + (long long)b * ldbeta;
  double bet[D], xa[D];
  const int ic = i < na ? i : na - 1;
#pragma unroll
  for (int k = 0; k < D; ++k) {
    bet[k] = k < d ? bb[k] : 0.0;
    xa[k] = k < d ? XA[(long long)ic * ldxa + k] : 0.0;
  }
  const double sb = s[b];
  const double db = delta ? delta[b] : 0.0;
  double* o = out + (long long)b * stride_o + i;
  const bool row_st = i < rows_out;
  const bool row_ok = i < na;
#pragma unroll 4
  for (int c = 0; c < kWCols; ++c) {
    const int j = jw + c;                          // uniform
    if (j >= cols_out) break;
    double v = 0.0;
    if (j < nb) {
      const double* xb = XB + (long long)j * ldxb;  // uniform: scalar loads
      double acc = 0.0;
#pragma unroll
      for (int k = 0; k < D; ++k) {
        const double t = xa[k] - (k < d ? xb[k] : 0.0);
        acc = fma(bet[k] * t, t, acc);
      }
      v = fma(sb, exp(-acc), (i == j) ? db : 0.0);
      v = row_ok ? v : 0.0;
    }
    if (row_st && (!lower || j <= i)) o[(long long)j * ldo] = v;
  }
}

template <int D>
hipError_t launch_ardse(const double* XA, int na, int ldxa, const double* XB, int nb, int ldxb,
                        int d, const double* beta, int ldbeta, const double* s,
                        const double* delta, double* out, int ldo, long long stride_o,
                        int rows_out, int cols_out, int batch, bool lower, hipStream_t st) {
  const int TR = gp_ceil_div(rows_out, kTile), TC = gp_ceil_div(cols_out, kTile);
  dim3 grid = lower ? dim3(TR * (TR + 1) / 2, 1, batch) : dim3(TR, TC, batch);
  hipLaunchKernelGGL((ardse_kernel<D>), grid, dim3(256), 0, st, XA, na, ldxa, XB, nb, ldxb,
                     d, beta, ldbeta, s, delta, out, ldo, stride_o, rows_out, cols_out,
                     lower);
  return hipGetLastError();
}

}  // namespace

// Internal entry shared with predict.hip: rows_out/cols_out may exceed na/nb (zero padding);
// `lower` writes only the lower triangle (j <= i) of a square Gram.
hipError_t gpfit_ardse_launch(const double* XA, int na, int ldxa, const double* XB, int nb,
                              int ldxb, int d, const double* beta, int ldbeta,
                              const double* s, const double* delta, double* out, int ldo,
                              long long stride_o, int rows_out, int cols_out, int batch,
                              hipStream_t st, bool lower) {
  if (d <= 8)
    return launch_ardse<8>(XA, na, ldxa, XB, nb, ldxb, d, beta, ldbeta, s, delta, out, ldo,
                           stride_o, rows_out, cols_out, batch, lower, st);
  if (d <= 16)
    return launch_ardse<16>(XA, na, ldxa, XB, nb, ldxb, d, beta, ldbeta, s, delta, out, ldo,
                            stride_o, rows_out, cols_out, batch, lower, st);
  return launch_ardse<32>(XA, na, ldxa, XB, nb, ldxb, d, beta, ldbeta, s, delta, out, ldo,
                          stride_o, rows_out, cols_out, batch, lower, st);
}

extern "C" int gp_version(void) { return 100; }

extern "C" int gp_padded_n(int n) { return n <= 0 ? 0 : gp_ceil_div(n, GPFIT_TILE) * GPFIT_TILE; }

namespace {
int gram_checked(const double* X, int n, int d, int ldx, const double* beta, int ldbeta,
                 const double* s, const double* delta, double* G, int ldg, long long strideG,
                 int batch, hipStream_t stream, bool lower) {
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
                                    strideG, n, n, batch, stream, lower);
  gpfit_prof_end(GP_PROF_GRAM, stream);
  return e == hipSuccess ? 0 : GPFIT_ERR_HIP - (int)e;
}

}  // namespace

extern "C" int gp_gram_ardse(const double* X, int n, int d, int ldx, const double* beta,
                             int ldbeta, const double* s, const double* delta, double* G,
                             int ldg, long long strideG, int batch, hipStream_t stream) {
  return gram_checked(X, n, d, ldx, beta, ldbeta, s, delta, G, ldg, strideG, batch, stream,
                      false);
}

// Lower triangle only (the factorisation never reads the upper one): half the exps and stores.
int gpfit_gram_lower(const double* X, int n, int d, int ldx, const double* beta, int ldbeta,
                     const double* s, const double* delta, double* G, int ldg,
                     long long strideG, int batch, hipStream_t stream) {
  return gram_checked(X, n, d, ldx, beta, ldbeta, s, delta, G, ldg, strideG, batch, stream,
                      true);
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
                                    ldk, strideK, n, m, batch, stream, false);
  return e == hipSuccess ? 0 : GPFIT_ERR_HIP - (int)e;
}
