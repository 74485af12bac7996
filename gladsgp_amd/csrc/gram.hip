// ARD squared-exponential Gram / cross-covariance build (HBM-write-bound).
//
// One kernel serves both (reference: examples/01...ipynb:135-141, SEPIA compute_cov_mat):
//   out[i + j*ldo] = s * exp(-sum_k beta_k (XA[i,k] - XB[j,k])^2) + delta*(i==j && diag)
// Work unit = one output column segment of a 64-row tile: 64 rows (lane = row, so a wave
// stores 512 contiguous bytes per unit) x 1 column.  The units of the whole job (every problem
// of the batch; the tiles on and below the diagonal only for a lower-triangle Gram) are cut into
// one contiguous range per wave of a grid sized to the chip's residency, so every wave runs the
// same number of units (+-1) in ONE residency round (the 64 x 64-tile grid it replaces put 2080
// blocks on 1792 block slots at n = 4096: a second round for 288 blocks doubled the kernel).
// Per range, a wave stages the design vectors of its next 64 / (D/8) columns through LDS (one
// lane-linear load, then wave-uniform broadcast reads: the "d-tile"), keeps its row's design
// vector and beta in registers, and walks its units in order, reloading them only when the
// (problem, row tile) changes.
//
// The weighted distance is taken on design vectors pre-scaled by sqrt(beta) (the row vector in
// registers and the staged d-tile, once per problem / segment): sum_k (a'_k - b'_k)^2 with
// a' = sqrt(beta) a costs 2 d ops per element instead of 3 d (beta >= 0, the ARD precisions);
// the rounding of the scaled values adds at most ~2 eps s to an element (|x| <= 1, beta <= 5),
// inside the 8 eps s Gram tolerance.
// Roofline: 8 B written per output element + 8 d B read per row/column vector (amortised),
// and per element ~37 fp64 VALU ops (2 d for the distance, 19 for exp_neg, the store
// address).  At n = 4096 (lower triangle, 133k column units of 64 elements) the stores
// alone take 12.3 us (5.5 TB/s) and the arithmetic alone 17 us in tools/dbg/gram_micro.hip:
// the kernel is bound by the fp64 VALU pipe, not by HBM (profiles/r02/gram_micro.txt).
#include "gpfit_common.h"
#include "gpfit_profile.h"
#include "gpfit_internal.h"
#include "../../include/gpfit.h"

namespace {

constexpr int kTile = 64;        // rows per unit (lane = row) and columns per tile
constexpr int kWaves = 4;        // waves per block


struct GramShape {
  int TR, TC;                    // tiles down / across
  int tiles;                     // tiles per problem (lower: TR (TR + 1) / 2)
  int units;                     // tiles * 64 per problem
  bool lower;
};

// Tile t of a problem -> (ti, tj); lower: t enumerates tj <= ti row by row.
GP_DEV void tile_of(const GramShape& g, int t, int& ti, int& tj) {
  if (g.lower) {
    int r = (int)((sqrt(8.0 * (double)t + 1.0) - 1.0) * 0.5);
    while (r * (r + 1) / 2 > t) --r;
    while ((r + 1) * (r + 2) / 2 <= t) ++r;
    ti = r;
    tj = t - r * (r + 1) / 2;
  } else {
    ti = t / g.TC;
    tj = t - ti * g.TC;
  }
}

template <int D>
__global__ __launch_bounds__(256) void ardse_kernel(
    const double* __restrict__ XA, int na, int ldxa,      // row points (output rows)
    const double* __restrict__ XB, int nb, int ldxb,      // column points (output columns)
    int d, const double* __restrict__ beta, int ldbeta,
    const double* __restrict__ s, const double* __restrict__ delta,
    double* __restrict__ out, int ldo, long long stride_o,
    int rows_out, int cols_out, GramShape g, int total) {
  __shared__ __attribute__((aligned(16))) double xs_all[kWaves][kTile * D];
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  double* xs = xs_all[w];
  const long long nw = (long long)gridDim.x * kWaves;
  const long long gw = (long long)blockIdx.x * kWaves + w;
  int u = (int)(total * gw / nw);
  const int u1 = (int)(total * (gw + 1) / nw);
  int cur_b = -1, cur_ti = -1;
  double xa[D], sq[D], sb = 0.0, db = 0.0;
#pragma unroll
  for (int k = 0; k < D; ++k) sq[k] = 0.0;
  while (u < u1) {
    // one segment: units u .. u + len - 1 share the problem b and the tile (ti, tj)
    const int b = u / g.units;
    const int rem = u - b * g.units;
    const int t = rem / kTile, c0 = rem - t * kTile;
    const int len = min(kTile - c0, u1 - u);
    int ti, tj;
    tile_of(g, t, ti, tj);
    // every load of the segment is issued before any of them is used: the row vector (on a
    // row-tile change), the d-tile's column vectors, and beta / s / delta (on a problem change)
    const int j0 = tj * kTile;
    const int jc = j0 + lane;
    const bool cok = lane >= c0 && lane < c0 + len && jc < nb;
    const double* src = XB + (long long)(cok ? jc : 0) * ldxb;
    double xb_raw[D];
#pragma unroll
    for (int k = 0; k < D; ++k) xb_raw[k] = (cok && k < d) ? src[k] : 0.0;
    const bool new_b = b != cur_b, new_row = new_b || ti != cur_ti;
    if (new_row) {
      const int ic = min(ti * kTile + lane, na - 1);
#pragma unroll
      for (int k = 0; k < D; ++k) xa[k] = k < d ? XA[(long long)ic * ldxa + k] : 0.0;
    }
    if (new_b) {
      // sqrt(beta) of problem b: lane k takes beta_k's root (one root per lane, in parallel),
      // then each is broadcast to the wave through SGPRs
      const double bl = lane < d ? beta[(long long)b * ldbeta + lane] : 0.0;
      const double rl = __builtin_sqrt(bl);               // NaN for a negative beta
#pragma unroll
      for (int k = 0; k < D; ++k) sq[k] = readlane_f64(rl, k);
      sb = s[b];
      db = delta ? delta[b] : 0.0;
    }
    if (new_row) {
#pragma unroll
      for (int k = 0; k < D; ++k) xa[k] *= sq[k];
      cur_b = b;
      cur_ti = ti;
    }
    // the d-tile: lane l stages column tj*64 + l's scaled design vector, read back as
    // broadcasts
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int k = 0; k < D; ++k) xs[lane * D + k] = xb_raw[k] * sq[k];
    __builtin_amdgcn_wave_barrier();
    const int i = ti * kTile + lane;
    const int cend = min(c0 + len, cols_out - j0);      // columns this segment stores
    double* o = out + (long long)b * stride_o + i;
    // interior segment (every row and column valid, strictly below the diagonal of a lower
    // Gram or off the diagonal tile, no jitter term): no per-element selects or store masks
    const bool interior = ti * kTile + kTile <= min(na, rows_out) && j0 + cend <= nb &&
                          (g.lower ? tj < ti : (ti != tj || !delta));
    if (interior) {
      for (int c = c0; c < cend; ++c) {
        const double* xb = xs + c * D;                   // wave-uniform: broadcast reads
        double acc = 0.0;
#pragma unroll
        for (int k = 0; k < D; ++k) {
          const double dt = xa[k] - xb[k];
          acc = fma(dt, dt, acc);
        }
        o[(long long)(j0 + c) * ldo] = sb * exp_neg(acc);
      }
    } else {
      const bool row_ok = i < na, row_st = i < rows_out;
      for (int c = c0; c < cend; ++c) {
        const int j = j0 + c;
        const double* xb = xs + c * D;
        double acc = 0.0;
#pragma unroll
        for (int k = 0; k < D; ++k) {
          const double dt = xa[k] - xb[k];
          acc = fma(dt, dt, acc);
        }
        double v = fma(sb, exp_neg(acc), (i == j) ? db : 0.0);
        v = (row_ok && j < nb) ? v : 0.0;
        if (row_st && (!g.lower || j <= i)) o[(long long)j * ldo] = v;
      }
    }
    u += len;
  }
}

template <int D>
int ardse_blocks_per_cu() {
  static const int occ = [] {
    int nb = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, ardse_kernel<D>, 256, 0) !=
            hipSuccess || nb <= 0)
      nb = 4;
    return nb;
  }();
  return occ;
}

int gram_num_cus() {
  static const int ncu = [] {
    int dev = 0, n = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
        n <= 0)
      n = 256;
    return n;
  }();
  return ncu;
}

template <int D>
hipError_t launch_ardse(const double* XA, int na, int ldxa, const double* XB, int nb, int ldxb,
                        int d, const double* beta, int ldbeta, const double* s,
                        const double* delta, double* out, int ldo, long long stride_o,
                        int rows_out, int cols_out, int batch, bool lower, hipStream_t st) {
  GramShape g;
  g.TR = gp_ceil_div(rows_out, kTile);
  g.TC = gp_ceil_div(cols_out, kTile);
  g.lower = lower;
  const long long tiles = lower ? (long long)g.TR * (g.TR + 1) / 2 : (long long)g.TR * g.TC;
  const long long total = tiles * kTile * batch;
  if (total >= (1LL << 31)) return hipErrorInvalidValue;   // > 16 G output elements
  g.tiles = (int)tiles;
  g.units = (int)(tiles * kTile);
  // one residency round: every wave of the grid is resident at once (or the grid is smaller
  // than that, when there are fewer than ~8 units per wave)
  const long long cap = (long long)gram_num_cus() * ardse_blocks_per_cu<D>();
  const long long want = gp_ceil_div(total, 8LL * kWaves);
  const int grid = (int)(want < cap ? want : cap);
  hipLaunchKernelGGL((ardse_kernel<D>), dim3(grid), dim3(256), 0, st, XA, na, ldxa, XB, nb, ldxb,
                     d, beta, ldbeta, s, delta, out, ldo, stride_o, rows_out, cols_out, g,
                     (int)total);
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
