// Fit-side dense kernels (fp64): general MFMA GEMM with split-K, column statistics and
// elementwise standardisation.  They implement the non-GP arithmetic of the drop-in surface:
//   src/svd.py:52-64   Y = X Omega, (X X^T) Y, Q^T X, U = Q U_B      (randomized SVD, A2)
//   src/model.py:60-72 mu = mean(Y, 0), sd = std(Y, ddof=1, 0) floored, Y_std      (A1)
//   src/model.py:101, 219-223  K = diag(S) Vh / sqrt(n), w = Y_std pinv(K)           (A3, A4)
//   SepiaEmulatorPrediction.get_y(): y = (w K) sd + mu                              (A9)
// GEMM: 64x64 output tiles, 256 threads = 4 waves (2x2 of 32x32, v_mfma_f64_16x16x4_f64),
// K staged through LDS 64 at a time with operand transposition folded into the staging;
// split-K over grid.z writes partial slabs that a second kernel reduces deterministically
// (no atomics), so X X^T with K = 1.35M still fills all 256 CUs.
#include "gpfit_common.h"
#include "../../include/gpfit.h"

namespace {

constexpr int TB = 64;
constexpr int TP = TB + 1;

// Operand staging of one 64 x 64 K-step: S[k][x] = op(M)(x, k) for the block at (x0, k0);
// NAT: M[x + k*ld], TRN: M[k + x*ld].  Thread slot q reads element (fast, slow) = (g & 63,
// g >> 6), g = tid + 256 q, so a wave reads 64 consecutive elements of memory; the element type
// E (double, or float widened exactly on load -- the fit's float32 ensembles are read as
// stored, without an fp64 copy) only changes the load.  Split in two phases so the next
// K-step's loads are in flight while the current one's MFMAs run.
template <bool TRN, typename E>
GP_DEV void stage_load(double (&r)[16], const E* __restrict__ M, int ld, int x0, int xmax,
                       int k0, int kmax) {
#pragma unroll
  for (int q = 0; q < 16; ++q) {
    const int g = threadIdx.x + 256 * q;
    const int fast = g & (TB - 1), slow = g >> 6;
    int x, k;
    if (!TRN) { x = fast; k = slow; } else { k = fast; x = slow; }
    const int gx = x0 + x, gk = k0 + k;
    r[q] = (gx < xmax && gk < kmax)
               ? static_cast<double>(TRN ? M[gk + (long long)gx * ld] : M[gx + (long long)gk * ld])
               : 0.0;
  }
}

template <bool TRN>
GP_DEV void stage_store(double* S, const double (&r)[16]) {
#pragma unroll
  for (int q = 0; q < 16; ++q) {
    const int g = threadIdx.x + 256 * q;
    const int fast = g & (TB - 1), slow = g >> 6;
    const int x = TRN ? slow : fast, k = TRN ? fast : slow;
    S[k * TP + x] = r[q];
  }
}

// opA(i,k): transa=0 -> A[i + k*lda] (NAT staging), 1 -> A[k + i*lda] (TRN staging)
// opB(k,j): transb=0 -> B[k + j*ldb] (TRN staging), 1 -> B[j + k*ldb] (NAT staging)
template <int TA, int TBT, typename EA, typename EB>
__global__ __launch_bounds__(256) void gemm_kernel(int M, int N, int K, int kchunk,
                                                   const EA* __restrict__ A, int lda,
                                                   const EB* __restrict__ B, int ldb,
                                                   double alpha, double beta,
                                                   double* __restrict__ C, int ldc,
                                                   double* __restrict__ part) {
  __shared__ double As[TB * TP];
  __shared__ double Bs[TB * TP];
  const int tilesM = gp_ceil_div(M, TB);
  const int ti = blockIdx.x % tilesM, tj = blockIdx.x / tilesM;
  const int i0 = ti * TB, j0 = tj * TB;
  const int kb = blockIdx.z * kchunk, ke = min(K, kb + kchunk);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int wr = w >> 1, wc = w & 1, li = lane & 15, lk = lane >> 4;
  f64x4 acc[2][2];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b) acc[a][b] = zero4();
  double ra[16], rb[16];
  if (kb < ke) {
    stage_load<TA != 0>(ra, A, lda, i0, M, kb, ke);
    stage_load<TBT == 0>(rb, B, ldb, j0, N, kb, ke);
  }
  for (int k0 = kb; k0 < ke; k0 += TB) {
    stage_store<TA != 0>(As, ra);
    stage_store<TBT == 0>(Bs, rb);
    __syncthreads();
    if (k0 + TB < ke) {          // the next K-step's operands, in flight under the MFMAs
      stage_load<TA != 0>(ra, A, lda, i0, M, k0 + TB, ke);
      stage_load<TBT == 0>(rb, B, ldb, j0, N, k0 + TB, ke);
    }
#pragma unroll 4
    for (int k4 = 0; k4 < TB / 4; ++k4) {
      const int k = k4 * 4 + lk;
      const double a0 = As[k * TP + wr * 32 + li], a1 = As[k * TP + wr * 32 + 16 + li];
      const double b0 = Bs[k * TP + wc * 32 + li], b1 = Bs[k * TP + wc * 32 + 16 + li];
      acc[0][0] = mfma16x16x4(a0, b0, acc[0][0]);
      acc[0][1] = mfma16x16x4(a0, b1, acc[0][1]);
      acc[1][0] = mfma16x16x4(a1, b0, acc[1][0]);
      acc[1][1] = mfma16x16x4(a1, b1, acc[1][1]);
    }
    __syncthreads();
  }
  // transpose through LDS for coalesced column-major stores
#pragma unroll
  for (int mi = 0; mi < 2; ++mi)
#pragma unroll
    for (int nj = 0; nj < 2; ++nj)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = wr * 32 + mi * 16 + lk + 4 * r, col = wc * 32 + nj * 16 + li;
        As[col * TP + row] = acc[mi][nj][r];
      }
  __syncthreads();
  for (int g = threadIdx.x; g < TB * TB; g += 256) {
    const int row = g & (TB - 1), col = g >> 6;
    const int gi = i0 + row, gj = j0 + col;
    if (gi >= M || gj >= N) continue;
    const double v = As[col * TP + row];
    if (part) {
      part[(long long)blockIdx.z * M * N + gi + (long long)gj * M] = v;
    } else {
      double* c = C + gi + (long long)gj * ldc;
      *c = (beta == 0.0) ? alpha * v : fma(alpha, v, beta * *c);
    }
  }
}

__global__ void splitk_reduce_kernel(const double* __restrict__ part, int splits, int M, int N,
                                     double alpha, double beta, double* __restrict__ C,
                                     int ldc) {
  const long long idx = (long long)blockIdx.x * 256 + threadIdx.x;
  if (idx >= (long long)M * N) return;
  const int gi = (int)(idx % M), gj = (int)(idx / M);
  double s = 0.0;
  for (int p = 0; p < splits; ++p) s += part[(long long)p * M * N + idx];
  double* c = C + gi + (long long)gj * ldc;
  *c = (beta == 0.0) ? alpha * s : fma(alpha, s, beta * *c);
}

// The tsk products' reduction (hundreds of slices over a small C: 256 x 512 x 25 at the fit):
// 32 outputs x 8 slice groups per block, group h summing its contiguous run of slices in order
// with eight loads in flight, then the eight group sums added in group order (a fixed order:
// deterministic).  splitk_reduce_kernel's thread per output summed 256 slices one load at a
// time on 50 CUs: 74 us per product (profiles/r05/r05_pmc_ts.txt).
constexpr int kRedGroups = 8;
__global__ __launch_bounds__(256) void splitk_reduce_wide_kernel(
    const double* __restrict__ part, int splits, int M, int N, double alpha, double beta,
    double* __restrict__ C, int ldc) {
  __shared__ double red[kRedGroups][33];
  const int o = threadIdx.x & 31, h = threadIdx.x >> 5;
  const long long MN = (long long)M * N;
  const long long idx = (long long)blockIdx.x * 32 + o;
  const int per = (splits + kRedGroups - 1) / kRedGroups;
  const int p0 = min(splits, h * per), p1 = min(splits, p0 + per);
  double s = 0.0;
  if (idx < MN) {
    const double* q = part + idx;
#pragma unroll 8
    for (int p = p0; p < p1; ++p) s += q[(long long)p * MN];
  }
  red[h][o] = s;
  __syncthreads();
  if (h == 0 && idx < MN) {
    double t = red[0][o];
#pragma unroll
    for (int g = 1; g < kRedGroups; ++g) t += red[g][o];
    const int gi = (int)(idx % M), gj = (int)(idx / M);
    double* c = C + gi + (long long)gj * ldc;
    *c = (beta == 0.0) ? alpha * t : fma(alpha, t, beta * *c);
  }
}

int choose_splits(int M, int N, int K) {
  const int tiles = gp_ceil_div(M, TB) * gp_ceil_div(N, TB);
  int s = 1;
  while (tiles * s < 512 && K / (s * 2) >= 256) s *= 2;
  return s;
}

// Per-location statistics over simulations of a C-order ensemble Y (n sims x ny locations,
// row stride ldy) — src/model.py:60-64: mu = mean(Y, 0), sd = std(Y, ddof=1, 0) floored at
// sd_floor.  Thread per location: each sweep over the n rows reads 256 consecutive locations
// per block row (coalesced); two passes (mean, then centred sum of squares) as numpy does.
__global__ __launch_bounds__(256) void simstats_kernel(const double* __restrict__ Y, int n,
                                                       int ny, long long ldy, double sd_floor,
                                                       double* __restrict__ mu,
                                                       double* __restrict__ sd) {
  const int c = blockIdx.x * 256 + threadIdx.x;
  if (c >= ny) return;
  double s = 0.0;
  for (int r = 0; r < n; ++r) s += Y[(long long)r * ldy + c];
  const double mean = s / n;
  double q = 0.0;
  for (int r = 0; r < n; ++r) {
    const double t = Y[(long long)r * ldy + c] - mean;
    q = fma(t, t, q);
  }
  double v = sqrt(q / (n > 1 ? n - 1 : 1));
  if (v < sd_floor) v = sd_floor;
  mu[c] = mean;
  sd[c] = v;
}

// The same statistics for a short field (ny below kSimStatsSplitNy: a thread per location would
// leave most CUs idle -- 40 blocks at C5's 10k nodes took 252 us, profiles/r06/
// r06b_c5_kernel_stats.csv): 64 locations per block, the rows in four consecutive quarters
// summed by four thread groups, the quarter sums added in quarter order (a fixed order:
// deterministic), for the mean and then the centred sum of squares.
constexpr int kSimStatsSplitNy = 1 << 16;
__global__ __launch_bounds__(256) void simstats_split_kernel(const double* __restrict__ Y, int n,
                                                             int ny, long long ldy,
                                                             double sd_floor,
                                                             double* __restrict__ mu,
                                                             double* __restrict__ sd) {
  __shared__ double part[4][64];
  const int cl = threadIdx.x & 63, g = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + cl;
  const int q = (n + 3) / 4, r0 = min(n, g * q), r1 = min(n, r0 + q);
  const double* y = Y + (c < ny ? c : 0);
  double s = 0.0;
  if (c < ny)
    for (int r = r0; r < r1; ++r) s += y[(long long)r * ldy];
  part[g][cl] = s;
  __syncthreads();
  const double mean = (((part[0][cl] + part[1][cl]) + part[2][cl]) + part[3][cl]) / n;
  __syncthreads();
  double t2 = 0.0;
  if (c < ny)
    for (int r = r0; r < r1; ++r) {
      const double t = y[(long long)r * ldy] - mean;
      t2 = fma(t, t, t2);
    }
  part[g][cl] = t2;
  __syncthreads();
  if (g == 0 && c < ny) {
    const double qs = ((part[0][cl] + part[1][cl]) + part[2][cl]) + part[3][cl];
    double v = sqrt(qs / (n > 1 ? n - 1 : 1));
    if (v < sd_floor) v = sd_floor;
    mu[c] = mean;
    sd[c] = v;
  }
}

// out[r*ldo + c] = (Y[r*ldy + c] - mu[c]) / sd[c]   (inverse = 0, src/model.py:72)
// out[r*ldo + c] =  Y[r*ldy + c] * sd[c] + mu[c]    (inverse = 1, get_y's back-transform)
__global__ void standardize_kernel(const double* __restrict__ Y, int n, int ny, long long ldy,
                                   const double* __restrict__ mu, const double* __restrict__ sd,
                                   double* __restrict__ out, long long ldo, int inverse) {
  const long long idx = (long long)blockIdx.x * 256 + threadIdx.x;
  if (idx >= (long long)n * ny) return;
  const int r = (int)(idx / ny), c = (int)(idx % ny);
  const double y = Y[(long long)r * ldy + c];
  out[(long long)r * ldo + c] = inverse ? fma(y, sd[c], mu[c]) : (y - mu[c]) / sd[c];
}

// A[i][i] += factor * trace(A) — the shift of shifted CholeskyQR (one block).
__global__ __launch_bounds__(256) void shift_diag_kernel(double* __restrict__ A, int r, int lda,
                                                         double factor) {
  __shared__ double red[4];
  double t = 0.0;
  for (int i = threadIdx.x; i < r; i += 256) t += A[i + (long long)i * lda];
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) t += __shfl_xor(t, o, 64);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = t;
  __syncthreads();
  const double tr = (red[0] + red[1]) + (red[2] + red[3]);
  for (int i = threadIdx.x; i < r; i += 256) A[i + (long long)i * lda] += factor * tr;
}

// scale row i of a column-major (rows x cols) matrix by f[i] (or 1/f[i] when inv=1, 0 if f=0)
__global__ void rowscale_kernel(double* __restrict__ M, int rows, int cols, int ld,
                                const double* __restrict__ f, int inv) {
  const long long idx = (long long)blockIdx.x * 256 + threadIdx.x;
  if (idx >= (long long)rows * cols) return;
  const int i = (int)(idx % rows), j = (int)(idx / rows);
  const double fi = f[i];
  const double g = inv ? (fi != 0.0 ? 1.0 / fi : 0.0) : fi;
  M[i + (long long)j * ld] *= g;
}

// Two-pass mean / variance of a long vector: grid-stride partial sums into work[blocks], one
// block reduces them; the second pass is centred (as numpy's var).
constexpr int kMVBlocks = 1024;
__global__ __launch_bounds__(256) void partial_sum_kernel(const double* __restrict__ x,
                                                          long long N,
                                                          const double* __restrict__ center,
                                                          double* __restrict__ work) {
  __shared__ double red[4];
  const double c = center ? center[0] : 0.0;
  double s = 0.0;
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < N;
       i += (long long)gridDim.x * 256) {
    const double t = x[i] - c;
    s += center ? t * t : t;
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) work[blockIdx.x] = (red[0] + red[1]) + (red[2] + red[3]);
}

__global__ __launch_bounds__(256) void finish_sum_kernel(const double* __restrict__ work,
                                                         int nb, double scale,
                                                         double* __restrict__ out) {
  __shared__ double red[4];
  double s = 0.0;
  for (int i = threadIdx.x; i < nb; i += 256) s += work[i];
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) out[0] = ((red[0] + red[1]) + (red[2] + red[3])) * scale;
}

}  // namespace

extern "C" int gp_mean_var(const double* x, long long N, int ddof, double* out, double* work,
                           hipStream_t stream) {
  if (!x) return -1;
  if (N < 1) return -2;
  if (ddof < 0 || ddof >= N) return -3;
  if (!out) return -4;
  if (!work) return -5;
  const int nb = (int)((N + 255) / 256 < kMVBlocks ? (N + 255) / 256 : kMVBlocks);
  hipLaunchKernelGGL(partial_sum_kernel, dim3(nb), dim3(256), 0, stream, x, N, nullptr, work);
  hipLaunchKernelGGL(finish_sum_kernel, dim3(1), dim3(256), 0, stream, work, nb, 1.0 / N, out);
  hipLaunchKernelGGL(partial_sum_kernel, dim3(nb), dim3(256), 0, stream, x, N, out, work);
  hipLaunchKernelGGL(finish_sum_kernel, dim3(1), dim3(256), 0, stream, work, nb,
                     1.0 / (double)(N - ddof), out + 1);
  hipError_t e = hipGetLastError();
  return e == hipSuccess ? 0 : GPFIT_ERR_HIP - (int)e;
}

extern "C" int gp_shift_diag(double* A, int r, int lda, double factor, hipStream_t stream) {
  if (!A) return -1;
  if (r < 0) return -2;
  if (lda < r || lda < 1) return -3;
  if (r == 0) return 0;
  hipLaunchKernelGGL(shift_diag_kernel, dim3(1), dim3(256), 0, stream, A, r, lda, factor);
  hipError_t e = hipGetLastError();
  return e == hipSuccess ? 0 : GPFIT_ERR_HIP - (int)e;
}

extern "C" int gp_rowscale(double* M, int rows, int cols, int ld, const double* f, int inv,
                           hipStream_t stream) {
  if (!M) return -1;
  if (rows < 0) return -2;
  if (cols < 0) return -3;
  if (ld < rows || ld < 1) return -4;
  if (!f) return -5;
  if (rows == 0 || cols == 0) return 0;
  const long long tot = (long long)rows * cols;
  hipLaunchKernelGGL(rowscale_kernel, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, stream,
                     M, rows, cols, ld, f, inv);
  hipError_t e = hipGetLastError();
  return e == hipSuccess ? 0 : GPFIT_ERR_HIP - (int)e;
}

namespace {

// ---- Tall-skinny products of the randomized SVD (src/svd.py:52-64 at the fit's shapes) ------
// The four products that stream the ensemble X (n_sims x ny, C-order: ny = 1,347,945 at the
// fit's 512 runs) against r = p + k <= 32 test vectors read X once each and are HBM-bound
// (5.5 GB in fp64; their fp64 MFMA time at r padded to 32 is ~0.6 ms, the read ~0.9 ms at
// 6 TB/s).  The 64 x 64-tile GEMM above reached 0.20-0.35 of HBM on them (r = 25 of 64 tile
// columns, one K-step of staging in flight: profiles/r04/r04k_prof_pca.log).  Two kernels keep
// the narrow side in registers / L2 and stream X with many loads in flight:
//   tsk (C = X W, K = ny long, C small): every block owns one K-slice of kTskRows rows, each
//       wave 64 rows (4 row tiles x 2 column tiles of 16 in MFMA accumulators).  X is loaded
//       row-contiguous (8 lanes read 8 consecutive k of one row: 64 B per row, 8 rows per
//       load), three K-groups ahead in registers, and transposed into the MFMA A layout through
//       a wave-private LDS tile; partial C per slice, then splitk_reduce_wide_kernel (fixed order:
//       deterministic).  (Round 5's first tsk loaded X straight into the A layout -- 16 rows x
//       32 B per load -- and reached 0.19-0.25 of HBM: profiles/r05/r05g_prof_pca.log.)
//   tsm (C = X^T Y or Q^T X, the big side is the output): every block owns kTsmRows rows of the
//       big dimension and the whole K <= kTsmMaxK (the narrow operand read through L1 / L2),
//       two blocks per CU; the accumulators go through LDS so the output is written as
//       contiguous runs.
// The operands' element types are template parameters (float32 X read as stored and widened
// exactly, as the general kernel does), so float32 and fp64 operands give the same bits.
#ifndef TSK_WAVES
#define TSK_WAVES 4
#endif
constexpr int kTskWaves = TSK_WAVES;           // waves per tsk block, 64 rows each
constexpr int kTskRows = 64 * kTskWaves;       // rows of C per tsk block
constexpr int kTskMinK = 1 << 16;
// 256 rows (4 waves x 64) at two blocks per CU: 0.53-0.56 of HBM on the fit's products, against
// 0.42-0.47 at 128 x 3, 0.29-0.31 at 64 x 4, 0.48-0.49 at 512 x 1 (profiles/r05/r05w_tsm*.log)
#ifndef TSM_ROWS
#define TSM_ROWS 256
#endif
#ifndef TSM_OCC
#define TSM_OCC 2
#endif
constexpr int kTsmRows = TSM_ROWS;   // rows of the big dimension per tsm block
constexpr int kTsmMaxK = 1024;   // K of a tsm product (the number of runs)
constexpr int kTsMaxN = 32;          // narrow side (two 16-wide MFMA column tiles)

// K-groups (16 k each) in flight ahead of the one being multiplied (a ring of kTsRing register
// buffers, indexed at compile time: the loops below are unrolled over the ring)
constexpr int kTsRing = 3;    // tsm
constexpr int kTskKG = 8;     // tsk: k per group (8 lanes read 64 contiguous bytes of a row)
constexpr int kTskRing = 4;   // tsk: groups in registers, three in flight ahead
constexpr int kTskPitch = 72; // tsk LDS transpose: doubles per k row of a wave's 64-row tile

// C(i, j) = sum_k P(i, k) W(k, j) for i < M (P(i,k) = P[k + i*ldp], contiguous in k), j < N <= 32,
// W(k, j) = W[k*wk + j*wj], k in this block's slice; partial C to part[slice][j*M + i].
template <typename EP, typename EW>
__global__ __launch_bounds__(64 * kTskWaves, 8 / kTskWaves) void gemm_tsk_kernel(int M, int N, int K, int kslice,
                                                          const EP* __restrict__ P, int ldp,
                                                          const EW* __restrict__ W, long long wk,
                                                          long long wj, double* __restrict__ part) {
  constexpr int G = kTskKG, R = kTskRing, NQ = 64 * G / 64;   // NQ loads of one group per lane
  __shared__ double xs[kTskWaves * G * kTskPitch];
  const int slice = blockIdx.x, rg = blockIdx.y;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int li = lane & 15, ks = lane >> 4;
  const int kk = lane % G, rr = lane / G;                // load slot: k offset, row offset
  const int kb = slice * kslice, ke = min(K, kb + kslice);
  const int row0 = rg * kTskRows + w * 64;
  double* xw = xs + w * G * kTskPitch;
  f64x4 acc[4][2];
#pragma unroll
  for (int t = 0; t < 4; ++t) acc[t][0] = acc[t][1] = zero4();
  // load q of a group: row row0 + (64 / G) q + rr, k = k0 + kk; rows >= M masked (never read)
  constexpr int RS = 64 / G;
  const EP* lrow = P + (long long)(row0 + rr) * ldp + kk;
  const long long qstep = (long long)RS * ldp;
  const int jc0 = li, jc1 = 16 + li;
  // FULL: the unmasked fast path of tsk16 / tsm (rows < M, whole groups; same bits)
  const int jc0c = jc0 < N ? jc0 : N - 1, jc1c = jc1 < N ? jc1 : N - 1;   // N < 16 too
  const EW* const wc0 = W + jc0c * wj;
  const EW* const wc1 = W + jc1c * wj;
  const long long wk4 = 4LL * wk;
  double xr[R][NQ], bv[R][G / 4][2];
  auto run = [&](auto fullc) {
    constexpr bool FULL = decltype(fullc)::value;
    auto load = [&](double (&xb)[NQ], double (&bb)[G / 4][2], int k0) {
      if constexpr (FULL) {
        const EP* lk = lrow + k0;
#pragma unroll
        for (int q = 0; q < NQ; ++q) xb[q] = static_cast<double>(lk[q * qstep]);
        const long long wo = (long long)(k0 + ks) * wk;
#pragma unroll
        for (int u = 0; u < G / 4; ++u) {
          bb[u][0] = static_cast<double>(wc0[wo + u * wk4]);
          bb[u][1] = static_cast<double>(wc1[wo + u * wk4]);
        }
      } else {
        const bool kok = k0 + kk < ke;
#pragma unroll
        for (int q = 0; q < NQ; ++q)
          xb[q] = (kok && row0 + RS * q + rr < M) ? static_cast<double>(lrow[q * qstep + k0])
                                                   : 0.0;
#pragma unroll
        for (int u = 0; u < G / 4; ++u) {
          const int k = k0 + 4 * u + ks;
          const bool ok = k < ke;
          bb[u][0] = (ok && jc0 < N) ? static_cast<double>(W[k * wk + jc0 * wj]) : 0.0;
          bb[u][1] = (ok && jc1 < N) ? static_cast<double>(W[k * wk + jc1 * wj]) : 0.0;
        }
      }
    };
    // prologue: only groups inside the slice (FULL loads are unmasked: a group at or past ke
    // would read up to 16 k past the slice, i.e. past X's last row and W's last k)
#pragma unroll
    for (int q = 0; q < R - 1; ++q)
      if (kb + G * q < ke) load(xr[q], bv[q], kb + G * q);
    for (int k0 = kb; k0 < ke; k0 += G * R) {
#pragma unroll
      for (int q = 0; q < R; ++q) {
        const int kq = k0 + G * q;
        if (kq >= ke) break;
        const int kn = kq + G * (R - 1);                    // the group R - 1 ahead
        if (kn < ke) load(xr[(q + R - 1) % R], bv[(q + R - 1) % R], kn);
        // transpose: xw[k][row] (one wave's LDS: its own DS instructions run in order)
#pragma unroll
        for (int i = 0; i < NQ; ++i) xw[kk * kTskPitch + RS * i + rr] = xr[q][i];
#pragma unroll
        for (int u = 0; u < G / 4; ++u) {
          double a[4];
#pragma unroll
          for (int t = 0; t < 4; ++t) a[t] = xw[(4 * u + ks) * kTskPitch + 16 * t + li];
#pragma unroll
          for (int t = 0; t < 4; ++t) {
            acc[t][0] = mfma16x16x4(a[t], bv[q][u][0], acc[t][0]);
            acc[t][1] = mfma16x16x4(a[t], bv[q][u][1], acc[t][1]);
          }
        }
      }
    }
  };
  if (rg * kTskRows + kTskRows <= M && (ke - kb) % G == 0) run(std::true_type{});
  else run(std::false_type{});
  // C layout: lane l, reg q holds C[(l >> 4) + 4q][l & 15] of each 16 x 16 tile
  double* pp = part + (long long)slice * M * N;
#pragma unroll
  for (int t = 0; t < 4; ++t)
#pragma unroll
    for (int jt = 0; jt < 2; ++jt)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int r = row0 + 16 * t + ks + 4 * q, j = 16 * jt + li;
        if (r < M && j < N) pp[(long long)j * M + r] = acc[t][jt][q];
      }
}

// C(i, j) = alpha sum_k P(i, k) Q(k, j) + beta C(i, j) for i < M (P(i,k) = P[i + k*ldp],
// contiguous in i), j < N <= 32, k < K <= kTsmMaxK, Q(k, j) = Q[k*qk + j*qj] (read through L1 /
// L2: 100 KB at the fit's 512 x 25), C(i, j) = C[i*ci + j*cj].  The block's rows are written
// through LDS as runs along whichever of i / j is contiguous in C.
template <typename EP, typename EQ>
__global__ __launch_bounds__(256, TSM_OCC) void gemm_tsm_kernel(int M, int N, int K,
                                                          const EP* __restrict__ P, int ldp,
                                                          const EQ* __restrict__ Q, long long qk,
                                                          long long qj, double alpha,
                                                          double beta, double* __restrict__ C,
                                                          long long ci, long long cj) {
  __shared__ double cs[kTsmRows * 33];            // the block's C rows, pitch 33
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int li = lane & 15, ks = lane >> 4;
  const long long i0 = (long long)blockIdx.x * kTsmRows;
  constexpr int T = kTsmRows / 64;                // row tiles of 16 per wave
  f64x4 acc[T][2];
#pragma unroll
  for (int t = 0; t < T; ++t) acc[t][0] = acc[t][1] = zero4();
  const long long rbase = i0 + w * 16 * T;
  const EP* pcol[T];
  bool rok[T];
#pragma unroll
  for (int t = 0; t < T; ++t) {
    const long long r = rbase + 16 * t + li;
    rok[t] = r < M;
    pcol[t] = P + (rok[t] ? r : 0);
  }
  const int jc0 = li, jc1 = 16 + li;
  // K-group of 16: lane (row li, slot ks) holds k = k0 + 4u + ks of its 4 row tiles.
  // FULL (every block row < M and K % 16 == 0, i.e. all but a product's last block): no
  // per-load masks and one 64-bit address per (group, u) -- the masked form's per-load
  // exec-mask branches and 64-bit multiplies outnumbered its MFMAs (r05_pmc_ts.txt: MFMA busy
  // 0.46 with waves waiting only 19% of their cycles).  Columns >= N then multiply a clamped,
  // finite column of Q into C columns that are never stored; every stored element sums the
  // same products in the same order, so the results are the masked form's bits.
  const int jc0c = jc0 < N ? jc0 : N - 1, jc1c = jc1 < N ? jc1 : N - 1;   // N < 16 too
  const long long ldp4 = 4LL * ldp, qk4 = 4LL * qk;
  const EQ* const qc0 = Q + jc0c * qj;
  const EQ* const qc1 = Q + jc1c * qj;
  double a[kTsRing][T][4], bv[kTsRing][4][2];
  auto run = [&](auto fullc) {
    constexpr bool FULL = decltype(fullc)::value;
    auto load = [&](double (&ab)[T][4], double (&bb)[4][2], int k0) {
      if constexpr (FULL) {
        const EP* pk = P + rbase + li + (long long)(k0 + ks) * ldp;
        const long long qo = (long long)(k0 + ks) * qk;
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const EP* pu = pk + u * ldp4;
#pragma unroll
          for (int t = 0; t < T; ++t) ab[t][u] = static_cast<double>(pu[16 * t]);
          bb[u][0] = static_cast<double>(qc0[qo + u * qk4]);
          bb[u][1] = static_cast<double>(qc1[qo + u * qk4]);
        }
      } else {
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const int k = k0 + 4 * u + ks;
          const bool kok = k < K;
#pragma unroll
          for (int t = 0; t < T; ++t)
            ab[t][u] = (kok && rok[t]) ? static_cast<double>(pcol[t][(long long)k * ldp]) : 0.0;
          bb[u][0] = (kok && jc0 < N) ? static_cast<double>(Q[k * qk + jc0 * qj]) : 0.0;
          bb[u][1] = (kok && jc1 < N) ? static_cast<double>(Q[k * qk + jc1 * qj]) : 0.0;
        }
      }
    };
    // prologue: only groups < K (FULL loads are unmasked; K = 16 would otherwise read P's
    // columns and Q's rows 16..31, past both operands)
#pragma unroll
    for (int q = 0; q < kTsRing - 1; ++q)
      if (16 * q < K) load(a[q], bv[q], 16 * q);
    for (int k0 = 0; k0 < K; k0 += 16 * kTsRing) {
#pragma unroll
      for (int q = 0; q < kTsRing; ++q) {
        const int kq = k0 + 16 * q;
        if (kq >= K) break;
        const int kn = kq + 16 * (kTsRing - 1);
        if (kn < K) load(a[(q + kTsRing - 1) % kTsRing], bv[(q + kTsRing - 1) % kTsRing], kn);
#pragma unroll
        for (int u = 0; u < 4; ++u)
#pragma unroll
          for (int t = 0; t < T; ++t) {
            acc[t][0] = mfma16x16x4(a[q][t][u], bv[q][u][0], acc[t][0]);
            acc[t][1] = mfma16x16x4(a[q][t][u], bv[q][u][1], acc[t][1]);
          }
      }
    }
  };
  if (i0 + kTsmRows <= M && K % 16 == 0) run(std::true_type{});
  else run(std::false_type{});
#pragma unroll
  for (int t = 0; t < T; ++t)
#pragma unroll
    for (int jt = 0; jt < 2; ++jt)
#pragma unroll
      for (int q = 0; q < 4; ++q)
        cs[(w * 16 * T + 16 * t + ks + 4 * q) * 33 + 16 * jt + li] = acc[t][jt][q];
  __syncthreads();
  const int rows = (int)min((long long)kTsmRows, M - i0);
  if (cj == 1) {                                // C(i, j) runs along j: rows of N doubles
    for (int e = threadIdx.x; e < rows * N; e += 256) {
      const int r = e / N, j = e - r * N;
      double* c = C + (i0 + r) * ci + j;
      const double v = alpha * cs[r * 33 + j];
      *c = (beta == 0.0) ? v : fma(beta, *c, v);
    }
  } else {                                      // runs along i: one column at a time
    for (int e = threadIdx.x; e < rows * N; e += 256) {
      const int j = e / rows, r = e - j * rows;
      double* c = C + (i0 + r) * ci + j * cj;
      const double v = alpha * cs[r * 33 + j];
      *c = (beta == 0.0) ? v : fma(beta, *c, v);
    }
  }
}

// ---- 16-byte form for fp64 ensembles whose rows start 16-B aligned (the fit's y_std is
// allocated with a padded row stride, emulator.py standardize_y) -------------------------------
// tsk16: as gemm_tsk_kernel, but 8 lanes read one row's 16 k as 16-B pairs (128 B per row, 8 rows
// per load; 64 B with 8-B loads); X three groups ahead, W two (a 6-group unrolled ring).
constexpr int kTsk16Pitch = 68;

template <typename EW>
__global__ __launch_bounds__(64 * kTskWaves, 8 / kTskWaves) void gemm_tsk16_kernel(int M, int N, int K, int kslice,
                                                            const double* __restrict__ P, int ldp,
                                                            const EW* __restrict__ W, long long wk,
                                                            long long wj,
                                                            double* __restrict__ part) {
  constexpr int G = 16, RX = 3, RW = 2;
  __shared__ double xs[kTskWaves * G * kTsk16Pitch];
  const int slice = blockIdx.x, rg = blockIdx.y;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int li = lane & 15, ks = lane >> 4;
  const int c = lane & 7, rr = lane >> 3;                // load slot: k pair 2c, row offset rr
  const int kb = slice * kslice, ke = min(K, kb + kslice);
  const int row0 = rg * kTskRows + w * 64;
  double* xw = xs + w * G * kTsk16Pitch;
  f64x4 acc[4][2];
#pragma unroll
  for (int t = 0; t < 4; ++t) acc[t][0] = acc[t][1] = zero4();
  const double* lrow = P + (long long)(row0 + rr) * ldp + 2 * c;
  const long long qstep = 8LL * ldp;
  const int jc0 = li, jc1 = 16 + li;
  // FULL (the block's rows < M and its k range whole groups of 16: all but a product's last
  // slice): loads without per-lane masks and one 64-bit multiply per W group, as in tsm
  // (the masked form spent more instructions on exec-mask branches and 64-bit address
  // arithmetic than on MFMAs: profiles/r05/r05_pmc_ts.txt, MFMA busy 0.49).  Columns >= N
  // read a clamped, finite column of W into C columns that are never stored: same bits.
  const int jc0c = jc0 < N ? jc0 : N - 1, jc1c = jc1 < N ? jc1 : N - 1;   // N < 16 too
  const EW* const wc0 = W + jc0c * wj;
  const EW* const wc1 = W + jc1c * wj;
  const long long wk4 = 4LL * wk;
  double2 xr[RX][8];
  double bv[RW][4][2];
  auto run = [&](auto fullc) {
    constexpr bool FULL = decltype(fullc)::value;
    // (k0 + 2c even < ke: the pair's second element is inside the padded row; zeroed past ke)
    auto load_x = [&](double2 (&xb)[8], int k0) {
      if constexpr (FULL) {
        const double* lk = lrow + k0;
#pragma unroll
        for (int q = 0; q < 8; ++q) xb[q] = *reinterpret_cast<const double2*>(lk + q * qstep);
      } else {
        const int k = k0 + 2 * c;
#pragma unroll
        for (int q = 0; q < 8; ++q) {
          double2 v = make_double2(0.0, 0.0);
          if (k < ke && row0 + 8 * q + rr < M)
            v = *reinterpret_cast<const double2*>(lrow + q * qstep + k0);
          if (k + 1 >= ke) v.y = 0.0;
          xb[q] = v;
        }
      }
    };
    auto load_w = [&](double (&bb)[4][2], int k0) {
      if constexpr (FULL) {
        const long long wo = (long long)(k0 + ks) * wk;
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          bb[u][0] = static_cast<double>(wc0[wo + u * wk4]);
          bb[u][1] = static_cast<double>(wc1[wo + u * wk4]);
        }
      } else {
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const int k = k0 + 4 * u + ks;
          const bool ok = k < ke;
          bb[u][0] = (ok && jc0 < N) ? static_cast<double>(W[k * wk + jc0 * wj]) : 0.0;
          bb[u][1] = (ok && jc1 < N) ? static_cast<double>(W[k * wk + jc1 * wj]) : 0.0;
        }
      }
    };
    load_x(xr[0], kb);
    load_w(bv[0], kb);
    if (kb + G < ke) load_x(xr[1], kb + G);      // a 16-long slice has no second group
    for (int k0 = kb; k0 < ke; k0 += G * RX * RW) {
      static_for<0, RX * RW, 1>([&](auto Q) {
        constexpr int q = decltype(Q)::value;
        const int kq = k0 + G * q;
        if (kq >= ke) return;
        if (kq + 2 * G < ke) load_x(xr[(q + 2) % RX], kq + 2 * G);
        if (kq + G < ke) load_w(bv[(q + 1) % RW], kq + G);
        // transpose: xw[k][row] (one wave's LDS: its own DS instructions run in order)
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          xw[(2 * c) * kTsk16Pitch + 8 * i + rr] = xr[q % RX][i].x;
          xw[(2 * c + 1) * kTsk16Pitch + 8 * i + rr] = xr[q % RX][i].y;
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          double a[4];
#pragma unroll
          for (int t = 0; t < 4; ++t) a[t] = xw[(4 * u + ks) * kTsk16Pitch + 16 * t + li];
#pragma unroll
          for (int t = 0; t < 4; ++t) {
            acc[t][0] = mfma16x16x4(a[t], bv[q % RW][u][0], acc[t][0]);
            acc[t][1] = mfma16x16x4(a[t], bv[q % RW][u][1], acc[t][1]);
          }
        }
      });
    }
  };
  if (rg * kTskRows + kTskRows <= M && (ke - kb) % G == 0) run(std::true_type{});
  else run(std::false_type{});
  double* pp = part + (long long)slice * M * N;
#pragma unroll
  for (int t = 0; t < 4; ++t)
#pragma unroll
    for (int jt = 0; jt < 2; ++jt)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int r = row0 + 16 * t + ks + 4 * q, j = 16 * jt + li;
        if (r < M && j < N) pp[(long long)j * M + r] = acc[t][jt][q];
      }
}

// The 16-B form applies to an fp64 big operand with a 16-B aligned base and an even leading
// dimension (a pair never reads past the row: an even ldp >= len rounds len up inside it).
// (A 16-B tsm, each lane reading rows 2i, 2i + 1 of a column, ran 2.4 vs 1.6 ms on the fit's
// products at its occupancy of 2 blocks per CU instead of 3: profiles/r05/r05j_prof_pca.log.)
template <typename E>
bool ts_vec_ok(const E* p, int ld, int len) {
  return sizeof(E) == 8 && (reinterpret_cast<uintptr_t>(p) & 15) == 0 && (ld & 1) == 0 &&
         ld >= ((len + 1) & ~1);
}

// Which tall-skinny kernel serves (transa, transb, m, n, k), if any:
//   1 tsk: transa = 1 (A's columns are C's rows), n <= 32, k >= kTskMinK;
//   2 tsm: transa = 0, n <= 32, k <= kTsmMaxK, m >= 8192 (the big side is C's rows);
//   3 tsm on the transpose: transb = 1, m <= 32, k <= kTsmMaxK, n >= 8192 (C^T's rows).
int ts_kind(int transa, int transb, int m, int n, int k) {
  if (transa == 1 && n <= kTsMaxN && k >= kTskMinK) return 1;
  if (transa == 0 && n <= kTsMaxN && k <= kTsmMaxK && m >= 8192) return 2;
  if (transb == 1 && m <= kTsMaxN && k <= kTsmMaxK && n >= 8192) return 3;
  return 0;
}

// tsk's K slices: eight waves per CU over all row groups, each slice a multiple of 16.
void tsk_shape(int m, int k, int& groups, int& slices, int& kslice) {
  groups = gp_ceil_div(m, kTskRows);
  slices = max(1, (2048 / kTskWaves) / groups);
  kslice = gp_ceil_div(gp_ceil_div(k, slices), 16) * 16;
  slices = gp_ceil_div(k, kslice);
}

}  // namespace

extern "C" long long gp_dgemm_ws_bytes(int m, int n, int k) {
  if (m <= 0 || n <= 0 || k <= 0) return 0;
  const int s = choose_splits(m, n, k);
  long long bytes = s > 1 ? (long long)s * m * n * 8 : 0;
  if (n <= kTsMaxN && k >= kTskMinK) {            // a tsk product (transa = 1)
    int g, sl, kc;
    tsk_shape(m, k, g, sl, kc);
    bytes = max(bytes, (long long)sl * m * n * 8);
  }
  return bytes;
}

namespace {
template <typename EA, typename EB>
hipError_t launch_ts(int kind, int transa, int transb, int m, int n, int k, double alpha,
                            const void* A, int lda, const void* B, int ldb, double beta,
                            double* C, int ldc, double* part, hipStream_t stream) {
  const EA* a = static_cast<const EA*>(A);
  const EB* b = static_cast<const EB*>(B);
  if (kind == 1) {
    int groups, slices, kslice;
    tsk_shape(m, k, groups, slices, kslice);
    // W(k, j) = opB(k, j): transb 0 -> B[k + j*ldb], 1 -> B[j + k*ldb]
    const long long wk = transb ? ldb : 1, wj = transb ? 1 : ldb;
    if constexpr (sizeof(EA) == 8) {
      if (ts_vec_ok(a, lda, k))
        hipLaunchKernelGGL((gemm_tsk16_kernel<EB>), dim3(slices, groups), dim3(64 * kTskWaves), 0, stream,
                           m, n, k, kslice, reinterpret_cast<const double*>(a), lda, b, wk, wj,
                           part);
      else
        hipLaunchKernelGGL((gemm_tsk_kernel<EA, EB>), dim3(slices, groups), dim3(64 * kTskWaves), 0, stream,
                           m, n, k, kslice, a, lda, b, wk, wj, part);
    } else {
      hipLaunchKernelGGL((gemm_tsk_kernel<EA, EB>), dim3(slices, groups), dim3(64 * kTskWaves), 0, stream, m,
                         n, k, kslice, a, lda, b, wk, wj, part);
    }
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    const long long tot = (long long)m * n;
    hipLaunchKernelGGL(splitk_reduce_wide_kernel, dim3((unsigned)((tot + 31) / 32)), dim3(256), 0,
                       stream, part, slices, m, n, alpha, beta, C, ldc);
    return hipGetLastError();
  }
  if (kind == 2) {
    // C(i, j) = sum_k A[i + k*lda] opB(k, j), C[i + j*ldc]
    const long long qk = transb ? ldb : 1, qj = transb ? 1 : ldb;
    hipLaunchKernelGGL((gemm_tsm_kernel<EA, EB>), dim3(gp_ceil_div(m, kTsmRows)), dim3(256), 0,
                       stream, m, n, k, a, lda, b, qk, qj, alpha, beta, C, 1LL, (long long)ldc);
  } else {
    // C^T(j, i) = sum_k B[j + k*ldb] opA(i, k), C[i + j*ldc]: the big operand is B
    const long long qk = transa ? 1 : lda, qj = transa ? lda : 1;
    hipLaunchKernelGGL((gemm_tsm_kernel<EB, EA>), dim3(gp_ceil_div(n, kTsmRows)), dim3(256), 0,
                       stream, n, m, k, b, ldb, a, qk, qj, alpha, beta, C, (long long)ldc, 1LL);
  }
  return hipGetLastError();
}

template <typename EA, typename EB>
static void launch_gemm(int transa, int transb, dim3 grid, hipStream_t stream, int m, int n,
                        int k, int kchunk, const void* A, int lda, const void* B, int ldb,
                        double alpha, double beta, double* C, int ldc, double* part) {
  const EA* a = static_cast<const EA*>(A);
  const EB* b = static_cast<const EB*>(B);
#define GP_GEMM(TA_, TB_)                                                                     \
  hipLaunchKernelGGL((gemm_kernel<TA_, TB_, EA, EB>), grid, dim3(256), 0, stream, m, n, k,     \
                     kchunk, a, lda, b, ldb, alpha, beta, C, ldc, part)
  if (transa == 0 && transb == 0) GP_GEMM(0, 0);
  else if (transa == 0 && transb == 1) GP_GEMM(0, 1);
  else if (transa == 1 && transb == 0) GP_GEMM(1, 0);
  else GP_GEMM(1, 1);
#undef GP_GEMM
}

}  // namespace

extern "C" int gp_gemm_ex(int transa, int transb, int m, int n, int k, double alpha,
                          const void* A, int a_f32, int lda, const void* B, int b_f32, int ldb,
                          double beta, double* C, int ldc, void* ws, long long ws_bytes,
                          hipStream_t stream) {
  if (transa != 0 && transa != 1) return -1;
  if (transb != 0 && transb != 1) return -2;
  if (m < 0) return -3;
  if (n < 0) return -4;
  if (k < 0) return -5;
  if (!A && k > 0) return -7;
  if (a_f32 != 0 && a_f32 != 1) return -8;
  if (lda < (transa ? k : m) || lda < 1) return -9;
  if (!B && k > 0) return -10;
  if (b_f32 != 0 && b_f32 != 1) return -11;
  if (ldb < (transb ? n : k) || ldb < 1) return -12;
  if (!C) return -14;
  if (ldc < m || ldc < 1) return -15;
  if (m == 0 || n == 0) return 0;
  const int tk = (k > 0) ? ts_kind(transa, transb, m, n, k) : 0;
  if (tk) {
    long long need = 0;
    if (tk == 1) {
      int g, sl, kc;
      tsk_shape(m, k, g, sl, kc);
      need = (long long)sl * m * n * 8;
    }
    if (tk != 1 || (ws && ws_bytes >= need)) {
      hipError_t e;
      double* part = static_cast<double*>(ws);
      if (a_f32 && b_f32)
        e = launch_ts<float, float>(tk, transa, transb, m, n, k, alpha, A, lda, B, ldb, beta, C,
                                    ldc, part, stream);
      else if (a_f32)
        e = launch_ts<float, double>(tk, transa, transb, m, n, k, alpha, A, lda, B, ldb, beta, C,
                                     ldc, part, stream);
      else if (b_f32)
        e = launch_ts<double, float>(tk, transa, transb, m, n, k, alpha, A, lda, B, ldb, beta, C,
                                     ldc, part, stream);
      else
        e = launch_ts<double, double>(tk, transa, transb, m, n, k, alpha, A, lda, B, ldb, beta,
                                      C, ldc, part, stream);
      return e == hipSuccess ? 0 : GPFIT_ERR_HIP - (int)e;
    }
  }
  int splits = (k > 0) ? choose_splits(m, n, k) : 1;
  if (splits > 1 && (!ws || ws_bytes < (long long)splits * m * n * 8)) splits = 1;
  const int kchunk = (k > 0) ? gp_ceil_div(gp_ceil_div(k, splits), TB) * TB : TB;
  splits = (k > 0) ? gp_ceil_div(k, kchunk) : 1;
  double* part = (splits > 1) ? static_cast<double*>(ws) : nullptr;
  dim3 grid(gp_ceil_div(m, TB) * gp_ceil_div(n, TB), 1, splits);
  if (a_f32 && b_f32)
    launch_gemm<float, float>(transa, transb, grid, stream, m, n, k, kchunk, A, lda, B, ldb,
                              alpha, beta, C, ldc, part);
  else if (a_f32)
    launch_gemm<float, double>(transa, transb, grid, stream, m, n, k, kchunk, A, lda, B, ldb,
                               alpha, beta, C, ldc, part);
  else if (b_f32)
    launch_gemm<double, float>(transa, transb, grid, stream, m, n, k, kchunk, A, lda, B, ldb,
                               alpha, beta, C, ldc, part);
  else
    launch_gemm<double, double>(transa, transb, grid, stream, m, n, k, kchunk, A, lda, B, ldb,
                                alpha, beta, C, ldc, part);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return GPFIT_ERR_HIP - (int)e;
  if (part) {
    const long long tot = (long long)m * n;
    hipLaunchKernelGGL(splitk_reduce_kernel, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0,
                       stream, part, splits, m, n, alpha, beta, C, ldc);
    e = hipGetLastError();
    if (e != hipSuccess) return GPFIT_ERR_HIP - (int)e;
  }
  return 0;
}

extern "C" int gp_dgemm(int transa, int transb, int m, int n, int k, double alpha,
                        const double* A, int lda, const double* B, int ldb, double beta,
                        double* C, int ldc, void* ws, long long ws_bytes, hipStream_t stream) {
  const int rc = gp_gemm_ex(transa, transb, m, n, k, alpha, A, 0, lda, B, 0, ldb, beta, C, ldc,
                            ws, ws_bytes, stream);
  // keep gp_dgemm's documented argument numbers (A, lda = 7, 8; B, ldb = 9, 10; C, ldc = 12, 13)
  static const int remap[16] = {0, -1, -2, -3, -4, -5, 0, -7, 0, -8, -9, 0, -10, 0, -12, -13};
  return (rc < 0 && rc > -16) ? remap[-rc] : rc;
}

extern "C" int gp_sim_stats(const double* Y, int n, int ny, long long ldy, double sd_floor,
                            double* mu, double* sd, hipStream_t stream) {
  if (!Y) return -1;
  if (n < 1) return -2;
  if (ny < 0) return -3;
  if (ldy < ny) return -4;
  if (!mu) return -6;
  if (!sd) return -7;
  if (ny == 0) return 0;
  if (ny < kSimStatsSplitNy)
    hipLaunchKernelGGL(simstats_split_kernel, dim3(gp_ceil_div(ny, 64)), dim3(256), 0, stream, Y,
                       n, ny, ldy, sd_floor, mu, sd);
  else
    hipLaunchKernelGGL(simstats_kernel, dim3(gp_ceil_div(ny, 256)), dim3(256), 0, stream, Y, n,
                       ny, ldy, sd_floor, mu, sd);
  hipError_t e = hipGetLastError();
  return e == hipSuccess ? 0 : GPFIT_ERR_HIP - (int)e;
}

extern "C" int gp_standardize(const double* Y, int n, int ny, long long ldy, const double* mu,
                              const double* sd, double* out, long long ldo, int inverse,
                              hipStream_t stream) {
  if (!Y) return -1;
  if (n < 0) return -2;
  if (ny < 0) return -3;
  if (ldy < ny) return -4;
  if (!mu) return -5;
  if (!sd) return -6;
  if (!out) return -7;
  if (ldo < ny) return -8;
  if (n == 0 || ny == 0) return 0;
  const long long tot = (long long)n * ny;
  hipLaunchKernelGGL(standardize_kernel, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0,
                     stream, Y, n, ny, ldy, mu, sd, out, ldo, inverse);
  hipError_t e = hipGetLastError();
  return e == hipSuccess ? 0 : GPFIT_ERR_HIP - (int)e;
}
