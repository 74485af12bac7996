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

extern "C" long long gp_dgemm_ws_bytes(int m, int n, int k) {
  if (m <= 0 || n <= 0 || k <= 0) return 0;
  const int s = choose_splits(m, n, k);
  return s > 1 ? (long long)s * m * n * 8 : 0;
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
  hipLaunchKernelGGL(simstats_kernel, dim3(gp_ceil_div(ny, 256)), dim3(256), 0, stream, Y, n, ny,
                     ldy, sd_floor, mu, sd);
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
