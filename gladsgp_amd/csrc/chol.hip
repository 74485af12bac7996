// Blocked right-looking Cholesky with a simultaneous triangular inverse (fp64, MFMA).
//
// Reference behaviour replaced: the SPD factorisation inside SEPIA's likelihood / prediction
// (LAPACK potrf), scipy.linalg.cholesky(lower=True) in examples/01...ipynb:66,144 and GPmodule's
// K_inv (examples/02...ipynb:232-233).  LAPACK semantics: info = first failing pivot (1-based).
//
// Algorithm (NB = 64 blocks, k = 0..N-1), X = L^-1 built alongside L:
//   diag   : L_kk = chol(A_kk) in LDS, D_k = L_kk^-1 (written as X_kk), logdet += 2 sum log
//   panel  : L_ik = A_ik D_k^T            (i > k)        — 64^3 MFMA tile GEMMs
//            X_kc = D_k R_kc              (c < k)        — R_kc accumulated in X's storage
//   update : A_ij -= L_ik L_jk^T          (k < j <= i)   — SYRK/GEMM trailing update
//            R_ic -= L_ik X_kc            (i > k, c<=k)  — drives the block forward
//                                                          substitution of L X = I
// Both products are n^3/3 flop; every tile product runs on v_mfma_f64_16x16x4_f64.
// Tile GEMM: 256 threads = 4 waves in a 2x2 grid of 32x32 sub-tiles (2x2 MFMA 16x16 each);
// operands staged into LDS k-major ([k][x], row pitch 65 doubles to spread banks), result
// transposed through LDS so global stores are coalesced down columns.
#include "gpfit_common.h"
#include "gpfit_profile.h"
#include "../../include/gpfit.h"

namespace {

constexpr int NB = 64;
constexpr int LP = NB + 1;  // LDS pitch (doubles)

// S[k][x]: NAT → src[x + k*ld] (x contiguous), TRN → src[k + x*ld] (k contiguous).
template <bool TRN>
GP_DEV void stage(double* S, const double* __restrict__ src, int ld, int xv, int kv) {
#pragma unroll 4
  for (int q = 0; q < (NB * NB) / 256; ++q) {
    const int g = threadIdx.x + 256 * q;
    const int fast = g & (NB - 1), slow = g >> 6;
    if (!TRN) {
      const int x = fast, k = slow;
      S[k * LP + x] = (x < xv && k < kv) ? src[x + (long long)k * ld] : 0.0;
    } else {
      const int k = fast, x = slow;
      S[k * LP + x] = (x < xv && k < kv) ? src[k + (long long)x * ld] : 0.0;
    }
  }
}

// acc (this wave's 32x32) = sum_k As[k][rows] * Bs[k][cols]
GP_DEV void mma64(const double* As, const double* Bs, f64x4 (&acc)[2][2]) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int wr = w >> 1, wc = w & 1, li = lane & 15, lk = lane >> 4;
#pragma unroll
  for (int mi = 0; mi < 2; ++mi)
#pragma unroll
    for (int nj = 0; nj < 2; ++nj) acc[mi][nj] = zero4();
#pragma unroll 4
  for (int k4 = 0; k4 < NB / 4; ++k4) {
    const int k = k4 * 4 + lk;
    const double a0 = As[k * LP + wr * 32 + li], a1 = As[k * LP + wr * 32 + 16 + li];
    const double b0 = Bs[k * LP + wc * 32 + li], b1 = Bs[k * LP + wc * 32 + 16 + li];
    acc[0][0] = mfma16x16x4(a0, b0, acc[0][0]);
    acc[0][1] = mfma16x16x4(a0, b1, acc[0][1]);
    acc[1][0] = mfma16x16x4(a1, b0, acc[1][0]);
    acc[1][1] = mfma16x16x4(a1, b1, acc[1][1]);
  }
}

// Write the block's 64x64 accumulator to C (column-major, ld), rows < rv, cols < cv.
// SUB: C -= acc, else C = acc.  LOWER: only row >= col (diagonal tiles of A).
template <bool SUB>
GP_DEV void epilogue(double* Cs, const f64x4 (&acc)[2][2], double* __restrict__ C, int ld,
                     int rv, int cv, bool lower) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int wr = w >> 1, wc = w & 1, li = lane & 15, lk = lane >> 4;
  __syncthreads();  // all waves done reading As/Bs (Cs aliases As)
#pragma unroll
  for (int mi = 0; mi < 2; ++mi)
#pragma unroll
    for (int nj = 0; nj < 2; ++nj)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = wr * 32 + mi * 16 + lk + 4 * r, col = wc * 32 + nj * 16 + li;
        Cs[col * LP + row] = acc[mi][nj][r];
      }
  __syncthreads();
#pragma unroll 4
  for (int q = 0; q < (NB * NB) / 256; ++q) {
    const int g = threadIdx.x + 256 * q;
    const int row = g & (NB - 1), col = g >> 6;
    if (row < rv && col < cv && (!lower || row >= col)) {
      double* p = C + row + (long long)col * ld;
      const double v = Cs[col * LP + row];
      *p = SUB ? (*p - v) : v;
    }
  }
}

__global__ __launch_bounds__(256) void chol_diag_kernel(
    double* __restrict__ A, int lda, long long sA, double* __restrict__ X, int ldx,
    long long sX, int n, int k, int* __restrict__ info, double* __restrict__ logdet) {
  const int b = blockIdx.x;
  if (info && info[b] != 0) return;
  __shared__ double T[NB * LP];
  __shared__ double U[NB * LP];
  const int k0 = k * NB;
  const int nb = min(NB, n - k0);
  double* Ab = A + b * sA + k0 + (long long)k0 * lda;
  double* Xb = X + b * sX + k0 + (long long)k0 * ldx;
  const int tid = threadIdx.x;
  // T[i][c] row-major in LDS (i = row): coalesced read down columns of A.
  for (int g = tid; g < NB * NB; g += 256) {
    const int i = g & (NB - 1), c = g >> 6;
    double v;
    if (i < nb && c < nb) v = Ab[i + (long long)c * lda];
    else v = (i == c) ? 1.0 : 0.0;   // identity padding keeps the edge block SPD
    T[i * LP + c] = v;
  }
  __syncthreads();
  const int row = tid & (NB - 1), cq = tid >> 6;
  for (int j = 0; j < NB; ++j) {
    const double piv = T[j * LP + j];
    if (!(piv > 0.0) || !isfinite(piv)) {  // uniform: every thread reads the same LDS word
      if (tid == 0 && j < nb && info) { info[b] = k0 + j + 1; }
      return;
    }
    const double sp = sqrt(piv);
    __syncthreads();  // everyone has read the pivot before it is overwritten
    if (tid == j) T[j * LP + j] = sp;
    if (tid > j && tid < NB) T[tid * LP + j] /= sp;
    __syncthreads();
    for (int c = j + 1 + cq; c <= row; c += 4) T[row * LP + c] -= T[row * LP + j] * T[c * LP + j];
    __syncthreads();
  }
  // D = L^-1 : thread c solves column c by forward substitution (its own column only).
  if (tid < NB) {
    const int c = tid;
    for (int i = 0; i < NB; ++i) {
      if (i < c) { U[i * LP + c] = 0.0; continue; }
      double acc = (i == c) ? 1.0 : 0.0;
      for (int p = c; p < i; ++p) acc -= T[i * LP + p] * U[p * LP + c];
      U[i * LP + c] = acc / T[i * LP + i];
    }
  }
  // logdet contribution (wave 0)
  if (tid < 64 && logdet) {
    double v = (tid < nb) ? 2.0 * log(T[tid * LP + tid]) : 0.0;
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
    if (tid == 0) logdet[b] += v;
  }
  __syncthreads();
  for (int g = tid; g < NB * NB; g += 256) {
    const int i = g & (NB - 1), c = g >> 6;
    if (i < nb && c < nb) {
      if (i >= c) Ab[i + (long long)c * lda] = T[i * LP + c];
      Xb[i + (long long)c * ldx] = U[i * LP + c];
    }
  }
}

__global__ __launch_bounds__(256) void chol_panel_kernel(
    double* __restrict__ A, int lda, long long sA, double* __restrict__ X, int ldx,
    long long sX, int n, int k, int nbelow, const int* __restrict__ info) {
  const int b = blockIdx.y;
  if (info && info[b] != 0) return;
  __shared__ double As[NB * LP];
  __shared__ double Bs[NB * LP];
  const int k0 = k * NB, kv = min(NB, n - k0);
  double* Ab = A + b * sA;
  double* Xb = X + b * sX;
  const double* Dk = Xb + k0 + (long long)k0 * ldx;   // D_k = X_kk (lower, zero upper)
  f64x4 acc[2][2];
  if ((int)blockIdx.x < nbelow) {
    // L_ik = A_ik D_k^T :  opA[r][p] = A_ik(r,p) (NAT), opB[p][c] = D_k(c,p) (NAT)
    const int i0 = (k + 1 + blockIdx.x) * NB, rv = min(NB, n - i0);
    double* Aik = Ab + i0 + (long long)k0 * lda;
    stage<false>(As, Aik, lda, rv, kv);
    stage<false>(Bs, Dk, ldx, kv, kv);
    __syncthreads();
    mma64(As, Bs, acc);
    epilogue<false>(As, acc, Aik, lda, rv, kv, false);
  } else {
    // X_kc = D_k R_kc :  opA[r][p] = D_k(r,p) (NAT), opB[p][c] = R_kc(p,c) (TRN)
    const int c0 = (blockIdx.x - nbelow) * NB;
    double* Rkc = Xb + k0 + (long long)c0 * ldx;
    stage<false>(As, Dk, ldx, kv, kv);
    stage<true>(Bs, Rkc, ldx, NB, kv);
    __syncthreads();
    mma64(As, Bs, acc);
    epilogue<false>(As, acc, Rkc, ldx, kv, NB, false);
  }
}

__global__ __launch_bounds__(256) void chol_update_kernel(
    double* __restrict__ A, int lda, long long sA, double* __restrict__ X, int ldx,
    long long sX, int n, int k, int T, const int* __restrict__ info) {
  const int b = blockIdx.y;
  if (info && info[b] != 0) return;
  __shared__ double As[NB * LP];
  __shared__ double Bs[NB * LP];
  const int k0 = k * NB, kv = min(NB, n - k0);
  double* Ab = A + b * sA;
  double* Xb = X + b * sX;
  const int ntri = T * (T + 1) / 2;
  const int idx = blockIdx.x;
  f64x4 acc[2][2];
  if (idx < ntri) {
    int ii = (int)((sqrt(8.0 * idx + 1.0) - 1.0) * 0.5);
    while (ii * (ii + 1) / 2 > idx) --ii;
    while ((ii + 1) * (ii + 2) / 2 <= idx) ++ii;
    const int jj = idx - ii * (ii + 1) / 2;
    const int i0 = (k + 1 + ii) * NB, j0 = (k + 1 + jj) * NB;
    const int rv = min(NB, n - i0), cv = min(NB, n - j0);
    // A_ij -= L_ik L_jk^T
    stage<false>(As, Ab + i0 + (long long)k0 * lda, lda, rv, kv);
    stage<false>(Bs, Ab + j0 + (long long)k0 * lda, lda, cv, kv);
    __syncthreads();
    mma64(As, Bs, acc);
    epilogue<true>(As, acc, Ab + i0 + (long long)j0 * lda, lda, rv, cv, ii == jj);
  } else {
    const int idx2 = idx - ntri;
    const int ii = idx2 / (k + 1), c = idx2 % (k + 1);
    const int i0 = (k + 1 + ii) * NB, c0 = c * NB, rv = min(NB, n - i0);
    // R_ic -= L_ik X_kc :  opB[p][cc] = X(k0+p, c0+cc) (TRN)
    stage<false>(As, Ab + i0 + (long long)k0 * lda, lda, rv, kv);
    stage<true>(Bs, Xb + k0 + (long long)c0 * ldx, ldx, NB, kv);
    __syncthreads();
    mma64(As, Bs, acc);
    epilogue<true>(As, acc, Xb + i0 + (long long)c0 * ldx, ldx, rv, NB, false);
  }
}

}  // namespace

extern "C" int gp_potrf_inv(double* A, int n, int lda, long long strideA, double* Linv,
                            int ldinv, long long strideInv, int batch, int* info,
                            double* logdet, hipStream_t stream) {
  if (!A) return -1;
  if (n < 0) return -2;
  if (lda < n || lda < 1) return -3;
  if (batch > 1 && strideA < (long long)lda * n) return -4;
  if (!Linv) return -5;
  const int npad = gp_padded_n(n);
  if (ldinv < npad || ldinv < 1) return -6;
  if (batch > 1 && strideInv < (long long)ldinv * npad) return -7;
  if (batch < 0) return -8;
  if (n == 0 || batch == 0) return 0;
  hipError_t e;
#define GP_CK(x) do { e = (x); if (e != hipSuccess) return GPFIT_ERR_HIP - (int)e; } while (0)
  if (info) GP_CK(hipMemsetAsync(info, 0, sizeof(int) * batch, stream));
  if (logdet) GP_CK(hipMemsetAsync(logdet, 0, sizeof(double) * batch, stream));
  // zero L^-1 (upper triangle + padding), one 2-D memset per problem
  for (int b = 0; b < batch; ++b)
    GP_CK(hipMemset2DAsync(Linv + b * strideInv, sizeof(double) * ldinv, 0,
                           sizeof(double) * npad, npad, stream));
  const int N = gp_ceil_div(n, NB);
  gpfit_prof_begin(GP_PROF_POTRF, stream);
  for (int k = 0; k < N; ++k) {
    hipLaunchKernelGGL(chol_diag_kernel, dim3(batch), dim3(256), 0, stream, A, lda, strideA,
                       Linv, ldinv, strideInv, n, k, info, logdet);
    GP_CK(hipGetLastError());
    const int T = N - k - 1;
    if (T + k > 0) {
      hipLaunchKernelGGL(chol_panel_kernel, dim3(T + k, batch), dim3(256), 0, stream, A, lda,
                         strideA, Linv, ldinv, strideInv, n, k, T, info);
      GP_CK(hipGetLastError());
    }
    if (T > 0) {
      const int nt = T * (T + 1) / 2 + T * (k + 1);
      hipLaunchKernelGGL(chol_update_kernel, dim3(nt, batch), dim3(256), 0, stream, A, lda,
                         strideA, Linv, ldinv, strideInv, n, k, T, info);
      GP_CK(hipGetLastError());
    }
  }
  gpfit_prof_end(GP_PROF_POTRF, stream);
#undef GP_CK
  return 0;
}
