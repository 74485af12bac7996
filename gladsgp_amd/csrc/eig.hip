// Small dense symmetric eigensolver (cyclic Jacobi, one workgroup) — the r x r core of the
// randomized SVD (src/svd.py:63 np.linalg.svd(B), B = Q^T X is r x ny with r = p + k <= 1024;
// the reference's calls use r = 25 (model.py:84), 100 (plot_PC_RMSE.py:91) and 2p when k=None):
// SVD(B) is taken from the eigendecomposition of B B^T = U_B S^2 U_B^T (an r x r problem; the
// r x ny products are MFMA GEMMs in blas.hip).
//
// Parallel tournament ordering: each round pairs all r indices disjointly (round-robin with
// index 0 fixed), computes the r/2 Jacobi rotations from the 2x2 pivots, applies them to rows
// (phase 1) and then columns (phase 2) of A and to columns of V.  Matrices live in global
// memory (L2-resident at these sizes); rotation parameters in LDS.  Sweeps stop when the
// off-diagonal Frobenius norm is below tol * ||A||_F or after max_sweeps.  Eigenvalues are
// returned in descending order with V's columns permuted to match.
#include "gpfit_common.h"
#include "../../include/gpfit.h"

namespace {

constexpr int kMaxR = 1024;   // LDS: rotations + pairing + sort keys, ~30 KB

__global__ __launch_bounds__(1024) void syevj_kernel(double* __restrict__ A, int r, int lda,
                                                     double* __restrict__ W,
                                                     double* __restrict__ V, int ldv,
                                                     int max_sweeps, double tol,
                                                     int* __restrict__ sweeps_out,
                                                     int want_sqrt) {
  __shared__ double cs[kMaxR / 2], sn[kMaxR / 2];
  __shared__ int pp[kMaxR / 2], qq[kMaxR / 2];
  __shared__ double red[17];
  __shared__ int perm[kMaxR];
  __shared__ double ws[kMaxR];
  __shared__ int done;
  const int tid = threadIdx.x, nt = blockDim.x;
  const int R = (r + 1) & ~1;          // padded to even; index r (if any) is a dummy
  const int npair = R / 2;
  // V = I
  for (int g = tid; g < r * r; g += nt) {
    const int i = g % r, j = g / r;
    V[i + (long long)j * ldv] = (i == j) ? 1.0 : 0.0;
  }
  __syncthreads();
  int sweep = 0;
  for (; sweep < max_sweeps; ++sweep) {
    // convergence check: off-diagonal vs total Frobenius norm
    double off = 0.0, tot = 0.0;
    for (int g = tid; g < r * r; g += nt) {
      const int i = g % r, j = g / r;
      const double a = A[i + (long long)j * lda];
      tot += a * a;
      if (i != j) off += a * a;
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      off += __shfl_xor(off, o, 64);
      tot += __shfl_xor(tot, o, 64);
    }
    if ((tid & 63) == 0) red[tid >> 6] = off;
    __syncthreads();
    if (tid == 0) {
      double so = 0.0;
      for (int q = 0; q < (nt + 63) / 64; ++q) so += red[q];
      red[16] = so;
    }
    __syncthreads();
    const double offs = red[16];
    __syncthreads();
    if ((tid & 63) == 0) red[tid >> 6] = tot;
    __syncthreads();
    if (tid == 0) {
      double st = 0.0;
      for (int q = 0; q < (nt + 63) / 64; ++q) st += red[q];
      done = (offs <= tol * tol * st) ? 1 : 0;
    }
    __syncthreads();
    if (done) break;
    for (int round = 0; round < R - 1; ++round) {
      // round-robin pairing: position 0 fixed, positions 1..R-1 rotate
      if (tid < npair) {
        const int a = tid, b = R - 1 - tid;
        auto idx = [&](int pos) { return pos == 0 ? 0 : 1 + (pos - 1 + round) % (R - 1); };
        int p = idx(a), q = idx(b);
        if (p > q) { const int t = p; p = q; q = t; }
        double c = 1.0, s = 0.0;
        if (q < r) {
          const double apq = A[p + (long long)q * lda];
          if (apq != 0.0) {
            const double app = A[p + (long long)p * lda], aqq = A[q + (long long)q * lda];
            const double theta = (aqq - app) / (2.0 * apq);
            const double t = (theta >= 0.0 ? 1.0 : -1.0) / (fabs(theta) + sqrt(1.0 + theta * theta));
            c = 1.0 / sqrt(1.0 + t * t);
            s = t * c;
          }
        }
        cs[tid] = c;
        sn[tid] = s;
        pp[tid] = p;
        qq[tid] = q;
      }
      __syncthreads();
      // phase 1: rows p, q of A   (A <- J^T A)
      for (int g = tid; g < npair * r; g += nt) {
        const int k = g / npair, t = g % npair;
        const int p = pp[t], q = qq[t];
        if (q >= r) continue;
        const double c = cs[t], s = sn[t];
        double* ap = A + p + (long long)k * lda;
        double* aq = A + q + (long long)k * lda;
        const double x = *ap, y = *aq;
        *ap = c * x - s * y;
        *aq = s * x + c * y;
      }
      __syncthreads();
      // phase 2: columns p, q of A (A <- A J) and of V (V <- V J)
      for (int g = tid; g < npair * r; g += nt) {
        const int k = g / npair, t = g % npair;
        const int p = pp[t], q = qq[t];
        if (q >= r) continue;
        const double c = cs[t], s = sn[t];
        double* ap = A + k + (long long)p * lda;
        double* aq = A + k + (long long)q * lda;
        double x = *ap, y = *aq;
        *ap = c * x - s * y;
        *aq = s * x + c * y;
        double* vp = V + k + (long long)p * ldv;
        double* vq = V + k + (long long)q * ldv;
        x = *vp;
        y = *vq;
        *vp = c * x - s * y;
        *vq = s * x + c * y;
      }
      __syncthreads();
    }
  }
  // sort eigenvalues descending; permute V's columns (stable selection by one thread)
  if (tid < r) ws[tid] = A[tid + (long long)tid * lda];
  __syncthreads();
  if (tid == 0) {
    for (int i = 0; i < r; ++i) perm[i] = i;
    for (int i = 0; i < r; ++i) {
      int best = i;
      for (int j = i + 1; j < r; ++j)
        if (ws[perm[j]] > ws[perm[best]]) best = j;
      const int t = perm[i]; perm[i] = perm[best]; perm[best] = t;
    }
    if (sweeps_out) *sweeps_out = sweep;
  }
  __syncthreads();
  if (tid < r) {
    const double ev = ws[perm[tid]];
    W[tid] = want_sqrt ? sqrt(ev > 0.0 ? ev : 0.0) : ev;   // singular values of B when A = B B^T
  }
  // permuted copy of V into A's storage, then back (A is scratch now)
  for (int g = tid; g < r * r; g += nt) {
    const int i = g % r, j = g / r;
    A[i + (long long)j * lda] = V[i + (long long)perm[j] * ldv];
  }
  __syncthreads();
  for (int g = tid; g < r * r; g += nt) {
    const int i = g % r, j = g / r;
    V[i + (long long)j * ldv] = A[i + (long long)j * lda];
  }
}

}  // namespace

extern "C" int gp_syevj(double* A, int r, int lda, double* W, double* V, int ldv,
                        int max_sweeps, double tol, int* sweeps, int want_sqrt,
                        hipStream_t stream) {
  if (!A) return -1;
  if (r < 0 || r > kMaxR) return -2;
  if (lda < r || lda < 1) return -3;
  if (!W) return -4;
  if (!V) return -5;
  if (ldv < r || ldv < 1) return -6;
  if (max_sweeps < 0) return -7;
  if (r == 0) return 0;
  hipLaunchKernelGGL(syevj_kernel, dim3(1), dim3(1024), 0, stream, A, r, lda, W, V, ldv,
                     max_sweeps, tol, sweeps, want_sqrt);
  hipError_t e = hipGetLastError();
  return e == hipSuccess ? 0 : GPFIT_ERR_HIP - (int)e;
}
