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
// r <= kLdsR: A and V live in LDS for the whole solve (2 x 64 x 65 doubles): a global round
// trip per phase (3 per round, 63 rounds per sweep at r = 64) made the L2-resident form take
// 3.35 ms for the C5 basis's 64 x 64 B B^T (profiles/r06/r06b_c5_kernel_stats.csv)
constexpr int kLdsR = 64;
constexpr int kLdsPitch = kLdsR + 1;

// column-major r x r matrix views: global (leading dimension) or LDS (fixed pitch)
struct GMat {
  double* p;
  int ld;
  GP_DEV double& operator()(int i, int j) const { return p[i + (long long)j * ld]; }
};
struct LMat {
  double* p;
  GP_DEV double& operator()(int i, int j) const { return p[i + j * kLdsPitch]; }
};

// The cyclic Jacobi sweep loop and the descending sort, on views A and V (the same operations
// in the same order whichever memory holds them: bit-identical results).
// FUSE (the LDS form): a round's row and column rotations in one phase, one thread per 2 x 2
// block (row pair t, column pair u) applying J_t^T then J_u to its four elements -- every
// element sees the two-phase form's operations in the same order, so the bits are the same --
// with V's column rotations beside them: two barriers per round instead of three.
template <bool FUSE, typename MA, typename MV>
GP_DEV int syevj_solve(MA A, MV V, int r, int max_sweeps, double tol, double* cs, double* sn,
                       int* pp, int* qq, double* red, int* done) {
  const int tid = threadIdx.x, nt = blockDim.x;
  const int R = (r + 1) & ~1;          // padded to even; index r (if any) is a dummy
  const int npair = R / 2;
  for (int g = tid; g < r * r; g += nt) {
    const int i = g % r, j = g / r;
    V(i, j) = (i == j) ? 1.0 : 0.0;
  }
  __syncthreads();
  int sweep = 0;
  for (; sweep < max_sweeps; ++sweep) {
    // convergence check: off-diagonal vs total Frobenius norm
    double off = 0.0, tot = 0.0;
    for (int g = tid; g < r * r; g += nt) {
      const int i = g % r, j = g / r;
      const double a = A(i, j);
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
      *done = (offs <= tol * tol * st) ? 1 : 0;
    }
    __syncthreads();
    if (*done) break;
    for (int round = 0; round < R - 1; ++round) {
      // round-robin pairing: position 0 fixed, positions 1..R-1 rotate
      if (tid < npair) {
        const int a = tid, b = R - 1 - tid;
        auto idx = [&](int pos) { return pos == 0 ? 0 : 1 + (pos - 1 + round) % (R - 1); };
        int p = idx(a), q = idx(b);
        if (p > q) { const int t = p; p = q; q = t; }
        double c = 1.0, s = 0.0;
        if (q < r) {
          const double apq = A(p, q);
          if (apq != 0.0) {
            const double app = A(p, p), aqq = A(q, q);
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
      if (FUSE) {
        for (int g = tid; g < npair * npair; g += nt) {
          const int t = g % npair, u = g / npair;
          const int p = pp[t], q = qq[t], pu = pp[u], qu = qq[u];
          const bool rq = q < r, cq = qu < r;
          // the block after J_t^T (rows p, q), column pu (suffix 0) and qu (suffix 1)
          double xp0 = A(p, pu), xp1 = cq ? A(p, qu) : 0.0;
          double xq0 = 0.0, xq1 = 0.0;
          if (rq) {
            const double c = cs[t], s = sn[t];
            const double y0 = A(q, pu), y1 = cq ? A(q, qu) : 0.0;
            xq0 = s * xp0 + c * y0;
            xp0 = c * xp0 - s * y0;
            xq1 = s * xp1 + c * y1;
            xp1 = c * xp1 - s * y1;
          }
          if (cq) {
            const double c = cs[u], s = sn[u];
            A(p, pu) = c * xp0 - s * xp1;
            A(p, qu) = s * xp0 + c * xp1;
            if (rq) {
              A(q, pu) = c * xq0 - s * xq1;
              A(q, qu) = s * xq0 + c * xq1;
            }
          } else {
            A(p, pu) = xp0;
            if (rq) A(q, pu) = xq0;
          }
        }
        for (int g = tid; g < npair * r; g += nt) {
          const int k = g / npair, t = g % npair;
          const int p = pp[t], q = qq[t];
          if (q >= r) continue;
          const double c = cs[t], s = sn[t];
          const double x = V(k, p), y = V(k, q);
          V(k, p) = c * x - s * y;
          V(k, q) = s * x + c * y;
        }
        __syncthreads();
        continue;
      }
      // phase 1: rows p, q of A   (A <- J^T A)
      for (int g = tid; g < npair * r; g += nt) {
        const int k = g / npair, t = g % npair;
        const int p = pp[t], q = qq[t];
        if (q >= r) continue;
        const double c = cs[t], s = sn[t];
        const double x = A(p, k), y = A(q, k);
        A(p, k) = c * x - s * y;
        A(q, k) = s * x + c * y;
      }
      __syncthreads();
      // phase 2: columns p, q of A (A <- A J) and of V (V <- V J)
      for (int g = tid; g < npair * r; g += nt) {
        const int k = g / npair, t = g % npair;
        const int p = pp[t], q = qq[t];
        if (q >= r) continue;
        const double c = cs[t], s = sn[t];
        double x = A(k, p), y = A(k, q);
        A(k, p) = c * x - s * y;
        A(k, q) = s * x + c * y;
        x = V(k, p);
        y = V(k, q);
        V(k, p) = c * x - s * y;
        V(k, q) = s * x + c * y;
      }
      __syncthreads();
    }
  }
  return sweep;
}

// sort eigenvalues descending (stable selection by one thread), W = eigenvalues or their square
// roots, the columns of V permuted to match and written to Vout (via the scratch view T)
template <typename MA, typename MV>
GP_DEV void syevj_finish(MA A, MV V, int r, int sweep, double* W, GMat Vout, int* perm,
                         double* ws, int* sweeps_out, int want_sqrt) {
  const int tid = threadIdx.x, nt = blockDim.x;
  if (tid < r) ws[tid] = A(tid, tid);
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
  // permuted copy of V into A's storage, then out (A is scratch now)
  for (int g = tid; g < r * r; g += nt) {
    const int i = g % r, j = g / r;
    A(i, j) = V(i, perm[j]);
  }
  __syncthreads();
  for (int g = tid; g < r * r; g += nt) {
    const int i = g % r, j = g / r;
    Vout(i, j) = A(i, j);
  }
}

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
  const GMat Ag{A, lda}, Vg{V, ldv};
  const int sweep = syevj_solve<false>(Ag, Vg, r, max_sweeps, tol, cs, sn, pp, qq, red, &done);
  syevj_finish(Ag, Vg, r, sweep, W, Vg, perm, ws, sweeps_out, want_sqrt);
}

// r <= kLdsR: the same solve on LDS copies of A and V; A (global) is left holding the
// eigenvalue-sorted V, as the global form leaves it
__global__ __launch_bounds__(1024) void syevj_lds_kernel(double* __restrict__ A, int r, int lda,
                                                         double* __restrict__ W,
                                                         double* __restrict__ V, int ldv,
                                                         int max_sweeps, double tol,
                                                         int* __restrict__ sweeps_out,
                                                         int want_sqrt) {
  __shared__ double al[kLdsR * kLdsPitch], vl[kLdsR * kLdsPitch];
  __shared__ double cs[kLdsR / 2], sn[kLdsR / 2];
  __shared__ int pp[kLdsR / 2], qq[kLdsR / 2];
  __shared__ double red[17];
  __shared__ int perm[kLdsR];
  __shared__ double ws[kLdsR];
  __shared__ int done;
  const int tid = threadIdx.x, nt = blockDim.x;
  const LMat Al{al}, Vl{vl};
  for (int g = tid; g < r * r; g += nt) {
    const int i = g % r, j = g / r;
    Al(i, j) = A[i + (long long)j * lda];
  }
  __syncthreads();
  const int sweep = syevj_solve<true>(Al, Vl, r, max_sweeps, tol, cs, sn, pp, qq, red, &done);
  syevj_finish(Al, Vl, r, sweep, W, GMat{V, ldv}, perm, ws, sweeps_out, want_sqrt);
  for (int g = tid; g < r * r; g += nt) {
    const int i = g % r, j = g / r;
    A[i + (long long)j * lda] = Al(i, j);
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
  if (r <= kLdsR)
    hipLaunchKernelGGL(syevj_lds_kernel, dim3(1), dim3(1024), 0, stream, A, r, lda, W, V, ldv,
                       max_sweeps, tol, sweeps, want_sqrt);
  else
    hipLaunchKernelGGL(syevj_kernel, dim3(1), dim3(1024), 0, stream, A, r, lda, W, V, ldv,
                       max_sweeps, tol, sweeps, want_sqrt);
  hipError_t e = hipGetLastError();
  return e == hipSuccess ? 0 : GPFIT_ERR_HIP - (int)e;
}
