// Blocked right-looking Cholesky with a simultaneous triangular inverse (fp64, MFMA).
//
// Reference behaviour replaced: the SPD factorisation inside SEPIA's likelihood / prediction
// (LAPACK potrf), scipy.linalg.cholesky(lower=True) in examples/01...ipynb:66,144 and GPmodule's
// K_inv (examples/02...ipynb:232-233).  LAPACK semantics: info = first failing pivot (1-based),
// the strict upper triangle of A is neither read nor written.
//
// Algorithm (NB = 64 blocks, k = 0..N-1), X = L^-1 built alongside L:
//   diag   : L_kk = chol(A_kk), D_k = L_kk^-1 (written as X_kk), logdet += 2 sum log L_ii
//   panel  : L_ik = A_ik D_k^T            (i > k)        — 64^3 MFMA tile GEMMs
//            X_kc = D_k R_kc              (c < k)        — R_kc accumulated in X's storage
//   update : A_ij -= L_ik L_jk^T          (k < j <= i)   — SYRK/GEMM trailing update
//            R_ic -= L_ik X_kc            (i > k, c<=k)  — block forward substitution of L X = I
// Lookahead: the update block that owns tile (k+1, k+1) factors and inverts it right after its
// own update (diag_factor_inv below), so each step is two launches (panel, update+diag) and the
// serial diagonal work overlaps the rest of the trailing update.
//
// diag_factor_inv: 4 waves, register resident (see the function for the scheme): X = L^-1
// comes out of the same right-looking sweep as L (X_j. = R_j. / L_jj, R_i. -= L_ij X_j.),
// one barrier and 16 FMAs per thread per column step.
#include "gpfit_common.h"
#include "gpfit_profile.h"
#include "../../include/gpfit.h"

#ifdef GPFIT_DIAG_STAMPS
__device__ unsigned long long gpfit_diag_stamps[16];
extern "C" int gp_diag_stamps(unsigned long long* host16) {
  return (int)hipMemcpyFromSymbol(host16, HIP_SYMBOL(gpfit_diag_stamps), 16 * 8);
}
#endif

namespace {

constexpr int NB = 64;
constexpr int LP = NB + 1;  // LDS pitch (doubles)

struct __align__(16) Smem {
  double As[NB * LP];
  double Bs[NB * LP];
  double VA[2][NB];    // L[.][j]   of the current pair (rows below the pivot)
  double VB[2][NB];    // L[.][j+1]
  double RR[2][NB];    // R[j][.]   (unscaled, c <= j)
  double RB[2][NB];    // R[j+1][.] (unscaled, c <= j+1)
  double sps[NB];      // L_jj
  double invs[NB];     // 1 / L_jj
  double inv[2];
  double inv1[2];
  double l10[2];
  double red[4];
  int bad[NB];         // per-column non-PD pivot flags (written once, scanned at the end)
  int fail;
};

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

// Scatter the block's accumulator into LDS as Cs[col][row] (pitch LP).
GP_DEV void acc_to_lds(double* Cs, const f64x4 (&acc)[2][2]) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int wr = w >> 1, wc = w & 1, li = lane & 15, lk = lane >> 4;
#pragma unroll
  for (int mi = 0; mi < 2; ++mi)
#pragma unroll
    for (int nj = 0; nj < 2; ++nj)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = wr * 32 + mi * 16 + lk + 4 * r, col = wc * 32 + nj * 16 + li;
        Cs[col * LP + row] = acc[mi][nj][r];
      }
}

// Coalesced tile element owned by thread for slot q: row = g & 63, col = g >> 6.
GP_DEV void slot_rc(int q, int& row, int& col) {
  const int g = threadIdx.x + 256 * q;
  row = g & (NB - 1);
  col = g >> 6;
}

// C = acc (STORE) for rows < rv, cols < cv.
GP_DEV void store_tile(double* Cs, const f64x4 (&acc)[2][2], double* __restrict__ C, int ld,
                       int rv, int cv) {
  __syncthreads();  // all waves done with As/Bs (Cs aliases As)
  acc_to_lds(Cs, acc);
  __syncthreads();
#pragma unroll 4
  for (int q = 0; q < 16; ++q) {
    int row, col;
    slot_rc(q, row, col);
    if (row < rv && col < cv) C[row + (long long)col * ld] = Cs[col * LP + row];
  }
}

// Factor + invert the 64x64 tile held (full, symmetric) in T[row * LP + col]; all 256 threads
// call it.  nb valid rows (rows/cols >= nb are identity padding).  On return T holds L (lower,
// zero upper), U holds L^-1 (lower, zero upper); returns 0 or the 1-based local index of the
// first non-PD pivot.
//
// Thread (row i = t & 63, wave cq = t >> 6) owns the 16 register slots w[u] of columns
// c = 16 cq + u.  Slot c holds A[i][c] until column c is factored and R[i][c] afterwards
// (R starts as I; X = L^-1 has rows R_i. / L_ii).  Columns are taken TWO at a time (a rank-2
// right-looking step): the wave owning columns (j, j+1) factors its 2x2 pivot block in
// registers (readlane pivots, rsqrt, the local column-j update of column j+1) and publishes
//   VA0 = L[.][j], VA1 = L[.][j+1]   (lanes below the pivots)     and    inv0, inv1, L[j+1][j]
// while lanes j and j+1 of every wave publish their R rows (unscaled).  After one barrier each
// thread applies, per slot c (the c-vs-j tests are wave-uniform),
//   c > j+1 :  A[i][c] -= L[i][j] L[c][j] + L[i][j+1] L[c][j+1]
//   c <= j+1:  R[i][c] -= L[i][j] X[j][c] + L[i][j+1] X[j+1][c]
// with X[j][c] = R[j][c]/L_jj and X[j+1][c] = (R[j+1][c] - L[j+1][j] X[j][c]) / L_j+1,j+1.
// 32 barriers per block instead of 64; the owner's two pivot chains per step are the critical
// path.  The pair loop is unrolled by 8 so owner wave and slots are compile-time.
GP_DEV int diag_factor_inv(Smem& sm, double* T, double* U, int nb, double* ld_out) {
  const int tid = threadIdx.x;
  const int i = tid & (NB - 1);
  const int cq = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int cb = cq * 16;
  double w[16];
#pragma unroll
  for (int u = 0; u < 16; ++u) w[u] = T[i * LP + cb + u];

  // publish pair (j, j+1): owner wave `own`, slots uj, uj+1 (compile-time), buffer q
  auto publish = [&](int j, int own, int uj, int q) {
    if (cq == own) {
      const double a0 = w[uj];
      const double piv0 = readlane_f64(a0, j);
      const double inv0 = rsqrt_nr(piv0);
      const double l0 = (i > j) ? a0 * inv0 : 0.0;               // L[i][j]
      const double L10 = readlane_f64(l0, j + 1);                 // L[j+1][j]
      const double a1 = fma(-l0, L10, w[uj + 1]);                 // A[i][j+1] after column j
      const double piv1 = readlane_f64(a1, j + 1);
      const double inv1 = rsqrt_nr(piv1);
      const double l1 = (i > j + 1) ? a1 * inv1 : 0.0;           // L[i][j+1]
      sm.VA[q][i] = l0;
      sm.VB[q][i] = l1;
      if (i > j) T[i * LP + j] = l0;                             // T's columns j, j+1 were read
      if (i > j + 1) T[i * LP + j + 1] = l1;                     // only by this wave
      w[uj] = (i == j) ? 1.0 : 0.0;                              // slots now hold R (= delta)
      w[uj + 1] = (i == j + 1) ? 1.0 : 0.0;
      if (i == 0) {
        sm.inv[q] = inv0;
        sm.inv1[q] = inv1;
        sm.l10[q] = L10;
        sm.invs[j] = inv0;
        sm.invs[j + 1] = inv1;
        sm.sps[j] = piv0 * inv0;
        sm.sps[j + 1] = piv1 * inv1;
        sm.bad[j] = (!(piv0 > 0.0) || !isfinite(piv0)) ? 1 : 0;
        sm.bad[j + 1] = (!(piv1 > 0.0) || !isfinite(piv1)) ? 1 : 0;
      }
    }
    // R rows j (c <= j) and j+1 (c <= j+1), unscaled; two uniform cases per wave
    if (i == j || i == j + 1) {
      double* dst = (i == j) ? sm.RR[q] : sm.RB[q];
      if (cq < own) {
#pragma unroll
        for (int u = 0; u < 16; u += 2) {
          double2 y;
          y.x = w[u];
          y.y = w[u + 1];
          *reinterpret_cast<double2*>(&dst[cb + u]) = y;
        }
      } else if (cq == own) {
#pragma unroll
        for (int u = 0; u < 16; ++u)
          if (u <= uj + 1) dst[cb + u] = w[u];
      }
    }
  };

  publish(0, 0, 0, 0);
#pragma unroll 1
  for (int jb = 0; jb < NB / 16; ++jb) {
#pragma unroll
    for (int jj = 0; jj < 16; jj += 2) {
      const int j = jb * 16 + jj;
      const int p = (jj >> 1) & 1;
      __syncthreads();
      const double inv0 = sm.inv[p], inv1 = sm.inv1[p], L10 = sm.l10[p];
      const double m0 = (i > j) ? sm.VA[p][i] : 0.0;             // L[i][j]
      const double m1 = (i > j + 1) ? sm.VB[p][i] : 0.0;         // L[i][j+1]
      // next pair's owner / slots (compile-time per jj); its two slots are updated first
      const int own1 = (jj < 14) ? jb : jb + 1, u1 = (jj + 2) & 15;
#pragma unroll
      for (int pass = 0; pass < 2; ++pass) {
#pragma unroll
        for (int u = 0; u < 16; u += 2) {
          const bool first = (cq == own1) && (u == u1);
          if ((pass == 0) != first) continue;
          const int c = cb + u;                                    // c, c+1 same side of j+1
          if (c > j + 1) {
            const double2 a = *reinterpret_cast<const double2*>(&sm.VA[p][c]);
            const double2 b = *reinterpret_cast<const double2*>(&sm.VB[p][c]);
            w[u] = fma(-m1, b.x, fma(-m0, a.x, w[u]));
            w[u + 1] = fma(-m1, b.y, fma(-m0, a.y, w[u + 1]));
          } else {
            const double2 r0 = *reinterpret_cast<const double2*>(&sm.RR[p][c]);
            const double2 r1 = *reinterpret_cast<const double2*>(&sm.RB[p][c]);
            // X[j][c] (zero for c = j+1), X[j+1][c]
            const double x0a = r0.x * inv0;
            const double x0b = (c + 1 <= j) ? r0.y * inv0 : 0.0;
            const double x1a = (r1.x - L10 * x0a) * inv1;
            const double x1b = (r1.y - L10 * x0b) * inv1;
            w[u] = fma(-m1, x1a, fma(-m0, x0a, w[u]));
            w[u + 1] = fma(-m1, x1b, fma(-m0, x0b, w[u + 1]));
          }
        }
      }
      if (j + 2 < NB) publish(j + 2, own1, u1, p ^ 1);
    }
  }
  __syncthreads();
  if (tid < 64) {
    const unsigned long long badm = __ballot(sm.bad[tid] != 0 && tid < nb);
    if (tid == 0) sm.fail = badm ? (__ffsll((long long)badm)) : 0;
  }
  __syncthreads();
  const int f = sm.fail;              // first bad pivot among the nb valid columns
  if (f) return f;
  const double inv_i = sm.invs[i];
#pragma unroll
  for (int u = 0; u < 16; ++u) {
    const int c = cb + u;
    U[i * LP + c] = (c <= i) ? w[u] * inv_i : 0.0;
    if (c >= i) T[i * LP + c] = (c == i) ? sm.sps[i] : 0.0;   // c < i: written by publish
  }
  double lg = (cq == 0 && i < nb) ? 2.0 * log(sm.sps[i]) : 0.0;
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) lg += __shfl_xor(lg, off, 64);
  if ((tid & 63) == 0) sm.red[tid >> 6] = lg;
  __syncthreads();
  if (ld_out) *ld_out = (sm.red[0] + sm.red[1]) + (sm.red[2] + sm.red[3]);
  return 0;
}

// Factor diagonal block k whose (updated, symmetric) tile is in sm.As as [row][col]; write
// L_kk into A, D_k into X, accumulate logdet, set info.
GP_DEV void diag_block(Smem& sm, double* __restrict__ Ab, int lda, double* __restrict__ Xb,
                       int ldx, int n, int k, int* info, double* logdet, int b) {
  const int k0 = k * NB, nb = min(NB, n - k0);
  double lg = 0.0;
  const int f = diag_factor_inv(sm, sm.As, sm.Bs, nb, &lg);
  if (f) {
    if (threadIdx.x == 0 && info) info[b] = k0 + f;
    return;
  }
  if (threadIdx.x == 0 && logdet) logdet[b] += lg;
  double* Akk = Ab + k0 + (long long)k0 * lda;
  double* Xkk = Xb + k0 + (long long)k0 * ldx;
#pragma unroll 4
  for (int q = 0; q < 16; ++q) {
    int row, col;
    slot_rc(q, row, col);
    if (row < nb && col < nb) {
      if (row >= col) Akk[row + (long long)col * lda] = sm.As[row * LP + col];
      Xkk[row + (long long)col * ldx] = sm.Bs[row * LP + col];
    }
  }
}

__global__ __launch_bounds__(256) void chol_diag_kernel(
    double* __restrict__ A, int lda, long long sA, double* __restrict__ X, int ldx,
    long long sX, int n, int k, int* __restrict__ info, double* __restrict__ logdet) {
  const int b = blockIdx.x;
  if (info && info[b] != 0) return;
  __shared__ Smem sm;
  const int k0 = k * NB, nb = min(NB, n - k0);
  double* Ab = A + b * sA;
  const double* Akk = Ab + k0 + (long long)k0 * lda;
  // symmetric tile from the lower triangle only (upper triangle of A is never read)
  for (int g = threadIdx.x; g < NB * NB; g += 256) {
    const int row = g & (NB - 1), col = g >> 6;
    double v;
    if (row < nb && col < nb) {
      v = (row >= col) ? Akk[row + (long long)col * lda] : Akk[col + (long long)row * lda];
    } else {
      v = (row == col) ? 1.0 : 0.0;
    }
    sm.As[row * LP + col] = v;
  }
  __syncthreads();
  diag_block(sm, Ab, lda, X + b * sX, ldx, n, k, info, logdet, b);
}

__global__ __launch_bounds__(256) void chol_panel_kernel(
    double* __restrict__ A, int lda, long long sA, double* __restrict__ X, int ldx,
    long long sX, int n, int k, int nbelow, const int* __restrict__ info) {
  const int b = blockIdx.y;
  if (info && info[b] != 0) return;
  __shared__ Smem sm;
  const int k0 = k * NB, kv = min(NB, n - k0);
  double* Ab = A + b * sA;
  double* Xb = X + b * sX;
  const double* Dk = Xb + k0 + (long long)k0 * ldx;   // D_k = X_kk (lower, zero upper)
  f64x4 acc[2][2];
  if ((int)blockIdx.x < nbelow) {
    // L_ik = A_ik D_k^T :  opA[r][p] = A_ik(r,p) (NAT), opB[p][c] = D_k(c,p) (NAT)
    const int i0 = (k + 1 + blockIdx.x) * NB, rv = min(NB, n - i0);
    double* Aik = Ab + i0 + (long long)k0 * lda;
    stage<false>(sm.As, Aik, lda, rv, kv);
    stage<false>(sm.Bs, Dk, ldx, kv, kv);
    __syncthreads();
    mma64(sm.As, sm.Bs, acc);
    store_tile(sm.As, acc, Aik, lda, rv, kv);
  } else {
    // X_kc = D_k R_kc :  opA[r][p] = D_k(r,p) (NAT), opB[p][c] = R_kc(p,c) (TRN)
    const int c0 = (blockIdx.x - nbelow) * NB;
    double* Rkc = Xb + k0 + (long long)c0 * ldx;
    stage<false>(sm.As, Dk, ldx, kv, kv);
    stage<true>(sm.Bs, Rkc, ldx, NB, kv);
    __syncthreads();
    mma64(sm.As, sm.Bs, acc);
    store_tile(sm.As, acc, Rkc, ldx, kv, NB);
  }
}

// Trailing update of step k.  Block 0 owns tile (k+1, k+1) and then factors it (lookahead).
__global__ __launch_bounds__(256) void chol_update_kernel(
    double* __restrict__ A, int lda, long long sA, double* __restrict__ X, int ldx,
    long long sX, int n, int k, int T, int* __restrict__ info, double* __restrict__ logdet) {
  const int b = blockIdx.y;
  if (info && info[b] != 0) return;
  __shared__ Smem sm;
  const int k0 = k * NB, kv = min(NB, n - k0);
  double* Ab = A + b * sA;
  double* Xb = X + b * sX;
  const int ntri = T * (T + 1) / 2;
  const int idx = blockIdx.x;
  double* Cp;
  int ldc, rv, cv, ldb;
  bool diag = false, trn;
  const double *Ap, *Bp;
  if (idx < ntri) {
    int ii = (int)((sqrt(8.0 * idx + 1.0) - 1.0) * 0.5);
    while (ii * (ii + 1) / 2 > idx) --ii;
    while ((ii + 1) * (ii + 2) / 2 <= idx) ++ii;
    const int jj = idx - ii * (ii + 1) / 2;
    const int i0 = (k + 1 + ii) * NB, j0 = (k + 1 + jj) * NB;
    rv = min(NB, n - i0);
    cv = min(NB, n - j0);
    Ap = Ab + i0 + (long long)k0 * lda;                 // L_ik
    Bp = Ab + j0 + (long long)k0 * lda;                 // L_jk  (opB[p][c] = L_jk(c,p), NAT)
    ldb = lda;
    trn = false;
    Cp = Ab + i0 + (long long)j0 * lda;
    ldc = lda;
    diag = (ii == jj);
  } else {
    const int idx2 = idx - ntri;
    const int ii = idx2 / (k + 1), c = idx2 % (k + 1);
    const int i0 = (k + 1 + ii) * NB, c0 = c * NB;
    rv = min(NB, n - i0);
    cv = NB;
    Ap = Ab + i0 + (long long)k0 * lda;                 // L_ik
    Bp = Xb + k0 + (long long)c0 * ldx;                 // X_kc (opB[p][cc] = X(k0+p,c0+cc), TRN)
    ldb = ldx;
    trn = true;
    Cp = Xb + i0 + (long long)c0 * ldx;
    ldc = ldx;
  }
  // prefetch the C tile (coalesced) while the operands are staged
  double cpre[16];
#pragma unroll
  for (int q = 0; q < 16; ++q) {
    int row, col;
    slot_rc(q, row, col);
    const bool ok = row < rv && col < cv && (!diag || row >= col);
    cpre[q] = ok ? Cp[row + (long long)col * ldc] : 0.0;
  }
  stage<false>(sm.As, Ap, lda, rv, kv);
  if (trn) stage<true>(sm.Bs, Bp, ldb, NB, kv);
  else stage<false>(sm.Bs, Bp, ldb, cv, kv);
  __syncthreads();
  f64x4 acc[2][2];
  mma64(sm.As, sm.Bs, acc);
  __syncthreads();
  acc_to_lds(sm.As, acc);      // As[col][row] = product
  __syncthreads();
  if (idx == 0) {
    // tile (k+1, k+1): updated lower values -> symmetric [row][col] tile in As, then factor
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      int row, col;
      slot_rc(q, row, col);
      cpre[q] -= sm.As[col * LP + row];
    }
    __syncthreads();
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      int row, col;
      slot_rc(q, row, col);
      if (row < rv && col < cv) {
        if (row >= col) {
          sm.As[row * LP + col] = cpre[q];
          sm.As[col * LP + row] = cpre[q];
        }
      } else {
        sm.As[row * LP + col] = (row == col) ? 1.0 : 0.0;
      }
    }
    __syncthreads();
    diag_block(sm, Ab, lda, Xb, ldx, n, k + 1, info, logdet, b);
    return;
  }
#pragma unroll
  for (int q = 0; q < 16; ++q) {
    int row, col;
    slot_rc(q, row, col);
    if (row < rv && col < cv && (!diag || row >= col))
      Cp[row + (long long)col * ldc] = cpre[q] - sm.As[col * LP + row];
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
  hipLaunchKernelGGL(chol_diag_kernel, dim3(batch), dim3(256), 0, stream, A, lda, strideA,
                     Linv, ldinv, strideInv, n, 0, info, logdet);
  GP_CK(hipGetLastError());
  for (int k = 0; k < N; ++k) {
    const int T = N - k - 1;
    if (T + k > 0) {
      hipLaunchKernelGGL(chol_panel_kernel, dim3(T + k, batch), dim3(256), 0, stream, A, lda,
                         strideA, Linv, ldinv, strideInv, n, k, T, info);
      GP_CK(hipGetLastError());
    }
    if (T > 0) {
      const int nt = T * (T + 1) / 2 + T * (k + 1);
      hipLaunchKernelGGL(chol_update_kernel, dim3(nt, batch), dim3(256), 0, stream, A, lda,
                         strideA, Linv, ldinv, strideInv, n, k, T, info, logdet);
      GP_CK(hipGetLastError());
    }
  }
  gpfit_prof_end(GP_PROF_POTRF, stream);
#undef GP_CK
  return 0;
}
