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
// diag_factor_inv: barrier-free symmetric elimination in one wave's registers (L), with a
// second wave applying the same row operations to I (L^-1); see the function.
//
// The kernels are templated on MODE, three C-ABI entry points over one sweep:
//   kPotrfInv (gp_potrf_inv): all of the above;
//   kPotrf    (gp_potrf)    : the L part only (no X_kc panels, no R tiles); D_k goes to a
//                             stream-ordered NB x n scratch (LAPACK dpotrf('L') contract);
//   kTrtri    (gp_trtri)    : the X part only, from a given L: every D_k = L_kk^-1 up front
//                             (trtri_diag_kernel, all blocks in parallel), then per step k the
//                             X_kc panels and R tiles (LAPACK dtrtri('L','N') + padding).
#include "gpfit_common.h"
#include <cstdlib>
#include "gpfit_profile.h"
#include "gpfit_internal.h"
#include "../../include/gpfit.h"


namespace {

constexpr int NB = 64;
constexpr int LP = NB + 1;  // LDS pitch (doubles)
constexpr int kPotrfInv = 0, kPotrf = 1, kTrtri = 2;

// D_k = L_kk^-1: X_kk inside L^-1 (kPotrfInv, kTrtri) or block k of the NB x n scratch
// (kPotrf, ldx = NB).
template <int MODE>
GP_DEV double* dk_ptr(double* Xb, int ldx, int k0) {
  return Xb + (MODE == kPotrf ? 0 : k0) + (long long)k0 * ldx;
}
#ifndef DIAG_PE
#define DIAG_PE 4           // diag factor: steps between step-counter publications
#endif

struct __align__(16) Smem {
  double As[NB * LP];
  double Bs[NB * LP];
  double invs[NB];     // 1 / L_jj
  double red[4];
  int step;            // diag sweep: elimination steps published by wave 0
  int fail;
};

// Operand tiles go global -> registers -> LDS in two phases so every load of a tile (and of
// the other operand) is in flight at once; the tile is walked as (fast, slow) index pairs with
// fast contiguous in memory, as 16-byte loads when the tile is full and aligned.
//   NAT: S[k][x] = src[x + k*ld] (fast = x),   TRN: S[k][x] = src[k + x*ld] (fast = k).
struct OpTile {
  double v[16];
};

GP_DEV void load_op(OpTile& t, const double* __restrict__ src, int ld, int fv, int sv) {
  const int tid = threadIdx.x;
  const bool full = fv == NB && sv == NB && (ld & 1) == 0 && (((size_t)src & 15) == 0);
  if (full) {
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const int g = tid + 256 * q;
      const int f = (g & 31) * 2, sl = g >> 5;
      const double2 x = *reinterpret_cast<const double2*>(src + f + (long long)sl * ld);
      t.v[2 * q] = x.x;
      t.v[2 * q + 1] = x.y;
    }
  } else {
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const int g = tid + 256 * q;
      const int f = (g & 31) * 2, sl = g >> 5;
      const bool ok = sl < sv;
      t.v[2 * q] = (ok && f < fv) ? src[f + (long long)sl * ld] : 0.0;
      t.v[2 * q + 1] = (ok && f + 1 < fv) ? src[f + 1 + (long long)sl * ld] : 0.0;
    }
  }
}

// load_op's full-tile walk with one 64-bit step per slot (the worker's hot path).
GP_DEV void load_full(OpTile& o, const double* __restrict__ src, int ld) {
  const int tid = threadIdx.x;
  const double* p = src + (tid & 31) * 2 + (long long)(tid >> 5) * ld;
  const long long step = 8LL * ld;
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    const double2 x = *reinterpret_cast<const double2*>(p + q * step);
    o.v[2 * q] = x.x;
    o.v[2 * q + 1] = x.y;
  }
}

template <bool TRN>
GP_DEV void store_op(double* S, const OpTile& t) {
  const int tid = threadIdx.x;
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    const int g = tid + 256 * q;
    const int f = (g & 31) * 2, sl = g >> 5;
    if (!TRN) {
      S[sl * LP + f] = t.v[2 * q];
      S[sl * LP + f + 1] = t.v[2 * q + 1];
    } else {
      S[f * LP + sl] = t.v[2 * q];
      S[(f + 1) * LP + sl] = t.v[2 * q + 1];
    }
  }
}

// acc (this wave's 32x32) = sum_k As[k][rows] * Bs[k][cols].  The MFMA's 4 k slots take rows
// k4, k4+16, k4+32, k4+48 rather than 4 consecutive rows.  Measured: the factorisation inside
// gp_fit_predict 3.47-3.49 -> 3.42-3.44 ms (same box, 3 reps, profiles/r01/ab_mma64_kslots.log);
// the tiles' LDS bank-conflict share did not move (21%: it is the transposed tile stores, the
// fragment reads are ds_read2_b64 and conflict-free either way).
GP_DEV void mma64(const double* As, const double* Bs, f64x4 (&acc)[2][2]) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int wr = w >> 1, wc = w & 1, li = lane & 15, lk = lane >> 4;
#pragma unroll
  for (int mi = 0; mi < 2; ++mi)
#pragma unroll
    for (int nj = 0; nj < 2; ++nj) acc[mi][nj] = zero4();
#pragma unroll 4
  for (int k4 = 0; k4 < NB / 4; ++k4) {
    const int k = k4 + (NB / 4) * lk;
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

using LdsSmem = __attribute__((address_space(3))) Smem;

// The one LDS block of every kernel in this file, at namespace scope so that it has the same
// fixed address in all of them and diag_factor_inv (a separate function) addresses it with
// immediate offsets instead of a runtime base register.
__shared__ Smem g_sm;
using lds_double = __attribute__((address_space(3))) double;
typedef double dvec2 __attribute__((ext_vector_type(2)));
using lds_dvec2 = __attribute__((address_space(3))) const dvec2;

// y[r] -= v[r] * x for r in [R0, NB), v[r] read as 16-byte LDS broadcasts from V (v[r] at
// V[r]) in batches of 8, software-pipelined: batch b+1 is issued before batch b is consumed.
// Rows below R0 are untouched (R0 may be odd: the pair holding R0 - 1 is read, half used).
template <int R0>
GP_DEV void bcast_axpy(double (&y)[NB], const lds_double* V, double x) {
  constexpr int P0 = R0 & ~1;              // first pair
  constexpr int NP = (NB - P0) / 2;        // pairs
  constexpr int BATCH = 8;
  constexpr int NBT = (NP + BATCH - 1) / BATCH;
  dvec2 buf[2][BATCH];
  auto load = [&](auto Bt) {
    constexpr int bt = decltype(Bt)::value;
    constexpr int b0 = bt * BATCH;
    constexpr int nb = (NP - b0 < BATCH) ? NP - b0 : BATCH;
    static_for<0, nb, 1>([&](auto Q) {
      constexpr int q = decltype(Q)::value;
      buf[bt & 1][q] = *reinterpret_cast<lds_dvec2*>(&V[P0 + 2 * (b0 + q)]);
    });
  };
  load(std::integral_constant<int, 0>{});
  static_for<0, NBT, 1>([&](auto Bt) {
    constexpr int bt = decltype(Bt)::value;
    if constexpr (bt + 1 < NBT) load(std::integral_constant<int, bt + 1>{});
    constexpr int b0 = bt * BATCH;
    constexpr int nb = (NP - b0 < BATCH) ? NP - b0 : BATCH;
    static_for<0, nb, 1>([&](auto Q) {
      constexpr int q = decltype(Q)::value;
      constexpr int r = P0 + 2 * (b0 + q);
      if constexpr (r >= R0) y[r] = fma(-buf[bt & 1][q].x, x, y[r]);
      y[r + 1] = fma(-buf[bt & 1][q].y, x, y[r + 1]);
    });
  });
}

// Factor + invert the 64x64 tile held (full, symmetric) in T = sm.As[row * LP + col]; all 256
// threads call it.  nb valid rows (rows/cols >= nb are identity padding).  On return T holds L
// (lower, zero upper), U = sm.Bs holds L^-1 (lower, zero upper); returns 0 or the 1-based local
// index of the first non-PD pivot.
//
// Symmetric Gaussian elimination A = Lt D Lt^T (Lt unit lower), no barriers inside the sweep:
//  * wave 0 holds the whole tile, lane c = column c (w[r] = A[r][c], 64 registers), and runs the
//    64 elimination steps.  Step j: pivot p = A[j][j], t_c = A[j][c] / p (lanes c > j, else 0),
//    A[r][c] -= A[r][j] t_c for r > j.  The trailing block stays symmetric, so A[r][j] is lane
//    r's own row-j value: every lane writes w[j] to LDS row S[j] and the column comes back as
//    16-byte broadcast reads (A[j+1][j] = lane j+1's w[j], which the next pivot needs, goes by
//    readlane).  Every row's factor comes from row j (the upper copy): the lower copies are
//    only read back as L at the end, so rounding asymmetry between the two never feeds back.
//    Critical path per column: readlane -> rcp + 2 Newton -> t -> one FMA; the broadcast reads
//    are issued before the chain.  Lane c's column freezes after step c and then holds
//    Lt[.][c] p_c, so L[r][c] = w[r] / sqrt(p_c).  t goes to LDS as the multiplier row M[j]
//    with a step counter after it.
//  * wave 1 applies the same row operations to I, lane c = column c of B:
//    B[r][c] -= M[j][r] B[j][c] (r > j), M[j] read as broadcasts, following the counter.
//    B = Lt^-1 and L^-1 = D^-1/2 B.
// Waves 2-3 only take part in the barriers.  S lives in T's storage (T is in registers during
// the sweep), M in U's (U is written after the barrier that ends both sweeps).
// noinline: inlined into a kernel that also has rolled loops, the 64-step straight-line sweep
// sends LLVM's CodeGenPrepare quadratic (minutes of compile time); as a callee it compiles alone.
__device__ __attribute__((noinline)) int diag_factor_inv(int nb, double* ld_out) {
  LdsSmem& sm = *(LdsSmem*)&g_sm;
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  lds_double* T = sm.As;
  lds_double* S = sm.As;
  lds_double* M = sm.Bs;
  if (tid == 0) sm.step = 0;
  __syncthreads();
  if (wv == 0) {
    double w[NB];
#pragma unroll
    for (int r = 0; r < NB; ++r) w[r] = T[r * LP + lane];
    __syncthreads();   // every wave has read T before S overwrites it
    double piv = 1.0;
    static_for<0, NB, 1>([&](auto J) {
      constexpr int j = decltype(J)::value;
      const double wj = w[j];
      const double p = readlane_f64(wj, j);
      piv = (lane == j) ? p : piv;
      if constexpr (j + 1 < NB) {
        S[j * NB + lane] = wj;
        const double t = (lane > j) ? wj * rcp_nr(p) : 0.0;
        // row j+1's factor A[j+1][j] is taken from the same copy as every other row's: row j
        // (lane j+1's w[j]), never lane j's own row j+1.  The trailing block is only
        // symmetric up to rounding, and mixing the two copies fed that asymmetry back through
        // the multipliers, amplified by |A|/p per step: on grid-like Grams whose pivots fall
        // to ~1e-4 |A| within a few columns (BASELINE C1, d = 1) L was wrong from column ~10.
        w[j + 1] = fma(-readlane_f64(wj, j + 1), t, w[j + 1]);
        M[j * NB + lane] = t;
        if constexpr (j + 2 < NB) bcast_axpy<j + 2>(w, &S[j * NB], t);
        // publish every DIAG_PE steps (and the last): the release store is a scheduling
        // barrier, and between publications the next column's pivot chain can overlap this
        // column's trailing FMAs
        if constexpr ((j + 1) % DIAG_PE == 0 || j + 2 == NB)
          __hip_atomic_store((int*)&sm.step, j + 1, __ATOMIC_RELEASE,
                             __HIP_MEMORY_SCOPE_WORKGROUP);
      }
    });
    const double rs = rsqrt_nr(piv);
    sm.invs[lane] = rs;
    const bool badc = lane < nb && (!(piv > 0.0) || !isfinite(piv));
    const unsigned long long badm = __ballot(badc);
    double lg = (lane < nb) ? log(piv) : 0.0;
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) lg += __shfl_xor(lg, off, 64);
    if (lane == 0) {
      sm.fail = badm ? __ffsll((long long)badm) : 0;
      sm.red[0] = lg;
    }
#pragma unroll
    for (int r = 0; r < NB; ++r)
      T[r * LP + lane] = (r > lane) ? w[r] * rs : ((r == lane) ? piv * rs : 0.0);
    __syncthreads();
  } else if (wv == 1) {
    __syncthreads();
    double bq[NB];
#pragma unroll
    for (int r = 0; r < NB; ++r) bq[r] = (r == lane) ? 1.0 : 0.0;
#ifndef DIAG_PROBE_NO_INV   // tools/probe_diag.hip only: time wave 0's sweep alone
    static_for<0, NB - 1, 1>([&](auto J) {
      constexpr int j = decltype(J)::value;
      if constexpr (j % DIAG_PE == 0)   // wave 0 publishes every DIAG_PE steps
        lds_wait_ge((int*)&sm.step, (j + DIAG_PE < NB - 1) ? j + DIAG_PE : NB - 1);
      bcast_axpy<j + 1>(bq, &M[j * NB], bq[j]);
    });
#endif
    __syncthreads();   // invs from wave 0; every M read done
#pragma unroll
    for (int r = 0; r < NB; ++r) sm.Bs[r * LP + lane] = bq[r] * sm.invs[r];
  } else {
    __syncthreads();
    __syncthreads();
  }
  __syncthreads();
  const int f = sm.fail;
  if (ld_out) *ld_out = sm.red[0];
  return f;
}

// Factor diagonal block k whose (updated, symmetric) tile is in sm.As as [row][col]; write
// L_kk into A, D_k into X (dk_ptr), accumulate logdet, set info.
template <int MODE>
GP_DEV void diag_block(Smem& sm, double* __restrict__ Ab, int lda, double* __restrict__ Xb,
                       int ldx, int n, int k, int* info, double* logdet, int b) {
  const int k0 = k * NB, nb = min(NB, n - k0);
  double lg = 0.0;
  const int f = diag_factor_inv(nb, &lg);
  if (f) {
    if (threadIdx.x == 0 && info) info[b] = k0 + f;
    return;
  }
  if (threadIdx.x == 0 && logdet) logdet[b] += lg;
  double* Akk = Ab + k0 + (long long)k0 * lda;
  double* Xkk = dk_ptr<MODE>(Xb, ldx, k0);
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

template <int MODE>
__global__ __launch_bounds__(256, 2) void chol_diag_kernel(
    double* __restrict__ A, int lda, long long sA, double* __restrict__ X, int ldx,
    long long sX, int n, int k, int* __restrict__ info, double* __restrict__ logdet) {
  const int b = blockIdx.x;
  if (info && info[b] != 0) return;
  Smem& sm = g_sm;
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
  diag_block<MODE>(sm, Ab, lda, X + b * sX, ldx, n, k, info, logdet, b);
}

// kTrtri: D_k = L_kk^-1 for every diagonal block at once (grid N x batch, one wave each).
// Lane c owns column c of D_k and runs the column-oriented forward substitution
//   x_j <- x_j / L_jj ;  x_r -= L_rj x_j (r > j)
// with column j of L_kk read as 16-byte LDS broadcasts (bcast_axpy).  info[b] = first exactly
// zero (or non-finite) diagonal entry, 1-based (LAPACK dtrtri).
__global__ __launch_bounds__(64) void trtri_diag_kernel(
    const double* __restrict__ A, int lda, long long sA, double* __restrict__ X, int ldx,
    long long sX, int n, int* __restrict__ info) {
  LdsSmem& sm = *(LdsSmem*)&g_sm;
  const int k = blockIdx.x, b = blockIdx.y;
  const int k0 = k * NB, nb = min(NB, n - k0);
  const int lane = threadIdx.x;
  const double* Akk = A + b * sA + k0 + (long long)k0 * lda;
  lds_double* Lc = sm.As;        // Lc[j * NB + r] = L[r][j], identity padding past nb
#pragma unroll 4
  for (int j = 0; j < NB; ++j) {
    double v;
    if (j < nb && lane < nb) v = (lane >= j) ? Akk[lane + (long long)j * lda] : 0.0;
    else v = (lane == j) ? 1.0 : 0.0;
    Lc[j * NB + lane] = v;
  }
  __syncthreads();
  const double dj = Lc[lane * NB + lane];
  const bool bad = lane < nb && !(dj != 0.0 && isfinite(dj));
  const unsigned long long badm = __ballot(bad);
  if (badm) {
    if (lane == 0 && info) atomicMin(&info[b], k0 + __ffsll((long long)badm));
    return;
  }
  sm.invs[lane] = 1.0 / dj;
  __syncthreads();
  double x[NB];
#pragma unroll
  for (int r = 0; r < NB; ++r) x[r] = (r == lane) ? 1.0 : 0.0;
  static_for<0, NB, 1>([&](auto J) {
    constexpr int j = decltype(J)::value;
    x[j] *= sm.invs[j];
    if constexpr (j + 1 < NB) bcast_axpy<j + 1>(x, &Lc[j * NB], x[j]);
  });
  // transpose through LDS (Bs[c][r]) so the global stores run down columns
  lds_double* T = sm.Bs;
#pragma unroll
  for (int r = 0; r < NB; ++r) T[lane * LP + r] = x[r];
  __syncthreads();
  double* Xkk = X + b * sX + k0 + (long long)k0 * ldx;
  if (lane < nb)
    for (int c = 0; c < nb; ++c) Xkk[lane + (long long)c * ldx] = T[c * LP + lane];
}

template <int MODE>
__global__ __launch_bounds__(256) void chol_panel_kernel(
    double* __restrict__ A, int lda, long long sA, double* __restrict__ X, int ldx,
    long long sX, int n, int k, int nbelow, const int* __restrict__ info) {
  const int b = blockIdx.y;
  if (info && info[b] != 0) return;
  Smem& sm = g_sm;
  const int k0 = k * NB, kv = min(NB, n - k0);
  double* Ab = A + b * sA;
  double* Xb = X + b * sX;
  const double* Dk = dk_ptr<MODE>(Xb, ldx, k0);      // D_k (lower, zero upper)
  // both tile kinds through one code path (a short kernel's cost is largely the code a cold
  // instruction cache streams, see upd_load):
  //   L_ik = A_ik D_k^T : opA = A_ik (NAT, rv rows), opB[p][c] = D_k(c,p) (NAT), C = A_ik
  //   X_kc = D_k R_kc   : opA = D_k (NAT),          opB[p][c] = R_kc(p,c) (TRN), C = R_kc
  const bool lt = MODE == kTrtri ? false : (MODE == kPotrf ? true : (int)blockIdx.x < nbelow);
  const double *pa, *pb;
  double* pc;
  int la, av, rv, cv;
  if (lt) {
    const int i0 = (k + 1 + blockIdx.x) * NB;
    rv = min(NB, n - i0);
    cv = kv;
    pc = Ab + i0 + (long long)k0 * lda;
    pa = pc;
    la = lda;
    av = rv;
    pb = Dk;
  } else {
    const int c0 = ((int)blockIdx.x - (MODE == kTrtri ? 0 : nbelow)) * NB;
    rv = kv;
    cv = NB;
    pc = Xb + k0 + (long long)c0 * ldx;
    pa = Dk;
    la = ldx;
    av = kv;
    pb = pc;
  }
  const int ld_c = lt ? lda : ldx;
  OpTile ta, tb;
  const bool full = rv == NB && cv == NB && kv == NB && ((lda | ldx) & 1) == 0 &&
                    ((((size_t)pa) | ((size_t)pb)) & 15) == 0;
  if (full) {
    load_full(ta, pa, la);
    load_full(tb, pb, ldx);
  } else {
    load_op(ta, pa, la, av, kv);
    if (lt) load_op(tb, pb, ldx, kv, kv);
    else load_op(tb, pb, ldx, kv, NB);
  }
  store_op<false>(sm.As, ta);
  if (lt) store_op<false>(sm.Bs, tb);
  else store_op<true>(sm.Bs, tb);
  __syncthreads();
  f64x4 acc[2][2];
  mma64(sm.As, sm.Bs, acc);
  __syncthreads();
  acc_to_lds(sm.As, acc);
  __syncthreads();
  const int tid = threadIdx.x;
  if (full) {
    const int row = tid & 63, col = tid >> 6;
    double* c = pc + row + (long long)col * ld_c;
    const long long cs = 4LL * ld_c;
#pragma unroll
    for (int q = 0; q < 16; ++q) c[q * cs] = sm.As[(col + 4 * q) * LP + row];
  } else {
#pragma unroll 4
    for (int q = 0; q < 16; ++q) {
      int row, col;
      slot_rc(q, row, col);
      if (row < rv && col < cv) pc[row + (long long)col * ld_c] = sm.As[col * LP + row];
    }
  }
}

// One tile of the trailing update of step k (tile index idx over the T(T+1)/2 lower tiles of
// A's trailing matrix, then the T(k+1) tiles of R): C -= opA * opB.
struct UpdTile {
  const double *Ap, *Bp;
  double* Cp;
  int ldb, ldc, rv, cv;
  bool diag, trn, full;   // full: 64 x 64 off-diagonal, 16-byte aligned (no per-element checks)
};

GP_DEV UpdTile upd_tile(double* Ab, int lda, double* Xb, int ldx, int n, int k, int T, int idx) {
  const int k0 = k * NB;
  const int ntri = T * (T + 1) / 2;
  UpdTile t;
  if (idx < ntri) {
    int ii = (int)((sqrt(8.0 * idx + 1.0) - 1.0) * 0.5);
    while (ii * (ii + 1) / 2 > idx) --ii;
    while ((ii + 1) * (ii + 2) / 2 <= idx) ++ii;
    const int jj = idx - ii * (ii + 1) / 2;
    const int i0 = (k + 1 + ii) * NB, j0 = (k + 1 + jj) * NB;
    t.rv = min(NB, n - i0);
    t.cv = min(NB, n - j0);
    t.Ap = Ab + i0 + (long long)k0 * lda;               // L_ik
    t.Bp = Ab + j0 + (long long)k0 * lda;               // L_jk  (opB[p][c] = L_jk(c,p), NAT)
    t.ldb = lda;
    t.trn = false;
    t.Cp = Ab + i0 + (long long)j0 * lda;
    t.ldc = lda;
    t.diag = (ii == jj);
  } else {
    const int idx2 = idx - ntri;
    const int ii = idx2 / (k + 1), c = idx2 % (k + 1);
    const int i0 = (k + 1 + ii) * NB, c0 = c * NB;
    t.rv = min(NB, n - i0);
    t.cv = NB;
    t.Ap = Ab + i0 + (long long)k0 * lda;               // L_ik
    t.Bp = Xb + k0 + (long long)c0 * ldx;               // X_kc (opB[p][cc] = X(k0+p,c0+cc), TRN)
    t.ldb = ldx;
    t.trn = true;
    t.Cp = Xb + i0 + (long long)c0 * ldx;
    t.ldc = ldx;
    t.diag = false;
  }
  t.full = t.rv == NB && t.cv == NB && !t.diag && ((lda | t.ldb | t.ldc) & 1) == 0 &&
           ((((size_t)t.Ap) | ((size_t)t.Bp)) & 15) == 0;
  return t;
}

// Global loads of one update tile into registers: the C tile (coalesced) and both operands.
// Full tiles take a branch-free path: the code a cold instruction cache has to stream per
// launch is what bounds these short kernels (tools/probe_update.hip: a worker's first tile
// 22 us, its second 7 us).
GP_DEV void upd_load(const UpdTile& t, int lda, int kv, OpTile& ta, OpTile& tb,
                     double (&cpre)[16]) {
  const int tid = threadIdx.x;
  if (t.full) {
    const double* c = t.Cp + (tid & 63) + (long long)(tid >> 6) * t.ldc;
    const long long cs = 4LL * t.ldc;
#pragma unroll
    for (int q = 0; q < 16; ++q) cpre[q] = c[q * cs];
    load_full(ta, t.Ap, lda);
    load_full(tb, t.Bp, t.ldb);
    return;
  }
#pragma unroll
  for (int q = 0; q < 16; ++q) {
    int row, col;
    slot_rc(q, row, col);
    const bool ok = row < t.rv && col < t.cv && (!t.diag || row >= col);
    cpre[q] = ok ? t.Cp[row + (long long)col * t.ldc] : 0.0;
  }
  load_op(ta, t.Ap, lda, t.rv, kv);
  if (t.trn) load_op(tb, t.Bp, t.ldb, kv, NB);
  else load_op(tb, t.Bp, t.ldb, t.cv, kv);
}

// C = cpre - product (product in Cs[col][row]), branch-free for full tiles.
GP_DEV void upd_store(const UpdTile& t, const double (&cpre)[16], const double* Cs) {
  const int tid = threadIdx.x;
  if (t.full) {
    const int row = tid & 63, col = tid >> 6;
    double* c = t.Cp + row + (long long)col * t.ldc;
    const long long cs = 4LL * t.ldc;
#pragma unroll
    for (int q = 0; q < 16; ++q) c[q * cs] = cpre[q] - Cs[(col + 4 * q) * LP + row];
    return;
  }
#pragma unroll
  for (int q = 0; q < 16; ++q) {
    int row, col;
    slot_rc(q, row, col);
    if (row < t.rv && col < t.cv && (!t.diag || row >= col))
      t.Cp[row + (long long)col * t.ldc] = cpre[q] - Cs[col * LP + row];
  }
}

// Trailing update of step k.  kPotrfInv / kPotrf: block 0 owns tile (k+1, k+1) and then
// factors it (lookahead), blocks 1.. walk the other tiles with stride gridDim.x - 1; kTrtri
// (no A tiles, D_k precomputed): every block walks the R tiles with stride gridDim.x.  The host
// caps the grid at two resident blocks per CU; each worker loads the next tile's operands and C
// into registers while the current tile's MFMAs run.
template <int MODE>
__global__ __launch_bounds__(256, 2) void chol_update_kernel(
    double* __restrict__ A, int lda, long long sA, double* __restrict__ X, int ldx,
    long long sX, int n, int k, int T, int* __restrict__ info, double* __restrict__ logdet) {
  const int b = blockIdx.y;
  if (info && info[b] != 0) return;
  Smem& sm = g_sm;
  const int k0 = k * NB, kv = min(NB, n - k0);
  double* Ab = A + b * sA;
  double* Xb = X + b * sX;
  const int ntri = T * (T + 1) / 2;
  // tile index space of upd_tile: [0, ntri) A tiles, [ntri, ntri + T(k+1)) R tiles
  const int t_lo = MODE == kTrtri ? ntri : 0;
  const int t_hi = ntri + (MODE == kPotrf ? 0 : T * (k + 1));
  const bool look = MODE != kTrtri;
  if (!look || blockIdx.x != 0) {
    // one call site each for the loads, the MFMAs, the epilogue and the LDS stores (compact
    // code), software-pipelined: tile i's loads are issued before tile i - stride's MFMAs
    const int stride = look ? gridDim.x - 1 : gridDim.x;
    OpTile ta, tb;
    double cpre[16], cnext[16];
    UpdTile cur, prev;
    bool started = false;
    for (int i = t_lo + blockIdx.x;; i += stride) {
      const bool have = i < t_hi;                     // uniform
      if (have) {
        cur = upd_tile(Ab, lda, Xb, ldx, n, k, T, i);
        upd_load(cur, lda, kv, ta, tb, cnext);
      }
      if (started) {
        f64x4 acc[2][2];
        mma64(sm.As, sm.Bs, acc);
        __syncthreads();
        acc_to_lds(sm.As, acc);                       // As[col][row] = product
        __syncthreads();
        upd_store(prev, cpre, sm.As);
      }
      if (!have) break;
      __syncthreads();                                // the epilogue has read As
      store_op<false>(sm.As, ta);
      if (cur.trn) store_op<true>(sm.Bs, tb);
      else store_op<false>(sm.Bs, tb);
      __syncthreads();
#pragma unroll
      for (int q = 0; q < 16; ++q) cpre[q] = cnext[q];
      prev = cur;
      started = true;
    }
    return;
  }
  // block 0: tile (k+1, k+1) (an A tile on the diagonal), then its factorisation
  const UpdTile t = upd_tile(Ab, lda, Xb, ldx, n, k, T, 0);
  const int rv = t.rv, cv = t.cv;
  double cpre[16];
  {
    OpTile ta, tb;
    upd_load(t, lda, kv, ta, tb, cpre);
    store_op<false>(sm.As, ta);
    store_op<false>(sm.Bs, tb);
  }
  __syncthreads();
  f64x4 acc[2][2];
  mma64(sm.As, sm.Bs, acc);
  __syncthreads();
  acc_to_lds(sm.As, acc);      // As[col][row] = product
  __syncthreads();
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
  diag_block<MODE>(sm, Ab, lda, Xb, ldx, n, k + 1, info, logdet, b);
}

// info sentinel (memset 0x7f) -> 0 for problems whose diagonal was fine (gp_trtri).
__global__ void trtri_info_kernel(int* __restrict__ info, int batch) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b < batch && info[b] == 0x7f7f7f7f) info[b] = 0;
}

}  // namespace

static_assert(GPFIT_POTRF_NB == NB, "gpfit_internal.h must match the blocking");

// Grid of chol_update_kernel for nt tiles per problem, capped at two resident blocks per CU
// over the whole batch so every worker is resident and walks several tiles.
static int update_grid(int nt, int batch) {
  static const int cap_all = [] {
    int dev = 0, ncu = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
        ncu <= 0)
      ncu = 256;
    return 2 * ncu;
  }();
  int cap = cap_all / (batch > 0 ? batch : 1);
  if (cap < 2) cap = 2;
  return nt < cap ? nt : cap;
}

#define GP_CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) return GPFIT_ERR_HIP - (int)e_; } while (0)

// The blocked sweep shared by the three entry points (arguments already validated; X is L^-1
// (kPotrfInv, kTrtri, zero-filled by the caller) or the D_k scratch (kPotrf)).
template <int MODE>
static int potrf_sweep(double* A, int n, int lda, long long sA, double* X, int ldx, long long sX,
                       int batch, int* info, double* logdet, hipStream_t stream, int k_ev,
                       hipEvent_t ev) {
  const int N = gp_ceil_div(n, NB);
  if (MODE != kTrtri) {   // kTrtri: every D_k is made up front by trtri_diag_kernel
    hipLaunchKernelGGL(chol_diag_kernel<MODE>, dim3(batch), dim3(256), 0, stream, A, lda, sA, X,
                       ldx, sX, n, 0, info, logdet);
    GP_CK(hipGetLastError());
  }
  for (int k = 0; k < N; ++k) {
    const int T = N - k - 1;
    const int npanel = MODE == kPotrfInv ? T + k : (MODE == kPotrf ? T : k);
    if (npanel > 0) {
      hipLaunchKernelGGL(chol_panel_kernel<MODE>, dim3(npanel, batch), dim3(256), 0, stream, A,
                         lda, sA, X, ldx, sX, n, k, T, info);
      GP_CK(hipGetLastError());
    }
    if (T > 0) {
      const int nt = (MODE == kTrtri ? 0 : T * (T + 1) / 2) + (MODE == kPotrf ? 0 : T * (k + 1));
      hipLaunchKernelGGL(chol_update_kernel<MODE>, dim3(update_grid(nt, batch), batch), dim3(256), 0, stream, A,
                         lda, sA, X, ldx, sX, n, k, T, info, logdet);
      GP_CK(hipGetLastError());
    }
    if (ev && (k == k_ev || (k == N - 1 && k_ev >= N))) GP_CK(hipEventRecord(ev, stream));
  }
  return 0;
}

// Zero L^-1 (upper triangle + padding): one memset for a packed batch, else one 2-D memset per
// problem.
static hipError_t zero_linv(double* Linv, int npad, int ldinv, long long strideInv, int batch,
                            hipStream_t stream) {
  if (ldinv == npad && (batch == 1 || strideInv == (long long)npad * npad))
    return hipMemsetAsync(Linv, 0, sizeof(double) * ((long long)(batch - 1) * strideInv +
                                                     (long long)ldinv * npad), stream);
  for (int b = 0; b < batch; ++b) {
    hipError_t e = hipMemset2DAsync(Linv + b * strideInv, sizeof(double) * ldinv, 0,
                                    sizeof(double) * npad, npad, stream);
    if (e != hipSuccess) return e;
  }
  return hipSuccess;
}

extern "C" int gp_potrf_inv(double* A, int n, int lda, long long strideA, double* Linv,
                            int ldinv, long long strideInv, int batch, int* info,
                            double* logdet, hipStream_t stream) {
  return gpfit_potrf_inv_event(A, n, lda, strideA, Linv, ldinv, strideInv, batch, info, logdet,
                               stream, -1, nullptr);
}

int gpfit_potrf_inv_event(double* A, int n, int lda, long long strideA, double* Linv,
                          int ldinv, long long strideInv, int batch, int* info, double* logdet,
                          hipStream_t stream, int k_ev, hipEvent_t ev) {
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
  if (info) GP_CK(hipMemsetAsync(info, 0, sizeof(int) * batch, stream));
  if (logdet) GP_CK(hipMemsetAsync(logdet, 0, sizeof(double) * batch, stream));
  GP_CK(zero_linv(Linv, npad, ldinv, strideInv, batch, stream));
  gpfit_prof_begin(GP_PROF_POTRF, stream);
  const int rc = potrf_sweep<kPotrfInv>(A, n, lda, strideA, Linv, ldinv, strideInv, batch, info,
                                        logdet, stream, k_ev, ev);
  gpfit_prof_end(GP_PROF_POTRF, stream);
  return rc;
}

extern "C" int gp_potrf(double* A, int n, int lda, long long strideA, int batch, int* info,
                        double* logdet, hipStream_t stream) {
  if (!A) return -1;
  if (n < 0) return -2;
  if (lda < n || lda < 1) return -3;
  if (batch > 1 && strideA < (long long)lda * n) return -4;
  if (batch < 0) return -5;
  if (n == 0 || batch == 0) return 0;
  if (info) GP_CK(hipMemsetAsync(info, 0, sizeof(int) * batch, stream));
  if (logdet) GP_CK(hipMemsetAsync(logdet, 0, sizeof(double) * batch, stream));
  // D_k scratch: NB x (N NB) per problem, stream-ordered (freed when the sweep has run)
  const int N = gp_ceil_div(n, NB);
  const long long sD = (long long)NB * N * NB;
  double* D = nullptr;
  GP_CK(hipMallocAsync(reinterpret_cast<void**>(&D), sizeof(double) * sD * batch, stream));
  const int rc = potrf_sweep<kPotrf>(A, n, lda, strideA, D, NB, sD, batch, info, logdet, stream,
                                     -1, nullptr);
  GP_CK(hipFreeAsync(D, stream));
  return rc;
}

extern "C" int gp_trtri(const double* L, int n, int ldl, long long strideL, double* Linv,
                        int ldinv, long long strideInv, int batch, int* info,
                        hipStream_t stream) {
  if (!L) return -1;
  if (n < 0) return -2;
  if (ldl < n || ldl < 1) return -3;
  if (batch > 1 && strideL < (long long)ldl * n) return -4;
  if (!Linv) return -5;
  const int npad = gp_padded_n(n);
  if (ldinv < npad || ldinv < 1) return -6;
  if (batch > 1 && strideInv < (long long)ldinv * npad) return -7;
  if (batch < 0) return -8;
  if (n == 0 || batch == 0) return 0;
  // trtri_diag_kernel lowers info[b] (atomicMin) from a "none" sentinel; the sweep's kernels
  // then skip every problem with info != 0
  if (info) GP_CK(hipMemsetAsync(info, 0x7f, sizeof(int) * batch, stream));
  GP_CK(zero_linv(Linv, npad, ldinv, strideInv, batch, stream));
  hipLaunchKernelGGL(trtri_diag_kernel, dim3(gp_ceil_div(n, NB), batch), dim3(64), 0, stream,
                     L, ldl, strideL, Linv, ldinv, strideInv, n, info);
  GP_CK(hipGetLastError());
  if (info) {
    hipLaunchKernelGGL(trtri_info_kernel, dim3(gp_ceil_div(batch, 256)), dim3(256), 0, stream,
                       info, batch);
    GP_CK(hipGetLastError());
  }
  return potrf_sweep<kTrtri>(const_cast<double*>(L), n, ldl, strideL, Linv, ldinv, strideInv,
                             batch, info, nullptr, stream, -1, nullptr);
}
#undef GP_CK
