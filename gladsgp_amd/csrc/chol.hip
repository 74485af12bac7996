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
#include <vector>
#include "gpfit_profile.h"
#include "gpfit_internal.h"
#include "../../include/gpfit.h"

#define GP_HD __host__ __device__

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

// mma64 with the B operand read transposed: acc = sum_k As[k][rows] * Bt[cols][k] (Bt held
// [row][col], e.g. a factor tile as diag_factor_blk leaves it).  Lanes li of a fragment read
// sit LP = 65 doubles apart: 16 distinct bank pairs, and the k slots 16 apart put the other
// lane groups on the other 32 banks (conflict-free).
GP_DEV void mma64_bt(const double* As, const double* Bt, f64x4 (&acc)[2][2]) {
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
    const double b0 = Bt[(wc * 32 + li) * LP + k], b1 = Bt[(wc * 32 + 16 + li) * LP + k];
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
// chain: L_j+1,j as [p][r] (opA layout) between steps, the two-wave leaf's multipliers during
// the diagonal factor; workers: the XT pair's third tile
__shared__ double g_keep[NB * LP];
// gp_loglik in-chain mode only (referenced by pp_kernel<true> alone): [0, 64) z_{j-1} (chain)
// or the current term's z_k (DP task), [64, 128) y_j, [128, 384) four 64-row partial sums
__shared__ double g_ll[6 * NB];
constexpr int kLLZ = 0, kLLY = NB, kLLPart = 2 * NB;
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
// TAG: one instantiation per caller family (the sweep's 2-wave/SIMD kernels, the persistent
// 1-wave/SIMD one), so each is register-allocated for its own occupancy.
template <int TAG>
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

// ---- Blocked 64x64 factor + inverse (the persistent chain's diagonal step) -------------------
// Same contract as diag_factor_inv (T = sm.As full symmetric [row][col] with identity padding
// past nb; on return T = L, U = sm.Bs = L^-1, both lower with zero upper), on 16 x 16 blocks:
//   for b = 0..3:  leaf16(b)                        wave 0: L_bb, Dinv_b = L_bb^-1
//                  L_rb = A_rb Dinv_b^T (r > b)     waves 1-3, one MFMA block each
//                  A_rs -= L_rb L_sb^T (b < s <= r) wave 0 takes (b+1, b+1) and goes straight on
//                                                   to the next leaf; waves 1-3 the rest
//   X_rc = -Dinv_r sum_{k=c}^{r-1} L_rk X_kc        row r of L^-1 by waves 1-2 beside leaf r+1,
//                                                   the last row by waves 0-2 after leaf 3
// The leaf is the 16-column symmetric elimination of diag_factor_inv held in ONE wave's
// registers (lanes 0-15 = columns of A, lanes 16-31 = columns of I for the inverse, same row
// operations), the broadcasts are readlanes instead of LDS round trips, and every block
// product is 4 v_mfma_f64_16x16x4.

// acc += (negA ? -A : A) B over one 16 x 16 x 16 block; A(i,k) = Ab[i*ai + k*ak],
// B(k,c) = Bb[k*bk + c*bc]  (C layout: lane l, reg q holds C[(l >> 4) + 4q][l & 15]).
GP_DEV void mm16(f64x4& acc, const lds_double* Ab, int ai, int ak, const lds_double* Bb, int bk,
                 int bc, bool negA) {
  const int lane = threadIdx.x & 63, i = lane & 15, kk = lane >> 4;
#pragma unroll
  for (int k0 = 0; k0 < 16; k0 += 4) {
    double a = Ab[i * ai + (k0 + kk) * ak];
    const double b = Bb[(k0 + kk) * bk + i * bc];
    acc = mfma16x16x4(negA ? -a : a, b, acc);
  }
}
GP_DEV f64x4 ld16(const lds_double* Cb) {          // row-major block, pitch LP
  const int lane = threadIdx.x & 63;
  f64x4 a;
#pragma unroll
  for (int q = 0; q < 4; ++q) a[q] = Cb[((lane >> 4) + 4 * q) * LP + (lane & 15)];
  return a;
}
GP_DEV void st16(lds_double* Cb, const f64x4& a, double sg) {
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int q = 0; q < 4; ++q) Cb[((lane >> 4) + 4 * q) * LP + (lane & 15)] = sg * a[q];
}

// One wave: factor + invert the 16 x 16 block at (o, o).  Writes L_bb into T's block and
// Dinv_b into U's block (lower, zero upper) and the 16 pivots p_c (L_cc = sqrt(p_c)) into
// piv[o + c]; the caller checks them.
//
// The block lives in MFMA C layout (lane l, reg q = element [(l >> 4) + 4q][l & 15]), so row j
// of the block is register j / 4 of lanes 16 (j % 4) .. + 15, which is at once the A operand's
// column k = j % 4 (A[i][k] from lane 16k + i) and the B operand's row k (B[k][c] from lane
// 16k + c).  Elimination step j is therefore ONE v_mfma_f64_16x16x4 on the whole block,
//   A[i][c] -= A[j][i] (A[j][c] / p_j)    (i, c > j; the other three k lanes zero),
// and one more applies the same row operation to W (= I at the start): W[i][c] -= m_i W[j][c],
// m_i = A[j][i] / p_j.  Both factors come from row j only, the same copy for every row (the
// rounding asymmetry of the trailing block never feeds back; see diag_factor_inv).  At the end
// A's lower triangle holds Lt[r][c] p_c and W = Lt^-1:  L = A D^-1/2 (columns), L^-1 = D^-1/2 W
// (rows).  Per step the dependent chain is readlane -> rcp + 2 Newton -> select -> MFMA; the
// register-resident form with one readlane pair per row and step (and the SGPR traffic that
// came with it) measured 8.5k cycles per leaf (tools/dbg/leaf_micro.hip).  Splitting the W
// row operations onto a second wave (multipliers handed over through LDS, a step counter)
// measured slower inside the chain: 14.6 vs 12.4 us per 64 x 64 factor
// (profiles/r03/pp_trace_pp4_pairs_splitleaf.txt).
GP_DEV void leaf16(lds_double* T, lds_double* U, int o, lds_double* piv) {
  const int lane = threadIdx.x & 63;
  const int r0 = lane >> 4, c = lane & 15;
  f64x4 A = ld16(T + o * LP + o);
  f64x4 W;
#pragma unroll
  for (int q = 0; q < 4; ++q) W[q] = (r0 + 4 * q == c) ? 1.0 : 0.0;
  double colpiv = 1.0;          // p_c of this lane's column
  double rowpiv[4];             // p_r of rows r0 + 4q
#pragma unroll
  for (int q = 0; q < 4; ++q) rowpiv[q] = 1.0;
  static_for<0, 16, 1>([&](auto J) {
    constexpr int j = decltype(J)::value;
    constexpr int q = j >> 2, k = j & 3;
    const double p = readlane_f64(A[q], 16 * k + j);
    colpiv = (c == j) ? p : colpiv;
    rowpiv[q] = (r0 == k) ? p : rowpiv[q];
    if constexpr (j < 15) {
      const double rp = rcp_nr(p);
      const bool sel = r0 == k && c > j;
      const double rowj = A[q];
      const double a = sel ? -rowj : 0.0;
      const double m = sel ? rowj * rp : 0.0;
      const double wj = W[q];
      A = mfma16x16x4(a, m, A);
      W = mfma16x16x4(-m, wj, W);
    }
  });
  const double rsc = rsqrt_nr(colpiv);
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int r = r0 + 4 * q;
    const double rsr = rsqrt_nr(rowpiv[q]);
    T[(o + r) * LP + o + c] = r >= c ? A[q] * rsc : 0.0;
    U[(o + r) * LP + o + c] = r >= c ? W[q] * rsr : 0.0;
  }
  if (lane < 16) piv[o + c] = colpiv;
}

#ifndef LEAF_MASKED
#define LEAF_MASKED 1
#endif
#ifndef PP_LEAF_BLOCKED
#define PP_LEAF_BLOCKED 1   // 0: leaf16 (one MFMA per column), 1: leaf16_blocked
#endif

// Blocked leaf (PP_LEAF_BLOCKED, the default): the same elimination four columns at a time.
// At the start of block q (columns 4q .. 4q+3, whose rows are register q: lane 16k + c = row
// 4q + k, column c) every row group receives all four of the block's rows (four lane shuffles
// for A, four for W), so lane 16k + c holds A[4q..4q+3][c]; the block's four elimination steps
// are then lane-local FMAs whose multipliers A[j][4q+k] / p_j are wave-uniform (readlanes of
// row j), and each lane takes its own row back.  ONE MFMA then applies the block's rank-4 update
// to every later row (A operand: lane 16k + i holds -M[i][4q+k] = -A[4q+k][i] / p_{4q+k} for
// i > 4q+3; B operand: the block's rows, masked to c > 4q + k), and one more to W.  Both
// factors still come from row j only.  The MFMA's latency is paid once per four columns instead
// of once per column: 4.08k vs 5.11k cycles per leaf, 23.4k vs 28.0k per 64 x 64 factor
// (tools/dbg/leafonly_micro.hip, diag_micro.hip); gp_potrf_inv n = 4096 1.813 -> 1.728 ms,
// 1024 x 32 0.997 -> 0.955, 2048 x 4 1.036 -> 0.988, fit 1.49-1.56 -> 1.45-1.47 ms per sweep
// (profiles/r04/r04f_*).  Broadcasting row j per step instead (LDS shuffles: 23.6k; gfx950's
// v_permlane16/32_swap: 28.4k) was no faster, nor was replaying W on wave 3 (idle during the
// leaves) from multipliers handed over through LDS per block: 28.0k.
GP_DEV void leaf16_blocked(lds_double* T, lds_double* U, int o, lds_double* piv) {
  const int lane = threadIdx.x & 63;
  const int r0 = lane >> 4, c = lane & 15;
  f64x4 A = ld16(T + o * LP + o);
  f64x4 W;
#pragma unroll
  for (int q = 0; q < 4; ++q) W[q] = (r0 + 4 * q == c) ? 1.0 : 0.0;
  double colpiv = 1.0;
  double rowpiv[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) rowpiv[q] = 1.0;
  static_for<0, 4, 1>([&](auto Q) {
    constexpr int q = decltype(Q)::value;
    double t[4], tw[4], rpk[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      t[k] = __shfl(A[q], 16 * k + c);
      tw[k] = __shfl(W[q], 16 * k + c);
      rpk[k] = 1.0;
    }
    static_for<0, 4, 1>([&](auto JJ) {
      constexpr int jj = decltype(JJ)::value;
      constexpr int j = 4 * q + jj;
      const double p = readlane_f64(t[jj], j);
      colpiv = (c == j) ? p : colpiv;
      rowpiv[q] = (r0 == jj) ? p : rowpiv[q];
#if LEAF_MASKED
      // row j masked to the columns it still updates (c > j) while the pivot's reciprocal is
      // formed: the update below then needs no select on its dependency chain (columns c <= j
      // get fma(-m, 0, t) = t)
      const double tjm = (c > j) ? t[jj] : 0.0;
#endif
      if constexpr (j < 15) {
        // 1 / p_j: v_rcp_f64's estimate (~2^-26: 1e-8 residuals alone) + one Newton step, as
        // accurate as two here (|LL^T - G| and |L^-1 L - I| unchanged on the micro-benchmark's
        // tiles) and one dependent FMA pair shorter: 22.7k vs 23.4k cycles per 64 x 64 factor
        // (profiles/r04/leaf_micro_nr*.log)
#ifndef LEAF_NR
#define LEAF_NR 1
#endif
        double rp = __builtin_amdgcn_rcp(p);
        if constexpr (LEAF_NR >= 1) rp = fma(rp, fma(-p, rp, 1.0), rp);
        if constexpr (LEAF_NR >= 2) rp = fma(rp, fma(-p, rp, 1.0), rp);
        rpk[jj] = rp;
        static_for<jj + 1, 4, 1>([&](auto K) {
          constexpr int k = decltype(K)::value;
          const double m = readlane_f64(t[jj], 4 * q + k) * rp;     // A[j][4q+k] / p_j
#if LEAF_MASKED
          t[k] = fma(-m, tjm, t[k]);
#else
          t[k] = (c > j) ? fma(-m, t[jj], t[k]) : t[k];
#endif
          tw[k] = fma(-m, tw[jj], tw[k]);
        });
      }
    });
    double mine = t[0], minew = tw[0], rp_row = rpk[0];
#pragma unroll
    for (int k = 1; k < 4; ++k) {
      mine = (r0 == k) ? t[k] : mine;
      minew = (r0 == k) ? tw[k] : minew;
      rp_row = (r0 == k) ? rpk[k] : rp_row;
    }
    A[q] = mine;
    W[q] = minew;
    if constexpr (q < 3) {
      const double a = (c > 4 * q + 3) ? -(mine * rp_row) : 0.0;
      const double b = (c > 4 * q + r0) ? mine : 0.0;
      A = mfma16x16x4(a, b, A);
      W = mfma16x16x4(a, minew, W);
    }
  });
  const double rsc = rsqrt_nr(colpiv);
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int r = r0 + 4 * q;
    const double rsr = rsqrt_nr(rowpiv[q]);
    T[(o + r) * LP + o + c] = r >= c ? A[q] * rsc : 0.0;
    U[(o + r) * LP + o + c] = r >= c ? W[q] * rsr : 0.0;
  }
  if (lane < 16) piv[o + c] = colpiv;
}

GP_DEV int diag_factor_blk(int nb, double* ld_out) {
  LdsSmem& sm = *(LdsSmem*)&g_sm;
  lds_double* T = sm.As;
  lds_double* U = sm.Bs;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  lds_double* piv = sm.invs;
  // X_rc = -Dinv_r sum_{k=c}^{r-1} L_rk X_kc (X_cc = Dinv_c) into U's block (r, c); the sum
  // passes through T's free upper block (c, r)
  auto inv_block = [&](int r, int c) {
    f64x4 acc = zero4();
    for (int k = c; k < r; ++k)
      mm16(acc, T + 16 * r * LP + 16 * k, LP, 1, U + 16 * k * LP + 16 * c, LP, 1, false);
    lds_double* tmp = T + 16 * c * LP + 16 * r;
    st16(tmp, acc, 1.0);
    __builtin_amdgcn_s_waitcnt(0xc07f);   // lgkmcnt(0): the block is in LDS before it is read
    f64x4 x = zero4();
    mm16(x, U + 16 * r * LP + 16 * r, LP, 1, tmp, LP, 1, false);
    st16(U + 16 * r * LP + 16 * c, x, -1.0);
  };
  static_for<0, 4, 1>([&](auto Bk) {
    constexpr int b = decltype(Bk)::value;
    // while wave 0 factors leaf b, waves 1-2 build row b-1 of the inverse (its inputs -- Dinv of
    // rows <= b-1, the final L_{b-1,k}, the rows above -- are all complete), which the serial
    // phase after the last leaf used to do
    if (w == 0) {
      if constexpr (PP_LEAF_BLOCKED) leaf16_blocked(T, U, 16 * b, piv);
      else leaf16(T, U, 16 * b, piv);
    }
    else if (b >= 2 && w <= b - 1) inv_block(b - 1, w - 1);
    else if (b == 3 && w == 3) {
      // the last row's sums over the rows already final (k = c .. 1), beside leaf 3, into the
      // blocks the last-row pass continues from (the same MFMA accumulation order: bit-identical)
#pragma unroll
      for (int c2 = 0; c2 < 2; ++c2) {
        f64x4 acc = zero4();
        for (int k = c2; k < 2; ++k)
          mm16(acc, T + 16 * 3 * LP + 16 * k, LP, 1, U + 16 * k * LP + 16 * c2, LP, 1, false);
        st16(T + 16 * c2 * LP + 16 * 3, acc, 1.0);
      }
    }
    __syncthreads();
    if constexpr (b < 3) {
      // panel: L_rb = A_rb Dinv_b^T, r = b + w
      if (w >= 1 && b + w <= 3) {
        const int r = b + w;
        f64x4 acc = zero4();
        mm16(acc, T + 16 * r * LP + 16 * b, LP, 1, U + 16 * b * LP + 16 * b, 1, LP, false);
        st16(T + 16 * r * LP + 16 * b, acc, 1.0);
      }
      __syncthreads();
      // trailing update of step b: (b+1, b+1) by wave 0, the other lower blocks by waves 1-3
      auto upd = [&](int r, int s2) {
        f64x4 acc = ld16(T + 16 * r * LP + 16 * s2);
        mm16(acc, T + 16 * r * LP + 16 * b, LP, 1, T + 16 * s2 * LP + 16 * b, 1, LP, true);
        st16(T + 16 * r * LP + 16 * s2, acc, 1.0);
      };
      if (w == 0) upd(b + 1, b + 1);
      int idx = 0;
      for (int r = b + 1; r <= 3; ++r)
        for (int s2 = b + 1; s2 <= r; ++s2) {
          if (r == b + 1 && s2 == b + 1) continue;
          if (w >= 1 && idx % 3 == w - 1) upd(r, s2);
          ++idx;
        }
    }
  });
  // the inverse's last row: wave c builds X_3c (rows 1 and 2 were built beside leaves 2 and 3;
  // X_cc = Dinv_c already in U).  Wave 3 meanwhile checks the 64 pivots and sums their logs.
  if (w == 3) {
    const int lane = threadIdx.x & 63;
    const double p = piv[lane];
    const bool bad = lane < nb && !(p > 0.0 && isfinite(p));
    const unsigned long long badm = __ballot(bad);
    double l = lane < nb ? log(p) : 0.0;
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) l += __shfl_xor(l, off, 64);
    if (lane == 0) {
      sm.fail = badm ? __ffsll((long long)badm) : 0;
      sm.red[0] = l;
    }
  }
  if (w < 3) {
    // the last row of the inverse (rows 1, 2: beside the leaves; this row's k < 2 terms too)
    lds_double* tmp = T + 16 * w * LP + 16 * 3;
    f64x4 acc = (w < 2) ? ld16(tmp) : zero4();
    mm16(acc, T + 16 * 3 * LP + 16 * 2, LP, 1, U + 16 * 2 * LP + 16 * w, LP, 1, false);
    st16(tmp, acc, 1.0);
    __builtin_amdgcn_s_waitcnt(0xc07f);
    f64x4 x = zero4();
    mm16(x, U + 16 * 3 * LP + 16 * 3, LP, 1, tmp, LP, 1, false);
    st16(U + 16 * 3 * LP + 16 * w, x, -1.0);
  }
  __syncthreads();
  // zero the strict upper blocks of L^-1 (the chain's GEMM and the D_j store read the whole
  // tile; L's upper blocks are never read: it is stored lower-only, then overwritten)
  for (int g = threadIdx.x; g < NB * NB; g += 256) {
    const int r = g >> 6, cc = g & 63;
    if ((cc >> 4) > (r >> 4)) U[r * LP + cc] = 0.0;
  }
  __syncthreads();
  const int f = sm.fail;
  if (ld_out) *ld_out = sm.red[0];
  __syncthreads();
  return f;
}

// Factor diagonal block k whose (updated, symmetric) tile is in sm.As as [row][col]; write
// L_kk into A, D_k into X (dk_ptr), accumulate logdet, set info.
template <int MODE>
GP_DEV void diag_block(Smem& sm, double* __restrict__ Ab, int lda, double* __restrict__ Xb,
                       int ldx, int n, int k, int* info, double* logdet, int b) {
  const int k0 = k * NB, nb = min(NB, n - k0);
  double lg = 0.0;
  const int f = diag_factor_inv<0>(nb, &lg);
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


// ------------------------------------------------------------------------------------------
// Persistent dataflow factorisation (gp_potrf_inv / gp_potrf for N = ceil(n/64) <= kPPMaxN).
//
// One launch replaces the 2N launches of potrf_sweep.  Left-looking on 64x64 tiles: every
// tile is finished by ONE workgroup that keeps its 64x64 accumulator in registers across all
// of its K steps (the trailing matrix is never re-read / re-written per step as in the
// right-looking sweep), and workgroups hand tiles to each other through per-tile flags.
//   chain (one workgroup per problem, for j = 0..N-1):
//     C_jj = P_jj - L_j,j-1 L_j,j-1^T ; (L_jj, D_j = L_jj^-1) = diag_factor_inv(C_jj) ;
//     L_j+1,j = P_j+1,j D_j^T  (kept in LDS for the next step's SYRK)
//   worker tasks, dequeued in one global order (schedule_kernel):
//     DP(j)  P_jj    = A_jj    - sum_{k<j-1} L_jk L_jk^T      (in place in A, for the chain)
//     SP(j)  P_j+1,j = A_j+1,j - sum_{k<j}   L_j+1,k L_jk^T   (in place in A, for the chain)
//     LT(i,j), i >= j+2:  L_ij = (A_ij - sum_{k<j} L_ik L_jk^T) D_j^T
//     XT(i,c), i > c:     X_ic = -D_i sum_{k=c}^{i-1} L_ik X_kc   (X = L^-1, X_cc = D_c)
// The dequeue order is topological (every task's inputs come from tasks earlier in the list,
// or from the chain, which only waits on DP/SP tasks that precede everything waiting on it),
// so the launch is deadlock-free for any residency; anti-diagonal keys put the tiles the
// chain needs next at the front.
// Hand-offs follow MI355X_MICROARCH.md's acquire-free form: produced tiles are stored with
// sc1 (write-through) 16-B stores, each storing wave waits vmcnt(0), the workgroup barriers,
// one lane stores the flag (sc1); consumers poll flags with sc1 loads.  Tiles that pass
// through in-place partial sums (near-diagonal L tiles) are read with sc1 loads; every other
// produced tile is written once and read only after its flag, with plain (L2-cached) loads --
// but only when no 128-B cache line straddles two tiles (PPArgs::plain: lda, ldx multiples of
// 16 doubles, 128-B aligned bases), since a line shared with a neighbouring tile could be
// cached by a reader of that neighbour before this tile was written.  Every wait also watches
// the problem's abort word (non-PD pivot) and a poll budget, so no path can spin forever; a
// spent budget is reported as info = -1 by the last workgroup to leave the launch.
// ------------------------------------------------------------------------------------------
constexpr int kPPMaxN = 240;          // schedule_kernel: one thread per key (4N+63 <= 1024)
constexpr int kTChain = 0, kTL = 1, kTDP = 2, kTSP = 3, kTX = 4;
// (LT(i,j) + LT(i+1,j) pairs sharing L_jk were tried: keyed at the second row's
// anti-diagonal they delayed the row tiles SP(j) waits on, chain waits 7.7 vs 1.9 us per step,
// profiles/r03/pp_trace_pp4_pairs_splitleaf.txt; removed)
// XT tasks of the last kPPXTailRows rows stay single: they run after the chain's end (the
// launch's tail), where a pair's doubled K loop is latency, not throughput (tail 330 vs 200 us,
// profiles/r03/pp_trace_pp5.txt).  Splitting the tail rows' long XT sums in two (the first half
// dequeued as soon as its inputs were) cut the tail to 194 us but slowed the chain's late phase
// more (n = 4096 2.07 vs 1.84 ms, profiles/r03/ab_libs_pp7.log): removed.
constexpr int kPPXTailRows = 8;
constexpr int kTX2 = 6;     // XT pair: X_ic and X_i,c+1 (one opA stream, two opB streams)
// Zero tasks (inv only): the parts of the padded L^-1 buffer the factorisation never writes --
// the upper tiles (r, c), r < c < NT = npad / 64, kPPZRun of them per task (one tile column), and
// when npad / 64 = N + 1 the pure-padding tile row N (kTZP, 8 tile columns per task) -- so the
// buffer meets gp_potrf_inv's contract (zero above the diagonal and in the padding) without the
// caller-stream memset of the whole npad^2 buffer (134 MB at n = 4096: 18 us ahead of every
// factorisation).  They sit in the first keys, which hold no other task: the workers take them
// while the chain factors its first diagonal block, which every other early task waits on.
constexpr int kTZ = 5, kTZP = 7;
constexpr int kPPZRun = 8;       // tiles per zero task (256 KB)
constexpr int kPPZKeys = 4;      // keys 0..3 (the first worker tasks are at key 4)
constexpr long long kPollBudget = 1ll << 22;   // default s_sleep polls before a wait gives up
// gp_set_poll_budget (test / diagnostics hook): polls per wait for later launches; < 0 starts
// every problem aborted (the deterministic abort path of the tests)
long long g_poll_budget = kPollBudget;
#ifdef GPFIT_PP_TRACE
int* g_trace_dbg = nullptr;         // gp_pp_trace_set (trace build only)
long long* g_trace_buf = nullptr;
#endif

__shared__ int g_msg[4];              // dequeued task / wait results broadcast to the workgroup

struct PPArgs {
  double* A; long long sA; int lda;
  double* X; long long sX; int ldx;   // L^-1 (inv) or the 64 x 64N D_k scratch (plain)
  int n, N, batch, inv;
  int plain;                          // produced tiles may be read with plain loads (above)
  long long budget;                   // polls per wait
  int* info; double* logdet;
  const int2* tasks; int ntasks;
  int groups;                         // 1: one shared queue; 8: per-XCD queues (pp_groups)
  int* head;                          // [0] dequeue counter, [1] workgroups that have left,
                                      // [32 + 4g] group g's dequeue counter
  int* flags; int fstride;            // per problem: FL[N*N], FX[N*N], DPF[N], SPF[N], abort
  // gp_loglik's in-chain mode (pp_kernel<true>, inv = 0): the right-hand sides w (problem b at
  // w + b ldw), the forward-substitution scratch zb (problem b at zb + b zld: z_j at j 64,
  // DP(j)'s partial sums zq_j at zq_off + j 64), per problem sum z^2 (zz), and the outputs
  // ll / status / info_out of gp_loglik.  FZ[j] (z_j stored) lives in the unused FX flags.
  const double* w; int ldw;
  double* zb; int zld, zq_off;
  double* zz; double* ll; int* status; int* info_out;
#ifdef GPFIT_PP_TRACE
  int* dbg;                           // trace build only: per-workgroup progress words
  long long* trace;                   // trace build only: per-task / per-chain-step stamps
#endif
};

GP_DEV long long pp_now() { return (long long)__builtin_amdgcn_s_memrealtime(); }
#ifdef GPFIT_PP_TRACE
// Diagnostics build only (libgpfit_trace.so, tools/dbg/pp_trace.py): timestamps per task and
// chain phase, progress words per workgroup.  The shipped library has none of this.
__shared__ long long g_stall;         // ticks thread 0 spent polling flags in the current task
constexpr int kPPTraceSlots = 6;      // per task: wg|stall<<8, start, K-loop end, end, kind, i|j
#define PP_TRACE(P, idx, val)                                                            \
  do {                                                                                   \
    if ((P).trace && threadIdx.x == 0) (P).trace[(idx)] = (val);                         \
  } while (0)
#define PP_MARK(P, code, val)                                                            \
  do {                                                                                   \
    if ((P).dbg && threadIdx.x == 0) {                                                   \
      __hip_atomic_store((P).dbg + blockIdx.x * 4 + 1, (code), __ATOMIC_RELAXED,         \
                         __HIP_MEMORY_SCOPE_SYSTEM);                                     \
      __hip_atomic_store((P).dbg + blockIdx.x * 4 + 2, (val), __ATOMIC_RELAXED,          \
                         __HIP_MEMORY_SCOPE_SYSTEM);                                     \
    }                                                                                    \
  } while (0)
#define PP_STALL_ADD(x) (g_stall += (x))
#define PP_STALL_RESET() do { if (threadIdx.x == 0) g_stall = 0; } while (0)
#define PP_STALL() g_stall
#else
#define PP_TRACE(P, idx, val) do { } while (0)
#define PP_MARK(P, code, val) do { } while (0)
#define PP_STALL_ADD(x) ((void)(x))
#define PP_STALL_RESET() do { } while (0)
#define PP_STALL() 0ll
#endif

// Give up problem `abort` after a spent poll budget (2), unless it already failed on a pivot.
GP_DEV void pp_give_up(int* abort) {
  int expected = 0;
  __hip_atomic_compare_exchange_strong(abort, &expected, 2, __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_AGENT);
}

GP_DEV __amdgpu_buffer_rsrc_t pp_rsrc(const void* base) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), 0, 0x7fffffff, 0x00020000);
}
GP_DEV int pp_ldflag(const int* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
GP_DEV void pp_stflag(int* p, int v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
typedef unsigned int pp_u4 __attribute__((ext_vector_type(4)));

// Tile load into registers (load_op's slot map) with sc1 loads: 16-B buffer loads for a full,
// aligned tile, else bounds-checked 8-B loads (zero outside fv x sv).
GP_DEV void pp_load(OpTile& t, const double* src, int ld, int fv, int sv, bool coh = true) {
  const int tid = threadIdx.x;
  const bool full = fv == NB && sv == NB && (ld & 1) == 0 && (((size_t)src & 15) == 0);
  if (full) {
    const __amdgpu_buffer_rsrc_t r = pp_rsrc(src);
    const int base = ((tid & 31) * 2 + (tid >> 5) * ld) * 8;
    pp_u4 x[8];
    if (coh) {
#pragma unroll
      for (int q = 0; q < 8; ++q)
        x[q] = __builtin_amdgcn_raw_buffer_load_b128(r, base + q * 64 * ld, 0, 16);
    } else {
#pragma unroll
      for (int q = 0; q < 8; ++q)
        x[q] = __builtin_amdgcn_raw_buffer_load_b128(r, base + q * 64 * ld, 0, 0);
    }
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      t.v[2 * q] = __longlong_as_double(((long long)x[q].y << 32) | x[q].x);
      t.v[2 * q + 1] = __longlong_as_double(((long long)x[q].w << 32) | x[q].z);
    }
  } else {
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const int g = tid + 256 * q;
      const int f = (g & 31) * 2, sl = g >> 5;
      const double* p = src + f + (long long)sl * ld;
      const bool ok = sl < sv;
      t.v[2 * q] = (ok && f < fv)
          ? __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0.0;
      t.v[2 * q + 1] = (ok && f + 1 < fv)
          ? __hip_atomic_load(p + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0.0;
    }
  }
}

// Store a tile held in LDS as Cs[col][row] (pitch LP) to dst (col-major, ld) with sc1 stores,
// rows < rv and cols < cv only (and row >= col with `lower`); `neg` stores -Cs.
GP_DEV void pp_store_cm(double* dst, int ld, const double* Cs, int rv, int cv, bool neg,
                        bool lower = false) {
  const int tid = threadIdx.x;
  const double sg = neg ? -1.0 : 1.0;
  const bool full = rv == NB && cv == NB && !lower && (ld & 1) == 0 &&
                    (((size_t)dst & 15) == 0);
  if (full) {
    const __amdgpu_buffer_rsrc_t r = pp_rsrc(dst);
    const int f = (tid & 31) * 2;
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const int sl = (tid >> 5) + 8 * q;
      const double a = sg * Cs[sl * LP + f], b = sg * Cs[sl * LP + f + 1];
      const unsigned long long ua = __double_as_longlong(a), ub = __double_as_longlong(b);
      pp_u4 x;
      x.x = (unsigned)ua; x.y = (unsigned)(ua >> 32); x.z = (unsigned)ub; x.w = (unsigned)(ub >> 32);
      __builtin_amdgcn_raw_buffer_store_b128(x, r, (f + sl * ld) * 8, 0, 16);
    }
  } else {
#pragma unroll 4
    for (int q = 0; q < 16; ++q) {
      int row, col;
      slot_rc(q, row, col);
      if (row < rv && col < cv && (!lower || row >= col))
        __hip_atomic_store(dst + row + (long long)col * ld, sg * Cs[col * LP + row],
                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

// Store the nb x nb tile held in LDS as T[row][col] (pitch LP) to dst (col-major, ld) with sc1
// stores: 16-B pairs of rows for a full aligned tile, else 8-B elements; `lower`: only
// row >= col (LAPACK: the strict upper triangle of A is never written).
GP_DEV void pp_store_rm(double* dst, int ld, const double* T, int nb, bool lower,
                        bool zpad = false) {
  const int tid = threadIdx.x;
  const bool full = nb == NB && (ld & 1) == 0 && (((size_t)dst & 15) == 0);
  if (full) {
    const __amdgpu_buffer_rsrc_t r = pp_rsrc(dst);
    const int f = (tid & 31) * 2;
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const int c = (tid >> 5) + 8 * q;
      const double a = T[f * LP + c], b = T[(f + 1) * LP + c];
      if (!lower || f >= c) {
        const unsigned long long ua = __double_as_longlong(a), ub = __double_as_longlong(b);
        pp_u4 x;
        x.x = (unsigned)ua; x.y = (unsigned)(ua >> 32); x.z = (unsigned)ub; x.w = (unsigned)(ub >> 32);
        __builtin_amdgcn_raw_buffer_store_b128(x, r, (f + c * ld) * 8, 0, 16);
      } else if (f + 1 == c) {
        __hip_atomic_store(dst + c + (long long)c * ld, b, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
      }
    }
  } else {
#pragma unroll 4
    for (int q = 0; q < 16; ++q) {
      int row, col;
      slot_rc(q, row, col);
      const bool in = row < nb && col < nb;
      if ((in && (!lower || row >= col)) || (zpad && !in))
        __hip_atomic_store(dst + row + (long long)col * ld, in ? T[row * LP + col] : 0.0,
                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

// Every storing wave drains its stores, then one lane raises the flag.
GP_DEV void pp_publish(int* flag) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) pp_stflag(flag, 1);
}

// acc (this wave's 32x32) += sum_k As[k][rows] * Bs[k][cols]   (mma64 without the zeroing)
GP_DEV void mma64_add(const double* As, const double* Bs, f64x4 (&acc)[2][2]) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int wr = w >> 1, wc = w & 1, li = lane & 15, lk = lane >> 4;
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

// The block's accumulator into LDS row-major: Cs[row][col] (pitch LP).
GP_DEV void acc_to_lds_rm(double* Cs, const f64x4 (&acc)[2][2]) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int wr = w >> 1, wc = w & 1, li = lane & 15, lk = lane >> 4;
#pragma unroll
  for (int mi = 0; mi < 2; ++mi)
#pragma unroll
    for (int nj = 0; nj < 2; ++nj)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = wr * 32 + mi * 16 + lk + 4 * r, col = wc * 32 + nj * 16 + li;
        Cs[row * LP + col] = acc[mi][nj][r];
      }
}

// Wait until the flag *f is set, or the problem aborted / the poll budget ran out (then
// false).  One lane polls; the verdict is broadcast through g_msg (all threads call).
GP_DEV bool pp_wait1(const int* f, int* abort, long long budget) {
  if (threadIdx.x == 0) {
    int ok = pp_ldflag(f) != 0;
    const long long ts = pp_now();
    for (long long it = 0; !ok && it < budget; ++it) {
      if (pp_ldflag(abort)) break;
      __builtin_amdgcn_s_sleep(2);
      ok = pp_ldflag(f) != 0;
    }
    PP_STALL_ADD(pp_now() - ts);
    if (!ok) pp_give_up(abort);   // budget spent (or aborted): give up the problem
    g_msg[1] = ok;
  }
  __syncthreads();
  const int ok = g_msg[1];
  __syncthreads();
  return ok != 0;
}

// Whether the flag *f is set now (no waiting); one lane reads, the workgroup gets the answer.
GP_DEV bool pp_test1(const int* f) {
  if (threadIdx.x == 0) g_msg[3] = pp_ldflag(f) != 0;
  __syncthreads();
  const int ok = g_msg[3];
  __syncthreads();
  return ok != 0;
}

// One K step of a worker task: opA tile (NAT), opB tile (NAT or TRN), the producer flags, and
// for the paired XT2 task a third tile: its second B (X_k,c+1, TRN; absent at the first term,
// X_c,c+1 = 0).
struct PPTerm {
  const double *a, *b, *c;
  const int *fa, *fb, *fc;
  int lda_, ldb_, ldc_, av, bv, cv;   // av / cv: valid rows of the NAT tiles; bv: of opB (NAT)
  bool btrn;
  bool ca, cb, cc;          // operand tile rewritten in place during the launch: sc1 load
};

struct PPTask {
  int kind, b, i, j, nterms, idx;
};

template <bool LL>
GP_DEV PPTerm pp_term(const PPArgs& P, const PPTask& T, int t) {
  const int N = P.N;
  double* Ab = P.A + T.b * P.sA;
  double* Xb = P.X + T.b * P.sX;
  const int* F = P.flags + (long long)T.b * P.fstride;
  auto atile = [&](int r, int c) { return Ab + r * NB + (long long)c * NB * P.lda; };
  auto rv = [&](int r) { return min(NB, P.n - r * NB); };
  PPTerm u;
  u.lda_ = P.lda;
  u.ldb_ = P.lda;
  u.ldc_ = P.lda;
  u.btrn = false;
  u.c = nullptr;
  u.fc = nullptr;
  u.cv = NB;
  u.cc = true;
  // L tiles (r, k) with r - k <= 1 pass through P partial sums in place (DP / SP tasks on any
  // XCD) before the chain writes L: read them with sc1 so no XCD's L2 serves a stale line.  Every
  // other operand tile is written once, by the XCD that alone read its old contents, and is
  // only read after its flag: plain loads, cached in each reader's L2 -- when P.plain says no
  // cache line spans two tiles (section comment), else sc1 as well.
  auto hz = [&](int r, int k) { return r - k <= 1 || !P.plain; };
  if (T.kind == kTL || T.kind == kTSP) {   // L_ik L_jk^T with (i, j) = (T.i, T.j)
    u.a = atile(T.i, t);  u.fa = F + T.i * N + t;  u.av = rv(T.i);  u.ca = hz(T.i, t);
    u.b = atile(T.j, t);  u.fb = F + T.j * N + t;  u.bv = rv(T.j);  u.cb = hz(T.j, t);
  } else if (T.kind == kTDP) {             // L_jk L_jk^T
    u.a = atile(T.j, t);  u.fa = F + T.j * N + t;  u.av = rv(T.j);  u.ca = hz(T.j, t);
    u.b = u.a;            u.fb = u.fa;             u.bv = u.av;     u.cb = u.ca;
    if constexpr (LL) u.fc = F + N * N + t;  // (+ L_jk z_k: z_k stored by chain step k, FZ[k])
  } else {                                 // XT: L_ik X_kc, k = c + t (X_cc = D_c)
    const int k = T.j + t;
    u.a = atile(T.i, k);  u.fa = F + T.i * N + k;  u.av = rv(T.i);  u.ca = hz(T.i, k);
    u.cb = !P.plain;
    u.b = Xb + k * NB + (long long)T.j * NB * P.ldx;
    u.ldb_ = P.ldx;
    u.fb = (k == T.j) ? F + k * N + k : F + N * N + k * N + T.j;
    u.bv = NB;                               // X is zero-padded to npad: always in bounds
    u.btrn = true;
    if (T.kind == kTX2 && k > T.j) {         // + L_ik X_k,c+1 (X_c+1,c+1 = D_c+1)
      const int c1 = T.j + 1;
      u.c = Xb + k * NB + (long long)c1 * NB * P.ldx;
      u.ldc_ = P.ldx;
      u.fc = (k == c1) ? F + k * N + k : F + N * N + k * N + c1;
      u.cc = !P.plain;
    }
  }
  return u;
}

// Lane-parallel readiness scan: the number of consecutive terms t0, t0+1, ... whose input
// flags are all set (wave 0, one term per lane), at least 1 unless the problem aborted (-1).
template <bool LL>
GP_DEV int pp_ready(const PPArgs& P, const PPTask& T, int t0, int* abort) {
  if (threadIdx.x < 64) {
    const int lane = threadIdx.x;
    int res = -1;
    const long long ts = pp_now();
    for (long long it = 0;; ++it) {
      const int t = t0 + lane;
      bool rdy = true;
      if (t < T.nterms) {
        const PPTerm u = pp_term<LL>(P, T, t);
        rdy = pp_ldflag(u.fa) != 0 && pp_ldflag(u.fb) != 0 && (!u.fc || pp_ldflag(u.fc) != 0);
      }
      const unsigned long long m = __ballot(rdy);
      const int lead = (~m == 0ull) ? 64 : __builtin_ctzll(~m);
      const int cnt = min(lead, T.nterms - t0);
      if (cnt > 0) { res = cnt; break; }
      if (it >= P.budget || pp_ldflag(abort)) break;
      __builtin_amdgcn_s_sleep(2);
    }
    if (res < 0 && lane == 0) pp_give_up(abort);
    if (lane == 0) g_msg[2] = res;
    if (lane == 0) PP_STALL_ADD(pp_now() - ts);
  }
  __syncthreads();
  const int r = g_msg[2];
  __syncthreads();
  return r;
}

GP_DEV void pp_load_term(const PPTerm& u, OpTile& ta, OpTile& tb, OpTile& tc) {
  pp_load(ta, u.a, u.lda_, u.av, NB, u.ca);
  if (u.b != u.a) pp_load(tb, u.b, u.ldb_, u.bv, NB, u.cb);
  if (u.c) pp_load(tc, u.c, u.ldc_, u.cv, NB, u.cc);
}

// Worker: accumulate the task's K steps in registers (software-pipelined: the next step's
// operands are loaded while the current step's MFMAs run, whenever its flags are known set).
// The paired XT2 accumulates its second output in acc2 from the third tile (staged in g_keep,
// which only the chain uses otherwise): acc2 += L_ik X_k,c+1, sharing opA: three tile loads
// per two tile-terms instead of four.
// LL (gp_loglik's in-chain mode) DP tasks also accumulate zq = sum_k L_jk z_k (this thread: row
// tid & 63, columns 16 (tid >> 6) .. + 15 of each term, k ascending) from the term's tile in LDS
// and z_k (staged in g_ll by the first wave with the tile; its flag FZ[k] is one of the term's).
template <bool LL>
GP_DEV bool pp_accumulate(const PPArgs& P, const PPTask& T, f64x4 (&acc)[2][2],
                          f64x4 (&acc2)[2][2], int* abort, double& zq) {
  Smem& sm = g_sm;
#pragma unroll
  for (int mi = 0; mi < 2; ++mi)
#pragma unroll
    for (int nj = 0; nj < 2; ++nj) {
      acc[mi][nj] = zero4();
      acc2[mi][nj] = zero4();
    }
  zq = 0.0;
  if (T.nterms == 0) return true;
  const bool lldp = LL && T.kind == kTDP;
  double zr = 0.0;                                   // z_k of the term in flight (tid < 64)
  auto ldz = [&](int t) {
    if (lldp && threadIdx.x < 64)
      zr = __hip_atomic_load(P.zb + (long long)T.b * P.zld + t * NB + threadIdx.x,
                             __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  };
  OpTile ta, tb, tc;
  int avail = pp_ready<LL>(P, T, 0, abort);  // terms [0, avail) are ready
  if (avail < 0) return false;
  PPTerm u = pp_term<LL>(P, T, 0);
  pp_load_term(u, ta, tb, tc);
  ldz(0);
  for (int t = 0; t < T.nterms; ++t) {
    const bool same = u.b == u.a;
    const bool trn = u.btrn;
    const bool third = u.c != nullptr;
    __syncthreads();                                   // the previous MFMAs have read the tiles
    store_op<false>(sm.As, ta);
    if (!same) {
      if (trn) store_op<true>(sm.Bs, tb);
      else store_op<false>(sm.Bs, tb);
    }
    if (third) store_op<true>(g_keep, tc);
    if (lldp && threadIdx.x < 64) g_ll[kLLZ + threadIdx.x] = zr;
    __syncthreads();
    const bool more = t + 1 < T.nterms;
    const bool pre = more && t + 1 < avail;
    if (pre) {
      u = pp_term<LL>(P, T, t + 1);
      pp_load_term(u, ta, tb, tc);
      ldz(t + 1);
    }
    mma64_add(sm.As, same ? sm.As : sm.Bs, acc);
    if (third) mma64_add(sm.As, g_keep, acc2);
    if (lldp) {
      const int r = threadIdx.x & 63, c0 = 16 * (threadIdx.x >> 6);
#pragma unroll
      for (int c = 0; c < 16; ++c) zq = fma(sm.As[(c0 + c) * LP + r], g_ll[kLLZ + c0 + c], zq);
    }
    if (more && !pre) {
      const int r = pp_ready<LL>(P, T, t + 1, abort);
      if (r < 0) return false;
      avail = t + 1 + r;
      u = pp_term<LL>(P, T, t + 1);
      pp_load_term(u, ta, tb, tc);
      ldz(t + 1);
    }
  }
  return true;
}

// C (As as [col][row]) = A tile - acc, for rows < rv / cols < cv (zero elsewhere).  lower:
// only row >= col is taken from A (diagonal tiles; the upper part of A is never read).  The A
// tile was loaded into registers (pp_load's slot map: column (tid >> 5) + 8q, rows
// 2 (tid & 31) + {0, 1}) when the task started, so its latency hides under the K loop.
GP_DEV void pp_sub_tile(const OpTile& a, int rv, int cv, bool lower, const f64x4 (&acc)[2][2]) {
  Smem& sm = g_sm;
  const int tid = threadIdx.x;
  __syncthreads();
  acc_to_lds(sm.As, acc);
  __syncthreads();
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    const int col = (tid >> 5) + 8 * q;
#pragma unroll
    for (int e = 0; e < 2; ++e) {
      const int row = (tid & 31) * 2 + e;
      const bool ok = row < rv && col < cv && (!lower || row >= col);
      sm.As[col * LP + row] = ok ? a.v[2 * q + e] - sm.As[col * LP + row] : 0.0;
    }
  }
  __syncthreads();
}

GP_DEV double* pp_dptr(const PPArgs& P, int b, int j, int& ld) {
  double* Xb = P.X + b * P.sX;
  if (P.inv) {
    ld = P.ldx;
    return Xb + j * NB + (long long)j * NB * P.ldx;
  }
  ld = NB;
  return Xb + (long long)j * NB * NB;
}

// The persistent kernel's two task families are inlined into its dispatch loop, where their
// register allocations add up (chain alone 344 VGPRs+AGPRs, workers alone 350, both 462: room
// for one 48-register cross-covariance wave per SIMD beside it).  As calls (PP_TASK_CALLS=1)
// the kernel takes 353 (+176 B of scratch per lane for the call frames), room for three; the
// cross-covariance then ran 1.09 instead of ~2 ms per C3 step, but the factorisation took 2.17
// instead of 1.81 ms alone and 2.40 beside it, and the C3 step got slower (27.05-27.21 ms,
// profiles/r04/r04d_*; same-box A/B in r04e_*).
#ifndef PP_TASK_CALLS
#define PP_TASK_CALLS 0
#endif
#if PP_TASK_CALLS
#define PP_TASK __device__ __attribute__((noinline))
#else
#define PP_TASK GP_DEV
#endif

template <bool LL>
PP_TASK void pp_worker(const PPArgs& P, const PPTask& T) {
  Smem& sm = g_sm;
  const int N = P.N;
  int* F = P.flags + (long long)T.b * P.fstride;
  int* abort = F + 2 * N * N + 2 * N;
  if (pp_ldflag(abort)) return;
  double* Ab = P.A + T.b * P.sA;
  double* Xb = P.X + T.b * P.sX;
  f64x4 acc[2][2], acc2[2][2];
  PP_MARK(P, 20 + T.kind, T.i * 1000 + T.j);
  PP_STALL_RESET();
  const long long tr = (long long)T.idx * 6;   // trace slots of this task (trace build)
  (void)tr;
  PP_TRACE(P, tr + 1, pp_now());
  PP_TRACE(P, tr + 4, T.kind | (T.b << 4));
  PP_TRACE(P, tr + 5, T.i | (T.j << 16));
  auto atile = [&](int r, int c) { return Ab + r * NB + (long long)c * NB * P.lda; };
  auto xtile = [&](int r, int c) { return Xb + r * NB + (long long)c * NB * P.ldx; };
  auto rv = [&](int r) { return min(NB, P.n - r * NB); };
  const bool xt = T.kind == kTX || T.kind == kTX2;
  // the task's own A tile (DP / SP: the chain's partial-sum tile; LT: A_ij), in flight from
  // here until the epilogue
  const int ar = T.kind == kTDP ? T.j : (T.kind == kTSP ? T.j + 1 : T.i);
  OpTile ta;
  if (!xt) pp_load(ta, atile(ar, T.j), P.lda, rv(ar), T.kind == kTL ? NB : rv(T.j));
  double zq;
  if (!pp_accumulate<LL>(P, T, acc, acc2, abort, zq)) return;
  PP_MARK(P, 30 + T.kind, T.i * 1000 + T.j);
  PP_TRACE(P, tr + 2, pp_now());
  // slot 0: workgroup | ticks polled before the K loop finished << 8
  PP_TRACE(P, tr + 0, blockIdx.x | (PP_STALL() << 8));
  if (T.kind == kTDP || T.kind == kTSP) {
    // partial sums for the chain, in place in A
    const int r = ar;
    double* dst = atile(r, T.j);
    pp_sub_tile(ta, rv(r), rv(T.j), T.kind == kTDP, acc);
    pp_store_cm(dst, P.lda, sm.As, rv(r), rv(T.j), false, T.kind == kTDP);
    if constexpr (LL) {
      if (T.kind == kTDP) {
        // zq_j = sum_{k < j-1} L_jk z_k for the chain's y_j: the four column quarters' partial
        // sums added in quarter order (a fixed order)
        g_ll[kLLPart + threadIdx.x] = zq;
        __syncthreads();
        if (threadIdx.x < 64 && threadIdx.x < rv(T.j)) {
          const double* pq = g_ll + kLLPart + threadIdx.x;
          __hip_atomic_store(P.zb + (long long)T.b * P.zld + P.zq_off + T.j * NB + threadIdx.x,
                             ((pq[0] + pq[64]) + pq[128]) + pq[192], __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_AGENT);
        }
      }
    }
    pp_publish(T.kind == kTDP ? F + 2 * N * N + T.j : F + 2 * N * N + N + T.j);
    PP_TRACE(P, tr + 3, pp_now());
    return;
  }
  if (T.kind == kTL) {
    // L_ij = (A_ij - acc) D_j^T
    double* dst = atile(T.i, T.j);
    pp_sub_tile(ta, rv(T.i), NB, false, acc);
    if (!pp_wait1(F + T.j * N + T.j, abort, P.budget)) return;
    int ldd;
    const double* D = pp_dptr(P, T.b, T.j, ldd);
    OpTile td;
    pp_load(td, D, ldd, NB, NB);                        // Bs[p][c] = D_j[c][p]
    store_op<false>(sm.Bs, td);
    __syncthreads();
    mma64(sm.As, sm.Bs, acc);
    __syncthreads();
    acc_to_lds(sm.As, acc);
    __syncthreads();
    pp_store_cm(dst, P.lda, sm.As, rv(T.i), NB, false);
    pp_publish(F + T.i * N + T.j);
    PP_TRACE(P, tr + 3, pp_now());
    return;
  }
  // XT: X_ic = -D_i S, S = acc (XT2: X_i,c+1 = -D_i S2, S2 = acc2), through g_keep
  __syncthreads();
  acc_to_lds_rm(sm.Bs, acc);                            // Bs[p][cc] = S[p][cc]
  if (!pp_wait1(F + T.i * N + T.i, abort, P.budget)) return;
  PP_MARK(P, 40, T.i * 1000 + T.j);
  int ldd;
  const double* D = pp_dptr(P, T.b, T.i, ldd);
  OpTile td;
  pp_load(td, D, ldd, NB, NB);                          // As[p][r] = D_i[r][p]
  store_op<false>(sm.As, td);
  __syncthreads();
  mma64(sm.As, sm.Bs, acc);
  __syncthreads();
  acc_to_lds(g_keep, acc);
  __syncthreads();
  pp_store_cm(xtile(T.i, T.j), P.ldx, g_keep, NB, NB, true);
  if (T.kind == kTX2) {
    acc_to_lds_rm(sm.Bs, acc2);                         // (the barrier above: Bs read)
    __syncthreads();                                    // ... and every wave's g_keep reads
    mma64(sm.As, sm.Bs, acc2);
    __syncthreads();
    acc_to_lds(g_keep, acc2);
    __syncthreads();
    pp_store_cm(xtile(T.i, T.j + 1), P.ldx, g_keep, NB, NB, true);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    pp_stflag(F + N * N + T.i * N + T.j, 1);
    if (T.kind == kTX2) pp_stflag(F + N * N + T.i * N + T.j + 1, 1);
  }
  PP_MARK(P, 41, T.i * 1000 + T.j);
  PP_TRACE(P, tr + 3, pp_now());
}

// The chain of problem b (see the section comment).
// gp_loglik's in-chain mode: z_j = D_j y_j (y_j = w_j - zq_j - L_j,j-1 z_j-1 in g_ll, D_j in
// sm.Bs as [row][col]) into g_ll's z slot and the problem's z scratch; sum z^2 accumulated in
// order on thread 0.  The four column quarters' partial sums are added in quarter order.
GP_DEV void ll_zstep(const PPArgs& P, int b, int j, int nb, double& zz) {
  Smem& sm = g_sm;
  const int r = threadIdx.x & 63, c0 = 16 * (threadIdx.x >> 6);
  double part = 0.0;
#pragma unroll
  for (int c = 0; c < 16; ++c) part = fma(sm.Bs[r * LP + c0 + c], g_ll[kLLY + c0 + c], part);
  g_ll[kLLPart + threadIdx.x] = part;
  __syncthreads();
  if (threadIdx.x < 64) {
    const double* pq = g_ll + kLLPart + r;
    const double z = r < nb ? ((pq[0] + pq[64]) + pq[128]) + pq[192] : 0.0;
    g_ll[kLLZ + r] = z;
    if (r < nb)
      __hip_atomic_store(P.zb + (long long)b * P.zld + j * NB + r, z, __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_AGENT);
    double q = z * z;
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) q += __shfl_xor(q, off, 64);
    if (r == 0) zz += q;
  }
  // (no barrier: z and the partial slots are next read / rewritten behind the step's own)
}

template <bool LL>
PP_TASK void pp_chain(const PPArgs& P, int b) {
  Smem& sm = g_sm;
  const int N = P.N;
  int* F = P.flags + (long long)b * P.fstride;
  int* abort = F + 2 * N * N + 2 * N;
  double* Ab = P.A + b * P.sA;
  auto atile = [&](int r, int c) { return Ab + r * NB + (long long)c * NB * P.lda; };
  double ld_sum = 0.0;
  double zz = 0.0;           // (LL) sum of z^2 so far (thread 0)
  OpTile tpj;                // P_jj, loaded by the previous step when its partials were ready
  bool pref = false;
  // L_j,j-1 L_j,j-1^T for step j, computed at the end of step j-1 while that step's stores
  // drain (zero for j = 0).  Exactly symmetric: element (r, c) and (c, r) sum the same products
  // in the same order.
  f64x4 syrk[2][2];
#pragma unroll
  for (int mi = 0; mi < 2; ++mi)
#pragma unroll
    for (int nj = 0; nj < 2; ++nj) syrk[mi][nj] = zero4();
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int wr = wv >> 1, wc = wv & 1, li = lane & 15, lk = lane >> 4;
  for (int j = 0; j < N; ++j) {
    const int nb = min(NB, P.n - j * NB);
    PP_MARK(P, 10, j);
    const long long tb0 = (long long)P.ntasks * 6 + ((long long)b * N + j) * 8;
    (void)tb0;
    PP_TRACE(P, tb0 + 0, pp_now());
    // (a) C_jj = P_jj - syrk into As as a full symmetric [row][col] tile: P_jj's lower triangle
    // staged in Bs ([col][row]), then every thread writes its own 16 accumulator positions
    // (mirrored to the lower element of P), identity padding past nb.
    if (!pref) {
      if (j >= 2 && !pp_wait1(F + 2 * N * N + j, abort, P.budget)) return;
      pp_load(tpj, atile(j, j), P.lda, nb, nb);
    }
    // (LL) this step's right-hand side w_j and DP(j)'s partial sum zq_j (its flag is set here)
    double wq = 0.0;
    if constexpr (LL) {
      if (threadIdx.x < 64 && threadIdx.x < nb) {
        wq = P.w[(long long)b * P.ldw + j * NB + threadIdx.x];
        if (j >= 2)
          wq -= __hip_atomic_load(P.zb + (long long)b * P.zld + P.zq_off + j * NB + threadIdx.x,
                                  __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    }
    PP_TRACE(P, tb0 + 1, pp_now());
    __syncthreads();
    store_op<false>(sm.Bs, tpj);                        // Bs[c][r] = P(r, c) (r >= c valid)
    __syncthreads();
#pragma unroll
    for (int mi = 0; mi < 2; ++mi)
#pragma unroll
      for (int nj = 0; nj < 2; ++nj)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int row = wr * 32 + mi * 16 + lk + 4 * q, col = wc * 32 + nj * 16 + li;
          const int R = row > col ? row : col, C = row > col ? col : row;
          const double v = R < nb ? sm.Bs[C * LP + R] - syrk[mi][nj][q]
                                  : (row == col ? 1.0 : 0.0);
          sm.As[row * LP + col] = v;
        }
    __syncthreads();
    if constexpr (LL) {
      // y_j = (w_j - zq_j) - L_j,j-1 z_j-1: the last term's four column-quarter partial sums
      // were formed beside step j-1's SYRK (read after that step's barriers; y is read after
      // diag_factor_blk's)
      if (threadIdx.x < 64) {
        const int r = threadIdx.x;
        const double* pq = g_ll + kLLPart + r;
        const double t = j >= 1 ? ((pq[0] + pq[64]) + pq[128]) + pq[192] : 0.0;
        g_ll[kLLY + r] = r < nb ? wq - t : 0.0;
      }
    }
    // (b) factor + invert
    PP_MARK(P, 11, j);
    PP_TRACE(P, tb0 + 2, pp_now());
    double lg = 0.0;
    const int f = diag_factor_blk(nb, &lg);
    PP_TRACE(P, tb0 + 3, pp_now());
    if (f) {
      if (threadIdx.x == 0) {
        if (P.info) P.info[b] = j * NB + f;
        pp_stflag(abort, 1);
      }
      return;
    }
    ld_sum += lg;
    PP_MARK(P, 12, j);
    int ldd;
    double* D = pp_dptr(P, b, j, ldd);
    if (j + 1 >= N) {
      // last step: D_j -> X_jj (or the D scratch), L_jj -> A (lower, LAPACK layout)
      pp_store_rm(D, ldd, sm.Bs, nb, false, true);
      pp_store_rm(atile(j, j), P.lda, sm.As, nb, true);
      if constexpr (LL) ll_zstep(P, b, j, nb, zz);
      pp_publish(F + j * N + j);
      PP_TRACE(P, tb0 + 4, pp_now());
      break;
    }
    // (c) D_j and L_jj are stored and D_j published right away: LT(j+2, j) -> SP(j+1) -> the
    // next step's (d) hang on it (publishing D_j after the GEMM instead moved 2-4 us per step
    // into the chain's wait for SP, profiles/r03/pp_trace_pp1.txt).  The loads of P_j+1,j and
    // the next P_j+1,j+1 go out with the stores when their partial sums are already published.
    PP_MARK(P, 13, j);
    const int nb1 = min(NB, P.n - (j + 1) * NB);
    // (zero padding past nb: X's rows >= n come out 0 in the XT tasks)
    pp_store_rm(D, ldd, sm.Bs, nb, false, true);
    OpTile tp;
    const bool spref = j < 1 || pp_test1(F + 2 * N * N + N + j);
    if (spref) pp_load(tp, atile(j + 1, j), P.lda, nb1, NB);
    pref = j + 1 < 2 || pp_test1(F + 2 * N * N + j + 1);
    if (pref) pp_load(tpj, atile(j + 1, j + 1), P.lda, nb1, nb1);
    pp_publish(F + j * N + j);                          // drains stores and loads alike
    // L_jj (read by nobody in this launch) after D_j's flag: its stores drain under the GEMM
    // instead of in front of the flag (n = 4096 1.812 vs 1.824 ms, n = 1024 x 32 0.994 vs
    // 0.998, bit-identical; profiles/r04/ab_zt_ljj.log)
    pp_store_rm(atile(j, j), P.lda, sm.As, nb, true);
    // (LL) z_j = D_j y_j (D_j in Bs) here, where the chain may wait for SP(j) below anyway
    if constexpr (LL) ll_zstep(P, b, j, nb, zz);
    __syncthreads();                                    // every wave has read As
    PP_TRACE(P, tb0 + 4, pp_now());
    if (!spref) {
      if (!pp_wait1(F + 2 * N * N + N + j, abort, P.budget)) return;
      pp_load(tp, atile(j + 1, j), P.lda, nb1, NB);    // As[p][r] = P[r][p]
    }
    store_op<false>(sm.As, tp);                         // (pp_publish's barrier: As is free)
    __syncthreads();
    PP_MARK(P, 14, j);
    PP_TRACE(P, tb0 + 5, pp_now());
    // (d) L_j+1,j = P_j+1,j D_j^T (D held [row][col] in Bs), kept in LDS for the next SYRK
    f64x4 acc[2][2];
    mma64_bt(sm.As, sm.Bs, acc);
    __syncthreads();
    acc_to_lds(g_keep, acc);                           // keep[c][r] = L_j+1,j(r, c)
    __syncthreads();
    PP_TRACE(P, tb0 + 6, pp_now());
    pp_store_cm(atile(j + 1, j), P.lda, g_keep, nb1, NB, false);
    // the next step's SYRK runs while L_j+1,j's stores drain, then its flag goes up
    mma64(g_keep, g_keep, syrk);
    if constexpr (LL) {
      // (LL) the quarter sums of L_j+1,j z_j for y_j+1, beside the SYRK (pp_publish's barrier
      // orders them before the next step reads them)
      const int r = threadIdx.x & 63, c0 = 16 * (threadIdx.x >> 6);
      double part = 0.0;
#pragma unroll
      for (int c = 0; c < 16; ++c) part = fma(g_keep[(c0 + c) * LP + r], g_ll[kLLZ + c0 + c], part);
      g_ll[kLLPart + threadIdx.x] = part;
    }
    pp_publish(F + (j + 1) * N + j);
    if constexpr (LL)
      if (threadIdx.x == 0) pp_stflag(F + N * N + j, 1);    // FZ[j]: z_j drained with the above
    PP_MARK(P, 15, j);
    PP_TRACE(P, tb0 + 7, pp_now());
  }
  if (threadIdx.x == 0 && P.logdet) P.logdet[b] = ld_sum;
  if constexpr (LL)
    if (threadIdx.x == 0) P.zz[b] = zz;
}

// The last workgroup to leave the launch (every task, chain and XT alike, has returned by then)
// reports a poll budget spent anywhere in problem b (abort word 2) as info[b] = -1: an internal
// error, never a pivot.  The acq_rel exit count orders every workgroup's abort / info stores
// before the reading workgroup's loads.
// In gp_loglik's in-chain mode it then writes every problem's log-likelihood, as
// nll_reduce_kernel does for the L^-1 path: -(1/2 sum z^2 + 1/2 logdet), -inf for a non-PD
// pivot (info > 0), NaN plus the sticky status word for an internal error (info = -1).
template <bool LL>
GP_DEV void pp_exit(const PPArgs& P) {
  if (threadIdx.x != 0) return;
  const int done = __hip_atomic_fetch_add(P.head + 1, 1, __ATOMIC_ACQ_REL,
                                          __HIP_MEMORY_SCOPE_AGENT);
  if (done != (int)gridDim.x - 1 || !P.info) return;
  for (int b = 0; b < P.batch; ++b) {
    const int* ab = P.flags + (long long)b * P.fstride + 2 * P.N * P.N + 2 * P.N;
    if (pp_ldflag(ab) == 2) P.info[b] = -1;
    if constexpr (LL) {
      const int f = P.info[b];
      const double v = 0.5 * P.zz[b] + 0.5 * P.logdet[b];
      P.ll[b] = f < 0 ? __builtin_nan("") : -(f > 0 ? __builtin_huge_val() : v);
      if (P.info_out) P.info_out[b] = f;
      if (f < 0 && P.status)
        __hip_atomic_fetch_or(P.status, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

// Zero task: plain stores (read only by later launches: the kernel boundary orders them).
// Wave w takes columns w, w + 4, ...; a column's run of rows is contiguous.  Kept minimal in
// registers: pp_kernel's allocation decides whether a cross-covariance wave still fits beside
// it on the SIMD (tests/test_capi.py::test_persistent_factorisation_leaves_room_for_cross).
GP_DEV void pp_zero(const PPArgs& P, const PPTask& T) {
  const bool zt = T.kind == kTZ;
  const int NT = (P.N + 1) & ~1;
  const int c0 = T.i;
  const int ncol = NB * (zt ? 1 : min(8, NT - c0));
  const int r0 = zt ? T.j : P.N;
  const int nrow = NB * (zt ? min(kPPZRun, T.i - T.j) : NT - P.N);
  double* base = P.X + T.b * P.sX + (long long)NB * r0 + (long long)NB * c0 * P.ldx;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  for (int col = w; col < ncol; col += 4) {
    double* cp = base + (long long)col * P.ldx;
    for (int e = lane; e < nrow; e += 64) cp[e] = 0.0;
  }
}

template <bool LL>
__global__ __launch_bounds__(256, 1) void pp_kernel(PPArgs P) {
  // per-XCD queues: workgroup w takes group w % 8's tasks, the global tasks 8k + g (pp_groups)
  const int g = (int)blockIdx.x % P.groups;
  for (;;) {
    if (threadIdx.x == 0)
      g_msg[0] = P.groups > 1 ? atomicAdd(P.head + 32 + 4 * g, 1) * P.groups + g
                              : atomicAdd(P.head, 1);
    __syncthreads();
    const int t = g_msg[0];
    __syncthreads();
#ifdef GPFIT_PP_TRACE
    if (P.dbg && threadIdx.x == 0)
      __hip_atomic_store(P.dbg + blockIdx.x * 4, t, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
#endif
    if (t >= P.ntasks) {
      PP_MARK(P, 99, 0);
      pp_exit<LL>(P);
      return;
    }
    const int2 e = P.tasks[t];
    PPTask T;
    T.kind = e.x & 15;
    T.b = e.x >> 4;
    T.i = e.y & 0xffff;
    T.j = e.y >> 16;
    if (T.kind == kTChain) {
      pp_chain<LL>(P, T.b);
      __syncthreads();
      continue;
    }
    T.idx = t;
    if (T.kind == kTZ || T.kind == kTZP) {
      PP_TRACE(P, (long long)t * 6 + 1, pp_now());
      pp_zero(P, T);
      PP_TRACE(P, (long long)t * 6 + 0, blockIdx.x);
      PP_TRACE(P, (long long)t * 6 + 2, pp_now());
      PP_TRACE(P, (long long)t * 6 + 3, pp_now());
      PP_TRACE(P, (long long)t * 6 + 4, T.kind | (T.b << 4));
      PP_TRACE(P, (long long)t * 6 + 5, T.i | (T.j << 16));
      continue;
    }
    T.nterms = T.kind == kTL ? T.j : T.kind == kTDP ? T.j - 1 : T.kind == kTSP ? T.j : T.i - T.j;
    pp_worker<LL>(P, T);
  }
}

// Task list: batch chain entries, then per key t = 0..4N-2+4(W+XD) (anti-diagonal order, see
// the section comment) the tasks of that key, each for every problem:
//   DP(j): t = 4j-2;  SP(j): t = 4j+1;  band LT(i,j), i-j <= kPPBand: t = 2(i+j)   ("early")
//   other LT(i,j): t = 2(i+j) + 4W;  XT(i,c): t = 4i+2 + 4(W+XD), c = 0 first
// XT tasks wait on whole rows of L (their last K step on L_i,i-1, a chain output): dequeued
// with the LT tasks (XD = 0) they sat polling in ~25% of the workers while the LT / SP tasks the
// chain waits on queued behind them (pp_trace: 145 ms of 588 ms worker time polling, the
// chain waiting 7-26 us per step for SP from step ~36 on); XD = kPPXDelay = 8 leaves those
// workers to the LT tasks (n = 4096: 2.12-2.17 vs 2.44-2.46 ms, profiles/r02/ab_pp_xt_delay.log).
// Emitting each row's longest XT (c = 0) first shortens the tail after the chain.
// The early tasks are what the chain waits on (its partials and the near-diagonal tiles the
// partials wait on): they are dequeued kPPLead = W chain steps ahead of their topological
// position, early enough to catch up on their K steps that are already available.  Only
// early tasks can wait on tasks not yet dequeued: per problem, those dequeued in the last 4W
// keys (W DP, W SP, 2W band LT).  With W = 0 the list is topological: every worker task waits
// only on earlier tasks and on chain steps whose own inputs are earlier still, so any grid with
// more workgroups than problems drains.  pp_lead() takes W = kPPLead only while every problem's
// blocked early tasks plus its chain fit in the grid with a worker to spare (batch 32 at
// n = 1024 on 256 workgroups deadlocked with W = 6 for every problem: 32 x 24 > 224).
// W = 4: n = 4096 1.855-1.857 ms median vs 1.880-1.890 at W = 6 and 1.896-1.909 at 8, batch 32
// unchanged (profiles/r02/ab_pp_lead_xd.log, XT delay 6 / 8 / 11 equal within noise).
constexpr int kPPLead = 4;
// per-problem bound on early tasks blocked on tasks not yet dequeued: W DP, W SP and 2W band
// LT in the 4W positions ahead, + 2 positions for the LT pairs keyed at their second row
constexpr int kPPLeadBlocked = 4 * kPPLead + 6;
constexpr int kPPBand = 3;
constexpr int kPPXDelay = 8;   // XT tasks: 8 chain steps after the late LT tasks of their row

// The tasks of key t in emission order (f(kind, i, j) per task; see pp_schedule_kernel):
//   early  DP(j): t = 4j-2;  SP(j): t = 4j+1;  band LT(i,j), 2 <= i-j <= kPPBand: t = 2(i+j)
//   late   (K = t - 4W)  XT(i,c): K = 4i+2 + 4XD;  LT(i,j), i-j > kPPBand: K = 2(i+j)
// Every input of a late task has a smaller key or is a chain step whose own inputs do (see the
// section comment).  Shared by the schedule kernel (count + emit) and the host's task count.
template <typename F>
GP_HD inline void pp_for_key(int t, int N, bool inv, int lead, int xd, F&& f) {
  if (inv && t < kPPZKeys) {
    const int NT = (N + 1) & ~1;                               // npad / 64
    for (int c = 1 + t; c < NT; c += kPPZKeys)
      for (int r0 = 0; r0 < c; r0 += kPPZRun) f(kTZ, c, r0);
    if (t == 0 && NT > N)
      for (int c0 = 0; c0 < NT; c0 += 8) f(kTZP, c0, 0);
  }
  // late tasks of this position first (K = t - 4W): a late task can be an input of an early
  // task of the same position, never the other way round
  const int K = t - 4 * lead;
  if (K >= 0) {
    const int KX = K - 4 * xd;
    if (inv && KX >= 0 && KX % 4 == 2 && (KX - 2) / 4 >= 1 && (KX - 2) / 4 <= N - 1) {
      const int i = (KX - 2) / 4;
      if (i + kPPXTailRows < N) {                              // pairs (c, c+1), longest first
        for (int c = 0; c + 1 < i; c += 2) f(kTX2, i, c);
        if (i & 1) f(kTX, i, i - 1);
      } else {                                                 // the last rows: singles
        for (int c = 0; c < i; ++c) f(kTX, i, c);
      }
    }
    if (K % 2 == 0) {                                          // late LT
      const int s = K / 2;
      const int jmin = s - (N - 1) > 0 ? s - (N - 1) : 0;
      for (int j = (s - kPPBand - 1) / 2; j >= jmin && s >= kPPBand + 1; --j) f(kTL, s - j, j);
    }
  }
  if (t % 4 == 2 && (t + 2) / 4 >= 2 && (t + 2) / 4 <= N - 1) f(kTDP, 0, (t + 2) / 4);
  if (t % 4 == 1 && (t - 1) / 4 >= 1 && (t - 1) / 4 <= N - 2) f(kTSP, (t - 1) / 4 + 1, (t - 1) / 4);
  if (t % 2 == 0 && t >= 4) {                                  // band LT on anti-diagonal s
    const int s = t / 2;
    const int jmin = (s - kPPBand + 1) / 2 > s - (N - 1) ? (s - kPPBand + 1) / 2 : s - (N - 1);
    for (int j = (s - 2) / 2; j >= jmin && j >= 0; --j) f(kTL, s - j, j);
  }
}

GP_HD inline int pp_nkeys(int N, int lead, int xd) { return 4 * N - 1 + 4 * (lead + xd); }

// Also zeroes the launch's flag words (dequeue head + per-tile flags) and info / logdet (in
// place of three memset launches ahead of it: ~30 us of a C3 step); `preset_abort` (the
// gp_set_poll_budget test hook) then marks every problem as having spent its poll budget.
// Block b of the grid writes the entries of problems b, b + gridDim.x, ... (every block runs
// the same per-key count and scan) and zeroes those problems' flag words; block 0 also the
// header.  One block per problem of a batch: the fit's 24 x 512 schedule took 10.4 us on one
// block (profiles/r05/r05t_prof_fit.txt), most of it one thread storing a key's tasks for
// every problem in turn.
__global__ __launch_bounds__(1024) void pp_schedule_kernel(int2* tasks, int N, int batch,
                                                           int inv, int lead, int xd,
                                                           int* head, int nhead,
                                                           int* info, double* logdet,
                                                           int* flags, int fstride,
                                                           int preset_abort) {
  __shared__ int cnt[2][1024];
  const int T = threadIdx.x;
  if (blockIdx.x == 0)
    for (int q = T; q < nhead; q += blockDim.x) head[q] = 0;
  for (int b = blockIdx.x; b < batch; b += gridDim.x) {
    for (int q = T; q < fstride; q += blockDim.x) flags[(long long)b * fstride + q] = 0;
    if (T == 0) {
      if (info) info[b] = 0;
      if (logdet) logdet[b] = 0.0;
    }
  }
  const int nk = pp_nkeys(N, lead, xd);
  int own = 0;
  if (T < nk) pp_for_key(T, N, inv != 0, lead, xd, [&](int, int, int) { ++own; });
  cnt[0][T] = own;
  __syncthreads();
  int src = 0;
  for (int off = 1; off < 1024; off <<= 1) {   // inclusive Hillis-Steele scan
    cnt[src ^ 1][T] = cnt[src][T] + (T >= off ? cnt[src][T - off] : 0);
    __syncthreads();
    src ^= 1;
  }
  // (after the barriers above: this block's zeroing is complete)
  if (T == 0)
    for (int b = blockIdx.x; b < batch; b += gridDim.x) {
      if (preset_abort) flags[(long long)b * fstride + 2 * N * N + 2 * N] = 2;
      tasks[b] = make_int2(kTChain | (b << 4), 0);
    }
  if (T >= nk) return;
  const int excl = cnt[src][T] - own;
  long long pos = batch + (long long)excl * batch;
  pp_for_key(T, N, inv != 0, lead, xd, [&](int kind, int i, int j) {
    for (int b = blockIdx.x; b < batch; b += gridDim.x)
      tasks[pos + b] = make_int2(kind | (b << 4), i | (j << 16));
    pos += batch;
  });
}

// Schedule blocks: one per problem up to one per CU (the rest loop)
static int pp_schedule_grid(int batch) { return batch < 256 ? batch : 256; }

// Tasks per problem, chain included (host side of the same enumeration; any lead gives the
// same total).
long long pp_task_count(int N, bool inv) {
  long long c = 1;
  for (int t = 0; t < pp_nkeys(N, 0, 0); ++t)
    pp_for_key(t, N, inv, 0, 0, [&](int, int, int) { ++c; });
  return c;
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

// gp_set_potrf_path (test / A-B hook): 1 forces the blocked sweep for later factorisations,
// 2 the persistent kernel with one shared queue for every batch
static int g_potrf_path = 0;

static int num_cus() {
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

// pp_kernel workgroups that can be resident at once on `stream`: its occupancy (1 per CU) x
// the CUs the stream's CU mask enables.  The dequeue lead and the eligibility test are bounded
// by this, not by the launched grid: a workgroup that is launched but never resident cannot
// take a task.
static int pp_resident(hipStream_t stream) {
  static const int occ = [] {
    int o = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&o, pp_kernel<false>, 256, 0) != hipSuccess ||
        o <= 0)
      o = 1;
    return o;
  }();
  int cus = num_cus();
  std::vector<uint32_t> mask((cus + 31) / 32, 0u);
  if (hipExtStreamGetCUMask(stream, (uint32_t)mask.size(), mask.data()) == hipSuccess) {
    int on = 0;
    for (uint32_t w : mask) on += __builtin_popcount(w);
    if (on > 0 && on < cus) cus = on;
  }
  return occ * cus;
}

// Dequeue lead (see pp_schedule_kernel): W = kPPLead while every problem's chain and blocked
// early tasks leave a resident worker free, else the topological order (W = 0).
static int pp_lead(int batch, int resident) {
  return (long long)batch * (kPPLeadBlocked + 1) < resident ? kPPLead : 0;
}

// Dequeue queues of a batched persistent factorisation.  Every task-list entry of problem b
// sits at an index congruent to b mod batch (the list is the batch's chains, then each task for
// b = 0..batch-1 in turn), so for batch % 8 == 0 the entries 8k + g are exactly the tasks of the
// problems b % 8 == g, in the list's order.  With 8 queues workgroup w dequeues only from queue
// w % 8: a problem's tasks all run on workgroups w, w + 8, ..., which the dispatcher places on
// one XCD (round-robin placement, MI355X_MICROARCH.md "Workgroup dispatch"), so the tiles they
// hand each other and re-read (every L_jk of a row, D_j) are served by that XCD's L2 instead of
// being fetched once per XCD from the Infinity Fabric.  Placement is a speed assumption only:
// each queue is a problem-closed, per-problem topological list served by grid / 8 workgroups,
// and the deadlock argument of pp_schedule_kernel holds per queue (pp_lead / pp_eligible scaled
// by 8 are the same inequalities).  Not for batch 1 (C3): one problem on one XCD would leave
// seven idle.
static int pp_groups(int batch, int grid) {
  return (g_potrf_path != 2 && batch >= 8 && batch % 8 == 0 && grid % 8 == 0) ? 8 : 1;
}

// Scratch of one persistent factorisation: the task list, a 256-B header (dequeue counters, exit
// counter) and the per-problem flag words.
struct PPScratch {
  long long ntasks;
  int fstride;
  size_t task_bytes, flag_bytes;
  size_t bytes() const { return task_bytes + flag_bytes; }
};

static PPScratch pp_scratch(int n, int batch, bool inv) {
  PPScratch s;
  const int N = gp_ceil_div(n, NB);
  s.ntasks = pp_task_count(N, inv) * batch;
  s.fstride = ((2 * N * N + 2 * N + 1 + 31) / 32) * 32;   // FL, FX, DPF, SPF, abort
  s.task_bytes = ((size_t)s.ntasks * sizeof(int2) + 255) / 256 * 256;
  s.flag_bytes = ((256 + (size_t)batch * s.fstride * sizeof(int)) + 255) / 256 * 256;
  return s;
}

static bool pp_shape_ok(int n, int batch) {
  const int N = gp_ceil_div(n, NB);
  return N <= kPPMaxN && pp_task_count(N, true) * (long long)batch < (1ll << 30);
}


static bool pp_eligible(int n, int batch, int resident) {
  // the chains hold `batch` workgroups for the whole launch: at least as many workers again
  return g_potrf_path != 1 && pp_shape_ok(n, batch) && 2 * batch <= resident;
}

// The persistent dataflow factorisation (pp_kernel) on `stream` in the caller's scratch `scr`
// (pp_scratch bytes, 256-B aligned): one schedule launch, one persistent launch with one
// workgroup per resident slot.  X is L^-1 (inv, zeroed by the caller) or the 64 x 64N D_k
// scratch (ldx = 64).
// gp_loglik's in-chain mode (gpfit_potrf_loglik): pp_kernel<true> with these PPArgs fields
struct PPLL {
  const double* w; int ldw;
  double* zb; int zld, zq_off;
  double* zz; double* ll; int* status; int* info_out;
};

static int pp_factor(double* A, int n, int lda, long long sA, double* X, int ldx, long long sX,
                     int batch, int* info, double* logdet, bool inv, char* scr, int resident,
                     hipStream_t stream, GpfitPre pre = GpfitPre(),
                     hipEvent_t ev_launch = nullptr, const PPLL* ll = nullptr) {
  const int N = gp_ceil_div(n, NB);
  const PPScratch s = pp_scratch(n, batch, inv);
  const int grid = (int)(s.ntasks < resident ? s.ntasks : resident);
  int2* tasks = reinterpret_cast<int2*>(scr);
  int* head = reinterpret_cast<int*>(scr + s.task_bytes);
  int* flags = reinterpret_cast<int*>(scr + s.task_bytes + 256);
  const int lead = pp_lead(batch, grid);
  const long long budget = g_poll_budget;
  // the schedule kernel also zeroes head + flags and info / logdet
  hipLaunchKernelGGL(pp_schedule_kernel, dim3(pp_schedule_grid(batch)), dim3(1024), 0, stream,
                     tasks, N, batch, inv ? 1 : 0, lead, kPPXDelay, head, 256 / (int)sizeof(int),
                     info, logdet, flags, s.fstride, budget < 0 ? 1 : 0);
  GP_CK(hipGetLastError());
  if (pre.fn) {
    const int prc = pre.fn(pre.arg);
    if (prc) return prc;
  }
  if (ev_launch) GP_CK(hipEventRecord(ev_launch, stream));   // after the Gram, before pp_kernel
  PPArgs P;
  P.A = A; P.sA = sA; P.lda = lda;
  P.X = X; P.sX = sX; P.ldx = ldx;
  P.n = n; P.N = N; P.batch = batch; P.inv = inv ? 1 : 0;
  // plain (L2-cached) loads of produced tiles only when no 128-B line spans two tiles
  auto al128 = [](const void* p) { return (reinterpret_cast<uintptr_t>(p) & 127) == 0; };
  P.plain = (lda % 16 == 0) && (ldx % 16 == 0) && al128(A) && al128(X) &&
            (batch == 1 || (sA % 16 == 0 && sX % 16 == 0));
  P.budget = budget > 0 ? budget : kPollBudget;
  P.info = info; P.logdet = logdet;
  P.tasks = tasks; P.ntasks = (int)s.ntasks;
  P.groups = pp_groups(batch, grid);
  P.head = head; P.flags = flags; P.fstride = s.fstride;
#ifdef GPFIT_PP_TRACE
  P.dbg = g_trace_dbg;
  P.trace = g_trace_buf;
#endif
  P.w = nullptr; P.ldw = 0; P.zb = nullptr; P.zld = 0; P.zq_off = 0;
  P.zz = nullptr; P.ll = nullptr; P.status = nullptr; P.info_out = nullptr;
  if (ll) {
    P.w = ll->w; P.ldw = ll->ldw; P.zb = ll->zb; P.zld = ll->zld; P.zq_off = ll->zq_off;
    P.zz = ll->zz; P.ll = ll->ll; P.status = ll->status; P.info_out = ll->info_out;
    hipLaunchKernelGGL(pp_kernel<true>, dim3(grid), dim3(256), 0, stream, P);
  } else {
    hipLaunchKernelGGL(pp_kernel<false>, dim3(grid), dim3(256), 0, stream, P);
  }
  GP_CK(hipGetLastError());
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

static bool ws_aligned(const void* ws) { return (reinterpret_cast<uintptr_t>(ws) & 255) == 0; }

long long gpfit_potrf_inv_ws_bytes(int n, int batch) {
  if (n <= 0 || batch <= 0 || !pp_shape_ok(n, batch)) return 0;
  return (long long)pp_scratch(n, batch, true).bytes();
}

extern "C" long long gp_potrf_inv_ws_bytes(int n, int batch) {
  if (n < 0 || batch < 0) return -1;
  return gpfit_potrf_inv_ws_bytes(n, batch);
}

extern "C" long long gp_potrf_ws_bytes(int n, int batch) {
  if (n < 0 || batch < 0) return -1;
  if (n == 0 || batch == 0) return 0;
  const long long sD = (long long)NB * gp_ceil_div(n, NB) * NB;
  const long long d = ((8LL * sD * batch) + 255) / 256 * 256;
  return d + (pp_shape_ok(n, batch) ? (long long)pp_scratch(n, batch, false).bytes() : 0);
}

static int potrf_inv_args(const double* A, int n, int lda, long long strideA, const double* Linv,
                          int ldinv, long long strideInv, int batch) {
  if (!A) return -1;
  if (n < 0) return -2;
  if (lda < n || lda < 1) return -3;
  if (batch > 1 && strideA < (long long)lda * n) return -4;
  if (!Linv) return -5;
  const int npad = gp_padded_n(n);
  if (ldinv < npad || ldinv < 1) return -6;
  if (batch > 1 && strideInv < (long long)ldinv * npad) return -7;
  if (batch < 0) return -8;
  return 0;
}

static int potrf_args(const double* A, int n, int lda, long long strideA, int batch) {
  if (!A) return -1;
  if (n < 0) return -2;
  if (lda < n || lda < 1) return -3;
  if (batch > 1 && strideA < (long long)lda * n) return -4;
  if (batch < 0) return -5;
  return 0;
}

int gpfit_potrf_inv_event(double* A, int n, int lda, long long strideA, double* Linv,
                          int ldinv, long long strideInv, int batch, int* info, double* logdet,
                          void* ws, long long ws_bytes, hipStream_t stream, int k_ev,
                          hipEvent_t ev, GpfitPre pre) {
  const int arc = potrf_inv_args(A, n, lda, strideA, Linv, ldinv, strideInv, batch);
  if (arc) return arc;
  if (n == 0 || batch == 0) return pre.fn ? pre.fn(pre.arg) : 0;
  const int npad = gp_padded_n(n);
  const int resident = pp_resident(stream);
  const bool pp = pp_eligible(n, batch, resident);
  if (pp) {
    if (!ws || !ws_aligned(ws)) return -11;
    if (ws_bytes < gpfit_potrf_inv_ws_bytes(n, batch)) return -12;
  } else {   // (pp_factor's schedule kernel zeroes them)
    if (pre.fn) {
      const int prc = pre.fn(pre.arg);
      if (prc) return prc;
    }
    if (info) GP_CK(hipMemsetAsync(info, 0, sizeof(int) * batch, stream));
    if (logdet) GP_CK(hipMemsetAsync(logdet, 0, sizeof(double) * batch, stream));
  }
  // the persistent kernel zeroes what it does not write itself (its zero tasks)
  if (!pp) GP_CK(zero_linv(Linv, npad, ldinv, strideInv, batch, stream));
  gpfit_prof_begin(GP_PROF_POTRF, stream);
  int rc;
  if (pp) {
    // one launch, no block steps: an event asked for at a step inside the factorisation is
    // recorded just before the persistent launch, after the schedule kernel and `pre` (whatever
    // waits on it runs beside the whole factorisation, not beside the Gram),
    // one asked for at k_ev >= N after it
    const int N = gp_ceil_div(n, NB);
    rc = pp_factor(A, n, lda, strideA, Linv, ldinv, strideInv, batch, info, logdet, true,
                   static_cast<char*>(ws), resident, stream, pre,
                   (ev && k_ev >= 0 && k_ev < N) ? ev : nullptr);
    if (rc == 0 && ev && !(k_ev >= 0 && k_ev < N)) GP_CK(hipEventRecord(ev, stream));
  } else {
    rc = potrf_sweep<kPotrfInv>(A, n, lda, strideA, Linv, ldinv, strideInv, batch, info, logdet,
                                stream, k_ev, ev);
  }
  gpfit_prof_end(GP_PROF_POTRF, stream);
  return rc;
}

// gp_loglik on the persistent kernel's in-chain mode (gpfit_internal.h).
long long gpfit_potrf_loglik_ws_bytes(int n, int batch) {
  return (long long)pp_scratch(n, batch, false).bytes();
}

int gpfit_potrf_loglik(double* G, int n, long long strideG, double* D, long long strideD,
                       const double* w, int ldw, double* zb, int zld, double* zz, int batch,
                       int* info, double* logdet, double* ll, int* status, int* info_out,
                       void* ws, long long ws_bytes, hipStream_t stream, GpfitPre pre) {
  const int resident = pp_resident(stream);
  if (!pp_eligible(n, batch, resident)) return 1;   // the caller's L^-1 path
  if (!ws || !ws_aligned(ws)) return -11;
  if (ws_bytes < gpfit_potrf_loglik_ws_bytes(n, batch)) return -12;
  const int N = gp_ceil_div(n, NB);
  if (strideD < (long long)NB * NB * N || zld < 2 * NB * N) return -13;
  PPLL L{w, ldw, zb, zld, NB * N, zz, ll, status, info_out};
  // (the profiler's POTRF pair brackets the Gram `pre` too on this path: it is enqueued
  // between the schedule kernel and pp_kernel; the fit's roofline subtracts nothing for it)
  gpfit_prof_begin(GP_PROF_POTRF, stream);
  const int rc = pp_factor(G, n, n, strideG, D, NB, strideD, batch, info, logdet, false,
                           static_cast<char*>(ws), resident, stream, pre, nullptr, &L);
  gpfit_prof_end(GP_PROF_POTRF, stream);
  return rc;
}

extern "C" int gp_potrf_inv_ws(double* A, int n, int lda, long long strideA, double* Linv,
                               int ldinv, long long strideInv, int batch, int* info,
                               double* logdet, void* ws, long long ws_bytes,
                               hipStream_t stream) {
  return gpfit_potrf_inv_event(A, n, lda, strideA, Linv, ldinv, strideInv, batch, info, logdet,
                               ws, ws_bytes, stream, -1, nullptr);
}

// The allocating forms: stream-ordered scratch (hipMallocAsync), freed behind the launches on
// every path, including a failed launch.
extern "C" int gp_potrf_inv(double* A, int n, int lda, long long strideA, double* Linv,
                            int ldinv, long long strideInv, int batch, int* info,
                            double* logdet, hipStream_t stream) {
  const int arc = potrf_inv_args(A, n, lda, strideA, Linv, ldinv, strideInv, batch);
  if (arc) return arc;
  const long long bytes = (n > 0 && batch > 0) ? gpfit_potrf_inv_ws_bytes(n, batch) : 0;
  void* ws = nullptr;
  if (bytes > 0) GP_CK(hipMallocAsync(&ws, (size_t)bytes, stream));
  const int rc = gp_potrf_inv_ws(A, n, lda, strideA, Linv, ldinv, strideInv, batch, info,
                                 logdet, ws, bytes, stream);
  if (ws) {
    const hipError_t e = hipFreeAsync(ws, stream);
    if (rc == 0 && e != hipSuccess) return GPFIT_ERR_HIP - (int)e;
  }
  return rc;
}

extern "C" int gp_potrf_ws(double* A, int n, int lda, long long strideA, int batch, int* info,
                           double* logdet, void* ws, long long ws_bytes, hipStream_t stream) {
  const int arc = potrf_args(A, n, lda, strideA, batch);
  if (arc) return arc;
  if (n == 0 || batch == 0) return 0;
  if (!ws || !ws_aligned(ws)) return -8;
  if (ws_bytes < gp_potrf_ws_bytes(n, batch)) return -9;
  const int resident = pp_resident(stream);
  const bool pp = pp_eligible(n, batch, resident);
  if (!pp) {   // (pp_factor's schedule kernel zeroes them)
    if (info) GP_CK(hipMemsetAsync(info, 0, sizeof(int) * batch, stream));
    if (logdet) GP_CK(hipMemsetAsync(logdet, 0, sizeof(double) * batch, stream));
  }
  // D_k scratch: NB x (N NB) per problem at the head of ws, then the persistent scratch
  const int N = gp_ceil_div(n, NB);
  const long long sD = (long long)NB * N * NB;
  double* D = static_cast<double*>(ws);
  char* scr = static_cast<char*>(ws) + ((8LL * sD * batch) + 255) / 256 * 256;
  return pp ? pp_factor(A, n, lda, strideA, D, NB, sD, batch, info, logdet, false, scr, resident,
                        stream)
            : potrf_sweep<kPotrf>(A, n, lda, strideA, D, NB, sD, batch, info, logdet, stream,
                                  -1, nullptr);
}

extern "C" int gp_potrf(double* A, int n, int lda, long long strideA, int batch, int* info,
                        double* logdet, hipStream_t stream) {
  const int arc = potrf_args(A, n, lda, strideA, batch);
  if (arc) return arc;
  const long long bytes = (n > 0 && batch > 0) ? gp_potrf_ws_bytes(n, batch) : 0;
  void* ws = nullptr;
  if (bytes > 0) GP_CK(hipMallocAsync(&ws, (size_t)bytes, stream));
  const int rc = gp_potrf_ws(A, n, lda, strideA, batch, info, logdet, ws, bytes, stream);
  if (ws) {
    const hipError_t e = hipFreeAsync(ws, stream);
    if (rc == 0 && e != hipSuccess) return GPFIT_ERR_HIP - (int)e;
  }
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

// Poll budget of the persistent factorisation's waits for later launches (process-wide test /
// diagnostics hook): polls > 0 sets it, 0 restores the default, < 0 makes every later
// factorisation start with its problems aborted (info = -1: the deterministic abort path).
// Returns the previous setting.
extern "C" long long gp_set_poll_budget(long long polls) {
  const long long prev = g_poll_budget;
  g_poll_budget = polls == 0 ? kPollBudget : polls;
  return prev;
}

// Factorisation path for later enqueues (process-wide test / A-B hook): 0 = automatic (the
// persistent kernel where eligible, per-XCD queues for batches of 8k), 1 = always the blocked
// sweep, 2 = the persistent kernel with one shared queue.  Returns the previous value.
extern "C" int gp_set_potrf_path(int path) {
  const int prev = g_potrf_path;
  g_potrf_path = (path == 1 || path == 2) ? path : 0;
  return prev;
}

#ifdef GPFIT_PP_TRACE
// Trace build only (libgpfit_trace.so): device buffers the next persistent launches fill.
extern "C" int gp_pp_trace_set(void* dbg, void* trace) {
  g_trace_dbg = static_cast<int*>(dbg);
  g_trace_buf = static_cast<long long*>(trace);
  return 0;
}
extern "C" long long gp_pp_trace_slots(int n, int batch) {
  const int N = gp_ceil_div(n, NB);
  return pp_scratch(n, batch, true).ntasks * kPPTraceSlots + (long long)batch * N * 8;
}
#endif
#undef GP_CK
