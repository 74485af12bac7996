// Posterior mean / marginal variance for batches of GPs (the dominant cost of the path).
//
// Reference replaced: SepiaEmulatorPrediction's predictive mean and covariance diagonal
// (analysis/time_predictions.py:76-78, assess_all_models.py:489, sensitivity_indices.py:85),
// i.e. examples/02...ipynb:232-233 restricted to the diagonal:
//   mean = K* A^-1 w ,  var = s_pred - diag(K* A^-1 K*^T),  A = L L^T.
// With X = L^-1 (from gp_potrf_inv) and V = X K*^T:  mean_j = z^T V[:,j] (z = X w) and
// var_j = s_pred - ||V[:,j]||^2, so ONE triangular matrix product per test-point chunk gives
// both; V is reduced in registers and never written.
//
// Per chunk of m_c test points:
//   1. cross_kp           Kt = s exp(-sum beta (X - Xs)^2), n_pad x m_c, k-major rows of m_c
//                         test points (the TRMM's LDS image row by row; exp once per element)
//   2. trmm_pair          for each 128x128 tile (I, C) of V: acc = sum_{k < 128(I+1)} X[I,k] Kt[k,C]
//                         on v_mfma_f64_16x16x4_f64 (row tiles NI-1-p and p in one block),
//                         epilogue: per-column partial sums of acc*z and acc^2 ->
//                         part[b][I][col]  (MFMA-bound: n^2 m flop)
//   3. finalize           mean = sum_I pm, var = s_pred - sum_I pv
// z = X w is a small lower-triangular gemv (linalg.hip trmv_kernel).
#include "gpfit_common.h"
#include <cstdlib>
#include "gpfit_profile.h"
#include "gpfit_internal.h"
#include "../../include/gpfit.h"
#include <atomic>
#include <new>
#include <vector>

namespace {

constexpr int BI = 128;   // V tile rows (L^-1 rows)
constexpr int BC = 128;   // V tile cols (test points)
constexpr int BK = 16;    // K step
constexpr long long kDefaultChunkElems = 256ll << 20;  // <= 2 GB of Kt per chunk
constexpr int kDefaultChunk = 8192;                   // test points per chunk (batches)
constexpr int kDefaultChunkSingle = 16384;            // ... and for one GP
// Non-temporal cross-covariance stores (the chunk, 2.15 GB at C4, is read back by the TRMM from
// HBM either way): C4 59.1-59.6 -> 58.7-58.8 ms per step, C3 unchanged
// (profiles/r06/r06ai_ab_cross_nt.log)
#ifndef CROSS_NT
#define CROSS_NT 1
#endif

// Cross-covariance chunk, k-major as the TRMM streams it:
//   Kt[k * mc + c] = s * exp(-sum beta (X[k] - Xs[c])^2)
// (exp by the 64-entry table, exp_neg_tab: the kernel is bound by its fp64 VALU work)
// (zero for k >= n or c >= mv).  Each thread owns one test point c (registers) and walks 32
// k-pairs whose design rows are broadcast from LDS; a wave stores 512 contiguous bytes per
// row k.  Both design vectors are pre-scaled by sqrt(beta) (beta >= 0): 2 d ops per element
// for the distance instead of 3 d (see gram.hip for the rounding bound).
template <int D>
__global__ __launch_bounds__(256) void cross_kp_kernel(
    const double* __restrict__ X, int n, int ldx, const double* __restrict__ Xs, int mv,
    int ldxs, int d, const double* __restrict__ beta, int ldbeta, const double* __restrict__ s,
    double* __restrict__ Kt2, int mc, long long sK) {
  const int b = blockIdx.z;
  const int c = blockIdx.x * 256 + threadIdx.x;
  const int kp0 = blockIdx.y * 32;
  __shared__ double xk[64][D];
  __shared__ double bs[D];
  __shared__ double tab[64];
  const double* bb = beta + (long long)b * ldbeta;
  if (threadIdx.x < D) bs[threadIdx.x] = (threadIdx.x < d) ? __builtin_sqrt(bb[threadIdx.x]) : 0.0;
  if (threadIdx.x < 64) tab[threadIdx.x] = kExp2Tab[threadIdx.x];
  __syncthreads();
  for (int t = threadIdx.x; t < 64 * D; t += 256) {
    const int kk = t / D, dd = t % D, k = 2 * kp0 + kk;
    xk[kk][dd] = (k < n && dd < d) ? X[(long long)k * ldx + dd] * bs[dd] : 0.0;
  }
  double xc[D];
#pragma unroll
  for (int dd = 0; dd < D; ++dd)
    xc[dd] = (c < mv && dd < d) ? Xs[(long long)c * ldxs + dd] * bs[dd] : 0.0;
  __syncthreads();
  if (c >= mc) return;
  const double sb = s[b];
  double* o = Kt2 + (long long)b * sK;
  const bool col_ok = c < mv;
#pragma unroll 2
  for (int kk = 0; kk < 32; ++kk) {
    const int k = 2 * (kp0 + kk);
    double e0 = 0.0, e1 = 0.0;
#pragma unroll
    for (int dd = 0; dd < D; ++dd) {
      const double t0 = xk[2 * kk][dd] - xc[dd], t1 = xk[2 * kk + 1][dd] - xc[dd];
      e0 = fma(t0, t0, e0);
      e1 = fma(t1, t1, e1);
    }
    // exp unconditionally, then select: padding rows / columns have finite (zeroed) inputs,
    // and a conditional exp costs an exec-mask branch around each call
    const double v0 = sb * exp_neg_tab(e0, tab), v1 = sb * exp_neg_tab(e1, tab);
#if CROSS_NT
    __builtin_nontemporal_store((col_ok && k < n) ? v0 : 0.0, o + (long long)k * mc + c);
    __builtin_nontemporal_store((col_ok && k + 1 < n) ? v1 : 0.0, o + (long long)(k + 1) * mc + c);
#else
    o[(long long)k * mc + c] = (col_ok && k < n) ? v0 : 0.0;
    o[(long long)(k + 1) * mc + c] = (col_ok && k + 1 < n) ? v1 : 0.0;
#endif
  }
}

// One 128x128 tile of V = Linv * Kt per block, 4 waves in 2 wave rows x 2 wave columns: a wave
// owns four 16-row MFMA row tiles (dealt in a snake, trmm_rtile) x 64 columns (4x4 MFMA tiles).
// Operands stream straight into LDS with global_load_lds (16 B per lane), double-buffered:
//   A step (16 k x 128 rows of L^-1): 16 rows of 1 KB, row pitch 1152 B (lanes 0-15 / 16-31
//     of a fragment read land 32 banks apart: conflict-free)
//   B step (16 k x 128 test points): 16 rows of 1 KB, the k-major rows of cross_kp_kernel, so
//     each 16-lane group of a fragment read covers 128 contiguous bytes (conflict-free; the
//     earlier k-pair-interleaved image put lanes li and li + 8 on one bank: 33% of LDS cycles
//     were bank conflicts, SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE).
// One barrier per K-step; ~69 KB of LDS and <= 256 VGPRs -> 2 blocks (8 waves) per CU.
constexpr int APITCH = 144;                    // doubles per staged A row (1152 B)
constexpr int ASTAGE = BK * APITCH;            // 2304 doubles
constexpr int BSTAGE = (BK / 2) * BC * 2;      // 2048 doubles
constexpr int STAGE = ASTAGE + BSTAGE;         // 4352 doubles = 34816 B

GP_DEV void glds16(const double* g, double* l) {
  __builtin_amdgcn_global_load_lds((const void __attribute__((address_space(1)))*)g,
                                   (void __attribute__((address_space(3)))*)l, 16, 0, 0);
}

// The 16-row MFMA tiles of a 128-row tile are dealt to the two wave rows in a snake,
// wave row wr owning tiles {wr, 3-wr, 4+wr, 7-wr}: inside the diagonal block, where tile r only
// meets nonzero L^-1 in the steps t <= r, both wave rows then run 18 of the block's 32
// tile-steps, instead of 10 and 26 with contiguous halves -- a step's barrier waits for the
// busier row, so the diagonal block took 6.5 steps' time for 4.5 steps of work.
GP_DEV constexpr int trmm_rtile(int mi, int wr) { return 2 * mi + ((mi & 1) ? 1 - wr : wr); }

// One staged K step (16 k) of a wave's four 16 x 64 MFMA row tiles.  TAIL: the step is step t
// of the tile's diagonal block of L^-1, where row tile r only meets nonzero L^-1 entries when
// r >= t.  The skipped products are exact zeros (L^-1 is zero above the diagonal), so the sums
// are unchanged and the SIMD goes to the co-resident block's waves instead.
template <bool TAIL>
GP_DEV void trmm_stage(const double* __restrict__ As, const double* __restrict__ Bs,
                       f64x4 (&acc)[4][4], int wr, int wc, int li, int lk, int t) {
#pragma unroll
  for (int k4 = 0; k4 < BK / 4; ++k4) {
    const int k = k4 * 4 + lk;
    double a[4], bb[4];
#pragma unroll
    for (int mi = 0; mi < 4; ++mi)
      if (!TAIL || trmm_rtile(mi, wr) >= t) a[mi] = As[k * APITCH + trmm_rtile(mi, wr) * 16 + li];
#pragma unroll
    for (int nj = 0; nj < 4; ++nj)
      bb[nj] = Bs[k * BC + wc * 64 + nj * 16 + li];
#pragma unroll
    for (int mi = 0; mi < 4; ++mi) {
      if (TAIL && trmm_rtile(mi, wr) < t) continue;
#pragma unroll
      for (int nj = 0; nj < 4; ++nj) acc[mi][nj] = mfma16x16x4(a[mi], bb[nj], acc[mi][nj]);
    }
  }
}

// blockIdx.x -> (pair p, panel C).  Blocks b and b + 8 share an XCD (dispatch is round-robin
// over the 8 XCDs), so with kXcdPanels = G > 0 the blocks of XCD slot x = b % 8 are laid out in
// its own order t = b / 8 as groups of G panels (x, x + 8, ...) x all pairs, pair-major.  An
// XCD's 64 resident blocks then hold G panels x 64/G pairs: each K* panel is read by 64/G
// blocks at once and each L^-1 pair by G.  G = 0: pair-major over all panels (p = b / NC,
// i.e. 16 panels x 4 pairs per XCD at C3, the K* panels re-fetched in every residency round).
// C3 TRMM fabric traffic (FETCH_SIZE x2): G = 0 5.09 GB per launch, G = 4 4.52, G = 8 4.18;
// launch time unchanged (profiles/r03/ab_map.log).
#ifndef TRMM_XCD_PANELS
#define TRMM_XCD_PANELS 8
#endif
constexpr int kXcdPanels = TRMM_XCD_PANELS;
// Diagonal-block steps (timing experiments only; 0 is the library): 1 = every MFMA of the step
// (exact for the padded layout, whose upper triangle is zero), 2 = none (wrong results)
#ifndef TRMM_DIAG_MODE
#define TRMM_DIAG_MODE 0
#endif
// XCD-local (problem, pair) units for batched launches (A/B build only): C4 TRMM 4.090 vs
// 4.105-4.125 ms per launch, but 9.44 vs 5.47 GB of fabric traffic per launch (every K* panel
// fetched by four XCDs; profiles/r05/r05m_umap.log, r05n_pmc_c4.log): not the default
#ifndef TRMM_UNIT_MAP
#define TRMM_UNIT_MAP 0
#endif

// The tile-packed L^-1 (GPFIT_LINV_PACKED, the single-GP broadcast's payload): column k of the
// padded npad x npad L^-1 from row 16 floor(k / 16) on, columns one after another, so every
// stored run starts on a 16-row MFMA tile and is a multiple of 16 doubles (128-B aligned).
// Element (r, k), r >= 16 floor(k / 16), sits at linv_col(k, npad) + r.  Rows below the start
// hold other columns' data: the TRMM's diagonal-block steps never use them (row tile r < t is
// skipped at step t) and the trmv masks them, so results equal the padded layout's bit for bit.
//   linv_col(k) = k npad - 16 sum_{j < k} floor(j / 16) - 16 floor(k / 16)
__host__ __device__ inline long long linv_col(long long k, long long npad) {
  const long long q = k >> 4;
  return k * npad - 128 * q * (q - 1) - 16 * q * (k - 16 * q) - 16 * q;
}
__host__ __device__ inline long long linv_packed_elems(long long npad) {
  const long long q = npad >> 4;
  return npad * npad - 128 * q * (q - 1);
}

// One TRMM launch covers `NCt` column panels of each of `batch` problems -- the panels of one
// test-point chunk, or of the last two chunks merged (a chunk whose blocks fill less than one
// residency round runs with the chunk before it, trmm_launch) -- numbered g = b * NCt + C
// (problem-major).  Panel C of the launch lies in chunk C / NCc (relative to the launch's first
// chunk), whose cross-covariance and partial sums are `slab` / `pslab` doubles after the first
// chunk's.
//
// The schedule (which blocks compute which tiles, trmm_sched) changes no sum: every tile (I, g)
// is computed by one block with the same K order wherever it runs (natural order, or for a tile
// that is the second of its row-tile pair, its diagonal block first: trmm_diag_first), so
// results are bit-identical whatever the chunking and the schedule.
struct TrmmArgs {
  const double* Linv;      // padded (column k at k * ld) or tile-packed (linv_col, PACKED)
  long long sL;
  const double* Kt2;       // the launch's first chunk's cross-covariance slab
  long long sK, slab;      // problem stride inside a slab; slab stride (chunk to chunk)
  const double* z;
  long long zld;           // z problem stride
  double* part;            // the launch's first chunk's partial-sum slab
  long long pslab;         // partial-sum slab stride
  int ld, mc, NCc, NCt, npad, NI;
  int Gp;                  // panels g < Gp: row-tile pair blocks (uniform 8 (NI + 1) K steps)
  int Gx;                  //   ... of which g < Gx (a multiple of 8 kXcdPanels) in the XCD order
  int Qc;                  // panels g >= Gp: one block per tile, longest tiles first
  int umap;                // batched launches: XCD-local (problem, pair) units (trmm_sched)
};

// A tile's K order: the second tile of a row-tile pair (I < NI - 1 - I) runs its diagonal block
// first (kDiagFirst, below); every other tile runs k = 0, 1, ... .
GP_DEV bool trmm_diag_first(int I, int NI);

// blockIdx.x -> (panel g, first tile I0, second tile I1 or -1).
//  * Pair blocks (bid < Gp NP): tiles (NI-1-p, g) then (p, g).  The first Gx panels in the
//    XCD-aware order: blocks b and b + 8 share an XCD (dispatch is round-robin over the 8 XCDs),
//    so the blocks of XCD slot x = b % 8 are laid out in their own order t = b / 8 as groups of
//    G = kXcdPanels panels (x, x + 8, ...) x all pairs, pair-major: an XCD's 64 resident blocks
//    hold G panels x 64/G pairs, each K* panel read by 64/G blocks at once and each L^-1 pair by
//    G (C3 TRMM fabric traffic, FETCH_SIZE x2: plain pair-major 5.09 GB per launch, G = 4 4.52,
//    G = 8 4.18; launch time unchanged, profiles/r03/ab_map.log).  The rest pair-major.
//  * Single-tile blocks (bid >= Gp NP): tile (I, g) for the last Qc panels, I descending (the
//    longest, 8 (I + 1) K steps, first): the dispatcher hands each freed slot the next block, so
//    the launch's last residency round is packed longest-first instead of leaving CUs idle
//    behind uniform pairs (trmm_sched).
GP_DEV void trmm_block_tiles(int bid, const TrmmArgs& a, int& g, int& I0, int& I1) {
  const int NP = (a.NI + 1) / 2;
  const int nA = a.Gp * NP;
  if (bid < nA) {
    int p;
    if (a.umap) {
      // unit u = (problem b, pair p) = u / NP, u % NP; XCD slot x takes units x, x + 8, ...,
      // each over all NCt panels of the launch in turn (t = bid / 8): one XCD's resident blocks
      // share one problem's pair p, i.e. two row tiles of L^-1 (<= 2 MB at n = 1024), where
      // problem-major panels spread a whole 8 MB L^-1 over every XCD's 4 MB L2
      const int x = bid & 7, t = bid >> 3, q = t / a.NCt;
      const int u = x + 8 * q, C = t - q * a.NCt;
      p = u % NP;
      g = (u / NP) * a.NCt + C;
    } else if (bid < a.Gx * NP) {
      const int x = bid & 7, t = bid >> 3, per = kXcdPanels * NP;
      const int grp = t / per, j = t - grp * per;
      p = j / kXcdPanels;
      g = x + 8 * (grp * kXcdPanels + j % kXcdPanels);
    } else {
      const int r = bid - a.Gx * NP, Gr = a.Gp - a.Gx;
      p = r / Gr;
      g = a.Gx + (r - p * Gr);
    }
    I0 = a.NI - 1 - p;
    I1 = (I0 == p) ? -1 : p;
    // (pair-order mixes -- reversed pairs in every other XCD group or block, or the pair's
    // diagonal-first tile first -- measured no different, profiles/r05/r05f_ab.log)
  } else {
    const int t = bid - nA;
    const int q = t / a.Qc;
    I0 = a.NI - 1 - q;
    g = a.Gp + (t - q * a.Qc);
    I1 = -1;
  }
}

// kDiagFirst: the second tile of a pair runs its diagonal block first.  A diagonal block's steps
// carry few MFMAs (row tile r only meets L^-1 at steps t <= r) and are bound by the next
// stage's load latency; with both tiles ending on their diagonal block every block of a
// residency round spent its last 8 steps there together (all co-resident blocks at once), while
// now pair p's two diagonal blocks sit back to back around step 8(NI - p), spread over the round.
// Measured: C4 TRMM 2.059 -> 2.051 ms per launch, C3 unchanged (profiles/r03/ab_df.log).
#ifndef TRMM_DIAG_FIRST
#define TRMM_DIAG_FIRST 1
#endif
constexpr bool kDiagFirst = TRMM_DIAG_FIRST;

GP_DEV bool trmm_diag_first(int I, int NI) { return kDiagFirst && 2 * I < NI - 1; }

// Row-tile pairs: block (p, g) computes tile (NI-1-p, g) and then tile (p, g), so every pair
// block runs 8(NI+1) K steps (uniform work: at C3 the 512 blocks of a residency round finish
// together) and the second tile's first stage is fetched under the first tile's last MFMAs;
// single-tile blocks (trmm_block_tiles) fill a launch's last round.  Per K step: the next
// stage's global_load_lds is issued, then the MFMAs of the current stage, then one vmcnt(0) +
// barrier.
template <bool PACKED>
__global__ __launch_bounds__(256, 2) void trmm_pair_kernel(const TrmmArgs a) {
  __shared__ __attribute__((aligned(16))) double smem[2 * STAGE];
  const int NI = a.NI, mc = a.mc, ld = a.ld;
  int g, Ifirst, Isecond;
  trmm_block_tiles(blockIdx.x, a, g, Ifirst, Isecond);
  const int b = g / a.NCt, Cl = g - b * a.NCt;       // problem, panel of the launch
  const int chr = Cl / a.NCc, C = Cl - chr * a.NCc;   // chunk (relative), panel in the chunk
  const int npass = (Isecond < 0) ? 1 : 2;
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = w >> 1, wc = w & 1, li = lane & 15, lk = lane >> 4;
  const double* Lb = a.Linv + b * a.sL + 2 * lane;                      // + I*BI + k*ld
  const double* K = a.Kt2 + chr * a.slab + b * a.sK + (long long)C * BC + 2 * lane;  // + k*mc
  double* const part = a.part + chr * a.pslab;

  auto issue = [&](const double* L, int s, double* st) {
    const int k0 = s * BK;
    // tile-packed: the step's 16 columns share their first stored row 16 s, so column k0 + kr
    // starts at linv_col(k0) + kr (npad - 16 s) (one multiply per row instead of linv_col's)
    const long long pbase = PACKED ? linv_col(k0, a.npad) : 0;
    const int pstride = PACKED ? a.npad - BK * s : 0;
#pragma unroll
    for (int r = 0; r < 4; ++r) {              // A rows k0 + 4w + r
      const int kr = 4 * w + r;
      const long long col = PACKED ? pbase + kr * pstride : (long long)(k0 + kr) * ld;
      glds16(L + col, st + kr * APITCH);
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) {              // B rows k0 + 4w + r
      const int kr = 4 * w + r;
      glds16(K + (long long)(k0 + kr) * mc, st + ASTAGE + kr * BC);
    }
  };
  // a tile's first K step: its diagonal block's when it runs that block first
  auto first_step = [&](int I) { return trmm_diag_first(I, NI) ? I * (BI / BK) : 0; };

  issue(Lb + Ifirst * BI, first_step(Ifirst), smem);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
#pragma unroll 1
  for (int pass = 0; pass < npass; ++pass) {
    const int I = pass ? Isecond : Ifirst;
    const double* L = Lb + I * BI;
    const int nsteps = (I + 1) * (BI / BK);   // even: the last step reads stage buffer 1
    f64x4 acc[4][4];
#pragma unroll
    for (int i4 = 0; i4 < 4; ++i4)
#pragma unroll
      for (int c = 0; c < 4; ++c) acc[i4][c] = zero4();
    const int s_diag = nsteps - BI / BK;
    int nst = nsteps;
    asm volatile("" : "+s"(nst));
    if (trmm_diag_first(I, NI)) {
      // the second tile: its diagonal block first (k-steps s_diag .., t = s), then k-steps 0 ..
      for (int s = 0; s < BI / BK; ++s) {
        double* cur = smem + (s & 1) * STAGE;
        if (s + 1 < BI / BK) issue(L, s_diag + s + 1, smem + ((s + 1) & 1) * STAGE);
        else if (nst > BI / BK) issue(L, 0, smem + ((s + 1) & 1) * STAGE);
        else if (pass + 1 < npass)               // (a diagonal-only first tile) next tile's
          issue(Lb + Isecond * BI, first_step(Isecond), smem);   // first stage
        if (TRMM_DIAG_MODE == 1) trmm_stage<false>(cur, cur + ASTAGE, acc, wr, wc, li, lk, 0);
        else if (TRMM_DIAG_MODE == 0 && s <= 7 - wr)
          trmm_stage<true>(cur, cur + ASTAGE, acc, wr, wc, li, lk, s);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
      }
      for (int s = BI / BK; s < nsteps; ++s) {
        double* cur = smem + (s & 1) * STAGE;
        if (s + 1 < nst) issue(L, s + 1 - BI / BK, smem + ((s + 1) & 1) * STAGE);
        else if (pass + 1 < npass)               // next tile's first stage
          issue(Lb + Isecond * BI, first_step(Isecond), smem);
        trmm_stage<false>(cur, cur + ASTAGE, acc, wr, wc, li, lk, 0);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
      }
    } else {
      int s = 0;
      for (; s < s_diag; ++s) {
        double* cur = smem + (s & 1) * STAGE;
        if (s + 1 < nst) issue(L, s + 1, smem + ((s + 1) & 1) * STAGE);
        trmm_stage<false>(cur, cur + ASTAGE, acc, wr, wc, li, lk, 0);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
      }
      for (; s < nsteps; ++s) {
        double* cur = smem + (s & 1) * STAGE;
        if (s + 1 < nst) issue(L, s + 1, smem + ((s + 1) & 1) * STAGE);
        else if (pass + 1 < npass)               // next tile's first stage
          issue(Lb + Isecond * BI, first_step(Isecond), smem);
        const int t = s - s_diag;               // the wave's last row tile is 7 - wr
        if (TRMM_DIAG_MODE == 1) trmm_stage<false>(cur, cur + ASTAGE, acc, wr, wc, li, lk, 0);
        else if (TRMM_DIAG_MODE == 0 && t <= 7 - wr)
          trmm_stage<true>(cur, cur + ASTAGE, acc, wr, wc, li, lk, t);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
      }
    }

    // epilogue in stage buffer 1 (buffer 0 may hold the next tile's first stage)
    double* red = smem + STAGE;
    const double* zb = a.z + b * a.zld + I * BI;
    double zr[4][4];
#pragma unroll
    for (int mi = 0; mi < 4; ++mi)
#pragma unroll
      for (int r = 0; r < 4; ++r) zr[mi][r] = zb[trmm_rtile(mi, wr) * 16 + lk + 4 * r];
#pragma unroll
    for (int nj = 0; nj < 4; ++nj) {
      double sm = 0.0, sv = 0.0;
#pragma unroll
      for (int mi = 0; mi < 4; ++mi)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const double v = acc[mi][nj][r];
          sm = fma(v, zr[mi][r], sm);
          sv = fma(v, v, sv);
        }
      sm += __shfl_xor(sm, 16, 64);
      sv += __shfl_xor(sv, 16, 64);
      sm += __shfl_xor(sm, 32, 64);
      sv += __shfl_xor(sv, 32, 64);
      if (lk == 0) {
        red[(wr * 2 + 0) * BC + wc * 64 + nj * 16 + li] = sm;
        red[(wr * 2 + 1) * BC + wc * 64 + nj * 16 + li] = sv;
      }
    }
    __syncthreads();
    if (tid < BC) {
      const int col = C * BC + tid;
      double* pm = part + ((long long)(b * 2 + 0) * NI + I) * mc;
      double* pv = part + ((long long)(b * 2 + 1) * NI + I) * mc;
      pm[col] = red[0 * BC + tid] + red[2 * BC + tid];
      pv[col] = red[1 * BC + tid] + red[3 * BC + tid];
    }
    __syncthreads();   // red (buffer 1) is read before the next tile's step 0 refills it
  }
}

// ------------------------------------------------------------------------------------------
// Column-resident prediction with the cross-covariance fused in, for npad <= 512 (C5's
// 512-point design, the fit's PC GPs).  At small n the pair kernel's 128 x 128 tiles spend 16
// of a block's 8 (NI + 1) K steps in diagonal blocks (16 of 40 at n = 512) whose stage loads
// and barriers cost a step each for 56% of a step's MFMAs, and its K* operand makes a round
// trip through HBM (the cross-covariance chunk written, then read by every row-tile pair).
// Here a panel is kResCols = 64 test points of one problem, and one block computes ALL npad
// rows of V = L^-1 K*^T for it:
//   * K*'s panel passes through a 2 RES_AHEAD-chunk LDS ring (6 chunks, 96 KB), produced 32
//     rows (a chunk) at a time, RES_AHEAD chunks ahead, by the block's own threads:
//     s exp(-sum (sqrt(beta)(x_k - x*_j))^2) with cross_kp_kernel's exact arithmetic (the same
//     Kt values bit for bit), one exp per element -- no cross-covariance kernel, no Kt slab in
//     HBM;
//   * L^-1 (1 MB lower triangle per problem at n = 512, L2-resident: panels are problem-major,
//     so the chip works through one problem's panels at a time) streams straight into
//     registers as MFMA A fragments by buffer loads (wave-uniform offset + four per-lane
//     offsets: no vector address arithmetic), one 16-k step ahead;
//   * 8 waves, wave w owning the 16-row tiles {w, 15 - w, 16 + w, 31 - w} (the first RT of
//     them: equal sums of (T + 1), i.e. equal MFMA work), all four 16-column MFMA tiles;
//   * tile T meets L^-1 at k-steps j <= T; activity is resolved per chunk (steps 2c, 2c + 1:
//     tile i takes part when T_i >= 2c, its step 2c + 1 then reading, when T_i = 2c, the zero
//     16 x 16 block above the diagonal -- zeroed by gp_potrf_inv / gp_trtri; the packed layout
//     does not store it, so those loads select 0).  T ascends with i, so the active tiles are
//     a suffix i >= F and the chunks split into segments of constant F, each its own
//     straight-line loop (no per-step branches, no accumulator copies);
//   * one block per panel (a persistent form that streamed a block's panels as one chunk
//     sequence, loading the next panel's inputs under the last chunks, measured no faster:
//     profiles/r06/r06ah_ab_res_persistent.log);
//   * one barrier per RES_AHEAD chunks, one more per panel for the epilogue, which reduces
//     sum V z and sum V^2 over the panel's rows and writes mean / var directly (no slab, no
//     finalize).
// Every global load is issued unconditionally (at a clamped in-bounds address when its value
// is not needed): the same number of loads on every path keeps the compiler's vmcnt waits
// counted, so prefetches stay in flight across the MFMAs.
// SLAB: K* read from a materialised cross-covariance chunk instead (gp_predict_solve after
// gp_predict_cross, and d > 8), RES_AHEAD chunks ahead through registers -- the same Kt
// values, so every entry point gives the same bits at npad <= 512.
// Sums run k ascending in every tile (the pair kernel runs some tiles diagonal-block first), so
// results equal the pair path to rounding, not bit for bit; they do not depend on the chunking.
#ifndef RES_COLS
#define RES_COLS 64
#endif
#ifndef RES_OCC
#define RES_OCC 2                              // waves per SIMD (launch bound)
#endif
constexpr int kResCols = RES_COLS;             // test points per panel
// RES_WIDE: 4 RT waves of two row tiles each (16 waves at npad = 512: 4 per SIMD); else 8
// waves of RT tiles
#ifndef RES_WIDE
#define RES_WIDE 0
#endif
// timing probes only (wrong results): 1 = no MFMAs, 2 = A fragments loaded once, 3 = no
// chunk barriers, 5 = no K* production in the chunks, 6 = neither production nor barriers
#ifndef RES_PROBE
#define RES_PROBE 0
#endif
#ifndef RES_XCD
#define RES_XCD 1
#endif
// RES_AHEAD = KA: K* produced KA chunks ahead into a 2 KA-slot LDS ring, design rows staged
// 2 KA chunks ahead, one barrier per KA chunks
#ifndef RES_AHEAD
#define RES_AHEAD 3
#endif
__host__ __device__ constexpr int res_waves(int RT) { return RES_WIDE ? 4 * RT : 8; }
constexpr int kResMaxWaves = 16;
constexpr int kResMaxPad = 512;
constexpr int kResD = 8;                       // design dimensions (d <= 8)

struct ResArgs {
  const double* Linv;      // padded (column k at k * ld) or tile-packed (linv_col, PACKED)
  long long sL;
  int ld;
  int n, d, mv, npanel;    // test points of this launch, ceil(mv / kResCols)
  int batch;
  const double* X;
  int ldx;
  const double* Xs;        // the launch's first test point
  int ldxs;
  const double* beta;
  int ldbeta;
  const double* s;
  const double* s_pred;
  const double* z;
  long long zld;
  double* mean;            // the launch's first test point's column
  double* var;
  int ldo;
  const double* kt;        // SLAB: the chunk's cross-covariance (row k of problem b at
  long long sK;            //   kt + b * sK + k * mc)
  int mc;
};

template <bool PACKED, int RT, bool SLAB>
__global__ __launch_bounds__(64 * res_waves(RT), RES_WIDE ? RT : RES_OCC) void trmm_res_kernel(
    const ResArgs a) {
  constexpr int NW = res_waves(RT);            // waves
  constexpr int kResThreads = 64 * NW;
  constexpr int TW = RT * 8 / NW;              // 16-row tiles per wave
  constexpr int NPAD = 128 * RT;
  constexpr int NCH = NPAD / 32;               // 32-row K* chunks per panel (even)
  constexpr int NJ = NPAD / 16;                // 16-k steps per panel
  constexpr int RING = 32 * kResD;             // one chunk's design rows
  constexpr int BCH = 32 * kResCols;           // one chunk of K*
  constexpr int NCT = kResCols / 16;           // 16-column MFMA tiles per panel
  constexpr int NPR = kResThreads / kResCols;  // K* rows one production pass covers
  constexpr int NH = (32 + NPR - 1) / NPR;     // production passes per chunk
  constexpr bool RAG = 32 % NPR != 0;          // (the last pass covers part of the chunk)
  constexpr int KA = RES_AHEAD;                // K* production distance (chunks)
  constexpr int KSL = 2 * KA;                  // K* ring slots
  // design-row staging distance: rows written at chunk c are read when chunk c + XA - KA
  // produces from them (needs XA >= 2 KA) and overwrite rows read at c + XA - 8 - KA (XA <= 8)
#ifdef RES_XA
  constexpr int XA = RES_XA;
#else
  constexpr int XA = 2 * KA;
#endif
  static_assert(XA >= 2 * KA && XA <= 8, "design-row ring has 8 slots");
  __shared__ __attribute__((aligned(16))) double Bs[KSL * BCH];   // K* chunks c .. c + KSL - 1
  __shared__ double tab[64];
  __shared__ double xring[9 * RING];           // design rows: chunk k in slot k & 7; scratch
  __shared__ double xsc[kResD * kResCols];     // sqrt(beta)-scaled test points, [dim][point]
  double* const red = Bs;                      // epilogue partial sums (K* ring is done)
  static_assert(NW * 2 * kResCols <= KSL * BCH, "epilogue sums alias the K* ring");
  __shared__ double zs[NPAD];
  // RES_XCD: the panels one XCD is dealt (blockIdx.x % 8 equal) are consecutive logical
  // panels, so a problem's L^-1 is fetched into one XCD's L2 instead of all eight
#if RES_XCD
  const int g = xcd_remap(blockIdx.x, gridDim.x);
#else
  const int g = blockIdx.x;
#endif
  const int b = g / a.npanel, P = g - b * a.npanel;
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int li = lane & 15, lk = lane >> 4;
  const int pc = tid & (kResCols - 1), rp = tid / kResCols;   // K* production: column, row
  const int xrow = tid >> 3, xd = tid & (kResD - 1);          // ring fill: design row, dim
  int T[TW];                                   // snake: equal sums of (T + 1) per wave
#pragma unroll
  for (int i = 0; i < TW; ++i) T[i] = (i & 1) ? NW * i + NW - 1 - w : NW * i + w;
  int voff[4];                                 // lane (li, lk): row li, column 4 q + lk
#pragma unroll
  for (int q = 0; q < 4; ++q) voff[q] = ((4 * q + lk) * a.ld + li) * 8;
  // raw inputs are loaded at clamped in-bounds indices and masked where they are stored
  const double bq = (!SLAB && xd < a.d)        // sqrt(beta[b][xd]), 0 past d
                        ? __builtin_sqrt(a.beta[(long long)b * a.ldbeta + xd]) : 0.0;
  auto xval = [&](int c) {                     // design row 32 c + xrow, dimension xd
    const int k = 32 * c + xrow;
    return a.X[(long long)(k < a.n ? k : a.n - 1) * a.ldx + (xd < a.d ? xd : 0)];
  };
  auto xscale = [&](int c, double v) {         // cross_kp's xk
    return (32 * c + xrow < a.n && xd < a.d) ? v * bq : 0.0;
  };
  const double* ktc = a.kt + b * a.sK + P * kResCols + pc;    // SLAB: column pc's chunk
  auto kval = [&](int c, int h) {
    const int r = rp + NPR * h;
    return ktc[(long long)(32 * c + (RAG && r >= 32 ? 31 : r)) * a.mc];
  };
  // K* chunk c in slot c & 1; row r's 64 doubles with the 16-column halves of each 32-column
  // group swapped in odd rows: the 16-lane groups of a B fragment read (rows k .. k+3) then
  // cover all 64 banks twice, conflict-free
  auto bslot = [&](int c, int h) {
    const int r = rp + NPR * h;
    return Bs + (c % KSL) * BCH + r * kResCols + (pc ^ (16 * (r & 1)));
  };
  const double sb = SLAB ? 0.0 : a.s[b];
  const bool col_ok = P * kResCols + pc < a.mv;
  // element h of chunk c of K*, from design-row slot `slot`
  auto produce_one = [&](int c, int slot, int h) {
    const int r = rp + NPR * h, k = 32 * c + r;
    if (RAG && r >= 32) return;
    const double* xc = xsc + pc;               // [dim][point]: consecutive lanes, banks
    const double* xk = xring + slot * RING + r * kResD;
    double e = 0.0;
#pragma unroll
    for (int dd = 0; dd < kResD; ++dd) {
      const double t = xk[dd] - xc[dd * kResCols];
      e = fma(t, t, e);
    }
    const double v = sb * exp_neg_tab(e, tab);
    *bslot(c, h) = (col_ok && k < a.n) ? v : 0.0;
  };
  auto produce = [&](int c, int slot) {
#pragma unroll
    for (int h = 0; h < NH; ++h) produce_one(c, slot, h);
  };

  // ---- L^-1 fragments (buffer loads: wave-uniform offset + per-lane voff)
  const __amdgpu_buffer_rsrc_t lrs = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<double*>(a.Linv + b * a.sL), 0, 0x7fffffff, 0x00020000);
  auto frag = [&](int i, int je, int q) -> double {
    if (PACKED) {
      const int k = 16 * je + 4 * q + lk;
      return (T[i] >= je) ? a.Linv[b * a.sL + linv_col(k, NPAD) + 16 * T[i] + li] : 0.0;
    }
    const auto v = __builtin_amdgcn_raw_buffer_load_b64(lrs, voff[q],
                                                        (16 * je * a.ld + 16 * T[i]) * 8, 0);
    return __longlong_as_double(((long long)v[1] << 32) | v[0]);
  };
  double av[TW][4];
  f64x4 acc[TW][NCT];
#pragma unroll
  for (int i = 0; i < TW; ++i)
#pragma unroll
    for (int ct = 0; ct < NCT; ++ct) acc[i][ct] = zero4();
  const int sw = 16 * (lk & 1);
  // step j's MFMAs for tiles F .. RT-1; each fragment, once used, is reloaded with step
  // j + 1's (one register set: the reload of substep q runs under substeps q + 1 .. 3 and the
  // next step's first substeps)
  auto mstep = [&](auto F, int j) {
    if constexpr (decltype(F)::value < TW) {
      const int jn = (j + 1 < NJ) ? j + 1 : NJ - 1;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const double* br = Bs + ((j >> 1) % KSL) * BCH + ((j & 1) * 16 + 4 * q + lk) * kResCols;
        double bv[NCT];
#pragma unroll
        for (int ct = 0; ct < NCT; ++ct) bv[ct] = br[(16 * ct + li) ^ sw];
        static_for<decltype(F)::value, TW, 1>([&](auto I) {
#if RES_PROBE != 1
#pragma unroll
          for (int ct = 0; ct < NCT; ++ct) acc[I][ct] = mfma16x16x4(av[I][q], bv[ct], acc[I][ct]);
#else
#pragma unroll
          for (int ct = 0; ct < NCT; ++ct) acc[I][ct][0] += av[I][q] * bv[ct];
#endif
#if RES_PROBE != 2
          av[I][q] = frag(I, jn, q);
#endif
        });
      }
    }
  };

  // ---- prologue: test points, z, design rows of chunks 0 .. XA - 1, K* chunks 0 .. KA - 1, A(0)
  {
    const double zv = a.z[b * a.zld + (tid < NPAD ? tid : 0)];
    if (SLAB) {
#pragma unroll
      for (int c = 0; c < KA; ++c)
#pragma unroll
        for (int h = 0; h < NH; ++h)
          if (c < NCH && (!RAG || rp + NPR * h < 32)) *bslot(c, h) = kval(c, h);
    } else {
      if (tid < 64) tab[tid] = kExp2Tab[tid];
      double xs[kResCols / 32];                // test points xrow + 32 h, dimension xd
#pragma unroll
      for (int h = 0; h < kResCols / 32; ++h) {
        const int c_ = P * kResCols + xrow + 32 * h;
        xs[h] = a.Xs[(long long)(c_ < a.mv ? c_ : a.mv - 1) * a.ldxs + (xd < a.d ? xd : 0)];
      }
      double x4[XA];
#pragma unroll
      for (int c = 0; c < XA; ++c) x4[c] = xval(c < NCH ? c : NCH - 1);
      if (tid < RING) {
#pragma unroll
        for (int h = 0; h < kResCols / 32; ++h)
          xsc[xd * kResCols + 32 * h + xrow] =
              (P * kResCols + xrow + 32 * h < a.mv && xd < a.d) ? xs[h] * bq : 0.0;
#pragma unroll
        for (int c = 0; c < XA; ++c) xring[c * RING + tid] = xscale(c, x4[c]);
      }
    }
    if (tid < NPAD) zs[tid] = zv;
#pragma unroll
    for (int i = 0; i < TW; ++i)
#pragma unroll
      for (int q = 0; q < 4; ++q) av[i][q] = frag(i, 0, q);
    __syncthreads();
    if (!SLAB) {
#pragma unroll
      for (int c = 0; c < KA; ++c)
        if (c < NCH) produce(c, c);
    }
    __syncthreads();
  }

  // ---- chunks: K* chunk c + KA (produced now; SLAB: loaded now, stored after the MFMAs) into
  // the slot chunk c - KA used, design rows of chunk c + 2 KA into slot (c + 2 KA) & 7 (read
  // when chunk c + KA produces from them; the rows it overwrites were read at chunk c + 2 KA -
  // 8 - KA <= c - KA), MFMAs of steps 2c and 2c + 1, and a barrier after chunks c = KA - 1
  // mod KA only: whatever chunk c writes is read from chunk c + KA on, and what it overwrites
  // was last read at chunk c - KA, so one barrier always lies between (a barrier per chunk cost
  // 6.5%: r06af, no-barrier probe).
  // Tile i takes part in chunk c when T_i >= 2c (its step 2c + 1 then reads,
  // when T_i = 2c, the zero 16 x 16 block above the diagonal -- zeroed by gp_potrf_inv /
  // gp_trtri; the packed layout does not store it, so those loads select 0).  T ascends with
  // i, so the active tiles are a suffix i >= F: the chunks split into segments of constant F,
  // each its own straight-line loop.
  auto chunk = [&](auto F, int c) {
    // (past the end: a harmless refill of the last chunk's slot with its own values)
    const int cf = (c + XA < NCH) ? c + XA : NCH - 1;
    double xn = 0.0, kn[NH];
    if (SLAB) {
      const int cn = (c + KA < NCH) ? c + KA : NCH - 1;
#pragma unroll
      for (int h = 0; h < NH; ++h) kn[h] = kval(cn, h);
    } else {
      xn = xval(cf);
    }
#if RES_PROBE != 5 && RES_PROBE != 6
    if (!SLAB && c + KA < NCH) produce(c + KA, (c + KA) & 7);
#endif
    mstep(F, 2 * c);
    mstep(F, 2 * c + 1);
    if (SLAB) {
      if (c + KA < NCH) {
#pragma unroll
        for (int h = 0; h < NH; ++h)
          if (!RAG || rp + NPR * h < 32) *bslot(c + KA, h) = kn[h];
      }
    } else {
      xring[(tid < RING ? (cf & 7) : 8) * RING + (tid & (RING - 1))] = xscale(cf, xn);
    }
#if RES_PROBE != 3 && RES_PROBE != 6
    if (c % KA == KA - 1) __syncthreads();
#endif
  };
  int c = 0;
  static_for<0, TW + 1, 1>([&](auto F) {
    constexpr int f = decltype(F)::value;
    int cend = (f < TW) ? T[f < TW ? f : 0] / 2 + 1 : NCH;   // chunks with T_f >= 2c
    if (cend > NCH) cend = NCH;
#pragma unroll 1
    for (; c < cend; ++c) chunk(F, c);
  });

  // ---- epilogue: per column sum V z and sum V^2 over the wave's rows (C layout: lane l, reg
  // r holds row 16 T + (l >> 4) + 4 r, column l & 15), then over the 8 waves in a fixed order
  double smv[NCT], svv[NCT];
#pragma unroll
  for (int ct = 0; ct < NCT; ++ct) {
    double sm = 0.0, sv = 0.0;
#pragma unroll
    for (int i = 0; i < TW; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const double v = acc[i][ct][r];
        sm = fma(v, zs[16 * T[i] + lk + 4 * r], sm);
        sv = fma(v, v, sv);
      }
    sm += __shfl_xor(sm, 16, 64);
    sv += __shfl_xor(sv, 16, 64);
    sm += __shfl_xor(sm, 32, 64);
    sv += __shfl_xor(sv, 32, 64);
    smv[ct] = sm;
    svv[ct] = sv;
  }
  // red overwrites the K* ring: every wave has finished its last chunk's reads (the last chunk
  // ends with a barrier only when NCH - 1 = KA - 1 mod KA)
  if ((NCH - 1) % KA != KA - 1) __syncthreads();
  if (lk == 0) {
#pragma unroll
    for (int ct = 0; ct < NCT; ++ct) {
      red[(w * 2 + 0) * kResCols + ct * 16 + li] = smv[ct];
      red[(w * 2 + 1) * kResCols + ct * 16 + li] = svv[ct];
    }
  }
  __syncthreads();
  if (tid < kResCols) {
    double sm = 0.0, sv = 0.0;
#pragma unroll
    for (int v = 0; v < NW; ++v) {
      sm += red[(v * 2 + 0) * kResCols + tid];
      sv += red[(v * 2 + 1) * kResCols + tid];
    }
    const int cg = P * kResCols + tid;
    if (cg < a.mv) {
      a.mean[(long long)b * a.ldo + cg] = sm;
      a.var[(long long)b * a.ldo + cg] = a.s_pred[b] - sv;
    }
  }
}

// mean / var of test points [j0, j0 + mv): column j's partial sums sit in the slab of chunk
// j / mc, counted from j0's chunk (slabs pslab doubles apart after `part`; pslab = 0 when every
// chunk reuses one slab).
__global__ __launch_bounds__(256) void finalize_kernel(const double* __restrict__ part, int NI,
                                                       int mc, long long pslab, int j0, int mv,
                                                       const double* __restrict__ s_pred,
                                                       double* __restrict__ mean,
                                                       double* __restrict__ var, int ldo) {
  const int b = blockIdx.y;
  const int jl = blockIdx.x * 256 + threadIdx.x;
  if (jl >= mv) return;
  const int j = j0 + jl, ch = j / mc, jj = j - ch * mc, chr = ch - j0 / mc;
  const double* pm = part + chr * pslab + (long long)(b * 2 + 0) * NI * mc + jj;
  const double* pv = part + chr * pslab + (long long)(b * 2 + 1) * NI * mc + jj;
  double sm = 0.0, sv = 0.0;
#pragma unroll 8
  for (int I = 0; I < NI; ++I) {
    sm += pm[(long long)I * mc];
    sv += pv[(long long)I * mc];
  }
  mean[(long long)b * ldo + j] = sm;
  var[(long long)b * ldo + j] = s_pred[b] - sv;
}

template <int D>
hipError_t cross_kp_launch_d(const double* X, int n, int ldx, const double* Xs, int mv,
                             int ldxs, int d, const double* beta, int ldbeta, const double* s,
                             double* Kt2, int mc, int npad, long long sK, int batch,
                             hipStream_t st) {
  // only the columns the chunk's TRMM reads (its ceil(mv / BC) column tiles; zeros past mv):
  // the 1696-point tail chunk of C3 no longer computes all 16384 columns (14.7% of a step's
  // cross-covariance work)
  const int cols = min(mc, gp_ceil_div(mv, BC) * BC);
  dim3 grid(gp_ceil_div(cols, 256), npad / 64, batch);
  hipLaunchKernelGGL((cross_kp_kernel<D>), grid, dim3(256), 0, st, X, n, ldx, Xs, mv, ldxs, d,
                     beta, ldbeta, s, Kt2, mc, sK);
  return hipGetLastError();
}

hipError_t cross_kp_launch(const double* X, int n, int ldx, const double* Xs, int mv, int ldxs,
                           int d, const double* beta, int ldbeta, const double* s, double* Kt2,
                           int mc, int npad, long long sK, int batch, hipStream_t st) {
  if (d <= 8)
    return cross_kp_launch_d<8>(X, n, ldx, Xs, mv, ldxs, d, beta, ldbeta, s, Kt2, mc, npad, sK,
                                batch, st);
  if (d <= 16)
    return cross_kp_launch_d<16>(X, n, ldx, Xs, mv, ldxs, d, beta, ldbeta, s, Kt2, mc, npad, sK,
                                 batch, st);
  return cross_kp_launch_d<32>(X, n, ldx, Xs, mv, ldxs, d, beta, ldbeta, s, Kt2, mc, npad, sK,
                               batch, st);
}

// z = L^-1 w for the prediction in two deterministic passes (the same arithmetic whatever the
// chunking, so results stay bit-identical across m_chunk).  z sits between the factorisation
// and the first TRMM, on the critical path of every step.  Round 4's form (64-row blocks x
// 128-column tiles, 32 loads of 512 B per wave at a 32 KB column stride) read the 71 MB
// triangle in 95 us alone, 140 us beside the cross-covariance (0.06 of HBM,
// profiles/r04/r04k_timeline.txt).  Here every load instruction of a block reads 4 KB of one
// column:
//   pass 1: block (rb, s) forms row block rb's kZR rows (2 per thread, one 16-B load per
//           column) times column strip s (kZS columns; strips right of the row block are zero
//           and skipped: 288 blocks at n = 4096), k ascending, into zp[s][r];
//   pass 2: z[r] = the sum over s = 0 .. last strip of r's row block of zp[s][r], as eight
//           in-order runs of strips combined in a fixed tree (trmv_sum_kernel).
// Every row r < npad is written (rows >= n are 0: L^-1 is zero-padded).  zp (batch *
// ceil(npad / kZS) * npad doubles, 2 MB per problem at n = 4096) is its own workspace region.
constexpr int kZR = 512;   // rows per pass-1 block
constexpr int kZS = 64;    // columns per strip

template <bool PACKED>
__global__ __launch_bounds__(256) void trmv_part_kernel(const double* __restrict__ Linv, int ld,
                                                        long long sL,
                                                        const double* __restrict__ w, int ldw,
                                                        double* __restrict__ zp, int npad,
                                                        int n) {
  const int b = blockIdx.z, rb = blockIdx.x * kZR, k0 = blockIdx.y * kZS;
  if (k0 > rb + kZR - 1 || k0 >= n) return;       // right of the row block: pass 2 skips it
  const int r = rb + 2 * threadIdx.x;
  if (r >= npad) return;                           // npad is even: both rows or neither
  const double* L = Linv + b * sL + r;
  const double* wb = w + (long long)b * ldw;
  const int ke = min(k0 + kZS, n);
  double a0 = 0.0, a1 = 0.0;
#pragma unroll 1
  for (int kb = k0; kb < ke; kb += 16) {
    // 16 columns' loads in flight before the first FMA
    double2 lv[16];
    double wk[16];
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      const int k = kb + j;
      // tile-packed: rows below column k's first stored tile are zero in L^-1 (the padded
      // layout's fma(0, w, acc) leaves acc unchanged, so skipping them changes no bit)
      const bool ok = k < ke && (!PACKED || r >= ((k >> 4) << 4));
      lv[j] = ok ? *reinterpret_cast<const double2*>(
                       L + (PACKED ? linv_col(k, npad) : (long long)k * ld))
                 : make_double2(0.0, 0.0);
      wk[j] = k < ke ? wb[k] : 0.0;
    }
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      a0 = fma(lv[j].x, wk[j], a0);
      a1 = fma(lv[j].y, wk[j], a1);
    }
  }
  *reinterpret_cast<double2*>(zp + ((long long)b * gridDim.y + blockIdx.y) * npad + r) =
      make_double2(a0, a1);
}

// Pass 2: 32 rows per block, 8 threads per row, thread g summing its row's strips
// g * per .. (g + 1) * per - 1 in order, the 8 partials combined in a fixed tree (one thread per
// row summing all 64 strips serially took 23 us at n = 4096, this 6 us:
// tools/dbg/trmv_micro.hip, profiles/r05/r05b_trmv_micro.log).
__global__ __launch_bounds__(256) void trmv_sum_kernel(const double* __restrict__ zp, int nst,
                                                       int npad, int n, double* __restrict__ z,
                                                       long long ldz) {
  __shared__ double red[8][32];
  const int b = blockIdx.y, rl = threadIdx.x & 31, g = threadIdx.x >> 5;
  const int r = blockIdx.x * 32 + rl;
  double acc = 0.0;
  if (r < npad) {
    const int rb = (r / kZR) * kZR;
    const int cnt = min(rb + kZR - 1, n - 1) / kZS + 1;   // pass 1's strips for r's row block
    const int per = (cnt + 7) / 8;
    const int s0 = g * per, s1 = min(cnt, s0 + per);
    const double* q = zp + (long long)b * nst * npad + r;
    for (int s = s0; s < s1; ++s) acc += q[(long long)s * npad];
  }
  red[g][rl] = acc;
  __syncthreads();
  if (g == 0 && r < npad)
    z[(long long)b * ldz + r] = ((red[0][rl] + red[1][rl]) + (red[2][rl] + red[3][rl])) +
                                ((red[4][rl] + red[5][rl]) + (red[6][rl] + red[7][rl]));
}

struct Plan {
  int npad, NI, mc, NC, nchunks, slabs;
  long long off_z, off_zp, off_kt, off_part, off_pot, bytes, slab_elems, part_elems;
};

// slabs = 1 (2 with a partial last chunk): one cross-covariance chunk and one partial-sum slab
// at a time (gp_predict, which finalises each chunk after its TRMM); slabs = nchunks: every
// chunk's cross-covariance and
// partial sums materialised (gp_predict_cross + gp_predict_solve, gp_fit_predict), so one
// finalize launch after the last TRMM covers all m points.  `potrf`: plus the factorisation's
// scratch (gp_fit_predict).
Plan make_plan(int n, int m, int batch, int m_chunk, bool all_slabs = false,
               bool potrf = false) {
  Plan p;
  p.npad = gp_padded_n(n);
  p.NI = p.npad / BI;
  const int mpad = gp_ceil_div(m, BC) * BC;
  int mc;
  if (m_chunk > 0) {
    mc = gp_ceil_div(m_chunk, BC) * BC;
  } else {
    // Test points per chunk: 8192 for batches (C4: 64 panels per GP, so the TRMM's XCD-aware
    // order applies; 60.2-62.1 vs 62.6-63.0 ms per step at 4096 in three same-box rounds,
    // profiles/r03/sweep_c4_chunk_r03.log -- round 1 had measured 4096 best with the plain
    // order) and 16384 for one GP (C3 with the row-pair TRMM: a launch is then 2048 blocks, four full
    // residency waves; 28.51-28.59 vs 28.72-28.81 ms per step at 4096, 32768 slower:
    // profiles/r01/sweep_c3_chunk_pair.log).  Shrunk only when the batch's cross-covariance
    // slab would exceed kDefaultChunkElems doubles.
    long long cap = kDefaultChunkElems / ((long long)p.npad * (batch > 0 ? batch : 1));
    mc = (int)((cap / BC) * BC);
    const int def = batch == 1 ? kDefaultChunkSingle : kDefaultChunk;
    if (mc > def) mc = def;
    if (mc < BC) mc = BC;
  }
  if (mc > mpad) mc = mpad;
  if (mc < BC) mc = BC;
  p.mc = mc;
  p.NC = mc / BC;
  p.nchunks = gp_ceil_div(m, mc);
  // gp_predict with a partial last chunk: two slabs, so that chunk's TRMM can run merged with
  // the chunk before it (trmm_merge_last)
  p.slabs = all_slabs ? p.nchunks : (p.nchunks >= 2 && m % mc != 0) ? 2 : 1;
  p.slab_elems = (long long)batch * mc * p.npad;
  long long z = (long long)batch * p.npad;
  long long zp = (long long)batch * gp_ceil_div(p.npad, kZS) * p.npad;   // trmv partials
  long long kt = p.slab_elems * p.slabs;
  p.part_elems = (long long)batch * 2 * p.NI * mc;
  const long long part = p.part_elems * p.slabs;
  p.off_z = 0;
  p.off_zp = ((z * 8 + 255) / 256) * 256;
  p.off_kt = p.off_zp + ((zp * 8 + 255) / 256) * 256;
  p.off_part = p.off_kt + ((kt * 8 + 255) / 256) * 256;
  p.off_pot = ((p.off_part + part * 8 + 255) / 256) * 256;
  p.bytes = p.off_pot + (potrf ? gpfit_potrf_inv_ws_bytes(n, batch) : 0);
  return p;
}

}  // namespace

extern "C" long long gp_predict_ws_bytes(int n, int m, int batch, int m_chunk) {
  if (n <= 0 || m <= 0 || batch <= 0) return 0;
  return make_plan(n, m, batch, m_chunk).bytes;
}

extern "C" long long gp_predict_prepared_ws_bytes(int n, int m, int batch, int m_chunk) {
  if (n <= 0 || m <= 0 || batch <= 0) return 0;
  return make_plan(n, m, batch, m_chunk, true).bytes;
}

extern "C" long long gp_fit_predict_ws_bytes(int n, int m, int batch, int m_chunk) {
  if (n <= 0 || m <= 0 || batch <= 0) return 0;
  return make_plan(n, m, batch, m_chunk, true, true).bytes;
}

namespace {

int check_common(const double* X, int ldx, const double* Xs, int ldxs, int n, int m, int d,
                 const double* beta, int ldbeta, const double* s, int batch) {
  if (!X) return -4;
  if (ldx < d) return -5;
  if (!Xs) return -6;
  if (ldxs < d) return -7;
  if (n < 0) return -8;
  if (m < 0) return -9;
  if (d < 1 || d > GPFIT_MAX_DIM) return -10;
  if (!beta) return -11;
  if (ldbeta < d && batch > 1) return -12;
  if (!s) return -13;
  if (batch < 0) return -20;
  return 0;
}

int check_solve(const double* Linv, int ldinv, long long strideInv, int n, const double* s_pred,
                const double* w_hat, int ldw, int m, double* mean, double* var, int ldo,
                int batch, bool packed = false) {
  if (!Linv || (reinterpret_cast<uintptr_t>(Linv) & 15)) return -1;
  const int npad = gp_padded_n(n);
  if (!packed && (ldinv < npad || ldinv < 1 || (ldinv & 1))) return -2;   // 16-B double2 loads
  const long long per = packed ? linv_packed_elems(npad) : (long long)ldinv * npad;
  if ((batch > 1 && strideInv < per) || (strideInv & 1)) return -3;
  if (!s_pred) return -14;
  if (!w_hat) return -15;
  if (ldw < n && batch > 1) return -16;
  if (!mean) return -17;
  if (!var) return -18;
  if (ldo < m && batch > 1) return -19;
  return 0;
}

struct WS {
  double *z, *zp, *kt, *part;
  char* pot;
};

WS carve(const Plan& p, void* ws) {
  char* base = static_cast<char*>(ws);
  return {reinterpret_cast<double*>(base + p.off_z), reinterpret_cast<double*>(base + p.off_zp),
          reinterpret_cast<double*>(base + p.off_kt), reinterpret_cast<double*>(base + p.off_part),
          base + p.off_pot};
}

// L^-1 as the prediction reads it: the padded buffer (column k at k * ld) or the tile-packed
// vector (linv_col); `stride` doubles from one problem to the next.
struct LinvRef {
  const double* p;
  int ld;
  long long stride;
  bool packed;
};

// z = L^-1 w into z (npad rows per problem, problem stride zld), two passes through zp (the same
// arithmetic whatever the chunking and the layout, so results stay bit-identical).
hipError_t trmv_pred(int npad, double* zp, const LinvRef& L, const double* w_hat, int ldw,
                     int n, int batch, double* z, long long zld, hipStream_t stream) {
  const int nst = gp_ceil_div(npad, kZS);
  const dim3 grid(gp_ceil_div(npad, kZR), nst, batch);
  if (L.packed)
    hipLaunchKernelGGL(trmv_part_kernel<true>, grid, dim3(256), 0, stream, L.p, L.ld, L.stride,
                       w_hat, ldw, zp, npad, n);
  else
    hipLaunchKernelGGL(trmv_part_kernel<false>, grid, dim3(256), 0, stream, L.p, L.ld, L.stride,
                       w_hat, ldw, zp, npad, n);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(trmv_sum_kernel, dim3(gp_ceil_div(npad, 32), batch), dim3(256), 0,
                     stream, zp, nst, npad, n, z, zld);
  return hipGetLastError();
}

hipError_t cross_chunk(const Plan& p, int ch, double* kt, const double* X, int ldx,
                       const double* Xs, int ldxs, int n, int m, int d, const double* beta,
                       int ldbeta, const double* s, int batch, hipStream_t stream) {
  const int c0 = ch * p.mc;
  const int mv = (m - c0 < p.mc) ? (m - c0) : p.mc;
  return cross_kp_launch(X, n, ldx, Xs + (long long)c0 * ldxs, mv, ldxs, d, beta, ldbeta, s, kt,
                         p.mc, p.npad, (long long)p.mc * p.npad, batch, stream);
}

// Residency slots of trmm_pair_kernel on the current device (CUs x blocks per CU), cached.
int trmm_slots() {
  static std::atomic<int> cache[64];
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) dev = 0;
  int v = cache[dev].load(std::memory_order_relaxed);
  if (v > 0) return v;
  int ncu = 0, nb = 0;
  if (hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
      ncu < 1)
    ncu = 256;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, trmm_pair_kernel<false>, 256, 0) !=
          hipSuccess ||
      nb < 1)
    nb = 2;
  v = ncu * nb;
  cache[dev].store(v, std::memory_order_relaxed);
  return v;
}

// The schedule of one launch over G = batch * NCt panels (T = G * NP pair blocks, S slots).
// Whole residency rounds of uniform pair blocks finish together; a partial last round would
// leave CUs idle for a whole pair block's time (C3's 1696-point tail: 224 blocks for 512
// slots, 0.535 ms against 0.414 at the full rate; a rank's 13,408 points at 8 ranks: 3.28
// rounds, the last 0.28 taking a full block's time).  So when T is not a multiple of S, the
// panels of the last round and one full round before it run as single-tile blocks, longest
// first: S blocks start on the longest tiles and every slot that frees takes the next, so the
// launch ends within about one short tile of T / S pair-block times.
void trmm_sched(TrmmArgs& a, int batch, int slots) {
  const int NP = (a.NI + 1) / 2;
  const long long G = (long long)batch * a.NCt;
  const long long T = G * NP;
  long long Gp = G;
  if (slots > 0 && T % slots != 0) {
    const long long full = T / slots;
    Gp = (full > 0 ? full - 1 : 0) * slots / NP;
  }
  a.Gp = (int)Gp;
  a.Qc = (int)(G - Gp);
  const int grp = 8 * kXcdPanels;
  a.Gx = grp > 0 ? (a.Gp / grp) * grp : 0;
  // XCD-local units for batches: every (problem, pair) unit spans whole launches' panels, and
  // the units split evenly over the 8 XCD slots
  a.umap = (TRMM_UNIT_MAP && batch > 1 && Gp == G && ((long long)batch * NP) % 8 == 0) ? 1 : 0;
}

// The last chunk's TRMM runs merged with the one before it when its blocks fill less than one
// residency round (the merged launch's schedule then packs that round with the previous
// chunk's panels).
bool trmm_merge_last(const Plan& p, int m, int batch) {
  if (p.nchunks < 2 || m % p.mc == 0) return false;
  const long long tail_panels = gp_ceil_div(m - (p.nchunks - 1) * p.mc, BC);
  return (long long)batch * tail_panels * ((p.NI + 1) / 2) < trmm_slots();
}

// TRMM of chunks ch0 .. ch1 (consecutive; each chunk's cross-covariance `slab` doubles after the
// one before, its partial sums `pslab` after) in one launch.
hipError_t trmm_launch(const Plan& p, int ch0, int ch1, const double* kt, long long slab,
                       double* part, long long pslab, const double* z, long long zld,
                       const LinvRef& L, int m, int batch, hipStream_t stream) {
  const int c1 = ch1 * p.mc;
  const int mv1 = (m - c1 < p.mc) ? (m - c1) : p.mc;
  TrmmArgs a;
  a.Linv = L.p;
  a.sL = L.stride;
  a.Kt2 = kt;
  a.sK = (long long)p.mc * p.npad;
  a.slab = slab;
  a.z = z;
  a.zld = zld;
  a.part = part;
  a.pslab = pslab;
  a.ld = L.ld;
  a.mc = p.mc;
  a.NCc = p.NC;
  a.NCt = (ch1 - ch0) * p.NC + gp_ceil_div(mv1, BC);
  a.npad = p.npad;
  a.NI = p.NI;
  trmm_sched(a, batch, trmm_slots());
  const long long blocks = (long long)a.Gp * ((p.NI + 1) / 2) + (long long)a.Qc * p.NI;
  if (L.packed)
    hipLaunchKernelGGL(trmm_pair_kernel<true>, dim3((unsigned)blocks), dim3(256), 0, stream, a);
  else
    hipLaunchKernelGGL(trmm_pair_kernel<false>, dim3((unsigned)blocks), dim3(256), 0, stream, a);
  return hipGetLastError();
}

// The column-resident kernel (trmm_res_kernel) serves every npad <= 512 prediction, with the
// cross-covariance fused in when d <= 8 (res_fused) and from a materialised chunk otherwise.
// gp_set_predict_path (A/B hook): 1 forces the cross-covariance + pair-TRMM path, 2 the
// column-resident kernel from materialised chunks for every d.
std::atomic<int> g_predict_path{0};
bool res_eligible(int npad) {
  return g_predict_path.load(std::memory_order_relaxed) != 1 && npad <= kResMaxPad;
}
bool res_fused(int d) { return g_predict_path.load(std::memory_order_relaxed) != 2 && d <= kResD; }

// mean / var of test points [j0, j0 + mv) of every problem in one launch (problem-major blocks).
hipError_t res_launch(int npad, const LinvRef& L, int n, int d, const double* X, int ldx,
                      const double* Xs, int ldxs, int j0, int mv, const double* beta,
                      int ldbeta, const double* s, const double* s_pred, const double* z,
                      long long zld, double* mean, double* var, int ldo, int batch,
                      const double* kt, long long sK, int mc, hipStream_t st) {
  ResArgs a;
  a.Linv = L.p;
  a.sL = L.stride;
  a.ld = L.ld;
  a.n = n;
  a.d = d;
  a.mv = mv;
  a.npanel = gp_ceil_div(mv, kResCols);
  a.batch = batch;
  a.X = X;
  a.ldx = ldx;
  a.Xs = Xs + (long long)j0 * ldxs;
  a.ldxs = ldxs;
  a.beta = beta;
  a.ldbeta = ldbeta;
  a.s = s;
  a.s_pred = s_pred;
  a.z = z;
  a.zld = zld;
  a.mean = mean + j0;
  a.var = var + j0;
  a.ldo = ldo;
  a.kt = kt;
  a.sK = sK;
  a.mc = mc;
  const long long total = (long long)batch * a.npanel;
#define GP_RES_K(PK, RT, SL)                                                               \
  hipLaunchKernelGGL((trmm_res_kernel<PK, RT, SL>), dim3((unsigned)total),                  \
                     dim3(64 * res_waves(RT)), \
                     0, st, a)
#define GP_RES(RT)                                                            \
  do {                                                                        \
    if (kt) {                                                                 \
      if (L.packed) GP_RES_K(true, RT, true); else GP_RES_K(false, RT, true); \
    } else {                                                                  \
      if (L.packed) GP_RES_K(true, RT, false); else GP_RES_K(false, RT, false); \
    }                                                                         \
  } while (0)
  switch (npad / 128) {
    case 1: GP_RES(1); break;
    case 2: GP_RES(2); break;
    case 3: GP_RES(3); break;
    case 4: GP_RES(4); break;
    default: return hipErrorInvalidValue;
  }
#undef GP_RES
#undef GP_RES_K
  return hipGetLastError();
}

// trmm_res_kernel over all m test points, one launch per plan chunk (another stream's kernels
// can interleave between launches, as with the TRMM chunks).  K* source: fused (d <= 8), the
// prepared slabs of gp_predict_cross, or each chunk's cross-covariance built into slab 0 just
// before its launch.
enum class ResSrc { Fused, Prepared, Serial };

hipError_t res_all(const Plan& p, const WS& w, ResSrc src, const LinvRef& L, int n, int m, int d,
                   const double* X, int ldx, const double* Xs, int ldxs, const double* beta,
                   int ldbeta, const double* s, const double* s_pred, const double* z,
                   long long zld, double* mean, double* var, int ldo, int batch,
                   hipStream_t st) {
  const bool one = src != ResSrc::Serial;    // one timing pair around all launches
  if (one) gpfit_prof_begin_n(GP_PROF_TRMM, st, p.nchunks);
  for (int ch = 0; ch < p.nchunks; ++ch) {
    const int j0 = ch * p.mc;
    const int mv = (m - j0 < p.mc) ? (m - j0) : p.mc;
    const double* kt = nullptr;
    hipError_t e;
    if (src == ResSrc::Prepared) {
      kt = w.kt + (long long)ch * p.slab_elems;
    } else if (src == ResSrc::Serial) {
      gpfit_prof_begin(GP_PROF_CROSS, st);
      if ((e = cross_chunk(p, ch, w.kt, X, ldx, Xs, ldxs, n, m, d, beta, ldbeta, s, batch,
                           st)) != hipSuccess)
        return e;
      gpfit_prof_end(GP_PROF_CROSS, st);
      kt = w.kt;
    }
    if (!one) gpfit_prof_begin(GP_PROF_TRMM, st);
    e = res_launch(p.npad, L, n, d, X, ldx, Xs, ldxs, j0, mv, beta, ldbeta, s, s_pred, z, zld,
                   mean, var, ldo, batch, kt, (long long)p.mc * p.npad, p.mc, st);
    if (e != hipSuccess) return e;
    if (!one) gpfit_prof_end(GP_PROF_TRMM, st);
  }
  if (one) gpfit_prof_end(GP_PROF_TRMM, st);
  return hipSuccess;
}

// Every chunk's TRMM into its own slab, then one finalize over all m points.  With `ready`
// (gp_fit_predict on a context), chunk ch's TRMM first waits for ready[ch], the event after
// that chunk's cross-covariance on the aux stream.
// Chunks from `late` on (gp_fit_predict with gp_ctx_set_aux_chunks) have no cross-covariance
// yet: `cross(ch)` enqueues it on `stream` just before that chunk's TRMM.
template <typename Cross>
hipError_t solve_all(const Plan& p, const WS& w, const LinvRef& L, const double* z,
                     long long zld, int m, const double* s_pred, double* mean, double* var,
                     int ldo, int batch, hipStream_t stream, const hipEvent_t* ready, int late,
                     Cross&& cross) {
  hipError_t e;
  if (ready && late > 0 && (e = hipStreamWaitEvent(stream, ready[0], 0)) != hipSuccess) return e;
  const bool merge = trmm_merge_last(p, m, batch);
  const int nlaunch = p.nchunks - (merge ? 1 : 0);
  // timing: one event pair spans the back-to-back TRMM launches (an event record between
  // launches costs a few us of stream time each); gp_profile_read reports it per launch.
  // With late cross-covariance chunks in between, one pair per launch.
  const bool split = late < p.nchunks;
  if (!split) gpfit_prof_begin_n(GP_PROF_TRMM, stream, nlaunch);
  for (int ch = 0; ch < p.nchunks;) {
    const int ch1 = (merge && ch == p.nchunks - 2) ? ch + 1 : ch;
    for (int c = ch; c <= ch1; ++c) {
      if (c >= late) {
        gpfit_prof_begin(GP_PROF_CROSS, stream);
        if ((e = cross(c)) != hipSuccess) return e;
        gpfit_prof_end(GP_PROF_CROSS, stream);
      } else if (ready && c == 1 &&
                 (e = hipStreamWaitEvent(stream, ready[late - 1], 0)) != hipSuccess) {
        // chunk 1 waits for the last aux chunk, which (aux is in order) covers every later
        // one: one queue barrier instead of one per launch (~4 us each beside the 1.7-1.9 us
        // kernel boundary, profiles/r05/r05p_timeline.txt); those chunks are long done when
        // the second TRMM is reached
        return e;
      }
    }
    if (split) gpfit_prof_begin(GP_PROF_TRMM, stream);
    e = trmm_launch(p, ch, ch1, w.kt + (long long)ch * p.slab_elems, p.slab_elems,
                    w.part + ch * p.part_elems, p.part_elems, z, zld, L, m, batch, stream);
    if (e != hipSuccess) return e;
    if (split) gpfit_prof_end(GP_PROF_TRMM, stream);
    ch = ch1 + 1;
  }
  if (!split) gpfit_prof_end(GP_PROF_TRMM, stream);
  hipLaunchKernelGGL(finalize_kernel, dim3(gp_ceil_div(m, 256), batch), dim3(256), 0, stream,
                     w.part, p.NI, p.mc, p.part_elems, 0, m, s_pred, mean, var, ldo);
  return hipGetLastError();
}

}  // namespace

extern "C" int gp_predict_ex(const double* Linv, int ldinv, long long strideInv,
                             const double* X, int ldx, const double* Xs, int ldxs, int n, int m,
                             int d, const double* beta, int ldbeta, const double* s,
                             const double* s_pred, const double* w_hat, int ldw, double* mean,
                             double* var, int ldo, int batch, void* ws, long long ws_bytes,
                             int m_chunk, int layout, const double* z, long long ldz,
                             hipStream_t stream) {
  if (layout != GPFIT_LINV_PADDED && layout != GPFIT_LINV_PACKED) return -24;
  const bool packed = layout == GPFIT_LINV_PACKED;
  int rc = check_common(X, ldx, Xs, ldxs, n, m, d, beta, ldbeta, s, batch);
  if (rc) return rc;
  // with z given, w_hat is not read
  rc = check_solve(Linv, ldinv, strideInv, n, s_pred, z ? s_pred : w_hat, ldw, m, mean, var, ldo,
                   batch, packed);
  if (rc) return rc;
  if (z && (batch > 1 && ldz < gp_padded_n(n))) return -26;
  if (n == 0 || m == 0 || batch == 0) return 0;
  if (m_chunk < 0) return -23;
  const Plan p = make_plan(n, m, batch, m_chunk);
  if (!ws) return -21;
  if (ws_bytes < p.bytes) return -22;
  const WS w = carve(p, ws);
  const LinvRef L{Linv, ldinv, strideInv, packed};
  const double* zz = z ? z : w.z;
  const long long zld = z ? ldz : p.npad;
  hipError_t e;
#define GP_CK(x) do { e = (x); if (e != hipSuccess) return GPFIT_ERR_HIP - (int)e; } while (0)
  if (!z) GP_CK(trmv_pred(p.npad, w.zp, L, w_hat, ldw, n, batch, w.z, p.npad, stream));
  if (res_eligible(p.npad)) {
    GP_CK(res_all(p, w, res_fused(d) ? ResSrc::Fused : ResSrc::Serial, L, n, m, d, X, ldx, Xs,
                  ldxs, beta, ldbeta, s, s_pred, zz, zld, mean, var, ldo, batch, stream));
    return 0;
  }
  // chunk by chunk: cross-covariance, TRMM, mean / var, reusing one slab -- except that a
  // merged last chunk (trmm_merge_last) has its own second slab, and its TRMM and finalize
  // cover the chunk before it too
  const bool merge = trmm_merge_last(p, m, batch);
  for (int ch = 0; ch < p.nchunks; ++ch) {
    const bool held = merge && ch == p.nchunks - 2;   // TRMM deferred to the merged launch
    const int sl = (merge && ch == p.nchunks - 1) ? 1 : 0;
    gpfit_prof_begin(GP_PROF_CROSS, stream);
    GP_CK(cross_chunk(p, ch, w.kt + sl * p.slab_elems, X, ldx, Xs, ldxs, n, m, d, beta, ldbeta,
                      s, batch, stream));
    gpfit_prof_end(GP_PROF_CROSS, stream);
    if (held) continue;
    const int ch0 = (merge && ch == p.nchunks - 1) ? ch - 1 : ch;
    gpfit_prof_begin(GP_PROF_TRMM, stream);
    GP_CK(trmm_launch(p, ch0, ch, w.kt, p.slab_elems, w.part, p.part_elems, zz, zld, L, m, batch,
                      stream));
    gpfit_prof_end(GP_PROF_TRMM, stream);
    const int j0 = ch0 * p.mc;
    const int mv = (m - j0 < (ch - ch0 + 1) * p.mc) ? m - j0 : (ch - ch0 + 1) * p.mc;
    hipLaunchKernelGGL(finalize_kernel, dim3(gp_ceil_div(mv, 256), batch), dim3(256), 0, stream,
                       w.part, p.NI, p.mc, p.part_elems, j0, mv, s_pred, mean, var, ldo);
    GP_CK(hipGetLastError());
  }
#undef GP_CK
  return 0;
}

extern "C" int gp_predict(const double* Linv, int ldinv, long long strideInv, const double* X,
                          int ldx, const double* Xs, int ldxs, int n, int m, int d,
                          const double* beta, int ldbeta, const double* s,
                          const double* s_pred, const double* w_hat, int ldw, double* mean,
                          double* var, int ldo, int batch, void* ws, long long ws_bytes,
                          int m_chunk, hipStream_t stream) {
  return gp_predict_ex(Linv, ldinv, strideInv, X, ldx, Xs, ldxs, n, m, d, beta, ldbeta, s,
                       s_pred, w_hat, ldw, mean, var, ldo, batch, ws, ws_bytes, m_chunk,
                       GPFIT_LINV_PADDED, nullptr, 0, stream);
}

// z = L^-1 w alone, with the prediction's arithmetic (the z gp_predict forms internally, bit
// for bit): rank 0 of the sharded single-GP path ships it with L^-1.  Scratch: the trmv
// partials.
extern "C" long long gp_predict_z_ws_bytes(int n, int batch) {
  if (n <= 0 || batch <= 0) return 0;
  const long long npad = gp_padded_n(n);
  return ((8LL * batch * gp_ceil_div(npad, kZS) * npad + 255) / 256) * 256;
}

extern "C" int gp_predict_z(const double* Linv, int ldinv, long long strideInv, int layout,
                            int n, const double* w_hat, int ldw, double* z, long long ldz,
                            int batch, void* ws, long long ws_bytes, hipStream_t stream) {
  if (!Linv || (reinterpret_cast<uintptr_t>(Linv) & 15)) return -1;
  if (layout != GPFIT_LINV_PADDED && layout != GPFIT_LINV_PACKED) return -4;
  const bool packed = layout == GPFIT_LINV_PACKED;
  if (n < 0) return -5;
  const int npad = gp_padded_n(n);
  if (!packed && (ldinv < npad || (ldinv & 1))) return -2;
  const long long per = packed ? linv_packed_elems(npad) : (long long)ldinv * npad;
  if ((batch > 1 && strideInv < per) || (strideInv & 1)) return -3;
  if (!w_hat) return -6;
  if (ldw < n && batch > 1) return -7;
  if (!z) return -8;
  if (ldz < npad && batch > 1) return -9;
  if (batch < 0) return -10;
  if (n == 0 || batch == 0) return 0;
  if (!ws) return -11;
  if (ws_bytes < gp_predict_z_ws_bytes(n, batch)) return -12;
  const hipError_t e = trmv_pred(npad, static_cast<double*>(ws), LinvRef{Linv, ldinv, strideInv,
                                 packed}, w_hat, ldw, n, batch, z, ldz, stream);
  return e == hipSuccess ? 0 : GPFIT_ERR_HIP - (int)e;
}

// The tile-packed layout (linv_col): gp_linv_packed_elems doubles per problem; pack from and
// unpack into the padded buffer (unpack writes every stored element: the rows below a column's
// first tile are left as they are, zero in a buffer prepared for gp_predict).
extern "C" long long gp_linv_packed_elems(int n) {
  if (n <= 0) return 0;
  return linv_packed_elems(gp_padded_n(n));
}

namespace {
__global__ __launch_bounds__(256) void linv_pack_kernel(const double* __restrict__ A, int npad,
                                                        long long ld, double* __restrict__ P,
                                                        int unpack) {
  const int c = blockIdx.x;
  const int r0 = (c >> 4) << 4;
  double* col = const_cast<double*>(A) + (long long)c * ld;
  double* pc = P + linv_col(c, npad);
  // 16-B vectors: r0, ld, npad and linv_col are even
  for (int r = r0 + 2 * threadIdx.x; r < npad; r += 512) {
    if (!unpack)
      *reinterpret_cast<double2*>(pc + r) = *reinterpret_cast<const double2*>(col + r);
    else
      *reinterpret_cast<double2*>(col + r) = *reinterpret_cast<const double2*>(pc + r);
  }
}
}  // namespace

extern "C" int gp_pack_linv(const double* Linv, int n, int ldinv, double* P, hipStream_t stream) {
  if (!Linv || (reinterpret_cast<uintptr_t>(Linv) & 15)) return -1;
  if (n < 0) return -2;
  const int npad = gp_padded_n(n);
  if (ldinv < npad || (ldinv & 1)) return -3;
  if (!P || (reinterpret_cast<uintptr_t>(P) & 15)) return -4;
  if (n == 0) return 0;
  hipLaunchKernelGGL(linv_pack_kernel, dim3(npad), dim3(256), 0, stream, Linv, npad,
                     (long long)ldinv, P, 0);
  const hipError_t e = hipGetLastError();
  return e == hipSuccess ? 0 : GPFIT_ERR_HIP - (int)e;
}

extern "C" int gp_unpack_linv(const double* P, int n, double* Linv, int ldinv,
                              hipStream_t stream) {
  if (!P || (reinterpret_cast<uintptr_t>(P) & 15)) return -1;
  if (n < 0) return -2;
  const int npad = gp_padded_n(n);
  if (!Linv || (reinterpret_cast<uintptr_t>(Linv) & 15)) return -3;
  if (ldinv < npad || (ldinv & 1)) return -4;
  if (n == 0) return 0;
  hipLaunchKernelGGL(linv_pack_kernel, dim3(npad), dim3(256), 0, stream, Linv, npad,
                     (long long)ldinv, const_cast<double*>(P), 1);
  const hipError_t e = hipGetLastError();
  return e == hipSuccess ? 0 : GPFIT_ERR_HIP - (int)e;
}

// Prediction path for later enqueues (process-wide A/B hook): 0 = automatic (trmm_res_kernel at
// npad <= 512, cross-covariance fused when d <= 8; else cross-covariance chunks + the pair TRMM),
// 1 = always chunks + pair TRMM, 2 = trmm_res_kernel from materialised chunks at npad <= 512.
// Returns the previous value.
extern "C" int gp_set_predict_path(int path) {
  return g_predict_path.exchange((path == 1 || path == 2) ? path : 0);
}

extern "C" int gp_predict_cross(const double* X, int ldx, const double* Xs, int ldxs, int n,
                                int m, int d, const double* beta, int ldbeta, const double* s,
                                int batch, void* ws, long long ws_bytes, int m_chunk,
                                hipStream_t stream) {
  int rc = check_common(X, ldx, Xs, ldxs, n, m, d, beta, ldbeta, s, batch);
  if (rc) return rc;
  if (n == 0 || m == 0 || batch == 0) return 0;
  if (m_chunk < 0) return -23;
  const Plan p = make_plan(n, m, batch, m_chunk, true);
  if (!ws) return -21;
  if (ws_bytes < p.bytes) return -22;
  const WS w = carve(p, ws);
  // one timing-event pair around all chunks (the stream runs nothing else in between)
  gpfit_prof_begin_n(GP_PROF_CROSS, stream, p.nchunks);
  for (int ch = 0; ch < p.nchunks; ++ch) {
    hipError_t e = cross_chunk(p, ch, w.kt + (long long)ch * p.slab_elems, X, ldx, Xs, ldxs, n,
                               m, d, beta, ldbeta, s, batch, stream);
    if (e != hipSuccess) return GPFIT_ERR_HIP - (int)e;
  }
  gpfit_prof_end(GP_PROF_CROSS, stream);
  return 0;
}

extern "C" int gp_predict_solve(const double* Linv, int ldinv, long long strideInv, int n,
                                int m, const double* s_pred, const double* w_hat, int ldw,
                                double* mean, double* var, int ldo, int batch, void* ws,
                                long long ws_bytes, int m_chunk, hipStream_t stream) {
  if (n < 0) return -4;
  if (m < 0) return -5;
  if (batch < 0) return -12;
  int rc = check_solve(Linv, ldinv, strideInv, n, s_pred, w_hat, ldw, m, mean, var, ldo, batch);
  if (rc) return rc;
  if (n == 0 || m == 0 || batch == 0) return 0;
  if (m_chunk < 0) return -23;
  const Plan p = make_plan(n, m, batch, m_chunk, true);
  if (!ws) return -21;
  if (ws_bytes < p.bytes) return -22;
  const WS w = carve(p, ws);
  hipError_t e;
#define GP_CK(x) do { e = (x); if (e != hipSuccess) return GPFIT_ERR_HIP - (int)e; } while (0)
  const LinvRef L{Linv, ldinv, strideInv, false};
  GP_CK(trmv_pred(p.npad, w.zp, L, w_hat, ldw, n, batch, w.z, p.npad, stream));
  if (res_eligible(p.npad)) {
    GP_CK(res_all(p, w, ResSrc::Prepared, L, n, m, 0, nullptr, 0, nullptr, 0, nullptr, 0,
                  nullptr, s_pred, w.z, p.npad, mean, var, ldo, batch, stream));
    return 0;
  }
  GP_CK(solve_all(p, w, L, w.z, p.npad, m, s_pred, mean, var, ldo, batch, stream, nullptr,
                  p.nchunks, [](int) { return hipSuccess; }));
#undef GP_CK
  return 0;
}

// ------------------------------------------------------------------------------------------
// gp_fit_predict: Gram -> Cholesky/L^-1 -> predict as one stream-ordered operation on `stream`.
// With a context (gp_ctx_create) the cross-covariance forks onto the context's stream:
//   `stream`: the factorisation's schedule kernel, the Gram, the factorisation (latency-bound,
//         few CUs busy), z = L^-1 w, and per chunk, once that chunk's cross-covariance is done,
//         the TRMM (all row tiles of the chunk, so its K* stays cached), and one mean / var
//         pass over all m points (round 4 forked the factorisation and the prediction onto
//         streams of their own too; each event hop cost 16-27 us of the step);
//   aux : the cross-covariance of every chunk (independent of the factorisation), CU-masked so
//         that it leaves aux_free_cus CUs to the factorisation, from the factorisation's
//         block step cross_start * n/64 on;
// each TRMM waits for its chunk's event, which joins aux back.  Without a context every step
// runs in order on `stream`.
struct gp_ctx_s {
  int device = -1;
  double cross_start = 0.4;
  int aux_chunks = -1;           // cross-covariance chunks on aux (-1: all; gp_ctx_set_aux_chunks)
  hipStream_t aux = nullptr;
  hipEvent_t e_late = nullptr;   // the factorisation has turned latency-bound
  std::vector<hipEvent_t> e_chunk;  // after chunk ch's cross-covariance (grown on demand)
};

namespace {

// Defaults measured at C3.  Round 1 (127-launch factorisation): the cross-covariance on all
// CUs at once doubled the early, bandwidth-bound trailing updates, so it ran CU-masked from 40%
// of the block steps (profiles/r01/ab_cross_select_exp.log).  With the persistent
// factorisation (1.9 ms, the cross-covariance's start event recorded before its launch) and
// per-chunk events, leaving 32 CUs free was best: 27.03-27.11 ms/step vs 27.03-27.14 for no
// mask, 27.31-27.57 for 64-96 and 27.79-27.88 for 128 (profiles/r02/sweep_cross_mask_r02e.log).
// Round 3's factorisation (1.82 ms alone) loses little to an unmasked cross-covariance, which
// then ends 0.3 ms sooner, before the first TRMM launch needs the GPU: no mask 26.68-26.71
// ms/step vs 26.87-26.95 for 32 CUs, 27.08-27.10 for 16, 27.05-27.19 for 48-64, two
// interleaved rounds on one box (profiles/r03/sweep_aux_cus_r03.log).
constexpr double kCrossStart = 0.4;
constexpr int kAuxFreeCUs = 0;

hipError_t ctx_init(gp_ctx_s* c, double cross_start, int aux_free_cus) {
  hipError_t e = hipGetDevice(&c->device);
  if (e != hipSuccess) return e;
  c->cross_start = cross_start < 0 ? kCrossStart : cross_start;
  const int fr = aux_free_cus < 0 ? kAuxFreeCUs : aux_free_cus;
  // logical CU i sits on XCD i % 8 (measured with a CU-mask probe in round 1), so masking off
  // the low CUs reserves CUs evenly per XCD
  int ncu = 0;
  if (fr > 0 &&
      hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, c->device) ==
          hipSuccess &&
      fr < ncu) {
    std::vector<uint32_t> m((ncu + 31) / 32, 0u);
    for (int i = fr; i < ncu; ++i) m[i / 32] |= 1u << (i % 32);
    if ((e = hipExtStreamCreateWithCUMask(&c->aux, (uint32_t)m.size(), m.data())) != hipSuccess)
      return e;
  } else if ((e = hipStreamCreateWithFlags(&c->aux, hipStreamNonBlocking)) != hipSuccess) {
    return e;
  }
  hipEvent_t* ev[1] = {&c->e_late};
  for (hipEvent_t* p : ev)
    if ((e = hipEventCreateWithFlags(p, hipEventDisableTiming)) != hipSuccess) return e;
  return hipSuccess;
}

hipError_t ctx_fini(gp_ctx_s* c) {
  hipError_t first = hipSuccess;
  auto keep = [&](hipError_t e) { if (first == hipSuccess && e != hipSuccess) first = e; };
  int dev0 = 0;
  keep(hipGetDevice(&dev0));
  if (c->device >= 0) keep(hipSetDevice(c->device));
  hipStream_t st[1] = {c->aux};
  for (hipStream_t x : st)
    if (x) {
      keep(hipStreamSynchronize(x));
      keep(hipStreamDestroy(x));
    }
  hipEvent_t ev[1] = {c->e_late};
  for (hipEvent_t x : ev)
    if (x) keep(hipEventDestroy(x));
  for (hipEvent_t x : c->e_chunk)
    if (x) keep(hipEventDestroy(x));
  c->e_chunk.clear();
  if (c->device >= 0) keep(hipSetDevice(dev0));
  return first;
}

}  // namespace

extern "C" int gp_ctx_create(double cross_start, int aux_free_cus, void** ctx) {
  if (cross_start > 1.0) return -1;
  if (!ctx) return -3;
  *ctx = nullptr;
  gp_ctx_s* c = new (std::nothrow) gp_ctx_s();
  if (!c) return GPFIT_ERR_HIP - (int)hipErrorOutOfMemory;
  const hipError_t e = ctx_init(c, cross_start, aux_free_cus);
  if (e != hipSuccess) {
    (void)ctx_fini(c);
    delete c;
    return GPFIT_ERR_HIP - (int)e;
  }
  *ctx = c;
  return 0;
}

extern "C" int gp_ctx_set_aux_chunks(void* ctx, int nchunks) {
  if (!ctx) return -1;
  if (nchunks < -1) return -2;
  static_cast<gp_ctx_s*>(ctx)->aux_chunks = nchunks;
  return 0;
}

extern "C" int gp_ctx_destroy(void* ctx) {
  if (!ctx) return 0;
  gp_ctx_s* c = static_cast<gp_ctx_s*>(ctx);
  const hipError_t e = ctx_fini(c);
  delete c;
  return e == hipSuccess ? 0 : GPFIT_ERR_HIP - (int)e;
}

extern "C" int gp_fit_predict(const double* X, int ldx, const double* Xs, int ldxs, int n,
                              int m, int d, const double* beta, int ldbeta, const double* s,
                              const double* delta, const double* s_pred, const double* w_hat,
                              int ldw, double* G, int ldg, long long strideG, double* Linv,
                              int ldinv, long long strideInv, int* info, double* logdet,
                              double* mean, double* var, int ldo, int batch, void* ws,
                              long long ws_bytes, int m_chunk, void* ctx, hipStream_t stream) {
  int rc = check_common(X, ldx, Xs, ldxs, n, m, d, beta, ldbeta, s, batch);
  if (rc) return rc;
  rc = check_solve(Linv, ldinv, strideInv, n, s_pred, w_hat, ldw, m, mean, var, ldo, batch);
  if (rc) return rc;
  if (!delta) return -24;
  if (!G) return -25;
  if (ldg < n || (batch > 1 && strideG < (long long)ldg * n)) return -26;
  if (n == 0 || m == 0 || batch == 0) return 0;
  if (m_chunk < 0) return -23;
  const Plan p = make_plan(n, m, batch, m_chunk, true, true);
  if (!ws || (reinterpret_cast<uintptr_t>(ws) & 255)) return -21;
  if (ws_bytes < p.bytes) return -22;
  const WS w = carve(p, ws);
  gp_ctx_s* S = static_cast<gp_ctx_s*>(ctx);
  hipError_t e;
#define GP_CK(x) do { e = (x); if (e != hipSuccess) return GPFIT_ERR_HIP - (int)e; } while (0)
  if (S) {
    int dev = -1;
    if (hipGetDevice(&dev) != hipSuccess || dev != S->device) return -29;
    while ((int)S->e_chunk.size() < p.nchunks) {
      hipEvent_t ev = nullptr;
      GP_CK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
      S->e_chunk.push_back(ev);
    }
  }
  // the factorisation and the prediction run on the caller's stream itself: z and the first
  // TRMM follow the factorisation, and the next call's Gram the last TRMM, without a
  // cross-stream hop (an event wait between pp_kernel and the trmv cost 16-20 us of every C3
  // step, profiles/r05/r05a_timeline.txt; the fork / join through a context stream another
  // ~27 us between steps, r05n_timeline.txt); only the cross-covariance forks onto aux
  hipStream_t fact = stream, aux = S ? S->aux : stream, pred = fact;
  // (the factorisation's schedule kernel,) Gram -> Cholesky / L^-1, with e_late once the
  // factorisation is latency-bound.  The Gram is enqueued from inside the factorisation's
  // setup, after its schedule kernel (GpfitPre): the schedule kernel's host-side preparation
  // then overlaps the Gram instead of leaving the GPU idle between Gram and factorisation
  // (16 us per C3 step, profiles/r05/r05n_timeline.txt)
  const int nblk = gp_ceil_div(n, GPFIT_POTRF_NB);
  const int k_late = S ? (int)(S->cross_start * nblk) : -1;
  struct GramPre {
    const double *X, *beta, *s, *delta;
    double* G;
    int ldx, ldbeta, n, d, ldg, batch;
    long long strideG;
    hipStream_t st;
    hipEvent_t late;
  } gp{X, beta, s, delta, G, ldx, ldbeta, n, d, ldg, batch, strideG, fact,
       (S && k_late <= 0) ? S->e_late : nullptr};
  GpfitPre pre;
  pre.arg = &gp;
  pre.fn = [](void* a) -> int {
    const GramPre& g = *static_cast<const GramPre*>(a);
    const int grc = gpfit_gram_lower(g.X, g.n, g.d, g.ldx, g.beta, g.ldbeta, g.s, g.delta, g.G,
                                     g.ldg, g.strideG, g.batch, g.st);
    if (grc) return grc;
    if (g.late) {
      const hipError_t er = hipEventRecord(g.late, g.st);
      if (er != hipSuccess) return GPFIT_ERR_HIP - (int)er;
    }
    return 0;
  };
  rc = gpfit_potrf_inv_event(G, n, ldg, strideG, Linv, ldinv, strideInv, batch, info, logdet,
                             w.pot, p.bytes - p.off_pot, fact, k_late > 0 ? k_late : -1,
                             (S && k_late > 0) ? S->e_late : nullptr, pre);
  if (rc) return rc;
  const LinvRef L{Linv, ldinv, strideInv, false};
  if (res_eligible(p.npad)) {
    // the cross-covariance is produced inside the prediction kernel (d <= 8; otherwise chunk
    // by chunk before each launch on pred): nothing forks onto aux
    GP_CK(trmv_pred(p.npad, w.zp, L, w_hat, ldw, n, batch, w.z, p.npad, pred));
    GP_CK(res_all(p, w, res_fused(d) ? ResSrc::Fused : ResSrc::Serial, L, n, m, d, X, ldx, Xs,
                  ldxs, beta, ldbeta, s, s_pred, w.z, p.npad, mean, var, ldo, batch, pred));
    return 0;
  }
  if (S) GP_CK(hipStreamWaitEvent(aux, S->e_late, 0));
  // chunks whose cross-covariance runs on aux, beside the factorisation and the earlier TRMMs
  // (all by default; the rest run on pred just before their TRMM: gp_ctx_set_aux_chunks)
  const int n_aux = (S && S->aux_chunks >= 0 && S->aux_chunks < p.nchunks) ? S->aux_chunks
                                                                            : p.nchunks;
  // aux: cross-covariance of those chunks (one timing-event pair around all of them)
  // (an event after each chunk: its TRMM waits for that chunk only, so the prediction starts
  // when the factorisation ends even if later chunks' cross-covariance is still running)
  if (n_aux > 0) gpfit_prof_begin_n(GP_PROF_CROSS, aux, n_aux);
  for (int ch = 0; ch < n_aux; ++ch) {
    GP_CK(cross_chunk(p, ch, w.kt + (long long)ch * p.slab_elems, X, ldx, Xs, ldxs, n, m, d,
                      beta, ldbeta, s, batch, aux));
    if (S && ch + 1 < n_aux) GP_CK(hipEventRecord(S->e_chunk[ch], aux));
  }
  if (n_aux > 0) gpfit_prof_end(GP_PROF_CROSS, aux);
  // pred: z, then TRMM + mean / var chunk by chunk.  One launch per chunk (not one for all):
  // the dispatcher interleaves another stream's kernels between launches, so a concurrent
  // factorisation is not starved behind a 25 ms grid (measured: 14 ms vs 3 ms per potrf).
  if (S && n_aux > 0) GP_CK(hipEventRecord(S->e_chunk[n_aux - 1], aux));   // after the end event
  GP_CK(trmv_pred(p.npad, w.zp, L, w_hat, ldw, n, batch, w.z, p.npad, pred));
  GP_CK(solve_all(p, w, L, w.z, p.npad, m, s_pred, mean, var, ldo, batch, pred,
                  S ? S->e_chunk.data() : nullptr, n_aux, [&](int ch) {
                    return cross_chunk(p, ch, w.kt + (long long)ch * p.slab_elems, X, ldx, Xs,
                                       ldxs, n, m, d, beta, ldbeta, s, batch, pred);
                  }));
  // (every chunk's cross-covariance on aux is joined by the TRMM that waits for its event)
#undef GP_CK
  return 0;
}

// gp_predict from a Cholesky factor L (LAPACK layout): L^-1 by gp_trtri into the head of the
// workspace, then gp_predict with the rest.
extern "C" long long gp_predict_chol_ws_bytes(int n, int m, int batch, int m_chunk) {
  if (n <= 0 || m <= 0 || batch <= 0) return 0;
  const long long npad = gp_padded_n(n);
  return ((8LL * npad * npad * batch + 255) / 256) * 256 + make_plan(n, m, batch, m_chunk).bytes;
}

extern "C" int gp_predict_chol(const double* L, int ldl, long long strideL, const double* X,
                               int ldx, const double* Xs, int ldxs, int n, int m, int d,
                               const double* beta, int ldbeta, const double* s,
                               const double* s_pred, const double* w_hat, int ldw, double* mean,
                               double* var, int ldo, int batch, int* info, void* ws,
                               long long ws_bytes, int m_chunk, hipStream_t stream) {
  if (!L) return -1;
  if (ldl < n || ldl < 1) return -2;
  if (batch > 1 && strideL < (long long)ldl * n) return -3;
  int rc = check_common(X, ldx, Xs, ldxs, n, m, d, beta, ldbeta, s, batch);
  if (rc) return rc;
  if (n == 0 || m == 0 || batch == 0) return 0;
  if (m_chunk < 0) return -24;
  if (!ws) return -22;
  if (ws_bytes < gp_predict_chol_ws_bytes(n, m, batch, m_chunk)) return -23;
  const long long npad = gp_padded_n(n);
  const long long head = ((8LL * npad * npad * batch + 255) / 256) * 256;
  double* Linv = static_cast<double*>(ws);
  rc = gp_trtri(L, n, ldl, strideL, Linv, (int)npad, npad * npad, batch, info, stream);
  if (rc) return rc;
  rc = gp_predict(Linv, (int)npad, npad * npad, X, ldx, Xs, ldxs, n, m, d, beta, ldbeta, s,
                  s_pred, w_hat, ldw, mean, var, ldo, batch, static_cast<char*>(ws) + head,
                  ws_bytes - head, m_chunk, stream);
  return rc;
}
