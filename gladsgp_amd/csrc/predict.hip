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
//   1. ardse (gram.hip)   Kt = s exp(-sum beta (X - Xs)^2), n_pad x m_c, column per test point
//                         (exp evaluated once per element; HBM-write-bound)
//   2. trmm_reduce        for each 128x128 tile (I, C) of V: acc = sum_{k < 128(I+1)} X[I,k] Kt[k,C]
//                         on v_mfma_f64_16x16x4_f64, epilogue: per-column partial sums of
//                         acc*z and acc^2 -> part[b][I][col]  (MFMA-bound: n^2 m flop)
//   3. finalize           mean = sum_I pm, var = s_pred - sum_I pv
// z = X w is a small lower-triangular gemv (linalg.hip trmv_kernel).
#include "gpfit_common.h"
#include "gpfit_profile.h"
#include "../../include/gpfit.h"

hipError_t gpfit_ardse_launch(const double* XA, int na, int ldxa, const double* XB, int nb,
                              int ldxb, int d, const double* beta, int ldbeta,
                              const double* s, const double* delta, double* out, int ldo,
                              long long stride_o, int rows_out, int cols_out, int batch,
                              hipStream_t st);
hipError_t gpfit_trmv_launch(const double* Linv, int ld, long long sL, const double* w,
                             int ldw, double* z, int ldz, int rows, int n, int batch,
                             hipStream_t st);

namespace {

constexpr int BI = 128;   // V tile rows (L^-1 rows)
constexpr int BC = 128;   // V tile cols (test points)
constexpr int BK = 16;    // K step
constexpr int PA = BI + 8;   // As pitch (doubles): [k][i]
constexpr int PB = BK + 1;   // Bs pitch (doubles): [c][k]
constexpr long long kDefaultChunkElems = 16ll << 20;   // ~128 MB of Kt per chunk (MALL-sized)

// One 128x128 tile of V = Linv * Kt per block; 4 waves in 2x2, each 64x64 = 4x4 MFMA tiles.
__global__ __launch_bounds__(256) void trmm_reduce_kernel(
    const double* __restrict__ Linv, int ld, long long sL, const double* __restrict__ Kt,
    int ldk, long long sK, const double* __restrict__ z, int npad, double* __restrict__ part,
    int NI, int NC, int mc) {
  const int b = blockIdx.y;
  const int t = blockIdx.x;
  const int I = NI - 1 - t / NC;     // heaviest row tiles dispatch first
  const int C = t % NC;
  const double* L = Linv + b * sL + I * BI;                  // rows I*BI.., column k
  const double* K = Kt + b * sK + (long long)C * BC * ldk;   // column c, rows k
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int wr = w >> 1, wc = w & 1, li = lane & 15, lk = lane >> 4;

  __shared__ double As[BK * PA];
  __shared__ double Bs[BC * PB];
  __shared__ double red[2][2][BC];

  f64x4 acc[4][4];
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int c = 0; c < 4; ++c) acc[a][c] = zero4();

  // register staging: A = 16 x 128 (i fast), B = 128 cols x 16 k (k fast); 8 doubles each.
  double2 ra[4], rb[4];
  const int kend = (I + 1) * BI;
  auto gload = [&](int k0) {
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int g = tid + 256 * q;           // 1024 double2 per operand
      const int i2 = (g & 63) * 2, ka = g >> 6;
      ra[q] = *reinterpret_cast<const double2*>(L + i2 + (long long)(k0 + ka) * ld);
      const int kb = (g & 7) * 2, c = g >> 3;
      rb[q] = *reinterpret_cast<const double2*>(K + k0 + kb + (long long)c * ldk);
    }
  };
  auto lstore = [&]() {
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int g = tid + 256 * q;
      const int i2 = (g & 63) * 2, ka = g >> 6;
      *reinterpret_cast<double2*>(&As[ka * PA + i2]) = ra[q];
      const int kb = (g & 7) * 2, c = g >> 3;
      Bs[c * PB + kb] = rb[q].x;
      Bs[c * PB + kb + 1] = rb[q].y;
    }
  };

  gload(0);
  for (int k0 = 0; k0 < kend; k0 += BK) {
    __syncthreads();
    lstore();
    __syncthreads();
    if (k0 + BK < kend) gload(k0 + BK);
#pragma unroll
    for (int k4 = 0; k4 < BK / 4; ++k4) {
      const int k = k4 * 4 + lk;
      double a[4], bb[4];
#pragma unroll
      for (int mi = 0; mi < 4; ++mi) a[mi] = As[k * PA + wr * 64 + mi * 16 + li];
#pragma unroll
      for (int nj = 0; nj < 4; ++nj) bb[nj] = Bs[(wc * 64 + nj * 16 + li) * PB + k];
#pragma unroll
      for (int mi = 0; mi < 4; ++mi)
#pragma unroll
        for (int nj = 0; nj < 4; ++nj) acc[mi][nj] = mfma16x16x4(a[mi], bb[nj], acc[mi][nj]);
    }
  }

  // epilogue: column partial sums of V*z and V^2 over this tile's 128 rows
  const double* zb = z + (long long)b * npad + I * BI + wr * 64;
  double zr[4][4];
#pragma unroll
  for (int mi = 0; mi < 4; ++mi)
#pragma unroll
    for (int r = 0; r < 4; ++r) zr[mi][r] = zb[mi * 16 + lk + 4 * r];
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
      red[wr][0][wc * 64 + nj * 16 + li] = sm;
      red[wr][1][wc * 64 + nj * 16 + li] = sv;
    }
  }
  __syncthreads();
  if (tid < BC) {
    const int col = C * BC + tid;
    double* pm = part + ((long long)(b * 2 + 0) * NI + I) * mc;
    double* pv = part + ((long long)(b * 2 + 1) * NI + I) * mc;
    pm[col] = red[0][0][tid] + red[1][0][tid];
    pv[col] = red[0][1][tid] + red[1][1][tid];
  }
}

__global__ __launch_bounds__(256) void finalize_kernel(const double* __restrict__ part, int NI,
                                                       int mc, int mv,
                                                       const double* __restrict__ s_pred,
                                                       double* __restrict__ mean,
                                                       double* __restrict__ var, int ldo,
                                                       int c0) {
  const int b = blockIdx.y;
  const int j = blockIdx.x * 256 + threadIdx.x;
  if (j >= mv) return;
  const double* pm = part + (long long)(b * 2 + 0) * NI * mc + j;
  const double* pv = part + (long long)(b * 2 + 1) * NI * mc + j;
  double sm = 0.0, sv = 0.0;
  for (int I = 0; I < NI; ++I) {
    sm += pm[(long long)I * mc];
    sv += pv[(long long)I * mc];
  }
  mean[(long long)b * ldo + c0 + j] = sm;
  var[(long long)b * ldo + c0 + j] = s_pred[b] - sv;
}

struct Plan {
  int npad, NI, mc, NC, nchunks;
  long long off_z, off_kt, off_part, bytes;
};

Plan make_plan(int n, int m, int batch, int m_chunk) {
  Plan p;
  p.npad = gp_padded_n(n);
  p.NI = p.npad / BI;
  const int mpad = gp_ceil_div(m, BC) * BC;
  int mc;
  if (m_chunk > 0) {
    mc = gp_ceil_div(m_chunk, BC) * BC;
  } else {
    long long cap = kDefaultChunkElems / ((long long)p.npad * (batch > 0 ? batch : 1));
    mc = (int)((cap / BC) * BC);
    if (mc < BC) mc = BC;
  }
  if (mc > mpad) mc = mpad;
  if (mc < BC) mc = BC;
  p.mc = mc;
  p.NC = mc / BC;
  p.nchunks = gp_ceil_div(m, mc);
  long long z = (long long)batch * p.npad;
  long long kt = (long long)batch * mc * p.npad;
  long long part = (long long)batch * 2 * p.NI * mc;
  p.off_z = 0;
  p.off_kt = ((z * 8 + 255) / 256) * 256;
  p.off_part = p.off_kt + ((kt * 8 + 255) / 256) * 256;
  p.bytes = p.off_part + part * 8;
  return p;
}

}  // namespace

extern "C" long long gp_predict_ws_bytes(int n, int m, int batch, int m_chunk) {
  if (n <= 0 || m <= 0 || batch <= 0) return 0;
  return make_plan(n, m, batch, m_chunk).bytes;
}

extern "C" int gp_predict(const double* Linv, int ldinv, long long strideInv, const double* X,
                          int ldx, const double* Xs, int ldxs, int n, int m, int d,
                          const double* beta, int ldbeta, const double* s,
                          const double* s_pred, const double* w_hat, int ldw, double* mean,
                          double* var, int ldo, int batch, void* ws, long long ws_bytes,
                          int m_chunk, hipStream_t stream) {
  if (!Linv || (reinterpret_cast<uintptr_t>(Linv) & 15)) return -1;
  const int npad = gp_padded_n(n);
  if (ldinv < npad || ldinv < 1 || (ldinv & 1)) return -2;   // 16-B aligned double2 loads
  if ((batch > 1 && strideInv < (long long)ldinv * npad) || (strideInv & 1)) return -3;
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
  if (!s_pred) return -14;
  if (!w_hat) return -15;
  if (ldw < n && batch > 1) return -16;
  if (!mean) return -17;
  if (!var) return -18;
  if (ldo < m && batch > 1) return -19;
  if (batch < 0) return -20;
  if (n == 0 || m == 0 || batch == 0) return 0;
  const Plan p = make_plan(n, m, batch, m_chunk);
  if (!ws) return -21;
  if (ws_bytes < p.bytes) return -22;
  if (m_chunk < 0) return -23;
  char* base = static_cast<char*>(ws);
  double* z = reinterpret_cast<double*>(base + p.off_z);
  double* kt = reinterpret_cast<double*>(base + p.off_kt);
  double* part = reinterpret_cast<double*>(base + p.off_part);
  hipError_t e;
#define GP_CK(x) do { e = (x); if (e != hipSuccess) return GPFIT_ERR_HIP - (int)e; } while (0)
  GP_CK(gpfit_trmv_launch(Linv, ldinv, strideInv, w_hat, ldw, z, p.npad, p.npad, n, batch,
                          stream));
  const long long sK = (long long)p.mc * p.npad;
  for (int ch = 0; ch < p.nchunks; ++ch) {
    const int c0 = ch * p.mc;
    const int mv = (m - c0 < p.mc) ? (m - c0) : p.mc;
    gpfit_prof_begin(GP_PROF_CROSS, stream);
    GP_CK(gpfit_ardse_launch(X, n, ldx, Xs + (long long)c0 * ldxs, mv, ldxs, d, beta, ldbeta,
                             s, nullptr, kt, p.npad, sK, p.npad, p.mc, batch, stream));
    gpfit_prof_end(GP_PROF_CROSS, stream);
    const int ncol_tiles = gp_ceil_div(mv, BC);
    gpfit_prof_begin(GP_PROF_TRMM, stream);
    hipLaunchKernelGGL(trmm_reduce_kernel, dim3(p.NI * ncol_tiles, batch), dim3(256), 0,
                       stream, Linv, ldinv, strideInv, kt, p.npad, sK, z, p.npad, part, p.NI,
                       ncol_tiles, p.mc);
    gpfit_prof_end(GP_PROF_TRMM, stream);
    GP_CK(hipGetLastError());
    hipLaunchKernelGGL(finalize_kernel, dim3(gp_ceil_div(mv, 256), batch), dim3(256), 0,
                       stream, part, p.NI, p.mc, mv, s_pred, mean, var, ldo, c0);
    GP_CK(hipGetLastError());
  }
#undef GP_CK
  return 0;
}
