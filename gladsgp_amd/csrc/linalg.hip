// Small fp64 linear-algebra helpers on the fit side of the path:
//   gp_trmv : z = L^-1 w            (triangular gemv, HBM-bound: reads n^2/2 doubles)
//   gp_nll  : 1/2 ||L^-1 w||^2 + 1/2 log|A|   — the GP negative log-likelihood of GPmodule
//             (examples/02...ipynb:70-72, no 2pi term) and the per-PC quadratic form + logdet
//             of SEPIA's logLik (src/model.py:234-235 drives it through do_mcmc).
#include "gpfit_common.h"
#include "gpfit_internal.h"
#include "../../include/gpfit.h"

namespace {

// z_b[r] = sum_{k<=r, k<n} Linv_b[r,k] w_b[k] for r0 <= r < rows.  1024 threads = 64 rows x 16
// k-slices: each wave reads 64 consecutive rows of one column (512 B, coalesced), the 16
// partial sums meet in LDS.  Reads the n^2/2 lower triangle once: HBM-bound.
constexpr int kTrmvSlices = 16;
__global__ __launch_bounds__(1024) void trmv_kernel(const double* __restrict__ Linv, int ld,
                                                    long long sL, const double* __restrict__ w,
                                                    int ldw, double* __restrict__ z, int ldz,
                                                    int r0, int rows, int n) {
  const int b = blockIdx.y;
  const int rb = r0 + blockIdx.x * 64;
  const int r = rb + (threadIdx.x & 63);
  const int ks = threadIdx.x >> 6;
  const double* L = Linv + b * sL;
  const double* wb = w + (long long)b * ldw;
  double acc0 = 0.0, acc1 = 0.0;
  const int kend = min(rb + 64, n);   // block-uniform bound; L is zero above r
  if (r < rows) {
    int k = ks;
    for (; k + kTrmvSlices < kend; k += 2 * kTrmvSlices) {
      acc0 = fma(L[r + (long long)k * ld], wb[k], acc0);
      acc1 = fma(L[r + (long long)(k + kTrmvSlices) * ld], wb[k + kTrmvSlices], acc1);
    }
    if (k < kend) acc0 = fma(L[r + (long long)k * ld], wb[k], acc0);
  }
  __shared__ double red[kTrmvSlices][64];
  red[ks][threadIdx.x & 63] = acc0 + acc1;
  __syncthreads();
  if (ks == 0 && r < rows) {
    const int t = threadIdx.x;
    double s = 0.0;
#pragma unroll
    for (int q = 0; q < kTrmvSlices; ++q) s += red[q][t];
    z[(long long)b * ldz + r] = s;
  }
}

// out[b] = sign * (1/2 ||z_b||^2 + 1/2 logdet[b]); a problem whose matrix is not positive
// definite (info[b] > 0, when info is given) gets sign * +inf, a factorisation that gave up
// (info[b] < 0, an internal error) NaN and raises the sticky `status` word (when given).
// info_out (when given) receives info[b]: gp_loglik's caller copy without a separate memcpy
// (one hipMemcpyAsync per Metropolis group before, ~5 us each).
__global__ __launch_bounds__(256) void nll_reduce_kernel(const double* __restrict__ z, int ldz,
                                                         int n,
                                                         const double* __restrict__ logdet,
                                                         const int* __restrict__ info,
                                                         double sign,
                                                         double* __restrict__ nll,
                                                         int* __restrict__ status,
                                                         int* __restrict__ info_out) {
  const int b = blockIdx.x;
  const double* zb = z + (long long)b * ldz;
  double acc = 0.0;
  for (int r = threadIdx.x; r < n; r += 256) acc = fma(zb[r], zb[r], acc);
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) acc += __shfl_xor(acc, off, 64);
  __shared__ double red[4];
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = acc;
  __syncthreads();
  if (threadIdx.x == 0) {
    const double v = 0.5 * ((red[0] + red[1]) + (red[2] + red[3])) + 0.5 * logdet[b];
    const int f = info ? info[b] : 0;
    nll[b] = f < 0 ? __builtin_nan("") : sign * (f > 0 ? __builtin_huge_val() : v);
    if (info_out) info_out[b] = f;
    if (f < 0 && status)
      __hip_atomic_fetch_or(status, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

}  // namespace

hipError_t gpfit_trmv_rows_launch(const double* Linv, int ld, long long sL, const double* w,
                                  int ldw, double* z, int ldz, int r0, int r1, int n, int batch,
                                  hipStream_t st) {
  if (r1 <= r0 || batch <= 0) return hipSuccess;
  hipLaunchKernelGGL(trmv_kernel, dim3(gp_ceil_div(r1 - r0, 64), batch), dim3(1024), 0, st,
                     Linv, ld, sL, w, ldw, z, ldz, r0, r1, n);
  return hipGetLastError();
}

hipError_t gpfit_trmv_launch(const double* Linv, int ld, long long sL, const double* w,
                             int ldw, double* z, int ldz, int rows, int n, int batch,
                             hipStream_t st) {
  return gpfit_trmv_rows_launch(Linv, ld, sL, w, ldw, z, ldz, 0, rows, n, batch, st);
}

extern "C" int gp_trmv(const double* Linv, int ldinv, long long strideInv, int n,
                       const double* w, int ldw, double* z, int ldz, int batch,
                       hipStream_t stream) {
  if (!Linv) return -1;
  if (ldinv < n || ldinv < 1) return -2;
  if (batch > 1 && strideInv < (long long)ldinv * n) return -3;
  if (n < 0) return -4;
  if (!w) return -5;
  if (ldw < n && batch > 1) return -6;
  if (!z) return -7;
  if (ldz < n && batch > 1) return -8;
  if (batch < 0) return -9;
  if (n == 0 || batch == 0) return 0;
  hipError_t e = gpfit_trmv_launch(Linv, ldinv, strideInv, w, ldw, z, ldz, n, n, batch, stream);
  return e == hipSuccess ? 0 : GPFIT_ERR_HIP - (int)e;
}

extern "C" int gp_nll(const double* Linv, int ldinv, long long strideInv, int n,
                      const double* w, int ldw, const double* logdet, double* nll,
                      double* work, int batch, hipStream_t stream) {
  if (!Linv) return -1;
  if (ldinv < n || ldinv < 1) return -2;
  if (batch > 1 && strideInv < (long long)ldinv * n) return -3;
  if (n < 0) return -4;
  if (!w) return -5;
  if (ldw < n && batch > 1) return -6;
  if (!logdet) return -7;
  if (!nll) return -8;
  if (!work) return -9;
  if (batch < 0) return -10;
  if (n == 0 || batch == 0) return 0;
  hipError_t e = gpfit_trmv_launch(Linv, ldinv, strideInv, w, ldw, work, n, n, n, batch, stream);
  if (e != hipSuccess) return GPFIT_ERR_HIP - (int)e;
  hipLaunchKernelGGL(nll_reduce_kernel, dim3(batch), dim3(256), 0, stream, work, n, n, logdet,
                     (const int*)nullptr, 1.0, nll, (int*)nullptr, (int*)nullptr);
  e = hipGetLastError();
  return e == hipSuccess ? 0 : GPFIT_ERR_HIP - (int)e;
}

namespace {
struct LoglikWs {
  double* G;
  double* Linv;      // L^-1 path: L^-1; in-chain path: the diagonal inverses D_j
  double* z;
  double* zb;        // in-chain path: z_j and the DP tasks' partial sums (2 npad per problem)
  double* zz;        // in-chain path: sum z^2 per problem
  double* logdet;
  int* info;
  int* status;       // sticky internal-error word (gp_loglik_status)
  char* pot;         // the factorisation's scratch
  long long pot_bytes;
  long long bytes;
};

LoglikWs loglik_carve(void* ws, int n, int batch) {
  const long long npad = gp_padded_n(n);
  auto up = [](long long b) { return (b + 255) & ~255LL; };
  LoglikWs w;
  char* p = static_cast<char*>(ws);
  long long off = 0;
  w.G = reinterpret_cast<double*>(p + off);
  off += up(8LL * batch * n * n);
  w.Linv = reinterpret_cast<double*>(p + off);
  off += up(8LL * batch * npad * npad);
  w.z = reinterpret_cast<double*>(p + off);
  off += up(8LL * batch * n);
  w.zb = reinterpret_cast<double*>(p + off);
  off += up(8LL * batch * 2 * npad);
  w.zz = reinterpret_cast<double*>(p + off);
  off += up(8LL * batch);
  w.logdet = reinterpret_cast<double*>(p + off);
  off += up(8LL * batch);
  w.info = reinterpret_cast<int*>(p + off);
  off += up(4LL * batch);
  w.status = reinterpret_cast<int*>(p + off);
  off += 256;
  w.pot = p + off;
  w.pot_bytes = gpfit_potrf_inv_ws_bytes(n, batch);
  if (gpfit_potrf_loglik_ws_bytes(n, batch) > w.pot_bytes)
    w.pot_bytes = gpfit_potrf_loglik_ws_bytes(n, batch);
  off += up(w.pot_bytes);
  w.bytes = off;
  return w;
}
}  // namespace

extern "C" long long gp_loglik_ws_bytes(int n, int batch) {
  if (n < 0 || batch < 0) return -1;
  return loglik_carve(nullptr, n, batch).bytes;
}

extern "C" int gp_loglik(const double* X, int n, int d, int ldx, const double* beta,
                         int ldbeta, const double* s, const double* delta, const double* w,
                         int ldw, int batch, void* ws, long long ws_bytes, double* ll,
                         int* info, hipStream_t stream) {
  if (!X) return -1;
  if (n < 0) return -2;
  if (d < 1) return -3;
  if (ldx < d) return -4;
  if (!beta) return -5;
  if (ldbeta < d) return -6;
  if (!s) return -7;
  if (!delta) return -8;
  if (!w) return -9;
  if (ldw < n && batch > 1) return -10;
  if (batch < 0) return -11;
  if (n == 0 || batch == 0) return 0;
  if (!ws || (reinterpret_cast<uintptr_t>(ws) & 255)) return -12;
  const LoglikWs c = loglik_carve(ws, n, batch);
  if (ws_bytes < c.bytes) return -13;
  if (!ll) return -14;
  const int npad = gp_padded_n(n);
  // In-chain path (the persistent factorisation's range): Gram -> factorisation whose chain
  // also solves z = L^-1 w by forward substitution over its diagonal inverses and writes ll
  // itself -- no L^-1 tasks, no trmv, no reduction launch (the fit's 24 x 512 gp_loglik: see
  // DESIGN.md "Metropolis fit").  The Gram is enqueued after the schedule kernel, as in
  // gp_fit_predict.
  struct GramArgs {
    const double *X, *beta, *s, *delta;
    double* G;
    int n, d, ldx, ldbeta, batch;
    hipStream_t st;
  } ga{X, beta, s, delta, c.G, n, d, ldx, ldbeta, batch, stream};
  GpfitPre pre;
  pre.arg = &ga;
  pre.fn = [](void* a) -> int {
    const GramArgs& g = *static_cast<const GramArgs*>(a);
    return gpfit_gram_lower(g.X, g.n, g.d, g.ldx, g.beta, g.ldbeta, g.s, g.delta, g.G, g.n,
                            (long long)g.n * g.n, g.batch, g.st);
  };
  int rc = gpfit_potrf_loglik(c.G, n, (long long)n * n, c.Linv, (long long)npad * npad, w,
                              batch > 1 ? ldw : n, c.zb, 2 * npad, c.zz, batch, c.info,
                              c.logdet, ll, c.status, info, c.pot, c.pot_bytes, stream, pre);
  if (rc <= 0) return rc;
  rc = gpfit_gram_lower(X, n, d, ldx, beta, ldbeta, s, delta, c.G, n, (long long)n * n,
                        batch, stream);
  if (rc) return rc;
  rc = gpfit_potrf_inv_event(c.G, n, n, (long long)n * n, c.Linv, npad, (long long)npad * npad,
                             batch, c.info, c.logdet, c.pot, c.pot_bytes, stream, -1, nullptr);
  if (rc) return rc;
  hipError_t e = gpfit_trmv_launch(c.Linv, npad, (long long)npad * npad, w, ldw, c.z, n, n, n,
                                   batch, stream);
  if (e != hipSuccess) return GPFIT_ERR_HIP - (int)e;
  hipLaunchKernelGGL(nll_reduce_kernel, dim3(batch), dim3(256), 0, stream, c.z, n, n, c.logdet,
                     (const int*)c.info, -1.0, ll, c.status, info);
  e = hipGetLastError();
  if (e != hipSuccess) return GPFIT_ERR_HIP - (int)e;
  return 0;
}

extern "C" int gp_loglik_status(void* ws, int n, int batch, int reset, hipStream_t stream) {
  if (!ws) return -1;
  if (n < 0) return -2;
  if (batch < 0) return -3;
  if (n == 0 || batch == 0) return 0;
  const LoglikWs c = loglik_carve(ws, n, batch);
  int host = 0;
  hipError_t e = hipMemcpyAsync(&host, c.status, sizeof(int), hipMemcpyDeviceToHost, stream);
  if (e == hipSuccess && reset) e = hipMemsetAsync(c.status, 0, sizeof(int), stream);
  if (e == hipSuccess) e = hipStreamSynchronize(stream);
  if (e != hipSuccess) return GPFIT_ERR_HIP - (int)e;
  return host ? GPFIT_ERR_INTERNAL : 0;
}
