// Internal (non-exported) entry points shared between the library's translation units.
#pragma once
#include <hip/hip_runtime.h>

// z_b[r] = sum_{k<=r, k<n} Linv_b[r,k] w_b[k] for r0 <= r < r1   (linalg.hip)
hipError_t gpfit_trmv_rows_launch(const double* Linv, int ld, long long sL, const double* w,
                                  int ldw, double* z, int ldz, int r0, int r1, int n, int batch,
                                  hipStream_t st);
hipError_t gpfit_trmv_launch(const double* Linv, int ld, long long sL, const double* w,
                             int ldw, double* z, int ldz, int rows, int n, int batch,
                             hipStream_t st);

constexpr int GPFIT_POTRF_NB = 64;   // column block of gp_potrf_inv (chol.hip NB)

// gp_potrf_inv_ws that also records `ev` on the stream once block step `k_ev` (NB = 64
// columns) has been enqueued (k_ev clamped to the last step); chol.hip.  Lets a caller start
// HBM-bound side work only when the factorisation turns latency-bound.  `ws` (256-B aligned)
// holds gpfit_potrf_inv_ws_bytes(n, batch) bytes: the persistent factorisation's task list and
// flags (nothing when n is beyond the persistent kernel's range).
// `pre` (optional) is enqueued on `stream` ahead of the factorisation proper -- on the
// persistent path after its schedule kernel (which reads nothing of A), so a caller can put the
// Gram that produces A there and the schedule kernel's host-side setup no longer sits between
// the Gram and the factorisation (gp_fit_predict).  A non-zero return aborts with that code.
struct GpfitPre {
  int (*fn)(void*) = nullptr;
  void* arg = nullptr;
};
int gpfit_potrf_inv_event(double* A, int n, int lda, long long strideA, double* Linv,
                          int ldinv, long long strideInv, int batch, int* info, double* logdet,
                          void* ws, long long ws_bytes, hipStream_t stream, int k_ev,
                          hipEvent_t ev, GpfitPre pre = GpfitPre());
long long gpfit_potrf_inv_ws_bytes(int n, int batch);

// gp_gram_ardse writing only the lower triangle (j <= i); the upper triangle is left untouched.
// For callers that factorise the result right away (gram.hip).
int gpfit_gram_lower(const double* X, int n, int d, int ldx, const double* beta, int ldbeta,
                     const double* s, const double* delta, double* G, int ldg,
                     long long strideG, int batch, hipStream_t stream);

// gp_loglik on the persistent factorisation's in-chain mode (chol.hip): G (lower triangle,
// strideG per problem, ld = n) factorised without L^-1; the chain solves z = L^-1 w by forward
// substitution over its diagonal inverses D_j (D: NB x NB N doubles per problem, strideD) with
// the DP tasks' partial sums, and the last workgroup writes ll = -(1/2 |z|^2 + 1/2 logdet)
// (-inf / NaN + status as nll_reduce) and info_out.  zb holds 2 NB N doubles per problem (zld),
// zz one double per problem.  Returns 1 (nothing enqueued) when the persistent kernel does not
// take (n, batch): the caller runs its L^-1 path.  `pre` (the Gram) as gpfit_potrf_inv_event.
long long gpfit_potrf_loglik_ws_bytes(int n, int batch);
int gpfit_potrf_loglik(double* G, int n, long long strideG, double* D, long long strideD,
                       const double* w, int ldw, double* zb, int zld, double* zz, int batch,
                       int* info, double* logdet, double* ll, int* status, int* info_out,
                       void* ws, long long ws_bytes, hipStream_t stream,
                       GpfitPre pre = GpfitPre());
