/*
 * libgpfit — MI355X (gfx950) fp64 Gaussian-process fit/predict kernels behind a C ABI.
 *
 * Drop-in boundary for timghill/GladsGP's GP hot path.  The reference is pure Python: its GP
 * arithmetic lives in the un-vendored SEPIA fork (requirements-cc.txt:55) and GPmodule
 * (requirements-cc.txt:20), called from src/model.py and the analysis drivers.  There is no FFI
 * in the reference, so each entry point below names the reference call it replaces; the
 * Python-side binding is gladsgp_amd/_capi.py (ctypes) and is shown in INTEGRATION.md.
 *
 * Conventions (all entry points):
 *  - every pointer is caller-owned DEVICE memory.  The library allocates nothing persistent:
 *    workspaces are sized by the *_ws_bytes() functions and passed in (256-byte aligned); the
 *    only library-owned objects are the streams/events of an explicit gp_ctx (gp_ctx_create /
 *    gp_ctx_destroy).  The two convenience forms gp_potrf_inv and gp_potrf take no workspace
 *    and use stream-ordered scratch of gp_potrf_inv_ws_bytes / gp_potrf_ws_bytes bytes instead
 *    (hipMallocAsync / hipFreeAsync inside the call, freed on every path); their _ws forms and
 *    every other entry point allocate nothing;
 *  - matrices are column-major with a leading dimension (LAPACK layout), element (i,j) at
 *    A[i + j*ld]; design matrices X (n x d) are row-major with row stride ldx >= d;
 *  - beta holds ARD precisions, beta >= 0 (the kernels take sqrt(beta); a negative entry
 *    yields NaN, which the factorisation reports through info);
 *  - `batch` independent problems share X / Xs; per-problem operands advance by the given
 *    stride (matrices), by ldbeta (beta rows), by 1 (s, delta, s_pred, info, logdet) and by
 *    ldw / ldo (w_hat, mean, var columns);
 *  - stream-ordered and asynchronous on `stream`; no host synchronisation, so calls can be
 *    captured into a hipGraph;
 *  - return 0 on success, -k when argument k is invalid (LAPACK style), or
 *    GPFIT_ERR_HIP - hipError_t for a launch failure.  A non-positive-definite pivot is not an
 *    error return: it is reported per problem in info[b] (LAPACK potrf semantics); info[b] = -1
 *    reports an internal error of the factorisation (a bounded wait of the persistent kernel
 *    gave up), never a pivot: the problem's outputs are then unspecified.
 */
#ifndef GPFIT_H
#define GPFIT_H

#include <hip/hip_runtime_api.h>

#ifdef __cplusplus
extern "C" {
#endif

#define GPFIT_ERR_HIP (-1000)
#define GPFIT_ERR_RCCL (-3000)  /* gp_comm_*: GPFIT_ERR_RCCL - ncclResult_t; RCCL not loadable */
#define GPFIT_ERR_INTERNAL (-2000)  /* a factorisation reported info = -1 (gp_loglik_status) */
#define GPFIT_MAX_DIM 32      /* largest input dimension d supported by the kernels      */
#define GPFIT_TILE 128        /* row padding of the L^-1 buffer (predict MFMA tile edge) */

/* Library version (major*10000 + minor*100 + patch). */
int gp_version(void);

/* Rows/columns of the L^-1 buffer gp_potrf_inv fills: n rounded up to GPFIT_TILE. */
int gp_padded_n(int n);

/*
 * ARD squared-exponential Gram with jitter, per problem b:
 *   G_b[i + j*ldg] = s[b] * exp(-sum_k beta_b[k] (X[i,k] - X[j,k])^2) + delta[b] * (i == j)
 * Replaces SEPIA SepiaDistCov.compute_cov_mat(beta, lamz, lams) (s = 1/lamUz,
 * delta = 1/lamWs + 1/(lamWOs*LamSim)) as used by SepiaModel.logLik and
 * SepiaEmulatorPrediction (src/model.py:106, analysis/time_predictions.py:76), the explicit
 * Gram of examples/01_Gaussian_random_fields.ipynb:135-141 and GPmodule's
 * squared_exponential (examples/02_univariate_GP_regression.ipynb:80).
 */
int gp_gram_ardse(const double* X, int n, int d, int ldx,
                  const double* beta, int ldbeta, const double* s, const double* delta,
                  double* G, int ldg, long long strideG, int batch, hipStream_t stream);

/*
 * Cross-covariance, transposed so each test point's column is contiguous:
 *   Kt_b[i + j*ldk] = s[b] * exp(-sum_k beta_b[k] (X[i,k] - Xs[j,k])^2),  i < n, j < m.
 * Replaces the Kvec / SigWWb cross-covariance of SepiaEmulatorPrediction and
 * examples/02...ipynb:226.
 */
int gp_cross_ardse(const double* X, int n, int ldx, const double* Xs, int m, int ldxs, int d,
                   const double* beta, int ldbeta, const double* s,
                   double* Kt, int ldk, long long strideK, int batch, hipStream_t stream);

/*
 * Blocked Cholesky with simultaneous triangular inverse, per problem b:
 *   A_b = L_b L_b^T (L_b overwrites the lower triangle of A_b; the strict upper triangle is
 *   left untouched, as LAPACK dpotrf('L')), Linv_b = L_b^-1 (lower; the upper triangle and the
 *   padding rows/cols n..gp_padded_n(n)-1 are zeroed), logdet[b] = log|A_b| = 2 sum log L_ii,
 *   info[b] = 0, or j (1-based) when the leading minor of order j is not positive definite
 *   (then L_b / Linv_b / logdet[b] are unspecified), or -1 for an internal error (above).
 * Linv_b needs ldinv >= gp_padded_n(n) and gp_padded_n(n) columns.  info / logdet may be NULL.
 * Replaces the dense SPD factorisation / solve inside SEPIA's likelihood and prediction
 * (LAPACK potrf/gesv), scipy.linalg.cholesky in examples/01...ipynb:66,144 and GPmodule's
 * K_inv (examples/02...ipynb:232).
 * gp_potrf_inv_ws is the same with caller-owned scratch `ws` of gp_potrf_inv_ws_bytes(n, batch)
 * bytes (the persistent factorisation's task list and flags; 0 bytes when n is beyond its
 * range); gp_potrf_inv allocates that scratch stream-ordered itself.
 */
long long gp_potrf_inv_ws_bytes(int n, int batch);
int gp_potrf_inv_ws(double* A, int n, int lda, long long strideA,
                    double* Linv, int ldinv, long long strideInv,
                    int batch, int* info, double* logdet, void* ws, long long ws_bytes,
                    hipStream_t stream);
int gp_potrf_inv(double* A, int n, int lda, long long strideA,
                 double* Linv, int ldinv, long long strideInv,
                 int batch, int* info, double* logdet, hipStream_t stream);

/*
 * Plain blocked Cholesky, LAPACK dpotrf('L') per problem: A_b = L_b L_b^T with L_b in the lower
 * triangle of A_b (strict upper triangle untouched), logdet[b] = log|A_b|, info[b] = 0 or the
 * 1-based order of the first non-positive-definite leading minor.  Same sweep and arithmetic as
 * gp_potrf_inv without the inverse (L is bit-identical to gp_potrf_inv's).  info / logdet may
 * be NULL.  Replaces the factorisation SURVEY §8b names gp_potrf (LAPACK potrf inside SEPIA's
 * likelihood, scipy.linalg.cholesky in examples/01...ipynb:66,144).  gp_potrf_ws takes the
 * scratch (the D_k = L_kk^-1 blocks and the persistent kernel's task list / flags) from the
 * caller: gp_potrf_ws_bytes(n, batch) bytes.
 */
long long gp_potrf_ws_bytes(int n, int batch);
int gp_potrf_ws(double* A, int n, int lda, long long strideA, int batch, int* info,
                double* logdet, void* ws, long long ws_bytes, hipStream_t stream);
int gp_potrf(double* A, int n, int lda, long long strideA, int batch, int* info,
             double* logdet, hipStream_t stream);

/*
 * Triangular inverse of a lower Cholesky factor, LAPACK dtrtri('L','N') into a padded buffer:
 * Linv_b = L_b^-1 (lower; upper triangle and padding to gp_padded_n(n) zeroed), so a caller
 * that already holds a LAPACK factor can call gp_predict without re-factorising.  info[b] =
 * 0, or the 1-based index of the first zero (or non-finite) diagonal entry (then Linv_b is
 * unspecified).  info may be NULL.
 */
int gp_trtri(const double* L, int n, int ldl, long long strideL, double* Linv, int ldinv,
             long long strideInv, int batch, int* info, hipStream_t stream);

/* Bytes of device workspace gp_predict needs for (n, m, batch) with test-point chunk m_chunk
 * (0 = library default).  Workspace contents are scratch (no state between calls).         */
long long gp_predict_ws_bytes(int n, int m, int batch, int m_chunk);

/*
 * Posterior mean and marginal variance of `batch` GPs at m test points:
 *   z_b = Linv_b w_b,  V = Linv_b Kt_b (never stored),
 *   mean_b[j] = sum_i V[i,j] z_b[i]          = k*_j^T A_b^-1 w_b
 *   var_b[j]  = s_pred[b] - sum_i V[i,j]^2   = s_pred[b] - k*_j^T A_b^-1 k*_j
 * with w_b = w_hat + b*ldw (n values), mean_b = mean + b*ldo, var_b = var + b*ldo (m values).
 * Linv comes from gp_potrf_inv with the same X, beta, s.  Replaces SepiaEmulatorPrediction's
 * predictive mean / covariance diagonal (analysis/time_predictions.py:76-78,
 * assess_all_models.py:489, sensitivity_indices.py:85) and examples/02...ipynb:232-233.
 */
int gp_predict(const double* Linv, int ldinv, long long strideInv,
               const double* X, int ldx, const double* Xs, int ldxs, int n, int m, int d,
               const double* beta, int ldbeta, const double* s, const double* s_pred,
               const double* w_hat, int ldw, double* mean, double* var, int ldo,
               int batch, void* ws, long long ws_bytes, int m_chunk, hipStream_t stream);

/*
 * gp_predict with the L^-1 layout and z = L^-1 w as options (the sharded single-GP path,
 * ranks >= 1 predict straight from the broadcast payload, no unpack and no trmv):
 *   layout GPFIT_LINV_PADDED: Linv as gp_predict (column k at Linv + k*ldinv);
 *   layout GPFIT_LINV_PACKED: Linv tile-packed (gp_pack_linv), ldinv ignored, strideInv >=
 *          gp_linv_packed_elems(n) between problems;
 *   z != NULL: z_b = z + b*ldz (gp_padded_n(n) values, from gp_predict_z) is used as L^-1 w and
 *          w_hat is not read; z == NULL: computed as gp_predict does.
 * Results are bit-identical to gp_predict's for every layout and z option.  Argument numbers
 * 1-23 as gp_predict; -24 layout, -26 ldz.  Workspace: gp_predict_ws_bytes.
 */
#define GPFIT_LINV_PADDED 0
#define GPFIT_LINV_PACKED 1
int gp_predict_ex(const double* Linv, int ldinv, long long strideInv,
                  const double* X, int ldx, const double* Xs, int ldxs, int n, int m, int d,
                  const double* beta, int ldbeta, const double* s, const double* s_pred,
                  const double* w_hat, int ldw, double* mean, double* var, int ldo,
                  int batch, void* ws, long long ws_bytes, int m_chunk, int layout,
                  const double* z, long long ldz, hipStream_t stream);

/*
 * z_b = Linv_b w_b (gp_padded_n(n) rows, zero past n) with exactly the arithmetic gp_predict
 * applies internally, into z + b*ldz: what rank 0 ships with L^-1 so the other ranks skip it.
 * `ws` holds gp_predict_z_ws_bytes(n, batch) bytes.  layout as gp_predict_ex.
 */
long long gp_predict_z_ws_bytes(int n, int batch);
int gp_predict_z(const double* Linv, int ldinv, long long strideInv, int layout, int n,
                 const double* w_hat, int ldw, double* z, long long ldz, int batch, void* ws,
                 long long ws_bytes, hipStream_t stream);

/*
 * The tile-packed L^-1: column c of the padded buffer from row 16*floor(c/16) on (every stored
 * run starts on a 16-row tile and is a multiple of 16 doubles, so the prediction's 16-B loads
 * and 16-row MFMA tiles read it in place), columns one after another:
 * gp_linv_packed_elems(n) = npad^2 - 128 q (q - 1) doubles, q = npad / 16, npad =
 * gp_padded_n(n) -- about half the padded square (67 MB at n = 4096).  Both buffers 16-B
 * aligned; gp_unpack_linv writes only the stored elements.
 */
long long gp_linv_packed_elems(int n);
int gp_pack_linv(const double* Linv, int n, int ldinv, double* P, hipStream_t stream);
int gp_unpack_linv(const double* P, int n, double* Linv, int ldinv, hipStream_t stream);

/*
 * gp_predict from the Cholesky factor L itself (the §8b form, LAPACK layout, lower): L^-1 by
 * gp_trtri into the head of `ws`, then gp_predict.  `ws` holds
 * gp_predict_chol_ws_bytes(n, m, batch, m_chunk) bytes; info as gp_trtri (mean / var of a
 * problem with info[b] != 0 are unspecified).
 */
long long gp_predict_chol_ws_bytes(int n, int m, int batch, int m_chunk);
int gp_predict_chol(const double* L, int ldl, long long strideL,
                    const double* X, int ldx, const double* Xs, int ldxs, int n, int m, int d,
                    const double* beta, int ldbeta, const double* s, const double* s_pred,
                    const double* w_hat, int ldw, double* mean, double* var, int ldo,
                    int batch, int* info, void* ws, long long ws_bytes, int m_chunk,
                    hipStream_t stream);

/*
 * Two-phase form of gp_predict.  The cross-covariance of every test-point chunk does not depend
 * on the factorisation, so it can be built on a second stream while gp_potrf_inv runs:
 *   gp_predict_cross : Kt chunks for all m points into ws (X, Xs, beta, s only)
 *   gp_predict_solve : z = Linv w, TRMM + mean/var per chunk from the prepared ws
 * Both take the same (n, m, batch, m_chunk) and a workspace of
 * gp_predict_prepared_ws_bytes(n, m, batch, m_chunk) bytes; results equal gp_predict's.
 */
long long gp_predict_prepared_ws_bytes(int n, int m, int batch, int m_chunk);
int gp_predict_cross(const double* X, int ldx, const double* Xs, int ldxs, int n, int m, int d,
                     const double* beta, int ldbeta, const double* s, int batch,
                     void* ws, long long ws_bytes, int m_chunk, hipStream_t stream);
int gp_predict_solve(const double* Linv, int ldinv, long long strideInv, int n, int m,
                     const double* s_pred, const double* w_hat, int ldw, double* mean,
                     double* var, int ldo, int batch, void* ws, long long ws_bytes,
                     int m_chunk, hipStream_t stream);

/*
 * z_b = Linv_b w_b (lower-triangular gemv, n rows), z_b = z + b*ldz.
 * Building block of the likelihood (quadratic form w^T A^-1 w = ||z||^2).
 */
int gp_trmv(const double* Linv, int ldinv, long long strideInv, int n,
            const double* w, int ldw, double* z, int ldz, int batch, hipStream_t stream);

/*
 * GP negative log-likelihood per problem:  nll[b] = 1/2 ||Linv_b w_b||^2 + 1/2 logdet[b]
 * (no 2*pi term), with Linv / logdet from gp_potrf_inv; `work` holds batch*n doubles.
 * Replaces GPmodule's MLE objective (examples/02_univariate_GP_regression.ipynb:80-83, known
 * answer fun = -3.989954265337257 at :70-72) and the per-PC Gaussian term of SEPIA's logLik
 * evaluated by SepiaModel.do_mcmc (src/model.py:234-235).
 */
int gp_nll(const double* Linv, int ldinv, long long strideInv, int n,
           const double* w, int ldw, const double* logdet, double* nll, double* work,
           int batch, hipStream_t stream);

/*
 * Execution context of gp_fit_predict, created and destroyed by the caller on the current
 * device: one stream for the cross-covariance (the factorisation and the prediction run on the
 * caller's stream) and its events (one per test-point chunk after its cross-covariance,
 * created on the first call that needs them).
 *   cross_start  : fraction of the factorisation's n/64 block steps after which the
 *                  cross-covariance starts (< 0: default 0.4; 0 = at once);
 *   aux_free_cus : CUs the cross-covariance stream leaves to the factorisation (CU mask;
 *                  < 0: default 0 = no mask).
 * gp_ctx_destroy drains the streams and frees them; call it before the HIP runtime is torn
 * down (e.g. before process exit).  A context serves one host thread at a time.
 */
int gp_ctx_create(double cross_start, int aux_free_cus, void** ctx);
int gp_ctx_destroy(void* ctx);
/*
 * How many test-point chunks' cross-covariance gp_fit_predict runs on the context's aux stream
 * (beside the factorisation and the earlier chunks' TRMMs); the remaining chunks' run on the
 * prediction stream just before their TRMM.  -1 (default): all chunks, the C3 schedule; a batch
 * of small GPs (C4) hides one chunk beside its factorisation and keeps the rest out of the
 * TRMMs' way.  Returns 0, -1 (ctx NULL), -2 (nchunks < -1).  Results are bit-identical for
 * every value.
 */
int gp_ctx_set_aux_chunks(void* ctx, int nchunks);

/*
 * Fit + predict in one call:
 *   G = gram(X) (caller buffer, L on return) -> L, L^-1, info, logdet (as gp_potrf_inv) ->
 *   mean / var at the m test points (as gp_predict).
 * With ctx == NULL every step runs in order on `stream`.  With a context the cross-covariance
 * of every chunk forks onto the context's stream, beside the factorisation (CU-masked if
 * asked), while `stream` runs the Gram + factorisation, z = L^-1 w and per chunk, once that
 * chunk's cross-covariance is done, its TRMM, then one mean/var pass: the caller sees one
 * stream-ordered operation.  `ws` holds
 * gp_fit_predict_ws_bytes(n, m, batch, m_chunk) bytes (the factorisation's scratch included).
 * The prediction runs whatever info says: mean / var of a problem with info[b] != 0 are
 * unspecified (check info; -1 is an internal error, see the conventions).
 * Replaces the reference's fit-then-predict sequence per GP (SEPIA likelihood factorisation +
 * SepiaEmulatorPrediction, time_predictions.py:76-79) at the bench configuration.
 */
long long gp_fit_predict_ws_bytes(int n, int m, int batch, int m_chunk);
int gp_fit_predict(const double* X, int ldx, const double* Xs, int ldxs, int n, int m, int d,
                   const double* beta, int ldbeta, const double* s, const double* delta,
                   const double* s_pred, const double* w_hat, int ldw, double* G, int ldg,
                   long long strideG, double* Linv, int ldinv, long long strideInv, int* info,
                   double* logdet, double* mean, double* var, int ldo, int batch, void* ws,
                   long long ws_bytes, int m_chunk, void* ctx, hipStream_t stream);

/*
 * Batched GP log-likelihood in one stream-ordered call: Gram (gp_gram_ardse) -> Cholesky
 * (gp_potrf_inv) -> ll[b] = -(1/2 ||L_b^-1 w_b||^2 + 1/2 log|G_b|), no 2*pi term, with
 * ll[b] = -inf where G_b is not positive definite (info[b] > 0: a proposal the sampler rejects)
 * and ll[b] = NaN where the factorisation gave up (info[b] = -1), which also raises a sticky
 * status word in `ws` (info optionally copied out to `info`).  `ws` is caller-owned device
 * scratch of gp_loglik_ws_bytes(n, batch) bytes, zero-filled before its first use.  Never
 * syncs, so a Metropolis sweep can be stream-ordered (and graph-captured) end to end;
 * gp_loglik_status reads the status word afterwards (it synchronises `stream`): 0, or
 * GPFIT_ERR_INTERNAL when any gp_loglik on this workspace since the last reset had an internal
 * factorisation error; `reset` clears the word.
 * Replaces the per-PC term of SEPIA's logLik evaluated by SepiaModel.do_mcmc /
 * tune_step_sizes (src/model.py:234-235): Sigma_j = s_j R(beta_j) + delta_j I, w = w_hat_j.
 */
long long gp_loglik_ws_bytes(int n, int batch);
int gp_loglik(const double* X, int n, int d, int ldx, const double* beta, int ldbeta,
              const double* s, const double* delta, const double* w, int ldw, int batch,
              void* ws, long long ws_bytes, double* ll, int* info, hipStream_t stream);
int gp_loglik_status(void* ws, int n, int batch, int reset, hipStream_t stream);

/*
 * Metropolis sweep steps around gp_loglik (the GPU sampler's speculative groups; replaces the
 * proposal / accept logic of SEPIA's SepiaModel.do_mcmc / tune_step_sizes that src/model.py:
 * 225-235 drives).  The chain state and its priors are described by a gp_mcmc_state of device
 * pointers (row-major: betaU and step_betaU (d+1) x P; lamUz, lamWs, ll, lam, step_lamUz,
 * step_lamWs P; lamWOs, step_lamWOs 1; acc (d+4) x P acceptance counters indexed by update
 * code; u the sweep's 2 ((d+1) P + 2 P + 1) uniforms, an update's proposal uniforms then its
 * acceptance uniforms, in update order; scratch 3 * GPFIT_MCMC_MAX_GROUP * P doubles) plus the
 * prior family / parameters / bounds and step type of each of betaU, lamUz, lamWs, lamWOs.
 * Update codes: 1..d betaU row, d+1 lamUz, d+2 lamWs, d+3 lamWOs.  For a group of g updates:
 *   gp_mcmc_group_prep   proposes them (first != 0: also the prior-only move of betaU row 0)
 *                        and writes the Gram inputs of the 2^g - 1 state sets, set
 *                        2^i - 1 + pat = update i proposed after the outcomes `pat` (bit q =
 *                        update q accepted) of updates 0..i-1, rows set * P + j of beta
 *                        (x d), s and delta: the batch for gp_loglik;
 *   gp_mcmc_group_decide takes the decisions in order from gp_loglik's ll_all (per GP; lamWOs
 *                        once on the sum), updates state, ll and counters in place and
 *                        (last != 0) writes the log posterior to lp;
 *   gp_mcmc_group_step   gp_mcmc_group_decide of one group (S, kinds, g, last, ll_all) then
 *                        gp_mcmc_group_prep of the next (S_next, kinds_next, g_next, first,
 *                        beta, s, delta) in one launch (one kernel boundary less per group);
 *                        the same results as the two calls in turn.  Argument errors of the
 *                        second group are its prep's codes - 10; S_next->P must equal S->P
 *                        (-18).
 * Single-workgroup launches (P <= 1024), stream-ordered, graph-capturable; 0 or < 0 (argument).
 */
#define GPFIT_MCMC_MAX_GROUP 4
#define GPFIT_MCMC_GAMMA 0        /* (a - 1) log x - b x                                      */
#define GPFIT_MCMC_BETA 1         /* Beta(a, b) on rho = min(exp(-x / 4), 0.999)              */
#define GPFIT_MCMC_NORMAL 2       /* -1/2 ((x - a) / b)^2                                     */
#define GPFIT_MCMC_UNIFORM 3      /* 0 (the bounds)                                           */
#define GPFIT_MCMC_STEP_UNIFORM 0 /* x' = x + step (u - 1/2)                                  */
#define GPFIT_MCMC_STEP_BETARHO 1 /* the same move on rho = exp(-x / 4)                       */
typedef struct {
  double* betaU;
  double* lamUz;
  double* lamWs;
  double* lamWOs;
  double* ll;
  const double* lam;
  const double* u;
  const double* step_betaU;
  const double* step_lamUz;
  const double* step_lamWs;
  const double* step_lamWOs;
  double* acc;
  double* lp;
  double* scratch;
  int P, d;
  int dist[4];        /* per parameter: betaU, lamUz, lamWs, lamWOs */
  int steptype[4];
  double pa[4], pb[4], lo[4], hi[4];
} gp_mcmc_state;
int gp_mcmc_group_prep(const gp_mcmc_state* S, const int* kinds, int g, int first,
                       double* beta, double* s, double* delta, hipStream_t stream);
int gp_mcmc_group_decide(const gp_mcmc_state* S, const int* kinds, int g, int last,
                         const double* ll_all, hipStream_t stream);
int gp_mcmc_group_step(const gp_mcmc_state* S, const int* kinds, int g, int last,
                       const double* ll_all, const gp_mcmc_state* S_next, const int* kinds_next,
                       int g_next, int first, double* beta, double* s, double* delta,
                       hipStream_t stream);

/*
 * Host-side (no device, no stream): `count` float32 deviates of numpy's legacy global
 * generator exactly as src/svd.py:51 draws randomized_svd's test matrix,
 * np.random.normal(size=...).astype(np.float32) -- MT19937 + the polar Box-Muller method
 * (numpy's legacy_gauss), bit-identical -- continued from and advancing the caller's state:
 * key[624] / pos (np.random.get_state()[1:3]) and the cached deviate has_gauss / gauss
 * ([3:5]).  Twist and candidate tests vectorised, the accepted pairs' log / sqrt on `nthreads`
 * host threads.  Returns 0, -1 (a state pointer NULL), -2 (pos outside [0, 624]), -5 (count < 0),
 * -6 (out NULL), -7 (a host thread or buffer could not be created; the state is then
 * undefined: restore it from a copy).
 */
int gp_host_legacy_normal_f32(unsigned int* key, int* pos, int* has_gauss, double* gauss,
                              long long count, float* out, int nthreads);

/*
 * One marginal realisation per entry: out[i] = mean[i] + sqrt(max(var[i], 0)) z_i, z_i ~ N(0,1)
 * from counter-based Philox4x32-10 keyed by `seed` (counter (i/2, offset); Box-Muller pairs),
 * so the draws depend only on (seed, offset, i).  out may alias mean.  The opt-in realize mode
 * of the prediction: SepiaEmulatorPrediction's .w is a random draw of the PC weights, whose
 * spread the reference's quantile / coverage statistics use (assess_all_models.py:489-500).
 */
int gp_realize(const double* mean, const double* var, long long N, unsigned long long seed,
               unsigned long long offset, double* out, hipStream_t stream);

/* ------------------------------------------------------------------------------------------
 * Fit-side dense kernels (src/model.py init_model and src/svd.py randomized_svd).
 * ---------------------------------------------------------------------------------------- */

/* C = alpha op(A) op(B) + beta C, column-major fp64 on MFMA; op = transpose when trans = 1.
 * Large-K products are split over K into `ws` (gp_dgemm_ws_bytes(m, n, k) bytes; with a smaller
 * or NULL ws the product runs unsplit).  Replaces the numpy GEMMs of src/svd.py:52-64
 * (X Omega, X X^T Y, Q^T X, Q U) and of src/model.py:101, 219-220. */
long long gp_dgemm_ws_bytes(int m, int n, int k);
int gp_dgemm(int transa, int transb, int m, int n, int k, double alpha,
             const double* A, int lda, const double* B, int ldb, double beta,
             double* C, int ldc, void* ws, long long ws_bytes, hipStream_t stream);

/* gp_dgemm with either operand stored as float32 (a_f32 / b_f32 = 1): the float32 elements are
 * widened to fp64 as they are loaded (exactly), the products and sums are fp64, so the result
 * is bit-identical to gp_dgemm on an fp64 copy of the operand -- from half its bytes and
 * without the copy.  src/svd.py:51-64 receives the float32 ensemble of fit_models /
 * load_model (src/model.py:184, 136) and multiplies it as stored; this is that product in fp64.
 * Same workspace rule as gp_dgemm; argument numbers as listed. */
int gp_gemm_ex(int transa, int transb, int m, int n, int k, double alpha,
               const void* A, int a_f32, int lda, const void* B, int b_f32, int ldb,
               double beta, double* C, int ldc, void* ws, long long ws_bytes, hipStream_t stream);

/* Per-location statistics over simulations of a C-order ensemble Y (n x ny, row stride ldy):
 * mu = mean over rows, sd = std(ddof=1) floored at sd_floor — src/model.py:60-64. */
int gp_sim_stats(const double* Y, int n, int ny, long long ldy, double sd_floor,
                 double* mu, double* sd, hipStream_t stream);

/* out = (Y - mu) / sd (inverse = 0, src/model.py:72) or out = Y sd + mu (inverse = 1, the
 * back-transform of SepiaEmulatorPrediction.get_y), both C-order n x ny with row strides. */
int gp_standardize(const double* Y, int n, int ny, long long ldy, const double* mu,
                   const double* sd, double* out, long long ldo, int inverse,
                   hipStream_t stream);

/* Field reconstruction, SepiaEmulatorPrediction.get_y() (time_predictions.py:79-90,
 * assess_all_models.py:489-500) in one pass:
 *   Y[r*ldy + c] = ((sum_j W[r*ldw + j] K[j*ldk + c]) + err[r]) * sd[c] + mu[c]
 * for r < rows (samples x test points), c < ncols (field nodes), j < P <= gp_field_max_pcs()
 * PCs; fp64 MFMA products, the back-transform and the optional error term (one scalar per row,
 * err may be NULL) in the epilogue, stored once as float32 (out_f32 = 1, the reference's
 * .w.astype(float32) path) or fp64.  sd and mu NULL together: Y = W K (+ err), the
 * standardised field.  Equal bit for bit to gp_dgemm (K <= 64) + gp_standardize(inverse = 1)
 * + a float32 cast.  Returns -4 for P outside [1, gp_field_max_pcs()]. */
int gp_field_max_pcs(void);
int gp_field(const double* W, long long ldw, int rows, int P, const double* K, long long ldk,
             int ncols, const double* sd, const double* mu, const double* err, void* Y,
             long long ldy, int out_f32, hipStream_t stream);

/* out[0] = mean(x), out[1] = var(x, ddof) of a length-N vector (two-pass, deterministic);
 * work holds 1024 doubles.  np.var of the PC truncation residual, src/model.py:222. */
int gp_mean_var(const double* x, long long N, int ddof, double* out, double* work,
                hipStream_t stream);

/* A[i][i] += factor * trace(A) (shifted CholeskyQR); row i of M scaled by f[i] or 1/f[i]. */
int gp_shift_diag(double* A, int r, int lda, double factor, hipStream_t stream);
int gp_rowscale(double* M, int rows, int cols, int ld, const double* f, int inv,
                hipStream_t stream);

/* Symmetric eigendecomposition A = V diag(W) V^T by cyclic Jacobi (r <= 1024, one workgroup),
 * eigenvalues descending (want_sqrt = 1: W = sqrt(max(eig, 0)), the singular values when
 * A = B B^T); A is destroyed.  `sweeps` (device int, may be NULL) receives the sweep count.
 * The r x r core of np.linalg.svd(B) in src/svd.py:63 (via B B^T). */
int gp_syevj(double* A, int r, int lda, double* W, double* V, int ldv, int max_sweeps,
             double tol, int* sweeps, int want_sqrt, hipStream_t stream);

/* ------------------------------------------------------------------------------------------
 * RCCL over xGMI for the sharded emulator: one communicator per process /
 * GPU.  The (sample, PC) GPs are independent, so the only exchanges are one broadcast of the
 * inputs (X, X*, w_hat, hyperparameters) from rank 0 and one gather of the (mean, var) shards
 * to rank 0.  librccl is opened at run time (dlopen); where it cannot be loaded these return
 * GPFIT_ERR_RCCL and the rest of the library is unaffected.  The reference has no distributed
 * code: a C caller uses these instead of torch.distributed (gladsgp_amd.dist.NativeComm).
 *   gp_comm_unique_id: rank 0 writes the 128-byte id every rank passes to gp_comm_init (the
 *                      caller ships it out of band);
 *   gp_bcast:          `bytes` from `root`'s buf to every rank's buf (stream-ordered);
 *   gp_gather:         every rank's `bytes` at `send` land at recv + rank * bytes on `root`.
 * ---------------------------------------------------------------------------------------- */
int gp_comm_available(void);
int gp_comm_unique_id(void* id128);
int gp_comm_init(int nranks, int rank, const void* id128, void** comm);
int gp_comm_destroy(void* comm);
int gp_bcast(void* comm, void* buf, long long bytes, int root, hipStream_t stream);

/* Lower triangle of a column-major n x n matrix (leading dimension ld; column c from row c
 * on) to / from a contiguous vector of n (n + 1) / 2 doubles, column after column (round 4's
 * single-GP broadcast payload; the payload is now gp_pack_linv's tile-packed layout, which the
 * prediction reads in place).
 * gp_unpack_tril writes only the lower triangle (the strict upper part of A is left as it
 * is: zero in a buffer prepared for gp_predict). */
int gp_pack_tril(const double* A, int n, int ld, double* out, hipStream_t stream);
int gp_unpack_tril(const double* in, int n, double* A, int ld, hipStream_t stream);
int gp_gather(void* comm, const void* send, long long bytes, void* recv, int root,
              hipStream_t stream);

/*
 * Optional kernel timing (diagnostics; not part of the reference surface).  When enabled with
 * capacity > 0, instrumented launches record a hipEvent pair on their own stream; after the
 * stream has drained, gp_profile_read returns the number of recorded launches of kernel `id`
 * and their summed / largest device time in milliseconds.  A run of back-to-back launches of
 * one kernel on one stream (gp_fit_predict's and gp_predict_solve's TRMM chunks, the cross-
 * covariance chunks) is bracketed by one pair and counted as that many launches, so the
 * events do not add stream time between them; `max_ms` is then the largest per-launch mean of
 * a run.  Host-side, single-threaded use.
 */
#define GP_PROF_GRAM 0        /* gram / cross-covariance build (ardse_kernel)            */
#define GP_PROF_POTRF 1       /* whole gp_potrf_inv sequence                             */
#define GP_PROF_TRMM 2        /* predict: trmm_pair_kernel (dominant kernel)             */
#define GP_PROF_CROSS 3       /* predict: per-chunk cross-covariance build               */
#define GP_PROF_NUM 4
int gp_profile_enable(int capacity);
/* Which kernels record (bit GP_PROF_* set; default all): a timed run can keep only the
 * dominant kernel's event pair on the critical path.  Returns the previous mask. */
unsigned gp_profile_select(unsigned mask);
int gp_profile_reset(void);
int gp_profile_read(int id, int* count, double* total_ms, double* max_ms);

/* Test / diagnostics hook, process-wide (the library's one mutable setting): the number of
 * polls a wait of the persistent factorisation makes before it gives up and reports info = -1
 * for the launches enqueued afterwards.  polls > 0 sets it, 0 restores the default (2^22, far
 * beyond any legitimate wait), < 0 makes every later factorisation start with its problems
 * given up (info = -1 deterministically: the tests of the internal-error path).  The value
 * is read when a factorisation is enqueued, so a captured HIP graph keeps the one it was
 * captured with.  Returns the previous setting. */
long long gp_set_poll_budget(long long polls);

/* Test / A-B hook, process-wide: the factorisation path of gp_potrf_inv / gp_potrf /
 * gp_fit_predict / gp_loglik enqueued afterwards.  0 = automatic (the persistent dataflow
 * kernel where eligible -- with per-XCD task queues for batches that are multiples of 8 --,
 * else the blocked sweep), 1 = always the blocked right-looking sweep, 2 = the persistent
 * kernel with one shared task queue for every batch.  Returns the previous setting. */
int gp_set_potrf_path(int path);

/* A-B hook, process-wide: the prediction path of gp_predict / gp_predict_ex / gp_fit_predict /
 * gp_predict_solve enqueued afterwards.  0 = automatic (at gp_padded_n(n) <= 512 the
 * column-resident kernel, the cross-covariance produced inside it when d <= 8 and read from
 * materialised chunks otherwise; above, cross-covariance chunks + the row-pair TRMM), 1 = always
 * cross-covariance chunks + the row-pair TRMM, 2 = the column-resident kernel from materialised
 * chunks at every d.  Paths 0 and 2 give the same bits; path 1 agrees to rounding.  Returns the
 * previous setting.  (Python: GPFIT_TRMM_RES=0 / 2 in the environment sets 1 / 2 at load.) */
int gp_set_predict_path(int path);

#ifdef __cplusplus
}
#endif
#endif /* GPFIT_H */
