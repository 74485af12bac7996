// Metropolis sweep steps of the GPU sampler (gladsgp_amd.mcmc.GPUSampler), replacing SEPIA's
// SepiaModel.do_mcmc / tune_step_sizes sweep as src/model.py:225-235 drives it.
//
// A sweep is component-wise Metropolis over mcmcList (betaU row by row, lamUz, lamWs, lamWOs).
// The sampler takes the likelihood-changing updates in speculative groups of g: ONE batched
// gp_loglik evaluates update i's proposal at each of the 2^i outcomes of the group's earlier
// updates (state set 2^i - 1 + pat, pat = bit j set when update j was accepted), and the
// decisions are then taken in order.  Around each gp_loglik this file puts two single-workgroup
// kernels (thread j = principal component j):
//   gp_mcmc_group_prep    proposals of the group's updates (and, for the sweep's first group,
//                         the prior-only move of betaU row 0), then the Gram inputs
//                         (beta, s = 1/lamUz, delta = 1/lamWs + 1/(lamWOs LamSim)) of every
//                         state set
//   gp_mcmc_group_decide  the accept / reject decisions in order (per GP; lamWOs once for all
//                         on the sum), state, per-GP likelihood and acceptance counters in place,
//                         and for the sweep's last group the log posterior
//   gp_mcmc_group_step    one group's decide and the next group's prep in one launch
// They replace some 100 elementwise launches per group of the tensor-op form of the same sweep
// (mcmc.py _sweep_torch, kept as the host-logic reference the CPU tests run).  Arithmetic is
// op-for-op that form's (no FMA contraction), so the chains agree with it and with the oracle
// (oracle/mcmc_ref.py) fed the same uniforms.
#include "gpfit_common.h"
#include "../../include/gpfit.h"

#pragma clang fp contract(off)

namespace {

constexpr double kRhoMax = 0.999;   // rho clipped in the Beta prior (mcmc.RHO_MAX)
constexpr int kLpTerms = 2048;      // log-posterior terms computed one per thread (LDS)

struct GroupArgs {
  gp_mcmc_state S;
  int kinds[GPFIT_MCMC_MAX_GROUP];
  int g;
  int flag;            // prep: first group of the sweep; decide: last group
};

// parameter index of an update code (1..d: betaU row, d+1 lamUz, d+2 lamWs, d+3 lamWOs; 0 is
// betaU row 0)
GP_DEV int param_of(int code, int d) { return code <= d ? 0 : code - d; }

GP_DEV double log_prior(const gp_mcmc_state& S, int p, double x) {
  const double a = S.pa[p], b = S.pb[p];
  switch (S.dist[p]) {
    case GPFIT_MCMC_GAMMA:
      return (a - 1.0) * log(x) - b * x;
    case GPFIT_MCMC_BETA: {
      const double rho = fmin(exp(-x / 4.0), kRhoMax);
      return (a - 1.0) * log(rho) + (b - 1.0) * log1p(-rho);
    }
    case GPFIT_MCMC_NORMAL: {
      const double t = (x - a) / b;
      return -0.5 * (t * t);
    }
    default:
      return 0.0;
  }
}

// current value, step and uniforms of update `code` for element j (j = 0 for lamWOs)
GP_DEV void update_refs(const gp_mcmc_state& S, int code, int j, double*& cur, double& step,
                        double& up, double& ua) {
  const int P = S.P, d = S.d;
  const long long off = 2LL * P * code;
  if (code <= d) {
    cur = S.betaU + (long long)code * P + j;
    step = S.step_betaU[(long long)code * P + j];
  } else if (code == d + 1) {
    cur = S.lamUz + j;
    step = S.step_lamUz[j];
  } else if (code == d + 2) {
    cur = S.lamWs + j;
    step = S.step_lamWs[j];
  } else {
    cur = S.lamWOs;
    step = S.step_lamWOs[0];
    up = S.u[off];
    ua = S.u[off + 1];
    return;
  }
  up = S.u[off + j];
  ua = S.u[off + P + j];
}

// proposal of parameter p from x (mcmc.propose): candidate (x when rejected by the bounds or
// rho's range), in-bounds flag and the prior difference
GP_DEV void propose(const gp_mcmc_state& S, int p, double x, double step, double up,
                    double& cand, bool& ok, double& dlp) {
  if (S.steptype[p] == GPFIT_MCMC_STEP_BETARHO) {
    const double rho = exp(-x / 4.0) + step * (up - 0.5);
    ok = (rho > 0.0) && (rho <= 1.0);
    cand = -4.0 * log(ok ? rho : 1.0);
  } else {
    cand = x + step * (up - 0.5);
    ok = true;
  }
  ok = ok && (cand >= S.lo[p]) && (cand <= S.hi[p]);
  cand = ok ? cand : x;
  dlp = log_prior(S, p, cand) - log_prior(S, p, x);
}

GP_DEV void prep_body(const GroupArgs& A, double* __restrict__ beta, double* __restrict__ s,
                      double* __restrict__ delta) {
  const gp_mcmc_state& S = A.S;
  const int j = threadIdx.x, P = S.P, d = S.d;
  double* cand = S.scratch;                               // [i][P]
  double* okf = S.scratch + GPFIT_MCMC_MAX_GROUP * P;
  double* dlp = S.scratch + 2 * GPFIT_MCMC_MAX_GROUP * P;
  // The prior-only move of betaU row 0 and the group's g proposals are independent (each reads
  // the current state of its own element only; the Gram inputs below never read row 0), so
  // thread t runs row 0's element t (t < P) or update t / P - 1's element t % P: one chain of
  // fp64 exp / log per thread instead of up to g + 1 in turn (the kernel was 9.6-10.6 us,
  // profiles/r05/r05_prof_fit2.txt).  The same arithmetic per element, so the same bits.
  for (int t = j; t < (A.g + 1) * P; t += blockDim.x) {
    const int i = t / P - 1, e = t - (t / P) * P;
    if (i < 0) {                                          // betaU row 0: prior only
      if (!A.flag) continue;
      double *cur, step, up, ua;
      update_refs(S, 0, e, cur, step, up, ua);
      double c, dl;
      bool ok;
      propose(S, 0, *cur, step, up, c, ok, dl);
      const bool acc = ok && (log(ua) < dl);
      if (acc) *cur = c;
      S.acc[e] += acc ? 1.0 : 0.0;
      continue;
    }
    const int code = A.kinds[i];
    if (code == d + 3 && e > 0) continue;                 // lamWOs: one element
    double *cur, step, up, ua;
    update_refs(S, code, e, cur, step, up, ua);
    double c, dl;
    bool ok;
    propose(S, param_of(code, d), *cur, step, up, c, ok, dl);
    cand[i * P + e] = c;
    okf[i * P + e] = ok ? 1.0 : 0.0;
    dlp[i * P + e] = dl;
  }
  __syncthreads();
  if (j >= P) return;
  const double lam = S.lam[j];
  for (int i = 0; i < A.g; ++i) {
    for (int pat = 0; pat < (1 << i); ++pat) {
      const int slot = (1 << i) - 1 + pat;
      const long long row = (long long)slot * P + j;
      double lUz = S.lamUz[j], lWs = S.lamWs[j], lWO = S.lamWOs[0];
      for (int r = 1; r <= d; ++r) {
        double v = S.betaU[(long long)r * P + j];
        for (int q = 0; q <= i; ++q)
          if ((q == i || ((pat >> q) & 1)) && A.kinds[q] == r) v = cand[q * P + j];
        beta[row * d + (r - 1)] = v;
      }
      for (int q = 0; q <= i; ++q) {
        if (!(q == i || ((pat >> q) & 1))) continue;
        const int code = A.kinds[q];
        if (code == d + 1) lUz = cand[q * P + j];
        else if (code == d + 2) lWs = cand[q * P + j];
        else if (code == d + 3) lWO = cand[q * P];
      }
      s[row] = 1.0 / lUz;
      delta[row] = 1.0 / lWs + 1.0 / (lWO * lam);
    }
  }
}

GP_DEV void decide_body(const GroupArgs& A, const double* __restrict__ ll_all) {
  const gp_mcmc_state& S = A.S;
  const int j = threadIdx.x, P = S.P, d = S.d;
  const double* cand = S.scratch;
  const double* okf = S.scratch + GPFIT_MCMC_MAX_GROUP * P;
  const double* dlp = S.scratch + 2 * GPFIT_MCMC_MAX_GROUP * P;
  __shared__ double sh[1024];
  __shared__ int sh_acc;
  int pat = 0;
  for (int i = 0; i < A.g; ++i) {
    const int code = A.kinds[i];
    const double lln = j < P ? ll_all[((long long)(1 << i) - 1 + pat) * P + j] : 0.0;
    bool acc = false;
    if (code == d + 3) {                       // lamWOs: one decision on the sum over GPs
      if (j < P) sh[j] = lln - S.ll[j];
      __syncthreads();
      if (j == 0) {
        double sum = 0.0;
        for (int q = 0; q < P; ++q) sum += sh[q];
        double *cur, step, up, ua;
        update_refs(S, code, 0, cur, step, up, ua);
        const bool a = okf[i * P] != 0.0 && (log(ua) < sum + dlp[i * P]);
        if (a) *cur = cand[i * P];
        S.acc[(long long)code * P] += a ? 1.0 : 0.0;
        sh_acc = a;
      }
      __syncthreads();
      acc = sh_acc != 0;
      if (acc && j < P) S.ll[j] = lln;
    } else if (j < P) {
      double *cur, step, up, ua;
      update_refs(S, code, j, cur, step, up, ua);
      acc = okf[i * P + j] != 0.0 && (log(ua) < lln - S.ll[j] + dlp[i * P + j]);
      if (acc) {
        *cur = cand[i * P + j];
        S.ll[j] = lln;
      }
      S.acc[(long long)code * P + j] += acc ? 1.0 : 0.0;
    }
    pat |= (acc ? 1 : 0) << i;
    __syncthreads();
  }
  if (!A.flag) return;
  // log posterior of the state reached (mcmc.GPUSampler.log_post).  The d + 3 prior terms of
  // each GP are independent: with room in LDS one thread per term, then thread j adds its GP's
  // terms in the serial order (same bits; d + 3 fp64 log / exp chains in turn before)
  __shared__ double terms[kLpTerms];
  const int nt = (d + 3) * P;
  if (nt <= kLpTerms) {
    for (int t = j; t < nt; t += blockDim.x) {
      const int q = t / P, e = t - q * P;
      terms[t] = q <= d ? log_prior(S, 0, S.betaU[(long long)q * P + e])
                        : (q == d + 1 ? log_prior(S, 1, S.lamUz[e]) : log_prior(S, 2, S.lamWs[e]));
    }
    __syncthreads();
    if (j < P) {
      double t = S.ll[j];
      for (int q = 0; q < d + 3; ++q) t += terms[q * P + j];
      sh[j] = t;
    }
  } else if (j < P) {
    double t = S.ll[j];
    for (int r = 0; r <= d; ++r) t += log_prior(S, 0, S.betaU[(long long)r * P + j]);
    t += log_prior(S, 1, S.lamUz[j]);
    t += log_prior(S, 2, S.lamWs[j]);
    sh[j] = t;
  }
  __syncthreads();
  if (j == 0) {
    double sum = 0.0;
    for (int q = 0; q < P; ++q) sum += sh[q];
    S.lp[0] = sum + log_prior(S, 3, S.lamWOs[0]);
  }
}

__global__ __launch_bounds__(1024) void mcmc_prep_kernel(GroupArgs A, double* __restrict__ beta,
                                                         double* __restrict__ s,
                                                         double* __restrict__ delta) {
  prep_body(A, beta, s, delta);
}

__global__ __launch_bounds__(1024) void mcmc_decide_kernel(GroupArgs A,
                                                           const double* __restrict__ ll_all) {
  decide_body(A, ll_all);
}

// A group's decisions, then the next group's proposals and Gram inputs, in one launch (the
// barrier orders the decisions' state and scratch reads before the proposals' writes)
__global__ __launch_bounds__(1024) void mcmc_step_kernel(GroupArgs D,
                                                         const double* __restrict__ ll_all,
                                                         GroupArgs A, double* __restrict__ beta,
                                                         double* __restrict__ s,
                                                         double* __restrict__ delta) {
  decide_body(D, ll_all);
  __syncthreads();
  prep_body(A, beta, s, delta);
}

int group_args(const gp_mcmc_state* S, const int* kinds, int g, int flag, GroupArgs& A) {
  if (!S) return -1;
  if (S->P < 1 || S->P > 1024) return -2;
  if (S->d < 1 || S->d > GPFIT_MAX_DIM) return -3;
  if (g < 1 || g > GPFIT_MCMC_MAX_GROUP || !kinds) return -4;
  if (!S->betaU || !S->lamUz || !S->lamWs || !S->lamWOs || !S->ll || !S->lam || !S->u ||
      !S->step_betaU || !S->step_lamUz || !S->step_lamWs || !S->step_lamWOs || !S->acc ||
      !S->lp || !S->scratch)
    return -5;
  A.S = *S;
  for (int i = 0; i < g; ++i) {
    if (kinds[i] < 1 || kinds[i] > S->d + 3) return -6;
    A.kinds[i] = kinds[i];
  }
  for (int i = g; i < GPFIT_MCMC_MAX_GROUP; ++i) A.kinds[i] = 0;
  A.g = g;
  A.flag = flag;
  return 0;
}

int block_for(int P) { return (P + 63) / 64 * 64; }

}  // namespace

extern "C" int gp_mcmc_group_prep(const gp_mcmc_state* S, const int* kinds, int g, int first,
                                  double* beta, double* s, double* delta, hipStream_t stream) {
  GroupArgs A;
  const int rc = group_args(S, kinds, g, first, A);
  if (rc) return rc;
  if (!beta || !s || !delta) return -7;
  hipLaunchKernelGGL(mcmc_prep_kernel, dim3(1), dim3(block_for(S->P)), 0, stream, A, beta, s,
                     delta);
  const hipError_t e = hipGetLastError();
  return e == hipSuccess ? 0 : GPFIT_ERR_HIP - (int)e;
}

extern "C" int gp_mcmc_group_step(const gp_mcmc_state* S, const int* kinds, int g, int last,
                                  const double* ll_all, const gp_mcmc_state* S_next,
                                  const int* kinds_next, int g_next, int first, double* beta,
                                  double* s, double* delta, hipStream_t stream) {
  GroupArgs D, A;
  int rc = group_args(S, kinds, g, last, D);
  if (rc) return rc;
  if (!ll_all) return -7;
  rc = group_args(S_next, kinds_next, g_next, first, A);
  if (rc) return rc - 10;
  if (!beta || !s || !delta) return -17;
  if (S_next->P != S->P) return -18;
  hipLaunchKernelGGL(mcmc_step_kernel, dim3(1), dim3(block_for(S->P)), 0, stream, D, ll_all, A,
                     beta, s, delta);
  const hipError_t e = hipGetLastError();
  return e == hipSuccess ? 0 : GPFIT_ERR_HIP - (int)e;
}

extern "C" int gp_mcmc_group_decide(const gp_mcmc_state* S, const int* kinds, int g, int last,
                                    const double* ll_all, hipStream_t stream) {
  GroupArgs A;
  const int rc = group_args(S, kinds, g, last, A);
  if (rc) return rc;
  if (!ll_all) return -7;
  hipLaunchKernelGGL(mcmc_decide_kernel, dim3(1), dim3(block_for(S->P)), 0, stream, A, ll_all);
  const hipError_t e = hipGetLastError();
  return e == hipSuccess ? 0 : GPFIT_ERR_HIP - (int)e;
}
