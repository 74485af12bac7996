// Marginal realisations of the posterior PC weights (opt-in realize mode of the prediction).
//
// Reference behaviour: SepiaEmulatorPrediction returns ONE random draw of the PC weights per
// (sample, PC), and the reference's accuracy statistics take quantiles over
// those draws (assess_all_models.py:489-500: preds.w -> get_y() + error draws).  The build
// returns the posterior mean by default; gp_realize turns (mean, var) into one marginal draw
//   out[i] = mean[i] + sqrt(max(var[i], 0)) * z_i ,   z_i ~ N(0, 1)
// so those quantiles keep their predictive spread.  (SEPIA draws jointly over the m_b points of
// a call; at m = 100k only the marginal is tractable — DESIGN.md.)
//
// z_i: counter-based Philox4x32-10 (Salmon et al., SC'11) keyed by `seed`, counter
// (i / 2, offset); the four 32-bit words make two 53-bit uniforms, Box-Muller gives z_{2j} =
// r cos(2 pi u2), z_{2j+1} = r sin(2 pi u2) with r = sqrt(-2 log(1 - u1)).  Deterministic
// for a (seed, offset) pair whatever the launch shape; restated in numpy by the test oracle.
// HBM-bound elementwise work: 24 B moved per element.
#include "gpfit_common.h"
#include "../../include/gpfit.h"

namespace {

GP_DEV void philox_round(uint32_t (&c)[4], uint32_t k0, uint32_t k1) {
  const uint64_t p0 = (uint64_t)0xD2511F53u * c[0];
  const uint64_t p1 = (uint64_t)0xCD9E8D57u * c[2];
  const uint32_t hi0 = (uint32_t)(p0 >> 32), lo0 = (uint32_t)p0;
  const uint32_t hi1 = (uint32_t)(p1 >> 32), lo1 = (uint32_t)p1;
  c[0] = hi1 ^ c[1] ^ k0;
  c[1] = lo1;
  c[2] = hi0 ^ c[3] ^ k1;
  c[3] = lo0;
}

GP_DEV void philox4x32_10(uint32_t (&c)[4], uint32_t k0, uint32_t k1) {
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    philox_round(c, k0, k1);
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
}

__global__ __launch_bounds__(256) void realize_kernel(const double* __restrict__ mean,
                                                      const double* __restrict__ var,
                                                      long long N, uint64_t seed,
                                                      uint64_t offset,
                                                      double* __restrict__ out) {
  const long long j = (long long)blockIdx.x * blockDim.x + threadIdx.x;   // pair index
  const long long i0 = 2 * j;
  if (i0 >= N) return;
  uint32_t c[4] = {(uint32_t)j, (uint32_t)((uint64_t)j >> 32), (uint32_t)offset,
                   (uint32_t)(offset >> 32)};
  philox4x32_10(c, (uint32_t)seed, (uint32_t)(seed >> 32));
  const double scale = 1.0 / 9007199254740992.0;   // 2^-53
  const double u1 = (double)((((uint64_t)c[0] << 32) | c[1]) >> 11) * scale;
  const double u2 = (double)((((uint64_t)c[2] << 32) | c[3]) >> 11) * scale;
  const double r = sqrt(-2.0 * log(1.0 - u1));
  double sn, cs;
  sincospi(2.0 * u2, &sn, &cs);
  out[i0] = mean[i0] + sqrt(fmax(var[i0], 0.0)) * (r * cs);
  if (i0 + 1 < N) out[i0 + 1] = mean[i0 + 1] + sqrt(fmax(var[i0 + 1], 0.0)) * (r * sn);
}

}  // namespace

extern "C" int gp_realize(const double* mean, const double* var, long long N,
                          unsigned long long seed, unsigned long long offset, double* out,
                          hipStream_t stream) {
  if (!mean) return -1;
  if (!var) return -2;
  if (N < 0) return -3;
  if (!out) return -6;
  if (N == 0) return 0;
  const long long pairs = (N + 1) / 2;
  hipLaunchKernelGGL(realize_kernel, dim3((unsigned)gp_ceil_div(pairs, 256)), dim3(256), 0,
                     stream, mean, var, N, (uint64_t)seed, (uint64_t)offset, out);
  const hipError_t e = hipGetLastError();
  return e == hipSuccess ? 0 : GPFIT_ERR_HIP - (int)e;
}
