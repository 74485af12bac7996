// Shared device helpers for libgpfit (gfx950 / CDNA4, fp64).
//
// MFMA used throughout: v_mfma_f64_16x16x4_f64 (64 cycles/SIMD on gfx950, ~70 TF/s measured
// chip-wide, tools/probe_f64.hip).  Lane maps, verified on hardware with exact integer,
// asymmetric operands (probe_f64 "LAYOUT ... 0 mismatches"):
//   A (16x4):  lane l holds A[l & 15][l >> 4]
//   B (4x16):  lane l holds B[l >> 4][l & 15]
//   C/D(16x16): lane l, reg r holds C[(l >> 4) + 4 r][l & 15]
#pragma once
#include <hip/hip_runtime.h>
#include <type_traits>
#include <stdint.h>

typedef double f64x4 __attribute__((ext_vector_type(4)));

#define GP_DEV __device__ __forceinline__

GP_DEV f64x4 mfma16x16x4(double a, double b, f64x4 c) {
  return __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0);
}

// Broadcast lane 0's double to an SGPR pair: tells the compiler a value is wave-uniform.
GP_DEV double uniform_f64(double x) {
  const unsigned long long u = __double_as_longlong(x);
  const unsigned lo = __builtin_amdgcn_readfirstlane((unsigned)u);
  const unsigned hi = __builtin_amdgcn_readfirstlane((unsigned)(u >> 32));
  return __longlong_as_double(((unsigned long long)hi << 32) | lo);
}

// v_readlane of a double: lane `l` (wave-uniform index) broadcast through SGPRs.
GP_DEV double readlane_f64(double x, int l) {
  const unsigned long long u = __double_as_longlong(x);
  const unsigned lo = __builtin_amdgcn_readlane((unsigned)u, l);
  const unsigned hi = __builtin_amdgcn_readlane((unsigned)(u >> 32), l);
  return __longlong_as_double(((unsigned long long)hi << 32) | lo);
}

// 1/sqrt(x) for x > 0: hardware v_rsq_f64 estimate + two Newton steps (<= 1 ulp typical);
// a short dependent chain, used where the pivot sits on a sequential critical path.
GP_DEV double rsqrt_nr(double x) {
  double y = __builtin_amdgcn_rsq(x);
  const double hx = 0.5 * x;
  y = y * fma(-hx * y, y, 1.5);
  y = y * fma(-hx * y, y, 1.5);
  return y;
}

// 1/x: hardware v_rcp_f64 estimate + two Newton steps (<= 1 ulp typical).
GP_DEV double rcp_nr(double x) {
  double y = __builtin_amdgcn_rcp(x);
  y = fma(y, fma(-x, y, 1.0), y);
  y = fma(y, fma(-x, y, 1.0), y);
  return y;
}

// Compile-time loop: f(std::integral_constant<int, i>) for i = B, B+S, ... < E (register
// arrays indexed by i stay in registers whatever the unroller decides).
template <int B, int E, int S, class F>
GP_DEV void static_for(F&& f) {
  if constexpr (B < E) {
    f(std::integral_constant<int, B>{});
    static_for<B + S, E, S>(f);
  }
}

// Spin (s_sleep between polls) until the LDS int *flag >= target.  Written as one asm block so
// it is opaque to the compiler: a visible loop splits the caller's straight-line, register-
// array code into basic blocks and the allocator then spills.  The memory clobber keeps the
// caller's later LDS reads below the wait.  The low 32 bits of a flat LDS address are its
// LDS offset (the shared aperture is 4 GiB aligned).
GP_DEV void lds_wait_ge(int* flag, int target) {
  const unsigned addr = (unsigned)(size_t)flag;
  int v;
  unsigned s;
  asm volatile(
      "1:\n"
      "  ds_read_b32 %0, %2\n"
      "  s_waitcnt lgkmcnt(0)\n"
      "  v_readfirstlane_b32 %1, %0\n"
      "  s_cmp_ge_i32 %1, %3\n"
      "  s_cbranch_scc1 2f\n"
      "  s_sleep 1\n"
      "  s_branch 1b\n"
      "2:\n"
      : "=&v"(v), "=&s"(s)
      : "v"(addr), "s"(target)
      : "memory", "scc");
}

GP_DEV f64x4 zero4() { f64x4 z = {0.0, 0.0, 0.0, 0.0}; return z; }

// exp(-a) for a >= 0 (a weighted squared distance), ~19 VALU ops: Cody-Waite reduction by ln 2,
// a degree-11 minimax polynomial for e^r (|r| <= ln2/2; the coefficients ocml's exp uses), and
// ldexp.  Every polynomial step is fma(p, r, c) with c a wave-uniform constant (an SGPR or
// literal operand), so no constant has to be re-materialised in a VGPR per call (ocml's fmac
// form overwrites its constant registers: 22 extra v_mov per exp inside a loop).  a is clamped
// to 1100 first: e^-1100 underflows to +0 through the ldexp, the only range check a
// non-negative argument needs.  v_min_f64 drops a NaN operand (IEEE minNum), so the result is
// finally passed through fma(a, 0, e): +0 for finite a (e unchanged), NaN for a NaN / Inf
// distance (NaN or Inf beta / design values), so bad inputs reach the factorisation's info
// instead of becoming a finite ~0.  Accuracy: within 1 ulp of exp (the same reduction and
// polynomial as ocml).
// fma(p, r, c) with c wave-uniform, pinned to VOP3 v_fma_f64 with c in an SGPR pair (the
// compiler otherwise keeps c in a VGPR and copies it before every v_fmac_f64).
GP_DEV double fma_sc(double p, double r, double c) {
  double o;
  asm("v_fma_f64 %0, %1, %2, %3" : "=v"(o) : "v"(p), "v"(r), "s"(c));
  return o;
}

GP_DEV double exp_neg(double a) {
  const double x = -fmin(a, 1100.0);
  const double k = __builtin_rint(x * 0x1.71547652b82fep+0);              // x log2(e)
  double r = fma(k, -0x1.62e42fefa39efp-1, x);                             // - k ln2 (hi)
  r = fma(k, -0x1.abc9e3b39803fp-56, r);                                   // - k ln2 (lo)
  double p = fma_sc(r, 0x1.ade156a5dcb37p-26, 0x1.28af3fca7ab0cp-22);
  p = fma_sc(p, r, 0x1.71dee623fde64p-19);
  p = fma_sc(p, r, 0x1.a01997c89e6b0p-16);
  p = fma_sc(p, r, 0x1.a01a014761f6ep-13);
  p = fma_sc(p, r, 0x1.6c16c1852b7b0p-10);
  p = fma_sc(p, r, 0x1.1111111122322p-7);
  p = fma_sc(p, r, 0x1.55555555502a1p-5);
  p = fma_sc(p, r, 0x1.5555555555511p-3);
  p = fma_sc(p, r, 0x1.000000000000bp-1);
  p = fma(p, r, 1.0);
  p = fma(p, r, 1.0);
  return fma(a, 0.0, __builtin_ldexp(p, (int)k));
}

// exp(-a) from a 64-entry table (the prediction's cross-covariance, predict.hip): with
// q = rint(-a 64 / ln2), exp(-a) = 2^(q >> 6) T[q & 63] exp(r), T[j] = 2^(j / 64) correctly
// rounded (kExp2Tab), r = -a - q ln2 / 64 (two-part constant), |r| <= ln2 / 128, exp(r) - 1 by
// its degree-5 Taylor polynomial (truncation 3.5e-17 relative) and T + T (exp(r) - 1) by one
// fma: within 1 ulp of ocml's exp (tools/dbg/cross_micro.hip: max 1.0 ulp over 67M values),
// 12 fp64 operations instead of exp_neg's 17 -- the cross-covariance of a batch is bound by its
// fp64 VALU work (C4 chunk 596 -> 472 us, profiles/r05/r05e_cross_micro.log).  `tab` is an
// LDS copy of kExp2Tab (per-lane indices).  NaN / Inf arguments propagate as in exp_neg.
static __constant__ double kExp2Tab[64] = {
    0x1.0000000000000p+0, 0x1.02c9a3e778061p+0, 0x1.059b0d3158574p+0, 0x1.0874518759bc8p+0,
    0x1.0b5586cf9890fp+0, 0x1.0e3ec32d3d1a2p+0, 0x1.11301d0125b51p+0, 0x1.1429aaea92de0p+0,
    0x1.172b83c7d517bp+0, 0x1.1a35beb6fcb75p+0, 0x1.1d4873168b9aap+0, 0x1.2063b88628cd6p+0,
    0x1.2387a6e756238p+0, 0x1.26b4565e27cddp+0, 0x1.29e9df51fdee1p+0, 0x1.2d285a6e4030bp+0,
    0x1.306fe0a31b715p+0, 0x1.33c08b26416ffp+0, 0x1.371a7373aa9cbp+0, 0x1.3a7db34e59ff7p+0,
    0x1.3dea64c123422p+0, 0x1.4160a21f72e2ap+0, 0x1.44e086061892dp+0, 0x1.486a2b5c13cd0p+0,
    0x1.4bfdad5362a27p+0, 0x1.4f9b2769d2ca7p+0, 0x1.5342b569d4f82p+0, 0x1.56f4736b527dap+0,
    0x1.5ab07dd485429p+0, 0x1.5e76f15ad2148p+0, 0x1.6247eb03a5585p+0, 0x1.6623882552225p+0,
    0x1.6a09e667f3bcdp+0, 0x1.6dfb23c651a2fp+0, 0x1.71f75e8ec5f74p+0, 0x1.75feb564267c9p+0,
    0x1.7a11473eb0187p+0, 0x1.7e2f336cf4e62p+0, 0x1.82589994cce13p+0, 0x1.868d99b4492edp+0,
    0x1.8ace5422aa0dbp+0, 0x1.8f1ae99157736p+0, 0x1.93737b0cdc5e5p+0, 0x1.97d829fde4e50p+0,
    0x1.9c49182a3f090p+0, 0x1.a0c667b5de565p+0, 0x1.a5503b23e255dp+0, 0x1.a9e6b5579fdbfp+0,
    0x1.ae89f995ad3adp+0, 0x1.b33a2b84f15fbp+0, 0x1.b7f76f2fb5e47p+0, 0x1.bcc1e904bc1d2p+0,
    0x1.c199bdd85529cp+0, 0x1.c67f12e57d14bp+0, 0x1.cb720dcef9069p+0, 0x1.d072d4a07897cp+0,
    0x1.d5818dcfba487p+0, 0x1.da9e603db3285p+0, 0x1.dfc97337b9b5fp+0, 0x1.e502ee78b3ff6p+0,
    0x1.ea4afa2a490dap+0, 0x1.efa1bee615a27p+0, 0x1.f50765b6e4540p+0, 0x1.fa7c1819e90d8p+0,
};

GP_DEV double exp_neg_tab(double a, const double* tab) {
  const double x = -fmin(a, 1100.0);
  const double q = __builtin_rint(x * 0x1.71547652b82fep+6);               // x 64 / ln2
  double r = fma(q, -0x1.62e42fefa39efp-7, x);                             // - q ln2/64 (hi)
  r = fma(q, -0x1.abc9e3b39803fp-62, r);                                   // - q ln2/64 (lo)
  double p = fma_sc(r, 0x1.1111111111111p-7, 0x1.5555555555555p-5);        // 1/120, 1/24
  p = fma_sc(p, r, 0x1.5555555555555p-3);                                  // 1/6
  p = fma_sc(p, r, 0.5);
  p = fma(p, r, 1.0);
  p = p * r;                                                               // exp(r) - 1
  const int qi = (int)q;
  const double t = tab[qi & 63];
  return fma(a, 0.0, __builtin_ldexp(fma(t, p, t), qi >> 6));
}

// Squared ARD distance sum_k beta_k (a_k - b_k)^2 ; D is a compile-time dimension bound.
template <int D>
GP_DEV double ard_dist(const double* __restrict__ a, const double* __restrict__ b,
                       const double* __restrict__ beta, int d) {
  double acc = 0.0;
#pragma unroll
  for (int k = 0; k < D; ++k) {
    if (k < d) {
      double t = a[k] - b[k];
      acc = fma(beta[k] * t, t, acc);
    }
  }
  return acc;
}

// Bijective XCD-aware remap of a 1-D block index (cdna_hip_programming.md §5 "XCD swizzle must
// be bijective"): blocks that the dispatcher deals to one XCD (b % 8 equal) get a contiguous
// range of logical ids, so neighbouring tiles share an L2.  Speed only, never correctness.
GP_DEV int xcd_remap(int b, int nwg) {
  const int nx = 8;
  int q = nwg / nx, r = nwg % nx;
  int xcd = b % nx, pos = b / nx;
  int base = (xcd < r) ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q;
  return base + pos;
}

__host__ __device__ inline int gp_ceil_div(long long a, long long b) { return (int)((a + b - 1) / b); }
