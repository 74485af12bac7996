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
#include <stdint.h>

typedef double f64x4 __attribute__((ext_vector_type(4)));

#define GP_DEV __device__ __forceinline__

GP_DEV f64x4 mfma16x16x4(double a, double b, f64x4 c) {
  return __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0);
}

GP_DEV f64x4 zero4() { f64x4 z = {0.0, 0.0, 0.0, 0.0}; return z; }

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

static inline int gp_ceil_div(long long a, long long b) { return (int)((a + b - 1) / b); }
