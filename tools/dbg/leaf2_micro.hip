// Microbenchmark (debug only): the 16 x 16 leaf of the chain's diagonal factor, cycles per
// variant on one workgroup (build like diag_micro.hip): leaf16 (one wave: A and W MFMAs), leaf16_elim alone (wave 0, the
// W handoff unused), leaf16_elim + leaf16_inv (waves 0 and 1), and the elimination without the
// multiplier stores / step releases.
#include "../../gladsgp_amd/csrc/chol.hip"
#include <cstdio>
#include <vector>

// round 4's two-wave leaf (not adopted: profiles/r04/ab_leaf2.log)
// ---- Two-wave leaf (round 4): the same elimination with the W (inverse) row operations on
// wave 1 and the next pivot's reciprocal off the MFMA path.  leaf16 runs two dependent f64
// MFMAs per step on ONE wave (A and W: 128 cycles of that SIMD's matrix pipe) and a pivot chain
// readlane -> rcp + 2 Newton -> multiplier -> MFMA after every step, ~310 cycles per step
// (profiles/r02/ab_mfma_leaf.log; neither change alone helped: ab_leaf_spec_pivot.log,
// DESIGN.md's two-wave leaf with a flag per step).  Here
//  * wave 0 (leaf16_elim) issues only the A updates.  The pivot of step j+1 is computed while
//    step j's MFMA runs, from the same values the MFMA combines:
//      p_{j+1} = fma(-A[j][j+1], A[j][j+1] * r_j, A[j+1][j+1])   (r_j = 1/p_j, the multiplier
//    lane j+1 uses), so step j+1 needs only A (MFMA -> VALU -> MFMA: multiplier = row * r) and
//    an r already in an SGPR pair.  Every pivot (L's diagonal and column scales, the checks, the
//    log) is that recurrence value.  The multipliers go to LDS (one 8-B slot per lane and step)
//    and a step counter is released every DIAG_PE steps;
//  * wave 1 (leaf16_inv) replays W = Lt^-1 from the published multipliers (the identical
//    W MFMA sequence of leaf16) on its own SIMD's matrix pipe, trailing wave 0 by < DIAG_PE
//    steps, then scales W's rows by the pivots wave 0 publishes last.
// Same arithmetic as leaf16 operation for operation where the f64 MFMA's single product
// accumulates exactly (fused, one rounding): bit-identical L and L^-1 then.
using lds_int = __attribute__((address_space(3))) int;

GP_DEV void leaf16_elim(lds_double* T, int o, lds_double* piv, lds_double* M, lds_int* step,
                        int base) {
  const int lane = threadIdx.x & 63;
  const int r0 = lane >> 4, c = lane & 15;
  f64x4 A = ld16(T + o * LP + o);
  double p = readlane_f64(A[0], 0);
  double r = rcp_nr(p);
  double colpiv = 1.0;
  static_for<0, 16, 1>([&](auto J) {
    constexpr int j = decltype(J)::value;
    constexpr int q = j >> 2, k = j & 3;
    colpiv = (c == j) ? p : colpiv;
    if constexpr (j < 15) {
      constexpr int q1 = (j + 1) >> 2, k1 = (j + 1) & 3;
      // critical path: MFMA j-1 -> multiplier -> MFMA j
      const double rowj = A[q];
      const double dg = A[q1];
      const bool sel = r0 == k && c > j;
      const double a = sel ? -rowj : 0.0;
      const double m = sel ? rowj * r : 0.0;
      A = mfma16x16x4(a, m, A);
      // everything below issues while MFMA j runs (the scheduler may not hoist it above)
      __builtin_amdgcn_sched_barrier(0);
      M[j * 64 + lane] = m;
      // release the multipliers of the previous group: their stores went out a step ago, so
      // the release's lgkmcnt(0) wait finds them done
      if constexpr (j % DIAG_PE == 0 && j > 0)
        __hip_atomic_store(step, base + j, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
      const double b = readlane_f64(rowj, 16 * k + j + 1);        // A[j][j+1]
      const double dd = readlane_f64(dg, 16 * k1 + j + 1);        // A[j+1][j+1]
      p = fma(-b, b * r, dd);
      r = rcp_nr(p);
      __builtin_amdgcn_sched_barrier(0);
    }
  });
  __hip_atomic_store(step, base + 15, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
  if (lane < 16) piv[o + c] = colpiv;
  const double rsc = rsqrt_nr(colpiv);
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int rr = r0 + 4 * q;
    T[(o + rr) * LP + o + c] = rr > c ? A[q] * rsc : (rr == c ? colpiv * rsc : 0.0);
  }
  __hip_atomic_store(step, base + 16, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
}

GP_DEV void leaf16_inv(lds_double* U, int o, const lds_double* piv, const lds_double* M,
                       lds_int* step, int base) {
  const int lane = threadIdx.x & 63;
  const int r0 = lane >> 4, c = lane & 15;
  f64x4 W;
#pragma unroll
  for (int q = 0; q < 4; ++q) W[q] = (r0 + 4 * q == c) ? 1.0 : 0.0;
  static_for<0, 15, 1>([&](auto J) {
    constexpr int j = decltype(J)::value;
    constexpr int q = j >> 2;
    if constexpr (j % DIAG_PE == 0)
      lds_wait_ge((int*)step, base + ((j + DIAG_PE < 15) ? j + DIAG_PE : 15));
    const double m = M[j * 64 + lane];
    const double wj = W[q];
    W = mfma16x16x4(-m, wj, W);
  });
  lds_wait_ge((int*)step, base + 16);
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int rr = r0 + 4 * q;
    const double rsr = rsqrt_nr(piv[o + rr]);
    U[(o + rr) * LP + o + c] = rr >= c ? W[q] * rsr : 0.0;
  }
}


__global__ __launch_bounds__(256, 1) void probe(const double* G, long long* out) {
  LdsSmem& sm = *(LdsSmem*)&g_sm;
  lds_double* Mx = (lds_double*)g_keep;
  const int w = threadIdx.x >> 6;
  for (int rep = 0; rep < 3; ++rep) {
    long long* o = out + rep * 16;
    // A: old leaf on wave 0
    for (int g = threadIdx.x; g < NB * NB; g += 256) sm.As[(g >> 6) * LP + (g & 63)] = G[g];
    if (threadIdx.x == 0) sm.step = 0;
    __syncthreads();
    long long t0 = __builtin_amdgcn_s_memtime();
    if (w == 0) leaf16(sm.As, sm.Bs, 0, sm.invs);
    long long t1 = __builtin_amdgcn_s_memtime();
    if (threadIdx.x == 0) o[0] = t1 - t0;
    __syncthreads();
    // B: elim alone on wave 0 (step releases go nowhere)
    for (int g = threadIdx.x; g < NB * NB; g += 256) sm.As[(g >> 6) * LP + (g & 63)] = G[g];
    if (threadIdx.x == 0) sm.step = 0;
    __syncthreads();
    t0 = __builtin_amdgcn_s_memtime();
    if (w == 0) leaf16_elim(sm.As, 0, sm.invs, Mx, (lds_int*)&sm.step, 0);
    t1 = __builtin_amdgcn_s_memtime();
    if (threadIdx.x == 0) o[1] = t1 - t0;
    __syncthreads();
    // C: elim (wave 0) + inv (wave 1)
    for (int g = threadIdx.x; g < NB * NB; g += 256) sm.As[(g >> 6) * LP + (g & 63)] = G[g];
    if (threadIdx.x == 0) sm.step = 0;
    __syncthreads();
    t0 = __builtin_amdgcn_s_memtime();
    if (w == 0) leaf16_elim(sm.As, 0, sm.invs, Mx, (lds_int*)&sm.step, 0);
    else if (w == 1) leaf16_inv(sm.Bs, 0, sm.invs, Mx, (lds_int*)&sm.step, 0);
    t1 = __builtin_amdgcn_s_memtime();
    if (threadIdx.x == 0) o[2] = t1 - t0;
    if (threadIdx.x == 64) o[3] = t1 - t0;
    __syncthreads();
    long long t2 = __builtin_amdgcn_s_memtime();
    if (threadIdx.x == 0) o[4] = t2 - t0;
    // D: dependent MFMA chain of 16 (srcC) and of 16 through srcB
    f64x4 a = zero4();
    double x = sm.As[threadIdx.x & 63];
    t0 = __builtin_amdgcn_s_memtime();
    if (w == 0) {
#pragma unroll
      for (int i = 0; i < 16; ++i) a = mfma16x16x4(x, x, a);
      asm volatile("" ::"v"(a));
    }
    t1 = __builtin_amdgcn_s_memtime();
    if (threadIdx.x == 0) o[5] = t1 - t0;
    t0 = __builtin_amdgcn_s_memtime();
    if (w == 0) {
#pragma unroll
      for (int i = 0; i < 16; ++i) a = mfma16x16x4(x, a[i & 3], a);
      asm volatile("" ::"v"(a));
    }
    t1 = __builtin_amdgcn_s_memtime();
    if (threadIdx.x == 0) o[6] = t1 - t0;
    // E: MFMA -> VALU mul -> MFMA chain of 16
    t0 = __builtin_amdgcn_s_memtime();
    if (w == 0) {
      double r = 1.0000001;
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const double m = a[i & 3] * r;
        a = mfma16x16x4(x, m, a);
      }
      asm volatile("" ::"v"(a));
    }
    t1 = __builtin_amdgcn_s_memtime();
    if (threadIdx.x == 0) o[7] = t1 - t0;
    // F: readlane -> rcp_nr chain of 16
    t0 = __builtin_amdgcn_s_memtime();
    if (w == 0) {
      double p = x + 2.0;
#pragma unroll
      for (int i = 0; i < 16; ++i) p = rcp_nr(readlane_f64(p, i)) + 1.5;
      asm volatile("" ::"v"(p));
    }
    t1 = __builtin_amdgcn_s_memtime();
    if (threadIdx.x == 0) o[8] = t1 - t0;
    __syncthreads();
  }
}

int main() {
  std::vector<double> G(NB * NB);
  for (int i = 0; i < NB; ++i)
    for (int j = 0; j < NB; ++j) {
      double s = 0.0;
      for (int k = 0; k < 8; ++k) {
        const double d = ((i * 37 + k * 11) % 64 - (j * 37 + k * 11) % 64) / 64.0;
        s += d * d;
      }
      G[i * NB + j] = exp(-s) + (i == j ? 1e-3 : 0.0);
    }
  double* dG; long long* dout;
  (void)hipMalloc(&dG, G.size() * 8); (void)hipMalloc(&dout, 48 * 8);
  (void)hipMemcpy(dG, G.data(), G.size() * 8, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(probe, dim3(1), dim3(256), 0, 0, dG, dout);
  std::vector<long long> o(48);
  (void)hipMemcpy(o.data(), dout, 48 * 8, hipMemcpyDeviceToHost);
  for (int r = 0; r < 3; ++r) {
    const long long* x = &o[r * 16];
    printf("rep %d: leaf16 %lld | elim alone %lld | elim+inv: w0 %lld w1 %lld all %lld | "
           "16 dep mfma (srcC) %lld | 16 dep via srcB %lld | mfma->mul->mfma x16 %lld | "
           "readlane->rcp_nr x16 %lld\n", r, x[0], x[1], x[2], x[3], x[4], x[5], x[6], x[7], x[8]);
  }
  return 0;
}
extern "C" int gp_padded_n(int n) { return n <= 0 ? 0 : gp_ceil_div(n, GPFIT_TILE) * GPFIT_TILE; }
void gpfit_prof_begin(int, hipStream_t) {}
void gpfit_prof_end(int, hipStream_t) {}
