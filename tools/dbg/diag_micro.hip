// Microbenchmark (debug only): cycles of the persistent chain's 64 x 64 diagonal factor +
// inverse (diag_factor_blk), of its leaf16, and of a dependent mm16 chain, on one workgroup.
#include "../../gladsgp_amd/csrc/chol.hip"
#include <cstdio>
#include <vector>

__global__ __launch_bounds__(256, 1) void probe(const double* G, long long* out) {
  LdsSmem& sm = *(LdsSmem*)&g_sm;
  for (int rep = 0; rep < 4; ++rep) {
    for (int g = threadIdx.x; g < NB * NB; g += 256) sm.As[(g >> 6) * LP + (g & 63)] = G[g];
    __syncthreads();
    const long long t0 = __builtin_amdgcn_s_memtime();
    double lg = 0.0;
    const int f = diag_factor_blk(NB, &lg);
    const long long t1 = __builtin_amdgcn_s_memtime();
    // leaf alone (wave 0), on the factored tile's block 0 (values irrelevant)
    for (int g = threadIdx.x; g < NB * NB; g += 256) sm.As[(g >> 6) * LP + (g & 63)] = G[g];
    __syncthreads();
    const long long t2 = __builtin_amdgcn_s_memtime();
    double lg2 = 0.0;
    int f2 = 0;
    if (threadIdx.x < 64) leaf16(sm.As, sm.Bs, 0, sm.invs);
    __syncthreads();
    const long long t3 = __builtin_amdgcn_s_memtime();
    // 8 dependent mm16 (wave 0)
    f64x4 acc = zero4();
    if (threadIdx.x < 64)
      for (int q = 0; q < 8; ++q) mm16(acc, sm.As, LP, 1, sm.Bs, 1, LP, false);
    __syncthreads();
    const long long t4 = __builtin_amdgcn_s_memtime();
    // mma64 (all 4 waves, 64x64x64)
    f64x4 a2[2][2];
    mma64(g_sm.As, g_sm.Bs, a2);
    __syncthreads();
    const long long t5 = __builtin_amdgcn_s_memtime();
    if (threadIdx.x == 0) {
      out[rep * 8 + 0] = t1 - t0; out[rep * 8 + 1] = t3 - t2; out[rep * 8 + 2] = t4 - t3;
      out[rep * 8 + 3] = t5 - t4; out[rep * 8 + 4] = f + f2;
      out[rep * 8 + 5] = (long long)(acc[0] + a2[0][0][0] + lg + lg2);
    }
    __syncthreads();
  }
}

int main() {
  std::vector<double> G(NB * NB);
  for (int i = 0; i < NB; ++i)
    for (int j = 0; j < NB; ++j) {
      double s = 0.0;
      for (int k = 0; k < 8; ++k) { const double d = ((i * 37 + k * 11) % 64 - (j * 37 + k * 11) % 64) / 64.0; s += d * d; }
      G[i * NB + j] = exp(-s) + (i == j ? 1e-3 : 0.0);
    }
  double* dG; long long* dout;
  (void)hipMalloc(&dG, G.size() * 8); (void)hipMalloc(&dout, 32 * 8);
  (void)hipMemcpy(dG, G.data(), G.size() * 8, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(probe, dim3(1), dim3(256), 0, 0, dG, dout);
  std::vector<long long> o(32);
  (void)hipMemcpy(o.data(), dout, 32 * 8, hipMemcpyDeviceToHost);
  for (int r = 0; r < 4; ++r)
    printf("rep %d: diag_factor_blk %lld cyc | leaf16 %lld | 8 dep mm16 %lld | mma64 %lld | fail %lld\n",
           r, o[r * 8], o[r * 8 + 1], o[r * 8 + 2], o[r * 8 + 3], o[r * 8 + 4]);
  return 0;
}
extern "C" int gp_padded_n(int n) { return n <= 0 ? 0 : gp_ceil_div(n, GPFIT_TILE) * GPFIT_TILE; }
void gpfit_prof_begin(int, hipStream_t) {}
void gpfit_prof_end(int, hipStream_t) {}
