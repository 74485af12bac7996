// Microbenchmark (debug only): cycles of the persistent chain's 64 x 64 diagonal factor +
// inverse (diag_factor_blk) on one workgroup, on three Gram-like tiles; the residuals
// |L L^T - G| and |L^-1 L - I| are checked on the host (lower triangles).
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -mllvm -amdgpu-mfma-vgpr-form \
//     -Xclang -target-feature -Xclang +enable-ds128 tools/dbg/diag_micro.hip -o tools/dbg/diag_micro
#include "../../gladsgp_amd/csrc/chol.hip"
#include <cmath>
#include <cstdio>
#include <vector>

__global__ __launch_bounds__(256, 1) void probe(const double* G, long long* out, double* Lo,
                                                double* Xo) {
  LdsSmem& sm = *(LdsSmem*)&g_sm;
  for (int rep = 0; rep < 4; ++rep) {
    for (int g = threadIdx.x; g < NB * NB; g += 256) sm.As[(g >> 6) * LP + (g & 63)] = G[g];
    __syncthreads();
    const long long t0 = __builtin_amdgcn_s_memtime();
    double lg = 0.0;
    const int f = diag_factor_blk(NB, &lg);
    const long long t1 = __builtin_amdgcn_s_memtime();
    if (threadIdx.x == 0) {
      out[rep * 4 + 0] = t1 - t0;
      out[rep * 4 + 1] = f;
      out[rep * 4 + 2] = (long long)(lg * 1e6);
    }
    __syncthreads();
  }
  for (int g = threadIdx.x; g < NB * NB; g += 256) {
    Lo[g] = sm.As[(g >> 6) * LP + (g & 63)];
    Xo[g] = sm.Bs[(g >> 6) * LP + (g & 63)];
  }
}

int main() {
  double* dG; long long* dout; double *dL, *dX;
  (void)hipMalloc(&dG, NB * NB * 8); (void)hipMalloc(&dout, 16 * 8);
  (void)hipMalloc(&dL, NB * NB * 8); (void)hipMalloc(&dX, NB * NB * 8);
  for (int mat = 0; mat < 3; ++mat) {
    std::vector<double> G(NB * NB);
    for (int i = 0; i < NB; ++i)
      for (int j = 0; j < NB; ++j) {
        double s = 0.0;
        for (int k = 0; k < 8; ++k) {
          const double xi = ((i * 37 + k * 11) % 64) / 64.0, xj = ((j * 37 + k * 11) % 64) / 64.0;
          const double d = xi - xj;
          s += (mat == 0 ? 1.0 : (mat == 1 ? 0.2 : 0.05)) * d * d;
        }
        G[i * NB + j] = exp(-s) + (i == j ? (mat == 2 ? 1e-6 : 1e-3) : 0.0);
      }
    (void)hipMemcpy(dG, G.data(), G.size() * 8, hipMemcpyHostToDevice);
    std::vector<double> L(NB * NB), X(NB * NB);
    hipLaunchKernelGGL(probe, dim3(1), dim3(256), 0, 0, dG, dout, dL, dX);
    std::vector<long long> o(16);
    (void)hipMemcpy(o.data(), dout, 16 * 8, hipMemcpyDeviceToHost);
    (void)hipMemcpy(L.data(), dL, NB * NB * 8, hipMemcpyDeviceToHost);
    (void)hipMemcpy(X.data(), dX, NB * NB * 8, hipMemcpyDeviceToHost);
    for (int r = 0; r < 4; ++r)
      printf("mat %d rep %d: diag_factor_blk %lld cyc | fail %lld | logdet*1e6 %lld\n", mat, r,
             o[r * 4], o[r * 4 + 1], o[r * 4 + 2]);
    double rl = 0, rx = 0, nl = 0;
    for (int i = 0; i < NB; ++i)
      for (int j = 0; j < NB; ++j) {
        double s = 0, t = 0;
        for (int k = 0; k <= (i < j ? i : j); ++k) s += L[i * NB + k] * L[j * NB + k];
        for (int k = j; k <= i; ++k) t += X[i * NB + k] * L[k * NB + j];
        rl = fmax(rl, fabs(s - G[i * NB + j]));
        nl = fmax(nl, fabs(G[i * NB + j]));
        rx = fmax(rx, fabs(t - (i == j ? 1.0 : 0.0)));
      }
    printf("mat %d: max|LL^T-G|/max|G| %.3e  max|L^-1 L - I| %.3e\n", mat, rl / nl, rx);
  }
  return 0;
}
extern "C" int gp_padded_n(int n) { return n <= 0 ? 0 : gp_ceil_div(n, GPFIT_TILE) * GPFIT_TILE; }
void gpfit_prof_begin(int, hipStream_t) {}
void gpfit_prof_end(int, hipStream_t) {}
