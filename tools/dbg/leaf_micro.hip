// Microbenchmark (debug only): where the cycles of the chain's 16 x 16 leaf go.  A copy of
// chol.hip's leaf16 with s_memtime stamps between its phases (load, elimination, rsqrt,
// stores, pivot check + log), run by one wave on one workgroup.
#include "../../gladsgp_amd/csrc/chol.hip"
#include <cstdio>
#include <vector>

template <int VAR>
GP_DEV int leaf16_st(lds_double* T, lds_double* U, int o, int nb, double& lg, long long* ts) {
  const int lane = threadIdx.x & 63;
  const int c = lane & 15;
  const bool fac = lane < 16;
  ts[0] = __builtin_amdgcn_s_memtime();
  double v[16];
#pragma unroll
  for (int r = 0; r < 16; ++r) v[r] = fac ? T[(o + r) * LP + o + c] : (r == c ? 1.0 : 0.0);
  __builtin_amdgcn_s_waitcnt(0xc07f);
  ts[1] = __builtin_amdgcn_s_memtime();
  double rsq[16];
  double mypiv = 1.0;
  static_for<0, 16, 1>([&](auto J) {
    constexpr int j = decltype(J)::value;
    const double p = readlane_f64(v[j], j);
    mypiv = (c == j) ? p : mypiv;
    const double rp = rcp_nr(p);
    const double y = (fac && c <= j) ? 0.0 : v[j] * rp;
    static_for<j + 1, 16, 1>([&](auto R) {
      constexpr int r = decltype(R)::value;
      v[r] = fma(-readlane_f64(v[j], r), y, v[r]);
    });
    rsq[j] = p;
  });
  asm volatile("" ::"v"(v[15]), "v"(mypiv));
  ts[2] = __builtin_amdgcn_s_memtime();
  double myrs;
  if (VAR == 0) {
#pragma unroll
    for (int r = 0; r < 16; ++r) rsq[r] = rsqrt_nr(rsq[r]);
    myrs = rsqrt_nr(mypiv);
  } else {
    myrs = rsqrt_nr(mypiv);
#pragma unroll
    for (int r = 0; r < 16; ++r) rsq[r] = readlane_f64(myrs, r);
  }
  asm volatile("" ::"v"(rsq[15]), "v"(myrs));
  ts[3] = __builtin_amdgcn_s_memtime();
  if (lane < 32) {
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      if (fac)
        T[(o + r) * LP + o + c] = r > c ? v[r] * myrs : (r == c ? mypiv * myrs : 0.0);
      else
        U[(o + r) * LP + o + c] = r >= c ? v[r] * rsq[r] : 0.0;
    }
  }
  __builtin_amdgcn_s_waitcnt(0xc07f);
  ts[4] = __builtin_amdgcn_s_memtime();
  const bool ok = !(lane < 16 && o + c < nb) || (mypiv > 0.0 && isfinite(mypiv));
  const unsigned long long bad = __ballot(!ok);
  double l = (lane < 16 && o + c < nb) ? log(mypiv) : 0.0;
#pragma unroll
  for (int off = 8; off > 0; off >>= 1) l += __shfl_xor(l, off, 64);
  lg += readlane_f64(l, 0);
  ts[5] = __builtin_amdgcn_s_memtime();
  return bad ? o + __ffsll((long long)bad) : 0;
}

__global__ __launch_bounds__(256, 1) void probe(const double* G, long long* out, double* res) {
  LdsSmem& sm = *(LdsSmem*)&g_sm;
  for (int rep = 0; rep < 4; ++rep) {
    for (int g = threadIdx.x; g < NB * NB; g += 256) sm.As[(g >> 6) * LP + (g & 63)] = G[g];
    __syncthreads();
    long long ts[6], ts2[6];
    double lg = 0.0;
    int f = 0;
    if (threadIdx.x < 64) f = leaf16_st<0>(sm.As, sm.Bs, 0, NB, lg, ts);
    __syncthreads();
    for (int g = threadIdx.x; g < NB * NB; g += 256) sm.As[(g >> 6) * LP + (g & 63)] = G[g];
    __syncthreads();
    if (threadIdx.x < 64) f += leaf16_st<1>(sm.As, sm.Bs, 0, NB, lg, ts2);
    __syncthreads();
    for (int g = threadIdx.x; g < 256; g += 256) {
      res[g] = sm.As[(g >> 4) * LP + (g & 15)];
      res[256 + g] = sm.Bs[(g >> 4) * LP + (g & 15)];
    }
    __syncthreads();
    // the library's MFMA leaf
    for (int g = threadIdx.x; g < NB * NB; g += 256) sm.As[(g >> 6) * LP + (g & 63)] = G[g];
    __syncthreads();
    long long tm0 = __builtin_amdgcn_s_memtime();
    if (threadIdx.x < 64) leaf16(sm.As, sm.Bs, 0, sm.invs);
    __builtin_amdgcn_s_waitcnt(0xc07f);
    long long tm1 = __builtin_amdgcn_s_memtime();
    __syncthreads();
    for (int g = threadIdx.x; g < 256; g += 256) {
      res[512 + g] = sm.As[(g >> 4) * LP + (g & 15)];
      res[768 + g] = sm.Bs[(g >> 4) * LP + (g & 15)];
    }
    if (threadIdx.x == 0) out[rep * 16 + 6] = tm1 - tm0;
    __syncthreads();
    if (threadIdx.x == 0) {
      for (int q = 0; q < 5; ++q) out[rep * 16 + q] = ts[q + 1] - ts[q];
      for (int q = 0; q < 5; ++q) out[rep * 16 + 8 + q] = ts2[q + 1] - ts2[q];
      out[rep * 16 + 5] = f + (long long)lg;
    }
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
  double* dG;
  long long* dout;
  (void)hipMalloc(&dG, G.size() * 8);
  (void)hipMalloc(&dout, 64 * 8);
  double* dres;
  (void)hipMalloc(&dres, 1024 * 8);
  (void)hipMemcpy(dG, G.data(), G.size() * 8, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(probe, dim3(1), dim3(256), 0, 0, dG, dout, dres);
  std::vector<double> res(1024);
  (void)hipMemcpy(res.data(), dres, 1024 * 8, hipMemcpyDeviceToHost);
  double dL = 0, dU = 0, mL = 0, mU = 0;
  for (int g = 0; g < 256; ++g) {
    dL = fmax(dL, fabs(res[g] - res[512 + g]));
    dU = fmax(dU, fabs(res[256 + g] - res[768 + g]));
    mL = fmax(mL, fabs(res[g]));
    mU = fmax(mU, fabs(res[256 + g]));
  }
  printf("mfma leaf vs register leaf: max |dL| %.3e (max |L| %.3e), max |dLinv| %.3e (max %.3e)\n",
         dL, mL, dU, mU);
  std::vector<long long> o(64);
  (void)hipMemcpy(o.data(), dout, 64 * 8, hipMemcpyDeviceToHost);
  const char* ph[5] = {"load", "elim", "rsqrt", "store", "check+log"};
  for (int r = 0; r < 4; ++r) {
    printf("rep %d  rsqrt x17:", r);
    for (int q = 0; q < 5; ++q) printf(" %s %lld", ph[q], o[r * 16 + q]);
    printf(" | readlane rsq:");
    for (int q = 0; q < 5; ++q) printf(" %s %lld", ph[q], o[r * 16 + 8 + q]);
    printf(" | mfma leaf (library) %lld\n", o[r * 16 + 6]);
  }
  return 0;
}
extern "C" int gp_padded_n(int n) { return n <= 0 ? 0 : gp_ceil_div(n, GPFIT_TILE) * GPFIT_TILE; }
void gpfit_prof_begin(int, hipStream_t) {}
void gpfit_prof_end(int, hipStream_t) {}
