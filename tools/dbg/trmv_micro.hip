// Microbenchmark (debug only): z = L^-1 w over the padded lower triangle at n = 4096 (71 MB
// read), the prediction's two-pass form (predict.hip trmv_part_kernel + trmv_sum_kernel) with
// its blocking varied: ZR rows per pass-1 block, ZS columns per strip, RPT rows per thread
// (one 16-B load per column for 2, two for 4), and pass 2 either one thread per row over every
// strip in order (SUM 0) or 8 threads per row over 8 strips each, combined in a fixed order
// (SUM 1).  Prints us per call (pass 1, pass 2) and the max |dz| against the first variant.
//   hipcc --offload-arch=gfx950 -O3 -o tools/dbg/trmv_micro tools/dbg/trmv_micro.hip
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <vector>

template <int ZR, int ZS, int RPT>
__global__ __launch_bounds__(256) void part(const double* __restrict__ L, int ld,
                                            const double* __restrict__ w, double* __restrict__ zp,
                                            int npad, int n) {
  const int rb = blockIdx.x * ZR, k0 = blockIdx.y * ZS;
  if (k0 > rb + ZR - 1 || k0 >= n) return;
  if (RPT * (int)threadIdx.x >= ZR) return;
  const int r = rb + RPT * threadIdx.x;
  if (r >= npad) return;
  const double* Lr = L + r;
  const int ke = min(k0 + ZS, n);
  double acc[RPT];
#pragma unroll
  for (int q = 0; q < RPT; ++q) acc[q] = 0.0;
#pragma unroll 1
  for (int kb = k0; kb < ke; kb += 16) {
    double2 lv[16][RPT / 2];
    double wk[16];
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      const bool ok = kb + j < ke;
#pragma unroll
      for (int h = 0; h < RPT / 2; ++h)
        lv[j][h] = ok ? *reinterpret_cast<const double2*>(Lr + (long long)(kb + j) * ld + 2 * h)
                      : make_double2(0.0, 0.0);
      wk[j] = ok ? w[kb + j] : 0.0;
    }
#pragma unroll
    for (int j = 0; j < 16; ++j)
#pragma unroll
      for (int h = 0; h < RPT / 2; ++h) {
        acc[2 * h] = fma(lv[j][h].x, wk[j], acc[2 * h]);
        acc[2 * h + 1] = fma(lv[j][h].y, wk[j], acc[2 * h + 1]);
      }
  }
#pragma unroll
  for (int h = 0; h < RPT / 2; ++h)
    *reinterpret_cast<double2*>(zp + (long long)blockIdx.y * npad + r + 2 * h) =
        make_double2(acc[2 * h], acc[2 * h + 1]);
}

template <int ZR, int ZS>
__global__ __launch_bounds__(256) void sum0(const double* __restrict__ zp, int npad, int n,
                                            double* __restrict__ z) {
  const int r = blockIdx.x * 256 + threadIdx.x;
  if (r >= npad) return;
  const int rb = (r / ZR) * ZR;
  const int last = min(rb + ZR - 1, n - 1) / ZS;
  const double* q = zp + r;
  double acc = 0.0;
  for (int s = 0; s <= last; ++s) acc += q[(long long)s * npad];
  z[r] = acc;
}

// 8 threads per row (g = tid >> 5 picks strips 8g .. 8g + 7 of 64), 32 rows per block
template <int ZR, int ZS>
__global__ __launch_bounds__(256) void sum1(const double* __restrict__ zp, int npad, int n,
                                            double* __restrict__ z) {
  __shared__ double red[8][32];
  const int rl = threadIdx.x & 31, g = threadIdx.x >> 5;
  const int r = blockIdx.x * 32 + rl;
  double acc = 0.0;
  if (r < npad) {
    const int rb = (r / ZR) * ZR;
    const int last = min(rb + ZR - 1, n - 1) / ZS;
    const int nst = last + 1, per = (nst + 7) / 8;
    const int s0 = g * per, s1 = min(nst, s0 + per);
    double v[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = (s0 + j < s1) ? zp[(long long)(s0 + j) * npad + r] : 0.0;
    for (int j = 8; s0 + j < s1; ++j) v[7] += zp[(long long)(s0 + j) * npad + r];
#pragma unroll
    for (int j = 0; j < 8; ++j) acc += v[j];
  }
  red[g][rl] = acc;
  __syncthreads();
  if (g == 0 && r < npad)
    z[r] = ((red[0][rl] + red[1][rl]) + (red[2][rl] + red[3][rl])) +
           ((red[4][rl] + red[5][rl]) + (red[6][rl] + red[7][rl]));
}

int main() {
  const int n = 4096, npad = 4096, ld = npad;
  std::vector<double> hL((size_t)ld * npad, 0.0), hw(n);
  for (int k = 0; k < n; ++k) {
    hw[k] = std::sin(0.37 * k);
    for (int r = k; r < n; ++r) hL[(size_t)k * ld + r] = std::cos(0.001 * r + 0.07 * k) / (1 + r - k);
  }
  double *L, *w, *zp, *z;
  hipMalloc(&L, hL.size() * 8);
  hipMalloc(&w, n * 8);
  hipMalloc(&zp, (size_t)128 * npad * 8);
  hipMalloc(&z, npad * 8);
  hipMemcpy(L, hL.data(), hL.size() * 8, hipMemcpyHostToDevice);
  hipMemcpy(w, hw.data(), n * 8, hipMemcpyHostToDevice);
  hipEvent_t a, b, c;
  hipEventCreate(&a); hipEventCreate(&b); hipEventCreate(&c);
  std::vector<double> z0(npad), zt(npad);
  int vi = 0;
  auto bench = [&](const char* name, auto p1, auto p2) {
    for (int r = 0; r < 3; ++r) { p1(); p2(); }
    float t1 = 0, t2 = 0;
    const int R = 20;
    for (int r = 0; r < R; ++r) {
      hipEventRecord(a); p1(); hipEventRecord(b); p2(); hipEventRecord(c);
      hipEventSynchronize(c);
      float x, y;
      hipEventElapsedTime(&x, a, b); hipEventElapsedTime(&y, b, c);
      t1 += x; t2 += y;
    }
    hipMemcpy(vi == 0 ? z0.data() : zt.data(), z, npad * 8, hipMemcpyDeviceToHost);
    double d = 0;
    if (vi) for (int r = 0; r < npad; ++r) d = fmax(d, fabs(zt[r] - z0[r]));
    printf("%-32s pass1 %7.1f us  pass2 %6.1f us  (%.0f GB/s pass 1)  max|dz| %.2e\n", name,
           1e3 * t1 / R, 1e3 * t2 / R, 8.0 * n * (n + 1) / 2 / (1e-3 * t1 / R) / 1e9, d);
    ++vi;
  };
#define V(ZR, ZS, RPT, SUM)                                                                     \
  bench("ZR=" #ZR " ZS=" #ZS " RPT=" #RPT " SUM=" #SUM,                                       \
        [&] { hipLaunchKernelGGL((part<ZR, ZS, RPT>), dim3((npad + ZR - 1) / ZR, npad / ZS),      \
                                 dim3(256), 0, 0, L, ld, w, zp, npad, n); },                      \
        [&] {                                                                                     \
          if (SUM == 0)                                                                           \
            hipLaunchKernelGGL((sum0<ZR, ZS>), dim3((npad + 255) / 256), dim3(256), 0, 0, zp,     \
                               npad, n, z);                                                       \
          else                                                                                    \
            hipLaunchKernelGGL((sum1<ZR, ZS>), dim3((npad + 31) / 32), dim3(256), 0, 0, zp, npad, \
                               n, z);                                                             \
        })
  V(512, 64, 2, 0);
  V(512, 64, 2, 1);
  V(512, 32, 2, 0);
  V(512, 32, 2, 1);
  V(256, 64, 1 * 2, 1);
  V(1024, 64, 4, 1);
  V(1024, 32, 4, 1);
  V(512, 128, 2, 1);
  V(256, 32, 2, 1);
  return 0;
}
