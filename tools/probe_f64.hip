// Hardware probe for gfx950 fp64 paths used by the GP kernels:
//  (1) v_mfma_f64_16x16x4_f64 operand/result lane maps (exact-integer, asymmetric operands)
//  (2) fp64 MFMA throughput, fp64 VALU FMA throughput, MFMA+VALU co-issue, exp() throughput
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cmath>
#include <vector>
typedef double d4 __attribute__((ext_vector_type(4)));
#define CK(x) do{hipError_t e=(x); if(e!=hipSuccess){printf("HIP error %s at %d\n",hipGetErrorString(e),__LINE__); exit(1);}}while(0)

// A: 16x4 (row i, k), B: 4x16 (k, col j). Hypothesis: lane l holds A[l&15][l>>4], B[l>>4][l&15]
__global__ void layout_k(const double* A, const double* B, double* D) {
  int l = threadIdx.x;
  double a = A[(l & 15) * 4 + (l >> 4)];
  double b = B[(l >> 4) * 16 + (l & 15)];
  d4 acc = {0, 0, 0, 0};
  acc = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc, 0, 0, 0);
  for (int r = 0; r < 4; r++) D[l * 4 + r] = acc[r];
}

__global__ void mfma_tp(double* out, int iters) {
  double a = threadIdx.x * 1e-3, b = 1.0 + blockIdx.x * 1e-6;
  d4 c0 = {0,0,0,0}, c1 = c0, c2 = c0, c3 = c0;
  for (int i = 0; i < iters; i++) {
    c0 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c0, 0, 0, 0);
    c1 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c1, 0, 0, 0);
    c2 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c2, 0, 0, 0);
    c3 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c3, 0, 0, 0);
  }
  d4 s = c0 + c1 + c2 + c3;
  if (s[0] == 12345.678) out[0] = s[1];
}

__global__ void valu_tp(double* out, int iters) {
  double x0 = threadIdx.x * 1e-3, x1 = x0 + 1, x2 = x0 + 2, x3 = x0 + 3, x4 = x0 + 4, x5 = x0 + 5, x6 = x0 + 6, x7 = x0 + 7;
  double m = 0.999999, c = 1e-7;
  for (int i = 0; i < iters; i++) {
    x0 = fma(x0, m, c); x1 = fma(x1, m, c); x2 = fma(x2, m, c); x3 = fma(x3, m, c);
    x4 = fma(x4, m, c); x5 = fma(x5, m, c); x6 = fma(x6, m, c); x7 = fma(x7, m, c);
  }
  double s = x0 + x1 + x2 + x3 + x4 + x5 + x6 + x7;
  if (s == 12345.678) out[0] = s;
}

// half of the waves do MFMA, half VALU FMA (wave-uniform split)
__global__ void mix_tp(double* out, int iters_m, int iters_v) {
  int w = threadIdx.x >> 6;
  if (w & 1) {
    double x0 = threadIdx.x * 1e-3, x1 = x0 + 1, x2 = x0 + 2, x3 = x0 + 3, x4 = x0 + 4, x5 = x0 + 5, x6 = x0 + 6, x7 = x0 + 7;
    double m = 0.999999, c = 1e-7;
    for (int i = 0; i < iters_v; i++) {
      x0 = fma(x0, m, c); x1 = fma(x1, m, c); x2 = fma(x2, m, c); x3 = fma(x3, m, c);
      x4 = fma(x4, m, c); x5 = fma(x5, m, c); x6 = fma(x6, m, c); x7 = fma(x7, m, c);
    }
    double s = x0 + x1 + x2 + x3 + x4 + x5 + x6 + x7;
    if (s == 12345.678) out[0] = s;
  } else {
    double a = threadIdx.x * 1e-3, b = 1.0 + blockIdx.x * 1e-6;
    d4 c0 = {0,0,0,0}, c1 = c0, c2 = c0, c3 = c0;
    for (int i = 0; i < iters_m; i++) {
      c0 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c0, 0, 0, 0);
      c1 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c1, 0, 0, 0);
      c2 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c2, 0, 0, 0);
      c3 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c3, 0, 0, 0);
    }
    d4 s = c0 + c1 + c2 + c3;
    if (s[0] == 12345.678) out[0] = s[1];
  }
}

__global__ void exp_tp(double* out, int iters) {
  double x = -(threadIdx.x & 63) * 1e-2, acc = 0;
  for (int i = 0; i < iters; i++) { acc += exp(x); x -= 1e-9; }
  if (acc == 12345.678) out[0] = acc;
}

static float time_ms(void (*launch)(void*), void* arg) {
  hipEvent_t a, b; CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
  launch(arg); CK(hipDeviceSynchronize());
  CK(hipEventRecord(a)); launch(arg); CK(hipEventRecord(b)); CK(hipEventSynchronize(b));
  float ms; CK(hipEventElapsedTime(&ms, a, b)); return ms;
}

double* g_out;
int g_blocks = 1024, g_threads = 256, g_iters = 4096;
void L_mfma(void*) { mfma_tp<<<g_blocks, g_threads>>>(g_out, g_iters); }
void L_valu(void*) { valu_tp<<<g_blocks, g_threads>>>(g_out, g_iters); }
void L_mix(void*) { mix_tp<<<g_blocks, 512>>>(g_out, g_iters, g_iters * 4); }
void L_exp(void*) { exp_tp<<<g_blocks, g_threads>>>(g_out, g_iters / 4); }

int main() {
  // (1) layout
  std::vector<double> A(64), B(64), D(256);
  for (int i = 0; i < 16; i++) for (int k = 0; k < 4; k++) A[i * 4 + k] = (i + 1) * 10 + k;         // asym
  for (int k = 0; k < 4; k++) for (int j = 0; j < 16; j++) B[k * 16 + j] = (k + 1) * 1000 + j * j;  // asym
  double *dA, *dB, *dD; CK(hipMalloc(&dA, 512)); CK(hipMalloc(&dB, 512)); CK(hipMalloc(&dD, 2048));
  CK(hipMemcpy(dA, A.data(), 512, hipMemcpyHostToDevice)); CK(hipMemcpy(dB, B.data(), 512, hipMemcpyHostToDevice));
  layout_k<<<1, 64>>>(dA, dB, dD); CK(hipDeviceSynchronize());
  CK(hipMemcpy(D.data(), dD, 2048, hipMemcpyDeviceToHost));
  int bad_h1 = 0, bad_h2 = 0;
  for (int l = 0; l < 64; l++) for (int r = 0; r < 4; r++) {
    int col = l & 15;
    int row1 = (l >> 4) + 4 * r;      // guide's f64 map
    int row2 = (l >> 4) * 4 + r;      // f32 16x16 map
    double e1 = 0, e2 = 0;
    for (int k = 0; k < 4; k++) { e1 += A[row1 * 4 + k] * B[k * 16 + col]; e2 += A[row2 * 4 + k] * B[k * 16 + col]; }
    if (D[l * 4 + r] != e1) bad_h1++;
    if (D[l * 4 + r] != e2) bad_h2++;
  }
  printf("LAYOUT f64 map row=(l>>4)+4r: %d mismatches; f32 map row=(l>>4)*4+r: %d mismatches\n", bad_h1, bad_h2);
  CK(hipMalloc(&g_out, 64));
  hipDeviceProp_t p; CK(hipGetDeviceProperties(&p, 0));
  printf("device %s CUs %d clock %d kHz\n", p.name, p.multiProcessorCount, p.clockRate);
  double waves = (double)g_blocks * g_threads / 64;
  float ms = time_ms(L_mfma, 0);
  double fl = waves * g_iters * 4 * 2048.0;
  printf("MFMA f64 16x16x4: %.3f ms  %.2f TFLOP/s\n", ms, fl / ms / 1e9);
  ms = time_ms(L_valu, 0);
  fl = (double)g_blocks * g_threads * g_iters * 8 * 2.0;
  printf("VALU f64 fma: %.3f ms  %.2f TFLOP/s\n", ms, fl / ms / 1e9);
  ms = time_ms(L_mix, 0);
  double flm = (double)g_blocks * 4 * g_iters * 4 * 2048.0, flv = (double)g_blocks * 256 * g_iters * 4 * 8 * 2.0;
  printf("MIX (4 mfma waves + 4 valu waves /WG): %.3f ms  mfma-part %.2f TF valu-part %.2f TF total %.2f TF\n", ms, flm / ms / 1e9, flv / ms / 1e9, (flm + flv) / ms / 1e9);
  ms = time_ms(L_exp, 0);
  double ne = (double)g_blocks * g_threads * (g_iters / 4);
  printf("exp f64: %.3f ms  %.2f Gexp/s\n", ms, ne / ms / 1e6);
  return 0;
}
