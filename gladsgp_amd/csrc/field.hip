// Field reconstruction (A9): SepiaEmulatorPrediction.get_y() -- y = (w K + e) sd + mu
// (time_predictions.py:79-90, assess_all_models.py:489-500) in one kernel.
//
// w (rows x P, rows = samples x test points) times the PC basis K (P x ncols, ncols = field
// nodes) is a GEMM with a short inner dimension (P <= 64 PCs) and a huge output (C5: 100k
// points x 10k nodes = 1e9 elements): the product is fp64-MFMA-bound (2 P flop per element,
// 1.28e11 flop at C5 = 1.6 ms at peak) against a 4-8 GB output write (0.5-1.0 ms at 8 TB/s).
// The generic path wrote the fp64 product (8 B per element), re-read it for the back-transform
// and again for the float32 narrowing -- ~4.5x the output's bytes.  Here the back-transform
// (fma(v, sd, mu), the same operation as gp_standardize's inverse), the optional error term
// (one scalar per row) and the narrowing run in the MFMA epilogue: every output element is
// written once, in its final dtype.
//
// Layout: block = 4 waves; every wave owns 64 consecutive output columns, the block 256.  A
// wave keeps its K panel (P x 64 doubles, the B operands of all its k-steps: 128 VGPRs at
// P = 64) in registers for the whole launch; the block streams 32-row tiles of w through LDS
// (double-buffered, the next tile's global loads in flight under the current tile's MFMAs),
// so w is read once per 256 columns (from L2 / MALL: w is 51 MB at C5).  Per tile and wave:
// 1-2 row sub-tiles x 4 column tiles x ceil(P/4) k-steps of v_mfma_f64_16x16x4_f64.
//
// Bits: every element is the k-ordered MFMA chain over k = 0, 4, 8, ... (k >= P contributes
// exact zeros), then v + e, then fma(v, sd, mu) -- the sums gp_dgemm's 64x64-tile kernel forms
// for K <= 64 (one accumulator, k in order, no split) followed by gp_standardize's inverse, so
// the fused path equals the generic one bit for bit (tests/test_gpu_emulator.py).
#include "gpfit_common.h"
#include "../../include/gpfit.h"

namespace {

// rows of w per tile: 32 (two 16-row MFMA sub-tiles) while the K panel leaves room for their
// accumulators, 16 at P > 32 (K panel 128 + accumulators 32 of 256 registers at P = 64)
#ifndef FIELD_ROWS_BIG
#define FIELD_ROWS_BIG 16
#endif
#ifndef FIELD_OCC
#define FIELD_OCC 3
#endif
// non-temporal output stores (the field is written once and not re-read by this kernel):
// 3.26 vs 3.78 ms at C5 (profiles/r06/r06c_field_ab.log), same bits
#ifndef FIELD_NT
#define FIELD_NT 1
#endif
template <int KS> constexpr int field_rows() { return KS <= 8 ? 32 : FIELD_ROWS_BIG; }
// float32 output staged through LDS and stored 16 B per lane (a wave's row segments written by
// one instruction each) instead of 4 B per lane from the MFMA C layout
#ifndef FIELD_ST16
#define FIELD_ST16 1
#endif
// timing probe only (no output): 1 = skip the stores
#ifndef FIELD_PROBE
#define FIELD_PROBE 0
#endif
typedef float f32x4_t __attribute__((ext_vector_type(4)));
#ifndef FIELD_WAVES
#define FIELD_WAVES 4
#endif
#ifndef FIELD_JT
#define FIELD_JT 2
#endif
constexpr int kFieldWaves = FIELD_WAVES;     // waves per block
constexpr int kFieldJT = FIELD_JT;           // 16-column MFMA tiles per wave
constexpr int kFieldThreads = 64 * kFieldWaves;
constexpr int kFieldWaveCols = 16 * kFieldJT;
constexpr int kFieldCols = kFieldWaves * kFieldWaveCols;   // output columns per block
constexpr int kFieldPitch = 68;              // LDS row pitch of a w tile (doubles)
constexpr int kFieldMaxP = 64;

// KS = k-steps of 4 (P <= 4 KS), F32 = narrow the output to float32.  Work units are (column
// panel, row tile) pairs, panel-major; block i takes units [i U / B, (i + 1) U / B) of the
// U = npanels x ntiles (one residency round of B blocks: no tail round), reloading its K panel
// when its range crosses into the next panel.
template <int KS, bool F32>
__global__ __launch_bounds__(kFieldThreads, FIELD_OCC) void field_kernel(const double* __restrict__ W,
                                                       long long ldw, int rows, int P,
                                                       const double* __restrict__ K,
                                                       long long ldk, int ncols,
                                                       const double* __restrict__ sd,
                                                       const double* __restrict__ mu,
                                                       const double* __restrict__ err,
                                                       void* __restrict__ Y, long long ldy,
                                                       long long ntiles, bool vec16) {
  constexpr int KP = 4 * KS;                              // padded inner dimension
  constexpr int kFieldRows = field_rows<KS>(), RS = kFieldRows / 16;
  constexpr int NLD = (kFieldRows * KP + kFieldThreads - 1) / kFieldThreads;   // per thread
  __shared__ double ws[2][kFieldRows * kFieldPitch];
  constexpr int kYP = kFieldWaveCols + 4;                 // staged row pitch (floats, 16-B rows)
  constexpr bool ST16 = F32 && FIELD_ST16;
  __shared__ __attribute__((aligned(16))) float ys[ST16 ? kFieldWaves * kFieldRows * kYP : 1];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int li = lane & 15, lk = lane >> 4;
  const long long npanels = (ncols + kFieldCols - 1) / kFieldCols;
  const long long units = npanels * ntiles;
  const long long u0 = units * blockIdx.x / gridDim.x;
  const long long u1 = units * (blockIdx.x + 1) / gridDim.x;
  if (u0 >= u1) return;                                  // block-uniform

  double b[KS][kFieldJT];
  long long cur = -1;                                    // the panel held in b
  auto load_panel = [&](long long panel) {
    const int c0 = (int)panel * kFieldCols + wv * kFieldWaveCols;   // this wave's first column
#pragma unroll
    for (int ks = 0; ks < KS; ++ks)
#pragma unroll
      for (int jt = 0; jt < kFieldJT; ++jt) {
        const int k = 4 * ks + lk, c = c0 + 16 * jt + li;
        b[ks][jt] = (k < P && c < ncols) ? K[(long long)k * ldk + c] : 0.0;
      }
    cur = panel;
  };

  // w tile t -> registers: element e = tid + 256 q is (row e / KP, k e % KP)
  double pre[NLD];
  auto load_tile = [&](long long t) {
    const long long r0 = t * kFieldRows;
#pragma unroll
    for (int q = 0; q < NLD; ++q) {
      const int e = threadIdx.x + kFieldThreads * q;
      const int r = e / KP, k = e % KP;
      pre[q] = (e < kFieldRows * KP && k < P && r0 + r < rows) ? W[(r0 + r) * ldw + k] : 0.0;
    }
  };
  auto store_tile = [&](int buf) {
#pragma unroll
    for (int q = 0; q < NLD; ++q) {
      const int e = threadIdx.x + kFieldThreads * q;
      if (e < kFieldRows * KP) ws[buf][(e / KP) * kFieldPitch + e % KP] = pre[q];
    }
  };

  long long panel = u0 / ntiles, t = u0 - panel * ntiles;  // unit u = panel * ntiles + t
  load_tile(t);
  store_tile(0);
  __syncthreads();
  int buf = 0;
  for (long long u = u0; u < u1; ++u) {
    if (panel != cur) load_panel(panel);
    const bool more = u + 1 < u1;
    const long long tn = t + 1 == ntiles ? 0 : t + 1;
    if (more) load_tile(tn);                             // in flight under the MFMAs
    f64x4 acc[RS][kFieldJT];
#pragma unroll
    for (int rs = 0; rs < RS; ++rs)
#pragma unroll
      for (int jt = 0; jt < kFieldJT; ++jt) acc[rs][jt] = zero4();
    const double* wt = ws[buf];
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
#pragma unroll
      for (int rs = 0; rs < RS; ++rs) {
        const double a = wt[(16 * rs + li) * kFieldPitch + 4 * ks + lk];
#pragma unroll
        for (int jt = 0; jt < kFieldJT; ++jt)
          acc[rs][jt] = mfma16x16x4(a, b[ks][jt], acc[rs][jt]);
      }
    }
    // epilogue: row 16 rs + lk + 4 q, column 16 jt + li of the tile
    const long long r0 = t * kFieldRows;
    const int c0 = (int)panel * kFieldCols + wv * kFieldWaveCols;
    // the back-transform's sd / mu of the wave's 4 columns: read per tile (L1 hits), not
    // held across the K loop (the K panel and accumulators take 192 of the 256 registers)
    double s_c[kFieldJT], m_c[kFieldJT];
#pragma unroll
    for (int jt = 0; jt < kFieldJT; ++jt) {
      const int c = c0 + 16 * jt + li;
      const bool ok = sd != nullptr && c < ncols;
      s_c[jt] = ok ? sd[c] : 1.0;
      m_c[jt] = ok ? mu[c] : 0.0;
    }
    if constexpr (ST16) {
      // the wave's kFieldRows x kFieldWaveCols float32 tile into its LDS slice (same values as
      // the direct path), then back as 16-B row pieces: 8 lanes per 128-B row segment
      float* yw = ys + wv * (kFieldRows * kYP);
#pragma unroll
      for (int rs = 0; rs < RS; ++rs)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int rr = 16 * rs + lk + 4 * q;
          const long long r = r0 + rr;
          const double e = (err && r < rows) ? err[r] : 0.0;
#pragma unroll
          for (int jt = 0; jt < kFieldJT; ++jt) {
            double v = acc[rs][jt][q];
            if (err) v = v + e;
            if (sd) v = fma(v, s_c[jt], m_c[jt]);
            yw[rr * kYP + 16 * jt + li] = static_cast<float>(v);
          }
        }
      constexpr int kPieces = kFieldWaveCols / 4;        // 16-B pieces per row
#pragma unroll
      for (int h = 0; h < kFieldRows * kPieces / 64; ++h) {
        const int idx = lane + 64 * h, rr = idx / kPieces, cc = 4 * (idx % kPieces);
        const f32x4_t v4 = *reinterpret_cast<const f32x4_t*>(yw + rr * kYP + cc);
        const long long r = r0 + rr;
        const int c = c0 + cc;
        if (r >= rows) continue;
        float* yp = static_cast<float*>(Y) + r * ldy + c;
#if FIELD_PROBE == 1
        if (v4[0] == 1234.5f) *yp = v4[1];
#else
        if (vec16 && c + 3 < ncols) {
          __builtin_nontemporal_store(v4, reinterpret_cast<f32x4_t*>(yp));
        } else {
#pragma unroll
          for (int i = 0; i < 4; ++i)
            if (c + i < ncols) __builtin_nontemporal_store(v4[i], yp + i);
        }
#endif
      }
    } else
#pragma unroll
    for (int rs = 0; rs < RS; ++rs)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const long long r = r0 + 16 * rs + lk + 4 * q;
        if (r >= rows) continue;
        const double e = err ? err[r] : 0.0;
#pragma unroll
        for (int jt = 0; jt < kFieldJT; ++jt) {
          const int c = c0 + 16 * jt + li;
          if (c >= ncols) continue;
          double v = acc[rs][jt][q];
          if (err) v = v + e;
          if (sd) v = fma(v, s_c[jt], m_c[jt]);
          if constexpr (F32) {
            float* yp = static_cast<float*>(Y) + r * ldy + c;
            if constexpr (FIELD_NT) __builtin_nontemporal_store(static_cast<float>(v), yp);
            else *yp = static_cast<float>(v);
          } else {
            double* yp = static_cast<double*>(Y) + r * ldy + c;
            if constexpr (FIELD_NT) __builtin_nontemporal_store(v, yp);
            else *yp = v;
          }
        }
      }
    if (more) {
      store_tile(buf ^ 1);                               // the other buffer: last read a tile ago
      __syncthreads();
      buf ^= 1;
    }
    if (tn == 0) ++panel;
    t = tn;
  }
}

int field_num_cus() {
  static const int ncu = [] {
    int dev = 0, n = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
        n <= 0)
      n = 256;
    return n;
  }();
  return ncu;
}

template <int KS, bool F32>
hipError_t launch_field(const double* W, long long ldw, int rows, int P, const double* K,
                        long long ldk, int ncols, const double* sd, const double* mu,
                        const double* err, void* Y, long long ldy, hipStream_t stream) {
  const long long npanels = gp_ceil_div(ncols, kFieldCols);
  constexpr int kFieldRows = field_rows<KS>();
  const long long ntiles = ((long long)rows + kFieldRows - 1) / kFieldRows;
  // one residency round: FIELD_OCC waves per SIMD (launch_bounds' second argument), 4 SIMDs
  long long blocks = (long long)field_num_cus() *
                     (FIELD_OCC * 4 >= kFieldWaves ? FIELD_OCC * 4 / kFieldWaves : 1);
  if (blocks > npanels * ntiles) blocks = npanels * ntiles;
  // 16-B stores need 16-B aligned rows
  const bool vec16 = ((reinterpret_cast<uintptr_t>(Y) & 15) == 0) && (ldy % 4 == 0);
  hipLaunchKernelGGL((field_kernel<KS, F32>), dim3((unsigned)blocks), dim3(kFieldThreads), 0, stream, W,
                     ldw, rows, P, K, ldk, ncols, sd, mu, err, Y, ldy, ntiles, vec16);
  return hipGetLastError();
}

template <bool F32>
hipError_t dispatch_field(const double* W, long long ldw, int rows, int P, const double* K,
                          long long ldk, int ncols, const double* sd, const double* mu,
                          const double* err, void* Y, long long ldy, hipStream_t stream) {
  const int ks = (P + 3) / 4;
  if (ks <= 2)
    return launch_field<2, F32>(W, ldw, rows, P, K, ldk, ncols, sd, mu, err, Y, ldy, stream);
  if (ks <= 4)
    return launch_field<4, F32>(W, ldw, rows, P, K, ldk, ncols, sd, mu, err, Y, ldy, stream);
  if (ks <= 8)
    return launch_field<8, F32>(W, ldw, rows, P, K, ldk, ncols, sd, mu, err, Y, ldy, stream);
  if (ks <= 12)
    return launch_field<12, F32>(W, ldw, rows, P, K, ldk, ncols, sd, mu, err, Y, ldy, stream);
  return launch_field<16, F32>(W, ldw, rows, P, K, ldk, ncols, sd, mu, err, Y, ldy, stream);
}

}  // namespace

extern "C" int gp_field_max_pcs(void) { return kFieldMaxP; }

extern "C" int gp_field(const double* W, long long ldw, int rows, int P, const double* K,
                        long long ldk, int ncols, const double* sd, const double* mu,
                        const double* err, void* Y, long long ldy, int out_f32,
                        hipStream_t stream) {
  if (!W) return -1;
  if (ldw < P || ldw < 1) return -2;
  if (rows < 0) return -3;
  if (P < 1 || P > kFieldMaxP) return -4;
  if (!K) return -5;
  if (ldk < ncols || ldk < 1) return -6;
  if (ncols < 0) return -7;
  if ((sd == nullptr) != (mu == nullptr)) return -8;
  if (!Y) return -11;
  if (ldy < ncols || ldy < 1) return -12;
  if (rows == 0 || ncols == 0) return 0;
  const hipError_t e = out_f32 ? dispatch_field<true>(W, ldw, rows, P, K, ldk, ncols, sd, mu,
                                                      err, Y, ldy, stream)
                               : dispatch_field<false>(W, ldw, rows, P, K, ldk, ncols, sd, mu,
                                                       err, Y, ldy, stream);
  return e == hipSuccess ? 0 : GPFIT_ERR_HIP - (int)e;
}
