// Host-side draw of randomized_svd's Gaussian test matrix exactly as the reference makes it:
// src/svd.py:51 `np.random.normal(size=(n, p + k)).astype(np.float32)` on numpy's global legacy
// RandomState (MT19937 + the polar Box-Muller method, numpy's legacy_gauss), continued from and
// advancing the caller's generator state, so a seeded np.random gives the reference's Omega bit
// for bit and leaves the generator where numpy would.
//
// numpy draws it one deviate at a time (~5 ns each, 0.34 s of init_model's 0.53 s at the fit
// config's 1.35M x 50).  Here the Mersenne Twister runs twist by twist with its 624-word
// recurrence and tempering vectorised (AVX2 when the host has it), the polar method's candidate
// pairs (four words each: two 53-bit doubles) are tested in bulk, and the accepted pairs'
// f = sqrt(-2 log r2 / r2) -- the libm log numpy calls -- and the float32 stores run on worker
// threads while the generator fills the next batch.  No fused multiply-adds anywhere (numpy's
// legacy code is built without): r2 = x1*x1 + x2*x2 must round twice.
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <thread>
#include <vector>
#include "../../include/gpfit.h"

#pragma clang fp contract(off)

namespace {

constexpr int kMtN = 624, kMtM = 397;
constexpr uint32_t kMtA = 0x9908b0dfu, kUpper = 0x80000000u, kLower = 0x7fffffffu;

// One MT19937 generation (numpy's mt19937_gen) then the 624 tempered outputs into w.  The
// recurrence's lag (397 / 227) is far beyond a vector's width, so both loops vectorise.
__attribute__((always_inline)) inline void twist_temper_body(uint32_t* __restrict__ k,
                                                             uint32_t* __restrict__ w) {
  for (int i = 0; i < kMtN - kMtM; ++i) {
    const uint32_t y = (k[i] & kUpper) | (k[i + 1] & kLower);
    k[i] = k[i + kMtM] ^ (y >> 1) ^ ((0u - (y & 1u)) & kMtA);
  }
  for (int i = kMtN - kMtM; i < kMtN - 1; ++i) {
    const uint32_t y = (k[i] & kUpper) | (k[i + 1] & kLower);
    k[i] = k[i + kMtM - kMtN] ^ (y >> 1) ^ ((0u - (y & 1u)) & kMtA);
  }
  const uint32_t y = (k[kMtN - 1] & kUpper) | (k[0] & kLower);
  k[kMtN - 1] = k[kMtM - 1] ^ (y >> 1) ^ ((0u - (y & 1u)) & kMtA);
  for (int i = 0; i < kMtN; ++i) {
    uint32_t t = k[i];
    t ^= t >> 11;
    t ^= (t << 7) & 0x9d2c5680u;
    t ^= (t << 15) & 0xefc60000u;
    t ^= t >> 18;
    w[i] = t;
  }
}
__attribute__((target("avx2"))) void twist_temper_avx2(uint32_t* k, uint32_t* w) {
  twist_temper_body(k, w);
}
void twist_temper_base(uint32_t* k, uint32_t* w) { twist_temper_body(k, w); }

inline uint32_t temper1(uint32_t t) {
  t ^= t >> 11;
  t ^= (t << 7) & 0x9d2c5680u;
  t ^= (t << 15) & 0xefc60000u;
  t ^= t >> 18;
  return t;
}

// numpy's mt19937_next_double from two consecutive words
inline double mt_double(uint32_t a, uint32_t b) {
  return ((double)(int32_t)(a >> 5) * 67108864.0 + (double)(int32_t)(b >> 6)) /
         9007199254740992.0;
}

// Polar-method candidates from nc <= kMaxGroups four-word groups of w: each accepted (x1, x2)
// appended to xy in order.  The tests run as one vectorisable pass, the compaction as a second.
// Returns the count and, in *last, the index of the group that gave the `want`-th acceptance
// (if reached; the compaction stops there).
constexpr int kMaxGroups = (kMtN + 3) / 4 + 1;
__attribute__((always_inline)) inline int accept_body(const uint32_t* __restrict__ w, int nc,
                                                      double* __restrict__ xy, int want,
                                                      int* last) {
  alignas(32) double X1[kMaxGroups], X2[kMaxGroups];
  alignas(32) int ok[kMaxGroups];
  for (int c = 0; c < nc; ++c) {
    const double x1 = 2.0 * mt_double(w[4 * c], w[4 * c + 1]) - 1.0;
    const double x2 = 2.0 * mt_double(w[4 * c + 2], w[4 * c + 3]) - 1.0;
    const double r2 = x1 * x1 + x2 * x2;
    X1[c] = x1;
    X2[c] = x2;
    ok[c] = (r2 < 1.0) & (r2 != 0.0);
  }
  int a = 0;
  for (int c = 0; c < nc; ++c) {
    xy[2 * a] = X1[c];
    xy[2 * a + 1] = X2[c];
    a += ok[c];
    if (a == want) {
      *last = c;
      return a;
    }
  }
  return a;
}
__attribute__((target("avx2"))) int accept_avx2(const uint32_t* w, int nc, double* xy, int want,
                                               int* last) {
  return accept_body(w, nc, xy, want, last);
}
int accept_base(const uint32_t* w, int nc, double* xy, int want, int* last) {
  return accept_body(w, nc, xy, want, last);
}

// Accepted pairs [p0, p1) of xy -> out[base + 2p] = f x2, out[base + 2p + 1] = f x1 (the second
// only below `count`; numpy returns f x2 first and keeps f x1 for the next call).
void transform(const double* xy, long long p0, long long p1, long long pair0, float* out,
               long long base, long long count) {
  for (long long p = p0; p < p1; ++p) {
    const double x1 = xy[2 * p], x2 = xy[2 * p + 1];
    const double r2 = x1 * x1 + x2 * x2;
    const double f = std::sqrt(-2.0 * std::log(r2) / r2);
    const long long o = base + 2 * (pair0 + p);
    out[o] = (float)(f * x2);
    if (o + 1 < count) out[o + 1] = (float)(f * x1);
  }
}

// Worker threads joined on every exit path (a joinable std::thread must not be destroyed).
struct Joiner {
  std::vector<std::thread> t;
  void join() {
    for (auto& x : t)
      if (x.joinable()) x.join();
    t.clear();
  }
  ~Joiner() { join(); }
};

int legacy_normal_impl(uint32_t* key, int* pos, int* has_gauss, double* gauss, long long count,
                       float* out, int nthreads) {
  const bool avx2 = __builtin_cpu_supports("avx2");
  auto twist = avx2 ? twist_temper_avx2 : twist_temper_base;
  auto accept = avx2 ? accept_avx2 : accept_base;

  long long base = 0;
  if (*has_gauss) {            // legacy_gauss: the cached deviate first
    out[0] = (float)*gauss;
    *has_gauss = 0;
    *gauss = 0.0;
    base = 1;
  }
  const long long rest = count - base;
  const long long pairs = (rest + 1) / 2;      // accepted pairs needed
  if (pairs == 0) return 0;

  // stream buffer: up to 3 carried words + the rest of the current twist / a new twist
  std::vector<uint32_t> sbuf(kMtN + 4);
  int carry = 0;
  // batches of accepted pairs, double-buffered against the transform threads
  constexpr long long kBatch = 1 << 20;                 // pairs per batch (16 MB)
  std::vector<double> xy[2] = {std::vector<double>(2 * (kBatch + kMtN)),
                               std::vector<double>(2 * (kBatch + kMtN))};
  Joiner pool;
  auto join = [&] { pool.join(); };
  long long done = 0;          // pairs handed to the transform
  int cur = 0;
  long long fill = 0;          // pairs in xy[cur]
  int p = *pos;
  bool first = true;
  double last_x1 = 0.0, last_x2 = 0.0;
  auto flush = [&](bool final) {
    join();
    const long long n = fill, pair0 = done;
    const double* src = xy[cur].data();
    const int T = (int)std::min<long long>(nthreads, std::max<long long>(1, n / 4096));
    for (int t = 0; t < T; ++t) {
      const long long a = n * t / T, b = n * (t + 1) / T;
      pool.t.emplace_back(transform, src, a, b, pair0, out, base, count);
    }
    done += n;
    fill = 0;
    cur ^= 1;
    if (final) join();
  };
  for (;;) {
    int nw;
    if (first && p < kMtN) {
      // the rest of the caller's current twist
      for (int i = p; i < kMtN; ++i) sbuf[i - p] = temper1(key[i]);
      nw = kMtN - p;
    } else {
      twist(key, sbuf.data() + carry);
      nw = carry + kMtN;
      p = 0;
    }
    const bool was_first = first && p != 0;
    first = false;
    const int nc = nw / 4;
    const long long want = pairs - done - fill;
    int last = -1;
    const int got = accept(sbuf.data(), nc, xy[cur].data() + 2 * fill,
                           (int)std::min<long long>(want, 1ll << 30), &last);
    fill += got;
    if (got == want) {
      // the final pair: state ends after its fourth word
      const int end_word = 4 * last + 4;                 // words of sbuf consumed
      last_x1 = xy[cur][2 * (fill - 1)];
      last_x2 = xy[cur][2 * (fill - 1) + 1];
      if (was_first) {
        *pos = p + end_word;
      } else {
        *pos = end_word - carry;                         // >= 1: the group ends in this twist
      }
      break;
    }
    // carry the incomplete group's words into the next twist's buffer
    const int used = 4 * nc;
    carry = nw - used;
    if (carry) std::memmove(sbuf.data(), sbuf.data() + used, carry * sizeof(uint32_t));
    if (was_first) p = kMtN;
    if (fill >= kBatch) flush(false);
  }
  flush(true);
  if (rest % 2 == 1) {         // odd: numpy keeps the last pair's f x1 for its next call
    const double r2 = last_x1 * last_x1 + last_x2 * last_x2;
    const double f = std::sqrt(-2.0 * std::log(r2) / r2);
    *has_gauss = 1;
    *gauss = f * last_x1;
  }
  return 0;
}

}  // namespace

extern "C" int gp_host_legacy_normal_f32(unsigned int* key, int* pos, int* has_gauss, double* gauss,
                                         long long count, float* out, int nthreads) {
  if (!key || !pos || !has_gauss || !gauss) return -1;
  if (*pos < 0 || *pos > kMtN) return -2;
  if (count < 0) return -5;
  if (count > 0 && !out) return -6;
  if (count == 0) return 0;
  if (nthreads < 1) nthreads = 1;
  try {
    return legacy_normal_impl(key, pos, has_gauss, gauss, count, out, nthreads);
  } catch (...) {   // thread or buffer allocation failed: nothing escapes the C ABI
    return -7;
  }
}
