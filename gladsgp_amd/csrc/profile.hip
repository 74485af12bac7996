// Optional in-library kernel timing with HIP events (off by default).
//
// When enabled, each instrumented launch records a start/stop hipEvent pair on the stream
// the kernel runs on, so bench.py can read per-kernel device time over its timed region
// without a profiler.  Host-side, single-threaded use; recording never synchronises.
#include "gpfit_common.h"
#include "gpfit_profile.h"
#include "../../include/gpfit.h"

#include <vector>

namespace {

struct Slot {
  std::vector<hipEvent_t> start, stop;
  std::vector<int> launches;   // launches bracketed by each pair
  int used = 0;
};

bool g_enabled = false;
unsigned g_mask = ~0u;             // kernels that record (gp_profile_select)
Slot g_slots[GP_PROF_NUM];

}  // namespace

void gpfit_prof_begin_n(int id, hipStream_t st, int launches) {
  if (!g_enabled || id < 0 || id >= GP_PROF_NUM || !(g_mask >> id & 1u)) return;
  Slot& s = g_slots[id];
  if (s.used >= (int)s.start.size()) return;   // capacity exhausted: stop recording
  s.launches[s.used] = launches > 0 ? launches : 1;
  (void)hipEventRecord(s.start[s.used], st);
}

void gpfit_prof_begin(int id, hipStream_t st) { gpfit_prof_begin_n(id, st, 1); }

void gpfit_prof_end(int id, hipStream_t st) {
  if (!g_enabled || id < 0 || id >= GP_PROF_NUM || !(g_mask >> id & 1u)) return;
  Slot& s = g_slots[id];
  if (s.used >= (int)s.start.size()) return;
  (void)hipEventRecord(s.stop[s.used], st);
  ++s.used;
}

extern "C" int gp_profile_enable(int capacity) {
  if (capacity < 0) return -1;
  for (auto& s : g_slots) {
    for (auto e : s.start) (void)hipEventDestroy(e);
    for (auto e : s.stop) (void)hipEventDestroy(e);
    s.start.clear();
    s.stop.clear();
    s.launches.assign(capacity, 1);
    s.used = 0;
    for (int i = 0; i < capacity; ++i) {
      hipEvent_t a, b;
      hipError_t e1 = hipEventCreate(&a), e2 = hipEventCreate(&b);
      if (e1 != hipSuccess) return GPFIT_ERR_HIP - (int)e1;
      if (e2 != hipSuccess) return GPFIT_ERR_HIP - (int)e2;
      s.start.push_back(a);
      s.stop.push_back(b);
    }
  }
  g_enabled = capacity > 0;
  return 0;
}

extern "C" unsigned gp_profile_select(unsigned mask) {
  const unsigned old = g_mask;
  g_mask = mask;
  return old;
}

extern "C" int gp_profile_reset(void) {
  for (auto& s : g_slots) s.used = 0;
  return 0;
}

extern "C" int gp_profile_read(int id, int* count, double* total_ms, double* max_ms) {
  if (id < 0 || id >= GP_PROF_NUM) return -1;
  Slot& s = g_slots[id];
  double tot = 0.0, mx = 0.0;
  int cnt = 0;
  for (int i = 0; i < s.used; ++i) {
    hipError_t e = hipEventSynchronize(s.stop[i]);
    if (e != hipSuccess) return GPFIT_ERR_HIP - (int)e;
    float ms = 0.f;
    e = hipEventElapsedTime(&ms, s.start[i], s.stop[i]);
    if (e != hipSuccess) return GPFIT_ERR_HIP - (int)e;
    tot += ms;
    cnt += s.launches[i];
    if (ms / s.launches[i] > mx) mx = ms / s.launches[i];
  }
  if (count) *count = cnt;
  if (total_ms) *total_ms = tot;
  if (max_ms) *max_ms = mx;
  return 0;
}
