// CU-mask probe: where do a stream's workgroups land for a given hipExtStreamCreateWithCUMask
// mask?  Each workgroup records HW_ID / XCC_ID and spins ~20 us so the grid spreads over every
// CU the mask allows.  Prints, per mask, the number of distinct CUs used, per-XCC counts and
// the launch time.  Used to choose the spatial split of gp_fit_predict's pipelined mode.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <set>
#include <vector>
#define CK(x) do{hipError_t e=(x); if(e!=hipSuccess){printf("HIP error %s line %d\n",hipGetErrorString(e),__LINE__); return 1;}}while(0)

__global__ void where(unsigned* out, int spin_ticks) {
  const unsigned hw = __builtin_amdgcn_s_getreg((31 << 11) | 4);    // HW_REG_HW_ID
  const unsigned xcc = __builtin_amdgcn_s_getreg((31 << 11) | 20);  // HW_REG_XCC_ID
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  while (__builtin_amdgcn_s_memrealtime() - t0 < (unsigned long long)spin_ticks) {}
  if (threadIdx.x == 0) { out[2 * blockIdx.x] = hw; out[2 * blockIdx.x + 1] = xcc; }
}

static int run(const char* name, const std::vector<unsigned>& mask, unsigned* d, int nblk) {
  hipStream_t s;
  if (mask.empty()) CK(hipStreamCreate(&s));
  else CK(hipExtStreamCreateWithCUMask(&s, (unsigned)mask.size(), mask.data()));
  unsigned got[8] = {0};
  CK(hipExtStreamGetCUMask(s, 8, got));
  hipEvent_t a, b; CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
  CK(hipEventRecord(a, s));
  hipLaunchKernelGGL(where, dim3(nblk), dim3(64), 0, s, d, 2000);  // 20 us per workgroup
  CK(hipEventRecord(b, s));
  CK(hipStreamSynchronize(s));
  float ms; CK(hipEventElapsedTime(&ms, a, b));
  std::vector<unsigned> h(2 * nblk);
  CK(hipMemcpy(h.data(), d, 8 * nblk, hipMemcpyDeviceToHost));
  std::set<unsigned> cus; int per_xcc[16] = {0}; std::set<unsigned> cu_x[16];
  for (int i = 0; i < nblk; ++i) {
    unsigned hw = h[2 * i], x = h[2 * i + 1] & 15;
    unsigned key = (x << 8) | (((hw >> 13) & 7) << 5) | (((hw >> 12) & 1) << 4) | ((hw >> 8) & 15);
    cus.insert(key); per_xcc[x]++; cu_x[x].insert(key);
  }
  printf("%-22s got-mask %08x %08x %08x %08x %08x %08x %08x %08x  %.3f ms  distinct CUs %zu  per-XCC wg/CUs:",
         name, got[0], got[1], got[2], got[3], got[4], got[5], got[6], got[7], ms, cus.size());
  for (int x = 0; x < 8; ++x) printf(" %d/%zu", per_xcc[x], cu_x[x].size());
  printf("\n");
  CK(hipStreamDestroy(s));
  return 0;
}

int main() {
  hipDeviceProp_t p; CK(hipGetDeviceProperties(&p, 0));
  printf("CUs %d\n", p.multiProcessorCount);
  const int nblk = 4096;
  unsigned* d; CK(hipMalloc(&d, 8 * nblk));
  auto bits = [](std::vector<int> idx) { std::vector<unsigned> m(8, 0); for (int i : idx) m[i / 32] |= 1u << (i % 32); return m; };
  auto comp = [](std::vector<unsigned> m) { for (auto& w : m) w = ~w; return m; };
  std::vector<int> bal, low, grp;
  for (int x = 0; x < 8; ++x) { bal.push_back(32 * x + x); bal.push_back(32 * x + x + 8); }
  for (int i = 0; i < 16; ++i) low.push_back(i);
  for (int x = 0; x < 8; ++x) { grp.push_back(32 * x); grp.push_back(32 * x + 1); }
  if (run("default", {}, d, nblk)) return 1;
  if (run("all", std::vector<unsigned>(8, ~0u), d, nblk)) return 1;
  if (run("balanced16", bits(bal), d, nblk)) return 1;
  if (run("~balanced16", comp(bits(bal)), d, nblk)) return 1;
  if (run("low16", bits(low), d, nblk)) return 1;
  if (run("grp16", bits(grp), d, nblk)) return 1;
  if (run("low8", bits({0, 1, 2, 3, 4, 5, 6, 7}), d, nblk)) return 1;
  return 0;
}
