// Debug helper (tools/prof_bcast_contention.py): a stand-in for the RCCL broadcast kernel that
// runs beside the prediction at N > 1 (rank 0 ships the next GP's packed L^-1, 67 MB at
// n = 4096, while every rank's TRMM runs).  RCCL moves a broadcast with one workgroup per
// channel copying through the ring; here `wgs` workgroups of 256 threads copy `bytes` from src
// to dst in 16-B vectors, each workgroup a contiguous slice, optionally throttled with s_sleep
// between 64 KB pieces so that the copy lasts about as long as an xGMI transfer would (the
// one-GPU box has no peer).  Not part of libgpfit.
//   hipcc --offload-arch=gfx950 -O3 -shared -fPIC -o tools/dbg/libbcast_standin.so \
//       tools/dbg/bcast_standin.hip
#include <hip/hip_runtime.h>

__global__ __launch_bounds__(256) void standin_copy_kernel(const int4* __restrict__ src,
                                                           int4* __restrict__ dst,
                                                           long long n16, int sleep_iters) {
  const long long per = (n16 + gridDim.x - 1) / gridDim.x;
  const long long a = blockIdx.x * per;
  const long long b = a + per < n16 ? a + per : n16;
  constexpr int kPiece = 4096;                       // 16-B vectors per throttle piece (64 KB)
  for (long long p = a; p < b; p += kPiece) {
    const long long e = p + kPiece < b ? p + kPiece : b;
    for (long long i = p + threadIdx.x; i < e; i += 256) dst[i] = src[i];
    for (int s = 0; s < sleep_iters; ++s) __builtin_amdgcn_s_sleep(127);
  }
}

extern "C" int standin_copy(const void* src, void* dst, long long bytes, int wgs,
                            int sleep_iters, hipStream_t stream) {
  if (!src || !dst || bytes <= 0 || (bytes & 15) || wgs < 1) return -1;
  hipLaunchKernelGGL(standin_copy_kernel, dim3(wgs), dim3(256), 0, stream,
                     static_cast<const int4*>(src), static_cast<int4*>(dst), bytes / 16,
                     sleep_iters);
  return hipGetLastError() == hipSuccess ? 0 : -2;
}
