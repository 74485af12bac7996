// RCCL over xGMI for the sharded emulator (gp_comm_init / gp_bcast / gp_gather;
// §8e: one broadcast of the inputs, one gather of the (mean, var) shards).
//
// One communicator per process / GPU (torchrun's layout).  librccl is resolved at run time with
// dlopen, so libgpfit loads, and its GP kernels run, where RCCL is absent; only gp_comm_* then
// return GPFIT_ERR_RCCL.  When PyTorch has already loaded RCCL, dlopen of the same soname
// returns that copy.
//
// The reference has no distributed code; these wrappers are what a C / ctypes
// caller of libgpfit uses instead of torch.distributed to shard (sample, PC) GPs over ranks.
#include "gpfit_common.h"
#include "../../include/gpfit.h"

#include <cstring>
#include <dlfcn.h>
#include <mutex>
#include <rccl/rccl.h>

namespace {

struct Api {
  decltype(&ncclGetUniqueId) get_unique_id = nullptr;
  decltype(&ncclCommInitRank) init_rank = nullptr;
  decltype(&ncclCommDestroy) destroy = nullptr;
  decltype(&ncclBroadcast) broadcast = nullptr;
  decltype(&ncclSend) send = nullptr;
  decltype(&ncclRecv) recv = nullptr;
  decltype(&ncclGroupStart) group_start = nullptr;
  decltype(&ncclGroupEnd) group_end = nullptr;
  bool ok = false;
};

std::mutex g_mu;
Api g_api;
bool g_tried = false;

const Api* api() {
  std::lock_guard<std::mutex> lk(g_mu);
  if (!g_tried) {
    g_tried = true;
    void* h = dlopen("librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
    if (!h) h = dlopen("librccl.so", RTLD_NOW | RTLD_GLOBAL);
    if (h) {
      Api a;
      a.get_unique_id = (decltype(a.get_unique_id))dlsym(h, "ncclGetUniqueId");
      a.init_rank = (decltype(a.init_rank))dlsym(h, "ncclCommInitRank");
      a.destroy = (decltype(a.destroy))dlsym(h, "ncclCommDestroy");
      a.broadcast = (decltype(a.broadcast))dlsym(h, "ncclBroadcast");
      a.send = (decltype(a.send))dlsym(h, "ncclSend");
      a.recv = (decltype(a.recv))dlsym(h, "ncclRecv");
      a.group_start = (decltype(a.group_start))dlsym(h, "ncclGroupStart");
      a.group_end = (decltype(a.group_end))dlsym(h, "ncclGroupEnd");
      a.ok = a.get_unique_id && a.init_rank && a.destroy && a.broadcast && a.send && a.recv &&
             a.group_start && a.group_end;
      g_api = a;
    }
  }
  return g_api.ok ? &g_api : nullptr;
}

struct Comm {
  ncclComm_t c;
  int nranks, rank;
};

int rc_of(ncclResult_t r) { return r == ncclSuccess ? 0 : GPFIT_ERR_RCCL - (int)r; }

}  // namespace

extern "C" int gp_comm_available(void) { return api() ? 1 : 0; }

extern "C" int gp_comm_unique_id(void* id) {
  if (!id) return -1;
  const Api* a = api();
  if (!a) return GPFIT_ERR_RCCL;
  ncclUniqueId u;
  const int rc = rc_of(a->get_unique_id(&u));
  if (rc) return rc;
  memcpy(id, &u, sizeof(u));
  return 0;
}

extern "C" int gp_comm_init(int nranks, int rank, const void* id, void** comm) {
  if (nranks < 1) return -1;
  if (rank < 0 || rank >= nranks) return -2;
  if (!id) return -3;
  if (!comm) return -4;
  const Api* a = api();
  if (!a) return GPFIT_ERR_RCCL;
  ncclUniqueId u;
  memcpy(&u, id, sizeof(u));
  ncclComm_t c = nullptr;
  const int rc = rc_of(a->init_rank(&c, nranks, u, rank));
  if (rc) return rc;
  *comm = new Comm{c, nranks, rank};
  return 0;
}

extern "C" int gp_comm_destroy(void* comm) {
  if (!comm) return -1;
  const Api* a = api();
  Comm* c = static_cast<Comm*>(comm);
  const int rc = a ? rc_of(a->destroy(c->c)) : GPFIT_ERR_RCCL;
  delete c;
  return rc;
}

extern "C" int gp_bcast(void* comm, void* buf, long long bytes, int root, hipStream_t stream) {
  if (!comm) return -1;
  if (!buf && bytes > 0) return -2;
  if (bytes < 0) return -3;
  Comm* c = static_cast<Comm*>(comm);
  if (root < 0 || root >= c->nranks) return -4;
  if (bytes == 0) return 0;
  const Api* a = api();
  if (!a) return GPFIT_ERR_RCCL;
  return rc_of(a->broadcast(buf, buf, (size_t)bytes, ncclInt8, root, c->c, stream));
}

extern "C" int gp_gather(void* comm, const void* send, long long bytes, void* recv, int root,
                         hipStream_t stream) {
  if (!comm) return -1;
  if (!send && bytes > 0) return -2;
  if (bytes < 0) return -3;
  Comm* c = static_cast<Comm*>(comm);
  if (c->rank == root && !recv && bytes > 0) return -4;
  if (root < 0 || root >= c->nranks) return -5;
  if (bytes == 0) return 0;
  const Api* a = api();
  if (!a) return GPFIT_ERR_RCCL;
  // NCCL has no gather: the root posts one receive per peer and every other rank one send, in
  // one group (point-to-point over xGMI, no all-to-all)
  if (c->rank == root) {
    char* r = static_cast<char*>(recv);
    const hipError_t e = hipMemcpyAsync(r + (long long)root * bytes, send, (size_t)bytes,
                                        hipMemcpyDeviceToDevice, stream);
    if (e != hipSuccess) return GPFIT_ERR_HIP - (int)e;
    if (c->nranks == 1) return 0;
    int rc = rc_of(a->group_start());
    if (rc) return rc;
    for (int p = 0; p < c->nranks && !rc; ++p)
      if (p != root)
        rc = rc_of(a->recv(r + (long long)p * bytes, (size_t)bytes, ncclInt8, p, c->c, stream));
    const int rc2 = rc_of(a->group_end());
    return rc ? rc : rc2;
  }
  int rc = rc_of(a->group_start());
  if (rc) return rc;
  rc = rc_of(a->send(send, (size_t)bytes, ncclInt8, root, c->c, stream));
  const int rc2 = rc_of(a->group_end());
  return rc ? rc : rc2;
}

// ---- Lower-triangle packing for the single-GP L^-1 broadcast (sharded.py) -------------------
// Column c of a column-major n x n buffer, rows c .. n-1, goes to out[c n - c (c - 1) / 2 ...]:
// n (n + 1) / 2 doubles, about half the padded square the prediction reads.  One block per
// column, lane-consecutive 8-B accesses (a wave moves 512 contiguous bytes each way).
namespace {
__global__ __launch_bounds__(256) void tril_copy_kernel(const double* __restrict__ A, int n,
                                                        long long ld, double* __restrict__ v,
                                                        int unpack) {
  const int c = blockIdx.x;
  const long long off = (long long)c * n - (long long)c * (c - 1) / 2;
  const int len = n - c;
  double* col = const_cast<double*>(A) + (long long)c * ld + c;
  if (!unpack) {
    for (int e = threadIdx.x; e < len; e += 256) v[off + e] = col[e];
  } else {
    for (int e = threadIdx.x; e < len; e += 256) col[e] = v[off + e];
  }
}
}  // namespace

extern "C" int gp_pack_tril(const double* A, int n, int ld, double* out, hipStream_t stream) {
  if (!A) return -1;
  if (n < 0) return -2;
  if (ld < n || ld < 1) return -3;
  if (!out) return -4;
  if (n == 0) return 0;
  hipLaunchKernelGGL(tril_copy_kernel, dim3(n), dim3(256), 0, stream, A, n, (long long)ld, out,
                     0);
  const hipError_t e = hipGetLastError();
  return e == hipSuccess ? 0 : GPFIT_ERR_HIP - (int)e;
}

extern "C" int gp_unpack_tril(const double* in, int n, double* A, int ld, hipStream_t stream) {
  if (!in) return -1;
  if (n < 0) return -2;
  if (!A) return -3;
  if (ld < n || ld < 1) return -4;
  if (n == 0) return 0;
  hipLaunchKernelGGL(tril_copy_kernel, dim3(n), dim3(256), 0, stream, A, n, (long long)ld,
                     const_cast<double*>(in), 1);
  const hipError_t e = hipGetLastError();
  return e == hipSuccess ? 0 : GPFIT_ERR_HIP - (int)e;
}
