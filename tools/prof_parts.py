"""Per-kernel device times (HIP events the library records, gp_profile_*) for the pieces of a
step, each alone on an idle GPU:
  * lower-triangle Gram at n (the factorising callers' form; gp_fit_predict's GP_PROF_GRAM);
  * cross-covariance of m test points (gp_predict_cross, all chunks, all CUs);
  * C4's batched cross-covariance (32 GPs, n = 1024, one 4096-point chunk).
    python tools/prof_parts.py [n] [m]
"""
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gladsgp_amd import _capi, kernels  # noqa: E402

dev = torch.device("cuda:0")
n = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
m = int(sys.argv[2]) if len(sys.argv) > 2 else 100000
T = lambda a: torch.as_tensor(np.ascontiguousarray(a), device=dev)  # noqa: E731


def prof(pid):
    c, t, mx = ctypes.c_int(0), ctypes.c_double(0), ctypes.c_double(0)
    _capi.call("gp_profile_read", pid, ctypes.addressof(c), ctypes.addressof(t),
               ctypes.addressof(mx))
    return c.value, t.value


X = T(np.random.default_rng(0).random((n, 8)))
beta = T(np.random.default_rng(3).uniform(0.5, 5, 8))
w = T(np.sin(np.random.default_rng(1).random(n)))
Xs = T(np.random.default_rng(2).random((m, 8)))
reps = 20
_capi.call("gp_profile_enable", 4096)
# lower Gram inside gp_fit_predict (serial path, few test points)
ws = kernels.Workspace()
for _ in range(3):
    kernels.fit_predict(X, Xs[:128], beta, 1.0, 1e-6, 1.0, w, workspace=ws, check=False)
torch.cuda.synchronize()
_capi.call("gp_profile_reset")
for _ in range(reps):
    kernels.fit_predict(X, Xs[:128], beta, 1.0, 1e-6, 1.0, w, workspace=ws, check=False)
torch.cuda.synchronize()
c, t = prof(_capi.PROF_GRAM)
g_us = 1e3 * t / max(c, 1)
g_bytes = 4.0 * n * (n + 1)
print(f"lower Gram n={n}: {g_us:7.2f} us/launch ({c} launches)  "
      f"{g_bytes / g_us / 1e3:7.1f} GB/s of its 4n(n+1) B", flush=True)
c, t = prof(_capi.PROF_POTRF)
print(f"factorisation n={n}: {1e3 * t / max(c, 1):8.1f} us/call", flush=True)
# cross-covariance of all m points on all CUs
pws = kernels.Workspace()
for _ in range(2):
    kernels.predict_prepare(X, Xs, beta, 1.0, workspace=pws)
torch.cuda.synchronize()
_capi.call("gp_profile_reset")
for _ in range(5):
    kernels.predict_prepare(X, Xs, beta, 1.0, workspace=pws)
torch.cuda.synchronize()
c, t = prof(_capi.PROF_CROSS)
npad = kernels.padded_n(n)
print(f"cross n={n} m={m}: {t / 5:7.3f} ms per {m} points ({c // 5} chunks)  "
      f"{8.0 * npad * m / (t / 5 * 1e-3) / 1e9:7.1f} GB/s", flush=True)
# C4: 32 GPs, n = 1024, one 4096-point chunk
B, n4 = 32, 1024
X4 = T(np.random.default_rng(0).random((n4, 8)))
b4 = T(np.stack([np.random.default_rng(10 + j).uniform(0.5, 5, 8) for j in range(B)]))
s4 = T(np.ones(B))
for _ in range(2):
    kernels.predict_prepare(X4, Xs[:4096], b4, s4, batch=B, workspace=pws)
torch.cuda.synchronize()
_capi.call("gp_profile_reset")
for _ in range(10):
    kernels.predict_prepare(X4, Xs[:4096], b4, s4, batch=B, workspace=pws)
torch.cuda.synchronize()
c, t = prof(_capi.PROF_CROSS)
print(f"C4 cross (32 GPs x 1024 x 4096 pts): {1e3 * t / 10:7.1f} us per chunk "
      f"({8.0 * B * n4 * 4096 / (t / 10 * 1e-3) / 1e9:7.1f} GB/s); x25 chunks = "
      f"{25 * t / 10:6.2f} ms", flush=True)
_capi.call("gp_profile_enable", 0)
