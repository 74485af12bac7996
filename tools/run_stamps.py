"""Diagnostic: per-phase cycles of the diagonal factorisation (stamps build)."""
import ctypes, os, sys
import numpy as np
import torch
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from gladsgp_amd import _capi
lib = ctypes.CDLL(os.path.join(ROOT, "tools", "libgpfit_stamps.so"))
for name, (res, args) in _capi.SIGNATURES.items():
    getattr(lib, name).restype = res; getattr(lib, name).argtypes = args
_capi._LIB = lib
from gladsgp_amd import kernels
dev = torch.device("cuda:0")
n = 64
X = torch.as_tensor(np.random.default_rng(0).random((n, 8)), device=dev)
beta = torch.as_tensor(np.random.default_rng(3).uniform(0.5, 5, 8), device=dev)
G = kernels.gram(X, beta, 1.0, 1e-3)
for _ in range(5):
    ch = kernels.cholesky_inverse(G.clone())
torch.cuda.synchronize()
h = (ctypes.c_ulonglong * 16)()
lib.gp_diag_stamps(h)
for w in range(4):
    print(f"wave {w}: barrier {h[4*w]/64:8.0f}  reads {h[4*w+1]/64:8.0f}  fma {h[4*w+2]/64:8.0f}  publish {h[4*w+3]/64:8.0f}  cycles/step")
