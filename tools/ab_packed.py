"""Same-process A/B of the TRMM reading L^-1 padded vs tile-packed (gp_predict_ex with z given, so
no trmv): interleaved rounds, per-launch TRMM device time from the library's own HIP events
(gp_profile_*), at the N = 8 rank block (13,408 points) and one full 16,384-point chunk.

    python tools/ab_packed.py
"""
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gladsgp_amd import _capi, kernels  # noqa: E402
from gladsgp_amd.sharded import LinvPacker  # noqa: E402

dev = torch.device("cuda:0")
n, d = 4096, 8
rng = np.random.default_rng(0)
X = torch.as_tensor(rng.random((n, d)), device=dev)
Xs = torch.as_tensor(rng.random((16384, d)), device=dev)
beta = torch.as_tensor(rng.uniform(0.5, 5, (1, d)), device=dev)
w = torch.as_tensor(np.sin(rng.random(n) * 6), device=dev).reshape(1, n)
ch = kernels.cholesky_inverse(kernels.gram(X, beta, 1.0, 1e-6))
ch.check()
npad = kernels.padded_n(n)
packer = LinvPacker(npad, dev, n=n)
payload = packer.buffer(dev)
packer.pack(ch.linv_buf, ch.info, payload, w=w)
view = packer.view(payload)
z = packer.z(payload).view(1, npad)
ws = kernels.Workspace()
_capi.call("gp_profile_enable", 4096)


def trmm_ms(src, pts, reps=5):
    Xc = Xs[:pts].contiguous()
    kernels.predict(src, X, Xc, beta, 1.0, 1.0, None, workspace=ws, z=z)
    torch.cuda.synchronize()
    _capi.call("gp_profile_reset")
    for _ in range(reps):
        kernels.predict(src, X, Xc, beta, 1.0, 1.0, None, workspace=ws, z=z)
    torch.cuda.synchronize()
    c, t, mx = ctypes.c_int(0), ctypes.c_double(0), ctypes.c_double(0)
    _capi.call("gp_profile_read", _capi.PROF_TRMM, ctypes.addressof(c), ctypes.addressof(t),
               ctypes.addressof(mx))
    return t.value / max(c.value, 1)


for pts in (13408, 16384):
    res = {"padded": [], "packed": []}
    for rnd in range(6):
        for name, src in (("padded", ch), ("packed", view)) if rnd % 2 == 0 else \
                (("packed", view), ("padded", ch)):
            res[name].append(trmm_ms(src, pts))
    mp, mk = np.median(res["padded"]), np.median(res["packed"])
    print(f"{pts} points: TRMM per launch padded {mp:.4f} ms, packed {mk:.4f} ms "
          f"(x{mk / mp:.3f}); rounds padded {np.round(res['padded'], 4).tolist()} packed "
          f"{np.round(res['packed'], 4).tolist()}", flush=True)
