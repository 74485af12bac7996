"""The factorisation with and without the inverse (VERDICT r03 Next #2's A/B): gp_potrf_inv_ws
(L and L^-1: the XT tasks included) vs gp_potrf_ws (L only, the persistent kernel without XT
tasks), median of HIP-event times over 10 calls, at n = 4096 (C3), n = 1024 x 32 (C4's batch)
and n = 512 x 8 (the fit's likelihood batch).

    python tools/prof_potrf_modes.py
"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gladsgp_amd import _capi, kernels  # noqa: E402

dev = torch.device("cuda:0")
st = torch.cuda.current_stream(dev).cuda_stream
for n, B in ((4096, 1), (1024, 32), (512, 8)):
    X = torch.as_tensor(np.random.default_rng(0).random((n, 8)), device=dev)
    betas = torch.as_tensor(np.stack([np.random.default_rng(10 + b).uniform(0.5, 5, 8)
                                      for b in range(B)]), device=dev)
    G0 = kernels.gram(X, betas, 1.0, 1e-6, batch=B)
    npad = kernels.padded_n(n)
    A = torch.empty_like(G0)
    Linv = torch.empty((B, npad, npad), dtype=torch.float64, device=dev)
    info = torch.empty(B, dtype=torch.int32, device=dev)
    logdet = torch.empty(B, dtype=torch.float64, device=dev)
    wsb = max(int(_capi.lib().gp_potrf_inv_ws_bytes(n, B)), int(_capi.lib().gp_potrf_ws_bytes(n, B)))
    ws = torch.empty(max(wsb, 256), dtype=torch.uint8, device=dev)
    res = {}
    for mode in ("potrf_inv", "potrf"):
        ts = []
        for rep in range(12):
            A.copy_(G0)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            if mode == "potrf_inv":
                _capi.call("gp_potrf_inv_ws", A.data_ptr(), n, n, n * n, Linv.data_ptr(), npad,
                           npad * npad, B, info.data_ptr(), logdet.data_ptr(), ws.data_ptr(),
                           ws.numel(), st)
            else:
                _capi.call("gp_potrf_ws", A.data_ptr(), n, n, n * n, B, info.data_ptr(),
                           logdet.data_ptr(), ws.data_ptr(), ws.numel(), st)
            e1.record()
            torch.cuda.synchronize()
            assert int(info.abs().max()) == 0
            if rep >= 2:
                ts.append(e0.elapsed_time(e1))
        res[mode] = float(np.median(ts))
    print(f"n={n} batch={B}: potrf_inv (L + L^-1) {res['potrf_inv']:.3f} ms | potrf (L only) "
          f"{res['potrf']:.3f} ms | inverse share {1 - res['potrf'] / res['potrf_inv']:.2f}",
          flush=True)
