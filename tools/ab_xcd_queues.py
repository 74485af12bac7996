"""Same-process A/B of the persistent factorisation's task queues (VERDICT r04 Next #4): per-XCD
queues (gp_set_potrf_path(0), batches of 8k) vs one shared queue (path 2), interleaved rounds,
median HIP-event time of gp_potrf_inv_ws (L + L^-1) and gp_potrf_ws (L only, the fit's
likelihood) per shape.  n = 4096 x 1 is the control (one queue either way).

    python tools/ab_xcd_queues.py
"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gladsgp_amd import _capi, kernels  # noqa: E402

dev = torch.device("cuda:0")
st = torch.cuda.current_stream(dev).cuda_stream
lib = _capi.lib()


def setup(n, B):
    X = torch.as_tensor(np.random.default_rng(0).random((n, 8)), device=dev)
    betas = torch.as_tensor(np.random.default_rng(1).uniform(0.5, 5, (B, 8)), device=dev)
    G0 = kernels.gram(X, betas, 1.0, 1e-6, batch=B)
    npad = kernels.padded_n(n)
    bufs = dict(G0=G0, A=torch.empty_like(G0),
                Linv=torch.empty((B, npad, npad), dtype=torch.float64, device=dev),
                info=torch.empty(B, dtype=torch.int32, device=dev),
                logdet=torch.empty(B, dtype=torch.float64, device=dev))
    wsb = max(int(lib.gp_potrf_inv_ws_bytes(n, B)), int(lib.gp_potrf_ws_bytes(n, B)))
    bufs["ws"] = torch.empty(max(wsb, 256), dtype=torch.uint8, device=dev)
    return bufs


def one(n, B, b, mode):
    b["A"].copy_(b["G0"])
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    if mode == "inv":
        npad = kernels.padded_n(n)
        _capi.call("gp_potrf_inv_ws", b["A"].data_ptr(), n, n, n * n, b["Linv"].data_ptr(), npad,
                   npad * npad, B, b["info"].data_ptr(), b["logdet"].data_ptr(),
                   b["ws"].data_ptr(), b["ws"].numel(), st)
    else:
        _capi.call("gp_potrf_ws", b["A"].data_ptr(), n, n, n * n, B, b["info"].data_ptr(),
                   b["logdet"].data_ptr(), b["ws"].data_ptr(), b["ws"].numel(), st)
    e1.record()
    torch.cuda.synchronize()
    assert int(b["info"].abs().max()) == 0
    return e0.elapsed_time(e1)


prev = lib.gp_set_potrf_path(0)
for n, B in ((512, 24), (1024, 32), (512, 8), (512, 128), (4096, 1)):
    b = setup(n, B)
    for mode in ("inv", "l"):
        res = {0: [], 2: []}
        for rnd in range(6):
            for path in ((0, 2) if rnd % 2 == 0 else (2, 0)):
                lib.gp_set_potrf_path(path)
                ts = [one(n, B, b, mode) for _ in range(8)]
                res[path].append(float(np.median(ts[2:])))
        lib.gp_set_potrf_path(0)
        m0, m2 = np.median(res[0]), np.median(res[2])
        print(f"n={n:5d} batch={B:4d} {'potrf_inv' if mode == 'inv' else 'potrf    '}: "
              f"per-XCD queues {m0 * 1e3:8.1f} us  shared queue {m2 * 1e3:8.1f} us  "
              f"(x{m0 / m2:.3f})  rounds {np.round(np.array(res[0]) * 1e3, 1).tolist()} vs "
              f"{np.round(np.array(res[2]) * 1e3, 1).tolist()}", flush=True)
lib.gp_set_potrf_path(prev)
