"""Same-box A/B of the factorisation between library builds (box-to-box variance is larger
than the differences being measured): every library given is loaded into this one process
(ctypes, RTLD_LOCAL: each keeps its own code objects), and gp_potrf_inv_ws runs on the same
Grams in interleaved rounds, timed with HIP events on the current stream.

    python tools/ab_libs.py libA.so libB.so [...]
Prints per library the median ms per call at n = 4096 (one GP) and n = 1024 x 32 (C4's batch),
and the max |L^-1 difference| against the first library."""
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gladsgp_amd import kernels  # noqa: E402  (torch's HIP runtime first)

libs = []
for path in sys.argv[1:]:
    h = ctypes.CDLL(os.path.abspath(path))
    if not hasattr(h, "gp_potrf_inv_ws"):      # a round-2 build: the allocating form only
        h.gp_potrf_inv.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int,
                                   ctypes.c_longlong, ctypes.c_void_p, ctypes.c_int,
                                   ctypes.c_longlong, ctypes.c_int, ctypes.c_void_p,
                                   ctypes.c_void_p, ctypes.c_void_p]
        h.ws_form = False
        libs.append((os.path.basename(path), h))
        continue
    h.ws_form = True
    h.gp_potrf_inv_ws.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_longlong,
                                  ctypes.c_void_p, ctypes.c_int, ctypes.c_longlong, ctypes.c_int,
                                  ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                  ctypes.c_longlong, ctypes.c_void_p]
    h.gp_potrf_inv_ws_bytes.argtypes = [ctypes.c_int, ctypes.c_int]
    h.gp_potrf_inv_ws_bytes.restype = ctypes.c_longlong
    libs.append((os.path.basename(path), h))
dev = torch.device("cuda:0")
st = torch.cuda.current_stream(dev).cuda_stream
for n, B in ((4096, 1), (1024, 32), (2048, 4), (512, 24)):
    X = torch.as_tensor(np.random.default_rng(0).random((n, 8)), device=dev)
    betas = torch.as_tensor(np.stack([np.random.default_rng(10 + b).uniform(0.5, 5, 8)
                                      for b in range(B)]), device=dev)
    G0 = kernels.gram(X, betas, 1.0, 1e-6, batch=B)
    npad = kernels.padded_n(n)
    A = torch.empty_like(G0)
    Linv = [torch.empty((B, npad, npad), dtype=torch.float64, device=dev) for _ in libs]
    info = torch.empty(B, dtype=torch.int32, device=dev)
    logdet = torch.empty(B, dtype=torch.float64, device=dev)
    wsb = max(h.gp_potrf_inv_ws_bytes(n, B) if h.ws_form else 0 for _, h in libs)
    ws = torch.empty(max(wsb, 256), dtype=torch.uint8, device=dev)
    times = [[] for _ in libs]
    for rnd in range(12):
        for k, (_, h) in enumerate(libs):
            A.copy_(G0)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            if h.ws_form:
                rc = h.gp_potrf_inv_ws(A.data_ptr(), n, n, n * n, Linv[k].data_ptr(), npad,
                                       npad * npad, B, info.data_ptr(), logdet.data_ptr(),
                                       ws.data_ptr(), ws.numel(), st)
            else:
                rc = h.gp_potrf_inv(A.data_ptr(), n, n, n * n, Linv[k].data_ptr(), npad,
                                    npad * npad, B, info.data_ptr(), logdet.data_ptr(), st)
            e1.record()
            torch.cuda.synchronize()
            assert rc == 0 and int(info.abs().max()) == 0, (rc, info)
            if rnd >= 2:
                times[k].append(e0.elapsed_time(e1))
    for k, (name, _) in enumerate(libs):
        d = float((Linv[k] - Linv[0]).abs().max())
        print(f"n={n} batch={B} {name:28s} median {np.median(times[k]):7.3f} ms "
              f"(min {min(times[k]):.3f})  max|dLinv| vs {libs[0][0]}: {d:.2e}", flush=True)
