"""Does the factorisation's CU-time shrink on fewer CUs?  (The question behind overlapping GP
k+1's factorisation with GP k's TRMM: worth it only if the factorisation, latency-bound on all
256 CUs, does the same work in fewer CU-milliseconds on a subset.)

  A. gp_potrf_inv_ws at n = 4096 on a CU-masked stream of c CUs (CU i sits on XCD i % 8, so the
     first c CUs are spread evenly over the XCDs): median time and time x c.
  B. the same factorisation on c CUs beside gp_predict_solve (the TRMM + mean/var of 32768
     test points from a prepared K*) on an unmasked stream: wall time of both vs each alone.

    python tools/prof_fact_cus.py
"""
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gladsgp_amd import _capi, kernels  # noqa: E402

dev = torch.device("cuda:0")
torch.cuda.init()
hip = ctypes.CDLL("libamdhip64.so")
NCU = torch.cuda.get_device_properties(dev).multi_processor_count


def masked_stream(c):
    mask = [0] * ((NCU + 31) // 32)
    for i in range(c):
        mask[i // 32] |= 1 << (i % 32)
    st = ctypes.c_void_p()
    arr = (ctypes.c_uint32 * len(mask))(*mask)
    rc = hip.hipExtStreamCreateWithCUMask(ctypes.byref(st), ctypes.c_uint32(len(mask)), arr)
    assert rc == 0, rc
    return torch.cuda.ExternalStream(st.value, device=dev)


n, d, m = 4096, 8, 32768
rng = np.random.default_rng(0)
X = torch.as_tensor(rng.random((n, d)), device=dev)
Xs = torch.as_tensor(rng.random((m, d)), device=dev)
beta = torch.as_tensor(rng.uniform(0.5, 5, (1, d)), device=dev)
one = torch.ones(1, dtype=torch.float64, device=dev)
G0 = kernels.gram(X, beta, 1.0, 1e-6)
npad = kernels.padded_n(n)
A = torch.empty_like(G0)
Linv = torch.zeros((1, npad, npad), dtype=torch.float64, device=dev)
Linv2 = torch.zeros_like(Linv)
info = torch.empty(1, dtype=torch.int32, device=dev)
logdet = torch.empty(1, dtype=torch.float64, device=dev)
wsf = torch.empty(int(_capi.lib().gp_potrf_inv_ws_bytes(n, 1)), dtype=torch.uint8, device=dev)
w = torch.as_tensor(rng.standard_normal((1, n)), device=dev)
mean = torch.empty((1, m), dtype=torch.float64, device=dev)
var = torch.empty_like(mean)
wsp = torch.empty(int(_capi.lib().gp_predict_prepared_ws_bytes(n, m, 1, 0)), dtype=torch.uint8,
                  device=dev)


def fact(st, out):
    A.copy_(G0)   # on the current stream, before the factorisation's stream waits
    ev = torch.cuda.Event()
    ev.record()
    st.wait_event(ev)
    _capi.call("gp_potrf_inv_ws", A.data_ptr(), n, n, n * n, out.data_ptr(), npad, npad * npad,
               1, info.data_ptr(), logdet.data_ptr(), wsf.data_ptr(), wsf.numel(),
               st.cuda_stream)


def solve(st):
    _capi.call("gp_predict_solve", Linv.data_ptr(), npad, npad * npad, n, m, one.data_ptr(),
               w.data_ptr(), n, mean.data_ptr(), var.data_ptr(), m, 1, wsp.data_ptr(),
               wsp.numel(), 0, st.cuda_stream)


main = torch.cuda.current_stream(dev)
fact(main, Linv)
_capi.call("gp_predict_cross", X.data_ptr(), d, Xs.data_ptr(), d, n, m, d, beta.data_ptr(), d,
           one.data_ptr(), 1, wsp.data_ptr(), wsp.numel(), 0, main.cuda_stream)
torch.cuda.synchronize()
assert int(info[0]) == 0


def timed(fn, reps=8):
    ts = []
    for r in range(reps + 2):
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(main)
        for s in streams_used:
            s.wait_event(e0)
        fn()
        for s in streams_used:
            ev = torch.cuda.Event()
            ev.record(s)
            main.wait_event(ev)
        e1.record(main)
        torch.cuda.synchronize()
        if r >= 2:
            ts.append(e0.elapsed_time(e1))
    return float(np.median(ts))


pred = torch.cuda.Stream(device=dev)
streams_used = [pred]
t_solve = timed(lambda: solve(pred))
print(f"gp_predict_solve, {m} points, all CUs: {t_solve:.3f} ms", flush=True)
ref = Linv.clone()
for c in (32, 64, 96, 128, 192, NCU):
    st = masked_stream(c) if c < NCU else torch.cuda.Stream(device=dev)
    streams_used = [st]
    tf = timed(lambda: fact(st, Linv2))
    if not (int(info[0]) == 0 and torch.equal(Linv2, ref)):
        print(f"  {c} CUs alone: info {int(info[0])}, L^-1 differs from the unmasked run")
    streams_used = [st, pred]
    tb = timed(lambda: (fact(st, Linv2), solve(pred)))
    ok = int(info[0]) == 0 and torch.equal(Linv2, ref)
    print(f"factorisation on {c:3d} CUs: {tf:.3f} ms alone ({tf * c:7.1f} CU-ms) | beside the "
          f"solve: both done in {tb:.3f} ms vs {tf + t_solve:.3f} one after the other "
          f"({tf + t_solve - tb:+.3f}){'' if ok else ' FACTORISATION FAILED'}", flush=True)
