"""Bit-for-bit comparison of gp_predict (cross-covariance + TRMM + mean/var) between library
builds loaded into one process: python tools/ab_predict_bits.py libA.so libB.so
Shapes: one GP (n = 1000, m = 20000, a ragged tail chunk) and a batch (n = 256 x 8, m = 5000),
d = 8 and d = 3; L^-1 is a random lower triangle (the kernels do not care that it is one)."""
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gladsgp_amd import kernels  # noqa: E402,F401  (torch's HIP runtime first)

P = ctypes.c_void_p
I = ctypes.c_int
LL = ctypes.c_longlong
libs = []
for path in sys.argv[1:]:
    h = ctypes.CDLL(os.path.abspath(path))
    h.gp_predict.argtypes = [P, I, LL, P, I, P, I, I, I, I, P, I, P, P, P, I, P, P, I, I, P, LL,
                             I, P]
    h.gp_predict_ws_bytes.argtypes = [I, I, I, I]
    h.gp_predict_ws_bytes.restype = LL
    h.gp_fit_predict.argtypes = [P, I, P, I, I, I, I, P, I, P, P, P, P, I, P, I, LL, P, I, LL, P,
                                 P, P, P, I, I, P, LL, I, P, P]
    h.gp_fit_predict_ws_bytes.argtypes = [I, I, I, I]
    h.gp_fit_predict_ws_bytes.restype = LL
    h.gp_ctx_create.argtypes = [ctypes.c_double, I, ctypes.POINTER(P)]
    h.gp_ctx_destroy.argtypes = [P]
    libs.append((os.path.basename(path), h))
dev = torch.device("cuda:0")
st = torch.cuda.current_stream(dev).cuda_stream
rng = np.random.default_rng(0)
bad = 0
for n, m, d, B, mch in ((1000, 20000, 8, 1, 0), (256, 5000, 8, 8, 0), (300, 7000, 3, 2, 2048)):
    npad = kernels.padded_n(n)
    L = np.tril(rng.standard_normal((B, npad, npad)) / n)
    L[:, n:, :] = 0.0
    L[:, :, n:] = 0.0
    Linv = torch.as_tensor(L.transpose(0, 2, 1).copy(), device=dev)   # column-major
    X = torch.as_tensor(rng.random((n, d)), device=dev)
    Xs = torch.as_tensor(rng.random((m, d)), device=dev)
    beta = torch.as_tensor(rng.uniform(0.5, 5, (B, d)), device=dev)
    s = torch.as_tensor(rng.uniform(0.5, 2, B), device=dev)
    w = torch.as_tensor(rng.standard_normal((B, n)), device=dev)
    outs = []
    for name, h in libs:
        mean = torch.empty((B, m), dtype=torch.float64, device=dev)
        var = torch.empty((B, m), dtype=torch.float64, device=dev)
        wsb = h.gp_predict_ws_bytes(n, m, B, mch)
        ws = torch.empty(wsb, dtype=torch.uint8, device=dev)
        rc = h.gp_predict(Linv.data_ptr(), npad, npad * npad, X.data_ptr(), d, Xs.data_ptr(), d,
                          n, m, d, beta.data_ptr(), d, s.data_ptr(), s.data_ptr(), w.data_ptr(),
                          n, mean.data_ptr(), var.data_ptr(), m, B, ws.data_ptr(), wsb, mch, st)
        torch.cuda.synchronize()
        assert rc == 0, (name, rc)
        outs.append((name, mean.cpu().numpy(), var.cpu().numpy()))
    for name, mu, va in outs[1:]:
        same = np.array_equal(mu, outs[0][1]) and np.array_equal(va, outs[0][2])
        bad += not same
        print(f"n={n} m={m} d={d} B={B} chunk={mch}: {name} vs {outs[0][0]}: "
              f"{'bit-identical' if same else 'DIFFERENT'} (max |dmean| "
              f"{np.max(np.abs(mu - outs[0][1])):.3g}, max |dvar| {np.max(np.abs(va - outs[0][2])):.3g})")
# gp_fit_predict (Gram + factorisation + cross-covariance + TRMM), with and without a gp_ctx,
# ragged last chunk
for n, m, d, B, mch in ((1000, 20000, 8, 1, 0), (512, 9000, 8, 2, 4096)):
    npad = kernels.padded_n(n)
    X = torch.as_tensor(rng.random((n, d)), device=dev)
    Xs = torch.as_tensor(rng.random((m, d)), device=dev)
    beta = torch.as_tensor(rng.uniform(0.5, 5, (B, d)), device=dev)
    s = torch.as_tensor(rng.uniform(0.5, 2, B), device=dev)
    delta = torch.full((B,), 1e-6, dtype=torch.float64, device=dev)
    w = torch.as_tensor(rng.standard_normal((B, n)), device=dev)
    for use_ctx in (False, True):
        outs = []
        for name, h in libs:
            G = torch.empty((B, n, n), dtype=torch.float64, device=dev)
            Linv = torch.empty((B, npad, npad), dtype=torch.float64, device=dev)
            info = torch.empty(B, dtype=torch.int32, device=dev)
            logdet = torch.empty(B, dtype=torch.float64, device=dev)
            mean = torch.empty((B, m), dtype=torch.float64, device=dev)
            var = torch.empty((B, m), dtype=torch.float64, device=dev)
            wsb = h.gp_fit_predict_ws_bytes(n, m, B, mch)
            ws = torch.empty(wsb, dtype=torch.uint8, device=dev)
            ctx = P()
            if use_ctx:
                assert h.gp_ctx_create(-1.0, -1, ctypes.byref(ctx)) == 0
            rc = h.gp_fit_predict(X.data_ptr(), d, Xs.data_ptr(), d, n, m, d, beta.data_ptr(), d,
                                  s.data_ptr(), delta.data_ptr(), s.data_ptr(), w.data_ptr(), n,
                                  G.data_ptr(), n, n * n, Linv.data_ptr(), npad, npad * npad,
                                  info.data_ptr(), logdet.data_ptr(), mean.data_ptr(),
                                  var.data_ptr(), m, B, ws.data_ptr(), wsb, mch, ctx, st)
            torch.cuda.synchronize()
            if use_ctx:
                h.gp_ctx_destroy(ctx)
            assert rc == 0 and int(info.abs().sum()) == 0, (name, rc, info)
            outs.append((name, mean.cpu().numpy(), var.cpu().numpy()))
        for name, mu, va in outs[1:]:
            same = np.array_equal(mu, outs[0][1]) and np.array_equal(va, outs[0][2])
            bad += not same
            print(f"fit_predict n={n} m={m} B={B} chunk={mch} ctx={use_ctx}: {name} vs "
                  f"{outs[0][0]}: {'bit-identical' if same else 'DIFFERENT'}")
sys.exit(1 if bad else 0)
