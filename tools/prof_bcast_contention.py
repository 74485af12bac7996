"""One-GPU rehearsal of the N > 1 step's contention (VERDICT r04 Next #3): every rank >= 1
predicts its block (13,408 points at N = 8 with the C3 split) while RCCL broadcasts the next GP's
packed L^-1 (67 MB at n = 4096) on RCCL's own stream.  A one-GPU box has no peer, so the
broadcast is a stand-in (tools/dbg/bcast_standin.hip): `wgs` workgroups copying 67 MB on a
second stream, either unthrottled (HBM-speed) or throttled to last about as long as an xGMI
transfer (target durations below).  Printed per configuration: the prediction's time (HIP
events on its stream, gp_predict_ex from the payload: cross-covariance + TRMM + finalize) alone and beside
the copy, and the copy's own completion time alone and beside the prediction; plus the
per-step extras of the N > 1 path measured alone: the payload's pack + z (rank 0), the unpack
the ranks > 0 no longer run, and the (mean, var) gather stand-in.

    python tools/prof_bcast_contention.py [points]
"""
import ctypes
import os
import subprocess
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from gladsgp_amd import _capi, kernels  # noqa: E402
from gladsgp_amd.sharded import LinvPacker  # noqa: E402

SO = os.path.join(ROOT, "tools", "dbg", "libbcast_standin.so")
if not os.path.exists(SO):
    subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-shared", "-fPIC",
                    "-o", SO, os.path.join(ROOT, "tools", "dbg", "bcast_standin.hip")],
                   check=True)
lib = ctypes.CDLL(SO)
lib.standin_copy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_longlong, ctypes.c_int,
                             ctypes.c_int, ctypes.c_void_p]

dev = torch.device("cuda:0")
n, d = 4096, 8
pts = int(sys.argv[1]) if len(sys.argv) > 1 else 13408
rng = np.random.default_rng(0)
X = torch.as_tensor(rng.random((n, d)), device=dev)
Xs = torch.as_tensor(rng.random((pts, d)), device=dev)
beta = torch.as_tensor(rng.uniform(0.5, 5, (1, d)), device=dev)
w = torch.as_tensor(np.sin(rng.random(n) * 6), device=dev).reshape(1, n)
ch = kernels.cholesky_inverse(kernels.gram(X, beta, 1.0, 1e-6))
ch.check()
npad = kernels.padded_n(n)
packer = LinvPacker(npad, dev, n=n)
nbytes = (packer.numel * 8 + 15) // 16 * 16
src = torch.empty(nbytes // 8, dtype=torch.float64, device=dev).fill_(1.0)
dst = torch.empty_like(src)
ws = kernels.Workspace()
s_pred = torch.cuda.Stream(dev)
s_copy = torch.cuda.Stream(dev)
out = (torch.empty((1, pts), dtype=torch.float64, device=dev),
       torch.empty((1, pts), dtype=torch.float64, device=dev))


def ev():
    return torch.cuda.Event(enable_timing=True)


payload = packer.buffer(dev)
packer.pack(ch.linv_buf, ch.info, payload, w=w)
view = packer.view(payload)


def predict():
    # a rank > 0's step: straight from the broadcast payload (tile-packed L^-1 + z)
    kernels.predict(view, X, Xs, beta, 1.0, 1.0, None, workspace=ws, out=out)


def copy(wgs, sl):
    rc = lib.standin_copy(src.data_ptr(), dst.data_ptr(), nbytes, wgs, sl, s_copy.cuda_stream)
    assert rc == 0


def run(wgs=None, sl=0, do_pred=True, reps=5):
    tp, tc = [], []
    for r in range(reps + 1):
        torch.cuda.synchronize()
        e = [ev() for _ in range(4)]
        if wgs is not None:
            with torch.cuda.stream(s_copy):
                e[2].record()
                copy(wgs, sl)
                e[3].record()
        if do_pred:
            with torch.cuda.stream(s_pred):
                e[0].record()
                predict()
                e[1].record()
        torch.cuda.synchronize()
        if r:
            if do_pred:
                tp.append(e[0].elapsed_time(e[1]))
            if wgs is not None:
                tc.append(e[2].elapsed_time(e[3]))
    med = lambda v: float(np.median(v)) if v else float("nan")  # noqa: E731
    return med(tp), med(tc)


# warm the clocks, then every configuration between two runs of the prediction alone (clock
# and power state drift between runs is as large as the effect measured)
for _ in range(3):
    run(reps=3)
base, _ = run(reps=7)
print(f"prediction of {pts} points at n = {n} alone: {base:.3f} ms", flush=True)
worst = 0.0
for wgs in (16, 32, 64):
    cfgs = [(0, None)]
    for target in (0.7, 1.4):
        sl, c = 1, 0.0
        while sl < 4096:
            _, c = run(wgs, sl, do_pred=False, reps=2)
            if c >= target:
                break
            sl *= 2
        cfgs.append((sl, c))
    for sl, c in cfgs:
        if c is None:
            _, c = run(wgs, 0, do_pred=False)
        a0, _ = run(reps=7)
        p, cp = run(wgs, sl, reps=7)
        a1, _ = run(reps=7)
        ratio = p / (0.5 * (a0 + a1))
        worst = max(worst, ratio)
        print(f"  wgs {wgs:3d} {'unthrottled' if sl == 0 else f'sleep {sl:4d}'}: copy alone "
              f"{c:.3f} ms, beside the prediction {cp:.3f} ms; prediction {p:.3f} ms beside vs "
              f"{a0:.3f} / {a1:.3f} alone before / after: x{ratio:.3f}", flush=True)
print(f"worst prediction slowdown beside the stand-in broadcast: x{worst:.3f}", flush=True)

# the per-step extras of the N > 1 path
linv = torch.zeros((1, npad, npad), dtype=torch.float64, device=dev)
packed = packer.buffer(dev)
for name, fn in (("gp_pack_linv + gp_predict_z (rank 0, round-5 payload)",
                  lambda: packer.pack(ch.linv_buf, ch.info, packed, w=w)),
                 ("gp_pack_linv alone", lambda: packer.pack(ch.linv_buf, ch.info, packed)),
                 ("gp_unpack_linv (not run any more: ranks >= 1 read the payload in place)",
                  lambda: packer.unpack(packed, linv)),
                 ("gather stand-in (2 x 8 B x points, D2D)",
                  lambda: out[0].copy_(out[1]))):
    ts = []
    for r in range(6):
        torch.cuda.synchronize()
        e0, e1 = ev(), ev()
        e0.record()
        fn()
        e1.record()
        torch.cuda.synchronize()
        if r:
            ts.append(e0.elapsed_time(e1))
    print(f"{name}: {np.median(ts) * 1e3:.1f} us", flush=True)
