"""Projection (not a measurement) of the C3 strong-scaling step at N = 2, 4, 8 from one GPU.

The per-rank work of `bench.py --gpus N` (sharded.PipelinedPredictor, round-5 payload) is timed
rank by rank on this GPU with HIP events, each piece median of 5:
  rank 0:    Gram + gp_potrf_inv of the next GP (t_fact), gp_pack_linv + gp_predict_z into the
             payload (t_pack), then its c0 points from its padded L^-1 with the shipped z;
  ranks > 0: their c1 points straight from the tile-packed payload with the shipped z (no
             unpack, no trmv), while RCCL receives the next GP's 67 MB payload beside them;
and the step is the slower of the two plus the gather.  The split is sharded.balanced_split on
these times (what calibrate_split picks on the GPUs).  Folded in from measurements on this GPU:
  * the broadcast's contention: the prediction beside a stand-in copy of the payload
    (tools/prof_bcast_contention.py: 16-64 workgroups, 67 MB, throttled to xGMI-like
    durations) -- the measured ratio, worst configuration, scales the ranks > 0 time;
  * the gather: a device-to-device copy of every rank's (mean, var) block (2 x 8 B x points)
    plus GATHER_LATENCY_US of collective latency (an assumption: RCCL small-message latency over
    xGMI is not measurable on one GPU);
Not included: GPU-to-GPU clock differences; whether the broadcast finishes within a step is
checked against the payload size at XGMI_GBS (an assumption, stated in the output).

    python tools/project_scaling.py [contention_ratio]
"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gladsgp_amd import kernels  # noqa: E402
from gladsgp_amd.sharded import LinvPacker, balanced_split  # noqa: E402

GATHER_LATENCY_US = 30.0     # assumed RCCL gather latency per step (1.6 MB in all)
XGMI_GBS = (48.0, 96.0)      # assumed effective ring-broadcast bandwidth range, GB/s

dev = torch.device("cuda:0")
n, m, d = 4096, 100000, 8
rng = np.random.default_rng(0)
X = torch.as_tensor(rng.random((n, d)), device=dev)
Xs = torch.as_tensor(rng.random((m, d)), device=dev)
beta = torch.as_tensor(rng.uniform(0.5, 5, (1, d)), device=dev)
w = torch.as_tensor(np.sin(rng.random(n) * 6), device=dev).reshape(1, n)
s, delta = 1.0, 1e-6
ws = kernels.PredictWorkspace()
npad = kernels.padded_n(n)
packer = LinvPacker(npad, dev, n=n)
payload = packer.buffer(dev)
contention = float(sys.argv[1]) if len(sys.argv) > 1 else 1.0


def med(fn, reps=5):
    fn()
    ts = []
    for _ in range(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize(dev)
        e0.record()
        fn()
        e1.record()
        torch.cuda.synchronize(dev)
        ts.append(e0.elapsed_time(e1) * 1e-3)
    return sorted(ts)[reps // 2]


ch = kernels.cholesky_inverse(kernels.gram(X, beta, s, delta))
ch.check()
t_fact = med(lambda: kernels.cholesky_inverse(kernels.gram(X, beta, s, delta)))
t_pack = med(lambda: packer.pack(ch.linv_buf, ch.info, payload, w=w))
view = packer.view(payload)
z = packer.z(payload).view(1, npad)
cache0, cache1 = {}, {}


def T0(p):          # rank 0: padded L^-1, shipped z
    if p <= 0:
        return 0.0
    if p not in cache0:
        Xc = Xs[:p].contiguous()
        cache0[p] = med(lambda: kernels.predict(ch, X, Xc, beta, s, s, None, workspace=ws, z=z),
                        reps=3)
    return cache0[p]


def T1(p):          # ranks > 0: the payload in place
    if p <= 0:
        return 0.0
    if p not in cache1:
        Xc = Xs[:p].contiguous()
        cache1[p] = med(lambda: kernels.predict(view, X, Xc, beta, s, s, None, workspace=ws),
                        reps=3)
    return cache1[p]


def gather_s(counts):
    mx = max(counts)
    src = torch.zeros((len(counts), 2, mx), dtype=torch.float64, device=dev)
    dst = torch.empty_like(src)
    return med(lambda: dst.copy_(src)) + GATHER_LATENCY_US * 1e-6


t_full = med(lambda: kernels.predict(ch, X, Xs, beta, s, s, w, workspace=ws))
t1 = t_fact + t_full
print(f"one GPU: factorisation {t_fact * 1e3:.3f} ms + prediction of {m} points "
      f"{t_full * 1e3:.3f} ms = {t1 * 1e3:.3f} ms per GP ({m / t1 / 1e6:.3f} M pred/s, serial "
      f"head); payload pack + z {t_pack * 1e6:.1f} us ({payload.numel() * 8 / 1e6:.1f} MB); "
      f"T(13408 points) padded+z {T0(13408) * 1e3:.3f} / packed+z {T1(13408) * 1e3:.3f} ms; "
      f"contention factor on ranks > 0: {contention:.3f}", flush=True)
for N in (2, 4, 8):
    counts = balanced_split(m, N, t_fact + t_pack, lambda p: contention * T1(p))
    r0 = t_fact + t_pack + T0(counts[0])
    rr = contention * max(T1(c) for c in counts[1:])
    g = gather_s(counts)
    step = max(r0, rr) + g
    bc = [payload.numel() * 8 / (b * 1e9) for b in XGMI_GBS]
    print(f"N={N}: counts rank0 {counts[0]} / others {max(counts[1:])}; rank 0 {r0 * 1e3:.3f} ms, "
          f"others {rr * 1e3:.3f} ms, gather {g * 1e6:.0f} us -> projected step "
          f"{step * 1e3:.3f} ms, {m / step / 1e6:.2f} M pred/s, {t1 / step / N:.2f} of N x the "
          f"serial one-GPU rate; the broadcast ({bc[1] * 1e3:.2f}-{bc[0] * 1e3:.2f} ms at "
          f"{XGMI_GBS[1]:.0f}-{XGMI_GBS[0]:.0f} GB/s) {'fits' if bc[0] < step else 'EXCEEDS'} "
          "the step", flush=True)
