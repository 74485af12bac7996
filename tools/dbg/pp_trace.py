"""Diagnostics: timestamp trace of the persistent factorisation (s_memrealtime, 100 MHz) at n.

Loads the trace build of the library (``python -m gladsgp_amd._build --trace`` ->
gladsgp_amd/libgpfit_trace.so; the shipped libgpfit.so has no trace code) and prints the
chain's per-step phases, how long the chain waited for its DP/SP partials, per-kind task
statistics and worker occupancy over time.  Every task records its own (kind, i, j), so the
task order is read from the trace, not recomputed here."""
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from gladsgp_amd import _build, _capi  # noqa: E402

if (not os.path.exists(_build.TRACE_LIB_PATH) or
        os.path.getmtime(_build.TRACE_LIB_PATH) < os.path.getmtime(_build.LIB_PATH)):
    # missing, or older than the shipped library (whose ABI _capi binds in full: a stale trace
    # build lacking a newer symbol would fail the bind); rebuild (stale objects only)
    print("rebuilding", _build.build_library(trace=True), file=sys.stderr)
_capi.LIB_PATH = _build.TRACE_LIB_PATH        # this process only: the diagnostics variant
from gladsgp_amd import kernels  # noqa: E402

lib = _capi.lib()
lib.gp_pp_trace_set.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
lib.gp_pp_trace_slots.argtypes = [ctypes.c_int, ctypes.c_int]
lib.gp_pp_trace_slots.restype = ctypes.c_longlong

n = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
N = (n + 63) // 64
SL = 6                                      # chol.hip kPPTraceSlots
dev = torch.device("cuda:0")
nslots = int(lib.gp_pp_trace_slots(n, 1))
nt = (nslots - N * 8) // SL
trace = torch.zeros(nslots, dtype=torch.int64, device=dev)
lib.gp_pp_trace_set(None, ctypes.c_void_p(trace.data_ptr()))
X = torch.as_tensor(np.random.default_rng(0).random((n, 8)), device=dev)
beta = torch.as_tensor(np.random.default_rng(3).uniform(0.5, 5, 8), device=dev)
for r in range(3):
    trace.zero_()
    ch = kernels.cholesky_inverse(kernels.gram(X, beta, 1.0, 1e-6))
    torch.cuda.synchronize()
ch.check()
lib.gp_pp_trace_set(None, None)
t = trace.cpu().numpy()
tk = t[: nt * SL].reshape(nt, SL).astype(np.float64)
kinds_raw = t[: nt * SL].reshape(nt, SL)[:, 4] & 15
ij = t[: nt * SL].reshape(nt, SL)[:, 5]
KN = {1: "L", 2: "DP", 3: "SP", 4: "X", 5: "Z", 6: "X2", 7: "ZP"}
tasks = [("C", 0, 0) if kinds_raw[k] == 0 else (KN[int(kinds_raw[k])], int(ij[k] & 0xffff),
                                                int(ij[k] >> 16)) for k in range(nt)]
cs = t[nt * SL:].reshape(N, 8).astype(np.float64)
t0 = cs[0, 0]
us = lambda x: (x - t0) / 100.0   # noqa: E731  (100 MHz -> us)
work = [k for k in range(nt) if tasks[k][0] != "C" and tk[k, 1] > 0]
print(f"n={n} N={N} tasks={nt}  chain end {us(cs[N-1, 4]):.1f} us; last task end "
      f"{us(tk[work, 3].max()):.1f} us")
ph = ["waitDP", "fill", "factor", "stD+pub", "waitSP+ldP", "gemm", "st+syrk", "->next"]
acc = np.zeros(8)
for j in range(N - 1):
    d = [(cs[j, q + 1] - cs[j, q]) / 100 for q in range(7)] + [(cs[j + 1, 0] - cs[j, 7]) / 100]
    acc += d
    if j % 8 == 0 or j > N - 4:
        print(f"j={j:3d} start {us(cs[j, 0]):8.1f} " +
              " ".join(f"{p}={x:5.1f}" for p, x in zip(ph, d)))
print("chain mean per step: " + " ".join(f"{p}={x / (N - 1):5.1f}" for p, x in zip(ph, acc)))
dur, ep, stall, terms = {}, {}, {}, {}
for k in work:
    kd, i, j = tasks[k]
    dur.setdefault(kd, []).append((tk[k, 2] - tk[k, 1]) / 100)
    ep.setdefault(kd, []).append((tk[k, 3] - tk[k, 2]) / 100)
    stall.setdefault(kd, []).append((int(t[k * SL]) >> 8) / 100)
    terms.setdefault(kd, []).append(      # 64^3 tile-terms (a pair does two per K step)
        j if kd in ("L", "SP") else j - 1 if kd == "DP" else 2 * (i - j) - 1 if kd == "X2"
        else i - j)
for kd, v in dur.items():
    nterm = np.sum(terms[kd])
    print(f"{kd}: {len(v)} tasks, accumulate mean {np.mean(v):.1f} us max {np.max(v):.1f}, "
          f"terms mean {np.mean(terms[kd]):.1f} -> {np.sum(v) / max(1, nterm):.2f} us/term; "
          f"epilogue mean {np.mean(ep[kd]):.1f} us; WG-time total {np.sum(v) + np.sum(ep[kd]):.0f} us; "
          f"polling for inputs inside the K loop {np.sum(stall[kd]):.0f} us "
          f"-> {(np.sum(v) - np.sum(stall[kd])) / max(1, nterm):.2f} us/term computing")
span = us(tk[work, 3].max())
edges = np.arange(0, span + 100, 100)
busy = np.zeros(len(edges))
for k in work:
    s0, s2 = us(tk[k, 1]), us(tk[k, 3])
    for bi, e in enumerate(edges):
        busy[bi] += max(0, min(s2, e + 100) - max(s0, e)) / 100
print("workers in a task per 100 us bucket:", " ".join(f"{x:.0f}" for x in busy))
rowsL, rowsX = {}, {}
for k in work:
    kd, i, j = tasks[k]
    end = us(tk[k, 3])
    if kd == "L":
        rowsL[i] = max(rowsL.get(i, 0), end)
    if kd in ("X", "X2"):
        rowsX[i] = max(rowsX.get(i, 0), end)
print("row: L done / X done (us)")
for r in range(0, N, 4):
    print(f"  {r:3d}: {rowsL.get(r, float('nan')):8.1f} {rowsX.get(r, float('nan')):8.1f}")
