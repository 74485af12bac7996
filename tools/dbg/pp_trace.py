"""Debug: timestamp trace of the persistent factorisation (s_memrealtime, 100 MHz) at n.
Prints the chain's per-step phases, how long the chain waited for its DP/SP partials, and
worker occupancy over time."""
import os, sys
import numpy as np
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
n = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
N = (n + 63) // 64
W, B = 6, 3  # chol.hip kPPLead, kPPBand
XD = 8      # chol.hip kPPXDelay
NBf = 0   # no block tasks
in_ltb = lambda i, j: (i >> 1) < NBf and (i >> 1) - (j >> 1) >= 3
in_xtb = lambda i, c: (i >> 1) < NBf and (i >> 1) > (c >> 1)
tasks = [("C", 0, 0)]
for t in range(4 * N - 1 + 4 * (W + XD)):          # chol.hip pp_for_key
    if t % 4 == 2 and 2 <= (t + 2) // 4 <= N - 1: tasks.append(("DP", 0, (t + 2) // 4))
    if t % 4 == 1 and 1 <= (t - 1) // 4 <= N - 2: tasks.append(("SP", (t - 1) // 4 + 1, (t - 1) // 4))
    if t % 2 == 0 and t >= 4:
        s_ = t // 2
        jmin = max((s_ - B + 1) // 2, s_ - (N - 1))
        tasks += [("L", s_ - j, j) for j in range((s_ - 2) // 2, max(jmin, 0) - 1, -1)]
    K = t - 4 * W
    if K < 0: continue
    KX = K - 4 * XD
    if KX >= 0 and KX % 4 == 2 and 1 <= (KX - 2) // 4 <= N - 1:
        i = (KX - 2) // 4
        tasks += [("X", i, c) for c in range(i) if not in_xtb(i, c)]
    if K % 8 == 2 and 1 <= (K - 2) // 8 < NBf:
        I = (K - 2) // 8
        tasks += [("XB", I, C) for C in range(I - 1, -1, -1)]
    if K % 2 == 0:
        s_ = K // 2
        jmin = max(s_ - (N - 1), 0)
        if s_ >= B + 1:
            tasks += [("L", s_ - j, j) for j in range((s_ - B - 1) // 2, jmin - 1, -1)
                      if not in_ltb(s_ - j, j)]
    if K % 4 == 0:
        S = K // 4
        jlo = max(S - NBf + 1, 0)
        if S >= 3:
            tasks += [("LB", S - J, J) for J in range((S - 3) // 2, jlo - 1, -1)]
nt = len(tasks)
dev = torch.device("cuda:0")
trace = torch.zeros(nt * 4 + N * 8, dtype=torch.int64, device=dev)
os.environ["GPFIT_PP_TRACE_PTR"] = str(trace.data_ptr())
from gladsgp_amd import kernels
X = torch.as_tensor(np.random.default_rng(0).random((n, 8)), device=dev)
beta = torch.as_tensor(np.random.default_rng(3).uniform(0.5, 5, 8), device=dev)
for r in range(3):
    trace.zero_()
    ch = kernels.cholesky_inverse(kernels.gram(X, beta, 1.0, 1e-6))
    torch.cuda.synchronize()
ch.check()
t = trace.cpu().numpy().astype(np.float64)
tk = t[: nt * 4].reshape(nt, 4)
cs = t[nt * 4:].reshape(N, 8)
t0 = cs[0, 0]
us = lambda x: (x - t0) / 100.0   # 100 MHz -> us
print(f"n={n} N={N} tasks={nt}  chain end {us(cs[N-1, 4]):.1f} us; last task end "
      f"{us(tk[1:, 3].max()):.1f} us")
ph = ["waitDP", "syrk+fill", "factor", "storeD", "waitSP", "ldP", "gemm+st", "->next"]
acc = np.zeros(8)
for j in range(N - 1):
    d = [(cs[j, q + 1] - cs[j, q]) / 100 for q in range(7)] + [(cs[j + 1, 0] - cs[j, 7]) / 100]
    acc += d
    if j % 8 == 0 or j > N - 4:
        print(f"j={j:3d} start {us(cs[j, 0]):8.1f} " + " ".join(f"{p}={x:5.1f}" for p, x in zip(ph, d)))
print("chain mean per step: " + " ".join(f"{p}={x / (N - 1):5.1f}" for p, x in zip(ph, acc)))
kinds = {}
ep = {}
stall = {}
for k in range(1, nt):
    kd = tasks[k][0]
    kinds.setdefault(kd, []).append((tk[k, 2] - tk[k, 1]) / 100)
    ep.setdefault(kd, []).append((tk[k, 3] - tk[k, 2]) / 100)
    stall.setdefault(kd, []).append((int(tk[k, 0]) >> 8) / 100)
for kd, v in kinds.items():
    nterm = [(x[2] if x[0] in ("L", "SP") else x[2] - 1 if x[0] == "DP" else x[1] - x[2] if x[0] == "X"
              else 2 * x[2] if x[0] == "LB" else 2 * (x[1] - x[2])) for x in tasks[1:] if x[0] == kd]
    print(f"{kd}: {len(v)} tasks, accumulate mean {np.mean(v):.1f} us max {np.max(v):.1f}, "
          f"terms mean {np.mean(nterm):.1f} -> {np.sum(v) / max(1, np.sum(nterm)):.2f} us/term; "
          f"epilogue mean {np.mean(ep[kd]):.1f} us; WG-time total {np.sum(v) + np.sum(ep[kd]):.0f} us; "
          f"polling for inputs inside the K loop {np.sum(stall[kd]):.0f} us "
          f"-> {(np.sum(v) - np.sum(stall[kd])) / max(1, np.sum(nterm)):.2f} us/term computing")
# occupancy: fraction of 255 workers inside a task (start..end) per 100 us bucket
span = us(tk[1:, 3].max())
edges = np.arange(0, span + 100, 100)
busy = np.zeros(len(edges))
accb = np.zeros(len(edges))
for k in range(1, nt):
    s0, s1, s2 = us(tk[k, 1]), us(tk[k, 2]), us(tk[k, 3])
    for bi, e in enumerate(edges):
        busy[bi] += max(0, min(s2, e + 100) - max(s0, e)) / 100
        accb[bi] += max(0, min(s2, e + 100) - max(s2 - (s2 - s1), e)) / 100
print("workers in a task per 100 us bucket:", " ".join(f"{x:.0f}" for x in busy))
# per tile row: when its last L and X tile finished (us), and the X column-0 chain
rowsL, rowsX, col0 = {}, {}, {}
for k in range(1, nt):
    kd, i, j = tasks[k]
    end = us(tk[k, 3])
    rows = [2 * i, 2 * i + 1] if kd in ("LB", "XB") else [i]
    for r in rows:
        if kd in ("L", "LB"): rowsL[r] = max(rowsL.get(r, 0), end)
        if kd in ("X", "XB"): rowsX[r] = max(rowsX.get(r, 0), end)
    if kd == "X" and j == 0: col0[i] = end
    if kd == "XB" and j == 0: col0[2 * i] = col0[2 * i + 1] = end
print("row: L done / X done / X col0 done (us)")
for r in range(0, N, 4):
    print(f"  {r:3d}: {rowsL.get(r, float('nan')):8.1f} {rowsX.get(r, float('nan')):8.1f} "
          f"{col0.get(r, float('nan')):8.1f}")
