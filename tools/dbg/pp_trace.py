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
def lt_range(s, band):
    jmin = max(0, s - (N - 1))
    if band:
        jmin = max(jmin, (s - B + 1) // 2); jmax = (s - 2) // 2
    else:
        jmax = (s - B - 1) // 2
    return (jmin, jmax) if s >= 2 else (0, -1)
tasks = [("C", 0, 0)]
for T in range(4 * N - 1 + 4 * W):
    if T % 4 == 2 and 2 <= (T + 2) // 4 <= N - 1: tasks.append(("DP", 0, (T + 2) // 4))
    if T % 4 == 1 and 1 <= (T - 1) // 4 <= N - 2: tasks.append(("SP", (T - 1) // 4 + 1, (T - 1) // 4))
    if T % 2 == 0:
        a, b = lt_range(T // 2, True)
        tasks += [("L", T // 2 - j, j) for j in range(b, a - 1, -1)]
    K = T - 4 * W
    if K < 0: continue
    if K % 4 == 2 and 1 <= (K - 2) // 4 <= N - 1:
        i = (K - 2) // 4
        tasks += [("X", i, c) for c in range(i - 1, -1, -1)]
    if K % 2 == 0:
        a, b = lt_range(K // 2, False)
        tasks += [("L", K // 2 - j, j) for j in range(b, a - 1, -1)]
nt = len(tasks)
dev = torch.device("cuda:0")
trace = torch.zeros(nt * 4 + N * 4, dtype=torch.int64, device=dev)
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
cs = t[nt * 4:].reshape(N, 4)
t0 = cs[0, 0]
us = lambda x: (x - t0) / 100.0   # 100 MHz -> us
print(f"n={n} N={N} tasks={nt}  chain span {us(cs[N-1, 2]):.1f} us; last task end "
      f"{us(tk[1:, 3].max()):.1f} us")
print("chain per step (us): a=wait DP+SYRK+fill, b=factor+store, c=wait SP+gemm+store")
for j in range(N):
    a = (cs[j, 1] - cs[j, 0]) / 100
    b = (cs[j, 2] - cs[j, 1]) / 100
    c = (cs[j, 3] - cs[j, 2]) / 100 if j + 1 < N else 0
    dp = [k for k, x in enumerate(tasks) if x[0] == "DP" and x[2] == j]
    sp = [k for k, x in enumerate(tasks) if x[0] == "SP" and x[2] == j]
    dpl = us(tk[dp[0], 3]) - us(cs[j, 0]) if dp else float("nan")
    spl = us(tk[sp[0], 3]) - us(cs[j, 2]) if sp else float("nan")
    if j % 4 == 0 or j > N - 5:
        print(f"j={j:3d} start {us(cs[j,0]):8.1f}  a {a:6.1f}  b {b:6.1f}  c {c:6.1f}   "
              f"DP ready {dpl:+7.1f}  SP ready {spl:+7.1f} (rel. to need)")
kinds = {}
for k in range(1, nt):
    kd = tasks[k][0]
    kinds.setdefault(kd, []).append((tk[k, 2] - tk[k, 1]) / 100)
for kd, v in kinds.items():
    print(f"{kd}: {len(v)} tasks, accumulate mean {np.mean(v):.1f} us max {np.max(v):.1f}")
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
