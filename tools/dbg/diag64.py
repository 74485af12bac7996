import sys, os
sys.path.insert(0, os.getcwd())
import numpy as np, torch
from gladsgp_amd import kernels
from oracle import gp_ref
dev = torch.device("cuda:0")
def run(A, tag):
    L = np.linalg.cholesky(A)
    Lg, info, ld = kernels.cholesky(torch.as_tensor(A.copy(), device=dev))
    Lg = Lg[0].cpu().numpy()
    err = np.abs(Lg - L) / np.abs(L).max()
    bad = np.argwhere(err > 1e-10)
    print(f"{tag:28s} cond {np.linalg.cond(A):.1e} info {int(info[0])} maxrel {err.max():.2e} first bad {bad[:3].tolist()}")
x = np.vstack(np.linspace(1/8, 7/8, 64))
for th1 in (0.02, 0.05, 0.1):
    s, b, d = gp_ref.gpmodule_theta_to_kernel([0.3, th1], 1e-3)
    run(gp_ref.gram_ardse(x, b, s, d), f"grid d=1 l={th1}")
rng = np.random.default_rng(0)
for c in (1e2, 1e4, 1e6, 1e8):
    Q, _ = np.linalg.qr(rng.standard_normal((64, 64)))
    ev = np.logspace(0, -np.log10(c), 64)
    run((Q * ev) @ Q.T, f"random Q cond {c:.0e}")
for c in (1e2, 1e6):
    ev = np.logspace(0, -np.log10(c), 64)
    run(np.diag(ev), f"diag cond {c:.0e}")
# tridiagonal-ish
T = np.eye(64) * 2 - np.eye(64, k=1) - np.eye(64, k=-1)
run(T, "tridiag 2,-1")
Xr = rng.random((64, 8))
run(gp_ref.gram_ardse(Xr, np.full(8, 0.3), 1.0, 1e-6), "random d=8 beta 0.3")
run(gp_ref.gram_ardse(Xr, np.full(8, 3.0), 1.0, 1e-6), "random d=8 beta 3")
