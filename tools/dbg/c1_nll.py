import sys, os
sys.path.insert(0, os.getcwd())
import numpy as np, torch, scipy.linalg as sla
from gladsgp_amd import kernels
from oracle import gp_ref
dev = torch.device("cuda:0")
x = np.vstack(np.linspace(1/8, 7/8, 64)); y = (x*np.sin(2*np.pi*x)).ravel()
for th in ([0.3, 0.05], [0.3, 0.2], [1.5, 0.35]):
    s, b, d = gp_ref.gpmodule_theta_to_kernel(th, 1e-3); b = float(b[0])
    G = gp_ref.gram_ardse(x, b, s, d)
    L = np.linalg.cholesky(G)
    Gg = kernels.gram(torch.as_tensor(x, device=dev), torch.full((1, 1), b, dtype=torch.float64, device=dev), s, d)
    print("gram maxdiff", float(np.abs(Gg[0].cpu().numpy() - G).max()))
    ch = kernels.cholesky_inverse(Gg)
    Lg = ch.L[0].cpu().numpy()
    print(th, "info", int(ch.info[0]), "L maxdiff", np.abs(Lg - L).max(), "logdet", float(ch.logdet[0]), 2*np.sum(np.log(np.diag(L))))
    Li = ch.Linv[0].cpu().numpy()
    print("  Linv@L - I", np.abs(Li @ L - np.eye(64)).max())
    bad = np.argwhere(np.abs(Lg - L) > 1e-8)
    print("  first bad", bad[:5])
    print("  nll", float(kernels.nll(ch, torch.as_tensor(y, device=dev))[0]), gp_ref.nll_gpmodule(np.array(th), x, y, 1e-3))
