"""GPU parity at BASELINE config 4's full size: the multivariate emulator's 32 independent PC
GPs (n = 1024, d = 8, m = 100k shared test points; SURVEY §8d recipe: X = rng(0),
beta_j = rng(10 + j), w_j = rng(100 + j), X* = rng(2), s = 1, delta = 1e-6).

* both production paths — gram -> gp_potrf_inv -> gp_predict (bench --workload c4) and
  gp_fit_predict on a context — against the numpy oracle for PCs 0, 9, 22, 31 on a ~3000-point
  sample (the first 2000 points, every 97th after them, the last 200: every chunk and the
  tail): max|dmean| <= 1e-8 max|mean|, max|dvar| <= 1e-8 s (kappa-limited);
* the two paths agree bit for bit over all 32 x 100k predictions;
* chunk invariance (1280-point vs the default 8192-point chunks) and prefix invariance: bit
  identical; bounds 0 <= var <= s;
* the 8-way round-robin PC deal of the sharded run (4 PCs per rank, as on 8 GPUs) predicted
  rank by rank and reassembled by emulator.unit_order equals the unsharded batch bit for bit.
"""
import numpy as np
import pytest
import torch

from oracle import gp_ref

pytestmark = pytest.mark.gpu

N, M, D, P = 1024, 100_000, 8, 32
SAMPLE = 2000
CHECK_PCS = (0, 9, 22, 31)


def _c4():
    X = np.random.default_rng(0).random((N, D))
    beta = np.stack([np.random.default_rng(10 + j).uniform(0.5, 5.0, D) for j in range(P)])
    W = np.stack([np.random.default_rng(100 + j).standard_normal(N) for j in range(P)])
    Xs = np.random.default_rng(2).random((M, D))
    return X, W, beta, Xs, np.ones(P), np.full(P, 1e-6)


@pytest.fixture(scope="module")
def c4():
    assert torch.cuda.is_available(), "GPU tests need a HIP device"
    from gladsgp_amd import kernels
    dev = torch.device("cuda:0")
    X, W, beta, Xs, s, delta = _c4()
    t = {k: torch.as_tensor(v, device=dev).contiguous() for k, v in
         dict(X=X, W=W, beta=beta, Xs=Xs, s=s, delta=delta).items()}

    def run_predict(sel=None, Xs_t=None, m_chunk=0):
        sel = list(range(P)) if sel is None else list(sel)
        idx = torch.as_tensor(sel, device=dev)
        b, sv, dl, w = (t[k][idx].contiguous() for k in ("beta", "s", "delta", "W"))
        G = kernels.gram(t["X"], b, sv, dl, batch=len(sel))
        ch = kernels.cholesky_inverse(G)
        ch.check()
        mean, var = kernels.predict(ch, t["X"], t["Xs"] if Xs_t is None else Xs_t, b, sv, sv, w,
                                    m_chunk=m_chunk)
        torch.cuda.synchronize()
        return mean, var

    mean, var = run_predict()
    return dict(X=X, W=W, beta=beta, Xs=Xs, s=s, delta=delta, t=t, dev=dev, run=run_predict,
                mean=mean, var=var)


def test_c4_predict_path_vs_oracle(c4):
    mean, var = c4["mean"].cpu().numpy(), c4["var"].cpu().numpy()
    # the first SAMPLE points plus points spread over every 8192-point chunk and the tail
    m = c4["Xs"].shape[0]
    idx = np.unique(np.concatenate([np.arange(SAMPLE), np.arange(SAMPLE, m, 97),
                                    np.arange(m - 200, m)]))
    for j in CHECK_PCS:
        mr, vr = gp_ref.predict(c4["X"], c4["Xs"][idx], c4["W"][j], c4["beta"][j], 1.0, 1e-6)
        dm = np.max(np.abs(mean[j, idx] - mr))
        dv = np.max(np.abs(var[j, idx] - vr))
        print(f"C4 PC {j}: max|dmean| = {dm:.3e}, max|dvar| = {dv:.3e}")
        assert dm <= 1e-8 * np.max(np.abs(mr))
        assert dv <= 1e-8


def test_c4_fit_predict_path_bitwise(c4):
    from gladsgp_amd import kernels
    t = c4["t"]
    for aux_chunks in (-1, 1):   # every chunk beside the factorisation / only the first
        with kernels.FitPredictContext(c4["dev"], aux_chunks=aux_chunks) as fctx:
            mean, var, ch = kernels.fit_predict(t["X"], t["Xs"], t["beta"], t["s"], t["delta"],
                                                t["s"], t["W"], ctx=fctx)
            torch.cuda.synchronize()
        assert torch.equal(mean, c4["mean"]) and torch.equal(var, c4["var"])
        assert int(ch.info.abs().sum()) == 0
        del mean, var, ch


def test_c4_bounds(c4):
    mean, var = c4["mean"], c4["var"]
    assert bool(torch.isfinite(mean).all()) and bool(torch.isfinite(var).all())
    assert float(var.min()) >= -1e-12 and float(var.max()) <= 1.0 + 1e-12


def test_c4_chunk_and_prefix_invariance(c4):
    mean, var = c4["run"](m_chunk=1280)
    assert torch.equal(mean, c4["mean"]) and torch.equal(var, c4["var"])
    mean, var = c4["run"](Xs_t=c4["t"]["Xs"][:SAMPLE].contiguous())
    assert torch.equal(mean, c4["mean"][:, :SAMPLE]) and torch.equal(var, c4["var"][:, :SAMPLE])


def test_c4_eight_way_deal_reassembles(c4):
    from gladsgp_amd import dist as gdist
    from gladsgp_amd.emulator import unit_order
    world = 8
    blocks_m, blocks_v = [], []
    for r in range(world):
        mine = gdist.shard_units(P, r, world)
        assert len(mine) == 4
        m_r, v_r = c4["run"](sel=mine)
        blocks_m.append(m_r)
        blocks_v.append(v_r)
    mean = unit_order(torch.cat(blocks_m), P, world)
    var = unit_order(torch.cat(blocks_v), P, world)
    assert torch.equal(mean, c4["mean"]) and torch.equal(var, c4["var"])
