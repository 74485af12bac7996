"""GPU parity of the TRMM schedule (predict.hip trmm_sched / trmm_merge_last, round 5).

A launch whose pair blocks do not fill whole residency rounds runs its last round (and one full
round before it) as single-tile blocks, longest first, and a last chunk smaller than one round
runs merged with the chunk before it (gp_fit_predict, gp_predict_solve, and gp_predict with its
second slab).  None of that may change a sum: every tile keeps its K order wherever it runs, so
the answers must be bit-identical across chunkings (m_chunk), across entry points (gp_predict
chunk by chunk vs gp_fit_predict's all-slab solve) and across prefixes of the test set, and
within the oracle tolerance (tests/test_gpu_kernels.py: |dmean| <= 1e-8 max|mean|,
|dvar| <= 1e-9 s) of gp_ref.predict on a sample.

Shapes: n = 1000 (NI = 8: 4 pairs, 512 / 4 blocks per round), n = 700 (npad 768, NI = 6: 3 pairs,
so rounds hold a non-integer number of panels), batches 1-3, m with a partial last chunk of a
few panels (merged) and of more than a round (not merged).
"""
import numpy as np
import pytest
import torch

from oracle import gp_ref

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def dev():
    assert torch.cuda.is_available(), "GPU tests need a HIP device"
    from gladsgp_amd import kernels  # noqa: F401
    return torch.device("cuda:0")


def _problem(n, m, B, seed):
    rng = np.random.default_rng(seed)
    X = rng.random((n, 8))
    Xs = rng.random((m, 8))
    betas = rng.uniform(0.5, 5.0, (B, 8))
    W = np.sin(X @ rng.uniform(0, 1, (8, B))).T.copy()      # (B, n)
    s = rng.uniform(0.8, 1.5, B)
    return X, Xs, betas, W, s, np.full(B, 1e-6)


@pytest.mark.parametrize("n,m,B", [
    (1000, 40000, 1),     # 2 chunks of 16384 + a 57-panel tail: 228 pair blocks, merged
    (1000, 16384 * 2 + 128 * 40, 1),   # tail of 40 panels: 160 pair blocks, merged
    (700, 30000, 2),      # 8192-point chunks for a batch; NP = 3: rounds of 170.7 panels
    (1000, 20000, 3),     # 2 chunks + a tail of 29 panels x 3 problems: 348 pair blocks, merged
])
def test_schedule_bit_identical_across_chunkings_and_paths(dev, n, m, B):
    from gladsgp_amd import kernels
    X, Xs, betas, W, s, delta = _problem(n, m, B, n + m + B)
    t = lambda a: torch.as_tensor(np.ascontiguousarray(a), device=dev)  # noqa: E731
    Xd, Xsd, bd, Wd, sd, dd = t(X), t(Xs), t(betas), t(W), t(s), t(delta)
    mean_f, var_f, ch = kernels.fit_predict(Xd, Xsd, bd, sd, dd, sd, Wd)   # all slabs, merged tail
    ch2 = kernels.cholesky_inverse(kernels.gram(Xd, bd, sd, dd, batch=B))
    ch2.check()
    assert torch.equal(ch.linv_buf, ch2.linv_buf)
    res = {"fit_predict": (mean_f, var_f)}
    res["predict"] = kernels.predict(ch2, Xd, Xsd, bd, sd, sd, Wd)        # chunk by chunk
    for mc in (1280, 4096, 12800):
        res[f"predict m_chunk={mc}"] = kernels.predict(ch2, Xd, Xsd, bd, sd, sd, Wd, m_chunk=mc)
        res[f"fit_predict m_chunk={mc}"] = kernels.fit_predict(Xd, Xsd, bd, sd, dd, sd, Wd,
                                                               m_chunk=mc)[:2]
    pre = 3000
    res_pre = kernels.predict(ch2, Xd, Xsd[:pre].contiguous(), bd, sd, sd, Wd)
    ref_m, ref_v = (r.cpu().numpy() for r in res["fit_predict"])
    for name, (mu, var) in res.items():
        assert np.array_equal(mu.cpu().numpy(), ref_m), name
        assert np.array_equal(var.cpu().numpy(), ref_v), name
    assert np.array_equal(res_pre[0].cpu().numpy(), ref_m[:, :pre])
    assert np.array_equal(res_pre[1].cpu().numpy(), ref_v[:, :pre])
    # oracle on a sample spread over every chunk (the merged tail included)
    idx = np.unique(np.concatenate([np.arange(0, m, max(1, m // 300)), np.arange(m - 200, m)]))
    for b in range(B):
        mr, vr = gp_ref.predict(X, Xs[idx], W[b], betas[b], s[b], delta[b], s_pred=s[b])
        assert np.max(np.abs(ref_m[b, idx] - mr)) <= 1e-8 * max(1.0, np.max(np.abs(mr))), b
        assert np.max(np.abs(ref_v[b, idx] - vr)) <= 1e-9 * s[b], b



@pytest.mark.parametrize("n,B", [(5, 1), (300, 2), (1000, 1), (4096, 1)])
def test_packed_linv_and_shipped_z_bit_identical(dev, n, B):
    """The sharded single-GP path's payload (sharded.LinvPacker): L^-1 tile-packed
    (gp_pack_linv, read in place by the TRMM and the trmv of gp_predict_ex) and z = L^-1 w from
    gp_predict_z give the padded path's answers bit for bit; the packed layout round-trips
    (gp_unpack_linv) and matches LinvPacker.order (host-documented layout)."""
    from gladsgp_amd import kernels
    from gladsgp_amd.sharded import LinvPacker
    m = 3000 if n < 4096 else 20000
    X, Xs, betas, W, s, delta = _problem(n, m, B, 7 * n + B)
    t = lambda a: torch.as_tensor(np.ascontiguousarray(a), device=dev)  # noqa: E731
    Xd, Xsd, bd, Wd, sd, dd = t(X), t(Xs), t(betas), t(W), t(s), t(delta)
    ch = kernels.cholesky_inverse(kernels.gram(Xd, bd, sd, dd, batch=B))
    ch.check()
    npad = kernels.padded_n(n)
    ref_m, ref_v = kernels.predict(ch, Xd, Xsd, bd, sd, sd, Wd)
    P = kernels.pack_linv(ch)
    assert P.shape == (B, kernels.linv_packed_elems(n))
    order = LinvPacker.order(npad).to(dev)
    for b in range(B):
        assert torch.equal(P[b], ch.linv_buf[b].reshape(-1)[order])
    z = kernels.predict_z(ch, Wd)
    pk = kernels.PackedLinv(n, P, ch.info)
    assert torch.equal(kernels.predict_z(pk, Wd), z)
    assert torch.all(z[:, n:] == 0)
    for name, (src, zz) in {"padded+z": (ch, z), "packed": (pk, None),
                            "packed+z": (pk, z)}.items():
        mu, var = kernels.predict(src, Xd, Xsd, bd, sd, sd, None if zz is not None else Wd, z=zz)
        assert torch.equal(mu, ref_m) and torch.equal(var, ref_v), name
    # chunked and merged-tail paths read the packed layout alike
    mu, var = kernels.predict(pk, Xd, Xsd, bd, sd, sd, Wd, m_chunk=1280)
    assert torch.equal(mu, ref_m) and torch.equal(var, ref_v)
    back = torch.zeros_like(ch.linv_buf)
    from gladsgp_amd import _capi
    for b in range(B):
        _capi.call("gp_unpack_linv", P[b].data_ptr(), n, back[b].data_ptr(), npad,
                   kernels._stream(dev))
    assert torch.equal(back, ch.linv_buf)
    # the payload as the pipelined predictor ships it (B = 1)
    if B == 1:
        packer = LinvPacker(npad, dev, n=n)
        buf = packer.buffer(dev)
        packer.pack(ch.linv_buf, ch.info, buf, w=Wd)
        assert torch.equal(packer.z(buf), z[0]) and packer.info(buf).tolist() == [0]
        mu, var = kernels.predict(packer.view(buf), Xd, Xsd, bd, sd, sd, None)
        assert torch.equal(mu, ref_m) and torch.equal(var, ref_v)
