"""CPU: the C-ABI library builds, loads, and exports every symbol include/gpfit.h declares.

No device work happens here: only host-side entry points (sizes, argument validation that
returns before any launch) are called.
"""
import ctypes
import os
import re
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "gpfit.h")


def _declared():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(gp_[a-z_0-9]+)\s*\(", src)))


@pytest.fixture(scope="module")
def lib():
    from gladsgp_amd import _build, _capi
    _build.build_library()
    return _capi.lib()


def test_header_declares_expected_entry_points():
    names = _declared()
    for must in ("gp_gram_ardse", "gp_cross_ardse", "gp_potrf_inv", "gp_predict",
                 "gp_predict_ws_bytes", "gp_nll", "gp_trmv", "gp_padded_n", "gp_version",
                 "gp_loglik", "gp_loglik_ws_bytes"):
        assert must in names


def test_every_declared_symbol_is_exported(lib):
    from gladsgp_amd import _build, _capi
    out = subprocess.run(["nm", "-D", "--defined-only", _build.LIB_PATH], capture_output=True,
                         text=True, check=True).stdout
    exported = set(re.findall(r"\bT (gp_[a-z_0-9]+)", out))
    for name in _declared():
        assert name in exported, name
        assert name in _capi.SIGNATURES, f"{name} lacks a ctypes signature"
    # _capi.lib() binds what it finds (older builds in same-box A/B runs): the shipped build
    # must export every signature it knows
    for name in _capi.SIGNATURES:
        assert name in exported, name
        assert getattr(lib, name).argtypes is not None or not _capi.SIGNATURES[name][1], name


def test_library_has_gfx950_code_object():
    from gladsgp_amd import _build
    data = open(_build.LIB_PATH, "rb").read()
    assert b"amdgcn-amd-amdhsa--gfx950" in data


def test_host_side_helpers(lib):
    assert lib.gp_version() >= 100
    assert lib.gp_padded_n(1) == 128
    assert lib.gp_padded_n(4096) == 4096
    assert lib.gp_padded_n(4097) == 4224
    assert lib.gp_padded_n(0) == 0
    ws = lib.gp_predict_ws_bytes(4096, 100000, 1, 0)
    assert ws > 4096 * 4096 * 8 // 4
    # a given chunk bounds the cross-covariance scratch
    small = lib.gp_predict_ws_bytes(4096, 100000, 1, 1024)
    assert small < ws
    assert lib.gp_predict_ws_bytes(0, 10, 1, 0) == 0


def test_argument_validation_returns_lapack_style_codes(lib):
    # invalid arguments are rejected on the host before any launch
    rc = lib.gp_gram_ardse(None, 10, 2, 2, None, 2, None, None, None, 10, 100, 1, None)
    assert rc == -1
    dummy = ctypes.c_void_p(16)
    rc = lib.gp_gram_ardse(dummy, 10, 0, 2, dummy, 2, dummy, dummy, dummy, 10, 100, 1, None)
    assert rc == -3   # d out of range
    rc = lib.gp_gram_ardse(dummy, 10, 2, 2, dummy, 2, dummy, dummy, dummy, 5, 100, 1, None)
    assert rc == -10  # ldg < n
    rc = lib.gp_potrf_inv(dummy, 100, 100, 10000, dummy, 64, 4096, 1, None, None, None)
    assert rc == -6   # ldinv < gp_padded_n(n)
    rc = lib.gp_predict(dummy, 128, 128 * 128, dummy, 2, dummy, 2, 100, 10, 2, dummy, 2, dummy,
                        dummy, dummy, 100, dummy, dummy, 10, 1, dummy, 0, 0, None)
    assert rc == -22  # workspace too small
    # zero-sized problems are a no-op
    assert lib.gp_potrf_inv(dummy, 0, 1, 0, dummy, 1, 0, 1, None, None, None) == 0
    # gp_loglik: workspace size grows with the batch; bad args rejected before any launch
    assert lib.gp_loglik_ws_bytes(512, 8) > lib.gp_loglik_ws_bytes(512, 1) > 512 * 512 * 8
    assert lib.gp_loglik_ws_bytes(-1, 1) == -1
    rc = lib.gp_loglik(dummy, 64, 0, 2, dummy, 2, dummy, dummy, dummy, 64, 1, dummy, 1 << 30,
                       dummy, None, None)
    assert rc == -3   # d < 1
    wsp = ctypes.c_void_p(256)                       # workspaces are 256-B aligned
    rc = lib.gp_loglik(dummy, 64, 2, 2, dummy, 2, dummy, dummy, dummy, 64, 2, wsp, 16,
                       dummy, None, None)
    assert rc == -13  # workspace too small
    rc = lib.gp_loglik(dummy, 64, 2, 2, dummy, 2, dummy, dummy, dummy, 64, 2, dummy, 1 << 30,
                       dummy, None, None)
    assert rc == -12  # workspace not 256-B aligned
    assert lib.gp_loglik(dummy, 0, 2, 2, dummy, 2, dummy, dummy, dummy, 0, 1, None, 0, dummy,
                         None, None) == 0
    # gp_fit_predict: validated before anything is enqueued
    assert lib.gp_fit_predict_ws_bytes(4096, 100000, 1, 0) >= lib.gp_predict_ws_bytes(4096,
                                                                                       100000,
                                                                                       1, 0)
    args = [dummy, 2, dummy, 2, 100, 10, 2, dummy, 2, dummy, dummy, dummy, dummy, 100,
            dummy, 100, 10000, dummy, 128, 128 * 128, None, None, dummy, dummy, 10, 1, wsp,
            1 << 40, 0, None, None]
    bad = list(args)
    bad[10] = None                                   # delta
    assert lib.gp_fit_predict(*bad) == -24
    bad = list(args)
    bad[15] = 50                                     # ldg < n
    assert lib.gp_fit_predict(*bad) == -26
    bad = list(args)
    bad[27] = 16                                     # workspace too small
    assert lib.gp_fit_predict(*bad) == -22
    bad[26] = ctypes.c_void_p(16)                    # workspace not 256-B aligned
    bad[27] = 1 << 40
    assert lib.gp_fit_predict(*bad) == -21


def test_new_entry_points_validate(lib):
    """gp_potrf / gp_trtri / gp_predict_chol / gp_ctx_*: argument checks before any launch."""
    dummy = ctypes.c_void_p(16)
    assert lib.gp_potrf(None, 4, 4, 16, 1, None, None, None) == -1
    assert lib.gp_potrf(dummy, 4, 3, 16, 1, None, None, None) == -3
    assert lib.gp_potrf(dummy, 4, 4, 8, 2, None, None, None) == -4
    assert lib.gp_potrf(dummy, 0, 1, 0, 1, None, None, None) == 0
    assert lib.gp_trtri(None, 4, 4, 16, dummy, 128, 128 * 128, 1, None, None) == -1
    assert lib.gp_trtri(dummy, 4, 4, 16, dummy, 64, 128 * 128, 1, None, None) == -6
    assert lib.gp_trtri(dummy, 4, 4, 16, None, 128, 128 * 128, 1, None, None) == -5
    assert lib.gp_predict_chol_ws_bytes(4096, 100000, 1, 0) == (
        8 * 4096 * 4096 + lib.gp_predict_ws_bytes(4096, 100000, 1, 0))
    args = [dummy, 100, 10000, dummy, 2, dummy, 2, 100, 10, 2, dummy, 2, dummy, dummy, dummy,
            100, dummy, dummy, 10, 1, None, dummy, 1 << 40, 0, None]
    bad = list(args)
    bad[0] = None
    assert lib.gp_predict_chol(*bad) == -1
    bad = list(args)
    bad[22] = 16                                     # workspace too small
    assert lib.gp_predict_chol(*bad) == -23
    assert lib.gp_ctx_create(2.0, 0, dummy) == -1
    assert lib.gp_ctx_create(0.4, 0, None) == -3
    assert lib.gp_ctx_destroy(None) == 0
    assert lib.gp_ctx_set_aux_chunks(None, 1) == -1
    assert lib.gp_ctx_set_aux_chunks(dummy, -5) == -2      # rejected before the handle is read


def test_mcmc_group_step_validates(lib):
    """gp_mcmc_group_step: both groups' arguments are checked before the launch (the second
    group's prep codes shifted by -10)."""
    from gladsgp_amd import _capi
    S = _capi.McmcState()
    for nm, _ in S._fields_[:14]:
        setattr(S, nm, 64)                           # non-null, never dereferenced here
    S.P, S.d = 4, 2
    T = _capi.McmcState()
    ctypes.pointer(T)[0] = S
    k = (ctypes.c_int * 2)(1, 2)
    dummy = ctypes.c_void_p(64)
    pS, pT = ctypes.addressof(S), ctypes.addressof(T)
    assert lib.gp_mcmc_group_step(None, k, 2, 0, dummy, pT, k, 2, 0, dummy, dummy, dummy,
                                  None) == -1
    assert lib.gp_mcmc_group_step(pS, k, 2, 0, None, pT, k, 2, 0, dummy, dummy, dummy,
                                  None) == -7
    assert lib.gp_mcmc_group_step(pS, k, 2, 0, dummy, None, k, 2, 0, dummy, dummy, dummy,
                                  None) == -11
    bad = (ctypes.c_int * 2)(1, 9)                   # update code > d + 3
    assert lib.gp_mcmc_group_step(pS, k, 2, 0, dummy, pT, bad, 2, 0, dummy, dummy, dummy,
                                  None) == -16
    assert lib.gp_mcmc_group_step(pS, k, 2, 0, dummy, pT, k, 2, 0, None, dummy, dummy,
                                  None) == -17
    T.P = 5
    assert lib.gp_mcmc_group_step(pS, k, 2, 0, dummy, pT, k, 2, 0, dummy, dummy, dummy,
                                  None) == -18


def test_comm_argument_validation(lib):
    # RCCL wrappers: bad arguments are rejected before librccl is touched
    dummy = ctypes.c_void_p(16)
    assert lib.gp_comm_init(0, 0, dummy, dummy) == -1
    assert lib.gp_comm_init(2, 2, dummy, dummy) == -2
    assert lib.gp_comm_init(1, 0, None, dummy) == -3
    assert lib.gp_comm_unique_id(None) == -1
    assert lib.gp_bcast(None, dummy, 8, 0, None) == -1
    assert lib.gp_gather(None, dummy, 8, dummy, 0, None) == -1
    assert lib.gp_comm_destroy(None) == -1
    assert lib.gp_comm_available() in (0, 1)


def test_product_path_fails_loudly_without_library(monkeypatch, tmp_path):
    from gladsgp_amd import _capi
    monkeypatch.setattr(_capi, "_LIB", None)
    monkeypatch.setattr(_capi, "LIB_PATH", str(tmp_path / "missing.so"))
    with pytest.raises(_capi.GPFitUnavailable):
        _capi.lib()


def test_factorisation_workspace_entry_points(lib):
    """gp_potrf_inv_ws / gp_potrf_ws: sized scratch, validated before any launch; the
    allocating forms validate before allocating."""
    dummy = ctypes.c_void_p(16)
    wsp = ctypes.c_void_p(256)
    inv = lib.gp_potrf_inv_ws_bytes(4096, 1)
    assert inv > 0 and lib.gp_potrf_inv_ws_bytes(4096, 8) > inv
    assert lib.gp_potrf_inv_ws_bytes(-1, 1) == -1
    assert lib.gp_potrf_inv_ws_bytes(64 * 241, 1) == 0          # beyond the persistent kernel
    assert lib.gp_potrf_ws_bytes(512, 4) > lib.gp_potrf_inv_ws_bytes(512, 4)
    # gp_fit_predict / gp_loglik carry the factorisation's scratch in their own workspace
    assert (lib.gp_fit_predict_ws_bytes(4096, 100000, 1, 0) >=
            lib.gp_predict_prepared_ws_bytes(4096, 100000, 1, 0) + inv)
    assert lib.gp_loglik_ws_bytes(512, 8) > lib.gp_potrf_inv_ws_bytes(512, 8)
    assert lib.gp_potrf_inv_ws(None, 10, 10, 100, dummy, 128, 128 * 128, 1, None, None, wsp,
                               1 << 30, None) == -1
    assert lib.gp_potrf_inv_ws(dummy, 100, 100, 10000, dummy, 64, 4096, 1, None, None, wsp,
                               1 << 30, None) == -6
    assert lib.gp_potrf_ws(dummy, 4, 3, 16, 1, None, None, wsp, 1 << 30, None) == -3
    assert lib.gp_potrf_ws(dummy, 0, 1, 0, 1, None, None, None, 0, None) == 0
    assert lib.gp_potrf(dummy, 4, 4, 8, 2, None, None, None) == -4   # before any allocation
    assert lib.gp_loglik_status(None, 4, 1, 0, None) == -1
    assert lib.gp_loglik_status(wsp, 0, 1, 0, None) == 0


def _kernel_resources():
    """Per-kernel register and LDS use read from the built library's gfx950 code objects
    (offload bundles -> AMDGPU metadata note, printed by llvm-readelf)."""
    import re
    import shutil
    import struct
    import subprocess
    import tempfile
    from gladsgp_amd import _build
    readelf = shutil.which("llvm-readelf") or "/opt/rocm/llvm/bin/llvm-readelf"
    if not os.path.exists(_build.LIB_PATH) or not os.path.exists(readelf):
        pytest.skip("built library or llvm-readelf missing")
    data = open(_build.LIB_PATH, "rb").read()
    out, pos = {}, 0
    while True:
        i = data.find(b"__CLANG_OFFLOAD_BUNDLE__", pos)
        if i < 0:
            break
        pos = i + 24
        n = struct.unpack_from("<Q", data, i + 24)[0]
        p = i + 32
        for _ in range(n):
            off, size, tl = struct.unpack_from("<QQQ", data, p)
            p += 24
            triple = data[p:p + tl].decode(errors="replace")
            p += tl
            if "gfx950" not in triple or not size:
                continue
            with tempfile.NamedTemporaryFile(suffix=".co") as f:
                f.write(data[i + off:i + off + size])
                f.flush()
                notes = subprocess.run([readelf, "--notes", f.name], capture_output=True,
                                       text=True, check=True).stdout
            for blk in notes.split("\n  - ")[1:]:
                name = re.search(r"\.name:\s+(\S+)", blk)
                if not name:
                    continue
                g = lambda k: int(re.search(r"\." + k + r":\s+(\d+)", blk).group(1))  # noqa
                out[name.group(1)] = {"vgpr": g("vgpr_count"), "agpr": g("agpr_count"),
                                      "lds": g("group_segment_fixed_size")}
    return out


def _alloc(r):
    """Registers a wave of the kernel holds per lane on gfx950 (unified VGPR/AGPR file: the
    metadata's .vgpr_count is the total, arch VGPRs + AGPRs), in granules of 8."""
    return -(-r["vgpr"] // 8) * 8


def test_persistent_factorisation_leaves_room_for_cross():
    """gp_fit_predict runs the cross-covariance (cross_kp_kernel<8>, every d <= 8 config) beside
    the persistent factorisation (pp_kernel, one 4-wave workgroup per CU); that overlap exists
    only while one wave of each fits on a SIMD: registers <= 512 per lane, LDS <= 160 KB per CU.
    Round 4 found it broken by 10 extra pp_kernel registers (C3 27.7 vs 26.8 ms per step: the
    cross-covariance waited for the whole factorisation) -- this guards the budget."""
    res = _kernel_resources()
    # pp_kernel<false>: the factorisation gp_fit_predict overlaps (pp_kernel<true> is
    # gp_loglik's in-chain mode, which runs with no cross-covariance beside it)
    pp = [v for k, v in res.items() if "pp_kernelILb0E" in k]
    cross = [v for k, v in res.items() if "cross_kp_kernelILi8E" in k]
    assert pp and cross, sorted(res)[:20]
    pp, cross = pp[0], cross[0]
    assert _alloc(pp) + _alloc(cross) <= 512, (pp, cross, _alloc(pp), _alloc(cross))
    assert pp["lds"] + cross["lds"] <= 160 * 1024, (pp, cross)


@pytest.mark.parametrize("seed,pre,shape", [
    (0, 0, (1,)), (0, 1, (1,)), (1, 0, (2,)), (2, 3, (3,)), (3, 0, (7, 5)), (4, 5, (1000,)),
    (5, 0, (624,)), (6, 623, (20001,)), (7, 0, (3000, 50)), (8, 311, (157,)), (9, 2, (0,)),
    # above 2 x kBatch (2^20 accepted pairs = 2^21 deviates per batch, host_rng.hip): the
    # double-buffered path -- flush(false), buffer swap, one batch's transform threads beside
    # the next batch's fill -- runs several times, as it does for the fit's 1.35M x 25 Omega
    (10, 7, (4_300_001,))])
def test_legacy_normal_matches_numpy(seed, pre, shape):
    """svd.legacy_normal_f32 (gp_host_legacy_normal_f32, host code: no GPU) == the reference's
    np.random.normal(size=...).astype(np.float32) (src/svd.py:51) bit for bit, from any
    generator position (pre draws: odd counts leave a cached deviate, pos anywhere in a twist),
    and numpy's global state afterwards equals the state numpy's own call leaves."""
    from gladsgp_amd.svd import legacy_normal_f32
    np.random.seed(seed)
    np.random.normal(size=pre)
    st = np.random.get_state()
    ref = np.random.normal(size=shape).astype(np.float32)
    st_ref = np.random.get_state()
    np.random.set_state(st)
    got = legacy_normal_f32(shape, threads=3)
    st_got = np.random.get_state()
    assert got.dtype == np.float32 and got.shape == ref.shape
    assert np.array_equal(got.view(np.uint32), ref.view(np.uint32))
    assert np.array_equal(st_got[1], st_ref[1]) and st_got[2:] == st_ref[2:]


def test_legacy_normal_draw_on_worker_thread():
    """svd.LegacyNormalDraw (init_model's Omega, drawn beside the upload): the same deviates as
    the reference's np.random.normal((ny, 25)).astype(float32) (src/svd.py:51), numpy's global
    state read on the calling thread when the draw starts and advanced there by result()."""
    from gladsgp_amd.svd import LegacyNormalDraw
    np.random.seed(11)
    st0 = np.random.get_state()
    ref = np.random.normal(size=(30001, 25)).astype(np.float32)
    st_ref = np.random.get_state()
    np.random.set_state(st0)
    draw = LegacyNormalDraw((30001, 25), threads=2)
    got = draw.result()
    assert np.array_equal(got.view(np.uint32), ref.view(np.uint32))
    st = np.random.get_state()
    assert np.array_equal(st[1], st_ref[1]) and st[2:] == st_ref[2:]
    assert draw.result() is got                 # result() advances the state once
    assert np.array_equal(np.random.get_state()[1], st_ref[1])


def test_legacy_normal_argument_validation(lib):
    key = (ctypes.c_uint * 624)()
    pos, hg, g = ctypes.c_int(624), ctypes.c_int(0), ctypes.c_double(0.0)
    out = (ctypes.c_float * 4)()
    f = lib.gp_host_legacy_normal_f32
    assert f(None, ctypes.byref(pos), ctypes.byref(hg), ctypes.byref(g), 4, out, 1) == -1
    bad = ctypes.c_int(625)
    assert f(key, ctypes.byref(bad), ctypes.byref(hg), ctypes.byref(g), 4, out, 1) == -2
    assert f(key, ctypes.byref(pos), ctypes.byref(hg), ctypes.byref(g), -1, out, 1) == -5
    assert f(key, ctypes.byref(pos), ctypes.byref(hg), ctypes.byref(g), 4, None, 1) == -6


def test_legacy_normal_reproduces_the_reference_omega():
    """The golden test matrices drawn by the reference's own src/svd.py:51 after
    np.random.seed(123) (tests/golden/svd_ref_64x500.npz, make_golden.py) come out of
    svd.legacy_normal_f32 bit for bit after the same seed."""
    from gladsgp_amd.svd import legacy_normal_f32
    g = np.load(os.path.join(os.path.dirname(__file__), "golden", "svd_ref_64x500.npz"))
    for tag in ("p8", "p25k0"):
        ref = g[f"{tag}_omega"]
        np.random.seed(123)
        got = legacy_normal_f32(ref.shape, threads=4)
        assert np.array_equal(got.view(np.uint32), ref.view(np.uint32)), tag


def test_predict_workspace_holds_the_merged_tail(lib):
    """gp_predict sizes two cross-covariance slabs exactly when the last chunk is partial (so it
    can run merged with the chunk before it), one otherwise."""
    full = lib.gp_predict_ws_bytes(1000, 32768, 1, 0)
    part = lib.gp_predict_ws_bytes(1000, 32768 + 128, 1, 0)
    one = lib.gp_predict_ws_bytes(1000, 16384, 1, 0)
    slab = 8 * 1024 * 16384                         # npad x chunk doubles
    assert part - full >= slab                      # the second slab (+ partial sums)
    assert full == one                              # whole chunks reuse one slab
