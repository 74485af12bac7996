"""A/B of gp_field variants (gladsgp_amd/csrc/field.hip compiled alone with -D flags) at the
C5 field shape: w (100k x 64) fp64, K (64 x 10k), sd / mu, float32 output.
    python tools/field_ab.py --build      # here: compile _ab/field_<name>.so
    python tools/field_ab.py              # GPU: interleaved timing, bit-equality vs the first
"""
import ctypes
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# round 6 first pass (profiles/r06/r06c_field_ab.log): base (plain stores) 3.78 ms, nt 3.26,
# 32-row tiles at one block per CU 4.52-4.75, one block per CU 5.27. Second pass
# (r06i_field_ab.log): JT 4 / 2 blocks per CU 3.13, JT 2 / 3 per CU 3.02 (adopted), 8-wave
# blocks 3.18-3.26, 32-row tiles at JT 2 3.13.  Late round 6: float32 output staged through LDS
# and stored 16 B per lane (FIELD_ST16) against the 4-B stores of the MFMA C layout.
VARIANTS = {
    "base": ["-DFIELD_ST16=0"],
    "st16": [],
    "nostore": ["-DFIELD_PROBE=1"],           # timing probe: no output written (bits differ)
}


def build():
    os.makedirs(os.path.join(ROOT, "_ab"), exist_ok=True)
    for name, flags in VARIANTS.items():
        out = os.path.join(ROOT, "_ab", f"field_{name}.so")
        cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC",
               "-shared", *flags, os.path.join(ROOT, "gladsgp_amd", "csrc", "field.hip"),
               "-o", out]
        subprocess.run(cmd, check=True)
        print(out)


def run(rows=100_000, P=64, ncols=10_000, reps=5, rounds=3):
    import numpy as np
    import torch
    dev = torch.device("cuda", 0)
    g = torch.Generator(device="cpu").manual_seed(0)
    W = torch.randn((rows, P), generator=g, dtype=torch.float64).to(dev)
    K = torch.randn((P, ncols), generator=g, dtype=torch.float64).to(dev)
    sd = (torch.rand(ncols, generator=g, dtype=torch.float64) + 0.5).to(dev)
    mu = torch.randn(ncols, generator=g, dtype=torch.float64).to(dev)
    libs = {}
    for name in VARIANTS:
        lib = ctypes.CDLL(os.path.join(ROOT, "_ab", f"field_{name}.so"))
        fn = lib.gp_field
        fn.restype = ctypes.c_int
        c_ll, c_int, c_p = ctypes.c_longlong, ctypes.c_int, ctypes.c_void_p
        fn.argtypes = [c_p, c_ll, c_int, c_int, c_p, c_ll, c_int, c_p, c_p, c_p, c_p, c_ll, c_int,
                       c_p]
        libs[name] = fn
    outs = {n: torch.empty((rows, ncols), dtype=torch.float32, device=dev) for n in libs}
    st = torch.cuda.current_stream().cuda_stream
    flop = 2.0 * rows * ncols * P
    res = {n: [] for n in libs}
    for r in range(rounds):
        order = list(libs) if r % 2 == 0 else list(libs)[::-1]
        for n in order:
            fn, Y = libs[n], outs[n]
            rc = fn(W.data_ptr(), P, rows, P, K.data_ptr(), ncols, ncols, sd.data_ptr(),
                    mu.data_ptr(), None, Y.data_ptr(), ncols, 1, st)
            assert rc == 0, (n, rc)
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(reps):
                fn(W.data_ptr(), P, rows, P, K.data_ptr(), ncols, ncols, sd.data_ptr(),
                   mu.data_ptr(), None, Y.data_ptr(), ncols, 1, st)
            e1.record()
            torch.cuda.synchronize()
            res[n].append(e0.elapsed_time(e1) / reps)
    base = outs["base"]
    for n in libs:
        ms = min(res[n])
        print(f"{n:12s} {ms:7.3f} ms  ({', '.join(f'{t:.3f}' for t in res[n])})  "
              f"{flop / ms / 1e9:7.1f} TF/s  {rows * ncols * 4 / ms / 1e6:7.0f} GB/s  "
              f"same bits as base: {bool(torch.equal(outs[n], base))}", flush=True)


if __name__ == "__main__":
    if "--build" in sys.argv:
        build()
    else:
        run()
