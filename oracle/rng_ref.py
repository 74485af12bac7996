"""CPU oracle (TEST INFRASTRUCTURE ONLY) for gp_realize: Philox4x32-10 + Box-Muller in numpy.

Only ``tests/`` import this.  It restates the published counter-based generator (Salmon, Moraes,
Dror, Shaw, "Parallel random numbers: as easy as 1, 2, 3", SC'11; Philox4x32 with 10 rounds,
multipliers 0xD2511F53 / 0xCD9E8D57, Weyl keys 0x9E3779B9 / 0xBB67AE85) and the mapping
``gladsgp_amd/csrc/rng.hip`` documents: pair j = i // 2 uses counter (j_lo, j_hi, offset_lo,
offset_hi) and key (seed_lo, seed_hi); u1, u2 are the top 53 bits of words (0,1) and (2,3);
z_{2j} = r cos(2 pi u2), z_{2j+1} = r sin(2 pi u2), r = sqrt(-2 log(1 - u1)).

Pinned by the generator's published known-answer vectors (Random123 kat_vectors, philox4x32
with 10 rounds) in ``tests/test_oracle.py``.
"""
from __future__ import annotations

import numpy as np

M0, M1 = np.uint64(0xD2511F53), np.uint64(0xCD9E8D57)
W0, W1 = np.uint32(0x9E3779B9), np.uint32(0xBB67AE85)
MASK32 = np.uint64(0xFFFFFFFF)


def philox4x32_10(ctr: np.ndarray, key: tuple[int, int]) -> np.ndarray:
    """ctr (N, 4) uint32 counters -> (N, 4) uint32 outputs."""
    c = [ctr[:, i].astype(np.uint64) for i in range(4)]
    k0, k1 = np.uint32(key[0]), np.uint32(key[1])
    with np.errstate(over="ignore"):
        for _ in range(10):
            p0 = M0 * c[0]
            p1 = M1 * c[2]
            hi0, lo0 = p0 >> np.uint64(32), p0 & MASK32
            hi1, lo1 = p1 >> np.uint64(32), p1 & MASK32
            c = [hi1 ^ c[1] ^ np.uint64(k0), lo1, hi0 ^ c[3] ^ np.uint64(k1), lo0]
            k0 = np.uint32(k0 + W0)
            k1 = np.uint32(k1 + W1)
    return np.stack([x.astype(np.uint32) for x in c], axis=1)


def normals(N: int, seed: int, offset: int = 0) -> np.ndarray:
    """z_0 .. z_{N-1} as gp_realize draws them."""
    pairs = (N + 1) // 2
    j = np.arange(pairs, dtype=np.uint64)
    ctr = np.stack([(j & MASK32).astype(np.uint32), (j >> np.uint64(32)).astype(np.uint32),
                    np.full(pairs, offset & 0xFFFFFFFF, dtype=np.uint32),
                    np.full(pairs, (offset >> 32) & 0xFFFFFFFF, dtype=np.uint32)], axis=1)
    out = philox4x32_10(ctr, (seed & 0xFFFFFFFF, (seed >> 32) & 0xFFFFFFFF)).astype(np.uint64)
    scale = 2.0 ** -53
    u1 = (((out[:, 0] << np.uint64(32)) | out[:, 1]) >> np.uint64(11)).astype(np.float64) * scale
    u2 = (((out[:, 2] << np.uint64(32)) | out[:, 3]) >> np.uint64(11)).astype(np.float64) * scale
    r = np.sqrt(-2.0 * np.log(1.0 - u1))
    z = np.empty(2 * pairs)
    z[0::2] = r * np.cos(2.0 * np.pi * u2)
    z[1::2] = r * np.sin(2.0 * np.pi * u2)
    return z[:N]


def realize(mean, var, seed: int, offset: int = 0) -> np.ndarray:
    mean = np.asarray(mean, dtype=np.float64)
    var = np.asarray(var, dtype=np.float64)
    z = normals(mean.size, seed, offset).reshape(mean.shape)
    return mean + np.sqrt(np.maximum(var, 0.0)) * z
