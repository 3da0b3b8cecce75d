"""Seed derivation of the reference pipeline (host side).

stage_prepare/prepare.cpp:549-562: std::seed_seq{master_seed}.generate(3 x u32) -> per-stage seeds
(anaphase, interphase, prometaphase).  Each stage driver then draws its BD seeds from
std::mt19937_64(stage_seed) (stage_interphase/simulation_driver.cpp:19; stage_interphase/simulation_driver_relaxation.cpp:53 takes the first
draw, simulation_driver_interphase.cpp:61 the second).  Both algorithms are standard-specified
([rand.util.seedseq], [rand.eng.mers]); tests/test_seeds.py pins them against g++ output.
"""
from __future__ import annotations

M32 = 0xFFFFFFFF
M64 = 0xFFFFFFFFFFFFFFFF


def seed_seq_generate(seeds, n_out):
    v = [s & M32 for s in seeds]
    s = len(v)
    n = n_out
    if n == 0:
        return []
    b = [0x8B8B8B8B] * n
    t = 11 if n >= 623 else 7 if n >= 68 else 5 if n >= 39 else 3 if n >= 7 else (n - 1) // 2
    p = (n - t) // 2
    q = p + t
    m = max(s + 1, n)
    for k in range(m):
        x = b[k % n] ^ b[(k + p) % n] ^ b[(k - 1) % n]
        r1 = (1664525 * (x ^ (x >> 27))) & M32
        if k == 0:
            r2 = (r1 + s) & M32
        elif k <= s:
            r2 = (r1 + k % n + v[k - 1]) & M32
        else:
            r2 = (r1 + k % n) & M32
        b[(k + p) % n] = (b[(k + p) % n] + r1) & M32
        b[(k + q) % n] = (b[(k + q) % n] + r2) & M32
        b[k % n] = r2
    for k in range(m, m + n):
        x = (b[k % n] + b[(k + p) % n] + b[(k - 1) % n]) & M32
        r3 = (1566083941 * (x ^ (x >> 27))) & M32
        r4 = (r3 - k % n) & M32
        b[(k + p) % n] ^= r3
        b[(k + q) % n] ^= r4
        b[k % n] = r4
    return b


class MT19937_64:
    """std::mt19937_64"""

    def __init__(self, seed: int):
        mt = [0] * 312
        mt[0] = seed & M64
        for i in range(1, 312):
            mt[i] = (6364136223846793005 * (mt[i - 1] ^ (mt[i - 1] >> 62)) + i) & M64
        self.mt = mt
        self.index = 312

    def __call__(self) -> int:
        mt = self.mt
        if self.index >= 312:
            for i in range(312):
                x = (mt[i] & 0xFFFFFFFF80000000) | (mt[(i + 1) % 312] & 0x7FFFFFFF)
                xa = x >> 1
                if x & 1:
                    xa ^= 0xB5026F5AA96619E9
                mt[i] = mt[(i + 156) % 312] ^ xa
            self.index = 0
        y = mt[self.index]
        self.index += 1
        y ^= (y >> 29) & 0x5555555555555555
        y ^= (y << 17) & 0x71D67FFFEDA60000
        y ^= (y << 37) & 0xFFF7EEE000000000
        y ^= y >> 43
        return y & M64


def stage_seeds(master_seed: int) -> dict:
    a, i, p = seed_seq_generate([master_seed], 3)
    return {"anaphase": a, "interphase": i, "prometaphase": p}


def interphase_bd_seeds(stage_seed: int) -> tuple[int, int]:
    """(relaxation seed, interphase seed): the first two draws of mt19937_64(stage_seed)."""
    g = MT19937_64(stage_seed)
    return g(), g()
