#!/usr/bin/env python3
"""Regenerate Go's ``math/rand`` ``rngCooked[607]`` table offline (TEST INFRASTRUCTURE).

Go (``go.mod:3`` pins go 1.22.0) seeds every ``rand.Source`` by XOR-ing a MINSTD
expansion of the seed with a constant table ``rngCooked``.  That table is *defined*
(Go's ``math/rand/gen_cooked.go``) as the state of the additive lagged-Fibonacci
generator ``y_m = y_{m-607} + y_{m-273} (mod 2^64)`` after 7.8e12 steps, started from
``srand(1)`` with gen-seed shifts 20/10 (not the 40/20 used by ``Seed``).  Go is
not installed in this image, so we restate that definition and jump 7.8e12 steps
ahead with polynomial arithmetic modulo ``x^607 - x^334 - 1`` over Z/2^64.

The result is pinned by the KATs in SURVEY.md Appendix B (first entries, last
entry, SHA-256 of the decimal list) and -- end to end -- by Go's published
``Int63`` outputs for seed 1 and by all 21 reference golden snapshots, which are
only reproduced with the exact Go stream (``snapshot_test.go:9,20``).

Usage: python oracle/gen_go_rng_cooked.py  -> writes
  tests/golden/go_rng_cooked.txt                       (607 signed decimals)
  oracle/go_rng_cooked.h                               (oracle's copy)
  <pkg>/csrc/go_rng_cooked.inc                         (product's copy)
"""
import hashlib
import os
import sys

import numpy as np

LEN, TAP = 607, 273
FEED0 = LEN - TAP          # 334
M31 = (1 << 31) - 1
STEPS = 7_800_000_000_000  # "7.8e12 calls to vrand" (gen_cooked.go)
MASK64 = (1 << 64) - 1

KAT_FIRST = [-4181792142133755926, -4576982950128230565, 1395769623340756751,
             5333664234075297259]
KAT_LAST = 4152330101494654406
KAT_SHA = "7c51f264024398f110804d3ad6925fde46207de08132b26bffaa2e9e09505997"

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = "chandy-lamport-distributed-snapshot-algorithm_amd"


def seedrand(x: int) -> int:
    """MINSTD step via Schrage's method, exactly as Go's seedrand (rng.go)."""
    hi, lo = divmod(x, 44488)
    x = 48271 * lo - 3399 * hi
    if x < 0:
        x += M31
    return x


def gen_srand_vec(seed: int):
    """gen_cooked.go srand(): shifts 20/10, no table XOR."""
    seed %= M31
    if seed == 0:
        seed = 89482311
    x = seed
    vec = [0] * LEN
    for i in range(-20, LEN):
        x = seedrand(x)
        if i >= 0:
            u = (x << 20) & MASK64
            x = seedrand(x)
            u ^= (x << 10) & MASK64
            x = seedrand(x)
            u ^= x
            vec[i] = u
    return vec


def polymulmod(a: np.ndarray, b: np.ndarray) -> np.ndarray:
    """(a*b) mod (x^607 - x^334 - 1), coefficients mod 2^64 (uint64 wraps)."""
    c = np.zeros(2 * LEN - 1, dtype=np.uint64)
    with np.errstate(over="ignore"):
        for i in np.nonzero(a)[0]:
            c[i:i + LEN] += a[i] * b
        # x^k = x^(k-607) * (x^334 + 1) for k >= 607, highest first
        for k in range(2 * LEN - 2, LEN - 1, -1):
            ck = c[k]
            if ck:
                c[k - LEN + FEED0] += ck
                c[k - LEN] += ck
                c[k] = 0
    return c[:LEN].copy()


def x_pow_mod(n: int) -> np.ndarray:
    result = np.zeros(LEN, dtype=np.uint64)
    result[0] = 1
    base = np.zeros(LEN, dtype=np.uint64)
    base[1] = 1
    while n:
        if n & 1:
            result = polymulmod(result, base)
        n >>= 1
        if n:
            base = polymulmod(base, base)
    return result


def cooked_table(steps: int = STEPS):
    vec0 = gen_srand_vec(1)
    # The state holds a window of the sequence z: slot (333 - i) mod 607 holds z_i,
    # initial window z_0..z_606; each vrand() writes z_{607+j} into slot of z_j.
    z = [vec0[(FEED0 - 1 - i) % LEN] for i in range(LEN)]
    for m in range(LEN, 2 * LEN - 1):
        z.append((z[m - LEN] + z[m - TAP]) & MASK64)
    coeff = [int(v) for v in x_pow_mod(steps)]
    out = [0] * LEN
    for i in range(LEN):
        s = 0
        for j, cj in enumerate(coeff):
            if cj:
                s += cj * z[i + j]
        zi = s & MASK64                      # z_{steps + i}
        out[(FEED0 - 1 - (steps + i)) % LEN] = zi
    return [v - (1 << 64) if v >= (1 << 63) else v for v in out]


def brute_force(steps: int):
    """Direct vrand() loop, used to self-check the jump for small step counts."""
    vec = gen_srand_vec(1)
    tap, feed = 0, FEED0
    for _ in range(steps):
        tap = (tap - 1) % LEN
        feed = (feed - 1) % LEN
        vec[feed] = (vec[feed] + vec[tap]) & MASK64
    return [v - (1 << 64) if v >= (1 << 63) else v for v in vec]


def main():
    for n in (0, 1, 5, 273, 607, 1500):
        assert cooked_table(n) == brute_force(n), f"jump-ahead self-check failed at {n}"
    tab = cooked_table()
    text = "\n".join(str(v) for v in tab)
    sha = hashlib.sha256(text.encode()).hexdigest()
    ok = tab[:4] == KAT_FIRST and tab[606] == KAT_LAST and sha == KAT_SHA
    print("rngCooked sha256", sha, "KAT", "OK" if ok else "MISMATCH")
    if not ok:
        sys.exit(1)
    with open(os.path.join(ROOT, "tests", "golden", "go_rng_cooked.txt"), "w") as f:
        f.write(text + "\n")
    body = ",\n".join(
        ", ".join(f"(int64_t){v}LL" if v != -(1 << 63) else "INT64_MIN" for v in tab[i:i + 3])
        for i in range(0, LEN, 3))
    hdr = ("/* GENERATED by oracle/gen_go_rng_cooked.py -- Go math/rand rngCooked[607]\n"
           f" * sha256(decimal list) = {sha} */\n")
    with open(os.path.join(ROOT, "oracle", "go_rng_cooked.h"), "w") as f:
        f.write(hdr + "#include <stdint.h>\nstatic const int64_t ORC_RNG_COOKED[607] = {\n"
                + body + "\n};\n")
    with open(os.path.join(ROOT, PKG, "csrc", "go_rng_cooked.inc"), "w") as f:
        f.write(hdr + body + "\n")


if __name__ == "__main__":
    main()
