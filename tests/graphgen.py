"""Independent numpy restatement of the synthetic workload generators.

TEST HELPER: the engine's host library generates the C4/C5 graphs itself
(cg_host.cpp); these functions restate the same specification so tests can check the
engine's edge lists and traffic decisions against an independent implementation.
"""
import numpy as np

M64 = (1 << 64) - 1
GOLD = 0x9E3779B97F4A7C15
K2 = 0xD6E8FEB86659FD93


def mix64(z):
    z &= M64
    z = ((z ^ (z >> 30)) * 0xbf58476d1ce4e5b9) & M64
    z = ((z ^ (z >> 27)) * 0x94d049bb133111eb) & M64
    return z ^ (z >> 31)


def counter_hash(seed, a, b):
    h = mix64(seed ^ ((a * GOLD) & M64))
    return mix64(h ^ ((b * K2) & M64))


def mix64_np(z):
    z = z.astype(np.uint64)
    with np.errstate(over="ignore"):
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xbf58476d1ce4e5b9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94d049bb133111eb)
    return z ^ (z >> np.uint64(31))


def counter_hash_np(seed, a, b):
    a = np.asarray(a, dtype=np.uint64)
    b = np.asarray(b, dtype=np.uint64)
    with np.errstate(over="ignore"):
        h = mix64_np(np.uint64(seed) ^ (a * np.uint64(GOLD)))
        return mix64_np(h ^ (b * np.uint64(K2)))


def mulhi(x, n):
    """floor(x * n / 2^64) for a 64-bit hash x: uniform index in [0, n)."""
    return (int(x) * int(n)) >> 64


def regular_graph(n, deg, seed):
    """deg random permutations (Fisher-Yates driven by counter_hash(seed, p, i)); edge
    v -> perm_p[v] for every p; self loops dropped, duplicates collapsed (AddLink)."""
    src, dst = [], []
    for p in range(deg):
        perm = list(range(n))
        for i in range(n - 1, 0, -1):
            j = mulhi(counter_hash(seed, p, i), i + 1)
            perm[i], perm[j] = perm[j], perm[i]
        src.extend(range(n))
        dst.extend(perm)
    return dedup(np.array(src, dtype=np.int32), np.array(dst, dtype=np.int32))


def powerlaw_graph(n, m, exponent, ring, seed):
    """m out-targets per node drawn from Zipf(exponent) over rank (P(k) ~ (k+1)^-s,
    sequential double CDF, inverse by upper bound on (h >> 11) * 2^-53 * total), plus
    ring edges v -> v+1 and v -> v-1 when ring."""
    w = np.arange(1, n + 1, dtype=np.float64) ** (-exponent)
    cdf = np.cumsum(w)
    total = cdf[-1]
    v = np.repeat(np.arange(n, dtype=np.uint64), m)
    i = np.tile(np.arange(m, dtype=np.uint64), n)
    h = counter_hash_np(seed, v, i)
    r = (h >> np.uint64(11)).astype(np.float64) * (1.0 / 9007199254740992.0) * total
    k = np.searchsorted(cdf, r, side="right").astype(np.int64)
    k = np.minimum(k, n - 1)
    src = [v.astype(np.int64)]
    dst = [k]
    if ring:
        a = np.arange(n, dtype=np.int64)
        src += [a, a]
        dst += [(a + 1) % n, (a + n - 1) % n]
    return dedup(np.concatenate(src).astype(np.int32), np.concatenate(dst).astype(np.int32))


def dedup(src, dst):
    keep = src != dst
    pairs = np.unique(np.stack([src[keep], dst[keep]], axis=1), axis=0)
    return pairs[:, 0].astype(np.int32), pairs[:, 1].astype(np.int32)
