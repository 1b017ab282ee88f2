"""Synthetic push workloads of BASELINE.json's configs.

No datasets are available offline; these generators reproduce the SHAPES
the reference's apps push (sorted unique uint64 keys per push, float
values), deterministically from a seed:

* cfg2 -- ``overlap_pushes``: N pushes of n keys, ``round(overlap*n)`` "hot"
  keys shared by every push plus fresh per-push keys; all keys are distinct
  splitmix64 outputs (2^64-1 excluded).  8 x 131,072 at 10 % -> U = 956,827.
* cfg3 -- ``zipf_pushes``: Zipf(1.1) ranks in [1, 1e9], redrawn until each
  push holds n unique ranks, keys = MurmurHash3_x64_128(rank, 512927377)
  folded o[0]^o[1] (reference data/example_parser.cc:205-208).
* cfg4 -- ``dense_pushes``: N pushes of the contiguous keys [0, n).
* cfg5 -- ``uniform_pushes``: N pushes of n unique uniform ranks in
  [0, 1e9), murmur-shuffled.

Values are uniform in [-1, 1) from 24-bit (f32) / 53-bit (f64) draws, so
every value is exactly representable.
"""
from __future__ import annotations

import numpy as np

MASK64 = np.uint64(0xFFFFFFFFFFFFFFFF)
GOLDEN = np.uint64(0x9E3779B97F4A7C15)
SHUFFLE_SEED = 512927377  # data/example_parser.cc:206


def splitmix64(seed: int, count: int, offset: int = 0) -> np.ndarray:
    """splitmix64 outputs x_{offset+1 .. offset+count} of state `seed`."""
    with np.errstate(over="ignore"):
        i = np.arange(offset + 1, offset + count + 1, dtype=np.uint64)
        z = np.uint64(seed) + i * GOLDEN
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        return z ^ (z >> np.uint64(31))


def uniform_values(seed: int, count: int, dtype=np.float32) -> np.ndarray:
    """Uniform [-1, 1) values, exactly representable in `dtype`."""
    x = splitmix64(seed ^ 0x5DEECE66D, count)
    if np.dtype(dtype) == np.float32:
        return ((x >> np.uint64(40)).astype(np.float32) * np.float32(2.0 ** -23)
                - np.float32(1.0))
    return (x >> np.uint64(11)).astype(np.float64) * 2.0 ** -52 - 1.0


def _rotl(x, r):
    return (x << np.uint64(r)) | (x >> np.uint64(64 - r))


def _fmix64(k):
    k = k ^ (k >> np.uint64(33))
    k = k * np.uint64(0xFF51AFD7ED558CCD)
    k = k ^ (k >> np.uint64(33))
    k = k * np.uint64(0xC4CEB9FE1A85EC53)
    return k ^ (k >> np.uint64(33))


def murmur_shuffle(ids: np.ndarray, seed: int = SHUFFLE_SEED) -> np.ndarray:
    """MurmurHash3_x64_128 of each 8-byte id, folded o[0]^o[1]
    (util/MurmurHash3.cc:255, data/example_parser.cc:205-208)."""
    with np.errstate(over="ignore"):
        k1 = np.asarray(ids, dtype=np.uint64).copy()
        c1 = np.uint64(0x87C37B91114253D5)
        c2 = np.uint64(0x4CF5AD432745937F)
        h1 = np.full(k1.shape, seed, dtype=np.uint64)
        h2 = h1.copy()
        k1 = k1 * c1
        k1 = _rotl(k1, 31)
        k1 = k1 * c2
        h1 ^= k1
        h1 ^= np.uint64(8)
        h2 ^= np.uint64(8)
        h1 = h1 + h2
        h2 = h2 + h1
        h1 = _fmix64(h1)
        h2 = _fmix64(h2)
        h1 = h1 + h2
        h2 = h2 + h1
        return h1 ^ h2


def _distinct_stream(seed: int, count: int) -> np.ndarray:
    """First `count` distinct splitmix64 outputs (stream order), != 2^64-1."""
    got = np.zeros(0, np.uint64)
    offset = 0
    while got.size < count:
        draw = splitmix64(seed, count - got.size + 64, offset)
        offset += draw.size
        cand = np.concatenate([got, draw[draw != MASK64]])
        _, first = np.unique(cand, return_index=True)
        got = cand[np.sort(first)]
    return got[:count]


def overlap_pushes(seed: int = 1, npush: int = 8, n: int = 131072,
                   overlap: float = 0.1, dtype=np.float32, m: int = 1):
    """cfg2.  Returns (D, [(keys, [vals]*m)] * npush); D = union (sorted)."""
    hot_n = int(round(overlap * n))
    own_n = n - hot_n
    U = hot_n + npush * own_n
    keys = _distinct_stream(seed, U)
    hot = keys[:hot_n]
    pushes = []
    for p in range(npush):
        own = keys[hot_n + p * own_n: hot_n + (p + 1) * own_n]
        k = np.sort(np.concatenate([hot, own]))
        vals = [uniform_values(seed * 1000003 + p * 17 + i, n, dtype) for i in range(m)]
        pushes.append((k, vals))
    return np.sort(keys), pushes


def shard_instance(seed: int, lo: int, hi: int, npush: int = 8, n: int = 131072,
                   overlap: float = 0.1, dtype=np.float32, m: int = 1):
    """A cfg2 aggregate whose keys all lie in the server key range [lo, hi)
    (what server shard [lo, hi) receives when workers slice their pushes,
    reference message.h:89-123).  For [0, 2^64-1) it is overlap_pushes."""
    width = np.uint64((hi - lo) & 0xFFFFFFFFFFFFFFFF)
    base = np.uint64(lo)
    for attempt in range(16):
        D, pushes = overlap_pushes(seed + attempt * 7919, npush, n, overlap, dtype, m)
        with np.errstate(over="ignore"):
            Dm = np.unique(base + D % width)
            if Dm.size != D.size:
                continue  # a modulo collision: take another seed
            out = []
            for k, vs in pushes:
                mk = base + k % width
                order = np.argsort(mk, kind="stable")
                out.append((mk[order], [v[order] for v in vs]))
        return Dm, out
    raise RuntimeError("could not draw a collision-free shard instance")


def zipf_pushes(seed: int = 3, npush: int = 64, n: int = 131072, a: float = 1.1,
                rank_max: int = 10 ** 9, dtype=np.float32, m: int = 1):
    """cfg3 (CTR shape).  Returns (D, pushes)."""
    rng = np.random.default_rng(seed)
    pushes = []
    allk = []
    for p in range(npush):
        ranks = np.zeros(0, np.uint64)
        while ranks.size < n:
            d = rng.zipf(a, size=2 * n).astype(np.uint64)
            d = d[d <= rank_max]
            ranks = np.unique(np.concatenate([ranks, d]))
        # keep the n smallest-index unique ranks deterministically
        ranks = ranks[:n] if ranks.size == n else rng.choice(ranks, n, replace=False)
        k = np.unique(murmur_shuffle(ranks))
        vals = [uniform_values(seed * 1000003 + p * 17 + i, k.size, dtype) for i in range(m)]
        pushes.append((k, vals))
        allk.append(k)
    return np.unique(np.concatenate(allk)), pushes


def dense_pushes(npush: int = 8, n: int = 16777216, seed: int = 4,
                 dtype=np.float32, m: int = 1):
    """cfg4: pushes of the contiguous keys [0, n)."""
    k = np.arange(n, dtype=np.uint64)
    pushes = [(k, [uniform_values(seed * 1000003 + p * 17 + i, n, dtype) for i in range(m)])
              for p in range(npush)]
    return k, pushes


def uniform_pushes(seed: int = 5, npush: int = 256, n: int = 262144,
                   rank_max: int = 10 ** 9, dtype=np.float32, m: int = 1, union: bool = True):
    """cfg5: unique uniform ranks in [0, rank_max), murmur-shuffled.
    Returns (D, pushes); D (the union) is None when ``union`` is False."""
    rng = np.random.default_rng(seed)
    pushes = []
    for p in range(npush):
        r = np.unique(rng.integers(0, rank_max, size=n + n // 8, dtype=np.uint64))
        while r.size < n:
            r = np.unique(np.concatenate([r, rng.integers(0, rank_max, size=n, dtype=np.uint64)]))
        r = rng.choice(r, n, replace=False)
        k = np.unique(murmur_shuffle(r))
        vals = [uniform_values(seed * 1000003 + p * 17 + i, k.size, dtype) for i in range(m)]
        pushes.append((k, vals))
    D = np.unique(np.concatenate([k for k, _ in pushes])) if union else None
    return D, pushes


def shard_pieces(pushes, bounds, shard: int):
    """Each push's piece for server shard [bounds[shard], bounds[shard+1]):
    the lower_bound cut of sliceKeyOrderedMsg (reference message.h:96-99)
    at Range::all().evenDivide bounds (range.h:85-98).  Zero-copy views."""
    lo, hi = np.uint64(bounds[shard]), np.uint64(bounds[shard + 1])
    out = []
    for k, vs in pushes:
        a, b = np.searchsorted(k, [lo, hi], side="left")
        out.append((k[a:b], [v[a:b] for v in vs]))
    return out


def cfg5_shard(shard: int = 0, nshards: int = 8, seed: int = 5, npush: int = 256,
               n: int = 262144, dtype=np.float32, m: int = 1):
    """cfg5 as server shard `shard` of `nshards` receives it when workers
    slice their pushes (mode A): (D_shard, [piece per push]), D_shard = the
    union of the pieces = the shard's slice of the global key set."""
    from .kv_vector import shard_bounds
    b = shard_bounds(nshards)
    _, pushes = uniform_pushes(seed, npush, n, dtype=dtype, m=m, union=False)
    pieces = shard_pieces(pushes, b, shard)
    D = np.unique(np.concatenate([k for k, _ in pieces]))
    return D, pieces
