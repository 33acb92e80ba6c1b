"""Synthetic key batches of the BASELINE.json shapes.

Counter-based splitmix64 (seed 0x5EED by default), so any shard of any config
can be regenerated anywhere without storing it.  Keys are packed the way the
C ABI takes them: a flat uint8 buffer (+16 bytes of slack) and, for
variable-length keys, uint64 offsets[n+1].
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np

GOLDEN = np.uint64(0x9E3779B97F4A7C15)
SEED = 0x5EED
H2_SEED = 17027509906831645879   # h2_seed of the reference's level_0/filter_0.sst
TIME_CONST = 1748963255          # its timeConst


def splitmix64(counter: np.ndarray) -> np.ndarray:
    """splitmix64 output for a uint64 counter array (vectorized, wrapping)."""
    with np.errstate(over="ignore"):
        z = counter * GOLDEN + GOLDEN
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        return z ^ (z >> np.uint64(31))


def _stream(seed: int, start: int, count: int) -> np.ndarray:
    base = np.uint64((seed * 0x100000001B3) & 0xFFFFFFFFFFFFFFFF)
    with np.errstate(over="ignore"):
        ctr = np.arange(start, start + count, dtype=np.uint64) + base
    return splitmix64(ctr)


def fixed_keys(n: int, key_len: int, seed: int = SEED, first: int = 0) -> np.ndarray:
    """n keys of key_len bytes (keys first..first+n of the stream), flat uint8 + 16 slack."""
    words_per_key = (key_len + 7) // 8
    w = _stream(seed, first * words_per_key, n * words_per_key).reshape(n, words_per_key)
    b = w.view(np.uint8).reshape(n, words_per_key * 8)[:, :key_len]
    out = np.empty(n * key_len + 16, dtype=np.uint8)
    out[: n * key_len] = b.reshape(-1)
    out[n * key_len:] = 0
    return out


def var_keys(n: int, lo: int = 8, hi: int = 64, seed: int = SEED):
    """n keys with length lo + (sm64(i) mod (hi-lo+1)) and uniform random bytes.
    Returns (flat uint8 buffer + 16 slack, uint64 offsets[n+1])."""
    lens = (_stream(seed ^ 0x1EA5, 0, n) % np.uint64(hi - lo + 1)) + np.uint64(lo)
    offs = np.zeros(n + 1, dtype=np.uint64)
    np.cumsum(lens, out=offs[1:])
    total = int(offs[-1])
    nw = (total + 7) // 8
    buf = np.empty(nw * 8 + 16, dtype=np.uint8)
    # shards of a var-length set are slices of (buf, offsets) of the whole set
    buf[: nw * 8] = _stream(seed ^ 0xB17E5, 0, nw).view(np.uint8)
    buf[nw * 8:] = 0
    return buf, offs


@dataclass(frozen=True)
class Workload:
    name: str
    n: int
    key_len: int          # 0 = variable length
    m: int
    k: int
    p: float
    lo: int = 8
    hi: int = 64


# BASELINE.json configs; m from the reference formulas, except C5
# whose m is explicit (the constructor would wrap to m=1,492,685,679, k=1).
C1 = Workload("c1_10k_x16B_k3", 10_000, 16, 47_926, 3, 0.1)
C2 = Workload("c2_10M_x16B_k7", 10_000_000, 16, 95_850_584, 7, 0.01)
C3 = Workload("c3_100M_var8-64B_k7", 100_000_000, 0, 958_505_838, 7, 0.01)
C4 = Workload("c4_100M_x16B_k7_per_gpu", 100_000_000, 16, 958_505_838, 7, 0.01)
C5 = Workload("c5_1B_x32B_k10_cooperative", 1_000_000_000, 32, 4_294_967_295, 10, 0.01)
WORKLOADS = {w.name.split("_")[0]: w for w in (C1, C2, C3, C4, C5)}


def keys_for(w: Workload, n: int | None = None, seed: int = SEED, first: int = 0):
    """(buf, offsets or None, key_len) for the first n keys of workload w."""
    n = w.n if n is None else n
    if w.key_len:
        return fixed_keys(n, w.key_len, seed, first), None, w.key_len
    buf, offs = var_keys(n, w.lo, w.hi, seed)
    return buf, offs, 0
