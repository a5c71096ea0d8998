"""Seeded synthetic-input generator (TEST INFRASTRUCTURE ONLY — see oracle/__init__.py).

SURVEY.md §8(d): base seed 0x48424247; per-instance stream = SplitMix64(seed ^
instance_id).  The same generator is implemented on the device
(``hbg_synth_bytes``) so bench inputs never cross PCIe; this module is the
host-side statement of it that tests compare against.

word k of stream (tag, instance) = mix64(seed(tag, instance) + (k + 1) * GAMMA)
bytes = little-endian concatenation of words.
"""
from __future__ import annotations

import numpy as np

BASE_SEED = 0x48424247
GAMMA = 0x9E3779B97F4A7C15
M64 = (1 << 64) - 1

TAG_PAYLOAD = 1
TAG_ERASURE = 2
TAG_TDEC = 3


def mix64(z: int) -> int:
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9 & M64
    z = (z ^ (z >> 27)) * 0x94D049BB133111EB & M64
    return z ^ (z >> 31)


def stream_seed(tag: int, instance: int) -> int:
    return (BASE_SEED ^ (tag << 48) ^ instance) & M64


def words(tag: int, instance: int, count: int, start: int = 0) -> np.ndarray:
    """Vectorised SplitMix64 words [start, start+count)."""
    s = np.uint64(stream_seed(tag, instance))
    k = np.arange(start + 1, start + count + 1, dtype=np.uint64)
    with np.errstate(over="ignore"):
        z = s + k * np.uint64(GAMMA)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        z = z ^ (z >> np.uint64(31))
    return z


def synth_bytes(tag: int, instance: int, nbytes: int) -> bytes:
    w = words(tag, instance, (nbytes + 7) // 8)
    return w.astype("<u8").tobytes()[:nbytes]


def payload(instance: int, nbytes: int) -> bytes:
    return synth_bytes(TAG_PAYLOAD, instance, nbytes)


class SplitMix64:
    def __init__(self, tag: int, instance: int):
        self.s = stream_seed(tag, instance)

    def next(self) -> int:
        self.s = (self.s + GAMMA) & M64
        return mix64(self.s)


def erasure_mask(instance: int, n: int, erase: int) -> list[bool]:
    """Seeded Fisher-Yates: exactly ``erase`` of ``n`` shards marked absent."""
    rng = SplitMix64(TAG_ERASURE, instance)
    perm = list(range(n))
    for i in range(n - 1, 0, -1):
        j = rng.next() % (i + 1)
        perm[i], perm[j] = perm[j], perm[i]
    gone = set(perm[:erase])
    return [i not in gone for i in range(n)]
