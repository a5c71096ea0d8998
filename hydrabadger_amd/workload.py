"""Seeded synthetic workload generation for the harness (bench / examples).

Implements SURVEY.md §8(d)'s input generator on the host side where inputs
are tiny (erasure patterns); bulk bytes come from the device kernel
``hbg_synth_bytes``.  Same streams as the test oracle's statement of the
generator (oracle/synth.py), which tests compare against.
"""
from __future__ import annotations

BASE_SEED = 0x48424247
GAMMA = 0x9E3779B97F4A7C15
M64 = (1 << 64) - 1
TAG_PAYLOAD, TAG_ERASURE, TAG_TDEC = 1, 2, 3


def _mix64(z: int) -> int:
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9 & M64
    z = (z ^ (z >> 27)) * 0x94D049BB133111EB & M64
    return z ^ (z >> 31)


class SplitMix64:
    def __init__(self, tag: int, instance: int):
        self.s = (BASE_SEED ^ (tag << 48) ^ instance) & M64

    def next(self) -> int:
        self.s = (self.s + GAMMA) & M64
        return _mix64(self.s)


def erasure_mask(instance: int, n: int, erase: int) -> list:
    """Exactly ``erase`` of ``n`` shards absent, by seeded Fisher-Yates."""
    rng = SplitMix64(TAG_ERASURE, instance)
    perm = list(range(n))
    for i in range(n - 1, 0, -1):
        j = rng.next() % (i + 1)
        perm[i], perm[j] = perm[j], perm[i]
    gone = set(perm[:erase])
    return [i not in gone for i in range(n)]
