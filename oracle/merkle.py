"""hbbft Merkle tree restatement (TEST INFRASTRUCTURE ONLY — see oracle/__init__.py).

Restates hbbft ``src/broadcast/merkle.rs`` [EXT, VegeBun-csj/hbbft master,
unpinned] as described in SURVEY.md §8(a) rows a4-a6 and a9:

* leaf = SHA3-256(value) with NO domain prefix (tiny-keccak ``sha3_256``);
* each level is ``chunks(2)``: a pair -> SHA3-256(left || right), a lone odd
  node is promoted unchanged; repeat until one digest (the root);
* ``proof(i)`` collects ``level[lvl_i ^ 1]`` when it exists, ``lvl_i /= 2``;
* ``Proof::validate(n)`` walks the same shape from the leaf.

Tree shape is "parity unpinned": no in-container hbbft source/fixture exists.
SHA3-256 itself is pinned by FIPS-202 (``hashlib.sha3_256``).
"""
from __future__ import annotations

import hashlib
from dataclasses import dataclass, field


def sha3(data: bytes) -> bytes:
    return hashlib.sha3_256(bytes(data)).digest()


def hash_pair(a: bytes, b: bytes) -> bytes:
    return sha3(bytes(a) + bytes(b))


@dataclass
class Proof:
    value: bytes
    index: int
    digests: list = field(default_factory=list)
    root_hash: bytes = b""

    def validate(self, n: int) -> bool:
        digest = sha3(self.value)
        lvl_i = self.index
        lvl_n = n
        it = iter(self.digests)
        while lvl_n > 1:
            if (lvl_i ^ 1) < lvl_n:
                sib = next(it, None)
                if sib is None:
                    return False  # not enough levels
                digest = hash_pair(sib, digest) if (lvl_i & 1) else hash_pair(digest, sib)
            lvl_i //= 2
            lvl_n = (lvl_n + 1) // 2
        if next(it, None) is not None:
            return False  # too many levels
        return digest == self.root_hash


class MerkleTree:
    def __init__(self, values: list):
        self.values = [bytes(v) for v in values]
        digests = [sha3(v) for v in self.values]
        self.levels: list[list[bytes]] = []
        while len(digests) > 1:
            nxt = []
            for k in range(0, len(digests), 2):
                if k + 1 < len(digests):
                    nxt.append(hash_pair(digests[k], digests[k + 1]))
                else:
                    nxt.append(digests[k])
            self.levels.append(digests)
            digests = nxt
        self.root_hash = digests[0] if digests else sha3(b"")

    @classmethod
    def from_vec(cls, values: list) -> "MerkleTree":
        return cls(values)

    def proof(self, index: int):
        if index >= len(self.values):
            return None
        lvl_i = index
        digests = []
        for level in self.levels:
            if (lvl_i ^ 1) < len(level):
                digests.append(level[lvl_i ^ 1])
            lvl_i //= 2
        return Proof(self.values[index], index, digests, self.root_hash)

    def flat_levels(self) -> list[bytes]:
        """All node digests level by level, root last (the GPU engine's
        ``levels`` output layout, see include/hbgpu.h)."""
        out = []
        for lv in self.levels:
            out.extend(lv)
        out.append(self.root_hash)
        return out


def num_nodes(n: int) -> int:
    """Digest count of ``flat_levels`` for n leaves (n >= 1)."""
    total = 0
    while n > 1:
        total += n
        n = (n + 1) // 2
    return total + 1


def depth(n: int) -> int:
    d = 0
    while n > 1:
        n = (n + 1) // 2
        d += 1
    return d
