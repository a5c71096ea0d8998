"""hbbft Broadcast glue restatement (TEST INFRASTRUCTURE ONLY — see oracle/__init__.py).

Restates hbbft ``src/broadcast/broadcast.rs`` [EXT, unpinned]:
``Broadcast::new`` (data = N - 2f, parity = 2f, ``Coding::Trivial`` when
parity == 0), ``send_shards``, ``decode_from_shards`` and ``glue_shards``
(SURVEY.md §8(a) rows a1, a2, a7, a8), reached from the reference at
``src/hydrabadger/state.rs:484`` (propose) and ``state.rs:486-487``
(handle_message).
"""
from __future__ import annotations

import struct

import numpy as np

from . import gf256
from .merkle import MerkleTree


def num_faulty(n: int) -> int:
    """hbbft ``NetworkInfo::num_faulty`` = (N - 1) / 3."""
    return (n - 1) // 3


def shard_counts(n: int) -> tuple[int, int]:
    f = num_faulty(n)
    parity = 2 * f
    return n - parity, parity


def shard_len(payload_len: int, data: int) -> int:
    return (payload_len + 4 + data - 1) // data


class Coding:
    """hbbft ``Coding`` enum: ReedSolomon(D, Q) or Trivial(D)."""

    def __init__(self, data: int, parity: int):
        self.data = data
        self.parity = parity
        self.rs = gf256.ReedSolomon(data, parity) if parity > 0 else None

    def encode(self, shards: np.ndarray) -> None:
        if self.rs is not None:
            self.rs.encode(shards)

    def reconstruct_shards(self, shards: list) -> None:
        if self.rs is not None:
            self.rs.reconstruct(shards)
        elif not all(s is not None for s in shards):
            raise gf256.TooFewShardsPresent()


def make_shards(payload: bytes, n: int) -> np.ndarray:
    """``send_shards`` up to (not including) ``Coding::encode``: 4-byte BE
    length prefix, zero pad to N*L, chunks of L."""
    data, parity = shard_counts(n)
    value = struct.pack(">I", len(payload)) + bytes(payload)
    L = (len(value) + data - 1) // data
    buf = np.zeros(L * n, dtype=np.uint8)
    buf[: len(value)] = np.frombuffer(value, dtype=np.uint8)
    return buf.reshape(n, L)


def send_shards(payload: bytes, n: int):
    """Returns (shards [N][L] uint8, MerkleTree) exactly as ``send_shards``
    builds them before emitting N ``Message::Value(proof(i))``."""
    data, parity = shard_counts(n)
    shards = make_shards(payload, n)
    Coding(data, parity).encode(shards)
    tree = MerkleTree.from_vec([bytes(s) for s in shards])
    return shards, tree


def glue_shards(values: list, data: int):
    """``glue_shards``: first D shards, BE u32 length, take len (truncating)."""
    joined = b"".join(bytes(v) for v in values[:data])
    if len(joined) < 4:
        return None
    ln = struct.unpack(">I", joined[:4])[0]
    return joined[4: 4 + ln]


def decode_from_shards(leaf_values: list, n: int, root_hash: bytes):
    """``decode_from_shards``: reconstruct, rebuild tree, compare root, glue.
    ``leaf_values``: list of Optional[np.ndarray]; modified in place."""
    data, parity = shard_counts(n)
    try:
        Coding(data, parity).reconstruct_shards(leaf_values)
    except (gf256.TooFewShardsPresent, gf256.IncorrectShardSize, gf256.EmptyShard,
            gf256.TooFewShards, gf256.TooManyShards):
        return None
    shards = [bytes(s) for s in leaf_values if s is not None]
    tree = MerkleTree.from_vec(shards)
    if tree.root_hash != root_hash:
        return None
    return glue_shards(tree.values, data)
