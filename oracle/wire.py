"""hbbft broadcast wire format restatement (TEST INFRASTRUCTURE ONLY — see
oracle/__init__.py).

bincode 1.x with its default configuration (the one hydrabadger's
``bincode::serialize`` / ``bincode::deserialize`` use, src/lib.rs:401-403 and
src/lib.rs:436-440): little-endian fixed-width integers, ``usize`` as u64,
sequence lengths as u64, enum variants as a u32 index, fixed arrays as tuples
(no length), trailing bytes after a complete value ignored.  Applied to hbbft
[EXT, VegeBun-csj/hbbft master, unvendored]:

* ``broadcast::Message`` (src/broadcast/message.rs): ``Value(Proof<Vec<u8>>)``
  = 0, ``Echo(Proof<Vec<u8>>)`` = 1, ``Ready(Digest)`` = 2,
  ``CanDecode(Digest)`` = 3, ``EchoHash(Digest)`` = 4;
* ``Proof<T> { value: T, index: usize, digests: Vec<Digest>, root_hash: Digest }``
  (src/broadcast/merkle.rs), ``Digest = [u8; 32]``.

Parity: the bincode encoding rules are the crate's documented format; the
hbbft type definitions (variant order, field order) are restated from
upstream and are "parity unpinned" (no in-container hbbft source or fixture).
"""
from __future__ import annotations

import struct

from . import merkle

VALUE, ECHO, READY, CAN_DECODE, ECHO_HASH = 0, 1, 2, 3, 4

# status codes (mirror include/hbgpu.h)
OK = 0
E_WIRE_EOF = -30
E_WIRE_TAG = -31
E_INCORRECT_SHARD_SIZE = -16


def proof_digests(n: int, index: int) -> int:
    """Digests MerkleTree::proof(index) carries in an n-leaf tree."""
    if index >= n:
        return 0
    k, ln, i = 0, n, index
    while ln > 1:
        if (i ^ 1) < ln:
            k += 1
        i //= 2
        ln = (ln + 1) // 2
    return k


def serialize_proof_msg(tag: int, proof: merkle.Proof) -> bytes:
    """bincode of Message::Value/Echo(proof)."""
    assert tag in (VALUE, ECHO)
    out = struct.pack("<IQ", tag, len(proof.value)) + bytes(proof.value)
    out += struct.pack("<QQ", proof.index, len(proof.digests))
    for d in proof.digests:
        assert len(d) == 32
        out += bytes(d)
    assert len(proof.root_hash) == 32
    return out + bytes(proof.root_hash)


def serialize_digest_msg(tag: int, digest: bytes) -> bytes:
    """bincode of Message::Ready/CanDecode/EchoHash(digest)."""
    assert tag in (READY, CAN_DECODE, ECHO_HASH) and len(digest) == 32
    return struct.pack("<I", tag) + bytes(digest)


def deserialize(msg: bytes):
    """bincode::deserialize::<Message>(msg) -> (status, tag, payload).

    payload is a merkle.Proof for Value/Echo, the 32-byte digest otherwise,
    None on error.  Value-length checks against a batch layout are the
    caller's (the GPU table reports them as E_INCORRECT_SHARD_SIZE)."""
    msg = bytes(msg)
    if len(msg) < 4:
        return E_WIRE_EOF, None, None
    (tag,) = struct.unpack_from("<I", msg, 0)
    if tag > ECHO_HASH:
        return E_WIRE_TAG, tag, None
    if tag >= READY:
        if len(msg) < 36:
            return E_WIRE_EOF, tag, None
        return OK, tag, msg[4:36]
    if len(msg) < 12:
        return E_WIRE_EOF, tag, None
    (vlen,) = struct.unpack_from("<Q", msg, 4)
    p = 12 + vlen
    if p + 16 > len(msg):
        return E_WIRE_EOF, tag, None
    index, k = struct.unpack_from("<QQ", msg, p)
    p += 16
    if p + 32 * k + 32 > len(msg):
        return E_WIRE_EOF, tag, None
    digests = [msg[p + 32 * j: p + 32 * j + 32] for j in range(k)]
    root = msg[p + 32 * k: p + 32 * k + 32]
    return OK, tag, merkle.Proof(msg[12:12 + vlen], index, digests, root)
