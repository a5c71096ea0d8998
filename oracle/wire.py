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


# ----------------------------------------------------------------------------- signed frames
# hydrabadger's own framing (in the reference: src/lib.rs:352-447):
# WireMessages::start_send = bincode(SignedWireMessage { message, sig }) in a
# tokio LengthDelimitedCodec frame (default: 4-byte big-endian length);
# WireMessages::poll verifies the signature only for WireMessageKind::Message
# (variant 7) and ::KeyGen (9) of the 11 variants at src/lib.rs:250-270.
# Signature serialises as its 96-byte compressed G2 point, a serde tuple
# (threshold_crypto serde_impl::projective) — no length; parity unpinned.
KIND_MESSAGE, KIND_KEYGEN, KIND_MAX = 7, 9, 10
# LengthDelimitedCodec::new() (tokio-io 0.1, src/lib.rs:369): default
# max_frame_length 8 MiB; a longer frame is an error on read and on write.
MAX_FRAME = 8 * 1024 * 1024
E_WIRE_FRAME = -32
E_INVALID_SIGNATURE = -33
E_UNKNOWN_PEER = -34
E_WIRE_VALUE = -35
E_INVALID_POINT = -22
INSTANCE_BUILTIN, INSTANCE_USER = 0, 1   # key_gen::InstanceId (src/hydrabadger/key_gen.rs:18-21)
KEYGEN_PART, KEYGEN_ACK = 0, 1           # key_gen::MessageKind (src/hydrabadger/key_gen.rs:25-28)


def _uid(m: bytes, p: int):
    """serde of hydrabadger's Uid(Uuid) (src/lib.rs:149; uuid 0.6, non-human-
    readable: serialize_bytes) under bincode: u64 length, the bytes; the uuid
    visitor rejects a length != 16 (after bincode has read the bytes)."""
    if len(m) < p + 8:
        return E_WIRE_EOF, p
    (n,) = struct.unpack_from("<Q", m, p)
    p += 8
    if n > len(m) - p:
        return E_WIRE_EOF, p
    if n != 16:
        return E_WIRE_VALUE, p
    return OK, p + 16


def body_status(message: bytes) -> int:
    """bincode::deserialize::<WireMessage>(message) (src/lib.rs:402-403) for the
    two verified kinds, as far as the reference tree defines their fields:
    Message(Uid, DhbMessage) — the Uid, then the (unvendored) hbbft message's
    u32 variant index must be present; KeyGen(InstanceId, key_gen::Message) —
    InstanceId (BuiltIn | User(Uid)), then MessageKind (Part | Ack) and the
    4 bytes of the first field of Part / Ack.  Unverified kinds: the index only."""
    m = bytes(message)
    (kind,) = struct.unpack_from("<I", m, 0)
    p = 4
    if kind == KIND_MESSAGE:
        st, p = _uid(m, p)
        if st:
            return st
        return OK if len(m) >= p + 4 else E_WIRE_EOF
    if kind == KIND_KEYGEN:
        if len(m) < p + 4:
            return E_WIRE_EOF
        (inst,) = struct.unpack_from("<I", m, p)
        p += 4
        if inst > INSTANCE_USER:
            return E_WIRE_TAG
        if inst == INSTANCE_USER:
            st, p = _uid(m, p)
            if st:
                return st
        if len(m) < p + 4:
            return E_WIRE_EOF
        (mk,) = struct.unpack_from("<I", m, p)
        if mk > KEYGEN_ACK:
            return E_WIRE_TAG
        return OK if len(m) >= p + 8 else E_WIRE_EOF
    return OK


def frame_len(msg_len: int) -> int:
    return 4 + 8 + msg_len + 96


def signed_frame(message: bytes, sig96: bytes) -> bytes:
    """One codec frame of SignedWireMessage { message, sig }."""
    body = struct.pack("<Q", len(message)) + bytes(message) + bytes(sig96)
    return struct.pack(">I", len(body)) + body


def poll_frame(frame: bytes, peer_pk=None) -> int:
    """WireMessages::poll outcome for one received frame: 0 or an E_* code.
    peer_pk: G1 point (oracle form) or None (unknown peer)."""
    from . import bls12_381 as B
    from . import tcrypto as T
    frame = bytes(frame)
    if len(frame) < 4:
        return E_WIRE_EOF
    head = struct.unpack_from(">I", frame, 0)[0]
    if head > MAX_FRAME or head != len(frame) - 4:  # codec: frame too big / not one whole frame
        return E_WIRE_FRAME
    if len(frame) < 12:
        return E_WIRE_EOF
    (mlen,) = struct.unpack_from("<Q", frame, 4)
    if mlen > len(frame) - 12 or len(frame) - 12 - mlen < 96:
        return E_WIRE_EOF
    message = frame[12:12 + mlen]
    try:
        sig = B.g2_decompress(frame[12 + mlen:12 + mlen + 96])
    except ValueError:
        return E_INVALID_POINT
    if mlen < 4:
        return E_WIRE_EOF
    (kind,) = struct.unpack_from("<I", message, 0)
    if kind > KIND_MAX:
        return E_WIRE_TAG
    st = body_status(message)  # poll deserialises the whole WireMessage before verifying
    if st:
        return st
    if kind in (KIND_MESSAGE, KIND_KEYGEN):
        if peer_pk is None:
            return E_UNKNOWN_PEER
        if not T.verify(peer_pk, sig, message):
            return E_INVALID_SIGNATURE
    return OK
