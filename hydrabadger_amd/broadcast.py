"""Drop-in mirror of hbbft's broadcast coding surfaces over the gfx950 engine.

Same names, argument meaning and error behaviour as hbbft
``src/broadcast/{broadcast.rs,merkle.rs}`` [EXT, VegeBun-csj/hbbft master]
(SURVEY.md §8(b)), which the reference reaches from
``/root/reference/src/hydrabadger/state.rs:484`` (``dhb.propose`` →
``Broadcast::send_shards``) and ``state.rs:486-487`` (``dhb.handle_message`` →
``Proof::validate`` / ``decode_from_shards``):

  Coding.new(data, parity)           -> rse ReedSolomon::new | Trivial   (a1)
  Coding.encode(shards)              -> rse encode, parity in place      (a3)
  Coding.reconstruct_shards(shards)  -> rse reconstruct                  (a7)
  MerkleTree.from_vec(values)        -> SHA3 leaves + pair tree          (a4)
  MerkleTree.proof(i) / root_hash()  ->                                  (a5)
  Proof.validate(n)                  ->                                  (a6)
  send_shards / decode_from_shards / glue_shards                         (a2, a7, a8)

Every computation runs in libhbgpu.so on the GPU (no CPU fallback).  Batched
forms (``*_batch``) take whole epochs of instances at once; the single-object
forms are n = 1 calls.
"""
from __future__ import annotations

import struct
from dataclasses import dataclass, field

import numpy as np

from . import _lib
from ._lib import HbgError, check, default_context, lib, ptr

# ----------------------------------------------------------------------------- errors
_RSE_NAMES = {
    _lib.HBG_E_TOO_FEW_DATA_SHARDS: "TooFewDataShards",
    _lib.HBG_E_TOO_FEW_PARITY_SHARDS: "TooFewParityShards",
    _lib.HBG_E_TOO_MANY_SHARDS: "TooManyShards",
    _lib.HBG_E_TOO_FEW_SHARDS: "TooFewShards",
    _lib.HBG_E_TOO_FEW_SHARDS_PRESENT: "TooFewShardsPresent",
    _lib.HBG_E_EMPTY_SHARD: "EmptyShard",
    _lib.HBG_E_INCORRECT_SHARD_SIZE: "IncorrectShardSize",
    _lib.HBG_E_SINGULAR_MATRIX: "SingularMatrix",
}


class RseError(HbgError):
    """reed-solomon-erasure ``Error``; ``.kind`` is the variant name."""

    @property
    def kind(self) -> str:
        return _RSE_NAMES.get(self.code, "Unknown")


def _rse_check(rc: int, what: str) -> None:
    if rc == _lib.HBG_OK:
        return
    if rc in _RSE_NAMES:
        raise RseError(rc, what)
    raise HbgError(rc, what)


def num_faulty(n: int) -> int:
    """hbbft ``NetworkInfo::num_faulty`` = (N - 1) / 3."""
    return _lib.num_faulty(n)


def shard_counts(n: int) -> tuple[int, int]:
    """``Broadcast::new``: (data, parity) = (N - 2f, 2f)."""
    p = 2 * num_faulty(n)
    return n - p, p


# ----------------------------------------------------------------------------- Coding
class Coding:
    """hbbft ``Coding``: ``ReedSolomon(D, Q)`` when Q > 0 else ``Trivial(D)``."""

    def __init__(self, data: int, parity: int, ctx: _lib.Context | None = None):
        self.data = data
        self.parity = parity
        self.ctx = ctx
        if parity > 0:
            _rse_check(lib().hbg_coding_matrix(data, parity, None), "Coding::new")

    @classmethod
    def new(cls, data: int, parity: int) -> "Coding":
        return cls(data, parity)

    def data_shard_count(self) -> int:
        return self.data

    def parity_shard_count(self) -> int:
        return self.parity

    def _ctx(self):
        return (self.ctx or default_context()).h

    def encode(self, shards) -> None:
        """``&mut [&mut [u8]]``: a [N][L] uint8 array (in place) or a list of
        equal-length mutable rows (bytearray / uint8 arrays, written back)."""
        if self.parity == 0:
            return
        arr, rows = _as_matrix(shards, self.data + self.parity)
        L = arr.shape[1]
        _rse_check(lib().hbg_rs_encode(self._ctx(), self.data, self.parity, L, ptr(arr), L, 1, 0), "Coding::encode")
        _write_back(arr, rows)

    def encode_batch(self, shards: np.ndarray) -> None:
        """[n][N][L] uint8, parity rows rewritten in place for every instance."""
        n, N, L = shards.shape
        if self.parity == 0:
            return
        if N != self.data + self.parity:
            raise RseError(_lib.HBG_E_TOO_MANY_SHARDS if N > self.data + self.parity else _lib.HBG_E_TOO_FEW_SHARDS)
        _rse_check(lib().hbg_rs_encode(self._ctx(), self.data, self.parity, L, ptr(shards), L, n, 0),
                   "Coding::encode")

    def reconstruct_shards(self, shards: list) -> None:
        """``&mut [Option<Box<[u8]>>]``: list of bytes/arrays or None; None
        slots are filled in place (present shards are kept as received)."""
        total = self.data + self.parity
        if self.parity == 0:
            if all(s is not None for s in shards):
                return
            raise RseError(_lib.HBG_E_TOO_FEW_SHARDS_PRESENT, "Coding::reconstruct_shards")
        if len(shards) != total:
            raise RseError(_lib.HBG_E_TOO_MANY_SHARDS if len(shards) > total else _lib.HBG_E_TOO_FEW_SHARDS)
        present = np.array([s is not None for s in shards], np.uint8)
        sizes = {len(s) for s in shards if s is not None}
        if len(sizes) > 1:
            raise RseError(_lib.HBG_E_INCORRECT_SHARD_SIZE)
        if present.all():
            return
        if present.sum() < self.data:
            raise RseError(_lib.HBG_E_TOO_FEW_SHARDS_PRESENT)
        L = sizes.pop()
        if L == 0:
            raise RseError(_lib.HBG_E_EMPTY_SHARD)
        arr = np.zeros((total, L), np.uint8)
        for i, s in enumerate(shards):
            if s is not None:
                arr[i] = np.frombuffer(bytes(s), np.uint8)
        st = np.zeros(1, np.int32)
        _rse_check(lib().hbg_rs_reconstruct(self._ctx(), self.data, self.parity, L, ptr(arr), L, ptr(present),
                                            ptr(st), 1, 0), "Coding::reconstruct_shards")
        _rse_check(int(st[0]), "Coding::reconstruct_shards")
        for i in range(total):
            if shards[i] is None:
                shards[i] = arr[i].copy()

    def reconstruct_batch(self, shards: np.ndarray, present: np.ndarray) -> np.ndarray:
        """[n][N][L] in place; present [n][N]; returns per-instance status (0 / HBG_E_*)."""
        n, N, L = shards.shape
        st = np.zeros(n, np.int32)
        pr = np.ascontiguousarray(present, dtype=np.uint8)
        _rse_check(lib().hbg_rs_reconstruct(self._ctx(), self.data, self.parity, L, ptr(shards), L, ptr(pr),
                                            ptr(st), n, 0), "Coding::reconstruct_shards")
        return st


def _as_matrix(shards, total: int):
    if isinstance(shards, np.ndarray) and shards.ndim == 2:
        if shards.shape[0] != total:
            raise RseError(_lib.HBG_E_TOO_MANY_SHARDS if shards.shape[0] > total else _lib.HBG_E_TOO_FEW_SHARDS)
        if shards.shape[1] == 0:
            raise RseError(_lib.HBG_E_EMPTY_SHARD)
        if not shards.flags.c_contiguous or shards.dtype != np.uint8:
            raise TypeError("shards must be a C-contiguous uint8 array")
        return shards, None
    rows = list(shards)
    if len(rows) != total:
        raise RseError(_lib.HBG_E_TOO_MANY_SHARDS if len(rows) > total else _lib.HBG_E_TOO_FEW_SHARDS)
    sizes = {len(r) for r in rows}
    if len(sizes) != 1:
        raise RseError(_lib.HBG_E_INCORRECT_SHARD_SIZE)
    if sizes.pop() == 0:
        raise RseError(_lib.HBG_E_EMPTY_SHARD)
    arr = np.stack([np.frombuffer(bytes(r), np.uint8) for r in rows])
    return np.ascontiguousarray(arr), rows


def _write_back(arr: np.ndarray, rows) -> None:
    if rows is None:
        return
    for i, r in enumerate(rows):
        r[:] = arr[i].tobytes() if isinstance(r, bytearray) else arr[i]


# ----------------------------------------------------------------------------- Merkle
@dataclass
class Proof:
    """hbbft ``Proof<T>``: value, index, sibling digests, root hash."""

    value: bytes
    index: int
    digests: list = field(default_factory=list)
    root_hash: bytes = b""

    def validate(self, n: int) -> bool:
        return bool(validate_proofs([self], n)[0])


def validate_proofs(proofs: list, n: int, ctx: _lib.Context | None = None) -> np.ndarray:
    """Batched ``Proof::validate(n)`` for proofs over one tree size; values of
    a batch must share one length (RBC shards of one instance always do)."""
    if not proofs:
        return np.zeros(0, np.uint8)
    L = len(proofs[0].value)
    if any(len(p.value) != L for p in proofs):
        out = np.zeros(len(proofs), np.uint8)
        for ln in sorted({len(p.value) for p in proofs}):
            idx = [k for k, p in enumerate(proofs) if len(p.value) == ln]
            out[idx] = validate_proofs([proofs[k] for k in idx], n, ctx)
        return out
    depth = _lib.merkle_depth(n)
    m = len(proofs)
    S = max(L, 1)
    vals = np.zeros((m, S), np.uint8)
    index = np.zeros(m, np.uint32)
    nd = np.zeros(m, np.uint32)
    dig = np.zeros((m, max(depth, 1), 32), np.uint8)
    roots = np.zeros((m, 32), np.uint8)
    ok = np.zeros(m, np.uint8)
    for k, p in enumerate(proofs):
        if L:
            vals[k] = np.frombuffer(bytes(p.value), np.uint8)
        index[k] = p.index
        ds = list(p.digests)
        if len(ds) > depth:  # more digests than any valid proof carries: hbbft returns false
            nd[k] = 0xFFFFFFFF
            ds = ds[:depth]
        else:
            nd[k] = len(ds)
        for j, d in enumerate(ds):
            dig[k, j] = np.frombuffer(bytes(d), np.uint8)
        roots[k] = np.frombuffer(bytes(p.root_hash), np.uint8) if len(p.root_hash) == 32 else 0
    h = (ctx or default_context()).h
    check(lib().hbg_merkle_validate(h, n, L, ptr(vals), S, ptr(index), ptr(dig), ptr(nd), ptr(roots), ptr(ok), m, 0),
          "Proof::validate")
    for k, p in enumerate(proofs):
        if len(p.root_hash) != 32:
            ok[k] = 0
    return ok


class MerkleTree:
    """hbbft ``MerkleTree<T>`` built on the GPU (``levels`` + root)."""

    def __init__(self, values: list, levels: np.ndarray):
        self._values = values
        self._flat = levels  # [nodes][32]
        n = len(values)
        self._level_start = []
        off, cnt = 0, n
        while cnt > 1:
            self._level_start.append((off, cnt))
            off += cnt
            cnt = (cnt + 1) // 2

    @classmethod
    def from_vec(cls, values: list, ctx: _lib.Context | None = None) -> "MerkleTree":
        n = len(values)
        if n == 0:
            raise ValueError("MerkleTree over zero values is not on the RBC path")
        L = len(values[0])
        if any(len(v) != L for v in values):
            raise ValueError("RBC shards of one tree must share one length")
        S = max(L, 1)
        arr = np.zeros((n, S), np.uint8)
        for i, v in enumerate(values):
            if L:
                arr[i] = np.frombuffer(bytes(v), np.uint8)
        levels = np.zeros((_lib.merkle_nodes(n), 32), np.uint8)
        h = (ctx or default_context()).h
        check(lib().hbg_merkle_build(h, n, L, ptr(arr), S, ptr(levels), 1, 0), "MerkleTree::from_vec")
        return cls([bytes(v) for v in values], levels)

    def root_hash(self) -> bytes:
        return self._flat[-1].tobytes()

    def values(self) -> list:
        return self._values

    def into_values(self) -> list:
        return self._values

    def levels(self) -> list:
        return [[self._flat[off + i].tobytes() for i in range(cnt)] for off, cnt in self._level_start]

    def proof(self, index: int):
        if index >= len(self._values):
            return None
        lvl_i = index
        digests = []
        for off, cnt in self._level_start:
            if (lvl_i ^ 1) < cnt:
                digests.append(self._flat[off + (lvl_i ^ 1)].tobytes())
            lvl_i //= 2
        return Proof(self._values[index], index, digests, self.root_hash())


# ----------------------------------------------------------------------------- Broadcast glue
def send_shards(value: bytes, n: int, ctx: _lib.Context | None = None):
    """``Broadcast::send_shards`` up to the N ``Message::Value(proof(i))``:
    returns (shards [N][L] uint8, MerkleTree)."""
    P = len(value)
    L = _lib.shard_len(n, P)
    pay = np.frombuffer(bytes(value), np.uint8).copy() if P else np.zeros(1, np.uint8)
    plen = np.array([P], np.uint64)
    shards = np.zeros((n, L), np.uint8)
    levels = np.zeros((_lib.merkle_nodes(n), 32), np.uint8)
    h = (ctx or default_context()).h
    check(lib().hbg_rbc_encode_merkle(h, n, ptr(pay), max(P, 1), ptr(plen), L, ptr(shards), L, ptr(levels), 1, 0),
          "send_shards")
    return shards, MerkleTree([s.tobytes() for s in shards], levels)


def glue_shards(values: list, data: int):
    """``glue_shards`` (pure byte glue; used by callers holding a tree)."""
    joined = b"".join(bytes(v) for v in values[:data])
    if len(joined) < 4:
        return None
    ln = struct.unpack(">I", joined[:4])[0]
    return joined[4: 4 + ln]


def decode_from_shards(leaf_values: list, coding: Coding, data_shard_num: int, root_hash: bytes,
                       ctx: _lib.Context | None = None):
    """``decode_from_shards``: reconstruct, rebuild the tree over all N shards,
    compare roots, glue.  Returns the payload bytes or None.  ``leaf_values`` is
    a list of Optional shards and is filled in place like the Rust slice."""
    n = len(leaf_values)
    present = [v for v in leaf_values if v is not None]
    if not present:
        return None
    L = len(present[0])
    if any(len(v) != L for v in present) or L == 0:
        return None
    arr = np.zeros((n, L), np.uint8)
    pres = np.zeros(n, np.uint8)
    for i, v in enumerate(leaf_values):
        if v is not None:
            arr[i] = np.frombuffer(bytes(v), np.uint8)
            pres[i] = 1
    root = np.frombuffer(bytes(root_hash), np.uint8).copy() if len(root_hash) == 32 else np.zeros(32, np.uint8)
    D = coding.data_shard_count()
    out = np.zeros(max(D * L, 4), np.uint8)
    plen = np.zeros(1, np.uint64)
    st = np.zeros(1, np.uint8)
    h = (ctx or default_context()).h
    check(lib().hbg_rbc_decode(h, n, L, ptr(arr), L, ptr(pres), ptr(root), ptr(out), out.shape[0], ptr(plen), ptr(st),
                               1, 0), "decode_from_shards")
    if coding.parity_shard_count() > 0 and pres.sum() >= D:
        for i in range(n):
            if leaf_values[i] is None:
                leaf_values[i] = arr[i].copy()
    if st[0] != _lib.HBG_DECODE_OK or len(root_hash) != 32:
        return None
    return out[: int(plen[0])].tobytes()


# ----------------------------------------------------------------------------- batched (engine) API
def rbc_encode_merkle_batch(n_nodes: int, payloads, payload_len, shard_len: int, shards, levels,
                            ctx: _lib.Context | None = None, device: bool = False, asynchronous: bool = False) -> None:
    """Whole-batch ``send_shards``.  Host numpy arrays, or (device=True) torch
    CUDA tensors: payloads [n][PS] u8, payload_len [n] u64 (int64 tensor),
    shards [n][N][S] u8, levels [n][nodes][32] u8."""
    n = payloads.shape[0]
    flags = (_lib.HBG_DEVICE if device else 0) | (_lib.HBG_ASYNC if asynchronous else 0)
    h = (ctx or default_context()).h
    check(lib().hbg_rbc_encode_merkle(h, n_nodes, ptr(payloads), payloads.shape[1], ptr(payload_len), shard_len,
                                      ptr(shards), shards.shape[-1], ptr(levels), n, flags), "rbc_encode_merkle")


def rbc_decode_batch(n_nodes: int, shard_len: int, shards, present, roots, payload_out, payload_len, status,
                     ctx: _lib.Context | None = None, device: bool = False, asynchronous: bool = False) -> None:
    n = shards.shape[0]
    flags = (_lib.HBG_DEVICE if device else 0) | (_lib.HBG_ASYNC if asynchronous else 0)
    h = (ctx or default_context()).h
    check(lib().hbg_rbc_decode(h, n_nodes, shard_len, ptr(shards), shards.shape[-1], ptr(present), ptr(roots),
                               ptr(payload_out), payload_out.shape[-1], ptr(payload_len), ptr(status), n, flags),
          "rbc_decode")


def merkle_build_batch(n_nodes: int, shard_len: int, shards, levels, ctx: _lib.Context | None = None,
                       device: bool = False, asynchronous: bool = False) -> None:
    n = shards.shape[0]
    flags = (_lib.HBG_DEVICE if device else 0) | (_lib.HBG_ASYNC if asynchronous else 0)
    h = (ctx or default_context()).h
    check(lib().hbg_merkle_build(h, n_nodes, shard_len, ptr(shards), shards.shape[-1], ptr(levels), n, flags),
          "merkle_build")


def synth_bytes(tag: int, first_instance: int, nbytes: int, out, ctx: _lib.Context | None = None,
                device: bool = False, asynchronous: bool = False) -> None:
    n = out.shape[0]
    flags = (_lib.HBG_DEVICE if device else 0) | (_lib.HBG_ASYNC if asynchronous else 0)
    h = (ctx or default_context()).h
    check(lib().hbg_synth_bytes(h, tag, first_instance, nbytes, ptr(out), out.shape[-1], n, flags), "synth_bytes")


# ----------------------------------------------------------------------------- wire format
@dataclass
class Message:
    """hbbft ``broadcast::Message``: ``kind`` is the bincode variant index
    (VALUE/ECHO carry a ``Proof``, READY/CAN_DECODE/ECHO_HASH a digest)."""

    VALUE, ECHO, READY, CAN_DECODE, ECHO_HASH = (_lib.HBG_MSG_VALUE, _lib.HBG_MSG_ECHO, _lib.HBG_MSG_READY,
                                                 _lib.HBG_MSG_CAN_DECODE, _lib.HBG_MSG_ECHO_HASH)
    kind: int
    payload: object  # Proof or 32-byte digest

    @classmethod
    def value(cls, proof: Proof) -> "Message":
        return cls(cls.VALUE, proof)

    @classmethod
    def echo(cls, proof: Proof) -> "Message":
        return cls(cls.ECHO, proof)

    @classmethod
    def ready(cls, digest: bytes) -> "Message":
        return cls(cls.READY, bytes(digest))


class WireError(HbgError):
    """bincode::Error of a broadcast message (UnexpectedEof / InvalidVariant)."""


def proof_msg_len(n: int, index: int, shard_len: int) -> int:
    return int(lib().hbg_proof_msg_len(n, index, shard_len))


def proof_msg_offsets(n: int, shard_len: int, index) -> np.ndarray:
    """out_off [m+1] (u64) for Value/Echo messages of leaves ``index`` laid end to end."""
    index = np.asarray(index, np.int64)
    lens = np.array([proof_msg_len(n, int(i), shard_len) for i in range(n)], np.uint64)
    off = np.zeros(index.shape[0] + 1, np.uint64)
    off[1:] = np.cumsum(lens[index])
    return off


def write_proof_msgs_batch(n_nodes: int, shard_len: int, shards, levels, tag: int, inst, index, out, out_off,
                           ctx: _lib.Context | None = None, device: bool = False, asynchronous: bool = False) -> None:
    """bincode ``Message::{Value,Echo}(tree[inst[j]].proof(index[j]))`` for
    every j, into out[out_off[j]:out_off[j+1]].  shards [n][N][S], levels
    [n][nodes][32] as produced by ``rbc_encode_merkle_batch``; inst u64/int64,
    index u32/int32, out_off u64/int64 [m+1]."""
    flags = (_lib.HBG_DEVICE if device else 0) | (_lib.HBG_ASYNC if asynchronous else 0)
    h = (ctx or default_context()).h
    check(lib().hbg_rbc_write_proof_msgs(h, n_nodes, shard_len, ptr(shards), shards.shape[-1], ptr(levels),
                                         shards.shape[0], tag, inst.shape[0], ptr(inst), ptr(index), ptr(out),
                                         ptr(out_off), flags), "write_proof_msgs")


def read_msgs_batch(n_nodes: int, shard_len: int, msgs, msg_off, tag, values, index, digests, ndigests, roots,
                    status, ctx: _lib.Context | None = None, device: bool = False,
                    asynchronous: bool = False) -> None:
    """``bincode::deserialize::<Message>`` of m messages (msgs[msg_off[j]:
    msg_off[j+1]]) into the ``validate_proofs`` table: tag/index/ndigests u32
    [m], values [m][S], digests [m][depth][32], roots [m][32], status i32 [m]."""
    m = msg_off.shape[0] - 1
    flags = (_lib.HBG_DEVICE if device else 0) | (_lib.HBG_ASYNC if asynchronous else 0)
    h = (ctx or default_context()).h
    check(lib().hbg_rbc_read_msgs(h, n_nodes, shard_len, ptr(msgs), ptr(msg_off), m, ptr(tag), ptr(values),
                                  values.shape[-1], ptr(index), ptr(digests), ptr(ndigests), ptr(roots), ptr(status),
                                  flags), "read_msgs")


def serialize_proof_messages(tree: MerkleTree, tag: int, indices=None, ctx: _lib.Context | None = None) -> list:
    """bincode of ``Message::Value/Echo(tree.proof(i))`` for each i (what
    ``Broadcast::send_shards`` hands to the transport), built on the GPU."""
    vals = tree.values()
    n = len(vals)
    L = len(vals[0])
    idx = np.arange(n, dtype=np.uint32) if indices is None else np.asarray(indices, np.uint32)
    shards = np.zeros((1, n, max(L, 1)), np.uint8)
    for i, v in enumerate(vals):
        if L:
            shards[0, i] = np.frombuffer(bytes(v), np.uint8)
    levels = tree._flat.reshape(1, -1, 32)
    off = proof_msg_offsets(n, L, idx)
    out = np.zeros(max(int(off[-1]), 1), np.uint8)
    inst = np.zeros(idx.shape[0], np.uint64)
    write_proof_msgs_batch(n, L, shards, levels, tag, inst, idx, out, off, ctx)
    return [out[int(off[j]):int(off[j + 1])].tobytes() for j in range(idx.shape[0])]


def deserialize_messages(msgs: list, n: int, shard_len: int, ctx: _lib.Context | None = None) -> list:
    """``bincode::deserialize::<Message>`` for each wire message of an n-node
    broadcast with shards of shard_len bytes, on the GPU.  Returns a Message,
    or raises-equivalent WireError objects in place of failed items (so a
    batch keeps its order); a proof whose value is not shard_len bytes is
    returned as WireError(HBG_E_INCORRECT_SHARD_SIZE)."""
    m = len(msgs)
    depth = max(_lib.merkle_depth(n), 1)
    off = np.zeros(m + 1, np.uint64)
    off[1:] = np.cumsum([len(b) for b in msgs]) if m else []
    buf = np.frombuffer(b"".join(bytes(b) for b in msgs) or b"\0", np.uint8).copy()
    S = max(shard_len, 1)
    tag = np.zeros(m, np.uint32)
    vals = np.zeros((m, S), np.uint8)
    index = np.zeros(m, np.uint32)
    dig = np.zeros((m, depth, 32), np.uint8)
    nd = np.zeros(m, np.uint32)
    roots = np.zeros((m, 32), np.uint8)
    st = np.zeros(m, np.int32)
    read_msgs_batch(n, shard_len, buf, off, tag, vals, index, dig, nd, roots, st, ctx)
    res = []
    for j in range(m):
        if st[j] != 0:
            res.append(WireError(int(st[j]), "bincode::deserialize"))
        elif tag[j] >= Message.READY:
            res.append(Message(int(tag[j]), roots[j].tobytes()))
        else:
            k = int(nd[j])
            if k == 0xFFFFFFFF:  # more digests than an n-leaf proof has: carried as an unvalidatable marker
                ds = [b"\0" * 32] * (_lib.merkle_depth(n) + 1)
            else:
                ds = [dig[j, q].tobytes() for q in range(k)]
            res.append(Message(int(tag[j]), Proof(vals[j, :shard_len].tobytes(), int(index[j]), ds,
                                                  roots[j].tobytes())))
    return res
