"""Drop-in mirror of hydrabadger's signed, length-delimited wire frames over
the gfx950 engine (SURVEY.md §8(f4) with §8(f2)'s signatures).

The reference (in-tree: /root/reference/src/lib.rs:352-447) wraps every
serialised ``WireMessage`` as ``bincode(SignedWireMessage { message, sig })``
in a tokio ``LengthDelimitedCodec`` frame (4-byte big-endian length):

  WireMessages::start_send(msg)  -> sign_frames / sign_frames_batch
  WireMessages::poll()           -> poll_frames  / poll_frames_batch

``poll`` verifies the signature only for ``WireMessageKind::Message`` (7) and
``::KeyGen`` (9) and fails with ``InvalidSignature`` /
``VerificationMessageReceivedUnknownPeer``; deserialisation failures are
``Serde`` errors (here ``UnexpectedEof`` / ``InvalidVariant`` / ``InvalidPoint``
status codes).  Everything runs in libhbgpu.so on the GPU; no CPU fallback.
"""
from __future__ import annotations

import numpy as np

from . import _lib
from ._lib import HbgError, check, default_context, lib, ptr
from .threshold import _scalar_bytes

KIND_MESSAGE, KIND_KEYGEN = _lib.HBG_WIRE_KIND_MESSAGE, _lib.HBG_WIRE_KIND_KEYGEN
UNKNOWN_PEER = 0xFFFFFFFF


class WireError(HbgError):
    """hydrabadger::Error of a received frame (InvalidSignature, Serde, …)."""


def frame_len(msg_len: int) -> int:
    return int(lib().hbg_wire_frame_len(msg_len))


def _offsets(lens) -> np.ndarray:
    off = np.zeros(len(lens) + 1, np.uint64)
    if len(lens):
        off[1:] = np.cumsum(np.asarray(lens, np.uint64))
    return off


def sign_frames_batch(sk32, msg_sk, msg, msg_off, frames, frame_off, ctx: _lib.Context | None = None,
                      device: bool = False, asynchronous: bool = False) -> None:
    """Batched WireMessages::start_send: sk32 [n_sk][32] LE scalars, msg_sk
    [n] u32, messages at msg_off [n+1], frames at frame_off [n+1] (each
    frame_len(len) bytes).  Host numpy arrays or (device=True) CUDA tensors."""
    n = msg_off.shape[0] - 1
    flags = (_lib.HBG_DEVICE if device else 0) | (_lib.HBG_ASYNC if asynchronous else 0)
    check(lib().hbg_wire_sign_frames((ctx or default_context()).h, sk32.shape[0], ptr(sk32), n, ptr(msg_sk),
                                     ptr(msg), ptr(msg_off), ptr(frames), ptr(frame_off), flags),
          "WireMessages::start_send")


def poll_frames_batch(pk48, frame_pk, frames, frame_off, status, ctx: _lib.Context | None = None,
                      device: bool = False, asynchronous: bool = False) -> None:
    """Batched WireMessages::poll: pk48 [n_pk][48], frame_pk [n] u32 (>= n_pk:
    unknown peer), frames at frame_off [n+1]; status [n] i32."""
    n = frame_off.shape[0] - 1
    flags = (_lib.HBG_DEVICE if device else 0) | (_lib.HBG_ASYNC if asynchronous else 0)
    check(lib().hbg_wire_verify_frames((ctx or default_context()).h, pk48.shape[0], ptr(pk48), n, ptr(frame_pk),
                                       ptr(frames), ptr(frame_off), ptr(status), flags), "WireMessages::poll")


def sign_frames(sks: list, items: list, ctx: _lib.Context | None = None) -> list:
    """items = [(sk index, serialised WireMessage)] -> codec frames (bytes)."""
    n = len(items)
    if n == 0:
        return []
    msgs = [bytes(m) for _, m in items]
    moff = _offsets([len(m) for m in msgs])
    foff = _offsets([frame_len(len(m)) for m in msgs])
    buf = np.frombuffer(b"".join(msgs) or b"\0", np.uint8).copy()
    sk = np.frombuffer(b"".join(_scalar_bytes(x) for x in sks), np.uint8).copy().reshape(len(sks), 32)
    ix = np.array([i for i, _ in items], np.uint32)
    out = np.zeros(int(foff[-1]), np.uint8)
    sign_frames_batch(sk, ix, buf, moff, out, foff, ctx)
    return [out[int(foff[k]):int(foff[k + 1])].tobytes() for k in range(n)]


def poll_frames(pk48s: list, items: list, ctx: _lib.Context | None = None) -> np.ndarray:
    """items = [(peer pk index or None, frame bytes)] -> status per frame
    (0: the WireMessage is accepted; else a negative HBG_E_* code)."""
    n = len(items)
    if n == 0:
        return np.zeros(0, np.int32)
    frames = [bytes(f) for _, f in items]
    foff = _offsets([len(f) for f in frames])
    buf = np.frombuffer(b"".join(frames) or b"\0", np.uint8).copy()
    pk = np.frombuffer(b"".join(bytes(p) for p in pk48s) or b"\0" * 48, np.uint8).copy().reshape(-1, 48)
    if not pk48s:
        pk = pk[:0]
    ix = np.array([UNKNOWN_PEER if p is None else p for p, _ in items], np.uint32)
    st = np.zeros(n, np.int32)
    poll_frames_batch(pk, ix, buf, foff, st, ctx)
    return st


def message_of(frame: bytes) -> bytes:
    """The serialised WireMessage inside an accepted frame."""
    ln = int.from_bytes(frame[4:12], "little")
    return bytes(frame[12:12 + ln])
