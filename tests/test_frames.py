"""SURVEY.md §8(f4) + §8(f2): hydrabadger's signed, length-delimited wire
frames (WireMessages::start_send / poll, /root/reference/src/lib.rs:352-447).

CPU tests pin oracle/wire.py's signed_frame / poll_frame against the committed
fixture tests/golden/frames_golden.json (generator make_golden_frames.py);
GPU tests run hbg_wire_sign_frames / hbg_wire_verify_frames through the C ABI
and must reproduce the fixture's frames byte for byte and its poll outcomes
code for code, then a device-resident batch at bench scale."""
from __future__ import annotations

import json
import os
import struct

import numpy as np
import pytest

from oracle import bls12_381 as B
from oracle import wire

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLD = json.load(open(os.path.join(ROOT, "tests", "golden", "frames_golden.json")))
UNMUTATED = {"message_ok", "keygen_ok", "message_wrong_key", "goodbye_wrong_key_exempt", "network_state_exempt",
             "message_unknown_peer", "bad_kind", "short_message", "empty_message", "message_bad_uid_len",
             "keygen_bad_instance_id", "message_truncated_body"}


def _sks():
    return [int.from_bytes(bytes.fromhex(h), "little") for h in GOLD["sk"]]


# ------------------------------------------------------------------ oracle (CPU)
def test_oracle_matches_fixture():
    pks = [B.g1_decompress(bytes.fromhex(h)) for h in GOLD["pk"]]
    for k, pk in zip(_sks(), pks):
        assert B.g1_mul(B.G1, k) == pk
    for c in GOLD["cases"]:
        f = bytes.fromhex(c["frame"])
        if c["name"] in UNMUTATED:
            assert wire.signed_frame(bytes.fromhex(c["message"]), bytes.fromhex(c["sig"])) == f, c["name"]
        peer = None if c["peer"] is None else pks[c["peer"]]
        assert wire.poll_frame(f, peer) == c["status"], c["name"]


def test_frame_layout():
    m = struct.pack("<I", 7) + b"abc"
    f = wire.signed_frame(m, bytes(96))
    assert len(f) == wire.frame_len(len(m)) == 4 + 8 + 7 + 96
    assert f[:4] == struct.pack(">I", 8 + 7 + 96) and f[4:12] == struct.pack("<Q", 7) and f[12:19] == m


def test_abi_frame_len_and_errors():
    from hydrabadger_amd import _lib
    l = _lib.lib()
    for n in (0, 1, 255, 1 << 20):
        assert l.hbg_wire_frame_len(n) == wire.frame_len(n)
    assert l.hbg_strerror(_lib.HBG_E_INVALID_SIGNATURE) == b"InvalidSignature"
    assert l.hbg_strerror(_lib.HBG_E_UNKNOWN_PEER) == b"VerificationMessageReceivedUnknownPeer"
    assert l.hbg_strerror(_lib.HBG_E_WIRE_VALUE) == b"InvalidValue"


def test_oracle_body_gate():
    """poll deserialises the WireMessage before verifying (src/lib.rs:400-416):
    the fields the reference tree defines for the verified kinds — Message's
    Uid (uuid: u64 length 16 + 16 bytes), KeyGen's InstanceId and
    key_gen::MessageKind (src/hydrabadger/key_gen.rs:18-33) — and the index
    of the hbbft body that follows; unverified kinds: the kind index only."""
    u = struct.pack("<Q", 16) + bytes(range(16))
    P = struct.pack
    assert wire.body_status(P("<I", 7) + u + P("<I", 0)) == wire.OK
    assert wire.body_status(P("<I", 7) + u + b"\0\0\0") == wire.E_WIRE_EOF       # the hbbft index cut short
    assert wire.body_status(P("<I", 7) + P("<Q", 15) + bytes(15) + bytes(8)) == wire.E_WIRE_VALUE
    assert wire.body_status(P("<I", 7) + P("<Q", 17) + bytes(17) + bytes(8)) == wire.E_WIRE_VALUE
    assert wire.body_status(P("<I", 7) + P("<Q", 1 << 40) + bytes(40)) == wire.E_WIRE_EOF  # bytes past the end
    assert wire.body_status(P("<I", 7) + bytes(7)) == wire.E_WIRE_EOF
    assert wire.body_status(P("<II", 9, 0) + P("<I", 1) + bytes(4)) == wire.OK      # BuiltIn, Ack
    assert wire.body_status(P("<II", 9, 1) + u + P("<I", 0) + bytes(4)) == wire.OK  # User(Uid), Part
    assert wire.body_status(P("<II", 9, 2) + bytes(40)) == wire.E_WIRE_TAG          # InstanceId index 2
    assert wire.body_status(P("<II", 9, 0) + P("<I", 2) + bytes(4)) == wire.E_WIRE_TAG  # MessageKind index 2
    assert wire.body_status(P("<II", 9, 0) + P("<I", 1)) == wire.E_WIRE_EOF
    assert wire.body_status(P("<I", 5)) == wire.OK                                   # Goodbye: no fields
    # the gate runs before the signature / peer checks: an unknown peer with a bad body is a Serde error
    f = wire.signed_frame(P("<IQ", 7, 3) + bytes(40), B.g2_compress(B.G2))
    assert wire.poll_frame(f, None) == wire.E_WIRE_VALUE


# ------------------------------------------------------------------ GPU (C ABI)
@pytest.mark.gpu
def test_gpu_sign_frames_match_fixture():
    from hydrabadger_amd import wire as hw
    cases = [c for c in GOLD["cases"] if c["name"] in UNMUTATED]
    frames = hw.sign_frames(_sks(), [(c["signer"], bytes.fromhex(c["message"])) for c in cases])
    for c, f in zip(cases, frames):
        assert f.hex() == c["frame"], c["name"]
        assert hw.message_of(f).hex() == c["message"]


@pytest.mark.gpu
def test_gpu_poll_frames_match_fixture():
    from hydrabadger_amd import wire as hw
    pks = [bytes.fromhex(h) for h in GOLD["pk"]]
    st = hw.poll_frames(pks, [(c["peer"], bytes.fromhex(c["frame"])) for c in GOLD["cases"]])
    assert [int(s) for s in st] == [c["status"] for c in GOLD["cases"]]


@pytest.mark.gpu
def test_gpu_poll_without_keys():
    """No peer keys at all: verified kinds -> unknown peer, exempt kinds pass."""
    from hydrabadger_amd import wire as hw
    cases = [c for c in GOLD["cases"] if c["name"] in ("message_ok", "network_state_exempt")]
    st = hw.poll_frames([], [(None, bytes.fromhex(c["frame"])) for c in cases])
    assert list(st) == [wire.E_UNKNOWN_PEER, 0]


def _torch():
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch


@pytest.mark.gpu
def test_gpu_device_batch_sign_poll():
    """4096 Message-kind frames of 256-B messages from 64 signers on the
    device: all accepted; 41 tampered frames (one byte of the message) are
    exactly the InvalidSignature ones; the signatures equal hbg_bls_sign's;
    two frames are re-checked by the oracle."""
    torch = _torch()
    from hydrabadger_amd import _lib, threshold as th, wire as hw
    from oracle import synth
    dev = torch.device("cuda:0")
    n, ln, n_sk = 4096, 256, 64
    sks = [(0x9E3779B97F4A7C15 * (i + 1)) % B.R for i in range(n_sk)]
    msgs = np.frombuffer(synth.synth_bytes(9, 3, n * ln), np.uint8).copy().reshape(n, ln)
    msgs[:, :4] = np.frombuffer(struct.pack("<I", wire.KIND_MESSAGE), np.uint8)
    msgs[:, 4:12] = np.frombuffer(struct.pack("<Q", 16), np.uint8)  # Message(Uid, ..): a 16-byte uuid
    msg_sk = (np.arange(n) % n_sk).astype(np.uint32)
    moff = np.arange(n + 1, dtype=np.uint64) * ln
    foff = np.arange(n + 1, dtype=np.uint64) * wire.frame_len(ln)
    sk = np.frombuffer(b"".join(th._scalar_bytes(k) for k in sks), np.uint8).copy().reshape(n_sk, 32)
    d = lambda a: torch.from_numpy(a.astype(np.int64) if a.dtype == np.uint64 else a.view(np.int32)
                                   if a.dtype == np.uint32 else a).to(dev)
    frames = torch.zeros(int(foff[-1]) + 16, dtype=torch.uint8, device=dev)
    hw.sign_frames_batch(d(sk), d(msg_sk), d(msgs.reshape(-1)), d(moff), frames, d(foff), device=True)
    torch.cuda.synchronize()
    bad = np.arange(7, n, 100)
    for k in bad:
        frames[int(foff[k]) + 12 + 4 + 24 + (k % 200)] ^= 1  # in the body past kind + Uid: still deserialises
    all_pk = np.frombuffer(b"".join(B.g1_compress(B.g1_mul(B.G1, k)) for k in sks), np.uint8).copy().reshape(n_sk, 48)
    st = torch.empty(n, dtype=torch.int32, device=dev)
    hw.poll_frames_batch(d(all_pk), d(msg_sk), frames, d(foff), st, device=True)
    torch.cuda.synchronize()
    expect = np.zeros(n, np.int32)
    expect[bad] = wire.E_INVALID_SIGNATURE
    assert np.array_equal(st.cpu().numpy(), expect)
    host = frames.cpu().numpy()
    spot = [0, 1, 4095]
    sigs = th.sign_batch(sks, [(int(msg_sk[k]), msgs[k].tobytes()) for k in spot])
    for k, s in zip(spot, sigs):
        f = host[int(foff[k]):int(foff[k + 1])].tobytes()
        assert f[-96:] == s and f[12:12 + ln] == msgs[k].tobytes()
    for k in (0, 7):
        f = host[int(foff[k]):int(foff[k + 1])].tobytes()
        pk = B.g1_mul(B.G1, sks[int(msg_sk[k])])
        assert wire.poll_frame(f, pk) == expect[k]
