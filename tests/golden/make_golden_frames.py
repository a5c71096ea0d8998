"""Regenerates tests/golden/frames_golden.json (SURVEY.md §8(f4) + §8(f2)):
hydrabadger's signed, length-delimited frames (src/lib.rs:352-447) from the
oracle (oracle/wire.py signed_frame / poll_frame, oracle/tcrypto.py sign).

    python tests/golden/make_golden_frames.py

Messages are bincode WireMessages: the u32 WireMessageKind variant (7 =
Message, 9 = KeyGen are verified; the others are not), then for Message the
Uid (u64 length 16 + 16 bytes) and for KeyGen the InstanceId (User(Uid)) and
key_gen::MessageKind (Part / Ack); the rest of each body (the unvendored hbbft
types) is synthetic.  poll deserialises the WireMessage before verifying
(src/lib.rs:400-416): two cases have a body that does not deserialise under a
valid signature.  Each case records the sender key index (None = unknown peer)
and the oracle's poll outcome.
"""
import json
import os
import struct
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from oracle import bls12_381 as B  # noqa: E402
from oracle import synth, tcrypto as T, wire  # noqa: E402


def le(x: int) -> str:
    return x.to_bytes(32, "little").hex()


def main():
    sks = [0x1234567890ABCDEF1122334455667788 % B.R, (7 << 200) + 12345]
    pks = [B.g1_mul(B.G1, k) for k in sks]
    def uid(seed):
        return struct.pack("<Q", 16) + synth.synth_bytes(6, seed, 16)

    def msg(kind, n, seed):
        body = synth.synth_bytes(5, seed, n)
        if kind == wire.KIND_MESSAGE:  # Message(Uid, hbbft DHB message)
            return struct.pack("<I", kind) + uid(seed) + body
        if kind == wire.KIND_KEYGEN:  # KeyGen(InstanceId::User(Uid), key_gen::Message { kind: Part(..) })
            return struct.pack("<II", kind, wire.INSTANCE_USER) + uid(seed) + struct.pack("<I", wire.KEYGEN_PART) + body
        return struct.pack("<I", kind) + body
    items = []  # (name, message, signer key for the sig, claimed peer (None = unknown), frame mutator)
    items.append(("message_ok", msg(7, 120, 1), 0, 0, None))
    items.append(("keygen_ok", msg(9, 40, 2), 1, 1, None))
    items.append(("message_wrong_key", msg(7, 64, 3), 1, 0, None))
    items.append(("goodbye_wrong_key_exempt", msg(5, 0, 4), 1, 0, None))
    items.append(("network_state_exempt", msg(4, 300, 5), 0, None, None))
    items.append(("message_unknown_peer", msg(7, 10, 6), 0, None, None))
    items.append(("bad_kind", msg(11, 10, 7), 0, 0, None))
    items.append(("short_message", b"\x07\x00", 0, 0, None))
    items.append(("empty_message", b"", 0, 0, None))
    items.append(("bad_prefix", msg(7, 20, 8), 0, 0, "prefix"))
    items.append(("truncated_sig", msg(7, 20, 9), 0, 0, "truncate"))
    items.append(("bad_sig_point", msg(7, 20, 10), 0, 0, "sigpoint"))
    items.append(("tampered_message", msg(7, 50, 11), 0, 0, "tamper"))
    items.append(("trailing_bytes", msg(9, 33, 12), 0, 0, "trailing"))
    # validly signed by the peer's key, but the WireMessage does not deserialise: Error::Serde before verify
    items.append(("message_bad_uid_len", struct.pack("<IQ", 7, 17) + synth.synth_bytes(6, 13, 17)
                  + synth.synth_bytes(5, 13, 40), 0, 0, None))
    items.append(("keygen_bad_instance_id", struct.pack("<II", 9, 2) + synth.synth_bytes(5, 14, 40), 1, 1, None))
    items.append(("message_truncated_body", struct.pack("<I", 7) + uid(15) + b"\x00\x00", 0, 0, None))
    cases = []
    for name, m, signer, peer, mut in items:
        sig = B.g2_compress(T.sign(sks[signer], m))
        f = bytearray(wire.signed_frame(m, sig))
        if mut == "prefix":
            f[3] ^= 1
        elif mut == "truncate":
            f = f[:-1]
            f[0:4] = struct.pack(">I", len(f) - 4)
        elif mut == "sigpoint":
            f[-96:] = b"\x80" + b"\xff" * 95  # x >= p: not a field element
        elif mut == "tamper":
            f[12 + 4 + 24 + 5] ^= 0x40  # inside the hbbft body (past kind + Uid): still deserialises
        elif mut == "trailing":
            body = bytes(f[4:]) + b"\x00\x01"
            f = bytearray(struct.pack(">I", len(body)) + body)
        st = wire.poll_frame(bytes(f), None if peer is None else pks[peer])
        cases.append({"name": name, "frame": bytes(f).hex(), "peer": peer, "signer": signer, "message": m.hex(),
                      "sig": sig.hex(), "status": st})
        print(name, st, flush=True)
    out = {"generator": "tests/golden/make_golden_frames.py", "oracle": "oracle/wire.py + oracle/tcrypto.py",
           "sk": [le(k) for k in sks], "pk": [B.g1_compress(p).hex() for p in pks], "cases": cases}
    path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "frames_golden.json")
    with open(path, "w") as fo:
        json.dump(out, fo, indent=1)
    print(path)


if __name__ == "__main__":
    main()
