"""Regenerates tests/golden/wire_golden.json from the oracle.

    python tests/golden/make_golden_wire.py

hbbft broadcast messages (bincode of ``Message::{Value,Echo}(Proof)`` /
``Ready(Digest)``) for small send_shards trees, plus malformed inputs with the
deserialisation outcome.  The reference (Rust, hbbft unvendored) cannot be
built here and holds no wire fixtures: these are the oracle's outputs
(oracle/wire.py: the bincode 1.x rules over the restated hbbft types), i.e.
"parity unpinned" for the hbbft type layout.
"""
import json
import os
import struct
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from oracle import rbc, synth, wire  # noqa: E402


def main():
    out = {"generator": "tests/golden/make_golden_wire.py", "oracle": "oracle/wire.py + oracle/rbc.py"}
    trees = []
    for N, P in [(1, 9), (4, 230), (5, 33), (7, 100), (16, 300)]:
        inst = 0x57 * N + P
        pl = synth.payload(inst, P)
        shards, tree = rbc.send_shards(pl, N)
        msgs = [wire.serialize_proof_msg(wire.VALUE if i % 2 == 0 else wire.ECHO, tree.proof(i)).hex()
                for i in range(N)]
        trees.append({"N": N, "P": P, "instance": inst, "L": int(shards.shape[1]), "root": tree.root_hash.hex(),
                      "shards_hex": shards.tobytes().hex(), "msgs": msgs,
                      "ready": wire.serialize_digest_msg(wire.READY, tree.root_hash).hex()})
    out["trees"] = trees
    # malformed / edge inputs against the N=7 tree (L from trees[3])
    t = trees[3]
    good = bytes.fromhex(t["msgs"][2])
    L = t["L"]
    bad = {
        "empty": b"",
        "short_tag": good[:3],
        "bad_tag": struct.pack("<I", 5) + good[4:],
        "huge_tag": struct.pack("<I", 0xFFFFFFFF) + good[4:],
        "no_len": good[:8],
        "value_cut": good[:12 + L - 1],
        "no_index": good[:12 + L + 7],
        "digests_cut": good[:-33],
        "root_cut": good[:-1],
        "huge_len": good[:4] + struct.pack("<Q", 1 << 62) + good[12:],
        "huge_k": good[:12 + L + 8] + struct.pack("<Q", 1 << 60) + good[12 + L + 16:],
        "short_value": wire.serialize_proof_msg(wire.VALUE, wire.deserialize(good)[2].__class__(
            good[12:12 + L - 1], 2, wire.deserialize(good)[2].digests, wire.deserialize(good)[2].root_hash)),
        "extra_digest": None,
        "trailing": good + b"\x01\x02\x03",
        "ready_cut": bytes.fromhex(t["ready"])[:35],
        "can_decode": wire.serialize_digest_msg(wire.CAN_DECODE, bytes(range(32))),
        "echo_hash": wire.serialize_digest_msg(wire.ECHO_HASH, bytes(range(32, 64))),
    }
    p = wire.deserialize(good)[2]
    bad["extra_digest"] = wire.serialize_proof_msg(wire.ECHO, p.__class__(p.value, p.index, p.digests + [b"\x07" * 32],
                                                                          p.root_hash))
    cases = []
    for name, b in bad.items():
        st, tag, payload = wire.deserialize(b)
        c = {"name": name, "hex": b.hex(), "status": st, "tag": tag}
        if st == wire.OK and tag is not None and tag <= wire.ECHO:
            c["value_len"] = len(payload.value)
            c["index"] = payload.index
            c["ndigests"] = len(payload.digests)
            c["root"] = payload.root_hash.hex()
            c["validates"] = bool(payload.validate(t["N"]))
        elif st == wire.OK:
            c["digest"] = payload.hex()
        cases.append(c)
    out["malformed"] = {"tree": 3, "cases": cases}
    path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "wire_golden.json")
    with open(path, "w") as f:
        json.dump(out, f, indent=1)
    print(path)


if __name__ == "__main__":
    main()
