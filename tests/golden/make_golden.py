"""Regenerates tests/golden/rbc_golden.json from the oracle (numpy restatement).

    python tests/golden/make_golden.py

The reference (Rust, hbbft unvendored) cannot be built or imported here and
ships no fixtures for this path; these vectors are the
oracle's own outputs, pinned by the Backblaze RS known answer and FIPS-202, and
are what the GPU tests and later rounds compare against.
"""
import hashlib
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from oracle import gf256, rbc, synth  # noqa: E402


def main():
    out = {"generator": "tests/golden/make_golden.py", "oracle": "oracle/gf256.py + oracle/merkle.py + oracle/rbc.py"}
    sh = np.zeros((10, 2), np.uint8)
    sh[:5] = [[0, 1], [4, 5], [2, 3], [6, 7], [8, 9]]
    gf256.ReedSolomon(5, 5).encode(sh)
    out["backblaze"] = {"data": sh[:5].tolist(), "parity": sh[5:].tolist()}
    cases = []
    for N, P in [(1, 10), (2, 0), (3, 7), (4, 230), (4, 0), (5, 33), (7, 100), (16, 1000), (16, 65536),
                 (64, 5000), (64, 1 << 20), (128, 3000)]:
        inst = N * 100003 + P
        pl = synth.payload(inst, P)
        shards, tree = rbc.send_shards(pl, N)
        c = {"N": N, "P": P, "instance": inst, "L": int(shards.shape[1]),
             "payload_sha3": hashlib.sha3_256(pl).hexdigest(),
             "shards_sha3": hashlib.sha3_256(shards.tobytes()).hexdigest(),
             "root": tree.root_hash.hex(), "proof_index": N // 2,
             "proof_digests": [d.hex() for d in tree.proof(N // 2).digests]}
        if shards.size <= 2048:
            c["shards_hex"] = shards.tobytes().hex()
        cases.append(c)
    out["send_shards"] = cases
    mats = []
    for D, Q in [(2, 2), (6, 10), (22, 42), (44, 84)]:
        m = np.array(gf256.build_matrix(D, Q), np.uint8)
        mats.append({"D": D, "Q": Q, "sha3": hashlib.sha3_256(m.tobytes()).hexdigest(),
                     "first_parity_rows": m[D:D + 2].tolist()})
    out["matrices"] = mats
    with open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "rbc_golden.json"), "w") as f:
        json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
