"""Regenerates tests/golden/tdec_golden.json from the oracle (BLS12-381 /
threshold_crypto restatement).  python tests/golden/make_golden_tdec.py

No reference fixtures exist for this path; these pin the
oracle's own outputs so later rounds (and a future Rust-side check against the
real crates) compare against fixed bytes."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from oracle import bls12_381 as B  # noqa: E402
from oracle import tcrypto as T  # noqa: E402
from tests.tdec_fixtures import scenario  # noqa: E402


def scenario_json(params):
    s = scenario(**params)
    return {
        "params": params, "t": s["t"],
        "pk_shares": [B.g1_compress(p).hex() for p in s["pk_shares"]],
        "cts": [{"U": B.g1_compress(ct.U).hex(), "V": ct.V.hex(), "W": B.g2_compress(ct.W).hex(),
                 "shares": [B.g1_compress(x).hex() for x in s["shares"][k]], "plaintext": s["msgs"][k].hex()}
                for k, ct in enumerate(s["cts"])],
    }


def main():
    here = os.path.dirname(os.path.abspath(__file__))
    # N=64, t=21 (BASELINE.json configs[3]) material for bench.py's TDec leg and
    # the size-64 GPU parity test: 4 ciphertexts x 64 shares, 256-B plaintexts.
    n64 = {"generator": "tests/golden/make_golden_tdec.py",
           "scenario": scenario_json({"n_nodes": 64, "n_ct": 4, "msg_len": 256, "seed": 2})}
    with open(os.path.join(here, "tdec_n64.json"), "w") as f:
        json.dump(n64, f)
    out = {"generator": "tests/golden/make_golden_tdec.py"}
    out["hash_g2"] = [{"msg": m.hex(), "point": B.g2_compress(T.hash_g2(m)).hex()}
                      for m in (b"", b"hydrabadger", bytes(range(70)))]
    out["scenario"] = scenario_json({"n_nodes": 7, "n_ct": 3, "msg_len": 40, "seed": 1})
    with open(os.path.join(here, "tdec_golden.json"), "w") as f:
        json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
