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
        # the key polynomial (Fr coefficients, 32-byte LE): lets a crate-side
        # check build the PublicKeySet / SecretKeyShares (rust/kat-gen)
        "poly": [c.to_bytes(32, "little").hex() for c in s["ks"].coeffs],
        "pk_shares": [B.g1_compress(p).hex() for p in s["pk_shares"]],
        "cts": [{"U": B.g1_compress(ct.U).hex(), "V": ct.V.hex(), "W": B.g2_compress(ct.W).hex(),
                 "shares": [B.g1_compress(x).hex() for x in s["shares"][k]], "plaintext": s["msgs"][k].hex()}
                for k, ct in enumerate(s["cts"])],
    }


def a18_cases():
    """hbbft ThresholdDecrypt arrival cases on the N=7 scenario (SURVEY.md §8
    a18), seen from node 0: `crate_arrival` is what hbbft's ThresholdDecrypt
    of node 0 receives (handle_message per entry, "ct" = set_ciphertext +
    start_decryption, which inserts node 0's own share before try_output; no
    "ct": before the first entry); `arrival` is the same history for
    hbg_tdec_threshold_decrypt, whose marker for a validator is
    ARRIVAL_OWN | 0 ("own").  The last case holds t+1 valid shares at the
    ciphertext already: node 0's own share is among the first t+1 by node id
    (accepted and interpolated) as in hbbft.  One share replaced by a bad one
    (`bad_sender`); status / outcomes / plaintext are the oracle's."""
    s = scenario(7, 3, 40, 1)
    t, pks = s["t"], s["pk_shares"]
    M = T.ARRIVAL_CIPHERTEXT
    cases = []
    OWN0 = T.ARRIVAL_OWN | 0
    for k, bad, crate in ((0, 1, [6, 6, 1, 5, 3, 2]), (1, 1, [3, 1, 3, M, 2, 4]), (2, 4, [5, 4, 6, M, 1, 2]),
                          (0, 1, [1, M, 1, 2]), (1, 2, [1, 2, 2, 3, 4, 5, 6]), (2, 4, [3, 5, 6, 4, M, 1, 2])):
        arrival = [OWN0 if a == M else a for a in crate] if M in crate else [OWN0] + list(crate)
        shares = list(s["shares"][k])
        shares[bad] = B.g1_add(shares[bad], B.G1)
        st, pt, oc = T.threshold_decrypt(t, s["cts"][k], pks, shares, arrival)
        cases.append({"ct": k, "bad_sender": bad, "bad_share": B.g1_compress(shares[bad]).hex(),
                      "crate_arrival": ["ct" if a == M else a for a in crate],
                      "arrival": ["own" if a == OWN0 else a for a in arrival], "status": st,
                      "outcome": oc, "plaintext": None if pt is None else pt.hex()})
    return {"outcome_codes": {"none": T.SHARE_NONE, "accepted": T.SHARE_ACCEPTED, "faulty": T.SHARE_FAULTY,
                              "ignored": T.SHARE_IGNORED, "repeat_flag": T.SHARE_REPEAT},
            "status_codes": {"ok": 0, "not_enough_shares": T.E_NOT_ENOUGH_SHARES,
                             "invalid_ciphertext": T.E_INVALID_CIPHERTEXT},
            "our_node": 0, "cases": cases}


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
    out["threshold_decrypt"] = a18_cases()
    with open(os.path.join(here, "tdec_golden.json"), "w") as f:
        json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
