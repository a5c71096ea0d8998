#!/usr/bin/env python3
"""SHA3(V) latency probe: threshold-encrypts `--n` messages of `--len` bytes
(the configs[4] proposer side: 128 contributions of 1 MiB) `--reps` times;
run it under `rocprofv3 --kernel-trace --stats` for tdec_v_digest_wave's
time per launch.  In a tool build with the A/B switches
(`python tools/build_variant.py ab -DHBG_TOOL_AB`, loaded with
HBG_LIB_PATH=tools/libhbgpu_ab.so) `HBG_SHA3_WAVE64=1` selects the round-3
(lo, hi)-per-lane sponge and `HBG_SHA3_3STAGE=1` the two-stage theta; the
product library has no environment switch.  The digests are checked against
hashlib through W's preimage on the host: every ciphertext must pass the
device Ciphertext::verify.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=128)
    ap.add_argument("--len", type=int, default=1 << 20)
    ap.add_argument("--reps", type=int, default=3)
    a = ap.parse_args()
    import random

    from oracle import bls12_381 as B
    from hydrabadger_amd import threshold as th
    rng = np.random.default_rng(7)
    # unaligned starts: every message one byte longer than the last
    msgs = [rng.integers(0, 256, a.len + (j % 5), dtype=np.uint8).tobytes() for j in range(a.n)]
    pk = B.g1_compress(B.g1_mul(B.G1, 12345))
    r = random.Random(3)
    rs = [r.randrange(1, B.R) for _ in msgs]
    times = []
    cts = None
    for _ in range(a.reps):
        t0 = time.perf_counter()
        cts = th.encrypt_batch(pk, msgs, rs)
        times.append((time.perf_counter() - t0) * 1e3)
    ok = bool(th.ct_verify_batch(cts).all())
    # the device digest feeds both W and ct_verify, so pin two W's on the oracle
    from oracle import tcrypto as T
    for j in (0, 3):
        u = B.g1_mul(B.G1, rs[j])
        ok = ok and cts[j].W == B.g2_compress(B.g2_mul(T.hash_g1_g2(u, cts[j].V), rs[j]))
    print(json.dumps({"n": a.n, "len": a.len, "wave64": bool(os.environ.get("HBG_SHA3_WAVE64")),
                      "encrypt_host_ms": times, "all_verify_and_oracle_W": ok}))
    if not ok:
        sys.exit(1)


if __name__ == "__main__":
    main()
