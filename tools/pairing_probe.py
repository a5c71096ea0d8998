#!/usr/bin/env python3
"""Pairing-stage probe: times the Miller loop, the final exponentiation and
the whole pairing on the device (hbg_test_bls ops 7 / 8 / 5, one lane per
pairing, every lane the same generator pair) and, with the instrumented
library, counts their Fp multiplications — so the TDec pairing kernels'
issue efficiency can be split between the two stages.

    python tools/pairing_probe.py --n 65536                      # product library
    HBG_LIB_PATH=tools/libhbgpu_fpcount.so python tools/pairing_probe.py --n 4096 --count

Run the first under `rocprofv3 --kernel-trace --stats` for the kernel times
(tdec_test launches in op order 7, 8, 5 after one warm-up launch each).
"""
from __future__ import annotations

import argparse
import ctypes as C
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=65536)
    ap.add_argument("--count", action="store_true", help="print the instrumented library's Fp counts")
    a = ap.parse_args()
    from oracle import bls12_381 as B
    from tests.tdec_fixtures import limbs
    from hydrabadger_amd import _lib, threshold as th
    p, q = B.G1, B.G2
    row = limbs(p[0]) + limbs(p[1]) + limbs(q[0][0]) + limbs(q[0][1]) + limbs(q[1][0]) + limbs(q[1][1])
    inp = np.tile(np.array(row, np.uint32), (a.n, 1))
    out = {"n": a.n}
    lib = _lib.lib()
    if a.count:
        lib.hbg_fp_count_report.argtypes = [C.c_char_p, C.c_uint64]
        lib.hbg_fp_count_report.restype = C.c_int

    def report():
        buf = C.create_string_buffer(1 << 16)
        assert lib.hbg_fp_count_report(buf, len(buf)) == 0
        return json.loads(buf.value.decode())

    ml = None
    for op, name in ((7, "miller_loop+g2_prepare"), (8, "final_exponentiation"), (5, "pairing")):
        x = ml if op == 8 else inp
        th.test_bls(op, x[:64], 144)  # warm-up
        if a.count:
            report()  # drain
        t0 = time.perf_counter()
        r = th.test_bls(op, x, 144)
        dt = time.perf_counter() - t0
        if op == 7:
            ml = r
        ent = {"host_call_ms": dt * 1e3}
        if a.count:
            k = report().get("tdec_test", [0, 0, 0])  # [fp_mul, fp_sqr, launches]
            ent["fp_mul_per_lane"] = k[0] / a.n
            ent["fp_sqr_per_lane"] = k[1] / a.n
            ent["fp_per_lane"] = (k[0] + k[1]) / a.n
        out[name] = ent
    print(json.dumps(out))


if __name__ == "__main__":
    main()
