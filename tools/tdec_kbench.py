#!/usr/bin/env python3
"""TDec kernel timing through the C ABI (bench.py's tdec_leg on its own).

    python tools/tdec_kbench.py --cts 1024 --reps 3

One JSON line: verify/combine ms and rates, plus the validity/plaintext checks
against the committed N=64 t=21 fixture.  Target of rocprofv3 --pmc passes.
"""
from __future__ import annotations

import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cts", type=int, default=1024)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--per-share", action="store_true",
                    help="also time the HBG_VERIFY_PER_SHARE schedule (off: the PMC passes profile the batched call)")
    a = ap.parse_args()
    import bench
    from hydrabadger_amd import _lib

    dev = torch.device("cuda", 0)
    st = torch.cuda.Stream(dev)
    torch.cuda.set_stream(st)
    ctx = _lib.Context(0)
    ctx.set_stream(st.cuda_stream)
    print(json.dumps(bench.tdec_leg(ctx, dev, a.cts, a.reps, per_share=a.per_share)[0]), flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
