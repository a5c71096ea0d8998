#!/usr/bin/env python3
"""Itemise one epoch of a rocprofv3 kernel trace (…_kernel_trace.csv): runs of
consecutive launches of the same kernel merged into one line
`start .. end  busy <ms> x <launches>  <kernel>` (ms from the window start),
then the busy sum and the span.  The window is the LAST `--epoch-ms`-long
stretch that starts at the earliest launch of `--first` (default: the
epoch's first kernel, merkle_build of the proposals) at most `--lead-ms`
before the last launch of `--needs` (the per-node epoch's combine).

    python tools/itemise_trace.py gpurun_out/r04u2/etrace/ep_kernel_trace.csv > profiles/.../itemised.txt
"""
from __future__ import annotations

import argparse
import csv
import re


def short(name: str) -> str:
    n = re.sub(r"\(.*$", "", name).replace("void ", "").replace("hbg::", "")
    if n.startswith("at::") or "at::native" in name:
        n = "torch " + n.split("::")[-1][:24]
    return n


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--first", default="merkle_build")
    ap.add_argument("--epoch-ms", type=float, default=700.0)
    ap.add_argument("--lead-ms", type=float, default=600.0)
    ap.add_argument("--needs", default="bls::tdec_combine",
                    help="a kernel the window must hold (default: the throughput-build combine of the "
                         "per-node epoch; the shared view's runs in bls_lat)")
    a = ap.parse_args()
    rows = list(csv.DictReader(open(a.trace)))
    ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"])) for r in rows)
    # the last epoch: the earliest `first` launch at most --lead-ms before the
    # last launch of `--needs`
    t_need = max(e[0] for e in ev if a.needs in e[2])
    cand = [e[0] for e in ev if a.first in e[2] and t_need - a.lead_ms * 1e6 <= e[0] <= t_need]
    t0 = min(cand) if cand else t_need
    win = [e for e in ev if t0 <= e[0] < t0 + a.epoch_ms * 1e6]
    lines, busy = [], 0.0
    cur = None
    for s, e, n in win:
        busy += (e - s) / 1e6
        if cur and cur[2] == n and s - cur[1] < 2e6:
            cur = [cur[0], max(cur[1], e), n, cur[3] + 1, cur[4] + (e - s) / 1e6]
        else:
            if cur:
                lines.append(cur)
            cur = [s, e, n, 1, (e - s) / 1e6]
    if cur:
        lines.append(cur)
    for s, e, n, c, b in lines:
        if b >= 1.0:
            print(f"{(s - t0) / 1e6:8.1f} .. {(e - t0) / 1e6:8.1f}  busy {b:7.1f} ms x {c:3d}  {n}")
    span = (max(e for _, e, _ in win) - t0) / 1e6
    print(f"kernel busy sum {busy:.1f} span {span:.1f}")


if __name__ == "__main__":
    main()
