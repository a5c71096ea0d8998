#!/usr/bin/env python3
"""Pack rocprofv3 PMC summaries (tools/pmc_summary.py output) into the
profile files bench.py reads, stamped with the kernels' source digest
(hydrabadger_amd.build.source_digest) so the bench line can say whether its
traffic figures were measured on the kernels it runs (`measured_at_head`).

    python tools/pack_profiles.py rbc  SUMMARY.json   # kbench --what decode --dec-fused 1 --instances 8192:
                                                      #   the fused encoder -> profiles/pmc_traffic.json,
                                                      #   the decode call   -> profiles/r06/pmc_decode_fused_8192.json
    python tools/pack_profiles.py rbc2 SUMMARY.json   # kbench --what encode --instances 8192: rs_encode_const and
                                                      #   merkle_build of the two-launch schedule -> pmc_traffic.json
    python tools/pack_profiles.py tdec SUMMARY.json   # tdec_kbench --cts 100000 -> profiles/r06/pmc_tdec_100k.json

Run it where the PMC passes ran (the GPU box), on the same tree; OUT_ROOT
(default the repo root) redirects the files, e.g. under gpurun_out/ so they
come back from the box (then copy them into profiles/).
"""
from __future__ import annotations

import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    from hydrabadger_amd.build import source_digest
    what, summary = sys.argv[1], sys.argv[2]
    s = json.load(open(summary))
    meta = {"csrc_sha16": source_digest(), "summary": os.path.relpath(summary, ROOT),
            "counters": "FETCH_SIZE x2 (gfx950 correction) + WRITE_SIZE, separate rocprofv3 --pmc passes"}
    out_root = os.environ.get("OUT_ROOT", ROOT)
    os.makedirs(os.path.join(out_root, "profiles", "r06"), exist_ok=True)
    if what == "rbc":
        enc = next(v for k, v in s.items() if k.startswith("rbc_encode_merkle<22, 42>"))
        d = json.load(open(os.path.join(ROOT, "profiles", "pmc_traffic.json")))
        path = os.path.join(out_root, "profiles", "pmc_traffic.json")
        rd, wr = enc["hbm_read_bytes_corrected"], enc["hbm_write_bytes"]
        d["rbc_encode_merkle_22_42"] = {
            "instances": 8192, "hbm_bytes_per_launch": rd + wr, "read": rd, "write": wr,
            "valu_insts_per_wave": enc.get("valu_insts_per_wave"),
            "summary": meta["summary"] + " (the fused encoder launch of tools/kbench.py --what decode "
                                         "--dec-fused 1 --instances 8192)",
            "csrc_sha16": meta["csrc_sha16"]}
        json.dump(d, open(path, "w"), indent=1)
        dec = {k: v for k, v in s.items() if not k.startswith("rbc_encode_merkle")}
        dec["_meta"] = meta
        json.dump(dec, open(os.path.join(out_root, "profiles", "r06", "pmc_decode_fused_8192.json"), "w"), indent=1)
    elif what == "rbc2":
        # the two-launch schedule (kbench --what encode --instances 8192):
        # rs_encode_const<22, 42, true> then merkle_build<0>
        src = os.path.join(out_root, "profiles", "pmc_traffic.json")  # pmcrbc's, when it ran first
        if not os.path.exists(src):
            src = os.path.join(ROOT, "profiles", "pmc_traffic.json")
        d = json.load(open(src))
        for key, prefix in (("rs_encode_const_22_42", "rs_encode_const<22, 42, true>"),
                            ("merkle_build", "merkle_build<0>")):
            v = next(v for k, v in s.items() if k.startswith(prefix))
            rd, wr = v["hbm_read_bytes_corrected"], v["hbm_write_bytes"]
            d[key] = {"instances": 8192, "hbm_bytes_per_launch": rd + wr, "read": rd, "write": wr,
                      "valu_insts_per_wave": v.get("valu_insts_per_wave"),
                      "summary": meta["summary"] + " (kbench --what encode --instances 8192: the two-launch "
                                                   "schedule)",
                      "csrc_sha16": meta["csrc_sha16"]}
        json.dump(d, open(os.path.join(out_root, "profiles", "pmc_traffic.json"), "w"), indent=1)
    elif what == "tdec":
        s["_meta"] = meta
        json.dump(s, open(os.path.join(out_root, "profiles", "r06", "pmc_tdec_100k.json"), "w"), indent=1)
    else:
        raise SystemExit(f"unknown kind {what}")
    print("packed", what, meta["csrc_sha16"])


if __name__ == "__main__":
    main()
