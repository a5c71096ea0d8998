#!/usr/bin/env python3
"""Print the headline and the main legs of a bench.py JSON line (GPU-run summaries)."""
import json
import sys

d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
r = d.get("roofline", {})
print("headline", round(d["value"], 1), d["unit"], round(d["ms_per_step"], 2), "ms", "frac", round(r.get("frac", 0), 3),
      {k: r[k] for k in ("clock_GHz", "frac_at_measured_clock") if k in r})
for k in ("decode", "tdec", "network_epoch", "config1_n16", "n128_encode_merkle"):
    v = d.get(k)
    if isinstance(v, dict):
        print(k, {a: b for a, b in v.items() if isinstance(b, (int, float, bool, str)) and len(str(b)) < 40})
print("leg_errors", d.get("leg_errors"))
