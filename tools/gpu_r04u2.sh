#!/bin/bash
# Round 4: the per-node epoch alone (bench --legs epoch) with its kernel trace
# at HEAD, itemised by tools/itemise_trace.py.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-r04u2}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/etrace" -o ep -- \
    python3 bench.py --steps 2 --warmup 1 --legs epoch --no-cpu --no-decode > "$OUT/epoch.json" 2> "$OUT/epoch.err" \
    || { tail -30 "$OUT/epoch.err"; exit 4; }
python3 - "$OUT/epoch.json" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
e = d.get("network_epoch") or {}
print(json.dumps({k: e.get(k) for k in ("epoch_ms", "phases_ms", "all_decrypted_ok")}))
PY
python3 tools/itemise_trace.py "$OUT/etrace/ep_kernel_trace.csv" > "$OUT/itemised.txt" && cat "$OUT/itemised.txt"
echo "== done"
