#!/bin/bash
# Round 4, call l: decoder diagnostics (tools/gpu_r04k.sh), the per-node
# epoch alone (bench --legs epoch) with its kernel trace, and a TDec 100 k
# kernel trace.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-r04l}
mkdir -p "$OUT"
export TMPDIR=/tmp
TAG=${TAG:-r04l} bash tools/gpu_r04k.sh || exit $?
echo "== epoch leg"
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/etrace" -o ep -- \
    python3 bench.py --steps 2 --warmup 1 --legs epoch --no-cpu --no-decode > "$OUT/epoch.json" 2> "$OUT/epoch.err" \
    || { tail -30 "$OUT/epoch.err"; exit 4; }
python3 - "$OUT/epoch.json" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
e = d.get("network_epoch") or {}
print(json.dumps({k: e.get(k) for k in ("epoch_ms", "phases_ms", "all_decrypted_ok")}))
print(json.dumps((e.get("shared_view") or {}).get("phases_ms")))
PY
echo "== TDec 100k trace"
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/ttrace" -o td -- \
    python3 tools/tdec_kbench.py --cts 100000 --reps 1 > "$OUT/tdec.json" 2> "$OUT/tdec.err" || { tail -30 "$OUT/tdec.err"; exit 5; }
cut -c1-400 "$OUT/tdec.json"
echo "== done"
