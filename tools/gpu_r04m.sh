#!/bin/bash
# Round 4, call m: spread one-item-per-lane BLS launches + vector keystream:
# BLS / epoch GPU tests, TDec at 100 k, the epoch leg (with kernel trace).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-r04m}
mkdir -p "$OUT"
export TMPDIR=/tmp
echo "== BLS + epoch tests"
timeout -k 10 900 python -u -m pytest tests/test_gpu_tdec.py tests/test_gpu_bls_ops.py tests/test_epoch.py tests/test_gpu_async.py \
    -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/pytest_bls.log" 2>&1 || { tail -40 "$OUT/pytest_bls.log"; exit 2; }
tail -2 "$OUT/pytest_bls.log"
echo "== TDec 100k"
timeout -k 10 600 python -u tools/tdec_kbench.py --cts 100000 --reps 2 > "$OUT/tdec.json" 2> "$OUT/tdec.err" \
    || { tail -30 "$OUT/tdec.err"; exit 3; }
cut -c1-300 "$OUT/tdec.json"
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
echo "== done"
