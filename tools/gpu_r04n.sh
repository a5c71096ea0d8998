#!/bin/bash
# Round 4, call n: TDec changes — BLS / TDec GPU tests, TDec at 100 k with a
# kernel trace (per-kernel times).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-r04n}
mkdir -p "$OUT"
export TMPDIR=/tmp
echo "== BLS / TDec tests"
timeout -k 10 900 python -u -m pytest tests/test_gpu_tdec.py tests/test_gpu_bls_ops.py tests/test_gpu_async.py \
    -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/pytest_bls.log" 2>&1 || { tail -40 "$OUT/pytest_bls.log"; exit 2; }
tail -2 "$OUT/pytest_bls.log"
echo "== TDec 100k (trace)"
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/ttrace" -o td -- \
    python3 tools/tdec_kbench.py --cts 100000 --reps 2 > "$OUT/tdec.json" 2> "$OUT/tdec.err" || { tail -30 "$OUT/tdec.err"; exit 3; }
cut -c1-420 "$OUT/tdec.json"
python3 - "$OUT/ttrace/td_kernel_stats.csv" <<'PY'
import csv, sys
for x in list(csv.DictReader(open(sys.argv[1])))[:12]:
    print(x["Name"][:60], x["Calls"], round(float(x["AverageNs"]) / 1e6, 2))
PY
echo "== done"
