#!/bin/bash
# Round 4, call z: the new many-pattern fused decode test, then the TDec
# kernel trace + PMC passes at the bench shape (100 k x 64) at HEAD.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-r04z}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_rbc.py -m gpu -x -q -k "many_erasure or fused_decode" --timeout 200 \
    --timeout-method thread > "$OUT/pytest_dec.log" 2>&1 || { tail -30 "$OUT/pytest_dec.log"; exit 2; }
tail -1 "$OUT/pytest_dec.log"
TAG=${TAG:-r04z}_pmc CTS=100000 bash tools/gpu_r03c.sh > "$OUT/pmc.log" 2>&1 || { tail -30 "$OUT/pmc.log"; exit 3; }
tail -c 400 "$OUT/pmc.log"; echo
echo "== done"
