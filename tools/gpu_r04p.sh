#!/bin/bash
# Round 4, call p: reproducible TDec roofline at HEAD — Fp-multiplication
# counts (instrumented build: the bench's 1 % profile and the 0 % floor), the
# TDec PMC passes at 100 k x 64 (tools/gpu_r03c.sh), then the whole GPU suite.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-r04p}
mkdir -p "$OUT"
export TMPDIR=/tmp
echo "== fpcount 1 %"
timeout -k 10 300 python -u tools/fpcount.py run --n-ct 2048 --out "$OUT/fpcount.json" > "$OUT/fpcount.log" 2>&1 \
    || { tail -20 "$OUT/fpcount.log"; exit 2; }
tail -c 300 "$OUT/fpcount.log"; echo
echo "== fpcount 0 %"
timeout -k 10 300 python -u tools/fpcount.py run --n-ct 2048 --bad-rate 0 --out "$OUT/fpcount_batched_0pct.json" \
    > "$OUT/fpcount0.log" 2>&1 || { tail -20 "$OUT/fpcount0.log"; exit 3; }
tail -c 300 "$OUT/fpcount0.log"; echo
TAG=${TAG:-r04p}_pmc CTS=100000 bash tools/gpu_r03c.sh > "$OUT/pmc.log" 2>&1 || { tail -30 "$OUT/pmc.log"; exit 4; }
tail -c 600 "$OUT/pmc.log"; echo
echo "== full GPU suite"
timeout -k 10 1200 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread \
    > "$OUT/pytest.log" 2>&1 || { tail -40 "$OUT/pytest.log"; exit 5; }
tail -3 "$OUT/pytest.log"
echo "== done"
