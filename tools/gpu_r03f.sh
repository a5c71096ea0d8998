#!/bin/bash
# Round 3: fused rbc_encode_merkle with the LDS parity ring — parity tests of
# the fused schedule, then A/B timing against the two-launch schedule.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-r03f}
mkdir -p "$OUT"
export TMPDIR=/tmp
echo "== pytest fused"
timeout -k 10 300 python -u -m pytest tests/test_gpu_rbc.py -m gpu -x -q -k "fused" --timeout 120 --timeout-method thread \
    > "$OUT/pytest.log" 2>&1 || { tail -40 "$OUT/pytest.log"; exit 2; }
tail -2 "$OUT/pytest.log"
echo "== kbench"
for i in 1 2; do
timeout -k 10 300 python -u tools/kbench.py --what encode,fused --instances 2048,8192 --reps 5 \
    >> "$OUT/kbench.jsonl" 2> "$OUT/kbench.err" || { tail -20 "$OUT/kbench.err"; exit 3; }
done
timeout -k 10 300 python -u tools/kbench.py --what encode,fused --instances 2048 --nodes 128 --reps 5 \
    >> "$OUT/kbench.jsonl" 2>> "$OUT/kbench.err" || { tail -20 "$OUT/kbench.err"; exit 4; }
timeout -k 10 300 python -u tools/kbench.py --what encode,fused --instances 10000 --nodes 16 --payload 65536 --reps 5 \
    >> "$OUT/kbench.jsonl" 2>> "$OUT/kbench.err" || { tail -20 "$OUT/kbench.err"; exit 4; }
cat "$OUT/kbench.jsonl"
echo "== done"
