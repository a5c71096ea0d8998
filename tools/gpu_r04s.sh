#!/bin/bash
# Round 4, call s: encoder in-sweep payload prefetch — RBC tests + timing.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-r04s}
mkdir -p "$OUT"
export TMPDIR=/tmp
echo "== RBC tests"
timeout -k 10 600 python -u -m pytest tests/test_gpu_rbc.py -m gpu -x -q --timeout 300 --timeout-method thread \
    > "$OUT/pytest_rbc.log" 2>&1 || { tail -40 "$OUT/pytest_rbc.log"; exit 2; }
tail -2 "$OUT/pytest_rbc.log"
echo "== encode / decode timing"
for i in 1 2; do
timeout -k 10 300 python -u tools/kbench.py --what fused --instances 8192 --reps 10 2> "$OUT/kbench_enc.err" \
    || { tail -20 "$OUT/kbench_enc.err"; exit 3; }
done
timeout -k 10 300 python -u tools/kbench.py --what decode --instances 8192 --dec-fused 1 --splits -1 --reps 5 2> "$OUT/kbench_dec.err" \
    || { tail -20 "$OUT/kbench_dec.err"; exit 4; }

echo "== throughput-build TDec probe (2,048 ct, every launch on the throughput build)"
timeout -k 10 300 python -u tools/tdec_throughput_probe.py --n-ct 2048 > "$OUT/probe.json" 2> "$OUT/probe.err" \
    || { tail -20 "$OUT/probe.err"; exit 5; }
cat "$OUT/probe.json"
echo "== done"
