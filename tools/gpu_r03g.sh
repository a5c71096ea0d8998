#!/bin/bash
# Round 3: 64-lane group combine (configs[4] t=42) and the LDS-ring fused
# rbc_encode_merkle — the GPU tests of the TDec / coin / glue / epoch / RBC
# paths, fused-vs-two-launch A/B timing, then the epoch + coin bench legs.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-r03g}
mkdir -p "$OUT"
export TMPDIR=/tmp
echo "== pytest"
timeout -k 10 900 python -u -m pytest tests/test_gpu_tdec.py tests/test_gpu_async.py tests/test_gpu_bls_ops.py \
    tests/test_tdec_glue.py tests/test_epoch.py tests/test_gpu_rbc.py -m gpu -x -q --timeout 300 --timeout-method thread \
    > "$OUT/pytest.log" 2>&1 || { tail -40 "$OUT/pytest.log"; exit 2; }
tail -2 "$OUT/pytest.log"
echo "== kbench fused A/B"
for i in 1 2; do
timeout -k 10 300 python -u tools/kbench.py --what encode,fused --instances 2048,8192 --reps 5 \
    >> "$OUT/kbench.jsonl" 2>> "$OUT/kbench.err" || { tail -20 "$OUT/kbench.err"; exit 3; }
done
timeout -k 10 300 python -u tools/kbench.py --what encode,fused --instances 2048 --nodes 128 --reps 5 \
    >> "$OUT/kbench.jsonl" 2>> "$OUT/kbench.err" || { tail -20 "$OUT/kbench.err"; exit 4; }
timeout -k 10 300 python -u tools/kbench.py --what encode,fused --instances 10000 --nodes 16 --payload 65536 --reps 5 \
    >> "$OUT/kbench.jsonl" 2>> "$OUT/kbench.err" || { tail -20 "$OUT/kbench.err"; exit 4; }
cat "$OUT/kbench.jsonl"
echo "== bench epoch + coin"
timeout -k 10 600 python -u bench.py --steps 3 --warmup 1 --legs epoch,coin --no-cpu --tdec-cts 0 > "$OUT/bench.json" \
    2> "$OUT/bench.err" || { tail -30 "$OUT/bench.err"; exit 6; }
python -c "import json; d=json.load(open('$OUT/bench.json')); print(json.dumps({k: d.get(k) for k in ('network_epoch', 'coin')})[:3000])"
echo "== done"
