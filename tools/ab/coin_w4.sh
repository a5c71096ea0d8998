#!/bin/bash
# BLS share-verification tests + coin and ThresholdDecrypt timing on the product library.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/${TAG:-coinw4}
mkdir -p "$OUT"
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_bls_ops.py tests/test_gpu_tdec.py tests/test_tdec_glue.py -m gpu -x -q \
    --timeout 300 --timeout-method thread > "$OUT/pytest.log" 2>&1 || { tail -30 "$OUT/pytest.log"; exit 2; }
tail -2 "$OUT/pytest.log"
timeout -k 10 400 python3 bench.py --no-cpu --legs coin --steps 3 --warmup 1 > "$OUT/bench.json" 2> "$OUT/bench.err" \
    || { tail -20 "$OUT/bench.err"; exit 3; }
python3 -c "
import json; d=json.loads(open('$OUT/bench.json').read().strip().splitlines()[-1]); print(json.dumps(d.get('coin')))"
timeout -k 10 300 python3 tools/tdec_kbench.py --cts 100000 --reps 2 > "$OUT/100k.json" 2>&1 || { tail -5 "$OUT/100k.json"; exit 4; }
tail -c 300 "$OUT/100k.json"
