#!/bin/bash
# Round-2 TDec session: glue + async tests, Fp-mul counts (instrumented build),
# bench TDec leg.  Each GPU step has its own time limit; the script stops at
# the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-r02b}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_tdec_glue.py tests/test_gpu_async.py -m gpu -x -v --timeout 300 \
    --timeout-method thread > "$OUT/pytest.log" 2>&1 || { tail -40 "$OUT/pytest.log"; exit 2; }
tail -3 "$OUT/pytest.log"
timeout -k 10 300 python tools/fpcount.py run --n-ct 2048 --out "$OUT/fpcount.json" > "$OUT/fpcount.log" 2>&1 \
    || { tail -30 "$OUT/fpcount.log"; exit 3; }
cp "$OUT/fpcount.json" profiles/fpcount.json
timeout -k 10 600 python bench.py --steps 3 --warmup 1 --legs tdec ${BENCH_ARGS:-} > "$OUT/bench.json" \
    2> "$OUT/bench.err" || { tail -30 "$OUT/bench.err"; exit 4; }
python -c "import json,sys; d=json.load(open('$OUT/bench.json')); print(json.dumps(d['tdec'], indent=1))"
