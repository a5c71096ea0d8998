#!/bin/bash
# Round 3: locate rounds in the batched share verifier — TDec parity (incl. the
# configs[3]-size test and the forced-batched cases), the TDec bench leg, and a
# kernel trace of one TDec step.
set -o pipefail
OUT=gpurun_out/${TAG:-r03aj}
mkdir -p $OUT
echo "== pytest"
timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
    tests/test_gpu_tdec.py tests/test_tdec_glue.py tests/test_gpu_async.py > $OUT/pytest.log 2>&1 \
    || { tail -30 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
ARGS="--steps 3 --warmup 1 --no-cpu --no-decode --legs tdec"
timeout -k 10 400 python -u bench.py $ARGS > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
python - <<'PY'
import json, os
o = os.environ.get("TAG", "r03aj")
d = json.loads(open(f"gpurun_out/{o}/bench.json").read().strip().splitlines()[-1])
t = d["tdec"]
print("tdec", round(t["value"]), round(t["threshold_decrypt_ms"], 1), t["ok_bits_match"], t["outcomes_match"],
      t["plaintexts_match"], d.get("leg_errors"))
PY
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $OUT/prof -o run -- \
    python3 bench.py $ARGS > $OUT/prof.json 2> $OUT/prof.err || { tail -20 $OUT/prof.err; exit 1; }
echo "== done"
