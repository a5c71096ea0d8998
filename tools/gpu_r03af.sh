#!/bin/bash
# Round 3: coin doc prepare on the latency build + the epoch's kernel timeline
# with the latency build.
set -o pipefail
OUT=gpurun_out/${TAG:-r03af}
mkdir -p $OUT
echo "== pytest"
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_bls_ops.py > $OUT/pytest.log 2>&1 \
    || { tail -30 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $OUT/prof -o run -- \
    python3 bench.py --steps 3 --warmup 1 --no-cpu --no-decode --legs epoch,coin --tdec-cts 0 > $OUT/bench.json 2> $OUT/bench.err \
    || { tail -20 $OUT/bench.err; exit 1; }
python - <<'PY'
import json, os
o = os.environ.get("TAG", "r03af")
d = json.loads(open(f"gpurun_out/{o}/bench.json").read().strip().splitlines()[-1])
e = d["network_epoch"]; c = d["coin"]
print("epoch", round(e["epoch_ms"], 1), {k: round(v, 1) for k, v in e["phases_ms"].items()})
print("coin", {k: round(v) for k, v in c.items() if isinstance(v, float)}, d.get("leg_errors"))
PY
echo "== done"
