#!/bin/bash
# Coin-share verification session: the §8(f3) GPU tests + a coin-only bench.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-coin}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_bls_ops.py -m gpu -x -v --timeout 120 --timeout-method thread > "$OUT/pytest.log" 2>&1
rc=$?; tail -15 "$OUT/pytest.log"; echo "pytest rc=$rc"
if [ $rc -ne 0 ]; then exit $rc; fi
HBG_TDEC_DEBUG=1 timeout -k 10 300 python bench.py --steps 2 --warmup 1 --instances 256 --no-cpu --no-decode --tdec-cts 0 --epoch-nodes 0 --wire-msgs 0 --f1-cts 0 > "$OUT/bench.json" 2> "$OUT/bench.err" || { tail -20 "$OUT/bench.err"; exit 5; }
python3 -c "import json; d=json.load(open('$OUT/bench.json')); print(d['coin'])"
grep "sig verify" "$OUT/bench.err" | sort | uniq -c | head
