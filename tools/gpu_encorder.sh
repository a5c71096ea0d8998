#!/bin/bash
# A/B of the encoder's block order (HBG_ENC_ORDER): RBC parity tests + kbench
# at the bench launch shape, one order after another.
#   ORDERS="0 1 0x200 0x201" bash tools/gpu_encorder.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-encorder}
mkdir -p "$OUT"
export TMPDIR=/tmp
for o in ${ORDERS:-0 1 0x200 0x201 0x400 0x401}; do
  echo "== order $o"
  HBG_ENC_ORDER=$o timeout -k 10 300 python -u -m pytest tests/test_gpu_rbc.py -m gpu -x -q --timeout 120 --timeout-method thread > "$OUT/pytest_$o.log" 2>&1
  rc=$?; tail -2 "$OUT/pytest_$o.log"; echo "pytest rc=$rc"
  if [ $rc -ne 0 ]; then exit $rc; fi
  HBG_ENC_ORDER=$o timeout -k 10 300 python tools/kbench.py --what merkle,encode,rs --instances 2048,8192 > "$OUT/kbench_$o.jsonl" 2> "$OUT/kbench_$o.err" || { tail -20 "$OUT/kbench_$o.err"; exit 4; }
  cat "$OUT/kbench_$o.jsonl"
done
echo "== done"
