#!/bin/bash
# Quick GPU iteration: selected parity tests, then kernel timings.
#   TAG=x TESTS="tests/test_gpu_rbc.py" KB_ARGS="--what encode,rs --instances 2048" bash tools/gpu_quick.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-quick}
mkdir -p "$OUT"
export TMPDIR=/tmp
if [ -n "${TESTS:-}" ]; then
  echo "== pytest $TESTS"
  timeout -k 10 600 python -u -m pytest $TESTS -m gpu -x -q --timeout 120 --timeout-method thread > "$OUT/pytest.log" 2>&1
  rc=$?; tail -15 "$OUT/pytest.log"; echo "pytest rc=$rc"
  if [ $rc -ne 0 ]; then exit $rc; fi
fi
if [ -n "${KB_ARGS:-}" ]; then
  echo "== kbench $KB_ARGS"
  timeout -k 10 600 python tools/kbench.py $KB_ARGS > "$OUT/kbench.jsonl" 2> "$OUT/kbench.err" || { tail -20 "$OUT/kbench.err"; exit 4; }
  cat "$OUT/kbench.jsonl"
fi
if [ -n "${BENCH_ARGS:-}" ]; then
  echo "== bench $BENCH_ARGS"
  timeout -k 10 600 python bench.py $BENCH_ARGS > "$OUT/bench.json" 2> "$OUT/bench.err" || { tail -20 "$OUT/bench.err"; exit 5; }
  cat "$OUT/bench.json"
fi
echo "== done"
