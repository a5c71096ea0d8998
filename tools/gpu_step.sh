#!/bin/bash
# One GPU iteration: selected parity tests, then a bench run with chosen legs.
#   TAG=name TESTS="tests/a.py tests/b.py" BENCH_ARGS="..." bash tools/gpu_step.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-step}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest ${TESTS:-tests} -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/pytest.log" 2>&1
rc=$?; tail -15 "$OUT/pytest.log"; echo "pytest rc=$rc"
if [ $rc -ne 0 ]; then exit $rc; fi
if [ -n "${BENCH_ARGS:-}" ]; then
  timeout -k 10 500 python bench.py $BENCH_ARGS > "$OUT/bench.json" 2> "$OUT/bench.err" || { tail -20 "$OUT/bench.err"; exit 4; }
  tail -4 "$OUT/bench.err"
  cat "$OUT/bench.json"
fi
