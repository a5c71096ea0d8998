#!/bin/bash
# One GPU session: parity tests, smoke, bench, rocprofv3 kernel stats.
# Every GPU step has its own time limit; a crash/timeout (rc >= 2 for pytest,
# != 0 for the others) stops the script before the next GPU step.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-r01}
mkdir -p "$OUT"
export TMPDIR=/tmp
echo "== pytest -m gpu"; timeout -k 10 900 python -m pytest tests -m gpu -x -q > "$OUT/pytest_gpu.log" 2>&1
rc=$?; tail -5 "$OUT/pytest_gpu.log"; echo "pytest rc=$rc"
if [ $rc -gt 1 ]; then exit $rc; fi
echo "== smoke"; timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || { cat "$OUT/smoke.log"; exit 3; }
cat "$OUT/smoke.log"
echo "== bench"; timeout -k 10 600 python bench.py ${BENCH_ARGS:-} > "$OUT/bench.json" 2> "$OUT/bench.err" || { tail -20 "$OUT/bench.err"; exit 4; }
cat "$OUT/bench.json"
if [ "${PROF:-1}" = "1" ]; then
  echo "== rocprofv3 kernel stats"
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o bench -- \
      python3 bench.py --steps 5 --warmup 1 --no-cpu > "$OUT/prof.log" 2>&1 || { tail -20 "$OUT/prof.log"; exit 5; }
  find "$OUT/prof" -name '*kernel_stats.csv' | head -3
fi
echo "== done"
