#!/bin/bash
# Round 3 re-entry validation of HEAD: full GPU suite, smoke, then the default
# bench line and a rocprofv3 kernel-trace summary of a short bench run.  Every
# GPU step has its own time limit; the script stops at the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-r03v}
mkdir -p "$OUT"
export TMPDIR=/tmp
echo "== pytest"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
    > "$OUT/pytest.log" 2>&1 || { tail -40 "$OUT/pytest.log"; exit 2; }
tail -3 "$OUT/pytest.log"
echo "== smoke"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 \
    || { tail -20 "$OUT/smoke.log"; exit 3; }
tail -2 "$OUT/smoke.log"
echo "== bench ${BENCH_ARGS:-}"
timeout -k 10 900 python -u bench.py ${BENCH_ARGS:-} > "$OUT/bench.json" 2> "$OUT/bench.err" \
    || { tail -30 "$OUT/bench.err"; exit 5; }
cut -c1-1500 "$OUT/bench.json"
if [ -z "${NO_PROF:-}" ]; then
  echo "== rocprofv3 kernel trace"
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- \
      python bench.py --steps 5 --warmup 1 --no-cpu > "$OUT/prof_bench.json" 2> "$OUT/prof.err" \
      || { tail -30 "$OUT/prof.err"; exit 6; }
fi
echo "== done"
