#!/bin/bash
# Round-3 first validation of HEAD: full GPU suite, smoke, TDec diag at the
# sizes that faulted in round 2, then the bench.  Every GPU step has its own
# time limit; the script stops at the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-r03a}
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
echo "== diag ${DIAG_SIZES:-8192,65536,100000}"
AMD_SERIALIZE_KERNEL=${SERIALIZE:-0} timeout -k 10 600 python -u tools/diag_tdec.py --n-ct "${DIAG_SIZES:-8192,65536,100000}" \
    > "$OUT/diag.log" 2> "$OUT/diag.err" || { cat "$OUT/diag.log"; tail -20 "$OUT/diag.err"; exit 4; }
cat "$OUT/diag.log"
if [ -n "${BENCH_ARGS:-}" ]; then
  echo "== bench $BENCH_ARGS"
  timeout -k 10 900 python -u bench.py $BENCH_ARGS > "$OUT/bench.json" 2> "$OUT/bench.err" \
      || { tail -30 "$OUT/bench.err"; exit 5; }
  cat "$OUT/bench.json"
fi
echo "== done"
