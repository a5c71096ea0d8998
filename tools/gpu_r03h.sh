#!/bin/bash
# Round 3: fused rbc_encode_merkle as the default step at N = 64 — full GPU
# suite, smoke, the default bench line, a rocprofv3 kernel trace (csv) of a
# short bench run, and PMC passes (HBM bytes, VALU counters) of the fused
# kernel at the bench's launch shape (8,192 x 1 MiB).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-r03h}
mkdir -p "$OUT"
export TMPDIR=/tmp
echo "== pytest"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
    > "$OUT/pytest.log" 2>&1 || { tail -40 "$OUT/pytest.log"; exit 2; }
tail -2 "$OUT/pytest.log"
echo "== smoke"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 \
    || { tail -20 "$OUT/smoke.log"; exit 3; }
echo "== bench"
timeout -k 10 900 python -u bench.py ${BENCH_ARGS:-} > "$OUT/bench.json" 2> "$OUT/bench.err" \
    || { tail -30 "$OUT/bench.err"; exit 5; }
cut -c1-1200 "$OUT/bench.json"
echo "== rocprofv3 kernel trace"
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- \
    python3 bench.py --steps 5 --warmup 1 --no-cpu > "$OUT/prof_bench.json" 2> "$OUT/prof.err" \
    || { tail -30 "$OUT/prof.err"; exit 6; }
echo "== pmc fused 8192"
TAG=${TAG:-r03h} KB_ARGS="--what fused --instances 8192 --reps 2" bash tools/pmc.sh > "$OUT/pmc.log" 2>&1 \
    || { tail -30 "$OUT/pmc.log"; exit 7; }
tail -30 "$OUT/pmc.log"
echo "== done"
