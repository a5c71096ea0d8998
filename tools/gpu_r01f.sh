#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-r01f}
mkdir -p "$OUT"
export TMPDIR=/tmp
echo "== gpu tests"; timeout -k 10 900 python -m pytest tests -m gpu -q -x --durations=12 > "$OUT/pytest_gpu.log" 2>&1
rc=$?; tail -22 "$OUT/pytest_gpu.log"; echo "pytest rc=$rc"
if [ $rc -gt 1 ]; then exit $rc; fi
echo "== kbench keccak A/B"
for impl in 0 1; do HBG_KECCAK_IMPL=$impl timeout -k 10 300 python tools/kbench.py --what merkle --instances 2048,4096 --reps 4 > "$OUT/kb_impl$impl.jsonl" 2>"$OUT/kb_impl$impl.err" || { tail "$OUT/kb_impl$impl.err"; exit 4; }; echo "impl=$impl"; cat "$OUT/kb_impl$impl.jsonl"; done
echo "== bench"; timeout -k 10 600 python bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" || { tail -20 "$OUT/bench.err"; exit 5; }
cat "$OUT/bench.json"
