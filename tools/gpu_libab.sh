#!/bin/bash
# A/B of alternative builds of libhbgpu.so (HBG_LIB_PATH): RBC parity tests + kbench.
#   LIBS="tools/var/libhbgpu_pf4.so ..." KB_ARGS="--what encode --instances 8192" bash tools/gpu_libab.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-libab}
mkdir -p "$OUT"
export TMPDIR=/tmp
for lib in ${LIBS}; do
  n=$(basename "$lib" .so)
  echo "== $lib"
  HBG_LIB_PATH=$PWD/$lib timeout -k 10 300 python -u -m pytest tests/test_gpu_rbc.py -m gpu -x -q --timeout 120 --timeout-method thread > "$OUT/pytest_$n.log" 2>&1 || { tail -20 "$OUT/pytest_$n.log"; exit 2; }
  tail -1 "$OUT/pytest_$n.log"
  HBG_LIB_PATH=$PWD/$lib timeout -k 10 300 python tools/kbench.py ${KB_ARGS} > "$OUT/kb_$n.jsonl" 2> "$OUT/kb_$n.err" || { tail -20 "$OUT/kb_$n.err"; exit 4; }
  cat "$OUT/kb_$n.jsonl"
done
echo "== done"
