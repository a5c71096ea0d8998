#!/bin/bash
# Round 3 re-entry, one call: (1) full validation of HEAD (tools/gpu_r03v.sh:
# whole GPU suite, smoke, default bench line, rocprofv3 kernel stats), (2) the
# TDec PMC passes at configs[3] size (tools/gpu_r03c.sh), (3) last, the
# locate-round prototype (tools/wip/tdec_locate.patch) as the debug variant
# tools/libhbgpu_locdbg.so (HBG_DEBUG_CHECKS: every step synchronised and
# named) on the batched-vs-per-share test.  Stops at the first failing step.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${TAG:-r03al}
TAG=$TAG bash tools/gpu_r03v.sh || exit 2
TAG=${TAG}_pmc CTS=100000 bash tools/gpu_r03c.sh || exit 3
OUT=gpurun_out/${TAG}_locdbg
mkdir -p $OUT
echo "== locate prototype (debug variant)"
HBG_LIB_PATH=tools/libhbgpu_locdbg.so timeout -k 10 300 python -u -m pytest -x -v --timeout 240 --timeout-method thread \
    -m gpu tests/test_gpu_tdec.py -k "batched_verify_equals_per_share" > $OUT/pytest.log 2>&1
echo "locdbg rc=$?"
grep -n "hbg\|FAIL\|passed\|failed" $OUT/pytest.log | head -40
echo "== all done"
