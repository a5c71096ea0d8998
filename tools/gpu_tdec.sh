#!/bin/bash
# GPU session: RBC + TDec parity tests, VALU probes.  Each GPU step time-limited.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-r01d}
mkdir -p "$OUT"
export TMPDIR=/tmp
echo "== ubench2"; timeout -k 10 120 tools/ubench2 > "$OUT/ubench2.txt" 2>&1; echo "rc=$?"
echo "== gpu tests"; timeout -k 10 900 python -m pytest tests -m gpu -q --durations=15 > "$OUT/pytest_tdec.log" 2>&1
rc=$?; tail -30 "$OUT/pytest_tdec.log"; echo "pytest rc=$rc"
if [ $rc -gt 1 ]; then exit $rc; fi
echo "== done"
