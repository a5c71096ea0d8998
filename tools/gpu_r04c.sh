#!/bin/bash
# Round 4, call c: TDec at configs[3] size after the register-resident tower —
# kernel trace (per-kernel times) and PMC passes (tools/gpu_r03c.sh), then the
# epoch tests (per-node views) and the rest of the GPU suite.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${TAG:-r04c}
TAG=${TAG}_pmc CTS=100000 bash tools/gpu_r03c.sh || exit 2
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
echo "== epoch tests"
timeout -k 10 900 python -u -m pytest tests/test_epoch.py -m gpu -x -q --timeout 600 --timeout-method thread \
    > "$OUT/pytest_epoch.log" 2>&1 || { tail -40 "$OUT/pytest_epoch.log"; exit 3; }
tail -3 "$OUT/pytest_epoch.log"
echo "== full GPU suite"
timeout -k 10 1200 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread \
    > "$OUT/pytest.log" 2>&1 || { tail -40 "$OUT/pytest.log"; exit 4; }
tail -3 "$OUT/pytest.log"
echo "== done"
