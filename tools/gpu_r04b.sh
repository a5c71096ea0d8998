#!/bin/bash
# Round 4, call b: the register-resident BLS tower (fixed-register Montgomery
# subroutines hbg_fpmul1/2/3, pairing / G2 kernels at one wave per SIMD).
# (1) the BLS GPU tests (fast fail), (2) TDec at configs[3] size, (3) the whole
# GPU suite.  Every step has its own time limit; stops at the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-r04b}
mkdir -p "$OUT"
export TMPDIR=/tmp
echo "== BLS tests"
timeout -k 10 600 python -u -m pytest tests/test_gpu_tdec.py tests/test_gpu_bls_ops.py -m gpu -x -q --timeout 300 \
    --timeout-method thread > "$OUT/pytest_bls.log" 2>&1 || { tail -40 "$OUT/pytest_bls.log"; exit 2; }
tail -3 "$OUT/pytest_bls.log"
echo "== TDec 100k"
timeout -k 10 600 python -u tools/tdec_kbench.py --cts ${CTS:-100000} --reps 2 > "$OUT/tdec.json" 2> "$OUT/tdec.err" \
    || { tail -30 "$OUT/tdec.err"; exit 3; }
cut -c1-1500 "$OUT/tdec.json"
echo "== full GPU suite"
timeout -k 10 1200 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
    > "$OUT/pytest.log" 2>&1 || { tail -40 "$OUT/pytest.log"; exit 4; }
tail -3 "$OUT/pytest.log"
echo "== done"
