#!/bin/bash
# Round 4, call i: software-pipelined carry counts in hbg_fpmul1/2/3 + paired
# G1 products (BLS tests, subroutine issue rates, TDec at 100 k), nt stores in
# the encode / decode kernels (RBC tests, encode + decode timing), the
# per-node epoch GPU tests.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-r04i}
mkdir -p "$OUT"
export TMPDIR=/tmp
echo "== fp subroutine issue rate"
timeout -k 10 120 ./tools/ubench6b > "$OUT/ubench6.json" 2>&1 || { cat "$OUT/ubench6.json"; exit 7; }
cat "$OUT/ubench6.json"
echo "== BLS tests"
timeout -k 10 600 python -u -m pytest tests/test_gpu_tdec.py tests/test_gpu_bls_ops.py -m gpu -x -q --timeout 300 \
    --timeout-method thread > "$OUT/pytest_bls.log" 2>&1 || { tail -40 "$OUT/pytest_bls.log"; exit 2; }
tail -2 "$OUT/pytest_bls.log"
echo "== RBC tests"
timeout -k 10 600 python -u -m pytest tests/test_gpu_rbc.py -m gpu -x -q --timeout 300 --timeout-method thread \
    > "$OUT/pytest_rbc.log" 2>&1 || { tail -40 "$OUT/pytest_rbc.log"; exit 3; }
tail -2 "$OUT/pytest_rbc.log"
echo "== encode / decode timing"
timeout -k 10 300 python -u tools/kbench.py --what fused --instances 8192 --reps 5 > "$OUT/kbench_enc.json" 2> "$OUT/kbench_enc.err" \
    || { tail -20 "$OUT/kbench_enc.err"; exit 4; }
cat "$OUT/kbench_enc.json"
timeout -k 10 300 python -u tools/kbench.py --what decode --instances 8192 --dec-fused 1 --splits -1 --reps 5 \
    > "$OUT/kbench_dec.json" 2> "$OUT/kbench_dec.err" || { tail -20 "$OUT/kbench_dec.err"; exit 5; }
cat "$OUT/kbench_dec.json"
echo "== TDec 100k"
timeout -k 10 600 python -u tools/tdec_kbench.py --cts 100000 --reps 2 > "$OUT/tdec.json" 2> "$OUT/tdec.err" \
    || { tail -30 "$OUT/tdec.err"; exit 6; }
cut -c1-1200 "$OUT/tdec.json"
echo "== epoch GPU tests"
timeout -k 10 600 python -u -m pytest tests/test_epoch.py -m gpu -x -q --timeout 300 --timeout-method thread \
    > "$OUT/pytest_epoch.log" 2>&1 || { tail -40 "$OUT/pytest_epoch.log"; exit 8; }
tail -2 "$OUT/pytest_epoch.log"
echo "== done"
