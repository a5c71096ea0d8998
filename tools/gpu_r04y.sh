#!/bin/bash
# Round 4, call y: the decoder's GPR-index-mode coder with an on/off pair per
# lookup (dseq2) and with idx switches separated by s_nop (dseq1): RBC tests
# and the 8,192-instance decode check + timing against the product.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-r04y}
mkdir -p "$OUT"
export TMPDIR=/tmp
for v in dseq2 dseq1; do
echo "== RBC tests on $v"
HBG_LIB_PATH=tools/libhbgpu_$v.so timeout -k 10 600 python -u -m pytest tests/test_gpu_rbc.py -m gpu -x -q \
    --timeout 300 --timeout-method thread > "$OUT/pytest_$v.log" 2>&1 || { tail -40 "$OUT/pytest_$v.log"; exit 2; }
tail -1 "$OUT/pytest_$v.log"
done
echo "== decode A/B"
for i in 1 2; do
for v in dseq2 dseq1 product; do
if [ $v = product ]; then unset HBG_LIB_PATH; else export HBG_LIB_PATH=tools/libhbgpu_$v.so; fi
echo -n "$v "
timeout -k 10 300 python -u tools/kbench.py --what decode --instances 8192 --dec-fused 1 --splits -1 --reps 5 \
    2> "$OUT/kbench_dec.err" || { tail -20 "$OUT/kbench_dec.err"; exit 3; }
done
done
echo "== done"
