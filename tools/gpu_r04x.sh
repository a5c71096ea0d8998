#!/bin/bash
# Round 4, call x: the decoder's GPR-index-mode coder (tools/libhbgpu_asmdec.so,
# one index dword per table lookup) — RBC tests on it, then decode timing A/B
# against the product library (compiler-lowered tab[i] selects).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-r04x}
mkdir -p "$OUT"
export TMPDIR=/tmp
echo "== RBC tests on the asm coder"
HBG_LIB_PATH=tools/libhbgpu_asmdec.so timeout -k 10 600 python -u -m pytest tests/test_gpu_rbc.py -m gpu -x -q \
    --timeout 300 --timeout-method thread > "$OUT/pytest_rbc.log" 2>&1 || { tail -40 "$OUT/pytest_rbc.log"; exit 2; }
tail -2 "$OUT/pytest_rbc.log"
echo "== decode A/B (asm = tools/libhbgpu_asmdec.so, cc = product)"
for i in 1 2 3; do
for v in asm cc; do
if [ $v = asm ]; then export HBG_LIB_PATH=tools/libhbgpu_asmdec.so; else unset HBG_LIB_PATH; fi
echo -n "$v "
timeout -k 10 300 python -u tools/kbench.py --what decode --instances 8192 --dec-fused 1 --splits -1 --reps 5 \
    2> "$OUT/kbench_dec.err" || { tail -20 "$OUT/kbench_dec.err"; exit 3; }
done
done
echo "== done"
