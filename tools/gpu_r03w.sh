#!/bin/bash
# Round 3: fused kernel A/B — product (vmcnt(0) only on edge passes) vs
# tools/libhbgpu_waitall.so (vmcnt(0) after every encode pass); parity first.
set -o pipefail
OUT=gpurun_out/${TAG:-r03w}
mkdir -p $OUT
echo "== pytest fused"
timeout -k 10 300 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu \
    tests/test_gpu_rbc.py -k "fused or roundtrip or batch_encode or mixed" > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
echo "== A/B"
for i in 1 2; do
  timeout -k 10 200 python -u tools/kbench.py --what fused --instances 8192 --reps 10 > $OUT/new_$i.jsonl 2>/dev/null || exit 1
  HBG_LIB_PATH=tools/libhbgpu_waitall.so timeout -k 10 200 python -u tools/kbench.py --what fused --instances 8192 --reps 10 > $OUT/old_$i.jsonl 2>/dev/null || exit 1
  echo "new $(cat $OUT/new_$i.jsonl)"
  echo "old $(cat $OUT/old_$i.jsonl)"
done
echo "== done"
