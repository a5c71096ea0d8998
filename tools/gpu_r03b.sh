#!/bin/bash
# Round 3, call b: Keccak rotation probes (tools/ubench4), the configs[3]-size
# TDec GPU test, the counter list, and PMC passes over the TDec kernels at the
# bench shape (100k ciphertexts x 64 shares).  Each GPU step is time-limited;
# the script stops at the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-r03b}
mkdir -p "$OUT"
export TMPDIR=/tmp
echo "== ubench4"
timeout -k 10 180 ./tools/ubench4 > "$OUT/ubench4.txt" 2>&1 || { tail -20 "$OUT/ubench4.txt"; exit 2; }
cat "$OUT/ubench4.txt"
echo "== pytest configs[3] size"
timeout -k 10 400 python -u -m pytest tests/test_tdec_glue.py -m gpu -x -v --timeout 300 --timeout-method thread \
    -k configs3 > "$OUT/pytest.log" 2>&1 || { tail -40 "$OUT/pytest.log"; exit 3; }
tail -3 "$OUT/pytest.log"
echo "== counters"
timeout -k 10 120 rocprofv3 -L > "$OUT/counters.txt" 2>&1 || echo "rocprofv3 -L rc=$?"
KB="--cts ${CTS:-100000} --reps 1"
i=0
for group in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY" \
             "SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INST_CYCLES_VMEM_RD" \
             "FETCH_SIZE" "WRITE_SIZE" "GRBM_GUI_ACTIVE GRBM_COUNT"; do
  i=$((i+1))
  echo "== pmc pass $i: $group"
  timeout -k 10 300 rocprofv3 --pmc $group --output-format csv -d "$OUT/pmc/p$i" -o pmc -- python3 tools/tdec_kbench.py $KB \
      > "$OUT/pmc/p$i.log" 2>&1 || { echo "pmc pass $i failed"; tail -20 "$OUT/pmc/p$i.log"; exit 6; }
done
python3 tools/pmc_summary.py "$OUT/pmc" > "$OUT/pmc_summary.json" && cat "$OUT/pmc_summary.json" | head -150
echo "== done"
