#!/bin/bash
# Round 3, call c: TDec at the bench shape (100k ciphertexts x 64 shares):
# rocprofv3 kernel trace + stats, then PMC passes (one counter group per run)
# for VALU utilisation, occupancy, scratch (FLAT) instructions and HBM bytes.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-r03c}
mkdir -p "$OUT/pmc"
export TMPDIR=/tmp
KB="--cts ${CTS:-100000} --reps 1"
echo "== kernel trace"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o tdec -- \
    python3 tools/tdec_kbench.py $KB > "$OUT/trace.log" 2>&1 || { tail -20 "$OUT/trace.log"; exit 2; }
grep -v "^[WEI]2026" "$OUT/trace.log" | tail -3
i=0
for group in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_FLAT SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES" \
             "SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_LEVEL_WAVES SQ_INSTS_LDS SQ_INSTS_SMEM" \
             "FETCH_SIZE" "WRITE_SIZE" "TCP_TCC_READ_REQ_sum TCP_TCC_WRITE_REQ_sum GRBM_GUI_ACTIVE GRBM_COUNT"; do
  i=$((i+1))
  echo "== pmc pass $i: $group"
  timeout -k 10 300 rocprofv3 --pmc $group --output-format csv -d "$OUT/pmc/p$i" -o pmc -- python3 tools/tdec_kbench.py $KB \
      > "$OUT/pmc/p$i.log" 2>&1 || { echo "pmc pass $i failed"; grep -v "^[WEI]2026" "$OUT/pmc/p$i.log" | tail -20; exit 6; }
done
python3 tools/pmc_summary.py "$OUT/pmc" > "$OUT/pmc_summary.json" && head -c 3000 "$OUT/pmc_summary.json"
echo "== done"
