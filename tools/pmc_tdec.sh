#!/bin/bash
# PMC passes over the TDec kernels (tools/tdec_kbench.py), one counter group per run.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-tdec_pmc}
mkdir -p "$OUT"
export TMPDIR=/tmp
KB=${KB_ARGS:---cts 256 --reps 1}
timeout -k 10 300 python tools/tdec_kbench.py $KB > "$OUT/plain.json" 2> "$OUT/plain.err" || { tail -5 "$OUT/plain.err"; exit 3; }
cat "$OUT/plain.json"
i=0
for group in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY" \
             "SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INST_CYCLES_VMEM_RD" \
             "GRBM_GUI_ACTIVE" ${EXTRA_GROUPS:-}; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $group --output-format csv -d "$OUT/p$i" -o pmc -- python3 tools/tdec_kbench.py $KB \
      > "$OUT/p$i.log" 2>&1 || { echo "pmc pass $i failed"; tail -20 "$OUT/p$i.log"; exit 6; }
done
python3 tools/pmc_summary.py "$OUT" > "$OUT/summary.txt" && cat "$OUT/summary.txt"
