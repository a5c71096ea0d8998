#!/bin/bash
# PMC passes (one counter group per rocprofv3 run, no tracing domains mixed in)
# over tools/kbench.py.  Usage: TAG=r01b KB_ARGS="--what merkle --instances 4096" bash tools/pmc.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-r01}/pmc
mkdir -p "$OUT"
export TMPDIR=/tmp
KB=${KB_ARGS:---what merkle,rs --instances 4096 --reps 2}
i=0
for group in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU" \
             "FETCH_SIZE" "WRITE_SIZE" ${EXTRA_GROUPS:-}; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $group --output-format csv -d "$OUT/p$i" -o pmc -- python3 tools/kbench.py $KB \
      > "$OUT/p$i.log" 2>&1 || { echo "pmc pass $i failed"; tail -20 "$OUT/p$i.log"; exit 6; }
done
python3 tools/pmc_summary.py "$OUT" > "$OUT/summary.txt" && cat "$OUT/summary.txt"
