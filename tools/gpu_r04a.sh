#!/bin/bash
# Round 4, call a: make the configs[2] / configs[3] rooflines reproducible at
# HEAD.  (1) Fp-multiplication counts of the ThresholdDecrypt kernels from the
# instrumented build (tools/libhbgpu_fpcount.so, built on the CPU beforehand):
# the bench's 1 % bad-share profile and the 0 % floor; (2) the decode path at
# the headline's 8,192 x 1 MiB (library-default schedule): kernel trace + PMC
# passes (one counter group per rocprofv3 run).  Stops at the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-r04a}
mkdir -p "$OUT/pmc"
export TMPDIR=/tmp
echo "== fpcount 1 %"
timeout -k 10 300 python -u tools/fpcount.py run --n-ct 2048 --out "$OUT/fpcount.json" > "$OUT/fpcount.log" 2>&1 \
    || { tail -20 "$OUT/fpcount.log"; exit 2; }
tail -c 400 "$OUT/fpcount.log"; echo
echo "== fpcount 0 %"
timeout -k 10 300 python -u tools/fpcount.py run --n-ct 2048 --bad-rate 0 --out "$OUT/fpcount_batched_0pct.json" \
    > "$OUT/fpcount0.log" 2>&1 || { tail -20 "$OUT/fpcount0.log"; exit 3; }
tail -c 400 "$OUT/fpcount0.log"; echo
KB="--what decode --instances ${INST:-8192} --splits -1 --reps 3"
echo "== decode kernel trace"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o dec -- \
    python3 tools/kbench.py $KB > "$OUT/trace.log" 2>&1 || { tail -20 "$OUT/trace.log"; exit 4; }
grep "^{" "$OUT/trace.log"
i=0
for group in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU" \
             "FETCH_SIZE" "WRITE_SIZE" "GRBM_GUI_ACTIVE GRBM_COUNT SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR"; do
  i=$((i+1))
  echo "== pmc pass $i: $group"
  timeout -k 10 300 rocprofv3 --pmc $group --output-format csv -d "$OUT/pmc/p$i" -o pmc -- python3 tools/kbench.py $KB \
      > "$OUT/pmc/p$i.log" 2>&1 || { echo "pmc pass $i failed"; tail -20 "$OUT/pmc/p$i.log"; exit 6; }
done
python3 tools/pmc_summary.py "$OUT/pmc" > "$OUT/pmc_summary.json" && head -c 2500 "$OUT/pmc_summary.json"
echo "== done"
