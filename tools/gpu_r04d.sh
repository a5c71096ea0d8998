#!/bin/bash
# Round 4, call d: the fused decoder (rbc_decode_merkle<22,42>): RBC GPU tests,
# decode timing fused vs three launches at 8,192 x 1 MiB, kernel trace and PMC
# passes of the fused decode, then the whole GPU suite.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-r04d}
mkdir -p "$OUT/pmc"
export TMPDIR=/tmp
echo "== RBC tests"
timeout -k 10 600 python -u -m pytest tests/test_gpu_rbc.py -m gpu -x -q --timeout 300 --timeout-method thread \
    > "$OUT/pytest_rbc.log" 2>&1 || { tail -40 "$OUT/pytest_rbc.log"; exit 2; }
tail -3 "$OUT/pytest_rbc.log"
echo "== decode timing"
timeout -k 10 300 python -u tools/kbench.py --what decode --instances 8192 --dec-fused 0,1 --splits -1 --reps 5 \
    > "$OUT/kbench.json" 2> "$OUT/kbench.err" || { tail -20 "$OUT/kbench.err"; exit 3; }
cat "$OUT/kbench.json"
KB="--what decode --instances 8192 --dec-fused 1 --splits -1 --reps 3"
echo "== decode kernel trace"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o dec -- \
    python3 tools/kbench.py $KB > "$OUT/trace.log" 2>&1 || { tail -20 "$OUT/trace.log"; exit 4; }
i=0
for group in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU" \
             "FETCH_SIZE" "WRITE_SIZE" "GRBM_GUI_ACTIVE GRBM_COUNT SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $group --output-format csv -d "$OUT/pmc/p$i" -o pmc -- python3 tools/kbench.py $KB \
      > "$OUT/pmc/p$i.log" 2>&1 || { echo "pmc pass $i failed"; tail -20 "$OUT/pmc/p$i.log"; exit 6; }
done
python3 tools/pmc_summary.py "$OUT/pmc" > "$OUT/pmc_summary.json"
python3 - "$OUT/pmc_summary.json" <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
for k, v in d.items():
    if v.get("avg_ms", 0) > 0.1:
        print(k[:40], round(v["avg_ms"], 2), "ms read", round(v.get("hbm_read_bytes_corrected", 0) / 1e9, 2),
              "GB write", round(v.get("hbm_write_bytes", 0) / 1e9, 2), "GB valu/wave", round(v.get("valu_insts_per_wave", 0)))
PY
[ -n "${SKIP_SUITE:-}" ] && { echo "== done (suite skipped)"; exit 0; }
echo "== full GPU suite"
timeout -k 10 1200 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread \
    > "$OUT/pytest.log" 2>&1 || { tail -40 "$OUT/pytest.log"; exit 5; }
tail -3 "$OUT/pytest.log"
echo "== done"
