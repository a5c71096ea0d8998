#!/bin/bash
# Round 4, call q: the encoder's pre-store block prefetch (RBC tests, encode /
# decode timing, one SQ pass), then the TDec roofline inputs and the suite
# (tools/gpu_r04p.sh).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-r04q}
mkdir -p "$OUT"
export TMPDIR=/tmp
echo "== RBC tests"
timeout -k 10 600 python -u -m pytest tests/test_gpu_rbc.py -m gpu -x -q --timeout 300 --timeout-method thread \
    > "$OUT/pytest_rbc.log" 2>&1 || { tail -40 "$OUT/pytest_rbc.log"; exit 2; }
tail -2 "$OUT/pytest_rbc.log"
echo "== encode / decode timing"
timeout -k 10 300 python -u tools/kbench.py --what fused --instances 8192 --reps 5 > "$OUT/kbench_enc.json" 2> "$OUT/kbench_enc.err" \
    || { tail -20 "$OUT/kbench_enc.err"; exit 3; }
cat "$OUT/kbench_enc.json"
KB="--what fused --instances 8192 --reps 3"
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU \
    --output-format csv -d "$OUT/pmc_enc" -o pmc -- python3 tools/kbench.py $KB > "$OUT/pmc_enc.log" 2>&1 || { tail -20 "$OUT/pmc_enc.log"; exit 4; }
python3 - "$OUT" <<'PY'
import csv, glob, sys
f = glob.glob(f"{sys.argv[1]}/pmc_enc/**/pmc_counter_collection.csv", recursive=True)
acc = {}
for r in csv.DictReader(open(f[0])):
    if "rbc_encode_merkle" in r["Kernel_Name"]:
        acc.setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
w = sum(acc["SQ_WAVES"]) / len(acc["SQ_WAVES"])
print("encoder per wave", {k: round(sum(x) / len(x) / w) for k, x in acc.items()})
PY
TAG=${TAG:-r04q} bash tools/gpu_r04p.sh || exit $?
