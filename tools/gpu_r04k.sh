#!/bin/bash
# Round 4, call k: fused-decoder diagnostics — the product library against
# variants without the payload stores (HBG_DEC_NO_PAYLOAD) and with
# default-policy stores (HBG_STORE_AUX=0): timing + one SQ counter pass each.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-r04k}
mkdir -p "$OUT"
export TMPDIR=/tmp
KB="--what decode --instances 8192 --dec-fused 1 --splits -1 --reps 3"
for v in product nopay st0; do
  if [ $v = product ]; then LIBP=""; else LIBP="$PWD/tools/libhbgpu_$v.so"; fi
  echo "== $v"
  HBG_LIB_PATH=$LIBP timeout -k 10 300 python3 tools/kbench.py $KB > "$OUT/kb_$v.json" 2> "$OUT/kb_$v.err" || { tail -20 "$OUT/kb_$v.err"; exit 2; }
  cat "$OUT/kb_$v.json"
  HBG_LIB_PATH=$LIBP timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU \
      --output-format csv -d "$OUT/pmc_$v" -o pmc -- python3 tools/kbench.py $KB > "$OUT/pmc_$v.log" 2>&1 || { tail -20 "$OUT/pmc_$v.log"; exit 3; }
done
python3 - "$OUT" <<'PY'
import csv, glob, sys
for v in ("product", "nopay", "st0"):
    f = glob.glob(f"{sys.argv[1]}/pmc_{v}/**/pmc_counter_collection.csv", recursive=True)
    acc = {}
    for r in csv.DictReader(open(f[0])):
        if "rbc_decode_merkle" not in r["Kernel_Name"]:
            continue
        acc.setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
    w = sum(acc["SQ_WAVES"]) / len(acc["SQ_WAVES"]) if acc.get("SQ_WAVES") else 1
    print(v, {k: round(sum(x) / len(x) / w) for k, x in acc.items()})
PY
echo "== done"
