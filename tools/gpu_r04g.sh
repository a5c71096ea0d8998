#!/bin/bash
# Round 4, call g: the fused decoder (tests, timing, PMC) then the pairing-stage
# probe (Miller loop / final exponentiation / pairing kernel times and their
# Fp-multiplication counts).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-r04g}
mkdir -p "$OUT"
export TMPDIR=/tmp
TAG=${TAG:-r04g} SKIP_SUITE=1 bash tools/gpu_r04d.sh || exit $?
echo "== pairing probe (trace)"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/ptrace" -o pp -- \
    python3 tools/pairing_probe.py --n 65536 > "$OUT/pairing_probe.json" 2> "$OUT/pairing_probe.err" || { tail -20 "$OUT/pairing_probe.err"; exit 8; }
cat "$OUT/pairing_probe.json"
echo "== pairing probe (counts)"
HBG_LIB_PATH=tools/libhbgpu_fpcount.so timeout -k 10 300 python3 tools/pairing_probe.py --n 4096 --count \
    > "$OUT/pairing_count.json" 2> "$OUT/pairing_count.err" || { tail -20 "$OUT/pairing_count.err"; exit 9; }
cat "$OUT/pairing_count.json"
python3 - "$OUT/ptrace" <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/pp_kernel_trace.csv", recursive=True)
rows = [r for r in csv.DictReader(open(f[0])) if "tdec_test" in r["Kernel_Name"]]
for r in rows:
    print("tdec_test grid", r.get("Grid_Size", r.get("Grid_Size_X", "?")), "ms", (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6)
PY
echo "== done"
