#!/bin/bash
# A/B: where Ciphertext::verify (aux stream) starts inside ThresholdDecrypt:
# with the batch round (product), after it (ctv1), after the first binary round (ctv2).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/${TAG:-ctv}
mkdir -p "$OUT"
for v in product ctv1 ctv2; do
    if [ "$v" = product ]; then lib=hydrabadger_amd/libhbgpu.so; else lib=tools/libhbgpu_$v.so; fi
    HBG_LIB_PATH=$lib timeout -k 10 300 python3 tools/tdec_kbench.py --cts 100000 --reps 2 > "$OUT/$v.100k.json" 2>&1 \
        || { tail -5 "$OUT/$v.100k.json"; exit 3; }
    HBG_LIB_PATH=$lib timeout -k 10 300 python3 tools/tdec_kbench.py --cts 16384 --reps 3 > "$OUT/$v.16k.json" 2>&1 \
        || { tail -5 "$OUT/$v.16k.json"; exit 4; }
    echo "$v"; python3 -c "
import json,sys
for f in sys.argv[1:]:
    d=json.loads(open(f).read().strip().splitlines()[-1]); print(f, round(d['threshold_decrypt_ms'],1), round(d['verify_ms'],1), d['ok_bits_match'], d['plaintexts_match'], d['outcomes_match'])" "$OUT/$v.100k.json" "$OUT/$v.16k.json"
done
