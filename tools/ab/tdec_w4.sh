#!/bin/bash
# ThresholdDecrypt tests + timing (configs[3] size and the epoch size) on the product library.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/${TAG:-w4}
mkdir -p "$OUT"
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_tdec.py tests/test_tdec_glue.py tests/test_gpu_bls_ops.py -m gpu -x -q \
    --timeout 300 --timeout-method thread > "$OUT/pytest.log" 2>&1 || { tail -30 "$OUT/pytest.log"; exit 2; }
tail -2 "$OUT/pytest.log"
timeout -k 10 300 python3 tools/tdec_kbench.py --cts 100000 --reps 2 > "$OUT/100k.json" 2>&1 || { tail -5 "$OUT/100k.json"; exit 3; }
timeout -k 10 300 python3 tools/tdec_kbench.py --cts 16384 --reps 3 > "$OUT/16k.json" 2>&1 || { tail -5 "$OUT/16k.json"; exit 4; }
python3 -c "
import json,sys
for f in sys.argv[1:]:
    d=json.loads(open(f).read().strip().splitlines()[-1]); print(f, round(d['threshold_decrypt_ms'],1), round(d['verify_ms'],1), d['ok_bits_match'], d['plaintexts_match'], d['outcomes_match'])" "$OUT/100k.json" "$OUT/16k.json"
