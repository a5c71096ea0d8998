#!/bin/bash
# Three-launch decoders at configs[1] and N = 128 with the product library (both splits).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/${TAG:-decnow}
mkdir -p "$OUT"
timeout -k 10 200 python3 tools/kbench.py --what decode --dec-fused 0 --splits 0,1 --nodes 16 --payload 65536 \
    --instances 10000 --reps 20 > "$OUT/16.json" 2>&1 || { tail -5 "$OUT/16.json"; exit 3; }
timeout -k 10 200 python3 tools/kbench.py --what decode --dec-fused 0 --splits 0,1 --nodes 128 --payload 1048576 \
    --instances 2048 --reps 5 > "$OUT/128.json" 2>&1 || { tail -5 "$OUT/128.json"; exit 4; }
timeout -k 10 200 python3 tools/kbench.py --what decode --dec-fused 0,1 --splits 1 --nodes 64 --payload 1048576 \
    --instances 2048 --reps 5 > "$OUT/64.json" 2>&1 || { tail -5 "$OUT/64.json"; exit 5; }
grep -h instances "$OUT"/*.json
