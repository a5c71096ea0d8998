#!/bin/bash
# A/B of the run-time coder's input load-ahead (HBG_IN_AHEAD) on the
# three-launch decoders (configs[1] N = 16, N = 128).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/${TAG:-movab}
mkdir -p "$OUT"
for v in product ia2 ia8; do
    if [ "$v" = product ]; then lib=hydrabadger_amd/libhbgpu.so; else lib=tools/libhbgpu_$v.so; fi
    HBG_LIB_PATH=$lib timeout -k 10 200 python3 tools/kbench.py --what decode --dec-fused 0 --splits 0,1 \
        --nodes 16 --payload 65536 --instances 10000 --reps 20 > "$OUT/$v.16.json" 2>&1 || { tail -5 "$OUT/$v.16.json"; exit 3; }
    HBG_LIB_PATH=$lib timeout -k 10 200 python3 tools/kbench.py --what decode --dec-fused 0 --splits 0,1 \
        --nodes 128 --payload 1048576 --instances 2048 --reps 5 > "$OUT/$v.128.json" 2>&1 || { tail -5 "$OUT/$v.128.json"; exit 4; }
    echo "$v"; grep -h instances "$OUT/$v.16.json" "$OUT/$v.128.json"
done
