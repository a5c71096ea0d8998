#!/bin/bash
# A/B of the store policy on the decoders (product build vs tools/libhbgpu_aux0.so).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/${TAG:-decab}
mkdir -p "$OUT"
for v in product aux0; do
    if [ "$v" = product ]; then lib=hydrabadger_amd/libhbgpu.so; else lib=tools/libhbgpu_$v.so; fi
    HBG_LIB_PATH=$lib timeout -k 10 200 python3 tools/kbench.py --what encode,fused,decode --dec-fused -1 --splits -1 \
        --nodes 64 --payload 1048576 --instances 8192 --reps 5 > "$OUT/$v.64.json" 2>&1 || { tail -5 "$OUT/$v.64.json"; exit 2; }
    HBG_LIB_PATH=$lib timeout -k 10 200 python3 tools/kbench.py --what encode,decode --dec-fused -1 --splits -1 \
        --nodes 16 --payload 65536 --instances 10000 --reps 20 > "$OUT/$v.16.json" 2>&1 || { tail -5 "$OUT/$v.16.json"; exit 3; }
    HBG_LIB_PATH=$lib timeout -k 10 200 python3 tools/kbench.py --what encode,decode --dec-fused -1 --splits -1 \
        --nodes 128 --payload 1048576 --instances 2048 --reps 5 > "$OUT/$v.128.json" 2>&1 || { tail -5 "$OUT/$v.128.json"; exit 4; }
    echo "$v"; grep -h instances "$OUT/$v.64.json" "$OUT/$v.16.json" "$OUT/$v.128.json"
done
