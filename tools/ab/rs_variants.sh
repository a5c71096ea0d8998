#!/bin/bash
# A/B of encoder build variants (tools/build_variant.py libraries) with kbench.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/${TAG:-rsab}
mkdir -p "$OUT"
for v in product aux0 pf10 pf3; do
    if [ "$v" = product ]; then lib=hydrabadger_amd/libhbgpu.so; else lib=tools/libhbgpu_$v.so; fi
    HBG_LIB_PATH=$lib timeout -k 10 200 python3 tools/kbench.py --what rs,encode,fused --nodes 64 --payload 1048576 \
        --instances 8192 --reps 5 > "$OUT/$v.64.json" 2>&1 || { tail -5 "$OUT/$v.64.json"; exit 2; }
    HBG_LIB_PATH=$lib timeout -k 10 200 python3 tools/kbench.py --what rs,encode --nodes 16 --payload 65536 \
        --instances 10000 --reps 20 > "$OUT/$v.16.json" 2>&1 || { tail -5 "$OUT/$v.16.json"; exit 3; }
    echo "$v"; grep instances "$OUT/$v.64.json" "$OUT/$v.16.json"
done
