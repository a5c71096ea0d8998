#!/bin/bash
# Round 3: latency build at 1 wave/SIMD register budget (tools/libhbgpu_latwpe1.so,
# dispatch up to 65,536 lanes) against the product latency build.
set -o pipefail
OUT=gpurun_out/${TAG:-r03ag}
mkdir -p $OUT
ARGS="--steps 3 --warmup 1 --no-cpu --no-decode --legs epoch,f1,wire --tdec-cts 0"
timeout -k 10 400 python -u bench.py $ARGS > $OUT/base.json 2> $OUT/base.err || { tail -20 $OUT/base.err; exit 1; }
HBG_LIB_PATH=tools/libhbgpu_latwpe1.so HBG_LAT_LANES=65536 timeout -k 10 400 python -u bench.py $ARGS > $OUT/wpe1.json 2> $OUT/wpe1.err || { tail -20 $OUT/wpe1.err; exit 1; }
python - <<'PY'
import json, os
o = os.environ.get("TAG", "r03ag")
for tag in ("base", "wpe1"):
    d = json.loads(open(f"gpurun_out/{o}/{tag}.json").read().strip().splitlines()[-1])
    e = d["network_epoch"]; f = d["tdec_inputs"]; w = d["wire_signatures"]
    print(tag, "epoch", round(e["epoch_ms"], 1), {k: round(v, 1) for k, v in e["phases_ms"].items()}, e["all_decrypted_ok"])
    print(tag, "f1 enc/s", round(f["encrypt_per_s"]), "wire sign/verify", round(w["sign_per_s"]), round(w["verify_per_s"]), d.get("leg_errors"))
PY
echo "== done"
