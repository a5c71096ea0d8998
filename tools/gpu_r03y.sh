#!/bin/bash
# Round 3: latency-bound BLS kernels — serial-chain Fp multiplication (product)
# vs 3 interleaved accumulators (tools/libhbgpu_k3.so) on the epoch / f1 /
# coin / wire legs.
set -o pipefail
OUT=gpurun_out/${TAG:-r03y}
mkdir -p $OUT
ARGS="--steps 3 --warmup 1 --no-cpu --no-decode --legs epoch,f1,coin,wire --tdec-cts 0"
for i in 1; do
  timeout -k 10 400 python -u bench.py $ARGS > $OUT/k1_$i.json 2> $OUT/k1_$i.err || { tail -20 $OUT/k1_$i.err; exit 1; }
  HBG_LIB_PATH=tools/libhbgpu_k3.so timeout -k 10 400 python -u bench.py $ARGS > $OUT/k3_$i.json 2> $OUT/k3_$i.err || { tail -20 $OUT/k3_$i.err; exit 1; }
done
python - <<'PY'
import json
for tag in ("k1_1", "k3_1"):
    d = json.loads(open(f"gpurun_out/{__import__('os').environ.get('TAG','r03y')}/{tag}.json").read().strip().splitlines()[-1])
    e = d["network_epoch"]
    print(tag, "epoch", round(e["epoch_ms"], 1), {k: round(v, 1) for k, v in e["phases_ms"].items()})
    print(tag, "f1", {k: round(v, 1) for k, v in d["tdec_inputs"].items() if k.endswith("_ms") or k.endswith("per_s")})
    print(tag, "coin", {k: round(v) for k, v in d["coin"].items() if isinstance(v, float)})
    print(tag, "wire", {k: round(v) for k, v in d["wire_signatures"].items() if isinstance(v, float)})
PY
echo "== done"
