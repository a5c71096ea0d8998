#!/bin/bash
# Round 3: BLS latency build (tdec_kernels_lat.hip) — full GPU suite (the BLS
# tests run on both builds), then the BLS legs with the default dispatch
# against the throughput build only (HBG_LAT_LANES=0).
set -o pipefail
OUT=gpurun_out/${TAG:-r03ae}
mkdir -p $OUT
echo "== pytest"
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > $OUT/pytest.log 2>&1 \
    || { tail -30 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
ARGS="--steps 3 --warmup 1 --no-cpu --no-decode --legs tdec,epoch,f1,coin,wire"
timeout -k 10 400 python -u bench.py $ARGS > $OUT/lat.json 2> $OUT/lat.err || { tail -20 $OUT/lat.err; exit 1; }
HBG_LAT_LANES=0 timeout -k 10 400 python -u bench.py $ARGS > $OUT/thr.json 2> $OUT/thr.err || { tail -20 $OUT/thr.err; exit 1; }
python - <<'PY'
import json, os
o = os.environ.get("TAG", "r03ae")
for tag in ("lat", "thr"):
    d = json.loads(open(f"gpurun_out/{o}/{tag}.json").read().strip().splitlines()[-1])
    t = d["tdec"]; e = d["network_epoch"]; f = d["tdec_inputs"]; c = d["coin"]; w = d["wire_signatures"]
    print(tag, "tdec", round(t["value"]), t["ok_bits_match"] and t["outcomes_match"] and t["plaintexts_match"],
          "epoch", round(e["epoch_ms"], 1), {k: round(v, 1) for k, v in e["phases_ms"].items()})
    print(tag, "f1 enc/s", round(f["encrypt_per_s"]), "dec/s", round(f["decrypt_shares_per_s"]),
          "wire sign/verify", round(w["sign_per_s"]), round(w["verify_per_s"]),
          "coin sign/verify/combine", round(c["share_sign_per_s"]), round(c["share_verify_per_s"]), round(c["combine_coins_per_s"]),
          d.get("leg_errors"))
PY
echo "== done"
