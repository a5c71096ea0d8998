#!/bin/bash
# Round 3: PublicKeySet::decrypt as a bucket MSM (tdec_combine_msm) — parity
# tests, then the TDec + epoch legs against tools/libhbgpu_grp.so
# (tdec_combine_grp, the per-lane joint double-and-add).
set -o pipefail
OUT=gpurun_out/${TAG:-r03z}
mkdir -p $OUT
echo "== pytest"
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
    tests/test_gpu_tdec.py tests/test_tdec_glue.py tests/test_epoch.py tests/test_gpu_bls_ops.py > $OUT/pytest.log 2>&1 \
    || { tail -30 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
ARGS="--steps 3 --warmup 1 --no-cpu --no-decode --legs tdec,epoch"
timeout -k 10 400 python -u bench.py $ARGS > $OUT/msm.json 2> $OUT/msm.err || { tail -20 $OUT/msm.err; exit 1; }
HBG_LIB_PATH=tools/libhbgpu_grp.so timeout -k 10 400 python -u bench.py $ARGS > $OUT/grp.json 2> $OUT/grp.err || { tail -20 $OUT/grp.err; exit 1; }
echo "== rocprof msm"
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o msm -- \
    python3 bench.py $ARGS > $OUT/prof.json 2> $OUT/prof.err || { tail -20 $OUT/prof.err; exit 1; }
python - <<'PY'
import json, os
o = os.environ.get("TAG", "r03z")
for tag in ("msm", "grp"):
    d = json.loads(open(f"gpurun_out/{o}/{tag}.json").read().strip().splitlines()[-1])
    t = d["tdec"]; e = d["network_epoch"]
    print(tag, "tdec", round(t["value"]), round(t["threshold_decrypt_ms"], 1), "ok", t["ok_bits_match"], t["outcomes_match"], t["plaintexts_match"],
          "epoch", round(e["epoch_ms"], 1), round(e["phases_ms"]["tdec"], 1), d.get("leg_errors"))
PY
grep -h "combine" $OUT/prof/*kernel_stats.csv | cut -d, -f1-4 | cut -c1-160
echo "== done"
