#!/bin/bash
# Round 4, call v: the interleaved SHA3(V) sponge with theta in one gather
# stage (13 gathers, two stages per round; the product default) against two
# stages (9 gathers, three stages: HBG_SHA3_3STAGE=1); RBC + BLS-ops tests on
# the reverted encoder / decoder schedule.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-r04v}
mkdir -p "$OUT"
export TMPDIR=/tmp
P="--kernel-trace --stats --output-format csv"
echo "== RBC + BLS-ops tests"
timeout -k 10 600 python -u -m pytest tests/test_gpu_rbc.py tests/test_gpu_bls_ops.py -m gpu -x -q --timeout 300 \
    --timeout-method thread > "$OUT/pytest_rbc_bls.log" 2>&1 || { tail -40 "$OUT/pytest_rbc_bls.log"; exit 2; }
tail -2 "$OUT/pytest_rbc_bls.log"
for v in 2 3 2 3; do
if [ $v = 3 ]; then export HBG_SHA3_3STAGE=1; else unset HBG_SHA3_3STAGE; fi
timeout -k 10 300 rocprofv3 $P -d "$OUT/sha3_s$v" -o run$v -- \
    python -u tools/sha3v_probe.py > "$OUT/sha3_s$v.json" 2> "$OUT/sha3_s$v.err" || { tail -20 "$OUT/sha3_s$v.err"; exit 3; }
echo -n "stages=$v "; cat "$OUT/sha3_s$v.json"
grep -h 'digest_wave' "$OUT/sha3_s$v/run${v}_kernel_stats.csv" | cut -c1-220 || true
done
echo "== done"
