#!/bin/bash
# A/B of the wave SHA3 theta (two gather stages vs one): long-V parity test and
# the configs[4] epoch leg with each build.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-r03o}
mkdir -p "$OUT"
export TMPDIR=/tmp
for lib in hydrabadger_amd/libhbgpu.so tools/libhbgpu_th1.so; do
  n=$(basename $lib .so)
  echo "== $lib"
  HBG_LIB_PATH=$PWD/$lib timeout -k 10 300 python -u -m pytest tests/test_gpu_bls_ops.py -m gpu -x -q -k long \
      --timeout 200 --timeout-method thread > "$OUT/pytest_$n.log" 2>&1 || { tail -30 "$OUT/pytest_$n.log"; exit 2; }
  tail -1 "$OUT/pytest_$n.log"
  HBG_LIB_PATH=$PWD/$lib timeout -k 10 300 python3 bench.py --steps 3 --warmup 1 --legs epoch --no-cpu --tdec-cts 0 \
      > "$OUT/bench_$n.json" 2> "$OUT/bench_$n.err" || { tail -30 "$OUT/bench_$n.err"; exit 3; }
  python3 -c "import json; d=json.load(open('$OUT/bench_$n.json')); e=d['network_epoch']; print(e['epoch_ms'], e['phases_ms']['propose_encode'], e['phases_ms']['tdec'], e['all_decrypted_ok'])"
done
echo "== done"
