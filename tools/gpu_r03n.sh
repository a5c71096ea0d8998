#!/bin/bash
# Round 3: wave-cooperative SHA3(V) (tdec_v_digest_wave) — the long-V / TDec /
# epoch GPU tests, then the epoch bench leg with a kernel trace.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-r03n}
mkdir -p "$OUT"
export TMPDIR=/tmp
echo "== pytest"
timeout -k 10 600 python -u -m pytest tests/test_gpu_bls_ops.py tests/test_epoch.py tests/test_tdec_glue.py tests/test_gpu_tdec.py \
    -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/pytest.log" 2>&1 || { tail -40 "$OUT/pytest.log"; exit 2; }
tail -2 "$OUT/pytest.log"
echo "== bench epoch"
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- \
    python3 bench.py --steps 3 --warmup 1 --legs epoch --no-cpu --tdec-cts 0 > "$OUT/bench.json" 2> "$OUT/bench.err" \
    || { tail -30 "$OUT/bench.err"; exit 6; }
python3 -c "import json; d=json.load(open('$OUT/bench.json')); e=d['network_epoch']; print(e['epoch_ms'], e['phases_ms'], e['all_decrypted_ok'])"
echo "== done"
