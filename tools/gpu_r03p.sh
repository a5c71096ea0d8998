#!/bin/bash
# Round 3: ct_verify forked onto the context's aux stream inside
# hbg_tdec_threshold_decrypt — TDec / glue / async / epoch GPU tests, then the
# epoch and TDec bench legs.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-r03p}
mkdir -p "$OUT"
export TMPDIR=/tmp
echo "== pytest"
timeout -k 10 600 python -u -m pytest tests/test_gpu_tdec.py tests/test_tdec_glue.py tests/test_gpu_async.py tests/test_epoch.py \
    tests/test_gpu_bls_ops.py -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/pytest.log" 2>&1 \
    || { tail -40 "$OUT/pytest.log"; exit 2; }
tail -2 "$OUT/pytest.log"
echo "== bench epoch + tdec"
timeout -k 10 600 python3 bench.py --steps 3 --warmup 1 --legs epoch,tdec --no-cpu > "$OUT/bench.json" 2> "$OUT/bench.err" \
    || { tail -30 "$OUT/bench.err"; exit 6; }
python3 -c "import json; d=json.load(open('$OUT/bench.json')); e=d['network_epoch']; t=d['tdec']; print(e['epoch_ms'], e['phases_ms'], e['all_decrypted_ok']); print(t['value'], t['threshold_decrypt_ms'], t['ok_bits_match'], t['outcomes_match'], t['plaintexts_match'])"
echo "== done"
