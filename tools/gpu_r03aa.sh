#!/bin/bash
# Round 3: TDec parity at head + Fp-multiplication counts of the MSM combine
# (instrumented tools/libhbgpu_fpcount.so), 1 % and 0 % bad shares.
set -o pipefail
OUT=gpurun_out/${TAG:-r03aa}
mkdir -p $OUT
echo "== pytest"
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
    tests/test_gpu_tdec.py tests/test_tdec_glue.py tests/test_gpu_async.py > $OUT/pytest.log 2>&1 \
    || { tail -30 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
echo "== fpcount"
timeout -k 10 300 python tools/fpcount.py run --n-ct 2048 --out "$OUT/fpcount.json" > "$OUT/fpcount.log" 2>&1 \
    || { tail -30 "$OUT/fpcount.log"; exit 4; }
timeout -k 10 300 python tools/fpcount.py run --n-ct 2048 --bad-rate 0 --out "$OUT/fpcount_min.json" \
    > "$OUT/fpcount_min.log" 2>&1 || { tail -30 "$OUT/fpcount_min.log"; exit 5; }
python -c "
import json
for f in ('fpcount', 'fpcount_min'):
    d = json.load(open('$OUT/' + f + '.json'))
    print(f, round(d['per_share_total'], 1), {k: round(v['per_share'], 1) for k, v in d['kernels'].items()})
"
echo "== done"
