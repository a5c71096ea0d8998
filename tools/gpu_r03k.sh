#!/bin/bash
# Round 3, call k: TDec schedule cutoff.  GPU tests of the TDec / coin / epoch
# paths (all schedules), batched-vs-per-share timing by size, Fp-mul counts of
# the batched schedule at 1 % and 0 % bad shares (instrumented build), and the
# tdec + epoch bench legs.  Each GPU step is time-limited; stops at the first
# failure.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-r03k}
mkdir -p "$OUT"
export TMPDIR=/tmp
echo "== pytest"
timeout -k 10 900 python -u -m pytest tests/test_gpu_tdec.py tests/test_gpu_async.py tests/test_gpu_bls_ops.py \
    tests/test_tdec_glue.py tests/test_epoch.py -m gpu -x -q --timeout 300 --timeout-method thread \
    > "$OUT/pytest.log" 2>&1 || { tail -40 "$OUT/pytest.log"; exit 2; }
tail -2 "$OUT/pytest.log"
echo "== schedule crossover"
timeout -k 10 600 python -u tools/tdec_sched.py --n-ct ${SCHED_SIZES:-512,2048,4096,6144,8192,12288} --reps 2 \
    > "$OUT/sched.jsonl" 2> "$OUT/sched.err" || { tail -20 "$OUT/sched.err"; exit 3; }
cat "$OUT/sched.jsonl"
echo "== fpcount"
timeout -k 10 300 python tools/fpcount.py run --n-ct 2048 --out "$OUT/fpcount.json" > "$OUT/fpcount.log" 2>&1 \
    || { tail -30 "$OUT/fpcount.log"; exit 4; }
timeout -k 10 300 python tools/fpcount.py run --n-ct 2048 --bad-rate 0 --out "$OUT/fpcount_min.json" \
    > "$OUT/fpcount_min.log" 2>&1 || { tail -30 "$OUT/fpcount_min.log"; exit 5; }
python -c "import json; a=json.load(open('$OUT/fpcount.json')); b=json.load(open('$OUT/fpcount_min.json')); print(a['per_share_total'], a['per_share_verify_total'], b['per_share_total'], b['per_share_verify_total'])"
echo "== bench tdec + epoch"
timeout -k 10 900 python -u bench.py --steps 3 --warmup 1 --legs tdec,epoch --no-cpu > "$OUT/bench.json" \
    2> "$OUT/bench.err" || { tail -30 "$OUT/bench.err"; exit 6; }
python -c "import json; d=json.load(open('$OUT/bench.json')); print(json.dumps({k: d[k] for k in ('tdec', 'network_epoch')})[:3000])"
echo "== done"
