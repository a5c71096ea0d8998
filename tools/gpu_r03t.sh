#!/bin/bash
# Round 3: reconstruct split schedule — parity tests, decode A/B, decode rocprof.
set -o pipefail
OUT=gpurun_out/${TAG:-r03t}
mkdir -p $OUT
echo "== pytest"
timeout -k 10 400 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu \
    tests/test_gpu_rbc.py > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
echo "== kbench decode A/B"
timeout -k 10 300 python -u tools/kbench.py --what decode --instances 2048 --reps 10 > $OUT/kbench.jsonl 2> $OUT/kbench.err || exit 1
timeout -k 10 300 python -u tools/kbench.py --what decode --nodes 16 --payload 65536 --instances 10000 --reps 10 >> $OUT/kbench.jsonl 2>> $OUT/kbench.err || exit 1
timeout -k 10 300 python -u tools/kbench.py --what decode --nodes 128 --instances 2048 --reps 5 >> $OUT/kbench.jsonl 2>> $OUT/kbench.err || exit 1
cat $OUT/kbench.jsonl
echo "== rocprof decode"
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o dec -- \
    python tools/kbench.py --what decode --instances 2048 --reps 5 > $OUT/prof.log 2>&1 || { tail -20 $OUT/prof.log; exit 1; }
find $OUT/prof -name "*kernel_stats.csv" | head -1 | xargs -I{} cp {} $OUT/decode_kernel_stats.csv
cut -d, -f1-4 $OUT/decode_kernel_stats.csv | head -12
echo "== done"
