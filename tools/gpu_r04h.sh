#!/bin/bash
# Round 4, call h: the driver's bench command, what outlives it, and a
# kernel-trace profile of the same command (profiles/r04/bench_*).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-r04h}
mkdir -p "$OUT"
export TMPDIR=/tmp
echo "== bench"
ps -u "$(id -u)" -o pid,ppid,etime,cmd > "$OUT/ps_before.txt" 2>&1
timeout -k 10 600 python3 bench.py --gpus 1 --steps 20 --warmup 5 > "$OUT/bench.json" 2> "$OUT/bench.err" || { tail -30 "$OUT/bench.err"; exit 2; }
tail -c 3000 "$OUT/bench.json"
sleep 2
echo "== processes after bench"
ps -u "$(id -u)" -o pid,ppid,etime,cmd > "$OUT/ps_after.txt" 2>&1
cat "$OUT/ps_after.txt"
echo "== bench kernel trace"
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o bench -- \
    python3 bench.py --gpus 1 --steps 5 --warmup 2 > "$OUT/trace_bench.json" 2> "$OUT/trace.err" || { tail -20 "$OUT/trace.err"; exit 3; }
echo "== done"
