#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-coinprof}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o coin -- \
  python3 bench.py --steps 2 --warmup 1 --instances 256 --no-cpu --no-decode --tdec-cts 0 --epoch-nodes 0 --wire-msgs 0 --f1-cts 0 > "$OUT/prof.log" 2>&1 || { tail -20 "$OUT/prof.log"; exit 5; }
python3 tools/trace_by_launch.py "$(find "$OUT/prof" -name '*kernel_trace.csv' | head -1)" > "$OUT/by_launch.csv"
head -20 "$OUT/by_launch.csv" | cut -c1-160
