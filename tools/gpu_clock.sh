#!/bin/bash
# Effective clock (GRBM_GUI_ACTIVE / 8 / wall) of the Merkle kernel for both
# Keccak implementations and of the RS encode kernel, then bench kernel stats.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-r01g}
mkdir -p "$OUT"
export TMPDIR=/tmp
for impl in 0 1; do
  d="$OUT/clk$impl"; mkdir -p "$d"
  HBG_KECCAK_IMPL=$impl timeout -k 10 300 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAVES SQ_INSTS_VALU SQ_BUSY_CYCLES --output-format csv -d "$d" -o pmc -- \
     python3 tools/kbench.py --what merkle,encode --instances 4096 --reps 20 > "$d/log" 2>&1 || { tail -20 "$d/log"; exit 6; }
  python3 tools/pmc_summary.py "$d" > "$d/summary.json"; echo "impl=$impl"; cat "$d/summary.json"; cat "$d/log" | grep '^{'
done
echo "== rocprofv3 kernel stats (bench)"
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o bench -- \
    python3 bench.py --steps 10 --warmup 2 --no-cpu > "$OUT/prof.log" 2>&1 || { tail -20 "$OUT/prof.log"; exit 5; }
grep '^{' "$OUT/prof.log"
find "$OUT/prof" -name '*kernel_stats.csv' -exec cat {} \;
