#!/bin/bash
# Round-5 GPU steps, one script (replaces the per-call gpu_r0*.sh scripts).
#   STEPS="tests smoke bench trace probe fpcount" TAG=r05a tools/gpu_r05.sh
# Each step runs under its own time limit; the script stops at the first
# failing step (no retries), output under gpurun_out/$TAG.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${TAG:-r05}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
STEPS=${STEPS:-"tests smoke bench"}
TESTS=${TESTS:-tests}

for s in $STEPS; do
    echo "== $s $(date +%T)"
    case $s in
    tests)
        timeout -k 10 900 python -u -m pytest $TESTS -m gpu -x -q --timeout 600 --timeout-method thread \
            > "$OUT/pytest.log" 2>&1 || { tail -40 "$OUT/pytest.log"; exit 2; }
        tail -2 "$OUT/pytest.log" ;;
    smoke)
        timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 \
            || { tail -20 "$OUT/smoke.log"; exit 3; }
        tail -1 "$OUT/smoke.log" ;;
    bench)
        timeout -k 10 600 python3 bench.py ${BENCH_ARGS:-} > "$OUT/bench.json" 2> "$OUT/bench.err" \
            || { tail -30 "$OUT/bench.err"; exit 4; }
        sleep 2
        ps -u "$(id -u)" -o pid,ppid,etime,cmd > "$OUT/ps_after.txt" 2>&1
        python3 tools/bench_summary.py "$OUT/bench.json" ;;
    trace)
        timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o bench -- \
            python3 bench.py --steps 5 --warmup 2 > "$OUT/trace_bench.json" 2> "$OUT/trace.err" \
            || { tail -20 "$OUT/trace.err"; exit 5; } ;;
    etrace)
        timeout -k 10 600 rocprofv3 --kernel-trace --output-format csv -d "$OUT/etrace" -o ep -- \
            python3 bench.py --steps 2 --warmup 1 --instances 512 --no-cpu --no-decode --legs ${ELEGS:-epoch} \
            > "$OUT/etrace_bench.json" 2> "$OUT/etrace.err" || { tail -20 "$OUT/etrace.err"; exit 8; }
        python3 tools/itemise_trace.py "$(ls "$OUT"/etrace/*/ep_kernel_trace.csv "$OUT"/etrace/ep_kernel_trace.csv 2>/dev/null | head -1)" \
            > "$OUT/epoch_itemised.txt" 2>&1 || true
        tail -40 "$OUT/epoch_itemised.txt"
        python3 tools/bench_summary.py "$OUT/etrace_bench.json" || true ;;
    probe)
        timeout -k 10 400 python3 -u tools/ctw_probe.py all ${PROBE_ARGS:-} > "$OUT/probe.log" 2>&1 \
            || { tail -60 "$OUT/probe.log"; exit 6; }
        tail -30 "$OUT/probe.log" ;;
    fpcount)
        timeout -k 10 400 python3 -u tools/fpcount.py run --n-ct 2048 --out "$OUT/fpcount.json" > "$OUT/fpcount.log" 2>&1 \
            || { tail -40 "$OUT/fpcount.log"; exit 7; }
        tail -c 600 "$OUT/fpcount.log" ;;
    *)
        echo "unknown step $s"; exit 9 ;;
    esac
done
echo "== done $(date +%T)"
