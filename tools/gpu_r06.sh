#!/bin/bash
# Round-6 GPU steps, one script (round 5's tools/gpu_r05.sh + the PMC /
# Fp-count re-measurement at HEAD, packed with the kernels' source digest).
#   STEPS="tests smoke bench trace pmcrbc pmctdec fpcount" TAG=r06x tools/gpu_r06.sh
# Packed profiles land in gpurun_out/$TAG/profiles/ (copy them into profiles/).
# Each step runs under its own time limit; the script stops at the first
# failing step (no retries), output under gpurun_out/$TAG.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${TAG:-r06}
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
        mkdir -p "$OUT/profiles/r06"
        timeout -k 10 400 python3 -u tools/fpcount.py run --n-ct 2048 --out "$OUT/profiles/fpcount.json" > "$OUT/fpcount.log" 2>&1 \
            || { tail -40 "$OUT/fpcount.log"; exit 7; }
        timeout -k 10 400 python3 -u tools/fpcount.py run --n-ct 2048 --bad-rate 0 \
            --out "$OUT/profiles/r06/fpcount_batched_0pct.json" > "$OUT/fpcount0.log" 2>&1 \
            || { tail -40 "$OUT/fpcount0.log"; exit 7; }
        tail -c 400 "$OUT/fpcount.log" ;;
    pmcrbc)
        # the fused encoder + the fused decode call at the bench shape (8,192 x 1 MiB, N = 64)
        TAG=$TAG/pmcrbc KB_ARGS="--what decode --dec-fused 1 --splits -1 --instances 8192 --reps 1" bash tools/pmc.sh \
            > "$OUT/pmcrbc.log" 2>&1 || { tail -30 "$OUT/pmcrbc.log"; exit 10; }
        OUT_ROOT="$OUT" python3 tools/pack_profiles.py rbc "gpurun_out/$TAG/pmcrbc/pmc/summary.txt" ;;
    pmcrbc2)
        # the two-launch schedule's kernels at the bench shape (after pmcrbc: updates its pmc_traffic.json)
        TAG=$TAG/pmcrbc2 KB_ARGS="--what encode --instances 8192 --reps 1" bash tools/pmc.sh \
            > "$OUT/pmcrbc2.log" 2>&1 || { tail -30 "$OUT/pmcrbc2.log"; exit 12; }
        OUT_ROOT="$OUT" python3 tools/pack_profiles.py rbc2 "gpurun_out/$TAG/pmcrbc2/pmc/summary.txt" ;;
    pmctdec)
        TAG=$TAG/pmctdec KB_ARGS="--cts 100000 --reps 1" EXTRA_GROUPS="FETCH_SIZE WRITE_SIZE" bash tools/pmc_tdec.sh \
            > "$OUT/pmctdec.log" 2>&1 || { tail -30 "$OUT/pmctdec.log"; exit 11; }
        OUT_ROOT="$OUT" python3 tools/pack_profiles.py tdec "gpurun_out/$TAG/pmctdec/summary.txt" ;;
    *)
        echo "unknown step $s"; exit 9 ;;
    esac
done
echo "== done $(date +%T)"
