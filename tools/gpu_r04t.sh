#!/bin/bash
# Round 4, call t: encoder in-sweep payload prefetch + decoder pre-store block
# load (RBC tests + timing) and the bit-interleaved SHA3(V) wave sponge
# (long-contribution test + A/B timing of 128 x 1 MiB against the round-3
# sponge).  The throughput-build TDec probe runs last.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-r04t}
mkdir -p "$OUT"
export TMPDIR=/tmp
echo "== RBC tests + long-contribution SHA3(V) test"
timeout -k 10 600 python -u -m pytest tests/test_gpu_rbc.py tests/test_gpu_bls_ops.py -m gpu -x -q --timeout 300 \
    --timeout-method thread > "$OUT/pytest_rbc_bls.log" 2>&1 || { tail -40 "$OUT/pytest_rbc_bls.log"; exit 2; }
tail -2 "$OUT/pytest_rbc_bls.log"
echo "== SHA3(V) 128 x 1 MiB: interleaved sponge, then the round-3 sponge"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/sha3_new" -o run -- \
    python -u tools/sha3v_probe.py > "$OUT/sha3_new.json" 2> "$OUT/sha3_new.err" || { tail -20 "$OUT/sha3_new.err"; exit 3; }
cat "$OUT/sha3_new.json"
HBG_SHA3_WAVE64=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/sha3_old" -o run -- \
    python -u tools/sha3v_probe.py > "$OUT/sha3_old.json" 2> "$OUT/sha3_old.err" || { tail -20 "$OUT/sha3_old.err"; exit 4; }
cat "$OUT/sha3_old.json"
echo "== SHA3(V) 16,384 x 64 KiB (the per-node epoch's item count): lane sponge, then the interleaved wave sponge"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/sha3_tp_lane" -o run -- \
    python -u tools/sha3v_probe.py --n 16384 --len 65536 --reps 2 > "$OUT/sha3_tp_lane.json" 2> "$OUT/sha3_tp_lane.err" \
    || { tail -20 "$OUT/sha3_tp_lane.err"; exit 3; }
HBG_VDIGEST_WAVE_MAX=100000 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/sha3_tp_wave" -o run -- \
    python -u tools/sha3v_probe.py --n 16384 --len 65536 --reps 2 > "$OUT/sha3_tp_wave.json" 2> "$OUT/sha3_tp_wave.err" \
    || { tail -20 "$OUT/sha3_tp_wave.err"; exit 3; }
for f in $(find "$OUT"/sha3_* -name '*kernel_stats.csv'); do echo "$f"; grep -h digest "$f" | cut -c1-200; done
echo "== encode / decode timing"
for i in 1 2; do
timeout -k 10 300 python -u tools/kbench.py --what fused --instances 8192 --reps 10 2> "$OUT/kbench_enc.err" \
    || { tail -20 "$OUT/kbench_enc.err"; exit 5; }
done
timeout -k 10 300 python -u tools/kbench.py --what decode --instances 8192 --dec-fused 1 --splits -1 --reps 5 2> "$OUT/kbench_dec.err" \
    || { tail -20 "$OUT/kbench_dec.err"; exit 6; }
echo "== throughput-build TDec probe (2,048 ct, every launch on the throughput build)"
timeout -k 10 300 python -u tools/tdec_throughput_probe.py --n-ct 2048 > "$OUT/probe.json" 2> "$OUT/probe.err" \
    || { tail -20 "$OUT/probe.err"; exit 7; }
cat "$OUT/probe.json"
echo "== done"
