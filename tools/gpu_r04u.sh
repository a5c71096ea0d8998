#!/bin/bash
# Round 4, call u: A/B in one box of (a) the encoder's in-sweep payload
# prefetch + the decoder's pre-store block load (product library) against the
# committed schedule (tools/libhbgpu_abold.so: -DHBG_ENC_NO_SWEEP_PD
# -DHBG_DEC_NO_PRESTORE), and (b) SHA3(V) kernel times of the interleaved wave
# sponge against the round-3 sponge and the lane sponge.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-r04u}
mkdir -p "$OUT"
export TMPDIR=/tmp
P="--kernel-trace --stats --output-format csv"
echo "== SHA3(V) 128 x 1 MiB: interleaved sponge, then the round-3 sponge"
timeout -k 10 300 rocprofv3 $P -d "$OUT/sha3_new" -o run -- \
    python -u tools/sha3v_probe.py > "$OUT/sha3_new.json" 2> "$OUT/sha3_new.err" || { tail -20 "$OUT/sha3_new.err"; exit 3; }
cat "$OUT/sha3_new.json"
HBG_SHA3_WAVE64=1 timeout -k 10 300 rocprofv3 $P -d "$OUT/sha3_old" -o run -- \
    python -u tools/sha3v_probe.py > "$OUT/sha3_old.json" 2> "$OUT/sha3_old.err" || { tail -20 "$OUT/sha3_old.err"; exit 4; }
cat "$OUT/sha3_old.json"
echo "== SHA3(V) 16,384 x 64 KiB: lane sponge, then the interleaved wave sponge"
timeout -k 10 300 rocprofv3 $P -d "$OUT/sha3_tp_lane" -o run -- \
    python -u tools/sha3v_probe.py --n 16384 --len 65536 --reps 2 > "$OUT/sha3_tp_lane.json" 2> "$OUT/sha3_tp_lane.err" \
    || { tail -20 "$OUT/sha3_tp_lane.err"; exit 5; }
cat "$OUT/sha3_tp_lane.json"
HBG_VDIGEST_WAVE_MAX=100000 timeout -k 10 300 rocprofv3 $P -d "$OUT/sha3_tp_wave" -o run -- \
    python -u tools/sha3v_probe.py --n 16384 --len 65536 --reps 2 > "$OUT/sha3_tp_wave.json" 2> "$OUT/sha3_tp_wave.err" \
    || { tail -20 "$OUT/sha3_tp_wave.err"; exit 6; }
cat "$OUT/sha3_tp_wave.json"
for f in $(find "$OUT" -name '*kernel_stats.csv'); do echo "$f"; grep -h 'digest' "$f" | cut -c1-220 || true; done
echo "== encode / decode A/B (new = product, old = abold)"
for i in 1 2 3; do
for v in new old; do
if [ $v = old ]; then export HBG_LIB_PATH=tools/libhbgpu_abold.so; else unset HBG_LIB_PATH; fi
echo -n "$v "
timeout -k 10 300 python -u tools/kbench.py --what fused --instances 8192 --reps 10 2> "$OUT/kbench_enc.err" \
    || { tail -20 "$OUT/kbench_enc.err"; exit 7; }
echo -n "$v "
timeout -k 10 300 python -u tools/kbench.py --what decode --instances 8192 --dec-fused 1 --splits -1 --reps 5 \
    2> "$OUT/kbench_dec.err" || { tail -20 "$OUT/kbench_dec.err"; exit 8; }
done
done
echo "== done"
