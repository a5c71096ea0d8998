#!/bin/bash
# Round 4, call w: validation of HEAD — the whole GPU suite, smoke(), the
# driver's default bench command (and what outlives it), and a kernel-trace
# profile of a shorter bench run.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-r04w}
mkdir -p "$OUT"
export TMPDIR=/tmp
echo "== full GPU suite"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread \
    > "$OUT/pytest.log" 2>&1 || { tail -40 "$OUT/pytest.log"; exit 2; }
tail -2 "$OUT/pytest.log"
echo "== smoke"
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > "$OUT/smoke.log" 2>&1 \
    || { tail -20 "$OUT/smoke.log"; exit 3; }
tail -1 "$OUT/smoke.log"
echo "== bench (driver default)"
timeout -k 10 600 python3 bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" || { tail -30 "$OUT/bench.err"; exit 4; }
sleep 2
ps -u "$(id -u)" -o pid,ppid,etime,cmd > "$OUT/ps_after.txt" 2>&1
python3 - "$OUT/bench.json" <<'EOF'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print("headline", round(d["value"], 1), d["unit"], round(d["ms_per_step"], 2), "ms", "frac", round(d["roofline"]["frac"], 3))
for k in ("decode", "tdec", "network_epoch", "config1_n16"):
    v = d.get(k)
    if isinstance(v, dict):
        print(k, {a: b for a, b in v.items() if isinstance(b, (int, float, bool, str)) and len(str(b)) < 40})
print("leg_errors", d.get("leg_errors"))
EOF
echo "== bench kernel trace"
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o bench -- \
    python3 bench.py --steps 5 --warmup 2 > "$OUT/trace_bench.json" 2> "$OUT/trace.err" || { tail -20 "$OUT/trace.err"; exit 5; }
echo "== done"
