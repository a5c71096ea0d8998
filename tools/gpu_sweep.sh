set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r01b
export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 -L > gpurun_out/r01b/counters.txt 2>&1
timeout -k 10 600 python tools/kbench.py --what merkle,encode,rs,decode --instances 1024,2048,3072,4096,5120,6144,8192 --reps 4 > gpurun_out/r01b/sweep.jsonl 2> gpurun_out/r01b/sweep.err || { tail gpurun_out/r01b/sweep.err; exit 3; }
cat gpurun_out/r01b/sweep.jsonl
TAG=r01b KB_ARGS="--what merkle,rs,encode --instances 4096 --reps 2" bash tools/pmc.sh
