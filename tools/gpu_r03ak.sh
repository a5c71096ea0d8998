#!/bin/bash
# Round 3 re-entry, one call: (1) the locate-round TDec checks (tools/gpu_r03aj.sh),
# (2) full validation of the tree (tools/gpu_r03v.sh: whole GPU suite, smoke,
# default bench line, rocprofv3 kernel stats), (3) the TDec PMC passes at
# configs[3] size (tools/gpu_r03c.sh).  Stops at the first failing step.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${TAG:-r03ak}
TAG=${TAG}_tdec bash tools/gpu_r03aj.sh || exit 1
TAG=$TAG NO_PROF=${NO_PROF:-} bash tools/gpu_r03v.sh || exit 2
TAG=${TAG}_pmc CTS=100000 bash tools/gpu_r03c.sh || exit 3
echo "== all done"
