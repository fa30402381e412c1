#!/bin/bash
# One GPU-box session at round granularity: the full -m gpu suite, smoke, then
# tools/gpu_profile.sh (bench + kernel trace + FETCH/WRITE PMC passes).  Stops at the first
# failing step.  Usage: bash tools/gpu_round.sh <tag>
set -u
TAG=${1:-r02}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd "$R"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
    > "$O/gpu_tests.log" 2>&1
rc=$?; tail -5 "$O/gpu_tests.log"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1
rc=$?; cat "$O/smoke.log" | tail -3; [ $rc -ne 0 ] && exit $rc
bash tools/gpu_profile.sh "$TAG"
