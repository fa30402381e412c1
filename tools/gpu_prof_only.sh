#!/bin/bash
# The profile half of tools/gpu_round.sh (kernel traces + PMC passes of the ResNet-18 bench
# only), without re-running the test suite.  Usage: bash tools/gpu_prof_only.sh <tag>
set -u
TAG=${1:-prof}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p "$O"
export TMPDIR=/tmp
cd "$R"
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/kt" -o kt -- \
    python3 "$R/bench.py" --steps 5 --warmup 2 --no-cpu-baseline --no-d1 --no-d4 --streams 1 --launch eager \
    > "$O/kt.log" 2>&1 || { tail -20 "$O/kt.log"; exit 1; }
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 600 rocprofv3 --pmc $C --output-format csv -d "$O/pmc_$C" -o pmc -- \
      python3 "$R/bench.py" --steps 2 --warmup 1 --no-cpu-baseline --no-d1 --no-d4 --streams 1 --launch eager \
      > "$O/pmc_$C.log" 2>&1 || { tail -20 "$O/pmc_$C.log"; exit 1; }
done
echo done
