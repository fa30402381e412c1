#!/bin/bash
# One GPU-box session: bench (JSON line), rocprofv3 kernel-trace/stats, and two separate PMC
# passes (FETCH_SIZE, WRITE_SIZE) of a short bench.  Outputs under gpurun_out/<tag>/.
# Usage: bash tools/gpu_profile.sh <tag> [bench args...]
set -u
TAG=${1:-r01}; shift || true
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p "$O"
export TMPDIR=/tmp
cd "$R"
echo "== bench"
timeout -k 10 600 python bench.py "$@" > "$O/bench.json" 2> "$O/bench.err"
rc=$?; if [ $rc -ne 0 ]; then echo "bench rc=$rc"; tail -20 "$O/bench.err"; exit $rc; fi
cat "$O/bench.json"
echo "== kernel trace"
# one stream, eager: the launches the bench's roofline pass times (its avg durations agree)
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/kt" -o kt -- \
    python3 "$R/bench.py" --steps 5 --warmup 2 --no-cpu-baseline --no-d1 --no-d4 --no-stem-leg --streams 1 --launch eager \
    > "$O/kt.log" 2>&1
rc=$?; if [ $rc -ne 0 ]; then echo "kt rc=$rc"; tail -20 "$O/kt.log"; exit $rc; fi
# the bench defaults (two chunk streams, hipGraph replay): the overlapped step timeline
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/kt2" -o kt -- \
    python3 "$R/bench.py" --steps 5 --warmup 2 --no-cpu-baseline --no-d1 --no-d4 --no-stem-leg > "$O/kt2.log" 2>&1
rc=$?; if [ $rc -ne 0 ]; then echo "kt2 rc=$rc"; tail -20 "$O/kt2.log"; exit $rc; fi
for C in FETCH_SIZE WRITE_SIZE; do
  echo "== pmc $C"
  timeout -k 10 600 rocprofv3 --pmc $C --output-format csv -d "$O/pmc_$C" -o pmc -- \
      python3 "$R/bench.py" --steps 2 --warmup 1 --no-cpu-baseline --no-d1 --no-d4 --no-stem-leg --streams 1 --launch eager \
      > "$O/pmc_$C.log" 2>&1
  rc=$?; if [ $rc -ne 0 ]; then echo "pmc $C rc=$rc"; tail -20 "$O/pmc_$C.log"; exit $rc; fi
done
find "$O" -name '*.csv' | head -20
echo done
