#!/bin/bash
# Kernel-level probes: VALU instruction rates, TR/conv microbench, SQ counters of the conv.
set -u
TAG=${1:-micro}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p "$O"
export TMPDIR=/tmp
cd "$R"
timeout -k 10 120 ./tools/valu_peak > "$O/valu_peak.txt" 2>&1; rc=$?
cat "$O/valu_peak.txt"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python tools/microbench.py > "$O/micro.txt" 2>&1; rc=$?
cat "$O/micro.txt"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_ANY --output-format csv -d "$O/sq" -o sq -- python3 "$R/tools/microbench.py" --iters 2 > "$O/sq.log" 2>&1; rc=$?
[ $rc -ne 0 ] && { tail -20 "$O/sq.log"; exit $rc; }
echo done
