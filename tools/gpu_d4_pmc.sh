#!/bin/bash
# Kernel trace + HBM counters of the fused MobileNet-V2 / EfficientNet-b0 executors
# (tools/bench_d4.py --fused-only): one rocprofv3 run for the trace, one per counter
# (FETCH_SIZE and WRITE_SIZE cannot share a pass), then per-kernel averages.
# Usage: bash tools/gpu_d4_pmc.sh <tag>
set -u
TAG=${1:-d4pmc}
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; O=gpurun_out/$TAG; mkdir -p $O
export TMPDIR=/tmp
for A in mobilenet_v2 efficientnet_b0; do
  timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$A/trace -o t -- \
      python3 tools/bench_d4.py --fused-only $A --steps 3 --warmup 1 > $O/$A.trace.log 2>&1 \
      || { tail -5 $O/$A.trace.log; exit 1; }
  for C in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 240 rocprofv3 --pmc $C --output-format csv -d $O/$A/$C -o p -- \
        python3 tools/bench_d4.py --fused-only $A --steps 3 --warmup 1 > $O/$A.$C.log 2>&1 \
        || { tail -5 $O/$A.$C.log; exit 1; }
  done
done
python3 tools/d4_pmc_report.py $O
