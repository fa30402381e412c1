#!/bin/bash
# r03n: per-launch kernel traces of the fused MobileNet-V2 / EfficientNet-b0 executors
# (tools/bench_d4.py), and every MobileNet-V2 depthwise shape alone (tools/dw_probe.py).
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; TAG=${1:-r03n}; O=gpurun_out/$TAG; mkdir -p $O
export TMPDIR=/tmp
for M in mobilenet_v2 efficientnet_b0; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_$M -o kt -- \
      python3 tools/bench_d4.py --only $M --steps 3 --warmup 2 > $O/kt_$M.log 2>&1 || { tail $O/kt_$M.log; exit 1; }
  tail -2 $O/kt_$M.log
done
for A in "32 112 1" "96 112 2" "144 56 1" "144 56 2" "192 28 1" "192 28 2" "384 14 1" "576 14 1" "576 14 2" "960 7 1"; do
  set -- $A
  timeout -k 10 120 python tools/dw_probe.py --c $1 --hw $2 --stride $3 --iters 20 2>>$O/err.log | tail -1 || exit 1
done | tee $O/dw_probe.txt
