#!/bin/bash
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; TAG=${1:-r03ad}; O=gpurun_out/$TAG; mkdir -p $O
S=144,24,1,1,56
for A in "--no-out" "" "--no-relu" "--no-relu --no-out" "--residual" "--no-relu --residual" "--codes 0"; do
  echo -n "[$A] "; timeout -k 10 120 python tools/conv_probe.py --shape $S --codes 1 $A --iters 20 2>>$O/err.log | tail -1
done | tee $O/probe.txt
echo -n "[TQ_LUT=0 --no-relu] "; TQ_LUT=0 timeout -k 10 120 python tools/conv_probe.py --shape $S --codes 1 --no-relu --iters 20 2>>$O/err.log | tail -1
