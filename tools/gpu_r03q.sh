#!/bin/bash
# r03q: engine choice per ResNet-18 layer (conv_probe configs: 0 heuristic, 7/8 patch
# 128/64-row, 9/10 direct 128/64-row, 11 strip)
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; TAG=${1:-r03q}; O=gpurun_out/$TAG; mkdir -p $O
for A in "1:0 8 10 11" "2:0 8 10 11" "6:0 7 8 10" "8:0 7 8 10" "11:0 7 10" "13:0 7 10"; do
  L=${A%%:*}; CFGS=${A#*:}
  RES=""; case $L in 2|4|8|13|18) RES="--residual";; esac
  for C in $CFGS; do
    timeout -k 10 120 python tools/conv_probe.py --layer $L --codes 1 $RES --config $C --iters 20 2>>$O/err.log | tail -1 || echo "layer $L cfg $C failed"
  done
done | tee $O/engines.txt
