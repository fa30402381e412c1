#!/bin/bash
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; TAG=${1:-r03ae}; O=gpurun_out/$TAG; mkdir -p $O
for A in "32 112 1" "144 56 1" "192 28 1" "384 14 1" "576 14 1" "960 7 1" "96 112 2" "144 56 2" "192 28 2" "576 14 2"; do
  set -- $A
  for M in 1 6 4 2 0; do
    [ $3 = 1 ] && [ $M = 2 ] && continue
    [ $3 = 2 ] && { [ $M = 6 ] || [ $M = 4 ]; } && continue
    echo -n "stream=$M "
    TQ_DW_STREAM=$M timeout -k 10 120 python tools/dw_probe.py --c $1 --hw $2 --stride $3 --iters 20 2>>$O/err.log | tail -1 || exit 1
  done
done | tee $O/dw_probe.txt
