#!/bin/bash
# Ring-engine rows-per-tile probe (TQ_RING_R): bash tools/gpu_ring_rows.sh "<layer:R,R..> ..."
# (TQ_RING_R was an A/B override, reverted after this probe: profiles/r05_ring_rows_probe.txt)
set -u
R0=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R0"
for spec in "$@"; do
  L=${spec%%:*}; RS=${spec#*:}
  for F in "--no-out" "--residual"; do
    for r in 0 ${RS//,/ }; do
      TQ_RING_R=$r timeout -k 10 120 python -u tools/conv_probe.py --layer $L --config 13 --codes 1 --nonneg $F --iters 30 2>/dev/null | grep layer | sed "s/^/$F R=$r /" || exit 1
    done
  done
done
