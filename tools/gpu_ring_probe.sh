#!/bin/bash
# Ring-engine check: its GPU parity tests, then per-layer timings against the default engines
# for the two epilogue forms of the fused ResNet executor (fp32 out + residual + codes, and
# codes only).  Usage: bash tools/gpu_ring_probe.sh <tag> "<layers>"
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; TAG=${1:-ring}; LAYERS=${2:-"6 8 11 13 16 18"}
O=$R/gpurun_out/$TAG; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_ring.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log; [ $rc -ne 0 ] && exit $rc
for L in $LAYERS; do
  for F in "--residual" "--no-out"; do
    for C in 0 13; do
      timeout -k 10 120 python -u tools/conv_probe.py --layer $L --config $C --codes 1 $F --iters 30 2>/dev/null | grep layer | sed "s/^/$F /" || exit 1
    done
  done
done
