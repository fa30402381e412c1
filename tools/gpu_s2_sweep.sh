#!/bin/bash
# MFMA config sweep of the ResNet-18 stride-2 convs at the bench batch (conv1 form: ReLU +
# codes; downsample form: fp32 out, no activation).  Usage: bash tools/gpu_s2_sweep.sh
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"
for L in 5 10 15; do
  for C in 0 1 2 3 4 5 6 9 10; do
    timeout -k 10 120 python -u tools/conv_probe.py --layer $L --config $C --codes 1 --no-out --nonneg --iters 20 2>/dev/null | grep layer || echo "layer $L cfg $C failed"
  done
done
for L in 7 12 17; do
  for C in 0 1 2 3 4 5 6 9 10 12; do
    timeout -k 10 120 python -u tools/conv_probe.py --layer $L --config $C --no-relu --nonneg --iters 20 2>/dev/null | grep layer || echo "layer $L cfg $C failed"
  done
done
