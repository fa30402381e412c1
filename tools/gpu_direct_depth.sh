#!/bin/bash
# Direct-engine K-steps in flight (TQ_DIR_DEPTH variant builds dd3 / dd4 vs the product's 2):
# the stride-2 conv1 and the downsample convs of ResNet-18, and MobileNet-V2 / EfficientNet-b0
# 1x1 project shapes, interleaved, two rounds.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"
run() {
  for r in 1 2; do for v in default dd3 dd4; do
    lib=""; [ "$v" != default ] && lib=$R/term-quantization_amd/lib/libtq_hip_$v.so
    TQ_LIB_PATH=$lib timeout -k 10 120 python -u tools/conv_probe.py "$@" --iters 30 2>/dev/null | grep layer | sed "s/^/r$r $v $* /" || exit 1
  done; done
}
run --layer 5 --config 0 --codes 1 --no-out --nonneg
run --layer 7 --config 0 --no-relu --nonneg
run --layer 12 --config 0 --no-relu --nonneg
run --shape 144,24,1,1,56 --config 0 --codes 1 --no-relu
run --shape 576,96,1,1,14 --config 0 --codes 1 --no-relu
