#!/bin/bash
# SQ counters of the three conv engines at batch 256: strip (layer 1 conv1-style), direct
# (layer 2 = layer1 conv2 with residual + fp32 out + codes), patch (layer 16, conv1-style).
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"
bash tools/gpu_sq2.sh r02e_strip --layer 1 --codes 1 --no-out || exit $?
bash tools/gpu_sq2.sh r02e_direct --layer 2 --codes 1 --residual || exit $?
bash tools/gpu_sq2.sh r02e_patch --layer 16 --codes 1 --no-out || exit $?
