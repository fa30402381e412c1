#!/bin/bash
# SQ counter passes at HEAD (tools/gpu_pmc_cmd.sh, three passes each) of the layer-1 c64 convs
# (conv1 form: ReLU + codes; conv2 form: + residual + fp32 out + codes) and the fused stem.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; O=gpurun_out/sq_head; mkdir -p $O
bash tools/gpu_pmc_cmd.sh sq_c64_conv1 conv2d_tp_c64 "python3 tools/conv_probe.py --layer 1 --config 15 --codes 1 --no-out --nonneg --iters 5" > $O/c64_conv1.txt 2>&1 || exit 1
bash tools/gpu_pmc_cmd.sh sq_c64_conv2 conv2d_tp_c64 "python3 tools/conv_probe.py --layer 1 --config 15 --codes 1 --residual --nonneg --iters 5" > $O/c64_conv2.txt 2>&1 || exit 1
bash tools/gpu_pmc_cmd.sh sq_stem stem_conv_pool "python3 tools/stem_probe.py --iters 3" > $O/stem.txt 2>&1 || exit 1
for f in c64_conv1 c64_conv2 stem; do echo "== $f"; cat $O/$f.txt; done
