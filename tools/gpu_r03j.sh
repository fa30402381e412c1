#!/bin/bash
# r03j: direct-engine ablations + PMC on ResNet-18 layer 8 (conv2-style)
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; TAG=${1:-r03j}; O=gpurun_out/$TAG; mkdir -p $O
export TMPDIR=/tmp
bash tools/gpu_ablate_direct.sh $TAG/abl > $O/abl.log 2>&1 || { tail $O/abl.log; exit 1; }
cat $O/abl.log
TQ_STRIP=0 bash tools/gpu_pmc.sh $TAG/pmc8 tools/conv_probe.py --layer 8 --codes 1 --residual || true
