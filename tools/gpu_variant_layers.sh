#!/bin/bash
# Parity + per-layer timing of one variant build against the product build:
#   bash tools/gpu_variant_layers.sh <tag> <variant> [pytest files...]
# runs the given GPU tests under the variant (TQ_LIB_PATH), then tools/layer_times.py twice
# per build, interleaved; outputs under gpurun_out/<tag>/.
set -u
TAG=$1; V=$2; shift 2
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; O=gpurun_out/$TAG; mkdir -p $O
export TMPDIR=/tmp
VL=$R/term-quantization_amd/lib/libtq_hip_$V.so
if [ $# -gt 0 ]; then
  TQ_LIB_PATH=$VL timeout -k 10 600 python -u -m pytest -x -q --timeout 120 \
    --timeout-method thread "$@" > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
  tail -2 $O/tests.txt
fi
for round in 1 2; do
  timeout -k 10 180 python tools/layer_times.py --steps 5 > $O/base_$round.txt 2>&1 || exit 1
  TQ_LIB_PATH=$VL timeout -k 10 180 python tools/layer_times.py --steps 5 > $O/${V}_$round.txt 2>&1 || exit 1
done
paste $O/base_2.txt $O/${V}_2.txt | tail -40
