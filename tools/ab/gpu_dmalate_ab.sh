#!/bin/bash
# A/B of the ring engine's DMA placement (RING_DMA_LATE variant build vs the product build):
# ring parity tests on the variant, then interleaved tools/layer_times.py runs.
# Usage: bash tools/ab/gpu_dmalate_ab.sh <tag>   (variant: bash tools/ab/variant.sh dmalate ...)
set -u
TAG=${1:-dmalate}
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; O=gpurun_out/$TAG; mkdir -p $O
V=$R/term-quantization_amd/lib/libtq_hip_dmalate.so
TQ_LIB_PATH=$V timeout -k 10 300 python -u -m pytest tests/test_gpu_ring.py -x -q --timeout 120 \
    --timeout-method thread > $O/ring_variant.log 2>&1 || { tail -5 $O/ring_variant.log; exit 1; }
tail -1 $O/ring_variant.log
for i in 1 2 3; do
  timeout -k 10 120 python -u tools/layer_times.py --steps 5 > $O/base_$i.txt 2>&1 || exit 1
  TQ_LIB_PATH=$V timeout -k 10 120 python -u tools/layer_times.py --steps 5 > $O/late_$i.txt 2>&1 || exit 1
done
for f in $O/base_*.txt $O/late_*.txt; do
  echo "$(basename $f): $(awk 'NR>1 && $3 ~ /^[0-9.]+$/ {printf "%s ", $3}' $f) $(tail -1 $f)"
done
