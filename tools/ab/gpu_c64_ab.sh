#!/bin/bash
# A/B of c64 engine variant builds (tools/ab/variant1.sh) on the layer-1 conv forms, interleaved,
# two rounds.  Usage: bash tools/ab/gpu_c64_ab.sh <tag> <variant>...
set -u
TAG=$1; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; O=gpurun_out/$TAG; mkdir -p $O
export TMPDIR=/tmp
FORMS=("--codes 1 --no-out" "--codes 1 --residual" "--codes 1 --residual --no-out")
for round in 1 2; do
  for i in 0 1 2; do
    for v in base "$@"; do
      if [ $v = base ]; then unset TQ_LIB_PATH; else export TQ_LIB_PATH=$R/term-quantization_amd/lib/libtq_hip_$v.so; fi
      r=$(timeout -k 10 120 python3 tools/conv_probe.py --layer 1 --nonneg --config 15 ${FORMS[$i]} --iters 30 2>&1 | tail -1) || { echo "$v failed: $r"; exit 1; }
      echo "round $round form $i $v: $r" | tee -a $O/ab.txt
    done
  done
done
