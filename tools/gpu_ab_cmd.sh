#!/bin/bash
# Interleaved A/B of variant builds (tools/variant1.sh) on one probe command, two rounds; the
# probe's last output line is recorded.  Usage: bash tools/gpu_ab_cmd.sh <tag> "<cmd>" <variant>...
set -u
TAG=$1; CMD=$2; shift 2
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; O=gpurun_out/$TAG; mkdir -p $O
export TMPDIR=/tmp
for round in 1 2; do
  for v in base "$@"; do
    if [ $v = base ]; then unset TQ_LIB_PATH; else export TQ_LIB_PATH=$R/term-quantization_amd/lib/libtq_hip_$v.so; fi
    r=$(timeout -k 10 120 $CMD 2>&1 | tail -1) || { echo "$v failed: $r"; exit 1; }
    echo "round $round $v: $r" | tee -a $O/ab.txt
  done
done
