#!/bin/bash
# Interleaved bench A/B of the default library against variant builds (TQ_LIB_PATH):
# Usage: bash tools/gpu_ab_lib.sh <tag> <rounds> <variant names...>   (lib/libtq_hip_<name>.so)
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; TAG=$1; N=$2; shift 2; O=gpurun_out/$TAG; mkdir -p $O
for i in $(seq 1 $N); do
  for v in default "$@"; do
    lib=""; [ "$v" != default ] && lib=$R/term-quantization_amd/lib/libtq_hip_$v.so
    TQ_LIB_PATH=$lib timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-d4 --no-d1 --no-stem-leg --steps 20 > $O/$v.$i.json 2> $O/$v.$i.err || { tail -5 $O/$v.$i.err; exit 1; }
    python3 -c "import json; d=json.loads(open('$O/$v.$i.json').read().strip().splitlines()[-1]); print('$v', $i, round(d['value']), 'conv', round(d['roofline']['avg_launch_us'],1), 'frac', round(d['roofline']['frac'],4), 'stem', round(d['roofline_tr']['avg_launch_us'],1))"
  done
done
