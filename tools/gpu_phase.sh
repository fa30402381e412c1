#!/bin/bash
# Per-workgroup phase timing of the direct engine (tools/phase_probe.py; build the trace
# library first: bash tools/variant.sh trace -DTQ_PHASE_TRACE=1)
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; TAG=${1:-phase}; O=gpurun_out/$TAG; mkdir -p $O
export TQ_LIB_PATH=$R/term-quantization_amd/lib/libtq_hip_trace.so
for A in "2 --residual" "1" "6" "8 --residual"; do
  timeout -k 10 120 python tools/phase_probe.py --layer $A 2>>$O/err.log || { tail $O/err.log; exit 1; }
done | tee $O/phase.txt
unset TQ_LIB_PATH
for L in 2 1; do timeout -k 10 120 python tools/conv_probe.py --layer $L --codes 1 --config 10 $([ $L = 2 ] && echo --residual) --iters 20 2>>$O/err.log | tail -1; done
