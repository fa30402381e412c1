#!/bin/bash
# r03y: phase traces of MobileNet-V2 1x1 shapes on the direct engine
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; TAG=${1:-r03y}; O=gpurun_out/$TAG; mkdir -p $O
export TQ_LIB_PATH=$R/term-quantization_amd/lib/libtq_hip_trace.so
for A in "16,96,1,1,112" "144,24,1,1,56" "32,16,1,1,112" "96,576,1,1,14"; do
  timeout -k 10 120 python tools/phase_probe.py --shape $A --no-out 2>>$O/err.log || { tail $O/err.log; exit 1; }
done | tee $O/phase.txt
