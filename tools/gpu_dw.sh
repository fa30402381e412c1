#!/bin/bash
# Depthwise kernels: bit-identity tests, every MobileNet-V2 shape, fused D4 images/s
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; TAG=${1:-dw}; O=gpurun_out/$TAG; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_models.py tests/test_gpu_fused_effnet.py tests/test_gpu_fused_mbv2.py \
    -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
bash tools/gpu_d4.sh 2>>$O/err.log | tail -2 | tee $O/d4.txt
TQ_DW_STREAM5=1 bash tools/gpu_d4.sh 2>>$O/err.log | tail -1 | sed "s/^/stream5 /" | tee -a $O/d4.txt
