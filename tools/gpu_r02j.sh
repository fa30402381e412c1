#!/bin/bash
# Stem with pre-split fp16 input planes: stem tests, then interleaved bench A/B vs the
# previous library (lib/libtq_hip_old.so).
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; O=gpurun_out/r02j; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_stem.py tests/test_gpu_fused_parity.py -x -q --timeout 120 --timeout-method thread > $O/t.log 2>&1; rc=$?; tail -2 $O/t.log; [ $rc -ne 0 ] && exit $rc
TAG=r02j R=3 STEPS=30 bash tools/gpu_ab2.sh
