#!/bin/bash
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; O=gpurun_out/r02n; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_fused_mbv2.py tests/test_gpu_models.py tests/test_gpu_fused.py -x -q --timeout 300 --timeout-method thread > $O/t.log 2>&1; rc=$?; tail -25 $O/t.log; exit $rc
