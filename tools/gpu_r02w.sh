#!/bin/bash
# EfficientNet-b0 fused executor: parity tests (+ MBV2 / ResNet fused tests after the
# epilogue activation change), then the D4 bench.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; O=gpurun_out/r02w; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_fused_effnet.py tests/test_gpu_fused_mbv2.py tests/test_gpu_fused.py tests/test_gpu_models.py -x -v --timeout 300 --timeout-method thread > $O/t.log 2>&1; rc=$?
grep -E "PASS|FAIL|Error|assert" $O/t.log | tail -30; [ $rc -ne 0 ] && { tail -40 $O/t.log; exit $rc; }
timeout -k 10 600 python tools/bench_d4.py > $O/d4.log 2>&1; rc=$?; tail -3 $O/d4.log | cut -c1-600; exit $rc
