#!/bin/bash
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; O=gpurun_out/r02l; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_lstm.py -x -q --timeout 120 --timeout-method thread > $O/t.log 2>&1; rc=$?; tail -15 $O/t.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python tools/bench_d4.py > $O/d4.log 2>&1; rc=$?; tail -3 $O/d4.log | cut -c1-700; exit $rc
