#!/bin/bash
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; O=gpurun_out/r02o; mkdir -p $O
timeout -k 10 600 python tools/bench_d4.py > $O/d4.log 2>&1; rc=$?; tail -3 $O/d4.log | cut -c1-400; exit $rc
