#!/bin/bash
# rocprofv3 kernel trace of the term-pair LSTM-650 chunk (BASELINE configs[2]):
#   bash tools/gpu_lstm_trace.sh <tag>   -> gpurun_out/<tag>/ (trace, stats, window, summary)
set -eu
TAG=$1
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; O=$R/gpurun_out/$TAG; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv \
  -- python3 tools/bench_d4.py --lstm-trace 20 > $O/window.json 2> $O/prof.log
T=$(find $O/prof -name 'run_kernel_trace.csv' | sort | tail -n 1)
S=$(find $O/prof -name 'run_kernel_stats.csv' | sort | tail -n 1)
cp $T $O/kernel_trace.csv; cp $S $O/kernel_stats.csv
python3 tools/trace_window.py $O/kernel_trace.csv $O/window.json $O/chunk.txt
