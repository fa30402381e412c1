#!/bin/bash
# Persistent LSTM seq2 launch: parity tests, then D4 LSTM tokens/s with TQ_LSTM_PERSIST 0 / 1
# (interleaved, two rounds) and a kernel trace of the persistent chunk.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; O=gpurun_out/lstmp; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_lstm.py > $O/tests.txt 2>&1
rc=$?; tail -12 $O/tests.txt; [ $rc -ne 0 ] && exit $rc
for r in 1 2; do
  for p in 0 1; do
    TQ_LSTM_PERSIST=$p timeout -k 10 300 python tools/bench_d4.py --lstm-trace 20 2>/dev/null | python3 -c "import sys,json; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('round $r persist $p', round(d['tokens_per_s']), round(d['ms_per_chunk'],4))" || exit 1
  done
done
bash tools/gpu_lstm_trace.sh lstmp_trace
