#!/bin/bash
# r03b: depthwise A/B (tools/gpu_dw_ab.sh), stem test + bench line (stem without scratch),
# LSTM-650 kernel trace.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; TAG=${1:-r03b}; O=gpurun_out/$TAG; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_stem.py tests/test_gpu_lstm.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/stem_tests.log 2>&1
rc=$?; tail -1 $O/stem_tests.log; [ $rc -ne 0 ] && { tail -30 $O/stem_tests.log; exit $rc; }
bash tools/gpu_dw_ab.sh $TAG/dw || exit $?
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-d4 --steps 20 > $O/bench.json 2> $O/bench.err || { tail $O/bench.err; exit 1; }
python3 -c "import json; d=json.loads(open('$O/bench.json').read().strip().splitlines()[-1]); print('bench', round(d['value']), 'conv', round(d['roofline']['avg_launch_us'],1), 'stem', round(d['roofline_tr']['avg_launch_us'],1))"
for v in "TQ_LSTM_SEQ=0" "TQ_LSTM_UPPER=miopen" "TQ_LSTM_SEQ=1"; do
  env $v timeout -k 10 300 python3 tools/lstm_trace.py --chunks 20 >> $O/lstm.log 2>&1 || { tail $O/lstm.log; exit 1; }
  echo "$v $(tail -1 $O/lstm.log)"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/lstm_kt -o kt -- python3 tools/lstm_trace.py --chunks 10 > $O/lstm_kt.log 2>&1 || { tail $O/lstm_kt.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/stem_kt -o kt -- python3 bench.py --no-cpu-baseline --no-d4 --no-d1 --steps 5 --warmup 2 --streams 1 --launch eager > $O/stem_kt.log 2>&1 || { tail $O/stem_kt.log; exit 1; }
echo done
