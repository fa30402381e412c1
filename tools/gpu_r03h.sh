#!/bin/bash
# r03h: LSTM branch-free step kernel; MobileNet-V2 fused line
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; TAG=${1:-r03h}; O=gpurun_out/$TAG; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_lstm.py tests/test_gpu_windows.py -m gpu -x -q --timeout 200 --timeout-method thread -k "lstm or pointwise" > $O/tests.log 2>&1
rc=$?; tail -1 $O/tests.log; [ $rc -ne 0 ] && { grep -E "FAIL|Error|assert" $O/tests.log | head -20; exit $rc; }
for v in "TQ_LSTM_SEQ=0" "TQ_LSTM_SEQ=1"; do
  env $v timeout -k 10 300 python3 tools/lstm_trace.py --chunks 20 > $O/lstm_$v.log 2>&1 || { tail $O/lstm_$v.log; exit 1; }
  echo "$v $(tail -1 $O/lstm_$v.log)"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/lstm_kt -o kt -- python3 tools/lstm_trace.py --chunks 10 > $O/lstm_kt.log 2>&1 || { tail $O/lstm_kt.log; exit 1; }
python3 - <<PY
import csv
rows=list(csv.DictReader(open('$O/lstm_kt/kt_kernel_stats.csv')))
for r in rows[:10]:
    print("%-80s %6s %9.1f us" % (r['Name'][:80], r['Calls'], float(r['AverageNs'])/1e3))
PY
bash tools/gpu_pmc.sh $TAG/dwpmc tools/dw_probe.py --c 144 --hw 56 --stride 1 --iters 20 || true
