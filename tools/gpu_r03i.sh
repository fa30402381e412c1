#!/bin/bash
# r03i: LSTM step kernel with batched staging
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; TAG=${1:-r03i}; O=gpurun_out/$TAG; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_lstm.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -1 $O/tests.log; [ $rc -ne 0 ] && { grep -E "FAIL|Error|assert" $O/tests.log | head -20; exit $rc; }
for v in "TQ_LSTM_SEQ=1"; do
  env $v timeout -k 10 300 python3 tools/lstm_trace.py --chunks 20 > $O/lstm_$v.log 2>&1 || { tail $O/lstm_$v.log; exit 1; }
  echo "$v $(tail -1 $O/lstm_$v.log)"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/lstm_kt -o kt -- python3 tools/lstm_trace.py --chunks 10 > $O/lstm_kt.log 2>&1 || { tail $O/lstm_kt.log; exit 1; }
python3 - <<PY
import csv
rows=list(csv.DictReader(open('$O/lstm_kt/kt_kernel_stats.csv')))
for r in rows[:6]:
    print("%-80s %6s %9.1f us" % (r['Name'][:80], r['Calls'], float(r['AverageNs'])/1e3))
# gaps between consecutive step kernels
tr=[r for r in csv.DictReader(open('$O/lstm_kt/kt_kernel_trace.csv')) if 'lstm_step' in r['Kernel_Name']]
tr.sort(key=lambda r:int(r['Start_Timestamp']))
g=[int(b['Start_Timestamp'])-int(a['End_Timestamp']) for a,b in zip(tr,tr[1:])]
g=sorted(x for x in g if x<50000)
print("step gap median %.2f us p10 %.2f p90 %.2f" % (g[len(g)//2]/1e3, g[len(g)//10]/1e3, g[9*len(g)//10]/1e3))
PY
