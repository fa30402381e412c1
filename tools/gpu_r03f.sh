#!/bin/bash
# r03f: LSTM step kernel + pointwise engine: tests, timings, A/B (TQ_PW=0/1) on MobileNet-V2 /
# EfficientNet fused lines and the ResNet bench
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; TAG=${1:-r03f}; O=gpurun_out/$TAG; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_lstm.py tests/test_gpu_windows.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -1 $O/tests.log; [ $rc -ne 0 ] && { grep -E "FAIL|Error|assert" $O/tests.log | head -20; exit $rc; }
for v in "TQ_LSTM_SEQ=0" "TQ_LSTM_SEQ=1"; do
  env $v timeout -k 10 300 python3 tools/lstm_trace.py --chunks 20 > $O/lstm_$v.log 2>&1 || { tail $O/lstm_$v.log; exit 1; }
  echo "$v $(tail -1 $O/lstm_$v.log)"
done
for pw in 0 1; do
  for arch in mobilenet_v2 efficientnet_b0; do
    TQ_PW=$pw timeout -k 10 300 python -u -c "
import sys, torch
sys.path.insert(0, 'tools')
import bench_d4
r = bench_d4.cnn_fused('$arch', 10, 3, 256, torch.device('cuda:0'))
k = r['kernels']
print('pw=$pw $arch %.0f img/s' % r['images_per_s'], {n: (round(v['avg_launch_us'], 1), v['launches_per_step'], round(v.get('frac') or 0, 3)) for n, v in k.items()})
" 2>/dev/null || exit 1
  done
done
for i in 1 2; do
  for pw in 0 1; do
    TQ_PW=$pw timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-d4 --no-d1 --steps 20 > $O/b$pw.$i.json 2> $O/b$pw.$i.err || { tail -5 $O/b$pw.$i.err; exit 1; }
    python3 -c "import json; d=json.loads(open('$O/b$pw.$i.json').read().strip().splitlines()[-1]); print('pw=$pw', $i, round(d['value']), 'conv', round(d['roofline']['avg_launch_us'],1), 'frac', round(d['roofline']['frac'],4))"
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/lstm_kt -o kt -- python3 tools/lstm_trace.py --chunks 10 > $O/lstm_kt.log 2>&1 || { tail $O/lstm_kt.log; exit 1; }
python3 - <<PY
import csv
rows=list(csv.DictReader(open('$O/lstm_kt/kt_kernel_stats.csv')))
for r in rows[:10]:
    print("%-80s %6s %9.1f us" % (r['Name'][:80], r['Calls'], float(r['AverageNs'])/1e3))
PY
