#!/bin/bash
# r03d: full GPU suite with the fp32 epilogue, bench A/B vs the fp64-epilogue build, D4 lines,
# LSTM timings.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; TAG=${1:-r03d}; O=gpurun_out/$TAG; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?; tail -2 $O/gpu_tests.log; [ $rc -ne 0 ] && { grep -E "FAIL|Error|assert" $O/gpu_tests.log | head -30; exit $rc; }
bash tools/gpu_ab_lib.sh $TAG/ab 2 epi64 || exit 1
for arch in mobilenet_v2 efficientnet_b0; do
  timeout -k 10 300 python -u -c "
import sys, torch
sys.path.insert(0, 'tools')
import bench_d4
r = bench_d4.cnn_fused('$arch', 10, 3, 256, torch.device('cuda:0'))
k = r['kernels']
print('$arch %.0f img/s' % r['images_per_s'], {n: (round(v['avg_launch_us'], 1), v['launches_per_step'], round(v.get('frac') or 0, 3)) for n, v in k.items()})
" 2>/dev/null || exit 1
done
for v in "TQ_LSTM_SEQ=0" "TQ_LSTM_SEQ=1"; do
  env $v timeout -k 10 300 python3 tools/lstm_trace.py --chunks 20 > $O/lstm_$v.log 2>&1 || { tail $O/lstm_$v.log; exit 1; }
  echo "$v $(tail -1 $O/lstm_$v.log)"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/lstm_kt -o kt -- python3 tools/lstm_trace.py --chunks 10 > $O/lstm_kt.log 2>&1 || { tail $O/lstm_kt.log; exit 1; }
echo done
