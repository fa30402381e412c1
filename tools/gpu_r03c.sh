#!/bin/bash
# r03c: dw window kernel + LSTM sweep fix (tests, A/B), MobileNet-V2 fused kernel trace,
# patch-engine ablations (layers 11, 16), per-layer config sweep.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; TAG=${1:-r03c}; O=gpurun_out/$TAG; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_models.py tests/test_gpu_lstm.py tests/test_gpu_fused_mbv2.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -1 $O/tests.log; [ $rc -ne 0 ] && { grep -E "FAIL|Error|assert" $O/tests.log | head -20; exit $rc; }
for m in 0 4; do
  TQ_DW_SLIDE=$m timeout -k 10 300 python -u -c "
import sys, torch
sys.path.insert(0, 'tools')
import bench_d4
r = bench_d4.cnn_fused('mobilenet_v2', 10, 3, 256, torch.device('cuda:0'))
k = r['kernels']
print('slide=$m mobilenet_v2 %.0f img/s' % r['images_per_s'], {n: (round(v['avg_launch_us'], 1), v['launches_per_step'], round(v.get('frac') or 0, 3)) for n, v in k.items()})
" 2>/dev/null || exit 1
done
for v in "TQ_LSTM_SEQ=0" "TQ_LSTM_UPPER=miopen" "TQ_LSTM_SEQ=1"; do
  env $v timeout -k 10 300 python3 tools/lstm_trace.py --chunks 20 > $O/lstm_$v.log 2>&1 || { tail $O/lstm_$v.log; exit 1; }
  echo "$v $(tail -1 $O/lstm_$v.log)"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/lstm_kt -o kt -- python3 tools/lstm_trace.py --chunks 10 > $O/lstm_kt.log 2>&1 || { tail $O/lstm_kt.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/mbv2_kt -o kt -- python3 tools/bench_d4.py --only mobilenet_v2 --steps 3 --warmup 1 > $O/mbv2_kt.log 2>&1 || { tail $O/mbv2_kt.log; exit 1; }
bash tools/gpu_ablate_patch.sh $TAG/abl > $O/abl.log 2>&1 || { tail $O/abl.log; exit 1; }
cat $O/abl.log
timeout -k 10 600 python -u tools/microbench.py --sweep --iters 10 > $O/sweep.log 2>&1 || { tail $O/sweep.log; exit 1; }
grep -E "sweep|total" $O/sweep.log | tail -25
echo done
