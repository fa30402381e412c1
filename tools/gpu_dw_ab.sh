#!/bin/bash
# Depthwise kernel A/B: the bit-identity test, the fused MobileNet-V2/EfficientNet tests, then
# tools/bench_d4.py fused lines under TQ_DW_SLIDE=0 (row-blocked), 4 and 8 (sliding window).
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; TAG=${1:-dwab}; O=gpurun_out/$TAG; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_models.py tests/test_gpu_fused_mbv2.py \
    tests/test_gpu_fused_effnet.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log; [ $rc -ne 0 ] && { grep -E "FAIL|Error|assert" $O/tests.log | head -20; exit $rc; }
for m in 0 4 8; do
  for arch in mobilenet_v2 efficientnet_b0; do
    TQ_DW_SLIDE=$m timeout -k 10 300 python -u -c "
import sys, json, torch
sys.path.insert(0, 'tools')
import bench_d4
r = bench_d4.cnn_fused('$arch', 10, 3, 256, torch.device('cuda:0'))
k = r['kernels']
print('slide=$m $arch %.0f img/s' % r['images_per_s'], {n: (round(v['avg_launch_us'], 1), v['launches_per_step'], round(v.get('frac') or 0, 3)) for n, v in k.items()})
" >> $O/ab.log 2>&1 || { tail -5 $O/ab.log; exit 1; }
  done
done
cat $O/ab.log
