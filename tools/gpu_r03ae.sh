#!/bin/bash
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; TAG=${1:-r03ae}; O=gpurun_out/$TAG; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_models.py tests/test_gpu_fused_mbv2.py tests/test_gpu_fused_effnet.py \
    -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for A in "32 112 1" "144 56 1" "192 28 1" "384 14 1" "576 14 1" "960 7 1" "96 112 2" "144 56 2" "192 28 2" "576 14 2"; do
  set -- $A
  for M in 1 2; do
    echo -n "stream=$M "
    TQ_DW_STREAM=$M timeout -k 10 120 python tools/dw_probe.py --c $1 --hw $2 --stride $3 --iters 20 2>>$O/err.log | tail -1 || exit 1
  done
done | tee $O/dw_probe.txt
timeout -k 10 300 python -c "
import sys, json, torch; sys.path.insert(0, 'tools'); import bench_d4
dev = torch.device('cuda:0')
for a in ('mobilenet_v2', 'efficientnet_b0'):
    r = bench_d4.cnn_fused(a, 10, 3, 256, dev)
    print(a, round(r['images_per_s']), json.dumps({k: round(v['avg_launch_us'], 1) for k, v in r['kernels'].items()}))
" 2>>$O/err.log | tee $O/d4.txt
