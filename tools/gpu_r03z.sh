#!/bin/bash
# r03z: persistent tile ranges for short-K direct-engine convs: tests, A/B (TQ_DIR_PERSIST=0
# one-shot vs 4 per CU) on MobileNet-V2 per-launch timings, fused D4, ResNet bench
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; TAG=${1:-r03z}; O=gpurun_out/$TAG; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_conv.py tests/test_gpu_fused.py tests/test_gpu_fused_mbv2.py \
    tests/test_gpu_fused_effnet.py tests/test_gpu_fused_parity.py -m gpu -x -q --timeout 300 --timeout-method thread \
    > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for P in 0 4 2 8; do
  echo "== TQ_DIR_PERSIST=$P"
  TQ_DIR_PERSIST=$P timeout -k 10 300 python tools/fused_layers.py --arch mobilenet_v2 > $O/mbv2_layers_$P.txt 2>&1 || { tail $O/mbv2_layers_$P.txt; exit 1; }
  sed -n 3,8p $O/mbv2_layers_$P.txt; tail -1 $O/mbv2_layers_$P.txt
done
for P in 4 0; do
  TQ_DIR_PERSIST=$P timeout -k 10 300 python -c "
import sys, json, torch; sys.path.insert(0, 'tools'); import bench_d4
dev = torch.device('cuda:0')
for a in ('mobilenet_v2', 'efficientnet_b0'):
    r = bench_d4.cnn_fused(a, 10, 3, 256, dev)
    print('persist $P', a, round(r['images_per_s']), json.dumps({k: round(v['avg_launch_us'], 1) for k, v in r['kernels'].items()}))
" 2>>$O/err.log
done | tee $O/d4.txt
for P in 4 0 4 0; do
  echo -n "persist $P "; TQ_DIR_PERSIST=$P timeout -k 10 300 python bench.py --no-cpu-baseline --no-d1 --no-d4 --steps 20 2>>$O/err.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('%.0f img/s conv %.1f us frac %.3f stem %.1f' % (d['value'], d['roofline']['avg_launch_us'], d['roofline']['frac'], d['roofline_tr']['avg_launch_us']))" || exit 1
done | tee $O/bench_ab.txt
