#!/bin/bash
# r03ac: signed code tables (no-activation epilogues): tests, MobileNet-V2 per-launch, D4
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; TAG=${1:-r03ac}; O=gpurun_out/$TAG; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_fused.py -k signed -m gpu -x -v --timeout 300 --timeout-method thread \
    > $O/tests_signed.log 2>&1 || { tail -40 $O/tests_signed.log; exit 1; }
tail -1 $O/tests_signed.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
    > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 python tools/fused_layers.py --arch mobilenet_v2 > $O/mbv2_layers.txt 2>&1 || { tail $O/mbv2_layers.txt; exit 1; }
sed -n 2,12p $O/mbv2_layers.txt; tail -1 $O/mbv2_layers.txt
timeout -k 10 300 python -c "
import sys, json, torch; sys.path.insert(0, 'tools'); import bench_d4
dev = torch.device('cuda:0')
for a in ('mobilenet_v2', 'efficientnet_b0'):
    r = bench_d4.cnn_fused(a, 10, 3, 256, dev)
    print(a, round(r['images_per_s']), json.dumps({k: round(v['avg_launch_us'], 1) for k, v in r['kernels'].items()}))
" 2>>$O/err.log | tee $O/d4.txt
