#!/bin/bash
# r03aa: fp32 epilogue arithmetic (lib/libtq_hip_f32.so, -DTQ_EPI_F32=1) vs the fp64 default:
# D4 fused images/s and the ResNet bench, interleaved
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; TAG=${1:-r03aa}; O=gpurun_out/$TAG; mkdir -p $O
export TMPDIR=/tmp
F32=$R/term-quantization_amd/lib/libtq_hip_f32.so
for V in f32 cur f32 cur; do
  case $V in f32) export TQ_LIB_PATH=$F32;; *) unset TQ_LIB_PATH;; esac
  timeout -k 10 300 python -c "
import sys, json, torch; sys.path.insert(0, 'tools'); import bench_d4
dev = torch.device('cuda:0')
for a in ('mobilenet_v2', 'efficientnet_b0'):
    r = bench_d4.cnn_fused(a, 10, 3, 256, dev)
    print('$V', a, round(r['images_per_s']), json.dumps({k: round(v['avg_launch_us'], 1) for k, v in r['kernels'].items()}))
" 2>>$O/err.log || exit 1
  echo -n "$V resnet "; timeout -k 10 300 python bench.py --no-cpu-baseline --no-d1 --no-d4 --steps 20 2>>$O/err.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('%.0f img/s conv %.1f us frac %.3f stem %.1f' % (d['value'], d['roofline']['avg_launch_us'], d['roofline']['frac'], d['roofline_tr']['avg_launch_us']))" || exit 1
done | tee $O/ab.txt
