#!/bin/bash
# dw: branch-free row kernel (in-tree) vs committed row kernel (ab) vs flat, D4 fused img/s;
# dw/fused tests on the in-tree build.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; O=gpurun_out/r02dw3; mkdir -p $O
L=$R/term-quantization_amd/lib
timeout -k 10 600 python -u -m pytest tests/test_gpu_models.py tests/test_gpu_fused_mbv2.py tests/test_gpu_fused_effnet.py -x -q --timeout 300 --timeout-method thread > $O/t.log 2>&1; rc=$?
tail -1 $O/t.log; [ $rc -ne 0 ] && { grep -E "Error|assert" $O/t.log | head; exit $rc; }
for v in new ab flat; do
  unset TQ_LIB_PATH TQ_DW_ROWS
  [ $v = ab ] && export TQ_LIB_PATH=$L/libtq_hip_ab.so
  [ $v = flat ] && export TQ_DW_ROWS=0
  for m in mobilenet_v2 efficientnet_b0; do
    timeout -k 10 600 python tools/bench_d4.py --only $m > $O/d4_${m}_$v.log 2>&1 || { tail $O/d4_${m}_$v.log; exit 1; }
    python - $O/d4_${m}_$v.log $v <<'PY'
import json,sys
for l in open(sys.argv[1]):
    if l.startswith('{'):
        d=json.loads(l); f=d.get('fused_executor')
        print(sys.argv[2], d['metric'], round(d['value']), 'fused', round(f['images_per_s']), 'dw', round(f['kernels']['dwconv2d_termpair']['avg_launch_us'],1))
PY
  done
done
