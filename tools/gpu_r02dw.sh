#!/bin/bash
# Row-blocked depthwise kernel: depthwise / fused tests, then D4 CNN lines with and without it.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; O=gpurun_out/r02dw; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_models.py tests/test_gpu_fused_mbv2.py tests/test_gpu_fused_effnet.py -x -q --timeout 300 --timeout-method thread > $O/t.log 2>&1; rc=$?
tail -1 $O/t.log; [ $rc -ne 0 ] && { grep -E "Error|assert" $O/t.log | head; exit $rc; }
for v in rows flat; do
  if [ $v = flat ]; then export TQ_DW_ROWS=0; else unset TQ_DW_ROWS; fi
  for m in mobilenet_v2 efficientnet_b0; do
    timeout -k 10 600 python tools/bench_d4.py --only $m > $O/d4_${m}_$v.log 2>&1 || { tail $O/d4_${m}_$v.log; exit 1; }
    python - $O/d4_${m}_$v.log $v <<'PY'
import json,sys
for l in open(sys.argv[1]):
    if l.startswith('{'):
        d=json.loads(l); f=d.get('fused_executor')
        print(sys.argv[2], d['metric'], round(d['value']), 'fused', f and round(f['images_per_s']), 'dw', round(d['kernels']['dwconv2d_termpair']['avg_launch_us'],1), f and round(f['kernels']['dwconv2d_termpair']['avg_launch_us'],1), f and round(f['kernels']['dwconv2d_termpair'].get('frac',0),3))
PY
  done
done
