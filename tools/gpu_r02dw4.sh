#!/bin/bash
# 5x5 depthwise: two output rows per lane (default) vs four (TQ_DW_ROWS=4); tests first.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; O=gpurun_out/r02dw4; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_models.py tests/test_gpu_fused_effnet.py -x -q --timeout 300 --timeout-method thread > $O/t.log 2>&1; rc=$?
tail -1 $O/t.log; [ $rc -ne 0 ] && { grep -E "Error|assert" $O/t.log | head; exit $rc; }
for rep in 1 2; do for v in 2 4; do
  if [ $v = 2 ]; then unset TQ_DW_ROWS; else export TQ_DW_ROWS=4; fi
  timeout -k 10 600 python tools/bench_d4.py --only efficientnet_b0 > $O/d4_$v.log 2>&1 || { tail $O/d4_$v.log; exit 1; }
  python - $O/d4_$v.log $v <<'PY'
import json,sys
for l in open(sys.argv[1]):
    if l.startswith('{'):
        d=json.loads(l); f=d.get('fused_executor')
        print('rows5x5=' + sys.argv[2], round(d['value']), 'fused', round(f['images_per_s']), 'dw', round(f['kernels']['dwconv2d_termpair']['avg_launch_us'],1))
PY
done; done
