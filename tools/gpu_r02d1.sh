#!/bin/bash
# 1x1 convs with Cp % 64 != 0 on the direct engine: conv + fused-executor tests, D4 CNNs.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; O=gpurun_out/r02d1; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_conv.py tests/test_gpu_models.py tests/test_gpu_fused_mbv2.py tests/test_gpu_fused_effnet.py tests/test_gpu_fused.py -x -q --timeout 300 --timeout-method thread > $O/t.log 2>&1; rc=$?
tail -1 $O/t.log; [ $rc -ne 0 ] && { grep -E "Error|assert|FAIL" $O/t.log | head -20; exit $rc; }
for m in mobilenet_v2 efficientnet_b0; do
  timeout -k 10 600 python tools/bench_d4.py --only $m > $O/d4_$m.log 2>&1 || { tail $O/d4_$m.log; exit 1; }
  python - $O/d4_$m.log <<'PY'
import json,sys
for l in open(sys.argv[1]):
    if l.startswith('{'):
        d=json.loads(l); f=d.get('fused_executor')
        print(d['metric'], round(d['value']), 'fused', f and round(f['images_per_s']), {k:round(v['avg_launch_us'],1) for k,v in f['kernels'].items()})
PY
done
