#!/bin/bash
# Fused stems of the MobileNet-V2 / EfficientNet executors: tests + D4.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; O=gpurun_out/r02st; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_fused_mbv2.py tests/test_gpu_fused_effnet.py tests/test_gpu_models.py -x -q --timeout 300 --timeout-method thread > $O/t.log 2>&1; rc=$?
tail -1 $O/t.log; [ $rc -ne 0 ] && { grep -E "Error|assert" $O/t.log | head -20; exit $rc; }
for m in mobilenet_v2 efficientnet_b0; do
  timeout -k 10 600 python tools/bench_d4.py --only $m > $O/d4_$m.log 2>&1 || { tail $O/d4_$m.log; exit 1; }
  python - $O/d4_$m.log <<'PY'
import json,sys
for l in open(sys.argv[1]):
    if l.startswith('{'):
        d=json.loads(l); f=d.get('fused_executor')
        print(d['metric'], round(d['value']), 'fused', round(f['images_per_s']))
PY
done
