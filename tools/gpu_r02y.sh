#!/bin/bash
# After moving swish out of the shared conv epilogue: fused + model tests, D4 mbv2 A/B vs
# lib/libtq_hip_old.so (pre-swish build), D4 efficientnet, bench.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; O=gpurun_out/r02y; mkdir -p $O
L=$R/term-quantization_amd/lib
timeout -k 10 600 python -u -m pytest tests/test_gpu_fused_effnet.py tests/test_gpu_fused_mbv2.py tests/test_gpu_fused.py tests/test_gpu_models.py tests/test_gpu_fused_parity.py -x -q --timeout 300 --timeout-method thread > $O/t.log 2>&1; rc=$?
tail -3 $O/t.log; [ $rc -ne 0 ] && { grep -E "Error|assert" $O/t.log | head -20; exit $rc; }
for v in new old; do
  if [ $v = old ]; then export TQ_LIB_PATH=$L/libtq_hip_old.so; else unset TQ_LIB_PATH; fi
  timeout -k 10 600 python tools/bench_d4.py --only mobilenet_v2 > $O/d4_mbv2_$v.log 2>&1 || { tail $O/d4_mbv2_$v.log; exit 1; }
done
unset TQ_LIB_PATH
timeout -k 10 600 python tools/bench_d4.py --only efficientnet_b0 > $O/d4_eff.log 2>&1 || { tail $O/d4_eff.log; exit 1; }
for f in $O/d4_*.log; do python - $f <<'PY'
import json,sys
for l in open(sys.argv[1]):
    if l.startswith('{'):
        d=json.loads(l); f=d.get('fused_executor')
        print(sys.argv[1].split('/')[-1], round(d['value']), 'fused', f and round(f['images_per_s']), f and {k:round(v['avg_launch_us'],1) for k,v in f['kernels'].items()})
PY
done
timeout -k 10 300 python bench.py --no-cpu-baseline --steps 20 > $O/bench.json 2>$O/bench.err || { tail $O/bench.err; exit 1; }
python -c "import json; d=json.loads(open('$O/bench.json').read().splitlines()[-1]); print('bench', round(d['value']), round(d['roofline']['frac'],4), round(d['roofline']['avg_launch_us'],1), round(d['roofline_tr']['avg_launch_us'],1))"
