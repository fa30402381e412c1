#!/bin/bash
# D4 A/B: current library vs lib/libtq_hip_old.so (before the swish epilogue), + bench
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; O=gpurun_out/r02x; mkdir -p $O
L=$R/term-quantization_amd/lib
timeout -k 10 300 python bench.py --no-cpu-baseline --steps 20 > $O/bench.json 2>$O/bench.err || { tail $O/bench.err; exit 1; }
python -c "import json; d=json.loads(open('$O/bench.json').read().splitlines()[-1]); print('bench', round(d['value']), round(d['roofline']['frac'],4), round(d['roofline']['avg_launch_us'],1), round(d['roofline_tr']['avg_launch_us'],1))"
for v in new old new; do
  if [ $v = old ]; then export TQ_LIB_PATH=$L/libtq_hip_old.so; else unset TQ_LIB_PATH; fi
  timeout -k 10 600 python tools/bench_d4.py --only mobilenet_v2 > $O/d4_$v.log 2>&1 || { tail $O/d4_$v.log; exit 1; }
  python - <<PY
import json
for l in open('$O/d4_$v.log'):
    if l.startswith('{'):
        d=json.loads(l); f=d.get('fused_executor')
        print('$v', d['metric'], round(d['value']), 'fused', f and round(f['images_per_s']), f and {k:round(v['avg_launch_us'],1) for k,v in f['kernels'].items()})
PY
done
