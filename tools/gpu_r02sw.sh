#!/bin/bash
# Swish in the direct engine's epilogue (EfficientNet expand convs): tests, D4, bench.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; O=gpurun_out/r02sw; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/t.log 2>&1; rc=$?
tail -1 $O/t.log; [ $rc -ne 0 ] && { grep -E "Error|assert|FAIL" $O/t.log | head -20; exit $rc; }
timeout -k 10 600 python tools/bench_d4.py > $O/d4.log 2>&1 || { tail $O/d4.log; exit 1; }
python - $O/d4.log <<'PY'
import json,sys
for l in open(sys.argv[1]):
    if l.startswith('{'):
        d=json.loads(l); f=d.get('fused_executor')
        print(d['metric'], round(d['value']), 'fused', f and round(f['images_per_s']), f and {k:round(v['avg_launch_us'],1) for k,v in f['kernels'].items()})
PY
timeout -k 10 300 python bench.py --no-cpu-baseline --steps 20 > $O/bench.json 2>$O/bench.err || { tail $O/bench.err; exit 1; }
python -c "import json; d=json.loads(open('$O/bench.json').read().splitlines()[-1]); print('bench', round(d['value']), round(d['roofline']['frac'],4))"
