#!/bin/bash
# D4 CNN lines with the fused executors also replayed as hipGraphs.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; O=gpurun_out/r02g; mkdir -p $O
timeout -k 10 900 python tools/bench_d4.py > $O/d4.log 2>&1 || { tail $O/d4.log; exit 1; }
python - $O/d4.log <<'PY'
import json,sys
for l in open(sys.argv[1]):
    if l.startswith('{'):
        d=json.loads(l); f=d.get('fused_executor')
        print(d['metric'], round(d['value']), 'fused', f and round(f['images_per_s']), 'graph', f and f.get('images_per_s_graph') and round(f['images_per_s_graph']))
PY
