#!/bin/bash
# Pipelined chunk graphs (half-step offset) vs lockstep two-stream graph, interleaved.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; O=gpurun_out/r02pl; mkdir -p $O
for rep in 1 2; do for L in pipeline graph; do for K in 20 50; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --steps $K --launch $L > $O/b_${L}_${K}_$rep.json 2>$O/b_$L.err || { tail -20 $O/b_$L.err; exit 1; }
  python -c "import json; d=json.loads(open('$O/b_${L}_${K}_$rep.json').read().splitlines()[-1]); print('$L K=$K', round(d['value']), d['config']['launch'][:40], d['accuracy_counters'])"
done; done; done
