#!/bin/bash
# Strip engine for the residual layer-1 conv2s (TQ_STRIP_RES=1) vs the direct engine, bench.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; O=gpurun_out/r02sr; mkdir -p $O
for rep in 1 2 3; do for v in 0 1; do
  export TQ_STRIP_RES=$v
  timeout -k 10 200 python bench.py --no-cpu-baseline --steps 40 > $O/b_${v}_$rep.json 2>$O/b.err || { tail $O/b.err; exit 1; }
  python -c "import json; d=json.loads(open('$O/b_${v}_$rep.json').read().splitlines()[-1]); print('TQ_STRIP_RES=$v', round(d['value']), round(d['roofline']['avg_launch_us'],1))"
done; done
