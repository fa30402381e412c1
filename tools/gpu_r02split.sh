#!/bin/bash
# Unequal chunk split for the two-stream bench (TQ_SPLIT = images of chunk 0).
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; O=gpurun_out/r02split; mkdir -p $O
for rep in 1 2; do for v in 0 160 192; do
  export TQ_SPLIT=$v
  timeout -k 10 200 python bench.py --no-cpu-baseline --steps 40 > $O/b_${v}_$rep.json 2>$O/b.err || { tail $O/b.err; exit 1; }
  python -c "import json; d=json.loads(open('$O/b_${v}_$rep.json').read().splitlines()[-1]); print('TQ_SPLIT=$v', round(d['value']))"
done; done
