#!/bin/bash
# Direct engine Cout tile 128 (TQ_DIRECT=2) vs 64 (default) under the two-stream bench.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; O=gpurun_out/r02mb; mkdir -p $O
for rep in 1 2; do for v in 0 2; do
  if [ $v = 0 ]; then unset TQ_DIRECT; else export TQ_DIRECT=$v; fi
  timeout -k 10 200 python bench.py --no-cpu-baseline --steps 40 > $O/b_${v}_$rep.json 2>$O/b.err || { tail $O/b.err; exit 1; }
  python -c "import json; d=json.loads(open('$O/b_${v}_$rep.json').read().splitlines()[-1]); print('TQ_DIRECT=$v', round(d['value']), round(d['roofline']['avg_launch_us'],1), round(d['roofline']['frac'],4))"
done; done
