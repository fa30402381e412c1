#!/bin/bash
# Batch split over HIP streams, eager vs hipGraph replay.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; O=gpurun_out/r02r; mkdir -p $O
for G in "" "--graph"; do for S in 1 2 3 4; do
  timeout -k 10 300 python bench.py --steps 30 --no-cpu-baseline --streams $S $G > $O/b${S}$G.json 2>$O/b$S.err || { tail -20 $O/b$S.err; exit 1; }
  python -c "import json; d=json.loads(open('$O/b${S}$G.json').read().splitlines()[-1]); print('streams=$S $G', round(d['value']), d['config']['launch'][:60], round(d['roofline']['avg_launch_us'],1), round(d['roofline_tr']['avg_launch_us'],1))"
done; done
