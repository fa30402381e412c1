#!/bin/bash
# Batch split over HIP streams (FusedResNet.forward_streams): bench at 1, 2, 4 streams, twice.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; O=gpurun_out/r02q; mkdir -p $O
for rep in 1 2; do for S in 1 2 4; do
  timeout -k 10 300 python bench.py --steps 30 --no-cpu-baseline --streams $S > $O/b${S}_$rep.json 2>$O/b$S.err || { tail -20 $O/b$S.err; exit 1; }
  python -c "import json; d=json.loads(open('$O/b${S}_$rep.json').read().splitlines()[-1]); print('streams=$S', round(d['value']), round(d['roofline']['avg_launch_us'],1), round(d['roofline_tr']['avg_launch_us'],1))"
done; done
