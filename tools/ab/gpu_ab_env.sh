#!/bin/bash
# Interleaved bench A/B of an environment switch: VAR=<name> A=<value> B=<value>, R rounds.
T=gpurun_out/${TAG:-abenv}
mkdir -p $T
for i in $(seq 1 ${R:-3}); do
  for v in $A $B; do
    env $VAR=$v timeout -k 10 200 python bench.py --no-cpu-baseline --steps ${STEPS:-50} > $T/b_${v}_$i.json 2> $T/b_${v}_$i.err || exit $?
    python3 -c "import json; d=json.loads(open('$T/b_${v}_$i.json').read().strip().splitlines()[-1]); print('$VAR=$v', round(d['value']), round(d['roofline']['avg_launch_us'],1), round(d['roofline_tr']['avg_launch_us'],1))"
  done
done
