#!/bin/bash
# Direct engine MB = 2 (128 x 128 tiles, config 9) vs MB = 1 (config 10) on the layer-2 convs
# now that the MB = 2 no-flush variant is scratch-free; then bench with TQ_DIRECT=2.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; O=gpurun_out/r02m; mkdir -p $O
for L in 5 6 7; do for m in "--codes 1 --no-out" "--codes 1 --residual"; do for c in 10 9; do
  echo -n "L$L cfg=$c $m: "; timeout -k 10 120 python tools/conv_probe.py --layer $L --config $c $m --iters 30 2>/dev/null | tail -1 || exit 1
done; done; done
for V in 2 1 2 1; do
  TQ_DIRECT=$V timeout -k 10 300 python bench.py --steps 20 --no-cpu-baseline > $O/b$V.json 2>$O/b$V.err || exit $?
  python -c "import json; d=json.loads(open('$O/b$V.json').read().splitlines()[-1]); print('direct_mb=$V', round(d['value']), round(d['roofline']['avg_launch_us'],1))"
done
