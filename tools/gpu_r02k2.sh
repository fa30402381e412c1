#!/bin/bash
# Layer-2 3x3 convs (128 -> 128, 28x28): direct (cfg 10) vs input-patch engine (cfg 7 = MB 2,
# cfg 8 = MB 1), conv1-style and residual epilogues; then the bench with the direct engine off.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; O=gpurun_out/r02k2; mkdir -p $O
for m in "--codes 1 --no-out" "--codes 1 --residual"; do for c in 10 7 8; do
  echo -n "cfg=$c $m: "; timeout -k 10 120 python tools/conv_probe.py --layer 6 --config $c $m --iters 30 2>/dev/null | tail -1 || exit 1
done; done
for V in 0 1 0 1; do
  if [ $V = 0 ]; then export TQ_DIRECT=0; else unset TQ_DIRECT; fi
  timeout -k 10 300 python bench.py --steps 20 --no-cpu-baseline > $O/b$V.json 2>$O/b$V.err || exit $?
  python -c "import json; d=json.loads(open('$O/b$V.json').read().splitlines()[-1]); print('direct=$V', round(d['value']), round(d['roofline']['avg_launch_us'],1))"
done
