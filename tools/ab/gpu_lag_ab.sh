#!/bin/bash
# bench.py headline with TQ_STREAM_LAG = 0 / 1 / 2 / 4 (chunk j starts j x L launches late),
# interleaved, two rounds.
set -u
cd ${GRAFT_REPO_ROOT:-$(pwd)}
for r in 1 2; do for L in 0 1 2 4; do
  TQ_STREAM_LAG=$L timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-d1 --no-d4 --no-stem-leg 2>/dev/null | python3 -c "import sys,json; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('round $r lag $L', round(d['value']), round(d['ms_per_step'],3))" || exit 1
done; done
