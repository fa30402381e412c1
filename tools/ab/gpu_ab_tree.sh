#!/bin/bash
# Interleaved bench A/B of this tree against another checkout of the repo (a git worktree
# under _ab/<name>, built in place): same lease, same box, alternating runs.
# Usage: bash tools/ab/gpu_ab_tree.sh <tag> <rounds> <worktree dir> [bench args...]
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; TAG=$1; N=$2; ALT=$3; shift 3; O=$R/gpurun_out/$TAG
mkdir -p $O
for i in $(seq 1 $N); do
  for v in head alt; do
    d=$R; [ "$v" = alt ] && d=$R/$ALT
    extra=""; [ "$v" = head ] && extra="--no-d4 --no-d1"
    (cd $d && timeout -k 10 300 python -u bench.py --no-cpu-baseline $extra "$@" > $O/$v.$i.json 2> $O/$v.$i.err) \
      || { tail -5 $O/$v.$i.err; exit 1; }
    python3 -c "import json; d=json.loads(open('$O/$v.$i.json').read().strip().splitlines()[-1]); r=d.get('roofline',{}); print('$v', $i, round(d['value']), 'ms', round(d['ms_per_step'],3), 'conv', round(r.get('avg_launch_us',0),1), 'frac', round(r.get('frac',0),4))"
  done
done
