#!/bin/bash
# Default bench (with the CPU baseline) and a sustained 2000-step run.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; O=gpurun_out/r02_sustain; mkdir -p $O
timeout -k 10 600 python bench.py > $O/bench_default.json 2>$O/b.err || { tail $O/b.err; exit 1; }
python -c "import json; d=json.loads(open('$O/bench_default.json').read().splitlines()[-1]); print('default', round(d['value']), round(d['roofline']['frac'],4), d['cpu_baseline']['value'])"
timeout -k 10 600 python bench.py --no-cpu-baseline --steps 2000 --warmup 20 > $O/bench_2000.json 2>$O/b2.err || { tail $O/b2.err; exit 1; }
python -c "import json; d=json.loads(open('$O/bench_2000.json').read().splitlines()[-1]); print('2000 steps', round(d['value']), round(d['ms_per_step'],3))"
