#!/bin/bash
# GPU tests (one process) then N bench runs (no CPU baseline): a quick check of a change.
# Usage: TAG=<dir> N=<runs> bash tools/gpu_quick.sh
T=gpurun_out/${TAG:-quick}
mkdir -p $T
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $T/gputests.log 2>&1
rc=$?; tail -2 $T/gputests.log; [ $rc -ne 0 ] && { tail -30 $T/gputests.log; exit $rc; }
for i in $(seq 1 ${N:-2}); do
  timeout -k 10 200 python bench.py --no-cpu-baseline --steps 20 > $T/b$i.json 2> $T/b$i.err || exit $?
  python3 -c "import json; d=json.loads(open('$T/b$i.json').read().strip().splitlines()[-1]); print(round(d['value']), round(d['roofline']['avg_launch_us'],1), round(d['roofline_tr']['avg_launch_us'],1))"
done
