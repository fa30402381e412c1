#!/bin/bash
# full -m gpu suite + smoke + bench (stem: BN after pool)
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; O=gpurun_out/r02v; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/gpu_tests.log 2>&1; rc=$?
tail -3 $O/gpu_tests.log; [ $rc -ne 0 ] && { grep -E "FAIL|Error" $O/gpu_tests.log | head -20; exit $rc; }
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
for i in 1 2; do
timeout -k 10 300 python bench.py --no-cpu-baseline --steps 20 > $O/bench$i.json 2>$O/bench.err || { tail $O/bench.err; exit 1; }
python -c "import json; d=json.loads(open('$O/bench$i.json').read().splitlines()[-1]); print(round(d['value']), round(d['roofline']['frac'],4), round(d['roofline']['avg_launch_us'],1), round(d['roofline_tr']['avg_launch_us'],1))"
done
