#!/bin/bash
# Last check at HEAD: full -m gpu suite, smoke, default bench.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; O=gpurun_out/r02_last; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?; tail -1 $O/gpu_tests.log; [ $rc -ne 0 ] && { grep -E "FAIL|Error" $O/gpu_tests.log | head; exit $rc; }
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 600 python bench.py > $O/bench.json 2>$O/b.err || { tail $O/b.err; exit 1; }
python -c "import json; d=json.loads(open('$O/bench.json').read().splitlines()[-1]); print('bench', round(d['value']), round(d['roofline']['frac'],4), round(d['roofline_tr']['frac'],4), d['cpu_baseline']['value'])"
