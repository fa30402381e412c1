#!/bin/bash
# A/B: the row-strip engine for the residual (block conv2) layer-1 convs, with code tables.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; O=gpurun_out/r02i; mkdir -p $O
fatal() { [ "$1" -ge 124 ] && { echo "fatal rc=$1 at $2"; exit "$1"; }; return 0; }
TQ_STRIP_RES=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_fused.py tests/test_gpu_fused_parity.py -x -q --timeout 120 --timeout-method thread > $O/t.log 2>&1; rc=$?; tail -2 $O/t.log; fatal $rc tests; [ $rc -ne 0 ] && exit $rc
for V in 0 1; do for m in "--codes 1 --residual" "--codes 1 --residual --no-out"; do
  echo -n "strip_res=$V $m: "; TQ_STRIP_RES=$V timeout -k 10 120 python tools/conv_probe.py --layer 2 $m --iters 30 2>/dev/null | tail -1; rc=$?; fatal $rc probe
done; done
for V in 1 0 1 0; do
  TQ_STRIP_RES=$V timeout -k 10 300 python bench.py --steps 20 --no-cpu-baseline > $O/bench_s$V.json 2>$O/bench_s$V.err
  rc=$?; fatal $rc bench; python -c "import json; d=json.loads(open('$O/bench_s$V.json').read().splitlines()[-1]); print('strip_res=$V', round(d['value']), round(d['roofline']['avg_launch_us'],1))"
done
