#!/bin/bash
# Patch-engine software pipelining: correctness (patch-engine GPU tests), per-layer timing
# pipelined vs not (conv_probe, layers 6/11/13/16), then bench A/B.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; O=gpurun_out/r02d; mkdir -p $O
fatal() { [ "$1" -ge 124 ] && { echo "fatal rc=$1 at $2"; exit "$1"; }; return 0; }
timeout -k 10 600 python -u -m pytest tests/test_gpu_conv.py tests/test_gpu_fused.py tests/test_gpu_windows.py -x -q --timeout 120 --timeout-method thread > $O/t.log 2>&1; rc=$?; tail -3 $O/t.log; fatal $rc tests; [ $rc -ne 0 ] && exit $rc
for L in 6 11 13 16; do for P in 0 1; do
  echo -n "pipe=$P "; TQ_PATCH_PIPE=$P timeout -k 10 120 python tools/conv_probe.py --layer $L --codes 1 --no-out --iters 30 2>/dev/null | tail -1; rc=$?; fatal $rc probe
done; done
for P in 1 0 1 0; do
  TQ_PATCH_PIPE=$P timeout -k 10 300 python bench.py --steps 20 --no-cpu-baseline > $O/bench_p$P.json 2>$O/bench_p$P.err
  rc=$?; fatal $rc bench; python -c "import json; d=json.loads(open('$O/bench_p$P.json').read().splitlines()[-1]); print('pipe=$P', round(d['value']), round(d['roofline']['avg_launch_us'],1))"
done
