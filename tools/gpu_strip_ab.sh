#!/bin/bash
# Strip-engine check: its parity tests, per-layer times with and without it, a bench A/B,
# then one full bench line (CPU baseline included).  TAG=<dir>
T=gpurun_out/${TAG:-strip}
mkdir -p $T
timeout -k 10 300 python -u -m pytest tests/test_gpu_windows.py -x -q --timeout 120 --timeout-method thread > $T/tests.log 2>&1
rc=$?; tail -2 $T/tests.log; [ $rc -ne 0 ] && { tail -30 $T/tests.log; exit $rc; }
for v in 1 0; do
  TQ_STRIP=$v timeout -k 10 200 python tools/layer_times.py --steps 5 > $T/layers_$v.txt 2>&1 || exit $?
done
VAR=TQ_STRIP A=1 B=0 R=2 TAG=${TAG:-strip}/ab bash tools/gpu_ab_env.sh || exit $?
timeout -k 10 400 python bench.py --steps 20 > $T/bench.json 2> $T/bench.err || exit $?
tail -1 $T/bench.json
