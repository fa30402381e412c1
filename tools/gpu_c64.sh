#!/bin/bash
# Cout-64 pixel-ring engine: parity tests, per-form timings against the default engines,
# per-launch times of the fused executor.  Usage: bash tools/gpu_c64.sh <tag> [pytest -k expr]
set -u
TAG=${1:-c64}
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; O=gpurun_out/$TAG; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_c64.py -x -q --timeout 120 --timeout-method thread ${2:+-k "$2"} > $O/tests.txt 2>&1
rc=$?; tail -15 $O/tests.txt; [ $rc -ne 0 ] && exit $rc
FORMS=("--codes 1 --no-out" "--codes 1 --residual" "--codes 1 --residual --no-out")
for i in 0 1 2; do
  for cfg in 0 15; do
    [ $cfg = 0 ] && export TQ_C64=0 || unset TQ_C64
    timeout -k 10 120 python3 tools/conv_probe.py --layer 1 --nonneg --config $cfg ${FORMS[$i]} --iters 30 > $O/probe${i}_$cfg.txt 2>&1 || { tail -5 $O/probe${i}_$cfg.txt; exit 1; }
    echo "form $i (${FORMS[$i]}): $(tail -1 $O/probe${i}_$cfg.txt)"
  done
done
unset TQ_C64
timeout -k 10 240 python3 tools/layer_times.py --steps 3 > $O/layers.txt 2>&1 || { tail -20 $O/layers.txt; exit 1; }
head -8 $O/layers.txt; tail -1 $O/layers.txt
