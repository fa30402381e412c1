#!/bin/bash
# Per-layer and bench A/B of the working tree against lib/libtq_hip_base.so (tools/base_variant.sh)
# (tests of the conv engines, conv_probe per ResNet-18 layer, bench.py without d1/d4/cpu).
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; TAG=${1:-ab}; O=gpurun_out/$TAG; mkdir -p $O
export TMPDIR=/tmp
BASE=$R/term-quantization_amd/lib/libtq_hip_base.so
timeout -k 10 600 python -u -m pytest tests/test_gpu_conv.py tests/test_gpu_fused.py tests/test_gpu_windows.py \
    tests/test_gpu_fused_parity.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for L in 2 4 5 6 7 8 9 12 17; do
  for V in base cur; do
    if [ $V = base ]; then export TQ_LIB_PATH=$BASE; else unset TQ_LIB_PATH; fi
    RES=""; case $L in 2|4|8|9|13|18) RES="--residual";; esac
    echo -n "$V "; timeout -k 10 120 python tools/conv_probe.py --layer $L --codes 1 $RES --iters 20 2>>$O/err.log | tail -1 || exit 1
  done
done | tee $O/probe.txt
for V in cur base cur base; do
  if [ $V = base ]; then export TQ_LIB_PATH=$BASE; else unset TQ_LIB_PATH; fi
  echo -n "$V "; timeout -k 10 300 python bench.py --no-cpu-baseline --no-d1 --no-d4 --steps 20 2>>$O/err.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('%.0f img/s conv %.1f us frac %.3f stem %.1f' % (d['value'], d['roofline']['avg_launch_us'], d['roofline']['frac'], d['roofline_tr']['avg_launch_us']))" || exit 1
done | tee $O/bench_ab.txt
