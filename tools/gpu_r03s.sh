#!/bin/bash
# r03s: direct-engine prefetch depth 3 (lib/libtq_hip_d3.so) vs 2 (product) vs HEAD~ (base)
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; TAG=${1:-r03s}; O=gpurun_out/$TAG; mkdir -p $O
export TMPDIR=/tmp
L3=$R/term-quantization_amd/lib/libtq_hip_d3.so
BASE=$R/term-quantization_amd/lib/libtq_hip_base.so
timeout -k 10 600 python -u -m pytest tests/test_gpu_conv.py tests/test_gpu_fused.py tests/test_gpu_fused_parity.py -m gpu -x -q --timeout 300 \
    --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
TQ_STRIP_RES=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_fused.py -m gpu -x -q --timeout 300 \
    --timeout-method thread > $O/tests_strip.log 2>&1 || { tail -30 $O/tests_strip.log; exit 1; }
tail -1 $O/tests_strip.log
tail -1 $O/tests.log
TQ_LIB_PATH=$L3 timeout -k 10 600 python -u -m pytest tests/test_gpu_conv.py tests/test_gpu_fused.py -m gpu -x -q --timeout 300 \
    --timeout-method thread > $O/tests_d3.log 2>&1 || { tail -30 $O/tests_d3.log; exit 1; }
tail -1 $O/tests_d3.log
for L in 2 5 6 8 9; do
  for V in base cur d3; do
    case $V in base) export TQ_LIB_PATH=$BASE;; d3) export TQ_LIB_PATH=$L3;; *) unset TQ_LIB_PATH;; esac
    RES=""; case $L in 2|4|8|9|13|18) RES="--residual";; esac
    echo -n "$V "; timeout -k 10 120 python tools/conv_probe.py --layer $L --codes 1 $RES --iters 20 2>>$O/err.log | tail -1 || exit 1
  done
done | tee $O/probe.txt
for L in 2 4; do
  for V in cur strip; do
    case $V in strip) export TQ_STRIP_RES=1;; *) unset TQ_STRIP_RES;; esac
    echo -n "$V "; timeout -k 10 120 python tools/conv_probe.py --layer $L --codes 1 --residual --iters 20 2>>$O/err.log | tail -1 || exit 1
  done
done | tee $O/strip_res.txt
unset TQ_STRIP_RES
for V in cur d3 cur d3; do
  case $V in d3) export TQ_LIB_PATH=$L3;; *) unset TQ_LIB_PATH;; esac
  echo -n "$V "; timeout -k 10 300 python bench.py --no-cpu-baseline --no-d1 --no-d4 --steps 20 2>>$O/err.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('%.0f img/s conv %.1f us frac %.3f stem %.1f' % (d['value'], d['roofline']['avg_launch_us'], d['roofline']['frac'], d['roofline_tr']['avg_launch_us']))" || exit 1
done | tee $O/bench_ab.txt
