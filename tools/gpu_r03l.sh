#!/bin/bash
# r03l: A/B of the working tree (patch-engine fragment schedule, direct-engine ring in
# dynamic LDS) against lib/libtq_hip_base.so (HEAD): per-layer conv_probe, the bench (no
# d1/d4/cpu), and hipBLASLt / MIOpen fp16 reference points (tools/gemm_ref.py).
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; TAG=${1:-r03l}; O=gpurun_out/$TAG; mkdir -p $O
export TMPDIR=/tmp
BASE=$R/term-quantization_amd/lib/libtq_hip_base.so
timeout -k 10 600 python -u -m pytest tests/test_gpu_conv.py tests/test_gpu_fused.py tests/test_gpu_windows.py \
    -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for L in 2 4 6 8 11 13 16 18; do
  for V in base cur; do
    if [ $V = base ]; then export TQ_LIB_PATH=$BASE; else unset TQ_LIB_PATH; fi
    RES=""; case $L in 2|4|8|13|18) RES="--residual";; esac
    echo -n "$V "; timeout -k 10 120 python tools/conv_probe.py --layer $L --codes 1 $RES --iters 20 2>>$O/err.log | tail -1 || exit 1
  done
done | tee $O/probe.txt
for V in cur base cur base; do
  if [ $V = base ]; then export TQ_LIB_PATH=$BASE; else unset TQ_LIB_PATH; fi
  echo -n "$V "; timeout -k 10 300 python bench.py --no-cpu-baseline --no-d1 --no-d4 --steps 20 2>>$O/err.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('%.0f img/s conv %.1f us frac %.3f stem %.1f' % (d['value'], d['roofline']['avg_launch_us'], d['roofline']['frac'], d['roofline_tr']['avg_launch_us']))" || exit 1
done | tee $O/bench_ab.txt
unset TQ_LIB_PATH
timeout -k 10 300 python tools/gemm_ref.py > $O/gemm_ref.txt 2>>$O/err.log; cat $O/gemm_ref.txt
