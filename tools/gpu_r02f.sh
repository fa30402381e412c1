#!/bin/bash
# Epilogue code tables: the whole -m gpu suite, per-layer probes and bench A/B (TQ_LUT).
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; O=gpurun_out/${TAG:-r02f}; mkdir -p $O
fatal() { [ "$1" -ge 124 ] && { echo "fatal rc=$1 at $2"; exit "$1"; }; return 0; }
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/t.log 2>&1; rc=$?; tail -3 $O/t.log; fatal $rc tests; [ $rc -ne 0 ] && exit $rc
for L in ${LAYERS:-1 2 6 11 16}; do for V in 0 1; do
  echo -n "lut=$V "; TQ_LUT=$V timeout -k 10 120 python tools/conv_probe.py --layer $L --codes 1 --no-out --iters 30 2>/dev/null | tail -1; rc=$?; fatal $rc probe
done; done
for V in 1 0 1 0; do
  TQ_LUT=$V timeout -k 10 300 python bench.py --steps 20 --no-cpu-baseline > $O/bench_l$V.json 2>$O/bench_l$V.err
  rc=$?; fatal $rc bench; python -c "import json; d=json.loads(open('$O/bench_l$V.json').read().splitlines()[-1]); print('lut=$V', round(d['value']), round(d['roofline']['avg_launch_us'],1), round(d['roofline_tr']['avg_launch_us'],1))"
done
bash tools/gpu_profile.sh ${TAG:-r02f}_prof
