#!/bin/bash
# Round-2 session: new GPU tests, the whole -m gpu suite, smoke, bench A/B of the fused
# downsample phase (TQ_FUSE_DS), then the profile set.  Ordinary test failures (rc 1) do not
# stop the script; a fault, abort or time limit does.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"
TAG=${1:-r02b}; O=gpurun_out/$TAG; mkdir -p $O
fatal() { [ "$1" -ge 124 ] && { echo "fatal rc=$1 at $2"; exit "$1"; }; return 0; }
timeout -k 10 300 python -u -m pytest tests/test_gpu_calib.py tests/test_gpu_fused.py -x -q \
  --timeout 120 --timeout-method thread -k "histc or linear_quantize or downsample_phase" > $O/new_tests.log 2>&1
rc=$?; tail -3 $O/new_tests.log; fatal $rc new_tests
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?; tail -3 $O/gpu_tests.log; fatal $rc gpu_tests
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
rc=$?; tail -1 $O/smoke.log; fatal $rc smoke
for v in 1 0 1 0; do
  TQ_FUSE_DS=$v timeout -k 10 300 python bench.py --steps 20 --no-cpu-baseline > $O/bench_ds$v.json 2>$O/bench_ds$v.err
  rc=$?; fatal $rc bench; python -c "import json,sys; d=json.loads(open('$O/bench_ds$v.json').read().splitlines()[-1]); print('ds=$v', round(d['value']), round(d['roofline']['avg_launch_us'],1), d['roofline']['launches'])"
done
bash tools/gpu_profile.sh $TAG
