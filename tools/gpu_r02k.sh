T=gpurun_out/r02m; mkdir -p $T
timeout -k 10 300 python -u -m pytest tests/test_gpu_windows.py -q --timeout 120 --timeout-method thread > $T/tests.log 2>&1; rc=$?; grep -E "Error|passed|failed" $T/tests.log | head -20; [ $rc -ne 0 ] && exit $rc
for m in "--codes 1 --no-out" "--codes 1 --residual"; do for c in 10 11; do
timeout -k 10 120 python tools/conv_probe.py --layer 1 --config $c $m --iters 50 || exit 1; done; done
TAG=r02m bash tools/gpu_strip_ab.sh
