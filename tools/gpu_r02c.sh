R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; O=gpurun_out/r02c; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_models.py tests/test_gpu_fused.py -q --timeout 120 --timeout-method thread -k "wide or depthwise_models or downsample" > $O/t.log 2>&1; rc=$?; tail -15 $O/t.log; [ $rc -ge 124 ] && exit $rc
timeout -k 10 600 python tools/bench_d4.py > $O/d4.log 2>&1; rc=$?; tail -5 $O/d4.log; [ $rc -ne 0 ] && exit $rc
bash tools/gpu_ablate_patch.sh r02c_abl > $O/abl.log 2>&1; rc=$?; cat $O/abl.log; exit $rc
