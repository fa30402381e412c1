set -u
O=gpurun_out/r06k; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_fused_parity.py -x -v -s -k "stem" --timeout 400 --timeout-method thread > $O/seam_tests.log 2>&1
rc=$?; grep -E "stem|passed|failed|Error" $O/seam_tests.log | tail -8; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python bench.py --no-d4 --no-cpu-baseline > $O/bench.json 2> $O/bench.err
rc=$?; [ $rc -ne 0 ] && { tail -20 $O/bench.err; exit $rc; }
python -c "import json; d=json.loads(open('$O/bench.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['roofline_tr']['avg_launch_us'], 'fp32', d['stem_fp32']['images_per_s'], 'exact', d['stem_exact']['images_per_s'])"
echo done
