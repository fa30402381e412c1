set -u
O=gpurun_out/r06f; mkdir -p $O
timeout -k 10 300 python -u tools/ab/stem_fix_count.py > $O/fix_count.log 2>&1
rc=$?; tail -8 $O/fix_count.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -u -m pytest tests/test_gpu_stem.py -x -q -s --timeout 300 --timeout-method thread -k exact > $O/stem_tests.log 2>&1
rc=$?; grep -E "exact stem|passed|failed|Error" $O/stem_tests.log | tail -8; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -u -m pytest tests/test_gpu_fused_parity.py -x -q -s -k "correctly_rounded" --timeout 400 --timeout-method thread > $O/seam_tests.log 2>&1
rc=$?; grep -E "stem|passed|failed|Error" $O/seam_tests.log | tail -5; [ $rc -ne 0 ] && exit $rc
echo done
