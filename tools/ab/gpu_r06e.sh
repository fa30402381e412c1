set -u
O=gpurun_out/r06e; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_stem.py -x -q -s --timeout 300 --timeout-method thread > $O/stem_tests.log 2>&1
rc=$?; grep -E "exact stem|passed|failed|Error" $O/stem_tests.log | tail -12; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -u -m pytest tests/test_gpu_fused_parity.py -x -v -s -k "stem" --timeout 400 --timeout-method thread > $O/seam_tests.log 2>&1
rc=$?; grep -E "stem|passed|failed|Error" $O/seam_tests.log | tail -20; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --no-d4 --no-cpu-baseline > $O/bench.json 2> $O/bench.err
rc=$?; [ $rc -ne 0 ] && { tail -20 $O/bench.err; exit $rc; }
python -c "import json; d=json.loads(open('$O/bench.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['stem_fp32']['images_per_s'], d['roofline_tr']['avg_launch_us'], d['config']['stem'][:30])"
timeout -k 10 300 python bench.py --no-d4 --no-cpu-baseline --no-d1 --stem split --no-stem-leg > $O/bench_split.json 2> $O/bench_split.err
rc=$?; [ $rc -ne 0 ] && { tail -20 $O/bench_split.err; exit $rc; }
python -c "import json; d=json.loads(open('$O/bench_split.json').read().strip().splitlines()[-1]); print('split', d['value'], d['ms_per_step'], d['roofline_tr']['avg_launch_us'])"
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o kt -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-d1 --no-d4 --no-stem-leg --streams 1 --launch eager > $O/kt.log 2>&1
rc=$?; [ $rc -ne 0 ] && { tail -20 $O/kt.log; exit $rc; }
python3 -c "
import csv
for r in csv.DictReader(open('$O/kt/kt_kernel_stats.csv')):
    if 'stem' in r['Name']: print(r['Name'][:60], r['Calls'], round(float(r['AverageNs'])/1000,1))
"
echo "== r05b reproduction: first c64 build, fused-parity file without the stem tests"
TQ_LIB_PATH=$PWD/term-quantization_amd/lib/libtq_hip_r05b.so timeout -k 10 400 python -u -m pytest tests/test_gpu_fused_parity.py -x -q -k "not stem" --timeout 300 --timeout-method thread > $O/r05b_parity.log 2>&1
rc=$?; tail -3 $O/r05b_parity.log
TQ_LIB_PATH=$PWD/term-quantization_amd/lib/libtq_hip_r05b.so timeout -k 10 400 python -u tools/ab/diag_streams.py 12 > $O/diag_r05b.log 2>&1
tail -6 $O/diag_r05b.log
echo done
