set -u
O=gpurun_out/r06m; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_stem.py -x -q --timeout 300 --timeout-method thread > $O/stem_tests.log 2>&1
rc=$?; tail -2 $O/stem_tests.log; [ $rc -ne 0 ] && exit $rc
for r in 1 2; do for v in base q64; do
  L=$PWD/term-quantization_amd/lib/libtq_hip.so; [ $v != base ] && L=$PWD/term-quantization_amd/lib/libtq_hip_$v.so
  TQ_LIB_PATH=$L timeout -k 10 300 python3 bench.py --no-d4 --no-d1 --no-cpu-baseline --no-stem-leg > $O/b_${v}_$r.json 2> $O/b_${v}_$r.err
  rc=$?; [ $rc -ne 0 ] && { tail -5 $O/b_${v}_$r.err; exit $rc; }
  python3 -c "import json; d=json.loads(open('$O/b_${v}_$r.json').read().strip().splitlines()[-1]); print('$v', round(d['value']), round(d['ms_per_step'],4), 'stem', round(d['roofline_tr']['avg_launch_us'],1), 'conv', round(d['roofline']['avg_launch_us'],2))"
done; done
echo done
